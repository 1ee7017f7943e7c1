// Kernel launch interface between the C-ABI (api.cpp) and the HIP kernels (trace.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "device_types.h"

namespace rtamd {

struct DeviceScene {  // device pointers (HBM), immutable after upload
	const DGeom* geoms;
	const DMaterial* mats;
	const DLight* lights;
	const DFaceGeo* fgeo;
	const DFaceNrm* fnrm;
	const int32_t* fid;
	const DBvhNode* nodes;
	DCamera cam;
	int32_t n_geoms, n_lights, n_nonambient;
	int32_t pad;
};

// One wavefront level of ray records (structure of arrays).
struct RayLevel {
	// ray in (unused at level 0: primary rays are generated from the pixel index)
	double *ox, *oy, *oz, *dx, *dy, *dz;
	uint8_t* inside;
	// node out
	double *cr, *cg, *cb;        // local colour, overwritten with the final colour by reduce
	double *kr, *kg, *kb;        // reflective weight (after TIR), valid when child_refl >= 0
	int32_t *child_refr, *child_refl;
	int64_t capacity;
};

struct FrameGeometry {
	int32_t width, height;
	int32_t row_begin, row_step;  // selected rows: row_begin + k*row_step
	int32_t chunk_row0;           // first selected-row ordinal of this chunk
	int32_t intersection_only;
};

// Device counters: first error code, next-level ray count, shaded hits (x non-ambient
// lights = shadow rays), running max (bits) for --intersection-only, children spawned
struct DeviceCounters {
	int32_t error;
	int32_t next_count;
	unsigned long long hits;
	unsigned long long max_bits;
	unsigned long long refl, refr;
	unsigned long long node_visits, tri_tests, candidates, sphere_tests;
};

hipError_t launch_trace_level(const DeviceScene& s, const FrameGeometry& fg, int level, int64_t n,
                              int remaining_depth, const RayLevel& cur, const RayLevel& next,
                              DeviceCounters* ctr, hipStream_t stream);
hipError_t launch_reduce_level(int64_t n, const RayLevel& cur, const RayLevel& next, hipStream_t stream);
hipError_t launch_output(int64_t n, const RayLevel& lvl0, double* out_rgb, uint8_t* out_rgb8,
                         int32_t intersection_only, DeviceCounters* ctr, hipStream_t stream);
hipError_t launch_normalize(int64_t n_values, double* rgb, double max_value, uint8_t* out_rgb8, hipStream_t stream);
hipError_t launch_selftest_math(int op, const double* x, const double* y, double* out, int64_t n, hipStream_t stream);

}  // namespace rtamd
