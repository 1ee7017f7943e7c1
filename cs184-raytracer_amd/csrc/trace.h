// Kernel launch interface between the C-ABI (api.cpp) and the HIP kernels (trace.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "device_types.h"

namespace rtamd {

// lights whose shadow verdicts fit the 64-bit mask of the fused level-0 shading (more
// lights use the light-major layout and k_shade)
constexpr int kMaxShadowLights = 64;

struct DeviceScene {  // device pointers (HBM), immutable after upload
	const DGeom* geoms;
	const DMaterial* mats;
	const DLight* lights;
	const DFaceGeo* fgeo;
	const DFaceNrm* fnrm;
	const DBvhNode* nodes;
	const int32_t* shadow_order;              // geometry order of the occlusion query
	// the camera (device copy): read where primary rays are made, not held in registers for
	// the kernel's lifetime as a 160-B by-value kernel argument would be
	const DCamera* cam;
	int32_t n_geoms, n_lights, n_nonambient;
	int32_t n_may_raise;                      // geometries with DGeom::may_raise
	int32_t n_meshes;                         // meshes of the scene
	int32_t n_faces, n_nodes;                 // records in fgeo, nodes (the L2 warm-up of level 0)
	int32_t mesh_kind;                        // kernels: 0 spheres only, 1 meshes without LBVHs, 2 with (intersect.h)
	const int32_t* shadow_light;              // j-th non-ambient light -> light index
	int32_t work_stats;                       // count the LBVH work (rt_counters node_visits ...); 0 = skip
};

// One wavefront level of ray records (structure of arrays).
struct RayLevel {
	// ray in (unused at level 0: primary rays are generated from the pixel index)
	double *ox, *oy, *oz, *dx, *dy, *dz;
	uint8_t* inside;
	// closest hit (k_closest -> k_shadow, k_shade)
	int32_t* hgeom;              // hit geometry, -1 = miss
	// hit records, compacted: entry h (0 <= h < counts[0]) is the h-th hit found, ray hit_list[h]
	double *hpx, *hpy, *hpz;     // world hit point
	double *hnx, *hny, *hnz;     // shading normal (flipped if inside, normalised)
	double *hdx, *hdy, *hdz;     // the ray's direction (the viewing ray of the Phong terms)
	uint8_t* hinside;            // bit 0: the ray's inside flag; bit 1: the material's DMaterial::zero_terms
	int32_t* hit_list;           // ray index of each hit (order of discovery)
	uint8_t* occl;               // [non-ambient light][hit] shadow verdicts (light j at j * capacity)
	// node out
	double *cr, *cg, *cb;        // local colour, overwritten with the final colour by reduce
	// (the reflective weight of a hit with a reflection child is its material's, or 1 on total
	// internal reflection: reduce_colour derives it from hgeom and child_refr, trace.hip)
	int32_t *child_refr, *child_refl;
	int32_t* counts;             // [0] hits of this level (k_closest), [1] children spawned
	int64_t capacity;
};

// A chunk holds the selected rows of one frame or of several frames of the same width,
// height and depth (rt_render_batch_device): small row selections, such as one GPU's share
// of row-partitioned frames, are then traced as one full-size wavefront.  Its rows are
// described by value, in the kernel arguments: a segment is a run of rows of one job, whose
// image rows and output rows follow from the ordinal arithmetically (scene.cpp:25-31: pixel
// -> (r, c) -> output(r, c)), so no kernel reads a row table from memory.
// Chunks are cut so that they never hold more segments than this (api.cpp plan_chunks).
#ifndef RT_MAX_ROW_SEGMENTS
#define RT_MAX_ROW_SEGMENTS 32
#endif
constexpr int kMaxRowSegments = RT_MAX_ROW_SEGMENTS;
struct RowSegment {
	double* out;          // the job's f64 rows: ordinal o at out + o * width * 3 (or null)
	uint8_t* out8;        // its RGB8 rows, the same layout (or null)
	int32_t q0;           // the chunk row of the segment's first row
	int32_t ord0;         // that row's ordinal in the job's row selection
	int32_t ord_end;      // the job's selected rows (ordinals at or past it: a corrupt descriptor)
	int32_t row_begin;    // image row of ordinal o: row_begin + (o / row_block) * row_span + o % row_block
	int32_t row_block;    // (rt_render_params: row_block >= 1, row_span = row_step * row_block;
	int32_t row_span;     //  the image row r gives rowFrac = (r + 0.5) / H, scene.cpp:28)
};
struct FrameGeometry {
	int32_t width, height;
	int32_t intersection_only;
	int32_t n_rows;       // rows of the chunk: pixel i is column i % width of chunk row i / width
	int32_t n_segs;       // 1 .. kMaxRowSegments, seg[k].q0 ascending from seg[0].q0 = 0
	int32_t pad;
	RowSegment seg[kMaxRowSegments];
};

// Row partition over devices (rt_partition_row): blocks of B rows interleaved over n
__host__ __device__ inline void partition_row(int64_t row, int n, int B, int* dev, int64_t* local) {
	B = B < 1 ? 1 : B;
	const int64_t blk = row / B;
	*dev = static_cast<int>(blk % n);
	*local = (blk / n) * B + row % B;
}

// Multi-GPU assembly on the first device: image row r (row_bytes each) comes from device
// partition_row(r)'s buffer src[dev] at its local row
constexpr int kMaxGpus = 16;
struct RowSources {
	const uint8_t* src[kMaxGpus];
};
hipError_t launch_deinterleave(uint8_t* dst, const RowSources& s, int n, int block, int64_t height, int64_t row_bytes,
                               hipStream_t stream);

// Device error word (first MathException code).  Ray and hit counts live per level
// (RayLevel::counts) so that levels in flight on different streams never share one.
struct DeviceCounters {
	int32_t error;
	int32_t pad[3];
};

// Statistics are sharded: a single word takes only ~88 atomics/us on MI355X
// (MI355X_MICROARCH.md, "dequeue"), so every block adds into shard blockIdx % kStatShards
// (one 128-B line each) and the host sums the shards.
constexpr int kStatShards = 256;
enum StatSlot : int {
	ST_HITS = 0, ST_REFL, ST_REFR, ST_MAX_BITS,
	ST_NODES0, ST_TRIS0, ST_CANDS0, ST_SPHERES0,   // k_closest
	ST_NODES1, ST_TRIS1, ST_CANDS1, ST_SPHERES1,   // k_shadow
	ST_ENTRIES0, ST_ENTRIES1,                      // LBVH traversals started
	ST_MAXNODES0, ST_MAXNODES1,                    // most node visits of one ray (max)
	ST_SHADOW_ZERO,                                // shadow rays whose Phong terms are zero (not traced)
	ST_RAYS,                                       // rays traced by k_closest (traceRay calls)
	ST_COUNT
};
constexpr int kStatStride = 32;  // u64 per shard (256 B)

// Level pipeline.  k_closest(L) finds the closest hits of level L, appends the hits to
// cur.hit_list (count cur.counts[0]) and spawns the reflection/refraction children into
// `next` (count cur.counts[1]).  The shading of level L (shadow rays, then Phong terms)
// depends only on k_closest(L), so it runs on a second stream while k_closest(L+1)
// traces the children: the latency-bound deep levels overlap with shading work.
// packet_mask selects wave-packet traversal per kernel and level class (N: every level
// >= 1; 1: level 1 only)
enum : int {
	kPacketClosest0 = 1, kPacketClosestN = 2, kPacketShadow0 = 4, kPacketShadowN = 8,
	kPacketClosest1 = 16, kPacketShadow1 = 32
};
// n: the level's ray count (level 0), or with n_dev (the previous level's child counter,
// read on the device) an upper bound used only to size the grid.  levels_dev: the device
// copy of the RayLevel records (level and level + 1 must be current).
// plan_last: the last level of a replayed plan (api.cpp): a child spawned there raises
// DERR_PLAN instead of being written (the plan had no further level for it)
hipError_t launch_closest(const DeviceScene& s, const FrameGeometry& fg, int level, int64_t n, const int32_t* n_dev,
                          int remaining_depth, const RayLevel* levels_dev, DeviceCounters* ctr,
                          unsigned long long* stats, hipStream_t stream, int packet_mask, int plan_last = 0,
                          hipEvent_t done = nullptr);
// Shading of one or more levels in one launch (the deep levels are shaded together once
// the closest-hit chain has finished).  Items of each level start on a wave boundary so
// that every wave belongs to one level.  levels_dev: device copy of the RayLevel records.
constexpr int kMaxBatch = 16;
struct ShadeBatch {
	int32_t n;                           // levels in the batch
	int32_t level[kMaxBatch];
	int64_t nh[kMaxBatch];               // hits of each level (cur.counts[0])
	int32_t all_lights;                  // k_shadow items: 1 = one per hit (all lights), 0 = per (light, hit)
	int32_t fused;                       // all_lights only: k_shadow also computes the Phong terms (no k_shade)
	int64_t shadow_begin[kMaxBatch + 1]; // k_shadow item ranges: (all_lights ? 1 : n_nonambient) x nh rounded up to 64
	int64_t shade_begin[kMaxBatch + 1];  // k_shade item ranges: nh each
	// Device-counted batch (the hipGraph plans of api.cpp): nh[k] is the level's hit counter
	// nh_dev[k][0], read by the kernels, which derive the item ranges themselves; the grid is
	// fixed and strides over the items.  nh / shadow_begin / shade_begin are then unused.
	int32_t dev_counts;
	const int32_t* nh_dev[kMaxBatch];
};


hipError_t launch_shadow(const DeviceScene& s, const ShadeBatch& b, const RayLevel* levels_dev, DeviceCounters* ctr,
                         unsigned long long* stats, hipStream_t stream, int packet_mask);
// ShadeBatch::fused may be set only when this holds (the wave-packet all-lights form; with
// per_lane also the per-lane one of scenes without LBVHs)
bool shadow_can_fuse(const DeviceScene& s, const ShadeBatch& b, int packet_mask, bool per_lane);
hipError_t launch_shade(const DeviceScene& s, const ShadeBatch& b, const RayLevel* levels_dev, DeviceCounters* ctr,
                        hipStream_t stream);
// n: the level's ray count, or with n_dev (the previous level's child counter) read on the
// device (a fixed grid strides over it)
// low non-null: two levels at once, cur's final colours from next's local colours reduced on
// the fly with low's final ones (next's final colours are not written)
hipError_t launch_reduce_level(const DeviceScene& s, int64_t n, const int32_t* n_dev, const RayLevel& cur,
                               const RayLevel& next, const RayLevel* low, hipStream_t stream);
// Where a fused level (launch_fused) puts its colours: final != 0 (a plan of one traced
// level): straight into the chunk's output rows (no k_output); else into the level's colours
// for k_reduce / k_output.  summary != null: the launch's last block reduces the statistics
// shards into it (launch_stats_finish's work without a launch; `done` counts the finished
// blocks and is reset by the last one).
struct FusedOut {
	int32_t final;
	int32_t pad;
	unsigned long long* summary;
	uint32_t* done;
};
// lvl1 non-null: level 0's reduction with level 1 (k_reduce) is fused into the output (lvl2
// non-null too: with levels 1 and 2, as launch_reduce_level's two-level form); pixels go to
// their rows' outputs (fg.seg); finish non-null: the statistics finish too
hipError_t launch_output(const DeviceScene& s, int64_t n, const FrameGeometry& fg, const RayLevel& lvl0,
                         const RayLevel* lvl1, const RayLevel* lvl2, unsigned long long* stats, hipStream_t stream,
                         DeviceCounters* ctr, const FusedOut* finish = nullptr);
// The reductions of a chunk of n_levels traced levels, deepest first, two levels per launch:
// {l, k} reduces level l with the k levels below it (l = 0: the output launch)
struct ReduceStep {
	int level, levels;
};
inline int reduce_steps(int n_levels, ReduceStep* out /* n_levels entries */) {
	int n = 0, j = n_levels - 1;  // j: the deepest level whose colours are final
	for (; j >= 2; j -= 2) out[n++] = {j - 2, 2};
	if (j == 1) out[n++] = {0, 1};
	if (n_levels == 1) out[n++] = {0, 0};
	return n;
}
// One level in one launch (k_fused): closest hits, children, and every hit's shadow rays and
// Phong terms from registers (the level's k_closest + k_shadow + k_shade); never for
// --intersection-only or counting renders.  Arguments as launch_closest.
hipError_t launch_fused(const DeviceScene& s, const FrameGeometry& fg, int level, int64_t n, const int32_t* n_dev,
                        int remaining_depth, const RayLevel* levels_dev, DeviceCounters* ctr, unsigned long long* stats,
                        hipStream_t stream, int packet_mask, int plan_last, const FusedOut& fo);
// End of a render: summary[k] = sum over the shards of statistic k (max for ST_MAX_BITS),
// summary[ST_COUNT] = the device error word; the shards and the error word are cleared for
// the next render.
hipError_t launch_stats_finish(unsigned long long* stats, DeviceCounters* ctr, unsigned long long* summary,
                               hipStream_t stream);
hipError_t launch_normalize(int64_t n_values, double* rgb, double max_value, uint8_t* out_rgb8, hipStream_t stream);
// n_words 16-byte words from src (device-readable, e.g. mapped pinned host memory) to dst
hipError_t launch_copy16(void* dst, const void* src, int64_t n_words, hipStream_t stream);
// Phase profile (builds with -DRT_PHASE_PROF=1 only, else zeros): per (stage, packet) pair
// (stage 0 k_closest, 1 k_shadow) 8 sums of per-lane shader-clock cycles (intersect.h
// PhaseSlot); copied and cleared.
constexpr int kPhaseSlots = 8;
hipError_t read_phase_profile(unsigned long long* out /* 4 * kPhaseSlots */);
// RT_DIAG_WAVETIME builds: the wave records since the last call (32 B each, intersect.h
// WaveTime), at most max_records, then cleared; 0 in other builds, -1 on a HIP error
int read_wave_times(void* out, int max_records);
// FETCH_SIZE calibration: reads `bytes` of buf once, `width` (1, 4, 8, 16) bytes per lane
// VALU issue calibration: kind 0 v_fma_f32, 1 v_pk_fma_f32, 2 v_fma_f64 chains at
// waves_per_simd waves on every SIMD
hipError_t launch_valu_peak(int iters, int kind, int waves_per_simd, void* sink, hipStream_t stream);
hipError_t launch_stream_read(const void* buf, int64_t bytes, int width, unsigned long long* sink, hipStream_t stream);
hipError_t launch_selftest_math(int op, const double* x, const double* y, double* out, int64_t n, hipStream_t stream);

}  // namespace rtamd
