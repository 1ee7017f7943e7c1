// TEST INFRASTRUCTURE ONLY — the CPU oracle for the ray-trace hot path.
//
// A plain-C++ restatement of the reference's render path (scene ingest + Whitted
// ray tracing), bit-exact in IEEE-754 binary64 against the unmodified reference
// (oracle/_ref/refharness, built from /root/reference/src by oracle/Makefile) and
// against the reference's shipped goldens (tests/golden/).  Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product
// (librtamd.so) never links or calls it.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_counters {
	int64_t trace_rays;      // Scene::traceRay calls (primary + reflection + refraction), scene.cpp:61
	int64_t shadow_rays;     // shadow castRay calls, scene.cpp:90-91
	int64_t reflect_rays;    // scene.cpp:130-135
	int64_t refract_rays;    // scene.cpp:124-127
	int64_t sphere_tests;    // Sphere::calculateIntNormInObjSpace calls, geometry.cpp:47
	int64_t mesh_tests;      // Mesh::calculateIntNormInObjSpace calls, geometry.cpp:69
	int64_t bbox_pass;       // mesh calls past the hitsBoundingBox gate, geometry.cpp:72-74
	int64_t face_tests;      // faces visited in the linear face loop, geometry.cpp:78
} oracle_counters;

// Renders rows row_begin, row_begin+row_step, ... < row_end of an H x W image of the scene made of the given
// .rti files (main.cpp:54-62: one parser per file), with bounce depth `bdepth` and the
// --intersection-only flag.  out: n_rows*W*3 doubles, row-major (selected rows in order).
// intersection-only normalisation (scene.cpp:50-58) is applied over the rendered rows
// only when they cover the whole image.  threads: std::threads with the reference's
// 2000-pixel block dispenser (scene.cpp:13-48, with the last block clamped).
// Returns 0, or 1 = parse error, 2 = math error (text in oracle_last_error()).
int oracle_render(const char* const* rti_files, int n_files, int W, int H, int bdepth,
                  int intersection_only, int threads, int row_begin, int row_end, int row_step,
                  double* out, oracle_counters* counters);
const char* oracle_last_error(void);
// Warnings the parser printed (ParseException::showWarning text, exceptions.h:15-17),
// newline separated, for the last oracle_render call.
const char* oracle_last_warnings(void);

// PNG byte conversion of writers.cpp:4-9: clamp to [0,1], *255, truncate.
void oracle_to_rgb8(const double* rgb, int64_t n_pixels, uint8_t* out);

#ifdef __cplusplus
}
#endif
