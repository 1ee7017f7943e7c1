/*
 * rtamd — MI355X-native Whitted ray tracer: the C-ABI drop-in boundary.
 *
 * Replaces the render path of gh2o/CS184-Raytracer (reference at /root/reference):
 *
 *   reference                                         this ABI
 *   ------------------------------------------------  ------------------------------------------
 *   Scene scene;                     main.cpp:53       rt_builder_create
 *   RTIParser(scene).parseFile(f)    parsers.cpp:93    rt_builder_parse_rti   (+ OBJParser, :253)
 *   scene.hasCamera()                scene.h:20        rt_builder_has_camera
 *   (geometry/lights live in Scene)  scene.h:35-38     rt_scene_create        (upload once to HBM)
 *   Scene::renderScene(img, ph)      scene.h:14,       rt_render              (host f64 image)
 *                                    scene.cpp:10-59   rt_render_device       (device buffers)
 *   ProgressHandler(int,int)         scene.h:12        rt_progress_fn (+ user pointer)
 *   programOptions.bounceDepth_ ...  options.h:10-16   rt_render_params
 *   PNGWriter(f).writeImage(img)     writers.cpp:11-21 rt_write_png           (byte-identical PNG)
 *   convertToRGBImage                writers.cpp:4-9   rt_to_rgb8
 *   MathException / ParseException  exceptions.h      return codes + rt_last_error()
 *
 * Plain pointers and sizes only; no HIP or torch types.  Images are row-major
 * H x W x 3 (the RasterImage layout, scene.h:11).  All functions return RT_OK (0) or
 * a negative RT_ERR_* code; rt_last_error() then holds the message text, identical to
 * the reference's exception what() where the reference throws.
 */
#ifndef RTAMD_H
#define RTAMD_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* The layout version of the structs below.  Round 4 appended fields to rt_scene_info
 * (level_bytes, build_ms, upload_ms) and rt_counters (host_ms, copy_ms): a caller built
 * against an older header would have those bytes written past its structs.  Check
 * rt_abi_version() == RTAMD_ABI_VERSION once after loading the library. */
#define RTAMD_ABI_VERSION 5
int rt_abi_version(void);

enum {
	RT_OK = 0,
	RT_ERR_PARSE = -1,   /* ParseException (exceptions.h:6-21): "line N: ..." / "file not found: ..." */
	RT_ERR_MATH = -2,    /* MathException (exceptions.h:23-26): "ray has no direction", ...          */
	RT_ERR_ARG = -3,     /* invalid argument (sizes, rows, null pointers)                            */
	RT_ERR_DEVICE = -4,  /* HIP runtime failure, or the HIP path is unavailable                      */
	RT_ERR_IO = -5       /* WriteException (exceptions.h:28-31) / output not writable                */
};

/* ---------------------------------------------------------------- ingest (host C++) */
typedef struct rt_builder rt_builder;

rt_builder* rt_builder_create(void);
void rt_builder_destroy(rt_builder* b);
/* One call = one `RTIParser parser(scene); parser.parseFile(path);` (main.cpp:54-62):
 * transform and material state restart for every file, geometry/lights accumulate. */
int rt_builder_parse_rti(rt_builder* b, const char* path);
int rt_builder_has_camera(const rt_builder* b);
/* Warnings printed by the reference (ParseException::showWarning), "Warning: ...\n" each. */
const char* rt_builder_warnings(const rt_builder* b);

typedef struct rt_scene_info {
	int32_t n_geometries, n_spheres, n_meshes, n_lights;
	int64_t n_faces;         /* triangles incl. the two faces of every `tri` line      */
	int64_t n_bvh_nodes;     /* flattened LBVH nodes over all meshes                  */
	int64_t device_bytes;    /* HBM held by the uploaded scene                        */
	int32_t max_bvh_depth;   /* deepest LBVH (root = depth 0)                          */
	int32_t reserved;
	int64_t level_bytes;     /* HBM held by the ray-level buffers of the renders so far
	                            (grown on demand, kept for later renders)              */
	double  build_ms;        /* host time of rt_scene_create's LBVH build + flattening  */
	double  upload_ms;       /* host time of its HBM allocations, copies and set-up     */
	int64_t level_bytes_peak;  /* most level-buffer HBM held at once so far (a host-driven
	                              trace sizes levels with one level of lookahead; after the
	                              call they are cut back to the rays the levels held)   */
	int64_t level_budget;    /* RTAMD_LEVEL_BUDGET (0: none): level_bytes never exceeds it;
	                            a render that would need more is traced in smaller chunks */
} rt_scene_info;

/* ---------------------------------------------------------------- flat scene descriptor */
/* The reference's in-memory Scene (scene.h:35-38) as plain arrays, for a caller that
 * already holds one (e.g. Scene::renderScene itself): no file, no
 * re-parse.  Every field is a member the reference's objects hold, in its own layout:
 *   - transforms are Eigen's Transform<double,3,Affine> storage, 16 doubles column-major
 *     (Transformable::forwardTransform().data(), rtbase.h:41-64);
 *   - Mesh faces are Mesh::Face verbatim (geometry.h:32: std::array<Vector4d,3> points_,
 *     normals_ = 24 doubles, 192 B), so mesh->faces_.data() can be passed as is;
 *   - camera corners and light vectors are the UNtransformed points/directions given to
 *     the setters (rtbase.h:69-73, lights.h:26,54): the library applies forwardTransform()
 *     once, in Eigen's order, instead of the reference's lazy (racy) caches. */
enum { RT_GEOM_SPHERE = 0, RT_GEOM_MESH = 1 };
enum { RT_LIGHT_POINT = 0, RT_LIGHT_DIRECTIONAL = 1, RT_LIGHT_AMBIENT = 2 };

typedef struct rt_xform_desc {      /* Transformable (rtbase.h:41-64)                        */
	double fwd[16];                 /* forwardTransform().data(), column-major 4x4          */
	double inv[16];                 /* inverseTransform().data()                             */
	double det;                     /* transformDeterminant()                                */
	int32_t derive;                 /* 1: inv and det are derived from fwd here, exactly as
	                                   Transformable::forwardTransform(xf) does (rtbase.h:51-54) */
	int32_t reserved;
} rt_xform_desc;

typedef struct rt_material_desc {   /* Material (rtbase.h:30-39), same field order           */
	double ambient[3], diffuse[3], specular[3], reflective[3];
	double specular_coefficient;
	double translucency[3];
	double index_of_refractivity;
} rt_material_desc;

typedef struct rt_face_desc {       /* Mesh::Face (geometry.h:32), object space; point w == 1 */
	double points[3][4];
	double normals[3][4];
} rt_face_desc;

typedef struct rt_geometry_desc {   /* Geometry (geometry.h:6-14)                            */
	int32_t kind;                   /* RT_GEOM_SPHERE (Sphere) or RT_GEOM_MESH (Mesh)        */
	int32_t reserved;
	rt_xform_desc xf;
	rt_material_desc material;      /* Geometry::material_                                   */
	double center[4];               /* Sphere::center_                                       */
	float radius;                   /* Sphere::radius_ (float, geometry.h:22)                */
	float reserved_f;
	const rt_face_desc* faces;      /* Mesh::faces_.data()                                   */
	int64_t n_faces;                /* Mesh::faces_.size()                                   */
	double bbox_min[4], bbox_max[4]; /* Mesh::boundingBoxMin_/Max_ (geometry.h:35-36): zero
	                                   unless Mesh::updateBoundingBox ran (obj meshes)        */
} rt_geometry_desc;

typedef struct rt_light_desc {      /* Light (lights.h:3-75)                                 */
	int32_t kind;                   /* RT_LIGHT_POINT / _DIRECTIONAL / _AMBIENT              */
	int32_t reserved;
	rt_xform_desc xf;               /* only forwardTransform() is used (lights.h:31,59)      */
	double color[3];                /* Light::color_                                         */
	double vec[4];                  /* PointLight::point_ / DirectionalLight::direction_      */
	double falloff;                 /* PointLight::falloffExponent_                          */
} rt_light_desc;

typedef struct rt_camera_desc {     /* Camera (rtbase.h:66-103)                              */
	rt_xform_desc xf;
	double eye[4], lower_left[4], lower_right[4], upper_left[4], upper_right[4];
} rt_camera_desc;

typedef struct rt_scene_desc {      /* Scene (scene.h:35-38)                                 */
	int32_t has_camera;             /* Scene::hasCamera()                                    */
	int32_t n_geometries;
	int32_t n_lights;
	int32_t reserved;
	rt_camera_desc camera;
	const rt_geometry_desc* geometries;  /* Scene::geometries_, insertion order (scene.cpp:147) */
	const rt_light_desc* lights;         /* Scene::lights_, definition order (scene.cpp:78)    */
} rt_scene_desc;

/* A parsed scene as a descriptor: views into the builder's memory, valid until the builder
 * is destroyed or parses another file (the transforms are those the parser computed). */
int rt_builder_get_desc(const rt_builder* b, rt_scene_desc* out);
/* Replaces the builder's scene by a copy of the descriptor's (the host scene that
 * rt_scene_create_desc uploads). */
int rt_builder_set_desc(rt_builder* b, const rt_scene_desc* d);

/* ---------------------------------------------------------------- device scene */
typedef struct rt_scene rt_scene;

/* Builds the per-mesh LBVHs and uploads geometry, materials, lights and camera to
 * HBM of HIP device `device` once; the scene is immutable afterwards. */
int rt_scene_create(const rt_builder* b, int device, rt_scene** out);
/* The same from a flat descriptor (the caller's own Scene, no file): equal to
 * rt_builder_set_desc + rt_scene_create.  The descriptor may be freed on return. */
int rt_scene_create_desc(const rt_scene_desc* d, int device, rt_scene** out);
void rt_scene_destroy(rt_scene* s);
int rt_scene_get_info(const rt_scene* s, rt_scene_info* info);

/* ---------------------------------------------------------------- render */
typedef void (*rt_progress_fn)(int complete, int total, void* user);

typedef struct rt_render_params {
	int32_t width, height;        /* -w / -h (options.h:13-14)                             */
	int32_t bounce_depth;         /* --bdepth (options.h:15), >= 0                         */
	int32_t intersection_only;    /* --intersection-only (options.h:16)                    */
	/* Rows rendered, in this order: blocks of row_block consecutive rows (0 or 1: single
	 * rows) starting at row_begin, row_begin + row_step*row_block, ... below row_end.  The
	 * multi-GPU partition gives rank k of N {k*B, H, N} with B = row_block: row r goes to
	 * rank (r / B) mod N.  {0, height, 1} renders the whole image. */
	int32_t row_begin, row_end, row_step;
	/* Pixels per wavefront pass (bounds queue memory); 0 = automatic. */
	int32_t chunk_pixels;
	int32_t row_block;            /* see row_begin; 0 = 1 */
	/* Nonzero: count the traversal work into rt_counters (node_visits, tri_tests, candidates,
	 * sphere_tests and their stage_* splits) with the counting instantiation of the
	 * traversal kernels, about 6% slower; 0 (the default): those counters read 0.  Images
	 * are bitwise equal either way.  Any nonzero entry of a batch counts the whole call;
	 * RTAMD_WORK_STATS=1 in the environment counts every call. */
	int32_t work_stats;
} rt_render_params;

typedef struct rt_counters {
	int64_t trace_rays;      /* Scene::traceRay calls: primary + reflection + refraction */
	int64_t shadow_rays;     /* shadow castRay calls (scene.cpp:90-91)                   */
	int64_t reflect_rays, refract_rays;
	int64_t pixels;
	double  intersection_max;   /* max over rendered pixels of maxCoeff (scene.cpp:50-53),
	                               only with intersection_only                          */
	double  kernel_ms;          /* device time of the per-level kernels (HIP events)     */
	int32_t levels;             /* wavefront levels executed (max over chunks)          */
	int32_t trace_launches;     /* per-level kernel launches                             */
	/* work done by the traversal kernels (algorithmic bytes/flops) */
	int64_t node_visits;        /* LBVH nodes visited (2 child boxes tested each)       */
	int64_t tri_tests;          /* ray-triangle (Cramer) tests                          */
	int64_t candidates;         /* tests that reached the normal fetch + facing test    */
	int64_t sphere_tests;       /* ray-sphere tests                                     */
	/* per-kernel split: [0] k_closest (camera/secondary rays), [1] k_shadow, [2] k_shade */
	double  stage_ms[3];
	int32_t stage_launches[3];
	int64_t stage_node_visits[2], stage_tri_tests[2], stage_candidates[2], stage_sphere_tests[2];
	int64_t stage_bvh_traversals[2];   /* mesh LBVH traversals started (the mesh gate is tested after) */
	int64_t stage_max_node_visits[2];  /* most LBVH nodes one ray visited (all meshes)       */
	int64_t shadow_rays_zero_terms;    /* shadow rays (counted in shadow_rays) whose diffuse and
	                                      specular terms are exact zeros, so the verdict cannot
	                                      change the colour: decided without traversal         */
	double  host_ms;   /* wall time of the call on the host, entry to return                 */
	double  copy_ms;   /* of which the image's device-to-host copy (rt_render, rt_render_rgb8) */
} rt_counters;

/* Scene::renderScene into a caller-owned host buffer of n_rows*W*3 doubles
 * (n_rows = rows selected by row_begin/row_end/row_step/row_block, in that order).
 * With intersection_only and the whole image selected, the output is normalised by
 * the global maximum exactly as scene.cpp:50-58; otherwise the raw 1/d^2 values are
 * returned with counters->intersection_max for the caller's global reduction. */
int rt_render(rt_scene* s, const rt_render_params* p, double* out_rgb,
              rt_progress_fn progress, void* user, rt_counters* counters);

/* Scene::renderScene + PNGWriter::convertToRGBImage (writers.cpp:4-9) into a caller-owned
 * host buffer of n_rows*W*3 bytes: the image is quantised on the device and only the RGB8
 * bytes cross PCIe (an eighth of rt_render's f64 copy).  --intersection-only needs the
 * whole image here (the global maximum normalises it first). */
int rt_render_rgb8(rt_scene* s, const rt_render_params* p, uint8_t* out_rgb8,
                   rt_progress_fn progress, void* user, rt_counters* counters);

/* Same, with outputs in device memory (either may be NULL): out_rgb_dev (n_rows*W*3
 * doubles) and out_rgb8_dev (n_rows*W*3 bytes, writers.cpp:4-9 quantisation fused).
 * `stream` is a hipStream_t; NULL = the scene's own non-blocking stream.  The call returns
 * when the work on the stream is complete. */
int rt_render_device(rt_scene* s, const rt_render_params* p, double* out_rgb_dev,
                     uint8_t* out_rgb8_dev, void* stream, rt_counters* counters);

/* A batch of n renders of the scene (params[k] -> out_rgb_dev[k], out_rgb8_dev[k]; either
 * array, or any entry, may be NULL), each equal to its own rt_render_device call.  Up to
 * RTAMD_BATCH_LANES (default 3) images are traced concurrently, so one image's
 * latency-bound deep reflection levels overlap the next image's wide first levels
 * (frame pipelining for throughput; the reference renders one image per renderScene).
 * intersection_only entries are rendered one at a time.  counters: sums over the batch. */
int rt_render_batch_device(rt_scene* s, int n, const rt_render_params* params,
                           double* const* out_rgb_dev, uint8_t* const* out_rgb8_dev,
                           void* stream, rt_counters* counters);

/* In-place scale of a device f64 image by 1/max (the --intersection-only tail of
 * scene.cpp:56, Color3d /= scalar == multiply by the reciprocal) + optional rgb8. */
int rt_normalize_device(rt_scene* s, double* rgb_dev, int64_t n_pixels, double max_value,
                        uint8_t* out_rgb8_dev, void* stream);

/* The multi-GPU row partition (rtamd_multi.h, rtamd/dist.py): with blocks of row_block
 * rows interleaved over n_devices, image row `row` is rendered by device *device as its
 * *local_row-th selected row, i.e. by rt_render_params {device * row_block, H, n_devices,
 * row_block} (the reference's block dispenser, scene.cpp:13-48, at GPU granularity). */
void rt_partition_row(int64_t row, int n_devices, int row_block, int* device, int64_t* local_row);

/* ---------------------------------------------------------------- output */
/* writers.cpp:4-9: clamp to [0,1], *255, truncate (NaN -> 0). */
void rt_to_rgb8(const double* rgb, int64_t n_pixels, uint8_t* out);
/* PNGWriter::writeImage (writers.cpp:11-21) byte for byte: libpng 1.6.13 simplified
 * write of 8-bit RGB, sRGB chunk, libpng's filter heuristic, zlib level 6 Z_FILTERED. */
int rt_write_png(const char* path, const uint8_t* rgb, int width, int height);

/* ---------------------------------------------------------------- diagnostics */
const char* rt_last_error(void);
const char* rt_version(void);
int rt_device_count(void);
/* Device math self-test: out[i] = pow(x[i], y[i]), sqrt(x[i]), x[i]/y[i] computed by the
 * kernels' own device routines (op 0 = pow, 1 = sqrt, 2 = div) for host comparison. */
int rt_selftest_math(int device, int op, const double* x, const double* y, double* out, int64_t n);

#ifdef __cplusplus
}
#endif
#endif /* RTAMD_H */
