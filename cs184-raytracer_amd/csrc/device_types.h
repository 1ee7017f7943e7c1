// Device-resident scene layout shared by the host uploader and the HIP kernels.
//
// HBM layout (all read-only after rt_scene_create):
//   DGeom[G]        per-geometry record, insertion order (scene.cpp:147 loop order)
//   DLight[L]       pre-transformed lights, definition order (scene.cpp:117)
//   DFaceGeo[F]     per face: p0, va = p1-p0, vb = p2-p0 (object space), the face's
//                   index within its mesh in the reference's order (tie-break) and its
//                   normals' cone for the facing pre-test                          96 B
//   DFaceNrm[F]     per face: n0, n1, n2 (object space, w == 0 dropped)       80 B
//   DBvhNode[N]     flattened binary LBVH, fp32 child boxes stored in the parent  64 B
// BVH meshes store their faces in LBVH leaf order; small meshes (<= kLinearFaces) keep
// the reference's order and are scanned linearly exactly like geometry.cpp:78.
#pragma once
#include <cstdint>

namespace rtamd {

enum : int32_t { DGEOM_SPHERE = 0, DGEOM_MESH = 1 };
enum : int32_t { DLIGHT_POINT = 0, DLIGHT_DIRECTIONAL = 1, DLIGHT_AMBIENT = 2 };

constexpr int kLinearFaces = 8;   // meshes up to this size are scanned linearly (no BVH)
#ifndef RT_LEAF_FACES
#define RT_LEAF_FACES 4
#endif
constexpr int kLeafFaces = RT_LEAF_FACES;  // faces per LBVH leaf
#ifndef RT_STACK_DEPTH
#define RT_STACK_DEPTH 32
#endif
constexpr int kStackDepth = RT_STACK_DEPTH;  // traversal stack entries per lane (LDS); LBVH depth <= kStackDepth - 2

struct alignas(16) DGeom {
	double fwd[3][4];     // forwardTransform rows
	double inv[3][4];     // inverseTransform rows
	double center[3];     // sphere centre (w == 1 implied)
	double rr;            // (double)(radius_ * radius_) with the product in fp32 (geometry.cpp:53)
	double bb_min[3], bb_max[3];   // Mesh bounding box (object space) for the gate
	double wlo[3], whi[3];         // padded world-space box of the geometry (culling only)
	int32_t kind;         // 0 sphere, 1 mesh
	int32_t flip;         // transformDeterminant() < 0 (geometry.cpp:42-43)
	int32_t gate;         // hitsBoundingBox gate active (geometry.cpp:72)
	int32_t bvh_root;     // root node index, -1 = linear face scan
	int32_t face_begin, face_count;
	int32_t mat;          // index into DMaterial
	// The inverse transform may map a unit direction to one the reference rejects as
	// "ray has no direction" (rtbase.h:17-23): every ray must then check this geometry,
	// even where culling or an early exit would skip it (bvh.cpp, intersect.h).
	int32_t may_raise;
};

struct alignas(16) DMaterial {   // rtbase.h:30-39
	double ka[3], kd[3], ks[3], kr[3], kt[3];
	double ns, ior;
	int32_t kt_nonzero;   // !translucencyColor.isZero()  (scene.cpp:115)
	int32_t kr_nonzero;   // !reflectiveColor.isZero()    (scene.cpp:130)
	// ns > 0 and kd, ks finite: a light whose diffuse factor max(N.L, 0) and specular base
	// max(-V.R, 0) are both zero adds exact zeros here (scene.cpp:96-106), whatever the
	// shadow ray finds (see k_shadow)
	int32_t zero_terms;
};

struct alignas(16) DLight {
	double color[3];
	double vec[3];        // point position or direction (both after the light's transform)
	double falloff;
	int32_t kind;         // 0 point, 1 directional, 2 ambient
	int32_t zero_terms;   // attenuated colour finite for every distance: directional, or point with falloff 0
};

// Facing pre-test margin, relative to |n_i|_1 (intersect.h face_facing_rejects)
constexpr double kFacingRel = 1e-5;

struct alignas(16) DFaceGeo {
	double p0[3], va[3], vb[3];
	int32_t id;           // the face's index in the reference's order within its mesh (tie-break)
	// Facing pre-test (never part of a result): the vertex normals lie within cone_r of the
	// fp32 vector cone_c; cone_tau = cone_r + margins, rounded up (+inf: no pre-test)
	float cone_tau;
	float cone_c[3];
	int32_t pad;
};
static_assert(sizeof(DFaceGeo) == 96, "face record: 96 B");

struct alignas(16) DFaceNrm {
	double n0[3], n1[3], n2[3];
	double pad;
};

// child c of a node: leaf when count[c] > 0 (faces [first[c], first[c]+count[c])),
// else inner node index first[c].  Boxes are padded outward and rounded outward to fp32
// (see bvh.cpp): one node is one 64-B half cache line.
struct alignas(64) DBvhNode {
	float lo[2][3];
	float hi[2][3];
	int32_t first[2];
	int32_t count[2];
};


struct DCamera {
	double eye[4], ll[4], lr[4], ul[4], ur[4];
};

// Device error codes -> MathException text (rtbase.h:14-22)
enum DeviceError : int32_t {
	DERR_NONE = 0,
	DERR_NO_DIRECTION = 1,      // "ray has no direction"
	DERR_POINT_DIRECTION = 2,   // "ray direction is a point vector"
	DERR_STACK = 3,             // traversal stack overflow (internal)
	DERR_ORIGIN_DIRECTION = 4,  // "ray origin is a direction vector" (camera eye with w == 0)
	DERR_PLAN = 5,              // a replayed launch plan did not fit the render (level capacity or
	                            // depth): nothing was written past a buffer, the host redoes it
	DERR_ROWS = 6,              // a chunk row descriptor names no selected row (internal; no pixel written)
};

}  // namespace rtamd
