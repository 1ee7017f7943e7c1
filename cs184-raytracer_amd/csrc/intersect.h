// Device-side intersection code of the hot path (included by trace.hip only).
//
// Numerics: binary64, -ffp-contract=off, every expression in the reference's Eigen 3.2.2
// evaluation order:
//   Vector4d dot   (a0 b0 + a2 b2) + (a1 b1 + a3 b3); for directions/normals the w products
//                  are exact zeros and are dropped (dot4z, sq4)
//   Vector3d norm  a0^2 + (a1^2 + a2^2)
//   T * v          rows sequential ((m0 v0 + m1 v1) + m2 v2) + m3 v3
//   invT * n       (M0k n0 + M2k n2) + (M1k n1 + M3k n3)
//   normalized()   division by the norm; normalize() multiplies by the reciprocal
//
// Acceleration (new design, exact): LBVH per mesh, world-space boxes per geometry, and
// conservative pre-tests that only ever skip work whose outcome is already decided.
#pragma once
#ifndef RT_PHASE_PROF
#define RT_PHASE_PROF 0
#endif
// Diagnostic builds only (tools/valu_breakdown.sh; the images are WRONG): skip a part of the
// packet kernels to measure its share of the vector instructions.  bit 0: the packet LBVH
// searches find nothing; bit 1: packet face tests skipped (node walk only); bit 2:
// occluded_packet decides nothing (returns false after the may-raise check).
#ifndef RT_DIAG_SKIP
#define RT_DIAG_SKIP 0
#endif
#include <hip/hip_runtime.h>
#include <cmath>
#include "device_types.h"
#include "trace.h"

namespace rtamd {
namespace dev {

// What the traversal kernels are instantiated for (template parameter kMesh, chosen on the
// host from the scene's content): spheres only, meshes all scanned face by face (no LBVH:
// a mesh of fewer faces than bvh.cpp's threshold, e.g. refraction3's floor triangle), or
// meshes with LBVHs.  Without the LBVH searches the kernels hold fewer registers.
constexpr int kMeshNone = 0, kMeshLinear = 1, kMeshBvh = 2;

#ifndef RT_BLOCK
#define RT_BLOCK 128
#endif
constexpr int kBlock = RT_BLOCK;  // threads per traversal block (2 waves); LDS stack = kStackDepth x kBlock x 4 B


// Scene data read at a wave-uniform address goes through the constant address space so
// it is fetched with scalar (SMEM) loads into SGPRs: one fetch per wave, no VGPRs.
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(4))) T* uniform_ptr(const T* p) {
	return (const __attribute__((address_space(4))) T*)(p);
}
// A pointer the compiler cannot see through at this point of the program: loads through it
// cannot be hoisted above here (e.g. out of a kernel's grid-stride loop, where the loaded
// values would occupy scalar registers for the whole kernel and spill).
template <typename T>
__device__ __forceinline__ const T* opaque(const T* p) {
	asm volatile("" : "+s"(p));
	return p;
}
template <bool kUniform, typename T>
__device__ __forceinline__ auto scene_ptr(const T* p) {
	if constexpr (kUniform)
		return uniform_ptr(p);
	else
		return p;
}

struct V3 {
	double x, y, z;
};
__device__ __forceinline__ V3 mk(double x, double y, double z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator-(V3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ V3 operator*(double s, V3 a) { return mk(s * a.x, s * a.y, s * a.z); }
template <typename P>
__device__ __forceinline__ V3 load3(P p) { return mk(p[0], p[1], p[2]); }

// Vector4d::dot of two vectors whose w is (+-)0: the w term contributes an exact zero
__device__ __forceinline__ double dot4z(V3 a, V3 b) { return (a.x * b.x + a.z * b.z) + a.y * b.y; }
// Vector4d::squaredNorm with w == 0: exact (y^2 + 0 == y^2)
__device__ __forceinline__ double sq4(V3 a) { return (a.x * a.x + a.z * a.z) + a.y * a.y; }
// isZero(): all |c| <= 1e-12 (w is zero)
__device__ __forceinline__ bool is_zero3(V3 a) { return fabs(a.x) <= 1e-12 && fabs(a.y) <= 1e-12 && fabs(a.z) <= 1e-12; }
__device__ __forceinline__ V3 div3(V3 a, double n) { return mk(a.x / n, a.y / n, a.z / n); }
// a.normalized() = a / |a| (Eigen divides by the norm): sqrt of ((x^2 + z^2) + y^2), then
// three quotients sharing the divisor
__device__ __forceinline__ V3 normalized3(V3 a, double* norm = nullptr) {
	const double n = sqrt((a.x * a.x + a.z * a.z) + a.y * a.y);  // sq4 (w == 0)
	if (norm) *norm = n;
	return div3(a, n);
}

template <typename M>
__device__ __forceinline__ V3 xf_point(M m, V3 p) {
	return mk(((m[0][0] * p.x + m[0][1] * p.y) + m[0][2] * p.z) + m[0][3],
	          ((m[1][0] * p.x + m[1][1] * p.y) + m[1][2] * p.z) + m[1][3],
	          ((m[2][0] * p.x + m[2][1] * p.y) + m[2][2] * p.z) + m[2][3]);
}
template <typename M>
__device__ __forceinline__ V3 xf_dir(M m, V3 d) {
	return mk((m[0][0] * d.x + m[0][1] * d.y) + m[0][2] * d.z, (m[1][0] * d.x + m[1][1] * d.y) + m[1][2] * d.z,
	          (m[2][0] * d.x + m[2][1] * d.y) + m[2][2] * d.z);
}
// inverseTransform().matrix().transpose() * n (geometry.cpp:40)
template <typename M>
__device__ __forceinline__ V3 xf_normal(M m, V3 n) {
	return mk((m[0][0] * n.x + m[2][0] * n.z) + m[1][0] * n.y, (m[0][1] * n.x + m[2][1] * n.z) + m[1][1] * n.y,
	          (m[0][2] * n.x + m[2][2] * n.z) + m[1][2] * n.y);
}

__device__ __forceinline__ void raise_error(DeviceCounters* c, int code) { atomicCAS(&c->error, 0, code); }

// Ray::direction(dir) (rtbase.h:17-23): reject |c| <= 1e-12, then dir.normalized()
__device__ __forceinline__ V3 ray_dir(V3 d, DeviceCounters* c) {
	if (is_zero3(d)) raise_error(c, DERR_NO_DIRECTION);
	return normalized3(d);
}

// Matrix3d::determinant of the matrix with columns c0, c1, c2 (LU/Determinant.h:61-69)
__device__ __forceinline__ double det3(V3 c0, V3 c1, V3 c2) {
	return (c0.x * (c1.y * c2.z - c2.y * c1.z) - c1.x * (c0.y * c2.z - c2.y * c0.z)) + c2.x * (c0.y * c1.z - c1.y * c0.z);
}

// hitsBoundingBox, verbatim (geometry.cpp:5-29)
template <typename P>
__device__ bool hits_bounding_box(V3 o, V3 d, P mn, P mx) {
	const double oa[3] = {o.x, o.y, o.z}, da[3] = {d.x, d.y, d.z};
#pragma unroll
	for (int axis = 0; axis < 3; axis++) {
#pragma unroll
		for (int bn = 0; bn < 2; bn++) {
			const double mag = da[axis];
			if (mag == 0.0) continue;
			const double t = ((bn ? mx : mn)[axis] - oa[axis]) / mag;
			if (t < 0) continue;
			bool inside = true;
#pragma unroll
			for (int a2 = 0; a2 < 3; a2++) {
				if (a2 == axis) continue;
				const double p = oa[a2] + t * da[a2];
				if (p < mn[a2] || p > mx[a2]) inside = false;
			}
			if (inside) return true;
		}
	}
	return false;
}

// Per-lane work counters (algorithmic bytes/flops of the roofline), counted
// only by the kernels instantiated with kCount (rt_render_params::work_stats): counting
// costs 6% of the traversal kernels' time, so renders that do not ask for
// the counts run kernels without them (WorkStats<false>: every member a no-op, reads 0).
// The counters live in the block's LDS, one slot per lane, bumped with ds_add (fewer VGPRs in
// the traversal loops, where every VGPR counts).
enum WorkCounter : int { W_NODES = 0, W_TRIS, W_CANDS, W_SPHERES, W_ENTRIES, W_COUNT };
template <bool kCount>
struct WorkStats {
	static constexpr bool kOn = kCount;
	uint32_t* c;  // this lane's counters: c[k * kBlock]
	__device__ __forceinline__ void init(uint32_t* lds) {
		if constexpr (kCount) {
			c = lds + threadIdx.x;
#pragma unroll
			for (int k = 0; k < W_COUNT; k++) c[k * kBlock] = 0;
		}
	}
	__device__ __forceinline__ void inc(int k) {
		if constexpr (kCount) atomicAdd(c + k * kBlock, 1u);
	}
	// counts a lane where b (the packet loops: every lane adds 0 or 1, no exec-mask
	// save/restore around the LDS atomic)
	__device__ __forceinline__ void add(int k, bool b) {
		if constexpr (kCount) atomicAdd(c + k * kBlock, static_cast<uint32_t>(b));
	}
	__device__ __forceinline__ uint32_t get(int k) const {
		if constexpr (kCount) return c[k * kBlock];
		return 0;
	}
#if RT_PHASE_PROF
	uint32_t ph[kPhaseSlots];  // shader-clock cycles per phase while this lane was active
#endif
};

// Phase profile (diagnostic builds, -DRT_PHASE_PROF=1): the wave's shader clock
// (s_memtime) around code regions, summed per lane.
enum PhaseSlot : int { PH_TOTAL = 0, PH_NODES, PH_FACES, PH_XFORM, PH_SPHERE, PH_WORLD, PH_SETUP, PH_GATE };
#if RT_PHASE_PROF
__device__ __forceinline__ uint32_t prof_t() {
	__builtin_amdgcn_sched_barrier(0);  // no instruction scheduled across the clock read
	const uint32_t t = static_cast<uint32_t>(__builtin_amdgcn_s_memtime());
	__builtin_amdgcn_sched_barrier(0);
	return t;
}
#define PROF_T() prof_t()
#define PROF_BEGIN(v) const uint32_t v = PROF_T()
#define PROF_END(ws, k, v) ((ws).ph[k] += PROF_T() - (v))
#else
#define PROF_BEGIN(v)
#define PROF_END(ws, k, v) ((void)0)
#endif

#ifndef RT_DIAG_LANES
#define RT_DIAG_LANES 0
#endif
// RT_DIAG_GEOMS (diagnostic build): per shadow-order position k, [2k] 64 x the packet
// shadow waves with a candidate lane there, [2k + 1] the candidate lanes
#ifndef RT_DIAG_GEOMS
#define RT_DIAG_GEOMS 0
#endif
// RT_DIAG_PACKET (diagnostic build, tools/packet_census.py): wave events of the packet
// searches, [2k] 64 x the waves, [2k + 1] the lanes taking part; k (PacketSlot): shadow
// (kAnyHit) node iterations, face tests and the stages of the predicated face test a wave
// gets through, LBVH entries, geometries entered, light verdicts; then the closest-hit ones
#ifndef RT_DIAG_PACKET
#define RT_DIAG_PACKET 0
#endif
enum PacketSlot : int {
	PK_NODE = 0, PK_FACE, PK_FACE_FACING, PK_FACE_DA, PK_FACE_DB, PK_FACE_DT, PK_FACE_CAND, PK_BVH, PK_GEOM, PK_LIGHT,
	PK_C_NODE, PK_C_FACE, PK_C_CAND, PK_C_BVH, PK_C_GEOM, PK_C_ITEM
};
#if RT_DIAG_PACKET
#define DIAG_PK(k, p) diag_lanes(2 * (k), (p))
#else
#define DIAG_PK(k, p) ((void)0)
#endif
#if RT_PHASE_PROF || RT_DIAG_LANES || RT_DIAG_GEOMS || RT_DIAG_PACKET
// RT_PHASE_PROF: [stage * 2 + packet][slot] shader cycles; RT_DIAG_LANES (diagnostic build):
// lane occupancy of the per-lane kernels, read by tools/lane_census.py
__device__ unsigned long long g_phase[4 * kPhaseSlots];
__device__ __forceinline__ void diag_lanes(int slot, bool p) {
	const unsigned long long m = __ballot(p);
	if (__lane_id() == __builtin_amdgcn_readfirstlane(__lane_id())) {
		atomicAdd(&g_phase[slot], 64ull);
		atomicAdd(&g_phase[slot + 1], (unsigned long long)__popcll(m));
	}
}
// [slot] 64 x the wave events, [slot + 1] 64 x those in which some lane has p
__device__ __forceinline__ void diag_any(int slot, bool p) {
	const unsigned long long m = __ballot(p);
	if (__lane_id() == __builtin_amdgcn_readfirstlane(__lane_id())) {
		atomicAdd(&g_phase[slot], 64ull);
		if (m) atomicAdd(&g_phase[slot + 1], 64ull);
	}
}
#endif

// RT_DIAG_WAVETIME (diagnostic build, tools/wave_times.py): every wave's item of the
// traversal launches (k_closest, k_fused, k_shadow) as one record: its start and end on the
// 100 MHz real-time clock, the kernel, level and first item, and the packet node iterations and
// face tests the wave made for it (counted per hardware wave slot: HW_ID and XCC_ID)
#ifndef RT_DIAG_WAVETIME
#define RT_DIAG_WAVETIME 0
#endif
#if RT_DIAG_WAVETIME
struct WaveTime {
	unsigned long long t0, t1;
	uint32_t tag;   // kernel (1 k_closest, 2 k_fused, 3 k_shadow) | packet << 4 | level << 8
	uint32_t item;  // the wave's first item
	uint32_t nodes, faces;
};
constexpr int kWaveTimes = 1 << 18;
__device__ WaveTime g_wt[kWaveTimes];
__device__ unsigned int g_wt_n;
__device__ uint32_t g_wt_slot[8 << 16][2];
__device__ __forceinline__ uint32_t wt_slot() {
	const uint32_t hw = __builtin_amdgcn_s_getreg((15 << 11) | 4);       // HW_ID[15:0]: wave, SIMD, CU, SH, SE
	const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7;  // XCC_ID[3:0]
	return (xcc << 16) | hw;
}
__device__ __forceinline__ void wt_count(int k) {
	if (__lane_id() == __builtin_amdgcn_readfirstlane(__lane_id())) g_wt_slot[wt_slot()][k]++;
}
__device__ __forceinline__ void wt_end(unsigned long long t0, uint32_t tag, int64_t item) {
	const unsigned long long t1 = wall_clock64();
	if (__lane_id() == __builtin_amdgcn_readfirstlane(__lane_id())) {
		uint32_t* c = g_wt_slot[wt_slot()];
		const uint32_t i = atomicAdd(&g_wt_n, 1u);
		if (i < kWaveTimes) g_wt[i] = WaveTime{t0, t1, tag, static_cast<uint32_t>(item), c[0], c[1]};
		c[0] = c[1] = 0;
	}
}
#define DIAG_WT(k) wt_count(k)
#define WT_BEGIN() const unsigned long long wt_t0 = wall_clock64()
#define WT_END(tag, item) wt_end(wt_t0, (tag), (item))
#else
#define DIAG_WT(k) ((void)0)
#define WT_BEGIN() ((void)0)
#define WT_END(tag, item) ((void)0)
#endif

// A mesh hit (face, barycentric a, b), or a sphere hit (face -1, ray parameter t in a)
struct FaceHit {
	int32_t face;
	double a, b;
};

struct MeshBest {
	double dist;
	int32_t face;   // global face index, -1 = none
	int32_t id;     // reference order within the mesh (tie-break)
	double a, b;    // barycentrics of the best face; its normal is interpolated again at the end
};

// Interpolated normal ((1 - a - b) n0 + a n1) + b n2 of face f (geometry.cpp:117-119)
template <bool kUniform = false>
__device__ __forceinline__ V3 face_normal(const DeviceScene& S, int32_t f, double a, double b) {
	const auto N = scene_ptr<kUniform>(S.fnrm) + f;
	const double w0 = (1.0 - a) - b;
	const V3 n0 = load3(N->n0), n1 = load3(N->n1), n2 = load3(N->n2);
	return mk((w0 * n0.x + a * n1.x) + b * n2.x, (w0 * n0.y + a * n1.y) + b * n2.y, (w0 * n0.z + a * n1.z) + b * n2.z);
}

// Exact pre-tests on q = num / den (den != 0): true only when the correctly rounded
// quotient certainly satisfies the predicate, so skipping the division cannot change a
// decision.  2^-1000 keeps clear of an underflow of the quotient to -0.
__device__ __forceinline__ bool quotient_surely_negative(double num, double den) {
	return ((num < 0) != (den < 0)) && fabs(num) > fabs(den) * 0x1p-1000;
}
// |num| > |den| * lim * 1.001 (same signs) implies fl(num / den) > lim; the threshold must
// be a normal number so that its own rounding stays below the 0.1% slack (lim >= 2^-900).
__device__ __forceinline__ bool quotient_surely_above(double num, double den, double lim) {
	const double thr = fabs(den) * (lim * 1.001);
	return ((num < 0) == (den < 0)) && thr >= 0x1p-1000 && fabs(num) > thr;
}

// ------------------------------------------------------------- facing pre-tests (exact)
// The reference accepts a face only if its interpolated normal tn = (w0 n0 + a n1) + b n2
// (w0 = (1 - a) - b, a, b in [0, 1]) passes the facing test `!front ^ reverse` with
// front = dot(tn, d) < 0 (geometry.cpp:117-122), after the whole Cramer test.  When
// dot(n_i, d) has one sign, with a margin, for all three vertex normals, so has dot(tn, d)
// (a convex combination; its rounding errs by ~10 ulp of sum w_i |n_i| |d|, far below the
// margins), and the facing test's outcome is known before any of the face's fp64 work.
// NaN or infinite barycentrics never reach acceptance (t and the distance are then NaN or
// infinite and fail the distance test), so only finite a, b matter.

// True when the facing test certainly rejects face F for the object-space unit direction d
// (|d| within 1e-15 of 1): every vertex normal lies within r of the fp32 vector c, so
// dot(n_i, d) lies within r of dot(c, d); the fp32 dot product of c with d rounded to fp32
// errs by < 5e-7 |c|_1, and tau = r + 2 (1e-5 max |n_i|_1 + 1e-6 |c|_1) (bvh.cpp
// facing_data) leaves every dot(n_i, d) beyond 1e-5 |n_i|_1 with the sign of dot(c, d).
// tau = +inf disables the face's test, a NaN compares false: never a rejection.
__device__ __forceinline__ float facing_dot(float c0, float c1, float c2, V3 d) {
	return fmaf(c2, static_cast<float>(d.z), fmaf(c1, static_cast<float>(d.y), c0 * static_cast<float>(d.x)));
}
__device__ __forceinline__ bool facing_rejects(float c0, float c1, float c2, float tau, V3 d, bool reverse) {
	const float s = facing_dot(c0, c1, c2, d);
	// s > tau: front false, rejected unless reverse; s < -tau: front true, rejected if reverse
	return reverse ? s < -tau : s > tau;
}
template <typename FP>
__device__ __forceinline__ bool face_facing_rejects(FP F, V3 d, bool reverse) {
	return facing_rejects(F->cone_c[0], F->cone_c[1], F->cone_c[2], F->cone_tau, d, reverse);
}
// One iteration of the face loop of geometry.cpp:78-124.  Accepts the face when it is
// strictly closer, or equally close with a smaller reference index: over any visiting
// order this selects the same face as the reference's in-order scan.
// Returns true when kAnyHit and the face passes (the caller's question is answered).
// Per lane (the packet traversal uses test_face_pred): the vertices are fetched only for
// faces the facing pre-test keeps.
template <bool kAnyHit, typename WS>
__device__ __forceinline__ bool test_face(const DeviceScene& S, int32_t f, V3 o, V3 d, V3 nd, double dn, bool reverse,
                                          double any_limit, MeshBest& best, WS& ws) {
	ws.inc(W_TRIS);
#if RT_DIAG_LANES
	diag_lanes(kAnyHit ? 12 : 14, true);  // [12]/[14] per-lane face tests (shadow/closest): wave slots, lanes
#endif
	const DFaceGeo* F = S.fgeo + f;
	if (face_facing_rejects(F, d, reverse)) return false;
	const V3 p0 = load3(F->p0), va = load3(F->va), vb = load3(F->vb);
	// id is fetched with the vertices: the compiler would otherwise issue its load where it is
	// first used (one more memory round trip per candidate face)
	const int32_t id = F->id;
	asm volatile("" ::"v"(id));
	const V3 rhs = o - p0;
	const double D = det3(va, vb, nd);
	if (D == 0) return false;
	const double Da = det3(rhs, vb, nd);
	if (quotient_surely_negative(Da, D) || quotient_surely_above(Da, D, 1.0)) return false;
	const double a = Da / D;
	if (a < 0 || a > 1) return false;
	const double Db = det3(va, rhs, nd);
	if (quotient_surely_negative(Db, D) || quotient_surely_above(Db, D, 1.0)) return false;
	const double b = Db / D;
	if (b < 0 || a + b > 1) return false;
	const double Dt = det3(va, vb, rhs);
	if (quotient_surely_negative(Dt, D)) return false;
	// dist = t * dn with dn = |d|_3 within a few ulps of 1: t > 1.001 * best * 1.001 cannot win
	if (best.dist < INFINITY && best.dist >= 0x1p-900 && quotient_surely_above(Dt, D, best.dist * 1.001)) return false;
	const double t = Dt / D;
	if (t < 0) return false;
	const double dist = t * dn;
	if (!(dist < best.dist || (dist == best.dist && id < best.id))) return false;
	ws.inc(W_CANDS);
	const V3 tn = face_normal(S, f, a, b);
	const bool front = dot4z(tn, d) < 0;
	if (!front ^ reverse) return false;
	best.dist = dist;
	best.face = f;
	best.id = id;
	best.a = a;
	best.b = b;
	return kAnyHit && dist < any_limit;
}

// The wave-packet form of test_face: the same decisions, but each lane's early exits
// become a running predicate and the wave leaves only when no lane is left (a wave-uniform
// branch).  The branchy form pays exec-mask bookkeeping (s_and_saveexec, s_cbranch_execz,
// the join) at every exit of every face test, in a kernel whose instruction stream is as
// much scalar as vector; here a lane that has failed just computes along, its results never
// selected.  The predicates combine with `&` (evaluated, never branched on: `&&` over an
// expensive right-hand side compiles to an exec-mask branch and a bool round trip through a
// VGPR), and the lanes taking part come and go as a wave mask (a scalar), not as a per-lane
// bool carried through the traversal loop (an i1 loop value costs exec-mask merges on every
// iteration).  Divisions of failed lanes may see D = 0 (inf/NaN, discarded).  The range
// tests keep the reference's form (geometry.cpp:93-106: a NaN a, b or t is not rejected).
// on: the lanes testing the face.  Returns the lanes for which kAnyHit && the face passes
// within any_limit (their question is answered).
__device__ __forceinline__ bool wave_any(bool p) { return __ballot(p) != 0; }
__device__ __forceinline__ bool lane_in(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }
// The lanes where a comparison holds.  A ballot of one comparison is the comparison's own
// result mask (v_cmp into an SGPR pair); a ballot of a combined bool costs a select and a
// compare to rebuild the mask, so predicates are combined as masks (s_and / s_xor).
#define BAL(c) static_cast<uint64_t>(__ballot(c))
// quotient_surely_negative / _above as lane masks (all lanes of the wave call them)
__device__ __forceinline__ uint64_t quotient_surely_negative_m(double num, double den) {
	return (BAL(num < 0) ^ BAL(den < 0)) & BAL(fabs(num) > fabs(den) * 0x1p-1000);
}
__device__ __forceinline__ uint64_t quotient_surely_above_m(double num, double den, double lim) {
	const double thr = fabs(den) * (lim * 1.001);
	return ~(BAL(num < 0) ^ BAL(den < 0)) & BAL(thr >= 0x1p-1000) & BAL(fabs(num) > thr);
}
template <bool kAnyHit, typename WS>
__device__ __forceinline__ uint64_t test_face_pred(const DeviceScene& S, int32_t f, V3 o, V3 d, V3 nd, double dn,
                                                   bool reverse, double any_limit, MeshBest& best, WS& ws,
                                                   uint64_t on) {
	ws.add(W_TRIS, lane_in(on));
	DIAG_WT(1);
	const auto F = uniform_ptr(S.fgeo) + f;
	const V3 p0 = load3(F->p0), va = load3(F->va), vb = load3(F->vb);
	const int32_t id = F->id;
	const float c0 = F->cone_c[0], c1 = F->cone_c[1], c2 = F->cone_c[2], tau = F->cone_tau;
	asm volatile("" ::"s"(p0.x), "s"(p0.y), "s"(p0.z), "s"(va.x), "s"(va.y), "s"(va.z), "s"(vb.x), "s"(vb.y),
	             "s"(vb.z), "s"(id), "s"(c0), "s"(c1), "s"(c2), "s"(tau));
	const float sf = facing_dot(c0, c1, c2, d);
	const uint64_t rev = BAL(reverse);  // (loop-invariant)
	uint64_t ok = on & ~((BAL(sf < -tau) & rev) | (BAL(sf > tau) & ~rev));
	DIAG_PK(kAnyHit ? PK_FACE : PK_C_FACE, lane_in(on));
	if (!ok) return 0;
	if (kAnyHit) DIAG_PK(PK_FACE_FACING, lane_in(ok));
	const V3 rhs = o - p0;
	const double D = det3(va, vb, nd);
	const double Da = det3(rhs, vb, nd);
	ok &= BAL(D != 0) & ~quotient_surely_negative_m(Da, D) & ~quotient_surely_above_m(Da, D, 1.0);
	if (!ok) return 0;
	if (kAnyHit) DIAG_PK(PK_FACE_DA, lane_in(ok));
	const double a = Da / D;
	const double Db = det3(va, rhs, nd);
	ok &= ~BAL(a < 0) & ~BAL(a > 1) & ~quotient_surely_negative_m(Db, D) & ~quotient_surely_above_m(Db, D, 1.0);
	if (!ok) return 0;
	if (kAnyHit) DIAG_PK(PK_FACE_DB, lane_in(ok));
	const double b = Db / D;
	const double Dt = det3(va, vb, rhs);
	// dist = t * dn with dn = |d|_3 within a few ulps of 1: t > 1.001 * best * 1.001 cannot win
	const uint64_t beyond =
	    BAL(best.dist < INFINITY) & BAL(best.dist >= 0x1p-900) & quotient_surely_above_m(Dt, D, best.dist * 1.001);
	ok &= ~BAL(b < 0) & ~BAL(a + b > 1) & ~quotient_surely_negative_m(Dt, D) & ~beyond;
	if (!ok) return 0;
	if (kAnyHit) DIAG_PK(PK_FACE_DT, lane_in(ok));
	const double t = Dt / D;
	const double dist = t * dn;
	ok &= ~BAL(t < 0) & (BAL(dist < best.dist) | (BAL(dist == best.dist) & BAL(id < best.id)));
	if (!ok) return 0;
	DIAG_PK(kAnyHit ? PK_FACE_CAND : PK_C_CAND, lane_in(ok));
	ws.add(W_CANDS, lane_in(ok));
	const V3 tn = face_normal<true>(S, f, a, b);
	// the reference's facing test !(!front ^ reverse) == front ^ reverse, front = dot(tn, d) < 0
	ok &= BAL(dot4z(tn, d) < 0) ^ BAL(reverse);
	if (lane_in(ok)) {
		best.dist = dist;
		best.face = f;
		best.id = id;
		best.a = a;
		best.b = b;
	}
	return kAnyHit ? ok & BAL(dist < any_limit) : 0;
}

// Slab test of a padded box; conservative: the interval is widened by a relative 1e-9.
template <typename P>
__device__ __forceinline__ bool slab(P lo, P hi, V3 o, V3 inv, double tlimit, double& tnear) {
	const double tx0 = (lo[0] - o.x) * inv.x, tx1 = (hi[0] - o.x) * inv.x;
	const double ty0 = (lo[1] - o.y) * inv.y, ty1 = (hi[1] - o.y) * inv.y;
	const double tz0 = (lo[2] - o.z) * inv.z, tz1 = (hi[2] - o.z) * inv.z;
	double tmin = fmax(fmax(fmin(tx0, tx1), fmin(ty0, ty1)), fmin(tz0, tz1));
	double tmax = fmin(fmin(fmax(tx0, tx1), fmax(ty0, ty1)), fmax(tz0, tz1));
	tmin -= 1e-9 * fabs(tmin);
	tmax += 1e-9 * fabs(tmax);
	tnear = tmin;
	return tmax >= tmin && tmax >= 0.0 && tmin <= tlimit;
}

// 1/x for the slab tests only (conservative, never part of a result): v_rcp_f64 refined by
// two Newton steps, relative error far below the slabs' 1e-9 widening.  |x| is clamped to
// >= 1e-300, so the operand and the result are normal numbers.
__device__ __forceinline__ double slab_rcp(double x) {
const double a = fabs(x) < 1e-300 ? copysign(1e-300, x) : x;
double r = __builtin_amdgcn_rcp(a);
r = fma(r, fma(-a, r, 1.0), r);
return fma(r, fma(-a, r, 1.0), r);
}
__device__ __forceinline__ V3 safe_inv(V3 d) { return mk(slab_rcp(d.x), slab_rcp(d.y), slab_rcp(d.z)); }

__device__ __forceinline__ double prune_limit(double best_dist) { return best_dist * (1.0 + 4e-9); }

// Per axis a, the computed plane parameter fma(lo, I, -fl(o' I)) errs from (lo - o') / d_a by
// at most 2^-23 |I| |o'_a| + 2^-23 |t| <= 1.5 * 2^-22 amax |I| (|o'_a|, |lo| <= amax, so
// |t| <= 2 amax |I|), while a face point inside the unpadded child box lies >= 2^-18 amax |I|
// in t from each padded plane: the test keeps every box such a point is in, with a margin
// of ten, without widening the interval (round 1's relative 2^-20 widening was dropped in
// round 2, +1.7%).
// fp32 node test.  The ray origin is first moved along the ray to where it enters the
// mesh's box (o' = o + s d, s >= 0; no face lies before it), so |o'| <= amax, the largest
// vertex coordinate magnitude; then t' = lo * I - o' * I in fp32 errs by at most about
// 6 * 2^-24 * amax in position, far inside the 2^-18 * amax the node boxes are padded by
// (bvh.cpp), and the relative 2^-22 in t' is inside it too.  A ray that
// misses the box finds no face whatever the node tests say.  |I| is clamped to 2^60:
// for a direction component below 2^-60 the clamped distances to the padded planes still
// exceed any face distance (the planes lie >= 2^-18 amax from every face).
struct Ray32 {
	float ix, iy, iz;     // I
	float oix, oiy, oiz;  // fl32(o') * I
	double s;             // the shift: t = t' + s
};
__device__ __forceinline__ float clamp_inv32(double inv) { return fminf(fmaxf(static_cast<float>(inv), -0x1p60f), 0x1p60f); }
template <typename GP>
__device__ __forceinline__ Ray32 ray32(GP G, V3 o, V3 d, V3 inv) {
	Ray32 r;
	double tb, s = 0;
	if (slab(G->bb_min, G->bb_max, o, inv, INFINITY, tb)) s = fmax(tb, 0.0);
	r.s = s;
	r.ix = clamp_inv32(inv.x);
	r.iy = clamp_inv32(inv.y);
	r.iz = clamp_inv32(inv.z);
	r.oix = static_cast<float>(o.x + s * d.x) * r.ix;
	r.oiy = static_cast<float>(o.y + s * d.y) * r.iy;
	r.oiz = static_cast<float>(o.z + s * d.z) * r.iz;
	return r;
}
// lim - s rounded up to fp32
__device__ __forceinline__ float limit32(double lim, double s) {
	const double l = lim - s;
	float f = static_cast<float>(l);
	if (static_cast<double>(f) < l) f = __uint_as_float(__float_as_uint(f) + (f > 0.0f ? 1u : (f == 0.0f ? 1u : 0xffffffffu)));
	return f;
}
// the lanes whose ray passes slab32 (packet traversal: every lane of the wave calls it)
template <typename P>
__device__ __forceinline__ uint64_t slab32_m(P lo, P hi, const Ray32& r, float lim, float& tnear) {
	const float tx0 = fmaf(lo[0], r.ix, -r.oix), tx1 = fmaf(hi[0], r.ix, -r.oix);
	const float ty0 = fmaf(lo[1], r.iy, -r.oiy), ty1 = fmaf(hi[1], r.iy, -r.oiy);
	const float tz0 = fmaf(lo[2], r.iz, -r.oiz), tz1 = fmaf(hi[2], r.iz, -r.oiz);
	const float tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1));
	const float tmax = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
	tnear = tmin;
	return static_cast<uint64_t>(__ballot(tmax >= tmin)) & static_cast<uint64_t>(__ballot(tmax >= 0.0f)) &
	       static_cast<uint64_t>(__ballot(tmin <= lim));
}
template <typename P>
__device__ __forceinline__ bool slab32(P lo, P hi, const Ray32& r, float lim, float& tnear) {
	const float tx0 = fmaf(lo[0], r.ix, -r.oix), tx1 = fmaf(hi[0], r.ix, -r.oix);
	const float ty0 = fmaf(lo[1], r.iy, -r.oiy), ty1 = fmaf(hi[1], r.iy, -r.oiy);
	const float tz0 = fmaf(lo[2], r.iz, -r.oiz), tz1 = fmaf(hi[2], r.iz, -r.oiz);
	const float tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1));
	const float tmax = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
	tnear = tmin;
	return tmax >= tmin && tmax >= 0.0f && tmin <= lim;
}


// A node record in registers: the child boxes and the child references
struct NodeRec {
	float lo[2][3], hi[2][3];
	int4 refs;  // first[0], first[1], count[0], count[1]
};
__device__ __forceinline__ void read_node(const DBvhNode* N, NodeRec& r) {
#pragma unroll
	for (int c = 0; c < 2; c++)
#pragma unroll
		for (int a = 0; a < 3; a++) {
			r.lo[c][a] = N->lo[c][a];
			r.hi[c][a] = N->hi[c][a];
		}
	r.refs = *reinterpret_cast<const int4*>(N->first);
}
__device__ __forceinline__ void fetch_node(const DeviceScene& S, int32_t ref, NodeRec& r) { read_node(S.nodes + ref, r); }

// The world cull of geometry G: its padded world box (a ray that misses it, or enters it
// beyond lim, cannot hit the geometry within lim)
template <typename GP>
__device__ __forceinline__ bool world_cull(GP G, V3 o, V3 winv, double lim) {
	double tw;
	return slab(G->wlo, G->whi, o, winv, lim, tw);
}

// Mesh::calculateIntNormInObjSpace (geometry.cpp:69-126) with an LBVH in place of the
// linear scan for large meshes.
//   kAnyHit = false: the reference's closest face (returns found, Po, No).
//   kAnyHit = true: shadow query; returns true as soon as a passing face has
//   dist < any_limit (the caller knows that settles occlusion); nodes beyond
//   prune_cap are skipped (faces there cannot decide it either).  Otherwise completes
//   like the closest-hit search restricted to dist <= prune_cap.
// The search itself, without the reference's bounding-box gate (see mesh_hit).
template <bool kAnyHit, int kMesh, typename GP, typename WS>
__device__ bool mesh_search(const DeviceScene& S, GP G, V3 o, V3 d, bool reverse, double any_limit,
                         double prune_cap, FaceHit& fh, bool& settled, double& found_dist, int32_t* stack,
                         DeviceCounters* ctr, WS& ws) {
	settled = false;
	const double dn = sqrt(d.x * d.x + (d.y * d.y + d.z * d.z));  // Vector3d::norm
	const V3 nd = -d;
	MeshBest best;
	best.dist = INFINITY;
	best.face = -1;
	best.id = 0x7fffffff;
	if (kMesh < kMeshBvh || G->bvh_root < 0) {
		PROF_BEGIN(tf);
		for (int32_t f = G->face_begin; f < G->face_begin + G->face_count; f++)
			if (test_face<kAnyHit>(S, f, o, d, nd, dn, reverse, any_limit, best, ws)) {
				PROF_END(ws, PH_FACES, tf);
				settled = true;
				return true;
			}
		PROF_END(ws, PH_FACES, tf);
	} else {
		// while-while traversal (Aila & Laine 2009): a lane first walks inner nodes until
		// it holds a leaf, then the lanes holding leaves test their faces together, so
		// node and face work do not interleave within a wave.  `ref` >= 0 is a node,
		// <= -2 a leaf (face offset << 3 | count), -1 done.  The far child of a node whose
		// two children are hit is pushed (LDS stack, kStackDepth entries per lane).
		ws.inc(W_ENTRIES);
#if RT_DIAG_LANES
		diag_lanes(kAnyHit ? 24 : 8, true);  // wave slots and lanes entering a per-lane LBVH search
#endif
		const V3 inv = safe_inv(d);
		const Ray32 r32 = ray32(G, o, d, inv);
		// the node-pruning limit in the shifted fp32 frame; it changes only with best.dist
		float lim = limit32(fmin(prune_limit(best.dist), prune_cap), r32.s);
		int32_t ref = G->bvh_root;
		int sp = 0;
		auto pop = [&]() { return sp > 0 ? stack[--sp * kBlock] : (int32_t)-1; };
		// Speculative (Aila & Laine 2009): a lane that reaches a leaf while other lanes are
		// still walking inner nodes postpones it (`leaf`) and keeps walking, so fewer lanes
		// idle in either phase.  Any visiting order selects the same face (test_face).
		int32_t leaf = -1;
		while (ref != -1 || leaf != -1) {
			PROF_BEGIN(tn);
			while (ref >= 0) {
				ws.inc(W_NODES);
				// the child references are read with the boxes (one memory round trip per node)
				NodeRec nr;
				fetch_node(S, ref, nr);
				const int4 refs = nr.refs;
				float tn0, tn1;
				const bool h0 = slab32(nr.lo[0], nr.hi[0], r32, lim, tn0);
				const bool h1 = slab32(nr.lo[1], nr.hi[1], r32, lim, tn1);
				if (h0 || h1) {
					const int c = (h0 && h1) ? (tn1 < tn0 ? 1 : 0) : (h1 ? 1 : 0);
					const int32_t cf = c ? refs.y : refs.x, cc = c ? refs.w : refs.z;
					const int32_t near_ref = cc > 0 ? -2 - ((cf << 3) | cc) : cf;
					if (h0 && h1) {
						const int32_t ff = c ? refs.x : refs.y, fc = c ? refs.z : refs.w;
						if (sp < kStackDepth) {
							stack[sp * kBlock] = fc > 0 ? -2 - ((ff << 3) | fc) : ff;
							sp++;
						} else {
							raise_error(ctr, DERR_STACK);
						}
					}
					ref = near_ref;
				} else {
					ref = pop();
				}
				if (ref <= -2 && leaf == -1) {
					leaf = ref;
					ref = pop();
				}
				if (__ballot(leaf == -1) == 0) break;  // every walking lane holds a leaf
			}
#if RT_DIAG_LANES
			diag_lanes(kAnyHit ? 26 : 10, leaf != -1);  // lanes holding a leaf when the face phase starts
#endif
			PROF_END(ws, PH_NODES, tn);
			// the postponed leaf, then a leaf the walk stopped on
			PROF_BEGIN(tf);
			while (leaf != -1) {
				const int32_t code = -2 - leaf;
				const int32_t f0 = G->face_begin + (code >> 3), f1 = f0 + (code & 7);
				for (int32_t f = f0; f < f1; f++)
					if (test_face<kAnyHit>(S, f, o, d, nd, dn, reverse, any_limit, best, ws)) {
						PROF_END(ws, PH_FACES, tf);
						settled = true;
						return true;
					}
				leaf = -1;
				if (ref <= -2) {
					leaf = ref;
					ref = pop();
				}
			}
			lim = limit32(fmin(prune_limit(best.dist), prune_cap), r32.s);
			PROF_END(ws, PH_FACES, tf);
		}
	}
	found_dist = best.dist;
	if (best.face < 0) return false;
	fh = FaceHit{best.face, best.a, best.b};
	return true;
}

// The reference tests a gated mesh only when hitsBoundingBox passes (geometry.cpp:72); the
// search has no side effects, so the gate (six divisions) is evaluated only for rays the
// search reports a hit (or occluder) for: the same outcome for fewer rays.
template <bool kAnyHit, int kMesh, typename GP, typename WS>
__device__ bool mesh_hit(const DeviceScene& S, GP G, V3 o, V3 d, bool reverse, double any_limit,
double prune_cap, FaceHit& fh, bool& settled, double& found_dist, int32_t* stack,
DeviceCounters* ctr, WS& ws) {
if (!mesh_search<kAnyHit, kMesh>(S, G, o, d, reverse, any_limit, prune_cap, fh, settled, found_dist, stack, ctr, ws))
return false;
PROF_BEGIN(tg);
const bool gate_miss = G->gate && !hits_bounding_box(o, d, G->bb_min, G->bb_max);
PROF_END(ws, PH_GATE, tg);
if (gate_miss) settled = false;
return !gate_miss;
}

// Sphere::calculateIntNormInObjSpace (geometry.cpp:47-67): the ray parameter t of the
// hit (point o + t d, normal point - center)
template <typename GP>
__device__ __forceinline__ bool sphere_hit(GP G, V3 o, V3 d, bool reverse, double& t) {
	const V3 oc = o - load3(G->center);
	const double a = sq4(d);
	const double b = 2 * dot4z(d, oc);
	const double cc = sq4(oc) - G->rr;
	const double disc = b * b - (4 * a) * cc;
	if (disc < 0) return false;
	t = reverse ? (-b + sqrt(disc)) / (2 * a) : (-b - sqrt(disc)) / (2 * a);
	return t >= 0;
}

// Object-space hit point of a mesh face (face.points_[0] + vec4dFrom3d(a * va + b * vb),
// geometry.cpp:121) or of a sphere (o + t d, t held in h.a)
__device__ __forceinline__ V3 face_point(const DeviceScene& S, const FaceHit& h) {
	const DFaceGeo* F = S.fgeo + h.face;
	const V3 p0 = load3(F->p0), va = load3(F->va), vb = load3(F->vb);
	return mk(p0.x + (h.a * va.x + h.b * vb.x), p0.y + (h.a * va.y + h.b * vb.y), p0.z + (h.a * va.z + h.b * vb.z));
}
template <int kMesh>
__device__ __forceinline__ V3 hit_point(const DeviceScene& S, const FaceHit& h, V3 oo, V3 dd) {
	return (!kMesh || h.face < 0) ? oo + h.a * dd : face_point(S, h);
}

// The closest-hit searches keep only (geometry, face, a, b) of the best hit so far; its
// world point and object-space normal are recomputed once at the end with the same
// expressions (bit-identical, fewer live registers during the traversals).
template <int kMesh>
__device__ __forceinline__ void winner_point_normal(const DeviceScene& S, int g, const FaceHit& h, V3 o, V3 d,
                                                    V3& Pw, V3& No) {
	const DGeom* G = S.geoms + g;
	V3 Po;
	if (!kMesh || h.face < 0) {
		const V3 oo = xf_point(G->inv, o);
		const V3 draw = xf_dir(G->inv, d);
		Po = oo + h.a * normalized3(draw);
		No = Po - load3(G->center);
	} else {
		Po = face_point(S, h);
		No = face_normal(S, h.face, h.a, h.b);
	}
	Pw = xf_point(G->fwd, Po);
}

// Every castRay transforms the ray into every geometry's object space, which throws for
// a vanishing direction (geometry.cpp:33, rtbase.h:17-23).  Culling and early exits skip
// geometries, so those whose transform can make a direction vanish (DGeom::may_raise,
// bvh.cpp) are checked here for every ray; for all others the check cannot fire.
__device__ __forceinline__ void check_may_raise(const DeviceScene& S, V3 d, bool on, DeviceCounters* ctr) {
	if (S.n_may_raise == 0) return;
	for (int g = 0; g < S.n_geoms; g++) {
		const auto G = uniform_ptr(S.geoms) + g;
		if (G->may_raise && on && is_zero3(xf_dir(G->inv, d))) raise_error(ctr, DERR_NO_DIRECTION);
	}
}

// Closest hit of Scene::castRay (scene.cpp:142-167): world distance, strict `<` in
// insertion order.  A geometry whose padded world box the ray misses, or enters beyond
// the current best distance, cannot be the answer and is skipped without its
// object-space transform.
// kMesh false: a scene of spheres only (DeviceScene::n_meshes == 0), instantiated without
// the mesh search (fewer registers for the sphere loop: DESIGN.md §4)
template <int kMesh, typename WS>
__device__ bool closest_hit(const DeviceScene& S, V3 o, V3 d, bool reverse, double& best_dist, int& best_geom, V3& hitP,
                            V3& hitNobj, int32_t* stack, DeviceCounters* ctr, WS& ws) {
	bool found = false;
	FaceHit best{-1, 0, 0};
	const V3 winv = safe_inv(d);
	check_may_raise(S, d, true, ctr);
	for (int g = 0; g < S.n_geoms; g++) {
		const auto G = uniform_ptr(S.geoms) + g;
		PROF_BEGIN(tw0);
		const bool wb = world_cull(G, o, winv, found ? prune_limit(best_dist) : INFINITY);
		PROF_END(ws, PH_WORLD, tw0);
#if RT_DIAG_LANES
		diag_lanes(2, true);  // [2] wave slots of the per-lane closest-hit geometry loop, [3] lanes in it
		diag_lanes(4, wb);    // [4], [5] lanes whose ray enters the geometry's world box
		diag_any(6, wb);      // [6], [7] iterations in which some lane enters it
#endif
		if (!wb) continue;
		// Geometry::calculateIntersectionNormal (geometry.cpp:31-45): object-space ray
		PROF_BEGIN(tx);
		const V3 oo = xf_point(G->inv, o);
		const V3 dd = ray_dir(xf_dir(G->inv, d), ctr);
		PROF_END(ws, PH_XFORM, tx);
		FaceHit h{-1, 0, 0};
		bool hit, settled;
		double fd;
		V3 Pw;
		if (!kMesh || G->kind == DGEOM_SPHERE) {
			ws.inc(W_SPHERES);
			PROF_BEGIN(ts);
			hit = sphere_hit(G, oo, dd, reverse, h.a);
			PROF_END(ws, PH_SPHERE, ts);
			if (!hit) continue;
			Pw = xf_point(G->fwd, oo + h.a * dd);
		} else {
			hit = mesh_hit<false, kMesh>(S, G, oo, dd, reverse, INFINITY, INFINITY, h, settled, fd, stack, ctr, ws);
			if (!hit) continue;
			Pw = xf_point(G->fwd, face_point(S, h));  // a mesh hit is a face (geometry.cpp:121)
		}
		const double dist = sqrt(sq4(Pw - o));
		if (found && dist >= best_dist) continue;
		found = true;
		best_dist = dist;
		best_geom = g;
		best = h;
	}
	if (found) winner_point_normal<kMesh>(S, best_geom, best, o, d, hitP, hitNobj);
	return found;
}

// Shadow test of scene.cpp:90-93: castRay(...) && distToOccluder <= distToLight, i.e.
// some geometry's hit (its reference-chosen face) lies within dist_light.  Meshes first
// try an any-hit search that decides the common cases exactly: a face with object-space
// t well inside the light distance occludes (the closest face is nearer still), and no
// face up to slightly beyond it means no occlusion.  Only a closest face within a
// relative 1e-7 of the light distance falls back to the reference's full comparison.
// geom_occludes: geometry G (its world box already passed) occludes the shadow ray.
template <int kMesh, typename GP, typename WS>
__device__ bool geom_occludes(const DeviceScene& S, GP G, V3 o, V3 d, bool reverse, double dist_light,
                              int32_t* stack, DeviceCounters* ctr, WS& ws) {
	const bool inf_light = dist_light == INFINITY;
	PROF_BEGIN(tx);
	const V3 oo = xf_point(G->inv, o);
	const V3 draw = xf_dir(G->inv, d);
	if (is_zero3(draw)) raise_error(ctr, DERR_NO_DIRECTION);
	double nrm;  // object-space length of the unit world direction
	const V3 dd = normalized3(draw, &nrm);
	PROF_END(ws, PH_XFORM, tx);
	FaceHit h{-1, 0, 0};
	bool hit, settled = false;
	double fd;
	if (!kMesh || G->kind == DGEOM_SPHERE) {
		ws.inc(W_SPHERES);
		PROF_BEGIN(ts);
		hit = sphere_hit(G, oo, dd, reverse, h.a);
		PROF_END(ws, PH_SPHERE, ts);
	} else if (inf_light) {
		hit = mesh_hit<true, kMesh>(S, G, oo, dd, reverse, INFINITY, INFINITY, h, settled, fd, stack, ctr, ws);
	} else {
		// world distance of object-space dist t is ~ t / nrm
		const double tl = dist_light * nrm;
		const double cap = tl * (1.0 + 1e-7) + 1e-300;
		hit = mesh_hit<true, kMesh>(S, G, oo, dd, reverse, tl * (1.0 - 1e-7), cap, h, settled, fd, stack, ctr, ws);
		// No face up to `cap` was missed by the capped search, so a closest face beyond
		// it lies beyond the light.  A closest face inside the 1e-7 band is decided
		// exactly from the reference's own face choice (full closest-face search).
		if (hit && !settled) {
			if (fd > cap) return false;
			hit = mesh_hit<false, kMesh>(S, G, oo, dd, reverse, INFINITY, INFINITY, h, settled, fd, stack, ctr, ws);
		}
	}
	if (!hit) return false;
	if (inf_light || settled) return true;
	const V3 Pw = xf_point(G->fwd, hit_point<kMesh>(S, h, oo, dd));
	return sqrt(sq4(Pw - o)) <= dist_light;
}

__device__ __forceinline__ double shadow_slab_limit(double dist_light) {
	return dist_light == INFINITY ? INFINITY : dist_light * (1.0 + 1e-6);
}

// The `any` over the geometries, cheap ones first (DeviceScene::shadow_order).
template <int kMesh, typename WS>
__device__ bool occluded(const DeviceScene& S, V3 o, V3 d, bool reverse, double dist_light, int32_t* stack,
                         DeviceCounters* ctr, WS& ws) {
	const V3 winv = safe_inv(d);
	const double lim = shadow_slab_limit(dist_light);
	check_may_raise(S, d, true, ctr);
	for (int k = 0; k < S.n_geoms; k++) {
		const int g = uniform_ptr(S.shadow_order)[k];
		const auto G = uniform_ptr(S.geoms) + g;
		PROF_BEGIN(tw0);
		const bool wb = world_cull(G, o, winv, lim);
		PROF_END(ws, PH_WORLD, tw0);
#if RT_DIAG_LANES
		diag_lanes(20, true);  // [20] wave slots of the per-lane shadow geometry loop, [21] lanes still searching
		diag_lanes(22, wb);    // [22], [23] lanes whose shadow ray enters the geometry's world box
		diag_any(30, wb);      // [30], [31] iterations in which some lane enters it
#endif
		if (wb && geom_occludes<kMesh>(S, G, o, d, reverse, dist_light, stack, ctr, ws)) return true;
	}
	return false;
}


// ---------------------------------------------------------------- wave-packet traversal
// For coherent rays (8x8 primary-ray tiles, shadow rays of such a tile towards one light)
// all 64 lanes of a wave traverse together: the wave visits the union of the nodes its
// lanes need, in one wave-uniform order (majority near-first), so node and face records
// are scalar loads (SGPRs) and the lanes never diverge on control flow.  Per-lane results
// are identical to the per-lane traversal: every lane still tests every face it would
// test there (pruning and tie-breaks are per lane), it may only test a few more.
// Callers must reach these functions with all lanes (inactive lanes pass on = false).

// A value every lane holds equally (node and face indices of the packet traversal): read
// from the first lane, so the compiler keeps it in an SGPR and the node/face records at
// that index are fetched with scalar loads instead of 64 identical vector loads.
__device__ __forceinline__ int32_t uniform_i32(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }

template <bool kAnyHit, int kMesh, typename GP, typename WS>
__device__ bool mesh_hit_packet(const DeviceScene& S, GP G, V3 o, V3 d, bool reverse, bool on, double any_limit,
                                double prune_cap, FaceHit& fh, bool& settled, double& found_dist,
                                int32_t* wstack, WS& ws) {
	const double dn = sqrt(d.x * d.x + (d.y * d.y + d.z * d.z));  // Vector3d::norm
	const V3 nd = -d;
	MeshBest best;
	best.dist = INFINITY;
	best.face = -1;
	best.id = 0x7fffffff;
	// lanes still searching, and lanes whose question a face answered (wave masks)
	uint64_t live = __ballot(on), done = 0;
	if (live) {
		if (kMesh < kMeshBvh || G->bvh_root < 0) {
			PROF_BEGIN(tf);
			for (int32_t f = G->face_begin; f < G->face_begin + G->face_count; f++) {
				const uint64_t h = test_face_pred<kAnyHit>(S, f, o, d, nd, dn, reverse, any_limit, best, ws, live);
				done |= h;
				live &= ~h;
			}
				PROF_END(ws, PH_FACES, tf);
		} else if (!(RT_DIAG_SKIP & 1)) {
			ws.add(W_ENTRIES, lane_in(live));
			DIAG_PK(kAnyHit ? PK_BVH : PK_C_BVH, lane_in(live));
			const V3 inv = safe_inv(d);
			const Ray32 r32 = ray32(G, o, d, inv);
			float lim = limit32(fmin(prune_limit(best.dist), prune_cap), r32.s);  // changes only with best.dist
			const auto nodes = uniform_ptr(S.nodes);
			const int32_t fbase = uniform_i32(G->face_begin);
			int32_t node = uniform_i32(G->bvh_root);
			int sp = 0;
			// the node record: the whole 64 B in one scalar load, both child boxes tested by
			// every lane (a lane that is done ignores its results)
			float box[2][2][3];  // [child][lo, hi][axis]
			int32_t rf0, rf1, rc0, rc1;
			auto fetch = [&](int32_t n) {
				const auto N = nodes + n;
#pragma unroll
				for (int c = 0; c < 2; c++)
#pragma unroll
					for (int a = 0; a < 3; a++) {
						box[c][0][a] = N->lo[c][a];
						box[c][1][a] = N->hi[c][a];
					}
				rf0 = N->first[0], rf1 = N->first[1], rc0 = N->count[0], rc1 = N->count[1];
			};
			fetch(node);
			// Child lane sets are wave masks (SGPRs); a lane's predicate is its bit (inverse
			// ballot, no instruction)
			for (;;) {
				PROF_BEGIN(tn);
				ws.add(W_NODES, lane_in(live));
				DIAG_PK(kAnyHit ? PK_NODE : PK_C_NODE, lane_in(live));
				DIAG_WT(0);
				float tn0 = 0, tn1 = 0;
				const uint64_t m0 = slab32_m(box[0][0], box[0][1], r32, lim, tn0) & live;
				const uint64_t m1 = slab32_m(box[1][0], box[1][1], r32, lim, tn1) & live;
				const uint64_t both = m0 & m1;
				// majority near-first: child 1 first when most lanes that need both see it nearer
				const bool first = 2 * __popcll(__ballot(tn1 < tn0) & both) > __popcll(both) || m0 == 0;
				const int32_t f_first = first ? rf1 : rf0, c_first = first ? rc1 : rc0;
				const int32_t f_second = first ? rf0 : rf1, c_second = first ? rc0 : rc1;
				const uint64_t w_first = first ? m1 : m0, w_second = first ? m0 : m1;
				PROF_END(ws, PH_NODES, tn);
				// inner children first, so the node to visit next is known (and its record
				// requested) before the leaf faces are tested: its memory round trip overlaps
				// theirs.  An inner second child keeps the node test's pruning limit (at most
				// one more node visit, never a different result).
				int32_t next = -1;
				if (w_first && c_first == 0) next = f_first;
				if (w_second && c_second == 0) {
					if (next < 0)
						next = f_second;
					else if (sp < kStackDepth)
						wstack[sp++] = f_second;  // LBVH depth <= kStackDepth - 2 (bvh.cpp)
				}
				if (next < 0 && sp > 0) next = uniform_i32(wstack[--sp]);
				if (next >= 0) fetch(next);
				// leaf children, in the same order; the second is tested again against the
				// limit the first one's faces may have lowered
				bool tested = false;
#pragma unroll
				for (int k = 0; k < 2; k++) {
					const int32_t cf = k ? f_second : f_first, cc = k ? c_second : c_first;
					if (cc <= 0 || (RT_DIAG_SKIP & 2)) continue;
					uint64_t want = (k ? w_second : w_first) & live;
					if (k == 1 && tested) want &= __ballot((first ? tn0 : tn1) <= lim);
					if (!want) continue;
					PROF_BEGIN(tf);
					const int32_t f0 = fbase + cf;
					for (int32_t f = f0; f < f0 + cc; f++) {
						const uint64_t h = test_face_pred<kAnyHit>(S, f, o, d, nd, dn, reverse, any_limit, best, ws,
						                                           want & live);
						done |= h;
						live &= ~h;
					}
					lim = limit32(fmin(prune_limit(best.dist), prune_cap), r32.s);
					tested = true;
					PROF_END(ws, PH_FACES, tf);
				}
				if (next < 0 || !live) break;
			}
		}
	}
	settled = lane_in(done);
	found_dist = best.dist;
	// the reference's gate (geometry.cpp:72), evaluated only for lanes with a result (see mesh_hit)
	bool keep = on && best.face >= 0;
	if (G->gate && wave_any(keep)) {
		PROF_BEGIN(tg);
		if (keep) keep = hits_bounding_box(o, d, G->bb_min, G->bb_max);
		PROF_END(ws, PH_GATE, tg);
		if (!keep) settled = false;
	}
	if (!keep) return false;
	fh = FaceHit{best.face, best.a, best.b};
	return true;
}

template <int kMesh, typename WS>
__device__ bool closest_hit_packet(const DeviceScene& S, V3 o, V3 d, bool reverse, bool on, double& best_dist,
                                   int& best_geom, V3& hitP, V3& hitNobj, int32_t* wstack, DeviceCounters* ctr,
                                   WS& ws) {
	bool found = false;
	FaceHit best{-1, 0, 0};
	const V3 winv = safe_inv(d);
	check_may_raise(S, d, on, ctr);
	for (int g = 0; g < S.n_geoms; g++) {
		const auto G = uniform_ptr(S.geoms) + g;
		PROF_BEGIN(tw0);
		const bool cand = on && world_cull(G, o, winv, found ? prune_limit(best_dist) : INFINITY);
		PROF_END(ws, PH_WORLD, tw0);
		if (!wave_any(cand)) continue;
		DIAG_PK(PK_C_GEOM, cand);
		PROF_BEGIN(tx);
		const V3 oo = xf_point(G->inv, o);
		const V3 draw = xf_dir(G->inv, d);
		if (cand && is_zero3(draw)) raise_error(ctr, DERR_NO_DIRECTION);
		const V3 dd = normalized3(draw);
		PROF_END(ws, PH_XFORM, tx);
		FaceHit h{-1, 0, 0};
		bool hit, settled;
		double fd;
		if (!kMesh || G->kind == DGEOM_SPHERE) {
			ws.add(W_SPHERES, cand);
			PROF_BEGIN(ts);
			hit = cand && sphere_hit(G, oo, dd, reverse, h.a);
		PROF_END(ws, PH_SPHERE, ts);
		} else {
			hit = mesh_hit_packet<false, kMesh>(S, G, oo, dd, reverse, cand, INFINITY, INFINITY, h, settled, fd, wstack, ws);
		}
		if (hit) {
			const V3 Pw = xf_point(G->fwd, hit_point<kMesh>(S, h, oo, dd));
			const double dist = sqrt(sq4(Pw - o));
			if (!(found && dist >= best_dist)) {
				found = true;
				best_dist = dist;
				best_geom = g;
				best = h;
			}
		}
	}
	if (found) winner_point_normal<kMesh>(S, best_geom, best, o, d, hitP, hitNobj);
	return found;
}

// Packet form of occluded(): same decisions per lane (see occluded()).
template <int kMesh, typename WS>
__device__ bool occluded_packet(const DeviceScene& S, V3 o, V3 d, bool reverse, double dist_light, bool on,
                                int32_t* wstack, DeviceCounters* ctr, WS& ws) {
	const bool inf_light = dist_light == INFINITY;
	const V3 winv = safe_inv(d);
	bool occ = false;
	check_may_raise(S, d, on, ctr);
	if (RT_DIAG_SKIP & 4) return false;
	for (int k = 0; k < S.n_geoms; k++) {
		const int g = uniform_ptr(S.shadow_order)[k];
		const auto G = uniform_ptr(S.geoms) + g;
		PROF_BEGIN(tw0);
		const bool cand = on && !occ && world_cull(G, o, winv, inf_light ? INFINITY : dist_light * (1.0 + 1e-6));
		PROF_END(ws, PH_WORLD, tw0);
		if (!wave_any(cand)) continue;
#if RT_DIAG_GEOMS
		if (k < 16) diag_lanes(2 * k, cand);
#endif
		DIAG_PK(PK_GEOM, cand);
		PROF_BEGIN(tx);
		const V3 oo = xf_point(G->inv, o);
		const V3 draw = xf_dir(G->inv, d);
		if (cand && is_zero3(draw)) raise_error(ctr, DERR_NO_DIRECTION);
		double nrm;
		const V3 dd = normalized3(draw, &nrm);
		PROF_END(ws, PH_XFORM, tx);
		FaceHit h{-1, 0, 0};
		bool hit, settled = false;
		double fd = INFINITY;
		if (!kMesh || G->kind == DGEOM_SPHERE) {
			ws.add(W_SPHERES, cand);
			PROF_BEGIN(ts);
			hit = cand && sphere_hit(G, oo, dd, reverse, h.a);
		PROF_END(ws, PH_SPHERE, ts);
		} else {
			const double tl = inf_light ? INFINITY : dist_light * nrm;
			const double cap = inf_light ? INFINITY : tl * (1.0 + 1e-7) + 1e-300;
			hit = mesh_hit_packet<true, kMesh>(S, G, oo, dd, reverse, cand, inf_light ? INFINITY : tl * (1.0 - 1e-7), cap, h,
			                            settled, fd, wstack, ws);
			// closest face inside the 1e-7 band around the light: the reference's exact choice
			const bool band = cand && hit && !settled && !inf_light && fd <= cap;
			if (cand && hit && !settled && !inf_light && fd > cap) hit = false;
			if (wave_any(band)) {
				bool s2;
				double fd2;
				FaceHit h2{-1, 0, 0};
				const bool hit2 = mesh_hit_packet<false, kMesh>(S, G, oo, dd, reverse, band, INFINITY, INFINITY, h2, s2, fd2,
				                                         wstack, ws);
				if (band) {
					hit = hit2;
					h = h2;
				}
			}
		}
		if (cand && hit) {
			if (inf_light || settled) {
				occ = true;
			} else {
				const V3 Pw = xf_point(G->fwd, hit_point<kMesh>(S, h, oo, dd));
				if (sqrt(sq4(Pw - o)) <= dist_light) occ = true;
			}
		}
	}
	return occ;
}

}  // namespace dev
}  // namespace rtamd
