// HIP kernels of the ray-trace hot path, gfx950 (MI355X).
//
// Wavefront formulation of the reference's recursive Scene::traceRay (scene.cpp:61-140).
// Level L holds every ray of recursion depth L; per level three launches:
//   k_closest  closest hit of every ray (castRay, scene.cpp:142-167); rays that hit are
//              appended to a hit list, their refraction/reflection children to level L+1
//              (scene.cpp:110-136), one atomic per block
//   k_shadow   one lane per (hit, non-ambient light), light-major so a wave traces rays
//              towards one light from neighbouring hits (scene.cpp:87-93)
//   k_shade    Phong terms in light order (scene.cpp:78-108), one lane per hit
// k_shadow/k_shade of level L run on a shading stream concurrently with k_closest(L+1).
// then colours are reduced bottom-up (k_reduce) in the reference's addition order:
// colour = (local + refraction) + reflection * kr (scene.cpp:127,134).
// Device arithmetic: see intersect.h; pow is glibc's (glibc_pow.h).
#include <algorithm>
#include <type_traits>
#include <hip/hip_ext.h>
#include "trace.h"
#include "glibc_pow.h"
#include "intersect.h"

namespace rtamd {
namespace {

using namespace dev;

// q = n / d for 0 <= n < 2^52, 0 < d (both exact in binary64): the quotient of the
// doubles, corrected by one step (the rounded quotient is within 1 of the exact one).
// A 64-bit integer division is a long emulated sequence on the GPU.
__device__ __forceinline__ int64_t div_small(int64_t n, int64_t d) {
	int64_t q = static_cast<int64_t>(static_cast<double>(n) / static_cast<double>(d));
	const int64_t r = n - q * d;
	q += (r < 0) ? -1 : (r >= d ? 1 : 0);
	return q;
}

constexpr int kShadeBlock = 512;
typedef __attribute__((address_space(3))) double lds_f64;
// an LDS address the compiler cannot see through: values are read back from LDS, not kept in
// registers from the store
__device__ __forceinline__ lds_f64* opaque_lds(lds_f64* p) {
	asm volatile("" : "+v"(p));
	return p;
}
#ifndef RT_FUSED_PARK
#define RT_FUSED_PARK 1
#endif
// entries of a wave-packet traversal's stack (LDS, one per wave)
constexpr int kWaveStack = kStackDepth;

// Occupancy targets of the traversal kernels (waves per SIMD, >= 1).  4 (<= 128 VGPRs, a
// few spills) measured 3 % faster than the compiler's 3 on C3; the wave-packet variants
// (node and face records in SGPRs) measured best at 4 as well: more waves of them starve
// the closest-hit chain.
#ifndef RT_TRAVERSAL_WAVES
#define RT_TRAVERSAL_WAVES 4
#endif
#ifndef RT_CLOSEST_WAVES
#define RT_CLOSEST_WAVES RT_TRAVERSAL_WAVES
#endif
#ifndef RT_PACKET_WAVES
#define RT_PACKET_WAVES RT_TRAVERSAL_WAVES
#endif
// A scene of spheres only: no LBVH search, so the closest-hit and per-lane shadow kernels fit
// 96 VGPRs without spills (5 waves per SIMD; the packet shadow kernel with its fused Phong
// terms keeps 4: at 96 VGPRs it spills 16)
#ifndef RT_SPHERE_WAVES
#define RT_SPHERE_WAVES 5
#endif
// Meshes scanned face by face only (kMeshLinear): no LBVH search either, but the fp64 face
// test's registers (at 5 waves the per-lane kernels spill 18-21 VGPRs)
#ifndef RT_LINEAR_WAVES
#define RT_LINEAR_WAVES 4
#endif

// Camera::calculateViewingRay (rtbase.h:74-84) for pixel (r, c) (scene.cpp:26-30)
__device__ __forceinline__ void primary_ray(const DCamera* camp, int r, int c, int W, int H, V3& o, V3& d,
                                            DeviceCounters* ctr) {
	const auto& cam = *uniform_ptr(opaque(camp));
	const double rF = (r + 0.5) / H;
	const double cF = (c + 0.5) / W;
	const double rI = 1.0 - rF, cI = 1.0 - cF;
	double p[4];
#pragma unroll
	for (int k = 0; k < 4; k++) p[k] = cF * (rF * cam.lr[k] + rI * cam.ur[k]) + cI * (rF * cam.ll[k] + rI * cam.ul[k]);
	// Ray(eye, P - eye) (rtbase.h:7-24): origin check, then isZero() over all four
	// components, then the w check; the first one that fails throws
	const double dw = p[3] - cam.eye[3];
	const V3 dv = mk(p[0] - cam.eye[0], p[1] - cam.eye[1], p[2] - cam.eye[2]);
	if (cam.eye[3] == 0)
		raise_error(ctr, DERR_ORIGIN_DIRECTION);
	else if (is_zero3(dv) && fabs(dw) <= 1e-12)
		raise_error(ctr, DERR_NO_DIRECTION);
	else if (dw != 0)
		raise_error(ctr, DERR_POINT_DIRECTION);
	o = load3(cam.eye);
	d = normalized3(dv);
}

// Chunk row q (FrameGeometry): the job's row ordinal, the image row (computed as the host's
// selected_row, api.cpp) and the job's outputs, from the segment holding q (the last one
// starting at or before it).  False when the descriptor names no selected row of the frame
// (corrupt): the caller raises DERR_ROWS and writes nothing.
// Every active lane of the wave calls it.  The common case is wave-uniform: the segment of
// the wave's first lane, found by a scalar search of the by-value descriptors, holds every
// lane's row (an 8x8 tile or 64 pixels of a row lie in one job's rows unless they straddle
// two jobs), and each lane only adds its offset.  Otherwise each lane selects its segment in
// a loop over them (uniform index, scalar loads, per-lane selects).  Neither indexes the
// argument block per lane (the compiler would copy it to scratch).  32-bit arithmetic: a
// chunk holds at most 2^22 pixels, an image at most 2^31 rows.
struct ChunkRowRef {
	int32_t ord, row;
	double* out;
	uint8_t* out8;
};
__device__ __forceinline__ bool chunk_row(const FrameGeometry& fg, int64_t q64, ChunkRowRef& r) {
	const int32_t q = static_cast<int32_t>(q64);
	// (the first index comes through an empty asm: the descriptors' loads cannot be hoisted out
	// of the grid-stride loops into scalar registers held through the traversals)
	int j = 0;
	asm volatile("" : "+s"(j));
	const int32_t qf = __builtin_amdgcn_readfirstlane(q);
	// binary search (scalar): the last segment starting at or before qf, in log2(n_segs)
	// dependent loads rather than n_segs (a GPU's row share of 16 frames is 16 segments)
	int k = j, hi = fg.n_segs - 1;
	while (k < hi) {
		const int mid = (k + hi + 1) >> 1;
		if (fg.seg[mid].q0 <= qf)
			k = mid;
		else
			hi = mid - 1;
	}
	const int32_t q_end = k + 1 < fg.n_segs ? fg.seg[k + 1].q0 : fg.n_rows;
	int32_t q0 = fg.seg[k].q0, ord0 = fg.seg[k].ord0, ord_end = fg.seg[k].ord_end;
	int32_t row_begin = fg.seg[k].row_begin, row_block = fg.seg[k].row_block, row_span = fg.seg[k].row_span;
	double* out = fg.seg[k].out;
	uint8_t* out8 = fg.seg[k].out8;
	if (__ballot(q < q0 || q >= q_end)) {  // the wave straddles segments: per lane
		for (; j < fg.n_segs; j++) {
			const RowSegment& sg = fg.seg[j];
			if (q >= sg.q0) {
				q0 = sg.q0, ord0 = sg.ord0, ord_end = sg.ord_end;
				row_begin = sg.row_begin, row_block = sg.row_block, row_span = sg.row_span;
				out = sg.out, out8 = sg.out8;
			}
		}
	}
	const int32_t ord = ord0 + (q - q0);
	int32_t row;
	if (row_block == 1) {  // blocks of one row: whole frames and interleaved rows, no division
		row = row_begin + ord * row_span;
	} else {
		const int32_t blk = row_block >= 1 ? row_block : 1;
		const int32_t nb = (ord >= 0 ? ord : 0) / blk;
		row = row_begin + nb * row_span + (ord - nb * blk);
	}
	r.ord = ord;
	r.row = row;
	r.out = out;
	r.out8 = out8;
	return q64 >= 0 && q < fg.n_rows && ord >= 0 && ord < ord_end && row_block >= 1 && row >= 0 && row < fg.height;
}

// kLevel0: the camera rays of level 0 (the traversal kernels are instantiated separately for
// it: the row look-up and the pixel writes stay out of the other levels' register allocation)
template <bool kLevel0, typename LV>
__device__ __forceinline__ void level_ray(const DeviceScene& S, const FrameGeometry& fg, int level, int64_t i,
                                          const LV& cur, V3& o, V3& d, bool& inside, DeviceCounters* ctr) {
	if constexpr (kLevel0) {
		const int64_t q = div_small(i, fg.width);
		ChunkRowRef rr;
		if (!chunk_row(fg, q, rr)) {
			raise_error(ctr, DERR_ROWS);
			rr.row = 0;  // a ray of a valid row: its pixel is never written (write_pixel checks again)
		}
		const int c = (int)(i - q * fg.width);
		primary_ray(S.cam, rr.row, c, fg.width, fg.height, o, d, ctr);
		inside = false;
	} else {
		o = mk(cur.ox[i], cur.oy[i], cur.oz[i]);
		d = mk(cur.dx[i], cur.dy[i], cur.dz[i]);
		inside = cur.inside[i];
	}
}

// Level-0 thread -> pixel mapping in 8x8 tiles (one wave = one tile), so primary rays,
// their shadow rays and their children are spatially coherent.  Returns -1 outside.
__device__ __forceinline__ int64_t tile_pixel(const FrameGeometry& fg, int64_t n, int64_t t) {
	const int64_t W = fg.width, R = div_small(n, fg.width);
	const int64_t tiles_x = (W + 7) / 8;
	const int64_t tile = t >> 6, l = t & 63;
	const int64_t ty = div_small(tile, tiles_x);
	const int64_t px = (tile - ty * tiles_x) * 8 + (l & 7), py = ty * 8 + (l >> 3);
	return (px < W && py < R) ? py * W + px : -1;
}
__host__ __device__ __forceinline__ int64_t tile_threads(int64_t n, int64_t width) {
	return ((width + 7) / 8) * ((n / width + 7) / 8) * 64;
}

// Workgroups are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, "Workgroup
// dispatch"), each with its own 4 MiB L2.  The logical block index gives XCD x (blocks
// b = x mod 8) runs of RT_XCD_GROUP consecutive blocks, so the rays one L2 serves at a
// time are neighbours and share BVH nodes and triangles, while every XCD still sweeps the
// whole image (balanced load).  Speed only: any bijection is correct.
#ifndef RT_XCD_GROUP
#define RT_XCD_GROUP 16
#endif
__device__ __forceinline__ int64_t xcd_block() {
	const int64_t nb = gridDim.x, b = blockIdx.x;
	if (RT_XCD_GROUP <= 0) return b;
	constexpr int64_t g = RT_XCD_GROUP, span = 8 * g;
	const int64_t base = (b / span) * span;
	if (base + span > nb) return b;  // tail: identity
	return base + (b & 7) * g + ((b - base) >> 3);
}

// L2 warm-up (RT_WARM_L2): the face and node records are fetched by scalar loads, one
// dependent round trip per node and per face, and a scalar-cache miss is served by the XCD's
// L2.  At the start of a frame that L2 holds the previous frame's output and ray levels, not
// the scene, so the first level's long traversals (a row share of C4: one round of waves
// whose slowest, with 75-120 node iterations, set the launch's length, ~1.4 us per
// iteration; profiles/round5/wave_times/) wait on the memory behind L2 at every step.  The
// first blocks of a level-0 launch therefore read the face and node records once per XCD
// (blocks b = x mod 8 run on XCD x) with coalesced vector loads before their own rays.
#ifndef RT_WARM_L2
#define RT_WARM_L2 1
#endif
constexpr uint32_t kWarmBlocksPerXcd = 64;
__device__ __forceinline__ void warm_l2(const DeviceScene& S) {
	const uint32_t nw = min(gridDim.x / 8, kWarmBlocksPerXcd), slice = blockIdx.x / 8;
	if (slice >= nw) return;
	const uint4* fg = reinterpret_cast<const uint4*>(S.fgeo);
	const uint4* nd = reinterpret_cast<const uint4*>(S.nodes);
	constexpr int64_t kF = sizeof(DFaceGeo) / 16, kN = sizeof(DBvhNode) / 16;
	const int64_t nf = int64_t(S.n_faces) * kF, total = nf + int64_t(S.n_nodes) * kN;
	uint32_t acc = 0;
	for (int64_t t = int64_t(slice) * blockDim.x + threadIdx.x; t < total; t += int64_t(nw) * blockDim.x) {
		const uint4 v = t < nf ? fg[t] : nd[t - nf];
		acc ^= v.x;
	}
	asm volatile("" ::"v"(acc));  // the loads are the point: keep them
}

// std::max(x, 0.0)
__device__ __forceinline__ double max0(double x) { return (x < 0.0) ? 0.0 : x; }

__device__ __forceinline__ unsigned long long* shard(unsigned long long* stats) {
	return stats + (blockIdx.x % kStatShards) * kStatStride;
}



template <typename WS>
__device__ __forceinline__ void flush_stats(const WS& ws, unsigned long long* stats, int stage, int packet = 0) {
#if RT_PHASE_PROF
#pragma unroll
	for (int k = 0; k < kPhaseSlots; k++) {
		unsigned long long v = ws.ph[k];
		for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
		if (__lane_id() == 0 && v) atomicAdd(&g_phase[(stage * 2 + packet) * kPhaseSlots + k], v);
	}
#endif
	if constexpr (!WS::kOn) return;
	unsigned long long w[5] = {ws.get(W_NODES), ws.get(W_TRIS), ws.get(W_CANDS), ws.get(W_SPHERES), ws.get(W_ENTRIES)};
	unsigned long long wmax = w[0];
#pragma unroll
	for (int k = 0; k < 5; k++)
		for (int o = 32; o > 0; o >>= 1) w[k] += __shfl_xor(w[k], o);
	for (int o = 32; o > 0; o >>= 1) {
		const unsigned long long v = __shfl_xor(wmax, o);
		wmax = v > wmax ? v : wmax;
	}
	if (__lane_id() == 0) {
		unsigned long long* sh = shard(stats);
		const int base = stage ? ST_NODES1 : ST_NODES0;
#pragma unroll
		for (int k = 0; k < 4; k++)
			if (w[k]) atomicAdd(sh + base + k, w[k]);
		if (w[4]) atomicAdd(sh + (stage ? ST_ENTRIES1 : ST_ENTRIES0), w[4]);
		if (wmax) atomicMax(sh + (stage ? ST_MAXNODES1 : ST_MAXNODES0), wmax);
	}
}

// Block-wide append to two counters: this thread contributes `a` (0/1) slots to counter
// ca and `b0 + b1` (0..2) slots to counter cb; one atomicAdd per counter per block returns
// the block's bases.  Every thread of the block must call it.
constexpr int kMaxWaves = 16;
struct AppendLds {
	int n[2][kMaxWaves + 1];
};
struct Slots {
	int a, b;
};
__device__ __forceinline__ Slots block_append2(bool a, bool b0, bool b1, int32_t* ca, int32_t* cb, AppendLds& lds) {
	const unsigned long long ma = __ballot(a), m0 = __ballot(b0), m1 = __ballot(b1);
	const int lane = __lane_id(), wave = threadIdx.x >> 6;
	const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
	if (lane == 0) {
		lds.n[0][wave] = __popcll(ma);
		lds.n[1][wave] = __popcll(m0) + __popcll(m1);
	}
	__syncthreads();
	if (threadIdx.x < 2) {
		const int k = threadIdx.x;
		const int nw = (blockDim.x + 63) >> 6;
		int total = 0;
		for (int w = 0; w < nw; w++) {
			const int c = lds.n[k][w];
			lds.n[k][w] = total;
			total += c;
		}
		lds.n[k][kMaxWaves] = total ? atomicAdd(k ? cb : ca, total) : 0;
	}
	__syncthreads();
	return Slots{lds.n[0][kMaxWaves] + lds.n[0][wave] + (int)__popcll(ma & below),
	             lds.n[1][kMaxWaves] + lds.n[1][wave] + (int)(__popcll(m0 & below) + __popcll(m1 & below))};
}

// writers.cpp:4-9: (uint8)(min(max(v,0),1) * 255), NaN -> 0
__device__ __forceinline__ uint8_t to_u8(double v) {
	v = (1.0 < v) ? 1.0 : v;
	v = (v < 0.0) ? 0.0 : v;
	v = v * 255.0;
	return (v == v) ? (uint8_t)(int)v : (uint8_t)0;
}

// pixel i of the chunk (column c of its row q) into that row's outputs: f64 and RGB8, at
// the job's row ordinal (a descriptor that names no selected row writes nothing)
__device__ __forceinline__ void write_pixel(const FrameGeometry& fg, int64_t i, const double v[3], bool rgb8,
                                            DeviceCounters* ctr) {
	const int64_t q = div_small(i, fg.width);
	const int64_t c = i - q * fg.width;
	ChunkRowRef rr;
	if (!chunk_row(fg, q, rr)) {
		raise_error(ctr, DERR_ROWS);
		return;
	}
	const int64_t at = (static_cast<int64_t>(rr.ord) * fg.width + c) * 3;
	double* out = rr.out;
	uint8_t* out8 = rr.out8;
	if (out) {
		out[at + 0] = v[0];
		out[at + 1] = v[1];
		out[at + 2] = v[2];
	}
	if (out8 && rgb8) {
		out8[at + 0] = to_u8(v[0]);
		out8[at + 1] = to_u8(v[1]);
		out8[at + 2] = to_u8(v[2]);
	}
}

template <bool kPacket, int kMesh, typename NV, typename DV, typename WS>
__device__ __forceinline__ void shade_in_place(const DeviceScene& S, bool on, int gi, V3 P, NV n_of, DV dir_of,
                                               bool inside, int32_t* stack, DeviceCounters* ctr,
                                               unsigned long long* stats, WS& ws, double col[3]);

// Closest hit (castRay, scene.cpp:142-167) + the bounce decisions of scene.cpp:110-136:
// the children's rays and the reflective weight depend only on the hit, not on the
// shading, so they are spawned here and level L+1 can be traced while level L is shaded.
// One item (thread t of the level's index space) of k_closest; every thread of the block
// calls it (block_append2 synchronises the block).
// kFused (k_fused): the hit is shaded right here, its shadow rays and Phong terms from the
// hit held in registers (no hit record, no k_shadow / k_shade launch), and the colour goes
// where fo says.  Never for --intersection-only.
template <bool kPacket, bool kCount, int kMesh, bool kLevel0, bool kFused = false>
__device__ __forceinline__ void closest_item(const DeviceScene& S, const FrameGeometry& fg, int level, int64_t n,
                                             int remaining, int plan_last, const RayLevel* levels,
                                             DeviceCounters* ctr, unsigned long long* stats, int64_t t,
                                             AppendLds& append_lds, int32_t* stack, uint32_t* stat_lds,
                                             const FusedOut* fo = nullptr, lds_f64* park = nullptr) {
	// the level records (~30 buffer pointers) are read where they are used, before and after
	// the traversal, not held in scalar registers through it
	const int next_level = remaining > 0 ? level + 1 : level;
	const int64_t i = (kLevel0 && kPacket) ? tile_pixel(fg, n, t) : (t < n ? t : -1);
	const bool active = i >= 0;
	WorkStats<kCount> ws{};
	ws.init(stat_lds);
	PROF_BEGIN(t_total);
	bool hit = false;
	int gi = -1;
	double dist = 0;
	V3 P = mk(0, 0, 0), N = mk(0, 0, 0), Nobj = mk(0, 0, 0);
	bool inside = false;
	V3 o = mk(0, 0, 0), d = mk(0, 0, 1);
	PROF_BEGIN(t_setup);
	if (active) level_ray<kLevel0>(S, fg, level, i, *uniform_ptr(opaque(levels) + level), o, d, inside, ctr);
	PROF_END(ws, PH_SETUP, t_setup);
#if RT_DIAG_LANES
	if (!kPacket) diag_lanes(0, active);  // [0] wave slots, [1] active lanes of k_closest<false>
#endif
	if (kPacket) DIAG_PK(PK_C_ITEM, active);
	if (kPacket)
		hit = closest_hit_packet<kMesh>(S, o, d, inside, active, dist, gi, P, Nobj, stack, ctr, ws);
	else if (active)
		hit = closest_hit<kMesh>(S, o, d, inside, dist, gi, P, Nobj, stack, ctr, ws);
	if (active) PROF_END(ws, PH_TOTAL, t_total);
	flush_stats(ws, stats, 0, kPacket);
	if (hit) {
		// Geometry::calculateIntersectionNormal tail (geometry.cpp:40-43) + scene.cpp:72-75
		N = xf_normal(S.geoms[gi].inv, Nobj);
		if (S.geoms[gi].flip) N = -N;
		if (inside) N = -N;
		const double rn = 1.0 / sqrt(sq4(N));  // targetNormal.normalize(): times 1/|N|
		N = rn * N;
	}
	const bool shade = hit && !fg.intersection_only;
	// bounce (scene.cpp:110-136): refraction first, then reflection with kr (1 on TIR)
	double kr[3] = {0, 0, 0};
	bool spawn_refr = false, spawn_refl = false;
	V3 refr_d = mk(0, 0, 0), refl_d = mk(0, 0, 0);
	if (shade && remaining > 0) {
		const DMaterial& M = S.mats[S.geoms[gi].mat];
		kr[0] = M.kr[0];
		kr[1] = M.kr[1];
		kr[2] = M.kr[2];
		bool kr_nz = M.kr_nonzero;
		if (M.kt_nonzero) {
			const double nr = inside ? M.ior : 1.0 / M.ior;
			const double cosI = dot4z(N, d);
			const double sinT2 = nr * nr * (1.0 - cosI * cosI);
			if (sinT2 > 1.0) {
				kr[0] = kr[1] = kr[2] = 1.0;  // total internal reflection
				kr_nz = true;
			} else {
				const double k2 = nr * cosI + sqrt(1.0 - sinT2);
				refr_d = ray_dir(nr * d - k2 * N, ctr);
				spawn_refr = true;
			}
		}
		if (kr_nz) {
			refl_d = ray_dir(d - (2 * dot4z(N, d)) * N, ctr);
			spawn_refl = true;
		}
	}
	const RayLevel* lv = opaque(levels);
	const auto& cur = *uniform_ptr(lv + level);
	const auto& next = *uniform_ptr(lv + next_level);
	// (a fused level keeps no hit list: its hit counter is not advanced)
	const Slots slot = block_append2(shade && !kFused, spawn_refr, spawn_refl, cur.counts, cur.counts + 1, append_lds);
	{
		const unsigned long long m_hit = __ballot(shade), m_refl = __ballot(spawn_refl), m_refr = __ballot(spawn_refr);
		if (__lane_id() == 0) {
			unsigned long long* sh = shard(stats);
			if (m_hit) atomicAdd(sh + ST_HITS, (unsigned long long)__popcll(m_hit));
			if (m_refl) atomicAdd(sh + ST_REFL, (unsigned long long)__popcll(m_refl));
			if (m_refr) atomicAdd(sh + ST_REFR, (unsigned long long)__popcll(m_refr));
		}
	}
	if (!kFused && !active) return;
	if (!kFused) {
		cur.hgeom[i] = hit ? gi : -1;
		if (fg.intersection_only) {  // scene.cpp:69-70
			const double v = hit ? 1.0 / (dist * dist) : 0.0;
			cur.cr[i] = cur.cg[i] = cur.cb[i] = v;
			cur.child_refr[i] = cur.child_refl[i] = -1;
			return;
		}
	}
	int32_t refr_idx = -1, refl_idx = -1;
	// the next level holds at most next.capacity rays: a child beyond it is not written and
	// the render is flagged (the host redoes it host-driven, api.cpp)
	// (plan_last: the last level of a replayed plan, whose children were never expected)
	if ((spawn_refr || spawn_refl) &&
	    (plan_last || slot.b + (spawn_refr && spawn_refl ? 1 : 0) >= next.capacity)) {
		raise_error(ctr, DERR_PLAN);
		spawn_refr = spawn_refl = false;
	}
	if (spawn_refr) {
		refr_idx = slot.b;
		next.ox[refr_idx] = P.x;
		next.oy[refr_idx] = P.y;
		next.oz[refr_idx] = P.z;
		next.dx[refr_idx] = refr_d.x;
		next.dy[refr_idx] = refr_d.y;
		next.dz[refr_idx] = refr_d.z;
		next.inside[refr_idx] = !inside;
	}
	if (spawn_refl) {
		refl_idx = slot.b + (spawn_refr ? 1 : 0);
		next.ox[refl_idx] = P.x;
		next.oy[refl_idx] = P.y;
		next.oz[refl_idx] = P.z;
		next.dx[refl_idx] = refl_d.x;
		next.dy[refl_idx] = refl_d.y;
		next.dz[refl_idx] = refl_d.z;
		next.inside[refl_idx] = inside;
		if constexpr (kFused) cur.hgeom[i] = gi;  // for reduce_colour's weight
	}
	if (!kFused || !fo->final) {
		if (active) {
			cur.child_refr[i] = refr_idx;
			cur.child_refl[i] = refl_idx;
		}
	}
	if constexpr (kFused) {
		// every lane of the wave takes part (the packet shadow searches are wave-uniform); a
		// miss is black (scene.cpp:66-67)
		WorkStats<false> ws{};
		double col[3] = {0.0, 0.0, 0.0};
		if constexpr (kPacket && RT_FUSED_PARK) {
			// the shading normal and the viewing direction wait in LDS through the shadow searches
			// (registers), read back where they are used (the per-lane form keeps them: its block's
			// LDS, the traversal stacks, already sets its occupancy)
			lds_f64* pk = park + threadIdx.x;
			pk[0 * kBlock] = N.x, pk[1 * kBlock] = N.y, pk[2 * kBlock] = N.z;
			pk[3 * kBlock] = d.x, pk[4 * kBlock] = d.y, pk[5 * kBlock] = d.z;
			auto n_of = [&]() {
				const lds_f64* q = opaque_lds(pk);
				return mk(q[0 * kBlock], q[1 * kBlock], q[2 * kBlock]);
			};
			auto d_of = [&]() {
				const lds_f64* q = opaque_lds(pk);
				return mk(q[3 * kBlock], q[4 * kBlock], q[5 * kBlock]);
			};
			shade_in_place<kPacket, kMesh>(S, shade, gi, P, n_of, d_of, inside, stack, ctr, stats, ws, col);
		} else {
			shade_in_place<kPacket, kMesh>(S, shade, gi, P, [&]() { return N; }, [&]() { return d; }, inside, stack, ctr,
			                               stats, ws, col);
		}
		if (!active) return;
		if (kLevel0 && fo->final) {  // (a plan of one traced level: level 0)
			write_pixel(fg, i, col, true, ctr);
		} else {
			cur.cr[i] = col[0];
			cur.cg[i] = col[1];
			cur.cb[i] = col[2];
		}
		return;
	}
	if (!hit) {  // background: black (scene.cpp:66-67); hits are coloured by k_shade
		cur.cr[i] = cur.cg[i] = cur.cb[i] = 0.0;
		return;
	}
	// the hit record, compacted at the hit's slot: k_shadow reads it without indirection
	const int64_t h = slot.a;
	cur.hpx[h] = P.x;
	cur.hpy[h] = P.y;
	cur.hpz[h] = P.z;
	cur.hnx[h] = N.x;
	cur.hny[h] = N.y;
	cur.hnz[h] = N.z;
	cur.hdx[h] = d.x;
	cur.hdy[h] = d.y;
	cur.hdz[h] = d.z;
	cur.hinside[h] = (inside ? 1 : 0) | (S.mats[S.geoms[gi].mat].zero_terms ? 2 : 0);
	cur.hit_list[h] = (int32_t)i;
}

// Level 0: one thread per pixel (n_dev null, exact grid).  Deeper levels are launched
// before the host knows their size: the ray count is read from the previous level's
// child counter (n_dev) and a fixed grid strides over it, so each level is queued behind
// the previous one without a host round trip.
template <bool kPacket, bool kCount, int kMesh, bool kLevel0>
__global__ void __launch_bounds__(kBlock)
    __attribute__((amdgpu_waves_per_eu(kMesh == kMeshNone ? RT_SPHERE_WAVES : kMesh == kMeshLinear ? RT_LINEAR_WAVES : kPacket ? RT_PACKET_WAVES : RT_CLOSEST_WAVES))) k_closest(DeviceScene S, FrameGeometry fg, int level,
                                                                      int64_t n_host, const int32_t* n_dev,
                                                                      int remaining, int plan_last,
                                                                      const RayLevel* levels, DeviceCounters* ctr,
                                                                      unsigned long long* stats) {
	__shared__ AppendLds append_lds;
	__shared__ uint32_t stat_lds[kCount ? W_COUNT * kBlock : 1];
	// the traversal stacks (LBVH searches: none in a scene of spheres only)
	__shared__ int32_t stack_mem[kMesh < kMeshBvh ? 1 : kPacket ? (kBlock / 64) * kWaveStack : kStackDepth * kBlock];
	int32_t* stack = kMesh < kMeshBvh ? stack_mem : kPacket ? stack_mem + (threadIdx.x / 64) * kWaveStack : stack_mem + threadIdx.x;
	// level records read through the constant address space (scalar loads at their uses)
	const auto& cur0 = *uniform_ptr(levels + level);
	const auto& next0 = *uniform_ptr(levels + (remaining > 0 ? level + 1 : level));
	// the level's rays: n_host, or the previous level's child counter, never more than the
	// level holds (children beyond its capacity were not written, see closest_item)
	const int64_t n = n_dev ? min(static_cast<int64_t>(*n_dev), cur0.capacity) : n_host;
	if (blockIdx.x == 0 && threadIdx.x == 0) {
		// the next level's counts start at zero (its k_closest appends to them)
		if (remaining > 0) next0.counts[0] = next0.counts[1] = 0;
		if (n) atomicAdd(stats + ST_RAYS, static_cast<unsigned long long>(n));  // traceRay calls
	}
	const int64_t limit = (kLevel0 && kPacket) ? tile_threads(n, fg.width) : n;
	const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
	if (RT_WARM_L2 && kMesh == kMeshBvh && kLevel0) warm_l2(S);
	for (int64_t base = xcd_block() * kBlock; base < limit; base += stride) {
		WT_BEGIN();
		closest_item<kPacket, kCount, kMesh, kLevel0>(S, fg, level, n, remaining, plan_last, levels, ctr, stats, base + threadIdx.x,
		                      append_lds, stack, stat_lds);
		WT_END(1 | kPacket << 4 | level << 8, base + (threadIdx.x & ~63));
	}
}

__device__ __forceinline__ bool stat_is_max(int k) { return k == ST_MAX_BITS || k == ST_MAXNODES0 || k == ST_MAXNODES1; }

// The statistics reduction by the last block of a launch (FusedOut::summary): k_stats_finish's
// work without a launch of its own.  Every block has added into the shards with device-scope
// atomics (performed beyond the XCDs' L2s, MI355X_MICROARCH.md "Inter-workgroup
// visibility"); each wave waits for its own to complete, the block then counts itself done,
// and the block whose count completes the grid reduces the shards (sc1 loads, L2-bypassing)
// into the summary (pinned host memory), clears them and the error word for the next render
// and resets the counters.  No L2 write-back or invalidation: the only data handed over are
// those atomics.  The count is sharded per XCD (blocks b with b mod 8 = x on counter x, one
// 128-B line each; the XCD whose last block arrives adds to a top counter): one device-scope
// counter takes only ~88 adds per us (MI355X_MICROARCH.md "dequeue").  Every thread of the
// block calls it.
constexpr int kFinishStride = 32;  // uint32 per counter line (128 B); FusedOut::done holds 9 lines
__device__ void last_block_finish(unsigned long long* stats, DeviceCounters* ctr, const FusedOut& fo) {
	__shared__ uint32_t last;
	__shared__ unsigned long long part[kMaxWaves][ST_COUNT];
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's statistics atomics are performed
	__syncthreads();
	if (threadIdx.x == 0) {
		const uint32_t nb = gridDim.x, x = blockIdx.x & 7, n_x = (nb - x + 7) / 8, n_xcd = nb < 8 ? nb : 8;
		uint32_t* cx = fo.done + (1 + x) * kFinishStride;
		last = 0;
		if (__hip_atomic_fetch_add(cx, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n_x - 1) {
			__hip_atomic_store(cx, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // every block of XCD x arrived
			last = __hip_atomic_fetch_add(fo.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n_xcd - 1;
		}
	}
	__syncthreads();
	if (!last) return;
	unsigned long long v[ST_COUNT];
#pragma unroll
	for (int k = 0; k < ST_COUNT; k++) v[k] = 0;
	for (int sh = threadIdx.x; sh < kStatShards; sh += blockDim.x) {
		unsigned long long* p = stats + sh * kStatStride;
#pragma unroll
		for (int k = 0; k < ST_COUNT; k++) {
			const unsigned long long x = __hip_atomic_load(p + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			v[k] = stat_is_max(k) ? (x > v[k] ? x : v[k]) : v[k] + x;
		}
#pragma unroll
		for (int k = 0; k < ST_COUNT; k++) p[k] = 0;
	}
	const int w = threadIdx.x >> 6;
#pragma unroll
	for (int k = 0; k < ST_COUNT; k++) {
		for (int off = 32; off > 0; off >>= 1) {
			const unsigned long long o = __shfl_xor(v[k], off);
			v[k] = stat_is_max(k) ? (o > v[k] ? o : v[k]) : v[k] + o;
		}
		if (__lane_id() == 0) part[w][k] = v[k];
	}
	__syncthreads();
	const int t = threadIdx.x, nw = (blockDim.x + 63) >> 6;
	if (t < ST_COUNT) {
		unsigned long long r = part[0][t];
		for (int q = 1; q < nw; q++) r = stat_is_max(t) ? (part[q][t] > r ? part[q][t] : r) : r + part[q][t];
		fo.summary[t] = r;
	}
	if (t == ST_COUNT) {
		fo.summary[t] = static_cast<unsigned long long>(
		    __hip_atomic_load(&ctr->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
		ctr->error = 0;
		__hip_atomic_store(fo.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
	// the summary is pinned host memory: visible at system scope before the kernel completes
	__threadfence_system();
}

// A whole level in one launch (small chunks and plans of one traced level, api.cpp): closest
// hits, children, and each hit's shadow rays and Phong terms from registers
// (closest_item<.., kFused>), with fo.final the output pixels too, and with fo.summary the
// statistics finish.  Level 0 traces 8x8 tiles as wave packets like k_closest.
#ifndef RT_FUSED_WAVES
#define RT_FUSED_WAVES 4
#endif
template <bool kPacket, int kMesh, bool kLevel0>
__global__ void __launch_bounds__(kBlock)
    __attribute__((amdgpu_waves_per_eu(RT_FUSED_WAVES))) k_fused(
        DeviceScene S, FrameGeometry fg, int level, int64_t n_host, const int32_t* n_dev, int remaining, int plan_last,
        const RayLevel* levels, DeviceCounters* ctr, unsigned long long* stats, FusedOut fo) {
	__shared__ AppendLds append_lds;
	__shared__ int32_t stack_mem[kMesh < kMeshBvh ? 1 : kPacket ? (kBlock / 64) * kWaveStack : kStackDepth * kBlock];
	__shared__ double park_mem[RT_FUSED_PARK && kPacket ? 6 * kBlock : 1];
	int32_t* stack = kMesh < kMeshBvh ? stack_mem : kPacket ? stack_mem + (threadIdx.x / 64) * kWaveStack : stack_mem + threadIdx.x;
	const auto& cur0 = *uniform_ptr(levels + level);
	const auto& next0 = *uniform_ptr(levels + (remaining > 0 ? level + 1 : level));
	const int64_t n = n_dev ? min(static_cast<int64_t>(*n_dev), cur0.capacity) : n_host;
	if (blockIdx.x == 0 && threadIdx.x == 0) {
		if (remaining > 0) next0.counts[0] = next0.counts[1] = 0;
		if (n) atomicAdd(stats + ST_RAYS, static_cast<unsigned long long>(n));
	}
	const int64_t limit = (kLevel0 && kPacket) ? tile_threads(n, fg.width) : n;
	const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
	if (RT_WARM_L2 && kMesh == kMeshBvh && kLevel0) warm_l2(S);
	for (int64_t base = xcd_block() * kBlock; base < limit; base += stride) {
		WT_BEGIN();
		closest_item<kPacket, false, kMesh, kLevel0, true>(S, fg, level, n, remaining, plan_last, levels, ctr, stats,
		                                          base + threadIdx.x, append_lds, stack, nullptr, &fo,
		                                          (lds_f64*)(park_mem));
		WT_END(2 | kPacket << 4 | level << 8, base + (threadIdx.x & ~63));
	}
	if (fo.summary) last_block_finish(stats, ctr, fo);
}

// Level of item t of a batch (wave-uniform: every level's items start on a wave boundary,
// so the level is found from the wave's first item, in scalar registers)
struct BatchItem {
	int32_t level;
	int64_t local, nh;
};
__device__ __forceinline__ int64_t wave_first(int64_t t) {
	return __builtin_amdgcn_readfirstlane(static_cast<int32_t>(t & ~int64_t(63))) |
	       (static_cast<int64_t>(__builtin_amdgcn_readfirstlane(static_cast<int32_t>(t >> 32))) << 32);
}
__device__ __forceinline__ int64_t wave_up64(int64_t x) { return (x + 63) & ~int64_t(63); }
// hits of level k of a device-counted batch (its k_closest has completed)
__device__ __forceinline__ int64_t batch_nh(const ShadeBatch& B, int k) { return *uniform_ptr(B.nh_dev[k]); }
// items per hit: k_shadow (all lights: 1, light-major: one per non-ambient light) or k_shade (1)
template <bool kShadow>
__device__ __forceinline__ int64_t batch_items_per_hit(const ShadeBatch& B, int nl) {
	return (kShadow && !B.all_lights) ? nl : 1;
}
template <bool kShadow>
__device__ __forceinline__ BatchItem batch_item(const ShadeBatch& B, int nl, int64_t t) {
	const int64_t t0 = wave_first(t);
	if (!B.dev_counts) {
		const int64_t* begin = kShadow ? B.shadow_begin : B.shade_begin;
		int k = 0;
		while (k + 1 < B.n && t0 >= begin[k + 1]) k++;
		return BatchItem{B.level[k], t - begin[k], B.nh[k]};
	}
	// ranges from the levels' hit counters: level k covers items_per_hit x nh rounded up to 64
	const int64_t per = batch_items_per_hit<kShadow>(B, nl);
	int64_t begin = 0, nh = batch_nh(B, 0);
	int k = 0;
	while (k + 1 < B.n && t0 >= begin + per * wave_up64(nh)) {
		begin += per * wave_up64(nh);
		nh = batch_nh(B, ++k);
	}
	return BatchItem{B.level[k], t - begin, nh};
}
// items of the whole batch
template <bool kShadow>
__device__ __forceinline__ int64_t batch_total(const ShadeBatch& B, int nl) {
	if (!B.dev_counts) return kShadow ? B.shadow_begin[B.n] : B.shade_begin[B.n];
	int64_t tot = 0;
	for (int k = 0; k < B.n; k++) tot += batch_items_per_hit<kShadow>(B, nl) * wave_up64(batch_nh(B, k));
	return tot;
}

// Phong terms in light order (scene.cpp:78-108) of a hit on geometry gi (hit point P,
// shading normal N, viewing direction d); occluded_j(j): the verdict of the j-th non-ambient
// light.  The colour goes to col.
template <typename OCC>
__device__ __forceinline__ void phong(const DeviceScene& S, int gi, V3 P, V3 N, V3 d, OCC occluded_j,
                                      const double* log_tab, const uint64_t* exp_tab, DeviceCounters* ctr,
                                      double col[3]) {
	col[0] = col[1] = col[2] = 0.0;
	const DMaterial& M = S.mats[S.geoms[gi].mat];
	int j = 0;
	for (int li = 0; li < S.n_lights; li++) {
		const DLight& L = S.lights[li];
		if (L.kind == DLIGHT_AMBIENT) {
#pragma unroll
			for (int k = 0; k < 3; k++) col[k] = col[k] + (1.0 * L.color[k]) * M.ka[k];
			continue;
		}
		const bool occ = occluded_j(j);
		j++;
		if (occ) continue;
		const bool point = L.kind == DLIGHT_POINT;
		const V3 lv = load3(L.vec);
		const V3 Ld = ray_dir(point ? lv - P : -lv, ctr);
		const double nl_dot = dot4z(N, Ld);
		const double dL = point ? sqrt(sq4(lv - P)) : INFINITY;
		// colorForDistance; glibc's pow(x, +-0) is exactly 1 and pow(x, 1) exactly x (its < 0.52-ulp
		// bound pins exact results; checked on 500k libm samples), so those exponents skip it
		const double fall = (point && L.falloff != 0.0) ? glibc_pow(dL, -L.falloff, log_tab, exp_tab) : 1.0;
		double att[3];
#pragma unroll
		for (int k = 0; k < 3; k++) att[k] = point ? fall * L.color[k] : L.color[k];
		const double diff = max0(nl_dot);
#pragma unroll
		for (int k = 0; k < 3; k++) col[k] = col[k] + (diff * att[k]) * M.kd[k];
		const V3 R = (2 * nl_dot) * N - Ld;
		const double sbase = max0(-dot4z(d, R));
		const double spec = M.ns == 1.0 ? sbase : glibc_pow(sbase, M.ns, log_tab, exp_tab);
#pragma unroll
		for (int k = 0; k < 3; k++) col[k] = col[k] + (spec * att[k]) * M.ks[k];
	}
}
// the same for hit slot hs of a level (hit records, compacted), into the ray's colour
template <typename LV, typename OCC>
__device__ __forceinline__ void shade_hit(const DeviceScene& S, const LV& cur, int64_t hs, V3 P, V3 N, V3 d,
                                          OCC occluded_j, const double* log_tab, const uint64_t* exp_tab,
                                          DeviceCounters* ctr) {
	const int64_t i = cur.hit_list[hs];
	double col[3];
	phong(S, cur.hgeom[i], P, N, d, occluded_j, log_tab, exp_tab, ctr, col);
	cur.cr[i] = col[0];
	cur.cg[i] = col[1];
	cur.cb[i] = col[2];
}

// The shadow verdict of the j-th non-ambient light for a hit at P with shading normal N
// (scene.cpp:87-93): occluded, or both Phong terms exact zeros.  Both Phong terms of this
// light (scene.cpp:96-106, the expressions of k_shade) are exact zeros when max(N.L, 0) and
// max(-V.R, 0) are (given ns > 0 and finite colours, DMaterial/DLight::zero_terms): the
// colour is the same bits whether the light is occluded or not (it is never -0), so that ray
// is not traced.  dv_of(): the viewing direction, read only for that test.  Every lane of
// the wave calls it (kPacket: the search is wave-uniform; lanes without a hit pass on false).
template <bool kPacket, int kMesh, typename NV, typename DV, typename WS>
__device__ __forceinline__ bool light_verdict(const DeviceScene& S, int j, V3 P, NV n_of, bool inside, bool zero_mat,
                                              bool on, DV dv_of, int32_t* stack, DeviceCounters* ctr,
                                              unsigned long long* stats, WS& ws) {
	V3 Ld = mk(0, 0, 1);
	bool rev = false, zero = false;
	double dL = 0;
	if (on) {
		const V3 N = n_of();
		const auto& L = *(uniform_ptr(S.lights) + uniform_ptr(S.shadow_light)[j]);
		const bool point = L.kind == DLIGHT_POINT;
		const V3 lv = load3(L.vec);
		Ld = ray_dir(point ? lv - P : -lv, ctr);  // Light::calculateRayToLight
		const double nl_dot = dot4z(N, Ld);
		rev = (nl_dot < 0) ^ inside;
		dL = point ? sqrt(sq4(lv - P)) : INFINITY;
		if (zero_mat && L.zero_terms && nl_dot <= 0.0) {
			const V3 R = (2 * nl_dot) * N - Ld;
			zero = -dot4z(dv_of(), R) <= 0.0;
		}
		// the reference's castRay still maps the ray into every object space (may raise)
		if (zero) check_may_raise(S, Ld, true, ctr);
	}
	const bool trace = on && !zero;
#if RT_DIAG_LANES
	if (!kPacket) {
		diag_lanes(16, on);     // [16] wave slots, [17] lanes with a hit of this level
		diag_lanes(18, trace);  // [18] wave slots, [19] lanes tracing (zero-term decided excluded)
	}
#endif
	bool occ = false;
	if (kPacket) DIAG_PK(PK_LIGHT, trace);
	if (kPacket)
		occ = occluded_packet<kMesh>(S, P, Ld, rev, dL, trace, stack, ctr, ws);
	else if (trace)
		occ = occluded<kMesh>(S, P, Ld, rev, dL, stack, ctr, ws);
	const unsigned long long mz = __ballot(zero);
	if (mz && __lane_id() == 0) atomicAdd(shard(stats) + ST_SHADOW_ZERO, (unsigned long long)__popcll(mz));
	return occ || zero;
}

// A fused level's shading (closest_item<.., kFused>): the verdicts of every light for the
// hit held in registers, then its Phong terms (scene.cpp:78-108) into col.  on: the lane has
// a hit to shade (every lane of the wave calls it).
template <bool kPacket, int kMesh, typename NV, typename DV, typename WS>
__device__ __forceinline__ void shade_in_place(const DeviceScene& S, bool on, int gi, V3 P, NV n_of, DV dir_of,
                                               bool inside, int32_t* stack, DeviceCounters* ctr,
                                               unsigned long long* stats, WS& ws, double col[3]) {
	const bool zero_mat = on && S.mats[S.geoms[gi].mat].zero_terms;
	unsigned long long verdicts = 0;  // bit j: the j-th non-ambient light's verdict (<= 64 lights)
	for (int j = 0; j < S.n_nonambient; j++)
		verdicts |= static_cast<unsigned long long>(
		                light_verdict<kPacket, kMesh>(S, j, P, n_of, inside, zero_mat, on, dir_of, stack, ctr, stats, ws))
		            << j;
	if (on)
		phong(S, gi, P, n_of(), dir_of(), [&](int j) { return static_cast<bool>((verdicts >> j) & 1); },
		      glibc_pow_data::kLogTab, glibc_pow_data::kExpTab, ctr, col);
}

// Shadow rays (scene.cpp:87-93), two item layouts (ShadeBatch::all_lights):
//  - light-major: item t of a level -> (light j, hit h) with t = j * nh64 + h, nh64 = nh
//    rounded up to a multiple of 64, so every wave traces rays towards ONE light;
//  - all lights: item t -> hit h = t, and the wave traces the shadow rays of its 64 hits
//    towards each light in turn (one light at a time, still wave-uniform), loading the hit
//    records once for all lights.
// The light record of the wave is read with scalar loads.
// Fused shading (ShadeBatch::fused, all lights per lane): the lane computes its hit's Phong
// terms from the verdicts held in registers (no k_shade).  kFuse: 1 the kernel always fuses (its
// own instantiation, without the light-major index mapping and the verdict stores: +0.6% on
// the batch bench), 0 never (per-lane kernels with LBVH searches), 2 as B.fused says.  The
// packet kernel's unfused launches (light-major, single frames) keep the form with both paths:
// an instantiation without the Phong terms finished its launches sooner and moved their k_shade
// onto the CUs the closest-hit chain needs (C3 frame 1.207 vs 1.169 ms, A/B).
template <bool kPacket, bool kCount, int kMesh, int kFuse>
__device__ __forceinline__ void shadow_item(const DeviceScene& S, const ShadeBatch& B, const RayLevel* levels,
                                            DeviceCounters* ctr, unsigned long long* stats, int64_t tg, int32_t* stack,
                                            uint32_t* stat_lds) {
	const int nl = S.n_nonambient;
	const BatchItem it = batch_item<true>(B, nl, tg);
	const int level = it.level;
	const int64_t t = it.local, nh = it.nh;
	WorkStats<kCount> ws{};
	ws.init(stat_lds);
	PROF_BEGIN(t_total);
	int j0 = 0, j1 = nl;
	int64_t h = t;
	const bool fused = kFuse == 1 || (kFuse == 2 && B.fused);
	if (kFuse != 1 && !B.all_lights) {
		const int64_t nh64 = (nh + 63) & ~int64_t(63);
		// the wave's light: j = t0 / nh64 for its first item t0 (a few scalar steps: nl <= 64)
		const int64_t t0 = t - (threadIdx.x & 63);
		int j = 0;
		while (j + 1 < nl && t0 >= (j + 1) * nh64) j++;
		j0 = __builtin_amdgcn_readfirstlane(j);
		j1 = j0 + 1;
		h = t - j0 * nh64;
	}
	const bool on = h < nh;
	V3 P = mk(0, 0, 0);
	bool inside = false, zero_mat = false;
	{
		// the level's record, read here and again where the verdicts are written (opaque: its
		// buffer pointers are not held in scalar registers through the traversals)
		const auto& cur = *uniform_ptr(opaque(levels) + level);
		if (on) {
			P = mk(cur.hpx[h], cur.hpy[h], cur.hpz[h]);
			const uint8_t fl = cur.hinside[h];
			inside = fl & 1;
			zero_mat = fl & 2;
		}
	}
	// the shading normal and the viewing direction are read from the hit record where they are
	// used (each light's set-up, the Phong terms), not held in registers through the searches
	auto n_of = [&]() {
		const auto& cur = *uniform_ptr(opaque(levels) + level);
		return mk(cur.hnx[h], cur.hny[h], cur.hnz[h]);
	};
	auto d_of = [&]() {
		const auto& cur = *uniform_ptr(opaque(levels) + level);
		return mk(cur.hdx[h], cur.hdy[h], cur.hdz[h]);
	};
	unsigned long long verdicts = 0;  // fused: bit j = the j-th light's verdict
	for (int j = j0; j < j1; j++) {
		const bool v = light_verdict<kPacket, kMesh>(S, j, P, n_of, inside, zero_mat, on, d_of, stack, ctr, stats, ws);
		// light-major: a wave writes 64 adjacent bytes; a zero-term light is skipped by k_shade
		if (fused) {
			verdicts |= static_cast<unsigned long long>(v) << j;
		} else if (on) {
			const auto& cur = *uniform_ptr(opaque(levels) + level);
			cur.occl[j * cur.capacity + h] = v;
		}
	}
	if (on) PROF_END(ws, PH_TOTAL, t_total);
	flush_stats(ws, stats, 1, kPacket);
	// fused shading (ShadeBatch::fused: all lights of the hit traced by this lane): the Phong
	// terms of k_shade from the verdicts in registers (per-lane kernels: without LBVH
	// searches only, whose registers leave room for them: 127 VGPRs without spills; the
	// sphere-only kernel, built for 5 waves, would spill 18)
	// (with LBVH searches it would spill 26 VGPRs; measured neutral on the batch and C3)
#if RT_DIAG_LANES
	if (!kPacket && fused) diag_lanes(28, on);  // [28] wave slots, [29] lanes shading in place
#endif
	if (kFuse != 0 && fused && on) {
		const auto& cur = *uniform_ptr(opaque(levels) + level);
		shade_hit(S, cur, h, P, n_of(), d_of(), [&](int j) { return static_cast<bool>((verdicts >> j) & 1); },
		          glibc_pow_data::kLogTab, glibc_pow_data::kExpTab, ctr);
	}
}

// Host-counted batches launch one thread per item; device-counted ones a fixed grid that
// strides over the items (the bound is block-uniform: no lane of a wave leaves early).
template <bool kPacket, bool kCount, int kMesh, int kFuse>
__global__ void __launch_bounds__(kBlock)
    __attribute__((amdgpu_waves_per_eu(kMesh == kMeshNone && !kPacket ? RT_SPHERE_WAVES : kMesh == kMeshLinear && !kPacket ? RT_LINEAR_WAVES : kPacket ? RT_PACKET_WAVES : RT_TRAVERSAL_WAVES))) k_shadow(DeviceScene S, ShadeBatch B,
                                                                     const RayLevel* levels, DeviceCounters* ctr,
                                                                     unsigned long long* stats) {
	__shared__ int32_t stack_mem[kMesh < kMeshBvh ? 1 : kPacket ? (kBlock / 64) * kWaveStack : kStackDepth * kBlock];
	__shared__ uint32_t stat_lds[kCount ? W_COUNT * kBlock : 1];
	int32_t* stack = kMesh < kMeshBvh ? stack_mem : kPacket ? stack_mem + (threadIdx.x / 64) * kWaveStack : stack_mem + threadIdx.x;
	const int64_t total = batch_total<true>(B, S.n_nonambient);
	const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
	for (int64_t base = xcd_block() * kBlock; base < total; base += stride) {
		WT_BEGIN();
		shadow_item<kPacket, kCount, kMesh, kFuse>(S, B, levels, ctr, stats, base + threadIdx.x, stack, stat_lds);
		WT_END(3 | kPacket << 4 | B.level[0] << 8, base + (threadIdx.x & ~63));
	}
}

// Phong terms in light order (scene.cpp:78-108), one thread per hit of the level
__global__ void __launch_bounds__(kShadeBlock) k_shade(DeviceScene S, ShadeBatch B, const RayLevel* levels,
                                                       DeviceCounters* ctr) {
	// glibc pow tables in LDS: the specular pow's two dependent table lookups per light
	// are LDS latency instead of divergent L2 gathers
	__shared__ double log_tab[512];
	__shared__ uint64_t exp_tab[256];
	for (int k = threadIdx.x; k < 512; k += blockDim.x) log_tab[k] = glibc_pow_data::kLogTab[k];
	for (int k = threadIdx.x; k < 256; k += blockDim.x) exp_tab[k] = glibc_pow_data::kExpTab[k];
	__syncthreads();
	const int64_t total = batch_total<false>(B, S.n_nonambient);
	const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
	for (int64_t base = xcd_block() * blockDim.x; base < total; base += stride) {
		const BatchItem it = batch_item<false>(B, S.n_nonambient, base + threadIdx.x);
		if (it.local >= it.nh) continue;
		const int level = it.level;
		const auto& cur = *uniform_ptr(levels + level);
		const int64_t hs = it.local;  // the hit's slot (hit records, verdicts)
		const V3 d = mk(cur.hdx[hs], cur.hdy[hs], cur.hdz[hs]);  // the viewing ray's direction
		const V3 P = mk(cur.hpx[hs], cur.hpy[hs], cur.hpz[hs]);
		const V3 N = mk(cur.hnx[hs], cur.hny[hs], cur.hnz[hs]);
		shade_hit(S, cur, hs, P, N, d, [&](int j) { return static_cast<bool>(cur.occl[j * cur.capacity + hs]); },
		          log_tab, exp_tab, ctr);
	}
}

// colour = (local + refraction) + reflection * kr, in place (scene.cpp:127,134).  kr is the
// hit material's reflective colour, or 1 on total internal reflection (scene.cpp:119-123):
// a refractive material's hit with a reflection child and no refraction child is exactly
// that case (k_closest spawns the refraction child whenever sinT2 <= 1), so kr is derived
// from the hit geometry instead of being stored per ray (24 B written and read per ray)
__device__ __forceinline__ void reduce_colour(int64_t i, const RayLevel& cur, const RayLevel& next,
                                              const DGeom* geoms, const DMaterial* mats, double c[3]) {
	c[0] = cur.cr[i];
	c[1] = cur.cg[i];
	c[2] = cur.cb[i];
	const int32_t t = cur.child_refr[i], r = cur.child_refl[i];
	if (t >= 0) {
		c[0] = c[0] + next.cr[t];
		c[1] = c[1] + next.cg[t];
		c[2] = c[2] + next.cb[t];
	}
	if (r >= 0) {
		const DMaterial& M = mats[geoms[cur.hgeom[i]].mat];
		const bool tir = M.kt_nonzero && t < 0;
		c[0] = c[0] + next.cr[r] * (tir ? 1.0 : M.kr[0]);
		c[1] = c[1] + next.cg[r] * (tir ? 1.0 : M.kr[1]);
		c[2] = c[2] + next.cb[r] * (tir ? 1.0 : M.kr[2]);
	}
}
// Two levels in one pass: cur's final colour from next's colours reduced on the fly with
// low's final ones (reduce_colour of each child, in registers): the same operations in the
// same order as reducing next in a launch of its own and then cur, without writing next's
// final colours (nothing else reads them) or a launch between the two
__device__ __forceinline__ void reduce_colour2(int64_t i, const RayLevel& cur, const RayLevel& next, const RayLevel& low,
                                               const DGeom* geoms, const DMaterial* mats, double c[3]) {
	c[0] = cur.cr[i];
	c[1] = cur.cg[i];
	c[2] = cur.cb[i];
	const int32_t t = cur.child_refr[i], r = cur.child_refl[i];
	if (t >= 0) {
		double m[3];
		reduce_colour(t, next, low, geoms, mats, m);
		c[0] = c[0] + m[0];
		c[1] = c[1] + m[1];
		c[2] = c[2] + m[2];
	}
	if (r >= 0) {
		double m[3];
		reduce_colour(r, next, low, geoms, mats, m);
		const DMaterial& M = mats[geoms[cur.hgeom[i]].mat];
		const bool tir = M.kt_nonzero && t < 0;
		c[0] = c[0] + m[0] * (tir ? 1.0 : M.kr[0]);
		c[1] = c[1] + m[1] * (tir ? 1.0 : M.kr[1]);
		c[2] = c[2] + m[2] * (tir ? 1.0 : M.kr[2]);
	}
}
// kLevels 1: cur's final colours from next's; 2: from next's and low's (reduce_colour2)
template <int kLevels>
__global__ void k_reduce(int64_t n_host, const int32_t* n_dev, RayLevel cur, RayLevel next, RayLevel low,
                         const DGeom* geoms, const DMaterial* mats) {
	const int64_t n = n_dev ? min(static_cast<int64_t>(*n_dev), cur.capacity) : n_host;
	const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
	for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
		if (cur.child_refr[i] < 0 && cur.child_refl[i] < 0) continue;
		double c[3];
		if constexpr (kLevels == 2)
			reduce_colour2(i, cur, next, low, geoms, mats, c);
		else
			reduce_colour(i, cur, next, geoms, mats, c);
		cur.cr[i] = c[0];
		cur.cg[i] = c[1];
		cur.cb[i] = c[2];
	}
}

// the image: level 0's colours, reduced on the fly with level 1 (kReduce 1: the last k_reduce
// fused into the output) or with levels 1 and 2 (kReduce 2, reduce_colour2); fo.summary: the
// last block finishes the statistics
template <int kReduce>
__global__ void k_output(int64_t n, FrameGeometry fg, RayLevel lvl0, RayLevel lvl1, RayLevel lvl2, const DGeom* geoms,
                         const DMaterial* mats, unsigned long long* stats, DeviceCounters* ctr, FusedOut fo) {
	const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
	const int32_t io = fg.intersection_only;
	// level 0's counts were read back; clear them for the lane's next chunk
	if (i == 0) lvl0.counts[0] = lvl0.counts[1] = 0;
	double v[3] = {0, 0, 0};
	if (i < n) {
		if constexpr (kReduce == 2) {
			reduce_colour2(i, lvl0, lvl1, lvl2, geoms, mats, v);
		} else if constexpr (kReduce == 1) {
			reduce_colour(i, lvl0, lvl1, geoms, mats, v);
		} else {
			v[0] = lvl0.cr[i];
			v[1] = lvl0.cg[i];
			v[2] = lvl0.cb[i];
		}
		write_pixel(fg, i, v, !io, ctr);
	}
	if (io) {  // running max of maxCoeff over positive doubles (bit order == value order)
		const double m = (i < n) ? fmax(fmax(v[0], v[1]), v[2]) : 0.0;
		unsigned long long bits = (m > 0.0) ? (unsigned long long)__double_as_longlong(m) : 0ull;
		for (int off = 32; off > 0; off >>= 1) {
			const unsigned long long o = __shfl_xor(bits, off);
			bits = o > bits ? o : bits;
		}
		if (__lane_id() == 0 && bits) atomicMax(shard(stats) + ST_MAX_BITS, bits);
	}
	if (fo.summary) last_block_finish(stats, ctr, fo);
}

// one block of kStatShards threads: thread t owns shard t; tree reduction in LDS
__global__ void k_stats_finish(unsigned long long* stats, DeviceCounters* ctr, unsigned long long* summary) {
	__shared__ unsigned long long red[kStatShards][ST_COUNT + 1];
	const int t = threadIdx.x;
	auto is_max = [](int k) { return k == ST_MAX_BITS || k == ST_MAXNODES0 || k == ST_MAXNODES1; };
#pragma unroll
	for (int k = 0; k < ST_COUNT; k++) {
		red[t][k] = stats[t * kStatStride + k];
		stats[t * kStatStride + k] = 0;
	}
	__syncthreads();
	for (int half = kStatShards / 2; half > 0; half >>= 1) {
		if (t < half)
#pragma unroll
			for (int k = 0; k < ST_COUNT; k++) {
				const unsigned long long a = red[t][k], b = red[t + half][k];
				red[t][k] = is_max(k) ? (a > b ? a : b) : a + b;
			}
		__syncthreads();
	}
	if (t < ST_COUNT) summary[t] = red[0][t];
	if (t == ST_COUNT) {
		summary[t] = static_cast<unsigned long long>(ctr->error);
		ctr->error = 0;
	}
	// summary may be pinned host memory (api.cpp summary_mapped): visible to the host at
	// system scope before the kernel completes
	__threadfence_system();
}

__global__ void k_normalize(int64_t n_values, double* rgb, double rcp, uint8_t* out8) {
	const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n_values) return;
	const double v = rgb[i] * rcp;
	rgb[i] = v;
	if (out8) out8[i] = to_u8(v);
}

__global__ void k_selftest(int op, const double* x, const double* y, double* out, int64_t n) {
	const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	if (op == 0) {
		out[i] = glibc_pow(x[i], y[i]);
	} else if (op == 1) {
		out[i] = sqrt(x[i]);
	} else if (op == 2) {
		out[i] = x[i] / y[i];
	} else if (op == 4) {  // normalized3 of the vector (x[i], y[i], x[i + n]) (component x; .y, .z below)
		out[i] = normalized3(mk(x[i], y[i], x[(i + n / 2) % n])).x;
	} else if (op == 5) {
		out[i] = normalized3(mk(x[i], y[i], x[(i + n / 2) % n])).y;
	} else {
		out[i] = normalized3(mk(x[i], y[i], x[(i + n / 2) % n])).z;
	}
}

// FETCH_SIZE calibration (profiles/, MI355X_MICROARCH.md: the counter is calibrated only
// for 16-B-per-lane streaming reads): every element of a buffer far larger than the
// Infinity Cache read once, W bytes per lane per load, coalesced like the ray and hit
// records (consecutive lanes, consecutive elements)
template <typename T>
__global__ void k_stream_read(const T* __restrict__ p, int64_t n, unsigned long long* sink) {
	unsigned long long acc = 0;
	const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
	for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
		const T v = p[i];
		acc += reinterpret_cast<const unsigned char*>(&v)[0];
	}
	if (acc == 0x7fffffffffffffffull) sink[0] = acc;  // keeps the loads; never true for the zeroed buffer
}

// VALU issue calibration (tools/valu_calibration.py, profiles/): every wave runs `iters`
// rounds of 32 independent chains, unrolled 4x (128 instructions per round, nothing else
// in the loop but the counter), on every CU at W waves per SIMD (grid 256 W blocks of 4
// waves).  K selects the instruction (kValuKinds): 0 v_fma_f32, 1 v_pk_fma_f32 (two f32
// FMAs per lane), 2 v_fma_f64, then the other instructions the traversal kernels are made
// of (--mix: 64-bit add/mul/max/compare/move, 32-bit select/integer add/move/compare, the
// f64 reciprocal; 13-16: v_cndmask_b32 with its mask in an SGPR pair set by a ballot, in
// VCC set by a compare before the loop, with two vector sources, and v_cmp_gt_f64 into an
// SGPR pair; 17-18: v_cndmask_b32 of two vector sources under VCC, VOP2 and VOP3 encodings;
// 19-25: the f64 division's v_div_fmas / v_div_scale / v_div_fixup, v_addc_co_u32 (VOP2,
// carry in VCC), v_readlane_b32 / v_writelane_b32 (SGPR spill traffic), v_sqrt_f64).
// Operands are the chain's own register and inline constants (the chains
// stay finite and normal), so no operand read limits issue.  rocprofv3 (SQ_INSTS_VALU,
// SQ_ACTIVE_INST_VALU, GRBM_GUI_ACTIVE + kernel trace), or the events of
// rt_debug_valu_rate, turn it into cycles per wave64 instruction per SIMD.
constexpr int kValuKinds = 26;
template <int K>
__device__ __forceinline__ void valu_op(float& x) {
	if constexpr (K == 0) asm volatile("v_fma_f32 %0, %0, 0.5, 1.0" : "+v"(x));
	if constexpr (K == 7) asm volatile("v_cndmask_b32 %0, 1.0, %0, vcc" : "+v"(x));
	if constexpr (K == 8) asm volatile("v_add_u32 %0, 1, %0" : "+v"(x));
	if constexpr (K == 9) asm volatile("v_mov_b32 %0, %0" : "+v"(x));
	if constexpr (K == 10) asm volatile("v_cmp_gt_f32 vcc, 1.0, %0" : "+v"(x)::"vcc");
}
template <int K>
__device__ __forceinline__ void valu_op(double& x) {
	if constexpr (K == 2) asm volatile("v_fma_f64 %0, %0, 0.5, 1.0" : "+v"(x));
	if constexpr (K == 3) asm volatile("v_add_f64 %0, %0, 1.0" : "+v"(x));
	if constexpr (K == 4) asm volatile("v_mul_f64 %0, %0, 1.0" : "+v"(x));
	if constexpr (K == 5) asm volatile("v_max_f64 %0, %0, 1.0" : "+v"(x));
	if constexpr (K == 6) asm volatile("v_cmp_gt_f64 vcc, 1.0, %0" : "+v"(x)::"vcc");
	if constexpr (K == 11) asm volatile("v_mov_b64 %0, %0" : "+v"(x));
	if constexpr (K == 12) asm volatile("v_rcp_f64 %0, %0" : "+v"(x));
}
template <int K>
__global__ void __launch_bounds__(256) k_valu_peak(int iters, float seed, float* sink) {
	if constexpr (K >= 13) {
		// select / compare forms with an explicit mask
		constexpr int kChains = 32;
		const unsigned long long mask = __ballot(threadIdx.x & 1);
		float a[kChains];
		double b[kChains];
#pragma unroll
		for (int k = 0; k < kChains; k++) a[k] = seed + threadIdx.x + k, b[k] = a[k];
		const float y = seed * 3;
		if constexpr (K == 14 || K == 17 || K == 18 || K == 19 || K == 22) asm volatile("v_cmp_gt_f32 vcc, 1.0, %0" ::"v"(y) : "vcc");
		for (int i = 0; i < iters; i++) {
#pragma unroll
			for (int u = 0; u < 4; u++)
#pragma unroll
				for (int k = 0; k < kChains; k++) {
					if constexpr (K == 13) asm volatile("v_cndmask_b32_e64 %0, 1.0, %0, %1" : "+v"(a[k]) : "s"(mask));
					if constexpr (K == 14) asm volatile("v_cndmask_b32 %0, 1.0, %0, vcc" : "+v"(a[k]));
					if constexpr (K == 15) asm volatile("v_cndmask_b32_e64 %0, %1, %0, %2" : "+v"(a[k]) : "v"(y), "s"(mask));
					if constexpr (K == 17) asm volatile("v_cndmask_b32_e32 %0, %1, %0, vcc" : "+v"(a[k]) : "v"(y));
					if constexpr (K == 18) asm volatile("v_cndmask_b32_e64 %0, %1, %0, vcc" : "+v"(a[k]) : "v"(y));
					if constexpr (K == 19) asm volatile("v_div_fmas_f64 %0, %0, 1.0, 1.0" : "+v"(b[k])::"vcc");
					if constexpr (K == 20) asm volatile("v_div_scale_f64 %0, vcc, %0, %0, 1.0" : "+v"(b[k])::"vcc");
					if constexpr (K == 21) asm volatile("v_div_fixup_f64 %0, %0, 1.0, 1.0" : "+v"(b[k]));
					if constexpr (K == 22) asm volatile("v_addc_co_u32_e32 %0, vcc, 0, %0, vcc" : "+v"(a[k])::"vcc");
					if constexpr (K == 23) {
						uint32_t t;
						asm volatile("v_readlane_b32 %0, %1, 5" : "=s"(t) : "v"(a[k]));
						asm volatile("" ::"s"(t));
					}
					if constexpr (K == 24) asm volatile("v_writelane_b32 %0, %1, 3" : "+v"(a[k]) : "s"((uint32_t)mask));
					if constexpr (K == 25) asm volatile("v_sqrt_f64 %0, %0" : "+v"(b[k]));
					if constexpr (K == 16) {
						unsigned long long m;
						asm volatile("v_cmp_gt_f64_e64 %0, 1.0, %1" : "=s"(m) : "v"(b[k]));
						asm volatile("" ::"s"(m));
					}
				}
		}
		float acc = 0;
#pragma unroll
		for (int k = 0; k < kChains; k++) acc += a[k] + (float)b[k];
		if (acc == -1.0f) sink[0] = acc;  // keeps the chains; never true
		return;
	}
	constexpr int kChains = 32;
	constexpr bool k64 = K == 2 || K == 3 || K == 4 || K == 5 || K == 6 || K == 11 || K == 12;
	using T = typename std::conditional<k64, double, float>::type;
	constexpr int kLanes = K == 1 ? 2 : 1;  // v_pk_fma_f32 works on a pair of f32 registers
	T a[kChains][kLanes];
#pragma unroll
	for (int k = 0; k < kChains; k++)
#pragma unroll
		for (int l = 0; l < kLanes; l++) a[k][l] = static_cast<T>(seed + threadIdx.x + k + l);
	for (int i = 0; i < iters; i++) {
#pragma unroll
		for (int u = 0; u < 4; u++)
#pragma unroll
			for (int k = 0; k < kChains; k++) {
				if constexpr (K == 1) {
					asm volatile("v_pk_fma_f32 %0, %0, 0.5, 1.0 op_sel_hi:[1,0,0]"
					             : "+v"(*reinterpret_cast<HIP_vector_base<float, 2>::Native_vec_*>(&a[k][0])));
				} else {
					valu_op<K>(a[k][0]);
				}
			}
	}
	T acc = 0;
#pragma unroll
	for (int k = 0; k < kChains; k++)
#pragma unroll
		for (int l = 0; l < kLanes; l++) acc += a[k][l];
	if (acc == static_cast<T>(-1)) sink[0] = static_cast<float>(acc);  // keeps the chains; never true
}

// multi-GPU image assembly on the first device: one thread per byte of the image, each
// row copied from its owner's buffer (partition_row)
__global__ void k_deinterleave(uint8_t* dst, RowSources s, int n, int block, int64_t height, int64_t row_bytes) {
	const int64_t total = height * row_bytes;
	const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
	for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
		const int64_t r = i / row_bytes, b = i - r * row_bytes;
		int dev;
		int64_t local;
		partition_row(r, n, block, &dev, &local);
		dst[i] = s.src[dev][local * row_bytes + b];
	}
}

inline unsigned grid_for(int64_t n, int block) { return (unsigned)((n + block - 1) / block); }
// grid of the stride loops: 8 blocks (16 waves) per CU, 4 waves per SIMD
constexpr int64_t kStrideBlocks = 256 * 8;

}  // namespace

// the traversal kernels' instantiation for the scene's geometry (kMeshNone / kMeshLinear /
// kMeshBvh, DeviceScene::mesh_kind): f(std::integral_constant<int, kind>)
template <typename F>
static void by_mesh_kind(const DeviceScene& s, F f) {
	switch (s.mesh_kind) {
		case kMeshNone: f(std::integral_constant<int, kMeshNone>{}); break;
		case kMeshLinear: f(std::integral_constant<int, kMeshLinear>{}); break;
		default: f(std::integral_constant<int, kMeshBvh>{}); break;
	}
}

hipError_t launch_closest(const DeviceScene& s, const FrameGeometry& fg, int level, int64_t n, const int32_t* n_dev,
                          int remaining_depth, const RayLevel* levels_dev, DeviceCounters* ctr,
                          unsigned long long* stats, hipStream_t stream, int packet_mask, int plan_last,
                          hipEvent_t done) {
	if (n <= 0) return done ? hipEventRecord(done, stream) : hipSuccess;
	const bool packet = packet_mask & (level == 0 ? kPacketClosest0 : level == 1 ? kPacketClosestN | kPacketClosest1 : kPacketClosestN);
	const int64_t threads = (level == 0 && packet) ? tile_threads(n, fg.width) : n;
	// with a device-side count, n is an upper bound: a grid of at most kStrideBlocks
	const unsigned grid = n_dev ? (unsigned)std::min<int64_t>(grid_for(threads, kBlock), kStrideBlocks)
	                            : grid_for(threads, kBlock);
	// the counting kernels only for renders that asked for the work counts (work_stats)
	// done: recorded by the launch itself (the kernel's own completion signal), not by a marker
	// packet queued behind it: a marker between two kernels of a queue costs ~7 us
	auto go = [&](auto kernel) {
		if (done)
			hipExtLaunchKernelGGL(kernel, dim3(grid), dim3(kBlock), 0, stream, nullptr, done, 0, s, fg, level, n, n_dev,
			                      remaining_depth, plan_last, levels_dev, ctr, stats);
		else
			hipLaunchKernelGGL(kernel, dim3(grid), dim3(kBlock), 0, stream, s, fg, level, n, n_dev, remaining_depth,
			                   plan_last, levels_dev, ctr, stats);
	};
	// instantiations: packet or per lane, counting or not, by the scene's geometry (mesh_kind)
	by_mesh_kind(s, [&](auto m) {
		constexpr int M = decltype(m)::value;
		if (packet)
			level == 0 ? (s.work_stats ? go(k_closest<true, true, M, true>) : go(k_closest<true, false, M, true>))
			           : (s.work_stats ? go(k_closest<true, true, M, false>) : go(k_closest<true, false, M, false>));
		else
			level == 0 ? (s.work_stats ? go(k_closest<false, true, M, true>) : go(k_closest<false, false, M, true>))
			           : (s.work_stats ? go(k_closest<false, true, M, false>) : go(k_closest<false, false, M, false>));
	});
	return hipGetLastError();
}

static bool shadow_packet(const ShadeBatch& b, int packet_mask) {
	const int lv = b.level[0];
	return packet_mask & (lv == 0 ? kPacketShadow0 : (lv == 1 && b.n == 1) ? kPacketShadowN | kPacketShadow1 : kPacketShadowN);
}

bool shadow_can_fuse(const DeviceScene& s, const ShadeBatch& b, int packet_mask, bool per_lane) {
	return b.all_lights && (shadow_packet(b, packet_mask) || (per_lane && s.mesh_kind == kMeshLinear));
}

// grid of a device-counted batch: one thread per item of `bound` (an upper bound of its
// items, from the levels' capacities); the blocks beyond the device count exit at once
#ifndef RT_DEV_GRID_CAP
#define RT_DEV_GRID_CAP (1 << 20)
#endif
inline unsigned dev_grid(int64_t bound, int block) {
	return (unsigned)std::max<int64_t>(1, std::min<int64_t>(grid_for(bound, block), RT_DEV_GRID_CAP));
}

hipError_t launch_shadow(const DeviceScene& s, const ShadeBatch& b, const RayLevel* levels_dev, DeviceCounters* ctr,
                         unsigned long long* stats, hipStream_t stream, int packet_mask) {
	const int64_t items = b.shadow_begin[b.n];  // device-counted: an upper bound
	if (items <= 0 || s.n_nonambient <= 0) return hipSuccess;
	const unsigned grid = b.dev_counts ? dev_grid(items, kBlock) : grid_for(items, kBlock);
	auto go = [&](auto kernel) {
		hipLaunchKernelGGL(kernel, dim3(grid), dim3(kBlock), 0, stream, s, b, levels_dev, ctr, stats);
	};
	by_mesh_kind(s, [&](auto m) {
		constexpr int M = decltype(m)::value;
		if (shadow_packet(b, packet_mask))
			b.fused ? (s.work_stats ? go(k_shadow<true, true, M, 1>) : go(k_shadow<true, false, M, 1>))
			        : (s.work_stats ? go(k_shadow<true, true, M, 2>) : go(k_shadow<true, false, M, 2>));
		else if constexpr (M == kMeshLinear)  // (per lane, fused only without LBVH searches: shadow_can_fuse)
			s.work_stats ? go(k_shadow<false, true, M, 2>) : go(k_shadow<false, false, M, 2>);
		else
			s.work_stats ? go(k_shadow<false, true, M, 0>) : go(k_shadow<false, false, M, 0>);
	});
	return hipGetLastError();
}

hipError_t launch_shade(const DeviceScene& s, const ShadeBatch& b, const RayLevel* levels_dev, DeviceCounters* ctr,
                        hipStream_t stream) {
	const int64_t items = b.shade_begin[b.n];  // device-counted: an upper bound
	if (items <= 0) return hipSuccess;
	const unsigned grid = b.dev_counts ? dev_grid(items, kShadeBlock) : grid_for(items, kShadeBlock);
	hipLaunchKernelGGL(k_shade, dim3(grid), dim3(kShadeBlock), 0, stream, s, b, levels_dev, ctr);
	return hipGetLastError();
}

hipError_t launch_reduce_level(const DeviceScene& s, int64_t n, const int32_t* n_dev, const RayLevel& cur,
                               const RayLevel& next, const RayLevel* low, hipStream_t stream) {
	if (n <= 0) return hipSuccess;
	const unsigned grid = n_dev ? dev_grid(n, 256) : grid_for(n, 256);
	if (low)
		hipLaunchKernelGGL(k_reduce<2>, dim3(grid), dim3(256), 0, stream, n, n_dev, cur, next, *low, s.geoms, s.mats);
	else
		hipLaunchKernelGGL(k_reduce<1>, dim3(grid), dim3(256), 0, stream, n, n_dev, cur, next, next, s.geoms, s.mats);
	return hipGetLastError();
}

hipError_t launch_output(const DeviceScene& s, int64_t n, const FrameGeometry& fg, const RayLevel& lvl0,
                         const RayLevel* lvl1, const RayLevel* lvl2, unsigned long long* stats, hipStream_t stream,
                         DeviceCounters* ctr, const FusedOut* finish) {
	if (n <= 0) return hipSuccess;
	const FusedOut fo = finish ? *finish : FusedOut{};
	const RayLevel& l1 = lvl1 ? *lvl1 : lvl0;
	const RayLevel& l2 = lvl2 ? *lvl2 : l1;
	auto go = [&](auto kernel) {
		hipLaunchKernelGGL(kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, n, fg, lvl0, l1, l2, s.geoms, s.mats,
		                   stats, ctr, fo);
	};
	if (lvl1 && lvl2)
		go(k_output<2>);
	else if (lvl1)
		go(k_output<1>);
	else
		go(k_output<0>);
	return hipGetLastError();
}

hipError_t launch_fused(const DeviceScene& s, const FrameGeometry& fg, int level, int64_t n, const int32_t* n_dev,
                        int remaining_depth, const RayLevel* levels_dev, DeviceCounters* ctr, unsigned long long* stats,
                        hipStream_t stream, int packet_mask, int plan_last, const FusedOut& fo) {
	if (n <= 0) return hipSuccess;
	const bool packet = packet_mask & (level == 0 ? kPacketClosest0 : level == 1 ? kPacketClosestN | kPacketClosest1 : kPacketClosestN);
	const int64_t threads = (level == 0 && packet) ? tile_threads(n, fg.width) : n;
	const unsigned grid = n_dev ? (unsigned)std::min<int64_t>(grid_for(threads, kBlock), kStrideBlocks)
	                            : grid_for(threads, kBlock);
	auto go = [&](auto kernel) {
		hipLaunchKernelGGL(kernel, dim3(grid), dim3(kBlock), 0, stream, s, fg, level, n, n_dev, remaining_depth,
		                   plan_last, levels_dev, ctr, stats, fo);
	};
	by_mesh_kind(s, [&](auto m) {
		constexpr int M = decltype(m)::value;
		if (level == 0)
			packet ? go(k_fused<true, M, true>) : go(k_fused<false, M, true>);
		else
			packet ? go(k_fused<true, M, false>) : go(k_fused<false, M, false>);
	});
	return hipGetLastError();
}

hipError_t launch_stats_finish(unsigned long long* stats, DeviceCounters* ctr, unsigned long long* summary,
                               hipStream_t stream) {
	hipLaunchKernelGGL(k_stats_finish, dim3(1), dim3(kStatShards), 0, stream, stats, ctr, summary);
	return hipGetLastError();
}

// 16-byte words from (mapped pinned) host memory to the device: the scene's arrays in one
// launch, without the copy engine (api.cpp upload batch)
__global__ void k_copy16(uint4* dst, const uint4* src, int64_t n) {
	const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
	for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = src[i];
}

hipError_t launch_copy16(void* dst, const void* src, int64_t n_words, hipStream_t stream) {
	if (n_words <= 0) return hipSuccess;
	const unsigned grid = static_cast<unsigned>(std::min<int64_t>(grid_for(n_words, 256), 4096));
	hipLaunchKernelGGL(k_copy16, dim3(grid), dim3(256), 0, stream, static_cast<uint4*>(dst), static_cast<const uint4*>(src),
	                   n_words);
	return hipGetLastError();
}

hipError_t launch_normalize(int64_t n_values, double* rgb, double max_value, uint8_t* out_rgb8, hipStream_t stream) {
	if (n_values <= 0) return hipSuccess;
	const double rcp = 1.0 / max_value;  // Color3d /= scalar: multiply by the reciprocal
	hipLaunchKernelGGL(k_normalize, dim3(grid_for(n_values, 256)), dim3(256), 0, stream, n_values, rgb, rcp, out_rgb8);
	return hipGetLastError();
}

hipError_t read_phase_profile(unsigned long long* out) {
#if RT_PHASE_PROF || RT_DIAG_LANES || RT_DIAG_GEOMS || RT_DIAG_PACKET
	hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(dev::g_phase), sizeof(dev::g_phase));
	if (e != hipSuccess) return e;
	static const unsigned long long zero[4 * kPhaseSlots] = {};
	return hipMemcpyToSymbol(HIP_SYMBOL(dev::g_phase), zero, sizeof(zero));
#else
	for (int k = 0; k < 4 * kPhaseSlots; k++) out[k] = 0;
	return hipSuccess;
#endif
}

int read_wave_times(void* out, int max_records) {
#if RT_DIAG_WAVETIME
	unsigned int n = 0;
	if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(dev::g_wt_n), sizeof(n)) != hipSuccess) return -1;
	n = std::min<unsigned int>(n, dev::kWaveTimes);
	const int m = std::min<int>(static_cast<int>(n), max_records);
	if (m > 0 && hipMemcpyFromSymbol(out, HIP_SYMBOL(dev::g_wt), m * sizeof(dev::WaveTime)) != hipSuccess) return -1;
	const unsigned int zero = 0;
	if (hipMemcpyToSymbol(HIP_SYMBOL(dev::g_wt_n), &zero, sizeof(zero)) != hipSuccess) return -1;
	return m;
#else
	(void)out;
	(void)max_records;
	return 0;
#endif
}

hipError_t launch_stream_read(const void* buf, int64_t bytes, int width, unsigned long long* sink, hipStream_t stream) {
	const unsigned grid = 256 * 8;
	switch (width) {
		case 1: hipLaunchKernelGGL(k_stream_read<uint8_t>, dim3(grid), dim3(256), 0, stream, (const uint8_t*)buf, bytes, sink); break;
		case 4: hipLaunchKernelGGL(k_stream_read<uint32_t>, dim3(grid), dim3(256), 0, stream, (const uint32_t*)buf, bytes / 4, sink); break;
		case 8: hipLaunchKernelGGL(k_stream_read<uint64_t>, dim3(grid), dim3(256), 0, stream, (const uint64_t*)buf, bytes / 8, sink); break;
		default: hipLaunchKernelGGL(k_stream_read<uint4>, dim3(grid), dim3(256), 0, stream, (const uint4*)buf, bytes / 16, sink); break;
	}
	return hipGetLastError();
}

hipError_t launch_valu_peak(int iters, int kind, int waves_per_simd, void* sink, hipStream_t stream) {
	const unsigned grid = 256 * std::max(1, waves_per_simd);  // blocks of 4 waves (one per SIMD) on every CU
	float* out = static_cast<float*>(sink);
	if (kind < 0 || kind >= kValuKinds) return hipErrorInvalidValue;
	auto go = [&](auto k) {
		hipLaunchKernelGGL(k_valu_peak<decltype(k)::value>, dim3(grid), dim3(256), 0, stream, iters, 1.0f, out);
	};
	switch (kind) {
		case 0: go(std::integral_constant<int, 0>{}); break;
		case 1: go(std::integral_constant<int, 1>{}); break;
		case 2: go(std::integral_constant<int, 2>{}); break;
		case 3: go(std::integral_constant<int, 3>{}); break;
		case 4: go(std::integral_constant<int, 4>{}); break;
		case 5: go(std::integral_constant<int, 5>{}); break;
		case 6: go(std::integral_constant<int, 6>{}); break;
		case 7: go(std::integral_constant<int, 7>{}); break;
		case 8: go(std::integral_constant<int, 8>{}); break;
		case 9: go(std::integral_constant<int, 9>{}); break;
		case 10: go(std::integral_constant<int, 10>{}); break;
		case 11: go(std::integral_constant<int, 11>{}); break;
		case 12: go(std::integral_constant<int, 12>{}); break;
		case 13: go(std::integral_constant<int, 13>{}); break;
		case 14: go(std::integral_constant<int, 14>{}); break;
		case 15: go(std::integral_constant<int, 15>{}); break;
		case 16: go(std::integral_constant<int, 16>{}); break;
		case 17: go(std::integral_constant<int, 17>{}); break;
		case 18: go(std::integral_constant<int, 18>{}); break;
		case 19: go(std::integral_constant<int, 19>{}); break;
		case 20: go(std::integral_constant<int, 20>{}); break;
		case 21: go(std::integral_constant<int, 21>{}); break;
		case 22: go(std::integral_constant<int, 22>{}); break;
		case 23: go(std::integral_constant<int, 23>{}); break;
		case 24: go(std::integral_constant<int, 24>{}); break;
		default: go(std::integral_constant<int, 25>{}); break;
	}
	return hipGetLastError();
}

hipError_t launch_deinterleave(uint8_t* dst, const RowSources& s, int n, int block, int64_t height, int64_t row_bytes,
                               hipStream_t stream) {
	const int64_t total = height * row_bytes;
	if (total <= 0) return hipSuccess;
	hipLaunchKernelGGL(k_deinterleave, dim3((unsigned)std::min<int64_t>(grid_for(total, 256), 8192)), dim3(256), 0,
	                   stream, dst, s, n, block, height, row_bytes);
	return hipGetLastError();
}

hipError_t launch_selftest_math(int op, const double* x, const double* y, double* out, int64_t n, hipStream_t stream) {
	if (n <= 0) return hipSuccess;
	hipLaunchKernelGGL(k_selftest, dim3(grid_for(n, 256)), dim3(256), 0, stream, op, x, y, out, n);
	return hipGetLastError();
}

}  // namespace rtamd
