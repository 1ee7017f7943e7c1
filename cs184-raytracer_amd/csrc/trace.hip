// HIP kernels of the ray-trace hot path, gfx950 (MI355X).
//
// Wavefront formulation of the reference's recursive Scene::traceRay (scene.cpp:61-140):
// level L holds every ray of recursion depth L; one launch per level finds the closest
// hit (castRay, scene.cpp:142-167), shades it with shadow rays in light order, and
// appends its refraction/reflection children to level L+1 through a wave-aggregated
// atomic.  Colours are then reduced bottom-up (reduce kernel) in the reference's
// addition order: colour = (local + refraction) + reflection * kr (scene.cpp:127,134).
//
// Numerics: binary64 throughout, compiled with -ffp-contract=off, every expression in
// the reference's Eigen 3.2.2 evaluation order:
//   Vector4d dot   (a0 b0 + a2 b2) + (a1 b1 + a3 b3); the w products are exact zeros for
//                  every direction/normal and are dropped (see dot4z)
//   Vector3d norm  a0^2 + (a1^2 + a2^2)
//   T * v          rows sequential ((m0 v0 + m1 v1) + m2 v2) + m3 v3
//   invT * n       (M0k n0 + M2k n2) + (M1k n1 + M3k n3)
//   normalized()   division by the norm; normalize() multiplies by the reciprocal
#include "trace.h"
#include "glibc_pow.h"
#include <cmath>

namespace rtamd {
namespace {

constexpr int kBlock = 128;  // 2 waves; LDS traversal stack = kStackDepth x kBlock x 4 B

struct V3 {
	double x, y, z;
};
__device__ __forceinline__ V3 mk(double x, double y, double z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator-(V3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ V3 operator*(double s, V3 a) { return mk(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ V3 load3(const double* p) { return mk(p[0], p[1], p[2]); }

// Vector4d::dot of two vectors whose w is (+-)0: the w term contributes an exact zero
__device__ __forceinline__ double dot4z(V3 a, V3 b) { return (a.x * b.x + a.z * b.z) + a.y * b.y; }
// Vector4d::squaredNorm with w == 0: exact (y^2 + 0 == y^2)
__device__ __forceinline__ double sq4(V3 a) { return (a.x * a.x + a.z * a.z) + a.y * a.y; }
// isZero(): all |c| <= 1e-12 (w is zero)
__device__ __forceinline__ bool is_zero3(V3 a) {
	return fabs(a.x) <= 1e-12 && fabs(a.y) <= 1e-12 && fabs(a.z) <= 1e-12;
}
__device__ __forceinline__ V3 div3(V3 a, double n) { return mk(a.x / n, a.y / n, a.z / n); }

__device__ __forceinline__ V3 xf_point(const double (*m)[4], V3 p) {
	return mk(((m[0][0] * p.x + m[0][1] * p.y) + m[0][2] * p.z) + m[0][3],
	          ((m[1][0] * p.x + m[1][1] * p.y) + m[1][2] * p.z) + m[1][3],
	          ((m[2][0] * p.x + m[2][1] * p.y) + m[2][2] * p.z) + m[2][3]);
}
__device__ __forceinline__ V3 xf_dir(const double (*m)[4], V3 d) {
	return mk((m[0][0] * d.x + m[0][1] * d.y) + m[0][2] * d.z, (m[1][0] * d.x + m[1][1] * d.y) + m[1][2] * d.z,
	          (m[2][0] * d.x + m[2][1] * d.y) + m[2][2] * d.z);
}
// inverseTransform().matrix().transpose() * n (geometry.cpp:40)
__device__ __forceinline__ V3 xf_normal(const double (*m)[4], V3 n) {
	return mk((m[0][0] * n.x + m[2][0] * n.z) + m[1][0] * n.y, (m[0][1] * n.x + m[2][1] * n.z) + m[1][1] * n.y,
	          (m[0][2] * n.x + m[2][2] * n.z) + m[1][2] * n.y);
}

__device__ __forceinline__ void raise_error(DeviceCounters* c, int code) { atomicCAS(&c->error, 0, code); }

// Ray::direction(dir) (rtbase.h:17-23): reject |c| <= 1e-12, then dir.normalized()
__device__ __forceinline__ V3 ray_dir(V3 d, DeviceCounters* c) {
	if (is_zero3(d)) raise_error(c, DERR_NO_DIRECTION);
	return div3(d, sqrt(sq4(d)));
}

// Matrix3d::determinant of the matrix with columns c0, c1, c2 (LU/Determinant.h:61-69)
__device__ __forceinline__ double det3(V3 c0, V3 c1, V3 c2) {
	return (c0.x * (c1.y * c2.z - c2.y * c1.z) - c1.x * (c0.y * c2.z - c2.y * c0.z)) + c2.x * (c0.y * c1.z - c1.y * c0.z);
}

// hitsBoundingBox, verbatim (geometry.cpp:5-29)
__device__ bool hits_bounding_box(V3 o, V3 d, const double* mn, const double* mx) {
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

// Per-lane work counters, reduced once per wave at the end of k_trace (algorithmic
// bytes/flops for the roofline).
struct WorkStats {
	uint32_t nodes, tris, cands, spheres;
};

struct MeshBest {
	double dist;
	int32_t face;   // global face index, -1 = none
	int32_t id;     // reference order within the mesh (tie-break)
	double a, b;
	V3 n;
};

// One iteration of the face loop of geometry.cpp:78-124.  Accepts the face when it is
// strictly closer, or equally close with a smaller reference index: over any visiting
// order this selects the same face as the reference's in-order scan.
template <bool kAnyHit>
__device__ __forceinline__ bool test_face(const DeviceScene& S, int32_t f, V3 o, V3 d, V3 nd, double dn,
                                          bool reverse, MeshBest& best, WorkStats& ws) {
	ws.tris++;
	const DFaceGeo* F = S.fgeo + f;
	const V3 p0 = load3(F->p0), va = load3(F->va), vb = load3(F->vb);
	const V3 rhs = o - p0;
	const double D = det3(va, vb, nd);
	if (D == 0) return false;
	const double a = det3(rhs, vb, nd) / D;
	if (a < 0 || a > 1) return false;
	const double b = det3(va, rhs, nd) / D;
	if (b < 0 || a + b > 1) return false;
	const double t = det3(va, vb, rhs) / D;
	if (t < 0) return false;
	const double dist = t * dn;
	const int32_t id = S.fid[f];
	if (!(dist < best.dist || (dist == best.dist && id < best.id))) return false;
	ws.cands++;
	const DFaceNrm* N = S.fnrm + f;
	const double w0 = (1.0 - a) - b;
	const V3 n0 = load3(N->n0), n1 = load3(N->n1), n2 = load3(N->n2);
	const V3 tn = mk((w0 * n0.x + a * n1.x) + b * n2.x, (w0 * n0.y + a * n1.y) + b * n2.y,
	                 (w0 * n0.z + a * n1.z) + b * n2.z);
	const bool front = dot4z(tn, d) < 0;
	if (!front ^ reverse) return false;
	best.dist = dist;
	best.face = f;
	best.id = id;
	best.a = a;
	best.b = b;
	best.n = tn;
	return kAnyHit;
}

// Slab test of a padded LBVH child box; conservative (never prunes a box the
// reference's scan could hit): the interval is widened by a relative 1e-9.
__device__ __forceinline__ bool slab(const double* lo, const double* hi, V3 o, V3 inv, double tlimit, double& tnear) {
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

__device__ __forceinline__ double prune_limit(double best_dist) { return best_dist * (1.0 + 4e-9); }

// Mesh::calculateIntNormInObjSpace (geometry.cpp:69-126) with an LBVH in place of the
// linear scan for large meshes.  kAnyHit: the caller only needs "some face passes"
// (shadow ray towards a directional light, distToLight = inf).
template <bool kAnyHit>
__device__ bool mesh_hit(const DeviceScene& S, const DGeom& G, V3 o, V3 d, bool reverse, V3& Po, V3& No,
                         int32_t* stack, DeviceCounters* ctr, WorkStats& ws) {
	if (G.gate && !hits_bounding_box(o, d, G.bb_min, G.bb_max)) return false;
	const double dn = sqrt(d.x * d.x + (d.y * d.y + d.z * d.z));  // Vector3d::norm
	const V3 nd = -d;
	MeshBest best;
	best.dist = INFINITY;
	best.face = -1;
	best.id = 0x7fffffff;
	if (G.bvh_root < 0) {
		for (int32_t f = G.face_begin; f < G.face_begin + G.face_count; f++)
			if (test_face<kAnyHit>(S, f, o, d, nd, dn, reverse, best, ws)) return true;
	} else {
		const V3 inv = mk(1.0 / (d.x != 0.0 ? d.x : copysign(1e-300, d.x)),
		                  1.0 / (d.y != 0.0 ? d.y : copysign(1e-300, d.y)),
		                  1.0 / (d.z != 0.0 ? d.z : copysign(1e-300, d.z)));
		int32_t node = G.bvh_root;
		int sp = 0;
		for (;;) {
			ws.nodes++;
			const DBvhNode* N = S.nodes + node;
			double tn0, tn1;
			const double lim = prune_limit(best.dist);
			const bool h0 = slab(N->lo[0], N->hi[0], o, inv, lim, tn0);
			const bool h1 = slab(N->lo[1], N->hi[1], o, inv, lim, tn1);
			const int first = (h0 && h1 && tn1 < tn0) ? 1 : 0;
			int32_t next = -1;
#pragma unroll
			for (int k = 0; k < 2; k++) {
				const int c = first ^ k;
				if (!(c ? h1 : h0)) continue;
				if (k == 1 && (c ? tn1 : tn0) > prune_limit(best.dist)) continue;
				const int32_t cf = N->first[c], cc = N->count[c];
				if (cc > 0) {
					const int32_t f0 = G.face_begin + cf;
					for (int32_t f = f0; f < f0 + cc; f++)
						if (test_face<kAnyHit>(S, f, o, d, nd, dn, reverse, best, ws)) return true;
				} else if (next < 0) {
					next = cf;
				} else if (sp < kStackDepth) {
					stack[sp++ * kBlock] = cf;
				} else {
					raise_error(ctr, DERR_STACK);
				}
			}
			if (next < 0) {
				if (sp == 0) break;
				next = stack[--sp * kBlock];
			}
			node = next;
		}
	}
	if (best.face < 0) return false;
	const DFaceGeo* F = S.fgeo + best.face;
	const V3 p0 = load3(F->p0), va = load3(F->va), vb = load3(F->vb);
	// face.points_[0] + vec4dFrom3d(a * va + b * vb)
	Po = mk(p0.x + (best.a * va.x + best.b * vb.x), p0.y + (best.a * va.y + best.b * vb.y),
	        p0.z + (best.a * va.z + best.b * vb.z));
	No = best.n;
	return true;
}

// Sphere::calculateIntNormInObjSpace (geometry.cpp:47-67)
__device__ __forceinline__ bool sphere_hit(const DGeom& G, V3 o, V3 d, bool reverse, V3& Po, V3& No) {
	const V3 c = load3(G.center);
	const V3 oc = o - c;
	const double a = sq4(d);
	const double b = 2 * dot4z(d, oc);
	const double cc = sq4(oc) - G.rr;
	const double disc = b * b - (4 * a) * cc;
	if (disc < 0) return false;
	const double t = reverse ? (-b + sqrt(disc)) / (2 * a) : (-b - sqrt(disc)) / (2 * a);
	if (t < 0) return false;
	Po = o + t * d;
	No = Po - c;
	return true;
}

// Scene::castRay (scene.cpp:142-167).  kShadow: return as soon as one geometry's hit
// lies within shadow_limit (occluded iff min over geometries <= distToLight).
template <bool kShadow>
__device__ bool cast_ray(const DeviceScene& S, V3 o, V3 d, bool reverse, double shadow_limit, double& best_dist,
                         int& best_geom, V3& hitP, V3& hitNobj, int32_t* stack, DeviceCounters* ctr,
                         WorkStats& ws) {
	bool found = false;
	for (int g = 0; g < S.n_geoms; g++) {
		const DGeom& G = S.geoms[g];
		// Geometry::calculateIntersectionNormal (geometry.cpp:31-45): object-space ray
		const V3 oo = xf_point(G.inv, o);
		const V3 dd = ray_dir(xf_dir(G.inv, d), ctr);
		V3 Po, No;
		bool hit;
		if (G.kind == DGEOM_SPHERE) {
			ws.spheres++;
			hit = sphere_hit(G, oo, dd, reverse, Po, No);
		}
		else if (kShadow && shadow_limit == INFINITY)
			hit = mesh_hit<true>(S, G, oo, dd, reverse, Po, No, stack, ctr, ws);
		else
			hit = mesh_hit<false>(S, G, oo, dd, reverse, Po, No, stack, ctr, ws);
		if (!hit) continue;
		if (kShadow && shadow_limit == INFINITY) return true;  // any finite hit is <= inf
		const V3 Pw = xf_point(G.fwd, Po);
		const double dist = sqrt(sq4(Pw - o));
		if (kShadow) {
			if (dist <= shadow_limit) return true;
			continue;
		}
		if (found && dist >= best_dist) continue;
		found = true;
		best_dist = dist;
		best_geom = g;
		hitP = Pw;
		hitNobj = No;
	}
	return found;
}

// Camera::calculateViewingRay (rtbase.h:74-84) for pixel (r, c) (scene.cpp:26-30)
__device__ __forceinline__ void primary_ray(const DCamera& cam, int r, int c, int W, int H, V3& o, V3& d,
                                            DeviceCounters* ctr) {
	const double rF = (r + 0.5) / H;
	const double cF = (c + 0.5) / W;
	const double rI = 1.0 - rF, cI = 1.0 - cF;
	double p[4];
#pragma unroll
	for (int k = 0; k < 4; k++)
		p[k] = cF * (rF * cam.lr[k] + rI * cam.ur[k]) + cI * (rF * cam.ll[k] + rI * cam.ul[k]);
	if (p[3] - cam.eye[3] != 0) raise_error(ctr, DERR_POINT_DIRECTION);
	o = load3(cam.eye);
	d = ray_dir(mk(p[0] - cam.eye[0], p[1] - cam.eye[1], p[2] - cam.eye[2]), ctr);
}

// std::max(x, 0.0)
__device__ __forceinline__ double max0(double x) { return (x < 0.0) ? 0.0 : x; }

__global__ void __launch_bounds__(kBlock) k_trace(DeviceScene S, FrameGeometry fg, int level, int64_t n, int remaining,
                                                  RayLevel cur, RayLevel next, DeviceCounters* ctr) {
	__shared__ int32_t stack_mem[kStackDepth * kBlock];
	int32_t* stack = stack_mem + threadIdx.x;
	const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
	const bool active = i < n;

	V3 o = mk(0, 0, 0), d = mk(0, 0, 1);
	bool inside = false;
	if (active) {
		if (level == 0) {
			const int64_t row_ord = fg.chunk_row0 + i / fg.width;
			const int r = fg.row_begin + (int)row_ord * fg.row_step;
			const int c = (int)(i % fg.width);
			primary_ray(S.cam, r, c, fg.width, fg.height, o, d, ctr);
		} else {
			o = mk(cur.ox[i], cur.oy[i], cur.oz[i]);
			d = mk(cur.dx[i], cur.dy[i], cur.dz[i]);
			inside = cur.inside[i];
		}
	}

	WorkStats ws{0, 0, 0, 0};
	double col[3] = {0.0, 0.0, 0.0};
	bool spawn_refr = false, spawn_refl = false;
	V3 P = mk(0, 0, 0), refr_d = mk(0, 0, 0), refl_d = mk(0, 0, 0);
	double kr[3] = {0, 0, 0};
	bool hit = false;
	if (active) {
		double dist = 0;
		int gi = -1;
		V3 Nobj;
		hit = cast_ray<false>(S, o, d, inside, 0.0, dist, gi, P, Nobj, stack, ctr, ws);
		if (hit && fg.intersection_only) {
			const double v = 1.0 / (dist * dist);  // scene.cpp:69-70
			col[0] = col[1] = col[2] = v;
		} else if (hit) {
			const DGeom& G = S.geoms[gi];
			V3 N = xf_normal(G.inv, Nobj);
			if (G.flip) N = -N;
			if (inside) N = -N;
			const double rn = 1.0 / sqrt(sq4(N));  // targetNormal.normalize() (scene.cpp:114)
			N = rn * N;
			const DMaterial& M = S.mats[G.mat];
			for (int li = 0; li < S.n_lights; li++) {
				const DLight& L = S.lights[li];
				if (L.kind == DLIGHT_AMBIENT) {
#pragma unroll
					for (int k = 0; k < 3; k++) col[k] = col[k] + (1.0 * L.color[k]) * M.ka[k];
					continue;
				}
				const bool point = L.kind == DLIGHT_POINT;
				const V3 lv = load3(L.vec);
				const V3 toL = point ? lv - P : -lv;
				const V3 Ld = ray_dir(toL, ctr);
				const double nl = dot4z(N, Ld);
				const bool lrev = nl < 0;
				const double dL = point ? sqrt(sq4(lv - P)) : INFINITY;
				double dummy_d;
				int dummy_g;
				V3 dP, dN;
				if (cast_ray<true>(S, P, Ld, lrev ^ inside, dL, dummy_d, dummy_g, dP, dN, stack, ctr, ws)) continue;
				const double fall = point ? glibc_pow(dL, -L.falloff) : 1.0;
				double att[3];
#pragma unroll
				for (int k = 0; k < 3; k++) att[k] = point ? fall * L.color[k] : L.color[k];
				const double diff = max0(nl);
#pragma unroll
				for (int k = 0; k < 3; k++) col[k] = col[k] + (diff * att[k]) * M.kd[k];
				const V3 R = (2 * nl) * N - Ld;
				const double spec = glibc_pow(max0(-dot4z(d, R)), M.ns);
#pragma unroll
				for (int k = 0; k < 3; k++) col[k] = col[k] + (spec * att[k]) * M.ks[k];
			}
			if (remaining > 0) {  // bounce (scene.cpp:114-136)
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
		}
	}

	// children -> level + 1: one atomic per wave (ballot prefix counts)
	const unsigned long long m_refr = __ballot(spawn_refr), m_refl = __ballot(spawn_refl);
	const unsigned long long m_hit = __ballot(hit && !fg.intersection_only);
	const int lane = __lane_id();
	const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
	const int total = __popcll(m_refr) + __popcll(m_refl);
	int base = 0;
	if (lane == 0) {
		if (total) base = atomicAdd(&ctr->next_count, total);
		if (m_hit) atomicAdd(&ctr->hits, (unsigned long long)__popcll(m_hit));
		if (m_refl) atomicAdd(&ctr->refl, (unsigned long long)__popcll(m_refl));
		if (m_refr) atomicAdd(&ctr->refr, (unsigned long long)__popcll(m_refr));
	}
	base = __shfl(base, 0);
	// work counters: one wave reduction, one atomic per counter per wave
	unsigned long long w4[4] = {ws.nodes, ws.tris, ws.cands, ws.spheres};
#pragma unroll
	for (int k = 0; k < 4; k++) {
		for (int o = 32; o > 0; o >>= 1) w4[k] += __shfl_xor(w4[k], o);
	}
	if (lane == 0) {
		atomicAdd(&ctr->node_visits, w4[0]);
		atomicAdd(&ctr->tri_tests, w4[1]);
		atomicAdd(&ctr->candidates, w4[2]);
		atomicAdd(&ctr->sphere_tests, w4[3]);
	}
	if (!active) return;
	int32_t refr_idx = -1, refl_idx = -1;
	const int off = __popcll(m_refr & below) + __popcll(m_refl & below);
	if (spawn_refr) {
		refr_idx = base + off;
		next.ox[refr_idx] = P.x;
		next.oy[refr_idx] = P.y;
		next.oz[refr_idx] = P.z;
		next.dx[refr_idx] = refr_d.x;
		next.dy[refr_idx] = refr_d.y;
		next.dz[refr_idx] = refr_d.z;
		next.inside[refr_idx] = !inside;
	}
	if (spawn_refl) {
		refl_idx = base + off + (spawn_refr ? 1 : 0);
		next.ox[refl_idx] = P.x;
		next.oy[refl_idx] = P.y;
		next.oz[refl_idx] = P.z;
		next.dx[refl_idx] = refl_d.x;
		next.dy[refl_idx] = refl_d.y;
		next.dz[refl_idx] = refl_d.z;
		next.inside[refl_idx] = inside;
		cur.kr[i] = kr[0];
		cur.kg[i] = kr[1];
		cur.kb[i] = kr[2];
	}
	cur.cr[i] = col[0];
	cur.cg[i] = col[1];
	cur.cb[i] = col[2];
	cur.child_refr[i] = refr_idx;
	cur.child_refl[i] = refl_idx;
}

// colour = (local + refraction) + reflection * kr, in place (scene.cpp:127,134)
__global__ void k_reduce(int64_t n, RayLevel cur, RayLevel next) {
	const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const int32_t t = cur.child_refr[i], r = cur.child_refl[i];
	if (t < 0 && r < 0) return;
	double c0 = cur.cr[i], c1 = cur.cg[i], c2 = cur.cb[i];
	if (t >= 0) {
		c0 = c0 + next.cr[t];
		c1 = c1 + next.cg[t];
		c2 = c2 + next.cb[t];
	}
	if (r >= 0) {
		c0 = c0 + next.cr[r] * cur.kr[i];
		c1 = c1 + next.cg[r] * cur.kg[i];
		c2 = c2 + next.cb[r] * cur.kb[i];
	}
	cur.cr[i] = c0;
	cur.cg[i] = c1;
	cur.cb[i] = c2;
}

// writers.cpp:4-9: (uint8)(min(max(v,0),1) * 255), NaN -> 0
__device__ __forceinline__ uint8_t to_u8(double v) {
	v = (1.0 < v) ? 1.0 : v;
	v = (v < 0.0) ? 0.0 : v;
	v = v * 255.0;
	return (v == v) ? (uint8_t)(int)v : (uint8_t)0;
}

__global__ void k_output(int64_t n, RayLevel lvl0, double* out, uint8_t* out8, int32_t io, DeviceCounters* ctr) {
	const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
	double v[3] = {0, 0, 0};
	if (i < n) {
		v[0] = lvl0.cr[i];
		v[1] = lvl0.cg[i];
		v[2] = lvl0.cb[i];
		if (out) {
			out[i * 3 + 0] = v[0];
			out[i * 3 + 1] = v[1];
			out[i * 3 + 2] = v[2];
		}
		if (out8 && !io) {
			out8[i * 3 + 0] = to_u8(v[0]);
			out8[i * 3 + 1] = to_u8(v[1]);
			out8[i * 3 + 2] = to_u8(v[2]);
		}
	}
	if (io) {  // running max of maxCoeff over positive doubles (bit order == value order)
		const double m = (i < n) ? fmax(fmax(v[0], v[1]), v[2]) : 0.0;
		unsigned long long bits = (m > 0.0) ? (unsigned long long)__double_as_longlong(m) : 0ull;
		for (int off = 32; off > 0; off >>= 1) {
			const unsigned long long o = __shfl_xor(bits, off);
			bits = o > bits ? o : bits;
		}
		if (__lane_id() == 0 && bits) atomicMax(&ctr->max_bits, bits);
	}
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
	if (op == 0)
		out[i] = glibc_pow(x[i], y[i]);
	else if (op == 1)
		out[i] = sqrt(x[i]);
	else
		out[i] = x[i] / y[i];
}

inline unsigned grid_for(int64_t n, int block) { return (unsigned)((n + block - 1) / block); }

}  // namespace

hipError_t launch_trace_level(const DeviceScene& s, const FrameGeometry& fg, int level, int64_t n, int remaining_depth,
                              const RayLevel& cur, const RayLevel& next, DeviceCounters* ctr, hipStream_t stream) {
	if (n <= 0) return hipSuccess;
	hipLaunchKernelGGL(k_trace, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, stream, s, fg, level, n, remaining_depth,
	                   cur, next, ctr);
	return hipGetLastError();
}

hipError_t launch_reduce_level(int64_t n, const RayLevel& cur, const RayLevel& next, hipStream_t stream) {
	if (n <= 0) return hipSuccess;
	hipLaunchKernelGGL(k_reduce, dim3(grid_for(n, 256)), dim3(256), 0, stream, n, cur, next);
	return hipGetLastError();
}

hipError_t launch_output(int64_t n, const RayLevel& lvl0, double* out_rgb, uint8_t* out_rgb8, int32_t io,
                         DeviceCounters* ctr, hipStream_t stream) {
	if (n <= 0) return hipSuccess;
	hipLaunchKernelGGL(k_output, dim3(grid_for(n, 256)), dim3(256), 0, stream, n, lvl0, out_rgb, out_rgb8, io, ctr);
	return hipGetLastError();
}

hipError_t launch_normalize(int64_t n_values, double* rgb, double max_value, uint8_t* out_rgb8, hipStream_t stream) {
	if (n_values <= 0) return hipSuccess;
	const double rcp = 1.0 / max_value;  // Color3d /= scalar: multiply by the reciprocal
	hipLaunchKernelGGL(k_normalize, dim3(grid_for(n_values, 256)), dim3(256), 0, stream, n_values, rgb, rcp, out_rgb8);
	return hipGetLastError();
}

hipError_t launch_selftest_math(int op, const double* x, const double* y, double* out, int64_t n, hipStream_t stream) {
	if (n <= 0) return hipSuccess;
	hipLaunchKernelGGL(k_selftest, dim3(grid_for(n, 256)), dim3(256), 0, stream, op, x, y, out, n);
	return hipGetLastError();
}

}  // namespace rtamd
