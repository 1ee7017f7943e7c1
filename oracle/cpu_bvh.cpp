// MEASUREMENT INFRASTRUCTURE ONLY — never linked into the product, never the checker.
//
// Same-algorithm CPU baseline (SURVEY.md §7 H6, §8d "vs a CPU BVH build"): the reference
// is a brute-force face loop, so the GPU/reference ratio mostly measures the algorithm
// change.  This program runs the HIP path's algorithm on the host cores instead: the
// product's own host ingest and per-mesh LBVH (cs184-raytracer_amd/csrc/scene_host.cpp,
// bvh.cpp), world-box culling, the any-hit shadow search with its exact early-outs and the
// zero-Phong-term decision (intersect.h, trace.hip k_shadow), evaluated per pixel
// recursively like scene.cpp:61-140 with one thread per core over a dynamic row queue.
// Node boxes are tested in binary64 (the kernels use fp32 with an origin shift; both are
// conservative against the same padded boxes, so both select the reference's faces).
// The image must equal the oracle's bit for bit (tests/test_cpu_bvh.py); bench.py reports
// its rate beside the reference's as cpu_baseline.same_algorithm.
//
// usage: cpu_bvh_cli scene.rti W H bdepth threads row_begin row_end row_step out.raw
// prints {"trace_rays": ..., "shadow_rays": ..., "render_s": ..., "setup_s": ...}
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>
#include "../cs184-raytracer_amd/csrc/bvh.h"
#include "../cs184-raytracer_amd/csrc/scene_host.h"

using namespace rtamd;

namespace {

struct V3 {
	double x, y, z;
};
V3 mk(double x, double y, double z) { return V3{x, y, z}; }
V3 operator+(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
V3 operator-(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
V3 operator-(V3 a) { return mk(-a.x, -a.y, -a.z); }
V3 operator*(double s, V3 a) { return mk(s * a.x, s * a.y, s * a.z); }
template <typename P>
V3 load3(const P* p) {
	return mk(p[0], p[1], p[2]);
}
// the evaluation orders of intersect.h (Eigen 3.2.2)
double dot4z(V3 a, V3 b) { return (a.x * b.x + a.z * b.z) + a.y * b.y; }
double sq4(V3 a) { return (a.x * a.x + a.z * a.z) + a.y * a.y; }
bool is_zero3(V3 a) { return std::fabs(a.x) <= 1e-12 && std::fabs(a.y) <= 1e-12 && std::fabs(a.z) <= 1e-12; }
V3 div3(V3 a, double n) { return mk(a.x / n, a.y / n, a.z / n); }
V3 xf_point(const double (*m)[4], V3 p) {
	return mk(((m[0][0] * p.x + m[0][1] * p.y) + m[0][2] * p.z) + m[0][3],
	          ((m[1][0] * p.x + m[1][1] * p.y) + m[1][2] * p.z) + m[1][3],
	          ((m[2][0] * p.x + m[2][1] * p.y) + m[2][2] * p.z) + m[2][3]);
}
V3 xf_dir(const double (*m)[4], V3 d) {
	return mk((m[0][0] * d.x + m[0][1] * d.y) + m[0][2] * d.z, (m[1][0] * d.x + m[1][1] * d.y) + m[1][2] * d.z,
	          (m[2][0] * d.x + m[2][1] * d.y) + m[2][2] * d.z);
}
V3 xf_normal(const double (*m)[4], V3 n) {
	return mk((m[0][0] * n.x + m[2][0] * n.z) + m[1][0] * n.y, (m[0][1] * n.x + m[2][1] * n.z) + m[1][1] * n.y,
	          (m[0][2] * n.x + m[2][2] * n.z) + m[1][2] * n.y);
}
std::atomic<int> g_error{0};
V3 ray_dir(V3 d) {
	if (is_zero3(d)) g_error = 1;
	return div3(d, std::sqrt(sq4(d)));
}
double det3(V3 c0, V3 c1, V3 c2) {
	return (c0.x * (c1.y * c2.z - c2.y * c1.z) - c1.x * (c0.y * c2.z - c2.y * c0.z)) + c2.x * (c0.y * c1.z - c1.y * c0.z);
}
bool hits_bounding_box(V3 o, V3 d, const double* mn, const double* mx) {  // geometry.cpp:5-29
	const double oa[3] = {o.x, o.y, o.z}, da[3] = {d.x, d.y, d.z};
	for (int axis = 0; axis < 3; axis++)
		for (int bn = 0; bn < 2; bn++) {
			const double mag = da[axis];
			if (mag == 0.0) continue;
			const double t = ((bn ? mx : mn)[axis] - oa[axis]) / mag;
			if (t < 0) continue;
			bool inside = true;
			for (int a2 = 0; a2 < 3; a2++) {
				if (a2 == axis) continue;
				const double p = oa[a2] + t * da[a2];
				if (p < mn[a2] || p > mx[a2]) inside = false;
			}
			if (inside) return true;
		}
	return false;
}

const FlatScene* S;
// LBVH work of this thread (node visits = nodes whose two child boxes were tested; face tests)
thread_local long long t_nodes = 0, t_tris = 0;

struct MeshBest {
	double dist;
	int32_t face, id;
	double a, b;
};

V3 face_normal(int32_t f, double a, double b) {
	const DFaceNrm& N = S->face_nrm[f];
	const double w0 = (1.0 - a) - b;
	const V3 n0 = load3(N.n0), n1 = load3(N.n1), n2 = load3(N.n2);
	return mk((w0 * n0.x + a * n1.x) + b * n2.x, (w0 * n0.y + a * n1.y) + b * n2.y, (w0 * n0.z + a * n1.z) + b * n2.z);
}

// geometry.cpp:78-124, one face; same acceptance as intersect.h test_face
bool test_face(bool any_hit, int32_t f, V3 o, V3 d, V3 nd, double dn, bool reverse, double any_limit, MeshBest& best) {
	t_tris++;
	const DFaceGeo& F = S->face_geo[f];
	const V3 p0 = load3(F.p0), va = load3(F.va), vb = load3(F.vb);
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
	if (!(dist < best.dist || (dist == best.dist && F.id < best.id))) return false;
	const bool front = dot4z(face_normal(f, a, b), d) < 0;
	if (!front ^ reverse) return false;
	best = MeshBest{dist, f, F.id, a, b};
	return any_hit && dist < any_limit;
}

template <typename P>
bool slab(const P* lo, const P* hi, V3 o, V3 inv, double tlimit, double& tnear) {
	const double tx0 = (lo[0] - o.x) * inv.x, tx1 = (hi[0] - o.x) * inv.x;
	const double ty0 = (lo[1] - o.y) * inv.y, ty1 = (hi[1] - o.y) * inv.y;
	const double tz0 = (lo[2] - o.z) * inv.z, tz1 = (hi[2] - o.z) * inv.z;
	double tmin = std::fmax(std::fmax(std::fmin(tx0, tx1), std::fmin(ty0, ty1)), std::fmin(tz0, tz1));
	double tmax = std::fmin(std::fmin(std::fmax(tx0, tx1), std::fmax(ty0, ty1)), std::fmax(tz0, tz1));
	tmin -= 1e-9 * std::fabs(tmin);
	tmax += 1e-9 * std::fabs(tmax);
	tnear = tmin;
	return tmax >= tmin && tmax >= 0.0 && tmin <= tlimit;
}
double safe_rcp(double x) { return 1.0 / (std::fabs(x) < 1e-300 ? std::copysign(1e-300, x) : x); }
V3 safe_inv(V3 d) { return mk(safe_rcp(d.x), safe_rcp(d.y), safe_rcp(d.z)); }
double prune_limit(double best) { return best * (1.0 + 4e-9); }

// Mesh search (intersect.h mesh_search): LBVH near-first with an explicit stack, or the
// linear scan for small meshes.  Returns the reference's face, or (any_hit) true as soon
// as a face within any_limit passes (settled).
bool mesh_search(bool any_hit, const DGeom& G, V3 o, V3 d, bool reverse, double any_limit, double prune_cap,
                 MeshBest& best, bool& settled) {
	settled = false;
	const double dn = std::sqrt(d.x * d.x + (d.y * d.y + d.z * d.z));
	const V3 nd = -d;
	best = MeshBest{INFINITY, -1, 0x7fffffff, 0, 0};
	if (G.bvh_root < 0) {
		for (int32_t f = G.face_begin; f < G.face_begin + G.face_count; f++)
			if (test_face(any_hit, f, o, d, nd, dn, reverse, any_limit, best)) return settled = true;
		return best.face >= 0;
	}
	const V3 inv = safe_inv(d);
	int32_t stack[64];
	int sp = 0;
	int32_t ref = G.bvh_root;  // >= 0 node, <= -2 leaf (-2 - (first << 3 | count))
	for (;;) {
		if (ref >= 0) {
			const DBvhNode& N = S->nodes[ref];
			t_nodes++;
			const double lim = std::fmin(prune_limit(best.dist), prune_cap);
			double t0, t1;
			const bool h0 = slab(N.lo[0], N.hi[0], o, inv, lim, t0), h1 = slab(N.lo[1], N.hi[1], o, inv, lim, t1);
			auto code = [&](int c) { return N.count[c] > 0 ? -2 - ((N.first[c] << 3) | N.count[c]) : N.first[c]; };
			if (h0 && h1) {
				const int c = t1 < t0 ? 1 : 0;
				stack[sp++] = code(c ^ 1);
				ref = code(c);
				continue;
			}
			if (h0 || h1) {
				ref = code(h1 ? 1 : 0);
				continue;
			}
		} else {
			const int32_t c = -2 - ref;
			const int32_t f0 = G.face_begin + (c >> 3), f1 = f0 + (c & 7);
			for (int32_t f = f0; f < f1; f++)
				if (test_face(any_hit, f, o, d, nd, dn, reverse, any_limit, best)) return settled = true;
		}
		if (sp == 0) break;
		ref = stack[--sp];
	}
	return best.face >= 0;
}

// the reference's hitsBoundingBox gate (geometry.cpp:72), evaluated for a reported hit
bool mesh_hit(bool any_hit, const DGeom& G, V3 o, V3 d, bool reverse, double any_limit, double prune_cap,
              MeshBest& best, bool& settled) {
	if (!mesh_search(any_hit, G, o, d, reverse, any_limit, prune_cap, best, settled)) return false;
	if (G.gate && !hits_bounding_box(o, d, G.bb_min, G.bb_max)) return settled = false;
	return true;
}

bool sphere_hit(const DGeom& G, V3 o, V3 d, bool reverse, double& t) {  // geometry.cpp:47-67
	const V3 oc = o - load3(G.center);
	const double a = sq4(d), b = 2 * dot4z(d, oc), cc = sq4(oc) - G.rr;
	const double disc = b * b - (4 * a) * cc;
	if (disc < 0) return false;
	t = reverse ? (-b + std::sqrt(disc)) / (2 * a) : (-b - std::sqrt(disc)) / (2 * a);
	return t >= 0;
}

V3 face_point(int32_t f, double a, double b) {
	const DFaceGeo& F = S->face_geo[f];
	const V3 p0 = load3(F.p0), va = load3(F.va), vb = load3(F.vb);
	return mk(p0.x + (a * va.x + b * vb.x), p0.y + (a * va.y + b * vb.y), p0.z + (a * va.z + b * vb.z));
}

// Scene::castRay closest hit (scene.cpp:142-167) with world-box culling
bool closest_hit(V3 o, V3 d, bool reverse, double& best_dist, int& best_geom, V3& P, V3& Nobj) {
	bool found = false;
	const V3 winv = safe_inv(d);
	for (size_t g = 0; g < S->geoms.size(); g++) {
		const DGeom& G = S->geoms[g];
		double tw;
		if (!slab(G.wlo, G.whi, o, winv, found ? prune_limit(best_dist) : INFINITY, tw)) continue;
		const V3 oo = xf_point(G.inv, o), dd = ray_dir(xf_dir(G.inv, d));
		V3 Po, No;
		if (G.kind == DGEOM_SPHERE) {
			double t;
			if (!sphere_hit(G, oo, dd, reverse, t)) continue;
			Po = oo + t * dd;
			No = Po - load3(G.center);
		} else {
			MeshBest mb;
			bool settled;
			if (!mesh_hit(false, G, oo, dd, reverse, INFINITY, INFINITY, mb, settled)) continue;
			Po = face_point(mb.face, mb.a, mb.b);
			No = face_normal(mb.face, mb.a, mb.b);
		}
		const V3 Pw = xf_point(G.fwd, Po);
		const double dist = std::sqrt(sq4(Pw - o));
		if (found && dist >= best_dist) continue;
		found = true;
		best_dist = dist;
		best_geom = static_cast<int>(g);
		P = Pw;
		Nobj = No;
	}
	return found;
}

// scene.cpp:90-93 as an `any` over the geometries (intersect.h geom_occludes / occluded)
bool occluded(V3 o, V3 d, bool reverse, double dist_light) {
	const V3 winv = safe_inv(d);
	const bool inf_light = dist_light == INFINITY;
	const double lim = inf_light ? INFINITY : dist_light * (1.0 + 1e-6);
	for (int32_t g : S->shadow_order) {
		const DGeom& G = S->geoms[g];
		double tw;
		if (!slab(G.wlo, G.whi, o, winv, lim, tw)) continue;
		const V3 oo = xf_point(G.inv, o), draw = xf_dir(G.inv, d);
		if (is_zero3(draw)) g_error = 1;
		const double nrm = std::sqrt(sq4(draw));
		const V3 dd = div3(draw, nrm);
		V3 Po;
		if (G.kind == DGEOM_SPHERE) {
			double t;
			if (!sphere_hit(G, oo, dd, reverse, t)) continue;
			if (inf_light) return true;
			Po = oo + t * dd;
		} else {
			MeshBest mb;
			bool settled, hit;
			if (inf_light) {
				if (mesh_hit(true, G, oo, dd, reverse, INFINITY, INFINITY, mb, settled)) return true;
				continue;
			}
			const double tl = dist_light * nrm, cap = tl * (1.0 + 1e-7) + 1e-300;
			hit = mesh_hit(true, G, oo, dd, reverse, tl * (1.0 - 1e-7), cap, mb, settled);
			if (hit && settled) return true;
			if (hit) {
				if (mb.dist > cap) continue;
				if (!mesh_hit(false, G, oo, dd, reverse, INFINITY, INFINITY, mb, settled)) continue;
			} else {
				continue;
			}
			Po = face_point(mb.face, mb.a, mb.b);
		}
		if (std::sqrt(sq4(xf_point(G.fwd, Po) - o)) <= dist_light) return true;
	}
	return false;
}

struct Counts {
	int64_t trace = 0, shadow = 0;
	long long nodes = 0, tris = 0;
};

double max0(double x) { return (x < 0.0) ? 0.0 : x; }

// Scene::traceRay (scene.cpp:61-140) with k_shade's / k_closest's expressions
void trace(V3 o, V3 d, int depth, bool inside, double col[3], Counts& cnt) {
	cnt.trace++;
	col[0] = col[1] = col[2] = 0.0;
	double dist;
	int gi;
	V3 P, Nobj;
	if (!closest_hit(o, d, inside, dist, gi, P, Nobj)) return;
	const DGeom& G = S->geoms[gi];
	const DMaterial& M = S->materials[G.mat];
	V3 N = xf_normal(G.inv, Nobj);
	if (G.flip) N = -N;
	if (inside) N = -N;
	N = (1.0 / std::sqrt(sq4(N))) * N;  // normalize(): times the reciprocal
	for (const DLight& L : S->lights) {
		if (L.kind == DLIGHT_AMBIENT) {
			for (int k = 0; k < 3; k++) col[k] = col[k] + (1.0 * L.color[k]) * M.ka[k];
			continue;
		}
		cnt.shadow++;
		const bool point = L.kind == DLIGHT_POINT;
		const V3 lv = load3(L.vec);
		const V3 Ld = ray_dir(point ? lv - P : -lv);
		const double nl_dot = dot4z(N, Ld);
		const double dL = point ? std::sqrt(sq4(lv - P)) : INFINITY;
		const V3 R = (2 * nl_dot) * N - Ld;
		const double sx = -dot4z(d, R);
		// both Phong additions exact zeros: the verdict cannot change the colour (k_shadow)
		if (M.zero_terms && L.zero_terms && nl_dot <= 0.0 && sx <= 0.0) continue;
		if (occluded(P, Ld, (nl_dot < 0) ^ inside, dL)) continue;
		const double fall = point ? std::pow(dL, -L.falloff) : 1.0;
		double att[3];
		for (int k = 0; k < 3; k++) att[k] = point ? fall * L.color[k] : L.color[k];
		const double diff = max0(nl_dot);
		for (int k = 0; k < 3; k++) col[k] = col[k] + (diff * att[k]) * M.kd[k];
		const double spec = std::pow(max0(sx), M.ns);
		for (int k = 0; k < 3; k++) col[k] = col[k] + (spec * att[k]) * M.ks[k];
	}
	if (depth <= 0) return;
	double kr[3] = {M.kr[0], M.kr[1], M.kr[2]};
	bool kr_nz = M.kr_nonzero;
	if (M.kt_nonzero) {
		const double nr = inside ? M.ior : 1.0 / M.ior;
		const double cosI = dot4z(N, d);
		const double sinT2 = nr * nr * (1.0 - cosI * cosI);
		if (sinT2 > 1.0) {
			kr[0] = kr[1] = kr[2] = 1.0;
			kr_nz = true;
		} else {
			const double k2 = nr * cosI + std::sqrt(1.0 - sinT2);
			double c[3];
			trace(P, ray_dir(nr * d - k2 * N), depth - 1, !inside, c, cnt);
			for (int k = 0; k < 3; k++) col[k] = col[k] + c[k];
		}
	}
	if (kr_nz) {
		double c[3];
		trace(P, ray_dir(d - (2 * dot4z(N, d)) * N), depth - 1, inside, c, cnt);
		for (int k = 0; k < 3; k++) col[k] = col[k] + c[k] * kr[k];
	}
}

}  // namespace

int main(int argc, char** argv) {
	if (argc != 10) {
		std::fprintf(stderr, "usage: %s scene.rti W H bdepth threads row_begin row_end row_step out.raw\n", argv[0]);
		return 2;
	}
	const int W = std::atoi(argv[2]), H = std::atoi(argv[3]), depth = std::atoi(argv[4]);
	const int threads = std::max(1, std::atoi(argv[5]));
	const int rb = std::atoi(argv[6]), re = std::atoi(argv[7]), rs = std::max(1, std::atoi(argv[8]));
	const auto t0 = std::chrono::steady_clock::now();
	Scene scene;
	try {
		parse_rti_file(scene, argv[1]);
	} catch (const ParseError& e) {
		std::fprintf(stderr, "Error: %s\n", e.msg.c_str());
		return 1;
	} catch (const MathError& e) {
		std::fprintf(stderr, "MathException: %s\n", e.msg.c_str());
		return 1;
	}
	if (!scene.has_camera) {
		std::fprintf(stderr, "Error: At least one camera must be specified.\n");
		return 1;
	}
	const FlatScene fs = flatten_scene(scene);
	S = &fs;
	std::vector<int> rows;
	for (int r = rb; r < re; r += rs) rows.push_back(r);
	std::vector<double> img(rows.size() * static_cast<size_t>(W) * 3);
	const auto t1 = std::chrono::steady_clock::now();
	std::atomic<size_t> next{0};
	std::vector<Counts> counts(threads);
	std::vector<std::thread> pool;
	for (int w = 0; w < threads; w++)
		pool.emplace_back([&, w] {
			for (size_t k; (k = next.fetch_add(1)) < rows.size();) {
				const int r = rows[k];
				for (int c = 0; c < W; c++) {
					// Camera::calculateViewingRay (rtbase.h:74-84) for pixel (r, c), scene.cpp:26-30
					const DCamera& cam = fs.camera;
					const double rF = (r + 0.5) / H, cF = (c + 0.5) / W;
					const double rI = 1.0 - rF, cI = 1.0 - cF;
					double p[4];
					for (int q = 0; q < 4; q++)
						p[q] = cF * (rF * cam.lr[q] + rI * cam.ur[q]) + cI * (rF * cam.ll[q] + rI * cam.ul[q]);
					if (p[3] - cam.eye[3] != 0) g_error = 2;
					const V3 d = ray_dir(mk(p[0] - cam.eye[0], p[1] - cam.eye[1], p[2] - cam.eye[2]));
					trace(load3(cam.eye), d, depth, false, &img[(k * W + c) * 3], counts[w]);
				}
			}
			counts[w].nodes = t_nodes;
			counts[w].tris = t_tris;
		});
	for (auto& t : pool) t.join();
	const auto t2 = std::chrono::steady_clock::now();
	if (g_error) {
		std::fprintf(stderr, "MathException (code %d)\n", g_error.load());
		return 3;
	}
	FILE* f = std::fopen(argv[9], "wb");
	if (!f || std::fwrite(img.data(), sizeof(double), img.size(), f) != img.size()) {
		std::perror("write");
		return 1;
	}
	std::fclose(f);
	Counts tot;
	for (const Counts& c : counts) {
		tot.trace += c.trace;
		tot.shadow += c.shadow;
		tot.nodes += c.nodes;
		tot.tris += c.tris;
	}
	std::printf("{\"trace_rays\": %lld, \"shadow_rays\": %lld, \"node_visits\": %lld, \"tri_tests\": %lld, "
	            "\"render_s\": %.6f, \"setup_s\": %.6f, \"threads\": %d}\n",
	            static_cast<long long>(tot.trace), static_cast<long long>(tot.shadow), tot.nodes, tot.tris,
	            std::chrono::duration<double>(t2 - t1).count(), std::chrono::duration<double>(t1 - t0).count(), threads);
	return 0;
}
