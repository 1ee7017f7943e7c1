// Scene flattening + per-mesh LBVH construction (host).
#include "bvh.h"
#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include "xform.h"

// Tree construction: binned SAH (1) or Morton radix splits (0); any tree gives the same
// results (intersect.h), the choice only moves traversal cost.
#ifndef RT_BVH_SAH
#define RT_BVH_SAH 1
#endif
#ifndef RT_SAH_BINS
#define RT_SAH_BINS 32
#endif
namespace rtamd {
namespace {

struct Box {
	double lo[3], hi[3];
	void empty() {
		for (int k = 0; k < 3; k++) {
			lo[k] = INFINITY;
			hi[k] = -INFINITY;
		}
	}
	void grow(const Box& b) {
		for (int k = 0; k < 3; k++) {
			lo[k] = std::min(lo[k], b.lo[k]);
			hi[k] = std::max(hi[k], b.hi[k]);
		}
	}
};

// directed conversions to fp32: the result bounds x from below / above
float round_down_f32(double x) {
	float f = static_cast<float>(x);
	if (static_cast<double>(f) > x) f = std::nextafter(f, -INFINITY);
	return f;
}
float round_up_f32(double x) {
	float f = static_cast<float>(x);
	if (static_cast<double>(f) < x) f = std::nextafter(f, INFINITY);
	return f;
}

// spread the low 21 bits of v to every third bit of a 63-bit word
uint64_t spread3(uint64_t v) {
	v &= 0x1fffff;
	v = (v | v << 32) & 0x1f00000000ffffULL;
	v = (v | v << 16) & 0x1f0000ff0000ffULL;
	v = (v | v << 8) & 0x100f00f00f00f00fULL;
	v = (v | v << 4) & 0x10c30c30c30c30c3ULL;
	v = (v | v << 2) & 0x1249249249249249ULL;
	return v;
}

struct Builder {
	const std::vector<Box>& boxes;   // per face (mesh-local index)
	std::vector<uint64_t> code;      // sorted Morton codes
	std::vector<int32_t> order;      // sorted face indices
	std::vector<DBvhNode>& nodes;
	std::vector<int32_t> leaf_order; // faces in leaf order
	double pad;
	int max_depth = 0;
	bool median_only = false;
	bool sah = true;

	struct Ref {
		Box box;
		int32_t first, count;  // count > 0: leaf
	};

	int split(int b, int e) const {  // [b, e) with e - b >= 2
		if (median_only || code[b] == code[e - 1]) return (b + e) / 2;
		const int prefix = __builtin_clzll(code[b] ^ code[e - 1]);
		int lo = b, hi = e - 1;  // find last index sharing > prefix bits with code[b]
		while (lo + 1 < hi) {
			const int mid = (lo + hi) / 2;
			if (__builtin_clzll(code[b] ^ code[mid]) > prefix)
				lo = mid;
			else
				hi = mid;
		}
		return lo + 1;
	}

	static double area(const Box& x) {
		const double dx = x.hi[0] - x.lo[0], dy = x.hi[1] - x.lo[1], dz = x.hi[2] - x.lo[2];
		return dx * dy + dy * dz + dz * dx;
	}

	// Binned surface-area-heuristic split of order[b, e) (reorders it in place): the split
	// between centroid bins minimising area(L) * |L| + area(R) * |R| over the three axes.
	int sah_split(int b, int e, double* cost = nullptr) {
		constexpr int kBins = RT_SAH_BINS;
		double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
		auto centre = [&](int32_t f, int a) { return 0.5 * (boxes[f].lo[a] + boxes[f].hi[a]); };
		for (int i = b; i < e; i++)
			for (int a = 0; a < 3; a++) {
				clo[a] = std::min(clo[a], centre(order[i], a));
				chi[a] = std::max(chi[a], centre(order[i], a));
			}
		double best = INFINITY;
		int best_axis = -1, best_bin = -1;
		for (int a = 0; a < 3; a++) {
			const double ext = chi[a] - clo[a];
			if (!(ext > 0)) continue;
			Box bb[kBins];
			int cnt[kBins] = {0};
			for (auto& x : bb) x.empty();
			for (int i = b; i < e; i++) {
				const int k = std::min(kBins - 1, static_cast<int>((centre(order[i], a) - clo[a]) / ext * kBins));
				cnt[k]++;
				bb[k].grow(boxes[order[i]]);
			}
			double right_area[kBins];
			int right_cnt[kBins];
			Box acc;
			acc.empty();
			int n = 0;
			for (int k = kBins - 1; k > 0; k--) {
				acc.grow(bb[k]);
				n += cnt[k];
				right_area[k] = area(acc);
				right_cnt[k] = n;
			}
			acc.empty();
			n = 0;
			for (int k = 0; k < kBins - 1; k++) {
				acc.grow(bb[k]);
				n += cnt[k];
				if (n == 0 || right_cnt[k + 1] == 0) continue;
				const double c = area(acc) * n + right_area[k + 1] * right_cnt[k + 1];
				if (c < best) {
					best = c;
					best_axis = a;
					best_bin = k;
				}
			}
		}
		if (cost) *cost = best;  // area(L) |L| + area(R) |R| (INFINITY: no split found)
		if (best_axis < 0) return (b + e) / 2;  // all centroids coincide
		const double ext = chi[best_axis] - clo[best_axis];
		auto* mid = std::partition(order.data() + b, order.data() + e, [&](int32_t f) {
			return std::min(kBins - 1, static_cast<int>((centre(f, best_axis) - clo[best_axis]) / ext * kBins)) <= best_bin;
		});
		const int m = static_cast<int>(mid - order.data());
		return (m == b || m == e) ? (b + e) / 2 : m;
	}

	Ref build(int b, int e, int depth) {
		max_depth = std::max(max_depth, depth);
		Ref r;
		r.box.empty();
		const bool leaf = e - b <= kLeafFaces;
		if (leaf) {
			r.first = static_cast<int32_t>(leaf_order.size());
			r.count = e - b;
			for (int i = b; i < e; i++) {
				leaf_order.push_back(order[i]);
				r.box.grow(boxes[order[i]]);
			}
			return r;
		}
		const int idx = static_cast<int>(nodes.size());
		nodes.emplace_back();
		const int m = (sah && !median_only) ? sah_split(b, e) : split(b, e);
		const Ref c[2] = {build(b, m, depth + 1), build(m, e, depth + 1)};
		DBvhNode& n = nodes[idx];
		std::memset(&n, 0, sizeof(n));
		for (int k = 0; k < 2; k++) {
			for (int a = 0; a < 3; a++) {
				n.lo[k][a] = round_down_f32(c[k].box.lo[a] - pad);
				n.hi[k][a] = round_up_f32(c[k].box.hi[a] + pad);
			}
			n.first[k] = c[k].first;
			n.count[k] = c[k].count;
			r.box.grow(c[k].box);
		}
		r.first = idx;
		r.count = 0;
		return r;
	}
};

// Padded world-space box of an object-space box (the eight corners through fwd).  Used
// only to skip geometries a ray cannot hit; a degenerate transform disables it.
void world_box(const Geometry& g, const double lo[3], const double hi[3], DGeom& d) {
	bool finite = std::isfinite(g.det) && g.det != 0;
	for (int i = 0; i < 3; i++)
		for (int j = 0; j < 4; j++) finite = finite && std::isfinite(g.fwd.m[i][j]) && std::isfinite(g.inv.m[i][j]);
	for (int k = 0; k < 3; k++) {
		d.wlo[k] = -INFINITY;
		d.whi[k] = INFINITY;
	}
	if (!finite) return;
	if (!(lo[0] <= hi[0] && lo[1] <= hi[1] && lo[2] <= hi[2])) {  // empty mesh: nothing to hit
		for (int k = 0; k < 3; k++) {
			d.wlo[k] = INFINITY;
			d.whi[k] = -INFINITY;
		}
		return;
	}
	double wl[3] = {INFINITY, INFINITY, INFINITY}, wh[3] = {-INFINITY, -INFINITY, -INFINITY};
	double amax = 0;
	for (int c = 0; c < 8; c++) {
		const double p[4] = {(c & 1) ? hi[0] : lo[0], (c & 2) ? hi[1] : lo[1], (c & 4) ? hi[2] : lo[2], 1.0};
		double w[4];
		affine_apply(g.fwd, p, w);
		for (int k = 0; k < 3; k++) {
			wl[k] = std::min(wl[k], w[k]);
			wh[k] = std::max(wh[k], w[k]);
			amax = std::max(amax, std::fabs(w[k]));
		}
	}
	const double pad = 1e-9 * amax + 1e-300;
	for (int k = 0; k < 3; k++) {
		d.wlo[k] = wl[k] - pad;
		d.whi[k] = wh[k] + pad;
	}
}

// True unless every unit world direction is certain to keep a component above 1e-12 in
// object space: |inv d| >= sigma_min(inv) >= |det(inv)| / ||inv||_F^2 (3x3 part).
bool direction_may_vanish(const Affine& inv) {
	double fro = 0;
	for (int i = 0; i < 3; i++)
		for (int j = 0; j < 3; j++) fro += inv.m[i][j] * inv.m[i][j];
	const double (*m)[4] = inv.m;
	const double det = m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) -
	                   m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0]) +
	                   m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]);
	if (!std::isfinite(fro) || !std::isfinite(det) || fro == 0) return true;
	const double sigma_min_bound = std::fabs(det) / fro;
	return !(sigma_min_bound > 4e-12);  // |v|_2 > sqrt(3) 1e-12 with margin for rounding
}

// Facing pre-test data of a face (DFaceGeo::cone_*): the fp32 mean c of the three vertex
// normals, their largest distance r from it, and tau = r + 2 (kFacingRel |n|_1 + 1e-6 |c|_1)
// with |n|_1 the largest normal's 1-norm, rounded up; tau = +inf (no pre-test) when a
// normal is not finite or zero, or the normals' magnitudes are far apart (the interpolated
// normal's rounding then scales with the largest one).  intersect.h face_facing_rejects.
void facing_data(const Face& f, DFaceGeo& fg) {
	long double c[3] = {0, 0, 0};
	double lo = INFINITY, hi = 0;
	bool ok = true;
	for (int v = 0; v < 3; v++) {
		double l1 = 0;
		for (int k = 0; k < 3; k++) {
			ok = ok && std::isfinite(f.n[v][k]);
			l1 += std::fabs(f.n[v][k]);
			c[k] += f.n[v][k] / 3.0L;
		}
		lo = std::min(lo, l1);
		hi = std::max(hi, l1);
	}
	ok = ok && lo > 1e-30 && hi < 1e30 && hi <= 1e6 * lo;
	fg.cone_tau = INFINITY;
	for (int k = 0; k < 3; k++) fg.cone_c[k] = ok ? static_cast<float>(c[k]) : 0.0f;
	if (!ok) return;
	long double r = 0, cl1 = 0;
	for (int k = 0; k < 3; k++) cl1 += std::fabs((long double)fg.cone_c[k]);
	for (int v = 0; v < 3; v++) {
		long double e = 0;
		for (int k = 0; k < 3; k++) {
			const long double x = (long double)f.n[v][k] - fg.cone_c[k];
			e += x * x;
		}
		r = std::max(r, std::sqrt(e));
	}
	const long double tau = (r * (1 + 1e-12L) + 2 * (kFacingRel * hi + 1e-6L * cl1));
	fg.cone_tau = round_up_f32(static_cast<double>(tau) * (1 + 1e-12));
}

}  // namespace

FlatScene flatten_scene(const Scene& s) {
	FlatScene fs;
	std::memset(&fs.camera, 0, sizeof(fs.camera));
	if (s.has_camera) {
		std::memcpy(fs.camera.eye, s.cam[0], sizeof(double) * 4);
		std::memcpy(fs.camera.ll, s.cam[1], sizeof(double) * 4);
		std::memcpy(fs.camera.lr, s.cam[2], sizeof(double) * 4);
		std::memcpy(fs.camera.ul, s.cam[3], sizeof(double) * 4);
		std::memcpy(fs.camera.ur, s.cam[4], sizeof(double) * 4);
	}
	for (const Light& l : s.lights) {
		DLight d;
		std::memset(&d, 0, sizeof(d));  // padding too: the scene digest hashes the bytes
		for (int k = 0; k < 3; k++) {
			d.color[k] = l.color[k];
			d.vec[k] = l.vec[k];
		}
		d.falloff = l.falloff;
		d.kind = l.kind;
		// colorForDistance (lights.h:24) is the colour itself: finite for every distance
		d.zero_terms = (l.kind == LIGHT_DIRECTIONAL || (l.kind == LIGHT_POINT && l.falloff == 0.0)) &&
		               std::isfinite(l.color[0]) && std::isfinite(l.color[1]) && std::isfinite(l.color[2]);
		fs.lights.push_back(d);
	}
	for (const Geometry& g : s.geoms) {
		DGeom d;
		std::memset(&d, 0, sizeof(d));
		std::memcpy(d.fwd, g.fwd.m, sizeof(d.fwd));
		std::memcpy(d.inv, g.inv.m, sizeof(d.inv));
		d.kind = g.kind;
		d.flip = g.det < 0;
		d.bvh_root = -1;
		d.may_raise = direction_may_vanish(g.inv);
		fs.n_may_raise += d.may_raise;
		DMaterial m;
		std::memset(&m, 0, sizeof(m));
		for (int k = 0; k < 3; k++) {
			m.ka[k] = g.mat.ka[k];
			m.kd[k] = g.mat.kd[k];
			m.ks[k] = g.mat.ks[k];
			m.kr[k] = g.mat.kr[k];
			m.kt[k] = g.mat.kt[k];
		}
		m.ns = g.mat.ns;
		m.ior = g.mat.ior;
		m.kt_nonzero = !is_zero(g.mat.kt, 3);
		m.kr_nonzero = !is_zero(g.mat.kr, 3);
		// pow(+-0, ns) is +-0 only for ns > 0; 0 * kd and 0 * ks are zeros only when finite
		m.zero_terms = g.mat.ns > 0;
		for (int k = 0; k < 3; k++) m.zero_terms = m.zero_terms && std::isfinite(g.mat.kd[k]) && std::isfinite(g.mat.ks[k]);
		d.mat = static_cast<int32_t>(fs.materials.size());
		fs.materials.push_back(m);
		if (g.kind == GEOM_SPHERE) {
			for (int k = 0; k < 3; k++) d.center[k] = g.center[k];
			const float rr = g.radius * g.radius;  // fp32 product, geometry.cpp:53
			d.rr = static_cast<double>(rr);
			// the reference's test compares against rr in object space: box radius sqrt(rr)
			const double rad = std::sqrt(static_cast<double>(rr)) * (1.0 + 1e-12);
			const double lo[3] = {g.center[0] - rad, g.center[1] - rad, g.center[2] - rad};
			const double hi[3] = {g.center[0] + rad, g.center[1] + rad, g.center[2] + rad};
			world_box(g, lo, hi, d);
			fs.geoms.push_back(d);
			continue;
		}
		// mesh
		bool box_differs = false;
		for (int k = 0; k < 4; k++) box_differs |= g.bb_min[k] != g.bb_max[k];
		d.gate = box_differs && g.face_count > 1;
		for (int k = 0; k < 3; k++) {
			d.bb_min[k] = g.bb_min[k];
			d.bb_max[k] = g.bb_max[k];
		}
		d.face_begin = static_cast<int32_t>(fs.face_geo.size());
		d.face_count = static_cast<int32_t>(g.face_count);
		{
			double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
			for (int64_t i = 0; i < g.face_count; i++)
				for (int v = 0; v < 3; v++)
					for (int k = 0; k < 3; k++) {
						lo[k] = std::min(lo[k], s.faces[g.face_begin + i].p[v][k]);
						hi[k] = std::max(hi[k], s.faces[g.face_begin + i].p[v][k]);
					}
			world_box(g, lo, hi, d);
		}
		auto emit = [&](int64_t local) {
			const Face& f = s.faces[g.face_begin + local];
			DFaceGeo fg;
			std::memset(&fg, 0, sizeof(fg));
			DFaceNrm fn;
			std::memset(&fn, 0, sizeof(fn));
			for (int k = 0; k < 3; k++) {
				fg.p0[k] = f.p[0][k];
				fg.va[k] = f.p[1][k] - f.p[0][k];  // face.points_[1] - face.points_[0] (geometry.cpp:80)
				fg.vb[k] = f.p[2][k] - f.p[0][k];
				fn.n0[k] = f.n[0][k];
				fn.n1[k] = f.n[1][k];
				fn.n2[k] = f.n[2][k];
			}
			facing_data(f, fg);
			fs.face_geo.push_back(fg);
			fs.face_nrm.push_back(fn);
			fs.face_geo.back().id = static_cast<int32_t>(local);
		};
		if (g.face_count <= kLinearFaces) {
			for (int64_t i = 0; i < g.face_count; i++) emit(i);
			fs.geoms.push_back(d);
			continue;
		}
		// LBVH over the object-space face boxes
		std::vector<Box> boxes(g.face_count);
		Box cb;
		cb.empty();
		double amax = 0;
		for (int64_t i = 0; i < g.face_count; i++) {
			const Face& f = s.faces[g.face_begin + i];
			boxes[i].empty();
			for (int v = 0; v < 3; v++)
				for (int k = 0; k < 3; k++) {
					boxes[i].lo[k] = std::min(boxes[i].lo[k], f.p[v][k]);
					boxes[i].hi[k] = std::max(boxes[i].hi[k], f.p[v][k]);
					amax = std::max(amax, std::fabs(f.p[v][k]));
				}
			Box c;
			for (int k = 0; k < 3; k++) c.lo[k] = c.hi[k] = 0.5 * (boxes[i].lo[k] + boxes[i].hi[k]);
			cb.grow(c);
		}
		std::vector<std::pair<uint64_t, int32_t>> keyed(g.face_count);
		for (int64_t i = 0; i < g.face_count; i++) {
			uint64_t q[3];
			for (int k = 0; k < 3; k++) {
				const double ext = cb.hi[k] - cb.lo[k];
				const double c = 0.5 * (boxes[i].lo[k] + boxes[i].hi[k]);
				double u = ext > 0 ? (c - cb.lo[k]) / ext : 0.5;
				u = std::min(std::max(u, 0.0), 1.0);
				q[k] = static_cast<uint64_t>(u * 2097151.0);
			}
			keyed[i] = {spread3(q[0]) << 2 | spread3(q[1]) << 1 | spread3(q[2]), static_cast<int32_t>(i)};
		}
		std::sort(keyed.begin(), keyed.end());
		// Conservative padding: the traversal may prune a node only when no face inside it
		// can pass the reference's Cramer test; 1e-9 of the largest coordinate magnitude is
		// ~10^7 ulps of slack for the fp64 slab and Cramer rounding (validated bit-exact
		// against the oracle over every shipped scene).  The padded boxes are then
		// rounded outward to fp32 (DBvhNode).
		// The node boxes get 2^-18 of amax more: the fp32 node test (intersect.h slab32)
		// errs by at most ~6 * 2^-24 * amax in position, well inside it.
		const double pad = (1e-9 + 0x1p-18) * amax + 1e-300;
		const size_t node_base = fs.nodes.size();
		for (int attempt = 0; attempt < 2; attempt++) {
			fs.nodes.resize(node_base);
			Builder bld{boxes, {}, {}, fs.nodes, {}, pad};
			bld.median_only = attempt == 1;
			bld.sah = RT_BVH_SAH;
			for (const auto& kv : keyed) {
				bld.code.push_back(kv.first);
				bld.order.push_back(kv.second);
			}
			bld.build(0, static_cast<int>(g.face_count), 0);
			if (bld.max_depth + 2 > kStackDepth && attempt == 0) continue;  // too deep: median splits
			// inner-node indices are global (fs.nodes); leaf face indices are relative to the mesh
			for (int32_t local : bld.leaf_order) emit(local);
			fs.max_bvh_depth = std::max(fs.max_bvh_depth, bld.max_depth);
			break;
		}
		d.bvh_root = static_cast<int32_t>(node_base);
		fs.geoms.push_back(d);
	}
	// shadow-test order: spheres and linear meshes first, then BVH meshes by size
	fs.shadow_order.resize(fs.geoms.size());
	std::iota(fs.shadow_order.begin(), fs.shadow_order.end(), 0);
	auto cost = [&](int32_t g) -> int64_t {
		const DGeom& d = fs.geoms[g];
		return (d.kind == GEOM_SPHERE || d.bvh_root < 0) ? 0 : d.face_count;
	};
	std::stable_sort(fs.shadow_order.begin(), fs.shadow_order.end(),
	                 [&](int32_t a, int32_t b) { return cost(a) < cost(b); });
	return fs;
}

}  // namespace rtamd
