// rt_scene_desc from an in-memory scene, the way a caller holding the reference's Scene
// (scene.h:35-38) would fill it, checked against the file route (rt_builder_parse_rti of
// an equivalent .rti/.obj pair written here).
//
//   desc_check <dir> digest   host only: the two routes give identical device scenes
//                             (rt_debug_builder_digest over the flattened upload)
//   desc_check <dir> render   + both scenes rendered on HIP device 0: identical f64 and RGB8
//                             images; the f64 image is written to <dir>/desc.raw for the
//                             caller's comparison with the oracle
//
// The in-memory scene is built with the reference's own construction rules, restated
// here as a caller would have them: Transform::translate/scale (Eigen 3.2.2,
// Transform.h:784-790,838-843), Mesh::addTriangle (geometry.cpp:128-143), OBJ fan
// triangulation with the normalised geometric normal (parsers.cpp:329-350) and
// Mesh::updateBoundingBox (geometry.cpp:145-162).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <limits>
#include <string>
#include <vector>
#include "../../include/rtamd.h"

extern "C" int rt_debug_builder_digest(const rt_builder* b, uint64_t* out);

namespace {

struct Xf {  // Transform<double,3,Affine>, row-major 3x4 here, column-major in the descriptor
	double m[3][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}};
	void translate(double x, double y, double z) {
		const double v[3] = {x, y, z};
		for (int k = 0; k < 3; k++) m[k][3] = m[k][3] + ((m[k][0] * v[0] + m[k][1] * v[1]) + m[k][2] * v[2]);
	}
	void scale(double x, double y, double z) {
		const double v[3] = {x, y, z};
		for (int i = 0; i < 3; i++)
			for (int j = 0; j < 3; j++) m[i][j] *= v[j];
	}
	rt_xform_desc desc() const {  // derive = 1: the library computes inverse and det as the reference
		rt_xform_desc x;
		std::memset(&x, 0, sizeof(x));
		for (int j = 0; j < 4; j++) {
			for (int i = 0; i < 3; i++) x.fwd[j * 4 + i] = m[i][j];
			x.fwd[j * 4 + 3] = j == 3 ? 1.0 : 0.0;
		}
		x.derive = 1;
		return x;
	}
};

double dot4(const double a[4], const double b[4]) { return (a[0] * b[0] + a[2] * b[2]) + (a[1] * b[1] + a[3] * b[3]); }
void cross(const double a[4], const double b[4], double o[4]) {
	o[0] = a[1] * b[2] - a[2] * b[1];
	o[1] = a[2] * b[0] - a[0] * b[2];
	o[2] = a[0] * b[1] - a[1] * b[0];
	o[3] = 0;
}

void set_material(rt_material_desc& m, const double p[17]) {  // `mat` line order (parsers.cpp:182-189)
	for (int k = 0; k < 3; k++) {
		m.ambient[k] = p[k];
		m.diffuse[k] = p[3 + k];
		m.specular[k] = p[6 + k];
		m.reflective[k] = p[10 + k];
		m.translucency[k] = p[13 + k];
	}
	m.specular_coefficient = p[9];
	m.index_of_refractivity = p[16];
}

std::string num(double v) {
	char b[40];
	std::snprintf(b, sizeof b, "%.17g", v);
	return b;
}

std::string mat_line(const double p[17]) {
	std::string s = "mat";
	for (int k = 0; k < 17; k++) s += " " + num(p[k]);
	return s + "\n";
}

struct Scene {
	rt_scene_desc desc{};
	std::vector<rt_geometry_desc> geoms;
	std::vector<rt_light_desc> lights;
	std::vector<std::vector<rt_face_desc>> faces;  // per mesh
	std::string rti, obj;
};

Scene build() {
	Scene S;
	S.faces.reserve(4);
	const double eye[4] = {0, 0, 6, 1}, ll[4] = {-1.6, -0.9, 2, 1}, lr[4] = {1.6, -0.9, 2, 1},
	             ul[4] = {-1.6, 0.9, 2, 1}, ur[4] = {1.6, 0.9, 2, 1};
	// camera under a translation
	Xf cx;
	cx.translate(0.25, -0.5, 0.125);
	std::memset(&S.desc, 0, sizeof(S.desc));
	S.desc.has_camera = 1;
	S.desc.camera.xf = cx.desc();
	std::memcpy(S.desc.camera.eye, eye, sizeof eye);
	std::memcpy(S.desc.camera.lower_left, ll, sizeof ll);
	std::memcpy(S.desc.camera.lower_right, lr, sizeof lr);
	std::memcpy(S.desc.camera.upper_left, ul, sizeof ul);
	std::memcpy(S.desc.camera.upper_right, ur, sizeof ur);
	S.rti += "xft 0.25 -0.5 0.125\ncam 0 0 6  -1.6 -0.9 2  1.6 -0.9 2  -1.6 0.9 2  1.6 0.9 2\nxfz\n";

	// lights: point, transformed point with falloff, directional, ambient
	auto light = [&](int kind, const Xf& x, const double vec[4], const double col[3], double falloff) {
		rt_light_desc l;
		std::memset(&l, 0, sizeof l);
		l.kind = kind;
		l.xf = x.desc();
		std::memcpy(l.vec, vec, 4 * sizeof(double));
		std::memcpy(l.color, col, 3 * sizeof(double));
		l.falloff = falloff;
		S.lights.push_back(l);
	};
	{
		const double p[4] = {4, 5, 6, 1}, c[3] = {0.6, 0.5, 0.4};
		light(RT_LIGHT_POINT, Xf(), p, c, 0.0);
		S.rti += "ltp 4 5 6  0.6 0.5 0.4\n";
		Xf t;
		t.translate(-1, 0.5, 0);
		const double p2[4] = {-3, 2, 1, 1}, c2[3] = {0.4, 0.6, 0.8};
		light(RT_LIGHT_POINT, t, p2, c2, 0.5);
		S.rti += "xft -1 0.5 0\nltp -3 2 1  0.4 0.6 0.8  0.5\nxfz\n";
		// ltd: direction normalised by its Vector3d norm, a0^2 + (a1^2 + a2^2) (parsers.cpp:156-161)
		const double raw[3] = {1, 1, -1};
		const double len = std::sqrt(raw[0] * raw[0] + (raw[1] * raw[1] + raw[2] * raw[2]));
		const double d[4] = {raw[0] / len, raw[1] / len, raw[2] / len, 0}, c3[3] = {0.3, 0.3, 0.3};
		light(RT_LIGHT_DIRECTIONAL, Xf(), d, c3, 0.0);
		S.rti += "ltd 1 1 -1  0.3 0.3 0.3\n";
		const double z[4] = {0, 0, 0, 0}, ca[3] = {0.1, 0.1, 0.1};
		light(RT_LIGHT_AMBIENT, Xf(), z, ca, 0.0);
		S.rti += "lta 0.1 0.1 0.1\n";
	}

	// OBJ torus of quads (fan-triangulated), reflective, translated and scaled
	{
		const double m[17] = {0.05, 0.02, 0.02, 0.5, 0.3, 0.2, 0.6, 0.6, 0.6, 12, 0.3, 0.3, 0.3, 0, 0, 0, 1};
		Xf x;
		x.translate(0.3, 0.1, -0.4);
		x.scale(1.5, 1.5, 0.75);
		const int nu = 16, nv = 10;
		std::vector<double> vx;
		for (int i = 0; i < nu; i++)
			for (int j = 0; j < nv; j++) {
				const double u = 2 * M_PI * i / nu, v = 2 * M_PI * j / nv;
				const double p[3] = {(1.0 + 0.35 * std::cos(v)) * std::cos(u), (1.0 + 0.35 * std::cos(v)) * std::sin(u),
				                     0.35 * std::sin(v)};
				for (int k = 0; k < 3; k++) {
					vx.push_back(std::stod(num(p[k])));  // what the parser reads back (%.17g round-trips)
					S.obj += (k == 0 ? "v " : " ") + num(p[k]);
				}
				S.obj += "\n";
			}
		std::vector<rt_face_desc> fs;
		auto vert = [&](int i, int j, double out[4]) {
			const int idx = ((i % nu) * nv + (j % nv)) * 3;
			out[0] = vx[idx];
			out[1] = vx[idx + 1];
			out[2] = vx[idx + 2];
			out[3] = 1.0;
		};
		for (int i = 0; i < nu; i++)
			for (int j = 0; j < nv; j++) {
				const int c[4][2] = {{i, j}, {i + 1, j}, {i + 1, j + 1}, {i, j + 1}};
				S.obj += "f";
				for (const auto& cc : c) S.obj += " " + std::to_string((cc[0] % nu) * nv + (cc[1] % nv) + 1);
				S.obj += "\n";
				for (int k = 1; k + 1 < 4; k++) {  // fan around corner 0
					double p[3][4];
					vert(c[0][0], c[0][1], p[0]);
					vert(c[k][0], c[k][1], p[1]);
					vert(c[k + 1][0], c[k + 1][1], p[2]);
					double e1[4], e2[4], n[4];
					for (int a = 0; a < 4; a++) {
						e1[a] = p[1][a] - p[0][a];
						e2[a] = p[2][a] - p[0][a];
					}
					cross(e1, e2, n);
					const double rcp = 1.0 / std::sqrt(dot4(n, n));  // normalize(): times 1/norm
					rt_face_desc f;
					for (int a = 0; a < 3; a++)
						for (int b = 0; b < 4; b++) {
							f.points[a][b] = p[a][b];
							f.normals[a][b] = n[b] * rcp;
						}
					fs.push_back(f);
				}
			}
		S.faces.push_back(fs);
		rt_geometry_desc g;
		std::memset(&g, 0, sizeof g);
		g.kind = RT_GEOM_MESH;
		g.xf = x.desc();
		set_material(g.material, m);
		// Mesh::updateBoundingBox (geometry.cpp:145-162)
		for (int k = 0; k < 4; k++) {
			g.bbox_min[k] = std::numeric_limits<double>::infinity();
			g.bbox_max[k] = -std::numeric_limits<double>::infinity();
		}
		for (const rt_face_desc& f : fs)
			for (int a = 0; a < 3; a++)
				for (int k = 0; k < 4; k++) {
					g.bbox_min[k] = std::min(g.bbox_min[k], f.points[a][k]);
					g.bbox_max[k] = std::max(g.bbox_max[k], f.points[a][k]);
				}
		S.geoms.push_back(g);
		S.rti += mat_line(m) + "xft 0.3 0.1 -0.4\nxfs 1.5 1.5 0.75\nobj torus.obj\nxfz\n";
	}
	// glass sphere under a non-uniform scale
	{
		const double m[17] = {0, 0, 0, 0.1, 0.1, 0.1, 0.5, 0.5, 0.5, 40, 0.1, 0.1, 0.1, 0.8, 0.9, 0.9, 1.5};
		Xf x;
		x.scale(0.5, 2, 1);
		rt_geometry_desc g;
		std::memset(&g, 0, sizeof g);
		g.kind = RT_GEOM_SPHERE;
		g.xf = x.desc();
		set_material(g.material, m);
		const double c[4] = {-1.2, 0.2, -1, 1};
		std::memcpy(g.center, c, sizeof c);
		g.radius = 0.4f;  // float radius_ (geometry.h:22)
		S.geoms.push_back(g);
		S.rti += mat_line(m) + "xfs 0.5 2 1\nsph -1.2 0.2 -1 0.4\nxfz\n";
	}
	// two-sided floor triangle: Mesh::addTriangle (geometry.cpp:128-143)
	{
		const double m[17] = {0.02, 0.02, 0.02, 0.6, 0.6, 0.6, 0, 0, 0, 1, 0.2, 0.2, 0.2, 0, 0, 0, 1};
		const double v[3][4] = {{-10, -1.2, 10, 1}, {10, -1.2, 10, 1}, {10, -1.2, -10, 1}};
		double e1[4], e2[4], n[4];
		for (int a = 0; a < 4; a++) {
			e1[a] = v[1][a] - v[0][a];
			e2[a] = v[2][a] - v[0][a];
		}
		cross(e1, e2, n);
		const double len = std::sqrt(dot4(n, n));
		for (int a = 0; a < 4; a++) n[a] = n[a] / len;  // normalized(): division
		double sum[4];
		for (int a = 0; a < 4; a++) sum[a] = (v[0][a] + v[1][a]) + v[2][a];
		const double sc = (std::numeric_limits<double>::epsilon() * std::sqrt(dot4(sum, sum))) / 3;
		std::vector<rt_face_desc> fs;
		for (int sgn = -1; sgn <= 1; sgn += 2) {
			rt_face_desc f;
			for (int k = 0; k < 3; k++)
				for (int a = 0; a < 4; a++) {
					f.points[k][a] = v[k][a] + sgn * (sc * n[a]);
					f.normals[k][a] = sgn * n[a];
				}
			fs.push_back(f);
		}
		S.faces.push_back(fs);
		rt_geometry_desc g;
		std::memset(&g, 0, sizeof g);
		g.kind = RT_GEOM_MESH;
		g.xf = Xf().desc();
		set_material(g.material, m);  // no updateBoundingBox for `tri`: the box stays zero
		S.geoms.push_back(g);
		S.rti += mat_line(m) + "tri -10 -1.2 10  10 -1.2 10  10 -1.2 -10\n";
	}
	size_t mesh = 0;
	for (rt_geometry_desc& g : S.geoms)
		if (g.kind == RT_GEOM_MESH) {
			g.faces = S.faces[mesh].data();
			g.n_faces = static_cast<int64_t>(S.faces[mesh].size());
			mesh++;
		}
	S.desc.n_geometries = static_cast<int32_t>(S.geoms.size());
	S.desc.geometries = S.geoms.data();
	S.desc.n_lights = static_cast<int32_t>(S.lights.size());
	S.desc.lights = S.lights.data();
	return S;
}

int die(const char* what) {
	std::fprintf(stderr, "desc_check: %s: %s\n", what, rt_last_error());
	return 1;
}

}  // namespace

int main(int argc, char** argv) {
	if (argc < 3) {
		std::fprintf(stderr, "usage: desc_check <dir> digest|render\n");
		return 2;
	}
	const std::string dir = argv[1], mode = argv[2];
	Scene S = build();
	{
		FILE* f = std::fopen((dir + "/scene.rti").c_str(), "w");
		FILE* g = std::fopen((dir + "/torus.obj").c_str(), "w");
		if (!f || !g) return die("cannot write the scene files");
		std::fputs(S.rti.c_str(), f);
		std::fputs(S.obj.c_str(), g);
		std::fclose(f);
		std::fclose(g);
	}
	rt_builder* file_b = rt_builder_create();
	if (rt_builder_parse_rti(file_b, (dir + "/scene.rti").c_str())) return die("parse");
	if (std::strlen(rt_builder_warnings(file_b))) return die("unexpected parser warnings");
	rt_builder* desc_b = rt_builder_create();
	if (rt_builder_set_desc(desc_b, &S.desc)) return die("rt_builder_set_desc");
	uint64_t h_file = 0, h_desc = 0;
	if (rt_debug_builder_digest(file_b, &h_file) || rt_debug_builder_digest(desc_b, &h_desc)) return die("digest");
	std::printf("{\"digest_file\": \"%016llx\", \"digest_desc\": \"%016llx\"", (unsigned long long)h_file,
	            (unsigned long long)h_desc);
	if (h_file != h_desc) {
		std::printf("}\n");
		std::fprintf(stderr, "desc_check: the descriptor route uploads a different scene\n");
		return 1;
	}
	if (mode == "render") {
		rt_scene *sd = nullptr, *sf = nullptr;
		if (rt_scene_create_desc(&S.desc, 0, &sd)) return die("rt_scene_create_desc");
		if (rt_scene_create(file_b, 0, &sf)) return die("rt_scene_create");
		rt_render_params p{};
		p.width = 160;
		p.height = 90;
		p.bounce_depth = 5;
		p.row_end = p.height;
		p.row_step = 1;
		const size_t n = static_cast<size_t>(p.width) * p.height * 3;
		std::vector<double> a(n), b(n);
		std::vector<uint8_t> a8(n), b8(n);
		rt_counters ca{}, cb{};
		if (rt_render(sd, &p, a.data(), nullptr, nullptr, &ca) || rt_render(sf, &p, b.data(), nullptr, nullptr, &cb))
			return die("rt_render");
		if (rt_render_rgb8(sd, &p, a8.data(), nullptr, nullptr, nullptr) ||
		    rt_render_rgb8(sf, &p, b8.data(), nullptr, nullptr, nullptr))
			return die("rt_render_rgb8");
		const bool same = std::memcmp(a.data(), b.data(), n * sizeof(double)) == 0 && a8 == b8 &&
		                  ca.trace_rays == cb.trace_rays && ca.shadow_rays == cb.shadow_rays;
		FILE* f = std::fopen((dir + "/desc.raw").c_str(), "wb");
		if (!f) return die("cannot write desc.raw");
		std::fwrite(a.data(), sizeof(double), n, f);
		std::fclose(f);
		std::printf(", \"trace_rays\": %lld, \"shadow_rays\": %lld, \"same_image\": %s",
		            (long long)ca.trace_rays, (long long)ca.shadow_rays, same ? "true" : "false");
		rt_scene_destroy(sd);
		rt_scene_destroy(sf);
		if (!same) {
			std::printf("}\n");
			return 1;
		}
	}
	std::printf("}\n");
	rt_builder_destroy(file_b);
	rt_builder_destroy(desc_b);
	return 0;
}
