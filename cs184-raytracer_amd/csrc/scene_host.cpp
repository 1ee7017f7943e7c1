// .rti / .obj ingest into the flat host scene (see scene_host.h).
//
// Grammar and error text follow the reference's RTIParser / OBJParser
// (parsers.cpp:5-374) and ParseException (exceptions.{h,cpp}); geometry set-up follows
// Mesh::addTriangle / Mesh::updateBoundingBox (geometry.cpp:128-162).
#include "scene_host.h"
#include <libgen.h>
#include <algorithm>
#include <array>
#include <cctype>
#include <cmath>
#include <fstream>
#include <limits>
#include <sstream>
#include <stdexcept>
#include "xform.h"

namespace rtamd {
namespace {

std::string at_line(const std::string& msg, int lineno) {  // ParseException::buildMessage
	return lineno > 0 ? "line " + std::to_string(lineno) + ": " + msg : msg;
}

// Tokenizer of parsers.cpp:24-75: whitespace separated, "quoted" tokens, an unquoted
// token starting with '#' ends the line.
class Tokens {
public:
	Tokens(const std::string& line, int lineno) : in_(line), lineno_(lineno) {}

	std::string next() {
		int c;
		for (;;) {
			c = in_.peek();
			if (c == EOF) return std::string();
			if (!std::isspace(c)) break;
			in_.get();
		}
		std::string tok;
		const bool quoted = in_.peek() == '"';
		if (quoted) {
			in_.get();
			while ((c = in_.get()) != '"') {
				if (c == EOF) throw ParseError{at_line("unclosed quotes", lineno_)};
				tok.push_back(static_cast<char>(c));
			}
		} else {
			while ((c = in_.get()) != EOF && !std::isspace(c)) tok.push_back(static_cast<char>(c));
		}
		if (!quoted && !tok.empty() && tok[0] == '#') {
			tok.clear();
			in_.ignore(std::numeric_limits<std::streamsize>::max());
		}
		return tok;
	}

	std::vector<std::string> rest() {
		std::vector<std::string> out;
		for (std::string t = next(); !t.empty(); t = next()) out.push_back(t);
		return out;
	}

	std::vector<double> numbers() {
		std::vector<double> out;
		for (const std::string& t : rest()) {
			try {
				out.push_back(std::stod(t));
			} catch (const std::logic_error&) {
				throw ParseError{at_line("invalid number " + t, lineno_)};
			}
		}
		return out;
	}

private:
	std::istringstream in_;
	int lineno_;
};

void warn(Scene& s, const std::string& msg, int lineno) { s.warnings += "Warning: " + at_line(msg, lineno) + "\n"; }

void sub4(const double a[4], const double b[4], double o[4]) {
	for (int i = 0; i < 4; i++) o[i] = a[i] - b[i];
}
void cross4(const double a[4], const double b[4], double o[4]) {  // Util::cross (util.h:22-26)
	o[0] = a[1] * b[2] - a[2] * b[1];
	o[1] = a[2] * b[0] - a[0] * b[2];
	o[2] = a[0] * b[1] - a[1] * b[0];
	o[3] = 0.0;
}

// Mesh::addTriangle (geometry.cpp:128-143): two one-sided faces offset by +-eps along n.
void add_triangle(Scene& s, Geometry& g, const double v[3][4]) {
	double e1[4], e2[4], n[4];
	sub4(v[1], v[0], e1);
	sub4(v[2], v[0], e2);
	cross4(e1, e2, n);
	const double len = std::sqrt(dot4(n, n));
	for (int i = 0; i < 4; i++) n[i] = n[i] / len;  // normalized(): division
	double sum[4];
	for (int i = 0; i < 4; i++) sum[i] = (v[0][i] + v[1][i]) + v[2][i];
	const double scale = (std::numeric_limits<double>::epsilon() * std::sqrt(dot4(sum, sum))) / 3;
	double ep[4];
	for (int i = 0; i < 4; i++) ep[i] = scale * n[i];
	for (int sgn = -1; sgn <= 1; sgn += 2) {
		Face f;
		for (int k = 0; k < 3; k++)
			for (int i = 0; i < 4; i++) {
				f.p[k][i] = v[k][i] + sgn * ep[i];
				f.n[k][i] = sgn * n[i];
			}
		s.faces.push_back(f);
		g.face_count++;
	}
}

// Mesh::updateBoundingBox (geometry.cpp:145-162)
void update_bounding_box(const Scene& s, Geometry& g) {
	g.box_valid = true;
	if (g.face_count == 0) {
		for (int i = 0; i < 4; i++) g.bb_min[i] = g.bb_max[i] = 0.0;
		return;
	}
	const double inf = std::numeric_limits<double>::infinity();
	for (int i = 0; i < 4; i++) {
		g.bb_min[i] = inf;
		g.bb_max[i] = -inf;
	}
	for (int64_t f = g.face_begin; f < g.face_begin + g.face_count; f++)
		for (int k = 0; k < 3; k++)
			for (int i = 0; i < 4; i++) {
				const double x = s.faces[f].p[k][i];
				g.bb_min[i] = (x < g.bb_min[i]) ? x : g.bb_min[i];  // std::min(cur, x)
				g.bb_max[i] = (g.bb_max[i] < x) ? x : g.bb_max[i];  // std::max(cur, x)
			}
	if (g.bb_min[3] != 1.0 || g.bb_max[3] != 1.0) throw MathError{"non-unity-homogeneous bounding box"};
}

// OBJParser::parseFile (parsers.cpp:253-374)
void parse_obj_file(Scene& s, Geometry& g, const std::string& path) {
	std::ifstream in(path);
	if (!in) throw ParseError{"file not found: " + path};
	std::vector<std::array<double, 4>> verts(1), norms(1);  // 1-indexed
	int lineno = 1;
	for (std::string line; std::getline(in, line); lineno++) {
		Tokens tk(line, lineno);
		const std::string kind = tk.next();
		if (kind.empty()) continue;
		if (kind == "v") {
			std::vector<double> p = tk.numbers();
			if (p.size() != 3 && p.size() != 4) throw ParseError{at_line("v requires 3 or 4 parameters", lineno)};
			p.push_back(1.0);
			if (p[3] == 0) throw ParseError{at_line("v must be a point vector", lineno)};
			verts.push_back({p[0], p[1], p[2], p[3]});
		} else if (kind == "vn") {
			std::vector<double> p = tk.numbers();
			if (p.size() != 3) throw ParseError{at_line("vn requires 3 parameters", lineno)};
			norms.push_back({p[0], p[1], p[2], 0.0});
		} else if (kind == "f") {
			const std::vector<std::string> toks = tk.rest();
			if (toks.size() < 3) throw ParseError{at_line("f requires at least 3 vertices", lineno)};
			std::vector<std::pair<int, int>> corner;  // (vertex, normal) indices, 0 = none
			for (const std::string& tok : toks) {
				int idx[3] = {0, 0, 0};
				int used = 0;
				size_t at = 0;
				while (used < 3 && at < tok.size()) {
					size_t slash = tok.find('/', at);
					if (slash == std::string::npos) slash = tok.size();
					const std::string part = tok.substr(at, slash - at);
					at = slash + 1;
					int value = 0;
					if (!part.empty()) {
						try {
							value = std::stoi(part);
						} catch (const std::logic_error&) {
							throw ParseError{at_line("invalid integer " + part, lineno)};
						}
						if (value <= 0) throw ParseError{at_line("index must be positive", lineno)};
					}
					idx[used++] = value;
				}
				if (idx[0] == 0) throw ParseError{at_line("vertex index is required", lineno)};
				if (static_cast<size_t>(idx[0]) >= verts.size()) throw ParseError{at_line("vertex index out of range", lineno)};
				if (idx[2] != 0 && static_cast<size_t>(idx[2]) >= norms.size())
					throw ParseError{at_line("normal index out of range", lineno)};
				corner.emplace_back(idx[0], idx[2]);
			}
			// fan triangulation around corner 0 (parsers.cpp:329-350)
			for (size_t k = 1; k + 1 < corner.size(); k++) {
				const std::pair<int, int>* tri[3] = {&corner[0], &corner[k], &corner[k + 1]};
				double e1[4], e2[4], n[4];
				sub4(verts[tri[1]->first].data(), verts[tri[0]->first].data(), e1);
				sub4(verts[tri[2]->first].data(), verts[tri[0]->first].data(), e2);
				cross4(e1, e2, n);
				if (is_zero(n, 4)) {
					warn(s, "degenerate face", lineno);
					continue;
				}
				// calculatedNormal.normalize(): `*this /= norm()` = multiply by 1/norm
				const double rcp = 1.0 / std::sqrt(dot4(n, n));
				for (int i = 0; i < 4; i++) n[i] = n[i] * rcp;
				Face f;
				for (int c = 0; c < 3; c++) {
					const double* nn = tri[c]->second ? norms[tri[c]->second].data() : n;
					for (int i = 0; i < 4; i++) {
						f.p[c][i] = verts[tri[c]->first][i];
						f.n[c][i] = nn[i];
					}
				}
				s.faces.push_back(f);
				g.face_count++;
			}
		} else {
			warn(s, "unknown obj line type " + kind, lineno);
		}
	}
}

struct LineSpec {
	const char* name;
	int pmin, pmax;
};
const LineSpec kSpecs[] = {  // RTIParser::LINE_TYPES (parsers.cpp:5-19)
    {"cam", 15, 15}, {"sph", 4, 4}, {"tri", 9, 9}, {"ltp", 6, 7}, {"ltd", 6, 6}, {"lta", 3, 3},
    {"mat", 13, 17}, {"xft", 3, 3}, {"xfr", 3, 3}, {"xfs", 3, 3}, {"xfz", 0, 0}};

std::string dir_of(const std::string& path) {  // Util::dirname (libgen)
	std::vector<char> buf(path.begin(), path.end());
	buf.push_back('\0');
	return std::string(::dirname(buf.data()));
}

}  // namespace

void parse_rti_file(Scene& s, const std::string& path) {
	std::ifstream in(path);
	if (!in) throw ParseError{"file not found: " + path};
	Affine xf = affine_identity();
	Material mat;  // zero until the first `mat` line (the reference leaves it indeterminate)
	int lineno = 1;
	for (std::string line; std::getline(in, line); lineno++) {
		Tokens tk(line, lineno);
		const std::string kind = tk.next();
		if (kind.empty()) continue;
		if (kind == "obj") {
			std::string file = tk.next();
			if (file.empty()) throw ParseError{at_line("obj requires a filename", lineno)};
			if (file[0] != '/') file = dir_of(path) + "/" + file;
			Geometry g{};
			g.kind = GEOM_MESH;
			g.fwd = xf;
			g.inv = affine_inverse(xf);
			g.det = affine_det4(xf);
			g.mat = mat;
			g.face_begin = static_cast<int64_t>(s.faces.size());
			parse_obj_file(s, g, file);
			update_bounding_box(s, g);
			s.geoms.push_back(g);
			continue;
		}
		const LineSpec* spec = nullptr;
		for (const LineSpec& ls : kSpecs)
			if (kind == ls.name) spec = &ls;
		if (!spec) {
			warn(s, "unknown line type " + kind, lineno);
			continue;
		}
		std::vector<double> p = tk.numbers();
		if (static_cast<int>(p.size()) < spec->pmin) {
			throw ParseError{at_line(kind + " requires " + (spec->pmin == spec->pmax ? "" : "at least ") +
			                             std::to_string(spec->pmin) + " parameters",
			                         lineno)};
		}
		if (static_cast<int>(p.size()) > spec->pmax) warn(s, "extra parameters found", lineno);
		while (static_cast<int>(p.size()) < spec->pmax) p.push_back(0.0);
		auto point = [&](int o, double out[4]) {  // hvec: (x, y, z, 1)
			out[0] = p[o];
			out[1] = p[o + 1];
			out[2] = p[o + 2];
			out[3] = 1.0;
		};
		auto color = [&](int o, double out[3]) {
			for (int i = 0; i < 3; i++) out[i] = p[o + i];
		};
		auto begin_geometry = [&](GeomKind k) {
			Geometry g{};
			g.kind = k;
			g.fwd = xf;
			g.inv = affine_inverse(xf);
			g.det = affine_det4(xf);
			g.mat = mat;
			return g;
		};
		if (kind == "xfz") {
			xf = affine_identity();
		} else if (kind == "xft") {
			affine_translate(xf, &p[0]);
		} else if (kind == "xfs") {
			affine_scale(xf, &p[0]);
		} else if (kind == "xfr") {
			if (!is_zero(&p[0], 3)) {
				const double len = norm3(&p[0]);
				const double axis[3] = {p[0] / len, p[1] / len, p[2] / len};
				double R[3][3];
				angle_axis(len * (2 * M_PI / 360.0), axis, R);
				affine_rotate(xf, R);
			}
		} else if (kind == "mat") {
			color(0, mat.ka);
			color(3, mat.kd);
			color(6, mat.ks);
			mat.ns = p[9];
			color(10, mat.kr);
			color(13, mat.kt);
			mat.ior = p[16];
		} else if (kind == "cam") {
			s.has_camera = true;
			s.cam_fwd = xf;
			for (int k = 0; k < 5; k++) {
				point(3 * k, s.cam_raw[k]);
				affine_apply(xf, s.cam_raw[k], s.cam[k]);
			}
		} else if (kind == "sph") {
			Geometry g = begin_geometry(GEOM_SPHERE);
			point(0, g.center);
			g.radius = static_cast<float>(p[3]);
			s.geoms.push_back(g);
		} else if (kind == "tri") {
			Geometry g = begin_geometry(GEOM_MESH);
			g.face_begin = static_cast<int64_t>(s.faces.size());
			double v[3][4];
			for (int k = 0; k < 3; k++) point(3 * k, v[k]);
			add_triangle(s, g, v);
			// no updateBoundingBox for `tri` (parsers.cpp:213-221): box stays zero -> no gate
			s.geoms.push_back(g);
		} else if (kind == "ltp") {
			Light l{};
			l.kind = LIGHT_POINT;
			l.fwd = xf;
			point(0, l.raw);
			affine_apply(xf, l.raw, l.vec);
			color(3, l.color);
			l.falloff = p[6];
			s.lights.push_back(l);
		} else if (kind == "ltd") {
			if (is_zero(&p[0], 3)) throw ParseError{at_line("zero direction specified", lineno)};
			const double len = norm3(&p[0]);
			const double d[4] = {p[0] / len, p[1] / len, p[2] / len, 0.0};
			Light l{};
			l.kind = LIGHT_DIRECTIONAL;
			l.fwd = xf;
			std::copy(d, d + 4, l.raw);
			affine_apply(xf, d, l.vec);
			color(3, l.color);
			s.lights.push_back(l);
		} else if (kind == "lta") {
			Light l{};
			l.kind = LIGHT_AMBIENT;
			l.fwd = xf;
			color(0, l.color);
			s.lights.push_back(l);
		}
	}
}

Affine affine_from_eigen(const double cm[16]) {
	Affine a;
	for (int i = 0; i < 3; i++)
		for (int j = 0; j < 4; j++) a.m[i][j] = cm[j * 4 + i];
	return a;
}

void affine_to_eigen(const Affine& a, double cm[16]) {
	for (int j = 0; j < 4; j++) {
		for (int i = 0; i < 3; i++) cm[j * 4 + i] = a.m[i][j];
		cm[j * 4 + 3] = j == 3 ? 1.0 : 0.0;  // Affine mode: last row (0 0 0 1)
	}
}

void apply_scene_transforms(Scene& s) {
	if (s.has_camera)
		for (int k = 0; k < 5; k++) affine_apply(s.cam_fwd, s.cam_raw[k], s.cam[k]);
	for (Light& l : s.lights)
		if (l.kind != LIGHT_AMBIENT) affine_apply(l.fwd, l.raw, l.vec);
}

}  // namespace rtamd
