// TEST INFRASTRUCTURE ONLY — CPU oracle (restatement of the reference render path).
//
// Follows, function by function:
//   scene ingest    /root/reference/src/parsers.cpp:5-374, geometry.cpp:128-162
//   transforms      rtbase.h:41-64 + Eigen 3.2.2 evaluation orders
//   render loop     scene.cpp:10-59
//   shading         scene.cpp:61-140 (traceRay), 142-167 (castRay)
//   intersection    geometry.cpp:5-126 (box gate, object-space transform, sphere, mesh)
//   camera/lights   rtbase.h:74-95, lights.h:3-75
// It is deliberately the reference's own brute-force algorithm (no BVH): it is the
// parity checker and the CPU baseline ("kind": "port") for bench.py.
//
// Differences that cannot change a pixel of any reference run that completes:
//   * camera/light transforms are computed once up front (the reference caches them
//     lazily and races under threads, rtbase.h:86-95, lights.h:28-33,56-61);
//   * the last 2000-pixel block is clamped (the reference aborts instead, scene.cpp:21-25);
//   * a geometry defined before any `mat` line gets an all-zero material (the
//     reference reads indeterminate memory, parsers.h:46 / rtbase.h:30-39);
//   * MathException is returned as an error code instead of std::terminate.
#include "oracle.h"
#include <libgen.h>
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace {

// ---------------------------------------------------------------- errors
struct ParseError : std::runtime_error { using std::runtime_error::runtime_error; };
struct MathError : std::runtime_error { using std::runtime_error::runtime_error; };

std::string g_last_error;
std::string g_warnings;

std::string lineMsg(const std::string& msg, int lineno) {  // exceptions.cpp:3-11
	if (lineno > 0) return "line " + std::to_string(lineno) + ": " + msg;
	return msg;
}
void warn(const std::string& msg, int lineno) { g_warnings += "Warning: " + lineMsg(msg, lineno) + "\n"; }

// ---------------------------------------------------------------- Eigen-order vector math
struct V4 { double x, y, z, w; };
struct V3 { double x, y, z; };
struct C3 { double r, g, b; };

inline V4 v4(double x, double y, double z, double w) { return V4{x, y, z, w}; }
inline V4 operator+(const V4& a, const V4& b) { return v4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
inline V4 operator-(const V4& a, const V4& b) { return v4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
inline V4 operator-(const V4& a) { return v4(-a.x, -a.y, -a.z, -a.w); }
inline V4 operator*(double s, const V4& a) { return v4(s * a.x, s * a.y, s * a.z, s * a.w); }
// Vector4d::dot / squaredNorm with SSE2 packets: (a0b0 + a2b2) + (a1b1 + a3b3)
inline double dot4(const V4& a, const V4& b) { return (a.x * b.x + a.z * b.z) + (a.y * b.y + a.w * b.w); }
inline double norm4(const V4& a) { return std::sqrt(dot4(a, a)); }
// normalized(): true division by the norm (Dot.h:139-145)
inline V4 normalized4(const V4& a) { double n = norm4(a); return v4(a.x / n, a.y / n, a.z / n, a.w / n); }
// normalize() is `*this /= norm()`, and DenseBase::operator/= multiplies by the
// reciprocal for floating scalars (SelfCwiseBinaryOp.h:181-193): a * (1/|a|)
inline V4 normalizeInPlace4(const V4& a) { double r = 1.0 / norm4(a); return v4(a.x * r, a.y * r, a.z * r, a.w * r); }
// isZero(): every |coeff| <= dummy_precision<double>() = 1e-12
inline bool isZero4(const V4& a) {
	return std::fabs(a.x) <= 1e-12 && std::fabs(a.y) <= 1e-12 && std::fabs(a.z) <= 1e-12 && std::fabs(a.w) <= 1e-12;
}
inline bool isZeroC(const C3& c) { return std::fabs(c.r) <= 1e-12 && std::fabs(c.g) <= 1e-12 && std::fabs(c.b) <= 1e-12; }
// Vector3d::dot / norm: a0b0 + (a1b1 + a2b2)
inline double norm3(const V3& a) { return std::sqrt(a.x * a.x + (a.y * a.y + a.z * a.z)); }
// Vector3d::cross
inline V4 cross4(const V4& a, const V4& b) {
	return v4(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x, 0.0);
}

inline C3 operator+(const C3& a, const C3& b) { return C3{a.r + b.r, a.g + b.g, a.b + b.b}; }
inline C3 operator*(const C3& a, const C3& b) { return C3{a.r * b.r, a.g * b.g, a.b * b.b}; }
inline C3 operator*(double s, const C3& a) { return C3{s * a.r, s * a.g, s * a.b}; }

// Transform<double,3,Affine>: 4x4 matrix, last row kept (0,0,0,1)
struct Xf {
	double m[4][4];
	static Xf identity() {
		Xf t;
		for (int i = 0; i < 4; i++)
			for (int j = 0; j < 4; j++) t.m[i][j] = (i == j) ? 1.0 : 0.0;
		return t;
	}
	// Transform::translate (Transform.h:838-843): t += L*v, row sums sequential
	void translate(const double v[3]) {
		for (int k = 0; k < 3; k++)
			m[k][3] = m[k][3] + ((m[k][0] * v[0] + m[k][1] * v[1]) + m[k][2] * v[2]);
	}
	// Transform::scale (Transform.h:784-790): L = L * diag(v)
	void scale(const double v[3]) {
		for (int i = 0; i < 3; i++)
			for (int j = 0; j < 3; j++) m[i][j] = m[i][j] * v[j];
	}
	// Transform::rotate (Transform.h:882-886): L = L * R
	void rotate(const double R[3][3]) {
		double L[3][3];
		for (int i = 0; i < 3; i++)
			for (int j = 0; j < 3; j++) L[i][j] = m[i][j];
		for (int i = 0; i < 3; i++)
			for (int j = 0; j < 3; j++) m[i][j] = (L[i][0] * R[0][j] + L[i][1] * R[1][j]) + L[i][2] * R[2][j];
	}
	// Transform::inverse(Affine) (Transform.h:1124-1151) with the 3x3 cofactor inverse
	// of LU/Inverse.h:117-159
	Xf inverse() const {
		auto a = [&](int i, int j) { return m[i][j]; };
		auto cof = [&](int i, int j) {
			int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
			return a(i1, j1) * a(i2, j2) - a(i1, j2) * a(i2, j1);
		};
		double c00 = cof(0, 0), c10 = cof(1, 0), c20 = cof(2, 0);
		double det = c00 * a(0, 0) + (c10 * a(1, 0) + c20 * a(2, 0));
		double invdet = 1.0 / det;
		Xf r = identity();
		r.m[0][0] = c00 * invdet; r.m[0][1] = c10 * invdet; r.m[0][2] = c20 * invdet;
		r.m[1][0] = cof(0, 1) * invdet; r.m[1][1] = cof(1, 1) * invdet; r.m[1][2] = cof(2, 1) * invdet;
		r.m[2][0] = cof(0, 2) * invdet; r.m[2][1] = cof(1, 2) * invdet; r.m[2][2] = cof(2, 2) * invdet;
		for (int k = 0; k < 3; k++)
			r.m[k][3] = ((-r.m[k][0]) * m[0][3] + (-r.m[k][1]) * m[1][3]) + (-r.m[k][2]) * m[2][3];
		return r;
	}
	// Matrix4d::determinant (LU/Determinant.h:71-83)
	double det4() const {
		auto h = [&](int j, int k, int p, int n) {
			return (m[j][0] * m[k][1] - m[k][0] * m[j][1]) * (m[p][2] * m[n][3] - m[n][2] * m[p][3]);
		};
		return ((((h(0, 1, 2, 3) - h(0, 2, 1, 3)) + h(0, 3, 1, 2)) + h(1, 2, 0, 3)) - h(1, 3, 0, 2)) + h(2, 3, 0, 1);
	}
	// Transform * Vector4d (Affine: Transform.h:1244-1267): top rows sequential, w copied
	V4 apply(const V4& v) const {
		double r[3];
		for (int k = 0; k < 3; k++) r[k] = ((m[k][0] * v.x + m[k][1] * v.y) + m[k][2] * v.z) + m[k][3] * v.w;
		return v4(r[0], r[1], r[2], v.w);
	}
	// matrix().transpose() * Vector4d: packet order (M0k n0 + M2k n2) + (M1k n1 + M3k n3)
	V4 applyTransposed(const V4& n) const {
		double r[4];
		for (int k = 0; k < 4; k++) r[k] = (m[0][k] * n.x + m[2][k] * n.z) + (m[1][k] * n.y + m[3][k] * n.w);
		return v4(r[0], r[1], r[2], r[3]);
	}
};

// AngleAxis<double>::toRotationMatrix (Eigen Geometry/AngleAxis.h:204-229)
void angleAxisMatrix(double angle, const V3& ax, double R[3][3]) {
	double s = std::sin(angle), c = std::cos(angle);
	V3 sa{s * ax.x, s * ax.y, s * ax.z};
	V3 ca{(1.0 - c) * ax.x, (1.0 - c) * ax.y, (1.0 - c) * ax.z};
	double t;
	t = ca.x * ax.y; R[0][1] = t - sa.z; R[1][0] = t + sa.z;
	t = ca.x * ax.z; R[0][2] = t + sa.y; R[2][0] = t - sa.y;
	t = ca.y * ax.z; R[1][2] = t - sa.x; R[2][1] = t + sa.x;
	R[0][0] = ca.x * ax.x + c; R[1][1] = ca.y * ax.y + c; R[2][2] = ca.z * ax.z + c;
}

// ---------------------------------------------------------------- scene model
struct Ray {  // rtbase.h:5-28
	V4 o, d;
	Ray(const V4& ori, const V4& dir) {
		if (ori.w == 0) throw MathError("ray origin is a direction vector");
		if (isZero4(dir)) throw MathError("ray has no direction");
		if (dir.w != 0) throw MathError("ray direction is a point vector");
		o = ori;
		d = normalized4(dir);
	}
};

struct Material {  // rtbase.h:30-39 (zero default, see header)
	C3 ka{0, 0, 0}, kd{0, 0, 0}, ks{0, 0, 0}, kr{0, 0, 0};
	double ns = 0;
	C3 kt{0, 0, 0};
	double ior = 0;
};

struct Face { V4 p[3], n[3]; };  // geometry.h:32

struct Geometry {  // geometry.h:6-37 (sphere + mesh in one record)
	bool isSphere = false;
	Xf fwd = Xf::identity(), inv = Xf::identity();
	double det = 1.0;
	Material mat;
	V4 center{0, 0, 0, 1};
	float radius = 0.f;
	std::vector<Face> faces;
	V4 bbMin{0, 0, 0, 0}, bbMax{0, 0, 0, 0};
	void setTransform(const Xf& xf) { fwd = xf; inv = xf.inverse(); det = fwd.det4(); }
};

enum LightKind { LIGHT_POINT, LIGHT_DIR, LIGHT_AMBIENT };
struct Light {  // lights.h
	LightKind kind;
	C3 color;
	V4 xfPoint, xfDir;  // precomputed fwd*point / fwd*direction
	double falloff = 0;
};

struct SceneData {
	bool hasCamera = false;
	V4 eye, ll, lr, ul, ur;  // transformed camera corners (rtbase.h:86-95)
	std::vector<Geometry> geoms;
	std::vector<Light> lights;
};

struct Counters {
	int64_t trace = 0, shadow = 0, refl = 0, refr = 0, sph = 0, mesh = 0, bbox = 0, face = 0;
};

// ---------------------------------------------------------------- parsing (parsers.cpp)
std::string extractToken(std::istream& s, int lineno) {  // parsers.cpp:24-64
	int c;
	while (true) {
		c = s.peek();
		if (c == EOF) return std::string();
		if (!std::isspace(c)) break;
		s.get();
	}
	bool quoted = s.peek() == '"';
	std::string str;
	if (quoted) {
		s.get();
		while (true) {
			c = s.get();
			if (c == EOF) throw ParseError(lineMsg("unclosed quotes", lineno));
			if (c == '"') break;
			str.push_back((char)c);
		}
	} else {
		while (true) {
			c = s.get();
			if (c == EOF || std::isspace(c)) break;
			str.push_back((char)c);
		}
	}
	if (!quoted && !str.empty() && str[0] == '#') {
		str.clear();
		s.ignore(std::numeric_limits<std::streamsize>::max());
	}
	return str;
}

std::vector<std::string> extractTokens(std::istream& s, int lineno) {
	std::vector<std::string> t;
	for (std::string tok; !(tok = extractToken(s, lineno)).empty();) t.push_back(tok);
	return t;
}

std::vector<double> extractDoubles(std::istream& s, int lineno) {  // parsers.cpp:77-91
	std::vector<double> out;
	for (const std::string& tok : extractTokens(s, lineno)) {
		try {
			out.push_back(std::stod(tok));
		} catch (std::logic_error&) {
			throw ParseError(lineMsg("invalid number " + tok, lineno));
		}
	}
	return out;
}

std::string dirnameOf(const std::string& path) {  // util.h:8-20
	std::vector<char> buf(path.begin(), path.end());
	buf.push_back('\0');
	return std::string(::dirname(buf.data()));
}

void updateBoundingBox(Geometry& g) {  // geometry.cpp:145-162
	if (g.faces.empty()) { g.bbMin = v4(0, 0, 0, 0); g.bbMax = v4(0, 0, 0, 0); return; }
	const double inf = std::numeric_limits<double>::infinity();
	V4 mn = v4(inf, inf, inf, inf), mx = v4(-inf, -inf, -inf, -inf);
	for (const Face& f : g.faces)
		for (const V4& p : f.p) {
			mn = v4(std::min(mn.x, p.x), std::min(mn.y, p.y), std::min(mn.z, p.z), std::min(mn.w, p.w));
			mx = v4(std::max(mx.x, p.x), std::max(mx.y, p.y), std::max(mx.z, p.z), std::max(mx.w, p.w));
		}
	if (mn.w != 1.0 || mx.w != 1.0) throw MathError("non-unity-homogeneous bounding box");
	g.bbMin = mn; g.bbMax = mx;
}

void addTriangle(Geometry& g, const V4& v0, const V4& v1, const V4& v2) {  // geometry.cpp:128-143
	V4 n = normalized4(cross4(v1 - v0, v2 - v0));
	V4 ep = ((std::numeric_limits<double>::epsilon() * norm4((v0 + v1) + v2)) / 3) * n;
	for (int s = -1; s <= 1; s += 2) {
		Face f;
		const V4 pts[3] = {v0, v1, v2};
		for (int i = 0; i < 3; i++) {
			f.p[i] = pts[i] + (double)s * ep;
			f.n[i] = (double)s * n;
		}
		g.faces.push_back(f);
	}
}

void parseObj(Geometry& mesh, const std::string& filename) {  // parsers.cpp:253-374
	std::ifstream stream(filename);
	if (!stream) throw ParseError("file not found: " + filename);
	std::vector<V4> verts(1), norms(1);  // 1-indexed
	int lineno = 1;
	for (std::string line; std::getline(stream, line); lineno++) {
		std::istringstream ss(line);
		std::string type = extractToken(ss, lineno);
		if (type.empty()) continue;
		if (type == "f") {
			std::vector<std::string> toks = extractTokens(ss, lineno);
			if (toks.size() < 3) throw ParseError(lineMsg("f requires at least 3 vertices", lineno));
			struct Pt { int vi, ni; };
			std::vector<Pt> pts;
			for (const std::string& s : toks) {
				int idx[3] = {0, 0, 0};
				int count = 0;
				size_t pos = 0;
				while (count < 3 && pos < s.length()) {
					size_t nd = s.find('/', pos);
					if (nd == std::string::npos) nd = s.length();
					std::string part = s.substr(pos, nd - pos);
					pos = nd + 1;
					int value = 0;
					if (!part.empty()) {
						try {
							value = std::stoi(part);
						} catch (std::logic_error&) {
							throw ParseError(lineMsg("invalid integer " + part, lineno));
						}
						if (value <= 0) throw ParseError(lineMsg("index must be positive", lineno));
					}
					idx[count++] = value;
				}
				if (idx[0] == 0) throw ParseError(lineMsg("vertex index is required", lineno));
				if ((size_t)idx[0] >= verts.size()) throw ParseError(lineMsg("vertex index out of range", lineno));
				if (idx[2] != 0 && (size_t)idx[2] >= norms.size())
					throw ParseError(lineMsg("normal index out of range", lineno));
				pts.push_back(Pt{idx[0], idx[2]});
			}
			// fan triangulation, parsers.cpp:329-350
			for (size_t k = 1; k + 1 < pts.size(); k++) {
				const Pt* tri[3] = {&pts[0], &pts[k], &pts[k + 1]};
				V4 nrm = cross4(verts[tri[1]->vi] - verts[tri[0]->vi], verts[tri[2]->vi] - verts[tri[0]->vi]);
				if (isZero4(nrm)) { warn("degenerate face", lineno); continue; }
				nrm = normalizeInPlace4(nrm);  // calculatedNormal.normalize(), parsers.cpp:340
				Face f;
				for (int i = 0; i < 3; i++) {
					f.p[i] = verts[tri[i]->vi];
					f.n[i] = tri[i]->ni ? norms[tri[i]->ni] : nrm;
				}
				mesh.faces.push_back(f);
			}
		} else if (type == "v") {
			std::vector<double> p = extractDoubles(ss, lineno);
			if (p.size() != 3 && p.size() != 4) throw ParseError(lineMsg("v requires 3 or 4 parameters", lineno));
			p.push_back(1.0);
			V4 v = v4(p[0], p[1], p[2], p[3]);
			if (v.w == 0) throw ParseError(lineMsg("v must be a point vector", lineno));
			verts.push_back(v);
		} else if (type == "vn") {
			std::vector<double> p = extractDoubles(ss, lineno);
			if (p.size() != 3) throw ParseError(lineMsg("vn requires 3 parameters", lineno));
			norms.push_back(v4(p[0], p[1], p[2], 0.0));
		} else {
			warn("unknown obj line type " + type, lineno);
		}
	}
}

void parseRti(SceneData& scene, const std::string& filename) {  // parsers.cpp:93-251
	struct LT { int pmin, pmax; };
	static const std::map<std::string, LT> kTypes = {
		{"cam", {15, 15}}, {"sph", {4, 4}}, {"tri", {9, 9}}, {"ltp", {6, 7}}, {"ltd", {6, 6}},
		{"lta", {3, 3}}, {"mat", {13, 17}}, {"xft", {3, 3}}, {"xfr", {3, 3}}, {"xfs", {3, 3}},
		{"xfz", {0, 0}}};
	std::ifstream stream(filename);
	if (!stream) throw ParseError("file not found: " + filename);
	Xf xf = Xf::identity();
	Material mat;
	int lineno = 1;
	for (std::string line; std::getline(stream, line); lineno++) {
		std::istringstream ss(line);
		std::string type = extractToken(ss, lineno);
		if (type.empty()) continue;
		if (type == "obj") {
			std::string fn = extractToken(ss, lineno);
			if (fn.empty()) throw ParseError(lineMsg("obj requires a filename", lineno));
			if (fn[0] != '/') fn = dirnameOf(filename) + "/" + fn;
			Geometry g;
			g.setTransform(xf);
			g.mat = mat;
			parseObj(g, fn);
			updateBoundingBox(g);
			scene.geoms.push_back(std::move(g));
			continue;
		}
		auto it = kTypes.find(type);
		if (it == kTypes.end()) { warn("unknown line type " + type, lineno); continue; }
		std::vector<double> p = extractDoubles(ss, lineno);
		const LT lt = it->second;
		if ((int)p.size() < lt.pmin) {
			throw ParseError(lineMsg(type + " requires " + (lt.pmin == lt.pmax ? "" : "at least ") +
			                         std::to_string(lt.pmin) + " parameters", lineno));
		} else if ((int)p.size() > lt.pmax) {
			warn("extra parameters found", lineno);
		}
		while ((int)p.size() < lt.pmax) p.push_back(0.0);
		auto C = [&](int o) { return C3{p[o], p[o + 1], p[o + 2]}; };
		auto H = [&](int o) { return v4(p[o], p[o + 1], p[o + 2], 1.0); };
		if (type == "xfz") {
			xf = Xf::identity();
		} else if (type == "xft") {
			xf.translate(&p[0]);
		} else if (type == "xfs") {
			xf.scale(&p[0]);
		} else if (type == "xfr") {
			V3 r{p[0], p[1], p[2]};
			if (!(std::fabs(r.x) <= 1e-12 && std::fabs(r.y) <= 1e-12 && std::fabs(r.z) <= 1e-12)) {
				double n = norm3(r);
				double R[3][3];
				angleAxisMatrix(n * (2 * M_PI / 360.0), V3{r.x / n, r.y / n, r.z / n}, R);
				xf.rotate(R);
			}
		} else if (type == "mat") {
			mat.ka = C(0); mat.kd = C(3); mat.ks = C(6); mat.kr = C(10); mat.kt = C(13);
			mat.ns = p[9]; mat.ior = p[16];
		} else if (type == "cam") {
			scene.hasCamera = true;
			scene.eye = xf.apply(H(0)); scene.ll = xf.apply(H(3)); scene.lr = xf.apply(H(6));
			scene.ul = xf.apply(H(9)); scene.ur = xf.apply(H(12));
		} else if (type == "sph") {
			Geometry g;
			g.isSphere = true;
			g.setTransform(xf);
			g.mat = mat;
			g.center = H(0);
			g.radius = (float)p[3];
			scene.geoms.push_back(std::move(g));
		} else if (type == "tri") {
			Geometry g;
			g.setTransform(xf);
			g.mat = mat;
			addTriangle(g, H(0), H(3), H(6));
			// the reference never calls updateBoundingBox for a `tri` mesh (parsers.cpp:213-221):
			// its box stays (0,0,0,0)-(0,0,0,0), so the gate at geometry.cpp:72 is skipped
			scene.geoms.push_back(std::move(g));
		} else if (type == "ltp") {
			Light l;
			l.kind = LIGHT_POINT;
			l.xfPoint = xf.apply(H(0));
			l.color = C(3);
			l.falloff = p[6];
			scene.lights.push_back(l);
		} else if (type == "ltd") {
			V3 c{p[0], p[1], p[2]};
			if (std::fabs(c.x) <= 1e-12 && std::fabs(c.y) <= 1e-12 && std::fabs(c.z) <= 1e-12)
				throw ParseError(lineMsg("zero direction specified", lineno));
			double n = norm3(c);
			Light l;
			l.kind = LIGHT_DIR;
			l.xfDir = xf.apply(v4(c.x / n, c.y / n, c.z / n, 0.0));
			l.color = C(3);
			scene.lights.push_back(l);
		} else if (type == "lta") {
			Light l;
			l.kind = LIGHT_AMBIENT;
			l.color = C(0);
			scene.lights.push_back(l);
		}
	}
}

// ---------------------------------------------------------------- intersection (geometry.cpp)
bool hitsBoundingBox(const Ray& ray, const V4& mn, const V4& mx) {  // geometry.cpp:5-29
	const double o[3] = {ray.o.x, ray.o.y, ray.o.z};
	const double d[3] = {ray.d.x, ray.d.y, ray.d.z};
	const double lo[3] = {mn.x, mn.y, mn.z}, hi[3] = {mx.x, mx.y, mx.z};
	for (int axis = 0; axis < 3; axis++) {
		for (int bn = 0; bn < 2; bn++) {
			double mag = d[axis];
			if (mag == 0.0) continue;
			double t = ((bn ? hi : lo)[axis] - o[axis]) / mag;
			if (t < 0) continue;
			bool inside = true;
			for (int a2 = 0; a2 < 3; a2++) {
				if (a2 == axis) continue;
				double p = o[a2] + t * d[a2];
				if (p < lo[a2] || p > hi[a2]) { inside = false; break; }
			}
			if (inside) return true;
		}
	}
	return false;
}

bool sphereObj(const Geometry& g, const Ray& r, V4& P, V4& N, bool reverse, Counters& c) {  // geometry.cpp:47-67
	c.sph++;
	V4 oc = r.o - g.center;
	double a = dot4(r.d, r.d);
	double b = 2 * dot4(r.d, oc);
	float rr = g.radius * g.radius;  // fp32 multiply (float radius_, geometry.h:22)
	double cc = dot4(oc, oc) - (double)rr;
	double disc = b * b - (4 * a) * cc;
	if (disc < 0) return false;
	double t = reverse ? (-b + std::sqrt(disc)) / (2 * a) : (-b - std::sqrt(disc)) / (2 * a);
	if (t < 0) return false;
	P = r.o + t * r.d;
	N = P - g.center;
	return true;
}

inline double det3cols(const double c0[3], const double c1[3], const double c2[3]) {
	// Matrix3d::determinant with columns c0,c1,c2 (LU/Determinant.h:61-69):
	// m(0,0)*(m11 m22 - m12 m21) - m(0,1)*(m10 m22 - m12 m20) + m(0,2)*(m10 m21 - m11 m20)
	return (c0[0] * (c1[1] * c2[2] - c2[1] * c1[2]) - c1[0] * (c0[1] * c2[2] - c2[1] * c0[2])) +
	       c2[0] * (c0[1] * c1[2] - c1[1] * c0[2]);
}

bool meshObj(const Geometry& g, const Ray& r, V4& P, V4& N, bool reverse, Counters& c) {  // geometry.cpp:69-126
	c.mesh++;
	bool boxDiffers = g.bbMin.x != g.bbMax.x || g.bbMin.y != g.bbMax.y || g.bbMin.z != g.bbMax.z || g.bbMin.w != g.bbMax.w;
	if (boxDiffers && g.faces.size() > 1)
		if (!hitsBoundingBox(r, g.bbMin, g.bbMax)) return false;
	c.bbox++;
	bool found = false;
	double best = std::numeric_limits<double>::infinity();
	const double dir[3] = {r.d.x, r.d.y, r.d.z};
	const double nd[3] = {-r.d.x, -r.d.y, -r.d.z};
	const double dnorm = norm3(V3{dir[0], dir[1], dir[2]});
	for (const Face& f : g.faces) {
		c.face++;
		const double va[3] = {f.p[1].x - f.p[0].x, f.p[1].y - f.p[0].y, f.p[1].z - f.p[0].z};
		const double vb[3] = {f.p[2].x - f.p[0].x, f.p[2].y - f.p[0].y, f.p[2].z - f.p[0].z};
		const double rhs[3] = {r.o.x - f.p[0].x, r.o.y - f.p[0].y, r.o.z - f.p[0].z};
		double D = det3cols(va, vb, nd);
		if (D == 0) continue;
		double a = det3cols(rhs, vb, nd) / D;
		if (a < 0 || a > 1) continue;
		double b = det3cols(va, rhs, nd) / D;
		if (b < 0 || a + b > 1) continue;
		double t = det3cols(va, vb, rhs) / D;
		if (t < 0) continue;
		double dist = t * dnorm;
		if (dist >= best) continue;
		double w0 = (1.0 - a) - b;
		V4 tn = v4((w0 * f.n[0].x + a * f.n[1].x) + b * f.n[2].x, (w0 * f.n[0].y + a * f.n[1].y) + b * f.n[2].y,
		           (w0 * f.n[0].z + a * f.n[1].z) + b * f.n[2].z, (w0 * f.n[0].w + a * f.n[1].w) + b * f.n[2].w);
		bool front = dot4(tn, r.d) < 0;
		if (!front ^ reverse) continue;
		found = true;
		best = dist;
		P = v4(f.p[0].x + (a * va[0] + b * vb[0]), f.p[0].y + (a * va[1] + b * vb[1]),
		       f.p[0].z + (a * va[2] + b * vb[2]), f.p[0].w + 0.0);
		N = tn;
	}
	return found;
}

bool intersect(const Geometry& g, const Ray& ray, V4& P, V4& N, bool reverse, Counters& c) {  // geometry.cpp:31-45
	Ray objRay(g.inv.apply(ray.o), g.inv.apply(ray.d));
	V4 Po, No;
	bool hit = g.isSphere ? sphereObj(g, objRay, Po, No, reverse, c) : meshObj(g, objRay, Po, No, reverse, c);
	if (!hit) return false;
	P = g.fwd.apply(Po);
	N = g.inv.applyTransposed(No);
	N.w = 0;
	if (g.det < 0) N = -N;
	return true;
}

// ---------------------------------------------------------------- shading (scene.cpp)
struct Tracer {
	const SceneData& s;
	int bdepth;
	bool intersectionOnly;
	Counters c;

	bool castRay(const Ray& ray, double* dist, int* geom, V4* P, V4* N, bool reverse) {  // scene.cpp:142-167
		bool hit = false;
		double best = 0;
		for (size_t i = 0; i < s.geoms.size(); i++) {
			V4 tp, tn;
			if (!intersect(s.geoms[i], ray, tp, tn, reverse, c)) continue;
			double d = norm4(tp - ray.o);
			if (hit && d >= best) continue;
			hit = true;
			best = d;
			if (geom) *geom = (int)i;
			if (P) *P = tp;
			if (N) *N = tn;
		}
		if (hit) *dist = best;
		return hit;
	}

	C3 traceRay(const Ray& ray, int depth, bool inside) {  // scene.cpp:61-140
		c.trace++;
		int gi = -1;
		V4 P, N;
		double dist;
		if (!castRay(ray, &dist, &gi, &P, &N, inside)) return C3{0, 0, 0};
		if (intersectionOnly) { double v = 1.0 / (dist * dist); return C3{v, v, v}; }
		if (inside) N = -N;
		N = normalizeInPlace4(N);  // targetNormal.normalize(), scene.cpp:114
		const Material& m = s.geoms[gi].mat;
		C3 color{0, 0, 0};
		for (const Light& L : s.lights) {
			if (L.kind == LIGHT_AMBIENT) {
				color = color + (1.0 * L.color) * m.ka;
				continue;
			}
			V4 toL = (L.kind == LIGHT_POINT) ? (L.xfPoint - P) : -L.xfDir;
			Ray lray(P, toL);
			bool lrev = dot4(N, lray.d) < 0;
			double dL = (L.kind == LIGHT_POINT) ? norm4(L.xfPoint - P) : std::numeric_limits<double>::infinity();
			c.shadow++;
			double dOcc;
			if (castRay(lray, &dOcc, nullptr, nullptr, nullptr, lrev ^ inside) && dOcc <= dL) continue;
			C3 att = (L.kind == LIGHT_POINT) ? std::pow(dL, -L.falloff) * L.color : L.color;
			double diff = std::max(dot4(N, lray.d), 0.0);
			color = color + (diff * att) * m.kd;
			double nl2 = 2 * dot4(N, lray.d);
			V4 R = nl2 * N - lray.d;
			double spec = std::pow(std::max(-dot4(ray.d, R), 0.0), m.ns);
			color = color + (spec * att) * m.ks;
		}
		const V4& I = ray.d;
		C3 kr = m.kr;
		if (depth > 0) {
			if (!isZeroC(m.kt)) {
				double n = m.ior;
				if (!inside) n = 1.0 / n;
				double cosI = dot4(N, I);
				double sinT2 = n * n * (1.0 - cosI * cosI);
				if (sinT2 > 1.0) {
					kr = C3{1.0, 1.0, 1.0};
				} else {
					V4 T = n * I - (n * cosI + std::sqrt(1.0 - sinT2)) * N;
					Ray tr(P, T);
					c.refr++;
					color = color + traceRay(tr, depth - 1, !inside);
				}
			}
			if (!isZeroC(kr)) {
				V4 Rd = I - (2 * dot4(N, I)) * N;
				Ray rr(P, Rd);
				c.refl++;
				color = color + traceRay(rr, depth - 1, inside) * kr;
			}
		}
		return color;
	}
};

Ray viewingRay(const SceneData& s, double rF, double cF) {  // rtbase.h:74-84
	V4 p = cF * (rF * s.lr + (1.0 - rF) * s.ur) + (1.0 - cF) * (rF * s.ll + (1.0 - rF) * s.ul);
	return Ray(s.eye, p - s.eye);
}

}  // namespace

extern "C" int oracle_render(const char* const* files, int n_files, int W, int H, int bdepth, int intersection_only,
                             int threads, int row_begin, int row_end, int row_step, double* out,
                             oracle_counters* counters) {
	g_last_error.clear();
	g_warnings.clear();
	SceneData scene;
	try {
		for (int i = 0; i < n_files; i++) parseRti(scene, files[i]);
	} catch (const ParseError& e) {
		g_last_error = e.what();
		return 1;
	} catch (const MathError& e) {
		g_last_error = e.what();
		return 2;
	}
	if (!scene.hasCamera) {
		g_last_error = "At least one camera must be specified.";
		return 1;
	}
	if (W <= 0 || H <= 0 || row_begin < 0 || row_end > H || row_begin > row_end || row_step <= 0) {
		g_last_error = "bad image geometry";
		return 3;
	}
	const int64_t n_rows = (row_end - row_begin + row_step - 1) / row_step;
	const int64_t total = n_rows * W;  // selected pixels, dispensed in 2000-pixel blocks
	const int64_t block = 2000;  // scene.cpp:13
	std::atomic<int64_t> next(0);
	std::mutex mu;
	Counters sum;
	std::string err;
	auto worker = [&]() {
		Tracer t{scene, bdepth, intersection_only != 0, Counters{}};
		try {
			while (true) {
				int64_t start = next.fetch_add(block);
				if (start >= total) break;
				int64_t end = std::min(start + block, total);
				for (int64_t i = start; i < end; i++) {
					int r = row_begin + (int)(i / W) * row_step, c = (int)(i % W);
					double rF = (r + 0.5) / H;  // scene.cpp:28-29
					double cF = (c + 0.5) / W;
					C3 v = t.traceRay(viewingRay(scene, rF, cF), bdepth, false);
					double* o = out + i * 3;
					o[0] = v.r; o[1] = v.g; o[2] = v.b;
				}
			}
		} catch (const MathError& e) {
			std::lock_guard<std::mutex> g(mu);
			if (err.empty()) err = e.what();
			next.store(total);
		}
		std::lock_guard<std::mutex> g(mu);
		sum.trace += t.c.trace; sum.shadow += t.c.shadow; sum.refl += t.c.refl; sum.refr += t.c.refr;
		sum.sph += t.c.sph; sum.mesh += t.c.mesh; sum.bbox += t.c.bbox; sum.face += t.c.face;
	};
	std::vector<std::thread> pool;
	for (int i = 0; i < std::max(1, threads); i++) pool.emplace_back(worker);
	for (auto& th : pool) th.join();
	if (!err.empty()) {
		g_last_error = err;
		return 2;
	}
	if (intersection_only && row_begin == 0 && row_end == H && row_step == 1) {  // scene.cpp:50-58
		double mx = std::numeric_limits<double>::min();
		for (int64_t i = 0; i < total; i++)
			mx = std::max(mx, std::max(std::max(out[i * 3], out[i * 3 + 1]), out[i * 3 + 2]));
		const double rcp = 1.0 / mx;  // Color3d /= scalar multiplies by the reciprocal
		for (int64_t i = 0; i < total * 3; i++) out[i] *= rcp;
	}
	if (counters) {
		counters->trace_rays = sum.trace; counters->shadow_rays = sum.shadow;
		counters->reflect_rays = sum.refl; counters->refract_rays = sum.refr;
		counters->sphere_tests = sum.sph; counters->mesh_tests = sum.mesh;
		counters->bbox_pass = sum.bbox; counters->face_tests = sum.face;
	}
	return 0;
}

extern "C" const char* oracle_last_error(void) { return g_last_error.c_str(); }
extern "C" const char* oracle_last_warnings(void) { return g_warnings.c_str(); }

extern "C" void oracle_to_rgb8(const double* rgb, int64_t n, uint8_t* out) {  // writers.cpp:4-9
	for (int64_t i = 0; i < n * 3; i++) {
		double v = rgb[i];
		v = (1.0 < v) ? 1.0 : v;  // cwiseMin(1): std::min(v, 1)
		v = (v < 0.0) ? 0.0 : v;  // cwiseMax(0): std::max(v, 0)
		v = v * 255.0;
		out[i] = (v == v) ? (uint8_t)(int)v : 0;  // NaN -> 0 as cvttsd2si does on x86-64
	}
}
