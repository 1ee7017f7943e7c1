// Eigen 3.2.2 evaluation orders for the host-side transform stack (bit-exact).
//
//   translate  Geometry/Transform.h:838-843   t_k += ((L_k0 v0 + L_k1 v1) + L_k2 v2)
//   scale      Geometry/Transform.h:784-790   L_ij *= v_j
//   rotate     Geometry/Transform.h:882-886   L = L * R, entries ((L_i0 R_0j + L_i1 R_1j) + L_i2 R_2j)
//   AngleAxis  Geometry/AngleAxis.h:204-229   Rodrigues terms exactly as written there
//   inverse    Geometry/Transform.h:1124-1151 + LU/Inverse.h:117-159 (cofactors * (1/det))
//   det        LU/Determinant.h:26-31,71-83  (4x4 "30 muls" form on the full matrix)
//   T * v      Geometry/Transform.h:1244-1267 (rows sequential, w copied)
// Compiled without FMA contraction (-ffp-contract=off, x86-64 baseline).
#pragma once
#include <cmath>
#include "scene_host.h"

namespace rtamd {

inline Affine affine_identity() {
	Affine a;
	for (int i = 0; i < 3; i++)
		for (int j = 0; j < 4; j++) a.m[i][j] = (i == j) ? 1.0 : 0.0;
	return a;
}

inline void affine_translate(Affine& a, const double v[3]) {
	for (int k = 0; k < 3; k++) {
		double lv = (a.m[k][0] * v[0] + a.m[k][1] * v[1]) + a.m[k][2] * v[2];
		a.m[k][3] = a.m[k][3] + lv;
	}
}

inline void affine_scale(Affine& a, const double v[3]) {
	for (int i = 0; i < 3; i++)
		for (int j = 0; j < 3; j++) a.m[i][j] *= v[j];
}

inline void affine_rotate(Affine& a, const double R[3][3]) {
	double L[3][3];
	for (int i = 0; i < 3; i++)
		for (int j = 0; j < 3; j++) L[i][j] = a.m[i][j];
	for (int i = 0; i < 3; i++)
		for (int j = 0; j < 3; j++) a.m[i][j] = (L[i][0] * R[0][j] + L[i][1] * R[1][j]) + L[i][2] * R[2][j];
}

// AngleAxis(angle, axis).toRotationMatrix()
inline void angle_axis(double angle, const double ax[3], double R[3][3]) {
	const double s = std::sin(angle), c = std::cos(angle), omc = 1.0 - c;
	const double sx = s * ax[0], sy = s * ax[1], sz = s * ax[2];
	const double cx = omc * ax[0], cy = omc * ax[1], cz = omc * ax[2];
	double t = cx * ax[1];
	R[0][1] = t - sz;
	R[1][0] = t + sz;
	t = cx * ax[2];
	R[0][2] = t + sy;
	R[2][0] = t - sy;
	t = cy * ax[2];
	R[1][2] = t - sx;
	R[2][1] = t + sx;
	R[0][0] = cx * ax[0] + c;
	R[1][1] = cy * ax[1] + c;
	R[2][2] = cz * ax[2] + c;
}

inline Affine affine_inverse(const Affine& a) {
	auto m = [&](int i, int j) { return a.m[i][j]; };
	// cofactor_3x3<i,j> (LU/Inverse.h:117-128)
	auto cof = [&](int i, int j) {
		const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
		return m(i1, j1) * m(i2, j2) - m(i1, j2) * m(i2, j1);
	};
	const double c0[3] = {cof(0, 0), cof(1, 0), cof(2, 0)};
	const double det = c0[0] * m(0, 0) + (c0[1] * m(1, 0) + c0[2] * m(2, 0));  // Vector3 sum a0+(a1+a2)
	const double invdet = 1.0 / det;
	Affine r;
	for (int rr = 0; rr < 3; rr++)
		for (int cc = 0; cc < 3; cc++) r.m[rr][cc] = (rr == 0 ? c0[cc] : cof(cc, rr)) * invdet;
	// translation: (-Linv) * t, inner sums sequential
	for (int k = 0; k < 3; k++)
		r.m[k][3] = ((-r.m[k][0]) * a.m[0][3] + (-r.m[k][1]) * a.m[1][3]) + (-r.m[k][2]) * a.m[2][3];
	return r;
}

inline double affine_det4(const Affine& a) {
	double M[4][4];
	for (int i = 0; i < 3; i++)
		for (int j = 0; j < 4; j++) M[i][j] = a.m[i][j];
	M[3][0] = M[3][1] = M[3][2] = 0.0;
	M[3][3] = 1.0;
	auto h = [&](int j, int k, int p, int n) {
		return (M[j][0] * M[k][1] - M[k][0] * M[j][1]) * (M[p][2] * M[n][3] - M[n][2] * M[p][3]);
	};
	return ((((h(0, 1, 2, 3) - h(0, 2, 1, 3)) + h(0, 3, 1, 2)) + h(1, 2, 0, 3)) - h(1, 3, 0, 2)) + h(2, 3, 0, 1);
}

inline void affine_apply(const Affine& a, const double v[4], double out[4]) {
	double r[3];
	for (int k = 0; k < 3; k++) r[k] = ((a.m[k][0] * v[0] + a.m[k][1] * v[1]) + a.m[k][2] * v[2]) + a.m[k][3] * v[3];
	out[0] = r[0];
	out[1] = r[1];
	out[2] = r[2];
	out[3] = v[3];
}

// Vector4d reductions with SSE2 packets: (a0 b0 + a2 b2) + (a1 b1 + a3 b3)
inline double dot4(const double a[4], const double b[4]) { return (a[0] * b[0] + a[2] * b[2]) + (a[1] * b[1] + a[3] * b[3]); }
// Vector3d reductions: a0 b0 + (a1 b1 + a2 b2)
inline double norm3(const double a[3]) { return std::sqrt(a[0] * a[0] + (a[1] * a[1] + a[2] * a[2])); }
// isZero(): |a_i| <= 1e-12 (NumTraits<double>::dummy_precision)
inline bool is_zero(const double* a, int n) {
	for (int i = 0; i < n; i++)
		if (!(std::fabs(a[i]) <= 1e-12)) return false;
	return true;
}

}  // namespace rtamd
