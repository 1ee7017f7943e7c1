// pow() with glibc's exact results, for host and device.
//
// The reference's specular term pow(max(-V.R, 0), ns) (scene.cpp:103) and light falloff
// pow(dist, -falloff) (lights.h:24) are evaluated by glibc 2.35's pow: the ARM
// optimized-routines algorithm (log_inline in double-double, exp_inline with a 2^(k/128)
// table), x86-64 ifunc variant __pow_fma (-mfma -mavx2, GCC contraction).  This is a
// restatement of that variant's dataflow — every fma() below is a vfmadd in __pow_fma,
// every other operation a separately rounded one — over the same tables
// (pow_tables.h, extracted by tools/gen_pow_tables.py).  ROCm's ocml pow is not
// bit-identical (differs in ~18% of results even for y = 1), so the kernels use this.
#pragma once
#include <cstdint>
#include "pow_tables.h"

#if defined(__HIPCC__) || defined(__HIP__)
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD inline __attribute__((always_inline))
#endif

namespace rtamd {
namespace glibc_pow_detail {

RT_HD uint64_t bits(double x) { return __builtin_bit_cast(uint64_t, x); }
RT_HD double dbl(uint64_t u) { return __builtin_bit_cast(double, u); }
RT_HD double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }
RT_HD uint32_t top12(double x) { return static_cast<uint32_t>(bits(x) >> 52); }

constexpr uint64_t kOff = 0x3fe6955500000000ULL;
constexpr uint32_t kSignBias = 0x800 << 7;

// The polynomial and reduction constants.  On the device they are read from constant memory
// through a pointer the compiler cannot see through (scalar loads where pow runs): as
// literals, a kernel that calls pow inside its grid-stride loop (the fused Phong terms of
// k_shadow) materialises all of them in vector registers before the loop and spills them.
struct PowConsts {
	double ln2hi, ln2lo, logpoly[7];
	double invln2n, shift, negln2hin, negln2lon, exppoly[4];
};
#if defined(__HIP_DEVICE_COMPILE__)
__constant__ PowConsts kPowConstsDev = {
    glibc_pow_data::kLn2hi, glibc_pow_data::kLn2lo,
    {glibc_pow_data::kLogPoly[0], glibc_pow_data::kLogPoly[1], glibc_pow_data::kLogPoly[2], glibc_pow_data::kLogPoly[3],
     glibc_pow_data::kLogPoly[4], glibc_pow_data::kLogPoly[5], glibc_pow_data::kLogPoly[6]},
    glibc_pow_data::kInvLn2N, glibc_pow_data::kShift, glibc_pow_data::kNegLn2hiN, glibc_pow_data::kNegLn2loN,
    {glibc_pow_data::kExpPoly[0], glibc_pow_data::kExpPoly[1], glibc_pow_data::kExpPoly[2], glibc_pow_data::kExpPoly[3]}};
__device__ __forceinline__ const __attribute__((address_space(4))) PowConsts& pow_consts() {
	const PowConsts* p = &kPowConstsDev;
	asm volatile("" : "+s"(p));
	return *(const __attribute__((address_space(4))) PowConsts*)(p);
}
#define RT_POW_CONSTS const auto& C = pow_consts()
#else
constexpr PowConsts kPowConstsHost = {
    glibc_pow_data::kLn2hi, glibc_pow_data::kLn2lo,
    {glibc_pow_data::kLogPoly[0], glibc_pow_data::kLogPoly[1], glibc_pow_data::kLogPoly[2], glibc_pow_data::kLogPoly[3],
     glibc_pow_data::kLogPoly[4], glibc_pow_data::kLogPoly[5], glibc_pow_data::kLogPoly[6]},
    glibc_pow_data::kInvLn2N, glibc_pow_data::kShift, glibc_pow_data::kNegLn2hiN, glibc_pow_data::kNegLn2loN,
    {glibc_pow_data::kExpPoly[0], glibc_pow_data::kExpPoly[1], glibc_pow_data::kExpPoly[2], glibc_pow_data::kExpPoly[3]}};
#define RT_POW_CONSTS const PowConsts& C = kPowConstsHost
#endif

// log(x) = hi + lo for the (normalised) bit pattern ix; kLogTab may live in LDS
RT_HD double log_inline(uint64_t ix, double* tail, const double* kLogTab) {
	RT_POW_CONSTS;
	const double kLn2hi = C.ln2hi, kLn2lo = C.ln2lo;
	const auto& kLogPoly = C.logpoly;
	const uint64_t tmp = ix - kOff;
	const int i = static_cast<int>((tmp >> 45) % 128);
	const int k = static_cast<int>(static_cast<int64_t>(tmp) >> 52);
	const uint64_t iz = ix - (tmp & 0xfffULL << 52);
	const double z = dbl(iz);
	const double kd = static_cast<double>(k);
	const double invc = kLogTab[4 * i], logc = kLogTab[4 * i + 2], logctail = kLogTab[4 * i + 3];
	const double r = fma_(z, invc, -1.0);
	const double t1 = fma_(kd, kLn2hi, logc);
	const double t2 = t1 + r;
	const double lo1 = fma_(kd, kLn2lo, logctail);
	const double lo2 = (t1 - t2) + r;
	const double ar = kLogPoly[0] * r;
	const double ar2 = r * ar;
	const double ar3 = r * ar2;
	const double hi = t2 + ar2;
	const double lo3 = fma_(ar, r, -ar2);
	const double lo4 = (t2 - hi) + ar2;
	const double q12 = fma_(r, kLogPoly[2], kLogPoly[1]);
	const double q34 = fma_(r, kLogPoly[4], kLogPoly[3]);
	const double q56 = fma_(r, kLogPoly[6], kLogPoly[5]);
	const double q = fma_(ar2, fma_(q56, ar2, q34), q12);
	const double lo = fma_(ar3, q, ((lo1 + lo2) + lo3) + lo4);
	const double y = hi + lo;
	*tail = (hi - y) + lo;
	return y;
}

RT_HD double math_oflow(uint32_t sign) { return sign ? -__builtin_inf() : __builtin_inf(); }
RT_HD double math_uflow(uint32_t sign) { return sign ? -0.0 : 0.0; }

// exp_inline's scale*(1+tmp) when 2^k over/underflows (optimized-routines specialcase)
RT_HD double specialcase(double tmp, uint64_t sbits, uint64_t ki) {
	if ((ki & 0x80000000) == 0) {
		sbits -= 1009ULL << 52;
		const double scale = dbl(sbits);
		return 0x1p1009 * fma_(scale, tmp, scale);
	}
	sbits += 1022ULL << 52;
	const double scale = dbl(sbits);
	const double st = tmp * scale;
	double y = scale + st;
	if (__builtin_fabs(y) < 1.0) {
		const double one = (y < 0.0) ? -1.0 : 1.0;
		double lo = (scale - y) + st;
		const double hi = y + one;
		lo = ((one - hi) + y) + lo;
		y = (lo + hi) - one;
		if (y == 0) y = dbl(sbits & 0x8000000000000000ULL);
	}
	return y * 0x1p-1022;
}

RT_HD double exp_inline(double x, double xtail, uint32_t sign_bias, const uint64_t* kExpTab) {
	RT_POW_CONSTS;
	const double kInvLn2N = C.invln2n, kShift = C.shift, kNegLn2hiN = C.negln2hin, kNegLn2loN = C.negln2lon;
	const auto& kExpPoly = C.exppoly;
	uint32_t abstop = top12(x) & 0x7ff;
	if (abstop - 0x3c9 >= 0x408 - 0x3c9) {  // |x| < 2^-54 or |x| >= 512
		if (static_cast<int32_t>(abstop - 0x3c9) < 0) {
			const double one = 1.0 + x;
			return sign_bias ? -one : one;
		}
		if (abstop >= 0x409) return (bits(x) >> 63) ? math_uflow(sign_bias) : math_oflow(sign_bias);
		abstop = 0;
	}
	double kd = fma_(x, kInvLn2N, kShift);
	const uint64_t ki = bits(kd);
	kd -= kShift;
	double r = fma_(kd, kNegLn2hiN, x);
	r = fma_(kd, kNegLn2loN, r);
	r = xtail + r;
	const uint64_t idx = 2 * (ki % 128);
	const uint64_t top = (ki + sign_bias) << 45;
	const double tail = dbl(kExpTab[idx]);
	const uint64_t sbits = kExpTab[idx + 1] + top;
	const double p23 = fma_(r, kExpPoly[1], kExpPoly[0]);
	const double tr = r + tail;
	const double r2 = r * r;
	const double p45 = fma_(r, kExpPoly[3], kExpPoly[2]);
	double tmp = fma_(p23, r2, tr);
	tmp = fma_(p45, r2 * r2, tmp);
	if (abstop == 0) return specialcase(tmp, sbits, ki);
	const double scale = dbl(sbits);
	return fma_(tmp, scale, scale);
}

// 0: not an integer, 1: odd integer, 2: even integer (iy finite, non-zero)
RT_HD int checkint(uint64_t iy) {
	const int e = static_cast<int>(iy >> 52 & 0x7ff);
	if (e < 0x3ff) return 0;
	if (e > 0x3ff + 52) return 2;
	if (iy & ((1ULL << (0x3ff + 52 - e)) - 1)) return 0;
	if (iy & (1ULL << (0x3ff + 52 - e))) return 1;
	return 2;
}

RT_HD bool zeroinfnan(uint64_t i) { return 2 * i - 1 >= 2 * 0x7ff0000000000000ULL - 1; }
RT_HD bool issignaling(double x) {
	return 2 * (bits(x) ^ 0x0008000000000000ULL) > 2 * 0x7ff8000000000000ULL;
}

}  // namespace glibc_pow_detail

// logtab/exptab: glibc_pow_data::kLogTab / kExpTab or copies of them (e.g. in LDS)
RT_HD double glibc_pow(double x, double y, const double* logtab = glibc_pow_data::kLogTab,
                       const uint64_t* exptab = glibc_pow_data::kExpTab) {
	using namespace glibc_pow_detail;
	uint32_t sign_bias = 0;
	uint64_t ix = bits(x), iy = bits(y);
	uint32_t topx = top12(x), topy = top12(y);
	if (topx - 0x001 >= 0x7ff - 0x001 || (topy & 0x7ff) - 0x3be >= 0x43e - 0x3be) {
		if (zeroinfnan(iy)) {
			if (2 * iy == 0) return issignaling(x) ? x + y : 1.0;
			if (ix == bits(1.0)) return issignaling(y) ? x + y : 1.0;
			if (2 * ix > 2 * bits(__builtin_inf()) || 2 * iy > 2 * bits(__builtin_inf())) return x + y;
			if (2 * ix == 2 * bits(1.0)) return 1.0;
			if ((2 * ix < 2 * bits(1.0)) == !(iy >> 63)) return 0.0;
			return y * y;
		}
		if (zeroinfnan(ix)) {
			double x2 = x * x;
			if ((ix >> 63) && checkint(iy) == 1) {
				x2 = -x2;
				sign_bias = 1;
			}
			if (2 * ix == 0 && (iy >> 63)) return (sign_bias ? -1.0 : 1.0) / 0.0;
			return (iy >> 63) ? 1 / x2 : x2;
		}
		if (ix >> 63) {
			const int yint = checkint(iy);
			if (yint == 0) return dbl(0xfff8000000000000ULL);  // __math_invalid: x86 default NaN
			if (yint == 1) sign_bias = kSignBias;
			ix &= 0x7fffffffffffffffULL;
			topx &= 0x7ff;
		}
		if ((topy & 0x7ff) - 0x3be >= 0x43e - 0x3be) {
			if (ix == bits(1.0)) return 1.0;
			if ((topy & 0x7ff) < 0x3be) return ix > bits(1.0) ? 1.0 + y : 1.0 - y;
			return (ix > bits(1.0)) == (topy < 0x800) ? math_oflow(0) : math_uflow(0);
		}
		if (topx == 0) {
			ix = bits(x * 0x1p52);
			ix &= 0x7fffffffffffffffULL;
			ix -= 52ULL << 52;
		}
	}
	double lo;
	const double hi = log_inline(ix, &lo, logtab);
	const double ehi = y * hi;
	const double elo = fma_(y, lo, fma_(hi, y, -ehi));
	return exp_inline(ehi, elo, sign_bias, exptab);
}

}  // namespace rtamd
