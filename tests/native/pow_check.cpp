// Host check of csrc/glibc_pow.h against the live libm pow(), bit for bit.
// Built and run by tests/test_host.py:  pow_check <n_random>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include "glibc_pow.h"

static uint64_t b(double x) { uint64_t u; std::memcpy(&u, &x, 8); return u; }

int main(int argc, char** argv) {
	const long n = argc > 1 ? std::atol(argv[1]) : 1000000;
	std::mt19937_64 rng(12345);
	std::uniform_real_distribution<double> u01(0.0, 1.0);
	long bad = 0, total = 0;
	auto check = [&](double x, double y) {
		total++;
		const double want = std::pow(x, y), got = rtamd::glibc_pow(x, y);
		if (b(want) != b(got) && !(std::isnan(want) && std::isnan(got))) {
			if (bad < 10) std::printf("MISMATCH pow(%a, %a): libm %a ours %a\n", x, y, want, got);
			bad++;
		}
	};
	const double ys[] = {0.0, -0.0, 1.0, 2.0, 3.0, 4.0, 5.0, 6.0, 10.0, 16.0, 30.0, 36.0, 160.0, 1000.0, 0.5, -1.0, -2.0, 1e-20, 1e20, 0.3};
	for (double y : ys)
		for (long i = 0; i < n / 20; i++) check(u01(rng), y);
	for (long i = 0; i < n / 4; i++) check(u01(rng) * 1e3, -u01(rng) * 4);              // falloff pow(d, -f)
	for (long i = 0; i < n / 4; i++) check(std::exp(u01(rng) * 1400 - 700), (u01(rng) - 0.5) * 20);
	for (long i = 0; i < n / 4; i++) check(u01(rng), u01(rng) * 2000);                  // deep underflow path
	const double xs[] = {0.0, -0.0, 1.0, -1.0, 2.0, 0.5, INFINITY, -INFINITY, NAN, 5e-324, 1e-310, 1e300, -2.0, -0.5};
	const double ys2[] = {0.0, -0.0, 1.0, -1.0, 2.0, 3.0, 0.5, -0.5, INFINITY, -INFINITY, NAN, 1e-300, 1e300, 5e-324, 1075.0, -1075.0};
	for (double x : xs)
		for (double y : ys2) check(x, y);
	std::printf("checked %ld bad %ld\n", total, bad);
	return bad ? 1 : 0;
}
