// Byte-exact PNG writer for the drop-in CLI.
//
// PNGWriter::writeImage (writers.cpp:11-21) calls libpng 1.6.13's simplified
// png_image_write_to_file(PNG_FORMAT_RGB).  For 8-bit RGB that produces:
//   signature, IHDR(8-bit, colour type 2), sRGB(intent 0)          pngwrite.c:2169-2206
//   rows filtered by the unweighted minimum-sum-of-absolute-
//   differences heuristic over None/Sub/Up/Avg/Paeth, first strict
//   minimum wins                                                   pngwutil.c:2323-2700
//   one zlib stream (level -1, windowBits 15 or less for images of
//   <= 16 KiB, memLevel 8, Z_FILTERED), fed one filtered row at a
//   time, split into 8192-byte IDAT chunks                         pngwutil.c:295-420,1005-1135
//   CMF window optimisation of the first IDAT for small images     pngwutil.c:251-288
//   IEND
// The filter choice of row y depends only on the raw rows y and y - 1, so the rows are
// filtered in parallel (bands of rows handed out in order to host threads) while the calling
// thread feeds the filtered rows to deflate in order, exactly as libpng does (one row per
// deflate call, Z_NO_FLUSH): only deflate stays serial.
// zlib is the system zlib (1.2.11 in this image, as on the reference's build).
#include <sched.h>
#include <zlib.h>
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <memory>
#include <vector>
#include "../../include/rtamd.h"

namespace {

void put32(std::vector<uint8_t>& v, uint32_t x) {
	v.push_back(x >> 24);
	v.push_back(x >> 16);
	v.push_back(x >> 8);
	v.push_back(x);
}

void chunk(std::vector<uint8_t>& out, const char* type, const uint8_t* data, size_t n) {
	put32(out, static_cast<uint32_t>(n));
	const size_t start = out.size();
	out.insert(out.end(), type, type + 4);
	if (n) out.insert(out.end(), data, data + n);
	const uLong crc = crc32(0L, out.data() + start, static_cast<uInt>(n + 4));
	put32(out, static_cast<uint32_t>(crc));
}

inline uint32_t cost(uint8_t v) { return v < 128 ? v : 256u - v; }

inline uint8_t paeth(int a, int b, int c) {
	int p = b - c, pc = a - c;
	const int pa = p < 0 ? -p : p;
	const int pb = pc < 0 ? -pc : pc;
	pc = (p + pc) < 0 ? -(p + pc) : (p + pc);
	return static_cast<uint8_t>((pa <= pb && pa <= pc) ? a : (pb <= pc) ? b : c);
}

// png_write_find_filter (pngwutil.c:2323-2700): the filtered row (filter byte first) of the
// smallest sum of |signed bytes|, the first strict minimum winning.  One pass sums the five
// candidates' costs, a second writes the chosen one into out[0..n].
void filter_row(const uint8_t* row, const uint8_t* prev, size_t n, uint8_t* out) {
	constexpr size_t bpp = 3;
	uint32_t sum[5] = {0, 0, 0, 0, 0};
	for (size_t i = 0; i < n; i++) {
		const int a = i >= bpp ? row[i - bpp] : 0;
		const int b = prev[i];
		const int c = i >= bpp ? prev[i - bpp] : 0;
		const int x = row[i];
		sum[0] += cost(static_cast<uint8_t>(x));
		sum[1] += cost(static_cast<uint8_t>(x - a));
		sum[2] += cost(static_cast<uint8_t>(x - b));
		sum[3] += cost(static_cast<uint8_t>(x - ((a + b) >> 1)));
		sum[4] += cost(static_cast<uint8_t>(x - paeth(a, b, c)));
	}
	uint32_t mins = 0xffffffffu >> 1;  // PNG_MAXSUM
	int best = 0;
	for (int f = 0; f < 5; f++)
		if (sum[f] < mins) {
			mins = sum[f];
			best = f;
		}
	out[0] = static_cast<uint8_t>(best);
	for (size_t i = 0; i < n; i++) {
		const int a = i >= bpp ? row[i - bpp] : 0;
		const int b = prev[i];
		const int c = i >= bpp ? prev[i - bpp] : 0;
		const int x = row[i];
		const int p = best == 0 ? 0 : best == 1 ? a : best == 2 ? b : best == 3 ? ((a + b) >> 1) : paeth(a, b, c);
		out[i + 1] = static_cast<uint8_t>(x - p);
	}
}

// host threads for the row filters: the process's CPUs, at most 16 (the GPU box's share)
int filter_threads() {
	int n = 1;
	cpu_set_t set;
	if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
	return std::max(1, std::min(n, 16));
}

// optimize_cmf (pngwutil.c:251-288)
void optimize_cmf(uint8_t* data, size_t data_size) {
	if (data_size > 16384) return;
	unsigned z_cmf = data[0];
	if ((z_cmf & 0x0f) != 8 || (z_cmf & 0xf0) > 0x70) return;
	unsigned z_cinfo = z_cmf >> 4;
	unsigned half = 1u << (z_cinfo + 7);
	if (data_size > half) return;
	do {
		half >>= 1;
		--z_cinfo;
	} while (z_cinfo > 0 && data_size <= half);
	z_cmf = (z_cmf & 0x0f) | (z_cinfo << 4);
	data[0] = static_cast<uint8_t>(z_cmf);
	unsigned tmp = data[1] & 0xe0;
	tmp += 0x1f - ((z_cmf << 8) + tmp) % 0x1f;
	data[1] = static_cast<uint8_t>(tmp);
}

}  // namespace

extern "C" int rt_encode_png(const uint8_t* rgb, int width, int height, std::vector<uint8_t>* out_ptr);

int rt_encode_png(const uint8_t* rgb, int width, int height, std::vector<uint8_t>* out_ptr) {
	std::vector<uint8_t>& out = *out_ptr;
	static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
	out.assign(sig, sig + 8);
	uint8_t ihdr[13];
	const uint32_t w = static_cast<uint32_t>(width), h = static_cast<uint32_t>(height);
	const uint8_t hdr[13] = {uint8_t(w >> 24), uint8_t(w >> 16), uint8_t(w >> 8), uint8_t(w),
	                         uint8_t(h >> 24), uint8_t(h >> 16), uint8_t(h >> 8), uint8_t(h),
	                         8, 2, 0, 0, 0};
	std::memcpy(ihdr, hdr, 13);
	chunk(out, "IHDR", ihdr, 13);
	const uint8_t srgb = 0;
	chunk(out, "sRGB", &srgb, 1);

	const size_t rowbytes = static_cast<size_t>(width) * 3;
	// png_image_size: (rowbytes + 1) * height when both fit in 15 bits
	const size_t image_size = (rowbytes < 32768 && h < 32768) ? (rowbytes + 1) * h : 0xffffffffu;
	int window_bits = 15;
	if (image_size <= 16384) {
		unsigned half = 1u << (window_bits - 1);
		while (image_size + 262 <= half) {
			half >>= 1;
			--window_bits;
		}
	}
	z_stream zs;
	std::memset(&zs, 0, sizeof(zs));
	if (deflateInit2(&zs, Z_DEFAULT_COMPRESSION, Z_DEFLATED, window_bits, 8, Z_FILTERED) != Z_OK) return RT_ERR_IO;
	std::vector<uint8_t> zbuf(8192);  // PNG_ZBUF_SIZE
	zs.next_out = zbuf.data();
	zs.avail_out = static_cast<uInt>(zbuf.size());
	bool have_idat = false;
	auto emit = [&](size_t n) {
		if (!have_idat) optimize_cmf(zbuf.data(), image_size);
		chunk(out, "IDAT", zbuf.data(), n);
		have_idat = true;
		zs.next_out = zbuf.data();
		zs.avail_out = static_cast<uInt>(zbuf.size());
	};
	// filtered rows, (rowbytes + 1) each: bands of kBand rows taken in order by the threads;
	// ready[k] is set when band k is written, and the calling thread deflates band after band
	constexpr uint32_t kBand = 8;
	const uint32_t n_bands = (h + kBand - 1) / kBand;
	std::vector<uint8_t> filt((rowbytes + 1) * h);
	std::unique_ptr<std::atomic<uint8_t>[]> ready(new std::atomic<uint8_t>[n_bands]);
	for (uint32_t k = 0; k < n_bands; k++) ready[k].store(0, std::memory_order_relaxed);
	std::atomic<uint32_t> next_band{0};
	const std::vector<uint8_t> zero_row(rowbytes, 0);
	auto work = [&]() {
		for (uint32_t k; (k = next_band.fetch_add(1, std::memory_order_relaxed)) < n_bands;) {
			for (uint32_t y = k * kBand; y < std::min(h, (k + 1) * kBand); y++)
				filter_row(rgb + static_cast<size_t>(y) * rowbytes, y ? rgb + static_cast<size_t>(y - 1) * rowbytes : zero_row.data(),
				           rowbytes, filt.data() + static_cast<size_t>(y) * (rowbytes + 1));
			ready[k].store(1, std::memory_order_release);
		}
	};
	// small images: no threads (their start costs more than the filtering)
	const int n_threads = static_cast<size_t>(h) * rowbytes >= (1u << 18) ? std::min<int>(filter_threads(), n_bands) : 0;
	std::vector<std::thread> pool;
	for (int t = 0; t < n_threads; t++) pool.emplace_back(work);
	if (n_threads == 0) work();
	int rc = RT_OK;
	for (uint32_t y = 0; y <= h && rc == RT_OK; y++) {
		const bool finish = y == h;
		if (!finish) {
			if (y % kBand == 0)
				while (!ready[y / kBand].load(std::memory_order_acquire)) std::this_thread::yield();
			zs.next_in = filt.data() + static_cast<size_t>(y) * (rowbytes + 1);
			zs.avail_in = static_cast<uInt>(rowbytes + 1);
		} else {
			zs.next_in = nullptr;
			zs.avail_in = 0;
		}
		for (;;) {
			const int ret = deflate(&zs, finish ? Z_FINISH : Z_NO_FLUSH);
			if (zs.avail_out == 0) {
				emit(zbuf.size());
				if (ret == Z_OK && finish) continue;
			}
			if (ret == Z_OK && !finish && zs.avail_in == 0) break;
			if (ret == Z_OK && !finish) continue;
			if (ret == Z_STREAM_END && finish) {
				emit(zbuf.size() - zs.avail_out);
				break;
			}
			if (ret == Z_BUF_ERROR && !finish && zs.avail_in == 0) break;
			if (ret != Z_OK) {
				rc = RT_ERR_IO;
				break;
			}
		}
	}
	if (rc != RT_OK) next_band.store(n_bands);  // the threads stop at their current band
	for (std::thread& t : pool) t.join();
	if (rc != RT_OK) {
		deflateEnd(&zs);
		return rc;
	}
	deflateEnd(&zs);
	chunk(out, "IEND", nullptr, 0);
	return RT_OK;
}

extern "C" void rt_to_rgb8(const double* rgb, int64_t n_pixels, uint8_t* out) {  // writers.cpp:4-9
	for (int64_t i = 0; i < n_pixels * 3; i++) {
		double v = rgb[i];
		v = (1.0 < v) ? 1.0 : v;  // cwiseMin(1)
		v = (v < 0.0) ? 0.0 : v;  // cwiseMax(0)
		v = v * 255.0;
		out[i] = (v == v) ? static_cast<uint8_t>(static_cast<int>(v)) : 0;  // cast<uint8_t>, NaN -> 0
	}
}
