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
// zlib is the system zlib (1.2.11 in this image, as on the reference's build).
#include <zlib.h>
#include <cstdio>
#include <cstring>
#include <string>
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

// png_write_find_filter: the filtered row (filter byte first) with the smallest cost
void filter_row(const uint8_t* row, const uint8_t* prev, size_t n, std::vector<uint8_t> cand[5], int& best) {
	const int bpp = 3;
	for (int f = 0; f < 5; f++) {
		cand[f].resize(n + 1);
		cand[f][0] = static_cast<uint8_t>(f);
	}
	for (size_t i = 0; i < n; i++) {
		const int a = i >= static_cast<size_t>(bpp) ? row[i - bpp] : 0;
		const int b = prev[i];
		const int c = i >= static_cast<size_t>(bpp) ? prev[i - bpp] : 0;
		const int x = row[i];
		cand[0][i + 1] = static_cast<uint8_t>(x);
		cand[1][i + 1] = static_cast<uint8_t>(x - a);
		cand[2][i + 1] = static_cast<uint8_t>(x - b);
		cand[3][i + 1] = static_cast<uint8_t>(x - ((a + b) >> 1));
		cand[4][i + 1] = static_cast<uint8_t>(x - paeth(a, b, c));
	}
	uint32_t mins = 0xffffffffu >> 1;  // PNG_MAXSUM
	best = 0;
	for (int f = 0; f < 5; f++) {
		uint32_t sum = 0;
		for (size_t i = 1; i <= n; i++) sum += cost(cand[f][i]);
		if (sum < mins) {
			mins = sum;
			best = f;
		}
	}
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
	std::vector<uint8_t> prev(rowbytes, 0), cand[5];
	for (uint32_t y = 0; y <= h; y++) {
		const bool finish = y == h;
		int best = 0;
		if (!finish) {
			const uint8_t* row = rgb + static_cast<size_t>(y) * rowbytes;
			filter_row(row, prev.data(), rowbytes, cand, best);
			std::memcpy(prev.data(), row, rowbytes);
			zs.next_in = cand[best].data();
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
				deflateEnd(&zs);
				return RT_ERR_IO;
			}
		}
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
