// TEST INFRASTRUCTURE ONLY — never linked into the product.
//
// Harness around the UNMODIFIED reference render path
// (/root/reference/src/{scene,geometry,parsers,exceptions,options}.cpp), built by
// oracle/Makefile into oracle/_ref/refharness.  It replaces only the reference's
// main.cpp (+ writers.cpp / libpng, which need generated headers and are therefore
// not built here) and dumps the raw f64 RasterImage instead of a PNG.
//
// Pixel loop: the reference's Scene::renderScene (scene.cpp:10-59) aborts when W*H is
// not a multiple of its 2000-pixel block (unclamped block overrun, scene.cpp:13,21-25,
// Eigen bounds assert).  Every pixel is a pure function of (r,c): the harness therefore
// evaluates exactly the per-pixel body of scene.cpp:26-31 through the reference's own
// public Camera::calculateViewingRay (rtbase.h:74-84) and Scene::traceRay
// (scene.cpp:61-140).  With RT_REF_MODE=renderScene (and W*H % 2000 == 0) it calls the
// reference's renderScene itself, which lets tests prove the two loops agree bit for bit.
//
// Parallelism: the reference's lazily cached transforms race under threads
// (rtbase.h:86-95, lights.h:28-33,56-61).  The harness forks single-threaded worker
// processes instead (each owns its caches), writing into a shared mapping.
//
// Output: <out> = H*W*3 little-endian doubles, row-major (RasterImage layout, scene.h:11).
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <limits>
#include <string>
#include "options.h"
#include "scene.h"
#include "parsers.h"

int main(int argc, char* argv[]) {
	if (!programOptions.parseCommandLine(argc, argv))
		return 1;
	Scene scene;
	for (const std::string& fn : programOptions.inputFilenames_) {
		RTIParser parser(scene);
		try {
			parser.parseFile(fn);
		} catch (const ParseException& e) {
			std::fprintf(stderr, "Error: %s\n", e.what());
			return 1;
		}
	}
	if (!scene.hasCamera()) {
		std::fprintf(stderr, "Error: At least one camera must be specified.\n");
		return 1;
	}
	const int rows = programOptions.renderHeight_;
	const int cols = programOptions.renderWidth_;
	const long total = (long)rows * cols;
	const size_t bytes = (size_t)total * 3 * sizeof(double);
	double* shared = (double*)mmap(nullptr, bytes, PROT_READ | PROT_WRITE,
			MAP_SHARED | MAP_ANONYMOUS, -1, 0);
	if (shared == MAP_FAILED) { std::perror("mmap"); return 1; }

	const char* mode = std::getenv("RT_REF_MODE");
	if (mode && std::string(mode) == "renderScene") {
		// the reference's own loop (requires W*H % 2000 == 0, see header)
		Scene::RasterImage image(rows, cols);
		scene.renderScene(image, nullptr);
		for (long i = 0; i < total; i++)
			for (int k = 0; k < 3; k++)
				shared[i * 3 + k] = image(i)(k);
	} else {
		const int workers = std::max(1, programOptions.renderThreadsCount_);
		const long block = 2000;  // scene.cpp:13
		// RT_REF_ROWS=begin:end:step renders only those rows (bench.py's bounded CPU
		// sample); the selected pixels are dealt in 2000-pixel blocks as above.
		long rb = 0, re = rows, rs = 1;
		if (const char* sel = std::getenv("RT_REF_ROWS")) {
			if (std::sscanf(sel, "%ld:%ld:%ld", &rb, &re, &rs) != 3 || rb < 0 || re > rows || rs <= 0) {
				std::fprintf(stderr, "refharness: bad RT_REF_ROWS\n");
				return 1;
			}
		}
		const long selected = (re > rb) ? ((re - rb + rs - 1) / rs) * cols : 0;
		for (int w = 0; w < workers; w++) {
			pid_t pid = fork();
			if (pid < 0) { std::perror("fork"); return 1; }
			if (pid == 0) {
				Camera cam = scene.camera();
				for (long start = (long)w * block; start < selected; start += (long)workers * block) {
					long end = std::min(start + block, selected);
					for (long k = start; k < end; k++) {
						int r = (int)(rb + (k / cols) * rs);
						int c = (int)(k % cols);
						long i = (long)r * cols + c;
						double rowFrac = (r + 0.5) / rows;  // scene.cpp:28
						double colFrac = (c + 0.5) / cols;  // scene.cpp:29
						Ray viewingRay = cam.calculateViewingRay(rowFrac, colFrac);
						Color3d v = scene.traceRay(viewingRay, programOptions.bounceDepth_);
						shared[i * 3 + 0] = v(0);
						shared[i * 3 + 1] = v(1);
						shared[i * 3 + 2] = v(2);
					}
				}
				_exit(0);
			}
		}
		int failed = 0;
		for (int w = 0; w < workers; w++) {
			int st = 0;
			wait(&st);
			if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) failed = st ? st : 1;
		}
		if (failed) {
			std::fprintf(stderr, "refharness: worker failed (status %d)\n", failed);
			return 2;
		}
		if (programOptions.intersectionOnly_) {
			// scene.cpp:50-58 (the renderScene branch normalises itself)
			double maxBrightness = std::numeric_limits<double>::min();
			for (long i = 0; i < total; i++) {
				Color3d v(shared[i * 3], shared[i * 3 + 1], shared[i * 3 + 2]);
				maxBrightness = std::max(maxBrightness, v.maxCoeff());
			}
			for (long i = 0; i < total; i++) {
				Color3d v(shared[i * 3], shared[i * 3 + 1], shared[i * 3 + 2]);
				v /= maxBrightness;  // the reference's own Eigen operator/= (scene.cpp:56)
				for (int k = 0; k < 3; k++) shared[i * 3 + k] = v(k);
			}
		}
	}
	FILE* f = std::fopen(programOptions.outputFilename_.c_str(), "wb");
	if (!f) { std::perror("fopen"); return 1; }
	if (std::fwrite(shared, 1, bytes, f) != bytes) { std::perror("fwrite"); return 1; }
	std::fclose(f);
	return 0;
}
