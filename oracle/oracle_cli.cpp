// TEST INFRASTRUCTURE ONLY — command-line front end of the CPU oracle.
// Same flags as the reference (options.cpp:7-16): -w -h -t -o --bdepth --intersection-only,
// positional .rti files.  Writes H*W*3 little-endian doubles to -o; prints counters.
#include <getopt.h>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include "oracle.h"

int main(int argc, char** argv) {
	int W = 500, H = 500, T = 1, bdepth = 10, io = 0;
	std::string out;
	static const struct option opts[] = {{"output", 1, 0, 'o'}, {"threads", 1, 0, 't'}, {"width", 1, 0, 'w'},
	                                     {"height", 1, 0, 'h'}, {"bdepth", 1, 0, 1},   {"intersection-only", 0, 0, 2},
	                                     {0, 0, 0, 0}};
	int c;
	while ((c = getopt_long(argc, argv, "t:w:h:o:", opts, nullptr)) != -1) {
		switch (c) {
			case 'o': out = optarg; break;
			case 't': T = std::atoi(optarg); break;
			case 'w': W = std::atoi(optarg); break;
			case 'h': H = std::atoi(optarg); break;
			case 1: bdepth = std::atoi(optarg); break;
			case 2: io = 1; break;
			default: return 1;
		}
	}
	std::vector<const char*> files;
	for (int i = optind; i < argc; i++) files.push_back(argv[i]);
	std::vector<double> img((size_t)W * H * 3);
	oracle_counters cnt;
	int rc = oracle_render(files.data(), (int)files.size(), W, H, bdepth, io, T, 0, H, 1, img.data(), &cnt);
	std::fputs(oracle_last_warnings(), stderr);
	if (rc) {
		std::fprintf(stderr, "Error: %s\n", oracle_last_error());
		return rc;
	}
	std::printf("COUNTERS trace=%lld shadow=%lld refl=%lld refr=%lld sphere=%lld mesh=%lld bbox=%lld face=%lld\n",
	            (long long)cnt.trace_rays, (long long)cnt.shadow_rays, (long long)cnt.reflect_rays,
	            (long long)cnt.refract_rays, (long long)cnt.sphere_tests, (long long)cnt.mesh_tests,
	            (long long)cnt.bbox_pass, (long long)cnt.face_tests);
	if (!out.empty()) {
		FILE* f = std::fopen(out.c_str(), "wb");
		if (!f) return 1;
		std::fwrite(img.data(), sizeof(double), img.size(), f);
		std::fclose(f);
	}
	return 0;
}
