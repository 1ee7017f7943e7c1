// Sanitizer driver (ASan + UBSan, tests/test_sanitizers.py) for the host C++ of the render
// path: .rti/.obj ingest (scene_host.cpp), flattening + LBVH build (bvh.cpp) and the PNG
// encoder (png.cpp) - the code that runs on the host before and after the kernels.
//   host_check <scene.rti>...   parses and flattens every scene, encodes PNGs of several
//                               sizes; prints one line per scene
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>
#include "../../cs184-raytracer_amd/csrc/bvh.h"
#include "../../cs184-raytracer_amd/csrc/scene_host.h"

extern "C" int rt_encode_png(const uint8_t* rgb, int width, int height, std::vector<uint8_t>* out);

int main(int argc, char** argv) {
	int scenes = 0, errors = 0;
	for (int i = 1; i < argc; i++) {
		rtamd::Scene s;
		try {
			rtamd::parse_rti_file(s, argv[i]);
		} catch (const rtamd::ParseError& e) {
			std::printf("%s: parse error: %s\n", argv[i], e.msg.c_str());
			errors++;
			continue;
		} catch (const rtamd::MathError& e) {
			std::printf("%s: math error: %s\n", argv[i], e.msg.c_str());
			errors++;
			continue;
		}
		const rtamd::FlatScene fs = rtamd::flatten_scene(s);
		std::printf("%s: %zu geometries, %zu faces, %zu nodes, depth %d\n", argv[i], fs.geoms.size(), fs.face_geo.size(),
		            fs.nodes.size(), fs.max_bvh_depth);
		scenes++;
	}
	const int sizes[][2] = {{1, 1}, {7, 5}, {73, 74}, {640, 480}};
	for (const auto& wh : sizes) {
		const int w = wh[0], h = wh[1];
		std::vector<uint8_t> rgb(static_cast<size_t>(w) * h * 3);
		for (size_t k = 0; k < rgb.size(); k++) rgb[k] = static_cast<uint8_t>((k * 37) % 251);
		std::vector<uint8_t> png;
		if (rt_encode_png(rgb.data(), w, h, &png) != 0 || png.size() < 8 || png[1] != 'P') {
			std::printf("png %dx%d failed\n", w, h);
			return 1;
		}
	}
	std::printf("ok %d scenes, %d rejected\n", scenes, errors);
	return 0;
}
