// rtamd — drop-in replacement for the reference's `as2` executable (main.cpp:40-85,
// options.cpp:7-90): same flags (-o/--output, -t/--threads, -w/--width, -h/--height,
// --bdepth, --intersection-only, positional .rti files), same messages and exit codes,
// byte-identical PNG.  Adds --device N (HIP device), --dump-raw FILE (f64 image) and
// --gpus N (devices --device .. --device+N-1 of this node, rows in --row-block blocks
// interleaved over them, gathered over RCCL: include/rtamd_multi.h) and --devices LIST
// (an explicit comma-separated device list for that path; a repeated device makes
// partitions sharing one GPU).  --timing FILE writes the host time of every phase of the run
// as JSON (HIP runtime start, parse, LBVH build, HBM upload, render, device-to-host copy,
// PNG): the drop-in's wall-clock split (tools/cli_bench.py).
// The render itself runs on the GPU through the C-ABI (include/rtamd.h).
#include <getopt.h>
#include <signal.h>
#include <sys/time.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <fstream>
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>
#include "../../include/rtamd.h"
#include "../../include/rtamd_multi.h"

namespace {

struct Options {  // options.h:10-16 defaults
	std::vector<std::string> inputs;
	std::string output, dump_raw, timing;
	int threads = 1, width = 500, height = 500, bdepth = 10, device = 0;
	int gpus = 0, row_block = 8;  // gpus 0: the single-device path
	std::vector<int> devices;     // --devices: explicit list for the multi-device path
	bool intersection_only = false;
};

enum { OPT_HELP = 0, OPT_BDEPTH = 256, OPT_IO, OPT_DEVICE, OPT_DUMP, OPT_GPUS, OPT_ROW_BLOCK, OPT_DEVICES, OPT_TIMING };

bool parse_int(const char* s, int& out) {
	try {
		out = std::stoi(s);
		return true;
	} catch (const std::logic_error&) {
		return false;
	}
}

bool parse_command_line(int argc, char** argv, Options& o) {  // options.cpp:18-86
	static const struct option opts[] = {{"help", 0, nullptr, OPT_HELP},     {"output", 1, nullptr, 'o'},
	                                     {"threads", 1, nullptr, 't'},       {"width", 1, nullptr, 'w'},
	                                     {"height", 1, nullptr, 'h'},        {"bdepth", 1, nullptr, OPT_BDEPTH},
	                                     {"intersection-only", 0, nullptr, OPT_IO},
	                                     {"device", 1, nullptr, OPT_DEVICE}, {"dump-raw", 1, nullptr, OPT_DUMP},
	                                     {"gpus", 1, nullptr, OPT_GPUS},     {"row-block", 1, nullptr, OPT_ROW_BLOCK},
	                                     {"devices", 1, nullptr, OPT_DEVICES}, {"timing", 1, nullptr, OPT_TIMING},
	                                     {nullptr, 0, nullptr, 0}};
	int c;
	while ((c = getopt_long(argc, argv, "t:w:h:o:", opts, nullptr)) != -1) {
		switch (c) {
			case 'o': o.output = optarg; break;
			case OPT_IO: o.intersection_only = true; break;
			case OPT_DUMP: o.dump_raw = optarg; break;
			case OPT_TIMING: o.timing = optarg; break;
			case 't':
				if (!parse_int(optarg, o.threads)) {
					std::cerr << "Error: Thread count is invalid." << std::endl;
					return false;
				}
				if (o.threads <= 0) {
					std::cerr << "Error: Thread count must be positive." << std::endl;
					return false;
				}
				break;
			case 'w':
			case 'h': {
				int& dest = c == 'w' ? o.width : o.height;
				if (!parse_int(optarg, dest)) {
					std::cerr << "Error: Width and/or height is invalid." << std::endl;
					return false;
				}
				if (dest <= 0) {
					std::cerr << "Error: Width and/or height must be positive." << std::endl;
					return false;
				}
				break;
			}
			case OPT_BDEPTH:
				if (!parse_int(optarg, o.bdepth)) {
					std::cerr << "Error: Bounce depth is invalid." << std::endl;
					return false;
				}
				if (o.bdepth < 0) {
					std::cerr << "Error: Bounce depth must be non-negative." << std::endl;
					return false;
				}
				break;
			case OPT_DEVICE:
				if (!parse_int(optarg, o.device) || o.device < 0) {
					std::cerr << "Error: Device index is invalid." << std::endl;
					return false;
				}
				break;
			case OPT_GPUS:
				if (!parse_int(optarg, o.gpus) || o.gpus < 1) {
					std::cerr << "Error: GPU count is invalid." << std::endl;
					return false;
				}
				break;
			case OPT_DEVICES: {
				o.devices.clear();
				std::string list = optarg;
				size_t pos = 0;
				while (pos <= list.size()) {
					const size_t e = std::min(list.find(',', pos), list.size());
					int d = -1;
					if (!parse_int(list.substr(pos, e - pos).c_str(), d) || d < 0) {
						std::cerr << "Error: Device list is invalid." << std::endl;
						return false;
					}
					o.devices.push_back(d);
					pos = e + 1;
				}
				o.gpus = static_cast<int>(o.devices.size());
				break;
			}
			case OPT_ROW_BLOCK:
				if (!parse_int(optarg, o.row_block) || o.row_block < 1) {
					std::cerr << "Error: Row block is invalid." << std::endl;
					return false;
				}
				break;
			default:
				std::cerr << "Usage: " << argv[0] << " [options] -o <output file> <input files>..." << std::endl;
				return false;
		}
	}
	while (optind < argc) o.inputs.push_back(argv[optind++]);
	if (o.inputs.empty()) {
		std::cerr << "Error: At least one input file must be specified." << std::endl;
		return false;
	}
	if (o.output.empty()) {
		std::cerr << "Error: An output file must be specified." << std::endl;
		return false;
	}
	return true;
}

volatile sig_atomic_t g_progress_signaled = 0;
void on_alarm(int) { g_progress_signaled = 1; }
void set_alarm(bool enable) {  // main.cpp:28-38: 4 Hz progress tick
	if (enable) signal(SIGALRM, on_alarm);
	struct itimerval itv = {{0, 0}, {0, 0}};
	itv.it_value.tv_usec = itv.it_interval.tv_usec = enable ? 1000000 / 4 : 0;
	setitimer(ITIMER_REAL, &itv, nullptr);
	if (!enable) signal(SIGALRM, SIG_DFL);
}
void update_progress(int complete, int total, void*) {  // main.cpp:12-22
	if (complete != total && !g_progress_signaled) return;
	std::putchar('\r');
	std::printf("Rendering scene (%d/%d) (%.1f%%) ...", complete, total, 100.0 * complete / total);
	std::fflush(stdout);
	if (complete == total) std::putchar('\n');
	g_progress_signaled = 0;
}

double now_ms() {
	using clk = std::chrono::steady_clock;
	return std::chrono::duration<double, std::milli>(clk::now().time_since_epoch()).count();
}

// host milliseconds of the run's phases (--timing): the top-level phases are consecutive
// and add up to main_ms; `detail` holds parts of them (scene_create = scene_build +
// scene_upload + the rest, render = render_gpu + d2h + the rest), not to be added again
struct Timing {
	double start = now_ms(), last = start;
	std::vector<std::pair<std::string, double>> phases, detail;
	void mark(const char* name) {
		const double t = now_ms();
		phases.emplace_back(name, t - last);
		last = t;
	}
	void write(const std::string& path) const {
		FILE* f = std::fopen(path.c_str(), "w");
		if (!f) return;
		std::fprintf(f, "{");
		for (const auto& p : phases) std::fprintf(f, "\"%s_ms\": %.3f, ", p.first.c_str(), p.second);
		std::fprintf(f, "\"main_ms\": %.3f, \"detail\": {", last - start);
		for (size_t k = 0; k < detail.size(); k++)
			std::fprintf(f, "%s\"%s_ms\": %.3f", k ? ", " : "", detail[k].first.c_str(), detail[k].second);
		std::fprintf(f, "}}\n");
		std::fclose(f);
	}
};

}  // namespace

int main(int argc, char** argv) {
	Timing tm;
	Options o;
	if (!parse_command_line(argc, argv, o)) return 1;
	if (!std::ofstream(o.output)) {  // main.cpp:45-51
		std::cerr << "Error: Output file is not writable." << std::endl;
		return 1;
	}
	std::remove(o.output.c_str());
	if (!o.timing.empty()) {
		(void)rt_device_count();  // starts the HIP runtime (otherwise inside rt_scene_create)
		tm.mark("hip_init");
	}
	rt_builder* b = rt_builder_create();
	for (const std::string& f : o.inputs) {
		const int rc = rt_builder_parse_rti(b, f.c_str());
		std::cerr << rt_builder_warnings(b);
		if (rc == RT_ERR_PARSE) {
			std::cerr << "Error: " << rt_last_error() << std::endl;
			return 1;
		}
		if (rc) {  // MathException escapes the reference's main (std::terminate)
			std::cerr << "terminate called after throwing an instance of 'MathException'\n  what():  "
			          << rt_last_error() << std::endl;
			std::abort();
		}
	}
	if (!rt_builder_has_camera(b)) {
		std::cerr << "Error: At least one camera must be specified." << std::endl;
		return 1;
	}
	tm.mark("parse");
	rt_scene* scene = nullptr;
	rt_multi* multi = nullptr;
	if (o.gpus > 0) {
		std::vector<int> devices = o.devices;
		if (devices.empty())
			for (int k = 0; k < o.gpus; k++) devices.push_back(o.device + k);
		if (rt_multi_create(b, o.gpus, devices.data(), o.row_block, &multi)) {
			std::cerr << "Error: " << rt_last_error() << std::endl;
			return 1;
		}
	} else if (rt_scene_create(b, o.device, &scene)) {
		std::cerr << "Error: " << rt_last_error() << std::endl;
		return 1;
	}
	if (scene) {
		rt_scene_info info{};
		rt_scene_get_info(scene, &info);
		tm.detail.emplace_back("scene_build", info.build_ms);
		tm.detail.emplace_back("scene_upload", info.upload_ms);
	}
	tm.mark("scene_create");
	rt_render_params p{};
	p.width = o.width;
	p.height = o.height;
	p.bounce_depth = o.bdepth;
	p.intersection_only = o.intersection_only;
	p.row_begin = 0;
	p.row_end = o.height;
	p.row_step = 1;
	// RGB8 quantised on the device (writers.cpp:4-9): only 3 bytes per pixel cross PCIe,
	// unless the raw f64 image is asked for (--dump-raw)
	const size_t n = static_cast<size_t>(o.width) * o.height * 3;
	std::vector<double> img(o.dump_raw.empty() ? 0 : n);
	std::vector<uint8_t> rgb(n);
	set_alarm(true);
	rt_counters cnt{};
	int rc = multi ? rt_multi_render(multi, &p, img.empty() ? nullptr : img.data(), rgb.data(), update_progress,
	                                 nullptr, nullptr)
	         : img.empty() ? rt_render_rgb8(scene, &p, rgb.data(), update_progress, nullptr, &cnt)
	                       : rt_render(scene, &p, img.data(), update_progress, nullptr, &cnt);
	set_alarm(false);
	if (scene) {
		tm.detail.emplace_back("render_gpu", cnt.host_ms - cnt.copy_ms);
		tm.detail.emplace_back("d2h", cnt.copy_ms);
	}
	tm.mark("render");
	if (rc == RT_ERR_MATH) {
		std::cerr << "terminate called after throwing an instance of 'MathException'\n  what():  " << rt_last_error()
		          << std::endl;
		std::abort();
	}
	if (rc) {
		std::cerr << "Error: " << rt_last_error() << std::endl;
		return 1;
	}
	if (!img.empty()) {
		FILE* f = std::fopen(o.dump_raw.c_str(), "wb");
		if (f) {
			std::fwrite(img.data(), sizeof(double), img.size(), f);
			std::fclose(f);
		}
		if (!multi) rt_to_rgb8(img.data(), static_cast<int64_t>(o.width) * o.height, rgb.data());
	}
	if (rt_write_png(o.output.c_str(), rgb.data(), o.width, o.height)) {
		std::cerr << "Error: " << rt_last_error() << std::endl;
		return 1;
	}
	tm.mark("png");
	if (scene) rt_scene_destroy(scene);
	if (multi) rt_multi_destroy(multi);
	rt_builder_destroy(b);
	tm.mark("teardown");
	if (!o.timing.empty()) tm.write(o.timing);
	return 0;
}
