// librtamd_multi: Scene::renderScene over several GPUs of one node from one process
// (include/rtamd_multi.h).  Each device holds the scene and renders its row blocks through
// librtamd (one host thread per device: rt_render_device blocks); the rows then go to the
// first device over RCCL (ncclSend/ncclRecv in one group, xGMI) and are de-interleaved
// there (k_deinterleave, trace.hip); --intersection-only all-reduces the maxima first.
// A device list that names one GPU more than once (several partitions sharing a GPU: the
// N > 1 path rehearsed on one device) cannot have an RCCL communicator (one rank per GPU):
// the rows then go to the first partition with device copies and the maxima are reduced on
// the host; everything else (row partition, per-partition normalisation, de-interleave) is
// the same code.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <algorithm>
#include <chrono>
#include <memory>
#include <cstring>
#include <set>
#include <string>
#include <thread>
#include <vector>
#include "../../include/rtamd.h"
#include "../../include/rtamd_multi.h"
#include "markers.h"
#include "trace.h"

namespace rtamd {
int set_error(int code, const std::string& msg);
}

namespace {

int fail(int code, const std::string& msg) { return rtamd::set_error(code, msg); }

#define HIP_TRY(expr)                                                                                    \
	do {                                                                                                 \
		hipError_t e_ = (expr);                                                                          \
		if (e_ != hipSuccess) return fail(RT_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
	} while (0)
#define NCCL_TRY(expr)                                                                                      \
	do {                                                                                                    \
		ncclResult_t r_ = (expr);                                                                           \
		if (r_ != ncclSuccess) return fail(RT_ERR_DEVICE, std::string(#expr ": ") + ncclGetErrorString(r_)); \
	} while (0)

template <typename T>
int ensure(T** p, int64_t* cap, int64_t n) {  // device buffer of at least n elements (current device)
	if (*cap >= n) return RT_OK;
	if (*p) HIP_TRY(hipFree(*p));
	*p = nullptr;
	*cap = 0;
	HIP_TRY(hipMalloc(reinterpret_cast<void**>(p), std::max<int64_t>(n, 1) * sizeof(T)));
	*cap = n;
	return RT_OK;
}

double now_ms() {
	return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

struct Device {
	int id = 0;
	rt_scene* scene = nullptr;
	ncclComm_t comm = nullptr;
	hipStream_t stream = nullptr;
	double* f64 = nullptr;        // this device's rows (f64), or on device 0 every rank's rows
	uint8_t* u8 = nullptr;
	int64_t f64_cap = 0, u8_cap = 0;
	double* recv64 = nullptr;     // device 0: rows received from this device
	uint8_t* recv8 = nullptr;
	int64_t recv64_cap = 0, recv8_cap = 0;
	double* maxv = nullptr;       // --intersection-only: this device's maximum, all-reduced
	double render_ms = 0;
};

struct rt_multi {
	int block = 8;
	std::vector<Device> dev;
	uint8_t* img = nullptr;       // device 0: the assembled image (bytes)
	int64_t img_cap = 0;
	double gather_ms = 0;
	bool rccl = true;             // distinct devices: RCCL; a shared device: copies (see top)
};

namespace {

int multi_init(rt_multi* m, int n, const int* devices, int row_block, const rt_builder* b, const rt_scene_desc* d) {
	if (n < 1 || n > rtamd::kMaxGpus || !devices) return fail(RT_ERR_ARG, "bad device list");
	m->block = row_block > 0 ? row_block : 8;
	m->dev.resize(n);
	for (int i = 0; i < n; i++) {
		Device& D = m->dev[i];
		D.id = devices[i];
		const int rc = b ? rt_scene_create(b, D.id, &D.scene) : rt_scene_create_desc(d, D.id, &D.scene);
		if (rc) return rc;
		HIP_TRY(hipSetDevice(D.id));
		HIP_TRY(hipStreamCreateWithFlags(&D.stream, hipStreamNonBlocking));
		HIP_TRY(hipMalloc(reinterpret_cast<void**>(&D.maxv), sizeof(double)));
	}
	m->rccl = std::set<int>(devices, devices + n).size() == static_cast<size_t>(n);
	if (!m->rccl) return RT_OK;
	std::vector<ncclComm_t> comms(n);
	NCCL_TRY(ncclCommInitAll(comms.data(), n, devices));
	for (int i = 0; i < n; i++) m->dev[i].comm = comms[i];
	return RT_OK;
}

// this device's rows of the image (rt_partition_row)
rt_render_params device_params(const rt_render_params* p, int i, int n, int block) {
	rt_render_params q = *p;
	q.row_begin = i * block;
	q.row_end = p->height;
	q.row_step = n;
	q.row_block = block;
	return q;
}

int64_t device_rows(int64_t H, int i, int n, int block) {
	int64_t k = 0;
	for (int64_t r = 0; r < H; r++) {
		int d;
		int64_t l;
		rtamd::partition_row(r, n, block, &d, &l);
		k += d == i;
	}
	return k;
}

}  // namespace

extern "C" {

int rt_multi_create(const rt_builder* b, int n_devices, const int* devices, int row_block, rt_multi** out) {
	if (!b || !out) return fail(RT_ERR_ARG, "null builder or output");
	*out = nullptr;
	rt_multi* m = new rt_multi();
	const int rc = multi_init(m, n_devices, devices, row_block, b, nullptr);
	if (rc) {
		rt_multi_destroy(m);
		return rc;
	}
	*out = m;
	return RT_OK;
}

int rt_multi_create_desc(const rt_scene_desc* d, int n_devices, const int* devices, int row_block, rt_multi** out) {
	if (!d || !out) return fail(RT_ERR_ARG, "null descriptor or output");
	*out = nullptr;
	rt_multi* m = new rt_multi();
	const int rc = multi_init(m, n_devices, devices, row_block, nullptr, d);
	if (rc) {
		rt_multi_destroy(m);
		return rc;
	}
	*out = m;
	return RT_OK;
}

void rt_multi_destroy(rt_multi* m) {
	if (!m) return;
	for (Device& D : m->dev) {
		(void)hipSetDevice(D.id);
		(void)hipDeviceSynchronize();
		if (D.comm) (void)ncclCommDestroy(D.comm);
		for (void* p : {(void*)D.f64, (void*)D.u8, (void*)D.recv64, (void*)D.recv8, (void*)D.maxv})
			if (p) (void)hipFree(p);
		if (D.stream) (void)hipStreamDestroy(D.stream);
		if (D.scene) rt_scene_destroy(D.scene);
	}
	if (!m->dev.empty() && m->img) {
		(void)hipSetDevice(m->dev[0].id);
		(void)hipFree(m->img);
	}
	delete m;
}

int rt_multi_render(rt_multi* m, const rt_render_params* p, double* out_rgb, uint8_t* out_rgb8,
                    rt_progress_fn progress, void* user, rt_counters* counters) {
	if (!m || !p) return fail(RT_ERR_ARG, "null multi-GPU scene or params");
	if (!out_rgb && !out_rgb8) return fail(RT_ERR_ARG, "null output");
	if (p->width <= 0 || p->height <= 0) return fail(RT_ERR_ARG, "Width and/or height must be positive.");
	if (p->row_begin != 0 || p->row_end != p->height || p->row_step != 1)
		return fail(RT_ERR_ARG, "rt_multi_render renders whole images");
	const int n = static_cast<int>(m->dev.size());
	const int64_t W = p->width, H = p->height;
	const bool io = p->intersection_only != 0;
	const bool want64 = out_rgb != nullptr || io;  // --intersection-only normalises the f64 image
	const int total = static_cast<int>(std::min<int64_t>(W * H, 0x7fffffff));
	if (progress) progress(0, total, user);
	std::vector<int64_t> rows(n);
	std::vector<rt_counters> cnt(n);
	std::vector<int> rcs(n, RT_OK);
	std::vector<std::string> errs(n);
	// 1. every device renders its row blocks (one host thread each)
	for (int i = 0; i < n; i++) {
		Device& D = m->dev[i];
		rows[i] = device_rows(H, i, n, m->block);
		HIP_TRY(hipSetDevice(D.id));
		int rc;
		if (want64 && (rc = ensure(&D.f64, &D.f64_cap, rows[i] * W * 3))) return rc;
		if (out_rgb8 && (rc = ensure(&D.u8, &D.u8_cap, rows[i] * W * 3))) return rc;
	}
	std::unique_ptr<rtamd::MarkerRange> phase(new rtamd::MarkerRange("rtamd_multi: devices render their row blocks"));
	std::vector<std::thread> th;
	for (int i = 0; i < n; i++)
		th.emplace_back([&, i]() {
			Device& D = m->dev[i];
			const double t0 = now_ms();
			if (hipSetDevice(D.id) != hipSuccess) {
				rcs[i] = RT_ERR_DEVICE;
				errs[i] = "hipSetDevice failed";
				return;
			}
			const rt_render_params q = device_params(p, i, n, m->block);
			// (a device holding the whole image normalises an --intersection-only render itself,
			// rt_render_device; the others return raw 1/d^2 values and their maximum)
			rcs[i] = rows[i] ? rt_render_device(D.scene, &q, want64 ? D.f64 : nullptr, out_rgb8 ? D.u8 : nullptr,
			                                    D.stream, &cnt[i])
			                 : RT_OK;
			if (rcs[i]) errs[i] = rt_last_error();
			D.render_ms = now_ms() - t0;
		});
	for (std::thread& t : th) t.join();
	for (int i = 0; i < n; i++)
		if (rcs[i]) return fail(rcs[i], errs[i]);
	phase.reset();  // the render range is popped before the next one is pushed (ranges nest)
	phase.reset(new rtamd::MarkerRange("rtamd_multi: max all-reduce + row gather + assembly"));
	const double tg = now_ms();
	// 2. --intersection-only: the global maximum (scene.cpp:50-58), then normalise on every device
	double gmax = 0.0;
	if (io) {
		// max initialised with DBL_MIN (scene.cpp:51); a device without rows contributes it
		std::vector<double> local(n, 2.2250738585072014e-308);
		for (int i = 0; i < n; i++)
			if (rows[i]) local[i] = std::max(cnt[i].intersection_max, local[i]);
		if (m->rccl) {
			// the local maxima reach the devices before the group (the renders have returned,
			// so a synchronous copy orders nothing else)
			for (int i = 0; i < n; i++) {
				HIP_TRY(hipSetDevice(m->dev[i].id));
				HIP_TRY(hipMemcpy(m->dev[i].maxv, &local[i], sizeof(double), hipMemcpyHostToDevice));
			}
			NCCL_TRY(ncclGroupStart());
			for (int i = 0; i < n; i++) {
				Device& D = m->dev[i];
				NCCL_TRY(ncclAllReduce(D.maxv, D.maxv, 1, ncclFloat64, ncclMax, D.comm, D.stream));
			}
			NCCL_TRY(ncclGroupEnd());
			for (int i = 0; i < n; i++) {
				Device& D = m->dev[i];
				HIP_TRY(hipSetDevice(D.id));
				HIP_TRY(hipStreamSynchronize(D.stream));
				HIP_TRY(hipMemcpy(&local[i], D.maxv, sizeof(double), hipMemcpyDeviceToHost));
			}
		} else {
			const double g = *std::max_element(local.begin(), local.end());
			std::fill(local.begin(), local.end(), g);
		}
		// a device's share is normalised by rt_render_device itself only when it is the whole
		// image (n == 1: row_step 1); with n > 1 every share holds raw 1/d^2 values, even one
		// that holds every row (H <= row_block)
		for (int i = 0; i < n; i++) {
			Device& D = m->dev[i];
			HIP_TRY(hipSetDevice(D.id));
			if (rows[i] && n > 1 &&
			    rt_normalize_device(D.scene, D.f64, rows[i] * W, local[i], out_rgb8 ? D.u8 : nullptr, D.stream) != RT_OK)
				return RT_ERR_DEVICE;
		}
		gmax = local[0];
	}
	// 3. rows to device 0 (one group of sends/receives: RCCL over xGMI)
	Device& D0 = m->dev[0];
	for (int i = 1; i < n; i++) {
		HIP_TRY(hipSetDevice(D0.id));
		int rc;
		if (out_rgb && (rc = ensure(&m->dev[i].recv64, &m->dev[i].recv64_cap, rows[i] * W * 3))) return rc;
		if (out_rgb8 && (rc = ensure(&m->dev[i].recv8, &m->dev[i].recv8_cap, rows[i] * W * 3))) return rc;
	}
	if (n > 1 && !m->rccl) {
		// partitions sharing a GPU: device copies into the first partition's buffers (the
		// renders and normalisations above have completed)
		for (int i = 1; i < n; i++) {
			Device& D = m->dev[i];
			if (!rows[i]) continue;
			const size_t c = static_cast<size_t>(rows[i] * W * 3);
			if (out_rgb)
				HIP_TRY(hipMemcpyPeerAsync(D.recv64, D0.id, D.f64, D.id, c * sizeof(double), D0.stream));
			if (out_rgb8) HIP_TRY(hipMemcpyPeerAsync(D.recv8, D0.id, D.u8, D.id, c, D0.stream));
		}
	} else if (n > 1) {
		NCCL_TRY(ncclGroupStart());
		for (int i = 1; i < n; i++) {
			Device& D = m->dev[i];
			if (!rows[i]) continue;
			const size_t c = static_cast<size_t>(rows[i] * W * 3);
			if (out_rgb) {
				NCCL_TRY(ncclSend(D.f64, c, ncclFloat64, 0, D.comm, D.stream));
				NCCL_TRY(ncclRecv(D.recv64, c, ncclFloat64, i, D0.comm, D0.stream));
			}
			if (out_rgb8) {
				NCCL_TRY(ncclSend(D.u8, c, ncclUint8, 0, D.comm, D.stream));
				NCCL_TRY(ncclRecv(D.recv8, c, ncclUint8, i, D0.comm, D0.stream));
			}
		}
		NCCL_TRY(ncclGroupEnd());
	}
	// 4. assemble on device 0 and copy to the host
	HIP_TRY(hipSetDevice(D0.id));
	const int64_t bytes64 = W * H * 3 * (int64_t)sizeof(double), bytes8 = W * H * 3;
	int rc;
	if ((rc = ensure(&m->img, &m->img_cap, std::max<int64_t>(out_rgb ? bytes64 : 0, bytes8)))) return rc;
	for (int pass = 0; pass < 2; pass++) {
		const bool f64 = pass == 0;
		if (f64 ? !out_rgb : !out_rgb8) continue;
		rtamd::RowSources src{};
		for (int i = 0; i < n; i++)
			src.src[i] = i == 0 ? (f64 ? reinterpret_cast<const uint8_t*>(D0.f64) : D0.u8)
			                    : (f64 ? reinterpret_cast<const uint8_t*>(m->dev[i].recv64) : m->dev[i].recv8);
		const int64_t row_bytes = W * 3 * (f64 ? (int64_t)sizeof(double) : 1);
		HIP_TRY(rtamd::launch_deinterleave(m->img, src, n, m->block, H, row_bytes, D0.stream));
		HIP_TRY(hipMemcpyAsync(f64 ? static_cast<void*>(out_rgb) : static_cast<void*>(out_rgb8), m->img,
		                       f64 ? bytes64 : bytes8, hipMemcpyDeviceToHost, D0.stream));
		HIP_TRY(hipStreamSynchronize(D0.stream));
	}
	for (int i = 1; i < n; i++) {
		HIP_TRY(hipSetDevice(m->dev[i].id));
		HIP_TRY(hipStreamSynchronize(m->dev[i].stream));
	}
	m->gather_ms = now_ms() - tg;
	if (counters) {
		rt_counters sum{};
		for (int i = 0; i < n; i++) {
			const rt_counters& c = cnt[i];
			sum.trace_rays += c.trace_rays;
			sum.shadow_rays += c.shadow_rays;
			sum.reflect_rays += c.reflect_rays;
			sum.refract_rays += c.refract_rays;
			sum.shadow_rays_zero_terms += c.shadow_rays_zero_terms;
			sum.pixels += c.pixels;
			sum.node_visits += c.node_visits;
			sum.tri_tests += c.tri_tests;
			sum.candidates += c.candidates;
			sum.sphere_tests += c.sphere_tests;
			sum.levels = std::max(sum.levels, c.levels);
		}
		sum.intersection_max = gmax;
		*counters = sum;
	}
	if (progress) progress(total, total, user);
	return RT_OK;
}

int rt_multi_last_times(const rt_multi* m, double* render_ms, double* gather_ms) {
	if (!m) return fail(RT_ERR_ARG, "null multi-GPU scene");
	if (render_ms)
		for (size_t i = 0; i < m->dev.size(); i++) render_ms[i] = m->dev[i].render_ms;
	if (gather_ms) *gather_ms = m->gather_ms;
	return RT_OK;
}

}  // extern "C"
