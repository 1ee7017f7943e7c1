// librtamd_diag.so: the render library plus test and measurement hooks.  None of these entry
// points is in include/rtamd.h or exported by librtamd.so: the tests that inject failures
// and the profiling tools (tools/) load this variant (rtamd.lib(diag=True)); the product
// path never does.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>
#include "bvh.h"
#include "render_state.h"

namespace {

int fail(int code, const std::string& msg) { return rtamd::set_error(code, msg); }

#define HIP_TRY(expr)                                                                         \
	do {                                                                                      \
		hipError_t e_ = (expr);                                                               \
		if (e_ != hipSuccess) return fail(RT_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
	} while (0)

// device scratch freed on every exit
struct DevBuf {
	void* p = nullptr;
	~DevBuf() {
		if (p) (void)hipFree(p);
	}
};

}  // namespace

extern "C" {

// CPU test hook (tests/test_host.py): the chunks a render call cuts `n` jobs into over
// `n_lanes` lanes (rt_render_batch_device: n_lanes = min(n, batch lanes)).  Segment k of
// the plan is out[4k..4k+3] = (chunk, job index in params, first row ordinal, rows); returns
// the number of segments, or -1 when out_cap segments do not suffice.  Needs no device.
int rt_debug_plan_chunks(int n, const rt_render_params* params, int n_lanes, int64_t batch_chunk_pixels, int balance,
                         int64_t* out, int out_cap) {
	std::vector<Job> jobs;
	std::vector<int> index;
	for (int k = 0; k < n; k++) {
		const Job j = make_job(params + k, nullptr, nullptr);
		if (j.n_rows <= 0) continue;
		jobs.push_back(j);
		index.push_back(k);
	}
	if (jobs.empty()) return 0;
	const auto chunks = plan_chunks(jobs, static_cast<size_t>(std::max(1, n_lanes)), jobs.size() > 1,
	                                batch_chunk_pixels, balance, 2);
	int q = 0;
	for (size_t c = 0; c < chunks.size(); c++)
		for (const Segment& sg : chunks[c]) {
			if (q >= out_cap) return -1;
			out[4 * q] = static_cast<int64_t>(c);
			out[4 * q + 1] = index[sg.job - jobs.data()];
			out[4 * q + 2] = sg.r0;
			out[4 * q + 3] = sg.rows;
			q++;
		}
	return q;
}

// FNV-1a digest of everything rt_scene_create would upload for the builder's scene
// (flattened geometry, LBVHs, materials, lights, camera), computed on the host only: equal
// digests = identical device scenes (tests of rt_builder_set_desc).
int rt_debug_builder_digest(const rt_builder* b, uint64_t* out) {
	if (!b || !out) return fail(RT_ERR_ARG, "null builder or output");
	const rtamd::FlatScene fs = rtamd::flatten_scene(b->scene);
	uint64_t h = 1469598103934665603ull;
	auto mix = [&](const void* p, size_t n) {
		const unsigned char* c = static_cast<const unsigned char*>(p);
		for (size_t i = 0; i < n; i++) h = (h ^ c[i]) * 1099511628211ull;
	};
	auto vec = [&](const auto& v) {
		const uint64_t n = v.size();
		mix(&n, sizeof(n));
		if (n) mix(v.data(), n * sizeof(v[0]));
	};
	vec(fs.geoms);
	vec(fs.materials);
	vec(fs.lights);
	vec(fs.face_geo);
	vec(fs.face_nrm);
	vec(fs.nodes);
	vec(fs.shadow_order);
	mix(&fs.camera, sizeof(fs.camera));
	*out = h;
	return RT_OK;
}

// The scene's next render fails after `launches` more closest-hit launches, as a device
// failure in the middle of a render would (tests of the error path: the render after it must
// be complete and exact).  -1 disables.
int rt_debug_fail_after(rt_scene* s, int launches) {
	if (!s) return fail(RT_ERR_ARG, "null scene");
	s->fail_after = launches;
	return RT_OK;
}

// The next chunk's row descriptors name rows no frame has (segment 0 moved past the image):
// the kernels must report DERR_ROWS (RT_ERR_DEVICE with its message) and write nothing.
int rt_debug_corrupt_rows(rt_scene* s) {
	if (!s) return fail(RT_ERR_ARG, "null scene");
	s->corrupt_rows = 1;
	return RT_OK;
}

// Phase profile of the traversal kernels (RT_PHASE_PROF builds; zeros otherwise), 4 x 8
// sums of per-lane shader-clock cycles (trace.h), read and cleared.
int rt_debug_phase_profile(int device, unsigned long long* out32) {
	HIP_TRY(hipSetDevice(device));
	HIP_TRY(hipDeviceSynchronize());
	HIP_TRY(rtamd::read_phase_profile(out32));
	return RT_OK;
}

// The per-wave timing records of an RT_DIAG_WAVETIME build (tools/wave_times.py; 32 B each:
// t0, t1 on the 100 MHz clock, tag, first item, node iterations, face tests), at most
// max_records, read and cleared; returns the count (0 in other builds).
int rt_debug_wave_times(int device, void* out, int max_records) {
	HIP_TRY(hipSetDevice(device));
	HIP_TRY(hipDeviceSynchronize());
	const int n = rtamd::read_wave_times(out, max_records);
	if (n < 0) return fail(RT_ERR_DEVICE, "wave time read-back failed");
	return n;
}

// FETCH_SIZE calibration.  Reads a fresh `bytes` buffer once per width in {1, 4, 8, 16} bytes
// per lane (one k_stream_read dispatch each, after a dispatch that streams another buffer of
// the same size through the caches); profiled with rocprofv3 --pmc FETCH_SIZE, the ratio of
// the counter to `bytes` per width corrects the path's own loads (tools/make_traffic.py).
int rt_debug_fetch_calibration(int device, int64_t bytes) {
	HIP_TRY(hipSetDevice(device));
	DevBuf b[3];
	HIP_TRY(hipMalloc(&b[0].p, bytes));
	HIP_TRY(hipMalloc(&b[1].p, bytes));
	HIP_TRY(hipMalloc(&b[2].p, 64));
	HIP_TRY(hipMemset(b[0].p, 0, bytes));
	HIP_TRY(hipMemset(b[1].p, 0, bytes));
	HIP_TRY(hipDeviceSynchronize());
	const int widths[4] = {1, 4, 8, 16};
	for (int w : widths) {
		// evict: stream the other buffer first (larger than the 256 MiB Infinity Cache)
		HIP_TRY(rtamd::launch_stream_read(b[1].p, bytes, 16, static_cast<unsigned long long*>(b[2].p), nullptr));
		HIP_TRY(rtamd::launch_stream_read(b[0].p, bytes, w, static_cast<unsigned long long*>(b[2].p), nullptr));
		HIP_TRY(hipDeviceSynchronize());
	}
	return RT_OK;
}

// VALU issue calibration.  k_valu_peak dispatches for each instruction kind (v_fma_f32,
// v_pk_fma_f32, v_fma_f64) at 1, 2, 4 and 8 waves per SIMD (each after a warm-up at the same
// shape), iterations scaled so that every dispatch issues the same instructions per SIMD;
// profiled with rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU
// GRBM_GUI_ACTIVE ..., they give cycles per wave64 instruction and the shader clock
// (tools/valu_calibration.py, tools/make_valu.py).
int rt_debug_valu_calibration(int device, int iters) {
	HIP_TRY(hipSetDevice(device));
	DevBuf sink;
	HIP_TRY(hipMalloc(&sink.p, 64));
	for (int kind = 0; kind < 3; kind++)
		for (int w = 1; w <= 8; w *= 2) {
			const int it = std::max(1, iters * 8 / w);
			HIP_TRY(rtamd::launch_valu_peak(std::max(1, it / 8), kind, w, sink.p, nullptr));  // warm-up (clocks)
			HIP_TRY(rtamd::launch_valu_peak(it, kind, w, sink.p, nullptr));
		}
	HIP_TRY(hipDeviceSynchronize());
	return RT_OK;
}

// k_valu_peak of one instruction kind (trace.hip kValuKinds) at `waves` waves per SIMD, timed
// with events after a warm-up launch; *ms = kernel time.  The kernel issues
// 256 * waves * 4 waves * iters * 128 instructions.
int rt_debug_valu_rate(int device, int kind, int waves, int iters, double* ms) {
	if (!ms || kind < 0 || waves < 1 || waves > 8 || iters < 1) return fail(RT_ERR_ARG, "bad calibration arguments");
	HIP_TRY(hipSetDevice(device));
	DevBuf sink;
	struct Events {
		hipEvent_t e0 = nullptr, e1 = nullptr;
		~Events() {
			if (e0) (void)hipEventDestroy(e0);
			if (e1) (void)hipEventDestroy(e1);
		}
	} ev;
	HIP_TRY(hipMalloc(&sink.p, 64));
	HIP_TRY(hipEventCreate(&ev.e0));
	HIP_TRY(hipEventCreate(&ev.e1));
	HIP_TRY(rtamd::launch_valu_peak(std::max(1, iters / 4), kind, waves, sink.p, nullptr));  // warm-up (clocks)
	HIP_TRY(hipEventRecord(ev.e0, nullptr));
	HIP_TRY(rtamd::launch_valu_peak(iters, kind, waves, sink.p, nullptr));
	HIP_TRY(hipEventRecord(ev.e1, nullptr));
	HIP_TRY(hipEventSynchronize(ev.e1));
	float f = 0;
	HIP_TRY(hipEventElapsedTime(&f, ev.e0, ev.e1));
	*ms = f;
	return RT_OK;
}

}  // extern "C"
