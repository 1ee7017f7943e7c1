// C-ABI of librtamd (include/rtamd.h): scene ingest, HBM upload, wavefront render
// driver, PNG output.  This is the drop-in for Scene::renderScene (scene.cpp:10-59).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>
#include "../../include/rtamd.h"
#include "bvh.h"
#include "scene_host.h"
#include "trace.h"

extern "C" int rt_encode_png(const uint8_t* rgb, int width, int height, std::vector<uint8_t>* out);

namespace {

thread_local std::string g_error;

int fail(int code, const std::string& msg) {
	g_error = msg;
	return code;
}

#define HIP_TRY(expr)                                                                         \
	do {                                                                                      \
		hipError_t e_ = (expr);                                                               \
		if (e_ != hipSuccess) return fail(RT_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
	} while (0)

const char* device_error_text(int code) {  // MathException what() (rtbase.h:14-22)
	switch (code) {
		case rtamd::DERR_NO_DIRECTION: return "ray has no direction";
		case rtamd::DERR_POINT_DIRECTION: return "ray direction is a point vector";
		case rtamd::DERR_STACK: return "internal: BVH traversal stack overflow";
		default: return "unknown device error";
	}
}

}  // namespace

struct rt_builder {
	rtamd::Scene scene;
};

struct LevelBuffers {
	rtamd::RayLevel lv{};
	void* block = nullptr;
};

struct rt_scene {
	int device = 0;
	hipStream_t stream = nullptr;
	rtamd::DeviceScene ds{};
	std::vector<void*> allocs;
	rt_scene_info info{};
	std::vector<LevelBuffers> levels;
	rtamd::DeviceCounters* ctr = nullptr;        // device
	rtamd::DeviceCounters* ctr_host = nullptr;   // pinned mirror
	unsigned long long* stats = nullptr;         // device, kStatShards x kStatStride
	std::vector<unsigned long long> stats_host;
	double* out_dev = nullptr;                   // staging for rt_render
	int64_t out_capacity = 0;
	// Shading streams: k_shadow + k_shade of level L < direct_levels run on
	// shade_streams[L % 3] while the render stream (high priority: it carries the critical
	// path) traces level L+1; the deeper, smaller levels are shaded together in batches on
	// shade_streams[3] once the closest-hit chain has finished.
	hipStream_t shade_streams[4] = {nullptr, nullptr, nullptr, nullptr};
	int direct_levels = 3;
	// RayLevel records of all levels for the batched shading kernels (pinned + device)
	rtamd::RayLevel* levels_pinned = nullptr;
	rtamd::RayLevel* levels_dev = nullptr;
	size_t levels_cap = 0;
	hipEvent_t fork_event = nullptr;             // caller's stream -> render stream
	// per level: [0] before k_closest, [1] after it (the shading streams wait on it);
	// per shading launch, in the events of its first level: [2] before k_shadow, [3] after
	// it, [4] after k_shade (the reduce waits on it)
	std::vector<std::array<hipEvent_t, 5>> level_events;
	int32_t* counts_host = nullptr;              // pinned: level counts + error word
	int packet_mask = rtamd::kPacketClosest0 | rtamd::kPacketShadow0;  // measured best on C3
};

namespace {

template <typename T>
int upload(rt_scene* s, const std::vector<T>& host, const T** dev) {
	*dev = nullptr;
	if (host.empty()) return RT_OK;
	void* p = nullptr;
	HIP_TRY(hipMalloc(&p, host.size() * sizeof(T)));
	s->allocs.push_back(p);
	HIP_TRY(hipMemcpy(p, host.data(), host.size() * sizeof(T), hipMemcpyHostToDevice));
	s->info.device_bytes += static_cast<int64_t>(host.size() * sizeof(T));
	*dev = static_cast<const T*>(p);
	return RT_OK;
}

// Level buffers grow on demand and are kept for later renders (HBM is plentiful:
// ~105 B per ray record).
int ensure_level(rt_scene* s, size_t level, int64_t capacity) {
	if (s->levels.size() <= level) s->levels.resize(level + 1);
	LevelBuffers& L = s->levels[level];
	if (L.lv.capacity >= capacity) return RT_OK;
	if (L.block) {
		HIP_TRY(hipDeviceSynchronize());
		HIP_TRY(hipFree(L.block));
		L.block = nullptr;
	}
	capacity = std::max<int64_t>(capacity, 1024);
	const int64_t n = capacity;
	const int64_t nl = std::max(8, s->ds.occl_stride);
	// 18 double arrays, 4 int32 arrays, inside flags, n x lights shadow verdicts and the
	// level's counts, each 256-B aligned
	auto align = [](int64_t b) { return (b + 255) & ~int64_t(255); };
	const int64_t bytes = 18 * align(n * 8) + 4 * align(n * 4) + align(n) + align(n * nl) + 256;
	HIP_TRY(hipMalloc(&L.block, bytes));
	char* p = static_cast<char*>(L.block);
	auto take = [&](int64_t b) {
		char* r = p;
		p += align(b);
		return r;
	};
	double** d[18] = {&L.lv.ox, &L.lv.oy, &L.lv.oz, &L.lv.dx, &L.lv.dy, &L.lv.dz, &L.lv.hpx, &L.lv.hpy, &L.lv.hpz,
	                  &L.lv.hnx, &L.lv.hny, &L.lv.hnz, &L.lv.cr, &L.lv.cg, &L.lv.cb, &L.lv.kr, &L.lv.kg, &L.lv.kb};
	for (double** q : d) *q = reinterpret_cast<double*>(take(n * 8));
	L.lv.hgeom = reinterpret_cast<int32_t*>(take(n * 4));
	L.lv.hit_list = reinterpret_cast<int32_t*>(take(n * 4));
	L.lv.child_refr = reinterpret_cast<int32_t*>(take(n * 4));
	L.lv.child_refl = reinterpret_cast<int32_t*>(take(n * 4));
	L.lv.inside = reinterpret_cast<uint8_t*>(take(n));
	L.lv.occl = reinterpret_cast<uint8_t*>(take(n * nl));
	L.lv.counts = reinterpret_cast<int32_t*>(take(256));
	L.lv.capacity = capacity;
	return RT_OK;
}

// Level `level` exists and its RayLevel record is in the pinned array (the record of an
// earlier level never changes while copies of it may be in flight).
int ensure_level_record(rt_scene* s, size_t level, int64_t capacity) {
	if (level + 1 > s->levels_cap) {
		HIP_TRY(hipDeviceSynchronize());
		const size_t cap = std::max<size_t>(16, 2 * (level + 1));
		rtamd::RayLevel *pin = nullptr, *dev = nullptr;
		HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&pin), cap * sizeof(rtamd::RayLevel), hipHostMallocDefault));
		HIP_TRY(hipMalloc(reinterpret_cast<void**>(&dev), cap * sizeof(rtamd::RayLevel)));
		if (s->levels_pinned) {
			std::memcpy(pin, s->levels_pinned, s->levels_cap * sizeof(rtamd::RayLevel));
			(void)hipHostFree(s->levels_pinned);
			(void)hipFree(s->levels_dev);
		}
		s->levels_pinned = pin;
		s->levels_dev = dev;
		s->levels_cap = cap;
	}
	int rc = ensure_level(s, level, capacity);
	if (rc) return rc;
	s->levels_pinned[level] = s->levels[level].lv;
	return RT_OK;
}

int ensure_events(rt_scene* s, size_t level) {
	while (s->level_events.size() <= level) {
		std::array<hipEvent_t, 5> ev{};
		for (hipEvent_t& e : ev) HIP_TRY(hipEventCreate(&e));
		s->level_events.push_back(ev);
	}
	return RT_OK;
}

int64_t selected_rows(const rt_render_params* p) {
	if (p->row_step <= 0 || p->row_end <= p->row_begin) return 0;
	return (p->row_end - p->row_begin + p->row_step - 1) / p->row_step;
}

int check_params(const rt_scene* s, const rt_render_params* p) {
	if (!s || !p) return fail(RT_ERR_ARG, "null scene or params");
	if (p->width <= 0 || p->height <= 0) return fail(RT_ERR_ARG, "Width and/or height must be positive.");
	if (p->bounce_depth < 0) return fail(RT_ERR_ARG, "Bounce depth must be non-negative.");
	if (p->row_begin < 0 || p->row_end > p->height || p->row_step <= 0 || p->row_begin > p->row_end)
		return fail(RT_ERR_ARG, "bad row selection");
	return RT_OK;
}

}  // namespace

extern "C" {

const char* rt_last_error(void) { return g_error.c_str(); }
const char* rt_version(void) { return "rtamd 0.1 (gfx950)"; }

rt_builder* rt_builder_create(void) { return new rt_builder(); }
void rt_builder_destroy(rt_builder* b) { delete b; }

int rt_builder_parse_rti(rt_builder* b, const char* path) {
	if (!b || !path) return fail(RT_ERR_ARG, "null builder or path");
	try {
		rtamd::parse_rti_file(b->scene, path);
	} catch (const rtamd::ParseError& e) {
		return fail(RT_ERR_PARSE, e.msg);
	} catch (const rtamd::MathError& e) {
		return fail(RT_ERR_MATH, e.msg);
	} catch (const std::exception& e) {
		return fail(RT_ERR_PARSE, e.what());
	}
	return RT_OK;
}

int rt_builder_has_camera(const rt_builder* b) { return b && b->scene.has_camera; }
const char* rt_builder_warnings(const rt_builder* b) { return b ? b->scene.warnings.c_str() : ""; }

int rt_device_count(void) {
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess) return 0;
	return n;
}

int rt_scene_create(const rt_builder* b, int device, rt_scene** out) {
	if (!b || !out) return fail(RT_ERR_ARG, "null builder or output");
	*out = nullptr;
	if (!b->scene.has_camera) return fail(RT_ERR_ARG, "At least one camera must be specified.");
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
		return fail(RT_ERR_DEVICE, "no HIP device available (the rtamd render path runs only on the GPU)");
	if (device < 0 || device >= ndev) return fail(RT_ERR_ARG, "bad device index");
	HIP_TRY(hipSetDevice(device));
	rtamd::FlatScene fs = rtamd::flatten_scene(b->scene);
	std::unique_ptr<rt_scene> s(new rt_scene());
	s->device = device;
	if (const char* pm = std::getenv("RTAMD_PACKET_MASK")) s->packet_mask = std::atoi(pm);  // tuning knobs
	if (const char* dl = std::getenv("RTAMD_DIRECT_LEVELS")) s->direct_levels = std::max(1, std::atoi(dl));
	int prio_low = 0, prio_high = 0;
	HIP_TRY(hipDeviceGetStreamPriorityRange(&prio_low, &prio_high));
	HIP_TRY(hipStreamCreateWithPriority(&s->stream, hipStreamNonBlocking, prio_high));
	for (hipStream_t& q : s->shade_streams) HIP_TRY(hipStreamCreateWithPriority(&q, hipStreamNonBlocking, prio_low));
	HIP_TRY(hipEventCreateWithFlags(&s->fork_event, hipEventDisableTiming));
	HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&s->counts_host), 4 * sizeof(int32_t), hipHostMallocDefault));
	int rc;
	if ((rc = upload(s.get(), fs.geoms, &s->ds.geoms)) || (rc = upload(s.get(), fs.materials, &s->ds.mats)) ||
	    (rc = upload(s.get(), fs.lights, &s->ds.lights)) || (rc = upload(s.get(), fs.face_geo, &s->ds.fgeo)) ||
	    (rc = upload(s.get(), fs.face_nrm, &s->ds.fnrm)) || (rc = upload(s.get(), fs.face_id, &s->ds.fid)) ||
	    (rc = upload(s.get(), fs.nodes, &s->ds.nodes)) || (rc = upload(s.get(), fs.shadow_order, &s->ds.shadow_order))) {
		rt_scene_destroy(s.release());
		return rc;
	}
	s->ds.cam = fs.camera;
	s->ds.n_geoms = static_cast<int32_t>(fs.geoms.size());
	s->ds.n_may_raise = fs.n_may_raise;
	s->ds.n_lights = static_cast<int32_t>(fs.lights.size());
	s->ds.n_nonambient = 0;
	for (size_t li = 0; li < fs.lights.size(); li++) {
		if (fs.lights[li].kind == rtamd::LIGHT_AMBIENT) continue;
		if (s->ds.n_nonambient >= rtamd::kMaxShadowLights) {
			rt_scene_destroy(s.release());
			return fail(RT_ERR_ARG, "too many non-ambient lights (max 64)");
		}
		s->ds.shadow_light[s->ds.n_nonambient++] = static_cast<int32_t>(li);
	}
	s->ds.occl_stride = (s->ds.n_nonambient + 7) / 8 * 8;
	void* c = nullptr;
	HIP_TRY(hipMalloc(&c, sizeof(rtamd::DeviceCounters)));
	s->allocs.push_back(c);
	s->ctr = static_cast<rtamd::DeviceCounters*>(c);
	HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&s->ctr_host), sizeof(rtamd::DeviceCounters), hipHostMallocDefault));
	void* st = nullptr;
	HIP_TRY(hipMalloc(&st, sizeof(unsigned long long) * rtamd::kStatShards * rtamd::kStatStride));
	s->allocs.push_back(st);
	s->stats = static_cast<unsigned long long*>(st);
	s->stats_host.resize(rtamd::kStatShards * rtamd::kStatStride);
	rt_scene_info& in = s->info;
	in.n_geometries = s->ds.n_geoms;
	for (const auto& g : fs.geoms) (g.kind == rtamd::GEOM_SPHERE ? in.n_spheres : in.n_meshes)++;
	in.n_lights = s->ds.n_lights;
	in.n_faces = static_cast<int64_t>(fs.face_geo.size());
	in.n_bvh_nodes = static_cast<int64_t>(fs.nodes.size());
	*out = s.release();
	return RT_OK;
}

void rt_scene_destroy(rt_scene* s) {
	if (!s) return;
	(void)hipSetDevice(s->device);
	(void)hipDeviceSynchronize();
	for (auto& L : s->levels)
		if (L.block) (void)hipFree(L.block);
	for (void* p : s->allocs) (void)hipFree(p);
	if (s->out_dev) (void)hipFree(s->out_dev);
	if (s->ctr_host) (void)hipHostFree(s->ctr_host);
	if (s->counts_host) (void)hipHostFree(s->counts_host);
	if (s->levels_pinned) (void)hipHostFree(s->levels_pinned);
	if (s->levels_dev) (void)hipFree(s->levels_dev);
	for (auto& ev : s->level_events)
		for (hipEvent_t e : ev) (void)hipEventDestroy(e);
	for (hipStream_t q : s->shade_streams)
		if (q) (void)hipStreamDestroy(q);
	if (s->fork_event) (void)hipEventDestroy(s->fork_event);
	if (s->stream) (void)hipStreamDestroy(s->stream);
	delete s;
}

int rt_scene_get_info(const rt_scene* s, rt_scene_info* info) {
	if (!s || !info) return fail(RT_ERR_ARG, "null scene or info");
	*info = s->info;
	return RT_OK;
}

int rt_render_device(rt_scene* s, const rt_render_params* p, double* out_rgb_dev, uint8_t* out_rgb8_dev, void* stream_v,
                     rt_counters* counters) {
	int rc = check_params(s, p);
	if (rc) return rc;
	HIP_TRY(hipSetDevice(s->device));
	// All work runs on the scene's streams; a caller's stream is joined first (its prior
	// work, e.g. the allocation of the output buffers, completes before ours starts) and
	// the call returns after the render stream has drained.
	hipStream_t caller = stream_v ? static_cast<hipStream_t>(stream_v) : s->stream;
	hipStream_t st = s->stream;
	if (caller != st) {
		HIP_TRY(hipEventRecord(s->fork_event, caller));
		HIP_TRY(hipStreamWaitEvent(st, s->fork_event, 0));
	}
	const int64_t W = p->width;
	const int64_t n_rows = selected_rows(p);
	const int io = p->intersection_only != 0;
	const int depth = io ? 0 : p->bounce_depth;
	int64_t chunk_pixels = p->chunk_pixels > 0 ? p->chunk_pixels : (int64_t)1 << 22;
	const int64_t chunk_rows = std::max<int64_t>(1, chunk_pixels / W);
	rt_counters cnt{};
	cnt.intersection_max = 2.2250738585072014e-308;  // numeric_limits<double>::min() (scene.cpp:51)
	HIP_TRY(hipMemsetAsync(s->ctr, 0, sizeof(rtamd::DeviceCounters), st));
	HIP_TRY(hipMemsetAsync(s->stats, 0, sizeof(unsigned long long) * s->stats_host.size(), st));
	std::vector<int64_t> level_n;
	float kernel_ms_total = 0.f;
	for (int64_t r0 = 0; r0 < n_rows; r0 += chunk_rows) {
		const int64_t rows = std::min(chunk_rows, n_rows - r0);
		const int64_t n0 = rows * W;
		rtamd::FrameGeometry fg{};
		fg.width = p->width;
		fg.height = p->height;
		fg.row_begin = p->row_begin;
		fg.row_step = p->row_step;
		fg.chunk_row0 = static_cast<int32_t>(r0);
		fg.intersection_only = io;
		level_n.assign(1, n0);
		if ((rc = ensure_level_record(s, 0, n0))) return rc;
		std::vector<int> shaded;                            // first level of each shading launch
		std::vector<std::pair<int, int64_t>> deferred;      // (level, hits) shaded after the chain
		// k_shadow + k_shade of the levels `lv` (their k_closest done) on stream q
		auto launch_shading = [&](const std::vector<std::pair<int, int64_t>>& lv, hipStream_t q) -> int {
			rtamd::ShadeBatch b{};
			const int64_t nl = s->ds.n_nonambient;
			auto wave_up = [](int64_t x) { return (x + 63) & ~int64_t(63); };
			int64_t so = 0, ho = 0;
			b.n = static_cast<int32_t>(lv.size());
			for (int k = 0; k < b.n; k++) {
				b.level[k] = lv[k].first;
				b.nh[k] = lv[k].second;
				b.shadow_begin[k] = so;
				b.shade_begin[k] = ho;
				so += wave_up(lv[k].second * nl);
				ho += wave_up(lv[k].second);
			}
			b.shadow_begin[b.n] = so;
			b.shade_begin[b.n] = ho;
			const int first = lv.front().first, last = lv.back().first;
			const auto& ev = s->level_events[first];
			HIP_TRY(hipStreamWaitEvent(q, s->level_events[last][1], 0));
			HIP_TRY(hipMemcpyAsync(s->levels_dev, s->levels_pinned, (last + 1) * sizeof(rtamd::RayLevel),
			                       hipMemcpyHostToDevice, q));
			HIP_TRY(hipEventRecord(ev[2], q));
			HIP_TRY(rtamd::launch_shadow(s->ds, b, s->levels_dev, s->ctr, s->stats, q, s->packet_mask));
			if (nl > 0) cnt.stage_launches[1]++;
			HIP_TRY(hipEventRecord(ev[3], q));
			HIP_TRY(rtamd::launch_shade(s->ds, fg, b, s->levels_dev, s->ctr, q));
			cnt.stage_launches[2]++;
			HIP_TRY(hipEventRecord(ev[4], q));
			shaded.push_back(first);
			return RT_OK;
		};
		bool error = false;
		for (int L = 0;; L++) {
			const int remaining = depth - L;
			const int64_t n = level_n[L];
			if (remaining > 0 && (rc = ensure_level_record(s, L + 1, 2 * n))) return rc;
			if ((rc = ensure_events(s, L))) return rc;
			const auto& ev = s->level_events[L];
			const rtamd::RayLevel& cur = s->levels[L].lv;
			const rtamd::RayLevel& next = remaining > 0 ? s->levels[L + 1].lv : cur;
			HIP_TRY(hipMemsetAsync(cur.counts, 0, 2 * sizeof(int32_t), st));
			HIP_TRY(hipEventRecord(ev[0], st));
			HIP_TRY(rtamd::launch_closest(s->ds, fg, L, n, remaining, cur, next, s->ctr, s->stats, st, s->packet_mask));
			cnt.stage_launches[0]++;
			HIP_TRY(hipEventRecord(ev[1], st));
			HIP_TRY(hipMemcpyAsync(s->counts_host, cur.counts, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, st));
			HIP_TRY(hipMemcpyAsync(s->counts_host + 2, &s->ctr->error, sizeof(int32_t), hipMemcpyDeviceToHost, st));
			HIP_TRY(hipStreamSynchronize(st));
			if (s->counts_host[2]) {
				error = true;
				break;
			}
			cnt.trace_rays += n;
			const int64_t nh = s->counts_host[0], nn = s->counts_host[1];
			if (nh > 0) {
				if (L < s->direct_levels) {  // big level: shade now, concurrent with k_closest(L+1)
					if ((rc = launch_shading({{L, nh}}, s->shade_streams[L % 3]))) return rc;
				} else {
					deferred.push_back({L, nh});
				}
			}
			if (remaining <= 0 || nn == 0) break;
			level_n.push_back(nn);
		}
		if (error) {
			HIP_TRY(hipDeviceSynchronize());
			break;
		}
		for (size_t k = 0; k < deferred.size(); k += rtamd::kMaxBatch) {
			const size_t e = std::min(deferred.size(), k + rtamd::kMaxBatch);
			if ((rc = launch_shading({deferred.begin() + k, deferred.begin() + e}, s->shade_streams[3]))) return rc;
		}
		for (int L : shaded) HIP_TRY(hipStreamWaitEvent(st, s->level_events[L][4], 0));
		for (int L = static_cast<int>(level_n.size()) - 2; L >= 0; L--)
			HIP_TRY(rtamd::launch_reduce_level(level_n[L], s->levels[L].lv, s->levels[L + 1].lv, st));
		HIP_TRY(rtamd::launch_output(n0, s->levels[0].lv, out_rgb_dev ? out_rgb_dev + r0 * W * 3 : nullptr,
		                             out_rgb8_dev ? out_rgb8_dev + r0 * W * 3 : nullptr, io, s->stats, st));
		// per-kernel device times of this chunk (events are re-recorded by the next chunk)
		HIP_TRY(hipStreamSynchronize(st));
		for (int L = 0; L < static_cast<int>(level_n.size()); L++) {
			const auto& ev = s->level_events[L];
			float ms = 0.f;
			HIP_TRY(hipEventElapsedTime(&ms, ev[0], ev[1]));
			cnt.stage_ms[0] += ms;
			kernel_ms_total += ms;
		}
		for (int L : shaded) {
			const auto& ev = s->level_events[L];
			for (int k = 0; k < 2; k++) {
				float ms = 0.f;
				HIP_TRY(hipEventElapsedTime(&ms, ev[2 + k], ev[3 + k]));
				cnt.stage_ms[1 + k] += ms;
				kernel_ms_total += ms;
			}
		}
		cnt.levels = std::max<int32_t>(cnt.levels, static_cast<int32_t>(level_n.size()));
		cnt.pixels += n0;
	}
	HIP_TRY(hipMemcpyAsync(s->ctr_host, s->ctr, sizeof(rtamd::DeviceCounters), hipMemcpyDeviceToHost, st));
	HIP_TRY(hipStreamSynchronize(st));
	if (s->ctr_host->error) return fail(RT_ERR_MATH, device_error_text(s->ctr_host->error));
	HIP_TRY(hipMemcpy(s->stats_host.data(), s->stats, sizeof(unsigned long long) * s->stats_host.size(),
	                  hipMemcpyDeviceToHost));
	unsigned long long sum[rtamd::ST_COUNT] = {0};
	for (int sh = 0; sh < rtamd::kStatShards; sh++)
		for (int k = 0; k < rtamd::ST_COUNT; k++) {
			const unsigned long long v = s->stats_host[sh * rtamd::kStatStride + k];
			sum[k] = (k == rtamd::ST_MAX_BITS) ? std::max(sum[k], v) : sum[k] + v;
		}
	cnt.shadow_rays = static_cast<int64_t>(sum[rtamd::ST_HITS]) * s->ds.n_nonambient;
	cnt.reflect_rays = static_cast<int64_t>(sum[rtamd::ST_REFL]);
	cnt.refract_rays = static_cast<int64_t>(sum[rtamd::ST_REFR]);
	for (int k = 0; k < 2; k++) {
		const int b = k ? rtamd::ST_NODES1 : rtamd::ST_NODES0;
		cnt.stage_node_visits[k] = static_cast<int64_t>(sum[b]);
		cnt.stage_tri_tests[k] = static_cast<int64_t>(sum[b + 1]);
		cnt.stage_candidates[k] = static_cast<int64_t>(sum[b + 2]);
		cnt.stage_sphere_tests[k] = static_cast<int64_t>(sum[b + 3]);
		cnt.stage_bvh_traversals[k] = static_cast<int64_t>(sum[k ? rtamd::ST_ENTRIES1 : rtamd::ST_ENTRIES0]);
		cnt.node_visits += cnt.stage_node_visits[k];
		cnt.tri_tests += cnt.stage_tri_tests[k];
		cnt.candidates += cnt.stage_candidates[k];
		cnt.sphere_tests += cnt.stage_sphere_tests[k];
	}
	cnt.trace_launches = cnt.stage_launches[0] + cnt.stage_launches[1] + cnt.stage_launches[2];
	if (io && sum[rtamd::ST_MAX_BITS]) {
		double m;
		const unsigned long long b = sum[rtamd::ST_MAX_BITS];
		std::memcpy(&m, &b, sizeof(m));
		cnt.intersection_max = std::max(cnt.intersection_max, m);
	}
	cnt.kernel_ms = kernel_ms_total;
	// full-image --intersection-only: normalise in place (scene.cpp:50-58)
	if (io && p->row_begin == 0 && p->row_end == p->height && p->row_step == 1 && out_rgb_dev) {
		HIP_TRY(rtamd::launch_normalize(n_rows * W * 3, out_rgb_dev, cnt.intersection_max, out_rgb8_dev, st));
		HIP_TRY(hipStreamSynchronize(st));
	}
	if (counters) *counters = cnt;
	return RT_OK;
}

int rt_render(rt_scene* s, const rt_render_params* p, double* out_rgb, rt_progress_fn progress, void* user,
              rt_counters* counters) {
	int rc = check_params(s, p);
	if (rc) return rc;
	if (!out_rgb) return fail(RT_ERR_ARG, "null output");
	HIP_TRY(hipSetDevice(s->device));
	const int64_t n = selected_rows(p) * p->width;
	if (s->out_capacity < n) {
		if (s->out_dev) HIP_TRY(hipFree(s->out_dev));
		s->out_dev = nullptr;
		HIP_TRY(hipMalloc(reinterpret_cast<void**>(&s->out_dev), std::max<int64_t>(n, 1) * 3 * sizeof(double)));
		s->out_capacity = n;
	}
	const int total = static_cast<int>(std::min<int64_t>(n, 0x7fffffff));
	if (progress) progress(0, total, user);
	rc = rt_render_device(s, p, s->out_dev, nullptr, nullptr, counters);
	if (rc) return rc;
	HIP_TRY(hipMemcpy(out_rgb, s->out_dev, n * 3 * sizeof(double), hipMemcpyDeviceToHost));
	if (progress) progress(total, total, user);
	return RT_OK;
}

int rt_normalize_device(rt_scene* s, double* rgb_dev, int64_t n_pixels, double max_value, uint8_t* out_rgb8_dev,
                        void* stream) {
	if (!s || !rgb_dev) return fail(RT_ERR_ARG, "null scene or image");
	HIP_TRY(hipSetDevice(s->device));
	hipStream_t st = stream ? static_cast<hipStream_t>(stream) : s->stream;
	HIP_TRY(rtamd::launch_normalize(n_pixels * 3, rgb_dev, max_value, out_rgb8_dev, st));
	HIP_TRY(hipStreamSynchronize(st));
	return RT_OK;
}

int rt_write_png(const char* path, const uint8_t* rgb, int width, int height) {
	if (!path || !rgb || width <= 0 || height <= 0) return fail(RT_ERR_ARG, "bad PNG arguments");
	std::vector<uint8_t> bytes;
	int rc = rt_encode_png(rgb, width, height, &bytes);
	if (rc) return fail(rc, "zlib failure");
	FILE* f = std::fopen(path, "wb");
	if (!f) return fail(RT_ERR_IO, std::string("can't open output file ") + path);
	const size_t w = std::fwrite(bytes.data(), 1, bytes.size(), f);
	std::fclose(f);
	if (w != bytes.size()) return fail(RT_ERR_IO, "write error");
	return RT_OK;
}

int rt_selftest_math(int device, int op, const double* x, const double* y, double* out, int64_t n) {
	if (n <= 0) return RT_OK;
	HIP_TRY(hipSetDevice(device));
	double *dx = nullptr, *dy = nullptr, *dout = nullptr;
	HIP_TRY(hipMalloc(reinterpret_cast<void**>(&dx), n * sizeof(double)));
	HIP_TRY(hipMalloc(reinterpret_cast<void**>(&dy), n * sizeof(double)));
	HIP_TRY(hipMalloc(reinterpret_cast<void**>(&dout), n * sizeof(double)));
	HIP_TRY(hipMemcpy(dx, x, n * sizeof(double), hipMemcpyHostToDevice));
	HIP_TRY(hipMemcpy(dy, y ? y : x, n * sizeof(double), hipMemcpyHostToDevice));
	HIP_TRY(rtamd::launch_selftest_math(op, dx, dy, dout, n, nullptr));
	HIP_TRY(hipMemcpy(out, dout, n * sizeof(double), hipMemcpyDeviceToHost));
	(void)hipFree(dx);
	(void)hipFree(dy);
	(void)hipFree(dout);
	return RT_OK;
}

}  // extern "C"
