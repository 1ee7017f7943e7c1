// C-ABI of librtamd (include/rtamd.h): scene ingest, HBM upload, wavefront render
// driver, PNG output.  This is the drop-in for Scene::renderScene (scene.cpp:10-59).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <functional>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>
#include "../../include/rtamd.h"
#include "bvh.h"
#include "markers.h"
#include "scene_host.h"
#include "trace.h"
#include "xform.h"

extern "C" int rt_encode_png(const uint8_t* rgb, int width, int height, std::vector<uint8_t>* out);

namespace {

thread_local std::string g_error;
constexpr size_t kFinDoneBytes = 9 * 128;  // rt_scene::fin_done: top + 8 per-XCD counters (trace.hip)

int fail(int code, const std::string& msg) {
	g_error = msg;
	return code;
}

double now_s() {
	using clk = std::chrono::steady_clock;
	return std::chrono::duration<double>(clk::now().time_since_epoch()).count();
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
		case rtamd::DERR_ORIGIN_DIRECTION: return "ray origin is a direction vector";
		case rtamd::DERR_PLAN: return "internal: a replayed launch plan did not fit the render";
		case rtamd::DERR_ROWS: return "internal: a chunk row descriptor names no selected row of the frame";
		default: return "unknown device error";
	}
}

}  // namespace

namespace rtamd {
// rt_last_error() text for the calling thread (librtamd_multi reports through it)
int set_error(int code, const std::string& msg) { return fail(code, msg); }
}  // namespace rtamd

#include "render_state.h"


namespace {

// Pinned host memory (staging, records, counts, the summary and the mapped image stage):
// fine-grained (coherent), so that no GPU cache holds a line of it between a kernel's write
// and the host's read (round 5: no measurable cost on the mapped image writes)
constexpr unsigned kPinned = hipHostMallocCoherent;
constexpr unsigned kPinnedMapped = hipHostMallocMapped | hipHostMallocCoherent;

template <typename T>
hipError_t dev_alloc(T** p, size_t bytes) {
	void* q = nullptr;
	const hipError_t e = hipMalloc(&q, bytes);
	*p = static_cast<T*>(q);
	return e;
}
hipError_t dev_free(void* p) { return hipFree(p); }

// The scene's arrays in one device block, filled in one launch from mapped pinned staging
// (RTAMD_UPLOAD 1): one allocation, no copy engine (its first use in a process costs ~16 ms
// and every pageable hipMemcpy ~3 ms; profiles/round4 CLI traces).  add() records where each
// array goes; commit() allocates, stages, copies and sets the device pointers.
struct UploadBatch {
	struct Item {
		const void* host;
		size_t bytes;
		std::function<void(const char*)> set;  // stores the array's device address
		size_t offset;
	};
	std::vector<Item> items;
	size_t total = 0;
	template <typename T>
	void add(const std::vector<T>& v, const T** dev) {
		*dev = nullptr;
		if (v.empty()) return;
		items.push_back({v.data(), v.size() * sizeof(T), [dev](const char* p) { *dev = reinterpret_cast<const T*>(p); }, total});
		total += (v.size() * sizeof(T) + 255) & ~size_t(255);
	}
	int commit(rt_scene* s) {
		if (total == 0) return RT_OK;
		void* block = nullptr;
		HIP_TRY(dev_alloc(&block, total));
		s->allocs.push_back(block);
		void* stage = nullptr;
		// coherent (fine-grained) by default (kPinnedMapped): the copy kernel's reads cannot hit
		// lines an XCD's L2 still holds from an earlier staging buffer at the same addresses
		HIP_TRY(hipHostMalloc(&stage, total, kPinnedMapped));
		void* stage_dev = nullptr;
		hipError_t e = hipHostGetDevicePointer(&stage_dev, stage, 0);
		std::memset(stage, 0, total);  // the padding between arrays too
		for (const Item& it : items) std::memcpy(static_cast<char*>(stage) + it.offset, it.host, it.bytes);
		if (e == hipSuccess) e = rtamd::launch_copy16(block, stage_dev, static_cast<int64_t>(total / 16), s->stream);
		if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
		(void)hipHostFree(stage);
		if (e != hipSuccess) return fail(RT_ERR_DEVICE, std::string("scene upload: ") + hipGetErrorString(e));
		for (const Item& it : items) {
			it.set(static_cast<const char*>(block) + it.offset);
			s->info.device_bytes += static_cast<int64_t>(it.bytes);
		}
		return RT_OK;
	}
};


// Level buffers grow on demand during a host-driven trace (one level of lookahead: up to
// four times the rays a level ends up holding), are cut back to what the lane's launch plans
// need once the call is done (right_size_levels), and are kept for later renders.
// bytes of one level buffer of `n` ray slots: 21 double arrays, 4 int32 arrays, two flag
// arrays, n x lights shadow verdicts and the level's counts, each 256-B aligned
// Clears device memory and waits for it.  hipMemset is asynchronous for device memory and
// runs on the null stream, which the library's non-blocking streams do not wait for: a
// kernel queued on a lane's stream right after it could otherwise run first.
hipError_t clear_device(void* p, size_t bytes) {
	hipError_t e = hipMemsetAsync(p, 0, bytes, nullptr);
	if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
	return e;
}

int64_t level_block_bytes(const rt_scene* s, int64_t n) {
	const int64_t nl = std::max(1, s->ds.n_nonambient);
	auto align = [](int64_t b) { return (b + 255) & ~int64_t(255); };
	return 18 * align(n * 8) + 4 * align(n * 4) + 2 * align(n) + align(n * nl) + 256;
}

constexpr int kBudgetMiss = 2;  // internal return code: RTAMD_LEVEL_BUDGET exceeded (render_jobs)

// (Re)allocates level `level` for `capacity` slots (at least 1024), larger or smaller than
// it was; kBudgetMiss when the lanes' level buffers would exceed RTAMD_LEVEL_BUDGET
int alloc_level(rt_scene* s, Lane& ln, size_t level, int64_t capacity) {
	LevelBuffers& L = ln.levels[level];
	capacity = std::max<int64_t>(capacity, 1024);
	const int64_t n = capacity;
	const int64_t nl = std::max(1, s->ds.n_nonambient);
	auto align = [](int64_t b) { return (b + 255) & ~int64_t(255); };
	const int64_t bytes = level_block_bytes(s, n);
	if (s->level_budget > 0 && s->info.level_bytes - L.bytes + bytes > s->level_budget) return kBudgetMiss;
	if (L.block) {
		HIP_TRY(hipDeviceSynchronize());
		HIP_TRY(dev_free(L.block));
		L.block = nullptr;
		s->info.level_bytes -= L.bytes;
		L.bytes = 0;
	}
	HIP_TRY(dev_alloc(&L.block, bytes));
	L.bytes = bytes;
	s->info.level_bytes += bytes;
	s->info.level_bytes_peak = std::max(s->info.level_bytes_peak, s->info.level_bytes);
	char* p = static_cast<char*>(L.block);
	auto take = [&](int64_t b) {
		char* r = p;
		p += align(b);
		return r;
	};
	double** d[18] = {&L.lv.ox,  &L.lv.oy,  &L.lv.oz,  &L.lv.dx,  &L.lv.dy,  &L.lv.dz,
	                  &L.lv.hpx, &L.lv.hpy, &L.lv.hpz, &L.lv.hnx, &L.lv.hny, &L.lv.hnz,
	                  &L.lv.hdx, &L.lv.hdy, &L.lv.hdz, &L.lv.cr,  &L.lv.cg,  &L.lv.cb};
	for (double** q : d) *q = reinterpret_cast<double*>(take(n * 8));
	L.lv.hgeom = reinterpret_cast<int32_t*>(take(n * 4));
	L.lv.hit_list = reinterpret_cast<int32_t*>(take(n * 4));
	L.lv.child_refr = reinterpret_cast<int32_t*>(take(n * 4));
	L.lv.child_refl = reinterpret_cast<int32_t*>(take(n * 4));
	L.lv.inside = reinterpret_cast<uint8_t*>(take(n));
	L.lv.hinside = reinterpret_cast<uint8_t*>(take(n));
	L.lv.occl = reinterpret_cast<uint8_t*>(take(n * nl));
	L.lv.counts = reinterpret_cast<int32_t*>(take(256));
	HIP_TRY(clear_device(L.lv.counts, 4 * sizeof(int32_t)));
	L.lv.capacity = capacity;
	return RT_OK;
}

int ensure_level(rt_scene* s, Lane& ln, size_t level, int64_t capacity) {
	if (ln.levels.size() <= level) ln.levels.resize(level + 1);
	if (ln.levels[level].lv.capacity >= capacity) return RT_OK;
	ln.grew = true;
	return alloc_level(s, ln, level, capacity);
}

// Level `level` exists and its RayLevel record is in the pinned array (the record of an
// earlier level never changes while copies of it may be in flight).
int ensure_level_record(rt_scene* s, Lane& ln, size_t level, int64_t capacity) {
	if (level + 1 > ln.levels_cap) {
		clear_plans(ln);
		HIP_TRY(hipDeviceSynchronize());
		const size_t cap = std::max<size_t>(16, 2 * (level + 1));
		rtamd::RayLevel *pin = nullptr, *dev = nullptr;
		int32_t* counts = nullptr;
		HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&pin), cap * sizeof(rtamd::RayLevel), kPinned));
		HIP_TRY(dev_alloc((&dev), cap * sizeof(rtamd::RayLevel)));
		HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&counts), 2 * cap * sizeof(int32_t), kPinned));
		std::memset(pin, 0, cap * sizeof(rtamd::RayLevel));
		if (ln.levels_pinned) {
			std::memcpy(pin, ln.levels_pinned, ln.levels_cap * sizeof(rtamd::RayLevel));
			std::memcpy(counts, ln.counts_host, 2 * ln.levels_cap * sizeof(int32_t));
			(void)hipHostFree(ln.levels_pinned);
			(void)hipHostFree(ln.counts_host);
			(void)dev_free(ln.levels_dev);
		}
		ln.counts_host = counts;
		// on the lane's stream, ahead of the per-level record updates queued there: a hipMemcpy
		// (the null stream, another hardware queue) could land after such an update and put a
		// zeroed record back
		HIP_TRY(hipMemcpyAsync(dev, pin, cap * sizeof(rtamd::RayLevel), hipMemcpyHostToDevice, ln.stream));
		ln.levels_pinned = pin;
		ln.levels_dev = dev;
		ln.levels_cap = cap;
	}
	int rc = ensure_level(s, ln, level, capacity);
	if (rc) return rc;
	if (std::memcmp(&ln.levels_pinned[level], &ln.levels[level].lv, sizeof(rtamd::RayLevel)) != 0) {
		// new buffers: the device copy is updated in stream order, ahead of any kernel of
		// this level (the entry itself changes only after a device-wide synchronisation)
		ln.levels_pinned[level] = ln.levels[level].lv;
		HIP_TRY(hipMemcpyAsync(ln.levels_dev + level, ln.levels_pinned + level, sizeof(rtamd::RayLevel),
		                       hipMemcpyHostToDevice, ln.stream));
	}
	return RT_OK;
}

int ensure_events(Lane& ln, size_t level) {
	while (ln.level_events.size() <= level) {
		std::array<hipEvent_t, 6> ev{};
		for (hipEvent_t& e : ev) HIP_TRY(hipEventCreate(&e));
		ln.level_events.push_back(ev);
	}
	return RT_OK;
}

// shading stream k of a lane, made at its first use: a stream costs 7-11 ms to create
// (profiles/round4: host traces), and a render of one traced level uses one of the four
hipStream_t shade_stream(Lane& ln, int k) {
	if (ln.minimal) return ln.stream;
	if (!ln.shade[k]) {
		if (hipStreamCreateWithPriority(&ln.shade[k], hipStreamNonBlocking, ln.prio_low) != hipSuccess) {
			ln.shade[k] = nullptr;
			return nullptr;
		}
		roctxNameHipStream("rtamd lane: shading", ln.shade[k]);
	}
	return ln.shade[k];
}

int lane_create(Lane& ln, int prio_low, int prio_high) {
	HIP_TRY(hipStreamCreateWithPriority(&ln.stream, hipStreamNonBlocking, prio_high));
	HIP_TRY(hipStreamCreateWithPriority(&ln.readback, hipStreamNonBlocking, prio_high));
	ln.prio_low = prio_low;  // the shading streams are made at their first use (shade_stream)
	HIP_TRY(hipEventCreateWithFlags(&ln.chunk_done, hipEventDisableTiming));
	roctxNameHipStream("rtamd lane: k_closest chain", ln.stream);
	roctxNameHipStream("rtamd lane: level counts read-back", ln.readback);
	return RT_OK;
}

void lane_destroy(Lane& ln) {
	clear_plans(ln);
	for (auto& L : ln.levels)
		if (L.block) (void)dev_free(L.block);
	if (ln.levels_pinned) (void)hipHostFree(ln.levels_pinned);
	if (ln.levels_dev) (void)dev_free(ln.levels_dev);
	if (ln.counts_host) (void)hipHostFree(ln.counts_host);
	for (auto& ev : ln.level_events)
		for (hipEvent_t e : ev) (void)hipEventDestroy(e);
	if (ln.chunk_done) (void)hipEventDestroy(ln.chunk_done);
	if (ln.minimal) return;  // the streams are the scene's
	for (hipStream_t q : ln.shade)
		if (q) (void)hipStreamDestroy(q);
	if (ln.readback) (void)hipStreamDestroy(ln.readback);
	if (ln.stream) (void)hipStreamDestroy(ln.stream);
}

// a minimal lane (the scene's first call) gets streams of its own; its buffers, events and
// plans stay (nothing of them is bound to a stream)
int upgrade_lane(Lane& ln, int prio_low, int prio_high) {
	if (!ln.minimal) return RT_OK;
	HIP_TRY(hipStreamSynchronize(ln.stream));
	ln.stream = ln.readback = nullptr;
	ln.minimal = false;
	HIP_TRY(hipStreamCreateWithPriority(&ln.stream, hipStreamNonBlocking, prio_high));
	HIP_TRY(hipStreamCreateWithPriority(&ln.readback, hipStreamNonBlocking, prio_high));
	ln.prio_low = prio_low;
	return RT_OK;
}

// image row of the selected-row ordinal q (rt_render_params: blocks of row_block rows)
int32_t selected_row(const rt_render_params* p, int64_t q) {
	const int64_t B = std::max(1, p->row_block);
	return static_cast<int32_t>(p->row_begin + (q / B) * p->row_step * B + q % B);
}

// The render of one rt_render_device / rt_render_batch_device call: chunks of rows of
// its jobs handed to lanes, each lane a small state machine advanced by the host as its
// events complete.
struct Render {
	rt_scene* s;
	int direct_levels = 2;  // rt_scene::direct_levels_single or _batch, for this call
	int deep_split = 0;     // rt_scene::deep_split_single or _batch, for this call
	int64_t light_major_below = 0;  // rt_scene::light_major_below_single or _batch, for this call
	rt_counters cnt{};
	float kernel_ms = 0.f;
	Progress* progress = nullptr;
	hipStream_t caller = nullptr;
	bool fork_recorded = false;
	bool direct_ok = false;    // the call is one chunk on one lane: it may run on the caller's stream
	bool stats_fused = false;  // the call's last kernel finishes the statistics (no k_stats_finish)
	bool finished = false;     // the plan issued last attached the statistics finish to a launch
	static constexpr int64_t kFinishBlocks = int64_t(1) << 30;

	// the caller's prior work before any of this lane's (the fork), once per call; a chunk
	// on the caller's own stream needs none
	int fork(Lane& ln) {
		if (ln.forked) return RT_OK;
		if (!fork_recorded) HIP_TRY(hipEventRecord(s->fork_event, caller));
		fork_recorded = true;
		HIP_TRY(hipStreamWaitEvent(ln.stream, s->fork_event, 0));
		ln.forked = true;
		return RT_OK;
	}

	// a replayed chunk of this plan is issued on one stream (issue_plan)
	bool one_stream(const Lane& ln, const Plan& pl) const {
		return ln.n0 <= s->one_stream_pixels || pl.n_levels == 1;
	}
	// its levels are fused launches (k_fused): shaded renders of at most 64 shadow lights,
	// without the work counters
	// (rt_scene::fused_min_pixels: not a small chunk of a mesh scene)
	bool fusable(const Lane& ln) const {
		return s->fused && !ln.io && !s->ds.work_stats && s->ds.n_nonambient <= rtamd::kMaxShadowLights &&
		       (s->ds.n_meshes == 0 || ln.n0 >= s->fused_min_pixels);
	}

	// k_closest of level L, then the read-back of its counts.  n: the level's ray count, or
	// with n_dev (the previous level's child counter) an upper bound: the level is queued
	// behind the previous one before the host knows its size (one level of lookahead).
	int launch_closest_level(Lane& ln, int L, int64_t n, const int32_t* n_dev) {
		const int remaining = ln.depth - L;
		int rc;
		// children of this level: at most 2 per ray
		if (remaining > 0 && (rc = ensure_level_record(s, ln, L + 1, 2 * n))) return rc;
		if ((rc = ensure_events(ln, L))) return rc;
		const auto& ev = ln.level_events[L];
		const rtamd::RayLevel& cur = ln.levels[L].lv;
		if (s->fail_after >= 0 && s->fail_after-- == 0) return fail(RT_ERR_DEVICE, "injected failure (rt_debug_fail_after)");
		// counts start at zero: level 0's are cleared at allocation and by the previous
		// chunk's k_output, deeper ones by the previous level's k_closest
		HIP_TRY(hipEventRecord(ev[0], ln.stream));
		HIP_TRY(rtamd::launch_closest(s->ds, ln.fg, L, n, n_dev, remaining, ln.levels_dev, s->ctr, s->stats, ln.stream,
		                              s->packet_mask));
		cnt.stage_launches[0]++;
		HIP_TRY(hipEventRecord(ev[1], ln.stream));
		HIP_TRY(hipStreamWaitEvent(ln.readback, ev[1], 0));
		HIP_TRY(hipMemcpyAsync(ln.counts_host + 2 * L, cur.counts, 2 * sizeof(int32_t), hipMemcpyDeviceToHost,
		                       ln.readback));
		HIP_TRY(hipEventRecord(ev[5], ln.readback));
		return RT_OK;
	}

	// k_shadow + k_shade of the levels `lv` (their k_closest done) on stream q
	int launch_shading(Lane& ln, const std::vector<std::pair<int, int64_t>>& lv, hipStream_t q) {
		rtamd::ShadeBatch b{};
		const int64_t nl = s->ds.n_nonambient;
		auto wave_up = [](int64_t x) { return (x + 63) & ~int64_t(63); };
		int64_t so = 0, ho = 0;
		b.n = static_cast<int32_t>(lv.size());
		int64_t hits = 0;
		for (const auto& l : lv) hits += l.second;
		b.all_lights = s->all_lights_for(lv.front().first, hits, light_major_below);
		for (int k = 0; k < b.n; k++) {
			b.level[k] = lv[k].first;
			b.nh[k] = lv[k].second;
			b.shadow_begin[k] = so;
			b.shade_begin[k] = ho;
			so += (b.all_lights ? 1 : nl) * wave_up(lv[k].second);  // every light's items start on a wave boundary
			ho += wave_up(lv[k].second);
		}
		b.shadow_begin[b.n] = so;
		b.shade_begin[b.n] = ho;
		if (s->serial) q = ln.stream;
		const int first = lv.front().first, last = lv.back().first;
		const auto& ev = ln.level_events[first];
		HIP_TRY(hipStreamWaitEvent(q, ln.level_events[last][1], 0));
		HIP_TRY(hipEventRecord(ev[2], q));
		// one level traced all-lights-per-lane: k_shadow computes the Phong terms itself
		b.fused = nl > 0 && nl <= 64 && rtamd::shadow_can_fuse(s->ds, b, s->packet_mask, true);
		HIP_TRY(rtamd::launch_shadow(s->ds, b, ln.levels_dev, s->ctr, s->stats, q, s->packet_mask));
		if (nl > 0) cnt.stage_launches[1]++;
		HIP_TRY(hipEventRecord(ev[3], q));
		if (!b.fused) {
			HIP_TRY(rtamd::launch_shade(s->ds, b, ln.levels_dev, s->ctr, q));
			cnt.stage_launches[2]++;
		}
		HIP_TRY(hipEventRecord(ev[4], q));
		ln.shaded.push_back(first);
		return RT_OK;
	}

	PlanKey key_of(const Lane& ln) const {
		PlanKey k{};
		k.width = ln.fg.width;
		k.height = ln.fg.height;
		k.depth = ln.depth;
		k.io = ln.io;
		k.direct_levels = direct_levels;
		k.deep_split = deep_split;
		k.light_major_below = light_major_below;
		k.work_stats = s->ds.work_stats;
		k.n0 = ln.n0;
		k.rows_hash = ln.rows_hash;
		return k;
	}

	Plan* find_plan(Lane& ln, const PlanKey& k) const {
		if (!s->plans || s->serial) return nullptr;
		for (Plan& p : ln.plans)
			if (p.key == k) return &p;
		return nullptr;
	}

	// shading of the levels `lv` with their hit counts read on the device (plans; the grid
	// from the plan's traced hits)
	int launch_shading_dev(Lane& ln, const std::vector<int>& lv, hipStream_t q, Plan& pl) {
		rtamd::ShadeBatch b{};
		const int64_t nl = s->ds.n_nonambient;
		auto wave_up = [](int64_t x) { return (x + 63) & ~int64_t(63); };
		int64_t so = 0, ho = 0;  // upper bounds (the levels' capacities): grid sizes only
		b.n = static_cast<int32_t>(lv.size());
		b.dev_counts = 1;
		int64_t hits = 0;
		for (int L : lv) hits += pl.hits[L];
		b.all_lights = s->all_lights_for(lv.front(), hits, light_major_below);
		for (int k = 0; k < b.n; k++) {
			const rtamd::RayLevel& L = ln.levels[lv[k]].lv;
			b.level[k] = lv[k];
			b.nh_dev[k] = L.counts;
			so += (b.all_lights ? 1 : nl) * wave_up(pl.hits[lv[k]]);
			ho += wave_up(pl.hits[lv[k]]);
		}
		// grid sizes from the traced chunk's hits (at least one block: the kernels stride)
		b.shadow_begin[b.n] = std::max<int64_t>(so, 64);
		b.shade_begin[b.n] = std::max<int64_t>(ho, 64);
		b.fused = nl > 0 && nl <= 64 && rtamd::shadow_can_fuse(s->ds, b, s->packet_mask, true);
		HIP_TRY(rtamd::launch_shadow(s->ds, b, ln.levels_dev, s->ctr, s->stats, q, s->packet_mask));
		if (nl > 0) pl.launches[1]++;
		if (!b.fused) {
			HIP_TRY(rtamd::launch_shade(s->ds, b, ln.levels_dev, s->ctr, q));
			pl.launches[2]++;
		}
		return RT_OK;
	}

	// The launch sequence of a planned chunk with device-read level sizes, issued at once
	// (no host round trip between levels): the same streams and dependencies as the
	// host-driven schedule: the chain on ln.stream, direct levels' shading on shade[L % 3]
	// as soon as their k_closest is done, the deep levels in batches on shade[3] after the
	// chain, then reductions and the output.
	int issue_plan(Lane& ln, Plan& pl, hipStream_t st, bool finish) {
		const int nlev = pl.n_levels, depth = ln.depth;
		int rc = RT_OK;
		if ((rc = ensure_events(ln, nlev))) return rc;
		// event slots as in the host-driven schedule: [L][1] k_closest(L) done, [L][4] the
		// shading launch starting at level L done
		auto ev = [&](int L, int k) -> hipEvent_t { return ln.level_events[L][k]; };
		auto step = [&](hipError_t e) {
			if (e != hipSuccess && rc == RT_OK) rc = fail(RT_ERR_DEVICE, std::string("planned launch: ") + hipGetErrorString(e));
		};
		int launches[3] = {0, 0, 0};
		std::vector<std::pair<hipEvent_t, hipStream_t>> joins;  // side shading done, on its stream
		Plan scratch = pl;
		// A small chunk (a small frame, or a GPU's row share of one) is issued on ONE stream:
		// the chain, then every level's shading in one batch, then the reductions.  Waits across
		// queues cost 6-19 us each between kernels of a few us (profiles/round3 timelines); a
		// large chunk's overlap of shading and tracing is worth them, a small one's is not.
		// A plan of one traced level (no bounce: bdepth 0, or nothing reflective was hit) has
		// nothing to overlap either: C2a 0.185 -> 0.179, C2b 0.334 -> 0.327, C4 0.357 -> 0.355 ms,
		// C4 2-way share 0.302 -> 0.290 ms (round 3)
		// the statistics finish inside the last launch (finish: a call of this one chunk): every
		// block counts itself done (per-XCD counters, trace.hip last_block_finish)
		rtamd::FusedOut fin{};
		fin.summary = s->summary_mapped;
		fin.done = s->fin_done;
		finished = false;
		auto finish_on = [&](int64_t threads, int block) {
			const bool on = finish && (threads + block - 1) / block <= kFinishBlocks;  // (grid sizes: unsigned)
			finished = finished || on;
			return on;
		};
		const int64_t tiles = ((ln.fg.width + 7) / 8) * ((ln.n0 / ln.fg.width + 7) / 8) * 64;  // level-0 packet threads
		if (one_stream(ln, pl) && fusable(ln)) {
			// every level in one launch (k_fused), level after level; a plan of one level writes
			// the pixels from there, else the reductions and k_output follow
			for (int L = 0; L < nlev && rc == RT_OK; L++) {
				const int remaining = depth - L;
				const int64_t bound = L == 0 ? ln.n0 : std::max<int64_t>(pl.level_n[L], 1);
				rtamd::FusedOut fo{};
				if (nlev == 1) {
					fo = finish_on((s->packet_mask & rtamd::kPacketClosest0) ? tiles : ln.n0, 128) ? fin : rtamd::FusedOut{};
					fo.final = 1;
				}
				step(rtamd::launch_fused(s->ds, ln.fg, L, bound, L == 0 ? nullptr : ln.levels[L - 1].lv.counts + 1,
				                         remaining, ln.levels_dev, s->ctr, s->stats, st, s->packet_mask,
				                         L == nlev - 1 && remaining > 0, fo));
				launches[0]++;
			}
			if (nlev > 1 && rc == RT_OK)
				step(reduce_and_output(ln, nlev, pl.level_n, true, st, finish_on(ln.n0, 256) ? &fin : nullptr));
			for (int k = 0; k < 3; k++) pl.launches[k] = launches[k];
			return rc;
		}
		if (one_stream(ln, pl)) {
			for (int L = 0; L < nlev && rc == RT_OK; L++) {
				const int remaining = depth - L;
				const int64_t bound = L == 0 ? ln.n0 : std::max<int64_t>(pl.level_n[L], 1);
				step(rtamd::launch_closest(s->ds, ln.fg, L, bound, L == 0 ? nullptr : ln.levels[L - 1].lv.counts + 1,
				                           remaining, ln.levels_dev, s->ctr, s->stats, st, s->packet_mask,
				                           L == nlev - 1 && remaining > 0));
				launches[0]++;
			}
			// levels 0 and 1 alone (their packet forms), the rest together
			for (int k = 0, e; k < nlev && rc == RT_OK; k = e) {
				e = k < 2 ? k + 1 : std::min(nlev, k + rtamd::kMaxBatch);
				std::vector<int> lv;
				for (int L = k; L < e; L++) lv.push_back(L);
				scratch.launches[1] = scratch.launches[2] = 0;
				rc = launch_shading_dev(ln, lv, st, scratch);
				launches[1] += scratch.launches[1];
				launches[2] += scratch.launches[2];
			}
		} else {
			for (int L = 0; L < nlev && rc == RT_OK; L++) {
				const int remaining = depth - L;
				const bool last = L == nlev - 1;
				const int64_t bound = L == 0 ? ln.n0 : std::max<int64_t>(pl.level_n[L], 1);
				// k_closest(L) done: only the side shading of a direct level waits on it; the
				// launch records it itself (no marker packet in the chain: ~7 us between two kernels)
				const bool waited = L < direct_levels && !last;
				hipEvent_t done = waited ? ev(L, 1) : nullptr;
				if (waited && !done) step(hipErrorOutOfMemory);
				const bool by_launch = done != nullptr;
				step(rtamd::launch_closest(s->ds, ln.fg, L, bound, L == 0 ? nullptr : ln.levels[L - 1].lv.counts + 1,
				                           remaining, ln.levels_dev, s->ctr, s->stats, st, s->packet_mask,
				                           last && remaining > 0, by_launch ? done : nullptr));
				launches[0]++;
				if (done && !by_launch) step(hipEventRecord(done, st));
				// shading beside the chain only where a later level's tracing can overlap it: a
				// wait on a not yet signalled event of another queue costs tens of microseconds
				if (L < direct_levels && rc == RT_OK) {
					const bool side = L < nlev - 1;
					hipStream_t q = side ? shade_stream(ln, L % 3) : st;
					if (side && !q && !ln.minimal) step(hipErrorOutOfMemory);  // (the chain's own st may be the null stream)
					if (side) step(hipStreamWaitEvent(q, done, 0));
					scratch.launches[1] = scratch.launches[2] = 0;
					if (rc == RT_OK) rc = launch_shading_dev(ln, {L}, q, scratch);
					launches[1] += scratch.launches[1];
					launches[2] += scratch.launches[2];
					if (side) {
						hipEvent_t sh = ev(L, 4);
						step(sh ? hipEventRecord(sh, q) : hipErrorOutOfMemory);
						joins.push_back({sh, q});
					}
				}
			}
			// the deep levels after the chain, on its own stream (the reductions wait for them)
			if (rc == RT_OK && nlev > direct_levels) {
				hipStream_t q = st;
				std::vector<int> deep;
				for (int L = direct_levels; L < nlev; L++) deep.push_back(L);
				for (size_t k = 0, e; k < deep.size() && rc == RT_OK; k = e) {
					e = std::min(deep.size(), k + (static_cast<int>(k) < deep_split ? 1 : rtamd::kMaxBatch));
					scratch.launches[1] = scratch.launches[2] = 0;
					rc = launch_shading_dev(ln, std::vector<int>(deep.begin() + k, deep.begin() + e), q, scratch);
					launches[1] += scratch.launches[1];
					launches[2] += scratch.launches[2];
				}
			}
		}
		// the chain joins the side shading once: the last side stream waits for the others (off
		// the chain's path, long after they finished) and records again; each wait in the chain's
		// queue costs ~5 us
		if (joins.size() > 1 && rc == RT_OK) {
			const auto last_join = joins.back();
			for (size_t k = 0; k + 1 < joins.size() && rc == RT_OK; k++)
				if (joins[k].second != last_join.second) step(hipStreamWaitEvent(last_join.second, joins[k].first, 0));
			step(hipEventRecord(last_join.first, last_join.second));
			joins.assign(1, last_join);
		}
		for (const auto& j : joins)
			if (rc == RT_OK) step(hipStreamWaitEvent(st, j.first, 0));
		if (rc == RT_OK) step(reduce_and_output(ln, nlev, pl.level_n, true, st, finish_on(ln.n0, 256) ? &fin : nullptr));
		for (int k = 0; k < 3; k++) pl.launches[k] = launches[k];
		return rc;
	}

	// A plan for the chunk just traced host-driven (its shape: ln.fg, ln.n0, the job's
	// depth; its levels: ln.level_n), kept by the lane and shared with the others
	int build_plan(Lane& ln) {
		Plan pl;
		pl.key = key_of(ln);
		pl.n_levels = static_cast<int>(ln.level_n.size());
		pl.level_n = ln.level_n;
		for (int L = 0; L < pl.n_levels; L++) pl.hits.push_back(ln.counts_host[2 * L]);
		for (int L = 0; L < pl.n_levels; L++) pl.capacity.push_back(std::max<int64_t>(pl.level_n[L], 1));
		if (s->plan_truncate && pl.n_levels > 1) pl.n_levels--;  // test hook: a plan that must miss
		keep_plan(ln, pl);
		bool known = false;
		for (const Plan& q : s->shared_plans) known = known || q.key == pl.key;
		if (!known) {
			if (s->shared_plans.size() >= kMaxPlans) s->shared_plans.erase(s->shared_plans.begin());
			s->shared_plans.push_back(pl);
		}
		return RT_OK;
	}

	// a lane keeps its kMaxPlans most recent plans (called while it replays none)
	static void keep_plan(Lane& ln, const Plan& pl) {
		if (ln.plans.size() >= kMaxPlans) ln.plans.erase(ln.plans.begin());
		ln.plans.push_back(pl);
	}

	// A plan of this chunk's shape built by another lane, made this lane's own: its level
	// buffers grown to the plan's capacities
	Plan* adopt_plan(Lane& ln, const PlanKey& k, int& rc) {
		rc = RT_OK;
		if (!s->plans || s->serial) return nullptr;
		for (const Plan& q : s->shared_plans) {
			if (!(q.key == k)) continue;
			// (and the level past the last: its k_closest clears that level's counts)
			for (int L = 0; L <= q.n_levels && rc == RT_OK; L++)
				rc = ensure_level_record(s, ln, L, L < q.n_levels ? q.capacity[L] : 1024);
			if (rc) return nullptr;
			keep_plan(ln, q);
			return &ln.plans.back();
		}
		return nullptr;
	}

	// The chunk's colours reduced bottom-up, two levels per launch (rtamd::reduce_steps), level
	// 0's reduction in the output launch.  device_counts: the level sizes are bounds and the
	// launches read the levels' ray counts on the device (replayed plans)
	hipError_t reduce_and_output(Lane& ln, int nlev, const std::vector<int64_t>& level_n, bool device_counts,
	                             hipStream_t st, const rtamd::FusedOut* fin) {
		std::vector<rtamd::ReduceStep> steps(std::max(1, nlev));
		const int n = rtamd::reduce_steps(nlev, steps.data());
		for (int k = 0; k < n; k++) {
			const int l = steps[k].level, m = steps[k].levels;
			const rtamd::RayLevel* low = m == 2 ? &ln.levels[l + 2].lv : nullptr;
			const hipError_t e =
			    l > 0 ? rtamd::launch_reduce_level(s->ds, device_counts ? std::max<int64_t>(level_n[l], 1) : level_n[l],
			                                       device_counts ? ln.levels[l - 1].lv.counts + 1 : nullptr, ln.levels[l].lv,
			                                       ln.levels[l + 1].lv, low, st)
			          : rtamd::launch_output(s->ds, ln.n0, ln.fg, ln.levels[0].lv, m >= 1 ? &ln.levels[1].lv : nullptr, low,
			                                 s->stats, st, s->ctr, fin);
			if (e != hipSuccess) return e;
		}
		return hipSuccess;
	}

	// The chunk's rows as by-value descriptors (FrameGeometry::seg, one per piece: the kernels
	// compute each row's image row and output address from them, trace.hip chunk_row), and the
	// hash of its image rows for the plan key.  plan_chunks never packs more than
	// kMaxRowSegments pieces into a chunk.
	int describe_rows(Lane& ln, const std::vector<Segment>& segs, int64_t n_rows) {
		if (segs.empty() || segs.size() > static_cast<size_t>(rtamd::kMaxRowSegments))
			return fail(RT_ERR_DEVICE, "internal: a chunk of " + std::to_string(segs.size()) + " row segments");
		rtamd::FrameGeometry& fg = ln.fg;
		const Job& first = *segs.front().job;
		fg = rtamd::FrameGeometry{};
		fg.width = first.p->width;
		fg.height = first.p->height;
		fg.intersection_only = first.io;
		fg.n_rows = static_cast<int32_t>(n_rows);
		fg.n_segs = static_cast<int32_t>(segs.size());
		uint64_t h = 1469598103934665603ull;
		int64_t q = 0;
		for (size_t k = 0; k < segs.size(); k++) {
			const Segment& sg = segs[k];
			const Job& job = *sg.job;
			const rt_render_params* p = job.p;
			rtamd::RowSegment& d = fg.seg[k];
			d.out = job.out_rgb_dev;
			d.out8 = job.out_rgb8_dev;
			d.q0 = static_cast<int32_t>(q);
			d.ord0 = static_cast<int32_t>(sg.r0);
			d.ord_end = static_cast<int32_t>(job.n_rows);
			d.row_begin = p->row_begin;
			d.row_block = std::max(1, p->row_block);
			d.row_span = p->row_step * d.row_block;
			for (int64_t r = 0; r < sg.rows; r++) h = (h ^ static_cast<uint32_t>(selected_row(p, sg.r0 + r))) * 1099511628211ull;
			q += sg.rows;
		}
		ln.rows_hash = h;
		if (s->corrupt_rows) {  // test hook (rt_debug_corrupt_rows): rows no frame has
			fg.seg[0].row_begin += fg.height;
			s->corrupt_rows = 0;
		}
		return RT_OK;
	}

	// a chunk: rows of one or several jobs of equal width, height, depth and io (render_jobs)
	int start_chunk(Lane& ln, const std::vector<Segment>& segs) {
		const Job& first = *segs.front().job;
		int64_t n_rows = 0;
		for (const Segment& sg : segs) n_rows += sg.rows;
		ln.segs = segs;
		ln.depth = first.depth;
		ln.io = first.io;
		ln.n0 = n_rows * first.W;
		int rc = describe_rows(ln, segs, n_rows);
		if (rc) return rc;
		ln.level = 0;
		ln.level_n.assign(1, ln.n0);
		ln.shaded.clear();
		ln.deferred.clear();
		ln.planned = nullptr;
		Plan* pl = find_plan(ln, key_of(ln));
		// the call's only chunk, replaying a plan of this lane's own: its chain runs on the
		// caller's stream (no fork, no join; side streams wait on its events as before);
		// otherwise on the lane's streams after the fork
		ln.direct = direct_ok && pl;
		const hipStream_t st = ln.direct ? caller : ln.stream;
		if (!ln.direct && (rc = fork(ln))) return rc;
		if (!pl && (pl = adopt_plan(ln, key_of(ln), rc), rc)) return rc;
		if (pl) {
			if (s->fail_after >= 0 && s->fail_after-- == 0) return fail(RT_ERR_DEVICE, "injected failure (rt_debug_fail_after)");
			// the call's only chunk finishes the statistics in its last kernel (pinned summary)
			const bool finish = direct_ok && s->summary_mapped;
			if ((rc = issue_plan(ln, *pl, st, finish))) return rc;
			stats_fused = stats_fused || (finish && finished);
			HIP_TRY(hipEventRecord(ln.chunk_done, st));
			ln.planned = pl;
			ln.phase = Lane::FINISHING;
			return RT_OK;
		}
		ln.phase = Lane::TRACING;
		rc = ensure_level_record(s, ln, 0, ln.n0);
		if (!rc) rc = launch_closest_level(ln, 0, ln.n0, nullptr);
		if (!rc && ln.depth >= 1) rc = launch_closest_level(ln, 1, 2 * ln.n0, ln.levels[0].lv.counts + 1);
		return rc;
	}

	// counts of the lane's level are on the host: launch the next level (the critical
	// path) first, then the shading of this one, or finish the chunk.  A device
	// MathException is reported after the render (the reference aborts; the GPU merely
	// finishes the chunk).
	int on_counts(Lane& ln) {
		const int depth = ln.depth;
		const int L = ln.level;
		const int64_t nh = ln.counts_host[2 * L], nn = ln.counts_host[2 * L + 1];
		int rc;
		// k_closest(L+1) is already queued; queue k_closest(L+2) behind it
		const bool more = depth - L > 0 && nn > 0;
		if (more) {
			ln.level_n.push_back(nn);
			ln.level++;
			if (L + 2 <= depth &&
			    (rc = launch_closest_level(ln, L + 2, 2 * nn, ln.levels[L + 1].lv.counts + 1)))
				return rc;
		}
		if (nh > 0) {
			if (L < direct_levels) {  // big level: shade now, concurrent with k_closest(L+1)
				hipStream_t q = shade_stream(ln, L % 3);
				if (!q && !ln.minimal) return fail(RT_ERR_DEVICE, "shading stream creation failed");
				if ((rc = launch_shading(ln, {{L, nh}}, q))) return rc;
			} else {
				ln.deferred.push_back({L, nh});
			}
		}
		if (more) return RT_OK;
		for (size_t k = 0, e; k < ln.deferred.size(); k = e) {
			e = std::min(ln.deferred.size(), k + (static_cast<int>(k) < deep_split ? 1 : rtamd::kMaxBatch));
			hipStream_t q = shade_stream(ln, 3);
			if (!q && !ln.minimal) return fail(RT_ERR_DEVICE, "shading stream creation failed");
			if ((rc = launch_shading(ln, {ln.deferred.begin() + k, ln.deferred.begin() + e}, q))) return rc;
		}
		for (int first : ln.shaded) HIP_TRY(hipStreamWaitEvent(ln.stream, ln.level_events[first][4], 0));
		HIP_TRY(reduce_and_output(ln, static_cast<int>(ln.level_n.size()), ln.level_n, false, ln.stream, nullptr));
		HIP_TRY(hipEventRecord(ln.chunk_done, ln.stream));
		ln.phase = Lane::FINISHING;
		return RT_OK;
	}

	// the chunk's work is complete: per-kernel device times (events are re-recorded by
	// the lane's next chunk)
	int on_done(Lane& ln) {
		if (ln.planned) {  // a replayed plan: no per-kernel events (its stage times are not measured)
			const Plan& pl = *ln.planned;
			for (int k = 0; k < 3; k++) cnt.stage_launches[k] += pl.launches[k];
			cnt.levels = std::max<int32_t>(cnt.levels, pl.n_levels);
			cnt.pixels += ln.n0;
			ln.planned = nullptr;
			ln.phase = Lane::IDLE;
			ln.segs.clear();
			if (progress) progress->done += ln.n0;
			return RT_OK;
		}
		if (ln.call_need.size() < ln.level_n.size()) ln.call_need.resize(ln.level_n.size(), 0);
		for (size_t L = 0; L < ln.level_n.size(); L++) ln.call_need[L] = std::max(ln.call_need[L], ln.level_n[L]);
		if (s->plans && !s->serial && !find_plan(ln, key_of(ln))) {
			const int rc = build_plan(ln);
			if (rc) return rc;
		}
		for (int L = 0; L < static_cast<int>(ln.level_n.size()); L++) {
			float ms = 0.f;
			HIP_TRY(hipEventElapsedTime(&ms, ln.level_events[L][0], ln.level_events[L][1]));
			cnt.stage_ms[0] += ms;
			kernel_ms += ms;
		}
		for (int first : ln.shaded) {
			const auto& ev = ln.level_events[first];
			for (int k = 0; k < 2; k++) {
				float ms = 0.f;
				HIP_TRY(hipEventElapsedTime(&ms, ev[2 + k], ev[3 + k]));
				cnt.stage_ms[1 + k] += ms;
				kernel_ms += ms;
			}
		}
		cnt.levels = std::max<int32_t>(cnt.levels, static_cast<int32_t>(ln.level_n.size()));
		cnt.pixels += ln.n0;
		ln.phase = Lane::IDLE;
		ln.segs.clear();
		if (progress) progress->done += ln.n0;
		return RT_OK;
	}
};

int64_t selected_rows(const rt_render_params* p) {
	if (p->row_step <= 0 || p->row_end <= p->row_begin) return 0;
	const int64_t B = std::max(1, p->row_block), span = (int64_t)p->row_step * B, len = p->row_end - p->row_begin;
	// whole periods of `span` rows hold B selected rows each; the last one min(B, rest)
	return (len / span) * B + std::min<int64_t>(B, len % span);
}

constexpr int kMaxLanes = 8;

// the scene has at least n lanes (each: streams, events; level buffers grow on use)
// minimal: a first lane may borrow the scene's stream (Lane::minimal)
int ensure_lanes(rt_scene* s, size_t n, bool minimal = false) {
	for (size_t k = 0; k < std::min(n, s->lanes.size()); k++)
		if (!minimal && s->lanes[k]->minimal) {
			const int rc = upgrade_lane(*s->lanes[k], s->prio_low, s->prio_high);
			if (rc) return rc;
		}
	while (s->lanes.size() < n) {
		std::unique_ptr<Lane> ln(new Lane());
		int rc;
		if (minimal && s->lanes.empty()) {
			ln->stream = ln->readback = s->stream;
			ln->minimal = true;
			rc = hipEventCreateWithFlags(&ln->chunk_done, hipEventDisableTiming) == hipSuccess
			         ? RT_OK
			         : fail(RT_ERR_DEVICE, "hipEventCreateWithFlags failed");
		} else {
			rc = lane_create(*ln, s->prio_low, s->prio_high);
		}
		if (rc) {
			lane_destroy(*ln);
			return rc;
		}
		s->lanes.push_back(std::move(ln));
	}
	return RT_OK;
}

int check_params(const rt_scene* s, const rt_render_params* p) {
	if (!s || !p) return fail(RT_ERR_ARG, "null scene or params");
	if (p->width <= 0 || p->height <= 0) return fail(RT_ERR_ARG, "Width and/or height must be positive.");
	if (p->bounce_depth < 0) return fail(RT_ERR_ARG, "Bounce depth must be non-negative.");
	// (row_begin >= row_end selects no row: a rank past the last row block of a partition)
	if (p->row_begin < 0 || p->row_end > p->height || p->row_step <= 0 || p->row_block < 0)
		return fail(RT_ERR_ARG, "bad row selection");
	return RT_OK;
}

// rt_scene_desc -> host scene (the reference's object model, scene.h:35-38): transforms
// from Eigen's column-major storage, faces verbatim, then the camera corners and lights
// transformed once (apply_scene_transforms) as the lazy caches of rtbase.h / lights.h would.
int scene_from_desc(const rt_scene_desc& d, rtamd::Scene& sc) {
	if (d.n_geometries < 0 || d.n_lights < 0) return fail(RT_ERR_ARG, "negative geometry or light count");
	if ((d.n_geometries > 0 && !d.geometries) || (d.n_lights > 0 && !d.lights))
		return fail(RT_ERR_ARG, "null geometry or light array");
	auto xf = [](const rt_xform_desc& x, rtamd::Affine& fwd, rtamd::Affine& inv, double& det) {
		fwd = rtamd::affine_from_eigen(x.fwd);
		if (x.derive) {  // Transformable::forwardTransform(xf): xf.inverse(), determinant()
			inv = rtamd::affine_inverse(fwd);
			det = rtamd::affine_det4(fwd);
		} else {
			inv = rtamd::affine_from_eigen(x.inv);
			det = x.det;
		}
	};
	sc = rtamd::Scene{};
	for (int32_t i = 0; i < d.n_geometries; i++) {
		const rt_geometry_desc& gd = d.geometries[i];
		if (gd.kind != RT_GEOM_SPHERE && gd.kind != RT_GEOM_MESH)
			return fail(RT_ERR_ARG, "geometry " + std::to_string(i) + ": unknown kind");
		rtamd::Geometry g{};
		g.kind = gd.kind == RT_GEOM_SPHERE ? rtamd::GEOM_SPHERE : rtamd::GEOM_MESH;
		xf(gd.xf, g.fwd, g.inv, g.det);
		const rt_material_desc& m = gd.material;
		for (int k = 0; k < 3; k++) {
			g.mat.ka[k] = m.ambient[k];
			g.mat.kd[k] = m.diffuse[k];
			g.mat.ks[k] = m.specular[k];
			g.mat.kr[k] = m.reflective[k];
			g.mat.kt[k] = m.translucency[k];
		}
		g.mat.ns = m.specular_coefficient;
		g.mat.ior = m.index_of_refractivity;
		if (g.kind == rtamd::GEOM_SPHERE) {
			std::memcpy(g.center, gd.center, sizeof(g.center));
			g.radius = gd.radius;
		} else {
			if (gd.n_faces < 0 || (gd.n_faces > 0 && !gd.faces))
				return fail(RT_ERR_ARG, "geometry " + std::to_string(i) + ": bad face array");
			g.face_begin = static_cast<int64_t>(sc.faces.size());
			g.face_count = gd.n_faces;
			for (int64_t f = 0; f < gd.n_faces; f++) {
				const rt_face_desc& fd = gd.faces[f];
				for (int k = 0; k < 3; k++)
					if (fd.points[k][3] != 1.0)  // the invariant Mesh::updateBoundingBox enforces (geometry.cpp:160-161)
						return fail(RT_ERR_ARG, "geometry " + std::to_string(i) + ": face point with w != 1");
				rtamd::Face hf;
				std::memcpy(&hf, &fd, sizeof(hf));
				sc.faces.push_back(hf);
			}
			std::memcpy(g.bb_min, gd.bbox_min, sizeof(g.bb_min));
			std::memcpy(g.bb_max, gd.bbox_max, sizeof(g.bb_max));
			g.box_valid = true;
		}
		sc.geoms.push_back(g);
	}
	for (int32_t i = 0; i < d.n_lights; i++) {
		const rt_light_desc& ld = d.lights[i];
		rtamd::Light l{};
		if (ld.kind == RT_LIGHT_POINT)
			l.kind = rtamd::LIGHT_POINT;
		else if (ld.kind == RT_LIGHT_DIRECTIONAL)
			l.kind = rtamd::LIGHT_DIRECTIONAL;
		else if (ld.kind == RT_LIGHT_AMBIENT)
			l.kind = rtamd::LIGHT_AMBIENT;
		else
			return fail(RT_ERR_ARG, "light " + std::to_string(i) + ": unknown kind");
		l.fwd = rtamd::affine_from_eigen(ld.xf.fwd);
		std::memcpy(l.color, ld.color, sizeof(l.color));
		std::memcpy(l.raw, ld.vec, sizeof(l.raw));
		l.falloff = ld.kind == RT_LIGHT_POINT ? ld.falloff : 0.0;
		sc.lights.push_back(l);
	}
	sc.has_camera = d.has_camera != 0;
	if (sc.has_camera) {
		sc.cam_fwd = rtamd::affine_from_eigen(d.camera.xf.fwd);
		const double* src[5] = {d.camera.eye, d.camera.lower_left, d.camera.lower_right, d.camera.upper_left,
		                        d.camera.upper_right};
		for (int k = 0; k < 5; k++) std::memcpy(sc.cam_raw[k], src[k], 4 * sizeof(double));
	}
	rtamd::apply_scene_transforms(sc);
	return RT_OK;
}

}  // namespace

extern "C" {

const char* rt_last_error(void) { return g_error.c_str(); }
int rt_abi_version(void) { return RTAMD_ABI_VERSION; }
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

int scene_create(const rtamd::Scene& scene, int device, rt_scene** out);

int rt_scene_create(const rt_builder* b, int device, rt_scene** out) {
	if (!b || !out) return fail(RT_ERR_ARG, "null builder or output");
	return scene_create(b->scene, device, out);
}

int rt_scene_create_desc(const rt_scene_desc* d, int device, rt_scene** out) {
	if (!d || !out) return fail(RT_ERR_ARG, "null descriptor or output");
	*out = nullptr;
	rtamd::Scene scene;
	const int rc = scene_from_desc(*d, scene);
	if (rc) return rc;
	return scene_create(scene, device, out);
}

int rt_builder_get_desc(const rt_builder* b, rt_scene_desc* out) {
	if (!b || !out) return fail(RT_ERR_ARG, "null builder or descriptor");
	rt_builder* mb = const_cast<rt_builder*>(b);  // the view arrays are builder-owned scratch
	const rtamd::Scene& sc = b->scene;
	std::memset(out, 0, sizeof(*out));
	auto xf = [](const rtamd::Affine& fwd, const rtamd::Affine* inv, double det, rt_xform_desc& x) {
		std::memset(&x, 0, sizeof(x));
		rtamd::affine_to_eigen(fwd, x.fwd);
		if (inv) {
			rtamd::affine_to_eigen(*inv, x.inv);
			x.det = det;
		} else {
			x.derive = 1;
		}
	};
	mb->desc_geoms.assign(sc.geoms.size(), rt_geometry_desc{});
	for (size_t i = 0; i < sc.geoms.size(); i++) {
		const rtamd::Geometry& g = sc.geoms[i];
		rt_geometry_desc& d = mb->desc_geoms[i];
		d.kind = g.kind == rtamd::GEOM_SPHERE ? RT_GEOM_SPHERE : RT_GEOM_MESH;
		xf(g.fwd, &g.inv, g.det, d.xf);
		const rtamd::Material& m = g.mat;
		for (int k = 0; k < 3; k++) {
			d.material.ambient[k] = m.ka[k];
			d.material.diffuse[k] = m.kd[k];
			d.material.specular[k] = m.ks[k];
			d.material.reflective[k] = m.kr[k];
			d.material.translucency[k] = m.kt[k];
		}
		d.material.specular_coefficient = m.ns;
		d.material.index_of_refractivity = m.ior;
		std::memcpy(d.center, g.center, sizeof(d.center));
		d.radius = g.radius;
		d.n_faces = g.face_count;
		d.faces = g.face_count ? reinterpret_cast<const rt_face_desc*>(&sc.faces[g.face_begin]) : nullptr;
		std::memcpy(d.bbox_min, g.bb_min, sizeof(d.bbox_min));
		std::memcpy(d.bbox_max, g.bb_max, sizeof(d.bbox_max));
	}
	mb->desc_lights.assign(sc.lights.size(), rt_light_desc{});
	for (size_t i = 0; i < sc.lights.size(); i++) {
		const rtamd::Light& l = sc.lights[i];
		rt_light_desc& d = mb->desc_lights[i];
		d.kind = l.kind == rtamd::LIGHT_POINT ? RT_LIGHT_POINT
		         : l.kind == rtamd::LIGHT_DIRECTIONAL ? RT_LIGHT_DIRECTIONAL : RT_LIGHT_AMBIENT;
		xf(l.fwd, nullptr, 0.0, d.xf);
		std::memcpy(d.color, l.color, sizeof(d.color));
		std::memcpy(d.vec, l.raw, sizeof(d.vec));
		d.falloff = l.falloff;
	}
	out->has_camera = sc.has_camera;
	out->n_geometries = static_cast<int32_t>(sc.geoms.size());
	out->n_lights = static_cast<int32_t>(sc.lights.size());
	if (sc.has_camera) {
		xf(sc.cam_fwd, nullptr, 0.0, out->camera.xf);
		double* dst[5] = {out->camera.eye, out->camera.lower_left, out->camera.lower_right, out->camera.upper_left,
		                  out->camera.upper_right};
		for (int k = 0; k < 5; k++) std::memcpy(dst[k], sc.cam_raw[k], 4 * sizeof(double));
	}
	out->geometries = mb->desc_geoms.empty() ? nullptr : mb->desc_geoms.data();
	out->lights = mb->desc_lights.empty() ? nullptr : mb->desc_lights.data();
	return RT_OK;
}

int rt_builder_set_desc(rt_builder* b, const rt_scene_desc* d) {
	if (!b || !d) return fail(RT_ERR_ARG, "null builder or descriptor");
	rtamd::Scene scene;
	const int rc = scene_from_desc(*d, scene);
	if (rc) return rc;
	b->scene = std::move(scene);
	return RT_OK;
}

int scene_create(const rtamd::Scene& scene, int device, rt_scene** out) {
	rtamd::MarkerRange mr("rtamd: scene LBVH build + upload");
	*out = nullptr;
	if (!scene.has_camera) return fail(RT_ERR_ARG, "At least one camera must be specified.");
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
		return fail(RT_ERR_DEVICE, "no HIP device available (the rtamd render path runs only on the GPU)");
	if (device < 0 || device >= ndev) return fail(RT_ERR_ARG, "bad device index");
	HIP_TRY(hipSetDevice(device));
	const double t_build = now_s();
	rtamd::FlatScene fs = rtamd::flatten_scene(scene);
	const double t_upload = now_s();
	std::unique_ptr<rt_scene> s(new rt_scene());
	s->device = device;
	// tuning knobs; lanes are created on first use
	if (const char* pm = std::getenv("RTAMD_PACKET_MASK")) s->packet_mask = std::atoi(pm);
	if (const char* dl = std::getenv("RTAMD_DIRECT_LEVELS"))
		s->direct_levels_single = s->direct_levels_two_lanes = s->direct_levels_batch = std::max(1, std::atoi(dl));
	if (const char* nl = std::getenv("RTAMD_LANES")) s->single_lanes = std::min(kMaxLanes, std::max(0, std::atoi(nl)));
	if (const char* bl = std::getenv("RTAMD_BATCH_LANES"))
		s->batch_lanes = std::min(kMaxLanes, std::max(1, std::atoi(bl)));
	if (const char* se = std::getenv("RTAMD_SERIAL")) s->serial = std::atoi(se);
	if (const char* al = std::getenv("RTAMD_SHADOW_ALL_LIGHTS")) s->shadow_all_lights = std::atoi(al);
	if (const char* lm = std::getenv("RTAMD_LIGHT_MAJOR_BELOW"))
		s->light_major_below_single = s->light_major_below_batch = std::atoll(lm);
	if (const char* os = std::getenv("RTAMD_ONE_STREAM_PIXELS")) s->one_stream_pixels = std::atoll(os);
	if (const char* fu = std::getenv("RTAMD_FUSED")) s->fused = std::atoi(fu);
	if (const char* fm = std::getenv("RTAMD_FUSED_MIN_PIXELS")) s->fused_min_pixels = std::atoll(fm);
	if (const char* pt = std::getenv("RTAMD_PLAN_TRUNCATE")) s->plan_truncate = std::atoi(pt);
	if (const char* bc = std::getenv("RTAMD_BATCH_CHUNK")) s->batch_chunk_pixels = std::max<int64_t>(1, std::atoll(bc));
	if (const char* lb = std::getenv("RTAMD_LEVEL_BUDGET")) s->level_budget = std::max<int64_t>(0, std::atoll(lb));
	s->info.level_budget = s->level_budget;
	HIP_TRY(hipDeviceGetStreamPriorityRange(&s->prio_low, &s->prio_high));
	// The scene's own non-blocking stream (work issued without a caller stream), made here: on
	// the null stream until the second call, C3's later single frames took 1.281 instead of
	// 1.214 ms (round 4, profiles/round4/ab/latency_scene_stream*.txt)
	HIP_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
	HIP_TRY(hipEventCreateWithFlags(&s->fork_event, hipEventDisableTiming));
	int rc;
	UploadBatch ub;
	std::vector<rtamd::DCamera> cam(1, fs.camera);
	std::vector<int32_t> shadow_light;  // j-th non-ambient light -> light index (any number of lights, as scene.cpp:77-108)
	for (size_t li = 0; li < fs.lights.size(); li++)
		if (fs.lights[li].kind != rtamd::LIGHT_AMBIENT) shadow_light.push_back(static_cast<int32_t>(li));
	ub.add(fs.geoms, &s->ds.geoms);
	ub.add(fs.materials, &s->ds.mats);
	ub.add(fs.lights, &s->ds.lights);
	ub.add(fs.face_geo, &s->ds.fgeo);
	ub.add(fs.face_nrm, &s->ds.fnrm);
	ub.add(fs.nodes, &s->ds.nodes);
	ub.add(fs.shadow_order, &s->ds.shadow_order);
	ub.add(cam, &s->ds.cam);
	ub.add(shadow_light, &s->ds.shadow_light);
	rc = ub.commit(s.get());
	if (rc) {
		rt_scene_destroy(s.release());
		return rc;
	}
	// light-major single frames pay off where a shadow ray is a long LBVH search; a scene
	// without LBVHs keeps the batch threshold (C2a, one sphere and 5 lights: 0.183 vs 0.217 ms;
	// C5, whose per-lane all-lights levels then shade in place: 20.41 vs 20.50 ms)
	bool lbvh = false;
	for (const auto& g : fs.geoms) lbvh = lbvh || (g.kind == rtamd::DGEOM_MESH && g.bvh_root >= 0);
	if (!lbvh) s->light_major_below_single = s->light_major_below_batch;
	s->ds.n_geoms = static_cast<int32_t>(fs.geoms.size());
	s->ds.n_faces = static_cast<int32_t>(fs.face_geo.size());
	s->ds.n_nodes = static_cast<int32_t>(fs.nodes.size());
	s->ds.n_may_raise = fs.n_may_raise;
	bool any_bvh = false;
	for (const auto& g : fs.geoms) {
		s->ds.n_meshes += g.kind == rtamd::DGEOM_MESH ? 1 : 0;
		any_bvh = any_bvh || (g.kind == rtamd::DGEOM_MESH && g.bvh_root >= 0);
	}
	s->ds.mesh_kind = s->ds.n_meshes == 0 ? 0 : any_bvh ? 2 : 1;
	// RTAMD_MESH_KIND: a more general instantiation than the scene needs (tests, A/B)
	if (const char* mk = std::getenv("RTAMD_MESH_KIND")) s->ds.mesh_kind = std::max(s->ds.mesh_kind, std::min(2, std::atoi(mk)));
	if (const char* ws = std::getenv("RTAMD_WORK_STATS")) s->force_work_stats = std::atoi(ws) != 0;
	s->ds.n_lights = static_cast<int32_t>(fs.lights.size());
	s->ds.n_nonambient = static_cast<int32_t>(shadow_light.size());
	void* c = nullptr;
	HIP_TRY(dev_alloc(&c, sizeof(rtamd::DeviceCounters)));
	s->allocs.push_back(c);
	s->ctr = static_cast<rtamd::DeviceCounters*>(c);
	void* st = nullptr;
	HIP_TRY(dev_alloc(&st, sizeof(unsigned long long) * rtamd::kStatShards * rtamd::kStatStride));
	s->allocs.push_back(st);
	s->stats = static_cast<unsigned long long*>(st);
	void* fd = nullptr;
	HIP_TRY(dev_alloc(&fd, kFinDoneBytes));
	s->allocs.push_back(fd);
	s->fin_done = static_cast<uint32_t*>(fd);
	HIP_TRY(clear_device(s->fin_done, kFinDoneBytes));
	void* sm = nullptr;
	HIP_TRY(dev_alloc(&sm, sizeof(unsigned long long) * (rtamd::ST_COUNT + 1)));
	s->allocs.push_back(sm);
	s->summary = static_cast<unsigned long long*>(sm);
	// written by the kernels, read by the host
	HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&s->summary_host), sizeof(unsigned long long) * (rtamd::ST_COUNT + 1),
	                      kPinned));
	{
		void* mapped = nullptr;
		if (hipHostGetDevicePointer(&mapped, s->summary_host, 0) == hipSuccess)
			s->summary_mapped = static_cast<unsigned long long*>(mapped);
		(void)hipGetLastError();
	}
	// statistics and the error word start cleared; k_stats_finish clears them after each render
	HIP_TRY(clear_device(s->ctr, sizeof(rtamd::DeviceCounters)));
	HIP_TRY(clear_device(s->stats, sizeof(unsigned long long) * rtamd::kStatShards * rtamd::kStatStride));
	rt_scene_info& in = s->info;
	in.n_geometries = s->ds.n_geoms;
	for (const auto& g : fs.geoms) (g.kind == rtamd::GEOM_SPHERE ? in.n_spheres : in.n_meshes)++;
	in.n_lights = s->ds.n_lights;
	in.n_faces = static_cast<int64_t>(fs.face_geo.size());
	in.n_bvh_nodes = static_cast<int64_t>(fs.nodes.size());
	in.max_bvh_depth = fs.max_bvh_depth;
	in.build_ms = (t_upload - t_build) * 1e3;
	in.upload_ms = (now_s() - t_upload) * 1e3;
	*out = s.release();
	return RT_OK;
}

void rt_scene_destroy(rt_scene* s) {
	if (!s) return;
	(void)hipSetDevice(s->device);
	(void)hipDeviceSynchronize();
	for (auto& ln : s->lanes) lane_destroy(*ln);
	for (void* p : s->allocs) (void)dev_free(p);
	if (s->out_dev) (void)dev_free(s->out_dev);
	if (s->out8_dev) (void)dev_free(s->out8_dev);
	if (s->mapped_stage) (void)hipHostFree(s->mapped_stage);
	if (s->summary_host) (void)hipHostFree(s->summary_host);
	if (s->fork_event) (void)hipEventDestroy(s->fork_event);
	if (s->stream) (void)hipStreamDestroy(s->stream);
	delete s;
}

int rt_scene_get_info(const rt_scene* s, rt_scene_info* info) {
	if (!s || !info) return fail(RT_ERR_ARG, "null scene or info");
	*info = s->info;
	return RT_OK;
}

}  // extern "C"

namespace {

// Renders `n` jobs: chunks of at most 4 M pixels are handed to idle lanes, so with several
// lanes the chunks (of one image, or whole images of a batch) are traced concurrently
// and one image's latency-bound deep levels overlap another's wide first levels.
// --intersection-only jobs come one per call (their maximum is a per-image statistic).

// After a failed render: nothing of it may outlive the call.  Queued kernels finish (they
// may still write the caller's buffers, which the caller must not free before this
// returns), every lane forgets its chunk (its Job lives in the failed call's frame), and
// the statistics shards and the device error word are cleared for the next render.
void reset_after_error(rt_scene* s) {
	(void)hipDeviceSynchronize();
	for (auto& ln : s->lanes) {
		ln->phase = Lane::IDLE;
		ln->segs.clear();
		ln->level = 0;
		ln->level_n.clear();
		ln->shaded.clear();
		ln->deferred.clear();
		for (auto& L : ln->levels)
			if (L.block) (void)hipMemset(L.lv.counts, 0, 2 * sizeof(int32_t));
		// the device copy of the level records again from the pinned one: whatever the failed render
		// left, the next one starts from the source
		if (ln->levels_dev && ln->levels_cap)
			(void)hipMemcpy(ln->levels_dev, ln->levels_pinned, ln->levels_cap * sizeof(rtamd::RayLevel),
			                hipMemcpyHostToDevice);
	}
	(void)hipMemset(s->stats, 0, sizeof(unsigned long long) * rtamd::kStatShards * rtamd::kStatStride);
	(void)hipMemset(s->ctr, 0, sizeof(rtamd::DeviceCounters));
	(void)hipMemset(s->fin_done, 0, kFinDoneBytes);
	(void)hipDeviceSynchronize();
	(void)hipGetLastError();
}

constexpr int kPlanMiss = 1;  // internal return code of render_jobs_impl (never returned by the ABI)

int render_jobs_impl(rt_scene* s, std::vector<Job>& jobs, hipStream_t caller, rt_counters* counters,
                     Progress* progress);
int render_jobs_once(rt_scene* s, std::vector<Job>& jobs, hipStream_t caller, rt_counters* counters,
                     Progress* progress);
constexpr int64_t kMinBudgetChunkPixels = 1 << 14;

// After a call whose host-driven traces grew level buffers: every lane's levels cut back to
// what its launch plans replay and this call traced (the exact ray counts of each level:
// a replay of a plan's chunk reproduces them), so that the one-level-lookahead bounds of the
// host-driven trace (up to four times a level's rays) are not kept between calls.  C5 held
// 59 GiB of level buffers after one frame in round 4 (missing 3).
int right_size_levels(rt_scene* s) {
	for (auto& lp : s->lanes) {
		Lane& ln = *lp;
		if (!ln.grew) continue;
		ln.grew = false;
		bool resized = false;
		std::vector<int64_t> need = ln.call_need;
		need.resize(ln.levels.size(), 0);
		for (const Plan& pl : ln.plans)
			for (int L = 0; L < pl.n_levels && L < static_cast<int>(need.size()); L++)
				need[L] = std::max(need[L], pl.capacity[L]);
		for (size_t L = 0; L < ln.levels.size(); L++) {
			const int64_t target = std::max<int64_t>(need[L], 1024);
			const int64_t cap = ln.levels[L].lv.capacity;
			if (cap <= target + target / 4 + 65536) continue;  // hysteresis: no churn for small differences
			int rc = alloc_level(s, ln, L, target);
			if (!rc) rc = ensure_level_record(s, ln, L, 0);  // the device copy of its RayLevel record
			if (rc) return rc;
			resized = true;
		}
		ln.call_need.clear();
		// the record copies were queued on the lane's stream; the next call's replay may run on the
		// caller's stream (Render::start_chunk, Lane::direct), which does not wait for it: they
		// complete here, before this call returns
		if (resized) HIP_TRY(hipStreamSynchronize(ln.stream));
	}
	return RT_OK;
}

// RTAMD_LEVEL_BUDGET exceeded: the call's work is dropped, every level buffer freed and the
// chunks halved (kept for later calls); fails when even small chunks do not fit
int shrink_for_budget(rt_scene* s) {
	reset_after_error(s);
	for (auto& lp : s->lanes) {
		Lane& ln = *lp;
		clear_plans(ln);
		for (size_t L = 0; L < ln.levels.size(); L++) {
			int rc = alloc_level(s, ln, L, 1024);
			if (rc == kBudgetMiss) return fail(RT_ERR_DEVICE, "RTAMD_LEVEL_BUDGET is smaller than the minimal level buffers");
			if (rc || (rc = ensure_level_record(s, ln, L, 0))) return rc;
		}
		ln.call_need.clear();
		ln.grew = false;
	}
	s->shared_plans.clear();
	// halved from the largest chunk the failed call planned (halving a larger nominal chunk size
	// might not change its chunks at all: another full render for nothing)
	const int64_t cur = s->budget_chunk_pixels > 0 ? std::min(s->budget_chunk_pixels, s->last_chunk_pixels)
	                                               : s->last_chunk_pixels;
	const int64_t next = cur / 2;
	if (next < kMinBudgetChunkPixels)
		return fail(RT_ERR_DEVICE, "the level buffers of a " + std::to_string(cur) +
		                               "-pixel chunk exceed RTAMD_LEVEL_BUDGET (" + std::to_string(s->level_budget) + " bytes)");
	s->budget_chunk_pixels = next;
	return RT_OK;
}

int render_jobs(rt_scene* s, std::vector<Job>& jobs, hipStream_t caller, rt_counters* counters,
                Progress* progress = nullptr) {
	int rc;
	for (;;) {
		rc = render_jobs_once(s, jobs, caller, counters, progress);
		if (rc != kBudgetMiss) break;
		if ((rc = shrink_for_budget(s))) break;
		if (progress) progress->done = 0;
	}
	if (rc == RT_OK) rc = right_size_levels(s);
	// a device MathException is reported after a complete render (nothing in flight, the
	// statistics already cleared by k_stats_finish); any other error may leave work queued
	if (rc && rc != RT_ERR_MATH) {
		const std::string err = g_error;
		reset_after_error(s);
		g_error = err;
	}
	return rc;
}

int render_jobs_once(rt_scene* s, std::vector<Job>& jobs, hipStream_t caller, rt_counters* counters,
                     Progress* progress) {
	int rc = render_jobs_impl(s, jobs, caller, counters, progress);
	if (rc == kPlanMiss) {
		// a replayed plan did not fit (DERR_PLAN: a level it lacked, or a level larger than
		// its buffer; nothing was written past a buffer): forget the plans and render the
		// whole call again host-driven, which sizes every level from the counts
		reset_after_error(s);
		for (auto& ln : s->lanes) clear_plans(*ln);
		s->shared_plans.clear();
		s->plans = false;
		if (progress) progress->done = 0;
		rc = render_jobs_impl(s, jobs, caller, counters, progress);
		s->plans = true;
		if (rc == kPlanMiss) rc = fail(RT_ERR_DEVICE, "internal: level capacity exceeded in a host-driven render");
	}
	return rc;
}

}  // namespace

// The chunks of a render call: every job's selected rows as segments, packed into chunks
// (render_jobs_impl; rt_debug_plan_chunks exposes it to the CPU tests).
// pixels of a job's chunks: its chunk_pixels (0: 4 M), at most max_chunk_pixels (> 0: the
// RTAMD_LEVEL_BUDGET cap, rt_scene::budget_chunk_pixels)
int64_t chunk_limit(const rt_render_params* p, int64_t max_chunk_pixels) {
	const int64_t lim = p->chunk_pixels > 0 ? p->chunk_pixels : (int64_t)1 << 22;
	return max_chunk_pixels > 0 ? std::min(lim, max_chunk_pixels) : lim;
}

std::vector<std::vector<Segment>> plan_chunks(const std::vector<Job>& jobs, size_t n_lanes, bool batch,
                                              int64_t batch_chunk_pixels, int batch_balance, int chunks_per_lane,
                                              int64_t max_chunk_pixels) {
	// Pieces: every job's selected rows cut into pieces of at most its chunk size (4 M
	// pixels by default: it bounds the level buffers); one image over several lanes is cut
	// so that every lane holds `chunks_per_lane` of its pieces.  Consecutive pieces of
	// different jobs with equal width, height, depth and io are packed into one chunk, up to
	// batch_chunk_pixels: rows of several frames traced as one wavefront (a GPU's share of
	// row-partitioned frames is a few rows of each frame).  A chunk holds at most
	// kMaxRowSegments pieces: its rows are described by value in the kernel arguments.
	std::vector<std::vector<Segment>> chunks;
	// Balanced batches (RTAMD_BATCH_BALANCE): jobs of one shape that make fewer than two
	// chunks per lane are cut into equal chunks whose number is a multiple of the lane count,
	// so that no lane traces a last chunk alone at the end of the call (a GPU's share of
	// row-partitioned frames); cuts fall on 8-row boundaries (whole 8x8 ray tiles).
	int64_t bal_rows = 0;
	if (batch && batch_balance) {
		const Job& j0 = jobs.front();
		int64_t limit_px = batch_chunk_pixels, total_rows = 0;
		bool uniform = true;
		for (const Job& job : jobs) {
			const rt_render_params* p = job.p;
			uniform = uniform && p->width == j0.p->width && p->height == j0.p->height && job.depth == j0.depth &&
			          job.io == j0.io;
			limit_px = std::min(limit_px, chunk_limit(p, max_chunk_pixels));
			total_rows += job.n_rows;
		}
		const int64_t lim_rows = (limit_px / j0.W) & ~int64_t(7);
		const int64_t lanes = static_cast<int64_t>(n_lanes);
		int64_t n = lim_rows >= 8 ? (total_rows + lim_rows - 1) / lim_rows : 0;
		// only a call of few chunks is balanced: with many, the last one's tail is a small
		// share of the call, and whole frames keep one chunk shape (one launch plan per lane)
		if (uniform && total_rows > 0 && n > 0 && n < 2 * lanes && n % lanes != 0) {
			n = (n + lanes - 1) / lanes * lanes;
			bal_rows = std::min(lim_rows, ((total_rows + n - 1) / n + 7) & ~int64_t(7));
		}
	}
	if (bal_rows > 0) {
		std::vector<Segment> cur;
		int64_t cur_rows = 0;
		for (const Job& job : jobs)
			for (int64_t r0 = 0; r0 < job.n_rows;) {
				const int64_t take = std::min(job.n_rows - r0, bal_rows - cur_rows);
				cur.push_back(Segment{&job, r0, take});
				r0 += take;
				cur_rows += take;
				if (cur_rows == bal_rows || cur.size() == static_cast<size_t>(rtamd::kMaxRowSegments)) {
					chunks.push_back(cur);
					cur.clear();
					cur_rows = 0;
				}
			}
		if (!cur.empty()) chunks.push_back(cur);
	} else {
		std::vector<Segment> cur;
		int64_t cur_px = 0, cur_limit = 0;
		for (const Job& job : jobs) {
			const rt_render_params* p = job.p;
			const int64_t limit_px = chunk_limit(p, max_chunk_pixels);
			const int64_t max_rows = std::max<int64_t>(1, limit_px / job.W);
			const int64_t want = (!batch && n_lanes > 1) ? static_cast<int64_t>(n_lanes) * chunks_per_lane : 1;
			const int64_t piece = std::min(max_rows, std::max<int64_t>(1, (job.n_rows + want - 1) / want));
			for (int64_t r0 = 0; r0 < job.n_rows; r0 += piece) {
				const Segment sg{&job, r0, std::min(piece, job.n_rows - r0)};
				const int64_t px = sg.rows * job.W;
				bool fits = false;
				if (!cur.empty()) {
					const Job& f = *cur.front().job;
					fits = cur.back().job != &job && f.p->width == p->width && f.p->height == p->height &&
					       f.depth == job.depth && f.io == job.io && cur.size() < static_cast<size_t>(rtamd::kMaxRowSegments) &&
					       cur_px + px <= std::min({cur_limit, limit_px, batch_chunk_pixels});
				}
				if (!fits && !cur.empty()) {
					chunks.push_back(cur);
					cur.clear();
					cur_px = 0;
				}
				cur_limit = cur.empty() ? limit_px : std::min(cur_limit, limit_px);
				cur.push_back(sg);
				cur_px += px;
			}
		}
		if (!cur.empty()) chunks.push_back(cur);
	}
	return chunks;
}

namespace {

int render_jobs_impl(rt_scene* s, std::vector<Job>& jobs, hipStream_t caller, rt_counters* counters,
                     Progress* progress) {
	const bool batch = jobs.size() > 1;
	const bool minimal = !batch && s->calls == 0 && s->lanes.empty() && s->single_lanes == 0;
	s->calls++;
	size_t n_lanes = batch ? std::min<size_t>(jobs.size(), s->batch_lanes) : static_cast<size_t>(s->single_lanes);
	int chunks_per_lane = s->chunks_per_lane;
	if (!batch && n_lanes == 0) {
		// auto: a frame (or row share) of more than one chunk is traced by two lanes, each
		// tracing whole chunks (C5, 4096^2 in four 4 M-pixel chunks: 22.6 vs 24.3 ms); a frame
		// of one chunk keeps one lane (cut in two, its chunks each pay the level chain's
		// latency: C3 1.44 vs 1.33 ms, C1 0.17 vs 0.09 ms)
		const Job& j = jobs.front();
		const int64_t limit = chunk_limit(j.p, s->budget_chunk_pixels);
		const int64_t max_rows = std::max<int64_t>(1, limit / std::max<int64_t>(1, j.W));
		const int64_t pieces = (j.n_rows + max_rows - 1) / max_rows;
		n_lanes = pieces > 1 ? 2 : 1;
		// each lane keeps level buffers of its own (~200 B per ray of a 4 M-pixel chunk per
		// level, kept after the render): a second lane only while free HBM holds it four times
		// over (C5, 4096^2 at depth 8: rt_scene_info.level_bytes)
		if (n_lanes == 2 && s->lanes.size() < 2) {
			size_t free_b = 0, total_b = 0;
			const double lane_bytes = 200.0 * static_cast<double>(std::min<int64_t>(limit, j.n_rows * j.W)) *
			                          std::min(j.depth + 1, 8);
			if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && static_cast<double>(free_b) < 4 * lane_bytes)
				n_lanes = 1;
		}
		chunks_per_lane = static_cast<int>(std::max<int64_t>(1, (pieces + 1) / 2));
		// the scene's first call (a CLI run renders one frame): one lane on the scene's own
		// stream, shading in the chain's stream order; the streams a lane makes cost more than
		// the frame (8-15 ms each, C3's GPU time is 1.2 ms: profiles/round4 CLI traces)
		if (minimal) {
			n_lanes = 1;
			chunks_per_lane = static_cast<int>(std::max<int64_t>(1, pieces));
		}
	}
	int rc = ensure_lanes(s, n_lanes, minimal);
	if (rc) return rc;
	Render R{s};
	R.direct_levels = batch ? s->direct_levels_batch : n_lanes > 1 ? s->direct_levels_two_lanes : s->direct_levels_single;
	R.deep_split = batch ? s->deep_split_batch : s->deep_split_single;
	R.light_major_below = batch || n_lanes > 1 ? s->light_major_below_batch : s->light_major_below_single;
	R.progress = progress;
	R.cnt.intersection_max = 2.2250738585072014e-308;  // numeric_limits<double>::min() (scene.cpp:51)
	// the caller's stream is joined first (its prior work, e.g. the allocation of the
	// output buffers, completes before ours starts: Render::fork, as a lane starts its first
	// chunk); the call returns when all is done
	R.caller = caller;
	for (size_t k = 0; k < n_lanes; k++) s->lanes[k]->forked = false;
	const std::vector<std::vector<Segment>> chunks =
	    plan_chunks(jobs, n_lanes, batch, s->batch_chunk_pixels, 1, chunks_per_lane, s->budget_chunk_pixels);
	R.direct_ok = n_lanes == 1 && chunks.size() == 1;
	s->last_chunk_pixels = 0;
	for (const auto& c : chunks) {
		int64_t px = 0;
		for (const Segment& sg : c) px += sg.rows * sg.job->W;
		s->last_chunk_pixels = std::max(s->last_chunk_pixels, px);
	}
	size_t next_chunk = 0;
	std::unique_ptr<rtamd::MarkerRange> trace_range(new rtamd::MarkerRange("rtamd: trace (levels, shading, output)"));
	// The statistics reduction is queued on the caller's stream, behind every lane's last
	// chunk, as soon as all of the call's launches are issued, not after the host has seen
	// them complete: a launch onto an idle GPU takes ~30 us to start, which is a third of a
	// small frame (profiles/round3 marker trace)
	bool stats_issued = false;
	auto issue_stats = [&]() -> int {
		stats_issued = true;
		if (R.stats_fused) return RT_OK;  // done by the call's last kernel (k_fused / k_output)
		for (size_t k = 0; k < n_lanes; k++)
			if (s->lanes[k]->forked) HIP_TRY(hipStreamWaitEvent(caller, s->lanes[k]->chunk_done, 0));
		if (s->summary_mapped) {
			HIP_TRY(rtamd::launch_stats_finish(s->stats, s->ctr, s->summary_mapped, caller));
		} else {
			HIP_TRY(rtamd::launch_stats_finish(s->stats, s->ctr, s->summary, caller));
			HIP_TRY(hipMemcpyAsync(s->summary_host, s->summary, sizeof(unsigned long long) * (rtamd::ST_COUNT + 1),
			                       hipMemcpyDeviceToHost, caller));
		}
		stats_issued = true;
		return RT_OK;
	};
	for (;;) {
		bool busy = false;
		for (size_t k = 0; k < n_lanes; k++) {
			Lane& ln = *s->lanes[k];
			if (ln.phase == Lane::IDLE) {
				if (next_chunk >= chunks.size()) continue;
				if ((rc = R.start_chunk(ln, chunks[next_chunk++]))) return rc;
				busy = true;
				continue;
			}
			busy = true;
			hipEvent_t e = ln.phase == Lane::TRACING ? ln.level_events[ln.level][5] : ln.chunk_done;
			const hipError_t q = hipEventQuery(e);
			if (q == hipErrorNotReady) continue;
			if (q != hipSuccess) return fail(RT_ERR_DEVICE, std::string("hipEventQuery: ") + hipGetErrorString(q));
			rc = ln.phase == Lane::TRACING ? R.on_counts(ln) : R.on_done(ln);
			if (rc) return rc;
		}
		if (!stats_issued && next_chunk >= chunks.size()) {
			bool issued = true;  // every lane idle or with its last chunk fully queued
			for (size_t k = 0; k < n_lanes; k++) issued = issued && s->lanes[k]->phase != Lane::TRACING;
			if (issued && (rc = issue_stats())) return rc;
		}
		if (progress && progress->fn && progress->done < progress->total) {
			const double t = now_s();
			if (t - progress->last >= 0.1) {  // scene.cpp:41-44 polls every 100 ms
				progress->last = t;
				progress->fn(static_cast<int>(progress->done), progress->total, progress->user);
			}
		}
		if (!busy) break;
	}
	trace_range.reset();
	rtamd::MarkerRange stats_range("rtamd: statistics read-back");
	// all lanes' work is complete (their events were observed); the statistics reduction is
	// queued behind it (above) and one small summary read back
	if (!stats_issued && (rc = issue_stats())) return rc;
	HIP_TRY(hipStreamSynchronize(caller));
	const unsigned long long* sum = s->summary_host;
	const int derr = static_cast<int>(sum[rtamd::ST_COUNT]);
	if (derr == rtamd::DERR_PLAN) return kPlanMiss;
	// MathException texts (rtbase.h:14-22) are the reference's; the internal checks are device failures
	if (derr == rtamd::DERR_STACK || derr == rtamd::DERR_ROWS)
		return fail(RT_ERR_DEVICE, device_error_text(derr));
	if (derr) return fail(RT_ERR_MATH, device_error_text(derr));
	rt_counters& cnt = R.cnt;
	cnt.trace_rays = static_cast<int64_t>(sum[rtamd::ST_RAYS]);
	cnt.shadow_rays = static_cast<int64_t>(sum[rtamd::ST_HITS]) * s->ds.n_nonambient;
	cnt.reflect_rays = static_cast<int64_t>(sum[rtamd::ST_REFL]);
	cnt.refract_rays = static_cast<int64_t>(sum[rtamd::ST_REFR]);
	cnt.shadow_rays_zero_terms = static_cast<int64_t>(sum[rtamd::ST_SHADOW_ZERO]);
	for (int k = 0; k < 2; k++) {
		const int b = k ? rtamd::ST_NODES1 : rtamd::ST_NODES0;
		cnt.stage_node_visits[k] = static_cast<int64_t>(sum[b]);
		cnt.stage_tri_tests[k] = static_cast<int64_t>(sum[b + 1]);
		cnt.stage_candidates[k] = static_cast<int64_t>(sum[b + 2]);
		cnt.stage_sphere_tests[k] = static_cast<int64_t>(sum[b + 3]);
		cnt.stage_bvh_traversals[k] = static_cast<int64_t>(sum[k ? rtamd::ST_ENTRIES1 : rtamd::ST_ENTRIES0]);
		cnt.stage_max_node_visits[k] = static_cast<int64_t>(sum[k ? rtamd::ST_MAXNODES1 : rtamd::ST_MAXNODES0]);
		cnt.node_visits += cnt.stage_node_visits[k];
		cnt.tri_tests += cnt.stage_tri_tests[k];
		cnt.candidates += cnt.stage_candidates[k];
		cnt.sphere_tests += cnt.stage_sphere_tests[k];
	}
	cnt.trace_launches = cnt.stage_launches[0] + cnt.stage_launches[1] + cnt.stage_launches[2];
	cnt.kernel_ms = R.kernel_ms;
	if (jobs.size() == 1 && jobs[0].io) {
		const Job& job = jobs[0];
		const rt_render_params* p = job.p;
		if (sum[rtamd::ST_MAX_BITS]) {
			double m;
			const unsigned long long b = sum[rtamd::ST_MAX_BITS];
			std::memcpy(&m, &b, sizeof(m));
			cnt.intersection_max = std::max(cnt.intersection_max, m);
		}
		// full-image --intersection-only: normalise in place (scene.cpp:50-58)
		if (p->row_begin == 0 && p->row_end == p->height && p->row_step == 1 && job.out_rgb_dev) {
			rtamd::MarkerRange nr("rtamd: --intersection-only normalisation");
			HIP_TRY(rtamd::launch_normalize(job.n_rows * job.W * 3, job.out_rgb_dev, cnt.intersection_max,
			                                job.out_rgb8_dev, caller));
			HIP_TRY(hipStreamSynchronize(caller));
		}
	}
	if (counters) *counters = cnt;
	return RT_OK;
}

}  // namespace

Job make_job(const rt_render_params* p, double* out_rgb_dev, uint8_t* out_rgb8_dev) {
	Job j{};
	j.p = p;
	j.out_rgb_dev = out_rgb_dev;
	j.out_rgb8_dev = out_rgb8_dev;
	j.io = p->intersection_only != 0;
	j.depth = j.io ? 0 : p->bounce_depth;
	j.W = p->width;
	j.n_rows = selected_rows(p);
	return j;
}

namespace {


void add_counters(rt_counters& a, const rt_counters& b) {
	a.trace_rays += b.trace_rays;
	a.shadow_rays += b.shadow_rays;
	a.reflect_rays += b.reflect_rays;
	a.refract_rays += b.refract_rays;
	a.shadow_rays_zero_terms += b.shadow_rays_zero_terms;
	a.pixels += b.pixels;
	a.intersection_max = std::max(a.intersection_max, b.intersection_max);
	a.kernel_ms += b.kernel_ms;
	a.levels = std::max(a.levels, b.levels);
	a.trace_launches += b.trace_launches;
	a.node_visits += b.node_visits;
	a.tri_tests += b.tri_tests;
	a.candidates += b.candidates;
	a.sphere_tests += b.sphere_tests;
	for (int k = 0; k < 3; k++) {
		a.stage_ms[k] += b.stage_ms[k];
		a.stage_launches[k] += b.stage_launches[k];
	}
	for (int k = 0; k < 2; k++) {
		a.stage_node_visits[k] += b.stage_node_visits[k];
		a.stage_tri_tests[k] += b.stage_tri_tests[k];
		a.stage_candidates[k] += b.stage_candidates[k];
		a.stage_sphere_tests[k] += b.stage_sphere_tests[k];
		a.stage_bvh_traversals[k] += b.stage_bvh_traversals[k];
		a.stage_max_node_visits[k] = std::max(a.stage_max_node_visits[k], b.stage_max_node_visits[k]);
	}
}


// device staging buffers of rt_render / rt_render_rgb8 (and of --intersection-only renders
// whose caller wants RGB8 only: the f64 image is needed for the global maximum)
int ensure_staging(rt_scene* s, int64_t n_pixels, bool f64, bool u8) {
	if (f64 && s->out_capacity < n_pixels) {
		if (s->out_dev) HIP_TRY(dev_free(s->out_dev));
		s->out_dev = nullptr;
		s->out_capacity = 0;
		HIP_TRY(dev_alloc((&s->out_dev), std::max<int64_t>(n_pixels, 1) * 3 * sizeof(double)));
		s->out_capacity = n_pixels;
	}
	if (u8 && s->out8_capacity < n_pixels) {
		if (s->out8_dev) HIP_TRY(dev_free(s->out8_dev));
		s->out8_dev = nullptr;
		s->out8_capacity = 0;
		HIP_TRY(dev_alloc((&s->out8_dev), std::max<int64_t>(n_pixels, 1) * 3));
		s->out8_capacity = n_pixels;
	}
	return RT_OK;
}

// The image to the caller's (pageable) host memory when it is not written into mapped
// memory (render_to_host): hipMemcpy stages pageable copies itself.  Pinning the destination
// for the copy, or staging through pinned memory the scene keeps, measured no faster
// (round 4, profiles/round4/ab/cli_startup_ab.txt).
hipError_t copy_to_host(void* dst, const void* src, size_t bytes) {
	return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost);
}

// mapped pinned host staging the kernels write the image into, for images of
// at most kMappedStageMax bytes (f64 + RGB8: a 2560x1600 frame; a 4096^2 f64 image, 400 MB,
// is copied instead of pinning that much host memory for the scene's lifetime)
#ifndef RT_MAPPED_STAGE_MAX
#define RT_MAPPED_STAGE_MAX (size_t(128) << 20)
#endif
constexpr size_t kMappedStageMax = RT_MAPPED_STAGE_MAX;
int ensure_mapped_stage(rt_scene* s, size_t bytes) {
	if (s->mapped_stage_bytes >= bytes) return RT_OK;
	if (s->mapped_stage) (void)hipHostFree(s->mapped_stage);
	s->mapped_stage = s->mapped_stage_dev = nullptr;
	s->mapped_stage_bytes = 0;
	// coherent: the kernels' image writes reach host memory, not an L2 line (see UploadBatch)
	if (hipHostMalloc(&s->mapped_stage, std::max<size_t>(bytes, 256), kPinnedMapped) !=
	    hipSuccess) {
		s->mapped_stage = nullptr;
		return fail(RT_ERR_DEVICE, "hipHostMalloc (mapped image stage) failed");
	}
	if (hipHostGetDevicePointer(&s->mapped_stage_dev, s->mapped_stage, 0) != hipSuccess) {
		(void)hipHostFree(s->mapped_stage);
		s->mapped_stage = s->mapped_stage_dev = nullptr;
		return fail(RT_ERR_DEVICE, "hipHostGetDevicePointer (mapped image stage) failed");
	}
	s->mapped_stage_bytes = bytes;
	return RT_OK;
}

bool whole_image(const rt_render_params* p) { return p->row_begin == 0 && p->row_end == p->height && p->row_step == 1; }
// (row_step 1 selects every row whatever row_block is)

int render_batch(rt_scene* s, int n, const rt_render_params* params, double* const* out_rgb_dev,
                 uint8_t* const* out_rgb8_dev, void* stream_v, rt_counters* counters, Progress* progress) {
	const double t0 = now_s();
	if (!s || !params || n < 0) return fail(RT_ERR_ARG, "null scene or params");
	for (int k = 0; k < n; k++) {
		const int rc = check_params(s, params + k);
		if (rc) return rc;
	}
	HIP_TRY(hipSetDevice(s->device));
	// no caller stream: the scene's own
	hipStream_t caller = stream_v ? static_cast<hipStream_t>(stream_v) : s->stream;
	// the traversal kernels' instantiation: with the work counters only when asked for
	s->ds.work_stats = s->force_work_stats;
	for (int k = 0; k < n; k++) s->ds.work_stats = s->ds.work_stats || params[k].work_stats != 0;
	rt_counters total{};
	total.intersection_max = 2.2250738585072014e-308;
	std::vector<Job> jobs;
	auto flush = [&]() -> int {
		if (jobs.empty()) return RT_OK;
		rt_counters c{};
		const int rc = render_jobs(s, jobs, caller, &c, progress);
		jobs.clear();
		if (!rc) add_counters(total, c);
		return rc;
	};
	for (int k = 0; k < n; k++) {
		Job j = make_job(params + k, out_rgb_dev ? out_rgb_dev[k] : nullptr, out_rgb8_dev ? out_rgb8_dev[k] : nullptr);
		if (j.n_rows <= 0) continue;
		int rc;
		if (j.io) {  // alone: its maximum is its own
			if (j.out_rgb8_dev && !j.out_rgb_dev) {
				// RGB8 of an --intersection-only image: normalised by the image's maximum
				// (scene.cpp:50-58) from an f64 staging image
				if (!whole_image(j.p))
					return fail(RT_ERR_ARG, "--intersection-only row subsets need out_rgb (the normalisation "
					                        "waits for the global maximum, rt_normalize_device)");
				if ((rc = ensure_staging(s, j.n_rows * j.W, true, false))) return rc;
				j.out_rgb_dev = s->out_dev;
			}
			if ((rc = flush())) return rc;
			jobs.push_back(j);
			if ((rc = flush())) return rc;
		} else {
			jobs.push_back(j);
		}
	}
	const int rc = flush();
	if (rc) return rc;
	total.host_ms = (now_s() - t0) * 1e3;
	if (counters) *counters = total;
	return RT_OK;
}

// rt_render / rt_render_rgb8: one image into staging buffers, then one copy to the host;
// progress as scene.cpp:41-44 (the calling thread, about every 100 ms, then complete)
int render_to_host(rt_scene* s, const rt_render_params* p, double* out_rgb, uint8_t* out_rgb8, rt_progress_fn progress,
                   void* user, rt_counters* counters) {
	int rc = check_params(s, p);
	if (rc) return rc;
	if (!out_rgb && !out_rgb8) return fail(RT_ERR_ARG, "null output");
	if (out_rgb8 && p->intersection_only && !whole_image(p))
		return fail(RT_ERR_ARG, "--intersection-only RGB8 needs the whole image (global maximum)");
	HIP_TRY(hipSetDevice(s->device));
	const int64_t n = selected_rows(p) * p->width;
	if ((rc = ensure_staging(s, n, out_rgb != nullptr || p->intersection_only, out_rgb8 != nullptr))) return rc;
	Progress pr;
	pr.fn = progress;
	pr.user = user;
	pr.total = static_cast<int>(std::min<int64_t>(n, 0x7fffffff));
	pr.last = now_s();
	if (progress) progress(0, pr.total, user);
	double* rgb_dev = (out_rgb || p->intersection_only) ? s->out_dev : nullptr;
	uint8_t* rgb8_dev = out_rgb8 ? s->out8_dev : nullptr;
	// the kernels write the image straight into mapped pinned host memory (no copy engine: its
	// first use in a process costs ~16 ms; the CLI's image copy 13-17 -> 0.2-2.2 ms,
	// profiles/round4/ab/cli_startup_ab.txt), then a host memcpy
	const size_t f64_bytes = out_rgb ? static_cast<size_t>(n) * 3 * sizeof(double) : 0, u8_bytes = out_rgb8 ? static_cast<size_t>(n) * 3 : 0;
	// Images above kMappedStageMax, or a failed pinned allocation, take the copy path instead:
	// the scene never holds more than that much pinned host memory for it.
	char* mapped = nullptr;
	if (f64_bytes + u8_bytes <= kMappedStageMax) {
		if (ensure_mapped_stage(s, f64_bytes + u8_bytes) == RT_OK && s->mapped_stage) {
			mapped = static_cast<char*>(s->mapped_stage);
			char* dev = static_cast<char*>(s->mapped_stage_dev);
			if (out_rgb) rgb_dev = reinterpret_cast<double*>(dev);
			if (out_rgb8) rgb8_dev = reinterpret_cast<uint8_t*>(dev + f64_bytes);
		} else {
			(void)hipGetLastError();  // the failed allocation is not the render's error: copy_to_host below
			g_error.clear();
		}
	}
	const double t0 = now_s();
	rc = render_batch(s, 1, p, &rgb_dev, &rgb8_dev, nullptr, counters, &pr);
	if (rc) return rc;
	rtamd::MarkerRange cr("rtamd: image to host (PCIe)");
	const double t_copy = now_s();
	if (mapped) {
		if (out_rgb) std::memcpy(out_rgb, mapped, f64_bytes);
		if (out_rgb8) std::memcpy(out_rgb8, mapped + f64_bytes, u8_bytes);
	} else {
		if (out_rgb) HIP_TRY(copy_to_host(out_rgb, s->out_dev, f64_bytes));
		if (out_rgb8) HIP_TRY(copy_to_host(out_rgb8, s->out8_dev, u8_bytes));
	}
	if (counters) {
		counters->copy_ms = (now_s() - t_copy) * 1e3;
		counters->host_ms = (now_s() - t0) * 1e3;
	}
	if (progress) progress(pr.total, pr.total, user);
	return RT_OK;
}

}  // namespace

extern "C" {

int rt_render_device(rt_scene* s, const rt_render_params* p, double* out_rgb_dev, uint8_t* out_rgb8_dev, void* stream_v,
                     rt_counters* counters) {
	return render_batch(s, 1, p, &out_rgb_dev, &out_rgb8_dev, stream_v, counters, nullptr);
}

int rt_render_batch_device(rt_scene* s, int n, const rt_render_params* params, double* const* out_rgb_dev,
                           uint8_t* const* out_rgb8_dev, void* stream_v, rt_counters* counters) {
	return render_batch(s, n, params, out_rgb_dev, out_rgb8_dev, stream_v, counters, nullptr);
}

int rt_render(rt_scene* s, const rt_render_params* p, double* out_rgb, rt_progress_fn progress, void* user,
              rt_counters* counters) {
	if (!out_rgb) return fail(RT_ERR_ARG, "null output");
	return render_to_host(s, p, out_rgb, nullptr, progress, user, counters);
}

int rt_render_rgb8(rt_scene* s, const rt_render_params* p, uint8_t* out_rgb8, rt_progress_fn progress, void* user,
                   rt_counters* counters) {
	if (!out_rgb8) return fail(RT_ERR_ARG, "null output");
	return render_to_host(s, p, nullptr, out_rgb8, progress, user, counters);
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

void rt_partition_row(int64_t row, int n_devices, int row_block, int* device, int64_t* local_row) {
	int d = 0;
	int64_t l = 0;
	rtamd::partition_row(row, n_devices < 1 ? 1 : n_devices, row_block, &d, &l);
	if (device) *device = d;
	if (local_row) *local_row = l;
}

int rt_write_png(const char* path, const uint8_t* rgb, int width, int height) {
	if (!path || !rgb || width <= 0 || height <= 0) return fail(RT_ERR_ARG, "bad PNG arguments");
	rtamd::MarkerRange mr("rtamd: PNG encode + write");
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
	if (!x || !out) return fail(RT_ERR_ARG, "null input or output");
	HIP_TRY(hipSetDevice(device));
	struct DeviceBuffers {  // freed on every exit, error paths included
		double* p[3] = {nullptr, nullptr, nullptr};
		~DeviceBuffers() {
			for (double* q : p)
				if (q) (void)dev_free(q);
		}
	} buf;
	for (double*& q : buf.p) HIP_TRY(dev_alloc((&q), n * sizeof(double)));
	double *dx = buf.p[0], *dy = buf.p[1], *dout = buf.p[2];
	HIP_TRY(hipMemcpy(dx, x, n * sizeof(double), hipMemcpyHostToDevice));
	HIP_TRY(hipMemcpy(dy, y ? y : x, n * sizeof(double), hipMemcpyHostToDevice));
	HIP_TRY(rtamd::launch_selftest_math(op, dx, dy, dout, n, nullptr));
	HIP_TRY(hipMemcpy(out, dout, n * sizeof(double), hipMemcpyDeviceToHost));
	return RT_OK;
}

}  // extern "C"
