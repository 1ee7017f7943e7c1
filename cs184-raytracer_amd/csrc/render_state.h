// Internal state of librtamd's render driver (api.cpp), shared with the diagnostic entry
// points of librtamd_diag.so (diag.cpp).  Not part of the C-ABI (include/rtamd.h).
#pragma once
#include <hip/hip_runtime.h>
#include <array>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>
#include "../../include/rtamd.h"
#include "scene_host.h"
#include "trace.h"

struct rt_builder {
	rtamd::Scene scene;
	// rt_builder_get_desc views (rebuilt on every call)
	std::vector<rt_geometry_desc> desc_geoms;
	std::vector<rt_light_desc> desc_lights;
};

static_assert(sizeof(rt_face_desc) == sizeof(rtamd::Face) && sizeof(rt_face_desc) == 192,
              "rt_face_desc is Mesh::Face (geometry.h:32) and the host Face");

// One image (or row selection) of a render call: its parameters and outputs.
struct Job {
	const rt_render_params* p;
	double* out_rgb_dev;
	uint8_t* out_rgb8_dev;
	int depth, io;
	int64_t W, n_rows;
};

// Rows [r0, r0 + rows) of a job's selected rows (ordinals), part of one chunk
struct Segment {
	const Job* job;
	int64_t r0, rows;
};

// Progress of a render call (scene.cpp:41-44: the calling thread reports completed pixels
// about every 100 ms): pixels of the chunks whose output kernel has finished, as seen by
// the host's event polling.
struct Progress {
	rt_progress_fn fn = nullptr;
	void* user = nullptr;
	int total = 0;
	int64_t done = 0;
	double last = -1.0;
};

struct LevelBuffers {
	rtamd::RayLevel lv{};
	void* block = nullptr;
	int64_t bytes = 0;
};

// A chunk shape traced once host-driven becomes a plan: the same launch sequence with every
// level size read on the device (k_closest's n from the previous level's child counter,
// the shading batches and reductions from the hit and child counters), issued at once for
// every later chunk of that shape, with no host round trip between levels.
// (Capturing that sequence into a hipGraph measured slower on this ROCm: graph replay
// serialised the branches and the lanes; round 2.)  Levels and
// capacities come from the traced chunk; a replay that would need more (a deeper level, a
// larger level) is caught on the device (DERR_PLAN, nothing written past a buffer) and the
// render is redone host-driven.
struct PlanKey {
	int32_t width, height, depth, io;
	int32_t direct_levels;  // the schedule's split of direct and batched shading (a graph bakes it in)
	int32_t deep_split;     // levels shaded alone after the chain (per call: single frame or batch)
	int32_t work_stats;     // the traversal kernels' counting instantiation (a graph bakes it in)
	int64_t light_major_below;  // shading launches' item layout (per call; a graph bakes it in)
	int64_t n0;
	uint64_t rows_hash;  // the chunk's image rows (they decide the level counts)
	bool operator==(const PlanKey& o) const {
		return width == o.width && height == o.height && depth == o.depth && io == o.io &&
		       direct_levels == o.direct_levels && deep_split == o.deep_split && work_stats == o.work_stats &&
		       light_major_below == o.light_major_below && n0 == o.n0 &&
		       rows_hash == o.rows_hash;
	}
};

// plans kept per lane and shared per scene (oldest dropped first): a batch of one shape has
// at most 2 x lanes chunk shapes
constexpr size_t kMaxPlans = 64;
struct Plan {
	PlanKey key{};
	int n_levels = 0;
	// rays and hits of every level in the traced chunk: they size the grids only (the kernels
	// read the actual counts and stride over them, so a difference costs time, not results)
	std::vector<int64_t> level_n, hits;
	// the level buffer capacities a replay needs (plan sharing, right-sizing): the traced
	// chunk's ray counts, which a replay of the same key reproduces exactly (same rows, same
	// scene), not the host-driven trace's one-level-lookahead bounds
	std::vector<int64_t> capacity;
	int launches[3] = {0, 0, 0};
};

// One render pipeline: its own level buffers, streams and events, tracing one chunk of
// rows (<= 4 M pixels) at a time as a host-polled state machine (Render below).  Several
// lanes can trace chunks of a frame concurrently (RTAMD_LANES); on C3 one lane is
// fastest, because every chunk pays the level chain's latency.
struct Lane {
	hipStream_t stream = nullptr;        // k_closest chain, reduce, output (high priority)
	hipStream_t readback = nullptr;      // level counts -> host, off the chain's stream
	// k_shadow + k_shade of level L < direct_levels on shade[L % 3]; the small deep levels
	// are shaded in batches on shade[3] once the chain has finished
	hipStream_t shade[4] = {nullptr, nullptr, nullptr, nullptr};
	int prio_low = 0;
	// a scene's first call borrows the scene's stream for everything (chain, read-back,
	// shading: no stream of its own, each costs 8-15 ms to make); the next call gives the
	// lane its own (upgrade_lane)
	bool minimal = false;
	std::vector<LevelBuffers> levels;
	// the largest ray count of each level traced host-driven during the current call, and
	// whether a level buffer grew in it (right_size_levels)
	std::vector<int64_t> call_need;
	bool grew = false;
	// RayLevel records of all levels, read by the kernels through the constant address space
	// (pinned host copy + device copy, updated in stream order when a level is reallocated)
	rtamd::RayLevel* levels_pinned = nullptr;
	rtamd::RayLevel* levels_dev = nullptr;
	size_t levels_cap = 0;
	// per level: [0] before k_closest, [1] after it (the shading streams wait on it),
	// [5] the level's counts copied to counts_host; per shading launch, in the events of
	// its first level: [2] before k_shadow, [3] after it, [4] after k_shade (the reduce
	// waits on it)
	std::vector<std::array<hipEvent_t, 6>> level_events;
	hipEvent_t chunk_done = nullptr;     // output of the chunk written
	int32_t* counts_host = nullptr;      // pinned, per level: hits, children (levels_cap x 2)
	// chunk state
	enum Phase { IDLE, TRACING, FINISHING } phase = IDLE;
	std::vector<Segment> segs;            // the chunk's rows: pieces of one or several jobs
	int depth = 0, io = 0;                // shared by the chunk's jobs
	uint64_t rows_hash = 0;               // the image rows of the chunk (plan key)
	rtamd::FrameGeometry fg{};
	int64_t n0 = 0;                       // pixels of the chunk (its rows x width)
	int level = 0;                        // the level whose counts are awaited
	std::vector<int64_t> level_n;         // ray counts of the levels known so far
	std::vector<int> shaded;                        // first level of each shading launch
	std::vector<std::pair<int, int64_t>> deferred;  // (level, hits) shaded after the chain
	// launch plans of the chunk shapes this lane has traced (plain data: the level buffers are
	// read from the lane when a plan is issued)
	std::vector<Plan> plans;
	const Plan* planned = nullptr;        // the plan replaying the current chunk, if any
	bool forked = false;                  // this call's caller stream joined into the lane's streams
	bool direct = false;                  // the current chunk runs on the caller's stream (Render::start_chunk)
};

inline void clear_plans(Lane& ln) {
	ln.plans.clear();
	ln.planned = nullptr;
}

struct rt_scene {
	int device = 0;
	hipStream_t stream = nullptr;                // default caller stream (rt_render, normalize)
	rtamd::DeviceScene ds{};
	std::vector<void*> allocs;
	rt_scene_info info{};
	std::vector<std::unique_ptr<Lane>> lanes;
	rtamd::DeviceCounters* ctr = nullptr;        // device
	unsigned long long* stats = nullptr;         // device, kStatShards x kStatStride
	unsigned long long* summary = nullptr;       // device, ST_COUNT + 1 (k_stats_finish)
	unsigned long long* summary_host = nullptr;  // pinned mirror
	// the pinned mirror's device address: k_stats_finish writes the summary straight into host
	// memory (no copy launch behind it on the call's critical path); null: copy from `summary`
	unsigned long long* summary_mapped = nullptr;
	double* out_dev = nullptr;                   // staging for rt_render (f64)
	int64_t out_capacity = 0;
	uint8_t* out8_dev = nullptr;                 // staging for rt_render_rgb8
	void* mapped_stage = nullptr;                // mapped pinned host image (render_to_host)
	void* mapped_stage_dev = nullptr;
	size_t mapped_stage_bytes = 0;
	int64_t out8_capacity = 0;
	// test hooks, set only through librtamd_diag.so (diag.cpp; rtamd.h has no entry point for them)
	int fail_after = -1;                         // rt_debug_fail_after: closest-hit launches left, then a failure
	int corrupt_rows = 0;                        // rt_debug_corrupt_rows: the next chunk's row descriptors made invalid
	hipEvent_t fork_event = nullptr;             // caller's stream -> lane streams
	// RTAMD_DIRECT_LEVELS: levels shaded beside the closest-hit chain; the rest are shaded in
	// batches after it.  Measured best on C3: 3 for one frame per call
	// (latency: level 1's shading overlaps levels 2+), 1 for batches (throughput: fewer,
	// larger shading launches while other frames fill the GPU).  A frame of more than one chunk,
	// traced by two lanes (single_lanes auto), takes 2: each lane's chain then shares the GPU
	// with the other lane's shading as well (round 6: C5 -2.9%, bunny and al at 4096^2 -3% and
	// -9%, al at 2896^2 -5%; one-chunk frames lose 1-3% with 2).  The variable sets all three.
	int direct_levels_single = 3;
	int direct_levels_two_lanes = 2;
	int direct_levels_batch = 1;
	int single_lanes = 0;                        // lanes one frame is split over (RTAMD_LANES); 0 = auto
	// chunk pipelines of a batch in flight (RTAMD_BATCH_LANES).  4 lanes gave the C3 bench
	// +0.2-1.2%, but single frames rendered after such a batch took 1.31-1.34 instead of
	// 1.16-1.18 ms (its 24 streams share the process's hardware queues differently); 8 lanes and
	// smaller chunks lose (profiles/round4/ab/batch_*)
	int batch_lanes = 3;
	int prio_low = 0, prio_high = 0;
	int chunks_per_lane = 2;
	int serial = 0;                              // RTAMD_SERIAL: shading on the chain's stream (solo kernel times)
	// launch plans of traced chunk shapes (false while a call whose plan missed is redone
	// host-driven, render_jobs_once)
	bool plans = true;
	int64_t batch_chunk_pixels = (int64_t)1 << 22;  // RTAMD_BATCH_CHUNK: most pixels of a chunk packed from several jobs
	// plans are plain data: a lane adopts a plan another lane built (growing its level buffers
	// to the plan's capacities) instead of tracing the chunk shape host-driven itself (+0.7%
	// whole frames, +1.3% on the 4-way share, round 2)
	std::vector<Plan> shared_plans;
	bool force_work_stats = false;               // RTAMD_WORK_STATS: every call counts (rt_render_params::work_stats)
	int plan_truncate = 0;                       // RTAMD_PLAN_TRUNCATE (tests): plans one level short, replays miss
	int shadow_all_lights = 3;                   // RTAMD_SHADOW_ALL_LIGHTS: bit 0 level 0, bit 1 deeper (ShadeBatch)
	// RTAMD_LIGHT_MAJOR_BELOW: a shading launch with fewer hits than this traces light-major
	// (one lane per (hit, light)) even where the all-lights layout is selected: a few waves per
	// SIMD each tracing every light in turn leave the GPU latency-bound (one GPU's row share
	// of a single frame); light-major gives n_lights times the waves, each a shorter chain
	// Per call like direct_levels: a single frame (or one device's row share of it) of a scene
	// with meshes traces light-major below 1 M hits (C4 0.401 -> 0.354 ms, C2b 0.349 -> 0.326,
	// C3 1.284 -> 1.259),
	// a batch below 128 K (its level-1 launch of 2-frame chunks, ~840 K hits, measured -7% as
	// light-major, and an 8-way row share -3 to -6%: DESIGN.md §4)
	// A frame traced by two lanes (more than one chunk) takes the batch's threshold: its
	// launches have the batch's size (round 6: al at 2896^2 / 4096^2 -3.4% / -2.6%, the bunny
	// at 4096^2 -0.5%)
	int64_t light_major_below_single = (int64_t)1 << 20;
	int64_t light_major_below_batch = (int64_t)1 << 17;
	// RTAMD_ONE_STREAM_PIXELS: a replayed chunk of at most this many pixels is issued on one
	// stream (Render::issue_plan)
	// (a plan of one traced level is issued on one stream too: it has no deeper level for its
	// shading to overlap; C4 0.365 -> 0.351 ms, round 3)
	int64_t one_stream_pixels = (int64_t)1 << 17;
	// RTAMD_FUSED: a replayed one-stream chunk traces every level in ONE launch (k_fused: closest
	// hits + shadow rays + Phong terms, and for a plan of one level the output pixels too)
	// instead of k_closest + k_shadow (+ k_shade) per level and k_output
	int fused = 1;
	// RTAMD_FUSED_MIN_PIXELS: a mesh scene's chunk of fewer pixels keeps the split launches.  Such
	// a chunk is one round of waves, so its time is its slowest tile's; fused, that tile also
	// traces every light's shadow rays in turn, split the shadow rays are spread over a second
	// launch of (hit, light) items: the C4 1/8 row share 0.234 -> 0.208 ms, C1-C4 unchanged
	// (profiles/round4/ab/latency_quad_fuse_knobs.txt)
	int64_t fused_min_pixels = 524288;
	// RTAMD_LEVEL_BUDGET: bytes of level buffers all lanes may hold together (0: no limit).  A
	// render whose host-driven trace would need more is redone with chunks of half as many
	// pixels (budget_chunk_pixels, kept for later calls) until it fits (render_jobs)
	int64_t level_budget = 0;
	int64_t budget_chunk_pixels = 0;
	int64_t last_chunk_pixels = 0;  // the largest chunk of the last call (shrink_for_budget)
	int64_t calls = 0;            // render calls so far
	uint32_t* fin_done = nullptr;  // device: blocks done of a launch that finishes the statistics (9 x 128 B)
	int all_lights_for(int first_level, int64_t hits, int64_t light_major_below) const {
		int al = (shadow_all_lights >> (first_level == 0 ? 0 : 1)) & 1;
		if (al && ds.n_nonambient > 1 && hits < light_major_below) al = 0;
		return al;
	}
	// RTAMD_DEEP_SPLIT: the first n levels after the direct ones are shaded alone, each in
	// its own launch after the chain, before one batch of the rest (a batch's first bounce
	// then traces its shadow rays as packets; per call like direct_levels)
	int deep_split_single = 0;
	int deep_split_batch = 1;
	// measured best on C3: packets for the camera rays and their first bounce, and
	// for the shadow rays of both (once the zero-term decision thinned the per-lane waves)
	int packet_mask =
	    rtamd::kPacketClosest0 | rtamd::kPacketClosest1 | rtamd::kPacketShadow0 | rtamd::kPacketShadow1;
};

// Shared with diag.cpp (defined in api.cpp)
namespace rtamd {
int set_error(int code, const std::string& msg);
}  // namespace rtamd
Job make_job(const rt_render_params* p, double* out_rgb_dev, uint8_t* out_rgb8_dev);
std::vector<std::vector<Segment>> plan_chunks(const std::vector<Job>& jobs, size_t n_lanes, bool batch,
                                              int64_t batch_chunk_pixels, int batch_balance, int chunks_per_lane,
                                              int64_t max_chunk_pixels = 0);
