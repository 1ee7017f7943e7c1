// roctx ranges around the host phases of a render (SURVEY.md §5 "Tracing / profiling"):
// `rocprofv3 --marker-trace` shows upload, trace, statistics read-back, normalisation,
// multi-GPU gather and PNG encoding on the host timeline beside the kernels.  The
// reference's only instrumentation is its progress ticker (main.cpp:24-38,
// scene.cpp:41-44).  Without a profiler attached a range costs two library calls.
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

namespace rtamd {

struct MarkerRange {
	explicit MarkerRange(const char* what) { roctxRangePushA(what); }
	~MarkerRange() { roctxRangePop(); }
	MarkerRange(const MarkerRange&) = delete;
	MarkerRange& operator=(const MarkerRange&) = delete;
};

}  // namespace rtamd
