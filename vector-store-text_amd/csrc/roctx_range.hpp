// roctx_range.hpp — a roctx range around every C-ABI entry point (SURVEY §5:
// "roctx ranges around each C-ABI call"), so `rocprofv3 --marker-trace` shows
// which library call a kernel belongs to.  Built in only with -DVSG_ROCTX
// (`make ROCTX=1`): production builds and the Rust / Python consumers do not
// depend on the profiler SDK; without the flag VSG_RANGE() is empty.
#pragma once
#ifdef VSG_ROCTX
#include <rocprofiler-sdk-roctx/roctx.h>

namespace vsg {
struct RoctxRange {
    explicit RoctxRange(const char* name) { roctxRangePushA(name); }
    ~RoctxRange() { roctxRangePop(); }
    RoctxRange(const RoctxRange&) = delete;
    RoctxRange& operator=(const RoctxRange&) = delete;
};
}  // namespace vsg

#define VSG_RANGE() ::vsg::RoctxRange vsg_range__(__func__)
#else
#define VSG_RANGE() ((void)0)
#endif
