// roctx_range.hpp — a roctx range around every C-ABI entry point (SURVEY §5:
// "roctx ranges around each C-ABI call"), so `rocprofv3 --marker-trace` shows
// which library call a kernel belongs to.  Without a profiler attached the
// push / pop are a few nanoseconds each.
#pragma once
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
