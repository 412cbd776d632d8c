// Tracing ranges for rocprofv3 (`--marker-trace`): one range per BFS run, per
// level and per phase (expand / update / exchange).  roctx calls are cheap
// no-ops unless a profiler is attached.  The reference has no tracing beyond
// std::chrono millisecond prints (bfs.cu:214-218, 551, 624-626).
#pragma once

#include <rocprofiler-sdk-roctx/roctx.h>

#include <string>

namespace dbfs {

class TraceRange {
 public:
  explicit TraceRange(const char* name) { roctxRangePushA(name); }
  explicit TraceRange(const std::string& name) { roctxRangePushA(name.c_str()); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

inline void trace_mark(const char* msg) { roctxMarkA(msg); }

}  // namespace dbfs
