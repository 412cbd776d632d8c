// Host spin on a device store into pinned, mapped memory (engine internals).
#pragma once

#include <chrono>

#include "dbfs/backend.hpp"

namespace dbfs {

// Spin until `ready()` (a store of the device into pinned, mapped memory).
// Every wait-watch period: the backend's watch runs (RCCL: async errors and
// the collective timeout), and a stream that has drained without `ready()`
// is an error (the stamping kernel did not run).
template <class Ready>
void spin_until(Backend& be, Ready ready, const char* what) {
  if (ready()) return;
  const auto t0 = std::chrono::steady_clock::now();
  const double period = be.wait_watch_period();
  double next = period;
  for (uint64_t spin = 1;; ++spin) {
    if (ready()) return;
    if ((spin & 0x3FF) != 0) continue;
    const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (waited < next) continue;
    if (be.stream_idle() && !ready()) throw Error(what);
    be.poll_wait_watch(waited);
    next = waited + period;
  }
}

}  // namespace dbfs
