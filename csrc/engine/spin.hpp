// Host spin on a device store into pinned, mapped memory (engine internals).
#pragma once

#include <algorithm>
#include <chrono>

#include "dbfs/backend.hpp"

namespace dbfs {

// Spin until `ready()` (a store of the device into pinned, mapped memory).
// Every wait-watch period: the backend's watch runs (RCCL: async errors and
// the collective timeout; peer windows: a timed-out device wait), then a
// stream that has drained without `ready()` is an error (the stamping kernel
// did not run).
template <class Ready>
void spin_until(Backend& be, Ready ready, const char* what) {
  if (ready()) return;
  const auto t0 = std::chrono::steady_clock::now();
  const double period = be.wait_watch_period();
  double next = period;
  double idle_since = -1.0;  // (seconds: when the stream was first seen drained without the stamp)
  for (uint64_t spin = 1;; ++spin) {
    if (ready()) return;
    if ((spin & 0x3FF) != 0) continue;
    const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (waited < next) continue;
    // (the watch first: a device wait that timed out also drains the stream,
    // and its error -- which rank, collective and peer -- is the real cause)
    be.poll_wait_watch(waited);
    // A drained stream without the stamp is an error only once it has stayed
    // so for a grace period: the stamp is a system-scope store into host
    // memory, and the completion signal the stream query reads can become
    // visible before it (a GPU suite run saw that race once).
    if (be.stream_idle() && !ready()) {
      if (idle_since < 0) idle_since = waited;
      else if (waited - idle_since > 0.2) throw Error(what);
    } else {
      idle_since = -1.0;
    }
    next = waited + std::min(period, 0.05);
  }
}

}  // namespace dbfs
