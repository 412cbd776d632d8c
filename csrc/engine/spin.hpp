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
// did not run, or ran without stamping).  No grace period: the stamp is a
// system-scope store, and a kernel's completion signal is raised only after
// its end-of-kernel release, so a drained stream has made every stamp
// visible.  (Round 5's "drained without the stamp" was not a visibility
// race: a late td_sparse workgroup had shifted the level ticket -- see
// DeviceLoop::sblk.)
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
    // (the watch first: a device wait that timed out also drains the stream,
    // and its error -- which rank, collective and peer -- is the real cause)
    be.poll_wait_watch(waited);
    // (idle first, then the stamp re-read: a stamp stored just before the
    // stream drained is seen)
    if (be.stream_idle() && !ready()) throw Error(what);
    next = waited + std::min(period, 0.05);
  }
}

}  // namespace dbfs
