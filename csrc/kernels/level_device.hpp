// Device-side level decisions shared by the traversal kernels
// (bfs_kernels.hip) and the peer-memory collectives (peer_kernels.hip), which
// finish a level in the same launch as its totals' all-reduce.
#pragma once

#include <hip/hip_runtime.h>

#include "dbfs/backend.hpp"
#include "wave.hpp"

namespace dbfs {
namespace kern {

// Level-end stamp of the host-mapped mailbox slot: values first (system
// scope), then the level with release semantics, so a host that observes the
// level reads that level's values.
__device__ __forceinline__ void stamp_mailbox(LevelMailbox* mb, const LevelCtrl& c, int32_t level) {
  __hip_atomic_store(&mb->done, c.done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(&mb->vis_deg), static_cast<unsigned long long>(c.vis_deg),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&mb->next_dir, c.dir, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(&mb->n_f), static_cast<unsigned long long>(c.n_f),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(&mb->m_f), static_cast<unsigned long long>(c.m_f),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(&mb->reached), static_cast<unsigned long long>(c.reached),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&mb->level, level, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Several ranks: the level's decision on its all-reduced totals
// (LevelFinishArgs; stats[2..3] final) -- one thread.
__device__ __forceinline__ void level_finish_device(const LevelFinishArgs& a) {
  if (!a.seed && !chain_live(*a.ctrl, a.expect_dir, a.expect_cap)) return;
  LevelCtrl c = a.seed ? a.ctrl_init : *a.ctrl;
  level_ctrl_finish(c, a.stats[2], a.stats[3], a.seed, a.seed ? nullptr : a.rec);
  if (!a.seed) {
    a.rec->t0 = c.t_start;
    a.rec->t1 = wall_clock64();
  }
  *a.ctrl = c;
  if (a.mailbox) stamp_mailbox(a.mailbox, c, a.seed ? -1 : a.level);
}

// Hub-split entries of the next level (HxAppendArgs), by one workgroup of
// kThreads: every thread takes kPer words of the frontier-hub bits, counts the
// hubs with a part on this rank and their edges, the workgroup scans those,
// and each thread appends its hubs' entries (qscan, qbase, qv, the edge
// blocks they start) behind the level's listed ones; thread 0 moves the end
// marker and the list totals.
template <int kThreads>
__device__ __forceinline__ void hx_append(const HxAppendArgs& h) {
  using namespace dev;
  constexpr int kPer = static_cast<int>((kTdMaxHubs / 64 + kThreads - 1) / kThreads);
  constexpr int kWaves = kThreads / kWave;
  __shared__ long long s_c[kWaves], s_e[kWaves];
  const int t = threadIdx.x;
  const int lane = lane_id();
  const int wv = t / kWave;
  const int64_t hw = (h.nhubs + 63) / 64;
  word_t wb[kPer];
  long long c = 0, e = 0;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t w = static_cast<int64_t>(t) * kPer + k;
    wb[k] = w < hw ? static_cast<word_t>(h.bits[w]) : 0ull;
    for (word_t m = wb[k]; m; m &= m - 1) {
      const int64_t hub = w * 64 + __ffsll(static_cast<long long>(m)) - 1;
      const eid_t d = h.hx_off[hub + 1] - h.hx_off[hub];
      if (d > 0) {
        ++c;
        e += d;
      } else {
        wb[k] &= ~(1ull << (hub & 63));  // (no part on this rank: no entry)
      }
    }
  }
  const long long ci = wave_incl_scan(c), ei = wave_incl_scan(e);
  if (lane == kWave - 1) {
    s_c[wv] = ci;
    s_e[wv] = ei;
  }
  __syncthreads();
  long long cb = ci - c, eb = ei - e, ctot = 0, etot = 0;
  for (int k = 0; k < kWaves; ++k) {
    if (k < wv) {
      cb += s_c[k];
      eb += s_e[k];
    }
    ctot += s_c[k];
    etot += s_e[k];
  }
  const long long q0 = h.list_stats[0], m0 = h.list_stats[1];
  long long p = q0 + cb, qs = m0 + eb;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t w = static_cast<int64_t>(t) * kPer + k;
    for (word_t m = wb[k]; m; m &= m - 1) {
      const int64_t hub = w * 64 + __ffsll(static_cast<long long>(m)) - 1;
      const eid_t rs = h.hx_off[hub], d = h.hx_off[hub + 1] - rs;
      const int64_t r = static_cast<int64_t>(h.hub_vertex[hub]) - h.lo;
      h.qscan[p] = qs;
      h.qbase[p] = rs - qs;
      h.qv[p] = r >= 0 && r < h.rows ? static_cast<vid_t>(r) : kNoRow;
      for (long long b = (qs + kTdEdgesPerBlock - 1) / kTdEdgesPerBlock; b * kTdEdgesPerBlock < qs + d; ++b)
        h.blk_vstart[b] = static_cast<int32_t>(p);
      ++p;
      qs += d;
    }
  }
  __syncthreads();  // (every thread has read list_stats)
  if (t == 0) {
    h.qscan[q0 + ctot] = m0 + etot;
    h.list_stats[0] = q0 + ctot;
    h.list_stats[1] = m0 + etot;
  }
}

// Several ranks: a level's end after its totals' all-reduce, by every thread
// of one workgroup of kThreads -- on a live chain (or the seed) the hub-split
// entries of the next level (fin.hx), then thread 0's decision.
// (the entries only after the decision, and only for a top-down next level:
// a bottom-up one reads no work list, and appending the thousands of frontier
// hubs of its input cost a P = 8 replay 300 us in this one workgroup)
template <int kThreads>
__device__ __forceinline__ void level_finish_block(const LevelFinishArgs& a) {
  if (!a.seed && !chain_live(*a.ctrl, a.expect_dir, a.expect_cap)) return;
  __shared__ int s_append;
  if (threadIdx.x == 0) {
    level_finish_device(a);
    s_append = a.hx.bits && !a.ctrl->done && a.ctrl->dir == 'T';
  }
  __syncthreads();
  if (s_append) hx_append<kThreads>(a.hx);
}

}  // namespace kern
}  // namespace dbfs
