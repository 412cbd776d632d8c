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
// level reads that level's values.  (Measured without the release -- values
// acknowledged by s_waitcnt, then a relaxed level store -- to skip its L2
// write-back: the 1024 x 1024 grid's levels 8.5 / 9.6 us either way, RMAT-26
// unchanged; the kernel's end-of-launch release writes the L2 back anyway.)
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

// A level record (host memory, read after the traversal's last stamp),
// system-scope write-through.
__device__ __forceinline__ void store_rec(LevelRecDev* rec, const LevelRecDev& r) {
  auto st64 = [](void* p, uint64_t v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), static_cast<unsigned long long>(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  };
  __hip_atomic_store(&rec->dir, r.dir, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  st64(&rec->n_f, static_cast<uint64_t>(r.n_f));
  st64(&rec->m_f, static_cast<uint64_t>(r.m_f));
  st64(&rec->discovered, static_cast<uint64_t>(r.discovered));
  st64(&rec->t0, r.t0);
  st64(&rec->t1, r.t1);
}

// A level's decision from its totals (count, degree sum of the new
// frontier), one thread: level_ctrl_finish on c (the control block as read),
// the level's record (not for the seed), the control block written back and
// the mailbox stamped.
__device__ __forceinline__ void finish_level(LevelCtrl* ctrl, LevelCtrl& c, int64_t cnt, int64_t deg, bool seed,
                                             LevelRecDev* rec, LevelMailbox* mailbox, int32_t level) {
  LevelRecDev r;
  level_ctrl_finish(c, cnt, deg, seed, &r);
  if (!seed && rec) {
    r.t0 = c.t_start;
    r.t1 = wall_clock64();
    store_rec(rec, r);
  }
  *ctrl = c;
  if (mailbox) stamp_mailbox(mailbox, c, seed ? -1 : level);
}

// Several ranks: the level's decision on its all-reduced totals
// (LevelFinishArgs; stats[2..3] final) -- one thread.
__device__ __forceinline__ void level_finish_device(const LevelFinishArgs& a) {
  if (!a.seed && !chain_live(*a.ctrl, a.expect_dir, a.expect_cap)) return;
  LevelCtrl c = a.seed ? a.ctrl_init : *a.ctrl;
  finish_level(a.ctrl, c, a.stats[2], a.stats[3], a.seed, a.rec, a.mailbox, a.level);
}

// ... for a kernel whose argument block holds `a` (level_finish_block: the
// peer collectives, level_finish_kernel): two plain copies instead of the
// select above, which takes the kernel argument's address and made those
// kernels copy their whole argument struct to scratch (752 B a lane in the
// peer unpack).  (The select stays where `a` is a kernel's own copy: the
// split form costs td_sparse a spill.)
__device__ __forceinline__ void level_finish_device_arg(const LevelFinishArgs& a) {
  if (!a.seed && !chain_live(*a.ctrl, a.expect_dir, a.expect_cap)) return;
  if (a.seed) {
    LevelCtrl c = a.ctrl_init;
    finish_level(a.ctrl, c, a.stats[2], a.stats[3], true, a.rec, a.mailbox, a.level);
  } else {
    LevelCtrl c = *a.ctrl;
    finish_level(a.ctrl, c, a.stats[2], a.stats[3], false, a.rec, a.mailbox, a.level);
  }
}

// Several ranks: a level's end after its totals' all-reduce, in one
// workgroup (the peer transport's fused collective): thread 0's decision.
// (The chain check is thread 0's alone -- it reads the control block the
// decision then writes.)
template <int kThreads>
__device__ __forceinline__ void level_finish_block(const LevelFinishArgs& a) {
  if (threadIdx.x == 0) level_finish_device_arg(a);
}

}  // namespace kern
}  // namespace dbfs
