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

// Several ranks: a level's end after its totals' all-reduce, in one
// workgroup (the peer transport's fused collective): thread 0's decision.
// (The chain check is thread 0's alone -- it reads the control block the
// decision then writes.)
template <int kThreads>
__device__ __forceinline__ void level_finish_block(const LevelFinishArgs& a) {
  if (threadIdx.x == 0) level_finish_device(a);
}

}  // namespace kern
}  // namespace dbfs
