// Device helpers shared by the traversal kernel files (bfs_kernels.hip:
// level bookkeeping, td_kernels.hip: top-down, bu_kernels.hip: bottom-up):
// the checked-build macro, level stores, last-arriver hand-offs, the scan
// finish, work-list block starts, the direct-exchange words and the folded
// level end.  Everything lives in an anonymous namespace: each kernel file
// gets its own copy (device globals such as g_check included).
#pragma once

#include <hip/hip_runtime.h>

#include "dbfs/backend.hpp"
#include "launch.hpp"
#include "level_device.hpp"
#include "wave.hpp"

namespace dbfs {
namespace kern {

// Compute units of the current device (bfs_kernels.hip).
int device_cus();
// Checked build: the first violation recorded by the top-down / bottom-up
// kernel files (cleared); bfs_kernels.hip's take_check_error reads all three.
unsigned long long take_check_td();
unsigned long long take_check_bu();
// A level's totals and finish from unscanned unit statistics, one workgroup
// (bfs_kernels.hip; bottom-up levels without the fused finish).
void totals_finish(const ScanArgs& a, hipStream_t st);

namespace {

using namespace dev;

// Device-checked build (make checked, -DDBFS_CHECKED): bounds
// of the work lists, owner lists and vertex ids are verified in the kernels
// and the first violation is recorded (code << 48 | detail) in g_check --
// never a trap: the host reads the word after every traversal and throws
// (HipBackend::device_checks), the GPU keeps running.  Off: no code.
#ifdef DBFS_CHECKED
__device__ unsigned long long g_check;
#define DBFS_DCHECK(cond, code, detail)                                                               \
  do {                                                                                                \
    if (!(cond))                                                                                      \
      atomicCAS(&g_check, 0ull,                                                                       \
                (static_cast<unsigned long long>(code) << 48) |                                       \
                    (static_cast<unsigned long long>(detail) & 0xFFFFFFFFFFFFull));                   \
  } while (0)
#else
#define DBFS_DCHECK(cond, code, detail) \
  do {                                  \
  } while (0)
#endif

// First kernel of a device-loop level chain: record its start (device wall
// clock) for the level's record (scan_units_kernel copies it to rec[L].t0).
// (The argument blocks carry the control block as const; this field is the
// one a level's kernels write.)
__device__ __forceinline__ void stamp_level_start(const LevelCtrl* c) {
  if (c && blockIdx.x == 0 && threadIdx.x == 0) const_cast<LevelCtrl*>(c)->t_start = wall_clock64();
}

// A new vertex's level: the narrow array when the run uses one (uniform
// branch), else the 32-bit array.  Narrow overflow (level > kNarrowMaxLevel)
// stores kNarrowUnreached; the engine reruns such a traversal with wide levels.
// (narrow: base + level; base + 63 flags a level too deep for the bytes)
__device__ __forceinline__ void store_level(lvl_t* wide, uint8_t* narrow, int64_t i, lvl_t level, uint8_t base) {
  if (narrow)
    narrow[i] = static_cast<uint8_t>(base + (level <= kNarrowMaxLevel ? level : kNarrowMaxLevel + 1));
  else
    wide[i] = level;
}

// Last-arriver hand-offs (scan_units, fused finishes, td_sparse): the last
// workgroup reads only values the others stored write-through (agent-scope
// stores / atomics) with agent-scope loads; the agent acquire fence is kept
// (measured no slower than without it).
__device__ __forceinline__ void last_arriver_acquire() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

constexpr int kBlock = 256;
constexpr int kUnitThreads = kUnitWaves * kWave;  // 256: 4 waves x 16 words
static_assert(kUnitThreads == 256 && kWaveWords <= kWave, "unit geometry");

// Unit geometry of update / compact / sparse-from-bitmap kernels: one wave
// per 64-word unit, kUnitsPerBlock units per workgroup.
constexpr int kUnitsPerBlock = kBlock / kWave;
static_assert(kUnitWords == kWave, "one word per lane in update/compact");

// The level's totals (count, degree sum of the new frontier) -> stats, the
// work list's end marker, the ticket reset and (device loop) the direction
// decision, level record and mailbox stamp.  One thread.
__device__ __forceinline__ void scan_finish(const ScanArgs& a, long long carry_c, long long carry_d) {
  DBFS_DCHECK(carry_c <= a.nunits * kUnitVertices, 7, carry_c);
  a.stats[0] = a.stats[2] = carry_c;
  a.stats[1] = a.stats[3] = carry_d;
  a.qscan[carry_c] = carry_d;
  *a.ticket = 0u;  // next launch is stream-ordered after this one
  if (a.ctrl && a.finish) {
    LevelCtrl c = *a.ctrl;
    finish_level(a.ctrl, c, carry_c, carry_d, a.seed, a.rec, a.mailbox, a.level);
  }
}

// blk[b] = p for every edge block b (kTdEdgesPerBlock edges) that starts in the
// entry's edge range [qs, qs + d) -- wave-uniform call.  Short ranges are
// written by their lane; long ones (a hub's row spans hundreds of blocks) by
// the whole wave, 64 blocks per step, instead of one lane looping alone.
__device__ __forceinline__ void wave_fill_blocks(int32_t* __restrict__ blk, bool take, long long qs, long long d,
                                                 long long p) {
  const long long b0 = take ? (qs + kTdEdgesPerBlock - 1) / kTdEdgesPerBlock : 0;
  const long long b1 = take ? (qs + d + kTdEdgesPerBlock - 1) / kTdEdgesPerBlock : 0;
  const bool wide = b1 - b0 > 4;
  if (!wide)
    for (long long b = b0; b < b1; ++b) blk[b] = static_cast<int32_t>(p);
  unsigned long long pending = __ballot(wide);
  while (pending) {
    const int l = __ffsll(static_cast<long long>(pending)) - 1;
    pending &= pending - 1;
    const long long lo = readlane_i64(b0, l), hi = readlane_i64(b1, l), pl = readlane_i64(p, l);
    for (long long b = lo + lane_id(); b < hi; b += kWave) blk[b] = static_cast<int32_t>(pl);
  }
}

// Cross-GPU hand-off words (direct owner-list exchange): system-scope relaxed
// accesses through global (not flat) instructions -- sc0 sc1 stores write
// through to the owner's memory, sc0 sc1 loads read it -- so neither side
// needs an L2 write-back or invalidate (MI355X_MICROARCH hand-off forms:
// write-through stores, every storing wave's vmcnt(0) before the signal, the
// reader's loads behind its poll and a workgroup barrier).
using gu32 = __attribute__((address_space(1))) uint32_t;
using gu64 = __attribute__((address_space(1))) uint64_t;
__device__ __forceinline__ void sys_store_u32(uint32_t* p, uint32_t v) {
  __hip_atomic_store((gu32*)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store_u64(uint64_t* p, uint64_t v) {
  __hip_atomic_store((gu64*)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t sys_load_u32(const uint32_t* p) {
  return __hip_atomic_load((gu32*)(const_cast<uint32_t*>(p)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t sys_load_u64(const uint64_t* p) {
  return __hip_atomic_load((gu64*)(const_cast<uint64_t*>(p)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

// Frontier push (backend.hpp FrontierTable): word w of this rank's slice to
// every peer's window, write-through.
__device__ __forceinline__ void push_frontier_word(const FrontierTable* t, int rank, int nranks, int64_t w,
                                                   uint64_t v) {
  for (int p = 0; p < nranks; ++p)
    if (p != rank) sys_store_u64(t->dst[p] + w, v);
}

// Append the kItems items of every lane (bit k of `act`: v[k]) to their
// owners' lists with ONE atomic per wave and owner for all of them (the
// per-item form takes one per item index and owner: up to kItems times as
// many returning atomics on the same count words).  Wave-uniform call.
template <int kItems>
__device__ __forceinline__ void owner_list_append_items(vid_t* lists, int64_t stride, int64_t part,
                                                        const vid_t (&v)[kItems], unsigned act,
                                                        const DirectTable* dt = nullptr) {
  const int lane = lane_id();
  int own[kItems];
  unsigned long long left = 0;
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    own[k] = ((act >> k) & 1u) ? static_cast<int>(static_cast<int64_t>(v[k]) / part) : -1;
    left |= __ballot(own[k] >= 0);
  }
  while (left) {
    // the next owner: the first active item of the first lane with one
    const int leader = __ffsll(static_cast<long long>(left)) - 1;
    int mine = -1;
#pragma unroll
    for (int k = kItems - 1; k >= 0; --k)
      if (own[k] >= 0) mine = own[k];
    const int o = __builtin_amdgcn_readfirstlane(__shfl(mine, leader, kWave));
    unsigned long long msk[kItems];
    unsigned tot = 0;
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      msk[k] = __ballot(own[k] == o);
      tot += static_cast<unsigned>(__popcll(msk[k]));
    }
    vid_t* list = lists + static_cast<int64_t>(o) * stride;
    unsigned base = 0;
    if (lane == leader) base = atomicAdd(list, tot);
    base = __shfl(base, leader, kWave);
    DBFS_DCHECK(base + tot < static_cast<unsigned long long>(stride), 3, base);
    unsigned before = 0;
    left = 0;
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      if (own[k] == o) {
        const unsigned at = 1u + base + before + mask_rank(msk[k]);
        if (dt) sys_store_u32(dt->dst[o] + at, v[k]);
        else list[at] = v[k];
        own[k] = -1;
      }
      before += static_cast<unsigned>(__popcll(msk[k]));
      left |= __ballot(own[k] >= 0);
    }
  }
}

// Workgroup-aggregated owner-list append: every wave of the workgroup calls
// it (uniform); lane items v[k] with bit k of `act` go to their owners' lists.
// Per owner the waves take their offsets with LDS atomics and the workgroup
// takes its slots with ONE atomic on the owner's count word -- with two ranks
// every wave of a 1 M-edge level appended to the same remote count word
// (thousands of returning atomics on one address, ~90 per us).
template <int kItems>
__device__ __forceinline__ void owner_list_append_wg(vid_t* lists, int64_t stride, int64_t part, int nranks,
                                                     const vid_t (&v)[kItems], unsigned act,
                                                     const DirectTable* dt = nullptr) {
  __shared__ unsigned s_oc[kern::kMaxPeers], s_ob[kern::kMaxPeers];
  const int t = threadIdx.x;
  const int lane = lane_id();
  if (t < nranks) s_oc[t] = 0u;
  __syncthreads();
  int own[kItems];
  unsigned off[kItems];
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    own[k] = ((act >> k) & 1u) ? static_cast<int>(static_cast<int64_t>(v[k]) / part) : -1;
    off[k] = 0u;
    unsigned long long pending = __ballot(own[k] >= 0);
    while (pending) {
      const int leader = __ffsll(static_cast<long long>(pending)) - 1;
      const int o = __builtin_amdgcn_readfirstlane(__shfl(own[k], leader, kWave));
      const unsigned long long msk = __ballot(own[k] == o);
      unsigned base = 0u;
      if (lane == leader) base = atomicAdd(&s_oc[o], static_cast<unsigned>(__popcll(msk)));
      base = __shfl(base, leader, kWave);
      if (own[k] == o) off[k] = base + mask_rank(msk);
      pending &= ~msk;
    }
  }
  __syncthreads();
  if (t < nranks) {
    const unsigned c = s_oc[t];
    s_ob[t] = c ? atomicAdd(lists + static_cast<int64_t>(t) * stride, c) : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    if (own[k] < 0) continue;
    const unsigned at = 1u + s_ob[own[k]] + off[k];
    DBFS_DCHECK(at < static_cast<unsigned long long>(stride), 3, at);
    if (dt) sys_store_u32(dt->dst[own[k]] + at, v[k]);
    else lists[static_cast<int64_t>(own[k]) * stride + at] = v[k];
  }
  __syncthreads();  // (s_oc / s_ob reused by the next call)
}

// Direct exchanges' tagged cells (backend.hpp DirectExchange).
__device__ __forceinline__ uint64_t cell_word0(uint64_t seq, uint64_t v) { return (seq << 32) | (v & 0xffffffffull); }
__device__ __forceinline__ uint64_t cell_word1(uint64_t seq, uint64_t v) {
  return ((seq & 0xffffffull) << 40) | (v & ((1ull << 40) - 1));
}
__device__ __forceinline__ bool cell_ok0(uint64_t w, uint64_t seq) { return (w >> 32) == (seq & 0xffffffffull); }
__device__ __forceinline__ bool cell_ok1(uint64_t w, uint64_t seq) { return (w >> 40) == (seq & 0xffffffull); }

// Direct owner lists, producer side (one workgroup, after every producing
// wave's write-through stores have drained): thread p publishes this rank's
// count for owner p in p's cell -- one store -- and zeroes the local count for
// the next list level.  A chain that is not live publishes empty lists: the
// peers wait all the same.
__device__ __forceinline__ void direct_publish(const DirectExchange& d, vid_t* lists, int64_t stride, bool live) {
  const int t = threadIdx.x;
  if (t < d.nranks && t != d.rank) {
    vid_t* cnt = lists + static_cast<int64_t>(t) * stride;
    const vid_t n = live ? __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    *cnt = 0u;
    sys_store_u64(d.table->cell_out[t], cell_word0(d.seq, n));
  }
}

// Direct exchange, consumer side (every thread of the workgroup calls it):
// threads p < nranks poll sender p's cell until both words asked for carry
// this exchange's tag and leave its payload in out0 / out1 [p] (this rank's
// own: 0).  Returns kWaitOk; kWaitTimeout after DirectExchange::timeout_ticks
// (the error word the host watches gets seq | (peer + 1) << 48: which
// exchange, and the first peer found missing), or at once when another wait
// of this rank already timed out (the error word is set: a dead peer stops
// every wait queued behind the first instead of each spending its own
// timeout); kWaitLater when a cell already carries a LATER exchange's tag:
// the peer has moved on, which it does only after this rank's next signal --
// so this exchange is over here (a workgroup of the apply that started after
// the level's end: it has nothing to do).  Data behind the cell is then read
// with sys loads.
constexpr int kWaitOk = 1, kWaitTimeout = 0, kWaitLater = -1;
__device__ __forceinline__ int direct_wait(const DirectExchange& d, uint64_t* out0, uint64_t* out1) {
  __shared__ int s_st, s_peer;
  const int t = threadIdx.x;
  if (t == 0) {
    s_st = kWaitOk;
    s_peer = -1;
  }
  __syncthreads();
  if (t < d.nranks) {
    uint64_t w0 = 0, w1 = 0;
    if (t != d.rank) {
      const uint64_t* c = d.table->cell_in[t];
      const uint64_t t0 = wall_clock64();
      for (uint32_t spin = 0;; ++spin) {
        w0 = sys_load_u64(c);
        if (out1) w1 = sys_load_u64(c + 1);
        if (cell_ok0(w0, d.seq) && (!out1 || cell_ok1(w1, d.seq))) break;
        if (static_cast<int32_t>(static_cast<uint32_t>(w0 >> 32) - static_cast<uint32_t>(d.seq)) > 0) {
          s_st = kWaitLater;  // (benign race: every writer stores the same)
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        if ((spin & 255) == 255) {
          if (wall_clock64() - t0 > d.timeout_ticks) {
            s_st = kWaitTimeout;
            s_peer = t;  // (benign race: any missing peer names the stall)
            break;
          }
          if (d.error && sys_load_u64(d.error) != 0) {
            s_st = kWaitTimeout;  // (an earlier wait already reported)
            break;
          }
        }
      }
      w0 &= 0xffffffffull;
      w1 &= (1ull << 40) - 1;
    }
    out0[t] = w0;
    if (out1) out1[t] = w1;
  }
  __syncthreads();
  const int st = s_st;
  if (st == kWaitTimeout && t == 0 && d.error && s_peer >= 0)
    sys_store_u64(d.error, (d.seq & kWaitSeqMask) | (static_cast<uint64_t>(s_peer + 1) << 48));
  return st;
}

// The level's end in the last workgroup of its last kernel (DirectExchange
// from Comm::direct_level_end; every thread of the workgroup calls it):
// threads p < nranks publish this rank's totals (c new vertices, g their
// degrees) in p's cell, every peer's cell is awaited, and thread 0 sums (or,
// shadow replay, takes the recorded sums) into stats[2..3] and makes the
// level's decision (level_finish_device, as Comm::level_end's).
// s_x: 2 x kMaxPeers words of LDS the caller lends (the bottom-up kernel has
// none to spare: two workgroups per CU fill the LDS to within 0.5 KiB).
__device__ __forceinline__ void direct_level_end(const DirectExchange& d, int64_t c, int64_t g, int64_t* stats,
                                                 const LevelFinishArgs& fin, uint64_t* s_x) {
  uint64_t* s_c = s_x;
  uint64_t* s_g = s_x + kern::kMaxPeers;
  const int t = threadIdx.x;
  DBFS_DCHECK(c >= 0 && c < (int64_t(1) << 32) && g >= 0 && g < (int64_t(1) << 40), 11, g);
  if (t < d.nranks && t != d.rank) {
    uint64_t* cell = d.table->cell_out[t];
    sys_store_u64(cell, cell_word0(d.seq, static_cast<uint64_t>(c)));
    sys_store_u64(cell + 1, cell_word1(d.seq, static_cast<uint64_t>(g)));
  }
  // (a level end is awaited by the one last workgroup of every rank: no peer
  // passes it before this rank's cell is read, so kWaitLater cannot occur)
  if (direct_wait(d, s_c, s_g) != kWaitOk || t != 0) return;
  uint64_t sc = static_cast<uint64_t>(c), sg = static_cast<uint64_t>(g);
  if (d.result) {
    sc = static_cast<uint64_t>(d.result[0]);
    sg = static_cast<uint64_t>(d.result[1]);
  } else {
    for (int p = 0; p < d.nranks; ++p) {
      sc += s_c[p];  // (this rank's own entries are 0)
      sg += s_g[p];
    }
  }
  stats[2] = static_cast<int64_t>(sc);
  stats[3] = static_cast<int64_t>(sg);
  level_finish_device(fin);
}

// Two-level last-arriver ticket (thread 0, the workgroup's stores drained):
// the workgroups of a kFusedGroup group count on their group's ticket (its own
// 128-B line), the group's last one re-zeroes it and counts on the level
// ticket -- a grid of thousands of workgroups queues ~64 atomics per address
// instead of all of them on one.  True in the level's last workgroup.
__device__ __forceinline__ bool group_ticket_last(unsigned* group_ticket, unsigned* ticket) {
  const unsigned grp = blockIdx.x / kFusedGroup;
  const unsigned gsz = min(static_cast<unsigned>(kFusedGroup), gridDim.x - grp * kFusedGroup);
  const unsigned ngroups = (gridDim.x + kFusedGroup - 1) / kFusedGroup;
  unsigned* gt = group_ticket + grp * kBuQueueStride;
  if (atomicAdd(gt, 1u) != gsz - 1) return false;
  atomicExch(gt, 0u);
  return atomicAdd(ticket, 1u) == ngroups - 1;
}

// n (<= kMaxWords) words of global memory staged into LDS by a workgroup of
// kThreads: every thread's words loaded at once, then stored -- one round
// trip instead of one per kThreads words (the loop's trip count is not known
// to the compiler, so it would not overlap them).
template <int kThreads, int kMaxWords>
__device__ __forceinline__ void stage_words(word_t* s, const word_t* __restrict__ g, int64_t n) {
  constexpr int kPer = (kMaxWords + kThreads - 1) / kThreads;
  word_t v[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t i = threadIdx.x + static_cast<int64_t>(k) * kThreads;
    v[k] = i < n ? g[i] : 0ull;
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t i = threadIdx.x + static_cast<int64_t>(k) * kThreads;
    if (i < n) s[i] = v[k];
  }
}

inline unsigned grid_for(int64_t work, int64_t per_block, int64_t cap = 1 << 30) {
  int64_t g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return static_cast<unsigned>(g);
}

// This file's first recorded device-check violation, cleared (0: none).
inline unsigned long long take_check_local() {
#ifdef DBFS_CHECKED
  unsigned long long h = 0, z = 0;
  (void)hipMemcpyFromSymbol(&h, HIP_SYMBOL(g_check), sizeof(h));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_check), &z, sizeof(z));
  return h;
#else
  return 0;
#endif
}

}  // namespace
}  // namespace kern
}  // namespace dbfs
