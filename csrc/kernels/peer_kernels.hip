// gfx950 kernels of the peer-memory communicator (PeerComm, csrc/comm/peer_comm.cpp).
//
// Every rank exports one window of uncached device memory (IPC) and maps its
// peers' windows; a collective is one launch (peer_fused_kernel: the three
// steps below in one grid; DBFS_PEER_FUSED=0 launches them separately), no
// host in the loop and no library protocol:
//   push   -- each rank stores its per-peer payloads straight into the peers'
//             windows over xGMI (slot [parity][sender]); the last workgroup to
//             finish (ticket) publishes `seq` into every peer's flag word for
//             this sender, behind a system-scope release;
//   wait   -- one wave polls the P flag words of its own window (system-scope
//             relaxed loads + s_sleep, bounded: a peer that never arrives sets
//             the error word the host watches instead of hanging the GPU);
//   unpack -- copy (or, for the all-reduce, sum) the landed slots into the
//             caller's buffers.
// The windows are uncached (hipDeviceMallocUncached), so the data a peer wrote
// is read from memory, not from a stale L2 line; the consumer's caches are the
// ordinary ones because unpack writes the caller's (cached) buffers.
// Reference call sites replaced: the per-pair synchronous cudaMemcpyPeer of
// bfs.cu:595-609 and MPI_Sendrecv of bfs_mpi.cu:614-621.
#include <hip/hip_runtime.h>

#include "launch.hpp"
#include "level_device.hpp"
#include "wave.hpp"

namespace dbfs {
namespace kern {
namespace {

using namespace dev;

constexpr int kBlock = 256;

// Copy `bytes` (a multiple of `unit`, 4 / 8 / 16) with every thread of the
// grid; `t` / `nt` = global thread index / count.
__device__ __forceinline__ void grid_copy(void* __restrict__ dst, const void* __restrict__ src, int64_t bytes, int unit,
                                          int64_t t, int64_t nt) {
  if (unit == 16) {
    uint4* d = static_cast<uint4*>(dst);
    const uint4* s = static_cast<const uint4*>(src);
    for (int64_t i = t; i < bytes / 16; i += nt) d[i] = s[i];
  } else if (unit == 8) {
    uint64_t* d = static_cast<uint64_t*>(dst);
    const uint64_t* s = static_cast<const uint64_t*>(src);
    for (int64_t i = t; i < bytes / 8; i += nt) d[i] = s[i];
  } else {
    uint32_t* d = static_cast<uint32_t*>(dst);
    const uint32_t* s = static_cast<const uint32_t*>(src);
    for (int64_t i = t; i < bytes / 4; i += nt) d[i] = s[i];
  }
}

// Bytes of segment 0 for peer p: fixed, or counted from the list's first word
// (n entries after it), rounded up to the copy granule, at most bytes[p].
__device__ __forceinline__ int64_t seg_bytes(int64_t cap, const uint32_t* count, int unit) {
  if (!count || cap <= 0) return cap;
  const int64_t b = (static_cast<int64_t>(*count) + 1) * 4;
  const int64_t r = (b + unit - 1) / unit * unit;
  return r < cap ? r : cap;
}

// The push of every piece by the grid: workgroups are dealt to peers
// round-robin (group g -> peer g % P), so every xGMI link carries its share at
// once instead of the grid streaming to one peer after another.
__device__ __forceinline__ void push_pieces(const PeerPushArgs& a, int nthreads) {
  const int P = a.npeers;
  const int t = threadIdx.x;
  const int groups = static_cast<int>(gridDim.x) / P;
  if (groups > 0) {
    const int p = static_cast<int>(blockIdx.x) % P;
    const int g = static_cast<int>(blockIdx.x) / P;
    if (g < groups) {
      const int64_t gt = static_cast<int64_t>(g) * nthreads + t, nt = static_cast<int64_t>(groups) * nthreads;
      const int64_t b = seg_bytes(a.bytes[p], a.count[p], a.unit);
      if (b > 0) grid_copy(a.dst[p], a.src[p], b, a.unit, gt, nt);
      if (a.bytes2 > 0 && a.dst2[p]) grid_copy(a.dst2[p], a.src2, a.bytes2, a.unit, gt, nt);
    }
  } else {
    const int64_t nt = static_cast<int64_t>(gridDim.x) * nthreads;
    const int64_t gt = static_cast<int64_t>(blockIdx.x) * nthreads + t;
    for (int q = 0; q < P; ++q) {
      const int64_t b = seg_bytes(a.bytes[q], a.count[q], a.unit);
      if (b > 0) grid_copy(a.dst[q], a.src[q], b, a.unit, gt, nt);
      if (a.bytes2 > 0 && a.dst2[q]) grid_copy(a.dst2[q], a.src2, a.bytes2, a.unit, gt, nt);
    }
  }
}

// The unpack of the landed slots (after the flags and an acquire): segment 0
// copied to the caller's buffers, segment 1 summed.
__device__ __forceinline__ void unpack_pieces(const PeerUnpackArgs& a, int64_t gt, int64_t nt) {
  if (a.has_finish) {
    // a level's end: the first workgroup sums the totals (and a hub-split
    // level's hub bits), then finishes the level -- thread 0's decision (the
    // stamp the host and the next level's kernels read), then for a top-down
    // next level its hub-split entries
    if (blockIdx.x == 0) {
      for (int64_t i = threadIdx.x; i < a.sum_count; i += blockDim.x) {
        uint64_t acc = 0;
        for (int p = 0; p < a.npeers; ++p) acc += static_cast<const uint64_t*>(a.sum_src[p])[i];
        static_cast<uint64_t*>(a.sum_out)[i] = acc;
      }
      __syncthreads();
      level_finish_block<kBlock>(a.finish);
    }
  } else if (a.sum_count > 0) {
    // all-reduce: out[i] = sum over ranks of slot[p][i] (wrapping, as RCCL)
    for (int64_t i = gt; i < a.sum_count; i += nt) {
      uint64_t acc = 0;
      for (int p = 0; p < a.npeers; ++p) acc += static_cast<const uint64_t*>(a.sum_src[p])[i];
      static_cast<uint64_t*>(a.sum_out)[i] = acc;
    }
  }
  for (int p = 0; p < a.npeers; ++p) {
    const int64_t b =
        seg_bytes(a.bytes[p], a.counted && a.bytes[p] > 0 ? static_cast<const uint32_t*>(a.src[p]) : nullptr, a.unit);
    if (b > 0) grid_copy(a.dst[p], a.src[p], b, a.unit, gt, nt);
  }
}

__global__ __launch_bounds__(kBlock) void peer_push_kernel(PeerPushArgs a) {
  __shared__ int s_last;
  push_pieces(a, kBlock);
  // every wave's stores complete, then the hand-off (cdna_hip_programming.md
  // Guideline 16, at system scope: the stores went to other GPUs' memory)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = atomicAdd(a.ticket, 1u);
    s_last = prev == gridDim.x - 1 ? 1 : 0;
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!s_last) return;
  if (threadIdx.x < a.npeers && a.flag[threadIdx.x])
    __hip_atomic_store(a.flag[threadIdx.x], a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (threadIdx.x == 0) *a.ticket = 0u;  // next push is stream-ordered after this one
}

// Lane p's wait for flags[p] >= seq (p < npeers, skip_self aside): 1 done,
// 0 timed out (that peer never arrived), -1 another wait of this rank timed
// out first (its error word is set: stop at once instead of spending a
// timeout of our own behind a dead peer).
__device__ __forceinline__ int peer_flag_wait(const PeerWaitArgs& a, int p) {
  const uint64_t t0 = wall_clock64();
  for (uint32_t spin = 0;; ++spin) {
    if (__hip_atomic_load(a.flags + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= a.seq) return 1;
    __builtin_amdgcn_s_sleep(2);
    if ((spin & 255) == 255) {
      if (wall_clock64() - t0 > a.timeout_ticks) return 0;
      if (a.error && __hip_atomic_load(a.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return -1;
    }
  }
}

// The error word of a timed-out wait (backend.hpp kWaitSeqMask): which
// collective, and the peer that never arrived.
__device__ __forceinline__ void peer_wait_error(const PeerWaitArgs& a, int peer) {
  if (a.error)
    __hip_atomic_store(a.error, (a.seq & kWaitSeqMask) | (static_cast<uint64_t>(peer + 1) << 48), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// One wave: lane p waits until flags[p] >= seq (p < npeers, skip_self aside).
__global__ void peer_wait_kernel(PeerWaitArgs a) {
  const int lane = lane_id();
  int st = 1;
  if (lane < a.npeers && lane != a.skip) st = peer_flag_wait(a, lane);
  const unsigned long long late = __ballot(st == 0);
  if (late || !__all(st == 1)) {
    if (lane == 0 && late) peer_wait_error(a, __ffsll(static_cast<long long>(late)) - 1);
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

__global__ __launch_bounds__(kBlock) void peer_unpack_kernel(PeerUnpackArgs a) {
  if (a.error && __hip_atomic_load(a.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return;
  unpack_pieces(a, static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x, static_cast<int64_t>(gridDim.x) * kBlock);
}

// A collective as ONE launch (the three above fused): push by every
// workgroup (groups dealt to peers round-robin), the ticket hand-off whose
// last workgroup publishes the flags behind a system-scope release, then
// every workgroup waits for the peers' flags itself (bounded as
// peer_wait_kernel) and unpacks its share after an acquire.  A workgroup
// waits only for flags: the peers' (which do not depend on this launch), and
// -- when this rank's own all-reduce input goes through its window -- its own,
// published by this launch's last workgroup; the grid (<= kPeerFusedGroups
// per peer) is far below the chip's residency, so that workgroup runs.
constexpr int kFusedThreads = 256;
__global__ __launch_bounds__(kFusedThreads) void peer_fused_kernel(PeerPushArgs pa, PeerWaitArgs wa, PeerUnpackArgs ua) {
  __shared__ int s_last, s_ok, s_late;
  const int t = threadIdx.x;
  const int P = pa.npeers;
  push_pieces(pa, kFusedThreads);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    s_ok = 1;
    s_late = -1;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = atomicAdd(pa.ticket, 1u);
    s_last = prev == gridDim.x - 1 ? 1 : 0;
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (s_last) {
    if (t < P && pa.flag[t]) __hip_atomic_store(pa.flag[t], pa.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (t == 0) *pa.ticket = 0u;  // next collective is stream-ordered after this one
  }
  if (t < wa.npeers && t != wa.skip) {
    const int st = peer_flag_wait(wa, t);
    if (st == 0) s_late = t;  // (benign race: any missing peer names the stall)
    if (st != 1) s_ok = 0;    // (benign race: every writer stores 0)
  }
  __syncthreads();
  if (!s_ok) {
    if (t == 0 && s_late >= 0) peer_wait_error(wa, s_late);
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  unpack_pieces(ua, static_cast<int64_t>(blockIdx.x) * kFusedThreads + t, static_cast<int64_t>(gridDim.x) * kFusedThreads);
}

inline unsigned grid_for_bytes(int64_t bytes, int unit) {
  int64_t g = (bytes / unit + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  if (g > 1024) g = 1024;
  return static_cast<unsigned>(g);
}

}  // namespace

void peer_push(const PeerPushArgs& a, hipStream_t st) {
  int64_t mx = 0;
  for (int p = 0; p < a.npeers; ++p) mx = a.bytes[p] + a.bytes2 > mx ? a.bytes[p] + a.bytes2 : mx;
  // one group of workgroups per peer, sized for the largest piece
  const int64_t per = (mx / a.unit + kBlock - 1) / kBlock;
  const int64_t groups = per < 1 ? 1 : (per > 128 ? 128 : per);
  peer_push_kernel<<<static_cast<unsigned>(groups * a.npeers), kBlock, 0, st>>>(a);
}

void peer_wait(const PeerWaitArgs& a, hipStream_t st) { peer_wait_kernel<<<1, 64, 0, st>>>(a); }

void peer_fused(const PeerPushArgs& push, const PeerWaitArgs& wait, const PeerUnpackArgs& unpack, hipStream_t st) {
  int64_t mx = 0;
  for (int p = 0; p < push.npeers; ++p) mx = push.bytes[p] + push.bytes2 > mx ? push.bytes[p] + push.bytes2 : mx;
  for (int p = 0; p < unpack.npeers; ++p) mx = unpack.bytes[p] > mx ? unpack.bytes[p] : mx;
  if (unpack.sum_count * 8 > mx) mx = unpack.sum_count * 8;
  // one group of workgroups per peer, sized for the largest piece (at most
  // kPeerFusedGroups per peer: the push of 1 MiB per peer keeps every link busy)
  const int64_t per = (mx / push.unit + kFusedThreads - 1) / kFusedThreads;
  const int64_t cap = push.max_groups > 0 && push.max_groups < kPeerFusedGroups ? push.max_groups : kPeerFusedGroups;
  const int64_t groups = per < 1 ? 1 : (per > cap ? cap : per);
  peer_fused_kernel<<<static_cast<unsigned>(groups * push.npeers), kFusedThreads, 0, st>>>(push, wait, unpack);
}

void peer_unpack(const PeerUnpackArgs& a, hipStream_t st) {
  int64_t tot = a.sum_count * 8;
  for (int p = 0; p < a.npeers; ++p) tot += a.bytes[p];
  if (tot <= 0) return;
  peer_unpack_kernel<<<grid_for_bytes(tot, a.unit), kBlock, 0, st>>>(a);
}

}  // namespace kern
}  // namespace dbfs
