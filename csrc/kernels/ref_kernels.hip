// Reference-algorithm mode (the measured MI355X baseline).
//
// A fresh HIP implementation of the reference's live kernel queueBfs
// (bfs.cu:134-165): one thread per frontier vertex walks its adjacency
// serially; a neighbour is claimed with atomicMin on a replicated int distance
// array; the winner appends it to its owner's bucket with one atomicAdd on a
// single counter per bucket.  Defects fixed: owners are in [0, P) for any N
// (D5), bucket capacity is per owner (D2), and received ids are de-duplicated
// by the owner (D4: the reference re-expands duplicates).
#include <hip/hip_runtime.h>

#include "launch.hpp"
#include "wave.hpp"

namespace dbfs {
namespace kern {
namespace {

constexpr int kRefBlock = 256;

__global__ __launch_bounds__(kRefBlock) void ref_expand_kernel(RefExpandArgs a) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kRefBlock + threadIdx.x;
  if (i >= a.q) return;
  const int64_t u = static_cast<int64_t>(a.queue[i]) - a.g.lo;
  for (eid_t e = a.g.row_off[u]; e < a.g.row_off[u + 1]; ++e) {
    const vid_t v = a.g.col[e];
    if (a.dist[v] == kUnreached && atomicMin(&a.dist[v], a.next_level) == kUnreached) {
      const int64_t owner = v / a.part;
      const unsigned long long pos =
          atomicAdd(reinterpret_cast<unsigned long long*>(a.bucket_cnt + owner), 1ull);
      a.buckets[owner * a.bucket_cap + static_cast<int64_t>(pos)] = v;
    }
  }
}

__global__ __launch_bounds__(kRefBlock) void ref_accept_kernel(RefAcceptArgs a) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kRefBlock + threadIdx.x;
  if (i >= a.total) return;
  const vid_t v = a.recv[i];
  bool keep;
  if (i >= a.self_begin && i < a.self_end) {
    keep = true;
  } else {
    keep = a.dist[v] == kUnreached && atomicMin(&a.dist[v], a.next_level) == kUnreached;
  }
  if (keep) {
    const unsigned long long pos = atomicAdd(reinterpret_cast<unsigned long long*>(a.qcount), 1ull);
    a.queue[pos] = v;
  }
}

// ---- scan mode (atomic-free frontier build) --------------
// One wave per frontier vertex; lanes stride its adjacency 64 edges at a time,
// so hubs are split across lanes instead of serialising one thread.  Owner
// grouping inside a 64-edge chunk loops over the distinct owners present
// (readlane + ballot); lane o carries owner o's counter, so nranks <= 64.
constexpr int kScanWavesPerBlock = 4;
constexpr int kScanBlock = kScanWavesPerBlock * dev::kWave;

__device__ __forceinline__ int64_t scan_wave_index() {
  return static_cast<int64_t>(blockIdx.x) * kScanWavesPerBlock + threadIdx.x / dev::kWave;
}

__global__ __launch_bounds__(kScanBlock) void scan_relax_kernel(ScanBfsArgs a) {
  const int64_t i = scan_wave_index();
  if (i >= a.q) return;
  const int64_t u = static_cast<int64_t>(a.queue[i]) - a.g.lo;
  const eid_t b = a.g.row_off[u], end = a.g.row_off[u + 1];
  for (eid_t e = b + dev::lane_id(); e < end; e += dev::kWave) {
    const vid_t v = a.g.col[e];
    // plain stores; concurrent claimers all write the same level and the
    // surviving claim names exactly one of them
    if (a.dist[v] == kUnreached) {
      a.dist[v] = a.next_level;
      a.claim[v] = e;
    }
  }
}

template <bool kAssign>
__global__ __launch_bounds__(kScanBlock) void scan_children_kernel(ScanBfsArgs a) {
  const int64_t i = scan_wave_index();
  if (i >= a.q) return;
  const int lane = dev::lane_id();
  const int64_t u = static_cast<int64_t>(a.queue[i]) - a.g.lo;
  const eid_t b = a.g.row_off[u], end = a.g.row_off[u + 1];
  // lane o keeps owner o's running count (count) / output cursor (assign)
  long long acc = 0;
  if (kAssign && lane < a.nranks) acc = a.offs[static_cast<int64_t>(lane) * a.q + i];
  for (eid_t base = b; base < end; base += dev::kWave) {
    const eid_t e = base + lane;
    int owner = -1;
    vid_t v = 0;
    if (e < end) {
      v = a.g.col[e];
      if (a.dist[v] == a.next_level && a.claim[v] == e) owner = static_cast<int>(v / a.part);
    }
    unsigned long long left = __ballot(owner >= 0);
    while (left) {
      const int leader = __builtin_ctzll(left);
      const int o = __builtin_amdgcn_readlane(owner, leader);
      const unsigned long long m = __ballot(owner == o);
      left &= ~m;
      if (kAssign) {
        const long long pos = dev::readlane_i64(acc, o);
        if (owner == o) a.out[pos + dev::mask_rank(m)] = v;
      }
      if (lane == o) acc += __popcll(m);
    }
  }
  if (!kAssign && lane < a.nranks) a.offs[static_cast<int64_t>(lane) * a.q + i] = acc;
}

__global__ void scan_bounds_kernel(ScanBfsArgs a) {
  for (int o = threadIdx.x; o <= a.nranks; o += blockDim.x) a.bounds[o] = a.offs[static_cast<int64_t>(o) * a.q];
  __syncthreads();
  for (int o = threadIdx.x; o < a.nranks; o += blockDim.x) a.counts[o] = a.bounds[o + 1] - a.bounds[o];
}

inline unsigned scan_grid(int64_t q) {
  return static_cast<unsigned>((q + kScanWavesPerBlock - 1) / kScanWavesPerBlock);
}

}  // namespace

void scan_relax(const ScanBfsArgs& a, hipStream_t st) {
  if (a.q <= 0) return;
  scan_relax_kernel<<<scan_grid(a.q), kScanBlock, 0, st>>>(a);
}

void scan_count(const ScanBfsArgs& a, hipStream_t st) {
  if (a.q <= 0) return;
  scan_children_kernel<false><<<scan_grid(a.q), kScanBlock, 0, st>>>(a);
}

void scan_bounds(const ScanBfsArgs& a, hipStream_t st) { scan_bounds_kernel<<<1, 64, 0, st>>>(a); }

void scan_assign(const ScanBfsArgs& a, hipStream_t st) {
  if (a.q <= 0) return;
  scan_children_kernel<true><<<scan_grid(a.q), kScanBlock, 0, st>>>(a);
}

void ref_expand(const RefExpandArgs& a, hipStream_t st) {
  if (a.q <= 0) return;
  ref_expand_kernel<<<static_cast<unsigned>((a.q + kRefBlock - 1) / kRefBlock), kRefBlock, 0, st>>>(a);
}

void ref_accept(const RefAcceptArgs& a, hipStream_t st) {
  if (a.total <= 0) return;
  ref_accept_kernel<<<static_cast<unsigned>((a.total + kRefBlock - 1) / kRefBlock), kRefBlock, 0, st>>>(a);
}

}  // namespace kern
}  // namespace dbfs
