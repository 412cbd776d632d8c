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

}  // namespace

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
