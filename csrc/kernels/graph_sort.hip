// Hub-first adjacency ordering (one-time graph preprocessing, untimed like the
// reference's CSR construction bfs.cu:829-880).
//
// Every row is sorted by (neighbour degree descending, neighbour id
// ascending).  The bottom-up step probes a vertex's neighbours in row order and
// stops at the first frontier member; frontier members at the dominant
// bottom-up level are overwhelmingly hubs, so hub-first rows cut the probes per
// vertex (RMAT-20, BFS level 2: first-probe hit rate 39% -> 76%) and the probes
// that remain hit a small, cache-resident set of hub bitmap words.
//
// Rows of 2..64 entries: one wave per row, 64-lane bitonic sort on 64-bit keys
// with __shfl_xor (no LDS).  Rows of 65..4096 entries: one workgroup per row,
// LDS bitonic sort (rows listed first by an atomic-append pass).  Longer rows
// (hubs, a handful) keep their order: hubs are visited in the first levels and
// their rows are never probed bottom-up.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "launch.hpp"
#include "wave.hpp"

namespace dbfs {
namespace kern {
namespace {

using namespace dev;

constexpr int kBlock = 256;
constexpr int kMaxLds = kSortedRowMax;

__device__ __forceinline__ unsigned long long sort_key(uint32_t deg, vid_t v) {
  return (static_cast<unsigned long long>(0xFFFFFFFFu - deg) << 32) | v;
}
// key_deg == nullptr: plain id order (top-down copy of the adjacency)
__device__ __forceinline__ unsigned long long row_key(const uint32_t* __restrict__ key_deg, vid_t v) {
  return sort_key(key_deg ? key_deg[v] : 0u, v);
}

__global__ __launch_bounds__(kBlock) void degrees_kernel(const eid_t* __restrict__ ro, int64_t rows,
                                                        uint32_t* __restrict__ out) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (r < rows) {
    const eid_t d = ro[r + 1] - ro[r];
    out[r] = d > 0xFFFFFFFFll ? 0xFFFFFFFFu : static_cast<uint32_t>(d);
  }
}

// Wave-per-row bitonic sort for rows of 2..64 entries (grid-stride over rows).
__global__ __launch_bounds__(kBlock) void sort_short_rows_kernel(const eid_t* __restrict__ ro, vid_t* __restrict__ col,
                                                                int64_t rows, const uint32_t* __restrict__ key_deg) {
  const int lane = lane_id();
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * (kBlock / kWave);
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * (kBlock / kWave) + (threadIdx.x >> 6); r < rows;
       r += nwaves) {
    const eid_t b = ro[r], e = ro[r + 1];
    const int64_t len = e - b;
    if (len < 2 || len > kWave) continue;
    unsigned long long k = ~0ull;
    if (lane < len) {
      const vid_t v = col[b + lane];
      k = row_key(key_deg, v);
    }
#pragma unroll
    for (int size = 2; size <= kWave; size <<= 1) {
#pragma unroll
      for (int j = size >> 1; j > 0; j >>= 1) {
        const unsigned long long o = __shfl_xor(k, j, kWave);
        const bool up = (lane & size) == 0;
        const bool lower = (lane & j) == 0;
        k = (lower == up) ? (k < o ? k : o) : (k > o ? k : o);
      }
    }
    if (lane < len) col[b + lane] = static_cast<vid_t>(k & 0xFFFFFFFFull);
  }
}

__global__ __launch_bounds__(kBlock) void list_medium_rows_kernel(const eid_t* __restrict__ ro, int64_t rows,
                                                                 int64_t* __restrict__ list,
                                                                 unsigned long long* __restrict__ count) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (r >= rows) return;
  const eid_t len = ro[r + 1] - ro[r];
  if (len > kWave && len <= kMaxLds) list[atomicAdd(count, 1ull)] = r;
}

__global__ __launch_bounds__(kBlock) void sort_medium_rows_kernel(const eid_t* __restrict__ ro, vid_t* __restrict__ col,
                                                                 const int64_t* __restrict__ list,
                                                                 const unsigned long long* __restrict__ count,
                                                                 const uint32_t* __restrict__ key_deg) {
  __shared__ unsigned long long s[kMaxLds];
  const unsigned long long nrows = *count;
  for (unsigned long long i = blockIdx.x; i < nrows; i += gridDim.x) {
    const int64_t r = list[i];
    const eid_t b = ro[r];
    const int len = static_cast<int>(ro[r + 1] - b);
    int n2 = 1;
    while (n2 < len) n2 <<= 1;
    for (int t = threadIdx.x; t < n2; t += kBlock) {
      if (t < len) {
        const vid_t v = col[b + t];
        s[t] = row_key(key_deg, v);
      } else {
        s[t] = ~0ull;
      }
    }
    __syncthreads();
    for (int size = 2; size <= n2; size <<= 1) {
      for (int j = size >> 1; j > 0; j >>= 1) {
        for (int t = threadIdx.x; t < n2; t += kBlock) {
          const int o = t ^ j;
          if (o > t) {
            const unsigned long long x = s[t], y = s[o];
            const bool up = (t & size) == 0;
            if ((x > y) == up) {
              s[t] = y;
              s[o] = x;
            }
          }
        }
        __syncthreads();
      }
    }
    for (int t = threadIdx.x; t < len; t += kBlock) col[b + t] = static_cast<vid_t>(s[t] & 0xFFFFFFFFull);
    __syncthreads();
  }
}

// Rows longer than kMaxLds in id order, approximately: a counting sort by the
// top 12 bits of the id range (4096 buckets, one workgroup per row, LDS
// histogram, scatter through `tmp`, copy back).  Within a bucket ids stay in
// arrival order; a bucket spans n / 4096 ids, so a top-down sweep of a hub's
// row walks the visited bitmap monotonically one bucket (<= a few cache lines
// at RMAT-22 ... 26) at a time.
constexpr int kLongThreads = 1024;
constexpr int kBuckets = 4096;

__global__ __launch_bounds__(kBlock) void list_long_rows_kernel(const eid_t* __restrict__ ro, int64_t rows,
                                                               int64_t* __restrict__ list,
                                                               unsigned long long* __restrict__ count) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (r >= rows) return;
  if (ro[r + 1] - ro[r] > kMaxLds) list[atomicAdd(count, 1ull)] = r;
}

__global__ __launch_bounds__(kLongThreads) void bucket_long_rows_kernel(const eid_t* __restrict__ ro,
                                                                       vid_t* __restrict__ col,
                                                                       const int64_t* __restrict__ list,
                                                                       const unsigned long long* __restrict__ count,
                                                                       vid_t* __restrict__ tmp, int shift) {
  __shared__ unsigned s_pos[kBuckets];
  __shared__ unsigned s_wave[kLongThreads / kWave];
  constexpr int kPer = kBuckets / kLongThreads;
  const unsigned long long nrows = *count;
  const int t = threadIdx.x;
  for (unsigned long long i = blockIdx.x; i < nrows; i += gridDim.x) {
    const int64_t r = list[i];
    const eid_t b = ro[r], e = ro[r + 1];
    for (int k = t; k < kBuckets; k += kLongThreads) s_pos[k] = 0;
    __syncthreads();
    for (eid_t x = b + t; x < e; x += kLongThreads) atomicAdd(&s_pos[col[x] >> shift], 1u);
    __syncthreads();
    // exclusive scan of the 4096 bucket sizes (kPer consecutive per thread)
    unsigned loc[kPer], sum = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      loc[k] = sum;
      sum += s_pos[t * kPer + k];
    }
    const unsigned incl = static_cast<unsigned>(wave_incl_scan(static_cast<long long>(sum)));
    if (lane_id() == kWave - 1) s_wave[t >> 6] = incl;
    __syncthreads();
    unsigned off = incl - sum;
    for (int w = 0; w < (t >> 6); ++w) off += s_wave[w];
#pragma unroll
    for (int k = 0; k < kPer; ++k) s_pos[t * kPer + k] = off + loc[k];
    __syncthreads();
    for (eid_t x = b + t; x < e; x += kLongThreads) {
      const vid_t v = col[x];
      tmp[b + atomicAdd(&s_pos[v >> shift], 1u)] = v;
    }
    __syncthreads();
    for (eid_t x = b + t; x < e; x += kLongThreads) col[x] = tmp[x];
    __syncthreads();
  }
}

__global__ __launch_bounds__(kBlock) void row_heads_kernel(const eid_t* __restrict__ ro, const vid_t* __restrict__ col,
                                                          int64_t rows, vid_t* __restrict__ head,
                                                          const uint32_t* __restrict__ hub_idx) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (r >= rows) return;
  vid_t h = 0;
  if (ro[r + 1] > ro[r]) {
    h = col[ro[r]];
    if (hub_idx) {
      const uint32_t k = hub_idx[h];
      if (k != 0xFFFFFFFFu) h = kHubFlag | k;
    }
  }
  head[r] = h;
}

__global__ __launch_bounds__(kBlock) void encode_hub_cols_kernel(const vid_t* __restrict__ col, int64_t nnz,
                                                                const uint32_t* __restrict__ hub_idx,
                                                                vid_t* __restrict__ out) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e < nnz; e += stride) {
    const vid_t v = col[e];
    const uint32_t k = hub_idx[v];
    out[e] = k != 0xFFFFFFFFu ? (kHubFlag | k) : v;
  }
}

// Non-empty rows per bitmap word: one wave per word.
__global__ __launch_bounds__(kBlock) void nz_count_kernel(const eid_t* __restrict__ ro, int64_t rows, int64_t words,
                                                         eid_t* __restrict__ counts) {
  const int64_t w = static_cast<int64_t>(blockIdx.x) * (kBlock / kWave) + (threadIdx.x >> 6);
  if (w >= words) return;
  const int64_t v = w * kWave + lane_id();
  const bool nz = v < rows && ro[v + 1] > ro[v];
  const unsigned long long m = __ballot(nz);
  if (lane_id() == 0) counts[w] = __popcll(m);
}

__global__ __launch_bounds__(kBlock) void nz_fill_kernel(const eid_t* __restrict__ ro, const vid_t* __restrict__ head,
                                                        int64_t rows, int64_t words, const eid_t* __restrict__ pref,
                                                        eid_t* __restrict__ nz_ro, vid_t* __restrict__ nz_head) {
  const int64_t w = static_cast<int64_t>(blockIdx.x) * (kBlock / kWave) + (threadIdx.x >> 6);
  if (w >= words) return;
  const int64_t v = w * kWave + lane_id();
  const bool nz = v < rows && ro[v + 1] > ro[v];
  const unsigned long long m = __ballot(nz);
  if (nz) {
    const int64_t k = pref[w] + mask_rank(m);
    nz_ro[k] = ro[v];
    nz_head[k] = head[v];
  }
  if (w == words - 1 && lane_id() == 0) nz_ro[pref[words]] = ro[rows];
}

// Packed records of the non-empty-row view: row k of unit U (vertices
// [4096 U, 4096 U + 4096)) -> {row start - unit_base[U], head}.
__global__ __launch_bounds__(kBlock) void nz_rec_kernel(const eid_t* __restrict__ ro, const vid_t* __restrict__ head,
                                                       int64_t rows, int64_t words, const eid_t* __restrict__ pref,
                                                       NzRec* __restrict__ rec) {
  const int64_t w = static_cast<int64_t>(blockIdx.x) * (kBlock / kWave) + (threadIdx.x >> 6);
  if (w >= words) return;
  const int64_t v = w * kWave + lane_id();
  const bool nz = v < rows && ro[v + 1] > ro[v];
  const unsigned long long m = __ballot(nz);
  if (nz) {
    const int64_t k = pref[w] + mask_rank(m);
    NzRec r;
    r.off = static_cast<uint32_t>(ro[v] - ro[(v / kUnitVertices) * kUnitVertices]);
    r.head = head[v];
    rec[k] = r;
  }
}

__global__ __launch_bounds__(kBlock) void unit_base_kernel(const eid_t* __restrict__ ro, int64_t rows, int64_t nunits,
                                                          eid_t* __restrict__ unit_base) {
  const int64_t u = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (u <= nunits) unit_base[u] = ro[min(u * kUnitVertices, rows)];
}

// Hubs = vertices of degree >= min_deg, indexed in wave-ballot order (one
// atomic per wave).
// Hub selection in two passes so that every rank numbers the hubs alike (hub
// index = number of hubs with a smaller vertex id): the split bottom-up levels
// of several ranks all-reduce hub frontier bits by index.
// Pass 1: hubs per 64-vertex word.
__global__ __launch_bounds__(kBlock) void hub_count_kernel(const uint32_t* __restrict__ deg, int64_t n,
                                                          uint32_t min_deg, eid_t* __restrict__ cnt) {
  const int64_t v = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  const unsigned long long m = __ballot(v < n && deg[v] >= min_deg);
  if (lane_id() == 0 && (v >> 6) * 64 < n) cnt[v >> 6] = __popcll(m);
}

// Pass 2 (cnt exclusive-scanned): index = hubs before the word + rank in it.
__global__ __launch_bounds__(kBlock) void hub_assign_kernel(const uint32_t* __restrict__ deg, int64_t n,
                                                           uint32_t min_deg, const eid_t* __restrict__ cnt,
                                                           vid_t* __restrict__ hub_vertex,
                                                           uint32_t* __restrict__ hub_idx) {
  const int64_t v = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  const bool hub = v < n && deg[v] >= min_deg;
  const unsigned long long m = __ballot(hub);
  if (v < n) {
    const unsigned long long slot = static_cast<unsigned long long>(cnt[v >> 6]) + mask_rank(m);
    if (hub) hub_vertex[slot] = static_cast<vid_t>(v);
    hub_idx[v] = hub ? static_cast<uint32_t>(slot) : 0xFFFFFFFFu;
  }
}

}  // namespace

void row_heads(const eid_t* row_off, const vid_t* col, int64_t rows, vid_t* head, const uint32_t* hub_idx,
               hipStream_t st) {
  if (rows <= 0) return;
  row_heads_kernel<<<static_cast<unsigned>((rows + kBlock - 1) / kBlock), kBlock, 0, st>>>(row_off, col, rows, head,
                                                                                          hub_idx);
}

void encode_hub_cols(const vid_t* col, int64_t nnz, const uint32_t* hub_idx, vid_t* out, hipStream_t st) {
  if (nnz <= 0) return;
  encode_hub_cols_kernel<<<static_cast<unsigned>(std::min<int64_t>((nnz + kBlock - 1) / kBlock, 1 << 16)), kBlock, 0,
                           st>>>(col, nnz, hub_idx, out);
}

void nz_word_counts(const eid_t* row_off, int64_t rows, int64_t words, eid_t* counts, hipStream_t st) {
  if (words <= 0) return;
  nz_count_kernel<<<static_cast<unsigned>((words + 3) / 4), kBlock, 0, st>>>(row_off, rows, words, counts);
}

void nz_fill(const eid_t* row_off, const vid_t* head, int64_t rows, int64_t words, const eid_t* nz_pref,
             eid_t* nz_row_off, vid_t* nz_head, hipStream_t st) {
  if (words <= 0) return;
  nz_fill_kernel<<<static_cast<unsigned>((words + 3) / 4), kBlock, 0, st>>>(row_off, head, rows, words, nz_pref,
                                                                          nz_row_off, nz_head);
}

void nz_records(const eid_t* row_off, const vid_t* head, int64_t rows, int64_t words, const eid_t* nz_pref,
                NzRec* rec, eid_t* unit_base, hipStream_t st) {
  if (rows <= 0) return;
  const int64_t nunits = (rows + kUnitVertices - 1) / kUnitVertices;
  unit_base_kernel<<<static_cast<unsigned>((nunits + 1 + kBlock - 1) / kBlock), kBlock, 0, st>>>(row_off, rows, nunits,
                                                                                                unit_base);
  nz_rec_kernel<<<static_cast<unsigned>((words + 3) / 4), kBlock, 0, st>>>(row_off, head, rows, words, nz_pref, rec);
}

void hub_count(const uint32_t* deg, int64_t n, uint32_t min_deg, eid_t* cnt, hipStream_t st) {
  if (n <= 0) return;
  hub_count_kernel<<<static_cast<unsigned>((n + kBlock - 1) / kBlock), kBlock, 0, st>>>(deg, n, min_deg, cnt);
}

void hub_assign(const uint32_t* deg, int64_t n, uint32_t min_deg, const eid_t* cnt, vid_t* hub_vertex,
                uint32_t* hub_idx, hipStream_t st) {
  if (n <= 0) return;
  hub_assign_kernel<<<static_cast<unsigned>((n + kBlock - 1) / kBlock), kBlock, 0, st>>>(deg, n, min_deg, cnt,
                                                                                        hub_vertex, hub_idx);
}

void degrees_u32(const eid_t* row_off, int64_t rows, uint32_t* out, hipStream_t st) {
  if (rows <= 0) return;
  degrees_kernel<<<static_cast<unsigned>((rows + kBlock - 1) / kBlock), kBlock, 0, st>>>(row_off, rows, out);
}

void sort_neighbors(const eid_t* row_off, vid_t* col, int64_t rows, const uint32_t* key_deg, int64_t* list,
                    unsigned long long* count, hipStream_t st) {
  if (rows <= 0) return;
  sort_short_rows_kernel<<<8192, kBlock, 0, st>>>(row_off, col, rows, key_deg);
  (void)hipMemsetAsync(count, 0, sizeof(unsigned long long), st);  // checked by the caller's hipGetLastError
  list_medium_rows_kernel<<<static_cast<unsigned>((rows + kBlock - 1) / kBlock), kBlock, 0, st>>>(row_off, rows,
                                                                                                  list, count);
  sort_medium_rows_kernel<<<4096, kBlock, 0, st>>>(row_off, col, list, count, key_deg);
}

void sort_rows_by_id(const eid_t* row_off, vid_t* col, int64_t rows, int64_t n, int64_t* list,
                     unsigned long long* count, vid_t* tmp, hipStream_t st) {
  if (rows <= 0) return;
  sort_neighbors(row_off, col, rows, nullptr, list, count, st);
  int bits = 0;
  while ((int64_t(1) << bits) < n) ++bits;
  const int shift = bits > 12 ? bits - 12 : 0;
  (void)hipMemsetAsync(count, 0, sizeof(unsigned long long), st);
  list_long_rows_kernel<<<static_cast<unsigned>((rows + kBlock - 1) / kBlock), kBlock, 0, st>>>(row_off, rows, list,
                                                                                                count);
  bucket_long_rows_kernel<<<1024, kLongThreads, 0, st>>>(row_off, col, list, count, tmp, shift);
}

}  // namespace kern
}  // namespace dbfs
