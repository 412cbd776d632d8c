// gfx950 graph-construction and validation kernels.
//
// The reference builds its CSR on the host from vector<vector<int>> and then
// copies the FULL graph to every device (bfs.cu:346-351).  Here a
// rank builds only its own shard on its own GPU, straight from the
// counter-based generator (dbfs/rmat.hpp): pass 1 counts owned endpoint
// degrees (device atomics), an exclusive scan turns degrees into row offsets,
// pass 2 regenerates the same edges and scatters them (atomic cursors).  No
// edge list is ever materialised, so RMAT-27 on 8 GPUs needs only the shard.
#include <hip/hip_runtime.h>

#include "launch.hpp"
#include "wave.hpp"

namespace dbfs {
namespace kern {
namespace {

using namespace dev;

constexpr int kBlock = 256;
constexpr int kScanItems = 16;
constexpr int kScanTile = kBlock * kScanItems;

__global__ __launch_bounds__(kBlock) void gen_count_kernel(GenParams p, int64_t lo, int64_t rows,
                                                          unsigned long long* __restrict__ deg) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < p.m; i += stride) {
    uint64_t u, v;
    gen_edge(p, static_cast<uint64_t>(i), u, v);
    const uint64_t ur = u - static_cast<uint64_t>(lo), vr = v - static_cast<uint64_t>(lo);
    if (ur < static_cast<uint64_t>(rows)) atomicAdd(deg + ur, 1ull);
    if (vr < static_cast<uint64_t>(rows)) atomicAdd(deg + vr, 1ull);
  }
}

__global__ __launch_bounds__(kBlock) void gen_fill_kernel(GenParams p, int64_t lo, int64_t rows,
                                                         unsigned long long* __restrict__ cursor,
                                                         vid_t* __restrict__ col) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < p.m; i += stride) {
    uint64_t u, v;
    gen_edge(p, static_cast<uint64_t>(i), u, v);
    const uint64_t ur = u - static_cast<uint64_t>(lo), vr = v - static_cast<uint64_t>(lo);
    if (ur < static_cast<uint64_t>(rows)) col[atomicAdd(cursor + ur, 1ull)] = static_cast<vid_t>(v);
    if (vr < static_cast<uint64_t>(rows)) col[atomicAdd(cursor + vr, 1ull)] = static_cast<vid_t>(u);
  }
}

// ---- CSR build from a file's edges (DeviceGraph::from_edges) ----------------
// Every input edge (u, v) yields the entries u -> v (owned by rank u / part) and
// v -> u (rank v / part).  Pass 1 counts the entries per destination rank,
// pass 2 scatters them into per-rank segments of the send buffer; both count
// in LDS first and touch the global counters once per workgroup and rank
// (device-scope atomics run at the memory side on MI355X: one per entry would
// cost more than the whole build).  Entry = row << 32 | neighbour.
constexpr int kMaxRouteRanks = 1024;

__global__ __launch_bounds__(kBlock) void route_count_kernel(const vid_t* __restrict__ u, const vid_t* __restrict__ v,
                                                            int64_t m, int64_t part, int nranks,
                                                            unsigned long long* __restrict__ counts) {
  __shared__ unsigned s_cnt[kMaxRouteRanks];
  for (int r = threadIdx.x; r < nranks; r += kBlock) s_cnt[r] = 0;
  __syncthreads();
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < m; i += stride) {
    atomicAdd(&s_cnt[u[i] / part], 1u);
    atomicAdd(&s_cnt[v[i] / part], 1u);
  }
  __syncthreads();
  for (int r = threadIdx.x; r < nranks; r += kBlock)
    if (s_cnt[r]) atomicAdd(counts + r, static_cast<unsigned long long>(s_cnt[r]));
}

// One tile of kBlock edges per step: LDS counts -> one reservation per rank
// -> stores.
__global__ __launch_bounds__(kBlock) void route_fill_kernel(const vid_t* __restrict__ u, const vid_t* __restrict__ v,
                                                           int64_t m, int64_t part, int nranks,
                                                           unsigned long long* __restrict__ cursor,
                                                           unsigned long long* __restrict__ out) {
  __shared__ unsigned s_cnt[kMaxRouteRanks];
  __shared__ unsigned long long s_base[kMaxRouteRanks];
  for (int64_t t0 = static_cast<int64_t>(blockIdx.x) * kBlock; t0 < m; t0 += static_cast<int64_t>(gridDim.x) * kBlock) {
    for (int r = threadIdx.x; r < nranks; r += kBlock) s_cnt[r] = 0;
    __syncthreads();
    const int64_t i = t0 + threadIdx.x;
    int ra = -1, rb = -1;
    unsigned ka = 0, kb = 0;
    vid_t a = 0, b = 0;
    if (i < m) {
      a = u[i];
      b = v[i];
      ra = static_cast<int>(a / part);
      rb = static_cast<int>(b / part);
      ka = atomicAdd(&s_cnt[ra], 1u);
      kb = atomicAdd(&s_cnt[rb], 1u);
    }
    __syncthreads();
    for (int r = threadIdx.x; r < nranks; r += kBlock)
      s_base[r] = s_cnt[r] ? atomicAdd(cursor + r, static_cast<unsigned long long>(s_cnt[r])) : 0ull;
    __syncthreads();
    if (i < m) {
      out[s_base[ra] + ka] = (static_cast<unsigned long long>(a) << 32) | b;
      out[s_base[rb] + kb] = (static_cast<unsigned long long>(b) << 32) | a;
    }
    __syncthreads();
  }
}

// Received entries -> row degrees of the shard (rows [lo, lo + rows)).
__global__ __launch_bounds__(kBlock) void entries_count_kernel(const unsigned long long* __restrict__ e, int64_t k,
                                                              int64_t lo, unsigned long long* __restrict__ deg) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < k; i += stride)
    atomicAdd(deg + (static_cast<int64_t>(e[i] >> 32) - lo), 1ull);
}

__global__ __launch_bounds__(kBlock) void entries_fill_kernel(const unsigned long long* __restrict__ e, int64_t k,
                                                             int64_t lo, unsigned long long* __restrict__ cursor,
                                                             vid_t* __restrict__ col) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < k; i += stride) {
    const unsigned long long x = e[i];
    col[atomicAdd(cursor + (static_cast<int64_t>(x >> 32) - lo), 1ull)] = static_cast<vid_t>(x & 0xFFFFFFFFull);
  }
}

// Block-wide exclusive scan of `items` (kScanItems per thread, blocked layout).
__device__ long long block_excl_scan(long long (&items)[kScanItems], long long* s_wave, long long& total) {
  long long sum = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const long long x = items[k];
    items[k] = sum;
    sum += x;
  }
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  const long long incl = wave_incl_scan(sum);
  if (lane == kWave - 1) s_wave[wv] = incl;
  __syncthreads();
  long long off = incl - sum;
  total = 0;
  for (int k = 0; k < kBlock / kWave; ++k) {
    if (k < wv) off += s_wave[k];
    total += s_wave[k];
  }
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) items[k] += off;
  return off;
}

__global__ __launch_bounds__(kBlock) void scan_single_kernel(eid_t* data, int64_t n) {
  __shared__ long long s_wave[kBlock / kWave];
  long long items[kScanItems];
  const int64_t base = static_cast<int64_t>(threadIdx.x) * kScanItems;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) items[k] = (base + k < n) ? data[base + k] : 0;
  long long total;
  block_excl_scan(items, s_wave, total);
#pragma unroll
  for (int k = 0; k < kScanItems; ++k)
    if (base + k < n) data[base + k] = items[k];
  if (threadIdx.x == 0) data[n] = total;
}

__global__ __launch_bounds__(kBlock) void scan_reduce_kernel(const eid_t* __restrict__ data, int64_t n,
                                                            eid_t* __restrict__ sums) {
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kScanTile;
  long long s = 0;
  for (int k = threadIdx.x; k < kScanTile; k += kBlock) {
    const int64_t i = base + k;
    if (i < n) s += data[i];
  }
  s = wave_sum(s);
  __shared__ long long s_wave[kBlock / kWave];
  if (lane_id() == 0) s_wave[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long t = 0;
    for (int k = 0; k < kBlock / kWave; ++k) t += s_wave[k];
    sums[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kBlock) void scan_apply_kernel(eid_t* data, int64_t n, const eid_t* __restrict__ offs,
                                                           int64_t nb) {
  __shared__ long long s_wave[kBlock / kWave];
  long long items[kScanItems];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kScanTile + static_cast<int64_t>(threadIdx.x) * kScanItems;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) items[k] = (base + k < n) ? data[base + k] : 0;
  long long total;
  block_excl_scan(items, s_wave, total);
  const long long off = offs[blockIdx.x];
#pragma unroll
  for (int k = 0; k < kScanItems; ++k)
    if (base + k < n) data[base + k] = items[k] + off;
  if (blockIdx.x == 0 && threadIdx.x == 0) data[n] = offs[nb];
}

// Thread per vertex for rows of at most kValidateLong entries; longer rows
// (RMAT hubs: up to millions of entries, which one thread scanned alone for
// ~88 ms on RMAT-22) are taken by the whole wave, 64 entries per step.
constexpr int64_t kValidateLong = 64;

__device__ __forceinline__ void validate_edge(lvl_t lu, lvl_t lv, long long& gap, long long& cross, bool& parent) {
  if (lu == kUnreached && lv == kUnreached) return;
  if ((lu == kUnreached) != (lv == kUnreached)) {
    ++cross;
    return;
  }
  if (lu - lv > 1 || lv - lu > 1) ++gap;
  if (lv == lu - 1) parent = true;
}

__global__ __launch_bounds__(kBlock) void validate_kernel(ValidateArgs a) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  const int lane = lane_id();
  const bool valid = r < a.g.rows;
  const int64_t u = a.g.lo + r;
  const lvl_t lu = valid ? a.level_global[u] : kUnreached;
  const eid_t b = valid ? a.g.row_off[r] : 0, e = valid ? a.g.row_off[r + 1] : 0;
  const bool longrow = e - b > kValidateLong;
  long long gap = 0, cross = 0, orphan = 0;
  bool has_parent = false;
  if (valid && !longrow)
    for (eid_t i = b; i < e; ++i) validate_edge(lu, a.level_global[a.g.col[i]], gap, cross, has_parent);
  // long rows: one at a time, the wave's lanes over its entries
  unsigned long long pending = __ballot(valid && longrow);
  while (pending) {
    const int leader = __ffsll(static_cast<long long>(pending)) - 1;
    pending &= pending - 1;
    const eid_t lb = __shfl(b, leader, kWave), le = __shfl(e, leader, kWave);
    const lvl_t llu = __shfl(lu, leader, kWave);
    bool par = false;
    for (eid_t i = lb + lane; i < le; i += kWave) validate_edge(llu, a.level_global[a.g.col[i]], gap, cross, par);
    if (__ballot(par) && lane == leader) has_parent = true;
  }
  if (valid) {
    if (lu != kUnreached && u != a.src && !has_parent) orphan = 1;
    if (u == a.src && lu != 0) orphan = 1;
  }
  if (gap) atomicAdd(reinterpret_cast<unsigned long long*>(a.out + 0), static_cast<unsigned long long>(gap));
  if (cross) atomicAdd(reinterpret_cast<unsigned long long*>(a.out + 1), static_cast<unsigned long long>(cross));
  if (orphan) atomicAdd(reinterpret_cast<unsigned long long*>(a.out + 2), 1ull);
}

// One wave per owned vertex: 64 neighbours per step, first match by ballot.
__global__ __launch_bounds__(kBlock) void parent_kernel(ParentArgs a) {
  const int lane = lane_id();
  const int64_t r = static_cast<int64_t>(blockIdx.x) * (kBlock / kWave) + (threadIdx.x >> 6);
  if (r >= a.g.rows) return;
  const int64_t v = a.g.lo + r;
  const lvl_t lv = a.level_global[v];
  if (v == a.src || lv == kUnreached) {
    if (lane == 0) a.parent[r] = (v == a.src) ? v : -1;
    return;
  }
  const eid_t b = a.g.row_off[r], e = a.g.row_off[r + 1];
  long long par = -1;
  for (eid_t base = b; base < e; base += kWave) {
    const eid_t idx = base + lane;
    vid_t u = 0;
    bool hit = false;
    if (idx < e) {
      u = a.g.col[idx];
      hit = a.level_global[u] == lv - 1;
    }
    const unsigned long long m = __ballot(hit);
    if (m) {
      const int l = __ffsll(static_cast<long long>(m)) - 1;
      // (ids up to 2^32 - 1: shuffled as unsigned, widened without sign)
      par = static_cast<long long>(static_cast<unsigned>(__shfl(static_cast<int>(u), l, kWave)));
      break;
    }
  }
  if (lane == 0) a.parent[r] = par;
}

__global__ __launch_bounds__(kBlock) void reached_deg_kernel(ShardView g, const lvl_t* __restrict__ level,
                                                            int64_t* out2) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  long long c = 0, d = 0;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; r < g.rows; r += stride) {
    if (level[r] != kUnreached) { ++c; d += g.row_off[r + 1] - g.row_off[r]; }
  }
  c = wave_sum(c);
  d = wave_sum(d);
  if (lane_id() == 0) {
    if (c) atomicAdd(reinterpret_cast<unsigned long long*>(out2 + 0), static_cast<unsigned long long>(c));
    if (d) atomicAdd(reinterpret_cast<unsigned long long*>(out2 + 1), static_cast<unsigned long long>(d));
  }
}

__global__ __launch_bounds__(kBlock) void degree_moments_kernel(ShardView g, int64_t* out2) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  long long s = 0, c = 0;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; r < g.rows; r += stride) {
    const long long d = g.row_off[r + 1] - g.row_off[r];
    s += d * d;
    c += d > 0 ? 1 : 0;
  }
  s = wave_sum(s);
  c = wave_sum(c);
  if (lane_id() == 0 && s) atomicAdd(reinterpret_cast<unsigned long long*>(out2), static_cast<unsigned long long>(s));
  if (lane_id() == 0 && c) atomicAdd(reinterpret_cast<unsigned long long*>(out2 + 1), static_cast<unsigned long long>(c));
}

inline unsigned capped_grid(int64_t work, int64_t cap) {
  int64_t g = (work + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return static_cast<unsigned>(g);
}

}  // namespace

void gen_count_degrees(const GenParams& p, int64_t lo, int64_t rows, eid_t* deg, hipStream_t st) {
  if (p.m <= 0 || rows <= 0) return;
  gen_count_kernel<<<capped_grid(p.m, 256 * 32), kBlock, 0, st>>>(p, lo, rows,
                                                                  reinterpret_cast<unsigned long long*>(deg));
}

void gen_fill(const GenParams& p, int64_t lo, int64_t rows, eid_t* cursor, vid_t* col, hipStream_t st) {
  if (p.m <= 0 || rows <= 0) return;
  gen_fill_kernel<<<capped_grid(p.m, 256 * 32), kBlock, 0, st>>>(
      p, lo, rows, reinterpret_cast<unsigned long long*>(cursor), col);
}

void route_edges_count(const vid_t* u, const vid_t* v, int64_t m, int64_t part, int nranks, int64_t* counts,
                       hipStream_t st) {
  if (m <= 0) return;
  route_count_kernel<<<capped_grid(m, 256 * 16), kBlock, 0, st>>>(u, v, m, part, nranks,
                                                                  reinterpret_cast<unsigned long long*>(counts));
}

void route_edges_fill(const vid_t* u, const vid_t* v, int64_t m, int64_t part, int nranks, int64_t* cursor,
                      uint64_t* out, hipStream_t st) {
  if (m <= 0) return;
  route_fill_kernel<<<capped_grid(m, 256 * 16), kBlock, 0, st>>>(
      u, v, m, part, nranks, reinterpret_cast<unsigned long long*>(cursor), reinterpret_cast<unsigned long long*>(out));
}

void entries_count(const uint64_t* e, int64_t k, int64_t lo, eid_t* deg, hipStream_t st) {
  if (k <= 0) return;
  entries_count_kernel<<<capped_grid(k, 256 * 32), kBlock, 0, st>>>(
      reinterpret_cast<const unsigned long long*>(e), k, lo, reinterpret_cast<unsigned long long*>(deg));
}

void entries_fill(const uint64_t* e, int64_t k, int64_t lo, eid_t* cursor, vid_t* col, hipStream_t st) {
  if (k <= 0) return;
  entries_fill_kernel<<<capped_grid(k, 256 * 32), kBlock, 0, st>>>(
      reinterpret_cast<const unsigned long long*>(e), k, lo, reinterpret_cast<unsigned long long*>(cursor), col);
}

int route_max_ranks() { return kMaxRouteRanks; }

int64_t scan_tmp_elems(int64_t n) {
  int64_t total = 0;
  while (n > kScanTile) {
    const int64_t nb = (n + kScanTile - 1) / kScanTile;
    total += nb + 1;
    n = nb;
  }
  return total + 1;
}

void exclusive_scan(eid_t* data, int64_t n, eid_t* tmp, hipStream_t st) {
  if (n <= kScanTile) {
    scan_single_kernel<<<1, kBlock, 0, st>>>(data, n);
    return;
  }
  const int64_t nb = (n + kScanTile - 1) / kScanTile;
  scan_reduce_kernel<<<static_cast<unsigned>(nb), kBlock, 0, st>>>(data, n, tmp);
  exclusive_scan(tmp, nb, tmp + nb + 1, st);
  scan_apply_kernel<<<static_cast<unsigned>(nb), kBlock, 0, st>>>(data, n, tmp, nb);
}

void validate_levels(const ValidateArgs& a, hipStream_t st) {
  if (a.g.rows <= 0) return;
  validate_kernel<<<static_cast<unsigned>((a.g.rows + kBlock - 1) / kBlock), kBlock, 0, st>>>(a);
}

void compute_parents(const ParentArgs& a, hipStream_t st) {
  if (a.g.rows <= 0) return;
  const int64_t wpb = kBlock / kWave;
  parent_kernel<<<static_cast<unsigned>((a.g.rows + wpb - 1) / wpb), kBlock, 0, st>>>(a);
}

void degree_moments(const ShardView& g, int64_t* out2, hipStream_t st) {
  if (g.rows <= 0) return;
  degree_moments_kernel<<<capped_grid(g.rows, 4096), kBlock, 0, st>>>(g, out2);
}

void reached_degree_sum(const ShardView& g, const lvl_t* level, int64_t* out2, hipStream_t st) {
  if (g.rows <= 0) return;
  reached_deg_kernel<<<capped_grid(g.rows, 4096), kBlock, 0, st>>>(g, level, out2);
}

}  // namespace kern
}  // namespace dbfs
