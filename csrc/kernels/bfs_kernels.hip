// gfx950 BFS primitives: frontier update (visited-bitmap update + level write),
// segment scan, frontier compaction (wave prefix sums), load-balanced top-down
// neighbour gather, bottom-up parent search.
//
// Reference counterpart: the single live kernel queueBfs (bfs.cu:134-165) --
// thread-per-frontier-vertex serial neighbour loop, atomicMin claim on an int
// distance array, and one global atomicAdd per discovered vertex on a single
// managed counter per owner bucket.  On CDNA4 that design is bound by (a) load
// imbalance of power-law degrees inside a 64-lane wave and (b) a contended
// device-scope counter (~88 returning atomics/us per word, MI355X_MICROARCH
// "dequeue" row).  Here:
//   * discoveries are bits (atomicOr on a 64-bit word, no counter at all);
//   * the next work list is built by wave prefix sums over bitmap segments
//     (one wave64 ballot per 64 vertices) -- deterministic, atomic-free;
//   * top-down work is split into equal edge ranges per workgroup
//     (kTdEdgesPerBlock) with an LDS owner map, so hubs and leaves cost the same
//     per edge and col[] is read fully coalesced;
//   * bottom-up scans each owned unvisited vertex's neighbours for a frontier
//     bit, per lane for the first few, then wave-cooperatively (64 neighbours per
//     step, ballot early exit) for the long ones.
#include <hip/hip_runtime.h>

#include "launch.hpp"
#include "wave.hpp"

namespace dbfs {
namespace kern {
namespace {

using namespace dev;

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void fill_level_kernel(lvl_t* __restrict__ level, int64_t n, lvl_t value,
                                                           bool aligned16) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  const int64_t n4 = aligned16 ? n / 4 : 0;
  int4* l4 = reinterpret_cast<int4*>(level);
  const int4 v4 = make_int4(value, value, value, value);
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n4; i += stride) l4[i] = v4;
  for (int64_t i = n4 * 4 + static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride)
    level[i] = value;
}

__global__ void set_bit_kernel(word_t* bm, int64_t bit) {
  if (threadIdx.x == 0) bm[bit >> 6] |= 1ull << (bit & 63);
}

// ---------------------------------------------------------------------------
// One wave per segment of 64 words.  Lane l owns word s*64+l for the bitmap
// update; then, for every non-zero new word (ballot over lanes), the wave
// switches to lane-per-vertex so level stores and row_off loads are coalesced.
__global__ __launch_bounds__(kBlock) void update_kernel(UpdateArgs a) {
  const int lane = lane_id();
  const int64_t s = static_cast<int64_t>(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6);
  const int64_t nseg = (a.words + kSegWords - 1) / kSegWords;
  if (s >= nseg) return;
  const int64_t w = s * kSegWords + lane;
  word_t nb = 0;
  if (w < a.words) {
    word_t c = 0;
    for (int r = 0; r < a.nchunks; ++r) c |= a.cand[r * a.cand_stride + w];
    const word_t vis = a.visited[w];
    nb = c & ~vis;
    if (nb) a.visited[w] = vis | nb;
    a.frontier[w] = nb;
  }
  long long cnt = 0, deg = 0;
  unsigned long long nz = __ballot(nb != 0);
  const eid_t* __restrict__ ro = a.g.row_off;
  while (nz) {
    const int j = __ffsll(static_cast<long long>(nz)) - 1;
    nz &= nz - 1;
    const word_t word = readlane64(nb, j);
    if ((word >> lane) & 1ull) {
      const int64_t v = (s * kSegWords + j) * 64 + lane;
      a.level[v] = a.new_level;
      const eid_t d = ro[v + 1] - ro[v];
      if (d > 0) { cnt += 1; deg += d; }
    }
  }
  cnt = wave_sum(cnt);
  deg = wave_sum(deg);
  if (lane == 0) {
    a.seg_cnt[s] = cnt;
    a.seg_deg[s] = deg;
  }
}

// ---------------------------------------------------------------------------
// Single workgroup exclusive scan over the segment counters (nseg is at most
// a few tens of thousands: 4096 vertices per segment).
constexpr int kScanThreads = 1024;
__global__ __launch_bounds__(kScanThreads) void scan_segments_kernel(ScanArgs a) {
  __shared__ long long s_c[kScanThreads / kWave];
  __shared__ long long s_d[kScanThreads / kWave];
  const int t = threadIdx.x;
  const int lane = lane_id();
  const int wv = t >> 6;
  const int64_t per = (a.nseg + kScanThreads - 1) / kScanThreads;
  const int64_t b = t * per;
  const int64_t e = min(a.nseg, b + per);
  long long c = 0, d = 0;
  for (int64_t i = b; i < e; ++i) { c += a.seg_cnt[i]; d += a.seg_deg[i]; }
  const long long ic = wave_incl_scan(c);
  const long long id = wave_incl_scan(d);
  if (lane == kWave - 1) { s_c[wv] = ic; s_d[wv] = id; }
  __syncthreads();
  long long oc = 0, od = 0;
  for (int k = 0; k < wv; ++k) { oc += s_c[k]; od += s_d[k]; }
  long long rc = oc + ic - c, rd = od + id - d;
  for (int64_t i = b; i < e; ++i) {
    const long long tc = a.seg_cnt[i], td = a.seg_deg[i];
    a.seg_cnt[i] = rc;
    a.seg_deg[i] = rd;
    rc += tc;
    rd += td;
  }
  if (t == kScanThreads - 1) {
    a.stats[0] = a.stats[2] = rc;
    a.stats[1] = a.stats[3] = rd;
    a.qscan[rc] = rd;
  }
}

// ---------------------------------------------------------------------------
// Frontier compaction: one wave per segment; per non-zero word, a wave-wide
// ballot gives each set bit its slot (mbcnt) and a wave prefix sum of degrees
// gives its edge offset.  Writes the top-down work list and the per-block start
// entries (blk_vstart) of the edge-balanced expansion.
__global__ __launch_bounds__(kBlock) void compact_kernel(CompactArgs a) {
  const int lane = lane_id();
  const int64_t s = static_cast<int64_t>(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6);
  const int64_t nseg = (a.words + kSegWords - 1) / kSegWords;
  if (s >= nseg) return;
  const int64_t w = s * kSegWords + lane;
  const word_t mine = (w < a.words) ? a.frontier[w] : 0ull;
  long long pos = a.seg_cnt_off[s];
  long long off = a.seg_deg_off[s];
  unsigned long long nz = __ballot(mine != 0);
  const eid_t* __restrict__ ro = a.g.row_off;
  while (nz) {
    const int j = __ffsll(static_cast<long long>(nz)) - 1;
    nz &= nz - 1;
    const word_t word = readlane64(mine, j);
    const int64_t v = (s * kSegWords + j) * 64 + lane;
    eid_t rs = 0, d = 0;
    if ((word >> lane) & 1ull) {
      rs = ro[v];
      d = ro[v + 1] - rs;
    }
    const bool take = d > 0;
    const unsigned long long tm = __ballot(take);
    const long long incl = wave_incl_scan(d);
    if (take) {
      const long long p = pos + mask_rank(tm);
      const long long qs = off + incl - d;
      a.qscan[p] = qs;
      a.qbase[p] = rs - qs;
      for (long long blk = (qs + kTdEdgesPerBlock - 1) / kTdEdgesPerBlock;
           blk * kTdEdgesPerBlock < qs + d; ++blk)
        a.blk_vstart[blk] = static_cast<int32_t>(p);
    }
    pos += __popcll(tm);
    off += readlane_i64(incl, kWave - 1);
  }
}

// ---------------------------------------------------------------------------
// Edge-balanced top-down expansion.  Workgroup b owns frontier edges
// [b*EPB, (b+1)*EPB).  The entries covering that range are [blk_vstart[b],
// blk_vstart[b+1]]; their start positions are scattered into an LDS owner map
// and max-scanned so every edge finds its entry with one LDS read.  col[] is
// then read in 256-lane coalesced sweeps.
__global__ __launch_bounds__(kTdThreads) void td_expand_kernel(TdArgs a) {
  __shared__ int32_t s_owner[kTdEdgesPerBlock];
  __shared__ long long s_base[kTdEdgesPerBlock + 1];
  __shared__ int32_t s_wmax[kTdThreads / kWave];
  const int t = threadIdx.x;
  const int lane = lane_id();
  const int wv = t >> 6;
  const long long e0 = static_cast<long long>(blockIdx.x) * kTdEdgesPerBlock;
  const long long e1 = min(static_cast<long long>(a.m), e0 + kTdEdgesPerBlock);
  const int cnt = static_cast<int>(e1 - e0);
  const long long v0 = a.blk_vstart[blockIdx.x];
  const long long vlast = (blockIdx.x + 1 < gridDim.x) ? a.blk_vstart[blockIdx.x + 1] : a.q - 1;
  const int nv = static_cast<int>(vlast - v0 + 1);

#pragma unroll
  for (int k = 0; k < kTdItems; ++k) s_owner[k * kTdThreads + t] = 0;
  __syncthreads();
  // Invariant (zero-degree vertices are never listed): nv <= EPB + 1.
  for (int i = t; i < nv && i <= kTdEdgesPerBlock; i += kTdThreads) {
    const long long qs = a.qscan[v0 + i];
    s_base[i] = a.qbase[v0 + i];
    const long long p = (qs > e0 ? qs : e0) - e0;
    if (p < cnt) s_owner[p] = i;
  }
  __syncthreads();
  // inclusive max-scan over s_owner: thread t owns entries [t*ITEMS, (t+1)*ITEMS)
  int vals[kTdItems];
  int run = 0;
#pragma unroll
  for (int k = 0; k < kTdItems; ++k) {
    run = max(run, s_owner[t * kTdItems + k]);
    vals[k] = run;
  }
  const int incl = wave_incl_max(run);
  if (lane == kWave - 1) s_wmax[wv] = incl;
  __syncthreads();
  int carry = 0;
  for (int k = 0; k < wv; ++k) carry = max(carry, s_wmax[k]);
  const int prev = __shfl_up(incl, 1, kWave);
  const int excl = lane > 0 ? max(carry, prev) : carry;
#pragma unroll
  for (int k = 0; k < kTdItems; ++k) s_owner[t * kTdItems + k] = max(vals[k], excl);
  __syncthreads();

  const vid_t* __restrict__ col = a.g.col;
  const word_t* __restrict__ visited = a.visited;
#pragma unroll
  for (int k = 0; k < kTdItems; ++k) {
    const int idx = k * kTdThreads + t;
    if (idx < cnt) {
      const int i = s_owner[idx];
      const vid_t v = col[e0 + idx + s_base[i]];
      const word_t bit = 1ull << (v & 63);
      if (!(visited[v >> 6] & bit)) atomicOr(a.next + (v >> 6), bit);
    }
  }
}

// ---------------------------------------------------------------------------
// Bottom-up parent search: one wave per owned bitmap word (64 vertices).
// Phase 1: each unvisited lane checks its first `lane_limit` neighbours (loads
// batched 4-wide for memory-level parallelism).  Phase 2: lanes still
// unresolved are scanned by the whole wave, 64 neighbours per step, ballot
// early exit.  The result word is assembled by a ballot: no atomics.
__global__ __launch_bounds__(kBlock) void bu_kernel(BuArgs a) {
  const int lane = lane_id();
  const int64_t w = static_cast<int64_t>(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6);
  if (w >= a.words) return;
  const word_t vis = a.visited[w];
  if (vis == ~0ull) {
    if (lane == 0) a.cand[w] = 0;
    return;
  }
  const int64_t v = w * 64 + lane;
  const eid_t* __restrict__ ro = a.g.row_off;
  const vid_t* __restrict__ col = a.g.col;
  const word_t* __restrict__ fr = a.frontier;
  eid_t p = 0, e = 0;
  if (v < a.g.rows && !((vis >> lane) & 1ull)) {
    p = ro[v];
    e = ro[v + 1];
  }
  bool found = false;
  const eid_t lim = min(e, p + static_cast<eid_t>(a.lane_limit));
  while (p < lim && !found) {
    vid_t u[4];
    bool ok[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      ok[k] = p + k < lim;
      u[k] = ok[k] ? col[p + k] : 0u;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) found |= ok[k] && test_bit(fr, u[k]);
    p += 4;
  }
  if (p > lim) p = lim;
  unsigned long long pending = __ballot(!found && p < e);
  while (pending) {
    const int l = __ffsll(static_cast<long long>(pending)) - 1;
    pending &= pending - 1;
    const long long ps = __shfl(static_cast<long long>(p), l, kWave);
    const long long pe = __shfl(static_cast<long long>(e), l, kWave);
    bool f = false;
    for (long long base = ps; base < pe; base += kWave) {
      const long long idx = base + lane;
      bool hit = false;
      if (idx < pe) hit = test_bit(fr, col[idx]);
      if (__ballot(hit)) { f = true; break; }
    }
    if (lane == l) found = f;
  }
  const word_t res = __ballot(found);
  if (lane == 0) a.cand[w] = res;
}

// ---------------------------------------------------------------------------
// Status-array top-down (Mode::Simple): thread per owned vertex.
__global__ __launch_bounds__(kBlock) void status_kernel(StatusArgs a) {
  const int64_t v = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (v >= a.g.rows) return;
  if (a.level[v] != a.cur) return;
  for (eid_t e = a.g.row_off[v]; e < a.g.row_off[v + 1]; ++e) {
    const vid_t u = a.g.col[e];
    const word_t bit = 1ull << (u & 63);
    if (!(a.visited[u >> 6] & bit)) atomicOr(a.next + (u >> 6), bit);
  }
}

__global__ __launch_bounds__(kBlock) void bitmap_or_kernel(word_t* __restrict__ dst, const word_t* __restrict__ src,
                                                         int64_t words) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < words; i += stride)
    dst[i] |= src[i];
}

inline unsigned grid_for(int64_t work, int64_t per_block, int64_t cap = 1 << 30) {
  int64_t g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return static_cast<unsigned>(g);
}

}  // namespace

void fill_level(lvl_t* level, int64_t n, lvl_t value, hipStream_t st) {
  if (n <= 0) return;
  const bool aligned16 = (reinterpret_cast<uintptr_t>(level) & 15u) == 0;
  fill_level_kernel<<<grid_for(n / 4 + 1, kBlock, 8192), kBlock, 0, st>>>(level, n, value, aligned16);
}

void set_bit(word_t* bm, int64_t bit, hipStream_t st) { set_bit_kernel<<<1, 64, 0, st>>>(bm, bit); }

void update_frontier(const UpdateArgs& a, hipStream_t st) {
  const int64_t nseg = (a.words + kSegWords - 1) / kSegWords;
  if (nseg == 0) return;
  update_kernel<<<grid_for(nseg, kWavesPerBlock), kBlock, 0, st>>>(a);
}

void scan_segments(const ScanArgs& a, hipStream_t st) {
  scan_segments_kernel<<<1, kScanThreads, 0, st>>>(a);
}

void compact_frontier(const CompactArgs& a, hipStream_t st) {
  const int64_t nseg = (a.words + kSegWords - 1) / kSegWords;
  if (nseg == 0) return;
  compact_kernel<<<grid_for(nseg, kWavesPerBlock), kBlock, 0, st>>>(a);
}

void td_expand(const TdArgs& a, hipStream_t st) {
  if (a.m <= 0 || a.q <= 0) return;
  td_expand_kernel<<<grid_for(a.m, kTdEdgesPerBlock), kTdThreads, 0, st>>>(a);
}

void bu_step(const BuArgs& a, hipStream_t st) {
  if (a.words <= 0) return;
  bu_kernel<<<grid_for(a.words, kWavesPerBlock), kBlock, 0, st>>>(a);
}

void status_expand(const StatusArgs& a, hipStream_t st) {
  if (a.g.rows <= 0) return;
  status_kernel<<<grid_for(a.g.rows, kBlock), kBlock, 0, st>>>(a);
}

void bitmap_or(word_t* dst, const word_t* src, int64_t words, hipStream_t st) {
  if (words <= 0) return;
  bitmap_or_kernel<<<grid_for(words, kBlock, 4096), kBlock, 0, st>>>(dst, src, words);
}

}  // namespace kern
}  // namespace dbfs
