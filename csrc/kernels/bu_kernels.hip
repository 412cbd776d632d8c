// gfx950 bottom-up kernels: the fused parent search (bu_kernel, and the
// persistent hub-LDS variants bu_hub_kernel with deferred row scans and the
// fused level finish) and the hub frontier gather.
//
// Reference counterpart: none -- the reference traverses top-down only
// (queueBfs, bfs.cu:134-165; the status scan, bfs.cu:102-125); the
// direction-optimising search follows Beamer et al.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "kernel_common.hpp"
#include "launch.hpp"
#include "level_device.hpp"
#include "wave.hpp"

namespace dbfs {
namespace kern {
namespace {

// Sum (cnt, deg) of the 4 waves of a unit workgroup; thread 0 writes them.
__device__ __forceinline__ void unit_stats_store(long long cnt, long long deg, int64_t unit, int64_t* unit_cnt,
                                                 int64_t* unit_deg) {
  __shared__ long long s_c[kUnitWaves], s_d[kUnitWaves];
  cnt = wave_sum(cnt);
  deg = wave_sum(deg);
  const int wv = threadIdx.x >> 6;
  if (lane_id() == 0) {
    s_c[wv] = cnt;
    s_d[wv] = deg;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long c = 0, d = 0;
#pragma unroll
    for (int k = 0; k < kUnitWaves; ++k) {
      c += s_c[k];
      d += s_d[k];
    }
    unit_cnt[unit] = c;
    unit_deg[unit] = d;
  }
}

// Rest of a bottom-up row after the head probe: phase 1, each unresolved lane
// checks its next `lane_limit` neighbours (loads batched kBuBatch-wide);
// phase 2, rows still unresolved are scanned by the whole wave, one row at a
// time, 64 neighbours per step with a ballot early exit.  Wave-uniform call
// (phase 2 is cooperative); returns the lane's `found`.
// (Rejected, measured on RMAT-26 in rounds 1-2 and removed: phase 2 as one
// packed multi-row edge stream -- 83 VGPRs, one workgroup per CU, 1238 ->
// 1069 GTEPS; 2-8 phase-2 steps in flight -- 1231 -> 1225-1188; non-temporal
// column loads; records prefetched two batches ahead.  Round 3: the wave's
// unresolved rows as one flattened stream, 128 entries per round found by a
// binary search over the rows' prefixes, per-row cap 4 x 4^round: coalesced
// loads and no serial phase 2, yet late-switch first levels 672 / 889 ->
// 700 / 875 us and the bench flat -- that level is bound by the ~44 M L2
// misses of its column lines and global frontier probes, not by the scan's
// round trips.)
constexpr int kBuBatch = 4;  // phase-1 column loads in flight per lane
constexpr int kCutLevels = 1, kCutClaims = 2;  // hub-cut variants (bu_hub_kernel's kCut)

// Deferred row-scan queue entries per wave (hub waves; 0 = scan in the
// probing step).  LDS: 16 waves x kBuQueue x 8 B next to the hub bits
// (kMaxHubs / 8 B) and the 8 KiB result words, two workgroups per CU.
constexpr int kBuQueue = 64;
static_assert(kBuQueue <= kWave, "one queued row per lane per flush");

#ifdef DBFS_BU_STATS
// Diagnostic build only (-DDBFS_BU_STATS, tools/gpu_bu_stats.sh): wave-level
// event counters of the bottom-up kernel, printed per dispatch by bu_step.
__device__ unsigned long long g_bu_stats[8];
#define BU_STAT(i, x)                                                   \
  do {                                                                  \
    const unsigned long long v_ = (x);                                  \
    if (lane_id() == 0 && v_) atomicAdd(&g_bu_stats[i], v_);            \
  } while (0)
#else
#define BU_STAT(i, x) \
  do {                \
  } while (0)
#endif

// Frontier test of a neighbour id that may be hub-encoded (kHub): hubs in the
// LDS copy of their frontier bits, the rest in the global bitmap.
template <bool kHub>
__device__ __forceinline__ bool bu_probe(const word_t* __restrict__ fr, const word_t* s_hub, vid_t u) {
  if constexpr (kHub) {
    const vid_t hb = u & ~kHubFlag;
    return (u & kHubFlag) ? ((s_hub[hb >> 6] >> (hb & 63)) & 1ull) : test_bit(fr, u);
  } else {
    return test_bit(fr, u);
  }
}

// kNoVertex pads a phase-2 step's tail (never a vertex or a hub-encoded id:
// ids < 2^31, hub codes < kHubFlag + kMaxHubs).
constexpr vid_t kNoVertex = 0xFFFFFFFFu;

// kCut (hub-cut level, `cut` set): the scan stops at the row's first non-hub
// neighbour (BuArgs::cut_edges) -- only hub prefixes are read, probed in LDS;
// rows longer than kSortedRowMax are not hub-first and are scanned whole.
template <bool kHub, bool kCut = false>
__device__ __forceinline__ bool bu_scan_row(const BuArgs& a, eid_t rs, eid_t e, bool found, const word_t* s_hub,
                                            bool cut = false) {
  const int lane = lane_id();
  // hub-encoded copy of the adjacency when present (kHub kernels only)
  const vid_t* __restrict__ col = (kHub && a.g.hub_col) ? a.g.hub_col : a.g.col;
  const word_t* __restrict__ fr = a.frontier;
  // positions relative to the row start: 32-bit (a row never holds 2^32 entries)
  const vid_t* __restrict__ row = col + rs;
  const uint32_t len = static_cast<uint32_t>(e - rs);
  uint32_t p = min(len, 1u);
  // (kCut: a row too long to be hub-first goes straight to the wave scan,
  // which decides per row)
  const uint32_t lim = min(len, cut && len > static_cast<uint32_t>(kSortedRowMax) ? 1u
                                                                                  : static_cast<uint32_t>(a.lane_limit));
  BU_STAT(3, __popcll(__ballot(p < lim && !found)));
  bool past_hubs = false;  // (kCut) the scan reached a non-hub neighbour
  while (p < lim && !found) {
    BU_STAT(4, 1);
    vid_t u[kBuBatch];
    bool ok[kBuBatch];
#pragma unroll
    for (int k = 0; k < kBuBatch; ++k) {
      ok[k] = p + k < lim;
      u[k] = ok[k] ? row[p + k] : 0u;
    }
    if constexpr (kCut) {
      if (cut) {
        bool stop = false;
#pragma unroll
        for (int k = 0; k < kBuBatch; ++k) {
          const bool hub = (u[k] & kHubFlag) != 0;
          found |= ok[k] && hub && ((s_hub[(u[k] & ~kHubFlag) >> 6] >> (u[k] & 63)) & 1ull);
          stop |= ok[k] && !hub;
        }
        past_hubs = stop;
        p = stop ? lim : p + kBuBatch;
        continue;
      }
    }
#pragma unroll
    for (int k = 0; k < kBuBatch; ++k) found |= ok[k] && bu_probe<kHub>(fr, s_hub, u[k]);
    p += kBuBatch;
  }
  if (p > lim) p = lim;
  // Phase 2: the wave scans each still-unresolved row in turn
  unsigned long long pending = __ballot(!found && !past_hubs && p < len);
  BU_STAT(5, __popcll(pending));
  while (pending) {
    const int l = __ffsll(static_cast<long long>(pending)) - 1;
    pending &= pending - 1;
    const vid_t* r = reinterpret_cast<const vid_t*>(__shfl(reinterpret_cast<long long>(row), l, kWave));
    const uint32_t ps = __shfl(p, l, kWave), pe = __shfl(len, l, kWave);
    const bool cut_row = cut && pe <= static_cast<uint32_t>(kSortedRowMax);  // (wave-uniform)
    bool f = false;
    for (uint32_t base = ps; base < pe; base += kWave) {
      BU_STAT(6, 1);
      const uint32_t idx = base + lane;
      const vid_t u = idx < pe ? r[idx] : kNoVertex;
      if constexpr (kCut) {
        if (cut_row) {
          const bool hub = u != kNoVertex && (u & kHubFlag);
          if (__ballot(hub && ((s_hub[(u & ~kHubFlag) >> 6] >> (u & 63)) & 1ull))) {
            f = true;
            break;
          }
          if (__ballot(u != kNoVertex && !hub)) break;  // past the hub prefix
          continue;
        }
      }
      if (__ballot(u != kNoVertex && bu_probe<kHub>(fr, s_hub, u))) {
        f = true;
        break;
      }
    }
    if (lane == l) found = f;
  }
  return found;
}

// ---------------------------------------------------------------------------
// Fused bottom-up step of one wave over kWords bitmap words from w0 (a whole
// 64-word unit, or 16 words when the shard is too small to fill the chip
// that way): the unvisited vertices of its words are numbered (per-word
// popcount prefix) and processed 64 at a time, one per lane, whatever word
// they sit in -- the per-step cost is a chain of dependent memory round trips
// nearly independent of how many lanes are active, so steps =
// ceil(unvisited / 64) instead of the words with any unvisited vertex.  Per
// step: row bounds and head (prefetched one step ahead), head probe, then the
// row scan.  Found bits are OR-ed into a per-wave LDS copy of the result words
// (s_res), written out once with the visited update; levels and unit
// statistics are written directly (no separate update pass).
// kQueue > 0: rows whose head probe failed are not scanned in the step that
// probed them (a handful of lanes per step, the rest idle through the scan's
// dependent loads) but queued in LDS (s_q, kQueue entries of row offset
// relative to the unit's first row / length / position) and scanned kQueue at
// a time; rows of 2^20+ entries (or units spanning 2^32 edges) are scanned in
// place.  kRec: row bounds and heads from the packed 8-byte records of the
// non-empty-row view (ShardView::nz_rec).
// kCut: the hub-cut variant (BuArgs::cut_edges; `cut` = *a.cut_flag, read
// once per kernel): vertices already claimed in a.pre are not scanned but
// join the output (their statistics from their row bounds), heads and rows
// stop at the first non-hub neighbour.
template <bool kHub, int kWords = kWaveWords, int kQueue = 0, bool kRec = false, int kCut = 0>
__device__ __forceinline__ void bu_wave_compact(const BuArgs& a, int64_t w0, word_t* s_res, const word_t* s_hub,
                                                long long& cnt, long long& deg, unsigned long long* s_q = nullptr,
                                                bool cut = false) {
  static_assert(kWords <= kWave, "one word per lane");
  const int lane = lane_id();
  const int64_t left = a.words - w0;
  const int nw = left <= 0 ? 0 : (left < kWords ? static_cast<int>(left) : kWords);
  // claimed by the hub-cut level's top-down part (kCut): unvisited vertices
  // whose level byte already holds this level, or (wide levels) whose claim
  // byte is set -- 64 bytes per lane, 16-B loads
  word_t pw = 0;
  if constexpr (kCut) {
    if (cut && lane < nw) {
      const uint8_t* src = kCut == kCutClaims ? a.cut_claim : a.level8;
      const uint4* lb = reinterpret_cast<const uint4*>(src + (w0 + lane) * 64);
      const uint64_t cur = kCut == kCutClaims ? 0ull
                                       : 0x0101010101010101ull *
                                             static_cast<uint8_t>(a.narrow_base + (a.new_level <= kNarrowMaxLevel
                                                                                       ? a.new_level
                                                                                       : kNarrowMaxLevel + 1));
      uint4 q[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) q[k] = lb[k];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint4& x = q[k >> 1];
        const uint64_t y = (k & 1 ? (static_cast<uint64_t>(x.w) << 32 | x.z) : (static_cast<uint64_t>(x.y) << 32 | x.x)) ^ cur;
        // high bit of each zero byte of y (exact), gathered into 8 bits
        const uint64_t z = ~(((y & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full) | y | 0x7F7F7F7F7F7F7F7Full);
        pw |= (((z >> 7) * 0x0102040810204080ull) >> 56) << (8 * k);
      }
      if constexpr (kCut == kCutClaims) pw = ~pw;  // (claim bytes: the non-zero ones)
      pw &= ~a.visited[w0 + lane];
    }
  }
  // unvisited bits of word `lane` (0 past the words); visited = ~um
  const word_t um = lane < nw ? ~a.visited[w0 + lane] & ~pw : 0ull;
  const int incl = static_cast<int>(wave_incl_scan(__popcll(um)));
  const int total = __builtin_amdgcn_readlane(incl, kWave - 1);
  if (lane < kWords) s_res[lane] = 0ull;
  // the claimed vertices: counted, their row lengths summed (wide levels:
  // their levels written and their claim bytes cleared)
  auto take_pre = [&]() {
    if constexpr (kCut) {
      if (pw) {
        if constexpr (kCut == kCutClaims) {
          uint4* cb = reinterpret_cast<uint4*>(a.cut_claim + (w0 + lane) * 64);
#pragma unroll
          for (int k = 0; k < 4; ++k) cb[k] = make_uint4(0u, 0u, 0u, 0u);
        }
        int c = 0;
        long long d = 0;
        for (word_t m = pw; m; m &= m - 1) {
          const int64_t v = (w0 + lane) * 64 + __builtin_ctzll(m);
          d += static_cast<long long>(a.g.row_off[v + 1] - a.g.row_off[v]);
          if constexpr (kCut == kCutClaims) a.level[v] = a.new_level;
          ++c;
        }
        cnt += c;
        deg += d;
      }
    }
  };
  if (total == 0) {
    if (lane < nw) {
      a.new_frontier[w0 + lane] = pw;
      if (pw) a.visited[w0 + lane] = ~um;  // (= visited | pw)
    }
    take_pre();
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const eid_t* __restrict__ ro = a.g.row_off;
  const vid_t* __restrict__ col = a.g.col;
  const word_t* __restrict__ fr = a.frontier;
  const vid_t* __restrict__ head = a.g.head;
  const eid_t* __restrict__ nz_ro = (head && a.g.nz_pref && a.zdeg) ? a.g.nz_row_off : nullptr;
  // packed records: the unit's base offset, span and end of its non-empty
  // rows are wave-uniform (one unit per wave range)
  // (kRec: the launcher checked that the view and its records exist)
  const NzRec* __restrict__ nz_rec = kRec ? a.g.nz_rec : nullptr;
  eid_t u_base = 0;
  uint32_t u_span = 0;
  int64_t u_nzend = 0;
  if constexpr (kRec) {
    // (readfirstlane: wave-uniform values in scalar registers)
    const int64_t unit = w0 / kUnitWords;
    const int64_t row_words = (a.g.rows + kWordBits - 1) / kWordBits;
    u_base = static_cast<eid_t>(readlane64(static_cast<unsigned long long>(a.g.unit_base[unit]), 0));
    u_span = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(a.g.unit_base[unit + 1] - u_base)));
    u_nzend = static_cast<int64_t>(readlane64(
        static_cast<unsigned long long>(a.g.nz_pref[min((unit + 1) * kUnitWords, row_words)]), 0));
  }
  // Unvisited vertex number 64 b + lane -> its position loc = 64 j + bit in the
  // wave's vertices (-1: no vertex), row bounds and head.
  // (row start, 32-bit length) keep the prefetched state small: the hub
  // kernel runs at 64 VGPRs (two 1024-thread workgroups per CU).
  auto fetch = [&](int b, int& loc, eid_t& rs, uint32_t& len, vid_t& u) {
    loc = -1;
    rs = 0;
    len = 0;
    u = 0;
    const int idx = b * kWave + lane;
    if (b * kWave >= total) return;  // uniform
    int j, bit;
    if constexpr (kWords == kWave) {
      const int p = wave_set_position(um, incl, idx);
      j = p >> 6;
      bit = p & 63;
    } else {
      // word j = number of words ending at or before idx; ex = where j starts
      int ex = 0;
      j = 0;
      for (int i = 0; i < nw; ++i) {
        const int end_i = __builtin_amdgcn_readlane(incl, i);
        if (end_i <= idx) {
          ++j;
          ex = end_i;
        }
      }
      j = min(j, nw - 1);
      const word_t umj = static_cast<word_t>(__shfl(static_cast<long long>(um), j, kWave));
      bit = select_bit(umj, idx - ex);
    }
    if (idx < total) {
      loc = j * 64 + bit;
      if (kRec || nz_ro) {
        // dense non-empty-row view: rank = non-empty rows before the word +
        // those below this bit (the word's prefix and zero-degree mask are
        // L1-resident: every lane of the wave reads one of <= 16 words)
        const int64_t k = a.g.nz_pref[w0 + j] + __popcll(~a.zdeg[w0 + j] & ((1ull << bit) - 1ull));
        if constexpr (kRec) {
          const NzRec r = nz_rec[k];
          const uint32_t end = k + 1 < u_nzend ? nz_rec[k + 1].off : u_span;
          rs = u_base + r.off;
          len = end - r.off;
          u = r.head;
        } else {
          rs = nz_ro[k];
          len = static_cast<uint32_t>(nz_ro[k + 1] - rs);
          u = a.g.nz_head[k];
        }
      } else {
        const int64_t v = w0 * 64 + loc;
        rs = ro[v];
        len = static_cast<uint32_t>(ro[v + 1] - rs);
        if (head) u = head[v];
      }
    }
  };
  const int nb = (total + kWave - 1) / kWave;
  int n_loc;
  eid_t n_rs;
  uint32_t n_len;
  vid_t n_u;
  fetch(0, n_loc, n_rs, n_len, n_u);
  if (!head) n_u = n_len ? col[n_rs] : 0u;
  int cnt32 = 0;
  // deferred row scans (kQueue): base = the unit's first row offset
  eid_t q_base = 0;
  bool q_span_ok = false;
  int qn = 0;
  if constexpr (kQueue > 0) {
    // (the non-empty-row view covers ceil(rows / 64) words; a shard's bitmap
    // slice may be longer -- padding words, all visited)
    const int64_t wend = min(w0 + nw, (a.g.rows + kWordBits - 1) / kWordBits);
    if constexpr (kRec) {
      q_base = u_base;  // (every row of the unit starts at or after it; span < 2^32)
      q_span_ok = true;
    } else if (nz_ro) {
      q_base = nz_ro[a.g.nz_pref[w0]];
      q_span_ok = nz_ro[a.g.nz_pref[wend]] - q_base < (eid_t(1) << 32);
    } else {
      const int64_t vend = min(wend * 64, a.g.rows);
      q_base = ro[w0 * 64];
      q_span_ok = ro[vend] - q_base < (eid_t(1) << 32);
    }
  }
  auto settle = [&](bool f, int l, eid_t r0, eid_t r1) {
    if (f) {
      store_level(a.level, a.level8, w0 * 64 + l, a.new_level, a.narrow_base);
      cnt32 += 1;
      deg += r1 - r0;
      __hip_atomic_fetch_or(s_res + (l >> 6), 1ull << (l & 63), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
  };
  // scan the queued rows, one per lane (wave-uniform)
  auto flush = [&]() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    int ql = 0;
    eid_t qrs = 0, qe = 0;
    if (lane < qn) {
      const unsigned long long ent = s_q[lane];
      ql = static_cast<int>(ent & 0xFFFu);
      qrs = q_base + static_cast<eid_t>(ent >> 32);
      qe = qrs + static_cast<eid_t>((ent >> 12) & 0xFFFFFu);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const bool f = bu_scan_row<kHub, (kCut != 0)>(a, qrs, qe, lane >= qn, s_hub, cut);
    settle(lane < qn && f, ql, qrs, qe);
    qn = 0;
  };
  for (int b = 0; b < nb; ++b) {
    const int loc = n_loc;
    const eid_t rs = n_rs, e = n_rs + n_len;
    const vid_t u0 = n_u;
    fetch(b + 1, n_loc, n_rs, n_len, n_u);  // in flight during this batch's probes
    bool found = false;
    bool cut_row = false;  // (kCut) a hub-first row with a non-hub head: nothing to scan
    if constexpr (kCut) {
      cut_row = cut && !(u0 & kHubFlag) && e - rs <= static_cast<eid_t>(kSortedRowMax);
      if (rs < e && !cut_row) found = bu_probe<kHub>(fr, s_hub, u0);
    } else {
      if (rs < e) found = bu_probe<kHub>(fr, s_hub, u0);
    }
    BU_STAT(0, 1);
    BU_STAT(1, __popcll(__ballot(loc >= 0)));
    BU_STAT(2, __popcll(__ballot(found)));
    if (!head) n_u = n_len ? col[n_rs] : 0u;
    if constexpr (kQueue > 0) {
      // found by the head: settled now; unresolved rows with more neighbours
      // are queued (huge rows / spans scanned in place)
      const bool need = !found && e - rs > 1 && !cut_row;
      const bool fits = q_span_ok && e - rs < (eid_t(1) << 20);
      // more unresolved rows than the queue holds (a sparse-hit level: most
      // lanes scan anyway, deferring gains nothing): all in place
      const bool direct = __popcll(__ballot(need && fits)) > kQueue;
      const bool inplace = need && (direct || !fits);
      if (__ballot(inplace)) {
        // (lanes not scanned here pass as resolved and keep their result)
        const bool f = bu_scan_row<kHub, (kCut != 0)>(a, rs, e, found || !inplace, s_hub, cut);
        if (inplace) found = f;
      }
      settle(found, loc, rs, e);
      const bool defer = need && !inplace;
      const unsigned long long dm = __ballot(defer);
      const int k = __popcll(dm);
      if (qn + k > kQueue) flush();
      if (defer)
        s_q[qn + mask_rank(dm)] = (static_cast<unsigned long long>(rs - q_base) << 32) |
                                  (static_cast<unsigned long long>(e - rs) << 12) | static_cast<unsigned>(loc);
      qn += k;
    } else {
      found = bu_scan_row<kHub, (kCut != 0)>(a, rs, e, found || cut_row, s_hub, cut) && !cut_row;
      BU_STAT(7, __popcll(__ballot(found)));
      settle(found, loc, rs, e);
    }
  }
  if constexpr (kQueue > 0) {
    if (qn) flush();
  }
  cnt += cnt32;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (lane < nw) {
    const word_t res = s_res[lane] | pw;
    a.new_frontier[w0 + lane] = res;
    if (res) a.visited[w0 + lane] = ~um | res;  // (~um holds pw)
  }
  take_pre();
}

// Graphs without hubs: a wave per 16 words, 4 waves (one unit) per workgroup.
__global__ __launch_bounds__(kUnitThreads) void bu_kernel(BuArgs a) {
  __shared__ word_t s_res[kUnitWaves * kWaveWords];
  if (a.ctrl && (a.ctrl->done || a.ctrl->dir != 'B')) return;
  stamp_level_start(a.ctrl);
  long long cnt = 0, deg = 0;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));  // (wave-uniform)
  const int64_t w0 = static_cast<int64_t>(blockIdx.x) * kUnitWords + wave * kWaveWords;
  bu_wave_compact<false>(a, w0, s_res + wave * kWaveWords, nullptr, cnt, deg);
  unit_stats_store(cnt, deg, blockIdx.x, a.unit_cnt, a.unit_deg);
}

// Hub variant: persistent workgroups (two per CU) that first stage the hub
// frontier bits (<= kMaxHubs bits, 64 KiB) in LDS; a hub-encoded head or
// neighbour is then probed in LDS instead of by a scattered load of the
// 8 MiB (RMAT-26) frontier bitmap -- at the dominant bottom-up level ~80% of
// the unvisited vertices resolve at their head, ~85% of heads are hubs.
// kWhole: one whole 64-word unit per wave (its statistics need no cross-wave
// reduction, so waves run independently) -- chosen when the shard has enough
// units to fill the chip that way (one GPU); small shards (many ranks) keep
// 16 words per wave, four waves per unit, for parallelism.
constexpr int kHubBuThreads = 1024;
static_assert(kHubBuThreads % kUnitThreads == 0, "hub workgroups hold whole unit groups");
constexpr int kHubWords = static_cast<int>(kMaxHubs / kWordBits);

// The fused finish of a bottom-up level (BuArgs::fuse_scan; every thread of
// the workgroup calls it): thread 0's workgroup totals (wc, wd) go to the
// workgroup's slot of tot (agent-scope stores: no same-address atomics but
// the ticket's), a ticket; the last workgroup sums the slots and finishes the
// level (scan_finish) -- and runs the level's end when it is folded in
// (a.end, several ranks).  s_c / s_d: kThreads / 64 LDS slots, reused; s_x:
// LDS for the level end (the kernel's result words, written out by then).
template <int kThreads, bool kEnd>
__device__ __forceinline__ void bu_fused_finish(const BuArgs& a, long long wc, long long wd, long long* s_c,
                                                long long* s_d, uint64_t* s_x) {
  constexpr int kWaves = kThreads / kWave;
  __shared__ int s_last;
  const int wave = static_cast<int>(threadIdx.x >> 6);
  if (threadIdx.x == 0) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.tot + 2 * blockIdx.x), static_cast<unsigned long long>(wc),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.tot + 2 * blockIdx.x + 1),
                       static_cast<unsigned long long>(wd), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // (measured: a two-level ticket here, as the update's, is no faster --
    // the workgroups of a bottom-up level do not arrive together)
    s_last = atomicAdd(a.scan.ticket, 1u) == gridDim.x - 1;
    if (s_last) last_arriver_acquire();
  }
  __syncthreads();
  if (!s_last) return;
  long long c = 0, d = 0;
  for (unsigned i = threadIdx.x; i < gridDim.x; i += kThreads) {
    c += static_cast<long long>(__hip_atomic_load(reinterpret_cast<unsigned long long*>(a.tot + 2 * i),
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    d += static_cast<long long>(__hip_atomic_load(reinterpret_cast<unsigned long long*>(a.tot + 2 * i + 1),
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
  c = wave_sum(c);
  d = wave_sum(d);
  __syncthreads();  // (s_c / s_d reused)
  if (lane_id() == 0) {
    s_c[wave] = c;
    s_d[wave] = d;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long tc = 0, td = 0;
    for (int k = 0; k < kWaves; ++k) {
      tc += s_c[k];
      td += s_d[k];
    }
    scan_finish(a.scan, tc, td);  // (resets the ticket)
    s_c[0] = tc;
    s_d[0] = td;
  }
  if constexpr (kEnd) {
    __syncthreads();
    direct_level_end(a.end, s_c[0], s_d[0], a.scan.stats, a.fin, s_x);
  }
}

// Pushed frontier words (BuArgs::push) of the words a wave wrote (w0 + lane,
// lane < nw): a pass of their own after the units, re-reading each lane's own
// stores, compiled only into the kPost variants -- inline in bu_wave_compact
// (or in every variant) they cost the hot loop registers (2 VGPRs spilled).
// Wave-uniform call.
__device__ __forceinline__ void bu_post_words(const BuArgs& a, int64_t w0, int nw) {
  const int lane = lane_id();
  if (lane >= nw || w0 + lane >= a.words) return;
  push_frontier_word(a.push, a.push_rank, a.push_nranks, w0 + lane, a.new_frontier[w0 + lane]);
}

// kEnd: the level's end folded in (BuArgs::end; several ranks only -- its
// code costs the one-rank kernels their spill-free 64 registers).
// kCut: the hub-cut variant (first bottom-up level of a run of them),
// kCutLevels (claims in the narrow level bytes) or kCutClaims (wide levels:
// claims in BuArgs::cut_claim).
// kPost: the output words pushed to the peers afterwards (BuArgs::push).
// kWW: words per wave when units are split over waves (!kWhole): 16, or 4 for
// shards too small to fill the chip at 16 (a soc-LiveJournal1-sized graph's
// 1184 units at 16 words per wave are 4736 waves, 18 per CU against 32 slots).
// XCD-aware unit walk: workgroup b takes the slot (b % 8) * (G / 8) + b / 8 of
// the grid-stride walk, so each XCD (workgroups dispatch round-robin over the
// 8) scans one contiguous eighth of every round's units -- its row records,
// level bytes and edge runs in its own L2 and translation caches -- instead
// of every eighth group of them.  Only when every round is full (units a
// multiple of G x per, as on the power-of-two RMAT shards): a partial last
// round remapped would sit on the first few XCDs only (a small shard's one
// partial round measured -10 % on the soc-LiveJournal1-sized graph).  Decided
// once, before the walk: a per-round choice cost the fused-finish variants
// 2-4 VGPRs and the cut variant a 12-B spill.
// Same-box A/B on RMAT-26 (profiles/r6_xcd_remap_ab.txt): flat to +0.5 %
// (the scan's traffic is streaming rows plus random frontier probes, which
// no mapping localises); DBFS_NO_XCD_REMAP restores the plain order.
__device__ __forceinline__ int64_t bu_block(int64_t nunits, int per) {
  const uint32_t g = gridDim.x, b = blockIdx.x;
#ifndef DBFS_NO_XCD_REMAP
  if (g % 8 == 0 && nunits % (static_cast<int64_t>(g) * per) == 0)
    return static_cast<int64_t>(b % 8) * (g / 8) + b / 8;
#endif
  return b;
}

template <bool kWhole, int kThreads = kHubBuThreads, int kQ = kBuQueue, bool kRec = false, bool kEnd = false,
          int kCut = 0, bool kPost = false, int kWW = kWaveWords>
__global__ __launch_bounds__(kThreads, 2 * kThreads / 256) void bu_hub_kernel(BuArgs a) {
  __shared__ word_t s_hub[kHubWords];
  __shared__ word_t s_res[(kThreads / kWave) * kUnitWords];
  __shared__ long long s_c[kThreads / kWave], s_d[kThreads / kWave];
  __shared__ unsigned long long s_q[kQ > 0 ? (kThreads / kWave) * kQ : 1];
  if (a.ctrl && (a.ctrl->done || a.ctrl->dir != 'B')) {
    // a folded level end is a collective: it runs on a no-op chain too
    if constexpr (kEnd) {
      if (blockIdx.x == 0)
        direct_level_end(a.end, a.scan.stats[2], a.scan.stats[3], a.scan.stats, a.fin,
                         reinterpret_cast<uint64_t*>(s_res));
    }
    return;
  }
  // a hub-cut level launches the cut variant alone: the device decision
  // (hub_gather's) picks the scan at run time -- the plain one when it says
  // no (rare: the level is enqueued only when predicted small), instead of a
  // second, plain launch that returned at once on every cut level (~4.5 us
  // of idle GPU per late-switch traversal)
  const bool cut = kCut != 0 && *a.cut_flag != 0;
  if (!a.hub_front) stamp_level_start(a.ctrl);
  const int64_t hw = (a.g.nhubs + kWordBits - 1) / kWordBits;
  stage_words<kThreads, kHubWords>(s_hub, a.hub_front, hw);
  __syncthreads();
  // (readfirstlane: the wave index, and the unit and word offsets derived
  // from it, are wave-uniform -- scalar registers, not vector ones)
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int64_t nunits = (a.words + kUnitWords - 1) / kUnitWords;
  if constexpr (kWhole) {
    constexpr int kWavesPerBlock = kThreads / kWave;
    // (fused finish: this wave's totals accumulate in its LDS slots)
    if (lane_id() == 0) {
      s_c[wave] = 0;
      s_d[wave] = 0;
    }
    // Static stride over the units.  (A dynamic unit queue measured slower:
    // RMAT-26 per level 387 / 182 / 104 against 346 / 137 / 30 us -- the
    // returning device-scope atomics cost more than the stride's imbalance.)
    const int64_t blk = bu_block(nunits, kWavesPerBlock);
    for (int64_t u = blk * kWavesPerBlock + wave; u < nunits; u += static_cast<int64_t>(gridDim.x) * kWavesPerBlock) {
      long long cnt = 0, deg = 0;
      bu_wave_compact<true, kUnitWords, kQ, kRec, kCut>(a, u * kUnitWords, s_res + wave * kUnitWords, s_hub, cnt,
                                                        deg, s_q + wave * kQ, cut);
      cnt = wave_sum(cnt);
      deg = wave_sum(deg);
      if (lane_id() == 0) {
        a.unit_cnt[u] = cnt;
        a.unit_deg[u] = deg;
        s_c[wave] += cnt;
        s_d[wave] += deg;
      }
    }
    if constexpr (kPost)
      for (int64_t u = blk * kWavesPerBlock + wave; u < nunits;
           u += static_cast<int64_t>(gridDim.x) * kWavesPerBlock)
        bu_post_words(a, u * kUnitWords, kUnitWords);
    if (!a.fuse_scan) return;
    // (pushed words: every wave's write-through stores drained before the
    // ticket, so a level end published after it covers them)
    if constexpr (kPost) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    long long wc = 0, wd = 0;
    if (threadIdx.x == 0)
      for (int k = 0; k < kWavesPerBlock; ++k) {
        wc += s_c[k];
        wd += s_d[k];
      }
    bu_fused_finish<kThreads, kEnd>(a, wc, wd, s_c, s_d, reinterpret_cast<uint64_t*>(s_res));
    return;
  }
  // kWW words per wave: unit groups of kUW waves walk the units; every
  // workgroup runs the same number of iterations (barriers stay uniform)
  constexpr int kUW = kUnitWords / kWW;  // waves per unit
  static_assert(kUnitWords % kWW == 0 && (kThreads / kWave) % kUW == 0, "whole unit groups per workgroup");
  constexpr int kGroups = (kThreads / kWave) / kUW;
  const int group = wave / kUW;
  const int wg = wave % kUW;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kGroups;
  // the unit groups' totals for the fused finish, in LDS (registers live
  // across the loop would spill)
  __shared__ long long s_acc[2 * kGroups];
  if (threadIdx.x < 2 * kGroups) s_acc[threadIdx.x] = 0;
  const int64_t blk = bu_block(nunits, kGroups);
  for (int64_t base = blk * kGroups; base < nunits; base += stride) {
    const int64_t u = base + group;
    long long cnt = 0, deg = 0;
    if (u < nunits)
      bu_wave_compact<true, kWW, kQ, kRec, kCut>(a, u * kUnitWords + wg * kWW, s_res + wave * kWW, s_hub, cnt, deg,
                                                 s_q + wave * kQ, cut);
    cnt = wave_sum(cnt);
    deg = wave_sum(deg);
    if (lane_id() == 0) {
      s_c[wave] = cnt;
      s_d[wave] = deg;
    }
    __syncthreads();
    if ((threadIdx.x & (kUW * kWave - 1)) == 0 && u < nunits) {
      long long c = 0, d = 0;
#pragma unroll
      for (int k = 0; k < kUW; ++k) {
        c += s_c[group * kUW + k];
        d += s_d[group * kUW + k];
      }
      a.unit_cnt[u] = c;
      a.unit_deg[u] = d;
      s_acc[2 * group] += c;
      s_acc[2 * group + 1] += d;
    }
    __syncthreads();
  }
  if constexpr (kPost)
    for (int64_t base = blk * kGroups; base < nunits; base += stride)
      if (base + group < nunits) bu_post_words(a, (base + group) * kUnitWords + wg * kWW, kWW);
  if (!a.fuse_scan) return;
  if constexpr (kPost) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (as above)
  __syncthreads();  // (an empty loop: the accumulators' zeroing)
  long long wc = 0, wd = 0;
  if (threadIdx.x == 0)
    for (int g = 0; g < kGroups; ++g) {
      wc += s_acc[2 * g];
      wd += s_acc[2 * g + 1];
    }
  bu_fused_finish<kThreads, kEnd>(a, wc, wd, s_c, s_d, reinterpret_cast<uint64_t*>(s_res));
}

// hub_front bit h = frontier bit of hub_vertex[h]: 4 hubs per thread, their
// loads issued together (the frontier bits are random 8-B reads of a bitmap
// far larger than the L2: one round trip per thread instead of four).
// Several ranks with bu_merge_visited: the whole grid then merges the gathered
// frontier into visited.
// kCut, a hub-cut level (BuArgs::cut_edges): the frontier hubs' degrees
// (their rows, or with several ranks g.hub_deg) summed per workgroup; the
// last-arriving workgroup (of ~128) totals them and stores the decision
// ctrl->m_f - hub edges <= cut_edges in *cut_flag -- the same on every rank
// (global frontier, global degrees).
// Pushed slices (HubGatherArgs::pull): the hubs' bits read from their owners'
// slices in this rank's window, and the whole grid copies the peers' slices
// into the global frontier (merging them into visited with the merge).
constexpr int kHgThreads = 1024, kHgPer = 4;
__device__ __forceinline__ bool pulled_bit(const HubGatherArgs& a, vid_t v) {
  const int64_t w = static_cast<int64_t>(v >> 6);
  const int p = static_cast<int>(w / a.pull_words);
  const word_t f = p == a.pull_rank ? a.frontier[w] : sys_load_u64(a.pull->src[p] + (w - p * a.pull_words));
  return (f >> (v & 63)) & 1ull;
}
// (kThreads x kPer hubs per workgroup: the plain gather one hub per thread
// over a grid that fills the chip, the cut decision 4 per thread over ~16
// workgroups -- fewer ticket arrivals)
template <bool kCut, int kThreads, int kPer>
__global__ __launch_bounds__(kThreads) void hub_gather_kernel(HubGatherArgs a) {
  if (a.ctrl && (a.ctrl->done || a.ctrl->dir != 'B')) return;
  stamp_level_start(a.ctrl);
  __shared__ long long s_d[kThreads / kWave];
  __shared__ int s_last;
  const int lane = lane_id();
  const int64_t base = static_cast<int64_t>(blockIdx.x) * (kThreads * kPer);
  vid_t hv[kPer];
  bool bit[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t h = base + k * kThreads + threadIdx.x;
    hv[k] = h < a.g.nhubs ? a.g.hub_vertex[h] : 0u;
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t h = base + k * kThreads + threadIdx.x;
    bit[k] = h < a.g.nhubs && (a.pull ? pulled_bit(a, hv[k]) : test_bit(a.frontier, hv[k]));
  }
  long long d = 0;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t h = base + k * kThreads + threadIdx.x;
    const int64_t h0 = base + k * kThreads + (threadIdx.x & ~(kWave - 1));
    const word_t m = __ballot(bit[k]);
    if (lane == 0 && h0 < a.g.nhubs) a.hub_front[h0 / kWave] = m;
    if (kCut && bit[k])
      d += a.g.hub_deg ? static_cast<long long>(a.g.hub_deg[h])
                       : static_cast<long long>(a.g.row_off[hv[k] + 1] - a.g.row_off[hv[k]]);
  }
  if (a.pull) {
    const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
    const int64_t gw = a.pull_words * a.pull_nranks;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < gw; i += stride) {
      const int p = static_cast<int>(i / a.pull_words);
      if (p == a.pull_rank) continue;
      const word_t f = sys_load_u64(a.pull->src[p] + (i - p * a.pull_words));
      a.pull_out[i] = f;
      if (a.visited && f) a.visited[i] |= f;
    }
  } else if (a.visited) {
    const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < a.words; i += stride) {
      const word_t f = a.frontier[i];
      if (f) a.visited[i] |= f;
    }
  }
  if constexpr (!kCut) return;
  d = wave_sum(d);
  if (lane == 0) s_d[threadIdx.x >> 6] = d;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long t = 0;
#pragma unroll
    for (int k = 0; k < kThreads / kWave; ++k) t += s_d[k];
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.cut_part + blockIdx.x), static_cast<unsigned long long>(t),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_last = atomicAdd(a.cut_ticket, 1u) == gridDim.x - 1;
    if (s_last) last_arriver_acquire();
  }
  __syncthreads();
  if (!s_last) return;
  long long t = 0;
  for (unsigned i = threadIdx.x; i < gridDim.x; i += kThreads)
    t += static_cast<long long>(__hip_atomic_load(reinterpret_cast<unsigned long long*>(a.cut_part + i),
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  t = wave_sum(t);
  __syncthreads();  // (s_d reused)
  if (lane == 0) s_d[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long hub_edges = 0;
#pragma unroll
    for (int k = 0; k < kThreads / kWave; ++k) hub_edges += s_d[k];
    *a.cut_flag = a.ctrl->m_f - hub_edges <= a.cut_edges ? 1 : 0;
    *a.cut_ticket = 0u;
  }
}

// The hub-cut level's top-down part (BuArgs::cut_edges; hub_gather decided):
// a wave per 64 frontier words finds their non-hub vertices and expands
// their rows one after another, the lanes striding over the row (four column
// loads, then four visited words, in flight per lane), writing the level
// byte of every unvisited neighbour -- plain byte stores, repeats harmless;
// the bottom-up kernel reads the claims back from the bytes.
// Measured on RMAT-26 (3 K non-hub frontier vertices, 0.66 M edges): 35-40 us
// (kernel trace; grid 256-4096 workgroups flat); a list of the vertices, a
// wave each, spent 109 us in the list's same-address appends alone; claims
// in a bitmap by device atomics 160 us.
// Several ranks (kX): a rank expands its own non-hub frontier vertices (its
// slice of the global frontier, BuArgs::cut_word_off), filters the targets by
// the replicated visited bitmap, claims the owned ones as above and marks the
// remote ones in the global byte map (BuArgs::cut_bytes), which pack_bytes
// turns into one bitmap slice per owner for the all-to-all; bu_cut_merge
// claims what arrives.  (Round 4 sent them as owner lists -- one returning
// atomic per claim -- and measured slower at P = 8.)
constexpr int kCutThreads = 1024;
template <bool kX>
__global__ __launch_bounds__(kCutThreads) void bu_cut_prep_kernel(BuArgs a) {
  if ((a.ctrl && (a.ctrl->done || a.ctrl->dir != 'B')) || !*a.cut_flag) return;
  const vid_t* __restrict__ col = a.g.col;
  const eid_t* __restrict__ ro = a.g.row_off;
  const word_t* __restrict__ fr = a.frontier + (kX ? a.cut_word_off : 0);
  const word_t* __restrict__ hub = a.g.hub_bits + (kX ? a.cut_word_off : 0);
  const word_t* __restrict__ vis = kX ? a.cut_vis : a.visited;
  const uint64_t lo = kX ? static_cast<uint64_t>(a.g.lo) : 0ull, rows = static_cast<uint64_t>(a.g.rows);
  const int lane = lane_id();
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kCutThreads;
  for (int64_t w0 = static_cast<int64_t>(blockIdx.x) * kCutThreads + (threadIdx.x & ~(kWave - 1)); w0 < a.words;
       w0 += stride) {
    const int64_t w = w0 + lane;
    word_t m = w < a.words ? fr[w] & ~hub[w] : 0ull;
    for (unsigned long long bm = __ballot(m != 0); bm; bm = __ballot(m != 0)) {
      const int l = __ffsll(static_cast<long long>(bm)) - 1;
      const int64_t v = (w0 + l) * 64 + __builtin_ctzll(static_cast<word_t>(__shfl(static_cast<long long>(m), l, kWave)));
      if (lane == l) m &= m - 1;
      const eid_t rs = ro[v], re = ro[v + 1];
      constexpr int kU = 4;
      for (eid_t b0 = rs + lane; b0 < re; b0 += kU * kWave) {
        vid_t t[kU];
        word_t vw[kU];
#pragma unroll
        for (int k = 0; k < kU; ++k) {
          const eid_t e = b0 + k * kWave;
          t[k] = e < re ? col[e] : kNoVertex;
        }
#pragma unroll
        for (int k = 0; k < kU; ++k) vw[k] = t[k] == kNoVertex ? ~0ull : vis[t[k] >> 6];
#pragma unroll
        for (int k = 0; k < kU; ++k) {
          if ((vw[k] >> (t[k] & 63)) & 1ull) continue;
          const uint64_t r = static_cast<uint64_t>(t[k]) - lo;
          if (kX && r >= rows) {
            a.cut_bytes[t[k]] = 1;  // (a remote claim: packed for its owner)
            continue;
          }
          if (a.cut_claim) a.cut_claim[r] = 1;  // (wide levels: the bottom-up kernel writes them)
          else store_level(nullptr, a.level8, static_cast<int64_t>(r), a.new_level, a.narrow_base);
        }
      }
    }
  }
}

// Several ranks, a live hub-cut level: owned word w's claims from the peers
// (OR of their slices in cut_recv, filtered by visited) into the claim bytes
// (narrow level bytes or cut_claim), and every slice of the packed bitmap
// zeroed (cut_next: the dense top-down levels' candidate bitmap, kept zero
// between users).
__global__ __launch_bounds__(kBlock) void bu_cut_merge_kernel(BuArgs a) {
  if ((a.ctrl && (a.ctrl->done || a.ctrl->dir != 'B')) || !*a.cut_flag) return;
  const int64_t w = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (w >= a.words) return;
  word_t c = 0;
  for (int p = 0; p < a.cut_nranks; ++p) {
    if (p == a.cut_rank) continue;
    c |= a.cut_recv[p * a.words + w];
    a.cut_next[p * a.words + w] = 0ull;
  }
  c &= ~a.visited[w];
  for (; c; c &= c - 1) {
    const int64_t r = w * 64 + __builtin_ctzll(c);
    if (a.cut_claim) a.cut_claim[r] = 1;
    else store_level(nullptr, a.level8, r, a.new_level, a.narrow_base);
  }
}

}  // namespace

#ifdef DBFS_BU_STATS
static void bu_stats_report(hipStream_t st) {
  unsigned long long h[8] = {0};
  (void)hipStreamSynchronize(st);
  (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_bu_stats), sizeof(h));
  const unsigned long long z[8] = {0};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bu_stats), z, sizeof(z));
  if (h[0])
    std::fprintf(stderr,
                 "[bu-stats] batches %llu active-lanes %llu head-found %llu p1-lanes %llu p1-iters %llu "
                 "p2-rows %llu p2-steps %llu found %llu\n",
                 h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
}
#endif

void bu_step(const BuArgs& a, hipStream_t st) {
#ifdef DBFS_BU_STATS
  struct Report {
    hipStream_t st;
    ~Report() { bu_stats_report(st); }
  } report{st};
#endif
  if (a.words <= 0) return;
  DBFS_CHECK((a.g.nhubs > 0 && a.hub_front) || !a.push, "bu_step: pushed words need the hub kernels");
  if (a.g.nhubs > 0 && a.hub_front) {
    const int64_t nunits = (a.words + kUnitWords - 1) / kUnitWords;
    // a whole 64-word unit per wave when the shard has enough units to fill
    // every resident wave slot (one GPU); small shards (many ranks) keep 16
    // words per wave for parallelism
    const int64_t slots = 2 * static_cast<int64_t>(device_cus()) * (kHubBuThreads / kWave);
    const bool whole = a.whole_units > 0 || (a.whole_units == 0 && nunits >= slots);
    // whole units in 1024-thread workgroups for every bottom-up level: a
    // level after another one (few unvisited vertices left, most of them
    // scanning rows) ran in 768-thread ones while that variant needed 80
    // VGPRs; at 60-65 now, 1024 threads measured the late-switch second
    // level 188-191 -> 160 us, RMAT-26 +2.4 % (held-out +1.7 %) on two boxes
    // (profiles/r6_follow_1024_ab.txt)
    const int threads = kHubBuThreads;
    // shards too small to fill the wave slots at 16 words per wave: 4 (one
    // unit per workgroup) for a first bottom-up level -- measured, the
    // soc-LiveJournal1-sized graph's first level 420 -> 295 us (do mode
    // 116 -> 146 GTEPS), RMAT-22's 45 -> 36 us; later levels, with few
    // unvisited vertices left, ran slower that way (21 -> 26 us) and keep 16
    const bool small = !whole && !a.follow_up &&
                       (a.small_waves > 0 || (a.small_waves == 0 && nunits * (kUnitWords / kWaveWords) < slots));
    const unsigned grid = grid_for(nunits, whole ? threads / kWave : (small ? 1 : kHubBuThreads / kUnitThreads),
                                   2 * device_cus());
    // packed row records (compile-time path: the view's fallback costs registers)
    const bool rec = a.g.nz_rec && a.g.unit_base && a.g.nz_pref && a.g.nz_row_off && a.zdeg && a.g.head;
    if (a.fuse_scan && grid > static_cast<unsigned>(kMaxFusedGrid)) {
      DBFS_CHECK(!a.end.active, "bu_step: a folded level end needs the fused finish");
      // (more workgroups than totals slots: finish in a kernel of its own)
      BuArgs b = a;
      b.fuse_scan = false;
      bu_step(b, st);
      totals_finish(a.scan, st);
      return;
    }
    // (every hub kernel runs the fused finish itself; a folded level end is
    // compiled only into the kEnd variants)
#define DBFS_BU_LAUNCH_WW(W, T, Q, R, WW)                                                                \
  do {                                                                                                   \
    if (a.end.active && a.push) bu_hub_kernel<W, T, Q, R, true, 0, true, WW><<<grid, T, 0, st>>>(a);     \
    else if (a.end.active) bu_hub_kernel<W, T, Q, R, true, 0, false, WW><<<grid, T, 0, st>>>(a);         \
    else if (a.push) bu_hub_kernel<W, T, Q, R, false, 0, true, WW><<<grid, T, 0, st>>>(a);               \
    else bu_hub_kernel<W, T, Q, R, false, 0, false, WW><<<grid, T, 0, st>>>(a);                          \
  } while (0)
#define DBFS_BU_LAUNCH(W, T, Q, R)                  \
  do {                                              \
    if (small) DBFS_BU_LAUNCH_WW(W, T, Q, R, 4);     \
    else DBFS_BU_LAUNCH_WW(W, T, Q, R, kWaveWords);  \
  } while (0)
    if (a.cut_edges > 0) {
      // a hub-cut level (a first bottom-up level: the engine only asks for
      // it there): the cut variant alone, which scans plain when the device
      // decision says no
      DBFS_CHECK(rec && !a.follow_up && a.cut_flag && (a.level8 || (a.cut_claim && a.level)) && a.g.hub_bits,
                 "bu_step: hub-cut level without packed records / flag / claim bytes");
      // (with the deferred row queue: without it, scans in place, the late-switch
      // levels measured 460-535 -> 505-560 us)
      constexpr int kCutQ = kBuQueue;
#define DBFS_CUT_LAUNCH(W, C)                                                                                   \
  do {                                                                                                        \
    if (a.end.active && a.push) bu_hub_kernel<W, kHubBuThreads, kCutQ, true, true, C, true><<<grid, kHubBuThreads, 0, st>>>(a); \
    else if (a.end.active) bu_hub_kernel<W, kHubBuThreads, kCutQ, true, true, C><<<grid, kHubBuThreads, 0, st>>>(a); \
    else if (a.push) bu_hub_kernel<W, kHubBuThreads, kCutQ, true, false, C, true><<<grid, kHubBuThreads, 0, st>>>(a); \
    else bu_hub_kernel<W, kHubBuThreads, kCutQ, true, false, C><<<grid, kHubBuThreads, 0, st>>>(a);          \
  } while (0)
      // (a small shard's first level -- 4 words per wave, one unit per
      // workgroup, as the plain launch below: the cut variant scans plain when
      // the decision says no, and the soc-LiveJournal1-sized graph's first
      // level then ran at 16 words per wave, do mode 154 -> 120 GTEPS)
      const bool small4 = small && !a.end.active && !a.push;
#define DBFS_CUT_LAUNCH4(C) bu_hub_kernel<false, kHubBuThreads, kCutQ, true, false, C, 0, 4><<<grid, kHubBuThreads, 0, st>>>(a)
      if (a.cut_claim) {
        if (whole) DBFS_CUT_LAUNCH(true, kCutClaims);
        else if (small4) DBFS_CUT_LAUNCH4(kCutClaims);
        else DBFS_CUT_LAUNCH(false, kCutClaims);
      } else {
        if (whole) DBFS_CUT_LAUNCH(true, kCutLevels);
        else if (small4) DBFS_CUT_LAUNCH4(kCutLevels);
        else DBFS_CUT_LAUNCH(false, kCutLevels);
      }
#undef DBFS_CUT_LAUNCH4
#undef DBFS_CUT_LAUNCH
      return;
    }
    if (whole) {
      if (rec) DBFS_BU_LAUNCH_WW(true, kHubBuThreads, kBuQueue, true, kWaveWords);
      else DBFS_BU_LAUNCH_WW(true, kHubBuThreads, kBuQueue, false, kWaveWords);
      return;
    }
    if (a.follow_up && rec) DBFS_BU_LAUNCH(false, kHubBuThreads, 0, true);
    else if (a.follow_up) DBFS_BU_LAUNCH(false, kHubBuThreads, 0, false);
    else if (rec) DBFS_BU_LAUNCH(false, kHubBuThreads, kBuQueue, true);
    else DBFS_BU_LAUNCH(false, kHubBuThreads, kBuQueue, false);
#undef DBFS_BU_LAUNCH
#undef DBFS_BU_LAUNCH_WW
    return;
  }
  DBFS_CHECK(!a.end.active, "bu_step: a folded level end needs the hub kernels' fused finish");
  bu_kernel<<<grid_for(a.words, kUnitWords), kUnitThreads, 0, st>>>(a);
  if (a.fuse_scan) totals_finish(a.scan, st);
}

void bu_cut_prep(const BuArgs& a, hipStream_t st) {
  DBFS_CHECK(a.cut_edges > 0 && a.cut_flag && (a.level8 || a.cut_claim) && a.g.hub_bits && a.ctrl,
             "bu_cut_prep: hub-cut arguments missing");
  const bool x = a.cut_bytes != nullptr;
  DBFS_CHECK(!x || (a.cut_vis && a.cut_word_off >= 0), "bu_cut_prep: several ranks' claim arguments missing");
  DBFS_CHECK(x || a.g.lo == 0, "bu_cut_prep: a shard past vertex 0 needs the several-rank arguments");
  // (grid measured flat from 256 to 4096 workgroups)
  const unsigned grid = grid_for(a.words, kCutThreads, 2 * device_cus());
  if (x) bu_cut_prep_kernel<true><<<grid, kCutThreads, 0, st>>>(a);
  else bu_cut_prep_kernel<false><<<grid, kCutThreads, 0, st>>>(a);
}

void bu_cut_merge(const BuArgs& a, hipStream_t st) {
  DBFS_CHECK(a.cut_flag && a.cut_recv && a.cut_next && (a.level8 || a.cut_claim) && a.cut_nranks > 1 &&
                 a.cut_rank >= 0 && a.cut_rank < a.cut_nranks && a.words > 0,
             "bu_cut_merge: several ranks' hub-cut arguments missing");
  bu_cut_merge_kernel<<<grid_for(a.words, kBlock), kBlock, 0, st>>>(a);
}

void hub_gather(const HubGatherArgs& a, hipStream_t st) {
  if (a.g.nhubs <= 0) return;
  DBFS_CHECK(!a.pull || (a.pull_out && a.pull_words > 0 && a.pull_nranks > 1 && a.pull_nranks <= kMaxDirectRanks &&
                         a.pull_rank >= 0 && a.pull_rank < a.pull_nranks),
             "hub_gather: pushed-slice arguments incomplete");
  // (with the visited merge or pushed slices: at least a grid striding over
  // the words well -- <= kHgCopyGrid workgroups, the cut decision's part sums
  // are sized for that)
  unsigned grid = grid_for(a.g.nhubs, kHgThreads * kHgPer);
  if (a.visited || a.pull)
    grid = std::max(grid, grid_for(a.pull ? a.pull_words * a.pull_nranks : a.words, kHgThreads, kHgCopyGrid));
  if (a.cut_part) {
    DBFS_CHECK(a.cut_flag && a.cut_ticket && a.ctrl, "hub_gather: the hub-cut decision needs a flag, a ticket and the level state");
    hub_gather_kernel<true, kHgThreads, kHgPer><<<grid, kHgThreads, 0, st>>>(a);
    return;
  }
  // (one hub per thread: 256 workgroups for 2^16 hubs, the loads of the
  // whole chip in flight -- 4 per thread over 16 workgroups measured 5.0 ->
  // 5.6 us a level)
  unsigned pgrid = grid_for(a.g.nhubs, kBlock);
  if (a.visited || a.pull)
    pgrid = std::max(pgrid, grid_for(a.pull ? a.pull_words * a.pull_nranks : a.words, kBlock, 4 * kHgCopyGrid));
  hub_gather_kernel<false, kBlock, 1><<<pgrid, kBlock, 0, st>>>(a);
}

unsigned long long take_check_bu() { return take_check_local(); }

}  // namespace kern
}  // namespace dbfs
