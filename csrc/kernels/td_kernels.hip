// gfx950 top-down kernels: edge-balanced expansion (td_expand), one-kernel
// sparse levels from a work list or straight from a bottom-up level's bitmap
// (td_sparse, td_sparse_bits), the owners' side of the owner-list exchange
// (td_sparse_apply, direct exchanges and their self-test), binned levels
// (propagation blocking) and the top-down hub marks.
//
// Reference counterpart: queueBfs (bfs.cu:134-165), a thread per frontier
// vertex walking its row serially with an atomicMin claim per edge.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <type_traits>

#include "kernel_common.hpp"
#include "launch.hpp"
#include "level_device.hpp"
#include "wave.hpp"

namespace dbfs {
namespace kern {
namespace {

// ---------------------------------------------------------------------------
// Edge-balanced top-down expansion.  Workgroup b owns frontier edges
// [b*EPB, (b+1)*EPB).  The entries covering that range are [blk_vstart[b],
// blk_vstart[b+1]]; their start positions are scattered into an LDS owner map
// and max-scanned so every edge finds its entry with one LDS read.  col[] is
// then read in 256-lane coalesced sweeps.  A discovered vertex costs one
// atomicOr only if neither `visited` nor the (possibly stale, only-growing)
// `next` word already has its bit.
enum class TdOut { Bits, Bytes, Lists, Dyn };  // Dyn: bits or bytes per ctrl->bytes

// Work-list owner map of edge block b (edges [b*EPB, min(m, (b+1)*EPB))):
// the entries covering the block are [blk_vstart[b], blk_vstart[b+1]]; their
// start positions are scattered into s_owner and max-scanned, so s_owner[i]
// is the block-local entry of edge i and s_base[entry] its qbase (col index =
// edge + qbase).  Returns the block's edge count; ends with a barrier.
// BaseT uint32_t: qbase kept modulo 2^32 (enough while the column array has
// at most 2^32 entries: the column index is then (edge + qbase) mod 2^32).
// kSpan > 1: super-block b of kSpan consecutive edge blocks (edges [b * kSpan
// * EPB, ...), nblocks still counting edge blocks): s_owner / s_base hold
// kSpan x EPB (+ 1) entries.
// OwnerT: int32_t, or uint16_t where LDS is tight (entries <= kSpan x EPB + 1
// < 2^16).
template <int kThreads, typename BaseT = long long, int kSpan = 1, typename OwnerT = int32_t>
__device__ __forceinline__ int td_block_owner_map(const int64_t* __restrict__ qscan, const int64_t* __restrict__ qbase,
                                                  const int32_t* __restrict__ blk_vstart, long long b,
                                                  long long nblocks, long long q, long long m, OwnerT* s_owner,
                                                  BaseT* s_base, int32_t* s_wmax) {
  static_assert(sizeof(OwnerT) >= 4 || kSpan * kTdEdgesPerBlock < 65535, "owner map entries fit OwnerT");
  constexpr int kEPB = kSpan * kTdEdgesPerBlock;
  constexpr int kItems = kEPB / kThreads;
  const int t = threadIdx.x;
  const int lane = lane_id();
  const int wv = t >> 6;
  const long long e0 = b * kEPB;
  const long long e1 = min(m, e0 + kEPB);
  const int cnt = static_cast<int>(e1 - e0);
  const long long v0 = blk_vstart[b * kSpan];
  const long long vlast = (b * kSpan + kSpan < nblocks) ? blk_vstart[b * kSpan + kSpan] : q - 1;
  const int nv = static_cast<int>(vlast - v0 + 1);

  // Invariant (zero-degree vertices are never listed): nv <= EPB + 1.  Every
  // entry's work-list words are loaded at once (a block of low-degree
  // vertices -- a sparse level's tail -- covers up to EPB + 1 entries, which
  // a strided loop fetched one dependent round trip after another), in
  // flight across the barriers of the owner map's zeroing.
  constexpr int kMapIter = (kEPB + kThreads) / kThreads;
  long long qs[kMapIter];
  BaseT qb[kMapIter];
#pragma unroll
  for (int k = 0; k < kMapIter; ++k) {
    const int i = t + k * kThreads;
    qs[k] = 0;
    qb[k] = 0;
    if (i < nv && i <= kEPB) {
      qs[k] = qscan[v0 + i];
      qb[k] = static_cast<BaseT>(qbase[v0 + i]);
    }
  }
  __syncthreads();  // LDS reuse across iterations
#pragma unroll
  for (int k = 0; k < kItems; ++k) s_owner[k * kThreads + t] = 0;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kMapIter; ++k) {
    const int i = t + k * kThreads;
    if (i < nv && i <= kEPB) {
      s_base[i] = qb[k];
      const long long p = (qs[k] > e0 ? qs[k] : e0) - e0;
      if (p < cnt) s_owner[p] = static_cast<OwnerT>(i);
    }
  }
  __syncthreads();
  // inclusive max-scan over s_owner: thread t owns entries [t*ITEMS, (t+1)*ITEMS)
  int vals[kItems];
  int run = 0;
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    run = max(run, static_cast<int>(s_owner[t * kItems + k]));
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
  for (int k = 0; k < kItems; ++k) s_owner[t * kItems + k] = static_cast<OwnerT>(max(vals[k], excl));
  __syncthreads();
  return cnt;
}

// kThreads: 256 (8 edges per thread) for big levels; 1024 (2 per thread) when
// the grid is too small to fill the chip -- 4x the waves in flight to cover the
// latency of the scattered loads/atomics.  The grid may be smaller than the
// number of edge blocks (device loop: fixed grid): workgroups stride over them.
#ifdef DBFS_TD_STATS
// Diagnostic build only (-DDBFS_TD_STATS): per-dispatch top-down counters
// (live edges, hub targets decoded unvisited, direct stores, filter on).
__device__ unsigned long long g_td_stats[4];
#define TD_STAT(i, x)                                              \
  do {                                                             \
    const unsigned long long v_ = (x);                             \
    if (lane_id() == 0 && v_) atomicAdd(&g_td_stats[i], v_);       \
  } while (0)
#else
#define TD_STAT(i, x) \
  do {                \
  } while (0)
#endif

// The items of one edge block (after td_block_owner_map): every item's
// column id loaded first (all in flight together: the items of a thread are
// independent, but the compiler cannot move a load above an earlier item's
// atomic, so one item at a time would cost kItems dependent round trips);
// then, with the hub filter, hub targets tested in the LDS snapshot: a
// visited hub is done here; an unvisited one is marked (td_hub_mark: its
// level byte stored by hub_apply) or decoded (hubnew: unvisited at the
// level's start, no global visited probe needed).  (Measured: claiming hubs
// in LDS as well, to store each once per workgroup, is slower -- few repeats
// per workgroup, LDS atomics on popular hubs serialise.)
template <int kThreads, bool kHubFilter, bool kBase32, typename BaseT, int kItems = kTdEdgesPerBlock / kThreads,
          typename OwnerT = int32_t>
__device__ __forceinline__ void td_load_items(const TdArgs& a, const vid_t* __restrict__ col, long long e0, int cnt,
                                              const OwnerT* s_owner, const BaseT* s_base, bool filter,
                                              const word_t* s_hubvis, vid_t (&vk)[kItems], bool (&live)[kItems],
                                              bool (&hubnew)[kItems]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    const int idx = k * kThreads + t;
    int64_t ci;
    if constexpr (kBase32)
      ci = static_cast<uint32_t>(static_cast<uint32_t>(e0 + idx) + s_base[s_owner[idx]]);
    else
      ci = e0 + idx + s_base[s_owner[idx]];
    vk[k] = idx < cnt ? __builtin_nontemporal_load(col + ci) : 0u;
    live[k] = idx < cnt;
    hubnew[k] = false;
  }
  if constexpr (kHubFilter) {
    if (filter) {
#pragma unroll
      for (int k = 0; k < kItems; ++k) {
        if (live[k] && (vk[k] & kHubFlag)) {
          const vid_t h = vk[k] & ~kHubFlag;
          if ((s_hubvis[h >> 6] >> (h & 63)) & 1ull) {
            live[k] = false;
          } else if (a.td_hub_mark) {
            a.td_hub_mark[h] = 1;  // claimed; hub_apply stores its level byte
            live[k] = false;
          } else {
            vk[k] = a.g.td_hub_vertex[h];
            hubnew[k] = true;
          }
        }
      }
    }
  }
}

// kFilter: the hub-filter variant (kTdMaxHubs / 8 bytes more LDS --
// launched only for levels that may use it).  kBase32: the owner map's column
// bases in 32 bits (graphs of at most 2^32 adjacency entries): 16 instead of
// 24 KiB of LDS per workgroup, 8 resident workgroups per CU instead of 6 (5
// instead of 4 with the filter).
// kUnvis: the unvisited-filter variant (TdArgs::unvis staged in LDS; 1024
// threads, no hub filter, Dyn output): a target whose filter bit is clear is
// visited, so only the others cost a `visited` probe.
template <TdOut kOut, int kThreads, bool kFilter = false, bool kBase32 = false, bool kUnvis = false>
__global__ __launch_bounds__(kThreads) void td_expand_kernel(TdArgs a) {
  // (the filter variant takes two edge blocks per step: its LDS allows two
  // workgroups per CU, so each keeps twice the edges in flight)
  constexpr int kSpan = kUnvis ? kUnvisSpan : 1;
  constexpr int kEPB = kSpan * kTdEdgesPerBlock;
  constexpr int kItems = kEPB / kThreads;
  constexpr bool kHubFilter = kFilter && kOut != TdOut::Lists && kThreads == kTdThreads;
  static_assert(!kUnvis || (!kFilter && kOut == TdOut::Dyn), "the unvisited filter replaces the hub filter");
  using BaseT = std::conditional_t<kBase32, uint32_t, long long>;
  // (the filter variant's owner map in 16 bits: 8 KiB more for the filter)
  using OwnerT = std::conditional_t<kUnvis, uint16_t, int32_t>;
  __shared__ OwnerT s_owner[kEPB];
  __shared__ BaseT s_base[kEPB + 1];
  __shared__ int32_t s_wmax[kThreads / kWave];
  __shared__ word_t s_hubvis[kHubFilter ? kTdMaxHubs / kWordBits : 1];
  __shared__ word_t s_unvis[kUnvis ? kUnvisWords : 1];
  __shared__ int s_unvis_on;
  long long q = a.q, m = a.m;
  bool bytes = kOut == TdOut::Bytes, check = a.check_visited;
  if (a.ctrl) {
    if (!chain_live(*a.ctrl, 'T', a.max_mf)) return;
    bytes = a.ctrl->bytes != 0;
    check = a.ctrl->check_visited != 0;
    q = a.dev_stats[0];
    m = a.dev_stats[1];
    if (a.clear_qv) stamp_level_start(a.ctrl);  // first kernel of the level (no compaction)
    if (a.clear_qv)
      for (int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i < q;
           i += static_cast<int64_t>(gridDim.x) * kThreads) {
        const vid_t r = a.clear_qv[i];
        a.clear_frontier[r >> 6] = 0ull;
      }
  }
  const long long nblocks = (m + kTdEdgesPerBlock - 1) / kTdEdgesPerBlock;
  const long long nsteps = (nblocks + kSpan - 1) / kSpan;
  // a split level's part (TdArgs::split_k): its run [s_lo, s_hi) of the steps
  const long long s_lo = a.split_k > 1 ? nsteps * a.split_i / a.split_k : 0;
  const long long s_hi = a.split_k > 1 ? nsteps * (a.split_i + 1) / a.split_k : nsteps;
  const int t = threadIdx.x;
  const int lane = lane_id();
  const word_t* __restrict__ visited = a.visited;
  // a level with an unvisited filter (TdArgs::unvis_pop) runs in exactly one
  // of the two variants launched for it: the filter one if the filter's set
  // bits are at most unvis_max_density of them, else the plain one
  if (a.unvis_pop) {
    if (t < kWave) {
      long long c = 0;
      for (int i = t; i < kUnvisChunks; i += kWave) c += a.unvis_pop[i];
      c = wave_sum(c);
      if (t == 0) s_unvis_on = static_cast<double>(c) <= a.unvis_max_density * static_cast<double>(kUnvisBits) ? 1 : 0;
    }
    __syncthreads();
    if ((s_unvis_on != 0) != kUnvis) return;
  }
  // large levels: hub targets tested in an LDS copy of the hubs' visited bits
  // (uniform: every workgroup sees the same m)
  bool filter = false;
  if constexpr (kHubFilter) {
    filter = a.td_hub_vis && a.g.td_col && m >= a.td_hub_min_edges && blockIdx.x < s_hi - s_lo &&
             (!a.ctrl || static_cast<double>(a.ctrl->vis_deg) >= a.td_hub_vis_frac * a.ctrl->total_directed);
    if (filter) {
      const int64_t hw = (a.g.td_nhubs + kWordBits - 1) / kWordBits;
      stage_words<kThreads, kTdMaxHubs / kWordBits>(s_hubvis, a.td_hub_vis, hw);
      // (td_block_owner_map starts with a barrier)
    }
  }
  const vid_t* __restrict__ col = filter ? a.g.td_col : a.g.col;
  // (td_block_owner_map starts with a barrier)
  if constexpr (kUnvis)
    if (blockIdx.x < s_hi - s_lo) stage_words<kThreads, kUnvisWords>(s_unvis, a.unvis, kUnvisWords);
  const uint64_t umult = a.unvis_mult;

  for (long long b = s_lo + blockIdx.x; b < s_hi; b += gridDim.x) {
    const long long e0 = b * kEPB;
    const int cnt = td_block_owner_map<kThreads, BaseT, kSpan, OwnerT>(a.qscan, a.qbase, a.blk_vstart, b, nblocks, q,
                                                                       m, s_owner, s_base, s_wmax);

    vid_t vk[kItems];
    bool live[kItems], hubnew[kItems];
    td_load_items<kThreads, kHubFilter, kBase32, BaseT, kItems, OwnerT>(a, col, e0, cnt, s_owner, s_base, filter,
                                                                        s_hubvis, vk, live, hubnew);
    if constexpr (kUnvis) {
      // filter bit clear: visited at the level's start -- no probe, no store
#pragma unroll
      for (int k = 0; k < kItems; ++k) {
        const uint32_t fi = unvis_index(vk[k], umult);
        live[k] = live[k] && ((s_unvis[fi >> 6] >> (fi & 63)) & 1ull);
      }
    }
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      DBFS_DCHECK(!live[k] || vk[k] < a.g.n, 2, vk[k]);
      TD_STAT(0, __popcll(__ballot(live[k])));
      TD_STAT(1, __popcll(__ballot(hubnew[k])));
    }
    TD_STAT(3, filter && t == 0 && b == blockIdx.x ? 1 : 0);
    if constexpr (kOut != TdOut::Lists) {
      if (!bytes) {
        word_t seen[kItems];
#pragma unroll
        for (int k = 0; k < kItems; ++k)
          seen[k] = live[k] ? (hubnew[k] ? 0ull : (visited[vk[k] >> 6] | a.next[vk[k] >> 6])) : ~0ull;
#pragma unroll
        for (int k = 0; k < kItems; ++k) {
          const word_t bit = 1ull << (vk[k] & 63);
          if (!(seen[k] & bit)) atomicOr(a.next + (vk[k] >> 6), bit);
        }
        continue;
      }
      if (a.level_direct) {
        // the level itself, for unreached candidates only: the level byte is
        // read instead of the visited bit (a reached vertex -- earlier level,
        // or claimed at this one -- reads something other than unreached), so
        // a target hit by many edges is stored about once instead of once per
        // edge (stores cost more than reads; a stale read in another XCD's L2
        // only repeats the same store)
        // The candidate's visited bit is tested (measured, RMAT-22 top-down
        // only: 65.0 GTEPS, against 60.0 testing the level byte, 58.0 both,
        // 55.3 with claims in `next`; the 43 M-edge level stores 29.8 M level
        // bytes for ~2 M new vertices, and removing the repeats with extra
        // reads costs more L2 requests than the writes, tools/gpu_td_stats_roots.sh).
        // Plain stores: write-through (sc1) or non-temporal ones measured slower,
        // RMAT-22 88.4 -> 74.8 / 69.3 GTEPS, LJ-sized 56.7 -> 51.4 / 52.0
        // (profiles/r4_s2_td_store_modes.txt).
        const uint8_t lv = static_cast<uint8_t>(a.narrow_base + a.new_level);
        bool keep[kItems];
#pragma unroll
        for (int k = 0; k < kItems; ++k)
          keep[k] = live[k] && (hubnew[k] || !(visited[vk[k] >> 6] & (1ull << (vk[k] & 63))));
#pragma unroll
        for (int k = 0; k < kItems; ++k) TD_STAT(2, __popcll(__ballot(keep[k])));
#pragma unroll
        for (int k = 0; k < kItems; ++k)
          if (keep[k]) a.level_direct[vk[k]] = lv;
        continue;
      }
      // byte map: with few visited vertices the check costs more than the
      // store it saves (random loads ~120 G/s vs byte stores ~88 G/s on
      // MI355X); the consuming update masks with ~visited anyway.  A byte
      // already marked is not stored again (RMAT rows repeat the same hubs,
      // and a read hit is cheaper than a byte write).
      bool keep[kItems];
#pragma unroll
      for (int k = 0; k < kItems; ++k)
        keep[k] = live[k] && (hubnew[k] || !check || !(visited[vk[k] >> 6] & (1ull << (vk[k] & 63))));
      uint8_t mark[kItems];
#pragma unroll
      for (int k = 0; k < kItems; ++k) mark[k] = keep[k] ? a.next_bytes[vk[k]] : 1;
#pragma unroll
      for (int k = 0; k < kItems; ++k)
        if (!mark[k]) a.next_bytes[vk[k]] = 1;
      continue;
    }
    bool actk[kItems];
#pragma unroll
    for (int k = 0; k < kItems; ++k)
      actk[k] = k * kThreads + t < cnt && !(visited[vk[k] >> 6] & (1ull << (vk[k] & 63)));
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      if constexpr (kOut == TdOut::Lists) {
        // wave-aggregated append to the owner lists (uniform loop over owners)
        const vid_t v = vk[k];
        const bool act = actk[k];
        const int owner = act ? static_cast<int>(v / a.part) : -1;
        unsigned long long pending = __ballot(act);
        while (pending) {
          const int leader = __ffsll(static_cast<long long>(pending)) - 1;
          const int o = __shfl(owner, leader, kWave);
          const unsigned long long msk = __ballot(owner == o);
          unsigned base = 0;
          vid_t* list = a.lists + static_cast<int64_t>(o) * (a.list_cap + 1);
          if (lane == leader) base = atomicAdd(list, static_cast<unsigned>(__popcll(msk)));
          base = __shfl(base, leader, kWave);
          DBFS_DCHECK(base + __popcll(msk) <= static_cast<unsigned long long>(a.list_cap), 3, base);
          if (owner == o) list[1 + base + mask_rank(msk)] = v;
          pending &= ~msk;
        }
      }
    }
  }
}

// The claimed, owned items of a lane (bit k of `claimed`: v[k], a global id
// of this shard): level, frontier bit, and the wave's work-list entries of
// the next level with one packed atomic (count << kSparseEdgeBits | edges)
// for all of them, so entries stay ordered by edge offset.  Wave-uniform call.
// kWg: a workgroup-uniform call (every wave of a workgroup of at most
// kSettleWaves waves): the waves' packed counts summed in LDS and ONE atomic
// per workgroup on the counter, each wave's base from the waves before it --
// a level settling thousands of waves' claims queued that many returning
// atomics on one address (~90 per us).
constexpr int kSettleWaves = 1024 / kWave;
template <int kItems, bool kWg = false>
__device__ __forceinline__ void sparse_settle(const TdSparseArgs& a, const vid_t (&v)[kItems], unsigned claimed) {
  constexpr unsigned long long kEdgeMask = (1ull << kSparseEdgeBits) - 1;
  if constexpr (!kWg) {
    if (!__ballot(claimed != 0)) return;
  }
  const int lane = lane_id();
  const eid_t* __restrict__ ro = a.g.row_off;
  const int64_t lo = a.g.lo;
  eid_t rs[kItems], re[kItems];
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    rs[k] = re[k] = 0;
    if (claimed & (1u << k)) {
      const int64_t r = static_cast<int64_t>(v[k]) - lo;
      DBFS_DCHECK(r >= 0 && r < a.g.rows, 10, v[k]);
      store_level(a.level, a.level8, r, a.new_level, a.narrow_base);
      rs[k] = ro[r];
      re[k] = ro[r + 1];
    }
  }
  unsigned long long tm[kItems];
  long long incl[kItems], cbase[kItems], ebase[kItems];
  long long ctot = 0, etot = 0;
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    const long long d = static_cast<long long>(re[k] - rs[k]);
    const bool take = d > 0;  // claimed (else rs == re)
    tm[k] = __ballot(take);
    if (take) {
      const int64_t r = static_cast<int64_t>(v[k]) - lo;
      atomicOr(a.frontier_out + (r >> 6), 1ull << (r & 63));
    }
    incl[k] = wave_incl_scan(take ? d : 0ll);
    cbase[k] = ctot;
    ebase[k] = etot;
    ctot += __popcll(tm[k]);
    etot += readlane_i64(incl[k], kWave - 1);
  }
  unsigned long long old = 0;
  const unsigned long long packed = (static_cast<unsigned long long>(ctot) << kSparseEdgeBits) +
                                    static_cast<unsigned long long>(etot);
  if constexpr (kWg) {
    __shared__ unsigned long long s_pk[kSettleWaves], s_pbase;
    const int wv = static_cast<int>(threadIdx.x >> 6);
    if (lane == 0) s_pk[wv] = packed;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long sum = 0;
      for (int k = 0; k < static_cast<int>(blockDim.x >> 6); ++k) sum += s_pk[k];
      s_pbase = sum ? atomicAdd(a.counter, sum) : 0ull;
    }
    __syncthreads();
    old = s_pbase;
    for (int k = 0; k < wv; ++k) old += s_pk[k];
    __syncthreads();  // (s_pk / s_pbase reused by the next call)
    if (!ctot) return;
  } else {
    if (!ctot) return;
    if (lane == 0) old = atomicAdd(a.counter, packed);
    old = __shfl(old, 0, kWave);
  }
  const long long p0 = static_cast<long long>(old >> kSparseEdgeBits);
  const long long q0 = static_cast<long long>(old & kEdgeMask);
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    const long long d = static_cast<long long>(re[k] - rs[k]);
    const long long p = p0 + cbase[k] + mask_rank(tm[k]);
    const long long qs = q0 + ebase[k] + incl[k] - d;
    DBFS_DCHECK(d <= 0 || p < a.g.rows, 4, p);
    if (d > 0) {
      a.oscan[p] = qs;
      a.obase[p] = rs[k] - qs;
      a.oqv[p] = static_cast<vid_t>(static_cast<int64_t>(v[k]) - lo);
    }
    wave_fill_blocks(a.oblk, d > 0, qs, d, p);
  }
}

// The level's local totals from the packed counter (one thread of the last
// workgroup): stats, the work list's end marker, counter and ticket reset.
__device__ __forceinline__ void sparse_totals(const TdSparseArgs& a, long long& cnt, long long& deg) {
  constexpr unsigned long long kEdgeMask = (1ull << kSparseEdgeBits) - 1;
  const unsigned long long tot = __hip_atomic_load(a.counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  cnt = static_cast<long long>(tot >> kSparseEdgeBits);
  deg = static_cast<long long>(tot & kEdgeMask);
  *a.counter = 0ull;
  *a.ticket = 0u;
  a.stats[0] = cnt;
  a.stats[1] = deg;
  a.oscan[cnt] = deg;
  a.stats[2] = cnt;
  a.stats[3] = deg;
}

// PeerComm::self_test of the direct exchanges (one workgroup): rank r sends
// peer p an owner list of (r + p + round) % 37 ids (+ 4000 in round 3) of a
// known pattern, then a level end of known totals; every count, id and sum
// checked against the pattern, mismatches counted in *err.
__device__ __forceinline__ uint32_t selftest_id(int from, int to, uint32_t i, int round) {
  return (static_cast<uint32_t>(from + 1) * 0x9E3779B9u) ^ (static_cast<uint32_t>(to + 7) << 20) ^ (i * 2654435761u) ^
         static_cast<uint32_t>(round * 977);
}
__device__ __forceinline__ uint32_t selftest_n(int from, int to, int round) {
  return static_cast<uint32_t>((from + to + round) % 37) + (round == 3 ? 4000u : 0u);
}
// The producer side runs as td_sparse's does: kSelftestGroups workgroups each
// store a strided share of every list (write-through, uneven: a workgroup's
// share depends on the list length), drain them, take a ticket, and the last
// arriver acquires and publishes the cells -- so the construction-time test
// covers the multi-workgroup publish path the sparse levels take, over the
// real links.  The last workgroup then runs the consumer side and the level end.
constexpr int kSelftestGroups = 8;
__global__ __launch_bounds__(256) void direct_selftest_kernel(DirectExchange l, DirectExchange e, int round,
                                                              unsigned* err, unsigned* ticket) {
  __shared__ uint64_t s_n[kern::kMaxPeers], s_x[2 * kern::kMaxPeers];
  __shared__ int s_last;
  const int t = threadIdx.x;
  const int me = l.rank, P = l.nranks;
  const uint32_t g0 = blockIdx.x * 256 + t, gs = gridDim.x * 256;
  for (int p = 0; p < P; ++p) {
    if (p == me) continue;
    const uint32_t n = selftest_n(me, p, round);
    for (uint32_t i = g0; i < n; i += gs) sys_store_u32(l.table->dst[p] + 1 + i, selftest_id(me, p, i, round));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    const unsigned prev = atomicAdd(ticket, 1u);
    s_last = prev == gridDim.x - 1 ? 1 : 0;
    if (s_last) {
      *ticket = 0u;
      last_arriver_acquire();
    }
  }
  __syncthreads();
  if (!s_last) return;
  if (t < P && t != me) sys_store_u64(l.table->cell_out[t], cell_word0(l.seq, selftest_n(me, t, round)));
  if (direct_wait(l, s_n, nullptr) != kWaitOk) {
    if (t == 0) atomicAdd(err, 1000000u);
    return;
  }
  unsigned bad = 0;
  for (int p = 0; p < P; ++p) {
    if (p == me) continue;
    const uint32_t n = selftest_n(p, me, round);
    if (t == 0 && s_n[p] != n) ++bad;
    const uint32_t m = min(static_cast<uint32_t>(s_n[p]), n);
    for (uint32_t i = t; i < m; i += 256)
      if (sys_load_u32(l.table->src[p] + 1 + i) != selftest_id(p, me, i, round)) ++bad;
  }
  // a level end of known totals: rank r contributes (r + round, r << 30 | round)
  const int64_t c = me + round, g = (static_cast<int64_t>(me) << 30) | round;
  if (t < P && t != me) {
    uint64_t* cell = e.table->cell_out[t];
    sys_store_u64(cell, cell_word0(e.seq, static_cast<uint64_t>(c)));
    sys_store_u64(cell + 1, cell_word1(e.seq, static_cast<uint64_t>(g)));
  }
  if (direct_wait(e, s_x, s_x + kern::kMaxPeers) != kWaitOk) {
    if (t == 0) atomicAdd(err, 1000000u);
    return;
  }
  if (t == 0) {
    int64_t sc = c, sg = g, wc = 0, wg = 0;
    for (int p = 0; p < P; ++p) {
      sc += p == me ? 0 : static_cast<int64_t>(s_x[p]);
      sg += p == me ? 0 : static_cast<int64_t>(s_x[kern::kMaxPeers + p]);
      wc += p + round;
      wg += (static_cast<int64_t>(p) << 30) | round;
    }
    if (sc != wc || sg != wg) ++bad;
  }
  if (bad) atomicAdd(err, bad);
}

// Several ranks, after the list exchange: the ids the other ranks claimed for
// this rank's vertices (recv_lists) are claimed here (fetch-or on the owned
// slice of `visited`; a vertex sent by several ranks, or claimed by this
// rank's own td_sparse, is settled once) and settled like td_sparse's owned
// claims; the last workgroup writes the level's local totals and zeroes the
// send lists' counts.  The lists' counts are loaded together (one per
// thread: they sit a stride apart, cold) and their entries form one index
// space the grid strides over.
// (bx / gx: this workgroup and the workgroups taking part -- the kernel's, or
// the one last workgroup of a fused tiny level, TdSparseArgs::fuse_apply)
// (live: called from a live td_sparse -- the chain check is not repeated: the
// level's own finish, the only writer of *ctrl, comes after it)
template <int kThreads, bool kWg = true>
__device__ __forceinline__ void sparse_apply(const TdSparseArgs& a, unsigned bx, unsigned gx, bool live = false) {
  constexpr int kItems = kTdEdgesPerBlock / kThreads;
  __shared__ int s_last;
  __shared__ long long s_end[kern::kMaxPeers];  // inclusive prefix of the counts
  __shared__ const vid_t* s_src[kern::kMaxPeers];
  __shared__ uint64_t s_cnt[kern::kMaxPeers];
  __shared__ uint64_t s_xend[2 * kern::kMaxPeers];
  // a direct exchange: the peers' cells (their counts) first, live chain or
  // not (every rank waits for every exchange: the window slots' reuse protocol)
  const bool dx = a.direct.active;
  if (dx && direct_wait(a.direct, s_cnt, nullptr) != kWaitOk) return;
  if (!live && !chain_live(*a.ctrl, 'T', a.max_mf)) {
    // a folded level end is a collective: it runs on a no-op chain too
    if (a.end.active && bx == 0) direct_level_end(a.end, a.stats[2], a.stats[3], a.stats, a.fin, s_xend);
    return;
  }
  const int t = threadIdx.x;
  if (t < kWave) {
    long long n = 0;
    if (t < a.nranks) {
      const vid_t* src = dx ? a.direct.table->src[t] : a.recv_lists + static_cast<int64_t>(t) * a.list_stride;
      s_src[t] = src;
      n = dx ? static_cast<long long>(s_cnt[t]) : static_cast<long long>(*src);
    }
    DBFS_DCHECK(n < a.list_stride, 5, n);
    const long long incl = wave_incl_scan(n);
    if (t < a.nranks) s_end[t] = incl;
  }
  __syncthreads();
  const long long total = s_end[a.nranks - 1];
  const int64_t span = static_cast<int64_t>(kThreads) * kItems;
  // only the workgroups with entries take part (at least one, for the finish)
  const int64_t need = (total + span - 1) / span;
  const unsigned active = static_cast<unsigned>(need < 1 ? 1 : (need < gx ? need : gx));
  if (bx >= active) return;
  for (int64_t i0 = static_cast<int64_t>(bx) * span; i0 < total; i0 += static_cast<int64_t>(active) * span) {
    vid_t v[kItems];
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int64_t j = i0 + static_cast<int64_t>(k) * kThreads + t;
      v[k] = 0u;
      if (j < total) {
        int r = 0;
        while (s_end[r] <= j) ++r;  // (<= kMaxPeers lists)
        const long long before = r > 0 ? s_end[r - 1] : 0;
        const vid_t* src = s_src[r] + 1 + (j - before);
        v[k] = dx ? sys_load_u32(src) : *(const gu32*)(src);
      }
    }
    // the received ids are claimed by fetch-or straight away: the senders
    // already dropped what their copy of `visited` held, so a visited pre-read
    // mostly found the bit clear and cost a round trip before the atomic
    // (shadow rank 0 of RMAT-26: P = 8 897-908 -> 888-893 us, P = 2 flat)
    unsigned claimed = 0;
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const word_t bit = 1ull << (v[k] & 63);
      if (i0 + static_cast<int64_t>(k) * kThreads + t < total && !(atomicOr(a.visited + (v[k] >> 6), bit) & bit))
        claimed |= 1u << k;
    }
    sparse_settle<kItems, kWg>(a, v, claimed);
  }
  __syncthreads();
  if (t == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // (one workgroup taking part -- a fused tiny level's, or a small level's:
    // trivially the last, no ticket)
    const unsigned prev = (gx == 1 || active == 1) ? 0u : atomicAdd(a.ticket, 1u);
    s_last = (prev == active - 1) ? 1 : 0;
    if (s_last && active > 1) last_arriver_acquire();
  }
  __syncthreads();
  if (!s_last) return;
  // the send lists were read by the exchange (stream-ordered before this
  // kernel): their counts restart from zero for the next list level (a
  // direct exchange's publisher zeroed them)
  if (!dx && t < a.nranks) a.lists[static_cast<int64_t>(t) * a.list_stride] = 0u;
  __shared__ long long s_tot[2];
  if (t == 0) {
    long long cnt = 0, deg = 0;
    sparse_totals(a, cnt, deg);
    s_tot[0] = cnt;
    s_tot[1] = deg;
  }
  if (!a.end.active) return;
  __syncthreads();
  direct_level_end(a.end, s_tot[0], s_tot[1], a.stats, a.fin, s_xend);
}

template <int kThreads>
__global__ __launch_bounds__(kThreads) void td_sparse_apply_kernel(TdSparseArgs a) {
  sparse_apply<kThreads>(a, blockIdx.x, gridDim.x);
}

// A direct exchange's wait on its own (Comm::split_waits: ranks sharing a
// GPU): one wave polls the peers' cells, and the consumer launched after it
// on the same stream finds them tagged at its first poll -- so no grid
// spins in every workgroup while a co-resident rank's producer waits for
// CUs.  (Ranks on separate GPUs keep the wait in the consumer: their
// producers never compete with it for a CU.)
__global__ __launch_bounds__(kWave) void direct_prewait_kernel(DirectExchange x) {
  __shared__ uint64_t s_n[kern::kMaxPeers];
  (void)direct_wait(x, s_n, nullptr);
}

// Sparse top-down level (TdSparseArgs): expansion as td_expand, then every
// claimed vertex is finished in place (level, frontier bit, output entry), so
// the level is one launch (one rank); with several ranks remote claims go to
// their owners' lists and td_sparse_apply finishes the level after the
// exchange.  kThreads = 1024: 2 edges per thread per block.
constexpr int kTdSparseThreads = 1024;
constexpr long long kTdWgSettleBlocks = 32;  // (one rank: td_sparse's per-workgroup settle from here)
// kWg: several ranks (owner lists) -- settles aggregated per workgroup
// (sparse_settle); one rank keeps the per-wave form (its registers).
template <int kThreads, bool kWg = false>
__global__ __launch_bounds__(kThreads) void td_sparse_kernel(TdSparseArgs a) {
  constexpr int kItems = kTdEdgesPerBlock / kThreads;
  __shared__ int32_t s_owner[kTdEdgesPerBlock];
  __shared__ long long s_base[kTdEdgesPerBlock + 1];
  __shared__ int32_t s_wmax[kThreads / kWave];
  __shared__ int s_last;
  // (kWg: several ranks -- the launcher's choice whenever there are owner
  // lists, so the one-rank variant compiles none of their code)
  const bool dx = kWg && a.lists && a.direct.active;
  if (a.late_ticks) {
    // fault injection: a workgroup that will take no ticket starts late
    const long long m0 = a.dev_stats[1];
    const long long nb0 = (m0 + kTdEdgesPerBlock - 1) / kTdEdgesPerBlock;
    if (static_cast<long long>(blockIdx.x) >= (nb0 < 1 ? 1 : nb0)) {
      const uint64_t t0 = wall_clock64();
      while (wall_clock64() - t0 < a.late_ticks) __builtin_amdgcn_s_sleep(8);
    }
  }
  // (the input totals loaded with the chain check: one round trip for both;
  // dev_stats is valid memory on a no-op chain too)
  const long long q = a.dev_stats[0], m = a.dev_stats[1];
  // uniform: the whole grid returns, no workgroup takes a ticket (a direct
  // exchange still publishes, empty)
  if (!chain_live(*a.ctrl, 'T', a.max_mf)) {
    if (dx && blockIdx.x == 0) {
      direct_publish(a.direct, a.lists, a.list_stride, false);
      // (the fused owner side waits for the peers all the same: a collective)
      if (a.fuse_apply) sparse_apply<kThreads, kWg>(a, 0, 1);
    }
    return;
  }
  if (a.first) stamp_level_start(a.ctrl);
  const long long nblocks = (m + kTdEdgesPerBlock - 1) / kTdEdgesPerBlock;
  // Only the workgroups that have an edge block take part (at least one, for
  // the finish): the others return before the ticket -- on a level of a few
  // blocks, 256 workgroups queueing on one ticket address cost several us.
  const unsigned active = static_cast<unsigned>(nblocks < 1 ? 1 : (nblocks < gridDim.x ? nblocks : gridDim.x));
  if (blockIdx.x >= active) return;
  // one rank, a level of many edge blocks: claims settled per workgroup too
  // (one counter atomic each, as with several ranks) -- hundreds of
  // workgroups' per-wave atomics on the one counter queue (~90 per us); a
  // small level keeps the per-wave form (the workgroup form's barriers cost
  // it ~2 us).  (Workgroup-uniform: nblocks is.)
#ifdef DBFS_NO_WG_SETTLE
  constexpr bool wg_settle = false;  // (diagnostic build: same-box A/B)
#else
  const bool wg_settle = nblocks >= kTdWgSettleBlocks;
#endif
  const int t = threadIdx.x;
  const int64_t gtid = static_cast<int64_t>(blockIdx.x) * kThreads + t;
  const int64_t gstride = static_cast<int64_t>(active) * kThreads;
  // the input vertices' frontier bits (the bitmap is not read here)
  for (int64_t i = gtid; i < q; i += gstride) {
    const vid_t r = a.qv[i];
    a.frontier_in[r >> 6] = 0ull;
  }

  const vid_t* __restrict__ col = a.g.col;
  const uint64_t lo = static_cast<uint64_t>(a.g.lo), rows = static_cast<uint64_t>(a.g.rows);
  for (long long b = blockIdx.x; b < nblocks; b += active) {
    const long long e0 = b * kTdEdgesPerBlock;
    const int cnt = td_block_owner_map<kThreads>(a.qscan, a.qbase, a.blk_vstart, b, nblocks, q, m, s_owner, s_base,
                                                 s_wmax);
    // (A) all items' claims in flight together: col, visited, fetch-or
    vid_t v[kItems];
    word_t seen[kItems];
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int idx = k * kThreads + t;
      v[k] = idx < cnt ? col[e0 + idx + s_base[s_owner[idx]]] : 0u;
    }
#pragma unroll
    for (int k = 0; k < kItems; ++k) seen[k] = k * kThreads + t < cnt ? a.visited[v[k] >> 6] : ~0ull;
    unsigned claimed = 0;  // bit k: item k claimed by this lane
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const word_t bit = 1ull << (v[k] & 63);
      if (!(seen[k] & bit) && !(atomicOr(a.visited + (v[k] >> 6), bit) & bit)) claimed |= 1u << k;
    }
    if (kWg && a.lists) {
      // several ranks: claimed remote targets to their owners' lists
      unsigned remote = 0;
#pragma unroll
      for (int k = 0; k < kItems; ++k)
        if (((claimed >> k) & 1u) && static_cast<uint64_t>(v[k]) - lo >= rows) remote |= 1u << k;
      claimed &= ~remote;
      if constexpr (kWg) {
        // (the whole workgroup: one count atomic per owner and block)
        owner_list_append_wg<kItems>(a.lists, a.list_stride, a.part, a.nranks, v, remote,
                                     dx ? a.direct.table : nullptr);
      } else if (__ballot(remote != 0)) {
        owner_list_append_items<kItems>(a.lists, a.list_stride, a.part, v, remote, dx ? a.direct.table : nullptr);
      }
    }
    // (B) finish the claimed vertices (the whole workgroup: one counter atomic)
    if constexpr (kWg) sparse_settle<kItems, true>(a, v, claimed);
    else if (wg_settle) sparse_settle<kItems, true>(a, v, claimed);
    else sparse_settle<kItems, false>(a, v, claimed);
  }
  if (kWg && a.lists) {
    // several ranks: td_sparse_apply finishes the level.  A direct exchange:
    // every wave's write-through stores drained, the workgroups' ticket, and
    // the last one publishes the counts and flags.
    if (!dx) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      // (one active workgroup -- a tiny level: trivially the last, no
      // ticket round trip; every wave drained its stores before the barrier)
      const unsigned prev = active == 1 ? 0u : atomicAdd(a.ticket, 1u);
      s_last = (prev == active - 1) ? 1 : 0;
      if (s_last && active > 1) {
        *a.ticket = 0u;  // (the apply's ticket next, stream-ordered)
        // the counts the publish reads were added by every workgroup's
        // waves; the ids are write-through stores every wave drained before
        // its workgroup's ticket (the peers read them with system-scope loads
        // behind the cell).  The acquire orders this workgroup's reads after
        // the ticket, as every other last arriver's.
        last_arriver_acquire();
      }
    }
    __syncthreads();
    if (!s_last) return;
    direct_publish(a.direct, a.lists, a.list_stride, true);
    // a tiny level (fuse_apply): this workgroup is also the owner side --
    // the peers' lists, their claims and the folded level end -- instead of
    // a td_sparse_apply launch
    if (a.fuse_apply) sparse_apply<kThreads, kWg>(a, 0, 1, true);
    return;
  }

  // last workgroup: the level's totals and decision (as scan_units_kernel)
  __syncthreads();
  if (t == 0) {
    // every wave's counter atomic has returned.  (No release: the last
    // workgroup reads only the counter, a device-scope atomic; the level's
    // stores are read by later launches.)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // (one active workgroup -- a tail level: trivially the last, no ticket
    // round trip; its own atomics are ordered by the s_waitcnt)
    const unsigned prev = active == 1 ? 0u : atomicAdd(a.ticket, 1u);
    s_last = (prev == active - 1) ? 1 : 0;
    if (s_last && active > 1) last_arriver_acquire();
  }
  __syncthreads();
  if (!s_last) return;
  if (t != 0) return;
  long long cnt = 0, deg = 0;
  sparse_totals(a, cnt, deg);
  LevelCtrl c = *a.ctrl;
  finish_level(a.ctrl, c, cnt, deg, false, a.rec, a.mailbox, a.level_index);
}

// Sparse top-down level read straight from the bitmap a bottom-up level left
// (TdSparseArgs::from_bits) -- in place of scan_units + compact + td_sparse,
// three launches whose scan must see every unit's count before any work list
// exists.  A wave per 64-word unit, grid-strided, kBitsPre units' words loaded
// at once (zeroed as read); a unit's frontier vertices 64 per step, their
// edges expanded kItems x 64 per round from the wave's prefix sum of their
// degrees (an edge's vertex by a binary search over the prefixes in LDS);
// claims, owner lists and settling as td_sparse.  The level ends in the last
// workgroup of a two-level ticket.
constexpr int kBitsPre = 4;
// kLists: several ranks (owner lists) -- the one-rank variant compiles none of
// their code (its registers).
template <int kItems, bool kLists>
__global__ __launch_bounds__(kBlock) void td_sparse_bits_kernel(TdSparseArgs a) {
  __shared__ long long s_incl[kBlock];  // per wave: the step's inclusive degree prefixes
  __shared__ eid_t s_rs[kBlock];        // ... and row starts
  __shared__ int s_last;
  const bool dx = kLists && a.lists && a.direct.active;
  if (!chain_live(*a.ctrl, 'T', a.max_mf)) {
    if (dx && blockIdx.x == 0) {
      direct_publish(a.direct, a.lists, a.list_stride, false);
      if (a.fuse_apply) sparse_apply<kBlock, false>(a, 0, 1);  // (a collective: as td_sparse)
    }
    return;
  }
  stamp_level_start(a.ctrl);
  const int t = threadIdx.x;
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(static_cast<int>(t >> 6));  // (wave-uniform)
  long long* w_incl = s_incl + wv * kWave;
  eid_t* w_rs = s_rs + wv * kWave;
  const int64_t nunits = (a.words + kUnitWords - 1) / kUnitWords;
  const int64_t wstride = static_cast<int64_t>(gridDim.x) * kUnitsPerBlock;
  const eid_t* __restrict__ ro = a.g.row_off;
  const vid_t* __restrict__ col = a.g.col;
  const uint64_t lo = static_cast<uint64_t>(a.g.lo), rows = static_cast<uint64_t>(a.g.rows);
  for (int64_t u0 = static_cast<int64_t>(blockIdx.x) * kUnitsPerBlock + wv; u0 < nunits; u0 += kBitsPre * wstride) {
    word_t fw[kBitsPre];
#pragma unroll
    for (int p = 0; p < kBitsPre; ++p) {
      const int64_t w = (u0 + p * wstride) * kUnitWords + lane;
      fw[p] = u0 + p * wstride < nunits && w < a.words ? a.frontier_in[w] : 0ull;
    }
    // the frontier vertices of the wave's kBitsPre units, numbered unit after
    // unit, 64 per step whatever unit they sit in (a tail level has about one
    // per unit: one step's chain of round trips instead of one per unit)
    int fincl[kBitsPre], ubase[kBitsPre + 1];
    ubase[0] = 0;
#pragma unroll
    for (int p = 0; p < kBitsPre; ++p) {
      if (fw[p]) a.frontier_in[(u0 + p * wstride) * kUnitWords + lane] = 0ull;
      fincl[p] = static_cast<int>(wave_incl_scan_u32(static_cast<unsigned>(__popcll(fw[p]))));
      ubase[p + 1] = ubase[p] + __builtin_amdgcn_readlane(fincl[p], kWave - 1);
    }
    const int ftotal = ubase[kBitsPre];
    for (int base = 0; base < ftotal; base += kWave) {
      const int idx = base + lane;
      int64_t r = -1;
#pragma unroll
      for (int p = 0; p < kBitsPre; ++p) {
        if (ubase[p + 1] == ubase[p]) continue;  // (uniform)
        const int vpos = wave_set_position(fw[p], fincl[p], idx - ubase[p]);
        if (idx >= ubase[p] && idx < ubase[p + 1]) r = (u0 + p * wstride) * kUnitWords * 64 + vpos;
      }
      eid_t rs = 0, d = 0;
      if (r >= 0) {
        rs = ro[r];
        d = ro[r + 1] - rs;
      }
      const long long incl = wave_incl_scan(static_cast<long long>(d));
      const long long E = readlane_i64(incl, kWave - 1);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      w_incl[lane] = incl;
      w_rs[lane] = rs;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      for (long long e0 = 0; e0 < E; e0 += kItems * kWave) {
        // (A) all items' claims in flight together: col, visited, fetch-or
        vid_t v[kItems];
        word_t seen[kItems];
#pragma unroll
        for (int k = 0; k < kItems; ++k) {
          const long long e = e0 + k * kWave + lane;
          v[k] = 0u;
          if (e < E) {
            int j = 0;  // the first lane whose inclusive prefix passes e
#pragma unroll
            for (int step = kWave / 2; step >= 1; step >>= 1)
              if (w_incl[j + step - 1] <= e) j += step;
            const long long ex = j > 0 ? w_incl[j - 1] : 0;
            v[k] = col[w_rs[j] + (e - ex)];
          }
        }
#pragma unroll
        for (int k = 0; k < kItems; ++k) seen[k] = e0 + k * kWave + lane < E ? a.visited[v[k] >> 6] : ~0ull;
        unsigned claimed = 0;
#pragma unroll
        for (int k = 0; k < kItems; ++k) {
          const word_t bit = 1ull << (v[k] & 63);
          if (!(seen[k] & bit) && !(atomicOr(a.visited + (v[k] >> 6), bit) & bit)) claimed |= 1u << k;
        }
        if (kLists && a.lists) {
          unsigned remote = 0;
#pragma unroll
          for (int k = 0; k < kItems; ++k)
            if (((claimed >> k) & 1u) && static_cast<uint64_t>(v[k]) - lo >= rows) remote |= 1u << k;
          claimed &= ~remote;
          // (one count atomic per wave and owner for all its items)
          if (__ballot(remote != 0))
            owner_list_append_items<kItems>(a.lists, a.list_stride, a.part, v, remote, dx ? a.direct.table : nullptr);
        }
        // (B) finish the wave's claimed vertices
        sparse_settle<kItems>(a, v, claimed);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();  // (the next step overwrites w_incl / w_rs)
    }
  }
  // every wave's stores and atomics drained, then the ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    s_last = group_ticket_last(a.group_ticket, a.ticket) ? 1 : 0;
    if (s_last) last_arriver_acquire();
  }
  __syncthreads();
  if (!s_last) return;
  if (kLists && a.lists) {
    // several ranks: td_sparse_apply finishes the level (a direct exchange:
    // the counts and flags published here)
    if (t == 0) *a.ticket = 0u;
    if (dx) direct_publish(a.direct, a.lists, a.list_stride, true);
    // a tiny level (fuse_apply): the owner side and the level end here too
    if (dx && a.fuse_apply) sparse_apply<kBlock, false>(a, 0, 1, true);
    return;
  }
  if (t != 0) return;
  long long cnt = 0, deg = 0;
  sparse_totals(a, cnt, deg);
  LevelCtrl c = *a.ctrl;
  finish_level(a.ctrl, c, cnt, deg, false, a.rec, a.mailbox, a.level_index);
}


// ---------------------------------------------------------------------------
// Binned top-down level (BinArgs).  Count and fill passes walk the same edge
// blocks per workgroup (b = blockIdx.x, += gridDim.x) with the td_expand owner
// map; a workgroup's targets of bin k land at bin_start[k] + wg_off[k * grid +
// g] plus an LDS slot.  1024-thread workgroups, 2 edges per thread per block.
constexpr int kBinThreads = 1024;
constexpr int kAggRounds = 4;

// slot = atomicAdd(&cnt[key], 1) for every active lane, with the lanes that
// share a key served by one LDS atomic (rows in id order put runs of targets
// in one bin, and 64 same-address LDS atomics serialise): up to kAggRounds
// distinct keys per wave aggregated, the rest per lane.  Wave-uniform call.
__device__ __forceinline__ unsigned lds_slot_add(unsigned* cnt, int key, bool active) {
  const int lane = lane_id();
  unsigned long long pending = __ballot(active);
  unsigned slot = 0;
#pragma unroll
  for (int r = 0; r < kAggRounds; ++r) {
    if (!pending) break;
    const int leader = __ffsll(static_cast<long long>(pending)) - 1;
    const int k = __shfl(key, leader, kWave);
    const unsigned long long m = __ballot(active && key == k) & pending;
    unsigned base = 0;
    if (lane == leader) base = atomicAdd(&cnt[k], static_cast<unsigned>(__popcll(m)));
    base = __shfl(base, leader, kWave);
    if ((m >> lane) & 1ull) slot = base + mask_rank(m);
    pending &= ~m;
  }
  if ((pending >> lane) & 1ull) slot = atomicAdd(&cnt[key], 1u);
  return slot;
}

template <bool kFill>
__global__ __launch_bounds__(kTdThreads) void bin_pass_kernel(BinArgs a) {
  constexpr int kItems = kTdEdgesPerBlock / kTdThreads;
  __shared__ int32_t s_owner[kTdEdgesPerBlock];
  __shared__ long long s_base[kTdEdgesPerBlock + 1];
  __shared__ int32_t s_wmax[kTdThreads / kWave];
  __shared__ unsigned s_cnt[kBinMaxBins];
  __shared__ long long s_start[kFill ? kBinMaxBins : 1];
  if (!chain_live(*a.ctrl, 'T', 0)) return;
  const long long q = a.dev_stats[0], m = a.dev_stats[1];
  const int t = threadIdx.x;
  if (!kFill && a.clear_qv) {
    stamp_level_start(a.ctrl);  // first kernel of the level (no compaction ran)
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kTdThreads + t; i < q;
         i += static_cast<int64_t>(gridDim.x) * kTdThreads)
      a.clear_frontier[a.clear_qv[i] >> 6] = 0ull;
  }
  for (int k = t; k < a.nbins; k += kTdThreads) s_cnt[k] = 0;
  if constexpr (kFill) {
    // bin starts: exclusive scan of the bin totals (<= kBinMaxBins), serial
    // per wave-chunk then across the 4 waves
    __shared__ long long s_part[kTdThreads / kWave];
    constexpr int kPer = kBinMaxBins / kTdThreads;
    long long c[kPer], sum = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int b = t * kPer + k;
      c[k] = b < a.nbins ? a.bin_total[b] : 0;
      sum += c[k];
    }
    const long long incl = wave_incl_scan(sum);
    if (lane_id() == kWave - 1) s_part[t >> 6] = incl;
    __syncthreads();
    long long off = incl - sum;
    for (int w = 0; w < (t >> 6); ++w) off += s_part[w];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int b = t * kPer + k;
      if (b < a.nbins) s_start[b] = off + a.cnt[static_cast<int64_t>(b) * a.grid + blockIdx.x];
      off += c[k];
    }
  }
  // (td_block_owner_map starts with a barrier)
  const long long nblocks = (m + kTdEdgesPerBlock - 1) / kTdEdgesPerBlock;
  const vid_t* __restrict__ col = a.g.col;
  for (long long b = blockIdx.x; b < nblocks; b += gridDim.x) {
    const long long e0 = b * kTdEdgesPerBlock;
    const int cnt = td_block_owner_map<kTdThreads>(a.qscan, a.qbase, a.blk_vstart, b, nblocks, q, m, s_owner,
                                                   s_base, s_wmax);
    vid_t v[kItems];
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int idx = k * kTdThreads + t;
      v[k] = idx < cnt ? col[e0 + idx + s_base[s_owner[idx]]] : 0u;
    }
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const bool act = k * kTdThreads + t < cnt;
      const int bin = static_cast<int>(v[k] >> a.shift);
      DBFS_DCHECK(!act || bin < a.nbins, 8, v[k]);
      const unsigned slot = lds_slot_add(s_cnt, bin, act);
      if constexpr (kFill) {
        if (act) a.buf[s_start[bin] + slot] = v[k];
      }
    }
  }
  if constexpr (!kFill) {
    __syncthreads();
    for (int k = t; k < a.nbins; k += kTdThreads) a.cnt[static_cast<int64_t>(k) * a.grid + blockIdx.x] = s_cnt[k];
  }
}

// One workgroup per bin: its row of workgroup counts made exclusive, the
// bin's total.
__global__ __launch_bounds__(kTdThreads) void bin_scan_kernel(BinArgs a) {
  __shared__ long long s_part[kTdThreads / kWave];
  if (!chain_live(*a.ctrl, 'T', 0)) return;
  uint32_t* row = a.cnt + static_cast<int64_t>(blockIdx.x) * a.grid;
  const int t = threadIdx.x;
  const int per = (a.grid + kTdThreads - 1) / kTdThreads;
  long long sum = 0;
  for (int k = 0; k < per; ++k) {
    const int g = t * per + k;
    if (g < a.grid) sum += row[g];
  }
  const long long incl = wave_incl_scan(sum);
  if (lane_id() == kWave - 1) s_part[t >> 6] = incl;
  __syncthreads();
  long long off = incl - sum, total = 0;
  for (int w = 0; w < kTdThreads / kWave; ++w) {
    if (w < (t >> 6)) off += s_part[w];
    total += s_part[w];
  }
  for (int k = 0; k < per; ++k) {
    const int g = t * per + k;
    if (g < a.grid) {
      const uint32_t c = row[g];
      row[g] = static_cast<uint32_t>(off);  // (a bin holds < 2^32 targets per level)
      off += c;
    }
  }
  if (t == 0) a.bin_total[blockIdx.x] = total;
}

// One workgroup per bin: the bin's visited slice in LDS, claims of the bin's
// targets with LDS atomics (lanes on one word aggregated; kApplyItems loads
// in flight per thread), then the bin's frontier / visited words.
constexpr int kApplyItems = 8;

__global__ __launch_bounds__(kBinThreads) void bin_apply_kernel(BinArgs a) {
  constexpr int kMaxWords = (1 << kBinMaxShift) / kWordBits;
  __shared__ word_t s_vis[kMaxWords];
  __shared__ word_t s_new[kMaxWords];
  __shared__ long long s_part[kBinThreads / kWave];
  if (!chain_live(*a.ctrl, 'T', 0)) return;
  const int t = threadIdx.x;
  const int lane = lane_id();
  const int64_t bin = blockIdx.x;
  const int64_t span_w = (int64_t(1) << a.shift) / kWordBits;
  const int64_t w0 = bin * span_w;
  const int nw = static_cast<int>(min<int64_t>(span_w, a.words - w0));
  if (nw <= 0) return;
  // this bin's start: the totals of the bins before it
  long long before = 0;
  for (int64_t b = t; b < bin; b += kBinThreads) before += a.bin_total[b];
  before = wave_sum(before);
  if (lane == 0) s_part[t >> 6] = before;
  for (int w = t; w < nw; w += kBinThreads) {
    s_vis[w] = a.visited[w0 + w];
    s_new[w] = 0ull;
  }
  __syncthreads();
  long long b0 = 0;
  for (int w = 0; w < kBinThreads / kWave; ++w) b0 += s_part[w];
  const long long b1 = b0 + a.bin_total[bin];
  const int64_t vlo = w0 * kWordBits;
  for (long long i0 = b0; i0 < b1; i0 += static_cast<long long>(kBinThreads) * kApplyItems) {
    vid_t v[kApplyItems];
#pragma unroll
    for (int k = 0; k < kApplyItems; ++k) {
      const long long j = i0 + static_cast<long long>(k) * kBinThreads + t;
      v[k] = j < b1 ? a.buf[j] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int k = 0; k < kApplyItems; ++k) {
      int w = 0;
      word_t bit = 0;
      if (v[k] != 0xFFFFFFFFu) {
        const int64_t l = static_cast<int64_t>(v[k]) - vlo;
        w = static_cast<int>(l >> 6);
        bit = 1ull << (l & 63);
        if (s_vis[w] & bit) bit = 0;  // visited: nothing to claim
      }
      unsigned long long pending = __ballot(bit != 0);
#pragma unroll
      for (int r = 0; r < kAggRounds; ++r) {
        if (!pending) break;
        const int leader = __ffsll(static_cast<long long>(pending)) - 1;
        const int kw = __shfl(w, leader, kWave);
        const unsigned long long msk = __ballot(bit != 0 && w == kw) & pending;
        if (__popcll(msk) == 1) break;  // no sharing left worth a reduction
        word_t mine = ((msk >> lane) & 1ull) ? bit : 0ull;
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) mine |= __shfl_xor(mine, off, kWave);
        if (lane == leader) atomicOr(&s_new[kw], mine);
        pending &= ~msk;
      }
      if ((pending >> lane) & 1ull) atomicOr(&s_new[w], bit);
    }
  }
  __syncthreads();
  for (int w = t; w < nw; w += kBinThreads) {
    const word_t nb = s_new[w];
    a.frontier[w0 + w] = nb;
    if (nb) a.visited[w0 + w] = s_vis[w] | nb;
  }
}

// out bit h = visited bit of td_hub_vertex[h]: one wave per hub word.
__global__ __launch_bounds__(kBlock) void hub_visited_kernel(HubVisitedArgs a) {
  if (a.ctrl && (!chain_live(*a.ctrl, 'T', 0) || a.ctrl->m_f < a.min_edges ||
                 static_cast<double>(a.ctrl->vis_deg) < a.vis_frac * a.ctrl->total_directed))
    return;
  const int64_t w = static_cast<int64_t>(blockIdx.x) * (kBlock / kWave) + (threadIdx.x >> 6);
  const int64_t h = w * kWave + lane_id();
  const bool bit = h < a.g.td_nhubs && test_bit(a.visited, a.g.td_hub_vertex[h]);
  const word_t m = __ballot(bit);
  if (lane_id() == 0 && w * kWave < a.g.td_nhubs) a.out[w] = m;
}

// UnvisArgs: a workgroup builds kUnvisChunk filter words in LDS from the
// visited words of their vertex run (coalesced; one LDS atomic per unvisited
// vertex and filter word its word's run touches), then stores them -- every
// filter word written, nothing to clear between levels.
constexpr int kUnvisChunk = 64;
__global__ __launch_bounds__(kBlock) void unvis_filter_kernel(UnvisArgs a) {
  if (a.ctrl && !chain_live(*a.ctrl, 'T', a.max_mf)) return;
  __shared__ word_t s_f[kUnvisChunk];
  const int t = threadIdx.x;
  const int64_t w0 = static_cast<int64_t>(blockIdx.x) * kUnvisChunk;
  const int64_t w1 = min(w0 + kUnvisChunk, kUnvisWords);
  if (t < kUnvisChunk) s_f[t] = 0ull;
  __syncthreads();
  const uint64_t n = static_cast<uint64_t>(a.n);
  const uint64_t v0 = unvis_first(static_cast<uint64_t>(w0) * 64, a.mult);
  const uint64_t v1 = min(n, unvis_first(static_cast<uint64_t>(w1) * 64, a.mult));
  if (v0 < v1) {
    const uint64_t j1 = (v1 - 1) >> 6;
    for (uint64_t j = (v0 >> 6) + t; j <= j1; j += kBlock) {
      word_t x = ~a.visited[j];
      if (j == (v0 >> 6)) x &= ~0ull << (v0 & 63);
      if (j == j1 && (v1 & 63)) x &= (1ull << (v1 & 63)) - 1;
      int64_t cur = -1;
      word_t acc = 0;
      while (x) {
        const uint64_t v = j * 64 + static_cast<uint64_t>(__builtin_ctzll(x));
        x &= x - 1;
        const int64_t i = static_cast<int64_t>(unvis_index(v, a.mult)) - w0 * 64;
        if ((i >> 6) != cur) {
          if (cur >= 0) atomicOr(&s_f[cur], acc);
          cur = i >> 6;
          acc = 0;
        }
        acc |= 1ull << (i & 63);
      }
      if (cur >= 0) atomicOr(&s_f[cur], acc);
    }
  }
  __syncthreads();
  if (t < kWave) {
    long long c = 0;
    if (t < w1 - w0) {
      a.out[w0 + t] = s_f[t];
      c = __popcll(s_f[t]);
    }
    c = wave_sum(c);
    if (t == 0 && a.pop) a.pop[blockIdx.x] = static_cast<uint32_t>(c);
  }
}

// HubApplyArgs: 16 marks per thread (kTdMaxHubs is a multiple of 16; the
// marks past td_nhubs stay zero).
__global__ __launch_bounds__(kBlock) void hub_apply_kernel(HubApplyArgs a) {
  if (a.ctrl && !chain_live(*a.ctrl, 'T', a.max_mf)) return;
  const uint8_t lv = static_cast<uint8_t>(a.narrow_base + a.new_level);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock * 16;
  for (int64_t i = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) * 16; i < a.g.td_nhubs; i += stride) {
    uint4* p = reinterpret_cast<uint4*>(a.mark + i);
    const uint4 m = *p;
    if ((m.x | m.y | m.z | m.w) == 0u) continue;
    const unsigned w[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if ((w[j >> 2] >> (8 * (j & 3))) & 0xFFu) {
        DBFS_DCHECK(i + j < a.g.td_nhubs, 9, i + j);
        const vid_t v = a.g.td_hub_vertex[i + j];
        a.level8[v] = lv;
      }
    *p = make_uint4(0u, 0u, 0u, 0u);
  }
}

}  // namespace

#ifdef DBFS_TD_STATS
static void td_stats_report(hipStream_t st) {
  unsigned long long h[4] = {0};
  (void)hipStreamSynchronize(st);
  (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_td_stats), sizeof(h));
  const unsigned long long z[4] = {0};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_td_stats), z, sizeof(z));
  if (h[0])
    std::fprintf(stderr, "[td-stats] live %llu hub-unvisited %llu direct-stores %llu filter-wgs %llu\n", h[0], h[1],
                 h[2], h[3]);
}
#endif

// Device-loop grid of a td_expand variant: at most the workgroups resident at
// once (a.grid is a cap).  A grid past residency runs a partial second wave of
// workgroups that start when the first ones finish their strided share: with
// 2048 workgroups and six resident per CU, RMAT-22 top-down 70 against 83
// GTEPS at 1536.
template <TdOut kOut, bool kFilter, bool kBase32, int kThreads = kTdThreads, bool kUnvis = false>
unsigned td_resident_grid(int64_t cap) {
  static const int per_cu = [] {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, td_expand_kernel<kOut, kThreads, kFilter, kBase32, kUnvis>,
                                                     kThreads, 0) != hipSuccess || n <= 0)
      n = 1;
    return n;
  }();
  return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(cap, static_cast<int64_t>(per_cu) * device_cus())));
}

void td_expand(const TdArgs& a, hipStream_t st) {
#ifdef DBFS_TD_STATS
  struct Report {
    hipStream_t st;
    ~Report() { td_stats_report(st); }
  } report{st};
#endif
  if (a.ctrl) {
    // device loop: fixed grid, size and output mode read on the device
    if (a.grid <= 0) return;
    const bool b32 = a.g.nnz <= (int64_t(1) << 32);
    const int64_t fgrid = a.grid_filter > 0 ? a.grid_filter : a.grid;
#define LAUNCH_TD_DEV(OUT, F, B) \
  td_expand_kernel<OUT, kTdThreads, F, B><<<td_resident_grid<OUT, F, B>(F ? fgrid : a.grid), kTdThreads, 0, st>>>(a)
    if (a.unvis && !a.lists) {
      // the filter variant, then the plain one: the level runs in one of
      // them (the filter's density, read by both)
      DBFS_CHECK(a.unvis_pop, "td_expand: an unvisited filter without its chunk counts");
      if (b32)
        td_expand_kernel<TdOut::Dyn, 1024, false, true, true>
            <<<td_resident_grid<TdOut::Dyn, false, true, 1024, true>(a.grid), 1024, 0, st>>>(a);
      else
        td_expand_kernel<TdOut::Dyn, 1024, false, false, true>
            <<<td_resident_grid<TdOut::Dyn, false, false, 1024, true>(a.grid), 1024, 0, st>>>(a);
    }
    if (a.lists)
      LAUNCH_TD_DEV(TdOut::Lists, false, false);
    else if (a.td_hub_vis && b32)
      LAUNCH_TD_DEV(TdOut::Dyn, true, true);
    else if (a.td_hub_vis)
      LAUNCH_TD_DEV(TdOut::Dyn, true, false);
    else if (b32)
      LAUNCH_TD_DEV(TdOut::Dyn, false, true);
    else
      LAUNCH_TD_DEV(TdOut::Dyn, false, false);
#undef LAUNCH_TD_DEV
    return;
  }
  if (a.m <= 0 || a.q <= 0) return;
  const unsigned grid = grid_for(a.m, kTdEdgesPerBlock);
  const bool wide = static_cast<int64_t>(grid) < a.wide_below_blocks;
#define LAUNCH_TD(OUT)                                                  \
  do {                                                                       \
    if (wide)                                                                \
      td_expand_kernel<OUT, 1024><<<grid, 1024, 0, st>>>(a);                 \
    else                                                                     \
      td_expand_kernel<OUT, kTdThreads><<<grid, kTdThreads, 0, st>>>(a);     \
  } while (0)
  if (a.lists)
    LAUNCH_TD(TdOut::Lists);
  else if (a.next_bytes)
    LAUNCH_TD(TdOut::Bytes);
  else
    LAUNCH_TD(TdOut::Bits);
#undef LAUNCH_TD
}

void td_binned(const BinArgs& a, hipStream_t st) {
  if (a.nbins <= 0 || a.grid <= 0 || a.nbins > kBinMaxBins) return;
  bin_pass_kernel<false><<<static_cast<unsigned>(a.grid), kTdThreads, 0, st>>>(a);
  bin_scan_kernel<<<static_cast<unsigned>(a.nbins), kTdThreads, 0, st>>>(a);
  bin_pass_kernel<true><<<static_cast<unsigned>(a.grid), kTdThreads, 0, st>>>(a);
  bin_apply_kernel<<<static_cast<unsigned>(a.nbins), kBinThreads, 0, st>>>(a);
}

void td_sparse(const TdSparseArgs& a, hipStream_t st) {
  if (a.from_bits) {
    // a wave per unit up to 4096 workgroups' worth, else kBitsPre units per
    // wave (RMAT-26, one rank: 1024 workgroups, 16 groups on the ticket)
    const int64_t nunits = (a.words + kUnitWords - 1) / kUnitWords;
    DBFS_CHECK(a.group_ticket, "td_sparse from a bitmap needs the group tickets");
    // (an empty shard still runs one workgroup: the level's finish)
    const unsigned grid = grid_for(nunits, kUnitsPerBlock, std::min<int64_t>(kMaxFusedGrid, 1024));
    if (a.lists) td_sparse_bits_kernel<4, true><<<grid, kBlock, 0, st>>>(a);
    else td_sparse_bits_kernel<4, false><<<grid, kBlock, 0, st>>>(a);
    return;
  }
  // 1024-thread workgroups, two edges per thread per block: a sparse level's
  // few blocks get four times the waves (measured against 256 threads / 8
  // edges: RMAT-26 1479 / 1469 -> 1502 / 1481 GTEPS, level 0 9.8 -> 6.7 us;
  // RMAT-22 top-down only 90.5 / 90.8 -> 91.8 / 92.2)
  const unsigned grid = static_cast<unsigned>(a.grid);
  if (a.lists) td_sparse_kernel<kTdSparseThreads, true><<<grid, kTdSparseThreads, 0, st>>>(a);
  else td_sparse_kernel<kTdSparseThreads><<<grid, kTdSparseThreads, 0, st>>>(a);
}

void direct_selftest(const DirectExchange& lists, const DirectExchange& end, int round, unsigned* err,
                     unsigned* ticket, hipStream_t st) {
  direct_selftest_kernel<<<kSelftestGroups, 256, 0, st>>>(lists, end, round, err, ticket);
}

namespace {
__device__ __forceinline__ uint64_t frontier_pat(int r, int64_t i, int round) {
  return (static_cast<uint64_t>(r + 1) << 48) ^ (static_cast<uint64_t>(i) * 0x9E3779B97F4A7C15ull) ^
         static_cast<uint64_t>(round);
}
__global__ __launch_bounds__(256) void frontier_selftest_kernel(const FrontierTable* t, int rank, int nranks,
                                                                int64_t words, int round, int phase, unsigned* err) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  unsigned bad = 0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < words; i += stride) {
    if (phase == 0) {
      push_frontier_word(t, rank, nranks, i, frontier_pat(rank, i, round));
      continue;
    }
    for (int p = 0; p < nranks; ++p)
      if (p != rank && sys_load_u64(t->src[p] + i) != frontier_pat(p, i, round)) ++bad;
  }
  if (bad) atomicAdd(err, bad);
}
}  // namespace

void frontier_selftest(const FrontierTable* t, int rank, int nranks, int64_t words, int round, int phase,
                       unsigned* err, hipStream_t st) {
  frontier_selftest_kernel<<<grid_for(words, 256, 64), 256, 0, st>>>(t, rank, nranks, words, round, phase, err);
}

void td_sparse_apply(const TdSparseArgs& a, hipStream_t st) {
  // (1024 threads, two ids each: as td_sparse)
  const unsigned grid = static_cast<unsigned>(std::max<int64_t>(1, a.grid));
  td_sparse_apply_kernel<kTdSparseThreads><<<grid, kTdSparseThreads, 0, st>>>(a);
}

void direct_prewait(const DirectExchange& x, hipStream_t st) {
  if (x.active) direct_prewait_kernel<<<1, kWave, 0, st>>>(x);
}

void hub_visited(const HubVisitedArgs& a, hipStream_t st) {
  if (a.g.td_nhubs <= 0) return;
  hub_visited_kernel<<<grid_for((a.g.td_nhubs + kWave - 1) / kWave, kBlock / kWave), kBlock, 0, st>>>(a);
}

void unvis_filter(const UnvisArgs& a, hipStream_t st) {
  DBFS_CHECK(a.mult == unvis_mult(a.n), "unvis_filter: multiplier of another vertex count");
  static_assert(kUnvisChunk == kWave, "a chunk's words are one wave's");
  unvis_filter_kernel<<<static_cast<unsigned>(kUnvisChunks), kBlock, 0, st>>>(a);
}

void hub_apply(const HubApplyArgs& a, hipStream_t st) {
  if (a.g.td_nhubs <= 0 || a.g.td_nhubs > kTdMaxHubs) return;  // (select_hubs: at most kTdMaxHubs)
  hub_apply_kernel<<<grid_for((a.g.td_nhubs + 15) / 16, kBlock), kBlock, 0, st>>>(a);
}

unsigned long long take_check_td() { return take_check_local(); }

}  // namespace kern
}  // namespace dbfs
