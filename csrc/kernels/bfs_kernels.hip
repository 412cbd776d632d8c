// gfx950 level bookkeeping of the BFS engine: per-run initialisation, the
// frontier update (visited-bitmap update + level write), the multi-block unit
// scan, frontier compaction (wave prefix sums) and the small utility kernels;
// the top-down kernels are in td_kernels.hip, the bottom-up ones in
// bu_kernels.hip (shared device helpers: kernel_common.hpp).
//
// Reference counterpart: the single live kernel queueBfs (bfs.cu:134-165) --
// thread-per-frontier-vertex serial neighbour loop, atomicMin claim on an int
// distance array, and one global atomicAdd per discovered vertex on a single
// managed counter per owner bucket.  On CDNA4 that design is bound by (a) load
// imbalance of power-law degrees inside a 64-lane wave and (b) a contended
// device-scope counter (~88 returning atomics/us per word, MI355X_MICROARCH
// "dequeue" row).  Here:
//   * discoveries are bits (atomicOr on a 64-bit word, no counter at all);
//   * one wave64 owns one bitmap word (64 vertices): ballots build words,
//     mbcnt gives slots, wave prefix sums give edge offsets -- no atomics;
//   * per-unit (16 words) counts are scanned by a multi-block scan that hands
//     its chunk totals to the last-arriving workgroup (agent-scope release /
//     acquire, cdna_hip_programming.md Guideline 16);
//   * top-down work is split into equal edge ranges per workgroup
//     (kTdEdgesPerBlock) with an LDS owner map, so hubs and leaves cost the same
//     per edge and col[] is read fully coalesced;
//   * bottom-up scans each owned unvisited vertex's neighbours for a frontier
//     bit, per lane for the first few, then wave-cooperatively (64 neighbours per
//     step, ballot early exit) for the long ones, and writes the new frontier,
//     visited word, levels and unit stats itself (no separate update pass).
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

// Zero fill, 16-B stores, grid-stride (one store per thread on the usual
// grid): an 8 MiB bitmap in ~2 us where the runtime's fill kernel takes ~5.
__global__ __launch_bounds__(kBlock) void zero16_kernel(uint4* __restrict__ p, int64_t n16) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n16; i += stride)
    p[i] = make_uint4(0u, 0u, 0u, 0u);
}

__global__ void ctrl_init_kernel(LevelCtrl* c, LevelCtrl init) {
  if (threadIdx.x == 0) *c = init;
}

__global__ void set_bit_kernel(word_t* bm, int64_t bit) {
  if (threadIdx.x == 0) bm[bit >> 6] |= 1ull << (bit & 63);
}

// Fused per-run initialisation (InitRunArgs).  Grid-stride over the level
// array (16-B stores), the global visited words and the owned frontier words;
// the element holding the source is written with its seeded value by the same
// thread that fills it, so no ordering between threads is needed.  Thread 0 of
// block 0 writes the seed's totals / work-list offsets / device-loop state.
__global__ __launch_bounds__(kBlock) void init_run_kernel(InitRunArgs a) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  const int64_t rows = a.g.rows;
  const int64_t src = a.src_local;
  if (a.level8 && a.level8_filled) {
    // already reads unreached for this run (prefilled, or an earlier epoch's
    // bytes): the source's byte only
    if (src >= 0 && t0 == 0) a.level8[src] = a.narrow_base;
  } else if (a.level8) {
    // narrow levels: rows / 16 uint4 stores of 0xFF (+ tail), the source's byte after
    const int64_t n16 = (reinterpret_cast<uintptr_t>(a.level8) & 15u) == 0 ? rows / 16 : 0;
    uint4* l16 = reinterpret_cast<uint4*>(a.level8);
    for (int64_t i = t0; i < n16; i += stride) {
      uint4 v = make_uint4(~0u, ~0u, ~0u, ~0u);
      if (src >= 0 && (src >> 4) == i) {
        const unsigned clear = ~(0xFFu << (8 * (src & 3)));
        const unsigned set = static_cast<unsigned>(a.narrow_base) << (8 * (src & 3));
        const int word = static_cast<int>((src >> 2) & 3);
        if (word == 0) v.x = (v.x & clear) | set;
        else if (word == 1) v.y = (v.y & clear) | set;
        else if (word == 2) v.z = (v.z & clear) | set;
        else v.w = (v.w & clear) | set;
      }
      l16[i] = v;
    }
    for (int64_t i = n16 * 16 + t0; i < rows; i += stride) a.level8[i] = i == src ? a.narrow_base : kNarrowUnreached;
  } else {
    // level: rows / 4 int4 stores (+ tail)
    const int64_t n4 = (reinterpret_cast<uintptr_t>(a.level) & 15u) == 0 ? rows / 4 : 0;
    int4* l4 = reinterpret_cast<int4*>(a.level);
    for (int64_t i = t0; i < n4; i += stride) {
      int4 v = make_int4(kUnreached, kUnreached, kUnreached, kUnreached);
      if (src >= 0 && (src >> 2) == i) {
        if ((src & 3) == 0) v.x = 0;
        else if ((src & 3) == 1) v.y = 0;
        else if ((src & 3) == 2) v.z = 0;
        else v.w = 0;
      }
      l4[i] = v;
    }
    for (int64_t i = n4 * 4 + t0; i < rows; i += stride) a.level[i] = i == src ? 0 : kUnreached;
  }
  // (the source's visited bit: in every rank's replicated bitmap when the
  // global id is known -- a seed without collective -- else on its owner)
  const int64_t sw = a.src_global >= 0 ? (a.src_global >> 6) : src >= 0 ? a.vis_word_base + (src >> 6) : -1;
  const word_t sbit = a.src_global >= 0 ? (1ull << (a.src_global & 63)) : src >= 0 ? (1ull << (src & 63)) : 0ull;
  for (int64_t w = t0; w < a.gwords; w += stride) a.visited[w] = a.zdeg[w] | (w == sw ? sbit : 0ull);
  if (a.frontier_global) {
    // a bottom-up first level reads the whole seed frontier: written here
    for (int64_t w = t0; w < a.gwords; w += stride) a.frontier_global[w] = w == sw ? sbit : 0ull;
  } else if (a.frontier_clean) {
    if (src >= 0 && t0 == 0) a.frontier[src >> 6] = 1ull << (src & 63);
  } else {
    const word_t obit = src >= 0 ? (1ull << (src & 63)) : 0ull;
    for (int64_t w = t0; w < a.words; w += stride) a.frontier[w] = (src >= 0 && w == (src >> 6)) ? obit : 0ull;
  }
  if (a.frontier_clear && !a.frontier_clean)
    for (int64_t w = t0; w < a.words; w += stride) a.frontier_clear[w] = 0ull;
  // the seed's work-list entry: edge blocks [0, ceil(d / EPB)) all start in it
  if (a.blk_vstart && src >= 0) {
    const eid_t d = a.g.row_off[src + 1] - a.g.row_off[src];
    for (int64_t b = t0; b * kTdEdgesPerBlock < d; b += stride) a.blk_vstart[b] = 0;
  }
  if (t0 != 0) return;
  int64_t cnt = 0, deg = 0;
  if (src >= 0) {
    const eid_t d = a.g.row_off[src + 1] - a.g.row_off[src];
    if (d > 0) {
      cnt = 1;
      deg = d;
    }
    const int64_t unit = (src >> 6) / kUnitWords;
    a.unit_cnt[unit] = 0;
    a.unit_deg[unit] = 0;
    a.part_cnt[unit / kScanChunk] = 0;
    a.part_deg[unit / kScanChunk] = 0;
  }
  a.stats[0] = a.stats[2] = cnt;
  a.stats[1] = a.stats[3] = deg;
  a.qscan[cnt] = deg;
  if (cnt && a.qbase) {
    a.qscan[0] = 0;
    a.qbase[0] = a.g.row_off[src];
    a.qv[0] = static_cast<vid_t>(src);
  }
  if (a.ctrl) {
    // the seed's global totals: this rank's own, or (several ranks) from the
    // replicated degree of the source
    int64_t gc = cnt, gd = deg;
    if (a.deg_all) {
      gd = a.deg_all[a.src_global];
      gc = gd > 0 ? 1 : 0;
      a.stats[2] = gc;
      a.stats[3] = gd;
    }
    LevelCtrl c = a.ctrl_init;
    finish_level(a.ctrl, c, gc, gd, true, nullptr, a.mailbox, -1);
  }
}

__global__ __launch_bounds__(kBlock) void level_finish_kernel(LevelFinishArgs a) { level_finish_block<kBlock>(a); }

// Level totals -> host-mapped mailbox: values first (system scope), then the
// sequence number with release semantics, so a host that observes `seq` reads
// the values of that level.
__global__ void publish_stats_kernel(const int64_t* __restrict__ stats, StatsMailbox* mb, int64_t seq) {
  if (threadIdx.x != 0) return;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(&mb->v[k]), static_cast<unsigned long long>(stats[k]),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(&mb->seq), static_cast<unsigned long long>(seq),
                     __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------
// Frontier update: a wave owns 16 consecutive words.  Lanes 0..15 update the
// bitmap words (one coalesced 128-B access per array); then, for every
// non-zero new word, the wave switches to lane-per-vertex so the level stores
// and row_off loads of that word are one coalesced access each.
//
// Geometry: one wave per 64-word unit (lane l owns word l of the unit), 4
// units per workgroup -- a sparse level then costs ~4K workgroups of dispatch
// instead of 16K, and the unit statistics need no cross-wave reduction.

// 64 candidate bytes (0/1, 64-byte aligned) -> one bitmap word; the bytes are
// cleared when any is set.  Four 16-B loads / stores per lane.
__device__ __forceinline__ word_t gather_byte_bits(uint8_t* p) {
  uint4* q = reinterpret_cast<uint4*>(p);
  word_t bits = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint4 x = q[k];
    const unsigned v[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if ((v[j] >> (8 * b)) & 0xFFu) bits |= 1ull << (k * 16 + j * 4 + b);
    }
  }
  if (bits) {
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = make_uint4(0u, 0u, 0u, 0u);
  }
  return bits;
}

// 64 level bytes (64-byte aligned) -> bit b set when byte b == lvl.
__device__ __forceinline__ word_t gather_level_bits(const uint8_t* p, uint8_t lvl) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  word_t bits = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint4 x = q[k];
    const unsigned v[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if (((v[j] >> (8 * b)) & 0xFFu) == lvl) bits |= 1ull << (k * 16 + j * 4 + b);
    }
  }
  return bits;
}

// A unit's statistics; write-through when the fused finish's last workgroup
// scans them (UpdateArgs::fold_scan: read there with agent-scope loads).
__device__ __forceinline__ void store_unit_stats(const UpdateArgs& a, int64_t unit, long long c, long long d) {
  if (a.fold_scan) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.unit_cnt + unit), static_cast<unsigned long long>(c),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.unit_deg + unit), static_cast<unsigned long long>(d),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    a.unit_cnt[unit] = c;
    a.unit_deg[unit] = d;
  }
}

// The fused finish's unit prefixes (UpdateArgs::fold_scan; every thread of the
// last workgroup of kBlock threads): unit_cnt / unit_deg become the exclusive
// prefixes over all units (at most kFoldScanUnits) and the chunk prefixes
// part_cnt / part_deg zero -- what scan_units_kernel leaves for the
// compaction.  The units are spread over all kBlock threads (a run of
// ceil(nunits / kBlock) each) and a run's agent-scope loads go out kFoldRun at
// a time: each batch is one round trip to memory (the stats were stored
// write-through by other XCDs' waves), so a run of up to kFoldRun units -- 2048
// units, a 2^23-vertex shard -- costs one round trip, its values kept in
// registers for the second pass.  (The first version gave each thread a run of
// kFoldScanUnits / kBlock units, four loads in flight: on a 2048-unit shard one
// wave made 16 dependent round trips -- the P = 8 post-bottom-up update 39.4 ->
// 33.8 us, RMAT-22 top-down only +2 %, profiles/r5_fold_scan_ab.txt.)
__device__ __forceinline__ long long agent_load_i64(const int64_t* p) {
  return static_cast<long long>(
      __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
constexpr int kFoldRun = 8;
__device__ __forceinline__ void fold_unit_scan(const ScanArgs& a) {
  __shared__ long long s_fc[kBlock / kWave], s_fd[kBlock / kWave];
  const int t = threadIdx.x, lane = lane_id(), wv = t >> 6;
  const int64_t n = a.nunits;
  const int64_t per = (n + kBlock - 1) / kBlock;
  const int64_t u0 = min(static_cast<int64_t>(t) * per, n);
  const int64_t u1 = min(u0 + per, n);
  long long c[kFoldRun], d[kFoldRun];
  long long sc = 0, sd = 0;
  for (int64_t b = u0; b < u1; b += kFoldRun) {
#pragma unroll
    for (int k = 0; k < kFoldRun; ++k) {
      const bool in = b + k < u1;
      c[k] = in ? agent_load_i64(a.unit_cnt + b + k) : 0ll;
      d[k] = in ? agent_load_i64(a.unit_deg + b + k) : 0ll;
    }
#pragma unroll
    for (int k = 0; k < kFoldRun; ++k) {
      sc += c[k];
      sd += d[k];
    }
  }
  const long long ic = wave_incl_scan(sc), id = wave_incl_scan(sd);
  __syncthreads();  // (s_fc / s_fd: the caller's earlier LDS use is done)
  if (lane == kWave - 1) {
    s_fc[wv] = ic;
    s_fd[wv] = id;
  }
  __syncthreads();
  long long oc = ic - sc, od = id - sd;
  for (int k = 0; k < wv; ++k) {
    oc += s_fc[k];
    od += s_fd[k];
  }
  for (int64_t b = u0; b < u1; b += kFoldRun) {
    if (per > kFoldRun) {
      // (a longer run: the batch again -- the registers hold the last one)
#pragma unroll
      for (int k = 0; k < kFoldRun; ++k) {
        const bool in = b + k < u1;
        c[k] = in ? agent_load_i64(a.unit_cnt + b + k) : 0ll;
        d[k] = in ? agent_load_i64(a.unit_deg + b + k) : 0ll;
      }
    }
#pragma unroll
    for (int k = 0; k < kFoldRun; ++k) {
      if (b + k < u1) {
        a.unit_cnt[b + k] = oc;
        a.unit_deg[b + k] = od;
      }
      oc += c[k];
      od += d[k];
    }
  }
  for (int64_t p = t; p * kScanChunk < a.nunits; p += kBlock) {
    a.part_cnt[p] = 0;
    a.part_deg[p] = 0;
  }
}

// One wave per 64-word unit, kUnitsPerBlock units per workgroup; with the
// fused finish a smaller grid strides over the units (fewer ticket arrivals).
// kSplit waves per unit (small graphs: 4, each over 16 of its words -- a
// graph of few units would leave most wave slots idle while each wave walks
// its unit's new vertices 64 per dependent step); `sub` = this wave's part.
// (kRanks: the several-rank extras -- pushed words, the send buffer re-zeroed
// -- compiled into a variant of their own: in every kernel they cost the
// one-rank update 2 us a level)
template <int kSplit = 1, bool kRanks = false>
__device__ __forceinline__ void update_unit(const UpdateArgs& a, int64_t unit, bool use_bytes, long long& cnt,
                                            long long& deg, int sub = 0) {
  constexpr int kWords = kUnitWords / kSplit;
  const int lane = lane_id();
  const int64_t w0 = unit * kUnitWords + sub * kWords;
  const int64_t wl = w0 + lane;
  word_t nb = 0;
  if (lane < kWords && wl < a.words) {
    word_t c = 0;
    if (use_bytes && a.level_direct) {
      c = gather_level_bits(a.level_direct + wl * 64, static_cast<uint8_t>(a.narrow_base + a.new_level));
    } else if (use_bytes) {
      c = gather_byte_bits(a.cand_bytes + wl * 64);
    } else {
      for (int r = 0; r < a.nchunks; ++r) c |= a.cand[r * a.cand_stride + wl];
    }
    const word_t vis = a.visited[wl];
    nb = a.force ? c : (c & ~vis);
    if (nb) a.visited[wl] = vis | nb;
    a.frontier[wl] = nb;
    if constexpr (kRanks) {
      if (a.push) push_frontier_word(a.push, a.push_rank, a.push_nranks, wl, nb);
      for (int p = 0; p < a.zero_slices; ++p) a.zero_next[p * a.words + wl] = 0ull;
    }
    if (a.clear_cand && c && !use_bytes) a.cand[wl] = 0;
  }
  // New vertices of the unit, 64 per step (one per lane, whatever word they
  // sit in): a sparse level has about one new vertex per word, and one word
  // per step would cost a dependent row_off round trip per new vertex.
  cnt = 0;
  deg = 0;
  const int incl = static_cast<int>(wave_incl_scan(__popcll(nb)));
  const int total = __builtin_amdgcn_readlane(incl, kWave - 1);
  const eid_t* __restrict__ ro = a.g.row_off;
  for (int base = 0; base < total; base += kWave) {
    const int idx = base + lane;
    const int pos = wave_set_position(nb, incl, idx);
    if (idx < total) {
      const int64_t v = w0 * 64 + pos;
      if (!(use_bytes && a.level_direct)) store_level(a.level, a.level8, v, a.new_level, a.narrow_base);
      const eid_t d = ro[v + 1] - ro[v];
      if (d > 0) {
        cnt += 1;
        deg += d;
      }
    }
  }
  cnt = wave_sum(cnt);
  deg = wave_sum(deg);
  if (kSplit == 1 && lane == 0) store_unit_stats(a, unit, cnt, deg);
}

// A unit per workgroup, its kSplit (= kUnitsPerBlock) waves each over a part
// (update_unit<kSplit>); the unit's statistics summed in LDS.
template <bool kRanks>
__device__ __forceinline__ void update_unit_split(const UpdateArgs& a, int64_t unit, bool use_bytes, long long& cnt,
                                                  long long& deg, long long* s_pc, long long* s_pd) {
  const int wv = static_cast<int>(threadIdx.x >> 6);
  update_unit<kUnitsPerBlock, kRanks>(a, unit, use_bytes, cnt, deg, wv);
  if (lane_id() == 0) {
    s_pc[wv] = cnt;
    s_pd[wv] = deg;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long c = 0, d = 0;
#pragma unroll
    for (int k = 0; k < kUnitsPerBlock; ++k) {
      c += s_pc[k];
      d += s_pd[k];
    }
    store_unit_stats(a, unit, c, d);
  }
  __syncthreads();  // (s_pc / s_pd reused by the next unit)
}

// kRanks: several ranks (UpdateArgs::push / zero_next / end).
template <bool kSplit, bool kRanks>
__global__ __launch_bounds__(kBlock) void update_kernel(UpdateArgs a) {
  __shared__ uint64_t s_x[kRanks ? 2 * kern::kMaxPeers : 1];  // (the folded level end's cells)
  bool use_bytes = a.cand_bytes != nullptr;
  if (a.ctrl) {
    if (!chain_live(*a.ctrl, 'T', a.max_mf)) {
      // a folded level end is a collective: it runs on a no-op chain too
      if constexpr (kRanks)
        if (a.end.active && blockIdx.x == 0)
          direct_level_end(a.end, a.scan.stats[2], a.scan.stats[3], a.scan.stats, a.fin, s_x);
      return;
    }
    use_bytes = use_bytes && a.ctrl->bytes != 0;
  }
  const int wv = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));  // (wave-uniform)
  const int64_t nunits = (a.words + kUnitWords - 1) / kUnitWords;
  __shared__ long long s_pc[kUnitsPerBlock], s_pd[kUnitsPerBlock];
  if (!a.fuse_scan) {
    long long cnt, deg;
    if constexpr (kSplit) {
      const int64_t unit = blockIdx.x;
      if (unit >= nunits) return;
      update_unit_split<kRanks>(a, unit, use_bytes, cnt, deg, s_pc, s_pd);
    } else {
      const int64_t unit = static_cast<int64_t>(blockIdx.x) * kUnitsPerBlock + wv;
      if (unit >= nunits) return;
      update_unit<1, kRanks>(a, unit, use_bytes, cnt, deg);
    }
    return;
  }
  // fused finish (as the whole-unit bottom-up kernel's): raw unit statistics,
  // the workgroup's totals in its slot of tot, a ticket; the last workgroup
  // sums the slots and finishes the level
  __shared__ long long s_c[kUnitsPerBlock], s_d[kUnitsPerBlock];
  __shared__ int s_last, s_level_last;  // (separate: waves read s_last while wave 0 decides the level)
  long long wc = 0, wd = 0;
  if constexpr (kSplit) {
    for (int64_t unit = blockIdx.x; unit < nunits; unit += gridDim.x) {
      long long cnt, deg;
      update_unit_split<kRanks>(a, unit, use_bytes, cnt, deg, s_pc, s_pd);
      wc += cnt;  // (this wave's part: the workgroup's totals are the waves' sum, as below)
      wd += deg;
    }
  } else {
    for (int64_t unit = static_cast<int64_t>(blockIdx.x) * kUnitsPerBlock + wv; unit < nunits;
         unit += static_cast<int64_t>(gridDim.x) * kUnitsPerBlock) {
      long long cnt, deg;
      update_unit<1, kRanks>(a, unit, use_bytes, cnt, deg);
      wc += cnt;
      wd += deg;
    }
  }
  if (lane_id() == 0) {
    s_c[wv] = wc;
    s_d[wv] = wd;
  }
  // (pushed words: every wave's write-through stores drained before the
  // ticket, so the level end published after it covers them; likewise the
  // unit statistics the last workgroup scans with fold_scan -- stored by
  // lane 0 of every wave, and a barrier does not wait for another wave's
  // stores)
  if constexpr (kRanks)
    if (a.push) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (a.fold_scan) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    long long c = 0, d = 0;
#pragma unroll
    for (int k = 0; k < kUnitsPerBlock; ++k) {
      c += s_c[k];
      d += s_d[k];
    }
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.tot + 2 * blockIdx.x), static_cast<unsigned long long>(c),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.tot + 2 * blockIdx.x + 1),
                       static_cast<unsigned long long>(d), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (a.group_ticket) {
      // the group's last workgroup sums the group (below), then takes the
      // level ticket
      const unsigned grp = blockIdx.x / kFusedGroup;
      const unsigned gsz = min(static_cast<unsigned>(kFusedGroup), gridDim.x - grp * kFusedGroup);
      const unsigned prev = atomicAdd(a.group_ticket + grp * kBuQueueStride, 1u);
      s_last = prev == gsz - 1;
      if (s_last) {
        atomicExch(a.group_ticket + grp * kBuQueueStride, 0u);
        last_arriver_acquire();
      }
    } else {
      const unsigned prev = atomicAdd(a.scan.ticket, 1u);
      s_last = prev == gridDim.x - 1;
      if (s_last) last_arriver_acquire();
    }
  }
  __syncthreads();
  if (!s_last) return;
  auto slot_sum = [&](const int64_t* slots, unsigned first, unsigned n, long long& c, long long& d) {
    c = 0;
    d = 0;
    for (unsigned g = threadIdx.x; g < n; g += kBlock) {
      c += static_cast<long long>(__hip_atomic_load(reinterpret_cast<const unsigned long long*>(slots + 2 * (first + g)),
                                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      d += static_cast<long long>(__hip_atomic_load(
          reinterpret_cast<const unsigned long long*>(slots + 2 * (first + g) + 1), __ATOMIC_RELAXED,
          __HIP_MEMORY_SCOPE_AGENT));
    }
  };
  long long c = 0, d = 0;
  if (a.group_ticket) {
    // group total (kFusedGroup slots: the first wave), then the level ticket
    const unsigned grp = blockIdx.x / kFusedGroup;
    const unsigned ngroups = (gridDim.x + kFusedGroup - 1) / kFusedGroup;
    if (wv == 0) {
      slot_sum(a.tot, grp * kFusedGroup, min(static_cast<unsigned>(kFusedGroup), gridDim.x - grp * kFusedGroup), c, d);
      c = wave_sum(c);
      d = wave_sum(d);
      if (lane_id() == 0) {
        int64_t* gt = a.tot + 2 * kMaxFusedGrid;
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(gt + 2 * grp), static_cast<unsigned long long>(c),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(gt + 2 * grp + 1), static_cast<unsigned long long>(d),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev = atomicAdd(a.scan.ticket, 1u);
        s_level_last = prev == ngroups - 1;
        if (s_level_last) last_arriver_acquire();
      }
    }
    __syncthreads();
    if (!s_level_last) return;
    slot_sum(a.tot + 2 * kMaxFusedGrid, 0, ngroups, c, d);
  } else {
    slot_sum(a.tot, 0, gridDim.x, c, d);
  }
  c = wave_sum(c);
  d = wave_sum(d);
  __syncthreads();  // (s_c / s_d reused)
  if (lane_id() == 0) {
    s_c[wv] = c;
    s_d[wv] = d;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long tc = 0, td = 0;
#pragma unroll
    for (int k = 0; k < kUnitsPerBlock; ++k) {
      tc += s_c[k];
      td += s_d[k];
    }
    scan_finish(a.scan, tc, td);
    s_c[0] = tc;
    s_d[0] = td;
  }
  if (a.fold_scan) fold_unit_scan(a.scan);
  if constexpr (kRanks) {
    if (a.end.active) {
      __syncthreads();
      direct_level_end(a.end, s_c[0], s_d[0], a.scan.stats, a.fin, s_x);
    }
  }
}


// Totals and finish of a level whose unit statistics stay unscanned (the
// fused bottom-up finish of kernels without the epilogue): one workgroup
// sums the units, thread 0 finishes.
__global__ __launch_bounds__(kScanChunk) void totals_finish_kernel(ScanArgs a) {
  __shared__ long long s_c[kScanChunk / kWave], s_d[kScanChunk / kWave];
  if (a.ctrl && !chain_live(*a.ctrl, a.expect_dir, a.expect_cap)) return;
  long long c = 0, d = 0;
  for (int64_t u = threadIdx.x; u < a.nunits; u += kScanChunk) {
    c += a.unit_cnt[u];
    d += a.unit_deg[u];
  }
  c = wave_sum(c);
  d = wave_sum(d);
  const int wv = threadIdx.x >> 6;
  if (lane_id() == 0) {
    s_c[wv] = c;
    s_d[wv] = d;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  long long tc = 0, td = 0;
  for (int k = 0; k < kScanChunk / kWave; ++k) {
    tc += s_c[k];
    td += s_d[k];
  }
  scan_finish(a, tc, td);
}

// ---------------------------------------------------------------------------
// Multi-block scan.  Workgroup b scans units [b*CH, (b+1)*CH) in place
// (exclusive, in-chunk) and publishes its chunk total; the last workgroup to
// arrive scans the chunk totals.  Hand-off: chunk totals stored agent-scope
// (write-through) by thread 0, `s_waitcnt vmcnt(0)`, then the ticket atomic
// (no agent release: it would write back the XCD's whole L2, microseconds on
// the level's critical path); the last arriver runs an agent acquire fence
// and reads the totals with agent-scope loads.
__global__ __launch_bounds__(kScanChunk) void scan_units_kernel(ScanArgs a) {
  __shared__ long long s_c[kScanChunk / kWave], s_d[kScanChunk / kWave];
  __shared__ int s_last;
  // uniform: no block takes a ticket
  if (a.ctrl && !chain_live(*a.ctrl, a.expect_dir, a.expect_cap)) return;
  const int t = threadIdx.x;
  const int lane = lane_id();
  const int wv = t >> 6;
  const int64_t u = static_cast<int64_t>(blockIdx.x) * kScanChunk + t;
  const long long c = u < a.nunits ? a.unit_cnt[u] : 0;
  const long long d = u < a.nunits ? a.unit_deg[u] : 0;
  const long long ic = wave_incl_scan(c), id = wave_incl_scan(d);
  if (lane == kWave - 1) {
    s_c[wv] = ic;
    s_d[wv] = id;
  }
  __syncthreads();
  long long oc = 0, od = 0, tc = 0, td = 0;
#pragma unroll
  for (int k = 0; k < kScanChunk / kWave; ++k) {
    if (k < wv) {
      oc += s_c[k];
      od += s_d[k];
    }
    tc += s_c[k];
    td += s_d[k];
  }
  if (u < a.nunits) {
    a.unit_cnt[u] = oc + ic - c;
    a.unit_deg[u] = od + id - d;
  }
  const unsigned nblk = gridDim.x;
  if (t == 0) {
    // chunk totals: agent-scope (sc1, write-through) stores
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.part_cnt + blockIdx.x),
                       static_cast<unsigned long long>(tc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.part_deg + blockIdx.x),
                       static_cast<unsigned long long>(td), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // (no agent release: the totals are the only bytes handed off, stored
    // write-through by this lane and read by agent-scope loads)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = atomicAdd(a.ticket, 1u);
    s_last = (prev == nblk - 1) ? 1 : 0;
    if (s_last) last_arriver_acquire();
  }
  __syncthreads();
  if (!s_last) return;
  // Last workgroup: exclusive scan of the chunk totals (loop for > 1024 chunks).
  long long carry_c = 0, carry_d = 0;
  for (unsigned base = 0; base < nblk; base += kScanChunk) {
    const unsigned i = base + t;
    // agent-scope loads of the other workgroups' chunk totals
    const long long pc = i < nblk ? static_cast<long long>(__hip_atomic_load(
        reinterpret_cast<unsigned long long*>(a.part_cnt + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) : 0;
    const long long pd = i < nblk ? static_cast<long long>(__hip_atomic_load(
        reinterpret_cast<unsigned long long*>(a.part_deg + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) : 0;
    const long long jc = wave_incl_scan(pc), jd = wave_incl_scan(pd);
    __syncthreads();
    if (lane == kWave - 1) {
      s_c[wv] = jc;
      s_d[wv] = jd;
    }
    __syncthreads();
    long long qc = 0, qd = 0, sc = 0, sd = 0;
#pragma unroll
    for (int k = 0; k < kScanChunk / kWave; ++k) {
      if (k < wv) {
        qc += s_c[k];
        qd += s_d[k];
      }
      sc += s_c[k];
      sd += s_d[k];
    }
    if (i < nblk) {
      a.part_cnt[i] = carry_c + qc + jc - pc;
      a.part_deg[i] = carry_d + qd + jd - pd;
    }
    carry_c += sc;
    carry_d += sd;
  }
  if (t == 0) scan_finish(a, carry_c, carry_d);
}


// ---------------------------------------------------------------------------
// Frontier compaction: one wave per 64-word unit (lane l loads word l), 4
// units per workgroup.  The unit's base slot and edge offset come from the
// scan; each set bit's slot from mbcnt and its edge offset from a wave prefix
// sum of degrees.  kSplit (graphs of few units): a unit per workgroup, 16
// words per wave; a first pass counts each part's entries and edges, the
// parts' bases are prefix-summed in LDS, and the second pass (row offsets now
// cache hits) writes -- twice the passes, a quarter of the steps each.
template <bool kSplit>
__global__ __launch_bounds__(kBlock) void compact_kernel(CompactArgs a) {
  if (a.ctrl && !chain_live(*a.ctrl, 'T', a.max_mf)) return;
  stamp_level_start(a.ctrl);
  constexpr int kWords = kSplit ? kWaveWords : kUnitWords;
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));  // (wave-uniform)
  const int64_t unit = kSplit ? static_cast<int64_t>(blockIdx.x) : static_cast<int64_t>(blockIdx.x) * kUnitsPerBlock + wv;
  const int64_t nunits = (a.words + kUnitWords - 1) / kUnitWords;
  if (unit >= nunits) return;  // (split: the whole workgroup)
  const int64_t w0 = unit * kUnitWords + (kSplit ? wv * kWaveWords : 0);
  const bool in = lane < kWords && w0 + lane < a.words;
  const word_t mine = in ? a.frontier[w0 + lane] : 0ull;
  if (a.clear_all && in) a.clear_all[w0 + lane] = 0ull;
  if (!kSplit && !__ballot(mine != 0)) return;
  if (a.clear && mine) a.clear[w0 + lane] = 0ull;  // read once: the next sparse level writes here
  const eid_t* __restrict__ ro = a.g.row_off;
  long long pos = a.unit_cnt_off[unit] + a.part_cnt[unit / kScanChunk];
  long long off = a.unit_deg_off[unit] + a.part_deg[unit / kScanChunk];
  // Frontier vertices of the unit in (word, bit) order, 64 per step (one per
  // lane, whatever word they sit in), so the work-list order is unchanged.
  const int fincl = static_cast<int>(wave_incl_scan(__popcll(mine)));
  const int ftotal = __builtin_amdgcn_readlane(fincl, kWave - 1);
  if constexpr (kSplit) {
    __shared__ long long s_pc[kUnitsPerBlock], s_pd[kUnitsPerBlock];
    long long pc = 0, pd = 0;
    for (int base = 0; base < ftotal; base += kWave) {
      const int idx = base + lane;
      const int vpos = wave_set_position(mine, fincl, idx);
      if (idx < ftotal) {
        const int64_t v = w0 * 64 + vpos;
        const eid_t d = ro[v + 1] - ro[v];
        pc += d > 0 ? 1 : 0;
        pd += d;
      }
    }
    pc = wave_sum(pc);
    pd = wave_sum(pd);
    if (lane == 0) {
      s_pc[wv] = pc;
      s_pd[wv] = pd;
    }
    __syncthreads();
    for (int k = 0; k < wv; ++k) {
      pos += s_pc[k];
      off += s_pd[k];
    }
  }
  for (int base = 0; base < ftotal; base += kWave) {
    const int idx = base + lane;
    const int vpos = wave_set_position(mine, fincl, idx);
    eid_t rs = 0, d = 0;
    if (idx < ftotal) {
      const int64_t v = w0 * 64 + vpos;
      rs = ro[v];
      d = ro[v + 1] - rs;
    }
    const bool take = d > 0;
    const unsigned long long tm = __ballot(take);
    const long long incl = wave_incl_scan(d);
    const long long p = pos + mask_rank(tm);
    const long long qs = off + incl - d;
    DBFS_DCHECK(!take || p < a.g.rows, 1, p);
    if (take) {
      a.qscan[p] = qs;
      a.qbase[p] = rs - qs;
      if (a.qv) a.qv[p] = static_cast<vid_t>(w0 * 64 + vpos);
    }
    wave_fill_blocks(a.blk_vstart, take, qs, d, p);
    pos += __popcll(tm);
    off += readlane_i64(incl, kWave - 1);
  }
}

// Narrow levels -> 32-bit levels (outside the timed traversal, on demand).
__global__ __launch_bounds__(kBlock) void widen_levels_kernel(const uint8_t* __restrict__ in, lvl_t* __restrict__ out,
                                                              int64_t n, uint8_t base) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
    const uint8_t v = static_cast<uint8_t>(in[i] - base);
    out[i] = v > kNarrowMaxLevel ? kUnreached : static_cast<lvl_t>(v);
  }
}

// Received owner lists -> candidate bits of the owned slice.
__global__ __launch_bounds__(kBlock) void list_scatter_kernel(ListScatterArgs a) {
  if (a.ctrl && !chain_live(*a.ctrl, 'T', a.max_mf)) return;
  const int r = blockIdx.y;
  // the send lists were read by the exchange (stream-ordered before this
  // kernel): their counts restart from zero for the next list-form chain
  if (a.reset_lists && blockIdx.x == 0 && threadIdx.x == 0) a.reset_lists[static_cast<int64_t>(r) * (a.list_cap + 1)] = 0;
  const vid_t* list = a.lists + static_cast<int64_t>(r) * (a.list_cap + 1);
  const int64_t n = list[0];
  DBFS_DCHECK(n <= a.list_cap, 5, n);
  for (int64_t k = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; k < n;
       k += static_cast<int64_t>(gridDim.x) * kBlock) {
    const int64_t v = static_cast<int64_t>(list[1 + k]) - a.lo;
    DBFS_DCHECK(v >= 0 && (a.words <= 0 || (v >> 6) < a.words), 6, list[1 + k]);
    atomicOr(a.cand + (v >> 6), 1ull << (v & 63));
  }
}

// Byte map -> bitmap for the multi-rank exchange (words of 64 vertices).
__global__ __launch_bounds__(kBlock) void pack_bytes_kernel(PackArgs a) {
  if (a.ctrl && (a.ctrl->done || (a.flag ? a.ctrl->dir != 'B' || !*a.flag : a.ctrl->dir != 'T' || !a.ctrl->bytes)))
    return;
  int64_t w = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (w >= a.skip_begin) w += a.skip_end - a.skip_begin;  // (the grid covers the other words only)
  if (w >= a.words) return;
  const word_t bits = gather_byte_bits(a.bytes + w * 64);
  if (bits) a.next[w] |= bits;
}

// Zero-degree / padding mask of the owned slice (computed once per graph).
__global__ __launch_bounds__(kBlock) void zero_degree_kernel(ZeroDegArgs a) {
  const int lane = lane_id();
  const int64_t w = static_cast<int64_t>(blockIdx.x) * (kBlock / kWave) + (threadIdx.x >> 6);
  if (w >= a.words) return;
  const int64_t v = w * 64 + lane;
  bool dead = true;
  if (v < a.g.rows) dead = !a.padding_only && a.g.row_off[v + 1] == a.g.row_off[v];
  const word_t m = __ballot(dead);
  if (lane == 0) a.out[w] = m;
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

// blockIdx.y = piece; 4-byte words, grid-stride over the piece.
__global__ __launch_bounds__(kBlock) void copy_pieces_kernel(Backend::CopyPieces c) {
  const int i = blockIdx.y;
  const int64_t n = c.bytes[i] / 4;
  const uint32_t* s = static_cast<const uint32_t*>(c.src[i]);
  uint32_t* d = static_cast<uint32_t*>(c.dst[i]);
  for (int64_t k = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; k < n;
       k += static_cast<int64_t>(gridDim.x) * kBlock)
    d[k] = s[k];
}

// RefreshArgs (a split top-down level): the claims of the parts so far into
// visited -- a word per thread, its 64 level bytes in four 16-byte loads.
__global__ __launch_bounds__(kBlock) void refresh_visited_kernel(RefreshArgs a) {
  if (a.ctrl && !chain_live(*a.ctrl, 'T', a.max_mf)) return;
  const uint8_t lv = static_cast<uint8_t>(a.narrow_base + a.new_level);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t w = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; w < a.words; w += stride) {
    const word_t m = gather_level_bits(a.level8 + w * 64, lv);
    if (m) a.visited[w] |= m;
  }
}

}  // namespace

void fill_level(lvl_t* level, int64_t n, lvl_t value, hipStream_t st) {
  if (n <= 0) return;
  const bool aligned16 = (reinterpret_cast<uintptr_t>(level) & 15u) == 0;
  fill_level_kernel<<<grid_for(n / 4 + 1, kBlock, 8192), kBlock, 0, st>>>(level, n, value, aligned16);
}

bool zero_fill(void* p, size_t bytes, hipStream_t st) {
  if ((reinterpret_cast<uintptr_t>(p) & 15u) != 0 || (bytes & 15u) != 0) return false;
  const int64_t n16 = static_cast<int64_t>(bytes / 16);
  zero16_kernel<<<grid_for(n16, kBlock, 4096), kBlock, 0, st>>>(static_cast<uint4*>(p), n16);
  return true;
}

void set_bit(word_t* bm, int64_t bit, hipStream_t st) { set_bit_kernel<<<1, 64, 0, st>>>(bm, bit); }

void level_ctrl_init(LevelCtrl* c, const LevelCtrl& init, hipStream_t st) { ctrl_init_kernel<<<1, 64, 0, st>>>(c, init); }

void init_run(const InitRunArgs& a, hipStream_t st) {
  const int64_t work = std::max<int64_t>(std::max<int64_t>(a.g.rows / 4, a.gwords), 1);
  init_run_kernel<<<grid_for(work, kBlock, 8 * device_cus()), kBlock, 0, st>>>(a);
}

void publish_stats(const int64_t* stats, StatsMailbox* mb, int64_t seq, hipStream_t st) {
  publish_stats_kernel<<<1, 64, 0, st>>>(stats, mb, seq);
}

// A graph of fewer units than kSplitUnits: a unit per workgroup, 16 words per
// wave (update_unit_split, compact_split) -- 4x the waves, a quarter of the
// dependent row_off steps each.
constexpr int64_t kSplitUnits = 4096;

void update_frontier(const UpdateArgs& a, hipStream_t st) {
  DBFS_CHECK(!a.end.active || (a.fuse_scan && a.ctrl && a.scan.stats), "update: a folded level end needs the fused finish");
  if (a.words <= 0) return;
  const int64_t nunits = (a.words + kUnitWords - 1) / kUnitWords;
  DBFS_CHECK(!a.fold_scan || (a.fuse_scan && a.scan.nunits == nunits && nunits <= kFoldScanUnits),
             "update: fold_scan needs the fused finish over at most kFoldScanUnits units");
  const bool split = nunits < kSplitUnits;
  const int64_t per = split ? kUnitWords : kUnitWords * kUnitsPerBlock;
  // fused finish: at most kMaxFusedGrid / 8 workgroups striding over the units
  // with one ticket; up to kMaxFusedGrid with the two-level ticket
  const unsigned grid = a.fuse_scan ? grid_for(a.words, per, a.group_ticket ? kMaxFusedGrid : kMaxFusedGrid / 8)
                                    : grid_for(a.words, per);
  const bool ranks = a.push || a.zero_next || a.end.active;
  if (split && ranks) update_kernel<true, true><<<grid, kBlock, 0, st>>>(a);
  else if (split) update_kernel<true, false><<<grid, kBlock, 0, st>>>(a);
  else if (ranks) update_kernel<false, true><<<grid, kBlock, 0, st>>>(a);
  else update_kernel<false, false><<<grid, kBlock, 0, st>>>(a);
}

void refresh_visited(const RefreshArgs& a, hipStream_t st) {
  if (a.words <= 0) return;
  refresh_visited_kernel<<<grid_for(a.words, kBlock, 4 * device_cus()), kBlock, 0, st>>>(a);
}

void totals_finish(const ScanArgs& a, hipStream_t st) { totals_finish_kernel<<<1, kScanChunk, 0, st>>>(a); }

void scan_units(const ScanArgs& a, hipStream_t st) {
  if (a.nunits <= 0) return;
  scan_units_kernel<<<grid_for(a.nunits, kScanChunk), kScanChunk, 0, st>>>(a);
}

void compact_frontier(const CompactArgs& a, hipStream_t st) {
  if (a.words <= 0) return;
  const int64_t nunits = (a.words + kUnitWords - 1) / kUnitWords;
  if (nunits < kSplitUnits) compact_kernel<true><<<grid_for(a.words, kUnitWords), kBlock, 0, st>>>(a);
  else compact_kernel<false><<<grid_for(a.words, kUnitWords * kUnitsPerBlock), kBlock, 0, st>>>(a);
}

void widen_levels(const uint8_t* in, lvl_t* out, int64_t n, uint8_t base, hipStream_t st) {
  if (n <= 0) return;
  widen_levels_kernel<<<grid_for(n, kBlock, 8 * device_cus()), kBlock, 0, st>>>(in, out, n, base);
}

void level_finish(const LevelFinishArgs& a, hipStream_t st) { level_finish_kernel<<<1, kBlock, 0, st>>>(a); }

void list_scatter(const ListScatterArgs& a, hipStream_t st) {
  if (a.nranks <= 0 || a.list_cap <= 0) return;
  const unsigned gx = grid_for(a.list_cap, kBlock, 256);
  list_scatter_kernel<<<dim3(gx, static_cast<unsigned>(a.nranks)), kBlock, 0, st>>>(a);
}

void pack_bytes(const PackArgs& a, hipStream_t st) {
  if (a.words - (a.skip_end - a.skip_begin) <= 0) return;
  DBFS_CHECK(a.skip_begin >= 0 && a.skip_begin <= a.skip_end && a.skip_end <= a.words, "pack_bytes: skipped range out of bounds");
  pack_bytes_kernel<<<grid_for(a.words - (a.skip_end - a.skip_begin), kBlock), kBlock, 0, st>>>(a);
}

// Compute units of the current device (cached per device id).
int device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) return 256;
  if (!cus[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

#ifdef DBFS_CHECKED
__global__ void check_fail_kernel(unsigned long long code) { DBFS_DCHECK(false, code, 0); }
#endif

void inject_check_failure(hipStream_t st) {
#ifdef DBFS_CHECKED
  check_fail_kernel<<<1, 1, 0, st>>>(99);
#else
  (void)st;
#endif
}

bool checks_enabled() {
#ifdef DBFS_CHECKED
  return true;
#else
  return false;
#endif
}

unsigned long long take_check_error() {
  // (each kernel file records into its own g_check; all are read and cleared)
  const unsigned long long h[3] = {take_check_local(), take_check_td(), take_check_bu()};
  for (unsigned long long x : h)
    if (x) return x;
  return 0;
}

void zero_degree_mask(const ZeroDegArgs& a, hipStream_t st) {
  if (a.words <= 0) return;
  zero_degree_kernel<<<grid_for(a.words, kBlock / kWave), kBlock, 0, st>>>(a);
}

void status_expand(const StatusArgs& a, hipStream_t st) {
  if (a.g.rows <= 0) return;
  status_kernel<<<grid_for(a.g.rows, kBlock), kBlock, 0, st>>>(a);
}

void copy_pieces(const Backend::CopyPieces& c, hipStream_t st) {
  int64_t mx = 0;
  for (int i = 0; i < c.n; ++i) mx = std::max(mx, c.bytes[i] / 4);
  if (c.n <= 0 || mx <= 0) return;
  copy_pieces_kernel<<<dim3(grid_for(mx, kBlock, 1024), static_cast<unsigned>(c.n)), kBlock, 0, st>>>(c);
}

void bitmap_or(word_t* dst, const word_t* src, int64_t words, hipStream_t st) {
  if (words <= 0) return;
  bitmap_or_kernel<<<grid_for(words, kBlock, 4096), kBlock, 0, st>>>(dst, src, words);
}

}  // namespace kern
}  // namespace dbfs
