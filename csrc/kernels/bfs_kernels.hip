// gfx950 BFS primitives: frontier update (visited-bitmap update + level write),
// multi-block unit scan, frontier compaction (wave prefix sums), load-balanced
// top-down neighbour gather, fused bottom-up parent search.
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
#include <type_traits>
#include <cstdio>

#include "launch.hpp"
#include "level_device.hpp"
#include "wave.hpp"

namespace dbfs {
namespace kern {
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
  const int64_t sw = src >= 0 ? a.vis_word_base + (src >> 6) : -1;
  const word_t sbit = src >= 0 ? (1ull << (src & 63)) : 0ull;
  for (int64_t w = t0; w < a.gwords; w += stride) a.visited[w] = a.zdeg[w] | (w == sw ? sbit : 0ull);
  for (int64_t w = t0; w < a.words; w += stride) a.frontier[w] = (src >= 0 && w == (src >> 6)) ? sbit : 0ull;
  if (a.frontier_clear)
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
    LevelCtrl c = a.ctrl_init;
    level_ctrl_finish(c, cnt, deg, true, nullptr);
    *a.ctrl = c;
    if (a.mailbox) stamp_mailbox(a.mailbox, c, -1);
  }
}

__global__ void level_finish_kernel(LevelFinishArgs a) {
  if (threadIdx.x == 0) level_finish_device(a);
}

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

// ---------------------------------------------------------------------------
// Frontier update: a wave owns 16 consecutive words.  Lanes 0..15 update the
// bitmap words (one coalesced 128-B access per array); then, for every
// non-zero new word, the wave switches to lane-per-vertex so the level stores
// and row_off loads of that word are one coalesced access each.
//
// Geometry: one wave per 64-word unit (lane l owns word l of the unit), 4
// units per workgroup -- a sparse level then costs ~4K workgroups of dispatch
// instead of 16K, and the unit statistics need no cross-wave reduction.
constexpr int kUnitsPerBlock = kBlock / kWave;
static_assert(kUnitWords == kWave, "one word per lane in update/compact");

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
    level_ctrl_finish(c, carry_c, carry_d, a.seed, a.seed ? nullptr : a.rec);
    if (!a.seed) {
      a.rec->t0 = c.t_start;
      a.rec->t1 = wall_clock64();
    }
    *a.ctrl = c;
    if (a.mailbox) stamp_mailbox(a.mailbox, c, a.level);
  }
}

// One wave per 64-word unit, kUnitsPerBlock units per workgroup; with the
// fused finish a smaller grid strides over the units (fewer ticket arrivals).
// kSplit waves per unit (small graphs: 4, each over 16 of its words -- a
// graph of few units would leave most wave slots idle while each wave walks
// its unit's new vertices 64 per dependent step); `sub` = this wave's part.
template <int kSplit = 1>
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
  if (kSplit == 1 && lane == 0) {
    a.unit_cnt[unit] = cnt;
    a.unit_deg[unit] = deg;
  }
}

// A unit per workgroup, its kSplit (= kUnitsPerBlock) waves each over a part
// (update_unit<kSplit>); the unit's statistics summed in LDS.
__device__ __forceinline__ void update_unit_split(const UpdateArgs& a, int64_t unit, bool use_bytes, long long& cnt,
                                                  long long& deg, long long* s_pc, long long* s_pd) {
  const int wv = static_cast<int>(threadIdx.x >> 6);
  update_unit<kUnitsPerBlock>(a, unit, use_bytes, cnt, deg, wv);
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
    a.unit_cnt[unit] = c;
    a.unit_deg[unit] = d;
  }
  __syncthreads();  // (s_pc / s_pd reused by the next unit)
}

template <bool kSplit>
__global__ __launch_bounds__(kBlock) void update_kernel(UpdateArgs a) {
  bool use_bytes = a.cand_bytes != nullptr;
  if (a.ctrl) {
    if (!chain_live(*a.ctrl, 'T', a.max_mf)) return;
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
      update_unit_split(a, unit, use_bytes, cnt, deg, s_pc, s_pd);
    } else {
      const int64_t unit = static_cast<int64_t>(blockIdx.x) * kUnitsPerBlock + wv;
      if (unit >= nunits) return;
      update_unit(a, unit, use_bytes, cnt, deg);
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
      update_unit_split(a, unit, use_bytes, cnt, deg, s_pc, s_pd);
      wc += cnt;  // (this wave's part: the workgroup's totals are the waves' sum, as below)
      wd += deg;
    }
  } else {
    for (int64_t unit = static_cast<int64_t>(blockIdx.x) * kUnitsPerBlock + wv; unit < nunits;
         unit += static_cast<int64_t>(gridDim.x) * kUnitsPerBlock) {
      long long cnt, deg;
      update_unit(a, unit, use_bytes, cnt, deg);
      wc += cnt;
      wd += deg;
    }
  }
  if (lane_id() == 0) {
    s_c[wv] = wc;
    s_d[wv] = wd;
  }
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
template <int kThreads, typename BaseT = long long>
__device__ __forceinline__ int td_block_owner_map(const int64_t* __restrict__ qscan, const int64_t* __restrict__ qbase,
                                                  const int32_t* __restrict__ blk_vstart, long long b,
                                                  long long nblocks, long long q, long long m, int32_t* s_owner,
                                                  BaseT* s_base, int32_t* s_wmax) {
  constexpr int kItems = kTdEdgesPerBlock / kThreads;
  const int t = threadIdx.x;
  const int lane = lane_id();
  const int wv = t >> 6;
  const long long e0 = b * kTdEdgesPerBlock;
  const long long e1 = min(m, e0 + kTdEdgesPerBlock);
  const int cnt = static_cast<int>(e1 - e0);
  const long long v0 = blk_vstart[b];
  const long long vlast = (b + 1 < nblocks) ? blk_vstart[b + 1] : q - 1;
  const int nv = static_cast<int>(vlast - v0 + 1);

  __syncthreads();  // LDS reuse across iterations
#pragma unroll
  for (int k = 0; k < kItems; ++k) s_owner[k * kThreads + t] = 0;
  __syncthreads();
  // Invariant (zero-degree vertices are never listed): nv <= EPB + 1.
  for (int i = t; i < nv && i <= kTdEdgesPerBlock; i += kThreads) {
    const long long qs = qscan[v0 + i];
    s_base[i] = static_cast<BaseT>(qbase[v0 + i]);
    const long long p = (qs > e0 ? qs : e0) - e0;
    if (p < cnt) s_owner[p] = i;
  }
  __syncthreads();
  // inclusive max-scan over s_owner: thread t owns entries [t*ITEMS, (t+1)*ITEMS)
  int vals[kItems];
  int run = 0;
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    run = max(run, s_owner[t * kItems + k]);
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
  for (int k = 0; k < kItems; ++k) s_owner[t * kItems + k] = max(vals[k], excl);
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

// kFilter: the hub-filter variant (kTdMaxHubs / 8 bytes more LDS --
// launched only for levels that may use it).  kBase32: the owner map's column
// bases in 32 bits (graphs of at most 2^32 adjacency entries): 16 instead of
// 24 KiB of LDS per workgroup, 8 resident workgroups per CU instead of 6 (5
// instead of 4 with the filter).
template <TdOut kOut, int kThreads, bool kFilter = false, bool kBase32 = false>
__global__ __launch_bounds__(kThreads) void td_expand_kernel(TdArgs a) {
  constexpr int kItems = kTdEdgesPerBlock / kThreads;
  constexpr bool kHubFilter = kFilter && kOut != TdOut::Lists && kThreads == kTdThreads;
  using BaseT = std::conditional_t<kBase32, uint32_t, long long>;
  __shared__ int32_t s_owner[kTdEdgesPerBlock];
  __shared__ BaseT s_base[kTdEdgesPerBlock + 1];
  __shared__ int32_t s_wmax[kThreads / kWave];
  __shared__ word_t s_hubvis[kHubFilter ? kTdMaxHubs / kWordBits : 1];
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
           i += static_cast<int64_t>(gridDim.x) * kThreads)
        a.clear_frontier[a.clear_qv[i] >> 6] = 0ull;
  }
  const long long nblocks = (m + kTdEdgesPerBlock - 1) / kTdEdgesPerBlock;
  const int t = threadIdx.x;
  const int lane = lane_id();
  const word_t* __restrict__ visited = a.visited;
  // large levels: hub targets tested in an LDS copy of the hubs' visited bits
  // (uniform: every workgroup sees the same m)
  bool filter = false;
  if constexpr (kHubFilter) {
    filter = a.td_hub_vis && a.g.td_col && m >= a.td_hub_min_edges && blockIdx.x < nblocks &&
             (!a.ctrl || static_cast<double>(a.ctrl->vis_deg) >= a.td_hub_vis_frac * a.ctrl->total_directed);
    if (filter) {
      const int64_t hw = (a.g.td_nhubs + kWordBits - 1) / kWordBits;
      for (int64_t i = t; i < hw; i += kThreads) s_hubvis[i] = a.td_hub_vis[i];
      // (td_block_owner_map starts with a barrier)
    }
  }
  const vid_t* __restrict__ col = filter ? a.g.td_col : a.g.col;

  for (long long b = blockIdx.x; b < nblocks; b += gridDim.x) {
    const long long e0 = b * kTdEdgesPerBlock;
    const int cnt = td_block_owner_map<kThreads, BaseT>(a.qscan, a.qbase, a.blk_vstart, b, nblocks, q, m, s_owner,
                                                        s_base, s_wmax);

    // All items' loads in flight together (column ids, then their visited /
    // next words), then the stores: the items of a thread are independent, but
    // the compiler cannot move a load above an earlier item's atomic, so one
    // item at a time costs kItems dependent round trips per block.
    vid_t vk[kItems];
    bool live[kItems];
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int idx = k * kThreads + t;
      int64_t ci;
      if constexpr (kBase32)
        ci = static_cast<uint32_t>(static_cast<uint32_t>(e0 + idx) + s_base[s_owner[idx]]);
      else
        ci = e0 + idx + s_base[s_owner[idx]];
      vk[k] = idx < cnt ? col[ci] : 0u;
      live[k] = idx < cnt;
    }
    // hub targets tested in the LDS snapshot: a visited hub is done here; an
    // unvisited one is decoded and needs no global visited probe (unvisited
    // at the level's start).  (Measured: claiming hubs in LDS as well, to
    // store each once per workgroup, is slower -- few repeats per workgroup,
    // LDS atomics on popular hubs serialise.)
    bool hubnew[kItems];
#pragma unroll
    for (int k = 0; k < kItems; ++k) hubnew[k] = false;
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

// Append v (act lanes) to its owner's list: one atomic per wave and owner on
// the count word (lists + owner * stride), the ids after it -- or, with a
// direct exchange table, after the count word of the owner's window slot
// (write-through stores over xGMI).  Wave-uniform call.
__device__ __forceinline__ void owner_list_append(vid_t* lists, int64_t stride, int64_t part, vid_t v, bool act,
                                                  const DirectTable* dt = nullptr) {
  const int lane = lane_id();
  const int owner = act ? static_cast<int>(static_cast<int64_t>(v) / part) : -1;
  unsigned long long pending = __ballot(act);
  while (pending) {
    const int leader = __ffsll(static_cast<long long>(pending)) - 1;
    const int o = __builtin_amdgcn_readfirstlane(__shfl(owner, leader, kWave));
    const unsigned long long msk = __ballot(owner == o);
    unsigned base = 0;
    vid_t* list = lists + static_cast<int64_t>(o) * stride;
    if (lane == leader) base = atomicAdd(list, static_cast<unsigned>(__popcll(msk)));
    base = __shfl(base, leader, kWave);
    DBFS_DCHECK(base + __popcll(msk) < static_cast<unsigned long long>(stride), 3, base);
    if (owner == o) {
      const unsigned at = 1 + base + mask_rank(msk);
      if (dt) sys_store_u32(dt->dst[o] + at, v);
      else list[at] = v;
    }
    pending &= ~msk;
  }
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
// (seq goes to the error word the host watches); kWaitLater when a cell
// already carries a LATER exchange's tag: the peer has moved on, which it
// does only after this rank's next signal -- so this exchange is over here
// (a workgroup of the apply that started after the level's end: it has
// nothing to do).  Data behind the cell is then read with sys loads.
constexpr int kWaitOk = 1, kWaitTimeout = 0, kWaitLater = -1;
__device__ __forceinline__ int direct_wait(const DirectExchange& d, uint64_t* out0, uint64_t* out1) {
  __shared__ int s_st;
  const int t = threadIdx.x;
  if (t == 0) s_st = kWaitOk;
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
        if ((spin & 255) == 255 && wall_clock64() - t0 > d.timeout_ticks) {
          s_st = kWaitTimeout;
          break;
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
  if (st == kWaitTimeout && t == 0 && d.error) sys_store_u64(d.error, d.seq);
  return st;
}

// The claimed, owned items of a lane (bit k of `claimed`: v[k], a global id
// of this shard): level, frontier bit, and the wave's work-list entries of
// the next level with one packed atomic (count << kSparseEdgeBits | edges)
// for all of them, so entries stay ordered by edge offset.  Wave-uniform call.
template <int kItems>
__device__ __forceinline__ void sparse_settle(const TdSparseArgs& a, const vid_t (&v)[kItems], unsigned claimed) {
  constexpr unsigned long long kEdgeMask = (1ull << kSparseEdgeBits) - 1;
  if (!__ballot(claimed != 0)) return;
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
  if (!ctot) return;
  unsigned long long old = 0;
  if (lane == 0)
    old = atomicAdd(a.counter, (static_cast<unsigned long long>(ctot) << kSparseEdgeBits) +
                                   static_cast<unsigned long long>(etot));
  old = __shfl(old, 0, kWave);
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
  a.stats[0] = a.stats[2] = cnt;
  a.stats[1] = a.stats[3] = deg;
  a.oscan[cnt] = deg;
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
__global__ __launch_bounds__(256) void direct_selftest_kernel(DirectExchange l, DirectExchange e, int round,
                                                              unsigned* err) {
  __shared__ uint64_t s_n[kern::kMaxPeers], s_x[2 * kern::kMaxPeers];
  const int t = threadIdx.x;
  const int me = l.rank, P = l.nranks;
  for (int p = 0; p < P; ++p) {
    if (p == me) continue;
    const uint32_t n = selftest_n(me, p, round);
    for (uint32_t i = t; i < n; i += 256) sys_store_u32(l.table->dst[p] + 1 + i, selftest_id(me, p, i, round));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
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

// Sparse top-down level (TdSparseArgs): expansion as td_expand, then every
// claimed vertex is finished in place (level, frontier bit, output entry), so
// the level is one launch (one rank); with several ranks remote claims go to
// their owners' lists and td_sparse_apply finishes the level after the
// exchange.  kThreads = 256: 8 edges per thread per block.
template <int kThreads>
__global__ __launch_bounds__(kThreads) void td_sparse_kernel(TdSparseArgs a) {
  constexpr int kItems = kTdEdgesPerBlock / kThreads;
  __shared__ int32_t s_owner[kTdEdgesPerBlock];
  __shared__ long long s_base[kTdEdgesPerBlock + 1];
  __shared__ int32_t s_wmax[kThreads / kWave];
  __shared__ int s_last;
  const bool dx = a.lists && a.direct.active;
  // uniform: the whole grid returns, no workgroup takes a ticket (a direct
  // exchange still publishes, empty)
  if (!chain_live(*a.ctrl, 'T', a.max_mf)) {
    if (dx && blockIdx.x == 0) direct_publish(a.direct, a.lists, a.list_stride, false);
    return;
  }
  if (a.first) stamp_level_start(a.ctrl);
  const long long q = a.dev_stats[0], m = a.dev_stats[1];
  const long long nblocks = (m + kTdEdgesPerBlock - 1) / kTdEdgesPerBlock;
  // Only the workgroups that have an edge block take part (at least one, for
  // the finish): the others return before the ticket -- on a level of a few
  // blocks, 256 workgroups queueing on one ticket address cost several us.
  const unsigned active = static_cast<unsigned>(nblocks < 1 ? 1 : (nblocks < gridDim.x ? nblocks : gridDim.x));
  if (blockIdx.x >= active) return;
  const int t = threadIdx.x;
  const int64_t gtid = static_cast<int64_t>(blockIdx.x) * kThreads + t;
  const int64_t gstride = static_cast<int64_t>(active) * kThreads;
  // the input vertices' frontier bits (the bitmap is not read here)
  for (int64_t i = gtid; i < q; i += gstride) a.frontier_in[a.qv[i] >> 6] = 0ull;

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
    if (a.lists) {
      // several ranks: claimed remote targets to their owners' lists
      unsigned remote = 0;
#pragma unroll
      for (int k = 0; k < kItems; ++k)
        if (((claimed >> k) & 1u) && static_cast<uint64_t>(v[k]) - lo >= rows) remote |= 1u << k;
      claimed &= ~remote;
      if (__ballot(remote != 0)) {
#pragma unroll
        for (int k = 0; k < kItems; ++k)
          owner_list_append(a.lists, a.list_stride, a.part, v[k], (remote >> k) & 1u, dx ? a.direct.table : nullptr);
      }
    }
    // (B) finish the wave's claimed vertices
    sparse_settle<kItems>(a, v, claimed);
  }
  if (a.lists) {
    // several ranks: td_sparse_apply finishes the level.  A direct exchange:
    // every wave's write-through stores drained, the workgroups' ticket, and
    // the last one publishes the counts and flags.
    if (!dx) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      const unsigned prev = atomicAdd(a.ticket, 1u);
      s_last = (prev == active - 1) ? 1 : 0;
      if (s_last) *a.ticket = 0u;  // (the apply's ticket next, stream-ordered)
    }
    __syncthreads();
    if (s_last) direct_publish(a.direct, a.lists, a.list_stride, true);
    return;
  }

  // last workgroup: the level's totals and decision (as scan_units_kernel)
  __syncthreads();
  if (t == 0) {
    // every wave's counter atomic has returned.  (No release: the last
    // workgroup reads only the counter, a device-scope atomic; the level's
    // stores are read by later launches.)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = atomicAdd(a.ticket, 1u);
    s_last = (prev == active - 1) ? 1 : 0;
    if (s_last) last_arriver_acquire();
  }
  __syncthreads();
  if (!s_last || t != 0) return;
  long long cnt = 0, deg = 0;
  sparse_totals(a, cnt, deg);
  LevelCtrl c = *a.ctrl;
  level_ctrl_finish(c, cnt, deg, false, a.rec);
  a.rec->t0 = c.t_start;
  a.rec->t1 = wall_clock64();
  *a.ctrl = c;
  if (a.mailbox) stamp_mailbox(a.mailbox, c, a.level_index);
}

// Several ranks, after the list exchange: the ids the other ranks claimed for
// this rank's vertices (recv_lists) are claimed here (fetch-or on the owned
// slice of `visited`; a vertex sent by several ranks, or claimed by this
// rank's own td_sparse, is settled once) and settled like td_sparse's owned
// claims; the last workgroup writes the level's local totals and zeroes the
// send lists' counts.  The lists' counts are loaded together (one per
// thread: they sit a stride apart, cold) and their entries form one index
// space the grid strides over.
template <int kThreads>
__global__ __launch_bounds__(kThreads) void td_sparse_apply_kernel(TdSparseArgs a) {
  constexpr int kItems = kTdItems;
  __shared__ int s_last;
  __shared__ long long s_end[kern::kMaxPeers];  // inclusive prefix of the counts
  __shared__ const vid_t* s_src[kern::kMaxPeers];
  __shared__ uint64_t s_cnt[kern::kMaxPeers];
  __shared__ uint64_t s_xend[2 * kern::kMaxPeers];
  // a direct exchange: the peers' cells (their counts) first, live chain or
  // not (every rank waits for every exchange: the window slots' reuse protocol)
  const bool dx = a.direct.active;
  if (dx && direct_wait(a.direct, s_cnt, nullptr) != kWaitOk) return;
  if (!chain_live(*a.ctrl, 'T', a.max_mf)) {
    // a folded level end is a collective: it runs on a no-op chain too
    if (a.end.active && blockIdx.x == 0) direct_level_end(a.end, a.stats[2], a.stats[3], a.stats, a.fin, s_xend);
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
  const unsigned active = static_cast<unsigned>(need < 1 ? 1 : (need < gridDim.x ? need : gridDim.x));
  if (blockIdx.x >= active) return;
  for (int64_t i0 = static_cast<int64_t>(blockIdx.x) * span; i0 < total; i0 += static_cast<int64_t>(active) * span) {
    vid_t v[kItems];
    word_t seen[kItems];
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
#pragma unroll
    for (int k = 0; k < kItems; ++k)
      seen[k] = i0 + static_cast<int64_t>(k) * kThreads + t < total ? a.visited[v[k] >> 6] : ~0ull;
    unsigned claimed = 0;
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const word_t bit = 1ull << (v[k] & 63);
      if (!(seen[k] & bit) && !(atomicOr(a.visited + (v[k] >> 6), bit) & bit)) claimed |= 1u << k;
    }
    sparse_settle<kItems>(a, v, claimed);
  }
  __syncthreads();
  if (t == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = atomicAdd(a.ticket, 1u);
    s_last = (prev == active - 1) ? 1 : 0;
    if (s_last) last_arriver_acquire();
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
  if (a.ctrl && (a.ctrl->done || a.ctrl->dir != 'T' || !a.ctrl->bytes)) return;
  const int64_t w = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (w >= a.words) return;
  const word_t bits = gather_byte_bits(a.bytes + w * 64);
  if (bits) a.next[w] |= bits;
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

template <bool kHub>
__device__ __forceinline__ bool bu_scan_row(const BuArgs& a, eid_t rs, eid_t e, bool found, const word_t* s_hub) {
  const int lane = lane_id();
  // hub-encoded copy of the adjacency when present (kHub kernels only)
  const vid_t* __restrict__ col = (kHub && a.g.hub_col) ? a.g.hub_col : a.g.col;
  const word_t* __restrict__ fr = a.frontier;
  // positions relative to the row start: 32-bit (a row never holds 2^32 entries)
  const vid_t* __restrict__ row = col + rs;
  const uint32_t len = static_cast<uint32_t>(e - rs);
  uint32_t p = min(len, 1u);
  const uint32_t lim = min(len, static_cast<uint32_t>(a.lane_limit));
  BU_STAT(3, __popcll(__ballot(p < lim && !found)));
  while (p < lim && !found) {
    BU_STAT(4, 1);
    vid_t u[kBuBatch];
    bool ok[kBuBatch];
#pragma unroll
    for (int k = 0; k < kBuBatch; ++k) {
      ok[k] = p + k < lim;
      u[k] = ok[k] ? row[p + k] : 0u;
    }
#pragma unroll
    for (int k = 0; k < kBuBatch; ++k) found |= ok[k] && bu_probe<kHub>(fr, s_hub, u[k]);
    p += kBuBatch;
  }
  if (p > lim) p = lim;
  // Phase 2: the wave scans each still-unresolved row in turn
  unsigned long long pending = __ballot(!found && p < len);
  BU_STAT(5, __popcll(pending));
  while (pending) {
    const int l = __ffsll(static_cast<long long>(pending)) - 1;
    pending &= pending - 1;
    const vid_t* r = reinterpret_cast<const vid_t*>(__shfl(reinterpret_cast<long long>(row), l, kWave));
    const uint32_t ps = __shfl(p, l, kWave), pe = __shfl(len, l, kWave);
    bool f = false;
    for (uint32_t base = ps; base < pe; base += kWave) {
      BU_STAT(6, 1);
      const uint32_t idx = base + lane;
      const vid_t u = idx < pe ? r[idx] : kNoVertex;
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
template <bool kHub, int kWords = kWaveWords, int kQueue = 0, bool kRec = false>
__device__ __forceinline__ void bu_wave_compact(const BuArgs& a, int64_t w0, word_t* s_res, const word_t* s_hub,
                                                long long& cnt, long long& deg, unsigned long long* s_q = nullptr) {
  static_assert(kWords <= kWave, "one word per lane");
  const int lane = lane_id();
  const int64_t left = a.words - w0;
  const int nw = left <= 0 ? 0 : (left < kWords ? static_cast<int>(left) : kWords);
  // unvisited bits of word `lane` (0 past the words); visited = ~um
  const word_t um = lane < nw ? ~a.visited[w0 + lane] : 0ull;
  const int incl = static_cast<int>(wave_incl_scan(__popcll(um)));
  const int total = __builtin_amdgcn_readlane(incl, kWave - 1);
  if (lane < kWords) s_res[lane] = 0ull;
  if (total == 0) {
    if (lane < nw) a.new_frontier[w0 + lane] = 0ull;
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
    const bool f = bu_scan_row<kHub>(a, qrs, qe, lane >= qn, s_hub);
    settle(lane < qn && f, ql, qrs, qe);
    qn = 0;
  };
  for (int b = 0; b < nb; ++b) {
    const int loc = n_loc;
    const eid_t rs = n_rs, e = n_rs + n_len;
    const vid_t u0 = n_u;
    fetch(b + 1, n_loc, n_rs, n_len, n_u);  // in flight during this batch's probes
    bool found = false;
    if (rs < e) found = bu_probe<kHub>(fr, s_hub, u0);
    BU_STAT(0, 1);
    BU_STAT(1, __popcll(__ballot(loc >= 0)));
    BU_STAT(2, __popcll(__ballot(found)));
    if (!head) n_u = n_len ? col[n_rs] : 0u;
    if constexpr (kQueue > 0) {
      // found by the head: settled now; unresolved rows with more neighbours
      // are queued (huge rows / spans scanned in place)
      const bool need = !found && e - rs > 1;
      const bool fits = q_span_ok && e - rs < (eid_t(1) << 20);
      // more unresolved rows than the queue holds (a sparse-hit level: most
      // lanes scan anyway, deferring gains nothing): all in place
      const bool direct = __popcll(__ballot(need && fits)) > kQueue;
      const bool inplace = need && (direct || !fits);
      if (__ballot(inplace)) {
        // (lanes not scanned here pass as resolved and keep their result)
        const bool f = bu_scan_row<kHub>(a, rs, e, found || !inplace, s_hub);
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
      found = bu_scan_row<kHub>(a, rs, e, found, s_hub);
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
    const word_t res = s_res[lane];
    a.new_frontier[w0 + lane] = res;
    if (res) a.visited[w0 + lane] = ~um | res;
  }
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
    const unsigned prev = atomicAdd(a.scan.ticket, 1u);
    s_last = prev == gridDim.x - 1;
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

// kEnd: the level's end folded in (BuArgs::end; several ranks only -- its
// code costs the one-rank kernels their spill-free 64 registers).
template <bool kWhole, int kThreads = kHubBuThreads, int kQ = kBuQueue, bool kRec = false, bool kEnd = false>
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
  if (!a.hub_front) stamp_level_start(a.ctrl);
  const int64_t hw = (a.g.nhubs + kWordBits - 1) / kWordBits;
  for (int64_t i = threadIdx.x; i < hw; i += kThreads) s_hub[i] = a.hub_front[i];
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
    for (int64_t u = static_cast<int64_t>(blockIdx.x) * kWavesPerBlock + wave; u < nunits;
         u += static_cast<int64_t>(gridDim.x) * kWavesPerBlock) {
      long long cnt = 0, deg = 0;
      bu_wave_compact<true, kUnitWords, kQ, kRec>(a, u * kUnitWords, s_res + wave * kUnitWords, s_hub, cnt, deg,
                                                  s_q + wave * kQ);
      cnt = wave_sum(cnt);
      deg = wave_sum(deg);
      if (lane_id() == 0) {
        a.unit_cnt[u] = cnt;
        a.unit_deg[u] = deg;
        s_c[wave] += cnt;
        s_d[wave] += deg;
      }
    }
    if (!a.fuse_scan) return;
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
  // 16 words per wave: unit groups of 4 waves walk the units; every workgroup
  // runs the same number of iterations (barriers stay uniform)
  constexpr int kGroups = kThreads / kUnitThreads;
  const int group = wave / kUnitWaves;
  const int wg = wave % kUnitWaves;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kGroups;
  // the unit groups' totals for the fused finish, in LDS (registers live
  // across the loop would spill)
  __shared__ long long s_acc[2 * kGroups];
  if (threadIdx.x < 2 * kGroups) s_acc[threadIdx.x] = 0;
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * kGroups; base < nunits; base += stride) {
    const int64_t u = base + group;
    long long cnt = 0, deg = 0;
    if (u < nunits)
      bu_wave_compact<true, kWaveWords, kQ, kRec>(a, u * kUnitWords + wg * kWaveWords, s_res + wave * kWaveWords, s_hub,
                                                  cnt, deg, s_q + wave * kQ);
    cnt = wave_sum(cnt);
    deg = wave_sum(deg);
    if (lane_id() == 0) {
      s_c[wave] = cnt;
      s_d[wave] = deg;
    }
    __syncthreads();
    if ((threadIdx.x & (kUnitThreads - 1)) == 0 && u < nunits) {
      long long c = 0, d = 0;
#pragma unroll
      for (int k = 0; k < kUnitWaves; ++k) {
        c += s_c[group * kUnitWaves + k];
        d += s_d[group * kUnitWaves + k];
      }
      a.unit_cnt[u] = c;
      a.unit_deg[u] = d;
      s_acc[2 * group] += c;
      s_acc[2 * group + 1] += d;
    }
    __syncthreads();
  }
  if (!a.fuse_scan) return;
  __syncthreads();  // (an empty loop: the accumulators' zeroing)
  long long wc = 0, wd = 0;
  if (threadIdx.x == 0)
    for (int g = 0; g < kGroups; ++g) {
      wc += s_acc[2 * g];
      wd += s_acc[2 * g + 1];
    }
  bu_fused_finish<kThreads, kEnd>(a, wc, wd, s_c, s_d, reinterpret_cast<uint64_t*>(s_res));
}

// hub_front bit h = frontier bit of hub_vertex[h]: one wave per hub word;
// several ranks: then the whole grid merges the frontier into visited.
__global__ __launch_bounds__(kBlock) void hub_gather_kernel(HubGatherArgs a) {
  if (a.ctrl && (a.ctrl->done || a.ctrl->dir != 'B')) return;
  stamp_level_start(a.ctrl);
  const int64_t w = static_cast<int64_t>(blockIdx.x) * (kBlock / kWave) + (threadIdx.x >> 6);
  const int64_t h = w * kWave + lane_id();
  const bool bit = h < a.g.nhubs && test_bit(a.frontier, a.g.hub_vertex[h]);
  const word_t m = __ballot(bit);
  if (lane_id() == 0 && w * kWave < a.g.nhubs) a.hub_front[w] = m;
  if (a.visited) {
    const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < a.words; i += stride) {
      const word_t f = a.frontier[i];
      if (f) a.visited[i] |= f;
    }
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

void level_ctrl_init(LevelCtrl* c, const LevelCtrl& init, hipStream_t st) { ctrl_init_kernel<<<1, 64, 0, st>>>(c, init); }

int device_cus();

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
  if (a.words <= 0) return;
  const int64_t nunits = (a.words + kUnitWords - 1) / kUnitWords;
  const bool split = nunits < kSplitUnits;
  const int64_t per = split ? kUnitWords : kUnitWords * kUnitsPerBlock;
  // fused finish: at most kMaxFusedGrid / 8 workgroups striding over the units
  // with one ticket; up to kMaxFusedGrid with the two-level ticket
  const unsigned grid = a.fuse_scan ? grid_for(a.words, per, a.group_ticket ? kMaxFusedGrid : kMaxFusedGrid / 8)
                                    : grid_for(a.words, per);
  if (split) update_kernel<true><<<grid, kBlock, 0, st>>>(a);
  else update_kernel<false><<<grid, kBlock, 0, st>>>(a);
}

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
template <TdOut kOut, bool kFilter, bool kBase32>
unsigned td_resident_grid(int64_t cap) {
  static const int per_cu = [] {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, td_expand_kernel<kOut, kTdThreads, kFilter, kBase32>,
                                                     kTdThreads, 0) != hipSuccess || n <= 0)
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
  td_sparse_kernel<kTdThreads><<<static_cast<unsigned>(a.grid), kTdThreads, 0, st>>>(a);
}

void direct_selftest(const DirectExchange& lists, const DirectExchange& end, int round, unsigned* err,
                     hipStream_t st) {
  direct_selftest_kernel<<<1, 256, 0, st>>>(lists, end, round, err);
}

void td_sparse_apply(const TdSparseArgs& a, hipStream_t st) {
  td_sparse_apply_kernel<kTdThreads><<<static_cast<unsigned>(std::max<int64_t>(1, a.grid)), kTdThreads, 0, st>>>(a);
}

void widen_levels(const uint8_t* in, lvl_t* out, int64_t n, uint8_t base, hipStream_t st) {
  if (n <= 0) return;
  widen_levels_kernel<<<grid_for(n, kBlock, 8 * device_cus()), kBlock, 0, st>>>(in, out, n, base);
}

void level_finish(const LevelFinishArgs& a, hipStream_t st) { level_finish_kernel<<<1, 64, 0, st>>>(a); }

void list_scatter(const ListScatterArgs& a, hipStream_t st) {
  if (a.nranks <= 0 || a.list_cap <= 0) return;
  const unsigned gx = grid_for(a.list_cap, kBlock, 256);
  list_scatter_kernel<<<dim3(gx, static_cast<unsigned>(a.nranks)), kBlock, 0, st>>>(a);
}

void pack_bytes(const PackArgs& a, hipStream_t st) {
  if (a.words <= 0) return;
  pack_bytes_kernel<<<grid_for(a.words, kBlock), kBlock, 0, st>>>(a);
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
  if (a.g.nhubs > 0 && a.hub_front) {
    const int64_t nunits = (a.words + kUnitWords - 1) / kUnitWords;
    // a whole 64-word unit per wave when the shard has enough units to fill
    // every resident wave slot (one GPU); small shards (many ranks) keep 16
    // words per wave for parallelism
    const int64_t slots = 2 * static_cast<int64_t>(device_cus()) * (kHubBuThreads / kWave);
    const bool whole = a.whole_units > 0 || (a.whole_units == 0 && nunits >= slots);
    // a bottom-up level after another one (few unvisited vertices left, most
    // of them scanning rows): whole units in 768-thread workgroups (80 VGPRs
    // instead of 64); 16-word waves without the row queue (measured)
    constexpr int kFollowThreads = 768;
    const int threads = whole ? (a.follow_up ? kFollowThreads : kHubBuThreads) : kHubBuThreads;
    const unsigned grid = grid_for(nunits, whole ? threads / kWave : kHubBuThreads / kUnitThreads, 2 * device_cus());
    // packed row records (compile-time path: the view's fallback costs registers)
    const bool rec = a.g.nz_rec && a.g.unit_base && a.g.nz_pref && a.g.nz_row_off && a.zdeg && a.g.head;
    if (a.fuse_scan && grid > static_cast<unsigned>(kMaxFusedGrid)) {
      DBFS_CHECK(!a.end.active, "bu_step: a folded level end needs the fused finish");
      // (more workgroups than totals slots: finish in a kernel of its own)
      BuArgs b = a;
      b.fuse_scan = false;
      bu_step(b, st);
      totals_finish_kernel<<<1, kScanChunk, 0, st>>>(a.scan);
      return;
    }
    // (every hub kernel runs the fused finish itself; a folded level end is
    // compiled only into the kEnd variants)
#define DBFS_BU_LAUNCH(W, T, Q, R)                                                          \
  do {                                                                                    \
    if (a.end.active) bu_hub_kernel<W, T, Q, R, true><<<grid, T, 0, st>>>(a);            \
    else bu_hub_kernel<W, T, Q, R, false><<<grid, T, 0, st>>>(a);                        \
  } while (0)
    if (whole) {
      if (a.follow_up && rec) DBFS_BU_LAUNCH(true, kFollowThreads, kBuQueue, true);
      else if (a.follow_up) DBFS_BU_LAUNCH(true, kFollowThreads, kBuQueue, false);
      else if (rec) DBFS_BU_LAUNCH(true, kHubBuThreads, kBuQueue, true);
      else DBFS_BU_LAUNCH(true, kHubBuThreads, kBuQueue, false);
      return;
    }
    if (a.follow_up && rec) DBFS_BU_LAUNCH(false, kHubBuThreads, 0, true);
    else if (a.follow_up) DBFS_BU_LAUNCH(false, kHubBuThreads, 0, false);
    else if (rec) DBFS_BU_LAUNCH(false, kHubBuThreads, kBuQueue, true);
    else DBFS_BU_LAUNCH(false, kHubBuThreads, kBuQueue, false);
#undef DBFS_BU_LAUNCH
    return;
  }
  DBFS_CHECK(!a.end.active, "bu_step: a folded level end needs the hub kernels' fused finish");
  bu_kernel<<<grid_for(a.words, kUnitWords), kUnitThreads, 0, st>>>(a);
  if (a.fuse_scan) totals_finish_kernel<<<1, kScanChunk, 0, st>>>(a.scan);
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
#ifdef DBFS_CHECKED
  unsigned long long h = 0, z = 0;
  (void)hipMemcpyFromSymbol(&h, HIP_SYMBOL(g_check), sizeof(h));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_check), &z, sizeof(z));
  return h;
#else
  return 0;
#endif
}

void hub_visited(const HubVisitedArgs& a, hipStream_t st) {
  if (a.g.td_nhubs <= 0) return;
  hub_visited_kernel<<<grid_for((a.g.td_nhubs + kWave - 1) / kWave, kBlock / kWave), kBlock, 0, st>>>(a);
}

void hub_apply(const HubApplyArgs& a, hipStream_t st) {
  if (a.g.td_nhubs <= 0 || a.g.td_nhubs > kTdMaxHubs) return;  // (select_hubs: at most kTdMaxHubs)
  hub_apply_kernel<<<grid_for((a.g.td_nhubs + 15) / 16, kBlock), kBlock, 0, st>>>(a);
}

void hub_gather(const HubGatherArgs& a, hipStream_t st) {
  if (a.g.nhubs <= 0) return;
  unsigned grid = grid_for((a.g.nhubs + kWave - 1) / kWave, kBlock / kWave);
  if (a.visited) grid = std::max(grid, grid_for(a.words, kBlock, 2048));
  hub_gather_kernel<<<grid, kBlock, 0, st>>>(a);
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
