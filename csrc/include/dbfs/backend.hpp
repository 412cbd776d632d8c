// Device abstraction the BFS engine is written against.
//
// Two implementations:
//   HipBackend  -- hand-written gfx950 HIP kernels on one HIP stream (the
//                  production path; csrc/backend/hip_backend.hip,
//                  csrc/kernels/*.hip).
//   CpuBackend  -- straightforward host loops with the identical semantics,
//                  used by the CPU test-suite (gloo multi-process tests) and
//                  the `--cpu` CLI path (csrc/backend/cpu_backend.cpp).
//
// Every primitive is asynchronous with respect to the host on the backend's
// stream (CpuBackend executes eagerly).  The reference has no such layer: its
// kernels take raw pointers pulled out of __managed__ tables (bfs.cu:252-269,
// 580-585).
#pragma once

#include <atomic>
#include <cstddef>
#include <functional>
#include <memory>
#include <string>
#include <utility>

#include "dbfs/common.hpp"
#include "dbfs/rmat.hpp"

namespace dbfs {

enum class DeviceKind { CPU, HIP };

// ---- kernel argument blocks -------------------------------------------------

// Local CSR shard: rows [lo, lo + rows) of an n-vertex graph, global column ids.
// Packed row record of the non-empty-row view (ShardView::nz_rec).
struct alignas(8) NzRec {
  uint32_t off;   // row start - unit_base[unit]
  vid_t head;     // the row's head (hub-encoded like ShardView::head)
};

struct ShardView {
  const eid_t* row_off = nullptr;  // rows + 1 (local)
  const vid_t* col = nullptr;      // row_off[rows]
  int64_t n = 0, lo = 0, rows = 0, nnz = 0;
  // Optional per-row copy of the first neighbour (col[row_off[r]]; any value
  // for empty rows), laid out per vertex so a wave's 64 first probes are one
  // coalesced 256-B load instead of 64 scattered col[] lines.
  const vid_t* head = nullptr;
  // Hub-encoded heads (nhubs > 0): the nhubs highest-degree vertices of the
  // whole graph get compact indices; head[r] = kHubFlag | index when the row's
  // first neighbour is a hub (hub_vertex[index] = its vertex id), else the
  // vertex id.  Bottom-up keeps the hubs' frontier bits in LDS.
  const vid_t* hub_vertex = nullptr;
  int64_t nhubs = 0;
  // Hub-encoded copy of col (same layout; hub neighbours as kHubFlag | index),
  // read by bottom-up so that probes of hub neighbours hit LDS too.
  const vid_t* hub_col = nullptr;
  // Optional non-empty-row view (Graph500 RMAT: about half the vertices have
  // no edges): nz_pref[w] = number of non-empty rows before bitmap word w,
  // nz_row_off / nz_head = row_off / head of the non-empty rows only (dense,
  // so a bottom-up wave touches half the cache lines).  Row k of the view is
  // [nz_row_off[k], nz_row_off[k + 1]).
  const eid_t* nz_pref = nullptr;
  const eid_t* nz_row_off = nullptr;
  const vid_t* nz_head = nullptr;
  // Packed non-empty-row records (optional, with the view): nz_rec[k] = {row
  // start relative to unit_base[U], head} for row k of unit U (4096
  // vertices); row k ends where row k + 1 starts, or at unit_base[U + 1] for
  // the unit's last non-empty row.  8 bytes per row instead of the view's
  // 8-byte offset + 4-byte head; present when every unit spans < 2^32 edges.
  const struct NzRec* nz_rec = nullptr;
  const eid_t* unit_base = nullptr;  // ceil(rows / 4096) + 1 entries: row_off of each unit's first vertex
  // Top-down copy of col (same layout, neighbour-id order) with the
  // td_nhubs highest-degree vertices encoded as kHubFlag | index
  // (td_hub_vertex[index] = the vertex): a large top-down level tests them in
  // an LDS copy of their visited bits and reads no visited word for them.
  const vid_t* td_col = nullptr;
  const vid_t* td_hub_vertex = nullptr;
  int64_t td_nhubs = 0;
  // One rank with hubs: bit v set when vertex v is a hub (the hubs are every
  // vertex of degree >= the hub threshold, so a hub-first row's hubs are a
  // prefix of it).  Read by the hub-cut bottom-up level (BuArgs::cut_edges).
  const word_t* hub_bits = nullptr;
  // Degree of every hub (nhubs entries; several ranks: a hub's row lives on
  // its owner, so the hub-cut decision sums these instead of row lengths).
  const uint32_t* hub_deg = nullptr;
};

// At most kTdMaxHubs top-down hubs (their visited bits, 8 KiB, sit in LDS
// next to the top-down owner map: five 256-thread workgroups per CU).
// Measured (RMAT-22 top-down only, hub marks on): 2^13 / 2^14 / 2^15 / 2^16
// / 2^17 / 2^18 hubs: 60 / 62 / 71 / 77 / 69 / 60 GTEPS.
#ifndef DBFS_TD_MAX_HUBS_LOG2
#define DBFS_TD_MAX_HUBS_LOG2 16
#endif
constexpr int64_t kTdMaxHubs = int64_t(1) << DBFS_TD_MAX_HUBS_LOG2;

// At most kMaxHubs hubs: their frontier bitmap (64 KiB) is staged in LDS by
// every bottom-up workgroup (two 1024-thread workgroups per CU fit in 160 KiB).
// (2^19 - 2^12: the 512 B below 64 KiB leave room for a 64-entry deferred-scan
// queue per wave next to the hub bits in two workgroups' LDS, see bu_hub_kernel)
#ifndef DBFS_MAX_HUBS
#define DBFS_MAX_HUBS ((int64_t(1) << 19) - (int64_t(1) << 12))
#endif
constexpr int64_t kMaxHubs = DBFS_MAX_HUBS;
constexpr vid_t kHubFlag = 0x80000000u;
// Rows of up to kSortedRowMax entries are sorted hub-first (neighbour degree
// descending, graph_sort); longer ones (a handful of hubs) keep their order.
constexpr int kSortedRowMax = 4096;
// Narrow (8-bit) level arrays: 0xFF = unreached, levels 0 .. 254.
constexpr uint8_t kNarrowUnreached = 0xFF;
// One-byte levels are stored as base + level, base = 64 x (run number mod
// kNarrowEpochs): a byte outside [base, base + kNarrowMaxLevel] reads as
// unreached, so the array is refilled with 0xFF only every kNarrowEpochs runs
// (base + 63 marks a level too deep for the narrow array: the traversal is
// repeated with 32-bit levels).
constexpr int kNarrowMaxLevel = 62;
constexpr int kNarrowEpochs = 4;

// Frontier bookkeeping is organised in "units" of 64 bitmap words (4096
// vertices): one 256-thread workgroup (4 waves) per unit, 16 consecutive words
// per wave64, in the HIP kernels.  (One wave per word would launch 1M waves for
// RMAT-26: dispatch alone then costs ~300 us per kernel on MI355X.)  Per-unit
// counts are scanned by a multi-block scan whose chunks hold kScanChunk units.
constexpr int kWaveWords = 16;
constexpr int kUnitWaves = 4;
constexpr int kUnitWords = kWaveWords * kUnitWaves;
constexpr int kUnitVertices = kUnitWords * kWordBits;
constexpr int kScanChunk = 1024;
// At most this many units are prefix-scanned by a fused finish's last
// workgroup (UpdateArgs::fold_scan): 32 per thread of a 256-thread workgroup.
constexpr int kFoldScanUnits = 8192;
// Top-down expansion handles kTdEdgesPerBlock frontier edges per workgroup.
constexpr int kTdThreads = 256;
constexpr int kTdItems = 8;
constexpr int kTdEdgesPerBlock = kTdThreads * kTdItems;

// ---- device-driven level loop (one rank) -------------------------------------
// The host enqueues level L+1 before level L has finished; every kernel of a
// level reads this block at entry and returns at once when the level is not
// its direction (or the traversal is done).  The scan's last workgroup turns
// the new frontier's totals into the next level's decision (level_ctrl_finish,
// the same Beamer switch as the host loop), so no per-level host round trip
// (~19 us of idle GPU on MI355X: D2H, host wake-up, next launch) remains.
struct LevelCtrl {
  // configuration (written once per run)
  int32_t mode = 2;             // 0 top-down only, 1 bottom-up only, 2 direction-optimising
  int32_t pad0 = 0;
  double alpha = 24.0, beta = 96.0;
  double n = 0.0, total_directed = 0.0;
  double td_byte_edges = 0.0, check_visited_min = 0.0;
  // state after the last finished level
  int32_t dir = 'T';            // direction of the next level
  int32_t bytes = 0;            // next top-down level writes the byte map
  int32_t check_visited = 1;    // ... with the visited pre-check
  int32_t done = 0;             // frontier empty: every later kernel returns
  int64_t n_f = 0, m_f = 0, prev_nf = 0, vis_deg = 0;
  int64_t reached = 0;          // vertices with degree > 0 reached so far (counts summed)
  // device wall clock (Backend::wall_clock_khz) when the running level's
  // first kernel started
  uint64_t t_start = 0;
  // Vertices with degree > 0 in the whole graph (configuration; 0: unknown --
  // directed graphs).  Once every one of them is reached no edge can discover
  // anything: the traversal is done without expanding its last frontier.
  int64_t n_active = 0;
};

// One record per finished level (device array; read after the run).
struct LevelRecDev {
  int32_t dir = 0, pad = 0;
  int64_t n_f = 0, m_f = 0, discovered = 0;
  uint64_t t0 = 0, t1 = 0;  // device wall clock: first kernel started, scan finished
};

// Host-visible mailbox slot (pinned, device-mapped), written by the scan's
// last workgroup of level L into slot L % kMailboxSlots.
struct LevelMailbox {
  int32_t level = -2;           // level that wrote this slot
  int32_t done = 0;
  int64_t vis_deg = 0;
  int32_t next_dir = 0;         // direction decided for the following level
  int32_t pad = 0;
  int64_t n_f = 0, m_f = 0;     // the following level's frontier (vertices, edges)
  int64_t reached = 0;          // LevelCtrl::reached
};
constexpr int kMailboxSlots = 8;

// Shared host/device decision logic (also used by the CPU backend).
DBFS_HD void level_ctrl_finish(LevelCtrl& c, int64_t count, int64_t degsum, bool seed, LevelRecDev* rec) {
  if (seed) {
    c.prev_nf = 0;
    c.vis_deg = degsum;
    c.reached = count;
  } else {
    rec->dir = c.dir;
    rec->n_f = c.n_f;
    rec->m_f = c.m_f;
    rec->discovered = count;
    c.prev_nf = c.n_f;
    c.vis_deg += degsum;
    c.reached += count;
  }
  c.n_f = count;
  c.m_f = degsum;
  c.done = count == 0 ? 1 : 0;
  if (!c.done && c.mode == 2) {
    const double m_u = c.total_directed - static_cast<double>(c.vis_deg);
    if (c.dir == 'T' && static_cast<double>(c.m_f) > m_u / c.alpha && c.n_f > c.prev_nf)
      c.dir = 'B';
    else if (c.dir == 'B' && static_cast<double>(c.n_f) < c.n / c.beta && c.n_f < c.prev_nf)
      c.dir = 'T';
  }
  // every vertex with an edge reached: the last frontier's edges can only
  // find visited vertices (levels, reached vertices and edges unchanged)
  if (c.n_active > 0 && c.reached >= c.n_active) c.done = 1;
  c.bytes = (c.dir == 'T' && static_cast<double>(c.m_f) >= c.td_byte_edges) ? 1 : 0;
  c.check_visited = static_cast<double>(c.vis_deg) >= c.check_visited_min * c.total_directed ? 1 : 0;
}

// Per-run initialisation of the bitmap engine in one pass (replaces a level
// fill, a visited copy, the seed update and its scan: ~8 dependent launches):
//   level[r] = kUnreached (0 for the source), visited = zdeg (+ source bit),
//   frontier (owned slice) = source bit only, and the seed's totals --
//   stats[0..3] = (count, degree sum) of {source} counting degree > 0 only,
//   qscan[count] = degree sum, the source unit's scan offsets = 0 -- exactly
//   what update + scan leave for a one-vertex frontier.  With ctrl, the
//   device-loop state is *ctrl = level_ctrl_finish(ctrl_init, seed) and the
//   mailbox slot of level -1 is stamped.
struct InitRunArgs {
  ShardView g;
  lvl_t* level = nullptr;          // rows
  // Narrow level array (one byte per vertex, kNarrowUnreached = not reached;
  // levels up to kNarrowMaxLevel): written instead of `level` when set, here
  // and by every bitmap-engine kernel that writes levels.
  uint8_t* level8 = nullptr;
  uint8_t narrow_base = 0;             // narrow level bytes of this run: base + level (kNarrowEpochs)
  bool level8_filled = false;      // level8 already holds kNarrowUnreached (prefilled): only the source's byte
  const word_t* zdeg = nullptr;    // global
  word_t* visited = nullptr;       // global
  int64_t gwords = 0;
  word_t* frontier = nullptr;      // owned slice of the seed frontier
  int64_t words = 0;
  int64_t src_local = -1;          // source row on this rank, -1 if not owned
  int64_t vis_word_base = 0;       // global word index of the owned slice
  int64_t* unit_cnt = nullptr;
  int64_t* unit_deg = nullptr;
  int64_t* part_cnt = nullptr;
  int64_t* part_deg = nullptr;
  int64_t* stats = nullptr;
  int64_t* qscan = nullptr;
  // Device loop: the seed's work-list entry (source vertex, qbase, the edge
  // blocks it covers) so a sparse first level can run without a compaction,
  // and frontier_clear (the first level's output bitmap) zeroed.
  int64_t* qbase = nullptr;
  int32_t* blk_vstart = nullptr;
  vid_t* qv = nullptr;
  word_t* frontier_clear = nullptr;
  // both owned frontier slices are known zero (the previous traversal ended
  // on a top-down level that found nothing: top-down levels clear their input
  // as they read it and set only new bits): only the seed's word is written
  // (the CPU backend checks the claim)
  bool frontier_clean = false;
  LevelCtrl* ctrl = nullptr;
  LevelCtrl ctrl_init;
  LevelMailbox* mailbox = nullptr;
  // Several ranks, seeded without a collective: every rank's replicated
  // degree array (deg_all, the global source id src_global) gives the seed's
  // global totals, so with ctrl / mailbox set each rank finishes the seed
  // itself -- the source's bit set in its replicated visited bitmap, and
  // (frontier_global, a bottom-up first level) the whole global seed
  // frontier written locally instead of all-gathered.
  const uint32_t* deg_all = nullptr;
  int64_t src_global = -1;
  word_t* frontier_global = nullptr;
};

// Multi-block exclusive scan of unit_cnt / unit_deg (in place, per chunk of
// kScanChunk units) plus chunk prefixes (part_cnt / part_deg, exclusive).  The
// last workgroup to finish (ticket, agent-scope release/acquire) scans the
// chunk totals and writes stats[0..1] = stats[2..3] = (count, degree sum) and
// the work-list end sentinel qscan[count] = degree sum.
struct ScanArgs {
  int64_t* unit_cnt = nullptr;
  int64_t* unit_deg = nullptr;
  int64_t nunits = 0;
  int64_t* part_cnt = nullptr;   // ceil(nunits / kScanChunk)
  int64_t* part_deg = nullptr;
  unsigned* ticket = nullptr;    // zero before the first launch; reset by the last block
  int64_t* stats = nullptr;
  int64_t* qscan = nullptr;
  // device-driven loop: skip everything when ctrl->done at entry; the last
  // workgroup runs level_ctrl_finish and fills rec / the mailbox slot
  LevelCtrl* ctrl = nullptr;
  LevelRecDev* rec = nullptr;       // this level's record
  LevelMailbox* mailbox = nullptr;  // device-mapped pinned slot
  int32_t level = 0;
  bool seed = false;
  // Device loop: the level's chain was enqueued for this direction (0: any);
  // when ctrl->dir differs, the chain was a no-op and so is the scan.
  int32_t expect_dir = 0;
  // ... and, for a multi-rank list-form top-down chain, only valid while the
  // level's global frontier edges fit its lists (ctrl->m_f <= expect_cap;
  // 0: no bound).
  int64_t expect_cap = 0;
  // Device loop: run level_ctrl_finish here (one rank); several ranks reduce
  // the totals first and finish in level_finish.
  bool finish = true;
};

// Device loop, several ranks: after the totals' all-reduce (stats[2..3] =
// global count / degree sum), one thread runs level_ctrl_finish (seed: from
// ctrl_init) and stamps rec / the mailbox, as the one-rank scan does.
struct LevelFinishArgs {
  const int64_t* stats = nullptr;
  LevelCtrl* ctrl = nullptr;
  LevelCtrl ctrl_init;
  LevelRecDev* rec = nullptr;
  LevelMailbox* mailbox = nullptr;
  int32_t level = 0;
  bool seed = false;
  int32_t expect_dir = 0;
  int64_t expect_cap = 0;  // see ScanArgs::expect_cap
};

// A device-loop chain's kernels run only when the chain is live: the level is
// not done, its direction is the one the chain was enqueued for, and (list-form
// top-down chains) the global frontier edges fit the chain's lists.
DBFS_HD bool chain_live(const LevelCtrl& c, int32_t dir, int64_t cap) {
  return !c.done && (dir == 0 || c.dir == dir) && (cap <= 0 || c.m_f <= cap);
}

// Host-loop statistics mailbox (pinned, device-mapped).  After a level's
// totals are final (scan, plus the all-reduce on several ranks) one tiny
// kernel copies stats[0..3] here with system-scope stores and then writes
// `seq` with release semantics; the host spins on `seq`.  This replaces a
// D2H copy + stream synchronisation per level (a copy-engine round trip and a
// host wake-up) by a store the spinning host sees within a microsecond.
struct StatsMailbox {
  int64_t seq = 0;
  int64_t v[4] = {0, 0, 0, 0};
};

// Owned frontier bitmap -> load-balanced top-down work list:
// qscan[i] = exclusive prefix of degrees, qbase[i] = row_off[v_i] - qscan[i],
// blk_vstart[b] = index of the entry covering edge b * kTdEdgesPerBlock.
struct CompactArgs {
  ShardView g;
  const word_t* frontier = nullptr;
  int64_t words = 0;
  const int64_t* unit_cnt_off = nullptr;  // scanned (in-chunk) unit offsets
  const int64_t* unit_deg_off = nullptr;
  const int64_t* part_cnt = nullptr;      // chunk prefixes
  const int64_t* part_deg = nullptr;
  int64_t* qscan = nullptr;
  int64_t* qbase = nullptr;
  int32_t* blk_vstart = nullptr;
  vid_t* qv = nullptr;              // optional: work-list entry -> vertex (local row)
  word_t* clear = nullptr;          // optional: zero the frontier words once read (== frontier)
  // optional: zero every word of this bitmap (a sparse level after a
  // bottom-up one writes its output into the bottom-up level's input)
  word_t* clear_all = nullptr;
  const LevelCtrl* ctrl = nullptr;  // device loop: runs only when ctrl->dir == 'T'
  int64_t max_mf = 0;               // ... and ctrl->m_f <= max_mf (0: any; a sparse chain's compaction)
};

// Sparse top-down level (device loop, one rank): one kernel instead of
// compact + td_expand + update + scan.  Expands the work list (qscan / qbase /
// blk_vstart / qv, totals in dev_stats[0..1]) edge-balanced like td_expand,
// claims each new vertex with a fetch-or on `visited`, writes its level, sets
// its bit in frontier_out (clean on entry) and appends it -- wave-aggregated,
// one packed atomic (count << kSparseEdgeBits | edges) per wave, so entries
// stay ordered by edge offset -- to the output work list (oscan / obase / oblk
// / oqv) the next level expands directly.  The input vertices' bits are
// cleared from frontier_in (keeps the bitmap the next sparse level writes
// clean).  The last workgroup publishes the totals (stats[0..3], oscan[q]),
// runs level_ctrl_finish and stamps rec / the mailbox like the scan.
constexpr int kSparseEdgeBits = 36;
// Direct exchanges (peer transport, Comm::direct_lists / direct_level_end):
// the kernels themselves move the data through the peers' windows, no
// exchange launch.  Every signal is a tagged cell of two 64-bit words in the
// receiver's window -- each word carries the exchange's sequence number next
// to its payload, so one write-through store publishes it and one poll both
// observes it and delivers the payload:
//   owner lists  word 0 = seq32 << 32 | count (the ids are in the slot,
//                stored and drained before the cell)
//   level end    word 0 = seq32 << 32 | new vertices (< 2^32 per rank),
//                word 1 = seq24 << 40 | their degree sum (< 2^40 per rank)
// The cells sit in the window's flag page, apart from every other
// collective's payload: a stale cell holds an older sequence number.
constexpr int kMaxDirectRanks = 16;
// Where the data goes and comes from, in device memory (the kernels index it
// with a wave-uniform rank): one table per window parity.
struct DirectTable {
  uint32_t* dst[kMaxDirectRanks];            // rank p's window slot for this rank (ids from word 1; [rank]: unused)
  uint64_t* cell_out[kMaxDirectRanks];       // rank p's cell for this rank ([rank]: unused)
  const uint32_t* src[kMaxDirectRanks];      // this rank's window slot of sender p
  const uint64_t* cell_in[kMaxDirectRanks];  // this rank's cell of sender p ([rank]: unused)
};
// Frontier slices pushed by the kernels that produce them (several ranks,
// peer transport, Comm::direct_frontier): each output word also goes,
// write-through, to every peer's window buffer for this rank's slice
// (dst[p]), and the next level's hub_gather copies the peers' slices from
// this rank's window (src[p]) into its global frontier -- the all-gather
// rides the producing kernel instead of a collective after it.  One table per
// buffer parity (the producing level's parity: a peer writes level L + 2's
// slice only after level L + 1's end, which this rank reaches after it has
// copied level L's); [rank] unused.
struct FrontierTable {
  uint64_t* dst[kMaxDirectRanks];
  const uint64_t* src[kMaxDirectRanks];
};

// A timed-out device wait's error word: the collective's sequence number
// (low 48 bits) and 1 + the peer it found missing (bits 48..55; 0: unknown).
constexpr uint64_t kWaitSeqMask = (uint64_t(1) << 48) - 1;

struct DirectExchange {
  int active = 0;  // 0: the exchange goes through a Comm collective instead
  int nranks = 1, rank = 0;
  uint64_t seq = 0;                     // this exchange's sequence number (the cells' tag)
  const DirectTable* table = nullptr;   // device memory
  uint64_t timeout_ticks = 0;           // a wait gives up after this many wall-clock ticks
  uint64_t* error = nullptr;            // ... and stores kWaitSeqMask & seq | (peer + 1) << 48 here (the host watches it)
  // a level end: the all-reduced totals as recorded (shadow replay) instead
  // of the peers' cells summed
  const int64_t* result = nullptr;
};

// new = (OR_r cand[r * cand_stride + w]) & ~visited[w] over the owned slice
// (force: new = cand, used to seed the source):  visited |= new;
// frontier = new; level[v] = new_level for v in new; unit_cnt[u] / unit_deg[u]
// = count / degree-sum of new vertices with degree > 0.  clear_cand zeroes the
// consumed cand words (single-chunk top-down: keeps `next` clean).
struct UpdateArgs {
  ShardView g;
  word_t* cand = nullptr;
  // Byte-map candidates (one byte per vertex, 0/1) instead of `cand`: used
  // after a byte-map top-down step on one rank; the bytes are cleared.
  uint8_t* cand_bytes = nullptr;
  int nchunks = 1;
  int64_t cand_stride = 0;       // words between chunks
  bool clear_cand = false;
  bool force = false;
  word_t* visited = nullptr;     // owned slice of the global visited bitmap
  word_t* frontier = nullptr;    // owned slice of the NEXT global frontier bitmap
  lvl_t* level = nullptr;        // rows
  uint8_t* level8 = nullptr;     // narrow levels (see InitRunArgs)
  uint8_t narrow_base = 0;             // narrow level bytes of this run: base + level (kNarrowEpochs)
  lvl_t new_level = 0;
  int64_t words = 0;             // words of the owned slice
  int64_t* unit_cnt = nullptr;   // nunits
  int64_t* unit_deg = nullptr;   // nunits
  // Device loop: runs only when ctrl->dir == 'T'; reads cand_bytes when
  // ctrl->bytes, else cand (both given).
  const LevelCtrl* ctrl = nullptr;
  int64_t max_mf = 0;  // list-form chain: live only while ctrl->m_f <= max_mf
  // With the byte-map levels of TdArgs::level_direct: candidates are the
  // unvisited vertices whose level already reads new_level (level8, padded to
  // whole words); cand_bytes is not read.
  const uint8_t* level_direct = nullptr;
  // One rank, device loop (as BuArgs::fuse_scan): totals and finish in the
  // last-arriving workgroup, unit statistics left unscanned (a following
  // compaction scans them first); tot[0..1] zero, reset by the last one.
  bool fuse_scan = false;
  // ... and (graphs of at most kFoldScanUnits units) the unit prefixes the
  // next compaction reads, scanned by the same last workgroup -- no
  // scan_units launch between the levels (the unit statistics are stored
  // write-through and read with agent-scope loads, as the totals)
  bool fold_scan = false;
  ScanArgs scan;
  int64_t* tot = nullptr;
  // ... with the ticket two-level: workgroups of kFusedGroup consecutive ids
  // share a group ticket (kBuQueueStride apart, zero between launches; the
  // group's last workgroup re-zeroes it, sums the group's slots into
  // tot[2 kMaxFusedGrid + 2 g] and takes the level ticket), so the grid can
  // be large without thousands of same-address atomics.  Null: one ticket
  // (grid capped at kMaxFusedGrid / 8).
  unsigned* group_ticket = nullptr;
  // several ranks: the new frontier words also pushed to the peers (FrontierTable)
  const FrontierTable* push = nullptr;
  int push_rank = 0, push_nranks = 1;
  // several ranks: the send buffer of the candidates' all-to-all (zero_slices
  // slices of `words` words) zeroed here -- word w of every slice by the lane
  // of w -- instead of a memset launch after the exchange
  word_t* zero_next = nullptr;
  int zero_slices = 0;
  // several ranks, fused finish: the level's end in the last workgroup
  // (Comm::direct_level_end; no frontier gathered, or a pushed one); it runs
  // on a no-op chain too (a collective)
  DirectExchange end;
  LevelFinishArgs fin;
};

struct TdSparseArgs {
  ShardView g;
  const int64_t* qscan = nullptr;
  const int64_t* qbase = nullptr;
  const int32_t* blk_vstart = nullptr;
  const vid_t* qv = nullptr;
  const int64_t* dev_stats = nullptr;  // [0] entries, [1] edges of the input list
  word_t* frontier_in = nullptr;       // owned slice
  word_t* frontier_out = nullptr;      // owned slice, zero on entry
  word_t* visited = nullptr;           // global
  lvl_t* level = nullptr;              // rows
  uint8_t* level8 = nullptr;           // narrow levels (see InitRunArgs)
  uint8_t narrow_base = 0;             // narrow level bytes of this run: base + level (kNarrowEpochs)
  int32_t new_level = 0;
  int64_t* oscan = nullptr;
  int64_t* obase = nullptr;
  int32_t* oblk = nullptr;
  vid_t* oqv = nullptr;
  unsigned long long* counter = nullptr;  // zero on entry; reset by the last workgroup
  unsigned* ticket = nullptr;             // zero on entry; reset by the last workgroup
  int64_t* stats = nullptr;
  LevelCtrl* ctrl = nullptr;
  LevelRecDev* rec = nullptr;
  LevelMailbox* mailbox = nullptr;
  int32_t level_index = 0;
  int64_t grid = 0;
  bool first = true;  // first kernel of the level (else a compaction ran before it)
  // live only while ctrl->m_f <= max_mf (0: any): a sparse chain enqueued for
  // a level that turns out large is a no-op and is re-enqueued dense
  int64_t max_mf = 0;
  // from_bits (a level right after a bottom-up one): the input frontier is the
  // bitmap frontier_in itself (`words` owned words, zeroed as read), not a
  // work list -- no unit scan, no compaction; qscan / qbase / blk_vstart / qv /
  // dev_stats are unused and frontier_out must be zero on entry.  The kernel's
  // workgroups end on a two-level ticket (group_ticket: kFusedGroups tickets
  // kBuQueueStride apart, zero between launches).
  bool from_bits = false;
  int64_t words = 0;
  // Fault injection (DBFS_FAULT_INJECT=kind=late_wg): the workgroups that
  // take no ticket (blockIdx >= the level's active count) first wait this
  // many wall-clock ticks, so they start after the level's last workgroup has
  // finished it -- the dispatch order a busy or cold GPU can produce.  0: off.
  uint64_t late_ticks = 0;
  // Several ranks, direct exchange with a folded level end, a tiny level:
  // td_sparse's last workgroup publishes the lists and then runs the owner
  // side itself (td_sparse_apply's work on one workgroup: nranks, end, fin
  // set) -- one launch per level instead of two.
  bool fuse_apply = false;
  unsigned* group_ticket = nullptr;
  // Several ranks: every target is claimed in the replicated `visited`
  // (fetch-or); an owned one is finished here, a remote one appended to its
  // owner's list (lists + owner * list_stride: count, then the ids; wave-
  // aggregated) -- claiming the remote bit too sends each target at most once
  // per rank.  The lists then travel (Comm::alltoall_lists) and
  // td_sparse_apply claims the received ids on their owner.  Only the apply
  // kernel finishes the level (totals to stats, no decision: the totals are
  // all-reduced first); with lists == nullptr td_sparse finishes it (one rank).
  vid_t* lists = nullptr;
  int64_t list_stride = 0;   // 32-bit words per owner list (count included)
  int64_t part = 0;          // vertices per rank (owner = v / part)
  // td_sparse_apply: the received lists (same layout, nranks of them) and the
  // send lists whose counts it zeroes for the next list level
  const vid_t* recv_lists = nullptr;
  int nranks = 1;
  // direct.active: the lists go straight into the owners' windows (td_sparse)
  // and are read from this rank's window (td_sparse_apply, after the flags)
  DirectExchange direct;
  // end.active (td_sparse_apply, several ranks): the level's end folded into
  // its last workgroup -- the totals (stats[2..3]) pushed to every peer's
  // window, the peers' awaited and summed, then the decision (`fin`), as
  // Comm::level_end without a frontier gather; no collective launch after.
  DirectExchange end;
  LevelFinishArgs fin;
};

// Binned top-down level (one rank, large frontiers; propagation blocking):
// instead of a random probe and a random store per frontier edge, the edges'
// targets are first written into nbins contiguous bins by target range
// (count pass: per-workgroup bin counts; scan; fill pass: each workgroup
// writes its targets at its scanned positions), then one workgroup per bin
// holds the bin's slice of `visited` in LDS, claims the unvisited targets with
// LDS atomics and writes the bin's frontier / visited words, the new
// vertices' levels and its units' statistics -- every random access of the
// level lands in one bin's LDS / L2-resident range.  Replaces td_expand; an
// update_frontier with force = true over the new frontier (cand = frontier)
// then writes the levels and unit statistics.  Correct for any frontier size.
struct BinArgs {
  ShardView g;
  const int64_t* qscan = nullptr;
  const int64_t* qbase = nullptr;
  const int32_t* blk_vstart = nullptr;
  const int64_t* dev_stats = nullptr;  // [0] work-list entries, [1] frontier edges
  // work list handed over by a sparse level: zero its vertices' input bits
  const vid_t* clear_qv = nullptr;
  word_t* clear_frontier = nullptr;
  const LevelCtrl* ctrl = nullptr;     // runs only when ctrl->dir == 'T'
  int shift = 12;                      // bin = vertex >> shift (bins align with 4096-vertex units)
  int nbins = 0;
  int grid = 0;                        // workgroups of the count / fill passes
  // count pass: cnt[k * grid + g] = targets of bin k in workgroup g's edges;
  // the scan (one workgroup per bin) makes each bin's row exclusive and sets
  // bin_total[k]; the fill pass and the apply derive the bin starts from
  // bin_total themselves
  uint32_t* cnt = nullptr;             // nbins * grid
  int64_t* bin_total = nullptr;        // nbins
  vid_t* buf = nullptr;                // >= frontier edges
  word_t* visited = nullptr;
  word_t* frontier = nullptr;          // next frontier (every word written)
  int64_t words = 0;
};
// Largest bin span (vertices) and bin count the kernels support.
constexpr int kBinMaxShift = 18;
constexpr int kBinMaxBins = 2048;

// For every edge (u, v) with u in the work list and v not visited: next[v] = 1.
struct TdArgs {
  ShardView g;
  const int64_t* qscan = nullptr;
  const int64_t* qbase = nullptr;
  const int32_t* blk_vstart = nullptr;
  int64_t q = 0;        // work-list entries
  int64_t m = 0;        // work-list edges (qscan[q])
  const word_t* visited = nullptr;  // global
  word_t* next = nullptr;           // global
  // Byte-map mode (large levels): next_bytes[v] = 1 with a plain byte store
  // instead of a scattered 64-bit atomicOr on next (the atomics bound the
  // top-down rate at ~40 G edges/s on MI355X).
  uint8_t* next_bytes = nullptr;
  // List mode (small levels, multi-rank): candidate v is appended to its
  // owner's list lists[o * (list_cap + 1) + 1 + k]; slot 0 of each list is its
  // count (wave-aggregated atomics, at most nranks per wave instruction).
  // list_cap >= global frontier edges guarantees no overflow.
  vid_t* lists = nullptr;
  int64_t list_cap = 0;
  int64_t part = 0;   // owner(v) = v / part
  // Byte mode only: skip the visited pre-check (few vertices visited yet).
  bool check_visited = true;
  // One rank, narrow levels, byte-map levels: instead of marking next_bytes,
  // store new_level straight into the level array of every unvisited
  // candidate (plain byte stores; the visited check is then always made) --
  // update_frontier(level_direct) derives the new frontier from it, nothing to
  // clear afterwards.
  uint8_t* level_direct = nullptr;
  lvl_t new_level = 0;
  uint8_t narrow_base = 0;  // (level_direct stores narrow_base + new_level)
  // Levels of at least td_hub_min_edges frontier edges read g.td_col and test
  // hub targets in an LDS copy of td_hub_vis (visited bits of the top-down
  // hubs, this level's snapshot: hub_visited); not with owner lists.
  const word_t* td_hub_vis = nullptr;
  int64_t td_hub_min_edges = 0;
  // ... and only once the visited vertices hold this fraction of all
  // adjacency entries (device loop: ctrl->vis_deg; earlier, most hub
  // targets are unvisited and decoding them costs a dependent load)
  double td_hub_vis_frac = 0.0;
  // With the filter and level_direct: a hub target unvisited at the level's
  // start is claimed by a byte store here (kTdMaxHubs bytes, L2-resident,
  // no decode of the hub id) instead of a level byte store scattered over
  // the whole level array; hub_apply turns the marks into level bytes.
  uint8_t* td_hub_mark = nullptr;
  // Unvisited filter (UnvisArgs, this level's snapshot): targets whose bit is
  // clear are visited without a `visited` probe (device loop, Dyn output; a
  // 1024-thread variant without the hub filter)
  const word_t* unvis = nullptr;
  uint64_t unvis_mult = 0;
  // ... its chunks' set bits (UnvisArgs::pop): the filter variant and the
  // plain one are both launched, and the level runs in the filter variant
  // iff at most unvis_max_density of the filter's bits are set
  const uint32_t* unvis_pop = nullptr;
  double unvis_max_density = 0.5;
  // Launch 1024-thread workgroups when the grid has fewer blocks than this.
  int64_t wide_below_blocks = 0;
  // Device loop: q / m come from dev_stats[0..1], bits vs bytes and the
  // visited pre-check from ctrl; the fixed grid loops over the edge blocks.
  const LevelCtrl* ctrl = nullptr;
  const int64_t* dev_stats = nullptr;
  int64_t grid = 0;
  int64_t grid_filter = 0;  // ... for the hub-filter variant (0: grid)
  // Device loop, work list handed over by a sparse level (no compaction ran):
  // zero the input vertices' words of clear_frontier (clear_qv: entry -> row).
  const vid_t* clear_qv = nullptr;
  word_t* clear_frontier = nullptr;
  // Device loop, several ranks, list form (`lists` set): live only while the
  // global frontier edges ctrl->m_f <= max_mf (= list_cap: no list can
  // overflow, every rank decides alike); else a no-op the host re-enqueues.
  int64_t max_mf = 0;
  // Split level (one rank, level_direct): this launch runs part split_i of
  // split_k equal runs of the level's edge blocks; between parts
  // refresh_visited ORs the vertices claimed so far into `visited`, so a
  // later part's probes skip them instead of storing their level byte again.
  int split_k = 1, split_i = 0;
};

// A split top-down level (TdArgs::split_k): visited |= the vertices whose level
// byte is narrow_base + new_level (claimed by the parts so far).  words:
// visited words (level8 holds 64 x words bytes).
struct RefreshArgs {
  const uint8_t* level8 = nullptr;
  uint8_t narrow_base = 0;
  lvl_t new_level = 0;
  word_t* visited = nullptr;
  int64_t words = 0;
  const LevelCtrl* ctrl = nullptr;
  int64_t max_mf = 0;  // chain predicate, as TdArgs::max_mf
};

// Received candidate lists (nranks lists of list_cap + 1 words, count first)
// -> bits in cand (owned slice), local index v - lo.
struct ListScatterArgs {
  const vid_t* lists = nullptr;
  int nranks = 1;
  int64_t list_cap = 0;
  int64_t lo = 0;
  word_t* cand = nullptr;
  int64_t words = 0;  // words of cand (bounds check of the checked build; 0: unchecked)
  // Device loop: the send lists' counts to zero once the exchange has read
  // them (the next list-form chain appends from zero), and the chain guard.
  vid_t* reset_lists = nullptr;
  const LevelCtrl* ctrl = nullptr;
  int64_t max_mf = 0;
};

// next[w] |= bits of bytes[64 w .. 64 w + 63]; bytes cleared (multi-rank
// byte-map top-down: the exchange stays a bitmap all-to-all).
struct PackArgs {
  uint8_t* bytes = nullptr;
  word_t* next = nullptr;
  int64_t words = 0;
  // device loop: runs only on a byte-map top-down level (ctrl->bytes) --
  // or, with `flag`, on a live bottom-up level whose *flag is set (the
  // several-rank hub cut's remote claims, BuArgs::cut_bytes)
  const LevelCtrl* ctrl = nullptr;
  const int* flag = nullptr;
  // words [skip_begin, skip_end) are left alone (the hub cut: this rank's own
  // slice, whose claims never go through the byte map)
  int64_t skip_begin = 0, skip_end = 0;
};

// Bottom-up step fused with the frontier update: for every owned unvisited v,
// if some neighbour u has frontier[u], v joins the new frontier: visited[v],
// new_frontier[v], level[v] = new_level, unit stats as in UpdateArgs.
// Slots of BuArgs::tot (one pair per workgroup of a fused bottom-up finish).
constexpr int kMaxFusedGrid = 4096;
// Group tickets kBuQueueStride uints apart (one 128-B line each: counters
// sharing a line serialise their atomics).
constexpr int kBuQueueStride = 32;
// Fused update finish, two-level ticket (UpdateArgs::group_ticket).
constexpr int kFusedGroup = 64;
constexpr int kFusedGroups = kMaxFusedGrid / kFusedGroup;

struct BuArgs {
  ShardView g;
  // Zero-degree / padding bits of the owned slice (needed with g.nz_pref).
  const word_t* zdeg = nullptr;
  // Hub frontier bits (g.nhubs bits, from hub_gather), staged in LDS.
  const word_t* hub_front = nullptr;
  word_t* visited = nullptr;         // owned slice
  const word_t* frontier = nullptr;  // current frontier, global
  word_t* new_frontier = nullptr;    // owned slice of the next frontier (fully overwritten)
  lvl_t* level = nullptr;
  uint8_t* level8 = nullptr;         // narrow levels (see InitRunArgs)
  uint8_t narrow_base = 0;             // narrow level bytes of this run: base + level (kNarrowEpochs)
  lvl_t new_level = 0;
  int64_t words = 0;
  int lane_limit = 32;               // neighbours scanned per lane before wave cooperation
  bool follow_up = false;            // the previous level was bottom-up too (launch shape)
  int whole_units = 0;               // hub kernel, compacted: 64 words per wave (1), 16 (-1), by shard size (0)
  int small_waves = 0;               // ... split units: 4 words per wave on a first level (1), never (-1), by shard size (0)
  int64_t* unit_cnt = nullptr;
  int64_t* unit_deg = nullptr;
  const LevelCtrl* ctrl = nullptr;   // device loop: runs only when ctrl->dir == 'B'
  // One rank, device loop: the level's totals and finish (ScanArgs: stats,
  // direction decision, record, mailbox) run in the bottom-up kernel's
  // last-arriving workgroup instead of a scan launch: workgroup g stores its
  // totals in tot[2g], tot[2g + 1] (kMaxFusedGrid slots).  The per-unit
  // prefixes are left to a scan_units (finish off) in the next chain, only
  // when it compacts the frontier (a top-down level).  Kernels without the
  // epilogue launch scan_units after themselves.
  bool fuse_scan = false;
  ScanArgs scan;
  int64_t* tot = nullptr;
  // several ranks, fuse_scan: the level's end folded into the last
  // workgroup (Comm::direct_level_end; no frontier gather), as td_sparse_apply
  DirectExchange end;
  LevelFinishArgs fin;
  // Hub-cut level (one rank, narrow levels, hub kernels with packed records,
  // cut_edges > 0; bu_cut_prep before it): when the level's frontier edges
  // outside the hubs -- ctrl->m_f minus the frontier hubs' degrees -- are at
  // most cut_edges, hub_gather sets *cut_flag and bu_cut_prep writes the level
  // byte of the non-hub frontier vertices' unvisited neighbours (top-down);
  // every row scan of the level then stops at its first non-hub neighbour (a
  // hub-first row's later neighbours cannot be in the frontier: rows with a
  // non-hub frontier neighbour were claimed).  Claimed vertices (unvisited,
  // level byte = this level) skip the scan and join the output with the
  // found ones.  *cut_flag = 0: a plain level.  Wide (32-bit) levels: the
  // claims are non-zero bytes of cut_claim (one per vertex, all zero between
  // levels), which the bottom-up kernel clears as it writes their levels.
  int64_t cut_edges = 0;
  int* cut_flag = nullptr;
  uint8_t* cut_claim = nullptr;
  // ... several ranks (bu_cut_prep): this rank's non-hub frontier is the
  // global frontier's words [cut_word_off, + words); a neighbour is skipped
  // when its bit in cut_vis (the replicated global visited bitmap) is set;
  // an owned one is claimed as above, a remote one gets its byte of
  // cut_bytes (the global byte map, packed per owner and all-to-all'ed).
  // bu_cut_merge then claims the received words (cut_recv: P slices of
  // `words`, this rank's own empty) and zeroes cut_next (the packed bitmap,
  // P slices) for the next user.
  uint8_t* cut_bytes = nullptr;
  const word_t* cut_vis = nullptr;
  int64_t cut_word_off = 0;
  const word_t* cut_recv = nullptr;
  word_t* cut_next = nullptr;
  int cut_rank = 0, cut_nranks = 1;
  // several ranks: the new frontier words also pushed to the peers (FrontierTable)
  const FrontierTable* push = nullptr;
  int push_rank = 0, push_nranks = 1;
};

// out bit h = visited bit of g.td_hub_vertex[h] (visited global): the
// snapshot a top-down level filters hub targets with; device loop: runs only
// when ctrl->dir == 'T' (and ctrl->m_f >= min_edges).
struct HubVisitedArgs {
  ShardView g;
  const word_t* visited = nullptr;
  word_t* out = nullptr;
  const LevelCtrl* ctrl = nullptr;
  int64_t min_edges = 0;
  double vis_frac = 0.0;  // as TdArgs::td_hub_vis_frac
};

// A dense top-down level's unvisited filter (this level's snapshot): bit i
// is set iff some vertex v with unvis_index(v) == i is unvisited, where
// unvis_index(v) = (v * mult) >> 32 maps the n vertices onto kUnvisBits bits
// in contiguous runs (mult = unvis_mult(n): at most 2^32, identity for n <=
// kUnvisBits).  td_expand (TdArgs::unvis) stages it in LDS and probes
// `visited` only for targets whose filter bit is set: late levels, where most
// targets are visited, trade most scattered L2 requests for LDS reads.
// 7104 words: with td_expand's owner map of two edge blocks (kUnvisSpan,
// 16-bit entries) two 1024-thread workgroups fill a CU's 160 KiB of LDS.
// Built in chunks of 64 words (kUnvisChunks), each chunk's set bits counted
// (UnvisArgs::pop).
constexpr int64_t kUnvisWords = 7104;
constexpr int64_t kUnvisBits = kUnvisWords * 64;
constexpr int kUnvisChunks = static_cast<int>(kUnvisWords / 64);
constexpr int kUnvisSpan = 2;
DBFS_HD uint64_t unvis_mult(int64_t n) {
  if (n <= kUnvisBits) return uint64_t(1) << 32;
  return (static_cast<uint64_t>(kUnvisBits) << 32) / static_cast<uint64_t>(n);
}
DBFS_HD uint32_t unvis_index(uint64_t v, uint64_t mult) { return static_cast<uint32_t>((v * mult) >> 32); }
// the first vertex with unvis_index >= i
DBFS_HD uint64_t unvis_first(uint64_t i, uint64_t mult) { return ((i << 32) + mult - 1) / mult; }
struct UnvisArgs {
  const word_t* visited = nullptr;  // global (n bits)
  int64_t n = 0;
  uint64_t mult = 0;
  word_t* out = nullptr;            // kUnvisWords
  uint32_t* pop = nullptr;          // kUnvisChunks: set bits per 64-word chunk
  const LevelCtrl* ctrl = nullptr;
  int64_t max_mf = 0;               // chain predicate, as TdArgs::max_mf
};

// level8[td_hub_vertex[h]] = narrow_base + new_level
// for every h with mark[h] != 0, which is cleared: td_expand's hub claims
// (TdArgs::td_hub_mark).  mark holds kTdMaxHubs bytes.
struct HubApplyArgs {
  ShardView g;
  uint8_t* mark = nullptr;
  uint8_t* level8 = nullptr;
  uint8_t narrow_base = 0;
  lvl_t new_level = 0;
  const LevelCtrl* ctrl = nullptr;
  int64_t max_mf = 0;  // chain predicate, as TdArgs::max_mf
};

// hub_gather copies (visited merge, pushed slices) with at most this many
// workgroups (the hub-cut part sums are sized for it)
constexpr int kHgCopyGrid = 512;

// hub_front bit h = frontier bit of g.hub_vertex[h] (frontier global); in the
// device loop only when ctrl->dir == 'B'.
struct HubGatherArgs {
  ShardView g;
  const word_t* frontier = nullptr;
  word_t* hub_front = nullptr;  // ceil(nhubs / 64) words
  const LevelCtrl* ctrl = nullptr;
  // several ranks: visited[0, words) |= frontier (the all-gathered remote
  // slices into the replicated visited bitmap) in the same launch
  word_t* visited = nullptr;
  int64_t words = 0;
  // hub-cut levels (BuArgs::cut_edges): cut_part[b] = the summed degrees of
  // the frontier hubs of workgroup b (kBlock hubs each); the last workgroup
  // (cut_ticket, zero between levels) stores the decision in *cut_flag
  int64_t* cut_part = nullptr;
  int64_t cut_edges = 0;
  int* cut_flag = nullptr;
  unsigned* cut_ticket = nullptr;
  // several ranks, the previous level's slices pushed (FrontierTable): the
  // peers' slices copied from this rank's window into pull_out (the global
  // frontier; `words` per slice) -- and merged into visited with `visited` --
  // and the hubs' bits read from their owners' slices directly
  const FrontierTable* pull = nullptr;
  word_t* pull_out = nullptr;
  int pull_rank = 0, pull_nranks = 1;
  int64_t pull_words = 0;
};

// Bits of the owned slice for vertices with degree 0 or beyond the shard
// (padding): they can never be discovered, so they start out "visited".
struct ZeroDegArgs {
  ShardView g;
  word_t* out = nullptr;  // owned slice
  int64_t words = 0;
  bool padding_only = false;  // directed graphs: only the padding past the shard
};

// Vertex-centric ("status array") top-down: every owned v with level[v] == cur
// marks its unvisited neighbours in next.  (The reference's simple/multiBfs
// variant, bfs.cu:101-130, made race-free.)
struct StatusArgs {
  ShardView g;
  const lvl_t* level = nullptr;
  lvl_t cur = 0;
  const word_t* visited = nullptr;  // global
  word_t* next = nullptr;           // global
};

// Reference-algorithm mode (bfs.cu:134-165): thread per frontier vertex,
// atomicMin claim on a replicated distance array, one atomic counter per owner
// bucket.
struct RefExpandArgs {
  ShardView g;
  const vid_t* queue = nullptr;  // global ids of owned frontier vertices
  int64_t q = 0;
  lvl_t next_level = 0;
  lvl_t* dist = nullptr;         // replicated, n entries
  int64_t part = 0;              // owner(v) = v / part
  int64_t* bucket_cnt = nullptr; // nranks
  vid_t* buckets = nullptr;      // nranks * bucket_cap
  int64_t bucket_cap = 0;
};

// Received ids: entries in [self_begin, self_end) were claimed locally and are
// kept; the others are kept iff this rank's atomicMin claim succeeds.  Kept ids
// are appended to queue (counter *qcount).
struct RefAcceptArgs {
  const vid_t* recv = nullptr;
  int64_t total = 0;
  int64_t self_begin = 0, self_end = 0;
  lvl_t next_level = 0;
  lvl_t* dist = nullptr;
  vid_t* queue = nullptr;
  int64_t* qcount = nullptr;
};

// Scan-mode BFS (the reference's single-GPU "scan" pipeline nextLayer /
// countDegrees / scanDegrees / assignVerticesNextQueue, bfs.cu:706-781 and
// H16c in SURVEY.md): an atomic-free frontier build.  relax writes
// dist[v] = next_level and claim[v] = e (shard-local edge index, last writer
// wins) with plain stores; count gives every frontier vertex i, per owner o,
// the number of edges e it won (offs[o * q + i]); an exclusive scan turns the
// counts into an owner-major output layout; assign writes the children there.
struct ScanBfsArgs {
  ShardView g;
  const vid_t* queue = nullptr;  // global ids of owned frontier vertices
  int64_t q = 0;
  lvl_t next_level = 0;
  lvl_t* dist = nullptr;         // replicated, n entries
  eid_t* claim = nullptr;        // replicated, n entries (no reset needed)
  int64_t part = 0;              // owner(v) = v / part
  int nranks = 1;
  eid_t* offs = nullptr;         // nranks * q + 1 entries
  eid_t* bounds = nullptr;       // scan_bounds: offs[o * q] for o in [0, nranks]
  int64_t* counts = nullptr;     // scan_bounds: per-owner child counts
  vid_t* out = nullptr;          // children, owner-major
};

// Graph500-style validation of a full level array against a shard: counts
// violations of (a) |level[u] - level[v]| <= 1 over every edge with both ends
// reached, (b) reached-unreached edges, (c) reached v != src without a
// neighbour at level[v] - 1.  out[0..2] += counts.
struct ValidateArgs {
  ShardView g;
  const lvl_t* level_global = nullptr;  // n entries
  int64_t src = 0;
  int64_t* out = nullptr;               // 3 counters (device)
};

// Graph500 parent tree from levels: parent[v] = first neighbour u with
// level[u] == level[v] - 1 (global vertex id), parent[src] = src, -1 if
// unreached.  Computed after a run from the all-gathered level array.
struct ParentArgs {
  ShardView g;
  const lvl_t* level_global = nullptr;  // n entries
  int64_t src = 0;
  int64_t* parent = nullptr;            // rows (owned slice)
};

// ---- backend ----------------------------------------------------------------

class Backend {
 public:
  virtual ~Backend() = default;
  virtual DeviceKind kind() const = 0;
  virtual std::string name() const = 0;
  virtual int device_id() const { return -1; }
  virtual void* stream_handle() { return nullptr; }
  // Communication stream.  Collectives are enqueued on comm_stream_handle():
  // the compute stream itself, unless a side region is open.  fork_side()
  // makes the side stream wait for everything enqueued on the compute stream
  // so far and routes the following collectives to it, so kernels enqueued
  // meanwhile overlap them; join_side() makes the compute stream wait for the
  // side stream's work and routes collectives back.  (CPU: no-ops.)
  virtual void* comm_stream_handle() { return stream_handle(); }
  virtual void fork_side() {}
  virtual void join_side() {}
  // Rate of the device wall clock the kernels stamp level records with (ticks
  // per ms; 0: no device clock, records carry no times).
  virtual double wall_clock_khz() const { return 0.0; }

  // Host waits on the device (to_host, to_device, synchronize) call
  // watch(seconds waited) about every period_s while the stream is still busy;
  // the watch may throw to abandon the wait.  A communicator installs one to
  // turn a dead peer into an error instead of a hang.
  const std::function<void(double)>& wait_watch() const { return wait_watch_; }
  void set_wait_watch(std::function<void(double)> watch, double period_s = 0.05) {
    wait_watch_ = std::move(watch);
    wait_period_ = period_s;
  }

  // memory (alloc/free are synchronous; copies/memsets are stream-ordered)
  virtual void* alloc(size_t bytes) = 0;
  virtual void dealloc(void* p) = 0;
  // Device and mapped frees held until the backend is destroyed (HIP: several
  // ranks of one process sharing a device -- a free waits for every stream of
  // the device, a peer's spinning collective included); a no-op elsewhere.
  virtual void set_deferred_frees(bool on) { (void)on; }
  virtual bool deferred_frees() const { return false; }
  // Bytes held in DBufs of this backend now and at most so far: one rank's
  // device footprint (graph shard + traversal state; the peer transport's
  // windows are allocated outside DBufs and not counted).
  int64_t device_bytes() const { return live_bytes_.load(std::memory_order_relaxed); }
  int64_t peak_device_bytes() const { return peak_bytes_.load(std::memory_order_relaxed); }
  void note_device_bytes(int64_t delta) {
    const int64_t now = live_bytes_.fetch_add(delta, std::memory_order_relaxed) + delta;
    int64_t pk = peak_bytes_.load(std::memory_order_relaxed);
    while (now > pk && !peak_bytes_.compare_exchange_weak(pk, now, std::memory_order_relaxed)) {
    }
  }
  virtual void memset_async(void* p, int value, size_t bytes) = 0;
  virtual void copy_async(void* dst, const void* src, size_t bytes) = 0;
  // Several device-to-device copies as one launch (4-byte multiples; the
  // shadow rank's replayed collectives: ReplayComm).
  struct CopyPieces {
    static constexpr int kMax = 16;
    void* dst[kMax] = {};
    const void* src[kMax] = {};
    int64_t bytes[kMax] = {};
    int n = 0;
  };
  virtual void copy_pieces(const CopyPieces& c) {
    for (int i = 0; i < c.n; ++i) copy_async(c.dst[i], c.src[i], static_cast<size_t>(c.bytes[i]));
  }
  virtual void to_host(void* host_dst, const void* dev_src, size_t bytes) = 0;   // blocking
  virtual void to_device(void* dev_dst, const void* host_src, size_t bytes) = 0; // blocking
  virtual void synchronize() = 0;
  // Non-blocking: true when all enqueued work has completed (raises on a
  // device error).
  virtual bool stream_idle() {
    synchronize();
    return true;
  }

  // timing: ms between two recorded points (events on HIP)
  virtual int record_event() = 0;
  virtual double elapsed_ms(int ev_begin, int ev_end) = 0;
  virtual void reset_events() = 0;

  // BFS primitives
  virtual void fill_level(lvl_t* level, int64_t n, lvl_t value) = 0;
  virtual void set_bit(word_t* bitmap, int64_t bit) = 0;
  virtual void update_frontier(const UpdateArgs& a) = 0;
  virtual void scan_units(const ScanArgs& a) = 0;
  // *ctrl = init (stream-ordered)
  virtual void level_ctrl_init(LevelCtrl* ctrl, const LevelCtrl& init) = 0;
  virtual void init_run(const InitRunArgs& a) = 0;
  // mb->v[0..3] = stats[0..3], then mb->seq = seq (release); mb is the device
  // pointer of an alloc_mapped block.
  virtual void publish_stats(const int64_t* stats, StatsMailbox* mb, int64_t seq) = 0;
  // Give an installed wait watch a chance to inspect a host-side wait that does
  // not go through the stream (mailbox spins).
  void poll_wait_watch(double waited) {
    if (wait_watch_) wait_watch_(waited);
  }
  double wait_watch_period() const { return wait_period_; }
  // Pinned host memory the device can store to (nullptr-safe free).
  virtual void* alloc_mapped(size_t bytes, void** device_ptr) = 0;
  virtual void free_mapped(void* host_ptr) = 0;
  virtual void zero_degree_mask(const ZeroDegArgs& a) = 0;
  virtual void compact_frontier(const CompactArgs& a) = 0;
  virtual void td_sparse(const TdSparseArgs& a) = 0;
  virtual void td_sparse_apply(const TdSparseArgs& a) = 0;
  virtual void level_finish(const LevelFinishArgs& a) = 0;
  virtual void td_expand(const TdArgs& a) = 0;
  // the passes of a binned top-down level (BinArgs), stream-ordered
  virtual void td_binned(const BinArgs& a) = 0;
  virtual void pack_bytes(const PackArgs& a) = 0;
  virtual void list_scatter(const ListScatterArgs& a) = 0;
  virtual void bu_step(const BuArgs& a) = 0;
  virtual void hub_gather(const HubGatherArgs& a) = 0;
  // Hub-cut level's top-down part (BuArgs::cut_edges): the unvisited
  // neighbours of the frontier's non-hub vertices claimed into a.pre.
  virtual void bu_cut_prep(const BuArgs& a) = 0;
  // ... several ranks: the claims the peers sent (BuArgs::cut_recv) into the
  // owned claim bytes, the packed bitmap zeroed -- on a live cut level only
  virtual void bu_cut_merge(const BuArgs& a) = 0;
  // A direct exchange's wait as a launch of its own, one wave (ranks sharing
  // a GPU, Comm::split_waits): the consumer after it finds the cells tagged.
  virtual void direct_prewait(const DirectExchange& x) { (void)x; }
  virtual void hub_visited(const HubVisitedArgs& a) = 0;
  virtual void unvis_filter(const UnvisArgs& a) = 0;
  virtual void hub_apply(const HubApplyArgs& a) = 0;
  virtual void refresh_visited(const RefreshArgs& a) = 0;
  // Device-checked build (make checked): whether the kernels verify their
  // bounds, the first recorded violation (code << 48 | detail; 0: none;
  // synchronises, clears), and a hook recording violation 99 (fault tests).
  virtual bool device_checks_enabled() const { return false; }
  virtual uint64_t take_device_check() { return 0; }
  virtual void inject_device_check() {}
  virtual void status_expand(const StatusArgs& a) = 0;
  virtual void bitmap_or(word_t* dst, const word_t* src, int64_t words) = 0;
  virtual void ref_expand(const RefExpandArgs& a) = 0;
  virtual void ref_accept(const RefAcceptArgs& a) = 0;
  virtual void scan_relax(const ScanBfsArgs& a) = 0;
  virtual void scan_count(const ScanBfsArgs& a) = 0;   // then exclusive_scan(offs, nranks * q)
  virtual void scan_bounds(const ScanBfsArgs& a) = 0;
  virtual void scan_assign(const ScanBfsArgs& a) = 0;  // consumes offs
  virtual void validate_levels(const ValidateArgs& a) = 0;
  virtual void compute_parents(const ParentArgs& a) = 0;

  // Hub-first adjacency: out[r] = degree of local row r (saturated to uint32);
  // then sort every row by (key_deg[neighbour] descending, neighbour ascending).
  virtual void degrees_u32(const eid_t* row_off, int64_t rows, uint32_t* out) = 0;
  virtual void sort_neighbors(const eid_t* row_off, vid_t* col, int64_t rows, const uint32_t* key_deg) = 0;
  // Every row in neighbour-id order (n: vertex count; the device orders rows
  // of more than 4096 entries by 4096 id buckets only).
  virtual void sort_rows_by_id(const eid_t* row_off, vid_t* col, int64_t rows, int64_t n) = 0;
  // head[r] = col[row_off[r]] (0 for empty rows); with hub_idx (one entry per
  // vertex, UINT32_MAX for non-hubs) a hub head is stored as kHubFlag | index.
  virtual void row_heads(const eid_t* row_off, const vid_t* col, int64_t rows, vid_t* head,
                         const uint32_t* hub_idx = nullptr) = 0;
  // Non-empty-row view: counts[w] = non-empty rows of bitmap word w (words
  // entries), then (after an exclusive scan into nz_pref) the dense row_off /
  // head copies.
  virtual void nz_word_counts(const eid_t* row_off, int64_t rows, int64_t words, eid_t* counts) = 0;
  virtual void nz_fill(const eid_t* row_off, const vid_t* head, int64_t rows, const eid_t* nz_pref, eid_t* nz_row_off,
                       vid_t* nz_head) = 0;
  // Packed records of the view (ShardView::nz_rec) and the unit bases
  // (ceil(rows / 4096) + 1 entries).
  virtual void nz_records(const eid_t* row_off, const vid_t* head, int64_t rows, const eid_t* nz_pref, NzRec* rec,
                          eid_t* unit_base) = 0;
  // out[e] = kHubFlag | hub_idx[col[e]] for hub neighbours, else col[e].
  virtual void encode_hub_cols(const vid_t* col, int64_t nnz, const uint32_t* hub_idx, vid_t* out) = 0;
  // Hubs = vertices of degree >= min_deg (deg_all has n entries): hub_vertex
  // receives their ids (in some order), hub_idx[v] their index or UINT32_MAX;
  // returns the count (blocking).
  virtual int64_t select_hubs(const uint32_t* deg_all, int64_t n, uint32_t min_deg, vid_t* hub_vertex,
                              uint32_t* hub_idx) = 0;

  // graph construction on the device
  // deg[r] += number of edge endpoints owned in rows [lo, lo + rows) (deg zeroed by caller)
  virtual void gen_count_degrees(const GenParams& p, int64_t lo, int64_t rows, eid_t* deg) = 0;
  // in-place exclusive scan of n+1 entries (data[n] receives the total)
  virtual void exclusive_scan(eid_t* data, int64_t n) = 0;
  // col[cursor[u - lo]++] = v for every generated endpoint u owned
  virtual void gen_fill(const GenParams& p, int64_t lo, int64_t rows, eid_t* cursor, vid_t* col) = 0;
  // CSR build from a file's edges (DeviceGraph::from_edges): every edge
  // (u, v) gives the entries u -> v and v -> u, routed to rank x / part as
  // (row << 32 | neighbour).  counts[r] += entries for rank r; then the
  // entries scattered into per-rank segments (cursor[r] = segment start,
  // advanced); at the owner deg[row - lo] += 1 per entry (deg zeroed by the
  // caller) and, after the scan, col[cursor[row - lo]++] = neighbour.
  virtual void route_edges_count(const vid_t* u, const vid_t* v, int64_t m, int64_t part, int nranks,
                                 int64_t* counts) = 0;
  virtual void route_edges_fill(const vid_t* u, const vid_t* v, int64_t m, int64_t part, int nranks,
                                int64_t* cursor, uint64_t* out) = 0;
  virtual void entries_count(const uint64_t* e, int64_t k, int64_t lo, eid_t* deg) = 0;
  virtual void entries_fill(const uint64_t* e, int64_t k, int64_t lo, eid_t* cursor, vid_t* col) = 0;
  // sum of degrees of vertices with level != kUnreached (device scalar out)
  virtual void reached_degree_sum(const ShardView& g, const lvl_t* level, int64_t* out2) = 0;
  // over the shard's rows: out2[0] = sum of degree^2, out2[1] = rows with degree > 0
  virtual void degree_moments(const ShardView& g, int64_t* out2) = 0;
  // out[i] = in[i] (narrow levels; kNarrowUnreached -> kUnreached)
  virtual void widen_levels(const uint8_t* in, lvl_t* out, int64_t n, uint8_t base) = 0;

 protected:
  std::function<void(double)> wait_watch_;
  double wait_period_ = 0.05;
  std::atomic<int64_t> live_bytes_{0}, peak_bytes_{0};
};

std::unique_ptr<Backend> make_cpu_backend();
std::unique_ptr<Backend> make_hip_backend(int device);
int hip_device_count();  // 0 when no GPU / runtime unavailable

// RAII device buffer.
template <class T>
class DBuf {
 public:
  DBuf() = default;
  DBuf(Backend& be, size_t n) : be_(&be), n_(n) {
    if (n_) {
      p_ = static_cast<T*>(be_->alloc(n_ * sizeof(T)));
      be_->note_device_bytes(static_cast<int64_t>(n_ * sizeof(T)));
    }
  }
  ~DBuf() { reset(); }
  DBuf(const DBuf&) = delete;
  DBuf& operator=(const DBuf&) = delete;
  DBuf(DBuf&& o) noexcept { *this = std::move(o); }
  DBuf& operator=(DBuf&& o) noexcept {
    if (this != &o) {
      reset();
      be_ = o.be_; p_ = o.p_; n_ = o.n_;
      o.be_ = nullptr; o.p_ = nullptr; o.n_ = 0;
    }
    return *this;
  }
  void reset() {
    if (p_ && be_) {
      be_->dealloc(p_);
      be_->note_device_bytes(-static_cast<int64_t>(n_ * sizeof(T)));
    }
    p_ = nullptr; n_ = 0;
  }
  T* data() const { return p_; }
  size_t size() const { return n_; }
  size_t bytes() const { return n_ * sizeof(T); }

 private:
  Backend* be_ = nullptr;
  T* p_ = nullptr;
  size_t n_ = 0;
};

}  // namespace dbfs
