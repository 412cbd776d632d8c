// Distributed level-synchronous BFS engine.
//
// Reference: runCudaQueueBfs (bfs.cu:542-629, bfs_mpi.cu:549-643) -- a host
// loop that per level launches queueBfs on every device, synchronises, copies
// owner buckets peer-to-peer and reads managed counters.  This engine keeps the
// level-synchronous, owner-computes structure but:
//   * shards the CSR (owned rows only) instead of replicating it per device;
//   * represents frontier / visited as bitmaps (64 vertices per wave ballot);
//   * exchanges discoveries as equal-size bitmap slices (ncclAllToAll) and the
//     new frontier with one ncclAllGather, so no count exchange is needed;
//   * switches direction (Beamer alpha/beta) between top-down load-balanced
//     expansion and bottom-up parent search;
//   * keeps the reference algorithm as Mode::Ref (the measured baseline) and
//     the status-array variant as Mode::Simple.
#pragma once

#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "dbfs/backend.hpp"
#include "dbfs/comm.hpp"
#include "dbfs/graph.hpp"
#include "dbfs/partition.hpp"

namespace dbfs {

enum class Mode { Ref, TopDown, BottomUp, DirOpt, Simple, Scan };
Mode parse_mode(const std::string& s);
const char* mode_name(Mode m);

// A CSR shard resident in backend memory.
class DeviceGraph {
 public:
  // `csr` is either the full graph (rows == n) or exactly this rank's shard.
  static std::unique_ptr<DeviceGraph> from_host(Backend& be, const HostCSR& csr, const Partition& part, int rank);
  // Generate this rank's shard of a synthetic graph directly on the device.
  static std::unique_ptr<DeviceGraph> generate(Backend& be, const GenParams& p, const Partition& part, int rank);
  // Build this rank's shard on the device from the edges this rank read (any
  // slice of the file, e.g. read_edge_shard): every edge's two entries are
  // routed to their owners (count -> all-to-all-v of (row, neighbour) pairs),
  // then count -> scan -> fill as generate().  Collective over `comm`.
  // input_edges: edges of the whole input (Graph500 TEPS numerator).
  static std::unique_ptr<DeviceGraph> from_edges(Backend& be, Comm& comm, const Partition& part, int rank,
                                                 int64_t input_edges, const vid_t* u, const vid_t* v,
                                                 int64_t m_local);
  // A file read in shards: edge list / MatrixMarket through read_edge_shard +
  // from_edges, a binary CSR cache through its rank's rows only.  Collective.
  static std::unique_ptr<DeviceGraph> from_file(Backend& be, Comm& comm, const std::string& path, int threads = 0);

  ShardView view() const;
  HostCSR to_host() const;  // the shard, copied back
  Backend& backend() const { return *be_; }
  const Partition& partition() const { return part_; }
  int rank() const { return rank_; }
  int64_t n() const { return part_.n; }
  int64_t lo() const { return lo_; }
  int64_t rows() const { return rows_; }
  int64_t nnz() const { return nnz_; }
  int64_t input_edges() const { return input_edges_; }
  std::vector<eid_t> degrees_of(const std::vector<int64_t>& local_rows) const;
  // Reorder every row hub-first (neighbour degree descending); collective over
  // `comm` (all ranks need every vertex's degree).  One-time preprocessing.
  // With `hubs`, the (up to kMaxHubs) highest-degree vertices of the graph are
  // also indexed and every row head naming one is hub-encoded (ShardView).
  // With hubs and `id_order`, bottom-up keeps the hub-first order in its
  // hub-encoded copy and `col` is then put in neighbour-id order for the
  // top-down sweeps (neighbours of one row probe the bitmaps monotonically).
  // ... and with `td_hubs` also the hub-encoded top-down copy td_col (the
  // kTdMaxHubs highest-degree vertices encoded; one more nnz x 4 B).
  void sort_neighbors_by_degree(Comm& comm, bool hubs = true, int64_t max_hubs = kMaxHubs, bool id_order = true,
                                bool td_hubs = true);
  bool hub_sorted() const { return hub_sorted_; }
  // col is in id order (bottom-up must scan hub_col, whose order is hub-first)
  bool col_by_id() const { return col_by_id_; }
  // share of all adjacency entries held by the top-down hubs' rows (0 without
  // them): graphs whose hubs are only slightly above the mean degree (uniform
  // random graphs) gain nothing from the top-down hub filter
  double td_hub_share() const { return td_hub_share_; }
  // every rank's shard has the packed row records (agreed at the degree sort)
  bool rec_all() const { return rec_all_; }
  int64_t nhubs() const { return nhubs_; }
  // from_file: the byte range [begin, end) of the file this rank parsed and
  // the edges it read (a binary cache: rows, -1 bytes); -1 when not from a file
  struct IngestInfo {
    int64_t byte_begin = -1, byte_end = -1, edges = -1;
  };
  const IngestInfo& ingest() const { return ingest_; }

 private:
  IngestInfo ingest_;
  Backend* be_ = nullptr;
  Partition part_;
  int rank_ = 0;
  int64_t lo_ = 0, rows_ = 0, nnz_ = 0, input_edges_ = 0;
  bool hub_sorted_ = false;
  bool col_by_id_ = false;
  int64_t nhubs_ = 0;
  bool rec_all_ = false;  // every rank has the packed row records (rec_all())
  void build_heads(const uint32_t* hub_idx = nullptr);
  DBuf<vid_t> head_, hub_vertex_, nz_head_, hub_col_, td_col_, td_hub_vertex_;
  double td_hub_share_ = 0.0;
  DBuf<uint32_t> hub_deg_;  // ShardView::hub_deg
  DBuf<word_t> hub_bits_;  // global vertex bitmap of the hubs
  int64_t td_nhubs_ = 0;
  DBuf<eid_t> nz_pref_, nz_row_off_;
  DBuf<NzRec> nz_rec_;      // packed view records (empty when a unit spans >= 2^32 edges)
  DBuf<eid_t> unit_base_;
  void build_nz_view();
  DBuf<eid_t> row_off_;
  DBuf<vid_t> col_;
};

struct EngineOptions {
  Mode mode = Mode::DirOpt;
  // Beamer's direction switch.  Defaults tuned on MI355X / RMAT-26 (sweeps in
  // profiles/): BU is cheap enough here that switching earlier than Beamer's
  // CPU value (14) pays.  alpha 40 (from 24, round 4): the same on the
  // bench's roots, +5 % on roots with a slower-growing frontier (a 64-root
  // tuning sample, seed 20261017; profiles/r4_final_alpha_sweep.txt), the
  // soc-LiveJournal1-sized graph unchanged.
  double alpha = 40.0;  // TD -> BU when m_f > m_u / alpha
  double beta = 384.0;  // BU -> TD when n_f < n / beta (and shrinking)
  // (384 since round 6, from 96: a shrinking frontier stays bottom-up
  // longer.  Asked to be a function of P -- a bottom-up level's cost per rank
  // shrinks with P, a sparse top-down level's does not -- the shadow replays
  // of RMAT-26 (ranks 0 and P - 1, four roots) found one value best at every
  // P: the late-switch roots' post-bottom-up level stays bottom-up (P = 8:
  // 103 -> 24 us), their traversals -12 % / -11 % / -19 % at P = 2 / 4 / 8,
  // early-switch ones unchanged, 768 and 1536 no better (profiles/
  // r6_policy_shadow_p*.txt); one GPU, 128 held-out roots, same box: 1498 /
  // 1494 -> 1506 / 1513 GTEPS (profiles/r6_beta_one_gpu_ab.txt).  alpha x 4
  // changed nothing at P = 8.)
  // neighbours a lane checks itself before rows go to wave-cooperative scans
  // (16: a first bottom-up level entered with a small frontier resolves more
  // rows per lane; RMAT-26 1240 -> 1259 GTEPS, 8 and 32 worse)
  int bu_lane_limit = 16;
  // Bottom-up waves take a whole 64-word unit (1), 16 words (-1), or by shard
  // size (0: whole units when they fill every resident wave slot).
  int bu_whole_units = 0;
  // ... units split over waves (small shards): a first bottom-up level at 4
  // words per wave instead of 16 (1), never (-1), when 16 would leave wave
  // slots idle (0)
  int bu_small_waves = 0;
  // Top-down levels with at least this many local frontier edges mark
  // discoveries in a byte map (plain stores) instead of bitmap atomics.
  int64_t td_byte_edges = int64_t(1) << 22;
  // Device loop, one rank, narrow levels: top-down levels with at least
  // td_direct_edges frontier edges store the new level straight into the
  // one-byte level array of every unvisited candidate (no byte map, nothing
  // to clear; the update reads the level bytes back) -- cheaper than the
  // candidate bitmap's memory-side atomics from ~64 K edges (RMAT-26: a
  // 1.7 M-edge level 115 -> 68 us).  Replaces td_byte_edges there.
  static constexpr bool td_direct = true;
  int64_t td_direct_edges = int64_t(1) << 16;
  // Device loop, one rank: top-down levels predicted to have at least this
  // many frontier edges run binned (BinArgs: targets binned by vertex range,
  // claimed per bin in LDS) instead of td_expand + update; 0 disables.  Only
  // on graphs of at least td_bin_min_rows vertices (level bytes and visited
  // bits far past the L2: a direct level's two random lines per edge go to
  // HBM; below, the direct level is faster -- RMAT-22 top-down) and only
  // before the run's first bottom-up level (the shrinking levels after it are
  // predicted from a falling frontier and are mostly far smaller).
  // Measured, RMAT-26 per root: a 28 M-edge second-level expansion 556 ->
  // 402 us; 1354 -> 1368 GTEPS with the bottom-up gate missing (post-bottom-up
  // levels of 200 K edges predicted at 2 M: 58 -> 80 us).
  // Not for levels the direct form does better since split top-down levels
  // (DeviceLoop::td_form): RMAT-26 top-down only 39.1 GTEPS binned against
  // 67.7 direct and split (its 0.5 B-edge level 5.6 -> 5.0 ms, the next one,
  // with the unvisited filter, 21.3 -> 10.8 ms; profiles/r5_td_binned_off_ab.txt).
  int64_t td_bin_edges = int64_t(1) << 21;
  // (2^26: RMAT-24, 2^24 vertices, measured 2 % slower binned -- 785 / 793
  // against 815 / 800 GTEPS; RMAT-26 +2-4 %; RMAT-27 flat)
  int64_t td_bin_min_rows = int64_t(1) << 26;
  // ... about 2^td_bin_log2_bins bins (of >= 4096 vertices, at most
  // kBinMaxBins; each bin's visited slice must fit LDS).  RMAT-26, the 28 M-edge
  // binned level: 256 / 512 / 1024 bins 407 / 417 / 441 us (more bins: the
  // fill pass scatters into more open lines).
  static constexpr int64_t td_bin_log2_bins = 8;
  // Dense top-down levels predicted at >= td_unvis_edges frontier edges that
  // start with >= td_unvis_vis_frac of the adjacency visited test targets in
  // an LDS unvisited filter first (UnvisArgs, TdArgs::unvis): a clear bit
  // means visited, so only the rest cost a scattered `visited` probe.  0
  // disables.
  int64_t td_unvis_edges = int64_t(1) << 22;
  double td_unvis_vis_frac = 0.6;
  // ... such a level runs with the filter iff at most this fraction of the
  // filter's bits are set (decided on the device from the built filter)
  double td_unvis_max_density = 0.5;
  // One rank, level-byte (level_direct) top-down levels predicted at >=
  // td_split_edges frontier edges run in td_split_parts parts (twice as many
  // from 16 x td_split_edges on graphs of >= 2^25 vertices: a smaller graph's
  // predicted level overshoots, and RMAT-22 runs 3 % slower in 8), the claims of the parts so far ORed into
  // `visited` between them (refresh_visited): a target reached by many
  // frontier edges stores its level byte about once per part instead of once
  // per edge.  0 disables.  RMAT-22 top-down only 98.5 -> 105.7 GTEPS (8 parts:
  // 103); RMAT-26 top-down only 55.8 -> 67.7 (its 0.5 B-edge level 9.4 -> 5.0
  // ms; 8 parts 69.5): profiles/r5_td_split_levels_ab.txt.
  int64_t td_split_edges = int64_t(1) << 23;
  int td_split_parts = 4;
  // Dense top-down levels with at least this many frontier edges test hub
  // targets in an LDS copy of the hubs' visited bits (ShardView::td_col);
  // 0 disables.
  // (RMAT-22 top-down-only, per root: levels of 75-90 M edges 440-511 ->
  // 397-474 us, the 43-58 M-edge levels before the visited fraction is
  // reached unchanged; below ~16 M edges the hub snapshot and its LDS staging
  // cost what they save)
  int64_t td_hub_edges = int64_t(1) << 24;
  // ... once the visited vertices hold this fraction of the adjacency.
  // Without hub marks (td_hub_mark) 0, i.e. also the earlier big levels, was
  // slower (58.9 against 63.5 GTEPS: decoding unvisited hubs costs a
  // dependent load); with them 0 is faster (69.0 against 65.9).
  double td_hub_vis_frac = 0.0;
  // ... only on graphs whose top-down hubs hold at least this share of the
  // adjacency entries (DeviceGraph::td_hub_share)
  static constexpr double td_hub_min_share = 0.0;
  // Direct-level top-down: hub targets claimed as one byte per hub (an
  // L2-resident 128 KiB array) and turned into level bytes after the
  // expansion (TdArgs::td_hub_mark, hub_apply).
  static constexpr bool td_hub_mark = true;
  // Byte-map levels skip the visited pre-check while the visited vertices
  // hold less than this fraction of all adjacency entries.
  double td_check_visited_min = 0.02;
  // Top-down grids of fewer workgroups than this use 1024-thread workgroups.
  int64_t td_wide_below_blocks = 2048;
  // Multi-rank top-down levels whose global frontier has at most this many
  // edges exchange owner lists instead of bitmap slices.
  int64_t sparse_max_edges = int64_t(1) << 17;
  // ... and only when the lists are smaller than half a bitmap slice (tests
  // switch this off to exercise the list path on small graphs).
  bool sparse_size_check = true;
  bool phase_timing = false;  // per-level device timing (adds events)
  // One rank, td/bu/do modes: device-driven level loop (LevelCtrl): the host
  // enqueues the next level before the current one finishes.
  bool device_loop = true;
  // ... also with several ranks: each level's chain carries its collectives
  // (frontier all-gather, candidate all-to-all, totals all-reduce), enqueued
  // ahead like the kernels; level_finish decides on the reduced totals.
  static constexpr bool device_loop_ranks = true;
  // ... enqueueing each level with an extrapolated direction prediction (else:
  // the previous level's direction, one more level ahead).
  bool device_loop_predict = true;
  // Host loop (several ranks, or device_loop off): read each level's totals
  // through a device-mapped mailbox the host spins on, instead of a D2H copy
  // plus a stream synchronisation.
  static constexpr bool stats_mailbox = true;
  // Device loop: top-down levels whose frontier is predicted to have at most
  // this many edges run as one sparse kernel (TdSparseArgs: direct claims, work list
  // handed to the next level) instead of compact + td_expand + update + scan;
  // 0 disables.  td_sparse_grid: its workgroups (RMAT-26, 256 / 512 / 1024:
  // 1504-1509 / 1506-1509 / 1492-1503 GTEPS held-out, profiles/r6_sparse_grid_ab.txt).
  int64_t td_sparse_edges = int64_t(1) << 16;
  static constexpr int64_t td_sparse_grid = 256;
  // ... several ranks: the owners' side (td_sparse_apply) at most this many
  // workgroups (sized by the level's expected received ids, ~512 each; only
  // those with ids take part).  Shadow rank 0 of RMAT-26 at P = 2, the 1.3
  // M-edge sparse level: 128 workgroups 91 us, 512 81 us.
  static constexpr int64_t td_apply_grid = 512;
  // A sparse chain stays live up to td_sparse_cap_factor x td_sparse_edges
  // frontier edges (0: any size); a larger level is re-enqueued dense.
  static constexpr double td_sparse_cap_factor = 8.0;
  // Device loop: workgroups of the dense top-down expansion grid (at most;
  // they stride over the level's edge blocks; the launcher also caps the grid
  // at the kernel's residency), without and with the hub filter.  Measured:
  // RMAT-26 (no filter levels) 1024 workgroups 1354 / 1334 against 1323 /
  // 1318 GTEPS at 2048; RMAT-22 top-down only (filter levels) 1024 / 1280 /
  // 1536 (= residency) 77 / 81 / 83 GTEPS.
  static constexpr int64_t td_grid_max = 1024;
  static constexpr int64_t td_grid_filter_max = 2048;
  // The sparse threshold for the first top-down level after a bottom-up one
  // (the extrapolated prediction of a shrinking frontier overshoots), and
  // how far such a chain stays live.  RMAT-26: the late-switch roots' level
  // after three bottom-up levels (0.2-0.6 M edges, predicted 2-6 M) 52-58 ->
  // 19-28 us sparse; a shared cap (td_sparse_cap_factor) would also keep
  // mispredicted early chains sparse (measured: 112 -> 331 us).
  static constexpr int64_t td_sparse_bu_edges = int64_t(1) << 23;
  // ... and that level reads the bottom-up level's output bitmap itself
  // (TdSparseArgs::from_bits: one kernel after a clear of its output bitmap,
  // instead of scan_units + compact + td_sparse).
  bool td_sparse_bits = true;
  // Device loop: a bottom-up level's unit scan (totals; one rank: direction
  // decision, mailbox stamp) runs in the bottom-up kernel's last-arriving
  // workgroup instead of a kernel of its own.
  static constexpr bool bu_fused_scan = true;
  // Device loop: a dense top-down level's update finishes the
  // level itself (as bu_fused_scan; per-workgroup totals slots, 512
  // workgroups striding over the units with one ticket, the full grid with
  // td_group_ticket): no scan launch unless a compaction follows.
  // RMAT-26 1344 / 1341 -> 1363 / 1353 GTEPS; top-down only equal within noise.
  // (A first version with one workgroup per 4 units and totals atomics on
  // one address: level 1 of RMAT-26 38 -> 117 us.)
  static constexpr bool td_fused_finish = true;
  // ... and on graphs of at most kFoldScanUnits 4096-vertex units (2^25
  // vertices) its last workgroup also scans the unit prefixes the next
  // compaction reads (UpdateArgs::fold_scan): one launch less per dense level
  static constexpr bool fold_scan = true;
  // ... with a two-level ticket (UpdateArgs::group_ticket): the update runs
  // a full grid (up to kMaxFusedGrid workgroups) instead of kMaxFusedGrid / 8.
  static constexpr bool td_group_ticket = true;
  // Device loop, several ranks: sparse top-down levels (td_sparse with owner
  // lists, the lists exchanged count-sized, td_sparse_apply on the owners)
  // for levels predicted at <= xsparse_edges global frontier edges; such a
  // chain stays live up to list_form_edges (the owner lists' capacity: P x
  // that many ids per rank, twice) and a larger level is re-enqueued dense.
  // 0 disables (dense top-down chains only).
  int64_t list_form_edges = int64_t(1) << 21;
  int64_t xsparse_edges = int64_t(1) << 20;
  // ... levels predicted at <= xfuse_edges (a chain then live up to 4x that):
  // with a direct exchange and a folded level end, td_sparse's last workgroup
  // runs the owner side too (TdSparseArgs::fuse_apply: one launch per level);
  // 0 disables.  (Validated over the peer transport with 4 processes on one
  // GPU, tests/test_gpu_engine.py::test_peer_multirank_options; shadow rank 0
  // of RMAT-26 at P = 8: level 0 11-19 -> 6-10 us.)
  int64_t xfuse_edges = int64_t(1) << 12;
  // Several ranks, bottom-up levels: merge the gathered frontier into the
  // replicated visited bitmap (the remote slices; folded into hub_gather).
  // Only top-down levels read remote visited bits, as a filter: a stale one
  // sends an id its owner drops, so the levels stay exact without it -- but
  // the top-down level after the bottom-up ones then claims and sends every
  // remote target the bottom-up levels reached.  Shadow rank 0 of RMAT-26
  // (profiles/r5_shadow_ab_merge_apply_grid.txt): that level 51-67 -> 21-24
  // us at P = 2 for 3-5 us per bottom-up level; traversal -6.6 % at P = 2,
  // -3.6 % at P = 8.
  bool bu_merge_visited = true;
  // Device loop, hubs: a first bottom-up level whose frontier has at most
  // bu_cut_edges edges outside the hubs claims those vertices' neighbours
  // top-down (bu_cut_prep) and scans only the rows' hub prefixes
  // (BuArgs::cut_edges) -- the late-switch level, whose frontier is a few
  // thousand vertices, mostly hubs.  0 disables.
  int64_t bu_cut_edges = int64_t(1) << 22;
  // ... with several ranks too, up to this many: every rank claims its own
  // non-hub frontier's neighbours, the remote ones in the byte map, packed
  // and sent to their owners as one bitmap all-to-all (bu_cut_merge applies
  // them) -- the top-down part shrinks with P as the bottom-up share does.
  // (Round 4's form sent the remote claims as owner lists and measured
  // slower at P = 8.)  Shadow replays of RMAT-26's late-switch roots
  // (profiles/r6_xcut_shadow_ab.txt, traversal us per rank): P = 2
  // 602-766 -> 530-620, P = 4 393-508 -> 397-453, P = 8 270-334 ->
  // 298-345 -- the cut's fixed launches (decision, top-down part, 64 MB byte
  // map pack, all-to-all, merge) outweigh what it saves a rank's 1/8 share
  // of the bottom-up scan at P = 8, so it stops at 4.
  int64_t bu_cut_ranks = 4;
  // ... enqueued (its decision and top-down launches) only for levels
  // predicted at <= bu_cut_mf_frac of the graph's directed edges (RMAT-26:
  // the late-switch first bottom-up levels have 4-15 % of them, the others
  // 37 % and more)
  double bu_cut_mf_frac = 0.25;
  // ... on a transport that ships the lists' capacity (RCCL / TCP fallback;
  // the peer windows ship their lengths), a chain's lists hold
  // list_cap_factor x the predicted edges (a power of two >= 1024)
  double list_cap_factor = 4.0;
  // Sparse chains on a transport with a direct exchange (peer windows,
  // Comm::direct_lists): td_sparse stores remote claims straight into their
  // owners' windows and td_sparse_apply waits for the flags -- no exchange
  // launch in between
  static constexpr bool direct_lists = true;
  // ... and their level's end folded into td_sparse_apply's last workgroup
  // (Comm::direct_level_end) when it gathers no frontier
  static constexpr bool direct_level_end = true;
  // Several ranks, a level whose frontier is all-gathered for a bottom-up
  // level next (graphs with hubs): the producing kernels push their output
  // words straight into the peers' windows (Comm::direct_frontier) and the
  // bottom-up level's hub_gather copies them in -- the level end carries only
  // its totals (and may fold into the bottom-up kernel): the frontier
  // exchange overlaps the kernels that produce it instead of following them.
  bool direct_frontier = true;
  // Bitmap engine (td / bu / do): levels kept in a one-byte-per-vertex array
  // during the traversal (a quarter of the per-run initialisation traffic),
  // widened to 32 bits when read; a traversal deeper than kNarrowMaxLevel is
  // rerun with 32-bit levels (and later runs keep them).
  bool narrow_levels = true;
  // Narrow level bytes stored as base + level with the base cycling through
  // kNarrowEpochs values, so only one run in kNarrowEpochs fills the byte
  // array (the others read the earlier epochs' bytes as unreached).
  static constexpr bool narrow_epochs = true;
  // Take the multi-rank exchange path (alltoall / allgather / alltoallv) even
  // with one rank: lets a 1-rank RCCL communicator exercise every collective
  // call on a single GPU (tests).
  bool force_exchange = false;
  // Directed input (CSR holds out-edges only): top-down modes only; vertices
  // without out-edges are not pre-marked visited; traversed edges = out-edges
  // of the reached vertices.
  bool directed = false;
};

// Named access to the numeric tuning options (alpha, beta, bu_lane_limit,
// td_byte_edges, td_wide_below_blocks, td_check_visited_min, sparse_max_edges,
// sparse_size_check, force_exchange, phase_timing); throws on unknown names.
void set_engine_option(EngineOptions& o, const std::string& name, double value);
std::vector<std::pair<std::string, double>> engine_option_map(const EngineOptions& o);

struct LevelRecord {
  int level = 0;
  char direction = 'T';  // 'T' top-down, 'B' bottom-up, 'R' reference, 'S' simple, 'C' scan
  int64_t frontier = 0;       // global frontier vertices expanded at this level
  int64_t frontier_edges = 0; // global sum of their degrees
  int64_t discovered = 0;     // global new vertices
  double ms = 0.0;            // device time of the level (phase_timing only)
  double comm_ms = 0.0;       // ... of which in collectives (host loop, phase_timing only)
  // Device loop, device clock: idle time between the previous level's scan
  // and this level's first kernel (launch gaps; -1 when unknown).
  double gap_ms = -1.0;
};

// One level chain the device loop enqueued (mispredicted ones included):
// form 'T' dense top-down, 'S' sparse top-down (`cap`: the global frontier
// edges it stays live for; several ranks: its owner lists' capacity), 'X'
// binned top-down, 'B' bottom-up; `gather` (several ranks): the chain's
// collective also all-gathered its output frontier.
struct ChainRecord {
  int level = 0;
  char form = 'T';
  int64_t cap = 0;
  bool gather = false;
  // several ranks: its output frontier pushed by its kernels (no gather in
  // its level end; EngineOptions::direct_frontier)
  bool push = false;
  // a dense top-down chain with the unvisited filter (TdArgs::unvis)
  bool unvis = false;
  // ... run in this many parts (TdArgs::split_k; 1: whole)
  int split = 1;
  // a bottom-up chain with the hub cut's launches (decided on the device)
  bool cut = false;
};

struct RunResult {
  int64_t source = 0;
  double ms = 0.0;             // wall time of the traversal (max over ranks)
  int64_t reached = 0;         // vertices reached (global)
  int64_t edges = 0;           // traversed undirected edges (Graph500)
  int depth = 0;               // number of levels (max level + 1)
  double gteps = 0.0;
  int mispredicts = 0;         // device loop: level chains enqueued for the wrong direction
  std::vector<LevelRecord> levels;
  std::vector<ChainRecord> chains;  // device loop: every chain enqueued, in order
};

// Fault injection for failure-detection tests (see Engine::inject_fault).
struct FaultSpec {
  int rank = -1, level = -1;
  std::string kind = "throw";
  int ms = 2000;  // kind=delay: how long the rank sleeps before enqueueing the level
  int us = 500;   // kind=late_wg: how long td_sparse's ticket-less workgroups wait (TdSparseArgs::late_ticks)
  static FaultSpec from_env();
};

class DeviceLoop;  // the device-driven level loop (csrc/engine/device_loop.cpp)

class Engine {
 public:
  Engine(DeviceGraph& g, Comm& comm, const EngineOptions& opt = {});
  ~Engine();
  RunResult run(int64_t source);
  // Owned slice of the last run's levels.
  std::vector<lvl_t> levels_local() const;
  // Full level array (all ranks participate).
  std::vector<lvl_t> gather_levels();
  // Graph500-style device validation of the last run; returns violation counts
  // {depth-gap, reached-unreached, orphan} summed over ranks (all must be 0).
  std::vector<int64_t> validate(int64_t source);
  // Graph500 parent tree of the last run (global vertex ids; -1 unreached):
  // owned slice, and the full array (all ranks participate in both).
  std::vector<int64_t> parents_local(int64_t source);
  std::vector<int64_t> gather_parents(int64_t source);
  int64_t global_directed_edges() const { return total_directed_; }
  const EngineOptions& options() const { return opt_; }
  void set_options(const EngineOptions& o) {
    opt_ = o;
  }

 private:
  friend class DeviceLoop;
  RunResult run_bitmap(int64_t source);
  RunResult run_bitmap_device(int64_t source);
  bool use_device_loop() const;
  RunResult run_ref(int64_t source);
  void alloc_bitmap_state();
  void begin_run_scratch();
  InitRunArgs init_args(int64_t source, word_t* seed_frontier, LevelCtrl* ctrl, const LevelCtrl& ctrl_init,
                        LevelMailbox* mailbox);
  bool scratch_dirty_ = true;  // cand / next / byte map may hold stale bits
  bool frontier_clean_ = false;  // the owned frontier slices are zero (InitRunArgs::frontier_clean)
  void alloc_ref_state();
  void gather_levels_device(DBuf<lvl_t>& full);
  bool exchange() const { return part_.nranks > 1 || opt_.force_exchange; }
  void inject_fault(int level);
  void check_device();

  DeviceGraph& g_;
  Comm& comm_;
  Backend& be_;
  EngineOptions opt_;
  Partition part_;
  FaultSpec fault_;
  int64_t total_directed_ = 0;

  DBuf<lvl_t> level_;
  DBuf<uint8_t> level8_;
  DBuf<uint32_t> td_group_ticket_;  // UpdateArgs::group_ticket
  DBuf<int64_t> bu_tot_;  // fused bottom-up finish: per-workgroup totals (BuArgs::tot)
  DBuf<int64_t> td_tot_;  // fused top-down finish: the level's totals (UpdateArgs::tot)
  DBuf<uint8_t> td_hub_mark_;  // TdArgs::td_hub_mark (kTdMaxHubs bytes; zero between levels)
  bool level8_filled_ = false;        // level8_ reads unreached for the current run without a fill
  uint8_t narrow_base_ = 0;           // the current run's level byte base (narrow_epochs)
  int64_t narrow_run_ = 0;            // narrow runs since level8_ was allocated
  bool narrow_failed_ = false;        // a traversal overflowed the narrow levels
  bool run_narrow_ = false;           // the current run writes level8_
  mutable bool levels_narrow_ = false;  // level_ is stale: level8_ holds the last run's levels
  bool use_narrow() const;
  void ensure_wide_levels() const;
  // bitmap engine state
  bool bitmap_ready_ = false;
  DBuf<word_t> visited_, zdeg_, frontier_[2], next_, recv_, cand_, hub_front_, td_hub_vis_, unvis_;
  DBuf<uint32_t> unvis_pop_;
  DBuf<uint32_t> deg_all_;  // several ranks: every vertex's degree (InitRunArgs::deg_all)
  // hub-cut bottom-up levels: per-workgroup frontier hub degrees, the
  // decision and its ticket (zero between levels)
  DBuf<int64_t> cut_part_;
  DBuf<int> cut_flag_;
  DBuf<uint8_t> cut_claim_;  // wide-level runs' claims
  DBuf<unsigned> cut_ticket_;
  DBuf<uint8_t> next_bytes_;  // lazily allocated (GW * 64 bytes)
  DBuf<vid_t> send_lists_, recv_lists_;  // sparse exchange, lazily allocated
  DBuf<int64_t> unit_cnt_, unit_deg_, part_cnt_, part_deg_, qscan_, qbase_, stats_;
  // Several ranks (device loop): level L's totals go to
  // stats block (L + 1) % kStatsBlocks, so a mispredicted chain's
  // (unpredicated) reduction never touches the block the re-enqueued chain
  // reads.  One rank: level L's totals in block (L + 1) % kStatsBlocks1, so a
  // level's input totals stay put while its own kernels finish it (see
  // DeviceLoop::sblk).  stats_stride_: int64 entries per block.
  static constexpr int kStatsBlocks = 3;
  static constexpr int kStatsBlocks1 = 2;
  int64_t stats_stride_ = 8;
  DBuf<vid_t> dl_send_lists_, dl_recv_lists_;  // device loop list form, stride list_stride_ + 1
  // binned top-down levels (one rank): bin counts / positions, bin starts, targets
  DBuf<int64_t> bin_total_;
  DBuf<uint32_t> bin_cnt_;
  DBuf<vid_t> bin_buf_;
  int64_t list_stride_ = 0;
  DBuf<unsigned> ticket_;
  DBuf<int32_t> blk_vstart_;
  // device loop, sparse top-down levels: a second work-list set (level L
  // reads set L & 1), entry -> vertex maps, output counters, a ticket
  bool sparse_ready_ = false;
  double excess_degree_ = 0.0;  // sum deg^2 / sum deg (level-1 edge prediction)
  int64_t n_active_ = -1;       // vertices with degree > 0 (global; -1: not computed yet)
  DBuf<int64_t> qscan2_, qbase2_;
  DBuf<int32_t> blk_vstart2_;
  DBuf<vid_t> qv_[2];
  DBuf<unsigned long long> sparse_cnt_;
  DBuf<unsigned> sparse_ticket_;
  bool sparse_enabled() const;
  int64_t nunits_ = 0;
  // device-driven loop state
  DBuf<LevelCtrl> ctrl_;
  // per-level records in pinned, device-mapped segments of kRecSeg levels
  // (host pointer, device pointer): the host reads them after the last stamp
  // without a copy or a stream synchronisation
  static constexpr int kRecSeg = 1024;
  std::vector<std::pair<LevelRecDev*, LevelRecDev*>> rec_segs_;
  LevelRecDev* rec_at(int level);  // device pointer of level's record
  LevelMailbox* mailbox_host_ = nullptr;  // pinned, device-mapped
  LevelMailbox* mailbox_dev_ = nullptr;
  // host-loop statistics mailbox
  StatsMailbox* stats_mb_host_ = nullptr;
  StatsMailbox* stats_mb_dev_ = nullptr;
  int64_t stats_seq_ = 0;
  void read_level_stats(int64_t* host_stats);
  // reference-mode state
  bool ref_ready_ = false;
  DBuf<lvl_t> dist_;
  DBuf<vid_t> queue_, buckets_, recvq_;
  DBuf<int64_t> bucket_cnt_, qcount_;
  DBuf<eid_t> claim_, scan_offs_;  // scan mode
};

}  // namespace dbfs
