// Device-driven level loop (Engine::run_bitmap_device): the host enqueues
// every level as a full predicated chain one level ahead of the device, which
// decides each level's direction itself (LevelCtrl) and stamps a mapped
// mailbox the host spins on.  Split into
//   * the planner: direction / frontier prediction (Beamer through the shared
//     level_ctrl_finish), the chain form of a top-down level (td_form) and
//     whether an enqueued chain is live for the level it turned out to be;
//   * the chain emitters, one per form: 'S' sparse top-down (emit_sparse),
//     'X' binned top-down (emit_binned), 'T' dense top-down (emit_dense),
//     'B' bottom-up (emit_bottom_up); with several ranks each chain also
//     enqueues its collectives and its level end (Comm::level_end, or the
//     direct exchanges the kernels run themselves).
// The reference's host loop (bfs.cu:569-620, bfs_mpi.cu:581-632) launches,
// synchronises, copies and reads managed counters once per level.
#include <algorithm>
#include <cmath>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "dbfs/engine.hpp"
#include "dbfs/trace.hpp"
#include "spin.hpp"

namespace dbfs {


class DeviceLoop {
 public:
  DeviceLoop(Engine& e, int64_t source)
      : e_(e), opt_(e.opt_), part_(e.part_), comm_(e.comm_), be_(e.be_), src_(source) {}
  RunResult run();

 private:
  // One enqueued level chain.
  struct Chain {
    int L = 0;
    char d = 'T';       // form: 'T', 'S', 'X', 'B'
    char pf = 'I';      // the previous level's form ('I': the seed)
    int64_t cap = 0;    // sparse: the global frontier edges it stays live for
    double mf_hint = -1;
    int cur = 0;        // input frontier buffer (level L reads frontier_[(L + 1) & 1])
    bool in_gathered = false;  // the input frontier is global already
    bool fused_scan = false;   // the chain's last kernel finishes the level
    bool level_ended = false;  // ... and also ran its level end (direct exchange)
    bool folded = false;       // ... and also scanned its unit prefixes (UpdateArgs::fold_scan)
    // several ranks: the output frontier pushed to the peers by the producing
    // kernel (EngineOptions::direct_frontier), and the input frontier's pushed
    // slices (the previous chain's table) for hub_gather to copy in
    const FrontierTable* push = nullptr;
    const FrontierTable* pull = nullptr;
  };

  Engine& e_;
  const EngineOptions& opt_;
  const Partition& part_;
  Comm& comm_;
  Backend& be_;
  const int64_t src_;

  // ---- run constants (setup) ----
  int64_t W_ = 0, GW_ = 0;
  int me_ = 0, P_ = 1;
  bool xc_ = false;        // several ranks (or a forced exchange): chains carry collectives
  ShardView gv_;
  bool direct_ = false;    // one rank, narrow levels: top-down levels write level bytes directly
  bool bytes_ok_ = false;
  int64_t byte_edges_ = 0;
  bool sparse_ = false;
  int64_t sparse_cap_ = 0;
  int64_t list_max_ = 0, xsparse_lim_ = 0, fuse_cap_ = 0;
  bool lists_unlimited_ = false, counted_ = false;
  double vis_hint_ = -1.0;  // the next enqueued level's visited degree sum at its start (< 0 unknown)
  double reach_hint_ = -1.0;  // ... and its reached vertices with an edge (< 0 unknown)
  int bin_shift_ = 12;
  int64_t nbins_ = 0;
  bool binned_ = false;
  static constexpr int kBinGrid = 1024;
  int64_t td_grid_ = 1, td_grid_filter_ = 1;
  bool seed_gather_ = false;
  uint64_t late_ticks_ = 0;  // DBFS_FAULT_INJECT=kind=late_wg (TdSparseArgs::late_ticks)
  LevelCtrl init_;
  UpdateArgs ua_;  // the update's fields common to every chain

  // ---- per-level records of what was enqueued ----
  std::vector<char> enq_dir_, enq_form_, enq_gather_, enq_fused_;
  std::vector<const FrontierTable*> enq_push_;  // level L's output pushed (Chain::push)
  std::vector<int64_t> enq_cap_;
  std::vector<std::pair<int, int>> evs_;
  RunResult res_;

  // ---- host timing (DBFS_HOST_TIMING=1: enqueue / stamp-wait timeline to stderr) ----
  const bool ht_ = [] {
    const char* e = std::getenv("DBFS_HOST_TIMING");
    return e && *e == '1';
  }();
  std::chrono::steady_clock::time_point t0_;
  std::vector<std::pair<std::string, double>> htl_;
  void hmark(const std::string& what);
  std::string describe(int waiting) const;

  void setup();
  word_t* fr_own(int k) const { return e_.frontier_[k].data() + me_ * W_; }
  // stats block of level L's output (L = -1: the seed): kStatsBlocks blocks
  // in turn with several ranks, two with one rank.  (One rank needs two: a
  // kernel that finishes its level in its last workgroup -- td_sparse -- has
  // workgroups that return before its ticket, past the level's active count,
  // and one dispatched after that finish re-reads its input totals.  With one
  // block it read the NEXT level's totals, ran them against this level's work
  // list and took a ticket the next sparse level then missed: round 5's wrong
  // levels and missing stamp, root 0 of RMAT-16.  With the input block apart
  // from the output block it finds the same active count and returns.
  // tests/test_gpu_engine.py::test_sparse_level_late_workgroups_gpu makes
  // every such workgroup late.)
  int64_t* sblk(int L) const {
    const int blocks = xc_ ? Engine::kStatsBlocks : Engine::kStatsBlocks1;
    return e_.stats_.data() + static_cast<int64_t>((L + 1) % blocks) * e_.stats_stride_;
  }
  static int slot(int level) { return (level + 1) % kMailboxSlots; }
  // work-list set k (level L reads set L & 1; one set without sparse levels)
  int64_t* qscan_set(int k) const { return sparse_ && (k & 1) ? e_.qscan2_.data() : e_.qscan_.data(); }
  int64_t* qbase_set(int k) const { return sparse_ && (k & 1) ? e_.qbase2_.data() : e_.qbase_.data(); }
  int32_t* blk_set(int k) const { return sparse_ && (k & 1) ? e_.blk_vstart2_.data() : e_.blk_vstart_.data(); }
  uint32_t* group_tickets();
  bool cells_fit() const { return e_.g_.rows() < (int64_t(1) << 32) && e_.g_.nnz() < (int64_t(1) << 40); }
  const volatile LevelMailbox* wait_stamp(int lv);
  LevelFinishArgs finish_args(int level, bool seed, char expect_dir, int64_t cap);
  void finish_ranks(int level, bool seed, char expect_dir, int64_t cap, bool gather);
  ScanArgs scan_args(int level, bool seed, char expect_dir, int64_t cap);

  // ---- planner ----
  char td_form(int L, double mf, int64_t* cap, bool exact) const;
  bool chain_valid(int L, char dir, int64_t mf) const;
  void predict(LevelCtrl& c, double nf, double mf, double pnf, double pmf, double reached, bool first, bool rising,
               double* enf, double* emf) const;

  // ---- emitters ----
  void enqueue_level(int L, char d, int64_t cap, double mf_hint, bool gather);
  void compact(const Chain& c, word_t* clear_all);
  void emit_sparse(Chain& c);
  void emit_binned(Chain& c);
  void emit_dense(Chain& c);
  void emit_bottom_up(Chain& c);
  void fuse_update(Chain& c, UpdateArgs& tu);

  RunResult collect(int nlev, std::chrono::steady_clock::time_point t1);
};

// A failed wait, self-described: the source, the level waited for, every
// chain enqueued (level, form, cap), the mailbox slots (level, direction, n_f,
// m_f, done) and the device records of the levels that finished.
std::string DeviceLoop::describe(int waiting) const {
  std::string s = "source " + std::to_string(src_) + ", waiting for level " + std::to_string(waiting) + "; chains";
  for (const auto& ch : res_.chains) s += " " + std::to_string(ch.level) + ch.form + ":" + std::to_string(ch.cap);
  s += "; mailbox";
  for (int i = 0; i < kMailboxSlots; ++i) {
    const volatile LevelMailbox* mb = e_.mailbox_host_ + i;
    if (mb->level < -1) continue;
    s += " [" + std::to_string(mb->level) + " " + static_cast<char>(mb->next_dir) + " nf=" + std::to_string(mb->n_f) +
         " mf=" + std::to_string(mb->m_f) + (mb->done ? " done" : "") + "]";
  }
  s += "; records";
  for (int L = 0; L < waiting && static_cast<size_t>(L / Engine::kRecSeg) < e_.rec_segs_.size(); ++L) {
    const volatile LevelRecDev* r = e_.rec_segs_[static_cast<size_t>(L / Engine::kRecSeg)].first + L % Engine::kRecSeg;
    s += " [" + std::to_string(L) + " " + static_cast<char>(r->dir) + " nf=" + std::to_string(r->n_f) +
         " mf=" + std::to_string(r->m_f) + " new=" + std::to_string(r->discovered) + "]";
  }
  return s;
}

void DeviceLoop::hmark(const std::string& what) {
  htl_.emplace_back(what, std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0_).count());
}

uint32_t* DeviceLoop::group_tickets() {
  // two-level tickets (fused update finish, sparse levels read from a bitmap):
  // zero between launches, each user re-zeroes what it took
  if (!e_.td_group_ticket_.data()) {
    e_.td_group_ticket_ = DBuf<uint32_t>(be_, static_cast<size_t>(kFusedGroups * kBuQueueStride));
    be_.memset_async(e_.td_group_ticket_.data(), 0, e_.td_group_ticket_.bytes());
  }
  return e_.td_group_ticket_.data();
}

// Allocations, run constants, the once-per-graph degree moments.
void DeviceLoop::setup() {
  e_.alloc_bitmap_state();
  W_ = part_.slice_words();
  GW_ = part_.global_words();
  me_ = comm_.rank();
  P_ = part_.nranks;
  xc_ = e_.exchange();
  gv_ = e_.g_.view();
  if (!e_.ctrl_.data()) e_.ctrl_ = DBuf<LevelCtrl>(be_, 1);
  if (!e_.mailbox_host_) {
    void* dptr = nullptr;
    e_.mailbox_host_ = static_cast<LevelMailbox*>(be_.alloc_mapped(sizeof(LevelMailbox) * kMailboxSlots, &dptr));
    e_.mailbox_dev_ = static_cast<LevelMailbox*>(dptr);
  }
  // one rank with narrow levels: byte-map levels write the levels directly
  direct_ = !xc_ && e_.run_narrow_ && opt_.td_direct;
  byte_edges_ = direct_ ? opt_.td_direct_edges : opt_.td_byte_edges;
  bytes_ok_ = opt_.mode != Mode::BottomUp && byte_edges_ <= e_.total_directed_;
  if (bytes_ok_ && !e_.next_bytes_.data()) {
    e_.next_bytes_ = DBuf<uint8_t>(be_, static_cast<size_t>(GW_) * kWordBits);
    be_.memset_async(e_.next_bytes_.data(), 0, e_.next_bytes_.bytes());
  }
  // (several ranks too: remote claims travel as owner lists, td_sparse_apply
  // settles them on their owner)
  sparse_ = e_.sparse_enabled();
  // A sparse chain is live up to this many frontier edges; a level that turns
  // out larger (a geometric prediction can be off by 100x on the second
  // level) is re-enqueued dense: fetch-or claims on every edge cost more than
  // a dense level's fixed passes from there on.
  // (Only with the predicting loop, which enqueues one chain ahead: without
  // prediction the next level's chain is already queued behind a chain found
  // invalid, and a chain of the right direction would run out of turn -- so
  // there only direction mismatches invalidate a chain, and level 0 is never
  // a list chain.)
  sparse_cap_ = opt_.device_loop_predict && opt_.td_sparse_cap_factor > 0
                    ? std::max<int64_t>(opt_.td_sparse_edges,
                                        static_cast<int64_t>(opt_.td_sparse_cap_factor *
                                                             static_cast<double>(opt_.td_sparse_edges)))
                    : 0;
  // Several ranks: a sparse chain is live while the level's global frontier
  // edges fit its owner lists (every rank sends any peer at most that many
  // ids); predicted levels up to xsparse_lim go sparse.
  // (a rank appends each remote vertex at most once per run -- it claims the
  // vertex's bit in its replicated visited bitmap first -- so no list ever
  // holds more than a rank's part: lists of that capacity never overflow)
  list_max_ = xc_ && sparse_ && opt_.list_form_edges > 0 ? std::min<int64_t>(opt_.list_form_edges, part_.part) : 0;
  lists_unlimited_ = list_max_ > 0 && list_max_ >= part_.part;
  xsparse_lim_ = std::min<int64_t>(opt_.xsparse_edges, list_max_);
  counted_ = comm_.counted_lists();
  // tiny sparse chains (several ranks, counted lists): live up to fuse_cap
  fuse_cap_ = xc_ && counted_ && opt_.xfuse_edges > 0 && 4 * opt_.xfuse_edges < list_max_ ? 4 * opt_.xfuse_edges : 0;
  if (list_max_ > 0 && e_.list_stride_ < list_max_ + 1) {
    // owner lists: count word + list_max ids, the stride a multiple of 4 words
    // (16-byte pieces for the count-sized exchange); counts zeroed once here
    // and by every td_sparse_apply after
    e_.list_stride_ = (list_max_ + 1 + 3) / 4 * 4;
    const size_t n = static_cast<size_t>(P_) * static_cast<size_t>(e_.list_stride_);
    e_.dl_send_lists_ = DBuf<vid_t>(be_, n);
    e_.dl_recv_lists_ = DBuf<vid_t>(be_, n);
    be_.memset_async(e_.dl_send_lists_.data(), 0, e_.dl_send_lists_.bytes());
    be_.memset_async(e_.dl_recv_lists_.data(), 0, e_.dl_recv_lists_.bytes());
  }
  if (sparse_ && !e_.sparse_ready_) {
    const size_t rows = static_cast<size_t>(std::max<int64_t>(e_.g_.rows(), 1));
    e_.qscan2_ = DBuf<int64_t>(be_, rows + 1);
    e_.qbase2_ = DBuf<int64_t>(be_, rows);
    e_.blk_vstart2_ = DBuf<int32_t>(be_, static_cast<size_t>(div_up(e_.g_.nnz(), kTdEdgesPerBlock) + 2));
    e_.qv_[0] = DBuf<vid_t>(be_, rows);
    e_.qv_[1] = DBuf<vid_t>(be_, rows);
    e_.sparse_cnt_ = DBuf<unsigned long long>(be_, 2);
    e_.sparse_ticket_ = DBuf<unsigned>(be_, 1);
    be_.memset_async(e_.sparse_cnt_.data(), 0, e_.sparse_cnt_.bytes());
    be_.memset_async(e_.sparse_ticket_.data(), 0, e_.sparse_ticket_.bytes());
    e_.sparse_ready_ = true;
  }
  // One rank, binned top-down levels: bins of 2^shift vertices (>= one
  // 4096-vertex unit, <= 2^kBinMaxShift so a bin's visited slice fits LDS),
  // about 256 of them (up to kBinMaxBins).
  {
    int bits = 0;
    while ((int64_t(1) << bits) < W_ * kWordBits) ++bits;
    bin_shift_ = std::min(std::max(bits - static_cast<int>(opt_.td_bin_log2_bins), 12), kBinMaxShift);
    while (bin_shift_ <= kBinMaxShift && div_up(W_ * kWordBits, int64_t(1) << bin_shift_) > kBinMaxBins) ++bin_shift_;
  }
  nbins_ = div_up(W_ * kWordBits, int64_t(1) << bin_shift_);
  binned_ = !xc_ && opt_.td_bin_edges > 0 && opt_.mode != Mode::BottomUp && bin_shift_ <= kBinMaxShift &&
            e_.g_.nnz() > 0 && e_.g_.rows() >= opt_.td_bin_min_rows;
  if (binned_ && (e_.bin_buf_.size() < static_cast<size_t>(e_.g_.nnz()) ||
                  e_.bin_cnt_.size() < static_cast<size_t>(nbins_ * kBinGrid))) {
    e_.bin_total_ = DBuf<int64_t>(be_, static_cast<size_t>(nbins_));
    e_.bin_cnt_ = DBuf<uint32_t>(be_, static_cast<size_t>(nbins_ * kBinGrid));
    e_.bin_buf_ = DBuf<vid_t>(be_, static_cast<size_t>(e_.g_.nnz()));  // a level's frontier edges <= nnz
  }
  if (e_.n_active_ < 0) {
    // (outside the timed window, once) the mean degree of an edge's endpoint
    // (sum deg^2 / sum deg) predicts the edges of level 1's frontier (the
    // source's neighbours) from the source's degree; the number of vertices
    // with edges bounds every later frontier by those not reached yet
    be_.degree_moments(gv_, e_.stats_.data() + 4);
    if (xc_) comm_.allreduce_sum_i64(e_.stats_.data() + 4, 2);
    int64_t mom[2] = {0, 0};
    be_.to_host(mom, e_.stats_.data() + 4, sizeof(mom));
    e_.excess_degree_ =
        e_.total_directed_ > 0 ? static_cast<double>(mom[0]) / static_cast<double>(e_.total_directed_) : 0.0;
    e_.n_active_ = mom[1];
  }
  const int64_t td_blocks = div_up(e_.g_.nnz(), kTdEdgesPerBlock);
  td_grid_ = std::max<int64_t>(1, std::min<int64_t>(td_blocks, opt_.td_grid_max));
  td_grid_filter_ = std::max<int64_t>(1, std::min<int64_t>(td_blocks, opt_.td_grid_filter_max));
  if (e_.fault_.kind == "late_wg")
    late_ticks_ = static_cast<uint64_t>(static_cast<double>(e_.fault_.us) * be_.wall_clock_khz() / 1000.0);
  // Mailbox stamps can be reset although the previous run did not end with a
  // synchronize: its trailing (speculative) chain may still be executing, but
  // every kernel that stamps a mailbox slot (scan_units, level_finish,
  // td_sparse, init_run with a ctrl) returns at entry once ctrl->done is set,
  // and the previous run's last stamp set it -- so nothing of that run writes
  // a slot again.  (tests/test_gpu_engine.py::test_back_to_back_runs_*)
  for (int i = 0; i < kMailboxSlots; ++i) {
    volatile LevelMailbox* mb = e_.mailbox_host_ + i;
    mb->level = -2;
  }
  e_.rec_at(0);  // the first record segment, outside the timed window
}

// Wait until level `lv` (-1 = seed) has stamped its mailbox slot.
const volatile LevelMailbox* DeviceLoop::wait_stamp(int lv) {
  const volatile LevelMailbox* mb = e_.mailbox_host_ + slot(lv);
  spin_until(be_, [&] { return __atomic_load_n(&mb->level, __ATOMIC_ACQUIRE) == lv; },
            "device level loop: a level finished without its mailbox stamp");
  return mb;
}

LevelFinishArgs DeviceLoop::finish_args(int level, bool seed, char expect_dir, int64_t cap) {
  LevelFinishArgs fa;
  fa.stats = sblk(level);
  fa.ctrl = e_.ctrl_.data();
  fa.ctrl_init = init_;
  fa.rec = seed ? nullptr : e_.rec_at(level);
  fa.mailbox = e_.mailbox_dev_ + slot(level);
  fa.level = level;
  fa.seed = seed;
  fa.expect_dir = expect_dir;
  fa.expect_cap = cap;
  return fa;
}

// Several ranks: the level's ONE collective -- its totals (stats block)
// all-reduced, and with `gather` (the next level is predicted bottom-up, or
// td mode, whose top-down levels filter with the replicated visited bitmap)
// in the same launch the level's output frontier slice all-gathered
// (Comm::allgather_allreduce) -- then level_finish decides and stamps.
// (bfs_mpi.cu:615-621 pays a Sendrecv and an Allreduce per level.)
void DeviceLoop::finish_ranks(int level, bool seed, char expect_dir, int64_t cap, bool gather) {
  int64_t* blk = sblk(level);
  // level L writes frontier_[L & 1] (the seed: frontier_[1])
  const int out = seed ? 1 : (level & 1);
  const LevelFinishArgs fa = finish_args(level, seed, expect_dir, cap);
  comm_.level_end(fr_own(out), e_.frontier_[out].data(), gather ? static_cast<size_t>(W_) * sizeof(word_t) : 0,
                  blk + 2, 2, fa);
}

ScanArgs DeviceLoop::scan_args(int level, bool seed, char expect_dir, int64_t cap) {
  ScanArgs sa;
  sa.unit_cnt = e_.unit_cnt_.data();
  sa.unit_deg = e_.unit_deg_.data();
  sa.nunits = e_.nunits_;
  sa.part_cnt = e_.part_cnt_.data();
  sa.part_deg = e_.part_deg_.data();
  sa.ticket = e_.ticket_.data();
  sa.stats = sblk(level);
  sa.qscan = qscan_set(level + 1);
  sa.ctrl = e_.ctrl_.data();
  sa.rec = seed ? nullptr : e_.rec_at(level);
  sa.mailbox = e_.mailbox_dev_ + slot(level);
  sa.level = level;
  sa.seed = seed;
  sa.expect_dir = expect_dir;
  sa.expect_cap = cap;
  sa.finish = !xc_;
  return sa;
}

// ---- planner ------------------------------------------------------------------

// Top-down form of level L whose frontier has (about) mf edges: sparse when
// small (right after a bottom-up level too: the compaction then zeroes the
// bottom-up input bitmap the sparse level writes into); *cap: the global
// frontier edges a sparse chain stays live for.  (exact: mf is the level's
// actual frontier edges -- a re-enqueue, which must be live.)
char DeviceLoop::td_form(int L, double mf, int64_t* cap, bool exact) const {
  *cap = 0;
  if (xc_) {
    if (list_max_ <= 0) return 'T';
    if (counted_) {
      // count-sized exchange: the largest lists cost nothing extra (cap 0:
      // lists of a whole part, live for any level)
      if (!exact && mf > static_cast<double>(xsparse_lim_)) return 'T';
      if (exact && !lists_unlimited_ && mf > static_cast<double>(list_max_)) return 'T';
      *cap = lists_unlimited_ ? 0 : list_max_;
      // tiny levels: chains capped at fuse_cap (fused into one launch on a
      // direct transport; the same chains on every transport, so a shadow
      // replay follows its recording)
      if (fuse_cap_ > 0 &&
          (exact ? mf <= static_cast<double>(fuse_cap_) : mf <= static_cast<double>(opt_.xfuse_edges)))
        *cap = fuse_cap_;
      return 'S';
    }
    // fixed-size exchange (cap + 1 ids per peer): lists sized for the
    // level, list_cap_factor x the prediction (at least the actual edges
    // of a re-enqueued level), a power of two >= 1024, and no larger than a
    // bitmap slice's worth of ids (past that the dense form ships less)
    const int64_t lim = std::min(list_max_, std::max<int64_t>(W_, 1024));
    const double want = std::max(1024.0, exact ? mf : mf * opt_.list_cap_factor);
    if (want > static_cast<double>(lim) || (!exact && mf > static_cast<double>(xsparse_lim_))) return 'T';
    int64_t c = 1024;
    while (static_cast<double>(c) < want) c <<= 1;
    *cap = std::min(c, lim);
    return 'S';
  }
  const char pf = L == 0 ? 'I' : enq_form_[static_cast<size_t>(L - 1)];
  // right after a bottom-up level: sparse up to td_sparse_bu_edges, the
  // chain live up to that many too (the prediction of a shrinking frontier
  // overshoots, and that level reads the bottom-up output bitmap directly);
  // elsewhere up to td_sparse_edges, live up to sparse_cap
  const bool post_bu = pf == 'B' && opt_.td_sparse_bu_edges > opt_.td_sparse_edges;
  int64_t lim = post_bu ? opt_.td_sparse_bu_edges : opt_.td_sparse_edges;
  const int64_t live = post_bu && sparse_cap_ > 0 ? std::max(sparse_cap_, opt_.td_sparse_bu_edges) : sparse_cap_;
  if (live > 0) lim = std::min(lim, live);  // (a sparse chain must stay live for mf)
  if (sparse_ && mf <= static_cast<double>(lim)) {
    *cap = live;
    return 'S';
  }
  bool after_bu = false;  // (binned only before the run's first bottom-up level)
  for (int k = 0; k < L && !after_bu; ++k) after_bu = enq_form_[static_cast<size_t>(k)] == 'B';
  // ... and not for a level the direct form does better: one of 16 x
  // td_split_edges or more (split in parts), or one late enough for the
  // unvisited filter (top-down only on RMAT-26: 0.5 B-edge level 5.6 -> 4.3
  // ms, the filter levels 21.3 -> 10.8 and 0.72 -> 0.42 ms)
  const bool huge = opt_.td_split_edges > 0 && mf >= 16.0 * static_cast<double>(opt_.td_split_edges);
  const bool late = opt_.td_unvis_edges > 0 && vis_hint_ >= opt_.td_unvis_vis_frac * static_cast<double>(e_.total_directed_);
  return binned_ && !after_bu && !huge && !late && mf >= static_cast<double>(opt_.td_bin_edges) ? 'X' : 'T';
}

// the chain enqueued for level L is live for a level with direction `dir`
// and mf global frontier edges
bool DeviceLoop::chain_valid(int L, char dir, int64_t mf) const {
  if (enq_dir_[L] != dir) return false;
  return enq_form_[L] != 'S' || enq_cap_[L] <= 0 || mf <= enq_cap_[L];
}

// One prediction step: from a level with frontier (nf, mf), its
// predecessor's (pnf, pmf) and `reached` vertices so far, the next level's
// frontier extrapolated geometrically (never more than the vertices with
// edges not reached yet) and its direction through level_ctrl_finish (c
// holds the known level's direction and totals on entry).
void DeviceLoop::predict(LevelCtrl& c, double nf, double mf, double pnf, double pmf, double reached, bool first,
                         bool rising, double* enf, double* emf) const {
  auto grow = [](double cur, double prev) { return prev <= 0 ? cur * cur : cur * (cur / prev); };
  const double unreached = std::max(0.0, static_cast<double>(e_.n_active_) - reached);
  *enf = std::min({grow(nf, pnf), static_cast<double>(part_.n), unreached});
  // level 1's frontier edges: the source's neighbours have the mean endpoint degree
  *emf = std::min(first ? mf * std::max(1.0, e_.excess_degree_) : grow(mf, pmf),
                  static_cast<double>(e_.total_directed_));
  const LevelCtrl c0 = c;
  LevelRecDev scratch;
  level_ctrl_finish(c, std::max<int64_t>(1, static_cast<int64_t>(*enf)), static_cast<int64_t>(*emf), false, &scratch);
  // Rising phase (no bottom-up level yet): each frontier edge finds about one
  // new vertex, of the mean endpoint degree.  Taken only when that estimate
  // turns the decision bottom-up -- a root whose few neighbours are hubs (1
  // -> 1 vertex but 1 -> 17 K edges: the vertex count's growth says
  // top-down; RMAT-26's late-switch roots, 91-153 M edges bottom-up, cost a
  // wasted chain and a host round trip each); the edge estimate would
  // otherwise oversize the forms of levels that stay top-down.
  // (A/B, same box, 128 held-out RMAT-26 roots twice each: mispredicted
  // levels 34 -> 19, 1489 / 1498 -> 1504 / 1506 GTEPS; profiles/r6_predictor_ab.txt)
  if (rising && !first && e_.n_active_ > 0 && c.dir != 'B') {
    const double e = std::min(mf, unreached);
    const double em = std::max(*emf, std::min(e * std::max(1.0, e_.excess_degree_), static_cast<double>(e_.total_directed_)));
    if (e > *enf) {
      LevelCtrl c2 = c0;
      level_ctrl_finish(c2, std::max<int64_t>(1, static_cast<int64_t>(e)), static_cast<int64_t>(em), false, &scratch);
      if (c2.dir == 'B') {
        c = c2;
        *enf = e;
        *emf = em;
      }
    }
  }
}

// ---- emitters -------------------------------------------------------------------

// mf_hint: the level's predicted (or, re-enqueued, actual) frontier edges
// (< 0 unknown); gather (several ranks): the chain's collective also
// all-gathers its output frontier, for a bottom-up level predicted next.
void DeviceLoop::enqueue_level(int L, char d, int64_t cap, double mf_hint, bool gather) {
  if (ht_) hmark("enqueue " + std::to_string(L) + d);
  comm_.set_level_tag(L);  // (a failed collective of this chain names its level)
  if (static_cast<size_t>(L) >= enq_dir_.size()) {
    e_.inject_fault(L);
    enq_dir_.resize(static_cast<size_t>(L) + 1);
    enq_form_.resize(static_cast<size_t>(L) + 1);
    enq_cap_.resize(static_cast<size_t>(L) + 1);
    enq_gather_.resize(static_cast<size_t>(L) + 1);
    enq_fused_.resize(static_cast<size_t>(L) + 1);
    enq_push_.resize(static_cast<size_t>(L) + 1);
    evs_.resize(static_cast<size_t>(L) + 1, {-1, -1});
  }
  Chain c;
  c.L = L;
  c.d = d;
  // the previous level's form decides what hands this one its work list
  c.pf = L == 0 ? 'I' : enq_form_[static_cast<size_t>(L - 1)];
  // the input frontier is already global: all-gathered by the previous
  // level's (or the seed's) collective
  c.in_gathered = L == 0 ? seed_gather_ : enq_gather_[static_cast<size_t>(L - 1)] != 0;
  enq_dir_[L] = d == 'B' ? 'B' : 'T';
  enq_form_[L] = d;
  enq_cap_[L] = d == 'S' ? cap : 0;
  enq_gather_[L] = xc_ && gather;
  // (the pushed slices are copied in by hub_gather: graphs with hubs; the
  // table's parity is the level's -- see FrontierTable)
  c.pull = L > 0 ? enq_push_[static_cast<size_t>(L - 1)] : nullptr;
  c.push = enq_gather_[L] && opt_.direct_frontier && gv_.nhubs > 0 && (d == 'T' || d == 'B')
               ? comm_.direct_frontier(static_cast<size_t>(W_), L & 1)
               : nullptr;
  enq_push_[L] = c.push;
  res_.chains.push_back({L, d, enq_cap_[L], enq_gather_[L] != 0});
  res_.chains.back().push = c.push != nullptr;
  c.cap = enq_cap_[L];
  c.mf_hint = mf_hint;
  c.cur = (L + 1) & 1;
  char trace_name[48];
  std::snprintf(trace_name, sizeof(trace_name), "bfs.level %d %c (enqueue)", L, d);
  TraceRange trace_level(trace_name);
  const int ev0 = opt_.phase_timing ? be_.record_event() : -1;
  // several ranks, bottom-up: the input frontier to every rank -- normally
  // gathered already by the previous level's collective; a chain enqueued
  // after a top-down prediction gathers it here (not predicated: on a no-op
  // chain it only refreshes bits every owner already has)
  if (xc_ && d == 'B') {
    if (!c.in_gathered)
      comm_.allgather(fr_own(c.cur), e_.frontier_[c.cur].data(), static_cast<size_t>(W_) * sizeof(word_t));
    // (bu_merge_visited: the remote slices merged into the replicated
    // visited bitmap -- by hub_gather with hubs)
    if (opt_.bu_merge_visited && gv_.nhubs == 0)
      be_.bitmap_or(e_.visited_.data(), e_.frontier_[c.cur].data(), GW_);
  }
  switch (d) {
    case 'S': emit_sparse(c); break;
    case 'X': emit_binned(c); break;
    case 'T': emit_dense(c); break;
    default: emit_bottom_up(c); break;
  }
  if (!c.fused_scan) be_.scan_units(scan_args(L, false, enq_dir_[L], c.cap));
  enq_fused_[L] = c.fused_scan && d != 'S' && !c.folded;
  if (xc_ && !c.level_ended)
    finish_ranks(L, false, enq_dir_[L], c.cap, enq_gather_[L] && !c.push);
  if (opt_.phase_timing) evs_[L] = {ev0, be_.record_event()};
  if (ht_) hmark("enqueued " + std::to_string(L));
}

// The frontier bitmap -> work list (set L & 1); with sparse levels also its
// vertex map, and the bitmap is zeroed as read (a later sparse level writes
// into it).
void DeviceLoop::compact(const Chain& c, word_t* clear_all) {
  const int L = c.L;
  if (L > 0 && enq_fused_[static_cast<size_t>(L - 1)]) {
    // the previous level only finished its totals: its unit prefixes now (no
    // finish; a no-op unless this chain is live)
    ScanArgs sa = scan_args(L - 1, false, 'T', c.d == 'S' ? c.cap : 0);
    sa.finish = false;
    be_.scan_units(sa);
  }
  CompactArgs ca;
  ca.g = gv_;
  ca.frontier = fr_own(c.cur);
  ca.words = W_;
  ca.unit_cnt_off = e_.unit_cnt_.data();
  ca.unit_deg_off = e_.unit_deg_.data();
  ca.part_cnt = e_.part_cnt_.data();
  ca.part_deg = e_.part_deg_.data();
  ca.qscan = qscan_set(L);
  ca.qbase = qbase_set(L);
  ca.blk_vstart = blk_set(L);
  if (sparse_) {
    ca.qv = e_.qv_[L & 1].data();
    ca.clear = fr_own(c.cur);
  }
  ca.clear_all = clear_all;
  ca.ctrl = e_.ctrl_.data();
  ca.max_mf = c.d == 'S' ? c.cap : 0;
  be_.compact_frontier(ca);
}

// 'S': a sparse top-down level -- td_sparse claims every target with a
// fetch-or on visited and settles it in place (one rank: the whole level in
// one launch); with several ranks remote claims go to their owners' lists,
// exchanged count-sized (or stored by the kernel into the owners' windows),
// and td_sparse_apply settles the received ids.
void DeviceLoop::emit_sparse(Chain& c) {
  const int L = c.L;
  DBFS_CHECK(sparse_, "sparse top-down level without sparse support");
  // after a bottom-up level the output bitmap is that level's input: zeroed
  // by the compaction (every other form leaves it clean)
  const bool compacted = c.pf == 'T' || c.pf == 'X' || c.pf == 'B';
  // right after a bottom-up level: the kernel reads that level's output
  // bitmap itself (no unit scan, no compaction); only the stale output bitmap
  // is cleared first
  const bool from_bits = c.pf == 'B' && opt_.td_sparse_bits;
  if (from_bits) be_.memset_async(fr_own(c.cur ^ 1), 0, static_cast<size_t>(W_) * sizeof(word_t));
  else if (compacted) compact(c, c.pf == 'B' ? fr_own(c.cur ^ 1) : nullptr);
  TdSparseArgs sp;
  sp.g = gv_;
  sp.qscan = qscan_set(L);
  sp.qbase = qbase_set(L);
  sp.blk_vstart = blk_set(L);
  sp.qv = e_.qv_[L & 1].data();
  sp.dev_stats = sblk(L - 1);
  sp.frontier_in = fr_own(c.cur);
  sp.frontier_out = fr_own(c.cur ^ 1);
  sp.visited = e_.visited_.data();
  sp.level = e_.level_.data();
  sp.level8 = e_.run_narrow_ ? e_.level8_.data() : nullptr;
  sp.narrow_base = e_.narrow_base_;
  sp.new_level = L + 1;
  sp.oscan = qscan_set(L + 1);
  sp.obase = qbase_set(L + 1);
  sp.oblk = blk_set(L + 1);
  sp.oqv = e_.qv_[(L + 1) & 1].data();
  sp.counter = e_.sparse_cnt_.data() + ((L + 1) & 1);
  sp.ticket = e_.sparse_ticket_.data();
  sp.stats = sblk(L);
  sp.ctrl = e_.ctrl_.data();
  sp.rec = e_.rec_at(L);
  sp.mailbox = e_.mailbox_dev_ + slot(L);
  sp.level_index = L;
  sp.grid = std::max<int64_t>(1, opt_.td_sparse_grid);
  sp.late_ticks = late_ticks_;
  sp.first = !compacted || from_bits;
  sp.max_mf = c.cap;
  if (from_bits) {
    sp.from_bits = true;
    sp.words = W_;
    sp.group_ticket = group_tickets();
  }
  c.fused_scan = true;
  if (!xc_) {
    be_.td_sparse(sp);
    return;
  }
  // remote claims to their owners' lists, the lists (count-sized) to their
  // owners, the received ids settled there; the totals go to the collective
  // (no decision in the kernels)
  DBFS_CHECK(list_max_ > 0 && c.cap <= list_max_, "sparse chain without owner lists");
  sp.lists = e_.dl_send_lists_.data();
  sp.list_stride = e_.list_stride_;
  sp.part = part_.part;
  sp.mailbox = nullptr;
  // the exchange itself: by the two kernels through the peers' windows
  // (direct), or a collective between them
  const size_t lcap = static_cast<size_t>(c.cap > 0 ? c.cap : list_max_);
  const bool direct = comm_.direct_lists(lcap, &sp.direct);
  sp.nranks = P_;
  // the owners' side sized by its expected ids (a rank receives about
  // mf (P - 1) / P^2 claims): ~512 per workgroup, up to td_apply_grid -- the
  // large levels' latency-bound claims spread over every CU, a tiny level's
  // launch stays small
  const double est_mf = c.mf_hint >= 0 ? c.mf_hint : static_cast<double>(c.cap > 0 ? c.cap : list_max_);
  const double est_ids = est_mf * static_cast<double>(P_ - 1) / (static_cast<double>(P_) * P_);
  int64_t apply_grid =
      std::max<int64_t>(1, std::min<int64_t>(opt_.td_apply_grid, static_cast<int64_t>(est_ids / 512.0) + 1));
  // (ranks sharing a GPU with the waits inside the apply -- every workgroup
  // spins on the peers' cells: at most 64 1024-thread workgroups over all of
  // them, an eighth of the chip's residency, so a peer's td_sparse always
  // finds CUs)
  if (comm_.coresident() > 1 && !comm_.split_waits())
    apply_grid = std::min<int64_t>(apply_grid, std::max(1, 64 / comm_.coresident()));
  // the level's end folded into the apply's last workgroup (no frontier
  // gather: that one is a bandwidth collective of its own)
  // (the cells carry < 2^32 new vertices and < 2^40 degrees per rank)
  const bool end_ok = direct && cells_fit() && !enq_gather_[L];
  // a tiny level (its chain capped at fuse_cap): td_sparse's last workgroup
  // also runs the owner side and the level end -- one launch (the direct
  // level end is taken in the same order as unfused)
  sp.fuse_apply = end_ok && fuse_cap_ > 0 && c.cap > 0 && c.cap <= fuse_cap_;
  if (sp.fuse_apply) {
    sp.recv_lists = nullptr;
    if (comm_.direct_level_end(2, &sp.end)) {
      sp.fin = finish_args(L, false, enq_dir_[L], c.cap);
      c.level_ended = true;
    } else {
      sp.fuse_apply = false;  // (not taken: the level ends in its collective)
    }
    be_.td_sparse(sp);
    sp.grid = apply_grid;
    if (!c.level_ended) be_.td_sparse_apply(sp);
    return;
  }
  be_.td_sparse(sp);
  if (!direct)
    comm_.alltoall_lists(e_.dl_send_lists_.data(), e_.dl_recv_lists_.data(), static_cast<size_t>(e_.list_stride_),
                         lcap);
  sp.recv_lists = direct ? nullptr : e_.dl_recv_lists_.data();
  if (end_ok && comm_.direct_level_end(2, &sp.end)) {
    sp.fin = finish_args(L, false, enq_dir_[L], c.cap);
    c.level_ended = true;
  }
  sp.grid = apply_grid;
  // ranks sharing a GPU: the wait for the peers' cells as a one-wave launch
  // first, so the apply's grid never spins in every workgroup while a peer's
  // td_sparse still needs CUs (Comm::split_waits)
  if (direct && comm_.split_waits()) be_.direct_prewait(sp.direct);
  be_.td_sparse_apply(sp);
}

// 'X': binned top-down (one rank): targets binned by vertex range, claimed
// per bin in LDS; a sparse level (or the seed) handed over the work list,
// else compact.
void DeviceLoop::emit_binned(Chain& c) {
  const int L = c.L;
  const bool listed = sparse_ && (c.pf == 'S' || c.pf == 'I');
  if (!listed) compact(c, nullptr);
  BinArgs xa;
  xa.g = gv_;
  xa.qscan = qscan_set(L);
  xa.qbase = qbase_set(L);
  xa.blk_vstart = blk_set(L);
  xa.dev_stats = sblk(L - 1);
  if (listed) {
    xa.clear_qv = e_.qv_[L & 1].data();
    xa.clear_frontier = fr_own(c.cur);
  }
  xa.ctrl = e_.ctrl_.data();
  xa.shift = bin_shift_;
  xa.nbins = static_cast<int>(nbins_);
  xa.grid = kBinGrid;
  xa.bin_total = e_.bin_total_.data();
  xa.cnt = e_.bin_cnt_.data();
  xa.buf = e_.bin_buf_.data();
  xa.visited = e_.visited_.data() + me_ * W_;
  xa.frontier = fr_own(c.cur ^ 1);
  xa.words = W_;
  be_.td_binned(xa);
  // levels and unit statistics of the new frontier (already claimed)
  UpdateArgs tu = ua_;
  tu.cand = fr_own(c.cur ^ 1);
  tu.cand_bytes = nullptr;
  tu.nchunks = 1;
  tu.clear_cand = false;
  tu.force = true;
  tu.frontier = fr_own(c.cur ^ 1);
  tu.new_level = L + 1;
  tu.ctrl = e_.ctrl_.data();
  be_.update_frontier(tu);
}

// The update's fused finish: the level's totals (and with one rank its
// decision) in its last workgroup, as bottom-up.
void DeviceLoop::fuse_update(Chain& c, UpdateArgs& tu) {
  if (!e_.td_tot_.data()) e_.td_tot_ = DBuf<int64_t>(be_, static_cast<size_t>(2 * kMaxFusedGrid + 2 * kFusedGroups));
  tu.fuse_scan = true;
  tu.scan = scan_args(c.L, false, enq_dir_[c.L], c.cap);
  // small graphs: the next compaction's unit prefixes too (no scan_units launch)
  tu.fold_scan = opt_.fold_scan && e_.nunits_ <= kFoldScanUnits;
  c.folded = tu.fold_scan;
  tu.tot = e_.td_tot_.data();
  if (opt_.td_group_ticket) tu.group_ticket = group_tickets();
  c.fused_scan = true;
}

// 'T': a dense top-down level -- compact (unless a sparse level or the seed
// handed over the work list) -> td_expand (edge-balanced, LDS owner map;
// large levels test hub targets in an LDS snapshot) -> [several ranks: the
// candidate slices to their owners] -> update (fused finish).
void DeviceLoop::emit_dense(Chain& c) {
  const int L = c.L;
  const bool listed = sparse_ && (c.pf == 'S' || c.pf == 'I');
  if (!listed) compact(c, nullptr);
  TdArgs ta;
  ta.g = gv_;
  ta.qscan = qscan_set(L);
  ta.qbase = qbase_set(L);
  ta.blk_vstart = blk_set(L);
  if (listed) {
    ta.clear_qv = e_.qv_[L & 1].data();
    ta.clear_frontier = fr_own(c.cur);
  }
  ta.visited = e_.visited_.data();
  ta.ctrl = e_.ctrl_.data();
  ta.dev_stats = sblk(L - 1);
  ta.grid = td_grid_;
  ta.grid_filter = td_grid_filter_;
  UpdateArgs tu = ua_;
  ta.next = e_.next_.data();
  ta.next_bytes = e_.next_bytes_.data();
  // late large levels: the unvisited filter (launched next to the plain
  // variant; the filter's density picks the one that runs)
  // (and, with the count of vertices with an edge known, a filter expected
  // at most 1.5 x td_unvis_max_density dense: u of the vertices unvisited,
  // n / kUnvisBits per bit -- so a hub-heavy level whose visited edges are
  // many but whose unvisited vertices are too launches nothing extra)
  bool unvis = opt_.td_unvis_edges > 0 && c.mf_hint >= static_cast<double>(opt_.td_unvis_edges) &&
               vis_hint_ >= opt_.td_unvis_vis_frac * static_cast<double>(e_.total_directed_);
  if (unvis && e_.n_active_ > 0 && reach_hint_ >= 0) {
    const double u = std::max(0.0, static_cast<double>(e_.n_active_) - reach_hint_) / static_cast<double>(gv_.n);
    const double per_bit = std::max(1.0, static_cast<double>(gv_.n) / static_cast<double>(kUnvisBits));
    unvis = 1.0 - std::pow(1.0 - std::min(u, 1.0), per_bit) <= 1.5 * opt_.td_unvis_max_density;
  }
  if (unvis) {
    res_.chains.back().unvis = true;
    if (!e_.unvis_.data()) {
      e_.unvis_ = DBuf<word_t>(be_, static_cast<size_t>(kUnvisWords));
      e_.unvis_pop_ = DBuf<uint32_t>(be_, static_cast<size_t>(kUnvisChunks));
    }
    UnvisArgs uv;
    uv.visited = e_.visited_.data();
    uv.n = gv_.n;
    uv.mult = unvis_mult(gv_.n);
    uv.out = e_.unvis_.data();
    uv.pop = e_.unvis_pop_.data();
    uv.ctrl = e_.ctrl_.data();
    uv.max_mf = 0;
    be_.unvis_filter(uv);
    ta.unvis = e_.unvis_.data();
    ta.unvis_mult = uv.mult;
    ta.unvis_pop = uv.pop;
    ta.unvis_max_density = opt_.td_unvis_max_density;
  }
  // (skipped for levels predicted well below the filter's threshold: the
  // snapshot kernel would only find its gate closed)
  if (gv_.td_nhubs > 0 && opt_.td_hub_edges > 0 && e_.g_.td_hub_share() >= opt_.td_hub_min_share &&
      (c.mf_hint < 0 || c.mf_hint * 4.0 >= static_cast<double>(opt_.td_hub_edges))) {
    // large levels: the hubs' visited bits, staged in LDS by td_expand
    if (!e_.td_hub_vis_.data())
      e_.td_hub_vis_ = DBuf<word_t>(be_, static_cast<size_t>(div_up(gv_.td_nhubs, kWordBits)));
    HubVisitedArgs hv;
    hv.g = gv_;
    hv.visited = e_.visited_.data();
    hv.out = e_.td_hub_vis_.data();
    hv.ctrl = e_.ctrl_.data();
    hv.min_edges = opt_.td_hub_edges;
    hv.vis_frac = opt_.td_hub_vis_frac;
    be_.hub_visited(hv);
    ta.td_hub_vis = e_.td_hub_vis_.data();
    ta.td_hub_min_edges = opt_.td_hub_edges;
    ta.td_hub_vis_frac = opt_.td_hub_vis_frac;
  }
  // (a level past kNarrowMaxLevel would store the unreached byte: the usual
  // path flags the overflow and the run is repeated wide)
  if (direct_ && e_.run_narrow_ && L + 1 <= kNarrowMaxLevel) {
    // byte-map levels write the level itself (nothing to clear after)
    ta.level_direct = e_.level8_.data();
    ta.narrow_base = e_.narrow_base_;
    ta.new_level = L + 1;
    tu.level_direct = e_.level8_.data();
    tu.narrow_base = e_.narrow_base_;
    if (ta.td_hub_vis) {
      if (!e_.td_hub_mark_.data()) {
        e_.td_hub_mark_ = DBuf<uint8_t>(be_, static_cast<size_t>(kTdMaxHubs));
        be_.memset_async(e_.td_hub_mark_.data(), 0, e_.td_hub_mark_.bytes());
      }
      ta.td_hub_mark = e_.td_hub_mark_.data();
    }
  }
  // large level-byte levels (one rank): the level in parts, the claims so far
  // ORed into visited between them (Options::td_split_edges)
  // (not with the unvisited filter: a late level claims few vertices, and
  // every part would stage the filter and launch both variants again --
  // RMAT-22's level 4 87 -> 134 us in 4 parts)
  const int parts = (ta.level_direct && !unvis && !xc_ && opt_.td_split_edges > 0 && opt_.td_split_parts > 1 &&
                     c.mf_hint >= static_cast<double>(opt_.td_split_edges))
                        ? opt_.td_split_parts * (c.mf_hint >= 16.0 * static_cast<double>(opt_.td_split_edges) &&
                                                         gv_.n >= (int64_t(1) << 25)
                                                     ? 2
                                                     : 1)
                        : 1;
  if (parts > 1) {
    res_.chains.back().split = parts;
    RefreshArgs ra;
    ra.level8 = ta.level_direct;
    ra.narrow_base = ta.narrow_base;
    ra.new_level = ta.new_level;
    ra.visited = e_.visited_.data();
    ra.words = GW_;
    ra.ctrl = e_.ctrl_.data();
    ra.max_mf = ta.max_mf;
    ta.split_k = parts;
    for (int i = 0; i < parts; ++i) {
      ta.split_i = i;
      be_.td_expand(ta);
      // (the input list's frontier words cleared, the level stamped: once)
      ta.clear_qv = nullptr;
      ta.clear_frontier = nullptr;
      if (i + 1 < parts) be_.refresh_visited(ra);
    }
  } else {
    be_.td_expand(ta);
  }
  if (ta.td_hub_mark) {
    HubApplyArgs ha;
    ha.g = gv_;
    ha.mark = ta.td_hub_mark;
    ha.level8 = ta.level_direct;
    ha.narrow_base = ta.narrow_base;
    ha.new_level = ta.new_level;
    ha.ctrl = e_.ctrl_.data();
    ha.max_mf = ta.max_mf;
    be_.hub_apply(ha);
  }
  tu.cand = e_.next_.data();
  tu.cand_bytes = e_.next_bytes_.data();
  if (xc_) {
    // candidates to their owners: the byte map (if this level used it)
    // packed into `next`, one bitmap slice per peer, `next` re-zeroed
    if (e_.next_bytes_.data()) {
      PackArgs pa;
      pa.bytes = e_.next_bytes_.data();
      pa.next = e_.next_.data();
      pa.words = GW_;
      pa.ctrl = e_.ctrl_.data();
      be_.pack_bytes(pa);
    }
    comm_.alltoall(e_.next_.data(), e_.recv_.data(), static_cast<size_t>(W_) * sizeof(word_t));
    // (`next` re-zeroed by the update, which runs after the exchange: on a
    // no-op chain nothing wrote it)
    tu.zero_next = e_.next_.data();
    tu.zero_slices = P_;
    tu.cand = e_.recv_.data();
    tu.cand_bytes = nullptr;
  }
  // (a split level: visited already holds the earlier parts' claims -- every
  // level byte of this level is a new vertex, as every `next` bit is)
  tu.force = parts > 1;
  tu.frontier = fr_own(c.cur ^ 1);
  tu.new_level = L + 1;
  tu.ctrl = e_.ctrl_.data();
  tu.push = c.push;
  tu.push_rank = me_;
  tu.push_nranks = P_;
  if (opt_.td_fused_finish) {
    // totals (and with one rank the decision) in the update's last
    // workgroup (as bottom-up)
    fuse_update(c, tu);
    // several ranks: the level's end in the same last workgroup (no frontier
    // gathered, or a pushed one)
    if (xc_ && cells_fit() && (!enq_gather_[L] || c.push) &&
        comm_.direct_level_end(2, &tu.end)) {
      tu.fin = finish_args(L, false, enq_dir_[L], c.cap);
      c.level_ended = true;
    }
  }
  be_.update_frontier(tu);
}

// 'B': a bottom-up level -- [hubs: hub_gather stages the frontier hubs' bits
// (several ranks: merges the gathered slices into visited; one rank, a first
// bottom-up level: decides the hub cut and bu_cut_prep expands the non-hub
// frontier top-down)] -> bu_step (fused finish; several ranks: the level end
// in its last workgroup when nothing is gathered).
void DeviceLoop::emit_bottom_up(Chain& c) {
  const int L = c.L;
  BuArgs ba;
  ba.g = gv_;
  ba.visited = e_.visited_.data() + me_ * W_;
  ba.frontier = e_.frontier_[c.cur].data();
  ba.new_frontier = fr_own(c.cur ^ 1);
  ba.level = e_.level_.data();
  ba.level8 = e_.run_narrow_ ? e_.level8_.data() : nullptr;
  ba.narrow_base = e_.narrow_base_;
  ba.new_level = L + 1;
  ba.words = W_;
  ba.lane_limit = opt_.bu_lane_limit;
  ba.whole_units = opt_.bu_whole_units;
  // the third and later bottom-up levels of a run (few unvisited vertices
  // left) scan whole units even on shards too small to fill the chip that
  // way: shadow ranks of P = 4 on RMAT-26, those levels 28-31 -> 22-24 us,
  // where the first two lost 4-10 % (profiles/r6_bu_whole_late_levels.txt)
  if (ba.whole_units == 0 && L >= 2 && enq_form_[static_cast<size_t>(L - 1)] == 'B' &&
      enq_form_[static_cast<size_t>(L - 2)] == 'B')
    ba.whole_units = 1;
  ba.small_waves = opt_.bu_small_waves;
  ba.zdeg = e_.zdeg_.data() + me_ * W_;
  ba.follow_up = c.pf == 'B';
  ba.unit_cnt = e_.unit_cnt_.data();
  ba.unit_deg = e_.unit_deg_.data();
  ba.ctrl = e_.ctrl_.data();
  ba.push = c.push;
  ba.push_rank = me_;
  ba.push_nranks = P_;
  bool cut = false;  // a hub-cut level was enqueued
  if (gv_.nhubs > 0) {
    HubGatherArgs hg;
    hg.g = gv_;
    hg.frontier = e_.frontier_[c.cur].data();
    hg.hub_front = e_.hub_front_.data();
    hg.ctrl = e_.ctrl_.data();
    if (c.pull) {
      // the peers' slices pushed by the previous level's kernels
      hg.pull = c.pull;
      hg.pull_out = e_.frontier_[c.cur].data();
      hg.pull_rank = me_;
      hg.pull_nranks = P_;
      hg.pull_words = W_;
    }
    // several ranks, bu_merge_visited: the gathered remote slices merged into
    // the replicated visited bitmap in the same launch
    if (xc_ && opt_.bu_merge_visited) {
      hg.visited = e_.visited_.data();
      hg.words = GW_;
    }
    // a first bottom-up level: the hub cut (decided on the device from the
    // frontier hubs' degrees hub_gather sums -- global, so the same on every
    // rank), enqueued for levels predicted at <= bu_cut_mf_frac of the
    // graph's edges (a first bottom-up level's non-hub frontier edges grow
    // with its frontier: the larger ones never cut, and skip its launches).
    // Several ranks (up to bu_cut_ranks): the remote claims as one bitmap
    // all-to-all (xcut).
    const bool xcut = P_ > 1;
    // (several ranks: every condition the same on every rank -- the chain
    // then carries the claims' collective)
    const bool shard_ok = P_ == 1 ? gv_.hub_bits && gv_.nz_rec && gv_.unit_base && gv_.nz_pref && gv_.nz_row_off &&
                                        gv_.head && ba.zdeg
                                  : xc_ && P_ <= opt_.bu_cut_ranks && e_.g_.rec_all();
    cut = opt_.bu_cut_edges > 0 && c.pf != 'B' &&
          (c.mf_hint < 0 || c.mf_hint <= opt_.bu_cut_mf_frac * static_cast<double>(e_.total_directed_)) && shard_ok;
    if (cut) {
      if (!e_.cut_part_.data()) {
        e_.cut_part_ = DBuf<int64_t>(be_, static_cast<size_t>(std::max<int64_t>(div_up(gv_.nhubs, int64_t(64)), kHgCopyGrid)));
        e_.cut_flag_ = DBuf<int>(be_, 1);
        e_.cut_ticket_ = DBuf<unsigned>(be_, 1);
        be_.memset_async(e_.cut_ticket_.data(), 0, e_.cut_ticket_.bytes());
      }
      hg.cut_part = e_.cut_part_.data();
      hg.cut_edges = opt_.bu_cut_edges;
      hg.cut_flag = e_.cut_flag_.data();
      hg.cut_ticket = e_.cut_ticket_.data();
    }
    be_.hub_gather(hg);
    ba.hub_front = e_.hub_front_.data();
    if (cut) {
      ba.cut_edges = opt_.bu_cut_edges;
      ba.cut_flag = e_.cut_flag_.data();
      if (!e_.run_narrow_) {
        // wide levels: claims in a byte array of their own (kept zero)
        if (!e_.cut_claim_.data()) {
          e_.cut_claim_ = DBuf<uint8_t>(be_, static_cast<size_t>(W_ * kWordBits));
          be_.memset_async(e_.cut_claim_.data(), 0, e_.cut_claim_.bytes());
        }
        ba.cut_claim = e_.cut_claim_.data();
      }
      res_.chains.back().cut = true;
      if (xcut) {
        // the remote claims: bytes of the global byte map (zero between its
        // users: every pack clears what it read)
        if (!e_.next_bytes_.data()) {
          e_.next_bytes_ = DBuf<uint8_t>(be_, static_cast<size_t>(GW_) * kWordBits);
          be_.memset_async(e_.next_bytes_.data(), 0, e_.next_bytes_.bytes());
        }
        ba.cut_bytes = e_.next_bytes_.data();
        ba.cut_vis = e_.visited_.data();
        ba.cut_word_off = me_ * W_;
      }
      be_.bu_cut_prep(ba);
      if (xcut) {
        // ... packed per owner into `next`, one bitmap all-to-all (a
        // collective: on a plain or no-op chain too, then empty), merged on
        // the owners; `next` re-zeroed by the merge
        PackArgs pa;
        pa.bytes = e_.next_bytes_.data();
        pa.next = e_.next_.data();
        pa.words = GW_;
        pa.ctrl = e_.ctrl_.data();
        pa.flag = e_.cut_flag_.data();
        pa.skip_begin = me_ * W_;
        pa.skip_end = (me_ + 1) * W_;
        be_.pack_bytes(pa);
        comm_.alltoall(e_.next_.data(), e_.recv_.data(), static_cast<size_t>(W_) * sizeof(word_t));
        ba.cut_recv = e_.recv_.data();
        ba.cut_next = e_.next_.data();
        ba.cut_rank = me_;
        ba.cut_nranks = P_;
        be_.bu_cut_merge(ba);
      }
    }
  }
  if (opt_.bu_fused_scan) {
    // the level's totals (and with one rank its finish) in the bottom-up
    // kernel's last workgroup; the unit prefixes only if a top-down chain
    // follows
    if (!e_.bu_tot_.data()) e_.bu_tot_ = DBuf<int64_t>(be_, static_cast<size_t>(2 * kMaxFusedGrid));
    ba.fuse_scan = true;
    ba.scan = scan_args(L, false, enq_dir_[L], c.cap);
    ba.tot = e_.bu_tot_.data();
    c.fused_scan = true;
    // several ranks: the level's end in the kernel's last workgroup too (no
    // frontier gather; the hub kernels' fused finish) -- on a hub-cut level
    // in whichever of its two kernels the decision runs (the plain one on a
    // no-op chain)
    if (xc_ && cells_fit() && gv_.nhubs > 0 && (!enq_gather_[L] || c.push) &&
        comm_.direct_level_end(2, &ba.end)) {
      ba.fin = finish_args(L, false, enq_dir_[L], c.cap);
      c.level_ended = true;
    }
  }
  be_.bu_step(ba);
}

// ---- the host loop ------------------------------------------------------------

RunResult DeviceLoop::run() {
  setup();
  TraceRange trace_run(std::string("bfs.run(device loop) mode=") + mode_name(opt_.mode) + " src=" +
                       std::to_string(src_));
  res_.source = src_;
  be_.reset_events();
  // Several ranks: the runs start together.  One rank: no synchronize -- the
  // previous run's speculative trailing chain may still be executing, and
  // this run's initialisation queues right behind it on the stream instead of
  // after a host wake-up (nothing below touches host-visible state the
  // trailing chain writes: see the mailbox note in setup).
  if (xc_ || opt_.phase_timing) comm_.barrier();
  t0_ = std::chrono::steady_clock::now();
  // (host timing: the host's time from the previous traversal's last stamp
  // to this one's start, i.e. the gap between back-to-back runs)
  static thread_local std::chrono::steady_clock::time_point prev_done{};
  if (ht_ && prev_done.time_since_epoch().count() != 0)
    htl_.emplace_back("since_prev_done", std::chrono::duration<double, std::micro>(t0_ - prev_done).count());

  e_.begin_run_scratch();
  init_.mode = opt_.mode == Mode::TopDown ? 0 : opt_.mode == Mode::BottomUp ? 1 : 2;
  init_.alpha = opt_.alpha;
  init_.beta = opt_.beta;
  init_.n = static_cast<double>(part_.n);
  init_.total_directed = static_cast<double>(e_.total_directed_);
  init_.td_byte_edges = bytes_ok_ ? static_cast<double>(byte_edges_) : 1e300;
  init_.check_visited_min = opt_.td_check_visited_min;
  init_.dir = opt_.mode == Mode::BottomUp ? 'B' : 'T';
  // (directed graphs: a vertex without out-edges can still be reached -- no
  // all-reached stop)
  init_.n_active = opt_.directed ? 0 : e_.n_active_;
  // one fused pass: levels, visited, the seed frontier (frontier_[1]), its
  // totals, the seeded LevelCtrl and the mailbox stamp of level -1 (+ with
  // sparse levels: the seed's work-list entry in set 0 and a clean
  // frontier_[0] for a sparse level 0 to write).  (Several ranks: the seed
  // totals are all-reduced first, then level_finish seeds the LevelCtrl and
  // stamps level -1.)
  // (several ranks: each rank seeds the traversal itself from the replicated
  // degree of the source -- no collective before level 0; a bottom-up level
  // 0 gets the whole seed frontier written locally)
  seed_gather_ = xc_ && init_.dir == 'B';
  InitRunArgs ia = e_.init_args(src_, fr_own(1), e_.ctrl_.data(), init_, e_.mailbox_dev_ + slot(-1));
  ia.stats = sblk(-1);
  if (xc_) {
    ia.deg_all = e_.deg_all_.data();
    ia.src_global = src_;
    if (seed_gather_) ia.frontier_global = e_.frontier_[1].data();
  }
  if (sparse_) {
    ia.qbase = e_.qbase_.data();
    ia.blk_vstart = e_.blk_vstart_.data();
    ia.qv = e_.qv_[0].data();
    ia.frontier_clear = fr_own(0);
  }
  // (the previous traversal left both owned slices zero: 16 B per vertex of
  // stores saved; cleared until this run completes)
  ia.frontier_clean = e_.frontier_clean_ && !seed_gather_;
  e_.frontier_clean_ = false;
  be_.init_run(ia);
  // (Top-down levels read only their owned slice; the replicated visited
  // bitmap filters candidates with whatever remote bits it has -- merged
  // frontiers, and the remote targets this rank claimed and sent -- so a
  // stale remote bit only costs an id its owner drops.)

  // Frontier double buffer: the seed is frontier_[1]; level L reads
  // frontier_[(L + 1) & 1] and writes the other one.
  ua_.g = gv_;
  ua_.nchunks = xc_ ? part_.nranks : 1;
  ua_.cand_stride = W_;
  ua_.clear_cand = !xc_;
  ua_.visited = e_.visited_.data() + me_ * W_;
  ua_.level = e_.level_.data();
  ua_.level8 = e_.run_narrow_ ? e_.level8_.data() : nullptr;
  ua_.narrow_base = e_.narrow_base_;
  ua_.words = W_;
  ua_.unit_cnt = e_.unit_cnt_.data();
  ua_.unit_deg = e_.unit_deg_.data();

  // Host loop, one level ahead of the device.  The stamp of level L - 1
  // carries the real direction of level L and its frontier; a mispredicted
  // level (a no-op chain, its scan skipped too) is enqueued again.
  //   device_loop_predict: after that stamp, level L + 1 is enqueued with the
  //     direction the device will choose if the frontier keeps its growth rate
  //     (n_f and m_f extrapolated geometrically, run through the same
  //     level_ctrl_finish): the Beamer switches of RMAT traversals are
  //     predicted exactly, so no chain is wasted.
  //   otherwise: level L + 1 is enqueued before the stamp, predicted to keep
  //     level L's direction (two wasted chains per direction change).
  // Several ranks: a top-down chain is sparse ('S': owner lists, live while
  // the level's global frontier edges fit them) or dense ('T'); a sparse
  // chain whose level turns out larger is a no-op and is re-enqueued dense,
  // like a mispredicted direction.  Each chain's collective also all-gathers
  // its output frontier when the level after it is predicted bottom-up (two
  // levels ahead of the stamp: the prediction is extrapolated twice).
  int nlev = 0;
  LevelCtrl hc = init_;  // host mirror for the prediction
  int64_t prev_nf = 0, prev_mf = 0;
  bool any_bu = init_.dir == 'B';  // a bottom-up level was decided (the rising phase is over)
  {
    int64_t cap0 = 0;
    const char f0 = init_.dir == 'B' ? 'B' : td_form(0, 0.0, &cap0, false);
    enqueue_level(0, f0, cap0, -1.0, init_.dir == 'B');
  }
  for (int L = 0;; ++L) {
    if (!opt_.device_loop_predict) {
      // dense top-down or bottom-up, one more level ahead
      enqueue_level(L + 1, enq_dir_[L], 0, -1.0, enq_dir_[L] == 'B');
    }
    const volatile LevelMailbox* mb = nullptr;
    try {
      mb = wait_stamp(L - 1);
    } catch (const Error& err) {
      throw Error(std::string(err.what()) + " (" + describe(L - 1) + ")");
    }
    if (ht_) hmark("stamp " + std::to_string(L - 1));
    if (mb->done) {
      nlev = L;
      break;
    }
    const char actual = static_cast<char>(mb->next_dir);
    const int64_t nf = mb->n_f, mf = mb->m_f;
    const bool valid = chain_valid(L, actual, mf);
    if (!valid) ++res_.mispredicts;
    if (!opt_.device_loop_predict) {
      if (!valid) {
        enqueue_level(L, actual, 0, -1.0, actual == 'B');
        enqueue_level(L + 1, actual, 0, -1.0, actual == 'B');
      }
      continue;
    }
    // level L + 1 extrapolated from the frontiers of L - 1 and L, then L + 2
    hc.dir = actual;
    hc.n_f = nf;
    hc.m_f = mf;
    hc.vis_deg = mb->vis_deg;
    hc.done = 0;
    double enf = 0, emf = 0, enf2 = 0, emf2 = 0;
    if (actual == 'B') any_bu = true;
    predict(hc, static_cast<double>(nf), static_cast<double>(mf), static_cast<double>(prev_nf),
            static_cast<double>(prev_mf), static_cast<double>(mb->reached), L == 0, !any_bu, &enf, &emf);
    const char d1 = static_cast<char>(hc.dir);
    LevelCtrl hc2 = hc;
    predict(hc2, enf, emf, static_cast<double>(nf), static_cast<double>(mf), static_cast<double>(mb->reached) + enf,
            false, !any_bu && d1 != 'B', &enf2, &emf2);
    const char d2 = static_cast<char>(hc2.dir);
    if (!valid) {
      int64_t cap = 0;
      const char f = actual == 'B' ? 'B' : td_form(L, static_cast<double>(mf), &cap, true);
      vis_hint_ = static_cast<double>(mb->vis_deg);  // (exact: level L's start)
      reach_hint_ = static_cast<double>(mb->reached);
      enqueue_level(L, f, cap, static_cast<double>(mf), d1 == 'B');
    }
    prev_nf = nf;
    prev_mf = mf;
    int64_t lcap = 0;
    const char f = d1 == 'B' ? 'B' : td_form(L + 1, emf, &lcap, false);
    vis_hint_ = static_cast<double>(mb->vis_deg) + emf;  // (level L + 1's frontier joins visited)
    reach_hint_ = static_cast<double>(mb->reached) + enf;
    enqueue_level(L + 1, f, lcap, emf, d2 == 'B');
  }
  // The traversal is complete once the last stamp is seen: the stamping
  // workgroup ran after all of that level's work (and every earlier level's).
  // The chain enqueued ahead of it is a no-op that drains on its own, ordered
  // before any later work on the stream -- no synchronisation needed.
  const auto t1 = std::chrono::steady_clock::now();
  prev_done = t1;
  comm_.set_level_tag(-1);
  return collect(nlev, t1);
}

// Totals and per-level records (outside the timed window), from the mapped
// record segments.
RunResult DeviceLoop::collect(int nlev, std::chrono::steady_clock::time_point t1) {
  if (opt_.phase_timing) be_.synchronize();
  e_.scratch_dirty_ = false;
  res_.ms = std::chrono::duration<double, std::milli>(t1 - t0_).count();
  if (xc_) res_.ms = comm_.max_host(res_.ms);
  if (ht_) {
    hmark("done");
    std::string line = "[host timing]";
    for (auto& [w, us] : htl_) line += " " + w + "@" + std::to_string(static_cast<int>(us));
    std::fprintf(stderr, "%s\n", line.c_str());
  }
  const int64_t vis_deg = e_.mailbox_host_[slot(nlev - 1)].vis_deg;
  std::vector<LevelRecDev> recs(static_cast<size_t>(nlev));
  for (int L = 0; L < nlev; ++L) {
    const volatile LevelRecDev* r = e_.rec_segs_[static_cast<size_t>(L / Engine::kRecSeg)].first + L % Engine::kRecSeg;
    recs[L].dir = r->dir;
    recs[L].n_f = r->n_f;
    recs[L].m_f = r->m_f;
    recs[L].discovered = r->discovered;
    recs[L].t0 = r->t0;
    recs[L].t1 = r->t1;
  }
  res_.reached = 1;
  const double khz = be_.wall_clock_khz();
  for (int L = 0; L < nlev; ++L) {
    LevelRecord r;
    r.level = L;
    r.direction = static_cast<char>(recs[L].dir);
    r.frontier = recs[L].n_f;
    r.frontier_edges = recs[L].m_f;
    r.discovered = recs[L].discovered;
    if (opt_.phase_timing && static_cast<size_t>(L) < evs_.size()) r.ms = be_.elapsed_ms(evs_[L].first, evs_[L].second);
    // device-clock times (kernels stamp them; no events, no overhead)
    if (khz > 0 && recs[L].t0 != 0 && recs[L].t1 >= recs[L].t0) {
      if (!opt_.phase_timing) r.ms = static_cast<double>(recs[L].t1 - recs[L].t0) / khz;
      if (L > 0 && recs[L - 1].t1 != 0)
        r.gap_ms = (static_cast<double>(recs[L].t0) - static_cast<double>(recs[L - 1].t1)) / khz;
    }
    res_.reached += r.discovered;
    res_.levels.push_back(r);
  }
  // the owned frontier slices are zero again when the last level was top-down
  // and found nothing (top-down levels clear their input as they read it and
  // set only new bits; a bottom-up level leaves its input, an all-reached
  // stop its last frontier)
  // (with sparse levels on: only then does the compaction clear as it reads)
  e_.frontier_clean_ = sparse_ && nlev > 0 && recs[nlev - 1].dir == 'T' && recs[nlev - 1].discovered == 0;
  res_.depth = nlev == 0 ? 1 : nlev;
  // (a traversal that stopped once every vertex with an edge was reached did
  // not expand its last frontier: its deepest level is the last record's + 1)
  if (nlev > 0 && recs[nlev - 1].discovered > 0) res_.depth = nlev + 1;
  res_.edges = vis_deg / 2;
  return std::move(res_);
}

RunResult Engine::run_bitmap_device(int64_t source) {
  DeviceLoop loop(*this, source);
  return loop.run();
}

}  // namespace dbfs
