// CPU implementation of the Backend primitives.
//
// Semantically identical to the HIP kernels (same work-list layout, same
// segment bookkeeping) so the engine's orchestration, partitioning and
// collectives are exercised by the CPU test-suite exactly as they run on the
// GPU.  Not a performance path.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#include "dbfs/backend.hpp"

namespace dbfs {
namespace {

// Level of a new vertex in the wide or the narrow array (HIP: store_level).
inline void put_level(lvl_t* wide, uint8_t* narrow, int64_t i, lvl_t level, uint8_t base) {
  if (narrow) narrow[i] = static_cast<uint8_t>(base + (level <= kNarrowMaxLevel ? level : kNarrowMaxLevel + 1));
  else wide[i] = level;
}

inline bool test_bit(const word_t* bm, uint64_t v) { return (bm[v >> 6] >> (v & 63)) & 1ull; }
inline word_t gather_bytes(uint8_t* p) {
  word_t bits = 0;
  for (int b = 0; b < 64; ++b)
    if (p[b]) bits |= 1ull << b;
  if (bits) std::memset(p, 0, 64);
  return bits;
}

class CpuBackend final : public Backend {
 public:
  DeviceKind kind() const override { return DeviceKind::CPU; }
  std::string name() const override { return "cpu"; }

  void* alloc(size_t bytes) override {
    void* p = std::aligned_alloc(64, round_up(std::max<size_t>(bytes, 64), 64));
    if (!p) raise_error(__FILE__, __LINE__, "host allocation failed");
    // DBFS_POISON_ALLOC=<byte>: as the HIP backend's (memory never written
    // reads as that byte instead of whatever the allocator hands back)
    static const int poison = [] {
      const char* e = std::getenv("DBFS_POISON_ALLOC");
      return e && *e ? static_cast<int>(std::strtol(e, nullptr, 0)) & 0xff : -1;
    }();
    if (poison >= 0) std::memset(p, poison, round_up(std::max<size_t>(bytes, 64), 64));
    return p;
  }
  void dealloc(void* p) override { std::free(p); }
  void memset_async(void* p, int v, size_t bytes) override { std::memset(p, v, bytes); }
  void copy_async(void* d, const void* s, size_t bytes) override {
    if (bytes) std::memmove(d, s, bytes);
  }
  void to_host(void* d, const void* s, size_t bytes) override { copy_async(d, s, bytes); }
  void to_device(void* d, const void* s, size_t bytes) override { copy_async(d, s, bytes); }
  void synchronize() override {}

  int record_event() override {
    events_.push_back(std::chrono::steady_clock::now());
    return static_cast<int>(events_.size() - 1);
  }
  double elapsed_ms(int a, int b) override {
    return std::chrono::duration<double, std::milli>(events_.at(b) - events_.at(a)).count();
  }
  void reset_events() override { events_.clear(); }

  void fill_level(lvl_t* level, int64_t n, lvl_t value) override { std::fill(level, level + n, value); }
  void set_bit(word_t* bm, int64_t bit) override { bm[bit >> 6] |= 1ull << (bit & 63); }

  void update_frontier(const UpdateArgs& a) override {
    if (a.fuse_scan) {
      // totals and finish right after the update, unit statistics unscanned
      UpdateArgs b = a;
      b.fuse_scan = false;
      update_frontier(b);
      const int64_t n = a.scan.nunits;
      std::vector<int64_t> c(a.scan.unit_cnt, a.scan.unit_cnt + n), d(a.scan.unit_deg, a.scan.unit_deg + n);
      scan_units(a.scan);
      if (a.fold_scan) return;  // (the prefixes stay: the next compaction reads them)
      std::copy(c.begin(), c.end(), a.scan.unit_cnt);
      std::copy(d.begin(), d.end(), a.scan.unit_deg);
      return;
    }
    bool use_bytes = a.cand_bytes != nullptr;
    if (a.ctrl) {
      if (!chain_live(*a.ctrl, 'T', a.max_mf)) return;
      use_bytes = use_bytes && a.ctrl->bytes != 0;
    }
    const int64_t nunits = div_up(a.words, kUnitWords);
    for (int64_t u = 0; u < nunits; ++u) {
      int64_t cnt = 0, deg = 0;
      for (int64_t w = u * kUnitWords; w < std::min<int64_t>(a.words, (u + 1) * kUnitWords); ++w) {
        word_t c = 0;
        if (use_bytes && a.level_direct) {
          for (int b = 0; b < 64; ++b)
            if (a.level_direct[w * 64 + b] == static_cast<uint8_t>(a.narrow_base + a.new_level)) c |= 1ull << b;
        } else if (use_bytes) {
          c = gather_bytes(a.cand_bytes + w * 64);
        } else {
          for (int r = 0; r < a.nchunks; ++r) c |= a.cand[r * a.cand_stride + w];
          if (a.clear_cand) a.cand[w] = 0;
        }
        const word_t nb = a.force ? c : (c & ~a.visited[w]);
        a.visited[w] |= nb;
        a.frontier[w] = nb;
        for (int p = 0; p < a.zero_slices; ++p) a.zero_next[p * a.words + w] = 0;
        word_t x = nb;
        while (x) {
          const int b = __builtin_ctzll(x);
          x &= x - 1;
          const int64_t v = w * 64 + b;
          put_level(a.level, a.level8, v, a.new_level, a.narrow_base);
          const eid_t d = a.g.row_off[v + 1] - a.g.row_off[v];
          if (d > 0) { ++cnt; deg += d; }
        }
      }
      a.unit_cnt[u] = cnt;
      a.unit_deg[u] = deg;
    }
  }

  void level_ctrl_init(LevelCtrl* c, const LevelCtrl& init) override { *c = init; }
  void init_run(const InitRunArgs& a) override {
    const int64_t src = a.src_local;
    if (a.level8 && a.level8_filled) {
      if (src >= 0) a.level8[src] = a.narrow_base;
    } else {
      for (int64_t i = 0; i < a.g.rows; ++i) {
        if (a.level8) a.level8[i] = i == src ? a.narrow_base : kNarrowUnreached;
        else a.level[i] = i == src ? 0 : kUnreached;
      }
    }
    for (int64_t w = 0; w < a.gwords; ++w) a.visited[w] = a.zdeg[w];
    if (a.frontier_clean && !a.frontier_global) {
      // (the claim the device kernel relies on, checked: no stale bit left)
      for (int64_t w = 0; w < a.words; ++w)
        DBFS_CHECK(a.frontier[w] == 0 && (!a.frontier_clear || a.frontier_clear[w] == 0),
                   "init_run: a frontier claimed clean holds a stale bit");
    }
    for (int64_t w = 0; w < a.words; ++w) a.frontier[w] = 0;
    if (a.frontier_global)
      for (int64_t w = 0; w < a.gwords; ++w) a.frontier_global[w] = 0;
    if (a.src_global >= 0) {
      // (a seed without collective: the source's bits on every rank)
      const word_t gbit = 1ull << (a.src_global & 63);
      a.visited[a.src_global >> 6] |= gbit;
      if (a.frontier_global) a.frontier_global[a.src_global >> 6] = gbit;
    }
    int64_t cnt = 0, deg = 0;
    if (src >= 0) {
      const word_t bit = 1ull << (src & 63);
      a.visited[a.vis_word_base + (src >> 6)] |= bit;
      a.frontier[src >> 6] = bit;
      const eid_t d = a.g.row_off[src + 1] - a.g.row_off[src];
      if (d > 0) { cnt = 1; deg = d; }
      const int64_t unit = (src >> 6) / kUnitWords;
      a.unit_cnt[unit] = a.unit_deg[unit] = 0;
      a.part_cnt[unit / kScanChunk] = a.part_deg[unit / kScanChunk] = 0;
    }
    a.stats[0] = a.stats[2] = cnt;
    a.stats[1] = a.stats[3] = deg;
    a.qscan[cnt] = deg;
    if (a.frontier_clear)
      for (int64_t w = 0; w < a.words; ++w) a.frontier_clear[w] = 0;
    if (cnt && a.qbase) {
      a.qscan[0] = 0;
      a.qbase[0] = a.g.row_off[src];
      a.qv[0] = static_cast<vid_t>(src);
      for (int64_t b = 0; b * kTdEdgesPerBlock < deg; ++b) a.blk_vstart[b] = 0;
    }
    if (a.ctrl) {
      int64_t gc = cnt, gd = deg;
      if (a.deg_all) {
        gd = a.deg_all[a.src_global];
        gc = gd > 0 ? 1 : 0;
        a.stats[2] = gc;
        a.stats[3] = gd;
      }
      LevelCtrl c = a.ctrl_init;
      level_ctrl_finish(c, gc, gd, true, nullptr);
      *a.ctrl = c;
      if (a.mailbox) {
        a.mailbox->done = c.done;
        a.mailbox->vis_deg = c.vis_deg;
        a.mailbox->next_dir = c.dir;
        a.mailbox->n_f = c.n_f;
        a.mailbox->m_f = c.m_f;
        a.mailbox->reached = c.reached;
        a.mailbox->level = -1;
      }
    }
  }
  void publish_stats(const int64_t* stats, StatsMailbox* mb, int64_t seq) override {
    for (int k = 0; k < 4; ++k) mb->v[k] = stats[k];
    __atomic_store_n(&mb->seq, seq, __ATOMIC_RELEASE);
  }
  void* alloc_mapped(size_t bytes, void** dptr) override {
    void* h = std::calloc(1, std::max<size_t>(bytes, 1));
    DBFS_CHECK(h != nullptr, "host allocation failed");
    *dptr = h;
    return h;
  }
  void free_mapped(void* h) override { std::free(h); }

  void scan_units(const ScanArgs& a) override {
    if (a.ctrl && !chain_live(*a.ctrl, a.expect_dir, a.expect_cap)) return;
    const int64_t nchunks = div_up(a.nunits, kScanChunk);
    int64_t c = 0, d = 0;
    for (int64_t k = 0; k < nchunks; ++k) {
      int64_t ic = 0, id = 0;
      for (int64_t u = k * kScanChunk; u < std::min<int64_t>(a.nunits, (k + 1) * kScanChunk); ++u) {
        const int64_t tc = a.unit_cnt[u], td = a.unit_deg[u];
        a.unit_cnt[u] = ic;
        a.unit_deg[u] = id;
        ic += tc;
        id += td;
      }
      a.part_cnt[k] = c;
      a.part_deg[k] = d;
      c += ic;
      d += id;
    }
    a.stats[0] = a.stats[2] = c;
    a.stats[1] = a.stats[3] = d;
    a.qscan[c] = d;
    if (a.ctrl && a.finish) {
      level_ctrl_finish(*a.ctrl, c, d, a.seed, a.seed ? nullptr : a.rec);
      if (a.mailbox) {
        a.mailbox->done = a.ctrl->done;
        a.mailbox->vis_deg = a.ctrl->vis_deg;
        a.mailbox->next_dir = a.ctrl->dir;
        a.mailbox->n_f = a.ctrl->n_f;
        a.mailbox->m_f = a.ctrl->m_f;
        a.mailbox->reached = a.ctrl->reached;
        a.mailbox->level = a.level;
      }
    }
  }

  void zero_degree_mask(const ZeroDegArgs& a) override {
    for (int64_t w = 0; w < a.words; ++w) {
      word_t m = 0;
      for (int b = 0; b < 64; ++b) {
        const int64_t v = w * 64 + b;
        if (v >= a.g.rows || (!a.padding_only && a.g.row_off[v + 1] == a.g.row_off[v])) m |= 1ull << b;
      }
      a.out[w] = m;
    }
  }

  void compact_frontier(const CompactArgs& a) override {
    if (a.ctrl && !chain_live(*a.ctrl, 'T', a.max_mf)) return;
    const int64_t nunits = div_up(a.words, kUnitWords);
    for (int64_t u = 0; u < nunits; ++u) {
      int64_t pos = a.unit_cnt_off[u] + a.part_cnt[u / kScanChunk];
      int64_t off = a.unit_deg_off[u] + a.part_deg[u / kScanChunk];
      for (int64_t w = u * kUnitWords; w < std::min<int64_t>(a.words, (u + 1) * kUnitWords); ++w) {
        word_t x = a.frontier[w];
        if (a.clear) a.clear[w] = 0;
        if (a.clear_all) a.clear_all[w] = 0;
        while (x) {
          const int b = __builtin_ctzll(x);
          x &= x - 1;
          const int64_t v = w * 64 + b;
          const eid_t rs = a.g.row_off[v], d = a.g.row_off[v + 1] - rs;
          if (d <= 0) continue;
          a.qscan[pos] = off;
          a.qbase[pos] = rs - off;
          if (a.qv) a.qv[pos] = static_cast<vid_t>(v);
          for (int64_t blk = div_up(off, kTdEdgesPerBlock); blk * kTdEdgesPerBlock < off + d; ++blk)
            a.blk_vstart[blk] = static_cast<int32_t>(pos);
          ++pos;
          off += d;
        }
      }
    }
  }

  void td_expand(const TdArgs& a) override {
    int64_t q = a.q;
    bool bytes = a.next_bytes != nullptr;
    if (a.ctrl) {
      if (!chain_live(*a.ctrl, 'T', a.max_mf)) return;
      q = a.dev_stats[0];
      bytes = a.ctrl->bytes != 0;
      if (a.clear_qv)
        for (int64_t i = 0; i < q; ++i)
          a.clear_frontier[a.clear_qv[i] >> 6] = 0;
    }
    // a split level's part (TdArgs::split_k): its run of the level's edges
    const int64_t m = a.ctrl ? a.dev_stats[1] : a.m;
    const int64_t e_lo = a.split_k > 1 ? m * a.split_i / a.split_k : 0;
    const int64_t e_hi = a.split_k > 1 ? m * (a.split_i + 1) / a.split_k : m;
    for (int64_t i = 0; i < q; ++i) {
      const int64_t b = std::max(a.qscan[i], e_lo), e = std::min(a.qscan[i + 1], e_hi);
      for (int64_t k = b; k < e; ++k) {
        const vid_t v = a.g.col[k + a.qbase[i]];
        // (the filter's clear bits are visited vertices: skipping on them
        // changes nothing -- and catches a filter that drops an unvisited one)
        if (a.unvis && !test_bit(a.unvis, unvis_index(v, a.unvis_mult))) continue;
        if (test_bit(a.visited, v)) continue;
        if (a.lists) {
          vid_t* list = a.lists + static_cast<int64_t>(v / a.part) * (a.list_cap + 1);
          list[1 + list[0]++] = v;
        } else if (bytes && a.level_direct) {
          a.level_direct[v] = static_cast<uint8_t>(a.narrow_base + a.new_level);
        } else if (bytes) {
          a.next_bytes[v] = 1;
        } else {
          a.next[v >> 6] |= 1ull << (v & 63);
        }
      }
    }
  }

  void td_binned(const BinArgs& a) override {
    if (!chain_live(*a.ctrl, 'T', 0)) return;
    const int64_t q = a.dev_stats[0];
    if (a.clear_qv)
      for (int64_t i = 0; i < q; ++i) a.clear_frontier[a.clear_qv[i] >> 6] = 0;
    std::vector<word_t> nb(static_cast<size_t>(a.words), 0);
    for (int64_t i = 0; i < q; ++i)
      for (int64_t k = a.qscan[i]; k < a.qscan[i + 1]; ++k) {
        const vid_t v = a.g.col[k + a.qbase[i]];
        if (!test_bit(a.visited, v)) nb[v >> 6] |= 1ull << (v & 63);
      }
    for (int64_t w = 0; w < a.words; ++w) {
      a.frontier[w] = nb[w];
      a.visited[w] |= nb[w];
    }
  }

  void level_finish(const LevelFinishArgs& a) override {
    if (!a.seed && !chain_live(*a.ctrl, a.expect_dir, a.expect_cap)) return;
    LevelCtrl c = a.seed ? a.ctrl_init : *a.ctrl;
    level_ctrl_finish(c, a.stats[2], a.stats[3], a.seed, a.seed ? nullptr : a.rec);
    *a.ctrl = c;
    if (a.mailbox) {
      a.mailbox->done = c.done;
      a.mailbox->vis_deg = c.vis_deg;
      a.mailbox->next_dir = c.dir;
      a.mailbox->n_f = c.n_f;
      a.mailbox->m_f = c.m_f;
      a.mailbox->reached = c.reached;
      a.mailbox->level = a.seed ? -1 : a.level;
    }
  }

  // Sparse top-down level (see the HIP kernel): claims in the replicated
  // visited bitmap; owned claims settled into the next work list (the running
  // totals in sparse_cnt_ / sparse_deg_), remote ones (several ranks) appended
  // to their owners' lists; without lists the level is finished here.
  void sparse_settle(const TdSparseArgs& a, vid_t v) {
    const int64_t r = static_cast<int64_t>(v) - a.g.lo;
    DBFS_CHECK(r >= 0 && r < a.g.rows, "sparse level: settled vertex outside this shard");
    put_level(a.level, a.level8, r, a.new_level, a.narrow_base);
    const eid_t rs = a.g.row_off[r], d = a.g.row_off[r + 1] - rs;
    if (d <= 0) return;
    a.frontier_out[r >> 6] |= 1ull << (r & 63);
    const int64_t cnt = sparse_cnt_, deg = sparse_deg_;
    a.oscan[cnt] = deg;
    a.obase[cnt] = rs - deg;
    a.oqv[cnt] = static_cast<vid_t>(r);
    for (int64_t blk = div_up(deg, kTdEdgesPerBlock); blk * kTdEdgesPerBlock < deg + d; ++blk)
      a.oblk[blk] = static_cast<int32_t>(cnt);
    ++sparse_cnt_;
    sparse_deg_ += d;
  }
  void sparse_finish_totals(const TdSparseArgs& a) {
    a.stats[0] = a.stats[2] = sparse_cnt_;
    a.stats[1] = a.stats[3] = sparse_deg_;
    a.oscan[sparse_cnt_] = sparse_deg_;
  }
  void td_sparse(const TdSparseArgs& a) override {
    DBFS_CHECK(!a.direct.active, "CpuBackend: no direct list exchange (peer windows are GPU memory)");
    if (!chain_live(*a.ctrl, 'T', a.max_mf)) return;
    // the input frontier's rows [col_begin, col_end), in work-list order (a
    // bitmap input: its set bits in (word, bit) order, as a compaction lists them)
    std::vector<std::pair<eid_t, eid_t>> rows;
    if (a.from_bits) {
      for (int64_t w = 0; w < a.words; ++w) {
        for (word_t m = a.frontier_in[w]; m; m &= m - 1) {
          const int64_t r = w * kWordBits + __builtin_ctzll(m);
          rows.emplace_back(a.g.row_off[r], a.g.row_off[r + 1]);
        }
        a.frontier_in[w] = 0;
      }
    } else {
      const int64_t q = a.dev_stats[0];
      for (int64_t i = 0; i < q; ++i) a.frontier_in[a.qv[i] >> 6] = 0;
      for (int64_t i = 0; i < q; ++i) rows.emplace_back(a.qscan[i] + a.qbase[i], a.qscan[i + 1] + a.qbase[i]);
    }
    sparse_cnt_ = sparse_deg_ = 0;
    for (const auto& [cb, ce] : rows) {
      for (eid_t k = cb; k < ce; ++k) {
        const vid_t v = a.g.col[k];
        if (test_bit(a.visited, v)) continue;
        a.visited[v >> 6] |= 1ull << (v & 63);
        const int64_t r = static_cast<int64_t>(v) - a.g.lo;
        if (a.lists && (r < 0 || r >= a.g.rows)) {
          vid_t* list = a.lists + (static_cast<int64_t>(v) / a.part) * a.list_stride;
          DBFS_CHECK(static_cast<int64_t>(list[0]) + 1 < a.list_stride, "owner list overflow");
          list[1 + list[0]++] = v;
          continue;
        }
        sparse_settle(a, v);
      }
    }
    if (a.lists) return;  // several ranks: td_sparse_apply finishes
    sparse_finish_totals(a);
    level_ctrl_finish(*a.ctrl, sparse_cnt_, sparse_deg_, false, a.rec);
    if (a.mailbox) {
      a.mailbox->done = a.ctrl->done;
      a.mailbox->vis_deg = a.ctrl->vis_deg;
      a.mailbox->next_dir = a.ctrl->dir;
      a.mailbox->n_f = a.ctrl->n_f;
      a.mailbox->m_f = a.ctrl->m_f;
      a.mailbox->reached = a.ctrl->reached;
      a.mailbox->level = a.level_index;
    }
  }
  void td_sparse_apply(const TdSparseArgs& a) override {
    DBFS_CHECK(!a.direct.active, "CpuBackend: no direct list exchange (peer windows are GPU memory)");
    if (!chain_live(*a.ctrl, 'T', a.max_mf)) return;
    for (int r = 0; r < a.nranks; ++r) {
      const vid_t* list = a.recv_lists + static_cast<int64_t>(r) * a.list_stride;
      for (vid_t k = 0; k < list[0]; ++k) {
        const vid_t v = list[1 + k];
        if (test_bit(a.visited, v)) continue;
        a.visited[v >> 6] |= 1ull << (v & 63);
        sparse_settle(a, v);
      }
    }
    for (int r = 0; r < a.nranks; ++r) a.lists[static_cast<int64_t>(r) * a.list_stride] = 0;
    sparse_finish_totals(a);
  }
  int64_t sparse_cnt_ = 0, sparse_deg_ = 0;  // the current sparse level's settled entries / their edges

  // (no device checks in the CPU kernels; the injected violation exercises
  // the engine's failure path on the CPU)
  uint64_t take_device_check() override { return std::exchange(check_, 0); }
  void inject_device_check() override { check_ = 99ull << 48; }
  uint64_t check_ = 0;

  void list_scatter(const ListScatterArgs& a) override {
    if (a.ctrl && !chain_live(*a.ctrl, 'T', a.max_mf)) return;
    if (a.reset_lists)
      for (int r = 0; r < a.nranks; ++r) a.reset_lists[static_cast<int64_t>(r) * (a.list_cap + 1)] = 0;
    for (int r = 0; r < a.nranks; ++r) {
      const vid_t* list = a.lists + static_cast<int64_t>(r) * (a.list_cap + 1);
      for (vid_t k = 0; k < list[0]; ++k) {
        const int64_t v = static_cast<int64_t>(list[1 + k]) - a.lo;
        a.cand[v >> 6] |= 1ull << (v & 63);
      }
    }
  }

  void pack_bytes(const PackArgs& a) override {
    if (a.ctrl && (a.ctrl->done || (a.flag ? a.ctrl->dir != 'B' || !*a.flag : a.ctrl->dir != 'T' || !a.ctrl->bytes)))
      return;
    for (int64_t w = 0; w < a.words; ++w)
      if (w < a.skip_begin || w >= a.skip_end) a.next[w] |= gather_bytes(a.bytes + w * 64);
  }

  void bu_step(const BuArgs& a) override {
    if (a.fuse_scan) {
      // totals and finish right after the step; the unit statistics stay
      // unscanned (as the HIP kernel's fused finish leaves them)
      BuArgs b = a;
      b.fuse_scan = false;
      bu_step(b);
      const int64_t n = a.scan.nunits;
      std::vector<int64_t> c(a.scan.unit_cnt, a.scan.unit_cnt + n), d(a.scan.unit_deg, a.scan.unit_deg + n);
      scan_units(a.scan);
      std::copy(c.begin(), c.end(), a.scan.unit_cnt);
      std::copy(d.begin(), d.end(), a.scan.unit_deg);
      return;
    }
    if (a.ctrl && (a.ctrl->done || a.ctrl->dir != 'B')) return;
    // hub-cut level (as the HIP kernel): claimed vertices join the output
    // unscanned, the others find parents among the frontier hubs only
    const bool cut = a.cut_edges > 0 && *a.cut_flag;
    const int64_t nunits = div_up(a.words, kUnitWords);
    for (int64_t u = 0; u < nunits; ++u) {
      int64_t cnt = 0, deg = 0;
      for (int64_t w = u * kUnitWords; w < std::min<int64_t>(a.words, (u + 1) * kUnitWords); ++w) {
        // claimed: unvisited with this level's level byte already
        word_t pw = 0;
        if (cut)
          for (int b = 0; b < 64 && w * 64 + b < a.g.rows; ++b) {
            const int64_t v = w * 64 + b;
            const bool claimed =
                a.cut_claim ? a.cut_claim[v] != 0
                            : a.level8[v] == static_cast<uint8_t>(a.narrow_base +
                                                                  std::min<lvl_t>(a.new_level, kNarrowMaxLevel + 1));
            if (!((a.visited[w] >> b) & 1ull) && claimed) {
              pw |= 1ull << b;
              if (a.cut_claim) {
                a.cut_claim[v] = 0;
                a.level[v] = a.new_level;
              }
            }
          }
        word_t out = pw;
        const word_t vis = a.visited[w] | pw;
        for (word_t m = pw; m; m &= m - 1) {
          const int64_t v = w * 64 + __builtin_ctzll(m);
          ++cnt;
          deg += a.g.row_off[v + 1] - a.g.row_off[v];
        }
        for (int b = 0; b < 64; ++b) {
          const int64_t v = w * 64 + b;
          if (v >= a.g.rows || ((vis >> b) & 1ull)) continue;
          for (eid_t e = a.g.row_off[v]; e < a.g.row_off[v + 1]; ++e) {
            if (test_bit(a.frontier, a.g.col[e]) && (!cut || test_bit(a.g.hub_bits, a.g.col[e]))) {
              out |= 1ull << b;
              put_level(a.level, a.level8, v, a.new_level, a.narrow_base);
              ++cnt;
              deg += a.g.row_off[v + 1] - a.g.row_off[v];
              break;
            }
          }
        }
        a.visited[w] = vis | out;
        a.new_frontier[w] = out;
      }
      a.unit_cnt[u] = cnt;
      a.unit_deg[u] = deg;
    }
  }

  void status_expand(const StatusArgs& a) override {
    for (int64_t v = 0; v < a.g.rows; ++v) {
      if (a.level[v] != a.cur) continue;
      for (eid_t e = a.g.row_off[v]; e < a.g.row_off[v + 1]; ++e) {
        const vid_t u = a.g.col[e];
        if (!test_bit(a.visited, u)) a.next[u >> 6] |= 1ull << (u & 63);
      }
    }
  }

  void bitmap_or(word_t* dst, const word_t* src, int64_t words) override {
    for (int64_t w = 0; w < words; ++w) dst[w] |= src[w];
  }

  void ref_expand(const RefExpandArgs& a) override {
    for (int64_t i = 0; i < a.q; ++i) {
      const int64_t u = static_cast<int64_t>(a.queue[i]) - a.g.lo;
      for (eid_t e = a.g.row_off[u]; e < a.g.row_off[u + 1]; ++e) {
        const vid_t v = a.g.col[e];
        if (a.dist[v] == kUnreached) {
          a.dist[v] = a.next_level;
          const int64_t owner = v / a.part;
          const int64_t pos = a.bucket_cnt[owner]++;
          a.buckets[owner * a.bucket_cap + pos] = v;
        }
      }
    }
  }

  void ref_accept(const RefAcceptArgs& a) override {
    for (int64_t i = 0; i < a.total; ++i) {
      const vid_t v = a.recv[i];
      bool keep;
      if (i >= a.self_begin && i < a.self_end) {
        keep = true;
      } else {
        keep = a.dist[v] == kUnreached;
        if (keep) a.dist[v] = a.next_level;
      }
      if (keep) a.queue[(*a.qcount)++] = v;
    }
  }

  // Scan mode: the same four passes as the HIP kernels (sequential, so the
  // claim is simply the first edge in queue order).
  void scan_relax(const ScanBfsArgs& a) override {
    for (int64_t i = 0; i < a.q; ++i) {
      const int64_t u = static_cast<int64_t>(a.queue[i]) - a.g.lo;
      for (eid_t e = a.g.row_off[u]; e < a.g.row_off[u + 1]; ++e) {
        const vid_t v = a.g.col[e];
        if (a.dist[v] == kUnreached) {
          a.dist[v] = a.next_level;
          a.claim[v] = e;
        }
      }
    }
  }
  void scan_count(const ScanBfsArgs& a) override {
    for (int64_t i = 0; i < a.q * a.nranks; ++i) a.offs[i] = 0;
    for (int64_t i = 0; i < a.q; ++i) {
      const int64_t u = static_cast<int64_t>(a.queue[i]) - a.g.lo;
      for (eid_t e = a.g.row_off[u]; e < a.g.row_off[u + 1]; ++e) {
        const vid_t v = a.g.col[e];
        if (a.dist[v] == a.next_level && a.claim[v] == e) ++a.offs[(v / a.part) * a.q + i];
      }
    }
  }
  void scan_bounds(const ScanBfsArgs& a) override {
    for (int o = 0; o <= a.nranks; ++o) a.bounds[o] = a.offs[o * a.q];
    for (int o = 0; o < a.nranks; ++o) a.counts[o] = a.bounds[o + 1] - a.bounds[o];
  }
  void scan_assign(const ScanBfsArgs& a) override {
    for (int64_t i = 0; i < a.q; ++i) {
      const int64_t u = static_cast<int64_t>(a.queue[i]) - a.g.lo;
      for (eid_t e = a.g.row_off[u]; e < a.g.row_off[u + 1]; ++e) {
        const vid_t v = a.g.col[e];
        if (a.dist[v] == a.next_level && a.claim[v] == e) a.out[a.offs[(v / a.part) * a.q + i]++] = v;
      }
    }
  }

  void validate_levels(const ValidateArgs& a) override {
    int64_t gap = 0, cross = 0, orphan = 0;
    for (int64_t r = 0; r < a.g.rows; ++r) {
      const int64_t u = a.g.lo + r;
      const lvl_t lu = a.level_global[u];
      bool has_parent = false;
      for (eid_t e = a.g.row_off[r]; e < a.g.row_off[r + 1]; ++e) {
        const lvl_t lv = a.level_global[a.g.col[e]];
        if (lu == kUnreached && lv == kUnreached) continue;
        if ((lu == kUnreached) != (lv == kUnreached)) { ++cross; continue; }
        if (lu - lv > 1 || lv - lu > 1) ++gap;
        if (lv == lu - 1) has_parent = true;
      }
      if (lu != kUnreached && u != a.src && !has_parent) ++orphan;
      if (u == a.src && lu != 0) ++orphan;
    }
    a.out[0] += gap;
    a.out[1] += cross;
    a.out[2] += orphan;
  }

  void compute_parents(const ParentArgs& a) override {
    for (int64_t r = 0; r < a.g.rows; ++r) {
      const int64_t v = a.g.lo + r;
      const lvl_t lv = a.level_global[v];
      int64_t par = -1;
      if (v == a.src) {
        par = v;
      } else if (lv != kUnreached) {
        for (eid_t e = a.g.row_off[r]; e < a.g.row_off[r + 1]; ++e) {
          if (a.level_global[a.g.col[e]] == lv - 1) { par = a.g.col[e]; break; }
        }
      }
      a.parent[r] = par;
    }
  }

  void degrees_u32(const eid_t* ro, int64_t rows, uint32_t* out) override {
    for (int64_t r = 0; r < rows; ++r) {
      const eid_t d = ro[r + 1] - ro[r];
      out[r] = d > 0xFFFFFFFFll ? 0xFFFFFFFFu : static_cast<uint32_t>(d);
    }
  }

  void sort_neighbors(const eid_t* ro, vid_t* col, int64_t rows, const uint32_t* key_deg) override {
    // Same policy as the device: rows of 2..4096 entries, (degree desc, id asc).
    for (int64_t r = 0; r < rows; ++r) {
      const eid_t len = ro[r + 1] - ro[r];
      if (len < 2 || len > 4096) continue;
      std::sort(col + ro[r], col + ro[r + 1], [&](vid_t x, vid_t y) {
        return key_deg[x] != key_deg[y] ? key_deg[x] > key_deg[y] : x < y;
      });
    }
  }

  void sort_rows_by_id(const eid_t* ro, vid_t* col, int64_t rows, int64_t n) override {
    (void)n;
    for (int64_t r = 0; r < rows; ++r) std::sort(col + ro[r], col + ro[r + 1]);
  }

  void encode_hub_cols(const vid_t* col, int64_t nnz, const uint32_t* hub_idx, vid_t* out) override {
    for (int64_t e = 0; e < nnz; ++e) out[e] = hub_idx[col[e]] != 0xFFFFFFFFu ? (kHubFlag | hub_idx[col[e]]) : col[e];
  }
  void nz_word_counts(const eid_t* ro, int64_t rows, int64_t words, eid_t* counts) override {
    for (int64_t w = 0; w < words; ++w) {
      eid_t c = 0;
      for (int64_t v = w * 64; v < std::min<int64_t>(rows, (w + 1) * 64); ++v) c += ro[v + 1] > ro[v] ? 1 : 0;
      counts[w] = c;
    }
  }
  void nz_fill(const eid_t* ro, const vid_t* head, int64_t rows, const eid_t* pref, eid_t* nz_ro,
               vid_t* nz_head) override {
    int64_t k = 0;
    for (int64_t v = 0; v < rows; ++v) {
      if (ro[v + 1] > ro[v]) {
        nz_ro[k] = ro[v];
        nz_head[k] = head[v];
        ++k;
      }
    }
    nz_ro[k] = rows > 0 ? ro[rows] : 0;
    (void)pref;
  }
  void nz_records(const eid_t* ro, const vid_t* head, int64_t rows, const eid_t* pref, NzRec* rec,
                  eid_t* unit_base) override {
    const int64_t nunits = div_up(std::max<int64_t>(rows, 1), kUnitVertices);
    for (int64_t u = 0; u <= nunits; ++u) unit_base[u] = ro[std::min<int64_t>(u * kUnitVertices, rows)];
    int64_t k = 0;
    for (int64_t v = 0; v < rows; ++v) {
      if (ro[v + 1] > ro[v]) {
        rec[k].off = static_cast<uint32_t>(ro[v] - unit_base[v / kUnitVertices]);
        rec[k].head = head[v];
        ++k;
      }
    }
    (void)pref;
  }
  int64_t select_hubs(const uint32_t* deg, int64_t n, uint32_t min_deg, vid_t* hub_vertex,
                      uint32_t* hub_idx) override {
    int64_t k = 0;
    for (int64_t v = 0; v < n; ++v) {
      if (deg[v] >= min_deg) {
        hub_vertex[k] = static_cast<vid_t>(v);
        hub_idx[v] = static_cast<uint32_t>(k++);
      } else {
        hub_idx[v] = 0xFFFFFFFFu;
      }
    }
    return k;
  }
  void hub_gather(const HubGatherArgs& a) override {
    if (a.ctrl && (a.ctrl->done || a.ctrl->dir != 'B')) return;
    for (int64_t w = 0; w < div_up(a.g.nhubs, 64); ++w) {
      word_t m = 0;
      int64_t d = 0;
      for (int b = 0; b < 64 && w * 64 + b < a.g.nhubs; ++b) {
        const vid_t hv = a.g.hub_vertex[w * 64 + b];
        if (test_bit(a.frontier, hv)) {
          m |= 1ull << b;
          if (a.cut_part) d += a.g.hub_deg ? a.g.hub_deg[w * 64 + b] : a.g.row_off[hv + 1] - a.g.row_off[hv];
        }
      }
      a.hub_front[w] = m;
      if (a.cut_part) a.cut_part[w] = d;
    }
    if (a.cut_part) {
      int64_t hub_edges = 0;
      for (int64_t w = 0; w < div_up(a.g.nhubs, 64); ++w) hub_edges += a.cut_part[w];
      *a.cut_flag = a.ctrl->m_f - hub_edges <= a.cut_edges ? 1 : 0;
    }
    if (a.visited)
      for (int64_t i = 0; i < a.words; ++i) a.visited[i] |= a.frontier[i];
  }
  void bu_cut_prep(const BuArgs& a) override {
    if (a.ctrl && (a.ctrl->done || a.ctrl->dir != 'B')) return;
    if (!*a.cut_flag) return;
    const bool x = a.cut_bytes != nullptr;
    DBFS_CHECK(x || a.g.lo == 0, "bu_cut_prep: a shard past vertex 0 needs the several-rank arguments");
    const int64_t lo = a.g.lo, off = x ? a.cut_word_off : 0;
    const word_t* vis = x ? a.cut_vis : a.visited;
    for (int64_t w = 0; w < a.words; ++w)
      for (word_t m = a.frontier[off + w] & ~a.g.hub_bits[off + w]; m; m &= m - 1) {
        const int64_t v = w * 64 + __builtin_ctzll(m);
        for (eid_t e = a.g.row_off[v]; e < a.g.row_off[v + 1]; ++e) {
          const vid_t t = a.g.col[e];
          if (test_bit(vis, t)) continue;
          const int64_t r = static_cast<int64_t>(t) - lo;
          if (r < 0 || r >= a.g.rows) {
            DBFS_CHECK(x, "bu_cut_prep: a remote neighbour without the several-rank arguments");
            a.cut_bytes[t] = 1;
            continue;
          }
          if (a.cut_claim) a.cut_claim[r] = 1;
          else put_level(nullptr, a.level8, r, a.new_level, a.narrow_base);
        }
      }
  }
  void bu_cut_merge(const BuArgs& a) override {
    DBFS_CHECK(a.cut_flag && a.cut_recv && a.cut_next && (a.level8 || a.cut_claim) && a.cut_nranks > 1,
               "bu_cut_merge: several ranks' hub-cut arguments missing");
    if (a.ctrl && (a.ctrl->done || a.ctrl->dir != 'B')) return;
    if (!*a.cut_flag) return;
    for (int64_t w = 0; w < a.words; ++w) {
      word_t c = 0;
      for (int p = 0; p < a.cut_nranks; ++p) {
        if (p == a.cut_rank) continue;
        c |= a.cut_recv[p * a.words + w];
        a.cut_next[p * a.words + w] = 0;
      }
      for (c &= ~a.visited[w]; c; c &= c - 1) {
        const int64_t r = w * 64 + __builtin_ctzll(c);
        if (a.cut_claim) a.cut_claim[r] = 1;
        else put_level(nullptr, a.level8, r, a.new_level, a.narrow_base);
      }
    }
  }
  void hub_apply(const HubApplyArgs& a) override {
    if (a.ctrl && !chain_live(*a.ctrl, 'T', a.max_mf)) return;
    for (int64_t h = 0; h < a.g.td_nhubs; ++h) {
      if (!a.mark[h]) continue;
      const vid_t v = a.g.td_hub_vertex[h];
      a.level8[v] = static_cast<uint8_t>(a.narrow_base + a.new_level);
      a.mark[h] = 0;
    }
  }
  void refresh_visited(const RefreshArgs& a) override {
    if (a.ctrl && !chain_live(*a.ctrl, 'T', a.max_mf)) return;
    const uint8_t lv = static_cast<uint8_t>(a.narrow_base + a.new_level);
    for (int64_t w = 0; w < a.words; ++w) {
      word_t m = 0;
      for (int b = 0; b < 64; ++b)
        if (a.level8[w * 64 + b] == lv) m |= 1ull << b;
      a.visited[w] |= m;
    }
  }
  void hub_visited(const HubVisitedArgs& a) override {
    if (a.ctrl && !chain_live(*a.ctrl, 'T', 0)) return;
    for (int64_t w = 0; w < div_up(a.g.td_nhubs, 64); ++w) {
      word_t m = 0;
      for (int b = 0; b < 64 && w * 64 + b < a.g.td_nhubs; ++b)
        if (test_bit(a.visited, a.g.td_hub_vertex[w * 64 + b])) m |= 1ull << b;
      a.out[w] = m;
    }
  }
  void unvis_filter(const UnvisArgs& a) override {
    if (a.ctrl && !chain_live(*a.ctrl, 'T', a.max_mf)) return;
    std::fill(a.out, a.out + kUnvisWords, word_t(0));
    for (int64_t v = 0; v < a.n; ++v)
      if (!test_bit(a.visited, static_cast<vid_t>(v))) {
        const uint32_t i = unvis_index(static_cast<uint64_t>(v), a.mult);
        a.out[i >> 6] |= 1ull << (i & 63);
      }
  }
  void row_heads(const eid_t* ro, const vid_t* col, int64_t rows, vid_t* head, const uint32_t* hub_idx) override {
    for (int64_t r = 0; r < rows; ++r) {
      vid_t h = ro[r + 1] > ro[r] ? col[ro[r]] : 0u;
      if (hub_idx && ro[r + 1] > ro[r] && hub_idx[h] != 0xFFFFFFFFu) h = kHubFlag | hub_idx[h];
      head[r] = h;
    }
  }

  void gen_count_degrees(const GenParams& p, int64_t lo, int64_t rows, eid_t* deg) override {
    for (int64_t i = 0; i < p.m; ++i) {
      uint64_t u, v;
      gen_edge(p, static_cast<uint64_t>(i), u, v);
      if (static_cast<int64_t>(u) >= lo && static_cast<int64_t>(u) < lo + rows) ++deg[u - lo];
      if (static_cast<int64_t>(v) >= lo && static_cast<int64_t>(v) < lo + rows) ++deg[v - lo];
    }
  }

  void exclusive_scan(eid_t* data, int64_t n) override {
    eid_t acc = 0;
    for (int64_t i = 0; i < n; ++i) {
      const eid_t t = data[i];
      data[i] = acc;
      acc += t;
    }
    data[n] = acc;
  }

  void route_edges_count(const vid_t* u, const vid_t* v, int64_t m, int64_t part, int nranks,
                         int64_t* counts) override {
    for (int64_t i = 0; i < m; ++i) {
      ++counts[u[i] / part];
      ++counts[v[i] / part];
    }
    (void)nranks;
  }
  void route_edges_fill(const vid_t* u, const vid_t* v, int64_t m, int64_t part, int nranks, int64_t* cursor,
                        uint64_t* out) override {
    // edge order within every destination segment (the reference's adjacency
    // order survives the exchange: segments arrive in rank = file order)
    for (int64_t i = 0; i < m; ++i) {
      out[cursor[u[i] / part]++] = (static_cast<uint64_t>(u[i]) << 32) | v[i];
      out[cursor[v[i] / part]++] = (static_cast<uint64_t>(v[i]) << 32) | u[i];
    }
    (void)nranks;
  }
  void entries_count(const uint64_t* e, int64_t k, int64_t lo, eid_t* deg) override {
    for (int64_t i = 0; i < k; ++i) ++deg[static_cast<int64_t>(e[i] >> 32) - lo];
  }
  void entries_fill(const uint64_t* e, int64_t k, int64_t lo, eid_t* cursor, vid_t* col) override {
    for (int64_t i = 0; i < k; ++i)
      col[cursor[static_cast<int64_t>(e[i] >> 32) - lo]++] = static_cast<vid_t>(e[i] & 0xFFFFFFFFull);
  }
  void gen_fill(const GenParams& p, int64_t lo, int64_t rows, eid_t* cursor, vid_t* col) override {
    // Same order as build_csr (edge order, u-side then v-side).
    for (int64_t i = 0; i < p.m; ++i) {
      uint64_t u, v;
      gen_edge(p, static_cast<uint64_t>(i), u, v);
      if (static_cast<int64_t>(u) >= lo && static_cast<int64_t>(u) < lo + rows)
        col[cursor[u - lo]++] = static_cast<vid_t>(v);
      if (static_cast<int64_t>(v) >= lo && static_cast<int64_t>(v) < lo + rows)
        col[cursor[v - lo]++] = static_cast<vid_t>(u);
    }
  }

  void widen_levels(const uint8_t* in, lvl_t* out, int64_t n, uint8_t base) override {
    for (int64_t i = 0; i < n; ++i) {
      const uint8_t v = static_cast<uint8_t>(in[i] - base);
      out[i] = v > kNarrowMaxLevel ? kUnreached : static_cast<lvl_t>(v);
    }
  }
  void degree_moments(const ShardView& g, int64_t* out2) override {
    int64_t s = 0, c = 0;
    for (int64_t r = 0; r < g.rows; ++r) {
      const int64_t d = g.row_off[r + 1] - g.row_off[r];
      s += d * d;
      c += d > 0 ? 1 : 0;
    }
    out2[0] = s;
    out2[1] = c;
  }
  void reached_degree_sum(const ShardView& g, const lvl_t* level, int64_t* out2) override {
    int64_t c = 0, d = 0;
    for (int64_t r = 0; r < g.rows; ++r)
      if (level[r] != kUnreached) { ++c; d += g.row_off[r + 1] - g.row_off[r]; }
    out2[0] = c;
    out2[1] = d;
  }

 private:
  std::vector<std::chrono::steady_clock::time_point> events_;
};

}  // namespace

std::unique_ptr<Backend> make_cpu_backend() { return std::make_unique<CpuBackend>(); }

}  // namespace dbfs
