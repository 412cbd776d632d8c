// Distributed BFS engine (see dbfs/engine.hpp for the design summary).
//
// Per level of the bitmap engine (rank r of P, W = slice words):
//   TD: compact(frontier[r]) -> work list; memset(next); td_expand -> next (N bits);
//       P > 1: alltoall(next slices) -> recv (P x W words, OR-reduced in update)
//   BU: bu_step(visited[r], frontier[*]) -> cand (W words)
//   update(cand) -> visited[r] |= new, frontier[r] = new, level[new] = L+1,
//                   per-segment counts/degree sums
//   scan -> work-list offsets + local totals
//   P > 1: allgather(frontier[r]) -> frontier[*]; visited |= frontier
//   allreduce(totals) -> host: termination + Beamer direction heuristic
// Reference per level (bfs.cu:569-620): kernel per device, full device sync,
// serialized peer copies per (i, j), host reads of managed counters, memset.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "dbfs/engine.hpp"
#include "dbfs/shard_reader.hpp"
#include "dbfs/trace.hpp"
#include "spin.hpp"

namespace dbfs {

Mode parse_mode(const std::string& s) {
  if (s == "ref" || s == "reference") return Mode::Ref;
  if (s == "td" || s == "topdown" || s == "top-down") return Mode::TopDown;
  if (s == "bu" || s == "bottomup" || s == "bottom-up") return Mode::BottomUp;
  if (s == "do" || s == "diropt" || s == "direction-optimizing" || s == "hybrid") return Mode::DirOpt;
  if (s == "simple" || s == "status") return Mode::Simple;
  if (s == "scan") return Mode::Scan;
  throw Error("unknown mode '" + s + "' (expected ref|td|bu|do|simple|scan)");
}

const char* mode_name(Mode m) {
  switch (m) {
    case Mode::Ref: return "ref";
    case Mode::TopDown: return "td";
    case Mode::BottomUp: return "bu";
    case Mode::DirOpt: return "do";
    case Mode::Simple: return "simple";
    case Mode::Scan: return "scan";
  }
  return "?";
}

void set_engine_option(EngineOptions& o, const std::string& name, double v) {
  if (name == "alpha") o.alpha = v;
  else if (name == "beta") o.beta = v;
  else if (name == "bu_lane_limit") o.bu_lane_limit = static_cast<int>(v);
  else if (name == "td_byte_edges") o.td_byte_edges = static_cast<int64_t>(v);
  else if (name == "td_check_visited_min") o.td_check_visited_min = v;
  else if (name == "td_wide_below_blocks") o.td_wide_below_blocks = static_cast<int64_t>(v);
  else if (name == "sparse_max_edges") o.sparse_max_edges = static_cast<int64_t>(v);
  else if (name == "sparse_size_check") o.sparse_size_check = v != 0;
  else if (name == "force_exchange") o.force_exchange = v != 0;
  else if (name == "phase_timing") o.phase_timing = v != 0;
  else if (name == "device_loop") o.device_loop = v != 0;
  else if (name == "device_loop_predict") o.device_loop_predict = v != 0;
  else if (name == "directed") o.directed = v != 0;
  else if (name == "bu_whole_units") o.bu_whole_units = static_cast<int>(v);
  else if (name == "bu_small_waves") o.bu_small_waves = static_cast<int>(v);
  else if (name == "narrow_levels") o.narrow_levels = v != 0;
  else if (name == "td_sparse_edges") o.td_sparse_edges = static_cast<int64_t>(v);
  else if (name == "td_sparse_bits") o.td_sparse_bits = v != 0;
  else if (name == "td_bin_edges") o.td_bin_edges = static_cast<int64_t>(v);
  else if (name == "td_bin_min_rows") o.td_bin_min_rows = static_cast<int64_t>(v);
  else if (name == "td_unvis_edges") o.td_unvis_edges = static_cast<int64_t>(v);
  else if (name == "td_unvis_vis_frac") o.td_unvis_vis_frac = v;
  else if (name == "td_unvis_max_density") o.td_unvis_max_density = v;
  else if (name == "td_split_edges") o.td_split_edges = static_cast<int64_t>(v);
  else if (name == "td_split_parts") o.td_split_parts = std::max(1, static_cast<int>(v));
  else if (name == "td_hub_edges") o.td_hub_edges = static_cast<int64_t>(v);
  else if (name == "td_hub_vis_frac") o.td_hub_vis_frac = v;
  else if (name == "td_direct_edges") o.td_direct_edges = static_cast<int64_t>(v);
  else if (name == "list_form_edges") o.list_form_edges = static_cast<int64_t>(v);
  else if (name == "xsparse_edges") o.xsparse_edges = static_cast<int64_t>(v);
  else if (name == "xfuse_edges") o.xfuse_edges = static_cast<int64_t>(v);
  else if (name == "bu_merge_visited") o.bu_merge_visited = v != 0;
  else if (name == "bu_cut_edges") o.bu_cut_edges = static_cast<int64_t>(v);
  else if (name == "bu_cut_mf_frac") o.bu_cut_mf_frac = v;
  else if (name == "bu_cut_ranks") o.bu_cut_ranks = static_cast<int64_t>(v);
  else if (name == "list_cap_factor") o.list_cap_factor = v;
  else if (name == "direct_frontier") o.direct_frontier = v != 0;
  else throw Error("unknown engine option '" + name + "'");
}

std::vector<std::pair<std::string, double>> engine_option_map(const EngineOptions& o) {
  return {{"alpha", o.alpha},
          {"beta", o.beta},
          {"bu_lane_limit", o.bu_lane_limit},
          {"td_byte_edges", static_cast<double>(o.td_byte_edges)},
          {"td_check_visited_min", o.td_check_visited_min},
          {"td_wide_below_blocks", static_cast<double>(o.td_wide_below_blocks)},
          {"sparse_max_edges", static_cast<double>(o.sparse_max_edges)},
          {"sparse_size_check", o.sparse_size_check ? 1.0 : 0.0},
          {"force_exchange", o.force_exchange ? 1.0 : 0.0},
          {"phase_timing", o.phase_timing ? 1.0 : 0.0},
          {"device_loop", o.device_loop ? 1.0 : 0.0},
          {"device_loop_predict", o.device_loop_predict ? 1.0 : 0.0},
          {"directed", o.directed ? 1.0 : 0.0},
          {"bu_whole_units", static_cast<double>(o.bu_whole_units)},
          {"bu_small_waves", static_cast<double>(o.bu_small_waves)},
          {"td_sparse_edges", static_cast<double>(o.td_sparse_edges)},
          {"td_sparse_bits", o.td_sparse_bits ? 1.0 : 0.0},
          {"narrow_levels", o.narrow_levels ? 1.0 : 0.0},
          {"td_bin_edges", static_cast<double>(o.td_bin_edges)},
          {"td_bin_min_rows", static_cast<double>(o.td_bin_min_rows)},
          {"td_unvis_edges", static_cast<double>(o.td_unvis_edges)},
          {"td_unvis_vis_frac", o.td_unvis_vis_frac},
          {"td_unvis_max_density", o.td_unvis_max_density},
          {"td_split_edges", static_cast<double>(o.td_split_edges)},
          {"td_split_parts", static_cast<double>(o.td_split_parts)},
          {"td_hub_edges", static_cast<double>(o.td_hub_edges)},
          {"td_hub_vis_frac", o.td_hub_vis_frac},
          {"td_direct_edges", static_cast<double>(o.td_direct_edges)},
          {"list_form_edges", static_cast<double>(o.list_form_edges)},
          {"xsparse_edges", static_cast<double>(o.xsparse_edges)},
          {"xfuse_edges", static_cast<double>(o.xfuse_edges)},
          {"bu_merge_visited", o.bu_merge_visited ? 1.0 : 0.0},
          {"bu_cut_edges", static_cast<double>(o.bu_cut_edges)},
          {"bu_cut_mf_frac", o.bu_cut_mf_frac},
          {"bu_cut_ranks", static_cast<double>(o.bu_cut_ranks)},
          {"list_cap_factor", o.list_cap_factor},
          {"direct_frontier", o.direct_frontier ? 1.0 : 0.0}};
}

// ---- DeviceGraph ----------------------------------------------------------------

std::unique_ptr<DeviceGraph> DeviceGraph::from_host(Backend& be, const HostCSR& csr, const Partition& part,
                                                    int rank) {
  DBFS_CHECK(csr.n == part.n, "partition vertex count does not match the graph");
  auto g = std::unique_ptr<DeviceGraph>(new DeviceGraph());
  g->be_ = &be;
  g->part_ = part;
  g->rank_ = rank;
  g->lo_ = part.lo(rank);
  g->rows_ = part.count(rank);
  g->input_edges_ = csr.input_edges;
  const eid_t* ro = nullptr;
  const vid_t* col = nullptr;
  std::vector<eid_t> rel;
  if (csr.row_lo == 0 && csr.rows == csr.n) {
    const eid_t base = csr.row_off[g->lo_];
    rel.resize(static_cast<size_t>(g->rows_ + 1));
    for (int64_t r = 0; r <= g->rows_; ++r) rel[r] = csr.row_off[g->lo_ + r] - base;
    ro = rel.data();
    col = csr.col.data() + base;
  } else {
    DBFS_CHECK(csr.row_lo == g->lo_ && csr.rows == g->rows_, "host shard does not match this rank's partition");
    ro = csr.row_off.data();
    col = csr.col.data();
  }
  g->nnz_ = ro[g->rows_];
  g->row_off_ = DBuf<eid_t>(be, static_cast<size_t>(g->rows_ + 1));
  g->col_ = DBuf<vid_t>(be, static_cast<size_t>(std::max<int64_t>(g->nnz_, 1)));
  be.to_device(g->row_off_.data(), ro, static_cast<size_t>(g->rows_ + 1) * sizeof(eid_t));
  if (g->nnz_) be.to_device(g->col_.data(), col, static_cast<size_t>(g->nnz_) * sizeof(vid_t));
  g->build_heads();
  return g;
}

std::unique_ptr<DeviceGraph> DeviceGraph::generate(Backend& be, const GenParams& p, const Partition& part, int rank) {
  DBFS_CHECK(p.n == part.n, "partition vertex count does not match the generator");
  DBFS_CHECK(p.n <= int64_t(UINT32_MAX), "generator vertex count exceeds 2^32");
  auto g = std::unique_ptr<DeviceGraph>(new DeviceGraph());
  g->be_ = &be;
  g->part_ = part;
  g->rank_ = rank;
  g->lo_ = part.lo(rank);
  g->rows_ = part.count(rank);
  g->input_edges_ = p.m;
  g->row_off_ = DBuf<eid_t>(be, static_cast<size_t>(g->rows_ + 1));
  be.memset_async(g->row_off_.data(), 0, g->row_off_.bytes());
  be.gen_count_degrees(p, g->lo_, g->rows_, g->row_off_.data());
  be.exclusive_scan(g->row_off_.data(), g->rows_);
  eid_t nnz = 0;
  be.to_host(&nnz, g->row_off_.data() + g->rows_, sizeof(eid_t));
  g->nnz_ = nnz;
  g->col_ = DBuf<vid_t>(be, static_cast<size_t>(std::max<int64_t>(nnz, 1)));
  {
    DBuf<eid_t> cursor(be, static_cast<size_t>(std::max<int64_t>(g->rows_, 1)));
    be.copy_async(cursor.data(), g->row_off_.data(), static_cast<size_t>(g->rows_) * sizeof(eid_t));
    be.gen_fill(p, g->lo_, g->rows_, cursor.data(), g->col_.data());
    be.synchronize();
  }
  g->build_heads();
  return g;
}

std::unique_ptr<DeviceGraph> DeviceGraph::from_edges(Backend& be, Comm& comm, const Partition& part, int rank,
                                                     int64_t input_edges, const vid_t* u, const vid_t* v,
                                                     int64_t m_local) {
  DBFS_CHECK(comm.size() == part.nranks && comm.rank() == rank, "communicator does not match the partition");
  DBFS_CHECK(m_local >= 0, "negative edge count");
  comm.bind_backend(&be);
  const int P = part.nranks;
  auto g = std::unique_ptr<DeviceGraph>(new DeviceGraph());
  g->be_ = &be;
  g->part_ = part;
  g->rank_ = rank;
  g->lo_ = part.lo(rank);
  g->rows_ = part.count(rank);
  g->input_edges_ = input_edges;
  // (1) this rank's edges -> entries per owner, grouped by owner
  std::vector<int64_t> sc(static_cast<size_t>(P), 0), rc(static_cast<size_t>(P), 0);
  DBuf<uint64_t> send;
  {
    DBuf<vid_t> du(be, static_cast<size_t>(std::max<int64_t>(m_local, 1)));
    DBuf<vid_t> dv(be, static_cast<size_t>(std::max<int64_t>(m_local, 1)));
    if (m_local) {
      be.to_device(du.data(), u, static_cast<size_t>(m_local) * sizeof(vid_t));
      be.to_device(dv.data(), v, static_cast<size_t>(m_local) * sizeof(vid_t));
    }
    DBuf<int64_t> cnt(be, static_cast<size_t>(P)), rcnt(be, static_cast<size_t>(P));
    be.memset_async(cnt.data(), 0, cnt.bytes());
    be.route_edges_count(du.data(), dv.data(), m_local, part.part, P, cnt.data());
    // (2) entry counts to their owners
    comm.alltoall(cnt.data(), rcnt.data(), sizeof(int64_t));
    be.to_host(sc.data(), cnt.data(), cnt.bytes());
    be.to_host(rc.data(), rcnt.data(), rcnt.bytes());
    std::vector<int64_t> sd(static_cast<size_t>(P), 0);
    for (int r = 1; r < P; ++r) sd[r] = sd[r - 1] + sc[r - 1];
    const int64_t total = sd[P - 1] + sc[P - 1];
    DBFS_CHECK(total == 2 * m_local, "edge routing lost entries");
    send = DBuf<uint64_t>(be, static_cast<size_t>(std::max<int64_t>(total, 1)));
    be.to_device(cnt.data(), sd.data(), sd.size() * sizeof(int64_t));  // cursors = segment starts
    be.route_edges_fill(du.data(), dv.data(), m_local, part.part, P, cnt.data(), send.data());
    be.synchronize();
  }
  // (3) all-to-all-v of the entries (in rank order: file order per owner)
  std::vector<int64_t> sd(static_cast<size_t>(P), 0), rd(static_cast<size_t>(P), 0);
  for (int r = 1; r < P; ++r) {
    sd[r] = sd[r - 1] + sc[r - 1];
    rd[r] = rd[r - 1] + rc[r - 1];
  }
  const int64_t nrecv = rd[P - 1] + rc[P - 1];
  DBuf<uint64_t> recv(be, static_cast<size_t>(std::max<int64_t>(nrecv, 1)));
  comm.alltoallv(send.data(), sc.data(), sd.data(), recv.data(), rc.data(), rd.data(), sizeof(uint64_t));
  be.synchronize();
  send.reset();
  // (4) the shard: degrees -> offsets -> fill
  g->row_off_ = DBuf<eid_t>(be, static_cast<size_t>(g->rows_ + 1));
  be.memset_async(g->row_off_.data(), 0, g->row_off_.bytes());
  be.entries_count(recv.data(), nrecv, g->lo_, g->row_off_.data());
  be.exclusive_scan(g->row_off_.data(), g->rows_);
  eid_t nnz = 0;
  be.to_host(&nnz, g->row_off_.data() + g->rows_, sizeof(eid_t));
  DBFS_CHECK(nnz == nrecv, "entries outside this rank's rows");
  g->nnz_ = nnz;
  g->col_ = DBuf<vid_t>(be, static_cast<size_t>(std::max<int64_t>(nnz, 1)));
  {
    DBuf<eid_t> cursor(be, static_cast<size_t>(std::max<int64_t>(g->rows_, 1)));
    be.copy_async(cursor.data(), g->row_off_.data(), static_cast<size_t>(g->rows_) * sizeof(eid_t));
    be.entries_fill(recv.data(), nrecv, g->lo_, cursor.data(), g->col_.data());
    be.synchronize();
  }
  g->build_heads();
  return g;
}

std::unique_ptr<DeviceGraph> DeviceGraph::from_file(Backend& be, Comm& comm, const std::string& path, int threads) {
  comm.bind_backend(&be);
  const int P = comm.size(), rank = comm.rank();
  if (is_binary_csr(path)) {
    const BinaryCsrInfo info = binary_csr_info(path);
    DBFS_CHECK(info.row_lo == 0 && info.rows == info.n, "a sharded read needs a whole-graph binary cache: " + path);
    const Partition part = Partition::block(info.n, P);
    const HostCSR shard = read_binary_csr_rows(path, part.lo(rank), part.lo(rank) + part.count(rank));
    auto g = from_host(be, shard, part, rank);
    g->ingest_.edges = shard.rows;
    return g;
  }
  const EdgeShard es = read_edge_shard(
      path, rank, P, [&comm](int64_t x) { return comm.allgather_host_i64(x); }, threads);
  const Partition part = Partition::block(es.n, P);
  auto g = from_edges(be, comm, part, rank, es.m, es.u.data(), es.v.data(), es.local_edges());
  g->ingest_ = {es.byte_begin, es.byte_end, es.local_edges()};
  return g;
}

ShardView DeviceGraph::view() const {
  ShardView v;
  v.row_off = row_off_.data();
  v.col = col_.data();
  v.n = part_.n;
  v.lo = lo_;
  v.rows = rows_;
  v.nnz = nnz_;
  v.head = head_.data();
  v.hub_vertex = hub_vertex_.data();
  v.nhubs = nhubs_;
  v.hub_col = hub_col_.data();
  v.hub_bits = hub_bits_.data();
  v.hub_deg = hub_deg_.data();
  v.nz_pref = nz_pref_.data();
  v.nz_row_off = nz_row_off_.data();
  v.nz_head = nz_head_.data();
  v.nz_rec = nz_rec_.data();
  v.unit_base = unit_base_.data();
  if (td_nhubs_ > 0) {
    v.td_col = td_col_.data();
    v.td_hub_vertex = td_hub_vertex_.data();
    v.td_nhubs = td_nhubs_;
  }
  return v;
}

HostCSR DeviceGraph::to_host() const {
  HostCSR h;
  h.n = part_.n;
  h.row_lo = lo_;
  h.rows = rows_;
  h.input_edges = input_edges_;
  h.row_off.resize(static_cast<size_t>(rows_ + 1));
  h.col.resize(static_cast<size_t>(nnz_));
  be_->to_host(h.row_off.data(), row_off_.data(), h.row_off.size() * sizeof(eid_t));
  if (nnz_) be_->to_host(h.col.data(), col_.data(), h.col.size() * sizeof(vid_t));
  return h;
}

std::vector<eid_t> DeviceGraph::degrees_of(const std::vector<int64_t>& local_rows) const {
  std::vector<eid_t> out;
  out.reserve(local_rows.size());
  for (int64_t r : local_rows) {
    DBFS_CHECK(r >= 0 && r < rows_, "row out of range");
    eid_t a[2];
    be_->to_host(a, row_off_.data() + r, sizeof(a));
    out.push_back(a[1] - a[0]);
  }
  return out;
}

// Smallest degree d >= 1 with |{v : deg(v) >= d}| <= cap (0: no vertex has
// degree >= 1).
static uint32_t hub_min_degree(const std::vector<uint32_t>& deg, int64_t cap) {
  constexpr uint32_t kCapDeg = 1u << 20;  // histogram range; larger degrees share the top bucket
  std::vector<int64_t> hist(kCapDeg + 1, 0);
  for (uint32_t d : deg) ++hist[std::min(d, kCapDeg)];
  int64_t acc = 0;
  uint32_t best = 0;
  for (uint32_t d = kCapDeg; d >= 1; --d) {
    acc += hist[d];
    if (acc > cap) break;
    best = d;
  }
  return best;
}

void DeviceGraph::sort_neighbors_by_degree(Comm& comm, bool hubs, int64_t max_hubs, bool id_order, bool td_hubs) {
  DBFS_CHECK(max_hubs >= 0 && max_hubs <= kMaxHubs, "max_hubs out of range");
  DBFS_CHECK(comm.size() == part_.nranks && comm.rank() == rank_, "communicator does not match the shard");
  comm.bind_backend(be_);
  const int P = part_.nranks;
  const int64_t part = part_.part;
  const int64_t nall = static_cast<int64_t>(P) * part;
  DBuf<uint32_t> mine(*be_, static_cast<size_t>(part)), all(*be_, static_cast<size_t>(nall));
  be_->memset_async(mine.data(), 0, mine.bytes());
  be_->degrees_u32(row_off_.data(), rows_, mine.data());
  comm.allgather(mine.data(), all.data(), static_cast<size_t>(part) * sizeof(uint32_t));
  be_->sort_neighbors(row_off_.data(), col_.data(), rows_, all.data());
  nhubs_ = 0;
  hub_vertex_.reset();
  hub_bits_.reset();
  hub_deg_.reset();
  hub_col_.reset();
  td_col_.reset();
  td_hub_vertex_.reset();
  td_nhubs_ = 0;
  td_hub_share_ = 0.0;
  col_by_id_ = false;
  // Hub encoding needs a free flag bit in the vertex ids.
  if (hubs && part_.n > 0 && nall <= static_cast<int64_t>(kHubFlag)) {
    std::vector<uint32_t> deg(static_cast<size_t>(nall));
    be_->to_host(deg.data(), all.data(), deg.size() * sizeof(uint32_t));
    const uint32_t min_deg = hub_min_degree(deg, max_hubs);
    if (min_deg > 0) {
      DBuf<uint32_t> hub_idx(*be_, static_cast<size_t>(nall));
      hub_vertex_ = DBuf<vid_t>(*be_, static_cast<size_t>(std::max<int64_t>(max_hubs, 1)));
      nhubs_ = be_->select_hubs(all.data(), nall, min_deg, hub_vertex_.data(), hub_idx.data());
      DBFS_CHECK(nhubs_ >= 0 && nhubs_ <= max_hubs, "hub selection exceeded its capacity");
      if (nhubs_ > 0) {
        // hub membership bitmap over all vertices (hub-cut bottom-up levels)
        std::vector<vid_t> hv(static_cast<size_t>(nhubs_));
        be_->to_host(hv.data(), hub_vertex_.data(), hv.size() * sizeof(vid_t));
        std::vector<word_t> bits(static_cast<size_t>(part_.global_words()), 0ull);
        for (vid_t v : hv) bits[v >> 6] |= 1ull << (v & 63);
        hub_bits_ = DBuf<word_t>(*be_, bits.size());
        be_->to_device(hub_bits_.data(), bits.data(), bits.size() * sizeof(word_t));
        // the hubs' degrees (several ranks: the hub-cut decision)
        std::vector<uint32_t> hd(hv.size());
        for (size_t i = 0; i < hv.size(); ++i) hd[i] = deg[hv[i]];
        hub_deg_ = DBuf<uint32_t>(*be_, hd.size());
        be_->to_device(hub_deg_.data(), hd.data(), hd.size() * sizeof(uint32_t));
      }
      // bottom-up's hub-encoded adjacency copy (one more nnz x 4 B: RMAT-26
      // 8.6 GB of the 288 GB HBM3E)
      hub_col_ = DBuf<vid_t>(*be_, static_cast<size_t>(std::max<int64_t>(nnz_, 1)));
      be_->encode_hub_cols(col_.data(), nnz_, hub_idx.data(), hub_col_.data());
      build_heads(hub_idx.data());
      // (only when bottom-up has the hub kernels -- the only ones that scan
      // hub_col -- i.e. at least one hub was selected)
      if (id_order && nhubs_ > 0) {
        be_->sort_rows_by_id(row_off_.data(), col_.data(), rows_, part_.n);
        col_by_id_ = true;
        if (td_hubs) {
          // top-down hubs: the kTdMaxHubs highest-degree vertices (their
          // visited bits fit LDS next to the top-down owner map)
          const uint32_t td_min = hub_min_degree(deg, std::min<int64_t>(kTdMaxHubs, max_hubs));
          if (td_min > 0) {
            DBuf<uint32_t> td_idx(*be_, static_cast<size_t>(nall));
            td_hub_vertex_ = DBuf<vid_t>(*be_, static_cast<size_t>(kTdMaxHubs));
            td_nhubs_ = be_->select_hubs(all.data(), nall, td_min, td_hub_vertex_.data(), td_idx.data());
            {
              double hub_sum = 0.0, all_sum = 0.0;
              for (uint32_t d : deg) {
                all_sum += d;
                if (d >= td_min) hub_sum += d;
              }
              td_hub_share_ = all_sum > 0 ? hub_sum / all_sum : 0.0;
            }
            if (td_nhubs_ > 0) {
              td_col_ = DBuf<vid_t>(*be_, static_cast<size_t>(std::max<int64_t>(nnz_, 1)));
              be_->encode_hub_cols(col_.data(), nnz_, td_idx.data(), td_col_.data());
            }
            be_->synchronize();
          }
        }
      }
    } else {
      build_heads();
    }
  } else {
    build_heads();
  }
  // whether every rank has the packed row records (a shard of no rows, or
  // with a unit of 2^32+ edges, has none): the several-rank hub cut needs
  // them on all (its chains carry a collective, so the choice must agree)
  {
    DBuf<int64_t> miss(*be_, 1);
    const int64_t m = nz_rec_.data() && unit_base_.data() ? 0 : 1;
    be_->to_device(miss.data(), &m, sizeof(m));
    if (P > 1) comm.allreduce_sum_i64(miss.data(), 1);
    int64_t h = 0;
    be_->to_host(&h, miss.data(), sizeof(h));
    rec_all_ = h == 0;
  }
  hub_sorted_ = true;
}

void DeviceGraph::build_heads(const uint32_t* hub_idx) {
  if (head_.size() < static_cast<size_t>(std::max<int64_t>(rows_, 1)))
    head_ = DBuf<vid_t>(*be_, static_cast<size_t>(std::max<int64_t>(rows_, 1)));
  be_->row_heads(row_off_.data(), col_.data(), rows_, head_.data(), hub_idx);
  build_nz_view();
  be_->synchronize();
}

// Dense copies of row_off / head over the non-empty rows (ShardView::nz_*),
// rebuilt whenever the heads change.
void DeviceGraph::build_nz_view() {
  const int64_t words = div_up(std::max<int64_t>(rows_, 1), kWordBits);
  nz_pref_ = DBuf<eid_t>(*be_, static_cast<size_t>(words + 1));
  be_->memset_async(nz_pref_.data(), 0, nz_pref_.bytes());
  be_->nz_word_counts(row_off_.data(), rows_, words, nz_pref_.data());
  be_->exclusive_scan(nz_pref_.data(), words);
  eid_t nzrows = 0;
  be_->to_host(&nzrows, nz_pref_.data() + words, sizeof(eid_t));
  nz_row_off_ = DBuf<eid_t>(*be_, static_cast<size_t>(nzrows + 1));
  nz_head_ = DBuf<vid_t>(*be_, static_cast<size_t>(std::max<eid_t>(nzrows, 1)));
  be_->nz_fill(row_off_.data(), head_.data(), rows_, nz_pref_.data(), nz_row_off_.data(), nz_head_.data());
  // packed records, when every unit's edges fit 32-bit relative offsets
  nz_rec_ = DBuf<NzRec>();
  unit_base_ = DBuf<eid_t>();
  if (rows_ <= 0) return;
  const int64_t nunits = div_up(rows_, kUnitVertices);
  unit_base_ = DBuf<eid_t>(*be_, static_cast<size_t>(nunits + 1));
  nz_rec_ = DBuf<NzRec>(*be_, static_cast<size_t>(std::max<eid_t>(nzrows, 1)));
  be_->nz_records(row_off_.data(), head_.data(), rows_, nz_pref_.data(), nz_rec_.data(), unit_base_.data());
  std::vector<eid_t> ub(static_cast<size_t>(nunits + 1));
  be_->to_host(ub.data(), unit_base_.data(), ub.size() * sizeof(eid_t));
  for (int64_t u = 0; u < nunits; ++u)
    if (ub[static_cast<size_t>(u + 1)] - ub[static_cast<size_t>(u)] >= (eid_t(1) << 32)) {
      nz_rec_ = DBuf<NzRec>();
      unit_base_ = DBuf<eid_t>();
      break;
    }
}

// ---- Engine ----------------------------------------------------------------------

Engine::Engine(DeviceGraph& g, Comm& comm, const EngineOptions& opt)
    : g_(g), comm_(comm), be_(g.backend()), opt_(opt), part_(g.partition()), fault_(FaultSpec::from_env()) {
  DBFS_CHECK(comm.size() == part_.nranks, "communicator size does not match the partition");
  DBFS_CHECK(comm.rank() == g.rank(), "communicator rank does not match the shard");
  comm_.bind_backend(&be_);
  total_directed_ = comm_.sum_host(g.nnz());
  level_ = DBuf<lvl_t>(be_, static_cast<size_t>(std::max<int64_t>(g.rows(), 1)));
  be_.fill_level(level_.data(), g.rows(), kUnreached);
}

Engine::~Engine() {
  if (mailbox_host_) be_.free_mapped(mailbox_host_);
  for (auto& seg : rec_segs_) be_.free_mapped(seg.first);
  if (stats_mb_host_) be_.free_mapped(stats_mb_host_);
}


// Totals of the level just scanned (stats[0..3]: local count, local degree
// sum, global count, global degree sum) to the host.
void Engine::read_level_stats(int64_t* host_stats) {
  if (!stats_mb_host_) {
    void* dptr = nullptr;
    stats_mb_host_ = static_cast<StatsMailbox*>(be_.alloc_mapped(sizeof(StatsMailbox), &dptr));
    stats_mb_dev_ = static_cast<StatsMailbox*>(dptr);
  }
  const int64_t seq = ++stats_seq_;
  be_.publish_stats(stats_.data(), stats_mb_dev_, seq);
  StatsMailbox* mb = stats_mb_host_;
  spin_until(be_, [&] { return __atomic_load_n(&mb->seq, __ATOMIC_ACQUIRE) == seq; },
             "level statistics mailbox: stream drained without the stamp");
  for (int k = 0; k < 4; ++k) host_stats[k] = __atomic_load_n(&mb->v[k], __ATOMIC_RELAXED);
}

// ---- fault injection -------------------------------------------
// DBFS_FAULT_INJECT="rank=R,level=L[,kind=throw|exit|hang]" makes rank R fail
// at the start of level L of every run: `throw` raises an Error (in-process
// ranks abort their group), `exit` ends the process with status 17 (a crashed
// rank), `hang` stops participating (peers must time out), `device` records
// a device-check violation (the run fails when it ends), `delay` enqueues the
// level ms late; kind=late_wg[,us=U] (every rank, every level) makes the
// workgroups of a sparse top-down level that take no ticket start U us late
// on the device (TdSparseArgs::late_ticks).  Used by the failure-detection
// and level-loop tests; unset in normal runs.
FaultSpec FaultSpec::from_env() {
  FaultSpec f;
  const char* e = std::getenv("DBFS_FAULT_INJECT");
  if (!e || !*e) return f;
  std::string s(e);
  size_t pos = 0;
  while (pos < s.size()) {
    size_t comma = s.find(',', pos);
    if (comma == std::string::npos) comma = s.size();
    const std::string kv = s.substr(pos, comma - pos);
    const size_t eq = kv.find('=');
    DBFS_CHECK(eq != std::string::npos, "DBFS_FAULT_INJECT: expected key=value, got '" + kv + "'");
    const std::string k = kv.substr(0, eq), v = kv.substr(eq + 1);
    if (k == "rank") f.rank = std::stoi(v);
    else if (k == "level") f.level = std::stoi(v);
    else if (k == "kind") f.kind = v;
    else if (k == "ms") f.ms = std::stoi(v);
    else if (k == "us") f.us = std::stoi(v);
    else DBFS_CHECK(false, "DBFS_FAULT_INJECT: unknown key '" + k + "'");
    pos = comma + 1;
  }
  DBFS_CHECK(f.kind == "throw" || f.kind == "exit" || f.kind == "hang" || f.kind == "device" || f.kind == "delay" ||
                 f.kind == "rccl_init" || f.kind == "peer_init" || f.kind == "late_wg",
             "DBFS_FAULT_INJECT: kind must be throw|exit|hang|device|delay|rccl_init|peer_init|late_wg");
  // (rccl_init / peer_init: the communicators' setup fails -- NcclComm /
  // PeerComm read them; late_wg: every sparse top-down level's ticket-less
  // workgroups start late, on every rank (DeviceLoop::emit_sparse) -- the
  // engine injects nothing at a level)
  if (f.kind == "rccl_init" || f.kind == "peer_init" || f.kind == "late_wg") f.rank = -1;
  return f;
}

// Device-checked build: the first bounds violation a kernel recorded during
// the traversal fails the run (codes: DBFS_DCHECK sites in the {bfs,td,bu}_kernels.hip files).
void Engine::check_device() {
  const uint64_t v = be_.take_device_check();
  if (v == 0) return;
  char buf[160];
  std::snprintf(buf, sizeof(buf), "device check failed on rank %d: code %llu, detail %llu", comm_.rank(),
                static_cast<unsigned long long>(v >> 48), static_cast<unsigned long long>(v & 0xFFFFFFFFFFFFull));
  throw Error(buf);
}

void Engine::inject_fault(int level) {
  if (fault_.rank != comm_.rank() || fault_.level != level) return;
  if (fault_.kind == "device") {
    // a kernel-side bounds violation (recorded, not raised: the traversal
    // completes and Engine::check_device fails it afterwards)
    be_.inject_device_check();
    return;
  }
  if (fault_.kind == "delay") {
    // this rank enqueues the level late (the host sleeps before its chain):
    // its peers' kernels of that level are already waiting for its
    // exchanges on the device -- the traversal must still complete exactly
    std::this_thread::sleep_for(std::chrono::milliseconds(fault_.ms));
    return;
  }
  const std::string what = "injected fault (" + fault_.kind + ") at level " + std::to_string(level) + " on rank " +
                           std::to_string(fault_.rank);
  std::fprintf(stderr, "[dbfs] %s\n", what.c_str());
  std::fflush(stderr);
  if (fault_.kind == "exit") std::_Exit(17);
  if (fault_.kind == "hang") {
    // bounded, so an unattended run still ends eventually
    for (int i = 0; i < 3600; ++i) std::this_thread::sleep_for(std::chrono::seconds(1));
  }
  throw Error(what);
}

void Engine::alloc_bitmap_state() {
  if (bitmap_ready_) return;
  const int64_t W = part_.slice_words(), GW = part_.global_words();
  visited_ = DBuf<word_t>(be_, static_cast<size_t>(GW));
  zdeg_ = DBuf<word_t>(be_, static_cast<size_t>(GW));
  frontier_[0] = DBuf<word_t>(be_, static_cast<size_t>(GW));
  frontier_[1] = DBuf<word_t>(be_, static_cast<size_t>(GW));
  next_ = DBuf<word_t>(be_, static_cast<size_t>(GW));
  if (exchange()) recv_ = DBuf<word_t>(be_, static_cast<size_t>(GW));
  cand_ = DBuf<word_t>(be_, static_cast<size_t>(W));
  nunits_ = div_up(W, kUnitWords);
  unit_cnt_ = DBuf<int64_t>(be_, static_cast<size_t>(nunits_ + 1));
  unit_deg_ = DBuf<int64_t>(be_, static_cast<size_t>(nunits_ + 1));
  part_cnt_ = DBuf<int64_t>(be_, static_cast<size_t>(div_up(nunits_, kScanChunk) + 1));
  part_deg_ = DBuf<int64_t>(be_, static_cast<size_t>(div_up(nunits_, kScanChunk) + 1));
  // (never read before written by a scan, except by a compaction of an empty
  // owned frontier, which ignores them: zeroed anyway)
  be_.memset_async(unit_cnt_.data(), 0, unit_cnt_.bytes());
  be_.memset_async(unit_deg_.data(), 0, unit_deg_.bytes());
  be_.memset_async(part_cnt_.data(), 0, part_cnt_.bytes());
  be_.memset_async(part_deg_.data(), 0, part_deg_.bytes());
  ticket_ = DBuf<unsigned>(be_, 4);
  be_.memset_async(ticket_.data(), 0, ticket_.bytes());
  qscan_ = DBuf<int64_t>(be_, static_cast<size_t>(g_.rows() + 1));
  qbase_ = DBuf<int64_t>(be_, static_cast<size_t>(std::max<int64_t>(g_.rows(), 1)));
  blk_vstart_ = DBuf<int32_t>(be_, static_cast<size_t>(div_up(g_.nnz(), kTdEdgesPerBlock) + 2));
  // kStatsBlocks (several ranks) or kStatsBlocks1 (one rank) blocks of
  // [local count, local degree sum, global count, global degree sum, ...]
  // (one 64-byte line each; block 0's [4..5] also hold the degree moments
  // before the first run)
  stats_stride_ = 8;
  stats_ = DBuf<int64_t>(be_, static_cast<size_t>((exchange() ? kStatsBlocks : kStatsBlocks1) * stats_stride_));
  be_.memset_async(stats_.data(), 0, stats_.bytes());
  if (g_.nhubs() > 0) hub_front_ = DBuf<word_t>(be_, static_cast<size_t>(div_up(g_.nhubs(), kWordBits)));
  // Zero-degree (and padding) vertices can never be discovered: they start out
  // visited, so bottom-up steps skip them without touching row_off.
  ZeroDegArgs za;
  za.g = g_.view();
  za.padding_only = opt_.directed;  // a directed vertex without out-edges can still be reached
  za.out = zdeg_.data() + comm_.rank() * W;
  za.words = W;
  be_.zero_degree_mask(za);
  if (exchange()) comm_.allgather(za.out, zdeg_.data(), static_cast<size_t>(W) * sizeof(word_t));
  if (exchange()) {
    // every vertex's degree on every rank (4 B per vertex): a traversal's
    // seed totals without a collective (InitRunArgs::deg_all)
    deg_all_ = DBuf<uint32_t>(be_, static_cast<size_t>(part_.nranks) * static_cast<size_t>(part_.part));
    DBuf<uint32_t> mine(be_, static_cast<size_t>(part_.part));
    be_.memset_async(mine.data(), 0, mine.bytes());
    be_.degrees_u32(g_.view().row_off, g_.rows(), mine.data());
    comm_.allgather(mine.data(), deg_all_.data(), static_cast<size_t>(part_.part) * sizeof(uint32_t));
    be_.synchronize();
  }
  be_.synchronize();
  bitmap_ready_ = true;
}

void Engine::alloc_ref_state() {
  const int P = part_.nranks;
  const int64_t cap = part_.part;
  if (opt_.mode == Mode::Scan && claim_.size() == 0) {
    DBFS_CHECK(P <= 64, "scan mode supports at most 64 ranks");
    claim_ = DBuf<eid_t>(be_, static_cast<size_t>(std::max<int64_t>(part_.n, 1)));
    scan_offs_ = DBuf<eid_t>(be_, static_cast<size_t>(P * cap + 1));
  }
  if (ref_ready_) return;
  dist_ =DBuf<lvl_t>(be_, static_cast<size_t>(std::max<int64_t>(part_.n, 1)));
  queue_ = DBuf<vid_t>(be_, static_cast<size_t>(std::max<int64_t>(cap, 1)));
  buckets_ = DBuf<vid_t>(be_, static_cast<size_t>(P * cap));
  recvq_ = DBuf<vid_t>(be_, static_cast<size_t>(P * cap));
  // [0, P) send counts, [P, 2P) receive counts, [2P, 3P] scan-mode bounds
  bucket_cnt_ = DBuf<int64_t>(be_, static_cast<size_t>(3 * P + 1));
  qcount_ = DBuf<int64_t>(be_, 1);
  ref_ready_ = true;
}

RunResult Engine::run(int64_t source) {
  DBFS_CHECK(source >= 0 && source < part_.n, "source vertex out of range");
  DBFS_CHECK(!opt_.directed || (opt_.mode != Mode::BottomUp && opt_.mode != Mode::DirOpt),
             "directed graphs need a top-down mode (bottom-up searches in-edges)");
  RunResult r;
  const bool ref = opt_.mode == Mode::Ref || opt_.mode == Mode::Scan;
  run_narrow_ = !ref && use_narrow();
  // (padded to whole bitmap words: a direct top-down update reads a word's
  // 64 level bytes; padding vertices are pre-set visited, so masked)
  const size_t l8_bytes = static_cast<size_t>(std::max<int64_t>(part_.slice_words() * kWordBits, 1));
  bool fresh = false;
  if (run_narrow_ && level8_.size() == 0) {
    level8_ = DBuf<uint8_t>(be_, l8_bytes);
    fresh = true;
  }
  level8_filled_ = false;
  narrow_base_ = 0;
  if (run_narrow_) {
    // Level bytes are stored as base + level with base cycling through
    // kNarrowEpochs values: the previous epochs' bytes (and the 0xFF fill)
    // lie outside this run's [base, base + kNarrowMaxLevel], so they already
    // read as unreached and only epoch 0 pays for the fill.
    if (fresh) narrow_run_ = 0;
    const int epoch = static_cast<int>(narrow_run_++ % kNarrowEpochs);
    narrow_base_ = static_cast<uint8_t>(epoch * (kNarrowMaxLevel + 2));
    level8_filled_ = epoch != 0;
  }
  r = ref ? run_ref(source) : (use_device_loop() ? run_bitmap_device(source) : run_bitmap(source));
  check_device();
  levels_narrow_ = run_narrow_;
  if (run_narrow_ && r.depth - 1 > kNarrowMaxLevel) {
    // deeper than the narrow levels hold (identical decision on every rank):
    // rerun with 32-bit levels; the reported time includes both traversals
    narrow_failed_ = true;
    run_narrow_ = levels_narrow_ = false;
    const double first_ms = r.ms;
    r = use_device_loop() ? run_bitmap_device(source) : run_bitmap(source);
    check_device();
    r.ms += first_ms;
  }
  if (ref || opt_.directed) {
    ensure_wide_levels();
    // Traversed-edge accounting outside the timed region (the bitmap engine
    // otherwise knows sum(deg) of every level's new vertices): Graph500's
    // undirected convention, or all out-edges of reached vertices (directed).
    DBuf<int64_t> acc(be_, 2);
    be_.reached_degree_sum(g_.view(), level_.data(), acc.data());
    comm_.allreduce_sum_i64(acc.data(), 2);
    int64_t h[2];
    be_.to_host(h, acc.data(), sizeof(h));
    r.reached = h[0];
    r.edges = opt_.directed ? h[1] : h[1] / 2;
  }
  r.gteps = r.ms > 0 ? static_cast<double>(r.edges) / (r.ms * 1e6) : 0.0;
  return r;
}

bool Engine::use_narrow() const {
  return opt_.narrow_levels && !narrow_failed_ &&
         (opt_.mode == Mode::TopDown || opt_.mode == Mode::BottomUp || opt_.mode == Mode::DirOpt);
}

// The last run's levels into level_ (32-bit) if it kept them narrow.
void Engine::ensure_wide_levels() const {
  if (!levels_narrow_) return;
  be_.widen_levels(level8_.data(), level_.data(), g_.rows(), narrow_base_);
  levels_narrow_ = false;
}

// Scratch bitmaps every consumer leaves zeroed (`next` bits cleared by the
// consuming update or re-zeroed after the exchange, the byte map by its
// gather, `cand` by its update): only a run that ended early (an error,
// injected fault) leaves them dirty, and then they are cleared here.
void Engine::begin_run_scratch() {
  if (scratch_dirty_) {
    be_.memset_async(cand_.data(), 0, cand_.bytes());
    be_.memset_async(next_.data(), 0, next_.bytes());
    if (next_bytes_.data()) be_.memset_async(next_bytes_.data(), 0, next_bytes_.bytes());
    if (td_hub_mark_.data()) be_.memset_async(td_hub_mark_.data(), 0, td_hub_mark_.bytes());
    if (td_group_ticket_.data()) be_.memset_async(td_group_ticket_.data(), 0, td_group_ticket_.bytes());
  }
  scratch_dirty_ = true;  // until the run completes
}

InitRunArgs Engine::init_args(int64_t source, word_t* seed_frontier, LevelCtrl* ctrl, const LevelCtrl& ctrl_init,
                              LevelMailbox* mailbox) {
  const int me = comm_.rank();
  InitRunArgs ia;
  ia.g = g_.view();
  ia.level = level_.data();
  ia.level8 = run_narrow_ ? level8_.data() : nullptr;
  ia.level8_filled = level8_filled_;
  ia.narrow_base = narrow_base_;
  ia.zdeg = zdeg_.data();
  ia.visited = visited_.data();
  ia.gwords = part_.global_words();
  ia.frontier = seed_frontier;
  ia.words = part_.slice_words();
  ia.src_local = part_.owner(source) == me ? source - g_.lo() : -1;
  ia.vis_word_base = static_cast<int64_t>(me) * part_.slice_words();
  ia.unit_cnt = unit_cnt_.data();
  ia.unit_deg = unit_deg_.data();
  ia.part_cnt = part_cnt_.data();
  ia.part_deg = part_deg_.data();
  ia.stats = stats_.data();
  ia.qscan = qscan_.data();
  ia.ctrl = ctrl;
  ia.ctrl_init = ctrl_init;
  ia.mailbox = mailbox;
  return ia;
}

RunResult Engine::run_bitmap(int64_t source) {
  alloc_bitmap_state();
  TraceRange trace_run(std::string("bfs.run mode=") + mode_name(opt_.mode) + " src=" + std::to_string(source));
  const int P = part_.nranks;
  const int me = comm_.rank();
  const int64_t W = part_.slice_words(), GW = part_.global_words();
  const int64_t lo = g_.lo();
  const ShardView gv = g_.view();
  word_t* vis_own = visited_.data() + me * W;
  // Frontier double buffer: `cur` is the frontier being expanded (global after
  // the all-gather), `nxt` receives the next one (bottom-up reads `cur` while
  // it writes `nxt`, so they must differ).
  int cur = 0;
  auto fr_cur = [&]() { return frontier_[cur].data(); };
  auto fr_nxt_own = [&]() { return frontier_[cur ^ 1].data() + me * W; };

  RunResult res;
  res.source = source;
  be_.reset_events();
  comm_.barrier();
  const auto t0 = std::chrono::steady_clock::now();

  // ---- init (inside the timed window): one fused pass, seed totals included ----
  begin_run_scratch();
  be_.init_run(init_args(source, frontier_[1].data() + me * W, nullptr, LevelCtrl(), nullptr));

  // Collectives of the current level, bracketed by events when phase timing is
  // on (LevelRecord::comm_ms).
  std::vector<std::pair<int, int>> comm_evs;
  auto timed_comm = [&](auto&& fn) {
    if (!opt_.phase_timing) {
      fn();
      return;
    }
    const int a = be_.record_event();
    fn();
    comm_evs.emplace_back(a, be_.record_event());
  };
  // Scan the unit statistics of the new frontier and reduce the totals to the
  // host (termination + direction decision).
  auto finish_level = [&](int64_t* host_stats) {
    ScanArgs sa;
    sa.unit_cnt = unit_cnt_.data();
    sa.unit_deg = unit_deg_.data();
    sa.nunits = nunits_;
    sa.part_cnt = part_cnt_.data();
    sa.part_deg = part_deg_.data();
    sa.ticket = ticket_.data();
    sa.stats = stats_.data();
    sa.qscan = qscan_.data();
    be_.scan_units(sa);
    cur ^= 1;
    if (exchange()) timed_comm([&] { comm_.allreduce_sum_i64(stats_.data() + 2, 2); });
    read_level_stats(host_stats);
  };
  // Publish the new frontier (all-gather of the owned slices) and merge it into
  // the replicated visited bitmap.  Bottom-up needs the global frontier; a
  // top-down level only reads its owned slice, and a stale remote `visited`
  // only lets some already-visited candidates through to their owners (which
  // filter them), so the direction-optimising engine skips the all-gather
  // before a top-down level.
  auto publish = [&](char next_dir) {
    if (!exchange() || (next_dir == 'T' && opt_.mode == Mode::DirOpt)) return;
    timed_comm([&] { comm_.allgather(fr_cur() + me * W, fr_cur(), static_cast<size_t>(W) * sizeof(word_t)); });
    be_.bitmap_or(visited_.data(), fr_cur(), GW);
  };
  auto update = [&](word_t* cand, int nchunks, bool clear, bool force, lvl_t new_level,
                    uint8_t* cand_bytes = nullptr) {
    UpdateArgs ua;
    ua.g = gv;
    ua.cand = cand;
    ua.cand_bytes = cand_bytes;
    ua.nchunks = nchunks;
    ua.cand_stride = W;
    ua.clear_cand = clear;
    ua.force = force;
    ua.visited = vis_own;
    ua.frontier = fr_nxt_own();
    ua.level = level_.data();
    ua.level8 = run_narrow_ ? level8_.data() : nullptr;
    ua.narrow_base = narrow_base_;
    ua.new_level = new_level;
    ua.words = W;
    ua.unit_cnt = unit_cnt_.data();
    ua.unit_deg = unit_deg_.data();
    be_.update_frontier(ua);
  };

  int64_t hs[4];
  // Seed totals (written by init_run; the source counts with degree > 0 only).
  cur ^= 1;
  if (exchange()) timed_comm([&] { comm_.allreduce_sum_i64(stats_.data() + 2, 2); });
  read_level_stats(hs);
  int64_t q_local = hs[0], m_local = hs[1], n_f = hs[2], m_f = hs[3];
  int64_t vis_deg = m_f;
  int64_t prev_nf = 0;

  char dir;
  switch (opt_.mode) {
    case Mode::BottomUp: dir = 'B'; break;
    case Mode::Simple: dir = 'S'; break;
    default: dir = 'T'; break;
  }
  const double n_d = static_cast<double>(part_.n);
  // Beamer's switch, evaluated on global totals (identical on every rank).
  auto decide = [&]() {
    if (opt_.mode != Mode::DirOpt) return;
    const double m_u = static_cast<double>(total_directed_ - vis_deg);
    // T -> B only while the frontier grows: in the tail m_u is just the edges
    // of unreachable components, and m_u / alpha would flip tiny frontiers to a
    // full bottom-up sweep.
    if (dir == 'T' && static_cast<double>(m_f) > m_u / opt_.alpha && n_f > prev_nf) {
      dir = 'B';
    } else if (dir == 'B' && static_cast<double>(n_f) < n_d / opt_.beta && n_f < prev_nf) {
      dir = 'T';
    }
  };
  decide();
  // A level's timing starts before the all-gather that publishes its frontier.
  int next_ev0 = -1;
  auto begin_next = [&]() {
    comm_evs.clear();
    if (opt_.phase_timing) next_ev0 = be_.record_event();
    publish(dir);
  };
  if (n_f > 0) begin_next();
  lvl_t L = 0;
  while (n_f > 0) {
    inject_fault(L);
    const int ev0 = opt_.phase_timing ? (next_ev0 >= 0 ? next_ev0 : be_.record_event()) : -1;
    next_ev0 = -1;
    char trace_name[48];
    std::snprintf(trace_name, sizeof(trace_name), "bfs.level %d %c", L, dir);
    TraceRange trace_level(trace_name);
    bool bytes_mode = false;
    // Sparse exchange: every rank sends at most m_f (global frontier edges)
    // candidates to any peer, so owner lists of capacity m_f cannot overflow;
    // used when they are smaller than half a bitmap slice.
    const bool list_mode =
        exchange() && dir == 'T' && m_f <= opt_.sparse_max_edges &&
        (!opt_.sparse_size_check ||
         (m_f + 1) * static_cast<int64_t>(sizeof(vid_t)) * 2 <= W * static_cast<int64_t>(sizeof(word_t)));
    const int64_t list_cap = m_f;
    if (list_mode) {
      if (send_lists_.size() < static_cast<size_t>(P) * (list_cap + 1)) {
        // grow geometrically (bounded by the option) so a run allocates O(1) times
        const int64_t per = std::min(opt_.sparse_max_edges, std::max<int64_t>(2 * list_cap, 4096));
        const size_t cap = static_cast<size_t>(P) * static_cast<size_t>(std::max(per, list_cap) + 1);
        send_lists_ = DBuf<vid_t>(be_, cap);
        recv_lists_ = DBuf<vid_t>(be_, cap);
      }
      be_.memset_async(send_lists_.data(), 0, static_cast<size_t>(P) * (list_cap + 1) * sizeof(vid_t));
    }
    if (dir == 'T' || dir == 'S') {
      // `next` is all-zero here: cleared at init and by every consuming update
      // (P == 1), or re-zeroed right after the exchange below (P > 1).
      if (dir == 'T') {
        if (q_local > 0) {
          CompactArgs ca;
          ca.g = gv;
          ca.frontier = fr_cur() + me * W;
          ca.words = W;
          ca.unit_cnt_off = unit_cnt_.data();
          ca.unit_deg_off = unit_deg_.data();
          ca.part_cnt = part_cnt_.data();
          ca.part_deg = part_deg_.data();
          ca.qscan = qscan_.data();
          ca.qbase = qbase_.data();
          ca.blk_vstart = blk_vstart_.data();
          be_.compact_frontier(ca);
          TdArgs ta;
          ta.g = gv;
          ta.qscan = qscan_.data();
          ta.qbase = qbase_.data();
          ta.blk_vstart = blk_vstart_.data();
          ta.q = q_local;
          ta.m = m_local;
          ta.visited = visited_.data();
          ta.next = next_.data();
          if (list_mode) {
            ta.lists = send_lists_.data();
            ta.list_cap = list_cap;
            ta.part = part_.part;
          } else if (m_local >= opt_.td_byte_edges) {
            if (!next_bytes_.data()) {
              next_bytes_ = DBuf<uint8_t>(be_, static_cast<size_t>(GW) * kWordBits);
              be_.memset_async(next_bytes_.data(), 0, next_bytes_.bytes());
            }
            ta.next_bytes = next_bytes_.data();
            ta.check_visited = static_cast<double>(vis_deg) >= opt_.td_check_visited_min * static_cast<double>(total_directed_);
            bytes_mode = true;
          }
          ta.wide_below_blocks = opt_.td_wide_below_blocks;
          be_.td_expand(ta);
        }
      } else {
        StatusArgs sa;
        sa.g = gv;
        sa.level = level_.data();
        sa.cur = L;
        sa.visited = visited_.data();
        sa.next = next_.data();
        be_.status_expand(sa);
      }
      if (list_mode) {
        timed_comm([&] {
          comm_.alltoall(send_lists_.data(), recv_lists_.data(), static_cast<size_t>(list_cap + 1) * sizeof(vid_t));
        });
        ListScatterArgs la;
        la.lists = recv_lists_.data();
        la.nranks = P;
        la.list_cap = list_cap;
        la.lo = lo;
        la.cand = cand_.data();
        la.words = part_.slice_words();
        be_.list_scatter(la);
        update(cand_.data(), 1, true, false, L + 1);
      } else if (exchange()) {
        if (bytes_mode) {
          PackArgs pa;
          pa.bytes = next_bytes_.data();
          pa.next = next_.data();
          pa.words = GW;
          be_.pack_bytes(pa);
        }
        timed_comm([&] { comm_.alltoall(next_.data(), recv_.data(), static_cast<size_t>(W) * sizeof(word_t)); });
        be_.memset_async(next_.data(), 0, next_.bytes());
        update(recv_.data(), P, false, false, L + 1);
      } else if (bytes_mode) {
        update(nullptr, 1, false, false, L + 1, next_bytes_.data());
      } else {
        update(next_.data(), 1, true, false, L + 1);
      }
    } else {
      BuArgs ba;
      ba.g = gv;
      ba.visited = vis_own;
      ba.frontier = fr_cur();
      ba.new_frontier = fr_nxt_own();
      ba.level = level_.data();
      ba.level8 = run_narrow_ ? level8_.data() : nullptr;
      ba.narrow_base = narrow_base_;
      ba.new_level = L + 1;
      ba.words = W;
      ba.lane_limit = opt_.bu_lane_limit;
      ba.whole_units = opt_.bu_whole_units;
      ba.small_waves = opt_.bu_small_waves;
      ba.zdeg = zdeg_.data() + comm_.rank() * W;
      ba.follow_up = !res.levels.empty() && res.levels.back().direction == 'B';
      ba.unit_cnt = unit_cnt_.data();
      ba.unit_deg = unit_deg_.data();
      if (gv.nhubs > 0) {
        HubGatherArgs hg;
        hg.g = gv;
        hg.frontier = fr_cur();
        hg.hub_front = hub_front_.data();
        be_.hub_gather(hg);
        ba.hub_front = hub_front_.data();
      }
      be_.bu_step(ba);
    }
    finish_level(hs);
    LevelRecord rec;
    rec.level = L;
    rec.direction = dir;
    rec.frontier = n_f;
    rec.frontier_edges = m_f;
    rec.discovered = hs[2];
    if (opt_.phase_timing) {
      const int ev1 = be_.record_event();
      rec.ms = be_.elapsed_ms(ev0, ev1);
      for (const auto& ce : comm_evs) rec.comm_ms += be_.elapsed_ms(ce.first, ce.second);
    }
    res.levels.push_back(rec);
    prev_nf = n_f;
    q_local = hs[0];
    m_local = hs[1];
    n_f = hs[2];
    m_f = hs[3];
    vis_deg += m_f;
    ++L;
    if (n_f > 0) {
      decide();
      begin_next();
    }
  }
  be_.synchronize();
  const auto t1 = std::chrono::steady_clock::now();
  scratch_dirty_ = false;
  const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  res.ms = comm_.max_host(ms);
  res.depth = res.levels.empty() ? 1 : static_cast<int>(res.levels.size());
  res.edges = vis_deg / 2;
  res.reached = 1;
  for (const auto& l : res.levels) res.reached += l.discovered;
  return res;
}

// Sparse top-down levels (device loop): the packed output counter holds
// 64 - kSparseEdgeBits bits of entries and kSparseEdgeBits of edges.
bool Engine::sparse_enabled() const {
  return opt_.td_sparse_edges > 0 && opt_.mode != Mode::BottomUp && g_.rows() < (int64_t(1) << (64 - kSparseEdgeBits)) &&
         g_.nnz() < (int64_t(1) << kSparseEdgeBits);
}

LevelRecDev* Engine::rec_at(int level) {
  const size_t seg = static_cast<size_t>(level / kRecSeg);
  while (rec_segs_.size() <= seg) {
    void* dptr = nullptr;
    auto* h = static_cast<LevelRecDev*>(be_.alloc_mapped(sizeof(LevelRecDev) * kRecSeg, &dptr));
    rec_segs_.emplace_back(h, static_cast<LevelRecDev*>(dptr));
  }
  return rec_segs_[seg].second + level % kRecSeg;
}

bool Engine::use_device_loop() const {
  return opt_.device_loop &&
         (opt_.mode == Mode::TopDown || opt_.mode == Mode::BottomUp || opt_.mode == Mode::DirOpt);
}

RunResult Engine::run_ref(int64_t source) {
  alloc_ref_state();
  const int P = part_.nranks;
  const int me = comm_.rank();
  const int64_t cap = part_.part;
  const ShardView gv = g_.view();
  RunResult res;
  res.source = source;
  be_.reset_events();
  comm_.barrier();
  const auto t0 = std::chrono::steady_clock::now();

  // initializeCudaBfs2 (bfs.cu:402-422): distance = INT_MAX everywhere, 0 at the
  // source on every rank; the source is queued on its owner only.
  be_.fill_level(dist_.data(), part_.n, kUnreached);
  be_.fill_level(dist_.data() + source, 1, 0);
  int64_t q = 0;
  if (part_.owner(source) == me) {
    const vid_t s = static_cast<vid_t>(source);
    be_.to_device(queue_.data(), &s, sizeof(s));
    q = 1;
  }
  int64_t total_q = 1;
  lvl_t L = 0;
  std::vector<int64_t> hcnt(static_cast<size_t>(P)), hrc(static_cast<size_t>(P)), sd(static_cast<size_t>(P)),
      rd(static_cast<size_t>(P)), hbuf(static_cast<size_t>(3 * P + 1));
  const bool scan = opt_.mode == Mode::Scan;
  while (total_q > 0) {
    inject_fault(L);
    const int ev0 = opt_.phase_timing ? be_.record_event() : -1;
    if (scan) {
      // relax -> count -> scan -> bounds -> assign: children land owner-major in
      // buckets_, bucket o at [bounds[o], bounds[o + 1])
      ScanBfsArgs sa;
      sa.g = gv;
      sa.queue = queue_.data();
      sa.q = q;
      sa.next_level = L + 1;
      sa.dist = dist_.data();
      sa.claim = claim_.data();
      sa.part = part_.part;
      sa.nranks = P;
      sa.offs = scan_offs_.data();
      sa.counts = bucket_cnt_.data();
      sa.bounds = bucket_cnt_.data() + 2 * P;
      sa.out = buckets_.data();
      be_.scan_relax(sa);
      be_.scan_count(sa);
      be_.exclusive_scan(sa.offs, P * q);
      be_.scan_bounds(sa);
      be_.scan_assign(sa);
      be_.to_host(hbuf.data(), bucket_cnt_.data(), hbuf.size() * sizeof(int64_t));
      for (int r = 0; r < P; ++r) {
        hcnt[r] = hbuf[r];
        sd[r] = hbuf[2 * P + r];
      }
    } else {
      be_.memset_async(bucket_cnt_.data(), 0, static_cast<size_t>(P) * sizeof(int64_t));
      RefExpandArgs ea;
      ea.g = gv;
      ea.queue = queue_.data();
      ea.q = q;
      ea.next_level = L + 1;
      ea.dist = dist_.data();
      ea.part = part_.part;
      ea.bucket_cnt = bucket_cnt_.data();
      ea.buckets = buckets_.data();
      ea.bucket_cap = cap;
      be_.ref_expand(ea);
      be_.to_host(hcnt.data(), bucket_cnt_.data(), static_cast<size_t>(P) * sizeof(int64_t));
      for (int r = 0; r < P; ++r) sd[r] = r * cap;
    }
    if (!exchange()) {
      if (scan) {
        std::swap(queue_, buckets_);  // P == 1: both hold cap entries
      } else {
        be_.copy_async(queue_.data(), buckets_.data(), static_cast<size_t>(hcnt[0]) * sizeof(vid_t));
      }
      q = hcnt[0];
    } else {
      // count exchange (the reference reads the peers' managed counters)
      comm_.alltoall(bucket_cnt_.data(), bucket_cnt_.data() + P, sizeof(int64_t));
      be_.to_host(hrc.data(), bucket_cnt_.data() + P, static_cast<size_t>(P) * sizeof(int64_t));
      int64_t tot = 0;
      for (int r = 0; r < P; ++r) {
        rd[r] = tot;
        tot += hrc[r];
      }
      comm_.alltoallv(buckets_.data(), hcnt.data(), sd.data(), recvq_.data(), hrc.data(), rd.data(), sizeof(vid_t));
      be_.memset_async(qcount_.data(), 0, sizeof(int64_t));
      RefAcceptArgs aa;
      aa.recv = recvq_.data();
      aa.total = tot;
      aa.self_begin = rd[me];
      aa.self_end = rd[me] + hrc[me];
      aa.next_level = L + 1;
      aa.dist = dist_.data();
      aa.queue = queue_.data();
      aa.qcount = qcount_.data();
      be_.ref_accept(aa);
      be_.to_host(&q, qcount_.data(), sizeof(int64_t));
    }
    LevelRecord rec;
    rec.level = L;
    rec.direction = scan ? 'C' : 'R';
    rec.frontier = total_q;
    total_q = exchange() ? comm_.sum_host(q) : q;
    rec.discovered = total_q;
    if (opt_.phase_timing) {
      const int ev1 = be_.record_event();
      rec.ms = be_.elapsed_ms(ev0, ev1);
    }
    res.levels.push_back(rec);
    ++L;
  }
  // Owned slice of the replicated distances is authoritative.
  be_.copy_async(level_.data(), dist_.data() + g_.lo(), static_cast<size_t>(g_.rows()) * sizeof(lvl_t));
  be_.synchronize();
  const auto t1 = std::chrono::steady_clock::now();
  res.ms = comm_.max_host(std::chrono::duration<double, std::milli>(t1 - t0).count());
  res.depth = static_cast<int>(res.levels.size());
  return res;
}

std::vector<lvl_t> Engine::levels_local() const {
  ensure_wide_levels();
  std::vector<lvl_t> h(static_cast<size_t>(g_.rows()));
  if (!h.empty()) be_.to_host(h.data(), level_.data(), h.size() * sizeof(lvl_t));
  return h;
}

std::vector<lvl_t> Engine::gather_levels() {
  ensure_wide_levels();
  const int P = part_.nranks;
  const int64_t part = part_.part;
  DBuf<lvl_t> send(be_, static_cast<size_t>(part)), recv(be_, static_cast<size_t>(P * part));
  be_.fill_level(send.data(), part, kUnreached);
  be_.copy_async(send.data(), level_.data(), static_cast<size_t>(g_.rows()) * sizeof(lvl_t));
  comm_.allgather(send.data(), recv.data(), static_cast<size_t>(part) * sizeof(lvl_t));
  std::vector<lvl_t> h(static_cast<size_t>(P * part));
  be_.to_host(h.data(), recv.data(), h.size() * sizeof(lvl_t));
  h.resize(static_cast<size_t>(part_.n));
  return h;
}

void Engine::gather_levels_device(DBuf<lvl_t>& full) {
  ensure_wide_levels();
  const int P = part_.nranks;
  const int64_t part = part_.part;
  DBuf<lvl_t> send(be_, static_cast<size_t>(part));
  full = DBuf<lvl_t>(be_, static_cast<size_t>(P * part));
  be_.fill_level(send.data(), part, kUnreached);
  be_.copy_async(send.data(), level_.data(), static_cast<size_t>(g_.rows()) * sizeof(lvl_t));
  comm_.allgather(send.data(), full.data(), static_cast<size_t>(part) * sizeof(lvl_t));
}

std::vector<int64_t> Engine::parents_local(int64_t source) {
  DBuf<lvl_t> full;
  gather_levels_device(full);
  DBuf<int64_t> par(be_, static_cast<size_t>(std::max<int64_t>(g_.rows(), 1)));
  ParentArgs pa;
  pa.g = g_.view();
  pa.level_global = full.data();
  pa.src = source;
  pa.parent = par.data();
  be_.compute_parents(pa);
  std::vector<int64_t> h(static_cast<size_t>(g_.rows()));
  if (!h.empty()) be_.to_host(h.data(), par.data(), h.size() * sizeof(int64_t));
  else be_.synchronize();
  return h;
}

std::vector<int64_t> Engine::gather_parents(int64_t source) {
  const int P = part_.nranks;
  const int64_t part = part_.part;
  std::vector<int64_t> mine = parents_local(source);
  mine.resize(static_cast<size_t>(part), -1);
  DBuf<int64_t> send(be_, static_cast<size_t>(part)), recv(be_, static_cast<size_t>(P * part));
  be_.to_device(send.data(), mine.data(), mine.size() * sizeof(int64_t));
  comm_.allgather(send.data(), recv.data(), static_cast<size_t>(part) * sizeof(int64_t));
  std::vector<int64_t> h(static_cast<size_t>(P * part));
  be_.to_host(h.data(), recv.data(), h.size() * sizeof(int64_t));
  h.resize(static_cast<size_t>(part_.n));
  return h;
}

std::vector<int64_t> Engine::validate(int64_t source) {
  DBuf<lvl_t> full;
  gather_levels_device(full);
  DBuf<int64_t> out(be_, 3);
  be_.memset_async(out.data(), 0, out.bytes());
  ValidateArgs va;
  va.g = g_.view();
  va.level_global = full.data();
  va.src = source;
  va.out = out.data();
  be_.validate_levels(va);
  comm_.allreduce_sum_i64(out.data(), 3);
  std::vector<int64_t> h(3);
  be_.to_host(h.data(), out.data(), 3 * sizeof(int64_t));
  return h;
}

}  // namespace dbfs
