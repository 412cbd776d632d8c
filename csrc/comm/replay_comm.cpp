// Record / replay communicators: one rank of a P-rank job measured alone on
// one GPU ("shadow rank").
//
// RecordComm wraps rank r's communicator in a real P-rank run (virtual ranks
// on one GPU, or processes) and keeps every collective's OUTPUT on the host,
// in call order: what the other ranks contributed, as this rank saw it.
// ReplayComm then stands in for the whole job with rank r running alone: each
// collective checks that it is the next recorded one (kind and sizes) and
// writes the recorded output with one stream-ordered device copy.  Rank r's
// kernels therefore see exactly the inputs they saw in the P-rank run (remote
// frontier slices, candidates, all-reduced totals -- the traversal is
// deterministic given them), but own the whole GPU: their times are the
// per-rank compute of a P-GPU job, which no single-GPU box can otherwise
// measure.  The per-device step of the reference being replaced is the
// launch-per-device + synchronize of bfs.cu:577-591 / bfs_mpi.cu:586-593.
#include <algorithm>
#include <climits>
#include <cstring>

#include "dbfs/comm.hpp"

namespace dbfs {

namespace {
const char* kind_name(int k) {
  switch (k) {
    case Comm::kAllToAll: return "alltoall";
    case Comm::kAllGather: return "allgather";
    case Comm::kAllReduce: return "allreduce";
    case Comm::kAllToAllV: return "alltoallv";
    case Comm::kBarrier: return "barrier";
    case CommTape::kLists: return "alltoall_lists";
  }
  return "?";
}
}  // namespace

int64_t CommTape::bytes() const {
  int64_t b = 0;
  for (const auto& r : recs) b += static_cast<int64_t>(r.data.size());
  return b;
}

// ---- RecordComm -------------------------------------------------------------

RecordComm::RecordComm(std::shared_ptr<Comm> inner) : inner_(std::move(inner)), tape_(std::make_shared<CommTape>()) {
  DBFS_CHECK(inner_ != nullptr, "RecordComm needs an inner communicator");
  tape_->rank = inner_->rank();
  tape_->size = inner_->size();
  tape_->counted_lists = inner_->counted_lists();
}

void RecordComm::push(int kind, int64_t a, int64_t b, const void* dev, size_t bytes) {
  CommTape::Rec r;
  r.kind = kind;
  r.a = a;
  r.b = b;
  r.data.resize(bytes);
  if (bytes) be_->to_host(&r.data[0], dev, bytes);  // (blocking: after the collective)
  tape_->recs.push_back(std::move(r));
}

void RecordComm::alltoall(const void* send, void* recv, size_t bytes) {
  note(kAllToAll, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(bytes));
  inner_->alltoall(send, recv, bytes);
  push(kAllToAll, static_cast<int64_t>(bytes), 0, recv, bytes * static_cast<size_t>(size()));
}

void RecordComm::allgather(const void* send, void* recv, size_t bytes) {
  note(kAllGather, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(bytes));
  inner_->allgather(send, recv, bytes);
  push(kAllGather, static_cast<int64_t>(bytes), 0, recv, bytes * static_cast<size_t>(size()));
}

void RecordComm::allreduce_sum_i64(int64_t* buf, size_t count) {
  note(kAllReduce, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(count) * 8);
  inner_->allreduce_sum_i64(buf, count);
  push(kAllReduce, static_cast<int64_t>(count), 0, buf, count * sizeof(int64_t));
}

void RecordComm::alltoallv(const void* send, const int64_t* sc, const int64_t* sd, void* recv, const int64_t* rc,
                           const int64_t* rd, size_t eb) {
  note_alltoallv(sc, eb);
  inner_->alltoallv(send, sc, sd, recv, rc, rd, eb);
  int64_t tot = 0, lo = INT64_MAX, hi = 0;
  bool ordered = true;
  for (int p = 0; p < size(); ++p) {
    tot += rc[p];
    if (rc[p] <= 0) continue;
    if (rd[p] < hi) ordered = false;
    lo = std::min(lo, rd[p]);
    hi = std::max(hi, rd[p] + rc[p]);
  }
  CommTape::Rec r;
  r.kind = kAllToAllV;
  r.a = tot;
  r.b = static_cast<int64_t>(eb);
  if (tot > 0 && ordered && hi - lo <= 2 * tot) {
    // pieces in rank order with small gaps (owner lists at a fixed stride):
    // the whole span, replayed as ONE copy (a gap is unused receive space)
    r.span = lo * static_cast<int64_t>(eb);
    r.data.resize(static_cast<size_t>(hi - lo) * eb);
    be_->to_host(&r.data[0], static_cast<const char*>(recv) + r.span, r.data.size());
  } else {
    // the received pieces in rank order, concatenated
    r.data.resize(static_cast<size_t>(tot) * eb);
    size_t off = 0;
    for (int p = 0; p < size(); ++p) {
      const size_t n = static_cast<size_t>(rc[p]) * eb;
      if (n) be_->to_host(&r.data[off], static_cast<const char*>(recv) + rd[p] * eb, n);
      r.pieces.push_back(static_cast<int64_t>(n));
      off += n;
    }
  }
  tape_->recs.push_back(std::move(r));
}

void RecordComm::alltoall_lists(const uint32_t* send, uint32_t* recv, size_t stride, size_t cap) {
  note(kAllToAllV, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(cap + 1) * 4);
  inner_->alltoall_lists(send, recv, stride, cap);
  // every received list's count word and entries (count-sized), replayed as
  // one multi-piece copy
  CommTape::Rec r;
  r.kind = CommTape::kLists;
  r.a = static_cast<int64_t>(stride);
  r.b = static_cast<int64_t>(cap);
  for (int p = 0; p < size(); ++p) {
    const uint32_t* list = recv + static_cast<size_t>(p) * stride;
    uint32_t n = 0;
    be_->to_host(&n, list, sizeof(n));
    const size_t bytes = (static_cast<size_t>(n) + 1) * sizeof(uint32_t);
    const size_t off = r.data.size();
    r.data.resize(off + bytes);
    be_->to_host(&r.data[off], list, bytes);
    r.pieces.push_back(static_cast<int64_t>(bytes));
  }
  tape_->recs.push_back(std::move(r));
}

void RecordComm::barrier() {
  note(kBarrier, 0);
  inner_->barrier();
  push(kBarrier, 0, 0, nullptr, 0);
}

double RecordComm::max_host(double x) { return inner_->max_host(x); }  // (timing only: not recorded)

// ---- ReplayComm -------------------------------------------------------------

ReplayComm::ReplayComm(std::shared_ptr<CommTape> tape, Backend& be) : tape_(std::move(tape)) {
  DBFS_CHECK(tape_ != nullptr, "ReplayComm needs a tape");
  bind_backend(&be);
  // every recorded output in one device buffer: a replayed collective is then
  // a device-to-device copy on the stream (no host round trip, no pinned
  // staging that would stall the enqueue-ahead level loop)
  const int64_t total = tape_->bytes();
  dev_ = DBuf<char>(be, static_cast<size_t>(std::max<int64_t>(total, 16)));
  off_.reserve(tape_->recs.size());
  int64_t off = 0;
  for (const auto& r : tape_->recs) {
    off_.push_back(off);
    if (!r.data.empty()) be.to_device(dev_.data() + off, r.data.data(), r.data.size());
    off += static_cast<int64_t>(r.data.size());
  }
  // direct exchanges (DirectExchange, sequence number 1): each recorded list
  // exchange as a table whose sources are the recorded lists in dev_ and
  // whose incoming cells hold their counts; outgoing data and cells go to a
  // sink (what this rank sends is not replayed anywhere); the level ends'
  // table has cells that have arrived (the kernel takes the recorded sums)
  if (be.kind() == DeviceKind::HIP && tape_->size <= kMaxDirectRanks) {
    int64_t cap_max = 0, nlists = 0;
    for (const auto& r : tape_->recs)
      if (r.kind == CommTape::kLists && static_cast<int>(r.pieces.size()) == tape_->size) {
        cap_max = std::max(cap_max, r.b);
        ++nlists;
      }
    // [sink for ids / cells][cells: one 16-B cell per rank and list record,
    // then the level ends' arrived cells]
    const int64_t sink_b = (std::max<int64_t>((cap_max + 1) * 4, 64 * 16) + 15) / 16 * 16;
    const int64_t ncells = (nlists + 1) * kMaxDirectRanks;
    dscratch_ = DBuf<char>(be, static_cast<size_t>(sink_b + ncells * 16));
    char* scr = dscratch_.data();
    uint64_t* cells = reinterpret_cast<uint64_t*>(scr + sink_b);
    std::vector<uint64_t> hcells(static_cast<size_t>(ncells * 2), 0);
    std::vector<DirectTable> tabs;
    auto sink_table = [&](DirectTable& t) {
      std::memset(&t, 0, sizeof(t));
      for (int p = 0; p < tape_->size; ++p) {
        t.dst[p] = reinterpret_cast<uint32_t*>(scr);
        t.cell_out[p] = reinterpret_cast<uint64_t*>(scr) + 2 * p;
      }
    };
    for (size_t i = 0; i < tape_->recs.size(); ++i) {
      const auto& r = tape_->recs[i];
      if (r.kind != CommTape::kLists || static_cast<int>(r.pieces.size()) != tape_->size) continue;
      DirectTable t;
      sink_table(t);
      const int64_t c0 = static_cast<int64_t>(tabs.size()) * kMaxDirectRanks;
      int64_t o = off_[i];
      size_t ho = 0;
      for (int p = 0; p < tape_->size; ++p) {
        uint32_t n = 0;
        std::memcpy(&n, r.data.data() + ho, sizeof(n));
        t.src[p] = reinterpret_cast<const uint32_t*>(dev_.data() + o);
        t.cell_in[p] = cells + 2 * (c0 + p);
        hcells[static_cast<size_t>(2 * (c0 + p))] = (uint64_t(1) << 32) | n;
        o += r.pieces[p];
        ho += static_cast<size_t>(r.pieces[p]);
      }
      dtab_index_[i] = static_cast<int64_t>(tabs.size());
      tabs.push_back(t);
    }
    DirectTable t;
    sink_table(t);
    const int64_t c0 = static_cast<int64_t>(tabs.size()) * kMaxDirectRanks;
    for (int p = 0; p < tape_->size; ++p) {
      t.src[p] = reinterpret_cast<const uint32_t*>(scr);
      t.cell_in[p] = cells + 2 * (c0 + p);
      hcells[static_cast<size_t>(2 * (c0 + p))] = uint64_t(1) << 32;
      hcells[static_cast<size_t>(2 * (c0 + p) + 1)] = uint64_t(1) << 40;
    }
    dtab_sink_ = static_cast<int64_t>(tabs.size());
    tabs.push_back(t);
    be.to_device(cells, hcells.data(), hcells.size() * sizeof(uint64_t));
    dtab_ = DBuf<char>(be, tabs.size() * sizeof(DirectTable));
    be.to_device(dtab_.data(), tabs.data(), tabs.size() * sizeof(DirectTable));
  }
}

bool ReplayComm::direct_level_end(size_t count, DirectExchange* x) {
  if (dtab_sink_ < 0 || pos_ >= tape_->recs.size()) return false;
  const auto& r = tape_->recs[pos_];
  if (r.kind != kAllReduce || r.a != static_cast<int64_t>(count)) return false;
  note(kAllReduce, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(count) * 8);
  x->active = 1;
  x->nranks = size();
  x->rank = rank();
  x->seq = 1;  // (every flag reads ~0)
  x->table = reinterpret_cast<const DirectTable*>(dtab_.data()) + dtab_sink_;
  x->timeout_ticks = ~uint64_t(0) >> 1;
  x->error = reinterpret_cast<uint64_t*>(dscratch_.data());
  x->result = reinterpret_cast<const int64_t*>(dev_.data() + off_[pos_]);  // the recorded sums
  ++pos_;
  return true;
}

bool ReplayComm::direct_lists(size_t cap, DirectExchange* x) {
  if (pos_ >= tape_->recs.size()) return false;
  const auto& r = tape_->recs[pos_];
  const auto it = dtab_index_.find(pos_);
  if (r.kind != CommTape::kLists || r.b != static_cast<int64_t>(cap) || it == dtab_index_.end()) return false;
  note(kAllToAllV, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(cap + 1) * 4);
  x->active = 1;
  x->nranks = size();
  x->rank = rank();
  x->seq = 1;  // (every flag reads ~0)
  x->table = reinterpret_cast<const DirectTable*>(dtab_.data()) + it->second;
  x->timeout_ticks = ~uint64_t(0) >> 1;
  x->error = reinterpret_cast<uint64_t*>(dscratch_.data());  // (never written: no wait times out)
  ++pos_;
  return true;
}

const CommTape::Rec& ReplayComm::next(int kind, int64_t a, int64_t b, size_t* idx) {
  DBFS_CHECK(pos_ < tape_->recs.size(), std::string("ReplayComm: tape exhausted at a ") + kind_name(kind) +
                                            " (the replayed rank issued more collectives than it recorded)");
  const auto& r = tape_->recs[pos_];
  if (r.kind != kind || r.a != a || r.b != b)
    throw Error("ReplayComm: collective " + std::to_string(pos_) + " is a " + kind_name(kind) + "(" + std::to_string(a) +
                ", " + std::to_string(b) + ") but the tape has a " + kind_name(r.kind) + "(" + std::to_string(r.a) +
                ", " + std::to_string(r.b) + ")");
  *idx = pos_++;
  return r;
}

void ReplayComm::alltoall(const void*, void* recv, size_t bytes) {
  note(kAllToAll, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(bytes));
  size_t i = 0;
  const auto& r = next(kAllToAll, static_cast<int64_t>(bytes), 0, &i);
  be_->copy_async(recv, dev_.data() + off_[i], r.data.size());
}

void ReplayComm::allgather(const void*, void* recv, size_t bytes) {
  note(kAllGather, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(bytes));
  size_t i = 0;
  const auto& r = next(kAllGather, static_cast<int64_t>(bytes), 0, &i);
  be_->copy_async(recv, dev_.data() + off_[i], r.data.size());
}

void ReplayComm::allreduce_sum_i64(int64_t* buf, size_t count) {
  note(kAllReduce, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(count) * 8);
  size_t i = 0;
  const auto& r = next(kAllReduce, static_cast<int64_t>(count), 0, &i);
  be_->copy_async(buf, dev_.data() + off_[i], r.data.size());
}

void ReplayComm::alltoallv(const void*, const int64_t* sc, const int64_t*, void* recv, const int64_t* rc,
                           const int64_t* rd, size_t eb) {
  note_alltoallv(sc, eb);
  int64_t tot = 0;
  for (int p = 0; p < size(); ++p) tot += rc[p];
  size_t i = 0;
  const auto& r = next(kAllToAllV, tot, static_cast<int64_t>(eb), &i);
  if (r.span >= 0) {
    be_->copy_async(static_cast<char*>(recv) + r.span, dev_.data() + off_[i], r.data.size());
    return;
  }
  int64_t off = off_[i];
  const bool words = eb % 4 == 0 && size() <= Backend::CopyPieces::kMax;
  Backend::CopyPieces cp;
  for (int p = 0; p < size(); ++p) {
    const size_t n = static_cast<size_t>(rc[p]) * eb;
    if (n && words) {
      cp.dst[cp.n] = static_cast<char*>(recv) + rd[p] * eb;
      cp.src[cp.n] = dev_.data() + off;
      cp.bytes[cp.n++] = static_cast<int64_t>(n);
    } else if (n) {
      be_->copy_async(static_cast<char*>(recv) + rd[p] * eb, dev_.data() + off, n);
    }
    off += static_cast<int64_t>(n);
  }
  if (cp.n) be_->copy_pieces(cp);
}

void ReplayComm::alltoall_lists(const uint32_t*, uint32_t* recv, size_t stride, size_t cap) {
  note(kAllToAllV, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(cap + 1) * 4);
  size_t i = 0;
  const auto& r = next(CommTape::kLists, static_cast<int64_t>(stride), static_cast<int64_t>(cap), &i);
  DBFS_CHECK(static_cast<int>(r.pieces.size()) == size() && size() <= Backend::CopyPieces::kMax,
             "ReplayComm: malformed list record");
  // one launch: every list at its stride, count-sized
  Backend::CopyPieces cp;
  int64_t off = off_[i];
  for (int p = 0; p < size(); ++p) {
    cp.dst[cp.n] = recv + static_cast<size_t>(p) * stride;
    cp.src[cp.n] = dev_.data() + off;
    cp.bytes[cp.n++] = r.pieces[p];
    off += r.pieces[p];
  }
  be_->copy_pieces(cp);
}

void ReplayComm::level_end(const void*, void* grecv, size_t gbytes, int64_t* buf, size_t count,
                           const LevelFinishArgs& fin) {
  Backend::CopyPieces cp;
  size_t i = 0;
  if (gbytes > 0) {
    note(kAllGather, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(gbytes));
    const auto& r = next(kAllGather, static_cast<int64_t>(gbytes), 0, &i);
    cp.dst[cp.n] = grecv;
    cp.src[cp.n] = dev_.data() + off_[i];
    cp.bytes[cp.n++] = static_cast<int64_t>(r.data.size());
  }
  note(kAllReduce, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(count) * 8);
  const auto& r = next(kAllReduce, static_cast<int64_t>(count), 0, &i);
  cp.dst[cp.n] = buf;
  cp.src[cp.n] = dev_.data() + off_[i];
  cp.bytes[cp.n++] = static_cast<int64_t>(r.data.size());
  be_->copy_pieces(cp);
  be_->level_finish(fin);
}

void ReplayComm::barrier() {
  note(kBarrier, 0);
  size_t i = 0;
  next(kBarrier, 0, 0, &i);
  be_->synchronize();
}

}  // namespace dbfs
