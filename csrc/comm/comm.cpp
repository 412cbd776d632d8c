// LocalComm, VirtualComm and the host-value helpers shared by every Comm.
//
// VirtualComm runs P ranks as threads of one process on any backend: the
// partitioned engine (shards, owner routing, bitmap exchange) is then testable
// on a single GPU or on the CPU, which the reference cannot do (its multi-GPU
// path needs >= 2 real GPUs with peer access).
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <vector>

#include "dbfs/comm.hpp"

namespace dbfs {

double comm_timeout_s() {
  const char* e = std::getenv("DBFS_COMM_TIMEOUT_S");
  // (a peer minutes late is dead: the default bounds a hung job at two
  // minutes per collective wait; the device-side waits give up after at most
  // 60 s of it)
  if (!e || !*e) return 120.0;
  return std::max(0.0, std::atof(e));
}

double bootstrap_timeout_s() {
  const char* e = std::getenv("DBFS_BOOTSTRAP_TIMEOUT_S");
  if (!e || !*e) return 600.0;
  return std::max(0.0, std::atof(e));
}

int64_t* Comm::scratch(size_t n) {
  DBFS_CHECK(be_ != nullptr, "comm has no backend bound");
  if (scratch_.size() < n) scratch_ = DBuf<int64_t>(*be_, std::max<size_t>(n, 64));
  return scratch_.data();
}

int64_t Comm::sum_host(int64_t x) {
  int64_t* b = scratch(1);
  be_->to_device(b, &x, sizeof(x));
  allreduce_sum_i64(b, 1);
  be_->to_host(&x, b, sizeof(x));
  return x;
}

double Comm::max_host(double x) {
  const int n = size();
  int64_t* b = scratch(static_cast<size_t>(n) + 1);
  be_->to_device(b, &x, sizeof(x));
  allgather(b, b + 1, sizeof(double));
  std::vector<double> h(static_cast<size_t>(n));
  be_->to_host(h.data(), b + 1, h.size() * sizeof(double));
  return *std::max_element(h.begin(), h.end());
}

std::vector<int64_t> Comm::allgather_host_i64(int64_t x) {
  const int n = size();
  int64_t* b = scratch(static_cast<size_t>(n) + 1);
  be_->to_device(b, &x, sizeof(x));
  allgather(b, b + 1, sizeof(int64_t));
  std::vector<int64_t> h(static_cast<size_t>(n));
  be_->to_host(h.data(), b + 1, h.size() * sizeof(int64_t));
  return h;
}

void Comm::alltoall_lists(const uint32_t* send, uint32_t* recv, size_t stride_words, size_t cap) {
  const int P = size();
  DBFS_CHECK(stride_words >= cap + 1, "alltoall_lists: stride below the list capacity");
  std::vector<int64_t> cnt(static_cast<size_t>(P), static_cast<int64_t>(cap + 1)), off(static_cast<size_t>(P));
  for (int p = 0; p < P; ++p) off[p] = static_cast<int64_t>(p) * static_cast<int64_t>(stride_words);
  alltoallv(send, cnt.data(), off.data(), recv, cnt.data(), off.data(), sizeof(uint32_t));
}

void Comm::allgather_allreduce(const void* send, void* recv, size_t bytes, int64_t* buf, size_t count) {
  group_start();
  allgather(send, recv, bytes);
  allreduce_sum_i64(buf, count);
  group_end();
  if (groups()) note_fused();
}

void Comm::level_end(const void* gsend, void* grecv, size_t gbytes, int64_t* buf, size_t count,
                     const LevelFinishArgs& fin) {
  if (gbytes > 0) allgather_allreduce(gsend, grecv, gbytes, buf, count);
  else allreduce_sum_i64(buf, count);
  be_->level_finish(fin);
}

// ---- LocalComm ----------------------------------------------------------------

void LocalComm::alltoall(const void* send, void* recv, size_t bytes) {
  if (send != recv) be_->copy_async(recv, send, bytes);
}
void LocalComm::allgather(const void* send, void* recv, size_t bytes) {
  if (send != recv) be_->copy_async(recv, send, bytes);
}
void LocalComm::alltoallv(const void* send, const int64_t* sc, const int64_t* sd, void* recv, const int64_t* rc,
                          const int64_t* rd, size_t eb) {
  DBFS_CHECK(sc[0] == rc[0], "LocalComm alltoallv count mismatch");
  be_->copy_async(static_cast<char*>(recv) + rd[0] * eb, static_cast<const char*>(send) + sd[0] * eb,
                  static_cast<size_t>(sc[0]) * eb);
}
void LocalComm::barrier() { be_->synchronize(); }

// ---- VirtualGroup / VirtualComm -----------------------------------------------

VirtualGroup::VirtualGroup(int nranks) : n_(nranks), slots_(static_cast<size_t>(nranks)) {
  DBFS_CHECK(nranks >= 1, "virtual group needs >= 1 rank");
}

void VirtualGroup::barrier() {
  std::unique_lock<std::mutex> lk(mu_);
  if (aborted_) throw Error("virtual rank group aborted: " + reason_);
  const uint64_t gen = generation_;
  if (++arrived_ == n_) {
    arrived_ = 0;
    ++generation_;
    cv_.notify_all();
    return;
  }
  auto done = [&] { return generation_ != gen || aborted_; };
  const double limit = comm_timeout_s();
  if (limit > 0) {
    if (!cv_.wait_for(lk, std::chrono::duration<double>(limit), done)) {
      aborted_ = true;
      reason_ = "barrier timed out after " + std::to_string(limit) + " s (a rank stopped participating)";
      cv_.notify_all();
    }
  } else {
    cv_.wait(lk, done);
  }
  if (generation_ == gen) throw Error("virtual rank group aborted: " + reason_);
}

void VirtualGroup::abort(const std::string& reason) {
  std::lock_guard<std::mutex> lk(mu_);
  if (!aborted_) {
    aborted_ = true;
    reason_ = reason;
  }
  cv_.notify_all();
}

bool VirtualGroup::aborted() const {
  std::lock_guard<std::mutex> lk(mu_);
  return aborted_;
}

GroupBootstrap::GroupBootstrap(std::shared_ptr<VirtualGroup> g, int rank) : g_(std::move(g)), rank_(rank) {
  DBFS_CHECK(g_ && rank >= 0 && rank < g_->size(), "group bootstrap: rank out of range");
}

std::vector<std::string> GroupBootstrap::allgather(const std::string& data) {
  // (the group's slots are shared with its VirtualComms: every rank makes the
  // same sequence of group calls, each ending in a barrier after the reads)
  auto& sl = g_->slots();
  sl[rank_].send = &data;
  g_->barrier();
  std::vector<std::string> out(static_cast<size_t>(size()));
  for (int r = 0; r < size(); ++r) out[r] = *static_cast<const std::string*>(sl[r].send);
  g_->barrier();
  return out;
}

std::string GroupBootstrap::broadcast(const std::string& data, int root) { return allgather(data)[root]; }

VirtualComm::VirtualComm(std::shared_ptr<VirtualGroup> g, int rank, Backend& be) : g_(std::move(g)), rank_(rank) {
  DBFS_CHECK(rank >= 0 && rank < g_->size(), "virtual rank out of range");
  bind_backend(&be);
}

void VirtualComm::alltoall(const void* send, void* recv, size_t bytes) {
  note(kAllToAll, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(bytes));
  be_->synchronize();
  auto& sl = g_->slots();
  sl[rank_].send = send;
  sl[rank_].be = be_;
  g_->barrier();
  for (int r = 0; r < size(); ++r)
    be_->copy_async(static_cast<char*>(recv) + r * bytes, static_cast<const char*>(sl[r].send) + rank_ * bytes, bytes);
  be_->synchronize();
  g_->barrier();
}

void VirtualComm::allgather(const void* send, void* recv, size_t bytes) {
  note(kAllGather, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(bytes));
  be_->synchronize();
  auto& sl = g_->slots();
  sl[rank_].send = send;
  g_->barrier();
  for (int r = 0; r < size(); ++r)
    be_->copy_async(static_cast<char*>(recv) + r * bytes, sl[r].send, bytes);
  be_->synchronize();
  g_->barrier();
}

void VirtualComm::allreduce_sum_i64(int64_t* buf, size_t count) {
  note(kAllReduce, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(count) * 8);
  be_->synchronize();
  auto& sl = g_->slots();
  sl[rank_].send = buf;
  g_->barrier();
  // wrapping (two's-complement) sums, as RCCL's (see TcpComm::allreduce_sum_i64)
  std::vector<uint64_t> acc(count, 0), tmp(count);
  for (int r = 0; r < size(); ++r) {
    be_->to_host(tmp.data(), sl[r].send, count * sizeof(int64_t));
    for (size_t i = 0; i < count; ++i) acc[i] += tmp[i];
  }
  g_->barrier();
  be_->to_device(buf, acc.data(), count * sizeof(int64_t));
  g_->barrier();
}

void VirtualComm::alltoallv(const void* send, const int64_t* sc, const int64_t* sd, void* recv, const int64_t* rc,
                            const int64_t* rd, size_t eb) {
  note_alltoallv(sc, eb);
  be_->synchronize();
  auto& sl = g_->slots();
  sl[rank_].send = send;
  sl[rank_].counts = sc;
  sl[rank_].displs = sd;
  g_->barrier();
  for (int r = 0; r < size(); ++r) {
    const int64_t n = sl[r].counts[rank_];
    DBFS_CHECK(n == rc[r], "VirtualComm alltoallv count mismatch");
    be_->copy_async(static_cast<char*>(recv) + rd[r] * eb,
                    static_cast<const char*>(sl[r].send) + sl[r].displs[rank_] * eb, static_cast<size_t>(n) * eb);
  }
  be_->synchronize();
  g_->barrier();
}

void VirtualComm::alltoall_lists(const uint32_t* send, uint32_t* recv, size_t stride, size_t cap) {
  note(kAllToAllV, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(cap + 1) * 4);
  be_->synchronize();
  auto& sl = g_->slots();
  sl[rank_].send = send;
  g_->barrier();
  for (int r = 0; r < size(); ++r) {
    const uint32_t* src = static_cast<const uint32_t*>(sl[r].send) + static_cast<size_t>(rank_) * stride;
    uint32_t n = 0;
    be_->to_host(&n, src, sizeof(n));
    DBFS_CHECK(n <= cap, "VirtualComm alltoall_lists: a list exceeds its capacity");
    be_->copy_async(recv + static_cast<size_t>(r) * stride, src, (static_cast<size_t>(n) + 1) * sizeof(uint32_t));
  }
  be_->synchronize();
  g_->barrier();
}

void VirtualComm::barrier() {
  note(kBarrier, 0);
  be_->synchronize();
  g_->barrier();
}

}  // namespace dbfs
