// RCCL communicator: the per-level exchange over xGMI.
//
// Reference call sites replaced: per-pair synchronous
// cudaMemcpyPeer (bfs.cu:595-609) and CUDA-aware MPI_Sendrecv / MPI_Allreduce
// (bfs_mpi.cu:614-621).  Every collective here is enqueued on the owning
// backend's HIP stream, so it is ordered after the expansion kernels without a
// host synchronisation.  On MI355X each GPU has 7 direct xGMI links, one per
// peer: all-to-all and all-gather drive all of them at once, which is why the
// engine exchanges equal-sized bitmap slices (ncclAllToAll / ncclAllGather)
// instead of ring all-reduces.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "dbfs/comm.hpp"

namespace dbfs {

#define NCCL_CHECK(expr)                                                                         \
  do {                                                                                           \
    ncclResult_t r_ = (expr);                                                                    \
    if (r_ != ncclSuccess)                                                                       \
      ::dbfs::raise_error(__FILE__, __LINE__,                                                    \
                          std::string("RCCL error ") + ncclGetErrorString(r_) + " in " #expr);   \
  } while (0)

#define HIP_CHECK(expr)                                                                          \
  do {                                                                                           \
    hipError_t e_ = (expr);                                                                      \
    if (e_ != hipSuccess)                                                                        \
      ::dbfs::raise_error(__FILE__, __LINE__, std::string("HIP error ") + hipGetErrorString(e_)); \
  } while (0)

// Calls on the (nonblocking) communicator: ncclInProgress settled by polling.
#define NCCL_Q(expr) settle(static_cast<int>(expr), #expr, __FILE__, __LINE__)

namespace {
inline ncclComm_t C(void* p) { return static_cast<ncclComm_t>(p); }
// Poll a nonblocking communicator until its pending operation is no longer
// in progress (or `limit` seconds pass: ncclInProgress returned).
ncclResult_t poll_comm(ncclComm_t c, double limit) {
  const auto t0 = std::chrono::steady_clock::now();
  for (int spin = 0;; ++spin) {
    ncclResult_t st = ncclSuccess;
    ncclCommGetAsyncError(c, &st);
    if (st != ncclInProgress) return st;
    if (limit > 0 && std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit)
      return ncclInProgress;
    if (spin > 1000) std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
}
double init_timeout_s() {
  const char* e = std::getenv("DBFS_RCCL_INIT_TIMEOUT_S");
  return e && *e ? std::max(0.0, std::atof(e)) : 60.0;
}
// collectives go to the backend's communication stream (the compute stream
// unless the engine opened a side region: Backend::fork_side)
inline hipStream_t S(Backend* be) { return static_cast<hipStream_t>(be->comm_stream_handle()); }
}  // namespace

std::string NcclComm::unique_id() {
  ncclUniqueId id;
  NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

NcclComm::NcclComm(const std::string& uid, int rank, int nranks, Backend& be) : rank_(rank), size_(nranks) {
  DBFS_CHECK(be.kind() == DeviceKind::HIP, "NcclComm requires a HIP backend");
  DBFS_CHECK(uid.size() == NCCL_UNIQUE_ID_BYTES, "bad RCCL unique id size");
  bind_backend(&be);
  HIP_CHECK(hipSetDevice(be.device_id()));
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
  // (DBFS_FAULT_INJECT="kind=rccl_init": tests of the setups that must not
  // depend on RCCL -- the peer transport runs on a TCP inner communicator)
  if (const char* f = std::getenv("DBFS_FAULT_INJECT"))
    DBFS_CHECK(std::string(f).find("kind=rccl_init") == std::string::npos, "injected fault (rccl_init)");
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclComm_t c = nullptr;
  const ncclResult_t r0 = ncclCommInitRankConfig(&c, nranks, id, rank, &cfg);
  if (r0 != ncclSuccess && r0 != ncclInProgress) {
    if (c) ncclCommAbort(c);
    NCCL_CHECK(r0);
  }
  const double limit = init_timeout_s();
  const ncclResult_t st = c ? poll_comm(c, limit) : ncclInternalError;
  if (st != ncclSuccess) {
    if (c) ncclCommAbort(c);
    DBFS_CHECK(st != ncclInProgress, "RCCL communicator setup did not complete within " +
                                         std::to_string(static_cast<int>(limit)) + " s on rank " +
                                         std::to_string(rank) + " (DBFS_RCCL_INIT_TIMEOUT_S)");
    NCCL_CHECK(st);
  }
  comm_ = c;
  install_watchdog();
}

void NcclComm::settle(int result, const char* what, const char* file, int line) {
  ncclResult_t r = static_cast<ncclResult_t>(result);
  if (r == ncclInProgress && comm_) r = poll_comm(C(comm_), 0.0);
  if (r != ncclSuccess) raise_error(file, line, std::string("RCCL error ") + ncclGetErrorString(r) + " in " + what);
}

// Failure detection: while the host waits on the stream, poll
// ncclCommGetAsyncError and bound the wait by comm_timeout_s(); on either, the
// communicator is aborted (ncclCommAbort releases the stuck kernels) and the
// wait throws, so a dead or hung peer ends the run with an error.
void NcclComm::install_watchdog() {
  const double limit = comm_timeout_s();
  be_->set_wait_watch([this, limit](double waited) {
    if (!comm_) return;
    ncclResult_t st = ncclSuccess;
    ncclCommGetAsyncError(C(comm_), &st);
    std::string why;
    if (st != ncclSuccess && st != ncclInProgress) why = std::string("RCCL async error: ") + ncclGetErrorString(st);
    else if (limit > 0 && waited > limit)
      why = "RCCL collective did not complete within " + std::to_string(limit) + " s (DBFS_COMM_TIMEOUT_S)";
    if (why.empty()) return;
    ncclCommAbort(C(comm_));
    comm_ = nullptr;
    throw Error(why + " on rank " + std::to_string(rank_));
  });
}

// One process, one communicator per backend (the reference's one process
// driving every GPU, bfs.cu:328-332): ncclCommInitAll's work as a group of
// nonblocking per-rank inits, so its setup is bounded like the multi-process
// one (DBFS_RCCL_INIT_TIMEOUT_S): a setup that cannot complete -- RCCL
// refusing two ranks on one device, a fabric problem -- aborts every
// communicator and fails instead of hanging the process.
std::vector<std::unique_ptr<NcclComm>> NcclComm::init_all(const std::vector<Backend*>& bes) {
  const int n = static_cast<int>(bes.size());
  for (int i = 0; i < n; ++i) DBFS_CHECK(bes[i]->kind() == DeviceKind::HIP, "NcclComm requires HIP backends");
  if (const char* f = std::getenv("DBFS_FAULT_INJECT"))
    DBFS_CHECK(std::string(f).find("kind=rccl_init") == std::string::npos, "injected fault (rccl_init)");
  ncclUniqueId id;
  NCCL_CHECK(ncclGetUniqueId(&id));
  std::vector<ncclComm_t> comms(static_cast<size_t>(n), nullptr);
  auto abort_all = [&] {
    for (auto& c : comms)
      if (c) ncclCommAbort(c);
  };
  ncclResult_t r0 = ncclGroupStart();
  for (int i = 0; i < n && (r0 == ncclSuccess || r0 == ncclInProgress); ++i) {
    HIP_CHECK(hipSetDevice(bes[i]->device_id()));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    r0 = ncclCommInitRankConfig(&comms[static_cast<size_t>(i)], n, id, i, &cfg);
  }
  const ncclResult_t r1 = ncclGroupEnd();
  if ((r0 != ncclSuccess && r0 != ncclInProgress) || (r1 != ncclSuccess && r1 != ncclInProgress)) {
    abort_all();
    NCCL_CHECK(r0 != ncclSuccess && r0 != ncclInProgress ? r0 : r1);
  }
  const double limit = init_timeout_s();
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) {
    const double left =
        limit > 0 ? std::max(0.001, limit - std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count())
                  : 0.0;
    const ncclResult_t st = comms[static_cast<size_t>(i)] ? poll_comm(comms[static_cast<size_t>(i)], left)
                                                          : ncclInternalError;
    if (st != ncclSuccess) {
      abort_all();
      DBFS_CHECK(st != ncclInProgress, "RCCL in-process setup (" + std::to_string(n) +
                                           " communicators) did not complete within " +
                                           std::to_string(static_cast<int>(limit)) + " s (DBFS_RCCL_INIT_TIMEOUT_S)");
      NCCL_CHECK(st);
    }
  }
  std::vector<std::unique_ptr<NcclComm>> out;
  for (int i = 0; i < n; ++i) {
    std::unique_ptr<NcclComm> c(new NcclComm());
    c->comm_ = comms[static_cast<size_t>(i)];
    c->rank_ = i;
    c->size_ = n;
    c->bind_backend(bes[i]);
    c->install_watchdog();
    out.push_back(std::move(c));
  }
  return out;
}

NcclComm::~NcclComm() {
  if (be_) be_->set_wait_watch(nullptr);
  if (comm_) ncclCommDestroy(C(comm_));
}

void NcclComm::check_alive() const {
  DBFS_CHECK(comm_ != nullptr, "RCCL communicator was aborted after a failure");
}

void NcclComm::alltoall(const void* send, void* recv, size_t bytes) {
  note(kAllToAll, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(bytes));
  check_alive();
  HIP_CHECK(hipSetDevice(be_->device_id()));
  NCCL_Q(ncclAllToAll(send, recv, bytes, ncclChar, C(comm_), S(be_)));
}

void NcclComm::allgather(const void* send, void* recv, size_t bytes) {
  note(kAllGather, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(bytes));
  check_alive();
  HIP_CHECK(hipSetDevice(be_->device_id()));
  NCCL_Q(ncclAllGather(send, recv, bytes, ncclChar, C(comm_), S(be_)));
}

void NcclComm::allreduce_sum_i64(int64_t* buf, size_t count) {
  note(kAllReduce, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(count) * 8);
  check_alive();
  HIP_CHECK(hipSetDevice(be_->device_id()));
  NCCL_Q(ncclAllReduce(buf, buf, count, ncclInt64, ncclSum, C(comm_), S(be_)));
}

void NcclComm::alltoallv(const void* send, const int64_t* sc, const int64_t* sd, void* recv, const int64_t* rc,
                         const int64_t* rd, size_t eb) {
  note_alltoallv(sc, eb);
  check_alive();
  HIP_CHECK(hipSetDevice(be_->device_id()));
  NCCL_Q(ncclGroupStart());
  for (int r = 0; r < size_; ++r) {
    if (sc[r] > 0)
      NCCL_Q(ncclSend(static_cast<const char*>(send) + sd[r] * eb, static_cast<size_t>(sc[r]) * eb, ncclChar, r,
                          C(comm_), S(be_)));
    if (rc[r] > 0)
      NCCL_Q(ncclRecv(static_cast<char*>(recv) + rd[r] * eb, static_cast<size_t>(rc[r]) * eb, ncclChar, r,
                          C(comm_), S(be_)));
  }
  NCCL_Q(ncclGroupEnd());
}

void NcclComm::group_start() { NCCL_Q(ncclGroupStart()); }
void NcclComm::group_end() { NCCL_Q(ncclGroupEnd()); }

void NcclComm::barrier() {
  note(kBarrier, 0);
  int64_t* b = scratch(1);
  allreduce_sum_i64(b, 1);  // value irrelevant: completion on every rank is the barrier
  be_->synchronize();
}

}  // namespace dbfs
