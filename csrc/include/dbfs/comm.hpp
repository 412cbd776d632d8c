// Communicator interface for the per-level frontier exchange.
//
// Replaces the reference's communication call sites:
//   X5 / M4  serialized cudaMemcpyPeer / MPI_Sendrecv of owner buckets
//            -> alltoall of equal-sized bitmap slices (bitmap engine) or
//               alltoallv of owner-routed vertex ids (reference mode)
//   X6 / M7  host sum / MPI_Allreduce for termination -> allreduce_sum_i64
//   X8 / M8  host min-merge of replicated distances -> not needed (owner
//            partitioned levels); allgather for gathering results
//   M2       MPI_Barrier -> barrier
//
// Implementations:
//   LocalComm    single rank (P = 1): copies only.
//   NcclComm     RCCL over xGMI, collectives enqueued on the backend's HIP
//                stream; one communicator per GPU (one process per GPU, or one
//                thread per GPU inside a process via ncclCommInitAll).
//   VirtualComm  P ranks as threads of one process on any backend (used to test
//                the partitioned engine on one GPU or on the CPU).
//   PyComm       (bindings) forwards to Python -- torch.distributed / gloo.
#pragma once

#include <condition_variable>
#include <functional>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "dbfs/backend.hpp"

namespace dbfs {

// Failure detection: a collective that waits longer than this
// for its peers fails with an error instead of hanging.  DBFS_COMM_TIMEOUT_S,
// default 120 s; 0 disables the limit.
double comm_timeout_s();
// The host bootstrap's socket timeout (TcpBootstrap, and TcpComm over it):
// DBFS_BOOTSTRAP_TIMEOUT_S, default 600 s (setup exchanges wait for every
// rank's ingest and CSR build); 0 disables it.
double bootstrap_timeout_s();

class Comm {
 public:
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual std::string name() const = 0;

  // All buffers live in backend memory; operations are ordered after earlier
  // work on the backend stream.
  // recv[r * bytes ... ] = send of rank r at offset rank() * bytes.
  virtual void alltoall(const void* send, void* recv, size_t bytes_per_peer) = 0;
  // recv[r * bytes ...] = send of rank r.
  virtual void allgather(const void* send, void* recv, size_t bytes_per_peer) = 0;
  virtual void allreduce_sum_i64(int64_t* buf, size_t count) = 0;
  // Variable-size exchange; counts/displacements in elements, host arrays.
  virtual void alltoallv(const void* send, const int64_t* send_counts, const int64_t* send_displs,
                         void* recv, const int64_t* recv_counts, const int64_t* recv_displs,
                         size_t elem_bytes) = 0;
  virtual void barrier() = 0;
  // Collectives issued between group_start/group_end may be fused into one
  // launch (ncclGroupStart/End); other communicators execute them in order.
  virtual void group_start() {}
  virtual void group_end() {}
  // group_start/group_end really fuse the collectives between them
  virtual bool groups() const { return false; }

  // Owner lists whose lengths live on the device (no host round trip): rank
  // r's list for peer p is the 32-bit words at send + p * stride_words -- word
  // 0 its length n <= cap, then n entries -- and lands at recv + r *
  // stride_words on peer p, length first.  The peer transport ships each
  // list's n + 1 words, sized on the device (count-sized, as the reference's
  // nextQueueSize-sized peer copies, bfs.cu:595-609 / bfs_mpi.cu:615-618);
  // the default ships cap + 1 words per peer (an all-to-all-v of uniform
  // counts).  The transport's choice may depend only on (stride, cap).
  virtual void alltoall_lists(const uint32_t* send, uint32_t* recv, size_t stride_words, size_t cap);
  // alltoall_lists ships each list's own length (else the capacity): the
  // engine then sizes its lists generously, otherwise by the prediction
  virtual bool counted_lists() const { return false; }
  // allgather(send, recv, bytes) and allreduce_sum_i64(buf, count) as ONE
  // collective where the transport can (peer windows: one launch, both
  // payloads in one slot; RCCL: one group); in order otherwise.
  virtual void allgather_allreduce(const void* send, void* recv, size_t bytes, int64_t* buf, size_t count);
  // The next owner-list exchange (alltoall_lists of `cap` ids per peer) done
  // by the kernels themselves (DirectExchange: producer stores into the peers'
  // windows, consumer waits for their flags): fills `x` and returns true, or
  // false when this transport cannot (the caller uses alltoall_lists).  The
  // choice depends only on `cap` (the same on every rank).
  virtual bool direct_lists(size_t cap, DirectExchange* x) {
    (void)cap;
    (void)x;
    return false;
  }
  // The next level end without a frontier gather -- level_end(nullptr,
  // nullptr, 0, buf, count, fin) -- done by the last workgroup of the level's
  // last kernel (DirectExchange: push the totals to every peer's window, wait
  // for theirs, sum, decide): fills `x` and returns true, or false (the caller
  // uses level_end).  The choice depends only on `count`.
  virtual bool direct_level_end(size_t count, DirectExchange* x) {
    (void)count;
    (void)x;
    return false;
  }
  // The frontier slices of `words` words each pushed by the producing kernels
  // themselves into the peers' windows (FrontierTable, buffer `parity`):
  // the device table, or nullptr when this transport cannot (the caller
  // all-gathers them with the level end).  The choice depends only on
  // `words` (the same on every rank).
  virtual const FrontierTable* direct_frontier(size_t words, int parity) {
    (void)words;
    (void)parity;
    return nullptr;
  }
  // A level's end on several ranks: its totals all-reduced (buf, count) --
  // with gbytes > 0 also its output frontier slice all-gathered (gsend ->
  // grecv) -- then the device continuation `fin`, the level's decision on the
  // reduced totals (Backend::level_finish).  The peer transport runs all of
  // it as ONE launch; the default is allgather_allreduce + level_finish.
  virtual void level_end(const void* gsend, void* grecv, size_t gbytes, int64_t* buf, size_t count,
                         const LevelFinishArgs& fin);

  // Host-value helpers built on the device collectives.
  virtual int64_t sum_host(int64_t x);
  virtual double max_host(double x);
  // Every rank's x, indexed by rank (one device all-gather).
  virtual std::vector<int64_t> allgather_host_i64(int64_t x);
  void bind_backend(Backend* be) {
    if (be != be_) scratch_.reset();
    be_ = be;
  }

  // Traffic of this rank since reset_traffic(): calls per collective and the
  // bytes this rank sends to the other ranks under a direct exchange --
  // alltoall / allgather (P - 1) x the per-peer bytes, all-reduce (P - 1) x
  // the vector, alltoallv the counts to other ranks; barriers count calls.
  // (docs/ARCHITECTURE.md §4 models these per level; tests check the model.)
  enum TrafficKind { kAllToAll = 0, kAllGather, kAllReduce, kAllToAllV, kBarrier, kTrafficKinds };
  struct Traffic {
    int64_t calls[kTrafficKinds] = {};
    int64_t bytes[kTrafficKinds] = {};
    // collectives that shared another's launch (allgather_allreduce): the
    // launches issued are sum(calls) - fused
    int64_t fused = 0;
  };
  const Traffic& traffic() const { return traffic_; }
  void reset_traffic() { traffic_ = Traffic{}; }

  // The level whose chain the engine is enqueueing (-1: none): a transport
  // names it when a collective of that chain fails or times out.
  void set_level_tag(int level) { level_tag_ = level; }
  // Ranks sharing a GPU (peer transport): a kernel that waits for a peer
  // must not spin in every workgroup of a large grid -- a co-resident rank's
  // producer may need those CUs -- so the waits run as one-wave launches
  // first (Backend::direct_prewait) and the collectives unfused.
  virtual bool split_waits() const { return false; }
  // Ranks of this communicator on this rank's GPU, itself included (peer
  // transport; 1 elsewhere): with the in-kernel waits (no split_waits) the
  // engine and the transport size every grid whose workgroups all spin on a
  // peer so the co-resident ranks' grids together leave the chip room for
  // the producers they wait for.
  virtual int coresident() const { return 1; }

 protected:
  int level_tag_ = -1;
  void note(TrafficKind k, int64_t bytes) {
    ++traffic_.calls[k];
    traffic_.bytes[k] += bytes;
  }
  void note_fused() { ++traffic_.fused; }
  void note_alltoallv(const int64_t* sc, size_t eb) {
    int64_t b = 0;
    for (int p = 0; p < size(); ++p)
      if (p != rank()) b += sc[p] * static_cast<int64_t>(eb);
    note(kAllToAllV, b);
  }
  Traffic traffic_;
  // Small persistent device scratch for the host-value helpers and barriers
  // (no hipMalloc/hipFree -- which synchronise the device -- per call).
  int64_t* scratch(size_t n_int64);
  Backend* be_ = nullptr;
  DBuf<int64_t> scratch_;
};

class LocalComm final : public Comm {
 public:
  explicit LocalComm(Backend& be) { bind_backend(&be); }
  int rank() const override { return 0; }
  int size() const override { return 1; }
  std::string name() const override { return "local"; }
  void alltoall(const void* send, void* recv, size_t bytes) override;
  void allgather(const void* send, void* recv, size_t bytes) override;
  void allreduce_sum_i64(int64_t*, size_t) override {}
  void alltoallv(const void* send, const int64_t* sc, const int64_t* sd, void* recv,
                 const int64_t* rc, const int64_t* rd, size_t eb) override;
  void barrier() override;
  int64_t sum_host(int64_t x) override { return x; }
  double max_host(double x) override { return x; }
  std::vector<int64_t> allgather_host_i64(int64_t x) override { return {x}; }
};

// Shared state of a group of virtual ranks living in one process.
class VirtualGroup {
 public:
  explicit VirtualGroup(int nranks);
  int size() const { return n_; }
  // Throws if the group was aborted (a rank failed) or the wait exceeds
  // comm_timeout_s().
  void barrier();
  // Mark the group failed and wake every waiting rank (they throw).
  void abort(const std::string& reason);
  bool aborted() const;
  struct Slot {
    const void* send = nullptr;
    void* recv = nullptr;
    const int64_t* counts = nullptr;
    const int64_t* displs = nullptr;
    Backend* be = nullptr;
  };
  std::vector<Slot>& slots() { return slots_; }
  std::vector<double>& scratch() { return scratch_; }

 private:
  int n_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  int arrived_ = 0;
  uint64_t generation_ = 0;
  bool aborted_ = false;
  std::string reason_;
  std::vector<Slot> slots_;
  std::vector<double> scratch_;
};

class VirtualComm final : public Comm {
 public:
  VirtualComm(std::shared_ptr<VirtualGroup> g, int rank, Backend& be);
  int rank() const override { return rank_; }
  int size() const override { return g_->size(); }
  std::string name() const override { return "virtual"; }
  void alltoall(const void* send, void* recv, size_t bytes) override;
  void allgather(const void* send, void* recv, size_t bytes) override;
  void allreduce_sum_i64(int64_t* buf, size_t count) override;
  void alltoallv(const void* send, const int64_t* sc, const int64_t* sd, void* recv,
                 const int64_t* rc, const int64_t* rd, size_t eb) override;
  void barrier() override;
  // count-sized, as the peer transport (so virtual ranks -- and the shadow
  // rank's recording -- take the peer transport's schedule)
  void alltoall_lists(const uint32_t* send, uint32_t* recv, size_t stride_words, size_t cap) override;
  bool counted_lists() const override { return true; }

 private:
  std::shared_ptr<VirtualGroup> g_;
  int rank_;
};

// Host-side rank group for setup exchanges (IPC handles, RCCL unique ids,
// agreed verdicts): TCP between processes (TcpBootstrap) or threads of one
// process (GroupBootstrap).
class Bootstrap {
 public:
  virtual ~Bootstrap() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual std::string broadcast(const std::string& data, int root = 0) = 0;
  virtual std::vector<std::string> allgather(const std::string& data) = 0;
  virtual void barrier() = 0;
  // every rank lives in this process: device pointers are shared directly
  // (peer access) instead of through IPC handles
  virtual bool in_process() const { return false; }
};

// The ranks of a VirtualGroup (one thread each) as a bootstrap.
class GroupBootstrap final : public Bootstrap {
 public:
  GroupBootstrap(std::shared_ptr<VirtualGroup> g, int rank);
  int rank() const override { return rank_; }
  int size() const override { return g_->size(); }
  std::string broadcast(const std::string& data, int root = 0) override;
  std::vector<std::string> allgather(const std::string& data) override;
  void barrier() override { g_->barrier(); }
  bool in_process() const override { return true; }

 private:
  std::shared_ptr<VirtualGroup> g_;
  int rank_;
};

// RCCL communicator (defined in csrc/comm/nccl_comm.cpp).
class NcclComm final : public Comm {
 public:
  // Multi-process: every rank passes the same 128-byte unique id.  The
  // communicator is nonblocking (ncclConfig_t::blocking = 0), so its
  // construction is bounded: DBFS_RCCL_INIT_TIMEOUT_S (default 60 s), then
  // ncclCommAbort and an error -- a bootstrap that never completes (a peer
  // that died, a fabric problem) fails the setup instead of hanging it.
  NcclComm(const std::string& unique_id, int rank, int nranks, Backend& be);
  ~NcclComm() override;
  static std::string unique_id();
  // Single process, one communicator per backend (one GPU each).
  static std::vector<std::unique_ptr<NcclComm>> init_all(const std::vector<Backend*>& bes);

  int rank() const override { return rank_; }
  int size() const override { return size_; }
  std::string name() const override { return "rccl"; }
  void alltoall(const void* send, void* recv, size_t bytes) override;
  void allgather(const void* send, void* recv, size_t bytes) override;
  void allreduce_sum_i64(int64_t* buf, size_t count) override;
  void alltoallv(const void* send, const int64_t* sc, const int64_t* sd, void* recv,
                 const int64_t* rc, const int64_t* rd, size_t eb) override;
  void barrier() override;
  void group_start() override;
  void group_end() override;
  bool groups() const override { return true; }

 private:
  NcclComm() = default;
  void install_watchdog();
  void check_alive() const;
  // a nonblocking communicator's call: ncclInProgress polled to completion
  void settle(int result, const char* what, const char* file, int line);
  void* comm_ = nullptr;  // ncclComm_t
  int rank_ = 0, size_ = 1;
};

// Every collective output one rank saw, in call order (RecordComm ->
// ReplayComm; csrc/comm/replay_comm.cpp).  kind: Comm::TrafficKind; (a, b):
// the call's sizes (bytes per peer / count / total elements, element bytes).
struct CommTape {
  struct Rec {
    int kind = 0;
    int64_t a = 0, b = 0;
    // alltoallv: >= 0 -- data is the receive buffer's span [span, span +
    // size) holding every piece (replayed as one copy); -1 -- the pieces
    // concatenated in rank order
    int64_t span = -1;
    // alltoall_lists (and alltoallv without a span): the received pieces'
    // byte sizes, concatenated in data in rank order
    std::vector<int64_t> pieces;
    std::string data;
  };
  int rank = 0, size = 1;
  bool counted_lists = false;  // the recorded communicator's Comm::counted_lists
  std::vector<Rec> recs;
  int64_t bytes() const;
  static constexpr int kLists = 100;  // Rec::kind of an alltoall_lists (a = stride, b = cap)
};

// Forwards to `inner` and records every output on the host (blocking copies:
// a recording run is not a timed one).
class RecordComm final : public Comm {
 public:
  explicit RecordComm(std::shared_ptr<Comm> inner);
  int rank() const override { return inner_->rank(); }
  int size() const override { return inner_->size(); }
  std::string name() const override { return "record+" + inner_->name(); }
  void alltoall(const void* send, void* recv, size_t bytes) override;
  void allgather(const void* send, void* recv, size_t bytes) override;
  void allreduce_sum_i64(int64_t* buf, size_t count) override;
  void alltoallv(const void* send, const int64_t* sc, const int64_t* sd, void* recv, const int64_t* rc,
                 const int64_t* rd, size_t eb) override;
  void barrier() override;
  void alltoall_lists(const uint32_t* send, uint32_t* recv, size_t stride_words, size_t cap) override;
  bool counted_lists() const override { return inner_->counted_lists(); }
  double max_host(double x) override;  // wall-time maxima: not part of the tape
  std::shared_ptr<CommTape> tape() const { return tape_; }

 private:
  void push(int kind, int64_t a, int64_t b, const void* dev, size_t bytes);
  std::shared_ptr<Comm> inner_;
  std::shared_ptr<CommTape> tape_;
};

// Rank tape->rank of a tape->size-rank job, alone: every collective must be
// the tape's next one and writes its recorded output (a device copy).
class ReplayComm final : public Comm {
 public:
  ReplayComm(std::shared_ptr<CommTape> tape, Backend& be);
  int rank() const override { return tape_->rank; }
  int size() const override { return tape_->size; }
  std::string name() const override { return "replay"; }
  void alltoall(const void* send, void* recv, size_t bytes) override;
  void allgather(const void* send, void* recv, size_t bytes) override;
  void allreduce_sum_i64(int64_t* buf, size_t count) override;
  void alltoallv(const void* send, const int64_t* sc, const int64_t* sd, void* recv, const int64_t* rc,
                 const int64_t* rd, size_t eb) override;
  void barrier() override;
  void alltoall_lists(const uint32_t* send, uint32_t* recv, size_t stride_words, size_t cap) override;
  bool counted_lists() const override { return tape_->counted_lists; }
  // the recorded frontier slices and totals as one multi-piece copy, then the
  // level's decision (two launches; the peer transport's level end is one)
  void level_end(const void* gsend, void* grecv, size_t gbytes, int64_t* buf, size_t count,
                 const LevelFinishArgs& fin) override;
  double max_host(double x) override { return x; }  // this rank's own time
  // a recorded list exchange as a direct one: the apply reads the recorded
  // lists in place (no copy launch), the kernels' own stores land in scratch
  bool direct_lists(size_t cap, DirectExchange* x) override;
  bool direct_level_end(size_t count, DirectExchange* x) override;
  size_t position() const { return pos_; }
  size_t length() const { return tape_->recs.size(); }

 private:
  const CommTape::Rec& next(int kind, int64_t a, int64_t b, size_t* idx);
  std::shared_ptr<CommTape> tape_;
  DBuf<char> dev_;
  DBuf<char> dtab_, dscratch_;                      // direct exchange tables / sinks
  std::unordered_map<size_t, int64_t> dtab_index_;  // record -> table
  int64_t dtab_sink_ = -1;                          // a table of sinks and arrived flags
  std::vector<int64_t> off_;
  size_t pos_ = 0;
};

class TcpBootstrap;

// Collectives through peer-mapped device memory (csrc/comm/peer_comm.cpp,
// csrc/kernels/peer_kernels.hip): every rank exports a window of uncached
// device memory over IPC and maps every peer's; a collective is a push kernel
// (remote stores over xGMI + a flag per sender), a one-wave wait kernel and an
// unpack kernel, all on the backend's communication stream -- a few
// microseconds of latency instead of a library collective's protocol.
// Payloads larger than a window slot go through the windows in slot-sized
// rounds; `inner` (RCCL, or TCP when ranks share a GPU) carries only the
// setup agreements and payloads that are not whole 4-byte words.  Requires:
// one HIP backend per rank, every window mappable.
class PeerComm final : public Comm {
 public:
  // (an in-process bootstrap: the ranks' windows are shared as device
  // pointers with peer access enabled between their devices)
  PeerComm(std::shared_ptr<Bootstrap> boot, Backend& be, std::shared_ptr<Comm> inner, size_t slot_bytes);
  ~PeerComm() override;
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  std::string name() const override;
  void alltoall(const void* send, void* recv, size_t bytes) override;
  void allgather(const void* send, void* recv, size_t bytes) override;
  void allreduce_sum_i64(int64_t* buf, size_t count) override;
  void alltoallv(const void* send, const int64_t* sc, const int64_t* sd, void* recv,
                 const int64_t* rc, const int64_t* rd, size_t eb) override;
  void barrier() override;
  void alltoall_lists(const uint32_t* send, uint32_t* recv, size_t stride_words, size_t cap) override;
  bool counted_lists() const override { return true; }
  bool direct_lists(size_t cap, DirectExchange* x) override;
  bool direct_level_end(size_t count, DirectExchange* x) override;
  const FrontierTable* direct_frontier(size_t words, int parity) override;
  void allgather_allreduce(const void* send, void* recv, size_t bytes, int64_t* buf, size_t count) override;
  void level_end(const void* gsend, void* grecv, size_t gbytes, int64_t* buf, size_t count,
                 const LevelFinishArgs& fin) override;
  size_t slot_bytes() const { return slot_; }
  // Every collective through the windows with known patterns (sizes up to a
  // full slot), checked on the host; the verdict is agreed over the inner
  // communicator, so every rank returns the same answer.
  bool self_test(std::string* why = nullptr);
  // collectives issued through the windows / delegated to the inner communicator
  int64_t peer_ops() const { return peer_ops_; }
  int64_t inner_ops() const { return inner_ops_; }
  // the direct exchanges are on (off: DBFS_PEER_DIRECT=0, or their self-test failed)
  bool direct_on() const { return dtab_ != nullptr; }
  // the pushed frontier slices are on (off: DBFS_PEER_FRONTIER_MB=0, or their self-test failed)
  bool frontier_on() const { return ftab_ != nullptr; }
  bool fused() const { return fused_; }
  bool split_waits() const override { return split_; }
  int coresident() const override { return coresident_; }
  // Topology seen at construction: every rank's PCI bus id, and access[r * P
  // + p] = 2 (ranks r and p share a GPU), 1 (rank r's GPU can access p's),
  // 0 (it cannot), -1 (p's GPU not visible to rank r's process).
  const std::vector<std::string>& bus_ids() const { return bus_; }
  const std::vector<int>& peer_access() const { return access_; }
  bool shared_device() const { return shared_; }
  // the last self_test's verdict ("ok" or why it failed; "" before one ran)
  const std::string& self_test_verdict() const { return verdict_; }

 private:
  struct Piece {
    const void* src = nullptr;
    void* dst = nullptr;  // final destination of a delivered piece (unpack)
    int64_t bytes = 0;
  };
  // One collective launch: segment 0, send[p] goes to rank p and recv[p] is
  // where rank p's piece lands here (empty: none; `counted`: pieces are owner
  // lists sized on the device, bytes = the most they may be; `self_direct`:
  // this rank's own piece is copied straight to recv[rank]); segment 1,
  // sum_count > 0: all-reduce of sum_buf (every rank's input through the
  // windows, summed in place).
  struct Plan {
    std::vector<Piece> send, recv;
    bool self_direct = true;
    bool counted = false;
    int64_t sum_count = 0;
    int64_t* sum_buf = nullptr;
    const LevelFinishArgs* finish = nullptr;  // then the level's decision (sum_count <= kPeerFinishMax)
    const char* op = "collective";            // (a timed-out wait names it)
  };
  void run(const Plan& plan);
  // pieces larger than a slot: nrounds launches of run(), slot-sized slices
  void rounds(const std::vector<const char*>& src, const std::vector<int64_t>& sb, const std::vector<char*>& dst,
              const std::vector<int64_t>& rb, int64_t nrounds, const char* op);
  int64_t nrounds(int64_t bytes) const;
  void direct_self_test();  // (self_test's second part)
  std::shared_ptr<Bootstrap> boot_;
  bool ipc_ = true;                     // peers' windows IPC-mapped (closed on release)
  std::shared_ptr<char> win_keep_;      // in-process: own window, shared-owned by the group
  std::vector<std::shared_ptr<char>> keep_;  // in-process: the peers' windows
  std::shared_ptr<Comm> inner_;
  int rank_ = 0, size_ = 1;
  size_t slot_ = 0;
  char* win_ = nullptr;                 // own window (uncached device memory)
  std::vector<char*> peer_;             // every rank's window as mapped here (peer_[rank_] == win_)
  unsigned* ticket_ = nullptr;
  uint64_t* err_host_ = nullptr;        // host-mapped error word (wait timeouts)
  uint64_t* err_dev_ = nullptr;
  uint64_t seq_ = 0;
  int64_t peer_ops_ = 0, inner_ops_ = 0;
  // every collective as one launch (DBFS_PEER_FUSED=0: push / wait / unpack)
  bool fused_ = true;
  // owner lists exchanged by the kernels themselves (DBFS_PEER_DIRECT=0: off):
  // the device tables of DirectExchange, one per parity
  DirectTable* dtab_ = nullptr;
  // pushed frontier slices: a region of 2 x P buffers of fslot_ bytes after
  // the slots (DBFS_PEER_FRONTIER_MB, default 8; 0: none) and its device
  // tables, one per parity
  size_t fslot_ = 0;
  FrontierTable* ftab_ = nullptr;
  void frontier_self_test();
  std::function<void(double)> prev_watch_;
  bool watch_installed_ = false;
  char* slot_ptr(int owner, int parity, int sender) const;
  void release();
  // several ranks on one physical GPU (bus ids): unfused collectives, split
  // waits (split_; DBFS_PEER_SPLIT=0 keeps the separate-GPU forms)
  bool shared_ = false, split_ = false;
  int coresident_ = 1;
  std::vector<std::string> bus_;
  std::vector<int> access_;
  std::string verdict_;
  // what each recent sequence number was (a timed-out wait names it)
  struct Tag {
    uint64_t seq = 0;
    int level = -1;
    const char* op = "";
  };
  std::vector<Tag> tags_ = std::vector<Tag>(1024);
  void tag(uint64_t seq, const char* op) { tags_[seq % tags_.size()] = Tag{seq, level_tag_, op}; }
  std::string describe_error(uint64_t word) const;
};

// Minimal TCP bootstrap (rank 0 hosts) used to ship the RCCL unique id and for
// host barriers when no MPI / torch store is wanted.  Single- or multi-node.
class TcpBootstrap;

// Host collectives over the TCP bootstrap (star through rank 0).  Device
// buffers are staged through host memory, so it works with any backend: used
// for multi-process CPU runs and as a debug fallback transport (DBFS_COMM=tcp).
class TcpComm final : public Comm {
 public:
  TcpComm(std::shared_ptr<TcpBootstrap> boot, Backend& be);
  int rank() const override;
  int size() const override;
  std::string name() const override { return "tcp"; }
  void alltoall(const void* send, void* recv, size_t bytes) override;
  void allgather(const void* send, void* recv, size_t bytes) override;
  void allreduce_sum_i64(int64_t* buf, size_t count) override;
  void alltoallv(const void* send, const int64_t* sc, const int64_t* sd, void* recv,
                 const int64_t* rc, const int64_t* rd, size_t eb) override;
  void barrier() override;

 private:
  std::string fetch(const void* p, size_t bytes);
  void store(void* p, const std::string& s, size_t off, size_t bytes);
  std::shared_ptr<TcpBootstrap> boot_;
};

class TcpBootstrap final : public Bootstrap {
 public:
  TcpBootstrap(const std::string& host, int port, int rank, int nranks, double timeout_s = 300.0);
  ~TcpBootstrap() override;
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  std::string broadcast(const std::string& data, int root = 0) override;
  std::vector<std::string> allgather(const std::string& data) override;
  void barrier() override;
  // allgather with every receive bounded by timeout_s (0: unbounded), `knob`
  // naming the setting in a timeout's error (TcpComm: DBFS_COMM_TIMEOUT_S)
  std::vector<std::string> allgather_within(const std::string& data, double timeout_s, const char* knob);

 private:
  int rank_, size_;
  int listen_fd_ = -1;
  std::vector<int> peers_;  // rank 0: fd per rank (index = rank); others: [0] = fd to root
};

}  // namespace dbfs
