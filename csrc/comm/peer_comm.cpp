// Peer-memory communicator: collectives as stream-ordered kernels over
// IPC-mapped windows (see dbfs/comm.hpp, csrc/kernels/peer_kernels.hip).
//
// Window layout (per rank, uncached device memory, exported over IPC):
//   [0, 4096)                       flag words, one per sender (monotonic seq)
//   4096 + ((parity * P) + s) * slot payload slot written by sender s
// Collective number `seq` uses parity seq & 1.  A sender reuses a parity slot
// (seq + 2) only after it has waited for every peer's seq + 1, which each peer
// pushed after it had unpacked seq -- so two slots per sender suffice, provided
// every collective involves every rank (all of these do) and a rank's
// collectives are totally ordered on its streams (the engine joins the side
// stream before issuing on the compute stream again).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "dbfs/comm.hpp"
#include "../kernels/launch.hpp"

namespace dbfs {

#define HIP_CHECK(expr)                                                                          \
  do {                                                                                           \
    hipError_t e_ = (expr);                                                                      \
    if (e_ != hipSuccess)                                                                        \
      ::dbfs::raise_error(__FILE__, __LINE__, std::string("HIP error ") + hipGetErrorString(e_) + \
                                                  " in " #expr);                                 \
  } while (0)

namespace {
// DBFS_FAULT_INJECT="kind=<k>" for a communicator's construction (tests):
// peer_init makes the peer transport's setup fail on every rank that sees it
bool fault_kind_is(const char* kind) {
  const char* e = std::getenv("DBFS_FAULT_INJECT");
  return e && std::string(e).find(std::string("kind=") + kind) != std::string::npos;
}
constexpr size_t kFlagBytes = 4096;
constexpr size_t kCellBase = 1024;  // direct exchange cells in the flag page (flags: bytes [0, 8 P))
static_assert(kCellBase + 2 * 16 * 16 <= kFlagBytes, "direct cells fit the flag page");
inline hipStream_t S(Backend* be) { return static_cast<hipStream_t>(be->comm_stream_handle()); }
}  // namespace

PeerComm::PeerComm(std::shared_ptr<Bootstrap> boot, Backend& be, std::shared_ptr<Comm> inner, size_t slot_bytes)
    : boot_(std::move(boot)), inner_(std::move(inner)), slot_(slot_bytes) {
  DBFS_CHECK(be.kind() == DeviceKind::HIP, "PeerComm requires a HIP backend");
  DBFS_CHECK(boot_ && inner_, "PeerComm needs a bootstrap and an inner communicator");
  rank_ = boot_->rank();
  size_ = boot_->size();
  ipc_ = !boot_->in_process();
  if (const char* e = std::getenv("DBFS_PEER_FUSED")) fused_ = std::string(e) != "0";
  DBFS_CHECK(size_ <= kern::kMaxPeers, "PeerComm supports at most 16 ranks");
  DBFS_CHECK(inner_->rank() == rank_ && inner_->size() == size_, "inner communicator does not match the bootstrap");
  DBFS_CHECK(slot_ >= 4096 && slot_ % 256 == 0, "PeerComm slot size must be a multiple of 256 B (>= 4 KiB)");
  bind_backend(&be);
  // Every step that can fail locally is agreed over the bootstrap, so all
  // ranks either build the communicator or all throw (no rank is left waiting
  // in a bootstrap exchange its peers never join).
  std::string local_err;
  hipIpcMemHandle_t h{};
  try {
    HIP_CHECK(hipSetDevice(be.device_id()));
    if (fault_kind_is("peer_init")) throw Error("injected fault (peer_init)");
    // the pushed frontier slices' region (Comm::direct_frontier)
    if (const char* fe = std::getenv("DBFS_PEER_FRONTIER_MB")) fslot_ = static_cast<size_t>(std::max(0L, std::atol(fe))) << 20;
    else fslot_ = size_t(8) << 20;
    const size_t total = kFlagBytes + 2 * static_cast<size_t>(size_) * (slot_ + fslot_);
    void* w = nullptr;
    HIP_CHECK(hipExtMallocWithFlags(&w, total, hipDeviceMallocUncached));
    win_ = static_cast<char*>(w);
    HIP_CHECK(hipMemset(win_, 0, total));
    HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&ticket_), sizeof(unsigned)));
    HIP_CHECK(hipMemset(ticket_, 0, sizeof(unsigned)));
    HIP_CHECK(hipDeviceSynchronize());
    void* dptr = nullptr;
    err_host_ = static_cast<uint64_t*>(be.alloc_mapped(sizeof(uint64_t), &dptr));
    err_dev_ = static_cast<uint64_t*>(dptr);
    if (ipc_) HIP_CHECK(hipIpcGetMemHandle(&h, win_));
  } catch (const std::exception& e) {
    local_err = e.what();
  }
  // what a peer needs to map this window: an IPC handle, or (one process)
  // the pointer and its device
  // (in-process: every rank keeps every window alive -- a window is freed
  // with the group's last communicator, so no rank waits for the others on
  // destruction)
  struct Local {
    char* win;
    int device;
    const std::shared_ptr<char>* keep;
  };
  if (!ipc_ && win_) win_keep_ = std::shared_ptr<char>(win_, [](char* w) { (void)hipFree(w); });
  const Local loc{win_, be.device_id(), &win_keep_};
  const std::string mine = !local_err.empty() ? std::string()
                           : ipc_ ? std::string(reinterpret_cast<const char*>(&h), sizeof(h))
                                  : std::string(reinterpret_cast<const char*>(&loc), sizeof(loc));
  const auto all = boot_->allgather(mine);
  auto agree = [&](const std::string& what) {
    // every rank's status; throw on all ranks if any failed
    const auto st = boot_->allgather(local_err);
    for (int p = 0; p < size_; ++p)
      if (!st[p].empty()) {
        release();
        throw Error("PeerComm " + what + " failed on rank " + std::to_string(p) + ": " + st[p]);
      }
  };
  agree("window allocation / export");
  peer_.assign(static_cast<size_t>(size_), nullptr);
  try {
    for (int p = 0; p < size_; ++p) {
      if (p == rank_) {
        peer_[p] = win_;
        continue;
      }
      if (!ipc_) {
        DBFS_CHECK(all[p].size() == sizeof(Local), "PeerComm: bad window record from a peer");
        Local pl;
        std::memcpy(&pl, all[p].data(), sizeof(pl));
        // threads of one process sharing a device cannot wait for each other in
        // kernels while any of them makes a device-wide synchronisation
        // (hipFree does: it waits for the other's spinning collective): only
        // with the backend's frees deferred (Backend::set_deferred_frees -- the
        // single-process CLI rehearsing --gpus P on one device, DBFS_DEVICE)
        DBFS_CHECK(pl.device != be.device_id() || be.deferred_frees(),
                   "PeerComm: in-process ranks " + std::to_string(rank_) + " and " + std::to_string(p) +
                       " share device " + std::to_string(pl.device) +
                       " (one device per rank, or one process per rank)");
        if (pl.device != be.device_id()) {
          int can = 0;
          HIP_CHECK(hipDeviceCanAccessPeer(&can, be.device_id(), pl.device));
          DBFS_CHECK(can, "PeerComm: device " + std::to_string(be.device_id()) + " cannot access device " +
                              std::to_string(pl.device));
          const hipError_t e = hipDeviceEnablePeerAccess(pl.device, 0);
          if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIP_CHECK(e);
          (void)hipGetLastError();  // (clear an already-enabled status)
        }
        peer_[p] = pl.win;
        keep_.push_back(*pl.keep);
        continue;
      }
      DBFS_CHECK(all[p].size() == sizeof(hipIpcMemHandle_t), "PeerComm: bad IPC handle from a peer");
      hipIpcMemHandle_t ph;
      std::memcpy(&ph, all[p].data(), sizeof(ph));
      void* m = nullptr;
      HIP_CHECK(hipIpcOpenMemHandle(&m, ph, hipIpcMemLazyEnablePeerAccess));
      peer_[p] = static_cast<char*>(m);
    }
  } catch (const std::exception& e) {
    local_err = e.what();
  }
  agree("window mapping");
  if (!ipc_) boot_->barrier();  // every rank holds every window before any may drop one
  // Topology: every rank's PCI bus id; ranks on one physical GPU (tests
  // rehearsing several ranks on one device) get unfused collectives and
  // split waits -- a collective that spins in every workgroup can hold the
  // CUs a co-resident rank's producer needs (Comm::split_waits)
  {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), be.device_id()) != hipSuccess) bus[0] = 0;
    bus_ = boot_->allgather(std::string(bus));
    std::string row;
    for (int p = 0; p < size_; ++p) {
      int a = -1;
      if (!bus_[p].empty() && bus_[p] == bus_[rank_]) {
        a = 2;
      } else {
        int d = -1, can = 0;
        if (!bus_[p].empty() && hipDeviceGetByPCIBusId(&d, bus_[p].c_str()) == hipSuccess && d >= 0 &&
            hipDeviceCanAccessPeer(&can, be.device_id(), d) == hipSuccess)
          a = can ? 1 : 0;
        (void)hipGetLastError();
      }
      row.push_back(static_cast<char>('0' + a + 1));
    }
    const auto rows = boot_->allgather(row);
    access_.assign(static_cast<size_t>(size_) * size_, -1);
    for (int r = 0; r < size_; ++r)
      for (int p = 0; p < size_ && p < static_cast<int>(rows[r].size()); ++p) access_[r * size_ + p] = rows[r][p] - '1';
    for (int p = 0; p < size_ && !shared_; ++p)
      for (int q = p + 1; q < size_; ++q)
        if (!bus_[p].empty() && bus_[p] == bus_[q]) shared_ = true;
    coresident_ = 0;
    for (int p = 0; p < size_; ++p) coresident_ += !bus_[rank_].empty() && bus_[p] == bus_[rank_] ? 1 : 0;
    coresident_ = std::max(coresident_, 1);
    // (DBFS_PEER_SPLIT=0: the separate-GPU forms on a shared GPU anyway --
    // tests of the fused collectives and in-kernel waits with two ranks,
    // which cannot starve each other of CUs)
    const char* sp = std::getenv("DBFS_PEER_SPLIT");
    split_ = shared_ && !(sp && std::string(sp) == "0");
    if (split_) fused_ = false;
  }
  // the direct exchange's tables (one per parity; DBFS_PEER_DIRECT=0: none)
  const char* de = std::getenv("DBFS_PEER_DIRECT");
  if (!de || std::string(de) != "0") {
    static_assert(kMaxDirectRanks == kern::kMaxPeers, "direct exchange and peer kernels share the rank bound");
    DirectTable t[2];
    // the direct exchanges' cells: flag page bytes [kCellBase, +2 x 16 x 16)
    auto cell = [&](char* win, int parity, int sender) {
      return reinterpret_cast<uint64_t*>(win + kCellBase + (static_cast<size_t>(parity) * kern::kMaxPeers + sender) * 16);
    };
    for (int b = 0; b < 2; ++b) {
      std::memset(&t[b], 0, sizeof(DirectTable));
      for (int p = 0; p < size_; ++p) {
        const bool self = p == rank_;
        t[b].dst[p] = self ? nullptr : reinterpret_cast<uint32_t*>(slot_ptr(p, b, rank_));
        t[b].cell_out[p] = self ? nullptr : cell(peer_[p], b, rank_);
        t[b].src[p] = reinterpret_cast<const uint32_t*>(slot_ptr(rank_, b, p));
        t[b].cell_in[p] = self ? nullptr : cell(win_, b, p);
      }
    }
    try {
      void* d = nullptr;
      HIP_CHECK(hipMalloc(&d, sizeof(t)));
      dtab_ = static_cast<DirectTable*>(d);
      HIP_CHECK(hipMemcpy(d, t, sizeof(t), hipMemcpyHostToDevice));
    } catch (const std::exception& e) {
      local_err = e.what();
    }
  }
  agree("direct exchange tables");  // (every rank has them, or none goes on)
  // the pushed frontier slices' tables (one per parity): [parity][sender]
  // buffers of fslot_ bytes after the slots
  if (dtab_ && fslot_ > 0) {
    FrontierTable t[2];
    auto buf = [&](char* win, int parity, int sender) {
      return reinterpret_cast<uint64_t*>(win + kFlagBytes + 2 * static_cast<size_t>(size_) * slot_ +
                                         (static_cast<size_t>(parity) * size_ + sender) * fslot_);
    };
    for (int b = 0; b < 2; ++b) {
      std::memset(&t[b], 0, sizeof(FrontierTable));
      for (int p = 0; p < size_; ++p) {
        t[b].dst[p] = p == rank_ ? nullptr : buf(peer_[p], b, rank_);
        t[b].src[p] = p == rank_ ? nullptr : buf(win_, b, p);
      }
    }
    try {
      void* d = nullptr;
      HIP_CHECK(hipMalloc(&d, sizeof(t)));
      ftab_ = static_cast<FrontierTable*>(d);
      HIP_CHECK(hipMemcpy(d, t, sizeof(t), hipMemcpyHostToDevice));
    } catch (const std::exception& e) {
      local_err = e.what();
    }
  }
  agree("frontier push tables");
  // a wait kernel that timed out leaves its seq in the error word: the host's
  // waits (stream synchronise, mailbox spins) turn it into an error
  prev_watch_ = be.wait_watch();
  auto prev = prev_watch_;
  uint64_t* eh = err_host_;
  be.set_wait_watch([this, eh, prev](double waited) {
    const uint64_t e = __atomic_load_n(eh, __ATOMIC_ACQUIRE);
    if (e) throw Error(describe_error(e));
    if (prev) prev(waited);
  });
  watch_installed_ = true;
  boot_->barrier();  // every rank has mapped every window
}

PeerComm::~PeerComm() {
  if (be_ && watch_installed_) {
    // collectives run on the communication stream, the kernels that write
    // into peers' windows directly on the compute stream: both drained
    hipStreamSynchronize(static_cast<hipStream_t>(be_->stream_handle()));
    hipStreamSynchronize(S(be_));
    be_->set_wait_watch(prev_watch_);
    // no rank unmaps or frees a window while a peer may still write into it
    // or read it (a peer that failed closes its socket: the barrier throws at
    // once and is ignored -- nothing of that peer is in flight any more).
    // After a timed-out wait (a peer hung) there is no barrier to reach: the
    // IPC allocations stay alive while any importer still maps them.
    // In-process the windows are shared-owned instead: the last rank frees.
    const bool peer_lost = err_host_ && __atomic_load_n(err_host_, __ATOMIC_ACQUIRE) != 0;
    if (ipc_ && !peer_lost) {
      try {
        boot_->barrier();
      } catch (const std::exception&) {
      }
    }
  }
  release();
}

void PeerComm::release() {
  for (int p = 0; p < static_cast<int>(peer_.size()); ++p)
    if (ipc_ && p != rank_ && peer_[p]) hipIpcCloseMemHandle(peer_[p]);
  peer_.clear();
  // (through the backend: deferred when it defers frees)
  if (ticket_) be_ ? be_->dealloc(ticket_) : (void)hipFree(ticket_);
  ticket_ = nullptr;
  if (dtab_) be_ ? be_->dealloc(dtab_) : (void)hipFree(dtab_);
  dtab_ = nullptr;
  if (ftab_) be_ ? be_->dealloc(ftab_) : (void)hipFree(ftab_);
  ftab_ = nullptr;
  keep_.clear();
  if (win_keep_) win_keep_.reset();  // (in-process: frees with the last holder)
  else if (win_) hipFree(win_);
  win_ = nullptr;
  if (be_ && err_host_) be_->free_mapped(err_host_);
  err_host_ = nullptr;
}

std::string PeerComm::name() const { return "peer+" + inner_->name(); }

// A timed-out device wait's error word (kWaitSeqMask) as a message: this
// rank, the collective's sequence number, what it was and for which level,
// and the peer that never arrived.
std::string PeerComm::describe_error(uint64_t word) const {
  const uint64_t seq = word & kWaitSeqMask;
  const int peer = static_cast<int>((word >> 48) & 0xFF) - 1;
  std::string what = "collective #" + std::to_string(seq);
  const Tag& t = tags_[seq % tags_.size()];
  if (t.seq == seq) {
    what += std::string(" (") + t.op;
    if (t.level >= 0) what += ", level " + std::to_string(t.level);
    what += ")";
  }
  const double limit = comm_timeout_s() > 0 ? std::min(comm_timeout_s(), 60.0) : 60.0;
  return "peer communicator: rank " + std::to_string(rank_) + " timed out in " + what + " waiting for " +
         (peer >= 0 ? "rank " + std::to_string(peer) : std::string("a peer")) + " (device wait bound " +
         std::to_string(static_cast<int>(limit)) + " s, DBFS_COMM_TIMEOUT_S)";
}

char* PeerComm::slot_ptr(int owner, int parity, int sender) const {
  return peer_[owner] + kFlagBytes + (static_cast<size_t>(parity) * size_ + sender) * slot_;
}

namespace {
int unit_for(uintptr_t x) { return (x % 16 == 0) ? 16 : (x % 8 == 0) ? 8 : 4; }
}  // namespace

void PeerComm::run(const Plan& plan) {
  const int P = size_;
  const uint64_t s = ++seq_;
  tag(s, plan.op);
  const int b = static_cast<int>(s & 1);
  const hipStream_t st = S(be_);
  HIP_CHECK(hipSetDevice(be_->device_id()));
  const bool has_copy = !plan.send.empty();
  const bool has_sum = plan.sum_count > 0;
  // slot layout per sender: [segment 0 (copy), padded to 16 B][segment 1 (sum input)]
  int64_t seg0_max = 0;
  if (has_copy)
    for (int p = 0; p < P; ++p) seg0_max = std::max(seg0_max, plan.send[p].bytes);
  const int64_t off2 = has_copy ? (seg0_max + 15) / 16 * 16 : 0;
  DBFS_CHECK(static_cast<size_t>(off2 + plan.sum_count * 8) <= slot_, "PeerComm: collective larger than a window slot");
  // this rank's own segment 0 goes straight to its destination (self_direct);
  // its all-reduce input goes through its own window like every peer's, so
  // then it waits for its own flag too
  const bool self_copy_direct = has_copy && plan.self_direct;
  const bool self_flag = has_sum || !self_copy_direct;
  int unit = 16;
  auto fit = [&](const void* x) { unit = std::min(unit, unit_for(reinterpret_cast<uintptr_t>(x))); };
  kern::PeerPushArgs pa;
  pa.npeers = P;
  pa.seq = s;
  pa.ticket = ticket_;
  kern::PeerUnpackArgs ua;
  ua.npeers = P;
  ua.counted = plan.counted;
  for (int p = 0; p < P; ++p) {
    char* slot = slot_ptr(p, b, rank_);
    const bool direct = self_copy_direct && p == rank_;
    if (has_copy) {
      pa.src[p] = plan.send[p].src;
      pa.bytes[p] = plan.send[p].bytes;
      pa.dst[p] = direct ? plan.recv[p].dst : slot;
      if (plan.counted) pa.count[p] = static_cast<const uint32_t*>(plan.send[p].src);
      if (direct && pa.src[p] == pa.dst[p]) pa.bytes[p] = 0;  // in place
      if (pa.bytes[p] > 0) {
        fit(pa.src[p]);
        fit(pa.dst[p]);
        unit = std::min(unit, unit_for(static_cast<uintptr_t>(pa.bytes[p])));
      }
      // unpack: the piece rank p left in this rank's window
      ua.src[p] = slot_ptr(rank_, b, p);
      ua.dst[p] = plan.recv[p].dst;
      ua.bytes[p] = (self_copy_direct && p == rank_) ? 0 : plan.recv[p].bytes;
      if (ua.bytes[p] > 0) {
        fit(ua.dst[p]);
        unit = std::min(unit, unit_for(static_cast<uintptr_t>(ua.bytes[p])));
      }
    }
    if (has_sum) {
      pa.dst2[p] = slot + off2;
      ua.sum_src[p] = slot_ptr(rank_, b, p) + off2;
    }
    pa.flag[p] = (p == rank_ && !self_flag) ? nullptr : reinterpret_cast<uint64_t*>(peer_[p]) + rank_;
  }
  if (has_sum) {
    pa.src2 = plan.sum_buf;
    pa.bytes2 = plan.sum_count * 8;
    fit(plan.sum_buf);
    unit = std::min(unit, 8);
    ua.sum_count = plan.sum_count;
    ua.sum_out = plan.sum_buf;
    if (plan.finish) {
      DBFS_CHECK(plan.sum_count <= kern::kPeerFinishMax, "PeerComm: a level end reduces at most 256 totals");
      ua.has_finish = true;
      ua.finish = *plan.finish;
    }
  }
  DBFS_CHECK(unit >= 4, "PeerComm payloads must be multiples of 4 bytes, 4-byte aligned");
  DBFS_CHECK(!plan.counted || unit >= 4, "PeerComm: counted lists need 4-byte granules");
  pa.unit = ua.unit = unit;
  const bool fused = fused_;
  if (!fused) {
    kern::peer_push(pa, st);
    HIP_CHECK(hipGetLastError());
  }
  kern::PeerWaitArgs wa;
  wa.flags = reinterpret_cast<const uint64_t*>(win_);
  wa.npeers = P;
  wa.skip = self_flag ? -1 : rank_;
  wa.seq = s;
  // (a peer that is minutes late is dead: the device-side wait gives up after
  // at most 60 s so a hung job frees the GPU and reports the error)
  const double limit = comm_timeout_s() > 0 ? std::min(comm_timeout_s(), 60.0) : 60.0;
  const double khz = be_->wall_clock_khz() > 0 ? be_->wall_clock_khz() : 100000.0;
  wa.timeout_ticks = static_cast<uint64_t>(limit * khz * 1000.0);
  wa.error = err_dev_;
  if (fused) {
    // ranks sharing a GPU (DBFS_PEER_SPLIT=0): every workgroup of a fused
    // launch spins on the peers' flags, so the co-resident ranks' launches
    // together stay a small part of the chip (<= kPeerFusedGroups x 256
    // threads per peer over all of them) -- a peer's producer always finds CUs
    pa.max_groups = coresident_ > 1 ? std::max<int>(1, static_cast<int>(kern::kPeerFusedGroups) / coresident_) : 0;
    kern::peer_fused(pa, wa, ua, st);
    HIP_CHECK(hipGetLastError());
    ++peer_ops_;
    return;
  }
  kern::peer_wait(wa, st);
  HIP_CHECK(hipGetLastError());
  // (a timed-out wait leaves its error word set: the unpack then copies
  // nothing and finishes no level -- the host's wait watch reports the stall)
  ua.error = err_dev_;
  kern::peer_unpack(ua, st);
  HIP_CHECK(hipGetLastError());
  ++peer_ops_;
}

// Payloads larger than a window slot go through the windows in rounds of at
// most one slot per peer (one launch each, in order on the comm stream; a
// round's parity slots are reused two rounds later, after the peers' flags of
// the round in between -- the same rule as any two consecutive collectives).
// The round count is a function of sizes every rank knows (or agreed first),
// so every rank issues the same sequence: RCCL is never needed for size.
// src[p] / sb[p]: the piece for rank p; dst[p] / rb[p]: where rank p's lands.
// (The reference copies each pair's bucket with one cudaMemcpyPeer,
// bfs.cu:604-605.)
void PeerComm::rounds(const std::vector<const char*>& src, const std::vector<int64_t>& sb,
                      const std::vector<char*>& dst, const std::vector<int64_t>& rb, int64_t nrounds, const char* op) {
  const int64_t slot = static_cast<int64_t>(slot_);
  for (int64_t k = 0; k < std::max<int64_t>(nrounds, 1); ++k) {
    const int64_t off = k * slot;
    auto piece = [&](int64_t total) { return std::max<int64_t>(0, std::min(slot, total - off)); };
    Plan pl;
    pl.op = op;
    pl.send.resize(static_cast<size_t>(size_));
    pl.recv.resize(static_cast<size_t>(size_));
    for (int p = 0; p < size_; ++p) {
      const int64_t sn = piece(sb[p]), rn = piece(rb[p]);
      pl.send[p] = {src[p] + (sn > 0 ? off : 0), nullptr, sn};
      pl.recv[p] = {nullptr, dst[p] + (rn > 0 ? off : 0), rn};
    }
    run(pl);
  }
}

int64_t PeerComm::nrounds(int64_t bytes) const {
  const int64_t slot = static_cast<int64_t>(slot_);
  return std::max<int64_t>(1, (bytes + slot - 1) / slot);
}

void PeerComm::alltoall(const void* send, void* recv, size_t bytes) {
  note(kAllToAll, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(bytes));
  if (bytes % 4) {
    ++inner_ops_;
    inner_->alltoall(send, recv, bytes);
    return;
  }
  std::vector<const char*> src(static_cast<size_t>(size_));
  std::vector<char*> dst(static_cast<size_t>(size_));
  std::vector<int64_t> n(static_cast<size_t>(size_), static_cast<int64_t>(bytes));
  for (int p = 0; p < size_; ++p) {
    src[p] = static_cast<const char*>(send) + p * bytes;
    dst[p] = static_cast<char*>(recv) + p * bytes;
  }
  rounds(src, n, dst, n, nrounds(static_cast<int64_t>(bytes)), "alltoall");
}

void PeerComm::allgather(const void* send, void* recv, size_t bytes) {
  note(kAllGather, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(bytes));
  if (bytes % 4) {
    ++inner_ops_;
    inner_->allgather(send, recv, bytes);
    return;
  }
  std::vector<const char*> src(static_cast<size_t>(size_), static_cast<const char*>(send));
  std::vector<char*> dst(static_cast<size_t>(size_));
  std::vector<int64_t> n(static_cast<size_t>(size_), static_cast<int64_t>(bytes));
  for (int p = 0; p < size_; ++p) dst[p] = static_cast<char*>(recv) + p * bytes;
  rounds(src, n, dst, n, nrounds(static_cast<int64_t>(bytes)), "allgather");
}

void PeerComm::allreduce_sum_i64(int64_t* buf, size_t count) {
  note(kAllReduce, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(count) * 8);
  if (count == 0) return;
  const size_t per = slot_ / sizeof(int64_t);
  for (size_t off = 0; off < count; off += per) {
    Plan pl;
    pl.op = "allreduce";
    pl.sum_count = static_cast<int64_t>(std::min(per, count - off));
    pl.sum_buf = buf + off;
    run(pl);
  }
}

void PeerComm::alltoallv(const void* send, const int64_t* sc, const int64_t* sd, void* recv, const int64_t* rc,
                         const int64_t* rd, size_t eb) {
  note_alltoallv(sc, eb);
  // The element size is the same on every rank; the counts are this rank's
  // own, so the number of rounds (the largest piece of any rank) is agreed
  // through the windows first.  (Host counts imply a host round trip
  // already; the engine's device-loop lists use alltoall_lists.)
  if (eb % 4 != 0) {
    ++inner_ops_;
    inner_->alltoallv(send, sc, sd, recv, rc, rd, eb);
    return;
  }
  const int64_t e = static_cast<int64_t>(eb);
  std::vector<const char*> src(static_cast<size_t>(size_));
  std::vector<char*> dst(static_cast<size_t>(size_));
  std::vector<int64_t> sb(static_cast<size_t>(size_)), rb(static_cast<size_t>(size_));
  int64_t mx = 0;
  for (int p = 0; p < size_; ++p) {
    src[p] = static_cast<const char*>(send) + sd[p] * e;
    dst[p] = static_cast<char*>(recv) + rd[p] * e;
    sb[p] = sc[p] * e;
    rb[p] = rc[p] * e;
    mx = std::max(mx, std::max(sb[p], rb[p]));
  }
  int64_t gmx = 0;
  for (int64_t x : allgather_host_i64(mx)) gmx = std::max(gmx, x);  // (one 8-byte round)
  rounds(src, sb, dst, rb, nrounds(gmx), "alltoallv");
}

void PeerComm::alltoall_lists(const uint32_t* send, uint32_t* recv, size_t stride_words, size_t cap) {
  const int64_t piece = static_cast<int64_t>(cap + 1) * 4;
  // (the choice depends only on the capacity, the same on every rank)
  if (static_cast<size_t>(piece) > slot_ || stride_words % 4 != 0 || stride_words < cap + 1) {
    // cap + 1 words per peer (the capacity: the same on every rank), in
    // slot-sized rounds through the windows
    note(kAllToAllV, static_cast<int64_t>(size_ - 1) * piece);
    DBFS_CHECK(stride_words >= cap + 1, "alltoall_lists: stride below the list capacity");
    std::vector<const char*> src(static_cast<size_t>(size_));
    std::vector<char*> dst(static_cast<size_t>(size_));
    std::vector<int64_t> n(static_cast<size_t>(size_), piece);
    for (int p = 0; p < size_; ++p) {
      src[p] = reinterpret_cast<const char*>(send + p * stride_words);
      dst[p] = reinterpret_cast<char*>(recv + p * stride_words);
    }
    rounds(src, n, dst, n, nrounds(piece), "owner lists");
    return;
  }
  // (traffic accounted at the capacity, as the default exchange: the device
  // counts are not read back)
  note(kAllToAllV, static_cast<int64_t>(size_ - 1) * piece);
  // count-sized: each piece is its list's n + 1 words, read on the device
  // (rounded up to 16 B, at most the stride)
  const int64_t stride_b = static_cast<int64_t>(stride_words) * 4;
  const int64_t cap_b = std::min<int64_t>((piece + 15) / 16 * 16, stride_b);
  Plan pl;
  pl.op = "owner lists";
  pl.counted = true;
  pl.send.resize(static_cast<size_t>(size_));
  pl.recv.resize(static_cast<size_t>(size_));
  for (int p = 0; p < size_; ++p) {
    pl.send[p] = {send + p * stride_words, nullptr, cap_b};
    pl.recv[p] = {nullptr, recv + p * stride_words, cap_b};
  }
  run(pl);
}

bool PeerComm::direct_lists(size_t cap, DirectExchange* x) {
  const int64_t piece = static_cast<int64_t>(cap + 1) * 4;
  if (static_cast<size_t>(piece) > slot_ || !dtab_) return false;
  note(kAllToAllV, static_cast<int64_t>(size_ - 1) * piece);  // (accounted at the capacity, as alltoall_lists)
  const uint64_t s = ++seq_;
  tag(s, "owner lists (direct)");
  x->active = 1;
  x->nranks = size_;
  x->rank = rank_;
  x->seq = s;
  x->table = dtab_ + (s & 1);
  const double limit = comm_timeout_s() > 0 ? std::min(comm_timeout_s(), 60.0) : 60.0;
  const double khz = be_->wall_clock_khz() > 0 ? be_->wall_clock_khz() : 100000.0;
  x->timeout_ticks = static_cast<uint64_t>(limit * khz * 1000.0);
  x->error = err_dev_;
  ++peer_ops_;
  return true;
}

const FrontierTable* PeerComm::direct_frontier(size_t words, int parity) {
  if (!ftab_ || words == 0 || words * sizeof(uint64_t) > fslot_) return nullptr;
  note(kAllGather, static_cast<int64_t>(size_ - 1) * static_cast<int64_t>(words * sizeof(uint64_t)));
  ++peer_ops_;
  return ftab_ + (parity & 1);
}

bool PeerComm::direct_level_end(size_t count, DirectExchange* x) {
  // (a level's totals: at most 2^32 new vertices and 2^40 of their degrees
  // per rank -- the cells' payload widths)
  if (!dtab_ || count != 2 || be_ == nullptr) return false;
  note(kAllReduce, static_cast<int64_t>(size_ - 1) * static_cast<int64_t>(count) * 8);
  const uint64_t s = ++seq_;
  tag(s, "level end (direct)");
  x->active = 1;
  x->nranks = size_;
  x->rank = rank_;
  x->seq = s;
  x->table = dtab_ + (s & 1);
  const double limit = comm_timeout_s() > 0 ? std::min(comm_timeout_s(), 60.0) : 60.0;
  const double khz = be_->wall_clock_khz() > 0 ? be_->wall_clock_khz() : 100000.0;
  x->timeout_ticks = static_cast<uint64_t>(limit * khz * 1000.0);
  x->error = err_dev_;
  x->result = nullptr;
  ++peer_ops_;
  return true;
}

void PeerComm::level_end(const void* gsend, void* grecv, size_t gbytes, int64_t* buf, size_t count,
                         const LevelFinishArgs& fin) {
  const size_t need = (gbytes + 15) / 16 * 16 + count * sizeof(int64_t);
  if (need > slot_ || gbytes % 4 || count == 0 || static_cast<int64_t>(count) > kern::kPeerFinishMax) {
    Comm::level_end(gsend, grecv, gbytes, buf, count, fin);
    return;
  }
  // one launch: the frontier slices and the totals pushed, the flags, the
  // slices unpacked, the totals summed and the level decided by one thread
  Plan pl;
  pl.op = gbytes > 0 ? "level end + frontier gather" : "level end";
  if (gbytes > 0) {
    note(kAllGather, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(gbytes));
    note_fused();
    pl.send.resize(static_cast<size_t>(size_));
    pl.recv.resize(static_cast<size_t>(size_));
    for (int p = 0; p < size_; ++p) {
      pl.send[p] = {gsend, nullptr, static_cast<int64_t>(gbytes)};
      pl.recv[p] = {nullptr, static_cast<char*>(grecv) + p * gbytes, static_cast<int64_t>(gbytes)};
    }
  }
  note(kAllReduce, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(count) * 8);
  pl.sum_count = static_cast<int64_t>(count);
  pl.sum_buf = buf;
  pl.finish = &fin;
  run(pl);
}

void PeerComm::allgather_allreduce(const void* send, void* recv, size_t bytes, int64_t* buf, size_t count) {
  const size_t need = (bytes + 15) / 16 * 16 + count * sizeof(int64_t);
  if (need > slot_ || bytes % 4 || count == 0) {
    allgather(send, recv, bytes);  // two collectives
    allreduce_sum_i64(buf, count);
    return;
  }
  note(kAllGather, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(bytes));
  note(kAllReduce, static_cast<int64_t>(size() - 1) * static_cast<int64_t>(count) * 8);
  note_fused();
  Plan pl;
  pl.op = "allgather + allreduce";
  pl.send.resize(static_cast<size_t>(size_));
  pl.recv.resize(static_cast<size_t>(size_));
  for (int p = 0; p < size_; ++p) {
    pl.send[p] = {send, nullptr, static_cast<int64_t>(bytes)};
    pl.recv[p] = {nullptr, static_cast<char*>(recv) + p * bytes, static_cast<int64_t>(bytes)};
  }
  pl.sum_count = static_cast<int64_t>(count);
  pl.sum_buf = buf;
  run(pl);
}

bool PeerComm::self_test(std::string* why) {
  const int P = size_, me = rank_;
  std::string err;
  auto pat = [](int from, int to, int64_t i, int round) {
    return static_cast<int64_t>((static_cast<uint64_t>(from + 1) * 0x9E3779B97F4A7C15ull) ^
                                (static_cast<uint64_t>(to + 3) << 40) ^ (static_cast<uint64_t>(i) * 2654435761ull) ^
                                static_cast<uint64_t>(round));
  };
  try {
    for (int round = 0; round < 4 && err.empty(); ++round) {
      // per-peer words: tiny, odd, and a whole slot
      const int64_t words = round == 0 ? 1 : round == 1 ? 257 : round == 2 ? 4099 : static_cast<int64_t>(slot_ / 8);
      const size_t n = static_cast<size_t>(words) * P;
      DBuf<int64_t> a(*be_, n), b(*be_, n);
      std::vector<int64_t> h(n), g(n);
      // alltoall
      for (int p = 0; p < P; ++p)
        for (int64_t i = 0; i < words; ++i) h[p * words + i] = pat(me, p, i, round);
      be_->to_device(a.data(), h.data(), n * 8);
      alltoall(a.data(), b.data(), static_cast<size_t>(words) * 8);
      be_->to_host(g.data(), b.data(), n * 8);
      for (int p = 0; p < P && err.empty(); ++p)
        for (int64_t i = 0; i < words; ++i)
          if (g[p * words + i] != pat(p, me, i, round)) {
            err = "alltoall mismatch (round " + std::to_string(round) + ", from rank " + std::to_string(p) + ")";
            break;
          }
      // in-place allgather
      for (int64_t i = 0; i < words; ++i) h[me * words + i] = pat(me, -1, i, round);
      be_->to_device(b.data() + me * words, h.data() + me * words, static_cast<size_t>(words) * 8);
      allgather(b.data() + me * words, b.data(), static_cast<size_t>(words) * 8);
      be_->to_host(g.data(), b.data(), n * 8);
      for (int p = 0; p < P && err.empty(); ++p)
        for (int64_t i = 0; i < words; ++i)
          if (g[p * words + i] != pat(p, -1, i, round)) {
            err = "allgather mismatch (round " + std::to_string(round) + ", from rank " + std::to_string(p) + ")";
            break;
          }
      // owner lists, count-sized: rank me sends peer p a list of
      // (me + p + round) % 37 ids (empty ones included), stride >= the most
      const int64_t stride = 64, cap = 60;
      {
        std::vector<uint32_t> hl(static_cast<size_t>(P * stride), 0xDEADBEEFu), gl(hl.size());
        for (int p = 0; p < P; ++p) {
          const uint32_t n = static_cast<uint32_t>((me + p + round) % 37);
          hl[p * stride] = n;
          for (uint32_t k = 0; k < n; ++k) hl[p * stride + 1 + k] = static_cast<uint32_t>(pat(me, p, k, round));
        }
        DBuf<uint32_t> la(*be_, hl.size()), lb(*be_, hl.size());
        be_->to_device(la.data(), hl.data(), hl.size() * 4);
        be_->memset_async(lb.data(), 0, lb.bytes());
        alltoall_lists(la.data(), lb.data(), static_cast<size_t>(stride), static_cast<size_t>(cap));
        be_->to_host(gl.data(), lb.data(), gl.size() * 4);
        for (int p = 0; p < P && err.empty(); ++p) {
          const uint32_t n = static_cast<uint32_t>((p + me + round) % 37);
          bool ok = gl[p * stride] == n;
          for (uint32_t k = 0; k < n && ok; ++k) ok = gl[p * stride + 1 + k] == static_cast<uint32_t>(pat(p, me, k, round));
          if (!ok) err = "alltoall_lists mismatch (round " + std::to_string(round) + ", from rank " + std::to_string(p) + ")";
        }
      }
      // all-gather + all-reduce in one launch
      {
        const int64_t gw = words < 4096 ? words : 4096, cnt2 = 2 + round;
        std::vector<int64_t> hg(static_cast<size_t>(gw * P)), hs(static_cast<size_t>(cnt2));
        for (int64_t i = 0; i < gw; ++i) hg[me * gw + i] = pat(me, -3, i, round);
        for (int64_t i = 0; i < cnt2; ++i) hs[i] = pat(me, -4, i, round);
        DBuf<int64_t> ga(*be_, hg.size()), sa(*be_, hs.size());
        be_->to_device(ga.data() + me * gw, hg.data() + me * gw, static_cast<size_t>(gw) * 8);
        be_->to_device(sa.data(), hs.data(), hs.size() * 8);
        allgather_allreduce(ga.data() + me * gw, ga.data(), static_cast<size_t>(gw) * 8, sa.data(),
                            static_cast<size_t>(cnt2));
        be_->to_host(hg.data(), ga.data(), hg.size() * 8);
        be_->to_host(hs.data(), sa.data(), hs.size() * 8);
        for (int p = 0; p < P && err.empty(); ++p)
          for (int64_t i = 0; i < gw; ++i)
            if (hg[p * gw + i] != pat(p, -3, i, round)) {
              err = "allgather_allreduce gather mismatch (round " + std::to_string(round) + ")";
              break;
            }
        for (int64_t i = 0; i < cnt2 && err.empty(); ++i) {
          uint64_t want = 0;
          for (int p = 0; p < P; ++p) want += static_cast<uint64_t>(pat(p, -4, i, round));
          if (static_cast<uint64_t>(hs[i]) != want)
            err = "allgather_allreduce sum mismatch (round " + std::to_string(round) + ")";
        }
      }
      // all-reduce (wrapping sums)
      const int64_t cnt = std::min<int64_t>(words, static_cast<int64_t>(slot_ / 8));
      for (int64_t i = 0; i < cnt; ++i) h[i] = pat(me, -2, i, round);
      be_->to_device(a.data(), h.data(), static_cast<size_t>(cnt) * 8);
      allreduce_sum_i64(a.data(), static_cast<size_t>(cnt));
      be_->to_host(g.data(), a.data(), static_cast<size_t>(cnt) * 8);
      for (int64_t i = 0; i < cnt && err.empty(); ++i) {
        uint64_t want = 0;
        for (int p = 0; p < P; ++p) want += static_cast<uint64_t>(pat(p, -2, i, round));
        if (static_cast<uint64_t>(g[i]) != want) err = "allreduce mismatch (round " + std::to_string(round) + ")";
      }
    }
    be_->synchronize();
  } catch (const std::exception& e) {
    err = e.what();
  }
  // agree over the inner communicator (the windows may be what is broken)
  const int64_t bad = inner_->sum_host(err.empty() ? 0 : 1);
  if (bad && err.empty()) err = "a peer's self-test failed";
  if (why) *why = err;
  verdict_ = bad == 0 ? "ok" : err;
  if (bad == 0) direct_self_test();
  if (bad == 0) frontier_self_test();
  return bad == 0;
}

// The pushed frontier slices: two rounds (both parities) of known words pushed
// by every rank, a barrier, every peer's checked; a failure anywhere (agreed)
// turns them off on every rank (the level ends then all-gather).
void PeerComm::frontier_self_test() {
  if (!ftab_) return;
  std::string err;
  try {
    const int64_t words = std::min<int64_t>(static_cast<int64_t>(fslot_ / 8), 4096 + 37);
    DBuf<unsigned> e(*be_, 1);
    be_->memset_async(e.data(), 0, sizeof(unsigned));
    for (int round = 0; round < 2; ++round) {
      kern::frontier_selftest(ftab_ + round, rank_, size_, words, round, 0, e.data(), S(be_));
      HIP_CHECK(hipGetLastError());
      be_->synchronize();
      HIP_CHECK(hipStreamSynchronize(S(be_)));
      inner_->sum_host(0);  // (every rank's pushes have landed)
      kern::frontier_selftest(ftab_ + round, rank_, size_, words, round, 1, e.data(), S(be_));
      HIP_CHECK(hipGetLastError());
    }
    unsigned h = 0;
    HIP_CHECK(hipStreamSynchronize(S(be_)));
    be_->to_host(&h, e.data(), sizeof(h));
    if (h) err = std::to_string(h) + " mismatched words";
  } catch (const std::exception& ex) {
    err = ex.what();
  }
  const int64_t bad = inner_->sum_host(err.empty() ? 0 : 1);
  if (bad == 0) return;
  if (rank_ == 0)
    std::fprintf(stderr, "[dbfs] peer communicator: frontier push off (self-test: %s)\n",
                 err.empty() ? "failed on a peer" : err.c_str());
  be_->dealloc(ftab_);
  ftab_ = nullptr;
}

// The direct exchanges (kernels writing into the peers' windows, tagged
// cells): four rounds of known lists and level ends on every rank; a failure
// anywhere (agreed) turns them off on every rank -- the engine then runs the
// collectives -- instead of failing the communicator.
void PeerComm::direct_self_test() {
  if (!dtab_) return;
  std::string err;
  try {
    DBuf<unsigned> e(*be_, 2);  // [0] mismatches, [1] the producers' ticket
    be_->memset_async(e.data(), 0, 2 * sizeof(unsigned));
    for (int round = 0; round < 4; ++round) {
      DirectExchange l, x;
      DBFS_CHECK(direct_lists(4100, &l) && direct_level_end(2, &x), "direct exchange unavailable");
      const double khz = be_->wall_clock_khz() > 0 ? be_->wall_clock_khz() : 100000.0;
      l.timeout_ticks = x.timeout_ticks = static_cast<uint64_t>(10.0 * khz * 1000.0);  // (10 s)
      kern::direct_selftest(l, x, round, e.data(), e.data() + 1, S(be_));
      HIP_CHECK(hipGetLastError());
    }
    unsigned h = 0;
    be_->to_host(&h, e.data(), sizeof(h));  // (synchronises)
    if (h) err = std::to_string(h) + " mismatches / timeouts";
  } catch (const std::exception& ex) {
    err = ex.what();
  }
  if (err_host_) __atomic_store_n(err_host_, uint64_t(0), __ATOMIC_RELEASE);  // (a timed-out wait's mark)
  const int64_t bad = inner_->sum_host(err.empty() ? 0 : 1);
  if (bad == 0) return;
  if (rank_ == 0)
    std::fprintf(stderr, "[dbfs] peer communicator: direct exchanges off (self-test: %s)\n",
                 err.empty() ? "failed on a peer" : err.c_str());
  be_->dealloc(dtab_);
  dtab_ = nullptr;
  if (ftab_) be_->dealloc(ftab_);  // (needs the direct exchanges' self-test passed too)
  ftab_ = nullptr;
}

void PeerComm::barrier() {
  note(kBarrier, 0);
  int64_t* b = scratch(1);
  allreduce_sum_i64(b, 1);  // value irrelevant: completion on every rank is the barrier
  be_->synchronize();
}

}  // namespace dbfs
