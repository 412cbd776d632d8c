// HIP backend: one gfx950 device, one non-blocking HIP stream; every primitive
// is a hand-written kernel launch (csrc/kernels/*.hip) enqueued on that stream.
//
// Replaces the reference's device runtime layer (initCuda2
// bfs.cu:308-360, __managed__ registry bfs.cu:252-269): explicit device
// allocations instead of managed memory, checked errors instead of the
// comma-expression idiom that discards them (bfs.cu:336-351, D3).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "dbfs/backend.hpp"
#include "../kernels/launch.hpp"

namespace dbfs {

#define HIP_CHECK(expr)                                                                              \
  do {                                                                                               \
    hipError_t e_ = (expr);                                                                          \
    if (e_ != hipSuccess)                                                                            \
      ::dbfs::raise_error(__FILE__, __LINE__, std::string("HIP error ") + hipGetErrorString(e_) +    \
                                                  " in " #expr);                                     \
  } while (0)

namespace {

class HipBackend final : public Backend {
 public:
  explicit HipBackend(int dev) : dev_(dev) {
    int n = 0;
    HIP_CHECK(hipGetDeviceCount(&n));
    DBFS_CHECK(dev >= 0 && dev < n, "HIP device " + std::to_string(dev) + " not present (" + std::to_string(n) + " visible)");
    HIP_CHECK(hipSetDevice(dev_));
    HIP_CHECK(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
    HIP_CHECK(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreateWithFlags(&fork_ev_, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&join_ev_, hipEventDisableTiming));
    hipDeviceProp_t prop{};
    HIP_CHECK(hipGetDeviceProperties(&prop, dev_));
    arch_ = prop.gcnArchName;
    cus_ = prop.multiProcessorCount;
    int khz = 0;
    HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev_));
    clock_khz_ = khz;
    HIP_CHECK(hipHostMalloc(&pinned_, kPinned, hipHostMallocDefault));
  }
  ~HipBackend() override {
    hipSetDevice(dev_);
    hipStreamSynchronize(st_);
    hipStreamSynchronize(side_);
    for (hipEvent_t e : events_) hipEventDestroy(e);
    hipEventDestroy(fork_ev_);
    hipEventDestroy(join_ev_);
    hipStreamDestroy(side_);
    if (scan_tmp_) hipFree(scan_tmp_);
    for (void* p : deferred_) hipFree(p);
    for (void* h : deferred_host_) hipHostFree(h);
    if (pinned_) hipHostFree(pinned_);
    hipStreamDestroy(st_);
  }

  DeviceKind kind() const override { return DeviceKind::HIP; }
  std::string name() const override {
    return "hip:" + std::to_string(dev_) + " (" + arch_ + ", " + std::to_string(cus_) + " CUs)";
  }
  int device_id() const override { return dev_; }
  double wall_clock_khz() const override { return clock_khz_; }
  void* stream_handle() override { return st_; }
  void* comm_stream_handle() override { return forked_ ? side_ : st_; }
  void fork_side() override {
    on();
    DBFS_CHECK(!forked_, "fork_side: a side region is already open");
    HIP_CHECK(hipEventRecord(fork_ev_, st_));
    HIP_CHECK(hipStreamWaitEvent(side_, fork_ev_, 0));
    forked_ = true;
  }
  void join_side() override {
    on();
    if (!forked_) return;
    HIP_CHECK(hipEventRecord(join_ev_, side_));
    HIP_CHECK(hipStreamWaitEvent(st_, join_ev_, 0));
    forked_ = false;
  }

  void* alloc(size_t bytes) override {
    on();
    void* p = nullptr;
    if (bytes == 0) bytes = 64;
    HIP_CHECK(hipMalloc(&p, bytes));
    // DBFS_POISON_ALLOC=<byte>: every allocation filled with that byte (a
    // debugging aid -- a read of memory never written shows up as a wrong
    // result in a fresh process too, not only after freed memory is reused)
    static const int poison = [] {
      const char* e = std::getenv("DBFS_POISON_ALLOC");
      return e && *e ? static_cast<int>(std::strtol(e, nullptr, 0)) & 0xff : -1;
    }();
    if (poison >= 0) {
      HIP_CHECK(hipMemsetAsync(p, poison, bytes, st_));
      HIP_CHECK(hipStreamSynchronize(st_));
    }
    return p;
  }
  void dealloc(void* p) override {
    on();
    hipStreamSynchronize(st_);
    hipStreamSynchronize(side_);
    release_(p);
  }
  // Frees deferred to the backend's destruction (Backend::set_deferred_frees):
  // hipFree waits for every stream of the device, and with several ranks of
  // one process on one device that includes a peer's kernel spinning on this
  // rank's next collective -- which this rank enqueues only after the free.
  void set_deferred_frees(bool on) override { defer_ = on; }
  bool deferred_frees() const override { return defer_; }
  void release_(void* p) {
    if (!p) return;
    if (defer_) deferred_.push_back(p);
    else hipFree(p);
  }
  void memset_async(void* p, int v, size_t bytes) override {
    if (!bytes) return;
    on();
    // large zero fills (bitmaps cleared inside a traversal) by a 16-B-store
    // kernel: about half the runtime fill kernel's time
    if (v == 0 && bytes >= (size_t(1) << 16) && kern::zero_fill(p, bytes, st_)) {
      chk();
      return;
    }
    HIP_CHECK(hipMemsetAsync(p, v, bytes, st_));
  }
  void copy_async(void* d, const void* s, size_t bytes) override {
    if (!bytes) return;
    on();
    HIP_CHECK(hipMemcpyAsync(d, s, bytes, hipMemcpyDefault, st_));
  }
  void copy_pieces(const CopyPieces& c) override {
    for (int i = 0; i < c.n; ++i)
      DBFS_CHECK(c.bytes[i] % 4 == 0 && reinterpret_cast<uintptr_t>(c.dst[i]) % 4 == 0 &&
                     reinterpret_cast<uintptr_t>(c.src[i]) % 4 == 0,
                 "copy_pieces: 4-byte pieces only");
    on();
    kern::copy_pieces(c, st_);
    chk();
  }
  void to_host(void* d, const void* s, size_t bytes) override {
    on();
    if (bytes && bytes <= kPinned) {
      // small (per-level statistics) copies: DMA into pinned memory, no staging
      HIP_CHECK(hipMemcpyAsync(pinned_, s, bytes, hipMemcpyDeviceToHost, st_));
      wait_stream();
      std::memcpy(d, pinned_, bytes);
      return;
    }
    if (bytes) HIP_CHECK(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToHost, st_));
    wait_stream();
  }
  void to_device(void* d, const void* s, size_t bytes) override {
    on();
    if (bytes) HIP_CHECK(hipMemcpyAsync(d, s, bytes, hipMemcpyHostToDevice, st_));
    wait_stream();
  }
  void synchronize() override {
    on();
    join_side();
    wait_stream();
  }
  bool stream_idle() override {
    const hipError_t e = hipStreamQuery(st_);
    if (e == hipSuccess) return true;
    if (e != hipErrorNotReady) HIP_CHECK(e);
    return false;
  }

  // Blocking wait on the stream.  With a wait watch installed (RCCL), poll so
  // the watch can inspect the communicator while a collective is in flight.
  void wait_stream() {
    if (!wait_watch_) {
      HIP_CHECK(hipStreamSynchronize(st_));
      return;
    }
    const auto t0 = std::chrono::steady_clock::now();
    double next = wait_period_;
    for (;;) {
      const hipError_t e = hipStreamQuery(st_);
      if (e == hipSuccess) return;
      if (e != hipErrorNotReady) HIP_CHECK(e);
      const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (waited >= next) {
        wait_watch_(waited);
        next = waited + wait_period_;
      }
    }
  }

  int record_event() override {
    on();
    if (ev_used_ == events_.size()) {
      hipEvent_t e;
      HIP_CHECK(hipEventCreate(&e));
      events_.push_back(e);
    }
    HIP_CHECK(hipEventRecord(events_[ev_used_], st_));
    return static_cast<int>(ev_used_++);
  }
  double elapsed_ms(int a, int b) override {
    on();
    HIP_CHECK(hipEventSynchronize(events_.at(b)));
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, events_.at(a), events_.at(b)));
    return ms;
  }
  void reset_events() override { ev_used_ = 0; }

  void fill_level(lvl_t* level, int64_t n, lvl_t value) override { on(); kern::fill_level(level, n, value, st_); chk(); }
  void set_bit(word_t* bm, int64_t bit) override { on(); kern::set_bit(bm, bit, st_); chk(); }
  void update_frontier(const UpdateArgs& a) override { on(); kern::update_frontier(a, st_); chk(); }
  void scan_units(const ScanArgs& a) override { on(); kern::scan_units(a, st_); chk(); }
  void level_ctrl_init(LevelCtrl* c, const LevelCtrl& init) override {
    on();
    kern::level_ctrl_init(c, init, st_);
    chk();
  }
  void init_run(const InitRunArgs& a) override { on(); kern::init_run(a, st_); chk(); }
  void publish_stats(const int64_t* stats, StatsMailbox* mb, int64_t seq) override {
    on();
    kern::publish_stats(stats, mb, seq, st_);
    chk();
  }
  void* alloc_mapped(size_t bytes, void** dptr) override {
    on();
    void* h = nullptr;
    HIP_CHECK(hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(h, 0, bytes);
    HIP_CHECK(hipHostGetDevicePointer(dptr, h, 0));
    return h;
  }
  void free_mapped(void* h) override {
    if (!h) return;
    on();
    hipStreamSynchronize(st_);
    if (defer_) deferred_host_.push_back(h);
    else hipHostFree(h);
  }
  void zero_degree_mask(const ZeroDegArgs& a) override { on(); kern::zero_degree_mask(a, st_); chk(); }
  void compact_frontier(const CompactArgs& a) override { on(); kern::compact_frontier(a, st_); chk(); }
  void td_sparse(const TdSparseArgs& a) override { on(); kern::td_sparse(a, st_); chk(); }
  void td_sparse_apply(const TdSparseArgs& a) override { on(); kern::td_sparse_apply(a, st_); chk(); }
  void level_finish(const LevelFinishArgs& a) override { on(); kern::level_finish(a, st_); chk(); }
  void widen_levels(const uint8_t* in, lvl_t* out, int64_t n, uint8_t base) override {
    on();
    kern::widen_levels(in, out, n, base, st_);
    chk();
  }
  void td_expand(const TdArgs& a) override { on(); kern::td_expand(a, st_); chk(); }
  void td_binned(const BinArgs& a) override { on(); kern::td_binned(a, st_); chk(); }
  void pack_bytes(const PackArgs& a) override { on(); kern::pack_bytes(a, st_); chk(); }
  void list_scatter(const ListScatterArgs& a) override { on(); kern::list_scatter(a, st_); chk(); }
  bool device_checks_enabled() const override { return kern::checks_enabled(); }
  uint64_t take_device_check() override {
    // (only the checked build has a word to read: otherwise no synchronize --
    // a traversal's speculative trailing chain keeps draining while the next
    // one is enqueued behind it)
    if (!kern::checks_enabled()) return 0;
    synchronize();
    return kern::take_check_error();
  }
  void inject_device_check() override { on(); kern::inject_check_failure(st_); chk(); }
  void bu_step(const BuArgs& a) override { on(); kern::bu_step(a, st_); chk(); }
  void hub_gather(const HubGatherArgs& a) override { on(); kern::hub_gather(a, st_); chk(); }
  void bu_cut_prep(const BuArgs& a) override { on(); kern::bu_cut_prep(a, st_); chk(); }
  void bu_cut_merge(const BuArgs& a) override { on(); kern::bu_cut_merge(a, st_); chk(); }
  void direct_prewait(const DirectExchange& x) override { on(); kern::direct_prewait(x, st_); chk(); }
  void hub_visited(const HubVisitedArgs& a) override { on(); kern::hub_visited(a, st_); chk(); }
  void unvis_filter(const UnvisArgs& a) override { on(); kern::unvis_filter(a, st_); chk(); }
  void hub_apply(const HubApplyArgs& a) override { on(); kern::hub_apply(a, st_); chk(); }
  void refresh_visited(const RefreshArgs& a) override { on(); kern::refresh_visited(a, st_); chk(); }
  void status_expand(const StatusArgs& a) override { on(); kern::status_expand(a, st_); chk(); }
  void bitmap_or(word_t* d, const word_t* s, int64_t w) override { on(); kern::bitmap_or(d, s, w, st_); chk(); }
  void ref_expand(const RefExpandArgs& a) override { on(); kern::ref_expand(a, st_); chk(); }
  void ref_accept(const RefAcceptArgs& a) override { on(); kern::ref_accept(a, st_); chk(); }
  void scan_relax(const ScanBfsArgs& a) override { on(); kern::scan_relax(a, st_); chk(); }
  void scan_count(const ScanBfsArgs& a) override { on(); kern::scan_count(a, st_); chk(); }
  void scan_bounds(const ScanBfsArgs& a) override { on(); kern::scan_bounds(a, st_); chk(); }
  void scan_assign(const ScanBfsArgs& a) override { on(); kern::scan_assign(a, st_); chk(); }
  void validate_levels(const ValidateArgs& a) override { on(); kern::validate_levels(a, st_); chk(); }
  void compute_parents(const ParentArgs& a) override { on(); kern::compute_parents(a, st_); chk(); }
  void degrees_u32(const eid_t* ro, int64_t rows, uint32_t* out) override {
    on();
    kern::degrees_u32(ro, rows, out, st_);
    chk();
  }
  void row_heads(const eid_t* ro, const vid_t* col, int64_t rows, vid_t* head, const uint32_t* hub_idx) override {
    on();
    kern::row_heads(ro, col, rows, head, hub_idx, st_);
    chk();
  }

  void encode_hub_cols(const vid_t* col, int64_t nnz, const uint32_t* hub_idx, vid_t* out) override {
    on();
    kern::encode_hub_cols(col, nnz, hub_idx, out, st_);
    chk();
  }
  void nz_word_counts(const eid_t* ro, int64_t rows, int64_t words, eid_t* counts) override {
    on();
    kern::nz_word_counts(ro, rows, words, counts, st_);
    chk();
  }
  void nz_records(const eid_t* ro, const vid_t* head, int64_t rows, const eid_t* pref, NzRec* rec,
                  eid_t* unit_base) override {
    on();
    kern::nz_records(ro, head, rows, div_up(rows, kWordBits), pref, rec, unit_base, st_);
    chk();
  }
  void nz_fill(const eid_t* ro, const vid_t* head, int64_t rows, const eid_t* pref, eid_t* nz_ro,
               vid_t* nz_head) override {
    on();
    kern::nz_fill(ro, head, rows, div_up(rows, kWordBits), pref, nz_ro, nz_head, st_);
    chk();
  }
  int64_t select_hubs(const uint32_t* deg, int64_t n, uint32_t min_deg, vid_t* hub_vertex,
                      uint32_t* hub_idx) override {
    on();
    // indices in vertex order (identical on every rank): per-word counts,
    // exclusive scan, assignment
    const int64_t words = div_up(std::max<int64_t>(n, 1), kWordBits);
    eid_t* cnt = nullptr;
    HIP_CHECK(hipMalloc(&cnt, static_cast<size_t>(words + 1) * sizeof(eid_t)));
    HIP_CHECK(hipMemsetAsync(cnt, 0, static_cast<size_t>(words + 1) * sizeof(eid_t), st_));
    kern::hub_count(deg, n, min_deg, cnt, st_);
    chk();
    exclusive_scan(cnt, words);
    kern::hub_assign(deg, n, min_deg, cnt, hub_vertex, hub_idx, st_);
    chk();
    eid_t h = 0;
    HIP_CHECK(hipMemcpyAsync(&h, cnt + words, sizeof(h), hipMemcpyDeviceToHost, st_));
    HIP_CHECK(hipStreamSynchronize(st_));
    release_(cnt);
    return static_cast<int64_t>(h);
  }
  void sort_neighbors(const eid_t* ro, vid_t* col, int64_t rows, const uint32_t* key_deg) override {
    on();
    int64_t* list = nullptr;
    unsigned long long* count = nullptr;
    HIP_CHECK(hipMalloc(&list, static_cast<size_t>(std::max<int64_t>(rows, 1)) * sizeof(int64_t)));
    HIP_CHECK(hipMalloc(&count, sizeof(unsigned long long)));
    kern::sort_neighbors(ro, col, rows, key_deg, list, count, st_);
    chk();
    HIP_CHECK(hipStreamSynchronize(st_));
    release_(list);
    release_(count);
  }

  void sort_rows_by_id(const eid_t* ro, vid_t* col, int64_t rows, int64_t n) override {
    on();
    eid_t nnz = 0;
    HIP_CHECK(hipMemcpyAsync(&nnz, ro + rows, sizeof(nnz), hipMemcpyDeviceToHost, st_));
    HIP_CHECK(hipStreamSynchronize(st_));
    int64_t* list = nullptr;
    unsigned long long* count = nullptr;
    vid_t* tmp = nullptr;
    HIP_CHECK(hipMalloc(&list, static_cast<size_t>(std::max<int64_t>(rows, 1)) * sizeof(int64_t)));
    HIP_CHECK(hipMalloc(&count, sizeof(unsigned long long)));
    HIP_CHECK(hipMalloc(&tmp, static_cast<size_t>(std::max<eid_t>(nnz, 1)) * sizeof(vid_t)));
    kern::sort_rows_by_id(ro, col, rows, n, list, count, tmp, st_);
    chk();
    HIP_CHECK(hipStreamSynchronize(st_));
    release_(list);
    release_(count);
    release_(tmp);
  }

  void gen_count_degrees(const GenParams& p, int64_t lo, int64_t rows, eid_t* deg) override {
    on();
    kern::gen_count_degrees(p, lo, rows, deg, st_);
    chk();
  }
  void exclusive_scan(eid_t* data, int64_t n) override {
    on();
    const size_t need = static_cast<size_t>(kern::scan_tmp_elems(n));
    if (need > scan_tmp_n_) {
      HIP_CHECK(hipStreamSynchronize(st_));
      if (scan_tmp_) release_(scan_tmp_);
      HIP_CHECK(hipMalloc(&scan_tmp_, need * sizeof(eid_t)));
      scan_tmp_n_ = need;
    }
    kern::exclusive_scan(data, n, scan_tmp_, st_);
    chk();
  }
  void route_edges_count(const vid_t* u, const vid_t* v, int64_t m, int64_t part, int nranks,
                         int64_t* counts) override {
    DBFS_CHECK(nranks <= kern::route_max_ranks(), "edge routing supports at most 1024 ranks");
    kern::route_edges_count(u, v, m, part, nranks, counts, st_);
    HIP_CHECK(hipGetLastError());
  }
  void route_edges_fill(const vid_t* u, const vid_t* v, int64_t m, int64_t part, int nranks, int64_t* cursor,
                        uint64_t* out) override {
    DBFS_CHECK(nranks <= kern::route_max_ranks(), "edge routing supports at most 1024 ranks");
    kern::route_edges_fill(u, v, m, part, nranks, cursor, out, st_);
    HIP_CHECK(hipGetLastError());
  }
  void entries_count(const uint64_t* e, int64_t k, int64_t lo, eid_t* deg) override {
    kern::entries_count(e, k, lo, deg, st_);
    HIP_CHECK(hipGetLastError());
  }
  void entries_fill(const uint64_t* e, int64_t k, int64_t lo, eid_t* cursor, vid_t* col) override {
    kern::entries_fill(e, k, lo, cursor, col, st_);
    HIP_CHECK(hipGetLastError());
  }
  void gen_fill(const GenParams& p, int64_t lo, int64_t rows, eid_t* cursor, vid_t* col) override {
    on();
    kern::gen_fill(p, lo, rows, cursor, col, st_);
    chk();
  }
  void degree_moments(const ShardView& g, int64_t* out2) override {
    on();
    HIP_CHECK(hipMemsetAsync(out2, 0, 2 * sizeof(int64_t), st_));
    kern::degree_moments(g, out2, st_);
    chk();
  }
  void reached_degree_sum(const ShardView& g, const lvl_t* level, int64_t* out2) override {
    on();
    HIP_CHECK(hipMemsetAsync(out2, 0, 2 * sizeof(int64_t), st_));
    kern::reached_degree_sum(g, level, out2, st_);
    chk();
  }

 private:
  // Other libraries (RCCL init, user code) may change the calling thread's
  // current device, so it is re-asserted on every call (a TLS write).
  void on() { HIP_CHECK(hipSetDevice(dev_)); }
  static void chk() { HIP_CHECK(hipGetLastError()); }

  static constexpr size_t kPinned = 4096;
  int dev_;
  void* pinned_ = nullptr;
  hipStream_t st_ = nullptr;
  // communication side stream (fork_side / join_side)
  hipStream_t side_ = nullptr;
  hipEvent_t fork_ev_ = nullptr, join_ev_ = nullptr;
  bool forked_ = false;
  std::string arch_;
  int cus_ = 0;
  double clock_khz_ = 0.0;
  std::vector<hipEvent_t> events_;
  size_t ev_used_ = 0;
  eid_t* scan_tmp_ = nullptr;
  size_t scan_tmp_n_ = 0;
  bool defer_ = false;
  std::vector<void*> deferred_, deferred_host_;
};

}  // namespace

std::unique_ptr<Backend> make_hip_backend(int device) { return std::make_unique<HipBackend>(device); }

int hip_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

}  // namespace dbfs
