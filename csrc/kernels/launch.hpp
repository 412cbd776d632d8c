// Host-side launchers of the gfx950 kernels (defined in csrc/kernels/*.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "dbfs/backend.hpp"

namespace dbfs {
namespace kern {

// bfs_kernels.hip, td_kernels.hip, bu_kernels.hip
void fill_level(lvl_t* level, int64_t n, lvl_t value, hipStream_t st);
// zero `bytes` at p with 16-B stores (false: p or bytes not 16-B aligned)
bool zero_fill(void* p, size_t bytes, hipStream_t st);
void set_bit(word_t* bm, int64_t bit, hipStream_t st);
void level_ctrl_init(LevelCtrl* c, const LevelCtrl& init, hipStream_t st);
void publish_stats(const int64_t* stats, StatsMailbox* mb, int64_t seq, hipStream_t st);
void init_run(const InitRunArgs& a, hipStream_t st);
void update_frontier(const UpdateArgs& a, hipStream_t st);
void scan_units(const ScanArgs& a, hipStream_t st);
void zero_degree_mask(const ZeroDegArgs& a, hipStream_t st);
void compact_frontier(const CompactArgs& a, hipStream_t st);
void td_expand(const TdArgs& a, hipStream_t st);
void td_sparse(const TdSparseArgs& a, hipStream_t st);
void td_sparse_apply(const TdSparseArgs& a, hipStream_t st);
// A direct exchange's wait as a one-wave launch (Comm::split_waits).
void direct_prewait(const DirectExchange& x, hipStream_t st);
// PeerComm::self_test of the direct exchanges (`round` 0..3; mismatches and
// timeouts counted in *err)
void direct_selftest(const DirectExchange& lists, const DirectExchange& end, int round, unsigned* err,
                     unsigned* ticket, hipStream_t st);
// PeerComm::self_test of the pushed frontier slices: phase 0 pushes `words`
// known words of this rank's slice, phase 1 (after a barrier) checks every
// peer's (mismatches counted in *err)
void frontier_selftest(const FrontierTable* t, int rank, int nranks, int64_t words, int round, int phase,
                       unsigned* err, hipStream_t st);
void td_binned(const BinArgs& a, hipStream_t st);
void level_finish(const LevelFinishArgs& a, hipStream_t st);
void widen_levels(const uint8_t* in, lvl_t* out, int64_t n, uint8_t base, hipStream_t st);
void pack_bytes(const PackArgs& a, hipStream_t st);
void list_scatter(const ListScatterArgs& a, hipStream_t st);
void bu_step(const BuArgs& a, hipStream_t st);
void hub_gather(const HubGatherArgs& a, hipStream_t st);
void bu_cut_prep(const BuArgs& a, hipStream_t st);
void bu_cut_merge(const BuArgs& a, hipStream_t st);
void hub_visited(const HubVisitedArgs& a, hipStream_t st);
void unvis_filter(const UnvisArgs& a, hipStream_t st);
void hub_apply(const HubApplyArgs& a, hipStream_t st);
void refresh_visited(const RefreshArgs& a, hipStream_t st);
// device-checked build (DBFS_CHECKED): whether checks are compiled in, the
// first recorded violation (code << 48 | detail, 0: none; cleared), and a
// test hook recording code 99
bool checks_enabled();
unsigned long long take_check_error();
void inject_check_failure(hipStream_t st);
void status_expand(const StatusArgs& a, hipStream_t st);
void bitmap_or(word_t* dst, const word_t* src, int64_t words, hipStream_t st);
void copy_pieces(const Backend::CopyPieces& c, hipStream_t st);

// peer_kernels.hip (PeerComm: collectives through peer-mapped windows)
constexpr int kMaxPeers = 16;
struct PeerPushArgs {
  // segment 0 of the piece for peer p: src[p] -> dst[p] (a peer's window slot,
  // or a local buffer for this rank's own piece)
  void* dst[kMaxPeers] = {};
  const void* src[kMaxPeers] = {};
  int64_t bytes[kMaxPeers] = {};    // (counted: the most it may be)
  // counted segment 0 (owner lists): its length is read on the device -- the
  // 32-bit word count[p] holds n, the piece is its n + 1 words (count first),
  // rounded up to `unit`, at most bytes[p]
  const uint32_t* count[kMaxPeers] = {};
  // segment 1 (the all-reduce input, the same for every peer): src2 -> dst2[p]
  void* dst2[kMaxPeers] = {};
  const void* src2 = nullptr;
  int64_t bytes2 = 0;
  uint64_t* flag[kMaxPeers] = {};   // flag word this rank owns in each peer's window (nullptr: none)
  int npeers = 0;
  int unit = 4;                     // copy granule (4, 8, 16 B; every size and address a multiple)
  uint64_t seq = 0;
  unsigned* ticket = nullptr;       // zero on entry; reset by the last workgroup
  // the fused launch's workgroups per peer at most (0: kPeerFusedGroups) --
  // ranks sharing a GPU with the in-kernel waits (PeerComm::coresident)
  int max_groups = 0;
};
struct PeerWaitArgs {
  const uint64_t* flags = nullptr;  // this rank's window: one word per sender
  int npeers = 0;
  int skip = -1;                    // sender not waited for (this rank, when it sent itself nothing)
  uint64_t seq = 0;
  uint64_t timeout_ticks = 0;       // device wall-clock ticks
  uint64_t* error = nullptr;        // host-mapped: set to seq on a timeout
};
struct PeerUnpackArgs {
  void* dst[kMaxPeers] = {};
  const void* src[kMaxPeers] = {};
  int64_t bytes[kMaxPeers] = {};
  bool counted = false;             // segment 0 counted (its first word holds n; n + 1 words, <= bytes[p])
  int npeers = 0;
  int unit = 4;
  int64_t sum_count = 0;            // > 0: all-reduce -- sum_out[i] = sum_p sum_src[p][i] (uint64, wrapping)
  const void* sum_src[kMaxPeers] = {};
  void* sum_out = nullptr;
  // then a level's end on the sums (sum_count <= kPeerFinishMax: the first
  // workgroup sums everything, then finishes the level: level_finish_block)
  bool has_finish = false;
  LevelFinishArgs finish;
  // the wait's error word (split collectives: the unpack is a launch of its
  // own, stream-ordered after the wait whatever its outcome): non-zero -- a
  // wait of this rank timed out -- and the unpack copies nothing and the
  // level is not finished on payloads that never arrived
  const uint64_t* error = nullptr;
};
constexpr int64_t kPeerFinishMax = 2048;
void peer_push(const PeerPushArgs& a, hipStream_t st);
void peer_wait(const PeerWaitArgs& a, hipStream_t st);
void peer_unpack(const PeerUnpackArgs& a, hipStream_t st);
// A collective as ONE launch (push, flags, wait, unpack fused) instead of
// three; up to kPeerFusedGroups workgroups per peer.
constexpr int64_t kPeerFusedGroups = 32;
void peer_fused(const PeerPushArgs& push, const PeerWaitArgs& wait, const PeerUnpackArgs& unpack, hipStream_t st);

// ref_kernels.hip (reference-algorithm mode)
void ref_expand(const RefExpandArgs& a, hipStream_t st);
void ref_accept(const RefAcceptArgs& a, hipStream_t st);
void scan_relax(const ScanBfsArgs& a, hipStream_t st);
void scan_count(const ScanBfsArgs& a, hipStream_t st);
void scan_bounds(const ScanBfsArgs& a, hipStream_t st);
void scan_assign(const ScanBfsArgs& a, hipStream_t st);

// graph_kernels.hip
void gen_count_degrees(const GenParams& p, int64_t lo, int64_t rows, eid_t* deg, hipStream_t st);
void gen_fill(const GenParams& p, int64_t lo, int64_t rows, eid_t* cursor, vid_t* col, hipStream_t st);
// CSR build from file edges: per-destination entry counts (counts[nranks],
// added to), the entries scattered by destination (cursor[r] = segment start,
// advanced), then the owner's row degrees (added to) and the row fill.
void route_edges_count(const vid_t* u, const vid_t* v, int64_t m, int64_t part, int nranks, int64_t* counts,
                       hipStream_t st);
void route_edges_fill(const vid_t* u, const vid_t* v, int64_t m, int64_t part, int nranks, int64_t* cursor,
                      uint64_t* out, hipStream_t st);
void entries_count(const uint64_t* e, int64_t k, int64_t lo, eid_t* deg, hipStream_t st);
void entries_fill(const uint64_t* e, int64_t k, int64_t lo, eid_t* cursor, vid_t* col, hipStream_t st);
int route_max_ranks();
// in-place exclusive scan of n + 1 entries; `tmp` must hold scan_tmp_elems(n) entries
int64_t scan_tmp_elems(int64_t n);
void exclusive_scan(eid_t* data, int64_t n, eid_t* tmp, hipStream_t st);
void validate_levels(const ValidateArgs& a, hipStream_t st);
void compute_parents(const ParentArgs& a, hipStream_t st);

// graph_sort.hip
void degrees_u32(const eid_t* row_off, int64_t rows, uint32_t* out, hipStream_t st);
void row_heads(const eid_t* row_off, const vid_t* col, int64_t rows, vid_t* head, const uint32_t* hub_idx,
               hipStream_t st);
void encode_hub_cols(const vid_t* col, int64_t nnz, const uint32_t* hub_idx, vid_t* out, hipStream_t st);
void nz_word_counts(const eid_t* row_off, int64_t rows, int64_t words, eid_t* counts, hipStream_t st);
void nz_records(const eid_t* row_off, const vid_t* head, int64_t rows, int64_t words, const eid_t* nz_pref,
                NzRec* rec, eid_t* unit_base, hipStream_t st);
void nz_fill(const eid_t* row_off, const vid_t* head, int64_t rows, int64_t words, const eid_t* nz_pref,
             eid_t* nz_row_off, vid_t* nz_head, hipStream_t st);
// hub selection: cnt[w] = hubs among vertices [64 w, 64 w + 64) (ceil(n / 64)
// entries); after an exclusive scan of cnt, hub index = hubs with a smaller id
void hub_count(const uint32_t* deg, int64_t n, uint32_t min_deg, eid_t* cnt, hipStream_t st);
void hub_assign(const uint32_t* deg, int64_t n, uint32_t min_deg, const eid_t* cnt, vid_t* hub_vertex,
                uint32_t* hub_idx, hipStream_t st);
// list must hold `rows` entries; count is one device counter
void sort_neighbors(const eid_t* row_off, vid_t* col, int64_t rows, const uint32_t* key_deg, int64_t* list,
                    unsigned long long* count, hipStream_t st);
// rows in id order (rows of 2..4096 exactly, longer rows by 4096 id buckets);
// tmp holds nnz entries
void sort_rows_by_id(const eid_t* row_off, vid_t* col, int64_t rows, int64_t n, int64_t* list,
                     unsigned long long* count, vid_t* tmp, hipStream_t st);
void reached_degree_sum(const ShardView& g, const lvl_t* level, int64_t* out2, hipStream_t st);
void degree_moments(const ShardView& g, int64_t* out2, hipStream_t st);

}  // namespace kern
}  // namespace dbfs
