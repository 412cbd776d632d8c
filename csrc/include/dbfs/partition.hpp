// 1D block vertex partition (owner-computes).
//
// Reference: getDev / in-kernel `v / part` (bfs.cu:29-32,148,585) uses
// part = N / P, which sends the tail vertices of N % P != 0 to a non-existent
// owner P.  Here `part` is ceil(N / P) rounded up to a
// whole bitmap word (64 vertices), so every vertex has an owner in [0, P) and
// every rank's slice of a global bitmap is a whole number of words -- the
// per-level all-to-all / all-gather of bitmap slices are then equal-sized
// collectives (RCCL ncclAllToAll / ncclAllGather) with no count exchange.
#pragma once

#include <algorithm>
#include "dbfs/common.hpp"

namespace dbfs {

struct Partition {
  int nranks = 1;
  int64_t n = 0;     // global vertex count
  int64_t part = 0;  // vertices per rank (multiple of 64), last rank may hold fewer

  static Partition block(int64_t n, int nranks) {
    DBFS_CHECK(nranks >= 1, "nranks must be >= 1");
    DBFS_CHECK(n >= 0, "negative vertex count");
    Partition p;
    p.nranks = nranks;
    p.n = n;
    p.part = std::max<int64_t>(kWordBits, round_up(div_up(std::max<int64_t>(n, 1), nranks), kWordBits));
    return p;
  }

  int owner(int64_t v) const { return static_cast<int>(v / part); }
  int64_t lo(int r) const { return std::min<int64_t>(n, static_cast<int64_t>(r) * part); }
  int64_t hi(int r) const { return std::min<int64_t>(n, static_cast<int64_t>(r + 1) * part); }
  int64_t count(int r) const { return hi(r) - lo(r); }
  // Words of one rank's bitmap slice (identical for every rank).
  int64_t slice_words() const { return part / kWordBits; }
  // Words of the padded global bitmap (nranks * slice_words).
  int64_t global_words() const { return static_cast<int64_t>(nranks) * slice_words(); }
};

}  // namespace dbfs
