// Sharded edge-list reading (see csrc/graph/shard_reader.cpp).
#pragma once

#include <functional>
#include <string>
#include <vector>

#include "dbfs/graph.hpp"

namespace dbfs {

// This rank's edges of a reference-format or MatrixMarket edge list: rank r
// parses bytes [byte_begin, byte_end) (cut at token / line boundaries) and the
// one token after it that completes its last edge.  Edges keep file order;
// first_edge is the global index of u[0].
struct EdgeShard {
  int64_t n = 0;           // vertices (header)
  int64_t m = 0;           // edges of the whole file (header)
  int64_t first_edge = 0;
  std::vector<vid_t> u, v;
  int64_t byte_begin = 0, byte_end = 0;
  FileFormat format = FileFormat::EdgeList;
  int64_t local_edges() const { return static_cast<int64_t>(u.size()); }
};

// One host value from every rank, in rank order (Comm::allgather_host_i64).
using HostAllgather = std::function<std::vector<int64_t>(int64_t)>;

// Every rank calls this collectively (the allgather agrees on token counts and
// errors: all ranks throw the same dbfs::Error).  threads = 0: up to 16.
EdgeShard read_edge_shard(const std::string& path, int rank, int nranks, const HostAllgather& allgather,
                          int threads = 0);

}  // namespace dbfs
