// Host-side graph containers, readers and CSR construction.
//
// Reference: struct Graph (bfs.cu:21-28) keeps three int32 vectors (adjacency,
// per-vertex offset, per-vertex degree).  Here the host CSR is the standard
// (n+1)-offset form with int64 offsets and uint32 column ids.  Adjacency order
// matches the reference reader exactly: for input edge (u, v) in file order, v
// is appended to adj(u) and u to adj(v) (bfs.cu:851-863); duplicates and
// self-loops are kept (a self-loop appears twice), numEdges = 2m (bfs.cu:875).
#pragma once

#include <string>
#include <vector>

#include "dbfs/common.hpp"

namespace dbfs {

// Undirected input edge list (u[i], v[i]) over vertices [0, n).
struct EdgeList {
  int64_t n = 0;
  std::vector<vid_t> u, v;
  int64_t m() const { return static_cast<int64_t>(u.size()); }
};

// Symmetrised CSR (rows [row_lo, row_lo + rows) of an n-vertex graph).
struct HostCSR {
  int64_t n = 0;          // global vertex count
  int64_t row_lo = 0;     // first row held (0 for a full graph)
  int64_t rows = 0;       // rows held
  std::vector<eid_t> row_off;  // rows + 1
  std::vector<vid_t> col;      // row_off[rows]
  int64_t input_edges = 0;     // undirected edges of the input (m)
  int64_t directed_edges() const { return static_cast<int64_t>(col.size()); }
  eid_t degree(int64_t local_row) const { return row_off[local_row + 1] - row_off[local_row]; }
};

enum class FileFormat { Auto, EdgeList, MatrixMarket, Binary };

struct ReadOptions {
  FileFormat format = FileFormat::Auto;
  bool verbose_reference_lines = false;  // print the reference's load lines
};

// Reference-format `n m` + m lines `u v` (0-based), or MatrixMarket
// (%%MatrixMarket header, % comments, 1-based, optional value column), or the
// binary CSR cache (see write_binary_csr).  Throws dbfs::Error on failure.
// path "-" reads the reference format (or MatrixMarket) from standard input.
EdgeList read_edge_list(const std::string& path, const ReadOptions& opt = {});
FileFormat detect_format(const std::string& path);

// Build a symmetrised CSR in reference adjacency order (stable counting sort).
// directed: u -> v entries only -- the reference's stdin reader `readGraph`
// (bfs.cu:882-920, dead there: main calls readGraphFromFile) reads the pairs as
// directed edges without symmetrising.
HostCSR build_csr(const EdgeList& el, bool directed = false);
// Rows [lo, hi) of a full CSR (shard extraction; column ids stay global).
HostCSR slice_rows(const HostCSR& full, int64_t lo, int64_t hi);

// Binary CSR cache: header {magic, version, n, rows, nnz, input_edges, checksum}
// then row_off (int64) and col (uint32).  SURVEY §5.4.
// Version 2 adds per-block checksums (row offsets and columns) so that a rank
// maps and verifies only its own rows; every read checks the header ranges,
// the offsets' monotonicity and span, and that column ids are < n.
void write_binary_csr(const std::string& path, const HostCSR& g);
HostCSR read_binary_csr(const std::string& path);
struct BinaryCsrInfo {
  int version = 0;
  int64_t n = 0, row_lo = 0, rows = 0, nnz = 0, input_edges = 0;
};
BinaryCsrInfo binary_csr_info(const std::string& path);
// Global rows [lo, hi) of the cache (a shard: row_lo = lo, rebased offsets).
HostCSR read_binary_csr_rows(const std::string& path, int64_t lo, int64_t hi);
bool is_binary_csr(const std::string& path);

// Reference-format edge list of a synthetic graph (generator edges in order),
// formatted by `threads` host threads (0: all cores).  Test / benchmark inputs
// for the file readers at scale (no dataset can be downloaded on the pool).
struct GenParams;
void write_generated_edge_list(const std::string& path, const GenParams& p, int threads = 0);

// Write per-vertex levels, one per line, 2147483647 for unreached.
void write_levels(const std::string& path, const std::vector<lvl_t>& levels);

// Sequential BFS oracle (bfs.cu:923-945): exact levels; parent[v] = index into
// col of the edge that discovered v (the reference's edge-index convention),
// parent[src] = -1.
struct CpuBfsResult {
  std::vector<lvl_t> level;
  std::vector<eid_t> parent_edge;
};
CpuBfsResult cpu_bfs(const HostCSR& g, int64_t src);

// Traversed undirected edges (Graph500 convention): sum of degrees over
// reached vertices / 2.
int64_t traversed_edges(const HostCSR& g, const std::vector<lvl_t>& level);

}  // namespace dbfs
