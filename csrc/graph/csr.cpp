// Host CSR construction and the sequential BFS oracle.
//
// build_csr reproduces the reference's adjacency order (bfs.cu:851-872:
// adj[u] += v; adj[v] += u per input edge, flattened in vertex order) with a
// stable two-pass counting sort instead of vector<vector<int>>.
// cpu_bfs is the oracle of bfs.cu:923-945 (std::queue BFS).
#include <algorithm>
#include <vector>

#include "dbfs/graph.hpp"

namespace dbfs {

HostCSR build_csr(const EdgeList& el, bool directed) {
  HostCSR g;
  g.n = el.n;
  g.row_lo = 0;
  g.rows = el.n;
  g.input_edges = el.m();
  g.row_off.assign(static_cast<size_t>(el.n + 1), 0);
  const int64_t m = el.m();
  for (int64_t i = 0; i < m; ++i) {
    ++g.row_off[el.u[i] + 1];
    if (!directed) ++g.row_off[el.v[i] + 1];
  }
  for (int64_t r = 0; r < el.n; ++r) g.row_off[r + 1] += g.row_off[r];
  g.col.resize(static_cast<size_t>(g.row_off[el.n]));
  std::vector<eid_t> cur(g.row_off.begin(), g.row_off.end() - 1);
  for (int64_t i = 0; i < m; ++i) {
    const vid_t a = el.u[i], b = el.v[i];
    g.col[cur[a]++] = b;
    if (!directed) g.col[cur[b]++] = a;
  }
  return g;
}

HostCSR slice_rows(const HostCSR& full, int64_t lo, int64_t hi) {
  DBFS_CHECK(full.row_lo == 0 && full.rows == full.n, "slice_rows expects a full CSR");
  DBFS_CHECK(0 <= lo && lo <= hi && hi <= full.n, "bad row range");
  HostCSR s;
  s.n = full.n;
  s.row_lo = lo;
  s.rows = hi - lo;
  s.input_edges = full.input_edges;
  s.row_off.resize(static_cast<size_t>(s.rows + 1));
  const eid_t base = full.row_off[lo];
  for (int64_t r = 0; r <= s.rows; ++r) s.row_off[r] = full.row_off[lo + r] - base;
  s.col.assign(full.col.begin() + base, full.col.begin() + full.row_off[hi]);
  return s;
}

CpuBfsResult cpu_bfs(const HostCSR& g, int64_t src) {
  DBFS_CHECK(g.row_lo == 0 && g.rows == g.n, "cpu_bfs expects a full CSR");
  DBFS_CHECK(src >= 0 && src < g.n, "source vertex out of range");
  CpuBfsResult r;
  r.level.assign(static_cast<size_t>(g.n), kUnreached);
  r.parent_edge.assign(static_cast<size_t>(g.n), -1);
  std::vector<vid_t> q;
  q.reserve(1024);
  q.push_back(static_cast<vid_t>(src));
  r.level[src] = 0;
  size_t head = 0;
  while (head < q.size()) {
    const vid_t u = q[head++];
    const lvl_t lu = r.level[u];
    for (eid_t e = g.row_off[u]; e < g.row_off[u + 1]; ++e) {
      const vid_t v = g.col[e];
      if (r.level[v] == kUnreached) {
        r.level[v] = lu + 1;
        r.parent_edge[v] = e;
        q.push_back(v);
      }
    }
  }
  return r;
}

int64_t traversed_edges(const HostCSR& g, const std::vector<lvl_t>& level) {
  int64_t s = 0;
  for (int64_t r = 0; r < g.rows; ++r)
    if (level[g.row_lo + r] != kUnreached) s += g.degree(r);
  return s / 2;
}

}  // namespace dbfs
