"""Debug: the long-row star graph of test_bottom_up_long_row_scanned_in_place_gpu
with the hub cut on / off, 16-word / whole-unit bottom-up waves."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_cuda_bfs_amd as dbfs
from distributed_cuda_bfs_amd.parallel.runtime import init_runtime
rt = init_runtime(sys.argv[1] if len(sys.argv) > 1 else "hip")
p = dbfs.rmat_params(16, 16, 9)
u0, v0 = (np.asarray(x, dtype=np.int64) for x in dbfs.generate_edges(p))
n0 = p.n; k = 1 << 21; c = n0
leaves = np.arange(n0 + 1, n0 + 1 + k, dtype=np.int64)
partners = n0 + 1 + ((leaves - n0 - 1) ^ 1); partners[-1] = 5; partners[-2] = n0 + 1 + k
keep = (leaves < partners) | (np.arange(k) >= k - 2)
u = np.concatenate([u0, np.full(k, c), leaves[keep]]); v = np.concatenate([v0, leaves, partners[keep]])
n = n0 + 2 + k
csr = dbfs.build_csr(n, u.astype(np.uint32), v.astype(np.uint32))
bfs = dbfs.BFS(csr, rt, mode="bu")
res = bfs.run(0); exp, _ = dbfs.cpu_bfs(csr, 0); got = bfs.levels()
ro = np.asarray(csr.row_off); col = np.asarray(csr.col); deg = np.diff(ro)
miss = np.nonzero((exp == 1) & (got != 1))[0]
print("missed", miss.tolist(), "hub threshold: nhubs", bfs.graph.nhubs, "deg>=3:", int((deg >= 3).sum()))
for v in miss[:3]:
    nb = col[ro[v]:ro[v + 1]]
    print(v, "deg", deg[v], "nbrs(deg)", sorted([(int(deg[x]), int(x)) for x in nb], reverse=True)[:20])
