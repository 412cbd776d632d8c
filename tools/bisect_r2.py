import os, sys, numpy as np
sys.path.insert(0, "/root/repo")
import distributed_cuda_bfs_amd as dbfs
from distributed_cuda_bfs_amd.parallel.runtime import run_virtual_ranks, init_runtime
p = dbfs.rmat_params(13, 16, 11)
csr = dbfs.host_csr_from_params(p)
src = 5
exp, _ = dbfs.cpu_bfs(csr, src)
mode = os.environ.get("MODE", "do")
P = int(os.environ.get("P", "2"))
knobs = {"list_form_edges": 0}
def body(rt):
    b = dbfs.BFS(p, rt, mode=mode, force_exchange=True)
    for k, v in knobs.items():
        b.engine.set_option(k, v)
    r = b.run(src)
    return b.levels(), [(l["dir"], l["frontier"], l["discovered"]) for l in r.levels], r.mispredicts
if P == 1:
    outs = [body(init_runtime("hip"))]
else:
    outs = run_virtual_ranks(P, body, device="hip")
ok = all(np.array_equal(o[0], exp) for o in outs)
bad = np.nonzero(outs[0][0] != exp)[0]
print(P, mode, os.environ.get("DBFS_DEBUG_BU_HEAD", "1"), "OK" if ok else f"BAD {bad.size}", outs[0][1], outs[0][2], flush=True)
