"""Repeat the byte-map top-down check (tests/test_gpu_engine.py::
test_td_byte_map_mode_gpu) REPS times against the package of one tree, and
print every mismatch (root, first differing vertex, got / expected levels)
instead of stopping at the first: tells a deterministic wrong level from a
timing-dependent one, and one build from another.

  python tools/byte_map_repeat.py [TREE] [REPS] [P] [mode] [knobs: 0/1/2]
"""
import os
import sys

tree = sys.argv[1] if len(sys.argv) > 1 else "."
sys.path.insert(0, tree)
import numpy as np  # noqa: E402

import distributed_cuda_bfs_amd as dbfs  # noqa: E402
from distributed_cuda_bfs_amd.parallel.runtime import run_virtual_ranks  # noqa: E402

reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
P = int(sys.argv[3]) if len(sys.argv) > 3 else 1
mode = sys.argv[4] if len(sys.argv) > 4 else "td"
knob_sets = [{}, {"td_check_visited_min": 2.0, "td_wide_below_blocks": 1 << 30},
             {"td_check_visited_min": 0.0, "td_wide_below_blocks": 0}]
knobs = knob_sets[int(sys.argv[5]) if len(sys.argv) > 5 else 1]
print("package", dbfs.__file__, "P", P, mode, knobs, flush=True)

p = dbfs.rmat_params(16, 16, 29)
csr = dbfs.host_csr_from_params(p)
srcs = [0, 5, 40000]
exp = [dbfs.cpu_bfs(csr, s)[0] for s in srcs]


def body(rt):
    bfs = dbfs.BFS(p, rt, mode=mode)
    bfs.engine.set_heuristics(24.0, 24.0, 8, td_byte_edges=0)
    for k, v in knobs.items():
        bfs.engine.set_option(k, v)
    out = []
    for _ in range(reps):
        for s in srcs:
            r = bfs.run(s)
            out.append((s, bfs.levels(), [tuple(c) for c in r.chains]))
    return out


bad = 0
for rank, rank_out in enumerate(run_virtual_ranks(P, body, device=os.environ.get("BMR_DEVICE", "hip"))):
    for i, (s, lv, ch) in enumerate(rank_out):
        e = exp[srcs.index(s)]
        if not np.array_equal(lv, e):
            bad += 1
            d = np.nonzero(lv != e)[0]
            print(f"rank {rank} run {i // len(srcs)} root {s}: {len(d)} wrong, first {d[:5].tolist()} "
                  f"got {lv[d[:5]].tolist()} exp {e[d[:5]].tolist()} chains {ch}", flush=True)
print(f"{bad} wrong of {P * reps * len(srcs)}", flush=True)
