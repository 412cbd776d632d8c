# Round-6 step: calibrate the shadow replay against real ranks -- the same roots traversed by
# P real processes sharing device 0 over the peer transport, and replayed rank by rank.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r6cal}; P=${P:-2}
ROOTS=${ROOTS:-8766153 17872028 13702079 43129764}
DBFS_DEVICE=0 DBFS_COMM=peer DBFS_COMM_TIMEOUT_S=120 timeout -k 10 600 python3 -u tools/real_ranks_levels.py --ranks $P --root-list $ROOTS --out gpurun_out/${T}_real > gpurun_out/${T}_real.log 2>&1 || { tail -20 gpurun_out/${T}_real.log; exit 1; }
timeout -k 10 600 python3 -u tools/shadow_rank.py --ranks-of $P --ranks $(seq 0 $((P - 1))) --root-list $ROOTS --json gpurun_out/${T}_shadow.json > gpurun_out/${T}_shadow.txt 2>&1 || { tail -20 gpurun_out/${T}_shadow.txt; exit 1; }
python3 - gpurun_out/${T} $P <<'PY'
import json, sys
t, P = sys.argv[1], int(sys.argv[2])
sh = json.load(open(f"{t}_shadow.json"))
real = [json.load(open(f"{t}_real_r{r}.json")) for r in range(P)]
print(f"# real ranks ({real[0]['comm']}, P = {P}, sharing one GPU) against their shadow replays: device-clock us per level, rank by rank")
for i, root in enumerate(sh["roots"]):
    print(f"\nroot {root}")
    print("lvl dir  frontier edges  " + "  ".join(f"real r{r} replay r{r}" for r in range(P)))
    rl = [real[r]["roots"][str(root)]["levels"] for r in range(P)]
    sl = {s["rank"]: s["levels"][i] for s in sh["ranks"]}
    n = max(len(x) for x in rl)
    tot = [[0.0, 0.0] for _ in range(P)]
    for L in range(n):
        d, _, mf = rl[0][L] if L < len(rl[0]) else ("-", 0, 0)
        row = f"{L:3d} {d:>3} {mf:15,d} "
        for r in range(P):
            a = rl[r][L][1] * 1e3 if L < len(rl[r]) else 0.0
            b = sl[r][L][1] * 1e3 if L < len(sl[r]) else 0.0
            tot[r][0] += a; tot[r][1] += b
            row += f"  {a:8.1f} {b:9.1f}"
        print(row)
    print("sum " + " " * 20 + "".join(f"  {a:8.1f} {b:9.1f}" for a, b in tot))
PY
