#!/usr/bin/env python3
"""Per-level communication table (docs/ARCHITECTURE.md §4) for a traversal
whose 1-GPU level profile is given, at several rank counts, from the model in
distributed_cuda_bfs_amd/utils/comm_model.py (checked against the
communicators' traffic counters by tests/test_comm_model.py).

  python3 tools/comm_table.py --scale 26 --levels T:5 T:547726 B:911126127 ...
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_cuda_bfs_amd.utils.comm_model import table  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--levels", nargs="+", required=True, help="DIR:FRONTIER_EDGES per level")
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--latency-us", type=float, default=10.0)
    ap.add_argument("--link-gbs", type=float, default=45.0)
    args = ap.parse_args()
    levels = [(x.split(":")[0], int(x.split(":")[1])) for x in args.levels]
    n = 1 << args.scale
    tabs = {P: table(levels, n, P, latency_us=args.latency_us, link_gbs=args.link_gbs) for P in args.ranks}
    hdr = "| level | dir | frontier edges | chain | collectives |" + "".join(
        f" MiB/rank P={P} |" for P in args.ranks) + f" est. µs P={args.ranks[-1]} |"
    print(hdr)
    print("|" + "---|" * (5 + len(args.ranks) + 1))
    last = tabs[args.ranks[-1]]
    tot = {P: 0.0 for P in args.ranks}
    for i, row in enumerate(last):
        kinds = " + ".join(f"{k}" if v == 1 else f"{v}x {k}" for k, v in sorted(row["kinds"].items()))
        cells = ""
        for P in args.ranks:
            r = tabs[P][i]
            cells += f" {r['mib_per_rank']:.3f} |"
            tot[P] += r["mib_per_rank"]
        fe = f"{row['frontier_edges']:,}" if row["dir"] != "-" else "(trailing chain)"
        print(f"| {row['level']} | {row['dir']} | {fe} | {row['form']} | {kinds} |{cells} {row['est_us']:.0f} |")
    est = sum(r["est_us"] for r in last)
    print(f"| total | | | | {sum(r['collectives'] for r in last)} |" + "".join(
        f" {tot[P]:.2f} |" for P in args.ranks) + f" {est:.0f} |")


if __name__ == "__main__":
    main()
