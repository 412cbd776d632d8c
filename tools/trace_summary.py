#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV as a per-kernel timeline.

Prints the last --last kernels (default: everything after the final
fill_level_kernel launch before the end, i.e. the last BFS) with their
duration and the idle gap since the previous kernel ended, so per-level host
round trips and launch gaps are visible.

Usage: python3 tools/trace_summary.py <kernel_trace.csv> [--last N] [--from-kernel NAME]
"""
import argparse
import csv
import re


def short(name: str) -> str:
    name = name.replace("dbfs::kern::(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "")
    return name[:60]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--from-kernel", default="fill_level_kernel",
                    help="start at the last launch of this kernel (a BFS run begins with it)")
    ap.add_argument("--runs", type=int, default=1, help="how many trailing runs to print")
    args = ap.parse_args()
    rows = []
    with open(args.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    if args.last:
        sel = rows[-args.last:]
    else:
        starts = [i for i, r in enumerate(rows) if args.from_kernel in r[2]]
        i0 = starts[-args.runs] if len(starts) >= args.runs else 0
        sel = rows[i0:]
    t_first = sel[0][0]
    prev_end = sel[0][0]
    busy = 0
    print(f"{'t_us':>9} {'gap_us':>8} {'dur_us':>8}  kernel")
    for s, e, n in sel:
        print(f"{(s - t_first) / 1e3:9.1f} {(s - prev_end) / 1e3:8.1f} {(e - s) / 1e3:8.1f}  {short(n)}")
        busy += e - s
        prev_end = max(prev_end, e)
    span = (prev_end - t_first) / 1e3
    print(f"span {span:.1f} us, kernels busy {busy / 1e3:.1f} us ({100 * busy / 1e3 / max(span, 1e-9):.0f}%)")


if __name__ == "__main__":
    main()
