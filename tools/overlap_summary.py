#!/usr/bin/env python3
"""Compute/communication overlap in a rocprofv3 kernel trace of one rank.

For every bottom-up head pass (bu_head_kernel) and every collective kernel
(peer_push / peer_wait / peer_unpack of the peer-memory communicator, or RCCL
kernels) on another HIP stream of the same process, prints how long they ran
at the same time, plus a short timeline around the first few head passes.

Usage: python3 tools/overlap_summary.py <kernel_trace.csv> [--timeline N]
"""
import argparse
import csv
import re


def short(name: str) -> str:
    name = name.replace("dbfs::kern::(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", name).replace("void ", "")[:44]


def is_comm(name: str) -> bool:
    return "peer_" in name or "nccl" in name.lower() or "rccl" in name.lower()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--timeline", type=int, default=2, help="head passes to show with their neighbourhood")
    args = ap.parse_args()
    ks = []
    with open(args.csv) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                       int(r.get("Stream_Id") or 0), int(r.get("Queue_Id") or 0)))
    ks.sort()
    heads = [k for k in ks if "bu_head_kernel" in k[2]]
    comm = [k for k in ks if is_comm(k[2])]
    tot_head = tot_ovl = 0
    for h in heads:
        ovl = sum(max(0, min(h[1], c[1]) - max(h[0], c[0])) for c in comm if c[3] != h[3])
        tot_head += h[1] - h[0]
        tot_ovl += min(ovl, h[1] - h[0])
    print(f"head passes {len(heads)}, collective kernels {len(comm)}")
    if heads:
        print(f"head-pass time {tot_head / 1e3:.1f} us, of which overlapped with collectives on another stream "
              f"{tot_ovl / 1e3:.1f} us ({100.0 * tot_ovl / max(tot_head, 1):.0f}%)")
    for h in heads[-args.timeline:]:
        t0 = h[0]
        near = [k for k in ks if k[1] >= h[0] - 40000 and k[0] <= h[1] + 40000]
        print(f"\n-- around a head pass (t = 0 at its start; stream, start us, end us, kernel)")
        for k in near:
            print(f"   s{k[3]:<3} {(k[0] - t0) / 1e3:9.1f} {(k[1] - t0) / 1e3:9.1f}  {short(k[2])}")


if __name__ == "__main__":
    main()
