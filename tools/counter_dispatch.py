#!/usr/bin/env python3
"""Per-dispatch hardware counters of one kernel (rocprofv3 --pmc runs).

Joins counter_collection.csv (Dispatch_Id, Counter_Name, Counter_Value) with
kernel_trace.csv (durations) and prints the N longest dispatches of kernels
whose name contains --kernel, one row per dispatch, plus derived rates.
Usage: counter_dispatch.py --kernel bu_hub <run_dir> [<run_dir> ...]
(each run_dir holds one pass' *_counter_collection.csv and *_kernel_trace.csv;
dispatches are matched across passes by their rank in time order).
"""
import argparse
import collections
import csv
import glob
import os


def load(run_dir, kernel):
    cc = glob.glob(os.path.join(run_dir, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(run_dir, "**", "*kernel_trace.csv"), recursive=True)
    counters = collections.defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(cc[0])):
        d = int(r["Dispatch_Id"])
        counters[d][r["Counter_Name"]] = counters[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    dur = {}
    for r in csv.DictReader(open(kt[0])):
        d = int(r["Dispatch_Id"])
        dur[d] = (int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = [(dur[d][0], d, dur[d][1], counters[d], names[d]) for d in counters
            if kernel in names[d] and d in dur]
    rows.sort()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--top", type=int, default=6)
    ap.add_argument("--timeline", type=int, default=0,
                    help="instead: the last N dispatches in time order (GRBM_GUI_ACTIVE / duration = clock)")
    ap.add_argument("dirs", nargs="+")
    a = ap.parse_args()
    passes = [load(d, a.kernel) for d in a.dirs]
    if a.timeline:
        rows = passes[0][-a.timeline:]
        t0 = rows[0][0]
        for start, d, us, c, name in rows:
            mhz = c.get("GRBM_GUI_ACTIVE", 0) / us if us else 0
            extra = " ".join(f"{k}={v:.4g}" for k, v in sorted(c.items()) if k != "GRBM_GUI_ACTIVE")
            print(f"{(start - t0) / 1e3:9.1f} {us:7.1f} us {mhz:7.0f} MHz  {name.split('(')[0][-36:]:36s} {extra}")
        return
    n = min(len(p) for p in passes)
    merged = []
    for i in range(n):
        c = {}
        for p in passes:
            c.update(p[i][3])
        merged.append((passes[0][i][2], c))  # (start, id, us, counters, name)
    merged.sort(key=lambda x: -x[0])
    keys = sorted({k for _, c in merged for k in c})
    print("us".rjust(8), *[k[:16].rjust(16) for k in keys])
    for us, c in merged[: a.top]:
        print(f"{us:8.1f}", *[f"{c.get(k, 0):16.4g}" for k in keys])
        extra = []
        if c.get("FETCH_SIZE"):
            extra.append(f"HBM read {c['FETCH_SIZE'] / 1e3 / us:.2f} TB/s ({c['FETCH_SIZE'] / 1e3:.0f} MB)")
        if c.get("WRITE_SIZE"):
            extra.append(f"written {c['WRITE_SIZE'] / 1e3:.0f} MB")
        if c.get("SQ_WAVE_CYCLES"):
            extra.append(f"wait {100 * c.get('SQ_WAIT_ANY', 0) / c['SQ_WAVE_CYCLES']:.0f}% of wave-cycles")
            extra.append(f"active-inst {100 * c.get('SQ_ACTIVE_INST_ANY', 0) / c['SQ_WAVE_CYCLES']:.0f}%")
        if c.get("TCC_HIT_sum") is not None and c.get("TCC_MISS_sum"):
            extra.append(f"L2 hit {100 * c['TCC_HIT_sum'] / (c['TCC_HIT_sum'] + c['TCC_MISS_sum']):.0f}%")
        if c.get("TCP_TCC_READ_REQ_sum"):
            extra.append(f"L2 read req {c['TCP_TCC_READ_REQ_sum'] / us / 1e3:.1f} G/s")
        if c.get("SQ_INSTS_VMEM_RD"):
            extra.append(f"vmem-rd wave-insts {c['SQ_INSTS_VMEM_RD'] / us / 1e3:.2f} G/s")
        print("         " + "; ".join(extra))


if __name__ == "__main__":
    main()
