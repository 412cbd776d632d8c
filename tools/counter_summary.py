#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --pmc CSV (counter_collection.csv).

Sums every counter over the dispatches of each kernel and prints the mean per
dispatch, plus derived ratios where the inputs are present:
  wait%     SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on memory / barriers)
  l2hit%    TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
Usage: python3 tools/counter_summary.py <counter_collection.csv> [...more csv]
"""
import collections
import csv
import re
import sys


def short(name: str) -> str:
    name = name.replace("dbfs::kern::(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", name).replace("void ", "")[:48]


def main() -> None:
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for path in sys.argv[1:]:
        with open(path) as f:
            for r in csv.DictReader(f):
                k = short(r["Kernel_Name"])
                sums[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add((path, r.get("Dispatch_Id") or r.get("Correlation_Id")))
    names = sorted({c for d in sums.values() for c in d})
    print("kernel".ljust(48), "disp", *[c[:14].rjust(14) for c in names], "wait%".rjust(7), "l2hit%".rjust(7))
    for k in sorted(sums, key=lambda k: -sum(sums[k].values())):
        n = max(1, len(disp[k]) // max(1, len(sys.argv) - 1))
        d = sums[k]
        wait = 100 * d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"] if d.get("SQ_WAVE_CYCLES") else float("nan")
        hits = d.get("TCC_HIT_sum", 0.0)
        miss = d.get("TCC_MISS_sum", 0.0)
        l2 = 100 * hits / (hits + miss) if hits + miss else float("nan")
        print(k.ljust(48), str(n).rjust(4), *[f"{d.get(c, 0.0) / n:14.4g}" for c in names], f"{wait:7.1f}", f"{l2:7.1f}")


if __name__ == "__main__":
    main()
