#!/usr/bin/env python3
"""Per-kernel register use of a HIP source for gfx950 (hipcc's
kernel-resource-usage remarks): VGPRs, scratch bytes per lane, VGPR / SGPR
spills and occupancy, one line per kernel -- the check that a change kept a
latency-bound kernel at its register budget (the bottom-up hub kernels run at
<= 64 VGPRs, two 1024-thread workgroups per CU).

    python tools/kernel_regs.py csrc/kernels/bu_kernels.hip [--filter bu_hub_kernel] [--include DIR]
"""
import argparse
import os
import re
import subprocess
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("source")
    ap.add_argument("--filter", default="")
    ap.add_argument("--include", default=None, help="repo root (default: two levels above the source)")
    args = ap.parse_args()
    root = args.include or os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(args.source))))
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", f"-I{root}/csrc/include", f"-I{root}/csrc/kernels",
           "--offload-arch=gfx950", "-munsafe-fp-atomics", "-c", args.source, "-o", os.devnull,
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True)
    if out.returncode != 0:
        sys.stderr.write(out.stderr[-4000:])
        return out.returncode
    rows, cur = [], None
    for line in out.stderr.splitlines():
        m = re.search(r"remark:\s+(.*?):\s+(\S+)\s+\[-Rpass", line)
        if not m:
            continue
        key, val = m.group(1).strip(), m.group(2)
        if key == "Function Name":
            cur = {"name": val}
            rows.append(cur)
        elif cur is not None:
            cur[key] = val
    for r in rows:
        name = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip() or r["name"]
        if args.filter and args.filter not in name:
            continue
        print(f"VGPR {r.get('VGPRs', '?'):>3} scratch {r.get('ScratchSize [bytes/lane]', '?'):>3} "
              f"vspill {r.get('VGPRs Spill', '?'):>2} sspill {r.get('SGPRs Spill', '?'):>3} "
              f"occ {r.get('Occupancy [waves/SIMD]', '?'):>2}  {name}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
