#!/bin/bash
# What the round-end driver runs: smoke(), then bench.py with no flags.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/drv_bench.json 2> gpurun_out/drv_bench.err || { tail -20 gpurun_out/drv_bench.err; exit 1; }
tail -1 gpurun_out/drv_bench.json | cut -c1-600
