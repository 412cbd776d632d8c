#!/bin/bash
# Hub-cut bound sweep (per-root level times of the late-switch roots) and a
# kernel timeline of two of them with the cut on.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q -m gpu -k "hub_cut or long_row or hub_lds" --timeout 200 --timeout-method thread > gpurun_out/cut_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/cut_pytest.log; [ $rc -eq 0 ] || exit $rc
ARGSETS="${ARGSETS}" ROOTS=20 STEPS=20 bash tools/gpu_ab_levels_args.sh > gpurun_out/cut_sweep.txt || { cat gpurun_out/cut_sweep.txt; exit 1; }
grep -E "GTEPS| (8766153|17872028|21909223|22823737|5467067|31770031|26246917|38084502) " gpurun_out/cut_sweep.txt
ROOTS="17872028 5467067 26246917" RUNS=3 bash tools/gpu_trace_roots.sh > gpurun_out/cut_trace.txt 2>&1 || { tail -30 gpurun_out/cut_trace.txt; exit 1; }
grep -E "bu_|hub_|ms|root" gpurun_out/cut_trace.txt | head -80
