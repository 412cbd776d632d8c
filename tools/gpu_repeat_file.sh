#!/bin/bash
# Run one GPU test file REPS times in fresh processes (a rare wrong result
# that needs the earlier tests' process state); stops at anything worse than
# a failed assertion (a fault, abort, time limit).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/repeat_file.txt
for r in $(seq 1 ${REPS:-3}); do
  kargs=(); [ -n "${KEXPR}" ] && kargs=(-k "${KEXPR}")
  timeout -k 10 ${LIMIT:-150} python -u -m pytest ${FILE:-tests/test_gpu_engine.py} -q -m gpu --timeout 120 --timeout-method thread "${kargs[@]}" ${PYARGS} \
    > gpurun_out/repeat_file_$r.log 2>&1
  rc=$?
  echo "run $r rc $rc: $(grep -E 'passed|failed' gpurun_out/repeat_file_$r.log | tail -n 1)" | tee -a gpurun_out/repeat_file.txt
  grep FAILED gpurun_out/repeat_file_$r.log | tee -a gpurun_out/repeat_file.txt
  [ $rc -le 1 ] || exit $rc
done
