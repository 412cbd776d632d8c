#!/bin/bash
# Byte-map top-down repeats (tools/byte_map_repeat.py) while a second process
# (the headline bench) keeps the GPU busy: workgroup scheduling shifts under
# contention, which is where a timing-dependent wrong level would show.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${BG_LIMIT:-240} python -u bench.py --steps 400 --warmup 2 --heldout-roots 0 --secondary none --no-int32-pass \
  > gpurun_out/stress_bg.json 2> gpurun_out/stress_bg.err &
bg=$!
sleep ${BG_DELAY:-25}
: > gpurun_out/stress.txt
rc=0
for cfg in "1 td 1" "1 td 0" "1 td 2" "1 do 1" "3 td 1" "3 do 2"; do
  set -- $cfg
  timeout -k 10 120 python -u tools/byte_map_repeat.py . ${REPS:-40} $1 $2 $3 > gpurun_out/stress_cfg.txt 2>&1
  rc=$?
  cat gpurun_out/stress_cfg.txt >> gpurun_out/stress.txt
  [ $rc -eq 0 ] || break
done
wait $bg
echo "bench rc $?" >> gpurun_out/stress.txt
exit $rc
