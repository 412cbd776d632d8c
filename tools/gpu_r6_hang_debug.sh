# Round-6 debug: the hung-rank peer test's three CLI ranks, outputs shown.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 0 1 2; do
  WORLD_SIZE=3 RANK=$r LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29710 DBFS_BOOTSTRAP_PORT=29711 DBFS_DEVICE=0 DBFS_COMM=peer \
  DBFS_PEER_SLOT_MB=4 DBFS_COMM_TIMEOUT_S=5 DBFS_FAULT_INJECT="rank=1,level=1,kind=hang" DBFS_HOST_TIMING=1 \
  timeout -k 5 40 ./bin/bfs --rmat 16 5 --no-oracle --json > gpurun_out/hang_$r.out 2> gpurun_out/hang_$r.err &
done
wait
for r in 0 1 2; do echo "== rank $r"; tail -c 1500 gpurun_out/hang_$r.err; grep -o '"depth":[0-9]*\|"levels":\[[^]]*\]' gpurun_out/hang_$r.out | head -c 600; echo; done
