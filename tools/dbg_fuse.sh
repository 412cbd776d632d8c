export DBFS_DEVICE=0 DBFS_COMM=peer DBFS_PEER_SLOT_MB=4 DBFS_COMM_TIMEOUT_S=20
run() { name=$1; shift; timeout -k 10 100 python bench.py --gpus 2 --scale 18 --steps 2 --warmup 1 --no-int32-pass --no-validate "$@" > gpurun_out/dbg_$name.json 2> gpurun_out/dbg_$name.err; echo "$name rc=$?"; grep -E "host timing|Error" gpurun_out/dbg_$name.err | head -6 | cut -c1-400; }
run nofuse --opt xfuse_edges=0
DBFS_DBG_NO_FUSE=1 run capnofuse
DBFS_HOST_TIMING=1 run fuse
