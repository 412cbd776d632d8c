#!/bin/bash
# Counters of chosen roots under a compile-time variant (a copy of the tree
# built with EXTRA_HIPFLAGS):  FLAGS="-DDBFS_X" ROOTS="..." tools/gpu_counters_variant.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
d=/tmp/cv_tree
rm -rf $d && mkdir -p $d && tar -C "$ROOT" --exclude=./gpurun_out --exclude=./build-asan -cf - . | tar -C $d -xf -
(cd $d && make clean > /dev/null && make -j16 EXTRA_HIPFLAGS="$FLAGS" > $ROOT/gpurun_out/cv_make.log 2>&1) || { tail -20 gpurun_out/cv_make.log; exit 1; }
cd $d && GRAFT_REPO_ROOT=$d bash tools/gpu_counters_roots.sh > $ROOT/gpurun_out/cv.log 2>&1; rc=$?
cp $d/gpurun_out/counters_roots.txt $ROOT/gpurun_out/counters_variant.txt 2>/dev/null
exit $rc
