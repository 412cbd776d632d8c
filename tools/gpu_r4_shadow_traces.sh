#!/bin/bash
# Round 4: kernel timelines of rank 0 of 8 replayed (tools/gpu_shadow_trace.sh)
# for one root per variant: "tag:root:opt=v,opt=v|..." (default: an early-switch
# and a late-switch root, new defaults against hub-split + multi-rank cut off).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
IFS='|' read -ra CS <<< "${CASES:-new13:13702079:|old13:13702079:hx_levels=0,bu_cut_ranks=0|new87:8766153:|old87:8766153:hx_levels=0,bu_cut_ranks=0}"
for c in "${CS[@]}"; do
  IFS=':' read -r tag root opts <<< "$c"
  sa="--root-list $root"
  if [ -n "$opts" ]; then IFS=',' read -ra kvs <<< "$opts"; for kv in "${kvs[@]}"; do sa="$sa --opt $kv"; done; fi
  echo "== $tag $root $opts"
  TAG=${TAG:-r4}_$tag SHADOW_ARGS="$sa" bash tools/gpu_shadow_trace.sh || exit 1
done
