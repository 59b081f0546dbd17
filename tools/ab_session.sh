#!/bin/bash
# A/B of library variants on the 128^3 seed-6 pass (tools/kernel_ms.py, HIP
# events per engine launch, median of 5 passes), alternating runs:
#   bash tools/ab_session.sh <rounds> <tag=lib[:ENV=val...]> ...
# e.g. bash tools/ab_session.sh 3 new=libtropical_hip.so old=libtropical_hip_r05.so
# Variants built from other sources load with TNP_LIB_ANY_BUILD=1.
# Output: gpurun_out/ab.jsonl (one line per run)
set -u
export TMPDIR=/tmp TNP_LIB_ANY_BUILD=1
mkdir -p gpurun_out
out=gpurun_out/ab.jsonl
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
  for spec in "$@"; do
    tag=${spec%%=*}; rest=${spec#*=}
    IFS=: read -r lib envs <<< "$rest"
    env_args=()
    if [ -n "${envs:-}" ]; then IFS=, read -ra env_args <<< "$envs"; fi
    timeout -k 10 150 env TNP_LIB="$lib" "${env_args[@]}" python tools/kernel_ms.py 128 6 "$tag" >> $out \
      2>> gpurun_out/ab.err || { echo "run $tag failed rc=$?"; exit 1; }
    echo "round $r $tag done"
  done
done
