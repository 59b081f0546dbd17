#!/bin/bash
# Parity subset on the main library, then an A/B bench + per-step profile of
# library variants / settings:
#   bash tools/gpu_ab.sh libtropical_hip.so libtropical_hip_<v>.so libtropical_hip.so:TNP_X=1 ...
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_ops.py -m gpu -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
for arg in "$@"; do
  v=${arg%%:*}; envs=""; [ "$arg" != "$v" ] && envs=${arg#*:}
  tag=$(echo "$arg" | tr ':=' '__')
  env TNP_LIB=$v $envs timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/ab_$tag.log 2>&1 || exit 1
  echo "$arg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$tag.log) $(grep -o '"kernel_ms_per_pass": {[^}]*}' gpurun_out/ab_$tag.log)"
  env TNP_LIB=$v $envs timeout -k 10 200 python tools/step_profile.py 128 6 > gpurun_out/sp_$tag.log 2>&1 || exit 1
  grep total gpurun_out/sp_$tag.log
done
