#!/bin/bash
# round 3: two-batch window tests + thresholded parallel window builder
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
run() { "$@" || { echo "step failed ($?): $*"; exit 1; }; }
run timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_curve.py -x -v \
  --timeout 300 --timeout-method thread -m gpu > gpurun_out/r03g_parity.log 2>&1
for k in 1 2; do
  run timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/r03g_bench_$k.json 2>&1
  echo "$k $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r03g_bench_$k.json) $(grep -o '"kernel_ms_per_pass": {[^}]*}' gpurun_out/r03g_bench_$k.json)" >> gpurun_out/r03g_ab.txt
done
TNP_LIB=libtropical_hip_phases.so run timeout -k 10 200 python -u tools/step_profile.py 128 6 \
  > gpurun_out/r03g_phases.log 2>&1
run timeout -k 10 200 python -u tools/small_profile.py 20 flat > gpurun_out/r03g_small.log 2>&1
