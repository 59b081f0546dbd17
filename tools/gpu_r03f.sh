#!/bin/bash
# round 3: workgroup-parallel window lists -- parity, A/B against the serial
# builder, per-phase clocks
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
run() { "$@" || { echo "step failed ($?): $*"; exit 1; }; }
run timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_curve.py -x -v \
  --timeout 300 --timeout-method thread -m gpu > gpurun_out/r03f_parity.log 2>&1
for v in libtropical_hip.so libtropical_hip_serialwin.so libtropical_hip.so libtropical_hip_serialwin.so; do
  TNP_LIB=$v run timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/r03f_ab_$v.json 2>&1
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r03f_ab_$v.json) $(grep -o '"kernel_ms_per_pass": {[^}]*}' gpurun_out/r03f_ab_$v.json)" >> gpurun_out/r03f_ab.txt
done
TNP_LIB=libtropical_hip_phases.so run timeout -k 10 200 python -u tools/step_profile.py 128 6 \
  > gpurun_out/r03f_phases.log 2>&1
run timeout -k 10 200 python -u tools/small_profile.py 20 flat > gpurun_out/r03f_small.log 2>&1
