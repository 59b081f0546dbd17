#!/bin/bash
# round 3: single-wave small buckets -- parity, then bunny-scale and 128^3
# profiles with and without (libtropical_hip_nosmall.so)
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
run() { "$@" || { echo "step failed ($?): $*"; exit 1; }; }
run timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_curve.py tests/test_gpu_multi_rank.py -x -v \
  --timeout 300 --timeout-method thread -m gpu > gpurun_out/r03e_parity.log 2>&1
for v in libtropical_hip.so libtropical_hip_nosmall.so; do
  TNP_LIB=$v run timeout -k 10 200 python -u tools/small_profile.py 20 > gpurun_out/r03e_small_$v.log 2>&1
done
run timeout -k 10 200 python -u tools/step_profile.py 128 6 > gpurun_out/r03e_step_profile.log 2>&1
