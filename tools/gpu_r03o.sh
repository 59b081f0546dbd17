#!/bin/bash
# packed bucket-group A/B: parity tests with every step packed, bench lines
# and per-step profiles never packed / packed below 16 entries per bucket
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
TNP_BG_PACK=100000000 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi_rank.py tests/test_gpu_curve.py -x -q -m gpu \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03o2_tests.log 2>&1 \
  || { echo "tests failed"; tail -15 gpurun_out/r03o2_tests.log; exit 1; }
tail -2 gpurun_out/r03o2_tests.log
for k in 1 2; do
  for v in 0 16; do
    TNP_BG_PACK=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/r03o2_$v.json 2>/dev/null || { echo "bench failed"; exit 1; }
    echo "$k $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r03o2_$v.json) $(grep -o '"kernel_ms_per_pass": {[^}]*}' gpurun_out/r03o2_$v.json)" >> gpurun_out/r03o2_ab.txt
  done
done
for v in 0 16; do
  TNP_BG_PACK=$v timeout -k 10 200 python -u tools/step_profile.py 128 6 > gpurun_out/r03o2_steps_$v.log 2>&1 || { echo "step profile failed"; exit 1; }
done
cat gpurun_out/r03o2_ab.txt
