#!/bin/bash
# small-key sort A/B: parity tests on the one-workgroup sort, bunny-scale
# profiles and bench lines with it off (0) / on (default)
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi_rank.py tests/test_gpu_curve.py tests/test_ops.py -x -q -m gpu \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03p2_tests.log 2>&1 \
  || { echo "tests failed"; tail -15 gpurun_out/r03p2_tests.log; exit 1; }
tail -2 gpurun_out/r03p2_tests.log
for k in 1 2; do
  for v in 0 16384; do
    TNP_SORT_SMALL=$v timeout -k 10 200 python -u tools/small_profile.py 20 > gpurun_out/r03p2_small_$v.log 2>&1 || { echo "small failed"; exit 1; }
    echo "$k $v $(grep -o '"median_ms": {[^}]*}' gpurun_out/r03p2_small_$v.log | tr '\n' ' ')" >> gpurun_out/r03p2_ab.txt
  done
done
for v in 0 16384; do
  TNP_SORT_SMALL=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/r03p2_$v.json 2>/dev/null || { echo "bench failed"; exit 1; }
  echo "bench $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r03p2_$v.json) $(grep -o '"kernel_ms_per_pass": {[^}]*}' gpurun_out/r03p2_$v.json)" >> gpurun_out/r03p2_ab.txt
done
cat gpurun_out/r03p2_ab.txt
