#!/bin/bash
# lazy-prune grid cap A/B (TNP_PL_BLOCKS): parity tests at the largest cap,
# bench lines at 1024 / 2048 / 4096 workgroups
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
TNP_PL_BLOCKS=4096 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi_rank.py -x -q -m gpu \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03t_tests.log 2>&1 \
  || { echo "tests failed"; tail -15 gpurun_out/r03t_tests.log; exit 1; }
tail -1 gpurun_out/r03t_tests.log
for k in 1 2; do
  for v in 1024 2048 4096; do
    TNP_PL_BLOCKS=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/r03t_$v.json 2>/dev/null || { echo "bench failed"; exit 1; }
    echo "$k $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r03t_$v.json) $(grep -o '"kernel_ms_per_pass": {[^}]*}' gpurun_out/r03t_$v.json)" >> gpurun_out/r03t_ab.txt
  done
done
cat gpurun_out/r03t_ab.txt
