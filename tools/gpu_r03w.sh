#!/bin/bash
# every GPU test on the current build, then the key-buffer A/B (WKEYS 448)
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r03w_tests.log 2>&1 || { echo "tests failed"; tail -15 gpurun_out/r03w_tests.log; exit 1; }
tail -1 gpurun_out/r03w_tests.log
for k in 1 2; do
  for v in libtropical_hip.so libtropical_hip_wk448.so; do
    TNP_LIB=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/r03w_$v.json 2>/dev/null || { echo "bench failed"; exit 1; }
    echo "$k $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r03w_$v.json) $(grep -o '"kernel_ms_per_pass": {[^}]*}' gpurun_out/r03w_$v.json)" >> gpurun_out/r03w_ab.txt
  done
done
cat gpurun_out/r03w_ab.txt
