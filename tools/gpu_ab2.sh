#!/bin/bash
# A/B of the working library against libtropical_hip_base.so (the previous
# commit's sources, tools: see session notes): parity first, then 128^3
# bench lines alternating, then the bunny-scale profile of both
# usage: tools/gpu_ab2.sh <tag> [pytest files...]
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
tag=$1; shift
tests=${@:-tests/test_gpu_parity.py tests/test_gpu_curve.py tests/test_gpu_multi_rank.py tests/test_ops.py}
run() { "$@" || { echo "step failed ($?): $*"; exit 1; }; }
run timeout -k 10 600 python -u -m pytest $tests -x -v -m gpu --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1
for k in 1 2; do
  for v in libtropical_hip.so libtropical_hip_base.so; do
    TNP_LIB=$v run timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/${tag}_$v.json 2>/dev/null
    echo "$k $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${tag}_$v.json) $(grep -o '"kernel_ms_per_pass": {[^}]*}' gpurun_out/${tag}_$v.json)" >> gpurun_out/${tag}_ab.txt
  done
done
for v in libtropical_hip.so libtropical_hip_base.so; do
  TNP_LIB=$v run timeout -k 10 200 python -u tools/small_profile.py 20 flat > gpurun_out/${tag}_small_$v.log 2>&1
done
