#!/bin/bash
# A/B of one run-time switch: bench lines with VAR=a and VAR=b alternating
# usage: tools/gpu_env_ab.sh <tag> <VAR> <a> <b> [pytest files...]
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
tag=$1; var=$2; va=$3; vb=$4; shift 4
run() { "$@" || { echo "step failed ($?): $*"; exit 1; }; }
if [ $# -gt 0 ]; then
  env $var=$vb timeout -k 10 600 python -u -m pytest "$@" -x -v -m gpu --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1 || { echo "tests failed"; tail -5 gpurun_out/${tag}_tests.log; exit 1; }
fi
for k in 1 2; do
  for v in $va $vb; do
    env $var=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/${tag}_$v.json 2>/dev/null || { echo "bench failed"; exit 1; }
    echo "$k $var=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${tag}_$v.json) $(grep -o '"kernel_ms_per_pass": {[^}]*}' gpurun_out/${tag}_$v.json)" >> gpurun_out/${tag}_ab.txt
  done
done
