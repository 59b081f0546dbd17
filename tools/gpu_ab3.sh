#!/bin/bash
# parity, then 128^3 bench lines of several library variants (TNP_LIB),
# then the bunny-scale profile of each and a kernel trace of the first
# usage: tools/gpu_ab3.sh <tag> <lib> [<lib>...]   (libs under tropical/_lib)
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
tag=$1; shift
libs="$@"
run() { "$@" || { echo "step failed ($?): $*"; exit 1; }; }
run timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_curve.py tests/test_gpu_multi_rank.py \
  tests/test_ops.py -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1
for k in 1 2; do
  for v in $libs; do
    TNP_LIB=$v run timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/${tag}_$v.json 2>/dev/null
    echo "$k $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${tag}_$v.json) $(grep -o '"kernel_ms_per_pass": {[^}]*}' gpurun_out/${tag}_$v.json)" >> gpurun_out/${tag}_ab.txt
  done
done
for v in $libs; do
  TNP_LIB=$v run timeout -k 10 200 python -u tools/small_profile.py 20 flat > gpurun_out/${tag}_small_$v.log 2>&1
done
first=$(echo $libs | cut -d' ' -f1)
cd /tmp && TNP_LIB=$first run timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof_small \
  -o small -- python3 $GRAFT_REPO_ROOT/tools/small_profile.py 5 flat > $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof_small.log 2>&1
