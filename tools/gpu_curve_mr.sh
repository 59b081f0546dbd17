#!/bin/bash
# the sharded curve branch: its new multi-rank tests, then the curve and
# multi-rank suites and the parity set
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi_rank.py -k curve -x -v -m gpu --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r03q_curve_mr.log 2>&1 || { tail -40 gpurun_out/r03q_curve_mr.log; exit 1; }
tail -1 gpurun_out/r03q_curve_mr.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi_rank.py tests/test_gpu_curve.py tests/test_gpu_parity.py tests/test_ops.py \
  -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03q_tests.log 2>&1 || { tail -30 gpurun_out/r03q_tests.log; exit 1; }
tail -1 gpurun_out/r03q_tests.log
