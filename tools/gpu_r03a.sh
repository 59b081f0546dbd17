#!/bin/bash
# round 3, first GPU session: the whole -m gpu suite, then one bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r03a_gpu_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --cpu-marks 48 > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err
