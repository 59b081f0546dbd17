#!/bin/bash
# round 3: net-shape generalisation on the GPU (parity + curve suites), then
# the whole suite and the smoke entry
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_curve.py -x -v --timeout 120 \
  --timeout-method thread -m gpu > gpurun_out/r03b_parity.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r03b_gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03b_smoke.log 2>&1
