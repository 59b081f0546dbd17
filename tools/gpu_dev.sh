#!/bin/bash
# Development loop on one GPU box: parity tests (stop on failure), then the
# per-step profile and a short bench.  Each GPU step under its own limit.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/dev_tests.log 2>&1 || { tail -30 gpurun_out/dev_tests.log; exit 1; }
tail -3 gpurun_out/dev_tests.log
timeout -k 10 200 python tools/step_profile.py 128 6 > gpurun_out/dev_sp.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/dev_bench.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/dev_bench.log
