#!/bin/bash
# GPU parity tests, then (only if they pass) a short bench; no retries.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -x -q -m gpu --timeout 200 -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench.log 2>&1
