#!/bin/bash
# round 3 (session 2): HEAD validation -- whole GPU suite, smoke, bench, phase clocks
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
run() { "$@" || { echo "step failed ($?): $*"; exit 1; }; }
run timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r03h_gpu_tests.log 2>&1
run timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03h_smoke.log 2>&1
run timeout -k 10 300 python -u bench.py > gpurun_out/r03h_bench.json 2>gpurun_out/r03h_bench.err
TNP_LIB=libtropical_hip_phases.so run timeout -k 10 200 python -u tools/step_profile.py 128 6 \
  > gpurun_out/r03h_phases.log 2>&1
run timeout -k 10 200 python -u tools/small_profile.py 20 flat > gpurun_out/r03h_small.log 2>&1
