#!/bin/bash
# round 3 (session 2): default bench (progress on stderr), phase clocks, bunny profile
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
run() { "$@" || { echo "step failed ($?): $*"; exit 1; }; }
run timeout -k 10 400 python -u bench.py > gpurun_out/r03i_bench.json 2>gpurun_out/r03i_bench.err
TNP_LIB=libtropical_hip_phases.so run timeout -k 10 200 python -u tools/step_profile.py 128 6 \
  > gpurun_out/r03i_phases.log 2>&1
run timeout -k 10 200 python -u tools/small_profile.py 20 flat > gpurun_out/r03i_small.log 2>&1
