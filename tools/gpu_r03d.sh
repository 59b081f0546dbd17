#!/bin/bash
# round 3: where k_bucket_group's time goes (per-phase shader-clock totals,
# diagnostic build) on the 128^3 headline pass
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
run() { "$@" || { echo "step failed ($?): $*"; exit 1; }; }
TNP_LIB=libtropical_hip_phases.so run timeout -k 10 200 python -u tools/step_profile.py 128 6 \
  > gpurun_out/r03d_phases.log 2>&1
