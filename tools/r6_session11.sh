#!/bin/bash
# round 6, session 11: HIP API + kernel trace of the bunny-scale flat
# subpoly() (where the finish's host turnaround goes)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/small_hip -o run -- \
  python tools/small_profile.py 3 flat > gpurun_out/small_hip.log 2>&1 || { echo trace failed; tail -20 gpurun_out/small_hip.log; exit 1; }
ls gpurun_out/small_hip
echo done
