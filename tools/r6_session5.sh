#!/bin/bash
# round-6 GPU session 5: forward_new shadow timings -- the real kernel (64)
# against the same kernel with an arithmetic stand-in for the marks search
# of the grid word (192), alternating; the shadow launch's own HIP-event
# time is printed at exit (net_lv.hip TNP_FWD_SHADOW).
set -u
export TMPDIR=/tmp TNP_LIB_ANY_BUILD=1
mkdir -p gpurun_out
out=gpurun_out/r6_shadow.txt
: > $out
for r in 1 2 3; do
  for m in 64 192; do
    TNP_LIB=libtropical_hip_shadow.so TNP_FWD_SHADOW=$m timeout -k 10 150 python tools/kernel_ms.py 128 6 shadow$m \
      >> $out 2>> gpurun_out/r6_shadow.err || { echo "shadow $m failed"; exit 1; }
    grep "fwd_shadow" gpurun_out/r6_shadow.err | tail -1
  done
done
echo done
