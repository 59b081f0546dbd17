#!/bin/bash
# forward_new timing experiments (shadow launches, tools/build_lv_variant.sh
# -DTNP_FWD_SHADOW) and the grouping kernel's phase clocks (-DTNP_BG_PHASES=1)
set -u
export TMPDIR=/tmp TNP_LIB_ANY_BUILD=1
mkdir -p gpurun_out
out=gpurun_out/exp_fwd.jsonl
: > $out
TNP_LIB=libtropical_hip.so timeout -k 10 120 python tools/kernel_ms.py 128 6 base >> $out || exit 1
for m in 0 1 3 5 9 17 33 29 61; do
  TNP_LIB=libtropical_hip_shadow.so TNP_FWD_SHADOW=$m timeout -k 10 120 python tools/kernel_ms.py 128 6 shadow$m >> $out || exit 1
done
TNP_LIB=libtropical_hip_phases.so timeout -k 10 120 python tools/kernel_ms.py 128 6 phases >> $out 2> gpurun_out/phases.err || exit 1
