#!/bin/bash
# A/B of library variants: kernel ms at 128^3 and the bunny-scale profile
set -u
export TMPDIR=/tmp TNP_LIB_ANY_BUILD=1
mkdir -p gpurun_out
for v in "$@"; do
  TNP_LIB=$v timeout -k 10 120 python tools/kernel_ms.py 128 6 $v >> gpurun_out/ab_kms.jsonl || exit 1
  TNP_LIB=$v timeout -k 10 120 python tools/small_profile.py 20 flat > gpurun_out/ab_small_$v.log 2>&1 || exit 1
done
