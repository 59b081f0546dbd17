#!/bin/bash
# A/B bench of in-tree library variants (TNP_LIB=<name> under tropical/_lib/):
#   bash tools/ab_bench.sh libtropical_hip.so libvariant.so ...
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  TNP_LIB=$v timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/ab_$v.log 2>&1 || exit 1
done
