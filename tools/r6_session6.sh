#!/bin/bash
# round-6 GPU session 6: the software-pipelined lazy prune -- the -m gpu
# suite, A/B against the unpipelined variant (TNP_LZ_PREFETCH=0).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/ab.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6f_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r6f_tests.log; exit 1; }
tail -1 gpurun_out/r6f_tests.log
bash tools/ab_session.sh 3 pf=libtropical_hip.so nopf=libtropical_hip_nopf.so || exit 1
echo done
