#!/bin/bash
# round-6 GPU session 4: the side-stream prune -- the -m gpu suite, A/B
# against the prune on the caller's stream (TNP_SIDE_PRUNE=0), step profile.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/ab.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6e_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r6e_tests.log; exit 1; }
tail -1 gpurun_out/r6e_tests.log
bash tools/ab_session.sh 3 side=libtropical_hip.so noside=libtropical_hip.so:TNP_SIDE_PRUNE=0 || exit 1
timeout -k 10 300 python -u tools/step_profile.py 128 6 > gpurun_out/r6e_step_profile128.log 2>&1 || { echo sp failed; exit 1; }
echo done
