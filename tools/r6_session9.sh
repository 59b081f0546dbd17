#!/bin/bash
# round 6, session 9: the live flags of a step with few members zeroed by
# one fill dispatch (bucket.hip, TNP_LIVE_FILL): the GPU suite, A/B against
# the count kernel's zeroing (TNP_LIVE_FILL=0) and the round's final build
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/ab.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6i_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r6i_tests.log; exit 1; }
tail -1 gpurun_out/r6i_tests.log
bash tools/ab_session.sh 3 new=libtropical_hip.so nolf=libtropical_hip.so:TNP_LIVE_FILL=0 h=libtropical_hip_r06h.so || exit 1
timeout -k 10 300 python -u tools/step_profile.py 128 6 > gpurun_out/r6i_step_profile128.log 2>&1 || { echo sp failed; exit 1; }
TNP_LIVE_FILL=0 timeout -k 10 300 python -u tools/step_profile.py 128 6 > gpurun_out/r6i_step_profile128_nolf.log 2>&1 || { echo sp failed; exit 1; }
echo done
