#!/bin/bash
# round 6, session 8: the two-stage key sort on by default (TNP_SORT_RUN=32)
# and the wave-merged bin adds in the one-workgroup member pass: the GPU
# suite, A/B against the round's final build (r06h) and run lengths 16 / 64,
# bunny-scale profiles of the new build, r06h and the unmerged variant (sbm0)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/ab.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6h_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r6h_tests.log; exit 1; }
tail -1 gpurun_out/r6h_tests.log
bash tools/ab_session.sh 3 new=libtropical_hip.so h=libtropical_hip_r06h.so run16=libtropical_hip.so:TNP_SORT_RUN=16 \
  run64=libtropical_hip.so:TNP_SORT_RUN=64 || exit 1
for r in 1 2; do
  for v in new=libtropical_hip.so h=libtropical_hip_r06h.so sbm0=libtropical_hip_sbm0.so; do
    tag=${v%%=*}; lib=${v#*=}
    echo "== $tag round $r" >> gpurun_out/r6h_small_ab.log
    timeout -k 10 300 env TNP_LIB=$lib TNP_LIB_ANY_BUILD=1 python -u tools/small_profile.py >> gpurun_out/r6h_small_ab.log 2>&1 \
      || { echo small $tag failed; exit 1; }
  done
done
timeout -k 10 300 python -u tools/step_profile.py 128 6 > gpurun_out/r6h_step_profile128.log 2>&1 || { echo sp failed; exit 1; }
echo done
