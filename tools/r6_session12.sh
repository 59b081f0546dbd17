#!/bin/bash
# round 6, session 12: the run loop's last readback of a step zeroes the
# counter words (k_publish clear) and the next split skips its memset: the
# GPU suite, bunny-scale profiles and the 128^3 pass against the committed
# build (r06f)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/ab.err gpurun_out/r6k_small_ab.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6k_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r6k_tests.log; exit 1; }
tail -1 gpurun_out/r6k_tests.log
for r in 1 2 3; do
  for v in new=libtropical_hip.so r06f=libtropical_hip_r06f.so; do
    tag=${v%%=*}; lib=${v#*=}
    echo "== $tag round $r" >> gpurun_out/r6k_small_ab.log
    timeout -k 10 300 env TNP_LIB=$lib TNP_LIB_ANY_BUILD=1 python -u tools/small_profile.py >> gpurun_out/r6k_small_ab.log 2>&1 \
      || { echo small $tag failed; exit 1; }
  done
done
bash tools/ab_session.sh 2 new=libtropical_hip.so r06f=libtropical_hip_r06f.so || exit 1
echo done
