#!/bin/bash
# round 6, session 7: wave-merged LDS bin adds in the member passes
# (bucket.hip merged_add), the 256-thread k_publish_sums and the two-stage
# key sort (sort.hip sort_keys_lex, TNP_SORT_RUN): the GPU suite on the new
# build, A/B against the round's final build (r06h) and the 0- / 1-round
# merge variants, then a kernel trace of the bunny-scale runs
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/ab.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6g_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r6g_tests.log; exit 1; }
tail -1 gpurun_out/r6g_tests.log
bash tools/ab_session.sh 3 agg2=libtropical_hip.so h=libtropical_hip_r06h.so lex32=libtropical_hip.so:TNP_SORT_RUN=32 \
  agg0=libtropical_hip_agg0.so agg1=libtropical_hip_agg1.so || exit 1
timeout -k 10 300 python -u tools/step_profile.py 128 6 > gpurun_out/r6g_step_profile128.log 2>&1 || { echo sp failed; exit 1; }
timeout -k 10 300 python -u tools/small_profile.py > gpurun_out/r6g_small_profile.log 2>&1 || { echo small failed; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/small_trace -o run -- python tools/small_profile.py \
  > gpurun_out/small_trace.log 2>&1 || { echo small trace failed; exit 1; }
echo done
