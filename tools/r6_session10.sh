#!/bin/bash
# round 6, session 10: steps of <= 8,192 connecting-edge keys sorted by one
# workgroup in LDS (sort.hip k_sort_small): the GPU suite, bunny-scale
# profiles against rocPRIM's merge sort (TNP_SORT_RUN=0 there), the 128^3
# pass against the build before the two-stage sort (r06h)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/ab.err gpurun_out/r6j_small_ab.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6j_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r6j_tests.log; exit 1; }
tail -1 gpurun_out/r6j_tests.log
for r in 1 2 3; do
  for v in new:1 rocprim:0; do
    tag=${v%%:*}; env=${v#*:}
    [ "$env" = 1 ] && e="" || e="TNP_SORT_RUN=0"
    echo "== $tag round $r" >> gpurun_out/r6j_small_ab.log
    timeout -k 10 300 env $e python -u tools/small_profile.py >> gpurun_out/r6j_small_ab.log 2>&1 || { echo small $tag failed; exit 1; }
  done
done
bash tools/ab_session.sh 2 new=libtropical_hip.so h=libtropical_hip_r06h.so || exit 1
echo done
