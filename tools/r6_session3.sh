#!/bin/bash
# round-6 GPU session 3 (the round's build): smoke, the -m gpu suite, the
# rocprofv3 kernel trace + counter passes (MFMA counters included), the
# default bench line, per-step / bunny-scale / finish profiles.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6d_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r6d_smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6d_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r6d_tests.log; exit 1; }
tail -1 gpurun_out/r6d_tests.log
bash tools/pmc_session.sh || { echo pmc failed; exit 1; }
echo pmc done
timeout -k 10 600 python -u bench.py > gpurun_out/r6d_bench.json 2> gpurun_out/r6d_bench.err || { echo bench failed; tail -20 gpurun_out/r6d_bench.err; exit 1; }
echo bench done
timeout -k 10 300 python -u tools/step_profile.py 128 6 > gpurun_out/r6d_step_profile128.log 2>&1 || { echo sp failed; exit 1; }
timeout -k 10 300 python -u tools/small_profile.py > gpurun_out/r6d_small_profile.log 2>&1 || { echo small failed; exit 1; }
timeout -k 10 300 python -u tools/finish_profile.py > gpurun_out/r6d_finish_profile.log 2>&1 || { echo finish failed; exit 1; }
echo done
