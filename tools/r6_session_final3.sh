#!/bin/bash
# round-6 final GPU session on the build with the two-stage key sort: smoke, the -m gpu suite,
# the rocprofv3 kernel trace + counter passes (tools/pmc_session.sh), the
# default bench line, per-step / bunny-scale / finish profiles, and the
# A/B against the build before the counter-clear change (r06f, three runs).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/ab.err
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6x_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r6x_smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6x_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r6x_tests.log; exit 1; }
tail -1 gpurun_out/r6x_tests.log
bash tools/pmc_session.sh || { echo pmc failed; exit 1; }
cp gpurun_out/pmc_table.json profiles/r06_bench128_seed6_pmc.json  # the bench line's traffic figures from this build
echo pmc done
bash tools/ab_session.sh 3 r06=libtropical_hip.so r06f=libtropical_hip_r06f.so || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r6x_bench.json 2> gpurun_out/r6x_bench.err || { echo bench failed; tail -20 gpurun_out/r6x_bench.err; exit 1; }
echo bench done
timeout -k 10 300 python -u tools/step_profile.py 128 6 > gpurun_out/r6x_step_profile128.log 2>&1 || { echo sp failed; exit 1; }
timeout -k 10 300 python -u tools/small_profile.py > gpurun_out/r6x_small_profile.log 2>&1 || { echo small failed; exit 1; }
timeout -k 10 300 python -u tools/finish_profile.py > gpurun_out/r6x_finish_profile.log 2>&1 || { echo finish failed; exit 1; }
echo done
