#!/bin/bash
# round-6 GPU session: smoke, the whole -m gpu suite, A/B of the forward_new
# variants, the grouping kernel's phase clocks, the default bench line with
# the 64^3 CPU baseline.  Stops at the first failure.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6c_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r6c_smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6c_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r6c_tests.log; exit 1; }
tail -2 gpurun_out/r6c_tests.log
bash tools/ab_session.sh 3 new=libtropical_hip.so nomfma=libtropical_hip_nomfma.so r05=libtropical_hip_r05.so || exit 1
bash tools/ab_session.sh 1 phases=libtropical_hip_phases.so || exit 1
TNP_CPU_MARKS=64 timeout -k 10 900 python -u bench.py > gpurun_out/r6c_bench.json 2> gpurun_out/r6c_bench.err || { echo bench failed; tail -20 gpurun_out/r6c_bench.err; exit 1; }
echo done
