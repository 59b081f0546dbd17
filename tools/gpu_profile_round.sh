#!/bin/bash
# Round-end evidence on one GPU box: every -m gpu test, smoke(), the rocprof
# kernel-trace stats and PMC passes of the bench workload (tools/pmc_session.sh),
# the default bench line priced with those counters, the per-step profile,
# and a 4-rank gloo rehearsal of the sharded bench on the one GPU against the
# unsharded run of the same lattice.  Outputs under gpurun_out/ (copied into
# profiles/ by hand).  Each GPU step has its own limit; the first failure ends it.
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r03}
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash tools/pmc_session.sh || exit 1
cp gpurun_out/pmc_table.json profiles/${R}_bench128_seed6_pmc.json
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { tail gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-300
