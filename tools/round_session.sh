#!/bin/bash
# This round's evidence on one GPU box: the GPU test suite, the rocprofv3
# kernel-trace + PMC passes of the headline workload (tools/pmc_session.sh),
# the PMC table copied where bench.py reads it, then the default bench line.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-r05}
bash tools/gpu.sh tests || exit 1
bash tools/pmc_session.sh || exit 1
cp gpurun_out/pmc_table.json "profiles/${tag}_bench128_seed6_pmc.json" || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || exit 1
tail -1 gpurun_out/bench_full.json
