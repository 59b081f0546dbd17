#!/bin/bash
# Full GPU check: every -m gpu test, smoke(), the 2-rank rehearsal.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 300 -p no:cacheprovider > gpurun_out/gpu_tests_full.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
bash tools/multi_rehearsal.sh
