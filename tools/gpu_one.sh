#!/bin/bash
# One GPU test file (argument), stop on the first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest "$@" -m gpu -x -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/one.log 2>&1
rc=$?
tail -40 gpurun_out/one.log
exit $rc
