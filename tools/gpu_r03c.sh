#!/bin/bash
# round 3: parity (net shapes + packed windows), whole suite, smoke, then an
# A/B of the packed window pass against the 32-stride one, and bunny-scale
# profiles
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
run() { "$@" || { echo "step failed ($?): $*"; exit 1; }; }
run timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_curve.py -x -v --timeout 120 \
  --timeout-method thread -m gpu > gpurun_out/r03c_parity.log 2>&1
run timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r03c_gpu_tests.log 2>&1
run timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03c_smoke.log 2>&1
for v in default nolazy strided default nolazy strided; do
  case $v in
    default) lib=libtropical_hip.so; lz=1 ;;
    nolazy) lib=libtropical_hip.so; lz=0 ;;
    strided) lib=libtropical_hip_strided.so; lz=1 ;;
  esac
  TNP_LIB=$lib TNP_LAZY_EDGES=$lz run timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/r03c_ab_$v.json 2>&1
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r03c_ab_$v.json) $(grep -o '"kernel_ms_per_pass": {[^}]*}' gpurun_out/r03c_ab_$v.json)" >> gpurun_out/r03c_ab.txt
done
run timeout -k 10 200 python -u tools/step_profile.py 128 6 > gpurun_out/r03c_step_profile.log 2>&1
run timeout -k 10 200 python -u tools/small_profile.py > gpurun_out/r03c_small_profile.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03c_small_trace -o small \
  -- python3 tools/small_profile.py 3 flat > gpurun_out/r03c_small_trace.log 2>&1
