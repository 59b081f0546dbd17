#!/bin/bash
# round 3: parity (net shapes + packed windows), whole suite, smoke, then an
# A/B of the packed window pass against the 32-stride one
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_curve.py -x -v --timeout 120 \
  --timeout-method thread -m gpu > gpurun_out/r03c_parity.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r03c_gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03c_smoke.log 2>&1 && \
for v in libtropical_hip.so libtropical_hip_strided.so libtropical_hip.so libtropical_hip_strided.so; do
  TNP_LIB=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/r03c_ab_$v.json 2>&1 || exit 1
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r03c_ab_$v.json) $(grep -o '"kernel_ms_per_pass": {[^}]*}' gpurun_out/r03c_ab_$v.json)" >> gpurun_out/r03c_ab.txt
done && \
timeout -k 10 200 python -u tools/step_profile.py 128 6 > gpurun_out/r03c_step_profile.log 2>&1 && \
timeout -k 10 200 python -u tools/small_profile.py > gpurun_out/r03c_small_profile.log 2>&1
