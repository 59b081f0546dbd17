#!/bin/bash
# round-6 GPU session 2: A/B of the window-table variants of the grouping
# kernel, failover frequency per step, the counter list, the 64^3 CPU baseline.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/ab.err
bash tools/ab_session.sh 2 base=libtropical_hip.so w1024k256=libtropical_hip_w1024k256.so \
  w768k320=libtropical_hip_w768k320.so w1024m4=libtropical_hip_w1024m4.so || exit 1
timeout -k 10 120 python -u -c "
import sys, os, json
sys.path[:0] = [os.getcwd(), 'tropical-nerf.pytorch_amd', 'tests']
import torch, bench
from tropical._engine import engine_for
net = bench.make_net(128, torch.device('cuda', 0), 6)
eng = engine_for(net)
st = []
eng.lattice(); eng.run_steps(st)
print(json.dumps([{k: s[k] for k in ('idx', 'S', 'override_applied', 'X')} for s in st]))
" > gpurun_out/r6_failover.json 2> gpurun_out/r6_failover.err || exit 1
timeout -k 10 60 rocprofv3 -L > gpurun_out/r6_counters.txt 2>&1 || echo "counter list rc=$?"
timeout -k 10 900 python -u tools/cpu_baseline.py 64 6 > gpurun_out/r6_cpu64.json 2> gpurun_out/r6_cpu64.err || { echo cpu64 failed; tail -5 gpurun_out/r6_cpu64.err; exit 1; }
echo done
