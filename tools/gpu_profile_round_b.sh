#!/bin/bash
# Round-end evidence, part B: per-step and bunny-scale profiles, a 203^3
# single-rank bench and its 4-rank gloo rehearsal on the one GPU.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/step_profile.py 128 6 > gpurun_out/step_profile.log 2>&1 || exit 1
timeout -k 10 200 python tools/small_profile.py 20 > gpurun_out/small_profile.log 2>&1 || exit 1
timeout -k 10 200 python tools/small_profile.py 20 curve > gpurun_out/small_profile_curve.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --marks 203 --steps 2 --warmup 1 --no-cpu > gpurun_out/b203_1rank.log 2>&1 || exit 1
TNP_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 4 --steps 2 --warmup 1 --no-cpu \
  > gpurun_out/b203_4rank.log 2>&1 || { tail gpurun_out/b203_4rank.log; exit 1; }
grep -o '"final_complex": {[^}]*}' gpurun_out/b203_1rank.log gpurun_out/b203_4rank.log
