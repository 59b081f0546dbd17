#!/bin/bash
# Rehearse the N>1 bench path on a one-GPU box: N=1 at the 2-GPU lattice
# size (161^3), then 2 ranks sharing the GPU with gloo collectives; the
# stitched complex of the 2-rank run must equal the N=1 final complex.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --marks 161 --steps 2 --warmup 1 --no-cpu > gpurun_out/b161.log 2>&1 && \
TNP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu > gpurun_out/b2.log 2>&1
