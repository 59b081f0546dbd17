#!/bin/bash
# `python -m tropical.stanford.train -e` on the stand-in small nets (sphere-
# and torus-fitted, committed fixtures): the real Stanford checkpoints are
# not available offline.  Flat (default) and curve (-f) runs.
export TMPDIR=/tmp
mkdir -p gpurun_out/eval
timeout -k 10 120 python - <<'PY'
import sys, torch
sys.path[:0] = [".", "tropical-nerf.pytorch_amd", "tests"]
from golden_io import load
from helpers import product_net
for name in ("small_sphere", "small_torus"):
    net = product_net(load(name), torch.device("cuda", 0))
    torch.save(net.state_dict(), f"gpurun_out/eval/{name}.pth")
PY
cd tropical-nerf.pytorch_amd || exit 1
for name in small_sphere small_torus; do
  timeout -k 10 300 python -m tropical.stanford.train -d bunny -m small -e \
    --weights ../gpurun_out/eval/$name.pth --out ../gpurun_out/eval/meshes_$name \
    > ../gpurun_out/eval/$name.log 2>&1 || exit $?
  timeout -k 10 300 python -m tropical.stanford.train -d bunny -m small -f \
    --weights ../gpurun_out/eval/$name.pth --out ../gpurun_out/eval/meshes_${name}_curve \
    > ../gpurun_out/eval/${name}_curve.log 2>&1 || exit $?
done
rm -rf ../gpurun_out/eval/meshes_*
