"""Diagnostic: where does the HIP forward differ from the oracle (per column)?"""
import sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "tropical-nerf.pytorch_amd"), os.path.join(os.getcwd(), "tests")]
import numpy as np, torch
from golden_io import load
from helpers import product_net, oracle_net
dev = torch.device("cuda", 0)
for name in ["small_sphere", "synth32"]:
    d = load(name)
    net, ref = product_net(d, dev), oracle_net(d)
    g = torch.Generator().manual_seed(1)
    x = torch.rand(20000, 3, generator=g) * 2 - 1
    enc_g = net.enc(((x + 1) / 2).to(dev)).cpu()
    with torch.no_grad():
        enc_c = ref.enc((x + 1) / 2)
        want = torch.cat(ref(x, gather=True)[1], -1)
    print(name, "enc mismatches", int((enc_g != enc_c).sum()), "of", enc_g.numel())
    got = torch.cat(net(x.to(dev), gather=True)[1], -1).cpu()
    bad = (got != want)
    print(name, "pre mismatches per col", bad.sum(0).tolist())
    # linear check with the oracle's encoding as input, on this CPU
    with torch.no_grad():
        a1 = ref.fc[0](enc_c)
    X = enc_c.numpy().astype(np.float64); W = ref.fc[0].weight.detach().numpy().astype(np.float64)
    acc = np.zeros((X.shape[0], W.shape[0]))
    for k in range(X.shape[1]):
        acc = (X[:, k:k+1] * W[None, :, k] + acc).astype(np.float32).astype(np.float64)
    h1 = (acc.astype(np.float32) + ref.fc[0].bias.detach().numpy()).astype(np.float32)
    print(name, "cpu Linear vs seq-fma mismatches", int((h1 != a1.numpy()).sum()))
import subprocess
print(subprocess.run(["bash", "-c", "lscpu | grep -i 'model name'"], capture_output=True, text=True).stdout)
print(torch.__config__.show()[:1500])
