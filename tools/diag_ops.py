import sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "tropical-nerf.pytorch_amd")]
import numpy as np, torch
from tropical import _hip
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
n = 1 << 20
a = torch.rand(n, generator=g) * 2; b = torch.rand(n, generator=g) + 0.1; c = torch.randn(n, generator=g)
out = torch.empty(n, 8, device=dev)
ad, bd, cd = a.to(dev), b.to(dev), c.to(dev)
import ctypes
_hip.check(_hip.lib().tnp_debug_ops(_hip.ptr(ad), _hip.ptr(bd), _hip.ptr(cd), n, _hip.ptr(out), ctypes.c_void_p(_hip.stream_ptr(dev))), "ops")
torch.cuda.synchronize()
o = out.cpu().numpy()
A, B, Cc = a.numpy().astype(np.float64), b.numpy().astype(np.float64), c.numpy().astype(np.float64)
sq = np.sqrt(A).astype(np.float32); dv = (A / B).astype(np.float32)
fm = (A * B + Cc).astype(np.float32)  # approx (double rounding rare)
print("sqrt_rn mism", int((o[:, 0] != sq).sum()), "div_rn mism", int((o[:, 1] != dv).sum()), "fma mism", int((o[:, 2] != fm).sum()))
print("mul mism", int((o[:, 3] != (a * b).numpy()).sum()), "add mism", int((o[:, 4] != (a + b).numpy()).sum()))
print("sqrtf mism", int((o[:, 5] != sq).sum()), "a/b mism", int((o[:, 6] != dv).sum()))
print("tanhf vs torch cpu", int((o[:, 7] != torch.tanh(a).numpy()).sum()))
