"""Diagnostic: compare HIP faces with the oracle's row by row (GPU box)."""
import sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "tropical-nerf.pytorch_amd"), os.path.join(os.getcwd(), "tests")]
import numpy as np, torch
import torch.nn.functional as F
from golden_io import load
from helpers import product_net, oracle_net
import oracle.subdivide as od
from tropical._engine import engine_for
from tropical.synthetic import lattice_edges, lattice_vertices

name = sys.argv[1] if len(sys.argv) > 1 else "synth32"
d = load(name)
dev = torch.device("cuda", 0)
net = product_net(d, dev); ref = oracle_net(d)
eng = engine_for(net)
n = int(d["lattice_n"])
eng.lattice(); eng.run_steps(); eng.surface()
v, e, _ = eng.export()
tri, fc = eng.faces()
tri = tri.cpu().numpy()
with torch.no_grad():
    V = torch.from_numpy(lattice_vertices(d["marks"])); E = torch.from_numpy(lattice_edges(n))
    V, E, c = od.run_steps(V, E, ref, 1e-4)
    Vs, Es, used = od.extract_surface(V, E, ref, 1e-4, c)
    cache = c[used]
    rgn, off, _ = ref.region(Vs, cache, 1e-4)
    rid, org = od.region_ids(rgn[:, :-1], off)
    lists = od.region_lists(rid, org).unique(dim=0)
    cnt = (lists != -1).sum(1)
    lists = lists[cnt >= 3]
    pts = Vs[lists + (lists == -1)]; pts[lists == -1] = 0
    centre = pts.sum(1) / (lists != -1).sum(1, keepdim=True)
normals = ref.normal(centre)
with torch.no_grad():
    faces, order = od.sort_polygons(pts, normals)
    rtri = od.fan_triangles(lists.gather(1, order))
print("verts equal", np.array_equal(v.cpu().numpy(), Vs.numpy()), "tri shapes", tri.shape, rtri.shape, "width", lists.shape[1])
R = lists.shape[0]
g0, r0 = tri[:R], rtri[:R]
print("first-vertex mismatch rows:", int((g0[:, 0] != r0[:, 0]).sum()), "any mismatch rows:", int((g0 != r0).any(1).sum()))
bad = np.nonzero((g0 != r0).any(1))[0]
# recompute the reference score for bad rows
valid = pts.norm(dim=-1, keepdim=True) > 0
k = valid.sum(dim=-2, keepdim=True); k[k == 0] = 1
u = pts - pts.sum(dim=-2, keepdim=True) / k
cr = torch.cross(u[:, 0:1].expand_as(u), u, dim=2)
cos = F.cosine_similarity(u[:, 0:1], u, dim=-1)
side = (cr @ normals.unsqueeze(-1)).squeeze(-1)
score = cos * ((side >= 0).float() * 2 - 1) + (side < 0).float() * 2
gn = torch.empty_like(centre)
gs = net.normal(centre.to(dev)).cpu()
print("normal max abs diff", (gs - normals).abs().max().item())
for b in bad[:6]:
    row = lists[b][lists[b] != -1].numpy()
    print("row", b, "members", row)
    print("   ref order", lists.gather(1, order)[b][:len(row)].numpy(), "gpu t0", g0[b], "ref t0", r0[b])
    print("   score", score[b][:len(row)].numpy(), "side", side[b][:len(row)].numpy())
    print("   cross", cr[b][:len(row)].numpy().tolist())

# --- isolate: reference scoring with the GPU's normals at the oracle's means
gn = net.normal(centre.to(dev)).cpu()
with torch.no_grad():
    faces2, order2 = od.sort_polygons(pts, gn)
    rtri2 = od.fan_triangles(lists.gather(1, order2))
print("ref-scoring with GPU normals: tri equal to GPU?", np.array_equal(rtri2, tri),
      "mismatch rows", int((tri[:R] != rtri2[:R]).any(1).sum()))
side2 = (cr @ gn.unsqueeze(-1)).squeeze(-1)
flip = ((side2 >= 0) != (side >= 0))
print("side sign flips (all entries incl pads):", int(flip.sum()))
for b in bad[:3]:
    print(" row", b, "n_ref", normals[b].tolist(), "n_gpu", gn[b].tolist())

import ctypes as C
from tropical import _hip
Fv, Wv = C.c_int64(), C.c_int64()
_hip.check(_hip.lib().tnp_engine_faces_debug(eng.h, None, 0, C.byref(Fv), C.byref(Wv), eng._s), "dbg")
buf = torch.empty(Fv.value * Wv.value, device=dev)
_hip.check(_hip.lib().tnp_engine_faces_debug(eng.h, _hip.ptr(buf), buf.numel(), C.byref(Fv), C.byref(Wv), eng._s), "dbg")
gs = buf.view(Fv.value, Wv.value).cpu()
print("F", Fv.value, "W", Wv.value, "score mismatches (all entries):", int((gs != score).sum()), "rows:", int((gs != score).any(1).sum()))
for b in bad[:3]:
    print(" row", b, "gpu", gs[b][:6].tolist(), "ref", score[b][:6].tolist())
