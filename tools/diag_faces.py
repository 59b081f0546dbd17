"""Diagnostic: compare HIP faces with the oracle's row by row."""
import sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "tropical-nerf.pytorch_amd"), os.path.join(os.getcwd(), "tests")]
import numpy as np, torch
from golden_io import load, sha
from helpers import product_net, oracle_net
import oracle.subdivide as od
from tropical._engine import engine_for
from tropical.synthetic import lattice_edges, lattice_vertices

def rows_from_fan(tri):
    rows = []
    n0 = None
    t = 0; i = 0
    # t=0 block: all rows
    # find block boundaries: block t has rows with c>=t+3, tri[first of block] v0 repeats
    blocks = []
    cur = []
    # reconstruct greedily: block t size = number of rows that continue
    return None

name = sys.argv[1] if len(sys.argv) > 1 else "synth32"
d = load(name)
dev = torch.device("cuda", 0)
net = product_net(d, dev); ref = oracle_net(d)
eng = engine_for(net)
n = int(d["lattice_n"])
eng.lattice()
eng.run_steps()
eng.surface()
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
    faces, order = od.sort_polygons(pts, normals)
    rtri = od.fan_triangles(lists.gather(1, order))
print("verts equal", np.array_equal(v.cpu().numpy(), Vs.numpy()), "tri shapes", tri.shape, rtri.shape)
R = lists.shape[0]
print("rows", R)
# block 0 = first R triangles: (p0, p1, p2) per row
g0, r0 = tri[:R], rtri[:R]
bad = np.nonzero((g0 != r0).any(1))[0]
print("rows whose first triangle differs:", len(bad))
for b in bad[:5]:
    row = lists[b][lists[b] != -1].numpy()
    print(" row", b, "members", row, "ref ordered", lists.gather(1, order)[b].numpy(), "gpu t0", g0[b], "ref t0", r0[b])
    # scores
    o = order[b]
    u = pts[b] - pts[b].sum(0) / max(1, int((pts[b].norm(dim=-1) > 0).sum()))
    print("  normal ref", normals[b].numpy())
