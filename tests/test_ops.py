"""``torch.ops.tropical_hip`` (tropical/ops.py): the dispatcher-registered
entry points of SURVEY §8(b).

CPU: every op is registered, its fake (meta) implementation gives the output
shapes, and a CPU tensor is refused (no CPU fallback).  GPU: each op equals
the drop-in surface it mirrors bitwise (which the parity suite pins to the
reference's goldens), and ``subpoly_step`` / ``subpoly`` reproduce the
reference's per-step hashes and faces.
"""
import numpy as np
import pytest
import torch

from golden_io import load, sha

import tropical.ops as ops


def _meta_args(L=2, P=1024, M=32, layers=3, hidden=16):
    nin = 2 * L
    sizes = [nin] + [hidden] * (layers - 1) + [2]
    nw = sum(a * b + b for a, b in zip(sizes[:-1], sizes[1:]))
    meta = torch.zeros(L, 4, dtype=torch.int32)
    return (torch.empty(P, device="meta"), meta, torch.ones(L), torch.empty(nw, device="meta"),
            torch.empty(M, device="meta"), 1e-4, layers, hidden)


def test_ops_registered():
    for name in ops.OPS:
        assert hasattr(torch.ops.tropical_hip, name), name


def test_fake_shapes():
    args = _meta_args()
    x = torch.empty(1000, 3, device="meta")
    pre, out2 = torch.ops.tropical_hip.encode_mlp(x, *args)
    assert pre.shape == (33, 1000) and out2.shape == (1000, 2)
    m, off = torch.ops.tropical_hip.region(x, pre, *args)
    assert m.shape == (1000, 36) and m.dtype == torch.int64 and off.shape == (1000, 3)
    y, J = torch.ops.tropical_hip.sdf_grad(x, *args)
    assert y.shape == (1000,) and J.shape == (1000, 3)


def test_cpu_tensors_refused():
    table = torch.zeros(64)
    args = (table, torch.zeros(2, 4, dtype=torch.int32), torch.ones(2), torch.zeros(386),
            torch.zeros(8), 1e-4, 3, 16)
    with pytest.raises(RuntimeError):
        torch.ops.tropical_hip.encode_mlp(torch.zeros(4, 3), *args)


# ---------------------------------------------------------------------------
# GPU: equal to the drop-in surface / the reference's goldens
# ---------------------------------------------------------------------------

def _pts(n, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(n, 3, generator=g) * 2 - 1


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["small_sphere", "synth32h"])
def test_ops_equal_dropin_surface(cuda, name):
    from helpers import product_net
    d = load(name)
    net = product_net(d, cuda)
    args = ops.net_args(net)
    x = _pts(5000, 3).to(cuda)
    pre, out2 = torch.ops.tropical_hip.encode_mlp(x, *args)
    out, planes = net(x, gather=True)
    assert torch.equal(pre.t(), torch.cat(planes, -1)) and torch.equal(out2, out)
    # the grouped (box-corner) forward
    pg, _ = torch.ops.tropical_hip.encode_mlp(x[:4096], *args, group=8)
    _, planes_g = net(x[:4096], gather=True, group=8)
    assert torch.equal(pg.t(), torch.cat(planes_g, -1))
    m, off = torch.ops.tropical_hip.region(x, pre, *args)
    m_ref, off_ref, _ = net.region(x)
    assert torch.equal(m, m_ref) and torch.equal(off, off_ref)
    y, J = torch.ops.tropical_hip.sdf_grad(x, *args)
    J_ref, y_ref = net.normal(x, return_y=True)
    assert torch.equal(y, y_ref[:, 0]) and torch.equal(J, J_ref)


@pytest.mark.gpu
def test_subpoly_step_op_reproduces_reference_steps(cuda):
    """The functional step op over the synth24 lattice: every state hash is
    the reference's, and the caller's tensors are left untouched."""
    from helpers import product_net
    from tropical.synthetic import lattice_edges, lattice_vertices
    d = load("synth24")
    net = product_net(d, cuda)
    args = ops.net_args(net)
    V = torch.from_numpy(lattice_vertices(d["marks"])).to(cuda)
    E = torch.from_numpy(lattice_edges(int(d["lattice_n"]))).to(cuda)
    # the cache as the reference hands it over: Net.forward's output, with a
    # graph (subpoly.py:93) -- the op detaches it; its outputs carry none
    o = torch.cat(net(V, gather=True)[1], -1)
    assert o.requires_grad
    for step, idx in enumerate(d["step_idx"][:12]):
        E_in = E.clone()
        V2, E2, o2 = torch.ops.tropical_hip.subpoly_step(V, E, o, *args, int(idx), True, True)
        assert torch.equal(E, E_in)
        assert not (V2.requires_grad or E2.requires_grad or o2.requires_grad)
        assert sha(V2.cpu().numpy(), E2.cpu().numpy(), o2.cpu().numpy()) == str(d["step_sha"][step])
        V, E, o = V2, E2, o2


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["small_sphere", "large_sphere"])
def test_subpoly_op_faces_match_reference(cuda, name):
    from helpers import product_net
    d = load(name)
    net = product_net(d, cuda)
    verts, tri, faces = torch.ops.tropical_hip.subpoly(*ops.net_args(net), 1.2, True)
    assert verts.shape[0] == int(d["n_surf"][0])
    assert sha(verts.cpu().numpy()) == str(d["sha_surf"])
    assert sha(tri.cpu().numpy().astype(np.int64)) == str(d["sha_tri"])
    assert sha(faces.cpu().numpy().astype(np.float32)) == str(d["sha_faces"])
