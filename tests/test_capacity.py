"""CPU: the engine's buffer capacity arithmetic (csrc/engine.cpp
buf_grow_bytes, connect_key_cap through tnp_debug_buf_growth -- host code, no
GPU call).

Round 4's 4-rank block run (2 x 2 x 1 blocks of 203^3) died with
hipMallocAsync of 66 GB: the connect phase's key capacity was the buffer's
size in keys rounded UP to the XS_N per-XCD regions, so once a 1.5x growth
left the buffer at a size that is not a multiple of 8 * XS_N bytes, every
step asked for a few bytes more than it had and grew it by another half.  The
capacity now rounds the buffer's own size DOWN (only the 4 M + 1024 floor
rounds up): a steady workload converges after its first step, for every
shard count the build allows (step.h: XS_N <= 63)."""
import ctypes as C

import pytest


def _growth(have, req, members, xs_n):
    from tropical import _hip
    g, k = C.c_int64(), C.c_int64()
    _hip.check(_hip.lib().tnp_debug_buf_growth(have, req, members, xs_n, C.byref(g), C.byref(k)),
               "tnp_debug_buf_growth")
    return g.value, k.value


def _simulate(members, xs_n, steps=60, have=0, overflow=None):
    """The connect phase's sizing per step (engine.cpp): cap from the
    buffer, ensure cap * 8 bytes, an overflow grows to X (rounded to the
    regions).  Returns the buffer size after every step."""
    sizes = []
    for _ in range(steps):
        _, cap = _growth(have, 0, members, xs_n)
        assert cap % xs_n == 0 and cap >= 4 * members + 1024
        if cap * 8 > have:
            have, _ = _growth(have, cap * 8, members, xs_n)
        if overflow is not None and overflow > cap:
            cap = -(-overflow // xs_n) * xs_n
            if cap * 8 > have:
                have, _ = _growth(have, cap * 8, members, xs_n)
        sizes.append(have)
    return sizes


@pytest.mark.parametrize("xs_n", [1, 6, 8, 12, 48, 63])
@pytest.mark.parametrize("members", [0, 1, 999, 4_000_003, 27_000_017])
def test_key_buffer_converges(xs_n, members):
    sizes = _simulate(members, xs_n)
    assert len(set(sizes[1:])) == 1, sizes[:6]


@pytest.mark.parametrize("xs_n", [6, 8, 63])
def test_key_buffer_converges_after_an_overflow(xs_n):
    """A step whose kept keys exceed the capacity grows the buffer (x1.5 or
    to the count); the same step repeated must not grow it again."""
    sizes = _simulate(1000, xs_n, overflow=123_457)
    assert len(set(sizes[1:])) == 1
    # and from any odd starting size the buffer holds what it is asked for
    for have in (8 * 4999 + 8, 1_234_567, 3 * 2**20 + 17 * 8):
        s2 = _simulate(1000, xs_n, have=have)
        assert len(set(s2)) == 1 and s2[0] >= have


def test_growth_is_geometric_in_whole_units():
    assert _growth(0, 1, 0, 8)[0] == 256
    assert _growth(1000, 1001, 0, 8)[0] == 1536  # 1.5 x 1000 = 1500 -> 6 units
    assert _growth(1000, 5000, 0, 8)[0] == 5120
    g, _ = _growth(2**30, 2**30 + 1, 0, 8)
    assert g == 3 * 2**29 and g % 256 == 0


def test_growth_rejects_bad_arguments():
    from tropical import _hip
    g, k = C.c_int64(), C.c_int64()
    assert _hip.lib().tnp_debug_buf_growth(0, 0, 0, 64, C.byref(g), C.byref(k)) == -1
    assert _hip.lib().tnp_debug_buf_growth(-1, 0, 0, 8, C.byref(g), C.byref(k)) == -1
