"""Reverse-engineer torch.linalg.eigvals (x86 MKL sgeev) on the 2x2
companion matrices of the curve path's quadratics: emulate sgebal + slahqr's
deflation test + slanv2 in float32 and compare bitwise (CPU only).
Usage: python tools/lapack2x2_probe.py [pq.pt]"""
import sys
import numpy as np
import torch

f32 = np.float32
EPS = f32(np.finfo(np.float32).eps / 2)      # slamch('P') = eps*base? ('E' relative machine eps = 2^-24), 'P' = eps*base = 2^-23
ULP = f32(2.0 ** -23)
SAFMIN = f32(np.finfo(np.float32).tiny)


def sign(a, b):
    return f32(abs(a)) if b >= 0 else f32(-abs(a))


def slapy2(x, y):
    x, y = abs(f32(x)), abs(f32(y))
    w, z = max(x, y), min(x, y)
    if z == 0 or w > f32(3.4e38):
        return w
    return f32(w * f32(np.sqrt(f32(f32(1) + f32(f32(z / w) * f32(z / w))))))


def slanv2(a, b, c, d):
    a, b, c, d = f32(a), f32(b), f32(c), f32(d)
    MULTPL = f32(4)
    eps = ULP
    if c == 0:
        pass
    elif b == 0:
        a, d = d, a
        b, c = f32(-c), f32(0)
    elif f32(a - d) == 0 and np.sign(b) != np.sign(c):
        pass
    else:
        temp = f32(a - d)
        p = f32(f32(0.5) * temp)
        bcmax = max(abs(b), abs(c))
        bcmis = f32(f32(min(abs(b), abs(c)) * sign(f32(1), b)) * sign(f32(1), c))
        scale = max(abs(p), bcmax)
        z = f32(f32(f32(p / scale) * p) + f32(f32(bcmax / scale) * bcmis))
        if z >= f32(MULTPL * eps):
            z = f32(p + sign(f32(f32(np.sqrt(scale)) * f32(np.sqrt(z))), p))
            a = f32(d + z)
            d = f32(d - f32(f32(bcmax / z) * bcmis))
            b = f32(b - c)
            c = f32(0)
        else:
            sigma = f32(b + c)
            p = f32(f32(0.5) * temp)
            tau = slapy2(sigma, temp)
            cs = f32(np.sqrt(f32(f32(0.5) * f32(f32(1) + f32(abs(sigma) / tau)))))
            sn = f32(f32(-f32(p / f32(tau * cs))) * sign(f32(1), sigma))
            aa = f32(f32(a * cs) + f32(b * sn))
            bb = f32(f32(-a * sn) + f32(b * cs))
            cc = f32(f32(c * cs) + f32(d * sn))
            dd = f32(f32(-c * sn) + f32(d * cs))
            a = f32(f32(aa * cs) + f32(cc * sn))
            b = f32(f32(bb * cs) + f32(dd * sn))
            c = f32(f32(-aa * sn) + f32(cc * cs))
            d = f32(f32(-bb * sn) + f32(dd * cs))
            temp = f32(f32(0.5) * f32(a + d))
            a = d = temp
            if c != 0:
                if b != 0:
                    if np.sign(b) == np.sign(c):
                        sab = f32(np.sqrt(abs(b)))
                        sac = f32(np.sqrt(abs(c)))
                        p = sign(f32(sab * sac), c)
                        a = f32(temp + p)
                        d = f32(temp - p)
                        b = f32(b - c)
                        c = f32(0)
                else:
                    b = f32(-c)
                    c = f32(0)
    r1r, r2r = a, d
    if c == 0:
        r1i = r2i = f32(0)
    else:
        r1i = f32(f32(np.sqrt(abs(b))) * f32(np.sqrt(abs(c))))
        r2i = -r1i
    return (r1r, r1i), (r2r, r2i)


def snrm2(v):
    v = [f32(x) for x in v]
    return f32(np.sqrt(np.float64(sum(np.float64(x) * np.float64(x) for x in v))))


def sgebal(A, variant="nrm2"):
    A = A.astype(np.float32).copy()
    n = 2
    # permutation: row with zero off-diagonal goes to the bottom
    k, l = 0, n - 1
    perm_done = False
    # row search (rows isolating an eigenvalue pushed down)
    while True:
        found = False
        for j in range(l, -1, -1):
            if all(A[j, i] == 0 for i in range(l + 1) if i != j):
                if j != l:
                    A[:, [j, l]] = A[:, [l, j]]
                    A[[j, l], :] = A[[l, j], :]
                if l == 0:
                    return A, 0, 0
                l -= 1
                found = True
                break
        if not found:
            break
    while True:
        found = False
        for j in range(k, l + 1):
            if all(A[i, j] == 0 for i in range(k, l + 1) if i != j):
                if j != k:
                    A[:, [j, k]] = A[:, [k, j]]
                    A[[j, k], :] = A[[k, j], :]
                k += 1
                found = True
                break
        if not found:
            break
    scale = [f32(1)] * n
    SCLFAC, FACTOR = f32(2), f32(0.95)
    SFMIN1 = f32(SAFMIN / ULP)
    SFMAX1 = f32(1) / SFMIN1
    SFMIN2 = f32(SFMIN1 * SCLFAC)
    SFMAX2 = f32(1) / SFMIN2
    while True:
        noconv = False
        for i in range(k, l + 1):
            if variant == "nrm2":
                c = snrm2(A[k:l + 1, i])
                r = snrm2(A[i, k:l + 1])
            else:  # old 1-norm excluding diagonal
                c = f32(sum(abs(A[j, i]) for j in range(k, l + 1) if j != i))
                r = f32(sum(abs(A[i, j]) for j in range(k, l + 1) if j != i))
            ca = max(abs(A[: l + 1, i]))
            ra = max(abs(A[i, k:]))
            if c == 0 or r == 0:
                continue
            g = f32(r / SCLFAC)
            f = f32(1)
            s = f32(c + r)
            while not (c >= g or max(f, c, ca) >= SFMAX2 or min(r, g, ra) <= SFMIN2):
                f = f32(f * SCLFAC); c = f32(c * SCLFAC); ca = f32(ca * SCLFAC)
                r = f32(r / SCLFAC); g = f32(g / SCLFAC); ra = f32(ra / SCLFAC)
            g = f32(c / SCLFAC)
            while not (g < r or max(r, ra) >= SFMAX2 or min(f, c, g, ca) <= SFMIN2):
                f = f32(f / SCLFAC); c = f32(c / SCLFAC); g = f32(g / SCLFAC); ca = f32(ca / SCLFAC)
                r = f32(r * SCLFAC); ra = f32(ra * SCLFAC)
            if f32(c + r) >= f32(FACTOR * s):
                continue
            if f < 1 and scale[i] < 1 and f32(f * scale[i]) <= SFMIN1:
                continue
            if f > 1 and scale[i] > 1 and scale[i] >= f32(SFMAX1 / f):
                continue
            gi = f32(f32(1) / f)
            scale[i] = f32(scale[i] * f)
            noconv = True
            A[i, k:] = (A[i, k:] * gi).astype(np.float32)
            A[: l + 1, i] = (A[: l + 1, i] * f).astype(np.float32)
        if not noconv:
            break
    return A, k, l


def eig2(C, variant="nrm2"):
    H, ilo, ihi = sgebal(C, variant)
    w = [None, None]
    for i in list(range(0, ilo)) + list(range(ihi + 1, 2)):
        w[i] = (H[i, i], f32(0))
    if ilo == ihi:
        w[ilo] = (H[ilo, ilo], f32(0))
        return w
    # slahqr deflation test on H(2,1)
    smlnum = f32(SAFMIN * f32(f32(2) / ULP))
    h21 = abs(H[1, 0])
    defl = h21 <= smlnum
    if not defl:
        tst = f32(abs(H[0, 0]) + abs(H[1, 1]))
        if h21 <= f32(ULP * tst):
            ab = max(h21, abs(H[0, 1])); ba = min(h21, abs(H[0, 1]))
            aa = max(abs(H[1, 1]), abs(f32(H[0, 0] - H[1, 1]))); bb = min(abs(H[1, 1]), abs(f32(H[0, 0] - H[1, 1])))
            s = f32(aa + ab)
            defl = f32(ba * f32(ab / s)) <= max(smlnum, f32(ULP * f32(bb * f32(aa / s))))
    if defl:
        return [(H[0, 0], f32(0)), (H[1, 1], f32(0))]
    return list(slanv2(H[0, 0], H[0, 1], H[1, 0], H[1, 1]))


if __name__ == "__main__":
    torch.set_num_threads(1)
    D = torch.load(sys.argv[1] if len(sys.argv) > 1 else "/tmp/pq.pt")
    g = torch.Generator().manual_seed(0)
    # random 2x2 companions spanning scales + the captured ones later
    rows = torch.randn(20000, 2, generator=g) * (10 ** (torch.randn(20000, 1, generator=g) * 2))
    C = torch.zeros(rows.shape[0], 2, 2)
    C[:, 0, 1] = 1
    C[:, 1] = rows
    ev = torch.linalg.eigvals(C)
    for variant in ("nrm2", "old"):
        bad = 0
        for i in range(C.shape[0]):
            w = eig2(C[i].numpy(), variant)
            got = np.array([complex(float(a), float(b)) for a, b in w], dtype=np.complex64)
            if not np.array_equal(got, ev[i].numpy()):
                bad += 1
                if bad <= 3:
                    print(variant, "mismatch", C[i].numpy().tolist(), ev[i].numpy(), got)
        print(variant, "bad", bad, "/", C.shape[0])
