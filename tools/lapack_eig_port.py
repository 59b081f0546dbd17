"""Reference-LAPACK sgeev (eigenvalues only) restated in fp32 for the small
companion matrices of the curve path (geometry.py:271-299): sgebal('B') ->
sgehd2 -> slahqr.  The EIGENVALUE ORDER is what the reference's "last real
root in [0, 1]" depends on; this script checks the restatement's order
against torch.linalg.eigvals (x86 MKL) on random companions:

    python tools/lapack_eig_port.py [n]

csrc/curve.hip eig_small<N> is the device version of the same code."""
import sys

import numpy as np

f32 = np.float32
SAFMIN = f32(1.17549435e-38)
ULP = f32(1.1920928955078125e-07)    # slamch('P')
EPS = f32(5.9604644775390625e-08)    # slamch('E')


def sign(a, b):
    return f32(abs(a)) if b >= 0 else f32(-abs(a))


def slapy2(x, y):
    x, y = f32(abs(x)), f32(abs(y))
    w, z = max(x, y), min(x, y)
    if z == 0 or w > f32(3.4e38):
        return w
    r = f32(z / w)
    return f32(w * f32(np.sqrt(f32(f32(1) + f32(r * r)))))


def snrm2(v):
    return f32(np.sqrt(np.sum(np.asarray(v, np.float64) ** 2)))


def slarfg(alpha, x):
    """-> (beta, tau, x scaled)"""
    n1 = len(x)
    if n1 == 0:
        return alpha, f32(0), x
    xnorm = snrm2(x)
    if xnorm == 0:
        return alpha, f32(0), x
    beta = -sign(slapy2(alpha, xnorm), alpha)
    tau = f32(f32(beta - alpha) / beta)
    sc = f32(f32(1) / f32(alpha - beta))
    x = [f32(xi * sc) for xi in x]
    return beta, tau, x


def sgebal(A):
    n = A.shape[0]
    A = A.copy()
    k, l = 0, n - 1
    # rows with zero off-diagonal (columns 0..l) pushed down
    while True:
        found = -1
        for j in range(l, -1, -1):
            if all(A[j, i] == 0 for i in range(l + 1) if i != j):
                found = j
                break
        if found < 0:
            break
        if found != l:
            A[:, [found, l]] = A[:, [l, found]]
            A[[found, l], :] = A[[l, found], :]
        if l == 0:
            return A, 0, 0
        l -= 1
    while True:
        found = -1
        for j in range(k, l + 1):
            if all(A[i, j] == 0 for i in range(k, l + 1) if i != j):
                found = j
                break
        if found < 0:
            break
        if found != k:
            A[:, [found, k]] = A[:, [k, found]]
            A[[found, k], :] = A[[k, found], :]
        k += 1
    if k >= l:
        return A, k, l
    SFMIN1 = f32(SAFMIN / ULP)
    SFMAX1 = f32(f32(1) / SFMIN1)
    SFMIN2 = f32(SFMIN1 * f32(2))
    SFMAX2 = f32(f32(1) / SFMIN2)
    scale = [f32(1)] * n
    for _ in range(100):
        noconv = False
        for i in range(k, l + 1):
            c = snrm2(A[k:l + 1, i])
            r = snrm2(A[i, k:l + 1])
            ica = np.argmax(np.abs(A[:l + 1, i]))
            ca = f32(abs(A[ica, i]))
            ira = k + np.argmax(np.abs(A[i, k:]))
            ra = f32(abs(A[i, ira]))
            if c == 0 or r == 0:
                continue
            g = f32(r / f32(2))
            f = f32(1)
            s = f32(c + r)
            while not (c >= g or max(f, c, ca) >= SFMAX2 or min(r, g, ra) <= SFMIN2):
                f, c, ca, r, g, ra = f32(f * 2), f32(c * 2), f32(ca * 2), f32(r / 2), f32(g / 2), f32(ra / 2)
            g = f32(c / f32(2))
            while not (g < r or max(r, ra) >= SFMAX2 or min(f, c, g, ca) <= SFMIN2):
                f, c, g, ca, r, ra = f32(f / 2), f32(c / 2), f32(g / 2), f32(ca / 2), f32(r * 2), f32(ra * 2)
            if f32(c + r) >= f32(f32(0.95) * s):
                continue
            if f < 1 and scale[i] < 1 and f32(f * scale[i]) <= SFMIN1:
                continue
            if f > 1 and scale[i] > 1 and scale[i] >= f32(SFMAX1 / f):
                continue
            gi = f32(f32(1) / f)
            scale[i] = f32(scale[i] * f)
            noconv = True
            A[i, k:] = (A[i, k:] * gi).astype(f32)
            A[:l + 1, i] = (A[:l + 1, i] * f).astype(f32)
        if not noconv:
            break
    return A, k, l


def sgehd2(A, ilo, ihi):
    n = A.shape[0]
    A = A.copy()
    for i in range(ilo, ihi):
        x = [A[j, i] for j in range(i + 2, ihi + 1)]
        beta, tau, x = slarfg(A[i + 1, i], x)
        for j, xv in zip(range(i + 2, ihi + 1), x):
            A[j, i] = xv
        A[i + 1, i] = beta
        if tau == 0:
            continue
        v = [f32(1)] + [A[j, i] for j in range(i + 2, ihi + 1)]
        rows = list(range(i + 1, ihi + 1))
        # right: C = A[0:ihi+1, i+1:ihi+1]; w = C v; C -= tau w v^T
        for r in range(0, ihi + 1):
            w = f32(0)
            for vv, cj in zip(v, rows):
                w = f32(w + f32(A[r, cj] * vv))
            for vv, cj in zip(v, rows):
                A[r, cj] = f32(A[r, cj] - f32(f32(tau * w) * vv))
        # left: C = A[i+1:ihi+1, i+1:n]; w = C^T v; C -= tau v w^T
        for cj in range(i + 1, n):
            w = f32(0)
            for vv, r in zip(v, rows):
                w = f32(w + f32(A[r, cj] * vv))
            for vv, r in zip(v, rows):
                A[r, cj] = f32(A[r, cj] - f32(f32(tau * vv) * w))
    for i in range(ilo, ihi):   # Hessenberg: below the subdiagonal is the reflectors' storage
        for j in range(i + 2, n):
            A[j, i] = f32(0)
    return A


def slanv2(a, b, c, d):
    a, b, c, d = f32(a), f32(b), f32(c), f32(d)
    if c == 0:
        pass
    elif b == 0:
        a, d, b, c = d, a, -c, f32(0)
    elif f32(a - d) == 0 and (b > 0) != (c > 0):
        pass
    else:
        temp = f32(a - d)
        p = f32(f32(0.5) * temp)
        bcmax = max(abs(b), abs(c))
        bcmis = f32(f32(min(abs(b), abs(c)) * sign(f32(1), b)) * sign(f32(1), c))
        scale = max(abs(p), bcmax)
        z = f32(f32(f32(p / scale) * p) + f32(f32(bcmax / scale) * bcmis))
        if z >= f32(4) * EPS * 2:   # 4*EPS with EPS = slamch('P')
            z = f32(p + sign(f32(f32(np.sqrt(scale)) * f32(np.sqrt(z))), p))
            a = f32(d + z)
            d = f32(d - f32(f32(bcmax / z) * bcmis))
            b = f32(b - c)
            c = f32(0)
        else:
            sigma = f32(b + c)
            tau = slapy2(sigma, temp)
            cs = f32(np.sqrt(f32(f32(0.5) * f32(f32(1) + f32(abs(sigma) / tau)))))
            sn = f32(-f32(p / f32(tau * cs)) * sign(f32(1), sigma))
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
                    if (b > 0) == (c > 0):
                        sab, sac = f32(np.sqrt(abs(b))), f32(np.sqrt(abs(c)))
                        p = sign(f32(sab * sac), c)
                        a = f32(temp + p)
                        d = f32(temp - p)
                        b = f32(b - c)
                        c = f32(0)
                else:
                    b, c = -c, f32(0)
    wr = [a, d]
    if c == 0:
        wi = [f32(0), f32(0)]
    else:
        w = f32(f32(np.sqrt(abs(b))) * f32(np.sqrt(abs(c))))
        wi = [w, -w]
    return wr, wi


def slahqr(H, ilo, ihi):
    n = H.shape[0]
    H = H.copy()
    wr = [f32(0)] * n
    wi = [f32(0)] * n
    for i in range(ilo):
        wr[i] = H[i, i]
    for i in range(ihi + 1, n):
        wr[i] = H[i, i]
    if ilo == ihi:
        wr[ilo] = H[ilo, ilo]
        return wr, wi, 0
    for j in range(ilo, ihi - 2):
        H[j + 2, j] = 0
        H[j + 3, j] = 0
    if ilo <= ihi - 2:
        H[ihi, ihi - 2] = 0
    nh = ihi - ilo + 1
    smlnum = f32(SAFMIN * f32(f32(nh) / ULP))
    itmax = 30 * max(10, nh)
    kdefl = 0
    i = ihi
    while i >= ilo:
        l = ilo
        converged = False
        for its in range(itmax + 1):
            k = i
            while k > l:
                if abs(H[k, k - 1]) <= smlnum:
                    break
                tst = f32(abs(H[k - 1, k - 1]) + abs(H[k, k]))
                if tst == 0:
                    if k - 2 >= ilo:
                        tst = f32(tst + abs(H[k - 1, k - 2]))
                    if k + 1 <= ihi:
                        tst = f32(tst + abs(H[k + 1, k]))
                if abs(H[k, k - 1]) <= f32(ULP * tst):
                    ab = max(abs(H[k, k - 1]), abs(H[k - 1, k]))
                    ba = min(abs(H[k, k - 1]), abs(H[k - 1, k]))
                    aa = max(abs(H[k, k]), abs(f32(H[k - 1, k - 1] - H[k, k])))
                    bb = min(abs(H[k, k]), abs(f32(H[k - 1, k - 1] - H[k, k])))
                    s = f32(aa + ab)
                    if f32(ba * f32(ab / s)) <= max(smlnum, f32(ULP * f32(bb * f32(aa / s)))):
                        break
                k -= 1
            l = k
            if l > ilo:
                H[l, l - 1] = 0
            if l >= i - 1:
                converged = True
                break
            kdefl += 1
            i1, i2 = l, i
            if kdefl % 20 == 0:
                s = f32(abs(H[i, i - 1]) + abs(H[i - 1, i - 2]))
                h11 = f32(f32(f32(0.75) * s) + H[i, i]); h12 = f32(f32(-0.4375) * s); h21 = s; h22 = h11
            elif kdefl % 10 == 0:
                s = f32(abs(H[l + 1, l]) + abs(H[l + 2, l + 1]))
                h11 = f32(f32(f32(0.75) * s) + H[l, l]); h12 = f32(f32(-0.4375) * s); h21 = s; h22 = h11
            else:
                h11, h21, h12, h22 = H[i - 1, i - 1], H[i, i - 1], H[i - 1, i], H[i, i]
            s = f32(f32(f32(abs(h11) + abs(h12)) + abs(h21)) + abs(h22))
            if s == 0:
                rt1r = rt1i = rt2r = rt2i = f32(0)
            else:
                h11, h21, h12, h22 = f32(h11 / s), f32(h21 / s), f32(h12 / s), f32(h22 / s)
                tr = f32(f32(h11 + h22) / f32(2))
                det = f32(f32(f32(h11 - tr) * f32(h22 - tr)) - f32(h12 * h21))
                rtdisc = f32(np.sqrt(abs(det)))
                if det >= 0:
                    rt1r = f32(tr * s); rt2r = rt1r; rt1i = f32(rtdisc * s); rt2i = -rt1i
                else:
                    rt1r = f32(tr + rtdisc); rt2r = f32(tr - rtdisc)
                    if abs(f32(rt1r - h22)) <= abs(f32(rt2r - h22)):
                        rt1r = f32(rt1r * s); rt2r = rt1r
                    else:
                        rt2r = f32(rt2r * s); rt1r = rt2r
                    rt1i = rt2i = f32(0)
            m = i - 2
            while True:
                h21s = H[m + 1, m]
                s = f32(f32(abs(f32(H[m, m] - rt2r)) + abs(rt2i)) + abs(h21s))
                h21s = f32(H[m + 1, m] / s)
                v1 = f32(f32(f32(h21s * H[m, m + 1]) + f32(f32(H[m, m] - rt1r) * f32(f32(H[m, m] - rt2r) / s)))
                         - f32(rt1i * f32(rt2i / s)))
                v2 = f32(h21s * f32(f32(f32(H[m, m] + H[m + 1, m + 1]) - rt1r) - rt2r))
                v3 = f32(h21s * H[m + 2, m + 1])
                s = f32(f32(abs(v1) + abs(v2)) + abs(v3))
                v = [f32(v1 / s), f32(v2 / s), f32(v3 / s)]
                if m == l:
                    break
                h00 = f32(abs(H[m, m - 1]) * f32(abs(v[1]) + abs(v[2])))
                h01 = f32(f32(ULP * abs(v[0])) * f32(f32(abs(H[m - 1, m - 1]) + abs(H[m, m])) + abs(H[m + 1, m + 1])))
                if h00 <= h01:
                    break
                m -= 1
            for k in range(m, i):
                nr = min(3, i - k + 1)
                if k > m:
                    v = [H[k + q, k - 1] for q in range(nr)] + [f32(0)] * (3 - nr)
                beta, t1, xs = slarfg(v[0], v[1:nr])
                v = [beta] + list(xs) + [f32(0)] * (3 - nr)
                if k > m:
                    H[k, k - 1] = v[0]
                    H[k + 1, k - 1] = 0
                    if k < i - 1:
                        H[k + 2, k - 1] = 0
                elif m > l:
                    H[k, k - 1] = f32(H[k, k - 1] * f32(f32(1) - t1))
                v2 = v[1]
                t2 = f32(t1 * v2)
                if nr == 3:
                    v3 = v[2]
                    t3 = f32(t1 * v3)
                    for j in range(k, i2 + 1):
                        sm = f32(f32(H[k, j] + f32(v2 * H[k + 1, j])) + f32(v3 * H[k + 2, j]))
                        H[k, j] = f32(H[k, j] - f32(sm * t1))
                        H[k + 1, j] = f32(H[k + 1, j] - f32(sm * t2))
                        H[k + 2, j] = f32(H[k + 2, j] - f32(sm * t3))
                    for j in range(i1, min(k + 3, i) + 1):
                        sm = f32(f32(H[j, k] + f32(v2 * H[j, k + 1])) + f32(v3 * H[j, k + 2]))
                        H[j, k] = f32(H[j, k] - f32(sm * t1))
                        H[j, k + 1] = f32(H[j, k + 1] - f32(sm * t2))
                        H[j, k + 2] = f32(H[j, k + 2] - f32(sm * t3))
                elif nr == 2:
                    for j in range(k, i2 + 1):
                        sm = f32(H[k, j] + f32(v2 * H[k + 1, j]))
                        H[k, j] = f32(H[k, j] - f32(sm * t1))
                        H[k + 1, j] = f32(H[k + 1, j] - f32(sm * t2))
                    for j in range(i1, i + 1):
                        sm = f32(H[j, k] + f32(v2 * H[j, k + 1]))
                        H[j, k] = f32(H[j, k] - f32(sm * t1))
                        H[j, k + 1] = f32(H[j, k + 1] - f32(sm * t2))
        if not converged:
            return wr, wi, i + 1
        if l == i:
            wr[i] = H[i, i]
            wi[i] = f32(0)
        else:
            (wr[i - 1], wr[i]), (wi[i - 1], wi[i]) = slanv2(H[i - 1, i - 1], H[i - 1, i], H[i, i - 1], H[i, i])
        kdefl = 0
        i = l - 1
    return wr, wi, 0


def sgeev_values(A):
    B, ilo, ihi = sgebal(np.asarray(A, f32))
    H = sgehd2(B, ilo, ihi)
    wr, wi, info = slahqr(H, ilo, ihi)
    return np.array(wr, np.float64) + 1j * np.array(wi, np.float64)


def companion(c):
    N = len(c) - 1
    C = np.zeros((N, N), f32)
    for i in range(N - 1):
        C[i, i + 1] = 1
    C[-1] = (-c[:-1] / c[-1]).astype(f32)
    return C


def last01(r):
    m = (np.abs(r.imag) <= 1e-9) & (r.real >= 0) & (r.real <= 1)
    idx = np.nonzero(m)[0]
    return None if len(idx) == 0 else r[idx[-1]].real


if __name__ == "__main__":
    import torch
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    rng = np.random.default_rng(3)
    agree = multi = magree = 0
    for t in range(n):
        N = int(rng.choice([3, 4]))
        roots = rng.uniform(-0.5, 1.5, N)
        c = (np.poly(roots)[::-1] * rng.uniform(0.5, 2)).astype(f32)
        C = companion(c)
        a = torch.linalg.eigvals(torch.from_numpy(C)).numpy()
        b = sgeev_values(C)
        la, lb = last01(a), last01(b)
        ok = (la is None and lb is None) or (la is not None and lb is not None and abs(la - lb) < 1e-4)
        agree += ok
        if ((np.abs(a.imag) <= 1e-9) & (a.real >= 0) & (a.real <= 1)).sum() > 1:
            multi += 1
            magree += ok
    print(f"last root in [0,1] agrees with torch (MKL): {agree}/{n}; multi-root cases {magree}/{multi}")
