"""numpy prototype of the two-stage symmetric eigensolver planned for the GPU.

Stage 1 (sy2sb): full -> band (half-bandwidth b) with TSQR panel QR (Householder
leaves of c rows + Householder root over the stacked R's) and the two-sided
compact-WY updates, exactly in the block-sparse form the GPU kernels use.
Stage 2 (sb2st): band -> tridiagonal by bulge chasing (one column per sweep).
Back-transformations: Q2 applied in blocks G(sweep group, step) in the valid
order derived in DESIGN.md, Q1 through the TSQR structure.

Design tool only (not test infrastructure, not product).
"""
import numpy as np


def house(x):
    """LAPACK dlarfg: H = I - tau v v^T, v[0] = 1, H x = beta e1."""
    alpha = x[0]
    xn = np.linalg.norm(x[1:])
    v = np.zeros_like(x)
    v[0] = 1.0
    if xn == 0.0:
        return v, 0.0, alpha
    beta = -np.copysign(np.hypot(alpha, xn), alpha)
    tau = (beta - alpha) / beta
    v[1:] = x[1:] / (alpha - beta)
    return v, tau, beta


def qr_house(P):
    """Householder QR of P (h x b): returns Y (h x kk unit lower), tau, R (kk x b)."""
    P = P.copy()
    h, b = P.shape
    kk = min(h, b)
    Y = np.zeros((h, kk))
    taus = np.zeros(kk)
    for j in range(kk):
        v, tau, beta = house(P[j:, j])
        Y[j:, j] = v
        taus[j] = tau
        P[j:, j:] -= tau * np.outer(v, v @ P[j:, j:])
        P[j + 1:, j] = 0.0
    return Y, taus, np.triu(P[:kk, :])


def larft(Y, taus):
    """Forward columnwise T: H_0 H_1 ... = I - Y T Y^T."""
    k = len(taus)
    T = np.zeros((k, k))
    G = Y.T @ Y
    for i in range(k):
        T[i, i] = taus[i]
        if i:
            T[:i, i] = T[:i, :i] @ (-taus[i] * G[:i, i])
    return T


def two_sided(A, Y, T):
    """A <- Q^T A Q, Q = I - Y T Y^T (A symmetric)."""
    X = A @ Y @ T
    W = X - 0.5 * Y @ (T.T @ (Y.T @ X))
    return A - Y @ W.T - W @ Y.T


def sy2sb(A, b, c=256):
    """Full -> band.  Returns band matrix and the list of panel transforms."""
    A = A.copy()
    n = A.shape[0]
    panels = []
    p = 0
    while p + b < n - 1:
        r0 = p + b
        m = n - r0
        P = A[r0:, p:p + b].copy()
        nc = max(1, m // c)
        bounds = [(I * c, (I + 1) * c if I < nc - 1 else m) for I in range(nc)]
        leaves = []
        Rs = []
        rrows = []
        for (a, e) in bounds:
            Y, taus, R = qr_house(P[a:e])
            T = larft(Y, taus)
            leaves.append((a, e, Y, T))
            Rs.append(R)
            rrows.extend(range(a, a + R.shape[0]))
        Rstack = np.vstack(Rs)
        Yr, taur, R = qr_house(Rstack)
        Tr = larft(Yr, taur)
        # two-sided: leaves (block diagonal), then root (embedded on rrows)
        A22 = A[r0:, r0:]
        Yd = np.zeros((m, sum(l[2].shape[1] for l in leaves)))
        Td = np.zeros((Yd.shape[1], Yd.shape[1]))
        col = 0
        for (a, e, Y, T) in leaves:
            kk = Y.shape[1]
            Yd[a:e, col:col + kk] = Y
            Td[col:col + kk, col:col + kk] = T
            col += kk
        A22 = two_sided(A22, Yd, Td)
        Ye = np.zeros((m, Yr.shape[1]))
        Ye[rrows, :] = Yr
        A22 = two_sided(A22, Ye, Tr)
        A[r0:, r0:] = A22
        newp = np.zeros((m, b))
        newp[:R.shape[0], :] = R
        A[r0:, p:p + b] = newp
        A[p:p + b, r0:] = newp.T
        panels.append((r0, Yd, Td, Ye, Tr))
        p += b
    return A, panels


def sb2st(B, b):
    """Band -> tridiagonal by bulge chasing.  Returns T (d, e) and the
    reflectors {(sweep, step): (row0, v, tau)} in application order."""
    B = B.copy()
    n = B.shape[0]
    refl = {}
    for j in range(n - 2):
        # first reflector of sweep j: rows [j+1, j+b], annihilates B[j+2:j+b+1, j]
        r1 = j + 1
        s = 0
        col = j
        while True:
            r2 = min(r1 + b, n)  # rows [r1, r2)
            if r2 - r1 < 2:
                break
            x = B[r1:r2, col]
            if np.all(x[1:] == 0):
                v, tau = np.zeros_like(x), 0.0
                v[0] = 1.0
            else:
                v, tau, beta = house(x)
            # two-sided on the window of rows/cols that can be nonzero
            lo = max(0, r1 - b)
            hi = min(n, r2 + b)
            Bw = B[r1:r2, lo:hi]
            B[r1:r2, lo:hi] = Bw - tau * np.outer(v, v @ Bw)
            Bw = B[lo:hi, r1:r2]
            B[lo:hi, r1:r2] = Bw - tau * np.outer(Bw @ v, v)
            refl[(j, s)] = (r1, v, tau)
            # bulge: column r1 now has nonzeros down to r2 - 1 + b; the next
            # reflector annihilates column r1 below its band (rows r1+b+1 ..)
            col = r1
            r1 = r1 + b
            s += 1
            if r1 >= n - 1:
                break
    d = np.diag(B).copy()
    e = np.diag(B, -1).copy()
    return d, e, B, refl


def apply_q2(Z, refl, n, b, g):
    """Z <- Q2 Z with Q2 = product of reflectors in application order, applied
    in blocks G(group, s) (sweep groups from last to first, steps ascending,
    within a block sweeps descending)."""
    Z = Z.copy()
    nsw = n - 2
    groups = list(range(0, nsw, g))
    for j0 in reversed(groups):
        j1 = min(j0 + g, nsw)
        s = 0
        while True:
            items = [(j, refl[(j, s)]) for j in range(j1 - 1, j0 - 1, -1) if (j, s) in refl]
            if not items:
                break
            for j, (r1, v, tau) in items:   # Z <- H(j0,s) ... H(j1-1,s) Z: apply j1-1 first
                L = len(v)
                Z[r1:r1 + L] -= tau * np.outer(v, v @ Z[r1:r1 + L])
            s += 1
    return Z


def apply_q2_sequential(Z, refl):
    Z = Z.copy()
    for key in sorted(refl.keys(), reverse=True):
        r1, v, tau = refl[key]
        L = len(v)
        Z[r1:r1 + L] -= tau * np.outer(v, v @ Z[r1:r1 + L])
    return Z


def apply_q1(Z, panels):
    Z = Z.copy()
    for (r0, Yd, Td, Ye, Tr) in reversed(panels):
        Zs = Z[r0:]
        Zs = Zs - Ye @ (Tr @ (Ye.T @ Zs))      # E first (Q = D E: Q Z = D (E Z))
        Zs = Zs - Yd @ (Td @ (Yd.T @ Zs))
        Z[r0:] = Zs
    return Z


if __name__ == "__main__":
    rng = np.random.default_rng(0)
    n, b = 300, 8
    X = rng.standard_normal((n + 40, n))
    A = X.T @ X / X.shape[0]
    Bm, panels = sy2sb(A, b, c=64)
    band_off = np.abs(np.tril(Bm, -b - 1)).max()
    print("stage1 outside-band max", band_off)
    L = np.linalg.eigvalsh(A)
    print("stage1 eig err", np.abs(np.linalg.eigvalsh((Bm + Bm.T) / 2) - L).max())
    d, e, Bt, refl = sb2st(Bm, b)
    print("stage2 off-tridiagonal max", np.abs(np.tril(Bt, -2)).max())
    T = np.diag(d) + np.diag(e, 1) + np.diag(e, -1)
    w, Zt = np.linalg.eigh(T)
    print("eig err", np.abs(w - L).max())
    Zs = apply_q2_sequential(Zt, refl)
    for g in (1, 3, 8):
        Zb = apply_q2(Zt, refl, n, b, g)
        print("q2 blocked vs sequential g=%d" % g, np.abs(Zb - Zs).max())
    V = apply_q1(Zs, panels)
    print("residual", np.abs(A @ V - V * w).max(), "orth", np.abs(V.T @ V - np.eye(n)).max())
