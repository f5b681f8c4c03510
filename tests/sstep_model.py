"""Numerical model of a two-vectors-per-pass Lanczos (design study for the next
update-pass design, DESIGN.md §3 "Next"; test infrastructure, not product code).

Today every Lanczos iteration j is one HBM pass that reads the whole basis
W_0..W_j to orthogonalise ONE new vector: sum_j (j+2) vector
transfers per basis, 119 at m = 16.  This model checks the algebra of a pass that
produces TWO new vectors from one read of the stored basis, which would cut the
update traffic to sum_p (2p+3) = 63 transfers at m = 16:

  stored raw vectors S_0..S_J (W = S C, C upper triangular, kept on the device),
  Arnoldi matrix H (H[k,i] = W_k^H L W_i) known for the columns i < J.
  One pass reads S_0..S_J once, plus L S_J and L^2 S_J (a radius-2 stencil of
  the last stored vector only), and writes
      X = L W_J - sigma W_J - sum_{k<J} conj(H[J,k]) W_k        (-> S_{J+1})
      Z = (L - sigma) X                                        (-> S_{J+2})
  as per-cell linear combinations of those inputs: L S_l (l < J) is never applied,
  it is rewritten through the Arnoldi relation L W_i = sum_k H[k,i] W_k.  The same
  pass measures the dots S_l^H X, S_l^H Z, X^H X, X^H Z, Z^H Z; the new columns of
  C (W_{J+1}, W_{J+2}) and of H (alpha_J, beta, alpha_{J+1}, ...) follow from
  those in coefficient space.  sigma (a shift, here the previous alpha) keeps the
  Gram-based norms free of cancellation.

Run: python tests/sstep_model.py  -- compares 20 steps of 3D/2D cubic NLSE against
oracle/np_ref.py's MGS Lanczos and prints the relative L2 differences and the
basis orthogonality (tests/test_sstep_model.py checks the same at small sizes).
Open: breakdown (nu -> 0) is not handled here.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import np_ref  # noqa: E402  (design study: compared against the oracle)


def lanczos2(apply, u, m, shift=True, nstore=None, raw=False):
    """T (m x m tridiagonal as the reference builds it), S (stored vectors), C, beta.
    nstore: stop once S_0..S_{nstore-1} are stored (the fused-tail end game);
    raw: return (S, C, H, G, beta) at that point instead of T."""
    u = np.asarray(u, dtype=np.complex128)
    beta = np.linalg.norm(u)
    S = [u / beta]
    C = np.zeros((m + 1, m + 1), complex)
    C[0, 0] = 1.0
    G = np.zeros((m + 1, m + 1), complex)  # Gram of the stored vectors
    G[0, 0] = np.vdot(S[0], S[0])
    H = np.zeros((m + 1, m + 1), complex)
    Cinv = np.zeros_like(C)
    J = 0
    sigma = 0.0
    mm = m if nstore is None else nstore
    while J + 1 < mm:
        n_s = J + 1
        Cb = C[:n_s, :n_s]
        Ci = np.linalg.inv(Cb)  # small upper-triangular inverse (device: back-substitution)
        # S-coefficients of L S_l for l < J:  L S_l = sum_{i<J} Ci[i,l] L W_i,  L W_i = S C H[:, i]
        LS = np.zeros((n_s, J), complex)
        if J > 0:
            LS = Cb @ H[:n_s, :J] @ Ci[:J, :J]
        # X = L W_J - sigma W_J - sum_{k<J} conj(H[J,k]) W_k
        #   = C[J,J] L S_J + sum_{l<J} C[l,J] L S_l - sigma W_J - ...
        aX = LS @ Cb[:J, J] if J > 0 else np.zeros(n_s, complex)
        aX = aX - sigma * Cb[:, J]
        for k in range(J):
            aX = aX - np.conj(H[J, k]) * Cb[:, k]
        bX1 = Cb[J, J]
        # Z = (L - sigma) X = sum_{l<J} aX[l] L S_l + aX[J] L S_J + bX1 L^2 S_J - sigma X
        aZ = (LS @ aX[:J] if J > 0 else np.zeros(n_s, complex)) - sigma * aX
        bZ1 = aX[J] - sigma * bX1
        bZ2 = bX1
        # ---- the pass: one read of S_0..S_J, stencils of S_J only ----
        SJ = S[J]
        L1 = apply(SJ)
        L2 = apply(L1)
        X = bX1 * L1
        Z = bZ2 * L2 + bZ1 * L1
        for l in range(n_s):
            X = X + aX[l] * S[l]
            Z = Z + aZ[l] * S[l]
        last = J + 2 >= mm  # only one more vector needed: no Z
        gX = np.array([np.vdot(S[l], X) for l in range(n_s)])
        gZ = np.array([np.vdot(S[l], Z) for l in range(n_s)])
        xx, xz, zz = np.vdot(X, X), np.vdot(X, Z), np.vdot(Z, Z)
        # ---- coefficient space (device: one small kernel) ----
        S.append(X)
        G[:n_s, J + 1] = gX
        G[J + 1, :n_s] = np.conj(gX)
        G[J + 1, J + 1] = xx
        p = Cb.conj().T @ gX  # p_k = W_k^H X
        nu1 = np.sqrt(max((xx - np.vdot(p, p)).real, 0.0))
        C[:, J + 1] = 0
        C[J + 1, J + 1] = 1.0
        C[:n_s, J + 1] -= Cb @ p
        C[:, J + 1] /= nu1
        # H column J: W_k^H L W_J = p_k + sigma delta_kJ + conj(H[J,k]) (k<J); H[J+1,J] = nu1
        for k in range(n_s):
            H[k, J] = p[k] + (sigma if k == J else 0.0) + (np.conj(H[J, k]) if k < J else 0.0)
        H[J + 1, J] = nu1
        if last:
            J += 1
            break
        S.append(Z)
        G[:n_s, J + 2] = gZ
        G[J + 2, :n_s] = np.conj(gZ)
        G[J + 1, J + 2] = xz
        G[J + 2, J + 1] = np.conj(xz)
        G[J + 2, J + 2] = zz
        n2 = J + 2
        C2 = C[:n2, :n2]
        q = C2.conj().T @ G[:n2, J + 2]  # q_k = W_k^H Z, k <= J+1
        nu2 = np.sqrt(max((zz - np.vdot(q, q)).real, 0.0))
        C[:, J + 2] = 0
        C[J + 2, J + 2] = 1.0
        C[:n2, J + 2] -= C2 @ q
        C[:, J + 2] /= nu2
        # H column J+1: L W_{J+1} = (L X - sum_{k<=J} p_k L W_k) / nu1
        #   L X = Z + sigma X;  L W_J = X + sigma W_J + sum_{k<J} conj(H[J,k]) W_k;
        #   L W_k (k<J) = sum_l H[l,k] W_l.  Project on W_i (i <= J+2):
        #   W_i^H X = p_i (i<=J), nu1 (i=J+1), 0 (i=J+2);  W_i^H Z = q_i (i<=J+1), nu2 (i=J+2)
        wx = np.zeros(J + 3, complex)
        wx[:n_s] = p
        wx[J + 1] = nu1
        wz = np.zeros(J + 3, complex)
        wz[:n2] = q
        wz[J + 2] = nu2
        col = wz + sigma * wx
        lwj = wx.copy()
        lwj[J] += sigma
        for k in range(J):
            lwj[k] += np.conj(H[J, k])
        col -= p[J] * lwj
        for k in range(J):
            col[:J + 1] -= p[k] * H[:J + 1, k]
        col /= nu1
        H[:J + 3, J + 1] = col
        if shift:
            sigma = H[J + 1, J + 1].real
        J += 2
    if raw:
        return S, C, H, G, beta
    # reference T: alpha_j on the diagonal (j < m-1), norms on the off-diagonals, T[m-1,m-1] = 0
    T = np.zeros((m, m))
    for j in range(m - 1):
        T[j, j] = H[j, j].real
        T[j + 1, j] = T[j, j + 1] = H[j + 1, j].real
    Cm = C[:m, :m]
    return T, S[:m], Cm, beta, G[:m, :m]


def krylov2(apply, u, t, m, func):
    T, S, C, beta, G = lanczos2(apply, u, m)
    lam, Q = np.linalg.eigh(T)
    c = Q @ (np_ref._f(func, lam, t) * Q[0, :])
    coef = C @ c  # over the stored vectors
    out = np.zeros_like(S[0])
    for l in range(m):
        out = out + coef[l] * S[l]
    return beta * out, C, G


def tail_coefficients(S, C, H, beta, a, l2, m, t, func):
    """Fused-tail end game of the two-vector scheme (the device's k_p2tail + k_tail):
    S_0..S_j stored (j = m-2), W = S C orthonormal, H columns < j known.  One alpha
    pass over S_j measures a = S_j^H L S_j and l2 = ||L S_j||^2; with y = L S_j,
      t_k = W_k^H y = sum_i conj(H[i,k]) D[i,j]             (k < j, D = C^-1)
      t_j = conj(C_jj) (a - sum_{i<j} conj(D[i,j]) t_i)
      lw  = -C_jj H[:, :j] D[:j, j]      (L W_j = C_jj y + sum_k lw_k W_k)
      H[k,j] = C_jj t_k + lw_k,  beta_{j+1} = |C_jj| sqrt(l2 - sum_k |t_k|^2)
      W_{j+1} = C_jj (y - sum_k t_k W_k) / beta_{j+1}
    returns (coef over S_0..S_j, coefficient of y, T)."""
    j = m - 2
    n = j + 1
    Cj = C[:n, :n]
    D = np.linalg.inv(Cj)
    cjj = Cj[j, j]
    tk = np.zeros(n, complex)
    for k in range(j):
        tk[k] = np.sum(np.conj(H[:k + 2, k]) * D[:k + 2, j])
    tk[j] = np.conj(cjj) * (a - np.sum(np.conj(D[:j, j]) * tk[:j]))
    lw = -cjj * (H[:n, :j] @ D[:j, j]) if j > 0 else np.zeros(n, complex)
    Hj = cjj * tk + lw
    bet = abs(cjj) * np.sqrt(max(l2 - np.sum(np.abs(tk) ** 2), 0.0))
    T = np.zeros((m, m))
    for i in range(j):
        T[i, i] = H[i, i].real
        T[i + 1, i] = T[i, i + 1] = H[i + 1, i].real
    T[j, j] = Hj[j].real
    T[j + 1, j] = T[j, j + 1] = bet
    lam, Q = np.linalg.eigh(T)
    c = Q @ (np_ref._f(func, lam, t) * Q[0, :])
    # result = beta (sum_{k<=j} c_k W_k + c_{j+1} W_{j+1})
    cw = c[:n] - c[j + 1] * cjj * tk / bet
    coefS = beta * (Cj @ cw)
    cy = beta * c[j + 1] * cjj / bet
    return coefS, cy, T


def krylov2_tail(apply, u, t, m, func):
    S, C, H, G, beta = lanczos2(apply, u, m, nstore=m - 1, raw=True)
    j = m - 2
    y = apply(S[j])
    a, l2 = np.vdot(S[j], y), np.vdot(y, y).real
    coefS, cy, T = tail_coefficients(S, C, H, beta, a, l2, m, t, func)
    out = cy * y
    for l in range(j + 1):
        out = out + coefS[l] * S[l]
    return out, T


def nlse_steps2_tail(dim, n, dx, u, dt, nsteps, m):
    nz = n if dim == 3 else 1
    ap = lambda v: np_ref.laplacian_apply(dim, n, n, nz, dx, dx, v)
    u = u.ravel().astype(np.complex128).copy()
    for _ in range(nsteps):
        r = np_ref.nonlin_half(u, dt)
        b, _ = krylov2_tail(ap, r, -1j * dt, m, np_ref.F_EXP_ABS)
        u = np_ref.nonlin_half(b, dt)
    return u


def nlse_steps2(dim, n, dx, u, dt, nsteps, m):
    nz = n if dim == 3 else 1
    ap = lambda v: np_ref.laplacian_apply(dim, n, n, nz, dx, dx, v)
    u = u.ravel().astype(np.complex128).copy()
    worst = 0.0
    for _ in range(nsteps):
        r = np_ref.nonlin_half(u, dt)
        b, C, G = krylov2(ap, r, -1j * dt, m, np_ref.F_EXP_ABS)
        Wg = C.conj().T @ G @ C  # Gram of W
        worst = max(worst, np.abs(Wg - np.eye(m)).max())
        u = np_ref.nonlin_half(b, dt)
    return u, worst


def main():
    rng = np.random.default_rng(0)
    for dim, n, m in ((3, 16, 16), (3, 20, 10), (2, 48, 16), (3, 16, 25), (2, 40, 30)):
        L = 10.0
        dx = 2 * L / (n - 1)
        shape = (n,) * dim
        x = np.linspace(-L, L, n)
        grids = np.meshgrid(*([x] * dim), indexing="ij")
        r2 = sum(g * g for g in grids)
        u = np.exp(-r2 / 4.0) * (1 + 0.1j) + 1e-3 * (rng.standard_normal(shape) + 1j * rng.standard_normal(shape))
        u = u.ravel()
        u /= np.sqrt(np.sum(np.abs(u) ** 2) * dx ** dim)
        dt = 1e-3
        nz = n if dim == 3 else 1
        ref = np_ref.nlse_steps(dim, n, n, nz, dx, dx, u, dt, 20, m)
        got, worst = nlse_steps2(dim, n, dx, u, dt, 20, m)
        rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
        print(f"dim={dim} n={n} m={m}: 20 steps rel L2 vs MGS oracle {rel:.2e}, max |W^H W - I| {worst:.2e}")


if __name__ == "__main__":
    main()
