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


# ---- s-step generalisation: one, two or three new vectors per pass ----------------
#
# A pass at J with ns new vectors writes V_1 = (L - sigma) W_J - sum_{k<J} conj(H[J,k]) W_k
# and V_{i+1} = (L - sigma) V_i, each V_i = sum_{l<=J} a_i[l] S_l + sum_p b_i[p] L^p S_J
# (p = 1..i: a radius-ns stencil of S_J only), and reduces S_l^H V_i and the Gram
# V_a^H V_b.  In coefficient space, with q^(i) = W^H V_i and nu_i its new norm,
#   C[:, J+i] = (e_{J+i} - C q^(i)) / nu_i,   D[:, J+i] = (q^(i), nu_i)
#   H[:, J] = q^(1) + sigma e_J + conj(H[J, :J]) (+ nu_1 e_{J+1})
#   H[:, J+i-1] = (wv_i + sigma wv_{i-1} - sum_{k < J+i-1} q^(i-1)_k H[:, k]) / nu_{i-1}   (i >= 2)
# (wv_i = (q^(i), nu_i)), and the next pass's W-coefficients follow the recurrence
#   w' = H[:, :j] w[:j] + w_j lw - sigma w,  b'_1 = w_j C_jj - sigma b_1,
#   b'_{p+1} = b_p - sigma b_{p+1}    (L W_j = C_jj L S_j + lw, lw = -C_jj H[:, :j] D[:j, j]).


def sstep_schedule(nstore, p3=(2, 5)):
    """[(J, ns)] of the passes storing S_0..S_{nstore-1}: two vectors per pass, three at
    the J in p3 (the device: J = 2 and 5, both or neither, when the basis reaches S_8,
    so the two-vector passes stay at even J), the last pass one or two; p3="all":
    three wherever they fit (from J = 1)."""
    use3 = p3 == "all" or nstore - 1 >= 8
    out, J = [], 0
    while J + 1 < nstore:
        left = nstore - 1 - J
        three = (J >= 1 if p3 == "all" else J in p3) and use3 and left >= 3
        ns = 3 if three else min(2, left)
        out.append((J, ns))
        J += ns
    return out


def pass_coefficients(C, D, H, sigma, j, ns):
    """S-basis coefficients a_i[0..j] and stencil coefficients b_i[1..i] of V_1..V_ns."""
    cjj = C[j, j]
    lw = -cjj * (H[:j + 1, :j] @ D[:j, j]) if j > 0 else np.zeros(j + 1, complex)
    w = lw.copy()
    w[j] -= sigma
    w[:j] -= np.conj(H[j, :j])
    b = np.zeros(6, complex)  # b[p]: coefficient of L^p S_j, p = 1..ns (ns <= 5)
    b[1] = cjj
    A, B = [], []
    for i in range(ns):
        A.append(C[:j + 1, :j + 1] @ w)
        B.append(b.copy())
        wn = (H[:j + 1, :j] @ w[:j] if j > 0 else np.zeros(j + 1, complex)) + w[j] * lw - sigma * w
        bn = np.zeros(6, complex)
        bn[1] = w[j] * cjj - sigma * b[1]
        for p in range(1, 5):
            bn[p + 1] = b[p] - sigma * b[p + 1]
        w, b = wn, bn
    return A, B


def coef_update(C, D, H, sigma, J, ns, g, G):
    """New columns of C, D, H from the pass's sums g[i][l] = S_l^H V_i (l <= J) and
    G[a][b] = V_a^H V_b; returns the next shift."""
    qs, nus = [], []
    for i in range(ns):
        n = J + 1 + i
        sv = np.concatenate([g[i], [G[a][i] for a in range(i)]])  # S_l^H V_i, l < n
        q = C[:n, :n].conj().T @ sv
        nu = np.sqrt(max((G[i][i] - np.vdot(q, q)).real, 0.0))
        C[:, n] = 0
        C[n, n] = 1.0
        C[:n, n] -= C[:n, :n] @ q
        C[:, n] /= nu
        D[:n, n] = q
        D[n, n] = nu
        qs.append(q)
        nus.append(nu)
    q1 = qs[0]
    for k in range(J + 1):
        H[k, J] = q1[k] + (sigma if k == J else 0.0) + (np.conj(H[J, k]) if k < J else 0.0)
    H[J + 1, J] = nus[0]
    for i in range(1, ns):
        c = J + i  # column J+i-1+1: L W_{J+i}
        n = c + 2
        wv = np.zeros(n, complex)
        wv[:c + 1] = qs[i]
        wv[c + 1] = nus[i]
        wp = np.zeros(n, complex)
        wp[:c] = qs[i - 1]
        wp[c] = nus[i - 1]
        col = wv + sigma * wp
        for k in range(c):
            col[:k + 2] -= qs[i - 1][k] * H[:k + 2, k]
        H[:n, c] = col / nus[i - 1]
    return H[J + ns - 1, J + ns - 1].real if ns > 1 else sigma


def lanczos_s(apply, u, m, p3=(2, 5), nstore=None, raw=False, sched=None):
    """lanczos2 with the s-step schedule (sstep_schedule, or an explicit [(J, ns)]); same returns."""
    u = np.asarray(u, dtype=np.complex128)
    beta = np.linalg.norm(u)
    S = [u / beta]
    M = m + 5
    C = np.zeros((M, M), complex)
    D = np.zeros((M, M), complex)
    H = np.zeros((M, M), complex)
    C[0, 0] = D[0, 0] = 1.0
    sigma = np.vdot(S[0], apply(S[0])).real  # the start's alpha pass
    mm = m if nstore is None else nstore
    for J, ns in (sched if sched is not None else sstep_schedule(mm, p3)):
        A, B = pass_coefficients(C, D, H, sigma, J, ns)
        Lp = [None, apply(S[J])]
        for p in range(2, ns + 1):
            Lp.append(apply(Lp[-1]))
        V = []
        for i in range(ns):
            v = sum(B[i][p] * Lp[p] for p in range(1, i + 2))
            for l in range(J + 1):
                v = v + A[i][l] * S[l]
            V.append(v)
        g = [np.array([np.vdot(S[l], V[i]) for l in range(J + 1)]) for i in range(ns)]
        G = [[np.vdot(V[a], V[b]) for b in range(ns)] for a in range(ns)]
        sigma = coef_update(C, D, H, sigma, J, ns, g, G)
        S.extend(V)
    if raw:
        return S, C, H, None, beta
    T = np.zeros((m, m))
    for j in range(m - 1):
        T[j, j] = H[j, j].real
        T[j + 1, j] = T[j, j + 1] = H[j + 1, j].real
    return T, S[:m], C[:m, :m], beta, None


def krylov_s_tail(apply, u, t, m, func, p3=(2, 5), sched=None):
    S, C, H, _, beta = lanczos_s(apply, u, m, p3, nstore=m - 1, raw=True, sched=sched)
    j = m - 2
    y = apply(S[j])
    a, l2 = np.vdot(S[j], y), np.vdot(y, y).real
    coefS, cy, T = tail_coefficients(S, C, H, beta, a, l2, m, t, func)
    out = cy * y
    for l in range(j + 1):
        out = out + coefS[l] * S[l]
    return out, T
