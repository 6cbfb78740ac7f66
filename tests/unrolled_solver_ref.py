"""numpy restatement of the constraint solve as the kernel runs it, with a tape, and the reverse sweep
of its unrolled iterations (the derivative jax.grad takes through MJX's fixed-count solver; train_apg.py:187-189
differentiates mjx.step with CG 4/4). TEST INFRASTRUCTURE: the algorithm reference of the HIP
VJP's unrolled mode (csrc/adjoint.hip `adj_solver_unrolled`), checked here against finite differences.

Forward = MJX solver.py `solve` + `_linesearch` (restated in oracle/physics.hpp Solver), with the
kernel's exact-segment and bracket-width exits (csrc/step_kernels.hip solver_linesearch).

Line-search derivative: every candidate step of the zoom search is either the Newton point of some
point p, alpha' = p.alpha - f'(p)/f''(p) = -Q1(A)/Q2(A) with A = p's active set, Q1 = c1 + sum_A D Jv jar,
Q2 = c2 + sum_A D Jv^2 (independent of p.alpha: d alpha'/d p.alpha = 1 - Q2/Q2 = 0), or a midpoint.
So the accepted alpha = sum_j w_j N(A_j) over the active sets the search visited ("recipe" w), and
d alpha = sum_j w_j (-dQ1_j / Q2_j + N_j dQ2_j / Q2_j).
"""
import numpy as np

MINVAL = 1e-15


class Problem:
    def __init__(self, M, J, D, aref, f, qws, solver="cg", iterations=4, ls_iterations=4, tolerance=1e-8,
                 ls_tolerance=0.01, meaninertia=1.0):
        self.M, self.J, self.D, self.aref, self.f, self.qws = M, J, D, aref, f, qws
        self.solver, self.iterations, self.ls_iterations = solver, iterations, ls_iterations
        self.tol, self.ls_tol = tolerance, ls_tolerance
        self.scale = 1.0 / (meaninertia * max(1, M.shape[0]))


def _cost(P, q, qsm):
    jar = P.J @ q - P.aref
    return 0.5 * (P.M @ q - P.f) @ (q - qsm) + 0.5 * np.sum(P.D * jar * jar * (jar < 0))


def _precond(P, act, g):
    if P.solver == "cg":
        return np.linalg.solve(P.M, g)
    H = P.M + (P.J * (P.D * act)[:, None]).T @ P.J
    return np.linalg.solve(H, g)


def _update(P, q):
    jar = P.J @ q - P.aref
    act = jar < 0
    force = -P.D * jar * act
    qfc = P.J.T @ force
    grad = P.M @ q - P.f - qfc
    return dict(q=q, jar=jar, act=act, force=force, qfc=qfc, grad=grad, Mg=_precond(P, act, grad))


def _linesearch(P, q, s):
    """Returns (alpha, weights over sets, sets [(active mask, Q1, Q2)], jar, Jv)."""
    jar, Jv, Mv = P.J @ q - P.aref, P.J @ s, P.M @ s
    c1, c2 = s @ (P.M @ q - P.f), s @ Mv
    sets = []

    def point(a, rec):
        A = jar + a * Jv < 0
        Q1 = c1 + np.sum((P.D * Jv * jar)[A])
        Q2 = c2 + np.sum((P.D * Jv * Jv)[A])
        d1 = Q2 + (MINVAL if Q2 == 0 else 0.0)
        cost = a * c1 + 0.5 * a * a * c2 + 0.5 * np.sum((P.D * (jar + a * Jv) ** 2)[A])
        return dict(a=a, d0=Q1 + a * Q2, d1=d1, cost=cost, A=A, Q1=Q1, Q2=Q2, rec=rec)

    def newton(p):
        sets.append((p["A"], p["Q1"], p["Q2"]))
        rec = np.zeros(64)
        rec[len(sets) - 1] = 1.0
        return point(p["a"] - p["d0"] / p["d1"], rec)

    gtol = P.tol * P.ls_tol * np.linalg.norm(s) / P.scale
    p0 = point(0.0, np.zeros(64))
    qn = newton(p0)
    if np.array_equal(p0["A"], qn["A"]):  # exact segment (kernel exit): q is the minimiser
        return qn["a"], qn["rec"], sets, jar, Jv
    lo, hi = (qn, p0) if qn["d0"] < p0["d0"] else (p0, qn)
    for _ in range(P.ls_iterations):
        if (lo["d0"] < 0 and lo["d0"] > -gtol) or (hi["d0"] > 0 and hi["d0"] < gtol):
            break
        if abs(hi["a"] - lo["a"]) <= 1e-6 * max(abs(lo["a"]), abs(hi["a"])):
            break
        lo_n, hi_n = newton(lo), newton(hi)
        mid = point(0.5 * (lo["a"] + hi["a"]), 0.5 * (lo["rec"] + hi["rec"]))
        s1 = lo["d0"] > 0 or lo["d0"] < lo_n["d0"]
        if s1:
            lo = lo_n
        s2 = mid["d0"] < 0 and lo["d0"] < mid["d0"]
        if s2:
            lo = mid
        s3 = hi["d0"] < 0 or hi["d0"] > hi_n["d0"]
        if s3:
            hi = hi_n
        s4 = mid["d0"] > 0 and hi["d0"] > mid["d0"]
        if s4:
            hi = mid
        if not (s1 or s2 or s3 or s4):
            break
    c0 = 0.0
    if not (lo["cost"] < c0 or hi["cost"] < c0):
        return 0.0, np.zeros(64), sets, jar, Jv
    best = lo if lo["cost"] < hi["cost"] else hi
    return best["a"], best["rec"], sets, jar, Jv


def solve(P):
    """Forward with tape. Returns (qacc, qfrc_constraint, tape)."""
    qsm = np.linalg.solve(P.M, P.f)
    wsel = 0 if _cost(P, P.qws, qsm) < _cost(P, qsm, qsm) else 1
    q = (P.qws if wsel == 0 else qsm).copy()
    u = _update(P, q)
    cost = _cost(P, q, qsm)
    ups, its = [u], []
    s = -u["Mg"]
    go = P.iterations == 1 or (P.iterations > 0 and P.scale * np.linalg.norm(u["grad"]) >= P.tol)
    k = 0
    while go:
        alpha, rec, sets, jar, Jv = _linesearch(P, q, s)
        its.append(dict(q=q.copy(), s=s.copy(), alpha=alpha, rec=rec, sets=sets, jar=jar, Jv=Jv))
        k += 1
        if alpha == 0.0:
            break
        q = q + alpha * s
        un = _update(P, q)
        old, cost = cost, _cost(P, q, qsm)
        beta, num, den = 0.0, 0.0, 0.0
        if P.solver == "cg":
            num = un["grad"] @ (un["Mg"] - u["Mg"])
            den = u["grad"] @ u["Mg"]
            beta = max(0.0, num / max(MINVAL, den))
            s = -un["Mg"] + beta * s
        else:
            s = -un["Mg"]
        un.update(beta=beta, num=num, den=den)
        ups.append(un)
        u = un
        go = P.iterations != 1 and k < P.iterations and P.scale * (old - cost) >= P.tol and \
            P.scale * np.linalg.norm(u["grad"]) >= P.tol
    return q, ups[-1]["qfc"], dict(ups=ups, its=its, wsel=wsel, qsm=qsm)


def solve_vjp(P, tape, qacc_b, qfc_b):
    """Cotangents of (M, J, D, aref, f) from those of the final qacc and qfrc_constraint."""
    M, J, D = P.M, P.J, P.D
    Mb, Jb = np.zeros_like(M), np.zeros_like(J)
    Db, arb, fb = np.zeros_like(D), np.zeros_like(D), np.zeros_like(P.f)
    ups, its = tape["ups"], tape["its"]
    K = len(ups) - 1
    qb = qacc_b.copy()
    sb = np.zeros_like(qb)     # cotangent of the search direction leaving update k
    gb = np.zeros_like(qb)     # of grad_k (from beta_{k+1}'s denominator)
    Mgb = np.zeros_like(qb)    # of Mgrad_k
    for k in range(K, -1, -1):
        u = ups[k]
        # direction s_k = -Mg_k + beta_k s_{k-1} (k >= 1), s_0 = -Mg_0: only if s_k was used
        sb_prev = np.zeros_like(qb)
        Mgb_prev, gb_prev = np.zeros_like(qb), np.zeros_like(qb)
        if k < len(its):
            Mgb = Mgb - sb
            if P.solver == "cg" and k >= 1:
                up = ups[k - 1]
                betab = sb @ its[k - 1]["s"]
                sb_prev += u["beta"] * sb
                den = max(MINVAL, u["den"])
                if u["num"] / den > 0:
                    nb = betab / den
                    gb = gb + nb * (u["Mg"] - up["Mg"])
                    Mgb = Mgb + nb * u["grad"]
                    Mgb_prev -= nb * u["grad"]
                    if u["den"] > MINVAL:
                        denb = -betab * u["num"] / den ** 2
                        gb_prev += denb * up["Mg"]
                        Mgb_prev += denb * up["grad"]
        # Mg_k = P_k^-1 grad_k
        if np.any(Mgb):
            act = u["act"]
            if P.solver == "cg":
                lam = np.linalg.solve(M, Mgb)
                Mb -= np.outer(lam, u["Mg"])
            else:
                H = M + (J * (D * act)[:, None]).T @ J
                lam = np.linalg.solve(H, Mgb)
                Hb = -np.outer(lam, u["Mg"])
                Mb += Hb
                Jl, Jm = J @ lam, J @ u["Mg"]
                Db -= act * Jl * Jm
                Jb -= (D * act)[:, None] * (np.outer(Jm, lam) + np.outer(Jl, u["Mg"]))
            gb = gb + lam
        # grad_k = M q_k - f - J' force_k (+ the final qfrc_constraint's cotangent at k = K)
        qfcb = -gb + (qfc_b if k == K else 0.0)
        fb -= gb
        qb += M @ gb
        Mb += np.outer(gb, u["q"])
        forceb = J @ qfcb
        Jb += np.outer(u["force"], qfcb)
        act = u["act"]
        Db -= act * forceb * u["jar"]
        jarb = -(act * forceb * D)
        Jb += np.outer(jarb, u["q"])
        qb += J.T @ jarb
        arb -= jarb
        if k == 0:
            break
        # q_k = q_{k-1} + alpha s_{k-1}
        it = its[k - 1]
        s = it["s"]
        alphab = qb @ s
        sb_prev += it["alpha"] * qb
        qprev = it["q"]
        # alpha = sum_j w_j N_j,  N_j = -Q1_j / Q2_j
        c1b = c2b = 0.0
        ra, rb = np.zeros_like(D), np.zeros_like(D)
        for j, (A, Q1, Q2) in enumerate(it["sets"]):
            w = it["rec"][j]
            if w == 0.0:
                continue
            q1b = alphab * w * (-1.0 / Q2)
            q2b = alphab * w * (Q1 / Q2 ** 2)
            c1b += q1b
            c2b += q2b
            ra += A * q1b
            rb += A * q2b
        jar, Jv = it["jar"], it["Jv"]
        Db += ra * Jv * jar + rb * Jv * Jv
        Jvb = ra * D * jar + 2 * rb * D * Jv
        jarb = ra * D * Jv
        Ms = M @ s
        sb_prev += c1b * (M @ qprev - P.f) + 2 * c2b * Ms
        qb += c1b * (M @ s)
        Mb += c1b * np.outer(s, qprev) + c2b * np.outer(s, s)
        fb -= c1b * s
        Jb += np.outer(Jvb, s)
        sb_prev += J.T @ Jvb
        Jb += np.outer(jarb, qprev)
        qb += J.T @ jarb
        arb -= jarb
        sb, gb, Mgb = sb_prev, gb_prev, Mgb_prev
    if tape["wsel"] == 1:  # q_0 = qacc_smooth = M^-1 f
        lam = np.linalg.solve(M, qb)
        fb += lam
        Mb -= np.outer(lam, tape["qsm"])
    return Mb, Jb, Db, arb, fb
