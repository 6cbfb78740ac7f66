"""The reverse sweep of the unrolled constraint solve (tests/unrolled_solver_ref.py, the algorithm the
HIP VJP's unrolled mode implements) against central finite differences of the same truncated solve.

jax.grad through mjx.step (train_apg.py:187-189, CG 4/4) differentiates MJX's solver iterations as
executed: branch decisions (active sets, bracket moves, the early exits) fixed, every arithmetic
step differentiated. A finite difference of the forward at a point where no decision flips
within +-eps measures exactly that derivative.
"""
import numpy as np
import pytest

from unrolled_solver_ref import Problem, solve, solve_vjp


def _problem(seed, nv=9, nefc=14, **kw):
    rng = np.random.default_rng(seed)
    A = rng.normal(size=(nv, nv))
    M = A @ A.T / nv + np.eye(nv)
    J = rng.normal(size=(nefc, nv))
    D = rng.uniform(5.0, 400.0, nefc)
    f = rng.normal(size=nv) * 5
    qsm = np.linalg.solve(M, f)
    aref = J @ qsm + rng.normal(size=nefc) * 3.0  # roughly half the rows active at the smooth solution
    qws = qsm + rng.normal(size=nv)
    return Problem(M, J, D, aref, f, qws, meaninertia=float(np.trace(M) / nv), **kw)


def _signature(tape):
    return ([tuple(u["act"]) for u in tape["ups"]],
            [(len(it["sets"]), tuple(np.round(it["rec"][:len(it["sets"])], 12)), it["alpha"] == 0.0) for it in tape["its"]],
            tape["wsel"])


@pytest.mark.parametrize("solver,it,ls", [("cg", 4, 4), ("newton", 1, 4), ("cg", 10, 20), ("newton", 3, 4)])
def test_unrolled_vjp_matches_finite_differences(solver, it, ls):
    checked = 0
    for seed in range(20):
        P = _problem(seed, solver=solver, iterations=it, ls_iterations=ls)
        q, qfc, tape = solve(P)
        rng = np.random.default_rng(100 + seed)
        qb, qfb = rng.normal(size=q.shape), rng.normal(size=q.shape)
        Mb, Jb, Db, arb, fb = solve_vjp(P, tape, qb, qfb)
        dM = rng.normal(size=P.M.shape)
        dM = dM + dM.T
        dirs = dict(M=dM, J=rng.normal(size=P.J.shape), D=rng.normal(size=P.D.shape) * 10,
                    aref=rng.normal(size=P.aref.shape), f=rng.normal(size=P.f.shape))
        an = np.sum(Mb * dM) + np.sum(Jb * dirs["J"]) + Db @ dirs["D"] + arb @ dirs["aref"] + fb @ dirs["f"]
        eps = 1e-7

        def run(sign):
            Q = Problem(P.M + sign * eps * dM, P.J + sign * eps * dirs["J"], P.D + sign * eps * dirs["D"],
                        P.aref + sign * eps * dirs["aref"], P.f + sign * eps * dirs["f"], P.qws, solver=solver,
                        iterations=it, ls_iterations=ls, meaninertia=1.0 / (P.scale * P.M.shape[0]))
            return solve(Q)

        qp, fp, tp = run(1)
        qm, fm, tm = run(-1)
        if _signature(tp) != _signature(tape) or _signature(tm) != _signature(tape):
            continue  # a decision flips within eps: not a differentiable point
        fd = (qb @ (qp - qm) + qfb @ (fp - fm)) / (2 * eps)
        assert an == pytest.approx(fd, rel=1e-5, abs=1e-6 * (1 + abs(fd))), (seed, an, fd)
        checked += 1
    assert checked >= 10


def test_truncated_solve_is_not_converged():
    """The case the unrolled mode exists for: CG 4/4 stops with a nonzero gradient, so the
    implicit-function derivative at the final active set differs from the unrolled one."""
    P = _problem(3, solver="cg", iterations=4, ls_iterations=4)
    q, qfc, tape = solve(P)
    assert np.linalg.norm(tape["ups"][-1]["grad"]) > 1e-3 * np.linalg.norm(P.f)
