"""scipy 1.7.3 `cg(A, b, x0, tol, maxiter, M, callback, atol=None)` restated in NumPy.

TEST INFRASTRUCTURE (see oracle/__init__.py).

scipy 1.7.3 (pinned by the reference, environment.yml:11) runs the Fortran
reverse-communication template CGREVCOM with a python driver.  Semantics kept
here, as used at src/sGDML/sgdml/solvers/iterative_solver.py:995-1005:

* atol=None ("legacy"): if ||A x0 - b|| <= tol return x0 (info 0, no callback);
  otherwise atol = tol * ||b|| (tol if ||b|| == 0).
* r0 = b - A x0 (skipped when ||x0|| == 0); if ||r0|| < atol: converged, 0 iterations.
* iteration ITER: z = M r; rho = r.z; p = z (ITER 1) or z + (rho/rho1) p;
  q = A p; alpha = rho / p.q; x += alpha p; r -= alpha q.
* stop test: resid = ||r|| <= atol; when it passes and ITER > 1 the wrapper
  recomputes r = b - A x and tests again ("avoid accumulating rounding error").
* ITER == maxiter without convergence -> info = maxiter.
* callback(x) fires at the start of iterations 2..m and once after the loop; the
  caller-frame local `resid` seen by a callback is the previous stop-test value.
"""
from __future__ import annotations

import numpy as np


def cg_legacy(matvec, b, x0=None, tol=1e-5, maxiter=None, psolve=None, callback=None,
              dot_fn=None):
    """Returns (x, info, trace, iters).  trace[0] = ||r0||, trace[j] = stop-test ||r_j||."""
    b = np.asarray(b, dtype=np.float64)
    n = b.size
    maxiter = 10 * n if maxiter is None else int(maxiter)
    dot = dot_fn if dot_fn is not None else (lambda u, v: float(np.dot(u, v)))
    norm = lambda u: float(np.sqrt(dot(u, u)))
    psolve = psolve if psolve is not None else (lambda v: v)
    x = np.zeros(n) if x0 is None else np.array(x0, dtype=np.float64)
    bnrm2 = norm(b)
    # _get_atol legacy
    resid0 = norm(matvec(x) - b)
    if resid0 <= tol:
        return x, 0, np.array([resid0]), 0
    atol = tol if bnrm2 == 0 else tol * bnrm2
    r = b.copy()
    if norm(x) != 0.0:
        r = r - matvec(x)
    trace = [norm(r)]
    if trace[0] < atol:
        if callback is not None:
            callback(x)
        return x, 0, np.array(trace), 0
    p = None
    rho1 = None
    it = 0
    info = 0
    resid = trace[0]
    while True:
        it += 1
        if callback is not None and it > 1:
            callback(x)
        z = psolve(r)
        rho = dot(r, z)
        if it > 1:
            beta = rho / rho1
            p = z + beta * p
        else:
            p = z.copy()
        q = matvec(p)
        alpha = rho / dot(p, q)
        x = x + alpha * p
        r = r - alpha * q
        resid = norm(r)
        conv = resid <= atol
        if conv and it > 1:
            r = b - matvec(x)
            resid = norm(r)
            conv = resid <= atol
        trace.append(resid)
        if conv:
            info = 0
            break
        if it == maxiter:
            info = maxiter
            break
        rho1 = rho
    if callback is not None:
        callback(x)
    return x, info, np.array(trace), it
