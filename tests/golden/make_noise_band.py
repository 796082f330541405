"""Noise band of the golden PCG solves: how far the reference's own algorithm moves under a
change of floating-point summation order alone.

For every golden solve of the reference (tests/golden/sgdml_*.npz, the same list as
tests/test_gpu_golden.py) the CPU oracle (oracle/: the reference's preconditioner build,
operator and scipy-1.7.3 CG recurrence restated in NumPy) is re-run with several
summation orders.  The reference's CG operator is the MATRIX-FREE K_op
(iterative_solver.py:383-445); a dense K @ v rounds differently (its errors scale with
||K|| ||v|| through the cancellations of the ill-conditioned K) and measurably shifts the
counts (+7 iterations on sgdml_ethanol_n270/cholesky for every BLAS order, 0 with
extended-precision products), so the variants are of the matrix-free operator:

  mf        oracle.sgdml.kernel_matvec_matrix_free, T.T @ (T @ r)   (the oracle's order)
  mf_rev    training points summed in reverse order, panel rows reversed
  mf_split  descriptor dot products in 4 chunks added in chunk order, 7-column-block panel
  mf_pair   pairwise einsum contractions, 512-column tiles of the panel (the GPU's width)
  ld        dense K with extended-precision (np.longdouble) products, rounded once
            (N <= 621: near-exact arithmetic)

and the spread against the reference's recorded solve is written to noise_band.json
(plus two cases without a recorded trace: the reference's trained model
sgdml_model_ethanol_n621 -- iterations and alphas only -- and the multi-rank tests' RBF
system rbf_n1003/{none,pivchol,nystrom}, whose reference is the oracle's own BLAS-order
solve, since those tests compare W GPU ranks with one):
iteration-count differences and the iteration at which the running-minimum residual first
crosses every half decade.  tests/parity.py holds the GPU to this band (scaled, see there).

Inputs are the committed fixtures only (the reference is not imported).  CPU only:
    python tests/golden/make_noise_band.py            (~5 min on 8 cores)
"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO)]

from oracle.pcg import cg_legacy  # noqa: E402
from oracle.precon import (nystrom_panel, pivoted_cholesky, svd_panel,  # noqa: E402
                           woodbury_panel)
from oracle.sgdml import assemble_kernel, descriptors, kernel_matvec_matrix_free  # noqa: E402

GOLDEN = REPO / "tests" / "golden"
PRECONS_270 = ["cholesky", "random_scores", "lev_scores", "inverse_lev", "lev_random",
               "truncated_cholesky", "truncated_cholesky_custom", "rank_k_lev_scores",
               "rank_k_lev_scores_custom", "eigvec_precon"]
CASES = [("sgdml_ethanol_n270", p) for p in PRECONS_270] + [
    ("sgdml_ethanol_n270_perms", p) for p in ["cholesky", "random_scores",
                                              "truncated_cholesky_custom"]] + [
    ("sgdml_ethanol_n621", p) for p in ["cholesky", "random_scores", "truncated_cholesky"]] + [
    ("sgdml_ethanol_n2997", p) for p in ["cholesky", "random_scores"]] + [
    ("sgdml_nanotube_n3330", p) for p in ["cholesky", "random_scores"]]


def half_decade_crossings(trace, top):
    """Iteration (1-based) at which the running minimum first reaches each half decade
    below `top` (log10 of the first residual)."""
    env = np.minimum.accumulate(np.asarray(trace))
    out = {}
    for lvl in np.arange(np.floor(top) - 0.5, np.log10(env[-1]) - 1e-12, -0.5):
        hit = np.nonzero(env <= 10 ** lvl)[0]
        if hit.size:
            out[f"{lvl:.1f}"] = int(hit[0])
    return out


def dense_K(f):
    if "K" in f.files:
        return np.array(f["K"])
    if "R_desc" in f.files:
        return assemble_kernel(f["R_desc"], f["R_d_desc"], f["tril_perms_lin"], float(f["sig"]))
    # nanotube: columns of the matrix-free operator (the reference's K_op), symmetrised
    Rd, Rdd = descriptors(f["R"])
    n = f["y"].size
    K = np.empty((n, n))
    e = np.zeros(n)
    for j in range(n):
        e[j] = 1.0
        K[:, j] = kernel_matvec_matrix_free(Rd, Rdd, f["perms"], float(f["sig"]), e)
        e[j] = 0.0
    return 0.5 * (K + K.T)


def panel(f, precon, K, lam):
    n = K.shape[0]
    S = -K
    k = int(int(f["k_rot"]) / n * n)
    if precon == "cholesky":
        L, piv = pivoted_cholesky(lambda i: S[:, i] + lam * (np.arange(n) == i),
                                  np.diag(S).copy(), k)
        return woodbury_panel(L, lam)
    if precon.startswith("eigvec"):
        return svd_panel(S, k, lam)
    idx = f[f"{precon}__inducing_pts_idxs"]
    return nystrom_panel(S[:, idx], idx, lam, 1 if precon.endswith("_custom") else 0)


def kop_variant(Rd, Rdd, perms, sig, order, threads=1):
    """v -> K v by the reference's matrix-free formulation (predict.py:72-234, restated in
    oracle.sgdml.kernel_matvec_matrix_free) in a given summation order.  `threads` > 1 splits the
    independent output rows i over a thread pool (numpy releases the GIL in the per-row array
    work); every y[i] keeps its summation order, so the result is bitwise the same."""
    from oracle.sgdml import desc_perm

    M, D = Rd.shape
    n = int((1 + np.sqrt(8 * D + 1)) / 2)
    P = np.array([desc_perm(p) for p in np.atleast_2d(perms)])
    s_at, t_at = np.tril_indices(n, k=-1)
    Rt = Rd[:, P]
    jorder = np.arange(M)[::-1] if order == "mf_rev" else np.arange(M)
    chunks = np.array_split(np.arange(D), 4) if order == "mf_split" else [np.arange(D)]
    sqrt5 = np.sqrt(5.0)

    def dot_d(a, b):  # sum over the last (descriptor) axis in the variant's order
        if order == "mf_pair":
            return np.einsum("...d,...d->...", a, b, optimize=False)
        out = 0.0
        for c in chunks:
            out = out + np.sum(a[..., c] * b[..., c], axis=-1)
        return out

    def mv(x):
        X = np.asarray(x).reshape(M, n, 3)
        z = np.einsum("mdc,mdc->md", Rdd, X[:, t_at, :] - X[:, s_at, :])
        Zt = z[:, P][jorder]                                  # j order of the sums
        Rtj = Rt[jorder]
        y = np.empty((M, n, 3))

        def rows(i0, i1):
            for i in range(i0, i1):
                row(i, Zt, Rtj, y)
        if threads > 1:
            from concurrent.futures import ThreadPoolExecutor
            edges = np.linspace(0, M, 4 * threads + 1).astype(int)
            with ThreadPoolExecutor(threads) as ex:
                list(ex.map(lambda ab: rows(*ab), zip(edges[:-1], edges[1:])))
        else:
            rows(0, M)
        return y.reshape(-1)

    def row(i, Zt, Rtj, y):
        if True:
            diff = Rd[i][None, None, :] - Rtj                 # M x n_perms x D
            norm = sqrt5 * np.sqrt(dot_d(diff, diff))
            m = np.exp(-norm / sig) * 5.0 / (3.0 * sig ** 4)
            w = (sig ** 2 + sig * norm) * m
            a = dot_d(diff, Zt)
            if order == "mf_pair":
                F = (np.einsum("jp,jpd->d", 5.0 * m * a, diff, optimize=False)
                     - np.einsum("jp,jpd->d", w, Zt, optimize=False))
            else:
                # axis-0 sums of a C-contiguous array accumulate row after row: j order
                terms = (5.0 * m * a)[..., None] * diff - w[..., None] * Zt
                F = terms.reshape(-1, D).sum(axis=0)
            contrib = Rdd[i] * F[:, None]
            yi = np.zeros((n, 3))
            np.add.at(yi, t_at, contrib)
            np.add.at(yi, s_at, -contrib)
            y[i] = yi
    return mv


def make_gemv(A, order):
    """v -> A @ v in a given summation order over the columns of A."""
    n = A.shape[1]
    if order == "blas":
        return lambda v: A @ v
    if order == "rev":
        Ar = np.ascontiguousarray(A[:, ::-1])
        return lambda v: Ar @ v[::-1]
    if order in ("blk7", "blk512"):
        edges = (np.linspace(0, n, 8).astype(int) if order == "blk7"
                 else np.arange(0, n + 512, 512).clip(max=n))
        blocks = [(a, b, np.ascontiguousarray(A[:, a:b])) for a, b in zip(edges[:-1], edges[1:])
                  if b > a]

        def f(v):
            y = np.zeros(A.shape[0])
            for a, b, Ab in blocks:
                y = y + Ab @ v[a:b]
            return y
        return f
    if order == "pair":
        return lambda v: np.einsum("ij,j->i", A, v)
    if order == "ld":
        Al = A.astype(np.longdouble)
        return lambda v: (Al @ v.astype(np.longdouble)).astype(np.float64)
    raise ValueError(order)


def run_case(name, precon, orders):
    f = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
    K = dense_K(f)
    y, lam, tol = f["y"], float(f["lam"]), float(f["solver_tol"])
    n = y.size
    T, sp = panel(f, precon, K, lam)
    ref_it = int(f[f"{precon}__num_iters"])
    ref_tr = f[f"{precon}__trace"]
    top = float(np.log10(np.minimum.accumulate(ref_tr)[0]))
    ref_cross = half_decade_crossings(ref_tr, top)
    out = {"n": n, "ref_iters": ref_it, "variants": {}}
    Rd, Rdd = (f["R_desc"], f["R_d_desc"]) if "R_desc" in f.files else descriptors(f["R"])
    panel_order = {"mf": "blas", "mf_rev": "rev", "mf_split": "blk7", "mf_pair": "blk512",
                   "ld": "ld"}
    for order in orders:
        mvK = (make_gemv(K, "ld") if order == "ld"
               else kop_variant(Rd, Rdd, f["perms"], float(f["sig"]), order))
        mvT = make_gemv(T, panel_order[order])
        mvTt = make_gemv(np.ascontiguousarray(T.T), panel_order[order])
        x, info, tr, it = cg_legacy(lambda v: -mvK(v) + lam * v, y, tol=tol, maxiter=5 * n,
                                    psolve=lambda r: sp * ((r - mvTt(mvT(r))) / lam))
        cross = half_decade_crossings(tr[1:], top)
        dc = [abs(cross[k] - ref_cross[k]) for k in ref_cross if k in cross]
        out["variants"][order] = {
            "iters": int(it), "info": int(info), "d_iters": int(it - ref_it),
            "max_d_crossing": int(max(dc) if dc else 0),
            "rel_dalpha": float(np.linalg.norm(-x - f[f"{precon}__alphas"])
                                / np.linalg.norm(f[f"{precon}__alphas"]))}
    v = out["variants"].values()
    out["band_iters"] = int(max(abs(e["d_iters"]) for e in v))
    out["band_crossing"] = int(max(e["max_d_crossing"] for e in v))
    out["band_rel_dalpha"] = float(max(e["rel_dalpha"] for e in v))
    return out


def run_model_case(orders):
    """sgdml_model_ethanol_n621: the reference's GDMLTrain.train model (harmonic labels, so the
    coefficients have prediction-neutral freedom; tol 1e-4, cholesky at the rule-of-thumb
    rank).  The model keeps no residual curve: the band is on the iteration count and on
    alphas_F only."""
    f = np.load(GOLDEN / "sgdml_model_ethanol_n621.npz", allow_pickle=False)
    Rd, Rdd = descriptors(f["R"])
    perms = np.atleast_2d(f["perms"])
    y = f["F"].ravel().copy()
    y /= np.std(y)
    n, lam, sig = y.size, 1e-10, float(f["model__sig"])
    mv0 = kop_variant(Rd, Rdd, perms, sig, "mf")
    cols = {}

    def col(i):  # columns of -K_op (the reference's get_col, iterative_cholesky.py:152-156)
        if i not in cols:
            e = np.zeros(n)
            e[i] = 1.0
            cols[i] = -mv0(e) + lam * e
        return cols[i]

    diag = np.array([-mv0(np.eye(1, n, i)[0])[i] for i in range(n)])
    k = int(int(f["k_rot"]) / n * n)
    L, piv = pivoted_cholesky(col, diag, k)
    T, sp = woodbury_panel(L, lam)
    a_ref = f["model__alphas_F"]
    ref_it = int(f["model__solver_iters"])
    panel_order = {"mf": "blas", "mf_rev": "rev", "mf_split": "blk7", "mf_pair": "blk512"}
    out = {"n": n, "ref_iters": ref_it, "variants": {},
           "pivots_equal_reference": bool(np.array_equal(piv, f["model__index_columns"]))}
    for order in orders:
        mvK = kop_variant(Rd, Rdd, perms, sig, order)
        mvT = make_gemv(T, panel_order[order])
        mvTt = make_gemv(np.ascontiguousarray(T.T), panel_order[order])
        x, info, tr, it = cg_legacy(lambda v: -mvK(v) + lam * v, y, tol=1e-4, maxiter=5 * n,
                                    psolve=lambda r: sp * ((r - mvTt(mvT(r))) / lam))
        out["variants"][order] = {"iters": int(it), "info": int(info), "d_iters": int(it - ref_it),
                                  "rel_dalpha": float(np.linalg.norm(-x - a_ref) / np.linalg.norm(a_ref))}
    v = out["variants"].values()
    out["band_iters"] = int(max(abs(e["d_iters"]) for e in v))
    out["band_crossing"] = None
    out["band_rel_dalpha"] = float(max(e["rel_dalpha"] for e in v))
    return out


def run_rbf_small_cases():
    """The multi-rank tests' RBF system (tests/test_gpu_multirank.py: N = 1003, x ~ U[0,1)^3
    default_rng(3), l = 0.2, lam = 0.1, tol 1e-8, rank-150 pivoted Cholesky / Nystrom on
    default_rng(5) columns / none): the oracle in the dense mat-vec's summation orders,
    against its own BLAS-order solve (the multi-rank tests compare W ranks with one rank)."""
    sys.path.insert(0, str(REPO / "mlff-preconditioner_amd"))
    from oracle.rbf import rbf_kernel
    from sgdml_amd import synthetic

    n, lam, k = 1003, 1e-1, 150
    X, b = synthetic.rbf_points(n, 3, 3)
    K = rbf_kernel(X, 0.2)
    idx = np.sort(np.random.default_rng(5).choice(n, k, replace=False))
    res = {}
    for precon in ("none", "pivchol", "nystrom"):
        if precon == "pivchol":
            L, _ = pivoted_cholesky(lambda i: K[:, i], np.diag(K).copy(), k)
            T, sp = woodbury_panel(L, lam)
        elif precon == "nystrom":
            T, sp = nystrom_panel(K[:, idx], idx, lam, 0)
        else:
            T, sp = None, 1.0  # no preconditioner
        runs = {}
        for order in ("blas", "rev", "blk7", "blk512", "pair"):
            mvK = make_gemv(K, order)
            if precon == "none":
                ps = None
            else:
                mvT = make_gemv(T, order)
                mvTt = make_gemv(np.ascontiguousarray(T.T), order)
                ps = (lambda mvT, mvTt: (lambda r: sp * ((r - mvTt(mvT(r))) / lam)))(mvT, mvTt)
            runs[order] = cg_legacy(lambda v: mvK(v) + lam * v, b, tol=1e-8, maxiter=5 * n,
                                    psolve=ps)
        x0, _, tr0, it0 = runs["blas"]
        top = float(np.log10(np.minimum.accumulate(tr0[1:])[0]))
        cr0 = half_decade_crossings(tr0[1:], top)
        var = {}
        for order, (x, info, tr, it) in runs.items():
            cr = half_decade_crossings(tr[1:], top)
            dc = [abs(cr[q] - cr0[q]) for q in cr0 if q in cr]
            var[order] = {"iters": int(it), "info": int(info), "d_iters": int(it - it0),
                          "max_d_crossing": int(max(dc) if dc else 0),
                          "rel_dalpha": float(np.linalg.norm(x - x0) / np.linalg.norm(x0))}
        v = var.values()
        res[f"rbf_n1003/{precon}"] = {
            "n": n, "ref_iters": int(it0), "variants": var,
            "band_iters": int(max(abs(e["d_iters"]) for e in v)),
            "band_crossing": int(max(e["max_d_crossing"] for e in v)),
            "band_rel_dalpha": float(max(e["rel_dalpha"] for e in v))}
        print(f"rbf_n1003 {precon:8s} ref {it0}  band it {res[f'rbf_n1003/{precon}']['band_iters']}",
              flush=True)
    return res


def main():
    res = {}
    for name, precon in CASES:
        t0 = time.time()
        n = int(np.load(GOLDEN / f"{name}.npz", allow_pickle=False)["y"].size)
        orders = ["mf", "mf_rev", "mf_split", "mf_pair"] + (["ld"] if n <= 621 else [])
        r = run_case(name, precon, orders)
        res[f"{name}/{precon}"] = r
        print(f"{name:28s} {precon:26s} ref {r['ref_iters']:5d}  "
              + " ".join(f"{o}:{e['d_iters']:+d}" for o, e in r["variants"].items())
              + f"  band it {r['band_iters']} cross {r['band_crossing']}  ({time.time() - t0:.1f} s)",
              flush=True)
    t0 = time.time()
    r = run_model_case(["mf", "mf_rev", "mf_split", "mf_pair"])
    res["sgdml_model_ethanol_n621/cholesky"] = r
    print(f"{'sgdml_model_ethanol_n621':28s} {'cholesky':26s} ref {r['ref_iters']:5d}  "
          + " ".join(f"{o}:{e['d_iters']:+d}" for o, e in r["variants"].items())
          + f"  band it {r['band_iters']} dalpha {r['band_rel_dalpha']:.1e}  ({time.time() - t0:.1f} s)",
          flush=True)
    res.update(run_rbf_small_cases())
    (GOLDEN / "noise_band.json").write_text(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
