"""configs[1] at its full size, pinned by the CPU oracle (BASELINE.json configs[1]: nanotube
N = 15540, rank-2701 pivoted-Cholesky PCG to relres 1e-6).

Geometry: sgdml_amd.synthetic.nanotube_like(14, seed=0) (the bench's --workload nanotube; the
reference's larger_aims_nanotube.npz is an HTTP download absent here), identity permutation,
sig = 10, lam = 1e-10 (train.py:866), y = F.ravel() / std (train.py:837-845).  Descriptors by
oracle.sgdml.descriptors on the host (the GPU test passes these same arrays to the device, so
both sides start from identical bits).

1. pivoted Cholesky (incomplete_cholesky.py:24-93) of the PSD operator -K_op to the rule-of-
   thumb rank k = 2701 (plot_data.py:1254-1258), get_col = -K_op e_i + lam e_i
   (iterative_cholesky.py:152-156) on the oracle's matrix-free operator, diagonal = -diag(K)
   without lam (iterative_cholesky.py:373).  Recorded per step: the pivot, its residual diagonal
   and the relative gap to the runner-up candidate (pivot sequences are compared up
   to the first near-tie).
2. Woodbury panel (iterative_cholesky.py:141-148) and the scipy-1.7.3 CG solve
   (iterative_solver.py:995-1009) to 1e-6 in three summation orders of the matrix-free operator
   and the panel apply (make_noise_band.kop_variant: mf, mf_rev, mf_split): the 'mf' solve is the
   reference trajectory (trace, alpha = -x), the spread of the others its noise band.

4. --compute-cache then --accurate (round 5): the accurate-panel band (QR / two-step panels in
   several summation orders) merged into the committed fixture as band["accurate"].

3. --panel-orders: more solves of the 'mf' operator with the Woodbury panel rounded another way
   (woodbury_gram_order): 'rev' / 'blk8' (Gram matrix in other orders) join the band; 'inverse',
   'noise', 'rownoise' (explicit triangular inverse; 2e-15 perturbations) are recorded beside it
   as "panel_perturbations": at lam = 1e-10 they take ~550-580 iterations against the LAPACK
   panels' ~365 (DESIGN.md 2, configs[1] at full size).  --cache keeps L (336 MB) outside the
   repository for such reruns.

Writes tests/golden/nanotube_n15540.npz and nanotube_n15540_band.json.  CPU only: 40 min on 4
cores (2701 operator applications for the columns, 30 min; three solves of 367 iterations); the
reference is not imported (its algorithm is the oracle's restatement).  First recorded run: 367 /
367 / 368 iterations, band b_it 1, b_cr 3, ||d alpha|| / ||alpha|| 2.0e-11, no near-tie among the
2701 pivots (smallest relative gap of the best two candidates 3.1e-7).  The committed fixture is
the round-4 rerun (2 BLAS threads: L differs in its last bits, 'mf' 369 iterations) with the
panel orders (profiles/r04/make_nanotube_full_r4.log).
"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "mlff-preconditioner_amd")]
GOLDEN = REPO / "tests" / "golden"
sys.path.insert(0, str(GOLDEN))

from make_noise_band import half_decade_crossings, kop_variant, make_gemv  # noqa: E402
from oracle.pcg import cg_legacy  # noqa: E402
from oracle.precon import woodbury_panel  # noqa: E402
from oracle.sgdml import descriptors, kernel_diag  # noqa: E402
from sgdml_amd import synthetic  # noqa: E402  (input generation only)

M, N_ATOMS, SIG, LAM, TOL, K_RANK = 14, 370, 10.0, 1e-10, 1e-6, 2701


def problem():
    ds = synthetic.nanotube_like(M, seed=0)
    Rd, Rdd = descriptors(ds["R"])
    y, _ = synthetic.labels(ds["F"])
    return ds["R"], Rd, Rdd, np.arange(N_ATOMS)[None, :], y


def pivoted_cholesky_logged(get_col, diagonal, max_rank):
    """oracle.precon.pivoted_cholesky (incomplete_cholesky.py:24-93) with the per-step pivot
    value and the relative gap between the largest and the second-largest candidate."""
    diag = np.array(diagonal, dtype=np.float64, copy=True)
    n = diag.size
    index_columns = np.arange(n)
    L = np.zeros((n, max_rank))
    piv_val = np.empty(max_rank)
    gap = np.empty(max_rank)
    t0 = time.time()
    for m in range(max_rank):
        cand = diag[index_columns][m:]
        i_argmax = int(np.argmax(cand) + m)                                  # :53
        top2 = np.partition(cand, -2)[-2:] if cand.size > 1 else np.array([0.0, cand[0]])
        gap[m] = (top2[1] - top2[0]) / top2[1]
        index_columns[m], index_columns[i_argmax] = index_columns[i_argmax], index_columns[m]
        m_pi = index_columns[m]
        i_pi = index_columns[m + 1:]
        pivot_element = diag[m_pi]
        piv_val[m] = pivot_element
        assert pivot_element > 0, "given matrix is not PSD"                  # :62
        L[m_pi, m] = np.sqrt(pivot_element)
        k = get_col(m_pi)
        schur = 0
        if m > 0:
            schur = L[i_pi, :m] @ L[m_pi, :m]                                # :72
        L[i_pi, m] = (k[i_pi] - schur) / L[m_pi, m]                           # :75
        diag[i_pi] -= L[i_pi, m] ** 2                                         # :78
        if (m + 1) % 250 == 0:
            print(f"  pivot {m + 1}/{max_rank}  {time.time() - t0:.0f} s", flush=True)
    return L, index_columns, piv_val, gap


PANEL_ORDERS = ["rev", "blk8", "chunk64dd", "pair", "ld", "inverse", "noise", "rownoise"]
# the Gram-matrix summation orders of the reference's one-step formula (round 6): the count of
# the one-step panel at an ill-conditioned [L; sqrt(lam) I] is set by how L^T L is rounded
# (DESIGN.md 2), so its band samples that rounding -- BLAS, reversed, 8 row slabs, 64-row
# chunks added exactly, pairwise, extended-precision products and sums
GRAM_ORDERS = ("rev", "blk8", "chunk64dd", "pair", "ld")


def _dd_accumulate(parts):
    """fl(sum of fp64 matrices) with every addition exact (TwoSum into a double-double
    accumulator, rounded once): the outer sum of a blocked Gram as k_gram_mfma_dd forms it.
    parts may be a generator (one k x k partial in memory at a time: 1172 of them at N = 74979)."""
    hi = lo = None
    for p in parts:
        if hi is None:
            hi = np.zeros_like(p)
            lo = np.zeros_like(p)
        s = hi + p
        bp = s - hi
        lo += (hi - (s - bp)) + (p - bp)
        hi = s
    return hi + lo


def gram_in_order(L, order):
    """L^T L (the Woodbury Gram matrix, iterative_cholesky.py:141) in a given summation order
    over the rows of L."""
    if order == "rev":
        Lr = np.ascontiguousarray(L[::-1])
        return Lr.T @ Lr
    if order == "blk8":
        return sum(L[b].T @ L[b] for b in np.array_split(np.arange(L.shape[0]), 8))
    if order == "chunk64dd":  # 64-row chunks in fp64, the chunk partials added exactly
        return _dd_accumulate(L[a:a + 64].T @ L[a:a + 64] for a in range(0, L.shape[0], 64))
    if order == "pair":  # pairwise over row halves down to 128-row leaves
        def pw(A):
            if A.shape[0] <= 128:
                return A.T @ A
            h = A.shape[0] // 2
            return pw(A[:h]) + pw(A[h:])
        return pw(L)
    if order == "ld":  # products and sums with a 64-bit significand, rounded once
        Ll = L.astype(np.longdouble)
        return (Ll.T @ Ll).astype(np.float64)
    return L.T @ L


def woodbury_gram_order(L, lam, order):
    """oracle.precon.woodbury_panel (iterative_cholesky.py:141-143) rounded another way:
    'rev' / 'blk8' / 'chunk64dd' / 'pair' / 'ld': the Gram matrix L^T L in another summation
    order (gram_in_order); 'inverse': T = inv(L2) L^T (the triangular inverse, then one GEMM)
    instead of the triangular solve; 'noise' / 'rownoise': the LAPACK panel with independent
    relative perturbations of 2e-15 per entry / with 2e-15 (E T), E a k x k Gaussian (a perturbed
    L2).  The PCG at lam = 1e-10 is sensitive to how the panel is rounded (scripts/dev/
    diag_config1[b,c].py): LAPACK-built panels take 364-366 iterations, the others 552-577."""
    import scipy.linalg

    k = L.shape[1]
    G = gram_in_order(L, order if order in GRAM_ORDERS else "blas")
    L2 = scipy.linalg.cholesky(lam * np.eye(k) + G, lower=True)
    if order == "inverse":
        return np.tril(scipy.linalg.solve_triangular(L2, np.eye(k), lower=True)) @ L.T
    T = scipy.linalg.solve_triangular(L2, L.T, lower=True)
    rng = np.random.default_rng(11)
    if order == "noise":
        return T * (1.0 + 2e-15 * rng.standard_normal(T.shape))
    if order == "rownoise":
        return T + 2e-15 * ((rng.standard_normal((k, k)) / np.sqrt(k)) @ T)
    return T


# the panels the reference's own formula gives under a change of summation order (LAPACK
# Cholesky + triangular solve): the band; the perturbed constructions are recorded beside it
PERTURBED = ("panel_inverse", "panel_noise", "panel_rownoise")


def band_json(n, it0, variants, gap):
    fam = [e for o, e in variants.items() if o not in PERTURBED]
    band = {"n": n, "k": K_RANK, "ref_order": "mf", "ref_iters": int(it0),
            "variants": {o: e for o, e in variants.items() if o not in PERTURBED},
            "panel_perturbations": {o: e for o, e in variants.items() if o in PERTURBED},
            "band_iters": int(max(abs(e["d_iters"]) for e in fam)),
            "band_crossing": int(max(e["max_d_crossing"] for e in fam)),
            "band_rel_dalpha": float(max(e["rel_dalpha"] for e in fam)),
            "first_gap_below_1e-12": int(np.argmax(gap < 1e-12)) if np.any(gap < 1e-12) else None,
            "min_gap": float(gap.min())}
    return band


_A = {}  # shared with the forked accurate-panel workers


def _accurate_solve(job):
    """(panel kind, operator order) -> the solve of an accurately evaluated Woodbury panel
    (make_ethanol_full.accurate_panel: Householder QR or two CholeskyQR steps), with the
    operator order's apply order or the device's rows apply order ('mf_rows')."""
    import threadpoolctl

    from make_ethanol_full import accurate_panel, rows_apply

    kind, order = job
    Rd, Rdd, perms, y, L = _A["Rd"], _A["Rdd"], _A["perms"], _A["y"], _A["L"]
    t0 = time.time()
    with threadpoolctl.threadpool_limits(limits=1, user_api="blas"):
        T = accurate_panel(L, LAM, kind)
        if order == "mf_rows":
            mvK = kop_variant(Rd, Rdd, perms, SIG, "mf")
            psolve = rows_apply(T, (K_RANK + 255) // 256)
        else:
            mvK = kop_variant(Rd, Rdd, perms, SIG, order)
            po = {"mf": "blas", "mf_rev": "rev", "mf_split": "blk7"}[order]
            mvT, mvTt = make_gemv(T, po), make_gemv(np.ascontiguousarray(T.T), po)
            psolve = lambda r: (r - mvTt(mvT(r))) / LAM  # noqa: E731
        x, info, tr, it = cg_legacy(lambda v: -mvK(v) + LAM * v, _A["y"], tol=TOL,
                                    maxiter=5 * y.size, psolve=psolve)
    print(f"accurate {kind}_{order}: iters {it} info {info} ({time.time() - t0:.0f} s)", flush=True)
    return job, x, info, tr, it


def accurate(cache, procs=5):
    """--accurate (needs --cache of a full run): the configs[1] solve with the Woodbury panel
    evaluated accurately (QR in three orders, the two-step panel with BLAS's and the device's
    apply order), recorded as band["accurate"] and the arrays accurate_* -- the band the device's
    default panel (two CholeskyQR steps on a double-double Gram) is held to beside
    the one-step LAPACK band."""
    import multiprocessing as mp

    _, Rd, Rdd, perms, y = problem()
    c = np.load(cache, allow_pickle=False)
    _A.update(Rd=Rd, Rdd=Rdd, perms=perms, y=y, L=np.ascontiguousarray(c["L"][:, :K_RANK]))
    jobs = [("qr", "mf"), ("qr", "mf_rev"), ("qr", "mf_split"), ("qr", "mf_rows"),
            ("refined", "mf"), ("refined", "mf_rows")]
    with mp.get_context("fork").Pool(procs) as pool:
        results = pool.map(_accurate_solve, jobs, chunksize=1)
    runs = {f"{kind}_{order}": (x, info, tr, it) for (kind, order), x, info, tr, it in results}
    x0, info0, tr0, it0 = runs["qr_mf"]
    top = float(np.log10(np.minimum.accumulate(tr0[1:])[0]))
    cr0 = half_decade_crossings(tr0[1:], top)
    variants = {}
    for name, (x, info, tr, it) in runs.items():
        cr = half_decade_crossings(tr[1:], top)
        dc = [abs(cr[q] - cr0[q]) for q in cr0 if q in cr]
        variants[name] = {"iters": int(it), "info": int(info), "d_iters": int(it - it0),
                          "max_d_crossing": int(max(dc) if dc else 0),
                          "rel_dalpha": float(np.linalg.norm(x - x0) / np.linalg.norm(x0))}
    v = variants.values()
    band = json.loads((GOLDEN / "nanotube_n15540_band.json").read_text())
    band["accurate"] = {"ref_order": "qr_mf", "ref_iters": int(it0), "variants": variants,
                        "band_iters": int(max(abs(e["d_iters"]) for e in v)),
                        "band_crossing": int(max(e["max_d_crossing"] for e in v)),
                        "band_rel_dalpha": float(max(e["rel_dalpha"] for e in v))}
    with np.load(GOLDEN / "nanotube_n15540.npz", allow_pickle=False) as f:
        arrays = {name: f[name] for name in f.files}
    arrays.update(accurate_trace=tr0, accurate_alphas=-x0, accurate_iters=np.int64(it0),
                  accurate_info=np.int64(info0))
    np.savez_compressed(GOLDEN / "nanotube_n15540.npz", **arrays)
    (GOLDEN / "nanotube_n15540_band.json").write_text(json.dumps(band, indent=1, sort_keys=True))
    print(json.dumps({q: band["accurate"][q] for q in ("ref_iters", "band_iters", "band_crossing",
                                                      "band_rel_dalpha")}), flush=True)


K4_RANK = 1024   # BASELINE configs[4]: the same nanotube, rank-1024 pivoted Cholesky
K4_TOLS = (1e-4, 1e-6)


def _k4_solve(job):
    """(operator order, Gram order, tol) -> the rank-1024 Woodbury PCG solve (iterative_cholesky.py:
    135-150, iterative_solver.py:995-1009) on the oracle's matrix-free operator."""
    import threadpoolctl

    order, po, tol = job
    Rd, Rdd, perms, y, L = _A["Rd"], _A["Rdd"], _A["perms"], _A["y"], _A["L"]
    t0 = time.time()
    with threadpoolctl.threadpool_limits(limits=1, user_api="blas"):
        T = woodbury_gram_order(L, LAM, po) if po else woodbury_panel(L, LAM)[0]
        mvK = kop_variant(Rd, Rdd, perms, SIG, order)
        pord = {"mf": "blas", "mf_rev": "rev", "mf_split": "blk7"}[order]
        mvT, mvTt = make_gemv(T, pord), make_gemv(np.ascontiguousarray(T.T), pord)
        x, info, tr, it = cg_legacy(lambda v: -mvK(v) + LAM * v, y, tol=tol, maxiter=5 * y.size,
                                    psolve=lambda r: (r - mvTt(mvT(r))) / LAM)
    name = order if not po else f"panel_{po}"
    print(f"k={K4_RANK} tol={tol:g} {name:16s} iters {it} info {info} ({time.time() - t0:.0f} s)",
          flush=True)
    return job, x, info, tr, it


def configs4(cache, procs=8):
    """--configs4 (needs --cache of a full run; round 6): BASELINE configs[4]'s solve pinned.  The
    rank-1024 factor is the first 1024 columns of the rank-2701 one (the greedy pivot sequence
    does not depend on max_rank; its pivots are the committed index_columns[:1024]).  Woodbury
    panel and PCG to 1e-4 and 1e-6 in three operator / apply orders and five Gram orders
    (GRAM_ORDERS): nanotube_n15540_k1024.npz (reference 'mf' trace, alpha, iters per tol) and
    nanotube_n15540_k1024_band.json (the band per tol)."""
    import multiprocessing as mp

    R, Rd, Rdd, perms, y = problem()
    c = np.load(cache, allow_pickle=False)
    with np.load(GOLDEN / "nanotube_n15540.npz", allow_pickle=False) as f:
        assert np.array_equal(c["piv"][:K4_RANK], f["index_columns"][:K4_RANK])
    _A.update(Rd=Rd, Rdd=Rdd, perms=perms, y=y, L=np.ascontiguousarray(c["L"][:, :K4_RANK]))
    del c
    jobs = [(o, "", tol) for tol in K4_TOLS for o in ("mf", "mf_rev", "mf_split")]
    jobs += [("mf", po, tol) for tol in K4_TOLS for po in GRAM_ORDERS]
    jobs.sort(key=lambda j: j[2] > 1e-5)  # the long solves first
    with mp.get_context("fork").Pool(procs) as pool:
        results = pool.map(_k4_solve, jobs, chunksize=1)
    arrays = {"R": R, "y": y, "index_columns": _A_piv(cache)}
    bands = {"n": int(y.size), "k": K4_RANK, "ref_order": "mf", "bands": {}}
    for tol in K4_TOLS:
        runs = {(o if not po else f"panel_{po}"): (x, info, tr, it)
                for (o, po, t), x, info, tr, it in results if t == tol}
        x0, info0, tr0, it0 = runs["mf"]
        top = float(np.log10(np.minimum.accumulate(tr0[1:])[0]))
        cr0 = half_decade_crossings(tr0[1:], top)
        variants = {}
        for name, (x, info, tr, it) in runs.items():
            cr = half_decade_crossings(tr[1:], top)
            dc = [abs(cr[q] - cr0[q]) for q in cr0 if q in cr]
            variants[name] = {"iters": int(it), "info": int(info), "d_iters": int(it - it0),
                              "max_d_crossing": int(max(dc) if dc else 0),
                              "rel_dalpha": float(np.linalg.norm(x - x0) / np.linalg.norm(x0))}
        v = variants.values()
        key = f"tol{tol:g}"
        bands["bands"][key] = {"tol": tol, "ref_order": "mf", "ref_iters": int(it0),
                               "variants": variants,
                               "band_iters": int(max(abs(e["d_iters"]) for e in v)),
                               "band_crossing": int(max(e["max_d_crossing"] for e in v)),
                               "band_rel_dalpha": float(max(e["rel_dalpha"] for e in v))}
        arrays.update({f"{key}_trace": tr0, f"{key}_alphas": -x0, f"{key}_iters": np.int64(it0),
                       f"{key}_info": np.int64(info0)})
        print(key, json.dumps({q: bands["bands"][key][q] for q in (
            "ref_iters", "band_iters", "band_crossing", "band_rel_dalpha")}),
              json.dumps({o: e["iters"] for o, e in variants.items()}), flush=True)
    np.savez_compressed(GOLDEN / "nanotube_n15540_k1024.npz", **arrays)
    (GOLDEN / "nanotube_n15540_k1024_band.json").write_text(json.dumps(bands, indent=1,
                                                                       sort_keys=True))


def _A_piv(cache):
    return np.load(cache, allow_pickle=False)["piv"][:K4_RANK]


def main(cache=None, panel_orders=()):
    """cache: .npz path (outside the repository: 336 MB) holding L and the pivot log, written
    on the first run and read by later ones; panel_orders: Gram-matrix orders of the Woodbury
    panel whose solves join the band (variants 'panel_<order>')."""
    t_all = time.time()
    R, Rd, Rdd, perms, y = problem()
    n = y.size
    assert n == 15540
    mv0 = kop_variant(Rd, Rdd, perms, SIG, "mf")

    def get_col(i):  # (-K_op) e_i (iterative_cholesky.py:152-156)
        e = np.zeros(n)
        e[i] = 1.0
        return -mv0(e) + LAM * e

    if cache is not None and Path(cache).exists():
        c = np.load(cache, allow_pickle=False)
        L, piv, piv_val, gap = c["L"], c["piv"], c["piv_val"], c["gap"]
    else:
        diag = -kernel_diag(Rd, Rdd, perms, SIG)
        L, piv, piv_val, gap = pivoted_cholesky_logged(get_col, diag, K_RANK)
        if cache is not None:
            np.savez(cache, L=L, piv=piv, piv_val=piv_val, gap=gap)
    print(f"pivoted Cholesky k={K_RANK}: {time.time() - t_all:.0f} s", flush=True)
    T, sp = woodbury_panel(L, LAM)
    panels = {"": T}
    for po in panel_orders:
        panels[po] = woodbury_gram_order(L, LAM, po)
    del L
    panel_order = {"mf": "blas", "mf_rev": "rev", "mf_split": "blk7"}
    runs = {}
    plan = [(o, "") for o in ("mf", "mf_rev", "mf_split")] + [("mf", po) for po in panel_orders]
    for order, po in plan:
        t0 = time.time()
        T = panels[po]
        mvK = kop_variant(Rd, Rdd, perms, SIG, order)
        mvT = make_gemv(T, panel_order[order])
        mvTt = make_gemv(np.ascontiguousarray(T.T), panel_order[order])
        x, info, tr, it = cg_legacy(lambda v: -mvK(v) + LAM * v, y, tol=TOL, maxiter=5 * n,
                                    psolve=lambda r: sp * ((r - mvTt(mvT(r))) / LAM))
        name = order if not po else f"panel_{po}"
        runs[name] = (x, info, tr, it)
        print(f"solve {name:8s} iters {it} info {info} ({time.time() - t0:.0f} s)", flush=True)
    x0, info0, tr0, it0 = runs["mf"]
    top = float(np.log10(np.minimum.accumulate(tr0[1:])[0]))
    cr0 = half_decade_crossings(tr0[1:], top)
    variants = {}
    for order, (x, info, tr, it) in runs.items():
        cr = half_decade_crossings(tr[1:], top)
        dc = [abs(cr[q] - cr0[q]) for q in cr0 if q in cr]
        variants[order] = {"iters": int(it), "info": int(info), "d_iters": int(it - it0),
                           "max_d_crossing": int(max(dc) if dc else 0),
                           "rel_dalpha": float(np.linalg.norm(x - x0) / np.linalg.norm(x0))}
    band = band_json(n, it0, variants, gap)
    np.savez_compressed(GOLDEN / "nanotube_n15540.npz", R=R, y=y, index_columns=piv[:K_RANK],
                        pivot_values=piv_val, pivot_gap=gap, trace=tr0, iters=np.int64(it0),
                        info=np.int64(info0), alphas=-x0)
    (GOLDEN / "nanotube_n15540_band.json").write_text(json.dumps(band, indent=1, sort_keys=True))
    print(json.dumps({q: band[q] for q in ("ref_iters", "band_iters", "band_crossing",
                                           "band_rel_dalpha", "first_gap_below_1e-12", "min_gap")}),
          flush=True)
    print(json.dumps({o: e["iters"] for o, e in band["panel_perturbations"].items()}), flush=True)
    print(f"total {time.time() - t_all:.0f} s", flush=True)


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--cache", default=None)
    ap.add_argument("--panel-orders", nargs="*", default=[], choices=PANEL_ORDERS)
    ap.add_argument("--accurate", action="store_true",
                    help="the accurate-panel band only (needs --cache from a full run)")
    ap.add_argument("--compute-cache", action="store_true",
                    help="compute the factor into --cache (no solves)")
    ap.add_argument("--configs4", action="store_true",
                    help="the rank-1024 (configs[4]) solve band (needs --cache from a full run)")
    ap.add_argument("--procs", type=int, default=8)
    a = ap.parse_args()
    if a.configs4:
        configs4(a.cache, a.procs)
    elif a.compute_cache:
        _, Rd, Rdd, perms, y = problem()
        mv0 = kop_variant(Rd, Rdd, perms, SIG, "mf")

        def get_col(i):
            e = np.zeros(y.size)
            e[i] = 1.0
            return -mv0(e) + LAM * e

        L, piv, piv_val, gap = pivoted_cholesky_logged(get_col, -kernel_diag(Rd, Rdd, perms, SIG),
                                                       K_RANK)
        np.savez(a.cache, L=L, piv=piv, piv_val=piv_val, gap=gap)
    elif a.accurate:
        accurate(a.cache)
    else:
        main(a.cache, a.panel_orders)
