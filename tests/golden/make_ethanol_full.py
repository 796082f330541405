"""Ethanol at the reference's published size, on energy-consistent labels, pinned by the CPU
oracle (BASELINE.md:22 publishes ethanol N = 15741: k = 3935 / 1476 / 554 / 150 ->
112 / 245 / 570 / 2395 iterations to tol 1e-4, data/data/cg_performance_n=15750/
2022-03-17_2333_ethanol_points583_meas31; train.py:309 solver_tol 1e-4).

Geometry: sgdml_amd.synthetic.ethanol_harmonic(583, seed=0) -- the bench's ethanol geometries
with forces F = -grad E of a pair-harmonic potential (the reference's MD dataset is an HTTP
download absent here; random force labels put 1e-6 at the system's attainable-accuracy floor,
VERDICT r4).  Identity permutation, sig = 10, lam = 1e-10 (train.py:866), y = F.ravel() / std
(train.py:837-845), descriptors by oracle.sgdml.descriptors on the host (the GPU test passes the
same arrays, so both sides start from identical bits).

1. pivoted Cholesky (incomplete_cholesky.py:24-93) of -K_op to k = 1264 (the rule of thumb,
   plot_data.py:1254-1258; get_col = -K_op e_i + lam e_i, iterative_cholesky.py:152-156) on the
   oracle's matrix-free operator, with per-step pivot values and top-two gaps.  The first 554
   steps are the rank-554 factor (a published k): the greedy pivot sequence does not depend on
   max_rank.
2. for k = 1264 and 554: Woodbury panel (iterative_cholesky.py:141-148) and the scipy-1.7.3 CG
   (iterative_solver.py:995-1009) to tol 1e-4 (the reference's training tolerance) and 1e-6 in
   three operator summation orders (mf, mf_rev, mf_split: make_noise_band.kop_variant) and two
   Gram orders of the panel (rev, blk8; make_nanotube_full.woodbury_gram_order) -- the 'mf' solve
   is the reference trajectory, the others its noise band.
3. in the same pass, the same solves with the Woodbury
   panel evaluated ACCURATELY -- T = Q1^T from a Householder QR of [L; sqrt(lam) I] ('qr'; the
   formula's exact value is T = L2^-1 L^T = (L R^-1)^T with R^T R = lam I + L^T L) and the one-step
   panel re-orthogonalised by a second CholeskyQR step ('refined', the device's default,
   DESIGN.md 2) -- in the 'mf', 'mf_rev' and 'mf_split' operator orders: the band of the
   reference's formula without the rounding of its one-step fp64 evaluation (at cond([L; sqrt(lam)
   I]) ~ 6e3 the one-step LAPACK panel is far from the formula's value).  Stored as
   bands[key]["accurate"] (reference order: qr / mf) and the arrays <key>_accurate_*.
4. --rows (after 1-3): the accurate panels once more with the device's one-pass apply order
   (groups of ceil(k / 256) rows, group partials added in order: rows_apply) merged into the
   accurate bands -- at lam = 1e-10 the count of an accurately evaluated preconditioner is set by
   the apply's rounding (the refined panel: 773 iterations with BLAS's order, 839 with this one).

Writes tests/golden/ethanol_n15741.npz and ethanol_n15741_band.json.  CPU only (~35 min on 7
processes, one BLAS thread each, after the 5-min pivoted Cholesky; --cache keeps L).
"""
from __future__ import annotations

import json
import multiprocessing as mp
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "mlff-preconditioner_amd")]
GOLDEN = REPO / "tests" / "golden"
sys.path.insert(0, str(GOLDEN))

from make_nanotube_full import pivoted_cholesky_logged, woodbury_gram_order  # noqa: E402
from make_noise_band import half_decade_crossings, kop_variant, make_gemv  # noqa: E402
from oracle.pcg import cg_legacy  # noqa: E402
from oracle.precon import woodbury_panel  # noqa: E402
from oracle.sgdml import descriptors, kernel_diag  # noqa: E402
from sgdml_amd import synthetic  # noqa: E402  (input generation only)

M, N_ATOMS, SIG, LAM = 583, 9, 10.0, 1e-10
K_RANKS = (1264, 554)
TOLS = (1e-4, 1e-6)
ORDERS = ("mf", "mf_rev", "mf_split")
PANEL_ORDERS = ("rev", "blk8")
MAXITER = 12000

_G = {}  # problem data shared with the forked solve workers


def problem():
    ds = synthetic.ethanol_harmonic(M, seed=0)
    Rd, Rdd = descriptors(ds["R"])
    y, _ = synthetic.labels(ds["F"])
    return ds["R"], Rd, Rdd, np.arange(N_ATOMS)[None, :], y


def accurate_panel(L, lam, kind):
    """The Woodbury panel T = chol(lam I + L^T L)^-1 L^T (iterative_cholesky.py:141-143)
    evaluated accurately: 'qr' -- T = Q1^T, Q1 the top block of the Householder QR of
    [L; sqrt(lam) I] (its R satisfies R^T R = lam I + L^T L, so T = (L R^-1)^T up to row signs,
    which T^T T does not see); 'refined' -- the one-step panel T1 and a second CholeskyQR step
    (C C^T = T1 T1^T + lam L2^-1 L2^-T, T = C^-1 T1), as the device builds it by default."""
    import scipy.linalg

    k = L.shape[1]
    if kind == "qr":
        A = np.vstack([L, np.sqrt(lam) * np.eye(k)])
        Q, _ = np.linalg.qr(A, mode="reduced")
        return np.ascontiguousarray(Q[:L.shape[0]].T)
    L2 = scipy.linalg.cholesky(lam * np.eye(k) + L.T @ L, lower=True)
    T1 = scipy.linalg.solve_triangular(L2, L.T, lower=True)
    Li = scipy.linalg.solve_triangular(L2, np.eye(k), lower=True)
    C = scipy.linalg.cholesky(T1 @ T1.T + lam * (Li @ Li.T), lower=True)
    return scipy.linalg.solve_triangular(C, T1, lower=True)


# rows per workgroup of the device's one-pass apply at these ranks when the fixture was made
# (lr_rows_per_wg was ceil(k / 256); round 5 later raised it to at least 7 -- another order of the
# same sums, which the band already samples)
ROWS_PER_GROUP = {1264: 5, 554: 3}


def rows_apply(T, rpw):
    """z = (r - T^T T r) / lam summed as the device's one-pass rows apply orders it (k_lr_rows /
    k_lr_fin): t_i row by row, the partial T_g^T t_g of each group of rpw consecutive rows, the
    group partials added in group order, then lam_inv (r - u) -- another summation order of the
    same formula."""
    k = T.shape[0]
    groups = [np.ascontiguousarray(T[a:min(a + rpw, k)]) for a in range(0, k, rpw)]
    lam_inv = 1.0 / LAM

    def f(r):
        u = np.zeros_like(r)
        for g in groups:
            u = u + g.T @ (g @ r)
        return lam_inv * (r - u)
    return f


def _solve(job):
    """One CG solve: (k, operator order, panel order, tol) -> trace, x, info, iters."""
    import threadpoolctl

    k, order, po, tol = job
    Rd, Rdd, perms, y, L = _G["Rd"], _G["Rdd"], _G["perms"], _G["y"], _G["L"]
    t0 = time.time()
    with threadpoolctl.threadpool_limits(limits=1, user_api="blas"):
        Lk = np.ascontiguousarray(L[:, :k])
        if not po:
            T = woodbury_panel(Lk, LAM)[0]
        elif po in ("qr", "refined"):
            T = accurate_panel(Lk, LAM, po)
        elif po == "subst":
            T = subst_panel(Lk, LAM)
        else:
            T = woodbury_gram_order(Lk, LAM, po)
        if order in ("mf_rows", "mf_rows7"):  # the device's one-pass apply order (rows_apply)
            mvK = kop_variant(Rd, Rdd, perms, SIG, "mf")
            psolve = rows_apply(T, ROWS_PER_GROUP[k] if order == "mf_rows" else 7)
        else:
            mvK = kop_variant(Rd, Rdd, perms, SIG, order)
            panel_order = {"mf": "blas", "mf_rev": "rev", "mf_split": "blk7"}[order]
            mvT = make_gemv(T, panel_order)
            mvTt = make_gemv(np.ascontiguousarray(T.T), panel_order)
            psolve = lambda r: (r - mvTt(mvT(r))) / LAM  # noqa: E731
        x, info, tr, it = cg_legacy(lambda v: -mvK(v) + LAM * v, y, tol=tol, maxiter=MAXITER,
                                    psolve=psolve)
    name = order if not po else f"panel_{po}" if po not in ("qr", "refined") else f"{po}_{order}"
    if po and po not in ("qr", "refined") and order != "mf":
        name += "_" + order
    print(f"k={k} tol={tol:g} {name:10s} iters {it} info {info} ({time.time() - t0:.0f} s)",
          flush=True)
    return job, x, info, tr, it


def subst_panel(L, lam):
    """The one-step Woodbury panel T = chol(lam I + L^T L)^-1 L^T (iterative_cholesky.py:141-143)
    in another evaluation order: the Gram matrix in 64-row chunks added exactly, the Cholesky
    factor column by column (left-looking dot products), T row by row by forward substitution
    (each row one dot product over the rows before it) -- the same formula with the factorisation's
    and the triangular solve's sums ordered unlike LAPACK's blocked dpotrf / dtrsm."""
    from make_nanotube_full import gram_in_order

    k = L.shape[1]
    A = gram_in_order(L, "chunk64dd") + lam * np.eye(k)
    L2 = np.zeros((k, k))
    for j in range(k):
        v = A[j:, j] - L2[j:, :j] @ L2[j, :j]
        L2[j, j] = np.sqrt(v[0])
        L2[j + 1:, j] = v[1:] / L2[j, j]
    Lt = np.ascontiguousarray(L.T)
    T = np.empty_like(Lt)
    for j in range(k):
        T[j] = (Lt[j] - L2[j, :j] @ T[:j]) / L2[j, j]
    return T


def band_of(runs, ref_name, tol):
    x0, info0, tr0, it0 = runs[ref_name]
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
    return {"tol": tol, "ref_order": ref_name, "ref_iters": int(it0), "variants": variants,
            "band_iters": int(max(abs(e["d_iters"]) for e in v)),
            "band_crossing": int(max(e["max_d_crossing"] for e in v)),
            "band_rel_dalpha": float(max(e["rel_dalpha"] for e in v))}


def merge_rows(cache, procs):
    """--rows: the accurate panels with the device's apply order ('refined_mf_rows', 'qr_mf_rows'),
    merged into the committed fixture's accurate bands (the reference solve of each band, qr / mf,
    is stored, so d_iters, crossings and d_alpha are measured against it as for the others)."""
    R, Rd, Rdd, perms, y = problem()
    c = np.load(cache, allow_pickle=False)
    _G.update(Rd=Rd, Rdd=Rdd, perms=perms, y=y, L=c["L"])
    out = json.loads((GOLDEN / "ethanol_n15741_band.json").read_text())
    with np.load(GOLDEN / "ethanol_n15741.npz", allow_pickle=False) as f:
        arrays = {name: f[name] for name in f.files}
    jobs = [(k, "mf_rows", po, tol) for k in K_RANKS for tol in TOLS for po in ("refined", "qr")]
    jobs.sort(key=lambda j: (j[3] > 1e-5, -j[0]))
    with mp.get_context("fork").Pool(procs) as pool:
        results = pool.map(_solve, jobs, chunksize=1)
    for (k, order, po, tol), x, info, tr, it in results:
        key = f"k{k}_tol{tol:g}"
        b = out["bands"][key]["accurate"]
        x0 = -arrays[f"{key}_accurate_alphas"]
        tr0, it0 = arrays[f"{key}_accurate_trace"], int(arrays[f"{key}_accurate_iters"])
        top = float(np.log10(np.minimum.accumulate(tr0[1:])[0]))
        cr0, cr = half_decade_crossings(tr0[1:], top), half_decade_crossings(tr[1:], top)
        dc = [abs(cr[q] - cr0[q]) for q in cr0 if q in cr]
        b["variants"][f"{po}_{order}"] = {
            "iters": int(it), "info": int(info), "d_iters": int(it - it0),
            "max_d_crossing": int(max(dc) if dc else 0),
            "rel_dalpha": float(np.linalg.norm(x - x0) / np.linalg.norm(x0))}
        v = b["variants"].values()
        b["band_iters"] = int(max(abs(e["d_iters"]) for e in v))
        b["band_crossing"] = int(max(e["max_d_crossing"] for e in v))
        b["band_rel_dalpha"] = float(max(e["rel_dalpha"] for e in v))
        print(key, "accurate", json.dumps({q: b[q] for q in ("ref_iters", "band_iters",
                                                            "band_crossing", "band_rel_dalpha")}),
              flush=True)
    (GOLDEN / "ethanol_n15741_band.json").write_text(json.dumps(out, indent=1, sort_keys=True))


def _factor(cache):
    """L of the rank-1264 pivoted Cholesky (from --cache when present), pivots checked against
    the committed fixture's."""
    R, Rd, Rdd, perms, y = problem()
    if cache is not None and Path(cache).exists():
        L = np.load(cache, allow_pickle=False)["L"]
    else:
        mv0 = kop_variant(Rd, Rdd, perms, SIG, "mf")

        def get_col(i):  # (-K_op) e_i (iterative_cholesky.py:152-156)
            e = np.zeros(y.size)
            e[i] = 1.0
            return -mv0(e) + LAM * e

        L, piv, piv_val, gap = pivoted_cholesky_logged(get_col, -kernel_diag(Rd, Rdd, perms, SIG),
                                                       max(K_RANKS))
        with np.load(GOLDEN / "ethanol_n15741.npz", allow_pickle=False) as f:
            assert np.array_equal(piv[:max(K_RANKS)], f["index_columns"])
        if cache is not None:
            np.savez(cache, L=L, piv=piv, piv_val=piv_val, gap=gap)
    return Rd, Rdd, perms, y, L


GRAM_JOBS_1 = [("mf", "chunk64dd"), ("mf", "pair"), ("mf", "ld")]
# the round's second pass: the one-step panel with the device's apply order (7 rows per group,
# lr_rows_per_wg) for three Gram orders, and the substitution-ordered factorisation / solve
GRAM_JOBS_2 = [("mf_rows7", "blas"), ("mf_rows7", "chunk64dd"), ("mf_rows7", "ld"),
               ("mf", "subst")]


def merge_gram(cache, procs, gram_jobs=GRAM_JOBS_1):
    """--gram (round 6): the reference's one-step panel (iterative_cholesky.py:141-143) with its
    Gram matrix L^T L in three more summation orders (make_nanotube_full.GRAM_ORDERS: 64-row
    chunks added exactly, pairwise, extended precision) merged into the one-step LAPACK bands at
    both ranks and both tolerances.  DESIGN.md 2 showed that this rounding, not the operator's,
    sets the one-step count at cond([L; sqrt(lam) I]) ~ 6e3; the band of rounds 5 sampled only
    BLAS / reversed / 8 slabs."""
    Rd, Rdd, perms, y, L = _factor(cache)
    _G.update(Rd=Rd, Rdd=Rdd, perms=perms, y=y, L=L)
    out = json.loads((GOLDEN / "ethanol_n15741_band.json").read_text())
    with np.load(GOLDEN / "ethanol_n15741.npz", allow_pickle=False) as f:
        arrays = {name: f[name] for name in f.files}
    jobs = [(k, order, po, tol) for k in K_RANKS for tol in TOLS for order, po in gram_jobs]
    jobs.sort(key=lambda j: (j[3] > 1e-5, -j[0]))
    with mp.get_context("fork").Pool(procs) as pool:
        results = pool.map(_solve, jobs, chunksize=1)
    for (k, order, po, tol), x, info, tr, it in results:
        key = f"k{k}_tol{tol:g}"
        b = out["bands"][key]
        x0 = -arrays[f"{key}_alphas"]
        tr0, it0 = arrays[f"{key}_trace"], int(arrays[f"{key}_iters"])
        top = float(np.log10(np.minimum.accumulate(tr0[1:])[0]))
        cr0, cr = half_decade_crossings(tr0[1:], top), half_decade_crossings(tr[1:], top)
        dc = [abs(cr[q] - cr0[q]) for q in cr0 if q in cr]
        vname = f"panel_{po}" if order == "mf" else f"panel_{po}_rows7"
        b["variants"][vname] = {
            "iters": int(it), "info": int(info), "d_iters": int(it - it0),
            "max_d_crossing": int(max(dc) if dc else 0),
            "rel_dalpha": float(np.linalg.norm(x - x0) / np.linalg.norm(x0))}
        v = [e for name, e in b["variants"].items()]
        b["band_iters"] = int(max(abs(e["d_iters"]) for e in v))
        b["band_crossing"] = int(max(e["max_d_crossing"] for e in v))
        b["band_rel_dalpha"] = float(max(e["rel_dalpha"] for e in v))
        xa = -arrays[f"{key}_accurate_alphas"]
        b["variants"][vname]["accurate_rel_dalpha"] = float(
            np.linalg.norm(x - xa) / np.linalg.norm(xa))
        print(key, "one-step", vname, it, json.dumps({q: b[q] for q in (
            "ref_iters", "band_iters", "band_crossing", "band_rel_dalpha")}), flush=True)
    (GOLDEN / "ethanol_n15741_band.json").write_text(json.dumps(out, indent=1, sort_keys=True))


def main(cache=None, procs=8):
    t_all = time.time()
    R, Rd, Rdd, perms, y = problem()
    n = y.size
    assert n == 15741
    mv0 = kop_variant(Rd, Rdd, perms, SIG, "mf")

    def get_col(i):  # (-K_op) e_i (iterative_cholesky.py:152-156)
        e = np.zeros(n)
        e[i] = 1.0
        return -mv0(e) + LAM * e

    kmax = max(K_RANKS)
    if cache is not None and Path(cache).exists():
        c = np.load(cache, allow_pickle=False)
        L, piv, piv_val, gap = c["L"], c["piv"], c["piv_val"], c["gap"]
    else:
        diag = -kernel_diag(Rd, Rdd, perms, SIG)
        L, piv, piv_val, gap = pivoted_cholesky_logged(get_col, diag, kmax)
        if cache is not None:
            np.savez(cache, L=L, piv=piv, piv_val=piv_val, gap=gap)
    print(f"pivoted Cholesky k={kmax}: {time.time() - t_all:.0f} s", flush=True)
    _G.update(Rd=Rd, Rdd=Rdd, perms=perms, y=y, L=L)
    jobs = []
    for k in K_RANKS:
        for tol in TOLS:
            jobs += [(k, o, "", tol) for o in ORDERS] + [(k, "mf", po, tol) for po in PANEL_ORDERS]
            jobs += [(k, o, "qr", tol) for o in ORDERS] + [(k, "mf", "refined", tol)]
    # the long solves first
    jobs.sort(key=lambda j: (j[3] > 1e-5, -j[0]))
    with mp.get_context("fork").Pool(procs) as pool:
        results = pool.map(_solve, jobs, chunksize=1)
    out = {"n": n, "M": M, "n_atoms": N_ATOMS, "sig": SIG, "lam": LAM, "k_max": kmax,
           "first_gap_below_1e-12": int(np.argmax(gap < 1e-12)) if np.any(gap < 1e-12) else None,
           "min_gap": float(gap.min()), "bands": {}}
    arrays = {"R": R, "y": y, "index_columns": piv[:kmax], "pivot_values": piv_val,
              "pivot_gap": gap}
    for k in K_RANKS:
        for tol in TOLS:
            runs, acc = {}, {}
            for (jk, order, po, jt), x, info, tr, it in results:
                if jk == k and jt == tol:
                    if po in ("qr", "refined"):
                        acc[f"{po}_{order}"] = (x, info, tr, it)
                    else:
                        runs[order if not po else f"panel_{po}"] = (x, info, tr, it)
            if not runs:
                continue
            key = f"k{k}_tol{tol:g}"
            out["bands"][key] = band_of(runs, "mf", tol)
            b = band_of(acc, "qr_mf", tol)
            x0 = acc["qr_mf"][0]
            b["lapack_onestep_rel_dalpha"] = float(np.linalg.norm(runs["mf"][0] - x0) / np.linalg.norm(x0))
            out["bands"][key]["accurate"] = b
            xa, infoa, tra, ita = acc["qr_mf"]
            arrays[f"{key}_accurate_trace"] = tra
            arrays[f"{key}_accurate_alphas"] = -xa
            arrays[f"{key}_accurate_iters"] = np.int64(ita)
            arrays[f"{key}_accurate_info"] = np.int64(infoa)
            print(key, "accurate", json.dumps({q: b[q] for q in ("ref_iters", "band_iters",
                                                                "band_crossing", "band_rel_dalpha")}),
                  flush=True)
            x0, info0, tr0, it0 = runs["mf"]
            arrays[f"{key}_trace"] = tr0
            arrays[f"{key}_alphas"] = -x0
            arrays[f"{key}_iters"] = np.int64(it0)
            arrays[f"{key}_info"] = np.int64(info0)
            print(key, json.dumps({q: out["bands"][key][q] for q in
                                   ("ref_iters", "band_iters", "band_crossing", "band_rel_dalpha")}),
                  flush=True)
    np.savez_compressed(GOLDEN / "ethanol_n15741.npz", **arrays)
    (GOLDEN / "ethanol_n15741_band.json").write_text(json.dumps(out, indent=1, sort_keys=True))
    print(f"total {time.time() - t_all:.0f} s", flush=True)


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--cache", default=None, help=".npz outside the repository for L (160 MB)")
    ap.add_argument("--procs", type=int, default=int(os.environ.get("PROCS", "8")))
    ap.add_argument("--rows", action="store_true",
                    help="merge the device-apply-order accurate solves into the committed fixture")
    ap.add_argument("--gram2", action="store_true",
                    help="merge the one-step apply-order / substitution variants into the fixture")
    ap.add_argument("--gram", action="store_true",
                    help="merge one-step solves with more Gram summation orders into the fixture")
    a = ap.parse_args()
    if a.gram2:
        merge_gram(a.cache, a.procs, GRAM_JOBS_2)
    elif a.gram:
        merge_gram(a.cache, a.procs)
    elif a.rows:
        merge_rows(a.cache, a.procs)
    else:
        main(a.cache, a.procs)
