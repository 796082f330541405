"""Ethanol at the reference's N = 75k point (BASELINE.md:24, data/rule_of_thumb.csv:9: M = 2777,
N = 74979, the rule-of-thumb k = 3752), pinned by the CPU oracle (round 6).

Geometry: sgdml_amd.synthetic.ethanol_harmonic(2777, seed=0) -- the bench's ethanol geometry at
this size, energy-consistent labels -- identity permutation, sig = 10, lam = 1e-10
(train.py:866), y = F.ravel() / std (train.py:837-845), descriptors by oracle.sgdml.descriptors.

1. pivoted Cholesky (incomplete_cholesky.py:24-93) of -K_op to k = 3752 with get_col = -K_op e_i
   + lam e_i (iterative_cholesky.py:152-156).  Each column comes from the one training point it
   touches (oracle.sgdml.kernel_column_matrix_free: the operator's own products without the zero
   terms, equal to K_op e_i to rounding -- test_column_restatement_matches_operator), so the
   3752 columns cost seconds instead of 3752 operator applications; L is kept column-major so the
   Schur GEMV L[:, :m] L[m_pi, :m] streams contiguous columns (another BLAS order of the same
   sums).  Per step: the pivot value and the relative gap of the best two candidates.
2. the reference's Woodbury panel (iterative_cholesky.py:141-148, one CholeskyQR step) and the
   scipy-1.7.3 CG (iterative_solver.py:995-1009) to tol 1e-6 in three operator orders (mf, mf_rev,
   mf_split: make_noise_band.kop_variant), with the panel's Gram matrix in 64-row chunks added
   exactly (chunk64dd, make_nanotube_full.gram_in_order) and with that Gram matrix factored and
   substituted in 64-wide blocks (blk64: right-looking blocked Cholesky, blocked forward
   substitution -- the device's factor orders); the count to the reference's training
   tolerance 1e-4 is each trace's first crossing of 1e-4 ||b||.  The 'mf' solve is the reference
   trajectory, the others its band.

Writes tests/golden/ethanol_n74979.npz and ethanol_n74979_band.json.  CPU only: ~10 min for the
factor (--cache keeps L: 2.25 GB), then ~1 h for the solves (each solve's result is kept next
to the cache as it finishes, so an interrupted run resumes).
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

from make_nanotube_full import gram_in_order  # noqa: E402
from make_noise_band import half_decade_crossings, kop_variant  # noqa: E402
from oracle.pcg import cg_legacy  # noqa: E402
from oracle.sgdml import descriptors, kernel_column_matrix_free, kernel_diag  # noqa: E402
from sgdml_amd import synthetic  # noqa: E402  (input generation only)

M, N_ATOMS, SIG, LAM, K_RANK, TOL = 2777, 9, 10.0, 1e-10, 3752, 1e-6
JOBS = [("mf", ""), ("mf_rev", ""), ("mf_split", ""), ("mf", "chunk64dd"), ("mf", "blk64")]
_G = {}


def problem():
    ds = synthetic.ethanol_harmonic(M, seed=0)
    Rd, Rdd = descriptors(ds["R"])
    y, _ = synthetic.labels(ds["F"])
    return ds["R"], Rd, Rdd, np.arange(N_ATOMS)[None, :], y


def pivoted_cholesky_colmajor(get_col, diagonal, max_rank):
    """incomplete_cholesky.py:24-93 (as make_nanotube_full.pivoted_cholesky_logged) with L
    column-major; pivot values and top-two gaps logged."""
    diag = np.array(diagonal, dtype=np.float64, copy=True)
    n = diag.size
    index_columns = np.arange(n)
    L = np.zeros((n, max_rank), order="F")
    piv_val = np.empty(max_rank)
    gap = np.empty(max_rank)
    t0 = time.time()
    for m in range(max_rank):
        cand = diag[index_columns][m:]
        i_argmax = int(np.argmax(cand) + m)                                  # :53
        top2 = np.partition(cand, -2)[-2:]
        gap[m] = (top2[1] - top2[0]) / top2[1]
        index_columns[m], index_columns[i_argmax] = index_columns[i_argmax], index_columns[m]
        m_pi = index_columns[m]
        i_pi = index_columns[m + 1:]
        pivot_element = diag[m_pi]
        piv_val[m] = pivot_element
        assert pivot_element > 0, "given matrix is not PSD"                  # :62
        L[m_pi, m] = np.sqrt(pivot_element)
        k = get_col(m_pi)
        schur = L[:, :m] @ L[m_pi, :m] if m > 0 else np.zeros(n)             # :72 (all rows)
        L[i_pi, m] = (k[i_pi] - schur[i_pi]) / L[m_pi, m]                     # :75
        diag[i_pi] -= L[i_pi, m] ** 2                                         # :78
        if (m + 1) % 250 == 0:
            print(f"  pivot {m + 1}/{max_rank}  {time.time() - t0:.0f} s", flush=True)
    return L, index_columns, piv_val, gap


def _chol_blocked(A, nb):
    """Right-looking blocked Cholesky (lower) in nb-wide panels."""
    import scipy.linalg

    A = np.array(A, copy=True)
    k = A.shape[0]
    for j0 in range(0, k, nb):
        j1 = min(j0 + nb, k)
        A[j0:j1, j0:j1] = np.linalg.cholesky(A[j0:j1, j0:j1])
        if j1 < k:
            A[j1:, j0:j1] = scipy.linalg.solve_triangular(A[j0:j1, j0:j1], A[j1:, j0:j1].T,
                                                          lower=True).T
            A[j1:, j1:] -= A[j1:, j0:j1] @ A[j1:, j0:j1].T
    return np.tril(A)


def _trsm_blocked(L2, B, nb):
    """L2^-1 B by blocked forward substitution in nb-row blocks."""
    import scipy.linalg

    T = np.empty_like(B)
    for j0 in range(0, B.shape[0], nb):
        j1 = min(j0 + nb, B.shape[0])
        rhs = B[j0:j1] - L2[j0:j1, :j0] @ T[:j0] if j0 else B[j0:j1]
        T[j0:j1] = scipy.linalg.solve_triangular(L2[j0:j1, j0:j1], rhs, lower=True)
    return T


def panel(L, lam, gram):
    """T = chol(lam I + L^T L)^-1 L^T (iterative_cholesky.py:141-143), Gram in `gram` order;
    'blk64' = the chunk64dd Gram factored and substituted in 64-wide blocks."""
    import scipy.linalg

    if gram == "blk64":
        G = lam * np.eye(L.shape[1]) + gram_in_order(L, "chunk64dd")
        return _trsm_blocked(_chol_blocked(G, 64), np.ascontiguousarray(L.T), 64)
    G = gram_in_order(L, gram) if gram else L.T @ L
    L2 = scipy.linalg.cholesky(lam * np.eye(L.shape[1]) + G, lower=True)
    return scipy.linalg.solve_triangular(L2, L.T, lower=True)


def _name(job):
    return job[0] if not job[1] else f"panel_{job[1]}"


def _solve(job):
    import threadpoolctl

    order, gram = job
    Rd, Rdd, perms, y = _G["Rd"], _G["Rdd"], _G["perms"], _G["y"]
    t0 = time.time()
    with threadpoolctl.threadpool_limits(limits=2, user_api="blas"):
        T = _G["T"][gram]
        mvK = kop_variant(Rd, Rdd, perms, SIG, order, threads=_G["threads"])
        psolve = lambda r: (r - T.T @ (T @ r)) / LAM  # noqa: E731
        x, info, tr, it = cg_legacy(lambda v: -mvK(v) + LAM * v, y, tol=TOL, maxiter=5 * y.size,
                                    psolve=psolve)
    print(f"solve {_name(job):16s} iters {it} info {info} ({time.time() - t0:.0f} s)", flush=True)
    if _G["keep"] is not None:
        np.savez(_G["keep"](job), x=x, info=info, tr=tr, it=it)
    return job, x, info, tr, it


def first_below(tr, tol):
    hit = np.nonzero(tr[1:] <= tol * tr[0])[0]
    return int(hit[0]) + 1 if hit.size else None


def main(cache, procs):
    t_all = time.time()
    R, Rd, Rdd, perms, y = problem()
    n = y.size
    assert n == 74979
    if cache is not None and Path(cache).exists():
        c = np.load(cache, allow_pickle=False)
        L, piv, piv_val, gap = np.asfortranarray(c["L"]), c["piv"], c["piv_val"], c["gap"]
    else:
        def get_col(i):  # (-K_op) e_i (iterative_cholesky.py:152-156)
            col = -kernel_column_matrix_free(Rd, Rdd, perms, SIG, i)
            col[i] += LAM
            return col

        L, piv, piv_val, gap = pivoted_cholesky_colmajor(
            get_col, -kernel_diag(Rd, Rdd, perms, SIG), K_RANK)
        if cache is not None:
            np.savez(cache, L=L, piv=piv, piv_val=piv_val, gap=gap)
    print(f"pivoted Cholesky k={K_RANK}: {time.time() - t_all:.0f} s, min gap {gap.min():.3g}",
          flush=True)
    L = np.ascontiguousarray(L)
    keep = None if cache is None else (lambda job: Path(cache).with_name(
        Path(cache).stem + f"_{_name(job)}.npz"))
    done, todo = [], []
    for job in JOBS:
        if keep is not None and keep(job).exists():
            r = np.load(keep(job), allow_pickle=False)
            done.append((job, r["x"], int(r["info"]), r["tr"], int(r["it"])))
        else:
            todo.append(job)
    T = {g: panel(L, LAM, g) for g in sorted({g for _, g in todo})}
    print(f"panels {sorted(T)}: {time.time() - t_all:.0f} s", flush=True)
    _G.update(Rd=Rd, Rdd=Rdd, perms=perms, y=y, T=T, threads=max(1, 8 // procs), keep=keep)
    with mp.get_context("fork").Pool(procs) as pool:
        results = done + pool.map(_solve, todo, chunksize=1)
    runs = {_name(job): (x, info, tr, it) for job, x, info, tr, it in results}
    x0, info0, tr0, it0 = runs["mf"]
    out = {"n": n, "M": M, "k": K_RANK, "lam": LAM, "sig": SIG, "ref_order": "mf",
           "first_gap_below_1e-12": int(np.argmax(gap < 1e-12)) if np.any(gap < 1e-12) else None,
           "min_gap": float(gap.min()), "bands": {}}
    for tol in (1e-4, 1e-6):
        it_ref = first_below(tr0, tol) if tol > TOL else it0
        top = float(np.log10(np.minimum.accumulate(tr0[1:])[0]))
        sub0 = tr0[1:it_ref + 1]
        cr0 = half_decade_crossings(sub0, top)
        variants = {}
        for name, (x, info, tr, it) in runs.items():
            itv = first_below(tr, tol) if tol > TOL else it
            cr = half_decade_crossings(tr[1:itv + 1], top)
            dc = [abs(cr[q] - cr0[q]) for q in cr0 if q in cr]
            e = {"iters": int(itv), "d_iters": int(itv - it_ref), "max_d_crossing": int(max(dc) if dc else 0)}
            if tol == TOL:
                e["info"] = int(info)
                e["rel_dalpha"] = float(np.linalg.norm(x - x0) / np.linalg.norm(x0))
            variants[name] = e
        v = variants.values()
        b = {"tol": tol, "ref_order": "mf", "ref_iters": int(it_ref), "variants": variants,
             "band_iters": int(max(abs(e["d_iters"]) for e in v)),
             "band_crossing": int(max(e["max_d_crossing"] for e in v))}
        if tol == TOL:
            b["band_rel_dalpha"] = float(max(e["rel_dalpha"] for e in v))
        out["bands"][f"k{K_RANK}_tol{tol:g}"] = b
        print(f"tol {tol:g}", json.dumps({q: b.get(q) for q in ("ref_iters", "band_iters",
                                                             "band_crossing", "band_rel_dalpha")}),
              json.dumps({o: e["iters"] for o, e in variants.items()}), flush=True)
    np.savez_compressed(GOLDEN / "ethanol_n74979.npz", R=R, y=y, index_columns=piv[:K_RANK],
                        pivot_values=piv_val, pivot_gap=gap, trace=tr0, iters=np.int64(it0),
                        info=np.int64(info0), alphas=-x0)
    (GOLDEN / "ethanol_n74979_band.json").write_text(json.dumps(out, indent=1, sort_keys=True))
    print(f"total {time.time() - t_all:.0f} s", flush=True)


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--cache", default=None, help=".npz outside the repository for L (2.25 GB)")
    ap.add_argument("--procs", type=int, default=2)
    a = ap.parse_args()
    main(a.cache, a.procs)
