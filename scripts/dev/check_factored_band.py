"""CPU check (oracle level) that the record-factored sGDML operator of kernels_mf.hip
(k_rec_g / k_rec_fin) rounds like a change of summation order, not like a dense K v:
every golden solve is re-run with

  mf      the reference's matrix-free K_op in the oracle's order (make_noise_band.kop_variant)
  plain   c = 5 m (v . x_j),  y = sum c u - J^T G    (the GPU's regrouping)
  ref0    as plain, v . (x_j - x_j[atom 0])          (translation-exact c)
  exactc  c from diff . Zt (reference order), y = sum c u - J^T G

and the iteration counts are printed next to the reference's and the noise band
(tests/golden/noise_band.json).  Result (profiles/r02/factored_band.txt): `plain` is inside
2 b_it + 2 on all 20 golden solves.  CPU only; the nanotube cases take ~10 min each.

    python scripts/dev/check_factored_band.py sgdml_ethanol_n270/cholesky ...
"""
import sys, json, time
import numpy as np
REPO = __import__("pathlib").Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "tests" / "golden")]
from make_noise_band import dense_K, panel, half_decade_crossings, kop_variant, make_gemv, GOLDEN
from oracle.pcg import cg_legacy
from oracle.sgdml import descriptors, desc_perm

def factored(Rd, Rdd, perms, sig, mode):
    M, D = Rd.shape
    n = int((1 + np.sqrt(8 * D + 1)) / 2)
    P = np.array([desc_perm(p) for p in np.atleast_2d(perms)])
    npm = P.shape[0]
    s_at, t_at = np.tril_indices(n, k=-1)
    Rt = Rd[:, P]  # M x np x D
    sqrt5 = np.sqrt(5.0)
    def JT(Rddi, F):
        contrib = Rddi * F[:, None]
        yi = np.zeros((n, 3))
        np.add.at(yi, t_at, contrib)
        np.add.at(yi, s_at, -contrib)
        return yi
    U = np.zeros((M, M, npm, n, 3)); V = np.zeros((M, M, npm, n, 3))
    m5 = np.zeros((M, M, npm)); W = np.zeros((M, M, npm))
    for i in range(M):
        for j in range(M):
            for p in range(npm):
                diff = Rd[i] - Rt[j, p]
                norm = sqrt5 * np.sqrt(np.sum(diff * diff))
                m = np.exp(-norm / sig) * 5.0 / (3.0 * sig ** 4)
                m5[i, j, p] = 5.0 * m; W[i, j, p] = (sig ** 2 + sig * norm) * m
                U[i, j, p] = JT(Rdd[i], diff)
                dp = np.zeros(D); dp[P[p]] = diff
                V[i, j, p] = JT(Rdd[j], dp)
    def mv(x):
        X = np.asarray(x).reshape(M, n, 3)
        z = np.einsum("mdc,mdc->md", Rdd, X[:, t_at, :] - X[:, s_at, :])
        Zt = z[:, P]  # M x np x D
        Xr = X - X[:, :1, :] if mode == "ref0" else X
        y = np.empty((M, n, 3))
        for i in range(M):
            if mode == "exactc":
                diff = Rd[i][None, None, :] - Rt
                c = m5[i] * np.sum(diff * Zt, axis=-1)
            else:
                c = m5[i] * np.einsum("jpac,jac->jp", V[i], Xr)
            G = np.einsum("jp,jpd->d", W[i], Zt)
            y[i] = np.einsum("jp,jpac->ac", c, U[i]) - JT(Rdd[i], G)
        return y.reshape(-1)
    return mv

def run(name, precon, modes):
    f = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
    K = dense_K(f)
    y, lam, tol = f["y"], float(f["lam"]), float(f["solver_tol"])
    n = y.size
    T, sp = panel(f, precon, K, lam)
    ref_it = int(f[f"{precon}__num_iters"])
    Rd, Rdd = (f["R_desc"], f["R_d_desc"]) if "R_desc" in f.files else descriptors(f["R"])
    res = {"ref": ref_it}
    for mode in modes:
        if mode == "mf":
            mvK = kop_variant(Rd, Rdd, f["perms"], float(f["sig"]), "mf")
        else:
            mvK = factored(Rd, Rdd, f["perms"], float(f["sig"]), mode)
        x, info, tr, it = cg_legacy(lambda v: -mvK(v) + lam * v, y, tol=tol, maxiter=5 * n,
                                    psolve=lambda r: sp * ((r - T.T @ (T @ r)) / lam))
        res[mode] = it
    return res

band = json.load(open(REPO / "tests" / "golden" / "noise_band.json"))
cases = [(a, b) for a, b in [l.split("/") for l in sys.argv[1:]]]
for name, precon in cases:
    t = time.time()
    r = run(name, precon, ["mf", "plain", "ref0", "exactc"])
    b = band.get(f"{name}/{precon}", {})
    print(name, precon, r, "band_it", b.get("band_iters"), {k: v["iters"] for k, v in b.get("variants", {}).items()}, f"{time.time()-t:.0f}s", flush=True)
