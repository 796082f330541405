import sys, time, json
import numpy as np, scipy.linalg
sys.path[:0] = ['/root/repo', '/root/repo/mlff-preconditioner_amd', '/root/repo/tests/golden']
from make_noise_band import kop_variant
from oracle.sgdml import descriptors, kernel_diag
from oracle.precon import pivoted_cholesky
from oracle.pcg import cg_legacy
from sgdml_amd import synthetic
from sgdml_amd.rule_of_thumb import get_params, rule_of_thumb
M = int(sys.argv[1]) if len(sys.argv) > 1 else 583
LAM, SIG = 1e-10, 10.0
ds = synthetic.ethanol_like(M, seed=0)
y, _ = synthetic.labels(ds["F"])
n = y.size
m, kmin, _ = get_params("ethanol")
k = int(rule_of_thumb(n=n, k_min=kmin, m=m))
Rd, Rdd = descriptors(ds["R"])
P = np.arange(9)[None, :]
mv = kop_variant(Rd, Rdd, P, SIG, "mf")
t0 = time.time()
def get_col(i):
    e = np.zeros(n); e[i] = 1.0
    return -mv(e) + LAM * e
L, piv = pivoted_cholesky(get_col, -kernel_diag(Rd, Rdd, P, SIG), k)
print("pivchol", k, time.time() - t0, flush=True)
sv = np.linalg.svd(L, compute_uv=False)
print("sigma2 max/min", sv[0]**2, sv[-1]**2, "cond_A", np.sqrt((sv[0]**2 + LAM) / (sv[-1]**2 + LAM)), flush=True)
G = LAM * np.eye(k) + L.T @ L
L2 = scipy.linalg.cholesky(G, lower=True)
T = scipy.linalg.solve_triangular(L2, L.T, lower=True)
Li = scipy.linalg.solve_triangular(L2, np.eye(k), lower=True)
G2 = T @ T.T + LAM * (Li @ Li.T)
print("G2-I max", np.abs(G2 - np.eye(k)).max(), flush=True)
C = scipy.linalg.cholesky(G2, lower=True)
T2 = scipy.linalg.solve_triangular(C, T, lower=True)
for name, TT in (("onestep", T), ("refined", T2)):
    t0 = time.time()
    x, info, tr, it = cg_legacy(lambda v: -mv(v) + LAM * v, y, tol=1e-6, maxiter=4000,
                                psolve=lambda r, TT=TT: (r - TT.T @ (TT @ r)) / LAM)
    print(name, it, info, tr[-1] / np.linalg.norm(y), time.time() - t0, flush=True)
