"""Quick device-time probe of the K mat-vec and a PCG iteration (development aid)."""
import sys, time
from pathlib import Path
REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "mlff-preconditioner_amd")]
import numpy as np
import sgdml_amd
from sgdml_amd import synthetic

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
k = int(sys.argv[2]) if len(sys.argv) > 2 else 256
X, b = synthetic.rbf_points(n, 3, 0)
s = sgdml_amd.KernelSolver(n)
t0 = time.time(); s.gen_rbf(X, 0.2); print(f"gen_rbf {time.time()-t0:.3f}s", flush=True)
s.set_operator(1.0, 1e-6)
idx = np.sort(np.random.default_rng(0).choice(n, k, replace=False))
t0 = time.time(); s.precon_nystrom(idx); print(f"nystrom build {time.time()-t0:.3f}s", flush=True)
s.pcg_start(b, tol=0.0, maxiter=10**6)
s.pcg_run(5, 5)
s.timing(True); s.timing_reset()
t0 = time.time(); s.pcg_run(50, 50); el = time.time() - t0
t = s.timing_read()
g = t["gemv_ms"] / t["gemv_count"]
bytes_mv = 8.0 * n * n + 16.0 * n
print(f"n={n} gemv {g:.3f} ms  {bytes_mv/g/1e6:.1f} GB/s  iter {t['iter_ms']/t['iter_count']:.3f} ms  wall/it {el/50*1e3:.3f} ms", flush=True)
s.precon_none()
s.pcg_start(b, tol=0.0, maxiter=10**6); s.pcg_run(3, 3); s.timing_reset()
s.pcg_run(50, 50); t = s.timing_read()
print(f"no-precon iter {t['iter_ms']/t['iter_count']:.3f} ms gemv {t['gemv_ms']/t['gemv_count']:.3f} ms", flush=True)
