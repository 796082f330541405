"""Build-time sweep of the persistent pivoted Cholesky (k_piv_persist) on the configs[1] nanotube:
grid sizes (MLFF_PIV_G) against the launch sequence (MLFF_PIVCHOL_PERSIST=0), with the per-phase
trace (MLFF_PIV_TRACE) on stderr.  Usage: python scripts/dev/piv_persist_sweep.py [k]"""
import os
import sys
import time

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", ".."),
                os.path.join(os.path.dirname(__file__), "..", "..", "mlff-preconditioner_amd")]
import sgdml_amd  # noqa: E402
from sgdml_amd import synthetic  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 2701
only = sys.argv[2] if len(sys.argv) > 2 else None  # e.g. "G=64": that configuration only
ds = synthetic.nanotube_like(14, seed=0)
Rd, Rdd = sgdml_amd.sgdml_descriptors(ds["R"])
y, _ = synthetic.labels(ds["F"])
n = y.size
ref = None
configs = [("legacy", {"MLFF_PIVCHOL_PERSIST": "0"})] + [
    (f"G={g}", {"MLFF_PIVCHOL_PERSIST": "1", "MLFF_PIV_G": str(g)}) for g in (256, 128, 64)]
if only is not None:
    configs = [c for c in configs if c[0] == only]
for rep in range(2):
    for name, env in configs:
        for key in ("MLFF_PIV_G", "MLFF_PIV_TRACE"):
            os.environ.pop(key, None)
        os.environ.update(env)
        if rep == 1 and name != "legacy":
            os.environ["MLFF_PIV_TRACE"] = "1"
        with sgdml_amd.KernelSolver(n) as s:
            s.sgdml_operator(Rd, Rdd, np.arange(370)[None, :], 10.0)
            s.set_operator(-1.0, 1e-10)
            piv, sec = s.precon_pivchol(k, build_woodbury=False)
            Lt = s.precon_panel()
        same = ""
        if ref is None:
            ref = (piv, Lt)
        else:
            same = "bitwise" if (np.array_equal(piv, ref[0]) and np.array_equal(Lt, ref[1])) else "DIFFERENT"
        print(f"rep {rep} {name:8s} k={k}: {sec:.4f} s  {1e6 * sec / k:.1f} us/step  {same}", flush=True)
