"""Residual traces of the nanotube n3330 drop-in solve (cholesky) with and without the
folded k_update_xr (MLFF_FUSE_XR), one child process each; prints where they part."""
import json
import os
import subprocess
import sys

import numpy as np

CHILD = r'''
import json, sys, numpy as np
sys.path.insert(0, "."); sys.path.insert(0, "mlff-preconditioner_amd")
import sgdml_amd as sg
from tests.test_gpu_golden import run_dropin, load, NANOTUBE
from pathlib import Path
f = load(Path("tests/golden"), NANOTUBE)
desc = sg.sgdml_descriptors(f["R"])
a, it, res, rmse, idx, conv, info = run_dropin(f, NANOTUBE, "cholesky", desc)
print(json.dumps({"iters": int(it), "trace": [float(v) for v in info["resid_trace"]]}))
'''

out = {}
for v in ("0", "1"):
    env = dict(os.environ, MLFF_FUSE_XR=v)
    p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True)
    line = [l for l in p.stdout.splitlines() if l.startswith("{")]
    if not line:
        print(p.stdout[-2000:], p.stderr[-3000:])
        sys.exit(1)
    out[v] = json.loads(line[-1])
a, b = np.array(out["0"]["trace"]), np.array(out["1"]["trace"])
print("iters", out["0"]["iters"], out["1"]["iters"], "len", a.size, b.size)
for i in range(max(a.size - 6, 0), min(a.size + 3, b.size)):
    print("tail", i, a[i] if i < a.size else None, b[i])
m = min(a.size, b.size)
rel = np.abs(a[:m] - b[:m]) / np.maximum(np.abs(a[:m]), 1e-300)
for i in range(min(m, 12)):
    print(i, a[i], b[i], rel[i])
bad = np.nonzero(rel > 1e-8)[0]
print("first index > 1e-8:", bad[:10])
