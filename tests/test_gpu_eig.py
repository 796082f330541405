"""The truncated eigensolver (csrc/kernels_eig.hip) behind the eigen preconditioners
(iterative_solver.py:1177-1329 `eigvec_precon*`, :1110-1175 `rank_k_lev_scores*`).

The reference decomposes all of K (scipy svd); here block subspace iteration on the
operator with Rayleigh-Ritz and a device Jacobi.  Checked against the oracle's exact
decomposition (numpy svd of the same S = -K): the k leading |eigenvalues|, the Woodbury
preconditioner it builds (which depends only on the k-dimensional invariant subspace)
and the row norms ||U[i, :k]||; on the matrix-free operator (no K assembled) and on
3 ranks (the same Q0 for every row split: results equal the one-rank run to rounding).
"""
import numpy as np
import pytest

from tests.conftest import load_golden
from tests.test_gpu_multirank import run_ranks

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sg():
    import sgdml_amd

    if sgdml_amd.device_count() < 1:
        pytest.fail("no GPU visible to libmlffpcg.so")
    return sgdml_amd


def _eig_case(sg, f, k, rank=0, world=1, key=None):
    n, lam = f["y"].size, float(f["lam"])
    v = np.random.default_rng(4).standard_normal(n)
    with sg.KernelSolver(n, device=0, rank=rank, world=world,
                         comm_id=key if world > 1 else None) as s:
        s.sgdml_operator(f["R_desc"], f["R_d_desc"], f["perms"], float(f["sig"]))
        s.set_operator(-1.0, lam)
        ev, rl = s.precon_eig(k, want_evals=True, want_rowlev=True)
        r0, r1 = s.row_range()
        z = s.precon_apply(np.ascontiguousarray(v[r0:r1]))
    return ev, rl, z, v


@pytest.mark.parametrize("name", ["sgdml_ethanol_n621", "sgdml_ethanol_n270_perms"])
def test_truncated_eig_matfree_vs_exact(sg, golden_dir, name):
    from oracle.precon import apply_panel, rank_k_lev_scores, svd_panel

    f = load_golden(golden_dir, name)
    k, lam = int(f["k_rot"]), float(f["lam"])
    ev, rl, z, v = _eig_case(sg, f, k)
    S = -np.asarray(f["K"])
    U, sv, _ = np.linalg.svd(S)
    np.testing.assert_allclose(ev, sv[:k], rtol=1e-9, atol=1e-12 * sv[0])
    np.testing.assert_allclose(rl, rank_k_lev_scores(S, k), rtol=1e-7, atol=1e-9)
    T, sp = svd_panel(S, k, lam)
    zref = apply_panel(T, sp, lam, v)
    assert np.linalg.norm(z - zref) <= 1e-6 * np.linalg.norm(zref)


@pytest.mark.parametrize("world", [2, 3])
def test_truncated_eig_sharded(sg, golden_dir, world):
    f = load_golden(golden_dir, "sgdml_ethanol_n621")
    k = int(f["k_rot"])
    ref = run_ranks(1, lambda r, w, key: _eig_case(sg, f, k, r, w, key))[0]
    outs = run_ranks(world, lambda r, w, key: _eig_case(sg, f, k, r, w, key))
    for ev, rl, _, _ in outs:
        np.testing.assert_allclose(ev, ref[0], rtol=1e-10)
        np.testing.assert_allclose(rl, ref[1], rtol=1e-8, atol=1e-10)
    z = np.concatenate([o[2] for o in outs])
    assert np.linalg.norm(z - ref[2]) <= 1e-6 * np.linalg.norm(ref[2])
