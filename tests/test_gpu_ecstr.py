"""Energy constraints (use_E_cstr) on the GPU against the reference's own outputs.

tests/golden/*_ecstr.npz (tests/golden/make_golden.py fx_ecstr) hold the reference's
_assemble_kernel_mat(use_E_cstr=True) (train.py:212-236: M energy rows / columns after the
3 n M force rows) and its operator closure _K_vec on an (N + M)-vector
(iterative_solver.py:416-443: forces from GDMLPredict with alphas_E, predict.py:206-218,
and the predicted energies with a flipped sign).  Its Iterative.solve itself raises with
use_E_cstr (the operator is sized 3 n M, the labels 3 n M + M), so the drop-in raises the
same ValueError; the energy-constrained system is solved here through KernelSolver, against
the oracle's dense K (parity of the solve itself: unpinned by the reference, which cannot
run it).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ECSTR = ["sgdml_ethanol_n270_ecstr", "sgdml_ethanol_n270_perms_ecstr"]


def load(golden_dir, name):
    return np.load(golden_dir / f"{name}.npz", allow_pickle=False)


@pytest.fixture(scope="module")
def sg():
    import sgdml_amd

    if sgdml_amd.device_count() < 1:
        pytest.fail("no GPU visible to libmlffpcg.so")
    return sgdml_amd


@pytest.mark.parametrize("name", ECSTR)
def test_ecstr_assembly_and_operators(sg, golden_dir, name):
    """Assembled K with the energy border vs the reference's (1e-13); the dense and the
    matrix-free operators vs the reference's _K_vec; the diagonal incl. K[E_i, E_i]."""
    f = load(golden_dir, name)
    N, lam = f["y"].size, float(f["lam"])
    with sg.KernelSolver(N) as s:
        s.assemble_sgdml(f["R_desc"], f["R_d_desc"], f["perms"], float(f["sig"]), use_E_cstr=True)
        K = s.get_matrix_rows()
        s.set_operator(-1.0, lam)
        out = {}
        for storage in ("dense", "matfree"):
            s.set_storage(storage)
            out[storage] = s.matvec(f["v"])
        d = s.diag()
    scale = np.abs(f["K"]).max()
    assert K.shape == f["K"].shape
    assert np.max(np.abs(K - f["K"])) <= 1e-13 * scale
    ref = f["Kop_v"]  # K v - lam v; ours: -K v + lam v
    for storage, Av in out.items():
        assert np.linalg.norm(-Av - ref) <= 1e-13 * np.linalg.norm(ref), storage
    np.testing.assert_allclose(d, -np.diag(f["K"]), rtol=1e-12)


@pytest.mark.parametrize("name", ECSTR)
def test_ecstr_matrix_free_only(sg, golden_dir, name):
    """The matrix-free operator alone (no assembly): _K_vec and the diagonal."""
    f = load(golden_dir, name)
    N, lam = f["y"].size, float(f["lam"])
    with sg.KernelSolver(N) as s:
        s.sgdml_operator(f["R_desc"], f["R_d_desc"], f["perms"], float(f["sig"]), use_E_cstr=True)
        s.set_operator(-1.0, lam)
        Av = s.matvec(f["v"])
        d = s.diag()
        assert s.storage_info()[0] == "matfree"
    ref = f["Kop_v"]
    assert np.linalg.norm(-Av - ref) <= 1e-13 * np.linalg.norm(ref)
    np.testing.assert_allclose(d, -np.diag(f["K"]), rtol=1e-12)


def test_ecstr_pivchol_pcg(sg, golden_dir):
    """The (3 n M + M) system solved through the matrix-free operator with a pivoted-Cholesky
    preconditioner whose columns are K_op e_g (energy columns included): the pivot sequence
    equals the oracle's on the reference's K up to its first near-tie, and the converged
    solution's true residual, recomputed on the host with the reference's K, meets the
    tolerance."""
    from oracle.precon import pivoted_cholesky

    f = load(golden_dir, "sgdml_ethanol_n270_ecstr")
    N, lam = f["y"].size, float(f["lam"])
    K = f["K"]
    S = -K
    k = 40
    _, piv_ref = pivoted_cholesky(lambda i: S[:, i] + lam * (np.arange(N) == i), np.diag(S).copy(), k)
    with sg.KernelSolver(N) as s:
        s.sgdml_operator(f["R_desc"], f["R_d_desc"], f["perms"], float(f["sig"]), use_E_cstr=True)
        s.set_operator(-1.0, lam)
        piv, _ = s.precon_pivchol(k)
        res = s.pcg(f["y"], tol=1e-6, maxiter=5 * N)
    # pivots: identical until the first near-tie of the reference's diagonal update
    same = int(np.argmax(piv[:k] != piv_ref[:k])) if np.any(piv[:k] != piv_ref[:k]) else k
    assert same >= 8, (piv[:12], piv_ref[:12])
    assert res.info == 0
    r = f["y"] - (S @ res.x + lam * res.x)
    assert np.linalg.norm(r) <= 1.05e-6 * np.linalg.norm(f["y"])


def test_ecstr_dropin_raises_like_reference(sg, golden_dir):
    """Iterative.solve with task['use_E_cstr'] raises ValueError, as the reference's does
    (recorded in the fixture for cholesky and eigvec_precon)."""
    from sgdml_amd.solvers import Iterative

    f = load(golden_dir, "sgdml_ethanol_n270_ecstr")
    M, n = f["R"].shape[:2]
    task = {"R_train": f["R"], "F_train": f["F"], "E_train": f["E"], "z": f["z"],
            "perms": f["perms"], "sig": 10.0, "lam": 1e-10, "solver_tol": 1e-4,
            "truncated_cholesky": 1500, "n_inducing_pts_init": 25, "use_E": True,
            "use_E_cstr": True}
    it = Iterative(None, None)
    with pytest.raises(ValueError):
        it.solve(task, f["R_desc"], f["R_d_desc"], f["tril_perms_lin"], f["y"], float(f["y_std"]),
                 break_percentage=0.2, str_preconditioner="cholesky")
    assert str(f["cholesky__error"]).startswith("ValueError")
