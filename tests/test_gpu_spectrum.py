"""Iterative.solve(flag_eigvals=True) against the reference's own spectra.

tests/golden/sgdml_ethanol_n270_eigvals.npz (make_golden.py fx_eigvals) holds, for three
preconditioners, the reference's info['eigvals'] = scipy.linalg.eigvals(P_op @ K) and
info['eigvals_K'] = eigvals(K), K = -K_op column by column (iterative_solver.py:978-989,
dev_utils.py:8-25), and its 10-iteration CG (:1002).  The reference's arrays are complex in
LAPACK order (imaginary parts <= 1.4e-6 of eigenvalues up to 7e5: rounding of the
non-symmetric eigensolver); the drop-in's are real and descending (P_op K is similar to a
symmetric matrix), compared sorted.  Tolerance: 1e-6 relative per eigenvalue + 1e-10 of the
largest.  Both codes form P_op ~ 1/lam = 1e10 and reach the eigenvalue-1 cluster (the
directions the preconditioner captures) through a cancellation of that scale: the
reference's own non-symmetric solver leaves imaginary parts up to 1.4e-6 there, and the
two spectra differ by up to 2.8e-6 in that cluster (measured), 1e-10 x 3.8e5 = 3.8e-5
above it.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NAME = "sgdml_ethanol_n270_eigvals"


@pytest.fixture(scope="module")
def fx(golden_dir):
    import sgdml_amd

    if sgdml_amd.device_count() < 1:
        pytest.fail("no GPU visible to libmlffpcg.so")
    return np.load(golden_dir / f"{NAME}.npz", allow_pickle=False)


def task_of(f):
    return {"R_train": f["R"], "F_train": f["F"], "E_train": f["E"], "z": f["z"],
            "perms": f["perms"], "sig": float(f["sig"]), "lam": float(f["lam"]),
            "solver_tol": float(f["solver_tol"]), "truncated_cholesky": 1500,
            "n_inducing_pts_init": 25, "use_E_cstr": False, "use_E": True}


def close_spectra(ours, ref):
    ref = np.sort(np.real(ref))[::-1]
    assert ours.shape == ref.shape
    tol = 1e-6 * np.abs(ref) + 1e-10 * np.abs(ref).max()
    bad = np.abs(ours - ref) > tol
    assert not bad.any(), (np.nonzero(bad)[0][:5], ours[bad][:5], ref[bad][:5])


@pytest.mark.parametrize("precon", ["cholesky", "random_scores", "eigvec_precon"])
def test_flag_eigvals_matches_reference(fx, precon):
    from sgdml_amd.solvers import Iterative

    f = fx
    n = f["y"].size
    np.random.seed(1003)  # the fixture generator's seed (host-side column draws)
    with Iterative(None, None, device=0) as it:
        alphas, num_iters, resid, rmse, idxs, is_conv, info = it.solve(
            task_of(f), f["R_desc"], f["R_d_desc"], f["tril_perms_lin"], f["y"], float(f["y_std"]),
            break_percentage=int(f["k_rot"]) / n, str_preconditioner=precon, flag_eigvals=True)
    # the reference stops its CG after 10 iterations when the spectra are requested (:1002)
    assert num_iters == int(f[f"{precon}__num_iters"]) == 10
    assert bool(is_conv) == bool(f[f"{precon}__is_conv"])
    close_spectra(info["eigvals_K"], f[f"{precon}__eigvals_K"])
    close_spectra(info["eigvals"], f[f"{precon}__eigvals"])
    if precon == "cholesky":
        np.testing.assert_array_equal(idxs, f[f"{precon}__inducing_pts_idxs"])
