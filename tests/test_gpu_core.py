"""GPU parity of the HIP kernels against the CPU oracle (small sizes).

Every test calls through the C ABI (sgdml_amd.KernelSolver -> libmlffpcg.so).
Tolerances: fp64 kernels whose summation order differs from NumPy's are held to
1e-12 relative (mat-vec, assembly) and the preconditioned PCG to identical
iteration counts with pointwise |log10(r_gpu / r_cpu)| <= 1e-4 and final
||dx|| / ||x|| <= 1e-6 (SURVEY.md 8(c) parity contract).
"""
import numpy as np
import pytest

from tests.parity import assert_pcg_parity

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sg():
    import sgdml_amd

    if sgdml_amd.device_count() < 1:
        pytest.fail("no GPU visible to libmlffpcg.so")
    return sgdml_amd


def _rbf(n, d=3, ell=0.2, seed=0):
    from sgdml_amd import synthetic

    return synthetic.rbf_points(n, d, seed)


def test_gen_rbf_matches_sklearn_recipe(sg):
    from oracle.rbf import rbf_kernel

    X, _ = _rbf(1001)
    with sg.KernelSolver(1001) as s:
        s.gen_rbf(X, length_scale=0.2, jitter=1e-10)
        K = s.get_matrix_rows()
    Kref = rbf_kernel(X, 0.2, jitter=1e-10)
    assert np.max(np.abs(K - Kref)) <= 4e-16
    assert np.array_equal(K, K.T)


def test_matvec_sigma_lam(sg):
    rng = np.random.default_rng(1)
    n = 777
    A = rng.standard_normal((n, n))
    K = A @ A.T / n
    v = rng.standard_normal(n)
    with sg.KernelSolver(n) as s:
        s.set_matrix(K)
        s.set_operator(-1.0, 1e-10)
        y = s.matvec(v)
        d = s.diag()
    yref = -(K @ v) + 1e-10 * v
    assert np.linalg.norm(y - yref) <= 1e-13 * np.linalg.norm(yref)
    assert np.allclose(d, -np.diag(K), rtol=0, atol=0)


def test_pcg_none_matches_oracle(sg):
    from oracle.pcg import cg_legacy
    from oracle.rbf import rbf_kernel

    n, lam = 900, 1e-2
    X, b = _rbf(n)
    K = rbf_kernel(X, 0.2)
    with sg.KernelSolver(n) as s:
        s.gen_rbf(X, length_scale=0.2)
        s.set_operator(1.0, lam)
        s.precon_none()
        res = s.pcg(b, tol=1e-8, maxiter=5 * n, chunk=7)
    x_ref, info, tr, it = cg_legacy(lambda v: K @ v + lam * v, b, tol=1e-8, maxiter=5 * n)
    assert res.info == info == 0
    # ~345 unpreconditioned iterations: chaotic regime (tests/parity.py)
    assert_pcg_parity(res.iters, res.trace[1:], res.x, it, tr[1:], x_ref, mode="chaotic",
                      x_tol=1e-6)


def test_pivchol_woodbury_and_pcg(sg):
    from oracle.pcg import cg_legacy
    from oracle.precon import apply_panel, pivoted_cholesky, woodbury_panel
    from oracle.rbf import rbf_kernel

    n, k, lam = 1200, 200, 1e-6
    X, b = _rbf(n)
    K = rbf_kernel(X, 0.2)
    with sg.KernelSolver(n) as s:
        s.gen_rbf(X, length_scale=0.2)
        s.set_operator(1.0, lam)
        piv, _ = s.precon_pivchol(k)
        T = s.precon_panel()
        r = np.random.default_rng(3).standard_normal(n)
        z = s.precon_apply(r)
        res = s.pcg(b, tol=1e-6, maxiter=5 * n)
    L, piv_ref = pivoted_cholesky(lambda i: K[:, i], np.diag(K).copy(), k)
    assert np.array_equal(piv[:k], piv_ref[:k])
    Tref, sp = woodbury_panel(L, lam)
    assert np.allclose(np.abs(T), np.abs(Tref), rtol=1e-8, atol=1e-10)
    zref = apply_panel(Tref, sp, lam, r)
    assert np.linalg.norm(z - zref) <= 1e-8 * np.linalg.norm(zref)
    x_ref, info, tr, it = cg_legacy(lambda v: K @ v + lam * v, b, tol=1e-6, maxiter=5 * n,
                                    psolve=lambda v: apply_panel(Tref, sp, lam, v))
    assert res.info == info == 0
    # ~1260 iterations at lam = 1e-6: the chaotic regime (CPU noise floor 1261-1268)
    assert_pcg_parity(res.iters, res.trace[1:], res.x, it, tr[1:], x_ref, mode="chaotic",
                      x_tol=1e-4)


@pytest.mark.parametrize("kind", ["pivchol", "nystrom0", "nystrom1"])
def test_pcg_stable_regime_exact(sg, kind):
    """Well-conditioned preconditioned system: identical iteration counts and
    pointwise residual curves (stable parity contract)."""
    from oracle.pcg import cg_legacy
    from oracle.precon import apply_panel, nystrom_panel, pivoted_cholesky, woodbury_panel
    from oracle.rbf import rbf_kernel

    n, k, lam = 1500, 200, 1e-1
    X, b = _rbf(n, seed=9)
    K = rbf_kernel(X, 0.2)
    idx = np.sort(np.random.default_rng(2).choice(n, k, replace=False))
    with sg.KernelSolver(n) as s:
        s.gen_rbf(X, length_scale=0.2)
        s.set_operator(1.0, lam)
        if kind == "pivchol":
            s.precon_pivchol(k)
            L, _ = pivoted_cholesky(lambda i: K[:, i], np.diag(K).copy(), k)
            T, sp = woodbury_panel(L, lam)
        else:
            v = int(kind[-1])
            s.precon_nystrom(idx, variant=v)
            T, sp = nystrom_panel(K[:, idx], idx, lam, v)
        res = s.pcg(b, tol=1e-8, maxiter=5 * n)
    x_ref, info, tr, it = cg_legacy(lambda v: K @ v + lam * v, b, tol=1e-8, maxiter=5 * n,
                                    psolve=lambda r: apply_panel(T, sp, lam, r))
    assert res.info == info == 0
    assert_pcg_parity(res.iters, res.trace[1:], res.x, it, tr[1:], x_ref, mode="stable")


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("form", ["auto", "one_pass", "cluster"])
def test_nystrom_apply(sg, monkeypatch, variant, form):
    """Nystrom applies (both variants, their opposite signs sigma_p) against the oracle, on
    the apply form the size selects, forced onto the one-pass rows form, and on the cluster
    form (N = 20000: rows longer than a workgroup)."""
    from oracle.precon import apply_panel, nystrom_panel
    from oracle.rbf import rbf_kernel

    n, k, lam = (20000, 400, 1e-6) if form == "cluster" else (1000, 64, 1e-6)
    if form == "one_pass":
        monkeypatch.setenv("MLFF_LR_ROWS", "1")
    X, _ = _rbf(n)
    K = rbf_kernel(X, 0.2)
    idx = np.sort(np.random.default_rng(5).choice(n, k, replace=False))
    r = np.random.default_rng(6).standard_normal(n)
    with sg.KernelSolver(n) as s:
        s.gen_rbf(X, length_scale=0.2)
        s.set_operator(1.0, lam)
        s.precon_nystrom(idx, variant=variant)
        if form != "auto":
            assert s.precon_apply_traffic()[0] == (1 if form == "one_pass" else 2)
        z = s.precon_apply(r)
    B, sp = nystrom_panel(K[:, idx], idx, lam, variant=variant)
    zref = apply_panel(B, sp, lam, r)
    assert np.linalg.norm(z - zref) <= 1e-6 * np.linalg.norm(zref)


def test_lev_scores(sg):
    from oracle.precon import lev_scores
    from oracle.rbf import rbf_kernel

    n, k, lam = 800, 40, 1e-10
    X, _ = _rbf(n)
    K = rbf_kernel(X, 0.3)
    idx = np.sort(np.random.default_rng(7).choice(n, k, replace=False))
    with sg.KernelSolver(n) as s:
        s.gen_rbf(X, length_scale=0.3)
        lev = s.lev_scores(idx, lam)
    ref = lev_scores(K[:, idx], idx, lam)
    assert np.allclose(lev, ref, rtol=1e-6, atol=1e-9)


def test_descriptors(sg):
    from oracle.sgdml import descriptors
    from sgdml_amd import synthetic, sgdml_descriptors

    d = synthetic.ethanol_like(6, seed=2)
    Rd, Rdd = sgdml_descriptors(d["R"])
    Rd0, Rdd0 = descriptors(d["R"])
    assert np.allclose(Rd, Rd0, rtol=1e-14, atol=0)
    assert np.allclose(Rdd, Rdd0, rtol=1e-13, atol=1e-16)


@pytest.mark.parametrize("perms", ["identity", "methyl", "c3group"])
def test_sgdml_assembly(sg, perms):
    from oracle.sgdml import assemble_kernel, descriptors, tril_perms_lin
    from sgdml_amd import synthetic

    d = synthetic.ethanol_like(7, seed=4)
    Rd, Rdd = descriptors(d["R"])
    P = np.arange(9)[None, :]
    if perms == "methyl":  # permute the methyl hydrogens (atoms 3, 4, 5)
        P = np.array([np.arange(9), [0, 1, 2, 4, 5, 3, 6, 7, 8], [0, 1, 2, 5, 3, 4, 7, 6, 8]])
    if perms == "c3group":  # a proper group: rotations of the methyl hydrogens
        P = np.array([np.arange(9), [0, 1, 2, 4, 5, 3, 6, 7, 8], [0, 1, 2, 5, 3, 4, 6, 7, 8]])
    K_ref = assemble_kernel(Rd, Rdd, tril_perms_lin(P), 10.0)
    n = K_ref.shape[0]
    with sg.KernelSolver(n) as s:
        s.assemble_sgdml(Rd, Rdd, P, 10.0)
        K = s.get_matrix_rows()
    scale = np.max(np.abs(K_ref))
    assert np.max(np.abs(K - K_ref)) <= 1e-12 * scale


@pytest.mark.parametrize("mask", [0, 1])
def test_eig_preconditioner_apply(sg, mask):
    """svd_preconditioner (iterative_solver.py:1313-1329): L = U sqrt(s)[:, :k] + Woodbury."""
    from oracle.precon import apply_panel, svd_panel
    from oracle.rbf import rbf_kernel

    n, k, lam = 700, 60, 1e-4
    X, _ = _rbf(n)
    K = rbf_kernel(X, 0.2)
    r = np.random.default_rng(8).standard_normal(n)
    with sg.KernelSolver(n) as s:
        s.gen_rbf(X, length_scale=0.2)
        s.set_operator(1.0, lam)
        ev, lev = s.precon_eig(k, mask_mode=mask, want_evals=True, want_rowlev=True)
        z = s.precon_apply(r)
    if mask == 1:  # block_diagonal zeroes the whole kernel: P = I / lam
        np.testing.assert_allclose(z, r / lam, rtol=1e-14)
        return
    T, sp = svd_panel(K, k, lam)
    zref = apply_panel(T, sp, lam, r)
    assert np.linalg.norm(z - zref) <= 1e-8 * np.linalg.norm(zref)
    U, sv, _ = np.linalg.svd(K)
    np.testing.assert_allclose(ev, sv[:k], rtol=1e-10, atol=1e-12 * sv[0])
    np.testing.assert_allclose(lev, np.linalg.norm(U[:, :k], axis=1), rtol=1e-7, atol=1e-10)


@pytest.mark.parametrize("case", ["warm", "early"])
def test_pcg_x0_legacy_semantics(sg, case):
    """Initial guess as scipy 1.7.3's cg treats it (iterative_solver.py:995-1005 passes
    x0 = -alphas0_F): r0 = b - A x0; the legacy pre-check ||A x0 - b|| <= tol returns x0
    untouched (no iteration, no callback)."""
    from oracle.pcg import cg_legacy
    from oracle.precon import apply_panel, pivoted_cholesky, woodbury_panel
    from oracle.rbf import rbf_kernel

    n, k, lam = 1500, 200, 1e-1
    X, b = _rbf(n, seed=9)
    K = rbf_kernel(X, 0.2)
    A = K + lam * np.eye(n)
    rng = np.random.default_rng(5)
    if case == "warm":
        x0, tol = 0.05 * rng.standard_normal(n), 1e-8
    else:
        x0, tol = np.linalg.solve(A, b), 1e-6
    with sg.KernelSolver(n) as s:
        s.gen_rbf(X, length_scale=0.2)
        s.set_operator(1.0, lam)
        s.precon_pivchol(k)
        res = s.pcg(b, x0, tol=tol, maxiter=5 * n)
    L, _ = pivoted_cholesky(lambda i: K[:, i], np.diag(K).copy(), k)
    T, sp = woodbury_panel(L, lam)
    x_ref, info, tr, it = cg_legacy(lambda v: A @ v, b, x0=x0, tol=tol, maxiter=5 * n,
                                    psolve=lambda r: apply_panel(T, sp, lam, r))
    assert res.info == info == 0
    if case == "early":
        assert res.early_exit and res.iters == it == 0 and res.callbacks == 0
        np.testing.assert_array_equal(res.x, x0)
        return
    assert not res.early_exit and res.iters > 0
    np.testing.assert_allclose(res.trace[0], tr[0], rtol=1e-12)
    assert_pcg_parity(res.iters, res.trace[1:], res.x, it, tr[1:], x_ref, mode="stable")


def test_call_order_and_argument_errors(sg):
    """State / argument errors surface as the reference's exception types
    (RuntimeError for call-order errors, ValueError for bad arguments) and leave the
    context usable."""
    from sgdml_amd import synthetic

    n = 300
    X, b = synthetic.rbf_points(n, 3, 1)
    with sg.KernelSolver(n) as s:
        with pytest.raises(RuntimeError):
            s.pcg(b, tol=1e-6)                      # no operator yet
        s.gen_rbf(X, 0.2)
        with pytest.raises(RuntimeError):
            s.precon_pivchol(10)                    # mlff_set_operator not called
        s.set_operator(1.0, 1e-2)
        with pytest.raises(ValueError):
            s.precon_nystrom(np.array([5, 3, 9]))   # unsorted (train.py:1197-1201)
        with pytest.raises(ValueError):
            s.precon_nystrom(np.array([1, 1, 2]))   # duplicate
        with pytest.raises(ValueError):
            s.precon_nystrom(np.array([0, n]))      # out of range
        with pytest.raises(ValueError):
            s.precon_pivchol(n + 1)
        with pytest.raises(ValueError):
            s.matvec(np.zeros(n + 1))
        s.precon_pivchol(20)                        # still usable
        res = s.pcg(b, tol=1e-8, maxiter=5 * n)
        assert res.info == 0


@pytest.mark.parametrize("n,k,clusters", [(1000, 3, 0), (1000, 800, 0), (5000, 1031, 0),
                                          (11000, 900, 0), (15540, 2701, 0),
                                          (20000, 400, 0), (40000, 301, 0), (40000, 301, 3),
                                          (70000, 40, 7)])
def test_one_pass_lowrank_apply(sg, monkeypatch, n, k, clusters):
    """The one-pass low-rank apply (k_lr_rows + k_lr_fin: each panel row read once, t_i
    kept in the workgroup) against the two-pass apply (T r, then T^T t) and NumPy, on
    every register-tile width (M = 4, 8, 12, 16 double2 per thread), ragged row groups
    (k = 1031: 207 groups of 5 rows, the last of 1) and k < one row per workgroup; rows
    longer than 16384 columns take the cluster form (k_lr_cluster: C = 3, 6, 10 workgroups per
    row, all resident clusters or MLFF_LR_CLUSTERS of them, ragged row ranges).  Then a
    PCG solve on both applies, held to the chaotic-regime contract of tests/parity.py (a
    random panel makes a poor preconditioner: the residual curves of two summation orders
    part after ~15 iterations, as they do on the CPU).
    Reference: iterative_cholesky.py:145-148 (z = (r - T^T T r) / lam)."""
    lam = 1.0
    X, b = _rbf(n)
    rng = np.random.default_rng(n + k)
    L = rng.standard_normal((k, n)) * 0.05
    r = rng.standard_normal(n)
    out = {}
    if clusters:
        monkeypatch.setenv("MLFF_LR_CLUSTERS", str(clusters))
    for mode in ("0", "1"):
        monkeypatch.setenv("MLFF_LR_ROWS", mode)
        with sg.KernelSolver(n) as s:
            s.gen_rbf(X, length_scale=0.2)
            s.set_operator(1.0, lam)
            s.precon_lowrank(L)
            form, _ = s.precon_apply_traffic()
            assert form == (0 if mode == "0" else (1 if n <= 16384 else 2))
            T = s.precon_panel()
            z = s.precon_apply(r)
            res = s.pcg(b, tol=1e-8, maxiter=5 * n)
        out[mode] = (T, z, res)
    T, z1, res1 = out["1"]
    _, z0, res0 = out["0"]
    zref = (r - T.T @ (T @ r)) / lam
    sgn = np.sign(np.dot(z0, zref))  # sigma_p of the low-rank operator
    assert np.linalg.norm(z0 - sgn * zref) <= 1e-12 * np.linalg.norm(zref)
    assert np.linalg.norm(z1 - z0) <= 1e-13 * np.linalg.norm(z0)
    assert res0.info == res1.info == 0
    assert_pcg_parity(res1.iters, res1.trace[1:], res1.x, res0.iters, res0.trace[1:], res0.x,
                      mode="chaotic", x_tol=1e-6)


def test_cluster_apply_fault_falls_back(sg, monkeypatch):
    """A cluster member that never publishes its partial (test hook MLFF_LC_TEST_MUTE) makes
    its cluster's hand-offs time out: the members leave after ~0.1 s instead of hanging the GPU,
    the apply is redone with two passes (correct z), the context stays on the two-pass form;
    in a PCG solve the faulted iteration is re-run with two passes and the solve converges to
    the result of a two-pass solve."""
    n, k, lam = 40000, 301, 1.0
    X, b = _rbf(n)
    rng = np.random.default_rng(5)
    L = rng.standard_normal((k, n)) * 0.05
    r = rng.standard_normal(n)
    with sg.KernelSolver(n) as s:
        s.gen_rbf(X, length_scale=0.2)
        s.set_operator(1.0, lam)
        s.precon_lowrank(L)
        T = s.precon_panel()
        ref = s.pcg(b, tol=1e-8, maxiter=2000)  # cluster form, no fault
        monkeypatch.setenv("MLFF_LC_TEST_MUTE", "3")
        s.precon_lowrank(L)  # a fresh panel: the cluster form again
        assert s.precon_apply_traffic()[0] == 2
        z = s.precon_apply(r)
        assert s.precon_apply_traffic()[0] == 0
        s.precon_lowrank(L)
        assert s.precon_apply_traffic()[0] == 2
        res = s.pcg(b, tol=1e-8, maxiter=2000)
        assert s.precon_apply_traffic()[0] == 0
        monkeypatch.delenv("MLFF_LC_TEST_MUTE")
    zref = (r - T.T @ (T @ r)) / lam
    sgn = np.sign(np.dot(z, zref))
    assert np.linalg.norm(z - sgn * zref) <= 1e-12 * np.linalg.norm(zref)
    assert ref.info == 0 and res.info == 0
    assert_pcg_parity(res.iters, res.trace[1:], res.x, ref.iters, ref.trace[1:], ref.x,
                      mode="chaotic", x_tol=1e-6)


def test_cluster_apply_fault_mid_chunk(sg, monkeypatch):
    """The cluster member goes silent only from the 6th apply on (MLFF_LC_TEST_MUTE=3@6), i.e.
    inside a chunk of PCG iterations whose stop tests are folded into the next iteration's
    first kernel: iterations 1-5 are the fault-free cluster solve's (residuals bit for bit),
    iteration 6 faults after its folded prologue already wrote iters / trace / rho1, the host
    re-runs it with two passes, and the rest of the solve equals a solve that ran the two-pass
    apply from iteration 6 on (same trace and x within the two-pass/one-pass rounding band)."""
    n, k, lam = 40000, 301, 1.0
    X, b = _rbf(n)
    L = np.random.default_rng(5).standard_normal((k, n)) * 0.05
    with sg.KernelSolver(n) as s:
        s.gen_rbf(X, length_scale=0.2)
        s.set_operator(1.0, lam)
        s.precon_lowrank(L)
        ref = s.pcg(b, tol=1e-8, maxiter=2000, chunk=16)  # cluster form throughout
        monkeypatch.setenv("MLFF_LC_TEST_MUTE", "3@6")
        s.precon_lowrank(L)
        assert s.precon_apply_traffic()[0] == 2
        res = s.pcg(b, tol=1e-8, maxiter=2000, chunk=16)
        assert s.precon_apply_traffic()[0] == 0  # fell back and stayed on two passes
        monkeypatch.delenv("MLFF_LC_TEST_MUTE")
        # the same switch made by hand: 5 cluster iterations, then two passes
        monkeypatch.setenv("MLFF_LR_ROWS", "0")
        s.precon_lowrank(L)
        assert s.precon_apply_traffic()[0] == 0
        two = s.pcg(b, tol=1e-8, maxiter=2000, chunk=16)
        monkeypatch.delenv("MLFF_LR_ROWS")
    assert ref.info == 0 and res.info == 0 and two.info == 0
    np.testing.assert_array_equal(res.trace[:6], ref.trace[:6])
    assert np.all(np.isfinite(res.trace)) and res.trace.size == res.iters + 1
    assert_pcg_parity(res.iters, res.trace[1:], res.x, ref.iters, ref.trace[1:], ref.x,
                      mode="chaotic", x_tol=1e-6)
    assert_pcg_parity(res.iters, res.trace[1:], res.x, two.iters, two.trace[1:], two.x,
                      mode="chaotic", x_tol=1e-6)


@pytest.mark.parametrize("steps", ["1", "2", "3"])
def test_woodbury_refine_steps(sg, monkeypatch, steps):
    """MLFF_WB_REFINE=<steps> (CholeskyQR2 and beyond): every refined panel T
    represents the same preconditioner as the exact formula -- T^T T = L (lam I + L^T L)^-1 L^T,
    evaluated on the host as Q1 Q1^T from a Householder QR of [L; sqrt(lam) I]
    (iterative_cholesky.py:141-148) -- to rounding, and steps >= 2 (the accumulated-inverse
    branch, Li <- C^-1 Li) agrees with the one-refinement panel to rounding."""
    n, k, lam = 1500, 96, 1e-6
    rng = np.random.default_rng(7)
    L = rng.standard_normal((n, k)) * np.logspace(0, -3, k)   # cond([L; sqrt(lam) I]) ~ 1e3
    A = np.vstack([L, np.sqrt(lam) * np.eye(k)])
    Q1 = np.linalg.qr(A, mode="reduced")[0][:n]
    P_ref = Q1 @ Q1.T
    panels = {}
    for st in ("1", steps):
        monkeypatch.setenv("MLFF_WB_REFINE", st)
        with sg.KernelSolver(n) as s:
            X, _ = _rbf(n)
            s.gen_rbf(X, 0.2)
            s.set_operator(1.0, lam)
            s.precon_lowrank(np.ascontiguousarray(L.T))
            panels[st] = s.precon_panel()
    for st, T in panels.items():
        err = np.abs(T.T @ T - P_ref).max()
        assert err <= 1e-12, (st, err)
        # the orthogonality the refinement restores: T T^T + lam L2^-1 L2^-T = I implies
        # T T^T <= I with the rest lam-sized
        assert np.linalg.eigvalsh(T @ T.T).max() <= 1.0 + 1e-12, st
    d = np.abs(panels[steps].T @ panels[steps] - panels["1"].T @ panels["1"]).max()
    assert d <= 1e-12, d


@pytest.mark.parametrize("k", [1, 13, 64, 200, 2701])
def test_potrf_wave_diag_bitwise(sg, monkeypatch, k):
    """The Woodbury build's Cholesky with the one-wave diagonal-block kernel (k_potrf_diag_wave,
    default) against the workgroup form (MLFF_POTRF_DIAG=0): the same operations in the same
    order, so the panel is bit-identical (and equals the LAPACK-pinned formula to rounding)."""
    n = max(3 * k, 600)
    rng = np.random.default_rng(k)
    L = rng.standard_normal((n, k)) * np.logspace(0, -2, k)
    X, _ = _rbf(n)
    panels = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("MLFF_POTRF_DIAG", mode)
        with sg.KernelSolver(n) as s:
            s.gen_rbf(X, 0.2)
            s.set_operator(1.0, 1e-6)
            s.precon_lowrank(np.ascontiguousarray(L.T))
            panels[mode] = s.precon_panel()
    np.testing.assert_array_equal(panels["1"], panels["0"])
    import scipy.linalg

    L2 = scipy.linalg.cholesky(1e-6 * np.eye(k) + L.T @ L, lower=True)
    T = scipy.linalg.solve_triangular(L2, L.T, lower=True)
    assert np.abs(panels["1"].T @ panels["1"] - T.T @ T).max() <= 1e-9
