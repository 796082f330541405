"""Symmetric tiled operator (csrc/kernels_sym.hip) against NumPy and the dense row GEMV.

The operator is the reference's K_op (src/sGDML/sgdml/solvers/iterative_solver.py:383-445)
evaluated from the lower block triangle of K only.  Tolerances: fp64 with a different
summation order than NumPy -> 1e-13 relative; PCG on a well-conditioned system ->
identical iteration counts and residual curves within 1e-10 relative.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sg():
    import sgdml_amd

    if sgdml_amd.device_count() < 1:
        pytest.fail("no GPU visible to libmlffpcg.so")
    return sgdml_amd


def _sym(n, seed):
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((n, n))
    return (A + A.T) / 2.0, rng.standard_normal(n)


@pytest.mark.parametrize("n", [1, 37, 512, 513, 1300, 2048, 2100])
def test_symtile_matvec(sg, n):
    K, v = _sym(n, n)
    ref = -(K @ v) + 0.5 * v
    out = {}
    with sg.KernelSolver(n) as s:
        s.set_matrix(K)
        s.set_operator(-1.0, 0.5)
        for mode in ("dense", "sym"):
            s.set_storage(mode)
            used, nbytes = s.storage_info()
            assert used == mode
            out[mode] = s.matvec(v)
        nt = -(-(-(-n // 64) * 64) // 512)
        assert nbytes == 8.0 * (nt * (nt + 1) // 2) * 512 * 512 + 16.0 * n
    scale = np.abs(K).sum(axis=1) @ np.abs(v) / n + 1e-300
    for mode, y in out.items():
        assert np.max(np.abs(y - ref)) <= 1e-13 * max(scale, np.abs(ref).max()), mode


def test_symtile_auto_and_asymmetric(sg):
    n = 700
    K, v = _sym(n, 1)
    K[3, 500] += 1e-9  # no longer symmetric
    with sg.KernelSolver(n) as s:
        s.set_matrix(K)
        s.set_operator(1.0, 1.0)
        assert s.storage_info()[0] == "dense"  # auto falls back to the row GEMV
        y = s.matvec(v)
        np.testing.assert_allclose(y, K @ v + v, rtol=1e-12, atol=1e-12)
        s.set_storage("sym")
        with pytest.raises(ValueError):
            s.matvec(v)
        # a symmetric matrix set afterwards is accepted
        s.set_matrix((K + K.T) / 2)
        assert s.storage_info()[0] == "sym"


def test_symtile_generated_kernel_is_auto(sg):
    from sgdml_amd import synthetic

    X, b = synthetic.rbf_points(3000, 3, 0)
    with sg.KernelSolver(3000) as s:
        s.gen_rbf(X, 0.2)
        s.set_operator(1.0, 1e-2)
        mode, _ = s.storage_info()
        assert mode == "sym"
        y_sym = s.matvec(b)
        s.set_storage("dense")
        y_dense = s.matvec(b)
    np.testing.assert_allclose(y_sym, y_dense, rtol=1e-13, atol=1e-13 * np.abs(y_dense).max())


def test_symtile_pcg_matches_dense(sg):
    from sgdml_amd import synthetic

    n, lam = 2500, 0.1
    X, b = synthetic.rbf_points(n, 3, 4)
    res = {}
    for mode in ("dense", "sym"):
        with sg.KernelSolver(n) as s:
            s.gen_rbf(X, 0.2)
            s.set_operator(1.0, lam)
            s.set_storage(mode)
            s.precon_pivchol(200)
            res[mode] = s.pcg(b, tol=1e-10, maxiter=5 * n)
    d, t = res["dense"], res["sym"]
    assert d.info == t.info == 0
    assert d.iters == t.iters
    # stable regime: identical counts, curves equal to ~1e-7 (fp64 summation order)
    np.testing.assert_allclose(t.trace, d.trace, rtol=1e-6, atol=1e-13 * d.trace[0])
    assert np.linalg.norm(t.x - d.x) <= 1e-9 * np.linalg.norm(d.x)


def test_symtile_sgdml_assembly(sg):
    """sGDML kernels are symmetric by construction (mirrored assembly)."""
    from oracle.sgdml import descriptors
    from sgdml_amd import synthetic

    d = synthetic.ethanol_like(40, seed=2)
    Rd, Rdd = descriptors(d["R"])
    n = 27 * 40
    v = np.random.default_rng(0).standard_normal(n)
    with sg.KernelSolver(n) as s:
        s.assemble_sgdml(Rd, Rdd, np.arange(9)[None, :], 10.0)
        s.set_operator(-1.0, 1e-10)
        assert s.storage_info()[0] == "matfree"  # auto: the cheaper matrix-free operator
        s.set_storage("sym")
        assert s.storage_info()[0] == "sym"
        y = s.matvec(v)
        K = s.get_matrix_rows()
    assert np.array_equal(K, K.T)
    ref = -(K @ v) + 1e-10 * v
    assert np.max(np.abs(y - ref)) <= 1e-13 * np.abs(ref).max()


@pytest.mark.parametrize("lsub", ["2", "4"])
@pytest.mark.parametrize("sched", ["dyn", "static"])
@pytest.mark.parametrize("n", [16384, 23040])
def test_symtile_quarter_tail_matches_dense(sg, n, sched, lsub, monkeypatch):
    """Tile counts past one round of 512 workgroups (528 and 1035 tiles: whole tiles plus
    sub-tile units for the remainder -- quarters, or 16 row slices with MLFF_SYM_LSUB=4),
    both launch schedules (counter-driven resident workgroups with cross-tile prefetch; one
    workgroup per unit), against the dense row GEMV."""
    from sgdml_amd import synthetic

    monkeypatch.setenv("MLFF_SYM_SCHED", sched)
    monkeypatch.setenv("MLFF_SYM_LSUB", lsub)

    X, _ = synthetic.rbf_points(n, 3, 11)
    v = np.random.default_rng(n).standard_normal(n)
    with sg.KernelSolver(n) as s:
        s.gen_rbf(X, 0.2)
        s.set_operator(1.0, 1e-3)
        s.set_storage("dense")
        yd = s.matvec(v)
        s.set_storage("sym")
        assert s.storage_info()[0] == "sym"
        ys = s.matvec(v)
        ys2 = s.matvec(v)
    np.testing.assert_array_equal(ys, ys2)  # deterministic
    assert np.max(np.abs(ys - yd)) <= 1e-13 * np.abs(yd).max()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n,k,forms", [(65536, 256, "cluster"), (4000, 300, "rows"),
                                        (20000, 256, "twopass")])
def test_symtile_fused_p_update_bitwise(sg, n, k, forms, monkeypatch):
    """One rank, symmetric tiles + low-rank apply (configs[2]'s iteration): p = z + beta p formed
    by the tile workgroups from the apply's gather block and written by the slot reduction
    (default, round 6) against the separate k_update_p launch (MLFF_FUSE_P=0): the same sums
    in the same order, so iterates, residual curve and stop decisions are bit-identical --
    through the one-pass rows, the cluster and the two-pass applies, with chunk boundaries.
    Ragged sizes (n not a multiple of the 512-row tile: the operand's tile padding lies past the
    gather block, round 6's out-of-bounds read at n = 1) read that padding as zeros."""
    from sgdml_amd import synthetic

    X, b = synthetic.rbf_points(n, 3, 0)
    idx = np.sort(np.random.default_rng(0).choice(n, k, replace=False))
    out = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("MLFF_FUSE_P", fuse)
        if forms == "twopass":
            monkeypatch.setenv("MLFF_LR_ROWS", "0")  # neither one-pass form
        with sg.KernelSolver(n) as s:
            s.gen_rbf(X, 0.2)
            s.set_operator(1.0, 1e-6)
            s.precon_nystrom(idx)
            assert s.storage_info()[0] == "sym"
            if forms is not None:
                form, _ = s.precon_apply_traffic()
                assert form == {"twopass": 0, "rows": 1, "cluster": 2}[forms], form
            # configs[2] itself for the cluster form: 300 iterations of it (info = maxiter)
            out[fuse] = s.pcg(b, tol=1e-6, maxiter=300 if n == 65536 else 5 * n, chunk=7)
    a, c = out["1"], out["0"]
    assert a.info == c.info and a.iters == c.iters
    np.testing.assert_array_equal(a.trace, c.trace)
    np.testing.assert_array_equal(a.x, c.x)
