"""BASELINE.json configs[0], [1] and [4] through the HIP path (size-true, -m gpu).

configs[0]  ethanol N = 2997, no preconditioner: the drop-in Iterative.solve against the
            reference's own unpreconditioned solve (tests/golden/sgdml_ethanol_n2997.npz,
            none_1e-04__*: 5N = 14985 iterations without reaching tol 1e-4).  Contract for
            unpreconditioned runs: same stopping outcome, the first residuals
            pointwise, the running-minimum envelope within 0.5 decade at every iteration.
configs[1]  nanotube N = 15540 (synthetic 370-atom geometry, M = 14), matrix-free operator:
            the first 64 pivots and L columns of the pivoted Cholesky against the oracle's
            (incomplete_cholesky.py:24-93 with get_col = -K_op e_i, iterative_cholesky.py:
            152-156, on oracle.sgdml.kernel_matvec_matrix_free), then the rule-of-thumb rank
            k = 2701 build and a solve to 1e-6 whose true residual ||b - A x|| is recomputed
            on the host with the oracle operator.
configs[4]  nanotube N = 15540, rank-1024 pivoted Cholesky on 8 ranks (in-process
            transport on one GPU, the same collectives as RCCL on 8 GPUs): pivots identical
            to the oracle's and the one-rank build's, panels within 1e-10, and the 1-rank and
            8-rank PCG solves held to the oracle's band (nanotube_n15540_k1024.npz).
"""
import numpy as np
import pytest

from tests.parity import assert_pcg_parity, noise_band

from tests.test_gpu_golden import load, run_dropin
from tests.test_gpu_multirank import run_ranks

pytestmark = pytest.mark.gpu

N_ATOMS, M_NANO, SIG, LAM = 370, 14, 10.0, 1e-10


@pytest.fixture(scope="module")
def sg():
    import sgdml_amd

    if sgdml_amd.device_count() < 1:
        pytest.fail("no GPU visible to libmlffpcg.so")
    return sgdml_amd


@pytest.fixture(scope="module")
def nanotube(sg):
    """configs[1] geometry (bench.py --workload nanotube): descriptors on the GPU."""
    from sgdml_amd import synthetic

    ds = synthetic.nanotube_like(M_NANO, seed=0)
    Rd, Rdd = sg.sgdml_descriptors(ds["R"])
    y, _ = synthetic.labels(ds["F"])
    return Rd, Rdd, np.arange(N_ATOMS)[None, :], y


@pytest.mark.timeout(600)
def test_config0_ethanol_n2997_unpreconditioned(sg, golden_dir):
    name = "sgdml_ethanol_n2997"
    f = load(golden_dir, name)
    n = f["y"].size
    alphas, num_iters, resid, rmse, idxs, is_conv, info = run_dropin(f, name, "none")
    ref = f["none_1e-04__trace"]
    # the reference stops at maxiter = 5N (iterative_solver.py:1002) without converging
    assert int(f["none_1e-04__info"]) == 5 * n and not is_conv
    assert num_iters == int(f["none_1e-04__callbacks"]) == 5 * n
    tr = info["resid_trace"][1:]
    assert tr.size == ref.size
    assert np.max(np.abs(np.log10(tr[:8] / ref[:8]))) <= 1e-6
    env, env_ref = np.minimum.accumulate(tr), np.minimum.accumulate(ref)
    assert np.max(np.abs(np.log10(env / env_ref))) <= 0.5
    assert idxs.size == 0


def _oracle_pivots(Rd, Rdd, perms, k):
    from oracle.precon import pivoted_cholesky
    from oracle.sgdml import kernel_diag, kernel_matvec_matrix_free

    n = Rd.shape[0] * 3 * N_ATOMS

    def get_col(i):  # (-K_op) e_i = -K e_i + lam e_i (iterative_cholesky.py:152-156)
        e = np.zeros(n)
        e[i] = 1.0
        return -kernel_matvec_matrix_free(Rd, Rdd, perms, SIG, e) + LAM * e

    diag = -kernel_diag(Rd, Rdd, perms, SIG)  # excludes lam (iterative_cholesky.py:373)
    return pivoted_cholesky(get_col, diag, k), diag


@pytest.mark.timeout(900)
def test_config1_nanotube_pivchol_and_solve(sg, nanotube):
    from oracle.sgdml import kernel_matvec_matrix_free

    Rd, Rdd, perms, y = nanotube
    n = y.size
    assert n == 15540
    kk = 64
    (L_ref, piv_ref), diag_ref = _oracle_pivots(Rd, Rdd, perms, kk)
    with sg.KernelSolver(n) as s:
        s.sgdml_operator(Rd, Rdd, perms, SIG)
        s.set_operator(-1.0, LAM)
        assert s.storage_info()[0] == "matfree"
        np.testing.assert_allclose(s.diag(), diag_ref, rtol=1e-12, atol=0)
        piv, _ = s.precon_pivchol(kk, build_woodbury=False)
        Lt = s.precon_panel()
        np.testing.assert_array_equal(piv[:kk], piv_ref[:kk])
        np.testing.assert_allclose(Lt.T, L_ref, rtol=0, atol=1e-10 * np.abs(L_ref).max())
        # the rule-of-thumb rank (plot_data.py:1254-1258: k = 2701 at N = 15540) and the solve
        k = 2701
        piv_full, _ = s.precon_pivchol(k)
        np.testing.assert_array_equal(piv_full[:kk], piv_ref[:kk])
        res = s.pcg(y, tol=1e-6, maxiter=5 * n)
    assert res.info == 0 and 0 < res.iters < 5 * n
    # the recheck guarantees the GPU's own ||b - A x|| <= tol ||b||; the oracle operator
    # (another summation order) must see the same to rounding of ||A|| ||x||
    Ax = -kernel_matvec_matrix_free(Rd, Rdd, perms, SIG, res.x) + LAM * res.x
    relres = np.linalg.norm(y - Ax) / np.linalg.norm(y)
    assert relres <= 1.05e-6, relres
    assert abs(res.resid / np.linalg.norm(y) - relres) <= 1e-2 * relres


@pytest.mark.timeout(1500)
def test_config4_nanotube_pivchol_rank1024_eight_ranks(sg, golden_dir):
    """configs[4]: the configs[1] nanotube with the rank-1024 pivoted Cholesky built on 8 ranks
    (in-process transport on one GPU, the same collectives as RCCL on 8 GPUs) and its PCG solve,
    against the CPU oracle's run of it (tests/golden/make_nanotube_full.py --configs4 ->
    nanotube_n15540_k1024.npz / _band.json: the rank-1024 factor is the first 1024 columns of the
    oracle's rank-2701 one; the reference's one-step Woodbury panel, iterative_cholesky.py:135-150,
    and the scipy-1.7.3 CG to 1e-4 and 1e-6 in three operator and five Gram orders).
    * all 1024 pivots equal the oracle's on 1 rank and on 8; the 8-rank factor and apply equal the
      one-rank ones to rounding;
    * the 1-rank and the 8-rank solves each held to the oracle's band at both tolerances
      (tests/parity.py rule: iterations, half-decade crossings, alpha)."""
    import json

    from oracle.sgdml import descriptors

    path = golden_dir / "nanotube_n15540_k1024.npz"
    if not path.exists():
        pytest.fail("tests/golden/nanotube_n15540_k1024.npz missing (make_nanotube_full.py --configs4)")
    f = np.load(path, allow_pickle=False)
    fx = json.loads((golden_dir / "nanotube_n15540_k1024_band.json").read_text())
    Rd, Rdd = descriptors(f["R"])
    y = f["y"]
    perms = np.arange(N_ATOMS)[None, :]
    n, k = y.size, int(fx["k"])
    assert (n, k) == (15540, 1024)

    def body(rank, world, key):
        with sg.KernelSolver(n, device=0, rank=rank, world=world,
                             comm_id=key if world > 1 else None) as s:
            s.sgdml_operator(Rd, Rdd, perms, SIG)
            s.set_operator(-1.0, LAM)
            piv, _ = s.precon_pivchol(k, build_woodbury=False)
            Lt = s.precon_panel()
            s.precon_pivchol(k)  # + Woodbury: the configs[4] preconditioner
            r0, r1 = s.row_range()
            b = np.ascontiguousarray(y[r0:r1])
            z = s.precon_apply(b)
            res = {tol: s.pcg(b, tol=tol, maxiter=5 * n) for tol in (1e-4, 1e-6)}
            return piv, Lt, z, res

    ref = run_ranks(1, body, timeout=900)[0]
    outs = run_ranks(8, body, timeout=1200)
    np.testing.assert_array_equal(ref[0][:k], f["index_columns"][:k])
    for piv, _, _, _ in outs:
        np.testing.assert_array_equal(piv[:k], ref[0][:k])
    Lt = np.concatenate([o[1] for o in outs], axis=1)
    np.testing.assert_allclose(Lt, ref[1], rtol=0, atol=1e-10 * np.abs(ref[1]).max())
    z = np.concatenate([o[2] for o in outs])
    err = np.abs(z - ref[2]).max() / np.abs(ref[2]).max()
    print(f"configs[4] Woodbury apply: max |dz| / max |z| = {err:.3e}")
    assert err <= 1e-11
    for tol in (1e-4, 1e-6):
        key = f"tol{tol:g}"
        b = fx["bands"][key]
        r1 = ref[3][tol]
        x8 = np.concatenate([o[3][tol].x for o in outs])
        r8 = outs[0][3][tol]
        print(f"configs[4] tol={tol:g}: GPU 1 rank {r1.iters}, 8 ranks {r8.iters} vs oracle "
              f"{int(f[key + '_iters'])} (band {b['band_iters']}, orders "
              f"{ {o: v['iters'] for o, v in b['variants'].items()} })")
        assert r1.info == r8.info == int(f[key + "_info"]) == 0
        for it, tr, x in ((r1.iters, r1.trace, r1.x), (r8.iters, r8.trace, x8)):
            assert_pcg_parity(it, tr[1:], -x, int(f[key + "_iters"]), f[key + "_trace"][1:],
                              f[key + "_alphas"], band=b)


@pytest.mark.timeout(900)
def test_nanotube_cluster_apply_solve(sg, monkeypatch):
    """The configs[1] geometry with one more training point (M = 15, N = 16650): its panel
    rows exceed one workgroup's registers, so the drop-in's default low-rank apply is the
    cluster one-pass form (k_lr_cluster, C = 3).  The rank-2850 pivoted-Cholesky PCG solve with
    it converges to 1e-6 with the true residual recomputed by the oracle operator, and takes
    the iteration count of the two-pass apply to within the chaotic-regime slack (the two
    applies sum in different orders).  Reference: iterative_cholesky.py:115-150."""
    from oracle.sgdml import kernel_matvec_matrix_free
    from sgdml_amd import synthetic

    ds = synthetic.nanotube_like(15, seed=0)
    Rd, Rdd = sg.sgdml_descriptors(ds["R"])
    y, _ = synthetic.labels(ds["F"])
    perms = np.arange(N_ATOMS)[None, :]
    n, k = y.size, 2850
    assert n == 16650
    out = {}
    for mode in ("0", "default"):
        if mode == "0":
            monkeypatch.setenv("MLFF_LR_ROWS", "0")
        else:
            monkeypatch.delenv("MLFF_LR_ROWS", raising=False)
        with sg.KernelSolver(n) as s:
            s.sgdml_operator(Rd, Rdd, perms, SIG)
            s.set_operator(-1.0, LAM)
            s.precon_pivchol(k)
            form, _ = s.precon_apply_traffic()
            assert form == (0 if mode == "0" else 2)
            out[mode] = s.pcg(y, tol=1e-6, maxiter=5 * n)
    r0, r1 = out["0"], out["default"]
    assert r0.info == 0 and r1.info == 0
    # two summation orders of the same solve: the measured band of the reference's nanotube
    # cholesky solve (noise_band.json, N = 3330: b_it = 1 of 322 iterations), scaled by the
    # iteration count, under the tests/parity.py rule
    b = noise_band("sgdml_nanotube_n3330/cholesky")
    scale = r0.iters / b["ref_iters"]
    band = {"band_iters": int(np.ceil(b["band_iters"] * scale)),
            "band_crossing": int(np.ceil(b["band_crossing"] * scale)),
            "band_rel_dalpha": b["band_rel_dalpha"]}
    print(f"cluster vs two-pass apply: {r1.iters} vs {r0.iters} iterations (band {band})")
    assert_pcg_parity(r1.iters, r1.trace[1:], r1.x, r0.iters, r0.trace[1:], r0.x, band=band)
    Ax = -kernel_matvec_matrix_free(Rd, Rdd, perms, SIG, r1.x) + LAM * r1.x
    relres = np.linalg.norm(y - Ax) / np.linalg.norm(y)
    assert relres <= 1.05e-6, relres


@pytest.mark.timeout(900)
def test_config1_full_size_against_oracle_fixture(sg, golden_dir):
    """configs[1] at its full size against the CPU oracle's own run of it
    (tests/golden/make_nanotube_full.py -> nanotube_n15540.npz / _band.json): the rank-2701
    pivoted Cholesky on the matrix-free operator (incomplete_cholesky.py:24-93 with get_col =
    -K_op e_i, iterative_cholesky.py:152-156) and the PCG solve to 1e-6 (iterative_solver.py:
    995-1009).  Both sides start from the same descriptors (oracle.sgdml.descriptors of the
    fixture's geometry).
    * pivots: identical up to the first near-tie of the oracle's residual diagonal (SURVEY 8(c):
      relative gap between the best two candidates < 1e-12); every pivot when there is none;
    * solve: iterations, residual trace and alpha under the tests/parity.py band rule with the
      band the oracle measured on this system (three summation orders of its operator, two of
      its Woodbury panel's Gram matrix: 366-369 iterations).  The fixture also records panels
      rounded differently (explicit inverse, 2e-15 perturbations: 564-578 iterations,
      "panel_perturbations"); the device's one-step panel fell there (571), its re-orthogonalised
      panel (the default) is held to the band."""
    import json

    from oracle.sgdml import descriptors
    from tests.parity import assert_pcg_parity

    path = golden_dir / "nanotube_n15540.npz"
    if not path.exists():
        pytest.fail("tests/golden/nanotube_n15540.npz missing (make_nanotube_full.py)")
    f = np.load(path, allow_pickle=False)
    band = json.loads((golden_dir / "nanotube_n15540_band.json").read_text())
    Rd, Rdd = descriptors(f["R"])
    y = f["y"]
    n, k = y.size, int(band["k"])
    with sg.KernelSolver(n) as s:
        s.sgdml_operator(Rd, Rdd, np.arange(N_ATOMS)[None, :], SIG)
        s.set_operator(-1.0, LAM)
        piv, _ = s.precon_pivchol(k)
        res = s.pcg(y, tol=1e-6, maxiter=5 * n)
    ref_piv, gap = f["index_columns"], f["pivot_gap"]
    diff = np.nonzero(piv[:k] != ref_piv[:k])[0]
    first_tie = np.nonzero(gap < 1e-12)[0]
    limit = int(first_tie[0]) if first_tie.size else k
    print(f"configs[1] pivots: first difference at {diff[0] if diff.size else None}, "
          f"first oracle near-tie at {limit if first_tie.size else None} of {k}")
    assert diff.size == 0 or diff[0] >= limit, (diff[:5], limit)
    assert res.info == 0 and int(f["info"]) == 0
    print(f"configs[1] solve: GPU {res.iters} vs oracle {int(f['iters'])} iterations "
          f"(band {band['band_iters']}, oracle orders "
          f"{ {o: v['iters'] for o, v in band['variants'].items()} })")
    assert_pcg_parity(res.iters, res.trace[1:], -res.x, int(f["iters"]), f["trace"][1:],
                      f["alphas"], band=band)
    if "accurate" in band:  # and the oracle's accurately evaluated panels (round 5: 363-366)
        acc = band["accurate"]
        print(f"configs[1] solve: GPU {res.iters} vs oracle accurate {acc['ref_iters']} "
              f"(band {acc['band_iters']}, {({o: v['iters'] for o, v in acc['variants'].items()})})")
        assert_pcg_parity(res.iters, res.trace[1:], -res.x, int(f["accurate_iters"]),
                          f["accurate_trace"][1:], f["accurate_alphas"], band=acc)



@pytest.mark.timeout(900)
@pytest.mark.parametrize("panel", ["onestep", "refined"])
@pytest.mark.parametrize("k", [1264, 554])
def test_ethanol_full_size_against_oracle_fixture(sg, golden_dir, monkeypatch, k, panel):
    """Ethanol at the reference's published size (N = 15741, M = 583; BASELINE.md:22) on
    energy-consistent labels, against the CPU oracle's run of it (tests/golden/
    make_ethanol_full.py -> ethanol_n15741.npz / _band.json): the pivoted Cholesky on the
    matrix-free operator to the rule-of-thumb k = 1264 and the published k = 554
    (incomplete_cholesky.py:24-93, iterative_cholesky.py:152-156), then the PCG to the reference's
    training tolerance 1e-4 (train.py:309) and to 1e-6 (iterative_solver.py:995-1009).  Pivots
    identical up to the oracle's first near-tie.  The Woodbury panel T = chol(lam I + L^T L)^-1 L^T
    (iterative_cholesky.py:141-143) at cond([L; sqrt(lam) I]) ~ 6e3:
    * 'onestep' (the default since round 6: the reference's formula, one CholeskyQR step, the
      Gram matrix summed in blocked double-double) is held to the band of the reference's one-step
      algorithm at both tolerances, alpha included.  The band samples what moves its count at
      this conditioning: three operator orders, six Gram orders (BLAS, reversed, 8
      slabs, 64-row chunks added exactly, pairwise, extended precision), the device's apply order,
      and the factorisation / triangular solve in substitution order (1202 vs LAPACK's 1351 at
      k = 1264, 1e-6);
    * 'refined' (MLFF_WB_REFINE=1, a second CholeskyQR step) is held to the band of the oracle's
      ACCURATE evaluations of the same formula (Householder-QR and two-step panels) at both
      tolerances, and to the one-step band at 1e-4, where every evaluation agrees.
    tests/parity.py rule for every compared solve."""
    import json

    from oracle.sgdml import descriptors

    path = golden_dir / "ethanol_n15741.npz"
    if not path.exists():
        pytest.fail("tests/golden/ethanol_n15741.npz missing (make_ethanol_full.py)")
    f = np.load(path, allow_pickle=False)
    fx = json.loads((golden_dir / "ethanol_n15741_band.json").read_text())
    Rd, Rdd = descriptors(f["R"])
    y = f["y"]
    n = y.size
    monkeypatch.setenv("MLFF_WB_REFINE", "1" if panel == "refined" else "0")
    res = {}
    with sg.KernelSolver(n) as s:
        s.sgdml_operator(Rd, Rdd, np.arange(9)[None, :], SIG)
        s.set_operator(-1.0, LAM)
        piv, _ = s.precon_pivchol(k)
        for tol in (1e-4, 1e-6):
            res[tol] = s.pcg(y, tol=tol, maxiter=12000)
    ref_piv, gap = f["index_columns"][:k], f["pivot_gap"][:k]
    diff = np.nonzero(piv[:k] != ref_piv)[0]
    first_tie = np.nonzero(gap < 1e-12)[0]
    limit = int(first_tie[0]) if first_tie.size else k
    print(f"ethanol k={k} pivots: first difference at {diff[0] if diff.size else None}, "
          f"first oracle near-tie at {limit if first_tie.size else None}")
    assert diff.size == 0 or diff[0] >= limit, (diff[:5], limit)
    for tol, r in res.items():
        key = f"k{k}_tol{tol:g}"
        if panel == "onestep":
            checks = {"one-step": (fx["bands"][key], "")}
        else:
            checks = {"accurate": (fx["bands"][key]["accurate"], "_accurate")}
            if tol == 1e-4:
                checks["one-step"] = (fx["bands"][key], "")
        for name, (b, sfx) in checks.items():
            print(f"ethanol k={k} tol={tol:g} {panel}: GPU {r.iters} vs oracle {name} "
                  f"{int(f[key + sfx + '_iters'])} iterations (band {b['band_iters']}, orders "
                  f"{ {o: v['iters'] for o, v in b['variants'].items()} })")
            assert r.info == int(f[key + sfx + "_info"]) == 0
            assert_pcg_parity(r.iters, r.trace[1:], -r.x, int(f[key + sfx + "_iters"]),
                              f[key + sfx + "_trace"][1:], f[key + sfx + "_alphas"], band=b)


@pytest.mark.timeout(900)
def test_ethanol_n74979_against_oracle_fixture(sg, golden_dir):
    """Ethanol at the reference's N = 75k point (BASELINE.md:24, data/rule_of_thumb.csv:9:
    M = 2777, N = 74979, rule-of-thumb k = 3752) against the CPU oracle's run of it (tests/golden/
    make_ethanol_75k.py -> ethanol_n74979.npz / _band.json): the pivoted
    Cholesky on the matrix-free operator (incomplete_cholesky.py:24-93 with get_col = -K_op e_i,
    iterative_cholesky.py:152-156; the oracle's columns from the one training point each touches),
    the reference's one-step Woodbury panel (iterative_cholesky.py:141-143) and the scipy-1.7.3
    PCG to 1e-6 (iterative_solver.py:995-1009).  Pivots identical up to the oracle's first
    near-tie; the solve held to the band of the oracle's three operator orders and two Gram /
    factorisation orders (tests/parity.py rule) at 1e-6, alpha included, and at the reference's
    training tolerance 1e-4 (each trace's first crossing, as the band was measured)."""
    import json

    from oracle.sgdml import descriptors

    path = golden_dir / "ethanol_n74979.npz"
    if not path.exists():
        pytest.fail("tests/golden/ethanol_n74979.npz missing (make_ethanol_75k.py)")
    f = np.load(path, allow_pickle=False)
    fx = json.loads((golden_dir / "ethanol_n74979_band.json").read_text())
    Rd, Rdd = descriptors(f["R"])
    y = f["y"]
    n, k = y.size, int(fx["k"])
    with sg.KernelSolver(n) as s:
        s.sgdml_operator(Rd, Rdd, np.arange(9)[None, :], SIG)
        s.set_operator(-1.0, LAM)
        piv, _ = s.precon_pivchol(k)
        res = s.pcg(y, tol=1e-6, maxiter=12000)
    ref_piv, gap = f["index_columns"][:k], f["pivot_gap"][:k]
    diff = np.nonzero(piv[:k] != ref_piv)[0]
    first_tie = np.nonzero(gap < 1e-12)[0]
    limit = int(first_tie[0]) if first_tie.size else k
    print(f"ethanol N={n} k={k} pivots: first difference at {diff[0] if diff.size else None}, "
          f"first oracle near-tie at {limit if first_tie.size else None}")
    assert diff.size == 0 or diff[0] >= limit, (diff[:5], limit)
    assert res.info == int(f["info"]) == 0
    tr, ref_tr = np.asarray(res.trace), np.asarray(f["trace"])
    for tol in (1e-4, 1e-6):
        b = fx["bands"][f"k{k}_tol{tol:g}"]
        it = int(np.argmax(tr[1:] <= tol * tr[0])) + 1
        print(f"ethanol N={n} k={k} tol={tol:g}: GPU {it} vs oracle {b['ref_iters']} iterations "
              f"(band {b['band_iters']}, orders { {o: v['iters'] for o, v in b['variants'].items()} })")
        if tol == 1e-6:
            assert it == res.iters
            assert_pcg_parity(res.iters, tr[1:], -res.x, int(f["iters"]), ref_tr[1:], f["alphas"],
                              band=b)
        else:
            assert_pcg_parity(it, tr[1:it + 1], None, b["ref_iters"], ref_tr[1:b["ref_iters"] + 1],
                              None, band=b)
