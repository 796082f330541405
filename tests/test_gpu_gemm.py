"""The library's fp64 GEMM (kernels_dense.hip: k_gemm on the vector ALUs, k_gemm_mfma on the
matrix cores) against numpy for every operand layout, with asymmetric data (a transposed
fragment or a swapped row/column in the MFMA result map fails it), through the
mlff_test_gemm hook.  The builds (Woodbury SYRK / TRSM, Nystrom, CholeskyQR, Rayleigh-Ritz,
spectrum) all run on it."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def solver():
    import sgdml_amd

    if sgdml_amd.device_count() < 1:
        pytest.fail("no GPU visible to libmlffpcg.so")
    with sgdml_amd.KernelSolver(64) as s:
        yield s


def run(solver, ta, tb, M, N, K, alpha, beta, splits=1, seed=0):
    from sgdml_amd import _native as nat

    rng = np.random.default_rng(seed)
    A = rng.standard_normal((K, M) if ta else (M, K)) + np.arange(M if not ta else K)[:, None] * 1e-3
    B = rng.standard_normal((N, K) if tb else (K, N))
    C = rng.standard_normal((M, N))
    opA = A.T if ta else A
    opB = B.T if tb else B
    ref = alpha * (opA @ opB) + beta * C
    if splits > 1:
        ref = C - alpha * (opA @ opB)
    out = np.ascontiguousarray(C.copy())
    A, B = np.ascontiguousarray(A), np.ascontiguousarray(B)
    solver._call("mlff_test_gemm", int(ta), int(tb), M, N, K, float(alpha), nat.dptr(A), A.shape[1],
                 nat.dptr(B), B.shape[1], float(beta), nat.dptr(out), N, int(splits))
    scale = np.abs(opA).max() * np.abs(opB).max() * K * abs(alpha) + abs(beta) * np.abs(C).max()
    assert np.max(np.abs(out - ref)) <= 1e-14 * scale, (ta, tb, M, N, K)


@pytest.mark.parametrize("ta", [0, 1])
@pytest.mark.parametrize("tb", [0, 1])
@pytest.mark.parametrize("shape", [(200, 300, 100), (64, 130, 40), (130, 129, 33),
                                   (257, 385, 77), (40, 50, 20), (128, 128, 16)])
def test_gemm_layouts(solver, ta, tb, shape):
    M, N, K = shape
    run(solver, ta, tb, M, N, K, 1.3, 0.7)


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1)])
def test_gemm_split_k_slabs(solver, ta, tb):
    run(solver, ta, tb, 64, 1000, 700, 1.0, 1.0, splits=4)
    run(solver, ta, tb, 150, 260, 100, 0.5, 1.0, splits=3)


def _two_prod(a, b):
    """Exact a * b = p + e (Dekker / Veltkamp, no fma needed), elementwise."""
    p = a * b
    c = 134217729.0  # 2^27 + 1
    def split(x):
        t = c * x
        hi = t - (t - x)
        return hi, x - hi
    ah, al = split(a)
    bh, bl = split(b)
    e = ((ah * bh - p) + ah * bl + al * bh) + al * bl
    return p, e


@pytest.mark.parametrize("k, ncols", [(70, 3001), (130, 1000), (9, 200)])
def test_woodbury_gram_modes(solver, k, ncols):
    """The Woodbury Gram matrix L^T L (mlff_test_gram): mode 2 (exact products,
    double-double sums) is the correctly rounded exact sum on every entry (within one ulp, exact
    on nearly all); mode 1 (the default: fp64 64-column chunks on the matrix cores, chunk sums in
    double-double) errs by at most a few ulps of its chunks' partial sums -- not of the full-length
    fp64 running sum, which is what the plain fp64 SYRK (mode 0) pays on the small entries; every
    mode is exactly symmetric.  Data with cancellation (mixed signs, a common offset)."""
    import math

    from sgdml_amd import _native as nat

    rng = np.random.default_rng(k)
    W = rng.standard_normal((k, ncols)) * np.exp(rng.uniform(-3, 3, (k, 1))) + 0.3
    W = np.ascontiguousarray(W)
    G = {}
    for mode in (0, 1, 2):
        out = np.zeros((k, k))
        solver._call("mlff_test_gram", nat.dptr(W), k, ncols, mode, nat.dptr(out))
        np.testing.assert_array_equal(out, out.T)
        G[mode] = out
    exact = np.empty((k, k))
    abs_sum = np.abs(W) @ np.abs(W).T
    for i in range(k):
        for j in range(i + 1):
            p, e = _two_prod(W[i], W[j])
            exact[i, j] = exact[j, i] = math.fsum(np.concatenate([p, e]))
    ulp = np.spacing(np.abs(exact))
    eps = np.finfo(float).eps
    err2 = np.abs(G[2] - exact)
    assert np.all(err2 <= ulp), (err2 / ulp).max()
    assert np.count_nonzero(err2) <= max(2, k * k // 200)
    # mode 1: fp64 only inside 64-column chunks (worst case 64 eps sum |products|, against
    # ncols eps sum |products| for one fp64 pass), and far below mode 0 on average
    err1 = np.abs(G[1] - exact)
    err0 = np.abs(G[0] - exact)
    assert np.all(err1 <= 64 * eps * abs_sum + ulp), (err1 / (eps * abs_sum)).max()
    assert err1.mean() <= err0.mean(), (err1.mean(), err0.mean())
    print(f"k={k} n={ncols}: max error / ulp of the entry: fp64 {np.max(err0 / ulp):.1f}, "
          f"chunked double-double {np.max(err1 / ulp):.1f}, exact products {np.max(err2 / ulp):.1f}")
