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
