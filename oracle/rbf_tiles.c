/* ORACLE — CPU restatement, TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
 *
 * The synthetic SPD RBF kernel of the reference (src/tools/utils.py:173-187: sklearn
 * RBF(length_scale) = exp(-0.5 * sqeuclidean(x_i / l, x_j / l)), diagonal 1) held as its
 * lower block triangle in 512 x 512 tiles, and the mat-vec y = K v over those tiles, for
 * CPU solves at sizes where a dense N x N NumPy array does not fit this container
 * (N = 65536: 17.3 GB of tiles instead of 34.4 GB).  Used by
 * tests/golden/make_rbf_band.py to record the oracle's solve of the configs[2] system
 * (iterations to relres 1e-6), never by the product.
 *
 *   gcc -O3 -fopenmp -shared -fPIC oracle/rbf_tiles.c -o oracle/_build/librbftiles.so -lm
 *
 * Tile (I, J), J <= I, lives at offset (I (I + 1) / 2 + J) * 512 * 512, row-major inside the
 * tile; rows / columns past N are zero.  The mat-vec is deterministic for a fixed thread
 * count: every thread sums its static share of tiles into a private vector, and the private
 * vectors are added in thread order.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define TB 512

static inline int64_t ntiles_of(int64_t n) {
  const int64_t nb = (n + TB - 1) / TB;
  return nb * (nb + 1) / 2;
}

int64_t rbf_tiles_count(int64_t n) { return ntiles_of(n); }

/* Xs: N x d points already divided by the length scale (as sklearn does). */
void rbf_tiles_gen(const double *Xs, int64_t n, int d, double *tiles) {
  const int64_t nb = (n + TB - 1) / TB;
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t I = 0; I < nb; ++I) {
    for (int64_t J = 0; J <= I; ++J) {
      double *t = tiles + (I * (I + 1) / 2 + J) * (int64_t)TB * TB;
      for (int64_t r = 0; r < TB; ++r) {
        const int64_t i = I * TB + r;
        for (int64_t c = 0; c < TB; ++c) {
          const int64_t j = J * TB + c;
          double v = 0.0;
          if (i < n && j < n) {
            if (i == j) {
              v = 1.0;
            } else {
              double s = 0.0;
              for (int k = 0; k < d; ++k) {
                const double e = Xs[i * d + k] - Xs[j * d + k];
                s += e * e;
              }
              v = exp(-0.5 * s);
            }
          }
          t[r * TB + c] = v;
        }
      }
    }
  }
}

/* K columns idx (k of them) as an N x k row-major panel, from the same tiles */
void rbf_tiles_cols(const double *tiles, int64_t n, const int64_t *idx, int64_t k, double *out) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    for (int64_t c = 0; c < k; ++c) {
      int64_t a = i, b = idx[c];
      if (b > a) {  // upper triangle: the symmetric entry
        const int64_t t = a;
        a = b;
        b = t;
      }
      const int64_t I = a / TB, J = b / TB;
      out[i * k + c] = tiles[(I * (I + 1) / 2 + J) * (int64_t)TB * TB + (a % TB) * TB + b % TB];
    }
  }
}

static void symv_impl(const double *tiles, int64_t n, const double *v, double *y, int reverse);

/* y = K v (N entries) */
void rbf_tiles_symv(const double *tiles, int64_t n, const double *v, double *y) {
  symv_impl(tiles, n, v, y, 0);
}

/* the same mat-vec in another summation order: tiles visited last to first (every thread's
 * private vector accumulates its share in reverse), rows of a tile last to first, and the
 * private vectors added in reverse thread order (a second oracle sample of the N = 65536 solve) */
void rbf_tiles_symv_rev(const double *tiles, int64_t n, const double *v, double *y) {
  symv_impl(tiles, n, v, y, 1);
}

static void symv_impl(const double *tiles, int64_t n, const double *v, double *y, int reverse) {
  const int64_t nb = (n + TB - 1) / TB;
  const int64_t np = nb * TB;
  const int64_t nt = ntiles_of(n);
  const int nth = omp_get_max_threads();
  double *acc = (double *)calloc((size_t)nth * np, sizeof(double));
  double *vp = (double *)calloc((size_t)np, sizeof(double));
  memcpy(vp, v, sizeof(double) * n);
#pragma omp parallel
  {
    const int th = omp_get_thread_num();
    double *ya = acc + (int64_t)th * np;
#pragma omp for schedule(static)
    for (int64_t tt = 0; tt < nt; ++tt) {
      const int64_t t = reverse ? nt - 1 - tt : tt;
      /* tile index -> (I, J) */
      int64_t I = (int64_t)((sqrt(8.0 * (double)t + 1.0) - 1.0) / 2.0);
      while (I * (I + 1) / 2 > t) --I;
      while ((I + 1) * (I + 2) / 2 <= t) ++I;
      const int64_t J = t - I * (I + 1) / 2;
      const double *A = tiles + t * (int64_t)TB * TB;
      const double *vj = vp + J * TB, *vi = vp + I * TB;
      double *yi = ya + I * TB, *yj = ya + J * TB;
      for (int64_t rr = 0; rr < TB; ++rr) {
        const int64_t r = reverse ? TB - 1 - rr : rr;
        const double *row = A + r * TB;
        double s = 0.0;
        for (int64_t c = 0; c < TB; ++c) s += row[c] * vj[c];
        yi[r] += s;
        if (I != J) {
          const double w = vi[r];
          for (int64_t c = 0; c < TB; ++c) yj[c] += row[c] * w;
        }
      }
    }
  }
  for (int64_t i = 0; i < n; ++i) {
    double s = 0.0;
    for (int k = 0; k < nth; ++k) s += acc[(int64_t)(reverse ? nth - 1 - k : k) * np + i];
    y[i] = s;
  }
  free(acc);
  free(vp);
}
