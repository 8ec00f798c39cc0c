/* san_oracle.c -- drives every entry point of the CPU oracle (tstar_oracle.c)
 * over the edge cases the parity tests use, under AddressSanitizer and
 * UndefinedBehaviorSanitizer (host ASan/UBSan on the CPU oracle).
 * TEST INFRASTRUCTURE ONLY; built by `make -C oracle sanitize`, run by
 * tests/test_sanitizers.py.  Exit 0 = every call completed with no report. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../tstar_oracle.h"

static uint64_t rs = 88172645463325252ull;
static double urand(void) {  /* xorshift64 */
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return (double)(rs >> 11) * (1.0 / 9007199254740992.0);
}

/* n rays of the given point counts in an m x n column-major NaN-padded layout */
static void rays(const int64_t *np, int64_t n, int64_t m, double **X, double **Y, double **Z, double **L,
                 double **U) {
    *X = malloc(sizeof(double) * (size_t)(m * n + 1));
    *Y = malloc(sizeof(double) * (size_t)(m * n + 1));
    *Z = malloc(sizeof(double) * (size_t)(m * n + 1));
    double *S = malloc(sizeof(double) * (size_t)(m * n + 1));
    *L = malloc(sizeof(double) * (size_t)((m - 1) * n + 1));
    *U = malloc(sizeof(double) * (size_t)((m - 1) * n + 1));
    for (int64_t r = 0; r < n; ++r)
        for (int64_t k = 0; k < m; ++k) {
            const int64_t i = r * m + k;
            const int in = k < np[r];
            (*X)[i] = in ? 1000.0 * urand() : NAN;
            (*Y)[i] = in ? 600.0 * urand() - 200.0 : NAN;
            (*Z)[i] = in ? 650.0 * urand() : NAN;
            S[i] = in ? 0.1 + 0.05 * urand() : NAN;
        }
    oracle_segments(*X, *Y, *Z, S, m, n, *L, *U);
    free(S);
}

int main(void) {
    const int64_t np[] = {0, 1, 2, 3, 15, 16, 17, 33, 131, 1025, 2100, 7};
    const int64_t n = (int64_t)(sizeof np / sizeof np[0]);
    int64_t m = 0;
    for (int64_t r = 0; r < n; ++r) m = np[r] > m ? np[r] : m;
    double *X, *Y, *Z, *L, *U;
    rays(np, n, m, &X, &Y, &Z, &L, &U);
    double tS[64], sig[64], ptS[64];
    for (int64_t r = 0; r < n; ++r) {
        tS[r] = urand();
        sig[r] = 0.04 + 0.5 * urand();
    }
    int64_t P = 0;
    for (int64_t r = 0; r < n; ++r) P += np[r];
    int32_t *near = malloc(sizeof(int32_t) * (size_t)(P + 1));
    const int64_t ncs[] = {0, 1, 5, 300};
    for (int c = 0; c < 4; ++c) {
        const int64_t N = ncs[c];
        double *xc = malloc(sizeof(double) * (size_t)(N + 1)), *yc = malloc(sizeof(double) * (size_t)(N + 1));
        double *zc = malloc(sizeof(double) * (size_t)(N + 1)), *ze = malloc(sizeof(double) * (size_t)(N + 1));
        for (int64_t j = 0; j < N; ++j) {
            xc[j] = 1000.0 * urand();
            yc[j] = 600.0 * urand() - 200.0;
            zc[j] = 650.0 * urand();
            ze[j] = 50.0 * urand();
        }
        if (N > 3) {  /* an exact duplicate and a cell beyond the 1e9 sentinel */
            xc[1] = xc[0];
            yc[1] = yc[0];
            zc[1] = zc[0];
            xc[2] = 1e6;
        }
        double phi = 0, lk = 0;
        if (oracle_evaluate(X, Y, Z, L, U, m, n, tS, sig, xc, yc, zc, ze, N, 0, ptS, &phi, &lk, near) != 0) return 2;
        if (oracle_evaluate(X, Y, Z, L, U, m, n, tS, sig, xc, yc, zc, ze, N, 1, ptS, &phi, &lk, NULL) != 0) return 3;
        /* Interpolation: full columns, broadcast Y/Z, a short Y (BoundsError) */
        double out[2200];
        int64_t idx[2200];
        for (int64_t r = 0; r < n; ++r) {
            const double *cx = X + r * m, *cy = Y + r * m, *cz = Z + r * m;
            (void)oracle_interpolation(xc, yc, zc, ze, N, cx, m, cy, m, cz, m, out, idx);
            (void)oracle_interpolation(xc, yc, zc, ze, N, cx, m, cy, 1, cz, 1, out, NULL);
        }
        if (oracle_interpolation(xc, yc, zc, ze, N, X + 10 * m, m, Y, 1, Z, 2, out, idx) != -1 && np[10] > 2)
            return 4;
        int64_t k;
        (void)oracle_v_nearest(1.0, 2.0, 3.0, xc, yc, zc, ze, N, &k);
        free(xc);
        free(yc);
        free(zc);
        free(ze);
    }
    /* Julia sum association at every length around the block boundaries */
    double *a = malloc(sizeof(double) * 5000);
    for (int i = 0; i < 5000; ++i) a[i] = urand() - 0.5;
    const int64_t lens[] = {0, 1, 15, 16, 17, 31, 32, 33, 1023, 1024, 1025, 2047, 2048, 2049, 4999};
    for (int i = 0; i < (int)(sizeof lens / sizeof lens[0]); ++i) (void)oracle_julia_sum(a, lens[i]);
    (void)oracle_chi2(ptS, tS, sig, n);
    (void)oracle_likelihood(sig, n);
    /* interp1 at the knots, between them, outside, at a repeated depth */
    const double kx[] = {0.0, 10.0, 10.0, 35.0, 210.0}, ky[] = {5.8, 5.8, 6.5, 6.5, 8.3};
    const double q[] = {-1.0, 0.0, 5.0, 10.0, 20.0, 35.0, 209.9, 210.0, 1e9, NAN};
    double qy[10];
    oracle_interp1(kx, ky, 5, q, 10, qy);
    oracle_interp1(kx, ky, 1, q, 10, qy);
    free(a);
    free(near);
    free(X);
    free(Y);
    free(Z);
    free(L);
    free(U);
    puts("san_oracle: ok");
    return 0;
}
