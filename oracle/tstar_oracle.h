/*
 * tstar_oracle.h -- CPU restatement of the reference's forward model (TEST
 * INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle for the MI355X path.  Only tests/, the smoke()
 * entry point and bench.py's cpu_baseline leg may load it, and only as the
 * checker / the timed CPU baseline -- never as a product code path.
 *
 * Every function restates one piece of /root/reference (Julia) and cites it.
 * Index conventions: cell indices are 0-based here (Julia is 1-based); -1
 * means "no cell closer than the 1e9 sentinel" (v_nearest returns 0.0 then).
 *
 * Pinning (see oracle/README.md):
 *   - chi^2 (MCsub.jl:169-172) and the likelihood expression
 *     (MCsub.jl:179-182) are pinned bit-exactly by the 100 saved models in
 *     /root/reference/model.jld (tests/golden/model_jld_kat.npz).
 *   - Julia's reassociated Base.sum order (VF=8 x IC=4 SIMD accumulators, see
 *     oracle_julia_sum) is pinned by the same file's likelihood value.
 *   - The nearest-cell search and the ray integral (MCsub.jl:142-163,247-263)
 *     have NO reference output to pin against (Julia is not installed and the
 *     487-ray geometry behind model.jld is not shipped): they are pinned only
 *     by an independent numpy restatement (oracle/oracle_np.py) and by
 *     hand-built adversarial cases.  Parity for those rows is "restatement-
 *     pinned", not reference-output-pinned.
 */
#ifndef TSTAR_ORACLE_H
#define TSTAR_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* MCsub.jl:247-263 v_nearest: value of the first cell (lowest index) at the
 * minimum squared distance ((mx-x)^2 + (my-y)^2) + (mz-z)^2 evaluated in FP64
 * without contraction; strict '<' against a running minimum initialised to
 * 1e9.  *idx_out (nullable) receives the 0-based index or -1. */
double oracle_v_nearest(double x, double y, double z, const double *mx, const double *my,
                        const double *mz, const double *mv, int64_t ncells, int64_t *idx_out);

/* MCsub.jl:312-316: index of the first NaN in X (0-based count of leading
 * non-NaN entries), or len if none. */
int64_t oracle_npoints(const double *X, int64_t len);

/* MCsub.jl:306-327 Interpolation with interp_style == 1.  ny/nz == 1 are
 * broadcast (MCsub.jl:317-322).  Writes npoints values to zeta_out (and the
 * chosen cell indices to idx_out if non-NULL).  Returns npoints, or -1 when Y
 * or Z is too short (Julia would throw a BoundsError). */
int64_t oracle_interpolation(const double *xc, const double *yc, const double *zc, const double *zeta,
                             int64_t ncells, const double *X, int64_t nx, const double *Y, int64_t ny,
                             const double *Z, int64_t nz, double *zeta_out, int64_t *idx_out);

/* Julia 1.5 Base.sum(::Vector{Float64}) association (reduce.jl
 * _mapreduce/mapreduce_impl): n<16 sequential; 16<=n<=1024 one @simd block
 * vectorised by LLVM as 4 interleaved 8-wide accumulators (AVX-512 host),
 * first element pair pre-added, tail sequential; n>1024 pairwise split. */
double oracle_julia_sum(const double *a, int64_t n);

/* MCsub.jl:169-172: C = 0; C += ((ptS[k]-tS[k])^2 * 1.0) / allSig[k]^2, k in order. */
double oracle_chi2(const double *ptS, const double *tS, const double *allSig, int64_t n);

/* MCsub.jl:179 (line 180 is a separate, discarded statement):
 * sum(-log.(allSig * sqrt(2pi)) * length(tS)) with Julia's sum order. */
double oracle_likelihood(const double *allSig, int64_t n);

/* load_data_Tonga.jl:66-69: rayL = sqrt((x1-x2)^2 + (y1-y2)^2 + (z1-z2)^2),
 * rayU = 0.5*(U1+U2); inputs m x n column-major, outputs (m-1) x n. */
void oracle_segments(const double *x, const double *y, const double *z, const double *U, int64_t m,
                     int64_t n, double *rayL, double *rayU);

/* MCsub.jl:54-74 interp1: piecewise-linear, half-open x[j] <= xx < x[j+1],
 * NaN outside.  (The reference loop reads x[j+1] past the end only when xx >=
 * x[end]; that case returns NaN here.) */
void oracle_interp1(const double *x, const double *y, int64_t nx, const double *xx, int64_t nxx,
                    double *yy);

/* MCsub.jl:123-185 evaluate (interp_style 1).  Arrays are the DataStruct
 * layout: rayX/Y/Z m x n column-major NaN tail-padded; rayL/rayU (m-1) x n.
 * Outputs ptS[n], *phi, *likelihood, and (nullable) nearest[P] = chosen cell
 * per valid point in ray-major order.  debug_prior==1 returns phi =
 * likelihood = 1 without touching data (MCsub.jl:134-136).  Returns 0, or -1
 * if a ray's rayL NaN prefix disagrees with its rayX NaN prefix (Julia would
 * throw DimensionMismatch). */
int oracle_evaluate(const double *rayX, const double *rayY, const double *rayZ, const double *rayL,
                    const double *rayU, int64_t m, int64_t n, const double *tS, const double *allSig,
                    const double *xc, const double *yc, const double *zc, const double *zeta,
                    int64_t ncells, int debug_prior, double *ptS, double *phi, double *likelihood,
                    int32_t *nearest);

#ifdef __cplusplus
}
#endif
#endif
