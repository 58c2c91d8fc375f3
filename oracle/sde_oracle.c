/*
 * sde_oracle.c -- CPU restatement of the WHDY/SceneDepthEstimation matching path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The
 * product path (scenedepthestimation_amd/) never links or calls it.
 *
 * Parity status
 *   - cost volume / WTA / WTA1: PINNED against golden vectors produced by the
 *     reference's own NumPy functions (tests/golden/make_golden.py executes
 *     process_functional.py:48-113 extracted with `ast`).
 *   - SGM penalties / 8-path SGM / LR check / LRC fill / median / tower:
 *     PARITY UNPINNED -- the reference implements them as Numba CUDA kernels
 *     and a TF1 graph, neither runnable here.  They are restated line-by-line
 *     from the reference source (citations below) and cross-checked against an
 *     independent literal Python restatement in tests/ (small sizes).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off: no FMA contraction, the
 * reference's NumPy products and sums are separately rounded).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))

/* OpenMP over independent lines / rows / pixels (bit-identical to a serial run: no loop
 * below reorders any per-element arithmetic).  Thread count: sdeo_set_threads (default 1). */
static int g_threads = 1;
EXPORT void sdeo_set_threads(int n) { g_threads = n > 0 ? n : 1; }
EXPORT int sdeo_get_threads(void) { return g_threads; }

/* ------------------------------------------------------------------------ */
/* NumPy float32 add.reduce: result = 0.0f + pairwise_sum(a, n).             */
/* numpy/_core/src/umath/loops_utils.h.src (pairwise_sum, PW_BLOCKSIZE 128); */
/* the leading 0.0f is add's reduction identity (turns a -0.0 sum into +0).  */
/* ------------------------------------------------------------------------ */
static float pw_sum_strided(const float *a, long n, long stride)
{
    if (n < 8) {
        float res = 0.0f;
        for (long i = 0; i < n; i++) res += a[i * stride];
        return res;
    } else if (n <= 128) {
        float r[8];
        for (int j = 0; j < 8; j++) r[j] = a[j * stride];
        long i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[(i + j) * stride];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i * stride];
        return res;
    } else {
        long n2 = n / 2;
        n2 -= n2 % 8;
        return pw_sum_strided(a, n2, stride) + pw_sum_strided(a + n2 * stride, n - n2, stride);
    }
}

EXPORT float sdeo_np_sum_f32(const float *a, long n)
{
    return 0.0f + pw_sum_strided(a, n, 1);
}

/* -(np.sum(np.multiply(l, r))) for one voxel: process_functional.py:58,72 */
static float np_neg_dot(const float *l, const float *r, int C, float *tmp)
{
    for (int c = 0; c < C; c++) tmp[c] = l[c] * r[c];
    float s = 0.0f + pw_sum_strided(tmp, C, 1);
    return -1.0f * s;   /* `-1 * left_cost_volume` (process_functional.py:72) */
}

/*
 * compute_cost_volume (process_functional.py:48-73): out[d][y][x] =
 * -(sum_c fl[y][x][c] * fr[y][x-d][c]) for x >= d, -0.0 otherwise.
 */
EXPORT void sdeo_cost_volume_dhw(const float *fl, const float *fr, int H, int W, int C, int D,
                                 float *out)
{
#pragma omp parallel num_threads(g_threads)
    {
        float *tmp = (float *)malloc(sizeof(float) * (C > 0 ? C : 1));
#pragma omp for schedule(static)
        for (int y = 0; y < H; y++)
            for (int d = 0; d < D; d++)
                for (int x = 0; x < W; x++) {
                    float *o = out + ((size_t)d * H + y) * W + x;
                    if (x >= d)
                        *o = np_neg_dot(fl + ((size_t)y * W + x) * C, fr + ((size_t)y * W + x - d) * C, C, tmp);
                    else
                        *o = -0.0f;   /* np.zeros then `-1 *` */
                }
        free(tmp);
    }
}

/*
 * GPU-path volume layout [H][W][D] (process_functional.py:120-131): left
 * L[y][x][d] = cost(x,d) for x >= d; right R[y][x-d][d] = cost(x,d); every
 * voxel never written keeps `invalid` (1.0 in the reference, :1111-1114).
 * Valid costs use the CPU-path numerics above.
 */
EXPORT void sdeo_cost_volume_hwd(const float *fl, const float *fr, int H, int W, int C, int D,
                                 float invalid, float *outl, float *outr)
{
#pragma omp parallel num_threads(g_threads)
    {
        float *tmp = (float *)malloc(sizeof(float) * (C > 0 ? C : 1));
        /* row y's voxels (left and right) are written by row y's thread only */
#pragma omp for schedule(static)
        for (int y = 0; y < H; y++) {
            const size_t r0 = (size_t)y * W * D, rn = (size_t)W * D;
            if (outl) for (size_t i = 0; i < rn; i++) outl[r0 + i] = invalid;
            if (outr) for (size_t i = 0; i < rn; i++) outr[r0 + i] = invalid;
            for (int x = 0; x < W; x++)
                for (int d = 0; d < D && d <= x; d++) {
                    float c = np_neg_dot(fl + ((size_t)y * W + x) * C, fr + ((size_t)y * W + x - d) * C, C, tmp);
                    if (outl) outl[((size_t)y * W + x) * D + d] = c;
                    if (outr) outr[((size_t)y * W + x - d) * D + d] = c;
                }
        }
        free(tmp);
    }
}

/* WTA1 (process_functional.py:96-113): first d with cost < running min (init +inf). */
EXPORT int sdeo_wta1_dhw(const float *cv, int D, int H, int W, float *disp)
{
    int bad = 0;
#pragma omp parallel for num_threads(g_threads) reduction(+ : bad) schedule(static)
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            float best = INFINITY;
            int arg = -1;
            for (int d = 0; d < D; d++) {
                float v = cv[((size_t)d * H + y) * W + x];
                if (v < best) { best = v; arg = d; }
            }
            if (arg < 0) bad++;
            disp[(size_t)y * W + x] = (float)arg;
        }
    return bad;   /* reference asserts arg >= 0 (:109) */
}

/* WTA (process_functional.py:76-93): same rule on an [H][W][D] volume. */
EXPORT int sdeo_wta_hwd(const float *cv, int H, int W, int D, float *disp)
{
    int bad = 0;
#pragma omp parallel for num_threads(g_threads) reduction(+ : bad) schedule(static)
    for (size_t p = 0; p < (size_t)H * W; p++) {
        float best = INFINITY;
        int arg = -1;
        for (int d = 0; d < D; d++) {
            float v = cv[p * D + d];
            if (v < best) { best = v; arg = d; }
        }
        if (arg < 0) bad++;
        disp[p] = (float)arg;
    }
    return bad;
}

/*
 * WTA_and_SupixelRefinement_kernel (process_functional.py:800-837): first-min
 * with `min_s > tmp`, initialised from d = 0 (not +inf).
 */
EXPORT void sdeo_wta_sgm_hwd(const float *S, int H, int W, int D, float *disp)
{
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (size_t p = 0; p < (size_t)H * W; p++) {
        float m = S[p * D];
        int arg = 0;
        for (int d = 1; d < D; d++) {
            float v = S[p * D + d];
            if (m > v) { m = v; arg = d; }
        }
        disp[p] = (float)arg;
    }
}

/*
 * Fused cost volume + first-min over a disparity shard [d0, d1) without
 * materialising the volume: min value and argmin (global d index, -1 if no
 * candidate beat +inf).  Invalid voxels (x < d) take -0.0 as in the CPU path.
 */
EXPORT void sdeo_cv_wta_shard(const float *fl, const float *fr, int H, int W, int C, int d0, int d1,
                              float *minv, int32_t *argmin)
{
#pragma omp parallel num_threads(g_threads)
    {
        float *tmp = (float *)malloc(sizeof(float) * (C > 0 ? C : 1));
#pragma omp for schedule(static)
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++) {
                float best = INFINITY;
                int arg = -1;
                for (int d = d0; d < d1; d++) {
                    float v = (x >= d) ? np_neg_dot(fl + ((size_t)y * W + x) * C, fr + ((size_t)y * W + x - d) * C, C,
                                                    tmp)
                                       : -0.0f;
                    if (v < best) { best = v; arg = d; }
                }
                minv[(size_t)y * W + x] = best;
                argmin[(size_t)y * W + x] = arg;
            }
        free(tmp);
    }
}

/* ------------------------------------------------------------------------ */
/* SGM penalties: sgm_penelty_kernel (process_functional.py:134-262).        */
/* Numba types uint8 - uint8 as uint64 (wraps), `-diff if diff < 0` is a     */
/* no-op, and `diff > threshold` compares as float64: reduced iff            */
/* nb < c or nb > c + thr.  The (y-1) block writes ch 2/3 but the (y+1)      */
/* block (:159-172) overwrites them, so ch 0/1 stay 0.                       */
/* ------------------------------------------------------------------------ */
EXPORT void sdeo_sgm_penalties(const uint8_t *img, int H, int W, double P1, double P2, long thr,
                               double lambda, float *pen)
{
    const float fP1 = (float)P1, fP2 = (float)P2;
    const float rP1 = (float)(P1 / lambda), rP2 = (float)(P2 / lambda);
    static const int nb[8][3] = {
        /* dy, dx, channel */
        {-1, 0, 2}, {+1, 0, 2}, {0, -1, 4}, {0, +1, 6},
        {+1, -1, 8}, {+1, +1, 10}, {-1, +1, 12}, {-1, -1, 14},
    };
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            float *p = pen + ((size_t)y * W + x) * 16;
            p[0] = 0.0f;
            p[1] = 0.0f;
            const uint64_t c = img[(size_t)y * W + x];
            for (int k = 0; k < 8; k++) {
                int yy = y + nb[k][0], xx = x + nb[k][1], ch = nb[k][2];
                if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
                    uint64_t diff = (uint64_t)img[(size_t)yy * W + xx] - c;
                    int red = (double)diff > (double)thr;
                    p[ch] = red ? rP1 : fP1;
                    p[ch + 1] = red ? rP2 : fP2;
                } else {
                    p[ch] = fP1;
                    p[ch + 1] = fP2;
                }
            }
        }
}

/* ------------------------------------------------------------------------ */
/* 8-path SGM (process_functional.py:265-797, launch order :1166-1203).      */
/* The reference runs one warp per scanline: lane j of the 32 holds the 4   */
/* disparities 4j..4j+3 (D = 128).  Its arithmetic, restated exactly so     */
/* that non-finite costs propagate as they do there:                        */
/*  - every `min(a, b)` is Numba's (= Python's) binary min: b if b < a else  */
/*    a (numba cpython/builtins.py do_minmax: select(v < acc, v, acc)), so a */
/*    NaN first argument sticks and a NaN second argument is ignored;       */
/*  - c_k += min(min(L(d-1) + P1, L(d)), min(L(d+1) + P1, mcP2)) - mc with  */
/*    L(d-1) := L(d) at d = 0 and L(d+1) := L(d) at d = D-1 (:300-303,        */
/*    :306-320);                                                            */
/*  - the minimum is per lane: m = min(min(c1, c2), min(c3, c4)), then       */
/*    m = min(m, shfl_xor(m, k)) for k = 1, 2, 4, 8, 16 (:329-338) -- with  */
/*    NaN present, lanes can end with different minima, and each lane uses */
/*    its own m and m + P2 at the next step.                                 */
/* For finite costs every lane's m is the global minimum and the chain's   */
/* value is the plain minimum, so the result does not depend on the        */
/* grouping.  Generic D (the reference has D = 128 only): lanes of 4        */
/* (missing disparities of the last lane act as +inf, which the binary min  */
/* ignores), the butterfly over the next power of two of ceil(D/4) lanes    */
/* with the padding lanes at +inf.                                          */
/* ------------------------------------------------------------------------ */
static inline double pymin(double a, double b) { return b < a ? b : a; }

typedef struct {
    double *L;      /* path cost of the previous pixel, fp64 (Numba-unified) */
    double *Ln;
    double *m;      /* per reference lane (4 disparities): min_cost */
    double *mP2;    /* per reference lane: min_cost + P2 */
    double *v;      /* butterfly scratch, nlp entries */
    int nlp;        /* reference lanes, rounded up to a power of two */
} sgm_state;

static int sgm_lanes_pow2(int D)
{
    int nl = (D + 3) / 4, p = 1;
    while (p < nl) p <<= 1;
    return p;
}

/* One SGM_Interation (:265-343) at pixel (r,c). */
static void sgm_step(const float *C, float *S, sgm_state *st, int D, int restart, double P1, double P2,
                     int calc_min)
{
    double *L = st->L, *Ln = st->Ln;
    if (restart) {
        for (int d = 0; d < D; d++) Ln[d] = (double)C[d];
    } else {
        for (int d = 0; d < D; d++) {
            const double self = L[d];
            const double lft = d > 0 ? L[d - 1] : self, rgt = d < D - 1 ? L[d + 1] : self;
            const double m1 = pymin(lft + P1, self);
            const double m2 = pymin(rgt + P1, st->mP2[d >> 2]);
            Ln[d] = (double)C[d] + (pymin(m1, m2) - st->m[d >> 2]);
        }
    }
    for (int d = 0; d < D; d++) S[d] = (float)((double)S[d] + Ln[d]);
    if (calc_min) {
        double *v = st->v;
        const int nlp = st->nlp;
        for (int j = 0; j < nlp; j++) {
            double c[4];
            for (int k = 0; k < 4; k++) c[k] = 4 * j + k < D ? Ln[4 * j + k] : INFINITY;
            v[j] = pymin(pymin(c[0], c[1]), pymin(c[2], c[3]));
        }
        for (int k = 1; k < nlp; k <<= 1) {
            /* simultaneous exchange: m_j = min(m_j, m_{j^k}); each pair computed from the old values */
            for (int j = 0; j < nlp; j++) {
                const int o = j ^ k;
                if (o < j) continue;
                const double a = v[j], b = v[o];
                v[j] = pymin(a, b);
                v[o] = pymin(b, a);
            }
        }
        for (int j = 0; j < nlp; j++) {
            st->m[j] = v[j];
            st->mP2[j] = v[j] + P2;
        }
    }
    st->L = Ln;
    st->Ln = L;
}

static void sgm_state_init(sgm_state *st, double *buf, int D)
{
    const int nlp = sgm_lanes_pow2(D);
    st->L = buf;
    st->Ln = buf + D;
    st->m = buf + 2 * D;
    st->mP2 = buf + 2 * D + nlp;
    st->v = buf + 2 * D + 2 * nlp;
    st->nlp = nlp;
    for (int d = 0; d < D; d++) st->L[d] = 1.0;     /* old_values = 1.0 (:359-364); unused at restart */
    for (int j = 0; j < nlp; j++) st->m[j] = st->mP2[j] = 1.0;
}

static inline int sgm_nsteps(int n) { return n - 1 > 2 ? n - 1 : 2; }

enum { SGM_UD = 0, SGM_DU, SGM_LR, SGM_RL, SGM_UDLR, SGM_DULR, SGM_UDRL, SGM_DURL };

/* One direction over one side: cv/pen/S are [H][W][D], [H][W][16], [H][W][D].  Lines are
 * independent (each pixel is visited once per direction), so they run in parallel. */
EXPORT void sdeo_sgm_direction(const float *cv, const float *pen, int H, int W, int D, int dir,
                               float *S)
{
#define CV(r, c) (cv + ((size_t)(r) * W + (c)) * D)
#define SS(r, c) (S + ((size_t)(r) * W + (c)) * D)
#define PEN(r, c, ch) ((double)pen[((size_t)(r) * W + (c)) * 16 + (ch)])
    const int nlp = sgm_lanes_pow2(D);
    const int nlines = (dir == SGM_LR || dir == SGM_RL) ? H : W;
#pragma omp parallel num_threads(g_threads)
    {
        double *buf = (double *)malloc(sizeof(double) * (2 * (size_t)D + 3 * (size_t)nlp));
#pragma omp for schedule(dynamic, 16)
        for (int line = 0; line < nlines; line++) {
            sgm_state st;
            sgm_state_init(&st, buf, D);
            if (dir == SGM_UD || dir == SGM_DU) {
                const int n = sgm_nsteps(H), c = line;
                for (int k = 0; k < n; k++) {
                    int r = dir == SGM_UD ? k : H - 1 - k;
                    double P1 = 0.0, P2;
                    if (dir == SGM_UD) { if (r - 1 >= 0) P1 = PEN(r - 1, c, 2); P2 = PEN(r, c, 3); }
                    else               { if (r + 1 < H)  P1 = PEN(r + 1, c, 0); P2 = PEN(r, c, 1); }
                    sgm_step(CV(r, c), SS(r, c), &st, D, k == 0, P1, P2, k < n - 1);
                }
            } else if (dir == SGM_LR || dir == SGM_RL) {
                const int n = sgm_nsteps(W), r = line;
                for (int k = 0; k < n; k++) {
                    int c = dir == SGM_LR ? k : W - 1 - k;
                    double P1 = 0.0, P2;
                    if (dir == SGM_LR) { if (c - 1 >= 0) P1 = PEN(r, c - 1, 6); P2 = PEN(r, c, 7); }
                    else               { if (c + 1 < W)  P1 = PEN(r, c + 1, 4); P2 = PEN(r, c, 5); }
                    sgm_step(CV(r, c), SS(r, c), &st, D, k == 0, P1, P2, k < n - 1);
                }
            } else {
                const int n = sgm_nsteps(H);
                const int down = (dir == SGM_UDLR || dir == SGM_UDRL);
                const int right = (dir == SGM_UDLR || dir == SGM_DULR);
                const int p1ch = dir == SGM_UDLR ? 10 : dir == SGM_DULR ? 12 : dir == SGM_UDRL ? 8 : 14;
                int c = line;
                for (int k = 0; k < n; k++) {
                    int r = down ? k : H - 1 - k;
                    int restart = (k == 0);
                    if (k > 0) {
                        c += right ? 1 : -1;
                        if (right && c >= W) { c = 0; restart = 1; }
                        if (!right && c < 0) { c = W - 1; restart = 1; }
                    }
                    int pr = down ? r - 1 : r + 1;
                    int pc = right ? c - 1 : c + 1;
                    double P1 = 0.0;
                    if (pr >= 0 && pr < H && pc >= 0 && pc < W) P1 = PEN(pr, pc, p1ch);
                    double P2 = PEN(r, c, p1ch + 1);
                    sgm_step(CV(r, c), SS(r, c), &st, D, restart, P1, P2, k < n - 1);
                }
            }
        }
        free(buf);
    }
#undef CV
#undef SS
#undef PEN
}

/* All 8 directions in the reference launch order; S is accumulated (caller zeroes it). */
EXPORT void sdeo_sgm_8path(const float *cv, const float *pen, int H, int W, int D, float *S)
{
    for (int dir = 0; dir < 8; dir++) sdeo_sgm_direction(cv, pen, H, W, D, dir, S);
}

/* ------------------------------------------------------------------------ */
/* Post-processing ("next" rows): is_error_match_kernel (:977-1000),        */
/* LRC_kernel (:1003-1088), Median_Filter_kernel (:840-879).                 */
/* uint8() index casts are restated as truncation toward zero then mod 256  */
/* (PARITY UNPINNED: Numba's float->uint8 out-of-range behaviour).           */
/* ------------------------------------------------------------------------ */
static inline int u8cast(double v) { long long t = (long long)v; return (int)(t & 255); }

EXPORT void sdeo_lr_check(const float *dl, const float *dr, int H, int W, uint8_t *lrcl, uint8_t *lrcr)
{
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            double ld = dl[(size_t)y * W + x];
            double rd = (double)x - ld;
            if (rd >= 0) {
                double r2 = dr[(size_t)y * W + u8cast(rd)];
                double mn = ld - r2;
                lrcl[(size_t)y * W + x] = (mn > 1 || mn < -1) ? 1 : 0;
            }
            double rd2 = dr[(size_t)y * W + x];
            double ld2 = (double)x + rd2;
            if (ld2 < W) {
                double l2 = dl[(size_t)y * W + u8cast(ld2)];
                double mn = rd2 - l2;
                lrcr[(size_t)y * W + x] = (mn > 1 || mn < -1) ? 1 : 0;
            }
        }
}

EXPORT void sdeo_lrc_fill(const float *dl, const uint8_t *lrcl, int H, int W, float *out)
{
#pragma omp parallel for num_threads(g_threads) schedule(dynamic, 4)
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            size_t p = (size_t)y * W + x;
            if (lrcl[p] == 1) {
                int number = 0;
                double sum = 0.0;   /* int 0 + float32 -> float64 in Numba */
                int iy = y;
                while (iy >= 0 && lrcl[(size_t)iy * W + x] == 1) iy--;
                if (iy >= 0) { number++; sum += dl[(size_t)iy * W + x]; }
                iy = y;
                while (iy < H && lrcl[(size_t)iy * W + x] == 1) iy++;
                if (iy < H) { number++; sum += dl[(size_t)iy * W + x]; }
                int ix = x;
                while (ix < W && lrcl[(size_t)y * W + ix] == 1) ix++;
                if (ix < W) { number++; sum += dl[(size_t)y * W + ix]; }
                ix = x;
                while (ix >= 0 && lrcl[(size_t)y * W + ix] == 1) ix--;
                if (ix >= 0) { number++; sum += dl[(size_t)y * W + ix]; }
                out[p] = number > 0 ? (float)(sum / number) : dl[p];
            } else {
                out[p] = dl[p];
            }
        }
}

/* 5x5 median of the interior (2-px border of `out` untouched): partial selection sort to the 13th. */
EXPORT void sdeo_median5(const float *in, int H, int W, float *out)
{
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (int y = 2; y < H - 2; y++)
        for (int x = 2; x + 2 < W; x++) {
            float w[25];
            for (int i = -2; i <= 2; i++)
                for (int j = -2; j <= 2; j++) w[(i + 2) * 5 + j + 2] = in[(size_t)(y + i) * W + x + j];
            float cur = 0.0f;
            for (int i = 0; i < 13; i++) {
                cur = w[i];
                int ci = i;
                for (int j = i + 1; j < 25; j++)
                    if (cur > w[j]) { cur = w[j]; ci = j; }
                w[ci] = w[i];
            }
            out[(size_t)y * W + x] = cur;
        }
}

/* ------------------------------------------------------------------------ */
/* MC-CNN-fast branch (mc_cnn_brunch.py:31-48,70-92) in fp64: 3x3 VALID      */
/* cross-correlation, HWIO weights, bias, ReLU on all but the last layer,    */
/* then tf.nn.l2_normalize(dim=-1) = x * rsqrt(max(sum x^2, 1e-12)).         */
/* ------------------------------------------------------------------------ */
EXPORT void sdeo_tower_forward(const float *img_pad, int Hp, int Wp, int nlayers, int nf,
                               const float *const *weights, const float *const *biases, float *out)
{
    int h = Hp, w = Wp, cin = 1;
    double *cur = (double *)malloc(sizeof(double) * (size_t)Hp * Wp);
    for (size_t i = 0; i < (size_t)Hp * Wp; i++) cur[i] = img_pad[i];
    for (int l = 0; l < nlayers; l++) {
        int ho = h - 2, wo = w - 2;
        double *nxt = (double *)malloc(sizeof(double) * (size_t)ho * wo * nf);
        const float *Wt = weights[l], *B = biases[l];
#pragma omp parallel for num_threads(g_threads) schedule(static)
        for (int y = 0; y < ho; y++)
            for (int x = 0; x < wo; x++)
                for (int n = 0; n < nf; n++) {
                    double s = 0.0;
                    for (int ky = 0; ky < 3; ky++)
                        for (int kx = 0; kx < 3; kx++)
                            for (int c = 0; c < cin; c++)
                                s += cur[((size_t)(y + ky) * w + (x + kx)) * cin + c] *
                                     (double)Wt[((ky * 3 + kx) * cin + c) * nf + n];
                    s += B[n];
                    if (l < nlayers - 1 && s < 0) s = 0;
                    nxt[((size_t)y * wo + x) * nf + n] = s;
                }
        free(cur);
        cur = nxt;
        h = ho;
        w = wo;
        cin = nf;
    }
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (size_t p = 0; p < (size_t)h * w; p++) {
        double ss = 0.0;
        for (int n = 0; n < nf; n++) ss += cur[p * nf + n] * cur[p * nf + n];
        double inv = 1.0 / sqrt(ss > 1e-12 ? ss : 1e-12);
        for (int n = 0; n < nf; n++) out[p * nf + n] = (float)(cur[p * nf + n] * inv);
    }
    free(cur);
}

/* ------------------------------------------------------------------------ */
/* Cross-based cost aggregation -- BUILD-DEFINED, PARITY UNPINNED.           */
/* The reference has none (only the buffer name          */
/* d_cost_volumel_after_aggr, process_functional.py:268,347, and an unused   */
/* timer label, match.py:98).  Definition v2 (round 4; MC-CNN-style cross    */
/* support of both images):                                                  */
/*  arms: for pixel p and direction left/right/up/down, the largest k in     */
/*   [0, L1-1] such that every q = p + j*dir, 1 <= j <= k, is inside the     */
/*   image and fabsf(I(p) - I(q)) < tau (fp32).  Packed l | r<<8 | u<<16 |   */
/*   d<<24.                                                                  */
/*  coordinates: volumes are aggregated in LEFT coordinates q (the left      */
/*   image's column): a left-referenced volume L(y,q,d) as it is, a right-   */
/*   referenced one through R(y,x',d) = L(y,x'+d,d).  Voxel (y,q,d) is valid */
/*   iff its right-image pixel q-d is inside the image (q >= d); an invalid  */
/*   voxel passes through every pass unchanged.                              */
/*  support arms of a valid voxel: per direction min(left-image arm at       */
/*   (y,q), right-image arm at (y,q-d)).  A right-referenced voxel and the   */
/*   left voxel it shears from have ONE support, so CBCA(R) = shear(CBCA(L)) */
/*   exactly whenever R = shear(L) (the GPU path's L/R volumes are).         */
/*  segments: every line is cut into segments of S = CBCA_SEG positions; the */
/*   prefix chain of segment k starts at b = max(kS - M, first valid         */
/*   position of the line) with M = L1 - 1 (the longest arm) and             */
/*   P(b-1) = 0, so both ends of every window of the segment lie on its own  */
/*   chain (a GPU wave can take any segment with an M-position pre-roll).    */
/*  horizontal pass, row y, disparity d, valid q in [d, W):                  */
/*   P(i) = P(i-1) + (double)C(y,i,d),  T(y,q,d) = (float)(P(q+hr) - P(q-hl-1)) */
/*  vertical pass, column q (valid), disparity d (rows; first valid row 0):  */
/*   Q(i) = Q(i-1) + (double)T(i,q,d),  N(i) = N(i-1) + hl + hr + 1 at (i,q,d) */
/*   C'(y,q,d) = (float)((Q(y+vd) - Q(y-vu-1)) * (1.0 / (double)cnt)),       */
/*   cnt = N(y+vd) - N(y-vu-1) (exact), 1.0/cnt the correctly rounded fp64   */
/*   reciprocal: the mean over the union of the horizontal segments hanging  */
/*   off the voxel's vertical segment.                                       */
/*  one iteration = horizontal pass, then vertical pass.                     */
/* (v1, rounds 1-3: prefixes from the line start, both volumes aggregated    */
/* independently, fp64 division.)                                            */
/* ------------------------------------------------------------------------ */
#define CBCA_SEG 256 /* = SDE_CBCA_SEG (include/sde.h; test_capi checks they agree) */
EXPORT int sdeo_cbca_seg(void) { return CBCA_SEG; }

EXPORT void sdeo_cbca_arms(const float *img, long pitch, int H, int W, int L1, float tau, uint32_t *arms)
{
    static const int dys[4] = {0, 0, -1, 1}, dxs[4] = {-1, 1, 0, 0};
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            const float c = img[(size_t)y * pitch + x];
            uint32_t packed = 0;
            for (int k = 0; k < 4; k++) {
                int len = 0;
                while (len + 1 <= L1 - 1) {
                    const int yy = y + (len + 1) * dys[k], xx = x + (len + 1) * dxs[k];
                    if (yy < 0 || yy >= H || xx < 0 || xx >= W) break;
                    if (!(fabsf(c - img[(size_t)yy * pitch + xx]) < tau)) break;
                    len++;
                }
                packed |= (uint32_t)len << (8 * k);
            }
            arms[(size_t)y * W + x] = packed;
        }
}

/* support arms of the valid left-coordinate voxel (y, q, d): al / ar = left / right image arms */
static inline void cbca_support(const uint32_t *al, const uint32_t *ar, int W, int y, int q, int d, int *a)
{
    const uint32_t p = al[(size_t)y * W + q], o = ar[(size_t)y * W + q - d];
    for (int k = 0; k < 4; k++) {
        const int u = (p >> (8 * k)) & 255, v = (o >> (8 * k)) & 255;
        a[k] = u < v ? u : v;
    }
}

static inline int imax(int a, int b) { return a > b ? a : b; }
static inline int imin(int a, int b) { return a < b ? a : b; }

/* Horizontal pass on a left-coordinate volume (src -> dst, [H][W][D]).  Loops run d innermost
 * (contiguous voxels); every (row, d, segment) chain is still accumulated sequentially in the
 * definition's order. */
EXPORT void sdeo_cbca_hpass(const float *src, float *dst, const uint32_t *al, const uint32_t *ar, int H, int W,
                            int D, int L1)
{
    const int M = L1 - 1, S = CBCA_SEG;
#pragma omp parallel num_threads(g_threads)
    {
        /* P[(i + 1) * D + d] = chain of (y, d, segment) through position i; P[b * D + d] = 0 */
        double *P = (double *)malloc(sizeof(double) * (size_t)(W + 1) * D);
#pragma omp for schedule(static)
        for (int y = 0; y < H; y++) {
            const size_t row = (size_t)y * W * D;
            for (int q = 0; q < W; q++)
                for (int d = q + 1; d < D; d++) dst[row + (size_t)q * D + d] = src[row + (size_t)q * D + d];
            for (int k = 0; k * S < W; k++) {
                const int t1 = imin((k + 1) * S, W), e = imin(t1 - 1 + M, W - 1), b0 = imax(k * S - M, 0);
                for (int d = 0; d < D && d <= e; d++) P[(size_t)imax(b0, d) * D + d] = 0.0;
                for (int i = b0; i <= e; i++)
                    for (int d = 0; d < D && d <= i; d++)   /* i >= b = max(b0, d) */
                        P[(size_t)(i + 1) * D + d] = P[(size_t)i * D + d] + (double)src[row + (size_t)i * D + d];
                for (int q = k * S; q < t1; q++)
                    for (int d = 0; d < D && d <= q; d++) {
                        int a[4];
                        cbca_support(al, ar, W, y, q, d, a);
                        dst[row + (size_t)q * D + d] =
                            (float)(P[(size_t)(q + a[1] + 1) * D + d] - P[(size_t)(q - a[0]) * D + d]);
                    }
            }
        }
        free(P);
    }
}

/* Vertical pass on a left-coordinate volume (src -> dst). */
EXPORT void sdeo_cbca_vpass(const float *src, float *dst, const uint32_t *al, const uint32_t *ar, int H, int W,
                            int D, int L1)
{
    const int M = L1 - 1, S = CBCA_SEG;
#pragma omp parallel num_threads(g_threads)
    {
        /* Q / N[(i + 1) * D + d]: chain of column (q, d, segment) through row i */
        double *Q = (double *)malloc(sizeof(double) * (size_t)(H + 1) * D);
        long *N = (long *)malloc(sizeof(long) * (size_t)(H + 1) * D);
#pragma omp for schedule(static)
        for (int q = 0; q < W; q++) {
            for (int y = 0; y < H; y++)
                for (int d = q + 1; d < D; d++) {
                    const size_t v = ((size_t)y * W + q) * D + d;
                    dst[v] = src[v];
                }
            const int dn = imin(D, q + 1);   /* valid disparities of this column: d <= q */
            for (int k = 0; k * S < H; k++) {
                const int t1 = imin((k + 1) * S, H), e = imin(t1 - 1 + M, H - 1), b = imax(k * S - M, 0);
                for (int d = 0; d < dn; d++) {
                    Q[(size_t)b * D + d] = 0.0;
                    N[(size_t)b * D + d] = 0;
                }
                for (int i = b; i <= e; i++)
                    for (int d = 0; d < dn; d++) {
                        int a[4];
                        cbca_support(al, ar, W, i, q, d, a);
                        const size_t u = (size_t)(i + 1) * D + d, w = (size_t)i * D + d;
                        Q[u] = Q[w] + (double)src[((size_t)i * W + q) * D + d];
                        N[u] = N[w] + a[0] + a[1] + 1;
                    }
                for (int y = k * S; y < t1; y++)
                    for (int d = 0; d < dn; d++) {
                        int a[4];
                        cbca_support(al, ar, W, y, q, d, a);
                        const size_t hi = (size_t)(y + a[3] + 1) * D + d, lo = (size_t)(y - a[2]) * D + d;
                        const double num = Q[hi] - Q[lo];
                        const long cnt = N[hi] - N[lo];
                        dst[((size_t)y * W + q) * D + d] = (float)(num * (1.0 / (double)cnt));
                    }
            }
        }
        free(Q);
        free(N);
    }
}

/* Per-disparity cyclic rotation of every row: out(y, x, d) = in(y, (x + s*d) mod W, d), s = +1 / -1.
 * s = -1 takes a right-referenced volume to left coordinates (its invalid voxels land on the
 * left-coordinate invalid ones, q < d), s = +1 takes it back. */
static void cbca_rotate(const float *in, float *out, int H, int W, int D, int s)
{
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++)
            for (int d = 0; d < D; d++) {
                const long src = (((long)x + s * (long)(d % W)) % W + W) % W;
                out[((size_t)y * W + x) * D + d] = in[((size_t)y * W + src) * D + d];
            }
}

/* iters x (horizontal pass, vertical pass) of one volume, in place in cv (tmp: scratch of the same
 * size).  side 1: left-referenced (arms_ref = left image, arms_other = right image); side 2:
 * right-referenced (arms_ref = right image, arms_other = left image), aggregated in left
 * coordinates through the rotation above. */
EXPORT void sdeo_cbca(float *cv, float *tmp, const uint32_t *ref, const uint32_t *oth, int H, int W, int D, int side,
                      int L1, int iters)
{
    if (side == 1) {
        for (int it = 0; it < iters; it++) {
            sdeo_cbca_hpass(cv, tmp, ref, oth, H, W, D, L1);
            sdeo_cbca_vpass(tmp, cv, ref, oth, H, W, D, L1);
        }
        return;
    }
    float *rot = (float *)malloc(sizeof(float) * (size_t)H * W * D);
    cbca_rotate(cv, rot, H, W, D, -1);
    for (int it = 0; it < iters; it++) {
        sdeo_cbca_hpass(rot, tmp, oth, ref, H, W, D, L1);
        sdeo_cbca_vpass(tmp, rot, oth, ref, H, W, D, L1);
    }
    cbca_rotate(rot, cv, H, W, D, +1);
    free(rot);
}

/* The GPU path's pair (sde_cbca_lr): the left volume aggregated in place, then every valid voxel of
 * the right volume set to its shear, cv_r(y, x', d) = cv_l(y, x'+d, d) for x'+d < W (invalid ones
 * untouched).  Equal to sdeo_cbca(cv_r, side 2) whenever cv_r's valid voxels are cv_l's shear. */
EXPORT void sdeo_cbca_lr(float *cv_l, float *cv_r, float *tmp, const uint32_t *al, const uint32_t *ar, int H, int W,
                         int D, int L1, int iters)
{
    sdeo_cbca(cv_l, tmp, al, ar, H, W, D, 1, L1, iters);
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++)
            for (int d = 0; d < D && x + d < W; d++)
                cv_r[((size_t)y * W + x) * D + d] = cv_l[((size_t)y * W + x + d) * D + d];
}
