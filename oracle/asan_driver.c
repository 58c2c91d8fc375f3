/*
 * asan_driver.c -- runs every sde_oracle.c entry point under AddressSanitizer +
 * UndefinedBehaviorSanitizer (the oracle is the parity checker of
 * every stage, so its own memory safety is checked).  TEST INFRASTRUCTURE ONLY.
 *
 * Build + run: `make -C oracle asan` (tests/test_oracle.py::test_oracle_asan).  Shapes
 * cover the edges the kernels' tests use: 1-pixel and 2-pixel lines, D > W, D not a
 * multiple of 4, C not a multiple of 8, L1 at its maximum, fully flagged LRC maps, and
 * non-finite costs in SGM.
 */
#include "sde_oracle.c"

#include <stdio.h>

static uint64_t g_rng = 0x9E3779B97F4A7C15ull;
static float frand(void)
{
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return (float)((g_rng >> 11) * (1.0 / 9007199254740992.0)) * 2.0f - 1.0f;
}

static float *fbuf(size_t n)
{
    float *p = (float *)malloc(sizeof(float) * (n ? n : 1));
    for (size_t i = 0; i < n; i++) p[i] = frand();
    return p;
}

static void run_cv(int H, int W, int C, int D)
{
    float *fl = fbuf((size_t)H * W * C), *fr = fbuf((size_t)H * W * C);
    float *dhw = fbuf((size_t)D * H * W), *l = fbuf((size_t)H * W * D), *r = fbuf((size_t)H * W * D);
    float *disp = fbuf((size_t)H * W), *mn = fbuf((size_t)H * W);
    int32_t *am = (int32_t *)malloc(sizeof(int32_t) * (size_t)H * W);
    sdeo_cost_volume_dhw(fl, fr, H, W, C, D, dhw);
    (void)sdeo_wta1_dhw(dhw, D, H, W, disp);
    sdeo_cost_volume_hwd(fl, fr, H, W, C, D, 1.0f, l, r);
    sdeo_cost_volume_hwd(fl, fr, H, W, C, D, 1.0f, l, NULL);
    (void)sdeo_wta_hwd(l, H, W, D, disp);
    sdeo_wta_sgm_hwd(l, H, W, D, disp);
    sdeo_cv_wta_shard(fl, fr, H, W, C, D / 3, D, mn, am);
    (void)sdeo_np_sum_f32(fl, (long)H * W * C);
    free(fl); free(fr); free(dhw); free(l); free(r); free(disp); free(mn); free(am);
}

static void run_sgm_post(int H, int W, int D, int nonfinite)
{
    uint8_t *img = (uint8_t *)malloc((size_t)H * W), *a = (uint8_t *)calloc((size_t)H * W, 1),
            *b = (uint8_t *)calloc((size_t)H * W, 1);
    for (size_t i = 0; i < (size_t)H * W; i++) img[i] = (uint8_t)(frand() * 127.5f + 127.5f);
    float *cv = fbuf((size_t)H * W * D), *pen = fbuf((size_t)H * W * 16), *S = (float *)calloc((size_t)H * W * D, 4);
    if (nonfinite)
        for (size_t i = 0; i < (size_t)H * W * D; i += 7) cv[i] = (i % 3) ? INFINITY : NAN;
    float *dl = fbuf((size_t)H * W), *dr = fbuf((size_t)H * W), *out = fbuf((size_t)H * W);
    sdeo_sgm_penalties(img, H, W, 2.3, 55.9, 30, 4.0, pen);
    if (H >= 2 && W >= 2) sdeo_sgm_8path(cv, pen, H, W, D, S);
    sdeo_wta_sgm_hwd(S, H, W, D, dl);
    for (size_t i = 0; i < (size_t)H * W; i++) dr[i] = (float)(int)((frand() + 1.0f) * 4.0f);
    sdeo_lr_check(dl, dr, H, W, a, b);
    sdeo_lrc_fill(dl, a, H, W, out);
    memset(a, 1, (size_t)H * W);                 /* fully flagged: every walk runs off the image */
    sdeo_lrc_fill(dl, a, H, W, out);
    sdeo_median5(out, H, W, dl);
    free(img); free(a); free(b); free(cv); free(pen); free(S); free(dl); free(dr); free(out);
}

static void run_tower(int H, int W, int L)
{
    const int nf = 64, Hp = H + 2 * L, Wp = W + 2 * L;
    float *img = fbuf((size_t)Hp * Wp), *out = fbuf((size_t)H * W * nf);
    float *ws[8], *bs[8];
    for (int l = 0; l < L; l++) {
        ws[l] = fbuf((size_t)9 * (l ? nf : 1) * nf);
        bs[l] = fbuf(nf);
    }
    sdeo_tower_forward(img, Hp, Wp, L, nf, (const float *const *)ws, (const float *const *)bs, out);
    for (int l = 0; l < L; l++) { free(ws[l]); free(bs[l]); }
    free(img); free(out);
}

static void run_cbca(int H, int W, int D, int L1)
{
    float *img = fbuf((size_t)H * W), *img2 = fbuf((size_t)H * W);
    for (size_t i = 0; i < (size_t)H * W; i++) img[i] *= 0.01f, img2[i] *= 0.01f;   /* long arms */
    uint32_t *a = (uint32_t *)malloc(4 * (size_t)H * W), *b = (uint32_t *)malloc(4 * (size_t)H * W);
    sdeo_cbca_arms(img, W, H, W, L1, 0.05f, a);
    sdeo_cbca_arms(img2, W, H, W, L1, 0.05f, b);
    float *cv = fbuf((size_t)H * W * D), *tmp = fbuf((size_t)H * W * D);
    float *cr = fbuf((size_t)H * W * D);
    sdeo_cbca(cv, tmp, a, b, H, W, D, 1, L1, 2);
    sdeo_cbca(cv, tmp, b, a, H, W, D, 2, L1, 1);
    sdeo_cbca_lr(cv, cr, tmp, a, b, H, W, D, L1, 1);
    free(img); free(img2); free(a); free(b); free(cv); free(tmp); free(cr);
}

int main(void)
{
    for (int t = 1; t <= 3; t += 2) {
        sdeo_set_threads(t);
        run_cv(1, 1, 64, 1);
        run_cv(3, 7, 64, 12);
        run_cv(4, 9, 20, 5);
        run_cv(2, 5, 136, 9);
        run_cv(2, 3, 1, 4);
        run_sgm_post(2, 2, 4, 0);
        run_sgm_post(6, 9, 12, 1);
        run_sgm_post(9, 3, 7, 0);
        run_sgm_post(3, 9, 130, 1);
        run_sgm_post(1, 6, 8, 0);
        run_tower(3, 4, 1);
        run_tower(5, 6, 3);
        run_cbca(9, 13, 6, 32);
        run_cbca(1, 40, 3, 14);
        run_cbca(40, 1, 3, 14);
        run_cbca(270, 300, 3, 14);     /* two segments each way (CBCA_SEG = 256) */
        run_cbca(3, 5, 9, 2);          /* D > W */
    }
    printf("asan driver ok\n");
    return 0;
}
