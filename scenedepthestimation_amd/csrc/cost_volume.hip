// cost_volume.hip -- disparity cost volume, fused cost+WTA and WTA kernels (gfx950).
//
// Replaces (WHDY/SceneDepthEstimation):
//   compute_cost_volume        process_functional.py:48-73   (CPU path, [D,H,W], -0.0 fill)
//   WTA1 / WTA                 process_functional.py:96-113 / 76-93
//   compute_cost_volume_kernel process_functional.py:120-131 ([H,W,D] L and R, 1.0 fill)
//   WTA_and_SupixelRefinement_kernel process_functional.py:800-837
//
// Numerics: every valid voxel is the CPU path's value bit for bit,
//   cost(x,d) = -(0.0f + pairwise8_c(fl[y][x][c] * fr[y][x-d][c]))
// -- products rounded to f32, 8 running f32 accumulators over channel blocks of
// 8, then ((a0+a1)+(a2+a3))+((a4+a5)+(a6+a7)) (NumPy's pairwise_sum for C=64).
// The library is compiled with -ffp-contract=off so no product is fused.
//
// Mapping (C = 64 fast path): a workgroup is 4 waves on one image row and 64
// consecutive "own" pixels (one per lane, its 64-float feature vector held in
// VGPRs).  The 127 "other" feature rows a 64-disparity chunk touches are staged
// in LDS (XOR-swizzled 256-B rows: the 16 lanes of a ds_read_b128 group read 16
// consecutive rows -> 16 distinct bank slots).  Wave w sweeps disparities
// [16w, 16w+16) of each chunk; the fused WTA merges the 4 per-wave first-minima
// by (value, index) at the end, which equals the sequential scan.
#include "sde_common.h"

namespace sde {

constexpr int CV_TX = 64;                    // own pixels per workgroup (= lanes)
constexpr int CV_WAVES = 4;                  // waves per workgroup
constexpr int CV_DC = 64;                    // disparities per LDS chunk
constexpr int CV_DW = CV_DC / CV_WAVES;      // disparities per wave per chunk
constexpr int CV_ROWS = CV_TX + CV_DC - 1;   // other-side rows per chunk

enum { OUT_WTA = 0, OUT_DHW = 1, OUT_HWD = 2 };

// Exact -(0 + pairwise8) of own[64] (registers) and one swizzled LDS row.
__device__ __forceinline__ float dot64_exact(const float (&own)[64], const float4 *__restrict__ win, int lr)
{
    float acc[8];
#pragma unroll
    for (int m = 0; m < 8; m++) {
        const float4 a = win[swz_row16(lr, 2 * m)];
        const float4 b = win[swz_row16(lr, 2 * m + 1)];
        const float p0 = own[8 * m + 0] * a.x, p1 = own[8 * m + 1] * a.y;
        const float p2 = own[8 * m + 2] * a.z, p3 = own[8 * m + 3] * a.w;
        const float p4 = own[8 * m + 4] * b.x, p5 = own[8 * m + 5] * b.y;
        const float p6 = own[8 * m + 6] * b.z, p7 = own[8 * m + 7] * b.w;
        if (m == 0) {
            acc[0] = p0; acc[1] = p1; acc[2] = p2; acc[3] = p3;
            acc[4] = p4; acc[5] = p5; acc[6] = p6; acc[7] = p7;
        } else {
            acc[0] += p0; acc[1] += p1; acc[2] += p2; acc[3] += p3;
            acc[4] += p4; acc[5] += p5; acc[6] += p6; acc[7] += p7;
        }
    }
    const float res = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    return -(0.0f + res);
}

// SIDE_LEFT : own = fl at x,  other = fr at x - d   (L[y][x][d])
// SIDE_RIGHT: own = fr at x', other = fl at x' + d  (R[y][x'][d] = cost(x'+d, d))
template <int SIDE, int OUT>
__global__ __launch_bounds__(256) void cv64_kernel(const float *__restrict__ own_feat,
                                                   const float *__restrict__ other_feat, int H, int W,
                                                   int d0, int d1, int Dvol, float invalid,
                                                   float *__restrict__ out, float *__restrict__ out_min,
                                                   int32_t *__restrict__ out_arg, float *__restrict__ out_disp)
{
    __shared__ float4 win[CV_ROWS * 16];
    __shared__ float otile[OUT == OUT_HWD ? CV_TX * (CV_DC + 1) : 1];

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int y = blockIdx.y;
    const int q0 = blockIdx.x * CV_TX;
    const int q = q0 + lane;
    const bool qok = q < W;

    float own[64];
    {
        const float4 *src = reinterpret_cast<const float4 *>(own_feat + ((size_t)y * W + (qok ? q : 0)) * 64);
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const float4 v = src[k];
            own[4 * k + 0] = v.x; own[4 * k + 1] = v.y; own[4 * k + 2] = v.z; own[4 * k + 3] = v.w;
        }
    }
    const float4 *other4 = reinterpret_cast<const float4 *>(other_feat) + (size_t)y * W * 16;

    float best = __builtin_inff();
    int arg = -1;

    for (int dc = d0; dc < d1; dc += CV_DC) {
        const int dce = min(dc + CV_DC, d1);
        const int rbase = (SIDE == SDE_SIDE_LEFT) ? q0 - (dc + CV_DC - 1) : q0 + dc;
        __syncthreads();   // previous chunk's LDS reads (win and otile) are complete
        for (int idx = threadIdx.x; idx < CV_ROWS * 16; idx += 256) {
            const int lr = idx >> 4, k = idx & 15, g = rbase + lr;
            if (g >= 0 && g < W) win[swz_row16(lr, k)] = other4[(size_t)g * 16 + k];
        }
        __syncthreads();
        const int ds = dc + wave * CV_DW;
        const int de = min(ds + CV_DW, dce);
        for (int d = ds; d < de; d++) {
            const int o = (SIDE == SDE_SIDE_LEFT) ? q - d : q + d;
            const bool valid = (SIDE == SDE_SIDE_LEFT) ? (o >= 0) : (o < W);
            float cost = invalid;
            if (qok && valid) cost = dot64_exact(own, win, o - rbase);
            if (OUT == OUT_WTA) {
                if (cost < best) { best = cost; arg = d; }
            } else if (OUT == OUT_DHW) {
                if (qok) out[((size_t)d * H + y) * W + q] = cost;
            } else {
                otile[lane * (CV_DC + 1) + (d - dc)] = cost;
            }
        }
        if (OUT == OUT_HWD) {
            __syncthreads();
            const int nd = dce - dc;
            for (int i = wave; i < CV_TX; i += CV_WAVES) {
                if (q0 + i < W && lane < nd)
                    out[((size_t)y * W + q0 + i) * Dvol + dc + lane] = otile[i * (CV_DC + 1) + lane];
            }
        }
    }

    if (OUT == OUT_WTA) {
        __shared__ float sm[CV_WAVES][CV_TX];
        __shared__ int sa[CV_WAVES][CV_TX];
        sm[wave][lane] = best;
        sa[wave][lane] = arg;
        __syncthreads();
        if (wave == 0 && qok) {
#pragma unroll
            for (int w = 1; w < CV_WAVES; w++) argmin_merge(best, arg, sm[w][lane], sa[w][lane]);
            const size_t p = (size_t)y * W + q;
            if (out_min) out_min[p] = best;
            if (out_arg) out_arg[p] = arg;
            if (out_disp) out_disp[p] = (float)arg;
        }
    }
}

// Any channel count: one lane per (pixel, d-range), features read from global
// memory, NumPy's full pairwise recursion.  Correctness path for C != 64.
template <int OUT>
__global__ __launch_bounds__(256) void cv_generic_kernel(const float *__restrict__ fl, const float *__restrict__ fr,
                                                         int H, int W, int C, int d0, int d1, int Dvol,
                                                         int sides, float invalid, float *__restrict__ outl,
                                                         float *__restrict__ outr, float *__restrict__ out_min,
                                                         int32_t *__restrict__ out_arg, float *__restrict__ out_disp)
{
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (int64_t)H * W) return;
    const int y = (int)(p / W), x = (int)(p % W);
    float best = __builtin_inff();
    int arg = -1;
    for (int d = d0; d < d1; d++) {
        float cost = invalid;
        if (x >= d) cost = np_neg_dot(fl + ((size_t)y * W + x) * C, fr + ((size_t)y * W + x - d) * C, C);
        if (OUT == OUT_WTA) {
            if (cost < best) { best = cost; arg = d; }
        } else if (OUT == OUT_DHW) {
            outl[((size_t)d * H + y) * W + x] = cost;
        } else {
            if (sides & SDE_SIDE_LEFT) outl[((size_t)y * W + x) * Dvol + d] = cost;
        }
        // right volume: R[y][x][d] = cost(x + d, d), computed by its own owner pixel x
        if (OUT == OUT_HWD && (sides & SDE_SIDE_RIGHT)) {
            float cr = invalid;
            if (x + d < W) cr = np_neg_dot(fl + ((size_t)y * W + x + d) * C, fr + ((size_t)y * W + x) * C, C);
            outr[((size_t)y * W + x) * Dvol + d] = cr;
        }
    }
    if (OUT == OUT_WTA) {
        if (out_min) out_min[p] = best;
        if (out_arg) out_arg[p] = arg;
        if (out_disp) out_disp[p] = (float)arg;
    }
}

// WTA over [D][H][W]: one lane per pixel, each d-slice read coalesced along W.
template <int RULE>
__global__ __launch_bounds__(256) void wta_dhw_kernel(const float *__restrict__ vol, int64_t npix, int D,
                                                      float *__restrict__ disp)
{
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npix) return;
    float best;
    int arg;
    if (RULE == SDE_WTA_INIT_D0) { best = vol[p]; arg = 0; }
    else { best = __builtin_inff(); arg = -1; }
    for (int d = (RULE == SDE_WTA_INIT_D0 ? 1 : 0); d < D; d++) {
        const float v = vol[(size_t)d * npix + p];
        if (v < best) { best = v; arg = d; }
    }
    disp[p] = (float)arg;
}

// WTA over [H][W][D]: 16 lanes per pixel (4 pixels per wave), each lane scans a
// strided subset in increasing d, then a (value, index) merge across the 16
// lanes reproduces the sequential scan.
template <int RULE>
__global__ __launch_bounds__(256) void wta_hwd_kernel(const float *__restrict__ vol, int64_t npix, int D,
                                                      float *__restrict__ disp)
{
    const int sub = threadIdx.x & 15;
    const int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const bool ok = p < npix;
    const float *v = vol + (size_t)(ok ? p : 0) * D;
    float best = __builtin_inff();
    int arg = -1;
    if (ok) {
        for (int d = sub; d < D; d += 16) {
            const float x = v[d];
            if (x < best) { best = x; arg = d; }
        }
    }
    // A lane with arg = -1 holds +inf; a lane with a winner holds a value < +inf,
    // so the plain (value, index) merge never lets -1 win against a real index.
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
        const float ob = __shfl_xor(best, off, 64);
        const int oa = __shfl_xor(arg, off, 64);
        argmin_merge(best, arg, ob, oa);
    }
    if (ok && sub == 0) {
        if (RULE == SDE_WTA_INIT_D0) {
            // best = v[0], `best > v[d]` (:805-811): identical to the +inf scan except that
            // "no winner" reads 0 and a NaN at d = 0 is never replaced.
            const float v0 = v[0];
            if (arg < 0 || v0 != v0) arg = 0;
        }
        disp[p] = (float)arg;
    }
}

__global__ __launch_bounds__(256) void argmin_merge_kernel(const float *__restrict__ mins,
                                                           const int32_t *__restrict__ args, int nshards,
                                                           int64_t npix, float *__restrict__ disp)
{
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npix) return;
    float best = mins[p];
    int arg = args[p];
    for (int s = 1; s < nshards; s++) {
        const float m = mins[(size_t)s * npix + p];
        const int a = args[(size_t)s * npix + p];
        if (m < best) { best = m; arg = a; }   // shards are ordered by d: ties keep the earlier one
    }
    disp[p] = (float)arg;
}

}  // namespace sde

using namespace sde;

SDE_EXPORT int sde_abi_version(void) { return SDE_ABI_VERSION; }

SDE_EXPORT const char *sde_status_string(int s)
{
    switch (s) {
    case SDE_OK: return "ok";
    case SDE_ERR_ARG: return "invalid argument";
    case SDE_ERR_LAUNCH: return "kernel launch failed";
    case SDE_ERR_WORKSPACE: return "workspace too small";
    default: return "unknown status";
    }
}

SDE_EXPORT int sde_cost_volume(const float *fl, const float *fr, int H, int W, int C, int D, int layout,
                               int sides, float invalid, float *out_left, float *out_right, void *stream)
{
    if (!fl || !fr || H <= 0 || W <= 0 || C <= 0 || D <= 0) return SDE_ERR_ARG;
    if (layout != SDE_LAYOUT_DHW && layout != SDE_LAYOUT_HWD) return SDE_ERR_ARG;
    if ((sides & ~(SDE_SIDE_LEFT | SDE_SIDE_RIGHT)) || !sides) return SDE_ERR_ARG;
    if ((sides & SDE_SIDE_LEFT) && !out_left) return SDE_ERR_ARG;
    if ((sides & SDE_SIDE_RIGHT) && !out_right) return SDE_ERR_ARG;
    if (layout == SDE_LAYOUT_DHW && (sides & SDE_SIDE_RIGHT)) return SDE_ERR_ARG;
    hipStream_t st = as_stream(stream);
    if (C == 64) {
        dim3 grid(cdiv(W, CV_TX), H);
        if (layout == SDE_LAYOUT_DHW) {
            cv64_kernel<SDE_SIDE_LEFT, OUT_DHW><<<grid, 256, 0, st>>>(fl, fr, H, W, 0, D, D, invalid, out_left,
                                                                       nullptr, nullptr, nullptr);
        } else {
            if (sides & SDE_SIDE_LEFT)
                cv64_kernel<SDE_SIDE_LEFT, OUT_HWD><<<grid, 256, 0, st>>>(fl, fr, H, W, 0, D, D, invalid,
                                                                           out_left, nullptr, nullptr, nullptr);
            if (sides & SDE_SIDE_RIGHT)
                cv64_kernel<SDE_SIDE_RIGHT, OUT_HWD><<<grid, 256, 0, st>>>(fr, fl, H, W, 0, D, D, invalid,
                                                                            out_right, nullptr, nullptr, nullptr);
        }
    } else {
        const int blocks = cdiv((int64_t)H * W, 256);
        if (layout == SDE_LAYOUT_DHW)
            cv_generic_kernel<OUT_DHW><<<blocks, 256, 0, st>>>(fl, fr, H, W, C, 0, D, D, sides, invalid, out_left,
                                                                nullptr, nullptr, nullptr, nullptr);
        else
            cv_generic_kernel<OUT_HWD><<<blocks, 256, 0, st>>>(fl, fr, H, W, C, 0, D, D, sides, invalid, out_left,
                                                                out_right, nullptr, nullptr, nullptr);
    }
    return launch_status();
}

SDE_EXPORT int sde_cv_wta(const float *fl, const float *fr, int H, int W, int C, int d0, int d1, float *disp,
                          float *min_cost, int32_t *argmin, void *stream)
{
    if (!fl || !fr || H <= 0 || W <= 0 || C <= 0 || d0 < 0 || d1 <= d0) return SDE_ERR_ARG;
    if (!disp && !min_cost && !argmin) return SDE_ERR_ARG;
    hipStream_t st = as_stream(stream);
    if (C == 64) {
        dim3 grid(cdiv(W, CV_TX), H);
        cv64_kernel<SDE_SIDE_LEFT, OUT_WTA><<<grid, 256, 0, st>>>(fl, fr, H, W, d0, d1, 0, -0.0f, nullptr,
                                                                   min_cost, argmin, disp);
    } else {
        const int blocks = cdiv((int64_t)H * W, 256);
        cv_generic_kernel<OUT_WTA><<<blocks, 256, 0, st>>>(fl, fr, H, W, C, d0, d1, 0, SDE_SIDE_LEFT, -0.0f,
                                                            nullptr, nullptr, min_cost, argmin, disp);
    }
    return launch_status();
}

SDE_EXPORT int sde_wta(const float *vol, int H, int W, int D, int layout, int rule, float *disp, void *stream)
{
    if (!vol || !disp || H <= 0 || W <= 0 || D <= 0) return SDE_ERR_ARG;
    if (rule != SDE_WTA_INIT_INF && rule != SDE_WTA_INIT_D0) return SDE_ERR_ARG;
    hipStream_t st = as_stream(stream);
    const int64_t npix = (int64_t)H * W;
    if (layout == SDE_LAYOUT_DHW) {
        const int blocks = cdiv(npix, 256);
        if (rule == SDE_WTA_INIT_INF) wta_dhw_kernel<SDE_WTA_INIT_INF><<<blocks, 256, 0, st>>>(vol, npix, D, disp);
        else wta_dhw_kernel<SDE_WTA_INIT_D0><<<blocks, 256, 0, st>>>(vol, npix, D, disp);
    } else if (layout == SDE_LAYOUT_HWD) {
        const int blocks = cdiv(npix * 16, 256);
        if (rule == SDE_WTA_INIT_INF) wta_hwd_kernel<SDE_WTA_INIT_INF><<<blocks, 256, 0, st>>>(vol, npix, D, disp);
        else wta_hwd_kernel<SDE_WTA_INIT_D0><<<blocks, 256, 0, st>>>(vol, npix, D, disp);
    } else {
        return SDE_ERR_ARG;
    }
    return launch_status();
}

SDE_EXPORT int sde_argmin_merge(const float *mins, const int32_t *args, int nshards, int64_t npix, float *disp,
                                void *stream)
{
    if (!mins || !args || !disp || nshards <= 0 || npix <= 0) return SDE_ERR_ARG;
    argmin_merge_kernel<<<cdiv(npix, 256), 256, 0, as_stream(stream)>>>(mins, args, nshards, npix, disp);
    return launch_status();
}
