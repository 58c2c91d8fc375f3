// cv_cert.h -- shared pieces of the certified fused cost volume + WTA (cost_volume.hip, cv_row.hip).
//
// Scores s(x,d) = fl[x] . fr[x-d] on the bf16 MFMA with every fp32 operand split
// into hi + lo bf16 parts; see cost_volume.hip for the error bound (FX_K) that
// certifies a fast argmax as the exact first-min.
#pragma once

#include "sde_common.h"

namespace sde {

typedef __bf16 fx_bf16x8 __attribute__((ext_vector_type(8)));
typedef float fx_floatx16 __attribute__((ext_vector_type(16)));

constexpr int FX_NX = 64;          // left pixels per workgroup
constexpr int FX_DCH = 128;        // disparities per window chunk
constexpr int FX_NT = 6;           // max M-tiles per chunk: ceil((128 + 63) / 32)
constexpr int FX_WIN = FX_NT * 32; // window pixels
constexpr float FX_K = 1e-4f;
constexpr float FX_ABS = 1e-30f;   // absolute slack (bf16 subnormal handling)

// Exact NumPy-order cost of two 64-float rows in global memory (16-B loads).
__device__ __forceinline__ float dot64_exact_global(const float4 *__restrict__ a, const float4 *__restrict__ b)
{
    float acc[8];
#pragma unroll
    for (int m = 0; m < 8; m++) {
        const float4 a0 = a[2 * m], a1 = a[2 * m + 1], b0 = b[2 * m], b1 = b[2 * m + 1];
        const float p[8] = {a0.x * b0.x, a0.y * b0.y, a0.z * b0.z, a0.w * b0.w,
                            a1.x * b1.x, a1.y * b1.y, a1.z * b1.z, a1.w * b1.w};
#pragma unroll
        for (int jj = 0; jj < 8; jj++) acc[jj] = (m == 0) ? p[jj] : acc[jj] + p[jj];
    }
    const float res = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    return -(0.0f + res);
}

// the same bits with at most two 32-byte steps of loads in flight (for kernels at tight VGPR budgets)
__device__ __forceinline__ float dot64_exact_global_lean(const float4 *__restrict__ a, const float4 *__restrict__ b)
{
    float acc[8];
    {
        const float4 a0 = a[0], a1 = a[1], b0 = b[0], b1 = b[1];
        acc[0] = a0.x * b0.x; acc[1] = a0.y * b0.y; acc[2] = a0.z * b0.z; acc[3] = a0.w * b0.w;
        acc[4] = a1.x * b1.x; acc[5] = a1.y * b1.y; acc[6] = a1.z * b1.z; acc[7] = a1.w * b1.w;
    }
#pragma unroll 1
    for (int m = 1; m < 8; m++) {
        const float4 a0 = a[2 * m], a1 = a[2 * m + 1], b0 = b[2 * m], b1 = b[2 * m + 1];
        const float p[8] = {a0.x * b0.x, a0.y * b0.y, a0.z * b0.z, a0.w * b0.w,
                            a1.x * b1.x, a1.y * b1.y, a1.z * b1.z, a1.w * b1.w};
#pragma unroll
        for (int jj = 0; jj < 8; jj++) acc[jj] = acc[jj] + p[jj];
    }
    const float res = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    return -(0.0f + res);
}

__device__ __forceinline__ int fx_slot(int r, int c8) { return r * 8 + (c8 ^ ((r >> 1) & 7)); }

__device__ __forceinline__ void fx_split(float x, __bf16 &h, __bf16 &l)
{
    h = (__bf16)x;
    l = (__bf16)(x - (float)h);
}

// merge (best, arg, second) of two disjoint candidate sets, scores in max-domain
__device__ __forceinline__ void fx_merge(float &b, int &a, float &s, float b2, int a2, float s2)
{
    const float ns = fmaxf(fminf(b, b2), fmaxf(s, s2));
    if (b2 > b || (b2 == b && a2 < a)) { b = b2; a = a2; }
    s = ns;
}

__device__ __forceinline__ int xcd_remap(int b, int nb)
{
    // bijective: blocks b, b+8, ... (one XCD under round-robin dispatch) get consecutive logical ids
    const int q = nb / 8, r = nb % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

constexpr float FX_NORM_UP = 1.000004f;

// the row-sweep kernel (cv_row.hip): window size limit and launcher
bool row_cert_supported(int d0, int d1);
void launch_row_cert(const float *fl, const float *fr, int H, int W, int d0, int d1, float *out_min, int32_t *out_arg,
                     float *out_disp, unsigned *counter, int32_t *list, hipStream_t st, const float *prev_min = nullptr);

}  // namespace sde
