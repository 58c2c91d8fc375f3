// cbca.hip -- cross-based cost aggregation on [H][W][D] volumes (gfx950).
//
// BUILD-DEFINED stage: the reference has no CBCA (only the
// buffer name d_cost_volumel_after_aggr, process_functional.py:268,347, and an
// unused timer label, match.py:98).  The definition -- cross arms on intensity
// + distance, support intersected with the other image's arms at x -/+ d,
// horizontal-then-vertical sums, mean over the support, N iterations -- is
// stated once in the CPU restatement under oracle/ (test infrastructure); these
// kernels reproduce it bit for bit (fp32 sums in ascending offset order from
// 0.0f, exact integer counts, one IEEE division).
//
// Mapping.  Both passes are line scans: one wave (one workgroup) walks one
// line -- a row for the horizontal pass, a column for the vertical one -- for
// one chunk of 64 disparities (lane = d, so each step moves one 256-B
// contiguous run of the HWD volume).  The fp64 prefix sum P of the definition
// is the wave's running state; the last 2R+2 prefixes live in a wave-private
// LDS ring, so each output is two LDS reads at per-lane offsets (its own arms)
// and one subtraction: O(1) work per voxel whatever the arm lengths.  The
// output trails the front by R positions (its right/down arm is at most R).
// Cost values and both images' arms are prefetched 8 positions ahead in a
// register ring (unconditional, clamped loads), and the support arms of the
// last R + 1 positions stay in registers for the trailing output.
#include "sde_common.h"

namespace sde {

__global__ __launch_bounds__(256) void cbca_arms_kernel(const float *__restrict__ img, int64_t pitch, int H, int W,
                                                        int L1, float tau, uint32_t *__restrict__ arms)
{
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (int64_t)H * W) return;
    const int y = (int)(p / W), x = (int)(p % W);
    const float c = img[(size_t)y * pitch + x];
    const int dys[4] = {0, 0, -1, 1}, dxs[4] = {-1, 1, 0, 0};
    uint32_t packed = 0;
#pragma unroll
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
    arms[p] = packed;
}

template <int R, bool VERT, int SIDE>
__global__ __launch_bounds__(64) void cbca_scan_kernel(const float *__restrict__ src, float *__restrict__ dst,
                                                       const uint32_t *__restrict__ ref,
                                                       const uint32_t *__restrict__ oth, int H, int W, int D)
{
    constexpr int RS = 2 * R + 2;      // prefix ring: positions [f - 2R - 1, f]; also the unroll
    constexpr int U = R + 1;           // support ring (trailing output reads the slot of f - R)
    constexpr int PF = 16;             // prefetch distance (vmcnt saturates at 63 outstanding ops)
    static_assert((RS & (RS - 1)) == 0 && RS % U == 0 && RS % PF == 0, "ring sizes");
    __shared__ double sP[RS * 64];
    __shared__ int sN[VERT ? RS * 64 : 1];
    const int lane = threadIdx.x;
    // Lanes past D work on d = D-1: they compute lane D-1's value and store it to the
    // same address, so no load, LDS access or store in the scan is predicated.
    const int d = min((int)blockIdx.x * 64 + lane, D - 1);
    const int line = blockIdx.y;
    const int len = VERT ? H : W;
    // opaque per-lane zero: keeps the (wave-uniform) reference-arm load a vector load,
    // ordered under vmcnt with the rest of the ring instead of a scalar load whose
    // out-of-order lgkmcnt (shared with the LDS ring) would serialise every step
    const int vz = __builtin_amdgcn_mbcnt_lo(0u, 0u);
    // per-position strides (elements) and per-line bases: position q of this line is
    // src/dst + cbase + q*cstride, ref + abase + q*astride, oth + abase + q*astride + o(q)
    const int cstride = VERT ? W * D : D, astride = VERT ? W : 1;
    const size_t cbase = VERT ? (size_t)line * D : (size_t)line * W * D;
    const size_t abase = VERT ? (size_t)line : (size_t)line * W;
    // vertical pass: the other pixel (line -/+ d) is fixed for the whole column
    const int ov = SIDE == SDE_SIDE_LEFT ? line - d : line + d;
    const bool vok = ov >= 0 && ov < W;
    const int ovc = (vok ? ov : 0) - line;          // offset from the reference pixel

    double P_acc = 0.0;
    int N_acc = 0;
    float cr[PF];
    uint32_t ar[PF], br[PF];
    uint32_t sup[U];    // VERT: (up | down << 8) of the last U positions; else (left | right << 8)
    auto issue = [&](int q, int slot) {
        const float *pc = src + cbase + (size_t)q * cstride;
        const uint32_t *pa = ref + abase + (size_t)q * astride;
        cr[slot] = pc[d];
        ar[slot] = pa[vz];
        int oo;
        if (VERT) {
            oo = ovc;
        } else {
            const int o = SIDE == SDE_SIDE_LEFT ? q - d : q + d;
            oo = (o < 0 ? 0 : (o >= W ? W - 1 : o)) - q;
        }
        br[slot] = pa[oo + (oth - ref)];
    };
    auto step = [&](int j, int f, bool tail) {
        const int slot = j % PF;
        const uint32_t a = ar[slot];
        uint32_t b = br[slot];
        if (VERT) {
            b = vok ? b : 0u;                       // no other pixel: support {p}
        } else {
            const int x = tail ? (f < len ? f : len - 1) : f;
            const bool ok = SIDE == SDE_SIDE_LEFT ? d <= x : d < W - x;
            b = ok ? b : 0u;
        }
        const int l = min(a & 255, b & 255), r = min((a >> 8) & 255, (b >> 8) & 255);
        // front: position f (tail positions >= len re-read the last one; never referenced)
        P_acc += (double)cr[slot];
        sP[j * 64 + lane] = P_acc;
        if (VERT) {
            N_acc += l + r + 1;
            sN[j * 64 + lane] = N_acc;
            sup[j % U] = min((a >> 16) & 255, (b >> 16) & 255) | (min(a >> 24, b >> 24) << 8);
        } else {
            sup[j % U] = (uint32_t)l | ((uint32_t)r << 8);
        }
        issue(tail ? min(f + PF, len - 1) : f + PF, slot);
        // trailing output y = f - R; its support arms from the ring slot of position y
        const int y = f - R;
        if (y >= 0 && (!tail || y < len)) {
            const uint32_t sy = sup[(j + 1) % U];
            const int lo = sy & 255, hi = sy >> 8;
            const int ib = ((j - R + hi) & (RS - 1)) * 64 + lane, ia = ((j - R - lo - 1) & (RS - 1)) * 64 + lane;
            const double pb = sP[ib], pa = sP[ia];
            float out;
            if (VERT) out = (float)((pb - pa) / (double)(sN[ib] - sN[ia]));
            else out = (float)(pb - pa);
            (dst + cbase + (size_t)y * cstride)[d] = out;
        }
    };
#pragma unroll
    for (int j = 0; j < PF; j++) issue(min(j, len - 1), j);
#pragma unroll
    for (int j = 0; j < U; j++) sup[j] = 0u;
    sP[(RS - 1) * 64 + lane] = 0.0;        // P(-1) = 0 (slot of position -1; rewritten at f = RS-1)
    if (VERT) sN[(RS - 1) * 64 + lane] = 0;
    int f0 = 0;
    // main blocks: every prefetched position is inside the line (no clamps)
    for (; f0 + RS + PF <= len; f0 += RS) {
#pragma unroll
        for (int j = 0; j < RS; j++) step(j, f0 + j, false);
    }
    for (; f0 < len + R; f0 += RS) {
#pragma unroll
        for (int j = 0; j < RS; j++) step(j, f0 + j, true);
    }
}

template <int R, int SIDE>
static void cbca_iters(float *cv, float *tmp, const uint32_t *ref, const uint32_t *oth, int H, int W, int D,
                       int iters, hipStream_t st)
{
    const int ndc = (D + 63) / 64;
    for (int it = 0; it < iters; it++) {
        cbca_scan_kernel<R, false, SIDE><<<dim3(ndc, H), 64, 0, st>>>(cv, tmp, ref, oth, H, W, D);
        cbca_scan_kernel<R, true, SIDE><<<dim3(ndc, W), 64, 0, st>>>(tmp, cv, ref, oth, H, W, D);
    }
}

}  // namespace sde

using namespace sde;

SDE_EXPORT int sde_cbca_arms(const float *img, int64_t pitch, int H, int W, int L1, float tau, uint32_t *arms,
                             void *stream)
{
    if (!img || !arms || H <= 0 || W <= 0 || pitch < W || L1 < 1 || L1 > SDE_CBCA_MAX_L1) return SDE_ERR_ARG;
    cbca_arms_kernel<<<cdiv((int64_t)H * W, 256), 256, 0, as_stream(stream)>>>(img, pitch, H, W, L1, tau, arms);
    return launch_status();
}

SDE_EXPORT int sde_cbca(float *cv, float *tmp, const uint32_t *arms_ref, const uint32_t *arms_other, int H, int W,
                        int D, int side, int L1, int iters, void *stream)
{
    if (!cv || !tmp || !arms_ref || !arms_other || H <= 0 || W <= 0 || D <= 0 || iters < 0 || L1 < 1 ||
        L1 > SDE_CBCA_MAX_L1 || (side != SDE_SIDE_LEFT && side != SDE_SIDE_RIGHT) || cv == tmp)
        return SDE_ERR_ARG;
    if (H > 65535 || W > 65535) return SDE_ERR_ARG;      // grid.y = lines
    hipStream_t st = as_stream(stream);
    if (side == SDE_SIDE_LEFT) {
        if (L1 <= 16) cbca_iters<15, SDE_SIDE_LEFT>(cv, tmp, arms_ref, arms_other, H, W, D, iters, st);
        else cbca_iters<31, SDE_SIDE_LEFT>(cv, tmp, arms_ref, arms_other, H, W, D, iters, st);
    } else {
        if (L1 <= 16) cbca_iters<15, SDE_SIDE_RIGHT>(cv, tmp, arms_ref, arms_other, H, W, D, iters, st);
        else cbca_iters<31, SDE_SIDE_RIGHT>(cv, tmp, arms_ref, arms_other, H, W, D, iters, st);
    }
    return launch_status();
}
