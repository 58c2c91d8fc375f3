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
// Mapping.  One wave = one d-chunk of 64 disparities (lane = d, so every load
// and store is a 256-B contiguous run of the HWD row) x one segment of NO
// outputs along a line (a row for the horizontal pass, a column for the
// vertical one).  The wave loads its NO + 2R window of cost rows into
// registers once and forms every output as a masked, fixed-order sum over the
// 2R + 1 taps, so each voxel is read from HBM about once (the halo hits L2:
// the four waves of a workgroup take four consecutive segments of the same
// line, and workgroups are remapped so neighbours share an XCD).  Arms of the
// reference pixel are wave-uniform (scalar loads); the other image's arms at
// x -/+ d are one coalesced 4-B gather per window row.
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

__device__ __forceinline__ int xcd_remap_cb(int b, int nb)
{
    const int q = nb / 8, r = nb % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// Support arms (l, r, u, d packed as bytes) of voxel (y, x, d): min of the
// reference arms at x and the other image's arms at x -/+ d, or 0 outside.
__device__ __forceinline__ uint32_t support(uint32_t a, const uint32_t *__restrict__ oth, size_t rowbase, int o,
                                            int W, int R)
{
    if (o < 0 || o >= W) return 0u;
    const uint32_t b = oth[rowbase + o];
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        int u = (a >> (8 * k)) & 255, v = (b >> (8 * k)) & 255;
        u = u < v ? u : v;
        u = u < R ? u : R;
        s |= (uint32_t)u << (8 * k);
    }
    return s;
}

template <int R, int NO, bool VERT>
__global__ __launch_bounds__(256) void cbca_pass_kernel(const float *__restrict__ src, float *__restrict__ dst,
                                                        const uint32_t *__restrict__ ref,
                                                        const uint32_t *__restrict__ oth, int H, int W, int D,
                                                        int side, int nseg, int ndc)
{
    constexpr int NWIN = NO + 2 * R;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int ngrp = (nseg + 3) / 4;
    const int lb = xcd_remap_cb(blockIdx.x, gridDim.x);
    const int grp = lb % ngrp;
    const int dc = (lb / ngrp) % ndc;
    const int line = lb / (ngrp * ndc);
    const int seg = grp * 4 + wave;
    if (seg >= nseg) return;                       // wave-uniform; no barriers below
    const int d = dc * 64 + lane;
    const bool dok = d < D;
    const int dl = dok ? d : D - 1;
    const int len = VERT ? H : W;                  // positions along the line
    const int p0 = seg * NO;
    const int dsgn = side == SDE_SIDE_LEFT ? -1 : 1;

    float v[NWIN];
    uint32_t sup[VERT ? NWIN : 1];
#pragma unroll
    for (int t = 0; t < NWIN; t++) {
        int q = p0 - R + t;
        q = q < 0 ? 0 : (q >= len ? len - 1 : q);
        const int y = VERT ? q : line, x = VERT ? line : q;
        v[t] = src[((size_t)y * W + x) * D + dl];
        if (VERT) {
            const size_t rb = (size_t)y * W;
            sup[t] = support(ref[rb + x], oth, rb, x + dsgn * d, W, R);
        }
    }
#pragma unroll
    for (int o = 0; o < NO; o++) {
        const int q = p0 + o;
        if (q < len) {
            const int y = VERT ? q : line, x = VERT ? line : q;
            uint32_t s;
            if (VERT) {
                s = sup[o + R];
            } else {
                const size_t rb = (size_t)y * W;
                s = support(ref[rb + x], oth, rb, x + dsgn * d, W, R);
            }
            const int lo = VERT ? (s >> 16) & 255 : s & 255;           // up / left
            const int hi = VERT ? (s >> 24) & 255 : (s >> 8) & 255;    // down / right
            float acc = 0.0f;
            int cnt = 0;
#pragma unroll
            for (int j = -R; j <= R; j++) {
                const bool in = j < 0 ? (-j <= lo) : (j <= hi);
                acc += in ? v[o + R + j] : 0.0f;
                if (VERT) {
                    const uint32_t sj = sup[o + R + j];
                    cnt += in ? (int)((sj & 255) + ((sj >> 8) & 255) + 1) : 0;
                }
            }
            if (dok) dst[((size_t)y * W + x) * D + d] = VERT ? acc / (float)cnt : acc;
        }
    }
}

template <int R, int NO, bool VERT>
static void launch_pass(const float *src, float *dst, const uint32_t *ref, const uint32_t *oth, int H, int W, int D,
                        int side, hipStream_t st)
{
    const int nlines = VERT ? W : H;
    const int len = VERT ? H : W;
    const int nseg = (len + NO - 1) / NO;
    const int ndc = (D + 63) / 64;
    const int64_t nblk = (int64_t)nlines * ndc * ((nseg + 3) / 4);
    cbca_pass_kernel<R, NO, VERT><<<(unsigned)nblk, 256, 0, st>>>(src, dst, ref, oth, H, W, D, side, nseg, ndc);
}

// NOH / NOV: outputs per wave of the horizontal / vertical pass (the vertical
// pass also keeps every window row's support arms, so it takes shorter segments
// to stay fully unrolled in registers).
template <int R, int NOH, int NOV>
static void cbca_iters(float *cv, float *tmp, const uint32_t *ref, const uint32_t *oth, int H, int W, int D, int side,
                       int iters, hipStream_t st)
{
    for (int it = 0; it < iters; it++) {
        launch_pass<R, NOH, false>(cv, tmp, ref, oth, H, W, D, side, st);
        launch_pass<R, NOV, true>(tmp, cv, ref, oth, H, W, D, side, st);
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
    if ((int64_t)H * W * ((D + 63) / 64) > ((int64_t)1 << 31) * 16) return SDE_ERR_ARG;
    hipStream_t st = as_stream(stream);
    if (L1 <= 16) cbca_iters<15, 32, 16>(cv, tmp, arms_ref, arms_other, H, W, D, side, iters, st);
    else cbca_iters<31, 16, 8>(cv, tmp, arms_ref, arms_other, H, W, D, side, iters, st);
    return launch_status();
}
