// sgm.hip -- semi-global matching and the GPU path's post-processing (gfx950).
//
// Replaces (process_functional.py):
//   sgm_penelty_kernel                :134-262
//   SGM_Interation + 8 SGM_*_kernel   :265-797  (launch order :1166-1203)
//   is_error_match_kernel / LRC_kernel :977-1088
//   Median_Filter_kernel               :840-879
//
// SGM recurrence, exactly as the reference computes it (Numba unifies the 1.0
// initialisers with the f32 loads, so the path state is float64):
//   L(p,d) = C(p,d)                                            first pixel / wrap restart
//   L(p,d) = C(p,d) + (min(L'(d), L'(d-1)+P1, L'(d+1)+P1, m'+P2') - m')   otherwise
//   S(p,d) = f32(f64(S(p,d)) + L(p,d));   m = min_d L(p,d)
// with P1 from the previous pixel's penalty channel, P2' read at the previous
// step, out-of-range neighbours (d = 0, D-1) dropped, n-1 pixels per line of n
// (>= 2), and diagonal lines wrapping around the image with a path restart.
//
// Mapping: one wave64 per scanline; lane l owns DPL = ceil(D/64) consecutive
// disparities (d = l*DPL + i) in registers, so d-1 / d+1 cross a lane boundary
// only at i = 0 / DPL-1 (one 64-bit shuffle each) and min_d is a 6-level xor
// butterfly.  The scanline's per-pixel loads (C and S, DPL floats per lane;
// the two penalties, wave-uniform) are prefetched PF steps ahead in a register
// ring so HBM latency overlaps the sequential DP.
#include "sde_common.h"

namespace sde {

// direction table in the reference launch order: step (dr, dc) and P1 channel
__constant__ int c_dir_dr[8] = {+1, -1, 0, 0, +1, -1, +1, -1};
__constant__ int c_dir_dc[8] = {0, 0, +1, -1, +1, +1, -1, -1};
__constant__ int c_dir_ch[8] = {2, 0, 6, 4, 10, 12, 8, 14};

struct PathGeom {
    int dir, dr, dc, ch, H, W, n;
};

// k-th pixel of scanline `line`; restart = first pixel or diagonal wrap.
__device__ __forceinline__ void path_pixel(const PathGeom &g, int line, int k, int &r, int &c, bool &restart)
{
    restart = (k == 0);
    if (g.dc == 0) {                       // vertical: line = column
        c = line;
        r = g.dr > 0 ? k : g.H - 1 - k;
    } else if (g.dr == 0) {                // horizontal: line = row
        r = line;
        c = g.dc > 0 ? k : g.W - 1 - k;
    } else {                               // diagonal: line = start column, wraps
        r = g.dr > 0 ? k : g.H - 1 - k;
        if (g.dc > 0) {
            c = (int)(((int64_t)line + k) % g.W);
            if (k > 0 && c == 0) restart = true;
        } else {
            int64_t cc = ((int64_t)line - k) % g.W;
            if (cc < 0) cc += g.W;
            c = (int)cc;
            if (k > 0 && c == g.W - 1) restart = true;
        }
    }
}

template <int DPL>
struct Slot {
    float cst[DPL];
    float s[DPL];
    double p1, p2;
    size_t off;     // voxel offset of (r, c, d = 0)
    bool restart;
};

template <int DPL>
__device__ __forceinline__ void issue(const PathGeom &g, int line, int k, const float *__restrict__ cv,
                                      const float *__restrict__ pen, const float *__restrict__ S, int D,
                                      int dbase, Slot<DPL> &sl)
{
    int r, c;
    bool restart;
    path_pixel(g, line, k, r, c, restart);
    sl.restart = restart;
    sl.off = ((size_t)r * g.W + c) * D;
    const int pr = r - g.dr, pc = c - g.dc;
    double p1 = 0.0;
    if (!restart && pr >= 0 && pr < g.H && pc >= 0 && pc < g.W) p1 = (double)pen[((size_t)pr * g.W + pc) * 16 + g.ch];
    sl.p1 = p1;
    sl.p2 = (double)pen[((size_t)r * g.W + c) * 16 + g.ch + 1];
#pragma unroll
    for (int i = 0; i < DPL; i++) {
        const int d = dbase + i;
        sl.cst[i] = d < D ? cv[sl.off + d] : 0.0f;
        sl.s[i] = d < D ? S[sl.off + d] : 0.0f;
    }
}

template <int DPL, int PF>
__global__ __launch_bounds__(256) void sgm_dir_kernel(const float *__restrict__ cv, const float *__restrict__ pen,
                                                      int H, int W, int D, int dir, float *__restrict__ S)
{
    PathGeom g;
    g.dir = dir; g.dr = c_dir_dr[dir]; g.dc = c_dir_dc[dir]; g.ch = c_dir_ch[dir];
    g.H = H; g.W = W;
    const int nlen = (g.dc != 0 && g.dr == 0) ? W : H;
    g.n = nlen - 1 > 2 ? nlen - 1 : 2;
    const int nlines = (g.dc != 0 && g.dr == 0) ? H : W;
    const int lane = threadIdx.x & 63;
    const int line = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (line >= nlines) return;            // whole wave leaves together
    const int dbase = lane * DPL;
    const double INF = __builtin_inf();

    Slot<DPL> ring[PF];
#pragma unroll
    for (int j = 0; j < PF; j++)
        if (j < g.n) issue<DPL>(g, line, j, cv, pen, S, D, dbase, ring[j]);

    double L[DPL];
    double m = 1.0, mP2 = 1.0;
#pragma unroll
    for (int i = 0; i < DPL; i++) L[i] = 1.0;

    for (int k0 = 0; k0 < g.n; k0 += PF) {
#pragma unroll
        for (int j = 0; j < PF; j++) {
            const int k = k0 + j;
            if (k >= g.n) break;
            Slot<DPL> &sl = ring[j];
            double Ln[DPL];
            if (sl.restart) {
#pragma unroll
                for (int i = 0; i < DPL; i++) Ln[i] = (double)sl.cst[i];
            } else {
                const double lo = __shfl_up(L[DPL - 1], 1, 64);     // L'(dbase - 1)
                const double hi = __shfl_down(L[0], 1, 64);         // L'(dbase + DPL)
#pragma unroll
                for (int i = 0; i < DPL; i++) {
                    const int d = dbase + i;
                    double b = L[i];
                    const double left = i > 0 ? L[i - 1] : lo;
                    const double right = i < DPL - 1 ? L[i + 1] : hi;
                    if (d > 0) { const double t = left + sl.p1; b = t < b ? t : b; }
                    if (d < D - 1) { const double t = right + sl.p1; b = t < b ? t : b; }
                    b = mP2 < b ? mP2 : b;
                    Ln[i] = (double)sl.cst[i] + (b - m);
                }
            }
#pragma unroll
            for (int i = 0; i < DPL; i++) {
                const int d = dbase + i;
                if (d < D) S[sl.off + d] = (float)((double)sl.s[i] + Ln[i]);
            }
            if (k < g.n - 1) {
                double mm = INF;
#pragma unroll
                for (int i = 0; i < DPL; i++)
                    if (dbase + i < D) mm = Ln[i] < mm ? Ln[i] : mm;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const double t = __shfl_xor(mm, o, 64);
                    mm = t < mm ? t : mm;
                }
                m = mm;
                mP2 = mm + sl.p2;
            }
            const double p2_unused = sl.p2;
            (void)p2_unused;
#pragma unroll
            for (int i = 0; i < DPL; i++) L[i] = Ln[i];
            if (k + PF < g.n) issue<DPL>(g, line, k + PF, cv, pen, S, D, dbase, ring[j]);
        }
    }
}

template <int DPL>
static void launch_dir(const float *cv, const float *pen, int H, int W, int D, int dir, float *S, hipStream_t st)
{
    const bool horiz = (dir == 2 || dir == 3);
    const int nlines = horiz ? H : W;
    sgm_dir_kernel<DPL, 8><<<cdiv(nlines, 4), 256, 0, st>>>(cv, pen, H, W, D, dir, S);
}

static int sgm_direction_impl(const float *cv, const float *pen, int H, int W, int D, int dir, float *S,
                              hipStream_t st)
{
    const int dpl = (D + 63) / 64;
    switch (dpl) {
    case 1: launch_dir<1>(cv, pen, H, W, D, dir, S, st); break;
    case 2: launch_dir<2>(cv, pen, H, W, D, dir, S, st); break;
    case 3: launch_dir<3>(cv, pen, H, W, D, dir, S, st); break;
    case 4: launch_dir<4>(cv, pen, H, W, D, dir, S, st); break;
    case 5: launch_dir<5>(cv, pen, H, W, D, dir, S, st); break;
    case 6: launch_dir<6>(cv, pen, H, W, D, dir, S, st); break;
    case 7: launch_dir<7>(cv, pen, H, W, D, dir, S, st); break;
    case 8: launch_dir<8>(cv, pen, H, W, D, dir, S, st); break;
    default: return SDE_ERR_ARG;
    }
    return SDE_OK;
}

// sgm_penelty_kernel: reduced (P1/lambda, P2/lambda) iff uint64(nb - c) > thr as
// float64, i.e. nb < c or nb > c + thr; channels 0/1 never written (stay 0).
__global__ __launch_bounds__(256) void sgm_penalty_kernel(const uint8_t *__restrict__ img, int H, int W, float fP1,
                                                          float fP2, float rP1, float rP2, double thr,
                                                          float *__restrict__ pen)
{
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (int64_t)H * W) return;
    const int y = (int)(p / W), x = (int)(p % W);
    const uint64_t c = img[p];
    const int dys[8] = {-1, +1, 0, 0, +1, +1, -1, -1};
    const int dxs[8] = {0, 0, -1, +1, -1, +1, +1, -1};
    const int chs[8] = {2, 2, 4, 6, 8, 10, 12, 14};
    float o[16];
    o[0] = 0.0f;
    o[1] = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int yy = y + dys[k], xx = x + dxs[k];
        float a = fP1, b = fP2;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
            const uint64_t diff = (uint64_t)img[(size_t)yy * W + xx] - c;
            if ((double)diff > thr) { a = rP1; b = rP2; }
        }
        o[chs[k]] = a;
        o[chs[k] + 1] = b;
    }
    float4 *dst = reinterpret_cast<float4 *>(pen + p * 16);
#pragma unroll
    for (int i = 0; i < 4; i++) dst[i] = make_float4(o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]);
}

__device__ __forceinline__ int u8cast(double v) { return (int)((long long)v & 255); }

__global__ __launch_bounds__(256) void lr_check_kernel(const float *__restrict__ dl, const float *__restrict__ dr,
                                                       int H, int W, uint8_t *__restrict__ lrcl,
                                                       uint8_t *__restrict__ lrcr)
{
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (int64_t)H * W) return;
    const int y = (int)(p / W), x = (int)(p % W);
    const double ld = dl[p];
    const double rd = (double)x - ld;
    if (rd >= 0) {
        const double mn = ld - (double)dr[(size_t)y * W + u8cast(rd)];
        lrcl[p] = (mn > 1 || mn < -1) ? 1 : 0;
    }
    const double rd2 = dr[p];
    const double ld2 = (double)x + rd2;
    if (ld2 < W) {
        const double mn = rd2 - (double)dl[(size_t)y * W + u8cast(ld2)];
        lrcr[p] = (mn > 1 || mn < -1) ? 1 : 0;
    }
}

__global__ __launch_bounds__(256) void lrc_fill_kernel(const float *__restrict__ dl, const uint8_t *__restrict__ f,
                                                       int H, int W, float *__restrict__ out)
{
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (int64_t)H * W) return;
    const int y = (int)(p / W), x = (int)(p % W);
    if (f[p] != 1) { out[p] = dl[p]; return; }
    int number = 0;
    double sum = 0.0;
    int iy = y;
    while (iy >= 0 && f[(size_t)iy * W + x] == 1) iy--;
    if (iy >= 0) { number++; sum += dl[(size_t)iy * W + x]; }
    iy = y;
    while (iy < H && f[(size_t)iy * W + x] == 1) iy++;
    if (iy < H) { number++; sum += dl[(size_t)iy * W + x]; }
    int ix = x;
    while (ix < W && f[(size_t)y * W + ix] == 1) ix++;
    if (ix < W) { number++; sum += dl[(size_t)y * W + ix]; }
    ix = x;
    while (ix >= 0 && f[(size_t)y * W + ix] == 1) ix--;
    if (ix >= 0) { number++; sum += dl[(size_t)y * W + ix]; }
    out[p] = number > 0 ? (float)(sum / number) : dl[p];
}

__global__ __launch_bounds__(256) void median5_kernel(const float *__restrict__ src, int H, int W,
                                                      float *__restrict__ dst)
{
    const int x = blockIdx.x * 16 + (threadIdx.x & 15) + 2;
    const int y = blockIdx.y * 16 + (threadIdx.x >> 4) + 2;
    if (y + 2 >= H || x + 2 >= W) return;
    float w[25];
#pragma unroll
    for (int i = -2; i <= 2; i++)
#pragma unroll
        for (int j = -2; j <= 2; j++) w[(i + 2) * 5 + j + 2] = src[(size_t)(y + i) * W + x + j];
    float cur = 0.0f;
    // partial selection sort to the 13th smallest, same swaps as the reference
    for (int i = 0; i < 13; i++) {
        cur = w[i];
        int ci = i;
        for (int j = i + 1; j < 25; j++)
            if (cur > w[j]) { cur = w[j]; ci = j; }
        w[ci] = w[i];
    }
    dst[(size_t)y * W + x] = cur;
}

}  // namespace sde

using namespace sde;

SDE_EXPORT int sde_sgm_penalties(const uint8_t *img, int H, int W, double P1, double P2, int64_t threshold,
                                 double lambda, float *pen, void *stream)
{
    if (!img || !pen || H <= 0 || W <= 0 || lambda == 0.0) return SDE_ERR_ARG;
    const int64_t n = (int64_t)H * W;
    sgm_penalty_kernel<<<cdiv(n, 256), 256, 0, as_stream(stream)>>>(img, H, W, (float)P1, (float)P2,
                                                                     (float)(P1 / lambda), (float)(P2 / lambda),
                                                                     (double)threshold, pen);
    return launch_status();
}

SDE_EXPORT int sde_sgm_direction(const float *cv, const float *pen, int H, int W, int D, int direction, float *S,
                                 void *stream)
{
    if (!cv || !pen || !S || H < 2 || W < 2 || D <= 0 || D > 512 || direction < 0 || direction > 7)
        return SDE_ERR_ARG;
    const int s = sgm_direction_impl(cv, pen, H, W, D, direction, S, as_stream(stream));
    if (s != SDE_OK) return s;
    return launch_status();
}

SDE_EXPORT int sde_sgm_8path(const float *cv, const float *pen, int H, int W, int D, float *S, void *stream)
{
    if (!cv || !pen || !S || H < 2 || W < 2 || D <= 0 || D > 512) return SDE_ERR_ARG;
    for (int dir = 0; dir < 8; dir++) {
        const int s = sgm_direction_impl(cv, pen, H, W, D, dir, S, as_stream(stream));
        if (s != SDE_OK) return s;
    }
    return launch_status();
}

SDE_EXPORT int sde_lr_check(const float *disp_l, const float *disp_r, int H, int W, uint8_t *lrc_l, uint8_t *lrc_r,
                            void *stream)
{
    if (!disp_l || !disp_r || !lrc_l || !lrc_r || H <= 0 || W <= 0) return SDE_ERR_ARG;
    lr_check_kernel<<<cdiv((int64_t)H * W, 256), 256, 0, as_stream(stream)>>>(disp_l, disp_r, H, W, lrc_l, lrc_r);
    return launch_status();
}

SDE_EXPORT int sde_lrc_fill(const float *disp_l, const uint8_t *lrc_l, int H, int W, float *out, void *stream)
{
    if (!disp_l || !lrc_l || !out || H <= 0 || W <= 0) return SDE_ERR_ARG;
    lrc_fill_kernel<<<cdiv((int64_t)H * W, 256), 256, 0, as_stream(stream)>>>(disp_l, lrc_l, H, W, out);
    return launch_status();
}

SDE_EXPORT int sde_median5(const float *src, int H, int W, float *dst, void *stream)
{
    if (!src || !dst || H <= 0 || W <= 0) return SDE_ERR_ARG;
    if (H < 5 || W < 5) return SDE_OK;   // no interior pixel
    dim3 grid(cdiv(W - 4, 16), cdiv(H - 4, 16));
    median5_kernel<<<grid, 256, 0, as_stream(stream)>>>(src, H, W, dst);
    return launch_status();
}
