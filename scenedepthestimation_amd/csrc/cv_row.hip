// cv_row.hip -- row-sweep certified fused cost volume + WTA (north-star kernel).
//
// Replaces (WHDY/SceneDepthEstimation) compute_cost_volume + WTA1,
// process_functional.py:48-73 + 96-113, fused: the disparity map is bit-identical
// to WTA1(compute_cost_volume(fl, fr, D)) (see cv_cert.h / cost_volume.hip for the
// certificate).  Built with -fno-honor-nans -mno-amdgpu-ieee (see _build.py): the
// per-score max / median / compare run without NaN canonicalisation, so every
// decision that must survive non-finite input is taken on integer bit tests.
#include "cv_cert.h"

#include <algorithm>
#include <type_traits>

namespace sde {

// ---------------------------------------------------------------------------
// Row-sweep certified CV + WTA on fp32 features (cv_wta_row_kernel).
//
// One 512-thread workgroup per image row walks the row in 256-pixel superstrips;
// wave w owns the 32 left pixels [256k + 32w, +32) (one MFMA N-tile) and sweeps
// every right tile of its disparity band itself, so a pixel's best / runner-up /
// argmin never leave the wave (no cross-wave merge).  The right-feature window of
// a superstrip (256 + D - 1 pixels, in 32-pixel tiles) lives in an LDS ring of
// hi/lo bf16 planes; advancing one superstrip retires 8 tiles and admits 8, so
// every right pixel is read from HBM once per row (the chunked kernel above
// re-stages ~5x the window).  New tiles are loaded one superstrip ahead into
// registers, then split into hi/lo (and their pixel norms and per-tile norm
// maximum computed) by the threads that loaded them: no pre-split pass -- the
// kernel's only HBM input is the two fp32 feature maps (the algorithmic minimum).
// Left operands are prefetched one superstrip ahead and split in registers.
// 12 MFMAs per 32x32 tile pair, then the certificate of cv_wta_cert_kernel: a
// pixel whose best fast score beats the runner-up by more than 2 eps gets its
// exact cost recomputed from the fp32 rows (L2-resident) when requested, the rest
// go to the fix-up list.  Outputs are bit-identical to the exact kernel.  Tiles
// left of the image are zero-filled, so an invalid voxel (x < d) scores exactly
// +0 = -(-0.0), like the CPU path.
// ---------------------------------------------------------------------------
// Arithmetic of the fast scores (unlike the chunked kernels of cost_volume.hip, which use bf16
// hi/lo): every operand is scaled by 2^RW_S (exact) and split into two fp16 parts, x*2^S = h + l
// + r; the three partial products run on v_mfma_f32_32x32x16_f16, the eight small-term MFMAs
// (l*h', h*l') of a tile before the four leading ones (h*h').  Bound per voxel (a = fl[x],
// b = fr[x-d], Cauchy-Schwarz as in cost_volume.hip):
//   split: |r| <= 2^-22 |x| 2^S (fp16 11-bit parts) and the dropped l*l' <= 2^-22 |ab| 2^2S
//          -> 3.001 * 2^-22 * sum|ab|                                         (7.2e-7)
//   accumulation, the conservative per-add model of cost_volume.hip (2^-23 of the running
//   sum per product): 128 small-term adds on partial sums <= 2.002 * 2^-11 sum|ab|, then 64
//   leading adds on partial sums <= 1.002 sum|ab|  -> (64 * 1.002 + 0.13) * 2^-23  (7.7e-6)
//   NumPy pairwise order of the exact cost: 10 * 2^-24                        (6.0e-7)
//   -> |s_fast - s_exact| <= RW_K * ||a|| ||b||, RW_K = 1.5e-5 (1.67x margin over 9.0e-6),
// plus 2^-30 (||a|| + ||b||) for parts that fall into fp16's subnormal range (absolute error
// 2^-25 per scaled element, 64 elements).  A pixel is certified only when its norm and the
// window's largest norm are below 2^(15-S) - 1: no part can overflow fp16.
constexpr int RW_S = 8;
constexpr float RW_SCALE = 256.0f;                 // 2^RW_S
constexpr float RW_K = 1.5e-5f;
constexpr float RW_ABS = 9.3132257e-10f;           // 2^-30
constexpr float RW_NMAX = 127.0f;                  // norm limit: 127 * 2^8 < 65504
typedef _Float16 rw_f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void rw_split(float x, _Float16 &h, _Float16 &l)
{
    const float xs = x * RW_SCALE;
    h = (_Float16)xs;
    l = (_Float16)(xs - (float)h);
}

constexpr int RW_T = 32;           // pixels per tile (= one MFMA N-tile of left pixels)
constexpr int RW_WAVES = 8;
constexpr int RW_NX = RW_T * RW_WAVES;   // left pixels per superstrip (256)
constexpr int RW_NEW = RW_NX / RW_T;     // tiles admitted per superstrip (8)

__device__ __forceinline__ int rw_slot(int T, int nt) { return ((T % nt) + nt) % nt; }

// one 16-B unit (pixel u>>4, channels 4(u&15)..+3) of right tile T (zero outside the row)
__device__ __forceinline__ float4 rw_load(const float *__restrict__ frrow, int W, int T, int u)
{
    const int xr = T * RW_T + (u >> 4);
    const bool ok = xr >= 0 && xr < W;
    const float4 v = reinterpret_cast<const float4 *>(frrow)[(size_t)(ok ? xr : 0) * 16 + (u & 15)];
    return ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
}

template <int CTRL>
__device__ __forceinline__ float rw_dpp(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

__device__ __forceinline__ bool rw_nonfinite(float x) { return (__float_as_uint(x) & 0x7f800000u) == 0x7f800000u; }

// split one unit into the ring slot's hi/lo planes; the pixel's 16 lanes reduce its squared norm
// and the tile's 32 pixels (512 units = 8 waves x 64 lanes -> 4 pixels per wave) its maximum
// (tmax) and whether any channel is non-finite (tbad).  Integer tests: this file is built with
// relaxed NaN handling, which may not be trusted to keep float NaN tests.
__device__ __forceinline__ void rw_store(uint4 *ring, unsigned *tmax, unsigned *tbad, int slot, int u, float4 v)
{
    const int px = u >> 4, q = u & 15;
    _Float16 h0, h1, h2, h3, l0, l1, l2, l3;
    rw_split(v.x, h0, l0); rw_split(v.y, h1, l1); rw_split(v.z, h2, l2); rw_split(v.w, h3, l3);
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    const h4 hv = {h0, h1, h2, h3}, lv = {l0, l1, l2, l3};
    char *base = reinterpret_cast<char *>(ring + slot * 512 + fx_slot(px, q >> 1)) + 8 * (q & 1);
    *reinterpret_cast<uint2 *>(base) = __builtin_bit_cast(uint2, hv);
    *reinterpret_cast<uint2 *>(base + 256 * 16) = __builtin_bit_cast(uint2, lv);
    // the pixel's 16 lanes sum their squares by DPP (no LDS round trips): lane ^ 1, lane ^ 2, then the
    // other quad of the 8 and the other 8 of the row by mirrors -- the partial sums are uniform
    // within each quad / 8 by then, so every add is the xor-butterfly's add (same bits)
    float ss = v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    ss += rw_dpp<0xB1>(ss);     // quad_perm [1,0,3,2]
    ss += rw_dpp<0x4E>(ss);     // quad_perm [2,3,0,1]
    ss += rw_dpp<0x141>(ss);    // row_half_mirror
    ss += rw_dpp<0x140>(ss);    // row_mirror
    // squared norms are non-negative: their bit patterns order like unsigned integers; one LDS
    // max per pixel (lane 16k) instead of a cross-row shuffle reduction
    const bool bad = rw_nonfinite(v.x) || rw_nonfinite(v.y) || rw_nonfinite(v.z) || rw_nonfinite(v.w);
    const uint64_t anybad = __ballot(bad);
    if ((threadIdx.x & 15) == 0) atomicMax(&tmax[slot], __float_as_uint(ss));
    if ((threadIdx.x & 63) == 0 && anybad) atomicOr(&tbad[slot], 1u);
}

template <bool WANT_MIN>
__global__ __launch_bounds__(512) void cv_wta_row_kernel(const float *__restrict__ fl, const float *__restrict__ fr,
                                                         int H, int W, int d0, int d1, int tlo0, int ntw,
                                                         float *__restrict__ out_min, int32_t *__restrict__ out_arg,
                                                         float *__restrict__ out_disp, unsigned *__restrict__ counter,
                                                         int32_t *__restrict__ list)
{
    extern __shared__ __attribute__((aligned(16))) uint4 rsm[];
    uint4 *ring = rsm;                                              // [ntw][2 planes][32 px][8 chunks]
    unsigned *tmax = reinterpret_cast<unsigned *>(ring + ntw * 512); // [ntw] max squared pixel norm (f32 bits)
    unsigned *tbad = tmax + ntw;                                    // [ntw] any non-finite channel

    const int y = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: tile loop runs on SALU
    const int j = lane & 31, h = lane >> 5;
    const float *flrow = fl + (size_t)y * W * 64;
    const float *frrow = fr + (size_t)y * W * 64;
    const size_t rowpix = (size_t)y * W;
    const int nss = (W + RW_NX - 1) / RW_NX;

    // prologue: the first superstrip's window
    for (int i = tid; i < ntw; i += 512) { tmax[i] = 0u; tbad[i] = 0u; }
    __syncthreads();
    {
        // all loads in flight before the first store (a load -> store chain per tile would serialise
        // ntw HBM latencies)
        constexpr int MAXT = 18;
        float4 pv[MAXT];
#pragma unroll
        for (int t = 0; t < MAXT; t++)
            if (t < ntw) pv[t] = rw_load(frrow, W, tlo0 + t, tid);
#pragma unroll
        for (int t = 0; t < MAXT; t++)
            if (t < ntw) rw_store(ring, tmax, tbad, rw_slot(tlo0 + t, ntw), tid, pv[t]);
    }
    // left operand (raw fp32: channels 16s+8h..+7 of pixel x), prefetched one superstrip ahead
    float4 lraw[8];
    auto load_left = [&](int kk) {
        const int xx = kk * RW_NX + RW_T * wave + j;
        const float4 *src = reinterpret_cast<const float4 *>(flrow) + (size_t)(xx < W ? xx : 0) * 16 + 2 * h;
#pragma unroll
        for (int s = 0; s < 4; s++) { lraw[2 * s] = src[4 * s]; lraw[2 * s + 1] = src[4 * s + 1]; }
    };
    load_left(0);
    __syncthreads();

    for (int k = 0; k < nss; k++) {
        const int tlo = tlo0 + RW_NEW * k;
        const bool more = k + 1 < nss;
        // the next superstrip's 8 new tiles: loaded now, stored after this superstrip's reads
        float4 nv[RW_NEW];
#pragma unroll
        for (int t = 0; t < RW_NEW; t++)
            nv[t] = more ? rw_load(frrow, W, tlo + ntw + t, tid) : make_float4(0.f, 0.f, 0.f, 0.f);

        const int xb = k * RW_NX + RW_T * wave;
        const int x = xb + j;
        const bool xok = x < W;
        float best = -__builtin_inff(), second = -__builtin_inff();
        int arg = -1;
        float nl = 0.0f;
        unsigned nmax2 = 0u, wbad = 0u;     // window: max squared norm (bits), any non-finite tile
        bool lbad = false;
        if (xb < W) {          // wave-uniform: waves past the row end only help with the ring
            rw_f16x8 bh[4], bl[4];
            float ssl = 0.0f;
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const float4 a = lraw[2 * s], b = lraw[2 * s + 1];
                const float v8[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
                for (int e = 0; e < 8; e++) {
                    _Float16 hh, ll;
                    rw_split(v8[e], hh, ll);
                    bh[s][e] = hh;
                    bl[s][e] = ll;
                    ssl += v8[e] * v8[e];
                    lbad |= rw_nonfinite(v8[e]);
                }
            }
            ssl += __shfl_xor(ssl, 32, 64);
            lbad |= __shfl_xor((int)lbad, 32, 64) != 0;
            nl = sqrtf(ssl) * FX_NORM_UP;
            if (more) load_left(k + 1);

            float b1[4], b2[4];
            int ag[4];
#pragma unroll
            for (int t = 0; t < 4; t++) { b1[t] = -__builtin_inff(); b2[t] = -__builtin_inff(); ag[t] = -1; }
            // right tiles of this N-tile's band: d = x - xr in [d0, d1)
            // right pixels xr in [xb - d1 + 1, xb + 31 - d0]: tiles floor(./32) (offset keeps it non-negative)
            const int Ta = (xb - d1 + 1 + RW_T * 4096) / RW_T - 4096;
            const int Tb = (xb + 31 - d0 + RW_T * 4096) / RW_T - 4096;
            const int T0 = max(Ta, tlo), T1 = min(Tb, tlo + ntw - 1);
            int slot = rw_slot(T0, ntw);                   // advanced incrementally (no division per tile)
            for (int T = T0; T <= T1; T++, slot = (slot + 1 == ntw) ? 0 : slot + 1) {
                const int dt = xb - RW_T * T;
                const int dlo = dt - 31, dhi = dt + 31;
                if (dhi < d0 || dlo >= d1) continue;     // wave-uniform
                nmax2 = max(nmax2, tmax[slot]);
                wbad |= tbad[slot];
                const uint4 *tp = ring + slot * 512;
                fx_floatx16 acc = {0};
                rw_f16x8 ah[4], al[4];
#pragma unroll
                for (int s = 0; s < 4; s++) {
                    const int sl = fx_slot(j, 2 * s + h);
                    ah[s] = __builtin_bit_cast(rw_f16x8, tp[sl]);
                    al[s] = __builtin_bit_cast(rw_f16x8, tp[256 + sl]);
                }
                // the small terms first, then the leading products (the order the bound assumes)
#pragma unroll
                for (int s = 0; s < 4; s++) {
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[s], bh[s], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[s], bl[s], acc, 0, 0, 0);
                }
#pragma unroll
                for (int s = 0; s < 4; s++) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[s], bh[s], acc, 0, 0, 0);
                const int dl = dt + j - 4 * h;             // d of register r is dl - ((r&3) + 8(r>>2))
                if (dlo >= d0 && dhi < d1) {
#pragma unroll
                    for (int r = 0; r < 16; r++) {
                        const int t = r & 3;
                        const int d = dl - ((r & 3) + 8 * (r >> 2));
                        const float sc = acc[r];
                        const bool gt = sc > b1[t];
                        ag[t] = gt ? d : ag[t];
                        b2[t] = __builtin_amdgcn_fmed3f(b1[t], b2[t], sc);
                        b1[t] = fmaxf(b1[t], sc);
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 16; r++) {
                        const int t = r & 3;
                        const int d = dl - ((r & 3) + 8 * (r >> 2));
                        const float sc = (d >= d0 && d < d1) ? acc[r] : -__builtin_inff();
                        const bool gt = sc > b1[t];
                        ag[t] = gt ? d : ag[t];
                        b2[t] = __builtin_amdgcn_fmed3f(b1[t], b2[t], sc);
                        b1[t] = fmaxf(b1[t], sc);
                    }
                }
            }
            best = b1[0]; second = b2[0]; arg = ag[0];
#pragma unroll
            for (int t = 1; t < 4; t++) fx_merge(best, arg, second, b1[t], ag[t], b2[t]);
            {
                const float bb = __shfl_xor(best, 32, 64), ss2 = __shfl_xor(second, 32, 64);
                const int aa = __shfl_xor(arg, 32, 64);
                fx_merge(best, arg, second, bb, aa, ss2);
            }
        }
        __syncthreads();       // every wave is done reading the retiring tiles
        if (more) {
            for (int t = tid; t < RW_NEW; t += 512) {
                tmax[rw_slot(tlo + ntw + t, ntw)] = 0u;
                tbad[rw_slot(tlo + ntw + t, ntw)] = 0u;
            }
            __syncthreads();
#pragma unroll
            for (int t = 0; t < RW_NEW; t++) rw_store(ring, tmax, tbad, rw_slot(tlo + ntw + t, ntw), tid, nv[t]);
        }
        // certificate and outputs (off the ring: overlaps the stores)
        if (xb < W && h == 0 && xok) {
            // scores are scaled by 2^2S (exact): compare against the scaled bound
            const float nr = sqrtf(__uint_as_float(nmax2)) * FX_NORM_UP;
            const float eps = (RW_K * nl * nr + RW_ABS * (nl + nr) + FX_ABS) * (RW_SCALE * RW_SCALE);
            const size_t p = rowpix + x;
            // certified only when every operand is finite and no fp16 part can overflow (then
            // every score and eps are finite too)
            // x < d0: no voxel of the band is inside the image -- every cost is the -0.0 fill, so the scan's
            // first minimum is d0 whatever the features hold (the chunked path's later chunks: x < 256 k)
            const bool none = x < d0;
            if (none || (!lbad && !wbad && nl < RW_NMAX && nr < RW_NMAX && (best - second) > 2.0f * eps && arg >= 0)) {
                if (none) arg = d0;
                if (WANT_MIN) {
                    float cost = -0.0f;
                    if (x - arg >= 0)
                        cost = dot64_exact_global(reinterpret_cast<const float4 *>(flrow + (size_t)x * 64),
                                                  reinterpret_cast<const float4 *>(frrow + (size_t)(x - arg) * 64));
                    out_min[p] = cost;
                }
                if (out_arg) out_arg[p] = arg;
                if (out_disp) out_disp[p] = (float)arg;
            } else {
                // near-ties and non-finite operands: the IEEE fix-up kernel's exact scan
                list[atomicAdd(counter, 1u)] = (int32_t)p;
            }
        }
        __syncthreads();
    }

}

// ---------------------------------------------------------------------------
// Warp-specialised row sweep (cv_wta_row2_kernel) -- the default.
//
// In cv_wta_row_kernel all eight waves stage the window's new tiles (split, norms, ring writes)
// and then all compute, in lock-step barrier phases around one 8-wave workgroup per CU (PMC:
// waves parked 38 % of their cycles, MFMA pipe ~10 % busy).  Here the roles are split: waves
// 0-3 compute (each owns 32 left pixels of a 128-pixel superstrip: left split, 12 MFMAs per
// right tile of its band, the certificate -- the same arithmetic and bound as above), waves 4-7
// stage: each admits one 32-pixel right tile per superstrip (fp32 loads issued a superstrip
// ahead, split into the ring's hi / lo planes, the tile's max squared norm and non-finite flag
// as whole-wave reductions, no atomics).  One barrier per superstrip: while the compute waves
// read window k, the stagers write window k+1's four new tiles into the slots of the tiles
// superstrip k-1 retired (ring = window + 4 tiles: 14 at D = 192, 112 KB).
// ---------------------------------------------------------------------------
constexpr int R2_NX = 128;                 // left pixels per superstrip (4 compute waves x 32)
#ifndef CV_FASTSPLIT
#define CV_FASTSPLIT 63                    // bits: 1 paired split, 2 norm-based flag, 4 swap merges, 8 norm total by shuffle,
                                           // 16 the stagers' flag from the pixel norm, 32 the stagers' paired split
                                           // (A/B builds)
#endif
constexpr int R2_NEW = R2_NX / RW_T;       // tiles admitted per superstrip (4)
#ifndef CV_LEAD
#define CV_LEAD 2                          // scores issued before the next tile's first MFMA (A/B builds: 2..8)
#endif

// one stager lane's 8 units (pixel u >> 4, channels 4 (u & 15) ..) of right tile T: unit u = lane + 64 i
__device__ __forceinline__ void r2_load(const float *__restrict__ frrow, int W, int T, int lane, float4 (&v)[8])
{
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = rw_load(frrow, W, T, lane + 64 * i);
}

// split a loaded tile into ring slot `slot`; its max squared pixel norm and non-finite flag
__device__ __forceinline__ void r2_store(uint4 *ring, unsigned *tmax, unsigned *tbad, int slot, int lane,
                                         const float4 (&v)[8])
{
    unsigned mx = 0u;
    bool bad = false;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int u = lane + 64 * i, px = u >> 4, q = u & 15;
        char *base = reinterpret_cast<char *>(ring + slot * 512 + fx_slot(px, q >> 1)) + 8 * (q & 1);
#if CV_FASTSPLIT & 32
        // rw_split's parts as the compute waves' left split: hi of a scaled pair by one packed convert, lo by
        // v_fma_mix{lo,hi} from it (x 2^S - hi exact in fp32: the same bits)
        const float xs[4] = {v[i].x * RW_SCALE, v[i].y * RW_SCALE, v[i].z * RW_SCALE, v[i].w * RW_SCALE};
        typedef _Float16 h2 __attribute__((ext_vector_type(2)));
        uint32_t hw[2], lw[2];
#pragma unroll
        for (int e = 0; e < 2; e++) {
            const h2 hh = {(_Float16)xs[2 * e], (_Float16)xs[2 * e + 1]};
            hw[e] = __builtin_bit_cast(uint32_t, hh);
            asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=&v"(lw[e]) : "v"(xs[2 * e]), "v"(hw[e]));
            asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(lw[e]) : "v"(xs[2 * e + 1]), "v"(hw[e]));
        }
        *reinterpret_cast<uint2 *>(base) = uint2{hw[0], hw[1]};
        *reinterpret_cast<uint2 *>(base + 256 * 16) = uint2{lw[0], lw[1]};
#else
        _Float16 h0, h1, h2, h3, l0, l1, l2, l3;
        rw_split(v[i].x, h0, l0); rw_split(v[i].y, h1, l1); rw_split(v[i].z, h2, l2); rw_split(v[i].w, h3, l3);
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        const h4 hv = {h0, h1, h2, h3}, lv = {l0, l1, l2, l3};
        *reinterpret_cast<uint2 *>(base) = __builtin_bit_cast(uint2, hv);
        *reinterpret_cast<uint2 *>(base + 256 * 16) = __builtin_bit_cast(uint2, lv);
#endif
        // the pixel's squared norm: its 16 lanes are one DPP row (same adds as rw_store)
        float ss = v[i].x * v[i].x + v[i].y * v[i].y + v[i].z * v[i].z + v[i].w * v[i].w;
        ss += rw_dpp<0xB1>(ss);
        ss += rw_dpp<0x4E>(ss);
        ss += rw_dpp<0x141>(ss);
        ss += rw_dpp<0x140>(ss);
        mx = max(mx, __float_as_uint(ss));          // non-negative: bit patterns order as unsigned
#if CV_FASTSPLIT & 16
        // a non-finite channel makes the pixel's sum of squares non-finite: one test per pixel (the norm
        // bound then fails the certificate as well: NaN / inf bits order above every finite square)
        bad |= rw_nonfinite(ss);
#else
        bad |= rw_nonfinite(v[i].x) || rw_nonfinite(v[i].y) || rw_nonfinite(v[i].z) || rw_nonfinite(v[i].w);
#endif
    }
    // whole-wave maximum (every lane holds its rows' pixel norms) and any-non-finite
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) mx = max(mx, (unsigned)__shfl_xor((int)mx, o, 64));
    const bool anybad = __ballot(bad) != 0;
    if (lane == 0) {
        tmax[slot] = mx;
        tbad[slot] = anybad ? 1u : 0u;
    }
}

// prev_min (chunked path, chunks after the first): the previous chunk's exact first-minimum cost per pixel.  A pixel
// whose every exact score here is provably below -prev_min (best fast score + eps, with a factor 2 for the add's
// rounding) has every cost above the previous chunk's minimum, so this chunk cannot win the in-order merge: it
// writes (+inf, -1) and skips the certificate and the fix-up.
template <bool WANT_MIN>
__global__ __launch_bounds__(512) void cv_wta_row2_kernel(const float *__restrict__ fl, const float *__restrict__ fr,
                                                          int H, int W, int d0, int d1, int tlo0, int nw, int nt,
                                                          float *__restrict__ out_min, int32_t *__restrict__ out_arg,
                                                          float *__restrict__ out_disp, unsigned *__restrict__ counter,
                                                          int32_t *__restrict__ list, const float *__restrict__ prev_min)
{
    extern __shared__ __attribute__((aligned(16))) uint4 rsm2[];
    uint4 *ring = rsm2;                                             // [nt][2 planes][32 px][8 chunks]
    unsigned *tmax = reinterpret_cast<unsigned *>(ring + nt * 512);  // [nt] max squared pixel norm (f32 bits)
    unsigned *tbad = tmax + nt;                                     // [nt] any non-finite channel
    const int y = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & 31, h = lane >> 5;
    const float *flrow = fl + (size_t)y * W * 64;
    const float *frrow = fr + (size_t)y * W * 64;
    const size_t rowpix = (size_t)y * W;
    const int nss = (W + R2_NX - 1) / R2_NX;
    auto slot_of = [&](int T) { int r = T % nt; return r < 0 ? r + nt : r; };

    if (wave >= 4) {
        // ---------------- stagers ----------------
        const int sw = wave - 4;
        // window 0 (nw tiles, tile tlo0 + t by wave t % 4) and this wave's tile of window 1
        // (nw <= 14: at most 4 prologue tiles per stager, all in flight together)
        constexpr int PB = 4;                          // tiles per batch
        float4 nv[8];
#pragma unroll
        for (int b = 0; b < 4 / PB; b++) {
            float4 pv[PB][8];
#pragma unroll
            for (int i = 0; i < PB; i++)
                if (sw + 4 * (PB * b + i) < nw) r2_load(frrow, W, tlo0 + sw + 4 * (PB * b + i), lane, pv[i]);
            if (b == 4 / PB - 1 && nss > 1) r2_load(frrow, W, tlo0 + nw + sw, lane, nv);
#pragma unroll
            for (int i = 0; i < PB; i++)
                if (sw + 4 * (PB * b + i) < nw) r2_store(ring, tmax, tbad, slot_of(tlo0 + sw + 4 * (PB * b + i)), lane, pv[i]);
        }
        __syncthreads();
        for (int k = 0; k < nss; k++) {
            // window k+1's new tile (loaded a superstrip ago) into the slot superstrip k-1 retired,
            // then the load of window k+2's
            if (k + 1 < nss) {
                const int T = tlo0 + R2_NEW * (k + 1) + nw - R2_NEW + sw;
                r2_store(ring, tmax, tbad, slot_of(T), lane, nv);
                if (k + 2 < nss) r2_load(frrow, W, T + R2_NEW, lane, nv);
            }
            __syncthreads();
        }
        return;
    }

    // ---------------- compute waves ----------------
    const int grp = wave & 3;                       // pixel group
    float4 lraw[8];
    auto load_left = [&](int kk) {
        const int xx = kk * R2_NX + RW_T * grp + j;
        const float4 *src = reinterpret_cast<const float4 *>(flrow) + (size_t)(xx < W ? xx : 0) * 16 + 2 * h;
#pragma unroll
        for (int s2 = 0; s2 < 4; s2++) { lraw[2 * s2] = src[4 * s2]; lraw[2 * s2 + 1] = src[4 * s2 + 1]; }
    };
    load_left(0);
    __syncthreads();

    for (int k = 0; k < nss; k++) {
        const int tlo = tlo0 + R2_NEW * k;
        const bool more = k + 1 < nss;
        const int xb = k * R2_NX + RW_T * grp;
        const int x = xb + j;
        const bool xok = x < W;
        float best = -__builtin_inff(), second = -__builtin_inff();
        float wcost = -0.0f;   // WANT_MIN: the winner's exact cost (computed before the barrier)
        int arg = -1;
        float nl = 0.0f;
        unsigned nmax2 = 0u, wbad = 0u;
        bool lbad = false;
        if (xb < W && xb + RW_T - 1 < d0) {
            // every pixel of the group is left of d0: no voxel of the band is in the image (the chunked path's
            // later chunks, disparity shards past the first); the certificate's `none` case writes (-0.0, d0)
            if (more) load_left(k + 1);
        } else if (xb < W) {   // wave-uniform
            rw_f16x8 bh[4], bl[4];
            float ssl = 0.0f;
#if CV_FASTSPLIT & 1
            // rw_split's parts two values at a time: hi by one packed convert of the scaled pair, lo =
            // f16(x 2^S - hi) by v_fma_mix{lo,hi} (x 2^S exact, x 2^S - hi exact in fp32: the same bits)
            const float scl = RW_SCALE;
#pragma unroll
            for (int s2 = 0; s2 < 4; s2++) {
                const float4 a = lraw[2 * s2], b = lraw[2 * s2 + 1];
                const float v8[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
                uint32_t hw[4], lw[4];
#pragma unroll
                for (int e = 0; e < 8; e += 2) {
                    const float x0 = v8[e] * scl, x1 = v8[e + 1] * scl;
                    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
                    const h2 hh = {(_Float16)x0, (_Float16)x1};
                    const uint32_t hv = __builtin_bit_cast(uint32_t, hh);
                    uint32_t lv;
                    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=&v"(lv) : "v"(x0), "v"(hv));
                    asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(lv) : "v"(x1), "v"(hv));
                    hw[e / 2] = hv;
                    lw[e / 2] = lv;
                    ssl += v8[e] * v8[e];
                    ssl += v8[e + 1] * v8[e + 1];
                }
                bh[s2] = __builtin_bit_cast(rw_f16x8, uint4{hw[0], hw[1], hw[2], hw[3]});
                bl[s2] = __builtin_bit_cast(rw_f16x8, uint4{lw[0], lw[1], lw[2], lw[3]});
            }
#else
#pragma unroll
            for (int s2 = 0; s2 < 4; s2++) {
                const float4 a = lraw[2 * s2], b = lraw[2 * s2 + 1];
                const float v8[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
                for (int e = 0; e < 8; e++) {
                    _Float16 hh, ll;
                    rw_split(v8[e], hh, ll);
                    bh[s2][e] = hh;
                    bl[s2][e] = ll;
                    ssl += v8[e] * v8[e];
                    if (!(CV_FASTSPLIT & 2)) lbad |= rw_nonfinite(v8[e]);
                }
            }
#endif
#if CV_FASTSPLIT & 2
            // a non-finite channel makes the sum of squares non-finite (an overflowing sum of finite squares
            // is flagged too: that pixel goes to the exact fix-up, same outputs).  The other half's partial
            // sum by the LDS shuffle (bit 8): with a permlane32 swap here the build's fix-up counts moved
            // (693 -> 709 at 512 x 2048, same maps) -- the swap's result in lanes 0-31 was not the other
            // half's sum in that schedule, so the norm bound would be wrong; not used
#if CV_FASTSPLIT & 8
            ssl += __shfl_xor(ssl, 32, 64);
#else
            ssl += __builtin_bit_cast(float, __builtin_amdgcn_permlane32_swap(__float_as_uint(ssl), __float_as_uint(ssl),
                                                                              false, false)[1]);
#endif
            lbad = rw_nonfinite(ssl);
#else
            ssl += __shfl_xor(ssl, 32, 64);
            lbad |= __shfl_xor((int)lbad, 32, 64) != 0;
#endif
            nl = sqrtf(ssl) * FX_NORM_UP;
            if (more) load_left(k + 1);

            float b1[4], b2[4];
            int ag[4];
#pragma unroll
            for (int t = 0; t < 4; t++) { b1[t] = -__builtin_inff(); b2[t] = -__builtin_inff(); ag[t] = -1; }
            const int Ta = (xb - d1 + 1 + RW_T * 4096) / RW_T - 4096;
            const int Tb = (xb + 31 - d0 + RW_T * 4096) / RW_T - 4096;
            const int T0 = max(Ta, tlo), T1 = min(Tb, tlo + nw - 1);
            int slot = slot_of(T0);
            {
                // software-pipelined sweep: tile i's 16 scores are interleaved with the 12 MFMAs of
                // tile i + 1 (after two scores that cover the fragment reads' LDS latency: one MFMA,
                // then the VALU of 1-2 scores, per gap -- the MFMA pipe runs while the scores issue).
                // Same scores, same order of score updates: the same outputs.
                // (every T in [T0, T1] is inside the band: Ta / Tb are its exact bounds)
                const int n = T1 - T0 + 1;
                // PD = 1: a tile's fragments are read at the start of the step before its MFMAs (PD = 2,
                // a whole step earlier in two fragment buffers, spilled and measured slower, round 3)
                constexpr int PD = 1;
                rw_f16x8 fh[PD][4], fo[PD][4];
                fx_floatx16 A[2];
                auto nxt = [&](int sl2) { return sl2 + 1 == nt ? 0 : sl2 + 1; };
                auto frag = [&](int sl2, rw_f16x8 (&ah)[4], rw_f16x8 (&al)[4]) {
                    const uint4 *tp = ring + sl2 * 512;
#pragma unroll
                    for (int s2 = 0; s2 < 4; s2++) {
                        const int sl = fx_slot(j, 2 * s2 + h);
                        ah[s2] = __builtin_bit_cast(rw_f16x8, tp[sl]);
                        al[s2] = __builtin_bit_cast(rw_f16x8, tp[256 + sl]);
                    }
                };
                // MFMA m (0..11) of a tile: the small terms first, then the leading products
                auto mfma = [&](int m, fx_floatx16 &acc, const rw_f16x8 (&ah)[4], const rw_f16x8 (&al)[4]) {
                    if (m == 0) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[0], bh[0], fx_floatx16{0}, 0, 0, 0);
                    else if (m < 8) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16((m & 1) ? ah[m >> 1] : al[m >> 1],
                                                                                (m & 1) ? bl[m >> 1] : bh[m >> 1],
                                                                                acc, 0, 0, 0);
                    else acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[m - 8], bh[m - 8], acc, 0, 0, 0);
                };
                // MODE 0: a full tile (every voxel in [d0, d1)); 1: only d < d1 can fail (d = dk - tt < d1 <=>
                // dk < d1 + tt: one compare against a per-tt scalar); 3: only d >= d0 can fail (dk >= d0 + tt);
                // 2: both
                auto score1 = [&](const fx_floatx16 &acc, int r, auto mode_c, const int (&dk)[4]) {
                    constexpr int MODE = decltype(mode_c)::value;
                    const int tt = r & 3;
                    const bool in = MODE == 0   ? true
                                    : MODE == 1 ? dk[r >> 2] < d1 + tt
                                    : MODE == 3 ? dk[r >> 2] >= d0 + tt
                                                : (dk[r >> 2] - tt) >= d0 && (dk[r >> 2] - tt) < d1;
                    const float sc = in ? acc[r] : -__builtin_inff();
                    const bool gt = sc > b1[tt];
                    ag[tt] = gt ? dk[r >> 2] : ag[tt];
                    b2[tt] = __builtin_amdgcn_fmed3f(b1[tt], b2[tt], sc);
                    b1[tt] = fmaxf(b1[tt], sc);
                };
                // scores of tile T (accumulators acc, ring slot sl2) interleaved with the MFMAs of the
                // next tile (slot nsl; fragments fb, read now when PD = 1) into accn; PD = 2: the
                // fragments of the tile after it (slot lsl) are read into lb first
                auto step = [&](auto issue_c, auto load_c, int T, int sl2, const fx_floatx16 &acc, int nsl,
                                fx_floatx16 &accn, rw_f16x8 (&fbh)[4], rw_f16x8 (&fbl)[4], int lsl,
                                rw_f16x8 (&lbh)[4], rw_f16x8 (&lbl)[4]) {
                    constexpr bool issue = decltype(issue_c)::value, load = decltype(load_c)::value;
                    if (PD == 1 && issue) frag(nsl, fbh, fbl);
                    if (PD == 2 && load) frag(lsl, lbh, lbl);
                    nmax2 = max(nmax2, tmax[sl2]);
                    wbad |= tbad[sl2];
                    const int dt = xb - RW_T * T;
                    const bool lowok = dt - 31 >= d0, highok = dt + 31 < d1;   // wave-uniform
                    const int dl = dt + j - 4 * h;
                    int dk[4];
#pragma unroll
                    for (int k2 = 0; k2 < 4; k2++) dk[k2] = dl - 8 * k2;
                    // CV_LEAD scores before the next tile's first MFMA (they cover its fragments' LDS reads), the
                    // other 16 - CV_LEAD spread over the 12 MFMA gaps
                    constexpr int LD = CV_LEAD, RS = 16 - CV_LEAD;
                    auto body = [&](auto mode_c) {
#pragma unroll
                        for (int r = 0; r < LD; r++) score1(acc, r, mode_c, dk);
#pragma unroll
                        for (int m = 0; m < 12; m++) {
                            if (issue) mfma(m, accn, fbh, fbl);
#pragma unroll
                            for (int r = LD + (RS * m) / 12; r < LD + (RS * (m + 1)) / 12; r++)
                                score1(acc, r, mode_c, dk);
                        }
                    };
                    if (lowok && highok) {
                        asm volatile("");
                        body(std::integral_constant<int, 0>{});
                    } else if (!WANT_MIN && lowok) {   // (WANT_MIN: the two extra bodies spill there)
                        body(std::integral_constant<int, 1>{});
                    } else if (!WANT_MIN && highok) {
                        body(std::integral_constant<int, 3>{});
                    } else {
                        body(std::integral_constant<int, 2>{});
                    }
                };
                if (n > 0) {
                    using yes = std::integral_constant<bool, true>;
                    using no = std::integral_constant<bool, false>;
                    constexpr int B1 = PD - 1;                 // the buffer of odd tiles
                    int sa = slot;                              // slot of tile T0 + i2
                    frag(sa, fh[0], fo[0]);
                    if (PD == 2 && n > 1) frag(nxt(sa), fh[B1], fo[B1]);
#pragma unroll
                    for (int m = 0; m < 12; m++) mfma(m, A[0], fh[0], fo[0]);
                    int i2 = 0;
                    for (; i2 + 3 < n; i2 += 2) {              // two tiles per trip: static buffers
                        const int sb = nxt(sa), sc2 = nxt(sb), sd = nxt(sc2);
                        step(yes{}, yes{}, T0 + i2, sa, A[0], sb, A[1], fh[B1], fo[B1], sc2, fh[0], fo[0]);
                        step(yes{}, yes{}, T0 + i2 + 1, sb, A[1], sc2, A[0], fh[0], fo[0], sd, fh[B1], fo[B1]);
                        sa = sc2;
                    }
                    // the last 1-3 tiles
                    const int sb = nxt(sa), sc2 = nxt(sb);
                    if (i2 + 2 < n) {
                        step(yes{}, yes{}, T0 + i2, sa, A[0], sb, A[1], fh[B1], fo[B1], sc2, fh[0], fo[0]);
                        step(yes{}, no{}, T0 + i2 + 1, sb, A[1], sc2, A[0], fh[0], fo[0], sc2, fh[B1], fo[B1]);
                        step(no{}, no{}, T0 + i2 + 2, sc2, A[0], sc2, A[1], fh[B1], fo[B1], sc2, fh[0], fo[0]);
                    } else if (i2 + 1 < n) {
                        step(yes{}, no{}, T0 + i2, sa, A[0], sb, A[1], fh[B1], fo[B1], sb, fh[0], fo[0]);
                        step(no{}, no{}, T0 + i2 + 1, sb, A[1], sb, A[0], fh[0], fo[0], sb, fh[B1], fo[B1]);
                    } else {
                        step(no{}, no{}, T0 + i2, sa, A[0], sa, A[1], fh[B1], fo[B1], sa, fh[0], fo[0]);
                    }
                }
            }
            // a chain that took a score holds d + t >= t >= 0; one that took none still holds -1
#pragma unroll
            for (int t = 0; t < 4; t++) ag[t] = ag[t] >= 0 ? ag[t] - t : -1;
            best = b1[0]; second = b2[0]; arg = ag[0];
#pragma unroll
            for (int t = 1; t < 4; t++) fx_merge(best, arg, second, b1[t], ag[t], b2[t]);
            {
#if CV_FASTSPLIT & 4
                // lanes 0-31 (the ones that store) take the other half's triple by permlane32 swaps
                auto up = [](uint32_t v) { return __builtin_amdgcn_permlane32_swap(v, v, false, false)[1]; };
                const float bb = __uint_as_float(up(__float_as_uint(best))), ss2 = __uint_as_float(up(__float_as_uint(second)));
                const int aa = (int)up((uint32_t)arg);
#else
                const float bb = __shfl_xor(best, 32, 64), ss2 = __shfl_xor(second, 32, 64);
                const int aa = __shfl_xor(arg, 32, 64);
#endif
                fx_merge(best, arg, second, bb, aa, ss2);
            }
            if constexpr (WANT_MIN) {
                // the winner's exact cost (used if the pixel certifies), by both lane halves and issued before the
                // barrier: lane (j, h) forms dot64_exact_global's partial sums acc[4h .. 4h+3] (channels 8m + 4h ..
                // 8m + 4h + 3 = float4 2m + h of each operand, all 16 loads in flight) and its half of the final tree,
                // ((acc0 + acc1) + (acc2 + acc3)) or ((acc4 + acc5) + (acc6 + acc7)); a permlane32 swap adds the
                // halves in that order: the same bits, one round of loads instead of dot64_exact_global_lean's eight
                const uint32_t lo_arg = __builtin_amdgcn_permlane32_swap((uint32_t)arg, (uint32_t)arg, false, false)[0];
                const int ab = h ? (int)lo_arg : arg;   // the upper half takes lane j's merged arg
                const int xr = x - ab;
                const bool ok = xok && ab >= 0 && xr >= 0;
                const float4 *la = reinterpret_cast<const float4 *>(flrow + (size_t)(xok ? x : 0) * 64) + h;
                const float4 *ra = reinterpret_cast<const float4 *>(frrow + (size_t)(ok ? xr : 0) * 64) + h;
                float4 lv[8], rv[8];
#pragma unroll
                for (int m = 0; m < 8; m++) {
                    lv[m] = la[2 * m];
                    rv[m] = ra[2 * m];
                }
                float a4[4];
#pragma unroll
                for (int m = 0; m < 8; m++) {
                    const float p4[4] = {lv[m].x * rv[m].x, lv[m].y * rv[m].y, lv[m].z * rv[m].z, lv[m].w * rv[m].w};
#pragma unroll
                    for (int e = 0; e < 4; e++) a4[e] = m == 0 ? p4[e] : a4[e] + p4[e];
                }
                const float half = (a4[0] + a4[1]) + (a4[2] + a4[3]);
                const float other = __uint_as_float(
                    __builtin_amdgcn_permlane32_swap(__float_as_uint(half), __float_as_uint(half), false, false)[1]);
                wcost = -(0.0f + (half + other));   // lanes 0-31: (lower half) + (upper half)
            }
        }
        // window k+1's new tiles go into the slots superstrip k-1 read (not this window's): one
        // barrier per superstrip orders both directions
        __syncthreads();
        if (xb < W && h == 0 && xok) {
            const float nr = sqrtf(__uint_as_float(nmax2)) * FX_NORM_UP;
            const float eps = (RW_K * nl * nr + RW_ABS * (nl + nr) + FX_ABS) * (RW_SCALE * RW_SCALE);
            const size_t p = rowpix + x;
            const bool none = x < d0;   // as in cv_wta_row_kernel: every cost the -0.0 fill, first minimum d0
            const bool fin = !lbad && !wbad && nl < RW_NMAX && nr < RW_NMAX;
            if (!none && fin && WANT_MIN && prev_min && best + 2.0f * eps < -prev_min[p] * (RW_SCALE * RW_SCALE)) {
                out_min[p] = __builtin_inff();
                if (out_arg) out_arg[p] = -1;
            } else if (none || (fin && (best - second) > 2.0f * eps && arg >= 0)) {
                if (none) arg = d0;
                if (WANT_MIN) {
                    float cost = -0.0f;
                    if (x - arg >= 0) cost = wcost;
                    out_min[p] = cost;
                }
                if (out_arg) out_arg[p] = arg;
                if (out_disp) out_disp[p] = (float)arg;
            } else {
                list[atomicAdd(counter, 1u)] = (int32_t)p;
            }
        }
    }
}

// tiles spanned by a superstrip's window and the first one (superstrip 0), floor division
static void row_window(int d0, int d1, int &tlo0, int &ntw)
{
    auto fdiv = [](int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); };
    tlo0 = fdiv(-(d1 - 1), RW_T);
    const int thi0 = fdiv(RW_NX - 1 - d0, RW_T);
    ntw = thi0 - tlo0 + 1;
}

static size_t row_smem(int ntw) { return (size_t)ntw * 512 * 16 + (size_t)ntw * 8; }

// the warp-specialised kernel's window (128-pixel superstrips) and ring (window + 4 tiles)
static void row2_window(int d0, int d1, int &tlo0, int &nw)
{
    auto fdiv = [](int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); };
    tlo0 = fdiv(-(d1 - 1), RW_T);
    nw = fdiv(R2_NX - 1 - d0, RW_T) - tlo0 + 1;
}

// the ring and its per-tile words
static size_t row2_smem(int nt) { return row_smem(nt); }

static bool row2_supported(int d0, int d1)
{
    int tlo0 = 0, nw = 0;
    row2_window(d0, d1, tlo0, nw);
    return nw <= 14;                      // prologue: <= 4 tiles per stager; ring <= 18 tiles
}

bool row_cert_supported(int d0, int d1)
{
    int tlo0 = 0, ntw = 0;
    row_window(d0, d1, tlo0, ntw);
    return ntw <= 18 || row2_supported(d0, d1);
}

void launch_row_cert(const float *fl, const float *fr, int H, int W, int d0, int d1, float *out_min, int32_t *out_arg,
                     float *out_disp, unsigned *counter, int32_t *list, hipStream_t st, const float *prev_min)
{
    static std::atomic<uint64_t> attr{0};
    constexpr int NT2 = 512;
    once_per_device(attr, [] {
        (void)hipFuncSetAttribute((const void *)cv_wta_row_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  150 * 1024);
        (void)hipFuncSetAttribute((const void *)cv_wta_row_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  150 * 1024);
        (void)hipFuncSetAttribute((const void *)cv_wta_row2_kernel<true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
        (void)hipFuncSetAttribute((const void *)cv_wta_row2_kernel<false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    });
    if (row2_supported(d0, d1)) {
        int tlo0 = 0, nw = 0;
        row2_window(d0, d1, tlo0, nw);
        const int nt = nw + R2_NEW;
        if (out_min)
            cv_wta_row2_kernel<true><<<H, NT2, row2_smem(nt), st>>>(fl, fr, H, W, d0, d1, tlo0, nw, nt,
                                                                          out_min, out_arg, out_disp, counter, list,
                                                                          prev_min);
        else
            cv_wta_row2_kernel<false><<<H, NT2, row2_smem(nt), st>>>(fl, fr, H, W, d0, d1, tlo0, nw, nt,
                                                                           nullptr, out_arg, out_disp, counter, list,
                                                                           nullptr);
        return;
    }
    int tlo0 = 0, ntw = 0;
    row_window(d0, d1, tlo0, ntw);
    if (out_min)
        cv_wta_row_kernel<true><<<H, 512, row_smem(ntw), st>>>(fl, fr, H, W, d0, d1, tlo0, ntw, out_min, out_arg,
                                                               out_disp, counter, list);
    else
        cv_wta_row_kernel<false><<<H, 512, row_smem(ntw), st>>>(fl, fr, H, W, d0, d1, tlo0, ntw, nullptr, out_arg,
                                                                out_disp, counter, list);
}

}  // namespace sde
