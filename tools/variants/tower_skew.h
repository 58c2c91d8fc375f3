// tower_skew.h -- f16x3 64->64 conv with the two M-tiles of a tile skewed by one c-block (gfx950).
// NOT BUILT (round 4): measured slower than conv64_x6p_kernel (248-254 vs 233 us per layer-image), removed
// from libsde.so; kept under tools/variants/ as the record of the experiment.
// Included by tower.hip after conv64_x6p_kernel, whose helpers it uses (same arithmetic, same bits).
//
// In conv64_x6p_kernel one MFMA wave per SIMD owns 4 output rows x all 64 output channels; at the
// end of every tile it runs the epilogue (bias, ReLU, bound, 32 KB of stores) while its SIMD's MFMA
// pipe idles -- about a fifth of a middle layer's cycles.  Here two MFMA waves share each SIMD,
// one per M-tile (output channels 0-31 / 32-63) of the same 4 rows, and the M-tile-1 waves trail
// the M-tile-0 waves by one c-block: while one wave of a SIMD runs its epilogue, the other is in
// the middle of a c-block's MFMAs.  768 threads: waves 0-7 MFMA (wave w: rows 4 (w & 3) .., M-tile
// w >> 2), waves 8-11 stage the input exactly as in conv64_x6p_kernel.  Three stage buffers (the
// f16x3 stage is the four (part, channel-half) planes, 39 KB): in barrier phase p the M-tile-0
// waves read stage p, the M-tile-1 waves stage p-1 and the stagers write stage p+1; one more phase
// than steps lets the trailing waves finish.  Every accumulator sees the same MFMAs in the same
// order as in conv64_x6p_kernel, so the outputs are bit-identical to it.  Not for the last layer
// (its L2 norm needs a pixel's 64 channels in one wave).
#pragma once

namespace sde {

#ifndef SK_PRIO
#define SK_PRIO 2      // s_setprio of the c-block that ends a tile (0: none)
#endif
constexpr int SK_STAGE = 4 * XP_PLANE;                      // 39,168 B
constexpr size_t SK_WIN_OFF = (size_t)3 * SK_STAGE;          // FIRST: one image window per stager wave
constexpr size_t SK_BIAS_OFF = SK_WIN_OFF + 4 * XP_WIN * sizeof(float);
constexpr size_t SK_SMEM = SK_BIAS_OFF + NF * sizeof(float);  // 129,280 B

// One c-block for one MFMA wave of the skewed kernel: 9 taps x 4 output rows = 36 row-steps of one
// M-tile (3 MFMAs each, small terms first), B fragments RD-1 row-steps ahead, A fragments 2 taps ahead.
__device__ __forceinline__ void sk_cblock(floatx16 (&acc)[4], XpFrag &a, XpFrag (&an)[2], const uint4 *__restrict__ wf,
                                          int mt, int cb, int ncb, int lane, const char *sb)
{
    constexpr int WR = 4, NS = 9 * WR, NP = 2, AL = 2, RD = XP_RING_F16;
    XpB ring[RD];
    auto boff = [&](int s) { return ((s / WR / 3 + s % WR) * XP_IX + (s / WR) % 3) * 16; };
#pragma unroll
    for (int k = 0; k < RD - 1; k++) ring[k] = xp_bfrag<NP>(sb + boff(k));
#pragma unroll
    for (int s = 0; s < NS; s++) {
        const int tap = s / WR, r = s % WR;
        if (r == 0 && tap > 0) {
            a = an[0];
            an[0] = an[1];
            const int t2 = tap + AL;
            an[1] = t2 < 9 ? xp_afrag<NP>(wf, mt, cb, t2, lane) : xp_afrag<NP>(wf, mt, ncb, t2 - 9, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
        const XpB &b = ring[s % RD];
        floatx16 &c = acc[r];
        c = mfma_h(a.p[1], b.p[0], c);
        c = mfma_h(a.p[0], b.p[1], c);
        c = mfma_h(a.p[0], b.p[0], c);
        if (s + RD - 1 < NS) ring[(s + RD - 1) % RD] = xp_bfrag<NP>(sb + boff(s + RD - 1));
    }
    a = an[0];
    an[0] = an[1];
    an[1] = xp_afrag<NP>(wf, mt, ncb, AL, lane);
}

// The stagers of the skewed kernel: xp_stager_loop's pipeline over three stage buffers, plus the
// trailing phase's barrier.
template <bool FIRST, bool IN_CB>
__device__ __forceinline__ void sk_stager_loop(char *xsm, const float *__restrict__ in, int Hin, int Win,
                                               const XpBatch &bt, int st, const float *__restrict__ in_amax,
                                               const float *__restrict__ hdr, const float *__restrict__ w1blob,
                                               float *win)
{
    const int tile0 = blockIdx.x, gstride = gridDim.x;
    const int nsteps = ((bt.ntiles - 1 - tile0) / gstride + 1) * XP_NCB;
    if (FIRST) {
        int sc_img = -1;
        float s = 1.0f, unscale = 1.0f;
        constexpr int WPL = (XP_WIN + 63) / 64;
        float wv[WPL];
        const int lane = st & 63;
        auto wload = [&](int t) {
            int img, ty0, tx0;
            xp_tile(bt, t, img, ty0, tx0);
            const float *src = in + img * bt.in_stride;
#pragma unroll
            for (int k = 0; k < WPL; k++) {
                const int idx = lane + 64 * k;
                const int iy = idx / XP_WX, ix = idx - iy * XP_WX;
                const int y = ty0 + iy, x = tx0 + ix;
                wv[k] = (idx < XP_WIN && y < Hin && x < Win) ? src[(size_t)y * Win + x] : 0.0f;
            }
        };
        auto fill = [&](int i) {
            const int t = tile0 + (i / XP_NCB) * gstride, im = t / bt.tiles_img, cb = i % XP_NCB;
            if (im != sc_img) {
                xp_scales(true, in_amax + im * bt.amax_stride, hdr, s, unscale);
                sc_img = im;
            }
            if (cb == 0) {
#pragma unroll
                for (int k = 0; k < WPL; k++)
                    if (lane + 64 * k < XP_WIN) win[lane + 64 * k] = wv[k];
                __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
                __builtin_amdgcn_wave_barrier();
            }
            xp_fill<true, false, true>(xsm + (i % 3) * SK_STAGE, in, Hin, Win, w1blob, t, bt, cb, st, s, win);
            if (cb == 1 && t + gstride < bt.ntiles) wload(t + gstride);
        };
        wload(tile0);
        fill(0);
        __syncthreads();
#pragma unroll 1
        for (int i = 0; i < nsteps; i++) {
            if (i + 1 < nsteps) fill(i + 1);
            __syncthreads();
        }
        __syncthreads();   // the trailing phase
        return;
    }
    auto load = [&](float4 (&v)[XP_UPT], int i) {
        const int t = tile0 + (i / XP_NCB) * gstride, cb = i % XP_NCB;
        int img, ty0, tx0;
        xp_tile(bt, t, img, ty0, tx0);
        const float *src = in + img * bt.in_stride;
#pragma unroll
        for (int k = 0; k < XP_UPT; k++) {
            const int u = st + k * XP_STAGERS;
            v[k] = u < XP_UNITS ? xp_load<IN_CB>(src, Hin, Win, ty0, tx0, cb, u) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    int sc_img = -1;
    float s = 1.0f, unscale = 1.0f;
    auto store = [&](const float4 (&v)[XP_UPT], int i) {
        const int im = (tile0 + (i / XP_NCB) * gstride) / bt.tiles_img;
        if (im != sc_img) {
            xp_scales(false, in_amax + im * bt.amax_stride, hdr, s, unscale);
            sc_img = im;
        }
        char *sb = xsm + (i % 3) * SK_STAGE;
#pragma unroll
        for (int k = 0; k < XP_UPT; k++) {
            const int u = st + k * XP_STAGERS;
            if (u < XP_UNITS) xp_store<true>(sb, u, v[k], s);
        }
    };
    float4 ra[XP_UPT], rb[XP_UPT];
    load(ra, 0);
    store(ra, 0);
    if (nsteps > 1) load(ra, 1);
    __syncthreads();
#pragma unroll 1
    for (int i = 0; i < nsteps; i += 2) {
        if (i + 2 < nsteps) load(rb, i + 2);
        if (i + 1 < nsteps) store(ra, i + 1);
        __syncthreads();
        if (i + 1 >= nsteps) break;
        if (i + 3 < nsteps) load(ra, i + 3);
        if (i + 2 < nsteps) store(rb, i + 2);
        __syncthreads();
    }
    __syncthreads();   // the trailing phase
}

template <bool FIRST, bool IN_CB, bool OUT_CB>
__global__ __launch_bounds__(768) void conv64_skew_kernel(const float *__restrict__ in, int Hin, int Win,
                                                          const float *__restrict__ w1blob,
                                                          const float *__restrict__ wkblob, float *__restrict__ out,
                                                          int Hout, int Wout, XpBatch bt,
                                                          const float *__restrict__ in_amax, float *__restrict__ out_amax)
{
    extern __shared__ __attribute__((aligned(16))) char xsm[];
    float *win = reinterpret_cast<float *>(xsm + SK_WIN_OFF) + ((threadIdx.x >> 6) & 3) * XP_WIN;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const float *hdr = wkblob + LK_F16 + LK_W;
    if (wave >= 8) {
        if (blockIdx.x < bt.ntiles)
            sk_stager_loop<FIRST, IN_CB>(xsm, in, Hin, Win, bt, tid - 512, in_amax, hdr, w1blob, win);
        return;
    }
    int tile = blockIdx.x;
    if (tile >= bt.ntiles) return;
    const int g = __builtin_amdgcn_readfirstlane(wave & 3);     // output rows 4g .. 4g+3 of the tile
    const int mt = __builtin_amdgcn_readfirstlane(wave >> 2);   // M-tile: output channels 32 mt ..
    const float *bias = wkblob;
    const uint4 *wf = reinterpret_cast<const uint4 *>(wkblob + LK_F16);
    const int bbase = (lane >> 5) * XP_PLANE + ((4 * g) * XP_IX + (lane & 31)) * 16;
    int sc_img = -1;
    float sc_s = 1.0f, sc_u = 1.0f;
    float *lbias = reinterpret_cast<float *>(xsm + SK_BIAS_OFF);
    if (wave == 0) lbias[lane] = bias[lane];   // published by the first barrier
    const float4 *lbias4 = reinterpret_cast<const float4 *>(lbias);
    XpFrag a, an[2];
    a = xp_afrag<2>(wf, mt, 0, 0, lane);
    an[0] = xp_afrag<2>(wf, mt, 0, 1, lane);
    an[1] = xp_afrag<2>(wf, mt, 0, 2, lane);
    __syncthreads();
    if (mt == 1) __syncthreads();              // M-tile 1 trails by one phase

    uint32_t amax_run = 0u;
    int amax_img = -1;
    auto flush_amax = [&]() {
        if (amax_img < 0) return;
        uint32_t am = amax_run;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) am = max(am, (uint32_t)__shfl_xor((int)am, o, 64));
        if (lane == 0) atomicMax(reinterpret_cast<unsigned int *>(out_amax + amax_img * bt.amax_stride), am);
        amax_run = 0u;
    };
    int step = 0;
    for (; tile < bt.ntiles; tile += gridDim.x) {
        int img, ty0, tx0;
        xp_tile(bt, tile, img, ty0, tx0);
        floatx16 acc[4];
#pragma unroll
        for (int r = 0; r < 4; r++) acc[r] = floatx16{0};
#pragma unroll 1
        for (int cb = 0; cb < XP_NCB; cb++, step++) {
            const int ncb = (cb + 1) & (XP_NCB - 1);
            // the wave that ends its tile in this phase issues its MFMAs at a higher priority, so it
            // reaches its epilogue while its SIMD partner (a c-block behind) still has MFMAs to issue
            if (SK_PRIO && cb == XP_NCB - 1) __builtin_amdgcn_s_setprio(SK_PRIO);
            sk_cblock(acc, a, an, wf, mt, cb, ncb, lane, xsm + (step % 3) * SK_STAGE + bbase);
            if (SK_PRIO && cb == XP_NCB - 1) __builtin_amdgcn_s_setprio(0);
            if (cb == XP_NCB - 1) {
                // epilogue: bias + ReLU, the f16x3 bound, stores (as conv64_x6p_kernel, one M-tile)
                int j = lane & 31, h = lane >> 5;
                asm volatile("" : "+v"(j), "+v"(h));
                const int im = tile / bt.tiles_img;
                if (im != sc_img) {
                    xp_scales(FIRST, in_amax + im * bt.amax_stride, hdr, sc_s, sc_u);
                    sc_img = im;
                }
                const float unscale = sc_u;
                const int x = tx0 + j;
                const bool xok = x < Wout;
                const int row0 = 4 * g;
                uint32_t amax = 0u;
                float *const outi = out + img * bt.out_stride;
                const uint32_t vo = xok ? (uint32_t)(x * (OUT_CB ? 64 : 256) + 16 * h) : XP_OOB;
                const size_t HW = (size_t)Hout * Wout;
                float4 b4[4];
#pragma unroll
                for (int q = 0; q < 4; q++) b4[q] = lbias4[(mt * 32 + 8 * q + 4 * h) >> 2];
#pragma unroll
                for (int qh = 0; qh < 2; qh++) {
                    const int cblk = 2 * mt + qh;
                    const __amdgpu_buffer_rsrc_t rs =
                        xp_rsrc(OUT_CB ? outi + ((size_t)cblk * HW + (size_t)ty0 * Wout) * 16 : outi + (size_t)ty0 * Wout * NF);
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const floatx16 &c = acc[r];
                        if (ty0 + row0 + r < Hout) {   // wave-uniform
                            const uint32_t so = (uint32_t)((row0 + r) * Wout) * (OUT_CB ? 64u : 256u);
#pragma unroll
                            for (int ql = 0; ql < 2; ql++) {
                                const int q = 2 * qh + ql;
                                const float bq[4] = {b4[q].x, b4[q].y, b4[q].z, b4[q].w};
                                float o4[4];
#pragma unroll
                                for (int e = 0; e < 4; e++) o4[e] = fmaxf(fmaf(c[4 * q + e], unscale, bq[e]), 0.f);
                                const float4 o = make_float4(o4[0], o4[1], o4[2], o4[3]);
                                amax = max(amax, max(__float_as_uint(o.x), __float_as_uint(o.y)));
                                amax = max(amax, max(__float_as_uint(o.z), __float_as_uint(o.w)));
                                xp_st4(o, rs, vo + (OUT_CB ? 32u * ql : 4u * (mt * 32 + 8 * q)), so);
                            }
                        }
                    }
                }
                if (!xok) amax = 0u;
                if (img != amax_img) {
                    flush_amax();
                    amax_img = img;
                }
                amax_run = max(amax_run, amax);
            }
            __syncthreads();
        }
    }
    if (mt == 0) __syncthreads();              // the trailing phase (M-tile 1's last step)
    flush_amax();
}

}  // namespace sde
