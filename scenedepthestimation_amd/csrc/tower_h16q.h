// tower_h16q.h -- the MC-CNN tower's middle 64 -> 64 layers (3..L-1; mc_cnn_brunch.py:31-48, conv :70-92) on
// split activations (SDE_TOWER_IN_SPLIT | SDE_TOWER_OUT_SPLIT), as a 4-wave kernel whose weights stay in
// registers (included by tower.hip after tower_h16.h; f16x3 arithmetic, v_mfma_f32_16x16x32_f16).
//
// Same arithmetic contract and tiles as conv64_h16_kernel (16 x 32 output tiles, 2 c-blocks of 32 input
// channels, the stage's 8 fp16 planes, lo*hi + hi*lo + hi*hi per product, small terms first), different
// work split.  conv64_h16_kernel's 8-wave form (4 MFMA waves over 4 output-row groups x all 64 channels,
// 4 stager waves) re-reads every A fragment from L2 for every c-block: 68 buffer loads per MFMA wave per
// c-block, queued in the same per-CU memory path as the input staging (without the
// A loads the split layer runs 9 % faster).  Here:
// * one 256-thread workgroup per CU (persistent over the batch's tiles), wave g owns output-channel
//   quarter g (16 channels) for all 16 rows x 32 columns of a tile: 16 rows x 2 halves = 32 accumulators
//   of 4 registers;
// * wave g's A fragments -- 16 output channels x 64 input channels x 9 taps x 2 parts -- are loaded once
//   (144 registers) and stay resident for the whole launch: no weight traffic in the loop;
// * with only 4 waves a wave may hold 512 registers (VGPRs + AGPRs), which is what makes that possible;
// * the stage is filled by the MFMA waves themselves with LDS-DMA (the split planes are copied, no
//   arithmetic): wave g copies planes 2g, 2g + 1 of step i + 1 (20 wave-instructions) at the start of
//   step i, and waits for them at the end of step i, before the barrier;
// * B fragments: each (tap, row, half) is read once per wave (2 ds_read_b128) and feeds that wave's 3
//   MFMAs: 576 LDS reads per wave per c-block, 2.3 MB per CU -- 67 % of the LDS's 256 B/clk over the
//   c-block's MFMA time;
// * epilogue: the lane's 4 channels 16g + 4 k4 .. + 3 of pixel (l & 15), split like h16_epilogue (lane
//   pairs swap halves, one 16-B store per lane per (row, half)), every store issued (rows / columns past
//   the output take the out-of-range offset), so the wait before the barrier can count them.
#pragma once

namespace sde {

// one step's LDS-DMA share of wave w (0..3): planes 2w, 2w + 1 of step k's stage (see h16_dma_stager_loop)
__device__ __forceinline__ void h16_dma_issue(char *hsm, const float *__restrict__ in, int Win, size_t PB,
                                              const XpBatch &bt, int tile0, int gstride, int k, int w, int lane,
                                              const uint32_t (&voff)[(XP_NPIX + 63) / 64])
{
    constexpr int ND = (XP_NPIX + 63) / 64, NLAST = XP_NPIX - 64 * (ND - 1);
    const int t = tile0 + (k >> 1) * gstride, cb = k & 1;
    int img, ty0, tx0;
    xp_tile(bt, t, img, ty0, tx0);
    const size_t org = ((size_t)ty0 * Win + tx0) * 16;
    const char *src = reinterpret_cast<const char *>(in + img * bt.in_stride) + (size_t)cb * 8 * PB + org;
    char *dst = hsm + (k & 1) * H16_STAGE;
#pragma unroll
    for (int pp = 0; pp < 2; pp++) {
        const int p = 2 * w + pp;
        const __amdgpu_buffer_rsrc_t rs = xp_rsrc_n(src + p * PB, (uint32_t)(PB - org));
        auto *lds = (__attribute__((address_space(3))) char *)(dst + p * H16_PLANE);
#pragma unroll
        for (int d = 0; d < ND - 1; d++)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, lds + d * 1024, 16, voff[d], 0, 0, 0);
        if (lane < NLAST) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, lds + (ND - 1) * 1024, 16, voff[ND - 1], 0, 0, 0);
    }
}

// the lane's per-DMA source offsets (tile-invariant)
__device__ __forceinline__ void h16_dma_offsets(int Win, int lane, uint32_t (&voff)[(XP_NPIX + 63) / 64])
{
#pragma unroll
    for (int d = 0; d < (XP_NPIX + 63) / 64; d++) {
        const int px = d * 64 + lane, iy = px / XP_IX, ix = px - iy * XP_IX;
        voff[d] = (uint32_t)((iy * Win + ix) * 16);
    }
}

// Work split (H16Q_NQ output-channel quarters x H16Q_NR rows per wave, NQ * NR = 16): NQ = 1 -- wave g owns
// quarter g, all 16 rows (each B fragment feeds 3 MFMAs, A 144 registers); NQ = 2 -- wave g owns quarters
// 2 (g & 1) + {0, 1} of rows 8 (g >> 1) .. + 7 (each B fragment feeds 6 MFMAs, half the LDS reads, but A
// takes 288 registers: 119 VGPRs spill at 512, so not built by default).
#ifndef H16Q_NQ
#define H16Q_NQ 1
#endif
constexpr int H16Q_NR = 16 / H16Q_NQ;
__device__ __forceinline__ int h16q_q0(int g) { return H16Q_NQ == 1 ? g : 2 * (g & 1); }
__device__ __forceinline__ int h16q_r0(int g) { return H16Q_NQ == 1 ? 0 : H16Q_NR * (g >> 1); }

// A fragments of wave g: [cb][tap][part][quarter], 16 B each (8 fp16 of the lane's k slots for output
// channel 16 (q0 + qq) + (l & 15)) from the F16 blob's [mtile][cblock16][tap][part][lane][8] order.
struct H16QA {
    f16x8 f[2][9][2][H16Q_NQ];
};

__device__ __forceinline__ void h16q_load_a(H16QA &a, const float *__restrict__ wkblob, int g, int lane)
{
    const __amdgpu_buffer_rsrc_t ra = xp_rsrc(wkblob + LK_F16);
    const int q0 = h16q_q0(g);
    const int ln = ((lane >> 4) & 1) * 32 + 16 * (q0 & 1) + (lane & 15);
    const uint32_t voff = (uint32_t)(((q0 >> 1) * XP_NCB + (lane >> 5)) * 18 * 64 + ln) * 16u;
#pragma unroll
    for (int cb = 0; cb < 2; cb++)
#pragma unroll
        for (int tap = 0; tap < 9; tap++)
#pragma unroll
            for (int p = 0; p < 2; p++)
#pragma unroll
                for (int qq = 0; qq < H16Q_NQ; qq++)   // quarter q0 + 1: the next 16 lanes of the M-tile
                    a.f[cb][tap][p][qq] = __builtin_bit_cast(
                        f16x8, __builtin_amdgcn_raw_buffer_load_b128(ra, voff, cb * H16_A_CB + (tap * 2 + p) * 1024 + 256 * qq, 0));
}

// B fragment of step b = (tap, row r, half ph); sb = the stage at the lane's base (plane lane >> 4, pixel
// lane & 15 of the wave's first row)
__device__ __forceinline__ H16B h16q_bfrag(const char *sb, int b)
{
    const int tap = b / (2 * H16Q_NR), r = (b >> 1) % H16Q_NR, ph = b & 1;
    const int off = ((r + tap / 3) * XP_IX + 16 * ph + tap % 3) * 16;
    H16B f;
    f.hi = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4 *>(sb + off));
    f.lo = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4 *>(sb + 4 * H16_PLANE + off));
    return f;
}

constexpr int H16Q_RD = 4;   // B ring depth

// one c-block of one wave: 9 taps x NR rows x 2 halves, 3 MFMAs per quarter each, acc[(r * 2 + ph) * NQ + qq]
template <int CB>
__device__ __forceinline__ void h16q_cblock(floatx4 (&acc)[32], const H16QA &a, const char *sb)
{
    constexpr int NB = 9 * 2 * H16Q_NR;
    H16B ring[H16Q_RD];
#pragma unroll
    for (int k = 0; k < H16Q_RD - 1; k++) ring[k] = h16q_bfrag(sb, k);
#pragma unroll
    for (int b = 0; b < NB; b++) {
        __builtin_amdgcn_sched_barrier(0);
        const int tap = b / (2 * H16Q_NR);
        const H16B &bf = ring[b % H16Q_RD];
#pragma unroll
        for (int qq = 0; qq < H16Q_NQ; qq++) {
            floatx4 &c = acc[(b % (2 * H16Q_NR)) * H16Q_NQ + qq];
            c = mfma16(a.f[CB][tap][1][qq], bf.hi, c);
            c = mfma16(a.f[CB][tap][0][qq], bf.lo, c);
            c = mfma16(a.f[CB][tap][0][qq], bf.hi, c);
        }
        if (b + H16Q_RD - 1 < NB) ring[(b + H16Q_RD - 1) % H16Q_RD] = h16q_bfrag(sb, b + H16Q_RD - 1);
    }
}

constexpr int H16Q_STORES = 32;   // epilogue stores per lane per tile (all issued)
// s_waitcnt immediate (gfx9 layout): vmcnt(n), expcnt / lgkmcnt not waited for
#define H16Q_VMCNT(n) (((n) & 15) | (((n) >> 4) << 14) | (7 << 4) | (15 << 8))

// epilogue of wave g: unscale + bias + ReLU, the bound, the split planes (see h16_epilogue's OSPL branch)
__device__ __forceinline__ void h16q_epilogue(const floatx4 (&acc)[32], int lane, int g, int img, int ty0, int tx0,
                                              float unscale, const float4 (&b4)[H16Q_NQ], float oscale,
                                              float *__restrict__ out, int Hout, int Wout, const XpBatch &bt,
                                              uint32_t &amax_run)
{
    uint32_t amax = 0u;
    int j = lane & 15, k4 = lane >> 4;
    asm volatile("" : "+v"(j), "+v"(k4));
    const size_t HW = (size_t)Hout * Wout;
    const uint32_t pb = (uint32_t)HW * 16u;
    const int q0 = h16q_q0(g), r0 = h16q_r0(g);
    // channels 16q + 4 k4 + e: 8-channel group 2q + (k4 >> 1), plane (q >> 1) * 8 + part * 4 + 2 (q & 1) + (k4 >> 1)
    const uint32_t lane_pl = (uint32_t)((k4 & 1) * 4 + (k4 >> 1)) * pb;
    char *outi = reinterpret_cast<char *>(out + img * bt.out_stride);
    u32x4 pin[32];
#pragma unroll
    for (int qq = 0; qq < H16Q_NQ; qq++) {
        const int q = q0 + qq;
        const __amdgpu_buffer_rsrc_t rs =
            xp_rsrc(outi + ((size_t)((q >> 1) * 8 + 2 * (q & 1)) * HW + (size_t)(ty0 + r0) * Wout) * 16);
        // the outputs scaled by 2^sigma straight from the accumulators (scale folded into the unscale and
        // the bias: exact), their bound unscaled at the end
        const float bq[4] = {b4[qq].x * oscale, b4[qq].y * oscale, b4[qq].z * oscale, b4[qq].w * oscale};
        const float us = unscale * oscale;
#pragma unroll
        for (int r = 0; r < H16Q_NR; r++) {
            const bool rok = ty0 + r0 + r < Hout;
            const uint32_t so = (uint32_t)(r * Wout) * 16u;
#pragma unroll
            for (int ph = 0; ph < 2; ph++) {
                const int x = tx0 + 16 * ph + j;
                const bool ok = rok && x < Wout;
                const floatx4 &c = acc[(r * 2 + ph) * H16Q_NQ + qq];
                float o4[4];
#pragma unroll
                for (int e = 0; e < 4; e++) o4[e] = fmaxf(fmaf(c[e], us, bq[e]), 0.f);
                const float4 o = make_float4(o4[0], o4[1], o4[2], o4[3]);
                if (ok) {   // the bound before the store: nothing writes o's registers after it
                    amax = max(amax, max(__float_as_uint(o.x), __float_as_uint(o.y)));
                    amax = max(amax, max(__float_as_uint(o.z), __float_as_uint(o.w)));
                }
                u32x2 hw2, lw2;
                xp_split16s(o, hw2, lw2);
                const int k = (qq * H16Q_NR + r) * 2 + ph;
                pin[k] = xp_pair_parts<false>(hw2, lw2);
                __builtin_amdgcn_raw_buffer_store_b128(pin[k], rs, ok ? lane_pl + (uint32_t)x * 16u : XP_OOB, so, 0);
                if (k >= XP_PIN - 1) asm volatile("" ::"v"(pin[k - (XP_PIN - 1)]));
            }
        }
    }
#pragma unroll
    for (int k = 32 - (XP_PIN - 1); k + 1 < 32; k++) asm volatile("" ::"v"(pin[k]));
    asm volatile("s_nop 4" ::"v"(pin[31]));
    // the bound of the scaled outputs, unscaled (exact: a power of two)
    amax_run = max(amax_run, __float_as_uint(__uint_as_float(amax) / oscale));
}

// Middle layers, split in and out.  wkblob: the layer's packed blob; in_amax / out_amax: the bound words
// (+ XP_SCALE_WORD: the input's / output's 2^sigma).
__global__ __launch_bounds__(256) void conv64_h16q_kernel(const float *__restrict__ in, int Hin, int Win,
                                                          const float *__restrict__ wkblob, float *__restrict__ out,
                                                          int Hout, int Wout, XpBatch bt,
                                                          const float *__restrict__ in_amax, float *__restrict__ out_amax)
{
    extern __shared__ __attribute__((aligned(16))) char hsm[];
    const int lane = threadIdx.x & 63;
    const int g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tile0 = blockIdx.x, gstride = gridDim.x;
    if (tile0 >= bt.ntiles) return;
    const int nsteps = ((bt.ntiles - 1 - tile0) / gstride + 1) * H16_NCB;
    const float *hdr = wkblob + LK_F16 + LK_W;
    xp_publish_scale(false, bt, in_amax, hdr, out_amax);

    uint32_t voff[(XP_NPIX + 63) / 64];
    h16_dma_offsets(Win, lane, voff);
    const size_t PB = (size_t)Hin * Win * 16;
    H16QA a;
    h16q_load_a(a, wkblob, g, lane);
    float4 b4[H16Q_NQ];
#pragma unroll
    for (int qq = 0; qq < H16Q_NQ; qq++)
        b4[qq] = *reinterpret_cast<const float4 *>(wkblob + 16 * (h16q_q0(g) + qq) + 4 * (lane >> 4));
    const char *bbase = hsm + (lane >> 4) * H16_PLANE + (h16q_r0(g) * XP_IX + (lane & 15)) * 16;

    h16_dma_issue(hsm, in, Win, PB, bt, tile0, gstride, 0, g, lane, voff);
    // waits as builtins, not inline asm: the compiler's own wait insertion then knows the A loads and the
    // DMAs before them have landed (it cannot read an asm's wait, and would re-wait for them in the loop)
    __builtin_amdgcn_s_waitcnt(H16Q_VMCNT(0));
    __builtin_amdgcn_s_barrier();

    int sc_img = -1;
    float sc_u = 1.0f, sc_o = 1.0f;
    uint32_t amax_run = 0u;
    int amax_img = -1;
    floatx4 acc[32];
#pragma unroll 1
    for (int i = 0; i < nsteps; i++) {
        if (i + 1 < nsteps) h16_dma_issue(hsm, in, Win, PB, bt, tile0, gstride, i + 1, g, lane, voff);
        const char *sb = bbase + (i & 1) * H16_STAGE;
        if ((i & 1) == 0) {
#pragma unroll
            for (int k = 0; k < 32; k++) acc[k] = floatx4{0.f, 0.f, 0.f, 0.f};
            h16q_cblock<0>(acc, a, sb);
            __builtin_amdgcn_s_waitcnt(H16Q_VMCNT(0));   // step i + 1's DMA
        } else {
            h16q_cblock<1>(acc, a, sb);
            int img, ty0, tx0;
            xp_tile(bt, tile0 + (i >> 1) * gstride, img, ty0, tx0);
            if (img != sc_img) {
                const float *am = in_amax + img * bt.amax_stride;
                sc_u = hdr[0] / am[XP_SCALE_WORD];   // the writer's published 2^sigma
                sc_o = xp_out_scale(false, am, hdr);
                sc_img = img;
            }
            if (img != amax_img) {
                xp_flush_amax(amax_run, amax_img, lane, out_amax, bt.amax_stride);
                amax_img = img;
            }
            h16q_epilogue(acc, lane, g, img, ty0, tx0, sc_u, b4, sc_o, out, Hout, Wout, bt, amax_run);
            // step i + 1's DMA was issued before the epilogue's H16Q_STORES stores (and at most one
            // bound atomic before them): counters retire in order, so this waits for the DMA only
            __builtin_amdgcn_s_waitcnt(H16Q_VMCNT(H16Q_STORES));
        }
        __builtin_amdgcn_s_barrier();
    }
    xp_flush_amax(amax_run, amax_img, lane, out_amax, bt.amax_stride);
}

}  // namespace sde
