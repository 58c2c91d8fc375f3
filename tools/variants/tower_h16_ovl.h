// PROBE COPY (tools/variants/, never built into the product): the tower header with the epilogue-overlap
// schedule (H16_OVL_K, h16_cblock_ovl, h16_store_half).  Bit-identical features; measured and not kept
// (layer 3 one image 207.7 us against 204.8 us for the product schedule; with its stores
// removed 189 us).  Build: bash tools/build_file_variant.sh tower.hip ovl \
//   -DSDE_H16_HEADER='"'$PWD/tools/variants/tower_h16_ovl.h'"'
// tower_h16.h -- the MC-CNN tower's 64 -> 64 layers (3..L; mc_cnn_brunch.py:31-48, conv :70-92) as
// a direct 3x3 implicit GEMM on v_mfma_f32_16x16x32_f16 (included by tower.hip; f16x3 arithmetic).
//
// Same arithmetic contract as conv64_x6p_kernel's F16 path: weights scaled by 2^tau on the host,
// activations by 2^sigma (from the input's bound word) on the device, each split exactly into two
// fp16 parts, the three leading partial products lo*hi + hi*lo + hi*hi accumulated in fp32 (small
// terms first), the accumulator unscaled by 2^-(tau+sigma) (exact) in the epilogue.  Why a second
// kernel: MI355X holds a lower clock under dense 32x32x16 MFMA streams than under 16x16x32 ones at
// equal cycles per FLOP (MI355X_MICROARCH.md, DVFS give-back item 7: 1.12-1.15x the FLOP/s on
// random operands), and the tower is clock-bound.
//
// Mapping (M = 64 output channels as 4 quarters of 16, N = pixels, K = 32 input channels of one
// c-block x one tap x one partial product):
// * persistent 512-thread workgroups over the batch's 16 x 32 output tiles; waves 0-3 are MFMA
//   waves (wave g owns output rows 4g .. 4g+3, all 32 columns as two 16-pixel halves, all 64
//   channels: 4 rows x 2 halves x 4 quarters = 32 accumulators of 4 VGPRs); waves 4-7 stage;
// * a tile is 2 c-blocks of 32 input channels; the stagers fill a stage of 8 planes (part 2 x
//   channel-quarter 4, 612 pixels x 8 fp16 each, planes 256-B aligned) one c-block ahead, double
//   buffered (2 x 78 KB), one barrier per c-block;
// * B fragment of (tap, row, half): lane l reads plane (part, l >> 4) at pixel (row + ky,
//   16 half + (l & 15) + kx): one conflict-free ds_read_b128, a per-lane base plus an immediate;
// * A fragments come straight from the F16 weight blob's [mtile][cblock16][tap][part][lane][8]
//   layout (no new packing): lane l of quarter q reads 16 B at a per-lane offset, from L2 -- by
//   default (h16_cblock12) a whole tap (4 quarters) one tap ahead, so each B fragment pair feeds 12
//   MFMAs; h16_cblock (H16_B12=0, and the last layer with split outputs) works in half-taps
//   (2 quarters each, 6 MFMAs per B pair) requested two half-taps ahead;
// * layer 2 (FIRST): the stagers compute conv1 from the tile's image window in LDS;
// * epilogue: a lane holds channels 16q + 4(l >> 4) .. +3 of pixel (l & 15): one dwordx4 store
//   per (row, half, quarter); the c-block-major output [cblk16][h][w][16] is written as 1 KB
//   runs; the last layer L2-normalises over the 4 lanes x 4 quarters that hold a pixel.
#pragma once

namespace sde {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int H16_PLANE = 9984;                           // 612 pixels x 16 B, rounded up to 256 B
constexpr int H16_STAGE = 8 * H16_PLANE;                  // [part 2][quarter 4] planes: 79,872 B
constexpr size_t H16_BIAS_OFF = 2 * (size_t)H16_STAGE;
constexpr size_t H16_SMEM = H16_BIAS_OFF + NF * sizeof(float);   // 160,000 B
constexpr int H16_NCB = 2;                                // 32-channel c-blocks per tile
constexpr int H16_HT = 18;                                // half-taps per c-block (9 taps x 2 quarter pairs)
constexpr int H16_RD = 3;                                 // B ring depth (fragments read RD-1 steps ahead)
static_assert(H16_PLANE >= XP_NPIX * 16 && H16_PLANE % 256 == 0, "plane size / bank alignment");
static_assert(H16_SMEM <= 163840, "LDS");
// layer 2 (FIRST): + the image window of the tile (20 x 36 fp32) behind the biases
constexpr size_t H16_WIN_OFF = H16_SMEM;
constexpr size_t H16_SMEM_FIRST = H16_WIN_OFF + XP_WIN * sizeof(float);   // 162,880 B
static_assert(H16_SMEM_FIRST <= 163840, "LDS (layer 2)");
// Timing-only diagnostic builds (no epilogue stores, no stager work, constant A or B operands, in-kernel
// clock stamps, ring-depth probes; wrong results) live in the probe copy tools/variants/tower_h16_diag.h,
// which tools/build_file_variant.sh substitutes for this header (-DSDE_H16_HEADER=...).
// Cache-policy bits of the stagers' activation loads: 1 (sc0) streams each activation past the CU's L1,
// which leaves the L1 to the A fragments all four MFMA waves re-read every tap.  Timing builds showed the
// MFMA waves waiting on those fragments (a probe build with the same loads issued but not consumed runs 149 us
// like no loads at all, 151, against 204 us).  Tower pair -8 to -30 us in three round-robin runs
// (profiles/r05/tower_act_aux_nt.txt); 2 (nt) does not help; 0 = the default policy.
#ifndef H16_ACT_AUX
#define H16_ACT_AUX 1
#endif

// Split 4 channels, scaled by s, into the stage's (part, quarter) planes at dst (the unit's byte offset
// in the stage, see h16_stager_loop): hi = f16(x s) by packed converts, lo = f16(x s - hi) by v_fma_mix from the
// packed hi half (xp_split16s; x s - hi is exact in fp32, so the same bits as the per-value split).  8 instead of
// 20 VALU per unit: the stagers' work per launch 222 -> 136 kcycles (profiles/r06/tower_phase_*.txt).
__device__ __forceinline__ void h16_put(char *dst, float4 v, float s)
{
    u32x2 hw, lw;
    xp_split16s(make_float4(v.x * s, v.y * s, v.z * s, v.w * s), hw, lw);
    *reinterpret_cast<uint2 *>(dst) = __builtin_bit_cast(uint2, hw);
    *reinterpret_cast<uint2 *>(dst + 4 * H16_PLANE) = __builtin_bit_cast(uint2, lw);
}

// Stage unit (pixel << 2 | 4-channel chunk) of stager thread st at iteration i: a wave's lanes take 16
// consecutive pixels x the 4 chunks, so each 32-lane half of a ds_write_b64 fills one quarter plane's 256
// contiguous bytes (the planes are 256-B aligned: lane-contiguous units would put both quarters of a pixel
// in one bank set), and the wave's loads still cover 1 KB of pixels contiguously.  Within a half the chunk
// pair of a pixel is the fastest index (lane = 32 plane + 16 pixel-octet + 2 pixel + chunk & 1): each
// 16-lane group of the write is then 128 contiguous bytes, one dword per bank (pixels at a 16-B stride put
// pixels 8 apart on one bank: 5.2e6 conflict cycles per launch by PMC, round 5).
__device__ __forceinline__ int h16_unit(int st, int i)
{
    const int l = st & 63;
    const int px = (i * (XP_STAGERS / 64) + (st >> 6)) * 16 + ((l >> 4) & 1) * 8 + ((l >> 1) & 7);
    return px * 4 + ((l >> 5) << 1 | (l & 1));
}
static_assert(XP_UPT * XP_STAGERS / 4 >= XP_NPIX, "the stager units cover the stage's pixels");

// Stager waves: half-steps k = (tile, 16-channel block cb16 = k % 4) in the MFMA waves' order; half-steps
// 2i, 2i+1 make c-block step i (stage i & 1).  Two register sets of one half-step each are loaded
// one c-block step ahead of their store.  One barrier per c-block step, like the MFMA waves.
// A unit's global and LDS offsets are tile-invariant: computed once; per half-step a wave-uniform
// buffer descriptor at the tile's origin (loads outside the input take an offset past the records
// and return the zero padding), and interior tiles skip the bound tests.
template <bool IN_CB>
__device__ __forceinline__ void h16_stager_loop(char *hsm, const float *__restrict__ in, int Hin, int Win,
                                                const XpBatch &bt, int st, const float *__restrict__ in_amax,
                                                const float *__restrict__ hdr)
{
    const int tile0 = blockIdx.x, gstride = gridDim.x;
    const int nsteps = ((bt.ntiles - 1 - tile0) / gstride + 1) * H16_NCB;
    const int nh = 2 * nsteps;
    uint32_t uoff[XP_UPT], uyx[XP_UPT], ulds[XP_UPT];
#pragma unroll
    for (int i = 0; i < XP_UPT; i++) {
        const int u = h16_unit(st, i), px = u >> 2, chunk = u & 3;
        const int iy = px / XP_IX, ix = px - iy * XP_IX;
        const bool ok = u < XP_UNITS;
        uoff[i] = ok ? (uint32_t)((iy * Win + ix) * (IN_CB ? 64 : 256) + 16 * chunk) : XP_OOB;
        uyx[i] = ok ? (uint32_t)(iy << 16 | ix) : 0xFFFF0000u;
        ulds[i] = ok ? (uint32_t)((chunk >> 1) * H16_PLANE + px * 16 + (chunk & 1) * 8) : 0u;
    }
    auto load = [&](float4 (&v)[XP_UPT], int k) {
        const int t = tile0 + (k >> 2) * gstride, cb16 = k & 3;
        int img, ty0, tx0;
        xp_tile(bt, t, img, ty0, tx0);
        const float *src = in + img * bt.in_stride;
        const __amdgpu_buffer_rsrc_t rs =
            xp_rsrc(IN_CB ? src + (((size_t)cb16 * Hin + ty0) * Win + tx0) * 16
                          : src + ((size_t)ty0 * Win + tx0) * 64 + cb16 * 16);
        const int ly = Hin - ty0, lx = Win - tx0;
        if (ly >= XP_IY && lx >= XP_IX) {   // wave-uniform: the tile's input window is inside the input
#pragma unroll
            for (int i = 0; i < XP_UPT; i++)
                v[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, uoff[i], 0, H16_ACT_AUX));
        } else {
#pragma unroll
            for (int i = 0; i < XP_UPT; i++) {
                const bool ok = (int)(uyx[i] >> 16) < ly && (int)(uyx[i] & 0xFFFFu) < lx;
                v[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? uoff[i] : XP_OOB, 0, H16_ACT_AUX));
            }
        }
    };
    int sc_img = -1;
    float s = 1.0f, unscale = 1.0f;
    auto store = [&](const float4 (&v)[XP_UPT], int k) {
        const int im = (tile0 + (k >> 2) * gstride) / bt.tiles_img;
        if (im != sc_img) {   // the tile's image changed: its bound word (tiles run image-major)
            xp_scales(false, in_amax + im * bt.amax_stride, hdr, s, unscale);
            sc_img = im;
        }
        // half h = k & 1 of the c-block: quarter planes 2h, 2h + 1
        char *sb = hsm + ((k >> 1) & 1) * H16_STAGE + (k & 1) * 2 * H16_PLANE;
#pragma unroll
        for (int i = 0; i < XP_UPT; i++)
            if (h16_unit(st, i) < XP_UNITS) h16_put(sb + ulds[i], v[i], s);
    };
    float4 ra[XP_UPT], rb[XP_UPT];
    load(ra, 0);
    load(rb, 1);
    store(ra, 0);
    store(rb, 1);
    if (2 < nh) load(ra, 2);
    if (3 < nh) load(rb, 3);
    __syncthreads();
    // step i: the MFMA waves consume stage i & 1; here step i+1's halves are stored and step
    // i+2's loaded
#pragma unroll 1
    for (int i = 0; i < nsteps; i++) {
        if (2 * i + 2 < nh) store(ra, 2 * i + 2);
        if (2 * i + 4 < nh) load(ra, 2 * i + 4);
        if (2 * i + 3 < nh) store(rb, 2 * i + 3);
        if (2 * i + 5 < nh) load(rb, 2 * i + 5);
        __syncthreads();
    }
}

// Stager waves, layer 2 (FIRST): the stage is conv1 (Cin = 1, 3x3, bias, ReLU; mc_cnn_brunch.py:31-48) of
// the padded image, computed here -- the same fmaf order as xp_conv1, so the same conv1 values as
// conv64_x6p_kernel's layer 2.  Same units, half-steps and barriers as h16_stager_loop; a lane's 4-channel
// chunk is the same in every unit, so a half-step's weights (9 taps + bias of 4 channels) are one register
// set, loaded a step ahead like the activations of the other layers.  The tile's image window (20 x 36)
// lives in LDS behind the biases, single-buffered: EVERY stager wave writes the whole window (identical
// values) at the tile's first half-step and then reads only what it wrote itself (a wave's LDS accesses
// complete in order), so no wave waits for another; the previous tile's window was last read in the step
// before, which the c-block barrier closes.  The window is loaded into registers a step ahead.
__device__ __forceinline__ void h16_conv1_stager_loop(char *hsm, const float *__restrict__ img, int Hin, int Win,
                                                      const XpBatch &bt, int st, const float *__restrict__ in_amax,
                                                      const float *__restrict__ hdr, const float *__restrict__ w1blob)
{
    const int tile0 = blockIdx.x, gstride = gridDim.x;
    const int nsteps = ((bt.ntiles - 1 - tile0) / gstride + 1) * H16_NCB;
    const int nh = 2 * nsteps;
    const int lane = st & 63;
    float *win = reinterpret_cast<float *>(hsm + H16_WIN_OFF);
    // a unit's window offset (its top-left tap), (iy, ix) in the tile and LDS offset: tile-invariant
    uint32_t uwin[XP_UPT], uyx[XP_UPT], ulds[XP_UPT];
#pragma unroll
    for (int i = 0; i < XP_UPT; i++) {
        const int u = h16_unit(st, i), px = u >> 2, chunk = u & 3;
        const int iy = px / XP_IX, ix = px - iy * XP_IX;
        const bool ok = u < XP_UNITS;
        uwin[i] = ok ? (uint32_t)(iy * XP_WX + ix) : 0u;
        uyx[i] = ok ? (uint32_t)(iy << 16 | ix) : 0xFFFF0000u;
        ulds[i] = ok ? (uint32_t)((chunk >> 1) * H16_PLANE + px * 16 + (chunk & 1) * 8) : 0u;
    }
    const int chunk = ((lane >> 5) << 1) | (lane & 1);   // = h16_unit(st, i) & 3 for every i
    constexpr int WPL = (XP_WIN + 63) / 64;
    float wv[WPL];
    auto wload = [&](int t) {
        int im, ty0, tx0;
        xp_tile(bt, t, im, ty0, tx0);
        const float *src = img + im * bt.in_stride;
#pragma unroll
        for (int k = 0; k < WPL; k++) {
            const int idx = lane + 64 * k;
            const int iy = idx / XP_WX, ix = idx - iy * XP_WX;
            const int y = ty0 + iy, x = tx0 + ix;
            wv[k] = (idx < XP_WIN && y < Hin && x < Win) ? src[(size_t)y * Win + x] : 0.0f;
        }
    };
    static_assert(XP_UPT >= 10, "a half-step's weights: 9 taps + the biases");
    // half-step k: channels 16 (k & 3) + 4 chunk .. +3; its tile's window at the tile's first half-step
    auto load = [&](float4 (&w)[XP_UPT], int k) {
        const int n0 = (k & 3) * 16 + chunk * 4;
#pragma unroll
        for (int t = 0; t < 9; t++) w[t] = *reinterpret_cast<const float4 *>(w1blob + NF + t * NF + n0);
        w[9] = *reinterpret_cast<const float4 *>(w1blob + n0);
        if ((k & 3) == 0) wload(tile0 + (k >> 2) * gstride);
    };
    int sc_img = -1;
    float s = 1.0f, unscale = 1.0f;
    auto store = [&](const float4 (&w)[XP_UPT], int k) {
        int im, ty0, tx0;
        xp_tile(bt, tile0 + (k >> 2) * gstride, im, ty0, tx0);
        if (im != sc_img) {
            xp_scales(true, in_amax + im * bt.amax_stride, hdr, s, unscale);
            sc_img = im;
        }
        if ((k & 3) == 0) {
#pragma unroll
            for (int k2 = 0; k2 < WPL; k2++)
                if (lane + 64 * k2 < XP_WIN) win[lane + 64 * k2] = wv[k2];
            __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the window's LDS writes have landed
            __builtin_amdgcn_wave_barrier();
        }
        char *sb = hsm + ((k >> 1) & 1) * H16_STAGE + (k & 1) * 2 * H16_PLANE;
        const int ly = Hin - 2 - ty0, lx = Win - 2 - tx0;   // conv1's output extent from the tile origin
#pragma unroll
        for (int i = 0; i < XP_UPT; i++) {
            if (h16_unit(st, i) >= XP_UNITS) continue;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if ((int)(uyx[i] >> 16) < ly && (int)(uyx[i] & 0xFFFFu) < lx) {
                float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
                const float *wp = win + uwin[i];
#pragma unroll
                for (int t = 0; t < 9; t++) {
                    const float x = wp[(t / 3) * XP_WX + t % 3];
                    s0 = fmaf(x, w[t].x, s0);
                    s1 = fmaf(x, w[t].y, s1);
                    s2 = fmaf(x, w[t].z, s2);
                    s3 = fmaf(x, w[t].w, s3);
                }
                v = make_float4(fmaxf(s0 + w[9].x, 0.f), fmaxf(s1 + w[9].y, 0.f), fmaxf(s2 + w[9].z, 0.f),
                                fmaxf(s3 + w[9].w, 0.f));
            }
            h16_put(sb + ulds[i], v, s);
        }
    };
    float4 ra[XP_UPT], rb[XP_UPT];
    load(ra, 0);
    load(rb, 1);
    store(ra, 0);
    store(rb, 1);
    if (2 < nh) load(ra, 2);
    if (3 < nh) load(rb, 3);
    __syncthreads();
#pragma unroll 1
    for (int i = 0; i < nsteps; i++) {
        if (2 * i + 2 < nh) store(ra, 2 * i + 2);
        if (2 * i + 4 < nh) load(ra, 2 * i + 4);
        if (2 * i + 3 < nh) store(rb, 2 * i + 3);
        if (2 * i + 5 < nh) load(rb, 2 * i + 5);
        __syncthreads();
    }
}

// Stager waves, split inputs (ISPL, SDE_TOWER_IN_SPLIT): a stage's 8 planes (part, quarter) are copies of
// input planes cb * 8 + (part * 4 + quarter) of the tile's 18 x 34 window, each [h][w][8 fp16] in HBM -- so a
// stage is filled by LDS-DMA with no arithmetic and no VGPR round trip: 1 KB (64 pixels, row-wrapped by the
// per-lane source offsets) per wave-instruction, stager wave w copying planes 2w and 2w + 1, 10
// instructions each (the last one 36 lanes).  The descriptor ends at the plane's end: a window pixel past the
// input's right edge reads the next row's pixel, one past the plane's end reads zero; both feed only
// outputs outside the image, which are never stored.  Same step / barrier pattern as h16_stager_loop.
__device__ __forceinline__ void h16_dma_stager_loop(char *hsm, const float *__restrict__ in, int Hin, int Win,
                                                    const XpBatch &bt, int st)
{
    const int tile0 = blockIdx.x, gstride = gridDim.x;
    const int nsteps = ((bt.ntiles - 1 - tile0) / gstride + 1) * H16_NCB;
    const int w = __builtin_amdgcn_readfirstlane(st >> 6), lane = st & 63;
    constexpr int ND = (XP_NPIX + 63) / 64, NLAST = XP_NPIX - 64 * (ND - 1);
    uint32_t voff[ND];
#pragma unroll
    for (int d = 0; d < ND; d++) {
        const int px = d * 64 + lane, iy = px / XP_IX, ix = px - iy * XP_IX;
        voff[d] = (uint32_t)((iy * Win + ix) * 16);
    }
    const size_t PB = (size_t)Hin * Win * 16;
    auto issue = [&](int k) {
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
    };
    issue(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll 1
    for (int i = 0; i < nsteps; i++) {
        if (i + 1 < nsteps) issue(i + 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
}

// A fragments of one half-tap (tap s >> 1, quarters 2 (s & 1) + qq) of 32-channel c-block cb: [part][qq],
// by buffer loads: ra = the layer's F16 A-fragment blob, voff = the lane's byte offset in its
// [mtile][cblock16][tap][part][lane][8] order, cbo = cb's byte offset (wave-uniform); the rest of the
// offset is a compile-time constant (no per-load VALU address arithmetic).
struct H16A {
    f16x8 f[2][2];
};
constexpr int H16_A_CB = 2 * 9 * 2 * 64 * 16;   // bytes per 32-channel c-block of one M-tile

__device__ __forceinline__ H16A h16_afrag(__amdgpu_buffer_rsrc_t ra, uint32_t voff, int cbo, int s)
{
    const int tap = s >> 1, hf = s & 1;
    H16A a;
#pragma unroll
    for (int p = 0; p < 2; p++)
#pragma unroll
        for (int qq = 0; qq < 2; qq++) {
            const int k = (((hf * XP_NCB * 9 + tap) * 2 + p) * 64 + 16 * qq) * 16;
            a.f[p][qq] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(ra, voff, cbo + k, 0));
        }
    return a;
}

struct H16B {
    f16x8 hi, lo;
};

// B fragment of step b = (half-tap b >> 3, row (b >> 1) & 3, pixel half b & 1); sb = the stage at the
// lane's base.
__device__ __forceinline__ H16B h16_bfrag(const char *sb, int b)
{
    const int tap = b >> 4, r = (b >> 1) & 3, ph = b & 1;
    const int off = ((r + tap / 3) * XP_IX + 16 * ph + tap % 3) * 16;
    H16B f;
    f.hi = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4 *>(sb + off));
    f.lo = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4 *>(sb + 4 * H16_PLANE + off));
    return f;
}

__device__ __forceinline__ floatx4 mfma16(f16x8 a, f16x8 b, floatx4 c)
{
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// One 32-channel c-block for one MFMA wave: 18 half-taps x 8 (row, half) steps, 6 MFMAs each.
// acc[(r * 2 + ph) * 4 + q].  A ring of three half-taps with static slots (18 = 6 x 3: every c-block
// starts in the same phase): on entry abuf[0] = A(cb, 0) and abuf[1] = A(cb, 1) are requested; half-tap s
// requests A(s + 2) into the slot A(s - 1) left; on exit abuf[0..1] = A(ncb, 0..1).
template <int NA>
__device__ __forceinline__ void h16_cblock(floatx4 (&acc)[32], H16A (&abuf)[NA], __amdgpu_buffer_rsrc_t ra,
                                           uint32_t avoff, int cb, int ncb, const char *sb)
{
    constexpr int NB = H16_HT * 8;
    static_assert(H16_HT % 3 == 0, "A ring phase");
    H16B ring[H16_RD];
#pragma unroll
    for (int k = 0; k < H16_RD - 1; k++) ring[k] = h16_bfrag(sb, k);
#pragma unroll
    for (int s = 0; s < H16_HT; s++) {
        abuf[(s + 2) % 3] = s + 2 < H16_HT ? h16_afrag(ra, avoff, cb * H16_A_CB, s + 2)
                                           : h16_afrag(ra, avoff, ncb * H16_A_CB, s + 2 - H16_HT);
        const H16A &a = abuf[s % 3];
        const int hf = s & 1;
#pragma unroll
        for (int rp = 0; rp < 8; rp++) {
            const int b = s * 8 + rp;
            __builtin_amdgcn_sched_barrier(0);
            const H16B &bf = ring[b % H16_RD];
#pragma unroll
            for (int qq = 0; qq < 2; qq++) {
                floatx4 &c = acc[rp * 4 + 2 * hf + qq];
                c = mfma16(a.f[1][qq], bf.hi, c);
                c = mfma16(a.f[0][qq], bf.lo, c);
                c = mfma16(a.f[0][qq], bf.hi, c);
            }
            if (b + H16_RD - 1 < NB) ring[(b + H16_RD - 1) % H16_RD] = h16_bfrag(sb, b + H16_RD - 1);
        }
    }
}

// The same c-block with each B fragment feeding all four quarters (H16_B12): 9 taps x 8 (row, half) steps of
// 12 MFMAs, so half the B reads from LDS per MFMA.  A ring of two whole taps (four half-tap slots, abuf[(h +
// PH) % 4] for half-tap h; 18 half-taps per c-block, so the two c-blocks of a tile run in phases 0 and 2):
// tap s requests tap s + 1 into the slots tap s - 1 left; on exit abuf holds A(ncb, tap 0) at phase PH + 2.
// Every accumulator takes the same MFMAs in the same order as h16_cblock: the same bits.
__device__ __forceinline__ H16B h16_bfrag12(const char *sb, int b)
{
    const int tap = b >> 3, r = (b >> 1) & 3, ph = b & 1;
    const int off = ((r + tap / 3) * XP_IX + 16 * ph + tap % 3) * 16;
    H16B f;
    f.hi = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4 *>(sb + off));
    f.lo = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4 *>(sb + 4 * H16_PLANE + off));
    return f;
}

// BRD: depth of the B ring (fragments read BRD - 1 (row, half) steps ahead).  Depth 3 (two steps, 24 MFMAs
// ahead) takes the MFMA waves' c-block loop from 280 to 249-274 kcycles per launch against the 232-kcycle MFMA floor
// (phase stamps, profiles/r06/tower_phase_*.txt): the LDS latency of a one-step-ahead read was showing.  The 8
// more VGPRs fit the middle layers' c-block-layout instantiation without spills; the others keep depth 2.
// NEXT = false (the c-block that ends a tile): the last tap does not request the next c-block's first tap; the
// caller's epilogue does, once half the accumulators are stored (h16_epilogue's `mid`), so those 32 VGPRs are not
// live across the whole epilogue -- what lets the 3-deep B ring fit layer 2 and the last layer without spills.
template <int PH, int BRD, bool NEXT = true>
__device__ __forceinline__ void h16_cblock12(floatx4 (&acc)[32], H16A (&abuf)[4], __amdgpu_buffer_rsrc_t ra,
                                             uint32_t avoff, int cb, int ncb, const char *sb)
{
    constexpr int NT = 9, NB = NT * 8;
    static_assert(NB % BRD == 0, "static B ring slots");
    H16B ring[BRD];
#pragma unroll
    for (int k = 0; k < BRD - 1; k++) ring[k] = h16_bfrag12(sb, k);
#pragma unroll
    for (int s = 0; s < NT; s++) {
#pragma unroll
        for (int hf = 0; hf < 2; hf++) {
            const int h = 2 * (s + 1) + hf;
            if (NEXT || h < H16_HT)
                abuf[(h + PH) % 4] = h < H16_HT ? h16_afrag(ra, avoff, cb * H16_A_CB, h)
                                                : h16_afrag(ra, avoff, ncb * H16_A_CB, h - H16_HT);
        }
#pragma unroll
        for (int rp = 0; rp < 8; rp++) {
            const int b = s * 8 + rp;
            __builtin_amdgcn_sched_barrier(0);
            const H16B &bf = ring[b % BRD];
            if (b + BRD - 1 < NB) ring[(b + BRD - 1) % BRD] = h16_bfrag12(sb, b + BRD - 1);
#pragma unroll
            for (int hf = 0; hf < 2; hf++) {
                const H16A &a = abuf[(2 * s + hf + PH) % 4];
#pragma unroll
                for (int qq = 0; qq < 2; qq++) {
                    floatx4 &c = acc[rp * 4 + 2 * hf + qq];
                    c = mfma16(a.f[1][qq], bf.hi, c);
                    c = mfma16(a.f[0][qq], bf.lo, c);
                    c = mfma16(a.f[0][qq], bf.hi, c);
                }
            }
        }
    }
}
// 2: every layer but the last one with split outputs (whose epilogue would spill), 1: the middle layers only,
// 0: none (A/B builds)
#ifndef H16_B12
#define H16_B12 2
#endif

// Tile epilogue of one MFMA wave (rows 4g ..): unscale + bias, then ReLU + c-block-major stores
// (+ the running bound word), or (LAST) the L2 norm and [h][w][64] stores.  Stored registers are
// pinned live for XP_PIN stores, as in xp_epilogue ("store-data overwrite").
template <bool LAST, bool OUT_CB, bool SPLIT, bool OSPL, typename MID>
__device__ __forceinline__ void h16_epilogue(const floatx4 (&acc)[32], int lane, int g, int img, int ty0, int tx0,
                                             float unscale, const float4 *lbias4, float *__restrict__ out, int Hout,
                                             int Wout, const XpBatch &bt, uint16_t *__restrict__ ohi,
                                             uint16_t *__restrict__ olo, float *__restrict__ onrm,
                                             uint32_t &amax_run, int &amax_img, float *__restrict__ out_amax,
                                             float oscale, MID &&mid)
{
    static_assert(!OSPL || (!LAST && !OUT_CB), "split outputs: intermediate layers");
    int j = lane & 15, k4 = lane >> 4;
    asm volatile("" : "+v"(j), "+v"(k4));
    const int row0 = 4 * g;
    constexpr int NPIN = 32;
    u32x4 pin[NPIN];
    if (!LAST) {
        uint32_t amax = 0u;
        float *const outi = out + img * bt.out_stride;
        const size_t HW = (size_t)Hout * Wout;
        // OSPL: channels 16q + 4 k4 + e are 8-channel group 2q + (k4 >> 1), plane (q >> 1) * 8 + part * 4 +
        // 2 (q & 1) + (k4 >> 1).  A lane pair (k4 even, k4 + 1) swaps halves (v_permlane16_swap, rows 2i <->
        // 2i + 1) so that the even lane holds the group's 8 hi parts and the odd one its 8 lo parts: one 16-B
        // store each, to plane part = k4 & 1
        const uint32_t pb = (uint32_t)HW * 16u;
        const uint32_t ospl_lane = (uint32_t)((k4 & 1) * 4 + (k4 >> 1)) * pb;
        // FULL: every row and column of the tile is inside the output (all but the last tile row and column):
        // no per-row branches, no per-lane range selects
        auto body = [&](auto fullc) {
        constexpr bool FULL = decltype(fullc)::value;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const float4 b4 = lbias4[4 * q + k4];
            const float bq[4] = {b4.x, b4.y, b4.z, b4.w};
            // OUT_CB: [cblk16 = q][h][w][16], one descriptor per c-block plane; else [h][w][64]
            const __amdgpu_buffer_rsrc_t rs =
                OSPL ? xp_rsrc(reinterpret_cast<char *>(outi) + ((size_t)((q >> 1) * 8 + 2 * (q & 1)) * HW + (size_t)ty0 * Wout) * 16)
                     : xp_rsrc(OUT_CB ? outi + ((size_t)q * HW + (size_t)ty0 * Wout) * 16
                                      : outi + (size_t)ty0 * Wout * NF);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const bool rok = FULL || ty0 + row0 + r < Hout;   // wave-uniform
                const uint32_t so = (uint32_t)((row0 + r) * Wout) * (OUT_CB ? 64u : 256u);
#pragma unroll
                for (int ph = 0; ph < 2; ph++) {
                    const int x = tx0 + 16 * ph + j;
                    const bool xok = FULL || x < Wout;
                    const floatx4 &c = acc[(r * 2 + ph) * 4 + q];
                    float o4[4];
                    // OSPL: the outputs scaled by 2^sigma straight from the accumulators (scale folded into
                    // the unscale and the bias: exact), their bound unscaled below
#pragma unroll
                    for (int e = 0; e < 4; e++)
                        o4[e] = fmaxf(fmaf(c[e], OSPL ? unscale * oscale : unscale, OSPL ? bq[e] * oscale : bq[e]), 0.f);
                    const float4 o = make_float4(o4[0], o4[1], o4[2], o4[3]);
                    const int k = (q * 4 + r) * 2 + ph;
                    if (OSPL) {
                        u32x2 hw2, lw2;
                        xp_split16s(o, hw2, lw2);
                        const u32x4 v4 = xp_pair_parts<false>(hw2, lw2);
                        pin[k] = v4;
                        if (rok) {
                            if (xok) {
                                amax = max(amax, max(__float_as_uint(o.x), __float_as_uint(o.y)));
                                amax = max(amax, max(__float_as_uint(o.z), __float_as_uint(o.w)));
                            }
                            const uint32_t v2 = xok ? ospl_lane + (uint32_t)x * 16u : XP_OOB;
                            const uint32_t s2 = (uint32_t)((row0 + r) * Wout) * 16u;
                            __builtin_amdgcn_raw_buffer_store_b128(v4, rs, v2, s2, 0);
                        }
                    } else {
                        pin[k] = __builtin_bit_cast(u32x4, o);
                        if (rok) {
                            if (xok) {   // the bound before the store: nothing writes o's registers after it
                                amax = max(amax, max(__float_as_uint(o.x), __float_as_uint(o.y)));
                                amax = max(amax, max(__float_as_uint(o.z), __float_as_uint(o.w)));
                            }
                            xp_st4(o, rs, xok ? (uint32_t)(OUT_CB ? x * 64 + 16 * k4 : x * 256 + 64 * q + 16 * k4) : XP_OOB, so);
                        }
                    }
                    asm volatile("s_nop 2" ::"v"(pin[k >= XP_PIN - 1 ? k - (XP_PIN - 1) : k]) : "memory");   // after each store: >= 9 wait states over XP_PIN stores
                }
            }
            if (q == 1) mid();   // half the accumulators stored
        }
#pragma unroll
        for (int k = NPIN - (XP_PIN - 1); k + 1 < NPIN; k++) asm volatile("" ::"v"(pin[k]));
        asm volatile("s_nop 7\n\ts_nop 1" ::"v"(pin[NPIN - 1]) : "memory");
        };
        if (ty0 + XP_TY <= Hout && tx0 + XP_TX <= Wout) body(std::true_type{});
        else body(std::false_type{});
        if (OSPL) amax = __float_as_uint(__uint_as_float(amax) / oscale);   // exact: a power of two
        // one atomic per wave and image (flushed when the tiles move to the next image and at the end)
        if (img != amax_img) {
            xp_flush_amax(amax_run, amax_img, lane, out_amax, bt.amax_stride);
            amax_img = img;
        }
        amax_run = max(amax_run, amax);
    } else {
        // a pixel's 64 channels: 4 quarters x 4 lanes (k4) x 4 registers of this wave
        const size_t pix0 = (size_t)img * bt.pix_stride + (size_t)ty0 * Wout;
        const __amdgpu_buffer_rsrc_t rs = xp_rsrc(out + pix0 * NF);
        auto body = [&](auto fullc) {   // FULL: as above
        constexpr bool FULL = decltype(fullc)::value;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const bool rok = FULL || ty0 + row0 + r < Hout;
            const uint32_t so = (uint32_t)((row0 + r) * Wout) * 256u;
#pragma unroll
            for (int ph = 0; ph < 2; ph++) {
                const int x = tx0 + 16 * ph + j;
                int kr = k4;
                asm volatile("" : "+v"(kr));   // per-step opaque copy: bias re-read from LDS per use
                float t[4][4];
                float ss = 0.0f;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const float4 b4 = lbias4[4 * q + kr];
                    const float bq[4] = {b4.x, b4.y, b4.z, b4.w};
                    const floatx4 &c = acc[(r * 2 + ph) * 4 + q];
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        t[q][e] = fmaf(c[e], unscale, bq[e]);
                        ss += t[q][e] * t[q][e];
                    }
                }
                ss += __shfl_xor(ss, 16, 64);
                ss += __shfl_xor(ss, 32, 64);
                const float inv = 1.0f / sqrtf(fmaxf(ss, 1e-12f));
                const bool xok = FULL || x < Wout;
                const uint32_t vo = xok ? (uint32_t)(x * 256 + 16 * k4) : XP_OOB;
                float s2 = 0.0f;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const float4 o = make_float4(t[q][0] * inv, t[q][1] * inv, t[q][2] * inv, t[q][3] * inv);
                    const int k = (r * 2 + ph) * 4 + q;
                    pin[k] = __builtin_bit_cast(u32x4, o);
                    if (rok) xp_st4(o, rs, vo + 64u * q, so);
                    asm volatile("s_nop 2" ::"v"(pin[k >= XP_PIN - 1 ? k - (XP_PIN - 1) : k]) : "memory");   // after each store: >= 9 wait states over XP_PIN stores
                    if (SPLIT) {   // bf16 split planes of the features (sde_cv_wta_split's input)
                        const float xs[4] = {o.x, o.y, o.z, o.w};
                        bf16x4 hv, lv;
#pragma unroll
                        for (int e = 0; e < 4; e++) {
                            const __bf16 hh = (__bf16)xs[e];
                            hv[e] = hh;
                            lv[e] = (__bf16)(xs[e] - (float)hh);
                            s2 += xs[e] * xs[e];
                        }
                        if (rok) {
                            const __amdgpu_buffer_rsrc_t rh = xp_rsrc(ohi + pix0 * NF), rl = xp_rsrc(olo + pix0 * NF);
                            const uint32_t o2 = xok ? (uint32_t)(x * 128 + 32 * q + 8 * k4) : XP_OOB;
                            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, hv), rh, o2, so / 2u, 0);
                            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, lv), rl, o2, so / 2u, 0);
                        }
                    }
                }
                if (SPLIT && onrm) {   // fp32 rounding bound of the 64-term sum
                    s2 += __shfl_xor(s2, 16, 64);
                    s2 += __shfl_xor(s2, 32, 64);
                    if (rok) {
                        const __amdgpu_buffer_rsrc_t rn = xp_rsrc(onrm + pix0);
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, sqrtf(s2) * 1.000004f), rn,
                                                              (xok && k4 == 0) ? (uint32_t)(x * 4) : XP_OOB, so / 64u, 0);
                    }
                }
            }
            if (r == 1) mid();   // half the accumulators stored
        }
#pragma unroll
        for (int k = NPIN - (XP_PIN - 1); k + 1 < NPIN; k++) asm volatile("" ::"v"(pin[k]));
        asm volatile("s_nop 7\n\ts_nop 1" ::"v"(pin[NPIN - 1]) : "memory");
        };
        if (ty0 + XP_TY <= Hout && tx0 + XP_TX <= Wout) body(std::true_type{});
        else body(std::false_type{});
    }
}

// Epilogue overlap (non-last layers; H16_OVL_K = K > 0).  With one MFMA wave per SIMD, a whole-tile epilogue
// (32 stores and their VALU) leaves the SIMD's matrix core idle: 13 % of the MFMA waves' cycles (phase stamps,
// profiles/r06/tower_phase_product_r6n.txt).  Here the 64 output channels are two halves H0 (quarters 0-1: half-tap
// 0 of every tap) and H1 (quarters 2-3: half-tap 1), and K taps at one end of each c-block run one half after the
// other (each B fragment then feeds 6 MFMAs, read twice), so that one half's accumulators are final, or free,
// while the other half's MFMAs run:
//   c-block 0: taps 0..K-1 half 0 [+ the previous tile's H1 stores], taps 0..K-1 half 1, taps K..8 whole;
//   c-block 1: taps 0..8-K whole, taps 9-K..8 half 0, taps 9-K..8 half 1 [+ this tile's H0 stores].
// Every accumulator takes the same MFMAs in the same order as in h16_cblock12 (taps ascending; the first MFMA of
// a tile on a zero accumulator): the same bits.  A fragments: items n (half-taps in consumption order, 36 per
// tile) in slot n % 4, each requested once, up to 3 items ahead.
#ifndef H16_OVL_K
#define H16_OVL_K 4
#endif

// item j of c-block cb in consumption order: its tap and half
__host__ __device__ constexpr int ovl_tap(int cb, int K, int j)
{
    return cb == 0 ? (j < 2 * K ? j % K : (j - 2 * K) / 2 + K) : (j < 2 * (9 - K) ? j / 2 : (j - 2 * (9 - K)) % K + 9 - K);
}
__host__ __device__ constexpr int ovl_hf(int cb, int K, int j)
{
    return cb == 0 ? (j < 2 * K ? j / K : (j - 2 * K) % 2) : (j < 2 * (9 - K) ? j % 2 : (j - 2 * (9 - K)) / K);
}
// groups (one half-tap, or a whole tap = 2 items): first item and size
__host__ __device__ constexpr int ovl_gstart(int cb, int K, int g)
{
    return cb == 0 ? (g < 2 * K ? g : 2 * K + 2 * (g - 2 * K)) : (g < 9 - K ? 2 * g : 2 * (9 - K) + (g - (9 - K)));
}
__host__ __device__ constexpr int ovl_gsize(int cb, int K, int g)
{
    return cb == 0 ? (g < 2 * K ? 1 : 2) : (g < 9 - K ? 2 : 1);
}
// last item requested before group g starts (items are requested up to the group's first + 3)
__host__ __device__ constexpr int ovl_req(int cb, int K, int g)
{
    return g > 0 ? 18 * cb + ovl_gstart(cb, K, g - 1) + 3 : cb == 0 ? 2 : ovl_gstart(0, K, 9 + K - 1) + 3;
}
static_assert(ovl_gstart(0, 4, 12) == 16 && ovl_gsize(0, 4, 12) == 2 && ovl_gstart(1, 4, 12) == 17, "ovl groups");
static_assert(ovl_tap(0, 4, 5) == 1 && ovl_hf(0, 4, 5) == 1 && ovl_tap(1, 4, 15) == 6 && ovl_hf(1, 4, 15) == 1,
              "ovl items");

// A fragments of tile-relative item n (n >= 36: the next tile's)
__device__ __forceinline__ H16A ovl_afrag(__amdgpu_buffer_rsrc_t ra, uint32_t avoff, int K, int n)
{
    const int m = n % 36, cb = m / 18, j = m % 18;
    return h16_afrag(ra, avoff, cb * H16_A_CB, 2 * ovl_tap(cb, K, j) + ovl_hf(cb, K, j));
}

// c-block CB of the overlapped schedule; epi(store_tag, e) issues epilogue store e (0..15) of the half being stored,
// one every K / 2 steps over the pass that carries them (c-block 0: the first half-0 pass, c-block 1: the last
// half-1 pass), after the step's MFMAs; epi(bias_tag, e) reads its bias at the step's start
template <int CB, int K, int BRD, typename EPI>
__device__ __forceinline__ void h16_cblock_ovl(floatx4 (&acc)[32], H16A (&abuf)[4], __amdgpu_buffer_rsrc_t ra,
                                               uint32_t avoff, const char *sb, EPI &&epi)
{
    constexpr int NG = 9 + K, NS = 8 * NG;
    constexpr int E0 = CB == 0 ? 0 : NS - 8 * K, EW = 8 * K;   // 16 stores, one every K / 2 steps
    auto bidx = [](int i) { return ovl_tap(CB, K, ovl_gstart(CB, K, i / 8)) * 8 + i % 8; };
    using bias_tag = std::integral_constant<int, 0>;
    using store_tag = std::integral_constant<int, 1>;
    auto sstep = [](int i) { return i >= E0 && i < E0 + EW && (i - E0) % (K / 2) == 0; };   // a store step
    H16B ring[BRD];
#pragma unroll
    for (int k = 0; k < BRD - 1; k++) ring[k] = h16_bfrag12(sb, bidx(k));
    // one group; WE: the group may carry epilogue work (only the pass's groups do: smaller loop bodies to unroll)
    auto group = [&](auto we_c, int g) {
        constexpr bool WE = decltype(we_c)::value;
        const int j0 = ovl_gstart(CB, K, g), gs = ovl_gsize(CB, K, g), n0 = 18 * CB + j0;
#pragma unroll
        for (int d = 1; d <= 3; d++) {   // constant trip count (unrolled before the group loop is)
            const int n = ovl_req(CB, K, g) + d;
            if (n <= n0 + 3) abuf[n % 4] = ovl_afrag(ra, avoff, K, n);
        }
#pragma unroll
        for (int rp = 0; rp < 8; rp++) {
            const int i = g * 8 + rp;
            __builtin_amdgcn_sched_barrier(0);
            // a store step: its bias (an LDS read) first, before this step's B read, the store after the MFMAs
            if (WE && sstep(i)) epi(bias_tag{}, (i - E0) / (K / 2));
            const H16B &bf = ring[i % BRD];
            if (i + BRD - 1 < NS) ring[(i + BRD - 1) % BRD] = h16_bfrag12(sb, bidx(i + BRD - 1));
#pragma unroll
            for (int u = 0; u < gs; u++) {
                const int hf = ovl_hf(CB, K, j0 + u), tap = ovl_tap(CB, K, j0 + u);
                const H16A &a = abuf[(n0 + u) % 4];
#pragma unroll
                for (int qq = 0; qq < 2; qq++) {
                    floatx4 &c = acc[rp * 4 + 2 * hf + qq];
                    c = mfma16(a.f[1][qq], bf.hi, CB == 0 && tap == 0 ? floatx4{0.f, 0.f, 0.f, 0.f} : c);
                    c = mfma16(a.f[0][qq], bf.lo, c);
                    c = mfma16(a.f[0][qq], bf.hi, c);
                }
            }
            if (WE && sstep(i)) epi(store_tag{}, (i - E0) / (K / 2));
        }
    };
    using yes = std::true_type;
    using no = std::false_type;
    constexpr int G0 = E0 / 8, G1 = (E0 + EW) / 8;   // the groups of the store pass
#pragma unroll
    for (int g = 0; g < G0; g++) group(no{}, g);
#pragma unroll
    for (int g = G0; g < G1; g++) group(yes{}, g);
#pragma unroll
    for (int g = G1; g < NG; g++) group(no{}, g);
}

// one tile's output as the overlapped epilogue needs it (the tile whose stores trail into the next tile)
struct H16Out {
    int img, ty0, tx0;
    float unscale, oscale;
};

// epilogue store e of half hh (quarters 2 hh, 2 hh + 1) of a non-last layer's tile: the same values, layout and
// bound as h16_epilogue's (!LAST) body, one store; its data registers are held for 9 wait states after it
__device__ __forceinline__ int h16_half_q(int hh, int e) { return 2 * hh + (e >> 3); }   // e: quarter-major

template <bool OUT_CB, bool OSPL>
__device__ __forceinline__ void h16_store_half(const floatx4 (&acc)[32], int hh, int e, int lane, int g, const H16Out &o,
                                               float4 b4, float *__restrict__ out, int Hout, int Wout,
                                               const XpBatch &bt, uint32_t &amax)
{
    // Always one store (rows past the output and a tile that does not exist, o.img < 0, store out of the
    // buffer's range: dropped).  A store under a branch would make the vector-memory count at the next A-fragment
    // wait path-dependent, and the compiler then waits as if the store had not been issued -- i.e. for it.
    const int j = lane & 15, k4 = lane >> 4;
    const int q = h16_half_q(hh, e), r = (e >> 1) & 3, ph = e & 1;   // as h16_epilogue's order
    const int row0 = 4 * g;
    float *const outi = out + (o.img < 0 ? 0 : o.img) * bt.out_stride;
    const size_t HW = (size_t)Hout * Wout;
    const float bq[4] = {b4.x, b4.y, b4.z, b4.w};
    const floatx4 &c = acc[(r * 2 + ph) * 4 + q];
    const bool rok = o.img >= 0 && o.ty0 + row0 + r < Hout;   // wave-uniform
    const int x = o.tx0 + 16 * ph + j;
    const bool ok = rok && x < Wout;
    float o4[4];
#pragma unroll
    for (int k = 0; k < 4; k++)
        o4[k] = fmaxf(fmaf(c[k], OSPL ? o.unscale * o.oscale : o.unscale, OSPL ? bq[k] * o.oscale : bq[k]), 0.f);
    const float4 ov = make_float4(o4[0], o4[1], o4[2], o4[3]);
    const uint32_t m = max(max(__float_as_uint(ov.x), __float_as_uint(ov.y)), max(__float_as_uint(ov.z), __float_as_uint(ov.w)));
    amax = ok ? max(amax, m) : amax;
    if (OSPL) {
        u32x2 hw2, lw2;
        xp_split16s(ov, hw2, lw2);
        const u32x4 v4 = xp_pair_parts<false>(hw2, lw2);
        const __amdgpu_buffer_rsrc_t rs =
            xp_rsrc(reinterpret_cast<char *>(outi) + ((size_t)((q >> 1) * 8 + 2 * (q & 1)) * HW + (size_t)o.ty0 * Wout) * 16);
        const uint32_t ospl_lane = (uint32_t)((k4 & 1) * 4 + (k4 >> 1)) * ((uint32_t)HW * 16u);
        __builtin_amdgcn_raw_buffer_store_b128(v4, rs, ok ? ospl_lane + (uint32_t)x * 16u : XP_OOB,
                                               (uint32_t)((row0 + r) * Wout) * 16u, 0);
        asm volatile("s_nop 7\n\ts_nop 1" ::"v"(v4) : "memory");
    } else {
        const __amdgpu_buffer_rsrc_t rs = xp_rsrc(OUT_CB ? outi + ((size_t)q * HW + (size_t)o.ty0 * Wout) * 16
                                                         : outi + (size_t)o.ty0 * Wout * NF);
        xp_st4(ov, rs, ok ? (uint32_t)(OUT_CB ? x * 64 + 16 * k4 : x * 256 + 64 * q + 16 * k4) : XP_OOB,
               (uint32_t)((row0 + r) * Wout) * (OUT_CB ? 64u : 256u));
        asm volatile("s_nop 7\n\ts_nop 1" ::"v"(__builtin_bit_cast(u32x4, ov)) : "memory");
    }
}

// Layers 3..L, f16x3; IN_CB / OUT_CB: c-block-major activations [cblk16][h][w][16] (the tower's
// intermediate layout) or [h][w][64]; LAST writes the [h][w][64] features (+ the optional split
// planes and norm bounds: SPLIT, the last layer only).
// FIRST: layer 2 -- `in` is the padded image (Hin x Win floats), w1blob conv1's weights, computed by the
// stagers (h16_conv1_stager_loop; launch with H16_SMEM_FIRST bytes of LDS); outputs in any of the three
// activation layouts (OSPL: the split planes).
template <bool LAST, bool IN_CB, bool OUT_CB, bool SPLIT, bool ISPL = false, bool OSPL = false, bool FIRST = false>
__global__ __launch_bounds__(512) void conv64_h16_kernel(const float *__restrict__ in, int Hin, int Win,
                                                         const float *__restrict__ wkblob, float *__restrict__ out,
                                                         int Hout, int Wout, uint16_t *__restrict__ ohi,
                                                         uint16_t *__restrict__ olo, float *__restrict__ onrm, XpBatch bt,
                                                         const float *__restrict__ in_amax, float *__restrict__ out_amax,
                                                         const float *__restrict__ w1blob)
{
    static_assert(!FIRST || (!ISPL && !SPLIT && !LAST), "layer 2: the fp32 image in, activations out");
    extern __shared__ __attribute__((aligned(16))) char hsm[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    int tile = blockIdx.x;
    if (tile >= bt.ntiles) return;
    const float *hdr = wkblob + LK_F16 + LK_W;
    if (wave >= 4) {
        if (FIRST) h16_conv1_stager_loop(hsm, in, Hin, Win, bt, tid - XP_STAGERS, in_amax, hdr, w1blob);
        else if (ISPL) h16_dma_stager_loop(hsm, in, Hin, Win, bt, tid - XP_STAGERS);
        else h16_stager_loop<IN_CB>(hsm, in, Hin, Win, bt, tid - XP_STAGERS, in_amax, hdr);
        return;
    }
    if (OSPL) xp_publish_scale(FIRST, bt, in_amax, hdr, out_amax);
    const int g = __builtin_amdgcn_readfirstlane(wave);
    float *lbias = reinterpret_cast<float *>(hsm + H16_BIAS_OFF);
    if (wave == 0) lbias[lane] = wkblob[lane];   // published by the first barrier below
    const float4 *lbias4 = reinterpret_cast<const float4 *>(lbias);
    const __amdgpu_buffer_rsrc_t ra = xp_rsrc(wkblob + LK_F16);
    // the lane's A-fragment byte offset: cb16 = 2 cb + (lane >> 5), channel half (lane >> 4) & 1, n & 15
    const uint32_t avoff = (uint32_t)((lane >> 5) * (9 * 2 * 64) + ((lane >> 4) & 1) * 32 + (lane & 15)) * 16u;
    // the lane's B base: plane quarter lane >> 4, pixel (4g, lane & 15) of the input tile
    const int bbase = (lane >> 4) * H16_PLANE + ((4 * g) * XP_IX + (lane & 15)) * 16;
    // c-blocks feeding each B fragment to all four quarters (h16_cblock12), except the last layer with
    // split outputs (its epilogue would spill 13 VGPRs with the 2-tap A ring)
    constexpr bool B12 = H16_B12 == 2 ? !(LAST && SPLIT) : H16_B12 == 1 ? !LAST && !FIRST : false;
    constexpr int BRD = 3;
    H16A abuf[4];   // h16_cblock: slots 0-2
    abuf[0] = h16_afrag(ra, avoff, 0, 0);
    abuf[1] = h16_afrag(ra, avoff, 0, 1);
    __syncthreads();

    int sc_img = -1;
    float sc_u = 1.0f, sc_o = 1.0f;
    uint32_t amax_run = 0u;
    int amax_img = -1;
    int cur = 0;
    // (not with split outputs: that store body is too large for the unrolled c-block; not in layer 2: spills)
#ifndef H16_OVL_FIRST
#define H16_OVL_FIRST 0
#endif
    constexpr bool OVL = H16_OVL_K > 0 && B12 && !LAST && !OSPL && (!FIRST || H16_OVL_FIRST);
    constexpr int OBRD = FIRST && H16_OVL_FIRST == 2 ? 2 : BRD;
    if constexpr (OVL) {
        constexpr int K = H16_OVL_K;
        static_assert(K >= 2 && K <= 8 && K % 2 == 0, "overlap depth: an even number of taps");
        abuf[1] = ovl_afrag(ra, avoff, K, 1);   // items 0..2 requested (item 0 above)
        abuf[2] = ovl_afrag(ra, avoff, K, 2);
        floatx4 acc[32];
#pragma unroll
        for (int i = 0; i < 32; i++) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
        H16Out prev{-1, 0, 0, 1.0f, 1.0f};
        float4 eb;   // the next epilogue store's bias
        // a half's bound into the running per-image word (flushed when the image changes, as h16_epilogue's)
        auto merge = [&](uint32_t a, const H16Out &o) {
            if (OSPL) a = __float_as_uint(__uint_as_float(a) / o.oscale);   // exact: a power of two
            if (o.img != amax_img) {
                xp_flush_amax(amax_run, amax_img, lane, out_amax, bt.amax_stride);
                amax_img = o.img;
            }
            amax_run = max(amax_run, a);
        };
        for (; tile < bt.ntiles; tile += gridDim.x) {
            H16Out cu;
            xp_tile(bt, tile, cu.img, cu.ty0, cu.tx0);
            uint32_t a1 = 0u;
            // c-block 0, carrying the previous tile's H1 stores
            h16_cblock_ovl<0, K, OBRD>(acc, abuf, ra, avoff, hsm + cur * H16_STAGE + bbase, [&](auto tag, int e) {
                // (the first tile of a wave: prev.img < 0, the stores fall out of range)
                if constexpr (decltype(tag)::value == 0) eb = lbias4[4 * h16_half_q(1, e) + (lane >> 4)];
                else h16_store_half<OUT_CB, OSPL>(acc, 1, e, lane, g, prev, eb, out, Hout, Wout, bt, a1);
            });
            if (prev.img >= 0) merge(a1, prev);
            __syncthreads();
            cur ^= 1;
            if (cu.img != sc_img) {
                const float *am = in_amax + cu.img * bt.amax_stride;
                if (ISPL) {
                    sc_u = hdr[0] / am[XP_SCALE_WORD];
                } else {
                    float s_unused;
                    xp_scales(FIRST, am, hdr, s_unused, sc_u);
                }
                if (OSPL) sc_o = xp_out_scale(FIRST, am, hdr);
                sc_img = cu.img;
            }
            cu.unscale = sc_u;
            cu.oscale = sc_o;
            uint32_t a0 = 0u;
            // c-block 1, carrying this tile's H0 stores
            h16_cblock_ovl<1, K, OBRD>(acc, abuf, ra, avoff, hsm + cur * H16_STAGE + bbase, [&](auto tag, int e) {
                if constexpr (decltype(tag)::value == 0) eb = lbias4[4 * h16_half_q(0, e) + (lane >> 4)];
                else h16_store_half<OUT_CB, OSPL>(acc, 0, e, lane, g, cu, eb, out, Hout, Wout, bt, a0);
            });
            merge(a0, cu);
            __syncthreads();
            cur ^= 1;
            prev = cu;
        }
        if (prev.img >= 0) {   // the last tile's H1
            uint32_t a1 = 0u;
#pragma unroll
            for (int e = 0; e < 16; e++)
                h16_store_half<OUT_CB, OSPL>(acc, 1, e, lane, g, prev, lbias4[4 * h16_half_q(1, e) + (lane >> 4)], out,
                                             Hout, Wout, bt, a1);
            merge(a1, prev);
        }
        xp_flush_amax(amax_run, amax_img, lane, out_amax, bt.amax_stride);
        return;
    }
    for (; tile < bt.ntiles; tile += gridDim.x) {
        int img, ty0, tx0;
        xp_tile(bt, tile, img, ty0, tx0);
        floatx4 acc[32];
#pragma unroll
        for (int i = 0; i < 32; i++) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
        // cb 0, then cb 1 and the epilogue (as a lambda: B12 unrolls the pair, the 3-slot form keeps a loop)
        auto cstep = [&](int cb) {
            if constexpr (B12) {
                if (cb == 0) h16_cblock12<0, BRD>(acc, abuf, ra, avoff, 0, 1, hsm + cur * H16_STAGE + bbase);
                else h16_cblock12<2, BRD, false>(acc, abuf, ra, avoff, 1, 0, hsm + cur * H16_STAGE + bbase);
            } else {
                h16_cblock(acc, abuf, ra, avoff, cb, cb ^ 1, hsm + cur * H16_STAGE + bbase);
            }
            if (cb == H16_NCB - 1) {
                if (img != sc_img) {
                    const float *am = in_amax + img * bt.amax_stride;
                    if (ISPL) {   // the writer's published 2^sigma
                        sc_u = hdr[0] / am[XP_SCALE_WORD];
                    } else {
                        float s_unused;
                        xp_scales(FIRST, am, hdr, s_unused, sc_u);
                    }
                    if (OSPL) sc_o = xp_out_scale(FIRST, am, hdr);
                    sc_img = img;
                }
                // B12: the next tile's first tap (c-block 0, phase 0: slots 0, 1), requested halfway through
                auto mid = [&]() {
                    if constexpr (B12) {
                        abuf[0] = h16_afrag(ra, avoff, 0, 0);
                        abuf[1] = h16_afrag(ra, avoff, 0, 1);
                    }
                };
                h16_epilogue<LAST, OUT_CB, SPLIT, OSPL>(acc, lane, g, img, ty0, tx0, sc_u, lbias4, out, Hout, Wout, bt, ohi,
                                                       olo, onrm, amax_run, amax_img, out_amax, sc_o, mid);
            }
            __syncthreads();
            cur ^= 1;
        };
        if constexpr (B12) {
            cstep(0);
            cstep(1);
        } else {
#pragma unroll 1
            for (int cb = 0; cb < H16_NCB; cb++) cstep(cb);
        }
    }
    if (!LAST) xp_flush_amax(amax_run, amax_img, lane, out_amax, bt.amax_stride);
}

}  // namespace sde
