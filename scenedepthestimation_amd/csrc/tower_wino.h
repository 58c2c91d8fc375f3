// tower_wino.h -- Winograd F(2x2, 3x3) for the MC-CNN tower's 64 -> 64 layers (included by
// tower.hip; f16x3 arithmetic).  Replaces, for layers 3..L (mc_cnn_brunch.py:31-48, conv
// :70-92), the direct conv64_x6p_kernel: per 2x2 output block the 3x3 correlation of a 4x4
// input patch d with the weights g is
//     Y = A^T [ sum_cin (G g G^T) .* (B^T d B) ] A,
//     B^T = [[1,0,-1,0],[0,1,1,0],[0,-1,1,0],[0,1,0,-1]],  G = [[1,0,0],[.5,.5,.5],[.5,-.5,.5],[0,0,1]],
//     A^T = [[1,1,1,0],[0,1,-1,-1]]
// -- 16 elementwise products per 4 outputs instead of 36: 2.25x fewer MFMA products.  The
// 16 "positions" xi = 4i + j are 16 independent GEMMs M[xi] = U[xi] (64 cout x 64 cin) x
// V[xi] (64 cin x tiles), run on v_mfma_f32_32x32x16_f16 with the same exact power-of-two
// scaled 2-part fp16 split as the direct kernel (3 partial products, fp32 accumulation):
// U = G g G^T is formed in fp64 on the host (sde_tower_pack_weights), scaled by 2^tau_u and
// split; V = B^T d B is formed in fp32 on the device (|V| <= 4 max|d|, so the activations'
// bound word times 4 sets sigma) and split by the threads that form it.
//
// Pass = 4 x 8 Winograd tiles = 8 x 16 outputs (10 x 18 input pixels).  512 threads, 8
// waves (two per SIMD), persistent over the batch's passes.  A pass is 4 steps, one per
// 16-channel c-block:
// * wave w owns positions xi = 2w, 2w+1 (row a = w >> 1 of the 4 x 4 grid) for all 64 output
//   channels (2 M-tiles) and the pass's 32 tiles (one N-tile): 4 accumulators, 12 MFMAs per
//   step.  Its U fragments -- 2 positions x 2 M-tiles x 4 c-blocks x 2 parts -- stay in 128
//   VGPRs for the whole kernel: no weight traffic after the prologue;
// * the raw input of a step (180 pixels x 64 B) is copied global -> LDS by buffer loads that
//   write LDS directly (no VGPRs), three steps ahead into a ring of three buffers; reads past
//   the input (right and bottom edges) return 0 -- the zero padding of the valid convolution;
// * V of step g+1 is formed from the raw ring while step g's MFMAs run: waves 0-3 the
//   transform rows 0-1 (positions 0-7), waves 4-7 rows 2-3, one (tile, channel pair) per
//   thread; two V stages [xi][part][channel half][tile][8 fp16] (a B fragment is one
//   conflict-free ds_read_b128; the halves padded so the transform's stores spread over 32
//   banks);
// * one barrier per step (raw s_barrier after counted vmcnt / lgkmcnt waits: the LDS-DMA
//   copies stay in flight across it);
// * epilogue, per M-tile: each wave folds its two positions of row a into the output
//   transform's column sums P_w[j] = sum_b M[a][b] A^T[j][b] and parks them in the stages;
//   every thread then sums the 8 waves' parts for 4 channels of one output column j of one
//   tile: Y[0][j] = sum_{a<3} (P_{2a} + P_{2a+1})[j], Y[1][j] = (P_2 + P_3 - P_4 - P_5 - P_6 -
//   P_7)[j]; unscale (exact), bias, ReLU + bound word, or (last layer) the L2 norm over the
//   64 channels of a pixel (8 lanes of one wave hold them).
// Error: V's fp32 transform rounds once or twice per value (2^-24 of |V| <= 4 max|d|), U is
// exact to 2^-22 after the split, the three partial products and fp32 accumulation as in
// the direct kernel, and the output transform adds <= 6 fp32 terms: fp32-level (measured
// against the fp64 restatement in the tests: below the direct kernel's error).
#pragma once

namespace sde {

constexpr int WN_TY = 8, WN_TX = 16;                  // outputs per pass
constexpr int WN_TTY = 4, WN_TTX = 8;                 // Winograd tiles per pass
constexpr int WN_NT = WN_TTY * WN_TTX;                // 32 tiles (one MFMA N-tile)
constexpr int WN_IY = WN_TY + 2, WN_IX = WN_TX + 2;   // input region 10 x 18
constexpr int WN_RAW_INS = 12;                        // LDS-DMA wave-instructions per step (768 >= 720 chunks)
constexpr int WN_RAW_BYTES = WN_RAW_INS * 64 * 16;    // 12 KB per raw buffer
constexpr int WN_HALF = 576;                          // bytes of one channel half of a (xi, part) plane (32 x 16 + pad)
constexpr int WN_PLANE = 2 * WN_HALF;
constexpr int WN_STAGE = 32 * WN_PLANE;               // [xi 16][part 2] planes: 36,864 B
constexpr size_t WN_RAW_OFF = 2 * (size_t)WN_STAGE;
#ifndef WN_RING
#define WN_RING 5                                     // raw buffers: LDS-DMA runs WN_RING - 2 steps ahead of use
#endif
static_assert(WN_RING == 3 || WN_RING == 5, "wait counts below are derived for rings of 3 and 5");
constexpr size_t WN_BIAS_OFF = WN_RAW_OFF + WN_RING * (size_t)WN_RAW_BYTES;
constexpr size_t WN_SMEM = WN_BIAS_OFF + NF * sizeof(float);
static_assert(8 * 2 * WN_NT * 32 * 4 <= 2 * WN_STAGE, "P exchange fits the stages");
static_assert(WN_RAW_INS * 64 >= WN_IY * WN_IX * 4, "raw chunks");

typedef float wn_f2 __attribute__((ext_vector_type(2)));
typedef _Float16 wn_h2 __attribute__((ext_vector_type(2)));
constexpr uint32_t WN_OOB = 0x80000000u;   // a voffset past num_records: the load returns 0
#ifndef WN_VALU_PER_MFMA
#define WN_VALU_PER_MFMA 5
#endif

__device__ __forceinline__ void wn_tile(const XpBatch &bt, int t, int &img, int &ty0, int &tx0)
{
    img = t / bt.tiles_img;
    const int tl = t - img * bt.tiles_img;
    ty0 = (tl / bt.tiles_x) * WN_TY;
    tx0 = (tl % bt.tiles_x) * WN_TX;
}

// 2^sigma for V of a tile: |V| <= 4 |input| (four-term sums), bound word * 4 in [2^14, 2^15)
__device__ __forceinline__ void wn_scales(const float *__restrict__ in_amax, float tau_inv, float &s, float &unscale)
{
    const float bound = 4.0f * *in_amax;
    int e = 0;
    if (bound >= 1.17549435e-38f && bound <= 3.40282347e38f) e = (int)((__float_as_uint(bound) >> 23) & 255u) - 127;
    const int sigma = min(max(14 - e, -100), 100);
    s = ldexpf(1.0f, sigma);
    unscale = ldexpf(tau_inv, -sigma);
}

// Buffer descriptor on a wave-uniform base with num_records bytes (range-checked accesses).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wn_rsrc(const void *base, uint32_t bytes)
{
    const uintptr_t b = (uintptr_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((uintptr_t)hi << 32) | lo), 0,
                                             (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// x * s split into two fp16 parts (x * s = h + l + r, |r| <= 2^-22 |x s|), a channel pair packed
// (the residual x s - h is exact in fp32; v_fma_mix_f32 forms it from the packed fp16 h directly:
// fma(xs, 1, -h) rounds once, to the same bits as widening h and subtracting)
__device__ __forceinline__ void wn_split(wn_f2 x, float s, uint32_t &h, uint32_t &l)
{
    const wn_f2 xs = x * s;
    h = __builtin_bit_cast(uint32_t, __builtin_convertvector(xs, wn_h2));
    float r0, r1;
    asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(r0) : "v"(xs.x), "v"(h));
    asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(r1) : "v"(xs.y), "v"(h));
    l = __builtin_bit_cast(uint32_t, __builtin_convertvector((wn_f2){r0, r1}, wn_h2));
}

// Epilogue LDS accesses as inline asm: the compiler's wait insertion treats any LDS access it
// cannot separate from an LDS-DMA target as dependent on it and drains vmcnt(0) -- every copy in
// flight -- before it.  The P exchange never touches the raw ring; its ordering is explicit
// (lgkmcnt waits + barriers).
__device__ __forceinline__ uint32_t wn_lds(const void *p)
{
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
typedef float wn_f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void wn_ds_write4(uint32_t a, float4 v)
{
    const wn_f4 x = {v.x, v.y, v.z, v.w};
    asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(x) : "memory");
}

// P_0..P_3 (+ the bias quad) and P_4..P_7 of the final phase: P_{2aa} at + aa * 16 KB,
// P_{2aa+1} at + 8 KB; one wait per batch
__device__ __forceinline__ void wn_read_p01(uint32_t pa, uint32_t ba, wn_f4 (&pr)[4], wn_f4 &b4)
{
    asm volatile(
        "ds_read_b128 %0, %5\n\tds_read_b128 %1, %5 offset:8192\n\t"
        "ds_read_b128 %2, %5 offset:16384\n\tds_read_b128 %3, %5 offset:24576\n\t"
        "ds_read_b128 %4, %6\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(pr[0]), "=&v"(pr[1]), "=&v"(pr[2]), "=&v"(pr[3]), "=&v"(b4)
        : "v"(pa), "v"(ba)
        : "memory");
}
__device__ __forceinline__ void wn_read_p23(uint32_t pa, wn_f4 (&pr)[4])
{
    asm volatile(
        "ds_read_b128 %0, %4 offset:32768\n\tds_read_b128 %1, %4 offset:40960\n\t"
        "ds_read_b128 %2, %4 offset:49152\n\tds_read_b128 %3, %4 offset:57344\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(pr[0]), "=&v"(pr[1]), "=&v"(pr[2]), "=&v"(pr[3])
        : "v"(pa)
        : "memory");
}

// LDS-DMA chunk of wave-instruction ins, lane ln: pixel (chunk >> 2) of the 10 x 18 region,
// channels 4 (chunk & 3).. -- its byte offset from the region's origin (WN_OOB past the region)
template <bool IN_CB>
__device__ __forceinline__ uint32_t wn_loff(int ins, int ln, int Win)
{
    const int ch = ins * 64 + ln, px = ch >> 2, q = ch & 3;
    const int iy = px / WN_IX, ix = px - iy * WN_IX;
    return px < WN_IY * WN_IX ? (uint32_t)(iy * Win + ix) * (IN_CB ? 64u : 256u) + 16u * q : WN_OOB;
}

struct WnA {
    f16x8 h, l;
};

// s_waitcnt immediates (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14])
constexpr int WN_LGKM0 = 0xC07F;                                     // lgkmcnt(0)
constexpr int WN_EPI_STORES = 4;   // buffer stores per thread in a pass's epilogue (unconditional)
constexpr int wn_vmcnt(int n) { return 0x0F70 | (n & 15) | ((n >> 4) << 14); }

template <bool LAST, bool IN_CB, bool OUT_CB>
__global__ __launch_bounds__(512) void wino_kernel(const float *__restrict__ in, int Hin, int Win,
                                                   const float *__restrict__ wkblob, float *__restrict__ out,
                                                   int Hout, int Wout, XpBatch bt, const float *__restrict__ in_amax,
                                                   float *__restrict__ out_amax)
{
    extern __shared__ __attribute__((aligned(16))) char wsm[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    if ((int)blockIdx.x >= bt.ntiles) return;
    const int npass = (bt.ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1;
    const int nsteps = 4 * npass;
    const float tau_inv = wkblob[LK_WHDR];
    float *lbias = reinterpret_cast<float *>(wsm + WN_BIAS_OFF);
    if (tid < NF) lbias[tid] = wkblob[tid];

    // resident U fragments: positions 2w + p, M-tile m, c-block cb, parts h / l
    WnA u[2][2][4];
    {
        const __amdgpu_buffer_rsrc_t ru = wn_rsrc(wkblob + LK_WINO, (uint32_t)LK_WU * 2u);
#pragma unroll
        for (int p = 0; p < 2; p++)
#pragma unroll
            for (int m = 0; m < 2; m++)
#pragma unroll
                for (int cb = 0; cb < 4; cb++) {
                    const int so = (((2 * w + p) * 2 + m) * XP_NCB + cb) * 2048;
                    u[p][m][cb].h = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(ru, 16u * lane, so, 0));
                    u[p][m][cb].l = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(ru, 16u * lane, so + 1024, 0));
                }
    }

    // LDS-DMA of step g's raw input into raw buffer g % 3: wave w copies chunks 64 ins + lane for
    // ins in {w, w + 8} (< 12) -- pixel (chunk >> 2) of the 10 x 18 region, channels 4 (chunk & 3)..
    // A pass's descriptor starts at its tile origin (per-pass SGPR work); the lane offsets are
    // fixed.  Reads past the bottom of the input return 0 (past num_records); a column past the
    // right edge reads the next row's first pixels instead -- they only reach M[.][3] (B^T d B's
    // column 3 holds d's column 3 alone), i.e. output column 1 of a tile whose column 1 is past
    // Wout and never stored.
    const int nins = w + 8 < WN_RAW_INS ? 2 : 1;
    // (lane offsets: recomputed per issue from an opaque lane copy, a few VALU; held across the
    // loop they would take registers next to the resident U fragments)
    const uint32_t plane_bytes = (uint32_t)Hin * Win * (IN_CB ? 64u : 256u);
    auto pass_src = [&](int pass, const float *&base, uint32_t &bytes) {
        int img, ty0, tx0;
        wn_tile(bt, (int)blockIdx.x + pass * (int)gridDim.x, img, ty0, tx0);
        const uint32_t o = (uint32_t)(ty0 * Win + tx0);
        base = in + (size_t)img * bt.in_stride + (size_t)o * (IN_CB ? 16 : 64);
        bytes = plane_bytes - o * (IN_CB ? 64u : 256u);
    };
    auto issue = [&](int g, const float *base, uint32_t bytes) {
        const int cb = g & 3;
        const __amdgpu_buffer_rsrc_t rs = IN_CB ? wn_rsrc(base + (size_t)cb * Hin * Win * 16, bytes)
                                                : wn_rsrc(base + cb * 16, bytes - 64u * cb);
        char *rb = wsm + WN_RAW_OFF + (size_t)(g % WN_RING) * WN_RAW_BYTES;
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const uint32_t lo0 = wn_loff<IN_CB>(w, ln, Win), lo1 = wn_loff<IN_CB>(w + 8, ln, Win);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void *)(rb + w * 1024), 16,
                                                 lo0, 0, 0, 0);
        if (nins == 2)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void *)(rb + (w + 8) * 1024),
                                                     16, lo1, 0, 0, 0);
    };
    // the end of a step: this wave's LDS stores done and every LDS-DMA copy older than the ones
    // just issued landed, then the barrier (its readers read after it)
    // after_epilogue (step 0 of a pass > 0): the previous pass's WN_EPI_STORES output stores were
    // issued after the copy this wait is for and before the one just issued; vmcnt retires in
    // issue order, so they need not have completed
    // The end of step g: the copy of step g + 2 (issued at step g + 2 - WN_RING) has landed -- the
    // WN_RING - 2 issues after it (nins copies each) may stay in flight, and so may the output
    // stores of an epilogue that ran in between (after_epilogue: WN_EPI_STORES of them; vmcnt
    // retires in issue order).  Past the last issue: drain.
    auto sync = [&](bool issued, bool after_epilogue) {
        constexpr int K = WN_RING - 2;
        if (issued) {
            if (after_epilogue) {
                if (nins == 2) __builtin_amdgcn_s_waitcnt(wn_vmcnt(2 * K + WN_EPI_STORES));
                else __builtin_amdgcn_s_waitcnt(wn_vmcnt(K + WN_EPI_STORES));
            } else {
                if (nins == 2) __builtin_amdgcn_s_waitcnt(wn_vmcnt(2 * K));
                else __builtin_amdgcn_s_waitcnt(wn_vmcnt(K));
            }
        } else {
            __builtin_amdgcn_s_waitcnt(wn_vmcnt(0));
        }
        __builtin_amdgcn_s_waitcnt(WN_LGKM0);
        __builtin_amdgcn_s_barrier();
    };

    // transform unit: tile (tty, ttx) of the pass, channel pair chp; half 0 forms rows 0-1 of V
    // (positions 0-7) from input rows 0-2, half 1 rows 2-3 from input rows 1-3
    const int half = __builtin_amdgcn_readfirstlane(tid >> 8), unit = tid & 255, chp = unit & 7, tl = unit >> 3, tty = tl >> 3, ttx = tl & 7;
    // The transform of a stage.  Rows of B^T d from three raw rows A, B, C (chosen per half; half
    // is wave-uniform):
    //   half 0: A = d0, B = d2, C = d1:  row 0 = A - B = d0 - d2,  row 1 = B + C = d1 + d2
    //   half 1: A = d2, B = d1, C = d3:  row 2 = A - B = d2 - d1,  row 3 = B - C = d1 - d3
    // (B + sg C as one fma with sg = +-1: exact product, one rounding -- the same bits as the
    // add / subtract), column by column; then (.) B along each row and the split of a position.
    const int traw = chp * 8 + ((2 * tty + half) * WN_IX + 2 * ttx) * 64;   // row d_{half}
    const int rowA = half == 0 ? 0 : 1, rowB = half == 0 ? 2 : 0, rowC = half == 0 ? 1 : 2;  // + d_{half}
    const float sgf = half == 0 ? 1.0f : -1.0f;
    const int tstage = (chp >> 2) * WN_HALF + tl * 16 + (chp & 3) * 4;
    auto transform = [&](int g, float s) {
        int tr = traw;   // opaque: one address add per step, not one hoisted register per ring buffer
        asm volatile("" : "+v"(tr));
        const char *rb = wsm + WN_RAW_OFF + (size_t)(g % WN_RING) * WN_RAW_BYTES + tr;
        const wn_f2 sg = {sgf, sgf};
        wn_f2 t[2][4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const wn_f2 ra = *reinterpret_cast<const wn_f2 *>(rb + (rowA * WN_IX + c) * 64);
            const wn_f2 rbv = *reinterpret_cast<const wn_f2 *>(rb + (rowB * WN_IX + c) * 64);
            const wn_f2 rc = *reinterpret_cast<const wn_f2 *>(rb + (rowC * WN_IX + c) * 64);
            t[0][c] = ra - rbv;
            t[1][c] = __builtin_elementwise_fma(rc, sg, rbv);
        }
        char *stage = wsm + (size_t)(g & 1) * WN_STAGE + tstage;
#pragma unroll
        for (int ii = 0; ii < 2; ii++) {
            const wn_f2 v[4] = {t[ii][0] - t[ii][2], t[ii][1] + t[ii][2], t[ii][2] - t[ii][1], t[ii][1] - t[ii][3]};
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int xi = 4 * (2 * half + ii) + j;
                uint32_t h, l;
                wn_split(v[j], s, h, l);
                *reinterpret_cast<uint32_t *>(stage + (size_t)(xi * 2 + 0) * WN_PLANE) = h;
                *reinterpret_cast<uint32_t *>(stage + (size_t)(xi * 2 + 1) * WN_PLANE) = l;
            }
        }
    };

    int sc_img = -1;
    float s = 1.0f, unscale = 1.0f;
    auto scales_of = [&](int pass) {
        const int img = ((int)blockIdx.x + pass * (int)gridDim.x) / bt.tiles_img;
        if (img != sc_img) {
            wn_scales(in_amax + img * bt.amax_stride, tau_inv, s, unscale);
            sc_img = img;
        }
    };

    // prologue: three steps' raw input in flight, step 0 transformed into stage 0
    const float *src_cur, *src_nxt;
    uint32_t rec_cur, rec_nxt;
    pass_src(0, src_cur, rec_cur);
    for (int g = 0; g < WN_RING && g < nsteps; g++) {   // nsteps >= 4
        if (g < 4) {
            issue(g, src_cur, rec_cur);
        } else {
            const float *b1;
            uint32_t r1;
            pass_src(1, b1, r1);
            issue(g, b1, r1);
        }
    }
    __builtin_amdgcn_s_waitcnt(wn_vmcnt(0));   // (the U fragments too)
    __builtin_amdgcn_s_waitcnt(WN_LGKM0);
    __builtin_amdgcn_s_barrier();
    scales_of(0);
    transform(0, s);
    __builtin_amdgcn_s_waitcnt(WN_LGKM0);
    __builtin_amdgcn_s_barrier();

    uint32_t amax_run = 0u;
    int amax_img = -1;
    auto flush_amax = [&]() {
        if (amax_img < 0) return;
        uint32_t a = amax_run;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) a = max(a, (uint32_t)__shfl_xor((int)a, o, 64));
        if (lane == 0) atomicMax(reinterpret_cast<unsigned int *>(out_amax + amax_img * bt.amax_stride), a);
        amax_run = 0u;
    };

    const int bh = lane >> 5;
#pragma unroll 1
    for (int pass = 0; pass < npass; pass++) {
        int img, ty0, tx0;
        wn_tile(bt, (int)blockIdx.x + pass * (int)gridDim.x, img, ty0, tx0);
        scales_of(pass);
        const float unscale_pass = unscale, s_pass = s;
        if (pass + 1 < npass) pass_src(pass + 1, src_nxt, rec_nxt);
        else { src_nxt = src_cur; rec_nxt = rec_cur; }
        const float *src_nn = src_nxt;   // two passes ahead (WN_RING 5, step 3)
        uint32_t rec_nn = rec_nxt;
        if (WN_RING > 4 && pass + 2 < npass) pass_src(pass + 2, src_nn, rec_nn);
        floatx16 acc[2][2];
#pragma unroll
        for (int p = 0; p < 2; p++)
#pragma unroll
            for (int m = 0; m < 2; m++) acc[p][m] = floatx16{0};
#pragma unroll
        for (int cb = 0; cb < 4; cb++) {
            const int g = 4 * pass + cb;
            const char *sb = wsm + (size_t)(cb & 1) * WN_STAGE + bh * WN_HALF + (lane & 31) * 16;
            f16x8 vh[2], vl[2];
            auto bfrag = [&](int p) {
                const char *b = sb + (2 * w + p) * 2 * WN_PLANE;
                vh[p] = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4 *>(b));
                vl[p] = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4 *>(b + WN_PLANE));
            };
            // 12 MFMAs, position-major (the B fragments of one position live at a time); within a
            // position the two M-tile chains alternate, the small products l.h', h.l' first
            auto mfma = [&](int k) {
                const int p = k / 6, L = (k % 6) >> 1, m = k & 1;
                floatx16 &c = acc[p][m];
                const WnA &a = u[p][m][cb];
                c = __builtin_amdgcn_mfma_f32_32x32x16_f16(L == 0 ? a.l : a.h, L == 1 ? vl[p] : vh[p], c, 0, 0, 0);
            };
            auto mfma_all = [&]() {
                bfrag(0);
                bfrag(1);
#pragma unroll
                for (int k = 0; k < 12; k++) mfma(k);
            };
            mfma_all();
            if (cb < 3) transform(g + 1, s_pass);
            const bool more = g + WN_RING < nsteps;
            if (more) {                  // into raw buffer g % WN_RING, read by transform(g) a step ago
                constexpr int ahead = WN_RING;
                const int tp = (cb + ahead) >> 2;            // passes ahead of this one (compile-time)
                if (tp == 0) issue(g + ahead, src_cur, rec_cur);
                else if (tp == 1) issue(g + ahead, src_nxt, rec_nxt);
                else issue(g + ahead, src_nn, rec_nn);
            }
            // stores of an epilogue between the wanted copy's issue (step g + 2 - WN_RING) and now
            sync(more, pass > 0 && (WN_RING == 3 ? cb == 0 : cb < 3));
        }

        // ---- epilogue: output transform, per M-tile ------------------------------------------
        // P_w[j][tile][cout]: lane holds tile lane & 31, couts 8q + 4 bh + e; the float4 slots of a
        // tile's 32 couts XOR-swizzled by the tile (the 8 consecutive tiles of a ds_write_b128
        // group hit 8 bank groups)
        float *P = reinterpret_cast<float *>(wsm);
        // final phase: cout quad fq, output column j of tile ft -- 16 consecutive lanes cover two
        // adjacent pixels, a wave 16 pixels of one row: full 64-B runs of every c-block plane
        // (opaque copy of the thread index: keeps the epilogue's addresses inside the epilogue --
        // hoisted out of the pass loop they would pin registers next to the resident U fragments)
        int tid_e = tid;
        asm volatile("" : "+v"(tid_e));
        const int fq = tid_e & 7, fj = (tid_e >> 3) & 1, ft = tid_e >> 4;
        const int oy = ty0 + 2 * (ft >> 3), ox = tx0 + 2 * (ft & 7) + fj;
        const __amdgpu_buffer_rsrc_t orsrc =
            wn_rsrc(LAST ? out + (size_t)img * bt.pix_stride * NF : out + img * bt.out_stride, (uint32_t)Hout * Wout * 256u);
        float4 ylast[2][2];
        uint32_t amax = 0u;
#pragma unroll
        for (int m = 0; m < 2; m++) {
            const int tt = tid_e & 31;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                float e0[4], e1[4];
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const float m0 = acc[0][m][4 * q + e], m1 = acc[1][m][4 * q + e];
                    if ((w & 1) == 0) { e0[e] = m0 + m1; e1[e] = m1; }      // b = 0, 1
                    else { e0[e] = m0; e1[e] = -m0 - m1; }                  // b = 2, 3
                }
                const int co = 4 * ((2 * q + bh) ^ (tt & 7));
                const uint32_t pa = wn_lds(P + ((size_t)(w * 2 + 0) * WN_NT + tt) * 32 + co);
                wn_ds_write4(pa, make_float4(e0[0], e0[1], e0[2], e0[3]));
                wn_ds_write4(pa + WN_NT * 32 * 4, make_float4(e1[0], e1[1], e1[2], e1[3]));
            }
            __builtin_amdgcn_s_waitcnt(WN_LGKM0);
            __builtin_amdgcn_s_barrier();
            const int co = 4 * (fq ^ (ft & 7));
            // P_{2aa} at + aa * 16 KB, P_{2aa+1} at + 8 KB (two batches of reads, one wait each)
            static_assert(4 * WN_NT * 32 * 4 == 16384 && 2 * WN_NT * 32 * 4 == 8192, "P offsets");
            const uint32_t pa = wn_lds(P + ((size_t)fj * WN_NT + ft) * 32 + co);
            wn_f4 pr[4], b4;
            float4 S[4];
            wn_read_p01(pa, wn_lds(lbias + 32 * m + 4 * fq), pr, b4);
#pragma unroll
            for (int aa = 0; aa < 2; aa++) {
                const wn_f4 a0 = pr[2 * aa], a1 = pr[2 * aa + 1];
                S[aa] = make_float4(a0.x + a1.x, a0.y + a1.y, a0.z + a1.z, a0.w + a1.w);
            }
            wn_read_p23(pa, pr);
#pragma unroll
            for (int aa = 2; aa < 4; aa++) {
                const wn_f4 a0 = pr[2 * aa - 4], a1 = pr[2 * aa - 3];
                S[aa] = make_float4(a0.x + a1.x, a0.y + a1.y, a0.z + a1.z, a0.w + a1.w);
            }
            float4 Y[2];
            Y[0] = make_float4(fmaf(S[0].x + S[1].x + S[2].x, unscale_pass, b4.x),
                               fmaf(S[0].y + S[1].y + S[2].y, unscale_pass, b4.y),
                               fmaf(S[0].z + S[1].z + S[2].z, unscale_pass, b4.z),
                               fmaf(S[0].w + S[1].w + S[2].w, unscale_pass, b4.w));
            Y[1] = make_float4(fmaf(S[1].x - S[2].x - S[3].x, unscale_pass, b4.x),
                               fmaf(S[1].y - S[2].y - S[3].y, unscale_pass, b4.y),
                               fmaf(S[1].z - S[2].z - S[3].z, unscale_pass, b4.z),
                               fmaf(S[1].w - S[2].w - S[3].w, unscale_pass, b4.w));
#pragma unroll
            for (int i = 0; i < 2; i++) {
                if (LAST) {
                    ylast[m][i] = Y[i];
                    continue;
                }
                const int c0 = 32 * m + 4 * fq;
                const int y = oy + i;
                const float4 o = make_float4(fmaxf(Y[i].x, 0.f), fmaxf(Y[i].y, 0.f), fmaxf(Y[i].z, 0.f), fmaxf(Y[i].w, 0.f));
                const bool ok = y < Hout && ox < Wout;
                if (ok)
                    amax = max(amax, max(max(__float_as_uint(o.x), __float_as_uint(o.y)),
                                         max(__float_as_uint(o.z), __float_as_uint(o.w))));
                // every lane stores (past the edge: an offset past num_records, dropped) -- a fixed
                // count of stores per wave for the next pass's vmcnt wait
                const uint32_t off = OUT_CB ? (((uint32_t)(c0 >> 4) * Hout + y) * Wout + ox) * 64u + 4u * (c0 & 15)
                                            : ((uint32_t)y * Wout + ox) * 256u + 4u * c0;
                const u32x4 od = __builtin_bit_cast(u32x4, o);
                __builtin_amdgcn_raw_buffer_store_b128(od, orsrc, ok ? off : WN_OOB, 0, 0);
                // the store's data registers stay untouched for >= 9 wait states ("store-data
                // overwrite"; _isa_lint.MFMA_STORE_DATA_WINDOW)
                asm volatile("s_nop 7\n\ts_nop 1" ::"v"(od));
            }
            __builtin_amdgcn_s_waitcnt(WN_LGKM0);
            __builtin_amdgcn_s_barrier();     // the P reads are done before P (or a stage) is rewritten
        }
        if (LAST) {
            // a pixel's 64 channels: the 8 consecutive lanes of one wave (fq) x 2 M-tiles x 4
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const float4 a = ylast[0][i], b = ylast[1][i];
                float ss = a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w + b.x * b.x + b.y * b.y + b.z * b.z + b.w * b.w;
                ss += __shfl_xor(ss, 1, 64);
                ss += __shfl_xor(ss, 2, 64);
                ss += __shfl_xor(ss, 4, 64);
                const float inv = 1.0f / sqrtf(fmaxf(ss, 1e-12f));
                const int y = oy + i;
                const uint32_t off = y < Hout && ox < Wout ? ((uint32_t)y * Wout + ox) * 256u + 16u * fq : WN_OOB;
                const u32x4 oa = __builtin_bit_cast(u32x4, make_float4(a.x * inv, a.y * inv, a.z * inv, a.w * inv));
                const u32x4 ob = __builtin_bit_cast(u32x4, make_float4(b.x * inv, b.y * inv, b.z * inv, b.w * inv));
                __builtin_amdgcn_raw_buffer_store_b128(oa, orsrc, off, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(ob, orsrc, off + 128u, 0, 0);
                asm volatile("s_nop 7\n\ts_nop 1" ::"v"(oa), "v"(ob));   // >= 9 wait states, as above
            }
        } else {
            // the bound word of an image: one atomic per wave and image (a flush when the passes move
            // to the next image and at the end), not per pass -- every workgroup maxes into the same
            // word, and per-pass atomics serialise on it
            if (img != amax_img) {
                flush_amax();
                amax_img = img;
            }
            amax_run = max(amax_run, amax);
        }
        // the next pass's first stage (its raw input landed at the wait of this pass's step 2)
        if (pass + 1 < npass) {
            scales_of(pass + 1);
            transform(4 * (pass + 1), s);
            __builtin_amdgcn_s_waitcnt(WN_LGKM0);
            __builtin_amdgcn_s_barrier();
        }
        src_cur = src_nxt;
        rec_cur = rec_nxt;
    }
    if (!LAST) flush_amax();
    // drain: no LDS-DMA copy may be in flight when the workgroup ends
    __builtin_amdgcn_s_waitcnt(wn_vmcnt(0));
}

}  // namespace sde
