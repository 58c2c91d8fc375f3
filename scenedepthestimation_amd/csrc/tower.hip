// tower.hip -- MC-CNN-fast Siamese branch on fp32 MFMA (gfx950).
//
// Replaces mc_cnn_brunch.py:31-48 (Net.construct) + :70-92 (conv) as run by
// compute_feature (process_functional.py:21-39): nlayers x [3x3 VALID conv,
// bias, ReLU] (no ReLU on the last), then tf.nn.l2_normalize over channels.
//
// Layers 2..n are an implicit GEMM on v_mfma_f32_32x32x2_f32 (exact f32 in /
// f32 accumulate, the 157 TF fp32 matrix rate): out[n][pixel] = sum over
// (tap, c) of W[tap][n][c] * in[pixel + tap][c].  A = weights (M = 64 output
// maps = 2 tiles of 32), B = input pixels (N = 32 pixels of one output row),
// K = 64 input maps per tap x 9 taps.
//
// Workgroup: 512 threads = 8 waves, output tile 8 rows x 32 columns, wave w
// owns output row w (2 accumulators of 32x32).  LDS: the (8+2) x (32+2) x 64
// input tile (87 KB) stays resident for all 9 taps; each tap's 64x64 weight
// slice (16 KB) is double-buffered (prefetched into registers during the
// previous tap's MFMAs).  Both LDS images are XOR-swizzled at 8-B granularity
// (pair slot ^= row & 31) so the 32 lanes of a ds_read_b64 half hit 64
// distinct banks.  Layer 1 (Cin = 1, 9 MACs per output) is computed on VALU
// straight into layer 2's LDS input tile, so its output never touches HBM; the
// last layer's epilogue L2-normalises each pixel (its 64 channels live in a
// lane pair l, l^32) before the store.
#include "sde_common.h"

#include <algorithm>
#include <cstring>

namespace sde {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int TW_TY = 8;                 // output rows per workgroup (one per wave)
constexpr int TW_TX = 32;                // output cols per workgroup (MFMA N)
constexpr int TW_IY = TW_TY + 2;         // input tile rows
constexpr int TW_IX = TW_TX + 2;         // input tile cols
constexpr int TW_NPIX = TW_IY * TW_IX;   // 340
constexpr int NF = 64;                   // feature maps (the reference's num_of_conv_feature_maps)
constexpr int L1_FLOATS = NF + 9 * NF;           // bias + [tap][n]
constexpr int LK_W = 9 * NF * NF;                // one [tap][n][c] plane, elements
// layer k >= 2: bias f32 [64] | W f32 [tap][n][c] | 3 bf16 planes [p][tap][n][c] (hi, mid, lo: W = hi+mid+lo)
constexpr int LK_FLOATS = NF + LK_W + 3 * LK_W / 2;

// float2 slot of channel pair `pair` (0..31) of pixel/row `p` in a swizzled 64-float row
__device__ __forceinline__ int pslot(int p, int pair) { return p * 32 + (pair ^ (p & 31)); }

// write channels 4q..4q+3 of row p (a float4) into the swizzled image
__device__ __forceinline__ void put4(float2 *img, int p, int q, float4 v)
{
    const int x = p & 31;
    const int unit = q ^ (x >> 1);
    float4 w = (x & 1) ? make_float4(v.z, v.w, v.x, v.y) : v;
    *reinterpret_cast<float4 *>(img + p * 32 + 2 * unit) = w;
}

// Load the 64x64 weight slice of one tap into registers (16 KB / 512 threads = 2 float4).
__device__ __forceinline__ void load_tap(const float *__restrict__ wk, int tap, float4 (&r)[2])
{
    const float4 *src = reinterpret_cast<const float4 *>(wk + (size_t)tap * NF * NF);
#pragma unroll
    for (int i = 0; i < 2; i++) r[i] = src[threadIdx.x + i * 512];
}

__device__ __forceinline__ void store_tap(float2 *wt, const float4 (&r)[2])
{
#pragma unroll
    for (int i = 0; i < 2; i++) {
        const int idx = threadIdx.x + i * 512;   // float4 index: n = idx / 16, q = idx % 16
        put4(wt, idx >> 4, idx & 15, r[i]);
    }
}

// Last-layer extras for the certified cost volume (see cost_volume.hip):
// bf16 hi/lo split planes of the output features (x = hi + lo + r, RNE) and
// an upper bound of each pixel's L2 norm.  A lane holds channels
// mt*32 + 8g + 4h + e (e = 0..3) of its pixel in v[mt][4g + e].
__device__ __forceinline__ void emit_split(const float (&v)[2][16], int h, size_t pix, uint16_t *ohi, uint16_t *olo)
{
    typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int mt = 0; mt < 2; mt++)
#pragma unroll
        for (int g = 0; g < 4; g++) {
            bf4 hv, lv;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const float x = v[mt][4 * g + e];
                const __bf16 hh = (__bf16)x;
                hv[e] = hh;
                lv[e] = (__bf16)(x - (float)hh);
            }
            const size_t o = pix * NF + mt * 32 + 8 * g + 4 * h;
            *reinterpret_cast<uint2 *>(ohi + o) = __builtin_bit_cast(uint2, hv);
            *reinterpret_cast<uint2 *>(olo + o) = __builtin_bit_cast(uint2, lv);
        }
}

__device__ __forceinline__ void emit_norm(const float (&v)[2][16], int h, size_t pix, float *onrm)
{
    float ss = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; r++) ss += v[0][r] * v[0][r] + v[1][r] * v[1][r];
    ss += __shfl_xor(ss, 32, 64);
    if (h == 0 && pix != (size_t)-1) onrm[pix] = sqrtf(ss) * 1.000004f;   // fp32 rounding bound (64 terms)
}

// FIRST: the input tile is conv1 (Cin = 1) of the padded image, computed here.
// LAST : no ReLU, L2-normalise over the 64 channels before the store.
template <bool FIRST, bool LAST>
__global__ __launch_bounds__(512) void conv64_mfma_kernel(const float *__restrict__ in, int Hin, int Win,
                                                          const float *__restrict__ w1blob,
                                                          const float *__restrict__ wkblob,
                                                          float *__restrict__ out, int Hout, int Wout,
                                                          uint16_t *__restrict__ ohi, uint16_t *__restrict__ olo,
                                                          float *__restrict__ onrm)
{
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    float2 *tile = smem;                          // TW_NPIX rows x 32 pairs
    float2 *wt0 = smem + TW_NPIX * 32;            // 64 rows x 32 pairs
    float2 *wt1 = wt0 + NF * 32;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int tx0 = blockIdx.x * TW_TX;
    const int ty0 = blockIdx.y * TW_TY;
    const float *bias = wkblob;
    const float *wk = wkblob + NF;

    float4 wreg[2];
    load_tap(wk, 0, wreg);

    // ---- input tile -> LDS ------------------------------------------------
    if (!FIRST) {
        // Hin x Win x 64 activations; tile pixel (iy, ix) = in[ty0+iy][tx0+ix]
        for (int idx = tid; idx < TW_NPIX * 16; idx += 512) {
            const int p = idx >> 4, q = idx & 15;
            const int iy = ty0 + p / TW_IX, ix = tx0 + p % TW_IX;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (iy < Hin && ix < Win) v = reinterpret_cast<const float4 *>(in + ((size_t)iy * Win + ix) * NF)[q];
            put4(tile, p, q, v);
        }
    } else {
        // `in` is the padded image (Hin x Win floats); conv1 output has (Hin-2) x (Win-2)
        // pixels.  Tile pixel (iy, ix) = relu(b1 + sum_tap img[ty0+iy+dy][tx0+ix+dx] * w1[tap][n]).
        const float *b1 = w1blob;
        const float *w1 = w1blob + NF;
        const int H1 = Hin - 2, W1 = Win - 2;
        for (int idx = tid; idx < TW_NPIX * 16; idx += 512) {
            const int p = idx >> 4, q = idx & 15;
            const int iy = ty0 + p / TW_IX, ix = tx0 + p % TW_IX;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (iy < H1 && ix < W1) {
                float im[9];
#pragma unroll
                for (int t = 0; t < 9; t++) im[t] = in[(size_t)(iy + t / 3) * Win + ix + t % 3];
                float a[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int n = 4 * q + j;
                    float s = 0.0f;
#pragma unroll
                    for (int t = 0; t < 9; t++) s = fmaf(im[t], w1[t * NF + n], s);
                    s += b1[n];
                    a[j] = s > 0.0f ? s : 0.0f;
                }
                v = make_float4(a[0], a[1], a[2], a[3]);
            }
            put4(tile, p, q, v);
        }
    }
    store_tap(wt0, wreg);
    __syncthreads();

    // ---- 9 taps x 16 k-quads x (2 M-tiles x 2 k-steps) MFMAs ----------------
    floatx16 acc0 = {0}, acc1 = {0};
    const int j = lane & 31;        // output column within the tile (B col / A row)
    const int h = lane >> 5;        // k half: channels 2h, 2h+1 of each k-quad
#pragma unroll 1
    for (int tap = 0; tap < 9; tap++) {
        const int ky = tap / 3, kx = tap - 3 * ky;
        float2 *wt = (tap & 1) ? wt1 : wt0;
        if (tap < 8) load_tap(wk, tap + 1, wreg);
        const int p = (wave + ky) * TW_IX + (j + kx);
#pragma unroll
        for (int t = 0; t < 16; t++) {
            const float2 b = tile[pslot(p, 2 * t + h)];
            const float2 a0 = wt[pslot(j, 2 * t + h)];
            const float2 a1 = wt[pslot(j + 32, 2 * t + h)];
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, b.x, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.x, b.x, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, b.y, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.y, b.y, acc1, 0, 0, 0);
        }
        if (tap < 8) store_tap((tap & 1) ? wt0 : wt1, wreg);
        __syncthreads();
    }

    // ---- epilogue: bias (+ReLU | L2-normalise), float4 stores ---------------
    // lane holds pixel column j, channels n = mt*32 + 8g + 4h + e in acc_mt[4g + e]
    float v[2][16];
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int n = 8 * (r >> 2) + 4 * h + (r & 3);
        v[0][r] = acc0[r] + bias[n];
        v[1][r] = acc1[r] + bias[32 + n];
    }
    if (!LAST) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
            v[0][r] = v[0][r] > 0.0f ? v[0][r] : 0.0f;
            v[1][r] = v[1][r] > 0.0f ? v[1][r] : 0.0f;
        }
    } else {
        float ss = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; r++) ss += v[0][r] * v[0][r] + v[1][r] * v[1][r];
        ss += __shfl_xor(ss, 32, 64);
        const float inv = 1.0f / sqrtf(fmaxf(ss, 1e-12f));
#pragma unroll
        for (int r = 0; r < 16; r++) { v[0][r] *= inv; v[1][r] *= inv; }
    }
    const int oy = ty0 + wave, ox = tx0 + j;
    if (oy < Hout && ox < Wout) {
        const size_t pix = (size_t)oy * Wout + ox;
        float *dst = out + pix * NF;
#pragma unroll
        for (int mt = 0; mt < 2; mt++)
#pragma unroll
            for (int g = 0; g < 4; g++)
                *reinterpret_cast<float4 *>(dst + mt * 32 + 8 * g + 4 * h) =
                    make_float4(v[mt][4 * g], v[mt][4 * g + 1], v[mt][4 * g + 2], v[mt][4 * g + 3]);
        if (LAST && ohi) emit_split(v, h, pix, ohi, olo);
    }
    if (LAST && onrm) emit_norm(v, h, oy < Hout && ox < Wout ? (size_t)oy * Wout + ox : (size_t)-1, onrm);
}

// ---------------------------------------------------------------------------
// bf16x6: fp32-accurate conv on the bf16 MFMA (v_mfma_f32_32x32x16_bf16).
// Every fp32 operand is split exactly into three bf16 parts, x = x0 + x1 + x2
// (RNE; each residual is exact in f32), and the six partial products with
// i + j <= 2 are accumulated in fp32 (the three dropped ones are < 2^-23 |ab|,
// below one fp32 rounding of the product).  16x the fp32 MFMA rate / 6 terms =
// 2.67x the fp32 matrix peak at fp32-level error.  Weights arrive pre-split
// (host packing); activations are split in registers from the fp32 LDS tile.
// Same tiling as conv64_mfma_kernel; LDS: fp32 tile (16-B XOR swizzle by pixel)
// + double-buffered 3 x [64 n][64 c] bf16 weight planes (16-B swizzle by n>>1).
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split3(float x, __bf16 &h, __bf16 &m, __bf16 &l)
{
    h = (__bf16)x;
    const float r1 = x - (float)h;
    m = (__bf16)r1;
    const float r2 = r1 - (float)m;
    l = (__bf16)r2;
}

// tile image: pixel p, 16-B chunk q (channels 4q..4q+3)
__device__ __forceinline__ int tslot(int p, int q) { return p * 16 + (q ^ (p & 15)); }
// weight plane image: row n, 16-B chunk c8 (channels 8c8..8c8+7)
__device__ __forceinline__ int wslot(int n, int c8) { return n * 8 + (c8 ^ ((n >> 1) & 7)); }

constexpr int X6_TILE_BYTES = TW_NPIX * NF * 4;             // 87,040
constexpr int X6_WBUF_BYTES = 3 * NF * NF * 2;              // 24,576 per tap buffer
constexpr size_t X6_SMEM = (size_t)X6_TILE_BYTES + 2 * X6_WBUF_BYTES;

template <bool FIRST, bool LAST>
__global__ __launch_bounds__(512) void conv64_x6_kernel(const float *__restrict__ in, int Hin, int Win,
                                                        const float *__restrict__ w1blob,
                                                        const float *__restrict__ wkblob,
                                                        float *__restrict__ out, int Hout, int Wout,
                                                        uint16_t *__restrict__ ohi, uint16_t *__restrict__ olo,
                                                        float *__restrict__ onrm)
{
    extern __shared__ __attribute__((aligned(16))) float4 smem4[];
    float4 *tile = smem4;                                                    // [340][16] float4
    uint4 *wbuf0 = reinterpret_cast<uint4 *>(smem4 + X6_TILE_BYTES / 16);    // [3][64][8] uint4
    uint4 *wbuf1 = wbuf0 + X6_WBUF_BYTES / 16;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int tx0 = blockIdx.x * TW_TX;
    const int ty0 = blockIdx.y * TW_TY;
    const float *bias = wkblob;
    const uint4 *planes = reinterpret_cast<const uint4 *>(wkblob + NF + LK_W);   // [3][9][64][8] uint4

    // weight prefetch: thread t moves chunk (n = t>>3, c8 = t&7) of each plane
    const int wn = tid >> 3, wc8 = tid & 7;
    const size_t wofs = (size_t)wn * 8 + wc8;
    constexpr size_t PSTRIDE = (size_t)9 * NF * 8;      // uint4 per plane
    uint4 wr0 = planes[wofs], wr1 = planes[PSTRIDE + wofs], wr2 = planes[2 * PSTRIDE + wofs];

    if (!FIRST) {
        for (int idx = tid; idx < TW_NPIX * 16; idx += 512) {
            const int p = idx >> 4, q = idx & 15;
            const int iy = ty0 + p / TW_IX, ix = tx0 + p % TW_IX;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (iy < Hin && ix < Win) v = reinterpret_cast<const float4 *>(in + ((size_t)iy * Win + ix) * NF)[q];
            tile[tslot(p, q)] = v;
        }
    } else {
        const float *b1 = w1blob;
        const float *w1 = w1blob + NF;
        const int H1 = Hin - 2, W1 = Win - 2;
        for (int idx = tid; idx < TW_NPIX * 16; idx += 512) {
            const int p = idx >> 4, q = idx & 15;
            const int iy = ty0 + p / TW_IX, ix = tx0 + p % TW_IX;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (iy < H1 && ix < W1) {
                float im[9];
#pragma unroll
                for (int t = 0; t < 9; t++) im[t] = in[(size_t)(iy + t / 3) * Win + ix + t % 3];
                float a[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int n = 4 * q + j;
                    float s = 0.0f;
#pragma unroll
                    for (int t = 0; t < 9; t++) s = fmaf(im[t], w1[t * NF + n], s);
                    s += b1[n];
                    a[j] = s > 0.0f ? s : 0.0f;
                }
                v = make_float4(a[0], a[1], a[2], a[3]);
            }
            tile[tslot(p, q)] = v;
        }
    }
    {
        const int ws = wslot(wn, wc8);
        wbuf0[ws] = wr0;
        wbuf0[NF * 8 + ws] = wr1;
        wbuf0[2 * NF * 8 + ws] = wr2;
    }
    __syncthreads();

    floatx16 acc0 = {0}, acc1 = {0};
    const int j = lane & 31;
    const int h = lane >> 5;
#pragma unroll 1
    for (int tap = 0; tap < 9; tap++) {
        const int ky = tap / 3, kx = tap - 3 * ky;
        const uint4 *wb = (tap & 1) ? wbuf1 : wbuf0;
        if (tap < 8) {
            const size_t o = (size_t)(tap + 1) * NF * 8 + wofs;
            wr0 = planes[o];
            wr1 = planes[PSTRIDE + o];
            wr2 = planes[2 * PSTRIDE + o];
        }
        const int p = (wave + ky) * TW_IX + (j + kx);
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const float4 x0 = tile[tslot(p, 4 * s + 2 * h)];
            const float4 x1 = tile[tslot(p, 4 * s + 2 * h + 1)];
            const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
            bf16x8 b0, b1, b2;
#pragma unroll
            for (int i = 0; i < 8; i++) {
                __bf16 hh, mm, ll;
                split3(xv[i], hh, mm, ll);
                b0[i] = hh; b1[i] = mm; b2[i] = ll;
            }
            const int c8 = 2 * s + h;
            const int s0 = wslot(j, c8), s1 = wslot(32 + j, c8);
            const bf16x8 a00 = __builtin_bit_cast(bf16x8, wb[s0]);
            const bf16x8 a01 = __builtin_bit_cast(bf16x8, wb[NF * 8 + s0]);
            const bf16x8 a02 = __builtin_bit_cast(bf16x8, wb[2 * NF * 8 + s0]);
            const bf16x8 a10 = __builtin_bit_cast(bf16x8, wb[s1]);
            const bf16x8 a11 = __builtin_bit_cast(bf16x8, wb[NF * 8 + s1]);
            const bf16x8 a12 = __builtin_bit_cast(bf16x8, wb[2 * NF * 8 + s1]);
            // small terms first, the leading product last
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a02, b0, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a12, b0, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a01, b1, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a11, b1, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a00, b2, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a10, b2, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a01, b0, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a11, b0, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a00, b1, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a10, b1, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a00, b0, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a10, b0, acc1, 0, 0, 0);
        }
        if (tap < 8) {
            uint4 *nb = (tap & 1) ? wbuf0 : wbuf1;
            const int ws = wslot(wn, wc8);
            nb[ws] = wr0;
            nb[NF * 8 + ws] = wr1;
            nb[2 * NF * 8 + ws] = wr2;
        }
        __syncthreads();
    }

    float v[2][16];
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int n = 8 * (r >> 2) + 4 * h + (r & 3);
        v[0][r] = acc0[r] + bias[n];
        v[1][r] = acc1[r] + bias[32 + n];
    }
    if (!LAST) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
            v[0][r] = v[0][r] > 0.0f ? v[0][r] : 0.0f;
            v[1][r] = v[1][r] > 0.0f ? v[1][r] : 0.0f;
        }
    } else {
        float ss = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; r++) ss += v[0][r] * v[0][r] + v[1][r] * v[1][r];
        ss += __shfl_xor(ss, 32, 64);
        const float inv = 1.0f / sqrtf(fmaxf(ss, 1e-12f));
#pragma unroll
        for (int r = 0; r < 16; r++) { v[0][r] *= inv; v[1][r] *= inv; }
    }
    const int oy = ty0 + wave, ox = tx0 + j;
    if (oy < Hout && ox < Wout) {
        const size_t pix = (size_t)oy * Wout + ox;
        float *dst = out + pix * NF;
#pragma unroll
        for (int mt = 0; mt < 2; mt++)
#pragma unroll
            for (int g = 0; g < 4; g++)
                *reinterpret_cast<float4 *>(dst + mt * 32 + 8 * g + 4 * h) =
                    make_float4(v[mt][4 * g], v[mt][4 * g + 1], v[mt][4 * g + 2], v[mt][4 * g + 3]);
        if (LAST && ohi) emit_split(v, h, pix, ohi, olo);
    }
    if (LAST && onrm) emit_norm(v, h, oy < Hout && ox < Wout ? (size_t)oy * Wout + ox : (size_t)-1, onrm);
}

// nlayers == 1: conv1 + L2 normalisation only (no ReLU on the last layer).
__global__ __launch_bounds__(256) void conv1_only_kernel(const float *__restrict__ img, int Hin, int Win,
                                                         const float *__restrict__ w1blob, float *__restrict__ out)
{
    const int Ho = Hin - 2, Wo = Win - 2;
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (int64_t)Ho * Wo) return;
    const int y = (int)(p / Wo), x = (int)(p % Wo);
    const float *b1 = w1blob, *w1 = w1blob + NF;
    float im[9];
    for (int t = 0; t < 9; t++) im[t] = img[(size_t)(y + t / 3) * Win + x + t % 3];
    float v[NF];
    float ss = 0.0f;
    for (int n = 0; n < NF; n++) {
        float s = 0.0f;
        for (int t = 0; t < 9; t++) s = fmaf(im[t], w1[t * NF + n], s);
        v[n] = s + b1[n];
        ss += v[n] * v[n];
    }
    const float inv = 1.0f / sqrtf(fmaxf(ss, 1e-12f));
    for (int n = 0; n < NF; n++) out[p * NF + n] = v[n] * inv;
}

// Per-image statistics: exact integer sum and sum of squares of the u8 pixels
// (one 64-bit atomic pair per workgroup), finalised in double by every reader.
__global__ __launch_bounds__(256) void image_sums_kernel(const uint8_t *__restrict__ img, int64_t n,
                                                         unsigned long long *__restrict__ sums)
{
    unsigned long long s = 0, q = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
    for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
        if (i + 3 < n && ((reinterpret_cast<uintptr_t>(img + i) & 3) == 0)) {
            const uint32_t w = *reinterpret_cast<const uint32_t *>(img + i);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const unsigned v = (w >> (8 * k)) & 255u;
                s += v;
                q += v * v;
            }
        } else {
            for (int64_t k = i; k < n && k < i + 4; k++) {
                const unsigned v = img[k];
                s += v;
                q += v * v;
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o, 64);
        q += __shfl_xor(q, o, 64);
    }
    __shared__ unsigned long long red[2][4];
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[0][wave] = s; red[1][wave] = q; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long ts = 0, tq = 0;
        for (int w = 0; w < 4; w++) { ts += red[0][w]; tq += red[1][w]; }
        atomicAdd(&sums[0], ts);
        atomicAdd(&sums[1], tq);
    }
}

// (I - mean) / std in float32 (match_single.py:40-41), zero border (process_functional.py:13-19).
__global__ __launch_bounds__(256) void znorm_pad_kernel(const uint8_t *__restrict__ img, int H, int W, int pad,
                                                        const unsigned long long *__restrict__ sums,
                                                        float *__restrict__ out)
{
    const int Wp = W + 2 * pad;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)(H + 2 * pad) * Wp) return;
    const double n = (double)H * W;
    const double mean_d = (double)sums[0] / n;
    const double var_d = fmax((double)sums[1] / n - mean_d * mean_d, 0.0);
    const float mean = (float)mean_d, stdv = (float)sqrt(var_d);
    const int y = (int)(i / Wp) - pad, x = (int)(i % Wp) - pad;
    float v = 0.0f;
    if (y >= 0 && y < H && x >= 0 && x < W) v = ((float)img[(size_t)y * W + x] - mean) / stdv;
    out[i] = v;
}

}  // namespace sde

using namespace sde;

static uint16_t f2bf_rne(float f)
{
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);   // NaN stays NaN
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

static float bf2f(uint16_t h)
{
    const uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

static constexpr size_t TW_SMEM = (size_t)(TW_NPIX * 32 + 2 * NF * 32) * sizeof(float2);

SDE_EXPORT int64_t sde_tower_packed_floats(int nlayers, int nf)
{
    if (nlayers < 1 || nf != NF) return -1;
    return (int64_t)L1_FLOATS + (int64_t)(nlayers - 1) * LK_FLOATS;
}

SDE_EXPORT int sde_tower_pack_weights(const float *const *hwio, const float *const *biases, int nlayers, int nf,
                                      float *packed)
{
    if (!hwio || !biases || !packed || nlayers < 1 || nf != NF) return SDE_ERR_ARG;
    float *o = packed;
    // layer 1: HWIO [3][3][1][64] is already [tap][n]
    for (int n = 0; n < NF; n++) o[n] = biases[0][n];
    for (int i = 0; i < 9 * NF; i++) o[NF + i] = hwio[0][i];
    o += L1_FLOATS;
    for (int l = 1; l < nlayers; l++) {
        for (int n = 0; n < NF; n++) o[n] = biases[l][n];
        float *w = o + NF;
        uint16_t *pl = reinterpret_cast<uint16_t *>(w + LK_W);
        for (int tap = 0; tap < 9; tap++)
            for (int c = 0; c < NF; c++)
                for (int n = 0; n < NF; n++) {
                    const size_t dsti = ((size_t)tap * NF + n) * NF + c;
                    const float x = hwio[l][((size_t)tap * NF + c) * NF + n];
                    w[dsti] = x;
                    const uint16_t h0 = f2bf_rne(x);
                    const float r1 = x - bf2f(h0);
                    const uint16_t h1 = f2bf_rne(r1);
                    const float r2 = r1 - bf2f(h1);
                    pl[dsti] = h0;
                    pl[LK_W + dsti] = h1;
                    pl[2 * (size_t)LK_W + dsti] = f2bf_rne(r2);
                }
        o += LK_FLOATS;
    }
    return SDE_OK;
}

SDE_EXPORT int64_t sde_tower_workspace_bytes(int H, int W, int nlayers, int nf)
{
    if (H <= 0 || W <= 0 || nlayers < 1 || nf != NF) return -1;
    if (nlayers <= 2) return 0;
    // two ping-pong activation buffers sized for layer 2's output
    const int64_t h2 = H + 2 * (nlayers - 2), w2 = W + 2 * (nlayers - 2);
    return 2 * h2 * w2 * NF * (int64_t)sizeof(float);
}

static void set_tower_attrs()
{
    static bool done = false;
    if (done) return;
    (void)hipFuncSetAttribute((const void *)conv64_mfma_kernel<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, TW_SMEM);
    (void)hipFuncSetAttribute((const void *)conv64_mfma_kernel<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, TW_SMEM);
    (void)hipFuncSetAttribute((const void *)conv64_mfma_kernel<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize, TW_SMEM);
    (void)hipFuncSetAttribute((const void *)conv64_mfma_kernel<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, TW_SMEM);
    (void)hipFuncSetAttribute((const void *)conv64_x6_kernel<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, X6_SMEM);
    (void)hipFuncSetAttribute((const void *)conv64_x6_kernel<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, X6_SMEM);
    (void)hipFuncSetAttribute((const void *)conv64_x6_kernel<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize, X6_SMEM);
    (void)hipFuncSetAttribute((const void *)conv64_x6_kernel<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, X6_SMEM);
    done = true;
}

// One launch: layer == 2 -> conv1+conv2 fused from the padded image (Hin x Win floats);
// layer > 2 -> one 64->64 conv on Hin x Win x 64 activations.  Output (Hin-4|Hin-2) x ... x 64.
static void launch_layer(const float *in, int Hin, int Win, const float *packed, int nlayers, int layer, float *out,
                         int flags, uint16_t *ohi, uint16_t *olo, float *onrm, hipStream_t st)
{
    set_tower_attrs();
    const bool last = (layer == nlayers);
    const bool x6 = (flags & SDE_TOWER_BF16X6) != 0;
    const float *w1 = packed;
    const float *wk = packed + L1_FLOATS + (int64_t)(layer - 2) * LK_FLOATS;
    const int hout = Hin - (layer == 2 ? 4 : 2), wout = Win - (layer == 2 ? 4 : 2);
    dim3 grid(cdiv(wout, TW_TX), cdiv(hout, TW_TY));
#define SDE_CONV(K, F, L, SM) K<F, L><<<grid, 512, SM, st>>>(in, Hin, Win, (F) ? w1 : nullptr, wk, out, hout, wout, \
                                                             (L) ? ohi : nullptr, (L) ? olo : nullptr, (L) ? onrm : nullptr)
    if (x6) {
        if (layer == 2) { if (last) SDE_CONV(conv64_x6_kernel, true, true, X6_SMEM); else SDE_CONV(conv64_x6_kernel, true, false, X6_SMEM); }
        else { if (last) SDE_CONV(conv64_x6_kernel, false, true, X6_SMEM); else SDE_CONV(conv64_x6_kernel, false, false, X6_SMEM); }
    } else {
        if (layer == 2) { if (last) SDE_CONV(conv64_mfma_kernel, true, true, TW_SMEM); else SDE_CONV(conv64_mfma_kernel, true, false, TW_SMEM); }
        else { if (last) SDE_CONV(conv64_mfma_kernel, false, true, TW_SMEM); else SDE_CONV(conv64_mfma_kernel, false, false, TW_SMEM); }
    }
#undef SDE_CONV
}

SDE_EXPORT int sde_tower_layer(const float *in, int Hin, int Win, const float *packed, int nlayers, int nf, int layer,
                               float *out, int flags, uint16_t *feat_hi, uint16_t *feat_lo, float *feat_norm,
                               void *stream)
{
    if (!in || !packed || !out || nf != NF || nlayers < 2 || layer < 2 || layer > nlayers) return SDE_ERR_ARG;
    if (Hin < (layer == 2 ? 5 : 3) || Win < (layer == 2 ? 5 : 3)) return SDE_ERR_ARG;
    if (flags & ~SDE_TOWER_BF16X6) return SDE_ERR_ARG;
    if ((feat_hi != nullptr) != (feat_lo != nullptr)) return SDE_ERR_ARG;
    launch_layer(in, Hin, Win, packed, nlayers, layer, out, flags, feat_hi, feat_lo, feat_norm, as_stream(stream));
    return launch_status();
}

SDE_EXPORT int sde_tower_forward(const float *img_pad, int H, int W, const float *packed, int nlayers, int nf,
                                 float *feat, void *workspace, int64_t workspace_bytes, int flags, uint16_t *feat_hi,
                                 uint16_t *feat_lo, float *feat_norm, void *stream)
{
    if ((feat_hi != nullptr) != (feat_lo != nullptr)) return SDE_ERR_ARG;
    if (nlayers == 1 && (feat_hi || feat_norm)) return SDE_ERR_ARG;
    if (!img_pad || !packed || !feat || H <= 0 || W <= 0 || nlayers < 1 || nf != NF) return SDE_ERR_ARG;
    if (flags & ~SDE_TOWER_BF16X6) return SDE_ERR_ARG;
    const int64_t need = sde_tower_workspace_bytes(H, W, nlayers, nf);
    if (need > 0 && (!workspace || workspace_bytes < need)) return SDE_ERR_WORKSPACE;
    hipStream_t st = as_stream(stream);
    const int Hp = H + 2 * nlayers, Wp = W + 2 * nlayers;
    if (nlayers == 1) {
        conv1_only_kernel<<<cdiv((int64_t)H * W, 256), 256, 0, st>>>(img_pad, Hp, Wp, packed, feat);
        return launch_status();
    }
    float *buf[2] = {nullptr, nullptr};
    if (nlayers > 2) {
        const int64_t h2 = H + 2 * (nlayers - 2), w2 = W + 2 * (nlayers - 2);
        buf[0] = reinterpret_cast<float *>(workspace);
        buf[1] = buf[0] + h2 * w2 * NF;
    }
    int hin = Hp, win = Wp;
    launch_layer(img_pad, hin, win, packed, nlayers, 2, nlayers == 2 ? feat : buf[0], flags, feat_hi, feat_lo, feat_norm,
                 st);
    hin -= 4; win -= 4;
    int cur = 0;
    for (int l = 3; l <= nlayers; l++) {
        float *o = (l == nlayers) ? feat : buf[cur ^ 1];
        launch_layer(buf[cur], hin, win, packed, nlayers, l, o, flags, feat_hi, feat_lo, feat_norm, st);
        hin -= 2; win -= 2;
        cur ^= 1;
    }
    return launch_status();
}

SDE_EXPORT int sde_preprocess_u8(const uint8_t *img, int H, int W, int pad, float *out_pad, void *scratch,
                                 void *stream)
{
    if (!img || !out_pad || !scratch || H <= 0 || W <= 0 || pad < 0) return SDE_ERR_ARG;
    hipStream_t st = as_stream(stream);
    unsigned long long *sums = reinterpret_cast<unsigned long long *>(scratch);
    if (hipMemsetAsync(sums, 0, 2 * sizeof(unsigned long long), st) != hipSuccess) return SDE_ERR_LAUNCH;
    const int64_t npix = (int64_t)H * W;
    const int blocks = (int)std::min<int64_t>(1024, std::max<int64_t>(1, cdiv(npix, 256 * 4 * 8)));
    image_sums_kernel<<<blocks, 256, 0, st>>>(img, npix, sums);
    const int64_t n = (int64_t)(H + 2 * pad) * (W + 2 * pad);
    znorm_pad_kernel<<<cdiv(n, 256), 256, 0, st>>>(img, H, W, pad, sums, out_pad);
    return launch_status();
}
