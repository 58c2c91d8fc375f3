// tower.hip -- MC-CNN-fast Siamese branch on the MFMA units (gfx950).
//
// Replaces mc_cnn_brunch.py:31-48 (Net.construct) + :70-92 (conv) as run by
// compute_feature (process_functional.py:21-39): nlayers x [3x3 VALID conv,
// bias, ReLU] (no ReLU on the last), then tf.nn.l2_normalize over channels.
// Layers 2..n are implicit GEMMs: out[n][pixel] = sum over (tap, c) of
// W[tap][n][c] * in[pixel + tap][c], M = 64 output maps, K = 9 taps x 64 maps.
// Layer 1 (Cin = 1, 9 MACs per output) is computed on VALU straight into layer
// 2's input staging, so its output never touches HBM; the last layer's epilogue
// L2-normalises each pixel (and can emit the certified cost volume's bf16 split
// planes and norm bounds).
//
// Two arithmetics (SDE_TOWER_FP32 / SDE_TOWER_BF16X6):
// * conv64_mfma_kernel: v_mfma_f32_32x32x2_f32 (exact f32 products, the 157 TF
//   fp32 matrix rate).  512 threads, output tile 8 rows x 32 columns, wave w owns
//   output row w (2 accumulators of 32x32); the (8+2) x (32+2) x 64 input tile
//   (87 KB) stays in LDS for all 9 taps, each tap's 64x64 weight slice is
//   double-buffered; both LDS images XOR-swizzled at 8-B granularity.
// * conv64_x6p_kernel (default): fp32 operands split exactly into three bf16
//   parts, six partial products on v_mfma_f32_32x32x16_bf16 -- see below.
#include "sde_common.h"

#include <atomic>

#include <vector>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <type_traits>

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
// layer k >= 2: bias f32 [64] | W f32 [tap][n][c] | bf16 parts (hi, mid, lo: W = hi+mid+lo) in A-fragment order
// [mtile 2][cblock 4][tap 9][part 3][lane 64][8] for conv64_x6p_kernel | fp16 parts of W * 2^tau (hi, lo)
// [mtile 2][cblock 4][tap 9][part 2][lane 64][8] for the F16 variant | F16 header {2^-tau, conv1 L1 bound,
// max |b1|, 0, L1 bound of this layer (max_n sum_{tap,c} |w|), its max |b|, 0, 0} (the conv1 terms are used
// by layer 2, which computes conv1; the layer's own terms bound its outputs for the split activations)
constexpr int LK_F16 = NF + LK_W + 3 * LK_W / 2;   // float offset of the fp16 parts
constexpr int LK_HDR = 8;                           // F16 header floats
// Winograd F(2x2,3x3) U = G g G^T (tower_wino.h): [xi 16][mtile 2][cblock 4][part 2][lane 64][8] fp16
// after the F16 header, then its own header {2^-tau_u, 0, 0, 0}
constexpr int LK_WINO = LK_F16 + LK_W + LK_HDR;
constexpr int LK_WU = 16 * NF * NF * 2;                // fp16 elements
constexpr int LK_WHDR = LK_WINO + LK_WU / 2;
constexpr int LK_FLOATS = LK_WHDR + 4;

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
// 2.67x the fp32 matrix peak at fp32-level error.
//
// conv64_x6p_kernel: persistent, one 512-thread workgroup per CU walking 16 x 32
// output tiles, warp-specialised:
// * waves 0-3 (one per SIMD) only issue MFMAs.  Wave w owns output channels
//   32*(w&1)..+31 and output rows 8*(w>>1)..+7 of the tile: 8 accumulators,
//   48 MFMAs per tap.  Weights never touch LDS: they are pre-arranged on the
//   host in A-fragment order [mtile][cblock][tap][part][lane][8] and read
//   straight into VGPRs one tap ahead (L2-resident, 221 KB per layer).
// * waves 4-7 (the "stagers") stream the input: the contraction is cut into
//   16-channel blocks (c-blocks); for one c-block the 18 x 34 input pixels are
//   loaded, split ONCE into bf16 parts and written to LDS as six planes (3 parts
//   x 2 channel halves, 8 bf16 per pixel) so that a B fragment is one contiguous,
//   conflict-free 1-KB ds_read_b128.  Two stage buffers: the stagers fill c-block
//   k+1 (or the next tile's first) while the MFMA waves consume c-block k; one
//   workgroup barrier per c-block.  Keeping the long-latency HBM loads in other
//   waves keeps them out of the MFMA waves' in-order vmcnt.
// Inter-layer activations use a c-block-major layout [4][h][w][16] (IN_CB /
// OUT_CB) so a stage reads contiguous 64-B pixel runs; the last layer writes the
// reference's [h][w][64].
//
// F16 (SDE_TOWER_F16X3): the same kernel with every operand split into TWO fp16
// parts after a power-of-two scaling, x*2^s = h + l (h = fp16(x*2^s), l =
// fp16(x*2^s - h), the residual exact in f32), and the three partial products
// h*h' + h*l' + l*h' on v_mfma_f32_32x32x16_f16.  fp16's 11-bit significand
// makes two parts carry 22 bits: the dropped l*l' term is < 2^-22 |ab| and each
// part's rounding 2^-23 relative -- the error of a few fp32 roundings per
// product, at half the MFMAs of bf16x6.  The scalings keep the parts in fp16's
// normal range without any chance of overflow:
// * weights: 2^tau per layer from the host (max |w| * 2^tau in [2^14, 2^15));
// * activations: 2^sigma per launch from a device word holding an upper bound
//   of |input| (the previous layer's epilogue atomically maxes its ReLU outputs
//   into it; for layer 2 the word holds max |image| and the kernel bounds conv1's
//   output by max|image| * max_n sum_t |w1[t][n]| + max |b1|), so that
//   bound * 2^sigma lies in [2^14, 2^15) < 65504.  Values far below the bound
//   lose relative precision only as fp16 subnormals do: absolute error
//   <= 2^-25 * 2^-sigma, i.e. <= 2^-40 of the layer's largest input.
// The epilogue multiplies the accumulators by 2^-(tau+sigma) (exact).
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split3(float x, __bf16 &h, __bf16 &m, __bf16 &l)
{
    h = (__bf16)x;
    const float r1 = x - (float)h;
    m = (__bf16)r1;
    const float r2 = r1 - (float)m;
    l = (__bf16)r2;
}

#ifndef XP_RING_F16
#define XP_RING_F16 3
#endif

constexpr int XP_TY = 16, XP_TX = 32;             // output tile
constexpr int XP_IY = XP_TY + 2, XP_IX = XP_TX + 2;
constexpr int XP_NPIX = XP_IY * XP_IX;            // 612 input pixels per tile
constexpr int XP_PLANE = XP_NPIX * 16;            // bytes of one (part, channel-half) plane
constexpr int XP_STAGE = 6 * XP_PLANE;            // one c-block stage: 58,752 B
constexpr int XP_UNITS = XP_NPIX * 4;             // (pixel, 4-channel chunk) units per stage
constexpr int XP_STAGERS = 256;                   // threads of the stager waves
constexpr int XP_UPT = (XP_UNITS + XP_STAGERS - 1) / XP_STAGERS;   // units per stager thread (10)
// MFMA wave mapping: WR output rows x 64 / (8 / WR)... per wave -- WR = 8: one M-tile (32 output
// channels) of 8 rows; WR = 4: both M-tiles of 4 rows (a pixel's 64 channels in one wave, as the
// last layer's L2 norm wants).  8 accumulators either way.
#ifndef XP_WR_MID
#define XP_WR_MID 4
#endif
#ifndef XP_WR_FIRST
#define XP_WR_FIRST 4
#endif
constexpr int XP_ACC = 8;                         // accumulators per MFMA wave
#define XP_AL(F16, WR) (((WR) == 8 || (F16)) ? 2 : 1)   // A fragments requested this many taps ahead
constexpr int XP_WX = XP_IX + 2, XP_WIN = (XP_IY + 2) * XP_WX;   // FIRST: image window of a tile (20 x 36)
// two stages | FIRST: one image window per stager wave
constexpr size_t XP_BIAS_OFF = (size_t)2 * XP_STAGE + 4 * XP_WIN * sizeof(float);
constexpr size_t XP_SMEM = XP_BIAS_OFF + NF * sizeof(float);     // + the layer's 64 biases
constexpr int XP_NCB = NF / 16;                   // c-blocks per pixel

// Split 4 channels and store them into the stage's six planes.
__device__ __forceinline__ void xp_put(char *sb, int u, float4 v)
{
    const int px = u >> 2, chunk = u & 3;
    bf16x4 p0, p1, p2;
    const float xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; e++) {
        __bf16 a, b, c;
        split3(xs[e], a, b, c);
        p0[e] = a; p1[e] = b; p2[e] = c;
    }
    char *dst = sb + (chunk >> 1) * XP_PLANE + px * 16 + (chunk & 1) * 8;
    *reinterpret_cast<uint2 *>(dst) = __builtin_bit_cast(uint2, p0);
    *reinterpret_cast<uint2 *>(dst + 2 * XP_PLANE) = __builtin_bit_cast(uint2, p1);
    *reinterpret_cast<uint2 *>(dst + 4 * XP_PLANE) = __builtin_bit_cast(uint2, p2);
}

// Tiles of a launch over a batch of images of one size: tile t -> image t / tiles_img, then
// row-major 16 x 32 output tiles.  Strides are per image (floats; pixels for the split outputs;
// floats between the images' F16 bound-word arrays).
struct XpBatch {
    int tiles_x, tiles_img, ntiles;
    int64_t in_stride, out_stride, pix_stride;
    int amax_stride;
};

__device__ __forceinline__ void xp_tile(const XpBatch &bt, int t, int &img, int &ty0, int &tx0)
{
    img = t / bt.tiles_img;
    const int tl = t - img * bt.tiles_img;
    ty0 = (tl / bt.tiles_x) * XP_TY;
    tx0 = (tl % bt.tiles_x) * XP_TX;
}

// F16: scale by 2^sigma (s), split into two fp16 parts, store planes (part, channel half).
__device__ __forceinline__ void xp_put16(char *sb, int u, float4 v, float s)
{
    const int px = u >> 2, chunk = u & 3;
    f16x4 p0, p1;
    const float xs[4] = {v.x * s, v.y * s, v.z * s, v.w * s};
#pragma unroll
    for (int e = 0; e < 4; e++) {
        const _Float16 h = (_Float16)xs[e];
        p0[e] = h;
        p1[e] = (_Float16)(xs[e] - (float)h);
    }
    char *dst = sb + (chunk >> 1) * XP_PLANE + px * 16 + (chunk & 1) * 8;
    *reinterpret_cast<uint2 *>(dst) = __builtin_bit_cast(uint2, p0);
    *reinterpret_cast<uint2 *>(dst + 2 * XP_PLANE) = __builtin_bit_cast(uint2, p1);
}

template <bool F16>
__device__ __forceinline__ void xp_store(char *sb, int u, float4 v, float s)
{
    if (F16) xp_put16(sb, u, v, s);
    else xp_put(sb, u, v);
}

// One stage unit of activations (zero outside the input).
template <bool IN_CB>
__device__ __forceinline__ float4 xp_load(const float *__restrict__ in, int Hin, int Win, int ty0, int tx0, int cb,
                                          int u)
{
    const int px = u >> 2, chunk = u & 3;
    const int iy = px / XP_IX, ix = px - iy * XP_IX;
    const int y = ty0 + iy, x = tx0 + ix;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (y < Hin && x < Win) {
        const float4 *in4 = reinterpret_cast<const float4 *>(in);
        const size_t i = IN_CB ? (((size_t)cb * Hin + y) * Win + x) * 4 + chunk : ((size_t)y * Win + x) * 16 + cb * 4 + chunk;
        v = in4[i];   // default cache policy: nontemporal loads / stores measured slower (the next layer
                      // re-reads the outputs from cache; round 2: layer 231 -> 234 / 242 / 250 us)
    }
    return v;
}

// conv1 (Cin = 1, 3x3, bias, ReLU) of the padded image for one stage unit; w = the 9 taps x
// 4 channels of the unit's chunk, b = their biases (a stager thread's chunk is fixed).
// The image values come from the stager wave's LDS window of the tile (win[iy][ix], 20 x 36).
__device__ __forceinline__ float4 xp_conv1(const float *win, int Hin, int Win, const float4 (&w)[9],
                                           float4 b, int ty0, int tx0, int u)
{
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    const int px = u >> 2;
    const int iy = px / XP_IX, ix = px - iy * XP_IX;
    const int y = ty0 + iy, x = tx0 + ix;
    if (y < Hin - 2 && x < Win - 2) {
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        const float *wp = win + iy * XP_WX + ix;
#pragma unroll
        for (int t = 0; t < 9; t++) {
            const float im = wp[(t / 3) * XP_WX + t % 3];
            s0 = fmaf(im, w[t].x, s0);
            s1 = fmaf(im, w[t].y, s1);
            s2 = fmaf(im, w[t].z, s2);
            s3 = fmaf(im, w[t].w, s3);
        }
        v = make_float4(fmaxf(s0 + b.x, 0.f), fmaxf(s1 + b.y, 0.f), fmaxf(s2 + b.z, 0.f), fmaxf(s3 + b.w, 0.f));
    }
    return v;
}

// Stager waves: fill one stage with c-block cb of tile t.
template <bool FIRST, bool IN_CB, bool F16>
__device__ __forceinline__ void xp_fill(char *sb, const float *__restrict__ in, int Hin, int Win,
                                        const float *__restrict__ w1blob, int t, const XpBatch &bt, int cb, int st,
                                        float s, float *win)
{
    // opaque to the optimiser: stops loop-invariant code motion from hoisting the per-unit
    // address arithmetic of all units out of the tile loop (it would pin ~40 VGPRs that the
    // MFMA waves' accumulators need)
    asm volatile("" : "+v"(st));
    int img, ty0, tx0;
    xp_tile(bt, t, img, ty0, tx0);
    in += img * bt.in_stride;
    if (FIRST) {
        // the tile's image window is already in the wave's LDS window (xp_stager_loop)
        // the thread's chunk is st & 3 for every unit (XP_STAGERS is a multiple of 4)
        const int n0 = cb * 16 + (st & 3) * 4;
        const float4 b = *reinterpret_cast<const float4 *>(w1blob + n0);
        float4 w[9];
#pragma unroll
        for (int t = 0; t < 9; t++) w[t] = *reinterpret_cast<const float4 *>(w1blob + NF + t * NF + n0);
#pragma unroll 2
        for (int i = 0; i < XP_UPT; i++) {
            const int u = st + i * XP_STAGERS;
            if (u < XP_UNITS) xp_store<F16>(sb, u, xp_conv1(win, Hin, Win, w, b, ty0, tx0, u), s);
        }
    } else {
        // two batches of 5 loads in flight (the stagers have time; registers are shared
        // with the MFMA waves' allocation)
        constexpr int HB = (XP_UPT + 1) / 2;
#pragma unroll
        for (int b0 = 0; b0 < XP_UPT; b0 += HB) {
            float4 v[HB];
#pragma unroll
            for (int i = 0; i < HB; i++) {
                const int u = st + (b0 + i) * XP_STAGERS;
                v[i] = u < XP_UNITS ? xp_load<IN_CB>(in, Hin, Win, ty0, tx0, cb, u) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int i = 0; i < HB; i++) {
                const int u = st + (b0 + i) * XP_STAGERS;
                if (u < XP_UNITS) xp_store<F16>(sb, u, v[i], s);
            }
        }
    }
}

// 2^sigma for a bound: bound * 2^sigma in [2^14, 2^15); a zero, subnormal or non-finite bound gives sigma = 14
__device__ __forceinline__ int xp_sigma(float bound)
{
    int e = 0;   // bound in [2^e, 2^(e+1))
    if (bound >= 1.17549435e-38f && bound <= 3.40282347e38f) e = (int)((__float_as_uint(bound) >> 23) & 255u) - 127;
    return min(max(14 - e, -100), 100);
}

// F16 scalings of one tile (see above): s = 2^sigma for the stagers, unscale = 2^-(tau+sigma).
// hdr: the layer blob's F16 header {2^-tau, max_n sum_t |w1[t][n]|, max |b1|, 0}.
__device__ __forceinline__ void xp_scales(bool first, const float *__restrict__ in_amax, const float *__restrict__ hdr,
                                          float &s, float &unscale)
{
    const float m = *in_amax;
    const int sigma = xp_sigma(first ? fmaf(m, hdr[1], hdr[2]) : m);
    s = ldexpf(1.0f, sigma);
    unscale = ldexpf(hdr[0], -sigma);
}

// Split activations (SDE_TOWER_OUT_SPLIT / SDE_TOWER_IN_SPLIT): a layer writes its ReLU outputs already
// scaled and split into the two fp16 parts its reader stages, so the reader's stagers copy them to LDS
// with LDS-DMA and no arithmetic.  The writer cannot know the measured maximum of its outputs before it
// writes them, so its 2^sigma comes from an a-priori bound: |out| <= max|b| + L1 * bound(|input|) (hdr[4],
// hdr[5], rounded up on the host; x 1.001 covers the f16x3 error of the computed outputs) -- bound * 2^sigma
// in [2^14, 2^15), no fp16 overflow.  The bound is looser than the measured maximum by the layer's L1 gain
// only (the input term is the measured bound word), which costs nothing here: values far below the bound
// lose precision only as fp16 subnormals do, an absolute error <= 2^-25 * 2^-sigma = 2^-39 of the bound.
// The writer publishes 2^sigma at its bound word + XP_SCALE_WORD (per image); the reader's unscale is
// 2^-tau / 2^sigma (exact).  Layout of a split activation (per image): 16 planes [cblk32 2][part 2][q 4],
// each [h][w][8 fp16] (16 B per pixel): the same 256 B per pixel as the fp32 [h][w][64].
constexpr int XP_SCALE_WORD = 32;
__device__ __forceinline__ float xp_out_scale(bool first, const float *__restrict__ in_amax,
                                              const float *__restrict__ hdr)
{
    const float m = *in_amax;
    const float bin = first ? fmaf(m, hdr[1], hdr[2]) : m;
    return ldexpf(1.0f, xp_sigma(fmaf(bin, hdr[4], hdr[5]) * 1.001f));
}

// the writer's 2^sigma into out_amax[img * stride + XP_SCALE_WORD] for every image of the launch
// (workgroup 0, wave 0; every workgroup would compute the same value)
__device__ __forceinline__ void xp_publish_scale(bool first, const XpBatch &bt, const float *__restrict__ in_amax,
                                                 const float *__restrict__ hdr, float *__restrict__ out_amax)
{
    if (blockIdx.x != 0 || threadIdx.x >= 64) return;
    const int nimg = bt.ntiles / bt.tiles_img;
    for (int im = threadIdx.x; im < nimg; im += 64)
        out_amax[im * bt.amax_stride + XP_SCALE_WORD] = xp_out_scale(first, in_amax + im * bt.amax_stride, hdr);
}

// Stager waves' own loop (non-FIRST layers): the pipeline of (tile, c-block) steps the MFMA
// waves consume, one stage ahead, with the HBM loads of step i+2 issued before step i+1's
// units are split and stored -- every load has a whole c-block period to land.  Runs the
// same barriers as the MFMA waves: one per c-block.
template <bool FIRST, bool IN_CB, bool F16>
__device__ __forceinline__ void xp_stager_loop(char *xsm, const float *__restrict__ in, int Hin, int Win,
                                               const XpBatch &bt, int st, const float *__restrict__ in_amax,
                                               const float *__restrict__ hdr, const float *__restrict__ w1blob,
                                               float *win)
{
    const int tile0 = blockIdx.x, gstride = gridDim.x;
    const int nsteps = ((bt.ntiles - 1 - tile0) / gstride + 1) * XP_NCB;
    if (FIRST) {
        // conv1 on the stagers: each step computed from the wave's LDS image window, one stage ahead
        int sc_img = -1;
        float s = 1.0f, unscale = 1.0f;
        // the image window of a tile, loaded into registers 3 steps before its first use (while
        // the previous tile's c-blocks are computed) and written to the wave's LDS window when
        // the tile's first c-block is filled -- the HBM latency stays off the stagers' path
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
            if (F16 && im != sc_img) {
                xp_scales(true, in_amax + im * bt.amax_stride, hdr, s, unscale);
                sc_img = im;
            }
            if (cb == 0) {   // a wave's LDS accesses complete in order: no barrier needed
#pragma unroll
                for (int k = 0; k < WPL; k++)
                    if (lane + 64 * k < XP_WIN) win[lane + 64 * k] = wv[k];
                __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the window's LDS writes have landed
                __builtin_amdgcn_wave_barrier();
            }
            xp_fill<true, false, F16>(xsm + (i & 1) * XP_STAGE, in, Hin, Win, w1blob, t, bt, cb, st, s, win);
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
        if (F16 && im != sc_img) {   // the tile's image changed: its bound word (tiles run image-major)
            xp_scales(false, in_amax + im * bt.amax_stride, hdr, s, unscale);
            sc_img = im;
        }
        char *sb = xsm + (i & 1) * XP_STAGE;
#pragma unroll
        for (int k = 0; k < XP_UPT; k++) {
            const int u = st + k * XP_STAGERS;
            if (u < XP_UNITS) xp_store<F16>(sb, u, v[k], s);
        }
    };
    auto sync_step = [&](int) {
        __syncthreads();
    };
    float4 ra[XP_UPT], rb[XP_UPT];
    load(ra, 0);
    store(ra, 0);
    if (nsteps > 1) load(ra, 1);
    __syncthreads();
    // step i: the MFMA waves consume stage i & 1; here step i+1 is stored and step i+2 loaded
#pragma unroll 1
    for (int i = 0; i < nsteps; i += 2) {
        if (i + 2 < nsteps) load(rb, i + 2);
        if (i + 1 < nsteps) store(ra, i + 1);
        sync_step(i);
        if (i + 1 >= nsteps) break;
        if (i + 3 < nsteps) load(ra, i + 3);
        if (i + 2 < nsteps) store(rb, i + 2);
        sync_step(i + 1);
    }
}

struct XpFrag {
    bf16x8 p[3];
};

// A fragments of one (c-block, tap): NP = 3 bf16 parts, or 2 fp16 parts (F16; the blob holds
// [mtile][cblock][tap][part NP][lane][8] for each arithmetic).  Unused parts stay untouched.
template <int NP>
__device__ __forceinline__ XpFrag xp_afrag(const uint4 *__restrict__ wf, int mt, int cb, int tap, int lane)
{
    const uint4 *src = wf + ((size_t)((mt * XP_NCB + cb) * 9 + tap) * NP) * 64 + lane;
    XpFrag f;
#pragma unroll
    for (int q = 0; q < NP; q++) f.p[q] = __builtin_bit_cast(bf16x8, src[q * 64]);
    return f;
}

// B fragments (three parts; two for F16) of one row-step.
struct XpB {
    bf16x8 p[3];
};

template <int NP>
__device__ __forceinline__ XpB xp_bfrag(const char *b)
{
    XpB f;
#pragma unroll
    for (int q = 0; q < NP; q++)
        f.p[q] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4 *>(b + 2 * q * XP_PLANE));
    return f;
}

__device__ __forceinline__ floatx16 mfma_h(bf16x8 a, bf16x8 b, floatx16 c)
{
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

// Epilogue stores: buffer descriptors on a per-tile base (wave-uniform), 32-bit per-lane byte
// offsets with an SGPR row offset; a lane outside the output (x >= Wout) gets XP_OOB, which the
// descriptor's range check drops -- no exec-mask branches, no 64-bit address math per store.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
constexpr uint32_t XP_NREC = 0x40000000u, XP_OOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t xp_rsrc(const void *base)
{
    const uintptr_t b = (uintptr_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((uintptr_t)hi << 32) | lo), 0, (int)XP_NREC, 0x00020000);
}

// the same with nrec bytes of records (loads past them return zero)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t xp_rsrc_n(const void *base, uint32_t nrec)
{
    const uintptr_t b = (uintptr_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((uintptr_t)hi << 32) | lo), 0,
                                             (int)__builtin_amdgcn_readfirstlane(nrec), 0x00020000);
}

__device__ __forceinline__ void xp_st4(float4 v, __amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so)
{
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, vo, so, 0);
}

// One c-block for one MFMA wave: 9 taps x 4 output rows = 36 row-steps; each step's B
// fragment (one input row segment, NP parts) feeds both M-tiles (output channels 0-31 and
// 32-63): 2 x 6 (bf16x6) or 2 x 3 (F16) MFMAs, small terms first, the leading product last.
// B fragments are read RD-1 row-steps ahead (a register ring); sched_barrier fences keep the
// scheduler from hoisting more, which bounds the live registers (8 accumulators = 128 of the
// 256 a wave may hold at 2 waves per SIMD).  A fragments (both M-tiles) are requested AL taps
// ahead.  Rows past the output edge run on zero-filled input and are discarded by the epilogue.
template <bool F16, int WR>
__device__ __forceinline__ void xp_cblock(floatx16 (&acc)[XP_ACC], XpFrag (&a)[8 / WR],
                                          XpFrag (&an)[XP_AL(F16, WR)][8 / WR], const uint4 *__restrict__ wf, int mt0,
                                          int cb, int ncb, int lane, const char *sb)
{
    constexpr int XP_WROWS = WR, MW = 8 / WR;
    constexpr int NS = 9 * XP_WROWS;
    constexpr int NP = F16 ? 2 : 3;
    constexpr int AL = XP_AL(F16, WR);
    constexpr int RD = F16 ? XP_RING_F16 : 3;   // ring depth: fragments read RD-1 row-steps ahead
    XpB ring[RD];
    auto boff = [&](int s) { return ((s / XP_WROWS / 3 + s % XP_WROWS) * XP_IX + (s / XP_WROWS) % 3) * 16; };
#pragma unroll
    for (int k = 0; k < RD - 1; k++) ring[k] = xp_bfrag<NP>(sb + boff(k));
#pragma unroll
    for (int s = 0; s < NS; s++) {
        const int tap = s / XP_WROWS, r = s % XP_WROWS;
        if (r == 0 && tap > 0) {
            // a = A(tap); an[k] = A(tap + 1 + k); request A(tap + AL) (the next c-block's past tap 8)
#pragma unroll
            for (int m = 0; m < MW; m++) {
                a[m] = an[0][m];
#pragma unroll
                for (int k = 0; k + 1 < AL; k++) an[k][m] = an[k + 1][m];
                const int t2 = tap + AL;
                an[AL - 1][m] = t2 < 9 ? xp_afrag<NP>(wf, mt0 + m, cb, t2, lane)
                                            : xp_afrag<NP>(wf, mt0 + m, ncb, t2 - 9, lane);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        const XpB &b = ring[s % RD];
#pragma unroll
        for (int m = 0; m < MW; m++) {
            floatx16 &c = acc[m * XP_WROWS + r];
            if (F16) {
                c = mfma_h(a[m].p[1], b.p[0], c);
                c = mfma_h(a[m].p[0], b.p[1], c);
                c = mfma_h(a[m].p[0], b.p[0], c);
            } else {
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[m].p[2], b.p[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[m].p[1], b.p[1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[m].p[0], b.p[2], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[m].p[1], b.p[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[m].p[0], b.p[1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[m].p[0], b.p[0], c, 0, 0, 0);
            }
        }
        if (s + RD - 1 < NS) ring[(s + RD - 1) % RD] = xp_bfrag<NP>(sb + boff(s + RD - 1));
    }
    // hand the c-block boundary over: a = A(next c-block, tap 0)
#pragma unroll
    for (int m = 0; m < MW; m++) {
        a[m] = an[0][m];
#pragma unroll
        for (int k = 0; k + 1 < AL; k++) an[k][m] = an[k + 1][m];
        an[AL - 1][m] = xp_afrag<NP>(wf, mt0 + m, ncb, AL, lane);
    }
}

// x (already scaled by 2^sigma) split exactly into two fp16 parts: hi = fp16(x) (v_cvt_pk_f16_f32), lo =
// fp16(x - hi) by v_fma_mix{lo,hi}_f16 straight from the packed hi half (x - hi is exact in fp32, so its one
// rounding gives the bits of (fp16)(x - (float)hi); 6 instructions per 4 values instead of 12)
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void xp_split16s(float4 x, u32x2 &hw, u32x2 &lw)
{
    const f16x2 h01 = {(_Float16)x.x, (_Float16)x.y}, h23 = {(_Float16)x.z, (_Float16)x.w};
    hw = u32x2{__builtin_bit_cast(uint32_t, h01), __builtin_bit_cast(uint32_t, h23)};
    uint32_t l01, l23;
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=&v"(l01) : "v"(x.x), "v"(hw.x));
    asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(l01) : "v"(x.y), "v"(hw.x));
    asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=&v"(l23) : "v"(x.z), "v"(hw.y));
    asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(l23) : "v"(x.w), "v"(hw.y));
    lw = u32x2{l01, l23};
}

// a lane pair (rows 2i, 2i + 1 of 16 lanes: SWAP32 = false; halves of 32: true) trades halves so that the
// even lane ends with both lanes' hi parts and the odd one with both lo parts (odd lanes' hi <-> even lanes' lo)
template <bool SWAP32>
__device__ __forceinline__ u32x4 xp_pair_parts(u32x2 hw, u32x2 lw)
{
#pragma unroll
    for (int w = 0; w < 2; w++) {
        const auto sw = SWAP32 ? __builtin_amdgcn_permlane32_swap(hw[w], lw[w], false, false)
                               : __builtin_amdgcn_permlane16_swap(hw[w], lw[w], false, false);
        hw[w] = sw[0];
        lw[w] = sw[1];
    }
    return u32x4{hw.x, hw.y, lw.x, lw.y};
}

// Tile epilogue of one MFMA wave (output rows WR*g .., M-tiles mt0 ..): bias (+ReLU | L2-normalise),
// stores, and (F16, !LAST) the running maximum of the stored outputs for the image's bound word
// (one atomic per wave and image, xp_flush_amax).  unscale undoes the F16 power-of-two scalings.
__device__ __forceinline__ void xp_flush_amax(uint32_t &amax_run, int &amax_img, int lane, float *out_amax,
                                              int amax_stride)
{
    if (amax_img < 0) return;
    uint32_t a = amax_run;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a = max(a, (uint32_t)__shfl_xor((int)a, o, 64));
    if (lane == 0) atomicMax(reinterpret_cast<unsigned int *>(out_amax + amax_img * amax_stride), a);
    amax_run = 0u;
}

constexpr int XP_PIN = 4;   // a stored float4's registers are not rewritten before XP_PIN - 1 more stores issue

template <bool LAST, bool OUT_CB, bool F16, int XP_WROWS, bool OSPL = false>
__device__ __forceinline__ void xp_epilogue(const floatx16 (&acc)[XP_ACC], int lane, int g, int mt0, int img,
                                            int ty0, int tx0, float unscale, const float4 *lbias4,
                                            float *__restrict__ out, int Hout, int Wout, const XpBatch &bt,
                                            uint16_t *__restrict__ ohi, uint16_t *__restrict__ olo,
                                            float *__restrict__ onrm, uint32_t &amax_run, int &amax_img,
                                            float *__restrict__ out_amax, float oscale = 1.0f)
{
    static_assert(!OSPL || (F16 && !LAST && !OUT_CB), "split outputs: F16 intermediate layers");
    constexpr int MW = 8 / XP_WROWS;
    // ---- epilogue (MFMA waves): bias (+ReLU | L2-normalise) ------------
    // lane holds pixel column j, channels m*32 + 8q + 4h + e in acc[m * XP_WROWS + r][4q + e]
    // opaque copies of the lane coordinates: keep the epilogue's bias loads and
    // addresses inside the loop (hoisted, they would pin registers for the whole kernel)
    int j = lane & 31, h = lane >> 5;
    asm volatile("" : "+v"(j), "+v"(h));
    const int x = tx0 + j;
    const bool xok = x < Wout;
    const int row0 = XP_WROWS * g;   // this wave's first row in the tile
    if (!LAST) {
        // F16: max of this lane's stored outputs of the tile, as float bits (outputs are >= +0
        // after the ReLU, so their bits order like their values: integer max3, no NaN quieting)
        uint32_t amax = 0u;
        float *const outi = out + img * bt.out_stride;
        // OUT_CB: [cblk][h][w][16] -> one descriptor per c-block plane, at the tile's first row;
        // else [h][w][64]
        const uint32_t vo = xok ? (uint32_t)(x * (OUT_CB ? 64 : 256) + 16 * h) : XP_OOB;
        const size_t HW = (size_t)Hout * Wout;
        // Store-data registers stay untouched for XP_PIN stores ("store-data overwrite"):
        // each stored float4 is pinned live by an empty asm placed after the store XP_PIN - 1 stores
        // later, and the epilogue's last pins carry an s_nop, so no VALU writes a register a dwordx4
        // store still reads within XP_PIN instructions -- the store's issue and its data read are not
        // one event when MFMA waves contend for the VGPR read ports.  _isa_lint.py checks the built
        // code objects for this schedule.
        constexpr int NPIN = MW * 2 * XP_WROWS * 2;
        u32x4 pin[NPIN];
#pragma unroll
        for (int m = 0; m < MW; m++) {
            float4 b4[4];
#pragma unroll
            for (int q = 0; q < 4; q++) b4[q] = lbias4[((mt0 + m) * 32 + 8 * q + 4 * h) >> 2];
#pragma unroll
            for (int qh = 0; qh < 2; qh++) {
                const int cblk = 2 * (mt0 + m) + qh;
                // OSPL: the hi planes of 32-channel block mt0 + m at the tile's first row (q and the part
                // ride in the SGPR offset: plane (cblk32 * 2 + part) * 4 + q)
                const __amdgpu_buffer_rsrc_t rs =
                    OSPL ? xp_rsrc(reinterpret_cast<char *>(outi) + (size_t)(mt0 + m) * 8 * HW * 16 + (size_t)ty0 * Wout * 16)
                         : xp_rsrc(OUT_CB ? outi + ((size_t)cblk * HW + (size_t)ty0 * Wout) * 16
                                          : outi + (size_t)ty0 * Wout * NF);
#pragma unroll
                for (int r = 0; r < XP_WROWS; r++) {
                    const floatx16 &c = acc[m * XP_WROWS + r];
                    const bool rok = ty0 + row0 + r < Hout;   // wave-uniform
                    const uint32_t so = (uint32_t)((row0 + r) * Wout) * (OUT_CB ? 64u : 256u);
#pragma unroll
                    for (int ql = 0; ql < 2; ql++) {
                        const int q = 2 * qh + ql;
                        const float bq[4] = {b4[q].x, b4[q].y, b4[q].z, b4[q].w};
                        float o4[4];
                        // OSPL: the outputs scaled by 2^sigma straight from the accumulators (the scale folded
                        // into the unscale and the bias: exact, powers of two), their bound unscaled at the flush
                        const float us = OSPL ? unscale * oscale : unscale;
#pragma unroll
                        for (int e = 0; e < 4; e++)
                            o4[e] = fmaxf((F16 ? fmaf(c[4 * q + e], us, OSPL ? bq[e] * oscale : bq[e]) : c[4 * q + e] + bq[e]), 0.f);
                        const float4 o = make_float4(o4[0], o4[1], o4[2], o4[3]);
                        const int k = ((m * 2 + qh) * XP_WROWS + r) * 2 + ql;
                        if (OSPL) {
                            // fp16 parts of channels 32 (mt0 + m) + 8q + 4h ..: the lane pair (h = 0, 1) swaps
                            // halves (v_permlane32_swap) so that lane h = 0 holds the group's 8 hi parts and
                            // h = 1 its 8 lo parts: one 16-B store each, to plane (mt0 + m) * 8 + h * 4 + q
                            u32x2 hw2, lw2;
                            xp_split16s(o, hw2, lw2);
                            const u32x4 v4 = xp_pair_parts<true>(hw2, lw2);
                            pin[k] = v4;
                            if (rok) {
                                amax = max(amax, max(__float_as_uint(o.x), __float_as_uint(o.y)));
                                amax = max(amax, max(__float_as_uint(o.z), __float_as_uint(o.w)));
                                const uint32_t pb = (uint32_t)HW * 16u;
                                const uint32_t v2 = xok ? (uint32_t)(x * 16) + (uint32_t)h * 4u * pb : XP_OOB;
                                const uint32_t s2 = (uint32_t)((row0 + r) * Wout) * 16u;
                                __builtin_amdgcn_raw_buffer_store_b128(v4, rs, v2, s2 + q * pb, 0);
                            }
                        } else {
                            pin[k] = __builtin_bit_cast(u32x4, o);
                            if (rok) {
                                if (F16) {   // the bound before the store: nothing writes o's registers after it
                                    amax = max(amax, max(__float_as_uint(o.x), __float_as_uint(o.y)));
                                    amax = max(amax, max(__float_as_uint(o.z), __float_as_uint(o.w)));
                                }
                                // byte offset within the descriptor: OUT_CB 32 (q & 1); else ch * 4
                                xp_st4(o, rs, vo + (OUT_CB ? 32u * ql : 4u * ((mt0 + m) * 32 + 8 * q)), so);
                            }
                        }
                        if (k >= XP_PIN - 1) asm volatile("" ::"v"(pin[k - (XP_PIN - 1)]));
                    }
                }
            }
        }
#pragma unroll
        for (int k = NPIN - (XP_PIN - 1); k + 1 < NPIN; k++) asm volatile("" ::"v"(pin[k]));
        asm volatile("s_nop 4" ::"v"(pin[NPIN - 1]));
        if (OSPL)   // the bound of the scaled outputs, unscaled (exact: a power of two)
            amax = __float_as_uint(__uint_as_float(amax) / oscale);
        if (F16) {
            if (!xok) amax = 0u;   // lanes past the output edge stored nothing
            // one atomic per wave and image (flushed when the tiles move to the next
            // image and at the end): every workgroup maxes into the same word
            if (img != amax_img) {
                xp_flush_amax(amax_run, amax_img, lane, out_amax, bt.amax_stride);
                amax_img = img;
            }
            amax_run = max(amax_run, amax);
        }
    } else {
        // a pixel's 64 channels live in this wave (two lanes): wave-local L2 norm.
        // Outputs [h][w][64] (+ bf16 planes, norm bound), descriptors at the tile's first row.
        const size_t pix0 = (size_t)img * bt.pix_stride + (size_t)ty0 * Wout;
        const __amdgpu_buffer_rsrc_t rs = xp_rsrc(out + pix0 * NF);
        const uint32_t vo = xok ? (uint32_t)(x * 256 + 16 * h) : XP_OOB;
#pragma unroll
        for (int r = 0; r < XP_WROWS; r++) {
            // biased value of channel m*32 + 8q + 4h + e (bias re-read from LDS per use: nothing
            // but the accumulators stays live across the row)
            int hr = h;
            asm volatile("" : "+v"(hr));   // per-row opaque copy: no CSE of bias reads across rows
            auto val4 = [&](int m, int q, float (&t)[4]) {
                const float4 bq4 = lbias4[(m * 32 + 8 * q + 4 * hr) >> 2];
                const float bq[4] = {bq4.x, bq4.y, bq4.z, bq4.w};
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const float cv = acc[m * XP_WROWS + r][4 * q + e];
                    t[e] = F16 ? fmaf(cv, unscale, bq[e]) : cv + bq[e];
                }
            };
            float ss = 0.0f;
#pragma unroll
            for (int m = 0; m < 2; m++)
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    float t[4];
                    val4(m, q, t);
#pragma unroll
                    for (int e = 0; e < 4; e++) ss += t[e] * t[e];
                }
            ss += __shfl_xor(ss, 32, 64);
            const float inv = 1.0f / sqrtf(fmaxf(ss, 1e-12f));
            float v[2][16];
#pragma unroll
            for (int m = 0; m < 2; m++)
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    float t[4];
                    val4(m, q, t);
#pragma unroll
                    for (int e = 0; e < 4; e++) v[m][4 * q + e] = t[e] * inv;
                }
            float s2 = 0.0f;
#pragma unroll
            for (int m = 0; m < 2; m++)
#pragma unroll
                for (int i = 0; i < 16; i++) s2 += v[m][i] * v[m][i];
            s2 += __shfl_xor(s2, 32, 64);
            if (ty0 + row0 + r < Hout) {   // wave-uniform
                const uint32_t rowp = (uint32_t)((row0 + r) * Wout);   // pixels from the tile's first row
#pragma unroll
                for (int m = 0; m < 2; m++)
#pragma unroll
                    for (int q = 0; q < 4; q++)
                        xp_st4(make_float4(v[m][4 * q], v[m][4 * q + 1], v[m][4 * q + 2], v[m][4 * q + 3]),
                               rs, vo + 4u * (m * 32 + 8 * q), rowp * 256u);
                if (ohi) {
                    const __amdgpu_buffer_rsrc_t rh = xp_rsrc(ohi + pix0 * NF), rl = xp_rsrc(olo + pix0 * NF);
                    const uint32_t vo2 = xok ? (uint32_t)(x * 128 + 8 * h) : XP_OOB;
#pragma unroll
                    for (int m = 0; m < 2; m++)
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            bf16x4 hv, lv;
#pragma unroll
                            for (int e = 0; e < 4; e++) {
                                const float xv = v[m][4 * q + e];
                                const __bf16 hh = (__bf16)xv;
                                hv[e] = hh;
                                lv[e] = (__bf16)(xv - (float)hh);
                            }
                            const uint32_t o2 = vo2 + 2u * (m * 32 + 8 * q);
                            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, hv), rh, o2, rowp * 128u, 0);
                            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, lv), rl, o2, rowp * 128u, 0);
                        }
                }
                // fp32 rounding bound of the 64-term sum
                if (onrm) {
                    const __amdgpu_buffer_rsrc_t rn = xp_rsrc(onrm + pix0);
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, sqrtf(s2) * 1.000004f), rn,
                                                          (xok && h == 0) ? (uint32_t)(x * 4) : XP_OOB, rowp * 4u, 0);
                }
            }
        }
    }
}

template <bool FIRST, bool LAST, bool IN_CB, bool OUT_CB, bool F16, bool OSPL = false>
__global__ __launch_bounds__(512) void conv64_x6p_kernel(const float *__restrict__ in, int Hin, int Win,
                                                         const float *__restrict__ w1blob,
                                                         const float *__restrict__ wkblob,
                                                         float *__restrict__ out, int Hout, int Wout,
                                                         uint16_t *__restrict__ ohi, uint16_t *__restrict__ olo,
                                                         float *__restrict__ onrm, XpBatch bt,
                                                         const float *__restrict__ in_amax, float *__restrict__ out_amax)
{
    extern __shared__ __attribute__((aligned(16))) char xsm[];
    // FIRST: the stager wave's image window
    float *win = reinterpret_cast<float *>(xsm + 2 * XP_STAGE) + ((threadIdx.x >> 6) & 3) * XP_WIN;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const bool mfma_wave = wave < 4;            // waves 4..7 stage the input
    constexpr int XP_WROWS = LAST ? 4 : (FIRST ? XP_WR_FIRST : XP_WR_MID), MW = 8 / XP_WROWS;
    static_assert(XP_WROWS == 4 || XP_WROWS == 8, "wave mapping");
    // MFMA wave: output rows XP_WROWS*g .. +XP_WROWS-1, M-tiles mt0 .. mt0+MW-1
    // wave-uniform by construction; readfirstlane tells the compiler (SGPR row offsets, scalar branches)
    const int g = __builtin_amdgcn_readfirstlane(XP_WROWS == 4 ? (wave & 3) : ((wave >> 1) & 1));
    const int mt0 = __builtin_amdgcn_readfirstlane(XP_WROWS == 4 ? 0 : (wave & 1));
    const int st = tid - XP_STAGERS;            // stager thread index (valid when !mfma_wave)
    constexpr int NP = F16 ? 2 : 3;
    constexpr int AL = XP_AL(F16, XP_WROWS);
    const float *bias = wkblob;
    const uint4 *wf = reinterpret_cast<const uint4 *>(wkblob + (F16 ? LK_F16 : NF + LK_W));
    // B fragment: plane (part, h), input row XP_WROWS*g + r + ky, pixel j + kx
    const int bbase = (lane >> 5) * XP_PLANE + ((XP_WROWS * g) * XP_IX + (lane & 31)) * 16;

    int tile = blockIdx.x;
    if (tile >= bt.ntiles) return;
    const float *hdr = wkblob + LK_F16 + LK_W;
    // F16 scalings of a tile (per image: each image has its own bound words; re-read only when
    // the tile's image changes -- tiles run image-major)
    int sc_img = -1;
    float sc_s = 1.0f, sc_u = 1.0f;
    auto scales = [&](int t, float &sc, float &usc) {
        if (F16) {
            const int im = t / bt.tiles_img;
            if (im != sc_img) {
                xp_scales(FIRST, in_amax + im * bt.amax_stride, hdr, sc_s, sc_u);
                sc_img = im;
            }
        }
        sc = sc_s;
        usc = sc_u;
    };
    if (!mfma_wave) {
        xp_stager_loop<FIRST, IN_CB, F16>(xsm, in, Hin, Win, bt, st, in_amax, hdr, w1blob, win);
        return;
    }
    if (OSPL) xp_publish_scale(FIRST, bt, in_amax, hdr, out_amax);
    float *lbias = reinterpret_cast<float *>(xsm + XP_BIAS_OFF);
    if (wave == 0) lbias[lane] = bias[lane];   // published by the first barrier below
    const float4 *lbias4 = reinterpret_cast<const float4 *>(lbias);
    XpFrag a[MW], an[AL][MW];
#pragma unroll
    for (int m = 0; m < MW; m++) {
        a[m] = xp_afrag<NP>(wf, mt0 + m, 0, 0, lane);
#pragma unroll
        for (int k = 0; k < AL; k++) an[k][m] = xp_afrag<NP>(wf, mt0 + m, 0, 1 + k, lane);
    }
    __syncthreads();

    uint32_t amax_run = 0u;
    int amax_img = -1, osc_img = -1;
    float osc = 1.0f;
    int cur = 0;
    for (; tile < bt.ntiles; tile += gridDim.x) {
        int img, ty0, tx0;
        xp_tile(bt, tile, img, ty0, tx0);
        floatx16 acc[XP_ACC];
#pragma unroll
        for (int r = 0; r < XP_ACC; r++) acc[r] = floatx16{0};

#pragma unroll 1
        for (int cb = 0; cb < XP_NCB; cb++) {
            const int ncb = (cb + 1) & (XP_NCB - 1);
            xp_cblock<F16, XP_WROWS>(acc, a, an, wf, mt0, cb, ncb, lane, xsm + cur * XP_STAGE + bbase);
            if (cb == XP_NCB - 1) {
                float unscale = 1.0f;
                if (F16) {
                    float s_unused;
                    scales(tile, s_unused, unscale);
                }
                float oscale = 1.0f;
                if (OSPL) {
                    if (img != osc_img) {
                        osc = xp_out_scale(FIRST, in_amax + img * bt.amax_stride, hdr);
                        osc_img = img;
                    }
                    oscale = osc;
                }
                xp_epilogue<LAST, OUT_CB, F16, XP_WROWS, OSPL>(acc, lane, g, mt0, img, ty0, tx0, unscale, lbias4, out,
                                                               Hout, Wout, bt, ohi, olo, onrm, amax_run, amax_img,
                                                               out_amax, oscale);
            }
            __syncthreads();
            cur ^= 1;
        }
    }
    if (F16 && !LAST) xp_flush_amax(amax_run, amax_img, lane, out_amax, bt.amax_stride);
}

}  // namespace sde
#include "tower_wino.h"
// A/B timing builds substitute a probe copy of this header (tools/build_file_variant.sh -DSDE_H16_HEADER=...)
#ifdef SDE_H16_HEADER
#include SDE_H16_HEADER
#else
#include "tower_h16.h"
#endif
#include "tower_h16q.h"
#ifndef SDE_H16_L2
#define SDE_H16_L2 1   // 0: layer 2 on conv64_x6p_kernel (32x32x16), for A/B builds
#endif
#ifndef SDE_H16Q
#define SDE_H16Q 1   // 0: timing builds only -- middle split layers on conv64_h16_kernel's 8-wave form
#endif
namespace sde {


// max |x| over n floats, atomically maxed (as float bits) into *amax (F16 tower scaling):
// float4 grid-stride loads, one atomic per workgroup.
__global__ __launch_bounds__(256) void absmax_kernel(const float *__restrict__ x, int64_t n, float *__restrict__ amax,
                                                     int amax_stride)
{
    x += blockIdx.y * n;        // batch: image blockIdx.y -> amax[blockIdx.y * amax_stride]
    amax += blockIdx.y * amax_stride;
    float m = 0.0f;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (int64_t)gridDim.x * blockDim.x;
    const int64_t head = std::min<int64_t>(n, (16 - (reinterpret_cast<uintptr_t>(x) & 15)) / 4 & 3);
    if (tid < head) m = fabsf(x[tid]);
    const float4 *x4 = reinterpret_cast<const float4 *>(x + head);
    const int64_t n4 = (n - head) / 4;
    for (int64_t i = tid; i < n4; i += nt) {
        const float4 v = x4[i];
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    for (int64_t i = head + 4 * n4 + tid; i < n; i += nt) m = fmaxf(m, fabsf(x[i]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    __shared__ float red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0)
        atomicMax(reinterpret_cast<unsigned int *>(amax),
                  __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
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

// Per-image statistics exactly as NumPy computes them for match_single.py:40-41 (float32 image,
// np.mean / np.std over axes (0, 1)): the reduction over both axes of a contiguous 2-D array adds,
// from 0.0f in order, the pairwise sums (numpy pairwise_sum: blocks <= 128 with 8 accumulators,
// larger blocks halved at a multiple of 8) of consecutive 8192-element pieces of the flattened
// image (np.getbufsize()); mean = S / n in float32; std = sqrt(S' / n) with S' the same reduction
// of (x - mean)^2 (float32 ops, no contraction: the library is built with -ffp-contract=off).
// Pinned against NumPy in tests (test_preprocess_u8: bit-identical at every config size).
// Scratch per image: [mean, std, -, -][piece sums][piece sums of squares].
constexpr int NP_PIECE = 8192;

__device__ __forceinline__ float np_val(const uint8_t *img, int64_t i, float mean, bool sq)
{
    const float x = (float)img[i];
    if (!sq) return x;
    const float d = x - mean;
    return d * d;
}

// numpy pairwise_sum of a block of len <= 128 elements at s
__device__ float np_leaf(const uint8_t *img, int64_t s, int len, float mean, bool sq)
{
    if (len < 8) {
        float res = 0.0f;
        for (int i = 0; i < len; i++) res += np_val(img, s + i, mean, sq);
        return res;
    }
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; j++) r[j] = np_val(img, s + j, mean, sq);
    int i = 8;
    for (; i < len - (len % 8); i += 8) {
#pragma unroll
        for (int j = 0; j < 8; j++) r[j] += np_val(img, s + i + j, mean, sq);
    }
    float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < len; i++) res += np_val(img, s + i, mean, sq);
    return res;
}

__device__ __forceinline__ int np_half(int len) { const int n2 = len / 2; return n2 - n2 % 8; }

// One wave per 8192-element piece: its pairwise sum into the image's scratch.  A full piece is a
// perfect tree of 64 blocks of 128 (lane l sums block l; the xor-butterfly adds adjacent subtrees,
// and float addition is commutative); the last, short piece walks numpy's recursion: every lane
// enumerates the blocks in order (lane k % 64 sums block k into LDS), lane 0 adds them up the tree.
// S = 0.0f + v[0] + v[1] + ... in order (np.mean's / np.std's float32 reduction of the piece sums), then the
// quotient: the wave loads the sums into LDS (one round of latency), lane 0 adds them.  NumPy 2.x divides
// the float32 sum by the intp count in float64 and rounds once to float32 (np.mean: ret.dtype.type(ret /
// rcount); _var: true_divide by an intp into a float32 out, and its final ret / rcount), so the quotient
// is formed in fp64 here too.  Below 2^24 pixels this equals the float32 quotient S / (float)n (fp64 has
// more than 2 * 24 + 2 bits: the double rounding is innocuous); above it (float)n would be inexact.
__device__ __forceinline__ float np_stat(const float *__restrict__ v, int npieces, int64_t n, float *buf, int lane)
{
    float q = 0.0f;
    for (int c0 = 0; c0 < npieces; c0 += 256) {   // LDS chunks of 256 sums
        const int m = min(256, npieces - c0);
        for (int c = lane; c < m; c += 64) buf[c] = v[c0 + c];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (lane == 0)
            for (int c = 0; c < m; c++) q += buf[c];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    q = __shfl(q, 0, 64);
    return (float)((double)q / (double)n);
}

// SQ: the pass over (x - mean)^2, the mean formed here from the first pass's piece sums (the launch of a
// separate statistics kernel saved); block 0 also stores it.  Scratch per image: [mean, std, -, -][piece
// sums][piece sums of squares].
template <bool SQ>
__global__ __launch_bounds__(64) void np_piece_kernel(const uint8_t *__restrict__ imgs, int64_t n, int sstride,
                                                      float *__restrict__ scratch)
{
    const uint8_t *img = imgs + blockIdx.y * n;
    float *st = scratch + (size_t)blockIdx.y * sstride;
    const int npieces = gridDim.x;
    __shared__ float sbuf[256];
    float mean = 0.0f;
    if (SQ) {
        mean = np_stat(st + 4, npieces, n, sbuf, threadIdx.x);
        if (blockIdx.x == 0 && threadIdx.x == 0) st[0] = mean;
    }
    const int lane = threadIdx.x;
    const int64_t c0 = (int64_t)blockIdx.x * NP_PIECE;
    const int m = (int)std::min<int64_t>(NP_PIECE, n - c0);
    float sum;
    if (m == NP_PIECE) {
        sum = np_leaf(img, c0 + 128 * lane, 128, mean, SQ);
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) sum += __shfl_xor(sum, o, 64);
    } else {
        __shared__ float leaf[256];
        {
            int ss[16], sl[16], sp = 0, k = 0;
            ss[0] = 0; sl[0] = m;
            while (sp >= 0) {
                const int s0 = ss[sp], len = sl[sp];
                sp--;
                if (len <= 128) {
                    if ((k & 63) == lane) leaf[k] = np_leaf(img, c0 + s0, len, mean, SQ);
                    k++;
                } else {
                    const int n2 = np_half(len);
                    ss[++sp] = s0 + n2; sl[sp] = len - n2;     // right, visited second
                    ss[++sp] = s0; sl[sp] = n2;                // left first
                }
            }
        }
        __syncthreads();
        sum = 0.0f;
        if (lane == 0) {
            // post-order evaluation of the same tree over the block sums
            int fl[16], fs[16], sp = 0, k = 0;
            float fv[16], ret = 0.0f;
            fl[0] = m; fs[0] = 0;
            while (sp >= 0) {
                const int len = fl[sp];
                if (len <= 128) {
                    ret = leaf[k++];
                    sp--;
                } else if (fs[sp] == 0) {
                    fs[sp] = 1;
                    ++sp; fl[sp] = np_half(len); fs[sp] = 0;
                    continue;
                } else if (fs[sp] == 1) {
                    fv[sp] = ret;
                    fs[sp] = 2;
                    const int n2 = np_half(len);
                    ++sp; fl[sp] = len - n2; fs[sp] = 0;
                    continue;
                } else {
                    ret = fv[sp] + ret;
                    sp--;
                }
                // deliver ret to the parent frame (handled at its next visit)
            }
            sum = ret;
        }
    }
    if (lane == 0) st[4 + (SQ ? npieces : 0) + blockIdx.x] = sum;
}

// (I - mean) / std in float32 (match_single.py:40-41), zero border (process_functional.py:13-19).
constexpr int ZN_PER = 8;   // padded pixels per thread of znorm_pad_kernel

// The std formed here (every block, from the second pass's piece sums: np_stat by its first wave) -- the
// launch of a separate statistics kernel saved; block 0 stores it in the scratch's std word.
__global__ __launch_bounds__(256) void znorm_pad_kernel(const uint8_t *__restrict__ img, int H, int W, int pad,
                                                        float *__restrict__ scratch, int sstride, int npieces,
                                                        float *__restrict__ out)
{
    const int Wp = W + 2 * pad;
    img += (size_t)blockIdx.y * H * W;      // batch: image blockIdx.y
    float *st = scratch + (size_t)blockIdx.y * sstride;
    out += (size_t)blockIdx.y * (H + 2 * pad) * Wp;
    __shared__ float sbuf[256];
    __shared__ float sstd;
    if (threadIdx.x < 64) {
        const float v = sqrtf(np_stat(st + 4 + npieces, npieces, (int64_t)H * W, sbuf, threadIdx.x));
        if (threadIdx.x == 0) {
            sstd = v;
            if (blockIdx.x == 0) st[1] = v;
        }
    }
    __syncthreads();
    const float mean = st[0], stdv = sstd;
    const int64_t np_ = (int64_t)(H + 2 * pad) * Wp;
#pragma unroll
    for (int k = 0; k < ZN_PER; k++) {   // ZN_PER pixels per thread: the block's statistics amortised
        const int64_t i = ((int64_t)blockIdx.x * ZN_PER + k) * blockDim.x + threadIdx.x;
        if (i >= np_) break;
        // the padded image has < 2^31 pixels (checked by sde_preprocess_u8_batch)
        const int ii = (int)i;
        const int y = ii / Wp - pad, x = ii % Wp - pad;
        float v = 0.0f;
        if (y >= 0 && y < H && x >= 0 && x < W) v = ((float)img[(size_t)y * W + x] - mean) / stdv;
        out[i] = v;
    }
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

static constexpr int64_t TOWER_AMAX_BYTES = 256;   // 64 bound words (nlayers <= 64)
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
    // conv1 output bound terms for the F16 scaling (layer 2 computes conv1)
    float l1 = 0.0f, bmax = 0.0f;
    for (int n = 0; n < NF; n++) {
        double s = 0.0;
        for (int t = 0; t < 9; t++) s += std::fabs((double)hwio[0][t * NF + n]);
        l1 = std::max(l1, (float)(s * (1.0 + 1e-6)));   // rounded up: a bound of the f32 conv1
        bmax = std::max(bmax, std::fabs(biases[0][n]));
    }
    for (int l = 1; l < nlayers; l++) {
        for (int n = 0; n < NF; n++) o[n] = biases[l][n];
        float *w = o + NF;
        uint16_t *pl = reinterpret_cast<uint16_t *>(w + LK_W);
        // F16 parts of W * 2^tau, max |W| * 2^tau in [2^14, 2^15)
        float wmax = 0.0f;
        for (size_t i = 0; i < (size_t)LK_W; i++) wmax = std::max(wmax, std::fabs(hwio[l][i]));
        const int tau = (wmax > 0.0f && std::isfinite(wmax)) ? std::min(std::max(14 - std::ilogb(wmax), -100), 100) : 0;
        _Float16 *ph = reinterpret_cast<_Float16 *>(o + LK_F16);
        float *hdr = o + LK_F16 + LK_W;
        hdr[0] = std::ldexp(1.0f, -tau);
        hdr[1] = l1;
        hdr[2] = bmax;
        hdr[3] = 0.0f;
        {   // this layer's output bound terms (rounded up: bounds of the f32 sums)
            float lk = 0.0f, bk = 0.0f;
            for (int n = 0; n < NF; n++) {
                double s = 0.0;
                for (int i = 0; i < 9 * NF; i++) s += std::fabs((double)hwio[l][(size_t)i * NF + n]);
                lk = std::max(lk, (float)(s * (1.0 + 1e-6)));
                bk = std::max(bk, std::fabs(biases[l][n]));
            }
            hdr[4] = lk;
            hdr[5] = bk;
            hdr[6] = hdr[7] = 0.0f;
        }
        for (int tap = 0; tap < 9; tap++)
            for (int c = 0; c < NF; c++)
                for (int n = 0; n < NF; n++) {
                    const float x = std::ldexp(hwio[l][((size_t)tap * NF + c) * NF + n], tau);
                    const _Float16 h0 = (_Float16)x;
                    const _Float16 parts[2] = {h0, (_Float16)(x - (float)h0)};
                    const int mt = n >> 5, cb = c >> 4, ln = ((c >> 3) & 1) * 32 + (n & 31);
                    for (int q = 0; q < 2; q++)
                        ph[((((size_t)(mt * XP_NCB + cb) * 9 + tap) * 2 + q) * 64 + ln) * 8 + (c & 7)] = parts[q];
                }
        {
            // Winograd U = G g G^T per (n, c) in fp64, scaled by 2^tau_u (max |U| 2^tau_u in [2^14, 2^15)) and
            // split into two fp16 parts (the residual taken in fp64)
            static const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
            std::vector<double> U((size_t)16 * NF * NF);
            double umax = 0.0;
            for (int c = 0; c < NF; c++)
                for (int n = 0; n < NF; n++) {
                    double g[3][3];
                    for (int ky = 0; ky < 3; ky++)
                        for (int kx = 0; kx < 3; kx++) g[ky][kx] = hwio[l][((size_t)(ky * 3 + kx) * NF + c) * NF + n];
                    for (int i = 0; i < 4; i++)
                        for (int j = 0; j < 4; j++) {
                            double u = 0.0;
                            for (int ky = 0; ky < 3; ky++)
                                for (int kx = 0; kx < 3; kx++) u += G[i][ky] * g[ky][kx] * G[j][kx];
                            U[((size_t)(4 * i + j) * NF + n) * NF + c] = u;
                            umax = std::max(umax, std::fabs(u));
                        }
                }
            const int tu = (umax > 0.0 && std::isfinite(umax)) ? std::min(std::max(14 - std::ilogb(umax), -100), 100) : 0;
            _Float16 *pu = reinterpret_cast<_Float16 *>(o + LK_WINO);
            float *wh = o + LK_WHDR;
            wh[0] = std::ldexp(1.0f, -tu);
            wh[1] = wh[2] = wh[3] = 0.0f;
            for (int xi = 0; xi < 16; xi++)
                for (int n = 0; n < NF; n++)
                    for (int c = 0; c < NF; c++) {
                        const double x = std::ldexp(U[((size_t)xi * NF + n) * NF + c], tu);
                        const _Float16 h0 = (_Float16)x;
                        const _Float16 parts[2] = {h0, (_Float16)(x - (double)h0)};
                        const int mt = n >> 5, cb = c >> 4, ln = ((c >> 3) & 1) * 32 + (n & 31);
                        for (int q = 0; q < 2; q++)
                            pu[((((size_t)(xi * 2 + mt) * XP_NCB + cb) * 2 + q) * 64 + ln) * 8 + (c & 7)] = parts[q];
                    }
        }
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
                    const uint16_t parts[3] = {h0, h1, f2bf_rne(r2)};
                    // A-fragment order [mtile][cblock][tap][part][lane][8] (conv64_x6p_kernel):
                    // lane = (c % 16 >= 8) * 32 + n % 32, element c % 8
                    const int mt = n >> 5, cb = c >> 4, ln = ((c >> 3) & 1) * 32 + (n & 31);
                    for (int q = 0; q < 3; q++)
                        pl[((((size_t)(mt * XP_NCB + cb) * 9 + tap) * 3 + q) * 64 + ln) * 8 + (c & 7)] = parts[q];
                }
        o += LK_FLOATS;
    }
    return SDE_OK;
}

SDE_EXPORT int64_t sde_tower_batch_workspace_bytes(int H, int W, int nimg, int nlayers, int nf)
{
    if (H <= 0 || W <= 0 || nimg <= 0 || nlayers < 1 || nf != NF) return -1;
    if (nlayers == 1) return 0;
    // two ping-pong activation buffers sized for layer 2's output (nimg images each), then the
    // F16X3 bound words (64 per image)
    const int64_t h2 = H + 2 * (nlayers - 2), w2 = W + 2 * (nlayers - 2);
    return (nlayers > 2 ? 2 * nimg * h2 * w2 * NF * (int64_t)sizeof(float) : 0) + nimg * TOWER_AMAX_BYTES;
}

SDE_EXPORT int64_t sde_tower_workspace_bytes(int H, int W, int nlayers, int nf)
{
    return sde_tower_batch_workspace_bytes(H, W, 1, nlayers, nf);
}

static void set_tower_attrs()
{
    static std::atomic<uint64_t> done{0};
    once_per_device(done, [] {
    (void)hipFuncSetAttribute((const void *)conv64_mfma_kernel<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, TW_SMEM);
    (void)hipFuncSetAttribute((const void *)conv64_mfma_kernel<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, TW_SMEM);
    (void)hipFuncSetAttribute((const void *)conv64_mfma_kernel<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize, TW_SMEM);
    (void)hipFuncSetAttribute((const void *)conv64_mfma_kernel<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, TW_SMEM);
#define SDE_X6P_ATTR1(F, L, I, O, H) (void)hipFuncSetAttribute((const void *)conv64_x6p_kernel<F, L, I, O, H>, \
                                                             hipFuncAttributeMaxDynamicSharedMemorySize, XP_SMEM)
#define SDE_X6P_ATTR(F, L, I, O) SDE_X6P_ATTR1(F, L, I, O, false); SDE_X6P_ATTR1(F, L, I, O, true)
    SDE_X6P_ATTR(true, false, false, true);
    SDE_X6P_ATTR(true, false, false, false);
    SDE_X6P_ATTR(true, true, false, false);
    SDE_X6P_ATTR(false, false, true, true);
    SDE_X6P_ATTR(false, false, false, false);
    SDE_X6P_ATTR(false, false, true, false);
    SDE_X6P_ATTR(false, false, false, true);
    SDE_X6P_ATTR(false, true, true, false);
    SDE_X6P_ATTR(false, true, false, false);
    (void)hipFuncSetAttribute((const void *)conv64_x6p_kernel<true, false, false, false, true, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, XP_SMEM);
#undef SDE_X6P_ATTR1
#undef SDE_X6P_ATTR
#define SDE_H16_ATTR(L, I, O, S, ...) (void)hipFuncSetAttribute((const void *)conv64_h16_kernel<L, I, O, S, ##__VA_ARGS__>, \
                                                                hipFuncAttributeMaxDynamicSharedMemorySize, H16_SMEM)
    SDE_H16_ATTR(false, false, false, false, true, true);
    (void)hipFuncSetAttribute((const void *)conv64_h16q_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, H16_SMEM);
    (void)hipFuncSetAttribute((const void *)conv64_h16_kernel<false, false, true, false, false, false, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, H16_SMEM_FIRST);
    (void)hipFuncSetAttribute((const void *)conv64_h16_kernel<false, false, false, false, false, false, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, H16_SMEM_FIRST);
    (void)hipFuncSetAttribute((const void *)conv64_h16_kernel<false, false, false, false, false, true, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, H16_SMEM_FIRST);
    SDE_H16_ATTR(true, false, false, false, true, false);
    SDE_H16_ATTR(true, false, false, true, true, false);
    SDE_H16_ATTR(true, true, false, false);
    SDE_H16_ATTR(true, false, false, false);
    SDE_H16_ATTR(true, true, false, true);
    SDE_H16_ATTR(true, false, false, true);
    SDE_H16_ATTR(false, true, true, false);
    SDE_H16_ATTR(false, true, false, false);
    SDE_H16_ATTR(false, false, true, false);
    SDE_H16_ATTR(false, false, false, false);
#undef SDE_H16_ATTR
#define SDE_WINO_ATTR(L, I, O) (void)hipFuncSetAttribute((const void *)wino_kernel<L, I, O>, \
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, WN_SMEM)
    SDE_WINO_ATTR(true, true, false);
    SDE_WINO_ATTR(true, false, false);
    SDE_WINO_ATTR(false, true, true);
    SDE_WINO_ATTR(false, true, false);
    SDE_WINO_ATTR(false, false, true);
    SDE_WINO_ATTR(false, false, false);
#undef SDE_WINO_ATTR
    });
}

// Persistent tower grids: one workgroup per CU (160 KB of LDS each), or g_grid_cus workgroups when set
// (sde_set_persistent_grid: the tower sharing the device with other work on CU-masked streams, where a
// workgroup per device CU would leave the last ones waiting for CUs the other stream holds).
static std::atomic<int> g_grid_cus{0};

static int cu_count()
{
    static int cached[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cached[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cached[dev] = n;
    }
    const int g = g_grid_cus.load(std::memory_order_relaxed);
    return g > 0 ? std::min(g, cached[dev]) : cached[dev];
}

// One launch: layer == 2 -> conv1+conv2 fused from the padded image (Hin x Win floats);
// layer > 2 -> one 64->64 conv on Hin x Win x 64 activations.  Output (Hin-4|Hin-2) x ... x 64.
// in_cb / out_cb: activations in the c-block-major layout [4][h][w][16] (bf16x6 / f16x3 paths).
// F16X3: in_amax = bound of |input| (|image| for layer 2), out_amax = max of the ReLU outputs
// (zeroed by the caller; unused by the last layer).
// nimg images per launch (split arithmetics: one tile space over the batch; fp32: one launch per
// image): image i at in + i * in_stride, out + i * out_stride, bound words + i * amax_stride.
static void launch_layer(const float *in, int Hin, int Win, const float *packed, int nlayers, int layer, float *out,
                         int flags, uint16_t *ohi, uint16_t *olo, float *onrm, bool in_cb, bool out_cb,
                         const float *in_amax, float *out_amax, hipStream_t st, int nimg = 1, int64_t in_stride = 0,
                         int64_t out_stride = 0, int amax_stride = 0, bool in_sp = false, bool out_sp = false)
{
    set_tower_attrs();
    const bool last = (layer == nlayers);
    const bool f16 = (flags & SDE_TOWER_F16X3) != 0;
    const bool x6 = f16 || (flags & SDE_TOWER_BF16X6) != 0;
    const float *w1 = packed;
    const float *wk = packed + L1_FLOATS + (int64_t)(layer - 2) * LK_FLOATS;
    const int hout = Hin - (layer == 2 ? 4 : 2), wout = Win - (layer == 2 ? 4 : 2);
    // the Winograd kernel's input / output descriptors span a whole image with 32-bit record
    // counts and offsets (tower_wino.h): planes of 4 GiB or more take the direct kernel, which
    // rebases its descriptors per tile (same f16x3 arithmetic, fp32-level error either way)
    const bool wino_fits = (int64_t)Hin * Win * 256 < ((int64_t)1 << 32) &&
                           (int64_t)hout * wout * 256 < ((int64_t)1 << 32);
    if (f16 && layer >= 3 && !ohi && !onrm && (flags & SDE_TOWER_WINOGRAD) && wino_fits) {
        // Winograd F(2x2, 3x3) for the 64 -> 64 layers (tower_wino.h)
        XpBatch bt;
        bt.tiles_x = cdiv(wout, WN_TX);
        bt.tiles_img = bt.tiles_x * cdiv(hout, WN_TY);
        bt.ntiles = bt.tiles_img * nimg;
        bt.in_stride = in_stride;
        bt.out_stride = out_stride;
        bt.pix_stride = (int64_t)hout * wout;
        bt.amax_stride = amax_stride;
        const int grid = std::min(bt.ntiles, cu_count());
#define SDE_WINO(L, I, O) wino_kernel<L, I, O><<<grid, 512, WN_SMEM, st>>>(in, Hin, Win, wk, out, hout, wout, bt, \
                                                                          in_amax, out_amax)
        if (last) { if (in_cb) SDE_WINO(true, true, false); else SDE_WINO(true, false, false); }
        else if (in_cb) { if (out_cb) SDE_WINO(false, true, true); else SDE_WINO(false, true, false); }
        else { if (out_cb) SDE_WINO(false, false, true); else SDE_WINO(false, false, false); }
#undef SDE_WINO
        return;
    }
    if (f16 && layer == 2 && !last && !(flags & SDE_TOWER_MFMA32) && SDE_H16_L2) {
        // layer 2 (conv1 on the stagers + conv2) on v_mfma_f32_16x16x32_f16 (tower_h16.h)
        XpBatch bt;
        bt.tiles_x = cdiv(wout, XP_TX);
        bt.tiles_img = bt.tiles_x * cdiv(hout, XP_TY);
        bt.ntiles = bt.tiles_img * nimg;
        bt.in_stride = in_stride;
        bt.out_stride = out_stride;
        bt.pix_stride = (int64_t)hout * wout;
        bt.amax_stride = amax_stride;
        const int grid = std::min(bt.ntiles, cu_count());
        if (out_sp)
            conv64_h16_kernel<false, false, false, false, false, true, true><<<grid, 512, H16_SMEM_FIRST, st>>>(
                in, Hin, Win, wk, out, hout, wout, nullptr, nullptr, nullptr, bt, in_amax, out_amax, w1);
        else if (out_cb)
            conv64_h16_kernel<false, false, true, false, false, false, true><<<grid, 512, H16_SMEM_FIRST, st>>>(
                in, Hin, Win, wk, out, hout, wout, nullptr, nullptr, nullptr, bt, in_amax, out_amax, w1);
        else
            conv64_h16_kernel<false, false, false, false, false, false, true><<<grid, 512, H16_SMEM_FIRST, st>>>(
                in, Hin, Win, wk, out, hout, wout, nullptr, nullptr, nullptr, bt, in_amax, out_amax, w1);
        return;
    }
    if (f16 && layer >= 3 && !(flags & SDE_TOWER_MFMA32)) {
        // the 64 -> 64 layers on v_mfma_f32_16x16x32_f16 (tower_h16.h; same tiles as the direct kernel)
        XpBatch bt;
        bt.tiles_x = cdiv(wout, XP_TX);
        bt.tiles_img = bt.tiles_x * cdiv(hout, XP_TY);
        bt.ntiles = bt.tiles_img * nimg;
        bt.in_stride = in_stride;
        bt.out_stride = out_stride;
        bt.pix_stride = (int64_t)hout * wout;
        bt.amax_stride = amax_stride;
        const int grid = std::min(bt.ntiles, cu_count());
#define SDE_H16(L, I, O, S, ...) conv64_h16_kernel<L, I, O, S, ##__VA_ARGS__><<<grid, 512, H16_SMEM, st>>>( \
        in, Hin, Win, wk, out, hout, wout, (S) ? ohi : nullptr, (S) ? olo : nullptr, (S) ? onrm : nullptr, bt, in_amax, out_amax, \
        nullptr)
        const bool split = ohi || olo || onrm;
        if (in_sp) {   // split activations in (and out, below the last layer): LDS-DMA stagers
            if (!last && SDE_H16Q)   // the 4-wave kernel with resident weights (tower_h16q.h)
                conv64_h16q_kernel<<<grid, 256, H16_SMEM, st>>>(in, Hin, Win, wk, out, hout, wout, bt, in_amax, out_amax);
            else if (!last) SDE_H16(false, false, false, false, true, true);
            else if (split) SDE_H16(true, false, false, true, true, false);
            else SDE_H16(true, false, false, false, true, false);
            return;
        }
        if (last && split) { if (in_cb) SDE_H16(true, true, false, true); else SDE_H16(true, false, false, true); }
        else if (last) { if (in_cb) SDE_H16(true, true, false, false); else SDE_H16(true, false, false, false); }
        else if (in_cb) { if (out_cb) SDE_H16(false, true, true, false); else SDE_H16(false, true, false, false); }
        else { if (out_cb) SDE_H16(false, false, true, false); else SDE_H16(false, false, false, false); }
#undef SDE_H16
        return;
    }
    if (x6) {
        XpBatch bt;
        bt.tiles_x = cdiv(wout, XP_TX);
        bt.tiles_img = bt.tiles_x * cdiv(hout, XP_TY);
        bt.ntiles = bt.tiles_img * nimg;
        bt.in_stride = in_stride;
        bt.out_stride = out_stride;
        bt.pix_stride = (int64_t)hout * wout;
        bt.amax_stride = amax_stride;
        const int grid = std::min(bt.ntiles, cu_count());
#define SDE_X6P(F, L, I, O, H, ...) conv64_x6p_kernel<F, L, I, O, H, ##__VA_ARGS__><<<grid, 512, XP_SMEM, st>>>( \
        in, Hin, Win, (F) ? w1 : nullptr, wk, out, hout, wout, (L) ? ohi : nullptr, (L) ? olo : nullptr, \
        (L) ? onrm : nullptr, bt, in_amax, out_amax)
        if (out_sp) {   // layer 2 writing split activations (f16x3; the callers check)
            SDE_X6P(true, false, false, false, true, true);
            return;
        }
#define SDE_X6P_ALL(H)                                                      \
        if (layer == 2) {                                                   \
            if (last) SDE_X6P(true, true, false, false, H);                 \
            else if (out_cb) SDE_X6P(true, false, false, true, H);          \
            else SDE_X6P(true, false, false, false, H);                     \
        } else if (last) {                                                  \
            if (in_cb) SDE_X6P(false, true, true, false, H);                \
            else SDE_X6P(false, true, false, false, H);                     \
        } else {                                                            \
            if (in_cb && out_cb) SDE_X6P(false, false, true, true, H);      \
            else if (in_cb) SDE_X6P(false, false, true, false, H);          \
            else if (out_cb) SDE_X6P(false, false, false, true, H);         \
            else SDE_X6P(false, false, false, false, H);                    \
        }
        if (f16) { SDE_X6P_ALL(true) } else { SDE_X6P_ALL(false) }
#undef SDE_X6P_ALL
#undef SDE_X6P
        return;
    }
    dim3 grid(cdiv(wout, TW_TX), cdiv(hout, TW_TY));
    const int64_t pix = (int64_t)hout * wout;
    for (int i = 0; i < nimg; i++) {
        const float *ini = in + i * in_stride;
        float *outi = out + i * out_stride;
        uint16_t *hi = ohi ? ohi + i * pix * NF : nullptr, *lo = olo ? olo + i * pix * NF : nullptr;
        float *nr = onrm ? onrm + i * pix : nullptr;
#define SDE_CONV(K, F, L, SM) K<F, L><<<grid, 512, SM, st>>>(ini, Hin, Win, (F) ? w1 : nullptr, wk, outi, hout, wout, \
                                                             (L) ? hi : nullptr, (L) ? lo : nullptr, (L) ? nr : nullptr)
        if (layer == 2) { if (last) SDE_CONV(conv64_mfma_kernel, true, true, TW_SMEM); else SDE_CONV(conv64_mfma_kernel, true, false, TW_SMEM); }
        else { if (last) SDE_CONV(conv64_mfma_kernel, false, true, TW_SMEM); else SDE_CONV(conv64_mfma_kernel, false, false, TW_SMEM); }
#undef SDE_CONV
    }
}

// split activations (SDE_TOWER_IN_SPLIT / OUT_SPLIT): the scale word sits at bound word + XP_SCALE_WORD (so
// the bound-word arrays hold 64 words per image and a tower at most 32 layers), and a plane's bytes
// (h w 16) times 8 fit the 32-bit buffer offsets
static constexpr int64_t SPLIT_MAX_PIX = (int64_t)1 << 24;
#ifndef SDE_SPLIT_ACT
// 1: sde_tower_forward* pass split activations between the f16x3 64->64 layers (conv64_h16q_kernel in the
// middle); 0 (the default): fp32 c-blocks.  Same time within 0.5 % on MI355X (the tower is
// power-capped, and the split path moves the fp16 split from the stagers into the MFMA waves' epilogue);
// ops.TOWER_SPLIT_ACT mirrors this for the layer-by-layer drivers.
#define SDE_SPLIT_ACT 0
#endif
static bool split_ok(int nlayers, int64_t pix) { return nlayers <= XP_SCALE_WORD && pix < SPLIT_MAX_PIX; }
// the kernels that exist: layer 2 may write split planes; a middle layer reads them iff it writes them; the
// last layer may read them
// the pixel limit applies to the split plane itself: the input plane for IN_SPLIT, the output plane (what the
// forward checks for layer 2's split outputs, h2 * w2) for OUT_SPLIT
static bool split_pairing_ok(bool in_sp, bool out_sp, int layer, int nlayers, int Hin, int Win)
{
    if (!in_sp && !out_sp) return true;
    const int sh = layer == 2 ? 4 : 2;
    if ((in_sp && !split_ok(nlayers, (int64_t)Hin * Win)) || (out_sp && !split_ok(nlayers, (int64_t)(Hin - sh) * (Win - sh))))
        return false;
    if ((in_sp && layer == 2) || (out_sp && layer == nlayers)) return false;
    return layer == 2 || layer == nlayers || in_sp == out_sp;
}

SDE_EXPORT int sde_tower_split_act(void) { return SDE_SPLIT_ACT; }

static bool tower_flags_ok(int flags, bool layer_api)
{
    if (flags & (SDE_TOWER_IN_SPLIT | SDE_TOWER_OUT_SPLIT)) {   // F16X3 on the 16x16x32 kernel (layer API only)
        if (!layer_api || !(flags & SDE_TOWER_F16X3) || (flags & (SDE_TOWER_WINOGRAD | SDE_TOWER_MFMA32))) return false;
        if ((flags & SDE_TOWER_IN_SPLIT && flags & SDE_TOWER_IN_CBLOCK) ||
            (flags & SDE_TOWER_OUT_SPLIT && flags & SDE_TOWER_OUT_CBLOCK)) return false;
        flags &= ~(SDE_TOWER_IN_SPLIT | SDE_TOWER_OUT_SPLIT);
    }
    if (flags & (SDE_TOWER_WINOGRAD | SDE_TOWER_MFMA32)) {   // F16X3 only: the 64 -> 64 layers' kernel choice
        if (!(flags & SDE_TOWER_F16X3) || (flags & SDE_TOWER_WINOGRAD && flags & SDE_TOWER_MFMA32)) return false;
        flags &= ~(SDE_TOWER_WINOGRAD | SDE_TOWER_MFMA32);
    }
    const int prec = flags & (SDE_TOWER_BF16X6 | SDE_TOWER_F16X3);
    if (prec == (SDE_TOWER_BF16X6 | SDE_TOWER_F16X3)) return false;
    const int layout = SDE_TOWER_IN_CBLOCK | SDE_TOWER_OUT_CBLOCK;
    if (!layer_api) return (flags & ~(SDE_TOWER_BF16X6 | SDE_TOWER_F16X3)) == 0;
    if (flags & ~(SDE_TOWER_BF16X6 | SDE_TOWER_F16X3 | layout)) return false;
    return !((flags & layout) && prec == 0);
}

SDE_EXPORT int sde_tower_layer_scaled(const float *in, int Hin, int Win, const float *packed, int nlayers, int nf,
                                      int layer, float *out, int flags, uint16_t *feat_hi, uint16_t *feat_lo,
                                      float *feat_norm, const float *in_absmax, float *out_absmax, void *stream)
{
    if (!in || !packed || !out || nf != NF || nlayers < 2 || layer < 2 || layer > nlayers) return SDE_ERR_ARG;
    if (Hin < (layer == 2 ? 5 : 3) || Win < (layer == 2 ? 5 : 3)) return SDE_ERR_ARG;
    if (!tower_flags_ok(flags, true)) return SDE_ERR_ARG;
    const bool in_cb = (flags & SDE_TOWER_IN_CBLOCK) != 0, out_cb = (flags & SDE_TOWER_OUT_CBLOCK) != 0;
    if ((in_cb && layer == 2) || (out_cb && layer == nlayers)) return SDE_ERR_ARG;
    if ((feat_hi != nullptr) != (feat_lo != nullptr)) return SDE_ERR_ARG;
    if ((flags & SDE_TOWER_F16X3) && (!in_absmax || (layer < nlayers && !out_absmax))) return SDE_ERR_ARG;
    const bool in_sp = (flags & SDE_TOWER_IN_SPLIT) != 0, out_sp = (flags & SDE_TOWER_OUT_SPLIT) != 0;
    if (!split_pairing_ok(in_sp, out_sp, layer, nlayers, Hin, Win)) return SDE_ERR_ARG;
    launch_layer(in, Hin, Win, packed, nlayers, layer, out, flags, feat_hi, feat_lo, feat_norm, in_cb, out_cb,
                 in_absmax, out_absmax, as_stream(stream), 1, 0, 0, 0, in_sp, out_sp);
    return launch_status();
}

SDE_EXPORT int sde_tower_layer_batch(const float *in, int nimg, int64_t in_stride, int Hin, int Win,
                                     const float *packed, int nlayers, int nf, int layer, float *out,
                                     int64_t out_stride, int flags, const float *in_absmax, float *out_absmax,
                                     int amax_stride, void *stream)
{
    if (!in || !packed || !out || nf != NF || nlayers < 2 || layer < 2 || layer > nlayers || nimg <= 0) return SDE_ERR_ARG;
    if (Hin < (layer == 2 ? 5 : 3) || Win < (layer == 2 ? 5 : 3)) return SDE_ERR_ARG;
    if (!tower_flags_ok(flags, true)) return SDE_ERR_ARG;
    const bool in_cb = (flags & SDE_TOWER_IN_CBLOCK) != 0, out_cb = (flags & SDE_TOWER_OUT_CBLOCK) != 0;
    if ((in_cb && layer == 2) || (out_cb && layer == nlayers)) return SDE_ERR_ARG;
    const int64_t hout = Hin - (layer == 2 ? 4 : 2), wout = Win - (layer == 2 ? 4 : 2);
    const int64_t in_need = layer == 2 ? (int64_t)Hin * Win : (int64_t)Hin * Win * NF;
    if (nimg > 1 && (in_stride < in_need || out_stride < hout * wout * NF ||
                     (layer == nlayers && out_stride != hout * wout * NF))) return SDE_ERR_ARG;
    if ((flags & SDE_TOWER_F16X3) && (!in_absmax || (layer < nlayers && !out_absmax) || (nimg > 1 && amax_stride < 1)))
        return SDE_ERR_ARG;
    const bool in_sp = (flags & SDE_TOWER_IN_SPLIT) != 0, out_sp = (flags & SDE_TOWER_OUT_SPLIT) != 0;
    // split activations: a layer's scale word sits 32 words past its bound word, which is column <= 31 of the
    // image's row; rows of fewer than 64 words would put image i's scale word on image i + 1's bound words
    if (!split_pairing_ok(in_sp, out_sp, layer, nlayers, Hin, Win) ||
        ((in_sp || out_sp) && nimg > 1 && amax_stride < (int)(TOWER_AMAX_BYTES / sizeof(float))))
        return SDE_ERR_ARG;
    launch_layer(in, Hin, Win, packed, nlayers, layer, out, flags, nullptr, nullptr, nullptr, in_cb, out_cb,
                 in_absmax, out_absmax, as_stream(stream), nimg, in_stride, out_stride, amax_stride, in_sp, out_sp);
    return launch_status();
}

SDE_EXPORT int sde_tower_layer(const float *in, int Hin, int Win, const float *packed, int nlayers, int nf, int layer,
                               float *out, int flags, uint16_t *feat_hi, uint16_t *feat_lo, float *feat_norm,
                               void *stream)
{
    if (flags & SDE_TOWER_F16X3) return SDE_ERR_ARG;   // needs the bound words: sde_tower_layer_scaled
    return sde_tower_layer_scaled(in, Hin, Win, packed, nlayers, nf, layer, out, flags, feat_hi, feat_lo, feat_norm,
                                  nullptr, nullptr, stream);
}

SDE_EXPORT int sde_set_persistent_grid(int cus)
{
    if (cus < 0) return SDE_ERR_ARG;
    g_grid_cus.store(cus, std::memory_order_relaxed);
    return SDE_OK;
}

SDE_EXPORT int sde_absmax_f32(const float *x, int64_t n, float *absmax, void *stream)
{
    if (!absmax || n < 0) return SDE_ERR_ARG;
    if (n == 0) return SDE_OK;
    if (!x) return SDE_ERR_ARG;
    const int blocks = (int)std::min<int64_t>(256, cdiv(n, 256 * 16));
    absmax_kernel<<<blocks, 256, 0, as_stream(stream)>>>(x, n, absmax, 0);
    return launch_status();
}

SDE_EXPORT int sde_absmax_f32_batch(const float *x, int nimg, int64_t n, float *absmax, int absmax_stride, void *stream)
{
    if (!absmax || n < 0 || nimg <= 0 || nimg > 65535 || absmax_stride < 0) return SDE_ERR_ARG;
    if (n == 0) return SDE_OK;
    if (!x) return SDE_ERR_ARG;
    const int blocks = (int)std::min<int64_t>(std::max(1, 256 / nimg), cdiv(n, 256 * 16));
    absmax_kernel<<<dim3(blocks, nimg), 256, 0, as_stream(stream)>>>(x, n, absmax, absmax_stride);
    return launch_status();
}

SDE_EXPORT int sde_tower_forward_batch(const float *img_pad, int nimg, int H, int W, const float *packed, int nlayers,
                                       int nf, float *feat, void *workspace, int64_t workspace_bytes, int flags,
                                       uint16_t *feat_hi, uint16_t *feat_lo, float *feat_norm, void *stream)
{
    if ((feat_hi != nullptr) != (feat_lo != nullptr)) return SDE_ERR_ARG;
    if (nlayers == 1 && (feat_hi || feat_norm)) return SDE_ERR_ARG;
    if (!img_pad || !packed || !feat || H <= 0 || W <= 0 || nimg <= 0 || nlayers < 1 || nf != NF) return SDE_ERR_ARG;
    if (!tower_flags_ok(flags, false)) return SDE_ERR_ARG;
    const int64_t need = sde_tower_batch_workspace_bytes(H, W, nimg, nlayers, nf);
    if (need > 0 && (!workspace || workspace_bytes < need)) return SDE_ERR_WORKSPACE;
    hipStream_t st = as_stream(stream);
    const int Hp = H + 2 * nlayers, Wp = W + 2 * nlayers;
    const int64_t img_stride = (int64_t)Hp * Wp, feat_stride = (int64_t)H * W * NF;
    if (nlayers == 1) {
        for (int i = 0; i < nimg; i++)
            conv1_only_kernel<<<cdiv((int64_t)H * W, 256), 256, 0, st>>>(img_pad + i * img_stride, Hp, Wp, packed,
                                                                         feat + i * feat_stride);
        return launch_status();
    }
    float *buf[2] = {nullptr, nullptr};
    const int64_t h2 = H + 2 * (nlayers - 2), w2 = W + 2 * (nlayers - 2);
    const int64_t act_stride = h2 * w2 * NF;   // per image, sized for layer 2's output
    if (nlayers > 2) {
        buf[0] = reinterpret_cast<float *>(workspace);
        buf[1] = buf[0] + nimg * act_stride;
    }
    // F16X3 bound words: amax[i * 64 + l - 2] bounds |input of layer l| of image i
    float *amax = reinterpret_cast<float *>(static_cast<char *>(workspace) +
                                            (nlayers > 2 ? 2 * nimg * act_stride * 4 : 0));
    constexpr int AS = (int)(TOWER_AMAX_BYTES / 4);
    const bool f16 = (flags & SDE_TOWER_F16X3) != 0;
    if (f16) {
        if (nlayers > AS) return SDE_ERR_ARG;
        if (hipMemsetAsync(amax, 0, nimg * TOWER_AMAX_BYTES, st) != hipSuccess) return SDE_ERR_LAUNCH;
        // one launch for the batch: per-image bound words amax[i * AS]
        const int blocks = (int)std::min<int64_t>(std::max<int64_t>(1, 256 / nimg), cdiv(img_stride, 256 * 16));
        absmax_kernel<<<dim3(blocks, nimg), 256, 0, st>>>(img_pad, img_stride, amax, AS);
    }
    int hin = Hp, win = Wp;
    // intermediate activations: f16x3 on the 16x16x32 kernel -- split (scaled fp16 parts, staged by LDS-DMA);
    // the other split paths -- c-block-major fp32
    const bool sp = SDE_SPLIT_ACT && f16 && !(flags & (SDE_TOWER_WINOGRAD | SDE_TOWER_MFMA32)) && nlayers > 2 &&
                    split_ok(nlayers, h2 * w2);
    const bool cbl = !sp && (flags & (SDE_TOWER_BF16X6 | SDE_TOWER_F16X3)) != 0;
    launch_layer(img_pad, hin, win, packed, nlayers, 2, nlayers == 2 ? feat : buf[0], flags, feat_hi, feat_lo, feat_norm,
                 false, cbl && nlayers > 2, amax, amax + 1, st, nimg, img_stride,
                 nlayers == 2 ? feat_stride : act_stride, AS, false, sp);
    hin -= 4; win -= 4;
    int cur = 0;
    for (int l = 3; l <= nlayers; l++) {
        float *o = (l == nlayers) ? feat : buf[cur ^ 1];
        launch_layer(buf[cur], hin, win, packed, nlayers, l, o, flags, feat_hi, feat_lo, feat_norm, cbl,
                     cbl && l < nlayers, amax + (l - 2), amax + (l - 1), st, nimg, act_stride,
                     l == nlayers ? feat_stride : act_stride, AS, sp, sp && l < nlayers);
        hin -= 2; win -= 2;
        cur ^= 1;
    }
    return launch_status();
}

SDE_EXPORT int sde_tower_forward(const float *img_pad, int H, int W, const float *packed, int nlayers, int nf,
                                 float *feat, void *workspace, int64_t workspace_bytes, int flags, uint16_t *feat_hi,
                                 uint16_t *feat_lo, float *feat_norm, void *stream)
{
    return sde_tower_forward_batch(img_pad, 1, H, W, packed, nlayers, nf, feat, workspace, workspace_bytes, flags,
                                   feat_hi, feat_lo, feat_norm, stream);
}

SDE_EXPORT int64_t sde_preprocess_scratch_bytes(int H, int W)
{
    if (H <= 0 || W <= 0) return -1;
    const int64_t pieces = ((int64_t)H * W + NP_PIECE - 1) / NP_PIECE;
    return ((4 + 2 * pieces) * 4 + 255) / 256 * 256;
}

SDE_EXPORT int sde_preprocess_u8_batch(const uint8_t *imgs, int nimg, int H, int W, int pad, float *out_pad,
                                       void *scratch, void *stream)
{
    if (!imgs || !out_pad || !scratch || nimg <= 0 || nimg > 65535 || H <= 0 || W <= 0 || pad < 0) return SDE_ERR_ARG;
    const int64_t n = (int64_t)(H + 2 * pad) * (W + 2 * pad);
    if (n >= ((int64_t)1 << 31)) return SDE_ERR_ARG;       // znorm_pad_kernel's 32-bit pixel index
    hipStream_t st = as_stream(stream);
    const int64_t npix = (int64_t)H * W;
    const int pieces = (int)((npix + NP_PIECE - 1) / NP_PIECE);
    const int sstride = (int)(sde_preprocess_scratch_bytes(H, W) / 4);
    float *sc = reinterpret_cast<float *>(scratch);
    np_piece_kernel<false><<<dim3(pieces, nimg), 64, 0, st>>>(imgs, npix, sstride, sc);
    np_piece_kernel<true><<<dim3(pieces, nimg), 64, 0, st>>>(imgs, npix, sstride, sc);
    znorm_pad_kernel<<<dim3((unsigned)cdiv(n, 256 * ZN_PER), nimg), 256, 0, st>>>(imgs, H, W, pad, sc, sstride, pieces,
                                                                                  out_pad);
    return launch_status();
}

SDE_EXPORT int sde_preprocess_u8(const uint8_t *img, int H, int W, int pad, float *out_pad, void *scratch,
                                 void *stream)
{
    return sde_preprocess_u8_batch(img, 1, H, W, pad, out_pad, scratch, stream);
}
