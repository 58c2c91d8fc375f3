// cbca.hip -- cross-based cost aggregation on [H][W][D] volumes (gfx950).
//
// BUILD-DEFINED stage: the reference has no CBCA (only the
// buffer name d_cost_volumel_after_aggr, process_functional.py:268,347, and an
// unused timer label, match.py:98).  The definition (v2, round 4) is stated once
// in the CPU restatement under oracle/ (test infrastructure); these kernels
// reproduce it bit for bit:
//  - every volume is aggregated in LEFT coordinates; a voxel is valid iff its
//    right-image pixel q - d is inside the image, and invalid voxels pass through;
//  - support arms = min(left-image arm at q, right-image arm at q - d), so the
//    right-referenced volume's aggregation is the shear of the left one's: the GPU
//    path aggregates ONE volume and writes the other as its shear (sde_cbca_lr);
//  - prefix chains (fp64, sequential) restart per segment of SDE_CBCA_SEG
//    positions at kS - M (M = L1 - 1): any wave can take any segment after an
//    M-position pre-roll, so the passes are persistent, load-balanced grids;
//  - the mean multiplies by the correctly rounded fp64 reciprocal of the exact
//    integer count (sde_cbca_reciprocals exposes the kernels' values).
//
// Mapping (both passes): one wave per (line, 64-disparity chunk, segment) item,
// lane = d, so each step moves one 256-B run of the HWD volume.  The chain P is the
// wave's running state; the last 2R+2 prefixes live in a wave-private LDS ring, so
// an output is two LDS reads at per-lane slots and one subtraction, trailing the
// front by R >= M positions.  Per step the only vector-memory operations are the
// cost load (prefetched a whole ring ahead, PF = 2R+2 positions: ~7 KB in flight
// per wave) and the output store; the arms come in once per ring block:
//  - horizontal pass: the left-image arms of the block's trailing positions are
//    one dword per lane, read back with v_readlane; the right-image arm of lane i
//    at position t is the value lane i-1 held at t-1, so it rides a DPP wave_shr:1
//    chain fed at lane 0;
//  - vertical pass: both images' arms come from a column-major copy in the
//    workspace (sde_cbca_workspace_bytes), the right image's as one dwordx4 per
//    lane per four rows.
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

// Column-major copy of the arms, aT[x * Hp + y] (Hp = H rounded up to 4: a lane's dwordx4 of four
// rows is 16-B aligned).  32 x 32 tiles through LDS.
__global__ __launch_bounds__(256) void cbca_transpose_kernel(const uint32_t *__restrict__ a, uint32_t *__restrict__ aT,
                                                             int H, int W, int Hp)
{
    __shared__ uint32_t t[32][33];
    const int x0 = blockIdx.x * 32, y0 = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
    for (int i = 0; i < 32; i += 8) {
        const int y = y0 + ty + i, x = x0 + tx;
        t[ty + i][tx] = (y < H && x < W) ? a[(size_t)y * W + x] : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 32; i += 8) {
        const int x = x0 + ty + i, y = y0 + tx;
        if (x < W && y < Hp) aT[(size_t)x * Hp + y] = t[tx][ty + i];
    }
}

// Cache policy of the cost streams (aux bit 1 = nt on gfx950): each voxel is read once and written
// once per pass (round 2: nontemporal both ways, 1.513 -> 1.468 ms per pair iteration).
#ifndef CBCA_NT
#define CBCA_NT 3
#endif
constexpr uint32_t CB_OOB = 0x80000000u;    // a voffset past every range: load 0, store dropped

// Buffer descriptor (wave-uniform inputs only) for raw dword loads/stores with a 32-bit per-lane
// voffset, an SGPR soffset and the hardware range check on voffset (>= bytes: load 0, store
// dropped; every range below is < 2^31, so a voffset of CB_OOB is always out of range).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t cb_rsrc(const void *base, uint32_t bytes)
{
    const uintptr_t b = (uintptr_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    void *p = (void *)(((uintptr_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, 0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t ruint(uint32_t v, int lane) { return (uint32_t)__builtin_amdgcn_readlane((int)v, lane); }

// (x + RS) mod RS for x in [-RS, RS): x + RS, then min_u32 with x + RS - RS (wraps huge when < 0)
template <int RS>
__device__ __forceinline__ uint32_t ring_slot(int x)
{
    const uint32_t u = (uint32_t)(x + RS);
    return min(u, u - (uint32_t)RS);
}

// Correctly rounded 1/c for the exact support counts (1 <= c <= (2*31+1)^2): v_rcp_f64 and two
// Newton steps; sde_cbca_reciprocals returns these values (the tests compare them with the IEEE
// quotient for every count).
__device__ __forceinline__ double cb_recip(uint32_t c)
{
    const double cd = (double)c;
    double r = __builtin_amdgcn_rcp(cd);
    double e = __builtin_fma(-cd, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-cd, r, 1.0);
    return __builtin_fma(r, e, r);
}

struct CbcaArgs {
    const float *src;
    float *dst;
    const uint32_t *al, *ar;       // row-major arms (left / right image): horizontal pass
    const uint32_t *alT, *arT;     // column-major arms (pitch Hp): vertical pass
    int H, W, D, M, Hp;
    int nseg, ndc;
    int64_t nitems;
    int per;                       // items per wave (contiguous range)
    int64_t chunk_first[9];        // vertical pass: first item of chunk c (valid columns only)
};

// ---------------------------------------------------------------------------------------------
// Horizontal pass: item = (row y, chunk c, segment k), k fastest, so a wave's consecutive items
// are consecutive segments of one row.
// ---------------------------------------------------------------------------------------------
// Opaque to the optimiser: keeps a per-step offset an incremented register instead of 2R+2
// block-invariant constants hoisted out of the loop (SGPR pressure, spills, drained prefetch).
__device__ __forceinline__ uint32_t opq_s(uint32_t v)
{
    asm volatile("" : "+s"(v));
    return v;
}
__device__ __forceinline__ uint32_t opq_v(uint32_t v)
{
    asm volatile("" : "+v"(v));
    return v;
}

template <int R>
__device__ __forceinline__ void cbca_h_item(const CbcaArgs &A, int y, int c, int k, double *__restrict__ sP)
{
    constexpr int RS = 2 * R + 2, PF = RS;
    const int lane = threadIdx.x;
    const int W = A.W, D = A.D, M = A.M;
    const int d0 = 64 * c, d = d0 + lane;
    const int t0 = k * SDE_CBCA_SEG, t1 = min(t0 + SDE_CBCA_SEG, W);
    if (t1 <= d0) return;                          // every voxel of the segment is invalid
    const int fs = max(t0 - M, d0);                // walk start = lane 0's chain base
    const int fe = t1 - 1 + R;                     // last front position (output t1 - 1)
    const uint32_t D4 = 4u * (uint32_t)D;
    const uint32_t dl4 = 4u * (uint32_t)min(d, D - 1);
    const uint32_t rowbytes = 4u * (uint32_t)W * (uint32_t)D;
    const __amdgpu_buffer_rsrc_t rc = cb_rsrc(A.src + (size_t)y * W * D, rowbytes);
    const __amdgpu_buffer_rsrc_t rd = cb_rsrc(A.dst + (size_t)y * W * D, rowbytes);
    const __amdgpu_buffer_rsrc_t ra = cb_rsrc(A.al + (size_t)y * W, 4u * W);
    const __amdgpu_buffer_rsrc_t rb = cb_rsrc(A.ar + (size_t)y * W, 4u * W);
    // a lane stores output t iff t >= th = max(t0, d) (valid voxel of this segment) and d < D
    const int th = d < D ? max(t0, d) : 0x7FFFFFFF;

    float cr[PF];
    // block arms: lane j (< RS) holds the left-image arm at the block's trailing position tb + j and
    // the right-image arm at tb + j - d0 (outside the row: 0, only ever used by invalid lanes)
    auto arms_blk = [&](int tb, uint32_t &av, uint32_t &bv) {
        av = __builtin_amdgcn_raw_buffer_load_b32(ra, 4u * (uint32_t)(tb + lane), 0, 0);
        bv = __builtin_amdgcn_raw_buffer_load_b32(rb, 4u * (uint32_t)(tb + lane - d0), 0, 0);
    };
#pragma unroll
    for (int j = 0; j < PF; j++)
        cr[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rc, dl4, (int)(D4 * (uint32_t)min(fs + j, W - 1)),
                                                                               CBCA_NT & 1 ? 2 : 0));
    uint32_t Ab, Bb, An, Bn;
    arms_blk(fs - R, Ab, Bb);
    // right-image arm of the trailing position, lane i = pixel t - d0 - i: the state before step fs
    uint32_t X = __builtin_amdgcn_raw_buffer_load_b32(rb, 4u * (uint32_t)(fs - R - 1 - d0 - lane), 0, 0);
    double P = 0.0;
    sP[(RS - 1) * 64 + lane] = 0.0;               // P(fs - 1) = 0: read before position fs + RS - 1 lands
    // per-lane store offset of output t (4d + 4tD), advanced every step
    uint32_t vst = 4u * (uint32_t)d + D4 * (uint32_t)(fs - R);

    // step j of a block at front f; CLAMP: prefetch positions may pass the row end (tail blocks)
    auto step = [&](int j, int f, uint32_t &sld, bool clamp) {
        const int slot = j % PF;
        // front: the chain of this lane starts at max(t0 - M, d) >= fs
        const float cv = cr[slot];
        P += f >= d ? (double)cv : 0.0;
        sP[j * 64 + lane] = P;
        const uint32_t so = clamp ? D4 * (uint32_t)min(f + PF, W - 1) : sld;
        cr[slot] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rc, dl4, (int)so, CBCA_NT & 1 ? 2 : 0));
        sld = opq_s(sld + D4);
        // trailing output t = f - R: left-image arm (uniform) and the right-image arm chain
        const int t = f - R;
        const uint32_t a = ruint(Ab, j);
        const uint32_t nb = ruint(Bb, j);
        X = (uint32_t)__builtin_amdgcn_update_dpp((int)nb, (int)X, 0x138, 0xF, 0xF, false);   // wave_shr:1, lane 0 <- nb
        const int hl = min(a & 255u, X & 255u), hr = min((a >> 8) & 255u, (X >> 8) & 255u);
        const uint32_t ib = ring_slot<RS>(j - R + hr), ia = ring_slot<RS>(j - R - hl - 1);
        const double pb = sP[ib * 64 + lane], pa = sP[ia * 64 + lane];
        const float out = (float)(pb - pa);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, out), rd, t >= th ? vst : CB_OOB, 0,
                                              CBCA_NT & 2 ? 2 : 0);
        vst = opq_v(vst + D4);
    };
    int fb = fs;
    // main blocks: every front and prefetch position inside the row
    for (; fb + RS - 1 <= fe && fb + RS - 1 + PF <= W - 1; fb += RS) {
        arms_blk(fb + RS - R, An, Bn);
        uint32_t sld = D4 * (uint32_t)(fb + PF);
#pragma unroll
        for (int j = 0; j < RS; j++) step(j, fb + j, sld, false);
        Ab = An;
        Bb = Bn;
    }
    for (; fb <= fe; fb += RS) {
        arms_blk(fb + RS - R, An, Bn);
        uint32_t sld = 0;
#pragma unroll
        for (int j = 0; j < RS; j++)
            if (fb + j <= fe) step(j, fb + j, sld, true);
        Ab = An;
        Bb = Bn;
    }
}

template <int R>
__global__ __launch_bounds__(64, 3) void cbca_h_kernel(const CbcaArgs A)
{
    __shared__ double sP[(2 * R + 2) * 64];
    const int64_t i0 = (int64_t)blockIdx.x * A.per, i1 = min(i0 + A.per, A.nitems);
    for (int64_t it = i0; it < i1; it++) {
        const int k = (int)(it % A.nseg);
        const int64_t r = it / A.nseg;
        cbca_h_item<R>(A, (int)(r / A.ndc), (int)(r % A.ndc), k, sP);
    }
}

// ---------------------------------------------------------------------------------------------
// Vertical pass: item = (chunk c, column x >= 64c, segment k), k fastest; only columns with at
// least one valid lane (x >= d0) are items.
// ---------------------------------------------------------------------------------------------
template <int R>
__device__ __forceinline__ void cbca_v_item(const CbcaArgs &A, int x, int c, int k, double *__restrict__ sP,
                                            uint16_t *__restrict__ sN)
{
    constexpr int RS = 2 * R + 2, PF = RS, U = R + 1, NQ = RS / 4;
    static_assert(RS % 4 == 0 && RS % U == 0, "ring sizes");
    const int lane = threadIdx.x;
    const int H = A.H, W = A.W, D = A.D, M = A.M, Hp = A.Hp;
    const int d0 = 64 * c, d = d0 + lane;
    const int t0 = k * SDE_CBCA_SEG, t1 = min(t0 + SDE_CBCA_SEG, H);
    const int fc = max(t0 - M, 0);               // chain base (every valid lane)
    const int fs = fc & ~3;                      // walk start: 16-B aligned dwordx4 of four rows
    const int fe = t1 - 1 + R;
    const bool lane_ok = d < D && d <= x;
    const uint32_t dl4 = 4u * (uint32_t)min(d, D - 1);
    const uint32_t rowv = 4u * (uint32_t)W * (uint32_t)D;       // one row of the volume
    // descriptors over the column, rebased on row fbase (loads) / fb - R (stores) every block, their
    // ranges covering the rows a block touches (< 2^31 bytes: the shape check)
    const uint32_t win = (uint32_t)(RS + PF + R + 1) * rowv;
    const __amdgpu_buffer_rsrc_t ra = cb_rsrc(A.alT + (size_t)x * Hp, 4u * (uint32_t)Hp);
    const __amdgpu_buffer_rsrc_t rb = cb_rsrc(A.arT, 4u * (uint32_t)W * (uint32_t)Hp);
    const uint32_t bcol = lane_ok ? 4u * (uint32_t)(x - d) * (uint32_t)Hp : CB_OOB;

    float cr[PF];
    u32x4 Bq[NQ];                // right-image arms of rows fb + 4m .. +3 (per lane); Bq[m] is
                                 // reloaded with the next block's rows once its last row is used
    uint32_t Ab, An;             // left-image arm of row fb + lane (lanes < RS)
    uint32_t sup[U];             // (vu | vd << 16) of the last U front positions
    auto arm_q = [&](int row) {  // rows row .. row + 3 of the right image at x - d
        const uint32_t off = bcol == CB_OOB ? CB_OOB : bcol + 4u * (uint32_t)row;
        return __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, 0);
    };
    {
        const __amdgpu_buffer_rsrc_t rc0 = cb_rsrc(A.src + ((size_t)fs * W + x) * D, win);
#pragma unroll
        for (int j = 0; j < PF; j++)
            cr[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                  rc0, dl4, (int)(rowv * (uint32_t)(min(fs + j, H - 1) - fs)), CBCA_NT & 1 ? 2 : 0));
    }
    Ab = __builtin_amdgcn_raw_buffer_load_b32(ra, 4u * (uint32_t)(fs + lane), 0, 0);
#pragma unroll
    for (int m = 0; m < NQ; m++) Bq[m] = arm_q(fs + 4 * m);
#pragma unroll
    for (int j = 0; j < U; j++) sup[j] = 0u;
    double P = 0.0;
    uint32_t N = 0;
    sP[(RS - 1) * 64 + lane] = 0.0;               // Q(fs - 1) = 0, N(fs - 1) = 0
    sN[(RS - 1) * 64 + lane] = 0;

    // step j of a block at front f; loads address rows relative to fbase, stores relative to fb - R
    auto step = [&](int j, int f, int fbase, __amdgpu_buffer_rsrc_t rc, __amdgpu_buffer_rsrc_t rd, uint32_t &sld,
                    uint32_t &sst, bool clamp) {
        const int slot = j % PF;
        // front f: chain (rows >= fc), count contribution and vertical support
        const uint32_t a = ruint(Ab, j);
        const uint32_t bw = Bq[j / 4][j % 4];
        const uint32_t a02 = a & 0x00FF00FFu, a13 = (a >> 8) & 0x00FF00FFu;
        const uint32_t b02 = bw & 0x00FF00FFu, b13 = (bw >> 8) & 0x00FF00FFu;
        // per 16-bit half: (min l, min u) and (min r, min d)
        const uint32_t m02 = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a02),
                                                                                    __builtin_bit_cast(u16x2, b02)));
        const uint32_t m13 = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a13),
                                                                                    __builtin_bit_cast(u16x2, b13)));
        const bool on = f >= fc;
        P += on ? (double)cr[slot] : 0.0;
        N += on ? ((m02 + m13) & 0xFFFFu) + 1u : 0u;
        sP[j * 64 + lane] = P;
        sN[j * 64 + lane] = (uint16_t)N;
        sup[j % U] = (m02 >> 16) | (m13 & 0xFFFF0000u);
        if (j % 4 == 3) Bq[j / 4] = arm_q(f + RS - 3);      // the next block's rows f + RS - 3 ..
        const uint32_t so = clamp ? rowv * (uint32_t)(min(f + PF, H - 1) - fbase) : sld;
        cr[slot] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rc, dl4, (int)so, CBCA_NT & 1 ? 2 : 0));
        sld = opq_s(sld + rowv);
        // trailing output t = f - R, support from the ring slot of position t
        const int t = f - R;
        const uint32_t sy = sup[(j + 1) % U];
        const int vu = sy & 0xFFFF, vd = sy >> 16;
        const uint32_t ib = ring_slot<RS>(j - R + vd), ia = ring_slot<RS>(j - R - vu - 1);
        const double num = sP[ib * 64 + lane] - sP[ia * 64 + lane];
        const uint32_t cnt = (uint16_t)(sN[ib * 64 + lane] - sN[ia * 64 + lane]);
        const float out = (float)(num * cb_recip(cnt));
        const uint32_t vo = (lane_ok && t >= t0) ? 4u * (uint32_t)d : CB_OOB;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, out), rd, vo, (int)sst, CBCA_NT & 2 ? 2 : 0);
        sst = opq_s(sst + rowv);
    };
    int fb = fs;
    for (; fb + RS - 1 <= fe && fb + RS - 1 + PF <= H - 1; fb += RS) {
        An = __builtin_amdgcn_raw_buffer_load_b32(ra, 4u * (uint32_t)(fb + RS + lane), 0, 0);
        // loads for positions fb + PF .. go against a descriptor rebased on row fb
        const __amdgpu_buffer_rsrc_t rc = cb_rsrc(A.src + ((size_t)fb * W + x) * D, win);
        const __amdgpu_buffer_rsrc_t rd = cb_rsrc(A.dst + ((size_t)(fb - R) * W + x) * D, win);
        uint32_t sld = rowv * (uint32_t)PF, sst = 0;
#pragma unroll
        for (int j = 0; j < RS; j++) step(j, fb + j, fb, rc, rd, sld, sst, false);
        Ab = An;
    }
    for (; fb <= fe; fb += RS) {
        An = __builtin_amdgcn_raw_buffer_load_b32(ra, 4u * (uint32_t)(fb + RS + lane), 0, 0);
        const int fbase = min(fb, H - 1);       // a tail block may start past the last row
        const __amdgpu_buffer_rsrc_t rc = cb_rsrc(A.src + ((size_t)fbase * W + x) * D, win);
        const __amdgpu_buffer_rsrc_t rd = cb_rsrc(A.dst + ((size_t)(fb - R) * W + x) * D, win);
        uint32_t sld = 0, sst = 0;
#pragma unroll
        for (int j = 0; j < RS; j++)
            if (fb + j <= fe) step(j, fb + j, fbase, rc, rd, sld, sst, true);
        Ab = An;
    }
}

template <int R>
__global__ __launch_bounds__(64, 3) void cbca_v_kernel(const CbcaArgs A)
{
    __shared__ double sP[(2 * R + 2) * 64];
    __shared__ uint16_t sN[(2 * R + 2) * 64];
    const int64_t i0 = (int64_t)blockIdx.x * A.per, i1 = min(i0 + A.per, A.nitems);
    for (int64_t it = i0; it < i1; it++) {
        int c = 0;
        while (c + 1 < A.ndc && it >= A.chunk_first[c + 1]) c++;
        const int64_t r = it - A.chunk_first[c];
        const int k = (int)(r % A.nseg);
        cbca_v_item<R>(A, 64 * c + (int)(r / A.nseg), c, k, sP, sN);
    }
}

// ---------------------------------------------------------------------------------------------
// Per-disparity rotation of the rows: out(y, x, d) = in(y, (x + s*d) mod W, d).  s = +1 with
// VALID_ONLY: the shear of an aggregated left volume into the right one's valid voxels (x + d <
// W; the others untouched); s = -1 / +1 over every voxel: a right-referenced volume into left
// coordinates and back (its invalid voxels ride on the left-coordinate invalid ones).
// Tile = (row, 64-disparity chunk, 64 output pixels); its 127 source pixels are staged in LDS
// (stride 64 floats: the diagonal reads hit 64 distinct banks), tiles sharing source pixels
// sit 8 blocks apart (one XCD under round-robin dispatch: L2 reuse, speed only).
// ---------------------------------------------------------------------------------------------
template <bool VEC4>
__global__ __launch_bounds__(256) void cbca_rotate_kernel(const float *__restrict__ in, float *__restrict__ out, int H,
                                                          int W, int D, int s, int valid_only, int64_t ntiles,
                                                          int64_t per_xcd)
{
    __shared__ float buf[127 * 64];
    const int64_t b = blockIdx.x;
    const int64_t tile = (b % 8) * per_xcd + b / 8;
    if (tile >= ntiles) return;
    const int nxs = (W + 63) / 64, ndc = (D + 63) / 64;
    const int xs = (int)(tile % nxs);
    const int64_t rem = tile / nxs;
    const int c = (int)(rem % ndc), y = (int)(rem / ndc);
    const int x0 = 64 * xs, d0 = 64 * c;
    const int tid = threadIdx.x;
    const uint32_t rowbytes = 4u * (uint32_t)W * (uint32_t)D;
    const __amdgpu_buffer_rsrc_t ri = cb_rsrc(in + (size_t)y * W * D, rowbytes);
    const __amdgpu_buffer_rsrc_t ro = cb_rsrc(out + (size_t)y * W * D, rowbytes);
    // source row r of the tile = pixel (base + r) mod W
    const int64_t base = s > 0 ? (int64_t)x0 + d0 : (int64_t)x0 - d0 - 63;
    auto srcpix = [&](int r) { return (int)((((base + r) % W) + W) % W); };
    if (VEC4) {
        // 16 lanes per 256-B run: thread t loads chunk t % 16 of rows t / 16 + 16 m
#pragma unroll
        for (int m = 0; m < 8; m++) {
            const int r = tid / 16 + 16 * m;
            if (r < 127) {
                const int col = 4 * (tid % 16);
                const uint32_t off = d0 + col < D ? 4u * ((uint32_t)srcpix(r) * D + d0 + col) : CB_OOB;
                const float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ri, off, 0, 0));
                *(float4 *)&buf[r * 64 + col] = v;
            }
        }
    } else {
#pragma unroll 4
        for (int m = 0; m < 32; m++) {
            const int r = tid / 64 + 4 * m;
            if (r < 127) {
                const int col = tid % 64;
                const uint32_t off = d0 + col < D ? 4u * ((uint32_t)srcpix(r) * D + d0 + col) : CB_OOB;
                buf[r * 64 + col] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ri, off, 0, 0));
            }
        }
    }
    __syncthreads();
    const int i = tid % 64, wv = tid / 64;
    const int d = d0 + i;
#pragma unroll 4
    for (int p = wv; p < 64; p += 4) {
        const int x = x0 + p;
        const int r = s > 0 ? p + i : p - i + 63;
        const bool ok = x < W && d < D && (!valid_only || x + d < W);
        const uint32_t off = ok ? 4u * ((uint32_t)x * D + d) : CB_OOB;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, buf[r * 64 + i]), ro, off, 0, 0);
    }
}

__global__ void cbca_recip_kernel(double *out, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = cb_recip((uint32_t)(i + 1));
}

// ---------------------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------------------
static inline int cb_hp(int H) { return (H + 3) & ~3; }

static size_t cbca_ws_bytes(int H, int W) { return 2 * sizeof(uint32_t) * (size_t)cb_hp(H) * (size_t)W; }

// Resident one-wave workgroups of a pass kernel (occupancy x CUs), per device and kernel.
template <typename K>
static int cb_resident(K kernel)
{
    int dev = 0, cus = 256, per = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, 64, 0) != hipSuccess || per <= 0) per = 8;
    return per * cus;
}

// Balanced static schedule: the fewest items per wave that fit the resident waves, then only as
// many waves as that needs (every wave gets the same count, so none idles while others finish).
static void cb_schedule(CbcaArgs &A, int resident, int &grid)
{
    const int64_t per = (A.nitems + resident - 1) / resident;
    A.per = (int)(per > 0 ? per : 1);
    grid = (int)((A.nitems + A.per - 1) / A.per);
}

// One left-coordinate volume: iters x (horizontal src -> tmp, vertical tmp -> src), in place.
template <int R>
static void cbca_left_iters(float *cv, float *tmp, const uint32_t *al, const uint32_t *ar, const uint32_t *alT,
                            const uint32_t *arT, int H, int W, int D, int L1, int iters, hipStream_t st)
{
    CbcaArgs h{};
    h.al = al, h.ar = ar, h.alT = alT, h.arT = arT;
    h.H = H, h.W = W, h.D = D, h.M = L1 - 1, h.Hp = cb_hp(H);
    h.ndc = (D + 63) / 64;
    CbcaArgs v = h;
    h.nseg = (W + SDE_CBCA_SEG - 1) / SDE_CBCA_SEG;
    h.nitems = (int64_t)H * h.ndc * h.nseg;
    v.nseg = (H + SDE_CBCA_SEG - 1) / SDE_CBCA_SEG;
    int64_t n = 0;
    for (int c = 0; c < v.ndc; c++) {
        v.chunk_first[c] = n;
        n += (int64_t)max(W - 64 * c, 0) * v.nseg;
    }
    v.chunk_first[v.ndc] = n;
    v.nitems = n;
    static std::atomic<int> res_h{0}, res_v{0};
    if (!res_h.load()) res_h = cb_resident(cbca_h_kernel<R>);
    if (!res_v.load()) res_v = cb_resident(cbca_v_kernel<R>);
    int gh = 0, gv = 0;
    cb_schedule(h, res_h.load(), gh);
    cb_schedule(v, res_v.load(), gv);
    h.src = cv, h.dst = tmp;
    v.src = tmp, v.dst = cv;
    for (int it = 0; it < iters; it++) {
        if (h.nitems > 0) cbca_h_kernel<R><<<gh, 64, 0, st>>>(h);
        if (v.nitems > 0) cbca_v_kernel<R><<<gv, 64, 0, st>>>(v);
    }
}

static void cbca_rotate(const float *in, float *out, int H, int W, int D, int s, bool valid_only, hipStream_t st)
{
    const int64_t ntiles = (int64_t)H * ((D + 63) / 64) * ((W + 63) / 64);
    const int64_t per = (ntiles + 7) / 8;
    const int64_t grid = 8 * per;
    if (D % 4 == 0)
        cbca_rotate_kernel<true><<<(unsigned)grid, 256, 0, st>>>(in, out, H, W, D, s, valid_only ? 1 : 0, ntiles, per);
    else
        cbca_rotate_kernel<false><<<(unsigned)grid, 256, 0, st>>>(in, out, H, W, D, s, valid_only ? 1 : 0, ntiles, per);
}

// Shapes the 32-bit offsets cover (refused with SDE_ERR_ARG otherwise): a row of the volume and a
// vertical-pass block window ((RS + PF + R + 1) rows, RS = PF = 2R + 2) below 2^31 bytes, the
// arms (and their column-major copy) below 2^31 bytes, at most 8 disparity chunks (D <= 512).
static int cbca_r(int L1) { return L1 <= 14 ? 13 : L1 <= 16 ? 15 : 31; }
static bool cbca_shape_ok(int H, int W, int D, int L1)
{
    if (H <= 0 || W <= 0 || D <= 0 || D > 512 || L1 < 1 || L1 > SDE_CBCA_MAX_L1) return false;
    const int R = cbca_r(L1);
    const int64_t row = 4 * (int64_t)W * D;
    return (int64_t)(5 * R + 5) * row < ((int64_t)1 << 31) && 4 * (int64_t)cb_hp(H) * W < ((int64_t)1 << 31) &&
           (int64_t)H * ((D + 63) / 64) * ((W + 63) / 64) < ((int64_t)1 << 31) - 8;
}

static int cbca_left(float *cv, float *tmp, const uint32_t *al, const uint32_t *ar, int H, int W, int D, int L1,
                     int iters, void *ws, hipStream_t st)
{
    if (iters == 0) return SDE_OK;
    const int Hp = cb_hp(H);
    uint32_t *alT = (uint32_t *)ws, *arT = alT + (size_t)Hp * W;
    const dim3 tg((W + 31) / 32, (Hp + 31) / 32);
    cbca_transpose_kernel<<<tg, 256, 0, st>>>(al, alT, H, W, Hp);
    cbca_transpose_kernel<<<tg, 256, 0, st>>>(ar, arT, H, W, Hp);
    switch (cbca_r(L1)) {
    case 13: cbca_left_iters<13>(cv, tmp, al, ar, alT, arT, H, W, D, L1, iters, st); break;
    case 15: cbca_left_iters<15>(cv, tmp, al, ar, alT, arT, H, W, D, L1, iters, st); break;
    default: cbca_left_iters<31>(cv, tmp, al, ar, alT, arT, H, W, D, L1, iters, st); break;
    }
    return launch_status();
}

// A right-referenced volume: rotated into left coordinates in tmp, aggregated there with cv as the
// scratch, rotated back.  al / ar: the left / right image's arms.
static int cbca_right(float *cv, float *tmp, const uint32_t *al, const uint32_t *ar, int H, int W, int D, int L1,
                      int iters, void *ws, hipStream_t st)
{
    if (iters == 0) return SDE_OK;
    cbca_rotate(cv, tmp, H, W, D, -1, false, st);
    const int s = cbca_left(tmp, cv, al, ar, H, W, D, L1, iters, ws, st);
    if (s != SDE_OK) return s;
    cbca_rotate(tmp, cv, H, W, D, +1, false, st);
    return launch_status();
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

SDE_EXPORT size_t sde_cbca_workspace_bytes(int H, int W)
{
    if (H <= 0 || W <= 0) return 0;
    return cbca_ws_bytes(H, W);
}

SDE_EXPORT int sde_cbca(float *cv, float *tmp, const uint32_t *arms_ref, const uint32_t *arms_other, int H, int W,
                        int D, int side, int L1, int iters, void *ws, size_t ws_bytes, void *stream)
{
    if (!cv || !tmp || !arms_ref || !arms_other || iters < 0 || (side != SDE_SIDE_LEFT && side != SDE_SIDE_RIGHT) ||
        cv == tmp || !cbca_shape_ok(H, W, D, L1) || (iters > 0 && (!ws || ws_bytes < cbca_ws_bytes(H, W))))
        return SDE_ERR_ARG;
    if (side == SDE_SIDE_LEFT)
        return cbca_left(cv, tmp, arms_ref, arms_other, H, W, D, L1, iters, ws, as_stream(stream));
    return cbca_right(cv, tmp, arms_other, arms_ref, H, W, D, L1, iters, ws, as_stream(stream));
}

SDE_EXPORT int sde_cbca_pair(float *cv_l, float *tmp_l, float *cv_r, float *tmp_r, const uint32_t *arms_l,
                             const uint32_t *arms_r, int H, int W, int D, int L1, int iters, void *ws, size_t ws_bytes,
                             void *stream)
{
    if (!cv_l || !tmp_l || !cv_r || !tmp_r || !arms_l || !arms_r || iters < 0 || !cbca_shape_ok(H, W, D, L1) ||
        (iters > 0 && (!ws || ws_bytes < cbca_ws_bytes(H, W))))
        return SDE_ERR_ARG;
    const float *b[4] = {cv_l, tmp_l, cv_r, tmp_r};
    for (int i = 0; i < 4; i++)
        for (int j = i + 1; j < 4; j++)
            if (b[i] == b[j]) return SDE_ERR_ARG;
    int s = cbca_left(cv_l, tmp_l, arms_l, arms_r, H, W, D, L1, iters, ws, as_stream(stream));
    if (s != SDE_OK) return s;
    return cbca_right(cv_r, tmp_r, arms_l, arms_r, H, W, D, L1, iters, ws, as_stream(stream));
}

SDE_EXPORT int sde_cbca_lr(float *cv_l, float *cv_r, float *tmp, const uint32_t *arms_l, const uint32_t *arms_r,
                           int H, int W, int D, int L1, int iters, void *ws, size_t ws_bytes, void *stream)
{
    if (!cv_l || !cv_r || !tmp || !arms_l || !arms_r || iters < 0 || cv_l == cv_r || cv_l == tmp || cv_r == tmp ||
        !cbca_shape_ok(H, W, D, L1) || (iters > 0 && (!ws || ws_bytes < cbca_ws_bytes(H, W))))
        return SDE_ERR_ARG;
    if (iters == 0) return SDE_OK;
    const int s = cbca_left(cv_l, tmp, arms_l, arms_r, H, W, D, L1, iters, ws, as_stream(stream));
    if (s != SDE_OK) return s;
    cbca_rotate(cv_l, cv_r, H, W, D, +1, true, as_stream(stream));
    return launch_status();
}

SDE_EXPORT int sde_cbca_reciprocals(double *out, int n, void *stream)
{
    if (!out || n <= 0) return SDE_ERR_ARG;
    cbca_recip_kernel<<<cdiv(n, 256), 256, 0, as_stream(stream)>>>(out, n);
    return launch_status();
}
