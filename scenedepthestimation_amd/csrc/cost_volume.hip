// cost_volume.hip -- disparity cost volume, fused cost+WTA and WTA kernels (gfx950).
//
// Replaces (WHDY/SceneDepthEstimation):
//   compute_cost_volume        process_functional.py:48-73   (CPU path, [D,H,W], -0.0 fill)
//   WTA1 / WTA                 process_functional.py:96-113 / 76-93
//   compute_cost_volume_kernel process_functional.py:120-131 ([H,W,D] L and R, 1.0 fill)
//   WTA_and_SupixelRefinement_kernel process_functional.py:800-837
//
// Numerics: every valid voxel is the CPU path's value bit for bit,
//   cost(x,d) = -(0.0f + pairwise8_c(fl[y][x][c] * fr[y][x-d][c]))
// -- products rounded to f32, 8 running f32 accumulators over channel blocks of
// 8, then ((a0+a1)+(a2+a3))+((a4+a5)+(a6+a7)) (NumPy's pairwise_sum for C=64).
// The library is compiled with -ffp-contract=off so no product is fused.
//
// Mapping (C = 64 fast path): a workgroup is 4 waves on one image row and 64
// consecutive "own" pixels (one per lane, its 64-float feature vector held in
// VGPRs).  The 127 "other" feature rows a 64-disparity chunk touches are staged
// in LDS (272-B padded rows: the 16 lanes of a ds_read_b128 group read 16
// consecutive rows -> 16 distinct bank slots).  Wave w sweeps disparities
// [16w, 16w+16) of each chunk; the fused WTA merges the 4 per-wave first-minima
// by (value, index) at the end, which equals the sequential scan.  The GPU
// path's L and R volumes come from one row sweep (cvlr3_kernel, below).
#include "sde_common.h"
#include "cv_cert.h"

#include <algorithm>

namespace sde {

constexpr int CV_TX = 64;                    // own pixels per workgroup (= lanes)
constexpr int CV_WAVES = 4;                  // waves per workgroup
constexpr int CV_DC = 64;                    // disparities per LDS chunk
constexpr int CV_DW = CV_DC / CV_WAVES;      // disparities per wave per chunk
constexpr int CV_ROWS = CV_TX + CV_DC - 1;   // other-side rows per chunk

enum { OUT_WTA = 0, OUT_DHW = 1, OUT_HWD = 2 };

// LDS image of the "other" rows: 64 floats + one 16-B pad per row (272 B), so the lanes of a
// ds_read_b128 group, which read the same chunk of consecutive rows, start 4 banks apart
// (conflict-free) and every chunk address is the row base plus an immediate offset.
constexpr int CV_RSTRIDE = 17;     // float4 per LDS row

// Exact -(0 + pairwise8) of own[64] (registers) and one padded LDS row.
__device__ __forceinline__ float dot64_exact(const float (&own)[64], const float4 *__restrict__ win, int lr)
{
    float acc[8];
    const float4 *row = win + lr * CV_RSTRIDE;
#pragma unroll
    for (int m = 0; m < 8; m++) {
        const float4 a = row[2 * m];
        const float4 b = row[2 * m + 1];
        const float p0 = own[8 * m + 0] * a.x, p1 = own[8 * m + 1] * a.y;
        const float p2 = own[8 * m + 2] * a.z, p3 = own[8 * m + 3] * a.w;
        const float p4 = own[8 * m + 4] * b.x, p5 = own[8 * m + 5] * b.y;
        const float p6 = own[8 * m + 6] * b.z, p7 = own[8 * m + 7] * b.w;
        if (m == 0) {
            acc[0] = p0; acc[1] = p1; acc[2] = p2; acc[3] = p3;
            acc[4] = p4; acc[5] = p5; acc[6] = p6; acc[7] = p7;
        } else {
            acc[0] += p0; acc[1] += p1; acc[2] += p2; acc[3] += p3;
            acc[4] += p4; acc[5] += p5; acc[6] += p6; acc[7] += p7;
        }
    }
    const float res = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    return -(0.0f + res);
}

// SIDE_LEFT : own = fl at x,  other = fr at x - d   (L[y][x][d])
// SIDE_RIGHT: own = fr at x', other = fl at x' + d  (R[y][x'][d] = cost(x'+d, d))
template <int SIDE, int OUT>
__global__ __launch_bounds__(256) void cv64_kernel(const float *__restrict__ own_feat,
                                                   const float *__restrict__ other_feat, int H, int W,
                                                   int d0, int d1, int Dvol, float invalid,
                                                   float *__restrict__ out, float *__restrict__ out_min,
                                                   int32_t *__restrict__ out_arg, float *__restrict__ out_disp)
{
    constexpr bool TILE = OUT == OUT_HWD;
    __shared__ float4 win[CV_ROWS * CV_RSTRIDE];
    __shared__ float otile[TILE ? CV_TX * (CV_DC + 1) : 1];

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int y = blockIdx.y;
    const int q0 = blockIdx.x * CV_TX;
    const int q = q0 + lane;
    const bool qok = q < W;

    float own[64];
    {
        const float4 *src = reinterpret_cast<const float4 *>(own_feat + ((size_t)y * W + (qok ? q : 0)) * 64);
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const float4 v = src[k];
            own[4 * k + 0] = v.x; own[4 * k + 1] = v.y; own[4 * k + 2] = v.z; own[4 * k + 3] = v.w;
        }
    }
    const float4 *other4 = reinterpret_cast<const float4 *>(other_feat) + (size_t)y * W * 16;

    float best = __builtin_inff();
    int arg = -1;

    for (int dc = d0; dc < d1; dc += CV_DC) {
        const int dce = min(dc + CV_DC, d1);
        const int rbase = (SIDE == SDE_SIDE_LEFT) ? q0 - (dc + CV_DC - 1) : q0 + dc;
        __syncthreads();   // previous chunk's LDS reads (win and otile) are complete
        for (int idx = threadIdx.x; idx < CV_ROWS * 16; idx += 256) {
            const int lr = idx >> 4, k = idx & 15, g = rbase + lr;
            if (g >= 0 && g < W) win[lr * CV_RSTRIDE + k] = other4[(size_t)g * 16 + k];
        }
        __syncthreads();
        const int ds = dc + wave * CV_DW;
        const int de = min(ds + CV_DW, dce);
#pragma unroll 2
        for (int d = ds; d < de; d++) {
            const int o = (SIDE == SDE_SIDE_LEFT) ? q - d : q + d;
            const bool valid = (SIDE == SDE_SIDE_LEFT) ? (o >= 0) : (o < W);
            float cost = invalid;
            if (qok && valid) cost = dot64_exact(own, win, o - rbase);
            if (OUT == OUT_WTA) {
                if (cost < best) { best = cost; arg = d; }
            } else if (OUT == OUT_DHW) {
                if (qok) out[((size_t)d * H + y) * W + q] = cost;
            } else {
                otile[lane * (CV_DC + 1) + (d - dc)] = cost;
            }
        }
        if (TILE) {
            __syncthreads();
            const int nd = dce - dc;
            for (int i = wave; i < CV_TX; i += CV_WAVES) {
                if (q0 + i < W && lane < nd)
                    out[((size_t)y * W + q0 + i) * Dvol + dc + lane] = otile[i * (CV_DC + 1) + lane];
            }
        }
    }

    if (OUT == OUT_WTA) {
        __shared__ float sm[CV_WAVES][CV_TX];
        __shared__ int sa[CV_WAVES][CV_TX];
        sm[wave][lane] = best;
        sa[wave][lane] = arg;
        __syncthreads();
        if (wave == 0 && qok) {
#pragma unroll
            for (int w = 1; w < CV_WAVES; w++) argmin_merge(best, arg, sm[w][lane], sa[w][lane]);
            const size_t p = (size_t)y * W + q;
            if (out_min) out_min[p] = best;
            if (out_arg) out_arg[p] = arg;
            if (out_disp) out_disp[p] = (float)arg;
        }
    }
}

// ---------------------------------------------------------------------------
// LDS-DMA helpers of the L/R volume sweep (cvlr3_kernel below).  Rounds 1-2 ran the sweep as
// cvlr_row_kernel (register-staged, 2 workgroups per CU) and cvlr_dma_kernel (one 512-thread
// workgroup per CU, LDS-DMA one dot loop ahead); both measured slower than cvlr3_kernel and were
// removed in round 4 (DESIGN.md sec. 3.1 keeps their measurements).  The padded 272-B rows, the
// 32-row DMA units (8.5 wave-instructions of 1 KiB; lane s loads chunk s % 17 of row s / 17, chunk
// 16 the pad) and the raw barriers below are theirs.
// ---------------------------------------------------------------------------
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int CD_RB = 272;                                // bytes per padded LDS row (17 chunks of 16 B)

__device__ __forceinline__ uint32_t cd_lds(const void *p)
{
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

typedef unsigned cd_u32x4 __attribute__((ext_vector_type(4)));
// raw buffer descriptor of `bytes` bytes at base (SGPRs): loads past the records return zeros
__device__ __forceinline__ cd_u32x4 cd_desc(const void *base, uint32_t bytes)
{
    const uintptr_t b = (uintptr_t)base;
    cd_u32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((uint32_t)b);
    r.y = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) & 0xffffu;
    r.z = __builtin_amdgcn_readfirstlane(bytes);
    r.w = 0x00020000u;
    return r;
}

// one LDS-DMA wave-instruction: 16 B per lane from byte offset voff of the buffer to lds_dst + 16 lane
__device__ __forceinline__ void cd_dma16(cd_u32x4 rs, uint32_t voff, uint32_t lds_dst)
{
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(rs), "s"(lds_dst)
                 : "memory");
}

// rows gbase + 2i (i = 0..31) of a feature row (the buffer) -> 32 padded LDS rows at lds_unit.  Lane
// s of the 8.5 instructions loads byte 256 (gbase + 2i) + 16 (s - 17 i), i = s / 17 (chunk 16, the
// pad, takes the next row's chunk 0); rows outside [0, W) -- negative ones wrap to huge offsets --
// are past the records and load zeros, never used.
__device__ __forceinline__ void cd_unit(cd_u32x4 rs, int gbase, uint32_t lds_unit, int lane)
{
    // (an opaque lane copy: the offsets are recomputed per issue, a few VALU, instead of being
    // hoisted out of the strip loop into registers the dot loop needs)
    asm volatile("" : "+v"(lane));
    const uint32_t rowoff = (uint32_t)gbase * 256u;
    const uint32_t lb = __builtin_amdgcn_readfirstlane(lds_unit);
#pragma unroll
    for (int n = 0; n < 9; n++) {
        const int sl = 64 * n + lane;
        const int i = (sl * 3856) >> 16;                // sl / 17 for sl < 544
        if (n < 8 || lane < 32) cd_dma16(rs, rowoff + 16u * sl + 240u * i, lb + 1024u * n);
    }
}

constexpr uint32_t CD_OOB = 0x80000000u;                 // past any row's records
__device__ __forceinline__ __amdgpu_buffer_rsrc_t cd_rsrc(const void *base, uint32_t bytes)
{
    const uintptr_t b = (uintptr_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((uintptr_t)hi << 32) | lo), 0,
                                             (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

__device__ __forceinline__ void cd_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ---------------------------------------------------------------------------
// L and R volumes in one row sweep, two workgroups per CU (C = 64, [H,W,D]) -- the default.
//
// Round 2's cvlr_dma_kernel held the whole CU (155 KB of LDS, 8 waves in lock-step barrier phases):
// its dot loops stopped at every strip boundary while the CU waited (PMC: waves parked 37 % of their
// cycles, VALU busy ~45 %).  Here a 256-thread workgroup (4 waves, one per SIMD) needs 69 KB of
// LDS, so two independent workgroups share each CU and one's barrier phases and exposed loads
// overlap the other's dots.  Workgroup = (row y, 64-disparity chunk dc), 64-pixel strips; the
// exact NumPy-order arithmetic and the two-pixel blocking are round 2's, the mapping is
// per pixel group: wave w, lane (p, h) = (lane & 7, lane >> 3): own pixels u = q0 + 16w + 2p,
// u + 1, disparities e = dc + 8h .. +7; rows o = u+1-e-j, j = 0..8, serve both pixels (the 16
// lanes of a ds_read_b128 group read 12 distinct padded rows in distinct bank slots).
//   * other-side rows: two parity sub-rings of 64 padded rows (272 B) = the strip's two 64-row
//     blocks [q0-dc-64, q0-dc+64); after the strip's dots the older block's slots take the next
//     strip's block by LDS-DMA (that latency is the one the co-resident workgroup covers);
//   * own pixels: LDS-DMA one strip ahead into two parity buffers of 32 padded pixels (coalesced
//     1 KiB pieces; as buffer loads straight into VGPRs the 8-fold re-reads of every line through
//     the texture path cost more than the dots' LDS traffic), copied to VGPRs at the strip start;
//   * every cost lands in a 64 x 65 LDS tile T[d][pixel] of the strip; at the next strip's start
//     each wave reads its 16 L rows (full 256-B runs L[y][x][dc..dc+63]) and the 16 R rows the
//     strip completes (R[y][xr][dc..] = cost(xr + d, d): an R row of the chunk spans at most two
//     strips) into registers; the part an R row got from the previous strip waits in a register
//     carry (16 VGPRs, lane = d; row xr belongs to wave (xr + 3) & 3 in every strip), so every
//     store is a whole 256-B run -- no partial lines; the 32 stores go out in the first four dot
//     rows and drain while the strip computes;
//   * per strip: wait for the DMA, barrier, own pixels -> VGPRs and tile -> registers, barrier,
//     the next own pixels' DMA, dots, barrier, the next rows' DMA.
// Voxels with x >= W are R's invalid fill; strips past the row end compute nothing.
// ---------------------------------------------------------------------------
// cvlr3_kernel's volume stores are nontemporal (cache-policy bits 2; round 3: 0.769 -> 0.756 ms, 1: 0.762)
constexpr int C3_AUX = 2;
constexpr int C3_NX = 64;                                  // own pixels per strip
constexpr int C3_RING = 64;                                // rows per parity sub-ring
constexpr int C3_TS = 65;                                  // tile stride (floats per disparity)
constexpr size_t C3_RING_BYTES = (size_t)2 * C3_RING * CD_RB;           // 34,816 B
constexpr size_t C3_OWN_BYTES = (size_t)2 * 32 * CD_RB;                 // 17,408 B
constexpr size_t C3_TILE_OFF = C3_RING_BYTES + C3_OWN_BYTES + 64 * 4;   // R reads reach 63 floats before T
constexpr size_t C3_SMEM = C3_TILE_OFF + (size_t)(64 * C3_TS + 64) * 4; // ... and 62 past it: 69,376 B

// instructions [n0, n1) of cd_unit's nine (a 32-row unit split over two waves)
__device__ __forceinline__ void c3_unit(cd_u32x4 rs, int gbase, uint32_t lds_unit, int lane, int n0, int n1)
{
    asm volatile("" : "+v"(lane));
    const uint32_t rowoff = (uint32_t)gbase * 256u;
    const uint32_t lb = __builtin_amdgcn_readfirstlane(lds_unit);
#pragma unroll
    for (int n = 0; n < 9; n++) {
        if (n < n0 || n >= n1) continue;
        const int sl = 64 * n + lane;
        const int i = (sl * 3856) >> 16;                // sl / 17 for sl < 544
        if (n < 8 || lane < 32) cd_dma16(rs, rowoff + 16u * sl + 240u * i, lb + 1024u * n);
    }
}

// WR: also the right volume.  Without it (the aggregation path: sde_cbca_lr writes the right volume as the
// aggregated left one's shear) the strips end at the row end and half the stores go.
template <bool WR>
__global__ __launch_bounds__(256, 2) void cvlr3_kernel(const float *__restrict__ fl, const float *__restrict__ fr,
                                                       int H, int W, int D, int nchunks, float invalid,
                                                       float *__restrict__ outl, float *__restrict__ outr)
{
    constexpr int NST = WR ? 32 : 16;                   // emission stores per strip
    extern __shared__ __attribute__((aligned(16))) char c3_sm[];
    const char *ring = c3_sm;
    const char *own = c3_sm + C3_RING_BYTES;
    float *T = reinterpret_cast<float *>(c3_sm + C3_TILE_OFF);
    const uint32_t ring_l = cd_lds(ring), own_l = cd_lds(own);

    const int job = xcd_remap(blockIdx.x, gridDim.x);   // the chunks of a row share an XCD's L2
    const int y = job / nchunks;
    const int dc = (job - y * nchunks) * CV_DC;
    const int nd = min(CV_DC, D - dc);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int p = lane & 7, h = lane >> 3;
    const int e = dc + 8 * h;                           // this lane's first disparity
    const size_t rowvox = (size_t)y * W;
    const cd_u32x4 rs_o = cd_desc(fl + rowvox * 64, (uint32_t)W * 256u);   // own pixels' feature row
    const cd_u32x4 rs_r = cd_desc(fr + rowvox * 64, (uint32_t)W * 256u);   // other side's
    // row y of each volume (the host guarantees 4 W D < CD_OOB)
    const __amdgpu_buffer_rsrc_t rl = cd_rsrc(outl + rowvox * D, (uint32_t)W * D * 4u);
    const __amdgpu_buffer_rsrc_t rr = cd_rsrc(WR ? outr + rowvox * D : outl, (uint32_t)W * D * 4u);
    // strips: the emission after strip k completes R rows [q0-dc-63, q0-dc] (whatever nd), so
    // the last strip holds x = W-1+dc+63 (left volume only: the last strip holds x = W-1)
    const int nstrips = WR ? (W + dc + 62) / C3_NX + 1 : (W + C3_NX - 1) / C3_NX;

    // a 64-row block of other-side rows at r (a multiple of 64): parity par, instructions [n0, n1)
    auto ring_unit = [&](int r, int par, int n0, int n1) {
        int k0 = (r >> 1) % C3_RING;
        if (k0 < 0) k0 += C3_RING;                      // a multiple of 32: the unit does not wrap
        c3_unit(rs_r, r + par, ring_l + (uint32_t)(par * C3_RING + k0) * CD_RB, lane, n0, n1);
    };
    // own pixels q + par + 2i (i < 32) -> parity buffer par
    auto own_unit = [&](int q, int par, int n0, int n1) {
        c3_unit(rs_o, q + par, own_l + (uint32_t)(par * 32) * CD_RB, lane, n0, n1);
    };

    // Emission of the tile of the strip at qp (lane = disparity dc + lane): L rows x = qp + wave + 4n,
    // R rows xr = qp - dc - 63 + i, i = 4n + wave (complete after this strip: lanes lane >= 63 - i
    // from the tile, the others from the carry), and the carry of the R rows this strip starts
    // (xr + 64, lanes lane <= 62 - i, for the next strip's emission).  Reads outside the tile land
    // in the slack words and are never selected.
    float vl[16], vr[16], cr[16];
#pragma unroll
    for (int n = 0; n < 16; n++) cr[n] = invalid;
    const float *tl = T + lane * C3_TS + wave;
    const float *tr = T + lane * (C3_TS + 1) + wave - 63;
    const uint32_t voff_d = lane < nd ? 4u * lane : CD_OOB;
    auto emit_load = [&]() {
#pragma unroll
        for (int n = 0; n < 16; n++) {
            vl[n] = tl[4 * n];
            const float t = tr[4 * n];
            vr[n] = lane >= 63 - (4 * n + wave) ? t : cr[n];
            cr[n] = tr[4 * n + 64];
        }
    };
    // stores 8j .. 8j+7 of the 32 (16 L, 16 R runs), issued in the first four dot rows so they
    // drain while the strip computes.  A row outside the image stores with voffset CD_OOB: the
    // buffer range check compares the voffset with the records (4 W D < CD_OOB) and drops it, with
    // or without the soffset counted in (row offsets < 2^31: the sum cannot wrap) -- one select per
    // store, no branch.
    auto emit_store = [&](int qp, int j) {
        const int rowstep = 16 * D;                         // 4 rows of the volume, bytes
#pragma unroll
        for (int n = 8 * j; n < 8 * j + 8 && n < NST; n++) {
            if (n < 16) {
                const int x = qp + wave + 4 * n;
                const bool in = x < W;
                const uint32_t so = in ? (uint32_t)(((qp + wave) * D + dc) * 4 + n * rowstep) : 0u;
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, vl[n]), rl, in ? voff_d : CD_OOB, so,
                                                      C3_AUX);
            } else {
                const int xr = qp - dc - 63 + 4 * (n - 16) + wave;
                const bool in = (uint32_t)xr < (uint32_t)W;
                const uint32_t so = in ? (uint32_t)(((qp - dc - 63 + wave) * D + dc) * 4 + (n - 16) * rowstep) : 0u;
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, vr[n - 16]), rr, in ? voff_d : CD_OOB,
                                                      so, C3_AUX);
            }
        }
    };

    // strip 0: rows [-dc-64, 64-dc) (two blocks x two parities, one unit per wave) and own pixels
    ring_unit(-dc - 64 + 64 * (wave >> 1), wave & 1, 0, 9);
    own_unit(0, wave & 1, (wave >> 1) ? 5 : 0, (wave >> 1) ? 9 : 5);

    for (int k = 0; k < nstrips; k++) {
        const int q0 = k * C3_NX;
        const bool more = k + 1 < nstrips;
        const bool compute = q0 + 16 * wave < W;            // wave-uniform
        const int u = q0 + 16 * wave + 2 * p;
        // this strip's rows and own pixels have landed (every wave's DMA, hence the barrier); the
        // previous strip's tile is complete.  Only the own pixels are waited for here --
        // per wave the ops after them are the previous strip's 32 emission stores (none before
        // strip 2) and this strip's 4-5 ring DMA instructions, and vmcnt retires in order -- so the
        // row block's DMA latency overlaps the own copy and the tile reads; the rows are waited for
        // before the second barrier.
        if (k == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (k == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else if (WR) asm volatile("s_waitcnt vmcnt(36)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
        cd_barrier();
        f32x2 own_a[32], own_b[32];
        if (compute) {
            const f32x4 *sa = reinterpret_cast<const f32x4 *>(own + (size_t)(8 * wave + p) * CD_RB);
            const f32x4 *sb = reinterpret_cast<const f32x4 *>(own + (size_t)(32 + 8 * wave + p) * CD_RB);
#pragma unroll
            for (int c = 0; c < 16; c++) {
                const f32x4 va = sa[c], vb = sb[c];
                own_a[2 * c] = va.xy; own_a[2 * c + 1] = va.zw;
                own_b[2 * c] = vb.xy; own_b[2 * c + 1] = vb.zw;
            }
        }
        if (k > 0) emit_load();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this strip's rows
        cd_barrier();                                       // the own buffers and the tile are free
        if (more) own_unit(q0 + C3_NX, wave & 1, (wave >> 1) ? 5 : 0, (wave >> 1) ? 9 : 5);
        {
            float *Tw = T + (e - dc) * C3_TS + 16 * wave + 2 * p;   // tile column of pixel u (u + 1: +1), disparity e
            const int obase = u + 1 - e;                    // odd: rows j even are odd, j odd even
            const int kb = (obase >> 1) & (C3_RING - 1);
            const bool aok = u < W, bok = u + 1 < W;
            // wave-uniform (lanes past nd compute values that are never stored): no exec masking, so
            // the nine rows are one straight-line block the scheduler can pipeline across
            if (compute) {
                // the 72 (row, 32-byte piece) steps with the pieces two steps ahead in flight
                auto piece = [&](int jj, int mm, f32x4 &a, f32x4 &b) {
                    const int kj = (kb - (jj >> 1)) & (C3_RING - 1);
                    const f32x4 *row = reinterpret_cast<const f32x4 *>(
                        ring + (size_t)(((jj & 1) ? 0 : C3_RING) + kj) * CD_RB);
                    a = row[2 * mm];
                    b = row[2 * mm + 1];
                };
                f32x4 pa[3], pb[3];
                piece(0, 0, pa[0], pb[0]);
                piece(0, 1, pa[1], pb[1]);
#pragma unroll
                for (int j = 0; j < 9; j++) {
                    const int o = obase - j;
                    f32x2 xa[4], xb[4];     // accumulators (0,1) (2,3) (4,5) (6,7)
#pragma unroll
                    for (int m = 0; m < 8; m++) {
                        const int st = 8 * j + m, nx = st + 2;
                        if (nx < 72) piece(nx >> 3, nx & 7, pa[nx % 3], pb[nx % 3]);
                        const f32x4 a = pa[st % 3], b = pb[st % 3];
                        const f32x2 r[4] = {a.xy, a.zw, b.xy, b.zw};
#pragma unroll
                        for (int t = 0; t < 4; t++) {
                            if (j <= 7) {
                                const f32x2 pr = own_b[4 * m + t] * r[t];
                                xb[t] = m == 0 ? pr : xb[t] + pr;
                            }
                            if (j >= 1) {
                                const f32x2 pr = own_a[4 * m + t] * r[t];
                                xa[t] = m == 0 ? pr : xa[t] + pr;
                            }
                        }
                    }
                    // the pairwise tree ((a0+a1)+(a2+a3))+((a4+a5)+(a6+a7)): the first level within
                    // each pixel's channel pairs as single adds, the rest packed across the two pixels
                    // (left to itself, the compiler packed the first level with three moves per add)
                    if (j >= 1 && j <= 7) {
                        f32x2 s[4];
#pragma unroll
                        for (int t = 0; t < 4; t++) {
                            float ua, ub;
                            asm("v_add_f32 %0, %1, %2" : "=v"(ua) : "v"(xa[t].x), "v"(xa[t].y));
                            asm("v_add_f32 %0, %1, %2" : "=v"(ub) : "v"(xb[t].x), "v"(xb[t].y));
                            s[t] = f32x2{ua, ub};
                        }
                        const f32x2 sm = f32x2{0.0f, 0.0f} + ((s[0] + s[1]) + (s[2] + s[3]));
                        Tw[j * C3_TS + 1] = (bok && o >= 0) ? -sm.y : invalid;
                        Tw[(j - 1) * C3_TS] = (aok && o >= 0) ? -sm.x : invalid;
                    } else {
                        const f32x2 *x = j == 0 ? xb : xa;
                        float u[4];
#pragma unroll
                        for (int t = 0; t < 4; t++) asm("v_add_f32 %0, %1, %2" : "=v"(u[t]) : "v"(x[t].x), "v"(x[t].y));
                        const float sm = 0.0f + ((u[0] + u[1]) + (u[2] + u[3]));
                        if (j == 0) Tw[1] = (bok && o >= 0) ? -sm : invalid;
                        else Tw[7 * C3_TS] = (aok && o >= 0) ? -sm : invalid;
                    }
                    if (k > 0) emit_store(q0 - C3_NX, j);     // the previous strip's runs
                }
            } else {
                // past the row end: R's invalid fill only
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    Tw[j * C3_TS] = invalid;
                    Tw[j * C3_TS + 1] = invalid;
                    if (k > 0) emit_store(q0 - C3_NX, j);
                }
            }
        }
        // every wave's dots are done: the older row block's slots take the next strip's block
        cd_barrier();
        if (more) ring_unit(q0 + C3_NX - dc, wave & 1, (wave >> 1) ? 5 : 0, (wave >> 1) ? 9 : 5);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    cd_barrier();
    emit_load();
#pragma unroll
    for (int j = 0; j < NST / 8; j++) emit_store((nstrips - 1) * C3_NX, j);
}

// Any channel count: one lane per (pixel, d-range), features read from global
// memory, NumPy's full pairwise recursion.  Correctness path for C != 64.
template <int OUT>
__global__ __launch_bounds__(256) void cv_generic_kernel(const float *__restrict__ fl, const float *__restrict__ fr,
                                                         int H, int W, int C, int d0, int d1, int Dvol,
                                                         int sides, float invalid, float *__restrict__ outl,
                                                         float *__restrict__ outr, float *__restrict__ out_min,
                                                         int32_t *__restrict__ out_arg, float *__restrict__ out_disp)
{
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (int64_t)H * W) return;
    const int y = (int)(p / W), x = (int)(p % W);
    float best = __builtin_inff();
    int arg = -1;
    for (int d = d0; d < d1; d++) {
        float cost = invalid;
        if (x >= d) cost = np_neg_dot(fl + ((size_t)y * W + x) * C, fr + ((size_t)y * W + x - d) * C, C);
        if (OUT == OUT_WTA) {
            if (cost < best) { best = cost; arg = d; }
        } else if (OUT == OUT_DHW) {
            outl[((size_t)d * H + y) * W + x] = cost;
        } else {
            if (sides & SDE_SIDE_LEFT) outl[((size_t)y * W + x) * Dvol + d] = cost;
        }
        // right volume: R[y][x][d] = cost(x + d, d), computed by its own owner pixel x
        if (OUT == OUT_HWD && (sides & SDE_SIDE_RIGHT)) {
            float cr = invalid;
            if (x + d < W) cr = np_neg_dot(fl + ((size_t)y * W + x + d) * C, fr + ((size_t)y * W + x) * C, C);
            outr[((size_t)y * W + x) * Dvol + d] = cr;
        }
    }
    if (OUT == OUT_WTA) {
        if (out_min) out_min[p] = best;
        if (out_arg) out_arg[p] = arg;
        if (out_disp) out_disp[p] = (float)arg;
    }
}

// WTA over [D][H][W]: one lane per pixel, each d-slice read coalesced along W.
template <int RULE>
__global__ __launch_bounds__(256) void wta_dhw_kernel(const float *__restrict__ vol, int64_t npix, int D,
                                                      float *__restrict__ disp)
{
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npix) return;
    float best;
    int arg;
    if (RULE == SDE_WTA_INIT_D0) { best = vol[p]; arg = 0; }
    else { best = __builtin_inff(); arg = -1; }
    for (int d = (RULE == SDE_WTA_INIT_D0 ? 1 : 0); d < D; d++) {
        const float v = vol[(size_t)d * npix + p];
        if (v < best) { best = v; arg = d; }
    }
    disp[p] = (float)arg;
}

// WTA over [H][W][D]: 16 lanes per pixel (4 pixels per wave), each lane scans a
// strided subset in increasing d, then a (value, index) merge across the 16
// lanes reproduces the sequential scan.
template <int RULE>
__global__ __launch_bounds__(256) void wta_hwd_kernel(const float *__restrict__ vol, int64_t npix, int D,
                                                      float *__restrict__ disp)
{
    const int sub = threadIdx.x & 15;
    const int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const bool ok = p < npix;
    const float *v = vol + (size_t)(ok ? p : 0) * D;
    float best = __builtin_inff();
    int arg = -1;
    if (ok) {
        for (int d = sub; d < D; d += 16) {
            const float x = v[d];
            if (x < best) { best = x; arg = d; }
        }
    }
    // A lane with arg = -1 holds +inf; a lane with a winner holds a value < +inf,
    // so the plain (value, index) merge never lets -1 win against a real index.
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
        const float ob = __shfl_xor(best, off, 64);
        const int oa = __shfl_xor(arg, off, 64);
        argmin_merge(best, arg, ob, oa);
    }
    if (ok && sub == 0) {
        if (RULE == SDE_WTA_INIT_D0) {
            // best = v[0], `best > v[d]` (:805-811): identical to the +inf scan except that
            // "no winner" reads 0 and a NaN at d = 0 is never replaced.
            const float v0 = v[0];
            if (arg < 0 || v0 != v0) arg = 0;
        }
        disp[p] = (float)arg;
    }
}

__global__ __launch_bounds__(256) void argmin_merge_kernel(const float *__restrict__ mins,
                                                           const int32_t *__restrict__ args, int nshards,
                                                           int64_t npix, float *__restrict__ disp)
{
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npix) return;
    float best = mins[p];
    int arg = args[p];
    for (int s = 1; s < nshards; s++) {
        const float m = mins[(size_t)s * npix + p];
        const int a = args[(size_t)s * npix + p];
        if (m < best) { best = m; arg = a; }   // shards are ordered by d: ties keep the earlier one
    }
    disp[p] = (float)arg;
}

// Chunked certified CV + WTA (sde_cv_wta, D past one row sweep's LDS window): chunk k's exact first-minimum
// (value, index) per pixel at mins / args + k * npix, chunks ordered by d; the pixel's first minimum over
// all of them (strict <: a later chunk wins only with a smaller cost -- a sequential scan over d), written
// to whichever outputs are requested.
__global__ __launch_bounds__(256) void argmin_chunks_kernel(const float *__restrict__ mins,
                                                            const int32_t *__restrict__ args, int nchunks,
                                                            int64_t npix, float *__restrict__ disp,
                                                            float *__restrict__ out_min, int32_t *__restrict__ out_arg)
{
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npix) return;
    float best = mins[p];
    int arg = args[p];
    for (int k = 1; k < nchunks; k++) {
        const float m = mins[(size_t)k * npix + p];
        if (m < best) { best = m; arg = args[(size_t)k * npix + p]; }
    }
    if (disp) disp[p] = (float)arg;
    if (out_min) out_min[p] = best;
    if (out_arg) out_arg[p] = arg;
}

// ===========================================================================
// Certified fast path for the fused cost volume + WTA (north-star kernel).
//
// Scores s(x,d) = fl[x] . fr[x-d] are computed on the bf16 MFMA
// (v_mfma_f32_32x32x16_bf16) with every fp32 operand split into hi + lo bf16
// parts and the three leading partial products (hh, hl, lh) accumulated in
// fp32.  Rigorous bound for every voxel of a pixel (Cauchy-Schwarz on |a|,|b|):
//   |s_fast - s_true| <= (3*2^-16 + 192*2^-23) * sum|a_c b_c|   (split + accumulation)
//   |s_exact - s_true| <= 10*2^-24 * sum|a_c b_c|               (NumPy pairwise order)
//   => |s_fast - s_exact| <= FX_K * sum|a_c b_c| <= FX_K * ||fl[x]||_2 * max_window ||fr||_2
//      (FX_K = 1e-4: 1.4x margin over 7e-5; the per-pixel L2 norms are fp32 sums of
//      squares inflated by 1 + 4e-6, an upper bound)
// If the best fast score beats the runner-up by more than 2 eps, the exact
// first-min is provably the fast argmax (no other d can tie or win exactly),
// and its exact cost is computed once (same arithmetic as cv64_kernel).  Any
// other pixel (near-ties, NaN/Inf features) goes to a work list that
// cv_wta_fixup_kernel resolves with the exact scan.  Outputs are therefore
// bit-identical to the exact kernel for every input.
//
// Mapping: workgroup = 4 waves on one row and 64 left pixels (2 N-tiles of 32);
// the right-feature window of a <=128-disparity chunk (<= 6 M-tiles of 32
// pixels) arrives pre-split as hi/lo bf16 planes (written by the tower's last
// epilogue or feature_split_kernel) and is staged into LDS by LDS-DMA
// (global_load_lds, swizzle applied to the source address); wave w owns N-tile
// w&1 and every other M-tile; the left operand lives in registers (hi/lo).
// Blocks are remapped so all blocks of a row run on one XCD (its L2 serves the
// overlapping windows).
// ===========================================================================
// Split of a feature map for the certified path: x = hi + lo + r with hi =
// bf16_rne(x), lo = bf16_rne(x - hi) (|r| <= 2^-16 |x|), plus an upper bound of
// each pixel's L2 norm (fp32 sum of 64 squares, relative error <= 64*2^-24,
// inflated by (1 + 4e-6)).  16 lanes per pixel, one float4 each.

__global__ __launch_bounds__(256) void feature_split_kernel(const float *__restrict__ f, int64_t npix,
                                                            uint16_t *__restrict__ hi, uint16_t *__restrict__ lo,
                                                            float *__restrict__ nrm)
{
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool ok = idx < npix * 16;
    const float4 v = ok ? reinterpret_cast<const float4 *>(f)[idx] : make_float4(0.f, 0.f, 0.f, 0.f);
    float ss = v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    ss += __shfl_xor(ss, 1, 64);
    ss += __shfl_xor(ss, 2, 64);
    ss += __shfl_xor(ss, 4, 64);
    ss += __shfl_xor(ss, 8, 64);
    if (!ok) return;
    __bf16 h0, h1, h2, h3, l0, l1, l2, l3;
    fx_split(v.x, h0, l0); fx_split(v.y, h1, l1); fx_split(v.z, h2, l2); fx_split(v.w, h3, l3);
    typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
    const bf4 hv = {h0, h1, h2, h3}, lv = {l0, l1, l2, l3};
    reinterpret_cast<uint2 *>(hi)[idx] = __builtin_bit_cast(uint2, hv);
    reinterpret_cast<uint2 *>(lo)[idx] = __builtin_bit_cast(uint2, lv);
    if ((idx & 15) == 0) nrm[idx >> 4] = sqrtf(ss) * FX_NORM_UP;
}

// Certified fast kernel on pre-split operands.  One workgroup per (row,
// 64-pixel strip), <= 128-disparity chunks (window <= 6 M-tiles = 192 pixels,
// 48 KB of hi/lo planes in LDS -> 3 workgroups per CU).  The window is staged
// by LDS-DMA (global_load_lds_dwordx4: no VGPRs, no VALU): each wave-instruction
// fills 1 KB of the swizzled image linearly, so the swizzle is applied to the
// per-lane SOURCE chunk.  Invalid voxels (x - d < 0: exact cost -0.0) are
// forced to score +0 in the edge-tile path.
__global__ __launch_bounds__(256) void cv_wta_cert_kernel(const float *__restrict__ fl, const float *__restrict__ fr,
                                                          const uint4 *__restrict__ lhi, const uint4 *__restrict__ llo,
                                                          const float *__restrict__ lnrm,
                                                          const uint4 *__restrict__ rhi, const uint4 *__restrict__ rlo,
                                                          const float *__restrict__ rnrm, int H, int W, int d0, int d1,
                                                          float *__restrict__ out_min, int32_t *__restrict__ out_arg,
                                                          float *__restrict__ out_disp, unsigned *__restrict__ counter,
                                                          int32_t *__restrict__ list)
{
    __shared__ uint4 pl[2 * FX_WIN * 8];            // [plane][pixel][8 chunks], swizzled
    __shared__ float mb[4][64];
    __shared__ int ma[4][64];
    __shared__ float ms[4][64];
    __shared__ unsigned nmax_bits;

    const int nbx = (W + FX_NX - 1) / FX_NX;
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int y = lb / nbx;
    const int x0 = (lb % nbx) * FX_NX;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = wave & 1, mpar = wave >> 1;
    const int j = lane & 31, h = lane >> 5;
    const int x = x0 + 32 * n + j;
    const bool xok = x < W;
    const size_t rowpix = (size_t)y * W;
    if (tid == 0) nmax_bits = 0u;

    // left operand: 16-B chunks 2s+h of this lane's pixel (channels 16s+8h..+7)
    fx_bf16x8 bh[4], bl[4];
    {
        const size_t pc = (rowpix + (xok ? x : 0)) * 8;
#pragma unroll
        for (int s = 0; s < 4; s++) {
            bh[s] = __builtin_bit_cast(fx_bf16x8, lhi[pc + 2 * s + h]);
            bl[s] = __builtin_bit_cast(fx_bf16x8, llo[pc + 2 * s + h]);
        }
    }
    const float nl = lnrm[rowpix + (xok ? x : 0)];

    float b1[4], b2[4];
    int ag[4];
#pragma unroll
    for (int t = 0; t < 4; t++) { b1[t] = -__builtin_inff(); b2[t] = -__builtin_inff(); ag[t] = -1; }

    for (int dc0 = d0; dc0 < d1; dc0 += FX_DCH) {
        const int dc1 = min(dc0 + FX_DCH, d1);
        const int nt = (dc1 - dc0 + 63 + 31) / 32;
        const int rb = x0 + FX_NX - dc0 - 32 * nt;     // right pixel of window row 0
        __syncthreads();                               // previous chunk's plane reads are done
        // LDS-DMA: 2 planes x nt*32 pixels x 8 chunks = nt*8 KB; 1 KB (8 pixels) per wave-instruction
        const int ninst = nt * 4 * 2;                  // per plane nt*4 instructions
        for (int ii = wave; ii < ninst; ii += 4) {
            const int plane = ii / (nt * 4);
            const int slot = (ii - plane * nt * 4) * 64 + lane;   // 16-B slot within the plane image
            const int r = slot >> 3, cs = slot & 7;
            const int c8 = cs ^ ((r >> 1) & 7);                  // source chunk for this LDS slot
            const int xr = min(max(rb + r, 0), W - 1);
            const uint4 *src = (plane ? rlo : rhi) + (rowpix + xr) * 8 + c8;
            __builtin_amdgcn_global_load_lds((const void *)src,
                                             (__attribute__((address_space(3))) void *)(pl + plane * FX_WIN * 8 +
                                                                                        (ii - plane * nt * 4) * 64),
                                             16, 0, 0);
        }
        // window norm bound: max over its pixels
        {
            float nm = 0.0f;
            for (int r = tid; r < nt * 32; r += 256) {
                const int xr = rb + r;
                if (xr >= 0 && xr < W) nm = fmaxf(nm, rnrm[rowpix + xr]);
            }
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) nm = fmaxf(nm, __shfl_xor(nm, o, 64));
            if (lane == 0) atomicMax(&nmax_bits, __float_as_uint(nm));   // non-negative: uint order
        }
        __syncthreads();                               // drains the DMA (vmcnt(0)) and publishes it

        const int xbase = x0 + 32 * n;
        for (int m = mpar; m < nt; m += 2) {
            const int dt = xbase - (rb + 32 * m);
            const int dlo = dt - 31, dhi = dt + 31;
            if (dhi < dc0 || dlo >= dc1) continue;     // wave-uniform
            fx_floatx16 acc = {0};
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const int sl = fx_slot(32 * m + j, 2 * s + h);
                const fx_bf16x8 ah = __builtin_bit_cast(fx_bf16x8, pl[sl]);
                const fx_bf16x8 al = __builtin_bit_cast(fx_bf16x8, pl[FX_WIN * 8 + sl]);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[s], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[s], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[s], acc, 0, 0, 0);
            }
            const int dl = dt + j - 4 * h;             // d of register r is dl - ((r&3) + 8(r>>2))
            const int xrl = rb + 32 * m + 4 * h;       // right pixel of register r is xrl + ((r&3) + 8(r>>2))
            if (dlo >= dc0 && dhi < dc1 && rb + 32 * m >= 0) {
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
                    const int ri = (r & 3) + 8 * (r >> 2);
                    const int d = dl - ri;
                    float sc = (xrl + ri < 0) ? 0.0f : acc[r];          // x < d: exact cost -0.0
                    sc = (d >= dc0 && d < dc1) ? sc : -__builtin_inff();
                    const bool gt = sc > b1[t];
                    ag[t] = gt ? d : ag[t];
                    b2[t] = __builtin_amdgcn_fmed3f(b1[t], b2[t], sc);
                    b1[t] = fmaxf(b1[t], sc);
                }
            }
        }
    }

    float best = b1[0], second = b2[0];
    int arg = ag[0];
#pragma unroll
    for (int t = 1; t < 4; t++) fx_merge(best, arg, second, b1[t], ag[t], b2[t]);
    {
        const float bb = __shfl_xor(best, 32, 64), ss = __shfl_xor(second, 32, 64);
        const int aa = __shfl_xor(arg, 32, 64);
        fx_merge(best, arg, second, bb, aa, ss);
    }
    mb[wave][lane] = best;
    ma[wave][lane] = arg;
    ms[wave][lane] = second;
    __syncthreads();
    if (wave < 2 && h == 0 && xok) {
        fx_merge(best, arg, second, mb[wave + 2][lane], ma[wave + 2][lane], ms[wave + 2][lane]);
        const float eps = FX_K * nl * __uint_as_float(nmax_bits) + FX_ABS;
        const size_t p = rowpix + x;
        if ((best - second) > 2.0f * eps && arg >= 0) {
            if (out_min) {
                float cost = -0.0f;
                if (x - arg >= 0)   // exact cost of the winner: NumPy pairwise order, as cv64_kernel
                    cost = dot64_exact_global(reinterpret_cast<const float4 *>(fl + p * 64),
                                              reinterpret_cast<const float4 *>(fr + (p - arg) * 64));
                out_min[p] = cost;
            }
            if (out_arg) out_arg[p] = arg;
            if (out_disp) out_disp[p] = (float)arg;
        } else {
            const unsigned e = atomicAdd(counter, 1u);
            list[e] = (int32_t)p;
        }
    }
}


// Exact resolution of the listed pixels, one 4-wave workgroup per pixel (persistent over the list).
// Wave v takes disparities [d0 + vQ, d0 + (v+1)Q), Q = 8 ceil(D / 32); each of its 8 lane groups of 8
// takes one disparity per iteration, lane jj of a group the products of channels 8m + jj, m = 0..7, in
// order -- dot64_exact_global's partial sum acc[jj] -- and the group's xor butterfly adds the 8 partial
// sums in that function's tree order (adds are commutative: the same bits).  A group scans its
// disparities in increasing d with a strict <, then (value, index) merges over the groups and the waves
// give the sequential first minimum.  All of a wave's iterations are in flight at once up to D = 256 (a
// chunk): one round of loads per pixel instead of a lane's three to four dependent 16-load dots, whose
// 64 lanes each read another pixel's 256 B (64 cache lines per load instruction).
constexpr int FX2_U = 8;   // iterations per round of loads
__global__ __launch_bounds__(256) void cv_wta_fixup_kernel(const float *__restrict__ fl, const float *__restrict__ fr,
                                                           int W, int d0, int d1, const unsigned *__restrict__ counter,
                                                           const int32_t *__restrict__ list, float *__restrict__ out_min,
                                                           int32_t *__restrict__ out_arg, float *__restrict__ out_disp)
{
    __shared__ float wb[4];
    __shared__ int wa[4];
    const unsigned cnt = *counter;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 3, jj = lane & 7;
    const int Q = (d1 - d0 + 31) / 32 * 8;
    const int dw = d0 + wave * Q, dwe = min(d1, dw + Q);
    for (unsigned e = blockIdx.x; e < cnt; e += gridDim.x) {
        const size_t p = (size_t)list[e];
        const int x = (int)(p % W);
        const size_t rowbase = p - x;
        float av[8];
#pragma unroll
        for (int m = 0; m < 8; m++) av[m] = fl[p * 64 + 8 * m + jj];
        float best = __builtin_inff();
        int arg = -1;
        for (int db = dw; db < dwe; db += 8 * FX2_U) {
            float bv[FX2_U][8];
#pragma unroll
            for (int u = 0; u < FX2_U; u++) {
                const int xr = x - (db + 8 * u + g);
                const float *b = fr + (rowbase + (xr >= 0 ? xr : 0)) * 64 + jj;
#pragma unroll
                for (int m = 0; m < 8; m++) bv[u][m] = b[8 * m];
            }
#pragma unroll
            for (int u = 0; u < FX2_U; u++) {
                const int d = db + 8 * u + g;
                float acc = av[0] * bv[u][0];
#pragma unroll
                for (int m = 1; m < 8; m++) acc = acc + av[m] * bv[u][m];
                acc = acc + __shfl_xor(acc, 1, 64);   // (acc0 + acc1), (acc2 + acc3), ...
                acc = acc + __shfl_xor(acc, 2, 64);   // ((acc0 + acc1) + (acc2 + acc3)), ...
                acc = acc + __shfl_xor(acc, 4, 64);
                const float c = x - d >= 0 ? -(0.0f + acc) : -0.0f;
                if (d < dwe && c < best) {
                    best = c;
                    arg = d;
                }
            }
        }
#pragma unroll
        for (int off = 8; off < 64; off <<= 1) {
            const float ob = __shfl_xor(best, off, 64);
            const int oa = __shfl_xor(arg, off, 64);
            argmin_merge(best, arg, ob, oa);
        }
        if (lane == 0) {
            wb[wave] = best;
            wa[wave] = arg;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            best = wb[0];
            arg = wa[0];
#pragma unroll
            for (int v = 1; v < 4; v++) argmin_merge(best, arg, wb[v], wa[v]);
            if (out_min) out_min[p] = best;
            if (out_arg) out_arg[p] = arg;
            if (out_disp) out_disp[p] = (float)arg;
        }
        __syncthreads();
    }
}

}  // namespace sde

using namespace sde;

SDE_EXPORT int sde_abi_version(void) { return SDE_ABI_VERSION; }

SDE_EXPORT const char *sde_status_string(int s)
{
    switch (s) {
    case SDE_OK: return "ok";
    case SDE_ERR_ARG: return "invalid argument";
    case SDE_ERR_LAUNCH: return "kernel launch failed";
    case SDE_ERR_WORKSPACE: return "workspace too small";
    default: return "unknown status";
    }
}

SDE_EXPORT int sde_cost_volume(const float *fl, const float *fr, int H, int W, int C, int D, int layout,
                               int sides, float invalid, float *out_left, float *out_right, void *stream)
{
    if (!fl || !fr || H <= 0 || W <= 0 || C <= 0 || D <= 0) return SDE_ERR_ARG;
    if (layout != SDE_LAYOUT_DHW && layout != SDE_LAYOUT_HWD) return SDE_ERR_ARG;
    if ((sides & ~(SDE_SIDE_LEFT | SDE_SIDE_RIGHT)) || !sides) return SDE_ERR_ARG;
    if ((sides & SDE_SIDE_LEFT) && !out_left) return SDE_ERR_ARG;
    if ((sides & SDE_SIDE_RIGHT) && !out_right) return SDE_ERR_ARG;
    if (layout == SDE_LAYOUT_DHW && (sides & SDE_SIDE_RIGHT)) return SDE_ERR_ARG;
    hipStream_t st = as_stream(stream);
    if (C == 64) {
        dim3 grid(cdiv(W, CV_TX), H);
        if (layout == SDE_LAYOUT_DHW) {
            cv64_kernel<SDE_SIDE_LEFT, OUT_DHW><<<grid, 256, 0, st>>>(fl, fr, H, W, 0, D, D, invalid, out_left,
                                                                       nullptr, nullptr, nullptr);
        } else if ((int64_t)W * D * 4 < (int64_t)CD_OOB) {
            // one row sweep per (row, 64-disparity chunk) writes both volumes (the left one alone: the
            // same sweep without the right volume's stores).  The >64 KB dynamic-LDS opt-in is set for
            // the kernel that launches, once per device.  (Rows of 2 GiB or more take the per-side
            // kernels below.)
            const int nchunks = cdiv(D, CV_DC);
            const dim3 grid1((unsigned)(nchunks * H));
            auto opt_in = [](std::atomic<uint64_t> &done, const void *k, size_t bytes) {
                return once_per_device(done, [k, bytes] {
                    return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) == hipSuccess;
                });
            };
            static std::atomic<uint64_t> a3l{0}, a3{0};
            if (sides == SDE_SIDE_LEFT) {
                if (!opt_in(a3l, reinterpret_cast<const void *>(cvlr3_kernel<false>), C3_SMEM)) return SDE_ERR_LAUNCH;
                cvlr3_kernel<false><<<grid1, 256, C3_SMEM, st>>>(fl, fr, H, W, D, nchunks, invalid, out_left, nullptr);
            } else if (sides == (SDE_SIDE_LEFT | SDE_SIDE_RIGHT)) {
                if (!opt_in(a3, reinterpret_cast<const void *>(cvlr3_kernel<true>), C3_SMEM)) return SDE_ERR_LAUNCH;
                cvlr3_kernel<true><<<grid1, 256, C3_SMEM, st>>>(fl, fr, H, W, D, nchunks, invalid, out_left, out_right);
            } else {
                cv64_kernel<SDE_SIDE_RIGHT, OUT_HWD><<<grid, 256, 0, st>>>(fr, fl, H, W, 0, D, D, invalid,
                                                                            out_right, nullptr, nullptr, nullptr);
            }
        } else {
            if (sides & SDE_SIDE_LEFT)
                cv64_kernel<SDE_SIDE_LEFT, OUT_HWD><<<grid, 256, 0, st>>>(fl, fr, H, W, 0, D, D, invalid,
                                                                           out_left, nullptr, nullptr, nullptr);
            if (sides & SDE_SIDE_RIGHT)
                cv64_kernel<SDE_SIDE_RIGHT, OUT_HWD><<<grid, 256, 0, st>>>(fr, fl, H, W, 0, D, D, invalid,
                                                                            out_right, nullptr, nullptr, nullptr);
        }
    } else {
        const int blocks = cdiv((int64_t)H * W, 256);
        if (layout == SDE_LAYOUT_DHW)
            cv_generic_kernel<OUT_DHW><<<blocks, 256, 0, st>>>(fl, fr, H, W, C, 0, D, D, sides, invalid, out_left,
                                                                nullptr, nullptr, nullptr, nullptr);
        else
            cv_generic_kernel<OUT_HWD><<<blocks, 256, 0, st>>>(fl, fr, H, W, C, 0, D, D, sides, invalid, out_left,
                                                                out_right, nullptr, nullptr, nullptr);
    }
    return launch_status();
}

// certified-mode workspace: [counters 256 B][list 4*npix][planes 4 x 128*npix][norms 2 x 4*npix]; the fix-up
// count of a call is the sum of the 64 counter words (one per disparity chunk, sde_cv_wta's chunked path)
constexpr int CERT_COUNTERS = 64;
static int64_t cert_ws_bytes(int H, int W, bool with_planes)
{
    const int64_t npix = (int64_t)H * W;
    int64_t b = 256 + ((4 * npix + 255) / 256) * 256;
    if (with_planes) b += 4 * 128 * npix + 2 * ((4 * npix + 255) / 256) * 256;
    return b;
}

SDE_EXPORT int64_t sde_cv_wta_workspace_bytes(int H, int W)
{
    if (H <= 0 || W <= 0) return -1;
    return cert_ws_bytes(H, W, true);
}

// chunked row sweep: [counter, list] then the chunks' (min, arg) planes; INT64_MAX when [d0, d1) does not split
// into row-sweep-supported chunks (the chunk kernel path then runs)
constexpr int ROW_CHUNK = 256;
static int64_t row_chunk_layout(int H, int W, int d0, int d1)
{
    const int K = cdiv(d1 - d0, ROW_CHUNK);
    if (K > CERT_COUNTERS) return INT64_MAX;
    for (int k = 0; k < K; k++)
        if (!row_cert_supported(d0 + k * ROW_CHUNK, std::min(d1, d0 + (k + 1) * ROW_CHUNK))) return INT64_MAX;
    return cert_ws_bytes(H, W, false) + (int64_t)K * 8 * H * W;
}

SDE_EXPORT int sde_feature_split(const float *feat, int64_t npix, int C, uint16_t *hi, uint16_t *lo, float *norm,
                                 void *stream)
{
    if (!feat || !hi || !lo || !norm || npix <= 0 || C != 64) return SDE_ERR_ARG;
    feature_split_kernel<<<cdiv(npix * 16, 256), 256, 0, as_stream(stream)>>>(feat, npix, hi, lo, norm);
    return launch_status();
}

static int launch_cert(const float *fl, const float *fr, const uint16_t *lhi, const uint16_t *llo, const float *lnrm,
                       const uint16_t *rhi, const uint16_t *rlo, const float *rnrm, int H, int W, int d0, int d1,
                       float *disp, float *min_cost, int32_t *argmin, void *ws, hipStream_t st)
{
    unsigned *counter = reinterpret_cast<unsigned *>(ws);
    int32_t *list = reinterpret_cast<int32_t *>(reinterpret_cast<char *>(ws) + 256);
    if (hipMemsetAsync(counter, 0, CERT_COUNTERS * sizeof(unsigned), st) != hipSuccess) return SDE_ERR_LAUNCH;
    cv_wta_cert_kernel<<<cdiv(W, FX_NX) * H, 256, 0, st>>>(
        fl, fr, reinterpret_cast<const uint4 *>(lhi), reinterpret_cast<const uint4 *>(llo), lnrm,
        reinterpret_cast<const uint4 *>(rhi), reinterpret_cast<const uint4 *>(rlo), rnrm, H, W, d0, d1, min_cost,
        argmin, disp, counter, list);
    cv_wta_fixup_kernel<<<1024, 256, 0, st>>>(fl, fr, W, d0, d1, counter, list, min_cost, argmin, disp);
    return SDE_OK;
}

SDE_EXPORT int64_t sde_cv_wta_split_workspace_bytes(int H, int W)
{
    if (H <= 0 || W <= 0) return -1;
    return cert_ws_bytes(H, W, false);
}

SDE_EXPORT int sde_cv_wta_split(const float *fl, const float *fr, const uint16_t *fl_hi, const uint16_t *fl_lo,
                                const float *fl_norm, const uint16_t *fr_hi, const uint16_t *fr_lo,
                                const float *fr_norm, int H, int W, int d0, int d1, float *disp, float *min_cost,
                                int32_t *argmin, void *workspace, int64_t workspace_bytes, void *stream)
{
    if (!fl || !fr || !fl_hi || !fl_lo || !fl_norm || !fr_hi || !fr_lo || !fr_norm) return SDE_ERR_ARG;
    if (H <= 0 || W <= 0 || d0 < 0 || d1 <= d0 || (!disp && !min_cost && !argmin)) return SDE_ERR_ARG;
    if (!workspace || workspace_bytes < cert_ws_bytes(H, W, false)) return SDE_ERR_WORKSPACE;
    const int s = launch_cert(fl, fr, fl_hi, fl_lo, fl_norm, fr_hi, fr_lo, fr_norm, H, W, d0, d1, disp, min_cost,
                              argmin, workspace, as_stream(stream));
    if (s != SDE_OK) return s;
    return launch_status();
}

SDE_EXPORT int sde_cv_wta(const float *fl, const float *fr, int H, int W, int C, int d0, int d1, float *disp,
                          float *min_cost, int32_t *argmin, int mode, void *workspace, int64_t workspace_bytes,
                          void *stream)
{
    if (!fl || !fr || H <= 0 || W <= 0 || C <= 0 || d0 < 0 || d1 <= d0) return SDE_ERR_ARG;
    if (!disp && !min_cost && !argmin) return SDE_ERR_ARG;
    if (mode != SDE_CV_EXACT && mode != SDE_CV_CERTIFIED) return SDE_ERR_ARG;
    hipStream_t st = as_stream(stream);
    if (C == 64 && mode == SDE_CV_CERTIFIED && row_cert_supported(d0, d1)) {
        // row-sweep kernel straight from the fp32 features (cv_row.hip)
        if (!workspace || workspace_bytes < sde_cv_wta_workspace_bytes(H, W)) return SDE_ERR_WORKSPACE;
        unsigned *counter = reinterpret_cast<unsigned *>(workspace);
        int32_t *list = reinterpret_cast<int32_t *>(reinterpret_cast<char *>(workspace) + 256);
        if (hipMemsetAsync(counter, 0, CERT_COUNTERS * sizeof(unsigned), st) != hipSuccess) return SDE_ERR_LAUNCH;
        launch_row_cert(fl, fr, H, W, d0, d1, min_cost, argmin, disp, counter, list, st);
        cv_wta_fixup_kernel<<<1024, 256, 0, st>>>(fl, fr, W, d0, d1, counter, list, min_cost, argmin, disp);
    } else if (C == 64 && mode == SDE_CV_CERTIFIED && row_chunk_layout(H, W, d0, d1) <= sde_cv_wta_workspace_bytes(H, W)) {
        // D past the row sweep's LDS window (e.g. BASELINE config 5, D = 512): ROW_CHUNK-disparity chunks, each
        // through the row-sweep kernel + its exact fix-ups (the same outputs as the exact kernel on that
        // range, as for the disparity shards of parallel.py), then the first minimum over the chunks in d order
        if (!workspace || workspace_bytes < sde_cv_wta_workspace_bytes(H, W)) return SDE_ERR_WORKSPACE;
        const int64_t npix = (int64_t)H * W;
        const int K = cdiv(d1 - d0, ROW_CHUNK);
        unsigned *counter = reinterpret_cast<unsigned *>(workspace);
        int32_t *list = reinterpret_cast<int32_t *>(reinterpret_cast<char *>(workspace) + 256);
        float *cmin = reinterpret_cast<float *>(reinterpret_cast<char *>(workspace) + cert_ws_bytes(H, W, false));
        int32_t *carg = reinterpret_cast<int32_t *>(cmin + (size_t)K * npix);
        // chunk k counts its fix-ups in counter word k (sde_cv_wta_fixups-style readers sum the words); the
        // list is reused: chunk k's fix-ups run before chunk k + 1's sweep
        if (hipMemsetAsync(counter, 0, CERT_COUNTERS * sizeof(unsigned), st) != hipSuccess) return SDE_ERR_LAUNCH;
        for (int k = 0; k < K; k++) {
            const int a = d0 + k * ROW_CHUNK, b = std::min(d1, a + ROW_CHUNK);
            launch_row_cert(fl, fr, H, W, a, b, cmin + (size_t)k * npix, carg + (size_t)k * npix, nullptr, counter + k,
                            list, st, k > 0 ? cmin + (size_t)(k - 1) * npix : nullptr);
            cv_wta_fixup_kernel<<<1024, 256, 0, st>>>(fl, fr, W, a, b, counter + k, list, cmin + (size_t)k * npix,
                                                      carg + (size_t)k * npix, nullptr);
        }
        argmin_chunks_kernel<<<cdiv(npix, 256), 256, 0, st>>>(cmin, carg, K, npix, disp, min_cost, argmin);
    } else if (C == 64 && mode == SDE_CV_CERTIFIED) {
        if (!workspace || workspace_bytes < sde_cv_wta_workspace_bytes(H, W)) return SDE_ERR_WORKSPACE;
        const int64_t npix = (int64_t)H * W;
        char *base = reinterpret_cast<char *>(workspace) + cert_ws_bytes(H, W, false);
        uint16_t *lhi = reinterpret_cast<uint16_t *>(base);
        uint16_t *llo = lhi + 64 * npix;
        uint16_t *rhi = llo + 64 * npix;
        uint16_t *rlo = rhi + 64 * npix;
        float *lnrm = reinterpret_cast<float *>(rlo + 64 * npix);
        float *rnrm = lnrm + ((npix + 63) / 64) * 64;
        feature_split_kernel<<<cdiv(npix * 16, 256), 256, 0, st>>>(fl, npix, lhi, llo, lnrm);
        feature_split_kernel<<<cdiv(npix * 16, 256), 256, 0, st>>>(fr, npix, rhi, rlo, rnrm);
        const int s = launch_cert(fl, fr, lhi, llo, lnrm, rhi, rlo, rnrm, H, W, d0, d1, disp, min_cost, argmin,
                                  workspace, st);
        if (s != SDE_OK) return s;
    } else if (C == 64) {
        dim3 grid(cdiv(W, CV_TX), H);
        cv64_kernel<SDE_SIDE_LEFT, OUT_WTA><<<grid, 256, 0, st>>>(fl, fr, H, W, d0, d1, 0, -0.0f, nullptr,
                                                                   min_cost, argmin, disp);
    } else {
        const int blocks = cdiv((int64_t)H * W, 256);
        cv_generic_kernel<OUT_WTA><<<blocks, 256, 0, st>>>(fl, fr, H, W, C, d0, d1, 0, SDE_SIDE_LEFT, -0.0f,
                                                            nullptr, nullptr, min_cost, argmin, disp);
    }
    return launch_status();
}

SDE_EXPORT int sde_wta(const float *vol, int H, int W, int D, int layout, int rule, float *disp, void *stream)
{
    if (!vol || !disp || H <= 0 || W <= 0 || D <= 0) return SDE_ERR_ARG;
    if (rule != SDE_WTA_INIT_INF && rule != SDE_WTA_INIT_D0) return SDE_ERR_ARG;
    hipStream_t st = as_stream(stream);
    const int64_t npix = (int64_t)H * W;
    if (layout == SDE_LAYOUT_DHW) {
        const int blocks = cdiv(npix, 256);
        if (rule == SDE_WTA_INIT_INF) wta_dhw_kernel<SDE_WTA_INIT_INF><<<blocks, 256, 0, st>>>(vol, npix, D, disp);
        else wta_dhw_kernel<SDE_WTA_INIT_D0><<<blocks, 256, 0, st>>>(vol, npix, D, disp);
    } else if (layout == SDE_LAYOUT_HWD) {
        const int blocks = cdiv(npix * 16, 256);
        if (rule == SDE_WTA_INIT_INF) wta_hwd_kernel<SDE_WTA_INIT_INF><<<blocks, 256, 0, st>>>(vol, npix, D, disp);
        else wta_hwd_kernel<SDE_WTA_INIT_D0><<<blocks, 256, 0, st>>>(vol, npix, D, disp);
    } else {
        return SDE_ERR_ARG;
    }
    return launch_status();
}

SDE_EXPORT int sde_argmin_merge(const float *mins, const int32_t *args, int nshards, int64_t npix, float *disp,
                                void *stream)
{
    if (!mins || !args || !disp || nshards <= 0 || npix <= 0) return SDE_ERR_ARG;
    argmin_merge_kernel<<<cdiv(npix, 256), 256, 0, as_stream(stream)>>>(mins, args, nshards, npix, disp);
    return launch_status();
}
