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

#include <algorithm>

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

// Chain arithmetic: fp64 (definition v2).  CBCA_P32 builds (timing probes, tools/build_file_variant.sh) run the
// chains, rings and the mean's reciprocal in fp32 -- different results, half the ring LDS.
#ifdef CBCA_P32
typedef float cb_p;
typedef float cb_r;
#else
typedef double cb_p;
typedef double cb_r;
#endif

struct CbcaArgs {
    const float *src;
    float *dst;
    const uint32_t *al, *ar;       // row-major arms (left / right image): horizontal pass
    const uint32_t *alT;           // column-major left-image arms (pitch Hp): vertical pass
    int H, W, D, M, Hp;
    int nseg, ndc;
    int64_t nitems;
    int64_t nper;                  // items per segment (vertical pass: valid (column, chunk) pairs only)
};

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

// ---------------------------------------------------------------------------------------------
// Horizontal pass: item = (segment k, row y, chunk c), c fastest; wave w takes items w, w + G, ...,
// so the waves in flight walk the same segment of consecutive rows, a pixel's chunks side by side.
// ---------------------------------------------------------------------------------------------
// SEL: some lane's chain starts inside the walk (d > fs: early segments); otherwise every front
// position is on every lane's chain and the per-step select goes
template <int R, bool SEL>
__device__ __forceinline__ void cbca_h_item(const CbcaArgs &A, int y, int c, int k, cb_p *__restrict__ sP)
{
    constexpr int RS = 2 * R + 2, PF = RS;
    const int lane = threadIdx.x & 63;
    const int W = A.W, D = A.D, M = A.M;
    const int d0 = 64 * c, d = d0 + lane;
    const int t0 = k * SDE_CBCA_SEG, t1 = min(t0 + SDE_CBCA_SEG, W);
    if (t1 <= d0) return;                          // every voxel of the segment is invalid
    const int fs = max(t0 - M, d0);                // walk start = lane 0's chain base
    // outputs trail the front by R + 1: a step issues its output's LDS reads first (every slot they
    // touch already holds its position -- the front's own slot still the one RS back) and consumes
    // them after the front's work, which hides their latency
    const int fe = t1 + R;                         // last front position (output t1 - 1)
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
    // the arms first: a loop-carried register loaded after the cost prefetch would make the entry
    // path's wait for it (merged into every block start) drain the whole prefetch
    uint32_t A0, B0, A1, B1;
    arms_blk(fs - R - 1, A0, B0);
    arms_blk(fs + RS - R - 1, A1, B1);
    // right-image arm of the trailing position, lane i = pixel t - d0 - i: the state before step fs
    uint32_t X = __builtin_amdgcn_raw_buffer_load_b32(rb, 4u * (uint32_t)(fs - R - 2 - d0 - lane), 0, 0);
#pragma unroll
    for (int j = 0; j < PF; j++)
        cr[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rc, dl4, (int)(D4 * (uint32_t)min(fs + j, W - 1)),
                                                                               CBCA_NT & 1 ? 2 : 0));
    cb_p P = 0.0;
    sP[(RS - 1) * 64 + lane] = 0.0;               // P(fs - 1) = 0: read before position fs + RS - 1 lands
    // per-lane store offset of output t (4d + 4tD), advanced every step
    uint32_t vst = 4u * (uint32_t)d + D4 * (uint32_t)(fs - R - 1);

    // step j of a block at front f; CLAMP: prefetch positions may pass the row end (tail blocks)
    auto step = [&](int j, int f, uint32_t Ab, uint32_t Bb, uint32_t &sld, bool clamp) {
        const int slot = j % PF;
        // trailing output t = f - R - 1: left-image arm (uniform) and the right-image arm chain;
        // its prefix reads before the front's write (slot j still holds position f - RS)
        const int t = f - R - 1;
        const uint32_t a = ruint(Ab, j);
        const uint32_t nb = ruint(Bb, j);
        X = (uint32_t)__builtin_amdgcn_update_dpp((int)nb, (int)X, 0x138, 0xF, 0xF, false);   // wave_shr:1, lane 0 <- nb
        const int hl = min(a & 255u, X & 255u), hr = min((a >> 8) & 255u, (X >> 8) & 255u);
        const uint32_t ib = ring_slot<RS>(j - R - 1 + hr), ia = ring_slot<RS>(j - R - 2 - hl);
        const cb_p pb = sP[ib * 64 + lane], pa = sP[ia * 64 + lane];
        __builtin_amdgcn_sched_barrier(0);   // (the reads' uses stay below the front's work)
        // front: the chain of this lane starts at max(t0 - M, d) >= fs
        const float cv = cr[slot];
        P += (!SEL || f >= d) ? (cb_p)cv : (cb_p)0.0;
        sP[j * 64 + lane] = P;
        const uint32_t so = clamp ? D4 * (uint32_t)min(f + PF, W - 1) : sld;
        cr[slot] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rc, dl4, (int)so, CBCA_NT & 1 ? 2 : 0));
        sld = opq_s(sld + D4);
        __builtin_amdgcn_sched_barrier(0);
        const float out = (float)(pb - pa);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, out), rd, t >= th ? vst : CB_OOB, 0,
                                              CBCA_NT & 2 ? 2 : 0);
        vst = opq_v(vst + D4);
    };
    // Blocks of RS steps.  The block arms alternate between two register pairs, each reloaded in
    // place at the end of the block it served with the arms of the block after next (issued a whole
    // block before use; no loop-carried copy of a register with a load in flight, which would wait
    // for it -- and, vmcnt retiring in order, drain the cost prefetch).  The first two blocks are
    // peeled and the loop runs two blocks per iteration, so the loop header merges steady-state
    // waits only.  Main blocks have every front and prefetch position inside the row; the tail
    // blocks clamp.
    int fb = fs;
    auto block = [&](uint32_t &Ap, uint32_t &Bp, bool clamp) {
        uint32_t sld = D4 * (uint32_t)(fb + PF);
#pragma unroll
        for (int j = 0; j < RS; j++)
            if (!clamp || fb + j <= fe) step(j, fb + j, Ap, Bp, sld, clamp);
        arms_blk(fb + 2 * RS - R - 1, Ap, Bp);
        fb += RS;
    };
    auto full = [&]() { return fb + RS - 1 <= fe && fb + RS - 1 + PF <= W - 1; };
    bool odd = false;
    if (full()) {
        block(A0, B0, false);
        odd = true;
        if (full()) {
            block(A1, B1, false);
            odd = false;
            while (full()) {
                block(A0, B0, false);
                if (!full()) {
                    odd = true;
                    break;
                }
                block(A1, B1, false);
            }
        }
    }
    while (fb <= fe) {
        if (odd) block(A1, B1, true);
        else block(A0, B0, true);
        odd = !odd;
    }
}

template <int R>
__global__ __launch_bounds__(64, 3) void cbca_h_kernel(const CbcaArgs A)
{
    __shared__ cb_p sP[(2 * R + 2) * 64];
    for (int64_t it = blockIdx.x; it < A.nitems; it += gridDim.x) {
        const int k = (int)(it / A.nper);
        const int64_t r = it - (int64_t)k * A.nper;
        const int c = (int)(r % A.ndc);
        if (k * SDE_CBCA_SEG - A.M >= 64 * c + 63)    // fs = max(t0 - M, d0) >= every lane's d
            cbca_h_item<R, false>(A, (int)(r / A.ndc), c, k, sP);
        else
            cbca_h_item<R, true>(A, (int)(r / A.ndc), c, k, sP);
    }
}

// Vertical-pass launch shape: WPB waves per workgroup, each with its own items and LDS rings; R = 13
// (L1 <= 14) adds a workgroup-shared table of the exact reciprocals 1/c, c <= (2R+1)^2 (one LDS
// read per voxel for the v_rcp_f64 + Newton chain; 4 waves x 17.5 KB + 5.7 KB: still two workgroups
// = 8 waves per CU).
template <int R> struct CbV {
    static constexpr int WPB = R == 13 ? 4 : 1;
    static constexpr bool TAB = R == 13;
    static constexpr int NT = TAB ? (2 * R + 1) * (2 * R + 1) + 1 : 1;
};

// ---------------------------------------------------------------------------------------------
// Vertical pass: item = (segment k, column x, chunk c <= x / 64), c fastest (only chunks with a
// valid lane are items); wave w takes items w, w + G, ...: the waves in flight walk the same rows
// of consecutive columns, so each row step reads whole pixels side by side.
// ---------------------------------------------------------------------------------------------
template <int R>
__device__ __forceinline__ void cbca_v_item(const CbcaArgs &A, int x, int c, int k, cb_p *__restrict__ sP,
                                            uint16_t *__restrict__ sN, const cb_r *__restrict__ tab)
{
    constexpr int RS = 2 * R + 2, PF = RS, U = R + 1;
    static_assert(RS % U == 0, "ring sizes");
    const int lane = threadIdx.x & 63;
    const int H = A.H, W = A.W, D = A.D, M = A.M, Hp = A.Hp;
    const int d0 = 64 * c, d = d0 + lane;
    const int t0 = k * SDE_CBCA_SEG, t1 = min(t0 + SDE_CBCA_SEG, H);
    const int fc = max(t0 - M, 0);               // chain base (every valid lane)
    const int fs = fc & ~3;                      // walk start: 16-B aligned dwordx4 of four rows
    const int fe = t1 + R;                       // outputs trail the front by R + 1 (as horizontally)
    const bool lane_ok = d < D && d <= x;
    const uint32_t dl4 = 4u * (uint32_t)min(d, D - 1);
    const uint32_t rowv = 4u * (uint32_t)W * (uint32_t)D;       // one row of the volume
    // descriptors over the column, rebased on row fbase (loads) / fb - R - 1 (stores) every block, their
    // ranges covering the rows a block touches (< 2^31 bytes: the shape check)
    const uint32_t win = (uint32_t)(RS + PF + R + 1) * rowv;
    const __amdgpu_buffer_rsrc_t ra = cb_rsrc(A.alT + (size_t)x * Hp, 4u * (uint32_t)Hp);
    // right-image arms from the ROW-major copy: at a row, lane d reads column x - d, so the wave's
    // 64 lanes read 64 adjacent words (one 256-B run) -- the column-major copy made every dwordx4
    // a gather of 64 cache lines
    const __amdgpu_buffer_rsrc_t rb = cb_rsrc(A.ar, 4u * (uint32_t)W * (uint32_t)H);
    const uint32_t bcol = lane_ok ? 4u * (uint32_t)(x - d) : CB_OOB;

    float cr[PF];
    uint32_t Bq[RS];             // right-image arm of row fb + j (per lane); slot j is reloaded with
                                 // the next block's row once step j has used it
    uint32_t A0, A1;             // left-image arm of row fb + lane (lanes < RS), pairs by block parity
    uint32_t sup[U];             // (vu | vd << 16) of the last U front positions
    auto arm_r = [&](int row) {  // row `row` of the right image at x - d (rows past H read 0)
        const uint32_t off = bcol == CB_OOB ? CB_OOB : bcol + 4u * (uint32_t)W * (uint32_t)row;
        return __builtin_amdgcn_raw_buffer_load_b32(rb, off, 0, 0);
    };
    // the arms first: loop-carried registers loaded after the cost prefetch would make the entry
    // path's waits for them (merged into every block start) drain the whole prefetch
    A0 = __builtin_amdgcn_raw_buffer_load_b32(ra, 4u * (uint32_t)(fs + lane), 0, 0);
    A1 = __builtin_amdgcn_raw_buffer_load_b32(ra, 4u * (uint32_t)(fs + RS + lane), 0, 0);
#pragma unroll
    for (int m = 0; m < RS; m++) Bq[m] = arm_r(fs + m);
    {
        const __amdgpu_buffer_rsrc_t rc0 = cb_rsrc(A.src + ((size_t)fs * W + x) * D, win);
#pragma unroll
        for (int j = 0; j < PF; j++)
            cr[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                  rc0, dl4, (int)(rowv * (uint32_t)(min(fs + j, H - 1) - fs)), CBCA_NT & 1 ? 2 : 0));
    }
#pragma unroll
    for (int j = 0; j < U; j++) sup[j] = 0u;
    cb_p P = 0.0;
    uint32_t N = 0;
    sP[(RS - 1) * 64 + lane] = 0.0;               // Q(fs - 1) = 0, N(fs - 1) = 0
    // count ring: lane l's u16 sits at (l % 32) * 2 + l / 32 of its slot row, so a 32-lane half
    // touches 32 different dwords of one row -- distinct banks whatever slot each lane reads (the
    // straight [slot][lane] layout put lanes 2k and 2k+1 in one bank: 2-way conflicts)
    const int ln = ((lane & 31) << 1) | (lane >> 5);
    sN[(RS - 1) * 64 + ln] = 0;

    // step j of a block at front f; loads address rows relative to fbase, stores relative to fb - R - 1
    // PRE: the walk's first block (its first fc - fs <= 3 positions precede the chain)
    auto step = [&](int j, int f, int fbase, uint32_t Ab, __amdgpu_buffer_rsrc_t rc, __amdgpu_buffer_rsrc_t rd,
                    uint32_t &sld, uint32_t &sst, bool clamp, bool pre) {
        const int slot = j % PF;
        // trailing output t = f - R - 1: its support from the ring slot of position t (the front
        // overwrites it below), its prefix / count reads before the front's writes
        const int t = f - R - 1;
        const uint32_t sy = sup[j % U];
        // the halves unpacked by opaque instructions: folded into SDWA adds, every step's slot
        // constant became a VGPR held across the loop (~70 registers)
        // (R = 31 keeps the plain form: with the asm its SGPR pressure forces an illegal VGPR-to-SGPR
        // copy in the compiler)
        uint32_t vu_u = sy & 0xFFFFu, vd_u = sy >> 16;
        if (R <= 15) {
            asm("v_and_b32 %0, 0xffff, %1" : "=v"(vu_u) : "v"(sy));
            asm("v_lshrrev_b32 %0, 16, %1" : "=v"(vd_u) : "v"(sy));
        }
        const int vu = (int)vu_u, vd = (int)vd_u;
        const uint32_t ib = ring_slot<RS>(j - R - 1 + vd), ia = ring_slot<RS>(j - R - 2 - vu);
        const cb_p pb = sP[ib * 64 + lane], pa = sP[ia * 64 + lane];
        const uint16_t nb = sN[ib * 64 + ln], na = sN[ia * 64 + ln];
        __builtin_amdgcn_sched_barrier(0);   // (the reads' uses stay below the front's work)
        // front f: chain (rows >= fc), count contribution and vertical support
        const uint32_t a = ruint(Ab, j);
        const uint32_t bw = Bq[j];
        const uint32_t a02 = a & 0x00FF00FFu, a13 = (a >> 8) & 0x00FF00FFu;
        const uint32_t b02 = bw & 0x00FF00FFu, b13 = (bw >> 8) & 0x00FF00FFu;
        // per 16-bit half: (min l, min u) and (min r, min d)
        const uint32_t m02 = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a02),
                                                                                    __builtin_bit_cast(u16x2, b02)));
        const uint32_t m13 = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a13),
                                                                                    __builtin_bit_cast(u16x2, b13)));
        const bool on = !pre || f >= fc;
        P += on ? (cb_p)cr[slot] : (cb_p)0.0;
        N += on ? ((m02 + m13) & 0xFFFFu) + 1u : 0u;
        sP[j * 64 + lane] = P;
        sN[j * 64 + ln] = (uint16_t)N;
        sup[j % U] = (m02 >> 16) | (m13 & 0xFFFF0000u);
        Bq[j] = arm_r(f + RS);                              // the next block's row
        const uint32_t so = clamp ? rowv * (uint32_t)(min(f + PF, H - 1) - fbase) : sld;
        cr[slot] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rc, dl4, (int)so, CBCA_NT & 1 ? 2 : 0));
        sld = opq_s(sld + rowv);
        __builtin_amdgcn_sched_barrier(0);
        // the output (row t = f - R - 1: soffset j rows on the block's store descriptor)
        const cb_p num = pb - pa;
        const uint32_t cnt = (uint16_t)(nb - na);
        // (an invalid lane's count may be anything: clamped into the table)
        const cb_r rcp = CbV<R>::TAB ? tab[min(cnt, (uint32_t)CbV<R>::NT - 1)] : (cb_r)cb_recip(cnt);
        const float out = (float)(num * rcp);
        const uint32_t vo = (lane_ok && t >= t0) ? 4u * (uint32_t)d : CB_OOB;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, out), rd, vo, (int)sst, CBCA_NT & 2 ? 2 : 0);
        sst = opq_s(sst + rowv);
    };
    int fb = fs;
    // blocks as in the horizontal pass: two alternating left-arm registers reloaded in place, the
    // first two blocks peeled, two blocks per loop iteration, clamped tail blocks
    auto block = [&](uint32_t &Ap, bool clamp, bool pre) {
        // loads for positions fb + PF .. go against a descriptor rebased on row fbase (a tail block
        // may start past the last row), stores against one rebased on row fb - R - 1
        const int fbase = clamp ? min(fb, H - 1) : fb;
        const __amdgpu_buffer_rsrc_t rc = cb_rsrc(A.src + ((size_t)fbase * W + x) * D, win);
        const __amdgpu_buffer_rsrc_t rd = cb_rsrc(A.dst + ((size_t)(fb - R - 1) * W + x) * D, win);
        uint32_t sld = rowv * (uint32_t)PF, sst = 0;
#pragma unroll
        for (int j = 0; j < RS; j++)
            if (!clamp || fb + j <= fe) step(j, fb + j, fbase, Ap, rc, rd, sld, sst, clamp, pre);
        Ap = __builtin_amdgcn_raw_buffer_load_b32(ra, 4u * (uint32_t)(fb + 2 * RS + lane), 0, 0);
        fb += RS;
    };
    auto full = [&]() { return fb + RS - 1 <= fe && fb + RS - 1 + PF <= H - 1; };
    bool odd = false;
    if (full()) {
        block(A0, false, true);
        odd = true;
        if (full()) {
            block(A1, false, false);
            odd = false;
            while (full()) {
                block(A0, false, false);
                if (!full()) {
                    odd = true;
                    break;
                }
                block(A1, false, false);
            }
        }
    }
    while (fb <= fe) {
        if (odd) block(A1, true, fb == fs);
        else block(A0, true, fb == fs);
        odd = !odd;
    }
}

template <int R>
__global__ __launch_bounds__(64 * CbV<R>::WPB, 2) void cbca_v_kernel(const CbcaArgs A)
{
    constexpr int WPB = CbV<R>::WPB;
    __shared__ cb_p sP[WPB][(2 * R + 2) * 64];
    __shared__ uint16_t sN[WPB][(2 * R + 2) * 64];
    __shared__ cb_r tab[CbV<R>::NT];
    const int wave = WPB > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
    if (CbV<R>::TAB) {
        for (int c = threadIdx.x; c < CbV<R>::NT; c += 64 * WPB) tab[c] = (cb_r)cb_recip((uint32_t)max(c, 1));
        __syncthreads();
    }
    for (int64_t it = (int64_t)blockIdx.x * WPB + wave; it < A.nitems; it += (int64_t)gridDim.x * WPB) {
        const int k = (int)(it / A.nper);
        int64_t r = it - (int64_t)k * A.nper;
        // columns [64(m-1), 64m) hold m valid chunks (m < ndc), the rest ndc
        int x = -1, c = 0;
        for (int m = 1; m < A.ndc; m++) {
            const int64_t n = (int64_t)max(0, min(64, A.W - 64 * (m - 1))) * m;
            if (r < n) {
                x = 64 * (m - 1) + (int)(r / m);
                c = (int)(r % m);
                break;
            }
            r -= n;
        }
        if (x < 0) {
            x = 64 * (A.ndc - 1) + (int)(r / A.ndc);
            c = (int)(r % A.ndc);
        }
        cbca_v_item<R>(A, x, c, k, sP[wave], sN[wave], tab);
    }
}

// ---------------------------------------------------------------------------------------------
// Per-disparity rotation of the rows: out(y, x, d) = in(y, (x + s*d) mod W, d).  s = +1 with
// VALID_ONLY: the shear of an aggregated left volume into the right one's valid voxels (x + d <
// W; the others untouched); s = -1 / +1 over every voxel: a right-referenced volume into left
// coordinates and back (its invalid voxels ride on the left-coordinate invalid ones).
// Tile = (row, RT_NP output pixels, RT_ND disparities): its sources form a parallelogram --
// source pixel r of the tile contributes the contiguous disparities whose outputs land in the
// tile -- so every source voxel is read by exactly one tile, as runs of <= RT_ND floats.  The
// tile is assembled in LDS as [pixel][d] (the runs' diagonal writes hit distinct banks, the
// output rows are read contiguously) and leaves as whole 256-B runs.  16-KB tiles: ten
// workgroups per CU, and each wave keeps its 16 loads of a batch in flight together.
// ---------------------------------------------------------------------------------------------
constexpr int RT_NP = 64, RT_ND = 64;
// S: the rotation's sign; WIDE: W >= 64 (a batch's pieces wrap the row at most once)
template <int S, bool WIDE>
__global__ __launch_bounds__(256) void cbca_rotate_kernel(const float *__restrict__ in, float *__restrict__ out, int H,
                                                          int W, int D, int valid_only, int64_t ntiles)
{
    __shared__ float rbuf[RT_NP * RT_ND + 64];   // + dump words for the lanes past a piece's run
    const int64_t tile = blockIdx.x;
    if (tile >= ntiles) return;
    const int nxs = (W + RT_NP - 1) / RT_NP, nds = (D + RT_ND - 1) / RT_ND;
    const int y = (int)(tile / ((int64_t)nxs * nds));
    const int rem = (int)(tile - (int64_t)y * nxs * nds);
    const int x0 = (rem / nds) * RT_NP, d0 = (rem % nds) * RT_ND;
    const int nd = min(RT_ND, D - d0);
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t rowbytes = 4u * (uint32_t)W * (uint32_t)D;
    const __amdgpu_buffer_rsrc_t ri = cb_rsrc(in + (size_t)y * W * D, rowbytes);
    const __amdgpu_buffer_rsrc_t ro = cb_rsrc(out + (size_t)y * W * D, rowbytes);
    // piece r (0 <= r < RT_NP + nd - 1): source pixel (x0 + base + r) mod W; output pixel p of relative
    // disparity e = d - d0 is p = r - e (S > 0) or p = r + e - (nd - 1) (S < 0)
    const int base = S > 0 ? d0 : -d0 - (nd - 1);
    const int np = RT_NP + nd - 1;
    constexpr int RB = 16;        // pieces per wave in flight: a batch's loads all issue before its LDS writes
    for (int r0 = wave; r0 < np; r0 += 4 * RB) {
        float v[RB];
        int at[RB];
        // source pixel of piece r0 in [0, W): one modulo per batch (scalar)
        int q0 = (x0 + base + r0) % W;
        if (q0 < 0) q0 += W;
        // the per-piece bookkeeping on the vector ALUs: as scalar code (one scalar unit per CU for
        // four SIMDs) it bound the kernel -- PMC 2.3e8 SALU instructions per launch
        int rv = r0, qv = q0;
        asm volatile("" : "+v"(rv), "+v"(qv));
#pragma unroll
        for (int b = 0; b < RB; b++) {
            const int r = rv + 4 * b;
            const int elo = S > 0 ? max(0, r - (RT_NP - 1)) : max(0, nd - 1 - r);
            const int ehi = S > 0 ? min(nd - 1, r) : min(nd - 1, nd - 1 - r + RT_NP - 1);
            const int e = elo + lane, d = d0 + e;
            const int p = S > 0 ? r - e : r + e - (nd - 1);
            const int x = x0 + p;
            int q = qv + 4 * b;
            if (WIDE) q = q >= W ? q - W : q;
            else q %= W;
            // the conditions as one signed minimum each (vector ops, no scalar mask algebra); the
            // offset computed before the select (not sunk into an exec-masked branch)
            const int in_m = min(ehi - e, np - 1 - r);                           // >= 0: inside the run
            const int ok_m = min(in_m, min(W - 1 - x, valid_only ? W - 1 - x - d : 0));
            uint32_t vraw = 4u * ((uint32_t)q * D + d);
            asm volatile("" : "+v"(vraw));
            v[b] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                 ri, ok_m >= 0 ? vraw : CB_OOB, 0, CBCA_NT & 1 ? 2 : 0));
            at[b] = in_m >= 0 ? p * RT_ND + e : RT_NP * RT_ND + lane;
        }
#pragma unroll
        for (int b = 0; b < RB; b++) rbuf[at[b]] = v[b];
    }
    __syncthreads();
    // output pixels x0 + p (wave w: pixels w, w + 4, ...), one run of nd floats each, WB per batch
    constexpr int WB = 8;
#pragma unroll
    for (int i0 = 0; i0 < RT_NP; i0 += 4 * WB) {
        float v[WB];
        uint32_t vo[WB];
#pragma unroll
        for (int b = 0; b < WB; b++) {
            const int p = i0 + 4 * b + wave, x = x0 + p, d = d0 + lane;
            const bool inr = x < W && lane < nd;
            v[b] = rbuf[p * RT_ND + lane];
            vo[b] = inr && (!valid_only || x + d < W) ? 4u * ((uint32_t)x * D + d) : CB_OOB;
        }
#pragma unroll
        for (int b = 0; b < WB; b++)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v[b]), ro, vo[b], 0, CBCA_NT & 2 ? 2 : 0);
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

static size_t cbca_ws_bytes(int H, int W) { return sizeof(uint32_t) * (size_t)cb_hp(H) * (size_t)W; }

// Resident workgroups of a pass kernel (occupancy x CUs), cached per device and kernel (`cache` is
// one slot per device id; a process driving GPUs with different CU counts sizes each grid for its own).
template <typename K>
static int cb_resident(std::atomic<int> (&cache)[64], K kernel, int threads = 64)
{
    int dev = 0, cus = 256, per = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    if (const int c = cache[dev].load(std::memory_order_relaxed)) return c;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, 0) != hipSuccess || per <= 0) per = 8;
    cache[dev].store(per * cus, std::memory_order_relaxed);
    return per * cus;
}

// Balanced static schedule: the fewest items per wave that fit the resident waves, then only as
// many waves as that needs (every wave gets the same count within one, so none idles long).
static int cb_grid(int64_t nitems, int resident)
{
    const int64_t per = std::max<int64_t>((nitems + resident - 1) / resident, 1);
    return (int)((nitems + per - 1) / per);
}

// One left-coordinate volume: iters x (horizontal src -> tmp, vertical tmp -> src), in place.
template <int R>
static void cbca_left_iters(float *cv, float *tmp, const uint32_t *al, const uint32_t *ar, const uint32_t *alT,
                            int H, int W, int D, int L1, int iters, hipStream_t st)
{
    CbcaArgs h{};
    h.al = al, h.ar = ar, h.alT = alT;
    h.H = H, h.W = W, h.D = D, h.M = L1 - 1, h.Hp = cb_hp(H);
    h.ndc = (D + 63) / 64;
    CbcaArgs v = h;
    h.nseg = (W + SDE_CBCA_SEG - 1) / SDE_CBCA_SEG;
    h.nper = (int64_t)H * h.ndc;
    h.nitems = h.nper * h.nseg;
    v.nseg = (H + SDE_CBCA_SEG - 1) / SDE_CBCA_SEG;
    v.nper = 0;
    for (int c = 0; c < v.ndc; c++) v.nper += (int64_t)max(W - 64 * c, 0);    // columns x >= 64c
    v.nitems = v.nper * v.nseg;
    static std::atomic<int> res_h[64], res_v[64];
    constexpr int VW = CbV<R>::WPB;
    const int gh = cb_grid(h.nitems, cb_resident(res_h, cbca_h_kernel<R>));
    const int gv = (cb_grid(v.nitems, cb_resident(res_v, cbca_v_kernel<R>, 64 * VW) * VW) + VW - 1) / VW;   // waves -> workgroups
    h.src = cv, h.dst = tmp;
    v.src = tmp, v.dst = cv;
    for (int it = 0; it < iters; it++) {
        if (h.nitems > 0) cbca_h_kernel<R><<<gh, 64, 0, st>>>(h);
        if (v.nitems > 0) cbca_v_kernel<R><<<gv, 64 * VW, 0, st>>>(v);
    }
}

static void cbca_rotate(const float *in, float *out, int H, int W, int D, int s, bool valid_only, hipStream_t st)
{
    const int64_t ntiles = (int64_t)H * ((W + RT_NP - 1) / RT_NP) * ((D + RT_ND - 1) / RT_ND);
    const int vo = valid_only ? 1 : 0;
    if (s > 0) {
        if (W >= 64) cbca_rotate_kernel<1, true><<<(unsigned)ntiles, 256, 0, st>>>(in, out, H, W, D, vo, ntiles);
        else cbca_rotate_kernel<1, false><<<(unsigned)ntiles, 256, 0, st>>>(in, out, H, W, D, vo, ntiles);
    } else {
        if (W >= 64) cbca_rotate_kernel<-1, true><<<(unsigned)ntiles, 256, 0, st>>>(in, out, H, W, D, vo, ntiles);
        else cbca_rotate_kernel<-1, false><<<(unsigned)ntiles, 256, 0, st>>>(in, out, H, W, D, vo, ntiles);
    }
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
    uint32_t *alT = (uint32_t *)ws;
    const dim3 tg((W + 31) / 32, (Hp + 31) / 32);
    cbca_transpose_kernel<<<tg, 256, 0, st>>>(al, alT, H, W, Hp);
    switch (cbca_r(L1)) {
    case 13: cbca_left_iters<13>(cv, tmp, al, ar, alT, H, W, D, L1, iters, st); break;
    case 15: cbca_left_iters<15>(cv, tmp, al, ar, alT, H, W, D, L1, iters, st); break;
    default: cbca_left_iters<31>(cv, tmp, al, ar, alT, H, W, D, L1, iters, st); break;
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
    // iters == 0 aggregates nothing but still defines cv_r as the shear of cv_l (as the oracle does)
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
