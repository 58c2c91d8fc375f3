// cbca.hip -- cross-based cost aggregation on [H][W][D] volumes (gfx950).
//
// BUILD-DEFINED stage: the reference has no CBCA (only the
// buffer name d_cost_volumel_after_aggr, process_functional.py:268,347, and an
// unused timer label, match.py:98).  The definition -- cross arms on intensity
// + distance, support intersected with the other image's arms at x -/+ d,
// horizontal-then-vertical sums, mean over the support, N iterations -- is
// stated once in the CPU restatement under oracle/ (test infrastructure); these
// kernels reproduce it bit for bit (fp32 sums in ascending offset order from
// 0.0f, exact integer counts, one IEEE division).
//
// Mapping.  Both passes are line scans: one wave (one workgroup) walks one
// line -- a row for the horizontal pass, a column for the vertical one -- for
// one chunk of 64 disparities (lane = d, so each step moves one 256-B
// contiguous run of the HWD volume).  The fp64 prefix sum P of the definition
// is the wave's running state; the last 2R+2 prefixes live in a wave-private
// LDS ring, so each output is two LDS reads at per-lane offsets (its own arms)
// and one subtraction: O(1) work per voxel whatever the arm lengths.  The
// output trails the front by R positions (its right/down arm is at most R).
// Cost values and both images' arms are prefetched 8 positions ahead in a
// register ring (unconditional, clamped loads), and the support arms of the
// last R + 1 positions stay in registers for the trailing output.
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

// Cache policy of the cost stream (aux bit 1 = nt on gfx950): 1 loads, 2 stores.  The volumes are
// streamed once per pass: nontemporal both ways, 1.513 -> 1.468 ms per pair iteration
// (tools/lib_variants.py; the arms stay cached -- every line re-reads them).
#ifndef CBCA_NT
#define CBCA_NT 3
#endif

// Buffer descriptor (wave-uniform inputs only) for raw dword loads/stores with a 32-bit
// per-lane voffset, an SGPR soffset and the hardware range check (voffset >= bytes -> 0 on
// load, dropped on store).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t cb_rsrc(const void *base, uint32_t bytes)
{
    const uintptr_t b = (uintptr_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    void *p = (void *)(((uintptr_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, 0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// One launch covers up to two volumes (grid.z): the left- and right-referenced volumes of a pair
// are independent, and one launch of both fills the machine in whole rounds of line-waves (a
// 1024^2 x 192 pass has 3072 line-waves per volume against 2048-2560 resident: alone, its second
// round runs half empty).
#ifndef CBCA_PF
#define CBCA_PF 16    // positions prefetched ahead (A/B builds: 8)
#endif
struct CbcaVolumes {
    const float *src[2];
    float *dst[2];
    const uint32_t *ref[2], *oth[2];
    int side[2];
};

// The scan of one line of one volume (SIDE compile-time: each launch holds both instantiations
// and picks one per workgroup).
template <int R, bool VERT, int SIDE>
__device__ __forceinline__ void cbca_scan(const float *__restrict__ src, float *__restrict__ dst,
                                          const uint32_t *__restrict__ ref, const uint32_t *__restrict__ oth,
                                          int H, int W, int D, double *__restrict__ sP, uint16_t *__restrict__ sN)
{
    constexpr int RS = 2 * R + 2;      // prefix ring: positions [f - 2R - 1, f]; also the unroll
    constexpr int U = R + 1;           // support ring (trailing output reads the slot of f - R)
    constexpr int PF = CBCA_PF;        // prefetch distance (vmcnt saturates at 63 outstanding ops)
    static_assert((RS & (RS - 1)) == 0 && RS % U == 0 && RS % PF == 0, "ring sizes");
    const int lane = threadIdx.x;
    // Lanes past D work on d = D-1: they compute lane D-1's value and store it to the
    // same address, so no load, LDS access or store in the scan is predicated.
    const int d = min((int)blockIdx.x * 64 + lane, D - 1);
    const int line = blockIdx.y;
    const int len = VERT ? H : W;
    // Addressing (all per-step offsets in SGPRs, per-lane parts fixed):
    //  H pass (line = row y): cost/out buffers over the row, voffset 4d, soffset 4qD; reference
    //   arms: voffset 0, soffset 4q; other arms: voffset 4(q -/+ d) -- outside the row it fails
    //   the range check and reads 0, i.e. "no other pixel: support {p}".
    //  V pass (line = column x): cost/out buffers rebased every RS rows (a column spans
    //   H*W*D*4 bytes, beyond 32-bit offsets), voffset 4d, soffset 4(q - q0)WD; arms: voffset 0 /
    //   4(x -/+ d) (masked when outside the row), soffset 4qW.
    const uint32_t d4 = 4u * d;
    // opaque per-lane zero for the (wave-uniform) reference-arm loads: keeps their value a VGPR,
    // so no readfirstlane (and no wait for it) lands on every step
    const uint32_t vz = __builtin_amdgcn_mbcnt_lo(0u, 0u);
    const int ov = SIDE == SDE_SIDE_LEFT ? line - d : line + d;
    const bool vok = ov >= 0 && ov < W;
    const uint32_t ov4 = 4u * (uint32_t)(vok ? ov : 0);
    const uint32_t linebytes = 4u * (uint32_t)W * (uint32_t)D;       // one row of the volume
    __amdgpu_buffer_rsrc_t rc, rd;
    __amdgpu_buffer_rsrc_t ra = cb_rsrc(ref + (VERT ? (size_t)line : (size_t)line * W), VERT ? 0xffffffffu : 4u * W);
    __amdgpu_buffer_rsrc_t rb = cb_rsrc(oth + (VERT ? 0 : (size_t)line * W), VERT ? 0xffffffffu : 4u * W);
    if (!VERT) {
        rc = cb_rsrc(src + (size_t)line * W * D, linebytes);
        rd = cb_rsrc(dst + (size_t)line * W * D, linebytes);
    }

    double P_acc = 0.0;
    uint32_t N_acc = 0;
    float cr[PF];
    uint32_t ar[PF], br[PF];
    uint32_t sup[U];    // VERT: (up | down << 8) of the last U positions; else (left | right << 8)
    // q: position (clamped by the caller in the tail); qb: the V pass's current rebase row
    auto issue = [&](int q, int qb, int slot) {
        if (VERT) {
            cr[slot] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                     rc, d4, (int)((uint32_t)(q - qb) * linebytes), CBCA_NT & 1 ? 2 : 0));
            ar[slot] = __builtin_amdgcn_raw_buffer_load_b32(ra, vz, 4 * q * W, 0);
            br[slot] = __builtin_amdgcn_raw_buffer_load_b32(rb, ov4, 4 * q * W, 0);
        } else {
            cr[slot] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rc, d4, 4 * q * D, CBCA_NT & 1 ? 2 : 0));
            ar[slot] = __builtin_amdgcn_raw_buffer_load_b32(ra, vz, 4 * q, 0);
            uint32_t o4 = SIDE == SDE_SIDE_LEFT ? 4u * (uint32_t)q - d4 : 4u * (uint32_t)q + d4;
            // opaque: the whole offset must reach the range check as voffset.  Left to itself the
            // compiler moves the step's constant part of q into the instruction offset, and a
            // voffset that wrapped below zero (x - d < 0 at the block start, >= 0 at this step)
            // then fails the check and reads 0 for a pixel inside the row.
            asm volatile("" : "+v"(o4));
            br[slot] = __builtin_amdgcn_raw_buffer_load_b32(rb, o4, 0, 0);
        }
    };
    auto step = [&](int j, int f, int qb, bool tail) {
        const int slot = j % PF;
        const uint32_t a = ar[slot];
        uint32_t b = br[slot];
        if (VERT) b = vok ? b : 0u;                 // no other pixel: support {p}
        const int l = min(a & 255, b & 255), r = min((a >> 8) & 255, (b >> 8) & 255);
        // front: position f (tail positions >= len re-read the last one; never referenced)
        P_acc += (double)cr[slot];
        sP[j * 64 + lane] = P_acc;
        if (VERT) {
            N_acc += (uint32_t)(l + r + 1);
            sN[j * 64 + lane] = (uint16_t)N_acc;
            sup[j % U] = min((a >> 16) & 255, (b >> 16) & 255) | (min(a >> 24, b >> 24) << 8);
        } else {
            sup[j % U] = (uint32_t)l | ((uint32_t)r << 8);
        }
        const int qn = tail ? min(f + PF, len - 1) : f + PF;
        issue(qn, qb, slot);
        // trailing output y = f - R; its support arms from the ring slot of position y
        const int y = f - R;
        if (y >= 0 && (!tail || y < len)) {
            const uint32_t sy = sup[(j + 1) % U];
            const int lo = sy & 255, hi = sy >> 8;
            const int ib = ((j - R + hi) & (RS - 1)) * 64 + lane, ia = ((j - R - lo - 1) & (RS - 1)) * 64 + lane;
            const double pb = sP[ib], pa = sP[ia];
            float out;
            if (VERT) out = (float)((pb - pa) / (double)(uint16_t)(sN[ib] - sN[ia]));
            else out = (float)(pb - pa);
            const int so = VERT ? (int)((uint32_t)(y - qb) * linebytes) : 4 * y * D;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, out), rd, d4, so, CBCA_NT & 2 ? 2 : 0);
        }
    };
    // V pass: (re)base the cost / output descriptors on row qb; soffsets then stay below
    // (2 RS + PF) rows of the volume
    auto rebase = [&](int qb) {
        if (VERT) {
            const size_t off = (size_t)qb * W * D + (size_t)line * D;
            rc = cb_rsrc(src + off, 0xffffffffu);
            rd = cb_rsrc(dst + off, 0xffffffffu);
        }
    };
    // V pass: the descriptors are rebased on row qb = f0 - R at every block start, so a block's
    // outputs (rows f0 - R ..) and loads (rows up to f0 + RS + PF) sit at small soffsets; loads
    // already in flight keep the addresses they were issued with.
    rebase(-R);
#pragma unroll
    for (int j = 0; j < PF; j++) issue(min(j, len - 1), -R, j);
#pragma unroll
    for (int j = 0; j < U; j++) sup[j] = 0u;
    sP[(RS - 1) * 64 + lane] = 0.0;        // P(-1) = 0 (slot of position -1; rewritten at f = RS-1)
    if (VERT) sN[(RS - 1) * 64 + lane] = 0;
    int f0 = 0;
    // main blocks: every prefetched position is inside the line (no clamps)
    for (; f0 + RS + PF <= len; f0 += RS) {
        const int qb = f0 - R;
        rebase(qb);
#pragma unroll
        for (int j = 0; j < RS; j++) step(j, f0 + j, qb, false);
    }
    for (; f0 < len + R; f0 += RS) {
        const int qb = f0 - R;
        rebase(qb);
#pragma unroll
        for (int j = 0; j < RS; j++) step(j, f0 + j, qb, true);
    }
}

template <int R, bool VERT>
__global__ __launch_bounds__(64) void cbca_scan_kernel(const CbcaVolumes vols, int H, int W, int D)
{
    constexpr int RS = 2 * R + 2;
    __shared__ double sP[RS * 64];
    // support-count prefixes mod 2^16: a support holds at most (2R+1)^2 < 2^16 pixels, so the
    // difference of two ring entries taken mod 2^16 is the exact count (half the LDS of int32:
    // more line-waves per CU)
    static_assert((2 * R + 1) * (2 * R + 1) < 65536, "support counts must fit 16 bits");
    __shared__ uint16_t sN[VERT ? RS * 64 : 1];
    const int z = blockIdx.z;
    if (vols.side[z] == SDE_SIDE_LEFT)
        cbca_scan<R, VERT, SDE_SIDE_LEFT>(vols.src[z], vols.dst[z], vols.ref[z], vols.oth[z], H, W, D, sP, sN);
    else
        cbca_scan<R, VERT, SDE_SIDE_RIGHT>(vols.src[z], vols.dst[z], vols.ref[z], vols.oth[z], H, W, D, sP, sN);
}

template <int R>
static void cbca_iters(const CbcaVolumes &fwd, const CbcaVolumes &bwd, int nvol, int H, int W, int D, int iters,
                       hipStream_t st)
{
    const int ndc = (D + 63) / 64;
    for (int it = 0; it < iters; it++) {
        cbca_scan_kernel<R, false><<<dim3(ndc, H, nvol), 64, 0, st>>>(fwd, H, W, D);
        cbca_scan_kernel<R, true><<<dim3(ndc, W, nvol), 64, 0, st>>>(bwd, H, W, D);
    }
}

// The scans address with 32-bit buffer offsets (signed soffsets): the H pass reaches 4*W*D bytes
// into a row and the V pass (q - qb) <= 3R + 17 rows of 4*W*D bytes past its rebase row (loads
// prefetched PF = 16 positions ahead of a 2R+2 block that starts R rows after qb); the V pass's
// arm loads reach 4*H*W bytes.  Beyond that an offset would wrap silently (the column
// descriptors carry no range limit), so such shapes are refused.
static bool cbca_shape_ok(int H, int W, int D, int L1)
{
    if (H > 65535 || W > 65535) return false;            // grid.y = lines
    const int R = L1 <= 16 ? 15 : 31;
    const int64_t row = 4 * (int64_t)W * D;
    return (3 * R + 18) * row < ((int64_t)1 << 31) && 4 * (int64_t)H * W < ((int64_t)1 << 31);
}

// fwd: horizontal pass cv -> tmp; bwd: vertical pass tmp -> cv
static int cbca_launch(float *const cv[2], float *const tmp[2], const uint32_t *const ref[2],
                       const uint32_t *const oth[2], const int side[2], int nvol, int H, int W, int D, int L1,
                       int iters, hipStream_t st)
{
    CbcaVolumes fwd{}, bwd{};
    for (int k = 0; k < nvol; k++) {
        fwd.src[k] = cv[k], fwd.dst[k] = tmp[k];
        bwd.src[k] = tmp[k], bwd.dst[k] = cv[k];
        fwd.ref[k] = bwd.ref[k] = ref[k];
        fwd.oth[k] = bwd.oth[k] = oth[k];
        fwd.side[k] = bwd.side[k] = side[k];
    }
    if (L1 <= 16) cbca_iters<15>(fwd, bwd, nvol, H, W, D, iters, st);
    else cbca_iters<31>(fwd, bwd, nvol, H, W, D, iters, st);
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

SDE_EXPORT int sde_cbca(float *cv, float *tmp, const uint32_t *arms_ref, const uint32_t *arms_other, int H, int W,
                        int D, int side, int L1, int iters, void *stream)
{
    if (!cv || !tmp || !arms_ref || !arms_other || H <= 0 || W <= 0 || D <= 0 || iters < 0 || L1 < 1 ||
        L1 > SDE_CBCA_MAX_L1 || (side != SDE_SIDE_LEFT && side != SDE_SIDE_RIGHT) || cv == tmp)
        return SDE_ERR_ARG;
    if (!cbca_shape_ok(H, W, D, L1)) return SDE_ERR_ARG;
    float *const cvs[2] = {cv, nullptr}, *const tmps[2] = {tmp, nullptr};
    const uint32_t *const refs[2] = {arms_ref, nullptr}, *const oths[2] = {arms_other, nullptr};
    const int sides[2] = {side, side};
    return cbca_launch(cvs, tmps, refs, oths, sides, 1, H, W, D, L1, iters, as_stream(stream));
}

SDE_EXPORT int sde_cbca_pair(float *cv_l, float *tmp_l, float *cv_r, float *tmp_r, const uint32_t *arms_l,
                             const uint32_t *arms_r, int H, int W, int D, int L1, int iters, void *stream)
{
    if (!cv_l || !tmp_l || !cv_r || !tmp_r || !arms_l || !arms_r || H <= 0 || W <= 0 || D <= 0 || iters < 0 ||
        L1 < 1 || L1 > SDE_CBCA_MAX_L1)
        return SDE_ERR_ARG;
    // four distinct buffers: each volume's passes run concurrently with the other's
    const float *b[4] = {cv_l, tmp_l, cv_r, tmp_r};
    for (int i = 0; i < 4; i++)
        for (int j = i + 1; j < 4; j++)
            if (b[i] == b[j]) return SDE_ERR_ARG;
    if (!cbca_shape_ok(H, W, D, L1)) return SDE_ERR_ARG;
    float *const cvs[2] = {cv_l, cv_r}, *const tmps[2] = {tmp_l, tmp_r};
    const uint32_t *const refs[2] = {arms_l, arms_r}, *const oths[2] = {arms_r, arms_l};
    const int sides[2] = {SDE_SIDE_LEFT, SDE_SIDE_RIGHT};
    return cbca_launch(cvs, tmps, refs, oths, sides, 2, H, W, D, L1, iters, as_stream(stream));
}
