// sgm_probe.hip -- PROBE COPY of scenedepthestimation_amd/csrc/sgm.hip with timing switches.  Never part of libsde.so.
// SGM_GAP = N: what sits between two passes of the pair (tools/sgm_gap_probe.py).
// SGM_SKEW = n > 0: line l's wave sleeps (l % SGM_SKEW_K) x n x 64 cycles before its first step, so the
// 2048 concurrent line streams of a pass do not walk their rows in lock step (tools/sgm_skew_probe.py).
// Build: SRC=tools/variants/sgm_probe.hip bash tools/build_file_variant.sh sgm.hip NAME -DSGM_GAP=N / -DSGM_SKEW=n.
// sgm.hip -- semi-global matching and the GPU path's post-processing (gfx950).
//
// Replaces (process_functional.py):
//   sgm_penelty_kernel                :134-262
//   SGM_Interation + 8 SGM_*_kernel   :265-797  (launch order :1166-1203)
//   is_error_match_kernel / LRC_kernel :977-1088
//   Median_Filter_kernel               :840-879
//
// SGM recurrence, exactly as the reference computes it (Numba unifies the 1.0
// initialisers with the f32 loads, so the path state is float64):
//   L(p,d) = C(p,d)                                            first pixel / wrap restart
//   L(p,d) = C(p,d) + (min(L'(d), L'(d-1)+P1, L'(d+1)+P1, m'+P2') - m')   otherwise
//   S(p,d) = f32(f64(S(p,d)) + L(p,d));   m = min_d L(p,d)
// with P1 from the previous pixel's penalty channel, P2' read at the previous
// step, out-of-range neighbours (d = 0, D-1) dropped, n-1 pixels per line of n
// (>= 2), and diagonal lines wrapping around the image with a path restart.
//
// Mapping: one wave64 (one workgroup) per scanline and image side, so the line,
// the pixel sequence and the penalty addresses are wave-uniform (scalar loads).
// Lane l owns DPL = ceil(D/64) consecutive disparities d = l*DPL + i in
// registers: d-1 / d+1 cross a lane only at i = 0 / DPL-1 (one DPP wave_shr /
// wave_shl per fp64 half), and min_d is a DPP butterfly (quad_perm, row_ror,
// row_bcast) ending in one readlane -- no LDS round trips on the serial chain.
// Each step's C and S rows (DPL floats per lane, one dwordx{DPL} load each,
// addresses clamped so no load is predicated) are prefetched PF steps ahead in
// a register ring, so HBM latency overlaps the sequential DP.  The left and
// right image sides (the reference's k loop) run in the same launch (grid.y).
#include "sde_common.h"

// The cost and S streams are touched once per pass: nontemporal loads and stores (1 | 2).  Both
// together: 6.44 -> 5.96 ms for the 7-launch pair (either alone: no change; tools/sgm_variants.py).
#ifndef SGM_NT
#define SGM_NT 3
#endif
// Fused WTA bookkeeping: 1 parks each step's S values in LDS and scans a pixel's D values in d
// order spread over the next block's steps (no per-step lane-local argmin, no index tie-breaks
// until the G-lane DPP merge); 0 the round-3 lane-partial form (A/B builds).
#ifndef SGM_WTA_PARK
#define SGM_WTA_PARK 1
#endif

#ifndef SGM_SKEW
#define SGM_SKEW 0
#endif
#ifndef SGM_SKEW_K
#define SGM_SKEW_K 8
#endif
namespace sde {

// direction table in the reference launch order: step (dr, dc) and P1 channel
__constant__ int c_dir_dr[8] = {+1, -1, 0, 0, +1, -1, +1, -1};
__constant__ int c_dir_dc[8] = {0, 0, +1, -1, +1, +1, -1, -1};
__constant__ int c_dir_ch[8] = {2, 0, 6, 4, 10, 12, 8, 14};

struct PathGeom {
    int dr, dc, ch, H, W, n;
};

// k-th pixel of scanline `line`; restart = first pixel or diagonal wrap.
__device__ __forceinline__ void path_pixel(const PathGeom &g, int line, int k, int &r, int &c, bool &restart)
{
    restart = (k == 0);
    if (g.dc == 0) {                       // vertical: line = column
        c = line;
        r = g.dr > 0 ? k : g.H - 1 - k;
    } else if (g.dr == 0) {                // horizontal: line = row
        r = line;
        c = g.dc > 0 ? k : g.W - 1 - k;
    } else {                               // diagonal: line = start column, wraps
        r = g.dr > 0 ? k : g.H - 1 - k;
        if (g.dc > 0) {
            c = (int)(((int64_t)line + k) % g.W);
            if (k > 0 && c == 0) restart = true;
        } else {
            int64_t cc = ((int64_t)line - k) % g.W;
            if (cc < 0) cc += g.W;
            c = (int)cc;
            if (k > 0 && c == g.W - 1) restart = true;
        }
    }
}

template <int N>
struct alignas(4) FVec {
    float v[N];
};

// DPP move of a double (two 32-bit halves); lanes outside ROW_MASK keep `v`.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ double dpp_f64(double v)
{
    const long long b = __builtin_bit_cast(long long, v);
    int lo = (int)b, hi = (int)(b >> 32);
    lo = __builtin_amdgcn_update_dpp(lo, lo, CTRL, ROW_MASK, 0xF, false);
    hi = __builtin_amdgcn_update_dpp(hi, hi, CTRL, ROW_MASK, 0xF, false);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

// DPP move of a double for reductions whose disabled lanes are never read: no `old` operand, so
// the compiler emits the two v_mov_b32_dpp into fresh registers (dpp_f64's old = v costs two
// v_mov copies per stage).  Lanes outside ROW_MASK hold unspecified values.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ double dpp_f64_nold(double v)
{
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, ROW_MASK, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, ROW_MASK, 0xF, false);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

// t < a ? t : a.  VMIN: one v_min_f64 instead of a compare and two selects.  The two differ
// only when a is NaN or both are zeros of opposite signs.  In the fast recurrence no operand
// is NaN (non-finite costs and penalties take the faithful path), and a zero's sign never
// changes a magnitude downstream (x + -0 = x + +0 for x != 0; comparisons ignore it): it can
// reach S only through S + L with S = -0, and S is never -0 unless the caller's accumulate
// input holds one -- so the callers that accumulate onto a caller's S keep the selects.
template <bool VMIN = false>
__device__ __forceinline__ double dmin(double a, double t)
{
    if (VMIN) {
        double r;
        asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(t), "v"(a));
        return r;
    }
    return t < a ? t : a;
}

// min over the 64 lanes, returned wave-uniform.  Only lane 63 is read: stages 1-4 move within
// rows (every lane valid); stage 5 updates rows 1 and 3 from lanes 15 and 47, stage 6 row 3 from
// lane 31 (row 1, valid after stage 5) -- the rows a stage leaves out hold unspecified values
// and never feed lane 63, so the moves need no `old` operand.
template <bool VMIN = false>
__device__ __forceinline__ double wave_min_f64(double v)
{
    v = dmin<VMIN>(v, dpp_f64_nold<0xB1>(v));          // quad_perm [1,0,3,2]
    v = dmin<VMIN>(v, dpp_f64_nold<0x4E>(v));          // quad_perm [2,3,0,1]
    v = dmin<VMIN>(v, dpp_f64_nold<0x124>(v));         // row_ror:4
    v = dmin<VMIN>(v, dpp_f64_nold<0x128>(v));         // row_ror:8   -> every lane holds its row's min
    v = dmin<VMIN>(v, dpp_f64_nold<0x142, 0xA>(v));    // row_bcast:15 -> rows 1, 3
    v = dmin<VMIN>(v, dpp_f64_nold<0x143, 0xC>(v));    // row_bcast:31 -> row 3 holds all four
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_readlane((int)b, 63);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

// ---------------------------------------------------------------------------
// Non-finite costs.  The fast recurrence above (min chain in any order, one wave-wide minimum)
// equals the reference's for finite costs: its minima are then plain minima.  With NaN / inf in
// the costs the reference's exact arithmetic decides where they propagate (SGM_Interation,
// process_functional.py:265-343): Numba's binary min(a, b) = b if b < a else a (a NaN first
// argument sticks, a NaN second one is ignored), the chain
//   c += min(min(L(d-1) + P1, L(d)), min(L(d+1) + P1, mcP2)) - mc
// with L(d-1) := L(d) at d = 0 and L(d+1) := L(d) at d = D-1, and the minimum kept PER
// reference lane of 4 disparities: min(min(c1, c2), min(c3, c4)), then an xor butterfly
// min(m, shfl_xor(m, k)), k = 1, 2, 4, .. -- with NaN present lanes can end with different
// minima, and each uses its own at the next step.  A line switches to this "faithful" step
// (sticky) at the first step whose costs are not all finite: every earlier state is finite, so
// it carries over exactly.  Generic D (the reference has D = 128 only): lanes of 4, missing
// disparities of the last lane and padding lanes up to a power of two act as +inf.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double pymin(double a, double b) { return b < a ? b : a; }

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int N>
struct SgmV {
    typedef float T __attribute__((ext_vector_type(N)));
};

template <int DPL>
__device__ __forceinline__ bool any_nonfinite(const float (&c)[DPL])
{
    bool nf = false;
#pragma unroll
    for (int i = 0; i < DPL; i++) nf |= __builtin_amdgcn_classf(c[i], 0x207);   // s/qNaN, -inf, +inf
    return __builtin_amdgcn_ballot_w64(nf) != 0;
}

// ... or a non-finite penalty (the fast recurrence's minima are the reference's for finite
// operands only)
template <int DPL>
__device__ __forceinline__ bool any_nonfinite(const float (&c)[DPL], float p1, float p2)
{
    bool nf = __builtin_amdgcn_classf(p1, 0x207) | __builtin_amdgcn_classf(p2, 0x207);
#pragma unroll
    for (int i = 0; i < DPL; i++) nf |= __builtin_amdgcn_classf(c[i], 0x207);
    return __builtin_amdgcn_ballot_w64(nf) != 0;
}
template <int DPL>
__device__ __forceinline__ bool any_nonfinite_v(const typename SgmV<DPL>::T &c, float p1, float p2)
{
    bool nf = __builtin_amdgcn_classf(p1, 0x207) | __builtin_amdgcn_classf(p2, 0x207);
#pragma unroll
    for (int i = 0; i < DPL; i++) nf |= __builtin_amdgcn_classf(c[i], 0x207);
    return __builtin_amdgcn_ballot_w64(nf) != 0;
}

// LDS of the faithful step (wave-private): the step's path costs, then one minimum per reference lane
template <int DPL>
struct FaithLds {
    double L[64 * DPL];
    double v[128];
};

// One SGM_Interation in the reference's exact arithmetic (see above).  mv / mpv: this lane's
// disparities' reference-lane minimum and minimum + P2 from the previous step; updated here.
template <int DPL>
__device__ __forceinline__ void faithful_step(double (&Ln)[DPL], const double (&L)[DPL], const float (&c)[DPL],
                                           bool restart, double p1, double p2, double (&mv)[DPL],
                                           double (&mpv)[DPL], int D, int dbase, FaithLds<DPL> &lds)
{
    const int lane = threadIdx.x & 63;
    if (restart) {
#pragma unroll
        for (int i = 0; i < DPL; i++) Ln[i] = (double)c[i];
    } else {
        const double lo = dpp_f64<0x138>(L[DPL - 1]);   // wave_shr:1 -> L'(dbase - 1)
        const double hi = dpp_f64<0x130>(L[0]);         // wave_shl:1 -> L'(dbase + DPL)
#pragma unroll
        for (int i = 0; i < DPL; i++) {
            const int d = dbase + i;
            const double self = L[i];
            const double lft = d > 0 ? (i > 0 ? L[i - 1] : lo) : self;
            const double rgt = d < D - 1 ? (i < DPL - 1 ? L[i + 1] : hi) : self;
            const double m1 = pymin(lft + p1, self);
            const double m2 = pymin(rgt + p1, mpv[i]);
            Ln[i] = (double)c[i] + (pymin(m1, m2) - mv[i]);
        }
    }
#pragma unroll
    for (int i = 0; i < DPL; i++)
        if (dbase + i < D) lds.L[dbase + i] = Ln[i];
    wave_sync();
    const int nl = (D + 3) / 4;
    int nlp = 1;
    while (nlp < nl) nlp <<= 1;
    double v[2];
#pragma unroll
    for (int t = 0; t < 2; t++) {
        const int j = lane + 64 * t;
        double q[4];
#pragma unroll
        for (int k = 0; k < 4; k++) q[k] = (j < nl && 4 * j + k < D) ? lds.L[4 * j + k] : __builtin_inf();
        v[t] = pymin(pymin(q[0], q[1]), pymin(q[2], q[3]));
    }
    for (int k = 1; k < nlp; k <<= 1) {
        if (k < 64) {
#pragma unroll
            for (int t = 0; t < 2; t++) v[t] = pymin(v[t], __shfl_xor(v[t], k, 64));
        } else {   // lanes j and j ^ 64 live in this lane
            const double a = v[0], b = v[1];
            v[0] = pymin(a, b);
            v[1] = pymin(b, a);
        }
    }
#pragma unroll
    for (int t = 0; t < 2; t++)
        if (lane + 64 * t < nlp) lds.v[lane + 64 * t] = v[t];
    wave_sync();
#pragma unroll
    for (int i = 0; i < DPL; i++) {
        const int d = min(dbase + i, D - 1);
        mv[i] = lds.v[d >> 2];
        mpv[i] = mv[i] + p2;
    }
    wave_sync();     // this step's LDS reads before the next step's writes
}

// One vertical line (column `line`) in the faithful arithmetic, no prefetch: the redo of a
// column whose costs are not all finite after a pass that folded DU into UD (the fold is exact
// for finite costs only).  down: UD (penalty ch 2/3) or DU (ch 0/1); accumulate: S += L,
// else S := f32(0 + L) and the rows the line does not visit are zeroed.
template <int DPL>
__device__ __noinline__ void faithful_vertical(const float *cv, const float *pen, float *S, int H, int W, int D,
                                               int line, bool down, bool accumulate, FaithLds<DPL> &lds)
{
    const int lane = threadIdx.x & 63, dbase = lane * DPL;
    const int n = H - 1 > 2 ? H - 1 : 2;
    double L[DPL], mv[DPL], mpv[DPL];
#pragma unroll
    for (int i = 0; i < DPL; i++) L[i] = mv[i] = mpv[i] = 1.0;
    for (int k = 0; k < n; k++) {
        const int r = down ? k : H - 1 - k;
        const int pr = down ? r - 1 : r + 1;
        const double p1 = (pr >= 0 && pr < H) ? (double)pen[((size_t)pr * W + line) * 16 + (down ? 2 : 0)] : 0.0;
        const double p2 = (double)pen[((size_t)r * W + line) * 16 + (down ? 3 : 1)];
        const size_t off = ((size_t)r * W + line) * D;
        float c[DPL];
#pragma unroll
        for (int i = 0; i < DPL; i++) c[i] = cv[off + min(dbase + i, D - 1)];
        double Ln[DPL];
        faithful_step<DPL>(Ln, L, c, k == 0, p1, p2, mv, mpv, D, dbase, lds);
#pragma unroll
        for (int i = 0; i < DPL; i++) {
            if (dbase + i < D) {
                const double s0 = accumulate ? (double)S[off + dbase + i] : 0.0;
                S[off + dbase + i] = (float)(s0 + Ln[i]);
            }
            L[i] = Ln[i];
        }
    }
    if (!accumulate)
        for (int r = down ? n : 0; down ? r < H : r < H - n; r++)
#pragma unroll
            for (int i = 0; i < DPL; i++)
                if (dbase + i < D) S[((size_t)r * W + line) * D + dbase + i] = 0.0f;
}

struct SgmSide {
    const float *cv;
    const float *pen;
    float *S;
    float *disp;    // WTA fused into the last direction (sde_sgm_8path_wta_pair), else unused
};

// DPP move of an int; lanes outside ROW_MASK keep `v`.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ int dpp_i32(int v)
{
    return __builtin_amdgcn_update_dpp(v, v, CTRL, ROW_MASK, 0xF, false);
}

// first-min merge of (value, index): b replaces a iff strictly smaller, or equal with a
// lower index -- the sequential `v < best` scan over increasing d (NaN never wins)
__device__ __forceinline__ void wta_merge(float &v, int &a, float v2, int a2)
{
    if (v2 < v || (v2 == v && a2 < a)) { v = v2; a = a2; }
}

// (min, first argmin) over the 64 lanes, valid in lane 63 (same DPP butterfly as wave_min_f64)
__device__ __forceinline__ void wave_argmin(float &v, int &a)
{
#define SDE_WTA_STEP(CTRL, RM)                                                               \
    {                                                                                        \
        const float v2 = __int_as_float(dpp_i32<CTRL, RM>(__float_as_int(v)));               \
        const int a2 = dpp_i32<CTRL, RM>(a);                                                 \
        wta_merge(v, a, v2, a2);                                                             \
    }
    SDE_WTA_STEP(0xB1, 0xF)
    SDE_WTA_STEP(0x4E, 0xF)
    SDE_WTA_STEP(0x124, 0xF)
    SDE_WTA_STEP(0x128, 0xF)
    SDE_WTA_STEP(0x142, 0xA)
    SDE_WTA_STEP(0x143, 0xC)
#undef SDE_WTA_STEP
}

// WTA_and_SupixelRefinement_kernel (process_functional.py:800-837) on one pixel whose S values
// are o[i] at d = dbase + i: best = S(0), `best > S(d)` for d = 1.. (== the +inf first-min scan,
// except that "no winner" and a NaN S(0) give 0); lane 63 holds the answer.
template <int DPL>
__device__ __forceinline__ int wta_pixel(const float (&o)[DPL], int dbase, int D)
{
    float best = __builtin_inff();
    int arg = 0x7fffffff;
#pragma unroll
    for (int i = 0; i < DPL; i++)
        if (dbase + i < D && o[i] < best) { best = o[i]; arg = dbase + i; }
    wave_argmin(best, arg);
    const float v0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(o[0]), 0));
    return (arg == 0x7fffffff || v0 != v0) ? 0 : arg;
}

// The end of one step's 64-way merge in the fused WTA: the G lanes of the step (a DPP row group)
// hold the merges of their PF partials each; quad_perm, quad_perm, row_half_mirror (and
// row_mirror for G = 16) leave every lane with the G-lane result -- the merge is a total order
// (first-min with index tie-break, no NaN partials), so any order agrees -- and lane q = 0 stores
// the disparity (rule of WTA_and_SupixelRefinement_kernel: "no winner" -> 0) unless px < 0.
template <int G>
__device__ __forceinline__ void wta_block_store(float bv, int ba, int px, int q, float *disp)
{
    static_assert(G == 8 || G == 16, "the fused WTA merge reduces 8 or 16 lanes per step");
#define SDE_WTA_DPP(CTRL)                                                           \
    {                                                                               \
        const float v2 = __int_as_float(dpp_i32<CTRL>(__float_as_int(bv)));         \
        const int a2 = dpp_i32<CTRL>(ba);                                           \
        wta_merge(bv, ba, v2, a2);                                                  \
    }
    SDE_WTA_DPP(0xB1)       // quad_perm [1,0,3,2]
    SDE_WTA_DPP(0x4E)       // quad_perm [2,3,0,1]
    SDE_WTA_DPP(0x141)      // row_half_mirror: the other quad of the 8
    if (G == 16) SDE_WTA_DPP(0x140)     // row_mirror: the other 8 of the 16
#undef SDE_WTA_DPP
    if (q == 0 && px >= 0) disp[px] = (float)(ba == 0x7fffffff ? 0 : ba);
}

// the destination of the S stores a step must not make (sgm_scan_kernel): one row of the widest lane
// block, rewritten by every wave that needs it, never read
__device__ float sgm_dump[64 * 16];

// a slot's DPL costs / S values as ONE vector value: as separate floats, the loop-header phis of
// the elements did not coalesce with the dwordx{DPL} load's register tuple, and the loop latch
// copied them back -- waiting for each slot's load, i.e. draining the prefetch ring
template <int DPL>
struct Slot {
    typename SgmV<DPL>::T c;
    typename SgmV<DPL>::T s;
    float p1, p2;   // p1 as loaded: the step applies `pin` (a select at issue would wait for the load);
                    // SGM_WALK: this pixel's P1 channel, the NEXT step's P1
    size_t off;     // voxel offset of (r, c, d = 0)
    int pix;        // pixel index r W + c (the fused WTA's output index; no 64-bit division by D per step)
    bool restart;
    bool pin;       // the previous pixel is inside the image (else P1 = 0); unused under SGM_WALK
};

// Incremental walk along a scanline (wave-uniform scalars; no divisions).  Same
// pixel sequence as path_pixel: diagonal lines wrap around the image with a
// path restart.  Steps past the end of the line are clamped into the image (the
// kernel re-reads valid memory there and stores nothing).
// SGM_WALK (the default): the pixel index itself advances (one 64-bit scalar add per step, and a
// +-W on a diagonal wrap) and stops at the line's last pixel, instead of clamping (r, c) and
// recomputing r W + c and the previous pixel's index with 64-bit multiplies on every step.  A
// step's predecessor on the path is the previous step's pixel unless the step restarts the path
// (line start, diagonal wrap), which is exactly when the reference's P1 pixel is outside the
// image -- so P1 is carried from the previous step and one 8-byte load per step fetches (P1, P2)
// of the pixel (channels ch, ch + 1; ch even).
#ifndef SGM_WALK
#define SGM_WALK 1
#endif
#ifndef SGM_EDGESEL
#define SGM_EDGESEL 1  // D = 64 DPL kernels: the edge lanes' missing neighbours by selects, not branches
#endif
struct Walker {
    int r, c;
    bool restart;
    int left;           // SGM_WALK: moves left before the line's last pixel
    long long dpx;      // SGM_WALK: pixel-index step dr W + dc
    size_t px;          // SGM_WALK: the pixel index r W + c
    __device__ __forceinline__ void init(const PathGeom &g, int line)
    {
        if (g.dc == 0) { c = line; r = g.dr > 0 ? 0 : g.H - 1; }
        else if (g.dr == 0) { r = line; c = g.dc > 0 ? 0 : g.W - 1; }
        else { r = g.dr > 0 ? 0 : g.H - 1; c = line; }
        restart = true;
        if (SGM_WALK) {
            const int nlen = (g.dc != 0 && g.dr == 0) ? g.W : g.H;
            left = min(g.n, nlen) - 1;
            dpx = (long long)g.dr * g.W + g.dc;
            px = (size_t)r * g.W + c;
        }
    }
    __device__ __forceinline__ void advance(const PathGeom &g)
    {
        if (SGM_WALK) {
            // selects, not branches (scalar s_cselect; the step is one basic block)
            const bool mv = left > 0;
            left -= mv ? 1 : 0;
            c += mv ? g.dc : 0;
            px += mv ? dpx : 0;
            restart = false;
            if (g.dr != 0 && g.dc != 0) {
                const bool wr = g.dc > 0 ? c >= g.W : c < 0;
                c = wr ? (g.dc > 0 ? 0 : g.W - 1) : c;
                px = wr ? (g.dc > 0 ? px - g.W : px + g.W) : px;
                restart = wr;
            }
            return;
        }
        r += g.dr;
        c += g.dc;
        restart = false;
        if (g.dr != 0 && g.dc != 0) {
            if (c >= g.W) { c = 0; restart = true; }
            else if (c < 0) { c = g.W - 1; restart = true; }
        }
    }
};

// VEC: D % DPL == 0, every lane's DPL disparities are all valid or all invalid
// and move as one dwordx{DPL}; otherwise per-element loads with clamped d.
template <int DPL, bool VEC, bool FIRST>
__device__ __forceinline__ void issue(const PathGeom &g, const Walker &w, const SgmSide &sd, int D, int dbase,
                                      Slot<DPL> &sl)
{
    size_t px;
    if (SGM_WALK) {
        px = w.px;
        const float2 pp = *reinterpret_cast<const float2 *>(sd.pen + px * 16 + g.ch);
        sl.p1 = pp.x;
        sl.p2 = pp.y;
    } else {
        const int r = min(max(w.r, 0), g.H - 1), c = min(max(w.c, 0), g.W - 1);
        px = (size_t)r * g.W + c;
        int pr = r - g.dr, pc = c - g.dc;
        const bool pin = pr >= 0 && pr < g.H && pc >= 0 && pc < g.W;
        pr = pin ? pr : r;
        pc = pin ? pc : c;
        sl.p1 = sd.pen[((size_t)pr * g.W + pc) * 16 + g.ch];
        sl.pin = pin;
        sl.p2 = sd.pen[px * 16 + g.ch + 1];
    }
    sl.restart = w.restart;
    sl.pix = (int)px;
    const size_t off = px * D;
    sl.off = off;
    if (VEC) {
        const size_t o = off + (dbase < D ? dbase : 0);
        if (SGM_NT & 1) {
            // wave-uniform row pointers + a 32-bit lane offset: the loads take the SGPR-base form
            const float *cvp = sd.cv + off, *sp = sd.S + off;
            const unsigned lo = (unsigned)(dbase < D ? dbase : 0);
#pragma unroll
            for (int i = 0; i < DPL; i++) sl.c[i] = __builtin_nontemporal_load(cvp + lo + i);
            if (!FIRST)
#pragma unroll
                for (int i = 0; i < DPL; i++) sl.s[i] = __builtin_nontemporal_load(sp + lo + i);
        } else {
        const FVec<DPL> cv = *reinterpret_cast<const FVec<DPL> *>(sd.cv + o);
#pragma unroll
        for (int i = 0; i < DPL; i++) sl.c[i] = cv.v[i];
        if (!FIRST) {
            const FVec<DPL> sv = *reinterpret_cast<const FVec<DPL> *>(sd.S + o);
#pragma unroll
            for (int i = 0; i < DPL; i++) sl.s[i] = sv.v[i];
        }
        }
    } else {
#pragma unroll
        for (int i = 0; i < DPL; i++) {
            const int d = dbase + i < D ? dbase + i : D - 1;
            sl.c[i] = sd.cv[off + d];
            if (!FIRST) sl.s[i] = sd.S[off + d];
        }
    }
}

// FIRST: S := f32(0 + L) (S is not read).  DU (direction UD only): also apply direction
// DU in the same pass.  With the penalty channels 0/1 zero -- sgm_penelty_kernel never
// writes them (:134-262) -- and finite costs, DU's recurrence collapses: b = m' exactly,
// so L_DU = C at its first pixel (row H-1) and C + 0.0 elsewhere; the reference adds
// it after UD (launch order :1166-1203), which per voxel is this same sequence.
// WTA (last direction only): the final S of each visited voxel is not stored; the pixel's
// first-min disparity (rule of WTA_and_SupixelRefinement_kernel) goes to sd.disp instead, and
// the pixels this direction never visits (its lines stop one short) take the WTA of the S
// already in memory.
template <int DPL, int PF, bool VEC, bool FIRST, bool DU, bool WTA, int DC, int DIRC, bool VMIN>
__global__ __launch_bounds__(64) void sgm_scan_kernel(SgmSide s0, SgmSide s1, int H, int W, int D, int dir)
{
    // DC != 0: D == DC == 64 * DPL is a compile-time constant -- every lane's disparities are
    // valid, so the per-disparity range guards and the pixel index's division fold away
    if (DC) D = DC;
    const SgmSide sd = blockIdx.y ? s1 : s0;
    PathGeom g;
    // DIRC >= 0: the direction is a compile-time constant (the walker's steps, wrap tests and the
    // penalty channel fold); the pair path's seven launches use these
    constexpr int kdr[8] = {+1, -1, 0, 0, +1, -1, +1, -1}, kdc[8] = {0, 0, +1, -1, +1, +1, -1, -1},
                  kch[8] = {2, 0, 6, 4, 10, 12, 8, 14};
    if (DIRC >= 0) {
        g.dr = kdr[DIRC & 7]; g.dc = kdc[DIRC & 7]; g.ch = kch[DIRC & 7];
    } else {
        g.dr = c_dir_dr[dir]; g.dc = c_dir_dc[dir]; g.ch = c_dir_ch[dir];
    }
    g.H = H; g.W = W;
    const int nlen = (g.dc != 0 && g.dr == 0) ? W : H;
    g.n = nlen - 1 > 2 ? nlen - 1 : 2;
    const int line = blockIdx.x;
    const int lane = threadIdx.x & 63;      // one wave per block: lane < 64 known to the compiler
#if SGM_SKEW > 0
    for (int k = line % SGM_SKEW_K; k > 0; k--) __builtin_amdgcn_s_sleep(SGM_SKEW);
#endif
    const int dbase = lane * DPL;
    const double INF = __builtin_inf();
    // fused WTA: per-step lane partials of the last PF steps (wave-private: one wave per block).
    // G = 64 / PF lanes merge one step; lane l's partial of step j sits at j * WS + (l % PF) * G +
    // l / PF with WS = 64 + G: the merge's reads (lane (st, q) takes partials q, q + G, .. of step
    // st) then hit 32 distinct banks per half-wave -- the straight j * 64 + l layout made the merge
    // reads 8-way conflicted (PMC: 65 % of the launch's LDS cycles were conflicts).  Within a step's
    // row, the G-word group of lane l % PF is XOR-swizzled by (l % PF) & 4: lanes l and l + 4 (same
    // l / PF, rows 32 words apart in bank space) then land in disjoint halves of their 8 banks, so
    // the per-step ds_write_b32s are conflict-free too (were 2-way: 28 % of the launch's LDS cycles)
    // The merge of a block of PF steps is spread over the next block's steps (one partial read and
    // merge per step, the G-lane DPP reduction and the store at its last step), so the loop body
    // stays one uniform step: a separate merge block after every PF steps made the compiler rotate
    // the prefetch ring's registers at the loop back-edge and drain it (vmcnt(0) every PF steps).
    // Partials and pixel indices are double-buffered by block parity.
    //
    // SGM_WTA_PARK (the default): each step parks its 64 DPL S values (+inf past D), value i of lane
    // l at word i IS + l of a row of RS words, and lane (st, q) scans pixel st's disparities
    // DPL (PF q + j) + i, i < DPL, at step j of the next block -- the values lane PF q + j parked --
    // in increasing d with a strict `<` (the reference's sequential scan over its chunk), so only the
    // G-lane DPP merge needs the index tie-break.  Banks (PF = 8): RS = 1 mod 64 puts pixel st's row
    // st banks over, lanes q of a read are 8 banks apart, and IS = 4 mod 64 sends the second word of
    // the compiler's paired `ds_read2_b32` to the other 4 banks of each 8: writes and reads are
    // conflict-free (a [lane][i] row with stride DPL had the pair's words collide: 12.6 M conflict
    // cycles per pair of launches).
    constexpr int IS = 68, RS = ((DPL * IS + 63) / 64) * 64 + 1;
    constexpr int G = 64 / PF, WS = 64 + G;
    constexpr bool PARK = SGM_WTA_PARK != 0;
    __shared__ float wbv[WTA ? 2 * PF * (PARK ? RS : WS) : 1];
    __shared__ int wba[WTA && !PARK ? 2 * PF * WS : 1];
    __shared__ int wpx[WTA ? 2 * PF : 1];
    __shared__ FaithLds<DPL> flds;

    if (DU && !FIRST) {
        // accumulate + DU fold: S's incoming values cannot be recovered after a folded pass, so a
        // column whose costs are not all finite is found first and runs both directions in the
        // reference's arithmetic (the fold is exact for finite costs only)
        // (and the UD penalties, channels 2/3: the fast recurrence's minima are the reference's
        // for finite operands only)
        bool bad = false;
        for (int r = 0; r < H && !bad; r++) {
            float c[DPL];
            const size_t px = (size_t)r * W + line, off = px * D;
#pragma unroll
            for (int i = 0; i < DPL; i++) c[i] = sd.cv[off + min(dbase + i, D - 1)];
            bad = any_nonfinite<DPL>(c, sd.pen[px * 16 + 2], sd.pen[px * 16 + 3]);
        }
        if (bad) {
            faithful_vertical<DPL>(sd.cv, sd.pen, sd.S, H, W, D, line, true, true, flds);
            faithful_vertical<DPL>(sd.cv, sd.pen, sd.S, H, W, D, line, false, true, flds);
            return;
        }
    }

    // Every load is unconditional (steps past the end re-read a clamped pixel):
    // a predicated load would make the ring slot a phi and force an early wait.  (Refilling the
    // ring two adjacent pixels at a time for the horizontal directions measured no gain in round 3
    // and was removed.)
    Slot<DPL> ring[PF];
    Walker ahead;
    ahead.init(g, line);
#pragma unroll
    for (int j = 0; j < PF; j++) {
        issue<DPL, VEC, FIRST>(g, ahead, sd, D, dbase, ring[j]);
        ahead.advance(g);
    }
    // the ring has landed before the loop: otherwise the loop header merges this entry path (the
    // fill's loads in another order, fewer ops after each) with the latch, and the waitcnt pass sizes
    // the first steps' waits for the entry path -- vmcnt(1..3) every PF steps, a drained ring.
    // Except in the first pass (cost loads, S stores, no S loads): there the drained ring is the
    // faster one, 619 against 646 us per launch (profiles/r04/sgm_ab_ring_waits.txt; PF 4 or 6:
    // 634 / 647 us) -- the other six launches gain from the full ring (DU-RL + WTA 670 -> 620 us)
    if (!(FIRST && DU)) __builtin_amdgcn_s_waitcnt(0xF70);          // vmcnt(0)

    double L[DPL];
    double m = 1.0, mP2 = 1.0;
    float p1c = 0.0f;              // SGM_WALK: the previous step's pixel's P1 channel
    int kf = -1;                   // first step with a non-finite cost: the line continues faithfully
    bool redo = false;             // DU fold (FIRST): recompute the column in the faithful arithmetic
#pragma unroll
    for (int i = 0; i < DPL; i++) L[i] = 1.0;

    // fused WTA: this lane's running merge over the previous block (lane (st, q) = (lane / G,
    // lane % G) merges the partials of lanes PF q .. PF q + PF - 1 of step st of that block)
    float mv_b = __builtin_inff();
    int mv_a = 0x7fffffff;
    const int wst = lane / G, wq = lane % G;
    for (int k0 = 0; k0 < g.n; k0 += PF) {
        const int buf = (k0 / PF) & 1;              // this block's partial buffer; buf ^ 1 = the previous block's
#pragma unroll
        for (int j = 0; j < PF; j++) {
            const int k = k0 + j;     // steps k >= n compute on a clamped pixel and store nothing
            const Slot<DPL> &sl = ring[j];
            const float p1f = SGM_WALK ? (sl.restart ? 0.0f : p1c) : (sl.pin ? sl.p1 : 0.0f);
            // (wave-uniform; into an SGPR for the reason given for p1c below)
            const float p2f = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, sl.p2)));
            // read before the slot's refill at the end of this step, into an SGPR: carried as the
            // slot's own VGPR it stayed live across the refill, so the refill took other registers and
            // the loop latch copied every slot's penalty pair back -- waiting for each load in turn,
            // which drained the prefetch ring once per PF steps
            if (SGM_WALK) p1c = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, sl.p1)));
            if (DU) {
                if (FIRST && !redo) redo = any_nonfinite_v<DPL>(sl.c, p1f, p2f);
            } else if (kf < 0 && k < g.n && any_nonfinite_v<DPL>(sl.c, p1f, p2f)) {
                // every state so far is finite; from step k on the line is redone in the reference's
                // exact arithmetic after this loop, which stores nothing more for it
                kf = k;
            }
            const bool keep = DU || kf < 0;
            double Ln[DPL];
            if (sl.restart) {
#pragma unroll
                for (int i = 0; i < DPL; i++) Ln[i] = (double)sl.c[i];
            } else {
                const double p1 = (double)p1f;
                const double lo = dpp_f64<0x138>(L[DPL - 1]);   // wave_shr:1 -> L'(dbase - 1)
                const double hi = dpp_f64<0x130>(L[0]);         // wave_shl:1 -> L'(dbase + DPL)
#pragma unroll
                for (int i = 0; i < DPL; i++) {
                    const int d = dbase + i;
                    double b = L[i];
                    const double left = i > 0 ? L[i - 1] : lo;
                    const double right = i < DPL - 1 ? L[i + 1] : hi;
                    if (DC && SGM_EDGESEL) {
                        // D = 64 DPL: only lane 0's first and lane 63's last disparity lack a
                        // neighbour -- a select of +inf (min(b, inf) = b) instead of an exec-masked
                        // branch per step
                        b = dmin<VMIN>(b, (i > 0 || d > 0) ? left + p1 : INF);
                        b = dmin<VMIN>(b, (i < DPL - 1 || d < D - 1) ? right + p1 : INF);
                    } else {
                        if (d > 0) b = dmin<VMIN>(b, left + p1);
                        if (d < D - 1) b = dmin<VMIN>(b, right + p1);
                    }
                    b = dmin<VMIN>(b, mP2);
                    Ln[i] = (double)sl.c[i] + (b - m);
                }
            }
            float o[DPL];
#pragma unroll
            for (int i = 0; i < DPL; i++)
                o[i] = FIRST ? (float)(0.0 + Ln[i]) : (float)((double)sl.s[i] + Ln[i]);
            if (DU && k >= H - g.n) {          // UD visits row k; DU visits rows H-n .. H-1
                const bool du_first = (k == H - 1);
#pragma unroll
                for (int i = 0; i < DPL; i++) {
                    const double c = (double)sl.c[i];
                    o[i] = (float)((double)o[i] + (du_first ? c : c + 0.0));
                }
            }
            if (WTA && PARK) {
                // this step's S values parked; one piece of the previous block's scan (below), off
                // the recurrence's serial chain
                float *row = wbv + (buf * PF + j) * RS + lane;
#pragma unroll
                for (int i = 0; i < DPL; i++) row[i * IS] = (DC || dbase + i < D) ? o[i] : __builtin_inff();
                if (lane == 0) wpx[buf * PF + j] = (k < g.n && keep) ? sl.pix : -1;
                if (k0 > 0) {
                    const int d0 = DPL * (PF * wq + j);
                    const float *src = wbv + ((buf ^ 1) * PF + wst) * RS + PF * wq + j;
#pragma unroll
                    for (int i = 0; i < DPL; i++) {
                        const float v2 = src[i * IS];
                        if (j == 0 && i == 0) {
                            // the chunk's first value; a NaN S(0) makes the pixel's answer 0
                            const bool w = v2 < __builtin_inff();
                            mv_b = w ? v2 : __builtin_inff();
                            mv_a = w ? d0 : 0x7fffffff;
                            if (wq == 0 && v2 != v2) { mv_b = -__builtin_inff(); mv_a = 0; }
                        } else if (v2 < mv_b) {
                            mv_b = v2;
                            mv_a = d0 + i;
                        }
                    }
                    if (j == PF - 1) wta_block_store<G>(mv_b, mv_a, wpx[(buf ^ 1) * PF + wst], wq, sd.disp);
                }
            } else if (WTA) {
                // lane-local first-min over this lane's disparities, parked in LDS; the 64-way
                // merge runs once per PF steps (below), off the recurrence's serial chain
                float bv = __builtin_inff();
                int ba = 0x7fffffff;
#pragma unroll
                for (int i = 0; i < DPL; i++)
                    if (dbase + i < D && o[i] < bv) { bv = o[i]; ba = dbase + i; }
                if (lane == 0 && o[0] != o[0]) { bv = -__builtin_inff(); ba = 0; }   // NaN S(0): d = 0
                const int slot = (buf * PF + j) * WS + (lane % PF) * G + ((lane / PF) ^ (lane % PF & 4));
                wbv[slot] = bv;
                wba[slot] = ba;
                if (lane == 0) wpx[buf * PF + j] = (k < g.n && keep) ? sl.pix : -1;
                // one step of the previous block's merge (nothing to merge in the first block)
                if (k0 > 0) {
                    const int rs = ((buf ^ 1) * PF + wst) * WS + j * G + (wq ^ (j & 4));
                    const float v2 = wbv[rs];
                    const int a2 = wba[rs];
                    if (j == 0) { mv_b = v2; mv_a = a2; }
                    else wta_merge(mv_b, mv_a, v2, a2);
                    if (j == PF - 1) wta_block_store<G>(mv_b, mv_a, wpx[(buf ^ 1) * PF + wst], wq, sd.disp);
                }
            } else if (VEC) {
                // every step stores: a step that must not (past the line's end, a line gone faithful)
                // writes the dump row instead.  A store behind a branch left the waitcnt pass unsure
                // how many stores were in flight, so it waited for loads issued 2-3 steps back
                // instead of PF: the prefetch ring was mostly idle.
                float *const sbase = (k < g.n && keep) ? sd.S + sl.off : sgm_dump;
                if (dbase < D) {
                    FVec<DPL> ov;
#pragma unroll
                    for (int i = 0; i < DPL; i++) ov.v[i] = o[i];
                    if (SGM_NT & 2) {
#pragma unroll
                        for (int i = 0; i < DPL; i++)
                            __builtin_nontemporal_store(o[i], sbase + (unsigned)dbase + i);
                    } else {
                        *reinterpret_cast<FVec<DPL> *>(sbase + dbase) = ov;
                    }
                }
            } else if (k < g.n && keep) {
                {
#pragma unroll
                    for (int i = 0; i < DPL; i++)
                        if (dbase + i < D) sd.S[sl.off + dbase + i] = o[i];
                }
            }
            double mm = INF;
#pragma unroll
            for (int i = 0; i < DPL; i++)
                if (dbase + i < D) mm = dmin<VMIN>(mm, Ln[i]);
            m = wave_min_f64<VMIN>(mm);
            mP2 = m + (double)p2f;
#pragma unroll
            for (int i = 0; i < DPL; i++) L[i] = Ln[i];
            // the slot is refilled after its use (not hoisted above it): its registers are reused,
            // with no moves -- and waits -- at the loop back-edge
            issue<DPL, VEC, FIRST>(g, ahead, sd, D, dbase, ring[j]);
            ahead.advance(g);
        }
    }
    // The parked values and pixel indices cross lanes through LDS: lanes read what other lanes of the
    // wave wrote one block earlier.  Inside the loop a read is always a whole step after the writes it
    // depends on and the compiler does not move LDS accesses of one iteration across another's; here,
    // right after the last writes, the ordering is made explicit (wavefront-scope release/acquire and a
    // wave barrier: no instruction with one wave per workgroup, a scheduling fence only).
    if (WTA && g.n > 0) wave_sync();
    if (WTA && PARK && g.n > 0) {
        // the last block's scan (its values are in buffer buf_last)
        const int buf = ((g.n - 1) / PF) & 1;
        const float *src = wbv + (buf * PF + wst) * RS + PF * wq;
        float b = __builtin_inff();
        int ba = 0x7fffffff;
#pragma unroll
        for (int t = 0; t < DPL * PF; t++) {
            const float v = src[(t % DPL) * IS + t / DPL];      // d = DPL (PF wq + t / DPL) + t % DPL
            if (v < b) { b = v; ba = DPL * PF * wq + t; }
        }
        if (wq == 0 && src[0] != src[0]) { b = -__builtin_inff(); ba = 0; }
        wta_block_store<G>(b, ba, wpx[buf * PF + wst], wq, sd.disp);
    } else if (WTA && g.n > 0) {
        // the last block's merge (its partials are in buffer buf_last)
        const int buf = ((g.n - 1) / PF) & 1;
        float b = wbv[(buf * PF + wst) * WS + wq];
        int ba = wba[(buf * PF + wst) * WS + wq];
#pragma unroll
        for (int t = 1; t < PF; t++) {
            const int rs = (buf * PF + wst) * WS + t * G + (wq ^ (t & 4));
            wta_merge(b, ba, wbv[rs], wba[rs]);
        }
        wta_block_store<G>(b, ba, wpx[buf * PF + wst], wq, sd.disp);
    }
    if (!DU && kf >= 0) {
        // the line again in the reference's exact arithmetic (no prefetch: rare path), storing from
        // step kf on: the replayed finite prefix reproduces the fast steps' state exactly
        double mv[DPL], mpv[DPL];
#pragma unroll
        for (int i = 0; i < DPL; i++) L[i] = mv[i] = mpv[i] = 1.0;
        for (int k = 0; k < g.n; k++) {
            int r, c;
            bool restart;
            path_pixel(g, line, k, r, c, restart);
            const int pr = r - g.dr, pc = c - g.dc;
            const bool pin = pr >= 0 && pr < H && pc >= 0 && pc < W;
            const double p1 = pin ? (double)sd.pen[((size_t)pr * W + pc) * 16 + g.ch] : 0.0;
            const double p2 = (double)sd.pen[((size_t)r * W + c) * 16 + g.ch + 1];
            const size_t off = ((size_t)r * W + c) * D;
            float cc[DPL];
#pragma unroll
            for (int i = 0; i < DPL; i++) cc[i] = sd.cv[off + min(dbase + i, D - 1)];
            double Ln[DPL];
            faithful_step<DPL>(Ln, L, cc, restart, p1, p2, mv, mpv, D, dbase, flds);
            if (k < kf) {
#pragma unroll
                for (int i = 0; i < DPL; i++) L[i] = Ln[i];
                continue;
            }
            float o[DPL];
#pragma unroll
            for (int i = 0; i < DPL; i++) {
                const double s0 = FIRST ? 0.0 : (double)sd.S[off + min(dbase + i, D - 1)];
                o[i] = (float)(s0 + Ln[i]);
                L[i] = Ln[i];
            }
            if (WTA) {
                const int a = wta_pixel<DPL>(o, dbase, D);
                if (lane == 63) sd.disp[off / D] = (float)a;
            } else {
#pragma unroll
                for (int i = 0; i < DPL; i++)
                    if (dbase + i < D) sd.S[off + dbase + i] = o[i];
            }
        }
    }
    if (WTA && g.n < nlen) {
        // pixels of this line's direction never visited: the last line position's successor.
        // DU-RL (the reference's last direction) walks rows H-1 .. 1 and never reaches row 0:
        // pixel (0, line) is one of them for every line; other directions map analogously.
        int r0, c0;
        if (g.dc == 0) { r0 = g.dr > 0 ? H - 1 : 0; c0 = line; }
        else if (g.dr == 0) { r0 = line; c0 = g.dc > 0 ? W - 1 : 0; }
        else { r0 = g.dr > 0 ? H - 1 : 0; c0 = line; }
        const size_t off = ((size_t)r0 * W + c0) * D;
        float o[DPL];
#pragma unroll
        for (int i = 0; i < DPL; i++) o[i] = sd.S[off + min(dbase + i, D - 1)];
        const int a = wta_pixel<DPL>(o, dbase, D);
        if (lane == 63) sd.disp[off / D] = (float)a;
    }
    if (FIRST || DU) {
        // rows UD never visits (it stops at row n-1): S := 0 (FIRST), then DU's term
        for (int r = g.n; r < H; r++) {
            const size_t off = ((size_t)r * W + line) * D;
#pragma unroll
            for (int i = 0; i < DPL; i++) {
                const int d = dbase + i;
                if (d < D) {
                    float v = FIRST ? 0.0f : sd.S[off + d];
                    if (DU) {
                        const float cf = sd.cv[off + d];
                        if (FIRST) redo |= (__float_as_uint(cf) & 0x7f800000u) == 0x7f800000u;
                        const double c = (double)cf;
                        v = (float)((double)v + (r == H - 1 ? c : c + 0.0));
                    }
                    sd.S[off + d] = v;
                }
            }
        }
    }
    if (DU && FIRST && __builtin_amdgcn_ballot_w64(redo) != 0) {
        // a non-finite cost in this column: the folded DU term is not the reference's -- redo UD
        // (overwrite) and DU (accumulate) in the faithful arithmetic
        faithful_vertical<DPL>(sd.cv, sd.pen, sd.S, H, W, D, line, true, false, flds);
        faithful_vertical<DPL>(sd.cv, sd.pen, sd.S, H, W, D, line, false, true, flds);
    }
}

// VMIN: S holds no -0.0 on entry (this library wrote it, or the pass overwrites it): the fast
// recurrence's minima may run on v_min_f64 (see dmin).  The other case (accumulating onto a
// caller's S) keeps the selects and the generic kernel.
template <int DPL, bool VEC, bool FIRST, bool DU, bool WTA, bool VMIN>
static void launch_scan(const SgmSide &a, const SgmSide &b, int nsides, int H, int W, int D, int dir,
                        hipStream_t st)
{
    const bool horiz = (dir == 2 || dir == 3);
    const int nlines = horiz ? H : W;
    constexpr int PF = DPL <= 4 ? 8 : 4;
    const dim3 grid(nlines, nsides);
#define SDE_SGM_LAUNCH(DC, DIRC) sgm_scan_kernel<DPL, PF, VEC, FIRST, DU, WTA, DC, DIRC, VMIN><<<grid, 64, 0, st>>>(a, b, H, W, D, dir)
    if constexpr (!VEC || !VMIN) {
        SDE_SGM_LAUNCH(0, -1);
    } else {
    if (D != 64 * DPL) {
        SDE_SGM_LAUNCH(0, -1);
        return;
    }
    constexpr int DC = 64 * DPL;
    // compile-time directions for the combinations sde_sgm_8path_wta_pair launches (UD + DU fold,
    // the five middle directions, DU-RL + WTA); any other stays generic
    if constexpr (DU) {
        if (dir == 0) SDE_SGM_LAUNCH(DC, 0);
        else SDE_SGM_LAUNCH(DC, -1);
    } else if constexpr (WTA) {
        if (dir == 7) SDE_SGM_LAUNCH(DC, 7);
        else SDE_SGM_LAUNCH(DC, -1);
    } else if constexpr (!FIRST) {
        switch (dir) {
        case 2: SDE_SGM_LAUNCH(DC, 2); break;
        case 3: SDE_SGM_LAUNCH(DC, 3); break;
        case 4: SDE_SGM_LAUNCH(DC, 4); break;
        case 5: SDE_SGM_LAUNCH(DC, 5); break;
        case 6: SDE_SGM_LAUNCH(DC, 6); break;
        default: SDE_SGM_LAUNCH(DC, -1); break;
        }
    } else {
        SDE_SGM_LAUNCH(DC, -1);
    }
    }
#undef SDE_SGM_LAUNCH
}

// mode: 0 accumulate, 1 first (S := 0 + L), 2 first + DU fold, 3 accumulate + DU fold,
// 4 accumulate + fused WTA (the last direction)
template <int DPL, bool VEC>
static void launch_mode(const SgmSide &a, const SgmSide &b, int nsides, int H, int W, int D, int dir, int mode,
                        bool vmin, hipStream_t st)
{
    switch (mode) {
    case 1: launch_scan<DPL, VEC, true, false, false, true>(a, b, nsides, H, W, D, dir, st); break;
    case 2: launch_scan<DPL, VEC, true, true, false, true>(a, b, nsides, H, W, D, dir, st); break;
    case 3:
        if (vmin) launch_scan<DPL, VEC, false, true, false, true>(a, b, nsides, H, W, D, dir, st);
        else launch_scan<DPL, VEC, false, true, false, false>(a, b, nsides, H, W, D, dir, st);
        break;
    case 4:
        if (vmin) launch_scan<DPL, VEC, false, false, true, true>(a, b, nsides, H, W, D, dir, st);
        else launch_scan<DPL, VEC, false, false, true, false>(a, b, nsides, H, W, D, dir, st);
        break;
    default:
        if (vmin) launch_scan<DPL, VEC, false, false, false, true>(a, b, nsides, H, W, D, dir, st);
        else launch_scan<DPL, VEC, false, false, false, false>(a, b, nsides, H, W, D, dir, st);
        break;
    }
}

template <int DPL>
static void launch_dpl(const SgmSide &a, const SgmSide &b, int nsides, int H, int W, int D, int dir, int mode,
                       bool vmin, hipStream_t st)
{
    if ((D % DPL) == 0) launch_mode<DPL, true>(a, b, nsides, H, W, D, dir, mode, vmin, st);
    else launch_mode<DPL, false>(a, b, nsides, H, W, D, dir, mode, vmin, st);
}

// One direction over one or two sides; first: S := f32(0 + L) (no S read); du (dir 0
// only): direction DU folded into the same pass; wta: the final S is reduced to the
// disparity map (sd.disp) instead of being stored (see sgm_scan_kernel).
static int sgm_direction_impl(const SgmSide &a, const SgmSide &b, int nsides, int H, int W, int D, int dir,
                              bool first, bool vmin, hipStream_t st, bool du = false, bool wta = false)
{
    const int mode = wta ? 4 : (first ? (du ? 2 : 1) : (du ? 3 : 0));
    if (wta && (first || du)) return SDE_ERR_ARG;
    switch ((D + 63) / 64) {
    case 1: launch_dpl<1>(a, b, nsides, H, W, D, dir, mode, vmin, st); break;
    case 2: launch_dpl<2>(a, b, nsides, H, W, D, dir, mode, vmin, st); break;
    case 3: launch_dpl<3>(a, b, nsides, H, W, D, dir, mode, vmin, st); break;
    case 4: launch_dpl<4>(a, b, nsides, H, W, D, dir, mode, vmin, st); break;
    case 5: launch_dpl<5>(a, b, nsides, H, W, D, dir, mode, vmin, st); break;
    case 6: launch_dpl<6>(a, b, nsides, H, W, D, dir, mode, vmin, st); break;
    case 7: launch_dpl<7>(a, b, nsides, H, W, D, dir, mode, vmin, st); break;
    case 8: launch_dpl<8>(a, b, nsides, H, W, D, dir, mode, vmin, st); break;
    default: return SDE_ERR_ARG;
    }
    return SDE_OK;
}

// sgm_penelty_kernel: reduced (P1/lambda, P2/lambda) iff uint64(nb - c) > thr as
// float64, i.e. nb < c or nb > c + thr; channels 0/1 never written (stay 0).
__global__ __launch_bounds__(256) void sgm_penalty_kernel(const uint8_t *__restrict__ img, int H, int W, float fP1,
                                                          float fP2, float rP1, float rP2, double thr,
                                                          float *__restrict__ pen)
{
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (int64_t)H * W) return;
    const int y = (int)(p / W), x = (int)(p % W);
    const uint64_t c = img[p];
    const int dys[8] = {-1, +1, 0, 0, +1, +1, -1, -1};
    const int dxs[8] = {0, 0, -1, +1, -1, +1, +1, -1};
    const int chs[8] = {2, 2, 4, 6, 8, 10, 12, 14};
    float o[16];
    o[0] = 0.0f;
    o[1] = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int yy = y + dys[k], xx = x + dxs[k];
        float a = fP1, b = fP2;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
            const uint64_t diff = (uint64_t)img[(size_t)yy * W + xx] - c;
            if ((double)diff > thr) { a = rP1; b = rP2; }
        }
        o[chs[k]] = a;
        o[chs[k] + 1] = b;
    }
    float4 *dst = reinterpret_cast<float4 *>(pen + p * 16);
#pragma unroll
    for (int i = 0; i < 4; i++) dst[i] = make_float4(o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]);
}

__device__ __forceinline__ int u8cast(double v) { return (int)((long long)v & 255); }

__global__ __launch_bounds__(256) void lr_check_kernel(const float *__restrict__ dl, const float *__restrict__ dr,
                                                       int H, int W, uint8_t *__restrict__ lrcl,
                                                       uint8_t *__restrict__ lrcr)
{
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (int64_t)H * W) return;
    const int y = (int)(p / W), x = (int)(p % W);
    const double ld = dl[p];
    const double rd = (double)x - ld;
    if (rd >= 0) {
        const double mn = ld - (double)dr[(size_t)y * W + u8cast(rd)];
        lrcl[p] = (mn > 1 || mn < -1) ? 1 : 0;
    }
    const double rd2 = dr[p];
    const double ld2 = (double)x + rd2;
    if (ld2 < W) {
        const double mn = rd2 - (double)dl[(size_t)y * W + u8cast(ld2)];
        lrcr[p] = (mn > 1 || mn < -1) ? 1 : 0;
    }
}

// LRC_kernel (:1003-1088): every flagged pixel takes the mean of the nearest unflagged
// pixel above, below, to the right and to the left (each only if it exists), summed in
// that order in float64.  The reference walks each direction pixel by pixel, which is
// quadratic in the length of a flagged run; here linear scans find the same four
// pixels.  Pass 1 (wave per column): nearest unflagged row above / below of every
// flagged pixel, parked in the output as two 16-bit row indices (0xFFFF = none).
// Pass 2 (wave per row): nearest unflagged column to the left (sweep left -> right) and
// to the right (sweep right -> left) by wave-wide max-scans over 64-pixel chunks; the
// right sweep, which runs second, has all four neighbours and writes the result.
constexpr uint32_t LRC_NONE = 0xFFFFu;

// inclusive max-scan over the 64 lanes
__device__ __forceinline__ int wave_max_scan(int v)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(v, o, 64);
        if (lane >= o) v = v > t ? v : t;
    }
    return v;
}

// Pass 1: one wave per column, 64 rows per step, wave-wide max-scans downwards (nearest
// unflagged row above, strictly) and upwards (below), carried across chunks.
__global__ __launch_bounds__(64) void lrc_cols_kernel(const uint8_t *__restrict__ f, int H, int W,
                                                      uint32_t *__restrict__ park)
{
    const int x = blockIdx.x;
    const int lane = threadIdx.x;
    const int nchunk = (H + 63) / 64;
    int carry = -1;
    for (int c = 0; c < nchunk; c++) {             // top -> bottom
        const int y = c * 64 + lane;
        const bool in = y < H;
        const bool flagged = in && f[(size_t)y * W + x] == 1;
        const int v = wave_max_scan(in && !flagged ? y : -1);
        int prev = __shfl_up(v, 1, 64);
        if (lane == 0) prev = -1;
        const int up = prev > carry ? prev : carry;
        const int last = __builtin_amdgcn_readlane(v, 63);
        carry = last > carry ? last : carry;
        if (flagged) park[(size_t)y * W + x] = up < 0 ? LRC_NONE : (uint32_t)up;
    }
    carry = -1;                                    // as H-1-y of the nearest unflagged row below
    for (int c = 0; c < nchunk; c++) {             // bottom -> top
        const int y = H - 1 - (c * 64 + lane);
        const bool in = y >= 0;
        const bool flagged = in && f[(size_t)(in ? y : 0) * W + x] == 1;
        const int v = wave_max_scan(in && !flagged ? H - 1 - y : -1);
        int prev = __shfl_up(v, 1, 64);
        if (lane == 0) prev = -1;
        const int dn = prev > carry ? prev : carry;
        const int last = __builtin_amdgcn_readlane(v, 63);
        carry = last > carry ? last : carry;
        if (flagged) park[(size_t)y * W + x] |= (dn < 0 ? LRC_NONE : (uint32_t)(H - 1 - dn)) << 16;
    }
}

__global__ __launch_bounds__(64) void lrc_rows_kernel(const float *__restrict__ dl, const uint8_t *__restrict__ f,
                                                      int H, int W, float *__restrict__ out)
{
    // nearest unflagged column left of x (LRC_NONE = none): 2 B per column of the row, W <= 65535
    extern __shared__ uint16_t sleft[];
    const int y = blockIdx.x;
    const int lane = threadIdx.x;
    const size_t row = (size_t)y * W;
    const uint32_t *park = reinterpret_cast<const uint32_t *>(out);
    const int nchunk = (W + 63) / 64;
    int carry = -1;
    for (int c = 0; c < nchunk; c++) {             // left -> right
        const int x = c * 64 + lane;
        const bool in = x < W;
        const bool clear = in && f[row + x] != 1;
        const int v = wave_max_scan(clear ? x : -1);
        int prev = __shfl_up(v, 1, 64);
        if (lane == 0) prev = -1;
        const int lft = prev > carry ? prev : carry;
        if (in) sleft[x] = lft < 0 ? (uint16_t)LRC_NONE : (uint16_t)lft;
        const int last = __builtin_amdgcn_readlane(v, 63);
        carry = last > carry ? last : carry;
    }
    __syncthreads();
    carry = -1;                                    // as W-1-x of the nearest unflagged column to the right
    for (int c = 0; c < nchunk; c++) {             // right -> left
        const int x = W - 1 - (c * 64 + lane);
        const bool in = x >= 0;
        const bool flagged = in && f[row + x] == 1;
        const int v = wave_max_scan(in && !flagged ? W - 1 - x : -1);
        int prev = __shfl_up(v, 1, 64);
        if (lane == 0) prev = -1;
        const int rr = prev > carry ? prev : carry;
        const int last = __builtin_amdgcn_readlane(v, 63);
        carry = last > carry ? last : carry;
        if (!in) continue;
        if (!flagged) {
            out[row + x] = dl[row + x];
            continue;
        }
        const uint32_t pk = park[row + x];
        const uint32_t up = pk & 0xFFFFu, down = pk >> 16;
        const int left = sleft[x] == LRC_NONE ? -1 : (int)sleft[x];
        int number = 0;
        double sum = 0.0;
        if (up != LRC_NONE) { number++; sum += dl[(size_t)up * W + x]; }
        if (down != LRC_NONE) { number++; sum += dl[(size_t)down * W + x]; }
        if (rr >= 0) { number++; sum += dl[row + (W - 1 - rr)]; }
        if (left >= 0) { number++; sum += dl[row + left]; }
        out[row + x] = number > 0 ? (float)(sum / number) : dl[row + x];
    }
}

__global__ __launch_bounds__(256) void median5_kernel(const float *__restrict__ src, int H, int W,
                                                      float *__restrict__ dst)
{
    const int x = blockIdx.x * 16 + (threadIdx.x & 15) + 2;
    const int y = blockIdx.y * 16 + (threadIdx.x >> 4) + 2;
    if (y + 2 >= H || x + 2 >= W) return;
    float w[25];
#pragma unroll
    for (int i = -2; i <= 2; i++)
#pragma unroll
        for (int j = -2; j <= 2; j++) w[(i + 2) * 5 + j + 2] = src[(size_t)(y + i) * W + x + j];
    float cur = 0.0f;
    // partial selection sort to the 13th smallest, same swaps as the reference
    for (int i = 0; i < 13; i++) {
        cur = w[i];
        int ci = i;
        for (int j = i + 1; j < 25; j++)
            if (cur > w[j]) { cur = w[j]; ci = j; }
        w[ci] = w[i];
    }
    dst[(size_t)y * W + x] = cur;
}

}  // namespace sde

using namespace sde;

SDE_EXPORT int sde_sgm_penalties(const uint8_t *img, int H, int W, double P1, double P2, int64_t threshold,
                                 double lambda, float *pen, void *stream)
{
    if (!img || !pen || H <= 0 || W <= 0 || lambda == 0.0) return SDE_ERR_ARG;
    const int64_t n = (int64_t)H * W;
    sgm_penalty_kernel<<<cdiv(n, 256), 256, 0, as_stream(stream)>>>(img, H, W, (float)P1, (float)P2,
                                                                     (float)(P1 / lambda), (float)(P2 / lambda),
                                                                     (double)threshold, pen);
    return launch_status();
}

SDE_EXPORT int sde_sgm_direction(const float *cv, const float *pen, int H, int W, int D, int direction, float *S,
                                 void *stream)
{
    if (!cv || !pen || !S || H < 2 || W < 2 || D <= 0 || D > 512 || direction < 0 || direction > 7)
        return SDE_ERR_ARG;
    const SgmSide a{cv, pen, S, nullptr};
    const int s = sgm_direction_impl(a, a, 1, H, W, D, direction, false, false, as_stream(stream));
    if (s != SDE_OK) return s;
    return launch_status();
}

SDE_EXPORT int sde_sgm_8path(const float *cv, const float *pen, int H, int W, int D, float *S, void *stream)
{
    return sde_sgm_8path_pair(cv, pen, S, nullptr, nullptr, nullptr, H, W, D, SDE_SGM_ACCUMULATE, stream);
}

static int sgm_pair(const float *cv_l, const float *pen_l, float *S_l, float *disp_l, const float *cv_r,
                    const float *pen_r, float *S_r, float *disp_r, int H, int W, int D, int flags, bool wta,
                    hipStream_t st)
{
    if (!cv_l || !pen_l || !S_l || H < 2 || W < 2 || D <= 0 || D > 512 ||
        (flags & ~(SDE_SGM_ACCUMULATE | SDE_SGM_ZERO_DU_PENALTIES)))
        return SDE_ERR_ARG;
    const bool two = cv_r || pen_r || S_r;
    if (two && (!cv_r || !pen_r || !S_r)) return SDE_ERR_ARG;
    if (wta && (!disp_l || (two && !disp_r))) return SDE_ERR_ARG;
    const SgmSide a{cv_l, pen_l, S_l, disp_l};
    const SgmSide b = two ? SgmSide{cv_r, pen_r, S_r, disp_r} : a;
    const bool fold_du = (flags & SDE_SGM_ZERO_DU_PENALTIES) != 0;
    for (int dir = 0; dir < 8; dir++) {
        if (dir == 1 && fold_du) continue;                               // applied in the UD pass
        const bool first = dir == 0 && !(flags & SDE_SGM_ACCUMULATE);   // UD: line = column
        // the caller's S is accumulated onto (ACCUMULATE): it may hold -0.0 -- no v_min (see dmin)
        const int s = sgm_direction_impl(a, b, two ? 2 : 1, H, W, D, dir, first, !(flags & SDE_SGM_ACCUMULATE), st,
                                         dir == 0 && fold_du,
                                         wta && dir == 7);
        if (s != SDE_OK) return s;
#ifdef SGM_GAP
        // probe builds (tools/sgm_gap_probe.py): what sits between two passes of the pair
        if (dir < 7) {
            if (SGM_GAP == 1) (void)hipStreamSynchronize(st);
            if (SGM_GAP == 2 || SGM_GAP == 3) {
                // 2: an event created with a system-scope release (L2 written back at the record)
                static hipEvent_t ev = nullptr;
                if (!ev) (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming |
                                                                 (SGM_GAP == 2 ? hipEventReleaseToSystem : 0));
                (void)hipEventRecord(ev, st);
            }
        }
#endif
    }
    return launch_status();
}

SDE_EXPORT int sde_sgm_8path_pair(const float *cv_l, const float *pen_l, float *S_l, const float *cv_r,
                                  const float *pen_r, float *S_r, int H, int W, int D, int flags, void *stream)
{
    return sgm_pair(cv_l, pen_l, S_l, nullptr, cv_r, pen_r, S_r, nullptr, H, W, D, flags, false, as_stream(stream));
}

SDE_EXPORT int sde_sgm_8path_wta_pair(const float *cv_l, const float *pen_l, float *S_l, float *disp_l,
                                      const float *cv_r, const float *pen_r, float *S_r, float *disp_r, int H, int W,
                                      int D, int flags, void *stream)
{
    return sgm_pair(cv_l, pen_l, S_l, disp_l, cv_r, pen_r, S_r, disp_r, H, W, D, flags, true, as_stream(stream));
}

SDE_EXPORT int sde_lr_check(const float *disp_l, const float *disp_r, int H, int W, uint8_t *lrc_l, uint8_t *lrc_r,
                            void *stream)
{
    if (!disp_l || !disp_r || !lrc_l || !lrc_r || H <= 0 || W <= 0) return SDE_ERR_ARG;
    lr_check_kernel<<<cdiv((int64_t)H * W, 256), 256, 0, as_stream(stream)>>>(disp_l, disp_r, H, W, lrc_l, lrc_r);
    return launch_status();
}

SDE_EXPORT int sde_lrc_fill(const float *disp_l, const uint8_t *lrc_l, int H, int W, float *out, void *stream)
{
    if (!disp_l || !lrc_l || !out || H <= 0 || W <= 0) return SDE_ERR_ARG;
    // 16-bit row / column indices (0xFFFF = none); the row pass keeps 2 B per column in LDS (<= 128 KB)
    if (H >= (int)LRC_NONE || W >= (int)LRC_NONE || out == disp_l) return SDE_ERR_ARG;
    hipStream_t st = as_stream(stream);
    const size_t smem = 2 * (size_t)W;
    if (smem > 64 * 1024) {
        static std::atomic<uint64_t> attr{0};
        once_per_device(attr, [] {
            (void)hipFuncSetAttribute((const void *)lrc_rows_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      2 * (int)LRC_NONE);
        });
    }
    lrc_cols_kernel<<<W, 64, 0, st>>>(lrc_l, H, W, reinterpret_cast<uint32_t *>(out));
    lrc_rows_kernel<<<H, 64, smem, st>>>(disp_l, lrc_l, H, W, out);
    return launch_status();
}

SDE_EXPORT int sde_median5(const float *src, int H, int W, float *dst, void *stream)
{
    if (!src || !dst || H <= 0 || W <= 0) return SDE_ERR_ARG;
    if (H < 5 || W < 5) return SDE_OK;   // no interior pixel
    dim3 grid(cdiv(W - 4, 16), cdiv(H - 4, 16));
    median5_kernel<<<grid, 256, 0, as_stream(stream)>>>(src, H, W, dst);
    return launch_status();
}
