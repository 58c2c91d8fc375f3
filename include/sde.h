/*
 * sde.h -- C ABI of the MI355X-native stereo matching path (libsde.so).
 *
 * Drop-in boundary for WHDY/SceneDepthEstimation's matching path.  The
 * reference's boundary is the Python function API of process_functional.py
 * (star-imported by match_single.py:9 / match.py:10); each entry point below
 * names the reference function or Numba kernel it replaces (file:line).
 *
 * Conventions
 *   - every pointer argument except host-side helpers is a DEVICE pointer owned
 *     by the caller; nothing here allocates, frees or synchronises, so every call
 *     is stream-ordered and capturable into a hipGraph;
 *   - `stream` is a hipStream_t passed as void* (NULL = the null stream);
 *   - feature maps are [H][W][C] float32 (channels-last, the layout
 *     compute_feature returns, process_functional.py:42-43);
 *   - return value: SDE_OK or a negative sde_status; errors are detected before
 *     any launch (argument checks) or right after it (hipGetLastError).
 *   - reentrant: no global state besides the HIP module the loader registers and the
 *     tower's grid cap (sde_set_persistent_grid, a tuning knob that does not change results).
 */
#ifndef SDE_H
#define SDE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDE_ABI_VERSION 4

typedef enum {
    SDE_OK = 0,
    SDE_ERR_ARG = -1,         /* bad size / null pointer / unsupported combination */
    SDE_ERR_LAUNCH = -2,      /* hipGetLastError() after a launch */
    SDE_ERR_WORKSPACE = -3,   /* workspace too small */
} sde_status;

typedef enum {
    SDE_LAYOUT_DHW = 0,   /* [D][H][W]: compute_cost_volume / WTA1 (process_functional.py:48,96) */
    SDE_LAYOUT_HWD = 1,   /* [H][W][D]: WTA and the GPU path (process_functional.py:76,120)      */
} sde_layout;

typedef enum {
    SDE_WTA_INIT_INF = 0, /* best=+inf, `v < best`; no winner -> -1 (WTA/WTA1, :83-110)             */
    SDE_WTA_INIT_D0 = 1,  /* best=v[0], `best > v` (WTA_and_SupixelRefinement_kernel, :805-811)      */
} sde_wta_rule;

typedef enum {
    SDE_SIDE_LEFT = 1,    /* L[y][x][d]   = cost(x, d)        (process_functional.py:130) */
    SDE_SIDE_RIGHT = 2,   /* R[y][x-d][d] = cost(x, d)        (process_functional.py:131) */
} sde_side;

/* ABI version (SDE_ABI_VERSION) and a static status string. */
int sde_abi_version(void);
const char *sde_status_string(int status);

/*
 * Cost volume, exact CPU-path numerics: cost(x,d) = -(0.0f + pairwise_sum_c
 * fl[y][x][c]*fr[y][x-d][c]) with NumPy's float32 pairwise order (no FMA).
 *   layout = SDE_LAYOUT_DHW, sides = LEFT, invalid = -0.0f
 *       replaces compute_cost_volume (process_functional.py:48-73), bit-exact;
 *   layout = SDE_LAYOUT_HWD, sides = LEFT|RIGHT, invalid = 1.0f
 *       replaces compute_cost_volume_kernel (process_functional.py:120-131)
 *       including its never-written voxels (:1111-1114).
 * out_left / out_right: D*H*W floats each (the one not requested may be NULL).
 */
int sde_cost_volume(const float *fl, const float *fr, int H, int W, int C, int D, int layout,
                    int sides, float invalid, float *out_left, float *out_right, void *stream);

/*
 * First-minimum over d of an existing volume -> disparity as float32.
 * Replaces WTA1 (process_functional.py:96-113, DHW), WTA (:76-93, HWD) and
 * WTA_and_SupixelRefinement_kernel (:800-837, HWD + SDE_WTA_INIT_D0).
 * A pixel without a winner (all NaN / +inf under INIT_INF) gets -1.0f; the
 * reference asserts there (:89,109) and the Python layer raises.
 */
int sde_wta(const float *vol, int H, int W, int D, int layout, int rule, float *disp, void *stream);

/* sde_cv_wta modes: both give identical (bit-exact) outputs. */
#define SDE_CV_EXACT 0       /* every voxel in NumPy's pairwise order on VALU                                */
#define SDE_CV_CERTIFIED 1   /* f16x3 (row sweep) or bf16x3 MFMA scores + rigorous error bound; pixels whose
                                winner is not certified by a 2*eps gap are resolved by the exact scan
                                (needs workspace) */

/* Workspace bytes sde_cv_wta needs in SDE_CV_CERTIFIED mode (work-list of unresolved pixels). */
int64_t sde_cv_wta_workspace_bytes(int H, int W);

/*
 * Fused cost volume + WTA over the disparity shard [d0, d1) without
 * materialising the volume: WTA1(compute_cost_volume(fl, fr, D)) bit-exact when
 * d0 = 0, d1 = D (process_functional.py:48-73 + :96-113).  Outputs (each
 * optional, NULL to skip): disp (float32 argmin), min_cost (float32 first-min
 * cost, bit-exact) and argmin (int32, -1 if none), [H][W].  Shards merge
 * bit-exactly with sde_argmin_merge (ties -> lower d).  mode: SDE_CV_EXACT or
 * SDE_CV_CERTIFIED (C == 64; other C always run exact).  The workspace's first
 * 256 bytes hold, after the call, 64 uint32 counters whose sum is the number of
 * pixels the certified mode resolved exactly (one per 256-disparity chunk when
 * d1 - d0 exceeds the row sweep's window, e.g. D = 512; word 0 otherwise).
 */
int sde_cv_wta(const float *fl, const float *fr, int H, int W, int C, int d0, int d1, float *disp,
               float *min_cost, int32_t *argmin, int mode, void *workspace, int64_t workspace_bytes,
               void *stream);

/*
 * Split a [npix][64] float32 feature map for SDE_CV_CERTIFIED: hi = bf16_rne(x),
 * lo = bf16_rne(x - hi) (both [npix][64] bf16 bit patterns) and norm[p] >= the
 * pixel's L2 norm.  The tower can emit the same three outputs from its last
 * layer (sde_tower_forward's feat_hi / feat_lo / feat_norm).
 */
int sde_feature_split(const float *feat, int64_t npix, int C, uint16_t *hi, uint16_t *lo, float *norm, void *stream);

/* Workspace bytes for sde_cv_wta_split (work-list of unresolved pixels). */
int64_t sde_cv_wta_split_workspace_bytes(int H, int W);

/*
 * SDE_CV_CERTIFIED on pre-split operands (no split pass): same outputs and
 * bit-exactness as sde_cv_wta.  fl / fr (float32) are read only for the exact
 * resolution of uncertified pixels and for min_cost.
 */
int sde_cv_wta_split(const float *fl, const float *fr, const uint16_t *fl_hi, const uint16_t *fl_lo,
                     const float *fl_norm, const uint16_t *fr_hi, const uint16_t *fr_lo, const float *fr_norm,
                     int H, int W, int d0, int d1, float *disp, float *min_cost, int32_t *argmin, void *workspace,
                     int64_t workspace_bytes, void *stream);

/*
 * Ordered merge of per-shard (min, argmin) pairs: shard s covers a disparity
 * range that precedes shard s+1's; strict `<` keeps the earliest on ties.
 * mins/args: [nshards][npix].  disp: float32 [npix].
 */
int sde_argmin_merge(const float *mins, const int32_t *args, int nshards, int64_t npix, float *disp,
                     void *stream);

/* ---------------------------------------------------------------------- */
/* MC-CNN-fast branch (mc_cnn_brunch.py:31-48; compute_feature's sess.run,   */
/* process_functional.py:11-45).  nlayers 3x3 VALID convs, nf = 64 maps.     */
/* ---------------------------------------------------------------------- */

/* Workgroups of the persistent tower kernels (default 0: one per CU of the device).  A positive value caps
 * the grid -- for a tower sharing the device with other work on CU-masked streams (hipExtStreamCreateWithCUMask),
 * where one workgroup per device CU would leave the last ones waiting for the other stream's CUs.  Process-wide;
 * results do not depend on it. */
int sde_set_persistent_grid(int cus);

/* Tower arithmetic (flags of sde_tower_forward / sde_tower_layer). */
#define SDE_TOWER_FP32 0      /* v_mfma_f32_32x32x2_f32: exact fp32 products, fp32 accumulation            */
#define SDE_TOWER_BF16X6 1    /* fp32 operands split exactly into 3 bf16 parts, the 6 leading partial products
                                 on v_mfma_f32_32x32x16_bf16, fp32 accumulation: fp32-level error, 2.67x rate */
#define SDE_TOWER_F16X3 8     /* operands scaled by powers of two and split exactly into 2 fp16 parts, the 3
                                 leading partial products on v_mfma_f32_32x32x16_f16, fp32 accumulation:
                                 ~2^-22 relative per product (fp32-level), 5.3x the fp32 matrix rate.
                                 The scalings need per-layer bound words: sde_tower_forward keeps them
                                 in its workspace; single layers go through sde_tower_layer_scaled. */
/* sde_tower_layer only, with SDE_TOWER_BF16X6 or SDE_TOWER_F16X3: intermediate activations in the c-block-major
 * layout [nf/16][h][w][16] that sde_tower_forward uses between layers (16-channel blocks
 * contiguous per pixel run).  IN: `in` of a layer >= 3; OUT: `out` of a layer < nlayers. */
/* With SDE_TOWER_F16X3 only: run the 64 -> 64 layers (3..L) with the Winograd F(2x2, 3x3) kernel
 * instead of the direct 3x3 kernel (same arithmetic contract and error class, 2.25x fewer MFMA
 * products, more VALU; slower than the direct kernel at 1024^2 on MI355X -- DESIGN.md 3.2). */
#define SDE_TOWER_WINOGRAD 16
/* With SDE_TOWER_F16X3 only: run the 64 -> 64 layers on the v_mfma_f32_32x32x16_f16 direct kernel instead of
 * the default v_mfma_f32_16x16x32_f16 one (same arithmetic contract). */
#define SDE_TOWER_MFMA32 32
#define SDE_TOWER_IN_CBLOCK 2
#define SDE_TOWER_OUT_CBLOCK 4
/* F16X3 split activations (sde_tower_layer_scaled / sde_tower_layer_batch; what sde_tower_forward uses
 * between the 64->64 layers of the default f16x3 tower): OUT_SPLIT writes a layer's ReLU outputs scaled by
 * 2^sigma and split exactly into two fp16 parts, per image 16 planes [cblk32 2][part 2][quarter 4] of
 * [h][w][8 fp16] (256 B per pixel, as fp32 [h][w][64]), and publishes 2^sigma at out_absmax[32] (per image);
 * IN_SPLIT reads that layout and in_absmax[32] (LDS-DMA staging, no arithmetic).  2^sigma comes from an
 * a-priori bound of the outputs (max |b| + L1 * input bound, no fp16 overflow).  Layers >= 3 (IN) and
 * < nlayers (OUT), a layer between them with both or neither; at most 32 layers, fewer than 2^24 input pixels; bound-word arrays extending >= 33 words past
 * the word passed (batches: amax_stride >= 64 words per image, so no image's scale word lands on the next image's row); not with the CBLOCK flag of the same side, WINOGRAD or MFMA32. */
#define SDE_TOWER_IN_SPLIT 64
#define SDE_TOWER_OUT_SPLIT 128

/* Number of floats of the packed (device-layout) weight blob (fp32 + pre-split bf16 planes). */
int64_t sde_tower_packed_floats(int nlayers, int nf);

/* 1 if this build's sde_tower_forward* pass split activations (SDE_TOWER_OUT_SPLIT / IN_SPLIT layouts) between
 * the default f16x3 tower's 64 -> 64 layers, 0 if they pass c-block-major fp32 (the default build).  Layer-by-layer
 * drivers that must reproduce the forward's bits (the row-band tower of the multi-GPU schemes) follow it. */
int sde_tower_split_act(void);

/*
 * HOST helper: pack TF HWIO weights ([3][3][Cin][nf], `conv{k}/weights:0`) and
 * biases ([nf], `conv{k}/biases:0`) of nlayers layers into `packed` (host memory,
 * sde_tower_packed_floats() floats).  Copy the blob to the device once.
 */
int sde_tower_pack_weights(const float *const *hwio, const float *const *biases, int nlayers, int nf,
                           float *packed);

/* Device workspace bytes needed by sde_tower_forward for an H x W output. */
int64_t sde_tower_workspace_bytes(int H, int W, int nlayers, int nf);

/*
 * img_pad: float32 [(H+2*nlayers)][(W+2*nlayers)] zero-padded normalised image
 * (process_functional.py:13-19).  feat: float32 [H][W][nf], L2-normalised per
 * pixel (mc_cnn_brunch.py:48).  packed: device copy of the packed weights.
 * feat_hi / feat_lo / feat_norm (optional, NULL to skip; nlayers >= 2): the
 * last layer's epilogue also writes the bf16 split planes and per-pixel norm
 * bound that sde_cv_wta_split consumes (same layout as sde_feature_split).
 */
int sde_tower_forward(const float *img_pad, int H, int W, const float *packed, int nlayers, int nf,
                      float *feat, void *workspace, int64_t workspace_bytes, int flags, uint16_t *feat_hi,
                      uint16_t *feat_lo, float *feat_norm, void *stream);

/*
 * sde_tower_forward over nimg images of one size in one set of launches (the
 * split arithmetics tile the whole batch in one persistent grid: fewer launches,
 * less tail imbalance).  img_pad: [nimg][H+2*nlayers][W+2*nlayers]; feat:
 * [nimg][H][W][nf]; feat_hi / feat_lo: [nimg][H][W][nf]; feat_norm: [nimg][H][W].
 * Each image gets the same result as sde_tower_forward on it alone.
 */
int64_t sde_tower_batch_workspace_bytes(int H, int W, int nimg, int nlayers, int nf);
int sde_tower_forward_batch(const float *img_pad, int nimg, int H, int W, const float *packed, int nlayers, int nf,
                            float *feat, void *workspace, int64_t workspace_bytes, int flags, uint16_t *feat_hi,
                            uint16_t *feat_lo, float *feat_norm, void *stream);

/*
 * One layer of the tower as a single kernel launch (for per-layer timing and
 * pipelining): layer == 2 -> conv1+conv2 fused, `in` = padded image Hin x Win
 * floats, out (Hin-4) x (Win-4) x nf; layer in 3..nlayers -> `in` = Hin x Win x
 * nf activations, out (Hin-2) x (Win-2) x nf.  Layer nlayers L2-normalises.
 */
int sde_tower_layer(const float *in, int Hin, int Win, const float *packed, int nlayers, int nf, int layer,
                    float *out, int flags, uint16_t *feat_hi, uint16_t *feat_lo, float *feat_norm, void *stream);

/*
 * sde_tower_layer with the SDE_TOWER_F16X3 bound words (ignored by the other
 * arithmetics): in_absmax -> device float, an upper bound of |input| (layer 2:
 * of |image|; the kernel bounds conv1's output from it); out_absmax -> device
 * float the launch atomically maxes its (non-negative) outputs into, zeroed by
 * the caller (may be NULL for the last layer).
 */
int sde_tower_layer_scaled(const float *in, int Hin, int Win, const float *packed, int nlayers, int nf, int layer,
                           float *out, int flags, uint16_t *feat_hi, uint16_t *feat_lo, float *feat_norm,
                           const float *in_absmax, float *out_absmax, void *stream);

/*
 * sde_tower_layer_scaled over nimg images per launch (no split outputs): image i
 * reads in + i * in_stride, writes out + i * out_stride (floats; the last layer's
 * out_stride must be (Hin-2)*(Win-2)*nf) and uses bound words in_absmax /
 * out_absmax + i * amax_stride.
 */
int sde_tower_layer_batch(const float *in, int nimg, int64_t in_stride, int Hin, int Win, const float *packed,
                          int nlayers, int nf, int layer, float *out, int64_t out_stride, int flags,
                          const float *in_absmax, float *out_absmax, int amax_stride, void *stream);

/* sde_absmax_f32 over nimg arrays of n floats (x + i * n) into absmax[i * absmax_stride]. */
int sde_absmax_f32_batch(const float *x, int nimg, int64_t n, float *absmax, int absmax_stride, void *stream);

/* *absmax = max(*absmax, max |x[i]|) over n floats (float bits compared as integers; *absmax >= +0). */
int sde_absmax_f32(const float *x, int64_t n, float *absmax, void *stream);

/*
 * Preprocess on device (match_single.py:34-43 + process_functional.py:13-19):
 * u8 image -> (I - mean) / std (population std, float32) written into the
 * interior of the zero-padded buffer out_pad [(H+2*pad)][(W+2*pad)] -- bit for bit
 * NumPy's np.mean / np.std over axes (0, 1) of the float32 image (its pairwise
 * float32 reduction order) and the float32 elementwise expression.
 * scratch: sde_preprocess_scratch_bytes(H, W) of device memory per image (the
 * statistics and NumPy's per-8192-element partial sums; no initialisation needed).
 */
int64_t sde_preprocess_scratch_bytes(int H, int W);
int sde_preprocess_u8(const uint8_t *img, int H, int W, int pad, float *out_pad, void *scratch,
                      void *stream);

/* sde_preprocess_u8 over nimg images per launch: imgs [nimg][H][W], out_pad
 * [nimg][H+2*pad][W+2*pad], scratch nimg * sde_preprocess_scratch_bytes(H, W). */
int sde_preprocess_u8_batch(const uint8_t *imgs, int nimg, int H, int W, int pad, float *out_pad, void *scratch,
                            void *stream);

/* ---------------------------------------------------------------------- */
/* Semi-global matching (GPU path of disparity_compute_by_gpu,               */
/* process_functional.py:1093-1267).                                         */
/* ---------------------------------------------------------------------- */

/* sgm_penelty_kernel (process_functional.py:134-262): pen [H][W][16] float32. */
int sde_sgm_penalties(const uint8_t *img, int H, int W, double P1, double P2, int64_t threshold,
                      double lambda, float *pen, void *stream);

/*
 * 8-path SGM for one side (SGM_*_kernel, process_functional.py:265-797, launch
 * order :1166-1203): S [H][W][D] += path costs, direction order UD, DU, LR, RL,
 * UD-LR, DU-LR, UD-RL, DU-RL; fp64 recurrence, float32 S.  The caller zeroes S
 * (the reference uploads np.zeros, :1116-1119).  cv: [H][W][D] with invalid
 * voxels = 1.0 (sde_cost_volume HWD).  Requires H >= 2, W >= 2.
 */
int sde_sgm_8path(const float *cv, const float *pen, int H, int W, int D, float *S, void *stream);

/*
 * Both image sides of the reference's per-direction k loop (:1166-1203) in one
 * launch per direction (the (cv_r, pen_r, S_r) triple may be all NULL for one
 * side).  flags = 0: S := the 8-path sum starting from zero, so the caller need
 * not zero S and the first direction does not read it (same values as zeroing
 * S then accumulating); SDE_SGM_ACCUMULATE: S += path costs as sde_sgm_8path.
 */
#define SDE_SGM_ACCUMULATE 1
/* The caller asserts that penalty channels 0/1 are zero (sde_sgm_penalties never writes
 * them, as the reference's sgm_penelty_kernel): direction DU then reduces to S += C (+0.0
 * off its first row) for finite costs and is folded into the UD pass (7 passes instead of
 * 8, same values).  A column holding a non-finite cost, or a non-finite UD penalty
 * (channels 2/3), is detected and recomputed for both directions in the reference's exact
 * arithmetic, so the fold gives the unfolded values for any costs. */
#define SDE_SGM_ZERO_DU_PENALTIES 2
int sde_sgm_8path_pair(const float *cv_l, const float *pen_l, float *S_l, const float *cv_r, const float *pen_r,
                       float *S_r, int H, int W, int D, int flags, void *stream);

/*
 * sde_sgm_8path_pair fused with WTA_and_SupixelRefinement_kernel (process_functional.py:800-837,
 * the same first-min rule as sde_wta(..., SDE_WTA_INIT_D0)): the last direction (DU-RL) reduces
 * each pixel's final S to its disparity in disp [H][W] float32 instead of storing S, so on
 * return S holds the sum of the first seven directions.  disp_r may be NULL only with the
 * right triple.  Same flags and values as sde_sgm_8path_pair followed by sde_wta.
 */
int sde_sgm_8path_wta_pair(const float *cv_l, const float *pen_l, float *S_l, float *disp_l, const float *cv_r,
                           const float *pen_r, float *S_r, float *disp_r, int H, int W, int D, int flags,
                           void *stream);

/* One direction (0..7 in the order above) of sde_sgm_8path. */
int sde_sgm_direction(const float *cv, const float *pen, int H, int W, int D, int direction, float *S,
                      void *stream);

/* ---------------------------------------------------------------------- */
/* Cross-based cost aggregation.  BUILD-DEFINED: the reference has none      */
/* (SURVEY.md sec. 0.3 -- only the buffer name d_cost_volumel_after_aggr,   */
/* process_functional.py:268,347, and an unused timer label, match.py:98);  */
/* the definition is restated on the CPU under oracle/ (parity unpinned vs */
/* the reference, bit-exact vs that restatement).                          */
/* ---------------------------------------------------------------------- */
#define SDE_CBCA_MAX_L1 32

/*
 * Cross arms of an f32 image (row pitch in elements, e.g. the z-normalised
 * interior of the tower's padded input): for left/right/up/down the largest
 * k <= L1-1 with |I(p) - I(p + j*dir)| < tau for all 1 <= j <= k inside the
 * image.  arms u32 [H][W] = l | r<<8 | u<<16 | d<<24.
 */
int sde_cbca_arms(const float *img, int64_t pitch, int H, int W, int L1, float tau, uint32_t *arms, void *stream);

/*
 * Definition v2 (round 4; the CPU restatement under oracle/ states it in full): volumes are
 * aggregated in LEFT coordinates (a right-referenced volume through
 * R(y,x',d) = L(y,x'+d,d)); voxels whose right-image pixel is outside the
 * image pass through unchanged; support arms = min(left-image arm, right-image
 * arm); fp64 prefix chains restart per segment of SDE_CBCA_SEG positions at
 * kS - (L1 - 1); the mean multiplies by the correctly rounded fp64 1/count.
 * Consequence: the aggregation of R = shear(L) is shear(aggregation of L).
 */
#define SDE_CBCA_SEG 256

/* Workspace of the aggregation entry points (a column-major copy of the left
 * image's arms for the vertical pass): 4 * W * roundup(H, 4) bytes (ABI 3 asked
 * for 8 *: larger buffers stay valid). */
size_t sde_cbca_workspace_bytes(int H, int W);

/*
 * iters x (horizontal pass, vertical pass) on an [H][W][D] volume, in place
 * in cv (tmp: same size, scratch).  side SDE_SIDE_LEFT: left-referenced volume,
 * the other pixel is x - d (arms_ref = left image arms, arms_other = right);
 * SDE_SIDE_RIGHT: x + d (arms_ref = right image, arms_other = left; done as a
 * rotation into left coordinates, the aggregation, and the rotation back).
 * L1 as given to sde_cbca_arms (arms must not exceed L1 - 1).
 */
int sde_cbca(float *cv, float *tmp, const uint32_t *arms_ref, const uint32_t *arms_other, int H, int W, int D,
             int side, int L1, int iters, void *ws, size_t ws_bytes, void *stream);

/*
 * sde_cbca on both volumes of a pair (same results as sde_cbca(cv_l, tmp_l,
 * arms_l, arms_r, SDE_SIDE_LEFT) and sde_cbca(cv_r, tmp_r, arms_r, arms_l,
 * SDE_SIDE_RIGHT)) for any two volumes; the four buffers must be distinct.
 * Build-defined like sde_cbca: the reference only names the aggregated
 * volumes d_cost_volumel/r_after_aggr (process_functional.py:268,347).
 */
int sde_cbca_pair(float *cv_l, float *tmp_l, float *cv_r, float *tmp_r, const uint32_t *arms_l,
                  const uint32_t *arms_r, int H, int W, int D, int L1, int iters, void *ws, size_t ws_bytes,
                  void *stream);

/*
 * The GPU path's pair (d_cost_volumel/r_after_aggr, process_functional.py:268,
 * 347): cv_l aggregated in place (tmp: scratch), then every valid voxel of cv_r
 * set to its shear, cv_r(y,x',d) = cv_l(y,x'+d,d) for x'+d < W (the others are
 * left as they are).  Equals sde_cbca_pair whenever cv_r's valid voxels are
 * the shear of cv_l's -- as sde_cost_volume(..., SDE_LAYOUT_HWD) writes them --
 * at half its traffic: one volume aggregated, one shear.
 */
int sde_cbca_lr(float *cv_l, float *cv_r, float *tmp, const uint32_t *arms_l, const uint32_t *arms_r, int H, int W,
                int D, int L1, int iters, void *ws, size_t ws_bytes, void *stream);
/* sde_cbca* shape limits (32-bit offsets, refused with SDE_ERR_ARG): D <= 512,
 * (5R + 5) * 4*W*D < 2^31 with R = 13 (L1 <= 14), 15 (L1 <= 16) or 31, and
 * 4 * roundup(H, 4) * W < 2^31. */

/* The fp64 reciprocals the aggregation multiplies by, out[i] = 1/(i+1) as the
 * kernels compute it (the tests check them against the IEEE quotient). */
int sde_cbca_reciprocals(double *out, int n, void *stream);

/* is_error_match_kernel (process_functional.py:977-1000): lrc_l/lrc_r u8 [H][W], caller-zeroed. */
int sde_lr_check(const float *disp_l, const float *disp_r, int H, int W, uint8_t *lrc_l, uint8_t *lrc_r,
                 void *stream);

/* LRC_kernel left output (process_functional.py:1003-1088).  Two linear scans instead of
 * the reference's per-pixel walks; `out` doubles as scratch, so out != disp_l.  Requires
 * H < 65535 and W < 65535 (16-bit row / column indices; the row pass keeps 2 B per column in LDS). */
int sde_lrc_fill(const float *disp_l, const uint8_t *lrc_l, int H, int W, float *out, void *stream);

/* Median_Filter_kernel (process_functional.py:840-879): 5x5 median of src into the interior of dst. */
int sde_median5(const float *src, int H, int W, float *dst, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SDE_H */
