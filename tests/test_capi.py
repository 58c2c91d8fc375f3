"""CPU: libsde.so loads, exports exactly what include/sde.h declares, and its host-side
entry points behave (no GPU needed: argument checks return before any launch)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from scenedepthestimation_amd import _lib
from scenedepthestimation_amd._build import LIB


def test_header_and_binding_agree():
    declared = set(_lib.header_functions())
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = set(_lib.header_functions()) - exported
    assert not missing, missing
    # nothing else leaks out of the C ABI (hidden visibility)
    extra = {s for s in exported if s.startswith("sde_")} - set(_lib.header_functions())
    assert not extra, extra


def test_version_and_status_strings():
    assert _lib.lib.sde_abi_version() == 4 == _lib.SDE_ABI_VERSION
    # the header's version is the binding's
    import re
    with open(_lib.os.path.join(_lib.INCLUDE, "sde.h")) as fh:
        assert int(re.search(r"#define SDE_ABI_VERSION (\d+)", fh.read()).group(1)) == _lib.SDE_ABI_VERSION


def test_cbca_segment_constant_matches_oracle():
    import re
    from oracle import oracle
    with open(_lib.os.path.join(_lib.INCLUDE, "sde.h")) as fh:
        assert int(re.search(r"#define SDE_CBCA_SEG (\d+)", fh.read()).group(1)) == oracle.cbca_seg()
    assert _lib.lib.sde_status_string(0) == b"ok"
    assert _lib.lib.sde_status_string(-1) == b"invalid argument"
    assert _lib.lib.sde_status_string(-3) == b"workspace too small"


def test_tower_packing_matches_layout():
    from scenedepthestimation_amd import mc_cnn, ops
    L = 3
    w = mc_cnn.synthetic_weights(L, seed=5)
    hw, hb = mc_cnn.layer_lists(w, L)
    packed = ops.pack_tower_weights(hw, hb)
    LW = 9 * 64 * 64
    LF = 64 + LW + 3 * LW // 2                    # bias | f32 [tap][n][c] | 3 bf16 parts
    LWINO = LF + LW + 8                           # | 2 fp16 parts of W * 2^tau | F16 header (8 floats)
    LK = LWINO + 16 * 64 * 64 + 4                 # | 2 fp16 parts of U * 2^tau_u (Winograd) | header
    assert packed.size == ops.tower_packed_floats(L) == 64 + 576 + 2 * LK
    assert np.array_equal(packed[:64], hb[0])
    assert np.array_equal(packed[64:640], hw[0].reshape(-1))
    for l in (1, 2):
        base = 640 + (l - 1) * LK
        assert np.array_equal(packed[base:base + 64], hb[l])
        blob = packed[base + 64:base + 64 + LW].reshape(9, 64, 64)            # [tap][n][c]
        ref = hw[l].reshape(9, 64, 64).transpose(0, 2, 1)                     # HWIO [tap][c][n] -> [tap][n][c]
        assert np.array_equal(blob, ref)
        # bf16 parts in A-fragment order [mtile 2][cblock 4][tap 9][part 3][lane 64][8]:
        # lane = ((c % 16) >= 8) * 32 + n % 32, element c % 8 (conv64_x6p_kernel)
        frag = packed[base + 64 + LW:base + LF].view(np.uint16).reshape(2, 4, 9, 3, 2, 32, 8)
        # -> [part][tap][n = mt*32 + lane%32][c = cb*16 + half*8 + e]
        planes = frag.transpose(3, 2, 0, 5, 1, 4, 6).reshape(3, 9, 64, 64)
        as_f32 = (planes.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
        # the three bf16 parts sum exactly to the fp32 weight (RNE splits, exact residuals)
        assert np.array_equal(as_f32.sum(0), ref.astype(np.float64))
        hi = as_f32[0]
        assert np.all(np.abs(ref - hi) <= np.abs(ref) * 2.0 ** -8)
        # F16X3: header {2^-tau, conv1 L1 bound, max |b1|, 0, L1 bound, max |b|, 0, 0}; two fp16 parts of
        # W * 2^tau in the same fragment order with 2 parts, max |W| * 2^tau in [2^14, 2^15)
        hdr = packed[base + LF + LW:base + LWINO]
        lk = np.abs(hw[l].reshape(9 * 64, 64).astype(np.float64)).sum(0).max()   # max_n sum_{tap,c} |w|
        assert lk <= hdr[4] <= lk * (1 + 4e-6) and hdr[5] == np.abs(hb[l]).max() and hdr[6] == hdr[7] == 0
        tau = -int(np.log2(hdr[0]))
        assert hdr[0] == 2.0 ** -tau and 2.0 ** 14 <= np.abs(ref).max() * 2.0 ** tau < 2.0 ** 15
        l1 = np.abs(hw[0].reshape(9, 64).astype(np.float64)).sum(0).max()
        assert l1 <= hdr[1] <= l1 * (1 + 4e-6) and hdr[2] == np.abs(hb[0]).max() and hdr[3] == 0
        f16 = packed[base + LF:base + LF + LW].view(np.float16).reshape(2, 4, 9, 2, 2, 32, 8)
        hparts = f16.transpose(3, 2, 0, 5, 1, 4, 6).reshape(2, 9, 64, 64).astype(np.float64)
        scaled = ref.astype(np.float64) * 2.0 ** tau
        assert np.array_equal(hparts[0], scaled.astype(np.float16).astype(np.float64))   # RNE hi part
        assert np.all(np.abs(hparts.sum(0) - scaled) <= np.abs(scaled) * 2.0 ** -22 + 2.0 ** -25)
        # Winograd F(2x2,3x3): U[xi = 4i + j][n][c] = (G g G^T)[i][j] formed in fp64, scaled by
        # 2^tau_u (max |U| 2^tau_u in [2^14, 2^15)), two fp16 parts in A-fragment order
        # [xi 16][mtile 2][cblock 4][part 2][lane 64][8]
        G = np.array([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]])
        g = hw[l].reshape(3, 3, 64, 64).astype(np.float64)                    # [ky][kx][c][n]
        U = np.einsum("ia,abcn,jb->ijnc", G, g, G).reshape(16, 64, 64)
        whdr = packed[base + LWINO + 16 * 64 * 64:base + LK]
        tau_u = -int(np.log2(whdr[0]))
        assert whdr[0] == 2.0 ** -tau_u and tuple(whdr[1:]) == (0, 0, 0)
        assert 2.0 ** 14 <= np.abs(U).max() * 2.0 ** tau_u < 2.0 ** 15
        u16 = packed[base + LWINO:base + LWINO + 16 * 64 * 64].view(np.float16).reshape(16, 2, 4, 2, 2, 32, 8)
        uparts = u16.transpose(3, 0, 1, 5, 2, 4, 6).reshape(2, 16, 64, 64).astype(np.float64)
        uscaled = U * 2.0 ** tau_u
        assert np.array_equal(uparts[0], uscaled.astype(np.float16).astype(np.float64))
        assert np.all(np.abs(uparts.sum(0) - uscaled) <= np.abs(uscaled) * 2.0 ** -22 + 2.0 ** -25)
    assert ops.tower_workspace_bytes(100, 80, 5) == 2 * 106 * 86 * 64 * 4 + 256
    assert ops.tower_workspace_bytes(100, 80, 2) == 256


def test_argument_validation_without_gpu():
    lib = _lib.lib
    ERR = -1
    assert lib.sde_cost_volume(None, None, 4, 4, 64, 4, 0, 1, ctypes.c_float(0.0), None, None, None) == ERR
    assert lib.sde_cost_volume(1, 1, 4, 4, 64, 4, 0, 2, ctypes.c_float(0.0), 1, 1, None) == ERR   # right needs HWD
    assert lib.sde_cv_wta(1, 1, 4, 4, 64, 5, 5, 1, None, None, 0, None, 0, None) == ERR           # empty shard
    assert lib.sde_cv_wta(1, 1, 4, 4, 64, 0, 5, 1, None, None, 1, None, 0, None) == -3            # workspace
    assert lib.sde_cv_wta(1, 1, 4, 4, 64, 0, 5, 1, None, None, 7, None, 0, None) == ERR           # mode
    assert lib.sde_wta(1, 4, 4, 4, 7, 0, 1, None) == ERR                                            # bad layout
    assert lib.sde_sgm_8path(1, 1, 1, 5, 8, 1, None) == ERR                                        # H < 2
    assert lib.sde_sgm_8path(1, 1, 5, 5, 513, 1, None) == ERR                                      # D > 512
    assert lib.sde_sgm_direction(1, 1, 5, 5, 8, 8, 1, None) == ERR                                 # direction
    N = None
    assert lib.sde_tower_forward(1, 8, 8, 1, 5, 32, 1, N, 0, 0, N, N, N, N) == ERR                 # nf != 64
    assert lib.sde_tower_forward(1, 8, 8, 1, 5, 64, 1, N, 0, 0, N, N, N, N) == -3                  # workspace
    assert lib.sde_tower_forward(1, 8, 8, 1, 5, 64, 1, 1, 1 << 30, 4, N, N, N, N) == ERR           # bad flags
    assert lib.sde_tower_forward(1, 8, 8, 1, 5, 64, 1, 1, 1 << 30, 16, N, N, N, N) == ERR          # Winograd w/o f16x3
    assert lib.sde_tower_forward(1, 8, 8, 1, 5, 64, 1, 1, 1 << 30, 17, N, N, N, N) == ERR          # ... with bf16x6
    assert lib.sde_tower_forward(1, 8, 8, 1, 5, 64, 1, 1, 1 << 30, 0, 1, N, N, N) == ERR           # hi without lo
    assert lib.sde_tower_layer(1, 8, 8, 1, 5, 64, 1, 1, 0, N, N, N, N) == ERR                      # layer 1
    assert lib.sde_tower_layer(1, 8, 8, 1, 5, 64, 3, 1, 8, N, N, N, N) == ERR                      # f16x3: bounds
    assert lib.sde_tower_layer_scaled(1, 8, 8, 1, 5, 64, 3, 1, 8, N, N, N, N, 1, N) == ERR         # no out bound
    assert lib.sde_tower_layer_scaled(1, 8, 8, 1, 5, 64, 3, 1, 9, N, N, N, 1, 1, N) == ERR         # two precisions
    assert lib.sde_tower_forward(1, 8, 8, 1, 5, 64, 1, 1, 1 << 30, 9, N, N, N, N) == ERR           # two precisions
    assert lib.sde_tower_forward(1, 8, 8, 1, 5, 64, 1, 1, 1 << 30, 8 | 2, N, N, N, N) == ERR       # layout flag
    assert lib.sde_tower_forward(1, 8, 8, 1, 5, 64, 1, 1, 1 << 30, 8 | 128, N, N, N, N) == ERR     # split flag
    scaled = lambda layer, flags, L=5: lib.sde_tower_layer_scaled(1, 8, 8, 1, L, 64, layer, 1, flags, N, N, N, 1, 1, N)
    assert scaled(3, 64) == ERR                         # split activations without f16x3
    assert scaled(2, 8 | 64) == ERR                     # layer 2 reads the image
    assert scaled(5, 8 | 128) == ERR                    # the last layer writes features
    assert scaled(3, 8 | 64) == ERR and scaled(3, 8 | 128) == ERR   # a middle layer: both or neither
    assert scaled(3, 8 | 64 | 128 | 2) == ERR           # IN_SPLIT with IN_CBLOCK
    assert scaled(3, 8 | 64 | 128 | 32) == ERR          # with the 32x32x16 kernel
    assert scaled(3, 8 | 64 | 128, L=33) == ERR         # the scale word needs <= 32 layers
    # split activations over a batch: image i's scale word (bound word + 32) must not reach image i + 1's row
    batch = lambda stride: lib.sde_tower_layer_batch(1, 2, 8 * 8 * 64, 8, 8, 1, 5, 64, 3, 1, 6 * 6 * 64,
                                                     8 | 64 | 128, 1, 1, stride, N)
    for stride in (33, 34, 35, 63):
        assert batch(stride) == ERR, stride
    # the split pixel limit is on the split plane: layer 2 writes a 4094 x 4092 plane (< 2^24) from a 4098 x 4096
    # image (> 2^24) -- accepted by the checks (no GPU here: the launch itself fails); a 4098 x 4096 split INPUT
    # plane is refused
    big = lambda layer, flags, h, w: lib.sde_tower_layer_scaled(1, h, w, 1, 5, 64, layer, 1, flags, N, N, N, 1, 1, N)
    assert big(2, 8 | 128, 4098, 4096) not in (ERR, 0)
    assert big(3, 8 | 64 | 128, 4098, 4096) == ERR
    from scenedepthestimation_amd import ops
    assert lib.sde_tower_split_act() in (0, 1) and ops.TOWER_SPLIT_ACT == bool(lib.sde_tower_split_act())
    assert lib.sde_absmax_f32(N, 4, 1, N) == ERR
    assert lib.sde_feature_split(1, 10, 32, 1, 1, 1, N) == ERR                                     # C != 64
    assert lib.sde_cv_wta_split(1, 1, 1, 1, 1, 1, 1, 1, 4, 4, 0, 4, 1, N, N, 1, 0, N) == -3        # workspace
    assert lib.sde_cv_wta_split(1, 1, N, 1, 1, 1, 1, 1, 4, 4, 0, 4, 1, N, N, 1, 1 << 20, N) == ERR
    assert lib.sde_preprocess_u8(1, 4, 4, 5, 1, None, None) == ERR
    assert lib.sde_preprocess_scratch_bytes(0, 4) == -1
    # [mean, std, -, -] + two floats per 8192-pixel piece (sums, sums of squares), rounded to 256 B
    assert lib.sde_preprocess_scratch_bytes(1024, 1024) == 1280 and lib.sde_preprocess_scratch_bytes(3, 5) == 256
    assert lib.sde_tower_packed_floats(0, 64) == -1
    W8 = lib.sde_cbca_workspace_bytes(4, 8)
    assert W8 == 4 * 8 * 4 and lib.sde_cbca_workspace_bytes(5, 7) == 4 * 7 * 8 and lib.sde_cbca_workspace_bytes(0, 7) == 0
    assert lib.sde_cbca_pair(1, 2, 3, 1, 5, 6, 4, 8, 8, 14, 1, 7, W8, N) == ERR                   # aliased buffers
    assert lib.sde_cbca_pair(1, 2, 3, 4, 5, 6, 4, 8, 8, 33, 1, 7, W8, N) == ERR                   # L1 > 32
    assert lib.sde_cbca_pair(1, 2, 3, 4, 5, 6, 4, 8, 8, 14, 1, 7, W8 - 1, N) == ERR               # workspace
    assert lib.sde_cbca_pair(1, 2, 3, 4, 5, 6, 4, 8, 8, 14, 1, N, W8, N) == ERR                   # no workspace
    assert lib.sde_cbca(1, 2, 3, 4, 4, 8, 513, 1, 14, 1, 7, W8, N) == ERR                         # D > 512
    assert lib.sde_cbca(1, 1, 3, 4, 4, 8, 8, 1, 14, 1, 7, W8, N) == ERR                           # cv == tmp
    assert lib.sde_cbca(1, 2, 3, 4, 4, 8, 8, 3, 14, 1, 7, W8, N) == ERR                           # side
    assert lib.sde_cbca_lr(1, 2, 2, 4, 5, 4, 8, 8, 14, 1, 7, W8, N) == ERR                        # cv_r == tmp
    assert lib.sde_cbca_lr(1, 2, 3, 4, 5, 4, 8, 8, 14, 1, 7, W8 - 4, N) == ERR                    # workspace
    assert lib.sde_cbca_reciprocals(N, 4, N) == ERR
    # 32-bit offsets: a vertical-pass block window of (5R + 5) rows of 4*W*D bytes stays below 2^31
    # (R = 13 for L1 <= 14: 70 rows; R = 31 for L1 > 16: 160 rows).  iters = 0 checks the shape only.
    assert lib.sde_cbca(1, 2, 3, 4, 2, 40000, 256, 1, 14, 0, N, 0, N) == ERR                      # 70 * 41 MB
    assert lib.sde_cbca_pair(1, 2, 3, 4, 5, 6, 2, 29960, 256, 14, 0, N, 0, N) == ERR              # just past
    assert lib.sde_cbca_pair(1, 2, 3, 4, 5, 6, 2, 29959, 256, 14, 0, N, 0, N) == 0                # just inside
    assert lib.sde_cbca_lr(1, 2, 3, 4, 5, 2, 13108, 256, 20, 0, N, 0, N) == ERR                   # R = 31
    # accepted by the argument checks (iters 0 still writes the shear: no GPU here, so the launch fails)
    assert lib.sde_cbca_lr(1, 2, 3, 4, 5, 2, 13107, 256, 20, 0, N, 0, N) != ERR
    assert lib.sde_lrc_fill(1, 2, 4, 65535, 3, N) == ERR                                          # 16-bit columns
    assert lib.sde_lrc_fill(1, 2, 65535, 4, 3, N) == ERR                                          # 16-bit rows


def test_ops_refuse_cpu_tensors():
    import torch
    from scenedepthestimation_amd import ops
    f = torch.zeros((2, 3, 64))
    with pytest.raises(ValueError, match="GPU"):
        ops.cv_wta(f, f, 0, 2)
    with pytest.raises(ValueError, match="GPU"):
        ops.cost_volume(f, f, 2)


def test_isa_lint_flags_store_data_overwrite():
    """The lint catches the round-4 schedule (a VALU write into a dwordx4 store's data right after
    it) and accepts it once the write is two instructions away or aimed elsewhere."""
    from scenedepthestimation_amd import _isa_lint
    head = "0000000000001000 <k>:\n"
    bad = head + ("\tbuffer_store_dwordx4 v[180:183], v206, s[28:31], s68 offen // 000000001000: x\n"
                  "\tv_max_u32_e32 v180, v176, v177 // 000000001008: x\n")
    near = head + ("\tbuffer_store_dwordx4 v[180:183], v206, s[28:31], s68 offen\n"
                   "\tv_mov_b32_e32 v1, v2\n\tv_lshlrev_b32_e32 v183, 2, v208\n")
    nop = head + ("\tglobal_store_dwordx4 v[0:1], v[4:7], off\n\ts_nop 1\n\tv_mov_b32_e32 v5, v2\n")
    far = head + ("\tbuffer_store_dwordx4 v[180:183], v206, s[28:31], s68 offen\n"
                  "\tv_mov_b32_e32 v1, v2\n\ts_nop 0\n\tv_max_u32_e32 v180, v176, v177\n")
    other = head + ("\tbuffer_store_dwordx2 v[180:181], v206, s[28:31], s68 offen\n\tv_mov_b32_e32 v180, v2\n")
    assert len(_isa_lint.lint_text(bad)) == 1
    assert len(_isa_lint.lint_text(near)) == 1
    assert _isa_lint.lint_text(nop) == []
    assert _isa_lint.lint_text(far) == []
    assert _isa_lint.lint_text(other) == []
    # kernels with MFMAs: a write is flagged until MFMA_STORE_DATA_WINDOW (9) wait states have passed;
    # AGPR store data is tracked like VGPR data
    mf = "\tv_mfma_f32_16x16x32_f16 v[0:3], v[4:7], v[8:11], v[0:3]\n"
    far_mfma = head + mf + ("\tbuffer_store_dwordx4 v[180:183], v206, s[28:31], s68 offen\n"
                            "\ts_nop 4\n\tv_max_u32_e32 v180, v176, v177\n")
    ok_mfma = head + mf + ("\tbuffer_store_dwordx4 v[180:183], v206, s[28:31], s68 offen\n"
                           "\ts_nop 7\n\ts_nop 0\n\tv_max_u32_e32 v180, v176, v177\n")
    agpr = head + mf + ("\tglobal_store_dwordx4 v[0:1], a[4:7], off\n\tv_accvgpr_write_b32 a6, v2\n")
    assert len(_isa_lint.lint_text(far_mfma)) == 1 and _isa_lint.lint_text(far) == []
    assert _isa_lint.lint_text(ok_mfma) == []
    assert len(_isa_lint.lint_text(agpr)) == 1
    # one function's MFMAs do not widen the window of the next one
    assert _isa_lint.lint_text(head + mf + "0000000000002000 <k2>:\n" + far.split("\n", 1)[1]) == []


def test_isa_lint_passes_on_the_built_library():
    from scenedepthestimation_amd import _isa_lint
    from scenedepthestimation_amd._build import OBJ
    objs = sorted(os.path.join(OBJ, f) for f in os.listdir(OBJ) if f.endswith(".o"))
    if not objs or not os.path.exists(_isa_lint.LLVM):
        pytest.skip("no built objects / ROCm LLVM tools")
    assert _isa_lint.lint_objects(objs) == []


def test_library_registers_no_exit_time_code(tmp_path):
    """code of ours inside exit() can reach the HIP runtime after it (or a profiler) has
    finalised -- the build refuses it.  The built library carries only the hipcc module destructors; a C++
    static with a destructor and a destructor-attribute function are both flagged."""
    import shutil
    import subprocess

    from scenedepthestimation_amd import _build
    if not os.path.exists(_build.LIB):
        pytest.skip("libsde.so not built")
    if not shutil.which("g++") or not shutil.which("readelf"):
        pytest.skip("no g++ / binutils")
    assert _build.exit_hooks(_build.LIB) == []
    src = tmp_path / "hooks.cpp"
    src.write_text("volatile int g;\nstruct S { ~S(); }; S::~S() {} static S s;\n"
                   "__attribute__((destructor)) static void bye() { g = 1; }\n"
                   "extern \"C\" int f() { static S t; return 1; }\n")
    so = tmp_path / "libhooks.so"
    subprocess.run(["g++", "-shared", "-fPIC", "-O1", str(src), "-o", str(so)], check=True)
    hooks = _build.exit_hooks(str(so))
    assert any(f == ".fini_array" for f, _ in hooks), hooks
    assert sum(1 for f, _ in hooks if f != ".fini_array") >= 2, hooks   # the static and the local static
