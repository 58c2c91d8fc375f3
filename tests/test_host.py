"""CPU: host-side logic -- product/oracle isolation, weights, synthetic data, image I/O, CLIs."""
import ast
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "scenedepthestimation_amd")


def _imports(path):
    tree = ast.parse(open(path).read())
    mods = set()
    for n in ast.walk(tree):
        if isinstance(n, ast.Import):
            mods |= {a.name.split(".")[0] for a in n.names}
        elif isinstance(n, ast.ImportFrom) and n.module and n.level == 0:
            mods.add(n.module.split(".")[0])
    return mods


def test_product_never_imports_the_oracle():
    for dp, _, files in os.walk(PKG):
        for f in files:
            if f.endswith(".py"):
                assert "oracle" not in _imports(os.path.join(dp, f)), f
            if f.endswith((".hip", ".h", ".cpp")):
                assert "sde_oracle" not in open(os.path.join(dp, f)).read(), f


def test_product_has_no_reference_dependency():
    for dp, _, files in os.walk(PKG):
        for f in files:
            if f.endswith((".py", ".hip", ".h")):
                assert "/root/reference" not in open(os.path.join(dp, f)).read(), f


def test_synthetic_weights_and_loading(tmp_path):
    from scenedepthestimation_amd import mc_cnn
    w = mc_cnn.synthetic_weights(5)
    assert w["conv1/weights:0"].shape == (3, 3, 1, 64)
    assert w["conv5/weights:0"].shape == (3, 3, 64, 64)
    assert np.allclose(w["conv3/biases:0"], 0.01)
    np.savez(tmp_path / "w.npz", **w)
    w2 = mc_cnn.load_weights(str(tmp_path / "w.npz"), 5)
    assert all(np.array_equal(w[k], w2[k]) for k in w)
    assert mc_cnn.load_weights("synthetic:1234", 5)["conv2/weights:0"].tobytes() == w["conv2/weights:0"].tobytes()
    with pytest.raises(FileNotFoundError):
        mc_cnn.load_weights("./check_points_11_11/model_epoch14.ckpt", 5)
    with pytest.raises(ValueError):
        mc_cnn.load_weights(str(tmp_path / "x.npy"), 5)
    bad = dict(w)
    del bad["conv4/biases:0"]
    with pytest.raises(KeyError):
        mc_cnn.load_weights(bad, 5)


def test_synthetic_pair_geometry():
    from scenedepthestimation_amd.synthetic import stereo_pair
    left, right, gt = stereo_pair(32, 200, 40, seed=2)
    assert left.dtype == np.uint8 and right.shape == left.shape and gt.max() < 40
    xr = np.arange(200)[None, :] - gt
    ys, xs = np.nonzero(xr >= 0)
    # right pixels hit by exactly one left pixel carry that pixel's intensity (occlusions excluded)
    hits = np.zeros_like(right, dtype=np.int32)
    np.add.at(hits, (ys, xr[ys, xs]), 1)
    uniq = hits[ys, xr[ys, xs]] == 1
    assert uniq.mean() > 0.8
    assert np.array_equal(right[ys[uniq], xr[ys, xs][uniq]], left[ys[uniq], xs[uniq]])


def test_imageio_cv2_gray_rule(tmp_path):
    from PIL import Image

    from scenedepthestimation_amd import imageio
    rgb = np.random.default_rng(0).integers(0, 256, (5, 7, 3)).astype(np.uint8)
    Image.fromarray(rgb, "RGB").save(tmp_path / "c.png")
    g = imageio.imread_gray(str(tmp_path / "c.png"))
    r, gg, b = (rgb[..., i].astype(np.uint32) for i in range(3))
    assert np.array_equal(g, ((r * 4899 + gg * 9617 + b * 1868 + 8192) >> 14).astype(np.uint8))
    gray = rgb[..., 0]
    imageio.imwrite(str(tmp_path / "sub" / "g.png"), gray)
    assert np.array_equal(imageio.imread_gray(str(tmp_path / "sub" / "g.png")), gray)
    assert imageio.imread_gray(str(tmp_path / "missing.png")) is None


def test_imageio_jpeg_gray_is_the_luma_plane():
    """cv2.imread(jpg, IMREAD_GRAYSCALE) has libjpeg emit a YCbCr JPEG's luma plane (match.py:48-52);
    imread_gray must return exactly that plane -- checked against the Y channel of a raw YCbCr decode
    of the committed fixture (tests/golden/make_jpeg.py), which the RGB -> gray route would miss."""
    from PIL import Image

    from scenedepthestimation_amd import imageio
    path = os.path.join(os.path.dirname(__file__), "golden", "ycbcr_4x2.jpg")
    raw = Image.open(path)
    raw.draft("YCbCr", raw.size)
    luma = np.asarray(raw)[..., 0]
    got = imageio.imread_gray(path)
    assert got.dtype == np.uint8 and got.shape == (24, 40)
    assert np.array_equal(got, luma)
    rgb = np.asarray(Image.open(path).convert("RGB")).astype(np.uint32)
    via_rgb = ((rgb[..., 0] * 4899 + rgb[..., 1] * 9617 + rgb[..., 2] * 1868 + 8192) >> 14).astype(np.uint8)
    assert (via_rgb != luma).sum() > 10          # the fixture tells the two routes apart


def test_cli_parsers_match_reference_flags():
    from scenedepthestimation_amd import match, match_single
    a = match_single.build_parser().parse_args([])
    assert (a.gpu, a.id, a.file, a.ui) == ("1,2", 0, "11_11", False)
    a = match_single.build_parser(ui=True).parse_args(["-i", "3", "-g", "0"])
    assert (a.gpu, a.id, a.file, a.ui) == ("0", 3, "UI_disparity", True)
    a = match.build_parser().parse_args([])
    assert a.gpu == "0,1,2,3,4,5,6,7" and a.pairs == 18


def test_cli_normalise_is_reference_numpy():
    from scenedepthestimation_amd.match_single import normalise
    img = np.random.default_rng(1).integers(0, 256, (9, 11)).astype(np.float32)
    x = normalise(img)
    ref = (img - np.mean(img, axis=(0, 1))) / np.std(img, axis=(0, 1))
    assert x.shape == (9, 11, 1) and x[..., 0].tobytes() == ref.tobytes()


def test_bench_mode_resolution():
    """bench.py --mode auto: dshard only where the sharded schemes apply (tower + CV/WTA at
    N > 1); the SGM workloads and one GPU run pair-DP; an explicit sharded mode on an SGM workload at N > 1
    is refused, at N = 1 it is the single-device path."""
    import bench
    assert bench.resolve_mode("auto", 1, "tower+cv_wta") == "pairdp"
    assert bench.resolve_mode("auto", 8, "tower+cv_wta") == "dshard"
    for w in ("c3", "north_star_sgm", "cones_sgm"):
        what = bench.WORKLOADS[w][3]
        assert bench.resolve_mode("auto", 8, what) == "pairdp"
        assert bench.resolve_mode("auto", 1, what) == "pairdp"
        with pytest.raises(SystemExit):
            bench.resolve_mode("dshard", 2, what)
    assert bench.resolve_mode("rowband", 4, "tower+cv_wta") == "rowband"


def test_split_batch_bound_rows_checked():
    """ops.tower_layer_batch refuses split activations over a batch whose bound-word rows are shorter than
    64 words (the scale word, 32 words past a layer's bound word, would land on the next image's
    row) before anything touches a device."""
    import torch

    from scenedepthestimation_amd import ops
    x = torch.zeros((2, 8, 8, 64))
    y = torch.zeros((2, 6, 6, 64))
    for stride in (33, 35, 63):
        words = torch.zeros(2 * stride + 64)[:2 * stride].view(2, stride)   # room for every scale word
        with pytest.raises(ValueError, match="rows of >= 64"):
            ops.tower_layer_batch(x, None, 5, 3, y, in_absmax=words, out_absmax=words[:, 1:], in_split=True,
                                  out_split=True)
