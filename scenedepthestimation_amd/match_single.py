"""Drop-in for the reference's match_single.py / match_single_ui.py entry points.

    python -m scenedepthestimation_amd.match_single [-g GPU] [-i ID] [-f FILE]
           [--checkpoint PATH|synthetic] [--cpu-path] [--ndisp N] [--ui]

Same flags, paths and outputs as match_single.py:15-57 (and, with --ui,
match_single_ui.py:20-58): reads ``./eval/left_{id}.png`` / ``right_{id}.png``
(``./UI_use/`` with --ui) as grayscale, z-normalises each image in NumPy exactly
as match_single.py:40-43, computes MC-CNN features (compute_feature), runs the
GPU path (disparity_compute_by_gpu) and writes ``./result/{file}/ld{id}.png`` as
``uint8(disparity)`` (x2 with --ui, match_single_ui.py:55).

--cpu-path selects the reference's commented CPU alternative
``WTA1(compute_cost_volume(fl, fr, 128))`` (match_single.py:51-53), computed by
the fused GPU kernel, bit-identical to the NumPy path.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

DEFAULT_CKPT = r"./check_points_11_11/model_epoch14.ckpt"   # match_single.py:46


def build_parser(ui: bool = False):
    p = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter,
                                description="stereo matching based on trained model and post-processing")
    p.add_argument("-g", "--gpu", type=str, default="1,2",
                   help="gpu id to use, multiple ids should be separated by commas (e.g. 0,1,2,3)")
    p.add_argument("-i", "--id", type=int, default=0, help="image_id")
    p.add_argument("-f", "--file", type=str, default="UI_disparity" if ui else "11_11", help="file to save result")
    p.add_argument("--checkpoint", type=str, default=DEFAULT_CKPT,
                   help="weights: .npz/.safetensors with conv{k}/weights:0, conv{k}/biases:0, or 'synthetic[:seed]'")
    p.add_argument("--cpu-path", action="store_true", help="WTA1(compute_cost_volume(...)) instead of the SGM path")
    p.add_argument("--ndisp", type=int, default=128, help="disparity range (the reference hard-codes 128)")
    p.add_argument("--ui", action="store_true", default=ui, help="match_single_ui.py paths and x2 output scaling")
    return p


def normalise(img_f32):
    """match_single.py:40-43: per-image (I - mean) / std over axes (0,1), then a channel axis."""
    x = (img_f32 - np.mean(img_f32, axis=(0, 1))) / np.std(img_f32, axis=(0, 1))
    return np.expand_dims(x, axis=2)


def run(args) -> str:
    # match_single.py:25 sets CUDA_VISIBLE_DEVICES; on ROCm the equivalent is HIP_VISIBLE_DEVICES,
    # set before torch initialises HIP.
    os.environ["HIP_VISIBLE_DEVICES"] = args.gpu
    from . import imageio
    from .process_functional import WTA1, compute_cost_volume, compute_feature, disparity_compute_by_gpu

    image_path = "./UI_use/" if args.ui else "./eval/"
    lp = os.path.join(image_path, "left_{}.png".format(args.id))
    rp = os.path.join(image_path, "right_{}.png".format(args.id))
    _left = imageio.imread_gray(lp)
    _right = imageio.imread_gray(rp)
    if _left is None or _right is None:
        # cv2.imread returns None and the reference then fails on `.astype` (AttributeError)
        raise AttributeError(f"'NoneType' object has no attribute 'astype' (cannot read {lp} / {rp})")
    left = normalise(_left.astype(np.float32))
    right = normalise(_right.astype(np.float32))
    fl, fr = compute_feature(left, right, 11, 11, 64, args.checkpoint)
    if args.cpu_path:
        disp = WTA1(compute_cost_volume(fl, fr, args.ndisp))
    else:
        detail_time = np.zeros(shape=[7], dtype=np.float32)
        disp, _, detail_time = disparity_compute_by_gpu(_left, _right, fl, fr, detail_time, ndisp=args.ndisp)
    out = disp.astype("uint8") * 2 if args.ui else disp.astype("uint8")
    path = "./result/{}/ld{}.png".format(args.file, args.id)
    imageio.imwrite(path, out)
    return path


def main(argv=None, ui: bool = False):
    args = build_parser(ui).parse_args(argv)
    path = run(args)
    print(path, file=sys.stderr)


def main_ui(argv=None):
    main(argv, ui=True)


if __name__ == "__main__":
    main()
