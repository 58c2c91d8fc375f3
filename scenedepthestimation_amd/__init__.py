"""MI355X-native stereo matching path (drop-in for WHDY/SceneDepthEstimation's matching pipeline).

Submodules
  _lib               ctypes binding of libsde.so (include/sde.h); raises if the library is missing
  ops                torch-tensor wrappers of every C-ABI entry point
  mc_cnn             MC-CNN-fast weights: reference variable names, synthetic init, loading, packing
  pipeline           StereoMatcher: device-resident hot path (tower -> fused cost volume + WTA, SGM path)
  process_functional the reference's function API (compute_feature, compute_cost_volume, WTA, WTA1,
                     disparity_compute_by_gpu)
  parallel           multi-GPU: pair data-parallel and disparity-sharded cost volume + RCCL all-gather
  match_single, match  the reference's CLI entry points
"""
__version__ = "0.1.0"


def build(force: bool = False) -> str:
    from ._build import build as _b
    return _b(force=force)
