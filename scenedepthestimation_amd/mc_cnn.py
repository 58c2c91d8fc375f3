"""MC-CNN-fast branch weights (mc_cnn_brunch.py) -- naming, synthetic init, loading, packing.

The reference builds `Net` (mc_cnn_brunch.py:4-67) with variables named
``conv{k}/weights:0`` (HWIO ``[3,3,Cin,nf]``) and ``conv{k}/biases:0`` (``[nf]``)
(`conv`, mc_cnn_brunch.py:70-92) and restores them from a TF1 checkpoint
(process_functional.py:24-33) or a ``.npy`` dict (`load_initial_weights`,
mc_cnn_brunch.py:51-58).  TF1 checkpoints are read without TensorFlow by
``tf_checkpoint.load_checkpoint``.  No checkpoint ships with the reference, so
the default here is a seeded synthetic He-normal initialisation of the same
architecture.  The device-side network is run by ``ops.tower_forward``.
"""
from __future__ import annotations

import os

import numpy as np

DEFAULT_NUM_FEATURE_MAPS = 64     # process_functional.py:23 / match_single.py:46
DEFAULT_PATCH = 11                # match_single.py:46 -> num_of_conv_layers = 11 // 2 = 5


def var_names(nlayers: int):
    return [(f"conv{k}/weights:0", f"conv{k}/biases:0") for k in range(1, nlayers + 1)]


def synthetic_weights(nlayers: int = 5, nf: int = DEFAULT_NUM_FEATURE_MAPS, seed: int = 1234,
                      bias: float = 0.01) -> dict:
    """He-normal HWIO weights and constant biases (SURVEY.md section 8d synthetic inputs)."""
    rng = np.random.default_rng(seed)
    out = {}
    for k, (wn, bn) in enumerate(var_names(nlayers), start=1):
        cin = 1 if k == 1 else nf
        std = np.sqrt(2.0 / (9 * cin))
        out[wn] = (rng.standard_normal((3, 3, cin, nf)) * std).astype(np.float32)
        out[bn] = np.full((nf,), bias, np.float32)
    return out


def load_weights(checkpoint, nlayers: int, allow_pickle: bool = False) -> dict:
    """Load a weights dict keyed like the reference's trainable variables.

    Accepted: a dict; ``synthetic`` / ``synthetic:<seed>`` / None; a ``.npz`` or
    ``.safetensors`` file with the reference variable names; a TF1 (Saver V2)
    checkpoint prefix such as ``model_epoch14.ckpt`` (``<prefix>.index`` +
    ``<prefix>.data-*``, read by tf_checkpoint.py); a ``.npy`` dict as written by
    ``Net.save_weights_dict`` (pickled, so only with allow_pickle=True for a file
    the caller trusts).  A missing checkpoint raises FileNotFoundError, like TF's
    restore.
    """
    if checkpoint is None:
        return synthetic_weights(nlayers)
    if isinstance(checkpoint, dict):
        w = dict(checkpoint)
    elif isinstance(checkpoint, str) and checkpoint.startswith("synthetic"):
        seed = int(checkpoint.split(":", 1)[1]) if ":" in checkpoint else 1234
        return synthetic_weights(nlayers, seed=seed)
    else:
        path = os.fspath(checkpoint)
        if path.endswith(".npz"):
            with np.load(path, allow_pickle=False) as z:
                w = {k: z[k] for k in z.files}
        elif path.endswith(".safetensors"):
            from safetensors.numpy import load_file
            w = load_file(path)
        elif path.endswith(".npy"):
            if not allow_pickle:
                raise ValueError(f"{path}: a .npy weights dict is a pickle; pass allow_pickle=True only for a "
                                 "file you trust, or convert it to .npz / .safetensors")
            w = np.load(path, allow_pickle=True, encoding="bytes").item()
        else:
            from . import tf_checkpoint
            names = [n for pair in var_names(nlayers) for n in pair]
            w = {n: v for n, v in zip(names, tf_checkpoint.load_checkpoint(path, names).values())}
    w = {(k.decode() if isinstance(k, bytes) else k): np.asarray(v, dtype=np.float32) for k, v in w.items()}
    for wn, bn in var_names(nlayers):
        if wn not in w or bn not in w:
            raise KeyError(f"weights dict lacks {wn} / {bn}")
    return w


def layer_lists(weights: dict, nlayers: int):
    names = var_names(nlayers)
    return [weights[wn] for wn, _ in names], [weights[bn] for _, bn in names]
