"""CPU oracle for the WHDY/SceneDepthEstimation matching path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this package, and only as the checker / the timed CPU baseline.  The
product package ``scenedepthestimation_amd`` never imports it (a test enforces that).

Parity: cost volume, WTA and WTA1 are pinned against golden vectors produced by
the reference's own NumPy code (tests/golden/make_golden.py).  SGM, penalties,
LR check, LRC fill, median and the tower are "parity unpinned" restatements of
Numba / TF1 code that cannot run here (see sde_oracle.c).
"""
from .oracle import *  # noqa: F401,F403
