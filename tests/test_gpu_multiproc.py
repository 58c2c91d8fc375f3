"""GPU: the product's multi-rank classes (parallel.py) at world 2 and 3 on the one GPU of the box.

Each rank is a fresh child process (subprocess: no exec of this process) on cuda:0 with the gloo
backend -- device tensors staged through host memory (parallel.all_gather_into / allreduce_max_);
on an 8-GPU node the same code runs one rank per GPU over RCCL.  Covers the band tower's bound-
word all-reduces, the feature all-gather, the partials all-gather + ordered merge, the replicated
-tower scheme's single all-gather, and the row-band gather, including an empty trailing band
(H = 3, world 3).  Every map must equal the single-device StereoMatcher's bit for bit."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("world,H,W,D", [(2, 70, 96, 64), (3, 40, 130, 96), (3, 3, 80, 32)])
def test_multirank_classes_on_one_gpu(gpu, world, H, W, D):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_worker.py"), str(H), str(W),
                                       str(D)], env=env, cwd=ROOT, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for r, (p, out) in enumerate(zip(procs, outs)):
        print(out)
        assert p.returncode == 0, f"rank {r} failed:\n{out[-3000:]}"


@pytest.mark.gpu
@pytest.mark.parametrize("mode,primary,scaling", [("auto", "dshard", "strong"), ("pairdp", "pairdp", "weak"),
                                                  ("dshard", "dshard", "strong"),
                                                  ("dshard_rep", "dshard_rep", "strong"),
                                                  ("rowband", "rowband", "strong")])
def test_bench_multirank_modes_on_one_gpu(gpu, tmp_path, mode, primary, scaling):
    """bench.py --gpus 2 exactly as the driver's scaling run launches it (torch.distributed.run, one
    process per rank), here both ranks on the box's one GPU over gloo (SDE_DIST_BACKEND=gloo; on an
    8-GPU node the same code runs one rank per GPU over RCCL): every mode the scaling run can use
    must come back with one JSON line whose n_gpus, scaling and parallelism say what ran, and its
    disparity map (rank 0's pair) must equal the single-device StereoMatcher's bit for bit.  The default
    (auto) line is the disparity-sharded scheme, with the other three schemes timed in its stages and
    their maps checked too."""
    import json

    import numpy as np
    import torch

    from scenedepthestimation_amd.pipeline import StereoMatcher
    from scenedepthestimation_amd.synthetic import stereo_pair
    port = _free_port()
    env = dict(os.environ, SDE_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    dump = str(tmp_path / "disp.npy")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--workload", "cones", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--dump-disp", dump]
    if mode != "auto":
        cmd += ["--mode", mode]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=110)
    if p.returncode != 0:
        print(p.stdout[-3000:], "\n---- stderr ----\n", "\n".join(l for l in p.stderr.splitlines() if "Gloo" not in l)[-6000:])
    assert p.returncode == 0, "bench.py --gpus 2 failed (output above)"
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == scaling
    assert line["config"]["parallelism"] == f"{primary}2"
    assert line["value"] > 0 and line["steps"] == 2
    H, W, D = 375, 450, 64          # bench.py's cones workload
    left, right, _ = stereo_pair(H, W, D, seed=0)
    m = StereoMatcher(H, W, D)
    m.load_images(left, right)
    want = m.match().cpu().numpy()
    assert np.array_equal(np.load(dump), want), f"{primary}: map differs from the single-device one"
    if mode == "auto":
        modes = line["stages"]["multi_gpu_modes"]
        assert set(modes) == {"dshard", "dshard_rep", "rowband", "pairdp"} and modes["dshard"]["primary"]
        for om in ("dshard_rep", "rowband", "pairdp"):
            assert modes[om]["ms_per_step"] > 0
            assert np.array_equal(np.load(f"{dump}.{om}.npy"), want), f"{om}: map differs from the single-device one"
    del m
    torch.cuda.empty_cache()


@pytest.mark.gpu
def test_bench_multirank_sgm_workload_default_mode(gpu, tmp_path):
    """bench.py --gpus 2 on an SGM workload with no --mode flag: auto resolves to pair-DP
    replicas (SGM needs every disparity per step), one JSON line, and rank 0's map equals the
    single-device whole GPU path's."""
    import json

    import numpy as np
    import torch

    import bench
    from scenedepthestimation_amd.pipeline import StereoMatcher
    from scenedepthestimation_amd.synthetic import stereo_pair
    port = _free_port()
    env = dict(os.environ, SDE_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    dump = str(tmp_path / "disp.npy")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--workload", "cones_sgm", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--dump-disp", dump]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=110)
    if p.returncode != 0:
        print(p.stdout[-3000:], "\n---- stderr ----\n", "\n".join(l for l in p.stderr.splitlines() if "Gloo" not in l)[-6000:])
    assert p.returncode == 0, "bench.py --gpus 2 --workload cones_sgm failed (output above)"
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and line["config"]["parallelism"] == "pairdp2"
    assert line["value"] > 0 and "multi_gpu_modes" not in line.get("stages", {})
    H, W, D, _ = bench.WORKLOADS["cones_sgm"]
    left, right, _ = stereo_pair(H, W, D, seed=0)
    m = StereoMatcher(H, W, D, sgm=True, cbca_iters=bench.CBCA_ITERS, cbca_L1=bench.CBCA_L1, cbca_tau=bench.CBCA_TAU)
    m.load_images(left, right)
    m.features()
    m.sgm_path(post=True)
    want = m.sgm_bufs["disp"][0].cpu().numpy()
    assert np.array_equal(np.load(dump), want), "pairdp SGM map differs from the single-device one"
    del m
    torch.cuda.empty_cache()
