"""The HIP renderer under more than one process (``-m gpu``).

Two ranks on device 0 (gloo control plane: the one-GPU test box cannot run RCCL with two
ranks on one card; the driver's N-GPU bench puts one rank per GPU over RCCL) each render
their contiguous ray range of a 3-frame NMR batch (tests/dist_render_worker.py).  The
assembled image must equal the single-process render bit for bit: sharding rays adds no
data-path collective and cannot change any ray's result.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_hip_render_equals_single_process(tmp_path):
    out = tmp_path / "dist_render.json"
    env = dict(os.environ, PNR_DIST_BACKEND="gloo", PNR_FORCE_DEVICE="0", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "dist_render_worker.py"), str(out)]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    res = json.loads(out.read_text())
    assert res["world"] == 2 and res["finite"]
    assert res["equal"], res


def test_bench_gpus_2_launches_its_own_ranks():
    """`python bench.py --gpus 2` -- the form the driver's scaling runs use -- starts its own 2
    ranks (torch.distributed.run as a child; both on device 0 with gloo here, one per GPU with
    RCCL on a node) and reports the whole batch over both ranks: n_gpus 2, rank 0's shard is half
    of the 98,304-ray cfg3 batch.  The cfg5 train leg runs with the encoder's BatchNorm
    synchronised over the 2 ranks (pnr.dist.SyncBatchNorm2d on HIP tensors)."""
    env = dict(os.environ, PNR_DIST_BACKEND="gloo", PNR_FORCE_DEVICE="0", OMP_NUM_THREADS="4")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(os.path.dirname(HERE), "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--train-steps", "2"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["rays_rank0"] == 49152 and res["value"] > 0
    assert res["config"]["rays_per_step"] == 98304
    tr = res["train"]
    assert tr["n_gpus"] == 2 and tr["config"]["encoder_batchnorm"].startswith("sync") and tr["value"] > 0
    assert tr["loss"] == tr["loss"]   # finite
