"""The training caller (pnr.trainer, scripts/train.py): the reference's train.py:193-283 step and
trainlib's loop / checkpoints.

CPU: util.bbox_sample against the reference's own draws (tests/golden/bbox_sample.npz, generated
by tests/golden/make_golden.py from /root/reference/src/util/util.py:220-235 with seeded torch
generators), and calc_losses' host logic (pixel / view picks, ray gather, source selection,
loss) with a recording stand-in for the model and renderer.  GPU: scripts/train.py end to end on
a synthetic SRN-layout dataset, then resumed from its checkpoints."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import fixtures
from pnr import trainer, util
from srn_synth import make_inputs, write_srn_dir

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bbox_sample_matches_reference_fixture():
    cfg, arr = fixtures.load("bbox_sample")
    torch.manual_seed(cfg["seed"])
    pix = util.bbox_sample(torch.as_tensor(np.asarray(arr["boxes"])), cfg["num_pix"])
    assert torch.equal(pix, torch.as_tensor(np.asarray(arr["pix"])))
    torch.manual_seed(cfg["iseed"])
    ipix = util.bbox_sample(torch.as_tensor(np.asarray(arr["iboxes"])), cfg["inum_pix"])
    assert torch.equal(ipix, torch.as_tensor(np.asarray(arr["ipix"])))


class _Net:
    def __init__(self):
        self.calls = []

    def encode(self, images, poses, focal, c=None):
        self.calls.append((images.clone(), poses.clone(), focal.clone(), None if c is None else c.clone()))


class _Render:
    """render_par stand-in: rgb = a learnable-free function of the rays (o + d), recorded."""

    def __init__(self, fine=True):
        self.fine = fine
        self.rays = None
        self.w = torch.ones((), requires_grad=True)   # a parameter for the backward to reach

    def __call__(self, rays, want_weights=False):
        assert want_weights
        self.rays = rays.clone()
        rgb = torch.sigmoid(rays[..., :3] + rays[..., 3:6]) * self.w
        out = {"coarse": {"rgb": rgb}}
        if self.fine:
            out["fine"] = {"rgb": rgb * 0.5}
        return out


def _batch(sb=2, nv=3, h=6, w=8, seed=0, bbox=False):
    g = torch.Generator().manual_seed(seed)
    images = torch.rand(sb, nv, 3, h, w, generator=g) * 2 - 1
    poses = torch.eye(4).repeat(sb, nv, 1, 1)
    poses[..., :3, 3] = torch.rand(sb, nv, 3, generator=g)
    data = dict(images=images, poses=poses, focal=torch.tensor([7.0, 9.0])[:sb],
                c=torch.tensor([[3.5, 2.5], [4.0, 3.0]])[:sb])
    if bbox:
        data["bbox"] = torch.tensor([[1.0, 1.0, 5.0, 4.0]]).repeat(sb, nv, 1)
    return data


@pytest.mark.parametrize("bbox,nviews", [(False, (1,)), (True, (2,)), (False, (1, 2, 3))])
def test_calc_losses_host_logic(bbox, nviews):
    """calc_losses draws its view / pixel picks from the host generators in the reference's
    order (train.py:214-245): reproduce them with the same seeds and check the rays the renderer
    got, the source views encode() got and the loss."""
    data = _batch(bbox=bbox)
    sb, nv, _, h, w = data["images"].shape
    rb = 10
    torch.manual_seed(11)
    np.random.seed(11)
    net, rp = _Net(), _Render()
    # is_train: the boxes are used only in training steps (train.py:205-206), and the loss is
    # back-propagated
    losses = trainer.calc_losses(net, rp, data, device="cpu", z_near=0.5, z_far=2.5, nviews=nviews,
                                 ray_batch_size=rb, use_bbox=bbox, is_train=True)
    assert rp.w.grad is not None
    # the same draws, by hand
    torch.manual_seed(11)
    np.random.seed(11)
    cur = nviews[torch.randint(0, len(nviews), ()).item()]
    order = torch.randint(0, nv, (sb, 1)) if cur == 1 else torch.empty((sb, cur), dtype=torch.long)
    want_rays, want_gt = [], []
    for o in range(sb):
        if cur > 1:
            order[o] = torch.from_numpy(np.random.choice(nv, cur, replace=False))
        rays = util.gen_rays(data["poses"][o], w, h, data["focal"][o], 0.5, 2.5, c=data["c"][o]).reshape(-1, 8)
        gt = (data["images"][o] * 0.5 + 0.5).permute(0, 2, 3, 1).reshape(-1, 3)
        if bbox:
            pix = util.bbox_sample(data["bbox"][o], rb)
            inds = pix[..., 0] * h * w + pix[..., 1] * w + pix[..., 2]
        else:
            inds = torch.randint(0, nv * h * w, (rb,))
        want_rays.append(rays[inds])
        want_gt.append(gt[inds])
    want_rays, want_gt = torch.stack(want_rays), torch.stack(want_gt)
    assert torch.equal(rp.rays, want_rays)
    imgs, poses, focal, c = net.calls[0]
    assert imgs.shape == (sb, cur, 3, h, w)
    assert torch.equal(imgs, util.batched_index_select_nd(data["images"], order))
    assert torch.equal(poses, util.batched_index_select_nd(data["poses"], order))
    rgb = torch.sigmoid(want_rays[..., :3] + want_rays[..., 3:6])
    mse = torch.nn.functional.mse_loss
    assert abs(losses["rc"] - mse(rgb, want_gt).item()) < 1e-6
    assert abs(losses["rf"] - mse(rgb * 0.5, want_gt).item()) < 1e-6
    assert abs(losses["t"] - (mse(rgb, want_gt) + mse(rgb * 0.5, want_gt)).item()) < 1e-6


def test_calc_losses_coarse_only():
    """No "fine" key (the renderer without a fine pass, nerf.py:305-316): the loss is the
    coarse term alone (train.py:262-270)."""
    data = _batch()
    losses = trainer.calc_losses(_Net(), _Render(fine=False), data, device="cpu", z_near=0.5, z_far=2.5,
                                 ray_batch_size=4, is_train=False, lambda_coarse=0.5)
    assert set(losses) == {"rc", "t"}
    assert abs(losses["rc"] - 0.5 * losses["t"]) < 1e-7


TRAIN_CONF = """
model {
    use_encoder = True
    use_xyz = True
    use_code = True
    code { num_freqs = 6, freq_factor = 1.5, include_input = True }
    use_viewdirs = True
    use_code_viewdirs = False
    mlp_coarse { type = resnet, n_blocks = 5, d_hidden = 512, combine_layer = 3, combine_type = average }
    mlp_fine { type = resnet, n_blocks = 5, d_hidden = 512, combine_layer = 3, combine_type = average }
    encoder { backbone = resnet34, pretrained = False, num_layers = 4 }
}
renderer {
    n_coarse = 32
    n_fine = 16
    n_fine_depth = 8
    depth_std = 0.01
    white_bkgd = True
}
loss {
    rgb { use_uncertainty = False }
    lambda_coarse = 1.0
    lambda_fine = 1.0
}
train {
    print_interval = 1
    save_interval = 2
    eval_interval = 2
    accu_grad = 1
}
"""


@pytest.mark.gpu
def test_train_script_end_to_end_and_resume(tmp_path):
    """scripts/train.py as a user runs it (train.py's flags, HOCON conf, SRN-layout train / val
    splits): 3 steps with bbox sampling, checkpoints every 2 batches; then --resume continues
    from the saved iteration with the saved weights and optimizer state."""
    inp = make_inputs(n_obj=4, n_views=3, size=24, seed=3)
    root = write_srn_dir(str(tmp_path), inp, stage="train")
    write_srn_dir(str(tmp_path), make_inputs(n_obj=2, n_views=3, size=24, seed=4), stage="val")
    write_srn_dir(str(tmp_path), make_inputs(n_obj=1, n_views=3, size=24, seed=5), stage="test")
    (tmp_path / "train.conf").write_text(TRAIN_CONF)
    common = [sys.executable, os.path.join(REPO, "scripts", "train.py"), "-c", str(tmp_path / "train.conf"),
              "-D", root, "-F", "srn", "-n", "synth", "--checkpoints_path", str(tmp_path / "ck"),
              "--visual_path", str(tmp_path / "vis"), "-B", "2", "-V", "1", "-R", "64", "--image_size", "24"]
    r = subprocess.run(common + ["--max_steps", "3"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "final losses" in r.stdout and "*** Eval" in r.stdout, r.stdout[-2000:]
    ck = tmp_path / "ck" / "synth"
    for f in ("pixel_nerf_latest", "_optim", "_iter", "_renderer"):
        assert (ck / f).exists(), f
    assert torch.load(str(ck / "_iter"), weights_only=True)["iter"] == 3
    sd = torch.load(str(ck / "pixel_nerf_latest"), weights_only=True)
    assert all(bool(torch.isfinite(v).all()) for v in sd.values() if v.is_floating_point())
    last = [l for l in r.stdout.splitlines() if l.startswith("final losses")][-1]
    vals = [float(t.split(":")[1]) for t in last.split()[2:]]
    assert vals and all(np.isfinite(vals))
    r2 = subprocess.run(common + ["--resume", "--max_steps", "2"], capture_output=True, text=True, timeout=300)
    assert r2.returncode == 0, r2.stderr[-3000:]
    assert "Load" in r2.stdout and "CONTINUE? yes" in r2.stdout
    assert torch.load(str(ck / "_iter"), weights_only=True)["iter"] == 5


# ---- Trainer over 2 gloo ranks (CPU): sampler sharding, gradient mean, rank-0 checkpoints --------
class _TinyNet(torch.nn.Module):
    """PixelNeRFNet stand-in: encode() keeps the mean source colour; the "render" is
    sigmoid(w * (o + d)) + that colour; an encoder BatchNorm for the SyncBN switch."""

    def __init__(self):
        super().__init__()
        self.encoder = torch.nn.Sequential(torch.nn.BatchNorm2d(3))
        self.w = torch.nn.Parameter(torch.full((3,), 0.5))
        self.col = None
        self.log = []

    def encode(self, images, poses, focal, c=None):
        self.col = images.mean(dim=(0, 1, 3, 4))
        self.log.append((int(images.shape[1]), bool(self.training)))   # (NS, train mode) per encode

    def load_weights(self, args, opt_init=False, strict=True, device=None):
        path = os.path.join(args.checkpoints_path, args.name, "pixel_nerf_latest")
        if args.resume and os.path.exists(path):
            self.load_state_dict(torch.load(path, weights_only=True))
        return self

    def save_weights(self, args, opt_init=False):
        torch.save(self.state_dict(), os.path.join(args.checkpoints_path, args.name, "pixel_nerf_latest"))


class _TinyRenderer(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.register_buffer("iter_idx", torch.zeros((), dtype=torch.long))

    def bind_parallel(self, net, gpus=None, simple_output=False):
        def render(rays, want_weights=False):
            return {"coarse": {"rgb": torch.sigmoid(net.w * (rays[..., :3] + rays[..., 3:6])) + 0.1 * net.col}}
        return render

    def sched_step(self, steps=1):
        self.iter_idx += steps


class _Objects(torch.utils.data.Dataset):
    z_near, z_far, lindisp = 0.5, 2.5, False

    def __init__(self, n=8, nv=3, size=6):
        g = torch.Generator().manual_seed(1)
        self.items = []
        for i in range(n):
            poses = torch.eye(4).repeat(nv, 1, 1)
            poses[:, :3, 3] = torch.rand(nv, 3, generator=g)
            self.items.append(dict(images=torch.rand(nv, 3, size, size, generator=g) * 2 - 1, poses=poses,
                                   focal=torch.tensor(5.0 + i), c=torch.tensor([3.0, 3.0]),
                                   bbox=torch.tensor([[1.0, 1.0, 4.0, 4.0]]).repeat(nv, 1), obj=torch.tensor(i)))

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        return self.items[i]


def _trainer_args(ck, resume=False, nviews=(1,)):
    import types

    return types.SimpleNamespace(checkpoints_path=ck, name="tiny", resume=resume, batch_size=2, lr=0.05,
                                 gamma=1.0, gamma_delay=0, epochs=2, ray_batch_size=16, nviews=list(nviews),
                                 no_bbox_step=100, seed=0)


def _trainer_worker(rank, world, port, ck, q):
    from pnr import dist as pdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    pdist.init_from_env("gloo")
    trainer.seed_everything(rank)
    net = _TinyNet()
    t = trainer.Trainer(net, _TinyRenderer(), _Objects(), None, _trainer_args(ck, nviews=(1, 2, 3)),
                        {"print_interval": 100, "save_interval": 100}, torch.device("cpu"), log=lambda *_: None)
    t.sampler.set_epoch(0)
    seen = [int(o) for d in t.loader for o in d["obj"]]
    last = t.start()
    # plain Python values: a tensor put on the queue is shared through a handle that dies with
    # this process
    q.put((rank, seen, net.w.detach().tolist(), type(net.encoder[0]).__name__, dict(last), net.log))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_trainer_two_rank_gloo(tmp_path):
    """pnr.trainer.Trainer at world_size 2 (gloo): each rank draws its own objects (together all
    of them, once), the gradient mean keeps the two ranks' parameters identical through Adam, the
    encoder BatchNorm became SyncBatchNorm2d, and only rank 0 wrote the checkpoints (_iter = the
    steps of one rank: 4 objects / 2 per batch)."""
    import multiprocessing

    from test_dist import _free_port

    ctx = multiprocessing.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ck = str(tmp_path / "ck")
    procs = [ctx.Process(target=_trainer_worker, args=(r, 2, port, ck, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, seen0, w0, bn0, l0, log0), (r1, seen1, w1, bn1, l1, log1) = res
    assert sorted(seen0 + seen1) == list(range(8)) and not set(seen0) & set(seen1)
    # -V "1 2 3": every step's view count is the same on both ranks (one draw per step for the whole
    # batch, as the reference's single process), and it varies over the steps; step 0 runs in eval
    # mode (train.py:93's render_par.eval()), the later steps in train mode
    assert [n for n, _ in log0] == [n for n, _ in log1] and len({n for n, _ in log0}) > 1, (log0, log1)
    assert [m for _, m in log0] == [False] + [True] * (len(log0) - 1)
    w0, w1 = torch.tensor(w0), torch.tensor(w1)
    assert torch.equal(w0, w1) and not torch.equal(w0, torch.full((3,), 0.5))
    assert bn0 == bn1 == "SyncBatchNorm2d"
    assert np.isfinite(l0["t"]) and np.isfinite(l1["t"])
    assert torch.load(os.path.join(ck, "tiny", "_iter"), weights_only=True)["iter"] == 4   # 2 epochs x 2
    assert torch.equal(torch.load(os.path.join(ck, "tiny", "pixel_nerf_latest"), weights_only=True)["w"], w0)


@pytest.mark.gpu
def test_train_script_two_ranks(tmp_path):
    """scripts/train.py under torch.distributed.run with 2 ranks (both on device 0 over gloo: the
    one-GPU box cannot run RCCL with two ranks on one card; a node puts one rank per GPU over
    RCCL): each rank trains its own objects with the encoder BatchNorm synchronised and the
    gradient mean over the ranks; rank 0 writes the checkpoints."""
    import socket

    inp = make_inputs(n_obj=4, n_views=3, size=24, seed=6)
    root = write_srn_dir(str(tmp_path), inp, stage="train")
    write_srn_dir(str(tmp_path), make_inputs(n_obj=2, n_views=3, size=24, seed=7), stage="val")
    write_srn_dir(str(tmp_path), make_inputs(n_obj=1, n_views=3, size=24, seed=8), stage="test")
    (tmp_path / "train.conf").write_text(TRAIN_CONF)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, PNR_DIST_BACKEND="gloo", PNR_FORCE_DEVICE="0", OMP_NUM_THREADS="4")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "scripts", "train.py"),
           "-c", str(tmp_path / "train.conf"), "-D", root, "-F", "srn", "-n", "synth2", "--checkpoints_path",
           str(tmp_path / "ck"), "--visual_path", str(tmp_path / "vis"), "-B", "1", "-V", "1", "-R", "32",
           "--image_size", "24", "--max_steps", "2"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.count("final losses") == 1, r.stdout[-2000:]
    ck = tmp_path / "ck" / "synth2"
    assert torch.load(str(ck / "_iter"), weights_only=True)["iter"] == 2
    sd = torch.load(str(ck / "pixel_nerf_latest"), weights_only=True)
    assert all(bool(torch.isfinite(v).all()) for v in sd.values() if v.is_floating_point())
