#!/usr/bin/env python
"""Generate golden input/output vectors by running the REFERENCE renderer.

This script is test infrastructure.  It imports the reference's own
``src/render/nerf.py`` and ``src/model/*`` from ``/root/reference`` (read-only)
with import-time stubs for the packages that are absent offline and that touch
no hot-path arithmetic:

* ``cv2``         — only ``cv2.COLORMAP_HOT`` for ``util.cmap`` (util.py:26-30)
* ``torchvision`` — transforms + ``models.resnet34`` (encoder.py:62-64); the CNN
                    is not run: the encoder latent is injected directly
* ``pyhocon``     — only the arg parser (args.py:6)
* ``dotmap``      — the renderer's output container (nerf.py:12)

Random draws (``torch.rand_like`` / ``torch.rand`` / ``torch.randn_like``,
nerf.py:111, 135, 141, 158) are replaced by explicitly injected streams, which
are stored in the fixture so every consumer replays them exactly.

Weights and latents come from ``pnr.synth`` hashes, so a fixture stores seeds,
not the 13.75 MB MLPs.  Nothing from the reference is written to the repo:
only inputs and outputs (``*.npz``).

Run:  python tests/golden/make_golden.py   (skips if /root/reference is absent)
"""
import contextlib
import json
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference/src"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))

from pnr import synth  # noqa: E402


# ---------------------------------------------------------------- stubs ----
def _install_stubs():
    cv2 = types.ModuleType("cv2")
    cv2.COLORMAP_HOT = 11
    sys.modules.setdefault("cv2", cv2)

    tv = types.ModuleType("torchvision")
    tvt = types.ModuleType("torchvision.transforms")
    tvm = types.ModuleType("torchvision.models")

    class _Any:
        def __init__(self, *a, **k):
            pass

        def __call__(self, x):
            return x

    for name in ("Compose", "ToTensor", "Normalize", "Resize", "ColorJitter"):
        setattr(tvt, name, _Any)
    tvt.functional = types.SimpleNamespace()

    def _resnet(**kw):
        return torch.nn.Module()

    tvm.resnet34 = _resnet
    tvm.resnet18 = _resnet
    tv.transforms = tvt
    tv.models = tvm
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.transforms", tvt)
    sys.modules.setdefault("torchvision.models", tvm)

    ph = types.ModuleType("pyhocon")
    ph.ConfigFactory = types.SimpleNamespace(parse_file=lambda *a, **k: None)
    sys.modules.setdefault("pyhocon", ph)

    dm = types.ModuleType("dotmap")

    class DotMap(dict):
        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError:
                raise AttributeError(k)

        def __setattr__(self, k, v):
            self[k] = v

        def toDict(self):
            return {k: (v.toDict() if isinstance(v, DotMap) else v) for k, v in self.items()}

    dm.DotMap = DotMap
    sys.modules.setdefault("dotmap", dm)


class Conf(dict):
    """pyhocon-like accessor over a nested dict (get_int / get_bool / ...)."""

    def __getitem__(self, k):
        v = dict.__getitem__(self, k)
        return Conf(v) if isinstance(v, dict) else v

    def _get(self, k, default=None):
        return self[k] if k in self else default

    get_int = get_float = get_bool = get_string = get_list = _get

    def get(self, k, default=None):
        return self._get(k, default)


def model_conf(d_hidden=512, num_layers=4, n_blocks=5, combine_layer=3, opts=None):
    """The shipped conf's model section; ``opts`` (the alt_* fixtures) sets the options the
    fused kernel does not implement: beta, combine_type, use_spade, use_code_viewdirs,
    index_padding / index_interp, global_latent_size (use_global_encoder)."""
    o = dict(opts or {})
    mlp = dict(type="resnet", n_blocks=n_blocks, d_hidden=d_hidden,
               combine_layer=combine_layer, combine_type=o.get("combine_type", "average"),
               beta=o.get("beta", 0.0), use_spade=o.get("use_spade", False))
    enc = dict(backbone="resnet34", pretrained=False, num_layers=num_layers,
               index_padding=o.get("index_padding", "border"), index_interp=o.get("index_interp", "bilinear"))
    conf = dict(
        use_encoder=True, use_global_encoder="global_latent_size" in o, use_xyz=True, canon_xyz=False,
        use_code=True, code=dict(num_freqs=6, freq_factor=1.5, include_input=True),
        use_viewdirs=True, use_code_viewdirs=o.get("use_code_viewdirs", False),
        mlp_coarse=dict(mlp), mlp_fine=dict(mlp), encoder=enc)
    if "global_latent_size" in o:
        conf["global_encoder"] = dict(backbone="resnet34", pretrained=False, latent_size=o["global_latent_size"])
    return Conf(conf)


def mlp_d_in(opts=None):
    """ResnetFC d_in of model_conf (models.py:49-60): xyz PE 39 + raw viewdirs 3, or the PE of
    (xyz, viewdirs) 6 + 72 with use_code_viewdirs."""
    return 78 if (opts or {}).get("use_code_viewdirs") else 42


@contextlib.contextmanager
def injected_rng(u_c, u_f, u_j, n_d):
    """Replace the renderer's random draws with the given streams, in order."""
    queue = [("rand_like", u_c)]
    if u_f.shape[1] > 0:
        queue += [("rand", u_f), ("rand_like", u_j)]
    if n_d.shape[1] > 0:
        queue += [("randn_like", n_d)]
    saved = (torch.rand_like, torch.rand, torch.randn_like)
    log = []

    def pop(kind, shape):
        # the coarse stream is drawn again by the fine pass? no: one queue per forward
        if not queue:
            raise RuntimeError("unexpected extra random draw " + kind)
        k, t = queue[0]
        if k != kind or tuple(t.shape) != tuple(shape):
            raise RuntimeError("draw mismatch: got %s%s, expected %s%s"
                               % (kind, tuple(shape), k, tuple(t.shape)))
        queue.pop(0)
        log.append(kind)
        return t.clone()

    torch.rand_like = lambda x, *a, **k: pop("rand_like", x.shape)
    torch.rand = lambda *s, **k: pop("rand", s if not isinstance(s[0], (tuple, list)) else s[0])
    torch.randn_like = lambda x, *a, **k: pop("randn_like", x.shape)
    try:
        yield log
    finally:
        torch.rand_like, torch.rand, torch.randn_like = saved
        if queue:
            raise RuntimeError("unused random streams: %s" % [q[0] for q in queue])


def build_reference_net(d_hidden, d_latent, seed, latent, poses, focal, c, width, height,
                        n_blocks=5, combine_layer=3, with_fine=True, opts=None, global_latent=None):
    from model import make_model  # reference src/model/__init__.py:4

    num_layers = {64: 1, 128: 2, 256: 3, 512: 4}[d_latent]
    o = opts or {}
    net = make_model(model_conf(d_hidden, num_layers, n_blocks, combine_layer, o))
    if not with_fine:
        net.mlp_fine = None
    sd = synth.pixelnerf_state(seed, d_in=mlp_d_in(o), d_latent=d_latent + o.get("global_latent_size", 0),
                               d_hidden=d_hidden, n_blocks=n_blocks, combine_layer=combine_layer,
                               with_fine=with_fine, use_spade=o.get("use_spade", False))
    missing, unexpected = net.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all(m.startswith("encoder.") or m.startswith("global_encoder.") for m in missing), missing
    enc = net.encoder
    if global_latent is not None:
        # what ImageEncoder.forward leaves behind (encoder.py:224-240): the latent is injected
        ge = net.global_encoder

        def fake_global(x):
            ge.latent = global_latent.clone()
            return ge.latent

        ge.forward = fake_global

    def fake_forward(x):
        # what SpatialEncoder.forward leaves behind (encoder.py:160-164)
        enc.latent = latent.clone()
        enc.latent_scaling[0] = enc.latent.shape[-1]
        enc.latent_scaling[1] = enc.latent.shape[-2]
        enc.latent_scaling = enc.latent_scaling / (enc.latent_scaling - 1) * 2.0
        return enc.latent

    enc.forward = fake_forward
    net.eval()
    if poses.dim() == 4:  # (SB, NS, 4, 4)
        images = torch.zeros(poses.shape[0], poses.shape[1], 3, height, width)
    else:
        images = torch.zeros(poses.shape[0], 3, height, width)
    net.encode(images, poses, focal, c=c)
    return net


def render_case(name, *, d_hidden, d_latent, seed, scene, n_coarse, n_fine, n_fine_depth,
                white_bkgd, lindisp=False, depth_std=0.01, sb=1, rng_seed=1,
                want_weights=True, force_u_high=0, with_fine=True, n_blocks=5,
                combine_layer=3, multi_obj_poses=None, focal_override=None, c_override=None,
                opts=None, global_latent=None):
    from render import NeRFRenderer  # reference src/render/__init__.py:1

    latent = scene["latent"]
    poses = scene["poses"] if multi_obj_poses is None else multi_obj_poses
    focal = scene["focal"] if focal_override is None else focal_override
    c = scene["c"] if c_override is None else c_override
    net = build_reference_net(d_hidden, d_latent, seed, latent, poses, focal, c,
                              scene["width"], scene["height"], n_blocks, combine_layer,
                              with_fine, opts, global_latent)
    renderer = NeRFRenderer(n_coarse=n_coarse, n_fine=n_fine, n_fine_depth=n_fine_depth,
                            depth_std=depth_std, white_bkgd=white_bkgd, lindisp=lindisp,
                            eval_batch_size=100000)
    rays = scene["rays"]
    B = rays.shape[0]
    assert B % sb == 0
    rays3 = rays.reshape(sb, B // sb, 8)
    u_c, u_f, u_j, n_d = synth.rng_streams(rng_seed, B, n_coarse, n_fine, n_fine_depth)
    if force_u_high and u_f.shape[1] > 0:
        u_f[:force_u_high, 0] = float(np.nextafter(np.float32(1.0), np.float32(0.0)))
    # capture what the renderer hands the model and what the model returns
    captured = {"z": [], "raw": []}
    orig_composite = renderer.composite

    def spy_composite(model, rays_, z_samp, coarse=True, sb=0):
        captured["z"].append(z_samp.detach().clone())
        return orig_composite(model, rays_, z_samp, coarse=coarse, sb=sb)

    renderer.composite = spy_composite
    orig_fwd = net.forward

    def spy_forward(xyz, coarse=True, viewdirs=None, far=False):
        out = orig_fwd(xyz, coarse=coarse, viewdirs=viewdirs, far=far)
        captured["raw"].append(out.detach().clone())
        return out

    net.forward = spy_forward
    with torch.no_grad(), injected_rng(u_c, u_f, u_j, n_d):
        out = renderer(net, rays3, want_weights=want_weights)
    cfg = dict(name=name, d_hidden=d_hidden, d_latent=d_latent, seed=seed,
               n_coarse=n_coarse, n_fine=n_fine, n_fine_depth=n_fine_depth,
               white_bkgd=bool(white_bkgd), lindisp=bool(lindisp), depth_std=depth_std,
               sb=sb, ns=int(latent.shape[0] // sb), width=scene["width"],
               height=scene["height"], near=scene["near"], far=scene["far"],
               latent_shape=list(latent.shape), rng_seed=rng_seed,
               force_u_high=force_u_high, with_fine=with_fine, n_blocks=n_blocks,
               combine_layer=combine_layer, latent_seed=scene["latent_seed"], opts=dict(opts or {}))
    arrays = dict(
        rays=rays3.numpy(), poses=poses.numpy(),
        focal=np.asarray(focal, dtype=np.float32),
        c=(np.asarray(c, dtype=np.float32) if c is not None else np.zeros(0, np.float32)),
        u_coarse=u_c.numpy(), u_fine=u_f.numpy(), u_fine_jit=u_j.numpy(), n_depth=n_d.numpy(),
        coarse_rgb=out.coarse.rgb.numpy(), coarse_depth=out.coarse.depth.numpy(),
        coarse_weights=out.coarse.weights.numpy(),
        z_coarse=captured["z"][0].numpy(),
    )
    if global_latent is not None:
        arrays["global_latent"] = global_latent.numpy()
    # model outputs of each pass, flattened to (SB*B'*K, 4) in ray-major order
    arrays["raw_coarse"] = torch.cat([r.reshape(-1, 4) for r in captured["raw"][:1]]).numpy()
    if "fine" in out:
        arrays.update(fine_rgb=out.fine.rgb.numpy(), fine_depth=out.fine.depth.numpy(),
                      fine_weights=out.fine.weights.numpy(), z_fine=captured["z"][1].numpy(),
                      raw_fine=torch.cat([r.reshape(-1, 4) for r in captured["raw"][1:]]).numpy())
    return cfg, arrays


def point_query_case(name, *, seed, scene, n_points, d_hidden=512, d_latent=512):
    """Direct model query (models.py:146-266) as eval.py:97-101 does it."""
    net = build_reference_net(d_hidden, d_latent, seed, scene["latent"], scene["poses"],
                              scene["focal"], scene["c"], scene["width"], scene["height"])
    xyz = torch.from_numpy(synth.hash_sym(seed + 99, (1, n_points, 3), 0.6))
    with torch.no_grad():
        out = net(xyz, coarse=True, viewdirs=torch.zeros(1, n_points, 3))
        out_f = net(xyz, coarse=False, viewdirs=torch.zeros(1, n_points, 3))
    cfg = dict(name=name, seed=seed, n_points=n_points, d_hidden=d_hidden,
               d_latent=d_latent, width=scene["width"], height=scene["height"],
               latent_shape=list(scene["latent"].shape), ns=1, sb=1,
               latent_seed=scene["latent_seed"])
    arrays = dict(xyz=xyz.numpy(), poses=scene["poses"].numpy(),
                  focal=np.asarray(scene["focal"], dtype=np.float32),
                  c=np.zeros(0, np.float32), out_coarse=out.numpy(), out_fine=out_f.numpy())
    return cfg, arrays


def composite_case(name, seed=5, B=48, K=24, white_bkgd=True):
    """Alpha composite on hand-made model outputs incl. all-zero sigma rows."""
    from render import NeRFRenderer

    g = torch.Generator().manual_seed(seed)
    near, far = 0.5, 3.0
    rays = torch.cat([torch.randn(B, 6, generator=g), torch.full((B, 1), near),
                      torch.full((B, 1), far)], 1)
    t = torch.sort(torch.rand(B, K, generator=g), -1)[0]
    z = near * (1 - t) + far * t
    raw = torch.rand(B, K, 4, generator=g)
    raw[..., 3] = torch.relu(torch.randn(B, K, generator=g) * 3.0)
    raw[:4, :, 3] = 0.0          # all-zero sigma rays
    raw[4:8, :, 3] = 1e4         # saturating rays
    r = NeRFRenderer(n_coarse=K, white_bkgd=white_bkgd)

    class M:
        use_viewdirs = False

        def __call__(self, pts, coarse=True):
            return raw.reshape(1, -1, 4)

    with torch.no_grad():
        w, rgb, depth = r.composite(M(), rays, z, coarse=True, sb=1)
    cfg = dict(name=name, B=B, K=K, white_bkgd=white_bkgd)
    return cfg, dict(rays=rays.numpy(), z=z.numpy(), raw=raw.numpy(), weights=w.numpy(),
                     rgb=rgb.numpy(), depth=depth.numpy())


def train_case(name, *, d_hidden=32, d_latent=64, seed=21, rng_seed=6, sb=2, rays_per_obj=12,
               n_coarse=16, n_fine=12, n_fine_depth=4, white_bkgd=True):
    """One training step's loss and gradients (train.py:182-283: MSE(coarse) + MSE(fine),
    lambda = 1) through the reference renderer + model under autograd, with the depth
    samples' gradient path (nerf.py:292, depth not detached).  The encoder latent is a
    leaf (what SpatialEncoder.forward would hand the trunk's backward)."""
    from render import NeRFRenderer

    sc = synth.scene_multiview(seed=9, n_views=sb, n_rays=sb * rays_per_obj, channels=d_latent,
                               h_l=6, w_l=7)
    poses = sc["poses"].reshape(sb, 1, 4, 4)
    focal = torch.tensor([[90.0, 95.0], [80.0, 85.0]])[:sb]
    c = torch.tensor([[31.0, 30.0], [33.0, 29.0]])[:sb]
    latent = sc["latent"].clone().requires_grad_(True)
    net = build_reference_net(d_hidden, d_latent, seed, latent, poses, focal, c, sc["width"],
                              sc["height"])
    net.train()
    for k, p in net.named_parameters():
        p.requires_grad_(not k.startswith("encoder."))
    # keep the latent leaf in the graph (fake_forward cloned it)
    net.encoder.latent = latent
    renderer = NeRFRenderer(n_coarse=n_coarse, n_fine=n_fine, n_fine_depth=n_fine_depth,
                            depth_std=0.05, white_bkgd=white_bkgd, eval_batch_size=100000)
    rays = sc["rays"].reshape(sb, rays_per_obj, 8)
    B = sb * rays_per_obj
    u_c, u_f, u_j, n_d = synth.rng_streams(rng_seed, B, n_coarse, n_fine, n_fine_depth)
    target = torch.from_numpy(synth.hash_uniform(rng_seed + 100, B * 3).astype(np.float32)).reshape(sb, -1, 3)
    with injected_rng(u_c, u_f, u_j, n_d):
        out = renderer(net, rays, want_weights=True)
    loss = torch.nn.functional.mse_loss(out.coarse.rgb, target) + \
        torch.nn.functional.mse_loss(out.fine.rgb, target)
    loss.backward()
    cfg = dict(name=name, d_hidden=d_hidden, d_latent=d_latent, seed=seed, rng_seed=rng_seed, sb=sb,
               n_coarse=n_coarse, n_fine=n_fine, n_fine_depth=n_fine_depth, depth_std=0.05,
               white_bkgd=white_bkgd, width=sc["width"], height=sc["height"],
               latent_seed=sc["latent_seed"])
    arrays = dict(rays=rays.numpy(), poses=poses.numpy(), focal=focal.numpy(), c=c.numpy(),
                  latent=latent.detach().numpy(), target=target.numpy(), u_coarse=u_c.numpy(),
                  u_fine=u_f.numpy(), u_fine_jit=u_j.numpy(), n_depth=n_d.numpy(),
                  loss=np.float32(loss.item()), coarse_rgb=out.coarse.rgb.detach().numpy(),
                  fine_rgb=out.fine.rgb.detach().numpy(), grad_latent=latent.grad.numpy())
    for k, p in net.named_parameters():
        if p.grad is not None:
            arrays["grad." + k] = p.grad.numpy()
    return cfg, arrays


def frame_case(name, *, seed=1, size=32, rng_seed=8):
    """gen_video.py:174-236 on one 32x32 frame: reference gen_rays -> render_par
    (bind_parallel(simple_output=True)) -> fine rgb frame -> uint8 by truncation.
    Shipped renderer conf (64 coarse + 32 fine incl. 16 depth, white background)."""
    import util
    from render import NeRFRenderer

    sc = synth.scene_srn(seed=0, n_rays=1)
    net = build_reference_net(512, 512, seed, sc["latent"], sc["poses"], sc["focal"], None,
                              sc["width"], sc["height"])
    renderer = NeRFRenderer(n_coarse=64, n_fine=32, n_fine_depth=16, depth_std=0.01,
                            white_bkgd=True, eval_batch_size=100000)
    render_par = renderer.bind_parallel(net, gpus=None, simple_output=True)
    focal = torch.tensor(131.25 * size / 128.0)
    rays = util.gen_rays(synth.srn_poses([40.0]), size, size, focal, 0.01, 4.0)   # (1, H, W, 8)
    B = size * size
    u_c, u_f, u_j, n_d = synth.rng_streams(rng_seed, B, 64, 32, 16)
    # what each composite pass saw and produced (fine-pass flips are classified on them)
    captured = []
    orig_composite = renderer.composite

    def spy_composite(model, rays_, z_samp, coarse=True, sb=0):
        res = orig_composite(model, rays_, z_samp, coarse=coarse, sb=sb)
        captured.append((z_samp.detach().clone(), res[0].detach().clone()))
        return res

    renderer.composite = spy_composite
    with torch.no_grad(), injected_rng(u_c, u_f, u_j, n_d):
        rgb, depth = render_par(rays.view(-1, 8)[None])
    frames = rgb[0].view(-1, size, size, 3)
    cfg = dict(name=name, seed=seed, size=size, rng_seed=rng_seed, latent_seed=sc["latent_seed"],
               width=sc["width"], height=sc["height"])
    return cfg, dict(rays=rays.numpy(), poses=sc["poses"].numpy(), focal=np.asarray(sc["focal"]),
                     u_coarse=u_c.numpy(), u_fine=u_f.numpy(), u_fine_jit=u_j.numpy(),
                     n_depth=n_d.numpy(), frames=frames.numpy(), depth=depth[0].numpy(),
                     frames_u8=(frames.numpy() * 255).astype(np.uint8),
                     coarse_weights=captured[0][1].numpy(),
                     z_fine=captured[1][0].numpy())


def gen_rays_case(name):
    """util.gen_rays (util.py:238-276): (fx, fy) + principal point, and scalar focal with
    the default image-centre principal point."""
    import util

    poses = synth.srn_poses([0.0, 37.0, 141.0], radius=1.7)
    focal = torch.tensor([52.0, 55.0])
    c = torch.tensor([19.5, 16.0])
    with torch.no_grad():
        r1 = util.gen_rays(poses, 40, 30, focal, 0.8, 1.8, c=c)
        r2 = util.gen_rays(poses[:2], 33, 21, torch.tensor(61.25), 0.01, 4.0)
    cfg = dict(name=name, w1=40, h1=30, near1=0.8, far1=1.8, w2=33, h2=21, near2=0.01, far2=4.0,
               focal2=61.25)
    return cfg, dict(poses=poses.numpy(), focal1=focal.numpy(), c1=c.numpy(), rays1=r1.numpy(),
                     rays2=r2.numpy())


def bbox_sample_case(name):
    """util.bbox_sample (util.py:220-235) from a seeded host generator: float boxes as the SRN
    loader makes them (and the area-resampled, non-integer ones), and integer boxes."""
    import util

    boxes = torch.tensor([[10.0, 12.0, 90.0, 100.0], [0.0, 0.0, 127.0, 127.0], [40.5, 33.25, 60.75, 70.5]])
    iboxes = torch.tensor([[3, 4, 20, 9], [0, 0, 0, 0]])
    torch.manual_seed(2024)
    pix = util.bbox_sample(boxes, 300)
    torch.manual_seed(7)
    ipix = util.bbox_sample(iboxes, 64)
    cfg = dict(name=name, seed=2024, num_pix=300, iseed=7, inum_pix=64)
    return cfg, dict(boxes=boxes.numpy(), pix=pix.numpy(), iboxes=iboxes.numpy(), ipix=ipix.numpy())


def save(cfg, arrays):
    path = os.path.join(HERE, cfg["name"] + ".npz")
    np.savez_compressed(path, config=np.array(json.dumps(cfg)), **arrays)
    print("wrote", os.path.relpath(path, REPO), "%.1f KB" % (os.path.getsize(path) / 1024))


def main():
    if not os.path.isdir(REF):
        print("reference not present; nothing to do")
        return 0
    _install_stubs()
    sys.path.insert(0, REF)
    torch.set_num_threads(os.cpu_count() or 1)
    only = set(sys.argv[1:])

    def want(n):
        return not only or n in only

    # --- reduced-width, fast cases (oracle pinning on CPU) --------------------
    if want("rw_ns1"):
        sc = synth.scene_srn(seed=3, n_rays=64, channels=64, h_l=8, w_l=8, pick="hash")
        save(*render_case("rw_ns1", d_hidden=64, d_latent=64, seed=11, scene=sc,
                          n_coarse=16, n_fine=16, n_fine_depth=8, white_bkgd=True,
                          force_u_high=5))
    if want("rw_lindisp"):
        sc = synth.scene_srn(seed=4, n_rays=48, channels=64, h_l=8, w_l=8, pick="hash",
                             near=0.8, far=1.8)
        save(*render_case("rw_lindisp", d_hidden=64, d_latent=64, seed=12, scene=sc,
                          n_coarse=16, n_fine=12, n_fine_depth=4, white_bkgd=False,
                          lindisp=True, rng_seed=2))
    if want("rw_ns3_sb2"):
        sc = synth.scene_multiview(seed=5, n_views=6, n_rays=64, channels=64, h_l=10, w_l=12)
        # two objects x three views: poses (SB, NS, 4, 4), per-object focal (SB, 2) and c
        poses = sc["poses"].reshape(2, 3, 4, 4)
        focal = torch.tensor([[300.0, 310.0], [280.0, 290.0]])
        c = torch.tensor([[195.0, 152.0], [200.0, 148.0]])
        save(*render_case("rw_ns3_sb2", d_hidden=64, d_latent=64, seed=13, scene=sc,
                          n_coarse=16, n_fine=16, n_fine_depth=0, white_bkgd=False, sb=2,
                          rng_seed=3, multi_obj_poses=poses, focal_override=focal,
                          c_override=c))
    if want("rw_coarse_only"):
        sc = synth.scene_srn(seed=6, n_rays=40, channels=64, h_l=8, w_l=8)
        save(*render_case("rw_coarse_only", d_hidden=64, d_latent=64, seed=14, scene=sc,
                          n_coarse=24, n_fine=0, n_fine_depth=0, white_bkgd=True,
                          rng_seed=4, with_fine=False))
    if want("composite_edge"):
        save(*composite_case("composite_edge"))
    # --- full-width cases (GPU parity pinning) ---------------------------------
    if want("fw_cfg2"):
        sc = synth.scene_srn(seed=0, n_rays=32, pick="hash")
        save(*render_case("fw_cfg2", d_hidden=512, d_latent=512, seed=1, scene=sc,
                          n_coarse=64, n_fine=64, n_fine_depth=0, white_bkgd=True))
    if want("fw_shipped"):
        sc = synth.scene_srn(seed=0, n_rays=32, pick="hash")
        save(*render_case("fw_shipped", d_hidden=512, d_latent=512, seed=1, scene=sc,
                          n_coarse=64, n_fine=32, n_fine_depth=16, white_bkgd=True,
                          rng_seed=7, force_u_high=2))
    if want("fw_cfg1"):
        sc = synth.scene_srn(seed=0, n_rays=256)
        save(*render_case("fw_cfg1", d_hidden=512, d_latent=512, seed=1, scene=sc,
                          n_coarse=32, n_fine=0, n_fine_depth=0, white_bkgd=True,
                          rng_seed=9, with_fine=False))
    if want("fw_dtu_ns3"):
        # cfg4 geometry at full size per view: latent (3, 512, 150, 200), 400x300 images
        sc = synth.scene_multiview(seed=8, n_views=3, n_rays=64, h_l=150, w_l=200)
        save(*render_case("fw_dtu_ns3", d_hidden=512, d_latent=512, seed=2, scene=sc,
                          n_coarse=64, n_fine=64, n_fine_depth=0, white_bkgd=False,
                          rng_seed=5, multi_obj_poses=sc["poses"][None],
                          focal_override=sc["focal"][None], c_override=sc["c"][None]))
    if want("fw_cfg3_nmr"):
        # cfg3: ShapeNet-NMR 64x64, latent 32x32, near/far 1.2/4.0, 64 + 64, white background
        sc = synth.scene_nmr(seed=3, n_rays=128)
        save(*render_case("fw_cfg3_nmr", d_hidden=512, d_latent=512, seed=3, scene=sc,
                          n_coarse=64, n_fine=64, n_fine_depth=0, white_bkgd=True, rng_seed=10,
                          force_u_high=2))
    if want("fw_cfg2_b128"):
        # cfg2 on 128 rays of the frame (hashed pixels), a second weight / stream seed
        sc = synth.scene_srn(seed=0, n_rays=128, pick="hash", theta_tgt=60.0)
        save(*render_case("fw_cfg2_b128", d_hidden=512, d_latent=512, seed=7, scene=sc,
                          n_coarse=64, n_fine=64, n_fine_depth=0, white_bkgd=True, rng_seed=11))
    if want("train_step"):
        save(*train_case("train_step"))
    if want("bbox_sample"):
        save(*bbox_sample_case("bbox_sample"))
    if want("gen_rays"):
        save(*gen_rays_case("gen_rays"))
    if want("frame32"):
        save(*frame_case("frame32"))
    # --- confs the fused kernel does not implement (the callback path) ----
    if want("alt_softplus"):
        sc = synth.scene_srn(seed=0, n_rays=32, pick="hash")
        save(*render_case("alt_softplus", d_hidden=512, d_latent=512, seed=31, scene=sc, n_coarse=64,
                          n_fine=32, n_fine_depth=16, white_bkgd=True, rng_seed=12, opts=dict(beta=100.0)))
    if want("alt_dh256"):
        sc = synth.scene_srn(seed=0, n_rays=32, pick="hash")
        save(*render_case("alt_dh256", d_hidden=256, d_latent=512, seed=32, scene=sc, n_coarse=64,
                          n_fine=64, n_fine_depth=0, white_bkgd=True, rng_seed=13))
    if want("alt_nl3"):
        sc = synth.scene_nmr(seed=3, n_rays=32, channels=256)
        save(*render_case("alt_nl3", d_hidden=512, d_latent=256, seed=33, scene=sc, n_coarse=64,
                          n_fine=64, n_fine_depth=0, white_bkgd=True, rng_seed=14))
    if want("alt_codevd"):
        sc = synth.scene_srn(seed=0, n_rays=32, pick="hash")
        save(*render_case("alt_codevd", d_hidden=512, d_latent=512, seed=34, scene=sc, n_coarse=64,
                          n_fine=32, n_fine_depth=16, white_bkgd=True, rng_seed=15,
                          opts=dict(use_code_viewdirs=True)))
    if want("alt_spade_max"):
        sc = synth.scene_multiview(seed=6, n_views=2, n_rays=32, channels=64, h_l=12, w_l=16)
        save(*render_case("alt_spade_max", d_hidden=128, d_latent=64, seed=35, scene=sc, n_coarse=32,
                          n_fine=16, n_fine_depth=0, white_bkgd=False, rng_seed=16,
                          multi_obj_poses=sc["poses"][None], focal_override=sc["focal"][None],
                          c_override=sc["c"][None], opts=dict(use_spade=True, combine_type="max")))
    if want("alt_global"):
        sc = synth.scene_srn(seed=0, n_rays=32, pick="hash", channels=64, h_l=16, w_l=16)
        gl = torch.from_numpy(synth.hash_normal(77, (1, 128)))
        save(*render_case("alt_global", d_hidden=256, d_latent=64, seed=36, scene=sc, n_coarse=32,
                          n_fine=32, n_fine_depth=0, white_bkgd=True, rng_seed=17,
                          opts=dict(global_latent_size=128), global_latent=gl))
    if want("alt_zeros_pad"):
        # grid_sample zeros padding: the target view sees past the source image's border
        sc = synth.scene_srn(seed=0, n_rays=32, pick="hash", theta_tgt=75.0, channels=64, h_l=16, w_l=16)
        save(*render_case("alt_zeros_pad", d_hidden=128, d_latent=64, seed=37, scene=sc, n_coarse=32,
                          n_fine=32, n_fine_depth=8, white_bkgd=True, rng_seed=18,
                          opts=dict(index_padding="zeros")))
    if want("fw_pointquery"):
        sc = synth.scene_srn(seed=0, n_rays=1)
        save(*point_query_case("fw_pointquery", seed=1, scene=sc, n_points=512))
    return 0


if __name__ == "__main__":
    sys.exit(main())
