"""Pin the oracle (oracle/ref_cpu.py) against vectors produced by the reference.

The fixtures in tests/golden/ were made by running the reference's own
NeRFRenderer/PixelNeRFNet (tests/golden/make_golden.py).  The oracle restates
the same op sequence on CPU fp32, so on the same machine it matches to
<= 1e-6 absolute.
"""
import pytest
import torch

import fixtures
from oracle import ref_cpu

RENDER_CASES = ["rw_ns1", "rw_lindisp", "rw_ns3_sb2", "rw_coarse_only",
                "fw_cfg2", "fw_shipped", "fw_cfg1", "fw_dtu_ns3", "fw_cfg3_nmr", "fw_cfg2_b128"]
ATOL = 1e-6


def oracle_render(cfg, arr):
    sd = fixtures.state_dict(cfg)
    scene = ref_cpu.Scene(fixtures.latent_of(cfg), arr["poses"], fixtures.focal_of(arr),
                          cfg["width"], cfg["height"], fixtures.c_or_none(arr))
    has_fine = cfg.get("with_fine", True)

    def model_fn(pts, coarse, dirs):
        return ref_cpu.pixelnerf_forward(sd, scene, pts, coarse, dirs,
                                         d_latent=cfg["d_latent"],
                                         n_blocks=cfg.get("n_blocks", 5),
                                         combine_layer=cfg.get("combine_layer", 3),
                                         has_fine=has_fine)

    streams = (arr["u_coarse"], arr["u_fine"], arr["u_fine_jit"], arr["n_depth"])
    return ref_cpu.render(model_fn, arr["rays"], cfg["n_coarse"], cfg["n_fine"],
                          cfg["n_fine_depth"], streams, cfg["white_bkgd"],
                          lindisp=cfg["lindisp"], depth_std=cfg["depth_std"])


@pytest.mark.parametrize("name", RENDER_CASES)
def test_oracle_render_matches_reference(name):
    torch.set_num_threads(4)
    cfg, arr = fixtures.load(name)
    with torch.no_grad():
        out = oracle_render(cfg, arr)
    c = out["coarse"]
    torch.testing.assert_close(c["z"], arr["z_coarse"], atol=ATOL, rtol=0)
    torch.testing.assert_close(c["raw"], arr["raw_coarse"], atol=ATOL, rtol=0)
    torch.testing.assert_close(c["rgb"], arr["coarse_rgb"], atol=ATOL, rtol=0)
    torch.testing.assert_close(c["depth"], arr["coarse_depth"], atol=ATOL, rtol=0)
    torch.testing.assert_close(c["weights"], arr["coarse_weights"], atol=ATOL, rtol=0)
    if cfg["n_fine"] > 0:
        f = out["fine"]
        torch.testing.assert_close(f["z"], arr["z_fine"], atol=ATOL, rtol=0)
        torch.testing.assert_close(f["raw"], arr["raw_fine"], atol=ATOL, rtol=0)
        torch.testing.assert_close(f["rgb"], arr["fine_rgb"], atol=ATOL, rtol=0)
        torch.testing.assert_close(f["depth"], arr["fine_depth"], atol=ATOL, rtol=0)
        torch.testing.assert_close(f["weights"], arr["fine_weights"], atol=ATOL, rtol=0)
    else:
        assert "fine" not in out


def test_oracle_forced_u_high_goes_past_far():
    """u >= cdf[-1] gives ind = Kc, i.e. a fine sample beyond far."""
    cfg, arr = fixtures.load("rw_ns1")
    assert cfg["force_u_high"] > 0
    far = arr["rays"].reshape(-1, 8)[:, 7]
    zf = arr["z_fine"]
    n_past = int((zf[: cfg["force_u_high"]] > far[: cfg["force_u_high"], None] + 1e-6).any(1).sum())
    assert n_past >= 1


def test_oracle_composite_edges():
    cfg, arr = fixtures.load("composite_edge")
    w, rgb, depth = ref_cpu.composite(arr["rays"], arr["z"], arr["raw"], cfg["white_bkgd"])
    torch.testing.assert_close(w, arr["weights"], atol=ATOL, rtol=0)
    torch.testing.assert_close(rgb, arr["rgb"], atol=ATOL, rtol=0)
    torch.testing.assert_close(depth, arr["depth"], atol=ATOL, rtol=0)
    # all-zero sigma rays: no weight, white background
    assert float(w[:4].abs().max()) == 0.0
    torch.testing.assert_close(rgb[:4], torch.ones(4, 3))


def test_oracle_point_query():
    torch.set_num_threads(4)
    cfg, arr = fixtures.load("fw_pointquery")
    sd = fixtures.state_dict(cfg)
    scene = ref_cpu.Scene(fixtures.latent_of(cfg), arr["poses"], fixtures.focal_of(arr),
                          cfg["width"], cfg["height"], None)
    vd = torch.zeros_like(arr["xyz"])
    with torch.no_grad():
        oc = ref_cpu.pixelnerf_forward(sd, scene, arr["xyz"], True, vd)
        of = ref_cpu.pixelnerf_forward(sd, scene, arr["xyz"], False, vd)
    torch.testing.assert_close(oc, arr["out_coarse"], atol=ATOL, rtol=0)
    torch.testing.assert_close(of, arr["out_fine"], atol=ATOL, rtol=0)


def test_host_gen_rays_matches_reference():
    """pnr.util.gen_rays on host tensors (the reference's host utility, restated) vs the
    reference's util.gen_rays output (tests/golden/gen_rays.npz)."""
    from pnr import util

    cfg, arr = fixtures.load("gen_rays")
    r1 = util.gen_rays(arr["poses"], cfg["w1"], cfg["h1"], arr["focal1"], cfg["near1"], cfg["far1"],
                       c=arr["c1"])
    r2 = util.gen_rays(arr["poses"][:2], cfg["w2"], cfg["h2"], torch.tensor(cfg["focal2"]),
                       cfg["near2"], cfg["far2"])
    assert r1.shape == arr["rays1"].shape and r2.shape == arr["rays2"].shape
    assert (r1 - arr["rays1"]).abs().max() <= 1e-6
    assert (r2 - arr["rays2"]).abs().max() <= 1e-6


def oracle_train_step(cfg, arr, sd, latent):
    """Loss of one training step (train.py:254-283) through the oracle under autograd."""
    scene = ref_cpu.Scene(latent, arr["poses"], arr["focal"], cfg["width"], cfg["height"], arr["c"])

    def model_fn(pts, coarse, dirs):
        return ref_cpu.pixelnerf_forward(sd, scene, pts, coarse, dirs, d_latent=cfg["d_latent"])

    streams = (arr["u_coarse"], arr["u_fine"], arr["u_fine_jit"], arr["n_depth"])
    out = ref_cpu.render(model_fn, arr["rays"], cfg["n_coarse"], cfg["n_fine"], cfg["n_fine_depth"],
                         streams, cfg["white_bkgd"], depth_std=cfg["depth_std"])
    mse = torch.nn.functional.mse_loss
    return mse(out["coarse"]["rgb"], arr["target"]) + mse(out["fine"]["rgb"], arr["target"]), out


def test_oracle_training_gradients_match_reference():
    """Oracle autograd reproduces the reference's training-step loss and every MLP / latent
    gradient (incl. the depth-sample path, nerf.py:292) of tests/golden/train_step.npz."""
    from pnr import synth

    torch.set_num_threads(4)
    cfg, arr = fixtures.load("train_step")
    sd = synth.pixelnerf_state(cfg["seed"], d_latent=cfg["d_latent"], d_hidden=cfg["d_hidden"])
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items() if k.startswith("mlp_")}
    sd.update(params)
    latent = arr["latent"].clone().requires_grad_(True)
    loss, out = oracle_train_step(cfg, arr, sd, latent)
    loss.backward()
    assert abs(loss.item() - float(arr["loss"])) <= 1e-6
    torch.testing.assert_close(out["fine"]["rgb"], arr["fine_rgb"], atol=1e-6, rtol=0)
    torch.testing.assert_close(latent.grad, arr["grad_latent"], atol=1e-6, rtol=1e-4)
    n = 0
    for k, p in params.items():
        ref = arr.get("grad." + k)
        assert ref is not None, k
        torch.testing.assert_close(p.grad, ref, atol=1e-6, rtol=1e-4, msg=k)
        n += 1
    assert n == len([k for k in arr if k.startswith("grad.mlp_")])
