"""Counter-mode draws (pnr_rng {seed, offset}, Philox4x32-10) and the a1 edge cases of the
fused march on an MI355X (``-m gpu``).

* pnr_rng_fill against the CPU restatement (oracle/philox.py): uniforms bit-exact,
  Box-Muller normals within 2e-6 (device logf / cosf vs numpy's);
* a counter-mode render is bit-identical to the injected-stream render of the same draws
  materialised by pnr_rng_fill, and matches the oracle renderer fed the oracle's Philox
  draws (fine pass classified by cause, oracle/parity.py);
* chunking a one-object batch (max_rays_per_call) leaves a counter-mode render unchanged;
* the draws' distribution: recovered stratified offsets U[0,1), sorted fine samples;
* using_fine with n_fine = 0 (fine MLP over the coarse samples, nerf.py:284-298) and
  training-mode sigma noise under no_grad (nerf.py:225-226) against the oracle.
"""
import numpy as np
import pytest
import torch

from oracle import parity, philox, ref_cpu
from pnr import _lib, ops, synth
from pnr.models import PixelNeRFNet
from pnr.renderer import NeRFRenderer

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
ATOL, RTOL = 5e-5, 1e-5


def close(a, b, atol=ATOL, rtol=RTOL):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return bool(((a - b).abs() <= atol + rtol * b.abs()).all())


def conf():
    mlp = dict(type="resnet", n_blocks=5, d_hidden=512, combine_layer=3, combine_type="average")
    return dict(use_encoder=True, use_xyz=True, use_code=True, code=dict(num_freqs=6, freq_factor=1.5),
                use_viewdirs=True, use_code_viewdirs=False, mlp_coarse=mlp, mlp_fine=dict(mlp),
                encoder=dict(backbone="resnet34", pretrained=False, num_layers=4))


def setup(n_rays=64, seed=0):
    sd = synth.pixelnerf_state(1)
    sc = synth.scene_srn(seed=seed, n_rays=n_rays, pick="hash")
    net = PixelNeRFNet(conf())
    net.load_state_dict(sd, strict=False)
    net = net.to(DEV).eval()
    net.encode_latent(sc["latent"].to(DEV), sc["poses"].to(DEV), sc["focal"].to(DEV), (128, 128))
    scene = ref_cpu.Scene(sc["latent"], sc["poses"], sc["focal"], 128, 128, None)
    model_fn = lambda p, c, d: ref_cpu.pixelnerf_forward(sd, scene, p, c, d)  # noqa: E731
    model_fn.scene = scene
    return net, sc, model_fn


def render(net, rays, kc, kf, kfd=0, streams=None, max_rays=None, **kw):
    r = NeRFRenderer(n_coarse=kc, n_fine=kf, n_fine_depth=kfd, white_bkgd=True, **kw)
    r.streams = streams
    r.return_z = True
    if max_rays:
        r.max_rays_per_call = max_rays
    with torch.no_grad():
        out = r(net, rays.to(DEV), want_weights=True)
    torch.cuda.synchronize()
    return r, out


def test_rng_fill_matches_philox_restatement():
    seed, off = 0xDEADBEEF12345678, 1000
    for s, width in ((philox.U_COARSE, 64), (philox.U_FINE, 48), (philox.U_FINE_JIT, 48), (philox.N_DEPTH, 16)):
        got = ops.rng_fill(seed, off, s, 777, width, DEV).cpu().numpy()
        want = philox.stream(seed, off, s, 777, width)
        if s == philox.N_DEPTH:
            assert np.abs(got - want).max() <= 2e-6 * (1.0 + np.abs(want).max())
        else:
            assert np.array_equal(got, want), s


def test_counter_render_equals_injected_replay_and_oracle():
    net, sc, model_fn = setup(64)
    torch.manual_seed(11)
    r, out = render(net, sc["rays"][None], 64, 32, 16)
    seed = r.last_seed
    streams = ops.rng_render_streams(seed, 0, 64, 64, 32, 16, DEV)
    _, rep = render(net, sc["rays"][None], 64, 32, 16, streams=streams)
    for p in ("coarse", "fine"):
        for k in ("rgb", "depth", "weights", "z"):
            assert torch.equal(out[p][k], rep[p][k]), (p, k)
    # reproducible under torch.manual_seed
    torch.manual_seed(11)
    _, again = render(net, sc["rays"][None], 64, 32, 16)
    assert torch.equal(out.fine.rgb, again.fine.rgb)
    # the oracle fed the oracle's own Philox draws
    st = tuple(torch.from_numpy(a) for a in philox.render_streams(seed, 0, 64, 64, 32, 16))
    with torch.no_grad():
        ref = ref_cpu.render(model_fn, sc["rays"][None], 64, 32, 16, st, True)
    assert close(out.coarse.rgb, ref["coarse"]["rgb"]) and close(out.coarse.weights, ref["coarse"]["weights"])
    z_exp = parity.expected_fine_sets(sc["rays"], out.coarse.z, out.coarse.weights, out.coarse.depth, st, 64, 32, 16)
    cls = parity.classify_fine(out.coarse.weights[0], ref["coarse"]["weights"][0], st[1], out.fine.z[0],
                               ref["fine"]["z"], z_exp)
    assert not cls["unexplained"].any() and not cls["inconsistent"].any() and len(cls["flip_idx"]) <= 1
    if cls["flip_idx"]:   # a flipped ray's outputs against the oracle fine pass at its own samples
        res = parity.check_flipped_outputs(synth.pixelnerf_state(1), model_fn.scene, sc["rays"], out.fine.z,
                                           out.fine.rgb, out.fine.depth, out.fine.weights, cls["flip_idx"], 64,
                                           True, w_coarse_hip=out.coarse.weights, u_fine=st[1])
        assert res["ok"], res
    keep = ~cls["flip"]
    assert close(out.fine.rgb[0].cpu()[keep], ref["fine"]["rgb"][0][keep])
    assert close(out.fine.depth[0].cpu()[keep], ref["fine"]["depth"][0][keep])


def test_counter_render_is_chunk_invariant():
    net, sc, _ = setup(256, seed=2)
    torch.manual_seed(5)
    _, whole = render(net, sc["rays"][None], 64, 64)
    torch.manual_seed(5)
    _, chunked = render(net, sc["rays"][None], 64, 64, max_rays=100)
    # eval_batch_size bounds a call's rays the same way (the reference's chunk knob)
    torch.manual_seed(5)
    _, ebs = render(net, sc["rays"][None], 64, 64, eval_batch_size=96)
    for p in ("coarse", "fine"):
        for k in ("rgb", "depth", "weights", "z"):
            assert torch.equal(whole[p][k], chunked[p][k]), (p, k)
            assert torch.equal(whole[p][k], ebs[p][k]), (p, k, "eval_batch_size")


def test_counter_draw_distribution():
    """4096 rays x 64 coarse samples: the stratified offsets recovered from z are U[0,1)
    (the kernels use the draws as sample_coarse does, nerf.py:109-113); fine z sorted."""
    sc = synth.scene_srn(seed=3, n_rays=4096, pick="hash")
    rays = sc["rays"].to(DEV)
    u = ops.rng_fill(99, 0, _lib.RNG_U_COARSE, 4096, 64, DEV)
    z = ops.sample_coarse(rays, 64, u, False)
    near, far = rays[:, 6:7], rays[:, 7:8]
    t = (z - near) / (far - near) * 64 - torch.arange(64, device=DEV)
    t = t.double()
    assert float(t.min()) > -1e-3 and float(t.max()) < 1 + 1e-3
    assert abs(float(t.mean()) - 0.5) < 3e-3 and abs(float(t.var()) - 1 / 12) < 2e-3
    net, _, _ = setup(64)
    _, out = render(net, sc["rays"][None, :512], 64, 64)
    zf = out.fine.z[0]
    assert bool((zf[:, 1:] >= zf[:, :-1]).all())


def test_fine_pass_over_coarse_samples_when_n_fine_is_zero():
    net, sc, model_fn = setup(48)
    streams = synth.rng_streams(4, 48, 64, 0, 0)
    r = NeRFRenderer(n_coarse=64, n_fine=16, white_bkgd=True)
    r.n_fine = 0                      # callers mutate n_fine after construction (gen_video.py:192-195)
    assert r.using_fine
    r.streams = streams
    with torch.no_grad():
        out = r(net, sc["rays"][None].to(DEV), want_weights=True)
        ref = ref_cpu.render(model_fn, sc["rays"][None], 64, 0, 0, streams, True, using_fine=True)
    assert out.fine.weights.shape[-1] == 64
    for p in ("coarse", "fine"):
        assert close(out[p].rgb, ref[p]["rgb"]) and close(out[p].depth, ref[p]["depth"])
        assert close(out[p].weights, ref[p]["weights"])
    assert not torch.equal(out.coarse.rgb, out.fine.rgb)   # the fine MLP ran


def test_training_mode_sigma_noise_without_grad():
    net, sc, model_fn = setup(32)
    B, kc, kf, kfd, std = 32, 64, 32, 16, 0.5
    r = NeRFRenderer(n_coarse=kc, n_fine=kf, n_fine_depth=kfd, noise_std=std, white_bkgd=True).train()
    torch.manual_seed(21)
    with torch.no_grad():
        out = r(net, sc["rays"][None].to(DEV), want_weights=True)
    # replay the reference's draw order (nerf.py:111, 226, 135, 141, 158, 226) on the device
    torch.manual_seed(21)
    u_c = torch.rand(B, kc, device=DEV)
    n_c = torch.randn(B, kc, device=DEV)
    u_f, u_j = torch.rand(B, kf - kfd, device=DEV), torch.rand(B, kf - kfd, device=DEV)
    n_d = torch.randn(B, kfd, device=DEV)
    n_f = torch.randn(B, kc + kf, device=DEV)
    st = tuple(t.cpu() for t in (u_c, u_f, u_j, n_d))
    with torch.no_grad():
        ref = ref_cpu.render(model_fn, sc["rays"][None], kc, kf, kfd, st, True,
                             sigma_noise=(n_c.cpu() * std, n_f.cpu() * std))
    assert close(out.coarse.rgb, ref["coarse"]["rgb"]) and close(out.coarse.weights, ref["coarse"]["weights"])
    # the fine pass: same rule as every fixture (flips proven from the coarse weights)
    z_ref = ref["fine"]["z"]
    bins_h = parity.fine_bins(out.coarse.weights[0], st[1])
    bins_r = parity.fine_bins(ref["coarse"]["weights"][0], st[1])
    keep = ~(bins_h != bins_r).any(-1)
    assert int((~keep).sum()) <= 1
    assert close(out.fine.rgb[0].cpu()[keep], ref["fine"]["rgb"][0][keep])
    with torch.no_grad():
        r.eval()
        quiet = r(net, sc["rays"][None].to(DEV))
    assert not torch.equal(quiet.coarse.rgb, out.coarse.rgb)   # the noise was applied
