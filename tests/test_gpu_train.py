"""Training step on the HIP path vs the oracle's autograd (``-m gpu``).

The oracle's training gradients are pinned to the reference's own autograd by
tests/test_oracle_golden.py::test_oracle_training_gradients_match_reference (reduced
width); here the HIP training path (pnr/train.py: saved-activation forward, per-layer
GEMM backward, composite / input-stage backward kernels) is compared with the oracle at
full width on identical rays, streams and targets, through the depth-sample gradient path.

Tolerance: every gradient tensor within 1e-4 of its own max-abs (fp32 GEMM arithmetic)
or 2e-4 (scaled-fp16 forward), and the loss within 1e-5 relative (measured: 9e-6 / 1.8e-5).
"""
import pytest
import torch

from oracle import ref_cpu
from pnr import synth
from pnr.models import PixelNeRFNet
from pnr.renderer import NeRFRenderer

pytestmark = pytest.mark.gpu
DEV = "cuda"


def conf(combine_layer=3):
    mlp = dict(type="resnet", n_blocks=5, d_hidden=512, combine_layer=combine_layer, combine_type="average")
    return dict(use_encoder=True, use_xyz=True, use_code=True,
                code=dict(num_freqs=6, freq_factor=1.5, include_input=True), use_viewdirs=True,
                use_code_viewdirs=False, mlp_coarse=dict(mlp), mlp_fine=dict(mlp),
                encoder=dict(backbone="resnet34", pretrained=False, num_layers=4))


def case(sb=2, rays_per_obj=8, kc=32, kf=24, kfd=8, seed=3, ns=1, combine_layer=3):
    sc = synth.scene_multiview(seed=seed, n_views=sb * ns, n_rays=sb * rays_per_obj, channels=512,
                               h_l=12, w_l=14)
    poses = sc["poses"].reshape(sb, ns, 4, 4) if ns > 1 else sc["poses"].reshape(sb, 4, 4)
    focal = torch.tensor([[300.0, 310.0], [290.0, 295.0]])[:sb]
    c = torch.tensor([[195.0, 152.0], [200.0, 148.0]])[:sb]
    rays = sc["rays"].reshape(sb, rays_per_obj, 8)
    B = sb * rays_per_obj
    streams = synth.rng_streams(seed + 1, B, kc, kf, kfd)
    target = torch.from_numpy(synth.hash_uniform(seed + 2, B * 3).astype("float32")).reshape(sb, -1, 3)
    return dict(sd=synth.pixelnerf_state(seed + 4, combine_layer=combine_layer), latent=sc["latent"], poses=poses, focal=focal, c=c,
                rays=rays, streams=streams, target=target, kc=kc, kf=kf, kfd=kfd,
                width=sc["width"], height=sc["height"])


def oracle_grads(cs):
    sd = dict(cs["sd"])
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items() if k.startswith("mlp_")}
    sd.update(params)
    latent = cs["latent"].clone().requires_grad_(True)
    poses = cs["poses"] if cs["poses"].dim() == 4 else cs["poses"][:, None]
    scene = ref_cpu.Scene(latent, poses, cs["focal"], cs["width"], cs["height"], cs["c"])

    def model_fn(pts, coarse, dirs):
        return ref_cpu.pixelnerf_forward(sd, scene, pts, coarse, dirs)

    out = ref_cpu.render(model_fn, cs["rays"], cs["kc"], cs["kf"], cs["kfd"], cs["streams"], True,
                         depth_std=0.05)
    mse = torch.nn.functional.mse_loss
    loss = mse(out["coarse"]["rgb"], cs["target"]) + mse(out["fine"]["rgb"], cs["target"])
    loss.backward()
    g = {k: p.grad for k, p in params.items()}
    g["latent"] = latent.grad
    return loss.item(), g


def hip_grads(cs, precision, wgrad_arith="f16x3"):
    net = PixelNeRFNet(conf())
    net.load_state_dict(cs["sd"], strict=False)
    net = net.to(DEV)
    net.mlp_precision = precision
    net.wgrad_arith = wgrad_arith
    latent = cs["latent"].to(DEV).requires_grad_(True)
    net.encode_latent(latent, cs["poses"].to(DEV), cs["focal"].to(DEV), (cs["width"], cs["height"]),
                      c=cs["c"].to(DEV), num_objs=cs["poses"].shape[0])
    r = NeRFRenderer(n_coarse=cs["kc"], n_fine=cs["kf"], n_fine_depth=cs["kfd"], depth_std=0.05,
                     white_bkgd=True).to(DEV)
    r.streams = cs["streams"]
    out = r(net, cs["rays"].to(DEV), want_weights=True)
    mse = torch.nn.functional.mse_loss
    tgt = cs["target"].to(DEV)
    loss = mse(out.coarse.rgb, tgt) + mse(out.fine.rgb, tgt)
    loss.backward()
    g = {k: p.grad.detach().cpu() for k, p in net.named_parameters()
         if k.startswith("mlp_") and p.grad is not None}
    g["latent"] = latent.grad.detach().cpu()
    return loss.item(), g


def compare(cs, precision, tol, wgrad_arith="f16x3"):
    ref_loss, ref = oracle_grads(cs)
    loss, got = hip_grads(cs, precision, wgrad_arith)
    assert abs(loss - ref_loss) <= 1e-5 * abs(ref_loss), (loss, ref_loss)
    assert set(ref) == set(got), set(ref) ^ set(got)
    worst = []
    for k in sorted(ref):
        a, b = got[k].reshape(-1).double(), ref[k].reshape(-1).double()
        scale = float(b.abs().max())
        err = float((a - b).abs().max())
        worst.append((err / max(scale, 1e-30), k))
        assert err <= tol * scale + 1e-9, "%s: max |d| %.3g vs max |ref| %.3g" % (k, err, scale)
    worst.sort()
    print("worst relative gradient error %.3g (%s)" % worst[-1])


@pytest.mark.parametrize("precision,tol,wgrad_arith", [("fp32", 1e-4, "f16x3"), ("f16x3", 2e-4, "f16x3"),
                                                       ("f16x3", 2e-4, "bf16x6")])
def test_training_step_gradients_match_oracle(precision, tol, wgrad_arith):
    torch.set_num_threads(8)
    compare(case(), precision, tol, wgrad_arith)


def test_fine_pass_depth_mask_changes_no_gradient(monkeypatch):
    """The fine pass's input backward computes dL/dz only for the depth samples (FinePass z_mask,
    pnr_points_input_backward_masked): every gradient equals the unmasked backward's (the other
    points' dL/dz never reaches the graph), up to the latent scatter's atomic order."""
    from pnr import train

    cs = case()
    loss_m, got = hip_grads(cs, "f16x3")
    orig = train.FinePass.__init__

    def unmasked(self, z_mask=None):
        orig(self, None)

    monkeypatch.setattr(train.FinePass, "__init__", unmasked)
    loss_u, ref = hip_grads(cs, "f16x3")
    assert loss_m == loss_u
    for k in ref:
        a, b = got[k].double(), ref[k].double()
        assert float((a - b).abs().max()) <= 1e-6 * float(b.abs().max()) + 1e-12, k


def conditioned(sd, margin=3.0, scale=0.1):
    """The state dict with every ReLU input held away from zero: weights scaled by `scale`,
    lin_in / fc_0 biases +-margin by a fixed sign pattern, the other biases 0 (sigma's
    lin_out bias 0.5).  A full-width network with hash weights has ~1e5 ReLU units carrying
    gradient, a few of them within fp32 rounding of zero; one that lands on the other side
    of the kink moves every gradient below it by percents (measured: a unit at 1.3e-6 in
    block 2).  Here no rounding can flip a mask, and both mask values still occur."""
    out = {}
    for k, v in sd.items():
        if not k.startswith("mlp_") or not v.is_floating_point():
            out[k] = v
            continue
        if k.endswith(".weight"):
            out[k] = v * scale
        elif k.endswith("lin_in.bias") or k.endswith("fc_0.bias"):
            sign = torch.where(torch.arange(v.numel()) % 3 == 0, -1.0, 1.0)
            out[k] = margin * sign
        elif k.endswith("lin_out.bias"):
            out[k] = torch.tensor([0.0, 0.0, 0.0, 0.5])
        else:
            out[k] = torch.zeros_like(v)
    return out


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-4), ("f16x3", 2e-4)])
def test_training_step_multiview_gradients_match_oracle(precision, tol):
    """train.py -V 2 (several source views per object, the DTU setting): SB = 2 objects x
    NS = 2 views with per-object focal / c; the view mean at combine_layer, per-view
    activation rows and the scatter into each view's latent.  Weights from `conditioned`."""
    torch.set_num_threads(8)
    cs = case(ns=2)
    cs["sd"] = conditioned(cs["sd"])
    compare(cs, precision, tol)


def capture_saves(monkeypatch):
    """Record the activation save of every RenderPoints forward (pnr/train.py) by pass."""
    from pnr import train

    caps = {}
    orig = train.RenderPoints.forward

    def forward(ctx, net, coarse, rays, z, latent_cl, *params):
        out = orig(ctx, net, coarse, rays, z, latent_cl, *params)
        save = ctx.to_save[3]   # save_for_backward(rays, z, out, save, latent_cl)
        caps[bool(coarse)] = dict(save=save.detach().clone(), P=z.numel(), ns=net.num_views_per_obj,
                                  nb=ctx.mlp.n_blocks, nc=ctx.mlp.combine_layer)
        return out

    monkeypatch.setattr(train.RenderPoints, "forward", staticmethod(forward))
    return caps


def margin_relu(caps, sb, margin_rel, stats):
    """ReLU-margin masking: the oracle's ReLU decides a unit itself unless its input is within
    margin_rel * max|input| of the kink, where it takes the HIP forward's decision (its saved
    relu output > 0).  Inside that band either side is a valid fp32 outcome; everywhere else
    a HIP mask that differs from the oracle's is a gradient error the comparison catches."""
    from pnr import train

    def for_pass(coarse):
        c = caps[coarse]
        P, ns, nb = c["P"], c["ns"], c["nb"]
        nc = min(c["nc"], nb) if ns > 1 else nb
        _, _, slot = train._save_views(c["save"], P, nb, ns=ns)

        def hip_mask(i, rows):
            m = (slot(i, rows) > 0).cpu()
            if rows == ns * P and ns > 1:   # HIP rows (view, object, point) -> oracle (object, view, point)
                m = m.reshape(ns, sb, P // sb, -1).transpose(0, 1).reshape(rows, -1)
            return m

        def relu(t, site):
            kind, b = site
            if kind == "xf":
                hip = hip_mask(2 * nb, P)
            else:
                rows = ns * P if b < nc else P
                hip = hip_mask(b if kind == "x" else nb + b, rows)
            assert hip.numel() == t.numel() and hip.shape[-1] == t.shape[-1], (site, hip.shape, t.shape)
            hip = hip.reshape(t.shape)   # after combine_layer the oracle's x is (objects, points, 512)
            band = t.detach().abs() < margin_rel * float(t.detach().abs().max())
            own = t.detach() > 0
            stats["band"] += int(band.sum())
            stats["adopted"] += int((band & (hip != own)).sum())
            stats["outside"] += int((~band & (hip != own)).sum())
            return t * torch.where(band, hip, own).to(t.dtype)

        return relu

    return {True: for_pass(True), False: for_pass(False)}


@pytest.mark.parametrize("precision,tol", [("fp32", 1e-4), ("f16x3", 2e-4)])
def test_training_step_multiview_unconditioned_relu_margin(precision, tol, monkeypatch):
    """SB = 2 x NS = 2 on the hash weights as drawn (no `conditioned` weights): ReLU units
    within 1e-4 of their layer's max |input| of the kink take the HIP forward's mask in the
    oracle (ReLU-margin masking, margin_relu); every other mask is the oracle's own, and all
    gradients are held to the same tolerance as the conditioned test."""
    torch.set_num_threads(8)
    cs = case(ns=2)
    caps = capture_saves(monkeypatch)
    loss, got = hip_grads(cs, precision)
    stats = dict(band=0, adopted=0, outside=0)
    relus = margin_relu(caps, cs["rays"].shape[0], 1e-4, stats)

    sd = dict(cs["sd"])
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items() if k.startswith("mlp_")}
    sd.update(params)
    latent = cs["latent"].clone().requires_grad_(True)
    scene = ref_cpu.Scene(latent, cs["poses"], cs["focal"], cs["width"], cs["height"], cs["c"])

    def model_fn(pts, coarse, dirs):
        return ref_cpu.pixelnerf_forward(sd, scene, pts, coarse, dirs, relu=relus[bool(coarse)])

    out = ref_cpu.render(model_fn, cs["rays"], cs["kc"], cs["kf"], cs["kfd"], cs["streams"], True,
                         depth_std=0.05)
    mse = torch.nn.functional.mse_loss
    ref_loss = mse(out["coarse"]["rgb"], cs["target"]) + mse(out["fine"]["rgb"], cs["target"])
    ref_loss.backward()
    ref = {k: p.grad for k, p in params.items()}
    ref["latent"] = latent.grad
    print("relu margin band %(band)d units, HIP decision adopted for %(adopted)d, "
          "masks differing outside the band %(outside)d" % stats)
    assert stats["outside"] == 0, stats
    assert abs(loss - ref_loss.item()) <= 1e-5 * abs(ref_loss.item()), (loss, ref_loss.item())
    assert set(ref) == set(got), set(ref) ^ set(got)
    for k in sorted(ref):
        a, b = got[k].reshape(-1).double(), ref[k].reshape(-1).double()
        scale = float(b.abs().max())
        err = float((a - b).abs().max())
        assert err <= tol * scale + 1e-9, "%s: max |d| %.3g vs max |ref| %.3g" % (k, err, scale)


def test_training_noise_std_draw_order_matches_reference():
    """noise_std > 0 in training mode (nerf.py:225-226): sigma noise per pass, with the
    reference's draw order u_coarse, coarse noise, u_fine, u_fine_jit, n_depth, fine noise."""
    cs = case(sb=1, rays_per_obj=4, kc=8, kf=6, kfd=2)
    net = PixelNeRFNet(conf())
    net.load_state_dict(cs["sd"], strict=False)
    net = net.to(DEV)
    lat = cs["latent"][:1].to(DEV).requires_grad_(True)
    net.encode_latent(lat, cs["poses"][:1].to(DEV), cs["focal"][:1].to(DEV), (cs["width"], cs["height"]),
                      c=cs["c"][:1].to(DEV), num_objs=1)
    r = NeRFRenderer(n_coarse=8, n_fine=6, n_fine_depth=2, noise_std=0.5, white_bkgd=True).to(DEV).train()
    log = []
    rand, randn = torch.rand, torch.randn

    def lrand(*s, **k):
        log.append(("rand", tuple(s[0]) if isinstance(s[0], (tuple, list)) else tuple(s)))
        return rand(*s, **k)

    def lrandn(*s, **k):
        log.append(("randn", tuple(s[0]) if isinstance(s[0], (tuple, list)) else tuple(s)))
        return randn(*s, **k)

    torch.rand, torch.randn = lrand, lrandn
    try:
        out = r(net, cs["rays"][:1].to(DEV), want_weights=True)
    finally:
        torch.rand, torch.randn = rand, randn
    B = 4
    assert log == [("rand", (B, 8)), ("randn", (B, 8)), ("rand", (B, 4)), ("rand", (B, 4)),
                   ("randn", (B, 2)), ("randn", (B, 14))], log
    loss = out.fine.rgb.sum() + out.coarse.rgb.sum()
    loss.backward()
    assert torch.isfinite(lat.grad).all()


@pytest.mark.parametrize("rays_per_obj,K,ns,comb", [(96, 41, 1, 3), (256, 64, 1, 3), (40, 41, 3, 3), (256, 64, 2, 3),
                                                     (40, 41, 3, 2)])
def test_fused_mlp_backward_matches_torch_backward(rays_per_obj, K, ns, comb):
    """pnr_mlp_backward_views (the f16x3 W^T chain: masks, residuals, lin_z latent gradient,
    bias column sums, the view mean's backward) plus the batched weight GEMMs against the
    per-layer fp32 torch backward (train.mlp_backward) on the same activation save: 7,872
    points (ragged last tile, one tile per workgroup), 32,768 (several tiles per workgroup: the
    bias partials add up across tiles), and NS = 3 / 2 source views per point (the DTU
    setting: per-view rows before combine_layer), per-point gradient magnitudes spread over
    2^-20 .. 1; combine_layer 2 as well as the default 3.  Tolerance 2e-5 of each tensor's
    max-abs."""
    from types import SimpleNamespace

    from pnr import train

    cs = case(sb=2, rays_per_obj=rays_per_obj, kc=K, ns=ns, combine_layer=comb)
    net = PixelNeRFNet(conf(comb))
    net.load_state_dict(cs["sd"], strict=False)
    net = net.to(DEV)
    net.mlp_precision = "f16x3"
    net.encode_latent(cs["latent"].to(DEV), cs["poses"].to(DEV), cs["focal"].to(DEV),
                      (cs["width"], cs["height"]), c=cs["c"].to(DEV), num_objs=cs["poses"].shape[0])
    rays = cs["rays"].to(DEV).reshape(-1, 8).contiguous()
    t = torch.linspace(0.0, 1.0, K, device=DEV)
    z = (rays[:, 6:7] + (rays[:, 7:8] - rays[:, 6:7]) * t).contiguous()
    ctx = SimpleNamespace()
    ctx.save_for_backward = lambda *ts: setattr(ctx, "saved", ts)
    params = train.mlp_params(net.mlp_coarse)
    with torch.no_grad():
        train.RenderPoints.forward(ctx, net, True, rays, z, net.encoder.latent_cl, *params)
    save = ctx.saved[3]
    P = rays.shape[0] * K
    gen = torch.Generator(device="cpu").manual_seed(7)
    d_o = torch.randn(P, 4, generator=gen) * torch.exp2(-20.0 * torch.rand(P, 1, generator=gen))
    d_o = d_o.to(DEV)
    with torch.no_grad():
        assert net.num_views_per_obj == ns
        g_ref, df_ref, dz_ref = train.mlp_backward(net.mlp_coarse, save, d_o, P, ns)
        g, df, dz = train.mlp_backward_fused(net.mlp_coarse, net.code, "f16x3", save, d_o, P, ns)
    worst = 0.0
    pairs = [(g[p], g_ref[p]) for p in g_ref] + [(df, df_ref), (dz, dz_ref)]
    for a, b in pairs:
        err = ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()
        worst = max(worst, err)
        assert err < 2e-5, err
    assert len(g) == len(g_ref) == len(params)
    print("fused MLP backward: worst relative error %.2e" % worst)


@pytest.mark.parametrize("arith", ["f16x3", "bf16x6"])
@pytest.mark.parametrize("P", [1, 33, 4133, 70000])
def test_weight_grad_matches_fp64(P, arith):
    """pnr_weight_grad (f16x3 on MFMA with running per-(chunk, channel) power-of-two scales,
    point-chunk partials + fixed-order reduce) against an fp64 GEMM: 3 layers, ragged point
    counts, magnitudes spread over 2^-30 .. 2^10 per row.  Tolerance 4e-6 of each result's
    max-abs (fp32 accumulation over up to 70k points)."""
    from pnr import train

    gen = torch.Generator(device="cpu").manual_seed(P)
    dys, xs = [], []
    for j in range(3):
        d = torch.randn(P, 512, generator=gen) * torch.exp2(-30 + 40 * torch.rand(P, 1, generator=gen))
        x = torch.relu(torch.randn(P, 512, generator=gen)) * torch.exp2(-8 * torch.rand(1, 512, generator=gen))
        dys.append(d.to(DEV))
        xs.append(x.to(DEV))
    g = train.weight_grad(dys, xs, P, arith)
    for j in range(3):
        ref = dys[j].double().t() @ xs[j].double()
        err = ((g[j].double() - ref).abs().max() / ref.abs().max()).item()
        print("weight_grad %s P=%d layer %d: relative error %.2e" % (arith, P, j, err))
        assert err < 4e-6, (j, err)
    # deterministic: same bits on a second call
    assert torch.equal(train.weight_grad(dys, xs, P, arith), g)


@pytest.mark.parametrize("case", ["growing", "late_channels", "huge_tiny", "zeros", "rays"])
def test_weight_grad_scale_moves(case):
    """The f16x3 weight gradient's running channel scales (csrc/wgrad.hip k_wgrad_h): data whose
    channel maxima grow along the points (every chunk moves its scales many times: rows ramp from
    2^-20 to 2^20), channels that stay zero for the first half of the points and then turn on,
    channel blocks 2^80 / 2^-60 apart (products from 2^117 down to 2^-113), and all-zero inputs.  Against an fp64 GEMM,
    4e-6 of each result's max-abs, and deterministic."""
    from pnr import train

    P = 9000
    gen = torch.Generator(device="cpu").manual_seed(7)
    d = torch.randn(P, 512, generator=gen)
    x = torch.relu(torch.randn(P, 512, generator=gen))
    if case == "growing":
        ramp = torch.exp2(torch.linspace(-20, 20, P)).unsqueeze(1)
        d = d * ramp
        x = x * ramp.flip(0).sqrt()
    elif case == "late_channels":
        d[: P // 2, ::3] = 0.0
        x[: P // 2, 1::2] = 0.0
        x[P // 2:, 1::2] *= 1e4
    elif case == "rays":
        # a training step's shape: per-point gradient magnitudes spread over 2^-30 .. 1 (the
        # transmittance along each 64-sample ray), sparse relu activations, channels that turn on
        k = torch.arange(P)
        u = torch.rand(P // 64 + 1, generator=gen)
        d = d * torch.exp2(-30.0 * u[k // 64] * (k % 64).float() / 63.0).unsqueeze(1)
        x = torch.relu(torch.randn(P, 512, generator=gen) - 1.5)
        x[: P // 3, 5::7] = 0.0
    elif case == "huge_tiny":
        d[:, :64] *= 2.0 ** 80
        d[:, 64:128] *= 2.0 ** -60
        x[:, :32] *= 2.0 ** -60
        x[:, 32:64] *= 2.0 ** 20
    else:
        d.zero_()
        x.zero_()
    dd, xd = d.to(DEV), x.to(DEV)
    g = train.weight_grad([dd], [xd], P)[0]
    ref = d.double().t() @ x.double()
    if case == "zeros":
        assert torch.equal(g.cpu(), torch.zeros(512, 512))
        return
    assert torch.isfinite(g).all()
    if case == "huge_tiny":
        # per block: the blocks' magnitudes differ by up to 2^230
        for rs in (slice(0, 64), slice(64, 128), slice(128, 512)):
            for cs in (slice(0, 32), slice(32, 64), slice(64, 512)):
                r = ref[rs, cs]
                err = ((g.double().cpu()[rs, cs] - r).abs().max() / r.abs().max()).item()
                assert err < 4e-6, (rs, cs, err)
    else:
        err = ((g.double().cpu() - ref).abs().max() / ref.abs().max()).item()
        print("weight_grad %s: relative error %.2e" % (case, err))
        assert err < 4e-6, err
    if case == "rays":
        # elementwise, against the fp32 GEMM error scale sum_p |dY_pi| |X_pj|
        scale = d.double().abs().t() @ x.double().abs()
        ew = ((g.double().cpu() - ref).abs() / scale.clamp_min(1e-300)).max().item()
        print("weight_grad rays: max |err| / sum |terms| %.2e" % ew)
        assert ew < 2.0 ** -17, ew
    assert torch.equal(train.weight_grad([dd], [xd], P)[0], g)


@pytest.mark.parametrize("arith", ["f16x3", "bf16x6"])
def test_weight_grad_wide_dynamic_range(arith):
    """an output element built ONLY from values far below their channel's
    maximum.  dY rows of the "far" points are scaled by 2^-15 .. 2^-25 (per point); X channels
    j = 0 mod 4 are nonzero only on those far points, so G_ij for those j has no term from a
    large dY.  bf16x6 (PNR_WGRAD_BF16X6) must hold every element to the fp32 GEMM error scale
    sum_p |dY_pi||X_pj|; f16x3 (the default) is held to the bound include/pnr_abi.h states: that
    scale plus ~2^-30 of the channel maxima times the other operand's column sums."""
    from pnr import train

    P = 9000
    gen = torch.Generator(device="cpu").manual_seed(21)
    d = torch.randn(P, 512, generator=gen)
    x = torch.relu(torch.randn(P, 512, generator=gen)) + 0.1
    far = torch.rand(P, generator=gen) < 0.5
    d[far] *= torch.exp2(-15.0 - 10.0 * torch.rand(int(far.sum()), 1, generator=gen))
    x[~far, 0::4] = 0.0
    g = train.weight_grad([d.to(DEV)], [x.to(DEV)], P, arith)[0].double().cpu()
    ref = d.double().t() @ x.double()
    scale = d.double().abs().t() @ x.double().abs()
    rel = ((g - ref).abs() / scale.clamp_min(1e-300))
    worst_far = rel[:, 0::4].max().item()
    worst_near = torch.cat([rel[:, 1::4], rel[:, 2::4], rel[:, 3::4]], 1).max().item()
    print("weight_grad %s wide range: max |err| / sum |terms|: far-only columns %.2e, others %.2e" % (
        arith, worst_far, worst_near))
    assert worst_near < 2.0 ** -17, worst_near
    if arith == "bf16x6":
        assert worst_far < 2.0 ** -17, worst_far
    else:
        mi = d.double().abs().max(0).values.unsqueeze(1)          # channel maxima (>= the chunk maxima)
        mj = x.double().abs().max(0).values.unsqueeze(0)
        bound = 2.0 ** -17 * scale + 2.0 ** -28 * (mi * x.double().abs().sum(0).unsqueeze(0)
                                                   + mj * d.double().abs().sum(0).unsqueeze(1))
        assert bool(((g - ref).abs() <= bound).all()), float(((g - ref).abs() / bound).max())
    assert torch.equal(train.weight_grad([d.to(DEV)], [x.to(DEV)], P, arith)[0].double().cpu(), g)


def test_weight_grad_arith_selects_kernel():
    """pnr_weight_grad_arith: both arithmetics agree to the fp32 level on ordinary data, and an
    unknown arithmetic is refused before any device work."""
    from pnr import train

    P = 2048
    gen = torch.Generator(device="cpu").manual_seed(3)
    d = torch.randn(P, 512, generator=gen).to(DEV)
    x = torch.relu(torch.randn(P, 512, generator=gen)).to(DEV)
    a = train.weight_grad([d], [x], P, "f16x3")[0]
    b = train.weight_grad([d], [x], P, "bf16x6")[0]
    assert ((a - b).abs().max() / b.abs().max()).item() < 4e-6
    from pnr import _lib

    lib = _lib.load()
    import ctypes

    arr = (ctypes.c_void_p * 1)(d.data_ptr())
    rc = lib.pnr_weight_grad_arith(arr, arr, arr, 1, P, 7, None, 0, None)
    assert rc == -1 and b"arithmetic" in lib.pnr_last_error()


@pytest.mark.parametrize("coarse", [True, False])
@pytest.mark.parametrize("precision", ["fp32", "f16x3"])
def test_grad_point_query_matches_oracle_autograd(precision, coarse):
    """The reference's callers query the net WITHOUT torch.no_grad() (eval/eval.py:100, the density
    grid; train/train.py:422): the output carries the autograd graph.  Here that query runs the
    training forward (PixelNeRFNet._forward_points_grad -> train.RenderPoints at z = 0); its values
    and its gradients (MLP parameters and latent, SB = 2 objects) against the oracle's autograd, at
    the training tests' tolerance, on `conditioned` weights (no ReLU within rounding of its kink:
    on the raw hash weights the f16x3 forward flips a few units the fp32 oracle does not, and each
    flip moves the latent gradient below it by ~1e-3 of its range, as the training tests found)."""
    cs = case(sb=2, rays_per_obj=8, seed=7)
    cs["sd"] = conditioned(cs["sd"])
    xyz = torch.from_numpy(synth.hash_sym(81, (2, 300, 3), 0.5))
    vd = torch.nn.functional.normalize(torch.from_numpy(synth.hash_sym(82, (2, 300, 3), 1.0)), dim=-1)
    wt = torch.from_numpy(synth.hash_sym(83, (2, 300, 4), 1.0))
    sd = dict(cs["sd"])
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items() if k.startswith("mlp_")}
    sd.update(params)
    latent = cs["latent"].clone().requires_grad_(True)
    scene = ref_cpu.Scene(latent, cs["poses"][:, None], cs["focal"], cs["width"], cs["height"], cs["c"])
    ref = ref_cpu.pixelnerf_forward(sd, scene, xyz, coarse, vd)
    (ref * wt).sum().backward()
    net = PixelNeRFNet(conf())
    net.load_state_dict(cs["sd"], strict=False)
    net = net.to(DEV)
    net.mlp_precision = precision
    lat_d = cs["latent"].to(DEV).requires_grad_(True)
    net.encode_latent(lat_d, cs["poses"].to(DEV), cs["focal"].to(DEV), (cs["width"], cs["height"]),
                      c=cs["c"].to(DEV), num_objs=2)
    out = net(xyz.to(DEV), coarse=coarse, viewdirs=vd.to(DEV))
    assert out.requires_grad and out.grad_fn is not None
    d = (out.detach().cpu() - ref.detach()).abs()
    assert bool((d <= 5e-5 + 1e-5 * ref.detach().abs()).all()), float(d.max())
    (out * wt.to(DEV)).sum().backward()
    tol = 1e-4 if precision == "fp32" else 2e-4
    used = "mlp_coarse." if (coarse or net.mlp_fine is None) else "mlp_fine."
    got = {k: p.grad.detach().cpu() for k, p in net.named_parameters() if k.startswith(used)}
    exp = {k: p.grad for k, p in params.items() if k.startswith(used)}
    got["latent"], exp["latent"] = lat_d.grad.detach().cpu(), latent.grad
    assert set(got) == set(exp), set(got) ^ set(exp)
    for k in sorted(exp):
        a, b = got[k].reshape(-1).double(), exp[k].reshape(-1).double()
        scale = float(b.abs().max())
        assert float((a - b).abs().max()) <= tol * scale + 1e-9, k
