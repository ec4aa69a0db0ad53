"""Training path: autograd over the HIP ray march (BASELINE cfg5).

The reference trains by running torch autograd through ``NeRFRenderer.forward``
(nerf.py:251-303) and ``PixelNeRFNet.forward`` (models.py:146-266); the training step is
train.py:182-283.  Here the same graph is built from HIP kernels:

* ``RenderPoints``: the model at the points ``o + z d`` of every ray.
  * **Forward** (``pnr_render_points``): the fused kernel, which saves the activations
    the backward needs: features, the sampled latent z, and relu(x) / relu(h) per block.
  * **Backward:**
    * the sigmoid / relu head;
    * ResnetFC as per-layer plain GEMMs on the saved activations (fp32 hipBLASLt via
      ``torch.mm``);
    * ``pnr_points_input_backward`` for the input stage: the bilinear scatter into the
      channels-last latent (grid_sample backward), and dL/dz of every sample through the
      PE and the projection.
* ``Composite``: ``pnr_composite`` forward and ``pnr_composite_backward``.

The renderer wires them as the reference's autograd graph does:
* the importance samples use the detached coarse weights (nerf.py:130);
* the depth samples keep their gradient to the coarse depth (nerf.py:150-161, 292);
* the fine depths are sorted with ``torch.sort`` (nerf.py:295), so the gradient follows
  the permutation.

Several source views per object (train.py -V, the DTU setting) are supported: the
activation save holds one row per (view, point) for the stages before combine_layer, the
backward sends dL/d(view mean) / NS to every view there (util.combine_interleaved,
util.py:461-471) and the input-stage backward scatters into each view's latent.  The fused
f16x3 backward chain (``pnr_mlp_backward_views``) covers any number of views; the fp32 / bf16
arithmetics run the ResnetFC backward as per-layer GEMMs (``mlp_backward``).
"""
import torch

from . import _lib, ops

__all__ = ["RenderPoints", "Composite", "mlp_backward", "mlp_backward_fused", "weight_grad", "mlp_params"]

# Measurement hook (bench.py train leg): None, or {kernel: [(start, end, flop)]} -- HIP events
# recorded on the launch stream around the training MLP kernels (torch's current stream, the one
# every ctypes launch here uses) with each launch's algorithmic FLOP.  No host synchronization.
KERNEL_EVENTS = None


def _ev_begin():
    if KERNEL_EVENTS is None:
        return None
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


def _ev_end(name, e0, flop):
    if e0 is not None:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        KERNEL_EVENTS.setdefault(name, []).append((e0, e1, float(flop)))


def mlp_params(mlp):
    """The ResnetFC parameters in registration order (what autograd tracks), also on an
    nn.DataParallel replica (bind_parallel, nerf.py:354-371)."""
    from .models import module_params

    return module_params(mlp)


def _on_device(dev, what, *tensors):
    """Every tensor handed to a training kernel by pointer must live on the launch device
    (the torch ops check this in C++, torch_ops.cpp; the ctypes calls check it here)."""
    for name, t in zip(what.split(), tensors):
        if t is not None and t.device != dev:
            raise ValueError("pnr: %s is on %s, the launch device is %s" % (name, t.device, dev))


def forward_flop(mlp, P, ns=1):
    """Algorithmic FLOP of the ResnetFC forward over P points with ns source views (the reference's
    per-point arithmetic, resnetfc.py:132-184: lin_in, lin_z and both block layers before
    combine_layer once per view, the rest once per point, lin_out)."""
    nb = mlp.n_blocks
    nc = min(mlp.combine_layer, nb) if ns > 1 else nb
    nz = len(getattr(mlp, "lin_z", []))
    H, d_in = 512, mlp.lin_in.weight.shape[1]
    per_view = 2 * H * d_in + 2 * H * H * (nz + 2 * nc)
    per_point = 2 * H * H * 2 * (nb - nc) + 2 * 4 * H
    return float(P) * (ns * per_view + per_point)


def backward_chain_flop(mlp, P, ns=1):
    """Algorithmic FLOP of k_mlp_bwd's input-gradient chain: W^T dY of every 512-wide layer (the
    blocks before combine_layer once per view) and d_o W_out; lin_in's d_feat is a torch GEMM."""
    nb = mlp.n_blocks
    nc = min(mlp.combine_layer, nb) if ns > 1 else nb
    nz = len(getattr(mlp, "lin_z", []))
    H = 512
    return float(P) * (ns * 2 * H * H * (nz + 2 * nc) + 2 * H * H * 2 * (nb - nc) + 2 * 4 * H)


def _save_views(save, P, n_blocks, H=512, ns=1):
    """Slices of the pnr_render_points activation save (include/pnr_abi.h): every region
    has R = ns * P rows, row v P + p = (view v, point p); ``slot(i, rows)`` takes the first
    ``rows`` rows of relu region i (P for the per-point stages after combine_layer)."""
    R = ns * P
    feat = save[: R * 64].view(R, 64)
    base = R * 64
    z = save[base: base + R * H].view(R, H)

    def slot(i, rows=R):
        o = base + R * H * (1 + i)
        return save[o: o + rows * H].view(rows, H)

    return feat, z, slot


def mlp_backward(mlp, save, d_o, P, ns=1, use_wgrad=False):
    """ResnetFC backward (resnetfc.py:132-184) given dL/d(pre-head output) ``d_o`` (P, 4),
    for ``ns`` source views per point.  Returns ({param: grad}, d_feat (ns P, 64),
    d_zlat (ns P, 512) or None), rows view-major like the activation save.
    The 512-wide GEMMs are fp32 hipBLASLt GEMMs (split-fp16 GEMMs assembled from torch
    ops measured 2x slower end to end: the split / scale passes cost more than they save);
    with ``use_wgrad`` the 512 x 512 weight gradients are ``pnr_weight_grad`` launches
    instead (one per row count: ns P rows before combine_layer, P after)."""
    mm = torch.mm
    jobs = {}   # rows -> [(param, dY, X)] for pnr_weight_grad

    def wgrad(param, dy, x):
        if use_wgrad:
            jobs.setdefault(dy.shape[0], []).append((param, dy, x))
        else:
            g[param] = mm(dy.t(), x)

    nb = mlp.n_blocks
    nc = min(mlp.combine_layer, nb) if ns > 1 else nb
    lin_z = list(getattr(mlp, "lin_z", []))
    feat, z, slot = _save_views(save, P, nb, ns=ns)
    g = {}
    xf = slot(2 * nb, P)
    W = mlp.lin_out.weight.detach()
    g[mlp.lin_out.weight] = d_o.t() @ xf
    g[mlp.lin_out.bias] = d_o.sum(0)
    dx = (d_o @ W) * (xf > 0)
    dz = None
    for b in reversed(range(nb)):
        blk = mlp.blocks[b]
        rows = ns * P if b < nc else P
        hb, xb = slot(nb + b, rows), slot(b, rows)
        w1, w0 = blk.fc_1.weight.detach(), blk.fc_0.weight.detach()
        wgrad(blk.fc_1.weight, dx, hb)
        g[blk.fc_1.bias] = dx.sum(0)
        dh = mm(dx, w1) * (hb > 0)
        wgrad(blk.fc_0.weight, dh, xb)
        g[blk.fc_0.bias] = dh.sum(0)
        dx = dx + mm(dh, w0) * (xb > 0)
        if b < len(lin_z):
            lz = lin_z[b]
            wgrad(lz.weight, dx, z)
            g[lz.bias] = dx.sum(0)
            t = mm(dx, lz.weight.detach())
            dz = t if dz is None else dz + t
        if b == nc and ns > 1:
            # x = mean over views at the start of block nc (combine_interleaved): every view's
            # row gets dL/d(mean) / ns, rows view-major
            dx = (dx / ns).repeat(ns, 1)
    d_in = mlp.lin_in.weight.shape[1]
    g[mlp.lin_in.weight] = _tall_mm(dx, feat)[:, :d_in]
    g[mlp.lin_in.bias] = dx.sum(0)
    d_feat = torch.zeros(ns * P, 64, device=dx.device, dtype=torch.float32)
    d_feat[:, :d_in] = dx @ mlp.lin_in.weight.detach()
    for rows, js in jobs.items():
        for i in range(0, len(js), 16):   # pnr_weight_grad: up to 16 layers per launch
            part = js[i:i + 16]
            gw = weight_grad([dy.contiguous() for _, dy, _ in part], [x for _, _, x in part], rows)
            for j, (param, _, _) in enumerate(part):
                g[param] = gw[j]
    return g, d_feat, dz


def weight_grad(dys, xs, P, arith="f16x3"):
    """``pnr_weight_grad_arith``: G[j] = dys[j]^T xs[j] (512 x 512) for (P, 512) fp32 matrices,
    in one launch, deterministic.  ``arith`` "f16x3" (default; csrc/wgrad.hip k_wgrad_h): fp16
    split products with running per-(chunk, channel) scales, fp32-level error relative to the
    channel scale (include/pnr_abi.h states the bound); "bf16x6" (k_wgrad): split-bf16 products,
    fp32-level error per element whatever the dynamic range."""
    import ctypes

    n = len(dys)
    dev = dys[0].device
    out = torch.empty(n, 512, 512, dtype=torch.float32, device=dev)
    lib = _lib.load()
    wsb = lib.pnr_weight_grad_workspace_bytes(n, P)
    if wsb == 0 and P > 0:
        _lib.check(-1, "pnr_weight_grad_workspace_bytes")
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)

    def arr(ts):
        for t in ts:
            assert t.is_contiguous() and t.shape == (P, 512) and t.dtype == torch.float32 and t.device == dev
        return (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])

    outs = (ctypes.c_void_p * n)(*[out[i].data_ptr() for i in range(n)])
    e0 = _ev_begin()
    _lib.check(lib.pnr_weight_grad_arith(arr(dys), arr(xs), outs, n, P, _lib.WGRAD_ARITH[arith], _lib.ptr(ws),
                                         wsb, _lib.stream_of(dev)), "pnr_weight_grad_arith")
    _ev_end("weight_grad", e0, 2.0 * 512 * 512 * n * P)
    return out


def _split(P, max_split=64):
    """Largest power-of-two split (<= max_split) of a point count P."""
    s = 1
    while s < max_split and P % (2 * s) == 0:
        s *= 2
    return s


def _tall_mm(a, b):
    """a^T b for tall a (P, m), b (P, n) with small m, n: split-K over the points as a batched
    GEMM plus one sum (hipBLASLt runs the plain (m x P)(P x n) product at a few TFLOP/s: its
    K = P reduction is not split; measured 4x faster, scripts/microbench_train_reductions.py)."""
    P = a.shape[0]
    s = _split(P)
    if s == 1:
        return a.t() @ b
    return (a.view(s, P // s, a.shape[1]).transpose(1, 2) @ b.view(s, P // s, b.shape[1])).sum(0)


def mlp_backward_fused(mlp, code, precision, save, d_o, P, ns=1, wgrad_arith="f16x3"):
    """``mlp_backward`` for f16x3 models: the input-gradient chain (masks, residual adds,
    every 512-wide W^T GEMM, the summed latent gradient, the view mean's backward for ``ns``
    source views) runs in one ``pnr_mlp_backward_views`` launch on the forward's split-fp16
    GEMM, which also sums every layer's output gradient over its rows (the bias gradients,
    without re-reading dy); the 512-wide weight gradients are ``pnr_weight_grad`` launches
    (fp16 split products, fp32-level), one per row count (ns P view rows before combine_layer, P
    after), over its per-layer output gradients and the activation save."""
    desc, packed, packed_t = mlp.packed_t(code, precision)
    nb = mlp.n_blocks
    nc = min(mlp.combine_layer, nb) if ns > 1 else nb
    lin_z = list(getattr(mlp, "lin_z", []))
    R = ns * P
    feat, z, slot = _save_views(save, P, nb, ns=ns)
    dev = d_o.device
    _on_device(dev, "packed packed_t save", packed, packed_t, save)
    d_o = d_o.contiguous()
    dy = torch.empty(2 * nb + 1, R, 512, dtype=torch.float32, device=dev)
    dzl = torch.empty(R, 512, dtype=torch.float32, device=dev) if lin_z else None
    w_out = mlp.lin_out.weight.detach().float().contiguous()
    sums = torch.empty(2 * nb + 1, 512, dtype=torch.float32, device=dev)   # bias gradients, dy's slot order
    lib = _lib.load()
    wsb = lib.pnr_mlp_backward_workspace_bytes(desc, P)
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
    e0 = _ev_begin()
    _lib.check(lib.pnr_mlp_backward_views(desc, _lib.ptr(packed), _lib.ptr(packed_t), _lib.ptr(w_out),
                                          _lib.ptr(save), _lib.ptr(d_o), P, ns, _lib.ptr(dy), _lib.ptr(dzl),
                                          _lib.ptr(sums), _lib.ptr(ws), wsb, _lib.stream_of(dev)),
               "pnr_mlp_backward_views")
    _ev_end("mlp_backward", e0, backward_chain_flop(mlp, P, ns))
    g = {}
    xf = slot(2 * nb, P)
    g[mlp.lin_out.weight] = _tall_mm(d_o, xf)
    g[mlp.lin_out.bias] = d_o.sum(0)
    # weight gradients grouped by row count: fc_0 (dY^T relu(x_b)), fc_1 (dY^T relu(h_b)),
    # lin_z (dY^T z)
    jobs = {}
    for b, blk in enumerate(mlp.blocks):
        rows = R if b < nc else P
        jobs.setdefault(rows, []).extend([(blk.fc_0.weight, dy[b, :rows], slot(b, rows)),
                                          (blk.fc_1.weight, dy[nb + 1 + b, :rows], slot(nb + b, rows))])
    for b, lz in enumerate(lin_z):
        rows = R if b < nc else P
        jobs.setdefault(rows, []).append((lz.weight, dy[nb + b, :rows], z[:rows]))
    for rows, js in jobs.items():
        for i in range(0, len(js), 16):   # pnr_weight_grad: up to 16 layers per launch
            part = js[i:i + 16]
            gw = weight_grad([d for _, d, _ in part], [x for _, _, x in part], rows, wgrad_arith)
            for j, (param, _, _) in enumerate(part):
                g[param] = gw[j]
    for b, blk in enumerate(mlp.blocks):
        g[blk.fc_0.bias] = sums[b]
        g[blk.fc_1.bias] = sums[nb + 1 + b]
    for b, lz in enumerate(lin_z):
        g[lz.bias] = sums[nb + b]
    dx = dy[nb]
    d_in = mlp.lin_in.weight.shape[1]
    g[mlp.lin_in.weight] = _tall_mm(dx, feat)[:, :d_in]
    g[mlp.lin_in.bias] = sums[nb]
    d_feat = torch.zeros(R, 64, device=dev, dtype=torch.float32)
    d_feat[:, :d_in] = dx @ mlp.lin_in.weight.detach()
    return g, d_feat, dzl


class FinePass:
    """The ``coarse`` argument of RenderPoints for a fine pass (false) carrying ``z_mask`` (n_rays,
    k) bool: the points whose dL/dz reaches the graph -- the depth samples of the sorted
    [importance, depth] fine depths (nerf.py:150-161, 292); the input backward computes the depth
    chain only there (``pnr_points_input_backward_masked``)."""

    def __init__(self, z_mask=None):
        self.z_mask = z_mask

    def __bool__(self):
        return False


class RenderPoints(torch.autograd.Function):
    """raw (B, K, 4) = PixelNeRFNet at o + z d (models.py:146-266, via nerf.py:182-216),
    differentiable in z, the encoder latent (channels-last) and the MLP parameters."""

    @staticmethod
    def forward(ctx, net, coarse, rays, z, latent_cl, *params):
        mlp = net.mlp_coarse if (coarse or net.mlp_fine is None) else net.mlp_fine
        desc, packed = mlp.packed(net.code, net.mlp_precision)
        sc = net.hip_scene()
        B, K = z.shape
        P = B * K
        lib = _lib.load()
        dev = z.device
        _on_device(dev, "packed rays latent cams", packed, rays, net.encoder.latent_cl, net.cams)
        ns = net.num_views_per_obj
        save = None
        # no activation save without a backward (no_grad); callers driving forward() by hand
        # (tests) pass a plain namespace and always get the save
        if any(getattr(ctx, "needs_input_grad", (True,))):
            n_save = lib.pnr_point_save_floats(desc, P * ns)
            if n_save == 0:
                _lib.check(-1, "pnr_point_save_floats")
            save = torch.empty(n_save, dtype=torch.float32, device=dev)
        ws_bytes = lib.pnr_point_query_workspace_bytes(sc, P)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        out = torch.empty(P, 4, dtype=torch.float32, device=dev)
        r = _lib.Rays(_lib.ptr(rays), B, B // net.num_objs)
        e0 = _ev_begin()
        _lib.check(lib.pnr_render_points(sc, desc, _lib.ptr(packed), r, _lib.ptr(z), K, _lib.ptr(out),
                                         _lib.ptr(save), _lib.ptr(ws), ws_bytes, _lib.stream_of(dev)),
                   "pnr_render_points")
        _ev_end("forward", e0, forward_flop(mlp, P, ns))
        ctx.save_for_backward(rays, z, out, save, latent_cl)
        ctx.net, ctx.mlp, ctx.desc, ctx.packed, ctx.params = net, mlp, desc, packed, params
        ctx.z_mask = getattr(coarse, "z_mask", None)
        return out.view(B, K, 4)

    @staticmethod
    def backward(ctx, d_out):
        rays, z, out, save, latent_cl = ctx.saved_tensors
        net, mlp = ctx.net, ctx.mlp
        B, K = z.shape
        P = B * K
        d_out = d_out.reshape(P, 4).float()
        # head: [sigmoid(rgb), relu(sigma)] (models.py:258-265)
        d_o = torch.cat([d_out[:, :3] * out[:, :3] * (1.0 - out[:, :3]),
                         d_out[:, 3:] * (out[:, 3:] > 0)], dim=1)
        ns = net.num_views_per_obj
        if net.mlp_precision == "f16x3":
            g, d_feat, d_zlat = mlp_backward_fused(mlp, net.code, net.mlp_precision, save, d_o, P, ns,
                                                   getattr(net, "wgrad_arith", "f16x3"))
        else:
            g, d_feat, d_zlat = mlp_backward(mlp, save, d_o, P, ns, use_wgrad=net.mlp_precision == "f16x3")
        need_z, need_lat = ctx.needs_input_grad[3], ctx.needs_input_grad[4]
        d_z = torch.empty(P, dtype=torch.float32, device=z.device) if need_z else None
        d_lat = torch.zeros_like(latent_cl) if need_lat else None
        if need_z or need_lat:
            if d_zlat is None:
                d_zlat = torch.zeros(ns * P, 512, dtype=torch.float32, device=z.device)
            lib = _lib.load()
            _on_device(z.device, "packed rays d_feat d_zlat d_latent cams latent", ctx.packed, rays, d_feat,
                       d_zlat, d_lat, net.cams, net.encoder.latent_cl)
            r = _lib.Rays(_lib.ptr(rays), B, B // net.num_objs)
            zm = getattr(ctx, "z_mask", None)
            if zm is not None:
                zm = zm.reshape(P).to(device=z.device, dtype=torch.uint8).contiguous()
            _lib.check(lib.pnr_points_input_backward_masked(
                net.hip_scene(), ctx.desc, _lib.ptr(ctx.packed), r, _lib.ptr(z), K, _lib.ptr(d_feat.contiguous()),
                _lib.ptr(d_zlat.contiguous()), _lib.ptr(d_lat), _lib.ptr(d_z), _lib.ptr(zm) if need_z else None,
                _lib.stream_of(z.device)), "pnr_points_input_backward_masked")
        grads = [g.get(p) for p in ctx.params]
        return (None, None, None, d_z.view(B, K) if need_z else None, d_lat, *grads)


class Composite(torch.autograd.Function):
    """(weights, rgb, depth) of NeRFRenderer.composite (nerf.py:225-247) with its backward."""

    @staticmethod
    def forward(ctx, z, raw, rays, white_bkgd):
        w, rgb, depth = ops.composite(z, raw, rays, white_bkgd, want_weights=True)
        ctx.save_for_backward(z, raw, rays)
        ctx.white_bkgd = white_bkgd
        return w, rgb, depth

    @staticmethod
    def backward(ctx, d_w, d_rgb, d_depth):
        z, raw, rays = ctx.saved_tensors
        B, K = z.shape
        if d_rgb is None:
            d_rgb = torch.zeros(B, 3, dtype=torch.float32, device=z.device)
        d_raw = torch.empty(B, K, 4, dtype=torch.float32, device=z.device)
        d_z = torch.empty(B, K, dtype=torch.float32, device=z.device) if ctx.needs_input_grad[0] else None
        _on_device(z.device, "raw rays d_rgb d_depth d_weights", raw, rays, d_rgb, d_depth, d_w)
        lib = _lib.load()
        _lib.check(lib.pnr_composite_backward(
            _lib.ptr(z), _lib.ptr(raw), _lib.ptr(rays), B, K, int(bool(ctx.white_bkgd)),
            _lib.ptr(d_rgb.contiguous()), _lib.ptr(d_depth.contiguous() if d_depth is not None else None),
            _lib.ptr(d_w.contiguous() if d_w is not None else None), _lib.ptr(d_raw), _lib.ptr(d_z),
            _lib.stream_of(z.device)), "pnr_composite_backward")
        return d_z, d_raw, None, None
