"""NeRFRenderer with the reference's interface (src/render/nerf.py:15-371).

``NeRFRenderer.forward(model, rays, want_weights)`` keeps the reference's
contract.  When ``model`` is a :class:`pnr.models.PixelNeRFNet` whose conf the fused
kernel implements, the whole coarse + fine march (sampling, fused point MLP,
compositing, inverse-CDF resampling) runs as one stream-ordered sequence in libpnr.so
(``pnr_render_forward``).  Any other model -- including a PixelNeRFNet with a conf the
kernel does not implement (``fused_conf_reason()``) -- goes through the reference's plug
point ``model(points, coarse, viewdirs)`` with sampling and compositing still on the HIP
kernels, and with autograd when gradients are on.

Random draws (nerf.py:111, 135, 141, 158), ``rng_mode``:
  "counter" (default on the fused path) -- the kernels draw on device from a
            Philox4x32-10 {seed, offset} (include/pnr_abi.h pnr_rng); the seed comes
            from torch's default CPU generator once per call, so torch.manual_seed
            still makes renders reproducible, and no stream tensors touch HBM;
  "torch"   -- torch.rand / torch.randn on the rays' device in the reference's order
            and shapes: with the same torch seed the generator is consumed exactly as
            the reference consumes it.
``streams`` (tests / benchmarks) injects explicit draws for one call.  The
model-callback and training paths always draw with torch in the reference's order.
"""
import torch

from . import _lib, ops
from .prof import ranged
from .conf import as_conf

__all__ = ["NeRFRenderer", "DotMap"]


class DotMap(dict):
    """Attribute-access dict with ``toDict`` (the reference returns dotmap.DotMap)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k)

    def __setattr__(self, k, v):
        self[k] = v

    def toDict(self):
        return {k: (v.toDict() if isinstance(v, DotMap) else v) for k, v in self.items()}


class _RenderWrapper(torch.nn.Module):
    """nerf.py:15-42."""

    def __init__(self, net, renderer, simple_output):
        super().__init__()
        self.net = net
        self.renderer = renderer
        self.simple_output = simple_output

    def forward(self, rays, want_weights=False):
        if rays.shape[0] == 0:
            return (torch.zeros(0, 3, device=rays.device), torch.zeros(0, device=rays.device))
        outputs = self.renderer(self.net, rays, want_weights=want_weights and not self.simple_output)
        if self.simple_output:
            part = outputs.fine if self.renderer.using_fine else outputs.coarse
            return part.rgb, part.depth
        return outputs.toDict()


# ray_order "auto": block the rays when the projected latent rows (views x H_l x W_l x 2 KB x lin_z
# stages) exceed this -- past the XCDs' L2s and a good part of the 256 MB Infinity Cache
ORDER_AUTO_BYTES = 128 << 20


def ray_block_order(rays, block=16):
    """A processing order for a pinhole ray batch (pnr_render_cfg.ray_order): rays grouped in
    block x block squares of neighbouring pixels, the squares row by row, the input order kept
    inside a square.  Rays sharing a square sample neighbouring latent pixels in every source
    view, so the scheduling units running at once on an XCD share its L2 (cfg4).
    The target camera is not known here: the image plane is the plane perpendicular to the mean
    direction, at unit distance, and the pixel rows' direction and pitch the median step between
    consecutive rays (one pixel along a row for row-major input, gen_video's / eval's frames).
    Computed on the rays' device without a host synchronisation: an int32 (B,) permutation, the
    input order itself when the rays do not look like one pinhole camera's; None below 4 blocks."""
    B = rays.shape[0]
    if B < 4 * block * block:
        return None
    o, d = rays[:, :3], rays[:, 3:6]
    axis = d.mean(0)
    axis = axis / axis.norm()
    cz = d @ axis
    up = torch.zeros(3, device=d.device, dtype=d.dtype)
    up.scatter_(0, torch.argmin(axis.abs()).reshape(1), 1.0)
    e1 = torch.linalg.cross(axis, up)
    e1 = e1 / e1.norm()
    e2 = torch.linalg.cross(axis, e1)
    t = d / cz.clamp_min(1e-3)[:, None]
    u, v = t @ e1, t @ e2
    # the pixel rows' direction and pitch: the median step between consecutive rays (one pixel
    # along a row for row-major input; the row wraps are outliers), so the blocks align with
    # the image's rows and columns
    du, dv = torch.diff(u).median(), torch.diff(v).median()
    pitch = torch.sqrt(du * du + dv * dv)
    r1 = (e1 * du + e2 * dv) / pitch.clamp_min(1e-30)
    r2 = torch.linalg.cross(axis, r1)
    u, v = t @ r1, t @ r2
    cell = block * pitch.clamp_min(1e-30)
    cu = torch.floor((u - u.min()) / cell).clamp(0, (1 << 20) - 1).long()
    cv = torch.floor((v - v.min()) / cell).clamp(0, (1 << 20) - 1).long()
    perm = torch.argsort((cv << 20) + cu, stable=True).to(torch.int32)
    ok = ((o - o[:1]).abs().amax() <= 1e-4 * (1.0 + o[0].abs().amax())) & (cz.amin() > 1e-3) & (pitch > 0) & \
        torch.isfinite(pitch)
    return torch.where(ok, perm, torch.arange(B, device=rays.device, dtype=torch.int32))


class NeRFRenderer(torch.nn.Module):
    """NeRF volume renderer (nerf.py:45-371)."""

    def __init__(self, n_coarse=128, n_fine=0, n_fine_depth=0, noise_std=0.0, depth_std=0.01,
                 eval_batch_size=100000, white_bkgd=False, lindisp=False, sched=None):
        super().__init__()
        self.n_coarse = n_coarse
        self.n_fine = n_fine
        self.n_fine_depth = n_fine_depth
        self.noise_std = noise_std
        self.depth_std = depth_std
        self.eval_batch_size = eval_batch_size
        self.white_bkgd = white_bkgd
        self.lindisp = lindisp
        if lindisp:
            print("Using linear displacement rays")
        self.using_fine = n_fine > 0
        self.sched = sched
        if sched is not None and len(sched) == 0:
            self.sched = None
        self.register_buffer("iter_idx", torch.tensor(0, dtype=torch.long), persistent=True)
        self.register_buffer("last_sched", torch.tensor(0, dtype=torch.long), persistent=True)
        # test / benchmark hook: explicit (u_coarse, u_fine, u_fine_jit, n_depth)
        self.streams = None
        self.rng_mode = "counter"
        self.last_seed = None
        # fused path: rays per library call (bounds the raw / z workspace, ~3 KB per ray at
        # 64 + 64 samples); counter-mode draws do not depend on the chunking
        self.max_rays_per_call = 1 << 20
        # test / benchmark hook: add each pass's sample depths ``z`` (SB, B', K) to the
        # output dicts (fine-pass parity is classified on them, oracle/parity.py)
        self.return_z = False
        # ray-march schedule of this renderer's fused calls (pnr_render_cfg.march_mode, ABI 3):
        # None = the library default (pnr_render_set_fused, initially 2), else 0, 1, 2 or 3; all
        # give bit-identical results; per call, so renderers in different threads may differ
        self.march_mode = None
        # the fused march's processing order (pnr_render_cfg.ray_order, ABI 8; results are
        # bit-identical in every order): "auto" = 16 x 16 blocks of neighbouring rays when the
        # scene's projected-latent rows outgrow the caches (ORDER_AUTO_BYTES; cfg4's 3 views x
        # 150 x 200 x 3 stages = 553 MB: -3.5 % frame time, profiles/r6c), else the input order;
        # "blocked" / "input" force one
        self.ray_order = "auto"

    # ---- random streams (nerf.py:111, 135, 141, 158) ---------------------------------
    def fine_counts(self):
        """(importance samples, depth samples) of the fine pass (nerf.py:284-293); (0, 0)
        with ``using_fine`` still means a fine pass, over the coarse samples only."""
        if not self.using_fine:
            return 0, 0
        return max(self.n_fine - self.n_fine_depth, 0), max(self.n_fine_depth, 0)

    def draw_streams(self, n_rays, device):
        if self.streams is not None:
            s = tuple(t.to(device=device, dtype=torch.float32).contiguous() for t in self.streams)
            self.streams = None
            return s
        nf, kfd = self.fine_counts()
        u_c = torch.rand(n_rays, self.n_coarse, device=device)
        empty = torch.zeros(n_rays, 0, device=device)
        u_f = u_j = n_d = empty
        if self.using_fine:
            if nf > 0:
                u_f = torch.rand(n_rays, nf, device=device)
                u_j = torch.rand(n_rays, nf, device=device)
            if kfd > 0:
                n_d = torch.randn(n_rays, kfd, device=device)
        return u_c, u_f, u_j, n_d

    # ---- building blocks (HIP) -------------------------------------------------------
    def sample_coarse(self, rays, u=None):
        if u is None:
            u = torch.rand(rays.shape[0], self.n_coarse, device=rays.device)
        return ops.sample_coarse(rays, self.n_coarse, u, self.lindisp)

    @ranged("renderer_composite")
    def composite(self, model, rays, z_samp, coarse=True, sb=0):
        """nerf.py:163-249 through the model callback; compositing on the HIP kernel."""
        B, K = z_samp.shape
        points = rays[:, None, :3] + z_samp.unsqueeze(2) * rays[:, None, 3:6]
        points = points.reshape(-1, 3)
        use_viewdirs = hasattr(model, "use_viewdirs") and model.use_viewdirs
        if sb > 0:
            points = points.reshape(sb, -1, 3)
            ebs = (self.eval_batch_size - 1) // sb + 1
            dim = 1
        else:
            ebs, dim = self.eval_batch_size, 0
        vals = []
        if use_viewdirs:
            vd = rays[:, None, 3:6].expand(-1, K, -1)
            vd = vd.reshape(sb, -1, 3) if sb > 0 else vd.reshape(-1, 3)
            for pts, dirs in zip(torch.split(points, ebs, dim=dim), torch.split(vd, ebs, dim=dim)):
                vals.append(model(pts, coarse=coarse, viewdirs=dirs))
        else:
            for pts in torch.split(points, ebs, dim=dim):
                vals.append(model(pts, coarse=coarse))
        out = torch.cat(vals, dim=dim).reshape(B, K, -1)
        if self.training and self.noise_std > 0.0:   # nerf.py:225-226 (sigma only)
            n = torch.randn_like(out[..., 3])
            out = torch.cat([out[..., :3], out[..., 3:4] + (n * self.noise_std).unsqueeze(-1), out[..., 4:]], -1)
        raw = out[..., :4].contiguous()
        if torch.is_grad_enabled() and (raw.requires_grad or z_samp.requires_grad):
            from .train import Composite   # the composite kernel with its backward kernel

            return Composite.apply(z_samp, raw, rays, self.white_bkgd)
        return ops.composite(z_samp, raw, rays, self.white_bkgd)

    # ---- forward (nerf.py:251-303) ---------------------------------------------------
    @ranged("renderer_forward")
    def forward(self, model, rays, want_weights=False):
        if self.sched is not None and self.last_sched.item() > 0:
            self.n_coarse = self.sched[1][self.last_sched.item() - 1]
            self.n_fine = self.sched[2][self.last_sched.item() - 1]
        assert len(rays.shape) == 3
        sb = rays.shape[0]
        rays = rays.reshape(-1, 8).contiguous()
        B = rays.shape[0]
        from .models import PixelNeRFNet

        if isinstance(model, PixelNeRFNet) and model.fused_conf_reason() is None:
            # the sigma noise of training mode (nerf.py:225-226) is added between the model
            # and the composite, which the fused march does not expose: the training
            # graph's kernels run it, with or without autograd
            noisy = self.training and self.noise_std > 0.0
            if noisy or (torch.is_grad_enabled() and model.needs_grad()):
                return self._forward_train(model, rays, sb, want_weights)
            if self.streams is None and self.rng_mode == "counter":
                return self._forward_fused(model, rays, sb, None, want_weights)
            return self._forward_fused(model, rays, sb, self.draw_streams(B, rays.device), want_weights)
        return self._forward_callback(model, rays, sb, want_weights)

    def _forward_train(self, net, rays, sb, want_weights):
        """The reference's autograd graph (nerf.py:251-303) over the HIP kernels
        (pnr/train.py): coarse pass, importance samples from the detached coarse weights
        (nerf.py:130), depth samples with their gradient (nerf.py:150-161), sort, fine pass.
        With noise_std > 0 in training mode, sigma noise is added before compositing
        (nerf.py:225-226) and the draws follow the reference's order: u_coarse, coarse
        noise, u_fine, u_fine_jit, n_depth, fine noise."""
        from .train import Composite, FinePass, RenderPoints, mlp_params

        r = net.hip_unsupported_reason()
        if r:
            raise NotImplementedError("pnr: " + r)
        if rays.device.type != "cuda":
            raise ValueError("pnr: rays must be on the HIP device")
        kc = self.n_coarse
        nf, kfd = self.fine_counts()
        kf = nf + kfd
        noisy = self.training and self.noise_std > 0.0
        B, dev = rays.shape[0], rays.device
        lazy = noisy and self.streams is None   # draws interleave with the noise draws
        if lazy:
            u_c = torch.rand(B, kc, device=dev)
        else:
            u_c, u_f, u_j, n_d = [t.contiguous() for t in self.draw_streams(B, dev)]

        def add_noise(raw):   # nerf.py:225-226 (sigma only; relu inside the composite)
            if not noisy:
                return raw
            n = torch.randn(raw.shape[:2], device=dev)
            return torch.cat([raw[..., :3], raw[..., 3:] + (n * self.noise_std).unsqueeze(-1)], -1)

        lat = net.encoder.latent_cl
        if net.stop_encoder_grad:
            lat = lat.detach()
        p_c = mlp_params(net.mlp_coarse)
        z_c = ops.sample_coarse(rays, kc, u_c, self.lindisp)
        raw_c = add_noise(RenderPoints.apply(net, True, rays, z_c, lat, *p_c))
        w_c, rgb_c, d_c = Composite.apply(z_c, raw_c.contiguous(), rays, self.white_bkgd)
        outputs = DotMap(coarse=self._pack_out(w_c, rgb_c, d_c, sb, want_weights, z_c))
        if self.using_fine:
            if lazy:
                empty = torch.zeros(B, 0, device=dev)
                u_f = torch.rand(B, nf, device=dev) if nf > 0 else empty
                u_j = torch.rand(B, nf, device=dev) if nf > 0 else empty
                n_d = torch.randn(B, kfd, device=dev) if kfd > 0 else empty
            with torch.no_grad():
                z_ci = (ops.sample_fine(rays, z_c, w_c.detach(), d_c.detach(), nf, 0, self.depth_std, u_f, u_j,
                                        None, self.lindisp) if nf > 0 else z_c)
            parts = [z_ci]
            if kfd > 0:
                z_d = d_c.unsqueeze(1).repeat((1, kfd)) + n_d * self.depth_std
                parts.append(torch.max(torch.min(z_d, rays[:, -1:]), rays[:, -2:-1]))
            z_f, order = torch.sort(torch.cat(parts, -1), -1)
            z_f = z_f.contiguous()
            # only the depth samples' dL/dz reaches the graph (the importance samples carry none)
            fine = FinePass(order >= z_ci.shape[1] if kfd > 0 else None)
            p_f = mlp_params(net.mlp_fine) if net.mlp_fine is not None else p_c
            raw_f = add_noise(RenderPoints.apply(net, fine, rays, z_f, lat, *p_f))
            w_f, rgb_f, d_f = Composite.apply(z_f, raw_f.contiguous(), rays, self.white_bkgd)
            outputs.fine = self._pack_out(w_f, rgb_f, d_f, sb, want_weights, z_f)
        return outputs

    def _pack_out(self, w, rgb, depth, sb, want_weights, z=None):
        d = DotMap(rgb=rgb.reshape(sb, -1, 3), depth=depth.reshape(sb, -1))
        if want_weights:
            d.weights = w.reshape(sb, -1, w.shape[-1])
        if self.return_z and z is not None:
            d.z = z.reshape(sb, -1, z.shape[-1])
        return d

    def _forward_fused(self, net, rays, sb, streams, want_weights):
        """The whole march in libpnr.so (pnr_render_forward_proj).  ``streams`` None =
        counter-mode draws.  With ``using_fine`` and no fine samples the fine pass runs the
        fine MLP over the coarse samples (nerf.py:284-298 with all_samps = [z_coarse]): a
        second coarse-only march with the fine model and the same draws."""
        net._require_hip()
        if rays.device.type != "cuda":
            raise ValueError("pnr: rays must be on the HIP device")
        B = rays.shape[0]
        kc = self.n_coarse
        nf, kfd = self.fine_counts()
        kf = nf + kfd
        seed = None
        if streams is None:
            seed = int(torch.randint(0, 2 ** 63 - 1, (1,), dtype=torch.int64).item())
            self.last_seed = seed   # the counter-mode key of the last call (tests replay it)
        # one object: ray chunks of at most eval_batch_size rays (the reference bounds a model
        # call to eval_batch_size points, nerf.py:191-201; the fused march keeps no per-point
        # activations in HBM, so the bound is on rays: its workspace is ~4 KB per ray) and
        # max_rays_per_call.  Several objects: one call, the scene record covers them all
        # (chunking inside each object would move the rays' counter-mode draw indices).
        step = max(1, min(int(self.max_rays_per_call), int(self.eval_batch_size))) if sb == 1 else max(B, 1)
        starts = list(range(0, max(B, 1), step))
        # every chunk's processing order before the first render is queued: the order's host
        # decisions (ray_block_order) then never wait for a chunk in flight
        orders = ([ray_block_order(rays[r0:min(B, r0 + step)]) for r0 in starts]
                  if sb == 1 and self._blocked_order(net) else [None] * len(starts))
        parts = []
        for r0, order in zip(starts, orders):
            r1 = min(B, r0 + step)
            st = None if streams is None else tuple(t[r0:r1] for t in streams)
            if self.using_fine and kf == 0:
                out = self._fused_call(net, rays[r0:r1], sb, st, seed, r0, kc, 0, 0, True, want_weights, order)
                fine = self._fused_call(net, rays[r0:r1], sb, st, seed, r0, kc, 0, 0, False, want_weights, order)
                out.fine = fine.coarse
            else:
                out = self._fused_call(net, rays[r0:r1], sb, st, seed, r0, kc, kf, kfd, True, want_weights, order)
            parts.append(out)
        if len(parts) == 1:
            return parts[0]
        return DotMap({p: DotMap({k: torch.cat([o[p][k] for o in parts], 1) for k in parts[0][p]})
                       for p in parts[0]})

    def _fused_call(self, net, rays, sb, streams, seed, offset, kc, kf, kfd, coarse, want_weights, order=None):
        """One torch.ops.pnr.render_rays call (pnr_render_forward_proj).  coarse=False: the
        fine MLP in the coarse slot (a coarse-only march with the fine model).  ``order``: the
        processing order (pnr_render_cfg.ray_order) or None."""
        from . import torchops

        ops_ = torchops.load()
        B = rays.shape[0]
        desc, pc = net.hip_mlp(coarse)
        pf = net.hip_mlp(False)[1] if kf > 0 else pc
        zc = net.hip_proj(coarse)
        zf = net.hip_proj(False) if kf > 0 else None
        if streams is None:
            u_c = u_f = u_j = n_d = None
        else:
            u_c, u_f, u_j, n_d = [t.contiguous() for t in streams]
        res = ops_.render_rays(*torchops.scene_args(net), torchops.desc_list(desc), pc, pf, zc, zf, rays,
                               B // sb, kc, kf, kfd, float(self.depth_std), bool(self.white_bkgd),
                               bool(self.lindisp), u_c, u_f, u_j, n_d, int(seed or 0), int(offset),
                               bool(want_weights), bool(self.return_z),
                               torchops.EVENTS_HOOK(B, kc, kf) if torchops.EVENTS_HOOK else [],
                               -1 if self.march_mode is None else int(self.march_mode), order)
        c_rgb, c_depth, c_w, f_rgb, f_depth, f_w, z_c, z_f = res
        outputs = DotMap(coarse=self._pack_out(c_w if want_weights else None, c_rgb, c_depth, sb, want_weights,
                                               z_c if self.return_z else None))
        if kf > 0:
            outputs.fine = self._pack_out(f_w if want_weights else None, f_rgb, f_depth, sb, want_weights,
                                          z_f if self.return_z else None)
        return outputs

    def _blocked_order(self, net):
        if self.ray_order == "input":
            return False
        if self.ray_order == "blocked":
            return True
        if self.ray_order != "auto":
            raise ValueError("ray_order must be 'auto', 'blocked' or 'input' (got %r)" % (self.ray_order,))
        lat = getattr(net.encoder, "latent_cl", None)
        if lat is None or lat.dim() != 4:
            return False
        stages = min(net.mlp_coarse.combine_layer, net.mlp_coarse.n_blocks) if hasattr(net.mlp_coarse, "n_blocks") else 1
        return lat.shape[0] * lat.shape[1] * lat.shape[2] * 512 * 4 * max(stages, 1) > ORDER_AUTO_BYTES

    def _forward_callback(self, model, rays, sb, want_weights):
        """nerf.py:251-303 through the plug point ``model(points, coarse, viewdirs)``; sampling
        and compositing on the HIP kernels.  Under autograd the depth samples keep their
        gradient to the coarse depth (nerf.py:150-161, 292) and the fine depths are sorted with
        torch.sort, as in the reference's graph.  With training-mode sigma noise the draws
        interleave with the noise draws in the reference's order."""
        B, dev = rays.shape[0], rays.device
        nf, kfd = self.fine_counts()
        lazy = self.training and self.noise_std > 0.0 and self.streams is None
        if lazy:
            u_c = torch.rand(B, self.n_coarse, device=dev)
        else:
            u_c, u_f, u_j, n_d = self.draw_streams(B, dev)
        z_c = self.sample_coarse(rays, u_c)
        w_c, rgb_c, depth_c = self.composite(model, rays, z_c, coarse=True, sb=sb)
        outputs = DotMap(coarse=self._pack_out(w_c, rgb_c, depth_c, sb, want_weights, z_c))
        if self.using_fine:
            if lazy:
                empty = torch.zeros(B, 0, device=dev)
                u_f = torch.rand(B, nf, device=dev) if nf > 0 else empty
                u_j = torch.rand(B, nf, device=dev) if nf > 0 else empty
                n_d = torch.randn(B, kfd, device=dev) if kfd > 0 else empty
            if nf + kfd == 0:
                z_f = z_c
            elif torch.is_grad_enabled() and kfd > 0 and depth_c.requires_grad:
                with torch.no_grad():
                    z_ci = (ops.sample_fine(rays, z_c, w_c.detach(), depth_c.detach(), nf, 0, self.depth_std, u_f,
                                            u_j, None, self.lindisp) if nf > 0 else z_c)
                z_d = depth_c.unsqueeze(1).repeat((1, kfd)) + n_d * self.depth_std
                z_d = torch.max(torch.min(z_d, rays[:, -1:]), rays[:, -2:-1])
                z_f = torch.sort(torch.cat([z_ci, z_d], -1), -1)[0].contiguous()
            else:
                z_f = ops.sample_fine(rays, z_c, w_c.detach(), depth_c.detach(), nf + kfd, kfd, self.depth_std,
                                      u_f, u_j, n_d, self.lindisp)
            w_f, rgb_f, depth_f = self.composite(model, rays, z_f, coarse=False, sb=sb)
            outputs.fine = self._pack_out(w_f, rgb_f, depth_f, sb, want_weights, z_f)
        return outputs

    # ---- schedule / construction / parallel (nerf.py:318-371) ------------------------
    def sched_step(self, steps=1):
        if self.sched is None:
            return
        self.iter_idx += steps
        while (self.last_sched.item() < len(self.sched[0])
               and self.iter_idx.item() >= self.sched[0][self.last_sched.item()]):
            self.n_coarse = self.sched[1][self.last_sched.item()]
            self.n_fine = self.sched[2][self.last_sched.item()]
            print("INFO: NeRF sampling resolution changed on schedule ==> c", self.n_coarse,
                  "f", self.n_fine)
            self.last_sched += 1

    @classmethod
    def from_conf(cls, conf, white_bkgd=False, lindisp=False, eval_batch_size=100000):
        conf = as_conf(conf)
        return cls(conf.get_int("n_coarse", 128), conf.get_int("n_fine", 0),
                   n_fine_depth=conf.get_int("n_fine_depth", 0),
                   noise_std=conf.get_float("noise_std", 0.0),
                   depth_std=conf.get_float("depth_std", 0.01),
                   white_bkgd=conf.get_float("white_bkgd", white_bkgd), lindisp=lindisp,
                   eval_batch_size=conf.get_int("eval_batch_size", eval_batch_size),
                   sched=conf.get_list("sched", None))

    def bind_parallel(self, net, gpus=None, simple_output=False):
        """nerf.py:354-371.  With several GPU ids this wraps in nn.DataParallel like the
        reference; the MI355X-native scaling path is one process per GPU
        (see pnr.dist / bench.py)."""
        wrapped = _RenderWrapper(net, self, simple_output=simple_output)
        if gpus is not None and len(gpus) > 1:
            print("Using multi-GPU", gpus)
            wrapped = torch.nn.DataParallel(wrapped, gpus, dim=1)
        return wrapped
