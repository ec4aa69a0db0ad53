"""PixelNeRFNet / ResnetFC / PositionalEncoding with the reference's interface.

Same constructor (``make_model(conf)``), ``encode``, ``forward``,
``load_weights`` / ``save_weights``, buffers and state-dict keys as the reference
(models.py:15-316, resnetfc.py:10-198, code.py:6-52) so checkpoints load
unchanged.  The per-point evaluation (``forward``, models.py:146-266) and the
full ray march (``pnr.renderer.NeRFRenderer``) run in libpnr.so on the HIP
device; the nn.Linear modules here are the parameter store the kernels read
(packed once per weight version by ``pnr_mlp_pack``).

Confs the fused kernel does not implement (``PixelNeRFNet.fused_conf_reason()``: softplus
``beta``, widths other than 512, ``use_code_viewdirs``, SPADE, max-combine, the global encoder,
other grid_sample modes) take the reference's callback path instead: the model
runs as device torch ops (``PixelNeRFNet.forward`` -> ``ResnetFC.forward``, hipBLASLt GEMMs)
and NeRFRenderer still samples and composites on the HIP kernels.  CPU tensors are refused on
both paths.
"""
import os
import os.path as osp
import warnings
import weakref

import numpy as np
import torch
from torch import nn

from . import _lib
from .consts import device_const
from .conf import as_conf
from .encoder import ImageEncoder, SpatialEncoder
from .prof import ranged
from .util import combine_interleaved, repeat_interleave

__all__ = ["PositionalEncoding", "ResnetBlockFC", "ResnetFC", "PixelNeRFNet", "make_model",
           "make_mlp", "make_encoder", "PRECISIONS"]

# Arithmetic of the 512-wide ResnetFC GEMMs (include/pnr_abi.h, PNR_PREC_*).  All modes
# take fp32 in / fp32 out with fp32 accumulation:
#   "fp32"   v_mfma_f32_16x16x4_f32
#   "bf16x9" exact 3-way bf16 split of both operands, all 9 products (exact products,
#            fp32 accumulation: numerically an fp32 GEMM)
#   "bf16x6" the 6 largest products of that split (error at the fp32 unit roundoff)
#   "f16x3"  power-of-two scaled operands (per layer / per activation column), each
#            split into two fp16 parts; 3 exact products on v_mfma_f32_16x16x32_f16
#            (error at the fp32 level, tools/precision_study.py)
PRECISIONS = {"fp32": 0, "f16x3": 3, "bf16x6": 6, "bf16x9": 9}


def _own_params(m):
    """The parameters registered directly on ``m``.  On an nn.DataParallel replica
    (torch.nn.parallel.replicate) ``_parameters`` is empty: the broadcast copies are plain
    attributes, listed in ``_former_parameters``."""
    if m._parameters or not getattr(m, "_is_replica", False):
        return list(m._parameters.values())
    return list(m.__dict__.get("_former_parameters", {}).values())


def module_params(mod, skip=None):
    """``mod.parameters()`` that also works on an nn.DataParallel replica (the tensors the
    replica's forward reads and autograd differentiates), in registration order; submodules
    named by ``skip`` (a direct child) are left out."""
    out, seen = [], set()
    skip_mod = mod._modules.get(skip) if skip else None
    excluded = set(id(m) for m in skip_mod.modules()) if skip_mod is not None else set()
    for m in mod.modules():
        if id(m) in excluded:
            continue
        for p in _own_params(m):
            if p is not None and id(p) not in seen:
                seen.add(id(p))
                out.append(p)
    return out


class PositionalEncoding(nn.Module):
    """NeRF sin/cos encoding (code.py:6-52); cos computed as sin(x + pi/2)."""

    def __init__(self, num_freqs=6, d_in=3, freq_factor=np.pi, include_input=True):
        super().__init__()
        self.num_freqs = num_freqs
        self.d_in = d_in
        self.freqs = freq_factor * 2.0 ** torch.arange(0, num_freqs)
        self.d_out = self.num_freqs * 2 * d_in + (d_in if include_input else 0)
        self.include_input = include_input
        self.register_buffer("_freqs", torch.repeat_interleave(self.freqs, 2).view(1, -1, 1))
        phases = torch.zeros(2 * self.num_freqs)
        phases[1::2] = np.pi * 0.5
        self.register_buffer("_phases", phases.view(1, -1, 1))

    @ranged("positional_enc")
    def forward(self, x):
        embed = x.unsqueeze(1).repeat(1, self.num_freqs * 2, 1)
        embed = torch.sin(torch.addcmul(self._phases, embed, self._freqs))
        embed = embed.view(x.shape[0], -1)
        return torch.cat((x, embed), dim=-1) if self.include_input else embed

    @classmethod
    def from_conf(cls, conf, d_in=3):
        return cls(conf.get_int("num_freqs", 6), d_in, conf.get_float("freq_factor", np.pi),
                   conf.get_bool("include_input", True))


class ResnetBlockFC(nn.Module):
    """x + fc_1(act(fc_0(act(x)))), act = relu or softplus(beta) (resnetfc.py:10-62).  The
    fused kernel reads the parameters; ``forward`` is the callback path's device evaluation."""

    def __init__(self, size_in, size_out=None, size_h=None, beta=0.0):
        super().__init__()
        size_out = size_in if size_out is None else size_out
        size_h = min(size_in, size_out) if size_h is None else size_h
        self.size_in, self.size_h, self.size_out = size_in, size_h, size_out
        self.fc_0 = nn.Linear(size_in, size_h)
        self.fc_1 = nn.Linear(size_h, size_out)
        nn.init.constant_(self.fc_0.bias, 0.0)
        nn.init.kaiming_normal_(self.fc_0.weight, a=0, mode="fan_in")
        nn.init.constant_(self.fc_1.bias, 0.0)
        nn.init.zeros_(self.fc_1.weight)
        self.beta = beta
        self.activation = nn.Softplus(beta=beta) if beta > 0 else nn.ReLU()
        self.shortcut = None
        if size_in != size_out:
            self.shortcut = nn.Linear(size_in, size_out, bias=False)

    @ranged("resblock")
    def forward(self, x):
        h = self.fc_0(self.activation(x))
        res = x if self.shortcut is None else self.shortcut(x)
        return res + self.fc_1(self.activation(h))


class ResnetFC(nn.Module):
    """ResnetFC (resnetfc.py:65-198): the parameter layout the fused kernel reads, and the
    callback path's device forward for confs the kernel does not implement."""

    def __init__(self, d_in, d_out=4, n_blocks=5, d_latent=0, d_hidden=128, beta=0.0,
                 combine_layer=1000, combine_type="average", use_spade=False):
        super().__init__()
        if d_in > 0:
            self.lin_in = nn.Linear(d_in, d_hidden)
            nn.init.constant_(self.lin_in.bias, 0.0)
            nn.init.kaiming_normal_(self.lin_in.weight, a=0, mode="fan_in")
        self.lin_out = nn.Linear(d_hidden, d_out)
        nn.init.constant_(self.lin_out.bias, 0.0)
        nn.init.kaiming_normal_(self.lin_out.weight, a=0, mode="fan_in")
        self.n_blocks, self.d_latent, self.d_in = n_blocks, d_latent, d_in
        self.d_out, self.d_hidden = d_out, d_hidden
        self.combine_layer, self.combine_type, self.use_spade = combine_layer, combine_type, use_spade
        self.beta = beta
        self.blocks = nn.ModuleList([ResnetBlockFC(d_hidden, beta=beta) for _ in range(n_blocks)])
        self.activation = nn.Softplus(beta=beta) if beta > 0 else nn.ReLU()
        if d_latent != 0:
            n_lin_z = min(combine_layer, n_blocks)
            self.lin_z = nn.ModuleList([nn.Linear(d_latent, d_hidden) for _ in range(n_lin_z)])
            for lz in self.lin_z:
                nn.init.constant_(lz.bias, 0.0)
                nn.init.kaiming_normal_(lz.weight, a=0, mode="fan_in")
            if use_spade:
                self.scale_z = nn.ModuleList([nn.Linear(d_latent, d_hidden) for _ in range(n_lin_z)])

    @ranged("resnetfc_infer")
    def forward(self, zx, combine_inner_dims=(1,), combine_index=None, dim_size=None):
        """(N, d_latent + d_in) -> (N', d_out) (resnetfc.py:132-184), as device torch ops: the
        callback path of PixelNeRFNet confs the fused kernel does not implement (the fused
        kernel evaluates the shipped conf inside the ray march).  ``combine_index`` /
        ``dim_size`` are the reference's disabled frustum-culling arguments (ignored there)."""
        z, x = zx[..., :self.d_latent], zx[..., self.d_latent:]
        x = self.lin_in(x) if self.d_in > 0 else torch.zeros(self.d_hidden, device=zx.device)
        for b, blk in enumerate(self.blocks):
            if b == self.combine_layer:
                x = combine_interleaved(x, combine_inner_dims, self.combine_type)
            if self.d_latent > 0 and b < self.combine_layer:
                t = self.lin_z[b](z)
                x = self.scale_z[b](z) * x + t if self.use_spade else x + t
            x = blk(x)
        return self.lin_out(self.activation(x))

    @classmethod
    def from_conf(cls, conf, d_in, **kwargs):
        return cls(d_in, n_blocks=conf.get_int("n_blocks", 5), d_hidden=conf.get_int("d_hidden", 128),
                   beta=conf.get_float("beta", 0.0), combine_layer=conf.get_int("combine_layer", 1000),
                   combine_type=conf.get_string("combine_type", "average"),
                   use_spade=conf.get_bool("use_spade", False), **kwargs)

    # ---- HIP packing -----------------------------------------------------------------
    def hip_unsupported_reason(self):
        if self.d_in <= 0 or self.d_latent != 512 or self.d_hidden != 512:
            return "d_hidden = d_latent = 512 and d_in > 0 required (got %d/%d/%d)" % (
                self.d_hidden, self.d_latent, self.d_in)
        if self.d_out != 4:
            return "d_out must be 4"
        if self.beta > 0:
            return "softplus activation (beta > 0) not implemented"
        if self.combine_type != "average":
            return "combine_type %r not implemented" % self.combine_type
        if self.use_spade:
            return "use_spade not implemented"
        if self.n_blocks > 8:
            return "n_blocks > 8"
        return None

    def desc(self, pe_n, precision="fp32"):
        return _lib.MlpDesc(self.d_in, self.d_latent, self.d_hidden, self.d_out, self.n_blocks,
                            self.combine_layer, pe_n, PRECISIONS[precision])

    def _weights(self, code, desc):
        """pnr_mlp_weights over fp32 contiguous views of the parameters (+ the temporaries
        that must outlive the pack launch)."""
        keep = []

        def p(t):
            t = t.detach().float().contiguous()
            keep.append(t)
            return t.data_ptr()

        w = _lib.MlpWeights()
        w.desc = desc
        w.lin_in_w, w.lin_in_b = p(self.lin_in.weight), p(self.lin_in.bias)
        w.lin_out_w, w.lin_out_b = p(self.lin_out.weight), p(self.lin_out.bias)
        for i, lz in enumerate(getattr(self, "lin_z", [])):
            w.lin_z_w[i], w.lin_z_b[i] = p(lz.weight), p(lz.bias)
        for i, blk in enumerate(self.blocks):
            w.fc0_w[i], w.fc0_b[i] = p(blk.fc_0.weight), p(blk.fc_0.bias)
            w.fc1_w[i], w.fc1_b[i] = p(blk.fc_1.weight), p(blk.fc_1.bias)
        w.pe_freqs, w.pe_phases = p(code._freqs.reshape(-1)), p(code._phases.reshape(-1))
        return w, keep

    def _cached(self, name):
        """This module's own entry of cache ``name`` (None if absent).  Every cache entry
        starts with a weak reference to the module that built it: nn.DataParallel's
        replicas (torch.nn.parallel.replicate -> _replicate_for_data_parallel) start from a
        copy of the original's __dict__, so without the owner check a replica would find
        the original's packs, which live on the original's device (nerf.py:354-371)."""
        c = self.__dict__.get(name)
        return c if c is not None and c[0]() is self else None

    def _pack_key(self, code, precision):
        # the submodule list is cached (nn.Module.parameters() walks and de-duplicates the
        # tree on every call: ~50 us of host time per MLP per render call); each submodule's
        # parameter dict is read live, so a reassigned parameter still changes the key.  The
        # snapshot belongs to the module that took it (a DataParallel replica inherits the
        # original's snapshot in its __dict__ copy and must take its own).
        snap = self.__dict__.get("_pnr_mods")
        if (snap is None or snap[0][0] is not self
                or any(tuple(m._modules.values()) != kids for m, kids in snap)):   # submodule swapped
            snap = [(m, tuple(m._modules.values())) for m in self.modules()]
            self.__dict__["_pnr_mods"] = snap
        params = [p for m, _ in snap for p in _own_params(m) if p is not None]
        dev = self.lin_out.weight.device
        return (precision, str(dev)) + tuple((p.data_ptr(), p._version)
                                             for p in params + [code._freqs, code._phases])

    def packed(self, code, precision="fp32"):
        """Packed fragment-order copy of the weights (re-packed when they change).  The
        pack is stream-ordered on the current stream: no host sync (the temporaries stay
        referenced by the cache until the next re-pack)."""
        key = self._pack_key(code, precision)
        cache = self._cached("_pnr_pack")
        if cache is not None and cache[1] == key:
            return cache[2], cache[3]
        pe_n = int(code._freqs.numel())
        desc = self.desc(pe_n, precision)
        lib = _lib.load()
        nbytes = lib.pnr_mlp_packed_bytes(desc)
        if nbytes == 0:
            _lib.check(-2, "pnr_mlp_packed_bytes")
        dev = self.lin_out.weight.device
        buf = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
        w, keep = self._weights(code, desc)
        _lib.check(lib.pnr_mlp_pack(w, _lib.ptr(buf), nbytes, _lib.stream_of(dev)), "pnr_mlp_pack")
        self.__dict__["_pnr_pack"] = (weakref.ref(self), key, desc, buf, keep)
        return desc, buf

    def packed_t(self, code, precision="f16x3"):
        """Transposed (backward) pack for pnr_mlp_backward, f16x3 only: (desc, packed,
        packed_t), re-packed with the forward pack."""
        desc, buf = self.packed(code, precision)
        key = self._pack_key(code, precision)
        cache = self._cached("_pnr_pack_t")
        if cache is not None and cache[1] == key:
            return desc, buf, cache[2]
        lib = _lib.load()
        nbytes = lib.pnr_mlp_packed_t_bytes(desc)
        if nbytes == 0:
            _lib.check(-2, "pnr_mlp_packed_t_bytes (f16x3 models only)")
        dev = self.lin_out.weight.device
        buf_t = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
        w, keep = self._weights(code, desc)
        _lib.check(lib.pnr_mlp_pack_t(w, _lib.ptr(buf), _lib.ptr(buf_t), nbytes, _lib.stream_of(dev)),
                   "pnr_mlp_pack_t")
        self.__dict__["_pnr_pack_t"] = (weakref.ref(self), key, buf_t, keep)
        return desc, buf, buf_t

    def latent_proj(self, code, scene, latent):
        """Projected latent of this MLP's lin_z layers for the encoded scene
        (pnr_latent_project: lin_z[b].weight . latent at every latent pixel, fp32), which the
        fused kernel blends per point instead of running the lin_z GEMMs (resnetfc.py:160-163;
        exact by linearity of grid_sample's bilinear blend).  Cached per (weight version,
        latent tensor + version); None if the MLP has no lin_z layers."""
        if len(getattr(self, "lin_z", [])) == 0:
            return None
        key = self._pack_key(code, None)
        cache = self._cached("_pnr_proj")
        if (cache is not None and cache[1] == key and cache[2]() is latent
                and cache[3] == latent._version):
            return cache[4]
        if latent.device != self.lin_out.weight.device:
            raise ValueError("pnr: latent on %s but the MLP weights on %s" % (latent.device,
                                                                              self.lin_out.weight.device))
        desc = self.desc(int(code._freqs.numel()))
        lib = _lib.load()
        nbytes = lib.pnr_latent_project_bytes(scene, desc)
        if nbytes == 0:
            _lib.check(-1, "pnr_latent_project_bytes")
        buf = torch.empty(nbytes // 4, dtype=torch.float32, device=latent.device)
        w, keep = self._weights(code, desc)
        _lib.check(lib.pnr_latent_project(scene, w, _lib.ptr(buf), nbytes, _lib.stream_of(latent.device)),
                   "pnr_latent_project")
        self.__dict__["_pnr_proj"] = (weakref.ref(self), key, weakref.ref(latent), latent._version, buf, keep)
        return buf

    def drop_latent_proj(self):
        self.__dict__.pop("_pnr_proj", None)


def make_mlp(conf, d_in, d_latent=0, allow_empty=False, **kwargs):
    """model_util.py:5-15 (type = resnet is the implemented MLP)."""
    mlp_type = conf.get_string("type", "mlp")
    if mlp_type == "resnet":
        return ResnetFC.from_conf(conf, d_in, d_latent=d_latent, **kwargs)
    if mlp_type == "empty" and allow_empty:
        return None
    raise NotImplementedError("Unsupported MLP type %r (pnr implements type = resnet)" % mlp_type)


def make_encoder(conf, **kwargs):
    enc_type = conf.get_string("type", "spatial")
    if enc_type == "spatial":
        return SpatialEncoder.from_conf(conf, **kwargs)
    raise NotImplementedError("Unsupported encoder type %r" % enc_type)


class PixelNeRFNet(nn.Module):
    """pixelNeRF network (models.py:15-316)."""

    def __init__(self, conf, stop_encoder_grad=False):
        super().__init__()
        conf = as_conf(conf)
        self.encoder = make_encoder(conf["encoder"])
        self.use_encoder = conf.get_bool("use_encoder", True)
        self.use_xyz = conf.get_bool("use_xyz", False)
        assert self.use_encoder or self.use_xyz
        self.normalize_z = conf.get_bool("normalize_z", True)
        self.stop_encoder_grad = stop_encoder_grad
        self.use_code = conf.get_bool("use_code", False)
        self.use_code_viewdirs = conf.get_bool("use_code_viewdirs", True)
        self.use_viewdirs = conf.get_bool("use_viewdirs", False)
        self.use_global_encoder = conf.get_bool("use_global_encoder", False)
        d_latent = self.encoder.latent_size if self.use_encoder else 0
        d_in = 3 if self.use_xyz else 1
        if self.use_viewdirs and self.use_code_viewdirs:
            d_in += 3
        self.code = None
        if self.use_code and d_in > 0:
            self.code = PositionalEncoding.from_conf(conf["code"], d_in=d_in)
            d_in = self.code.d_out
        if self.use_viewdirs and not self.use_code_viewdirs:
            d_in += 3
        if self.use_global_encoder:
            # global image feature (models.py:62-66); the model then takes the callback path
            self.global_encoder = ImageEncoder.from_conf(conf["global_encoder"])
            self.global_latent_size = self.global_encoder.latent_size
            d_latent += self.global_latent_size
        d_out = 4
        self.latent_size = self.encoder.latent_size
        self.mlp_coarse = make_mlp(conf["mlp_coarse"], d_in, d_latent, d_out=d_out)
        self.mlp_fine = make_mlp(conf["mlp_fine"], d_in, d_latent, d_out=d_out, allow_empty=True)
        self.register_buffer("poses", torch.empty(1, 3, 4), persistent=False)
        self.register_buffer("image_shape", torch.empty(2), persistent=False)
        self.d_in, self.d_out, self.d_latent = d_in, d_out, d_latent
        self.register_buffer("focal", torch.empty(1, 2), persistent=False)
        self.register_buffer("c", torch.empty(1, 2), persistent=False)
        # HIP-side scene: per-(object, view) camera records (SB*NS, 16)
        self.register_buffer("cams", torch.empty(0, 16), persistent=False)
        self.num_objs = 0
        self.num_views_per_obj = 1
        # GEMM arithmetic of the fused kernel (see PRECISIONS): the scaled split-fp16 mode
        # has fp32-level error at 3.2x the f32-MFMA throughput
        self.mlp_precision = "f16x3"
        # inference: fold lin_z into the latent once per (scene, weights) and blend four
        # projected rows per point (ResnetFC.latent_proj) instead of the per-point lin_z GEMMs
        self.use_latent_proj = True
        # arithmetic of the training backward's 512 x 512 weight gradients (pnr_weight_grad_arith):
        # "f16x3" (fast; fp32-level relative to each channel's scale, include/pnr_abi.h) or
        # "bf16x6" (fp32-level per element whatever the dynamic range, ~1.4x the kernel time)
        self.wgrad_arith = "f16x3"

    # ---- encode ---------------------------------------------------------------------
    def encode(self, images, poses, focal, z_bounds=None, c=None):
        """models.py:89-144: run the encoder CNN, then set world->camera poses and
        intrinsics.  images (NS, 3, H, W) or (SB, NS, 3, H, W)."""
        self.num_objs = images.size(0)
        if len(images.shape) == 5:
            assert len(poses.shape) == 4 and poses.size(1) == images.size(1)
            self.num_views_per_obj = images.size(1)
            images = images.reshape(-1, *images.shape[2:])
            poses = poses.reshape(-1, 4, 4)
        else:
            self.num_views_per_obj = 1
        self.encoder(images)
        self._set_cameras(poses, focal, c, images.shape[-1], images.shape[-2])
        if self.use_global_encoder:
            self.global_encoder(images)

    def encode_latent(self, latent, poses, focal, image_size, c=None, num_objs=1, global_latent=None):
        """Install a precomputed feature map (SB*NS, C, H_l, W_l) instead of running the
        CNN; ``image_size`` = (W, H) of the source images.  ``global_latent`` (SB*NS, L): the
        global encoder's output (use_global_encoder), likewise precomputed."""
        ns = latent.shape[0] // num_objs
        self.num_objs = num_objs
        self.num_views_per_obj = ns
        if poses.dim() == 4:
            poses = poses.reshape(-1, 4, 4)
        self.encoder.set_latent(latent.float().contiguous())
        self._set_cameras(poses, focal, c, image_size[0], image_size[1])
        if self.use_global_encoder:
            if global_latent is None:
                raise ValueError("use_global_encoder: pass the global latent (SB*NS, %d)" % self.global_latent_size)
            self.global_encoder.latent = global_latent.float()

    def _set_cameras(self, poses, focal, c, width, height):
        dev = self.encoder.latent.device
        poses = poses.to(dev).float()
        rot = poses[:, :3, :3].transpose(1, 2)
        trans = -torch.bmm(rot, poses[:, :3, 3:])
        self.poses = torch.cat((rot, trans), dim=-1)
        self.image_shape = device_const((width, height), dev)
        self._image_wh = (float(width), float(height))   # host copy: hip_scene() never syncs
        focal = torch.as_tensor(focal).to(dev)
        if focal.dim() == 0:
            focal = focal[None, None].repeat((1, 2))
        elif focal.dim() == 1:
            focal = focal.unsqueeze(-1).repeat((1, 2))
        else:
            focal = focal.clone()
        self.focal = focal.float()
        self.focal[..., 1] *= -1.0
        if c is None:
            c = (self.image_shape * 0.5).unsqueeze(0)
        else:
            c = torch.as_tensor(c).to(dev).float()
            if c.dim() == 0:
                c = c[None, None].repeat((1, 2))
            elif c.dim() == 1:
                c = c.unsqueeze(-1).repeat((1, 2))
        self.c = c
        self._build_cams()

    def _build_cams(self):
        sb, ns = self.num_objs, self.num_views_per_obj
        n = self.poses.shape[0]
        if n != sb * ns:
            raise ValueError("poses (%d) != objects (%d) x views (%d)" % (n, sb, ns))
        obj = torch.arange(n, device=self.poses.device) // ns

        def per_obj(t, name):
            if t.shape[0] == 1:
                return t.expand(n, 2)
            if t.shape[0] == sb:
                return t[obj]
            raise ValueError("%s has %d rows; expected 1 or %d (one per object)" % (name, t.shape[0], sb))

        f = per_obj(self.focal, "focal")
        c = per_obj(self.c, "c")
        self.cams = torch.cat([self.poses[:, :, :3].reshape(n, 9), self.poses[:, :, 3], f, c],
                              dim=1).float().contiguous()

    # ---- HIP scene ------------------------------------------------------------------
    def fused_conf_reason(self):
        """Why the fused HIP kernel cannot evaluate this model's CONFIGURATION (None: it can).
        Such a model takes the reference's callback path: device torch ops for
        the model, HIP kernels for sampling and compositing."""
        if not (self.use_encoder and self.use_xyz and self.normalize_z and self.use_code
                and self.use_viewdirs and not self.use_code_viewdirs):
            return ("the fused kernel implements use_encoder, use_xyz, normalize_z, use_code, "
                    "use_viewdirs with use_code_viewdirs = False (the shipped confs)")
        if self.use_global_encoder:
            return "use_global_encoder"
        if self.code is None or not self.code.include_input:
            return "positional encoding must include the input"
        if self.encoder.index_interp != "bilinear" or self.encoder.index_padding != "border":
            return "the fused gather implements bilinear / border indexing"
        for mlp in (self.mlp_coarse, self.mlp_fine):
            if mlp is not None:
                r = mlp.hip_unsupported_reason()
                if r:
                    return r
        return None

    def hip_unsupported_reason(self):
        """fused_conf_reason(), or a scene the fused path cannot render yet."""
        r = self.fused_conf_reason()
        if r:
            return r
        if self.encoder.latent_cl.numel() == 0:
            return "encode() has not been called"
        if self.num_views_per_obj > 1 and self.mlp_coarse.combine_layer >= self.mlp_coarse.n_blocks:
            return "multi-view input needs combine_layer < n_blocks"
        return None

    def needs_grad(self):
        """Does a forward now have to build the autograd graph (training)?"""
        lat = self.encoder.latent_cl
        return any(p.requires_grad for p in module_params(self, skip="encoder")) \
            or (lat.requires_grad and not self.stop_encoder_grad)

    def _require_hip(self):
        r = self.hip_unsupported_reason()
        if r:
            raise NotImplementedError("pnr: " + r)

    def hip_scene(self):
        lat = self.encoder.latent_cl
        sc = _lib.Scene()
        sc.latent = lat.data_ptr()
        sc.cams = self.cams.data_ptr()
        sc.n_obj = self.num_objs
        sc.n_views = self.num_views_per_obj
        sc.latent_h, sc.latent_w, sc.latent_c = lat.shape[1], lat.shape[2], lat.shape[3]
        wh = self.__dict__.get("_image_wh")
        if wh is None:   # image_shape installed without _set_cameras (e.g. a state dict)
            wh = (float(self.image_shape[0]), float(self.image_shape[1]))
        sc.image_w, sc.image_h = wh
        return sc

    def hip_mlp(self, coarse):
        mlp = self.mlp_coarse if (coarse or self.mlp_fine is None) else self.mlp_fine
        if self.mlp_precision not in PRECISIONS:
            raise ValueError("mlp_precision must be one of %s" % sorted(PRECISIONS))
        return mlp.packed(self.code, self.mlp_precision)

    def hip_proj(self, coarse, scene=None):
        """Device pointer-holder of the projected latent for the coarse / fine MLP, or None
        (use_latent_proj off, or no lin_z layers)."""
        if not self.use_latent_proj:
            return None
        mlp = self.mlp_coarse if (coarse or self.mlp_fine is None) else self.mlp_fine
        return mlp.latent_proj(self.code, scene if scene is not None else self.hip_scene(),
                               self.encoder.latent_cl)

    def drop_latent_proj(self):
        """Forget the cached projections (they are rebuilt on the next render)."""
        for mlp in (self.mlp_coarse, self.mlp_fine):
            if mlp is not None:
                mlp.drop_latent_proj()

    # ---- forward (point query) -----------------------------------------------------
    @ranged("model_inference")
    def forward(self, xyz, coarse=True, viewdirs=None, far=False):
        """(SB, B, 3) world points -> (SB, B, 4) [sigmoid(rgb), relu(sigma)]
        (models.py:146-266) on the HIP device: the fused kernel for the confs it implements,
        device torch ops (the callback path) for the others.

        With grad enabled and trainable parameters (or a latent that carries gradient) the output
        carries the reference's autograd graph, as the reference's does: eval/eval.py:100 and
        train/train.py:422 query without torch.no_grad().  The query then runs the training
        forward (``train.RenderPoints`` on rays o = xyz, d = viewdirs at z = 0, so o + z d = xyz
        exactly), differentiable in the MLP parameters and the latent; a query whose xyz or
        viewdirs themselves require grad takes the device torch ops (differentiable in them too)."""
        if self.fused_conf_reason() is not None:
            return self._forward_torch(xyz, coarse, viewdirs)
        self._require_hip()
        SB, B, _ = xyz.shape
        if SB != self.num_objs:
            raise ValueError("xyz has %d objects but encode() saw %d" % (SB, self.num_objs))
        if torch.is_grad_enabled() and self.needs_grad():
            if xyz.requires_grad or (viewdirs is not None and viewdirs.requires_grad):
                return self._forward_torch(xyz, coarse, viewdirs)
            return self._forward_points_grad(xyz, coarse, viewdirs)
        from .ops import _dev

        from . import torchops

        xyz = _dev(xyz, "xyz")
        vd = _dev(viewdirs.reshape(SB, B, 3), "viewdirs") if viewdirs is not None else None
        desc, packed = self.hip_mlp(coarse)
        proj = self.hip_proj(coarse)
        return torchops.load().point_query(*torchops.scene_args(self), torchops.desc_list(desc), packed, proj,
                                           xyz, vd)

    def _forward_points_grad(self, xyz, coarse, viewdirs):
        """The point query with its autograd graph (see forward): one training-forward sample per
        point, rays [xyz, viewdirs, 0, 0] at z = 0."""
        from .ops import _dev
        from .train import RenderPoints, mlp_params

        SB, B, _ = xyz.shape
        xyz = _dev(xyz, "xyz").detach().float()
        vd = (_dev(viewdirs, "viewdirs").detach().float().reshape(SB, B, 3) if viewdirs is not None
              else torch.zeros_like(xyz))
        rays = torch.cat((xyz, vd, torch.zeros(SB, B, 2, device=xyz.device)), -1).reshape(SB * B, 8).contiguous()
        z = torch.zeros(SB * B, 1, device=xyz.device)
        lat = self.encoder.latent_cl
        if self.stop_encoder_grad:
            lat = lat.detach()
        mlp = self.mlp_coarse if (coarse or self.mlp_fine is None) else self.mlp_fine
        raw = RenderPoints.apply(self, coarse, rays, z, lat, *mlp_params(mlp))
        return raw.reshape(SB, B, 4)

    def _forward_torch(self, xyz, coarse, viewdirs):
        """models.py:146-266 as device torch ops (hipBLASLt GEMMs, grid_sample): the callback
        path of confs the fused kernel does not implement.  Differentiable (training through
        NeRFRenderer's callback path).  CPU tensors are refused as on the fused path."""
        if xyz.device.type != "cuda":
            raise ValueError("pnr: xyz must be on a HIP device (got %s); the HIP path has no CPU "
                             "fallback" % xyz.device)
        SB, B, _ = xyz.shape
        NS = self.num_views_per_obj
        rot = self.poses[:, None, :3, :3]
        xyz = repeat_interleave(xyz, NS)                          # (SB NS, B, 3)
        xyz_rot = torch.matmul(rot, xyz.unsqueeze(-1))[..., 0]
        xyz = xyz_rot + self.poses[:, None, :3, 3]
        feats = None
        if self.d_in > 0:
            p = xyz_rot if self.normalize_z else xyz
            feats = p.reshape(-1, 3) if self.use_xyz else -p[..., 2].reshape(-1, 1)
            if self.use_code and not self.use_code_viewdirs:
                feats = self.code(feats)
            if self.use_viewdirs:
                assert viewdirs is not None
                vd = repeat_interleave(viewdirs.reshape(SB, B, 3, 1), NS)
                feats = torch.cat((feats, torch.matmul(rot, vd).reshape(-1, 3)), dim=1)
            if self.use_code and self.use_code_viewdirs:
                feats = self.code(feats)
        mlp_input = feats
        if self.use_encoder:
            uv = -xyz[:, :, :2] / xyz[:, :, 2:]
            uv = uv * repeat_interleave(self.focal.unsqueeze(1), NS if self.focal.shape[0] > 1 else 1)
            uv = uv + repeat_interleave(self.c.unsqueeze(1), NS if self.c.shape[0] > 1 else 1)
            lat = self.encoder.index(uv, None, self.image_shape)     # (SB NS, C, B)
            if self.stop_encoder_grad:
                lat = lat.detach()
            lat = lat.transpose(1, 2).reshape(-1, self.latent_size)
            mlp_input = lat if feats is None else torch.cat((lat, feats), dim=-1)
        if self.use_global_encoder:
            gl = self.global_encoder.latent
            gl = repeat_interleave(gl, mlp_input.shape[0] // gl.shape[0])
            mlp_input = torch.cat((gl, mlp_input), dim=-1)
        mlp = self.mlp_coarse if (coarse or self.mlp_fine is None) else self.mlp_fine
        out = mlp(mlp_input, combine_inner_dims=(NS, B)).reshape(-1, B, self.d_out)
        return torch.cat((torch.sigmoid(out[..., :3]), torch.relu(out[..., 3:4])), dim=-1).reshape(SB, B, -1)

    # ---- checkpoints (models.py:268-316) -------------------------------------------
    def load_weights(self, args, opt_init=False, strict=True, device=None):
        if opt_init and not args.resume:
            return
        ckpt_name = "pixel_nerf_init" if opt_init or not args.resume else "pixel_nerf_latest"
        model_path = "%s/%s/%s" % (args.checkpoints_path, args.name, ckpt_name)
        if device is None:
            device = self.poses.device
        if os.path.exists(model_path):
            print("Load", model_path)
            self.load_state_dict(torch.load(model_path, map_location=device, weights_only=True),
                                 strict=strict)
        elif not opt_init:
            warnings.warn("WARNING: {} does not exist, not loaded!! Model will be "
                          "re-initialized.".format(model_path))
        return self

    def save_weights(self, args, opt_init=False):
        from shutil import copyfile

        ckpt_name = "pixel_nerf_init" if opt_init else "pixel_nerf_latest"
        backup_name = "pixel_nerf_init_backup" if opt_init else "pixel_nerf_backup"
        ckpt_path = osp.join(args.checkpoints_path, args.name, ckpt_name)
        ckpt_backup_path = osp.join(args.checkpoints_path, args.name, backup_name)
        if osp.exists(ckpt_path):
            copyfile(ckpt_path, ckpt_backup_path)
        torch.save(self.state_dict(), ckpt_path)
        return self


def make_model(conf, *args, **kwargs):
    """model/__init__.py:4-11."""
    conf = as_conf(conf)
    model_type = conf.get_string("type", "pixelnerf")
    if model_type == "pixelnerf":
        return PixelNeRFNet(conf, *args, **kwargs)
    raise NotImplementedError("Unsupported model type", model_type)
