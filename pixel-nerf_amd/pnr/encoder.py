"""Image encoder that produces the latent the ray march gathers from.

Mirrors the interface of the reference's ``SpatialEncoder`` (encoder.py:13-177):
a ResNet34 trunk (conv1 .. layer3 used; layer4 present for checkpoint
compatibility), every stage upsampled to the conv1 resolution and concatenated
into a 512-channel feature map (``num_layers = 4``).  The trunk is defined here
with torchvision-compatible parameter names (``encoder.model.layer1.0.conv1.weight``
...) because torchvision is absent offline; it runs on PyTorch-ROCm (MIOpen) once
per scene and is not part of the per-ray hot path.

The hot path consumes the latent channels-LAST; ``latent_cl`` keeps that copy.
"""
import ctypes
import warnings
import weakref

import torch
import torch.nn.functional as F
from torch import nn

from .consts import device_const
from .prof import ranged

__all__ = ["SpatialEncoder", "ImageEncoder", "resnet34_trunk"]


def _nhwc(maps):
    """Every map channels-last in memory (the trunk's convolutions in channels-last format)."""
    return all(t.is_contiguous(memory_format=torch.channels_last) and not t.is_contiguous() for t in maps)


def _latent_channels_last(maps):
    from . import _lib

    maps = [t.float() for t in maps]
    nhwc = _nhwc(maps)
    if not nhwc:
        maps = [t.contiguous() for t in maps]
    n, (h, w) = maps[0].shape[0], maps[0].shape[-2:]
    c_total = sum(t.shape[1] for t in maps)
    out = torch.empty(n, h, w, c_total, dtype=torch.float32, device=maps[0].device)
    k = len(maps)
    ptrs = (ctypes.c_void_p * k)(*[t.data_ptr() for t in maps])
    ch = (ctypes.c_int32 * k)(*[t.shape[1] for t in maps])
    hs = (ctypes.c_int32 * k)(*[t.shape[2] for t in maps])
    ws = (ctypes.c_int32 * k)(*[t.shape[3] for t in maps])
    name = "pnr_latent_channels_last_nhwc" if nhwc else "pnr_latent_channels_last"
    _lib.check(getattr(_lib.load(), name)(ptrs, ch, hs, ws, k, n, _lib.ptr(out), h, w, _lib.stream_of(out.device)),
               name)
    return out


class LatentChannelsLast(torch.autograd.Function):
    """(n, h, w, sum C_i) = cat_i(upsample_bilinear_align_corners(map_i, (h, w))) channels-last
    (encoder.py:150-160) in one HIP kernel; the backward is each map's bilinear-upsample
    adjoint on its channel slice of the incoming gradient (what autograd of F.interpolate +
    torch.cat runs)."""

    @staticmethod
    def forward(ctx, *maps):
        ctx.shapes = [tuple(t.shape) for t in maps]
        ctx.nhwc = _nhwc(maps)
        return _latent_channels_last(maps)

    @staticmethod
    def backward(ctx, g):
        if g.is_cuda and ctx.nhwc and g.dtype == torch.float32:
            # channels-last maps (the trunk's layout): pnr_latent_channels_last_backward, one
            # deterministic gather launch for every map
            from . import _lib

            g = g.contiguous()
            n, h, w = g.shape[:3]
            grads = [torch.empty(shp, dtype=torch.float32, device=g.device, memory_format=torch.channels_last)
                     for shp in ctx.shapes]
            k = len(grads)
            ptrs = (ctypes.c_void_p * k)(*[t.data_ptr() for t in grads])
            ch = (ctypes.c_int32 * k)(*[s[1] for s in ctx.shapes])
            hs = (ctypes.c_int32 * k)(*[s[2] for s in ctx.shapes])
            ws = (ctypes.c_int32 * k)(*[s[3] for s in ctx.shapes])
            _lib.check(_lib.load().pnr_latent_channels_last_backward(
                _lib.ptr(g), ptrs, ch, hs, ws, k, n, h, w, _lib.stream_of(g.device)),
                "pnr_latent_channels_last_backward")
            return tuple(grads)
        gn = g.permute(0, 3, 1, 2)   # NCHW view of the channels-last gradient
        h, w = gn.shape[-2:]
        grads, c0 = [], 0
        for shp in ctx.shapes:
            gi = gn[:, c0:c0 + shp[1]]
            c0 += shp[1]
            if tuple(shp[-2:]) == (h, w):
                # the map's own layout (a channels-last trunk's backward convolutions take NHWC)
                grads.append(gi.contiguous(memory_format=torch.channels_last if ctx.nhwc else torch.contiguous_format))
            else:
                grads.append(torch.ops.aten.upsample_bilinear2d_backward(
                    gi, [h, w], list(shp), True, None, None))
        return tuple(grads)


class _BnFold(ctypes.Structure):
    """include/pnr_abi.h pnr_bn_fold."""
    _fields_ = [("conv_w", ctypes.c_void_p), ("gamma", ctypes.c_void_p), ("beta", ctypes.c_void_p),
                ("mean", ctypes.c_void_p), ("var", ctypes.c_void_p), ("w_out", ctypes.c_void_p),
                ("b_out", ctypes.c_void_p), ("n_out", ctypes.c_int64), ("per_out", ctypes.c_int64),
                ("eps", ctypes.c_float), ("pad_", ctypes.c_int32)]


def _ptr(t):
    return None if t is None else t.data_ptr()


def _bn_foldable(module):
    """Every BatchNorm of ``module`` (itself included) is affine and tracks running statistics: the
    fold (k_fold_bn) reads all four tensors, and an eval-mode BatchNorm without running statistics
    normalizes by the batch's, which no fold represents -- such an encoder runs the module path."""
    for b in module.modules():
        if isinstance(b, nn.modules.batchnorm._BatchNorm) and (
                b.running_mean is None or b.running_var is None or b.weight is None or b.bias is None):
            return False
    return True


class InferenceTrunk:
    """The encoder trunk for rendering (eval mode, no autograd; encoder.py:135-164's forward with
    the BatchNorms on their running statistics, what gen_video.py / eval.py run after .eval()):

    * every BatchNorm is folded into the convolution before it, W' = W s and b' = beta - mu s with
      s = gamma / sqrt(var + eps) per output channel (the same affine map, one rounding apart), by
      ONE ``pnr_fold_batchnorm`` launch over all pairs at the head of every encode;
    * ReLUs and residual adds run in place;
    * the fold, the trunk and the channels-last latent kernel (``pnr_latent_channels_last``) are
      captured once per input shape as one HIP graph and replayed: the eval encode is ~140 small
      launches whose host-side issue, not their GPU time, sets its duration (the fixed per-rank
      cost at N = 8).

    Because the fold runs inside every replay from the live storage of the convolution weights and
    BatchNorm tensors, every in-place change is seen -- optimizer steps, ``load_state_dict``,
    ``p.data.copy_`` (which a tensor version counter does not record).  The (conv, bn) pairs and
    their storage pointers are re-read from the module on every encode: a replaced tensor
    (``load_state_dict(assign=True)``) or a swapped module rebuilds the fold table, and a changed
    shape drops the captured graphs.  ``SpatialEncoder.invalidate_inference_cache()`` drops
    everything explicitly."""

    def __init__(self, enc, device):
        self.owner = weakref.ref(enc)
        self.device = device
        self.key = None
        self.folded = []          # per pair position: (w', b')
        self.table = None         # device copy of the pnr_bn_fold records
        self.n_folds, self.max_elems = 0, 0
        self.graphs = {}          # (shape, dtype, strides) -> (graph, static input, static latent)
        self.use_graph = True

    def _pairs(self):
        m = self.owner().model
        self.layers = [m.layer1, m.layer2, m.layer3, m.layer4][:max(self.owner().num_layers - 1, 0)]
        pairs = [(m.conv1, m.bn1)]
        for layer in self.layers:
            for blk in layer:
                pairs += [(blk.conv1, blk.bn1), (blk.conv2, blk.bn2)]
                if blk.downsample is not None:
                    pairs.append((blk.downsample[0], blk.downsample[1]))
        return pairs

    def refresh(self):
        """Re-read the (conv, bn) pairs from the module; rebuild the fold table when any tensor
        object, storage or eps changed (~40 us of host work per encode)."""
        pairs = self._pairs()
        self.pairs = pairs
        key = tuple((id(c), _ptr(c.weight), _ptr(b.weight), _ptr(b.bias), _ptr(b.running_mean),
                     _ptr(b.running_var), float(b.eps)) for c, b in pairs)
        if key == self.key:
            return
        for i, (c, b) in enumerate(pairs):
            if not _bn_foldable(b):   # k_fold_bn reads mean / var / weight / bias
                raise ValueError("pnr: the folded trunk needs every BatchNorm2d affine with running "
                                 "statistics (%r)" % (b,))
            w = c.weight
            if w.dtype != torch.float32 or w.device != self.device or not (
                    w.is_contiguous() or w.is_contiguous(memory_format=torch.channels_last)):
                raise ValueError("pnr: encoder conv weights must be dense fp32 on %s" % self.device)
            if i >= len(self.folded) or self.folded[i][0].shape != w.shape or self.folded[i][0].stride() != w.stride():
                if i < len(self.folded):
                    self.folded[i] = None
                else:
                    self.folded.append(None)
                self.graphs.clear()   # the captured convolutions read the old buffers
            if self.folded[i] is None:
                self.folded[i] = (torch.empty_like(w), torch.empty(c.out_channels, device=self.device))
        del self.folded[len(pairs):]
        recs = (_BnFold * len(pairs))()
        for i, (c, b) in enumerate(pairs):
            w_out, b_out = self.folded[i]
            recs[i] = _BnFold(_ptr(c.weight), _ptr(b.weight), _ptr(b.bias), _ptr(b.running_mean), _ptr(b.running_var),
                              _ptr(w_out), _ptr(b_out), c.out_channels, c.weight[0].numel(), float(b.eps), 0)
        host = torch.frombuffer(bytearray(bytes(recs)), dtype=torch.uint8)
        if self.table is None or self.table.numel() != host.numel():
            self.table = torch.empty(host.numel(), dtype=torch.uint8, device=self.device)
            self.graphs.clear()   # the captured fold reads the old table
        self.table.copy_(host)    # stream-ordered before the next fold (a replay reads it in place)
        self.n_folds = len(pairs)
        self.max_elems = max(c.weight.numel() for c, _ in pairs)
        self.key = key

    def fold(self):
        from . import _lib

        _lib.check(_lib.load().pnr_fold_batchnorm(self.table.data_ptr(), self.n_folds, self.max_elems,
                                                  _lib.stream_of(self.device)), "pnr_fold_batchnorm")

    # conv + bias + relu and conv + bias + residual + relu as MIOpen's fused forward ops
    # (torch.miopen_convolution_relu / _add_relu); False: F.conv2d + in-place relu / add.
    # Off: on the channels-last trunk F.conv2d is fastest (cfg3 encode 0.51 ms against 0.58 ms
    # NCHW and 0.60 ms fused NCHW; the fused ops on NHWC take 44 ms, a fallback kernel:
    # profiles/r4k/encode_ab_cl.txt), so they are never used on channels-last input
    fused = False

    def trunk(self, x):
        enc = self.owner()
        m = enc.model
        f = {id(c): wb for (c, _), wb in zip(self.pairs, self.folded)}
        fused = self.fused
        self.fold()

        def conv(c, x, relu=True, add=None):
            w, b = f[id(c)]
            if fused and relu:
                if add is None:
                    return torch.miopen_convolution_relu(x, w, b, c.stride, c.padding, c.dilation, c.groups)
                return torch.miopen_convolution_add_relu(x, w, add, 1.0, b, c.stride, c.padding, c.dilation,
                                                         c.groups)
            y = F.conv2d(x, w, b, c.stride, c.padding, c.dilation, c.groups)
            if add is not None:
                y = y.add_(add)
            return torch.relu_(y) if relu else y

        fused = fused and not x.is_contiguous(memory_format=torch.channels_last)
        x = conv(m.conv1, x)
        maps = [x]
        if self.layers and enc.use_first_pool:
            x = m.maxpool(x)
        for layer in self.layers:
            for blk in layer:
                idt = x if blk.downsample is None else conv(blk.downsample[0], x, relu=False)
                x = conv(blk.conv2, conv(blk.conv1, x), add=idt)
            maps.append(x)
        return _latent_channels_last(maps)

    def _capture(self, x, key):
        xin = x.clone()
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):   # MIOpen solver search and allocator warm-up, outside the capture
            try:
                self.trunk(xin)
            except RuntimeError as e:   # a fused op MIOpen refuses for this shape: the unfused form
                if not self.fused:
                    raise
                warnings.warn("pnr: MIOpen fused conv+relu unavailable (%s); unfused convolutions" % e)
                self.fused = False
            self.trunk(xin)
        torch.cuda.current_stream(self.device).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        try:
            # thread_local: other threads' HIP calls (the RCCL process group's watchdog at N > 1)
            # do not invalidate this thread's capture
            with torch.cuda.graph(graph, capture_error_mode="thread_local"):
                out = self.trunk(xin)
        except RuntimeError as e:   # a library call that cannot be captured: eager launches from now on
            warnings.warn("pnr: encoder trunk graph capture failed (%s); eager launches" % e)
            self.use_graph = False
            return None
        self.graphs[key] = (graph, xin, out)
        return self.graphs[key]

    def run(self, x):
        """(NS, H_l, W_l, C) channels-last latent of images x (NS, 3, H, W)."""
        self.refresh()
        key = (tuple(x.shape), x.dtype, x.stride())
        g = self.graphs.get(key)
        if g is None and self.use_graph:
            g = self._capture(x, key)
        if g is None:
            return self.trunk(x)
        graph, xin, out = g
        xin.copy_(x)
        graph.replay()
        return out.clone()   # the graph's output buffer is rewritten by the next replay


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, norm_layer=nn.BatchNorm2d):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = norm_layer(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = norm_layer(planes)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + idt)


class ResNetTrunk(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), norm_layer=nn.BatchNorm2d):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = norm_layer(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make(64, layers[0], 1, norm_layer)
        self.layer2 = self._make(128, layers[1], 2, norm_layer)
        self.layer3 = self._make(256, layers[2], 2, norm_layer)
        self.layer4 = self._make(512, layers[3], 2, norm_layer)
        self.avgpool = nn.Sequential()
        self.fc = nn.Sequential()
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make(self, planes, blocks, stride, norm_layer):
        down = None
        if stride != 1 or self.inplanes != planes:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes, 1, stride, bias=False),
                                 norm_layer(planes))
        layers = [BasicBlock(self.inplanes, planes, stride, down, norm_layer)]
        self.inplanes = planes
        layers += [BasicBlock(planes, planes, norm_layer=norm_layer) for _ in range(1, blocks)]
        return nn.Sequential(*layers)


def resnet34_trunk(pretrained=False, norm_layer=nn.BatchNorm2d):
    if pretrained:
        warnings.warn("pnr: ImageNet ResNet34 weights cannot be downloaded offline; the "
                      "encoder starts from random init (load a pixelNeRF checkpoint instead)")
    return ResNetTrunk(norm_layer=norm_layer)


def _norm_layer(norm_type):
    if norm_type == "batch":
        return nn.BatchNorm2d
    if norm_type == "instance":
        return lambda c: nn.InstanceNorm2d(c, affine=False, track_running_stats=False)
    if norm_type == "group":
        return lambda c: nn.GroupNorm(32, c)
    raise NotImplementedError("normalization layer [%s] is not found" % norm_type)


class SpatialEncoder(nn.Module):
    """Pixel-aligned encoder (encoder.py:13-177)."""

    def __init__(self, backbone="resnet34", pretrained=True, num_layers=4, index_interp="bilinear",
                 index_padding="border", upsample_interp="bilinear", feature_scale=1.0,
                 use_first_pool=True, norm_type="batch"):
        super().__init__()
        if backbone != "resnet34":
            raise NotImplementedError("pnr SpatialEncoder implements backbone=resnet34 only")
        # index_interp / index_padding other than bilinear / border: the fused kernel's gather
        # does not implement them, so such models take the callback path (F.grid_sample in
        # index(), PixelNeRFNet.fused_conf_reason)
        self.feature_scale = feature_scale
        self.use_first_pool = use_first_pool
        # channels-last (NHWC) trunk: MIOpen's NHWC convolutions, without the NCHW<->NHWC
        # transposes it otherwise wraps around them; the eval encode 0.58 -> 0.51 ms (cfg3) and the
        # cfg5 training step 14.8 -> 14.4 ms (profiles/r4k).  Same parameters and state-dict values.
        self.model = resnet34_trunk(pretrained, _norm_layer(norm_type)).to(memory_format=torch.channels_last)
        self.latent_size = [0, 64, 128, 256, 512, 1024][num_layers]
        self.num_layers = num_layers
        self.index_interp = index_interp
        self.index_padding = index_padding
        self.upsample_interp = upsample_interp
        self.register_buffer("latent", torch.empty(1, 1, 1, 1), persistent=False)
        self.register_buffer("latent_scaling", torch.empty(2, dtype=torch.float32), persistent=False)
        # channels-last copy (NS, H_l, W_l, C) read by the HIP gather; a buffer so that
        # nn.DataParallel replicas get their own device copy
        self.register_buffer("latent_cl", torch.empty(0), persistent=False)
        # eval-mode encodes on the device run the folded, graph-replayed trunk (InferenceTrunk)
        self.infer_fast = True
        self._infer = None

    def invalidate_inference_cache(self):
        """Drop the eval-mode inference trunk (its fold table and captured HIP graphs); the next
        eval-mode encode rebuilds it from the module as it is then."""
        self._infer = None

    def __getstate__(self):
        # the inference trunk holds HIP graphs and a weak reference: never copied or pickled
        # (copy.deepcopy / pickle of an encoded model); a copy rebuilds its own on first use
        state = super().__getstate__().copy()
        state["_infer"] = None
        return state

    def set_latent(self, latent):
        """Install a feature map (NS, C, H_l, W_l) as forward() would (encoder.py:160-163)."""
        self.latent = latent
        ls = device_const((latent.shape[-1], latent.shape[-2]), latent.device)
        self.latent_scaling = ls / (ls - 1) * 2.0
        self.latent_cl = latent.permute(0, 2, 3, 1).contiguous()
        return latent

    def forward(self, x):
        if self.feature_scale != 1.0:
            x = F.interpolate(x, scale_factor=self.feature_scale,
                              mode="bilinear" if self.feature_scale > 1.0 else "area",
                              align_corners=True if self.feature_scale > 1.0 else None,
                              recompute_scale_factor=True)
        x = x.to(device=self.latent.device)
        if x.dim() == 4:   # the trunk's channels-last layout (a no-op for a channels-last input)
            x = x.contiguous(memory_format=torch.channels_last)
        if self._use_infer(x):
            return self.set_latent_cl(self._infer.run(x))
        m = self.model
        x = m.relu(m.bn1(m.conv1(x)))
        latents = [x]
        if self.num_layers > 1:
            if self.use_first_pool:
                x = m.maxpool(x)
            x = m.layer1(x)
            latents.append(x)
        if self.num_layers > 2:
            x = m.layer2(x)
            latents.append(x)
        if self.num_layers > 3:
            x = m.layer3(x)
            latents.append(x)
        if self.num_layers > 4:
            x = m.layer4(x)
            latents.append(x)
        if x.is_cuda and self.upsample_interp == "bilinear" and len(latents) <= 8:
            return self.set_latent_maps(latents)
        size = latents[0].shape[-2:]
        for i in range(len(latents)):
            latents[i] = F.interpolate(latents[i], size, mode=self.upsample_interp,
                                       align_corners=True)
        return self.set_latent(torch.cat(latents, dim=1))

    def _use_infer(self, x):
        """The eval-mode inference trunk (InferenceTrunk) applies: no autograd, module in eval
        mode (BatchNorm on its running statistics), BatchNorm layers, a HIP device, the
        bilinear channels-last latent."""
        if not (self.infer_fast and x.is_cuda and not self.training and not torch.is_grad_enabled()
                and self.upsample_interp == "bilinear" and isinstance(self.model.bn1, nn.BatchNorm2d)
                and _bn_foldable(self.model)):
            return False
        if self._infer is None or self._infer.device != x.device or self._infer.owner() is not self:
            self._infer = InferenceTrunk(self, x.device)
        return True

    def set_latent_cl(self, out):
        """Install a channels-last latent (NS, H_l, W_l, C) with its NCHW view."""
        h, w = out.shape[1], out.shape[2]
        self.latent = out.permute(0, 3, 1, 2)
        ls = device_const((w, h), out.device)
        self.latent_scaling = ls / (ls - 1) * 2.0
        self.latent_cl = out
        return self.latent

    def set_latent_maps(self, maps):
        """encoder.py:150-163 on the HIP device without the NCHW concat + transpose:
        ``pnr_latent_channels_last`` upsamples (bilinear, align_corners) and concatenates
        the trunk maps straight into the channels-last latent the ray march reads;
        ``latent`` is its NCHW view (no copy).  Under autograd the gradient flows back
        through each map's upsample adjoint (``LatentChannelsLast``)."""
        return self.set_latent_cl(LatentChannelsLast.apply(*maps))

    @ranged("encoder_index")
    def index(self, uv, cam_z=None, image_size=(), z_bounds=None):
        """Bilinear feature lookup at image points (encoder.py:80-109); utility only —
        the ray march does this gather inside the fused HIP kernel."""
        if uv.shape[0] == 1 and self.latent.shape[0] > 1:
            uv = uv.expand(self.latent.shape[0], -1, -1)
        if len(image_size) > 0:
            if len(image_size) == 1:
                image_size = (image_size, image_size)
            scale = self.latent_scaling / image_size
            uv = uv * scale - 1.0
        samples = F.grid_sample(self.latent, uv.unsqueeze(2), align_corners=True,
                                mode=self.index_interp, padding_mode=self.index_padding)
        return samples[:, :, :, 0]

    @classmethod
    def from_conf(cls, conf):
        return cls(conf.get_string("backbone"), pretrained=conf.get_bool("pretrained", True),
                   num_layers=conf.get_int("num_layers", 4),
                   index_interp=conf.get_string("index_interp", "bilinear"),
                   index_padding=conf.get_string("index_padding", "border"),
                   upsample_interp=conf.get_string("upsample_interp", "bilinear"),
                   feature_scale=conf.get_float("feature_scale", 1.0),
                   use_first_pool=conf.get_bool("use_first_pool", True))


class ImageEncoder(nn.Module):
    """Global image encoder (encoder.py:180-240): the ResNet34 trunk through layer4 and a global
    average pool, then ``fc`` to ``latent_size`` when that is not 512.  Its latent (B, L) is
    concatenated to every point's MLP input (models.py:229-235); models using it take the
    callback path (PixelNeRFNet.fused_conf_reason)."""

    def __init__(self, backbone="resnet34", pretrained=True, latent_size=128):
        super().__init__()
        if backbone != "resnet34":
            raise NotImplementedError("pnr ImageEncoder implements backbone=resnet34 only")
        self.model = resnet34_trunk(pretrained)
        self.model.avgpool = nn.AdaptiveAvgPool2d((1, 1))   # torchvision's; fc replaced as the reference does
        self.register_buffer("latent", torch.empty(1, 1), persistent=False)
        self.latent_size = latent_size
        if latent_size != 512:
            self.fc = nn.Linear(512, latent_size)

    def index(self, uv, cam_z=None, image_size=(), z_bounds=()):
        """(B, L, N): the global latent for each of uv's N points (uv only gives the shape)."""
        return self.latent.unsqueeze(-1).expand(-1, -1, uv.shape[1])

    def forward(self, x):
        x = x.to(device=self.latent.device)
        m = self.model
        x = m.maxpool(m.relu(m.bn1(m.conv1(x))))
        x = m.layer4(m.layer3(m.layer2(m.layer1(x))))
        x = torch.flatten(m.avgpool(x), 1)
        if self.latent_size != 512:
            x = self.fc(x)
        self.latent = x
        return self.latent

    @classmethod
    def from_conf(cls, conf):
        return cls(conf.get_string("backbone"), pretrained=conf.get_bool("pretrained", True),
                   latent_size=conf.get_int("latent_size", 128))
