"""Train-mode BatchNorm(+residual add)(+ReLU) kernels (csrc/bn.hip, ``pnr.encoder.BatchNormTrain``)
against torch's nn.BatchNorm2d + add + relu in fp32 on the same device (``-m gpu``).

The trunk's training-mode layers (encoder.py:135-149 over torchvision's BasicBlock): forward
output, running mean / variance (momentum, unbiased variance), num_batches_tracked, and the
gradients of the map, the residual, gamma and beta.  Tolerance: fp32 rounding of the
normalisation (torch reduces in fp32 Welford, the kernels in double): outputs within 2e-5 of
their max-abs or of gamma invstd |y| (the conditioning of y - mean in fp32), gradients within 1e-4
of their max-abs (dy: of its terms' scale gamma invstd |dz|), running statistics within 1e-5.
"""
import copy

import pytest
import torch
from torch import nn

from pnr import encoder as pe

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


@pytest.mark.parametrize("shape", [(4, 64, 64, 64), (4, 128, 16, 16), (3, 256, 7, 9), (2, 64, 1, 1), (2, 512, 4, 4)])
@pytest.mark.parametrize("relu,add", [(True, False), (True, True), (False, False)])
def test_fused_batchnorm_matches_torch(shape, relu, add):
    g = torch.Generator().manual_seed(sum(shape) + 2 * relu + add)
    n, c, h, w = shape
    y0 = (torch.randn(shape, generator=g) * 1.7 + 0.4).to(DEV).contiguous(memory_format=torch.channels_last)
    i0 = torch.randn(shape, generator=g).to(DEV).contiguous(memory_format=torch.channels_last) if add else None
    bn = nn.BatchNorm2d(c).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(c, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(c, generator=g) * 0.3)
        bn.running_mean.copy_(torch.randn(c, generator=g))
        bn.running_var.copy_(torch.rand(c, generator=g) + 0.5)
        bn.num_batches_tracked.fill_(7)
    ref = copy.deepcopy(bn)
    assert pe._fused_bn_ok(bn, y0, i0)

    y = y0.clone().requires_grad_(True)
    idt = i0.clone().requires_grad_(True) if add else None
    out = pe.BatchNormTrain.apply(y, idt, bn.weight, bn.bias, bn, relu)
    yr = y0.clone().requires_grad_(True)
    ir = i0.clone().requires_grad_(True) if add else None
    o = ref(yr)
    if add:
        o = o + ir
    outr = torch.relu(o) if relu else o
    assert out.is_contiguous(memory_format=torch.channels_last)
    # fp32 conditioning of the normalisation: y - mean rounds at the scale of |y|, so the output
    # error scales with gamma invstd |y| (large at M = 2 where the two values of a channel are close)
    var = y0.double().var(dim=(0, 2, 3), unbiased=False)
    gis = (bn.weight.double().abs() / (var + bn.eps).sqrt()).max().item()
    assert (out - outr).abs().max().item() < 2e-5 * max(outr.abs().max().item(), gis * y0.abs().max().item())
    assert _rel(bn.running_mean, ref.running_mean) < 1e-5
    assert _rel(bn.running_var, ref.running_var) < 1e-5
    assert int(bn.num_batches_tracked) == int(ref.num_batches_tracked) == 8

    dout = torch.randn(shape, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
    out.backward(dout)
    outr.backward(dout)
    # dy is a difference of terms of size gamma invstd |dz|: measured against that scale (at M = 2
    # the exact dy is 0 and both sides are rounding noise of it)
    term = gis * dout.abs().max().item()
    # ... plus x_hat's own rounding, amplified by invstd |y| (y - mean at the scale of |y|): large
    # only when a channel's values nearly coincide (M = 2)
    cond = (y0.abs().max().double() / (var + bn.eps).sqrt().min()).item()
    tol = 1e-4 + 64 * 2.0 ** -24 * cond
    assert (y.grad - yr.grad).abs().max().item() < tol * max(yr.grad.abs().max().item(), term)
    assert _rel(bn.weight.grad, ref.weight.grad) < 1e-4
    assert _rel(bn.bias.grad, ref.bias.grad) < 1e-4
    if add:
        assert torch.equal(idt.grad, ir.grad) or _rel(idt.grad, ir.grad) < 1e-6


def test_fused_batchnorm_without_running_stats():
    c = 64
    y0 = torch.randn(2, c, 8, 8, device=DEV).contiguous(memory_format=torch.channels_last)
    bn = nn.BatchNorm2d(c, track_running_stats=False).to(DEV)
    out = pe.BatchNormTrain.apply(y0, None, bn.weight, bn.bias, bn, True)
    assert _rel(out, torch.relu(bn(y0))) < 2e-5


def test_fused_batchnorm_refuses_what_it_does_not_implement():
    bn = nn.BatchNorm2d(96).to(DEV)   # 96 / 4 = 24 does not divide 256
    y = torch.randn(2, 96, 4, 4, device=DEV).contiguous(memory_format=torch.channels_last)
    assert not pe._fused_bn_ok(bn, y, None)
    assert not pe._fused_bn_ok(nn.BatchNorm2d(64).to(DEV).eval(), y[:, :64].contiguous(
        memory_format=torch.channels_last), None)
    assert not pe._fused_bn_ok(nn.BatchNorm2d(64, momentum=None).to(DEV), y[:, :64].contiguous(
        memory_format=torch.channels_last), None)
    assert not pe._fused_bn_ok(nn.BatchNorm2d(64).to(DEV), y[:, :64].contiguous(), None)   # NCHW (4 x 4 maps)
    # the ABI refuses a channel count it cannot tile, loudly
    with pytest.raises(RuntimeError, match="batchnorm"):
        pe.BatchNormTrain.apply(y, None, bn.weight, bn.bias, bn, True)


def test_train_mode_encoder_fused_matches_unfused(monkeypatch):
    """The whole trunk in training mode (encode + backward through the latent) with the fused
    kernels and with torch's modules: the same latent, running statistics and gradients."""
    torch.manual_seed(5)
    enc = pe.SpatialEncoder(pretrained=False).to(DEV).train()
    twin = copy.deepcopy(enc)
    x = torch.rand(4, 3, 128, 128, device=DEV) * 2 - 1
    calls = []
    orig = pe.BatchNormTrain.forward

    def counted(ctx, *a):
        calls.append(1)
        return orig(ctx, *a)

    monkeypatch.setattr(pe.BatchNormTrain, "forward", staticmethod(counted))
    lat = enc(x)
    n_bn = sum(isinstance(m, nn.BatchNorm2d) for m in enc.model.modules()) - 2 * 3 - 1   # layer4 unused
    assert len(calls) == n_bn
    monkeypatch.setattr(pe, "FUSED_TRAIN_BN", False)
    latr = twin(x)
    assert _rel(lat, latr) < 1e-4
    g = torch.randn_like(lat)
    lat.backward(g)
    latr.backward(g)
    for (name, p), (_, pr) in zip(enc.named_parameters(), twin.named_parameters()):
        if pr.grad is None:
            assert p.grad is None, name
            continue
        assert _rel(p.grad, pr.grad) < 2e-3, name
    for (name, b), (_, br) in zip(enc.model.named_buffers(), twin.model.named_buffers()):
        if b.dtype == torch.int64:
            assert torch.equal(b, br), name
        else:
            assert _rel(b, br) < 1e-4, name
