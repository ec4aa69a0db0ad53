"""Profiler ranges with the reference's names (nerf.py:175, 264, models.py:156,
encoder.py:90, resnetfc.py:54, 139, code.py:36) around the same calls, on the host path
(the callback modules run on the CPU)."""
import pytest
import torch

from pnr.encoder import SpatialEncoder
from pnr.models import PositionalEncoding, ResnetFC


def _names(fn):
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        fn()
    return {e.name for e in prof.events()}


def test_reference_range_names():
    pe = PositionalEncoding(6, 3, 1.5, True)
    mlp = ResnetFC(d_in=42, d_out=4, n_blocks=2, d_latent=8, d_hidden=16, combine_layer=1)
    enc = SpatialEncoder(pretrained=False)
    enc.set_latent(torch.rand(1, 512, 4, 4))
    with torch.no_grad():
        names = _names(lambda: (pe(torch.rand(5, 3)), mlp(torch.rand(5, 50)),
                                enc.index(torch.rand(1, 5, 2), image_size=torch.tensor([8.0, 8.0]))))
    for n in ("positional_enc", "resnetfc_infer", "resblock", "encoder_index"):
        assert n in names, (n, sorted(names)[:40])


@pytest.mark.gpu
def test_renderer_ranges_on_the_callback_path():
    """NeRFRenderer.forward / composite keep the reference's range names (renderer_forward,
    renderer_composite) on the callback path a plain model takes (its sampling and composite
    are HIP kernels: GPU)."""
    from pnr.renderer import NeRFRenderer

    class Plain(torch.nn.Module):
        use_viewdirs = True

        def forward(self, xyz, coarse=True, viewdirs=None):
            return torch.cat([torch.sigmoid(xyz), torch.relu(xyz[..., :1])], -1).contiguous()

    r = NeRFRenderer(n_coarse=8, n_fine=0).cuda()
    rays = torch.cat([torch.zeros(1, 4, 3), torch.tensor([0.0, 0.0, 1.0]).expand(1, 4, 3),
                      torch.full((1, 4, 1), 0.5), torch.full((1, 4, 1), 2.0)], -1).cuda()
    with torch.no_grad():
        names = _names(lambda: r(Plain(), rays))
    assert "renderer_forward" in names and "renderer_composite" in names
