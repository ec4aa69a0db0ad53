"""Diagnostic (GPU): the cfg3 eval encode (bench.py's per-step net.encode: 1 NMR 64x64 source
image, use_first_pool=False) in three forms, alternating, HIP events around 50 encodes each:
    module   the module's conv / BN / relu launches (net.encoder.infer_fast = False)
    folded   InferenceTrunk, BN folded, F.conv2d + in-place relu / add, one HIP graph
    fused    InferenceTrunk with MIOpen's fused conv + bias (+ add) + relu ops, one HIP graph
each in NCHW and in channels-last (NHWC) memory format (trunk weights and input image), and each
form's latent against the module's.   python tools/encode_ab.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402
from pnr.encoder import InferenceTrunk  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
torch.backends.cudnn.benchmark = True
torch.manual_seed(0)
net = bench.make_net(dev, "f16x3", True, use_first_pool=False)
img, src, focal, _ = bench.nmr_inputs(dev)


def setup(form, cl):
    net.encoder.infer_fast = form != "module"
    net.encoder._infer = None
    InferenceTrunk.fused = form == "fused"
    net.encoder.model.to(memory_format=torch.channels_last if cl else torch.contiguous_format)


def time_form(form, cl, n=50):
    setup(form, cl)
    x = img.contiguous(memory_format=torch.channels_last) if cl else img
    with torch.no_grad():
        for _ in range(5):
            net.encode(x, src, focal)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            net.encode(x, src, focal)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n, net.encoder.latent_cl.clone()


ref = None
for rnd in range(2):
    for form in ("module", "folded", "fused"):
        for cl in (False, True):
            ms, lat = time_form(form, cl)
            if ref is None:
                ref = lat
            d = (lat - ref).abs().max().item() / ref.abs().max().item()
            used = net.encoder._infer
            print("%-7s %-4s %.4f ms per encode   max|d| / max|ref| %.2e   graph %s fused %s" % (
                form, "nhwc" if cl else "nchw", ms, d, used is not None and used.use_graph and bool(used.graphs),
                used is not None and used.fused), flush=True)
