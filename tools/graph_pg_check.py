"""Diagnostic (GPU): the eval encode's HIP graph capture (pnr.encoder.InferenceTrunk) with an RCCL
process group alive in the process (world size 1, one all-reduce issued first so that its watchdog
has work), as every bench.py rank at N > 1 has.  Prints the capture state and the latent's
difference from the module path.   python tools/graph_pg_check.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pixel-nerf_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pnr.encoder import SpatialEncoder  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1)
t = torch.ones(4, device=dev)
dist.all_reduce(t)
torch.manual_seed(0)
enc = SpatialEncoder(pretrained=False).to(dev).eval()
img = torch.rand(1, 3, 64, 64, device=dev) * 2 - 1
with torch.no_grad():
    enc.infer_fast = False
    ref = enc(img).clone()
    enc.infer_fast = True
    for _ in range(3):
        got = enc(img).clone()
    dist.all_reduce(t)
torch.cuda.synchronize()
print("graph used:", enc._infer.use_graph, "graphs:", len(enc._infer.graphs),
      "max|d| vs module path: %.3g (scale %.3g)" % ((got - ref).abs().max().item(), ref.abs().max().item()))
dist.destroy_process_group()
