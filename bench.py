#!/usr/bin/env python
"""Benchmark: pixelNeRF coarse + fine ray march (64 + 64 samples) on MI355X.

Workload (BASELINE.json configs[1], "cfg2"): SRN-cars 128x128 frame, 1 source
view, rendered as 4096-ray chunks x (64 coarse + 64 fine), fp32.  One step =
one full 128x128 frame (16,384 rays = 4 chunks) through
``render_par(rays[None])`` exactly as eval/gen_video.py:213-217 drives it.
Inputs are synthetic (hash-initialised MLP weights and latent) and
already resident in HBM when the timed region starts.

Multi-GPU (launched by torch.distributed.run): one process per GPU, every rank
renders its own frame (a different target pose) — weak scaling, no data-path
collective; a barrier + all_reduce(MAX) of the elapsed time bracket the region.

The MLP arithmetic is --precision (default f16x3: fp32-accurate GEMMs from split-fp16
products, include/pnr_abi.h); `dtype` stays "f32" (fp32 in / out / accumulation).

The JSON line also carries
  roofline     — the dominant kernel (fine-pass fused point MLP, k_point_mlp):
                 algorithmic fp32 FLOP per launch / its average duration measured with
                 HIP events recorded on the launch stream inside the timed region,
                 against the precision's fp32-equivalent MFMA peak (f16x3: 2500 / 3),
                 plus the raw MFMA issue rate; `traffic` from the committed PMC pass;
  composite    — the standalone alpha-composite kernel's HBM roofline (bytes per
                 ray x rays / duration vs 8 TB/s) on a 1 M-ray batch;
  extra_configs — cfg2 with the shipped conf, cfg3 (NMR 64x64) and cfg4 (DTU, 3 source
                 views) on 1 GPU (informational; skip with --no-extra);
  value_fp32_mfma — the same frame with the plain f32-MFMA arithmetic;
  cpu_baseline — the CPU oracle (oracle/ref_cpu.py, a restatement of the
                 reference's PyTorch path) on a bounded sample of the same frame,
                 timed on this host, rank 0 at N = 1 only;
  psnr_vs_reference_path — SURVEY §8(d)'s PSNR delta: the HIP render of that sample
                 with the same injected random streams against the oracle's render.
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pnr import _lib, synth, util  # noqa: E402
from pnr import dist as pdist  # noqa: E402
from pnr.models import PRECISIONS, PixelNeRFNet  # noqa: E402
from pnr.renderer import NeRFRenderer  # noqa: E402

MFMA_F32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: Peak FP32 (matrix)
MFMA_BF16_PEAK_TFLOPS = 2500.0 # MI355X_MICROARCH.md: Peak BF16 MFMA, dense
# fp32-equivalent peak of each ResnetFC arithmetic mode (pnr.models.PRECISIONS): the
# split modes issue 6 / 9 bf16 MFMA products per fp32 multiply-add
PEAK_BY_PRECISION = {"fp32": (MFMA_F32_PEAK_TFLOPS, 1), "f16x3": (MFMA_BF16_PEAK_TFLOPS / 3, 3),
                     "bf16x6": (MFMA_BF16_PEAK_TFLOPS / 6, 6),
                     "bf16x9": (MFMA_BF16_PEAK_TFLOPS / 9, 9)}
ARITHMETIC = {
    "fp32": "v_mfma_f32_16x16x4_f32 (fp32 products, fp32 accumulate)",
    "bf16x6": "exact 3-way bf16 split of both fp32 operands, 6 largest products on "
              "v_mfma_f32_16x16x32_bf16, fp32 accumulate (error at fp32 unit roundoff; "
              "profiles/r1/precision_study.json)",
    "bf16x9": "exact 3-way bf16 split, all 9 products (exact), fp32 accumulate",
    "f16x3": "power-of-two scaled operands split into two fp16 parts, 3 exact products on "
             "v_mfma_f32_16x16x32_f16 (f16 MFMA rate = bf16 rate), fp32 accumulate "
             "(error at the fp32 level; profiles/*/precision_study.json)",
}
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E peak (spec)
FLOP_PER_POINT_NS1 = 4761600 + 2101248   # NS*4,761,600 + 2,101,248
# FLOP the fused kernel executes per point with the projected latent (lin_z folded into the
# latent per scene): lin_in + 5 blocks x (fc_0 + fc_1) + lin_out
KERNEL_FLOP_PER_POINT_NS1 = 2 * 42 * 512 + 5 * 2 * 2 * 512 * 512 + 2 * 512 * 4   # 5,289,984
PROJ_FLOP_PER_SCENE = 2 * 3 * 64 * 64 * 512 * 512   # 3 lin_z layers x 4096 latent pixels
KC, KF = 64, 64
CHUNK = 4096
W = H = 128


def model_conf():
    mlp = dict(type="resnet", n_blocks=5, d_hidden=512, combine_layer=3, combine_type="average")
    return dict(use_encoder=True, use_xyz=True, use_code=True,
                code=dict(num_freqs=6, freq_factor=1.5, include_input=True), use_viewdirs=True,
                use_code_viewdirs=False, mlp_coarse=mlp, mlp_fine=mlp,
                encoder=dict(backbone="resnet34", pretrained=False, num_layers=4))


class HipEvents:
    """hipEvent_t handles from the HIP runtime torch already loaded."""

    def __init__(self):
        self.hip = ctypes.CDLL("libamdhip64.so.7")
        self.hip.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        self.hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p,
                                                 ctypes.c_void_p]
        self.hip.hipEventDestroy.argtypes = [ctypes.c_void_p]

    def create(self, n):
        evs = []
        for _ in range(n):
            e = ctypes.c_void_p()
            assert self.hip.hipEventCreate(ctypes.byref(e)) == 0
            evs.append(e)
        return evs

    def elapsed_ms(self, a, b):
        ms = ctypes.c_float()
        rc = self.hip.hipEventElapsedTime(ctypes.byref(ms), a, b)
        assert rc == 0, rc
        return ms.value


def build_scene(dev, rank):
    sd = synth.pixelnerf_state(1)
    net = PixelNeRFNet(model_conf())
    net.load_state_dict(sd, strict=False)
    net = net.to(dev).eval()
    lat = synth.latent(0, 1, 512, 64, 64).to(dev)
    net.encode_latent(lat, synth.srn_poses([0.0]).to(dev), torch.tensor(131.25, device=dev), (W, H))
    tgt = synth.srn_poses([30.0 + 15.0 * rank])
    rays = util.gen_rays(tgt, W, H, torch.tensor(131.25), 0.01, 4.0).reshape(-1, 8).to(dev)
    return sd, net, rays.contiguous()


def cpu_baseline(sd, rays_cpu, n_rays):
    """Oracle (CPU restatement of the reference path) on a bounded sample."""
    from oracle import ref_cpu

    torch.set_num_threads(min(16, os.cpu_count() or 1))
    scene = ref_cpu.Scene(synth.latent(0, 1, 512, 64, 64), synth.srn_poses([0.0]),
                          torch.tensor(131.25), W, H, None)
    rays = rays_cpu[:n_rays][None].contiguous()
    streams = synth.rng_streams(2, n_rays, KC, KF, 0)
    fn = lambda p, c, d: ref_cpu.pixelnerf_forward(sd, scene, p, c, d)  # noqa: E731
    with torch.no_grad():
        ref_cpu.render(fn, rays[:, :8], KC, KF, 0, tuple(s[:8] for s in streams), True)  # warm-up
        t0 = time.perf_counter()
        ref = ref_cpu.render(fn, rays, KC, KF, 0, streams, True)
        dt = time.perf_counter() - t0
    return dict(value=round(n_rays / dt, 2), unit="rays/s", cores=torch.get_num_threads(),
                kind="port",
                sample="%d rays of the cfg2 frame x (64+64) samples, oracle/ref_cpu.py, %.1f s" % (
                    n_rays, dt)), ref, streams


def psnr_vs_reference_path(net, rays_dev, ref, streams, dev):
    """SURVEY §8(d)'s PSNR delta: the HIP render of the cpu_baseline rays with the SAME
    injected random streams, against the oracle's render of them (oracle/ref_cpu.py, the
    CPU restatement pinned to the reference).  `agreement_db` = PSNR(HIP, oracle);
    `delta_db` = PSNR(HIP, target) - PSNR(oracle, target) for a seeded U(0,1) target image
    (no ground-truth frames offline).  Fine-pass rays are excluded from the `_excl_flips`
    figures only for a searchsorted bin flip PROVEN from the two sets of coarse weights
    (oracle/parity.py); `unexplained_rays` (fine samples that differ without one) must be 0."""
    from oracle import parity

    n = rays_dev.shape[0]
    r = NeRFRenderer(n_coarse=KC, n_fine=KF, n_fine_depth=0, white_bkgd=True).to(dev)
    r.streams = tuple(t.to(dev) for t in streams)
    r.return_z = True
    with torch.no_grad():
        out = r(net, rays_dev[None].contiguous(), want_weights=True)
    tgt = torch.from_numpy(synth.hash_uniform(5, n * 3).astype("float32")).reshape(n, 3)
    cls = parity.classify_fine(out.coarse.weights[0], ref["coarse"]["weights"][0], streams[1],
                               out.fine.z[0], ref["fine"]["z"])

    def psnr(a, b):   # util.psnr (util.py:474-481), +inf for identical images
        return float("inf") if float(((a - b) ** 2).mean()) == 0.0 else float(util.psnr(a, b))

    res = {}
    for name in ("coarse", "fine"):
        mine = getattr(out, name).rgb[0].float().cpu()
        theirs = ref[name]["rgb"][0].float()
        agree = psnr(mine, theirs)
        flip = cls["flip"] if name == "fine" else torch.zeros(n, dtype=torch.bool)
        keep = ~flip
        agree_kept = psnr(mine[keep], theirs[keep]) if bool(keep.any()) else float("inf")
        d = (mine - theirs).abs()
        res[name] = dict(agreement_db=round(agree, 2) if agree < float("inf") else None,
                         delta_db=round(psnr(mine, tgt) - psnr(theirs, tgt), 6),
                         max_abs_rgb=float(d.max()),
                         bin_flip_rays=int(flip.sum()),
                         agreement_db_excl_flips=round(agree_kept, 2) if agree_kept < float("inf") else None,
                         max_abs_rgb_excl_flips=float(d[keep].max()) if bool(keep.any()) else 0.0,
                         rays_outside_tol_excl_flips=int(((d > 5e-5 + 1e-5 * theirs.abs()).any(-1) & keep).sum()))
    res["fine"]["flip_rays"] = cls["flip_idx"][:16]
    res["fine"]["unexplained_rays"] = int(cls["unexplained"].sum())
    res["rays"] = n
    res["flip_rule"] = ("fine-bin flip = searchsorted bins recomputed from the HIP and the oracle "
                        "coarse weights with the same u differ (oracle/parity.py)")
    return res


def composite_roofline(dev, ev):
    """Standalone composite kernel on 1 M rays x 128 samples (HBM-bound)."""
    from pnr import ops

    B, K = 1 << 20, 128
    g = torch.Generator(device=dev).manual_seed(0)
    rays = torch.zeros(B, 8, device=dev)
    rays[:, 6] = 0.01
    rays[:, 7] = 4.0
    z = torch.sort(torch.rand(B, K, device=dev, generator=g) * 3.9 + 0.05, -1)[0]
    raw = torch.rand(B, K, 4, device=dev, generator=g)
    lib = _lib.load()
    rgb = torch.empty(B, 3, device=dev)
    depth = torch.empty(B, device=dev)
    w = torch.empty(B, K, device=dev)
    st = _lib.stream_of(dev)
    evs = ev.create(2)
    res = {}
    for want_w in (False, True):
        for _ in range(2):
            ops.composite(z, raw, rays, True, want_weights=want_w)
        times = []
        for _ in range(5):
            ev.hip.hipEventRecord(evs[0], st)
            _lib.check(lib.pnr_composite(_lib.ptr(z), _lib.ptr(raw), _lib.ptr(rays), B, K, 1,
                                         _lib.ptr(w) if want_w else None, _lib.ptr(rgb),
                                         _lib.ptr(depth), st), "pnr_composite")
            ev.hip.hipEventRecord(evs[1], st)
            torch.cuda.synchronize(dev)
            times.append(ev.elapsed_ms(evs[0], evs[1]))
        ms = sorted(times)[len(times) // 2]
        per_ray = 4 * K + 16 * K + 4 + 12 + 4 + (4 * K if want_w else 0)
        gbs = per_ray * B / (ms * 1e-3) / 1e9
        res["weights" if want_w else "no_weights"] = dict(
            ms=round(ms, 4), bytes_per_ray=per_ray, achieved=round(gbs, 1), peak=HBM_PEAK_GBS,
            unit="GB/s", frac=round(gbs / HBM_PEAK_GBS, 4))
    return res


def _time_render(net, renderer, rays, chunk, passes=2):
    """Seconds per pass over `rays` (N, 8) in `chunk`-ray render_par calls (warm, synced)."""
    render_par = renderer.bind_parallel(net, simple_output=True).eval()

    def once():
        net.drop_latent_proj()   # per-scene projection rebuilt in every timed pass
        for r in torch.split(rays, chunk, dim=0):
            render_par(r[None])

    with torch.no_grad():
        once()
        torch.cuda.synchronize(rays.device)
        t0 = time.perf_counter()
        for _ in range(passes):
            once()
        torch.cuda.synchronize(rays.device)
    return (time.perf_counter() - t0) / passes


def extra_configs(dev, precision, latent_proj=True):
    """The other SURVEY §8(d) workloads on 1 GPU (informational, not `value`):
    cfg2 with the shipped conf (64 + 32 incl. 16 depth samples), cfg3 NMR 64x64 (latent
    32x32, 24 frames x 4096 rays), cfg4 DTU 400x300 with NS = 3 source views (one 120,000-
    ray frame, the multi-view mean path), chunked as gen_video.py does (50,000 rays)."""
    res = {}
    sd = synth.pixelnerf_state(1)

    def make(latent, poses, focal, size, c=None, n_obj=1):
        net = PixelNeRFNet(model_conf())
        net.load_state_dict(sd, strict=False)
        net = net.to(dev).eval()
        net.mlp_precision = precision
        net.use_latent_proj = latent_proj
        net.encode_latent(latent.to(dev), poses.to(dev), focal.to(dev), size,
                          c=c.to(dev) if c is not None else None, num_objs=n_obj)
        return net

    # cfg2, shipped renderer conf
    net = make(synth.latent(0, 1, 512, 64, 64), synth.srn_poses([0.0]), torch.tensor(131.25), (W, H))
    rays = util.gen_rays(synth.srn_poses([30.0]).to(dev), W, H, torch.tensor(131.25), 0.01, 4.0).reshape(-1, 8)
    r = NeRFRenderer(n_coarse=64, n_fine=32, n_fine_depth=16, depth_std=0.01, white_bkgd=True).to(dev)
    s = _time_render(net, r, rays, CHUNK)
    res["cfg2_shipped_64_32_16"] = dict(rays_per_s=round(rays.shape[0] / s, 1), ms_per_frame=round(s * 1e3, 3),
                                        gflop_per_ray=round(160 * FLOP_PER_POINT_NS1 / 1e9, 4))
    # cfg2 as eval_approx.py --coarse renders it: mlp_fine = None, 64 + 128 samples (the fine
    # pass reuses the coarse pass's outputs for the 64 coarse samples)
    net.mlp_fine = None
    r = NeRFRenderer(n_coarse=64, n_fine=128, white_bkgd=True).to(dev)
    s = _time_render(net, r, rays, CHUNK)
    res["cfg2_coarse_as_fine_64_128"] = dict(rays_per_s=round(rays.shape[0] / s, 1),
                                             ms_per_frame=round(s * 1e3, 3))
    # cfg3, NMR 64x64: 24 target views of one object
    net = make(synth.latent(3, 1, 512, 32, 32), synth.srn_poses([0.0], radius=2.7), torch.tensor(70.0), (64, 64))
    rays = util.gen_rays(synth.srn_poses([15.0 * i for i in range(24)], radius=2.7).to(dev), 64, 64,
                         torch.tensor(70.0), 1.2, 4.0).reshape(-1, 8)
    r = NeRFRenderer(n_coarse=64, n_fine=64, white_bkgd=True).to(dev)
    s = _time_render(net, r, rays, 16384)
    res["cfg3_nmr64_24frames"] = dict(rays_per_s=round(rays.shape[0] / s, 1), ms_per_batch=round(s * 1e3, 3),
                                      rays=int(rays.shape[0]))
    # cfg4, DTU 400x300, 3 source views
    sc = synth.scene_multiview(seed=8, n_views=3, n_rays=1)
    net = make(synth.latent(8, 3, 512, 150, 200), sc["poses"][None], sc["focal"][None], (400, 300),
               c=sc["c"][None])
    rays = util.gen_rays(synth.srn_poses([10.0], phi=-12.0, radius=2.0).to(dev), 400, 300, sc["focal"],
                         0.1, 5.0, c=sc["c"]).reshape(-1, 8)
    r = NeRFRenderer(n_coarse=64, n_fine=64, white_bkgd=False).to(dev)
    s = _time_render(net, r, rays, 50000, passes=1)
    res["cfg4_dtu_ns3_frame"] = dict(rays_per_s=round(rays.shape[0] / s, 1), ms_per_frame=round(s * 1e3, 3),
                                     gflop_per_ray=round(192 * (3 * 4761600 + 2101248) / 1e9, 4))
    return res


L2_PEAK_TBS = 34.5            # MI355X_MICROARCH.md, L2 (per XCD): ~34.5 TB/s aggregate
L2_GATHER_LOOP_TBS = 18.8     # same guide: a 64-row LDS gather loop from the XCD's L2 at <= 72 KiB in
                              # flight per CU reads 16.8-18.8 TB/s chip-wide (a lower bound)


def l2_stream(points, launch_ms, precision, latent_proj):
    """The fused MLP's second roofline: every 64-point tile streams the whole packed network
    from L2 (each CU reads each weight fragment once per tile) plus, with the projected
    latent, three 4-corner blends of 2 KB rows per point.  Bytes per launch / launch time
    against the guide's aggregate L2 rate (and, for scale, its measured gather-loop rate)."""
    if precision != "f16x3":
        return None
    tiles = (points + 63) // 64
    # packed 512x512 layers (10, or 13 with the per-point lin_z GEMMs), lin_in, lin_out
    weights = (10 if latent_proj else 13) * (1 << 20) + (128 << 10) + (32 << 10)
    gather = 3 * 64 * 4 * 2048   # 3 blends x 64 points x 4 corners x 2 KB rows (P or the latent)
    total = tiles * (weights + gather)
    tbs = total / (launch_ms * 1e-3) / 1e12
    return {"kernel": "k_point_mlp (fine pass)", "bytes_per_tile": weights + gather, "tiles": tiles,
            "achieved": round(tbs, 2), "peak": L2_PEAK_TBS, "unit": "TB/s (L2 -> CU)",
            "frac": round(tbs / L2_PEAK_TBS, 4),
            "frac_of_gather_loop": round(tbs / L2_GATHER_LOOP_TBS, 4),
            "note": "packed weight fragments per 64-point tile + 4-corner latent rows; peak is the "
                    "guide's aggregate L2 figure; frac_of_gather_loop compares with its measured "
                    "L2 gather loop (16.8-18.8 TB/s at <= 72 KiB in flight per CU)"}


def pmc_traffic(kernel, render_pass):
    """Mean HBM bytes per launch of `kernel` in `render_pass` ("fine" / "coarse") from the
    newest committed PMC summary that has it (rocprofv3 counters cannot be read live from
    inside the process).  Returns (bytes, summary path) or (None, None)."""
    import csv
    import glob

    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*", "pmc_summary.csv")), reverse=True):
        vals = []
        with open(path) as fh:
            rows = [f for f in csv.reader(l for l in fh if not l.startswith("#") and not l.startswith("kernel,"))]
        for f in rows:   # kernel names are quoted (they contain commas: k_point_mlp<3, true>)
            if f and f[0].endswith(kernel) and len(f) > 6 and f[6] == render_pass:
                vals.append(int(f[5]))
        if vals:
            return sum(vals) // len(vals), os.path.relpath(path, REPO)
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-rays", type=int, default=4096)   # ~13 s of oracle work on 16 cores
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-composite", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the cfg2-shipped / cfg3 / cfg4 lines")
    ap.add_argument("--no-compare", action="store_true",
                    help="skip the f32-MFMA comparison frame (profiling runs)")
    ap.add_argument("--precision", default="f16x3", choices=sorted(PEAK_BY_PRECISION))
    ap.add_argument("--no-latent-proj", action="store_true",
                    help="per-point lin_z GEMMs on the gathered latent (A/B against the projection)")
    args = ap.parse_args()

    rank, world, local = pdist.init_from_env("nccl")   # RCCL on ROCm; control plane only
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    sd, net, rays = build_scene(dev, rank)
    net.mlp_precision = args.precision
    net.use_latent_proj = not args.no_latent_proj
    renderer = NeRFRenderer(n_coarse=KC, n_fine=KF, n_fine_depth=0, white_bkgd=True,
                            eval_batch_size=CHUNK).to(dev)
    render_par = renderer.bind_parallel(net, [local], simple_output=True).eval()
    lib = _lib.load()
    chunks = list(torch.split(rays, CHUNK, dim=0))
    ev = HipEvents()

    # instrument the fused render: record events around every kernel of each chunk
    orig = lib.pnr_render_forward_proj
    pool = []
    recording = {"on": False}

    def render_with_events(*a):
        if not recording["on"]:
            return orig(*a)
        evs = ev.create(7)
        pool.append(evs)
        arr = (ctypes.c_void_p * 7)(*[e.value for e in evs])
        return orig(*a[:-1], arr)

    lib.pnr_render_forward_proj = render_with_events

    def step():
        # the per-scene latent projection (lin_z folded into the latent) is rebuilt inside
        # every timed frame: nothing beyond the encoder latent is carried across steps
        net.drop_latent_proj()
        frame = []
        for r in chunks:
            rgb, _depth = render_par(r[None])
            frame.append(rgb[0])
        return torch.cat(frame)

    torch.manual_seed(1234 + rank)
    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        recording["on"] = True
        t0 = time.perf_counter()
        for _ in range(args.steps):
            img = step()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        recording["on"] = False
        if world > 1:
            dist.barrier()
    elapsed = pdist.max_over_ranks(t1 - t0, device=dev)
    assert bool(torch.isfinite(img).all())

    # per-kernel durations from the events recorded in the timed region
    names = ["sample_coarse", "mlp_coarse", "composite_coarse", "sample_fine", "mlp_fine",
             "composite_fine"]
    per = {n: [] for n in names}
    for evs in pool:
        for i, n in enumerate(names):
            per[n].append(ev.elapsed_ms(evs[i], evs[i + 1]))
    avg = {n: sum(v) / len(v) for n, v in per.items()}
    pts_fine = CHUNK * (KC + KF)
    kflop = KERNEL_FLOP_PER_POINT_NS1 if net.use_latent_proj else FLOP_PER_POINT_NS1
    flop_fine = pts_fine * kflop
    achieved = flop_fine / (avg["mlp_fine"] * 1e-3) / 1e12
    ref_equiv = pts_fine * FLOP_PER_POINT_NS1 / (avg["mlp_fine"] * 1e-3) / 1e12
    peak, terms = PEAK_BY_PRECISION[args.precision]

    # same frame with the plain f32-MFMA arithmetic, for comparison (N = 1 only)
    value_fp32 = None
    if world == 1 and args.precision != "fp32" and not args.no_compare:
        net.mlp_precision = "fp32"
        with torch.no_grad():
            step()
            torch.cuda.synchronize(dev)
            t2 = time.perf_counter()
            for _ in range(2):
                step()
            torch.cuda.synchronize(dev)
            value_fp32 = round(2 * W * H / (time.perf_counter() - t2), 1)
        net.mlp_precision = args.precision

    prec_code = PRECISIONS[args.precision]
    kname = "k_point_mlp<%d, %s>" % (prec_code, "true" if net.use_latent_proj else "false")
    traffic, traffic_src = pmc_traffic(kname, "fine")
    rays_total = W * H * args.steps * world
    value = rays_total / elapsed
    out = {
        "metric": "rays/sec (coarse+fine, 64+64 samples)",
        "value": round(value, 1),
        "unit": "rays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "arithmetic": ARITHMETIC[args.precision],
        "value_fp32_mfma": value_fp32,
        "data": "synthetic (hash-initialised ResnetFC weights + latent; SRN geometry)",
        "config": {"workload": "cfg2: SRN-cars 128x128 frame, 1 source view, 4096-ray chunks x "
                               "(64 coarse + 64 fine)", "frame": [W, H], "chunk_rays": CHUNK,
                   "n_coarse": KC, "n_fine": KF, "n_views": 1, "rays_per_step_per_gpu": W * H,
                   "parallelism": "rays sharded by frame, 1 process per GPU"},
        "latent_proj": {"on": bool(net.use_latent_proj),
                        "flop_per_scene_per_mlp": PROJ_FLOP_PER_SCENE,
                        "note": "lin_z of every latent pixel (pnr_latent_project), rebuilt for both "
                                "MLPs inside every timed step; the kernel blends 4 projected rows per "
                                "point instead of 3 per-point 512x512 lin_z GEMMs"},
        "roofline": {"kernel": "k_point_mlp (fine pass)", "bound": "mfma",
                     "achieved": round(achieved, 2), "peak": round(peak, 1),
                     "unit": "TFLOP/s (fp32-equivalent: the kernel's algorithmic FLOP per launch / "
                             "launch time; %d FLOP per point)" % kflop,
                     "reference_equivalent_tflops": round(ref_equiv, 2),
                     "frac": round(achieved / peak, 4),
                     "mfma_issue": {"tflops": round(achieved * terms, 1),
                                    "peak": MFMA_F32_PEAK_TFLOPS if terms == 1 else MFMA_BF16_PEAK_TFLOPS,
                                    "products_per_fma": terms},
                     "traffic": traffic,
                     "traffic_source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this "
                                       "bench, fine-pass launches of %s (%s, FETCH x2 "
                                       "gfx950 correction)" % (kname, traffic_src),
                     "flop_per_launch": flop_fine,
                     "launch_ms": round(avg["mlp_fine"], 4)},
        "kernel_ms": {n: round(v, 4) for n, v in avg.items()},
        "l2_stream": l2_stream(pts_fine, avg["mlp_fine"], args.precision, net.use_latent_proj),
    }
    if rank == 0 and world == 1 and not args.no_composite:
        out["composite"] = composite_roofline(dev, ev)
    if rank == 0 and world == 1 and not args.no_extra:
        out["extra_configs"] = extra_configs(dev, args.precision, not args.no_latent_proj)
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"], ref, streams = cpu_baseline(sd, rays.cpu(), args.cpu_rays)
        out["psnr_vs_reference_path"] = psnr_vs_reference_path(net, rays[:args.cpu_rays], ref, streams, dev)
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
