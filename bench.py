#!/usr/bin/env python
"""Benchmark: pixelNeRF coarse + fine ray march (64 + 64 samples) on 1/2/4/8 MI355X.

Headline workload (`value`; BASELINE.json configs[2], SURVEY §8(d)/(e) "cfg3"): one
ShapeNet-NMR batch of 24 target frames x 64x64 = 98,304 rays, 1 source view, 64 coarse +
64 fine samples, STRONG scaling: the batch is fixed and each of the N ranks (one process
per GPU) takes its contiguous ray range (pnr.dist.shard_range; the reference scatters rays
the same way, nerf.py:367-371).  One step, per rank:
  * encode the source image (the ResNet34 trunk, use_first_pool=False as
    conf/exp/sn64.conf:4-8 sets it -> a 32x32 channels-last latent; models.py:89-144);
  * the per-scene latent projection of both MLPs (lin_z folded into the latent,
    pnr_latent_project) -- rebuilt every step, because the latent is new;
  * render the rank's rays through ``render_par(rays[None])`` in gen_video.py's
    ray_batch_size chunks of 50,000 (gen_video.py:213-217; args.py:19);
  * copy the rank's rgb to the host (the launcher assembles the frames).
No data-path collective: a barrier and an all_reduce(MAX) of the elapsed time bracket
the timed region.  `value` = 98,304 x steps / max-over-ranks time, the same config at
every N (N = 1 included), so the driver's SCALE runs compare with BENCH directly.

The MLP arithmetic is --precision (default f16x3: fp32-accurate GEMMs from split-fp16
products, include/pnr_abi.h); `dtype` stays "f32" (fp32 in / out / accumulation).
Inputs are synthetic (hash-initialised MLP weights, random-init encoder, hashed source
image), resident in HBM when the timed region starts.

The JSON line also carries
  roofline     -- the dominant kernel (fine-pass fused point MLP, k_point_mlp): its
                  algorithmic FLOP per launch / its mean launch duration, both from HIP
                  events recorded on the launch stream around every kernel inside the timed
                  region; `traffic` from the committed rocprofv3 PMC pass;
  train        -- cfg5 (BASELINE configs[4]): the training step (encoder, coarse + fine
                  render, backward, bucketed RCCL gradient all-reduce, Adam), 4 x 256 rays
                  per rank (weak scaling: 8 ranks = 8192 rays), at every N;
  cfg2         -- (N = 1) BASELINE configs[1]: one SRN 128x128 frame as 4 x 4096-ray
                  chunks, with its own roofline (the round-1 headline);
  composite    -- (N = 1) the standalone alpha-composite kernel's HBM roofline;
  extra_configs -- (N = 1) cfg2 with the shipped conf, mlp_fine=None, cfg4 (DTU, NS = 3);
  cpu_baseline -- (N = 1, rank 0) the CPU oracle (oracle/ref_cpu.py) on a bounded sample
                  of the headline batch, median of 3, plus cfg1 at full size and a cfg2
                  subset, with os.cpu_count() and torch.get_num_threads() stated;
  psnr_vs_reference_path -- SURVEY §8(d)'s PSNR delta: the HIP render of that sample with
                  the same injected random streams against the oracle's render; fine-pass
                  bin flips are proven from the coarse weights (oracle/parity.py).
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "pixel-nerf_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pnr import _lib, synth, torchops, util  # noqa: E402
from pnr import dist as pdist  # noqa: E402
from pnr.models import PRECISIONS, PixelNeRFNet  # noqa: E402
from pnr.renderer import NeRFRenderer  # noqa: E402

MFMA_F32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: Peak FP32 (matrix)
MFMA_BF16_PEAK_TFLOPS = 2500.0 # MI355X_MICROARCH.md: Peak BF16 MFMA, dense
# fp32-equivalent peak of each ResnetFC arithmetic mode (pnr.models.PRECISIONS): the
# split modes issue 3 / 6 / 9 16-bit MFMA products per fp32 multiply-add
PEAK_BY_PRECISION = {"fp32": (MFMA_F32_PEAK_TFLOPS, 1), "f16x3": (MFMA_BF16_PEAK_TFLOPS / 3, 3),
                     "bf16x6": (MFMA_BF16_PEAK_TFLOPS / 6, 6),
                     "bf16x9": (MFMA_BF16_PEAK_TFLOPS / 9, 9)}
# the arithmetic type of the path: fp32 in / fp32 out with fp32 accumulation everywhere; the
# parenthesis names the matrix-core products the fp32 GEMMs are built from (ARITHMETIC)
DTYPE = {"fp32": "f32", "f16x3": "f32 (f16x3)", "bf16x6": "f32 (bf16x6)", "bf16x9": "f32 (bf16x9)"}
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


def flop_per_point(ns=1, latent_proj=True, n_blocks=5, combine_layer=3, d_in=42):
    """ResnetFC FLOP per point with ns source views (resnetfc.py:132-184): lin_in, the lin_z
    GEMMs (not executed with the projected latent: k_latent_proj folds them per latent pixel) and
    both block layers before combine_layer once per view, the later blocks once per point, lin_out.
    ns = 1, latent_proj False: FLOP_PER_POINT_NS1; True: KERNEL_FLOP_PER_POINT_NS1."""
    H = 512
    nc = min(combine_layer, n_blocks) if ns > 1 else n_blocks
    nz = min(combine_layer, n_blocks)
    per_view = 2 * H * d_in + 2 * H * H * (2 * nc + (0 if latent_proj else nz))
    return ns * per_view + 2 * H * H * 2 * (n_blocks - nc) + 2 * H * 4
KC, KF = 64, 64
# cfg3 (headline): ShapeNet-NMR 64x64, 24 target frames, latent 32x32
NMR_SIZE, NMR_FRAMES, NMR_FOCAL, NMR_NEAR, NMR_FAR, NMR_RADIUS = 64, 24, 70.0, 1.2, 4.0, 2.7
RAY_BATCH = 50000              # gen_video.py --ray_batch_size default (args.py:19)
# cfg2: SRN 128x128 frame in 4096-ray chunks
CHUNK = 4096
W = H = 128
FUSED_MARCH = True   # pnr_render_set_fused(2) (main: --unfused / --fused-mode)
# why the single-launch march (mode 3, north_star's "one fused kernel") is selectable but not the
# default (measured in round 4)
MARCH_MODE_BOUND = {
    "default_mode": 2, "single_launch_mode": 3,
    "mode3_upside_bound_pct": 0.15,
    "why": "mode 3 can only save what mode 2 spends outside its two k_point_mlp launches: the k_sample_fine "
           "launch (0.06 ms per 50,000-ray chunk) and one launch tail (~0.1 ms), ~0.15 % of a ~106 ms chunk; "
           "it pays the fine draws on one wave while seven wait (~0.6 % of tile work) and measured 0.8 % "
           "slower. Mode 3 is bit-identical to modes 0-2 (tests/test_gpu_parity.py::"
           "test_fused_march_matches_unfused) and runs with --fused-mode 3."}
MARCH_MODE = 2       # the fused mode (3: both passes in one launch)
KERNELS = ["sample_coarse", "mlp_coarse", "composite_coarse", "sample_fine", "mlp_fine", "composite_fine"]


def model_conf(use_first_pool=True):
    mlp = dict(type="resnet", n_blocks=5, d_hidden=512, combine_layer=3, combine_type="average")
    return dict(use_encoder=True, use_xyz=True, use_code=True,
                code=dict(num_freqs=6, freq_factor=1.5, include_input=True), use_viewdirs=True,
                use_code_viewdirs=False, mlp_coarse=mlp, mlp_fine=mlp,
                encoder=dict(backbone="resnet34", pretrained=False, num_layers=4,
                             use_first_pool=use_first_pool))


class HipEvents:
    """hipEvent_t handles from the HIP runtime torch already loaded."""

    def __init__(self):
        self.hip = ctypes.CDLL("libamdhip64.so.7")
        self.hip.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        self.hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p,
                                                 ctypes.c_void_p]
        self.hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]

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


class RenderProbe:
    """Records HIP events around every kernel of each fused render call while `on`
    (torch.ops.pnr.render_rays' `events` argument, through pnr.torchops.EVENTS_HOOK: no host
    synchronization is added), and the call's ray count, so per-launch durations and
    algorithmic work come from the same launches as the timed region."""

    def __init__(self, ev):
        self.ev = ev
        self.on = False
        self.calls = []      # (events, n_rays, n_coarse, n_fine)
        self.saved = None    # (avg, roofline) kept across a comparison run (cfg2_leg)

        def hook(n_rays, n_coarse, n_fine):
            if not self.on:
                return []
            evs = ev.create(7)
            self.calls.append((evs, int(n_rays), int(n_coarse), int(n_fine)))
            return [int(e.value) for e in evs]

        torchops.EVENTS_HOOK = hook

    def reset(self):
        self.calls = []

    def summary(self, precision, latent_proj, ns=1):
        """Per-kernel mean ms, and the fine MLP's roofline over the recorded launches (ns source
        views per point: the multi-view FLOP count)."""
        per = {n: [] for n in KERNELS}
        pts = []
        single = False
        for evs, n, kc, kf in self.calls:
            for i, name in enumerate(KERNELS):
                per[name].append(self.ev.elapsed_ms(evs[i], evs[i + 1]))
            # march mode 3 runs both passes in the launch events [1]-[2] time
            single = FUSED_MARCH and MARCH_MODE == 3 and latent_proj and kc == 64 and kc + kf == 128
            pts.append(n * (kc + kc + kf) if single else n * (kc + kf))
        avg = {k: sum(v) / len(v) for k, v in per.items() if v}
        kflop = flop_per_point(ns, latent_proj)
        ref_flop = flop_per_point(ns, False)
        pts_per_launch = sum(pts) / len(pts)
        flop = pts_per_launch * kflop
        ms = avg["mlp_coarse"] if single else avg["mlp_fine"]
        achieved = flop / (ms * 1e-3) / 1e12
        peak, terms = PEAK_BY_PRECISION[precision]
        # the fine pass (K = 128) runs the fused-march instantiation unless --unfused
        kname = "k_point_mlp<%d, %s, %s>" % (PRECISIONS[precision], "true" if latent_proj else "false",
                                             "true" if FUSED_MARCH else "false")
        return avg, {
            "kernel": "k_point_mlp (single-launch march: coarse + fine pass)" if single else "k_point_mlp (fine pass)",
            "bound": "mfma",
            "achieved": round(achieved, 2), "peak": round(peak, 1),
            "unit": "TFLOP/s (fp32-equivalent: algorithmic FLOP per launch (%d FLOP per point x points "
                    "per launch) / mean launch duration, HIP events on the launch stream)" % kflop,
            "reference_equivalent_tflops": round(pts_per_launch * ref_flop / (ms * 1e-3) / 1e12, 2),
            "frac": round(achieved / peak, 4),
            "mfma_issue": {"tflops": round(achieved * terms, 1),
                           "peak": MFMA_F32_PEAK_TFLOPS if terms == 1 else MFMA_BF16_PEAK_TFLOPS,
                           "products_per_fma": terms},
            "points_per_launch": round(pts_per_launch, 1), "launches": len(pts),
            "flop_per_launch": int(flop), "launch_ms": round(ms, 4),
            "kernel_name": kname,
        }


class ClockSampler:
    """The GPU's graphics clock sampled from the SMI library (amdsmi) in a background thread while
    `on` -- the sustained clock of the timed region, recorded in the line so a reader can place
    a run within the box-to-box spread (MI355X_MICROARCH.md "DVFS give-back": the SMI clock reads up
    to ~10 % above the in-kernel clock; profiles/<run>/clock.csv holds the GRBM_GUI_ACTIVE-derived
    one of the same lease).  The device is matched by PCI bus id; any failure leaves it off."""

    def __init__(self, dev, period_s=0.05):
        self.samples, self.err, self.h, self.period = [], None, None, period_s
        self._stop = None
        try:
            import amdsmi

            self.smi = amdsmi
            amdsmi.amdsmi_init()
            props = torch.cuda.get_device_properties(dev)
            bus = getattr(props, "pci_bus_id", None)
            for h in amdsmi.amdsmi_get_processor_handles():
                bdf = str(amdsmi.amdsmi_get_gpu_device_bdf(h))    # "0000:75:00.0"
                if bus is None or int(bdf.split(":")[1], 16) == int(bus):
                    self.h = h
                    self.bdf = bdf
                    break
            if self.h is None:
                self.err = "no SMI handle with PCI bus %s" % bus
        except Exception as e:   # noqa: BLE001 -- the clock is an annotation, never a failure
            self.err = "%s: %s" % (type(e).__name__, e)

    def _read(self):
        m = self.smi.amdsmi_get_gpu_metrics_info(self.h)
        xs = [v for v in (m.get("current_gfxclks") or []) if isinstance(v, (int, float)) and 0 < v < 10000]
        if xs:
            return sum(xs) / len(xs)
        v = m.get("current_gfxclk")
        if isinstance(v, (int, float)) and 0 < v < 10000:
            return float(v)
        return float(self.smi.amdsmi_get_clock_info(self.h, self.smi.AmdSmiClkType.GFX)["clk"])

    def start(self):
        import threading

        if self.h is None:
            return
        self.samples = []
        self._stop = threading.Event()

        def loop():
            while not self._stop.is_set():
                try:
                    self.samples.append(self._read())
                except Exception as e:   # noqa: BLE001
                    self.err = "%s: %s" % (type(e).__name__, e)
                    return
                self._stop.wait(self.period)

        self._t = threading.Thread(target=loop, daemon=True)
        self._t.start()

    def stop(self):
        if self._stop is None:
            return
        self._stop.set()
        self._t.join()
        self._stop = None

    def summary(self):
        if not self.samples:
            return {"mhz_mean": None, "error": self.err or "no samples"}
        s = sorted(self.samples)
        return {"mhz_mean": round(sum(s) / len(s), 1), "mhz_median": s[len(s) // 2], "mhz_min": s[0],
                "mhz_max": s[-1], "samples": len(s), "device_bdf": getattr(self, "bdf", None),
                "source": "amdsmi gpu_metrics current_gfxclk(s), sampled every %d ms over the timed region"
                          % int(self.period * 1000)}


def timed(fn, steps, warmup, dev, world, clock=None):
    """W untimed steps, then K timed steps between barrier + synchronize; max over ranks."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    if clock is not None:
        clock.start()
    t0 = time.perf_counter()
    for _ in range(steps):
        res = fn()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if clock is not None:
        clock.stop()
    if world > 1:
        dist.barrier()
    return pdist.max_over_ranks(t1 - t0, device=dev), res


# ----------------------------------------------------------------- cfg3 --------------
def nmr_inputs(dev):
    """cfg3 inputs: a hashed 64x64 source image, its pose, and the 24-frame ray batch."""
    img = torch.from_numpy(synth.hash_sym(31, (1, 3, NMR_SIZE, NMR_SIZE), 1.0)).to(dev)
    src = synth.srn_poses([0.0], phi=-20.0, radius=NMR_RADIUS).to(dev)
    tgt = synth.srn_poses([15.0 * i for i in range(NMR_FRAMES)], phi=-20.0, radius=NMR_RADIUS).to(dev)
    focal = torch.tensor(NMR_FOCAL, device=dev)
    rays = util.gen_rays(tgt, NMR_SIZE, NMR_SIZE, focal, NMR_NEAR, NMR_FAR).reshape(-1, 8).contiguous()
    return img, src, focal, rays


def make_net(dev, precision, latent_proj, use_first_pool=True):
    torch.manual_seed(0)   # the random-init encoder is identical on every rank
    net = PixelNeRFNet(model_conf(use_first_pool))
    net.load_state_dict(synth.pixelnerf_state(1), strict=False)
    net = net.to(dev).eval()
    net.mlp_precision = precision
    net.use_latent_proj = latent_proj
    return net


def cfg3_leg(args, dev, rank, world, probe, clock=None):
    net = make_net(dev, args.precision, not args.no_latent_proj, use_first_pool=False)
    # the eval encode runs the BN-folded trunk replayed as one HIP graph (pnr.encoder.InferenceTrunk);
    # --encoder-eager: the module's own conv / BN / relu launches (A/B)
    net.encoder.infer_fast = not getattr(args, "encoder_eager", False)
    img, src, focal, rays = nmr_inputs(dev)
    n_all = rays.shape[0]
    start, end = pdist.shard_range(n_all, rank, world)
    mine = rays[start:end]
    renderer = NeRFRenderer(n_coarse=KC, n_fine=KF, white_bkgd=True, eval_batch_size=RAY_BATCH).to(dev)
    render_par = renderer.bind_parallel(net, simple_output=True).eval()
    host = torch.empty(end - start, 3, pin_memory=True)
    enc_ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def step():
        enc_ev[0].record()
        net.encode(img, src, focal)          # ResNet34 trunk -> channels-last latent, cameras
        enc_ev[1].record()
        outs = [render_par(r[None])[0][0] for r in torch.split(mine, RAY_BATCH, dim=0)]
        rgb = torch.cat(outs)
        host.copy_(rgb, non_blocking=True)   # the rank's shard lands in host memory
        return rgb

    torch.backends.cudnn.benchmark = True
    torch.manual_seed(1234 + rank)
    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        probe.reset()
        probe.on = True
        elapsed, rgb = timed(step, args.steps, 0, dev, world, clock=clock)
        probe.on = False
    assert bool(torch.isfinite(rgb).all())
    avg, roof = probe.summary(args.precision, net.use_latent_proj)
    enc = enc_ev[0].elapsed_time(enc_ev[1])   # the last timed step's encode
    return net, (img, src, focal, rays), elapsed, avg, roof, enc, (start, end)


# ----------------------------------------------------------------- cfg2 --------------
def cfg2_leg(args, dev, probe):
    """BASELINE configs[1]: one SRN 128x128 frame, 4 x 4096-ray chunks (N = 1)."""
    net = make_net(dev, args.precision, not args.no_latent_proj)
    net.encode_latent(synth.latent(0, 1, 512, 64, 64).to(dev), synth.srn_poses([0.0]).to(dev),
                      torch.tensor(131.25, device=dev), (W, H))
    rays = util.gen_rays(synth.srn_poses([30.0]).to(dev), W, H, torch.tensor(131.25), 0.01, 4.0)
    chunks = list(torch.split(rays.reshape(-1, 8).contiguous(), CHUNK, dim=0))
    renderer = NeRFRenderer(n_coarse=KC, n_fine=KF, white_bkgd=True, eval_batch_size=CHUNK).to(dev)
    render_par = renderer.bind_parallel(net, simple_output=True).eval()

    def step():
        net.drop_latent_proj()   # per-scene projection rebuilt inside every timed frame
        return torch.cat([render_par(r[None])[0][0] for r in chunks])

    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        probe.reset()
        probe.on = True
        elapsed, img = timed(step, args.steps, 0, dev, 1)
        probe.on = False
        value_fp32, roof_fp32 = None, None
        if args.precision != "fp32" and not args.no_compare:
            # the same frame with plain fp32 MFMA products, with its own fine-MLP roofline
            # against the fp32 matrix peak (events on the same launches)
            avg_main, roof_main = probe.summary(args.precision, net.use_latent_proj)
            net.mlp_precision = "fp32"
            for _ in range(1):
                step()
            probe.reset()
            probe.on = True
            t_fp32, _ = timed(step, 3, 0, dev, 1)
            probe.on = False
            value_fp32 = round(3 * W * H / t_fp32, 1)
            _, rf = probe.summary("fp32", net.use_latent_proj)
            roof_fp32 = {k: rf[k] for k in ("achieved", "peak", "frac", "launch_ms", "kernel_name")}
            roof_fp32["unit"] = "TFLOP/s (fp32 products on v_mfma_f32_16x16x4_f32)"
            net.mlp_precision = args.precision
            probe.calls = []   # the headline summary below comes from the main precision's launches
            probe.saved = (avg_main, roof_main)
    assert bool(torch.isfinite(img).all())
    if getattr(probe, "saved", None) is not None:
        (avg, roof), probe.saved = probe.saved, None
    else:
        avg, roof = probe.summary(args.precision, net.use_latent_proj)
    return dict(value=round(W * H * args.steps / elapsed, 1), unit="rays/s",
                ms_per_frame=round(1e3 * elapsed / args.steps, 3),
                workload="cfg2: SRN-cars 128x128 frame, 1 source view, 4096-ray chunks x (64 + 64)",
                roofline=roof, kernel_ms={k: round(v, 4) for k, v in avg.items()},
                value_fp32_mfma=value_fp32, roofline_fp32_mfma=roof_fp32,
                l2_stream=l2_stream(roof["points_per_launch"], roof["launch_ms"], args.precision,
                                    net.use_latent_proj))


# ----------------------------------------------------------------- cfg5 --------------
def train_leg(dev, rank, world, steps, warmup, precision="f16x3", sb=4, per=256, ns=1, graph=False,
              sync_debug=False, bn=None):
    """cfg5 (BASELINE configs[4]; the reference's train.py:182-283) on synthetic SRN-shaped
    data: encode SB x NS source images (ResNet34 trunk), render SB x B' rays with the shipped
    conf (64 coarse + 32 fine incl. 16 depth, white background) through the HIP training path
    (pnr/train.py), MSE(coarse) + MSE(fine) (conf/default.conf:77-78), backward, bucketed
    gradient mean over RCCL/xGMI overlapped with the backward (pnr.dist.GradReducer), Adam lr 1e-4
    (trainer.py:49).
    Weak scaling: SB x B' rays per rank.  Returns the result dict (max-over-ranks timing)."""
    from pnr.models import make_model

    torch.manual_seed(1234 + rank)
    torch.backends.cudnn.benchmark = True   # MIOpen solver search for the encoder convolutions
    net = make_model(model_conf()).to(dev)
    net.load_state_dict(synth.pixelnerf_state(0), strict=False)
    net.mlp_precision = precision
    # encoder BatchNorm over ranks: the reference encodes the whole step's objects in one batch
    # (train.py:257-262), so at N > 1 the statistics are synchronised over the ranks
    bn = bn or ("sync" if world > 1 else "batch")
    pdist.set_batchnorm_mode(net.encoder, bn)
    net.train()
    renderer = NeRFRenderer(n_coarse=64, n_fine=32, n_fine_depth=16, depth_std=0.01, white_bkgd=True).to(dev)
    # fused Adam: one multi-tensor kernel per step (the reference uses torch.optim.Adam, same update);
    # capturable keeps the step counter on the device so the update replays inside a graph
    opt = torch.optim.Adam(net.parameters(), lr=1e-4, fused=True, capturable=graph)
    params = list(net.parameters())
    focal = torch.tensor(131.25, device=dev)
    src_poses = synth.srn_poses([float(15 * i + 7 * rank + 40 * v) for i in range(sb) for v in range(ns)]).to(dev)
    if ns > 1:
        src_poses = src_poses.reshape(sb, ns, 4, 4)
    tgt_poses = synth.srn_poses([float(15 * i + 7 * rank + 90) for i in range(sb)]).to(dev)
    g = torch.Generator(device=dev).manual_seed(rank)
    images = (torch.rand(sb, 3, H, W, device=dev, generator=g) * 2 - 1 if ns == 1 else
              torch.rand(sb, ns, 3, H, W, device=dev, generator=g) * 2 - 1)
    all_rays = util.gen_rays(tgt_poses, W, H, focal, 0.8, 1.8).reshape(sb, -1, 8)   # on device
    pix = torch.randint(0, W * H, (sb, per), device=dev, generator=g)
    rays = torch.gather(all_rays, 1, pix[..., None].expand(-1, -1, 8)).contiguous()
    target = torch.rand(sb, per, 3, device=dev, generator=g)
    mse = torch.nn.functional.mse_loss

    # gradient mean overlapped with the backward: buckets go out from the grad hooks as they fill
    # (the MLP buckets under the encoder's backward), the rest after backward()
    reducer = pdist.GradReducer(params, world)

    def step():
        opt.zero_grad(set_to_none=True)
        net.encode(images, src_poses, focal)
        out = renderer(net, rays, want_weights=True)
        loss = mse(out.coarse.rgb, target) + mse(out.fine.rgb, target)
        reducer.arm()
        loss.backward()
        reducer.finish()
        opt.step()
        return loss

    run = step
    if graph:
        # HIP graph of the whole step: warm-up on a side stream (MIOpen solver search, pack
        # caches, allocator), then capture; inputs are static tensors
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(max(warmup, 2)):
                step()
        torch.cuda.current_stream(dev).wait_stream(side)
        cg = torch.cuda.CUDAGraph()
        opt.zero_grad(set_to_none=True)
        with torch.cuda.graph(cg):
            static_loss = step()

        def run():
            cg.replay()
            return static_loss

        warmup = 1
    for _ in range(warmup):
        run()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    from pnr import train as ptrain

    ptrain.KERNEL_EVENTS = None if graph else {}   # HIP events around the MLP kernels (eager only)
    t0 = time.perf_counter()
    if sync_debug:
        torch.cuda.set_sync_debug_mode("warn")
    for _ in range(steps):
        loss = run()
    if sync_debug:
        torch.cuda.set_sync_debug_mode("default")
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    kev, ptrain.KERNEL_EVENTS = ptrain.KERNEL_EVENTS, None
    if world > 1:
        dist.barrier()
    elapsed = pdist.max_over_ranks(t1 - t0, dev)
    rays_total = sb * per * steps * world
    # roofline of the step: algorithmic FLOP = forward + input gradient + weight gradient of every
    # ResnetFC layer, 3 x 6,862,848 per point (NS = 1; §8(d)), over the step's points
    # (SB x B' rays x (64 coarse + 96 fine)); peak = the f16x3 fp32-equivalent 833 TFLOP/s
    pts = sb * per * (renderer.n_coarse + renderer.n_coarse + renderer.n_fine)
    step_flop = 3.0 * FLOP_PER_POINT_NS1 * pts * ns if ns == 1 else None
    ms_step = elapsed / steps * 1e3
    peak = PEAK_BY_PRECISION[precision][0]
    roof = None
    if step_flop is not None:
        kernels = {}
        for name, evs in (kev or {}).items():
            ms = sum(a.elapsed_time(b) for a, b, _ in evs) / steps
            fl = sum(f for _, _, f in evs) / steps
            kernels[name] = {"ms_per_step": round(ms, 4), "launches_per_step": len(evs) // steps,
                             "tflops": round(fl / (ms * 1e-3) / 1e12, 1), "frac": round(fl / (ms * 1e-3) / 1e12 / peak, 4)}
        roof = {"bound": "mfma", "achieved": round(step_flop / (ms_step * 1e-3) / 1e12, 2), "peak": round(peak, 1),
                "unit": "TFLOP/s (fp32-equivalent: 3 x %d FLOP per point (forward + input gradient + weight "
                        "gradient) x %d points per step / ms_per_step)" % (FLOP_PER_POINT_NS1, pts),
                "frac": round(step_flop / (ms_step * 1e-3) / 1e12 / peak, 4), "flop_per_step": int(step_flop),
                "kernels": kernels,
                "kernel_note": "HIP events on the launch stream: forward = k_point_mlp<3, false, false> with the "
                               "activation save, mlp_backward = k_mlp_bwd (+ k_bias_reduce), weight_grad = "
                               "k_wgrad_h (+ k_wgrad_reduce); frac of each against the same peak"}
    arith = (precision + " forward + f16x3 fused input-gradient chain%s + f16x3 weight gradients (running "
             "per-channel power-of-two scales, csrc/wgrad.hip k_wgrad_h)"
             % (" (NS = %d views)" % ns if ns > 1 else "")
             if precision == "f16x3" else precision + " forward, fp32 GEMM backward")
    return {
        "metric": "training rays/sec (cfg5: encoder + coarse/fine render + backward + grad all-reduce + Adam)",
        "value": round(rays_total / elapsed, 1), "unit": "rays/s", "n_gpus": world, "steps": steps,
        "ms_per_step": round(elapsed / steps * 1e3, 3), "scaling": "weak",
        "arithmetic": arith + " (pnr/train.py)",
        "config": {"workload": "cfg5: SB=%d objects x %d rays per rank, %d source view(s), 64 coarse + 32 fine "
                               "(16 depth)" % (sb, per, ns), "global_batch_rays": sb * per * world,
                   "parallelism": "data parallel, 1 process per GPU, bucketed RCCL all-reduce (32 MB buckets) "
                                  "launched from the backward's grad hooks",
                   "encoder_batchnorm": bn + (" (statistics all-reduced over the ranks, pnr.dist.SyncBatchNorm2d)"
                                              if bn == "sync" else ""),
                   "launch": "one HIP graph per step" if graph else "eager"},
        "loss": round(float(loss.item()), 6),
        "roofline": roof,
    }


# ----------------------------------------------------------------- roofline helpers --
def composite_roofline(dev, ev, pmc_path=None, same_lease=False):
    """Standalone composite kernel on 1 M rays x 128 samples (HBM-bound): algorithmic bytes
     / HIP-event time, and -- when a PMC summary holds this leg's launches
    (workload composite_1M, scripts/summarize_profile.py) -- the counter bytes per launch and
    counter GB/s (counter bytes / the same HIP-event time) beside them (north_star: "rocprof HBM
    GB/s on the composite step")."""
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
        for _ in range(11):   # the median of 11 launches (one launch varies by a few % on a box)
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
        key = "weights" if want_w else "no_weights"
        res[key] = dict(
            ms=round(ms, 4), bytes_per_ray=per_ray, achieved=round(gbs, 1), peak=HBM_PEAK_GBS,
            unit="GB/s", frac=round(gbs / HBM_PEAK_GBS, 4))
        if pmc_path and os.path.exists(pmc_path):
            rows = [(b, dms) for k, g, dms, b, p, w in pmc_rows(pmc_path)
                    if "k_composite" in k and w == "composite_1M" and p == key]
            if rows:
                tb = sum(b for b, _ in rows) / len(rows)
                res[key]["pmc"] = dict(
                    hbm_bytes_per_launch=int(tb), algorithmic_bytes_per_launch=per_ray * B,
                    traffic_over_algorithmic=round(tb / (per_ray * B), 4),
                    counter_gbs=round(tb / (ms * 1e-3) / 1e9, 1),
                    counter_frac=round(tb / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    launches=len(rows), source=pmc_source_label(pmc_path, same_lease))
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


def density_grid_leg(net, dev, precision, latent_proj, res=256, chunk=65536):
    """eval/eval.py's density grid (eval.py:93-103; scripts/eval.py): relu(sigma) of the coarse net
    at res^3 points over [-1, 1]^3 through PixelNeRFNet.forward (the point query, SURVEY §8(a)
    a17) in the caller's 65,536-point chunks.  Timed with events around the whole pass (res^3 /
    chunk launches with their host glue), so its rate includes each launch's ramp and tail."""
    grid = torch.linspace(-1, 1, res, device=dev)
    pts = torch.stack(torch.meshgrid(grid, grid, grid, indexing="ij"), -1).reshape(-1, 3)
    vd = torch.zeros(1, chunk, 3, device=dev)
    sig = torch.empty(pts.shape[0], device=dev)

    def grid_pass():
        for i in range(0, pts.shape[0], chunk):
            p = pts[i:i + chunk][None]
            sig[i:i + chunk] = net(p, coarse=True, viewdirs=vd[:, :p.shape[1]])[0, :, 3]

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.no_grad():
        grid_pass()
        torch.cuda.synchronize(dev)
        e0.record()
        grid_pass()
        e1.record()
        torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1)
    assert bool(torch.isfinite(sig).all())
    n = pts.shape[0]
    flop = n * flop_per_point(1, latent_proj)
    peak = PEAK_BY_PRECISION[precision][0]
    return dict(points_per_s=round(n / ms * 1e3, 1), ms_per_grid=round(ms, 3), points=n, chunk=chunk,
                workload="eval.py density grid: %d^3 points of the coarse net, %d-point point-query calls" % (res, chunk),
                roofline=dict(achieved=round(flop / (ms * 1e-3) / 1e12, 2), peak=round(peak, 1),
                              frac=round(flop / (ms * 1e-3) / 1e12 / peak, 4),
                              unit="TFLOP/s (fp32-equivalent: %d FLOP per point x points / the whole pass, "
                                   "launch ramps and host glue included)" % flop_per_point(1, latent_proj)))


def extra_configs(dev, precision, latent_proj=True, probe=None, oracle_rays=64):
    """Other SURVEY §8(d) workloads on 1 GPU (informational, not `value`): cfg2 with the
    shipped conf (64 + 32 incl. 16 depth samples), cfg2 as eval_approx.py --coarse renders it
    (mlp_fine = None, 64 + 128), cfg4 DTU 400x300 with NS = 3 source views (one 120,000-ray
    frame, the multi-view mean path) in gen_video's 50,000-ray chunks -- with its fine-launch
    roofline (HIP events, NS = 3 FLOP per point as the kernel executes it) and an oracle agreement
    leg on ``oracle_rays`` rays of the frame (the CPU oracle, same injected streams)."""
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

    net = make(synth.latent(0, 1, 512, 64, 64), synth.srn_poses([0.0]), torch.tensor(131.25), (W, H))
    rays = util.gen_rays(synth.srn_poses([30.0]).to(dev), W, H, torch.tensor(131.25), 0.01, 4.0).reshape(-1, 8)
    r = NeRFRenderer(n_coarse=64, n_fine=32, n_fine_depth=16, depth_std=0.01, white_bkgd=True).to(dev)
    s = _time_render(net, r, rays, CHUNK)
    res["cfg2_shipped_64_32_16"] = dict(rays_per_s=round(rays.shape[0] / s, 1), ms_per_frame=round(s * 1e3, 3),
                                        gflop_per_ray=round(160 * FLOP_PER_POINT_NS1 / 1e9, 4))
    net.mlp_fine = None
    r = NeRFRenderer(n_coarse=64, n_fine=128, white_bkgd=True).to(dev)
    s = _time_render(net, r, rays, CHUNK)
    res["cfg2_coarse_as_fine_64_128"] = dict(rays_per_s=round(rays.shape[0] / s, 1),
                                             ms_per_frame=round(s * 1e3, 3))
    res["eval_density_grid_256"] = density_grid_leg(net, dev, precision, latent_proj)
    sc = synth.scene_multiview(seed=8, n_views=3, n_rays=1)
    net = make(synth.latent(8, 3, 512, 150, 200), sc["poses"][None], sc["focal"][None], (400, 300),
               c=sc["c"][None])
    rays = util.gen_rays(synth.srn_poses([10.0], phi=-12.0, radius=2.0).to(dev), 400, 300, sc["focal"],
                         0.1, 5.0, c=sc["c"]).reshape(-1, 8)
    r = NeRFRenderer(n_coarse=64, n_fine=64, white_bkgd=False, eval_batch_size=RAY_BATCH).to(dev)
    with torch.no_grad():   # warm-up (packs, projections, allocator)
        r(net, rays[None])
    torch.cuda.synchronize(dev)
    if probe is not None:
        probe.reset()
        probe.on = True
    with torch.no_grad():
        t0 = time.perf_counter()
        r(net, rays[None])
        torch.cuda.synchronize(dev)
        s = time.perf_counter() - t0
    cfg4 = dict(rays_per_s=round(rays.shape[0] / s, 1), ms_per_frame=round(s * 1e3, 3),
                gflop_per_ray=round(192 * flop_per_point(3, False) / 1e9, 4),
                workload="cfg4: DTU 400x300 frame, 3 source views (150x200 latent each), 64 + 64, "
                         "gen_video's %d-ray chunks" % RAY_BATCH,
                ray_order="%s (%s)" % (r.ray_order, "16 x 16 pixel blocks: the projected rows exceed the caches"
                                       if r._blocked_order(net) else "input order"))
    if probe is not None:
        probe.on = False
        avg, roof = probe.summary(precision, latent_proj, ns=3)
        roof["kernel"] = "k_point_mlp (fine pass, NS = 3: lin_in and blocks 0-2 per view, mean, blocks 3-4)"
        cfg4["roofline"] = roof
        cfg4["kernel_ms"] = {k: round(v, 4) for k, v in avg.items()}
    if oracle_rays:
        cfg4["oracle_agreement"] = cfg4_oracle_leg(net, rays, sc, sd, dev, oracle_rays)
    res["cfg4_dtu_ns3_frame"] = cfg4
    return res


def cfg4_oracle_leg(net, rays, sc, sd, dev, n):
    """The HIP render of n rays spread over the cfg4 frame against the CPU oracle's render of the
    same rays with the same injected streams (NS = 3 multi-view mean path; black background)."""
    from oracle import ref_cpu

    idx = torch.linspace(0, rays.shape[0] - 1, n).round().long()
    sub = rays[idx.to(dev)].contiguous()
    streams = synth.rng_streams(41, n, 64, 64, 0)
    scene = ref_cpu.Scene(net.encoder.latent.detach().float().cpu().contiguous(), sc["poses"][None],
                          sc["focal"][None], 400, 300, sc["c"][None])
    with torch.no_grad():
        ref = ref_cpu.render(lambda p, c, d: ref_cpu.pixelnerf_forward(sd, scene, p, c, d), sub.cpu()[None],
                             64, 64, 0, streams, False)
    return psnr_vs_reference_path(net, sub, ref, streams, dev, sd, scene, white_bkgd=False)


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
    tiles = int((points + 63) // 64)
    # packed 512x512 layers (10, or 13 with the per-point lin_z GEMMs), lin_in, lin_out
    weights = (10 if latent_proj else 13) * (1 << 20) + (128 << 10) + (32 << 10)
    gather = 3 * 64 * 4 * 2048   # 3 blends x 64 points x 4 corners x 2 KB rows (P or the latent)
    total = tiles * (weights + gather)
    tbs = total / (launch_ms * 1e-3) / 1e12
    return {"kernel": "k_point_mlp (fine pass)", "bytes_per_tile": weights + gather, "tiles": tiles,
            "achieved": round(tbs, 2), "peak": L2_PEAK_TBS, "unit": "TB/s (L2 -> CU)",
            "frac": round(tbs / L2_PEAK_TBS, 4),
            "frac_of_gather_loop": round(tbs / L2_GATHER_LOOP_TBS, 4)}


def pmc_rows(path):
    """Rows of a pmc_summary.csv (scripts/summarize_profile.py): (kernel, grid, dispatch_ms,
    hbm_bytes_corrected, pass, workload)."""
    import csv

    with open(path) as fh:
        rows = list(csv.reader(ln for ln in fh if not ln.startswith("#") and not ln.startswith("kernel,")))
    return [(f[0], int(f[1]), float(f[2]), int(f[5]), f[6], f[7]) for f in rows if f and len(f) > 7]


def pmc_summary_path(explicit=None):
    """The PMC summary the line's `traffic` figures come from: --traffic-from (a summary written
    by the same GPU lease, scripts/gpu_session.sh `evidence`), else the newest committed
    profiles/*/pmc_summary.csv.  Returns (path, same_lease)."""
    import glob

    if explicit:
        return explicit, True
    paths = sorted(glob.glob(os.path.join(REPO, "profiles", "*", "pmc_summary.csv")), reverse=True)
    return (paths[0], False) if paths else (None, False)


def pmc_traffic(kernel, render_pass, workload, path):
    """Mean HBM bytes per launch of `kernel` in `render_pass` of `workload` in the PMC summary at
    `path` (rocprofv3 counters cannot be read live from inside the process).  Returns bytes or None."""
    if not path or not os.path.exists(path):
        return None
    vals = [b for k, _, _, b, p, w in pmc_rows(path) if k.endswith(kernel) and p == render_pass and w == workload]
    return sum(vals) // len(vals) if vals else None


def pmc_source_label(path, same_lease):
    if path is None:
        return None
    rel = os.path.relpath(path, REPO)
    if same_lease:
        return ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes run in the same GPU lease as this bench, just "
                "before it (%s; FETCH x2 gfx950 correction)" % rel)
    return ("committed PMC summary %s from an EARLIER lease, not measured in this run (FETCH x2 gfx950 "
            "correction)" % rel)


# ----------------------------------------------------------------- CPU baseline -----
def cpu_baselines(sd, nmr, net3, dev, n_rays):
    """The oracle (oracle/ref_cpu.py, the CPU restatement of the reference path, pinned to
    the reference's outputs) on the box's host cores, median of 3 after a warm-up:
      * the headline's bounded sample: n_rays rays spread evenly over the cfg3 batch x (64+64),
        on the latent the GPU leg's encoder produced;
      * cfg1 at full size (256 rays x 32 coarse samples; BASELINE configs[0]);
      * cfg2 on a 512-ray subset of the 128x128 frame x (64+64), extrapolated per ray.
    Returns (baseline dict, oracle render of the cfg3 sample, its ray indices, its streams, the
    oracle scene of the sample)."""
    from oracle import ref_cpu

    def median_run(fn, give_up=None):
        """Median of 3 timed runs after a warm-up; one run only when it already takes longer
        than ``give_up`` seconds (a thread count far slower than one already measured)."""
        fn(warm=True)
        times, out = [], None
        for _ in range(3):
            t0 = time.perf_counter()
            out = fn(warm=False)
            times.append(time.perf_counter() - t0)
            if give_up is not None and times[-1] > give_up:
                break
        return statistics.median(times), times, out

    def runner(scene, rays, streams, kc, kf):
        def run(warm):
            rr, ss = (rays[:8], tuple(s[:8] for s in streams)) if warm else (rays, streams)
            with torch.no_grad():
                return ref_cpu.render(lambda p, c, d: ref_cpu.pixelnerf_forward(sd, scene, p, c, d),
                                      rr[None], kc, kf, 0, ss, True)
        return run

    img, src, focal, rays3 = nmr
    idx = torch.linspace(0, rays3.shape[0] - 1, n_rays).round().long().to(dev)
    scene3 = ref_cpu.Scene(net3.encoder.latent.detach().float().cpu().contiguous(), src.cpu(),
                           torch.tensor(NMR_FOCAL), NMR_SIZE, NMR_SIZE, None)
    st3 = synth.rng_streams(2, n_rays, KC, KF, 0)
    # torch.set_num_threads(os.cpu_count()).  On a shared box the process may
    # be held to fewer CPUs (affinity / the job's CPU share, OMP_NUM_THREADS) than the host
    # has, so the headline sample is timed at both counts; `value` is the faster, and both
    # are reported
    share = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "0")) or 1 << 30)
    counts = [share]
    if (os.cpu_count() or 1) != share:
        counts.append(os.cpu_count() or 1)
    by_threads = {}
    for n in counts:
        torch.set_num_threads(n)
        fastest = min((v[0] for v in by_threads.values()), default=None)
        t, runs, out = median_run(runner(scene3, rays3[idx].cpu(), st3, KC, KF),
                                  give_up=None if fastest is None else 3 * fastest)
        by_threads[n] = (t, runs, out)
    best = min(by_threads, key=lambda n: by_threads[n][0])
    torch.set_num_threads(best)
    t3, runs3, ref3 = by_threads[best]
    sc1 = synth.scene_srn(seed=0, n_rays=256)
    scene1 = ref_cpu.Scene(sc1["latent"], sc1["poses"], sc1["focal"], W, H, None)
    t1, runs1, _ = median_run(runner(scene1, sc1["rays"], synth.rng_streams(9, 256, 32, 0, 0), 32, 0))
    sc2 = synth.scene_srn(seed=0, n_rays=512, pick="hash")
    scene2 = ref_cpu.Scene(sc2["latent"], sc2["poses"], sc2["focal"], W, H, None)
    t2, runs2, _ = median_run(runner(scene2, sc2["rays"], synth.rng_streams(3, 512, KC, KF, 0), KC, KF))
    fmt = lambda ts: ", ".join("%.2f" % t for t in ts)  # noqa: E731
    base = dict(value=round(n_rays / t3, 2), unit="rays/s", cores=torch.get_num_threads(), kind="port",
                os_cpu_count=os.cpu_count(), torch_num_threads=torch.get_num_threads(),
                cpus_allowed=len(os.sched_getaffinity(0)),
                by_threads={str(n): dict(value=round(n_rays / v[0], 2), runs_s=[round(x, 3) for x in v[1]])
                            for n, v in by_threads.items()},
                sample="%d rays spread evenly over the cfg3 98,304-ray batch x (64+64) samples, "
                       "oracle/ref_cpu.py, median of 3 runs (%s s) at %d threads (the faster of "
                       "os.cpu_count() and the process's CPU share, by_threads; a count 3x slower than "
                       "the faster after one run is not repeated)"
                       % (n_rays, fmt(runs3), best),
                cfg1_full=dict(value=round(256 / t1, 2), unit="rays/s",
                               sample="cfg1 at full size: 256 rays x 32 coarse, median of 3 (%s s)" % fmt(runs1)),
                cfg2_subset=dict(value=round(512 / t2, 2), unit="rays/s",
                                 sample="cfg2: 512 hashed rays of the 128x128 frame x (64+64), median of 3 "
                                        "(%s s), extrapolated per ray" % fmt(runs2)))
    return base, ref3, idx, st3, scene3


def psnr_vs_reference_path(net, rays_dev, ref, streams, dev, sd, scene, white_bkgd=True):
    """SURVEY §8(d)'s PSNR delta: the HIP render of the cpu_baseline rays with the SAME
    injected random streams, against the oracle's render of them (oracle/ref_cpu.py, the
    CPU restatement pinned to the reference).  `agreement_db` = PSNR(HIP, oracle);
    `delta_db` = PSNR(HIP, target) - PSNR(oracle, target) for a seeded U(0,1) target image
    (no ground-truth frames offline).  Fine-pass rays are excluded from the `_excl_flips`
    figures only for a searchsorted bin flip PROVEN from the two sets of coarse weights
    (oracle/parity.py); `unexplained_rays` (fine samples that differ without one) must be 0."""
    from oracle import parity

    n = rays_dev.shape[0]
    r = NeRFRenderer(n_coarse=KC, n_fine=KF, n_fine_depth=0, white_bkgd=white_bkgd).to(dev)
    r.streams = tuple(t.to(dev) for t in streams)
    r.return_z = True
    with torch.no_grad():
        out = r(net, rays_dev[None].contiguous(), want_weights=True)
    tgt = torch.from_numpy(synth.hash_uniform(5, n * 3).astype("float32")).reshape(n, 3)
    z_exp = parity.expected_fine_sets(rays_dev, out.coarse.z, out.coarse.weights, out.coarse.depth, streams,
                                   KC, KF, 0)
    cls = parity.classify_fine(out.coarse.weights[0], ref["coarse"]["weights"][0], streams[1],
                               out.fine.z[0], ref["fine"]["z"], z_exp)

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
    # no ray escapes an output check: a flipped ray's rgb / depth / weights against the oracle
    # fine pass at its own (HIP) fine samples, with each flip's draw-to-boundary distance
    chk = parity.check_flipped_outputs(sd, scene, rays_dev.cpu(), out.fine.z, out.fine.rgb, out.fine.depth,
                                       out.fine.weights, cls["flip_idx"], n, white_bkgd,
                                       w_coarse_hip=out.coarse.weights, u_fine=streams[1])
    res["fine"]["flipped_rays_vs_oracle_at_own_samples"] = dict(
        ok=chk["ok"], max_abs=chk["max_abs"], bad_rays=chk.get("bad_rays", []),
        boundary_distance=chk.get("boundary_distance", []))
    res["fine"]["unexplained_rays"] = int(cls["unexplained"].sum())
    res["fine"]["flips_not_following_own_coarse_weights"] = int(cls["inconsistent"].sum())
    res["rays"] = n
    res["flip_rule"] = ("fine-bin flip = searchsorted bins recomputed from the HIP and the oracle "
                        "coarse weights with the same u differ (oracle/parity.py)")
    return res


# ----------------------------------------------------------------- launcher ----------
def _free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_argv(n_gpus, bench_argv, port, python=sys.executable, script=None):
    """Command that runs this bench as `n_gpus` ranks, one process per GPU, under
    torch.distributed.run on this node (the reference scatters rays over the listed GPUs
    itself, nerf.py:367-371; here every GPU gets its own process)."""
    script = script or os.path.abspath(__file__)
    return [python, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(int(n_gpus)),
            "--master-addr", "127.0.0.1", "--master-port", str(int(port)), script] + list(bench_argv)


def check_world(n_gpus, env=os.environ):
    """In a rank: the launcher's WORLD_SIZE must be the --gpus the bench was asked for.
    Returns True when this process must launch the ranks itself (--gpus N > 1 and no
    torch.distributed.run around it)."""
    if "WORLD_SIZE" not in env:
        return n_gpus > 1
    world = int(env["WORLD_SIZE"])
    if world != n_gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d (launch N ranks for --gpus N)" % (n_gpus, world))
    return False


def spawn_ranks(n_gpus, bench_argv):
    """Run the N ranks as a CHILD process (torch.distributed.run) and return its exit code.
    The calling process has not touched HIP, and it never exec()s: it waits for the child,
    whose ranks print the JSON line (rank 0) to the inherited stdout."""
    import subprocess

    cmd = launcher_argv(n_gpus, bench_argv, _free_port())
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    return subprocess.call(cmd, env=env)


# ----------------------------------------------------------------- main --------------
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-rays", type=int, default=512, help="oracle sample of the headline batch")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-composite", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the cfg2-shipped / coarse-as-fine / cfg4 lines")
    ap.add_argument("--no-cfg2", action="store_true", help="skip the cfg2 frame leg")
    ap.add_argument("--no-train", action="store_true", help="skip the cfg5 training leg")
    ap.add_argument("--no-compare", action="store_true", help="skip the f32-MFMA comparison frame")
    ap.add_argument("--train-steps", type=int, default=5)
    ap.add_argument("--precision", default="f16x3", choices=sorted(PEAK_BY_PRECISION))
    ap.add_argument("--encoder-eager", action="store_true",
                    help="cfg3 encode by the module's conv / BN / relu launches instead of the folded trunk's graph")
    ap.add_argument("--no-latent-proj", action="store_true",
                    help="per-point lin_z GEMMs on the gathered latent (A/B against the projection)")
    ap.add_argument("--unfused", action="store_true",
                    help="separate sample / MLP / composite kernels instead of the fused ray march (A/B)")
    ap.add_argument("--traffic-from", default=None,
                    help="pmc_summary.csv written by this GPU lease (scripts/gpu_session.sh evidence); default: "
                         "the newest committed profiles/*/pmc_summary.csv, labelled as such")
    ap.add_argument("--no-clock", action="store_true", help="do not sample the GPU clock (amdsmi)")
    ap.add_argument("--fused-mode", type=int, default=2,
                    help="pnr_render_set_fused: 2 fused passes + fine-draw kernel (default), 1 fine draws "
                         "in the coarse epilogue too, 3 both passes in one launch")
    args = ap.parse_args()
    # `python bench.py --gpus N` (N > 1) outside torch.distributed.run: launch the N ranks as
    # a child before anything here touches the GPU, and exit with their status
    if check_world(args.gpus):
        sys.stdout.flush()
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    global FUSED_MARCH, MARCH_MODE
    FUSED_MARCH = not args.unfused
    MARCH_MODE = 0 if args.unfused else args.fused_mode
    if hasattr(_lib.load(), "pnr_render_set_fused"):   # absent only in A/B builds of older revisions
        _lib.load().pnr_render_set_fused(0 if args.unfused else args.fused_mode)

    rank, world, local = pdist.init_from_env("nccl")   # RCCL on ROCm; control plane only
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    ev = HipEvents()
    probe = RenderProbe(ev)

    clock = None if args.no_clock else ClockSampler(dev)
    net3, nmr, elapsed, avg, roof, enc_ms, (start, end) = cfg3_leg(args, dev, rank, world, probe, clock)
    n_batch = nmr[3].shape[0]
    pmc_path, same_lease = pmc_summary_path(args.traffic_from)
    roof["traffic"] = pmc_traffic(roof["kernel_name"], "fine", "cfg3", pmc_path)
    roof["traffic_source"] = pmc_source_label(pmc_path, same_lease)
    out = {
        "metric": "rays/sec (coarse+fine, 64+64 samples)",
        "value": round(n_batch * args.steps / elapsed, 1),
        "unit": "rays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": DTYPE[args.precision],
        "arithmetic": ARITHMETIC[args.precision],
        "march": ("separate sample / MLP / composite kernels" if args.unfused else
                  "fused (mode 3): ONE k_point_mlp launch per batch -- a ray's coarse tile (coarse draws in "
                  "its prologue, composite + fine draws in its epilogue, fine depths kept in LDS), then its two "
                  "fine tiles (composite in the epilogue); roofline.launch_ms is that launch"
                  if args.fused_mode == 3 else
                  "fused (mode %d): one k_point_mlp launch per pass, coarse draws in its prologue, the "
                  "composite in its epilogue (roofline.launch_ms includes them); fine draws %s"
                  % (args.fused_mode, "in the coarse epilogue" if args.fused_mode == 1 else "in their own kernel")),
        "data": "synthetic (hash-initialised ResnetFC weights, random-init ResNet34 encoder on a hashed "
                "64x64 source image; NMR geometry)",
        "config": {"workload": "cfg3: ShapeNet-NMR 64x64, 1 source view, 24 frames = 98,304 rays per step "
                               "x (64 coarse + 64 fine), ray-batch sharded over the GPUs",
                   "frames": NMR_FRAMES, "frame": [NMR_SIZE, NMR_SIZE], "rays_per_step": n_batch,
                   "rays_rank0": end - start if rank == 0 else None, "ray_batch_size": RAY_BATCH,
                   "n_coarse": KC, "n_fine": KF, "n_views": 1, "latent": [32, 32],
                   "near_far": [NMR_NEAR, NMR_FAR], "focal": NMR_FOCAL,
                   "parallelism": "contiguous ray ranges, 1 process per GPU, no data-path collective",
                   "per_step": "encode (ResNet34) + latent projection + render + device->host copy"},
        "encode_ms": round(enc_ms, 3),
        "roofline": roof,
        "box_clock": clock.summary() if clock is not None else None,
        "march_mode_bound": MARCH_MODE_BOUND,
        "kernel_ms": {k: round(v, 4) for k, v in avg.items()},
        "l2_stream": l2_stream(roof["points_per_launch"], roof["launch_ms"], args.precision,
                               not args.no_latent_proj),
    }
    if not args.no_train:
        out["train"] = train_leg(dev, rank, world, args.train_steps, 2, precision=args.precision)
    if rank == 0 and world == 1:
        if not args.no_cfg2:
            out["cfg2"] = cfg2_leg(args, dev, probe)
        if not args.no_composite:
            out["composite"] = composite_roofline(dev, ev, pmc_path, same_lease)
        if not args.no_extra:
            out["extra_configs"] = extra_configs(dev, args.precision, not args.no_latent_proj, probe,
                                                 0 if args.no_cpu else 64)
        if not args.no_cpu:
            sd = synth.pixelnerf_state(1)
            out["cpu_baseline"], ref, idx, streams, scene3 = cpu_baselines(sd, nmr, net3, dev, args.cpu_rays)
            out["psnr_vs_reference_path"] = psnr_vs_reference_path(net3, nmr[3][idx], ref, streams, dev, sd,
                                                                   scene3)
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
