"""SRN-layout loader and the PSNR / SSIM evaluation harness.

CPU: the loader against the reference loader's outputs (tests/golden/srn_loader.npz, made
by tests/golden/make_srn_golden.py from src/data/SRNDataset.py), SSIM against a brute-force
window sum, the eval view selection.  GPU: eval_approx end to end on a synthetic dataset.
"""
import numpy as np
import pytest
import torch

from srn_synth import write_srn_dir
from pnr import evaluate
from pnr.data import SRNDataset, get_split_dataset


def _golden():
    import os

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "srn_loader.npz")
    return dict(np.load(path))


def test_srn_loader_matches_reference_fixture(tmp_path):
    g = _golden()
    root = write_srn_dir(str(tmp_path), g)
    for tag, kw in (("native", {}), ("resized", dict(image_size=(12, 12))), ("scaled", dict(world_scale=1.5))):
        d = SRNDataset(root, stage="test", **{"image_size": (24, 24), **kw})
        assert len(d) == g["images"].shape[0]
        np.testing.assert_array_equal(np.array([d.z_near, d.z_far], np.float32), g["%s_near_far" % tag])
        for i in range(len(d)):
            item = d[i]
            for k in ("focal", "c", "images", "masks", "bbox", "poses"):
                ref = g["%s_%d_%s" % (tag, i, k)]
                got = item[k].numpy()
                assert got.shape == ref.shape, (tag, i, k)
                np.testing.assert_allclose(got, ref, rtol=0, atol=1e-6, err_msg="%s %d %s" % (tag, i, k))


def test_get_split_dataset(tmp_path):
    g = _golden()
    root = write_srn_dir(str(tmp_path), g, stage="val")
    d = get_split_dataset("srn", root, want_split="val", training=False)
    assert isinstance(d, SRNDataset) and d.stage == "val" and len(d) == 2
    with pytest.raises(FileNotFoundError):
        get_split_dataset("srn", root, want_split="test")


def _ssim_brute(x, y, win=7, k1=0.01, k2=0.03):
    """Windowed SSIM by explicit sums over each interior 7 x 7 window (sample covariance)."""
    h, w, c = x.shape
    r = win // 2
    n = win * win
    out = []
    for ch in range(c):
        vals = []
        for i in range(r, h - r):
            for j in range(r, w - r):
                a = x[i - r:i + r + 1, j - r:j + r + 1, ch].astype(np.float64).ravel()
                b = y[i - r:i + r + 1, j - r:j + r + 1, ch].astype(np.float64).ravel()
                ma, mb = a.mean(), b.mean()
                va = ((a - ma) ** 2).sum() / (n - 1)
                vb = ((b - mb) ** 2).sum() / (n - 1)
                cov = ((a - ma) * (b - mb)).sum() / (n - 1)
                c1, c2 = k1 ** 2, k2 ** 2
                vals.append((2 * ma * mb + c1) * (2 * cov + c2) / ((ma ** 2 + mb ** 2 + c1) * (va + vb + c2)))
        out.append(np.mean(vals))
    return float(np.mean(out))


def test_ssim_matches_window_sums():
    rng = np.random.default_rng(0)
    x = rng.random((20, 17, 3))
    y = np.clip(x + 0.1 * rng.normal(size=x.shape), 0, 1)
    assert abs(evaluate.ssim(x, y) - _ssim_brute(x, y)) < 1e-10
    assert abs(evaluate.ssim(x, x) - 1.0) < 1e-12
    assert evaluate.psnr_np(x, x) == float("inf")
    assert abs(evaluate.psnr_np(x, y) - (-10 * np.log10(np.mean((x - y) ** 2)))) < 1e-9


def test_select_views_never_picks_a_source():
    torch.manual_seed(0)
    for source in ([64], [3, 10], [-1]):
        for _ in range(20):
            src, dst = evaluate.select_views(5, 100, source)
            assert src.shape[0] == 5 and dst.shape == (5, 1)
            assert bool((dst >= 0).all()) and bool((dst < 100).all())
            assert not bool((src == dst).any())


@pytest.mark.gpu
def test_eval_approx_end_to_end(tmp_path):
    """eval_approx on a synthetic 2-object dataset: finite scores, deterministic for a seed,
    and each object's PSNR equals a direct render of the same target view under the same
    seed (the harness adds no error of its own)."""
    from pnr import synth, util
    from pnr.models import PixelNeRFNet
    from pnr.renderer import NeRFRenderer

    g = _golden()
    root = write_srn_dir(str(tmp_path), g)
    dset = SRNDataset(root, stage="test", image_size=(24, 24))
    dev = torch.device("cuda", 0)
    mlp = dict(type="resnet", n_blocks=5, d_hidden=512, combine_layer=3, combine_type="average")
    conf = dict(use_encoder=True, use_xyz=True, use_code=True, code=dict(num_freqs=6, freq_factor=1.5),
                use_viewdirs=True, use_code_viewdirs=False, mlp_coarse=mlp, mlp_fine=mlp,
                encoder=dict(backbone="resnet34", pretrained=False, num_layers=4))
    torch.manual_seed(0)
    net = PixelNeRFNet(conf)
    net.load_state_dict(synth.pixelnerf_state(2), strict=False)
    net = net.to(dev).eval()

    def run():
        r = NeRFRenderer(n_coarse=32, n_fine=16, white_bkgd=True).to(dev)
        return evaluate.eval_approx(net, r, dset, dev, source=[1], batch_size=2, seed=7)

    res = run()
    assert res["objects"] == 2 and np.isfinite(res["mean_psnr"]) and -1 <= res["mean_ssim"] <= 1
    # repeatable up to the encoder convolutions' fp32 spread (MIOpen may pick another
    # algorithm once its solver search has run)
    np.testing.assert_allclose(run()["psnr"], res["psnr"], rtol=0, atol=1e-5)
    # direct render of object 0's target view with the same draws (the DataLoader iterator
    # takes one draw for its base seed, in eval_approx.py as here)
    torch.random.manual_seed(7)
    data = next(iter(torch.utils.data.DataLoader(dset, batch_size=2, shuffle=False)))
    src, dst = evaluate.select_views(2, 3, [1])
    poses = util.batched_index_select_nd(data["poses"], dst).reshape(-1, 4, 4)
    rays = util.gen_rays(poses, 24, 24, data["focal"][0], dset.z_near, dset.z_far).reshape(2, -1, 8)
    net.encode(util.batched_index_select_nd(data["images"], src).to(dev),
               util.batched_index_select_nd(data["poses"], src).to(dev), data["focal"][0].to(dev))
    r = NeRFRenderer(n_coarse=64, n_fine=16, white_bkgd=True).to(dev)   # eval_approx raises n_coarse to 64
    with torch.no_grad():
        rgb, _ = r.bind_parallel(net, None, simple_output=True)(rays.to(dev))
    gt = util.batched_index_select_nd(data["images"] * 0.5 + 0.5, dst).reshape(2, 3, 24, 24)
    p0 = evaluate.psnr_np(rgb.reshape(2, 24, 24, 3)[0].cpu().numpy(), gt.permute(0, 2, 3, 1)[0].numpy())
    assert abs(p0 - res["psnr"][0]) < 1e-5



@pytest.mark.gpu
def test_eval_approx_psnr_matches_oracle(tmp_path):
    """pnr.evaluate.eval_approx against the oracle restatement of eval_approx.py's scoring
    loop (oracle/eval_ref.py): the same encoded latent, rays and counter-mode draws (replayed
    from the renderer's seed through oracle/philox.py) rendered by the CPU oracle; every
    object's PSNR agrees within 0.01 dB (the north star's PSNR bar)."""
    from oracle import eval_ref, philox
    from pnr import synth
    from pnr.models import PixelNeRFNet
    from pnr.renderer import NeRFRenderer

    g = _golden()
    root = write_srn_dir(str(tmp_path), g)
    dset = SRNDataset(root, stage="test", image_size=(16, 16))
    dev = torch.device("cuda", 0)
    mlp = dict(type="resnet", n_blocks=5, d_hidden=512, combine_layer=3, combine_type="average")
    conf = dict(use_encoder=True, use_xyz=True, use_code=True, code=dict(num_freqs=6, freq_factor=1.5),
                use_viewdirs=True, use_code_viewdirs=False, mlp_coarse=mlp, mlp_fine=mlp,
                encoder=dict(backbone="resnet34", pretrained=False, num_layers=4))
    torch.manual_seed(0)
    sd = synth.pixelnerf_state(2)
    net = PixelNeRFNet(conf)
    net.load_state_dict(sd, strict=False)
    net = net.to(dev).eval()
    rec = []
    enc = net.encode

    def encode(images, poses, focal, *a, **k):
        rec.append(dict(poses=poses.cpu(), focal=focal.cpu(), images=images.cpu()))
        return enc(images, poses, focal, *a, **k)

    net.encode = encode

    class RecRenderer(NeRFRenderer):
        def forward(self, model, rays, want_weights=False):
            out = super().forward(model, rays, want_weights)
            rec[-1].update(rays=rays.cpu(), seed=self.last_seed, latent=model.encoder.latent.detach().cpu())
            return out

    r = RecRenderer(n_coarse=32, n_fine=16, white_bkgd=True).to(dev)
    res = evaluate.eval_approx(net, r, dset, dev, source=[1], batch_size=2, seed=7)
    assert r.rng_mode == "counter" and len(rec) == 1
    b = rec[0]
    SB, HW = b["rays"].shape[:2]
    streams = tuple(torch.from_numpy(a) for a in philox.render_streams(b["seed"], 0, SB * HW, 64, 16, 0))
    # the ground truth as eval_approx picks it (same seed, same draws)
    torch.random.manual_seed(7)
    data = next(iter(torch.utils.data.DataLoader(dset, batch_size=2, shuffle=False)))
    src, dst = evaluate.select_views(2, data["images"].shape[1], [1])
    from pnr import util

    gt = util.batched_index_select_nd(data["images"] * 0.5 + 0.5, dst).reshape(SB, 3, 16, 16).permute(0, 2, 3, 1)
    ps, _ = eval_ref.score_batch(sd, b["latent"], b["poses"].reshape(SB, 1, 4, 4), b["focal"], 16, 16,
                                 b["rays"], streams, gt, 64, 16)
    np.testing.assert_allclose(res["psnr"], ps, rtol=0, atol=0.01)
    print("eval_approx PSNR hip %s oracle %s" % (res["psnr"], ps))


CLI_CONF = """
model {
    use_encoder = True
    use_xyz = True
    use_code = True
    code { num_freqs = 6, freq_factor = 1.5, include_input = True }
    use_viewdirs = True
    use_code_viewdirs = False
    mlp_coarse { type = resnet, n_blocks = 5, d_hidden = 512, combine_layer = 3, combine_type = average }
    mlp_fine { type = resnet, n_blocks = 5, d_hidden = 512, combine_layer = 3, combine_type = average }
    encoder { backbone = resnet34, pretrained = False, num_layers = 4 }
}
renderer {
    n_coarse = 32
    n_fine = 16
    n_fine_depth = 8
    depth_std = 0.01
    white_bkgd = True
}
"""


@pytest.mark.gpu
def test_eval_and_video_scripts_end_to_end(tmp_path):
    """scripts/eval_approx.py and scripts/gen_video.py as a user runs them: HOCON conf,
    checkpoint through load_weights, SRN-layout dataset, on the HIP device."""
    import os
    import subprocess
    import sys

    from pnr import synth

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    g = _golden()
    root = write_srn_dir(str(tmp_path), g)
    (tmp_path / "exp.conf").write_text(CLI_CONF)
    ck = tmp_path / "ck" / "synthnet"
    ck.mkdir(parents=True)
    sd = {k: v for k, v in synth.pixelnerf_state(2).items()}
    # a full state dict: encoder weights from a fresh (random, pretrained=False) encoder
    from pnr.models import make_model
    from pnr.conf import parse_file

    net = make_model(parse_file(str(tmp_path / "exp.conf"))["model"])
    full = net.state_dict()
    full.update(sd)
    torch.save(full, str(ck / "pixel_nerf_latest"))
    common = ["-c", str(tmp_path / "exp.conf"), "-D", root, "-n", "synthnet",
              "--checkpoints_path", str(tmp_path / "ck"), "--split", "test"]
    r = subprocess.run([sys.executable, os.path.join(repo, "scripts", "eval_approx.py"), *common, "-P", "1",
                        "--batch_size", "2"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "final psnr" in r.stdout
    r = subprocess.run([sys.executable, os.path.join(repo, "scripts", "gen_video.py"), *common, "-P", "1",
                        "-S", "1", "--num_views", "3", "--visual_path", str(tmp_path / "vis")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    frames = sorted(os.listdir(tmp_path / "vis" / "synthnet" / "videot0001_v001"))
    assert frames == ["0000.png", "0001.png", "0002.png"]
    assert (tmp_path / "vis" / "synthnet" / "videot0001_v001.gif").exists()


@pytest.mark.gpu
def test_eval_script_density_grid_and_compare(tmp_path):
    """scripts/eval.py (eval/eval.py): the density grid of each object (the point query over a
    res^3 grid in 65,536-point chunks) equals PixelNeRFNet.forward at the same points in this
    process, and --compare writes eval.py's finish.txt line per object."""
    import os
    import subprocess
    import sys

    from pnr import synth
    from pnr.conf import parse_file
    from pnr.models import make_model

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    g = _golden()
    root = write_srn_dir(str(tmp_path), g)
    (tmp_path / "exp.conf").write_text(CLI_CONF)
    ck = tmp_path / "ck" / "synthnet"
    ck.mkdir(parents=True)
    net = make_model(parse_file(str(tmp_path / "exp.conf"))["model"])
    full = net.state_dict()
    full.update(synth.pixelnerf_state(2))
    torch.save(full, str(ck / "pixel_nerf_latest"))
    res = 20
    r = subprocess.run([sys.executable, os.path.join(repo, "scripts", "eval.py"), "-c", str(tmp_path / "exp.conf"),
                        "-D", root, "-n", "synthnet", "--checkpoints_path", str(tmp_path / "ck"), "--split", "test",
                        "-P", "0 1", "--mesh_res", str(res), "--compare", "-O", str(tmp_path / "out")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    dset = get_split_dataset("srn", root, want_split="test", training=False)
    lines = (tmp_path / "out" / "finish.txt").read_text().strip().splitlines()
    assert len(lines) == len(dset)
    dev = torch.device("cuda")
    net.load_state_dict(full)
    net = net.to(dev).eval()
    for i in range(len(dset)):
        data = dset[i]
        name = os.path.basename(data["path"])
        sig = np.load(str(tmp_path / "out" / name / (name + "_sigma.npy")))
        assert sig.shape == (res, res, res) and np.isfinite(sig).all() and (sig >= 0).all()
        fields = lines[i].split()
        assert fields[0] == name and fields[3] == "1" and np.isfinite(float(fields[1]))
        focal = torch.as_tensor(data["focal"], dtype=torch.float32)[None].to(dev)
        with torch.no_grad():
            net.encode(data["images"][:2].to(dev)[None], data["poses"][:2].to(dev)[None], focal,
                       c=data["c"].to(dev)[None])
            grid = torch.linspace(-1, 1, res, device=dev)
            idx = torch.tensor([[0, 0, 0], [3, 7, 11], [19, 19, 19], [10, 2, 17]])
            pts = grid[idx.to(dev)]
            got = torch.relu(net(pts[None], coarse=True, viewdirs=torch.zeros_like(pts[None]))[0, :, 3]).cpu()
        want = torch.from_numpy(sig[idx[:, 0], idx[:, 1], idx[:, 2]])
        assert torch.equal(got, want), (got, want)


# ------------------------------------------------------- DVR / multi-object loaders ----
def _dvr_golden():
    import os

    return dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "dvr_loader.npz")))


def _dvr_inputs(g, tag):
    cams = []
    for o in range(g["%s_images_in" % tag].shape[0]):
        pre = "%s_cam%d_" % (tag, o)
        cams.append({k[len(pre):]: v for k, v in g.items() if k.startswith(pre)})
    return {"images": g["%s_images_in" % tag], "masks": g.get("%s_masks_in" % tag), "cams": cams}


def _check_item(item, g, key_prefix, atol=1e-5):
    for k in ("focal", "c", "images", "masks", "bbox", "poses"):
        ref = g.get(key_prefix + k)
        if ref is None:
            v = item.get(k)
            assert v is None or (isinstance(v, list) and not v), (key_prefix, k)
            continue
        v = item[k]
        got = np.zeros((0,), np.float32) if isinstance(v, list) and not v else np.asarray(
            v.numpy() if torch.is_tensor(v) else v)
        assert got.shape == ref.shape, (key_prefix, k, got.shape, ref.shape)
        np.testing.assert_allclose(got, ref, rtol=1e-6, atol=atol, err_msg=key_prefix + k)


@pytest.mark.parametrize("tag", ["nmr", "nmr_nomask", "nmr_resized", "dtu", "dtu_resized"])
def test_dvr_loader_matches_reference_fixture(tmp_path, tag):
    """pnr.data.DVRDataset against the reference's DVRDataset.py on the same synthetic
    ShapeNet-NMR / DTU directories (tests/golden/make_dvr_golden.py)."""
    import dvr_synth
    from pnr.data import DVRDataset

    g = _dvr_golden()
    kw = {"nmr": {}, "nmr_nomask": {}, "nmr_resized": dict(image_size=(10, 10)),
          "dtu": dict(list_prefix="new_", sub_format="dtu", scale_focal=False, z_near=0.1, z_far=5.0),
          "dtu_resized": dict(list_prefix="new_", sub_format="dtu", scale_focal=False, image_size=(10, 10))}[tag]
    root = dvr_synth.write_dvr_dir(str(tmp_path), _dvr_inputs(g, tag), list_prefix=kw.get("list_prefix", "softras_"))
    d = DVRDataset(root, stage="test", **kw)
    n, near, far = g["%s_meta" % tag]
    assert len(d) == int(n) and d.z_near == near and d.z_far == far and d.lindisp is False
    for i in range(len(d)):
        # DTU poses come from an RQ decomposition: both sides solve the same exact decomposition
        _check_item(d[i], g, "%s_%d_" % (tag, i), atol=2e-5 if tag.startswith("dtu") else 1e-6)


def test_multiobj_loader_matches_reference_fixture(tmp_path):
    import os

    import dvr_synth
    from pnr.data import MultiObjectDataset

    g = _dvr_golden()
    inp = {"images": g["multi_images_in"], "poses": g["multi_poses_in"], "angle": g["multi_angle_in"]}
    d = MultiObjectDataset(dvr_synth.write_multiobj_dir(str(tmp_path), inp), stage="test")
    assert len(d) == inp["images"].shape[0]
    for i in range(len(d)):
        item = d[i]
        _check_item(item, g, "multi_%s_" % os.path.basename(item["path"]))


def test_get_split_dataset_formats(tmp_path):
    import dvr_synth
    from pnr.data import ColorJitterDataset, DVRDataset, MultiObjectDataset

    g = _dvr_golden()
    inp = _dvr_inputs(g, "dtu")
    for st in ("train", "val", "test"):
        root = dvr_synth.write_dvr_dir(str(tmp_path / "dtu"), inp, list_prefix="new_", stage=st)
    tr, va, te = get_split_dataset("dvr_dtu", root)
    assert isinstance(tr, ColorJitterDataset) and isinstance(va, DVRDataset) and isinstance(te, DVRDataset)
    # training=True caps every split at 49 views, as the reference's shared flags do (data/__init__.py:41-42)
    assert tr.base_dset.max_imgs == 49 and va.max_imgs == 49 and tr.sub_format == "dtu"
    assert (tr.z_near, tr.z_far, va.scale_focal) == (0.1, 5.0, False)
    assert get_split_dataset("dvr_dtu", root, want_split="test", training=False).max_imgs == 100000
    inp = _dvr_inputs(g, "nmr")
    root = dvr_synth.write_dvr_dir(str(tmp_path / "gen"), inp, list_prefix="gen_", stage="val")
    assert len(get_split_dataset("dvr_gen", root, want_split="val")) == 2
    m = get_split_dataset("multi_obj", dvr_synth.write_multiobj_dir(str(tmp_path), dvr_synth.make_multiobj_inputs(),
                                                                     stage="val"), want_split="val")
    assert isinstance(m, MultiObjectDataset) and len(m) == 2
    with pytest.raises(NotImplementedError):
        get_split_dataset("llff", str(tmp_path))


def test_color_jitter_is_the_tensor_colour_transform():
    """ColorJitterDataset: zero ranges leave images unchanged; the HSV round trip is the identity;
    brightness / saturation / contrast are the clamped blends; one draw per object."""
    from pnr import data as pdata

    x = torch.rand(2, 3, 6, 7)
    hsv = pdata._rgb_to_hsv(x)
    torch.testing.assert_close(pdata._hsv_to_rgb(hsv), x, atol=1e-6, rtol=0)
    # pure hues land on h = 0, 1/3, 2/3
    prim = torch.eye(3).reshape(3, 3, 1, 1)
    torch.testing.assert_close(pdata._rgb_to_hsv(prim)[:, 0, 0, 0], torch.tensor([0.0, 1 / 3, 2 / 3]))

    class Base(torch.utils.data.Dataset):
        z_near, z_far, lindisp, base_path, image_to_tensor = 1.0, 2.0, False, "b", None

        def __len__(self):
            return 1

        def __getitem__(self, i):
            return {"images": x.clone() * 2 - 1}

    same = pdata.ColorJitterDataset(Base(), 0.0, 0.0, 0.0, 0.0)
    torch.testing.assert_close(same[0]["images"], x * 2 - 1, atol=1e-6, rtol=0)
    j = pdata.ColorJitterDataset(Base())
    np.random.seed(3)
    out = j[0]["images"]
    np.random.seed(3)
    hue, sat, bri, con = (np.random.uniform(-0.1, 0.1), np.random.uniform(0.9, 1.1),
                          np.random.uniform(0.9, 1.1), np.random.uniform(0.9, 1.1))
    y = x[0]
    gray = 0.2989 * y[0] + 0.587 * y[1] + 0.114 * y[2]
    y = (sat * y + (1 - sat) * gray).clamp(0, 1)
    h = pdata._rgb_to_hsv(y)
    y = pdata._hsv_to_rgb(torch.stack(((h[0] + hue) % 1.0, h[1], h[2])))
    m = (0.2989 * y[0] + 0.587 * y[1] + 0.114 * y[2]).mean()
    y = (con * y + (1 - con) * m).clamp(0, 1)
    y = (bri * y).clamp(0, 1)
    torch.testing.assert_close(out[0], y * 2 - 1, atol=1e-6, rtol=0)
    assert float(out.min()) >= -1 and float(out.max()) <= 1


@pytest.mark.parametrize("fmt,tag", [("dvr", "nmr"), ("dvr_dtu", "dtu")])
def test_train_script_keeps_the_loader_image_size(tmp_path, fmt, tag):
    """scripts/train.py: without --image_size the DVR loaders run at their native size
    with their own intrinsics, as train.py:74 calls get_split_dataset with no size; the items equal
    the reference loader's on the same directory (tests/golden/dvr_loader.npz)."""
    import importlib.util
    import os

    import dvr_synth

    spec = importlib.util.spec_from_file_location(
        "pnr_train_script", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts",
                                         "train.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    g = _dvr_golden()
    prefix = "new_" if tag == "dtu" else "softras_"
    for st in ("train", "val", "test"):
        root = dvr_synth.write_dvr_dir(str(tmp_path), _dvr_inputs(g, tag), list_prefix=prefix, stage=st)
    tr, va, te = mod.load_datasets(fmt, root)
    base = tr.base_dset if hasattr(tr, "base_dset") else tr
    item = te[0]
    assert tuple(item["images"].shape[-2:]) == tuple(g["%s_0_images" % tag].shape[-2:])
    _check_item(item, g, "%s_0_" % tag, atol=2e-5 if tag == "dtu" else 1e-6)   # images, focal, c, poses
    assert base.image_size is None
    # an explicit --image_size still resamples
    _, _, te2 = mod.load_datasets(fmt, root, 10)
    assert tuple(te2[0]["images"].shape[-2:]) == (10, 10)
