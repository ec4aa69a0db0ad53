"""CPU-only tests: the C-ABI library's exports, host-side API plumbing, config
parsing, RNG stream order and the no-fallback guarantee."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

import fixtures
from pnr import _lib, conf, ops, synth
from pnr.models import PixelNeRFNet, make_model
from pnr.renderer import DotMap, NeRFRenderer

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "pnr_abi.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pnr_[a-z_]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    names = header_functions()
    assert len(names) >= 12, names
    lib = ctypes.CDLL(_lib.LIB_PATH)  # loads without a GPU; no compute call is made
    for n in names:
        assert hasattr(lib, n), "libpnr.so does not export %s" % n
    # the Python binding declares exactly the header's functions
    assert sorted(_lib.SIGNATURES) == names


def test_abi_version_and_error_channel():
    lib = _lib.load()
    assert lib.pnr_abi_version() == 8
    assert lib.pnr_fold_batchnorm(None, 3, 10, None) == -1 and b"NULL" in lib.pnr_last_error()
    assert lib.pnr_latent_channels_last_backward(None, None, None, None, None, 1, 1, 4, 4, None) == -1
    assert b"NULL" in lib.pnr_last_error()
    # an invalid call fails with a message, without touching the GPU
    rc = lib.pnr_composite(None, None, None, 4, 0, 0, None, None, None, None)
    assert rc == -1
    assert b"bad sizes" in lib.pnr_last_error()
    assert lib.pnr_mlp_packed_bytes(_lib.MlpDesc(42, 256, 256, 4, 5, 3, 12)) == 0
    assert b"512" in lib.pnr_last_error()
    sz = lib.pnr_mlp_packed_bytes(_lib.MlpDesc(42, 512, 512, 4, 5, 3, 12))
    # 13 K=512 layers + lin_in (4 k-blocks) + lin_out + biases, in bytes
    assert 13 * 512 * 512 * 4 < sz < 13 * 512 * 512 * 4 + 600000


def test_ops_refuse_cpu_tensors():
    with pytest.raises(ValueError, match="HIP device"):
        ops.composite(torch.zeros(2, 3), torch.zeros(2, 3, 4), torch.zeros(2, 8), True)
    with pytest.raises(ValueError, match="HIP device"):
        ops.sample_coarse(torch.zeros(2, 8), 4, torch.zeros(2, 4))


def _conf_dict():
    mlp = dict(type="resnet", n_blocks=5, d_hidden=512, combine_layer=3, combine_type="average")
    return dict(use_encoder=True, use_xyz=True, use_code=True,
                code=dict(num_freqs=6, freq_factor=1.5, include_input=True), use_viewdirs=True,
                use_code_viewdirs=False, mlp_coarse=mlp, mlp_fine=dict(mlp),
                encoder=dict(backbone="resnet34", pretrained=False, num_layers=4))


def test_model_state_dict_matches_reference_layout():
    net = make_model(_conf_dict())
    sd = net.state_dict()
    ours = sorted(k for k in sd if not k.startswith("encoder."))
    ref = sorted(synth.pixelnerf_state(0).keys())
    assert ours == ref and len(ours) == 62
    for k in ref:
        assert tuple(sd[k].shape) == tuple(synth.pixelnerf_state(0)[k].shape), k
    assert net.d_in == 42 and net.d_latent == 512
    # torchvision resnet34 minus fc: 216 encoder tensors
    assert sum(1 for k in sd if k.startswith("encoder.model.")) == 216


def test_encode_builds_camera_records():
    cfg, arr = fixtures.load("rw_ns3_sb2")
    net = make_model(_conf_dict())
    lat = torch.zeros(6, 512, 4, 5)
    net.encode_latent(lat, arr["poses"], arr["focal"], (cfg["width"], cfg["height"]), c=arr["c"],
                      num_objs=2)
    assert net.num_objs == 2 and net.num_views_per_obj == 3
    cams = net.cams
    assert cams.shape == (6, 16)
    # R_wc = R^T, t_wc = -R^T t (models.py:112-114); fy negated (models.py:130)
    p = arr["poses"].reshape(6, 4, 4)
    R = p[:, :3, :3].transpose(1, 2)
    torch.testing.assert_close(cams[:, :9], R.reshape(6, 9))
    torch.testing.assert_close(cams[:, 9:12], -(R @ p[:, :3, 3:])[..., 0])
    torch.testing.assert_close(cams[3:, 12:14], torch.tensor([[280.0, -290.0]] * 3))
    torch.testing.assert_close(cams[:3, 14:16], torch.tensor([[195.0, 152.0]] * 3))
    assert net.encoder.latent_cl.shape == (6, 4, 5, 512)
    # the HIP path refuses CPU tensors loudly (no CPU fallback)
    with torch.no_grad(), pytest.raises(ValueError, match="HIP device"):
        net(torch.zeros(2, 4, 3), coarse=True, viewdirs=torch.zeros(2, 4, 3))


def test_grad_point_query_routes_to_training_forward_and_refuses_cpu():
    """eval/eval.py:100 and train/train.py:422 query the net with grad enabled: the query builds
    its autograd graph through train.RenderPoints (tests/test_gpu_parity.py checks its values and
    gradients on the device); CPU tensors are refused loudly, as on every HIP path."""
    net = make_model(_conf_dict())
    net.encode_latent(torch.zeros(1, 512, 4, 4), synth.srn_poses([0.0]), torch.tensor(50.0), (32, 32))
    assert torch.is_grad_enabled() and net.needs_grad()
    with pytest.raises(ValueError, match="HIP device"):
        net(torch.zeros(1, 2, 3), coarse=True, viewdirs=torch.zeros(1, 2, 3))


def test_renderer_draws_streams_in_reference_order():
    """Same seed -> the same four streams the fixtures replay (nerf.py:111,135,141,158)."""
    r = NeRFRenderer(n_coarse=16, n_fine=16, n_fine_depth=8)
    torch.manual_seed(1)
    got = r.draw_streams(64, torch.device("cpu"))
    exp = synth.rng_streams(1, 64, 16, 16, 8)
    for a, b in zip(got, exp):
        assert torch.equal(a, b)
    cfg, arr = fixtures.load("rw_lindisp")   # streams as stored by make_golden.py
    r2 = NeRFRenderer(n_coarse=cfg["n_coarse"], n_fine=cfg["n_fine"], n_fine_depth=cfg["n_fine_depth"])
    torch.manual_seed(cfg["rng_seed"])
    got = r2.draw_streams(arr["rays"].reshape(-1, 8).shape[0], torch.device("cpu"))
    for a, k in zip(got, ["u_coarse", "u_fine", "u_fine_jit", "n_depth"]):
        assert torch.equal(a, arr[k]), k


def test_renderer_from_conf_and_sched():
    c = conf.Conf(dict(n_coarse=64, n_fine=32, n_fine_depth=16, depth_std=0.01, white_bkgd=True,
                       sched=[[10, 20], [32, 16], [16, 8]]))
    r = NeRFRenderer.from_conf(c, lindisp=False, eval_batch_size=5000)
    assert (r.n_coarse, r.n_fine, r.n_fine_depth, r.using_fine, r.eval_batch_size) == (64, 32, 16, True, 5000)
    r.sched_step(10)
    assert (r.n_coarse, r.n_fine) == (32, 16)
    r.sched_step(15)
    assert (r.n_coarse, r.n_fine) == (16, 8) and int(r.last_sched) == 2
    sd = r.state_dict()
    assert set(sd) == {"iter_idx", "last_sched"}


def test_dotmap_todict():
    d = DotMap(coarse=DotMap(rgb=1), x=2)
    assert d.coarse.rgb == 1 and d.toDict() == {"coarse": {"rgb": 1}, "x": 2}


def test_hocon_subset_parser(tmp_path):
    (tmp_path / "base.conf").write_text(
        "# base\nmodel {\n  use_xyz = True\n  code { num_freqs = 6\n freq_factor = 1.5 }\n"
        "  mlp_coarse { type = resnet  # comment\n n_blocks = 3 }\n}\nrenderer { sched = [] }\n")
    (tmp_path / "exp.conf").write_text(
        'include required("base.conf")\nmodel {\n  mlp_coarse { n_blocks = 5, d_hidden = 512 }\n}\n'
        "renderer.n_coarse = 64\n")
    c = conf.parse_file(str(tmp_path / "exp.conf"))
    m = c["model"]
    assert m.get_bool("use_xyz") is True and m["code"].get_float("freq_factor") == 1.5
    assert m["mlp_coarse"].get_string("type") == "resnet"
    assert m["mlp_coarse"].get_int("n_blocks") == 5 and m["mlp_coarse"].get_int("d_hidden") == 512
    assert c["renderer"].get_int("n_coarse") == 64 and c["renderer"].get_list("sched") == []
    assert c.get_int("missing", 7) == 7


@pytest.mark.skipif(not os.path.isdir("/root/reference/conf"), reason="reference confs absent")
def test_parser_reads_reference_confs():
    for name in ("srn", "sn64", "dtu"):
        c = conf.parse_file("/root/reference/conf/exp/%s.conf" % name)
        net = PixelNeRFNet(dict(c["model"], encoder=dict(c["model"]["encoder"], pretrained=False)))
        assert net.d_in == 42 and net.mlp_coarse.n_blocks == 5
        assert net.hip_unsupported_reason() == "encode() has not been called"


def test_torch_ops_registered_with_meta_shapes():
    """torch.ops.pnr.{render_rays, point_query, composite} (libpnr_torch.so, TORCH_LIBRARY over
    the C ABI) load on the CPU host and give their output shapes on meta tensors (FakeTensor /
    torch.compile tracing) -- no compute without a GPU."""
    import torch

    from pnr import torchops

    ops = torchops.load()
    m = dict(device="meta")
    rays = torch.empty(6, 8, **m)
    w, rgb, depth = ops.composite(torch.empty(6, 9, **m), torch.empty(6, 9, 4, **m), rays, True, True)
    assert (w.shape, rgb.shape, depth.shape) == ((6, 9), (6, 3), (6,))
    lat, cams, pk = torch.empty(1, 32, 32, 512, **m), torch.empty(1, 16, **m), torch.empty(8, **m)
    desc = [42, 512, 512, 4, 5, 3, 12, 3]
    out = ops.render_rays(lat, cams, 1, 1, 64.0, 64.0, desc, pk, pk, None, None, rays, 6, 64, 32, 16, 0.01,
                          True, False, None, None, None, None, 7, 0, True, True, [], 1)
    assert [tuple(t.shape) for t in out] == [(6, 3), (6,), (6, 64), (6, 3), (6,), (6, 96), (6, 64), (6, 96)]
    q = ops.point_query(lat, cams, 1, 1, 64.0, 64.0, desc, pk, None, torch.empty(1, 10, 3, **m), None)
    assert tuple(q.shape) == (1, 10, 4)


def test_pack_key_tracks_weight_changes():
    """ResnetFC._pack_key (the packed-weight cache of the HIP path) changes on an in-place
    update, a reassigned parameter and a swapped submodule, and stays put otherwise (the
    cached submodule list keeps its per-call host cost at ~30 us instead of ~100 us)."""
    import copy

    from pnr.models import PixelNeRFNet

    mlp = dict(type="resnet", n_blocks=5, d_hidden=512, combine_layer=3, combine_type="average")
    conf = dict(use_encoder=True, use_xyz=True, use_code=True, code=dict(num_freqs=6, freq_factor=1.5),
                use_viewdirs=True, use_code_viewdirs=False, mlp_coarse=mlp, mlp_fine=mlp,
                encoder=dict(backbone="resnet34", pretrained=False, num_layers=4))
    net = PixelNeRFNet(conf)
    m = net.mlp_coarse
    k0 = m._pack_key(net.code, "f16x3")
    assert m._pack_key(net.code, "f16x3") == k0
    assert m._pack_key(net.code, "fp32") != k0
    with torch.no_grad():
        m.blocks[0].fc_0.weight.mul_(1.0)
    k1 = m._pack_key(net.code, "f16x3")
    assert k1 != k0
    m.lin_out.bias = torch.nn.Parameter(m.lin_out.bias.detach().clone())
    k2 = m._pack_key(net.code, "f16x3")
    assert k2 != k1
    m.blocks[2] = copy.deepcopy(m.blocks[2])
    assert m._pack_key(net.code, "f16x3") != k2


def test_render_set_fused_modes():
    """pnr_render_set_fused (host state only, no device work): default 2, returns the previous
    mode, out-of-range values select the default; pnr._lib.fused_march restores the mode."""
    lib = _lib.load()
    prev = lib.pnr_render_set_fused(2)
    try:
        assert lib.pnr_render_set_fused(0) == 2
        assert lib.pnr_render_set_fused(1) == 0
        assert lib.pnr_render_set_fused(3) == 1
        assert lib.pnr_render_set_fused(7) == 3     # invalid -> default
        assert lib.pnr_render_set_fused(2) == 2
        with _lib.fused_march(0):
            assert lib.pnr_render_set_fused(0) == 0
        assert lib.pnr_render_set_fused(2) == 2
    finally:
        lib.pnr_render_set_fused(prev)


def test_render_cfg_march_mode_is_per_call():
    """ABI 3: pnr_render_cfg.march_mode names the march schedule of one call; a value outside
    -1..3 is refused before any device work (host-side validation only: the pointers below
    are never dereferenced), and the refusal does not touch the process default."""
    lib = _lib.load()
    assert ctypes.sizeof(_lib.RenderCfg) == 40   # ABI 8: + ray_order (8-B aligned at 32)
    buf = ctypes.create_string_buffer(4096 + 16)
    p = ctypes.c_void_p((ctypes.addressof(buf) + 15) & ~15)   # 16-B aligned, never read
    sc = _lib.Scene(p, p, 1, 1, 4, 4, 512, 64.0, 64.0)
    desc = _lib.MlpDesc(42, 512, 512, 4, 5, 3, 12, 3)
    rays = _lib.Rays(p, 4, 4)
    rng = _lib.Rng(None, None, None, None, 1, 0)
    out = _lib.RenderOut(p, p, None, p, p, None, None, None)
    prev = lib.pnr_render_set_fused(2)
    try:
        for bad in (-2, 4, 7):
            cfg = _lib.RenderCfg(64, 64, 0, 0.01, 1, 0, bad)
            rc = lib.pnr_render_forward_proj(ctypes.byref(sc), ctypes.byref(desc), p, p, None, None,
                                             ctypes.byref(rays), ctypes.byref(rng), ctypes.byref(cfg),
                                             ctypes.byref(out), p, 0, None, None)
            assert rc == -1 and b"march_mode" in lib.pnr_last_error(), (bad, rc, lib.pnr_last_error())
        assert lib.pnr_render_set_fused(2) == 2
    finally:
        lib.pnr_render_set_fused(prev)


def test_callback_confs_and_state_dict_layout():
    """Confs the fused kernel does not implement are recognised (fused_conf_reason), keep the
    reference's state-dict layout (scale_z with use_spade, global_encoder.* with the global
    encoder), and the callback forward refuses CPU tensors like the fused path."""
    base = _conf_dict()
    cases = {
        "softplus": dict(base, mlp_coarse=dict(base["mlp_coarse"], beta=100.0)),
        "d_hidden": dict(base, mlp_fine=dict(base["mlp_fine"], d_hidden=256)),
        "latent": dict(base, encoder=dict(base["encoder"], num_layers=3)),
        "viewdirs": dict(base, use_code_viewdirs=True),
        "spade": dict(base, mlp_coarse=dict(base["mlp_coarse"], use_spade=True)),
        "combine": dict(base, mlp_coarse=dict(base["mlp_coarse"], combine_type="max")),
        "global": dict(base, use_global_encoder=True,
                       global_encoder=dict(backbone="resnet34", pretrained=False, latent_size=128)),
        "padding": dict(base, encoder=dict(base["encoder"], index_padding="zeros")),
    }
    for name, c in cases.items():
        net = PixelNeRFNet(c)
        assert net.fused_conf_reason() is not None, name
        with pytest.raises(ValueError, match="HIP device"):
            net(torch.zeros(1, 2, 3), coarse=True, viewdirs=torch.zeros(1, 2, 3))
    assert PixelNeRFNet(base).fused_conf_reason() is None
    sd = PixelNeRFNet(cases["spade"]).state_dict()
    assert sd["mlp_coarse.scale_z.2.weight"].shape == (512, 512) and "mlp_fine.scale_z.0.weight" not in sd
    g = PixelNeRFNet(cases["global"])
    assert g.d_latent == 640 and g.mlp_coarse.lin_z[0].weight.shape == (512, 640)
    assert g.state_dict()["global_encoder.fc.weight"].shape == (128, 512)
    assert PixelNeRFNet(cases["viewdirs"]).d_in == 78


def test_inference_trunk_fold_table_follows_the_module():
    """pnr.encoder.InferenceTrunk (the eval-mode encode) builds its pnr_fold_batchnorm records from
    the LIVE module on every encode: one record per (conv, bn) pair with the tensors' current
    storage, and a new table when a tensor is replaced (load_state_dict(assign=True)) or a module
    swapped -- the cases a version-counter key misses.  The fold arithmetic itself and
    the graph replay run on the device (tests/test_gpu_parity.py::test_eval_encode_*); a deepcopy /
    pickle of an encoder never carries the trunk's graphs."""
    import copy
    import pickle

    from pnr.encoder import InferenceTrunk, SpatialEncoder, _BnFold

    enc = SpatialEncoder(pretrained=False).eval()
    t = InferenceTrunk(enc, torch.device("cpu"))
    t.refresh()
    assert len(t.pairs) == 1 + 2 * (3 + 4 + 6) + 2   # conv1, layer1-3 blocks, 2 downsamples

    def records():
        return (_BnFold * len(t.pairs)).from_buffer_copy(t.table.numpy().tobytes())

    for r, (conv, bn), (w_out, b_out) in zip(records(), t.pairs, t.folded):
        assert r.conv_w == conv.weight.data_ptr() and r.var == bn.running_var.data_ptr()
        assert r.gamma == bn.weight.data_ptr() and r.w_out == w_out.data_ptr() and r.b_out == b_out.data_ptr()
        assert (r.n_out, r.per_out) == (conv.out_channels, conv.weight[0].numel()) and abs(r.eps - bn.eps) < 1e-12
        assert w_out.shape == conv.weight.shape and w_out.stride() == conv.weight.stride()
    assert t.max_elems == max(c.weight.numel() for c, _ in t.pairs)
    key = t.key
    with torch.no_grad():
        enc.model.layer1[0].conv1.weight.data.copy_(torch.randn_like(enc.model.layer1[0].conv1.weight))
    t.refresh()
    assert t.key == key   # same storage: the in-kernel fold reads the new values on the next replay
    sd = {k: v.clone() for k, v in enc.state_dict().items()}
    enc.load_state_dict(sd, assign=True)
    t.refresh()
    assert t.key != key and records()[0].conv_w == enc.model.conv1.weight.data_ptr()
    enc.model.layer3[0].bn1 = torch.nn.BatchNorm2d(256, eps=1e-3)   # a swapped module
    t.refresh()
    i = next(k for k, (_, b) in enumerate(t.pairs) if b is enc.model.layer3[0].bn1)
    assert abs(records()[i].eps - 1e-3) < 1e-9 and records()[i].var == enc.model.layer3[0].bn1.running_var.data_ptr()
    enc._infer = t
    assert copy.deepcopy(enc)._infer is None and enc._infer is t
    assert pickle.loads(pickle.dumps(enc))._infer is None
    enc.invalidate_inference_cache()
    assert enc._infer is None


def test_inference_trunk_refuses_batchnorm_without_running_stats():
    """a BatchNorm with track_running_stats=False (running_mean / running_var None) or
    affine=False has no tensors for k_fold_bn to read, and in eval mode normalizes by the batch's
    statistics, which no fold represents: such an encoder takes the module path (_use_infer is
    False on any device), and the trunk itself raises instead of handing the kernel NULL."""
    from pnr.encoder import InferenceTrunk, SpatialEncoder, _bn_foldable

    enc = SpatialEncoder(pretrained=False).eval()
    assert _bn_foldable(enc.model)
    for bad in (torch.nn.BatchNorm2d(128, track_running_stats=False), torch.nn.BatchNorm2d(128, affine=False)):
        enc.model.layer2[1].bn2 = bad
        assert not _bn_foldable(enc.model)
        with pytest.raises(ValueError, match="running"):
            InferenceTrunk(enc, torch.device("cpu")).refresh()
        with torch.no_grad():   # the module path still encodes (on the CPU here)
            assert torch.isfinite(enc(torch.rand(1, 3, 32, 32))).all()


_LINT_BAD = """\
_ZN3pnr4mlpk11k_point_mlpILi6ELb1ELb1EEEvNS0_4ArgsE:
\tv_mov_b32_e32 v5, v0
\tv_cmp_eq_u32_e64 s[10:11], 0, v5
\ts_mov_b64 s[6:7], exec
\ts_and_b64 s[10:11], s[6:7], s[10:11]
\ts_mov_b64 exec, s[10:11]
\ts_cbranch_execz .LBB12_21
; %bb.7:
\tglobal_atomic_add v3, v0, v3, s[24:25] sc0
.LBB12_21:
\ts_mov_b32 s20, s34
\tscratch_store_dword off, v5, off offset:4 ; 4-byte Folded Spill
\ts_or_b64 exec, exec, s[6:7]
\ts_barrier
\tscratch_load_dword v49, off, off offset:4 ; 4-byte Folded Reload
.Lfunc_end12:
"""


def test_isa_lint_flags_a_spill_under_a_branch_mask(tmp_path):
    """pixel-nerf_amd/isa_lint.py (the build's check): the round-5 fault pattern --
    k_point_mlp<6,true,true> of the 8299515 tree spilled the thread id in the join block of
    `if (tid == 0)` before the EXEC restore -- is rejected; the same spill after the restore, or a
    spill inside a region (after its own EXEC write), is not."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("isa_lint", os.path.join(REPO, "pixel-nerf_amd", "isa_lint.py"))
    lint = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(lint)
    bad = tmp_path / "bad.s"
    bad.write_text(_LINT_BAD)
    hits = lint.lint_file(str(bad))
    assert len(hits) == 1 and "offset:4" in hits[0][2] and hits[0][0].endswith("ArgsE")
    assert lint.main([str(bad)]) == 1
    good = tmp_path / "good.s"
    good.write_text(_LINT_BAD.replace("\tscratch_store_dword off, v5, off offset:4 ; 4-byte Folded Spill\n"
                                      "\ts_or_b64 exec, exec, s[6:7]\n",
                                      "\ts_or_b64 exec, exec, s[6:7]\n"
                                      "\tscratch_store_dword off, v5, off offset:4 ; 4-byte Folded Spill\n"))
    assert lint.lint_file(str(good)) == [] and lint.main([str(good)]) == 0
    inside = tmp_path / "inside.s"   # a reload inside the region: its own mask write comes first
    inside.write_text(_LINT_BAD.replace("\ts_mov_b32 s20, s34\n", "\ts_and_saveexec_b64 s[8:9], vcc\n"))
    assert lint.lint_file(str(inside)) == []
    wwm = tmp_path / "wwm.s"   # a whole-wave SGPR-spill section between the spill and the restore
    wwm.write_text(_LINT_BAD.replace("\ts_or_b64 exec, exec, s[6:7]\n",
                                     "\ts_or_saveexec_b64 s[10:11], -1\n\tscratch_store_dword off, v255, off\n"
                                     "\ts_mov_b64 exec, s[10:11]\n\ts_or_b64 exec, exec, s[6:7]\n"))
    hits = lint.lint_file(str(wwm))
    assert len(hits) == 1 and "v5" in hits[0][2]


def test_built_device_code_passes_isa_lint():
    """Every device object of the in-tree build (the Makefile keeps each one's assembly as
    build/<source>.gfx950.s) is free of spills under a branch's lane mask."""
    import glob
    import importlib.util

    files = sorted(glob.glob(os.path.join(REPO, "pixel-nerf_amd", "build", "*.gfx950.s")))
    if not files:
        pytest.skip("no in-tree build (make -C pixel-nerf_amd)")
    names = {os.path.basename(f) for f in files}
    assert {"mlp.hip.gfx950.s", "march.hip.gfx950.s", "train.hip.gfx950.s", "wgrad.hip.gfx950.s"} <= names
    spec = importlib.util.spec_from_file_location("isa_lint", os.path.join(REPO, "pixel-nerf_amd", "isa_lint.py"))
    lint = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(lint)
    for f in files:
        assert lint.lint_file(f) == [], f


def test_ray_block_order_groups_neighbouring_pixels():
    """pnr.renderer.ray_block_order (the ray_order heuristic, ABI 8): on a pinhole camera's
    row-major frame (util.gen_rays) it is a permutation whose every run of 256 consecutive rays
    covers a compact pixel block (a row-major run spans 256 pixels of one or two rows), for the
    frame and for gen_video's 50,000-ray chunks of it; it keeps the input order for rays without
    a common centre of projection; "auto" blocks only scenes
    whose projected-latent rows exceed ORDER_AUTO_BYTES."""
    from pnr import renderer as rmod
    from pnr import util

    W, H = 400, 300
    rays = util.gen_rays(synth.srn_poses([10.0], phi=-12.0, radius=2.0), W, H, torch.tensor(300.0), 0.1, 5.0)
    rays = rays.reshape(-1, 8)
    order = rmod.ray_block_order(rays)
    assert order.dtype == torch.int32 and torch.equal(torch.sort(order.long())[0], torch.arange(W * H))
    ys, xs = order.long() // W, order.long() % W
    spans = []
    for i in range(0, W * H - 255, 256):
        y, x = ys[i:i + 256], xs[i:i + 256]
        spans.append(max(int(y.max() - y.min()), int(x.max() - x.min())))
    spans.sort()
    assert spans[len(spans) // 2] <= 40, spans[len(spans) // 2]   # ~16-32 px blocks, not 256-px rows
    for r0 in (0, 50000, 100000):   # gen_video's chunks (each a row-major band of the frame)
        o = rmod.ray_block_order(rays[r0:r0 + 50000]).long() + r0
        y, x = o // W, o % W
        med = sorted(max(int(y[i:i + 256].max() - y[i:i + 256].min()), int(x[i:i + 256].max() - x[i:i + 256].min()))
                     for i in range(0, len(o) - 255, 256))[len(o) // 512]
        assert med <= 40, (r0, med)
    rnd = rays.clone()
    rnd[:, :3] += torch.randn(W * H, 3)   # no common centre of projection: the input order
    assert torch.equal(rmod.ray_block_order(rnd), torch.arange(W * H, dtype=torch.int32))
    assert rmod.ray_block_order(rays[:100]) is None

    class Enc:
        latent_cl = torch.empty(3, 150, 200, 512)

    class Mlp:
        combine_layer, n_blocks = 3, 5

    class Net:
        encoder, mlp_coarse = Enc(), Mlp()

    r = rmod.NeRFRenderer()
    assert r.ray_order == "auto" and r._blocked_order(Net())   # cfg4: 553 MB of projected rows
    Net.encoder.latent_cl = torch.empty(1, 32, 32, 512)
    assert not r._blocked_order(Net())                           # cfg3: 6 MB
    r.ray_order = "blocked"
    assert r._blocked_order(Net())
    r.ray_order = "sideways"
    with pytest.raises(ValueError):
        r._blocked_order(Net())


def _torchvision_resnet34_keys():
    """torchvision.models.resnet34's state-dict names and shapes (BasicBlock x [3, 4, 6, 3],
    widths 64 / 128 / 256 / 512, a 1x1-conv + BatchNorm downsample on the first block of layers
    2-4), without fc: the reference replaces fc and avgpool by empty Sequentials (encoder.py:66-67).
    Restated from torchvision's published architecture (torchvision is absent offline)."""
    keys = {"conv1.weight": (64, 3, 7, 7)}

    def bn(prefix, c):
        for n in ("weight", "bias", "running_mean", "running_var"):
            keys["%s.%s" % (prefix, n)] = (c,)
        keys[prefix + ".num_batches_tracked"] = ()

    bn("bn1", 64)
    cin = 64
    for li, (blocks, c) in enumerate(zip((3, 4, 6, 3), (64, 128, 256, 512)), 1):
        for b in range(blocks):
            p = "layer%d.%d" % (li, b)
            keys[p + ".conv1.weight"] = (c, cin if b == 0 else c, 3, 3)
            bn(p + ".bn1", c)
            keys[p + ".conv2.weight"] = (c, c, 3, 3)
            bn(p + ".bn2", c)
            if b == 0 and li > 1:
                keys[p + ".downsample.0.weight"] = (c, cin, 1, 1)
                bn(p + ".downsample.1", c)
        cin = c
    return keys


def test_encoder_state_dict_matches_torchvision_resnet34_names_and_shapes():
    """A reference checkpoint's ``encoder.model.*`` entries load by name and shape (models.py:268-298,
    strict): every key of the in-repo trunk is torchvision ResNet-34's, with its shape, in its order."""
    from pnr.encoder import SpatialEncoder

    got = {k: tuple(v.shape) for k, v in SpatialEncoder(pretrained=False).model.state_dict().items()}
    exp = _torchvision_resnet34_keys()
    assert list(got) == list(exp)
    assert got == exp
    net_keys = [k for k in PixelNeRFNet(_conf_dict()).state_dict() if k.startswith("encoder.")]
    assert net_keys == ["encoder.model." + k for k in exp]


def _encoder_fixture():
    import json
    import os

    g = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "encoder_fw.npz")))
    return g, json.loads(bytes(g["cases"]).decode())


def test_encoder_forward_matches_reference_fixture_cpu():
    """The module path of pnr.encoder.SpatialEncoder.forward on the CPU against the reference's own
    SpatialEncoder.forward (encoder.py:111-164; tests/golden/make_encoder_golden.py): feature_scale,
    use_first_pool, num_layers 3 / 4, the align_corners upsample + concat and latent_scaling, in eval
    mode and in train mode (batch statistics, and the running-statistics update)."""
    from pnr.encoder import SpatialEncoder

    g, cases = _encoder_fixture()
    imgs = torch.from_numpy(g["images"])
    for i, c in enumerate(cases):
        enc = SpatialEncoder(pretrained=False, num_layers=c["num_layers"], feature_scale=c["feature_scale"],
                             use_first_pool=c["use_first_pool"])
        enc.model.load_state_dict(synth.encoder_state(int(g["weight_seed"]), enc.model.state_dict()))
        enc.train(c["train"])
        with torch.no_grad():
            lat = enc(imgs if c["train"] else imgs[:1])
        ref = torch.from_numpy(g["latent_%d" % i])
        assert lat.shape == ref.shape, (c, lat.shape)
        scale = float(ref.abs().max())
        # eval: 1e-6 of the latent's range (measured 2e-7); train: batch statistics over 2 x 12 x 12
        # values amplify the convolutions' fp32 reordering (channels-last here) to ~1.2e-5
        tol = 3e-5 if c["train"] else 1e-6
        assert float((lat - ref).abs().max()) <= tol * scale + 1e-7, (c, float((lat - ref).abs().max()), scale)
        torch.testing.assert_close(enc.latent_scaling, torch.from_numpy(g["latent_scaling_%d" % i]))
        if c["train"]:
            torch.testing.assert_close(enc.model.bn1.running_mean, torch.from_numpy(g["running_mean_after_%d" % i]))
