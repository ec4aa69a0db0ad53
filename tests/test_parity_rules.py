"""The fine-pass flip rule of the parity tests (oracle/parity.py), on CPU.

A searchsorted bin flip is proven from the coarse weights: these tests perturb the
reference's coarse weights of a fixture (as the HIP reduction order does, but larger),
redraw the fine samples from the perturbed weights with the reference algorithm, and check
that the classifier flags exactly the rays whose bins moved, and catches both kinds of
kernel bug: a fine sample set that differs without a flip, and a flipped ray whose samples
do not follow its own coarse weights.
"""
import torch

import fixtures
from oracle import parity


def _case(scale):
    cfg, arr = fixtures.load("fw_cfg2_b128")
    B = arr["rays"].reshape(-1, 8).shape[0]
    w_ref = arr["coarse_weights"].reshape(B, -1)
    g = torch.Generator().manual_seed(3)
    w_hip = w_ref * (1.0 + scale * torch.randn(w_ref.shape, generator=g))
    streams = (arr["u_coarse"], arr["u_fine"], arr["u_fine_jit"], arr["n_depth"])
    z_hip = parity.expected_fine_z(arr["rays"], arr["z_coarse"], w_hip, arr["coarse_depth"], streams,
                                   cfg["n_coarse"], cfg["n_fine"], cfg["n_fine_depth"])
    return cfg, arr, B, w_ref, w_hip, z_hip


def test_expected_fine_z_reproduces_the_reference_samples():
    cfg, arr, B, w_ref, _, _ = _case(0.0)
    streams = (arr["u_coarse"], arr["u_fine"], arr["u_fine_jit"], arr["n_depth"])
    z = parity.expected_fine_z(arr["rays"], arr["z_coarse"], w_ref, arr["coarse_depth"], streams,
                               cfg["n_coarse"], cfg["n_fine"], cfg["n_fine_depth"])
    torch.testing.assert_close(z, arr["z_fine"].reshape(B, -1), atol=1e-6, rtol=0)


def test_flips_are_exactly_the_rays_whose_bins_moved():
    cfg, arr, B, w_ref, w_hip, z_hip = _case(2e-3)
    bins_moved = (parity.fine_bins(w_hip, arr["u_fine"]) != parity.fine_bins(w_ref, arr["u_fine"])).any(-1)
    assert 0 < int(bins_moved.sum()) < B
    cls = parity.classify_fine(w_hip, w_ref, arr["u_fine"], z_hip, arr["z_fine"], z_hip)
    assert torch.equal(cls["flip"], bins_moved)
    assert not cls["unexplained"].any() and not cls["inconsistent"].any()
    # every ray without a flip has the reference's samples
    keep = ~cls["flip"]
    torch.testing.assert_close(z_hip[keep], arr["z_fine"].reshape(B, -1)[keep], atol=1e-6, rtol=0)


def test_classifier_catches_sample_errors():
    cfg, arr, B, w_ref, w_hip, z_hip = _case(2e-3)
    cls = parity.classify_fine(w_hip, w_ref, arr["u_fine"], z_hip, arr["z_fine"], z_hip)
    ok_ray = int(torch.nonzero(~cls["flip"])[0])
    flip_ray = int(torch.nonzero(cls["flip"])[0])
    bad = z_hip.clone()
    bad[ok_ray, 5] += 1e-3          # a sample moved on a ray whose bins did not
    cls = parity.classify_fine(w_hip, w_ref, arr["u_fine"], bad, arr["z_fine"], z_hip)
    assert cls["unexplained"].nonzero().reshape(-1).tolist() == [ok_ray]
    bad = z_hip.clone()
    bad[flip_ray, 7] += 1e-3        # a flipped ray that does not follow its own weights
    cls = parity.classify_fine(w_hip, w_ref, arr["u_fine"], bad, arr["z_fine"], z_hip)
    assert cls["inconsistent"].nonzero().reshape(-1).tolist() == [flip_ray]


def test_marginal_draws_may_take_either_neighbouring_bin():
    """A draw ON a cdf boundary (fw_shipped's force_u_high rays: u = 1 - 2^-24 against
    cdf[-1] = 1 +- ulp) may land in either bin from the same weights, because the device
    sums the normaliser in another order; the alternative set moves exactly those draws, and
    a sample set that is neither the expected nor the alternative still fails."""
    cfg, arr = fixtures.load("fw_shipped")
    B = arr["rays"].reshape(-1, 8).shape[0]
    w = arr["coarse_weights"].reshape(B, -1)
    streams = (arr["u_coarse"], arr["u_fine"], arr["u_fine_jit"], arr["n_depth"])
    args = (arr["rays"], arr["z_coarse"], w, arr["coarse_depth"], streams, cfg["n_coarse"], cfg["n_fine"],
            cfg["n_fine_depth"], cfg.get("depth_std", 0.01))
    z0, z1 = parity.expected_fine_sets(*args)
    marginal = parity.boundary_distance(w, arr["u_fine"]) <= parity.MARGIN
    moved = (z0 != z1).any(-1)
    assert int(marginal[: cfg["force_u_high"]].sum()) == cfg["force_u_high"]
    assert torch.equal(moved, moved & marginal) and bool(moved.any())
    # a HIP ray that took the other bin of a boundary draw, with flip evidence: consistent
    flip_w = w.clone()
    cls = parity.classify_fine(flip_w, w, arr["u_fine"], z1, z0, (z0, z1))
    assert not cls["inconsistent"].any()
    # a set that follows neither is inconsistent wherever it is flagged as flipped
    bad = z1.clone()
    bad[:, 3] += 1e-2
    cls = parity.classify_fine(w, w, arr["u_fine"], bad, z0, (z0, z1))
    assert bool((cls["inconsistent"] == cls["flip"]).all())


def test_marginal_rule_needs_expected_sets():
    """without z_expected_hip a marginal draw does not excuse differing samples --
    they are unexplained unless the bins themselves differ."""
    cfg, arr = fixtures.load("fw_shipped")
    B = arr["rays"].reshape(-1, 8).shape[0]
    w = arr["coarse_weights"].reshape(B, -1)
    streams = (arr["u_coarse"], arr["u_fine"], arr["u_fine_jit"], arr["n_depth"])
    z0, z1 = parity.expected_fine_sets(arr["rays"], arr["z_coarse"], w, arr["coarse_depth"], streams,
                                       cfg["n_coarse"], cfg["n_fine"], cfg["n_fine_depth"],
                                       cfg.get("depth_std", 0.01))
    moved = (z0 != z1).any(-1)
    cls = parity.classify_fine(w, w, arr["u_fine"], z1, z0)
    assert torch.equal(cls["unexplained"], moved) and not cls["flip"].any()
    cls = parity.classify_fine(w, w, arr["u_fine"], z1, z0, (z0, z1))
    assert torch.equal(cls["flip"], moved) and not cls["unexplained"].any()


def test_flipped_ray_outputs_are_checked_against_the_oracle_fine_pass():
    """check_flipped_outputs recomputes the oracle fine pass at the given (HIP) fine samples:
    the fixture's own outputs at the fixture's samples pass, a perturbed rgb or weight fails
    and names its ray, and multi-object batches are split per object."""
    from oracle import ref_cpu

    for name in ("rw_ns1", "rw_ns3_sb2"):
        cfg, arr = fixtures.load(name)
        sd = fixtures.state_dict(cfg)
        scene = ref_cpu.Scene(fixtures.latent_of(cfg), arr["poses"], fixtures.focal_of(arr), cfg["width"],
                              cfg["height"], fixtures.c_or_none(arr))
        kw = dict(d_latent=cfg["d_latent"], n_blocks=cfg.get("n_blocks", 5),
                  combine_layer=cfg.get("combine_layer", 3), has_fine=cfg.get("with_fine", True))
        B = arr["rays"].reshape(-1, 8).shape[0]
        rpo = B // cfg.get("sb", 1)
        idx = [0, 3, B - 1]
        args = (sd, scene, arr["rays"], arr["z_fine"], arr["fine_rgb"], arr["fine_depth"], arr["fine_weights"])
        res = parity.check_flipped_outputs(*args, idx, rpo, bool(cfg["white_bkgd"]), kw,
                                           w_coarse_hip=arr["coarse_weights"], u_fine=arr["u_fine"])
        assert res["ok"], (name, res)
        assert len(res["boundary_distance"]) == 3
        rgb = arr["fine_rgb"].clone().reshape(B, 3)
        rgb[B - 1, 1] += 1e-3
        res = parity.check_flipped_outputs(sd, scene, arr["rays"], arr["z_fine"], rgb, arr["fine_depth"],
                                           arr["fine_weights"], idx, rpo, bool(cfg["white_bkgd"]), kw)
        assert not res["ok"] and res["bad_rays"] == [B - 1], (name, res)
