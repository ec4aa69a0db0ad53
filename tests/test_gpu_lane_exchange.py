"""Cross-lane exchanges of the fused epilogue and the relu publish.

k_point_mlp's epilogue (composite_wave / sample_fine_wave: DPP row_shr / row_bcast scans and
sums) and its relu publish (rows_max: v_permlane16/32_swap) exchange values between lanes
without LDS; the register sort keeps ds_bpermute (march_dev.h lane_xor) after a DPP / permlane
version of it measured wrong inside the GEMM region in round 2.  pixel-nerf_amd/csrc/selftest.hip
runs both exchange families -- ds_bpermute and DPP quad_perm / row shifts with bank masks /
permlane swaps -- in three placements (wave-uniform; a lane-divergent branch; right after a
16-accumulator MFMA chain that stays live across them) and these tests hold them to the
exchange semantics computed on the host.  Built by `make -C pixel-nerf_amd`
(pnr/libpnr_selftest.so, a diagnostic library: nothing in the render path loads it)."""
import ctypes
import os

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "pixel-nerf_amd", "pnr", "libpnr_selftest.so")

pytestmark = pytest.mark.gpu

NW = 4   # waves
ACTIVE = np.array([(l * 7) % 5 != 0 for l in range(64)])   # placement 1's EXEC


def run(variant, placement, x):
    lib = ctypes.CDLL(LIB)
    lib.pnr_selftest_lane_exchange.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    xin = torch.from_numpy(x).to(dev)
    out = torch.full((NW * 8 * 64 + NW * 64,), float("nan"), device=dev)
    wts = torch.from_numpy(np.random.default_rng(5).standard_normal(256 * 8).astype(np.float16)).to(dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    rc = lib.pnr_selftest_lane_exchange(variant, placement, xin.data_ptr(), out.data_ptr(), wts.data_ptr(), NW,
                                        ctypes.c_void_p(stream))
    torch.cuda.synchronize(dev)
    assert rc == 0
    return out[:NW * 8 * 64].reshape(NW, 8, 64).cpu().numpy()


def inputs(seed=0):
    x = np.random.default_rng(seed).standard_normal(NW * 64).astype(np.float32)
    x[7] = x[9]          # ties in the sort
    x[70] = -0.0
    return x


def host_xor(x, j):
    return x.reshape(NW, 64)[:, np.arange(64) ^ j]


@pytest.mark.parametrize("placement", [0, 2])
@pytest.mark.parametrize("variant", [0, 1])
def test_exchanges_and_sort_exact(variant, placement):
    """Wave-uniform control flow, alone (0) and with a live MFMA chain around it (2): every
    exchange is the exact lane ^ J permutation and the register bitonic sort is np.sort."""
    x = inputs()
    o = run(variant, placement, x)
    for t, j in enumerate((1, 2, 4, 8, 16, 32)):
        np.testing.assert_array_equal(o[:, t], host_xor(x, j), err_msg="lane ^ %d" % j)
    np.testing.assert_array_equal(o[:, 6], np.sort(x.reshape(NW, 64), axis=1))


@pytest.mark.parametrize("placement", [0, 2])
def test_dpp_scans_identical_across_variants_and_placements(placement):
    """The epilogue's DPP scan / sum and the publish's permlane row maximum give bit-identical
    lanes whatever exchange family surrounds them and wherever they sit."""
    x = inputs(1)
    ref = run(0, 0, x)[:, 7]
    assert np.isfinite(ref).all()
    for v in (0, 1):
        np.testing.assert_array_equal(run(v, placement, x)[:, 7], ref)


@pytest.mark.parametrize("variant", [0, 1])
def test_divergent_branch_active_pairs(variant):
    """Inside a lane-divergent branch: an active lane whose partner lane is active gets the
    partner's value from both families.  (What a lane reads from an INACTIVE partner is where
    the families may differ -- DPP / permlane read the partner's register as it is, the result
    the tests do not rely on; no exchange in the render path runs under a divergent EXEC.)"""
    x = inputs(2)
    o = run(variant, 1, x)
    for t, j in enumerate((1, 2, 4, 8, 16, 32)):
        partner = np.arange(64) ^ j
        m = ACTIVE & ACTIVE[partner]
        np.testing.assert_array_equal(o[:, t][:, m], host_xor(x, j)[:, m], err_msg="lane ^ %d" % j)
        assert np.isnan(o[:, t][:, ~ACTIVE]).all()   # inactive lanes wrote nothing
