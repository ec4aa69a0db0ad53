"""Counter-mode random streams (pnr_rng {seed, offset}; oracle/philox.py) on the CPU:
the Philox4x32-10 restatement against the Random123 known-answer vectors, and the
stream mapping's properties.  The device side is tests/test_gpu_rng.py."""
import numpy as np

from oracle import philox

# Random123 kat_vectors, "philox4x32 10": (counter, key) -> output
KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff),
     (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


def test_philox_known_answers():
    for ctr, key, want in KAT:
        got = tuple(int(x) for x in philox.philox4x32_10(ctr, key))
        assert got == want, (ctr, key, [hex(g) for g in got])


def test_streams_are_chunk_invariant_and_distinct():
    seed = 0x1234_5678_9abc_def0
    full = philox.stream(seed, 0, philox.U_COARSE, 300, 64)
    assert np.array_equal(full[100:300], philox.stream(seed, 100, philox.U_COARSE, 200, 64))
    assert not np.array_equal(full, philox.stream(seed, 0, philox.U_FINE, 300, 64))
    assert not np.array_equal(full, philox.stream(seed + 1, 0, philox.U_COARSE, 300, 64))


def test_stream_moments():
    u = philox.stream(7, 0, philox.U_FINE_JIT, 4096, 64).astype(np.float64)
    assert u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 3e-3 and abs(u.var() - 1.0 / 12.0) < 2e-3
    n = philox.stream(7, 0, philox.N_DEPTH, 4096, 64).astype(np.float64)
    assert np.isfinite(n).all()
    assert abs(n.mean()) < 1e-2 and abs(n.var() - 1.0) < 2e-2
    assert abs(((n - n.mean()) ** 3).mean()) < 3e-2            # symmetric
    assert abs((n ** 4).mean() / n.var() ** 2 - 3.0) < 0.1      # Gaussian kurtosis
