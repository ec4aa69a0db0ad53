"""ORACLE — test infrastructure only; never imported by the product path.

CPU restatement of the counter-mode random streams of ``pnr_rng`` (include/pnr_abi.h):
Philox4x32-10 as published by Salmon, Moraes, Dror and Shaw, "Parallel random numbers:
as easy as 1, 2, 3" (SC'11), with the Random123 round and key-schedule constants, and the
library's mapping of (seed, offset, stream, ray, k) to a counter and of the output words
to U[0,1) / N(0,1).  Pinned by the Random123 known-answer vectors (tests/test_rng.py).

The reference draws these values with torch.rand / torch.randn (nerf.py:111, 135, 141,
158); counter mode replaces the generator, not the distribution, so parity of a render in
counter mode is checked by materialising the streams (pnr_rng_fill) and replaying them
through the injected-stream path and the oracle renderer.
"""
import numpy as np

MASK = np.uint64(0xFFFFFFFF)
M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
U_COARSE, U_FINE, U_FINE_JIT, N_DEPTH = 0, 1, 2, 3


def philox4x32_10(ctr, key):
    """ctr: 4 arrays (or ints) of 32-bit words, key: 2; returns the 4 output words (uint64
    arrays holding 32-bit values)."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) & MASK for c in ctr)
    k0, k1 = (np.asarray(k, dtype=np.uint64) & MASK for k in key)
    for r in range(10):
        if r:
            k0 = (k0 + W0) & MASK
            k1 = (k1 + W1) & MASK
        p0 = M0 * c0            # < 2^64: exact in uint64
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
    return c0, c1, c2, c3


def stream(seed, offset, stream_id, n_rays, width):
    """The (n_rays, width) draws of stream ``stream_id`` for rays offset .. offset + n_rays - 1
    (pnr_rng_fill): counter (lo32 e, hi32 e, stream, 0), e = (offset + b) * width + k."""
    b = np.arange(n_rays, dtype=np.uint64)[:, None]
    k = np.arange(width, dtype=np.uint64)[None, :]
    e = (np.uint64(offset) + b) * np.uint64(width) + k
    x0, x1, _, _ = philox4x32_10((e & MASK, e >> np.uint64(32), np.uint64(stream_id), np.uint64(0)),
                                 (np.uint64(seed) & MASK, np.uint64(seed) >> np.uint64(32)))
    two24 = np.float32(2.0 ** -24)
    if stream_id != N_DEPTH:
        return (x0 >> np.uint64(8)).astype(np.float32) * two24
    u1 = ((x0 >> np.uint64(8)) + np.uint64(1)).astype(np.float32) * two24
    u2 = (x1 >> np.uint64(8)).astype(np.float32) * two24
    return (np.sqrt(np.float32(-2.0) * np.log(u1)) * np.cos(np.float32(6.28318530717958647) * u2)).astype(np.float32)


def render_streams(seed, offset, n_rays, n_coarse, n_fine, n_fine_depth):
    """(u_coarse, u_fine, u_fine_jit, n_depth) as a counter-mode render draws them."""
    nf = max(n_fine - n_fine_depth, 0)
    return (stream(seed, offset, U_COARSE, n_rays, n_coarse), stream(seed, offset, U_FINE, n_rays, nf),
            stream(seed, offset, U_FINE_JIT, n_rays, nf), stream(seed, offset, N_DEPTH, n_rays, n_fine_depth))
