"""Philox4x32-10 jitter stream, restated in numpy (TEST INFRASTRUCTURE ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s CPU legs may import this
module; the product package never does.

The reference jitters each (pixel, dof, aa) sample's origin by
``0.1 (dx + dy) normalize(vec3(rand(), rand(), rand()))`` with three unseeded
``np.random.rand()`` draws (provided/scene.py:63-65), so its jittered frames are not
reproducible. The product's production mode (``RTX_JITTER_PHILOX``) draws the three
uniforms from a counter-based generator instead; this module produces the same uniforms,
in the layout of the parity mode's replayed noise table ([column][row][dof][aa][3],
provided/scene.py:47-65 loop order), so the oracle -- which applies them exactly as the
reference applies its draws -- renders the frame the Philox kernel must produce, bit for
bit.

Generator: Philox4x32 with 10 rounds (Salmon, Moraes, Dror, Shaw, "Parallel random
numbers: as easy as 1, 2, 3", SC'11; Random123 1.x): per round
``(c0, c1, c2, c3) <- (hi(M1 c2) ^ c1 ^ k0, lo(M1 c2), hi(M0 c0) ^ c3 ^ k1, lo(M0 c0))``
with M0 = 0xD2511F53, M1 = 0xCD9E8D57, then the key is bumped by (0x9E3779B9, 0xBB67AE85).
``KAT`` holds Random123's published known-answer vectors for it.

Stream layout (the product's contract, include/rtx.h RTX_JITTER_PHILOX): sample
s = kd * n_aa + ka of image column X (0-based, full frame) and reference row j (0 =
bottom, provided/scene.py:48) takes half s & 1 of the block with counter (X, j, s >> 1, 0)
and key (seed & 0xFFFFFFFF, seed >> 32). Each block gives six 21-bit integers u, each
used as u * 2^-21 (exact in fp32 and fp64):
- half 0: the top 21 bits of words 0, 1, 2;
- half 1: the low 11 bits of words 0, 1, 2, each joined (as bits 11..20) with the
  consecutive 10-bit fields 0..9, 10..19, 20..29 of word 3.
"""
import numpy as np

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
_MASK = 0xFFFFFFFF

# Random123 kat_vectors, "philox4x32 10": (counter, key, expected output)
KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF),
     (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def philox4x32_10(ctr, key):
    """Philox4x32-10 of counters ``ctr`` (uint32 [..., 4]) under one key (k0, k1).
    Returns uint32 [..., 4]."""
    c = [np.asarray(ctr, np.uint64)[..., i] & _MASK for i in range(4)]
    k0, k1 = int(key[0]) & _MASK, int(key[1]) & _MASK
    for r in range(10):
        if r:
            k0, k1 = (k0 + W0) & _MASK, (k1 + W1) & _MASK
        p0 = np.uint64(M0) * c[0]  # < 2^64: exact in uint64
        p1 = np.uint64(M1) * c[2]
        c = [(p1 >> np.uint64(32)) ^ c[1] ^ np.uint64(k0), p1 & np.uint64(_MASK),
             (p0 >> np.uint64(32)) ^ c[3] ^ np.uint64(k1), p0 & np.uint64(_MASK)]
    return np.stack(c, axis=-1).astype(np.uint32)


def sample_uniforms(block, half):
    """The three 21-bit integers of one sample from its block (uint32 [..., 4]) and its
    half (0 or 1, array-like), as uint32 [..., 3]."""
    w = np.asarray(block, np.uint32)
    half = np.asarray(half)
    top = w[..., :3] >> np.uint32(11)
    w3 = w[..., 3:4]
    fields = np.concatenate([w3 & np.uint32(0x3FF), (w3 >> np.uint32(10)) & np.uint32(0x3FF),
                             (w3 >> np.uint32(20)) & np.uint32(0x3FF)], axis=-1)
    low = (w[..., :3] & np.uint32(0x7FF)) | (fields << np.uint32(11))
    return np.where(half[..., None] != 0, low, top)


def jitter_noise(seed, col0, ncols, height, n_dof, n_aa):
    """The uniforms the Philox kernel draws for the strip of columns col0 .. col0+ncols-1,
    as the parity mode's noise table: float64 [ncols * height * n_dof * n_aa * 3] in
    (column, reference row, dof, aa, xyz) order -- what ``noise=`` of the oracle and
    ``Scene.jitter_noise`` expect."""
    X, J, S = np.meshgrid(np.arange(col0, col0 + ncols, dtype=np.uint64), np.arange(height, dtype=np.uint64),
                          np.arange(n_dof * n_aa, dtype=np.uint64), indexing="ij")
    ctr = np.stack([X, J, S >> np.uint64(1), np.zeros_like(X)], axis=-1)
    blocks = philox4x32_10(ctr, (seed & _MASK, (seed >> 32) & _MASK))
    u = sample_uniforms(blocks, (S & np.uint64(1)).astype(np.uint32))
    return (u.astype(np.float64) * 2.0 ** -21).ravel()
