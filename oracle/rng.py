"""CPU restatement of the engine's counter-based randomness (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package.

The reference draws every random number from TensorFlow's unseeded, stateful global generator
(layers/rf_layers.py:22 z~N(0,1); layers/GP_weight_layers.py:9 W~N(0,1); models/dgp.py:210,212,240
momenta and SGHMC noise) and shuffles minibatches with tf.data (experiments/utils_dataset.py:38-42).
That stream cannot be reproduced without TF, so the MI355X engine replaces it with
  * Philox4x32-10 (Salmon et al., SC'11; Random123) + Box-Muller for N(0,1) draws, and
  * a keyed 4-round Feistel permutation (cycle-walking) for per-epoch drop-remainder batching.
This module restates both bit-exactly (uint32 arithmetic in numpy) so the GPU tests can check the
device generator bit-for-bit (uint32 words, minibatch indices) and to ~1e-6 (normals).
Philox is pinned by the published Random123 known-answer vectors (tests/test_oracle_rng.py).
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = 0x9E3779B9
W1 = 0xBB67AE85
MASK32 = np.uint64(0xFFFFFFFF)

PURPOSE_NOISE = 1      # dgprf.h DGPRF_RNG_NOISE
PURPOSE_RESAMPLE = 2
PURPOSE_Z = 3
PURPOSE_W = 4
PURPOSE_MOMENTS = 5


def philox4x32_10(ctr, key):
    """Vectorised Philox4x32-10.  ctr: uint32 array [..., 4]; key: (k0, k1) ints or arrays."""
    c = np.asarray(ctr, dtype=np.uint64) & MASK32
    x, y, z, w = c[..., 0], c[..., 1], c[..., 2], c[..., 3]
    k0 = np.asarray(key[0], dtype=np.uint64) & MASK32
    k1 = np.asarray(key[1], dtype=np.uint64) & MASK32
    for _ in range(10):
        p0 = M0 * x
        p1 = M1 * z
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        x, y, z, w = (hi1 ^ y ^ k0) & MASK32, lo1, (hi0 ^ w ^ k1) & MASK32, lo0
        k0 = (k0 + np.uint64(W0)) & MASK32
        k1 = (k1 + np.uint64(W1)) & MASK32
    return np.stack([x, y, z, w], axis=-1).astype(np.uint32)


def _box_muller(a, b):
    u1 = ((a.astype(np.float64) // 256) + 1.0) * 2.0 ** -24
    u2 = (b.astype(np.float64) // 256) * 2.0 ** -24
    r = np.sqrt(-2.0 * np.log(u1))
    return r * np.cos(2.0 * np.pi * u2), r * np.sin(2.0 * np.pi * u2)


def philox_words(n_quads, seed, sub, purpose, tag):
    q = np.arange(n_quads, dtype=np.uint64)
    ctr = np.zeros((n_quads, 4), dtype=np.uint64)
    ctr[:, 0] = q & MASK32
    ctr[:, 1] = np.uint64(sub) & MASK32
    ctr[:, 2] = (np.uint64(sub) >> np.uint64(32)) & MASK32
    ctr[:, 3] = np.uint64(((purpose & 0xFF) << 24) | (tag & 0x00FFFFFF))
    return philox4x32_10(ctr, (seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF))


def philox_normal(n, seed, sub, purpose, tag=0):
    """N(0,1) stream of dgprf_philox_normal / the update kernel (float64 result).

    Element i uses counter quad i // 4 and output word i % 4 (words (0,1) and (2,3) are
    Box-Muller pairs giving (r cos, r sin)).
    """
    nq = (n + 3) // 4
    w = philox_words(nq, seed, sub, purpose, tag)
    z0, z1 = _box_muller(w[:, 0], w[:, 1])
    z2, z3 = _box_muller(w[:, 2], w[:, 3])
    z = np.stack([z0, z1, z2, z3], axis=1).reshape(-1)
    return z[:n]


def fmix32(h):
    h = np.asarray(h, dtype=np.uint64) & MASK32
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & MASK32
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & MASK32
    h ^= h >> np.uint64(16)
    return h


def feistel_key(seed, chain, epoch, rnd):
    mix = ((seed >> 32) + chain * 0x632BE5AB + (epoch & 0xFFFFFFFF) * 0x9E3779B9
           + (epoch >> 32) * 0x85EBCA6B + rnd * 0x27D4EB2F) & 0xFFFFFFFF
    return int(fmix32(np.uint64((seed & 0xFFFFFFFF) ^ int(fmix32(np.uint64(mix))))))


def feistel_perm(x, n, seed, chain, epoch):
    """Vectorised keyed permutation of [0, n) (dgprf_device.h feistel_perm)."""
    bits = 2
    while bits < 32 and (1 << bits) < n:
        bits += 2
    half = bits // 2
    mask = np.uint64((1 << half) - 1)
    keys = [np.uint64(feistel_key(seed, chain, epoch, r)) for r in range(4)]
    x = np.asarray(x, dtype=np.uint64).copy()
    todo = np.ones(x.shape, dtype=bool)
    while todo.any():
        xs = x[todo]
        L = xs >> np.uint64(half)
        R = xs & mask
        for k in keys:
            t = L ^ (fmix32((R * np.uint64(0x9E3779B1) + k) & MASK32) & mask)
            L, R = R, t
        xs = (L << np.uint64(half)) | R
        x[todo] = xs
        todo = x >= np.uint64(n)
    return x.astype(np.int64)


def batch_rows(step, B, n_data, iters, perm_seed, chain=0):
    """Dataset rows of the minibatch at `step` (DGPRF_BATCH_EPOCH)."""
    epoch, pos0 = divmod(int(step), int(iters))
    pos = np.arange(B, dtype=np.uint64) + np.uint64(pos0 * B)
    return feistel_perm(pos, n_data, perm_seed, chain, epoch)
