"""Oracle RNG pins: Philox4x32-10 against the published Random123 known-answer vectors; the
keyed Feistel minibatch permutation is a bijection with drop-remainder epochs."""
import numpy as np

from oracle import rng as R

# Random123 kat_vectors, philox4x32_10
KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def test_philox_kat():
    for ctr, key, exp in KAT:
        got = R.philox4x32_10(np.array([ctr], dtype=np.uint64), key)[0]
        assert [int(x) for x in got] == list(exp)


def test_normal_moments():
    z = R.philox_normal(200_000, seed=123, sub=7, purpose=R.PURPOSE_NOISE)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01
    # different purpose / subsequence -> different stream
    z2 = R.philox_normal(1000, seed=123, sub=8, purpose=R.PURPOSE_NOISE)
    assert not np.allclose(z[:1000], z2)


def test_feistel_is_bijection():
    for n in (1, 2, 3, 133, 1000, 4097, 1 << 16):
        p = R.feistel_perm(np.arange(n), n, seed=99, chain=3, epoch=5)
        assert sorted(p.tolist()) == list(range(n))


def test_epoch_batches_cover_drop_remainder():
    n, B = 1003, 10
    iters = n // B
    rows = np.concatenate([R.batch_rows(t, B, n, iters, perm_seed=4) for t in range(iters)])
    assert len(set(rows.tolist())) == iters * B  # no repeats inside an epoch
    nxt = R.batch_rows(iters, B, n, iters, perm_seed=4)  # next epoch reshuffles
    assert not np.array_equal(nxt, R.batch_rows(0, B, n, iters, perm_seed=4))
