"""CPU check of the arithmetic behind the f32 convs' bf16 three-term form (va_seg.hip split3_bf16 /
conv2_kernel SPL): h = bf16(x), m = bf16(x - h), l = bf16(x - h - m) with round-to-nearest-even reproduces every
f32 x exactly as h + m + l, each term product of two such terms is exact in f32, and the three products the
6-term form leaves out are below 2^-22 of |a b| together."""
import numpy as np


def bf16_rne(x: np.ndarray) -> np.ndarray:
    """f32 -> bf16 (round to nearest even) -> f32, as v_cvt_pk_bf16_f32 does for finite values."""
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return r.view(np.float32)


def split3(x: np.ndarray):
    x = x.astype(np.float32)
    h = bf16_rne(x)
    r = (x - h).astype(np.float32)
    m = bf16_rne(r)
    l_ = (r - m).astype(np.float32)
    lb = bf16_rne(l_)
    return h, m, l_, lb


def _samples(n=400_000, seed=0):
    g = np.random.default_rng(seed)
    u = g.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    x = u.view(np.float32)
    x = x[np.isfinite(x) & (np.abs(x) > 1e-30) & (np.abs(x) < 1e30)]
    return np.concatenate([x, g.standard_normal(n).astype(np.float32),
                           np.float32([1.0, -1.0, 3.0, 1 + 2**-23, -(1 + 2**-23), 255.99998, 65504.0])])


def test_split_is_exact():
    x = _samples()
    h, m, l_, lb = split3(x)
    assert np.array_equal(lb, l_), "the last remainder must be exact in bf16"
    s = h.astype(np.float64) + m.astype(np.float64) + l_.astype(np.float64)
    assert np.array_equal(s, x.astype(np.float64))


def test_term_products_exact_and_dropped_terms_small():
    g = np.random.default_rng(1)
    a = g.standard_normal(100_000).astype(np.float32) * np.float32(3.7)
    b = g.standard_normal(100_000).astype(np.float32)
    ah, am, al, _ = split3(a)
    bh, bm, bl, _ = split3(b)
    for p, q in ((ah, bh), (ah, bm), (am, bh), (ah, bl), (am, bm), (al, bh), (am, bl), (al, bm), (al, bl)):
        exact = p.astype(np.float64) * q.astype(np.float64)
        assert np.array_equal((p * q).astype(np.float64), exact)  # 8 x 8 significand bits fit f32
    ab = a.astype(np.float64) * b.astype(np.float64)
    six = sum(p.astype(np.float64) * q.astype(np.float64)
              for p, q in ((ah, bh), (ah, bm), (am, bh), (ah, bl), (am, bm), (al, bh)))
    nz = ab != 0
    rel = np.abs(six - ab)[nz] / np.abs(ab)[nz]
    assert rel.max() < 2.0 ** -22


def test_host_split_of_the_weights_matches_the_device_split():
    """seg.split3_bf16 (the pre-split weights of va_conv_args.w3, conv3t_kernel) gives the same three terms as the
    device's split (restated above) and h + m + l == x exactly, in the [K/8][3][8] layout."""
    import torch

    from vision_assist_amd.seg import split3_bf16
    x = _samples(20_000)
    x = x[: (len(x) // 64) * 64].reshape(-1, 64)
    t = split3_bf16(torch.from_numpy(x)).float().numpy()  # [rows, 8, 3, 8]
    h, m, _, lb = split3(x)
    g = x.shape[:-1] + (8, 8)
    assert np.array_equal(t[..., 0, :], h.reshape(g))
    assert np.array_equal(t[..., 1, :], m.reshape(g))
    assert np.array_equal(t[..., 2, :], lb.reshape(g))
    s = (t[..., 0, :].astype(np.float64) + t[..., 1, :] + t[..., 2, :]).reshape(x.shape)
    assert np.array_equal(s, x.astype(np.float64))
