"""Statistics of the attention dropout hash (one 32-bit hash per (query, key quad), one
byte per key; tests/dropout_hash.py mirrors csrc/hip/attention.hip bit for bit): keep
rate at the quantised p, byte uniformity, and no correlation between neighbouring
scores along the key axis (inside a quad: bytes of one hash; across quads), the query
axis and the diagonal.  CPU only."""
import pytest
import torch

from dropout_hash import hash_bytes, keep_mask, thr8


@pytest.fixture(scope="module")
def grid():
    return hash_bytes(2, 2, 512, 1234, SK=512).double()   # 2 x 2 x 512 x 512 = 1M scores


@pytest.mark.parametrize("p", [0.1, 0.25, 0.5])
def test_keep_rate_matches_quantised_p(p):
    keep, scale = keep_mask(2, 3, 256, 99, p)
    pq = thr8(p) / 256.0
    rate = 1.0 - keep.double().mean().item()
    n = keep.numel()
    assert abs(rate - pq) < 5 * (pq * (1 - pq) / n) ** 0.5, (rate, pq)
    assert abs(scale * (1 - pq) - 1.0) < 1e-12   # unbiased for the quantised rate
    assert abs(pq - p) <= 1 / 512


def test_byte_uniformity(grid):
    counts = torch.bincount(grid.flatten().long(), minlength=256).double()
    exp = grid.numel() / 256
    chi2 = ((counts - exp) ** 2 / exp).sum().item()
    assert chi2 < 255 + 6 * (2 * 255) ** 0.5, chi2    # ~6 sigma of chi2(255)


@pytest.mark.parametrize("dq,dk", [(0, 1), (0, 2), (0, 3), (0, 4), (0, 5), (1, 0), (2, 0),
                                   (1, 1), (1, -1), (4, 4)])
def test_neighbour_correlation(grid, dq, dk):
    """Correlation of the byte at (q, k) with the byte at (q + dq, k + dk), dq >= 0."""
    x = grid - grid.mean()
    S = x.shape[-1]
    ka = slice(0, S - dk) if dk >= 0 else slice(-dk, S)
    kb = slice(dk, S) if dk >= 0 else slice(0, S + dk)
    a = x[..., 0:S - dq, ka]
    b = x[..., dq:S, kb]
    r = (a * b).mean().item() / x.var().item()
    assert abs(r) < 6 / a.numel() ** 0.5, (dq, dk, r)


def test_keep_bits_within_quad_independent():
    """Joint keep probability of the 4 keys of a quad = product of the marginals."""
    keep, _ = keep_mask(2, 2, 512, 7, 0.5)
    k = keep.view(2, 2, 512, 128, 4).double()
    both = (k[..., 0] * k[..., 1]).mean().item()
    m0, m1 = k[..., 0].mean().item(), k[..., 1].mean().item()
    assert abs(both - m0 * m1) < 6 * (m0 * m1 / k[..., 0].numel()) ** 0.5
