"""CPU checks of the sampled-softmax restatement (oracle/models.py) — the
build-defined C3 loss has no reference counterpart, so the
oracle's draw and loss are pinned here against independent formulations."""
import numpy as np
import torch

from oracle.models import sample_uniform, sampled_ce

M = (1 << 64) - 1


def _mix(z):
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


def _draw_bigint(seed, ctr, S, A):
    return [(_mix((seed + 0x9E3779B97F4A7C15 * (ctr * S + s + 1)) & M) * A) >> 64 for s in range(S)]


def test_sample_uniform_matches_bigint_formula():
    for seed, ctr, S, A in [(0, 0, 64, 1_000_000), (11, 3, 50, 37), (2**63 + 5, 2**40, 20, 2**31 - 1)]:
        assert sample_uniform(seed, ctr, S, A).tolist() == _draw_bigint(seed, ctr, S, A)


def test_sample_uniform_is_uniform_and_in_range():
    x = sample_uniform(7, 0, 200_000, 100)
    assert x.min() >= 0 and x.max() < 100
    cnt = np.bincount(x, minlength=100)
    chi2 = ((cnt - 2000.0) ** 2 / 2000.0).sum()
    assert chi2 < 160  # 99 dof; p ~ 1e-4 bound
    assert not np.array_equal(sample_uniform(7, 0, 50, 100), sample_uniform(7, 1, 50, 100))


def test_sampled_ce_matches_explicit_formula():
    g = torch.Generator().manual_seed(0)
    B, A, H, S = 9, 40, 8, 30
    h = torch.randn(B, H, generator=g, dtype=torch.float64)
    W = torch.randn(A, H, generator=g, dtype=torch.float64)
    b = torch.randn(A, generator=g, dtype=torch.float64)
    a = torch.randint(0, A, (B,), generator=g)
    neg = torch.from_numpy(sample_uniform(1, 0, S, A))
    got = float(sampled_ce(h, W, b, a, neg))
    hn, Wn, bn = h.numpy(), W.numpy(), b.numpy()
    tot = 0.0
    for i in range(B):
        zs = [hn[i] @ Wn[a[i]] + bn[a[i]]] + [hn[i] @ Wn[j] + bn[j] for j in neg.tolist()]
        m = max(zs)
        tot += m + np.log(sum(np.exp(z - m) for z in zs)) - zs[0]
    assert abs(got - tot / B) < 1e-12


def test_oracle_bpr_matches_pairwise_formula():
    """oracle.sampled_bpr against the BPR definition written out in float64
    numpy: mean over rows and negatives of log(1 + exp(z_neg - z_pos))."""
    import torch
    from oracle.models import sampled_bpr
    g = torch.Generator().manual_seed(3)
    B, S, A, H = 17, 40, 90, 8
    h = torch.randn(B, H, generator=g, dtype=torch.float64)
    W = torch.randn(A, H, generator=g, dtype=torch.float64)
    b = torch.randn(A, generator=g, dtype=torch.float64)
    a = torch.randint(0, A, (B,), generator=g)
    neg = torch.randint(0, A, (S,), generator=g)
    got = float(sampled_bpr(h, W, b, a, neg))
    hn, Wn, bn = h.numpy(), W.numpy(), b.numpy()
    zp = (hn * Wn[a.numpy()]).sum(1) + bn[a.numpy()]
    zn = hn @ Wn[neg.numpy()].T + bn[neg.numpy()]
    want = np.log1p(np.exp(zn - zp[:, None])).mean()
    assert abs(got - want) < 1e-12
