"""The bucket-reduction algebra the MSM kernels rely on, checked on CPU with
bucket sums modelled as integers mod r (the group law is the same Z-module
structure, so any identity of coefficients that holds here holds for points):

* the segment form of the weighted bucket sum (k_bucket_runsum + the batched
  reduction, msm_impl.cuh msm_finish): sum_b (b + 1) S_b = sum_t D_t +
  L sum_t (t + 1) R_t, with R_t the plain sum of segment t and D_t = A_t - L R_t;
* bucket stripes (gg_msm_stripe): stripe r of N = 2^s keeps the buckets
  b = N j + r, renumbered j; its share of the whole is
  N sum_j (j + 1) T_j - (N - 1 - r) sum_j T_j, and the N shares add up to the
  whole weighted sum;
* precompute groups: the group sums recombine with the factors 2^(j c)."""
import random

import pytest

R = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001


def weighted(S, off=1):
    return sum((b + off) * s for b, s in enumerate(S)) % R


def segment_form(S, logL):
    L = 1 << logL
    assert len(S) % L == 0
    D, Rs = [], []
    for t in range(len(S) // L):
        seg = S[t * L:(t + 1) * L]
        run = acc = 0
        for s in reversed(seg):  # k_bucket_runsum walks the segment from the top
            run = (run + s) % R
            acc = (acc + run) % R
        Rs.append(run)
        D.append((acc - L * run) % R)
    return (sum(D) + L * weighted(Rs)) % R


@pytest.mark.parametrize("nb,logL", [(16, 1), (64, 2), (256, 4), (1 << 12, 3)])
def test_segment_form(nb, logL):
    rng = random.Random(nb + logL)
    S = [rng.randrange(R) if rng.random() < 0.8 else 0 for _ in range(nb)]
    assert segment_form(S, logL) == weighted(S)


@pytest.mark.parametrize("nb,slog", [(8, 1), (64, 2), (256, 3), (1 << 11, 4)])
def test_stripes_add_up(nb, slog):
    rng = random.Random(7 * nb + slog)
    S = [rng.randrange(R) for _ in range(nb)]
    N = 1 << slog
    total = 0
    for r in range(N):
        T = S[r::N]  # buckets b = N j + r, j = b >> slog
        ws = weighted(T)
        ps = sum(T) % R
        share = (N * ws - (N - 1 - r) * ps) % R
        assert share == sum((b + 1) * S[b] for b in range(r, nb, N)) % R
        # the kernels' route: the stripe's segment form, scaled, plus the plain term
        if len(T) >= 4:
            assert (N * segment_form(T, 1)) % R == (N * ws) % R
        total = (total + share) % R
    assert total == weighted(S)


@pytest.mark.parametrize("G,c", [(2, 4), (4, 3)])
def test_precompute_groups_recombine(G, c):
    # window w = G w' + j adds into group j with the copy shifted by 2^(c G w'),
    # so the group-j sum carries the missing factor 2^(c j)
    rng = random.Random(G * 100 + c)
    W = 2 * G
    digits = [rng.randrange(1, 1 << (c - 1)) for _ in range(W)]
    point = rng.randrange(1, R)
    want = sum(d << (c * w) for w, d in enumerate(digits)) * point % R
    groups = [0] * G
    for w, d in enumerate(digits):
        j, wp = w % G, w // G
        groups[j] = (groups[j] + d * ((point << (c * G * wp)) % R)) % R
    assert sum(gs << (c * j) for j, gs in enumerate(groups)) % R == want
