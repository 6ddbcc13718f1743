"""Exact outcome law of the reference round loop under its admissible inputs.

TEST INFRASTRUCTURE ONLY (third, independent check of the oracle and kernel).

Derivation (from src/nodes/node.ts:43-163 and
launchNodes.ts:12-13): with exactly F crash-faulty nodes, every live receiver
tallies the same m = N - F live values in every phase.  A round whose live
x-multiset is not tied makes every node propose the majority v
(node.ts:63-69); all m votes then equal v, so every live node decides v in
that round iff m > F (node.ts:99-105), else adopts v (node.ts:106-109) and x
freezes.  A tied round (m even, c0 == c1) makes every node propose "?"; the
P-phase then sees c0 == c1 == 0 and every node flips its own coin
(node.ts:111).  The coin is one uniform Philox bit, so P(coin = 1) = 1/2
exactly (the reference's Math.random() > 0.5 ? 0 : 1 gives 1/2 + 2^-53).
"""
from __future__ import annotations

from math import comb

import numpy as np

P_COIN1 = 0.5


def tie_prob(m: int, p: float = 0.5) -> float:
    """P(c0 == c1) for m iid Bernoulli(p) values."""
    if m % 2:
        return 0.0
    h = m // 2
    if p == 0.5:
        return comb(m, h) / (1 << m)          # exact big-integer ratio: no overflow at m in the thousands
    return comb(m, h) * (p ** h) * ((1 - p) ** h)


def hist_probs(N: int, F: int, k_max: int) -> np.ndarray:
    """Probability of each histogram bin (layout of oracle_run_trials, without
    the trailing disagreement counter) for iid Bernoulli(1/2) initial values."""
    m = N - F
    H = (k_max + 1) * 3
    pr = np.zeros(H, dtype=np.float64)
    if m <= 0:
        pr[2] = 1.0
        return pr
    q1 = tie_prob(m, 0.5)          # round 1: initial values
    qc = tie_prob(m, P_COIN1)      # later rounds: coin values
    # probability that rounds 1..r-1 all tie and round r does not
    decides = m > F
    alive = 1.0                     # P(all previous rounds tied)
    for r in range(1, k_max + 1):
        q = q1 if r == 1 else qc
        p = 0.5 if r == 1 else P_COIN1
        nontie = alive * (1 - q)
        # majority value distribution given not tied: symmetric at p = 1/2;
        # for the coin rounds P(c1 > c0 | no tie)
        if p == 0.5:
            p1 = 0.5
        else:
            s1 = sum(comb(m, j) * p ** j * (1 - p) ** (m - j) for j in range(m // 2 + 1, m + 1))
            p1 = s1 / (1 - q) if q < 1 else 0.5
        if decides:
            pr[r * 3 + 0] += nontie * (1 - p1)
            pr[r * 3 + 1] += nontie * p1
        else:
            pr[0] += nontie * (1 - p1)
            pr[1] += nontie * p1
        alive *= q
    # every round tied: final x are the round-k_max coins
    p = P_COIN1 if k_max >= 1 else 0.5
    all1 = p ** m
    all0 = (1 - p) ** m
    # conditional on the last round's coins being drawn (the tie happened in
    # round k_max), x are iid coins; unconditional weight is `alive`.
    pr[0] += alive * all0
    pr[1] += alive * all1
    pr[2] += alive * (1 - all0 - all1)
    return pr


def expected_rounds(N: int, F: int) -> float:
    """E[R] for N > 2F with Bernoulli(1/2) inputs (geometric law)."""
    m = N - F
    q = tie_prob(m)
    return 1.0 / (1.0 - q)


def rounds_cdf(probs: np.ndarray, k_max: int) -> np.ndarray:
    """CDF of the rounds-to-decision R over 1..k_max+1 from bin probabilities
    (R = k_max + 1 stands for "not decided within k_max rounds")."""
    pr = np.asarray(probs, dtype=np.float64)[: (k_max + 1) * 3].reshape(k_max + 1, 3).sum(axis=1)
    pmf = np.concatenate([pr[1:], pr[:1]])             # R = 1..k_max, then undecided
    return np.cumsum(pmf)


def ks_rounds_pvalue(counts: np.ndarray, probs: np.ndarray, k_max: int) -> float:
    """Kolmogorov-Smirnov test of the rounds-to-decision distribution (the
    histogram summed over decided values) against the exact law.

    R is discrete, so the statistic D = max |F_n(r) - F(r)| is taken over the
    support points and its p-value from the Kolmogorov distribution of n
    samples (scipy.stats.kstwo) is conservative: P(D >= d) is never larger
    under H0 than for a continuous law."""
    from scipy import stats

    c = np.asarray(counts, dtype=np.float64)[: (k_max + 1) * 3].reshape(k_max + 1, 3).sum(axis=1)
    n = c.sum()
    emp = np.cumsum(np.concatenate([c[1:], c[:1]])) / n
    d = float(np.max(np.abs(emp - rounds_cdf(probs, k_max))))
    return float(stats.kstwo.sf(d, int(n))) if d > 0 else 1.0


def chi2_pvalue(counts: np.ndarray, probs: np.ndarray, min_expected: float = 5.0) -> float:
    """Pearson chi-square goodness of fit, pooling bins with small expectation."""
    from scipy import stats

    counts = np.asarray(counts, dtype=np.float64)
    n = counts.sum()
    exp = probs * n
    order = np.argsort(-exp)
    obs_b, exp_b = [], []
    acc_o = acc_e = 0.0
    for i in order:
        if exp[i] >= min_expected:
            obs_b.append(counts[i])
            exp_b.append(exp[i])
        else:
            acc_o += counts[i]
            acc_e += exp[i]
    if acc_e > 0:
        if acc_e >= min_expected or not obs_b:
            obs_b.append(acc_o)
            exp_b.append(acc_e)
        else:
            obs_b[-1] += acc_o
            exp_b[-1] += acc_e
    if len(obs_b) < 2:
        return 1.0 if all(abs(o - e) < 1e-9 for o, e in zip(obs_b, exp_b)) else 0.0
    stat, pval = stats.chisquare(np.array(obs_b), np.array(exp_b))
    return float(pval)
