"""The key generator's and encryption's Gaussian noise follows the reference's sampler: sigma = 3.19
by DiscreteGaussianGeneratorImpl's inversion method (discretegaussiangenerator-impl.h:78-132, used for
every error and Gaussian secret, lwe-pke.cpp:54,90,114,324).  Our draws (GAUSSIAN-keyDist secrets of
STD128_LMKCDEY, fhe_hip_keygen_secret) against 10^6 draws of the reference's own generator
(oracle/_ref ref_dgg_samples) and against the exact probabilities of its table."""
import ctypes
import math

import numpy as np
import pytest

from oracle_lib import Ref, ref_available

SIGMA = 3.19
STD128_LMKCDEY, LMKCDEY = 21, 3


def exact_pmf(xmax):
    """the reference table's probabilities: P(x) = a exp(-x^2 / (2 sigma^2)), |x| <= fin"""
    fin = math.ceil(SIGMA * 12.00610553538285)
    w = [math.exp(-(x * x) / (2 * SIGMA * SIGMA)) for x in range(fin + 1)]
    a = 1.0 / (2 * sum(w[1:]) + 1.0)
    return {x: a * w[abs(x)] for x in range(-xmax, xmax + 1)}


def our_samples(count):
    from fhe_amd import binfhe as bf
    P = bf.params(STD128_LMKCDEY, LMKCDEY)
    out, s = [], 1
    while sum(len(o) for o in out) < count:
        # scattered seeds: the streams of seeds d apart are d draws apart (keygen.h rng_state)
        seed = (s * 0xD1B54A32D192ED03 + 0x5DEECE66D) % (1 << 64)
        sk = bf.keygen_secret(STD128_LMKCDEY, LMKCDEY, seed).astype(np.int64)
        out.append(np.where(sk > P.qKS // 2, sk - P.qKS, sk))
        s += 1
    return np.concatenate(out)[:count]


def binned(x, xmax=10):
    """counts of -xmax..xmax, the two tails merged into the end bins"""
    x = np.clip(x, -xmax, xmax)
    return np.bincount(x + xmax, minlength=2 * xmax + 1).astype(np.float64)


def chi2_p(stat, dof):
    from scipy.stats import chi2
    return float(chi2.sf(stat, dof))


def test_our_noise_matches_the_reference_table():
    n = 400_000
    x = our_samples(n)
    assert abs(x.std() - SIGMA) < 0.03 and abs(x.mean()) < 0.03
    assert np.abs(x).max() <= math.ceil(SIGMA * 12.00610553538285)
    pmf = exact_pmf(10)
    exp = np.array([pmf[v] for v in range(-10, 11)])
    tail = (1 - exp.sum()) / 2
    exp[0] += tail
    exp[-1] += tail
    exp = exp * n
    obs = binned(x)
    stat = float(((obs - exp) ** 2 / exp).sum())
    assert chi2_p(stat, len(obs) - 1) > 1e-4, stat


@pytest.mark.skipif(not ref_available(), reason="oracle/_ref not built")
def test_our_noise_vs_reference_generator_two_sample():
    n = 1_000_000
    ref = Ref(None, None)
    r = np.zeros(n, np.int64)
    assert ref.L.ref_dgg_samples(ctypes.c_size_t(n), r.ctypes.data_as(ctypes.c_void_p)) == 0, ref.err()
    x = our_samples(n)
    a, b = binned(x), binned(r)
    keep = (a + b) > 0
    a, b = a[keep], b[keep]
    stat = float((((a - b) ** 2) / (a + b)).sum())      # equal-size two-sample chi-square
    assert chi2_p(stat, len(a) - 1) > 1e-4, (stat, a, b)
    assert abs(r.std() - x.std()) < 0.02
