"""ModSwitch (RoundqQ, lwe-pke.cpp:41-46: floor(0.5 + double(v) double(q) / double(Q)) mod q) at
moduli outside the STD128 path, on values next to the rounding ties, where the exact-integer
form floor((2 v q + Q) / (2 Q)) and the reference's IEEE-double form can disagree:
  * the standalone fhe_hip_modswitch_batch (any moduli, evaluated in double like the reference);
  * the key-switch epilogue's ModSwitch(qKS -> fmod) of BootstrapFunc at fmod up to 2^40;
  * EvalFunc with an arbitrary LUT at small q (beta = 128 >= 2q: the reference's
    EvalAddConstEq leaves b + beta - 2q unreduced, ModSub in BootstrapFuncCore reduces it)."""
import numpy as np
import pytest

from oracle_lib import Ref, ref_available

# (q_from, q_to): odd and power-of-two moduli whose product exceeds 2^53
PAIRS = [((1 << 40) - 87, (1 << 20) - 3), ((1 << 39) + 1, 1 << 19), ((1 << 45) - 55, 1 << 14), (1 << 14, (1 << 40) - 5),
         (134215681, 16384), (268369921, (1 << 30) + 7)]


def near_ties(q_from, q_to, count=256, seed=0):
    """values v < q_from with v q_to / q_from within a few ulps of k + 1/2, plus random ones"""
    rng = np.random.default_rng(seed + q_from % 1000)
    out = []
    for _ in range(count):
        k = int(rng.integers(0, q_to))
        c = ((2 * k + 1) * q_from) // (2 * q_to)       # floor of the tie point
        for d in (-1, 0, 1, 2):
            v = c + d
            if 0 <= v < q_from:
                out.append(v)
    out += [int(x) for x in rng.integers(0, q_from, 64, dtype=np.uint64)] + [0, q_from - 1]
    return np.array(out, np.uint64)


def round_qQ(v, q, Q):
    """lwe-pke.cpp:41-46 in IEEE double (numpy float64 ops are IEEE, no contraction)"""
    x = (v.astype(np.float64) * np.float64(q)) / np.float64(Q)
    return (np.floor(np.float64(0.5) + x).astype(np.uint64)) % np.uint64(q)


def test_integer_form_differs_from_double_somewhere():
    """the test values do reach the region where only the double form is the reference's"""
    diff = 0
    for qf, qt in PAIRS[:4]:
        v = near_ties(qf, qt)
        exact = np.array([((2 * int(x) * qt + qf) // (2 * qf)) % qt for x in v], np.uint64)
        diff += int(np.sum(exact != round_qQ(v, qt, qf)))
    assert diff > 0


@pytest.mark.skipif(not ref_available(), reason="reference oracle not built")
def test_numpy_round_qQ_matches_reference_modswitch():
    ref = Ref(3, 2)
    for qf, qt in PAIRS:
        v = near_ties(qf, qt)
        a = v.reshape(-1, 1).copy()
        ao, bo = ref.modswitch(qf, qt, a, v.copy())
        assert np.array_equal(ao.ravel(), round_qQ(v, qt, qf)), (qf, qt)
        assert np.array_equal(bo, round_qQ(v, qt, qf))


@pytest.mark.gpu
def test_gpu_modswitch_any_moduli_equals_reference_double():
    from fhe_amd import binfhe as bf
    e = bf.GateEngine(bf.STD128, bf.GINX, device=0)
    for qf, qt in PAIRS:
        v = near_ties(qf, qt)
        L = 4
        n = len(v) // L
        a = v[:n * L].reshape(n, L).copy()
        b = v[:n].copy()
        ao, bo = e.modswitch(qf, qt, a, b)
        assert np.array_equal(ao.ravel(), round_qQ(a.ravel(), qt, qf)), (qf, qt)
        assert np.array_equal(bo, round_qQ(b, qt, qf)), (qf, qt)
    e.close()


@pytest.mark.gpu
def test_gpu_bootstrap_func_large_fmod_vs_oracle(restatement):
    """BootstrapFunc's final ModSwitch(qKS -> fmod) at fmod > 2^38 (double path of the key-switch
    epilogue) against the restatement, whose RoundqQ is the reference's double expression"""
    from fhe_amd import binfhe as bf
    from oracle_lib import Restatement
    ps, m = bf.STD128, bf.GINX
    keys = bf.keygen(ps, m, 0xB0070000 + ps)
    O = Restatement(ps, m)
    e = bf.GateEngine(ps, m, device=0)
    e.load_keys(keys.bsk, keys.kskA, keys.kskB)
    rng = np.random.default_rng(5)
    q = 1024
    for fmod in ((1 << 40) - 3, (1 << 39) + 11, 1 << 40):
        a, b = bf.encrypt(ps, m, keys.sk, rng.integers(0, 4, 37), 900 + fmod % 97)
        f = rng.integers(0, 1 << 12, q).astype(np.uint64) * np.uint64(fmod >> 12)
        ga, gb = e.bootstrap_func(a, b, q, f, fmod)
        oa, ob = O.bootstrap_func(keys.bsk, keys.kskA, keys.kskB, a, b, q, (O.Q // fmod) * f, fmod)
        assert np.array_equal(ga, oa) and np.array_equal(gb, ob), fmod
    e.close()


@pytest.mark.gpu
@pytest.mark.skipif(not ref_available(), reason="reference oracle not built")
@pytest.mark.parametrize("q_in", [32, 64, 128])
def test_gpu_eval_func_arbitrary_small_q_vs_reference(q_in):
    """arbitrary-function EvalFunc at q <= 64 (dq <= 128 = beta): the reference itself, run on the
    same keys and ciphertexts (oracle/_ref), against the GPU"""
    from fhe_amd import binfhe as bf
    ps, m = bf.STD128, bf.GINX
    keys = bf.keygen(ps, m, 0xB0070000 + ps)
    p = max(2, q_in // 16)
    lut = np.array([(q_in // p) * (((i * p) // q_in) ** 3 % p) for i in range(q_in)], np.uint64)
    ms = np.arange(2 * p) % p
    a, b = bf.encrypt(ps, m, keys.sk, ms, 4000 + q_in, p, q_in)
    e = bf.GateEngine(ps, m, device=0)
    e.load_keys(keys.bsk, keys.kskA, keys.kskB)
    ga, gb = e.eval_func(a, b, q_in, lut)
    e.close()
    ref = Ref(ps, m)
    ref.load_keys(keys.bsk, keys.kskA, keys.kskB)
    ra, rb = ref.eval_func(a, b, q_in, lut)
    assert np.array_equal(ga, ra) and np.array_equal(gb, rb)
