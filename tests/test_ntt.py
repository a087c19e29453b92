"""Negacyclic NTT parity: oracle pinned to the reference's golden vectors (CPU)
and the HIP kernel vs the oracle / golden vectors (GPU)."""
import hashlib
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = ["q60", "std128", "lmkcdey"]


def gold(name):
    return np.load(os.path.join(GOLD, f"ntt_{name}.npz"))


def inputs(g):
    Q = int(g["Q"])
    rng = np.random.default_rng(int(g["seed"]))
    x = rng.integers(0, Q, size=(64, 1024), dtype=np.uint64)
    x[0] = 0
    x[1] = Q - 1
    return Q, int(g["psi"]), x


def inputs4096(g):
    """BASELINE config 2's whole batch (tests/golden/make_golden.py ntt4096_inputs)"""
    Q = int(g["Q"])
    return Q, np.random.default_rng(int(g["seed4096"])).integers(0, Q, size=(4096, 1024), dtype=np.uint64)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.uint64).tobytes()).hexdigest()


def negacyclic_mul(a, b, Q):
    """schoolbook a*b mod (X^N + 1, Q) (python ints, exact)."""
    N = len(a)
    r = [0] * N
    for i in range(N):
        ai = int(a[i])
        if ai == 0:
            continue
        for j in range(N):
            k = i + j
            if k < N:
                r[k] += ai * int(b[j])
            else:
                r[k - N] -= ai * int(b[j])
    return np.array([v % Q for v in r], dtype=np.uint64)


# ----------------------------------------------------------------- CPU ----
@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_reference_golden(restatement, name):
    g = gold(name)
    Q, psi, x = inputs(g)
    assert np.array_equal(x[:4], g["x"])
    fwd = restatement.ntt(Q, psi, x)
    inv = restatement.ntt(Q, psi, x, inverse=True)
    assert np.array_equal(fwd[:4], g["fwd"]) and sha(fwd) == str(g["fwd_sha"])
    assert np.array_equal(inv[:4], g["inv"]) and sha(inv) == str(g["inv_sha"])


def test_oracle_roots_match_reference(restatement):
    for name in NAMES:
        g = gold(name)
        assert restatement.L.tfo_root_of_unity(2048, int(g["Q"])) == int(g["psi"])


def test_oracle_kat_unittesttransform(restatement):
    """Known-answer test of the reference (src/core/unittest/UnitTestTransform.cpp:57-91):
    modulus 113, m = 8, (1 + 2x + 4x^2 + x^3)^2 -> {94, 109, 11, 18}."""
    Q = 113
    psi = restatement.L.tfo_root_of_unity(8, Q)
    a = np.array([[1, 2, 4, 1]], dtype=np.uint64)
    A = restatement.ntt(Q, psi, a)
    AB = (A.astype(object) * A.astype(object)) % Q
    r = restatement.ntt(Q, psi, AB.astype(np.uint64), inverse=True)
    assert list(r[0]) == [94, 109, 11, 18]


@pytest.mark.parametrize("name", NAMES)
def test_oracle_ntt4096_matches_reference_hash(name, restatement):
    """the restatement on config 2's 4096-polynomial batch == the reference's SwitchFormat (hashes)"""
    g = gold(name)
    Q, x = inputs4096(g)
    psi = int(g["psi"])
    assert sha(restatement.ntt(Q, psi, x)) == str(g["fwd4096_sha"])
    assert sha(restatement.ntt(Q, psi, x, inverse=True)) == str(g["inv4096_sha"])


# ----------------------------------------------------------------- GPU ----
@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_ntt4096_matches_reference_hash(name):
    """config 2 as measured (one 4096-polynomial launch per direction: k_ntt1024w / k_ntt1024w64) ==
    the reference's SwitchFormat on the same 4096 polynomials, forward and inverse"""
    from fhe_amd import NttPlan
    g = gold(name)
    Q, x = inputs4096(g)
    plan = NttPlan(Q)
    assert sha(plan.forward(x)) == str(g["fwd4096_sha"])
    assert sha(plan.inverse(x)) == str(g["inv4096_sha"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_ntt_matches_golden(name):
    from fhe_amd import NttPlan
    g = gold(name)
    Q, psi, x = inputs(g)
    plan = NttPlan(Q)          # psi chosen by the library exactly as the reference does
    assert plan.psi == psi
    fwd = plan.forward(x)
    inv = plan.inverse(x)
    assert np.array_equal(fwd[:4], g["fwd"]) and sha(fwd) == str(g["fwd_sha"])
    assert np.array_equal(inv[:4], g["inv"]) and sha(inv) == str(g["inv_sha"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_ntt_roundtrip_and_ragged(name, restatement):
    from fhe_amd import NttPlan
    g = gold(name)
    Q, psi, _ = inputs(g)
    plan = NttPlan(Q)
    rng = np.random.default_rng(7)
    for count in (1, 3, 7, 9, 33, 4096):   # ragged batches (partial workgroups)
        x = rng.integers(0, Q, size=(count, 1024), dtype=np.uint64)
        f = plan.forward(x)
        if count <= 33:
            assert np.array_equal(f, restatement.ntt(Q, psi, x))
        assert np.array_equal(plan.inverse(f), x)


@pytest.mark.gpu
def test_gpu_ntt_negacyclic_product():
    """size-independent property: iNTT(NTT(a) . NTT(b)) = a*b mod (X^N+1)."""
    from fhe_amd import NttPlan
    Q = 134215681
    plan = NttPlan(Q)
    rng = np.random.default_rng(3)
    a = rng.integers(0, Q, size=(1, 1024), dtype=np.uint64)
    b = np.zeros((1, 1024), dtype=np.uint64)
    b[0, rng.integers(0, 1024, 6)] = rng.integers(0, Q, 6, dtype=np.uint64)
    A, B = plan.forward(a), plan.forward(b)
    AB = ((A.astype(object) * B.astype(object)) % Q).astype(np.uint64)
    assert np.array_equal(plan.inverse(AB)[0], negacyclic_mul(a[0], b[0], Q))


@pytest.mark.gpu
def test_gpu_ntt_empty_and_bad_params():
    from fhe_amd import FheHipError, NttPlan
    plan = NttPlan(134215681)
    assert plan.forward(np.zeros((0, 1024), np.uint64)).shape == (0, 1024)
    with pytest.raises(FheHipError):
        NttPlan(134215683)   # not prime


@pytest.mark.gpu
@pytest.mark.parametrize("Q", [1073707009, 2147473409, 1152921504606830593, 4611686018427322369])
def test_gpu_ntt_lazy_bound_moduli(Q, restatement):
    """moduli at the edge of the 32-bit lazy path (4Q < 2^32 needs Q < 2^30; larger Q
    takes the 64-bit path), the 60-bit poly-benchmark prime 2^60 - 2^14 + 1 (the Sol60 butterflies:
    values grow to just below 16 Q between planned folds) and a 62-bit prime (Lazy64), with
    all-(Q-1) rows as the worst case for lazy bounds."""
    from fhe_amd import NttPlan
    plan = NttPlan(Q)
    rng = np.random.default_rng(17)
    x = rng.integers(0, Q, size=(9, 1024), dtype=np.uint64)
    x[0] = Q - 1
    x[1, ::2] = Q - 1
    f = plan.forward(x)
    assert np.array_equal(f, restatement.ntt(Q, plan.psi, x))
    assert np.array_equal(plan.inverse(x), restatement.ntt(Q, plan.psi, x, inverse=True))
    assert np.array_equal(plan.inverse(f), x)


@pytest.mark.gpu
@pytest.mark.parametrize("Q", [134215681, 1152921504606830593])
def test_gpu_ntt_multi_iteration_out_of_place(restatement, Q):
    """a batch larger than the persistent grid (every wave loops, odd tail pair),
    out-of-place on device buffers == in-place host path; sampled rows vs the oracle."""
    import ctypes
    from fhe_amd import NttPlan
    from fhe_amd._lib import check, lib, ptr, vp
    plan = NttPlan(Q)
    count = 20001
    rng = np.random.default_rng(23)
    x = rng.integers(0, Q, size=(count, 1024), dtype=np.uint64)
    ref = plan.forward(x)
    dx, dy = vp(), vp()
    check(lib().fhe_hip_alloc(0, x.nbytes, ctypes.byref(dx)))
    check(lib().fhe_hip_alloc(0, x.nbytes, ctypes.byref(dy)))
    try:
        check(lib().fhe_hip_copy_to_device(dx, ptr(x), x.nbytes))
        plan.run_device(dx.value, dy.value, count, False)
        check(lib().fhe_hip_synchronize(0))
        y = np.zeros_like(x)
        xin = np.zeros_like(x)
        check(lib().fhe_hip_copy_to_host(ptr(y), dy, x.nbytes))
        check(lib().fhe_hip_copy_to_host(ptr(xin), dx, x.nbytes))
    finally:
        lib().fhe_hip_free(dx)
        lib().fhe_hip_free(dy)
    assert np.array_equal(y, ref)
    assert np.array_equal(xin, x)   # input untouched
    rows = [0, 1, 4095, 4096, 12345, count - 2, count - 1]
    assert np.array_equal(ref[rows], restatement.ntt(Q, plan.psi, x[rows]))
    assert np.array_equal(plan.inverse(ref), x)
