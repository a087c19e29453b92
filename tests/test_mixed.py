"""Ciphertexts mod Q as gate and bootstrap inputs: the reference key-switches every
input whose modulus is Q before the gate (binfhe-base-scheme.cpp:92-93 two-input gates, :150-152 ctvector
gates, :200-201 Bootstrap, whose b constant is the ORIGINAL modulus >> 2), and inputs mod q and mod Q may be
mixed within one call.  Golden vectors are the reference's own outputs (tests/golden/make_golden.py mixed) on
the flows of UnitTestFHEWExtended.cpp:37-153 (extended outputs chained into the next gate, SMALL_DIM and
LARGE_DIM encryptions mixed) and on every 2-input gate, MAJORITY, CMUX and Bootstrap with mixed columns."""
import ctypes
import hashlib
import os
import sys

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLD)
SETS = [s for s in ("std128", "lmkcdey", "std192", "std256q") if os.path.exists(os.path.join(GOLD, f"mixed_{s}.npz"))]
TRUTH = {"OR": lambda a, b: a | b, "AND": lambda a, b: a & b, "NOR": lambda a, b: 1 - (a | b),
         "NAND": lambda a, b: 1 - (a & b), "XOR": lambda a, b: a ^ b, "XNOR": lambda a, b: 1 - (a ^ b)}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.uint64).tobytes()).hexdigest()


_cache = {}


def fixture(name):
    if name not in _cache:
        from make_golden import mixed_cases
        g = np.load(os.path.join(GOLD, f"mixed_{name}.npz"))
        keys, skN, cases = mixed_cases(int(g["paramset"]), int(g["method"]), int(g["key_seed"]))
        _cache[name] = (g, keys, skN, cases)
    return _cache[name]


def columns(case):
    op, p, bits, c = case
    return op, p, bits, [x[0] for x in c], [x[1] for x in c], [x[2] for x in c]


# ----------------------------------------------------------------- CPU ----
@pytest.mark.parametrize("name", SETS)
def test_mixed_inputs_deterministic_and_reference_truth(name):
    """our seeded keys, RLWE secret and inputs are the ones the goldens were made from, and the reference's
    outputs decrypt to the truth tables (mod-q rows of Bootstrap: the input bit)"""
    g, keys, skN, cases = fixture(name)
    assert sha(keys.bsk) + sha(keys.kskA) + sha(keys.kskB) == str(g["keys_sha"])
    assert sha(skN) == str(g["skN_sha"])
    for cname, case in cases.items():
        op, p, bits, A, B, F = columns(case)
        assert "".join(sha(x) for x in A + B) == str(g[f"{cname}_in_sha"]), cname
        assert np.array_equal(np.array(F), g[f"{cname}_flags"])
        dec = g[f"{cname}_dec"]
        if cname.startswith("gate_"):
            assert np.array_equal(dec, TRUTH[cname[5:]](bits[0], bits[1])), cname
        elif cname == "majority":
            assert np.array_equal(dec, (bits.sum(0) >= 2).astype(np.int64))
        elif cname == "cmux":
            assert np.array_equal(dec, np.where(bits[2] == 1, bits[1], bits[0]))
        elif cname == "boot":   # a mod-q input refreshes to its bit (:190-220)
            assert np.array_equal(dec[F[0] == 0], bits[0][F[0] == 0])
        elif cname == "flow2":  # NAND(OR(s, l), AND(l, s)) = NAND(s, l) (UnitTestFHEWExtended.cpp:53-65)
            assert np.array_equal(dec, 1 - (bits[0] & bits[1]))


def test_large_dim_encryptions_decrypt_under_skN():
    """LARGE_DIM encryptions (dimension N, mod Q) decrypt under skN; SwitchCTtoqn's key is made from it"""
    from fhe_amd import binfhe as bf
    ps, m = bf.STD128, bf.GINX
    P = bf.params(ps, m)
    skN = bf.keygen_ring_secret(ps, m, 77)
    bits = np.random.default_rng(1).integers(0, 2, 64)
    for p in (4, 6, 8):
        a, b = bf.encrypt_large(ps, m, skN, bits % p, 99, p)
        assert a.shape == (64, P.N) and int(a.max()) < P.Q and int(b.max()) < P.Q
        assert np.array_equal(bf.decrypt(ps, m, skN, a, b, mod=P.Q, p=p), bits % p)


def test_mixed_capi_exported_and_validates():
    from fhe_amd import binfhe as bf
    L = bf.L()
    for sym in ("fhe_hip_switch_to_qn_batch", "fhe_hip_switch_to_qn_batch_device", "fhe_hip_eval_mixed_batch",
                "fhe_hip_eval_mixed_batch_device", "fhe_hip_keygen_ring_secret", "fhe_hip_encrypt_large"):
        assert hasattr(L, sym), sym
    # null context / arrays are rejected without touching a device
    assert L.fhe_hip_eval_mixed_batch(None, 1, 2, 4, 1, None, None, None, None, None, 0) == -1
    assert L.fhe_hip_switch_to_qn_batch(None, 1, None, None, None, None) == -1


# ----------------------------------------------------------------- GPU ----
_eng = {}


def engine(name):
    if name not in _eng:
        from fhe_amd import binfhe as bf
        g, keys, skN, cases = fixture(name)
        e = bf.GateEngine(int(g["paramset"]), int(g["method"]), 0)
        e.load_keys(keys.bsk, keys.kskA, keys.kskB)
        _eng[name] = e
    return _eng[name]


@pytest.mark.gpu
@pytest.mark.parametrize("name", SETS)
def test_gpu_mixed_inputs_bit_exact_vs_reference(name):
    """every 2-input gate, MAJORITY, CMUX and Bootstrap (p = 4 and 8) on columns mixing ciphertexts mod q and
    mod Q: final outputs and ctExt == the reference, through the C-ABI (fhe_hip_eval_mixed_batch)"""
    from fhe_amd import binfhe as bf
    g, keys, skN, cases = fixture(name)
    e = engine(name)
    for cname, case in cases.items():
        if cname.startswith("flow"):
            continue
        op, p, bits, A, B, F = columns(case)
        ao, bo = e.eval_mixed(op, A, B, F, p)
        assert np.array_equal(ao, g[f"{cname}_out_a"]) and np.array_equal(bo, g[f"{cname}_out_b"]), (name, cname)
        if op != bf.CMUX:
            ea, eb = e.eval_mixed(op, A, B, F, p, extended=True)
            assert sha(ea) + sha(eb) == str(g[f"{cname}_ext_sha"]), (name, cname)
            assert np.array_equal(ea[0], g[f"{cname}_ext_a0"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", SETS)
def test_gpu_extended_flows_chained_bit_exact(name):
    """UnitTestFHEWExtended.cpp:37-136 as batches: G1(v, extended), G2(v, extended) on SMALL_DIM / LARGE_DIM
    inputs, then NAND of the two ctExt (both mod Q) -- each stage == the reference"""
    from make_golden import FLOW_GATES
    g, keys, skN, cases = fixture(name)
    e = engine(name)
    for cname, (g1, g2) in FLOW_GATES.items():
        op, p, bits, A, B, F = columns(cases[cname])
        e1 = e.eval_mixed(g1, A, B, F, p, extended=True)
        if cname == "flow2":
            e2 = e.eval_mixed(g2, A[::-1], B[::-1], F[::-1], p, extended=True)
        else:
            e2 = e.eval_mixed(g2, A, B, F, p, extended=True)
        assert sha(e1[0]) + sha(e1[1]) == str(g[f"{cname}_ext1_sha"]), (name, cname)
        assert sha(e2[0]) + sha(e2[1]) == str(g[f"{cname}_ext2_sha"]), (name, cname)
        ones = np.ones(len(B[0]), np.uint8)
        ao, bo = e.eval_mixed(3, [e1[0], e2[0]], [e1[1], e2[1]], [ones, ones], 4)
        assert np.array_equal(ao, g[f"{cname}_out_a"]) and np.array_equal(bo, g[f"{cname}_out_b"]), (name, cname)


@pytest.mark.gpu
@pytest.mark.parametrize("name", SETS[:2])
def test_gpu_switch_to_qn_equals_reference_stages(name):
    """SwitchCTtoqn alone (fhe_hip_switch_to_qn_batch) == the reference's ModSwitch -> KeySwitch -> ModSwitch
    on LARGE_DIM ciphertexts"""
    from oracle_lib import Ref, ref_available
    if not ref_available():
        pytest.skip("reference oracle not built")
    from fhe_amd import binfhe as bf
    g, keys, skN, cases = fixture(name)
    ps, m = int(g["paramset"]), int(g["method"])
    e = engine(name)
    a, b = bf.encrypt_large(ps, m, skN, np.arange(40) % 2, 5, 4)
    ga, gb = e.switch_to_qn(a, b)
    ref = Ref(ps, m)
    ref.load_keys(keys.bsk, keys.kskA, keys.kskB)
    ma, mb = ref.modswitch(ref.Q, ref.qKS, a, b)
    ka, kb = ref.keyswitch(ma, mb)
    ra, rb = ref.modswitch(ref.qKS, ref.q, ka, kb)
    assert np.array_equal(ga, ra) and np.array_equal(gb, rb)
    assert np.array_equal(bf.decrypt(ps, m, keys.sk, ga, gb), np.arange(40) % 2)


@pytest.mark.gpu
def test_gpu_mixed_device_entry_point_matches_host():
    """fhe_hip_eval_mixed_batch_device (device columns and flags, the context's stream) == the host entry"""
    from fhe_amd import binfhe as bf
    from fhe_amd._lib import check, vp
    g, keys, skN, cases = fixture("std128")
    e = engine("std128")
    L = bf.L()
    op, p, bits, A, B, F = columns(cases["gate_XOR"])
    bufs = []

    def dev(x):
        x = np.ascontiguousarray(x)
        d = vp()
        check(L.fhe_hip_alloc(0, max(x.nbytes, 8), ctypes.byref(d)))
        check(L.fhe_hip_copy_to_device(d, x.ctypes.data, x.nbytes))
        bufs.append(d)
        return d

    P = e.params
    da, db, dl = [dev(x) for x in A], [dev(x) for x in B], [dev(np.asarray(x, np.uint8)) for x in F]
    cnt = len(B[0])
    dao, dbo = dev(np.zeros((cnt, P.n), np.uint64)), dev(np.zeros(cnt, np.uint64))
    pa = (vp * 2)(*[d.value for d in da])
    pb = (vp * 2)(*[d.value for d in db])
    pl = (vp * 2)(*[d.value for d in dl])
    check(L.fhe_hip_eval_mixed_batch_device(e._h, op, 2, p, cnt, pa, pb, pl, dao, dbo, 0, None))
    check(L.fhe_hip_synchronize(0))
    ao, bo = np.zeros((cnt, P.n), np.uint64), np.zeros(cnt, np.uint64)
    check(L.fhe_hip_copy_to_host(ao.ctypes.data, dao, ao.nbytes))
    check(L.fhe_hip_copy_to_host(bo.ctypes.data, dbo, bo.nbytes))
    for d in bufs:
        L.fhe_hip_free(d)
    assert np.array_equal(ao, g["gate_XOR_out_a"]) and np.array_equal(bo, g["gate_XOR_out_b"])


@pytest.mark.gpu
def test_gpu_unittest_fhew_extended_through_the_mirror():
    """UnitTestFHEWExtended.cpp:37-153 verbatim through the BinFHEContext mirror (TOY, GINX): moduli of
    every intermediate and the final decryptions"""
    from fhe_amd import binfhe as bf
    cc = bf.BinFHEContext()
    cc.GenerateBinFHEContext(bf.TOY, bf.GINX)
    sk = cc.KeyGen()
    cc.BTKeyGen(sk)
    Q = cc.params.Q
    for p, gates, expect in ((4, None, 0), (6, (bf.OR3, bf.AND3), 1), (8, (bf.OR4, bf.AND4), 1)):
        small = cc.Encrypt(sk, 1, bf.SMALL_DIM, p)
        large = cc.Encrypt(sk, 1, bf.LARGE_DIM, p)
        assert small.modulus != Q and large.modulus == Q
        if gates is None:   # EvalBinGate2
            ct11 = cc.EvalBinGate(bf.OR, small, large, True)
            ct12 = cc.EvalBinGate(bf.AND, large, small, True)
        else:
            v = [small, large, cc.Encrypt(sk, 0, bf.SMALL_DIM, p)]
            if p == 8:
                v.append(cc.Encrypt(sk, 1, bf.LARGE_DIM, p))
            ct11 = cc.EvalBinGate(gates[0], v, True)
            ct12 = cc.EvalBinGate(gates[1], v, True)
            assert ct11.p == p and ct12.p == p
        assert ct11.modulus == Q and ct12.modulus == Q
        ct2 = cc.EvalBinGate(bf.NAND, ct11, ct12, False)
        assert ct2.modulus != Q and ct2.p == 4
        assert cc.Decrypt(sk, ct2) == expect, p
    ct1 = cc.Bootstrap(cc.Encrypt(sk, 1, bf.SMALL_DIM, 4), True)
    ct0 = cc.Bootstrap(cc.Encrypt(sk, 0, bf.LARGE_DIM, 4), True)
    assert ct1.modulus == Q and ct0.modulus == Q
