"""Multi-input gates and CMUX: EvalBinGate(gate, ctvector) for MAJORITY,
AND3, OR3, AND4, OR4 (binfhe-base-scheme.cpp:129-171) and CMUX (:172-182), against golden
vectors produced by the reference itself (tests/golden/make_golden.py multi) on every input
combination, and against the oracle restatement."""
import hashlib
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SETS = ["std128", "lmkcdey"]
TRUTH = {
    "MAJORITY": lambda b: (b.sum(1) >= 2),
    "AND3": lambda b: b.all(1),
    "OR3": lambda b: b.any(1),
    "AND4": lambda b: b.all(1),
    "OR4": lambda b: b.any(1),
    "CMUX": lambda b: np.where(b[:, 2] == 1, b[:, 1], b[:, 0]),   # ctvector[2] ? ctvector[1] : ctvector[0]
}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.uint64).tobytes()).hexdigest()


_cache = {}


def fixture(name):
    if name not in _cache:
        import sys
        sys.path.insert(0, GOLD)
        from make_golden import multi_inputs
        g = np.load(os.path.join(GOLD, f"gates_multi_{name}.npz"))
        keys, cases = multi_inputs(int(g["paramset"]), int(g["method"]), int(g["key_seed"]))
        _cache[name] = (g, keys, cases)
    return _cache[name]


# ----------------------------------------------------------------- CPU ----
@pytest.mark.parametrize("name", SETS)
def test_multi_inputs_deterministic_and_reference_truth(name):
    g, keys, cases = fixture(name)
    assert sha(keys.bsk) + sha(keys.kskA) + sha(keys.kskB) == str(g["keys_sha"])
    for gname, (gate, k, p, bits, A, B) in cases.items():
        assert "".join(sha(x) for x in A + B) == str(g[f"{gname}_in_sha"]), gname
        assert np.array_equal(g[f"{gname}_bits"], bits)
        # the reference's outputs decrypt (with p) to the gate's truth table
        assert np.array_equal(g[f"{gname}_dec"], TRUTH[gname](bits).astype(np.int64)), gname


@pytest.mark.parametrize("name", SETS)
def test_our_decrypt_of_reference_outputs(name):
    from fhe_amd import binfhe as bf
    g, keys, cases = fixture(name)
    ps, m = int(g["paramset"]), int(g["method"])
    for gname, (gate, k, p, bits, A, B) in cases.items():
        dec = bf.decrypt(ps, m, keys.sk, g[f"{gname}_out_a"].astype(np.uint64), g[f"{gname}_out_b"].astype(np.uint64),
                         p=p)
        assert np.array_equal(dec, g[f"{gname}_dec"]), gname


@pytest.mark.slow
@pytest.mark.parametrize("name", SETS)
def test_oracle_multi_matches_reference_golden(name, restatement):
    from oracle_lib import Restatement
    g, keys, cases = fixture(name)
    O = Restatement(int(g["paramset"]), int(g["method"]))
    for gname, (gate, k, p, bits, A, B) in cases.items():
        if gname == "CMUX":
            ao, bo = O.eval_cmux(keys.bsk, keys.kskA, keys.kskB, A[0], B[0], A[1], B[1], A[2], B[2])
        else:
            ao, bo = O.eval_gate_multi(keys.bsk, keys.kskA, keys.kskB, gate, A, B, p)
            ea, eb = O.eval_gate_multi(keys.bsk, keys.kskA, keys.kskB, gate, A, B, p, stage=1)
            assert sha(ea) + sha(eb) == str(g[f"{gname}_ext_sha"]), gname
        assert np.array_equal(ao, g[f"{gname}_out_a"]) and np.array_equal(bo, g[f"{gname}_out_b"]), gname


# ----------------------------------------------------------------- GPU ----
_engines = {}


def engine(name):
    from fhe_amd import binfhe as bf
    if name not in _engines:
        g, keys, _ = fixture(name)
        e = bf.GateEngine(int(g["paramset"]), int(g["method"]))
        e.load_keys(keys.bsk, keys.kskA, keys.kskB)
        _engines[name] = e
    return _engines[name]


@pytest.mark.gpu
@pytest.mark.parametrize("name", SETS)
def test_gpu_multi_gates_bit_exact_vs_reference(name):
    g, keys, cases = fixture(name)
    e = engine(name)
    for gname, (gate, k, p, bits, A, B) in cases.items():
        if gname == "CMUX":
            ao, bo = e.eval_cmux(A[0], B[0], A[1], B[1], A[2], B[2])
        else:
            ao, bo = e.eval_gate_multi(gate, A, B, p)
            ea, eb = e.eval_gate_multi(gate, A, B, p, extended=True)
            assert sha(ea) + sha(eb) == str(g[f"{gname}_ext_sha"]), gname
        assert np.array_equal(ao, g[f"{gname}_out_a"]), gname
        assert np.array_equal(bo, g[f"{gname}_out_b"]), gname


@pytest.mark.gpu
@pytest.mark.parametrize("name", SETS)
def test_gpu_multi_ragged_vs_oracle_and_large_truth(name, restatement):
    """ragged batch sizes vs the oracle, and a 4096-tuple batch (tiled key switch, 2 x 4096-gate
    CMUX first level) checked by decryption."""
    from fhe_amd import binfhe as bf
    from oracle_lib import Restatement
    g, keys, _ = fixture(name)
    ps, m = int(g["paramset"]), int(g["method"])
    O = Restatement(ps, m)
    e = engine(name)
    rng = np.random.default_rng(31)
    for count, gname, gate, k, p in ((5, "AND4", 9, 4, 8), (3, "OR3", 8, 3, 6), (7, "CMUX", 13, 3, 4)):
        bits = rng.integers(0, 2, (count, k))
        ins = [bf.encrypt(ps, m, keys.sk, bits[:, j], 500 + 10 * count + j, p) for j in range(k)]
        A, B = [x[0] for x in ins], [x[1] for x in ins]
        if gate == 13:
            ao, bo = e.eval_cmux(A[0], B[0], A[1], B[1], A[2], B[2])
            oa, ob = O.eval_cmux(keys.bsk, keys.kskA, keys.kskB, A[0], B[0], A[1], B[1], A[2], B[2])
        else:
            ao, bo = e.eval_gate_multi(gate, A, B, p)
            oa, ob = O.eval_gate_multi(keys.bsk, keys.kskA, keys.kskB, gate, A, B, p)
        assert np.array_equal(ao, oa) and np.array_equal(bo, ob), gname
        assert np.array_equal(bf.decrypt(ps, m, keys.sk, ao, bo, p=p), TRUTH[gname](bits).astype(np.int64))
    count = 4096
    for gname, gate, k, p in (("MAJORITY", 6, 3, 4), ("CMUX", 13, 3, 4)):
        bits = rng.integers(0, 2, (count, k))
        ins = [bf.encrypt(ps, m, keys.sk, bits[:, j], 900 + j, p) for j in range(k)]
        A, B = [x[0] for x in ins], [x[1] for x in ins]
        if gate == 13:
            ao, bo = e.eval_cmux(A[0], B[0], A[1], B[1], A[2], B[2])
        else:
            ao, bo = e.eval_gate_multi(gate, A, B, p)
        assert np.array_equal(bf.decrypt(ps, m, keys.sk, ao, bo, p=p), TRUTH[gname](bits).astype(np.int64)), gname


@pytest.mark.gpu
def test_gpu_binfhecontext_multiinput_and_cmux():
    """UnitTestFHEW.cpp:411-500 (MULTIINPUT, CMUX) through the BinFHEContext mirror."""
    from fhe_amd import binfhe as bf
    from fhe_amd._lib import FheHipError
    cc = bf.BinFHEContext()
    cc.GenerateBinFHEContext(bf.STD128, bf.GINX)
    sk = cc.KeyGen()
    cc.BTKeyGen(sk)
    for gate, k, p, exp in ((bf.AND3, 3, 6, 0), (bf.OR3, 3, 6, 1), (bf.AND4, 4, 8, 0), (bf.OR4, 4, 8, 1),
                            (bf.MAJORITY, 3, 4, 1)):
        msgs = [1, 1, 0] if k == 3 else [1, 0, 0, 0]
        cts = [cc.Encrypt(sk, x, None, p) for x in msgs]
        assert cc.Decrypt(sk, cc.EvalBinGate(gate, cts), p) == exp, gate
    c1, c2, c3, c4 = (cc.Encrypt(sk, x) for x in (1, 1, 0, 0))
    assert cc.Decrypt(sk, cc.EvalBinGate(bf.CMUX, [c1, c3, c4])) == 1
    assert cc.Decrypt(sk, cc.EvalBinGate(bf.CMUX, [c1, c3, c2])) == 0
    assert cc.Decrypt(sk, cc.EvalNOT(c1)) == 0 and cc.Decrypt(sk, cc.EvalNOT(c3)) == 1
    with pytest.raises(FheHipError):
        cc.EvalBinGate(bf.AND3, [c1, c1, c2])
    with pytest.raises(FheHipError):
        cc.EvalBinGate(bf.CMUX, [c1, c2])
    with pytest.raises(FheHipError):     # 2-input gate through the vector API
        cc.engine.eval_gate_multi(bf.AND, [c1.a[None], c2.a[None]], [np.array([c1.b], np.uint64),
                                                                      np.array([c2.b], np.uint64)], 4)
