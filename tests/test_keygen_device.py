"""BTKeyGen on the GPU (KeyGenCGGI rgsw-acc-cggi.cpp:71-96, KeyGenDM
rgsw-acc-dm.cpp:80-114, KeyGenLMKCDEY / KeyGenAuto rgsw-acc-lmkcdey.cpp:160-226, KeySwitchGen
lwe-pke.cpp:264-344).  The device generator reproduces the seeded host generator bit for bit, so the
keys it produces hash to the keys the reference itself was run on for the gate goldens
(tests/golden/gates_*.npz keys_sha), and gates evaluated with them reproduce the reference's outputs."""
import hashlib
import os
import time

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SETS = ["std128", "lmkcdey", "ap"]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.uint64).tobytes()).hexdigest()


def test_keygen_secret_is_keygen_sk():
    from fhe_amd import binfhe as bf
    g = np.load(os.path.join(GOLD, "gates_std128.npz"))
    ps, m, seed = int(g["paramset"]), int(g["method"]), int(g["key_seed"])
    assert np.array_equal(bf.keygen_secret(ps, m, seed), bf.keygen(ps, m, seed).sk)


@pytest.mark.gpu
@pytest.mark.parametrize("name", SETS)
def test_gpu_keygen_matches_reference_keys_and_gates(name):
    import sys
    sys.path.insert(0, GOLD)
    from make_golden import gate_inputs_for
    from fhe_amd import binfhe as bf
    g = np.load(os.path.join(GOLD, f"gates_{name}.npz"))
    ps, m, seed = int(g["paramset"]), int(g["method"]), int(g["key_seed"])
    sk = bf.keygen_secret(ps, m, seed)
    e = bf.GateEngine(ps, m)
    ks = e.keygen_device(sk, seed, export=True)
    assert sha(ks.bsk) + sha(ks.kskA) + sha(ks.kskB) == str(g["keys_sha"])
    del ks
    e2 = bf.GateEngine(ps, m)
    t0 = time.perf_counter()
    e2.keygen_device(sk, seed)                    # keys stay on the device
    print(f"{name}: device BTKeyGen {1e3 * (time.perf_counter() - t0):.1f} ms")
    bits1, bits2, a1, b1, a2, b2 = gate_inputs_for(ps, m, seed, sk)
    pg = g["bits1"].shape[1]
    for i, gate in enumerate(g["gates"]):
        sl = slice(i * pg, (i + 1) * pg)
        ao, bo = e2.eval_gate(int(gate), a1[sl], b1[sl], a2[sl], b2[sl])
        assert np.array_equal(ao, g["out_a"][sl]) and np.array_equal(bo, g["out_b"][sl]), int(gate)


@pytest.mark.gpu
def test_gpu_binfhecontext_btkeygen_on_device():
    from fhe_amd import binfhe as bf
    for ps, m in ((bf.STD128, bf.GINX), (bf.STD128_LMKCDEY, bf.LMKCDEY)):
        cc = bf.BinFHEContext()
        cc.GenerateBinFHEContext(ps, m)
        sk = cc.KeyGen()
        cc.BTKeyGen(sk)
        for x in range(2):
            for y in range(2):
                r = cc.EvalBinGate(bf.NAND, cc.Encrypt(sk, x), cc.Encrypt(sk, y))
                assert cc.Decrypt(sk, r) == 1 - (x & y)
