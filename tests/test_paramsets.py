"""The other BINFHE_PARAMSET rows (binfhecontext.cpp:113-159) on the device path, bit-exact against
the reference's own outputs for the same keys and ciphertexts (tests/golden/gates_<set>.npz, made by
tests/golden/make_golden.py wider from oracle/_ref):

  * the 32-bit kernels (N = 1024, Q < 2^28, digitsG = 3): MEDIUM (GINX, AP, LMKCDEY),
    STD128_3_LMKCDEY, STD128Q_LMKCDEY, LPF_STD128_LMKCDEY (n = 556: 1024-column key-switching rows,
    qKS = 2^15);
  * the 64-bit kernel (bootstrap_wide.hip) for every other GINX set: digitsG = 4 / 5 (STD128_3/4,
    STD128Q, LPF_STD128/Q, STD256*), N = 2048 with 29- to 50-bit Q (STD128Q_3/4, STD192*, STD256*),
    qKS up to 2^21;
  * its op-list form (k_blind_rotate_wide_ops) for every other LMKCDEY set: STD128_4, STD128Q_3/4,
    STD192*, STD256*, LPF_STD128Q _LMKCDEY (digitsG 2-5, N = 1024 / 2048, n up to 1320);
  * TOY (N = 512) with GINX, AP (the DM op list) and LMKCDEY, SIGNED_MOD_TEST: the prime qKS of
    modKS = PRIME, STD256Q_3: baseKS = 21 (key-switching digits by remainders).
Six gate types per set, final outputs and the extended ctExt."""
import hashlib
import os
import sys

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLD)
from make_golden import GATES, WIDER_PER_GATE, WIDER_SETS  # noqa: E402

TRUTH = {0: lambda a, b: a | b, 1: lambda a, b: a & b, 2: lambda a, b: 1 - (a | b), 3: lambda a, b: 1 - (a & b),
         4: lambda a, b: a ^ b, 5: lambda a, b: 1 - (a ^ b)}
SETS = [s for s in WIDER_SETS if os.path.exists(os.path.join(GOLD, f"gates_{s}.npz"))]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.uint64).tobytes()).hexdigest()


def golden(name):
    return np.load(os.path.join(GOLD, f"gates_{name}.npz"))


def test_wider_goldens_present():
    assert len(SETS) >= 40, SETS


@pytest.mark.parametrize("name", SETS)
def test_reference_wider_outputs_decrypt_to_truth_table(name):
    """the reference, run on our keys, computes every gate correctly (its own decryptions)"""
    g = golden(name)
    pg = WIDER_PER_GATE
    for i, gate in enumerate(g["gates"]):
        exp = TRUTH[int(gate)](g["bits1"][i], g["bits2"][i])
        assert np.array_equal(g["ref_dec"][i * pg:(i + 1) * pg], exp), (name, int(gate))


@pytest.mark.gpu
@pytest.mark.parametrize("name", SETS)
def test_gpu_wider_paramset_gates_bit_exact_vs_reference(name):
    from fhe_amd import binfhe as bf
    from make_golden import gate_inputs
    g = golden(name)
    ps, m = int(g["paramset"]), int(g["method"])
    pg = WIDER_PER_GATE
    keys, bits1, bits2, a1, b1, a2, b2 = gate_inputs(ps, m, int(g["key_seed"]), pg)
    assert sha(keys.bsk) + sha(keys.kskA) + sha(keys.kskB) == str(g["keys_sha"])
    assert sha(a1) + sha(b1) + sha(a2) + sha(b2) == str(g["in_sha"])
    e = bf.GateEngine(ps, m, device=0)
    e.load_keys(keys.bsk, keys.kskA, keys.kskB)
    del keys
    outs, outb, exts = [], [], []
    for i, gate in enumerate(GATES.values()):
        sl = slice(i * pg, (i + 1) * pg)
        ao, bo = e.eval_gate(gate, a1[sl], b1[sl], a2[sl], b2[sl])
        ea, eb = e.eval_gate_extended(gate, a1[sl], b1[sl], a2[sl], b2[sl])
        outs.append(ao); outb.append(bo); exts.append(ea)
    e.close()
    assert np.array_equal(np.concatenate(outs), g["out_a"].astype(np.uint64))
    assert np.array_equal(np.concatenate(outb), g["out_b"].astype(np.uint64))
    assert sha(np.concatenate(exts)) == str(g["ext_sha"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["std128_3", "std128q", "std128_4", "lpf_std128", "lpf_std128q", "std128_4_lmkcdey",
                                  "std128q_3_lmkcdey", "lpf_std128q_lmkcdey"])
def test_gpu_digitsg4_split_kernel_matches_64bit_accumulator(name, monkeypatch):
    """digitsG = 4 at N = 1024, Q < 2^27 (q = 1024, and q = 2N: the full monomial table): the 32-bit
    split kernels with three digits per component (launch_blind_rotate_ginx3; LMKCDEY:
    launch_blind_rotate_lmk3, the default) against the 64-bit accumulator the set ran on before
    (FHE_HIP_GINX3=0, bootstrap_wide.hip) on 777 gates of every 2-input type, final outputs and
    extended ctExt; both also decrypt to the truth table"""
    from fhe_amd import binfhe as bf
    from make_golden import GATE_SETS
    ps, m = GATE_SETS[name]
    keys = bf.keygen(ps, m, 31)
    B = 777
    rng = np.random.default_rng(5)
    x1, x2 = rng.integers(0, 2, B), rng.integers(0, 2, B)
    a1, b1 = bf.encrypt(ps, m, keys.sk, x1, 11)
    a2, b2 = bf.encrypt(ps, m, keys.sk, x2, 12)
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("FHE_HIP_GINX3", flag)
        e = bf.GateEngine(ps, m, device=0)
        e.load_keys(keys.bsk, keys.kskA, keys.kskB)
        res[flag] = [(e.eval_gate(gate, a1, b1, a2, b2), e.eval_gate_extended(gate, a1, b1, a2, b2))
                     for gate in GATES.values()]
        e.close()
    for (gname, gate), (fast, ref) in zip(GATES.items(), zip(res["1"], res["0"])):
        for u, v in zip(fast, ref):
            for s, t in zip(u, v):
                assert np.array_equal(s, t), (name, gname)
        dec = bf.decrypt(ps, m, keys.sk, fast[0][0], fast[0][1])
        assert np.array_equal(dec, TRUTH[gate](x1, x2)), (name, gname)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["std128_3", "std128q", "std256q_3", "toy", "signed_mod_test"])
def test_gpu_digitsg4_keyswitch_vs_reference(name):
    """the 32-bit key switch these sets now use (u16 rows of 1024 columns; gate-tiled with 64 staged
    slices at baseKS = 64 (STD128_3), 32 at baseKS = 32 (STD128Q); row split below 4096) on uniform
    inputs mod qKS, incl. a ragged last tile, vs the reference's own LWEEncryptionScheme::KeySwitch
    (oracle/_ref, the restatement covers the STD128 sets only).  STD256Q_3 (round 5): baseKS 21, its
    four digits by division, 21 staged slices, 1408-column rows at n = 1400.  TOY / SIGNED_MOD_TEST (round 6):
    the prime qKS (modKS = PRIME, qKS = Q) on the u32-row tiled kernel with sums kept mod qKS, baseKS 25 with six /
    seven digits by division, 512-gate tiles"""
    from fhe_amd import binfhe as bf
    from make_golden import GATE_SETS
    from oracle_lib import Ref
    ps, m = GATE_SETS[name]
    keys = bf.keygen(ps, m, 41)
    O = Ref(ps, m)
    O.load_keys(keys.bsk, keys.kskA, keys.kskB)
    e = bf.GateEngine(ps, m, device=0)
    e.load_keys(keys.bsk, keys.kskA, keys.kskB)
    P = e.params
    rng = np.random.default_rng(78)
    for count in (300, 4096 + 259):
        a = rng.integers(0, P.qKS, (count, P.N), dtype=np.uint64)
        b = rng.integers(0, P.qKS, count, dtype=np.uint64)
        ga, gb = e.keyswitch(a, b)
        oa, ob = O.keyswitch(a, b)
        assert np.array_equal(ga, oa) and np.array_equal(gb, ob), count
    e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["std128_3", "std128_4_lmkcdey"])
def test_gpu_digitsg4_multi_input_gates_vs_reference(name):
    """MAJORITY / AND3 / OR3 / AND4 / OR4 / CMUX (binfhe-base-scheme.cpp:129-187) on the split kernels
    (K1s GINX, K1m LMKCDEY) over every input combination, against the reference's own
    EvalBinGate(gate, ctvector) (oracle/_ref) on the same keys and ciphertexts"""
    from fhe_amd import binfhe as bf
    from make_golden import GATE_SETS, multi_inputs
    from oracle_lib import Ref
    truth = {"MAJORITY": lambda b: b.sum(1) >= 2, "AND3": lambda b: b.all(1), "OR3": lambda b: b.any(1),
             "AND4": lambda b: b.all(1), "OR4": lambda b: b.any(1),
             "CMUX": lambda b: np.where(b[:, 2] == 1, b[:, 1], b[:, 0])}
    ps, m = GATE_SETS[name]
    keys, cases = multi_inputs(ps, m, 0xD4 + ps)
    ref = Ref(ps, m)
    ref.load_keys(keys.bsk, keys.kskA, keys.kskB)
    e = bf.GateEngine(ps, m, device=0)
    e.load_keys(keys.bsk, keys.kskA, keys.kskB)
    for gname, (gate, k, p, bits, A, B) in cases.items():
        if gname == "CMUX":
            ao, bo = e.eval_cmux(A[0], B[0], A[1], B[1], A[2], B[2])
        else:
            ao, bo = e.eval_gate_multi(gate, A, B, p)
        ra, rb = ref.eval_gate_multi(gate, A, B, p)
        assert np.array_equal(ao, ra) and np.array_equal(bo, rb), (name, gname)
        dec = bf.decrypt(ps, m, keys.sk, ao, bo, p=p)
        assert np.array_equal(dec, truth[gname](bits).astype(np.int64)), (name, gname)
    e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["std256q", "std256q_lmkcdey", "std256q_3_lmkcdey", "std256_3_lmkcdey",
                                  "std256_4_lmkcdey", "std256q_4_lmkcdey", "std256", "std256_3",
                                  "std256_4", "std256q_3", "std256q_4"])
def test_gpu_n2k_kernel_matches_64bit_accumulator(monkeypatch, name):
    """N = 2048, Q < 2^27, digitsG = 4: K1w, the register-resident two-waves-per-gate accumulators
    (STD256Q, q = 1024: launch_blind_rotate_n2k; STD256Q_LMKCDEY (28-bit Q) / STD256Q_3_LMKCDEY:
    launch_blind_rotate_lmk2k with 2 / 3 retained digits; STD256_3 / STD256_4_LMKCDEY: 29-bit Q, the forward
    transform reduced after stages 3, 6 and 9; the default),
    against the one-gate-per-workgroup accumulator the sets ran on before (FHE_HIP_N2K=0,
    bootstrap_wide.hip A32) on 333 gates of every 2-input type (final and extended outputs) and on the seam's
    BlindRotate (random accumulators, ciphertexts mod q for GINX and mod 2N for LMKCDEY, as EvalAcc reads
    them); the gates also decrypt to the truth table.  The reference goldens of the sets run in
    test_gpu_wider_paramset_gates_bit_exact_vs_reference on the default kernel."""
    from fhe_amd import binfhe as bf
    ps, m = WIDER_SETS[name]
    assert bf.kernel_path(ps, m) == 4
    keys = bf.keygen(ps, m, 41)
    P = bf.params(ps, m)
    B = 333
    rng = np.random.default_rng(9)
    x1, x2 = rng.integers(0, 2, B), rng.integers(0, 2, B)
    a1, b1 = bf.encrypt(ps, m, keys.sk, x1, 21)
    a2, b2 = bf.encrypt(ps, m, keys.sk, x2, 22)
    amod = 2 * P.N if m == 3 else P.q
    acc_a = rng.integers(0, amod, (5, P.n), dtype=np.uint64)
    acc = rng.integers(0, P.Q, (5, 2, P.N), dtype=np.uint64)
    # GINX seam calls at a second ciphertext modulus (EvalAcc reads a_i with the ciphertext's modulus): 2N on the
    # half-resolution rows (no even exponents: K5 must take them), N / 2 on the q = 2N rows (their
    # full-resolution kernel takes any modulus)
    acc_a2 = rng.integers(0, 2 * P.N, (5, P.n), dtype=np.uint64)
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("FHE_HIP_N2K", flag)
        e = bf.GateEngine(ps, m, device=0)
        e.load_keys(keys.bsk, keys.kskA, keys.kskB)
        res[flag] = [(e.eval_gate(gate, a1, b1, a2, b2), e.eval_gate_extended(gate, a1, b1, a2, b2))
                     for gate in GATES.values()]
        res[flag].append(((e.blind_rotate_acc(acc_a, amod, acc),), ))
        if m == 2:   # the other ciphertext modulus of the table's resolution: 2N (half table) or q / 2 (full)
            amod2 = 2 * P.N if amod != 2 * P.N else P.N // 2
            res[flag].append(((e.blind_rotate_acc(acc_a2 % amod2, amod2, acc),), ))
        e.close()
    for (gname, gate), (fast, ref) in zip(GATES.items(), zip(res["1"], res["0"])):
        for u, v in zip(fast, ref):
            for s, t in zip(u, v):
                assert np.array_equal(s, t), gname
        dec = bf.decrypt(ps, m, keys.sk, fast[0][0], fast[0][1])
        assert np.array_equal(dec, TRUTH[gate](x1, x2)), gname
    for u, v in zip(res["1"][len(GATES):], res["0"][len(GATES):]):
        assert np.array_equal(u[0][0], v[0][0])


def test_integration_kernel_table_matches_params():
    """INTEGRATION.md's "Which kernel serves a parameter set" table lists every compatible (set, method) pair of
    binfhecontext.cpp:113-159 exactly once, with the `kernel` fhe_hip_params_get reports for it (default kernel
    settings: the FHE_HIP_* knobs unset)"""
    import re
    from fhe_amd import binfhe as bf
    for k in ("FHE_HIP_GINX3", "FHE_HIP_N2K", "FHE_HIP_NARROW"):
        assert k not in os.environ, k
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    text = open(os.path.join(root, "INTEGRATION.md")).read()
    sec = text[text.index("## Which kernel serves a parameter set"):text.index("## Raw key layout")]
    methods = {"AP": bf.AP, "GINX": bf.GINX, "LMKCDEY": bf.LMKCDEY}
    seen = {}
    for line in sec.splitlines():
        cells = [c.strip() for c in line.strip().strip("|").split("|")]
        if len(cells) < 3 or cells[1] not in methods:
            continue
        kernel = int(cells[2])
        for name in (n.strip() for n in cells[0].split(",")):
            ps, m = bf.PARAMSETS.index(name), methods[cells[1]]
            assert (ps, m) not in seen, (name, cells[1])
            assert bf.method_compatible(ps, m), (name, cells[1])
            seen[(ps, m)] = kernel
            assert bf.params(ps, m).kernel == kernel, (name, cells[1], bf.params(ps, m).kernel, kernel)
    want = {(ps, m) for ps in range(len(bf.PARAMSETS)) for m in methods.values() if bf.method_compatible(ps, m)}
    assert set(seen) == want, sorted(want - set(seen))
    assert re.search(r"1 = K1, 2 = K1s / K1m, 3 = K5 A32, 4 = K1w, 0 = K5 A64", sec)
