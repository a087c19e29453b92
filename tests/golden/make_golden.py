"""Generates the committed golden vectors in tests/golden/ by running the
REFERENCE itself (oracle/_ref/libfhe_ref.so, compiled from /root/reference by
oracle/Makefile) on seeded inputs.  Run here (where the reference exists):

    make -C oracle -j8 && python tests/golden/make_golden.py [ntt|gates|all]

Fixtures are data only (inputs + the reference's outputs + hashes).
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle_lib import AP, GINX, LMKCDEY, STD128, STD128_AP, STD128_LMKCDEY, Ref  # noqa: E402

NTT_MODULI = {
    "q60": 1152921504606830593,   # poly-benchmark-1k (benchmark/src/poly-benchmark-1k.cpp:40-50)
    "std128": 134215681,          # STD128 Q = LastPrime(27, 2048)
    "lmkcdey": 268369921,         # STD128_LMKCDEY Q = LastPrime(28, 2048)
}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.uint64).tobytes()).hexdigest()


def make_ntt():
    ref = Ref(None, None)
    for name, Q in NTT_MODULI.items():
        rng = np.random.default_rng(0x5EED0001)
        x = rng.integers(0, Q, size=(64, 1024), dtype=np.uint64)
        x[0] = 0
        x[1] = Q - 1
        fwd, psi = ref.ntt(Q, x, inverse=False)
        inv, _ = ref.ntt(Q, x, inverse=True)   # x taken as EVALUATION input
        np.savez(os.path.join(HERE, f"ntt_{name}.npz"), Q=np.uint64(Q), psi=np.uint64(psi), seed=np.uint64(0x5EED0001),
                 x=x[:4], fwd=fwd[:4], inv=inv[:4],
                 fwd_sha=np.array(sha(fwd)), inv_sha=np.array(sha(inv)))
        print(name, Q, psi, "ok")


def ntt4096_inputs(Q):
    """BASELINE config 2's batch: 4096 polynomials uniform in [0, Q) (seed 0x5EED0002)"""
    return np.random.default_rng(0x5EED0002).integers(0, Q, size=(4096, 1024), dtype=np.uint64)


def make_ntt4096():
    """the reference's SwitchFormat (transformnat-impl.h:302-373, 511-624) on config 2's whole 4096-polynomial
    batch, forward and inverse, as hashes added to tests/golden/ntt_<name>.npz (other fields kept)"""
    ref = Ref(None, None)
    for name, Q in NTT_MODULI.items():
        f = os.path.join(HERE, f"ntt_{name}.npz")
        g = dict(np.load(f))
        x = ntt4096_inputs(Q)
        fwd, psi = ref.ntt(Q, x, inverse=False)
        inv, _ = ref.ntt(Q, x, inverse=True)
        assert psi == int(g["psi"])
        g.update(fwd4096_sha=np.array(sha(fwd)), inv4096_sha=np.array(sha(inv)), seed4096=np.uint64(0x5EED0002))
        np.savez(f, **g)
        print(name, "4096 ok", flush=True)


# cryptoContext archives (Serial::Serialize(cc, BINARY), boolean-serial-binary.cpp:65-71) the reference writes
CONTEXTS = {"std128": (STD128, GINX), "lmkcdey": (STD128_LMKCDEY, LMKCDEY), "ap": (STD128_AP, AP),
            "std128_3": (4, GINX), "std192": (9, GINX), "std128_4_lmkcdey": (23, LMKCDEY), "toy_lmkcdey": (0, LMKCDEY)}


def make_contexts():
    import ctypes
    for name, (ps, m) in CONTEXTS.items():
        ref = Ref(ps, m)
        out = ctypes.create_string_buffer(1 << 16)
        size = ctypes.c_size_t()
        ref.L.ref_serialize_context.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        assert ref.L.ref_serialize_context(ref.h, out, 1 << 16, ctypes.byref(size)) == 0, ref.err()
        with open(os.path.join(HERE, f"context_{name}.bin"), "wb") as f:
            f.write(out.raw[:size.value])
        print("context", name, size.value, flush=True)


GATE_SETS = {"std128": (STD128, GINX), "lmkcdey": (STD128_LMKCDEY, LMKCDEY), "ap": (STD128_AP, AP)}
# the other BINFHE_PARAMSET rows (binfhecontext.cpp:113-159) the device path covers: GINX on every
# non-LMKCDEY set with N = 1024 / 2048 and a power-of-two baseKS / qKS, LMKCDEY on the N = 1024,
# digitsG = 3 sets; reference enum values (binfhe-constants.h:49-95)
WIDER_SETS = {"medium": (1, GINX), "medium_ap": (1, AP), "medium_lmkcdey": (1, LMKCDEY),
              "std128_3": (4, GINX), "std128_4": (5, GINX), "std128q": (6, GINX),
              "std128q_3": (7, GINX), "std128q_4": (8, GINX), "std192": (9, GINX), "std192_3": (10, GINX),
              "std192_4": (11, GINX), "std192q": (12, GINX), "std192q_3": (13, GINX), "std192q_4": (14, GINX),
              "std256": (15, GINX), "std256_3": (16, GINX), "std256_4": (17, GINX), "std256q": (18, GINX),
              "std256q_4": (20, GINX), "std128_3_lmkcdey": (22, LMKCDEY), "std128q_lmkcdey": (24, LMKCDEY),
              "lpf_std128": (39, GINX), "lpf_std128q": (40, GINX), "lpf_std128_lmkcdey": (41, LMKCDEY),
              # LMKCDEY on the 64-bit accumulator (k_blind_rotate_wide_ops): digitsG 2-5, N = 2048
              "std128_4_lmkcdey": (23, LMKCDEY), "std128q_3_lmkcdey": (25, LMKCDEY),
              "std128q_4_lmkcdey": (26, LMKCDEY), "std192_lmkcdey": (27, LMKCDEY), "std192_3_lmkcdey": (28, LMKCDEY),
              "std192_4_lmkcdey": (29, LMKCDEY), "std192q_lmkcdey": (30, LMKCDEY),
              "std192q_3_lmkcdey": (31, LMKCDEY), "std192q_4_lmkcdey": (32, LMKCDEY),
              "std256_lmkcdey": (33, LMKCDEY), "std256_3_lmkcdey": (34, LMKCDEY), "std256_4_lmkcdey": (35, LMKCDEY),
              "std256q_lmkcdey": (36, LMKCDEY), "std256q_3_lmkcdey": (37, LMKCDEY),
              "std256q_4_lmkcdey": (38, LMKCDEY), "lpf_std128q_lmkcdey": (42, LMKCDEY),
              # N = 512 (TOY: all three methods), prime qKS (TOY, SIGNED_MOD_TEST), baseKS = 21 (STD256Q_3)
              "toy": (0, GINX), "toy_ap": (0, AP), "toy_lmkcdey": (0, LMKCDEY), "signed_mod_test": (43, GINX),
              "std256q_3": (19, GINX)}
GATE_SETS.update(WIDER_SETS)
WIDER_PER_GATE = 2
GATES = {"OR": 0, "AND": 1, "NOR": 2, "NAND": 3, "XOR": 4, "XNOR": 5}
PER_GATE = 8


def gate_inputs(ps, m, key_seed, per_gate=PER_GATE):
    """Deterministic keys (fhe_amd host keygen, seeded) + encrypted inputs."""
    from fhe_amd import binfhe as bf
    keys = bf.keygen(ps, m, key_seed)
    return (keys,) + gate_inputs_for(ps, m, key_seed, keys.sk, per_gate)


def gate_inputs_for(ps, m, key_seed, sk, per_gate=PER_GATE):
    """the encrypted inputs of gate_inputs() under the secret key sk (= keygen(key_seed).sk)"""
    from fhe_amd import binfhe as bf
    rng = np.random.default_rng(key_seed)
    bits1 = rng.integers(0, 2, size=(len(GATES), per_gate))
    bits2 = rng.integers(0, 2, size=(len(GATES), per_gate))
    a1, b1 = bf.encrypt(ps, m, sk, bits1.ravel(), key_seed + 1)
    a2, b2 = bf.encrypt(ps, m, sk, bits2.ravel(), key_seed + 2)
    return bits1, bits2, a1, b1, a2, b2


def gate_key_seed(ps, m):
    return 0xB0070000 + ps + (0 if m in (GINX,) or ps in (STD128_LMKCDEY, STD128_AP) else m << 8)


def make_gates(names=("std128", "lmkcdey")):
    for name in names:
        ps, m = GATE_SETS[name]
        key_seed = gate_key_seed(ps, m)
        pg = WIDER_PER_GATE if name in WIDER_SETS else PER_GATE
        keys, bits1, bits2, a1, b1, a2, b2 = gate_inputs(ps, m, key_seed, pg)
        ref = Ref(ps, m)
        ref.load_keys(keys.bsk, keys.kskA, keys.kskB)
        outs, exts, extb, outb = [], [], [], []
        for gi, (gname, g) in enumerate(GATES.items()):
            sl = slice(gi * pg, (gi + 1) * pg)
            ao, bo = ref.eval_gate(g, a1[sl], b1[sl], a2[sl], b2[sl])
            ea, eb = ref.eval_gate(g, a1[sl], b1[sl], a2[sl], b2[sl], extended=True)
            outs.append(ao); outb.append(bo); exts.append(ea); extb.append(eb)
        outs, outb, exts, extb = map(np.concatenate, (outs, outb, exts, extb))
        # intermediates of SwitchCTtoqn on ctExt: ModSwitch(Q -> qKS), KeySwitch, ModSwitch(qKS -> q)
        ms_a, ms_b = ref.modswitch(ref.Q, ref.qKS, exts, extb)
        ks_a, ks_b = ref.keyswitch(ms_a, ms_b)
        dec = np.array([ref.decrypt(keys.sk, outs[i], outb[i], ref.q) for i in range(len(outb))])
        np.savez_compressed(os.path.join(HERE, f"gates_{name}.npz"), paramset=ps, method=m, key_seed=np.uint64(key_seed),
                            gates=np.array(list(GATES.values())), bits1=bits1, bits2=bits2,
                            out_a=outs.astype(np.uint16), out_b=outb.astype(np.uint16),
                            ext_a=exts[::pg // 2].astype(np.uint64 if ref.Q >= 1 << 32 else np.uint32),
                            ext_b=extb.astype(np.uint64),
                            ext_sha=np.array(sha(exts)), ks_sha=np.array(sha(ks_a) + sha(ks_b)),
                            ms_sha=np.array(sha(ms_a) + sha(ms_b)), ref_dec=dec,
                            keys_sha=np.array(sha(keys.bsk) + sha(keys.kskA) + sha(keys.kskB)),
                            in_sha=np.array(sha(a1) + sha(b1) + sha(a2) + sha(b2)))
        print(name, "ok", outs.shape, flush=True)


# multi-input gates (binfhe-base-scheme.cpp:129-187): (gate, k, plaintext modulus) as the
# reference's UnitTestFHEW.cpp:202-224 uses them; every input combination once
MULTI = {"MAJORITY": (6, 3, 4), "AND3": (7, 3, 6), "OR3": (8, 3, 6), "AND4": (9, 4, 8), "OR4": (10, 4, 8),
         "CMUX": (13, 3, 4)}


def multi_inputs(ps, m, key_seed):
    """keys + per gate: bits [2^k][k] (all combinations) and k encrypted input arrays."""
    from fhe_amd import binfhe as bf
    keys = bf.keygen(ps, m, key_seed)
    cases = {}
    for gi, (gname, (g, k, p)) in enumerate(MULTI.items()):
        bits = np.array([[(c >> j) & 1 for j in range(k)] for c in range(1 << k)])
        ins = [bf.encrypt(ps, m, keys.sk, bits[:, j], key_seed + 100 + 8 * gi + j, p) for j in range(k)]
        cases[gname] = (g, k, p, bits, [x[0] for x in ins], [x[1] for x in ins])
    return keys, cases


def make_multi(names=("std128", "lmkcdey")):
    for name in names:
        ps, m = GATE_SETS[name]
        key_seed = 0xB0070000 + ps
        keys, cases = multi_inputs(ps, m, key_seed)
        ref = Ref(ps, m)
        ref.load_keys(keys.bsk, keys.kskA, keys.kskB)
        out = {"paramset": ps, "method": m, "key_seed": np.uint64(key_seed),
               "keys_sha": np.array(sha(keys.bsk) + sha(keys.kskA) + sha(keys.kskB))}
        for gname, (g, k, p, bits, A, B) in cases.items():
            ao, bo = ref.eval_gate_multi(g, A, B, p)
            out[f"{gname}_out_a"] = ao.astype(np.uint16)
            out[f"{gname}_out_b"] = bo.astype(np.uint16)
            out[f"{gname}_bits"] = bits
            out[f"{gname}_in_sha"] = np.array("".join(sha(x) for x in A + B))
            if g != 13:   # CMUX ignores `extended` in the reference (it returns the final NAND)
                ea, eb = ref.eval_gate_multi(g, A, B, p, extended=True)
                out[f"{gname}_ext_sha"] = np.array(sha(ea) + sha(eb))
            dec = [ref.decrypt(keys.sk, ao[i], bo[i], ref.q, p) for i in range(len(bo))]
            out[f"{gname}_dec"] = np.array(dec)
            print(name, gname, "decrypts:", dec)
        np.savez_compressed(os.path.join(HERE, f"gates_multi_{name}.npz"), **out)
        print(name, "multi ok")


# functional bootstrapping (binfhe-base-scheme.cpp:241-521): beta = 128, p = q / 256
FB_LARGE_MOD = 1 << 14


def fb_luts(q, p, N):
    """LUTs as GenerateLUTviaFunction builds them (binfhecontext.cpp:372-390)"""
    def lut_of(f):
        return np.array([(q // p) * f((i * p) // q, p) for i in range(q)], np.uint64)
    luts = {"neg": lut_of(lambda x, p: 1 if x < p // 2 else p - 1),   # negacyclic
            "per": lut_of(lambda x, p: x % 2)}                          # periodic
    if q <= N:
        luts["cube"] = lut_of(lambda x, p: (x ** 3) % p)                # arbitrary (eval-function.cpp)
    return luts


def fb_inputs(ps, m, key_seed):
    """keys; small-precision inputs (every m < p twice, mod q, plaintext modulus p) and
    large-precision inputs (mod 2^14, plaintext modulus P = p 2^14 / q, values around P/2)."""
    from fhe_amd import binfhe as bf
    keys = bf.keygen(ps, m, key_seed)
    P = bf.params(ps, m)
    q = P.q
    p = q // 256
    ms = np.arange(2 * p) % p
    sa, sb = bf.encrypt(ps, m, keys.sk, ms, key_seed + 300, p)
    PL = p * (FB_LARGE_MOD // q)
    xs = np.array([PL // 2 + i - 4 for i in range(8)] + [3, PL - 3, 0, PL // 4])
    la, lb = bf.encrypt(ps, m, keys.sk, xs, key_seed + 301, PL, FB_LARGE_MOD)
    return keys, q, p, ms, sa, sb, PL, xs, la, lb


def make_fb(names=("std128", "lmkcdey")):
    for name in names:
        ps, m = GATE_SETS[name]
        key_seed = 0xB0070000 + ps
        keys, q, p, ms, sa, sb, PL, xs, la, lb = fb_inputs(ps, m, key_seed)
        ref = Ref(ps, m)
        ref.load_keys(keys.bsk, keys.kskA, keys.kskB)
        out = {"paramset": ps, "method": m, "key_seed": np.uint64(key_seed), "ms": ms, "xs": xs,
               "in_sha": np.array(sha(sa) + sha(sb) + sha(la) + sha(lb))}
        for lname, lut in fb_luts(q, p, ref.N).items():
            # one thread: the reference's LMKCDEY EvalFunc crashes under its own OpenMP parallel loop
            # (reproduced with 16 ciphertexts; fine ciphertext by ciphertext)
            ao, bo = ref.eval_func(sa, sb, q, lut, nthreads=1)
            out[f"func_{lname}_a"], out[f"func_{lname}_b"] = ao.astype(np.uint16), bo.astype(np.uint16)
        for rb in (0, 1):
            ao, bo = ref.eval_floor(sa, sb, q, rb)
            out[f"floor{rb}_a"], out[f"floor{rb}_b"] = ao.astype(np.uint16), bo.astype(np.uint16)
        ao, bo = ref.eval_floor(la, lb, FB_LARGE_MOD, 0)
        out["floorL_a"], out["floorL_b"] = ao.astype(np.uint16), bo.astype(np.uint16)
        for ss in (0, 1):
            ao, bo = ref.eval_sign(la, lb, FB_LARGE_MOD, bool(ss))
            out[f"sign{ss}_a"], out[f"sign{ss}_b"] = ao.astype(np.uint16), bo.astype(np.uint16)
        ao, bo = ref.eval_decomp(la, lb, FB_LARGE_MOD)
        out["decomp_a"], out["decomp_b"] = ao.astype(np.uint16), bo.astype(np.uint16)
        np.savez_compressed(os.path.join(HERE, f"fb_{name}.npz"), **out)
        print(name, "fb ok", sorted(k for k in out if k.endswith("_a")))


# the large-precision family GenerateBinFHEContext(set, arbFunc, logQ, N, GINX) (binfhecontext.cpp:55-104):
# name -> (set, arbFunc, logQ); covers every baseG regime (2^27 / 2^18 / 2^14 at N = 2048) and
# logQ = 11 (27-bit Q, N = 1024, baseG = 2^5); one STD128 (n = 1305) case
LARGE_SETS = {"toy12arb": (0, True, 12), "toy17": (0, False, 17), "toy29": (0, False, 29), "toy11": (0, False, 11),
              "std29": (3, False, 29),
              # timeOptimization (:292-303): the three-key map; EvalSign / EvalDecomp from 2^29 walk
              # 2^14 -> 2^18 -> 2^27, from 2^17 they go 2^18 -> 2^27 (binfhe-base-scheme.cpp:409-431)
              "toy29t": (0, False, 29, True), "toy17t": (0, False, 17, True)}


def large_inputs(name):
    """keys (seeded host keygen) and the inputs of each large-family fixture: gate bits (mod q),
    and values mod 2^logQ with plaintext modulus P = 2^logQ / (q / (2 beta)) around P/2"""
    from fhe_amd import binfhe as bf
    st, arb, logQ, *topt = LARGE_SETS[name]
    topt = bool(topt and topt[0])
    ps = bf.large_paramset(st, arb, logQ, 0, topt)
    key_seed = 0xB1600000 + logQ + (st << 8) + (int(arb) << 7) + (int(topt) << 6)
    keys = bf.keygen(ps, GINX, key_seed)
    P = bf.params(ps, GINX)
    cnt = 2 if st == 3 else 4
    rng = np.random.default_rng(key_seed)
    bits1, bits2 = rng.integers(0, 2, cnt), rng.integers(0, 2, cnt)
    g1 = bf.encrypt(ps, GINX, keys.sk, bits1, key_seed + 1)
    g2 = bf.encrypt(ps, GINX, keys.sk, bits2, key_seed + 2)
    mod = 1 << logQ
    PL = mod // (P.q // 256) if mod > P.q else P.q // 256
    xs = np.array([PL // 2 - 1, PL // 2, 3, PL - 3, PL // 4, 0][:cnt + (2 if st != 3 else 0)])
    la, lb = bf.encrypt(ps, GINX, keys.sk, xs, key_seed + 3, PL, mod)
    return ps, key_seed, keys, P, bits1, bits2, g1, g2, mod, PL, xs, la, lb


def make_large(names=tuple(LARGE_SETS)):
    for name in names:
        ps, key_seed, keys, P, bits1, bits2, (a1, b1), (a2, b2), mod, PL, xs, la, lb = large_inputs(name)
        ref = Ref(ps, GINX)
        assert (ref.n, ref.N, ref.q, ref.Q, ref.qKS, ref.baseG) == (P.n, P.N, P.q, P.Q, P.qKS, P.baseG)
        ref.load_keys(keys.bsk, keys.kskA, keys.kskB)
        out = {"paramset": ps, "key_seed": np.uint64(key_seed), "bits1": bits1, "bits2": bits2, "xs": xs,
               "mod": np.uint64(mod), "PL": np.uint64(PL),
               "in_sha": np.array(sha(a1) + sha(b1) + sha(a2) + sha(b2) + sha(la) + sha(lb))}
        if name != "std29":
            out["keys_sha"] = np.array(sha(keys.bsk) + sha(keys.kskA) + sha(keys.kskB))
        for gname, g in (("AND", 1), ("XOR", 4)):
            ao, bo = ref.eval_gate(g, a1, b1, a2, b2)
            out[f"{gname}_a"], out[f"{gname}_b"] = ao, bo
            ea, eb = ref.eval_gate(g, a1, b1, a2, b2, extended=True)
            out[f"{gname}_ext_a"], out[f"{gname}_ext_b"] = ea, eb
        if mod > P.q:
            ao, bo = ref.eval_floor(la, lb, mod, 0)
            out["floor_a"], out["floor_b"] = ao, bo
            ao, bo = ref.eval_sign(la, lb, mod, False)
            out["sign_a"], out["sign_b"] = ao, bo
            if name != "std29":
                ao, bo = ref.eval_decomp(la, lb, mod)
                out["decomp_a"], out["decomp_b"] = ao, bo
        if P.q <= P.N:   # arbitrary-function LUT (eval-function.cpp): x^3 mod p on inputs mod q
            p = P.q // 256
            lut = np.array([(P.q // p) * (((i * p) // P.q) ** 3 % p) for i in range(P.q)], np.uint64)
            ms = np.arange(p)
            fa, fb = __import__("fhe_amd.binfhe", fromlist=["x"]).encrypt(ps, GINX, keys.sk, ms, key_seed + 4, p)
            ao, bo = ref.eval_func(fa, fb, P.q, lut)
            out["func_in_sha"] = np.array(sha(fa) + sha(fb))
            out["func_ms"], out["func_a"], out["func_b"] = ms, ao, bo
        np.savez_compressed(os.path.join(HERE, f"large_{name}.npz"), **out)
        print(name, "large ok", sorted(k for k in out if k.endswith("_a")))


# BASELINE configs 4 and 5 at their stated size: 65,536 AND gates through one context (the
# global batch of the 8-GPU run); hashes of the reference's outputs, whole and per 8192-gate shard
FULL_GATES = 65536
FULL_SHARD = 8192


def full_inputs(name, count=FULL_GATES):
    """keys (same seed as gates_<name>.npz) and `count` seeded AND-gate input pairs"""
    from fhe_amd import binfhe as bf
    ps, m = GATE_SETS[name]
    key_seed = 0xB0070000 + ps
    keys = bf.keygen(ps, m, key_seed)
    rng = np.random.default_rng(0xF011 + ps)
    bits1, bits2 = rng.integers(0, 2, count), rng.integers(0, 2, count)
    a1, b1 = bf.encrypt(ps, m, keys.sk, bits1, 0xF0110000 + ps)
    a2, b2 = bf.encrypt(ps, m, keys.sk, bits2, 0xF0120000 + ps)
    return ps, m, key_seed, keys, bits1, bits2, a1, b1, a2, b2


def _full_slice(args):
    """one process's share of a full batch, single-threaded (the reference's LMKCDEY EvalAcc crashes
    under its OpenMP gate loop with these keys; separate processes share nothing)"""
    name, lo, hi = args
    ps, m, key_seed, keys, bits1, bits2, a1, b1, a2, b2 = full_inputs(name)
    ref = Ref(ps, m)
    ref.load_keys(keys.bsk, keys.kskA, keys.kskB)
    return ref.eval_gate(GATES["AND"], a1[lo:hi], b1[lo:hi], a2[lo:hi], b2[lo:hi], nthreads=1)


def make_full(names=("std128", "lmkcdey"), nthreads=8):
    import time
    for name in names:
        ps, m, key_seed, keys, bits1, bits2, a1, b1, a2, b2 = full_inputs(name)
        t0 = time.time()
        if GATE_SETS[name][1] == LMKCDEY:
            import multiprocessing as mp
            step = FULL_GATES // nthreads
            with mp.get_context("spawn").Pool(nthreads) as pool:
                parts = pool.map(_full_slice, [(name, s, s + step) for s in range(0, FULL_GATES, step)])
            ao = np.concatenate([p[0] for p in parts])
            bo = np.concatenate([p[1] for p in parts])
            ref = Ref(ps, m)
        else:
            ref = Ref(ps, m)
            ref.load_keys(keys.bsk, keys.kskA, keys.kskB)
            ao, bo = ref.eval_gate(GATES["AND"], a1, b1, a2, b2, nthreads=nthreads)
        dt = time.time() - t0
        dec = np.array([ref.decrypt(keys.sk, ao[i], bo[i], ref.q) for i in range(0, FULL_GATES, 97)])
        assert np.array_equal(dec, (bits1 & bits2)[::97]), "reference AND outputs do not decrypt"
        shards = [sha(ao[s:s + FULL_SHARD]) + sha(bo[s:s + FULL_SHARD]) for s in range(0, FULL_GATES, FULL_SHARD)]
        np.savez_compressed(os.path.join(HERE, f"full_{name}.npz"), paramset=ps, method=m,
                            key_seed=np.uint64(key_seed), count=FULL_GATES, shard=FULL_SHARD, gate=GATES["AND"],
                            out_sha=np.array(sha(ao) + sha(bo)), shard_sha=np.array(shards),
                            out_a_head=ao[:16].astype(np.uint16), out_b_head=bo[:16].astype(np.uint16),
                            keys_sha=np.array(sha(keys.bsk) + sha(keys.kskA) + sha(keys.kskB)),
                            in_sha=np.array(sha(a1) + sha(b1) + sha(a2) + sha(b2)),
                            ref_seconds=dt, ref_threads=nthreads)
        print(name, "full ok", FULL_GATES, f"{dt:.0f} s on {nthreads} threads", flush=True)


# BASELINE config 3 (1024 STD128 GINX AND gates on one GPU): the first 1024 gates of full_inputs drawn
# at count = 1024 (bench.py's config-3 object uses the same seeds), one shard
C3_GATES = 1024


def make_config3(nthreads=8):
    ps, m, key_seed, keys, bits1, bits2, a1, b1, a2, b2 = full_inputs("std128", C3_GATES)
    ref = Ref(ps, m)
    ref.load_keys(keys.bsk, keys.kskA, keys.kskB)
    ao, bo = ref.eval_gate(GATES["AND"], a1, b1, a2, b2, nthreads=nthreads)
    dec = np.array([ref.decrypt(keys.sk, ao[i], bo[i], ref.q) for i in range(C3_GATES)])
    assert np.array_equal(dec, bits1 & bits2), "reference AND outputs do not decrypt"
    np.savez_compressed(os.path.join(HERE, "full_std128_b1024.npz"), paramset=ps, method=m,
                        key_seed=np.uint64(key_seed), count=C3_GATES, shard=C3_GATES, gate=GATES["AND"],
                        out_sha=np.array(sha(ao) + sha(bo)), shard_sha=np.array([sha(ao) + sha(bo)]),
                        out_a_head=ao[:16].astype(np.uint16), out_b_head=bo[:16].astype(np.uint16),
                        keys_sha=np.array(sha(keys.bsk) + sha(keys.kskA) + sha(keys.kskB)),
                        in_sha=np.array(sha(a1) + sha(b1) + sha(a2) + sha(b2)), ref_threads=nthreads)
    print("config3 ok", C3_GATES, flush=True)


# Ciphertexts mod Q as inputs (binfhe-base-scheme.cpp:92-93, 150-152, 200-201): the flows of the
# reference's UnitTestFHEWExtended.cpp:37-153 (extended = true outputs chained into the next gate, SMALL_DIM
# and LARGE_DIM encryptions mixed within one call) as batches, plus every 2-input gate, MAJORITY and CMUX on
# mixed inputs.  LARGE_DIM ciphertexts are encryptions under the keys' RLWE secret skN (dimension N, mod Q),
# what Encrypt(pk, m, LARGE_DIM, p) makes (binfhecontext.cpp:236-252).
MIXED_SETS = {"std128": (STD128, GINX), "lmkcdey": (STD128_LMKCDEY, LMKCDEY), "std192": (9, GINX),
              "std256q": (18, GINX)}
MIXED_COUNT = 8
OP_BOOTSTRAP = -1


def mixed_column(ps, m, sk, skN, bits, flags, seed, p):
    """one input column: rows of N words; flagged rows are LARGE_DIM encryptions (mod Q), the others
    SMALL_DIM ones (mod q, first n words)"""
    from fhe_amd import binfhe as bf
    P = bf.params(ps, m)
    sa, sb = bf.encrypt(ps, m, sk, bits, seed, p)
    la, lb = bf.encrypt_large(ps, m, skN, bits, seed + 0x1000, p)
    a = np.zeros((len(bits), P.N), np.uint64)
    a[:, :P.n] = sa
    a[flags == 1] = la[flags == 1]
    b = np.where(flags == 1, lb, sb).astype(np.uint64)
    return a, b


def mixed_cases(ps, m, key_seed, count=MIXED_COUNT):
    """keys, skN and the input-only cases: name -> (op, ptmod, bits [k][count], columns [(a, b, flags)])"""
    from fhe_amd import binfhe as bf
    keys = bf.keygen(ps, m, key_seed)
    skN = bf.keygen_ring_secret(ps, m, key_seed)
    rng = np.random.default_rng(key_seed ^ 0x3D)
    cases = {}

    def cols(name, op, k, p, pattern=None):
        bits = rng.integers(0, 2, size=(k, count))
        fl = rng.integers(0, 2, size=(k, count)).astype(np.uint8) if pattern is None else np.array(pattern, np.uint8)
        fl[:, 0] = 1   # every column has a ciphertext mod Q and (below) one mod q
        fl[:, 1] = 0
        base = key_seed + 0x500 + 16 * len(cases)
        c = [mixed_column(ps, m, keys.sk, skN, bits[j], fl[j], base + j, p) + (fl[j],) for j in range(k)]
        cases[name] = (op, p, bits, c)

    for gname, g in GATES.items():
        cols(f"gate_{gname}", g, 2, 4)
    cols("majority", 6, 3, 4)
    cols("cmux", 13, 3, 4)
    cols("boot", OP_BOOTSTRAP, 1, 4)
    cols("boot_p8", OP_BOOTSTRAP, 1, 8)
    # UnitTestFHEWExtended flows: EvalBinGate2 (p = 4: small, large), EvalBinGate3 (p = 6: small, large, small),
    # EvalBinGate4 (p = 8: small, large, small, large); the BootStrap test is "boot" with its large rows
    cols("flow2", None, 2, 4, [[0] * count, [1] * count])
    cols("flow3", None, 3, 6, [[0] * count, [1] * count, [0] * count])
    cols("flow4", None, 4, 8, [[0] * count, [1] * count, [0] * count, [1] * count])
    return keys, skN, cases


FLOW_GATES = {"flow2": (0, 1), "flow3": (8, 7), "flow4": (10, 9)}   # (OR, AND), (OR3, AND3), (OR4, AND4)


def make_mixed(names=("std128", "lmkcdey")):
    for name in names:
        ps, m = MIXED_SETS[name]
        key_seed = 0xB00E0000 + ps + (m << 8)
        keys, skN, cases = mixed_cases(ps, m, key_seed)
        ref = Ref(ps, m)
        ref.load_keys(keys.bsk, keys.kskA, keys.kskB)
        out = {"paramset": ps, "method": m, "key_seed": np.uint64(key_seed),
               "keys_sha": np.array(sha(keys.bsk) + sha(keys.kskA) + sha(keys.kskB)), "skN_sha": np.array(sha(skN))}
        for cname, (op, p, bits, c) in cases.items():
            A = [x[0] for x in c]
            B = [x[1] for x in c]
            F = [x[2] for x in c]
            out[f"{cname}_in_sha"] = np.array("".join(sha(x) for x in A + B))
            out[f"{cname}_bits"] = bits
            out[f"{cname}_flags"] = np.array(F)
            if cname in FLOW_GATES:
                # UnitTestFHEWExtended.cpp:53-59: ct11 = G1(v, extended), ct12 = G2(v, extended) with the
                # 2-input form taking (small, large) then (large, small), then NAND(ct11, ct12, false)
                g1, g2 = FLOW_GATES[cname]
                if cname == "flow2":
                    e1 = ref.eval_mixed(g1, A, B, F, p, extended=True)
                    e2 = ref.eval_mixed(g2, A[::-1], B[::-1], F[::-1], p, extended=True)
                else:
                    e1 = ref.eval_mixed(g1, A, B, F, p, extended=True)
                    e2 = ref.eval_mixed(g2, A, B, F, p, extended=True)
                ones = np.ones(len(B[0]), np.uint8)
                fo = ref.eval_mixed(3, [e1[0], e2[0]], [e1[1], e2[1]], [ones, ones], 4)
                out[f"{cname}_ext1_sha"] = np.array(sha(e1[0]) + sha(e1[1]))
                out[f"{cname}_ext2_sha"] = np.array(sha(e2[0]) + sha(e2[1]))
                out[f"{cname}_out_a"], out[f"{cname}_out_b"] = fo
                out[f"{cname}_dec"] = np.array([ref.decrypt(keys.sk, fo[0][i], fo[1][i], ref.q) for i in range(len(fo[1]))])
                print(name, cname, "NAND of the chained outputs decrypts:", list(out[f"{cname}_dec"]), flush=True)
                continue
            ao, bo = ref.eval_mixed(op, A, B, F, p)
            out[f"{cname}_out_a"], out[f"{cname}_out_b"] = ao, bo
            out[f"{cname}_dec"] = np.array([ref.decrypt(keys.sk, ao[i], bo[i], ref.q, p if op == OP_BOOTSTRAP else 4)
                                            for i in range(len(bo))])
            if op != 13:   # CMUX ignores extended
                ea, eb = ref.eval_mixed(op, A, B, F, p, extended=True)
                out[f"{cname}_ext_sha"] = np.array(sha(ea) + sha(eb))
                out[f"{cname}_ext_a0"] = ea[0]
            print(name, cname, "decrypts:", list(out[f"{cname}_dec"]), flush=True)
        np.savez_compressed(os.path.join(HERE, f"mixed_{name}.npz"), **out)
        print(name, "mixed ok", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "config3":
        make_config3()
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what == "full":   # ~15 min per set on 8 cores
        make_full(sys.argv[2:] or ("std128", "lmkcdey"))
    if what in ("ntt", "all"):
        make_ntt()
    if what in ("ntt", "ntt4096", "all"):
        make_ntt4096()
    if what in ("contexts", "all"):
        make_contexts()
    if what in ("gates", "all"):
        make_gates(sys.argv[2:] or ("std128",))
    if what == "wider":   # one process per call keeps the reference's memory bounded
        make_gates(sys.argv[2:] or tuple(WIDER_SETS))
    if what in ("multi", "all"):
        make_multi(sys.argv[2:] or ("std128", "lmkcdey"))
    if what == "fb":   # one parameter set per process (see tests/test_fb.py)
        make_fb(sys.argv[2:] or ("std128",))
    if what == "large":
        make_large(sys.argv[2:] or tuple(LARGE_SETS))
    if what == "mixed":
        make_mixed(sys.argv[2:] or tuple(MIXED_SETS))
    sys.stdout.flush()
    os._exit(0)   # skip interpreter teardown: two OpenMP runtimes (reference + fhe_amd) in one process
