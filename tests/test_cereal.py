"""The reference's serialized objects (cereal, binfhecontext-ser.h:42-52;
Serial::Serialize(..., SerType::BINARY), utils/serial.h:95-125): our reader / writer against the
reference's own serializer, compiled from its sources into oracle/_ref.  Keys written by the reference
(both keys it generated itself and keys it loaded) are read bit-exactly; our writer's bytes are
identical to the reference's; the reference deserializes our bytes; gates run on keys loaded from
reference files reproduce the reference's outputs (golden)."""
import hashlib
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.uint64).tobytes()).hexdigest()


def need_ref():
    from oracle_lib import ref_available
    if not ref_available():
        pytest.skip("reference oracle not built")


@pytest.mark.parametrize("is_key,mod", [(False, 1024), (False, 2048), (False, 1 << 14), (True, 1 << 14)])
def test_lwe_objects_match_reference_bytes(is_key, mod):
    need_ref()
    from oracle_lib import ref_deserialize_ct, ref_serialize_lwe
    from fhe_amd import binfhe as bf
    rng = np.random.default_rng(mod + is_key)
    for n in (503, 447, 1, 0):
        a = rng.integers(0, mod, n, dtype=np.uint64)
        b = None if is_key else int(rng.integers(0, mod))
        ours = bf.cereal_write_lwe(a, b, mod, is_key)
        theirs = ref_serialize_lwe(a, b, mod, is_key)
        assert ours == theirs
        ra, rb, rmod = bf.cereal_read_lwe(theirs, is_key)
        assert np.array_equal(ra, a) and rb == b and rmod == mod
        if not is_key:
            assert ref_deserialize_ct(ours)[1:] == (b, mod)
            assert np.array_equal(ref_deserialize_ct(ours)[0], a)


def test_lwe_stream_errors():
    from fhe_amd import binfhe as bf
    from fhe_amd._lib import FheHipError
    good = bf.cereal_write_lwe(np.arange(5, dtype=np.uint64), 3, 1024)
    for bad in (good[:-1], good + b"\0", b"\x00" + good[1:], good[:1] + b"\0\0\0\0" + good[5:]):
        with pytest.raises(FheHipError):
            bf.cereal_read_lwe(bad)


@pytest.mark.slow
@pytest.mark.parametrize("name", ["std128", "lmkcdey"])
def test_keys_byte_identical_and_read_back(name):
    """reference-serialized keys (loaded from our raw keys) == our writer's bytes; our reader
    recovers the raw keys; a wrong parameter set is refused"""
    need_ref()
    import sys
    sys.path.insert(0, GOLD)
    from make_golden import gate_inputs
    from oracle_lib import Ref, ref_serialize_key
    from fhe_amd import binfhe as bf
    from fhe_amd._lib import FheHipError
    g = np.load(os.path.join(GOLD, f"gates_{name}.npz"))
    ps, m = int(g["paramset"]), int(g["method"])
    keys = gate_inputs(ps, m, int(g["key_seed"]))[0]
    ref = Ref(ps, m)
    ref.load_keys(keys.bsk, keys.kskA, keys.kskB)
    r_ref, s_ref = ref_serialize_key(ref, 0), ref_serialize_key(ref, 1)
    r_ours, s_ours = bf.cereal_write_keys(ps, m, keys)
    assert r_ours == r_ref and s_ours == s_ref
    ks = bf.cereal_read_keys(ps, m, r_ref, s_ref)
    assert sha(ks.bsk) + sha(ks.kskA) + sha(ks.kskB) == str(g["keys_sha"])
    other = (bf.STD128_LMKCDEY, bf.LMKCDEY) if name == "std128" else (bf.STD128, bf.GINX)
    with pytest.raises(FheHipError):
        bf.cereal_read_keys(*other, r_ref, s_ref)
    with pytest.raises(FheHipError):
        bf.cereal_read_keys(ps, m, r_ref[:-8], s_ref)


@pytest.mark.slow
@pytest.mark.parametrize("ps_m", ["std128", "lmkcdey"])
def test_reference_generated_keys_read_and_our_bytes_deserialize(ps_m):
    """keys the reference generated itself (BLAKE2 keygen) and serialized are read bit-exactly;
    the reference deserializes our re-serialization of them and evaluates gates correctly"""
    need_ref()
    from oracle_lib import Ref, ref_deserialize_keys, ref_serialize_key
    from fhe_amd import binfhe as bf
    ps, m = (bf.STD128, bf.GINX) if ps_m == "std128" else (bf.STD128_LMKCDEY, bf.LMKCDEY)
    ref = Ref(ps, m)
    sk, bsk, A, B = ref.keygen()
    r_ref, s_ref = ref_serialize_key(ref, 0), ref_serialize_key(ref, 1)
    ks = bf.cereal_read_keys(ps, m, r_ref, s_ref)
    assert np.array_equal(ks.bsk, bsk) and np.array_equal(ks.kskA, A) and np.array_equal(ks.kskB, B)
    r_ours, s_ours = bf.cereal_write_keys(ps, m, ks)
    ref2 = Ref(ps, m)
    ref_deserialize_keys(ref2, r_ours, s_ours)
    bits = np.array([0, 1, 0, 1]), np.array([0, 0, 1, 1])
    a1, b1 = bf.encrypt(ps, m, sk, bits[0], 5)
    a2, b2 = bf.encrypt(ps, m, sk, bits[1], 6)
    ao, bo = ref2.eval_gate(1, a1, b1, a2, b2)
    assert np.array_equal(bf.decrypt(ps, m, sk, ao, bo), bits[0] & bits[1])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["std128", "lmkcdey"])
def test_gpu_gates_on_keys_loaded_from_reference_files(name):
    import sys
    sys.path.insert(0, GOLD)
    from make_golden import gate_inputs
    from oracle_lib import Ref, ref_available, ref_serialize_key
    from fhe_amd import binfhe as bf
    g = np.load(os.path.join(GOLD, f"gates_{name}.npz"))
    ps, m = int(g["paramset"]), int(g["method"])
    keys, bits1, bits2, a1, b1, a2, b2 = gate_inputs(ps, m, int(g["key_seed"]))
    if ref_available():
        ref = Ref(ps, m)
        ref.load_keys(keys.bsk, keys.kskA, keys.kskB)
        files = ref_serialize_key(ref, 0), ref_serialize_key(ref, 1)
        del ref
    else:                                   # writer pinned byte-for-byte by the CPU tests
        files = bf.cereal_write_keys(ps, m, keys)
    e = bf.GateEngine(ps, m)
    e.load_keys_cereal(*files)
    pg = g["bits1"].shape[1]
    for i, gate in enumerate(g["gates"]):
        sl = slice(i * pg, (i + 1) * pg)
        ao, bo = e.eval_gate(int(gate), a1[sl], b1[sl], a2[sl], b2[sl])
        assert np.array_equal(ao, g["out_a"][sl]) and np.array_equal(bo, g["out_b"][sl]), int(gate)


@pytest.mark.gpu
def test_gpu_boolean_serial_binary_flow(tmp_path):
    """boolean-serial-binary.cpp: the reference generates keys, a secret key and a ciphertext and
    serializes them; our BinFHEContext deserializes everything and evaluates AND on the GPU."""
    need_ref()
    from oracle_lib import Ref, ref_serialize_key, ref_serialize_lwe
    from fhe_amd import binfhe as bf
    ref = Ref(bf.STD128, bf.GINX)
    sk, *_ = ref.keygen()
    ct_a, ct_b = ref.encrypt([1])
    files = {"refreshKey": ref_serialize_key(ref, 0), "ksKey": ref_serialize_key(ref, 1),
             "sk1": ref_serialize_lwe(sk, None, ref.qKS, is_key=True),
             "ct1": ref_serialize_lwe(ct_a[0], int(ct_b[0]), ref.q)}
    del ref
    for k, v in files.items():
        (tmp_path / f"{k}.txt").write_bytes(v)
    cc = bf.BinFHEContext()
    cc.GenerateBinFHEContext(bf.STD128, bf.GINX)
    S = bf.Serial
    refresh = S.DeserializeFromFile(tmp_path / "refreshKey.txt", bf.SerializedKey)
    ks = S.DeserializeFromFile(tmp_path / "ksKey.txt", bf.SerializedKey)
    cc.BTKeyLoad(refresh, ks)
    key = S.DeserializeFromFile(tmp_path / "sk1.txt", bf.LWEPrivateKey)
    ct = S.DeserializeFromFile(tmp_path / "ct1.txt", bf.LWECiphertext)
    res = cc.EvalBinGate(bf.AND, ct, cc.Encrypt(key, 1))
    assert cc.Decrypt(key, res) == 1
    assert cc.Decrypt(key, cc.EvalBinGate(bf.AND, ct, cc.Encrypt(key, 0))) == 0
    S.SerializeToFile(tmp_path / "out.txt", res)        # the reference reads what we write (CPU tests)
    back = S.DeserializeFromFile(tmp_path / "out.txt", bf.LWECiphertext)
    assert np.array_equal(back.a, res.a) and back.b == res.b


# ---- the cryptoContext archive (BinFHEContext -> BinFHECryptoParams -> LWE / RingGSW parameters) ------
CONTEXTS = {"std128": (3, 2), "lmkcdey": (21, 3), "ap": (2, 1), "std128_3": (4, 2), "std192": (9, 2),
            "std128_4_lmkcdey": (23, 3), "toy_lmkcdey": (0, 3)}


def same_row(x, y):
    """two rows with the same parameters (STD128 and STD128_AP, for one, differ only in name)"""
    import dataclasses
    return dataclasses.replace(x, paramset=0) == dataclasses.replace(y, paramset=0)


def context_fixture(name):
    with open(os.path.join(GOLD, f"context_{name}.bin"), "rb") as f:
        return f.read()


@pytest.mark.parametrize("name", list(CONTEXTS))
def test_context_fixture_read_and_rewritten_byte_identically(name):
    """the reference's own archive (tests/golden/make_golden.py contexts) names its row; our writer
    reproduces its bytes"""
    from fhe_amd import binfhe as bf
    data = context_fixture(name)
    ps, m = CONTEXTS[name]
    rps, rm = bf.cereal_read_context(data)
    assert rm == m and same_row(bf.params(rps, rm), bf.params(ps, m))
    assert bf.cereal_write_context(rps, rm) == data
    assert bf.cereal_write_context(ps, m) == data


def test_context_archive_errors():
    from fhe_amd import binfhe as bf
    from fhe_amd._lib import FheHipError
    good = context_fixture("std128")
    bad_q = bytearray(good)
    bad_q[29] ^= 0x40      # Q of the LWE parameters: inconsistent with the ring's
    for bad in (good[:-1], good + b"\0", b"\x00" + good[1:], bytes(bad_q)):
        with pytest.raises(FheHipError):
            bf.cereal_read_context(bad)
    with pytest.raises(FheHipError):
        bf.cereal_write_context(3, 3)    # STD128 x LMKCDEY: isMethodCompatible refuses it


@pytest.mark.slow
def test_context_archive_every_row_vs_reference():
    """every compatible (set, method) row: our bytes == Serial::Serialize(cc, BINARY) of the reference's
    context; our reader maps the reference's archive to a row with the same parameters; the reference
    deserializes our bytes into a context that serializes back to them"""
    need_ref()
    import ctypes
    from oracle_lib import REF_SO, Ref
    from fhe_amd import binfhe as bf
    from fhe_amd._lib import FheHipError
    L = ctypes.CDLL(REF_SO)
    vp = ctypes.c_void_p
    L.ref_serialize_context.argtypes = [vp, vp, ctypes.c_size_t, vp]
    L.ref_ctx_from_archive.restype = vp
    L.ref_ctx_from_archive.argtypes = [vp, ctypes.c_size_t]
    L.ref_ctx_destroy.argtypes = [vp]

    def ser(h):
        out, size = ctypes.create_string_buffer(1 << 16), ctypes.c_size_t()
        assert L.ref_serialize_context(h, out, 1 << 16, ctypes.byref(size)) == 0
        return out.raw[:size.value]

    rows = 0
    for ps in range(44):
        for m in (1, 2, 3):
            try:
                ours = bf.cereal_write_context(ps, m)
            except FheHipError:
                continue     # incompatible (set, method): the reference refuses it too
            ref = Ref(ps, m)      # held: its context is destroyed with the object
            theirs = ser(ref.h)
            assert ours == theirs, (ps, m)
            rps, rm = bf.cereal_read_context(theirs)
            assert rm == m and same_row(bf.params(rps, rm), bf.params(ps, m)), (ps, m, rps)
            h = L.ref_ctx_from_archive(ours, len(ours))
            assert h, (ps, m)
            assert ser(vp(h)) == ours
            L.ref_ctx_destroy(vp(h))
            rows += 1
    assert rows == 70    # 24 rows x {AP, GINX} + 22 rows x LMKCDEY


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["std128", "lmkcdey"])
def test_gpu_context_from_reference_archive_evaluates_gate_goldens(name):
    """boolean-serial-binary.cpp:108: a GPU context built from the reference's cryptoContext archive alone
    (no parameter set given), keys loaded, reproduces the reference's gate outputs (tests/golden/gates_*)"""
    import sys
    sys.path.insert(0, GOLD)
    from make_golden import gate_inputs
    from fhe_amd import binfhe as bf
    g = np.load(os.path.join(GOLD, f"gates_{name}.npz"))
    keys, _, _, a1, b1, a2, b2 = gate_inputs(int(g["paramset"]), int(g["method"]), int(g["key_seed"]))
    e = bf.GateEngine.from_cereal(context_fixture(name))
    assert (e.params.n, e.params.Q) == (bf.params(int(g["paramset"]), int(g["method"])).n,
                                        bf.params(int(g["paramset"]), int(g["method"])).Q)
    e.load_keys(keys.bsk, keys.kskA, keys.kskB)
    pg = g["bits1"].shape[1]
    for i, gate in enumerate(g["gates"]):
        sl = slice(i * pg, (i + 1) * pg)
        ao, bo = e.eval_gate(int(gate), a1[sl], b1[sl], a2[sl], b2[sl])
        assert np.array_equal(ao, g["out_a"][sl]) and np.array_equal(bo, g["out_b"][sl]), int(gate)
    e.close()
