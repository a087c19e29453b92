"""The reference's packed GPU-transfer format (src/binfhe/include/backend/packed.h,
src/binfhe/lib/backend/packed.cpp): LWE batches byte-compatible with the reference's own
PackLWEBatch / UnpackLWEBatch (sequential and interleaved), packed keys (whose reference packers are
TODO stubs) defined on the same header, and gates evaluated straight from packed batches."""
import os
import struct

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sample(count=7, n=503, seed=3):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 1024, (count, n), dtype=np.uint64), rng.integers(0, 1024, count, dtype=np.uint64)


@pytest.mark.parametrize("flags", [0, 1])
def test_pack_matches_reference_bytes(flags):
    from oracle_lib import ref_available, ref_pack_lwe_batch, ref_unpack_lwe_batch
    from fhe_amd import binfhe as bf
    if not ref_available():
        pytest.skip("reference oracle not built")
    a, b = sample()
    ours = bf.pack_lwe_batch(a, b, flags)
    theirs = ref_pack_lwe_batch(a, b, flags)
    assert ours == theirs                                     # byte for byte
    ua, ub = bf.unpack_lwe_batch(theirs)                      # we read theirs
    assert np.array_equal(ua, a) and np.array_equal(ub, b)
    ra, rb = ref_unpack_lwe_batch(ours, a.shape[1], len(b))   # they read ours
    assert np.array_equal(ra, a) and np.array_equal(rb, b)


def test_packed_header_layout_and_validation():
    from fhe_amd import binfhe as bf
    from fhe_amd._lib import FheHipError
    a, b = sample(count=3, n=5)
    buf = bf.pack_lwe_batch(a, b, 1)
    magic, ver, typ, total, count, flags = struct.unpack_from("<IHHQQI", buf, 0)
    assert (magic, ver, typ, total, count, flags) == (0x4C555846, 1, 2, len(buf), 3, 1)
    n, log_q, q, cnt, stride = struct.unpack_from("<IIQQI", buf, 32)
    assert (n, cnt, stride) == (5, 3, 48) and len(buf) == 64 + 3 * 6 * 8
    for bad in (b"XXXX" + buf[4:], buf[:len(buf) - 8], buf[:4] + struct.pack("<H", 9) + buf[6:]):
        with pytest.raises(FheHipError):
            bf.unpack_lwe_batch(bad)


def test_packed_keys_layout():
    from fhe_amd import binfhe as bf
    keys = bf.keygen(bf.STD128, bf.GINX, 99)
    pb, pk = bf.pack_keys(bf.STD128, bf.GINX, keys)
    magic, ver, typ, total, count, flags = struct.unpack_from("<IHHQQI", pb.tobytes(), 0)
    assert (magic, typ, total, flags) == (0x4C555846, 5, pb.size, bf.GINX)
    lwe_n, log_q, N, limbs, levels, base_log, key_size, layout = struct.unpack_from("<IIIIIIQI", pb.tobytes(), 32)
    assert (lwe_n, log_q, N, limbs, levels, base_log, key_size, layout) == (503, 10, 1024, 1, 4, 9, keys.bsk.size * 8, 2)
    assert np.array_equal(np.frombuffer(pb.tobytes()[72:], np.uint64), keys.bsk)
    typ = struct.unpack_from("<H", pk.tobytes(), 6)[0]
    in_n, out_n, levels, base_log, Q = struct.unpack_from("<IIIIQ", pk.tobytes(), 32)
    assert (typ, in_n, out_n, levels, base_log, Q) == (6, 1024, 503, 3, 5, 16384)
    body = np.frombuffer(pk.tobytes()[64:], np.uint64)
    assert np.array_equal(body[:keys.kskA.size], keys.kskA) and np.array_equal(body[keys.kskA.size:], keys.kskB)


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, 1])
def test_gpu_gates_from_reference_packed_batches(flags):
    """reference-packed inputs -> EvalBinGate on the GPU -> packed output the reference unpacks
    == the reference's own EvalBinGate outputs (golden); keys loaded from the packed key format."""
    import sys
    sys.path.insert(0, GOLD)
    from make_golden import gate_inputs
    from oracle_lib import ref_available, ref_pack_lwe_batch, ref_unpack_lwe_batch
    from fhe_amd import binfhe as bf
    g = np.load(os.path.join(GOLD, "gates_std128.npz"))
    ps, m = int(g["paramset"]), int(g["method"])
    keys, bits1, bits2, a1, b1, a2, b2 = gate_inputs(ps, m, int(g["key_seed"]))
    e = bf.GateEngine(ps, m)
    e.load_keys_packed(*bf.pack_keys(ps, m, keys))
    pg = g["bits1"].shape[1]
    pack = ref_pack_lwe_batch if ref_available() else bf.pack_lwe_batch
    for i, gate in enumerate(g["gates"]):
        sl = slice(i * pg, (i + 1) * pg)
        out = e.eval_gate_packed(int(gate), pack(a1[sl], b1[sl], flags), pack(a2[sl], b2[sl], flags), flags)
        oa, ob = ref_unpack_lwe_batch(out, 503, pg) if ref_available() else bf.unpack_lwe_batch(out)
        assert np.array_equal(oa, g["out_a"][sl]) and np.array_equal(ob, g["out_b"][sl]), int(gate)


@pytest.mark.parametrize("ps,m", [(0, 2), (19, 2), (43, 2), (3, 2), (21, 3)])
def test_packed_keys_roundtrip(ps, m):
    """pack / unpack of the keys for sets with a non-power-of-two baseKS (TOY 25, STD256Q_3 21,
    SIGNED_MOD_TEST 25) and the STD128 sets; a short output buffer is refused"""
    from fhe_amd import binfhe as bf
    from fhe_amd._lib import FheHipError
    keys = bf.keygen(ps, m, 0x9AC0 + ps)
    pb, pk = bf.pack_keys(ps, m, keys)
    back = bf.unpack_keys(ps, m, pb, pk)
    assert np.array_equal(back.bsk, keys.bsk)
    assert np.array_equal(back.kskA, keys.kskA) and np.array_equal(back.kskB, keys.kskB)
    import ctypes
    short = np.zeros(len(keys.kskB) - 1, np.uint64)
    A = np.zeros_like(keys.kskA)
    with pytest.raises(FheHipError):
        bf.check(bf.L().fhe_hip_unpack_keys(ps, m, None, 0, None, 0, pk.ctypes.data_as(ctypes.c_void_p), pk.size,
                                            A.ctypes.data_as(ctypes.c_void_p), A.size,
                                            short.ctypes.data_as(ctypes.c_void_p), short.size))
