"""Host-side mirror of the reference's binfhe API over the HIP C-ABI.

Names and argument meaning follow lux::fhe::BinFHEContext
(src/binfhe/include/binfhecontext.h) and the batch API
(src/binfhe/include/batch/binfhe-batch.h) so tests read like the reference's:

    cc = BinFHEContext()
    cc.GenerateBinFHEContext(STD128, GINX)
    sk = cc.KeyGen(); cc.BTKeyGen(sk)
    ct1, ct2 = cc.Encrypt(sk, 1), cc.Encrypt(sk, 0)
    r = cc.EvalBinGate(AND, ct1, ct2)          # runs on the MI355X
    cc.Decrypt(sk, r)

Every evaluation goes through libfhe_amd.so on the GPU; there is no CPU
fallback.  Key generation / encryption / decryption are host C++ (seeded).
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from ._lib import FheHipError, check, lib, ptr, sz, u64, vp

# reference enum values (src/binfhe/include/binfhe-constants.h:49-126)
TOY, STD128_AP, STD128, STD128_LMKCDEY = 0, 2, 3, 21
# every BINFHE_PARAMSET name in enum order (binfhe-constants.h:49-95)
PARAMSETS = ("TOY MEDIUM STD128_AP STD128 STD128_3 STD128_4 STD128Q STD128Q_3 STD128Q_4 STD192 STD192_3 STD192_4 "
             "STD192Q STD192Q_3 STD192Q_4 STD256 STD256_3 STD256_4 STD256Q STD256Q_3 STD256Q_4 STD128_LMKCDEY "
             "STD128_3_LMKCDEY STD128_4_LMKCDEY STD128Q_LMKCDEY STD128Q_3_LMKCDEY STD128Q_4_LMKCDEY STD192_LMKCDEY "
             "STD192_3_LMKCDEY STD192_4_LMKCDEY STD192Q_LMKCDEY STD192Q_3_LMKCDEY STD192Q_4_LMKCDEY STD256_LMKCDEY "
             "STD256_3_LMKCDEY STD256_4_LMKCDEY STD256Q_LMKCDEY STD256Q_3_LMKCDEY STD256Q_4_LMKCDEY LPF_STD128 "
             "LPF_STD128Q LPF_STD128_LMKCDEY LPF_STD128Q_LMKCDEY SIGNED_MOD_TEST").split()


def method_compatible(paramset, method):
    """GenerateBinFHEContext(set, method) accepts the pair (binfhecontext.cpp:113-159: the *_LMKCDEY rows, TOY
    and MEDIUM take LMKCDEY; the CGGI rows, TOY .. STD256Q_4, LPF_STD128/Q and SIGNED_MOD_TEST take GINX and AP)"""
    lmk = paramset in (0, 1, 41, 42) or 21 <= paramset <= 38
    cggi = paramset <= 20 or paramset in (39, 40, 43)
    return lmk if method == 3 else cggi if method in (1, 2) else False
LARGE = 1 << 30
TIMEOPT = 1 << 14


def large_paramset(paramset, arbFunc, logQ, N=0, timeOptimization=False):
    """paramset code of GenerateBinFHEContext(paramset, arbFunc, logQ, N, GINX, timeOptimization)
    (binfhecontext.cpp:55-104), the large-precision family (54-bit Q, N = 2048, qKS = 2^35).  With
    timeOptimization (logQ != 11) the bootstrapping key is the map of BTKeyGen (:285-307): one key per
    baseG 2^14, 2^18, 2^27, concatenated in that order (Params.bsk_words covers all three)"""
    logN = 0 if not N else N.bit_length() - 1
    if N and N != 1 << logN:
        raise ValueError("N must be a power of two")
    return (LARGE | (paramset << 16) | (int(bool(arbFunc)) << 15) | (TIMEOPT if timeOptimization else 0) |
            (logN << 8) | int(logQ))
AP, GINX, LMKCDEY = 1, 2, 3
OR, AND, NOR, NAND, XOR, XNOR, MAJORITY, AND3, OR3, AND4, OR4, XOR_FAST, XNOR_FAST, CMUX = range(14)
GATE_NAMES = {"OR": OR, "AND": AND, "NOR": NOR, "NAND": NAND, "XOR": XOR, "XNOR": XNOR, "MAJORITY": MAJORITY,
              "AND3": AND3, "OR3": OR3, "AND4": AND4, "OR4": OR4, "CMUX": CMUX}
MULTI_GATES = (MAJORITY, AND3, OR3, AND4, OR4)
OP_BOOTSTRAP = -1      # fhe_hip_eval_mixed_batch: BinFHEScheme::Bootstrap
LARGE_DIM, SMALL_DIM = 3, 4   # BINFHE_OUTPUT (binfhe-constants.h:103-109): Encrypt's output dimension


class _Params(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint32) for f in ("paramset", "method", "n", "N", "q", "baseKS", "digitsKS",
                                               "baseG", "digitsG", "numAutoKeys", "keyDist", "kernel")] + \
               [(f, ctypes.c_uint64) for f in ("Q", "psi", "qKS", "bsk_words", "ksk_rows")]


def _setup(L):
    if getattr(L, "_binfhe_ready", False):
        return L
    P = ctypes.POINTER(_Params)
    L.fhe_hip_params_get.argtypes = [ctypes.c_int, ctypes.c_int, P]
    L.fhe_hip_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
    L.fhe_hip_destroy.argtypes = [vp]
    L.fhe_hip_destroy.restype = None
    L.fhe_hip_get_params.argtypes = [vp, P]
    L.fhe_hip_stream.argtypes = [vp]
    L.fhe_hip_stream.restype = vp
    L.fhe_hip_load_bsk.argtypes = [vp, vp, sz]
    L.fhe_hip_load_ksk.argtypes = [vp, vp, sz, vp, sz]
    L.fhe_hip_eval_bingate_batch.argtypes = [vp, ctypes.c_int, sz, vp, vp, vp, vp, vp, vp]
    L.fhe_hip_eval_bingate_batch_device.argtypes = [vp, ctypes.c_int, sz, vp, vp, vp, vp, vp, vp, vp]
    L.fhe_hip_blind_rotate_batch_device.argtypes = [vp, ctypes.c_int, sz, vp, vp, vp, vp, vp]
    L.fhe_hip_keyswitch_workspace_device.argtypes = [vp, sz, vp, vp, vp]
    L.fhe_hip_eval_bingate_extended.argtypes = [vp, ctypes.c_int, sz, vp, vp, vp, vp, vp, vp]
    L.fhe_hip_keyswitch_batch.argtypes = [vp, sz, vp, vp, vp, vp]
    L.fhe_hip_modswitch_batch.argtypes = [vp, u64, u64, ctypes.c_uint32, sz, vp, vp, vp, vp]
    L.fhe_hip_keygen.argtypes = [ctypes.c_int, ctypes.c_int, u64, vp, vp, vp, vp]
    L.fhe_hip_encrypt.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, sz, u64, vp, vp]
    L.fhe_hip_decrypt.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, vp, sz, ctypes.c_uint32, u64, vp]
    L.fhe_hip_eval_gate_multi_batch.argtypes = [vp, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, sz, vp, vp, vp,
                                                vp, ctypes.c_int]
    L.fhe_hip_eval_gate_multi_batch_device.argtypes = [vp, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, sz, vp,
                                                       vp, vp, vp, vp]
    L.fhe_hip_eval_cmux_batch.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp, vp, vp]
    L.fhe_hip_eval_cmux_batch_device.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.fhe_hip_encrypt_ptmod.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, sz, u64, ctypes.c_uint32, vp, vp]
    L.fhe_hip_encrypt_mod.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, sz, u64, ctypes.c_uint32, u64, vp, vp]
    L.fhe_hip_decrypt_ptmod.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, vp, sz, ctypes.c_uint32, u64,
                                        ctypes.c_uint32, vp]
    L.fhe_hip_eval_func_batch.argtypes = [vp, sz, vp, vp, u64, vp, sz, vp, vp]
    L.fhe_hip_eval_func_batch_device.argtypes = [vp, sz, vp, vp, u64, vp, sz, vp, vp, vp]
    L.fhe_hip_eval_floor_batch.argtypes = [vp, sz, vp, vp, u64, ctypes.c_uint32, vp, vp]
    L.fhe_hip_eval_sign_batch.argtypes = [vp, sz, vp, vp, u64, ctypes.c_int, vp, vp]
    L.fhe_hip_eval_decomp_parts.argtypes = [vp, u64, vp]
    L.fhe_hip_eval_decomp_batch.argtypes = [vp, sz, vp, vp, u64, vp, vp]
    L.fhe_hip_bootstrap_func_batch.argtypes = [vp, sz, vp, vp, ctypes.c_uint32, vp, u64, vp, vp]
    L.fhe_hip_btkeygen_device.argtypes = [vp, vp, sz, u64, vp, vp, vp]
    L.fhe_hip_keygen_secret.argtypes = [ctypes.c_int, ctypes.c_int, u64, vp]
    L.fhe_hip_load_keys_cereal.argtypes = [vp, vp, sz, vp, sz]
    L.fhe_hip_cereal_read_keys.argtypes = [ctypes.c_int, ctypes.c_int, vp, sz, vp, sz, vp, vp, vp]
    L.fhe_hip_cereal_write_keys.argtypes = [ctypes.c_int, ctypes.c_int, vp, sz, vp, vp, vp, sz, vp, vp, sz, vp]
    L.fhe_hip_cereal_read_lwe.argtypes = [vp, sz, ctypes.c_int, vp, ctypes.c_uint32, vp, vp, vp]
    L.fhe_hip_cereal_write_lwe.argtypes = [vp, ctypes.c_uint32, u64, u64, ctypes.c_int, vp, sz, vp]
    L.fhe_hip_cereal_read_context.argtypes = [vp, sz, vp, vp, vp]
    L.fhe_hip_cereal_write_context.argtypes = [ctypes.c_int, ctypes.c_int, vp, sz, vp]
    L.fhe_hip_create_from_cereal.argtypes = [vp, sz, ctypes.c_int, vp]
    L.fhe_hip_bootstrap_batch.argtypes = [vp, sz, vp, vp, vp, vp]
    L.fhe_hip_pack_lwe_batch.argtypes = [ctypes.c_uint32, sz, vp, vp, ctypes.c_uint32, vp, sz, vp]
    L.fhe_hip_unpack_lwe_batch.argtypes = [vp, sz, vp, vp, vp, vp]
    L.fhe_hip_eval_bingate_packed.argtypes = [vp, ctypes.c_int, vp, sz, vp, sz, ctypes.c_uint32, vp, sz, vp]
    L.fhe_hip_pack_keys.argtypes = [ctypes.c_int, ctypes.c_int, vp, sz, vp, vp, vp, sz, vp, vp, sz, vp]
    L.fhe_hip_load_keys_packed.argtypes = [vp, vp, sz, vp, sz]
    L.fhe_hip_multi_create.argtypes = [ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, ctypes.POINTER(vp)]
    L.fhe_hip_multi_destroy.argtypes = [vp]
    L.fhe_hip_multi_destroy.restype = None
    L.fhe_hip_multi_load_keys.argtypes = [vp, vp, sz, vp, sz, vp, sz]
    L.fhe_hip_multi_eval_bingate_batch.argtypes = [vp, ctypes.c_int, sz, vp, vp, vp, vp, vp, vp]
    L.fhe_hip_blind_rotate_acc_batch.argtypes = [vp, sz, vp, u64, vp]
    L.fhe_hip_blind_rotate_acc_batch_device.argtypes = [vp, sz, vp, u64, vp, vp]
    L.fhe_hip_external_product_batch.argtypes = [vp, sz, vp, vp, vp]
    L.fhe_hip_external_product_batch_device.argtypes = [vp, sz, vp, vp, vp, vp]
    L.fhe_hip_max_batch_size.argtypes = [vp, vp]
    L.fhe_hip_device_memory.argtypes = [ctypes.c_int, vp, vp]
    L.fhe_hip_unpack_keys.argtypes = [ctypes.c_int, ctypes.c_int, vp, sz, vp, sz, vp, sz, vp, sz, vp, sz]
    L.fhe_hip_switch_to_qn_batch.argtypes = [vp, sz, vp, vp, vp, vp]
    L.fhe_hip_switch_to_qn_batch_device.argtypes = [vp, sz, vp, vp, vp, vp, vp]
    L.fhe_hip_eval_mixed_batch.argtypes = [vp, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, sz, vp, vp, vp, vp, vp,
                                           ctypes.c_int]
    L.fhe_hip_eval_mixed_batch_device.argtypes = [vp, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, sz, vp, vp, vp,
                                                  vp, vp, ctypes.c_int, vp]
    L.fhe_hip_eval_func_multi_batch.argtypes = [vp, sz, vp, vp, u64, vp, sz, ctypes.c_uint32, vp, vp]
    L.fhe_hip_eval_func_multi_batch_device.argtypes = [vp, sz, vp, vp, u64, vp, sz, ctypes.c_uint32, vp, vp, vp]
    L.fhe_hip_keygen_ring_secret.argtypes = [ctypes.c_int, ctypes.c_int, u64, vp]
    L.fhe_hip_encrypt_large.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, sz, u64, ctypes.c_uint32, vp, vp]
    L.fhe_hip_gate_kernel.argtypes = [vp, sz, ctypes.POINTER(ctypes.c_char_p)]
    L.fhe_hip_copy_keys.argtypes = [vp, vp]
    L._binfhe_ready = True
    return L


def L():
    return _setup(lib())


@dataclass(frozen=True)
class Params:
    paramset: int
    method: int
    n: int
    N: int
    q: int
    baseKS: int
    digitsKS: int
    baseG: int
    digitsG: int
    numAutoKeys: int
    keyDist: int
    kernel: int
    Q: int
    psi: int
    qKS: int
    bsk_words: int
    ksk_rows: int


def params(paramset, method):
    p = _Params()
    check(L().fhe_hip_params_get(paramset, method, ctypes.byref(p)))
    return Params(**{f: int(getattr(p, f)) for f, _ in _Params._fields_})


def kernel_path(paramset, method):
    """the accumulator kernels (paramset, method) runs on, as the engine chooses them
    (fhe_hip_params.kernel): 1 = 32-bit one-wave, 2 = 32-bit split (digitsG = 4), 3 = one gate per
    workgroup in 32-bit residues, 4 = GINX gates at N = 2048 on the register-resident split kernel (the
    rest as 3), 0 = one gate per workgroup in 64-bit residues"""
    return params(paramset, method).kernel


def uses_fast_kernels(paramset, method):
    """True when (paramset, method) runs on one of the register-resident 32-bit accumulator kernels
    (one wave or two waves per gate)"""
    return kernel_path(paramset, method) in (1, 2)


def _u64(a):
    return np.ascontiguousarray(a, dtype=np.uint64)


@dataclass
class KeySet:
    sk: np.ndarray
    bsk: np.ndarray
    kskA: np.ndarray
    kskB: np.ndarray


def keygen(paramset, method, seed):
    """Deterministic (sk, bsk, kskA, kskB) in the reference's raw layouts."""
    P = params(paramset, method)
    sk = np.zeros(P.n, np.uint64)
    bsk = np.zeros(P.bsk_words, np.uint64)
    A = np.zeros(P.ksk_rows * P.n, np.uint64)
    B = np.zeros(P.ksk_rows, np.uint64)
    check(L().fhe_hip_keygen(paramset, method, seed, ptr(sk), ptr(bsk), ptr(A), ptr(B)))
    return KeySet(sk, bsk, A, B)


def keygen_secret(paramset, method, seed):
    """KeyGen: the LWE secret only (the same sk keygen(seed) returns)."""
    sk = np.zeros(params(paramset, method).n, np.uint64)
    check(L().fhe_hip_keygen_secret(paramset, method, seed, ptr(sk)))
    return sk


def encrypt(paramset, method, sk, bits, seed, p=4, mod=0):
    """LWE encryptions of `bits` (messages mod p) under sk, modulo `mod` (0: q) (lwe-pke.cpp:103-128)."""
    P = params(paramset, method)
    bits = np.ascontiguousarray(bits, dtype=np.int32)
    a = np.zeros((len(bits), P.n), np.uint64)
    b = np.zeros(len(bits), np.uint64)
    check(L().fhe_hip_encrypt_mod(paramset, method, ptr(_u64(sk)), ptr(bits), len(bits), seed, p, mod, ptr(a),
                                  ptr(b)))
    return a, b


def keygen_ring_secret(paramset, method, seed):
    """skN[N] of keygen(seed) (KeyGenN's key) stored mod qKS: the LWE secret of dimension-N ciphertexts
    mod Q (decrypt(..., skN, a, b, mod=Q) with a of N columns)"""
    skN = np.zeros(params(paramset, method).N, np.uint64)
    check(L().fhe_hip_keygen_ring_secret(paramset, method, seed, ptr(skN)))
    return skN


def encrypt_large(paramset, method, skN, bits, seed, p=4):
    """Encrypt(pk, m, LARGE_DIM, p) (binfhecontext.cpp:236-252): dimension N, modulus Q, under skN"""
    P = params(paramset, method)
    bits = np.ascontiguousarray(bits, dtype=np.int32)
    a = np.zeros((len(bits), P.N), np.uint64)
    b = np.zeros(len(bits), np.uint64)
    check(L().fhe_hip_encrypt_large(paramset, method, ptr(_u64(skN)), ptr(bits), len(bits), seed, p, ptr(a), ptr(b)))
    return a, b


def decrypt(paramset, method, sk, a, b, mod=None, p=4):
    P = params(paramset, method)
    a = _u64(np.atleast_2d(a))
    b = _u64(np.atleast_1d(b))
    out = np.zeros(len(b), np.int64)
    check(L().fhe_hip_decrypt_ptmod(paramset, method, ptr(_u64(sk)), ptr(a), ptr(b), len(b), a.shape[1],
                                    mod if mod is not None else P.q, p, ptr(out)))
    return out


def _ptrs(arrs):
    t = (vp * len(arrs))()
    for j, x in enumerate(arrs):
        t[j] = x.ctypes.data if isinstance(x, np.ndarray) else x
    return t


# ---- the reference's packed transfer format (backend/packed.h) ----
LWE_PACK_INTERLEAVED = 1


def pack_lwe_batch(a, b, flags=0):
    """PackLWEBatch-compatible bytes (backend/packed.cpp:144-211)."""
    a, b = _u64(np.atleast_2d(a)), _u64(np.atleast_1d(b))
    size = ctypes.c_size_t()
    check(L().fhe_hip_pack_lwe_batch(a.shape[1], len(b), ptr(a), ptr(b), flags, None, 0, ctypes.byref(size)))
    out = np.zeros(size.value, np.uint8)
    check(L().fhe_hip_pack_lwe_batch(a.shape[1], len(b), ptr(a), ptr(b), flags, ptr(out), out.size,
                                     ctypes.byref(size)))
    return out.tobytes()


def unpack_lwe_batch(data):
    buf = np.frombuffer(data, np.uint8)
    n, cnt = ctypes.c_uint32(), ctypes.c_size_t()
    check(L().fhe_hip_unpack_lwe_batch(ptr(buf), buf.size, ctypes.byref(n), ctypes.byref(cnt), None, None))
    a = np.zeros((cnt.value, n.value), np.uint64)
    b = np.zeros(cnt.value, np.uint64)
    check(L().fhe_hip_unpack_lwe_batch(ptr(buf), buf.size, ctypes.byref(n), ctypes.byref(cnt), ptr(a), ptr(b)))
    return a, b


def pack_keys(paramset, method, keys):
    """(packed bootstrapping key, packed switching key) bytes."""
    bsk, A, B = _u64(keys.bsk), _u64(keys.kskA), _u64(keys.kskB)
    s1, s2 = ctypes.c_size_t(), ctypes.c_size_t()
    check(L().fhe_hip_pack_keys(paramset, method, ptr(bsk), bsk.size, ptr(A), ptr(B), None, 0, ctypes.byref(s1), None,
                                0, ctypes.byref(s2)))
    ob, ok = np.zeros(s1.value, np.uint8), np.zeros(s2.value, np.uint8)
    check(L().fhe_hip_pack_keys(paramset, method, ptr(bsk), bsk.size, ptr(A), ptr(B), ptr(ob), ob.size,
                                ctypes.byref(s1), ptr(ok), ok.size, ctypes.byref(s2)))
    return ob, ok


def unpack_keys(paramset, method, bsk_packed, ksk_packed):
    """the raw KeySet (sk = None) of packed keys (Backend::UnpackBootstrappingKey)"""
    P = params(paramset, method)
    ob, ok = _buf(bsk_packed), _buf(ksk_packed)
    bsk = np.zeros(P.bsk_words, np.uint64)
    A, B = np.zeros(P.ksk_rows * P.n, np.uint64), np.zeros(P.ksk_rows, np.uint64)
    check(L().fhe_hip_unpack_keys(paramset, method, ptr(ob), ob.size, ptr(bsk), bsk.size, ptr(ok), ok.size, ptr(A),
                                  A.size, ptr(B), B.size))
    return KeySet(None, bsk, A, B)


# ---- the reference's serialized objects (Serial::Serialize(..., SerType::BINARY)) ----
def _buf(data):
    return np.frombuffer(data, np.uint8) if not isinstance(data, np.ndarray) else data


def cereal_read_keys(paramset, method, refresh, switching):
    """raw KeySet (sk = None) from a serialized RingGSWACCKey and LWESwitchingKey"""
    P = params(paramset, method)
    r, w = _buf(refresh), _buf(switching)
    ks = KeySet(None, np.zeros(P.bsk_words, np.uint64), np.zeros(P.ksk_rows * P.n, np.uint64),
                np.zeros(P.ksk_rows, np.uint64))
    check(L().fhe_hip_cereal_read_keys(paramset, method, ptr(r), r.size, ptr(w), w.size, ptr(ks.bsk), ptr(ks.kskA),
                                       ptr(ks.kskB)))
    return ks


def cereal_write_keys(paramset, method, keys):
    """(refresh key bytes, switching key bytes) as the reference's SerializeToFile writes them"""
    bsk, A, B = _u64(keys.bsk), _u64(keys.kskA), _u64(keys.kskB)
    s1, s2 = ctypes.c_size_t(), ctypes.c_size_t()
    args = (paramset, method, ptr(bsk), bsk.size, ptr(A), ptr(B))
    check(L().fhe_hip_cereal_write_keys(*args, None, 0, ctypes.byref(s1), None, 0, ctypes.byref(s2)))
    o1, o2 = np.zeros(s1.value, np.uint8), np.zeros(s2.value, np.uint8)
    check(L().fhe_hip_cereal_write_keys(*args, ptr(o1), o1.size, ctypes.byref(s1), ptr(o2), o2.size,
                                        ctypes.byref(s2)))
    return o1.tobytes(), o2.tobytes()


def cereal_read_lwe(data, is_key=False):
    """(a, b, modulus) of a serialized LWECiphertext, or (s, None, modulus) of an LWEPrivateKey"""
    d = _buf(data)
    n, b, mod = ctypes.c_uint32(), ctypes.c_uint64(), ctypes.c_uint64()
    check(L().fhe_hip_cereal_read_lwe(ptr(d), d.size, int(is_key), None, 0, ctypes.byref(n), ctypes.byref(b),
                                      ctypes.byref(mod)))
    a = np.zeros(n.value, np.uint64)
    check(L().fhe_hip_cereal_read_lwe(ptr(d), d.size, int(is_key), ptr(a), a.size, ctypes.byref(n), ctypes.byref(b),
                                      ctypes.byref(mod)))
    return a, (None if is_key else int(b.value)), int(mod.value)


def cereal_write_lwe(a, b, mod, is_key=False):
    a = _u64(a)
    size = ctypes.c_size_t()
    check(L().fhe_hip_cereal_write_lwe(ptr(a), a.size, int(b or 0), mod, int(is_key), None, 0, ctypes.byref(size)))
    out = np.zeros(size.value, np.uint8)
    check(L().fhe_hip_cereal_write_lwe(ptr(a), a.size, int(b or 0), mod, int(is_key), ptr(out), out.size,
                                       ctypes.byref(size)))
    return out.tobytes()


def cereal_read_context(data):
    """(paramset, method) of the GenerateBinFHEContext row a serialized BinFHEContext (the cryptoContext
    archive of boolean-serial-binary.cpp) holds"""
    d = _buf(data)
    ps, m = ctypes.c_int(), ctypes.c_int()
    check(L().fhe_hip_cereal_read_context(ptr(d), d.size, ctypes.byref(ps), ctypes.byref(m), None))
    return ps.value, m.value


def cereal_write_context(paramset, method):
    """the bytes Serial::Serialize(cc, SerType::BINARY) writes for a context of this row"""
    size = ctypes.c_size_t()
    check(L().fhe_hip_cereal_write_context(paramset, method, None, 0, ctypes.byref(size)))
    out = np.zeros(size.value, np.uint8)
    check(L().fhe_hip_cereal_write_context(paramset, method, ptr(out), out.size, ctypes.byref(size)))
    return out.tobytes()


class GateEngine:
    """One MI355X context (fhe_hip_ctx): resident keys + batched gate bootstrapping."""

    def __init__(self, paramset, method, device=0, _handle=None):
        self._h = vp()
        if _handle is None:
            check(L().fhe_hip_create(paramset, method, device, ctypes.byref(self._h)))
        else:
            self._h = _handle
        self.params = params(paramset, method)
        self.device = device

    @classmethod
    def from_cereal(cls, data, device=0):
        """a context built from a serialized BinFHEContext alone (fhe_hip_create_from_cereal)"""
        d = _buf(data)
        h = vp()
        check(L().fhe_hip_create_from_cereal(ptr(d), d.size, device, ctypes.byref(h)))
        ps, m = cereal_read_context(d)
        return cls(ps, m, device, _handle=h)

    def bootstrap(self, a, b):
        """BinFHEContext::Bootstrap over a batch (fhe_hip_bootstrap_batch)"""
        a, b = _u64(a), _u64(b)
        ao, bo = np.zeros_like(a), np.zeros_like(b)
        check(L().fhe_hip_bootstrap_batch(self._h, b.size, ptr(a), ptr(b), ptr(ao), ptr(bo)))
        return ao, bo

    def gate_kernel(self, count):
        """the blind-rotation kernel a gate batch of `count` runs on in this context (fhe_hip_gate_kernel)"""
        name = ctypes.c_char_p()
        check(L().fhe_hip_gate_kernel(self._h, count, ctypes.byref(name)))
        return name.value.decode()

    def kernel(self):
        """fhe_hip_params::kernel of this context (its own kernel flags, fhe_hip_get_params)"""
        p = _Params()
        check(L().fhe_hip_get_params(self._h, ctypes.byref(p)))
        return p.kernel

    def copy_keys_from(self, src):
        """the resident keys of another context of the same set (fhe_hip_copy_keys)"""
        check(L().fhe_hip_copy_keys(self._h, src._h))

    def close(self):
        if self._h:
            L().fhe_hip_destroy(self._h)
            self._h = vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self):
        return L().fhe_hip_stream(self._h)

    def load_keys(self, bsk, kskA, kskB):
        bsk, kskA, kskB = _u64(bsk), _u64(kskA), _u64(kskB)
        check(L().fhe_hip_load_bsk(self._h, ptr(bsk), bsk.size))
        check(L().fhe_hip_load_ksk(self._h, ptr(kskA), kskA.size, ptr(kskB), kskB.size))

    def eval_gate(self, gate, a1, b1, a2, b2):
        a1, b1, a2, b2 = _u64(a1), _u64(b1), _u64(a2), _u64(b2)
        cnt = len(b1)
        ao = np.zeros((cnt, self.params.n), np.uint64)
        bo = np.zeros(cnt, np.uint64)
        check(L().fhe_hip_eval_bingate_batch(self._h, gate, cnt, ptr(a1), ptr(b1), ptr(a2), ptr(b2), ptr(ao),
                                             ptr(bo)))
        return ao, bo

    def keygen_device(self, sk, seed, export=False):
        """BTKeyGen on this engine's device; keys identical to keygen(seed) for its sk.  With
        export=True the raw layouts come back as a KeySet."""
        sk = _u64(sk)
        P = self.params
        if export:
            ks = KeySet(sk.copy(), np.zeros(P.bsk_words, np.uint64), np.zeros(P.ksk_rows * P.n, np.uint64),
                        np.zeros(P.ksk_rows, np.uint64))
            check(L().fhe_hip_btkeygen_device(self._h, ptr(sk), sk.size, seed, ptr(ks.bsk), ptr(ks.kskA),
                                              ptr(ks.kskB)))
            return ks
        check(L().fhe_hip_btkeygen_device(self._h, ptr(sk), sk.size, seed, None, None, None))
        return None

    def eval_gate_packed(self, gate, in1, in2, out_flags=0):
        """EvalBinGate on two PackLWEBatch buffers; returns the packed result."""
        p1, p2 = np.frombuffer(in1, np.uint8), np.frombuffer(in2, np.uint8)
        size = ctypes.c_size_t()
        check(L().fhe_hip_eval_bingate_packed(self._h, gate, ptr(p1), p1.size, ptr(p2), p2.size, out_flags, None, 0,
                                              ctypes.byref(size)))
        out = np.zeros(size.value, np.uint8)
        check(L().fhe_hip_eval_bingate_packed(self._h, gate, ptr(p1), p1.size, ptr(p2), p2.size, out_flags, ptr(out),
                                              out.size, ctypes.byref(size)))
        return out.tobytes()

    def load_keys_cereal(self, refresh, switching):
        """BTKeyLoad of the reference's serialized refresh / switching keys"""
        r, w = _buf(refresh), _buf(switching)
        check(L().fhe_hip_load_keys_cereal(self._h, ptr(r), r.size, ptr(w), w.size))

    def load_keys_packed(self, bsk_packed, ksk_packed):
        check(L().fhe_hip_load_keys_packed(self._h, ptr(bsk_packed), bsk_packed.size, ptr(ksk_packed),
                                           ksk_packed.size))

    def eval_gate_extended(self, gate, a1, b1, a2, b2):
        a1, b1, a2, b2 = _u64(a1), _u64(b1), _u64(a2), _u64(b2)
        cnt = len(b1)
        ao = np.zeros((cnt, self.params.N), np.uint64)
        bo = np.zeros(cnt, np.uint64)
        check(L().fhe_hip_eval_bingate_extended(self._h, gate, cnt, ptr(a1), ptr(b1), ptr(a2), ptr(b2), ptr(ao),
                                                ptr(bo)))
        return ao, bo

    def eval_gate_device(self, gate, count, d_a1, d_b1, d_a2, d_b2, d_ao, d_bo, stream=None):
        check(L().fhe_hip_eval_bingate_batch_device(self._h, gate, count, vp(d_a1), vp(d_b1), vp(d_a2), vp(d_b2),
                                                    vp(d_ao), vp(d_bo), vp(stream) if stream else None))

    def blind_rotate_device(self, gate, count, d_a1, d_b1, d_a2, d_b2, stream=None):
        check(L().fhe_hip_blind_rotate_batch_device(self._h, gate, count, vp(d_a1), vp(d_b1), vp(d_a2), vp(d_b2),
                                                    vp(stream) if stream else None))

    def keyswitch_workspace_device(self, count, d_ao, d_bo, stream=None):
        check(L().fhe_hip_keyswitch_workspace_device(self._h, count, vp(d_ao), vp(d_bo),
                                                     vp(stream) if stream else None))

    def eval_gate_multi(self, gate, a_list, b_list, p, extended=False):
        """EvalBinGate(gate, ctvector) for MAJORITY/AND3/OR3/AND4/OR4 over a batch of k-tuples:
        a_list[j] [count][n], b_list[j] [count]; p = plaintext modulus of the inputs."""
        a_list = [_u64(a) for a in a_list]
        b_list = [_u64(b) for b in b_list]
        cnt = len(b_list[0])
        ao = np.zeros((cnt, self.params.N if extended else self.params.n), np.uint64)
        bo = np.zeros(cnt, np.uint64)
        check(L().fhe_hip_eval_gate_multi_batch(self._h, gate, len(a_list), p, cnt, _ptrs(a_list), _ptrs(b_list),
                                                ptr(ao), ptr(bo), int(extended)))
        return ao, bo

    def eval_cmux(self, a0, b0, a1, b1, a2, b2):
        """EvalBinGate(CMUX, {ct0, ct1, ct2}) = ct2 ? ct1 : ct0 over a batch."""
        a0, b0, a1, b1, a2, b2 = (_u64(x) for x in (a0, b0, a1, b1, a2, b2))
        cnt = len(b0)
        ao = np.zeros((cnt, self.params.n), np.uint64)
        bo = np.zeros(cnt, np.uint64)
        check(L().fhe_hip_eval_cmux_batch(self._h, cnt, ptr(a0), ptr(b0), ptr(a1), ptr(b1), ptr(a2), ptr(b2),
                                          ptr(ao), ptr(bo)))
        return ao, bo

    def eval_gate_multi_device(self, gate, count, p, d_a_list, d_b_list, d_ao, d_bo, stream=None):
        check(L().fhe_hip_eval_gate_multi_batch_device(self._h, gate, len(d_a_list), p, count, _ptrs(d_a_list),
                                                       _ptrs(d_b_list), vp(d_ao), vp(d_bo),
                                                       vp(stream) if stream else None))

    def switch_to_qn(self, a, b):
        """SwitchCTtoqn (lwe-pke.cpp:170-178): a [count][N], b [count] mod Q -> (n, q)"""
        a, b = _u64(a), _u64(b)
        cnt = len(b)
        ao = np.zeros((cnt, self.params.n), np.uint64)
        bo = np.zeros(cnt, np.uint64)
        check(L().fhe_hip_switch_to_qn_batch(self._h, cnt, ptr(a), ptr(b), ptr(ao), ptr(bo)))
        return ao, bo

    def eval_mixed(self, op, a_list, b_list, large=None, ptmod=4, extended=False):
        """fhe_hip_eval_mixed_batch: op a gate or OP_BOOTSTRAP over k columns whose rows may be mod Q.
        a_list[j]: [count][n] (column all mod q) or [count][N] with large[j][g] = 1 marking the rows mod Q
        (large[j] None: the column is mod q)"""
        a_list = [_u64(a) for a in a_list]
        b_list = [_u64(b) for b in b_list]
        k, cnt = len(a_list), len(b_list[0])
        flags = [None if large is None or large[j] is None else np.ascontiguousarray(large[j], np.uint8)
                 for j in range(k)]
        for j in range(k):
            want = self.params.N if flags[j] is not None else self.params.n
            if a_list[j].shape != (cnt, want):
                raise FheHipError(-2, f"column {j}: rows of {want} words expected")
        wide = extended and op != CMUX
        ao = np.zeros((cnt, self.params.N if wide else self.params.n), np.uint64)
        bo = np.zeros(cnt, np.uint64)
        lp = (vp * k)(*[f.ctypes.data if f is not None else None for f in flags])
        check(L().fhe_hip_eval_mixed_batch(self._h, op, k, ptmod, cnt, _ptrs(a_list), _ptrs(b_list), lp, ptr(ao),
                                           ptr(bo), int(extended)))
        return ao, bo

    def eval_cmux_device(self, count, d_a0, d_b0, d_a1, d_b1, d_a2, d_b2, d_ao, d_bo, stream=None):
        check(L().fhe_hip_eval_cmux_batch_device(self._h, count, vp(d_a0), vp(d_b0), vp(d_a1), vp(d_b1), vp(d_a2),
                                                 vp(d_b2), vp(d_ao), vp(d_bo), vp(stream) if stream else None))

    # ---- functional bootstrapping (binfhe-base-scheme.cpp:241-521) ----
    def _fb_out(self, b, parts=1):
        cnt = len(b)
        return np.zeros((parts, cnt, self.params.n), np.uint64), np.zeros((parts, cnt), np.uint64)

    def eval_func(self, a, b, q_in, lut):
        a, b, lut = _u64(a), _u64(b), _u64(lut)
        ao, bo = self._fb_out(b)
        check(L().fhe_hip_eval_func_batch(self._h, len(b), ptr(a), ptr(b), q_in, ptr(lut), len(lut), ptr(ao), ptr(bo)))
        return ao[0], bo[0]

    def eval_func_multi(self, a, b, q_in, luts):
        """EvalFuncMultiOutputBatch: every LUT of luts [L][q_in] on every input; rows i L + j"""
        a, b = _u64(a), _u64(b)
        luts = _u64(np.atleast_2d(luts))
        L_, cnt = luts.shape[0], len(b)
        ao, bo = np.zeros((cnt * L_, self.params.n), np.uint64), np.zeros(cnt * L_, np.uint64)
        check(L().fhe_hip_eval_func_multi_batch(self._h, cnt, ptr(a), ptr(b), q_in, ptr(luts), luts.shape[1], L_,
                                                 ptr(ao), ptr(bo)))
        return ao, bo

    def eval_floor(self, a, b, mod, roundbits=0):
        a, b = _u64(a), _u64(b)
        ao, bo = self._fb_out(b)
        check(L().fhe_hip_eval_floor_batch(self._h, len(b), ptr(a), ptr(b), mod, roundbits, ptr(ao), ptr(bo)))
        return ao[0], bo[0]

    def eval_sign(self, a, b, mod, scheme_switch=False):
        a, b = _u64(a), _u64(b)
        ao, bo = self._fb_out(b)
        check(L().fhe_hip_eval_sign_batch(self._h, len(b), ptr(a), ptr(b), mod, int(scheme_switch), ptr(ao), ptr(bo)))
        return ao[0], bo[0]

    def eval_decomp(self, a, b, mod):
        a, b = _u64(a), _u64(b)
        k = ctypes.c_uint32()
        check(L().fhe_hip_eval_decomp_parts(self._h, mod, ctypes.byref(k)))
        ao, bo = self._fb_out(b, k.value)
        check(L().fhe_hip_eval_decomp_batch(self._h, len(b), ptr(a), ptr(b), mod, ptr(ao), ptr(bo)))
        return ao, bo

    def bootstrap_func(self, a, b, ctmod, f, fmod):
        a, b, f = _u64(a), _u64(b), _u64(f)
        ao, bo = self._fb_out(b)
        check(L().fhe_hip_bootstrap_func_batch(self._h, len(b), ptr(a), ptr(b), ctmod, ptr(f), fmod, ptr(ao),
                                               ptr(bo)))
        return ao[0], bo[0]

    def keyswitch(self, a, b):
        a, b = _u64(a), _u64(b)
        cnt = len(b)
        ao = np.zeros((cnt, self.params.n), np.uint64)
        bo = np.zeros(cnt, np.uint64)
        check(L().fhe_hip_keyswitch_batch(self._h, cnt, ptr(a), ptr(b), ptr(ao), ptr(bo)))
        return ao, bo

    # ---- the Backend seam (backend.h:131-192) ----
    def blind_rotate_acc(self, a, ctmod, acc):
        """Backend::BlindRotateBatch = EvalAcc: a [count][n] mod ctmod, acc [count][2][N] EVALUATION
        (canonical mod Q) -> the rotated accumulators (a new array)."""
        a = _u64(np.atleast_2d(a))
        out = np.array(acc, dtype=np.uint64, copy=True, order="C").reshape(len(a), 2, self.params.N)
        check(L().fhe_hip_blind_rotate_acc_batch(self._h, len(a), ptr(a), ctmod, ptr(out)))
        return out

    def external_product(self, rgsw, rlwe):
        """Backend::ExternalProductBatch: rgsw [count][digitsG2][2][N], rlwe [count][2][N] (EVALUATION)
        -> rgsw (x) rlwe [count][2][N]."""
        N, d2 = self.params.N, 2 * (self.params.digitsG - 1)
        rgsw = _u64(rgsw).reshape(-1, d2, 2, N)
        rlwe = _u64(rlwe).reshape(-1, 2, N)
        out = np.zeros_like(rlwe)
        check(L().fhe_hip_external_product_batch(self._h, len(rlwe), ptr(rgsw), ptr(rlwe), ptr(out)))
        return out

    def max_batch_size(self):
        v = ctypes.c_size_t()
        check(L().fhe_hip_max_batch_size(self._h, ctypes.byref(v)))
        return v.value

    def modswitch(self, q_from, q_to, a, b):
        a, b = _u64(a), _u64(b)
        cnt, ln = a.shape
        ao = np.zeros_like(a)
        bo = np.zeros_like(b)
        check(L().fhe_hip_modswitch_batch(self._h, q_from, q_to, ln, cnt, ptr(a), ptr(b), ptr(ao), ptr(bo)))
        return ao, bo


class MultiGateEngine:
    """Single-process multi-GPU gate bootstrapping (fhe_hip_multi): one host thread + stream
    per device, contiguous shards, keys replicated, no collectives."""

    def __init__(self, paramset, method, devices):
        self._h = vp()
        devs = np.ascontiguousarray(devices, dtype=np.int32)
        check(L().fhe_hip_multi_create(paramset, method, ptr(devs), len(devs), ctypes.byref(self._h)))
        self.params = params(paramset, method)
        self.devices = list(devices)

    def close(self):
        if self._h:
            L().fhe_hip_multi_destroy(self._h)
            self._h = vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_keys(self, bsk, kskA, kskB):
        bsk, kskA, kskB = _u64(bsk), _u64(kskA), _u64(kskB)
        check(L().fhe_hip_multi_load_keys(self._h, ptr(bsk), bsk.size, ptr(kskA), kskA.size, ptr(kskB), kskB.size))

    def eval_gate(self, gate, a1, b1, a2, b2):
        a1, b1, a2, b2 = _u64(a1), _u64(b1), _u64(a2), _u64(b2)
        cnt = len(b1)
        ao = np.zeros((cnt, self.params.n), np.uint64)
        bo = np.zeros(cnt, np.uint64)
        check(L().fhe_hip_multi_eval_bingate_batch(self._h, gate, cnt, ptr(a1), ptr(b1), ptr(a2), ptr(b2), ptr(ao),
                                                   ptr(bo)))
        return ao, bo


# ------------------------------------------------------------------------------------------
# BinFHEContext mirror (binfhecontext.h)
# ------------------------------------------------------------------------------------------
@dataclass
class LWECiphertext:
    a: np.ndarray
    b: int
    modulus: int
    p: int = 4  # plaintext modulus (GetptModulus)


@dataclass
class LWEPrivateKey:
    s: np.ndarray  # stored mod qKS, as the reference stores it


@dataclass
class SerializedKey:
    """a RingGSWACCKey ("refresh") or LWESwitchingKey stream as Serial::SerializeToFile writes it"""
    data: bytes


class Serial:
    """Serial::SerializeToFile / DeserializeFromFile with SerType::BINARY (utils/serial.h:95-125) for
    the objects of boolean-serial-binary.cpp: BinFHEContext (the cryptoContext archive), LWECiphertext,
    LWEPrivateKey and the two key streams."""

    @staticmethod
    def SerializeToFile(path, obj):
        if isinstance(obj, LWECiphertext):
            data = cereal_write_lwe(obj.a, obj.b, obj.modulus)
        elif isinstance(obj, LWEPrivateKey):
            data = cereal_write_lwe(obj.s, None, 1 << 14, is_key=True)
        elif isinstance(obj, SerializedKey):
            data = obj.data
        elif isinstance(obj, BinFHEContext):   # the key-independent cryptoContext archive
            data = cereal_write_context(obj.paramset, obj.method)
        else:
            raise TypeError(f"cannot serialize {type(obj).__name__}")
        with open(path, "wb") as f:
            f.write(data)
        return True

    @staticmethod
    def DeserializeFromFile(path, cls):
        with open(path, "rb") as f:
            data = f.read()
        if cls is LWECiphertext:
            a, b, mod = cereal_read_lwe(data)
            return LWECiphertext(a, b, mod)
        if cls is LWEPrivateKey:
            return LWEPrivateKey(cereal_read_lwe(data, is_key=True)[0])
        if cls is SerializedKey:
            return SerializedKey(data)
        if cls is BinFHEContext:   # boolean-serial-binary.cpp:108: the parameters come from the archive
            cc = BinFHEContext()
            cc.engine = GateEngine.from_cereal(data, cc.device)
            cc.paramset, cc.method = cereal_read_context(data)
            cc.params = params(cc.paramset, cc.method)
            return cc
        raise TypeError(f"cannot deserialize {cls.__name__}")


class BinFHEContext:
    def __init__(self, device=0, seed=0x5EED):
        self.device = device
        self._seed = seed
        self._ctr = 0
        self.engine = None

    def GenerateBinFHEContext(self, paramset=STD128, method=GINX, *args, logQ=None, N=0, timeOptimization=False):
        """GenerateBinFHEContext(set, method) (binfhecontext.cpp:106-179), or the large-precision
        overload GenerateBinFHEContext(set, arbFunc, logQ = 11, N = 0, method = GINX,
        timeOptimization = False) (:55-104) when the second argument is a bool"""
        if isinstance(method, bool):
            arb = method
            rest = list(args)
            logQ = rest.pop(0) if rest else (11 if logQ is None else logQ)
            N = rest.pop(0) if rest else N
            method = rest.pop(0) if rest else GINX
            timeOptimization = rest.pop(0) if rest else timeOptimization
            paramset = large_paramset(paramset, arb, logQ, N, timeOptimization)
        self.paramset, self.method = paramset, method
        self.params = params(paramset, method)
        self.engine = GateEngine(paramset, method, self.device)

    def _next_seed(self):
        self._ctr += 1
        return (self._seed * 1000003 + self._ctr) & 0xFFFFFFFFFFFFFFFF

    def KeyGen(self):
        return LWEPrivateKey(keygen_secret(self.paramset, self.method, self._next_seed()))

    def BTKeyGen(self, sk):
        """keys generated on the device (fhe_hip_btkeygen_device); nothing crosses PCIe"""
        self._key_seed = self._next_seed()
        self.engine.keygen_device(sk.s, self._key_seed)

    def BTKeyLoad(self, bsk, kskA, kskB=None):
        """raw arrays (bsk, kskA, kskB), or the deserialized refresh / switching keys
        (SerializedKey, SerializedKey) as in boolean-serial-binary.cpp"""
        if isinstance(bsk, SerializedKey):
            self.engine.load_keys_cereal(bsk.data, kskA.data)
        else:
            self.engine.load_keys(bsk, kskA, kskB)
        # the loaded keys may come from elsewhere: their RLWE secret is not the one BTKeyGen's seed derives,
        # so LARGE_DIM encryption (which needs it) refuses until the next BTKeyGen
        self._key_seed = None

    def Encrypt(self, sk, m, output=None, p=4, mod=0):
        """Encrypt(sk, m, SMALL_DIM, p, mod) (binfhecontext.cpp:220-234).  output = LARGE_DIM: a
        dimension-N ciphertext mod Q like the one Encrypt(pk, m, LARGE_DIM, p) makes (:236-252), under the RLWE
        secret of the keys BTKeyGen generated (refused after BTKeyLoad: the loaded keys' secret is unknown).
        The reference's LARGE_DIM encryption is public-key (EncryptN); this one is symmetric under that
        secret, so it decrypts and bootstraps the same but its noise distribution is not the reference's
        (parity of the distribution is unpinned; outputs of gates on it are pinned by tests/test_mixed.py)"""
        if output == LARGE_DIM:
            if getattr(self, "_key_seed", None) is None:
                raise FheHipError(-11, "LARGE_DIM encryption needs the keys of BTKeyGen")
            skN = keygen_ring_secret(self.paramset, self.method, self._key_seed)
            a, b = encrypt_large(self.paramset, self.method, skN, [int(m)], self._next_seed(), p)
            return LWECiphertext(a[0], int(b[0]), self.params.Q, p)
        a, b = encrypt(self.paramset, self.method, sk.s, [int(m)], self._next_seed(), p, mod)
        return LWECiphertext(a[0], int(b[0]), mod or self.params.q, p)

    def Decrypt(self, sk, ct, p=4):
        return int(decrypt(self.paramset, self.method, sk.s, ct.a[None, :], [ct.b], ct.modulus, p)[0])

    # ---- functional bootstrapping (binfhecontext.cpp:340-392) ----
    def GetBeta(self):
        return 128

    def GetMaxPlaintextSpace(self):
        return self.params.q // (2 * self.GetBeta())

    def GenerateLUTviaFunction(self, f, p):
        """GenerateLUTviaFunction (binfhecontext.cpp:372-390): lut[i] = (q/p) f(i p / q, p)"""
        if p & (p - 1):
            raise FheHipError(-2, "plaintext p not power of two")
        q = self.params.q
        lut = []
        for i in range(q):
            v = (q // p) * int(f((i * p) // q, p))
            if v >= q:
                raise FheHipError(-2, "input function should output in Z_{p_output}")
            lut.append(v)
        return np.array(lut, np.uint64)

    def _one(self, ct):
        return ct.a[None, :], np.array([ct.b], np.uint64)

    def EvalFunc(self, ct, lut):
        ao, bo = self.engine.eval_func(*self._one(ct), ct.modulus, lut)
        return LWECiphertext(ao[0], int(bo[0]), ct.modulus, ct.p)

    def EvalFloor(self, ct, roundbits=0):
        ao, bo = self.engine.eval_floor(*self._one(ct), ct.modulus, roundbits)
        return LWECiphertext(ao[0], int(bo[0]), ct.modulus, ct.p)

    def EvalSign(self, ct, schemeSwitch=False):
        ao, bo = self.engine.eval_sign(*self._one(ct), ct.modulus, schemeSwitch)
        return LWECiphertext(ao[0], int(bo[0]), self.params.q)

    def EvalDecomp(self, ct):
        ao, bo = self.engine.eval_decomp(*self._one(ct), ct.modulus)
        mods, mod, q = [], ct.modulus, self.params.q
        while mod > q:
            mods.append(q)
            mod = mod // q * 2 * self.GetBeta()
        mods.append(mod)
        return [LWECiphertext(ao[k][0], int(bo[k][0]), mods[k]) for k in range(len(mods))]

    def EvalNOT(self, ct):
        """EvalNOT (binfhe-base-scheme.cpp:223-236): (q - a, q/4 - b) mod q"""
        q = ct.modulus
        a = np.where(ct.a == 0, 0, q - ct.a.astype(np.uint64)).astype(np.uint64)
        return LWECiphertext(a, int(((q >> 2) - ct.b) % q), q, ct.p)

    def EvalBinGate(self, gate, ct1, ct2=None, extended=False):
        """EvalBinGate(gate, ct1, ct2, extended) or EvalBinGate(gate, ctvector, extended)
        (binfhecontext.h:305-315).  Inputs mod q or mod Q (extended outputs, LARGE_DIM encryptions) are
        switched to (n, q) on the GPU first, as the reference does (binfhe-base-scheme.cpp:92-93, 150-152)."""
        if ct2 is None or isinstance(ct2, bool):
            return self._eval_vector(gate, list(ct1), bool(ct2) if isinstance(ct2, bool) else extended)
        if ct1 is ct2:
            raise FheHipError(-8, "Input ciphertexts should be independant")
        if extended or self._large(ct1) or self._large(ct2):
            ao, bo = self._mixed(gate, [ct1, ct2], 4, extended)
            return self._out(ao, bo, extended, 4)
        return self.EvalBinGateBatch(gate, [ct1], [ct2])[0]

    def Bootstrap(self, ct, extended=False):
        """BinFHEContext::Bootstrap (binfhe-base-scheme.cpp:190-220): a ciphertext mod q or mod Q;
        ctExt (dimension N, mod Q) when extended"""
        ao, bo = self._mixed(OP_BOOTSTRAP, [ct], ct.p, extended)
        return self._out(ao, bo, extended, ct.p)

    def _large(self, ct):
        return ct.modulus == self.params.Q

    def _mixed(self, op, cts, p, extended):
        cols_a, cols_b, large = [], [], []
        P = self.params
        for c in cts:
            if self._large(c):
                if len(c.a) != P.N:
                    raise FheHipError(-2, "ciphertext mod Q of dimension N expected")
                cols_a.append(c.a[None, :]); large.append(np.ones(1, np.uint8))
            else:
                cols_a.append(c.a[None, :]); large.append(None)
            cols_b.append(np.array([c.b], np.uint64))
        return self.engine.eval_mixed(op, cols_a, cols_b, large, p, extended)

    def _out(self, ao, bo, extended, p):
        mod = self.params.Q if extended else self.params.q
        return LWECiphertext(ao[0], int(bo[0]), mod, p)

    def _eval_vector(self, gate, cts, extended=False):
        for i in range(len(cts)):
            for j in range(i + 1, len(cts)):
                if cts[i] is cts[j]:
                    raise FheHipError(-8, "Input ciphertexts should be independent")
        if gate in MULTI_GATES:
            p = cts[0].p
            if extended or any(self._large(c) for c in cts):
                ao, bo = self._mixed(gate, cts, p, extended)
                return self._out(ao, bo, extended, p)
            ao, bo = self.engine.eval_gate_multi(gate, [c.a[None, :] for c in cts],
                                                 [np.array([c.b], np.uint64) for c in cts], p)
            return LWECiphertext(ao[0], int(bo[0]), self.params.q, p)
        if gate == CMUX:
            if len(cts) != 3:
                raise FheHipError(-8, "CMUX gate implemented for ciphertext vectors of size 3")
            if any(self._large(c) for c in cts):   # CMUX ignores extended (:180-182)
                ao, bo = self._mixed(CMUX, cts, 4, False)
                return self._out(ao, bo, False, 4)
            return self.EvalCMUXBatch([cts[0]], [cts[1]], [cts[2]])[0]
        raise FheHipError(-8, "This gate is not implemented for vector of ciphertexts at this time")

    def EvalCMUXBatch(self, ct_sel, ct_true, ct_false):
        """EvalCMUXBatch (batch.cpp:212-249): EvalBinGate(CMUX, {sel, true, false}) per element,
        which the reference evaluates as ctvector[2] ? ctvector[1] : ctvector[0]."""
        if not (len(ct_sel) == len(ct_true) == len(ct_false)):
            raise FheHipError(-2, "Input size mismatch")
        if not ct_sel:
            return []
        st = lambda cs: (np.stack([c.a for c in cs]), np.array([c.b for c in cs], np.uint64))  # noqa: E731
        (a0, b0), (a1, b1), (a2, b2) = st(ct_sel), st(ct_true), st(ct_false)
        ao, bo = self.engine.eval_cmux(a0, b0, a1, b1, a2, b2)
        return [LWECiphertext(ao[i], int(bo[i]), self.params.q) for i in range(len(bo))]

    def EvalBinGateBatch(self, gate, ct1, ct2):
        """EvalBinGateBatch (src/binfhe/lib/batch/batch.cpp:176-210) on the GPU."""
        if len(ct1) != len(ct2):
            raise FheHipError(-2, "Input size mismatch")
        if not ct1:
            return []
        a1 = np.stack([c.a for c in ct1])
        a2 = np.stack([c.a for c in ct2])
        b1 = np.array([c.b for c in ct1], np.uint64)
        b2 = np.array([c.b for c in ct2], np.uint64)
        ao, bo = self.engine.eval_gate(gate, a1, b1, a2, b2)
        return [LWECiphertext(ao[i], int(bo[i]), self.params.q) for i in range(len(bo))]
