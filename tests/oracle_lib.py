"""ctypes wrappers for the TEST-ONLY oracles (never imported by fhe_amd).

* ``Ref``  -> oracle/_ref/libfhe_ref.so : the reference itself, compiled from
  /root/reference by oracle/Makefile (only present where it was built; the
  built .so travels to the GPU box with the snapshot).
* ``Restatement`` -> oracle/_ref/libtfhe_oracle.so : our C restatement
  (oracle/tfhe_oracle.c), pinned against ``Ref`` and tests/golden/.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# FHE_REF_SO: a private copy of the reference library (long golden regenerations, tools/regen_goldens.sh)
REF_SO = os.environ.get("FHE_REF_SO") or os.path.join(ROOT, "oracle", "_ref", "libfhe_ref.so")
RESTATE_SO = os.path.join(ROOT, "oracle", "_ref", "libtfhe_oracle.so")
# the reference + our BackendHIP (integration/backend_hip.cpp) registered in its BackendRegistry
BACKEND_SO = os.path.join(ROOT, "oracle", "_ref", "libbackend_hip.so")

u64p = ctypes.POINTER(ctypes.c_uint64)
vp = ctypes.c_void_p

TOY, STD128_AP, STD128, STD128_LMKCDEY = 0, 2, 3, 21
AP, GINX, LMKCDEY = 1, 2, 3
GATES = {"OR": 0, "AND": 1, "NOR": 2, "NAND": 3, "XOR": 4, "XNOR": 5}
MAJORITY, AND3, OR3, AND4, OR4, CMUX = 6, 7, 8, 9, 10, 13


def _ptrs(arrs):
    """array of k uint64 pointers (const uint64_t* const*) to the given arrays"""
    t = (vp * len(arrs))()
    for j, a in enumerate(arrs):
        t[j] = _p(a)
    return t


def _p(a):
    if a is None:
        return None
    assert a.dtype == np.uint64 and a.flags.c_contiguous
    return a.ctypes.data_as(vp)


def ref_pack_lwe_batch(a, b, flags=0):
    """the reference's own PackLWEBatch (backend/packed.cpp:144-211) on raw arrays"""
    L = ctypes.CDLL(REF_SO)
    a, b = np.ascontiguousarray(a, np.uint64), np.ascontiguousarray(b, np.uint64)
    size = ctypes.c_size_t()
    out = np.zeros(64 + a.size * 8 + b.size * 8, np.uint8)
    rc = L.ref_pack_lwe_batch(ctypes.c_uint32(a.shape[1]), ctypes.c_size_t(len(b)), _p(a), _p(b), ctypes.c_uint32(flags),
                              out.ctypes.data_as(vp), ctypes.c_size_t(out.size), ctypes.byref(size))
    assert rc == 0
    return out[:size.value].tobytes()


def ref_unpack_lwe_batch(data, n, count):
    """the reference's own UnpackLWEBatch (backend/packed.cpp:214-279)"""
    L = ctypes.CDLL(REF_SO)
    buf = np.frombuffer(data, np.uint8)
    a = np.zeros((count, n), np.uint64)
    b = np.zeros(count, np.uint64)
    rc = L.ref_unpack_lwe_batch(buf.ctypes.data_as(vp), ctypes.c_size_t(buf.size), ctypes.c_uint32(n),
                                ctypes.c_size_t(count), _p(a), _p(b))
    assert rc == 0
    return a, b


def ref_serialize_key(ref, which):
    """the reference's Serial::Serialize(BINARY) of its loaded refresh (0) / switching (1) key"""
    L = ctypes.CDLL(REF_SO)
    size = ctypes.c_size_t()
    fn = L.ref_serialize_key
    fn.argtypes = [vp, ctypes.c_int, vp, ctypes.c_size_t, vp]
    assert fn(ref.h, which, None, 0, ctypes.byref(size)) == 0
    out = np.zeros(size.value, np.uint8)
    assert fn(ref.h, which, out.ctypes.data_as(vp), out.size, ctypes.byref(size)) == 0
    return out.tobytes()


def ref_deserialize_keys(ref, refresh, switching):
    """Serial::Deserialize both keys and BTKeyLoad them into the reference context"""
    L = ctypes.CDLL(REF_SO)
    fn = L.ref_deserialize_keys
    fn.argtypes = [vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t]
    ref._chk(fn(ref.h, refresh, len(refresh), switching, len(switching)))


def ref_serialize_lwe(a, b, mod, is_key=False):
    L = ctypes.CDLL(REF_SO)
    a = np.ascontiguousarray(a, np.uint64)
    size = ctypes.c_size_t()
    out = np.zeros(64 + a.size * 8, np.uint8)
    if is_key:
        fn = L.ref_serialize_sk
        fn.argtypes = [ctypes.c_uint32, vp, ctypes.c_uint64, vp, ctypes.c_size_t, vp]
        assert fn(a.size, _p(a), mod, out.ctypes.data_as(vp), out.size, ctypes.byref(size)) == 0
    else:
        fn = L.ref_serialize_ct
        fn.argtypes = [ctypes.c_uint32, vp, ctypes.c_uint64, ctypes.c_uint64, vp, ctypes.c_size_t, vp]
        assert fn(a.size, _p(a), b, mod, out.ctypes.data_as(vp), out.size, ctypes.byref(size)) == 0
    return out[:size.value].tobytes()


def ref_deserialize_ct(data, cap_n=4096):
    L = ctypes.CDLL(REF_SO)
    fn = L.ref_deserialize_ct
    fn.argtypes = [vp, ctypes.c_size_t, ctypes.c_uint32, vp, vp, vp, vp]
    a = np.zeros(cap_n, np.uint64)
    b, n, mod = ctypes.c_uint64(), ctypes.c_uint32(), ctypes.c_uint64()
    assert fn(data, len(data), cap_n, _p(a), ctypes.byref(b), ctypes.byref(n), ctypes.byref(mod)) == 0
    return a[:n.value], int(b.value), int(mod.value)


def ref_available():
    return os.path.exists(REF_SO)


def restatement_available():
    return os.path.exists(RESTATE_SO)


def backend_available():
    return os.path.exists(BACKEND_SO)


class Ref:
    def __init__(self, paramset, method, so=REF_SO):
        self.L = ctypes.CDLL(so)
        L = self.L
        L.ref_ctx_create.restype = vp
        L.ref_ctx_create.argtypes = [ctypes.c_int, ctypes.c_int]
        L.ref_last_error.restype = ctypes.c_char_p
        L.ref_bsk_len.restype = ctypes.c_size_t
        L.ref_bsk_len.argtypes = [vp]
        L.ref_ntt_bench.restype = ctypes.c_double
        L.ref_ntt_bench.argtypes = [ctypes.c_uint64, ctypes.c_uint32, vp, ctypes.c_int]
        L.ref_time_gates.restype = ctypes.c_double
        L.ref_time_gates.argtypes = [vp, ctypes.c_int, ctypes.c_size_t, vp, vp, vp, vp, vp, vp, ctypes.c_int]
        self.h = vp(L.ref_ctx_create(paramset, method)) if paramset is not None else None
        if self.h is not None and not self.h.value:
            raise RuntimeError(self.err())
        if self.h is not None:
            info = np.zeros(12, np.uint64)
            self._chk(L.ref_ctx_info(self.h, _p(info)))
            (self.n, self.N, self.q, self.Q, self.qKS, self.baseKS, self.digitsKS, self.baseG,
             self.digitsG, self.psi, self.numAutoKeys, self.keyDist) = [int(x) for x in info]
            self.method_is_ginx = method == GINX
            # timeOptimization (paramset code bit 14, logQ != 11): three switching keys in the raw layout
            self.ksk_keys = 3 if (paramset & (1 << 30) and paramset & (1 << 14) and (paramset & 0xff) != 11) else 1

    def err(self):
        return self.L.ref_last_error().decode()

    def _chk(self, rc):
        if rc != 0:
            raise RuntimeError("reference error: " + self.err())

    def __del__(self):
        try:
            if self.h is not None:
                self.L.ref_ctx_destroy(self.h)
        except Exception:
            pass

    def bsk_len(self):
        return int(self.L.ref_bsk_len(self.h))

    def ntt(self, Q, polys, inverse=False):
        polys = np.ascontiguousarray(polys, dtype=np.uint64).copy()
        cnt, N = polys.shape
        psi = ctypes.c_uint64()
        self._chk(self.L.ref_ntt(ctypes.c_uint64(Q), ctypes.c_uint32(N), _p(polys), ctypes.c_size_t(cnt),
                                 int(inverse), ctypes.byref(psi)))
        return polys, psi.value

    def keygen(self):
        sk = np.zeros(self.n, np.uint64)
        bsk = np.zeros(self.bsk_len(), np.uint64)
        rows = self.N * self.baseKS * self.digitsKS * self.ksk_keys
        A = np.zeros(rows * self.n, np.uint64)
        B = np.zeros(rows, np.uint64)
        self._chk(self.L.ref_keygen(self.h, _p(sk), _p(bsk), _p(A), _p(B)))
        return sk, bsk, A, B

    def encrypt(self, bits):
        a = np.zeros((len(bits), self.n), np.uint64)
        b = np.zeros(len(bits), np.uint64)
        for i, m in enumerate(bits):
            self._chk(self.L.ref_encrypt(self.h, int(m), _p(a[i]), ctypes.byref(ctypes.c_uint64.from_buffer(b, 8 * i))))
        return a, b

    def load_keys(self, bsk, A, B):
        self._chk(self.L.ref_load_keys(self.h, _p(bsk), _p(A), _p(B)))

    def eval_gate(self, gate, a1, b1, a2, b2, extended=False, nthreads=0):
        cnt = a1.shape[0]
        L = self.N if extended else self.n
        ao = np.zeros((cnt, L), np.uint64)
        bo = np.zeros(cnt, np.uint64)
        self._chk(self.L.ref_eval_gate(self.h, ctypes.c_int(gate), ctypes.c_size_t(cnt), _p(a1), _p(b1), _p(a2),
                                       _p(b2), _p(ao), _p(bo), ctypes.c_int(int(extended)), ctypes.c_int(nthreads)))
        return ao, bo

    def eval_gate_multi(self, gate, a_list, b_list, ptmod, extended=False, nthreads=0):
        """EvalBinGate(gate, ctvector, extended) per k-tuple (gate = MAJORITY..OR4 or CMUX)."""
        cnt = a_list[0].shape[0]
        L = self.N if extended else self.n
        ao = np.zeros((cnt, L), np.uint64)
        bo = np.zeros(cnt, np.uint64)
        self._chk(self.L.ref_eval_gate_multi(self.h, ctypes.c_int(gate), ctypes.c_uint32(len(a_list)),
                                             ctypes.c_uint32(ptmod), ctypes.c_size_t(cnt), _ptrs(a_list),
                                             _ptrs(b_list), _p(ao), _p(bo), ctypes.c_int(int(extended)),
                                             ctypes.c_int(nthreads)))
        return ao, bo

    def eval_mixed(self, op, a_list, b_list, large, ptmod=4, extended=False, nthreads=0):
        """ref_eval_mixed: EvalBinGate / EvalBinGate(ctvector) / Bootstrap (op = -1) on columns whose rows may
        be mod Q (large[j][g] = 1; such a column has rows of N words, large[j] None: rows of n words mod q)"""
        cnt = len(b_list[0])
        L = self.N if (extended and op != 13) else self.n
        ao = np.zeros((cnt, L), np.uint64)
        bo = np.zeros(cnt, np.uint64)
        a_list = [np.ascontiguousarray(x, np.uint64) for x in a_list]
        b_list = [np.ascontiguousarray(x, np.uint64) for x in b_list]
        flags = [None if large is None or large[j] is None else np.ascontiguousarray(large[j], np.uint8)
                 for j in range(len(a_list))]
        lp = (vp * len(flags))(*[f.ctypes.data if f is not None else None for f in flags])
        self._chk(self.L.ref_eval_mixed(self.h, ctypes.c_int(op), ctypes.c_uint32(len(a_list)), ctypes.c_uint32(ptmod),
                                        ctypes.c_size_t(cnt), _ptrs(a_list), _ptrs(b_list), lp, _p(ao), _p(bo),
                                        ctypes.c_int(int(extended)), ctypes.c_int(nthreads)))
        return ao, bo

    def decrypt(self, sk, a, b, mod, ptmod=4):
        r = ctypes.c_int64()
        self._chk(self.L.ref_decrypt_p(self.h, _p(np.ascontiguousarray(sk, np.uint64)),
                                       _p(np.ascontiguousarray(a, np.uint64)), ctypes.c_uint64(int(b)),
                                       ctypes.c_uint32(len(a)), ctypes.c_uint64(mod), ctypes.c_uint32(ptmod),
                                       ctypes.byref(r)))
        return r.value

    # functional bootstrapping through BinFHEContext (binfhecontext.cpp:340-370)
    def eval_func(self, a, b, ct_mod, lut, nthreads=0):
        ao, bo = np.zeros_like(a), np.zeros_like(b)
        lut = np.ascontiguousarray(lut, np.uint64)
        self._chk(self.L.ref_eval_func(self.h, ctypes.c_size_t(len(b)), _p(a), _p(b), ctypes.c_uint64(ct_mod), _p(lut),
                                       ctypes.c_size_t(len(lut)), _p(ao), _p(bo), ctypes.c_int(nthreads)))
        return ao, bo

    def eval_floor(self, a, b, ct_mod, roundbits=0, nthreads=0):
        ao, bo = np.zeros_like(a), np.zeros_like(b)
        self._chk(self.L.ref_eval_floor(self.h, ctypes.c_size_t(len(b)), _p(a), _p(b), ctypes.c_uint64(ct_mod),
                                        ctypes.c_uint32(roundbits), _p(ao), _p(bo), ctypes.c_int(nthreads)))
        return ao, bo

    def eval_sign(self, a, b, ct_mod, scheme_switch=False):
        ao, bo = np.zeros_like(a), np.zeros_like(b)
        self._chk(self.L.ref_eval_sign(self.h, ctypes.c_size_t(len(b)), _p(a), _p(b), ctypes.c_uint64(ct_mod),
                                       ctypes.c_int(int(scheme_switch)), _p(ao), _p(bo)))
        return ao, bo

    def eval_decomp(self, a, b, ct_mod, max_parts=16):
        cnt, n = a.shape
        ao = np.zeros((max_parts, cnt, n), np.uint64)
        bo = np.zeros((max_parts, cnt), np.uint64)
        parts = ctypes.c_size_t()
        self._chk(self.L.ref_eval_decomp(self.h, ctypes.c_size_t(cnt), _p(a), _p(b), ctypes.c_uint64(ct_mod),
                                         ctypes.c_size_t(max_parts), _p(ao), _p(bo), ctypes.byref(parts)))
        k = parts.value
        return np.ascontiguousarray(ao.reshape(-1)[:k * cnt * n].reshape(k, cnt, n)), np.ascontiguousarray(
            bo.reshape(-1)[:k * cnt].reshape(k, cnt))

    def time_gates(self, gate, a1, b1, a2, b2, nthreads=0):
        cnt = a1.shape[0]
        ao = np.zeros((cnt, self.n), np.uint64)
        bo = np.zeros(cnt, np.uint64)
        t = self.L.ref_time_gates(self.h, gate, cnt, _p(a1), _p(b1), _p(a2), _p(b2), _p(ao), _p(bo), nthreads)
        if t < 0:
            raise RuntimeError(self.err())
        return t, ao, bo

    def modswitch(self, q_from, q_to, a, b):
        cnt, L = a.shape
        ao = np.zeros_like(a)
        bo = np.zeros_like(b)
        self._chk(self.L.ref_modswitch(self.h, ctypes.c_uint64(q_from), ctypes.c_uint64(q_to), ctypes.c_uint32(L),
                                       ctypes.c_size_t(cnt), _p(a), _p(b), _p(ao), _p(bo)))
        return ao, bo

    def keyswitch(self, a, b):
        cnt = a.shape[0]
        ao = np.zeros((cnt, self.n), np.uint64)
        bo = np.zeros(cnt, np.uint64)
        self._chk(self.L.ref_keyswitch(self.h, ctypes.c_size_t(cnt), _p(a), _p(b), _p(ao), _p(bo)))
        return ao, bo


class _Params(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint32) for f in
                ("n", "N", "q", "qKS", "baseKS", "digitsKS", "baseG", "gBits", "digitsG", "numAutoKeys",
                 "method", "paramset", "baseR", "digitsR")] + [("Q", ctypes.c_uint64), ("psi", ctypes.c_uint64)]


class Restatement:
    """Our C restatement of the reference path (oracle/tfhe_oracle.c)."""

    def __init__(self, paramset=None, method=None):
        self.L = ctypes.CDLL(RESTATE_SO)
        self.L.tfo_last_prime.restype = ctypes.c_uint64
        self.L.tfo_root_of_unity.restype = ctypes.c_uint64
        self.L.tfo_root_of_unity.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        self.L.tfo_decrypt.restype = ctypes.c_int64
        self.L.tfo_decrypt.argtypes = [vp, ctypes.c_uint64, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64]
        self.L.tfo_decrypt_p.restype = ctypes.c_int64
        self.L.tfo_decrypt_p.argtypes = [vp, ctypes.c_uint64, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                         ctypes.c_uint32]
        self.p = None
        if paramset is not None:
            self.p = _Params()
            rc = self.L.tfo_params_init(paramset, method, ctypes.byref(self.p))
            if rc != 0:
                raise ValueError("bad params")
            for f, _ in _Params._fields_:
                setattr(self, f, getattr(self.p, f))

    def ntt(self, Q, psi, polys, inverse=False, nthreads=8):
        polys = np.ascontiguousarray(polys, dtype=np.uint64).copy()
        cnt, N = polys.shape
        self.L.tfo_ntt_batch(_p(polys), ctypes.c_size_t(cnt), ctypes.c_uint32(N), ctypes.c_uint64(Q),
                             ctypes.c_uint64(psi), int(inverse), nthreads)
        return polys

    def eval_gate(self, bsk, A, B, gate, a1, b1, a2, b2, stage=0, nthreads=8):
        cnt = a1.shape[0]
        L = self.N if stage == 1 else self.n
        ao = np.zeros((cnt, L), np.uint64)
        bo = np.zeros(cnt, np.uint64)
        self.L.tfo_eval_gate_batch(ctypes.byref(self.p), _p(bsk), _p(A), _p(B), ctypes.c_int(gate),
                                   ctypes.c_size_t(cnt), _p(a1), _p(b1), _p(a2), _p(b2), _p(ao), _p(bo),
                                   ctypes.c_int(stage), ctypes.c_int(nthreads))
        return ao, bo

    def eval_gate_multi(self, bsk, A, B, gate, a_list, b_list, ptmod, stage=0, nthreads=8):
        cnt = a_list[0].shape[0]
        L = self.N if stage == 1 else self.n
        ao = np.zeros((cnt, L), np.uint64)
        bo = np.zeros(cnt, np.uint64)
        rc = self.L.tfo_eval_gate_multi_batch(ctypes.byref(self.p), _p(bsk), _p(A), _p(B), ctypes.c_int(gate),
                                              ctypes.c_uint32(len(a_list)), ctypes.c_uint32(ptmod),
                                              ctypes.c_size_t(cnt), _ptrs(a_list), _ptrs(b_list), _p(ao), _p(bo),
                                              ctypes.c_int(stage), ctypes.c_int(nthreads))
        if rc != 0:
            raise ValueError("tfo_eval_gate_multi_batch: bad arguments")
        return ao, bo

    def eval_cmux(self, bsk, A, B, a0, b0, a1, b1, a2, b2, nthreads=8):
        cnt = a0.shape[0]
        ao = np.zeros((cnt, self.n), np.uint64)
        bo = np.zeros(cnt, np.uint64)
        self.L.tfo_eval_cmux_batch(ctypes.byref(self.p), _p(bsk), _p(A), _p(B), ctypes.c_size_t(cnt), _p(a0), _p(b0),
                                   _p(a1), _p(b1), _p(a2), _p(b2), _p(ao), _p(bo), ctypes.c_int(nthreads))
        return ao, bo

    # functional bootstrapping restatement (oracle/tfhe_oracle.c)
    def bootstrap_func(self, bsk, A, B, a, b, ctmod, tv, fmod, nthreads=8):
        ao, bo = np.zeros_like(a), np.zeros_like(b)
        tv = np.ascontiguousarray(tv, np.uint64)
        rc = self.L.tfo_bootstrap_func_batch(ctypes.byref(self.p), _p(bsk), _p(A), _p(B), ctypes.c_size_t(len(b)),
                                             _p(a), _p(b), ctypes.c_uint64(ctmod), _p(tv), ctypes.c_uint64(fmod),
                                             _p(ao), _p(bo), ctypes.c_int(nthreads))
        if rc:
            raise ValueError("tfo_bootstrap_func_batch")
        return ao, bo

    def eval_func(self, bsk, A, B, a, b, ct_mod, lut, nthreads=8):
        ao, bo = np.zeros_like(a), np.zeros_like(b)
        lut = np.ascontiguousarray(lut, np.uint64)
        rc = self.L.tfo_eval_func_batch(ctypes.byref(self.p), _p(bsk), _p(A), _p(B), ctypes.c_size_t(len(b)), _p(a),
                                        _p(b), ctypes.c_uint64(ct_mod), _p(lut), _p(ao), _p(bo), ctypes.c_int(nthreads))
        if rc:
            raise ValueError("tfo_eval_func_batch")
        return ao, bo

    def eval_floor(self, bsk, A, B, a, b, ct_mod, roundbits=0, nthreads=8):
        ao, bo = np.zeros_like(a), np.zeros_like(b)
        self.L.tfo_eval_floor_batch(ctypes.byref(self.p), _p(bsk), _p(A), _p(B), ctypes.c_size_t(len(b)), _p(a),
                                    _p(b), ctypes.c_uint64(ct_mod), ctypes.c_uint32(roundbits), _p(ao), _p(bo),
                                    ctypes.c_int(nthreads))
        return ao, bo

    def eval_sign(self, bsk, A, B, a, b, ct_mod, scheme_switch=False, nthreads=8):
        ao, bo = np.zeros_like(a), np.zeros_like(b)
        rc = self.L.tfo_eval_sign_batch(ctypes.byref(self.p), _p(bsk), _p(A), _p(B), ctypes.c_size_t(len(b)), _p(a),
                                        _p(b), ctypes.c_uint64(ct_mod), ctypes.c_int(int(scheme_switch)), _p(ao),
                                        _p(bo), ctypes.c_int(nthreads))
        if rc:
            raise ValueError("tfo_eval_sign_batch")
        return ao, bo

    def eval_decomp(self, bsk, A, B, a, b, ct_mod, nthreads=8):
        cnt, n = a.shape
        self.L.tfo_eval_decomp_parts.restype = ctypes.c_uint32
        k = self.L.tfo_eval_decomp_parts(ctypes.byref(self.p), ctypes.c_uint64(ct_mod))
        ao = np.zeros((k, cnt, n), np.uint64)
        bo = np.zeros((k, cnt), np.uint64)
        rc = self.L.tfo_eval_decomp_batch(ctypes.byref(self.p), _p(bsk), _p(A), _p(B), ctypes.c_size_t(cnt), _p(a),
                                          _p(b), ctypes.c_uint64(ct_mod), _p(ao), _p(bo), ctypes.c_int(nthreads))
        if rc:
            raise ValueError("tfo_eval_decomp_batch")
        return ao, bo

    def modswitch(self, q_from, q_to, a, b):
        cnt, L = a.shape
        ao = np.zeros_like(a)
        bo = np.zeros_like(b)
        self.L.tfo_modswitch(ctypes.c_uint64(q_from), ctypes.c_uint64(q_to), ctypes.c_uint32(L), ctypes.c_size_t(cnt),
                             _p(a), _p(b), _p(ao), _p(bo))
        return ao, bo

    def keyswitch(self, A, B, a, b):
        cnt = a.shape[0]
        ao = np.zeros((cnt, self.n), np.uint64)
        bo = np.zeros(cnt, np.uint64)
        self.L.tfo_keyswitch(ctypes.byref(self.p), _p(A), _p(B), ctypes.c_size_t(cnt), _p(a), _p(b), _p(ao), _p(bo))
        return ao, bo

    def decrypt(self, sk, skmod, a, b, mod, ptmod=4):
        a = np.ascontiguousarray(a, np.uint64)
        return int(self.L.tfo_decrypt_p(_p(np.ascontiguousarray(sk, np.uint64)), ctypes.c_uint64(skmod), _p(a),
                                        ctypes.c_uint64(int(b)), ctypes.c_uint32(len(a)), ctypes.c_uint64(mod),
                                        ctypes.c_uint32(ptmod)))
