"""The drop-in boundary as the reference sees it: our BackendHIP (integration/backend_hip.cpp), built
against the reference's own backend.h (oracle/Makefile -> oracle/_ref/libbackend_hip.so), is
registered in the reference's BackendRegistry and every seam operation is run through
CurrentBackend() on the GPU and through the reference's CPU path on the same objects
(oracle/bh_driver.cpp):

  BlindRotateBatch      vs RingGSWAccumulator{CGGI,LMKCDEY,DM}::EvalAcc on arbitrary accumulators
  BlindRotateBatch with null accumulators (what BootstrapBatch passes) vs BootstrapGateCore(AND,
                        ct + q/4), the restated test vector pinned by the reference's Bootstrap(ct, true);
                        lux::fhe::BootstrapBatch itself with BackendHIP as the default
  ExternalProductBatch  vs AddToAccLMKCDEY (SignedDigitDecompose + NativePoly products)
  lux::fhe::KeySwitchBatch / ModSwitchBatch (batch.cpp:251-314) with BackendHIP as the default
  KeySwitchBatch        vs LWEEncryptionScheme::KeySwitch
  ModSwitchBatch        vs LWEEncryptionScheme::ModSwitch (Q -> qKS, qKS -> q)
  EvalBinGateBatch      vs lux::fhe::EvalBinGateBatch (batch.cpp), directly and routed through the registry
  Pack/Unpack{BootstrappingKey,Ciphertexts}, memory calls, info calls.
Parameter sets: STD128 / STD128_LMKCDEY / STD128_AP on the 32-bit kernels, STD128_3 (GINX, digitsG = 4)
and STD128_4_LMKCDEY (the split-layout sets, whose seam calls run on the 64-bit accumulator), STD192 and
STD192_LMKCDEY (N = 2048).  Keys: our seeded keys (as the goldens use) and, for STD128 GINX, keys the
reference generated itself."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from oracle_lib import BACKEND_SO, Ref, backend_available

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "fhe_amd", "libfhe_amd.so")
vp = ctypes.c_void_p
sz = ctypes.c_size_t
u64 = ctypes.c_uint64
STD128, STD128_LMKCDEY, GINX, LMKCDEY = 3, 21, 2, 3
BH = ["bh_register", "bh_unregister", "bh_info", "bh_memory_roundtrip", "bh_blind_rotate", "bh_external_product",
      "bh_keyswitch", "bh_modswitch", "bh_eval_gates", "bh_pack_roundtrip", "bh_last_error", "bh_bootstrap_init",
      "bh_batch_callers", "bh_eval_gates_routed", "bh_eval_mixed_routed"]
STD128_AP, AP = 2, 1
# name -> (paramset, method) (binfhe-constants.h:49-95); "_refkeys": keys from the reference's BTKeyGen
BACKEND_SETS = {"std128": (STD128, GINX), "lmkcdey": (STD128_LMKCDEY, LMKCDEY), "std128_refkeys": (STD128, GINX),
                "ap": (STD128_AP, AP), "std128_3": (4, GINX), "std128_4_lmkcdey": (23, LMKCDEY),
                "std192": (9, GINX), "std192_lmkcdey": (27, LMKCDEY),
                # K1w (N = 2048, accumulator in registers, accumulator-I/O instantiations): seam parity with the
                # reference's EvalAcc directly, not only with the K5 GPU path
                "std256q": (18, GINX), "std256q_3_lmkcdey": (37, LMKCDEY)}

needs_backend = pytest.mark.skipif(not backend_available(), reason="oracle/_ref/libbackend_hip.so not built")


def P(a):
    assert a.dtype == np.uint64 and a.flags.c_contiguous
    return a.ctypes.data_as(vp)


def dyn_symbols(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if ln.strip()}


def undefined_symbols(path):
    out = subprocess.run(["nm", "-D", "--undefined-only", path], capture_output=True, text=True, check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if ln.strip()}


# ----------------------------------------------------------------- CPU ----
def test_product_library_links_nothing_from_the_reference():
    """libfhe_amd.so neither needs nor defines any reference (lux::fhe) symbol"""
    needed = subprocess.run(["readelf", "-d", LIB], capture_output=True, text=True, check=True).stdout
    assert "fhe_ref" not in needed and "backend_hip" not in needed
    assert not [s for s in dyn_symbols(LIB) | undefined_symbols(LIB) if "3lux3fhe" in s]


@needs_backend
def test_backend_library_exports_and_binds_through_the_c_abi():
    syms = dyn_symbols(BACKEND_SO)
    assert all(s in syms for s in BH)
    # BackendHIP reaches libfhe_amd only through the C-ABI of include/fhe_hip.h
    used = {s for s in undefined_symbols(BACKEND_SO) if s.startswith("fhe_hip_")}
    hdr = open(os.path.join(ROOT, "include", "fhe_hip.h")).read()
    assert used and all(s + "(" in hdr for s in used), used
    # every pure virtual of backend.h is overridden (the class compiled as concrete: it is instantiated)
    src = open(os.path.join(ROOT, "integration", "backend_hip.h")).read()
    for m in ("Type", "Name", "IsAvailable", "MaxBatchSize", "DeviceMemory", "Allocate", "Free", "CopyToDevice",
              "CopyToHost", "Synchronize", "BlindRotate", "ExternalProduct", "KeySwitch", "ModSwitch",
              "BlindRotateBatch", "ExternalProductBatch", "KeySwitchBatch", "ModSwitchBatch", "PackBootstrappingKey",
              "UnpackBootstrappingKey", "PackCiphertexts", "UnpackCiphertexts"):
        assert f" {m}(" in src and "override" in src.split(f" {m}(")[1].split(";")[0], m


# ----------------------------------------------------------------- GPU ----
class Backend:
    """ctypes view of oracle/_ref/libbackend_hip.so for one parameter set"""

    def __init__(self, paramset, method, keys=None):
        self.ref = Ref(paramset, method, so=BACKEND_SO)
        self.L = self.ref.L
        self.L.bh_last_error.restype = ctypes.c_char_p
        if os.environ.get("FHE_SEGV_TRACE") == "1":   # native stack of a fault (oracle/bh_driver.cpp)
            self.L.bh_install_fault_trace()
        self.ps, self.m = paramset, method
        if keys is None:     # the reference's own key generation
            self.sk, bsk, A, B = self.ref.keygen()
            self.ref.load_keys(bsk, A, B)
        else:
            self.sk = keys.sk
            self.ref.load_keys(keys.bsk, keys.kskA, keys.kskB)
        self.chk(self.L.bh_register(paramset, method, 0))

    def chk(self, rc):
        if rc != 0:
            raise RuntimeError("bh: " + self.L.bh_last_error().decode())

    def close(self):
        self.chk(self.L.bh_unregister())

    @property
    def h(self):
        return self.ref.h


_backends = {}


def backend(name):
    from fhe_amd import binfhe as bf
    if name not in _backends:
        for b in _backends.values():
            b.close()
        _backends.clear()
        ps, m = BACKEND_SETS[name]
        keys = None if name.endswith("refkeys") else bf.keygen(ps, m, 0xB0070000 + ps)
        _backends[name] = Backend(ps, m, keys)
    return _backends[name]


@pytest.fixture(scope="module", autouse=True)
def _release():
    yield
    for b in _backends.values():
        b.close()
    _backends.clear()


SETS = list(BACKEND_SETS)


@pytest.fixture(scope="module", params=SETS)
def bset(request):
    """the parameter set under test; module scope with params makes pytest run every test of one set
    before the next set is set up (one key generation and registration per set)"""
    return request.param


NOREF = [x for x in SETS if x != "std128_refkeys"]


@pytest.mark.gpu
@needs_backend
@pytest.mark.parametrize("bset", ("std128", "lmkcdey"), indirect=True)
def test_gpu_backend_registered_info_and_memory(bset):
    name = bset
    b = backend(name)
    out = np.zeros(5, np.uint64)
    buf = ctypes.create_string_buffer(256)
    b.chk(b.L.bh_info(P(out), buf, sz(256)))
    assert out[0] == 4 and out[1] == 1 and out[4] == 1       # kBackendHIP, available, in the registry
    assert out[2] >= 65536 and out[3] > 100e9                 # MaxBatchSize, DeviceMemory (bytes)
    assert b"HIP" in buf.value
    src = np.random.default_rng(3).integers(0, 256, 1 << 20, dtype=np.uint8)
    back = np.zeros_like(src)
    b.chk(b.L.bh_memory_roundtrip(src.ctypes.data_as(vp), sz(src.size), back.ctypes.data_as(vp)))
    assert np.array_equal(src, back)


@pytest.mark.gpu
@needs_backend
def test_gpu_backend_blind_rotate_equals_evalacc(bset):
    name = bset
    """BlindRotateBatch on arbitrary accumulators (uniform mod Q, EVALUATION) and ragged counts"""
    b = backend(name)
    r = b.ref
    rng = np.random.default_rng(11)
    mods = [r.q, 2 * r.N] if r.method_is_ginx else [r.q] if b.m == AP else [2 * r.N]
    for ctmod in mods:
        for count in (1, 6):
            a = rng.integers(0, ctmod, (count, r.n), dtype=np.uint64)
            acc = rng.integers(0, r.Q, (count, 2, r.N), dtype=np.uint64)
            g, ref = np.zeros_like(acc), np.zeros_like(acc)
            b.chk(b.L.bh_blind_rotate(b.h, sz(count), P(a), u64(ctmod), P(acc), P(g), P(ref), 0))
            assert np.array_equal(g, ref), (name, ctmod, count)


@pytest.mark.gpu
@needs_backend
@pytest.mark.parametrize("bset", NOREF, indirect=True)
def test_gpu_backend_external_product_equals_reference(bset):
    name = bset
    b = backend(name)
    r = b.ref
    rng = np.random.default_rng(12)
    dG2 = 2 * (r.digitsG - 1)
    for count in (1, 7):
        rgsw = rng.integers(0, r.Q, (count, dG2, 2, r.N), dtype=np.uint64)
        rlwe = rng.integers(0, r.Q, (count, 2, r.N), dtype=np.uint64)
        g, ref = np.zeros_like(rlwe), np.zeros_like(rlwe)
        b.chk(b.L.bh_external_product(b.h, sz(count), P(rgsw), P(rlwe), P(g), P(ref)))
        assert np.array_equal(g, ref), (name, count)


@pytest.mark.gpu
@needs_backend
@pytest.mark.parametrize("bset", NOREF, indirect=True)
def test_gpu_backend_keyswitch_and_modswitch_equal_reference(bset):
    name = bset
    b = backend(name)
    r = b.ref
    rng = np.random.default_rng(13)
    count = 9
    a = rng.integers(0, r.qKS, (count, r.N), dtype=np.uint64)
    bb = rng.integers(0, r.qKS, count, dtype=np.uint64)
    ga, gb = np.zeros((count, r.n), np.uint64), np.zeros(count, np.uint64)
    ra, rb = np.zeros_like(ga), np.zeros_like(gb)
    b.chk(b.L.bh_keyswitch(b.h, sz(count), P(a), P(bb), P(ga), P(gb), P(ra), P(rb)))
    assert np.array_equal(ga, ra) and np.array_equal(gb, rb)
    for mod, ln, to in ((r.Q, r.N, r.qKS), (r.qKS, r.n, r.q)):
        a = rng.integers(0, mod, (count, ln), dtype=np.uint64)
        bb = rng.integers(0, mod, count, dtype=np.uint64)
        ga, gb = np.zeros_like(a), np.zeros_like(bb)
        ra, rb = np.zeros_like(a), np.zeros_like(bb)
        mo = ctypes.c_uint64()
        b.chk(b.L.bh_modswitch(b.h, sz(count), ctypes.c_uint32(ln), u64(mod), P(a), P(bb), P(ga), P(gb), P(ra),
                               P(rb), ctypes.byref(mo)))
        assert mo.value == to
        assert np.array_equal(ga, ra) and np.array_equal(gb, rb), (mod, to)


@pytest.mark.gpu
@needs_backend
def test_gpu_backend_gate_batch_equals_reference_evalbingatebatch(bset):
    name = bset
    from fhe_amd import binfhe as bf
    b = backend(name)
    r = b.ref
    count = 12
    rng = np.random.default_rng(14)
    x1, x2 = rng.integers(0, 2, count), rng.integers(0, 2, count)
    a1, b1 = bf.encrypt(b.ps, b.m, b.sk, x1, 501)
    a2, b2 = bf.encrypt(b.ps, b.m, b.sk, x2, 502)
    for gate, truth in ((1, x1 & x2), (4, x1 ^ x2), (3, 1 - (x1 & x2))):
        ga, gb = np.zeros((count, r.n), np.uint64), np.zeros(count, np.uint64)
        ra, rb = np.zeros_like(ga), np.zeros_like(gb)
        b.chk(b.L.bh_eval_gates(b.h, gate, sz(count), P(a1), P(b1), P(a2), P(b2), P(ga), P(gb), P(ra), P(rb)))
        assert np.array_equal(ga, ra) and np.array_equal(gb, rb), gate
        assert np.array_equal(bf.decrypt(b.ps, b.m, b.sk, ga, gb), truth), gate


@pytest.mark.gpu
@needs_backend
@pytest.mark.parametrize("bset", ("std128", "lmkcdey"), indirect=True)
def test_gpu_backend_pack_roundtrips(bset):
    name = bset
    b = backend(name)
    r = b.ref
    rng = np.random.default_rng(15)
    count = 33
    a = rng.integers(0, r.q, (count, r.n), dtype=np.uint64)
    bb = rng.integers(0, r.q, count, dtype=np.uint64)
    ok = ctypes.c_int()
    b.chk(b.L.bh_pack_roundtrip(b.h, sz(count), P(a), P(bb), ctypes.byref(ok)))
    assert ok.value == 3, ok.value


@pytest.mark.gpu
@needs_backend
def test_gpu_backend_null_accumulators_and_bootstrapbatch(bset):
    name = bset
    """BlindRotateBatch with null accumulators (BootstrapBatch, batch.cpp:77-86) ==
    BootstrapGateCore(AND, ct + q/4); its extraction == the reference's Bootstrap(ct, true); and the
    reference's BootstrapBatch succeeds with BackendHIP as the default"""
    from fhe_amd import binfhe as bf
    b = backend(name)
    r = b.ref
    for count, seed in ((1, 21), (5, 22)):
        bits = np.random.default_rng(seed).integers(0, 2, count)
        a, bb = bf.encrypt(b.ps, b.m, b.sk, bits, 700 + seed)
        g = np.zeros((count, 2, r.N), np.uint64)
        ref = np.zeros_like(g)
        flags = ctypes.c_int()
        b.chk(b.L.bh_bootstrap_init(b.h, sz(count), P(a), P(bb), P(g), P(ref), ctypes.byref(flags)))
        assert flags.value == 3, (name, flags.value)
        assert np.array_equal(g, ref), (name, count)


@pytest.mark.gpu
@needs_backend
@pytest.mark.parametrize("bset", NOREF, indirect=True)
def test_gpu_backend_reference_batch_callers(bset):
    name = bset
    """lux::fhe::KeySwitchBatch / ModSwitchBatch (batch.cpp:251-314) through the registry == the
    reference's LWEEncryptionScheme::KeySwitch / ModSwitch"""
    b = backend(name)
    r = b.ref
    rng = np.random.default_rng(16)
    count = 7
    ka = rng.integers(0, r.qKS, (count, r.N), dtype=np.uint64)
    kb = rng.integers(0, r.qKS, count, dtype=np.uint64)
    ma = rng.integers(0, r.Q, (count, r.N), dtype=np.uint64)
    mb = rng.integers(0, r.Q, count, dtype=np.uint64)
    gka, gkb = np.zeros((count, r.n), np.uint64), np.zeros(count, np.uint64)
    rka, rkb = np.zeros_like(gka), np.zeros_like(gkb)
    gma, gmb = np.zeros_like(ma), np.zeros_like(mb)
    rma, rmb = np.zeros_like(ma), np.zeros_like(mb)
    ok = ctypes.c_int()
    b.chk(b.L.bh_batch_callers(b.h, sz(count), P(ka), P(kb), P(gka), P(gkb), P(rka), P(rkb), P(ma), P(mb), P(gma),
                               P(gmb), P(rma), P(rmb), ctypes.byref(ok)))
    assert ok.value == 1
    assert np.array_equal(gka, rka) and np.array_equal(gkb, rkb), name
    assert np.array_equal(gma, rma) and np.array_equal(gmb, rmb), name


@pytest.mark.gpu
@needs_backend
@pytest.mark.parametrize("bset", ["std128", "lmkcdey", "std128_3", "std192"], indirect=True)
def test_gpu_backend_routed_gate_batch_equals_reference(bset):
    name = bset
    """EvalBinGateBatchHIP (the routing INTEGRATION.md proposes for batch.cpp:176-210) with BackendHIP as the
    default == the reference's EvalBinGateBatch"""
    from fhe_amd import binfhe as bf
    b = backend(name)
    r = b.ref
    count = 9
    rng = np.random.default_rng(17)
    x1, x2 = rng.integers(0, 2, count), rng.integers(0, 2, count)
    a1, b1 = bf.encrypt(b.ps, b.m, b.sk, x1, 601)
    a2, b2 = bf.encrypt(b.ps, b.m, b.sk, x2, 602)
    for gate, truth in ((0, x1 | x2), (5, 1 - (x1 ^ x2))):
        ga, gb = np.zeros((count, r.n), np.uint64), np.zeros(count, np.uint64)
        ra, rb = np.zeros_like(ga), np.zeros_like(gb)
        ok = ctypes.c_int()
        b.chk(b.L.bh_eval_gates_routed(b.h, gate, sz(count), P(a1), P(b1), P(a2), P(b2), P(ga), P(gb), P(ra), P(rb),
                                       ctypes.byref(ok)))
        assert ok.value == 1
        assert np.array_equal(ga, ra) and np.array_equal(gb, rb), (name, gate)
        assert np.array_equal(bf.decrypt(b.ps, b.m, b.sk, ga, gb), truth), (name, gate)


# ---- the reference's other batch callers and its public C API, routed to the GPU ---------------------
ROUTED = ["std128", "lmkcdey", "std128_3"]


@needs_backend
def test_c_api_library_exports_the_reference_c_api():
    """integration/c_api_hip.cpp defines every function of the reference's include/lux/fhe/c_api.h (when the
    reference is present to read the header from) and the batch forms of integration/c_api_hip.h"""
    import re
    syms = dyn_symbols(BACKEND_SO)
    ours = open(os.path.join(ROOT, "integration", "c_api_hip.h")).read()
    want = set(re.findall(r"LUX_FHE_API[^;(]*?\b(lux_fhe_\w+)\s*\(", ours))
    hdr = "/root/reference/include/lux/fhe/c_api.h"
    if os.path.exists(hdr):
        want |= set(re.findall(r"LUX_FHE_API[^;(]*?\b(lux_fhe_\w+)\s*\(", open(hdr).read()))
        assert len(want) == 36, sorted(want)   # 33 of the reference + 3 batch forms
    assert want and not (want - syms), sorted(want - syms)


class CApi:
    """ctypes view of the C API in oracle/_ref/libbackend_hip.so (integration/c_api_hip.cpp)"""

    def __init__(self):
        L = ctypes.CDLL(BACKEND_SO)
        for f in ("lux_fhe_context_new", "lux_fhe_keygen_secret", "lux_fhe_keygen_bootstrap", "lux_fhe_encrypt",
                  "lux_fhe_decrypt", "lux_fhe_and", "lux_fhe_or", "lux_fhe_xor", "lux_fhe_nand", "lux_fhe_nor",
                  "lux_fhe_xnor", "lux_fhe_mux", "lux_fhe_bootstrap", "lux_fhe_gate_batch", "lux_fhe_mux_batch",
                  "lux_fhe_bootstrap_batch", "capi_ref_eval", "capi_ct_equal", "capi_on_gpu",
                  "lux_fhe_ciphertext_marshal", "lux_fhe_ciphertext_unmarshal"):
            getattr(L, f).restype = ctypes.c_int
        L.lux_fhe_context_n.restype = ctypes.c_uint32
        L.lux_fhe_context_ring_dim.restype = ctypes.c_uint32
        L.lux_fhe_context_modulus.restype = ctypes.c_uint64
        L.lux_fhe_strerror.restype = ctypes.c_char_p
        # pointer arguments as pointers (a bare Python int would be passed as a 32-bit int)
        L.lux_fhe_decrypt.argtypes = [vp, vp, vp, vp]
        L.lux_fhe_ciphertext_free.argtypes = [vp]
        L.capi_ct_equal.argtypes = [vp, vp]
        L.capi_ref_eval.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp]
        self.L = L

    def ok(self, rc):
        assert rc == 0, self.L.lux_fhe_strerror(rc).decode()


@needs_backend
def test_c_api_parameter_mapping_and_errors():
    """c_api.cpp:44-68: STD128 is STD128_LMKCDEY, so GINX / AP on it are incompatible
    (isMethodCompatible) and lux_fhe_context_new reports LUX_FHE_ERR_ALLOC; null pointers report
    LUX_FHE_ERR_NULL_PTR.  CPU only: no bootstrapped call is made."""
    C = CApi()
    ctx = vp()
    C.ok(C.L.lux_fhe_context_new(ctypes.byref(ctx), 2, 2))          # STD128 x LMKCDEY
    assert (C.L.lux_fhe_context_n(ctx), C.L.lux_fhe_context_ring_dim(ctx), C.L.lux_fhe_context_modulus(ctx)) == \
        (447, 1024, 2048)
    assert C.L.capi_on_gpu(ctx) == 0                                    # the device context comes with the gates
    other = vp()
    assert C.L.lux_fhe_context_new(ctypes.byref(other), 2, 1) == -3   # STD128 x GINX
    assert C.L.lux_fhe_context_new(None, 2, 2) == -1
    bsk = vp()
    assert C.L.lux_fhe_and(ctx, bsk, None, None, ctypes.byref(vp())) == -1
    C.L.lux_fhe_context_free(ctx)


@pytest.mark.gpu
@needs_backend
@pytest.mark.parametrize("bset", ROUTED, indirect=True)
def test_gpu_backend_routed_eval_func_batches(bset):
    """EvalFuncBatchHIP / EvalFuncMultiOutputBatchHIP (BackendHIP as the default) == the reference's
    EvalFuncBatch / EvalFuncMultiOutputBatch (batch.cpp:106-174) on uniformly random ciphertexts mod q,
    for the negacyclic, periodic and (q <= N) arbitrary LUTs GenerateLUTviaFunction builds"""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_golden import fb_luts
    name = bset
    b = backend(name)
    r = b.ref
    luts = np.stack(list(fb_luts(r.q, r.q // 256 if r.q >= 512 else 2, r.N).values())).astype(np.uint64)
    L = luts.shape[0]
    rng = np.random.default_rng(31)
    for count in (1, 7):
        a = rng.integers(0, r.q, (count, r.n), dtype=np.uint64)
        bb = rng.integers(0, r.q, count, dtype=np.uint64)
        for multi in (0, 1):
            ga, gb = np.zeros((L * count, r.n), np.uint64), np.zeros(L * count, np.uint64)
            ra, rb = np.zeros_like(ga), np.zeros_like(gb)
            ok = ctypes.c_int()
            b.chk(b.L.bh_eval_func_routed(b.h, multi, sz(count), P(a), P(bb), u64(r.q), P(luts), sz(L),
                                          sz(r.q), P(ga), P(gb), P(ra), P(rb), ctypes.byref(ok)))
            assert ok.value == 1, (name, multi)
            assert np.array_equal(ga, ra) and np.array_equal(gb, rb), (name, count, multi)


@pytest.mark.gpu
@needs_backend
@pytest.mark.parametrize("bset", ROUTED, indirect=True)
def test_gpu_backend_routed_cmux_and_refresh(bset):
    """EvalCMUXBatchHIP == the reference's EvalCMUXBatch (batch.cpp:212-249; rows {sel, true, false} as it
    passes them, so the result is false ? true : sel), and BackendHIP::RefreshBatch == BinFHEContext::
    Bootstrap, on every input combination"""
    from fhe_amd import binfhe as bf
    name = bset
    b = backend(name)
    r = b.ref
    bits = np.array([[x >> 2 & 1, x >> 1 & 1, x & 1] for x in range(8)] * 2)
    count = len(bits)
    cts = [bf.encrypt(b.ps, b.m, b.sk, bits[:, j], 811 + j) for j in range(3)]
    ga, gb = np.zeros((count, r.n), np.uint64), np.zeros(count, np.uint64)
    ra, rb = np.zeros_like(ga), np.zeros_like(gb)
    ok = ctypes.c_int()
    b.chk(b.L.bh_eval_cmux_routed(b.h, sz(count), P(cts[0][0]), P(cts[0][1]), P(cts[1][0]), P(cts[1][1]),
                                  P(cts[2][0]), P(cts[2][1]), P(ga), P(gb), P(ra), P(rb), ctypes.byref(ok)))
    assert ok.value == 1
    assert np.array_equal(ga, ra) and np.array_equal(gb, rb), name
    want = np.where(bits[:, 2] == 1, bits[:, 1], bits[:, 0])
    assert np.array_equal(bf.decrypt(b.ps, b.m, b.sk, ga, gb), want), name
    ga, gb = np.zeros((count, r.n), np.uint64), np.zeros(count, np.uint64)
    ra, rb = np.zeros_like(ga), np.zeros_like(gb)
    b.chk(b.L.bh_refresh(b.h, sz(count), P(cts[0][0]), P(cts[0][1]), P(ga), P(gb), P(ra), P(rb)))
    assert np.array_equal(ga, ra) and np.array_equal(gb, rb), name
    assert np.array_equal(bf.decrypt(b.ps, b.m, b.sk, ga, gb), bits[:, 0]), name


@pytest.mark.gpu
@needs_backend
@pytest.mark.parametrize("bset", ROUTED, indirect=True)
def test_gpu_backend_routed_inputs_mod_Q(bset):
    """Ciphertexts mod Q (dimension N: extended outputs, LARGE_DIM encryptions) mixed with ones mod q in one
    batch through the routed callers: EvalBinGateBatchHIP (every 2-input gate), EvalCMUXBatchHIP and
    BackendHIP::RefreshBatch (plaintext moduli 4 and 8) == the reference's EvalBinGateBatch / EvalCMUXBatch /
    Bootstrap, which switch those inputs first (binfhe-base-scheme.cpp:92-93, 180-182, 200-201)"""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_golden import mixed_column
    from fhe_amd import binfhe as bf
    name = bset
    b = backend(name)
    r = b.ref
    skN = bf.keygen_ring_secret(b.ps, b.m, 0xB0070000 + b.ps)
    rng = np.random.default_rng(47)
    count = 12

    def run(op, k, p):
        bits = rng.integers(0, 2, (k, count))
        fl = rng.integers(0, 2, (k, count)).astype(np.uint8)
        fl[:, 0], fl[:, 1] = 1, 0
        cols = [mixed_column(b.ps, b.m, b.sk, skN, bits[j], fl[j], 900 + 10 * k + j, p) for j in range(k)]
        A = [c[0] for c in cols]
        B = [c[1] for c in cols]
        ptr = lambda xs: (vp * k)(*[x.ctypes.data for x in xs])   # noqa: E731
        ga, gb = np.zeros((count, r.n), np.uint64), np.zeros(count, np.uint64)
        ra, rb = np.zeros_like(ga), np.zeros_like(gb)
        ok = ctypes.c_int()
        b.chk(b.L.bh_eval_mixed_routed(b.h, op, k, p, sz(count), ptr(A), ptr(B), ptr(list(fl)), P(ga), P(gb), P(ra),
                                       P(rb), ctypes.byref(ok)))
        assert ok.value == 1, (name, op)
        assert np.array_equal(ga, ra) and np.array_equal(gb, rb), (name, op, p)
        return bits, fl, ga, gb

    for gate in range(6):
        run(gate, 2, 4)
    bits, fl, ga, gb = run(13, 3, 4)
    assert np.array_equal(bf.decrypt(b.ps, b.m, b.sk, ga, gb), np.where(bits[2] == 1, bits[1], bits[0])), name
    for p in (4, 8):   # p = 8: the reference's window stays p = 4's (:205), only b uses p (:210): parity only
        bits, fl, ga, gb = run(-1, 1, p)
        small = fl[0] == 0
        if p == 4:
            assert np.array_equal(bf.decrypt(b.ps, b.m, b.sk, ga, gb)[small], bits[0][small]), name


@pytest.mark.gpu
@needs_backend
@pytest.mark.parametrize("params", [2, 0])    # LUX_FHE_PARAMS_STD128 (= STD128_LMKCDEY), TOY
def test_gpu_c_api_gates_mux_bootstrap_vs_reference(params):
    """The reference's public C API (c_api.h) over the GPU: every gate, lux_fhe_mux and lux_fhe_bootstrap
    (single and batch forms) == the reference's own cc.EvalBinGate / EvalBinGate(CMUX, ..) / Bootstrap on
    the same context, keys (the reference's BTKeyGen) and ciphertexts, and decrypt to the truth tables"""
    for bname in list(_backends):      # one registry default at a time: release the seam tests' backend
        _backends.pop(bname).close()
    C = CApi()
    L = C.L
    ctx, sk, bsk = vp(), vp(), vp()
    C.ok(L.lux_fhe_context_new(ctypes.byref(ctx), params, 2))
    C.ok(L.lux_fhe_keygen_secret(ctx, ctypes.byref(sk)))
    C.ok(L.lux_fhe_keygen_bootstrap(ctx, sk, ctypes.byref(bsk)))
    bits = np.array([[x >> 2 & 1, x >> 1 & 1, x & 1] for x in range(8)])
    cts = [[vp() for _ in range(8)] for _ in range(3)]
    for j in range(3):
        for i in range(8):
            C.ok(L.lux_fhe_encrypt(ctx, sk, ctypes.c_bool(bool(bits[i, j])), ctypes.byref(cts[j][i])))

    def dec(ct):
        v = ctypes.c_bool()
        C.ok(L.lux_fhe_decrypt(ctx, sk, ct, ctypes.byref(v)))
        return int(v.value)

    def same_as_ref(out, code, x, y=None, z=None):
        ref = vp()
        assert L.capi_ref_eval(ctx, code, x, y, z, ctypes.byref(ref)) == 0
        assert L.capi_ct_equal(out, ref) == 1, code
        L.lux_fhe_ciphertext_free(ref)

    gates = {"or": (0, lambda x, y: x | y), "and": (1, lambda x, y: x & y), "nor": (2, lambda x, y: 1 - (x | y)),
             "nand": (3, lambda x, y: 1 - (x & y)), "xor": (4, lambda x, y: x ^ y), "xnor": (5, lambda x, y: 1 - (x ^ y))}
    for gname, (code, f) in gates.items():
        fn = getattr(L, f"lux_fhe_{gname}")
        for i in (0, 3, 5, 6):
            out = vp()
            C.ok(fn(ctx, bsk, cts[0][i], cts[1][i], ctypes.byref(out)))
            assert dec(out) == f(bits[i, 0], bits[i, 1]), (gname, i)
            same_as_ref(out, code, cts[0][i], cts[1][i])
            L.lux_fhe_ciphertext_free(out)
        arr = (vp * 8)
        outs = arr()
        C.ok(L.lux_fhe_gate_batch(ctx, bsk, code, arr(*cts[0]), arr(*cts[1]), sz(8), outs))
        for i in range(8):
            assert dec(vp(outs[i])) == f(bits[i, 0], bits[i, 1]), (gname, i)
            same_as_ref(vp(outs[i]), code, cts[0][i], cts[1][i])
            L.lux_fhe_ciphertext_free(vp(outs[i]))
    assert L.capi_on_gpu(ctx) == 1
    arr = (vp * 8)
    outs = arr()
    C.ok(L.lux_fhe_mux_batch(ctx, bsk, arr(*cts[0]), arr(*cts[1]), arr(*cts[2]), sz(8), outs))
    for i in range(8):   # EvalBinGate(CMUX, {sel, a, b}) = b ? a : sel
        assert dec(vp(outs[i])) == (bits[i, 1] if bits[i, 2] else bits[i, 0]), i
        same_as_ref(vp(outs[i]), 6, cts[0][i], cts[1][i], cts[2][i])
        L.lux_fhe_ciphertext_free(vp(outs[i]))
    one = vp()
    C.ok(L.lux_fhe_mux(ctx, bsk, cts[0][5], cts[1][5], cts[2][5], ctypes.byref(one)))
    same_as_ref(one, 6, cts[0][5], cts[1][5], cts[2][5])
    C.ok(L.lux_fhe_bootstrap_batch(ctx, bsk, arr(*cts[0]), sz(8), outs))
    for i in range(8):
        assert dec(vp(outs[i])) == bits[i, 0], i
        same_as_ref(vp(outs[i]), 7, cts[0][i])
        L.lux_fhe_ciphertext_free(vp(outs[i]))
    C.ok(L.lux_fhe_bootstrap(ctx, bsk, cts[1][6], ctypes.byref(one)))
    same_as_ref(one, 7, cts[1][6])
    # a bootstrap key that was never generated: LUX_FHE_ERR_NOT_INIT, nothing evaluated
    fake = ctypes.create_string_buffer(8)
    assert L.lux_fhe_and(ctx, fake, cts[0][0], cts[1][0], ctypes.byref(vp())) == -11
    for j in range(3):
        for i in range(8):
            L.lux_fhe_ciphertext_free(cts[j][i])
    L.lux_fhe_bootstrapkey_free(bsk)
    L.lux_fhe_secretkey_free(sk)
    L.lux_fhe_context_free(ctx)
