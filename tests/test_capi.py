"""C-ABI: the library loads and exports every symbol include/fhe_hip.h declares
(no compute call, so this runs without a GPU)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "fhe_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fhe_hip_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "fhe_hip_ntt_batch" in syms and len(syms) >= 10


def test_library_exports_every_declared_symbol():
    from fhe_amd import lib_path
    assert os.path.exists(lib_path), "run fhe_amd.build.build() first"
    L = ctypes.CDLL(lib_path)
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing


def test_product_does_not_reference_oracle():
    """the product path never links/calls the oracle (oracle/ is test-only)."""
    for d, _, files in os.walk(os.path.join(ROOT, "fhe_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h", "Makefile")):
                txt = open(os.path.join(d, f), errors="ignore").read()
                assert "tfhe_oracle" not in txt and "libfhe_ref" not in txt and "oracle_lib" not in txt, f


def test_kernel_path_per_parameter_set():
    """fhe_hip_params.kernel names the accumulator the engine picks (Engine::fast_path / g3_set /
    narrow_set): no GPU needed, the parameter table is host data"""
    from fhe_amd import binfhe as bf
    STD128_3, STD192, STD256 = 4, 9, 15   # binfhe-constants.h:49-89
    assert bf.kernel_path(bf.STD128, bf.GINX) == 1
    assert bf.kernel_path(bf.STD128_LMKCDEY, bf.LMKCDEY) == 1
    assert bf.kernel_path(STD128_3, bf.GINX) == 2
    assert bf.kernel_path(STD256, bf.GINX) == 4       # N = 2048, 29-bit Q, q = 2048: K1w, forward reduced 3x
    assert bf.kernel_path(16, bf.GINX) == 4           # STD256_3 (3 retained digits)
    assert bf.kernel_path(17, bf.GINX) == 4           # STD256_4: q = 2N, the full-resolution monomials
    assert bf.kernel_path(19, bf.GINX) == 4           # STD256Q_3: q = 2N, 4 retained digits
    assert bf.kernel_path(20, bf.GINX) == 4           # STD256Q_4
    assert bf.kernel_path(STD192, bf.GINX) == 0       # 37-bit Q: 64-bit residues
    assert bf.kernel_path(18, bf.GINX) == 4           # STD256Q: K1w (N = 2048, accumulator in registers)
    assert bf.kernel_path(37, bf.LMKCDEY) == 4        # STD256Q_3_LMKCDEY: K1w's LMKCDEY form
    assert bf.kernel_path(36, bf.LMKCDEY) == 4        # STD256Q_LMKCDEY (28-bit Q, 2 digits): the C API's STD256Q
    assert bf.kernel_path(38, bf.LMKCDEY) == 4        # STD256Q_4_LMKCDEY (4 retained digits): K1w
    assert bf.kernel_path(33, bf.LMKCDEY) == 3        # STD256_LMKCDEY (30-bit Q): K5 A32
    assert bf.kernel_path(34, bf.LMKCDEY) == 4        # STD256_3_LMKCDEY (29-bit Q, 3 digits): K1w, forward reduced 3x
    assert bf.kernel_path(35, bf.LMKCDEY) == 4        # STD256_4_LMKCDEY (29-bit Q, 3 digits)
    assert bf.uses_fast_kernels(bf.STD128, bf.GINX) and not bf.uses_fast_kernels(STD256, bf.GINX)


def test_no_stream_ordered_pool_allocations():
    """Round 4's zero read-back ("A block read back as zeros"): a seam call's device scratch came
    from the stream-ordered pool (hipMallocAsync / hipFreeAsync per call), whose default release threshold
    of 0 lets a stream / event synchronize hand pool memory back to the driver.  No product code uses that
    allocator now: every device buffer is a hipMalloc'd, context-owned, grow-only allocation freed only after
    the context's streams are synchronised (Engine::grow / ensure_work, fhe_hip_ctx::scratch)."""
    import subprocess
    from fhe_amd import lib_path
    und = subprocess.run(["nm", "-D", "--undefined-only", lib_path], capture_output=True, text=True,
                         check=True).stdout
    assert "hipMallocAsync" not in und and "hipFreeAsync" not in und and "hipMallocFromPoolAsync" not in und
    for d in ("fhe_amd/csrc", "integration"):
        for f in os.listdir(os.path.join(ROOT, d)):
            if f.endswith((".cpp", ".hip", ".h")):
                txt = re.sub(r"//.*", "", open(os.path.join(ROOT, d, f)).read())
                assert "hipMallocAsync" not in txt and "hipFreeAsync" not in txt, f


import numpy as np  # noqa: E402
import pytest  # noqa: E402


@pytest.mark.gpu
@pytest.mark.parametrize("ps,m", [(27, 3), (3, 2)])   # STD192_LMKCDEY (where r04 saw the zeros), STD128 GINX
def test_gpu_seam_call_sequence_repeats_on_one_context(ps, m):
    """the host-buffer seam calls (ExternalProduct, BlindRotate, BlindRotate with null accumulators, gates,
    SwitchCTtoqn) interleaved three times on ONE context, each call's output equal to its first run: the
    sequence that read a block back as zeros in round 4 (test_backend's std192_lmkcdey null accumulators)"""
    from fhe_amd import binfhe as bf
    from fhe_amd._lib import check, ptr
    L = bf.L()
    L.fhe_hip_blind_rotate_init_batch.argtypes = [ctypes.c_void_p, ctypes.c_size_t] + [ctypes.c_void_p] * 3
    keys = bf.keygen(ps, m, 0xB0070000 + ps)
    P = bf.params(ps, m)
    e = bf.GateEngine(ps, m, 0)
    e.load_keys(keys.bsk, keys.kskA, keys.kskB)
    rng = np.random.default_rng(5)
    bits = rng.integers(0, 2, 5)
    a, b = bf.encrypt(ps, m, keys.sk, bits, 3)
    amod = 2 * P.N if m == 3 else P.q
    acc_a = rng.integers(0, amod, (5, P.n), dtype=np.uint64)
    acc = rng.integers(0, P.Q, (5, 2, P.N), dtype=np.uint64)
    rgsw = rng.integers(0, P.Q, (3, 2 * (P.digitsG - 1), 2, P.N), dtype=np.uint64)
    rlwe = rng.integers(0, P.Q, (3, 2, P.N), dtype=np.uint64)
    skN = bf.keygen_ring_secret(ps, m, 0xB0070000 + ps)
    la, lb = bf.encrypt_large(ps, m, skN, bits, 4)

    def init(cnt):
        out = np.zeros((cnt, 2, P.N), np.uint64)
        check(L.fhe_hip_blind_rotate_init_batch(e._h, cnt, ptr(a[:cnt].copy()), ptr(b[:cnt].copy()), ptr(out)))
        return out

    def round_():
        return [e.external_product(rgsw, rlwe), e.blind_rotate_acc(acc_a, amod, acc), init(1), init(5),
                e.eval_gate(bf.AND, a, b, a[::-1].copy(), b[::-1].copy()), init(1), e.switch_to_qn(la, lb)]

    first = round_()
    assert np.any(first[2] != 0) and np.any(first[3] != 0)
    for _ in range(2):
        for x, y in zip(round_(), first):
            for u, v in zip(x if isinstance(x, tuple) else (x,), y if isinstance(y, tuple) else (y,)):
                assert np.array_equal(u, v)
    e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("ps,m", [(3, 2), (21, 3), (9, 2), (18, 2), (37, 3)])
def test_gpu_copy_keys_fan_out_matches_host_load(ps, m):
    """fhe_hip_copy_keys (MultiEngine's key fan-out): a context that received another context's resident keys
    device to device computes the same gates as one that packed the host keys itself (STD128, STD128_LMKCDEY,
    the 64-bit STD192, the K1w STD256Q / STD256Q_3_LMKCDEY layouts)"""
    from fhe_amd import binfhe as bf
    from fhe_amd._lib import check
    L = bf.L()
    L.fhe_hip_copy_keys.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    keys = bf.keygen(ps, m, 0xB0070000 + ps)
    a1, b1 = bf.encrypt(ps, m, keys.sk, np.arange(37) % 2, 1)
    a2, b2 = bf.encrypt(ps, m, keys.sk, np.arange(37) // 2 % 2, 2)
    src = bf.GateEngine(ps, m, 0)
    src.load_keys(keys.bsk, keys.kskA, keys.kskB)
    dst = bf.GateEngine(ps, m, 0)
    check(L.fhe_hip_copy_keys(dst._h, src._h))
    for gate in (bf.AND, bf.XOR):
        ra, rb = src.eval_gate(gate, a1, b1, a2, b2)
        ga, gb = dst.eval_gate(gate, a1, b1, a2, b2)
        assert np.array_equal(ra, ga) and np.array_equal(rb, gb), gate
    other = bf.GateEngine(3 if ps != 3 else 21, 2 if ps != 3 else 3, 0)
    assert L.fhe_hip_copy_keys(other._h, src._h) == -2   # another parameter set
    for e in (src, dst, other):
        e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("ps,m,knob,val", [(3, 2, "FHE_HIP_GINX_KERNEL", "wave"), (0, 2, "FHE_HIP_NARROW", "0")])
def test_gpu_copy_keys_refuses_contexts_of_other_kernel_layouts(ps, m, knob, val, monkeypatch):
    """contexts created under different FHE_HIP_* kernel settings pack their keys in different layouts (STD128:
    the two-wave kernels' repacked BSK or none; TOY: u32 or u64 words of the 64-bit-path BSK): fhe_hip_copy_keys
    refuses the pair with FHE_HIP_ERR_INVALID_PARAM instead of handing a kernel a buffer of another layout; the
    contexts' own kernel fields differ accordingly where the knob changes the accumulator (TOY)"""
    from fhe_amd import binfhe as bf
    from fhe_amd._lib import check
    L = bf.L()
    keys = bf.keygen(ps, m, 0xB0070000 + ps)
    src = bf.GateEngine(ps, m, 0)
    src.load_keys(keys.bsk, keys.kskA, keys.kskB)
    monkeypatch.setenv(knob, val)
    dst = bf.GateEngine(ps, m, 0)
    monkeypatch.delenv(knob)
    assert L.fhe_hip_copy_keys(dst._h, src._h) == -2
    assert "different layouts" in L.fhe_hip_last_error().decode()
    same = bf.GateEngine(ps, m, 0)
    check(L.fhe_hip_copy_keys(same._h, src._h))
    if knob == "FHE_HIP_NARROW":
        assert (src.kernel(), dst.kernel()) == (3, 0)
    for e in (src, dst, same):
        e.close()


@pytest.mark.gpu
def test_gpu_gate_kernel_reports_the_launched_kernel(monkeypatch):
    """fhe_hip_gate_kernel: the STD128 GINX context runs K1q (k_blind_rotate_ginx4x, four waves per gate) up to one
    gate per CU, K1x (k_blind_rotate_ginx2x) up to two and K1 above; FHE_HIP_GINX_KERNEL pins it; LMKCDEY runs
    K1m-4 (k_blind_rotate_lmk4x) up to one gate per CU, K1m's two-digit form (k_blind_rotate_lmk3) up to two and
    its op-list kernel above"""
    from fhe_amd import binfhe as bf
    keys = bf.keygen(bf.STD128, bf.GINX, 5)
    e = bf.GateEngine(bf.STD128, bf.GINX, 0)
    e.load_keys(keys.bsk, keys.kskA, keys.kskB)
    assert e.gate_kernel(1) == "k_blind_rotate_ginx4x" and e.gate_kernel(65536) == "k_blind_rotate_ginx"

    def switch(k, kernels):  # the last count launching one of `kernels`
        lo, hi = 1, 65536
        while hi - lo > 1:
            mid = (lo + hi) // 2
            lo, hi = (mid, hi) if k.gate_kernel(mid) in kernels else (lo, mid)
        return lo
    q = switch(e, ("k_blind_rotate_ginx4x",))
    x = switch(e, ("k_blind_rotate_ginx4x", "k_blind_rotate_ginx2x"))
    assert 64 <= q <= 512 and x == 2 * q and e.gate_kernel(q + 1) == "k_blind_rotate_ginx2x", (q, x)   # CUs, 2 x CUs
    assert e.kernel() == 1
    for val, name in (("wave", "k_blind_rotate_ginx"), ("split", "k_blind_rotate_ginx2"), ("xsplit", "k_blind_rotate_ginx2x"),
                      ("qsplit", "k_blind_rotate_ginx4x")):
        monkeypatch.setenv("FHE_HIP_GINX_KERNEL", val)
        p = bf.GateEngine(bf.STD128, bf.GINX, 0)
        p.load_keys(keys.bsk, keys.kskA, keys.kskB)
        assert p.gate_kernel(4096) == name, val
        p.close()
    monkeypatch.delenv("FHE_HIP_GINX_KERNEL")
    lk = bf.keygen(bf.STD128_LMKCDEY, bf.LMKCDEY, 5)
    l = bf.GateEngine(bf.STD128_LMKCDEY, bf.LMKCDEY, 0)
    l.load_keys(lk.bsk, lk.kskA, lk.kskB)
    assert l.gate_kernel(1024) == "k_blind_rotate_lmk" and l.gate_kernel(1) == "k_blind_rotate_lmk4x"
    assert switch(l, ("k_blind_rotate_lmk4x",)) == q and switch(l, ("k_blind_rotate_lmk4x", "k_blind_rotate_lmk3")) == x
    for x in (e, l):
        x.close()
