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
