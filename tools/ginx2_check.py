"""Split-kernel check: STD128 GINX gates through k_blind_rotate_ginx2 (FHE_HIP_GINX_KERNEL=split) vs
the one-wave kernel and the reference goldens, then timing of both kernels at a few batch sizes."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
sys.path.insert(0, "tests/golden")
from fhe_amd import binfhe as bf  # noqa: E402


def engine(kind, ps, m, keys):
    os.environ["FHE_HIP_GINX_KERNEL"] = kind
    e = bf.GateEngine(ps, m)
    e.load_keys(keys.bsk, keys.kskA, keys.kskB)
    return e


from make_golden import gate_inputs  # noqa: E402
g = np.load("tests/golden/gates_std128.npz")
keys, bits1, bits2, a1, b1, a2, b2 = gate_inputs(3, 2, int(g["key_seed"]))
es, ew = engine("split", 3, 2, keys), engine("wave", 3, 2, keys)
ok = True
for i, gate in enumerate(g["gates"]):
    sl = slice(i * 8, (i + 1) * 8)
    ao, bo = es.eval_gate(int(gate), a1[sl], b1[sl], a2[sl], b2[sl])
    good = np.array_equal(ao, g["out_a"][sl].astype(np.uint64)) and np.array_equal(bo, g["out_b"][sl].astype(np.uint64))
    ok &= good
    print("gate", int(gate), "split == reference:", good, flush=True)
rng = np.random.default_rng(5)
for B in (1, 7, 1024, 3000):
    x1, x2 = rng.integers(0, 2, B), rng.integers(0, 2, B)
    c1, d1 = bf.encrypt(3, 2, keys.sk, x1, 11 + B)
    c2, d2 = bf.encrypt(3, 2, keys.sk, x2, 12 + B)
    sa, sb = es.eval_gate(1, c1, d1, c2, d2)
    wa, wb = ew.eval_gate(1, c1, d1, c2, d2)
    same = np.array_equal(sa, wa) and np.array_equal(sb, wb)
    ok &= same
    print("B", B, "split == wave:", same, flush=True)
print("ALL OK" if ok else "MISMATCH", flush=True)
