"""GPU workload for rocprofv3 --pmc passes: one STD128 GINX gate batch, one LMKCDEY
batch and a 4096-polynomial NTT pass (device-resident)."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, ".")
from fhe_amd import NttPlan  # noqa: E402
from fhe_amd import binfhe as bf  # noqa: E402
from fhe_amd._lib import check, lib, ptr, vp  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192


def dalloc(x):
    d = vp()
    check(lib().fhe_hip_alloc(0, x.nbytes, ctypes.byref(d)))
    check(lib().fhe_hip_copy_to_device(d, ptr(x), x.nbytes))
    return d.value


for ps, m in ((bf.STD128, bf.GINX), (bf.STD128_LMKCDEY, bf.LMKCDEY)):
    keys = bf.keygen(ps, m, 99)
    e = bf.GateEngine(ps, m)
    e.load_keys(keys.bsk, keys.kskA, keys.kskB)
    x = np.random.default_rng(1).integers(0, 2, B)
    a1, b1 = bf.encrypt(ps, m, keys.sk, x, 1)
    a2, b2 = bf.encrypt(ps, m, keys.sk, x, 2)
    d = [dalloc(v) for v in (a1, b1, a2, b2)]
    ao = dalloc(np.zeros((B, e.params.n), np.uint64))
    bo = dalloc(np.zeros(B, np.uint64))
    e.eval_gate_device(bf.AND, B, *d, ao, bo)
    check(lib().fhe_hip_synchronize(0))
    e.close()

Q = 134215681
plan = NttPlan(Q)
xs = np.random.default_rng(2).integers(0, Q, size=(4096, 1024), dtype=np.uint64)
dx = dalloc(xs)
for _ in range(3):
    plan.run_device(dx, dx, 4096, False)
check(lib().fhe_hip_synchronize(0))
print("pmc workload done")
