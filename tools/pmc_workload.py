"""GPU workload for rocprofv3 --pmc passes (tools/pmc_run.sh): one STD128 GINX and one
STD128_LMKCDEY AND batch of B gates (device-resident, as bench.py runs them), and 4096-polynomial
forward + inverse NTT passes for the STD128 modulus (k_ntt1024w) and the 60-bit prime (k_ntt1024w64)."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, ".")
from fhe_amd import NttPlan  # noqa: E402
from fhe_amd import binfhe as bf  # noqa: E402
from fhe_amd._lib import check, lib, ptr, vp  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
NTT = not (len(sys.argv) > 2 and sys.argv[2] == "nontt")   # "nontt": the gate batches only


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

for Q in ((134215681, 1152921504606830593) if NTT else ()):
    plan = NttPlan(Q)
    xs = np.random.default_rng(2).integers(0, Q, size=(4096, 1024), dtype=np.uint64)
    dx = dalloc(xs)
    for inv in (False, True):
        for _ in range(3):
            plan.run_device(dx, dx, 4096, inv)
    check(lib().fhe_hip_synchronize(0))
    plan.close()
print("pmc workload done")
