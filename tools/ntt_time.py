"""Quick device-resident NTT timing (wall clock over many launches)."""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from fhe_amd import NttPlan  # noqa: E402
from fhe_amd._lib import check, lib, ptr, vp  # noqa: E402

count = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200
oop = len(sys.argv) > 3 and sys.argv[3] == "oop"      # out-of-place (separate output buffer)
qs = [int(q) for q in sys.argv[4].split(",")] if len(sys.argv) > 4 else [134215681, 1152921504606830593]
for Q in qs:
    plan = NttPlan(Q)
    x = np.random.default_rng(1).integers(0, Q, size=(count, 1024), dtype=np.uint64)
    d = vp()
    check(lib().fhe_hip_alloc(0, x.nbytes, ctypes.byref(d)))
    check(lib().fhe_hip_copy_to_device(d, ptr(x), x.nbytes))
    o = vp()
    check(lib().fhe_hip_alloc(0, x.nbytes, ctypes.byref(o)))
    dst = o.value if oop else d.value
    for inv in (0, 1):
        for _ in range(5):
            plan.run_device(d.value, dst, count, inv)
        check(lib().fhe_hip_synchronize(0))
        t = time.perf_counter()
        for _ in range(iters):
            plan.run_device(d.value, dst, count, inv)
        check(lib().fhe_hip_synchronize(0))
        dt = (time.perf_counter() - t) / iters
        print(f"{'oop' if oop else 'ip'} Q={Q} inv={inv} count={count}: {dt*1e6:.2f} us/pass  {2*x.nbytes/dt/1e9:.1f} GB/s")
    check(lib().fhe_hip_free(d))
    check(lib().fhe_hip_free(o))
