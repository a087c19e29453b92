"""Quick device-resident gate-bootstrap timing (wall clock around device launches)."""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from fhe_amd import binfhe as bf  # noqa: E402
from fhe_amd._lib import check, lib, ptr, vp  # noqa: E402

SETS = {"ginx": (bf.STD128, bf.GINX), "lmk": (bf.STD128_LMKCDEY, bf.LMKCDEY), "ap": (bf.STD128_AP, bf.AP)}
ps, m = SETS[sys.argv[1] if len(sys.argv) > 1 else "ginx"]
batches = [int(x) for x in sys.argv[2:]] or [1024, 8192]
t0 = time.time()
keys = bf.keygen(ps, m, 1234)
print(f"keygen {time.time()-t0:.1f}s", flush=True)
e = bf.GateEngine(ps, m)
t0 = time.time()
e.load_keys(keys.bsk, keys.kskA, keys.kskB)
print(f"load {time.time()-t0:.1f}s", flush=True)
P = e.params


def dalloc(nbytes):
    d = vp()
    check(lib().fhe_hip_alloc(0, nbytes, ctypes.byref(d)))
    return d.value


for B in batches:
    rng = np.random.default_rng(B)
    x1, x2 = rng.integers(0, 2, B), rng.integers(0, 2, B)
    a1, b1 = bf.encrypt(ps, m, keys.sk, x1, 7)
    a2, b2 = bf.encrypt(ps, m, keys.sk, x2, 8)
    bufs = [dalloc(x.nbytes) for x in (a1, b1, a2, b2)]
    for d, x in zip(bufs, (a1, b1, a2, b2)):
        check(lib().fhe_hip_copy_to_device(vp(d), ptr(x), x.nbytes))
    dao, dbo = dalloc(B * P.n * 8), dalloc(B * 8)
    e.eval_gate_device(bf.AND, B, *bufs, dao, dbo)
    check(lib().fhe_hip_synchronize(0))
    reps = 3
    t = time.perf_counter()
    for _ in range(reps):
        e.eval_gate_device(bf.AND, B, *bufs, dao, dbo)
    check(lib().fhe_hip_synchronize(0))
    dt = (time.perf_counter() - t) / reps
    ao = np.zeros((B, P.n), np.uint64)
    bo = np.zeros(B, np.uint64)
    check(lib().fhe_hip_copy_to_host(ptr(ao), vp(dao), ao.nbytes))
    check(lib().fhe_hip_copy_to_host(ptr(bo), vp(dbo), bo.nbytes))
    dec = bf.decrypt(ps, m, keys.sk, ao, bo)
    ok = np.array_equal(dec, (x1 & x2).astype(np.int64))
    print(f"B={B}: {dt*1e3:.2f} ms/batch  {B/dt:.0f} gates/s  correct={ok}", flush=True)
    for d in bufs + [dao, dbo]:
        check(lib().fhe_hip_free(vp(d)))
