"""Key switch alone (K2: KeySwitch + ModSwitch of the workspace the blind rotation left), STD128 GINX:
one blind rotation of B gates, then `reps` key switches of its workspace timed with a device sync
around them; the outputs are decrypted and hashed (variants must agree).

  python tools/ks_time.py [B] [reps]
"""
import ctypes
import hashlib
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from fhe_amd import binfhe as bf  # noqa: E402
from fhe_amd._lib import check, lib, ptr, vp  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ps, m = bf.STD128, bf.GINX
keys = bf.keygen(ps, m, 1234)
e = bf.GateEngine(ps, m)
e.load_keys(keys.bsk, keys.kskA, keys.kskB)
P = e.params
rng = np.random.default_rng(B)
x1, x2 = rng.integers(0, 2, B), rng.integers(0, 2, B)
a1, b1 = bf.encrypt(ps, m, keys.sk, x1, 7)
a2, b2 = bf.encrypt(ps, m, keys.sk, x2, 8)


def dalloc(nbytes):
    d = vp()
    check(lib().fhe_hip_alloc(0, nbytes, ctypes.byref(d)))
    return d.value


bufs = [dalloc(x.nbytes) for x in (a1, b1, a2, b2)]
for d, x in zip(bufs, (a1, b1, a2, b2)):
    check(lib().fhe_hip_copy_to_device(vp(d), ptr(x), x.nbytes))
dao, dbo = dalloc(B * P.n * 8), dalloc(B * 8)
e.blind_rotate_device(bf.AND, B, *bufs)
e.keyswitch_workspace_device(B, dao, dbo)
check(lib().fhe_hip_synchronize(0))
t = time.perf_counter()
for _ in range(reps):
    e.keyswitch_workspace_device(B, dao, dbo)
check(lib().fhe_hip_synchronize(0))
ms = (time.perf_counter() - t) / reps * 1e3
ao = np.zeros((B, P.n), np.uint64)
bo = np.zeros(B, np.uint64)
check(lib().fhe_hip_copy_to_host(ptr(ao), vp(dao), ao.nbytes))
check(lib().fhe_hip_copy_to_host(ptr(bo), vp(dbo), bo.nbytes))
ok = np.array_equal(bf.decrypt(ps, m, keys.sk, ao, bo), (x1 & x2).astype(np.int64))
h = hashlib.sha256(ao.tobytes() + bo.tobytes()).hexdigest()[:16]
print(f"B={B}: keyswitch {ms:.3f} ms  correct={ok} sha={h}", flush=True)
