"""Gate-bootstrap throughput of the other parameter sets on one GPU (device-resident AND batches,
wall time around eval_gate_device, reps reported individually to expose launch-time spread).
usage: python tools/bench_sets.py [name ...]   (names of tests/golden/make_golden.py WIDER_SETS)"""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests/golden")
from fhe_amd import binfhe as bf  # noqa: E402
from fhe_amd._lib import check, lib, ptr, vp  # noqa: E402
from make_golden import GATE_SETS  # noqa: E402


def dalloc(x):
    d = vp()
    check(lib().fhe_hip_alloc(0, x.nbytes, ctypes.byref(d)))
    check(lib().fhe_hip_copy_to_device(d, ptr(x), x.nbytes))
    return d.value


names = sys.argv[1:] or ["medium", "std128_3", "std128q", "std128_4", "lpf_std128", "lpf_std128q", "std192", "std256", "std256q_4",
                         "std128_3_lmkcdey", "std128q_lmkcdey", "medium_ap"]
for name in names:
    ps, m = GATE_SETS[name]
    P = bf.params(ps, m)
    t0 = time.time()
    keys = bf.keygen(ps, m, 7)
    e = bf.GateEngine(ps, m)
    e.load_keys(keys.bsk, keys.kskA, keys.kskB)
    B = 8192 if P.N == 1024 and P.Q < (1 << 28) else 2048  # the 32-bit kernels (incl. the digitsG = 4 split one)
    x = np.random.default_rng(1).integers(0, 2, B)
    a1, b1 = bf.encrypt(ps, m, keys.sk, x, 1)
    a2, b2 = bf.encrypt(ps, m, keys.sk, x, 2)
    d = [dalloc(v) for v in (a1, b1, a2, b2)]
    ao, bo = dalloc(np.zeros((B, P.n), np.uint64)), dalloc(np.zeros(B, np.uint64))
    e.eval_gate_device(bf.AND, B, *d, ao, bo)
    check(lib().fhe_hip_synchronize(0))
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        e.eval_gate_device(bf.AND, B, *d, ao, bo)
        check(lib().fhe_hip_synchronize(0))
        ts.append(time.perf_counter() - t)
    h = np.zeros((B, P.n), np.uint64)
    hb = np.zeros(B, np.uint64)
    check(lib().fhe_hip_copy_to_host(ptr(h), vp(ao), h.nbytes))
    check(lib().fhe_hip_copy_to_host(ptr(hb), vp(bo), hb.nbytes))
    ok = np.array_equal(bf.decrypt(ps, m, keys.sk, h, hb), x)
    print(f"{name:18s} n={P.n:5d} N={P.N} Q={P.Q.bit_length()}b dG={P.digitsG} B={B}: "
          f"{B / min(ts):9.0f} gates/s  runs_ms={[round(t * 1e3, 1) for t in ts]}  correct={ok}  "
          f"setup {time.time() - t0:.0f}s", flush=True)
    for p in d + [ao, bo]:
        check(lib().fhe_hip_free(vp(p)))
    e.close()
