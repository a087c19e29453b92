"""Small-batch latency of the paths the two-wave kernels serve (round 6): the seam's BlindRotate, BootstrapFunc at
ciphertext moduli q and 2N, EvalFunc with an arbitrary LUT, and gates, for the default context (K1x for GINX,
K1m's two-digit form for LMKCDEY, up to two gates per CU) and with FHE_HIP_{GINX,LMK}_KERNEL=wave (K1).
Host-buffer entry points, median of `reps` calls.
usage: python tools/small_batch_time.py [reps] [paramset name] [GINX | LMKCDEY]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from fhe_amd import binfhe as bf  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
ps = bf.PARAMSETS.index(sys.argv[2]) if len(sys.argv) > 2 else bf.STD128
m = bf.LMKCDEY if len(sys.argv) > 3 and sys.argv[3] == "LMKCDEY" else bf.GINX
knob = "FHE_HIP_LMK_KERNEL" if m == bf.LMKCDEY else "FHE_HIP_GINX_KERNEL"
keys = bf.keygen(ps, m, 3)
P = bf.params(ps, m)
rng = np.random.default_rng(5)


def med(f):
    f()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t)
    return sorted(ts)[len(ts) // 2] * 1e3


for kind in ("default", "wave"):
    if kind == "wave":
        os.environ[knob] = "wave"
    e = bf.GateEngine(ps, m, device=0)
    os.environ.pop(knob, None)
    e.load_keys(keys.bsk, keys.kskA, keys.kskB)
    out = []
    for cnt in (1, 64, 512):
        a = rng.integers(0, P.q, (cnt, P.n), dtype=np.uint64)
        b = rng.integers(0, P.q, cnt, dtype=np.uint64)
        a2 = rng.integers(0, 2 * P.N, (cnt, P.n), dtype=np.uint64)
        acc = rng.integers(0, P.Q, (cnt, 2, P.N), dtype=np.uint64)
        f = rng.integers(0, 8, P.q, dtype=np.uint64)
        f2 = rng.integers(0, 8, 2 * P.N, dtype=np.uint64)
        lut = (np.arange(P.q) * 37 % P.q).astype(np.uint64)
        r = {"gate": med(lambda: e.eval_gate(bf.AND, a, b, a[::-1].copy(), b[::-1].copy())),
             # LMKCDEY's seam takes a_i mod 2N
             "BlindRotate": med(lambda: e.blind_rotate_acc(a2, 2 * P.N, acc) if m == bf.LMKCDEY
                                else e.blind_rotate_acc(a, P.q, acc)),
             "BootstrapFunc q": med(lambda: e.bootstrap_func(a, b, P.q, f, 8)),
             "BootstrapFunc 2N": med(lambda: e.bootstrap_func(a2, b, 2 * P.N, f2, 8))}
        if P.q <= P.N:  # arbitrary functions need q <= N
            r["EvalFunc arbitrary"] = med(lambda: e.eval_func(a, b, P.q, lut))
        out.append(f"  {cnt:4d} ciphertexts ({e.gate_kernel(cnt)}): " + ", ".join(f"{k} {v:.2f} ms" for k, v in r.items()))
    print(kind)
    print("\n".join(out), flush=True)
    e.close()
