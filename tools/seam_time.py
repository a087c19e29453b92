"""Host-buffer (PCIe-inclusive) vs device-resident gate bootstrapping, and the latency of the
Backend seam's single-ciphertext calls ("BlindRotate for one ciphertext is a
full device round-trip ... unmeasured").

  python tools/seam_time.py [ginx|lmk] [B ...]

Per batch size B (STD128 AND gates, every output decrypted and checked):
  host   fhe_hip_eval_bingate_batch: H2D of the two inputs, prep + K1 + K2, D2H of the result
         (what BinFHEContext::EvalBinGateBatch / BackendHIP callers see)
  device fhe_hip_eval_bingate_batch_device on HBM-resident inputs (what bench.py times)
then the seam ops on one ciphertext / accumulator (fhe_hip_blind_rotate_acc_batch = Backend::
BlindRotate, fhe_hip_keyswitch_batch = Backend::KeySwitch), median of 20 calls.
"""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from fhe_amd import binfhe as bf  # noqa: E402
from fhe_amd._lib import check, lib, ptr, vp  # noqa: E402

SETS = {"ginx": (bf.STD128, bf.GINX), "lmk": (bf.STD128_LMKCDEY, bf.LMKCDEY)}
name = sys.argv[1] if len(sys.argv) > 1 else "ginx"
ps, m = SETS[name]
batches = [int(x) for x in sys.argv[2:]] or [1, 16, 256, 1024, 8192, 65536]
keys = bf.keygen(ps, m, 1234)
e = bf.GateEngine(ps, m)
e.load_keys(keys.bsk, keys.kskA, keys.kskB)
P = e.params


def dalloc(nbytes):
    d = vp()
    check(lib().fhe_hip_alloc(0, nbytes, ctypes.byref(d)))
    return d.value


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        check(lib().fhe_hip_synchronize(0))
        ts.append(time.perf_counter() - t)
    return float(np.median(ts))


print(f"set {name}: n={P.n} N={P.N}", flush=True)
for B in batches:
    rng = np.random.default_rng(B)
    x1, x2 = rng.integers(0, 2, B), rng.integers(0, 2, B)
    a1, b1 = bf.encrypt(ps, m, keys.sk, x1, 7)
    a2, b2 = bf.encrypt(ps, m, keys.sk, x2, 8)
    reps = 20 if B <= 1024 else 3
    # the C-ABI call itself on caller-owned, already-touched output buffers (the Python wrapper's
    # fresh np.zeros outputs would add first-touch page faults to every call)
    hao, hbo = np.ones((B, P.n), np.uint64), np.ones(B, np.uint64)

    def host_call():
        check(lib().fhe_hip_eval_bingate_batch(e._h, bf.AND, B, ptr(a1), ptr(b1), ptr(a2), ptr(b2), ptr(hao),
                                               ptr(hbo)))
    host_call()  # warm-up (workspace, staging)
    th = timed(host_call, reps)
    res = {"h": (hao, hbo)}
    ok_h = np.array_equal(bf.decrypt(ps, m, keys.sk, *res["h"]), (x1 & x2).astype(np.int64))
    bufs = [dalloc(x.nbytes) for x in (a1, b1, a2, b2)]
    for d, x in zip(bufs, (a1, b1, a2, b2)):
        check(lib().fhe_hip_copy_to_device(vp(d), ptr(x), x.nbytes))
    dao, dbo = dalloc(B * P.n * 8), dalloc(B * 8)
    td = timed(lambda: e.eval_gate_device(bf.AND, B, *bufs, dao, dbo), reps)
    ao = np.zeros((B, P.n), np.uint64)
    bo = np.zeros(B, np.uint64)
    check(lib().fhe_hip_copy_to_host(ptr(ao), vp(dao), ao.nbytes))
    check(lib().fhe_hip_copy_to_host(ptr(bo), vp(dbo), bo.nbytes))
    ok_d = np.array_equal(ao, res["h"][0]) and np.array_equal(bo, res["h"][1])
    for d in bufs + [dao, dbo]:
        check(lib().fhe_hip_free(vp(d)))
    io = (2 * (P.n + 1) + (P.n + 1)) * 8 * B
    print(f"B={B}: host {th*1e3:.3f} ms ({B/th:.0f} gates/s)  device {td*1e3:.3f} ms ({B/td:.0f} gates/s)  "
          f"host/device {th/td:.3f}  PCIe bytes {io}  correct={ok_h} host==device={ok_d}", flush=True)

# the seam's one-ciphertext calls
rng = np.random.default_rng(5)
a = rng.integers(0, P.q, (1, P.n), dtype=np.uint64)
acc = rng.integers(0, P.Q, (1, 2, P.N), dtype=np.uint64)
e.blind_rotate_acc(a, P.q, acc)
t_br = timed(lambda: e.blind_rotate_acc(a, P.q, acc), 20)
ka = rng.integers(0, P.qKS, (1, P.N), dtype=np.uint64)
kb = rng.integers(0, P.qKS, 1, dtype=np.uint64)
e.keyswitch(ka, kb)
t_ks = timed(lambda: e.keyswitch(ka, kb), 20)
a1, b1 = bf.encrypt(ps, m, keys.sk, np.array([1]), 7)
a2, b2 = bf.encrypt(ps, m, keys.sk, np.array([1]), 8)
t_g1 = timed(lambda: e.eval_gate(bf.AND, a1, b1, a2, b2), 20)
print(f"seam, one item: BlindRotate {t_br*1e3:.3f} ms  KeySwitch {t_ks*1e3:.3f} ms  EvalBinGate {t_g1*1e3:.3f} ms",
      flush=True)
