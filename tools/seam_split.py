"""Backend::BlindRotateBatch (fhe_hip_blind_rotate_acc_batch_device: EvalAcc on HBM-resident RLWE
accumulators) on the digitsG = 4 sets whose gates run the split kernels: the accumulator-I/O
instantiations of K1s (GINX) / K1m (LMKCDEY) against the 64-bit accumulator K5 they replaced
(FHE_HIP_GINX3=0), same inputs, outputs compared.

  python tools/seam_split.py [B]      (each set once per process mode; prints items/s)
"""
import ctypes
import os
import subprocess
import sys
import time

import numpy as np

sys.path.insert(0, ".")
SETS = {"STD128_3": (4, 2), "STD128_4_LMKCDEY": (23, 3), "STD128Q": (6, 2)}


def run(name, B):
    from fhe_amd import binfhe as bf
    from fhe_amd._lib import check, lib, ptr, vp
    ps, m = SETS[name]
    keys = bf.keygen(ps, m, 4321)
    e = bf.GateEngine(ps, m)
    e.load_keys(keys.bsk, keys.kskA, keys.kskB)
    P = e.params
    ctmod = 2 * P.N if m == bf.LMKCDEY else P.q
    rng = np.random.default_rng(5)
    a = rng.integers(0, ctmod, (B, P.n), dtype=np.uint64)
    acc = rng.integers(0, P.Q, (B, 2, P.N), dtype=np.uint64)
    da, dacc = vp(), vp()
    check(lib().fhe_hip_alloc(0, a.nbytes, ctypes.byref(da)))
    check(lib().fhe_hip_alloc(0, acc.nbytes, ctypes.byref(dacc)))
    check(lib().fhe_hip_copy_to_device(da, ptr(a), a.nbytes))
    ts = []
    for rep in range(4):
        check(lib().fhe_hip_copy_to_device(dacc, ptr(acc), acc.nbytes))
        check(lib().fhe_hip_synchronize(0))
        t = time.perf_counter()
        check(lib().fhe_hip_blind_rotate_acc_batch_device(e._h, B, da, ctmod, dacc, None))
        check(lib().fhe_hip_synchronize(0))
        ts.append(time.perf_counter() - t)
    out = np.zeros_like(acc)
    check(lib().fhe_hip_copy_to_host(ptr(out), dacc, out.nbytes))
    dt = min(ts[1:])
    return B / dt, out


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        name, B = sys.argv[2], int(sys.argv[3])
        rate, out = run(name, B)
        np.save(f"/tmp/seam_split_{name}_{os.environ.get('FHE_HIP_GINX3', '1')}.npy", out)
        print(f"{rate:.1f}", flush=True)
        sys.exit(0)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    for name in SETS:
        res = {}
        for mode in ("1", "0"):
            env = dict(os.environ, FHE_HIP_GINX3=mode)
            r = subprocess.run([sys.executable, __file__, "--child", name, str(B)], env=env, capture_output=True,
                               text=True, timeout=300)
            if r.returncode:
                print(name, mode, "failed", r.stderr[-800:], flush=True)
                sys.exit(1)
            res[mode] = float(r.stdout.strip().split()[-1])
        same = np.array_equal(np.load(f"/tmp/seam_split_{name}_1.npy"), np.load(f"/tmp/seam_split_{name}_0.npy"))
        print(f"{name}: BlindRotateBatch B={B}: split kernel {res['1']:.0f} /s, K5 (FHE_HIP_GINX3=0) {res['0']:.0f} /s,"
              f" x{res['1'] / res['0']:.2f}, outputs identical: {same}", flush=True)
