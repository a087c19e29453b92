"""EvalFuncMultiOutputBatch timing: one fused call (fhe_hip_eval_func_multi_batch) for L LUTs
against L sequential EvalFunc calls (what the routed caller did before), and against L = 1, per batch size.
    python tools/multi_time.py [std128|lmkcdey]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from fhe_amd import binfhe as bf  # noqa: E402
from make_golden import fb_luts  # noqa: E402

SETS = {"std128": (bf.STD128, bf.GINX), "lmkcdey": (bf.STD128_LMKCDEY, bf.LMKCDEY)}
ps, m = SETS[sys.argv[1] if len(sys.argv) > 1 else "std128"]
P = bf.params(ps, m)
keys = bf.keygen(ps, m, 5)
e = bf.GateEngine(ps, m, 0)
e.load_keys(keys.bsk, keys.kskA, keys.kskB)
q = P.q
p = q // 256
luts = fb_luts(q, p, P.N)
for cls in ("neg", "per", "cube"):
    tab1 = luts[cls][None, :]
    tab4 = np.stack([luts[cls]] * 4)
    for B in (1, 16, 256, 2048):
        a, b = bf.encrypt(ps, m, keys.sk, np.arange(B) % p, 9, p)

        def t(fn, reps=3):
            fn()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            return (time.perf_counter() - t0) / reps * 1e3

        one = t(lambda: e.eval_func_multi(a, b, q, tab1))
        four = t(lambda: e.eval_func_multi(a, b, q, tab4))
        seq = t(lambda: [e.eval_func(a, b, q, tab4[j]) for j in range(4)])
        print(f"{cls:4s} B={B:5d}  L=1 {one:8.2f} ms  L=4 fused {four:8.2f} ms ({four / one:4.2f}x)  "
              f"L=4 as 4 calls {seq:8.2f} ms ({seq / one:4.2f}x)", flush=True)
