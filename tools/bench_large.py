"""Throughput of the large-precision family on one GPU (bootstrap_wide.hip): EvalBinGate(AND)
batches and EvalSign on the STD128 large set GenerateBinFHEContext(STD128, false, logQ) (n = 1305,
N = 2048, 54-bit Q, qKS = 2^35).  Synthetic seeded keys and inputs; host round trip included
(inputs are 10 KB per ciphertext, negligible next to a 1305-step blind rotation).

    python tools/bench_large.py [--logq 29] [--batch 2048] [--steps 3] [--time-opt]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--logq", type=int, default=29)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--sign-batch", type=int, default=256)
    ap.add_argument("--toy", action="store_true")
    ap.add_argument("--time-opt", action="store_true", help="timeOptimization: the three-key map")
    args = ap.parse_args()
    from fhe_amd import binfhe as bf
    ps = bf.large_paramset(bf.TOY if args.toy else bf.STD128, False, args.logq, 0, args.time_opt)
    t0 = time.time()
    keys = bf.keygen(ps, bf.GINX, 0x1A46E)
    e = bf.GateEngine(ps, bf.GINX)
    e.load_keys(keys.bsk, keys.kskA, keys.kskB)
    P = e.params
    setup = time.time() - t0
    rng = np.random.default_rng(3)
    B = args.batch
    x1, x2 = rng.integers(0, 2, B), rng.integers(0, 2, B)
    a1, b1 = bf.encrypt(ps, bf.GINX, keys.sk, x1, 5)
    a2, b2 = bf.encrypt(ps, bf.GINX, keys.sk, x2, 6)
    e.eval_gate(1, a1[:64], b1[:64], a2[:64], b2[:64])  # warm-up (workspace, code objects)
    t = time.perf_counter()
    for _ in range(args.steps):
        ao, bo = e.eval_gate(1, a1, b1, a2, b2)
    gate_s = (time.perf_counter() - t) / args.steps
    ok = bool(np.array_equal(bf.decrypt(ps, bf.GINX, keys.sk, ao, bo), x1 & x2))
    mod = 1 << args.logq
    PL = mod // (P.q // 256)
    S = args.sign_batch
    xs = rng.integers(0, PL, S)
    la, lb = bf.encrypt(ps, bf.GINX, keys.sk, xs, 7, PL, mod)
    t = time.perf_counter()
    sa, sb = e.eval_sign(la, lb, mod)
    sign_s = time.perf_counter() - t
    far = np.abs(xs - PL // 2) > PL // 16
    far &= (xs > PL // 16) & (xs < PL - PL // 16)
    sign_ok = bool(np.array_equal(bf.decrypt(ps, bf.GINX, keys.sk, sa, sb, mod=P.q, p=2)[far], (xs >= PL // 2)[far]))
    print(json.dumps({"workload": f"{'TOY' if args.toy else 'STD128'} large-precision logQ={args.logq}", "n": P.n, "N": P.N,
                      "Q_bits": P.Q.bit_length(), "digitsG": P.digitsG,
                      "time_optimization": args.time_opt, "batch": B, "gates_per_s": B / gate_s,
                      "ms_per_batch": gate_s * 1e3, "gates_decrypt_ok": ok, "evalsign_batch": S,
                      "evalsign_per_s": S / sign_s, "evalsign_ok": sign_ok, "setup_s": setup}))


if __name__ == "__main__":
    main()
