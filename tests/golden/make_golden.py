"""Generates the committed golden vectors in tests/golden/ by running the
REFERENCE itself (oracle/_ref/libfhe_ref.so, compiled from /root/reference by
oracle/Makefile) on seeded inputs.  Run here (where the reference exists):

    make -C oracle -j8 && python tests/golden/make_golden.py [ntt|gates|all]

Fixtures are data only (inputs + the reference's outputs + hashes).
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from oracle_lib import GINX, LMKCDEY, STD128, STD128_LMKCDEY, Ref  # noqa: E402

NTT_MODULI = {
    "q60": 1152921504606830593,   # poly-benchmark-1k (benchmark/src/poly-benchmark-1k.cpp:40-50)
    "std128": 134215681,          # STD128 Q = LastPrime(27, 2048)
    "lmkcdey": 268369921,         # STD128_LMKCDEY Q = LastPrime(28, 2048)
}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.uint64).tobytes()).hexdigest()


def make_ntt():
    ref = Ref(None, None)
    for name, Q in NTT_MODULI.items():
        rng = np.random.default_rng(0x5EED0001)
        x = rng.integers(0, Q, size=(64, 1024), dtype=np.uint64)
        x[0] = 0
        x[1] = Q - 1
        fwd, psi = ref.ntt(Q, x, inverse=False)
        inv, _ = ref.ntt(Q, x, inverse=True)   # x taken as EVALUATION input
        np.savez(os.path.join(HERE, f"ntt_{name}.npz"), Q=np.uint64(Q), psi=np.uint64(psi), seed=np.uint64(0x5EED0001),
                 x=x[:4], fwd=fwd[:4], inv=inv[:4],
                 fwd_sha=np.array(sha(fwd)), inv_sha=np.array(sha(inv)))
        print(name, Q, psi, "ok")


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what in ("ntt", "all"):
        make_ntt()
