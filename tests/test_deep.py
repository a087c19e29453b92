"""Deep-chain noise regression in the style of the reference's UnitTestFHEWDeep.cpp:72-116
(AND_GINX_VERY_LONG): 2000 dependent STD128 GINX AND levels, decrypting every level, here on 1024
independent chains at once (one 1024-gate batch per dependent step, inputs and outputs resident on
the GPU).  Per level, as the reference does:  b = AND(s1, s2);  s1 <- b;  s2 <- AND(b, d)  with
d = AND(E(1), E(1)) bootstrapped once.  Run on keys the reference generated itself (its Gaussian
noise, oracle/_ref ref_keygen) and on our seeded keys (the same sigma 3.19 DGG):
zero decryption failures over 2 x 1024 x 2000 bootstraps each."""
import ctypes

import numpy as np
import pytest

from oracle_lib import Ref, ref_available

CHAINS, LEVELS = 1024, 2000


class Dev:
    """device buffers through the C-ABI's memory calls (Backend::Allocate/CopyTo*)"""

    def __init__(self):
        from fhe_amd._lib import lib
        self.L = lib()
        self.ptrs = []

    def alloc(self, nbytes):
        from fhe_amd._lib import check, vp
        d = vp()
        check(self.L.fhe_hip_alloc(0, nbytes, ctypes.byref(d)))
        self.ptrs.append(d.value)
        return d.value

    def put(self, x):
        from fhe_amd._lib import check, ptr
        x = np.ascontiguousarray(x)
        d = self.alloc(x.nbytes)
        check(self.L.fhe_hip_copy_to_device(ctypes.c_void_p(d), ptr(x), x.nbytes))
        return d

    def get(self, d, out):
        from fhe_amd._lib import check, ptr
        check(self.L.fhe_hip_synchronize(0))
        check(self.L.fhe_hip_copy_to_host(ptr(out), ctypes.c_void_p(d), out.nbytes))
        return out

    def free(self):
        for p in self.ptrs:
            self.L.fhe_hip_free(ctypes.c_void_p(p))
        self.ptrs = []


def run_chains(sk, bsk, A, B, seed):
    from fhe_amd import binfhe as bf
    ps, m, AND = bf.STD128, bf.GINX, bf.AND
    n = bf.params(ps, m).n
    eng = bf.GateEngine(ps, m, device=0)
    eng.load_keys(bsk, A, B)
    rng = np.random.default_rng(seed)
    x1, x2 = rng.integers(0, 2, CHAINS), rng.integers(0, 2, CHAINS)
    dev = Dev()
    a1, b1 = bf.encrypt(ps, m, sk, x1, seed + 1)
    a2, b2 = bf.encrypt(ps, m, sk, x2, seed + 2)
    o1, ob1 = bf.encrypt(ps, m, sk, np.ones(CHAINS, int), seed + 3)
    o2, ob2 = bf.encrypt(ps, m, sk, np.ones(CHAINS, int), seed + 4)
    s1 = (dev.put(a1), dev.put(b1))
    s2 = (dev.put(a2), dev.put(b2))
    one1, one2 = (dev.put(o1), dev.put(ob1)), (dev.put(o2), dev.put(ob2))
    d = (dev.alloc(CHAINS * n * 8), dev.alloc(CHAINS * 8))
    eng.eval_gate_device(AND, CHAINS, *one1, *one2, *d)
    P = [(dev.alloc(CHAINS * n * 8), dev.alloc(CHAINS * 8)) for _ in range(2)]
    Qb = [(dev.alloc(CHAINS * n * 8), dev.alloc(CHAINS * 8)) for _ in range(2)]
    ha, hb = np.zeros((CHAINS, n), np.uint64), np.zeros(CHAINS, np.uint64)
    v = (x1 & x2).astype(np.int64)
    fails = 0
    first_fail = None
    for it in range(LEVELS):
        b, s2n = P[it & 1], Qb[it & 1]
        eng.eval_gate_device(AND, CHAINS, *s1, *s2, *b)          # b = AND(s1, s2)
        eng.eval_gate_device(AND, CHAINS, *b, *d, *s2n)         # s2 <- AND(b, d)
        dec = bf.decrypt(ps, m, sk, dev.get(b[0], ha), dev.get(b[1], hb))
        bad = int(np.sum(dec != v))
        if bad and first_fail is None:
            first_fail = it
        fails += bad
        s1, s2 = b, s2n       # the value is carried: v stays v1 & v2 of the previous level
    eng.close()
    dev.free()
    return fails, first_fail


@pytest.mark.gpu
@pytest.mark.skipif(not ref_available(), reason="reference oracle not built")
def test_gpu_deep_and_chain_reference_keys():
    ref = Ref(3, 2)   # STD128, GINX
    sk, bsk, A, B = ref.keygen()   # the reference's own KeyGen + BTKeyGen (Gaussian noise)
    fails, first = run_chains(sk, bsk, A, B, 0xDEE0)
    assert fails == 0, f"{fails} decryption failures, first at level {first}"


@pytest.mark.gpu
def test_gpu_deep_and_chain_our_keys():
    from fhe_amd import binfhe as bf
    keys = bf.keygen(bf.STD128, bf.GINX, 0xDEE1)
    fails, first = run_chains(keys.sk, keys.bsk, keys.kskA, keys.kskB, 0xDEE2)
    assert fails == 0, f"{fails} decryption failures, first at level {first}"
