"""BASELINE configs 4 and 5 at their stated size: 65,536 AND gates (STD128 GINX and
STD128_LMKCDEY) through one context and through the multi-device engine with 8 contexts
(the 8-shard split and reassembly of the 8-GPU run, here on device 0), checked against the
SHA-256 of the reference's own outputs for the same gates (tests/golden/full_*.npz, made by
tests/golden/make_golden.py full from oracle/_ref, the reference built from its sources)."""
import hashlib
import os
import sys

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SETS = ["std128", "lmkcdey"]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.uint64).tobytes()).hexdigest()


_cache = {}


def full(name):
    if name not in _cache:
        sys.path.insert(0, GOLD)
        from make_golden import full_inputs
        g = np.load(os.path.join(GOLD, f"full_{name}.npz"))
        _cache[name] = (g, full_inputs(name, int(g["count"])))
    return _cache[name]


@pytest.mark.parametrize("name", SETS)
def test_full_inputs_and_keys_match_golden(name):
    g, (ps, m, key_seed, keys, bits1, bits2, a1, b1, a2, b2) = full(name)
    assert int(g["paramset"]) == ps and int(g["key_seed"]) == key_seed
    assert sha(keys.bsk) + sha(keys.kskA) + sha(keys.kskB) == str(g["keys_sha"])
    assert sha(a1) + sha(b1) + sha(a2) + sha(b2) == str(g["in_sha"])
    assert len(g["shard_sha"]) == int(g["count"]) // int(g["shard"]) == 8


@pytest.mark.parametrize("name", SETS)
def test_full_golden_head_decrypts(name):
    """the first reference outputs (kept in full) decrypt to AND of the inputs"""
    from fhe_amd import binfhe as bf
    g, (ps, m, key_seed, keys, bits1, bits2, a1, b1, a2, b2) = full(name)
    dec = bf.decrypt(ps, m, keys.sk, g["out_a_head"].astype(np.uint64), g["out_b_head"].astype(np.uint64))
    assert np.array_equal(dec, (bits1 & bits2)[:16])


@pytest.mark.gpu
@pytest.mark.parametrize("name", SETS)
def test_gpu_full_batch_one_context_bit_exact(name):
    from fhe_amd import binfhe as bf
    g, (ps, m, key_seed, keys, bits1, bits2, a1, b1, a2, b2) = full(name)
    eng = bf.GateEngine(ps, m, device=0)
    eng.load_keys(keys.bsk, keys.kskA, keys.kskB)
    ao, bo = eng.eval_gate(int(g["gate"]), a1, b1, a2, b2)
    eng.close()
    S = int(g["shard"])
    bad = [k for k in range(len(g["shard_sha"])) if sha(ao[k * S:(k + 1) * S]) + sha(bo[k * S:(k + 1) * S])
           != str(g["shard_sha"][k])]
    assert not bad, f"shards differing from the reference: {bad}"
    assert sha(ao) + sha(bo) == str(g["out_sha"])
    assert np.array_equal(ao[:16], g["out_a_head"].astype(np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("name", SETS)
def test_gpu_full_batch_eight_shards_bit_exact(name):
    """MultiGateEngine with 8 contexts (one host thread + stream each) on device 0: the
    contiguous 8192-gate shards of the 8-GPU run, reassembled in order"""
    from fhe_amd import binfhe as bf
    g, (ps, m, key_seed, keys, bits1, bits2, a1, b1, a2, b2) = full(name)
    me = bf.MultiGateEngine(ps, m, [0] * 8)
    me.load_keys(keys.bsk, keys.kskA, keys.kskB)
    ao, bo = me.eval_gate(int(g["gate"]), a1, b1, a2, b2)
    me.close()
    assert sha(ao) + sha(bo) == str(g["out_sha"])


# ---- BASELINE config 3: 1024 STD128 GINX AND gates (the batch bench.py's config3 object runs) ----
def config3():
    if "c3" not in _cache:
        sys.path.insert(0, GOLD)
        from make_golden import full_inputs
        g = np.load(os.path.join(GOLD, "full_std128_b1024.npz"))
        _cache["c3"] = (g, full_inputs("std128", int(g["count"])))
    return _cache["c3"]


def test_config3_inputs_match_golden_and_head_decrypts():
    from fhe_amd import binfhe as bf
    g, (ps, m, key_seed, keys, bits1, bits2, a1, b1, a2, b2) = config3()
    assert int(g["count"]) == 1024 and int(g["paramset"]) == ps
    assert sha(keys.bsk) + sha(keys.kskA) + sha(keys.kskB) == str(g["keys_sha"])
    assert sha(a1) + sha(b1) + sha(a2) + sha(b2) == str(g["in_sha"])
    dec = bf.decrypt(ps, m, keys.sk, g["out_a_head"].astype(np.uint64), g["out_b_head"].astype(np.uint64))
    assert np.array_equal(dec, (bits1 & bits2)[:16])


@pytest.mark.gpu
def test_gpu_config3_batch_bit_exact():
    """the 1024-gate batch at its own size (row-split key switch, one wave per gate) == the reference"""
    from fhe_amd import binfhe as bf
    g, (ps, m, key_seed, keys, bits1, bits2, a1, b1, a2, b2) = config3()
    eng = bf.GateEngine(ps, m, device=0)
    eng.load_keys(keys.bsk, keys.kskA, keys.kskB)
    ao, bo = eng.eval_gate(int(g["gate"]), a1, b1, a2, b2)
    eng.close()
    assert sha(ao) + sha(bo) == str(g["out_sha"])
    assert np.array_equal(ao[:16], g["out_a_head"].astype(np.uint64))
