"""The closed-form op offsets of k_prep_lmk_w (fhe_amd/csrc/bootstrap.hip, round 5) against the
reference's sequential nSkips emission (RingGSWAccumulatorLMKCDEY::EvalAcc,
src/binfhe/lib/rgsw-acc-lmkcdey.cpp:99-157), as host models of both: for random group counts per logGen
position (empty, sparse, dense, every position non-empty) and automorphism-key caps 1..600 the two give
the same op list.  CPU-only; the kernel itself is checked bit-exact by the LMKCDEY GPU tests."""
import random

import pytest


def sequential(cnts, nh, cap):
    """rgsw-acc-lmkcdey.cpp:99-157: groups in position order, AUTO(nSkips) before a non-empty group when
    nSkips != 0, and after a position when nSkips reaches cap or i == 1; AUTO(0) after the -1 group"""
    out, ns = [], 0
    for half in range(2):
        base = nh * half
        for t in range(nh - 1):
            i, p = nh - 1 - t, base + t
            if cnts[p]:
                if ns:
                    out.append(("A", ns))
                    ns = 0
                out += [("G", p, r) for r in range(cnts[p])]
            ns += 1
            if ns == cap or i == 1:
                out.append(("A", ns))
                ns = 0
        if half == 0:
            out += [("G", nh - 1, r) for r in range(cnts[nh - 1])]
            out.append(("A", 0))
        else:
            out += [("G", 2 * nh - 1, r) for r in range(cnts[2 * nh - 1])]
    return out


def closed_form(cnts, nh, cap):
    """the kernel's per-64-position form: skip counter before lane from the last non-empty lane below (or
    the carry), at most two AUTO ops per position, offsets from the AUTO counts of lower lanes"""
    start = [0]
    for c in cnts:
        start.append(start[-1] + c)
    n, A, o, fill = start[-1], 0, {}, [0] * (2 * nh)
    for half in range(2):
        base, ns = nh * half, 0
        for tb in range(0, nh - 1, 64):
            last_ne, below_autos, lanes = None, 0, []
            for lane in range(64):
                t = tb + lane
                p, ok = base + t, t < nh - 1
                s, e = (start[p], start[p + 1]) if ok else (0, 0)
                ne = ok and e > s
                nsb = (lane - last_ne) % cap if last_ne is not None else (ns + lane) % cap
                pre = ne and nsb != 0
                aft = 1 if ne else nsb + 1
                cap_e = ok and (aft == cap or t == nh - 2)
                ab = A + below_autos
                if pre:
                    o[s + ab] = ("A", nsb)
                if ok:
                    fill[p] = s + ab + pre
                if cap_e:
                    o[e + ab + pre] = ("A", aft)
                below_autos += pre + cap_e
                if ne:
                    last_ne = lane
                lanes.append(0 if cap_e else aft)
            A += below_autos
            ns = lanes[min(64, nh - 1 - tb) - 1]
        if half == 0:
            fill[nh - 1] = start[nh - 1] + A
            o[start[nh] + A] = ("A", 0)
            A += 1
        else:
            fill[2 * nh - 1] = start[2 * nh - 1] + A
    for p in range(2 * nh):
        for r in range(cnts[p]):
            o[fill[p] + r] = ("G", p, r)
    assert sorted(o) == list(range(n + A))  # no slot written twice or left empty
    return [o[k] for k in range(n + A)]


@pytest.mark.parametrize("seed", range(6))
def test_closed_form_offsets_match_sequential_emission(seed):
    rng = random.Random(seed)
    for _ in range(12):
        nh = rng.choice([256, 512, 1024])
        cap = rng.choice([1, 2, 3, 10, 64, 100, 600])
        kind = rng.choice(["sparse", "half", "dense", "full", "empty"])
        if kind == "empty":
            cnts = [0] * (2 * nh)
        elif kind == "full":
            cnts = [rng.randint(1, 3) for _ in range(2 * nh)]
        elif kind == "dense":
            cnts = [rng.randint(0, 5) for _ in range(2 * nh)]
        else:
            d = 0.02 if kind == "sparse" else 0.5
            cnts = [rng.randint(1, 3) if rng.random() < d else 0 for _ in range(2 * nh)]
        assert closed_form(cnts, nh, cap) == sequential(cnts, nh, cap), (nh, cap, kind)
