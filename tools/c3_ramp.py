"""Per-step times of config 3 (1024 STD128 GINX gates, device-resident) right after the host-side setup:
shows the clock ramp from idle that a short warmup leaves inside the timed region.
usage: python tools/c3_ramp.py [steps]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from fhe_amd import binfhe as bf  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 120
ps, m, B = bf.STD128, bf.GINX, 1024
keys = bf.keygen(ps, m, 7)
P = bf.params(ps, m)
rng = np.random.default_rng(1)
x1, x2 = rng.integers(0, 2, B), rng.integers(0, 2, B)
a1, b1 = bf.encrypt(ps, m, keys.sk, x1, 1)
a2, b2 = bf.encrypt(ps, m, keys.sk, x2, 2)
dev = torch.device("cuda:0")
e = bf.GateEngine(ps, m, device=0)
e.load_keys(keys.bsk, keys.kskA, keys.kskB)
st = torch.cuda.Stream(dev)
d = [torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).to(dev) for x in (a1, b1, a2, b2)]
ao = torch.empty((B, P.n), dtype=torch.int64, device=dev)
bo = torch.empty((B,), dtype=torch.int64, device=dev)
torch.cuda.synchronize()
time.sleep(3.0)  # idle, as after the bench's host-side setup
evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(steps)]
for k in range(steps):
    evs[k][0].record(st)
    e.blind_rotate_device(bf.AND, B, *[t.data_ptr() for t in d], stream=st.cuda_stream)
    e.keyswitch_workspace_device(B, ao.data_ptr(), bo.data_ptr(), stream=st.cuda_stream)
    evs[k][1].record(st)
torch.cuda.synchronize()
ms = [a.elapsed_time(b) for a, b in evs]
print("per-step ms:", " ".join(f"{x:.2f}" for x in ms))
cum = np.cumsum(ms)
for lo, hi in ((0, 10), (10, 20), (20, 40), (40, 80), (80, steps)):
    print(f"steps {lo}-{hi} (t = {cum[lo]:.0f} ms ..): mean {np.mean(ms[lo:hi]):.3f} ms")
e.close()
