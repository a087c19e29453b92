"""Batched negacyclic NTT (N = 1024) on the GPU -- mirrors NativePoly::SwitchFormat
(src/core/include/lattice/hal/default/poly-impl.h:420-440 in the reference)."""
import ctypes

import numpy as np

from ._lib import check, lib, ptr, u64, vp


class NttPlan:
    def __init__(self, Q, psi=0, N=1024, device=0):
        self._h = vp()
        psi_out = u64()
        check(lib().fhe_hip_ntt_plan_create(Q, psi, N, device, ctypes.byref(self._h), ctypes.byref(psi_out)))
        self.Q, self.psi, self.N, self.device = int(Q), int(psi_out.value), N, device

    def close(self):
        if self._h:
            lib().fhe_hip_ntt_plan_destroy(self._h)
            self._h = vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self):
        return lib().fhe_hip_ntt_plan_stream(self._h)

    def forward(self, polys):
        """COEFFICIENT -> EVALUATION (bit-reversed); returns a new uint64 array."""
        return self._run(polys, 0)

    def inverse(self, polys):
        return self._run(polys, 1)

    def _run(self, polys, inv):
        a = np.array(polys, dtype=np.uint64, copy=True, order="C")
        if a.ndim != 2 or a.shape[1] != self.N:
            raise ValueError(f"expected shape (count, {self.N})")
        check(lib().fhe_hip_ntt_batch(self._h, ptr(a), a.shape[0], inv))
        return a

    def run_device(self, d_in, d_out, count, inverse=False, stream=None):
        """Asynchronous transform of device buffers (raw device pointers as ints)."""
        check(lib().fhe_hip_ntt_batch_device(self._h, vp(d_in), vp(d_out), count, int(inverse),
                                             vp(stream) if stream else None))
