// ntt.h -- host-side plan for the batched N=1024 negacyclic NTT (ntt.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fhe_amd {

struct NttPlan {
    uint64_t Q = 0, psi = 0;
    uint32_t N = 0;
    bool wide = false;  // Q >= 2^30: 64-bit arithmetic path (the 32-bit path keeps values < 4Q)
    // device tables: Table[i] / TableI[i] (reference order, transformnat-impl.h:777-831)
    // paired with Shoup precon; uint2 (32-bit path) or ulonglong2 (64-bit path)
    void* d_tab_fwd = nullptr;
    void* d_tab_inv = nullptr;
    uint64_t ninv = 0, ninv_pre = 0, w1ninv = 0, w1ninv_pre = 0;
    // Q = 2^60 - (2^S - 1) (the poly-benchmark prime, S = 14): S, which selects the Sol60 butterflies
    // of k_ntt1024w64 (shift-only q Q); 0 for any other 64-bit modulus
    uint32_t sol_shift = 0;
    // Q < 2^27: Table / TableI in Montgomery form (u32, x 2^32 mod Q) for the signed kernel
    void* d_tabm_fwd = nullptr;
    void* d_tabm_inv = nullptr;
    uint32_t qinvp = 0, oneR = 0, ninvR = 0, w1ninvR = 0;
    int device = 0;
    int cus = 256;      // compute units of the device (grid sizing)
};

// Builds tables on the host and uploads them; psi == 0 selects the reference's
// minimal primitive 2N-th root of unity (nbtheory-impl.h:183-228).
hipError_t ntt_plan_init(NttPlan& p, uint64_t Q, uint64_t psi, uint32_t N, int device);
void ntt_plan_free(NttPlan& p);
hipError_t ntt1024_launch(const NttPlan& p, const uint64_t* in, uint64_t* out, uint32_t count, bool inverse,
                          hipStream_t s);

}  // namespace fhe_amd
