// keyswitch.hip -- LWE key switching (LWEEncryptionScheme::KeySwitch,
// src/binfhe/lib/lwe-pke.cpp:348-372) fused with the final ModSwitch(qKS -> q)
// (:254-261) of SwitchCTtoqn (:170-178).
//
// out = (0, b) - sum_{i<N, j<digitsKS} KSK[i][digit_j(a_i)][j]   (mod qKS)
// One workgroup per ciphertext; thread t owns columns 2t, 2t+1 of the
// (n+1)-wide rows (A row + B stored at column n, u16, padded to 512).  Each
// of the N*digitsKS row gathers is one fully coalesced 1 KiB read.  qKS is a
// power of two (2^14 in both STD128 sets), so the row sums are accumulated in
// plain u32 (3072 * 2^14 < 2^32) and reduced once.
#include "arith.h"
#include "boot.h"

namespace fhe_amd {

__global__ void __launch_bounds__(256)
    k_keyswitch(GateArgs g, uint32_t logBase, uint32_t digitsKS, const uint32_t* __restrict__ ksk,
                const uint32_t* __restrict__ ms_a, const uint32_t* __restrict__ ms_b, uint32_t q_out,
                uint64_t* __restrict__ a_out, uint64_t* __restrict__ b_out) {
    __shared__ uint32_t s_a[1024];
    const uint32_t gate = blockIdx.x, t = threadIdx.x;
    for (uint32_t i = t; i < g.N; i += 256) s_a[i] = ms_a[(size_t)gate * g.N + i];
    __syncthreads();
    const uint32_t base = 1u << logBase, mask = base - 1;
    uint32_t lo = 0, hi = 0;
#pragma unroll 4
    for (uint32_t i = 0; i < g.N; ++i) {
        const uint32_t ai = s_a[i];
        for (uint32_t j = 0; j < digitsKS; ++j) {
            const uint32_t dig = (ai >> (logBase * j)) & mask;
            const uint32_t row = (i * base + dig) * digitsKS + j;
            const uint32_t w   = ksk[(size_t)row * 256 + t];
            lo += w & 0xffffu;
            hi += w >> 16;
        }
    }
    const uint32_t qm = g.qKS - 1;
    const uint32_t c0 = 2 * t, c1 = 2 * t + 1;
    const uint32_t b  = ms_b[gate];
    uint32_t v0 = ((c0 == g.n ? b : 0u) - lo) & qm;
    uint32_t v1 = ((c1 == g.n ? b : 0u) - hi) & qm;
    if (q_out) {  // ModSwitch qKS -> q: floor((2 v q + qKS) / (2 qKS)) mod q (exact, see bootstrap.hip)
        v0 = ((2 * v0 * q_out + g.qKS) / (2 * g.qKS)) % q_out;
        v1 = ((2 * v1 * q_out + g.qKS) / (2 * g.qKS)) % q_out;
    }
    uint64_t* oa = a_out + (size_t)gate * g.n;
    if (c0 < g.n) oa[c0] = v0;
    else if (c0 == g.n) b_out[gate] = v0;
    if (c1 < g.n) oa[c1] = v1;
    else if (c1 == g.n) b_out[gate] = v1;
}

hipError_t launch_keyswitch(const GateArgs& g, uint32_t baseKS, uint32_t digitsKS, const uint16_t* ksk,
                            const uint32_t* ms_a, const uint32_t* ms_b, uint32_t q_out, uint64_t* a_out,
                            uint64_t* b_out, hipStream_t s) {
    if (g.count == 0) return hipSuccess;
    if (baseKS & (baseKS - 1)) return hipErrorInvalidValue;
    if (g.qKS & (g.qKS - 1) || g.qKS > 65536 || g.n >= 512 || g.N > 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_keyswitch, dim3(g.count), dim3(256), 0, s, g, (uint32_t)__builtin_ctz(baseKS), digitsKS,
                       reinterpret_cast<const uint32_t*>(ksk), ms_a, ms_b, q_out, a_out, b_out);
    return hipGetLastError();
}

}  // namespace fhe_amd
