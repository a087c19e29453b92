// ntt_plan.cpp -- builds and uploads the twiddle tables for ntt.hip.
#include <vector>

#include "nt.h"
#include "ntt.h"

namespace fhe_amd {

hipError_t ntt_plan_init(NttPlan& p, uint64_t Q, uint64_t psi, uint32_t N, int device) {
    if (N != 1024) return hipErrorInvalidValue;
    if (Q < 3 || Q >= (1ull << 62) || (Q - 1) % (2 * N) != 0 || !is_prime(Q)) return hipErrorInvalidValue;
    if (psi == 0) psi = root_of_unity(2 * N, Q);
    if (powmod(psi, N, Q) != Q - 1) return hipErrorInvalidValue;  // must be a primitive 2N-th root
    HostNtt h;
    h.init(N, Q, psi);
    p.Q = Q; p.psi = psi; p.N = N; p.device = device;
    p.wide = Q >= (1ull << 30);  // the 32-bit path keeps lazy values below 4Q < 2^32
    const uint64_t w1 = h.tabI[1];
    p.ninv = h.ninv;
    p.w1ninv = mulmod(w1, h.ninv, Q);
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return e;
    if ((e = hipDeviceGetAttribute(&p.cus, hipDeviceAttributeMultiprocessorCount, device)) != hipSuccess) return e;
    if (!p.wide) {
        std::vector<uint32_t> f(2 * N), iv(2 * N);
        for (uint32_t i = 0; i < N; ++i) {
            f[2 * i] = (uint32_t)h.tab[i];  f[2 * i + 1] = shoup32(h.tab[i], Q);
            iv[2 * i] = (uint32_t)h.tabI[i]; iv[2 * i + 1] = shoup32(h.tabI[i], Q);
        }
        p.ninv_pre = shoup32(p.ninv, Q);
        p.w1ninv_pre = shoup32(p.w1ninv, Q);
        if ((e = hipMalloc(&p.d_tab_fwd, f.size() * 4)) != hipSuccess) return e;
        if ((e = hipMalloc(&p.d_tab_inv, iv.size() * 4)) != hipSuccess) return e;
        if ((e = hipMemcpy(p.d_tab_fwd, f.data(), f.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) return e;
        if ((e = hipMemcpy(p.d_tab_inv, iv.data(), iv.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) return e;
        if (Q < (1ull << 27)) {
            auto mont = [&](uint64_t x) { return (uint32_t)(((x % Q) << 32) % Q); };
            std::vector<uint32_t> fm(N), im(N);
            for (uint32_t i = 0; i < N; ++i) {
                fm[i] = mont(h.tab[i]);
                im[i] = mont(h.tabI[i]);
            }
            uint32_t inv = 1;  // Q^-1 mod 2^32 by Newton iteration
            for (int k = 0; k < 5; ++k) inv *= 2u - (uint32_t)Q * inv;
            p.qinvp = inv;
            p.oneR = mont(1);
            p.ninvR = mont(p.ninv);
            p.w1ninvR = mont(p.w1ninv);
            if ((e = hipMalloc(&p.d_tabm_fwd, N * 4)) != hipSuccess) return e;
            if ((e = hipMalloc(&p.d_tabm_inv, N * 4)) != hipSuccess) return e;
            if ((e = hipMemcpy(p.d_tabm_fwd, fm.data(), N * 4, hipMemcpyHostToDevice)) != hipSuccess) return e;
            if ((e = hipMemcpy(p.d_tabm_inv, im.data(), N * 4, hipMemcpyHostToDevice)) != hipSuccess) return e;
        }
    } else {
        std::vector<uint64_t> f(2 * N), iv(2 * N);
        for (uint32_t i = 0; i < N; ++i) {
            f[2 * i] = h.tab[i];  f[2 * i + 1] = shoup64(h.tab[i], Q);
            iv[2 * i] = h.tabI[i]; iv[2 * i + 1] = shoup64(h.tabI[i], Q);
        }
        p.ninv_pre = shoup64(p.ninv, Q);
        p.w1ninv_pre = shoup64(p.w1ninv, Q);
        for (uint32_t S = 1; S < 20; ++S)
            if (Q == (1ull << 60) - ((1ull << S) - 1)) p.sol_shift = S;
        if ((e = hipMalloc(&p.d_tab_fwd, f.size() * 8)) != hipSuccess) return e;
        if ((e = hipMalloc(&p.d_tab_inv, iv.size() * 8)) != hipSuccess) return e;
        if ((e = hipMemcpy(p.d_tab_fwd, f.data(), f.size() * 8, hipMemcpyHostToDevice)) != hipSuccess) return e;
        if ((e = hipMemcpy(p.d_tab_inv, iv.data(), iv.size() * 8, hipMemcpyHostToDevice)) != hipSuccess) return e;
    }
    return hipSuccess;
}

void ntt_plan_free(NttPlan& p) {
    if (p.d_tab_fwd) (void)hipFree(p.d_tab_fwd);
    if (p.d_tab_inv) (void)hipFree(p.d_tab_inv);
    if (p.d_tabm_fwd) (void)hipFree(p.d_tabm_fwd);
    if (p.d_tabm_inv) (void)hipFree(p.d_tabm_inv);
    p.d_tab_fwd = p.d_tab_inv = p.d_tabm_fwd = p.d_tabm_inv = nullptr;
}

}  // namespace fhe_amd
