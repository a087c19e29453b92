// keygen_dev.hip -- BTKeyGen on the device (KeyGenCGGI rgsw-acc-cggi.cpp:71-96,
// KeyGenDM rgsw-acc-dm.cpp:80-114, KeyGenLMKCDEY / KeyGenAuto rgsw-acc-lmkcdey.cpp:160-226,
// KeySwitchGen lwe-pke.cpp:264-344).
//
// Bit-identical to the host generator keygen_bootstrap() (keygen.cpp) for the same seed: the
// generator is counter-based, so every draw of every stream is computed independently here.
// The keys are written straight into the engine's resident layouts (packed Montgomery u32 BSK,
// u16 KSK rows), with the reference raw layouts as an optional export.
//
// Per RGSW row pair (row0 = A + msg?, row1 = A * S + NTT(e) + msg?):
//   k_kg_sample  A uniform mod Q (drawn in EVALUATION), e the reference's discrete Gaussian, message monomial
//                folded into e (row1 message) or kept as M (row0 message)  -> [E, M] per pair
//   ntt1024      forward NTT of every E and M (the batched kernel of ntt.hip)
//   k_kg_finish  row1 = A*S + E (- skAuto*g for automorphism keys), row0 = A + M
// KSK: one wave per row, n uniform draws, <a, s> by wave reduction, b = e + <a,s> + s'_i j B^k.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <vector>

#include "engine.h"
#include "keygen.h"
#include "nt.h"
#include "ntt.h"

namespace fhe_amd {
namespace {

struct KgDesc {
    uint64_t s0;        // rng_state of the stream
    uint32_t rp;        // row pair: words [rp * 2N, (rp + 1) * 2N) in both BSK layouts
    uint32_t call;      // first draw of this row pair in the stream
    uint32_t mm, mval;  // message mval * X^mm (mval = 0: none)
    uint32_t odd;       // message on row 1 (else on row 0)
    int32_t aidx;       // automorphism key: index of its permuted secret (else -1)
    uint32_t g;         // automorphism key gadget power
    uint32_t pad;
};
static_assert(sizeof(KgDesc) == 40, "descriptor layout");

__device__ __forceinline__ uint64_t draw(uint64_t s0, uint64_t k) { return mix64(s0 + (k + 2) * kRngGamma); }
__device__ __forceinline__ uint64_t draw_uniform(uint64_t s0, uint64_t k, uint64_t m) {
    return __umul64hi(draw(s0, k), m);
}
// the reference's discrete Gaussian (keygen.h dgg_sample) on the host's table, lifted mod m
__device__ __forceinline__ uint64_t draw_dgg(uint64_t s0, uint64_t k, uint64_t m, const DggTable& t) {
    const int64_t v = dgg_sample(draw(s0, k), t);
    return v < 0 ? (uint64_t)(v + (int64_t)m) : (uint64_t)v;
}

__global__ void __launch_bounds__(256) k_kg_sample(const KgDesc* __restrict__ D, uint32_t N, uint64_t Q,
                                                   uint64_t* __restrict__ A, uint64_t* __restrict__ T, DggTable dg) {
    const KgDesc k = D[blockIdx.x];
    uint64_t* a = A + (size_t)blockIdx.x * N;
    uint64_t* e = T + (size_t)blockIdx.x * 2 * N;
    uint64_t* m = e + N;
    for (uint32_t j = threadIdx.x; j < N; j += blockDim.x) {
        a[j] = draw_uniform(k.s0, k.call + j, Q);
        uint64_t ev = draw_dgg(k.s0, k.call + N + j, Q, dg);
        uint64_t mv = (k.mval && j == k.mm) ? k.mval : 0;
        if (k.odd) {
            ev += mv;
            ev = ev >= Q ? ev - Q : ev;
            mv = 0;
        }
        e[j] = ev;
        m[j] = mv;
    }
}

__global__ void __launch_bounds__(256) k_kg_finish(const KgDesc* __restrict__ D, uint32_t N, uint64_t Q,
                                                   const uint64_t* __restrict__ S,
                                                   const uint64_t* __restrict__ skAuto,
                                                   const uint64_t* __restrict__ A, const uint64_t* __restrict__ T,
                                                   uint64_t ninv, uint32_t* __restrict__ bsk,
                                                   uint64_t* __restrict__ raw, uint32_t ginx_u4) {
    const KgDesc k = D[blockIdx.x];
    const uint64_t* a = A + (size_t)blockIdx.x * N;
    const uint64_t* e = T + (size_t)blockIdx.x * 2 * N;
    const uint64_t* m = e + N;
    const size_t base = (size_t)k.rp * 2 * N;
    for (uint32_t j = threadIdx.x; j < N; j += blockDim.x) {
        const uint64_t av = a[j];
        uint64_t r1 = (av * S[j]) % Q + e[j];
        r1 = r1 >= Q ? r1 - Q : r1;
        if (k.aidx >= 0) {
            const uint64_t t = (skAuto[(size_t)k.aidx * N + j] * k.g) % Q;
            r1 = r1 >= t ? r1 - t : r1 + Q - t;
        }
        uint64_t r0 = av + m[j];
        r0 = r0 >= Q ? r0 - Q : r0;
        // engine layout (Engine::load_bsk): slot c = l*32 + 2kk + e of component h at
        // ((kk * 64 + h * 32 + l) * 2 + e), values x * N^-1 in Montgomery form (* 2^32 mod Q)
        const uint32_t l = j >> 5, kk = (j & 31) >> 1, el = j & 1;
        const uint32_t v0 = (uint32_t)((((r0 * ninv) % Q) << 32) % Q), v1 = (uint32_t)((((r1 * ninv) % Q) << 32) % Q);
        // component 1 of row rp sits at position rp ^ 1 with kBskHalfSwap (boot.h)
        const uint32_t rp1 = kBskHalfSwap ? k.rp ^ 1 : k.rp;
        if (ginx_u4) {
            // rp = (2 i + ks) dG2 + row with dG2 = 4 (boot.h ginx_u4_off)
            const size_t bi = (size_t)(k.rp >> 3) * 16 * N;
            bsk[bi + ginx_u4_off((k.rp >> 2) & 1, k.rp & 3, kk, l, el)]       = v0;
            bsk[bi + ginx_u4_off((k.rp >> 2) & 1, rp1 & 3, kk, 32 + l, el)]   = v1;
        } else {
            bsk[base + row_off(0, kk, l, el)]                  = v0;
            bsk[(size_t)rp1 * 2 * N + row_off(0, kk, 32 + l, el)] = v1;
        }
        if (raw) {
            raw[base + j] = r0;
            raw[base + N + j] = r1;
        }
    }
}

// one wave per KSK row [N][baseKS][digitsKS]; rows of the u16 layout are ksk_width(n) wide (A, B, zeros)
__global__ void __launch_bounds__(256) k_kg_ksk(uint64_t seed, uint32_t rows, uint32_t n, uint32_t bKS, uint32_t dKS,
                                                uint64_t qk, const uint64_t* __restrict__ sv,
                                                const uint64_t* __restrict__ svN, const uint64_t* __restrict__ dig,
                                                uint16_t* __restrict__ ksk, uint64_t* __restrict__ rawA,
                                                uint64_t* __restrict__ rawB, DggTable dg) {
    const uint32_t row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= rows) return;
    const uint64_t s0 = rng_state(seed, T_KSK, row);
    uint64_t acc = 0;
    const uint32_t W = ksk_width(n);
    for (uint32_t t = lane; t < W; t += 64) {
        const uint64_t v = t < n ? draw_uniform(s0, t, qk) : 0;
        acc += v * sv[t];
        if (t != n) ksk[(size_t)row * W + t] = (uint16_t)v;
        if (rawA && t < n) rawA[(size_t)row * n + t] = v;
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) {
        const uint32_t i = row / (bKS * dKS), j = (row / dKS) % bKS, kk = row % dKS;
        uint64_t b = draw_dgg(s0, n, qk, dg);
        b = (b + svN[i] * ((j * dig[kk]) % qk)) % qk;
        b = (b + acc % qk) % qk;
        ksk[(size_t)row * W + n] = (uint16_t)b;
        if (rawB) rawB[row] = b;
    }
}

inline int64_t signed_of(uint64_t x, uint64_t m) { return x > (m >> 1) ? (int64_t)x - (int64_t)m : (int64_t)x; }
inline uint64_t lift(int64_t v, uint64_t m) {
    const int64_t r = v % (int64_t)m;
    return (uint64_t)(r < 0 ? r + (int64_t)m : r);
}

template <class T>
struct DevBuf {
    T* p = nullptr;
    explicit DevBuf(size_t count) { FHE_HIP_CHECK(hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(T))); }
    ~DevBuf() { (void)hipFree(p); }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
};

// message monomial of KeyGenDM / KeyGenLMKCDEY: m mod q on X^(m * 2N/q), negated past N
inline void monomial(const Params& p, int64_t m, uint32_t row, uint32_t& mm, uint32_t& mval) {
    int64_t e = ((m % (int64_t)p.q) + p.q) % p.q * (2 * p.N / p.q);
    const uint64_t g = p.gpow[(row >> 1) + 1];
    bool neg = false;
    if (e >= (int64_t)p.N) { e -= p.N; neg = true; }
    mm = (uint32_t)e;
    mval = (uint32_t)(neg ? p.Q - g : g);
}

}  // namespace

void keygen_bootstrap_device(const Params& p, const std::vector<uint64_t>& sk, uint64_t seed, int device,
                             uint32_t* d_bsk, uint16_t* d_ksk, uint64_t* raw_bsk, uint64_t* raw_kskA,
                             uint64_t* raw_kskB, void* stream) {
    if (sk.size() != p.n) throw std::invalid_argument("secret key has wrong length");
    for (uint64_t v : sk)
        if (v >= p.qKS) throw std::invalid_argument("secret key not reduced mod qKS");
    if (p.N != 1024 || p.digitsG2 != 4) throw std::invalid_argument("device key generation expects N = 1024, digitsG = 3");
    if (p.Q >= (1ull << 31)) throw std::invalid_argument("device key generation expects Q < 2^31");
    const uint32_t n = p.n, N = p.N, dG2 = p.digitsG2;
    const uint64_t Q = p.Q;
    hipStream_t s = static_cast<hipStream_t>(stream);
    FHE_HIP_CHECK(hipSetDevice(device));

    // ring secret and its EVALUATION form (host: N coefficients)
    std::vector<uint64_t> skN, S;
    keygen_ring_secret(p, seed, skN);
    S = skN;
    HostNtt ntt;
    ntt.init(N, Q, p.psi);
    ntt.forward(S.data());

    // one descriptor per RGSW row pair, in the order keygen_bootstrap() draws them
    std::vector<KgDesc> desc;
    std::vector<uint64_t> skAuto;
    auto add = [&](uint64_t st, uint32_t rp, uint32_t row, uint32_t mm, uint32_t mval, int32_t aidx, uint32_t g) {
        desc.push_back(KgDesc{st, rp, row * 2 * N, mm, mval, row & 1u, aidx, g, 0});
    };
    if (p.method == M_GINX) {
        for (uint32_t i = 0; i < n; ++i) {
            const int64_t si = signed_of(sk[i], p.qKS);
            for (uint32_t ks = 0; ks < 2; ++ks) {
                const bool m = ks == 0 ? si == 1 : si == -1;
                const uint64_t st = rng_state(seed, T_BSK, (uint64_t)i * 2 + ks);
                for (uint32_t row = 0; row < dG2; ++row)   // G^(row/2+1) on X^0: constant in EVALUATION
                    add(st, (i * 2 + ks) * dG2 + row, row, 0, m ? (uint32_t)p.gpow[(row >> 1) + 1] : 0, -1, 0);
            }
        }
    } else if (p.method == M_AP) {
        const uint32_t bR = p.baseR, dR = p.digitsR;
        desc.reserve((size_t)n * (bR - 1) * dR * dG2);
        for (uint32_t i = 0; i < n; ++i) {
            const int64_t si = signed_of(sk[i], p.qKS);
            int64_t rk = 1;
            for (uint32_t k = 0; k < dR; ++k, rk *= bR)
                for (uint32_t j = 1; j < bR; ++j) {
                    const uint32_t slot = (i * bR + j) * dR + k;
                    const uint64_t st = rng_state(seed, T_BSK, slot);
                    for (uint32_t row = 0; row < dG2; ++row) {
                        uint32_t mm, mval;
                        monomial(p, si * (int64_t)j * rk, row, mm, mval);
                        add(st, slot * dG2 + row, row, mm, mval, -1, 0);
                    }
                }
        }
    } else {
        for (uint32_t i = 0; i < n; ++i) {
            const int64_t si = signed_of(sk[i], p.qKS);
            const uint64_t st = rng_state(seed, T_BSK, i);
            for (uint32_t row = 0; row < dG2; ++row) {
                uint32_t mm, mval;
                monomial(p, (int64_t)lift(si, p.q), row, mm, mval);
                add(st, i * dG2 + row, row, mm, mval, -1, 0);
            }
        }
        // automorphism keys: [0] for -5 (2N - 5), [k] for 5^k (KeyGenAuto)
        const uint32_t dA = p.digitsG - 1;
        skAuto.resize((size_t)(p.numAutoKeys + 1) * N);
        for (uint32_t k = 0; k <= p.numAutoKeys; ++k) {
            const uint32_t kk = k == 0 ? 2 * N - 5 : (uint32_t)powmod(5, k, 2 * N);
            auto_eval(p, kk, S.data(), skAuto.data() + (size_t)k * N);
            const uint64_t st = rng_state(seed, T_AUTO, k);
            for (uint32_t row = 0; row < dA; ++row)
                add(st, n * dG2 + k * dA + row, row, 0, 0, (int32_t)k, (uint32_t)p.gpow[row + 1]);
        }
    }

    const size_t words = p.bsk_words();
    FHE_HIP_CHECK(hipMemsetAsync(d_bsk, 0, words * 4, s));  // AP: the j = 0 slots stay zero
    if (raw_bsk) FHE_HIP_CHECK(hipMemsetAsync(raw_bsk, 0, words * 8, s));
    DevBuf<KgDesc> dd(desc.size());
    DevBuf<uint64_t> dS(N), dAuto(skAuto.size());
    FHE_HIP_CHECK(hipMemcpyAsync(dd.p, desc.data(), desc.size() * sizeof(KgDesc), hipMemcpyHostToDevice, s));
    FHE_HIP_CHECK(hipMemcpyAsync(dS.p, S.data(), N * 8, hipMemcpyHostToDevice, s));
    if (!skAuto.empty())
        FHE_HIP_CHECK(hipMemcpyAsync(dAuto.p, skAuto.data(), skAuto.size() * 8, hipMemcpyHostToDevice, s));
    NttPlan plan;
    FHE_HIP_CHECK(ntt_plan_init(plan, Q, p.psi, N, device));
    struct PlanGuard { NttPlan& p; ~PlanGuard() { ntt_plan_free(p); } } guard{plan};
    const size_t chunk = std::min<size_t>(desc.size(), 32768);
    DevBuf<uint64_t> dA(chunk * N), dT(chunk * 2 * N);
    for (size_t c0 = 0; c0 < desc.size(); c0 += chunk) {
        const uint32_t nc = (uint32_t)std::min(chunk, desc.size() - c0);
        k_kg_sample<<<nc, 256, 0, s>>>(dd.p + c0, N, Q, dA.p, dT.p, dgg_table());
        FHE_HIP_CHECK(hipGetLastError());
        FHE_HIP_CHECK(ntt1024_launch(plan, dT.p, dT.p, 2 * nc, false, s));
        k_kg_finish<<<nc, 256, 0, s>>>(dd.p + c0, N, Q, dS.p, dAuto.p, dA.p, dT.p, invmod(N, Q), d_bsk, raw_bsk,
                                       (kGinxU4 && p.method == M_GINX) ? 1u : 0u);
        FHE_HIP_CHECK(hipGetLastError());
    }

    // key-switching key
    const uint64_t qk = p.qKS;
    const uint32_t rows = (uint32_t)p.ksk_rows();
    const uint32_t W = ksk_width(n);
    std::vector<uint64_t> sv(W, 0), svN(N), dig(p.digitsKS);
    for (uint32_t i = 0; i < n; ++i) sv[i] = sk[i] % qk;
    for (uint32_t i = 0; i < N; ++i) svN[i] = lift(signed_of(skN[i], Q), qk);
    for (uint32_t k = 0, v = 1; k < p.digitsKS; ++k, v *= p.baseKS) dig[k] = v;
    DevBuf<uint64_t> dsv(W), dsvN(N), ddig(dig.size());
    FHE_HIP_CHECK(hipMemcpyAsync(dsv.p, sv.data(), W * 8, hipMemcpyHostToDevice, s));
    FHE_HIP_CHECK(hipMemcpyAsync(dsvN.p, svN.data(), N * 8, hipMemcpyHostToDevice, s));
    FHE_HIP_CHECK(hipMemcpyAsync(ddig.p, dig.data(), dig.size() * 8, hipMemcpyHostToDevice, s));
    k_kg_ksk<<<(rows + 3) / 4, 256, 0, s>>>(seed, rows, n, p.baseKS, p.digitsKS, qk, dsv.p, dsvN.p, ddig.p, d_ksk,
                                            raw_kskA, raw_kskB, dgg_table());
    FHE_HIP_CHECK(hipGetLastError());
    FHE_HIP_CHECK(hipStreamSynchronize(s));  // temporaries are freed on return
}

}  // namespace fhe_amd
