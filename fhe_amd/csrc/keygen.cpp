// keygen.cpp -- see keygen.h.
#include "keygen.h"

#include <omp.h>

#include <cmath>
#include <stdexcept>

#include "nt.h"

namespace fhe_amd {
namespace {

// counter-based generator: splitmix64 over (seed, tag, stream, counter)
struct Rng {
    uint64_t s;
    Rng(uint64_t seed, uint64_t tag, uint64_t stream) {
        s = rng_state(seed, tag, stream);
        next();
    }
    uint64_t next() { return mix64(s += kRngGamma); }
    uint64_t uniform(uint64_t m) { return (uint64_t)(((u128)next() * m) >> 64); }
    int64_t dgg() { return dgg_sample(next(), dgg_table()); }  // the reference's DGG, sigma 3.19
    int64_t ternary() { return (int64_t)uniform(3) - 1; }
};

inline uint64_t lift(int64_t v, uint64_t m) {
    int64_t r = v % (int64_t)m;
    return (uint64_t)(r < 0 ? r + (int64_t)m : r);
}
// signed value of x stored mod m (SwitchModulus semantics, mubintvecnat.cpp:109-122)
inline int64_t signed_of(uint64_t x, uint64_t m) { return x > (m >> 1) ? (int64_t)x - (int64_t)m : (int64_t)x; }

}  // namespace

const DggTable& dgg_table() {
    static const DggTable t = [] {
        DggTable d{};
        const double M = 12.00610553538285;
        d.fin = (int)std::ceil(kDggSigma * M);
        if (d.fin > kDggMaxFin) throw std::logic_error("DGG table size");
        const double variance = 2 * kDggSigma * kDggSigma;
        double cusum = 0.0;
        for (int x = 1; x <= d.fin; ++x) {
            cusum += std::exp(-((double)(x * x) / variance));
            d.vals[x - 1] = cusum;
        }
        d.a = 1.0 / (2 * cusum + 1.0);
        for (int x = 0; x < d.fin; ++x) d.vals[x] *= d.a;
        return d;
    }();
    return t;
}

void auto_eval(const Params& p, uint32_t k, const uint64_t* in, uint64_t* out) {
    // AutomorphismTransform(k) in EVALUATION (poly-impl.h:350-356)
    const uint32_t N = p.N, logN = ilog2(N), mask = N - 1;
    for (uint32_t j = 0; j < N; ++j) {
        uint32_t jk = (2 * j + 1) * k;
        out[reverse_bits(j, logN)] = in[reverse_bits((jk >> 1) & mask, logN)];
    }
}

void keygen_ring_secret(const Params& p, uint64_t seed, std::vector<uint64_t>& skN) {
    skN.assign(p.N, 0);
    Rng r(seed, T_SKN, 0);
    for (uint32_t i = 0; i < p.N; ++i) skN[i] = lift(p.keyDist == KD_GAUSSIAN ? r.dgg() : r.ternary(), p.Q);
}

void keygen_secret(const Params& p, uint64_t seed, std::vector<uint64_t>& sk) {
    sk.assign(p.n, 0);
    Rng r(seed, T_SK, 0);
    for (uint32_t i = 0; i < p.n; ++i)
        sk[i] = lift(p.keyDist == KD_GAUSSIAN ? r.dgg() : r.ternary(), p.qKS);
}

namespace {
void keygen_one(const Params& p, const std::vector<uint64_t>& sk, uint64_t seed, uint64_t bseed, bool with_ksk,
                KeySet& out);
}

// timeOptimization (BTKeyGen, binfhecontext.cpp:285-307): one whole key per baseG of the map, as the
// reference's KeyGen per base makes it -- its own RLWE secret skN, bootstrapping key and switching
// key; the key of the context's own baseG is the one keygen without timeOptimization makes from the
// same seed (out.skN is that base's secret)
void keygen_bootstrap(const Params& p, const std::vector<uint64_t>& sk, uint64_t seed, KeySet& out) {
    if (!p.timeopt) {
        keygen_one(p, sk, seed, seed, true, out);
        return;
    }
    out.bsk.assign(p.bsk_words(), 0);
    out.kskA.assign(p.ksk_rows_all() * p.n, 0);
    out.kskB.assign(p.ksk_rows_all(), 0);
    for (uint32_t bg : kSignBases) {
        Params pb = p.with_base(bg);
        pb.timeopt = false;
        KeySet t;
        const bool own = bg == p.baseG;
        const uint64_t sb = own ? seed : seed ^ ((uint64_t)bg * kRngGamma);
        keygen_one(pb, sk, sb, sb, true, t);
        const size_t k = p.ksk_index(bg), rows = p.ksk_rows();
        std::copy(t.bsk.begin(), t.bsk.end(), out.bsk.begin() + p.bsk_offset(bg));
        std::copy(t.kskA.begin(), t.kskA.end(), out.kskA.begin() + k * rows * p.n);
        std::copy(t.kskB.begin(), t.kskB.end(), out.kskB.begin() + k * rows);
        if (own) {
            out.sk = std::move(t.sk);
            out.skN = std::move(t.skN);
        }
    }
}

namespace {
// seed: skN and the switching key; bseed: the bootstrapping key's randomness
void keygen_one(const Params& p, const std::vector<uint64_t>& sk, uint64_t seed, uint64_t bseed, bool with_ksk,
                KeySet& out) {
    if (sk.size() != p.n) throw std::invalid_argument("secret key has wrong length");
    const uint32_t n = p.n, N = p.N, dG2 = p.digitsG2;
    const uint64_t Q = p.Q;
    out.sk = sk;
    HostNtt ntt;
    ntt.init(N, Q, p.psi);

    // RLWE secret skN and its EVAL form
    keygen_ring_secret(p, seed, out.skN);
    std::vector<uint64_t> S(out.skN);
    ntt.forward(S.data());

    // ---- bootstrapping key
    out.bsk.assign(p.bsk_words(), 0);
    auto rgsw_row_pair = [&](uint64_t* row0, uint64_t* row1, Rng& r, const uint64_t* msg_eval, int msg_slot) {
        // row0 = A (+msg), row1 = A*S + NTT(e) (+msg)   (KeyGenCGGI/KeyGenLMKCDEY structure)
        std::vector<uint64_t> e(N);
        for (uint32_t j = 0; j < N; ++j) row0[j] = r.uniform(Q);
        for (uint32_t j = 0; j < N; ++j) e[j] = lift(r.dgg(), Q);
        ntt.forward(e.data());
        for (uint32_t j = 0; j < N; ++j) row1[j] = addmod(mulmod(row0[j], S[j], Q), e[j], Q);
        if (msg_eval) {
            uint64_t* dst = msg_slot == 0 ? row0 : row1;
            for (uint32_t j = 0; j < N; ++j) dst[j] = addmod(dst[j], msg_eval[j], Q);
        }
    };
    const size_t rg = (size_t)dG2 * 2 * N;
    if (p.method == M_GINX) {
#pragma omp parallel for schedule(dynamic, 4)
        for (int64_t i = 0; i < (int64_t)n; ++i) {
            const int64_t s = signed_of(sk[i], p.qKS);
            std::vector<uint64_t> msg(N);
            for (int ks = 0; ks < 2; ++ks) {
                const bool m = ks == 0 ? s == 1 : s == -1;  // 0 -> {0,0}, 1 -> {1,0}, -1 -> {0,1}
                Rng r(bseed, T_BSK, (uint64_t)i * 2 + ks);
                uint64_t* key = out.bsk.data() + ((size_t)i * 2 + ks) * rg;
                for (uint32_t row = 0; row < dG2; ++row) {
                    // message G^{(row>>1)+1} on coefficient 0: constant in EVALUATION domain
                    for (uint32_t j = 0; j < N; ++j) msg[j] = p.gpow[(row >> 1) + 1];
                    rgsw_row_pair(key + (size_t)row * 2 * N, key + ((size_t)row * 2 + 1) * N, r,
                                  m ? msg.data() : nullptr, row & 1);
                }
            }
        }
    } else if (p.method == M_AP) {
        // KeyGenAcc DM (rgsw-acc-dm.cpp:39-58): key [i][j][k] = KeyGenDM(s_i * j * baseR^k) for
        // j in [1, baseR), k < digitsR; KeyGenDM (:80-114): +-G on X^mm, mm = (m mod q) * (2N/q)
        const uint32_t bR = p.baseR, dR = p.digitsR;
#pragma omp parallel for schedule(dynamic, 1)
        for (int64_t i = 0; i < (int64_t)n; ++i) {
            const int64_t s = signed_of(sk[i], p.qKS);
            std::vector<uint64_t> msg(N);
            int64_t rk = 1;
            for (uint32_t k = 0; k < dR; ++k, rk *= bR)
                for (uint32_t j = 1; j < bR; ++j) {
                    const int64_t m = s * (int64_t)j * rk;
                    int64_t mm = (((m % (int64_t)p.q) + p.q) % p.q) * (2 * N / p.q);
                    bool neg = false;
                    if (mm >= (int64_t)N) { mm -= N; neg = true; }
                    const size_t slot = ((size_t)i * bR + j) * dR + k;
                    Rng r(bseed, T_BSK, slot);
                    uint64_t* key = out.bsk.data() + slot * rg;
                    for (uint32_t row = 0; row < dG2; ++row) {
                        std::fill(msg.begin(), msg.end(), 0);
                        const uint64_t g = p.gpow[(row >> 1) + 1];
                        msg[mm] = neg ? Q - g : g;
                        ntt.forward(msg.data());
                        rgsw_row_pair(key + (size_t)row * 2 * N, key + ((size_t)row * 2 + 1) * N, r, msg.data(),
                                      row & 1);
                    }
                }
        }
    } else {
#pragma omp parallel for schedule(dynamic, 4)
        for (int64_t i = 0; i < (int64_t)n; ++i) {
            // KeyGenLMKCDEY(m = s_i): +-G on X^mm, mm = (m mod q) * (2N/q)
            const int64_t s = signed_of(sk[i], p.qKS);
            int64_t mm = lift(s, p.q) * (2 * N / p.q);
            bool neg = false;
            if (mm >= (int64_t)N) { mm -= N; neg = true; }
            Rng r(bseed, T_BSK, (uint64_t)i);
            uint64_t* key = out.bsk.data() + (size_t)i * rg;
            std::vector<uint64_t> msg(N);
            for (uint32_t row = 0; row < dG2; ++row) {
                std::fill(msg.begin(), msg.end(), 0);
                uint64_t g = p.gpow[(row >> 1) + 1];
                msg[mm] = neg ? Q - g : g;
                ntt.forward(msg.data());
                rgsw_row_pair(key + (size_t)row * 2 * N, key + ((size_t)row * 2 + 1) * N, r, msg.data(), row & 1);
            }
        }
        // automorphism keys: [0] for -5 (2N-5), [k] for 5^k, k = 1..numAutoKeys (KeyGenAuto)
        uint64_t* autok = out.bsk.data() + (size_t)n * rg;
        const size_t ak = (size_t)(p.digitsG - 1) * 2 * N;
        for (uint32_t k = 0; k <= p.numAutoKeys; ++k) {
            uint32_t kk = k == 0 ? 2 * N - 5 : (uint32_t)powmod(5, k, 2 * N);
            std::vector<uint64_t> skAuto(N), e(N);
            auto_eval(p, kk, S.data(), skAuto.data());
            Rng r(bseed, T_AUTO, k);
            uint64_t* key = autok + k * ak;
            for (uint32_t row = 0; row + 1 < p.digitsG; ++row) {
                uint64_t* r0 = key + (size_t)row * 2 * N;
                uint64_t* r1 = r0 + N;
                for (uint32_t j = 0; j < N; ++j) r0[j] = r.uniform(Q);
                for (uint32_t j = 0; j < N; ++j) e[j] = lift(r.dgg(), Q);
                ntt.forward(e.data());
                const uint64_t g = p.gpow[row + 1];
                for (uint32_t j = 0; j < N; ++j)
                    r1[j] = addmod(submod(e[j], mulmod(skAuto[j], g, Q), Q), mulmod(r0[j], S[j], Q), Q);
            }
        }
    }

    if (!with_ksk) return;
    // ---- key-switching key (KeySwitchGen): rows [N][baseKS][digitsKS], A row of n, B
    const uint64_t qk = p.qKS;
    out.kskA.assign(p.ksk_rows() * n, 0);
    out.kskB.assign(p.ksk_rows(), 0);
    std::vector<uint64_t> digitsKS(p.digitsKS);
    {
        uint64_t v = 1;
        for (uint32_t k = 0; k < p.digitsKS; ++k, v *= p.baseKS) digitsKS[k] = v;
    }
    std::vector<uint64_t> sv(n);
    for (uint32_t i = 0; i < n; ++i) sv[i] = sk[i] % qk;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)N; ++i) {
        const uint64_t svN = lift(signed_of(out.skN[i], Q), qk);
        for (uint32_t j = 0; j < p.baseKS; ++j)
            for (uint32_t k = 0; k < p.digitsKS; ++k) {
                const size_t row = ((size_t)i * p.baseKS + j) * p.digitsKS + k;
                Rng r(seed, T_KSK, row);
                uint64_t* a = out.kskA.data() + row * n;
                u128 acc = 0;
                for (uint32_t t = 0; t < n; ++t) {
                    a[t] = r.uniform(qk);
                    acc += (u128)a[t] * sv[t];
                }
                uint64_t b = lift(r.dgg(), qk);
                b = addmod(b, mulmod(svN, (j * digitsKS[k]) % qk, qk), qk);
                b = addmod(b, (uint64_t)(acc % qk), qk);
                out.kskB[row] = b;
            }
    }
}
}  // namespace

void encrypt(const Params& p, const uint64_t* sk, const int* bits, size_t count, uint64_t seed, uint64_t* a,
             uint64_t* b, uint32_t ptmod, uint64_t mod, uint32_t len) {
    const uint64_t q = mod ? mod : p.q;
    const uint32_t n = len ? len : p.n;
    if (ptmod < 2 || ptmod > q) throw std::invalid_argument("plaintext modulus out of range");
#pragma omp parallel for schedule(static) if (count > 64)
    for (int64_t g = 0; g < (int64_t)count; ++g) {
        Rng r(seed, T_ENC, (uint64_t)g);
        uint64_t* ag = a + (size_t)g * n;
        u128 acc = 0;
        for (uint32_t i = 0; i < n; ++i) {
            ag[i] = r.uniform(q);
            acc += (u128)ag[i] * lift(signed_of(sk[i], p.qKS), q);
        }
        // b = (m mod p) (q / p) + e + <a, s>   (lwe-pke.cpp:103-128)
        uint64_t m = ((uint64_t)(uint32_t)bits[g] % ptmod) * (q / ptmod);
        b[g] = (m + lift(r.dgg(), q) + (uint64_t)(acc % q)) % q;
    }
}

int64_t decrypt(const Params& p, const uint64_t* sk, const uint64_t* a, uint64_t b, uint32_t len, uint64_t mod,
                uint32_t ptmod) {
    u128 acc = 0;
    for (uint32_t i = 0; i < len; ++i) acc += (u128)(a[i] % mod) * lift(signed_of(sk[i], p.qKS), mod);
    uint64_t inner = (uint64_t)(acc % mod);
    uint64_t r = submod(b % mod, inner, mod);
    // Round(p/q x) = Floor(p/q (x + q/(2p)))   (lwe-pke.cpp:209-215)
    r = addmod(r, mod / (2 * (uint64_t)ptmod), mod);
    return (int64_t)(((u128)ptmod * r) / mod);
}

}  // namespace fhe_amd
