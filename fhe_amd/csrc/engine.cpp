// engine.cpp -- see engine.h.
#include "engine.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "keygen.h"
#include "nt.h"

namespace fhe_amd {

namespace {
inline uint32_t to_mont(uint64_t x, uint64_t Q) { return (uint32_t)(((u128)(x % Q) << 32) % Q); }
inline uint32_t neg_inv32(uint32_t Q) {  // -Q^-1 mod 2^32 (Newton)
    uint32_t x = Q;                        // Q * Q = 1 mod 8
    for (int i = 0; i < 5; ++i) x *= 2 - Q * x;
    return (uint32_t)(0u - x);
}
}  // namespace

bool Engine::fast_path(const Params& p) {
    const bool pow2q = !(p.q & (p.q - 1)), pow2ks = !(p.qKS & (p.qKS - 1));
    return !is_large(p.paramset) && p.N == 1024 && p.Q < (1ull << 28) && p.digitsG == 3 && pow2q && pow2ks &&
           p.qKS <= 65536 && p.n < 1024;
}

bool Engine::narrow_set(const Params& p) {
    // the 64-bit accumulator's 32-bit policy (bootstrap_wide.hip A32): residues and digit x key sums
    // (< digitsG2 Q^2 < Q 2^32) in 32-bit words
    return p.Q < (1ull << 30) && (uint64_t)p.digitsG2 * p.Q < (1ull << 32);
}

bool Engine::g3_set(const Params& p) {
    // digit fields of d + C in 32 bits (bootstrap.hip decompose_n): 4 g <= 32 and C + Q < 2^32
    const uint64_t g = p.gBits, h = 1ull << (g - 1);
    const uint64_t C = h * (1 + (1ull << g) + (1ull << (2 * g)) + (1ull << (3 * g)));
    return !is_large(p.paramset) && !p.timeopt && (p.method == M_GINX || p.method == M_LMKCDEY) && p.N == 1024 &&
           p.Q < (1ull << 27) &&
           p.digitsG == 4 && g >= 2 && 4 * g <= 32 && C + p.Q < (1ull << 32) && p.qKS <= 65536 && p.n < 1024;
}

constexpr bool kN2kExtended = true;
bool Engine::n2k_set(const Params& p) {
    // K1w at N = 2048: GINX with digitsG = 4 (q < 2N: the half-resolution table), and under
    // FHE_HIP_N2K_EXT (default on) digitsG 3 / 4 at 29-bit Q and q = 2N (the negated half-range table,
    // digitsG 4 / 5); LMKCDEY with digitsG = 4, and under FHE_HIP_N2K_EXT digitsG 3 (Q < 2^29) and 5
    // (Q < 2^27); the digit fields of d + C in 32 bits
    const uint64_t g = p.gBits, h = 1ull << (g - 1);
    const char* ext = std::getenv("FHE_HIP_N2K_EXT");
    const bool wide_rows = ext ? std::string(ext) == "1" : kN2kExtended;
    // GINX: digitsG 4 at Q < 2^27 (STD256Q); digitsG 3 / 4 at 2^27 <= Q < 2^29 (STD256, STD256_3, STD256_4:
    // the forward transform reduced three times); digitsG 5 at q = 2N (STD256Q_3, STD256Q_4)
    const bool ginx = p.method == M_GINX &&
                      (p.q < 2 * p.N || (p.q == 2 * p.N && (p.Q >= (1ull << 27) || p.digitsG == 5))) &&
                      (p.digitsG == 4 || (p.digitsG == 3 && p.Q >= (1ull << 27) && p.q < 2 * p.N) ||
                       (p.digitsG == 5 && p.q == 2 * p.N && wide_rows));
    // digitsG 3 with 2^27 <= Q < 2^28 (STD256Q_LMKCDEY) measured 24.0K -> 32.7K gates/s
    // (profiles/r04_ext_bench.txt); FHE_HIP_N2K_EXT=0 keeps it on K5
    const bool lmk = p.method == M_LMKCDEY && (p.digitsG == 4 || (wide_rows && (p.digitsG == 3 || p.digitsG == 5)));
    if (lmk && p.Q >= (1ull << 27) && (!wide_rows || p.digitsG == 5)) return false;  // reduced forward: 2-3 digits
    // LMKCDEY: Q < 2^29 (the forward transform reduced once at Q >= 2^27, three times at Q >= 2^28: the
    // 29-bit STD256_3 / STD256_4_LMKCDEY); GINX: Q < 2^27
    const uint64_t qmax = wide_rows ? (1ull << 29) : (1ull << 27);
    if (is_large(p.paramset) || p.timeopt || !(ginx || lmk) || p.N != 2048 || p.Q >= qmax || g < 2 ||
        (uint64_t)p.digitsG * g > 32)
        return false;
    uint64_t C = 0;
    for (uint32_t j = 0; j < p.digitsG; ++j) C += h << (j * g);
    return C + p.Q < (1ull << 32);
}

namespace {
bool knob_off(const char* name) {
    const char* e = std::getenv(name);
    return e && std::string(e) == "0";
}
}  // namespace

uint32_t Engine::kernel_kind(const Params& p) {
    if (fast_path(p)) return 1;
    if (g3_set(p) && !knob_off("FHE_HIP_GINX3")) return 2;
    if (n2k_set(p) && !knob_off("FHE_HIP_N2K")) return 4;
    if (narrow_set(p) && !knob_off("FHE_HIP_NARROW")) return 3;
    return 0;
}

uint32_t Engine::kernel() const {
    if (!wide_) return 1;
    if (g3_) return 2;
    if (n2k_) return 4;
    if (narrow_) return 3;
    return 0;
}

int Engine::ginx_choice(const GateArgs& g) const {
    if (!d_bsk2_) return 1;
    if (ginx_kernel_ == 2) return ginx2_supported(g, tabs_) ? 2 : 1;
    // K1x: gates, BootstrapFunc tables and the seam's accumulators, ciphertext modulus q or 2N; K1q (four waves
    // per gate) up to one gate per CU
    if (!ginx2x_supported(g, tabs_)) return 1;
    if (ginx_kernel_ == 4 || (ginx_kernel_ == 0 && 2 * (size_t)g.count <= x_batch_)) return 4;
    if (ginx_kernel_ == 3 || (ginx_kernel_ == 0 && g.count <= x_batch_)) return 3;
    return 1;
}

int Engine::lmk_choice(const GateArgs& g) const {
    if (p_.method != M_LMKCDEY || wide_ || !d_bsk2_ || lmk_kernel_ == 1 || !lmkx_supported(g, tabs_)) return 1;
    if (lmk_kernel_ == 4 || (lmk_kernel_ == 0 && 2 * (size_t)g.count <= x_batch_)) return 4;
    return lmk_kernel_ == 2 || g.count <= x_batch_ ? 2 : 1;
}

const char* Engine::gate_kernel(size_t count) const {
    const GateArgs g = gate_args(G_AND, count ? count : 1);
    const int nd = (int)p_.digitsG - 1;
    const bool lmk = p_.method == M_LMKCDEY;
    if (wide_) {  // rotate_device's order
        if (g3_ && lmk) return "k_blind_rotate_lmk3";
        if (n2k_ && lmk && lmk2k_supported(g, tabs2k_, nd)) return "k_blind_rotate_lmk2k";
        if (lmk || p_.method == M_AP) return "k_blind_rotate_wide_ops";
        if (n2k_ && n2k_supported(g, tabs2k_, nd)) return "k_blind_rotate_n2k";
        if (g3_ && ginx3_supported(g, tabs_)) return "k_blind_rotate_ginx2";
        return "k_blind_rotate_wide";
    }
    if (p_.method != M_GINX) {
        const int k = lmk_choice(g);
        return k == 4 ? "k_blind_rotate_lmk4x" : k == 2 ? "k_blind_rotate_lmk3" : "k_blind_rotate_lmk";
    }
    const int k = ginx_choice(g);
    return k == 2 ? "k_blind_rotate_ginx2" : k == 3 ? "k_blind_rotate_ginx2x" : k == 4 ? "k_blind_rotate_ginx4x"
                                                                                  : "k_blind_rotate_ginx";
}

bool Engine::ks32_set(const Params& p) {
    const bool pow2ks = !(p.qKS & (p.qKS - 1));
    // the tiled shapes (keyswitch.hip launch_keyswitch): baseKS 32 / 64 with digitsKS 3, 16 with 4, and 21 with 4
    // (STD256Q_3, digits by division)
    const bool shape = ((p.baseKS == 32 || p.baseKS == 64) && p.digitsKS == 3) ||
                       ((p.baseKS == 16 || p.baseKS == 21) && p.digitsKS == 4);
    return !is_large(p.paramset) && !p.timeopt && pow2ks && shape && p.qKS <= 65536 && p.n < 2048 && p.N <= 2048;
}

bool Engine::ks32w_set(const Params& p) {
    const bool pow2ks = p.qKS && !(p.qKS & (p.qKS - 1));
    // qKS < 2^32: GateArgs::qKS is a u32 word (launch_keyswitch_w32 reads it from there).  Round 6: also the prime
    // qKS of TOY / SIGNED_MOD_TEST (modKS = PRIME: qKS = Q < 2^28, baseKS 25), whose u32 sums are kept mod qKS
    const bool prime = p.baseKS == 25 && (p.qKS & 1) && p.qKS < (1ull << 28);
    return !is_large(p.paramset) && !p.timeopt && (prime || (pow2ks && p.qKS > 65536 && p.qKS < (1ull << 32))) &&
           keyswitch_w32_shape(p.baseKS, p.digitsKS) && p.n < 2048 && p.N <= 2048;
}

// K1w tables (bootstrap.hip k_blind_rotate_n2k): Table / TableI (2048 words each, u32 Montgomery; the
// uniform stages read words 0..31 of them), the half-resolution monomial pairs psi^(2f) - 1 for
// f in [0, 2048] at f + (f >> 5)
void Engine::build_tables_n2k() {
    const uint64_t Q = p_.Q;
    HostNtt h;
    h.init(p_.N, Q, p_.psi);
    constexpr size_t kMono = 2048 + 1 + 64;
    std::vector<uint32_t> t(2048 + 2048 + 2 * kMono, 0);
    uint32_t* tabF = t.data();
    uint32_t* tabI = tabF + 2048;
    uint32_t* mono = tabI + 2048;
    uint32_t* monoP = mono + kMono;
    for (uint32_t i = 0; i < 2048; ++i) {
        tabF[i] = to_mont(h.tab[i], Q);
        tabI[i] = to_mont(h.tabI[i], Q);
    }
    // q = 2N (odd exponents): psi^g - 1 for g in [0, 2048], the kernel negating past 2048 (FULL)
    const uint64_t psi2 = p_.q == 2 * p_.N ? p_.psi : mulmod(p_.psi, p_.psi, Q);
    uint64_t x = 1;
    for (uint32_t f = 0; f <= 2048; ++f) {
        mono[f + (f >> 5)]  = to_mont(submod(x, 1, Q), Q);
        monoP[f + (f >> 5)] = (uint32_t)submod(x, 1, Q);
        x = mulmod(x, psi2, Q);
    }
    FHE_HIP_CHECK(hipSetDevice(device_));
    FHE_HIP_CHECK(hipMalloc(&d_tables2k_, t.size() * 4));
    FHE_HIP_CHECK(hipMemcpy(d_tables2k_, t.data(), t.size() * 4, hipMemcpyHostToDevice));
    const uint32_t* d = static_cast<const uint32_t*>(d_tables2k_);
    tabs2k_ = BootTables{};
    tabs2k_.tabF = d;
    tabs2k_.tabI = d + 2048;
    tabs2k_.twA_fwd = tabs2k_.tabF;
    tabs2k_.twA_inv = tabs2k_.tabI;
    tabs2k_.mono = d + 4096;
    tabs2k_.monoP = tabs2k_.mono + kMono;
    tabs2k_.Q = (uint32_t)Q;
    tabs2k_.Q2 = (uint32_t)(2 * Q);
    tabs2k_.qinv = neg_inv32((uint32_t)Q);
    tabs2k_.ninvR = to_mont(h.ninv, Q);
    tabs2k_.w1R = to_mont(h.tabI[1], Q);
    tabs2k_.oneR = to_mont(1, Q);
    tabs2k_.nR = to_mont(p_.N, Q);
}

// K1w key layout, u32 Montgomery with N^-1 folded in, per index i and wave c:
// [c][q < 6][k2 < 16][64][4] = (K+[r], K+[r+1], K-[r], K-[r+1]), r = 2 k2 + e, slot x(L, r) of layout C,
// q = 2 j + o: digit row 2 j + c, column c (o = 0) or 1 - c (o = 1); raw BSK [n][2][dG2 = 6][2][N]
// LMKCDEY (k_blind_rotate_lmk2k): ek [i][c][q < 6][k4 < 8][64][4], register r = 4 k4 + e4 of lane L is
// slot x(L, r), q = 2 j + o: row 2 j + c, column c (o = 0) or 1 - c (o = 1), from [n][dG2 = 6][2][N];
// then ak [t][q < 6][k4][64][4], q = 2 d + column, from [numAutoKeys + 1][3][2][N]
void Engine::pack_n2k(const uint64_t* bsk) {
    const uint32_t n = p_.n, N = p_.N, dG2 = p_.digitsG2;
    const uint64_t Q = p_.Q, ninv = invmod(N, Q);
    auto word = [&](uint64_t v) { return to_mont(mulmod(v % Q, ninv, Q), Q); };
    auto slot = [](uint32_t L, uint32_t r) { return ((r >> 1) << 7) | (L << 1) | (r & 1); };
    if (p_.method == M_LMKCDEY) {
        const uint32_t nd = p_.digitsG - 1, kq = 2 * nd;  // retained digits, key vectors per slot
        const size_t per = (size_t)2 * kq * 8 * 64 * 4, aper = (size_t)kq * 8 * 64 * 4;
        const size_t nauto = (size_t)p_.numAutoKeys + 1;
        std::vector<uint32_t> dev((size_t)n * per + nauto * aper);
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < (int64_t)n; ++i)
            for (uint32_t c = 0; c < 2; ++c)
                for (uint32_t q = 0; q < kq; ++q)
                    for (uint32_t k4 = 0; k4 < 8; ++k4)
                        for (uint32_t L = 0; L < 64; ++L)
                            for (uint32_t e = 0; e < 4; ++e) {
                                const uint32_t row = 2 * (q >> 1) + c, col = (q & 1) ? 1 - c : c;
                                const size_t src = (((size_t)i * dG2 + row) * 2 + col) * N + slot(L, 4 * k4 + e);
                                dev[(size_t)i * per + ((((c * kq + q) * 8 + k4) * 64 + L) * 4 + e)] = word(bsk[src]);
                            }
        const uint64_t* asrc = bsk + (size_t)n * dG2 * 2 * N;
        uint32_t* adst = dev.data() + (size_t)n * per;
        for (size_t t = 0; t < nauto; ++t)
            for (uint32_t q = 0; q < kq; ++q)
                for (uint32_t k4 = 0; k4 < 8; ++k4)
                    for (uint32_t L = 0; L < 64; ++L)
                        for (uint32_t e = 0; e < 4; ++e) {
                            const uint32_t d = q >> 1, col = q & 1;
                            adst[t * aper + (((q * 8 + k4) * 64 + L) * 4 + e)] =
                                word(asrc[((t * nd + d) * 2 + col) * N + slot(L, 4 * k4 + e)]);
                        }
        FHE_HIP_CHECK(hipSetDevice(device_));
        if (d_bsk2_) FHE_HIP_CHECK(hipFree(d_bsk2_));
        d_bsk2_ = nullptr;
        FHE_HIP_CHECK(hipMalloc(&d_bsk2_, dev.size() * 4));
        FHE_HIP_CHECK(hipMemcpy(d_bsk2_, dev.data(), dev.size() * 4, hipMemcpyHostToDevice));
        return;
    }
    const uint32_t kq = 2 * (p_.digitsG - 1);  // retained digits x 2 columns
    const size_t per = (size_t)2 * kq * 16 * 64 * 4;
    std::vector<uint32_t> dev((size_t)n * per);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i)
        for (uint32_t c = 0; c < 2; ++c)
            for (uint32_t q = 0; q < kq; ++q)
                for (uint32_t k2 = 0; k2 < 16; ++k2)
                    for (uint32_t L = 0; L < 64; ++L)
                        for (uint32_t e4 = 0; e4 < 4; ++e4) {
                            const uint32_t r = 2 * k2 + (e4 & 1), ks = e4 >> 1;
                            const uint32_t x = ((r >> 1) << 7) | (L << 1) | (r & 1);
                            const uint32_t row = 2 * (q >> 1) + c, col = (q & 1) ? 1 - c : c;
                            const size_t src = ((((size_t)i * 2 + ks) * dG2 + row) * 2 + col) * N + x;
                            dev[(size_t)i * per + ((((c * kq + q) * 16 + k2) * 64 + L) * 4 + e4)] =
                                to_mont(mulmod(bsk[src] % Q, ninv, Q), Q);
                        }
    FHE_HIP_CHECK(hipSetDevice(device_));
    if (d_bsk2_) FHE_HIP_CHECK(hipFree(d_bsk2_));
    d_bsk2_ = nullptr;
    FHE_HIP_CHECK(hipMalloc(&d_bsk2_, dev.size() * 4));
    FHE_HIP_CHECK(hipMemcpy(d_bsk2_, dev.data(), dev.size() * 4, hipMemcpyHostToDevice));
}

// the split kernels' nd = 3 key layouts, u32 Montgomery with N^-1 folded in (as the resident 32-bit
// layouts).  GINX (boot.h g2_key_word) from the raw BSK [n][2][dG2 = 8][2][N]; LMKCDEY
// (launch_blind_rotate_lmk3) from [n][dG2][2][N] ++ [numAutoKeys + 1][3][2][N]
void Engine::pack_ginx3(const uint64_t* bsk) {
    const uint32_t n = p_.n, N = p_.N, dG2 = p_.digitsG2;
    const uint64_t Q = p_.Q, ninv = invmod(N, Q);
    const bool lmk = p_.method == M_LMKCDEY;
    const size_t per = lmk ? 12288 : 8192 * 3, nauto = lmk ? (size_t)p_.numAutoKeys + 1 : 0;
    std::vector<uint32_t> dev((size_t)n * per + nauto * 6144);
    auto word = [&](uint64_t v) { return to_mont(mulmod(v % Q, ninv, Q), Q); };
    if (lmk) {
        // ek [i][c][p < 6][k4 < 4][64][4]: register r = 4 k4 + e of lane L is slot x(L, r)
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < (int64_t)n; ++i)
            for (uint32_t c = 0; c < 2; ++c)
                for (uint32_t p = 0; p < 6; ++p)
                    for (uint32_t k4 = 0; k4 < 4; ++k4)
                        for (uint32_t L = 0; L < 64; ++L)
                            for (uint32_t e = 0; e < 4; ++e) {
                                const uint32_t x = (k4 << 8) | (L << 2) | e;
                                const size_t src = (((size_t)i * dG2 + g2_row(c, p, 3)) * 2 + c) * N + x;
                                dev[(size_t)i * per + ((((c * 6 + p) * 4 + k4) * 64 + L) * 4 + e)] = word(bsk[src]);
                            }
        // ak [t][c][d < 3][k4][64][4]
        const uint64_t* asrc = bsk + (size_t)n * dG2 * 2 * N;
        uint32_t* adst = dev.data() + (size_t)n * per;
        for (size_t t = 0; t < nauto; ++t)
            for (uint32_t c = 0; c < 2; ++c)
                for (uint32_t dd = 0; dd < 3; ++dd)
                    for (uint32_t k4 = 0; k4 < 4; ++k4)
                        for (uint32_t L = 0; L < 64; ++L)
                            for (uint32_t e = 0; e < 4; ++e) {
                                const uint32_t x = (k4 << 8) | (L << 2) | e;
                                adst[t * 6144 + ((((c * 3 + dd) * 4 + k4) * 64 + L) * 4 + e)] =
                                    word(asrc[((t * 3 + dd) * 2 + c) * N + x]);
                            }
    } else
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i)
        for (uint32_t c = 0; c < 2; ++c)
            for (uint32_t p = 0; p < 6; ++p)
                for (uint32_t k2 = 0; k2 < 8; ++k2)
                    for (uint32_t L = 0; L < 64; ++L)
                        for (uint32_t e4 = 0; e4 < 4; ++e4) {
                            const uint32_t r = 2 * k2 + (e4 & 1), ks = e4 >> 1;
                            const uint32_t x = ((r >> 2) << 8) | (L << 2) | (r & 3);
                            const size_t src = ((((size_t)i * 2 + ks) * dG2 + g2_row(c, p, 3)) * 2 + c) * N + x;
                            dev[(size_t)i * per + g2_key_word(3, c, p, k2, L, e4)] = to_mont(mulmod(bsk[src] % Q, ninv, Q), Q);
                        }
    FHE_HIP_CHECK(hipSetDevice(device_));
    if (d_bsk2_) FHE_HIP_CHECK(hipFree(d_bsk2_));
    d_bsk2_ = nullptr;
    FHE_HIP_CHECK(hipMalloc(&d_bsk2_, dev.size() * 4));
    FHE_HIP_CHECK(hipMemcpy(d_bsk2_, dev.data(), dev.size() * 4, hipMemcpyHostToDevice));
}

Engine::Engine(int paramset, int method, int device) : p_(make_params(paramset, method)), device_(device) {
    // Two accumulator kernels: the 32-bit one (bootstrap.hip) for N = 1024, Q < 2^28, digitsG = 3 (the
    // STD128 / MEDIUM / STD128*_LMKCDEY sets); the 64-bit one (bootstrap_wide.hip) for every other
    // GINX set with N = 1024 / 2048 (any digitsG, Q up to 2^62) and the large-precision family.
    if (is_large(paramset) || !fast_path(p_)) {
        wide_ = true;
        if (p_.N != 512 && p_.N != 1024 && p_.N != 2048)
            throw std::invalid_argument("device path supports ring dimension N = 512 / 1024 / 2048");
        if ((double)p_.digitsG2 * (double)p_.Q >= 18446744073709551616.0)
            throw std::invalid_argument("device path: digitsG2 * Q must stay below 2^64");
        if (p_.q & (p_.q - 1)) throw std::invalid_argument("device path needs a power-of-two q");
        if (p_.n > 2048) throw std::invalid_argument("device path supports n <= 2048");
        FHE_HIP_CHECK(hipSetDevice(device_));
        FHE_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
        const char* nw = std::getenv("FHE_HIP_NARROW");  // "0": keep 64-bit residues (A/B, tests)
        narrow_ = !(nw && std::string(nw) == "0") && narrow_set(p_);
        build_tables_wide();
        set_base(p_.baseG);
        if (g3_set(p_)) {
            const char* e = std::getenv("FHE_HIP_GINX3");
            g3_ = !(e && std::string(e) == "0");
            if (g3_) build_tables();
        }
        if (n2k_set(p_)) {
            const char* e = std::getenv("FHE_HIP_N2K");
            n2k_ = !(e && std::string(e) == "0");
            if (n2k_) build_tables_n2k();
        }
        if (g3_) {
            ks32_ = true;
        } else if (ks32_set(p_)) {
            const char* e = std::getenv("FHE_HIP_KS32");
            ks32_ = !(e && std::string(e) == "0");
        } else if (ks32w_set(p_)) {  // measured +5-15% (profiles/r04_ksw_bench.txt)
            const char* e = std::getenv("FHE_HIP_KS32");
            ks32w_ = !(e && std::string(e) == "0");
        }
        if (method == M_LMKCDEY) {  // op lists (k_prep_lmk_w) for k_blind_rotate_wide_ops
            if (p_.n > 2048 || (p_.numAutoKeys + 1) > 0x7fff) throw std::invalid_argument("device path: LMKCDEY n <= 2048");
            build_loggen();
            maxops_ = p_.N + p_.n + 128;
        } else if (method == M_AP) {  // op lists (k_prep_dm_w): at most digitsR ops per index
            if ((size_t)p_.n * p_.baseR * p_.digitsR > 0x8000u) throw std::invalid_argument("device path: AP keys");
            maxops_ = std::max<uint32_t>(p_.N + p_.n + 128, p_.n * p_.digitsR);
        }
        return;
    }
    if (!fast_path(p_))
        throw std::invalid_argument(
            "device path for AP / LMKCDEY: N = 1024, Q < 2^28, digitsG = 3, power-of-two q and qKS <= 2^16, n < 1024");
    FHE_HIP_CHECK(hipSetDevice(device_));
    FHE_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    build_tables();
    maxops_ = p_.N + p_.n + 128;
    // FHE_HIP_GINX_KERNEL = wave | split | xsplit: pin the GINX blind-rotation kernel (tests, A/B); default by
    // batch size (K1x below kXBatch gates, K1 above)
    if (const char* k = std::getenv("FHE_HIP_GINX_KERNEL")) {
        const std::string v(k);
        ginx_kernel_ = v == "split" ? 2 : v == "wave" ? 1 : v == "xsplit" ? 3 : v == "qsplit" ? 4 : 0;
    }
    if (const char* k = std::getenv("FHE_HIP_LMK_KERNEL")) {
        const std::string v(k);
        lmk_kernel_ = v == "split" ? 2 : v == "wave" ? 1 : v == "qsplit" ? 4 : 0;
    }
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device_) == hipSuccess && cus > 0)
        x_batch_ = 2 * (uint32_t)cus;   // K1x: one two-gate workgroup per CU
}

Engine::~Engine() {
    (void)hipSetDevice(device_);
    if (stream_) (void)hipStreamSynchronize(stream_);
    for (void* ptr : {(void*)d_tables_, d_bsk_, (void*)d_ksk_, (void*)d_idx_, (void*)d_tvb_, (void*)d_ext_a_,
                      (void*)d_ext_b_, (void*)d_io_, (void*)d_l1_, (void*)d_mix_, (void*)d_mixio_, (void*)d_tvbuf_, (void*)d_fb_, (void*)d_logGen_, (void*)d_ops_, (void*)d_nops_,
                      d_wtables_, (void*)d_wksk_, (void*)d_wext_a_, (void*)d_wext_b_,
                      (void*)d_epk_, (void*)d_epops_, (void*)d_epn_, d_bsk2_, (void*)d_kspart_, d_tables2k_,
                      (void*)d_ksk32_})
        if (ptr) (void)hipFree(ptr);
    if (order_ev_) (void)hipEventDestroy(order_ev_);
    if (stream_) (void)hipStreamDestroy(stream_);
}

hipStream_t Engine::use_stream(hipStream_t s) {
    if (!s) s = stream_;
    if (last_stream_ && s != last_stream_) {  // order after the previous call's work on its stream
        FHE_HIP_CHECK(hipSetDevice(device_));
        // the context's own stream is alive for the context's lifetime: its ordering point is taken
        // now (it covers a synchronous call that threw after enqueueing work); a caller's stream was
        // marked by that call's end_call (capi CallOrder, on every exit path)
        if (last_stream_ == stream_) end_call(stream_);
        if (pending_) FHE_HIP_CHECK(hipStreamWaitEvent(s, order_ev_, 0));
    }
    last_stream_ = s;
    return s;
}

void Engine::end_call(hipStream_t s) {
    FHE_HIP_CHECK(hipSetDevice(device_));
    if (!order_ev_) FHE_HIP_CHECK(hipEventCreateWithFlags(&order_ev_, hipEventDisableTiming));
    FHE_HIP_CHECK(hipEventRecord(order_ev_, s));
    pending_ = true;
}

void Engine::sync_streams() {
    FHE_HIP_CHECK(hipSetDevice(device_));
    FHE_HIP_CHECK(hipStreamSynchronize(stream_));
    if (pending_) FHE_HIP_CHECK(hipEventSynchronize(order_ev_));
}

void Engine::build_tables() {
    const uint64_t Q = p_.Q;
    HostNtt h;
    h.init(p_.N, Q, p_.psi);
    std::vector<uint32_t> t(32 + 32 + 992 + 992 + 2 * (kMonoHalfWords + kMonoTableWords) + 2048, 0);
    uint32_t* twAf = t.data();
    uint32_t* twAi = twAf + 32;
    uint32_t* twBf = twAi + 32;
    uint32_t* twBi = twBf + 992;
    uint32_t* mono = twBi + 992;
    uint32_t* monoF = mono + kMonoHalfWords;
    uint32_t* monoP = monoF + kMonoTableWords;
    uint32_t* monoPF = monoP + kMonoHalfWords;
    uint32_t* tabI = monoPF + kMonoTableWords;
    uint32_t* tabF = tabI + 1024;
    for (uint32_t i = 0; i < 1024 && i < p_.N; ++i) {
        tabI[i] = to_mont(h.tabI[i], Q);
        tabF[i] = to_mont(h.tab[i], Q);
    }
    for (int i = 0; i < 32; ++i) {
        twAf[i] = to_mont(h.tab[i], Q);
        twAi[i] = to_mont(h.tabI[i], Q);
    }
    // lane-major tables of the stages on bits 4..0 (bootstrap.hip, twb_off)
    for (int b = 4; b >= 0; --b) {
        const int per = 1 << (4 - b), off = 32 * (per - 1);
        for (int k = 0; k < per; ++k)
            for (int l = 0; l < 32; ++l) {
                const size_t idx = (size_t)(1 << (9 - b)) + (size_t)l * per + k;
                twBf[off + k * 32 + l] = to_mont(h.tab[idx], Q);
                twBi[off + k * 32 + l] = to_mont(h.tabI[idx], Q);
            }
    }
    // EVAL(X^m - 1) at slot j = omega_j^m - 1 with omega_j = psi^(2 brv(j) + 1) (bootstrap.hip,
    // monomial addressing).  Gates (m = a_i * 2N/q, 2N/q = 2) have even exponents: the
    // half-resolution table psi^(2f) - 1, f in [0, 2N].  BootstrapFunc with ciphertext modulus
    // 2N has any exponent: the full table psi^e - 1, e in [0, 4N].  Entry k at k + (k >> 5).
    {
        const uint64_t psi2 = mulmod(p_.psi, p_.psi, Q);
        uint64_t x = 1;
        for (uint32_t f = 0; f <= 2 * p_.N; ++f) {
            mono[f + (f >> 5)] = to_mont(submod(x, 1, Q), Q);
            monoP[f + (f >> 5)] = (uint32_t)submod(x, 1, Q);
            x = mulmod(x, psi2, Q);
        }
        x = 1;
        for (uint32_t e = 0; e <= 4 * p_.N; ++e) {
            monoF[e + (e >> 5)] = to_mont(submod(x, 1, Q), Q);
            monoPF[e + (e >> 5)] = (uint32_t)submod(x, 1, Q);
            x = mulmod(x, p_.psi, Q);
        }
    }
    if (p_.method == M_LMKCDEY) build_loggen();
    FHE_HIP_CHECK(hipMalloc(&d_tables_, t.size() * 4));
    FHE_HIP_CHECK(hipMemcpy(d_tables_, t.data(), t.size() * 4, hipMemcpyHostToDevice));
    const uint32_t* d = static_cast<const uint32_t*>(d_tables_);
    tabs_.twA_fwd = d;
    tabs_.twA_inv = d + 32;
    tabs_.twB_fwd = d + 64;
    tabs_.twB_inv = d + 64 + 992;
    tabs_.mono = d + 64 + 1984;                     // kMonoHalfWords words
    tabs_.mono_full = tabs_.mono + kMonoHalfWords;  // kMonoTableWords words
    tabs_.monoP = tabs_.mono_full + kMonoTableWords;
    tabs_.monoP_full = tabs_.monoP + kMonoHalfWords;
    tabs_.tabI = tabs_.monoP_full + kMonoTableWords;
    tabs_.tabF = tabs_.tabI + 1024;
    tabs_.Q = (uint32_t)Q;
    tabs_.Q2 = (uint32_t)(2 * Q);
    tabs_.qinv = neg_inv32((uint32_t)Q);
    tabs_.ninvR = to_mont(h.ninv, Q);
    tabs_.w1R = to_mont(h.tabI[1], Q);
    tabs_.oneR = to_mont(1, Q);
    tabs_.nR = to_mont(p_.N, Q);
}

// logGen of rgsw-cryptoparameters.cpp:115-127 (k_prep_lmk_w's group positions)
void Engine::build_loggen() {
    if (d_logGen_) return;
    const uint32_t M = 2 * p_.N;
    std::vector<int16_t> lg(M, 0);
    uint32_t gp = 1;
    lg[M - gp] = (int16_t)M;
    for (uint32_t i = 1; i < p_.N / 2; ++i) {
        gp = (gp * 5) % M;
        lg[gp] = (int16_t)i;
        lg[M - gp] = (int16_t)-(int32_t)i;
    }
    FHE_HIP_CHECK(hipMalloc(&d_logGen_, M * sizeof(int16_t)));
    FHE_HIP_CHECK(hipMemcpy(d_logGen_, lg.data(), M * sizeof(int16_t), hipMemcpyHostToDevice));
}

void Engine::set_base(uint32_t bg) {
    cur_ = p_.timeopt ? p_.with_base(bg) : p_;
    cur_off_ = p_.bsk_offset(bg);
    cur_ksk_off_ = p_.ksk_index(bg) * p_.ksk_rows() * ((size_t)p_.n + 1);
}

void Engine::build_tables_wide() {
    const uint64_t Q = p_.Q;
    const uint32_t N = p_.N;
    HostNtt h;
    h.init(N, Q, p_.psi);
    std::vector<uint64_t> t(6 * (size_t)N);
    for (uint32_t i = 0; i < N; ++i) {
        t[i] = h.tab[i];
        t[N + i] = shoup64(h.tab[i], Q);
        t[2 * N + i] = h.tabI[i];
        t[3 * N + i] = shoup64(h.tabI[i], Q);
    }
    const uint64_t R = (uint64_t)(((u128)1 << 64) % Q);  // Montgomery 1
    uint64_t x = 1;
    for (uint32_t e = 0; e < 2 * N; ++e) {
        t[4 * N + e] = mulmod(x, R, Q);
        x = mulmod(x, p_.psi, Q);
    }
    // the 32-bit policy's copies (A32): Shoup quotients floor(w 2^32 / Q), psi^e 2^32 mod Q
    const size_t w32 = narrow_ ? 6 * (size_t)N : 0;  // tab, tabS, tabI, tabIS (N each), psiM (2N)
    std::vector<uint64_t> t32((w32 + 1) / 2, 0);
    uint32_t* n32 = reinterpret_cast<uint32_t*>(t32.data());
    if (narrow_) {
        auto shoup32 = [&](uint64_t w) { return (uint32_t)(((u128)w << 32) / Q); };
        for (uint32_t i = 0; i < N; ++i) {
            n32[i] = (uint32_t)h.tab[i];
            n32[N + i] = shoup32(h.tab[i]);
            n32[2 * N + i] = (uint32_t)h.tabI[i];
            n32[3 * N + i] = shoup32(h.tabI[i]);
        }
        const uint64_t R32 = (1ull << 32) % Q;
        uint64_t y = 1;
        for (uint32_t e = 0; e < 2 * N; ++e) {
            n32[4 * N + e] = (uint32_t)mulmod(y, R32, Q);
            y = mulmod(y, p_.psi, Q);
        }
        wtabs_.narrow = 1;
        wtabs_.Q32 = (uint32_t)Q;
        wtabs_.qinv32 = neg_inv32((uint32_t)Q);
        wtabs_.ninv32 = (uint32_t)h.ninv;
        wtabs_.ninvS32 = shoup32(h.ninv);
        wtabs_.oneM32 = (uint32_t)R32;
        wtabs_.r2_32 = (uint32_t)mulmod(R32, R32, Q);
    }
    t.insert(t.end(), t32.begin(), t32.end());
    FHE_HIP_CHECK(hipMalloc(&d_wtables_, t.size() * 8));
    FHE_HIP_CHECK(hipMemcpy(d_wtables_, t.data(), t.size() * 8, hipMemcpyHostToDevice));
    const uint64_t* d = static_cast<const uint64_t*>(d_wtables_);
    if (narrow_) {
        const uint32_t* d32 = reinterpret_cast<const uint32_t*>(d + 6 * (size_t)N);
        wtabs_.tab32 = d32;
        wtabs_.tabS32 = d32 + N;
        wtabs_.tabI32 = d32 + 2 * N;
        wtabs_.tabIS32 = d32 + 3 * N;
        wtabs_.psiM32 = d32 + 4 * N;
    }
    wtabs_.tab = d;
    wtabs_.tabS = d + N;
    wtabs_.tabI = d + 2 * N;
    wtabs_.tabIS = d + 3 * N;
    wtabs_.psiM = d + 4 * N;
    wtabs_.Q = Q;
    uint64_t inv = Q;  // Q^-1 mod 2^64 (Newton)
    for (int i = 0; i < 6; ++i) inv *= 2 - Q * inv;
    wtabs_.qinv = 0 - inv;
    wtabs_.ninv = h.ninv;
    wtabs_.ninvS = shoup64(h.ninv, Q);
    wtabs_.oneM = R;
    wtabs_.r2 = mulmod(R, R, Q);
}

void Engine::load_bsk(const uint64_t* bsk, size_t words) {
    if (!bsk) throw std::invalid_argument("bsk is null");
    if (words != p_.bsk_words()) throw std::invalid_argument("bsk has wrong length");
    if (wide_) {  // raw layout [n][2][dG2][2][N], Montgomery form K R mod Q (bootstrap_wide.hip), R = 2^64
                  // (u64 words) or 2^32 (u32 words, narrow_)
        const uint64_t Q = p_.Q;
        const unsigned sh = narrow_ ? 32 : 64;
        const size_t wb = narrow_ ? 4 : 8;
        std::vector<uint64_t> dev((words * wb + 7) / 8);
        uint32_t* d32 = reinterpret_cast<uint32_t*>(dev.data());
        bool bad = false;
#pragma omp parallel for schedule(static) reduction(|| : bad)
        for (int64_t i = 0; i < (int64_t)words; ++i) {
            bad = bad || bsk[i] >= Q;
            const uint64_t v = (uint64_t)(((u128)(bsk[i] % Q) << sh) % Q);
            if (narrow_) d32[i] = (uint32_t)v;
            else dev[i] = v;
        }
        if (bad) throw std::invalid_argument("bsk coefficient not reduced mod Q");
        FHE_HIP_CHECK(hipSetDevice(device_));
        if (d_bsk_) FHE_HIP_CHECK(hipFree(d_bsk_));
        d_bsk_ = nullptr;
        FHE_HIP_CHECK(hipMalloc(&d_bsk_, words * wb));
        FHE_HIP_CHECK(hipMemcpy(d_bsk_, dev.data(), words * wb, hipMemcpyHostToDevice));
        if (g3_) pack_ginx3(bsk);
        if (n2k_) pack_n2k(bsk);
        return;
    }
    const uint32_t n = p_.n, N = p_.N, dG2 = p_.digitsG2;
    const uint64_t Q = p_.Q;
    if (dG2 != 4) throw std::invalid_argument("device path expects digitsG = 3");
    // device uint2 blocks [..][d][16][64 lanes]: lane = h*32 + l holds slots l*32 + 2k, +1 of
    // component h -- one 512-byte coalesced load per wave-instruction in the kernels.  With
    // kBskHalfSwap the half-1 lanes of position d hold row d ^ 1 (rows come in pairs).
    //   GINX   raw [n][2][dG2][2][N]                 -> [n][2][dG2][16][64]
    //   LMKCDEY raw [n][dG2][2][N] ++ [nA+1][2][2][N] -> [n][dG2][16][64] ++ [nA+1][2][16][64]
    //   AP     raw [n][baseR][digitsR][dG2][2][N]    -> [n][baseR][digitsR][dG2][16][64]
    const size_t nrgsw = p_.method == M_GINX ? (size_t)n * 2
                         : p_.method == M_AP ? (size_t)n * p_.baseR * p_.digitsR
                                             : (size_t)n;  // RGSW keys of dG2 rows
    const size_t nauto = p_.method == M_LMKCDEY ? (size_t)p_.numAutoKeys + 1 : 0;
    const uint32_t dA = p_.digitsG - 1;
    std::vector<uint32_t> dev(nrgsw * dG2 * 2 * N + nauto * dA * 2 * N);
    // keys carry N^-1 (BootTables::w1R): the kernels' last inverse stage skips the N^-1 multiply
    const uint64_t ninv = invmod(N, Q);
    auto pack = [&](const uint64_t* src_key, uint32_t rows, uint32_t* dst_key) {
        for (uint32_t d = 0; d < rows; ++d)
            for (uint32_t k = 0; k < 16; ++k)
                for (uint32_t lane = 0; lane < 64; ++lane) {
                    const uint32_t h = lane >> 5, l = lane & 31;
                    const uint32_t row = kBskHalfSwap ? d ^ h : d;  // boot.h kBskHalfSwap
                    const size_t src = ((size_t)row * 2 + h) * N + l * 32 + 2 * k;
                    const size_t dst = row_off(d, k, lane, 0);  // boot.h
                    dst_key[dst] = to_mont(mulmod(src_key[src] % Q, ninv, Q), Q);
                    dst_key[dst + 1] = to_mont(mulmod(src_key[src + 1] % Q, ninv, Q), Q);
                }
    };
    if (kGinxU4 && p_.method == M_GINX) {
        // (BSK+, BSK-) of index i interleaved per lane (boot.h ginx_u4_off)
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < (int64_t)n; ++i)
            for (uint32_t ks = 0; ks < 2; ++ks) {
                const uint64_t* src_key = bsk + ((size_t)i * 2 + ks) * dG2 * 2 * N;
                uint32_t* dst_key = dev.data() + (size_t)i * 2 * dG2 * 2 * N;
                for (uint32_t d = 0; d < dG2; ++d)
                    for (uint32_t k = 0; k < 16; ++k)
                        for (uint32_t lane = 0; lane < 64; ++lane) {
                            const uint32_t h = lane >> 5, l = lane & 31;
                            const uint32_t row = kBskHalfSwap ? d ^ h : d;
                            const size_t src = ((size_t)row * 2 + h) * N + l * 32 + 2 * k;
                            for (uint32_t e = 0; e < 2; ++e)
                                dst_key[ginx_u4_off(ks, d, k, lane, e)] = to_mont(mulmod(src_key[src + e] % Q, ninv, Q), Q);
                        }
            }
    } else {
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < (int64_t)nrgsw; ++i)
            pack(bsk + (size_t)i * dG2 * 2 * N, dG2, dev.data() + (size_t)i * dG2 * 2 * N);
    }
    const uint64_t* asrc = bsk + nrgsw * dG2 * 2 * N;
    uint32_t* adst = dev.data() + nrgsw * dG2 * 2 * N;
    for (size_t t = 0; t < nauto; ++t) pack(asrc + t * dA * 2 * N, dA, adst + t * dA * 2 * N);
    for (size_t i = 0; i < words; ++i)
        if (bsk[i] >= Q) throw std::invalid_argument("bsk coefficient not reduced mod Q");
    FHE_HIP_CHECK(hipSetDevice(device_));
    if (d_bsk_) FHE_HIP_CHECK(hipFree(d_bsk_));
    d_bsk_ = nullptr;
    FHE_HIP_CHECK(hipMalloc(&d_bsk_, dev.size() * 4));
    FHE_HIP_CHECK(hipMemcpy(d_bsk_, dev.data(), dev.size() * 4, hipMemcpyHostToDevice));
    d_autok_ = static_cast<uint32_t*>(d_bsk_) + nrgsw * dG2 * 2 * N;
    repack_ginx2();
}

// the two-wave GINX kernels' key layouts, repacked on the device from the resident one: K1s's
// (k_blind_rotate_ginx2, FHE_HIP_GINX_KERNEL=split) or K1x's (k_blind_rotate_ginx2x, the small-batch default)
void Engine::repack_ginx2() {
    if (p_.method == M_LMKCDEY && !wide_ && d_bsk_ && lmk_kernel_ != 1) {  // K1m's two-digit form
        FHE_HIP_CHECK(hipSetDevice(device_));
        const uint32_t nauto = p_.numAutoKeys + 1;
        if (!d_bsk2_) FHE_HIP_CHECK(hipMalloc(&d_bsk2_, ((size_t)p_.n * 8192 + (size_t)nauto * 4096) * 4));
        FHE_HIP_CHECK(launch_repack_lmkx(d_bsk_, p_.n, nauto, d_bsk2_, stream_));
        FHE_HIP_CHECK(hipStreamSynchronize(stream_));
        return;
    }
    if (p_.method != M_GINX || wide_ || !d_bsk_ || ginx_kernel_ == 1 || (ginx_kernel_ == 0 && x_batch_ == 0)) return;
    FHE_HIP_CHECK(hipSetDevice(device_));
    if (!d_bsk2_) FHE_HIP_CHECK(hipMalloc(&d_bsk2_, (size_t)p_.n * 16384 * 4));
    if (ginx_kernel_ == 2) FHE_HIP_CHECK(launch_repack_ginx2(d_bsk_, p_.n, d_bsk2_, stream_));
    else FHE_HIP_CHECK(launch_repack_ginx2x(d_bsk_, p_.n, d_bsk2_, stream_));
    FHE_HIP_CHECK(hipStreamSynchronize(stream_));
}

void Engine::load_ksk(const uint64_t* A, size_t nA, const uint64_t* B, size_t nB) {
    if (!A || !B) throw std::invalid_argument("ksk is null");
    const size_t rows = p_.ksk_rows();
    if (nA != p_.ksk_rows_all() * p_.n || nB != p_.ksk_rows_all())
        throw std::invalid_argument(p_.timeopt ? "ksk has wrong length (timeOptimization: the map's three switching keys)"
                                               : "ksk has wrong length");
    if (wide_) {  // u64 A [rows][n] ++ B [rows] as given, per key of the map
        bool bad = false;
#pragma omp parallel for schedule(static) reduction(|| : bad)
        for (int64_t r = 0; r < (int64_t)nA; ++r) bad = bad || A[r] >= p_.qKS;
        for (size_t r = 0; r < nB; ++r) bad = bad || B[r] >= p_.qKS;
        if (bad) throw std::invalid_argument("ksk value not reduced mod qKS");
        FHE_HIP_CHECK(hipSetDevice(device_));
        if (d_wksk_) FHE_HIP_CHECK(hipFree(d_wksk_));
        d_wksk_ = nullptr;
        FHE_HIP_CHECK(hipMalloc(&d_wksk_, (nA + nB) * 8));
        const size_t one = rows * ((size_t)p_.n + 1);
        for (size_t k = 0; k < p_.ksk_keys(); ++k) {
            FHE_HIP_CHECK(hipMemcpy(d_wksk_ + k * one, A + k * rows * p_.n, rows * p_.n * 8, hipMemcpyHostToDevice));
            FHE_HIP_CHECK(hipMemcpy(d_wksk_ + k * one + rows * p_.n, B + k * rows, rows * 8, hipMemcpyHostToDevice));
        }
        if (ks32w_) {  // u32 rows of launch_keyswitch_w32: A then B at column n, zero-padded
            const size_t W = ksk_width(p_.n);
            std::vector<uint32_t> dev(rows * W, 0);
#pragma omp parallel for schedule(static)
            for (int64_t r = 0; r < (int64_t)rows; ++r) {
                for (uint32_t k = 0; k < p_.n; ++k) dev[(size_t)r * W + k] = (uint32_t)A[(size_t)r * p_.n + k];
                dev[(size_t)r * W + p_.n] = (uint32_t)B[r];
            }
            if (d_ksk32_) FHE_HIP_CHECK(hipFree(d_ksk32_));
            d_ksk32_ = nullptr;
            FHE_HIP_CHECK(hipMalloc(&d_ksk32_, dev.size() * 4));
            FHE_HIP_CHECK(hipMemcpy(d_ksk32_, dev.data(), dev.size() * 4, hipMemcpyHostToDevice));
            return;
        }
        if (!ks32_) return;
        // ks32_: also the u16 rows of the 32-bit key switch (qKS <= 2^16; ks32_set)
    }
    const size_t W = ksk_width(p_.n);
    std::vector<uint16_t> dev(rows * W, 0);
    bool bad = false;
#pragma omp parallel for schedule(static) reduction(|| : bad)
    for (int64_t r = 0; r < (int64_t)rows; ++r) {
        for (uint32_t k = 0; k < p_.n; ++k) {
            const uint64_t v = A[(size_t)r * p_.n + k];
            bad = bad || v >= p_.qKS;
            dev[(size_t)r * W + k] = (uint16_t)v;
        }
        bad = bad || B[r] >= p_.qKS;
        dev[(size_t)r * W + p_.n] = (uint16_t)B[r];
    }
    if (bad) throw std::invalid_argument("ksk value not reduced mod qKS");
    FHE_HIP_CHECK(hipSetDevice(device_));
    if (d_ksk_) FHE_HIP_CHECK(hipFree(d_ksk_));
    d_ksk_ = nullptr;
    FHE_HIP_CHECK(hipMalloc(&d_ksk_, dev.size() * 2));
    FHE_HIP_CHECK(hipMemcpy(d_ksk_, dev.data(), dev.size() * 2, hipMemcpyHostToDevice));
}

void Engine::copy_keys_from(const Engine& src) {
    if (src.p_.paramset != p_.paramset || src.p_.method != p_.method)
        throw std::invalid_argument("copy_keys_from: another parameter set");
    // the packed layouts also follow knobs each context read from the environment at creation (word size of
    // the wide keys, which layout d_bsk2_ holds, the key switch's row form): a copy between contexts created
    // under different knobs would hand a kernel buffers of another layout
    const int two_src = src.ginx_kernel_ == 1 ? 0 : src.ginx_kernel_ == 2 ? 2 : 3;
    const int two_dst = ginx_kernel_ == 1 ? 0 : ginx_kernel_ == 2 ? 2 : 3;
    if (src.wide_ != wide_ || src.narrow_ != narrow_ || src.g3_ != g3_ || src.n2k_ != n2k_ || src.ks32_ != ks32_ ||
        src.ks32w_ != ks32w_ || (!wide_ && p_.method == M_GINX && two_src != two_dst) ||
        (!wide_ && p_.method == M_LMKCDEY && (src.lmk_kernel_ == 1) != (lmk_kernel_ == 1)))
        throw std::invalid_argument("copy_keys_from: the contexts pack their keys in different layouts "
                                    "(created under different FHE_HIP_* kernel settings)");
    if (!src.ready()) throw std::logic_error("copy_keys_from: the source context has no keys");
    if (src.device_ != device_) {
        int can = 0;
        FHE_HIP_CHECK(hipDeviceCanAccessPeer(&can, device_, src.device_));
        if (can) {
            FHE_HIP_CHECK(hipSetDevice(device_));
            const hipError_t e = hipDeviceEnablePeerAccess(src.device_, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) throw HipError(e, "hipDeviceEnablePeerAccess");
            (void)hipGetLastError();
        }
    }
    auto dup = [&](void*& dst, const void* from) {
        FHE_HIP_CHECK(hipSetDevice(device_));
        if (dst) FHE_HIP_CHECK(hipFree(dst));
        dst = nullptr;
        if (!from) return;
        hipDeviceptr_t base = nullptr;
        size_t bytes = 0;
        FHE_HIP_CHECK(hipSetDevice(src.device_));
        FHE_HIP_CHECK(hipMemGetAddressRange(&base, &bytes, const_cast<void*>(from)));
        if (base != from) throw std::logic_error("copy_keys_from: not an allocation base");
        FHE_HIP_CHECK(hipSetDevice(device_));
        FHE_HIP_CHECK(hipMalloc(&dst, bytes));
        if (src.device_ == device_)
            FHE_HIP_CHECK(hipMemcpyAsync(dst, from, bytes, hipMemcpyDeviceToDevice, stream_));
        else
            FHE_HIP_CHECK(hipMemcpyPeerAsync(dst, device_, from, src.device_, bytes, stream_));
    };
    sync_streams();
    const_cast<Engine&>(src).sync_streams();
    dup(d_bsk_, src.d_bsk_);
    d_autok_ = src.d_autok_ ? static_cast<char*>(d_bsk_) + (static_cast<const char*>(src.d_autok_) -
                                                            static_cast<const char*>(src.d_bsk_))
                            : nullptr;
    dup(d_bsk2_, src.d_bsk2_);
    void* k = d_ksk_;
    dup(k, src.d_ksk_);
    d_ksk_ = static_cast<uint16_t*>(k);
    k = d_ksk32_;
    dup(k, src.d_ksk32_);
    d_ksk32_ = static_cast<uint32_t*>(k);
    k = d_wksk_;
    dup(k, src.d_wksk_);
    d_wksk_ = static_cast<uint64_t*>(k);
    FHE_HIP_CHECK(hipStreamSynchronize(stream_));
}

void Engine::keygen_device(const uint64_t* sk, size_t n, uint64_t seed, uint64_t* bsk_out, uint64_t* kskA_out,
                           uint64_t* kskB_out) {
    if (!sk) throw std::invalid_argument("secret key is null");
    if (n != p_.n) throw std::invalid_argument("secret key has wrong length");
    const std::vector<uint64_t> s(sk, sk + n);
    if (wide_) {  // large-precision family: the host generator (keygen.cpp), then the upload
        KeySet ks;
        keygen_bootstrap(p_, s, seed, ks);
        load_bsk(ks.bsk.data(), ks.bsk.size());
        load_ksk(ks.kskA.data(), ks.kskA.size(), ks.kskB.data(), ks.kskB.size());
        if (bsk_out) std::copy(ks.bsk.begin(), ks.bsk.end(), bsk_out);
        if (kskA_out) std::copy(ks.kskA.begin(), ks.kskA.end(), kskA_out);
        if (kskB_out) std::copy(ks.kskB.begin(), ks.kskB.end(), kskB_out);
        return;
    }
    const size_t words = p_.bsk_words(), rows = p_.ksk_rows();
    FHE_HIP_CHECK(hipSetDevice(device_));
    if (d_bsk_) FHE_HIP_CHECK(hipFree(d_bsk_));
    if (d_ksk_) FHE_HIP_CHECK(hipFree(d_ksk_));
    d_bsk_ = d_autok_ = nullptr;
    d_ksk_ = nullptr;
    void* raw = nullptr;
    uint64_t *rb = nullptr, *ra = nullptr, *rk = nullptr;
    try {
        FHE_HIP_CHECK(hipMalloc(&d_bsk_, words * 4));
        FHE_HIP_CHECK(hipMalloc(&d_ksk_, rows * ksk_width(p_.n) * 2));
        const size_t raw_words = (bsk_out ? words : 0) + (kskA_out ? rows * p_.n : 0) + (kskB_out ? rows : 0);
        if (raw_words) FHE_HIP_CHECK(hipMalloc(&raw, raw_words * 8));
        uint64_t* cur = static_cast<uint64_t*>(raw);
        if (bsk_out) { rb = cur; cur += words; }
        if (kskA_out) { ra = cur; cur += rows * p_.n; }
        if (kskB_out) rk = cur;
        keygen_bootstrap_device(p_, s, seed, device_, static_cast<uint32_t*>(d_bsk_), d_ksk_, rb, ra, rk, stream_);
        if (rb) FHE_HIP_CHECK(hipMemcpy(bsk_out, rb, words * 8, hipMemcpyDeviceToHost));
        if (ra) FHE_HIP_CHECK(hipMemcpy(kskA_out, ra, rows * p_.n * 8, hipMemcpyDeviceToHost));
        if (rk) FHE_HIP_CHECK(hipMemcpy(kskB_out, rk, rows * 8, hipMemcpyDeviceToHost));
    } catch (...) {
        if (raw) (void)hipFree(raw);
        if (d_bsk_) (void)hipFree(d_bsk_);
        if (d_ksk_) (void)hipFree(d_ksk_);
        d_bsk_ = nullptr;
        d_ksk_ = nullptr;
        throw;
    }
    if (raw) FHE_HIP_CHECK(hipFree(raw));
    const size_t nrgsw = p_.method == M_GINX ? (size_t)p_.n * 2
                         : p_.method == M_AP ? (size_t)p_.n * p_.baseR * p_.digitsR
                                             : (size_t)p_.n;
    d_autok_ = static_cast<uint32_t*>(d_bsk_) + nrgsw * p_.digitsG2 * 2 * p_.N;
    repack_ginx2();
}

GateArgs Engine::gate_args(int gate, size_t count, uint32_t p, bool multi) const {
    switch (gate) {
        case G_OR: case G_AND: case G_NOR: case G_NAND: case G_XOR: case G_XNOR: case G_XOR_FAST: case G_XNOR_FAST:
            if (multi) throw std::invalid_argument("EvalBinGate(ctvector): AND3, OR3, AND4, OR4, MAJORITY or CMUX only");
            break;
        case G_MAJORITY: case G_AND3: case G_OR3: case G_AND4: case G_OR4:
            if (!multi) throw std::invalid_argument("EvalBinGate: multi-input gates take a ciphertext vector");
            break;
        default:
            throw std::invalid_argument("EvalBinGate: unsupported gate");
    }
    if (count > 0x7fffffffull) throw std::invalid_argument("batch too large");
    if (p < 2 || 2 * p > p_.q) throw std::invalid_argument("plaintext modulus out of range");
    GateArgs g{};
    g.count = (uint32_t)count;
    g.n = p_.n;
    g.N = p_.N;
    g.q = p_.q;
    g.qKS = p_.qKS;
    g.ctmod = p_.q;
    g.tv = nullptr;
    // BootstrapGateCore window (binfhe-base-scheme.cpp:535-553); Q2p = Q/(2p) + 1 (:555-556)
    const uint64_t q = p_.q, qHalf = q >> 1, Q = p_.Q;
    const uint64_t q1 = p_.gate_const(gate), q2 = (q1 + qHalf) % q;
    const bool swap = q1 >= q2;
    g.lb = (uint32_t)(swap ? q2 : q1);
    g.ub = (uint32_t)(swap ? q1 : q2);
    const uint64_t Q2p = Q / (2 * p) + 1, Q2pNeg = Q - Q2p;
    g.lv = (uint32_t)(swap ? Q2p : Q2pNeg);
    g.uv = (uint32_t)(swap ? Q2pNeg : Q2p);
    g.factor = (uint32_t)(p_.N / qHalf);
    // b = Q/8 + 1 for 2-input gates (:118, hardcoded p = 4), Q/(2p) + 1 for ctvector gates (:162)
    g.b_const = (uint32_t)(multi ? Q / (2 * p) + 1 : (Q >> 3) + 1);
    g.lv64 = swap ? Q2p : Q2pNeg;
    g.uv64 = swap ? Q2pNeg : Q2p;
    g.b64 = multi ? Q / (2 * p) + 1 : (Q >> 3) + 1;
    g.tv64 = nullptr;
    g.xor_double = (gate == G_XOR || gate == G_XNOR || gate == G_XOR_FAST || gate == G_XNOR_FAST) ? 1 : 0;
    g.msb_out = 1;
    g.gbits = p_.gBits;
    return g;
}

void Engine::ensure_work(size_t count) {
    if (count <= cap_) return;
    sync_streams();
    for (void* ptr : {(void*)d_idx_, (void*)d_tvb_, (void*)d_ext_a_, (void*)d_ext_b_, (void*)d_wext_a_, (void*)d_wext_b_})
        if (ptr) FHE_HIP_CHECK(hipFree(ptr));
    d_idx_ = nullptr; d_tvb_ = nullptr; d_ext_a_ = nullptr; d_ext_b_ = nullptr; cap_ = 0; rot_count_ = 0;
    d_wext_a_ = nullptr; d_wext_b_ = nullptr;
    FHE_HIP_CHECK(hipMalloc(&d_idx_, count * p_.n * sizeof(uint16_t)));
    FHE_HIP_CHECK(hipMalloc(&d_tvb_, count * sizeof(uint32_t)));
    if (wide_) {
        FHE_HIP_CHECK(hipMalloc(&d_wext_a_, count * p_.N * sizeof(uint64_t)));
        FHE_HIP_CHECK(hipMalloc(&d_wext_b_, count * sizeof(uint64_t)));
    }
    if (!wide_ || ks32_ || ks32w_) {  // ks32_ / ks32w_: the tiled key switch's u32 input (keyswitch_ext)
        FHE_HIP_CHECK(hipMalloc(&d_ext_a_, count * p_.N * sizeof(uint32_t)));
        FHE_HIP_CHECK(hipMalloc(&d_ext_b_, count * sizeof(uint32_t)));
    }
    if (p_.method == M_LMKCDEY || p_.method == M_AP) {
        for (void* ptr : {(void*)d_ops_, (void*)d_nops_})
            if (ptr) FHE_HIP_CHECK(hipFree(ptr));
        d_ops_ = nullptr; d_nops_ = nullptr;
        FHE_HIP_CHECK(hipMalloc(&d_ops_, count * maxops_ * sizeof(uint16_t)));
        FHE_HIP_CHECK(hipMalloc(&d_nops_, count * sizeof(uint32_t)));
    }
    cap_ = count;
}

void Engine::ensure_host_stage(size_t count) {
    if (count <= hcap_) return;
    sync_streams();
    if (d_io_) FHE_HIP_CHECK(hipFree(d_io_));
    d_io_ = nullptr;
    hcap_ = 0;
    const size_t words = count * (4 * ((size_t)p_.n + 1) + p_.N + 1);
    FHE_HIP_CHECK(hipMalloc(&d_io_, words * 8));
    hcap_ = count;
}

void Engine::prep_device(const GateArgs& g, const GateInputs& in, size_t offset, hipStream_t s) {
    if (p_.method == M_GINX) {
        FHE_HIP_CHECK(launch_prep_ginx(g, in, d_idx_ + offset * p_.n, d_tvb_ + offset, s));
    } else if (p_.method == M_AP) {
        if (g.ctmod != p_.q)  // EvalAcc DM reads a_i modulo the parameter q (rgsw-acc-dm.cpp:64-69)
            throw std::invalid_argument("AP accumulator: ciphertext modulus must be q");
        FHE_HIP_CHECK(launch_prep_dm(g, in, d_ops_ + offset * maxops_, d_nops_ + offset, d_tvb_ + offset, maxops_,
                                     p_.baseR, p_.digitsR, s));
    } else {
        FHE_HIP_CHECK(launch_prep_lmk(g, in, d_logGen_, d_ops_ + offset * maxops_,
                                      d_nops_ + offset, d_tvb_ + offset, maxops_, p_.numAutoKeys, s));
    }
}

void Engine::rotate_device(const GateArgs& g, hipStream_t s) {
    rot_count_ = g.count;
    if (wide_) {
        WideArgs w{};
        w.count = g.count;
        w.n = g.n;
        w.N = g.N;
        w.ctmod = g.ctmod;
        w.factor = g.factor;
        w.lb = g.lb;
        w.ub = g.ub;
        w.digitsG = cur_.digitsG;
        w.gbits = cur_.gBits;
        w.msb_out = g.msb_out;
        w.lv = g.lv64;
        w.uv = g.uv64;
        w.b_const = g.b64;
        w.qKS = p_.qKS;
        w.tv = g.tv64;
        w.acc_io = g.acc_io;
        w.acc_tv = g.acc_tv;
        w.tv_mod = g.tv_mod;
        if (g3_ && p_.method == M_LMKCDEY && d_bsk2_ && g.lv == g.lv64 && g.uv == g.uv64 && g.b_const == g.b64 &&
            !g.tv && !g.tv64) {
            const uint32_t* ek = static_cast<const uint32_t*>(d_bsk2_);
            FHE_HIP_CHECK(launch_blind_rotate_lmk3(g, tabs_, ek, ek + (size_t)p_.n * 12288, d_ops_, d_nops_, maxops_,
                                                   d_tvb_, d_wext_a_, d_wext_b_, s));
            return;
        }
        const int nd = (int)p_.digitsG - 1;
        if (n2k_ && p_.method == M_LMKCDEY && d_bsk2_ && lmk2k_supported(g, tabs2k_, nd) && g.lv == g.lv64 &&
            g.uv == g.uv64 && g.b_const == g.b64) {
            const uint32_t* ek = static_cast<const uint32_t*>(d_bsk2_);
            const size_t per = (size_t)2 * 2 * nd * 8 * 64 * 4;  // pack_n2k's ek words per index
            FHE_HIP_CHECK(launch_blind_rotate_lmk2k(g, tabs2k_, ek, ek + (size_t)p_.n * per, d_ops_, d_nops_, maxops_,
                                                    d_tvb_, d_wext_a_, d_wext_b_, nd, s));
            return;
        }
        if (p_.method == M_LMKCDEY || p_.method == M_AP) {
            const bool dm = p_.method == M_AP;
            FHE_HIP_CHECK(launch_blind_rotate_wide_ops(w, wtabs_, wkey(0), wkey(dm ? 0 : (size_t)p_.n * p_.digitsG2 * 2 * p_.N),
                                                       d_ops_, d_nops_, maxops_, d_tvb_, d_wext_a_, d_wext_b_, dm, s));
            return;
        }
        if (n2k_ && d_bsk2_ && n2k_supported(g, tabs2k_, (int)p_.digitsG - 1) && g.lv == g.lv64 && g.uv == g.uv64 &&
            g.b_const == g.b64) {
            FHE_HIP_CHECK(launch_blind_rotate_n2k(g, tabs2k_, d_bsk2_, d_idx_, d_tvb_, d_wext_a_, d_wext_b_,
                                                  (int)p_.digitsG - 1, s));
            return;
        }
        if (g3_ && d_bsk2_ && ginx3_supported(g, tabs_) && g.lv == g.lv64 && g.uv == g.uv64 && g.b_const == g.b64) {
            FHE_HIP_CHECK(launch_blind_rotate_ginx3(g, tabs_, d_bsk2_, d_idx_, d_tvb_, d_wext_a_, d_wext_b_, s));
            return;
        }
        FHE_HIP_CHECK(launch_blind_rotate_wide(w, wtabs_, wkey(cur_off_), d_idx_, d_tvb_, d_wext_a_, d_wext_b_, s));
        return;
    }
    // the kernels' digit decomposition (bootstrap.hip decompose2) works on d + C in 32 bits
    const uint64_t h = 1ull << (g.gbits - 1);
    if (g.gbits < 2 || h * (1 + (1ull << g.gbits) + (1ull << (2 * g.gbits))) + p_.Q >= (1ull << 32))
        throw std::invalid_argument("device path expects log2(baseG) <= 10");
    if (p_.method == M_GINX) {
        // two waves per gate up to x_batch_ gates (K1x: small batches would leave SIMDs idle), else one
        const int k = ginx_choice(g);
        if (k == 2)
            FHE_HIP_CHECK(launch_blind_rotate_ginx2(g, tabs_, d_bsk2_, d_idx_, d_tvb_, d_ext_a_, d_ext_b_, s));
        else if (k == 4)
            FHE_HIP_CHECK(launch_blind_rotate_ginx4x(g, tabs_, d_bsk2_, d_idx_, d_tvb_, d_ext_a_, d_ext_b_, s));
        else if (k == 3)
            FHE_HIP_CHECK(launch_blind_rotate_ginx2x(g, tabs_, d_bsk2_, d_idx_, d_tvb_, d_ext_a_, d_ext_b_,
                                                     2 * (size_t)g.count <= x_batch_ ? 1 : 2, s));
        else
            FHE_HIP_CHECK(launch_blind_rotate_ginx(g, tabs_, d_bsk_, d_idx_, d_tvb_, d_ext_a_, d_ext_b_, s));
    } else if (lmk_choice(g) == 4) {
        // four waves per gate up to one gate per CU (K1m-4, as K1q for GINX)
        FHE_HIP_CHECK(launch_blind_rotate_lmk4x(g, tabs_, d_bsk2_, p_.n, d_ops_, d_nops_, maxops_, d_tvb_, d_ext_a_,
                                                d_ext_b_, s));
    } else if (lmk_choice(g) == 2) {
        // two waves per gate up to x_batch_ gates (as K1x for GINX): one gate per 128-thread workgroup up to one
        // per CU, two per 256-thread workgroup above (bootstrap.hip k_blind_rotate_lmk3's GW)
        FHE_HIP_CHECK(launch_blind_rotate_lmkx(g, tabs_, d_bsk2_, p_.n, d_ops_, d_nops_, maxops_, d_tvb_, d_ext_a_,
                                               d_ext_b_, 2 * (size_t)g.count <= x_batch_ ? 1 : 2, s));
    } else {
        FHE_HIP_CHECK(launch_blind_rotate_lmk(g, tabs_, d_bsk_, d_autok_, d_ops_, d_nops_, maxops_, d_tvb_, d_ext_a_,
                                              d_ext_b_, p_.method == M_AP, s));
    }
}

void Engine::bootstrap_device(int gate, size_t count, const uint64_t* a1, const uint64_t* b1, const uint64_t* a2,
                              const uint64_t* b2, bool modswitch, hipStream_t s) {
    if (!d_bsk_) throw std::logic_error("bootstrapping key not loaded");
    GateArgs g = gate_args(gate, count);
    g.msb_out = modswitch ? 1 : 0;
    if (count == 0) return;
    ensure_work(count);
    FHE_HIP_CHECK(hipSetDevice(device_));
    GateInputs in{{a1, a2, nullptr, nullptr}, {b1, b2, nullptr, nullptr}, 2, 0, 0};
    prep_device(g, in, 0, s);
    rotate_device(g, s);
}

void Engine::blind_rotate_acc_device(size_t count, const uint64_t* a, uint32_t ctmod, uint64_t* acc, hipStream_t s) {
    if (!d_bsk_) throw std::logic_error("bootstrapping key not loaded");
    if (ctmod < 2 || (ctmod & (ctmod - 1)) || ctmod > 2 * p_.N)
        throw std::invalid_argument("BlindRotate: ciphertext modulus must be a power of two <= 2N");
    if (p_.method == M_AP && ctmod != p_.q)  // EvalAcc DM reads a_i modulo q (rgsw-acc-dm.cpp:64-69)
        throw std::invalid_argument("BlindRotate (AP): ciphertext modulus must be q");
    if (p_.method == M_LMKCDEY && ctmod != 2 * p_.N)  // a_i are taken mod M = 2N (rgsw-acc-lmkcdey.cpp:84-86)
        throw std::invalid_argument("BlindRotate (LMKCDEY): ciphertext modulus must be 2N");
    if (count == 0) return;
    if (!a || !acc) throw std::invalid_argument("null argument");
    if (count > 0x7fffffffull) throw std::invalid_argument("batch too large");
    ensure_work(count);
    FHE_HIP_CHECK(hipSetDevice(device_));
    GateArgs g{};
    g.count = (uint32_t)count;
    g.n = p_.n;
    g.N = p_.N;
    g.q = p_.q;
    g.qKS = p_.qKS;
    g.ctmod = ctmod;
    g.factor = 2 * p_.N / ctmod;
    g.gbits = p_.gBits;
    g.acc_io = acc;
    // the prep kernels read one input ciphertext; its b only feeds the (unused) test vector
    GateInputs in{{a, nullptr, nullptr, nullptr}, {a, nullptr, nullptr, nullptr}, 1, 0, 0};
    prep_device(g, in, 0, s);
    rotate_device(g, s);
    rot_count_ = 0;  // no ctExt left in the workspace
}

void Engine::blind_rotate_init_device(size_t count, const uint64_t* a, const uint64_t* b, uint64_t* acc, hipStream_t s) {
    if (!d_bsk_) throw std::logic_error("bootstrapping key not loaded");
    if (count == 0) return;
    if (!a || !b || !acc) throw std::invalid_argument("null argument");
    GateArgs g = gate_args(G_AND, count);  // BootstrapGateCore's AND window (Bootstrap, :205)
    ensure_work(count);
    FHE_HIP_CHECK(hipSetDevice(device_));
    g.acc_io = acc;
    g.acc_tv = 1;
    // ct + q/4 (EvalAddConstEq, binfhe-base-scheme.cpp:201): the b offset of the prep
    GateInputs in{{a, nullptr, nullptr, nullptr}, {b, nullptr, nullptr, nullptr}, 1, 0, p_.q >> 2};
    prep_device(g, in, 0, s);
    rotate_device(g, s);
    rot_count_ = 0;
}

void Engine::external_product_device(size_t count, const uint64_t* rgsw, const uint64_t* rlwe, uint64_t* result,
                                     hipStream_t s) {
    if (!wide_ && p_.digitsG2 != 4) throw std::invalid_argument("device path expects digitsG = 3");
    if (count == 0) return;
    if (!rgsw || !rlwe || !result) throw std::invalid_argument("null argument");
    FHE_HIP_CHECK(hipSetDevice(device_));
    constexpr size_t kChunk = 0x8000;   // op codes hold key indices < 0x8000
    const size_t keyw = (size_t)p_.digitsG2 * 2 * p_.N;
    const size_t wpk = wide_ && !narrow_ ? 2 : 1;   // u32 words per packed key word (u64 Montgomery on the 64-bit path)
    const size_t cap = std::min(count, kChunk);
    if (cap > epcap_) {
        sync_streams();
        for (void* ptr : {(void*)d_epk_, (void*)d_epops_, (void*)d_epn_})
            if (ptr) FHE_HIP_CHECK(hipFree(ptr));
        d_epk_ = nullptr; d_epops_ = nullptr; d_epn_ = nullptr; epcap_ = 0;
        FHE_HIP_CHECK(hipMalloc(&d_epk_, cap * keyw * wpk * sizeof(uint32_t)));
        FHE_HIP_CHECK(hipMalloc(&d_epops_, cap * sizeof(uint16_t)));
        FHE_HIP_CHECK(hipMalloc(&d_epn_, cap * sizeof(uint32_t)));
        epcap_ = cap;
    }
    const uint32_t ninv_mont = wide_ ? 0u : to_mont(invmod(p_.N, p_.Q), p_.Q);
    for (size_t off = 0; off < count; off += kChunk) {
        const size_t c = std::min(kChunk, count - off);
        if (result + off * 2 * p_.N != rlwe + off * 2 * p_.N)
            FHE_HIP_CHECK(hipMemcpyAsync(result + off * 2 * p_.N, rlwe + off * 2 * p_.N, c * 2 * p_.N * 8,
                                         hipMemcpyDeviceToDevice, s));
        FHE_HIP_CHECK(launch_single_ops(d_epops_, d_epn_, (uint32_t)c, 1, s));
        if (wide_) {
            // the wide DM op loop (k_blind_rotate_wide_ops): one EXT op per item with its own key
            FHE_HIP_CHECK(launch_pack_rgsw_wide(rgsw + off * keyw, c * keyw, wtabs_, d_epk_, s));
            WideArgs w{};
            w.count = (uint32_t)c;
            w.n = p_.n;
            w.N = p_.N;
            w.ctmod = p_.q;
            w.factor = 1;
            w.digitsG = p_.digitsG;
            w.gbits = p_.gBits;
            w.qKS = p_.qKS;
            w.acc_io = result + off * 2 * p_.N;
            FHE_HIP_CHECK(launch_blind_rotate_wide_ops(w, wtabs_, d_epk_, d_epk_, d_epops_, d_epn_, 1, nullptr, nullptr,
                                                       nullptr, true, s));
            continue;
        }
        FHE_HIP_CHECK(launch_pack_rgsw(rgsw + off * keyw, c, p_.N, (uint32_t)p_.Q, ninv_mont, d_epk_, s));
        GateArgs g{};
        g.count = (uint32_t)c;
        g.n = p_.n;
        g.N = p_.N;
        g.q = p_.q;
        g.qKS = p_.qKS;
        g.ctmod = p_.q;
        g.factor = 1;
        g.gbits = p_.gBits;
        g.acc_io = result + off * 2 * p_.N;
        // the DM op loop: each item's list is the one external product with its own key
        FHE_HIP_CHECK(launch_blind_rotate_lmk(g, tabs_, d_epk_, nullptr, d_epops_, d_epn_, 1, nullptr, nullptr,
                                              nullptr, true, s));
    }
}

size_t Engine::max_batch() const {
    size_t fr = 0, tot = 0;
    if (hipSetDevice(device_) != hipSuccess || hipMemGetInfo(&fr, &tot) != hipSuccess) return 0;
    // workspace per gate: monomial indices / op list, ctExt, test-vector b, staged I/O
    const size_t per = (size_t)p_.n * 2 + (size_t)maxops_ * 2 + ((size_t)p_.N + 1) * (wide_ ? 8 : 4) + 4 +
                       (4 * ((size_t)p_.n + 1) + p_.N + 1) * 8;
    return std::min<size_t>(0x7fffffffull, fr / 2 / per);
}

void Engine::eval_gate_multi_device(int gate, size_t count, uint32_t k, const uint64_t* const* a,
                                    const uint64_t* const* b, uint32_t p, uint64_t* a_out, uint64_t* b_out,
                                    hipStream_t s) {
    if (!ready()) throw std::logic_error("keys not loaded (load_bsk / load_ksk)");
    if (k < 2 || k > 4) throw std::invalid_argument("EvalBinGate(ctvector): 2 to 4 ciphertexts");
    GateArgs g = gate_args(gate, count, p, true);
    if (count == 0) return;
    ensure_work(count);
    FHE_HIP_CHECK(hipSetDevice(device_));
    GateInputs in{};
    for (uint32_t j = 0; j < k; ++j) {
        if (!a[j] || !b[j]) throw std::invalid_argument("null ciphertext array");
        in.a[j] = a[j];
        in.b[j] = b[j];
    }
    in.k = k;
    g.msb_out = a_out ? 1 : 0;
    prep_device(g, in, 0, s);
    rotate_device(g, s);
    if (a_out) keyswitch_workspace_device(count, a_out, b_out, s);
}

void Engine::refresh_device(size_t count, const uint64_t* a, const uint64_t* b, uint64_t* a_out, uint64_t* b_out,
                            hipStream_t s) {
    if (!ready()) throw std::logic_error("keys not loaded (load_bsk / load_ksk)");
    GateArgs g = gate_args(G_AND, count);  // BootstrapGateCore's AND window; b = Q/(2p) + 1, p = 4 (:211)
    if (count == 0) return;
    if (!a || !b || !a_out || !b_out) throw std::invalid_argument("null argument");
    ensure_work(count);
    FHE_HIP_CHECK(hipSetDevice(device_));
    // ct + q/4 (EvalAddConstEq, :201) as the prep's b offset
    GateInputs in{{a, nullptr, nullptr, nullptr}, {b, nullptr, nullptr, nullptr}, 1, 0, p_.q >> 2};
    prep_device(g, in, 0, s);
    rotate_device(g, s);
    keyswitch_workspace_device(count, a_out, b_out, s);
}

void Engine::eval_cmux_device(size_t count, const uint64_t* a0, const uint64_t* b0, const uint64_t* a1,
                              const uint64_t* b1, const uint64_t* a2, const uint64_t* b2, uint64_t* a_out,
                              uint64_t* b_out, hipStream_t s) {
    if (!ready()) throw std::logic_error("keys not loaded (load_bsk / load_ksk)");
    if (count == 0) return;
    if (2 * count > 0x7fffffffull) throw std::invalid_argument("batch too large");
    ensure_work(2 * count);
    FHE_HIP_CHECK(hipSetDevice(device_));
    cmux_levels(count, a0, b0, a1, b1, a2, b2, nullptr, nullptr, a_out, b_out, s);
}

uint64_t* Engine::grow(uint64_t*& ptr, size_t& cap, size_t bytes) {
    if (bytes <= cap) return ptr;
    sync_streams();
    if (ptr) FHE_HIP_CHECK(hipFree(ptr));
    ptr = nullptr;
    cap = 0;
    FHE_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&ptr), bytes));
    cap = bytes;
    return ptr;
}

void Engine::cmux_levels(size_t count, const uint64_t* a0, const uint64_t* b0, const uint64_t* a1, const uint64_t* b1,
                         const uint64_t* a2, const uint64_t* b2, const uint64_t* a2n, const uint64_t* b2n,
                         uint64_t* a_out, uint64_t* b_out, hipStream_t s) {
    const size_t n = p_.n;
    uint64_t* l1 = grow(d_l1_, ccap_, 2 * count * (n + 1) * 8);
    uint64_t* l1a = l1;                 // [2 count][n]: NAND(ct0, NOT ct2) | NAND(ct1, ct2)
    uint64_t* l1b = l1 + 2 * count * n; // [2 count]
    const GateArgs gh = gate_args(G_NAND, count);
    // ct0 + NOT ct2: EvalNOT (:223-236) folded into the input combination (ct0 - ct2, b offset q/4; exact
    // mod the power-of-two q), or the explicit NOT column when ct2 was switched from Q
    const GateInputs lo = a2n ? GateInputs{{a0, a2n, nullptr, nullptr}, {b0, b2n, nullptr, nullptr}, 2, 0u, 0u}
                              : GateInputs{{a0, a2, nullptr, nullptr}, {b0, b2, nullptr, nullptr}, 2, 2u, p_.q >> 2};
    const GateInputs hi{{a1, a2, nullptr, nullptr}, {b1, b2, nullptr, nullptr}, 2, 0u, 0u};
    prep_device(gh, lo, 0, s);
    prep_device(gh, hi, count, s);
    rotate_device(gate_args(G_NAND, 2 * count), s);
    keyswitch_workspace_device(2 * count, l1a, l1b, s);
    const GateInputs top{{l1a, l1a + count * n, nullptr, nullptr}, {l1b, l1b + count, nullptr, nullptr}, 2, 0u, 0u};
    prep_device(gh, top, 0, s);
    rotate_device(gh, s);
    keyswitch_workspace_device(count, a_out, b_out, s);
}

void Engine::ext_to_device(size_t count, uint64_t* a_out, uint64_t* b_out, hipStream_t s) {
    if (count > rot_count_) throw std::logic_error("ctExt of more ciphertexts than the last blind rotation produced");
    if (wide_) {
        FHE_HIP_CHECK(hipMemcpyAsync(a_out, d_wext_a_, count * p_.N * 8, hipMemcpyDeviceToDevice, s));
        FHE_HIP_CHECK(hipMemcpyAsync(b_out, d_wext_b_, count * 8, hipMemcpyDeviceToDevice, s));
        return;
    }
    FHE_HIP_CHECK(launch_widen_u64(d_ext_a_, d_ext_b_, a_out, b_out, p_.N, count, s));
}

void Engine::switch_column_device(size_t count, const uint64_t* a, const uint64_t* b, uint32_t stride,
                                  const uint8_t* large, bool negate, bool set_b, uint64_t b_large, uint64_t* a_out,
                                  uint64_t* b_out, hipStream_t s) {
    // ModSwitch(Q -> qKS) into the key switch's input, KeySwitch + ModSwitch(qKS -> q) (K2's epilogue) into
    // the output column, then the rows that were mod q already copied in (lwe-pke.cpp:170-178)
    FHE_HIP_CHECK(launch_switch_in(a, b, stride, large, p_.Q, p_.qKS, p_.N, count, negate,
                                   wide_ ? (void*)d_wext_a_ : (void*)d_ext_a_, wide_ ? (void*)d_wext_b_ : (void*)d_ext_b_,
                                   wide_, s));
    keyswitch_ext(count, p_.q, a_out, b_out, s);
    FHE_HIP_CHECK(launch_switch_out(a, b, stride, large, p_.n, p_.q, count, negate, set_b, b_large, a_out, b_out, s));
    rot_count_ = 0;  // the workspace no longer holds a blind rotation's ctExt
}

void Engine::switch_to_qn_device(size_t count, const uint64_t* a, const uint64_t* b, uint64_t* a_out, uint64_t* b_out,
                                 hipStream_t s) {
    if (!d_ksk_ && !d_wksk_) throw std::logic_error("key-switching key not loaded");
    if (count == 0) return;
    if (!a || !b || !a_out || !b_out) throw std::invalid_argument("null argument");
    if (count > 0x7fffffffull) throw std::invalid_argument("batch too large");
    ensure_work(count);
    FHE_HIP_CHECK(hipSetDevice(device_));
    switch_column_device(count, a, b, p_.N, nullptr, false, false, 0, a_out, b_out, s);
}

void Engine::eval_mixed_device(int op, uint32_t k, uint32_t ptmod, size_t count, const uint64_t* const* a,
                               const uint64_t* const* b, const uint8_t* const* large, uint64_t* a_out, uint64_t* b_out,
                               bool extended, hipStream_t s) {
    if (!ready()) throw std::logic_error("keys not loaded (load_bsk / load_ksk)");
    const bool multi = op == G_MAJORITY || op == G_AND3 || op == G_OR3 || op == G_AND4 || op == G_OR4;
    if (op == kOpBootstrap) {
        if (k != 1) throw std::invalid_argument("Bootstrap takes one ciphertext");
        if (ptmod < 1) throw std::invalid_argument("plaintext modulus out of range");
    } else if (op == G_CMUX) {
        if (k != 3) throw std::invalid_argument("CMUX gate implemented for ciphertext vectors of size 3");
    } else if (multi) {
        if (k < 2 || k > 4) throw std::invalid_argument("EvalBinGate(ctvector): 2 to 4 ciphertexts");
        gate_args(op, count, ptmod, true);
    } else {
        if (k != 2) throw std::invalid_argument("EvalBinGate: two ciphertexts");
        gate_args(op, count);
    }
    if (count == 0) return;
    if (!a || !b || !a_out || !b_out) throw std::invalid_argument("null argument");
    for (uint32_t j = 0; j < k; ++j)
        if (!a[j] || !b[j]) throw std::invalid_argument("null ciphertext array");
    if ((op == G_CMUX ? 2 : 1) * count > 0x7fffffffull) throw std::invalid_argument("batch too large");
    ensure_work(op == G_CMUX ? 2 * count : count);
    FHE_HIP_CHECK(hipSetDevice(device_));
    const size_t n = p_.n, col = count * (n + 1);
    bool any = false;
    for (uint32_t j = 0; j < k; ++j) any |= large && large[j];
    const bool cmux_not = op == G_CMUX && large && large[2];
    uint64_t* mix = any ? grow(d_mix_, mixcap_, (k + (cmux_not ? 1 : 0)) * col * 8) : nullptr;
    // Bootstrap (:199-201): ct + (ct->GetModulus() >> 2) by ModAddFast at the switched ciphertext's modulus q.
    // For an input mod Q that sum is b_sw + Q/4 - q >= 1.5 q, and BootstrapGateCore's window walk
    // (:562-567, ModSubFast by 1 from there) never wraps and never enters [lb, ub < q): every test-vector
    // slot is uv.  The device prep adds q/4 mod q to b; the b its window test then sees, (lb - 1) mod q,
    // walks exactly the complement of [lb, ub), so the same all-uv test vector results.
    const GateArgs gand = gate_args(G_AND, count);
    if (op == kOpBootstrap && any && (p_.Q >> 2) < 2 * (uint64_t)p_.q + (p_.q >> 1))
        throw std::invalid_argument("Bootstrap of a ciphertext mod Q needs Q/4 >= 2.5 q");
    const uint64_t q = p_.q, b_large = ((uint64_t)gand.lb + 2 * q - 1 - (q >> 2)) % q;
    const uint64_t* ia[4] = {};
    const uint64_t* ib[4] = {};
    for (uint32_t j = 0; j < k; ++j) {
        if (large && large[j]) {
            uint64_t* ca = mix + j * col;
            uint64_t* cb = ca + count * n;
            switch_column_device(count, a[j], b[j], p_.N, large[j], false, op == kOpBootstrap, b_large, ca, cb, s);
            ia[j] = ca;
            ib[j] = cb;
        } else {
            ia[j] = a[j];
            ib[j] = b[j];
        }
    }
    if (op == G_CMUX) {
        const uint64_t *a2n = nullptr, *b2n = nullptr;
        if (cmux_not) {  // EvalNOT at ct2's own modulus (:180, :223-236), then the NAND's SwitchCTtoqn
            uint64_t* ca = mix + k * col;
            uint64_t* cb = ca + count * n;
            switch_column_device(count, a[2], b[2], p_.N, large[2], true, false, 0, ca, cb, s);
            a2n = ca;
            b2n = cb;
        }
        cmux_levels(count, ia[0], ib[0], ia[1], ib[1], ia[2], ib[2], a2n, b2n, a_out, b_out, s);
        return;
    }
    if (op == kOpBootstrap) {
        // the window and its values are p = 4's (the switched / copied ciphertext's default plaintext
        // modulus, lwe-ciphertext.h:161); the extraction's b uses the input's own (:210-211)
        GateArgs g = gand;
        g.b_const = (uint32_t)(p_.Q / (2 * (uint64_t)ptmod) + 1);
        g.b64 = p_.Q / (2 * (uint64_t)ptmod) + 1;
        g.msb_out = extended ? 0 : 1;
        const GateInputs in{{ia[0], nullptr, nullptr, nullptr}, {ib[0], nullptr, nullptr, nullptr}, 1, 0, p_.q >> 2};
        prep_device(g, in, 0, s);
        rotate_device(g, s);
    } else if (multi) {
        GateArgs g = gate_args(op, count, ptmod, true);
        g.msb_out = extended ? 0 : 1;
        GateInputs in{};
        for (uint32_t j = 0; j < k; ++j) {
            in.a[j] = ia[j];
            in.b[j] = ib[j];
        }
        in.k = k;
        prep_device(g, in, 0, s);
        rotate_device(g, s);
    } else {
        bootstrap_device(op, count, ia[0], ib[0], ia[1], ib[1], !extended, s);
    }
    if (extended)
        ext_to_device(count, a_out, b_out, s);
    else
        keyswitch_workspace_device(count, a_out, b_out, s);
}

void Engine::eval_mixed_host(int op, uint32_t k, uint32_t ptmod, size_t count, const uint64_t* const* a,
                             const uint64_t* const* b, const uint8_t* const* large, uint64_t* a_out, uint64_t* b_out,
                             bool extended) {
    if (k < 1 || k > 4) throw std::invalid_argument("1 to 4 ciphertext columns");
    if (count == 0) return;
    const size_t n = p_.n, N = p_.N;
    // staged columns (rows of N words where flagged), flags, and the output
    size_t words = 0;
    for (uint32_t j = 0; j < k; ++j) words += count * ((large && large[j] ? N : n) + 1) + (count + 7) / 8;
    const size_t outw = count * ((extended && op != G_CMUX ? N : n) + 1);
    uint64_t* d = grow(d_mixio_, mixiocap_, (words + outw) * 8);
    FHE_HIP_CHECK(hipSetDevice(device_));
    const uint64_t* da[4] = {};
    const uint64_t* db[4] = {};
    const uint8_t* dl[4] = {};
    uint64_t* cur = d;
    for (uint32_t j = 0; j < k; ++j) {
        if (!a[j] || !b[j]) throw std::invalid_argument("null ciphertext array");
        const bool lg = large && large[j];
        const size_t len = lg ? N : n;
        FHE_HIP_CHECK(hipMemcpyAsync(cur, a[j], count * len * 8, hipMemcpyHostToDevice, stream_));
        da[j] = cur;
        cur += count * len;
        FHE_HIP_CHECK(hipMemcpyAsync(cur, b[j], count * 8, hipMemcpyHostToDevice, stream_));
        db[j] = cur;
        cur += count;
        if (lg) {
            FHE_HIP_CHECK(hipMemcpyAsync(cur, large[j], count, hipMemcpyHostToDevice, stream_));
            dl[j] = reinterpret_cast<const uint8_t*>(cur);
        }
        cur += (count + 7) / 8;
    }
    uint64_t* dao = cur;
    uint64_t* dbo = dao + (outw - count);
    eval_mixed_device(op, k, ptmod, count, da, db, dl, dao, dbo, extended, stream_);
    FHE_HIP_CHECK(hipMemcpyAsync(a_out, dao, (outw - count) * 8, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(b_out, dbo, count * 8, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipStreamSynchronize(stream_));
}

void Engine::switch_to_qn_host(size_t count, const uint64_t* a, const uint64_t* b, uint64_t* a_out, uint64_t* b_out) {
    if (count == 0) return;
    const size_t n = p_.n, N = p_.N;
    uint64_t* d = grow(d_mixio_, mixiocap_, count * (N + 1 + n + 1) * 8);
    FHE_HIP_CHECK(hipSetDevice(device_));
    uint64_t* dbi = d + count * N;
    uint64_t* dao = dbi + count;
    uint64_t* dbo = dao + count * n;
    FHE_HIP_CHECK(hipMemcpyAsync(d, a, count * N * 8, hipMemcpyHostToDevice, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(dbi, b, count * 8, hipMemcpyHostToDevice, stream_));
    switch_to_qn_device(count, d, dbi, dao, dbo, stream_);
    FHE_HIP_CHECK(hipMemcpyAsync(a_out, dao, count * n * 8, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(b_out, dbo, count * 8, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipStreamSynchronize(stream_));
}

void Engine::keyswitch_workspace_device(size_t count, uint64_t* a_out, uint64_t* b_out, hipStream_t s) {
    if (!d_ksk_ && !d_wksk_) throw std::logic_error("key-switching key not loaded");
    if (count == 0) return;
    if (count > rot_count_)
        throw std::invalid_argument("key switch of more ciphertexts than the last blind rotation produced");
    FHE_HIP_CHECK(hipSetDevice(device_));
    keyswitch_ext(count, p_.q, a_out, b_out, s);
}

void Engine::keyswitch_ext(size_t count, uint64_t q_out, uint64_t* a_out, uint64_t* b_out, hipStream_t s) {
    if (wide_ && ks32_ && d_ksk_ && d_ext_a_ && count <= cap_) {
        // the u64 ctExt mod qKS narrowed to u32, then the 32-bit (u16-row, gate-tiled) key switch instead
        // of u64 row gathers
        FHE_HIP_CHECK(launch_narrow_u32(d_wext_a_, d_wext_b_, d_ext_a_, d_ext_b_, p_.N, count, s));
        GateArgs g = gate_args(G_AND, count);
        FHE_HIP_CHECK(launch_keyswitch(g, p_.baseKS, p_.digitsKS, d_ksk_, d_ext_a_, d_ext_b_, q_out, a_out, b_out, s,
                                       ks_part(count), kKsPartWords));
        return;
    }
    if (wide_ && ks32w_ && d_ksk32_ && d_ext_a_ && count <= cap_) {
        FHE_HIP_CHECK(launch_narrow_u32(d_wext_a_, d_wext_b_, d_ext_a_, d_ext_b_, p_.N, count, s));
        GateArgs g = gate_args(G_AND, count);
        FHE_HIP_CHECK(launch_keyswitch_w32(g, p_.baseKS, p_.digitsKS, d_ksk32_, d_ext_a_, d_ext_b_, q_out, a_out, b_out,
                                           s, ks_part(count), kKsPartWords));
        return;
    }
    if (wide_) {
        const size_t rows = p_.ksk_rows();
        const uint64_t* ksk = d_wksk_ + cur_ksk_off_;  // timeOptimization: the switching key of the current base
        FHE_HIP_CHECK(launch_keyswitch_wide(count, p_.n, p_.N, p_.baseKS, p_.digitsKS, p_.qKS, ksk, ksk + rows * p_.n,
                                            d_wext_a_, d_wext_b_, q_out, a_out, b_out, s));
        return;
    }
    GateArgs g = gate_args(G_AND, count);
    FHE_HIP_CHECK(launch_keyswitch(g, p_.baseKS, p_.digitsKS, d_ksk_, d_ext_a_, d_ext_b_, q_out, a_out, b_out, s,
                                   ks_part(count), kKsPartWords));
}

// scratch of the row-split key switch (launch_keyswitch, below 4096 gates): S count <= 2^16 for
// every count, so 2^16 partial rows of ksk_width / 2 words
uint32_t* Engine::ks_part(size_t count) {
    if (count >= 4096) return nullptr;
    if (!d_kspart_) {
        sync_streams();
        FHE_HIP_CHECK(hipMalloc(&d_kspart_, kKsPartWords * sizeof(uint32_t)));
    }
    return d_kspart_;
}

void Engine::copy_ext_host(size_t count, uint64_t* ext_a, uint64_t* ext_b) {
    const size_t N = p_.N;
    if (wide_) {
        FHE_HIP_CHECK(hipMemcpyAsync(ext_a, d_wext_a_, count * N * 8, hipMemcpyDeviceToHost, stream_));
        FHE_HIP_CHECK(hipMemcpyAsync(ext_b, d_wext_b_, count * 8, hipMemcpyDeviceToHost, stream_));
        FHE_HIP_CHECK(hipStreamSynchronize(stream_));
        return;
    }
    std::vector<uint32_t> ha(count * N), hb(count);
    FHE_HIP_CHECK(hipMemcpyAsync(ha.data(), d_ext_a_, count * N * 4, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(hb.data(), d_ext_b_, count * 4, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipStreamSynchronize(stream_));
    for (size_t i = 0; i < count * N; ++i) ext_a[i] = ha[i];
    for (size_t i = 0; i < count; ++i) ext_b[i] = hb[i];
}

void Engine::eval_gate_device(int gate, size_t count, const uint64_t* a1, const uint64_t* b1, const uint64_t* a2,
                              const uint64_t* b2, uint64_t* a_out, uint64_t* b_out, hipStream_t s) {
    if (!ready()) throw std::logic_error("keys not loaded (load_bsk / load_ksk)");
    if (count == 0) return;
    bootstrap_device(gate, count, a1, b1, a2, b2, true, s);
    keyswitch_workspace_device(count, a_out, b_out, s);
}

void Engine::eval_gate_host(int gate, size_t count, const uint64_t* a1, const uint64_t* b1, const uint64_t* a2,
                            const uint64_t* b2, uint64_t* a_out, uint64_t* b_out) {
    if (count == 0) return;
    ensure_host_stage(count);
    const size_t n = p_.n;
    uint64_t* da1 = d_io_;
    uint64_t* db1 = da1 + count * n;
    uint64_t* da2 = db1 + count;
    uint64_t* db2 = da2 + count * n;
    uint64_t* dao = db2 + count;
    uint64_t* dbo = dao + count * p_.N;
    FHE_HIP_CHECK(hipSetDevice(device_));
    FHE_HIP_CHECK(hipMemcpyAsync(da1, a1, count * n * 8, hipMemcpyHostToDevice, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(db1, b1, count * 8, hipMemcpyHostToDevice, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(da2, a2, count * n * 8, hipMemcpyHostToDevice, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(db2, b2, count * 8, hipMemcpyHostToDevice, stream_));
    eval_gate_device(gate, count, da1, db1, da2, db2, dao, dbo, stream_);
    FHE_HIP_CHECK(hipMemcpyAsync(a_out, dao, count * n * 8, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(b_out, dbo, count * 8, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipStreamSynchronize(stream_));
}

void Engine::bootstrap_extended_host(int gate, size_t count, const uint64_t* a1, const uint64_t* b1,
                                     const uint64_t* a2, const uint64_t* b2, uint64_t* ext_a, uint64_t* ext_b) {
    if (count == 0) return;
    ensure_host_stage(count);
    const size_t n = p_.n, N = p_.N;
    uint64_t* da1 = d_io_;
    uint64_t* db1 = da1 + count * n;
    uint64_t* da2 = db1 + count;
    uint64_t* db2 = da2 + count * n;
    FHE_HIP_CHECK(hipSetDevice(device_));
    FHE_HIP_CHECK(hipMemcpyAsync(da1, a1, count * n * 8, hipMemcpyHostToDevice, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(db1, b1, count * 8, hipMemcpyHostToDevice, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(da2, a2, count * n * 8, hipMemcpyHostToDevice, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(db2, b2, count * 8, hipMemcpyHostToDevice, stream_));
    bootstrap_device(gate, count, da1, db1, da2, db2, false, stream_);
    (void)N;
    copy_ext_host(count, ext_a, ext_b);
}

void Engine::keyswitch_host(size_t count, const uint64_t* a, const uint64_t* b, uint64_t* a_out, uint64_t* b_out) {
    if (!d_ksk_ && !d_wksk_) throw std::logic_error("key-switching key not loaded");
    if (count == 0) return;
    ensure_work(count);
    ensure_host_stage(count);
    const size_t N = p_.N;
    if (wide_) {
        for (size_t i = 0; i < count * N; ++i)
            if (a[i] >= p_.qKS) throw std::invalid_argument("keyswitch input not reduced mod qKS");
        for (size_t i = 0; i < count; ++i)
            if (b[i] >= p_.qKS) throw std::invalid_argument("keyswitch input not reduced mod qKS");
        uint64_t* dao = d_io_;
        uint64_t* dbo = dao + count * p_.n;
        FHE_HIP_CHECK(hipSetDevice(device_));
        FHE_HIP_CHECK(hipMemcpyAsync(d_wext_a_, a, count * N * 8, hipMemcpyHostToDevice, stream_));
        FHE_HIP_CHECK(hipMemcpyAsync(d_wext_b_, b, count * 8, hipMemcpyHostToDevice, stream_));
        keyswitch_ext(count, 0, dao, dbo, stream_);
        FHE_HIP_CHECK(hipMemcpyAsync(a_out, dao, count * p_.n * 8, hipMemcpyDeviceToHost, stream_));
        FHE_HIP_CHECK(hipMemcpyAsync(b_out, dbo, count * 8, hipMemcpyDeviceToHost, stream_));
        FHE_HIP_CHECK(hipStreamSynchronize(stream_));
        return;
    }
    std::vector<uint32_t> ha(count * N), hb(count);
    for (size_t i = 0; i < count * N; ++i) {
        if (a[i] >= p_.qKS) throw std::invalid_argument("keyswitch input not reduced mod qKS");
        ha[i] = (uint32_t)a[i];
    }
    for (size_t i = 0; i < count; ++i) {
        if (b[i] >= p_.qKS) throw std::invalid_argument("keyswitch input not reduced mod qKS");
        hb[i] = (uint32_t)b[i];
    }
    uint64_t* dao = d_io_;
    uint64_t* dbo = dao + count * p_.n;
    FHE_HIP_CHECK(hipSetDevice(device_));
    FHE_HIP_CHECK(hipMemcpyAsync(d_ext_a_, ha.data(), count * N * 4, hipMemcpyHostToDevice, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(d_ext_b_, hb.data(), count * 4, hipMemcpyHostToDevice, stream_));
    GateArgs g = gate_args(G_AND, count);
    FHE_HIP_CHECK(launch_keyswitch(g, p_.baseKS, p_.digitsKS, d_ksk_, d_ext_a_, d_ext_b_, 0, dao, dbo, stream_,
                                   ks_part(count), kKsPartWords));
    FHE_HIP_CHECK(hipMemcpyAsync(a_out, dao, count * p_.n * 8, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(b_out, dbo, count * 8, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipStreamSynchronize(stream_));
}

void Engine::stage_inputs(size_t count, uint32_t k, const uint64_t* const* a, const uint64_t* const* b,
                          const uint64_t** da, const uint64_t** db) {
    const size_t n = p_.n;
    uint64_t* cur = d_io_;
    for (uint32_t j = 0; j < k; ++j) {
        if (!a[j] || !b[j]) throw std::invalid_argument("null ciphertext array");
        FHE_HIP_CHECK(hipMemcpyAsync(cur, a[j], count * n * 8, hipMemcpyHostToDevice, stream_));
        da[j] = cur;
        cur += count * n;
        FHE_HIP_CHECK(hipMemcpyAsync(cur, b[j], count * 8, hipMemcpyHostToDevice, stream_));
        db[j] = cur;
        cur += count;
    }
}

void Engine::eval_gate_multi_host(int gate, size_t count, uint32_t k, const uint64_t* const* a,
                                  const uint64_t* const* b, uint32_t p, uint64_t* a_out, uint64_t* b_out,
                                  bool extended) {
    if (k < 2 || k > 4) throw std::invalid_argument("EvalBinGate(ctvector): 2 to 4 ciphertexts");
    gate_args(gate, count, p, true);  // validate before any transfer
    if (count == 0) return;
    ensure_host_stage(count);
    FHE_HIP_CHECK(hipSetDevice(device_));
    const uint64_t* da[4] = {};
    const uint64_t* db[4] = {};
    stage_inputs(count, k, a, b, da, db);
    const size_t n = p_.n, N = p_.N;
    uint64_t* dao = d_io_ + count * 4 * (n + 1);
    uint64_t* dbo = dao + count * n;
    if (!extended) {
        eval_gate_multi_device(gate, count, k, da, db, p, dao, dbo, stream_);
        FHE_HIP_CHECK(hipMemcpyAsync(a_out, dao, count * n * 8, hipMemcpyDeviceToHost, stream_));
        FHE_HIP_CHECK(hipMemcpyAsync(b_out, dbo, count * 8, hipMemcpyDeviceToHost, stream_));
        FHE_HIP_CHECK(hipStreamSynchronize(stream_));
        return;
    }
    eval_gate_multi_device(gate, count, k, da, db, p, nullptr, nullptr, stream_);
    (void)N;
    copy_ext_host(count, a_out, b_out);
}

void Engine::refresh_host(size_t count, const uint64_t* a, const uint64_t* b, uint64_t* a_out, uint64_t* b_out) {
    if (count == 0) return;
    ensure_host_stage(count);
    FHE_HIP_CHECK(hipSetDevice(device_));
    const uint64_t* ha[1] = {a};
    const uint64_t* hb[1] = {b};
    const uint64_t* da[4] = {};
    const uint64_t* db[4] = {};
    stage_inputs(count, 1, ha, hb, da, db);
    const size_t n = p_.n;
    uint64_t* dao = d_io_ + count * 4 * (n + 1);
    uint64_t* dbo = dao + count * n;
    refresh_device(count, da[0], db[0], dao, dbo, stream_);
    FHE_HIP_CHECK(hipMemcpyAsync(a_out, dao, count * n * 8, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(b_out, dbo, count * 8, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipStreamSynchronize(stream_));
}

void Engine::eval_cmux_host(size_t count, const uint64_t* a0, const uint64_t* b0, const uint64_t* a1,
                            const uint64_t* b1, const uint64_t* a2, const uint64_t* b2, uint64_t* a_out,
                            uint64_t* b_out) {
    if (count == 0) return;
    ensure_host_stage(count);
    FHE_HIP_CHECK(hipSetDevice(device_));
    const uint64_t* ha[3] = {a0, a1, a2};
    const uint64_t* hb[3] = {b0, b1, b2};
    const uint64_t* da[4] = {};
    const uint64_t* db[4] = {};
    stage_inputs(count, 3, ha, hb, da, db);
    const size_t n = p_.n;
    uint64_t* dao = d_io_ + count * 4 * (n + 1);
    uint64_t* dbo = dao + count * n;
    eval_cmux_device(count, da[0], db[0], da[1], db[1], da[2], db[2], dao, dbo, stream_);
    FHE_HIP_CHECK(hipMemcpyAsync(a_out, dao, count * n * 8, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(b_out, dbo, count * 8, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipStreamSynchronize(stream_));
}

}  // namespace fhe_amd
