// params.cpp -- see params.h.
#include "params.h"

#include <cmath>
#include <stdexcept>

#include "nt.h"

namespace fhe_amd {

size_t Params::bsk_words() const {
    if (!timeopt) return bsk_words_one();
    size_t w = 0;
    for (uint32_t bg : kSignBases) w += with_base(bg).bsk_words_one();
    return w;
}

size_t Params::bsk_offset(uint32_t bg) const {
    if (!timeopt) {
        if (bg != baseG) throw std::invalid_argument("no bootstrapping key for this baseG");
        return 0;
    }
    size_t w = 0;
    for (uint32_t b : kSignBases) {
        if (b == bg) return w;
        w += with_base(b).bsk_words_one();
    }
    throw std::invalid_argument("no bootstrapping key for this baseG");
}

size_t Params::ksk_index(uint32_t bg) const {
    if (!timeopt) return 0;
    for (size_t k = 0; k < 3; ++k)
        if (kSignBases[k] == bg) return k;
    throw std::invalid_argument("no switching key for this baseG");
}

Params Params::with_base(uint32_t bg) const {
    Params p = *this;
    p.baseG = bg;
    p.gBits = ilog2(bg);
    p.digitsG = (uint32_t)std::ceil(std::log((double)p.Q) / std::log((double)bg));  // rgsw-cryptoparameters.h:226-228
    p.digitsG2 = (p.digitsG - 1) * 2;
    p.gpow.clear();
    uint64_t v = 1;
    for (uint32_t i = 0; i < p.digitsG; ++i) {
        p.gpow.push_back(v);
        v = mulmod(v, bg, p.Q);
    }
    return p;
}

size_t Params::bsk_words_one() const {
    if (method == M_GINX) return (size_t)n * 2 * digitsG2 * 2 * N;
    // AP: [n][baseR][digitsR][digitsG2][2][N], the j = 0 slots unused (rgsw-acc-dm.cpp:39-58)
    if (method == M_AP) return (size_t)n * baseR * digitsR * digitsG2 * 2 * N;
    return (size_t)n * digitsG2 * 2 * N + (size_t)(numAutoKeys + 1) * (digitsG - 1) * 2 * N;
}

uint64_t Params::gate_const(int gate) const {
    switch (gate) {
        case G_OR: return 5ull * (q >> 3);
        case G_AND: return 7ull * (q >> 3);
        case G_NOR: return 1ull * (q >> 3);
        case G_NAND: return 3ull * (q >> 3);
        case G_XOR: return 6ull * (q >> 3);
        case G_XNOR: return 2ull * (q >> 3);
        case G_MAJORITY: return 7ull * (q >> 3);
        case G_AND3: return 11ull * (q / 12);
        case G_OR3: return 7ull * (q / 12);
        case G_AND4: return 15ull * (q >> 4);
        case G_OR4: return 9ull * (q >> 4);
        case G_XOR_FAST: return 6ull * (q >> 3);
        case G_XNOR_FAST: return 2ull * (q >> 3);
        default: throw std::invalid_argument("unsupported gate");
    }
}

namespace {
// GenerateBinFHEContext(set, arbFunc, logQ, N, method, timeOptimization = false)
// (binfhecontext.cpp:55-104): Q = LastPrime(54 (27 for logQ = 11), 2N), N the smallest ring
// dimension of the ternary / 128-bit-classic table for log Q' (stdlatticeparms.cpp:169-172:
// 1024 -> 27 bits, 2048 -> 54 bits) or the caller's larger N, q = N (arbFunc) or 2N,
// qKS = 2^35, baseKS = 32, baseG by logQ, baseR = 23, uniform ternary secret, n = 1305 (TOY: 32)
Params make_params_large(int code, int method) {
    const int set = (code >> 16) & 0xff;
    const bool arb = ((code >> 15) & 1) != 0;
    const uint32_t logN = (code >> 8) & 0x1f, logQ = code & 0xff;
    if (method != M_GINX) throw std::invalid_argument("CGGI is the only supported method");
    if (set != PS_STD128 && set != PS_TOY) throw std::invalid_argument("STD128 and TOY are the only supported sets");
    if (logQ > 29) throw std::invalid_argument("logQ > 29 is not supported");
    if (logQ < 11) throw std::invalid_argument("logQ < 11 is not supported");
    uint32_t logQp = 54, bg;
    if (logQ > 25) bg = 1u << 14;
    else if (logQ > 16) bg = 1u << 18;
    else if (logQ > 11) bg = 1u << 27;
    else { bg = 1u << 5; logQp = 27; }
    const uint32_t minN = logQp <= 27 ? 1024 : 2048;
    const uint32_t N = logN && (1u << logN) > minN ? 1u << logN : minN;
    Params p;
    p.paramset = code;
    p.method = method;
    p.n = set == PS_TOY ? 32 : 1305;
    p.N = N;
    p.q = arb ? N : 2 * N;
    p.Q = last_prime(logQp, 2 * N);
    p.qKS = 1ull << 35;
    p.baseKS = 32;
    p.digitsKS = (uint32_t)std::ceil(std::log((double)p.qKS) / std::log((double)p.baseKS));  // lwe-pke.cpp:354
    p.baseG = bg;
    p.gBits = ilog2(bg);
    p.digitsG = (uint32_t)std::ceil(std::log((double)p.Q) / std::log((double)bg));  // rgsw-cryptoparameters.h:93-94
    p.digitsG2 = (p.digitsG - 1) * 2;
    p.numAutoKeys = 10;
    p.keyDist = KD_UNIFORM_TERNARY;
    p.timeopt = (code & kTimeOpt) != 0 && logQ != 11;  // RingGSWCryptoParams(..., signEval = logQ != 11 && timeOpt)
    p.baseR = 23;
    p.digitsR = (uint32_t)std::ceil(std::log((double)p.q) / std::log((double)p.baseR));
    p.psi = root_of_unity(2 * N, p.Q);
    uint64_t v = 1;
    for (uint32_t i = 0; i < p.digitsG; ++i) {
        p.gpow.push_back(v);
        v = mulmod(v, bg, p.Q);
    }
    return p;
}
}  // namespace

namespace {
// BinFHEContext::GenerateBinFHEContext(set, method) rows (binfhecontext.cpp:113-159), indexed by
// BINFHE_PARAMSET (binfhe-constants.h:49-95).  qks = 0: modKS = PRIME (the ring modulus Q).
struct Row {
    uint32_t bits, cyc, n, q, qks, bks, bg, brk, nauto;
    int kd;
};
constexpr int G_ = KD_GAUSSIAN, T_ = KD_UNIFORM_TERNARY;
constexpr Row kRows[] = {
    {27, 1024, 64, 512, 0, 25, 512, 23, 9, T_},                  // TOY
    {28, 2048, 422, 1024, 16384, 128, 1024, 32, 10, T_},         // MEDIUM
    {27, 2048, 503, 1024, 16384, 32, 512, 32, 10, T_},           // STD128_AP
    {27, 2048, 503, 1024, 16384, 32, 512, 32, 10, T_},           // STD128
    {27, 2048, 595, 1024, 65536, 64, 128, 32, 10, T_},           // STD128_3
    {27, 2048, 595, 2048, 65536, 64, 128, 64, 10, T_},           // STD128_4
    {25, 2048, 534, 1024, 16384, 32, 128, 32, 10, T_},           // STD128Q
    {50, 4096, 600, 2048, 32768, 32, 33554432, 64, 10, T_},      // STD128Q_3
    {50, 4096, 641, 2048, 65536, 64, 33554432, 64, 10, T_},      // STD128Q_4
    {37, 4096, 790, 2048, 16384, 32, 524288, 64, 10, T_},        // STD192
    {37, 4096, 875, 4096, 65536, 64, 524288, 64, 10, T_},        // STD192_3
    {37, 4096, 875, 4096, 65536, 64, 8192, 64, 10, T_},          // STD192_4
    {35, 4096, 875, 1024, 32768, 32, 4096, 32, 10, T_},          // STD192Q
    {34, 4096, 922, 2048, 65536, 16, 4096, 64, 10, T_},          // STD192Q_3
    {34, 4096, 980, 2048, 131072, 16, 4096, 64, 10, T_},         // STD192Q_4
    {29, 4096, 1076, 2048, 32768, 32, 1024, 64, 10, T_},         // STD256
    {29, 4096, 1145, 2048, 65536, 64, 256, 64, 10, T_},          // STD256_3
    {29, 4096, 1145, 4096, 65536, 64, 256, 64, 10, T_},          // STD256_4
    {27, 4096, 1225, 1024, 65536, 16, 128, 32, 10, T_},          // STD256Q
    {27, 4096, 1400, 4096, 65536, 21, 64, 64, 10, T_},           // STD256Q_3
    {27, 4096, 1625, 4096, 2097152, 16, 64, 64, 10, T_},         // STD256Q_4
    {28, 2048, 447, 2048, 16384, 32, 1024, 64, 10, G_},          // STD128_LMKCDEY
    {27, 2048, 556, 2048, 32768, 32, 512, 64, 10, T_},           // STD128_3_LMKCDEY
    {27, 2048, 595, 2048, 65536, 64, 128, 64, 10, T_},           // STD128_4_LMKCDEY
    {27, 2048, 483, 2048, 16384, 32, 512, 64, 10, G_},           // STD128Q_LMKCDEY
    {25, 2048, 643, 2048, 65536, 64, 128, 64, 10, T_},           // STD128Q_3_LMKCDEY
    {50, 4096, 641, 4096, 65536, 64, 33554432, 64, 10, T_},      // STD128Q_4_LMKCDEY
    {39, 4096, 716, 2048, 32768, 32, 1048576, 64, 10, G_},       // STD192_LMKCDEY
    {39, 4096, 771, 4096, 65536, 64, 1048576, 64, 10, G_},       // STD192_3_LMKCDEY
    {37, 4096, 875, 4096, 65536, 64, 8192, 64, 10, T_},          // STD192_4_LMKCDEY
    {36, 4096, 776, 4096, 32768, 32, 262144, 64, 10, G_},        // STD192Q_LMKCDEY
    {36, 4096, 834, 4096, 65536, 64, 4096, 64, 10, G_},          // STD192Q_3_LMKCDEY
    {34, 4096, 949, 4096, 65536, 64, 4096, 64, 10, T_},          // STD192Q_4_LMKCDEY
    {30, 4096, 939, 2048, 32768, 32, 1024, 64, 10, G_},          // STD256_LMKCDEY
    {29, 4096, 1076, 4096, 32768, 32, 256, 64, 10, T_},          // STD256_3_LMKCDEY
    {29, 4096, 1145, 4096, 65536, 64, 256, 64, 10, T_},          // STD256_4_LMKCDEY
    {28, 4096, 1019, 4096, 32768, 32, 1024, 64, 10, G_},         // STD256Q_LMKCDEY
    {26, 4096, 1242, 4096, 65536, 64, 128, 64, 10, T_},          // STD256Q_3_LMKCDEY
    {26, 4096, 1320, 4096, 131072, 64, 64, 64, 10, T_},          // STD256Q_4_LMKCDEY
    {27, 2048, 556, 2048, 32768, 32, 128, 64, 10, T_},           // LPF_STD128
    {25, 2048, 645, 2048, 65536, 64, 128, 64, 10, T_},           // LPF_STD128Q
    {27, 2048, 556, 2048, 32768, 32, 512, 64, 10, T_},           // LPF_STD128_LMKCDEY
    {25, 2048, 600, 2048, 32768, 32, 128, 64, 10, T_},           // LPF_STD128Q_LMKCDEY
    {28, 2048, 512, 1024, 0, 25, 128, 23, 10, T_},               // SIGNED_MOD_TEST
};
constexpr int kNumRows = (int)(sizeof(kRows) / sizeof(kRows[0]));
}  // namespace

int paramset_rows() { return kNumRows; }

bool method_compatible(int paramset, int method) {
    if (paramset < 0 || paramset >= kNumRows) return false;
    const bool lmk_row = paramset == PS_TOY || paramset == 1 || (paramset >= PS_STD128_LMKCDEY && paramset <= 38) ||
                         paramset == 41 || paramset == 42;   // TOY, MEDIUM, *_LMKCDEY, LPF_*_LMKCDEY
    const bool cggi_row = paramset <= 20 || paramset == 39 || paramset == 40 || paramset == 43;  // .. SIGNED_MOD_TEST
    if (method == M_LMKCDEY) return lmk_row;
    if (method == M_AP || method == M_GINX) return cggi_row;
    return false;
}

Params make_params(int paramset, int method) {
    if (is_large(paramset)) return make_params_large(paramset, method);
    if (paramset < 0 || paramset >= kNumRows) throw std::invalid_argument("unknown parameter set");
    const Row& R = kRows[paramset];
    const uint32_t bits = R.bits, cyc = R.cyc, n = R.n, q = R.q, qks = R.qks, bks = R.bks, bg = R.bg;
    const uint32_t nauto = R.nauto;
    const int kd = R.kd;
    if (method != M_GINX && method != M_LMKCDEY && method != M_AP)
        throw std::invalid_argument("unsupported method (AP, GINX, LMKCDEY)");
    Params p;
    p.paramset = paramset;
    p.method = method;
    p.n = n;
    p.N = cyc / 2;
    p.q = q;
    p.Q = last_prime(bits, cyc);
    p.qKS = qks ? qks : p.Q;  // modKS == PRIME -> Q
    p.baseKS = bks;
    p.digitsKS = (uint32_t)std::ceil(std::log((double)p.qKS) / std::log((double)bks));  // lwe-pke.cpp:354
    p.baseG = bg;
    p.gBits = ilog2(bg);
    p.digitsG = (uint32_t)std::ceil(std::log((double)p.Q) / std::log((double)bg));      // rgsw-cryptoparameters.h:93-94
    p.digitsG2 = (p.digitsG - 1) * 2;
    p.numAutoKeys = nauto;
    p.keyDist = kd;
    p.baseR = R.brk;  // the baseRK column (binfhecontext.cpp:113-159)
    p.digitsR = (uint32_t)std::ceil(std::log((double)q) / std::log((double)p.baseR));
    p.psi = root_of_unity(cyc, p.Q);
    uint64_t v = 1;
    for (uint32_t i = 0; i < p.digitsG; ++i) {
        p.gpow.push_back(v);
        v = mulmod(v, bg, p.Q);
    }
    return p;
}

}  // namespace fhe_amd
