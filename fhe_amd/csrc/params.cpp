// params.cpp -- see params.h.
#include "params.h"

#include <cmath>
#include <stdexcept>

#include "nt.h"

namespace fhe_amd {

size_t Params::bsk_words() const {
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

Params make_params(int paramset, int method) {
    if (is_large(paramset)) return make_params_large(paramset, method);
    //            bits cyc   n    q     qKS    Bks  Bg    nAuto keyDist   (binfhecontext.cpp:113-159)
    uint32_t bits, cyc, n, q, qks, bks, bg, nauto;
    int kd;
    switch (paramset) {
        case PS_TOY:            bits = 27; cyc = 1024; n = 64;  q = 512;  qks = 0;     bks = 25; bg = 512;  nauto = 9;  kd = KD_UNIFORM_TERNARY; break;
        case PS_STD128_AP:
        case PS_STD128:         bits = 27; cyc = 2048; n = 503; q = 1024; qks = 16384; bks = 32; bg = 512;  nauto = 10; kd = KD_UNIFORM_TERNARY; break;
        case PS_STD128_LMKCDEY: bits = 28; cyc = 2048; n = 447; q = 2048; qks = 16384; bks = 32; bg = 1024; nauto = 10; kd = KD_GAUSSIAN; break;
        default: throw std::invalid_argument("unsupported parameter set (TOY, STD128_AP, STD128, STD128_LMKCDEY)");
    }
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
    p.baseR = 32;  // baseRK column of every row (binfhecontext.cpp:113-159)
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
