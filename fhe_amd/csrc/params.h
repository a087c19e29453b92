// params.h -- binfhe parameter sets (host).  Mirrors the rows of
// BinFHEContext::GenerateBinFHEContext (src/binfhe/lib/binfhecontext.cpp:113-179)
// and the derived constants of LWECryptoParams / RingGSWCryptoParams
// (src/binfhe/include/lwe-cryptoparameters.h:66-86, rgsw-cryptoparameters.h:77-97,
// src/binfhe/lib/rgsw-cryptoparameters.cpp:36-128).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace fhe_amd {

// reference enum values (src/binfhe/include/binfhe-constants.h:49-126)
enum ParamSet : int { PS_TOY = 0, PS_STD128_AP = 2, PS_STD128 = 3, PS_STD128_LMKCDEY = 21 };
// The large-precision family GenerateBinFHEContext(set, arbFunc, logQ, N, GINX, false)
// (binfhecontext.cpp:55-104) as one paramset code:
//   kLargeFamily | set << 16 | arbFunc << 15 | log2(N) << 8 (0: the minimum secure N) | logQ
constexpr int kLargeFamily = 1 << 30;
inline int large_paramset(int set, bool arbFunc, uint32_t logQ, uint32_t logN = 0) {
    return kLargeFamily | (set << 16) | ((arbFunc ? 1 : 0) << 15) | (int)(logN << 8) | (int)logQ;
}
inline bool is_large(int paramset) { return (paramset & kLargeFamily) != 0; }
enum Method : int { M_AP = 1, M_GINX = 2, M_LMKCDEY = 3 };
enum Gate : int { G_OR = 0, G_AND, G_NOR, G_NAND, G_XOR, G_XNOR, G_MAJORITY, G_AND3, G_OR3, G_AND4, G_OR4,
                  G_XOR_FAST, G_XNOR_FAST, G_CMUX };
enum KeyDist : int { KD_GAUSSIAN = 0, KD_UNIFORM_TERNARY = 1 };

struct Params {
    int paramset = 0, method = 0;
    uint32_t n = 0, N = 0, q = 0, baseKS = 0, digitsKS = 0;
    uint64_t qKS = 0;  // 2^14 (STD128 sets), 2^35 (large-precision family)
    uint32_t baseG = 0, gBits = 0, digitsG = 0, digitsG2 = 0, numAutoKeys = 0;
    uint32_t baseR = 0, digitsR = 0;  // AP/DM refresh base and digit count (rgsw-cryptoparameters.cpp:37-46)
    int keyDist = KD_UNIFORM_TERNARY;
    uint64_t Q = 0, psi = 0;
    std::vector<uint64_t> gpow;  // Gpow[i] = baseG^i mod Q (rgsw-cryptoparameters.cpp:69-74)

    // raw (reference-layout) key sizes in u64 words
    size_t bsk_words() const;
    size_t ksk_rows() const { return (size_t)N * baseKS * digitsKS; }
    uint64_t gate_const(int gate) const;  // rgsw-cryptoparameters.cpp:78-92
};

// Throws std::invalid_argument on an unsupported set/method.
Params make_params(int paramset, int method);

}  // namespace fhe_amd
