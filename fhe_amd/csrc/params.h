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
// timeOptimization = true (binfhecontext.cpp:55-104, BTKeyGen :285-307): for logQ != 11 the
// context holds one bootstrapping key per baseG in {2^14, 2^18, 2^27} (m_BTKey_map), and
// EvalSign / EvalDecomp change the base as the modulus shrinks (binfhe-base-scheme.cpp:409-431)
constexpr int kTimeOpt = 1 << 14;
inline int large_paramset(int set, bool arbFunc, uint32_t logQ, uint32_t logN = 0, bool timeopt = false) {
    return kLargeFamily | (set << 16) | ((arbFunc ? 1 : 0) << 15) | (timeopt ? kTimeOpt : 0) | (int)(logN << 8) |
           (int)logQ;
}
constexpr uint32_t kSignBases[3] = {1u << 14, 1u << 18, 1u << 27};  // rgsw-cryptoparameters.cpp:50
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
    bool timeopt = false;        // the three-key map of timeOptimization (kSignBases)

    // raw (reference-layout) key sizes in u64 words; with timeopt the map's keys, concatenated in
    // the map's (ascending baseG) order
    size_t bsk_words() const;
    size_t bsk_words_one() const;            // one key at this baseG
    size_t bsk_offset(uint32_t bg) const;    // timeopt: first word of the key for baseG bg
    // RingGSWCryptoParams::Change_BaseG (rgsw-cryptoparameters.h:222-229): baseG, digitsG, Gpow
    Params with_base(uint32_t bg) const;
    size_t ksk_rows() const { return (size_t)N * baseKS * digitsKS; }   // rows of one switching key
    // timeOptimization: BTKeyGen's map holds one whole key per base (binfhecontext.cpp:292-296 calls
    // KeyGen per base: its own RLWE secret and switching key); the raw layouts concatenate the three
    // switching keys (A rows then B per key array, kSignBases order)
    size_t ksk_keys() const { return timeopt ? 3 : 1; }
    size_t ksk_rows_all() const { return ksk_rows() * ksk_keys(); }
    size_t ksk_index(uint32_t bg) const;   // timeopt: which of the map's switching keys baseG bg uses
    uint64_t gate_const(int gate) const;  // rgsw-cryptoparameters.cpp:78-92
};

// Throws std::invalid_argument on an unsupported set/method.
Params make_params(int paramset, int method);
// the rows of the GenerateBinFHEContext(set, method) table (paramset codes 0 .. count - 1) and
// isMethodCompatible (binfhe-constants-impl.cpp:266-330)
int paramset_rows();
bool method_compatible(int paramset, int method);

}  // namespace fhe_amd
