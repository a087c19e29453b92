// keygen.h -- deterministic, seeded host key generation / encryption / decryption.
//
// Produces keys with exactly the reference's structure and raw layout, so that
// the reference itself can consume them through BTKeyLoad
// (src/binfhe/include/binfhecontext.h:273-275):
//   LWE secret  : LWEEncryptionScheme::KeyGen / KeyGenGaussian   (lwe-pke.cpp:48-56), stored mod qKS
//   RLWE secret : skN (BinFHEScheme::KeyGen, binfhe-base-scheme.cpp:39-73), stored mod Q
//   GINX BSK    : RingGSWAccumulatorCGGI::KeyGenAcc/KeyGenCGGI   (rgsw-acc-cggi.cpp:39-96)
//   LMKCDEY BSK : RingGSWAccumulatorLMKCDEY::KeyGenAcc/KeyGenLMKCDEY/KeyGenAuto
//                                                                (rgsw-acc-lmkcdey.cpp:39-226)
//   KSK         : LWEEncryptionScheme::KeySwitchGen             (lwe-pke.cpp:264-344)
//   Encrypt     : LWEEncryptionScheme::Encrypt                  (lwe-pke.cpp:116-146)
// Differences from the reference, which do not affect evaluation parity
// (evaluation is deterministic given the keys): randomness comes from a
// seeded counter-based generator instead of BLAKE2, Gaussian samples are a
// centred binomial with k = 20 (sigma ~ 3.16 vs the reference's 3.19), and the
// uniform mask of each RGSW row is drawn directly in the EVALUATION domain
// (the NTT of a uniform polynomial is uniform).
#pragma once
#include <stdint.h>

#include <vector>

#include "params.h"

namespace fhe_amd {

struct KeySet {
    std::vector<uint64_t> sk;    // n, mod qKS
    std::vector<uint64_t> skN;   // N, mod Q
    std::vector<uint64_t> bsk;   // Params::bsk_words()
    std::vector<uint64_t> kskA;  // ksk_rows() * n
    std::vector<uint64_t> kskB;  // ksk_rows()
};

// counter-based generator: stream (seed, tag, stream) yields out_k = mix(rng_state(..) + (k + 2) * kRngGamma)
// for its k-th draw, so the device key generation (keygen_dev.hip) reproduces any draw independently
enum RngTag : uint64_t { T_SK = 1, T_SKN, T_BSK, T_KSK, T_ENC, T_AUTO };
constexpr uint64_t kRngGamma = 0x9E3779B97F4A7C15ull;
inline uint64_t rng_state(uint64_t seed, uint64_t tag, uint64_t stream) {
    return seed * kRngGamma ^ (tag << 56) ^ (stream * 0xD1B54A32D192ED03ull);
}

void keygen_secret(const Params& p, uint64_t seed, std::vector<uint64_t>& sk);
// RLWE secret skN (mod Q) of BTKeyGen
void keygen_ring_secret(const Params& p, uint64_t seed, std::vector<uint64_t>& skN);
// AutomorphismTransform(k) of an EVALUATION-domain polynomial (poly-impl.h:350-356)
void auto_eval(const Params& p, uint32_t k, const uint64_t* in, uint64_t* out);
void keygen_bootstrap(const Params& p, const std::vector<uint64_t>& sk, uint64_t seed, KeySet& out);
// the same keys generated on a device (keygen_dev.hip): BSK in the engine's packed Montgomery
// layout (d_bsk, bsk_words u32) and KSK in its u16 row layout (d_ksk, ksk_rows x 512); when the
// raw_* device pointers are non-null the reference raw layouts are written there as well
void keygen_bootstrap_device(const Params& p, const std::vector<uint64_t>& sk, uint64_t seed, int device,
                             uint32_t* d_bsk, uint16_t* d_ksk, uint64_t* raw_bsk, uint64_t* raw_kskA,
                             uint64_t* raw_kskB, void* stream);
// LWEEncryptionScheme::Encrypt / Decrypt (lwe-pke.cpp:103-128, 181-226) with plaintext modulus
// ptmod and ciphertext modulus mod (0: q)
void encrypt(const Params& p, const uint64_t* sk, const int* bits, size_t count, uint64_t seed, uint64_t* a,
             uint64_t* b, uint32_t ptmod = 4, uint64_t mod = 0);
int64_t decrypt(const Params& p, const uint64_t* sk, const uint64_t* a, uint64_t b, uint32_t len, uint64_t mod,
                uint32_t ptmod = 4);

}  // namespace fhe_amd
