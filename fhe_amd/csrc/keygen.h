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
// Gaussian samples (errors, and the secrets of the GAUSSIAN key distribution) follow the reference's
// own sampler for sigma = 3.19 < KARNEY_THRESHOLD: DiscreteGaussianGeneratorImpl's inversion method
// (discretegaussiangenerator-impl.h:78-132) with its table, thresholds and sign rule, one uniform
// double per sample.  Differences from the reference, which do not affect evaluation parity
// (evaluation is deterministic given the keys): randomness comes from a seeded counter-based
// generator instead of BLAKE2, and the uniform mask of each RGSW row is drawn directly in the
// EVALUATION domain (the NTT of a uniform polynomial is uniform).
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

#if defined(__HIPCC__)
#define FHE_HD __host__ __device__
#else
#define FHE_HD
#endif
// counter-based generator: stream (seed, tag, stream) yields out_k = mix64(rng_state(..) + (k + 2) * kRngGamma)
// for its k-th draw, so the device key generation (keygen_dev.hip) reproduces any draw independently.
// The stream's state is a hash of (seed, tag, stream): nearby seeds give unrelated streams.
enum RngTag : uint64_t { T_SK = 1, T_SKN, T_BSK, T_KSK, T_ENC, T_AUTO };
constexpr uint64_t kRngGamma = 0x9E3779B97F4A7C15ull;
FHE_HD inline uint64_t mix64(uint64_t z) {  // splitmix64's finaliser
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
FHE_HD inline uint64_t rng_state(uint64_t seed, uint64_t tag, uint64_t stream) {
    return mix64(mix64(seed ^ (tag << 56)) + stream * 0xD1B54A32D192ED03ull);
}

// DiscreteGaussianGeneratorImpl::Initialize for sigma = STD_DEV = 3.19 (discretegaussiangenerator-impl.h:
// 78-97; binfhecontext.cpp:107-179 uses it for every error and Gaussian secret): fin = ceil(sigma M),
// M = 12.00610553538285, vals[x - 1] = a sum_{1 <= y <= x} exp(-y^2 / (2 sigma^2)), a = 1 / (2 sum + 1)
constexpr double kDggSigma = 3.19;
constexpr int kDggMaxFin = 40;
struct DggTable {
    double a;
    int fin;
    double vals[kDggMaxFin];
};
const DggTable& dgg_table();  // the host's table (computed once, exactly as the reference computes it)
// GenerateIntVector's inversion step (:120-131) on one 64-bit draw r: u = r 2^-64 in [0, 1) at double
// precision, seed = u - 1/2, tmp = |seed| - a/2; 0 if tmp <= 0, else +-(1 + the index of the first
// vals[i] >= tmp) with the sign of seed (the reference throws past the table end, a 2^-100 event: here
// the last value)
FHE_HD inline int64_t dgg_sample(uint64_t r, const DggTable& t) {
    const double u = (double)(r >> 11) * 0x1p-53;
    const double seed = u - 0.5;
    const double tmp = (seed < 0 ? -seed : seed) - t.a / 2;
    if (tmp <= 0) return 0;
    int lo = 0, hi = t.fin;  // lower_bound
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (t.vals[mid] < tmp) lo = mid + 1;
        else hi = mid;
    }
    const int64_t v = lo < t.fin ? lo + 1 : t.fin;
    return seed > 0 ? v : -v;
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
// ptmod and ciphertext modulus mod (0: q); len: the dimension (0: n; N with skN for EncryptN's LARGE_DIM)
void encrypt(const Params& p, const uint64_t* sk, const int* bits, size_t count, uint64_t seed, uint64_t* a,
             uint64_t* b, uint32_t ptmod = 4, uint64_t mod = 0, uint32_t len = 0);
int64_t decrypt(const Params& p, const uint64_t* sk, const uint64_t* a, uint64_t b, uint32_t len, uint64_t mod,
                uint32_t ptmod = 4);

}  // namespace fhe_amd
