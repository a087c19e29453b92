// cereal.h -- the reference's serialized key / ciphertext files.
//
// Reads and writes the byte streams Serial::Serialize(obj, stream, SerType::BINARY)
// produces (src/core/include/utils/serial.h:95-125; types registered in
// src/binfhe/include/binfhecontext-ser.h): a cereal PortableBinary archive
// (one endianness byte, little-endian scalars) of
//   RingGSWACCKey   (rgsw-acckey.h:136-155)   -> raw BSK layout (include/fhe_hip.h)
//   LWESwitchingKey (lwe-keyswitchkey.h:102-125) -> raw KSK A / B
//   LWECiphertext   (lwe-ciphertext.h:134-156) -> a[n], b, modulus
//   LWEPrivateKey   (lwe-privatekey.h:92-110)  -> s[n], modulus
// Archive rules the streams follow (cereal's own, vendored under
// install/include/openfhe/cereal): a class's u32 version is written the first
// time the class appears; a polymorphic shared_ptr whose dynamic type is its
// static type is u32 0x40000000 then u32 pointer id (bit 31 set: first
// occurrence, object follows; 0 id word: null); std::vector is a u64 size then
// the elements; a unique_ptr is a u8 "valid" flag then the object.
// Native code, no reference source: written from the observed archive layout
// and pinned byte-for-byte against the reference's own serializer (tests/test_cereal.py).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "params.h"

namespace fhe_amd {

// keys: Params decides the expected shapes (method, n, N, Q, qKS, digits)
void cereal_read_bsk(const Params& p, const uint8_t* data, size_t size, std::vector<uint64_t>& bsk);
void cereal_read_ksk(const Params& p, const uint8_t* data, size_t size, std::vector<uint64_t>& A,
                     std::vector<uint64_t>& B);
std::string cereal_write_bsk(const Params& p, const uint64_t* bsk);
std::string cereal_write_ksk(const Params& p, const uint64_t* A, const uint64_t* B);

// LWE ciphertext (is_key = false) or LWE secret key (is_key = true): a NativeVector (+ b)
struct CerealLwe {
    std::vector<uint64_t> a;
    uint64_t b = 0, mod = 0;
};
CerealLwe cereal_read_lwe(const uint8_t* data, size_t size, bool is_key);
std::string cereal_write_lwe(const uint64_t* a, uint32_t n, uint64_t b, uint64_t mod, bool is_key);

// The key-independent cryptoContext archive: Serial::Serialize(BinFHEContext) (boolean-serial-binary.cpp:
// 65-71, 108) = BinFHEContext (binfhecontext.h:410-422) -> shared_ptr<BinFHECryptoParams>
// (binfhe-base-params.h:103-116) -> shared_ptr<LWECryptoParams> (lwe-cryptoparameters.h:182-212) and
// shared_ptr<RingGSWCryptoParams> (rgsw-cryptoparameters.h:181-214, its ILNativeParams as in the keys)
struct CerealContext {
    uint32_t n = 0, N = 0, baseKS = 0;                       // LWECryptoParams
    uint64_t q = 0, Q = 0, qKS = 0;
    double sigma = 0, sigmaKS = 0;
    uint32_t rN = 0, baseR = 0, baseG = 0, method = 0, digitsG = 0, numAutoKeys = 0;  // RingGSWCryptoParams
    uint64_t rQ = 0, rq = 0;
    double rsigma = 0;
    uint32_t order = 0, ringDim = 0;                          // ILNativeParams
    uint64_t mod = 0, root = 0, bigMod = 0, bigRoot = 0;
};
CerealContext cereal_read_context(const uint8_t* data, size_t size);
std::string cereal_write_context(const Params& p);
// the GenerateBinFHEContext(set, method) row whose parameters the archive holds (the archive records no
// set name); false when no supported row matches
bool cereal_context_paramset(const CerealContext& c, int& paramset, int& method);

}  // namespace fhe_amd
