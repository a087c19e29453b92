// packed.h -- the reference's packed GPU-transfer format (src/binfhe/include/backend/packed.h:
// 29-307, implementation src/binfhe/lib/backend/packed.cpp), byte for byte: a 32-byte common
// header ("LUXF", version 1, type, total size, element count, flags) followed by a type-specific
// block and little-endian u64 words.
//   LWE_BATCH (2):          64-byte header block (n, log_q, q, count, stride); coefficients
//                           sequential [ct][a_0 .. a_{n-1}, b] or, with flag INTERLEAVED (1),
//                           [j][ct] for the a's followed by all b's (PackLWEBatch, packed.cpp:144-211)
//   BOOTSTRAPPING_KEY (5):  72-byte block; the reference's packer is a TODO (packed.cpp:284-307).
//                           Defined here: header.flags = BINFHE_METHOD, lwe_n = n, lwe_log_q =
//                           log2 q, rlwe_N = N, rlwe_num_limbs = 1, decomp_levels = digitsG2,
//                           decomp_base_log = log2 baseG, key_size = bytes of key data,
//                           key_layout = KEY_LAYOUT_NTT; then the raw u64 key (include/fhe_hip.h).
//   SWITCHING_KEY (6):      64-byte block (input_n = N, output_n = n, decomp_levels = digitsKS,
//                           decomp_base_log = floor(log2 baseKS), reserved[0] = baseKS, Q = qKS,
//                           header.element_count = rows); then A [N][baseKS][digitsKS][n] and
//                           B [N][baseKS][digitsKS] u64 (timeOptimization: the map's three keys, A
//                           then B) (the reference's packer is a TODO, packed.cpp:313-328).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace fhe_amd {

constexpr uint32_t kPackedMagic   = 0x4C555846;  // "LUXF"
constexpr uint16_t kPackedVersion = 1;
enum PackedType : uint16_t { PT_LWE = 1, PT_LWE_BATCH = 2, PT_BSK = 5, PT_KSK = 6 };
enum : uint32_t { LWE_PACK_INTERLEAVED = 1u, KEY_LAYOUT_NTT = 2u };

#pragma pack(push, 1)
struct PackedHeader {
    uint32_t magic;
    uint16_t version;
    uint16_t type;
    uint64_t total_size;
    uint64_t element_count;
    uint32_t flags;
    uint32_t reserved;
};
struct PackedLWEBatchHdr {
    PackedHeader h;
    uint32_t n, log_q;
    uint64_t q, count;
    uint32_t stride, reserved;
};
struct PackedBskHdr {
    PackedHeader h;
    uint32_t lwe_n, lwe_log_q, rlwe_N, rlwe_num_limbs, decomp_levels, decomp_base_log;
    uint64_t key_size;
    uint32_t key_layout, reserved;
};
struct PackedKskHdr {
    PackedHeader h;
    uint32_t input_n, output_n, decomp_levels, decomp_base_log;
    uint64_t Q;
    uint32_t reserved[2];
};
#pragma pack(pop)
static_assert(sizeof(PackedHeader) == 32, "PackedHeader");
static_assert(sizeof(PackedLWEBatchHdr) == 64, "PackedLWEBatch");
static_assert(sizeof(PackedBskHdr) == 72, "PackedBootstrappingKey");
static_assert(sizeof(PackedKskHdr) == 64, "PackedSwitchingKey");

// LWE batches
size_t packed_lwe_batch_size(uint32_t n, size_t count);
void pack_lwe_batch(uint32_t n, size_t count, const uint64_t* a, const uint64_t* b, uint32_t flags, uint8_t* out);
// parses and validates; a/b may be null to query n and count only
void unpack_lwe_batch(const uint8_t* data, size_t size, uint32_t* n, size_t* count, uint64_t* a, uint64_t* b);

// keys (formats defined above); unpack returns views into `data`
struct Params;
std::vector<uint8_t> pack_bsk(const Params& p, const uint64_t* bsk, size_t words);
const uint64_t* unpack_bsk(const Params& p, const uint8_t* data, size_t size, size_t* words);
std::vector<uint8_t> pack_ksk(const Params& p, const uint64_t* A, const uint64_t* B);
void unpack_ksk(const Params& p, const uint8_t* data, size_t size, const uint64_t** A, const uint64_t** B);

}  // namespace fhe_amd
