// nt.h -- host number theory for parameter setup (init only, never on the hot path).
// Restates the reference's LastPrime (src/core/include/math/nbtheory-impl.h:350-371),
// RootOfUnity (:183-228, minimal primitive root) and ReverseBits (nbtheory.h:135).
#pragma once
#include <stdint.h>

#include <vector>

namespace fhe_amd {

typedef unsigned __int128 u128;

inline uint64_t mulmod(uint64_t a, uint64_t b, uint64_t m) { return (uint64_t)(((u128)a * b) % m); }
inline uint64_t addmod(uint64_t a, uint64_t b, uint64_t m) { uint64_t s = a + b; return s >= m ? s - m : s; }
inline uint64_t submod(uint64_t a, uint64_t b, uint64_t m) { return a >= b ? a - b : a + m - b; }
uint64_t powmod(uint64_t b, uint64_t e, uint64_t m);
inline uint64_t invmod(uint64_t a, uint64_t m) { return powmod(a, m - 2, m); }  // m prime
bool is_prime(uint64_t n);
uint64_t last_prime(uint32_t bits, uint64_t m);
uint64_t root_of_unity(uint64_t m, uint64_t Q);
inline uint32_t reverse_bits(uint32_t x, uint32_t bits) {
    uint32_t r = 0;
    for (uint32_t i = 0; i < bits; ++i) r |= ((x >> i) & 1u) << (bits - 1 - i);
    return r;
}
inline uint32_t ilog2(uint64_t x) { uint32_t r = 0; while (x > 1) { x >>= 1; ++r; } return r; }
inline uint32_t shoup32(uint64_t w, uint64_t Q) { return (uint32_t)(((u128)w << 32) / Q); }
inline uint64_t shoup64(uint64_t w, uint64_t Q) { return (uint64_t)(((u128)w << 64) / Q); }

// Host NTT (same transform as the device kernels) for key generation.
struct HostNtt {
    uint32_t N = 0, logN = 0;
    uint64_t Q = 0, psi = 0, ninv = 0;
    std::vector<uint64_t> tab, tabI;  // Table[brv(i)] = psi^i, TableI[brv(i)] = psi^-i
    void init(uint32_t N, uint64_t Q, uint64_t psi);
    void forward(uint64_t* a) const;
    void inverse(uint64_t* a) const;
};

}  // namespace fhe_amd
