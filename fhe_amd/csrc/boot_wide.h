// boot_wide.h -- the wide accumulator (bootstrap_wide.hip): the large-precision parameter family, and
// every parameter set outside the 32-bit register-resident kernels (A32 policy below Q < 2^30).
// The large-precision family:
// GenerateBinFHEContext(set, arbFunc, logQ, N, GINX, false) (binfhecontext.cpp:55-104) with a
// 54-bit accumulator modulus Q (27-bit for logQ = 11), N = 2048 (1024), qKS = 2^35, n = 1305.
// The accumulator works in 64-bit residues: Shoup products for the NTT twiddles, 128-bit digit x
// key sums with one Montgomery (R = 2^64) reduction per slot; the key switch sums u64 rows mod
// 2^35.  ModSwitch (RoundqQ, lwe-pke.cpp:41-46) is evaluated in IEEE double exactly as the
// reference writes it: v * q / Q with v up to 2^54 is not exact in double, so no integer form.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "boot.h"

namespace fhe_amd {

struct WideTables {
    const uint64_t* tab;    // Table[N]: psi^i at bit-reversed i (transformnat-impl.h:777-831)
    const uint64_t* tabS;   // floor(Table * 2^64 / Q) (Shoup quotients)
    const uint64_t* tabI;   // TableI[N]: psi^-i at bit-reversed i
    const uint64_t* tabIS;
    const uint64_t* psiM;   // psi^e * 2^64 mod Q, e in [0, 2N): EVAL(X^m) at slot j = psi^((2 brv(j) + 1) m)
    uint64_t Q, qinv;       // qinv = -Q^-1 mod 2^64
    uint64_t ninv, ninvS;   // N^-1 and its Shoup quotient
    uint64_t oneM;          // 2^64 mod Q
    uint64_t r2;            // 2^128 mod Q (keys into Montgomery form)
    // narrow = 1: the 32-bit policy (Q < 2^30, digitsG2 Q < 2^32): the same tables one word wide,
    // Shoup quotients floor(w 2^32 / Q), Montgomery R = 2^32, and every key array in u32 words
    uint32_t narrow;
    const uint32_t *tab32, *tabS32, *tabI32, *tabIS32, *psiM32;
    uint32_t Q32, qinv32, ninv32, ninvS32, oneM32, r2_32;
};

// one bootstrap launch: the blind rotation of GINX (rgsw-acc-cggi.cpp:59-151) over the monomial
// exponents prep wrote (launch_prep_ginx), its test vector, and the extraction of ctExt
// (binfhe-base-scheme.cpp:110-121 / :624-626), optionally ModSwitch(Q -> qKS)
struct WideArgs {
    uint32_t count, n, N, ctmod, factor;
    uint32_t lb, ub;             // gate test-vector window (BootstrapGateCore)
    uint32_t digitsG, gbits;
    uint32_t msb_out;            // 1: ext mod-switched to qKS; 0: raw mod Q
    uint64_t lv, uv;             // window values
    uint64_t b_const;            // added to acc1[0]
    uint64_t qKS;
    const uint64_t* tv;          // BootstrapFunc test vector (Q / fmod) f(x), x < ctmod; null: gate window
    // Backend::BlindRotate / ExternalProduct seam (GateArgs::acc_io / acc_tv): non-null = the final
    // accumulator goes to acc_io[count][2][N] (EVALUATION, canonical) instead of the extraction; the
    // initial one is read from there too unless acc_tv (then the test vector above, as for a gate)
    uint64_t* acc_io;
    uint32_t acc_tv;
    uint32_t tv_mod;             // GateArgs::tv_mod: gate g reads table tv + (g % tv_mod) ctmod
};

// bsk: [n][2][dG2][2][N] Montgomery keys, u64 words (u32 with t.narrow)
hipError_t launch_blind_rotate_wide(const WideArgs& g, const WideTables& t, const void* bsk, const uint16_t* idx,
                                    const uint32_t* tvb, uint64_t* ext_a, uint64_t* ext_b, hipStream_t s);
// LMKCDEY / DM on the wide accumulator: the op lists of launch_prep_lmk / launch_prep_dm
// (k_blind_rotate_wide_ops); bsk = the EXT keys [keys][digitsG2][2][N], autok = [numAutoKeys +
// 1][digitsG - 1][2][N], Montgomery form (u64, or u32 with t.narrow)
hipError_t launch_blind_rotate_wide_ops(const WideArgs& g, const WideTables& t, const void* bsk, const void* autok,
                                        const uint16_t* ops, const uint32_t* nops, uint32_t maxops, const uint32_t* tvb,
                                        uint64_t* ext_a, uint64_t* ext_b, bool dm, hipStream_t s);
// ExternalProduct seam: raw RGSW words (< Q) -> the Montgomery form of the op-list kernel's keys
// (u64 words, u32 with t.narrow)
hipError_t launch_pack_rgsw_wide(const uint64_t* raw, size_t words, const WideTables& t, void* out, hipStream_t s);
// KeySwitch (lwe-pke.cpp:348-372) mod qKS = 2^k with u64 rows A [rows][n], B [rows], then
// ModSwitch(qKS -> q_out) (q_out = 0: none); ms_a [count][N], ms_b [count] mod qKS
hipError_t launch_keyswitch_wide(size_t count, uint32_t n, uint32_t N, uint32_t baseKS, uint32_t digitsKS, uint64_t qKS,
                                 const uint64_t* A, const uint64_t* B, const uint64_t* ms_a, const uint64_t* ms_b,
                                 uint64_t q_out, uint64_t* a_out, uint64_t* b_out, hipStream_t s);

}  // namespace fhe_amd
