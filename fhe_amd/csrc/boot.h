// boot.h -- device-side argument blocks and launchers for the gate bootstrap
// (bootstrap.hip) and the LWE key switch (keyswitch.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fhe_amd {

// Twiddle/monomial tables for the fused accumulator kernels (all u32,
// Montgomery form x * 2^32 mod Q).
// monomial tables (N = 1024, entries padded by one word per 32, 16-byte rounded):
//   half resolution: psi^(2f) - 1 for f in [0, 2N] at f + (f >> 5)  (exponents a * 2N/ctmod even)
//   full resolution: psi^e - 1 for e in [0, 4N] at e + (e >> 5)     (ctmod = 2N: any exponent)
constexpr int kMonoHalfWords = 2176;
constexpr int kMonoTableWords = 4228;

struct BootTables {
    const uint32_t* twA_fwd;  // Table[0..31]   (uniform stages on bits 9..5)
    const uint32_t* twA_inv;  // TableI[0..31]
    const uint32_t* twB_fwd;  // 992 words: lane-major Table entries of the stages on bits 4..0
    const uint32_t* twB_inv;  // 992 words: same for TableI
    const uint32_t* mono;     // kMonoHalfWords: psi^(2f) - 1 -> EVAL(X^m - 1) = omega_j^m - 1, m even
    const uint32_t* mono_full;  // kMonoTableWords: psi^e - 1, any m
    const uint32_t* monoP;       // plain (non-Montgomery) copies of mono / mono_full: the signed
    const uint32_t* monoP_full;  // accumulator multiplies the unreduced 64-bit digit-key sums by both
    const uint32_t* tabI;        // TableI[0..1023] (the LMKCDEY automorphism's wave-wide inverse NTT)
    const uint32_t* tabF;        // Table[0..1023] (the split GINX kernel's wave-wide forward NTT)
    uint32_t Q, Q2, qinv;     // qinv = -Q^-1 mod 2^32
    // The resident keys carry a factor N^-1 (folded in at packing), so the EVALUATION accumulator
    // is N^-1 * acc and the last inverse stage needs no N^-1 multiply: it scales by TableI[1] only.
    uint32_t ninvR;  // N^-1 (Montgomery): scales the initial accumulator
    uint32_t w1R;    // TableI[1] (Montgomery) for the last iNTT stage
    uint32_t oneR;   // 2^32 mod Q (Montgomery 1): x -> x mod Q by one signed Montgomery product
    uint32_t nR;     // N (Montgomery): undoes the N^-1 scaling when the accumulator is written out
};

// Digit exchange between the half-waves in the external products: ds_bpermute of the other half's
// digits, with the key rows of half 1 stored swapped in pairs (row d at position d ^ 1) so that every
// lane multiplies (own, other) digits in the same order.  Engine::load_bsk and the device key
// generator write this layout.
constexpr bool kBskHalfSwap = true;
// GINX: the two ternary keys of an index (BSK+ / BSK-) interleaved per lane as one 16-byte
// vector (K+[2k], K+[2k+1], K-[2k], K-[2k+1]) per digit row and slot pair: one load per digit
constexpr bool kGinxU4 = true;
// op-list methods (LMKCDEY, AP/DM, automorphism keys): the 4 slots l*32 + 4kk .. +3 of a lane as
// one 16-byte vector per row; word offset within a key of (row d, slot pair k = 0..15, lane, e)
__host__ __device__ constexpr size_t row_off(uint32_t d, uint32_t k, uint32_t lane, uint32_t e) {
    return (((size_t)d * 8 + (k >> 1)) * 64 + lane) * 4 + (k & 1) * 2 + e;
}
// word offset, within index i's 2 * dG2 * 2N words, of (sign ks, row d, slot pair k, lane, e)
__host__ __device__ constexpr size_t ginx_u4_off(uint32_t ks, uint32_t d, uint32_t k, uint32_t lane, uint32_t e) {
    return (((size_t)d * 16 + k) * 64 + lane) * 4 + ks * 2 + e;
}

// u16 key-switching-key rows: A[n] then B at column n, zero-padded to 512 columns (n < 512, both
// STD128 sets), 1024 (n < 1024: STD128_3, LPF_STD128, ...) or the next multiple of 128 (STD256Q:
// n = 1225 -> 1280)
__host__ __device__ constexpr uint32_t ksk_width(uint32_t n) {
    return n < 512 ? 512u : n < 1024 ? 1024u : (n + 1 + 127) / 128 * 128;  // n >= 1024: the N = 2048 rows
}

struct GateArgs {
    uint32_t count, n, N, q, qKS;
    uint32_t ctmod;                   // modulus of the bootstrapped ct's a (q; 2q for BootstrapFunc), power of 2
    uint32_t lb, ub, lv, uv, factor;  // BootstrapGateCore test-vector window (binfhe-base-scheme.cpp:535-567)
    const uint32_t* tv;               // BootstrapFuncCore test vector (binfhe-base-scheme.cpp:596-608): tv[x] =
                                      // (Q / fmod) f(x) for x < ctmod; null: gate window lb/ub/lv/uv
    uint32_t b_const;                 // Q/(2p) + 1 (binfhe-base-scheme.cpp:118-120, :162-163)
    uint32_t xor_double;              // XOR/XNOR: 2 (ct1 + ct2)
    uint32_t msb_out;                 // 1: write ctExt mod-switched to qKS; 0: raw ctExt mod Q
    uint32_t gbits;                   // log2(baseG)
    // the large-precision family (boot_wide.h): the same window / test vector / b with 64-bit Q
    uint64_t lv64, uv64, b64;
    const uint64_t* tv64;
    // Backend::BlindRotate / ExternalProduct seam (backend.h:131-146, 177-192): non-null selects the
    // accumulator-I/O instantiation of the blind-rotation kernels.  The initial accumulator is read
    // from acc_io[count][2][N] (EVALUATION, bit-reversed as the reference stores it, canonical mod Q)
    // instead of being built from the test vector, and the final one is written back there in the
    // same form instead of the extraction / ModSwitch epilogue.
    uint64_t* acc_io;
    // with acc_io: 1 = the initial accumulator is BootstrapGateCore's test vector (0, NTT(m))
    // (binfhe-base-scheme.cpp:556-575) from the gate window and tvb, as for a gate, instead of acc_io's
    // contents -- the seam's null accumulators (BootstrapBatch, batch.cpp:77-86); the final
    // accumulator still goes to acc_io
    uint32_t acc_tv;
    // BootstrapFunc with several tables (EvalFuncMultiOutputBatch, batch.cpp:141-174): tv_mod > 1 cycles
    // gate g through table g % tv_mod, at tv + (g % tv_mod) ctmod (tv64 likewise); 0 / 1: the one table
    uint32_t tv_mod;
};

// The LWE ciphertext a gate bootstraps: ct = sum_j (-1)^{neg_j} ct_j + (0, boff) mod q, then
// doubled for XOR/XNOR.  2-input gates: k = 2 (binfhe-base-scheme.cpp:95-107); AND3/OR3/AND4/
// OR4/MAJORITY: k = 3..4 (:146-150); CMUX's NAND(ct0, NOT ct2): neg = {ct2}, boff = q/4
// (EvalNOT :223-236 folded into the sum).  Inputs are u64 [count][n] / [count], mod q.
struct GateInputs {
    const uint64_t* a[4];
    const uint64_t* b[4];
    uint32_t k;         // 1..4
    uint32_t neg_mask;  // bit j: subtract input j
    uint32_t boff;      // added to b
};

// GINX/CGGI: inputs -> monomial exponents + test-vector b
hipError_t launch_prep_ginx(const GateArgs& g, const GateInputs& in, uint16_t* idx, uint32_t* tvb, hipStream_t s);
// GINX with two waves per gate (one RLWE component each): keys repacked from the resident GINX
// layout (launch_repack_ginx2); launched for gate batches with Q < 2^27 and ciphertext modulus q < 2N
hipError_t launch_repack_ginx2(const void* bsk, uint32_t n, void* bsk2, hipStream_t s);
hipError_t launch_blind_rotate_ginx2(const GateArgs& g, const BootTables& t, const void* bsk2, const uint16_t* idx,
                                     const uint32_t* tvb, uint32_t* ext_a, uint32_t* ext_b, hipStream_t s);
bool ginx2_supported(const GateArgs& g, const BootTables& t);
// K1x: two waves per gate with K1w's one-word exchange (the small-batch GINX kernel), same support as K1s;
// keys repacked from the resident layout into [i][c][q < 4][k2 < 8][64 lanes][4 words] (launch_repack_ginx2x)
hipError_t launch_repack_ginx2x(const void* bsk, uint32_t n, void* bskx, hipStream_t s);
// gw gates per workgroup: 1 (up to one gate per CU) or 2 (FHE_X_GATES)
hipError_t launch_blind_rotate_ginx2x(const GateArgs& g, const BootTables& t, const void* bskx, const uint16_t* idx,
                                      const uint32_t* tvb, uint32_t* ext_a, uint32_t* ext_b, int gw, hipStream_t s);
// K1x's range: Q < 2^27, N = 1024, ciphertext modulus <= 2N (gates, BootstrapFunc tables, the seam's accumulators)
bool ginx2x_supported(const GateArgs& g, const BootTables& t);
// K1q: four waves per gate (component x retained digit), one gate per 256-thread workgroup, K1x's keys and range:
// the latency kernel for batches of up to one gate per CU
hipError_t launch_blind_rotate_ginx4x(const GateArgs& g, const BootTables& t, const void* bskx, const uint16_t* idx,
                                      const uint32_t* tvb, uint32_t* ext_a, uint32_t* ext_b, hipStream_t s);
// The same split kernel with three retained digits per component (digitsG = 4 at N = 1024, Q < 2^27:
// STD128_3, STD128Q; with q = 2N: STD128_4, LPF_STD128, LPF_STD128Q) for the sets whose keys otherwise
// live on the 64-bit accumulator: keys in the g2_key_word layout (nd = 3), u64 ctExt into that
// path's workspace (launch_keyswitch_wide reads it)
hipError_t launch_blind_rotate_ginx3(const GateArgs& g, const BootTables& t, const void* bsk3, const uint16_t* idx,
                                     const uint32_t* tvb, uint64_t* ext_a, uint64_t* ext_b, hipStream_t s);
bool ginx3_supported(const GateArgs& g, const BootTables& t);
// LMKCDEY on the same split layout (k_blind_rotate_lmk3) for the digitsG = 4 LMKCDEY sets at N = 1024,
// Q < 2^27 (STD128_4_LMKCDEY, STD128Q_3_LMKCDEY, LPF_STD128Q_LMKCDEY): op lists of launch_prep_lmk,
// keys ek [n][c][p < 6][k4 < 4][64][4] (rows g2_row(c, p, 3)) and ak [numAutoKeys + 1][c][d < 3][k4][64][4]
// (Engine::pack_ginx3), u64 ctExt into the 64-bit path's workspace
hipError_t launch_blind_rotate_lmk3(const GateArgs& g, const BootTables& t, const void* ek, const void* ak,
                                    const uint16_t* ops, const uint32_t* nops, uint32_t maxops, const uint32_t* tvb,
                                    uint64_t* ext_a, uint64_t* ext_b, hipStream_t s);
// Its two-digit form (K1m, ND = 2) as the small-batch LMKCDEY kernel of the fast path (digitsG = 3, N = 1024,
// Q < 2^28: STD128_LMKCDEY, STD128_3_LMKCDEY, STD128Q_LMKCDEY, LPF_STD128_LMKCDEY, MEDIUM): keys repacked on the
// device from the resident layout (launch_repack_lmkx: n * 8192 + nauto * 4096 words), u32 ctExt, tables g.tv;
// gw gates per workgroup (1 or 2: k_blind_rotate_lmk3)
hipError_t launch_repack_lmkx(const void* bsk, uint32_t n, uint32_t nauto, void* bskx, hipStream_t s);
hipError_t launch_blind_rotate_lmkx(const GateArgs& g, const BootTables& t, const void* ekx, uint32_t n,
                                    const uint16_t* ops, const uint32_t* nops, uint32_t maxops, const uint32_t* tvb,
                                    uint32_t* ext_a, uint32_t* ext_b, int gw, hipStream_t s);
bool lmkx_supported(const GateArgs& g, const BootTables& t);
// K1m-4: four waves per gate (component x retained digit), one gate per 256-thread workgroup, the same keys
// (launch_repack_lmkx) and range: the LMKCDEY latency kernel for batches of up to one gate per CU
hipError_t launch_blind_rotate_lmk4x(const GateArgs& g, const BootTables& t, const void* ekx, uint32_t n,
                                     const uint16_t* ops, const uint32_t* nops, uint32_t maxops, const uint32_t* tvb,
                                     uint32_t* ext_a, uint32_t* ext_b, hipStream_t s);
// split-kernel key layout, per index i (8192 nd words): [c][p < 2 nd][k2 < 8][64 lanes][4 words]
// = (K+[r], K+[r+1], K-[r], K-[r+1]) of component c, digit row g2_row(c, p, nd), r = 2 k2, EVAL slot
// x(L, r) = ((r >> 2) << 8) | (L << 2) | (r & 3): wave c multiplies (own digits D_c, D_{2+c}, ..,
// partner digits D_{1-c}, D_{3-c}, ..) in that order
__host__ __device__ constexpr uint32_t g2_row(uint32_t c, uint32_t p, uint32_t nd) {
    return p < nd ? 2 * p + c : 2 * (p - nd) + 1 - c;
}
__host__ __device__ constexpr uint32_t g2_key_word(uint32_t nd, uint32_t c, uint32_t p, uint32_t k2, uint32_t L,
                                                   uint32_t e4) {
    return (((c * 2 * nd + p) * 8 + k2) * 64 + L) * 4 + e4;
}
// K1w: GINX at N = 2048, Q < 2^27, digitsG = 4, q < 2N (STD256Q) with the accumulator in registers
// (two waves per gate); keys in Engine::pack_n2k's layout, tables of Engine::build_tables_n2k (BootTables
// with 2048-word tabF / tabI and the 2113-pair half monomial table), u64 ctExt into the 64-bit path's
// workspace
hipError_t launch_blind_rotate_n2k(const GateArgs& g, const BootTables& t, const void* keys, const uint16_t* idx,
                                   const uint32_t* tvb, uint64_t* ext_a, uint64_t* ext_b, int nd, hipStream_t s);
bool n2k_supported(const GateArgs& g, const BootTables& t, int nd);
// K1w for LMKCDEY (k_blind_rotate_lmk2k<nd>): N = 2048, Q < 2^27, digitsG = nd + 1 = 4 or 5
// (STD256Q_3_LMKCDEY, STD256Q_4_LMKCDEY); op lists of launch_prep_lmk, keys in Engine::pack_n2k's
// LMKCDEY layout (ek per index, then ak per automorphism key), tables as launch_blind_rotate_n2k
hipError_t launch_blind_rotate_lmk2k(const GateArgs& g, const BootTables& t, const void* ek, const void* ak,
                                     const uint16_t* ops, const uint32_t* nops, uint32_t maxops, const uint32_t* tvb,
                                     uint64_t* ext_a, uint64_t* ext_b, int nd, hipStream_t s);
bool lmk2k_supported(const GateArgs& g, const BootTables& t, int nd);
// fused blind rotation (EvalAcc CGGI) + Transpose + iNTT + b fix-up + ModSwitch(Q -> qKS)
hipError_t launch_blind_rotate_ginx(const GateArgs& g, const BootTables& t, const void* bsk, const uint16_t* idx,
                                    const uint32_t* tvb, uint32_t* ext_a, uint32_t* ext_b, hipStream_t s);
// LMKCDEY: per-gate op schedule (EXT(i) / AUTO(t)), then the fused accumulator
hipError_t launch_prep_lmk(const GateArgs& g, const GateInputs& in, const int16_t* logGen,
                           uint16_t* ops, uint32_t* nops, uint32_t* tvb, uint32_t maxops, uint32_t numAutoKeys,
                           hipStream_t s);
// dm = true: the AP/DM accumulator (rgsw-acc-dm.cpp:62-77) -- an op list of external products only
hipError_t launch_blind_rotate_lmk(const GateArgs& g, const BootTables& t, const void* bsk, const void* autok,
                                   const uint16_t* ops, const uint32_t* nops, uint32_t maxops, const uint32_t* tvb,
                                   uint32_t* ext_a, uint32_t* ext_b, bool dm, hipStream_t s);
// AP/DM: per-gate op list EXT((i baseR + a0) digitsR + k) over the nonzero base-baseR digits a0 of
// (q - a_i) mod q (rgsw-acc-dm.cpp:62-77), + test-vector b
hipError_t launch_prep_dm(const GateArgs& g, const GateInputs& in, uint16_t* ops, uint32_t* nops, uint32_t* tvb,
                          uint32_t maxops, uint32_t baseR, uint32_t digitsR, hipStream_t s);
// ExternalProduct seam: raw RGSW keys [count][dG2 = 4][2][N] (EVAL, u64) -> the op-list kernel's
// resident layout (row_off, half-swapped rows, Montgomery with N^-1 folded in), key g at
// out + g * 4 * 2 * N words
hipError_t launch_pack_rgsw(const uint64_t* raw, size_t count, uint32_t N, uint32_t Q, uint32_t ninv_mont,
                            uint32_t* out, hipStream_t s);
// one op per item: ops[g * maxops] = g, nops[g] = 1 (ExternalProduct through the DM op loop)
hipError_t launch_single_ops(uint16_t* ops, uint32_t* nops, uint32_t count, uint32_t maxops, hipStream_t s);
// KeySwitch (lwe-pke.cpp:348-372) + ModSwitch(qKS -> q_out) (:254-261), KSK as u16 rows of 512;
// q_out = 0: no final switch (output mod qKS)
// part: optional scratch of part_words u32 for the row-split tiled kernel below 4096 gates (null:
// the per-gate kernel there)
hipError_t launch_keyswitch(const GateArgs& g, uint32_t baseKS, uint32_t digitsKS, const uint16_t* ksk,
                            const uint32_t* ms_a, const uint32_t* ms_b, uint64_t q_out, uint64_t* a_out,
                            uint64_t* b_out, hipStream_t s, uint32_t* part = nullptr, size_t part_words = 0);
// the row-split factor launch_keyswitch uses for count gates with that scratch
uint32_t keyswitch_split(size_t count, uint32_t n, uint32_t N, size_t part_words);
// the u32-sum form of the tiled kernel (u32 rows of ksk_width(n), any power-of-two qKS <= 2^32) for the
// (baseKS, digitsKS) shapes keyswitch_w32_shape accepts: (16, 5), (16, 6), (64, 3)
bool keyswitch_w32_shape(uint32_t baseKS, uint32_t digitsKS);
hipError_t launch_keyswitch_w32(const GateArgs& g, uint32_t baseKS, uint32_t digitsKS, const uint32_t* ksk,
                                const uint32_t* ms_a, const uint32_t* ms_b, uint64_t q_out, uint64_t* a_out,
                                uint64_t* b_out, hipStream_t s, uint32_t* part = nullptr, size_t part_words = 0);
// LWE element-wise operations on [count][len] / [count] u64 arrays (lwe.hip):
//   reduce: (a, b) mod m (LWECiphertextImpl::SetModulus, lwe-ciphertext.h:116-120)
//   sub:    x - y mod m, inputs < m (EvalSubEq / EvalSubEq2, lwe-pke.cpp:234-242); outputs may alias
//   addb:   b = (b + c) mod m, c < m (EvalAddConstEq / EvalSubConstEq as m - c, :230-246)
hipError_t launch_lwe_reduce(const uint64_t* a, const uint64_t* b, uint64_t* ao, uint64_t* bo, uint64_t m,
                             uint32_t len, size_t count, hipStream_t s);
hipError_t launch_lwe_sub(const uint64_t* xa, const uint64_t* xb, const uint64_t* ya, const uint64_t* yb, uint64_t* oa,
                          uint64_t* ob, uint64_t m, uint32_t len, size_t count, hipStream_t s);
hipError_t launch_lwe_addb(uint64_t* b, uint64_t c, uint64_t m, size_t count, hipStream_t s);
//   repeat: row i of [count][n] to rows i L .. i L + L - 1 of [count L][n] (EvalFuncMultiOutput's copies)
hipError_t launch_lwe_repeat(const uint64_t* a, const uint64_t* b, uint32_t n, size_t count, uint32_t L, uint64_t* ao,
                             uint64_t* bo, hipStream_t s);
// u64 [count][len] / [count] values below 2^32 -> u32 (the 64-bit path's ctExt mod qKS <= 2^16 into
// the 32-bit key switch's input, for the digitsG = 4 sets of launch_blind_rotate_ginx3)
hipError_t launch_narrow_u32(const uint64_t* a, const uint64_t* b, uint32_t* ao, uint32_t* bo, uint32_t len, size_t count,
                             hipStream_t s);
// u32 [count][len] / [count] -> u64 (the 32-bit path's ctExt out of the workspace)
hipError_t launch_widen_u64(const uint32_t* a, const uint32_t* b, uint64_t* ao, uint64_t* bo, uint32_t len, size_t count,
                            hipStream_t s);
// Ciphertexts mod Q as gate / bootstrap inputs (binfhe-base-scheme.cpp:92-93, 150-152, 200): SwitchCTtoqn
// (lwe-pke.cpp:170-178) of the rows of a column that are mod Q.  A column holds `count` ciphertexts as
// rows of `stride` u64 words (a) and count words (b); large[g] != 0 marks a ciphertext mod Q of dimension N,
// 0 one mod q of dimension n (its first n words); large == nullptr: every row is mod Q.
//   switch_in:  ModSwitch(Q -> qKS) (RoundqQ in IEEE double, lwe-pke.cpp:41-46, 254-261) of the flagged rows
//               into the key switch's input ext [count][N] (u32, or u64 when ext64) / [count]; other rows 0.
//               negate: EvalNOT at modulus Q first (binfhe-base-scheme.cpp:223-236; CMUX's NOT ct2, :180)
//   switch_out: after KeySwitch + ModSwitch(qKS -> q) of ext into (a_out, b_out) [count][n] / [count], the
//               unflagged rows copied in from the input (negated at q when negate); set_b: b_out of the
//               flagged rows = b_large instead (Bootstrap's test-vector offset, Engine::eval_mixed_device)
hipError_t launch_switch_in(const uint64_t* a, const uint64_t* b, uint32_t stride, const uint8_t* large, uint64_t Q,
                            uint64_t qKS, uint32_t N, size_t count, bool negate, void* ext_a, void* ext_b, bool ext64,
                            hipStream_t s);
hipError_t launch_switch_out(const uint64_t* a, const uint64_t* b, uint32_t stride, const uint8_t* large, uint32_t n,
                             uint64_t q, size_t count, bool negate, bool set_b, uint64_t b_large, uint64_t* a_out,
                             uint64_t* b_out, hipStream_t s);
// ModSwitch on u64 vectors (lwe-pke.cpp:41-46, 254-261)
hipError_t launch_modswitch(uint64_t q_from, uint64_t q_to, uint32_t len, uint32_t count, const uint64_t* a,
                            const uint64_t* b, uint64_t* a_out, uint64_t* b_out, hipStream_t s);

}  // namespace fhe_amd
