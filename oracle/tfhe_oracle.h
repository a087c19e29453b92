/*
 * tfhe_oracle.h -- CPU restatement of the reference's TFHE gate-bootstrap path
 * (luxcpp/fhe = OpenFHE 1.4.2 fork), in plain C.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this (as libtfhe_oracle.so), and only as the checker
 * or the CPU baseline.  The fhe_amd product never links or calls it.
 *
 * Parity pinning: every function here is checked bit-for-bit against the
 * reference itself, compiled from /root/reference into oracle/_ref/libfhe_ref.so
 * (oracle/Makefile + oracle/ref_driver.cpp), by tests/test_oracle_vs_reference.py,
 * and against the golden vectors in tests/golden/ that script produced.
 *
 * Raw layouts (u64 words, polynomials of N coefficients; EVALUATION-domain
 * polynomials in the reference's bit-reversed order):
 *   GINX    bsk : [n][2 (s=+1,s=-1)][digitsG2][2][N]      rgsw-acc-cggi.cpp:39-57
 *   AP bsk      : [n][baseR][digitsR][digitsG2][2][N]  (j = 0 slots unused)  rgsw-acc-dm.cpp:39-58
 *   LMKCDEY bsk : [n][digitsG2][2][N] ++ [numAutoKeys+1][digitsG-1][2][N]
 *                                                          rgsw-acc-lmkcdey.cpp:39-68
 *   ksk A : [N][baseKS][digitsKS][n],  ksk B : [N][baseKS][digitsKS]
 *                                                          lwe-pke.cpp:264-344
 *   LWE ciphertexts: a[count][len], b[count]
 */
#ifndef TFHE_ORACLE_H
#define TFHE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* reference enum values (src/binfhe/include/binfhe-constants.h:49-126) */
enum { TFO_TOY = 0, TFO_STD128_AP = 2, TFO_STD128 = 3, TFO_STD128_LMKCDEY = 21 };
enum { TFO_AP = 1, TFO_GINX = 2, TFO_LMKCDEY = 3 };

typedef struct {
    uint32_t n, N, q, qKS, baseKS, digitsKS, baseG, gBits, digitsG, numAutoKeys, method, paramset;
    uint32_t baseR, digitsR;  /* AP/DM refresh decomposition of a_i (rgsw-cryptoparameters.cpp:37-46) */
    uint64_t Q, psi;
} tfo_params;

/* LastPrime (src/core/include/math/nbtheory-impl.h:350-371) */
uint64_t tfo_last_prime(uint32_t bits, uint64_t m);
/* RootOfUnity: minimal primitive m-th root of unity (nbtheory-impl.h:183-228) */
uint64_t tfo_root_of_unity(uint64_t m, uint64_t Q);
/* GenerateBinFHEContext parameter rows (src/binfhe/lib/binfhecontext.cpp:113-179) */
int tfo_params_init(int paramset, int method, tfo_params* p);

/* Merged negacyclic NTT/iNTT, bit-reversed twiddles
 * (src/core/include/math/hal/intnat/transformnat-impl.h:302-373, 511-624, 777-831).
 * inverse=0: COEFFICIENT -> EVALUATION (bit-reversed); inverse=1: back. */
int tfo_ntt_batch(uint64_t* polys, size_t count, uint32_t N, uint64_t Q, uint64_t psi, int inverse, int nthreads);

/* EvalBinGate on `count` gate pairs (src/binfhe/lib/binfhe-base-scheme.cpp:76-126).
 * stage = 0: final output (n, q).  stage = 1: ctExt (N, Q) (extended=true).
 * Output a_out[count][stage ? N : n], b_out[count]. */
int tfo_eval_gate_batch(const tfo_params* p, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB,
                        int gate, size_t count, const uint64_t* a1, const uint64_t* b1, const uint64_t* a2,
                        const uint64_t* b2, uint64_t* a_out, uint64_t* b_out, int stage, int nthreads);

/* EvalBinGate(gate, ctvector) for MAJORITY=6/AND3=7/OR3=8/AND4=9/OR4=10 (binfhe-base-scheme.cpp:129-171):
 * k inputs a_in[j][count][n], b_in[j][count] summed mod q; ptmod = their plaintext modulus. */
int tfo_eval_gate_multi_batch(const tfo_params* p, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB,
                              int gate, uint32_t k, uint32_t ptmod, size_t count, const uint64_t* const* a_in,
                              const uint64_t* const* b_in, uint64_t* a_out, uint64_t* b_out, int stage, int nthreads);
/* EvalBinGate(CMUX, {ct0, ct1, ct2}) (binfhe-base-scheme.cpp:172-182) */
int tfo_eval_cmux_batch(const tfo_params* p, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB,
                        size_t count, const uint64_t* a0, const uint64_t* b0, const uint64_t* a1, const uint64_t* b1,
                        const uint64_t* a2, const uint64_t* b2, uint64_t* a_out, uint64_t* b_out, int nthreads);

/* Functional bootstrapping (binfhe-base-scheme.cpp:241-521, 589-648).
 * BootstrapFunc: a [count][n] mod ctmod (power of 2, <= 2N), test vector tv[x] = (Q/fmod) f(x) for
 * x < ctmod, output [count][n] mod fmod. */
int tfo_bootstrap_func_batch(const tfo_params* p, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB,
                             size_t count, const uint64_t* a, const uint64_t* b, uint64_t ctmod, const uint64_t* tv,
                             uint64_t fmod, uint64_t* a_out, uint64_t* b_out, int nthreads);
/* EvalFunc: inputs and outputs mod q_in, lut[q_in] */
int tfo_eval_func_batch(const tfo_params* p, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB,
                        size_t count, const uint64_t* a, const uint64_t* b, uint64_t q_in, const uint64_t* lut,
                        uint64_t* a_out, uint64_t* b_out, int nthreads);
/* EvalFloor: inputs and outputs mod `mod` */
int tfo_eval_floor_batch(const tfo_params* p, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB,
                         size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod, uint32_t roundbits,
                         uint64_t* a_out, uint64_t* b_out, int nthreads);
/* EvalSign: inputs mod `mod` > q, outputs mod q */
int tfo_eval_sign_batch(const tfo_params* p, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB,
                        size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod, int scheme_switch,
                        uint64_t* a_out, uint64_t* b_out, int nthreads);
/* EvalDecomp: a_out [parts][count][n], b_out [parts][count] */
uint32_t tfo_eval_decomp_parts(const tfo_params* p, uint64_t mod);
int tfo_eval_decomp_batch(const tfo_params* p, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB,
                          size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod, uint64_t* a_out,
                          uint64_t* b_out, int nthreads);

/* LWEEncryptionScheme::ModSwitch (lwe-pke.cpp:41-46, 254-261) */
void tfo_modswitch(uint64_t q_from, uint64_t q_to, uint32_t len, size_t count, const uint64_t* a, const uint64_t* b,
                   uint64_t* a_out, uint64_t* b_out);
/* LWEEncryptionScheme::KeySwitch (lwe-pke.cpp:348-372): (N, qKS) -> (n, qKS) */
void tfo_keyswitch(const tfo_params* p, const uint64_t* kskA, const uint64_t* kskB, size_t count, const uint64_t* a,
                   const uint64_t* b, uint64_t* a_out, uint64_t* b_out);
/* LWEEncryptionScheme::Decrypt (lwe-pke.cpp:181-226) with p = 4; sk stored mod qKS */
int64_t tfo_decrypt(const uint64_t* sk, uint64_t skmod, const uint64_t* a, uint64_t b, uint32_t len, uint64_t mod);
/* the same with plaintext modulus ptmod */
int64_t tfo_decrypt_p(const uint64_t* sk, uint64_t skmod, const uint64_t* a, uint64_t b, uint32_t len, uint64_t mod,
                      uint32_t ptmod);

#ifdef __cplusplus
}
#endif
#endif
