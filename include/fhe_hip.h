/*
 * fhe_hip.h -- C-ABI of the fhe_amd MI355X (gfx950) TFHE bootstrapping engine.
 *
 * Drop-in boundary for the reference's binfhe GPU-backend seam
 * lux::fhe::backend::Backend (src/binfhe/include/backend/backend.h:73-247 in
 * luxcpp/fhe) and for the gate path BinFHEContext::EvalBinGate
 * (src/binfhe/lib/binfhecontext.cpp:309-317) / EvalBinGateBatch
 * (src/binfhe/lib/batch/batch.cpp:176-210).  Plain pointers and sizes only.
 *
 * Conventions (mirroring the reference C API, include/lux/fhe/c_api.h:57-70):
 *   - every entry point returns 0 (FHE_HIP_OK) or a negative FHE_HIP_ERR_*;
 *     no C++ exception ever crosses this boundary (c_api.cpp:224-235);
 *   - the caller owns host buffers; a context owns its device copies;
 *   - host-buffer calls are synchronous; *_device calls are asynchronous on the
 *     given HIP stream (NULL = the context's own stream).  A context has one
 *     device workspace: a call on a different stream than the context's previous
 *     asynchronous call first waits for that call's work (an event recorded on its
 *     stream), so the calls on one context always execute in issue order;
 *   - a context is bound to one device and is not thread-safe: use one per
 *     host thread / device (BinFHEContext is likewise used per process).
 * Integers are the reference's u64 words (NativeInteger, NATIVEINT=64).
 */
#ifndef FHE_HIP_H
#define FHE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* error codes: same meanings as LuxFheError (c_api.h:57-70), plus device errors */
enum {
    FHE_HIP_OK = 0,
    FHE_HIP_ERR_NULL_PTR = -1,
    FHE_HIP_ERR_INVALID_PARAM = -2,
    FHE_HIP_ERR_ALLOC = -3,
    FHE_HIP_ERR_BOOTSTRAP = -7,
    FHE_HIP_ERR_GATE = -8,
    FHE_HIP_ERR_NOT_INIT = -11,
    FHE_HIP_ERR_DEVICE = -20
};

/* ------------------------------------------------------------------------ */
/* Batched negacyclic NTT (NativePoly::SwitchFormat,                         */
/*   src/core/include/lattice/hal/default/poly-impl.h:420-440;               */
/*   transformnat-impl.h:302-373 forward, :511-624 inverse).                 */
/* ------------------------------------------------------------------------ */
typedef struct fhe_hip_ntt_plan fhe_hip_ntt_plan;

/* N must be 1024; Q prime, Q = 1 mod 2N, Q < 2^62.  psi = 0 picks the
 * reference's root (minimal primitive 2N-th root, nbtheory-impl.h:183-228);
 * *psi_out (optional) receives the root used. */
int fhe_hip_ntt_plan_create(uint64_t Q, uint64_t psi, uint32_t N, int device, fhe_hip_ntt_plan** out,
                            uint64_t* psi_out);
void fhe_hip_ntt_plan_destroy(fhe_hip_ntt_plan* plan);
/* in-place on host memory: polys[count][N], canonical inputs (< Q).
 * inverse = 0: COEFFICIENT -> EVALUATION (bit-reversed); 1: back. */
int fhe_hip_ntt_batch(fhe_hip_ntt_plan* plan, uint64_t* polys, size_t count, int inverse);
/* device memory, asynchronous on `stream` (hipStream_t; NULL = plan stream);
 * d_in may equal d_out. */
int fhe_hip_ntt_batch_device(fhe_hip_ntt_plan* plan, const uint64_t* d_in, uint64_t* d_out, size_t count,
                             int inverse, void* stream);
/* the plan's stream (hipStream_t) */
void* fhe_hip_ntt_plan_stream(fhe_hip_ntt_plan* plan);

/* ------------------------------------------------------------------------ */
/* Gate bootstrapping context (one per device).                             */
/*   Replaces BinFHEContext::EvalBinGate / EvalBinGateBatch and the seam's   */
/*   BlindRotateBatch + KeySwitchBatch + ModSwitchBatch (backend.h:177-211). */
/* Parameter sets / methods / gates use the reference's enum values         */
/*   (src/binfhe/include/binfhe-constants.h:49-126):                         */
/*   paramset TOY=0, STD128=3, STD128_LMKCDEY=21; method GINX=2, LMKCDEY=3;   */
/*   gate OR=0 AND=1 NOR=2 NAND=3 XOR=4 XNOR=5 MAJORITY=6 AND3=7 OR3=8       */
/*   AND4=9 OR4=10 XOR_FAST=11 XNOR_FAST=12 CMUX=13.                        */
/* Raw key layouts (u64 words, the reference's values):                     */
/*   GINX bsk    [n][2 (s=+1, s=-1)][digitsG2][2][N]  EVAL (bit-reversed)   */
/*               = (*BSkey)[0][0..1][i] (rgsw-acc-cggi.cpp:39-57)           */
/*   LMKCDEY bsk [n][digitsG2][2][N] ++ [numAutoKeys+1][digitsG-1][2][N]    */
/*               = (*BSkey)[0][0][i] ++ (*BSkey)[0][1][k] (rgsw-acc-lmkcdey.cpp:39-68) */
/*   ksk A [N][baseKS][digitsKS][n], ksk B [N][baseKS][digitsKS]            */
/*               = LWESwitchingKeyImpl::GetElementsA/B (lwe-keyswitchkey.h:49) */
/* Ciphertexts: a[count][len], b[count] (len n for gate inputs/outputs).    */
/* ------------------------------------------------------------------------ */
typedef struct fhe_hip_ctx fhe_hip_ctx;

typedef struct {
    uint32_t paramset, method, n, N, q, baseKS, digitsKS, baseG, digitsG, numAutoKeys, keyDist;
    uint32_t kernel;  /* the accumulator kernels the set runs on: 1 = 32-bit, one wave per gate (N = 1024,
                         Q < 2^28, digitsG = 3); 2 = 32-bit split, two waves per gate (digitsG = 4, N = 1024,
                         Q < 2^27); 3 = the one-gate-per-workgroup accumulator with 32-bit residues
                         (Q < 2^30, digitsG2 Q < 2^32: the N = 2048 STD256 / STD256Q rows, TOY, ...);
                         4 = GINX gates at N = 2048, Q < 2^27, digitsG = 4, q < 2N (STD256Q) with the
                         accumulator in registers, two waves per gate (the rest as 3);
                         0 = the same accumulator with 64-bit residues (every other set, the
                         large-precision family) */
    uint64_t Q, psi, qKS, bsk_words, ksk_rows;  /* ksk_rows: of the raw layout (timeOptimization: 3 keys) */
} fhe_hip_params;
/* The large-precision family GenerateBinFHEContext(set, arbFunc, logQ, N, GINX, false)
 * (binfhecontext.cpp:55-104: Q = LastPrime(54, 2N), N = 2048, qKS = 2^35, n = 1305 (TOY: 32),
 * baseG 2^14 / 2^18 / 2^27 by logQ) is addressed by the paramset code
 *   FHE_HIP_LARGE | set << 16 | arbFunc << 15 | FHE_HIP_TIMEOPT? | log2(N) << 8 (0: minimum N) | logQ
 * in every entry point that takes a paramset.  FHE_HIP_TIMEOPT is timeOptimization = true: for
 * logQ != 11 the bootstrapping key is BTKeyGen's map (binfhecontext.cpp:285-307), one key per baseG
 * 2^14, 2^18, 2^27 concatenated in that order in the raw bsk (bsk_words covers the three), and
 * EvalSign / EvalDecomp switch keys as the modulus shrinks (binfhe-base-scheme.cpp:409-431, 498-514);
 * gates and the other operations use the key of the set's own baseG. */
#define FHE_HIP_LARGE (1 << 30)
#define FHE_HIP_TIMEOPT (1 << 14)

/* parameters of a set (host only; GenerateBinFHEContext, binfhecontext.cpp:107-179) */
int fhe_hip_params_get(int paramset, int method, fhe_hip_params* out);
int fhe_hip_create(int paramset, int method, int device, fhe_hip_ctx** out);
void fhe_hip_destroy(fhe_hip_ctx* ctx);
/* the context's parameters; its kernel field reports the kernels THIS context runs (the FHE_HIP_* kernel
 * settings it was created under), fhe_hip_params_get's the default for the set */
int fhe_hip_get_params(const fhe_hip_ctx* ctx, fhe_hip_params* out);
/* the blind-rotation kernel a 2-input gate batch of `count` ciphertexts runs on in this context (a static
 * string, e.g. "k_blind_rotate_ginx" / "k_blind_rotate_ginx2x": the rocprof kernel name) */
int fhe_hip_gate_kernel(const fhe_hip_ctx* ctx, size_t count, const char** name);
/* the context's stream (hipStream_t) */
void* fhe_hip_stream(fhe_hip_ctx* ctx);
/* upload keys (BTKeyLoad, binfhecontext.h:273-275; Backend::PackBootstrappingKey) */
int fhe_hip_load_bsk(fhe_hip_ctx* ctx, const uint64_t* bsk, size_t n_words);
int fhe_hip_load_ksk(fhe_hip_ctx* ctx, const uint64_t* A, size_t nA, const uint64_t* B, size_t nB);
/* The resident keys of src (same parameter set and method, any device) into dst: device-to-device copies of
 * the packed key buffers (xGMI peer copies between GPUs), no host repacking -- the per-device key fan-out of
 * fhe_hip_multi_load_keys */
int fhe_hip_copy_keys(fhe_hip_ctx* dst, const fhe_hip_ctx* src);
/* BTKeyGen on the context's device (BinFHEContext::BTKeyGen binfhecontext.cpp:185-200 -> KeyGenAcc
 * rgsw-acc-cggi.cpp:39-96 / rgsw-acc-dm.cpp:39-114 / rgsw-acc-lmkcdey.cpp:39-226, KeySwitchGen
 * lwe-pke.cpp:264-344): generates and loads the keys for sk[n] (mod qKS); bit-identical to
 * fhe_hip_keygen(..., seed, ...) for the sk it returns.  bsk / kskA / kskB (raw layouts, may be
 * NULL) receive a host copy. */
int fhe_hip_btkeygen_device(fhe_hip_ctx* ctx, const uint64_t* sk, size_t n, uint64_t seed, uint64_t* bsk,
                            uint64_t* kskA, uint64_t* kskB);
/* ---- the reference's packed transfer format (src/binfhe/include/backend/packed.h:29-307) ----
 * LWE batches byte-compatible with PackLWEBatch / UnpackLWEBatch (backend/packed.cpp:144-279):
 * 64-byte header ("LUXF", type LWE_BATCH = 2), u64 coefficients, sequential or INTERLEAVED (flag 1).
 * pack: out = NULL reports *size.  unpack: a/b = NULL report *n and *count. */
int fhe_hip_pack_lwe_batch(uint32_t n, size_t count, const uint64_t* a, const uint64_t* b, uint32_t flags,
                           uint8_t* out, size_t capacity, size_t* size);
int fhe_hip_unpack_lwe_batch(const uint8_t* data, size_t size, uint32_t* n, size_t* count, uint64_t* a, uint64_t* b);
/* ---- the reference's serialized objects: Serial::Serialize(obj, s, SerType::BINARY) streams
 * (utils/serial.h:95-125, cereal PortableBinary; binfhecontext-ser.h registrations) ----
 * RingGSWACCKey "refresh key" (cc.GetRefreshKey()) + LWESwitchingKey (cc.GetSwitchKey()): loaded
 * straight into the context (BTKeyLoad of deserialized keys, boolean-serial-binary.cpp flow). */
int fhe_hip_load_keys_cereal(fhe_hip_ctx* ctx, const uint8_t* refresh, size_t refresh_size, const uint8_t* sw,
                             size_t sw_size);
/* the same streams to / from the raw layouts (out = NULL reports the sizes) */
int fhe_hip_cereal_read_keys(int paramset, int method, const uint8_t* refresh, size_t refresh_size, const uint8_t* sw,
                             size_t sw_size, uint64_t* bsk, uint64_t* kskA, uint64_t* kskB);
int fhe_hip_cereal_write_keys(int paramset, int method, const uint64_t* bsk, size_t bsk_words, const uint64_t* kskA,
                              const uint64_t* kskB, uint8_t* refresh_out, size_t refresh_cap, size_t* refresh_size,
                              uint8_t* sw_out, size_t sw_cap, size_t* sw_size);
/* LWECiphertext (is_key = 0: a[n], b, modulus) or LWEPrivateKey (is_key = 1: s[n], modulus);
 * read with a = NULL reports *n */
int fhe_hip_cereal_read_lwe(const uint8_t* data, size_t size, int is_key, uint64_t* a, uint32_t cap_n, uint32_t* n,
                            uint64_t* b, uint64_t* mod);
int fhe_hip_cereal_write_lwe(const uint64_t* a, uint32_t n, uint64_t b, uint64_t mod, int is_key, uint8_t* out,
                             size_t cap, size_t* size);
/* The key-independent cryptoContext archive Serial::Serialize(BinFHEContext, BINARY) (boolean-serial-binary.cpp:
 * 65-71 writes it, :108 reads it back): BinFHEContext -> BinFHECryptoParams -> LWECryptoParams,
 * RingGSWCryptoParams (binfhecontext-ser.h:43,49,52-53).  read: the GenerateBinFHEContext(set, method) row
 * whose parameters the archive holds (the archive names none; FHE_HIP_ERR_INVALID_PARAM if no supported row
 * matches), with its parameters (out may be NULL).  write: the reference's bytes for a row (out = NULL
 * reports *size).  create_from_cereal: fhe_hip_create on the row a cryptoContext archive describes. */
int fhe_hip_cereal_read_context(const uint8_t* data, size_t size, int* paramset, int* method, fhe_hip_params* out);
int fhe_hip_cereal_write_context(int paramset, int method, uint8_t* out, size_t cap, size_t* size);
int fhe_hip_create_from_cereal(const uint8_t* data, size_t size, int device, fhe_hip_ctx** out);
/* EvalBinGate on two packed batches, result packed with out_flags (out = NULL reports *size) */
int fhe_hip_eval_bingate_packed(fhe_hip_ctx* ctx, int gate, const uint8_t* in1, size_t size1, const uint8_t* in2,
                                size_t size2, uint32_t out_flags, uint8_t* out, size_t capacity, size_t* size);
/* Packed keys: PackedBootstrappingKey (type 5) / PackedSwitchingKey (type 6) headers of
 * backend/packed.h (the reference's packers are TODO stubs, packed.cpp:284-328) followed by the
 * raw u64 layouts above; header.flags of the BSK = BINFHE_METHOD.  NULL outputs report sizes. */
int fhe_hip_pack_keys(int paramset, int method, const uint64_t* bsk, size_t bsk_words, const uint64_t* A,
                      const uint64_t* B, uint8_t* bsk_out, size_t bsk_cap, size_t* bsk_size, uint8_t* ksk_out,
                      size_t ksk_cap, size_t* ksk_size);
int fhe_hip_load_keys_packed(fhe_hip_ctx* ctx, const uint8_t* bsk, size_t bsk_size, const uint8_t* ksk,
                             size_t ksk_size);

/* EvalBinGate over count independent pairs (binfhe-base-scheme.cpp:76-126).
 * Inputs mod q, dimension n; outputs likewise.  ct1 and ct2 must not alias
 * (the reference's ct1 == ct2 check, :85-86, becomes a documented precondition). */
int fhe_hip_eval_bingate_batch(fhe_hip_ctx* ctx, int gate, size_t count, const uint64_t* a1, const uint64_t* b1,
                               const uint64_t* a2, const uint64_t* b2, uint64_t* a_out, uint64_t* b_out);
/* same on device buffers, asynchronous on stream (NULL = context stream) */
int fhe_hip_eval_bingate_batch_device(fhe_hip_ctx* ctx, int gate, size_t count, const uint64_t* d_a1,
                                      const uint64_t* d_b1, const uint64_t* d_a2, const uint64_t* d_b2,
                                      uint64_t* d_a_out, uint64_t* d_b_out, void* stream);
/* The two stages of fhe_hip_eval_bingate_batch_device, separately launchable:
 * blind_rotate leaves the mod-switched ctExt (N+1 values mod qKS per gate) in
 * the context's workspace; keyswitch consumes it (count must not exceed the
 * count of the last blind rotation: FHE_HIP_ERR_INVALID_PARAM otherwise). */
int fhe_hip_blind_rotate_batch_device(fhe_hip_ctx* ctx, int gate, size_t count, const uint64_t* d_a1,
                                      const uint64_t* d_b1, const uint64_t* d_a2, const uint64_t* d_b2, void* stream);
int fhe_hip_keyswitch_workspace_device(fhe_hip_ctx* ctx, size_t count, uint64_t* d_a_out, uint64_t* d_b_out,
                                       void* stream);
/* EvalBinGate(..., extended = true): ctExt before SwitchCTtoqn, dimension N, mod Q */
int fhe_hip_eval_bingate_extended(fhe_hip_ctx* ctx, int gate, size_t count, const uint64_t* a1, const uint64_t* b1,
                                  const uint64_t* a2, const uint64_t* b2, uint64_t* ext_a, uint64_t* ext_b);
/* EvalBinGate(gate, ctvector, extended) for gate in {MAJORITY, AND3, OR3, AND4, OR4}
 * (binfhe-base-scheme.cpp:129-171): k (2..4) inputs a_in[j] [count][n], b_in[j] [count]
 * mod q, summed; ptmod = the inputs' plaintext modulus (GetptModulus of ctvector[0]:
 * 6 for AND3/OR3, 8 for AND4/OR4, 4 for MAJORITY in the reference's tests).
 * extended = 0: outputs [count][n] mod q; extended = 1: ctExt [count][N] mod Q. */
int fhe_hip_eval_gate_multi_batch(fhe_hip_ctx* ctx, int gate, uint32_t k, uint32_t ptmod, size_t count,
                                  const uint64_t* const* a_in, const uint64_t* const* b_in, uint64_t* a_out,
                                  uint64_t* b_out, int extended);
int fhe_hip_eval_gate_multi_batch_device(fhe_hip_ctx* ctx, int gate, uint32_t k, uint32_t ptmod, size_t count,
                                         const uint64_t* const* d_a_in, const uint64_t* const* d_b_in,
                                         uint64_t* d_a_out, uint64_t* d_b_out, void* stream);
/* BinFHEContext::Bootstrap (binfhecontext.cpp; BinFHEScheme::Bootstrap, binfhe-base-scheme.cpp:190-218):
 * BootstrapGateCore(AND, ct + q/4), extraction (b = Q/8 + 1 + acc1[0]) and SwitchCTtoqn -- the refresh of
 * lux_fhe_bootstrap (c_api.cpp:263-276).  Ciphertexts a[count][n], b[count] mod q, plaintext modulus 4. */
int fhe_hip_bootstrap_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b, uint64_t* a_out,
                            uint64_t* b_out);
int fhe_hip_bootstrap_batch_device(fhe_hip_ctx* ctx, size_t count, const uint64_t* d_a, const uint64_t* d_b,
                                   uint64_t* d_a_out, uint64_t* d_b_out, void* stream);
/* EvalBinGate(CMUX, {ct0, ct1, ct2}) = NAND(NAND(ct0, NOT ct2), NAND(ct1, ct2)), i.e. ct2 ? ct1 : ct0
 * (binfhe-base-scheme.cpp:172-182; EvalCMUXBatch, batch.cpp:212-249, passes {sel, true, false}). */
int fhe_hip_eval_cmux_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a0, const uint64_t* b0,
                            const uint64_t* a1, const uint64_t* b1, const uint64_t* a2, const uint64_t* b2,
                            uint64_t* a_out, uint64_t* b_out);
int fhe_hip_eval_cmux_batch_device(fhe_hip_ctx* ctx, size_t count, const uint64_t* d_a0, const uint64_t* d_b0,
                                   const uint64_t* d_a1, const uint64_t* d_b1, const uint64_t* d_a2,
                                   const uint64_t* d_b2, uint64_t* d_a_out, uint64_t* d_b_out, void* stream);
/* ---- ciphertexts mod Q (extended outputs, LARGE_DIM encryptions) as inputs ----
 * BinFHEScheme::EvalBinGate / EvalBinGate(ctvector) / Bootstrap switch every input whose modulus is Q
 * to (n, q) first (binfhe-base-scheme.cpp:92-93, 150-152, 200: SwitchCTtoqn), and inputs of either
 * modulus may be mixed within one call.
 * SwitchCTtoqn (lwe-pke.cpp:170-178; BinFHEContext::SwitchCTtoqn, binfhecontext.cpp:254-264):
 *   a[count][N], b[count] mod Q -> a_out[count][n], b_out[count] mod q. */
int fhe_hip_switch_to_qn_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b, uint64_t* a_out,
                               uint64_t* b_out);
int fhe_hip_switch_to_qn_batch_device(fhe_hip_ctx* ctx, size_t count, const uint64_t* d_a, const uint64_t* d_b,
                                      uint64_t* d_a_out, uint64_t* d_b_out, void* stream);
/* op: OR..XNOR / XOR_FAST / XNOR_FAST (k = 2; EvalBinGate(gate, ct1, ct2, extended), :76-126),
 * MAJORITY / AND3 / OR3 / AND4 / OR4 (k = 2..4, inputs' plaintext modulus ptmod; :129-175), CMUX (k = 3,
 * {ct0, ct1, ct2} -> ct2 ? ct1 : ct0, extended ignored as the reference ignores it, :176-182), or
 * FHE_HIP_OP_BOOTSTRAP (k = 1, Bootstrap(ct, extended), :190-220, the input's plaintext modulus ptmod).
 * Column j: count ciphertexts a_in[j], b_in[j]; large == NULL or large[j] == NULL: rows of n words, all mod q;
 * otherwise rows of N words, large[j][g] = 1 marking a ciphertext mod Q (dimension N), 0 one mod q (its first
 * n words used).  Outputs [count][n] mod q, or ctExt [count][N] mod Q when extended.
 * Bootstrap of an input mod Q keeps the reference's constant ct->GetModulus() >> 2 (:201), added at q by
 * ModAddFast, so its test vector is the window's constant uv.  That shortcut needs
 * Q / 4 >= 2.5 q, true for every parameter row (the smallest ratio is far above it); a set below it is refused
 * with FHE_HIP_ERR_INVALID_PARAM rather than computed differently from the reference. */
#define FHE_HIP_OP_BOOTSTRAP (-1)
int fhe_hip_eval_mixed_batch(fhe_hip_ctx* ctx, int op, uint32_t k, uint32_t ptmod, size_t count,
                             const uint64_t* const* a_in, const uint64_t* const* b_in, const uint8_t* const* large,
                             uint64_t* a_out, uint64_t* b_out, int extended);
/* device buffers (large[j] device arrays too), asynchronous on stream */
int fhe_hip_eval_mixed_batch_device(fhe_hip_ctx* ctx, int op, uint32_t k, uint32_t ptmod, size_t count,
                                    const uint64_t* const* d_a_in, const uint64_t* const* d_b_in,
                                    const uint8_t* const* d_large, uint64_t* d_a_out, uint64_t* d_b_out, int extended,
                                    void* stream);

/* ---- functional bootstrapping (binfhe-base-scheme.cpp:241-521, 589-648) ----
 * Batches of `count` LWE ciphertexts a[count][n], b[count] under the context's keys; beta = 128
 * (BinFHEContext::GetBeta).  Moduli are powers of two.
 * EvalFunc (binfhecontext.cpp:340-344): inputs/outputs mod q_in; lut[lut_len = q_in] as from
 *   GenerateLUTviaFunction; negacyclic / periodic / arbitrary LUTs as checkInputFunction
 *   classifies them (arbitrary needs q_in <= N). */
int fhe_hip_eval_func_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b, uint64_t q_in,
                            const uint64_t* lut, size_t lut_len, uint64_t* a_out, uint64_t* b_out);
int fhe_hip_eval_func_batch_device(fhe_hip_ctx* ctx, size_t count, const uint64_t* d_a, const uint64_t* d_b,
                                   uint64_t q_in, const uint64_t* lut, size_t lut_len, uint64_t* d_a_out,
                                   uint64_t* d_b_out, void* stream);
/* EvalFuncMultiOutputBatch (batch.cpp:141-174): EvalFunc(ct_i, luts[j]) for every input i and each of num_luts
 * LUTs luts[num_luts][lut_len = q_in]; output j of input i at row i * num_luts + j of a_out [count * num_luts][n],
 * b_out [count * num_luts].  The LUT-independent first bootstrap of EvalFunc's periodic / arbitrary forms runs
 * once per input and class; the LUT-dependent last bootstraps of a class run as one launch. */
int fhe_hip_eval_func_multi_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b, uint64_t q_in,
                                  const uint64_t* luts, size_t lut_len, uint32_t num_luts, uint64_t* a_out,
                                  uint64_t* b_out);
int fhe_hip_eval_func_multi_batch_device(fhe_hip_ctx* ctx, size_t count, const uint64_t* d_a, const uint64_t* d_b,
                                         uint64_t q_in, const uint64_t* luts, size_t lut_len, uint32_t num_luts,
                                         uint64_t* d_a_out, uint64_t* d_b_out, void* stream);
/* EvalFloor (binfhecontext.cpp:346-357): inputs/outputs mod `mod` (<= 2^31) */
int fhe_hip_eval_floor_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod,
                             uint32_t roundbits, uint64_t* a_out, uint64_t* b_out);
/* EvalSign (binfhecontext.cpp:359-364): inputs mod `mod` (q < mod <= 2^31), outputs mod q */
int fhe_hip_eval_sign_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod,
                            int scheme_switch, uint64_t* a_out, uint64_t* b_out);
/* EvalDecomp (binfhecontext.cpp:366-370): *parts ciphertexts per input; a_out [parts][count][n],
 * b_out [parts][count]; parts - 1 of them mod q, the last one mod its own reduced modulus */
int fhe_hip_eval_decomp_parts(fhe_hip_ctx* ctx, uint64_t mod, uint32_t* parts);
int fhe_hip_eval_decomp_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod,
                              uint64_t* a_out, uint64_t* b_out);
/* BootstrapFunc (binfhe-base-scheme.cpp:617-642): a mod ctmod (<= 2N), f[ctmod] with f(x) <= fmod,
 * outputs mod fmod (<= 2^40) */
int fhe_hip_bootstrap_func_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b,
                                 uint32_t ctmod, const uint64_t* f, uint64_t fmod, uint64_t* a_out, uint64_t* b_out);

/* ---- the reference GPU seam lux::fhe::backend::Backend (src/binfhe/include/backend/backend.h) ----
 * Backend::BlindRotate / BlindRotateBatch (backend.h:131-136, 177-182) = the accumulator's EvalAcc
 * (rgsw-acc-cggi.cpp:59-68, rgsw-acc-lmkcdey.cpp:70-158, rgsw-acc-dm.cpp:62-77) on `count` pairs:
 * a[count][n] mod ctmod (the LWE ciphertext's modulus: a power of two <= 2N; 2N for LMKCDEY, q for
 * AP), acc[count][2][N] in/out (RLWECiphertext elements 0 and 1, EVALUATION, bit-reversed as the
 * reference stores them, canonical mod Q).  Every parameter set and method of the context. */
int fhe_hip_blind_rotate_acc_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, uint64_t ctmod, uint64_t* acc);
int fhe_hip_blind_rotate_acc_batch_device(fhe_hip_ctx* ctx, size_t count, const uint64_t* d_a, uint64_t ctmod,
                                          uint64_t* d_acc, void* stream);
/* BlindRotateBatch with null accumulators -- what BootstrapBatch (batch/batch.cpp:53-104) passes
 * ("initialize accumulators with LUT (identity for bootstrap)", :77-86): the accumulator of
 * BinFHEScheme::Bootstrap (binfhe-base-scheme.cpp:190-205), i.e. BootstrapGateCore(AND, ct + q/4)
 * (:525-583): the AND window's test vector at b + q/4, NTT'd, then EvalAcc over a.  Ciphertexts
 * a[count][n], b[count] mod q; acc[count][2][N] out (EVALUATION, canonical mod Q). */
int fhe_hip_blind_rotate_init_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b,
                                    uint64_t* acc);
int fhe_hip_blind_rotate_init_batch_device(fhe_hip_ctx* ctx, size_t count, const uint64_t* d_a, const uint64_t* d_b,
                                           uint64_t* d_acc, void* stream);
/* Backend::ExternalProduct / ExternalProductBatch (backend.h:141-146, 187-192): RGSW x RLWE -> RLWE,
 * result[g] = sum_d D_d(rlwe[g]) * rgsw[g][d] with D = SignedDigitDecompose (rgsw-acc.cpp:54-91) --
 * AddToAccLMKCDEY / AddToAccDM (rgsw-acc-lmkcdey.cpp:228-254, rgsw-acc-dm.cpp:119-145) under the
 * context's baseG.  rgsw[count][digitsG2][2][N] (RingGSWEvalKeyImpl rows, EVALUATION), rlwe and
 * result [count][2][N] (EVALUATION), canonical mod Q; result may equal rlwe. */
int fhe_hip_external_product_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* rgsw, const uint64_t* rlwe,
                                   uint64_t* result);
int fhe_hip_external_product_batch_device(fhe_hip_ctx* ctx, size_t count, const uint64_t* d_rgsw,
                                          const uint64_t* d_rlwe, uint64_t* d_result, void* stream);
/* Backend::MaxBatchSize (backend.h:86): gates one call can take given the device's free memory */
int fhe_hip_max_batch_size(fhe_hip_ctx* ctx, size_t* max_count);
/* Backend::UnpackBootstrappingKey (backend.h:229-233): packed keys (fhe_hip_pack_keys) back to the
 * raw layouts; either key may be skipped (NULL); *_cap = the output buffers' sizes in u64 words
 * (FHE_HIP_ERR_INVALID_PARAM when too small) */
int fhe_hip_unpack_keys(int paramset, int method, const uint8_t* bsk_packed, size_t bsk_size, uint64_t* bsk,
                        size_t bsk_cap, const uint8_t* ksk_packed, size_t ksk_size, uint64_t* kskA, size_t kskA_cap,
                        uint64_t* kskB, size_t kskB_cap);

/* LWEEncryptionScheme::KeySwitch (lwe-pke.cpp:348-372): (N, qKS) -> (n, qKS) */
int fhe_hip_keyswitch_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b, uint64_t* a_out,
                            uint64_t* b_out);
/* LWEEncryptionScheme::ModSwitch (lwe-pke.cpp:254-261): RoundqQ in IEEE double exactly as the
 * reference evaluates it (lwe-pke.cpp:41-46), for any nonzero moduli */
int fhe_hip_modswitch_batch(fhe_hip_ctx* ctx, uint64_t q_from, uint64_t q_to, uint32_t len, size_t count,
                            const uint64_t* a, const uint64_t* b, uint64_t* a_out, uint64_t* b_out);

/* Single-process multi-device: one host thread + stream per device,
 * contiguous shards, keys replicated on every device, no collectives.
 * devices may repeat (several contexts on one GPU). */
typedef struct fhe_hip_multi fhe_hip_multi;
int fhe_hip_multi_create(int paramset, int method, const int* devices, int ndev, fhe_hip_multi** out);
void fhe_hip_multi_destroy(fhe_hip_multi* m);
int fhe_hip_multi_load_keys(fhe_hip_multi* m, const uint64_t* bsk, size_t n_words, const uint64_t* A, size_t nA,
                            const uint64_t* B, size_t nB);
int fhe_hip_multi_eval_bingate_batch(fhe_hip_multi* m, int gate, size_t count, const uint64_t* a1, const uint64_t* b1,
                                     const uint64_t* a2, const uint64_t* b2, uint64_t* a_out, uint64_t* b_out);

/* ------------------------------------------------------------------------ */
/* Deterministic host key material (KeyGen / BTKeyGen / Encrypt / Decrypt,   */
/*   binfhecontext.cpp:185-307) -- seeded, same structure as the reference. */
/* ------------------------------------------------------------------------ */
/* KeyGen (binfhecontext.cpp:185-190): sk[n] (mod qKS) only */
int fhe_hip_keygen_secret(int paramset, int method, uint64_t seed, uint64_t* sk);
/* sk[n] (mod qKS), bsk[bsk_words], kskA[ksk_rows*n], kskB[ksk_rows] */
int fhe_hip_keygen(int paramset, int method, uint64_t seed, uint64_t* sk, uint64_t* bsk, uint64_t* kskA,
                   uint64_t* kskB);
/* a[count][n], b[count] mod q, plaintext modulus 4 */
int fhe_hip_encrypt(int paramset, int method, const uint64_t* sk, const int* bits, size_t count, uint64_t seed,
                    uint64_t* a, uint64_t* b);
int fhe_hip_decrypt(int paramset, int method, const uint64_t* sk, const uint64_t* a, const uint64_t* b, size_t count,
                    uint32_t len, uint64_t mod, int64_t* out);
/* the same with an explicit plaintext modulus (Encrypt/Decrypt(..., p), lwe-pke.cpp:103-128, 181-226) */
int fhe_hip_encrypt_ptmod(int paramset, int method, const uint64_t* sk, const int* bits, size_t count, uint64_t seed,
                          uint32_t ptmod, uint64_t* a, uint64_t* b);
/* ... and an explicit ciphertext modulus mod (Encrypt(sk, m, SMALL_DIM, p, mod), binfhecontext.cpp:220-234) */
int fhe_hip_encrypt_mod(int paramset, int method, const uint64_t* sk, const int* bits, size_t count, uint64_t seed,
                        uint32_t ptmod, uint64_t mod, uint64_t* a, uint64_t* b);
int fhe_hip_decrypt_ptmod(int paramset, int method, const uint64_t* sk, const uint64_t* a, const uint64_t* b,
                          size_t count, uint32_t len, uint64_t mod, uint32_t ptmod, int64_t* out);
/* The RLWE secret skN[N] of fhe_hip_keygen(..., seed, ...) (KeyGenN's key, binfhecontext.cpp:203-208), stored
 * mod qKS as the key switch holds it (lwe-pke.cpp:285-286): the LWE secret of dimension-N ciphertexts mod Q.
 * fhe_hip_decrypt_ptmod with len = N, mod = Q decrypts them under it. */
int fhe_hip_keygen_ring_secret(int paramset, int method, uint64_t seed, uint64_t* skN);
/* Encrypt(pk, m, LARGE_DIM, p) (binfhecontext.cpp:236-252, EncryptN): a[count][N], b[count] mod Q under skN
 * (a symmetric encryption under the key the public key belongs to; uniform a, the reference's Gaussian) */
int fhe_hip_encrypt_large(int paramset, int method, const uint64_t* skN, const int* bits, size_t count, uint64_t seed,
                          uint32_t ptmod, uint64_t* a, uint64_t* b);

/* ------------------------------------------------------------------------ */
/* Device memory (Backend::Allocate/Free/CopyToDevice/CopyToHost/Synchronize, */
/*   backend.h:94-114)                                                       */
/* ------------------------------------------------------------------------ */
int fhe_hip_alloc(int device, size_t bytes, void** d_ptr);
int fhe_hip_free(void* d_ptr);
int fhe_hip_copy_to_device(void* d_dst, const void* h_src, size_t bytes);
int fhe_hip_copy_to_host(void* h_dst, const void* d_src, size_t bytes);
int fhe_hip_synchronize(int device);
int fhe_hip_device_count(int* count);
/* Backend::DeviceMemory (backend.h:87): free / total bytes of the device (either may be NULL) */
int fhe_hip_device_memory(int device, size_t* free_bytes, size_t* total_bytes);
/* message of the last error on this host thread */
const char* fhe_hip_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* FHE_HIP_H */
