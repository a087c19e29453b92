// engine.h -- one MI355X device context for the gate-bootstrap path.
//
// Mirrors the reference's backend seam (src/binfhe/include/backend/backend.h:73-247):
// key packing (PackBootstrappingKey), BlindRotateBatch + KeySwitchBatch +
// ModSwitchBatch fused into one EvalBinGateBatch launch sequence.  Keys are
// uploaded once and stay resident in HBM in kernel-native layouts:
//   BSK : u32 Montgomery form, grouped per accumulator iteration, slot order
//         matching the kernel's register ownership (one 512 B coalesced load per
//         wave-instruction);  GINX 32.9 MB, LMKCDEY 14.8 MB.
//   KSK : u16 rows of 512 (A row + B), 100.7 MB (qKS = 2^14).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "boot.h"
#include "boot_wide.h"
#include "params.h"

namespace fhe_amd {

struct HipError : std::runtime_error {
    hipError_t code;
    HipError(hipError_t e, const std::string& what)
        : std::runtime_error(what + ": " + hipGetErrorString(e)), code(e) {}
};
#define FHE_HIP_CHECK(expr)                                   \
    do {                                                      \
        hipError_t _e = (expr);                               \
        if (_e != hipSuccess) throw HipError(_e, #expr);      \
    } while (0)

class Engine {
public:
    Engine(int paramset, int method, int device);
    ~Engine();
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;

    const Params& params() const { return p_; }
    int device() const { return device_; }
    hipStream_t stream() const { return stream_; }
    // The stream a call runs on (nullptr: the context's own).  All calls share one workspace, so
    // a call on a different stream than the previous call first waits for that stream's work.
    // (end_call records the point a later call on another stream waits for).
    hipStream_t use_stream(hipStream_t s);
    void end_call(hipStream_t s);
    void sync_streams();  // waits for the context's stream and the last asynchronous call
    bool ready() const { return d_bsk_ && (d_ksk_ || d_wksk_); }
    // the 64-bit accumulator (boot_wide.h): the large-precision family and the GINX sets outside
    // the 32-bit kernel's range
    bool wide() const { return wide_; }
    // the 32-bit kernels' range: N = 1024, Q < 2^28, digitsG = 3, power-of-two q, qKS <= 2^16, n < 1024
    static bool fast_path(const Params& p);
    static bool narrow_set(const Params& p);  // the 64-bit accumulator runs its 32-bit policy (A32)
    // the digitsG = 4 sets at N = 1024, Q < 2^27 the split kernels take (K1s / K1m)
    static bool g3_set(const Params& p);
    static bool n2k_set(const Params& p);     // GINX gates on K1w (N = 2048 in registers)
    // 64-bit-path sets whose key switch runs on the 32-bit tiled kernel (u16 rows): qKS <= 2^16 a power
    // of two and a tiled shape (baseKS 32 / 64 with digitsKS 3, baseKS 16 with digitsKS 4), n < 2048
    static bool ks32_set(const Params& p);
    // the u32-sum form for power-of-two qKS above 2^16 (launch_keyswitch_w32 shapes)
    static bool ks32w_set(const Params& p);
    // the accumulator kernels a context of this set runs on (fhe_hip_params::kernel), with the A/B
    // environment knobs a context reads at creation (FHE_HIP_GINX3, FHE_HIP_N2K, FHE_HIP_NARROW)
    static uint32_t kernel_kind(const Params& p);
    // the same for this context: its own kernel flags, read from the environment when it was created
    uint32_t kernel() const;
    // the blind-rotation kernel a 2-input gate batch of `count` ciphertexts runs on in this context
    const char* gate_kernel(size_t count) const;

    // raw reference layouts (see include/fhe_hip.h)
    void load_bsk(const uint64_t* bsk, size_t words);
    void load_ksk(const uint64_t* A, size_t nA, const uint64_t* B, size_t nB);
    // BTKeyGen on this device (keygen_dev.hip): keys bit-identical to keygen_bootstrap(sk, seed),
    // generated in place in the resident layouts; non-null host pointers receive the raw layouts
    void keygen_device(const uint64_t* sk, size_t n, uint64_t seed, uint64_t* bsk_out, uint64_t* kskA_out,
                       uint64_t* kskB_out);
    // the resident keys of another context of the same parameter set (any device): every packed key buffer
    // copied device to device (hipMemcpyPeerAsync over xGMI between GPUs), no host repacking
    void copy_keys_from(const Engine& src);

    // EvalBinGate on `count` pairs; device pointers, asynchronous on `s`
    void eval_gate_device(int gate, size_t count, const uint64_t* a1, const uint64_t* b1, const uint64_t* a2,
                          const uint64_t* b2, uint64_t* a_out, uint64_t* b_out, hipStream_t s);
    // stage outputs on device: ctExt (count x N, mod Q) or mod-switched to qKS
    void bootstrap_device(int gate, size_t count, const uint64_t* a1, const uint64_t* b1, const uint64_t* a2,
                          const uint64_t* b2, bool modswitch, hipStream_t s);
    // KeySwitch + ModSwitch(qKS -> q) of the workspace left by bootstrap_device(modswitch = true)
    void keyswitch_workspace_device(size_t count, uint64_t* a_out, uint64_t* b_out, hipStream_t s);
    const uint32_t* ext_a() const { return d_ext_a_; }
    const uint32_t* ext_b() const { return d_ext_b_; }

    // ---- the Backend seam (backend.h:131-192) ----
    // BlindRotate[Batch] = EvalAcc (rgsw-acc-cggi.cpp:59-68 / rgsw-acc-lmkcdey.cpp:70-158 /
    // rgsw-acc-dm.cpp:62-77): acc [count][2][N] (EVALUATION, canonical mod Q) in/out, a [count][n]
    // mod ctmod (a power of two <= 2N; EvalAcc reads a_i with the ciphertext's modulus)
    void blind_rotate_acc_device(size_t count, const uint64_t* a, uint32_t ctmod, uint64_t* acc, hipStream_t s);
    // the seam's null accumulators (BootstrapBatch, batch.cpp:77-86): BinFHEScheme::Bootstrap's
    // accumulator, BootstrapGateCore(AND, ct + q/4) (binfhe-base-scheme.cpp:190-205, 525-583) on
    // ciphertexts (a [count][n], b [count]) mod q -- the test vector of the AND window at b + q/4,
    // EvalAcc over a -- written to acc [count][2][N] (EVALUATION, canonical mod Q)
    void blind_rotate_init_device(size_t count, const uint64_t* a, const uint64_t* b, uint64_t* acc, hipStream_t s);
    // ExternalProduct[Batch] = AddToAccLMKCDEY / AddToAccDM (rgsw-acc-lmkcdey.cpp:228-254,
    // rgsw-acc-dm.cpp:119-145): result[g] = rgsw[g] (x) rlwe[g]; rgsw [count][digitsG2][2][N] and
    // rlwe / result [count][2][N], EVALUATION, canonical mod Q; result may alias rlwe
    void external_product_device(size_t count, const uint64_t* rgsw, const uint64_t* rlwe, uint64_t* result,
                                 hipStream_t s);
    // upper bound on the batch one call can take on this device (Backend::MaxBatchSize)
    size_t max_batch() const;

    // EvalBinGate(gate, ctvector) for AND3 / OR3 / AND4 / OR4 / MAJORITY (binfhe-base-scheme.cpp:129-171):
    // k inputs a[j] [count][n], b[j] [count] (mod q), plaintext modulus p of the inputs
    void eval_gate_multi_device(int gate, size_t count, uint32_t k, const uint64_t* const* a,
                                const uint64_t* const* b, uint32_t p, uint64_t* a_out, uint64_t* b_out, hipStream_t s);
    // EvalBinGate(CMUX, {ct0, ct1, ct2}) = NAND(NAND(ct0, NOT ct2), NAND(ct1, ct2)) (:172-182):
    // one 2*count-gate NAND level, then one count-gate NAND level
    // BinFHEScheme::Bootstrap (binfhe-base-scheme.cpp:190-218): BootstrapGateCore(AND, ct + q/4), extraction,
    // SwitchCTtoqn; ciphertexts mod q of plaintext modulus 4
    void refresh_device(size_t count, const uint64_t* a, const uint64_t* b, uint64_t* a_out, uint64_t* b_out,
                        hipStream_t s);
    void eval_cmux_device(size_t count, const uint64_t* a0, const uint64_t* b0, const uint64_t* a1, const uint64_t* b1,
                          const uint64_t* a2, const uint64_t* b2, uint64_t* a_out, uint64_t* b_out, hipStream_t s);

    // ---- ciphertexts mod Q as inputs (binfhe-base-scheme.cpp:92-93, 150-152, 200-201) ----
    // SwitchCTtoqn (lwe-pke.cpp:170-178) of `count` ciphertexts a [count][N], b [count] mod Q into
    // [count][n] / [count] mod q: ModSwitch(Q -> qKS), KeySwitch, ModSwitch(qKS -> q)
    void switch_to_qn_device(size_t count, const uint64_t* a, const uint64_t* b, uint64_t* a_out, uint64_t* b_out,
                             hipStream_t s);
    // The reference's gate entry points on inputs of either modulus.  op: a 2-input gate (k = 2),
    // MAJORITY / AND3 / OR3 / AND4 / OR4 (k = 2..4, plaintext modulus ptmod), CMUX (k = 3) or kOpBootstrap
    // (BinFHEScheme::Bootstrap, k = 1, the input's plaintext modulus ptmod).  Column j: count ciphertexts,
    // large[j] == nullptr: rows of n words mod q; otherwise rows of N words, large[j][g] != 0 marking a
    // ciphertext mod Q (dimension N), 0 one mod q (its first n words).  Outputs [count][n] mod q, or
    // ctExt [count][N] mod Q when extended (CMUX ignores extended, as the reference does: :180-182).
    // Device pointers (large[j] too), asynchronous on s.
    static constexpr int kOpBootstrap = -1;
    void eval_mixed_device(int op, uint32_t k, uint32_t ptmod, size_t count, const uint64_t* const* a,
                           const uint64_t* const* b, const uint8_t* const* large, uint64_t* a_out, uint64_t* b_out,
                           bool extended, hipStream_t s);
    // the same on host buffers (synchronous)
    void eval_mixed_host(int op, uint32_t k, uint32_t ptmod, size_t count, const uint64_t* const* a,
                         const uint64_t* const* b, const uint8_t* const* large, uint64_t* a_out, uint64_t* b_out,
                         bool extended);
    void switch_to_qn_host(size_t count, const uint64_t* a, const uint64_t* b, uint64_t* a_out, uint64_t* b_out);

    // ---- functional bootstrapping (binfhe-base-scheme.cpp:241-521, 589-648); fb.cpp ----
    // BootstrapFunc: a [count][n] mod ctmod (power of two <= 2N), f[x] = f(x) < fmod for x < ctmod;
    // output [count][n] mod fmod
    void bootstrap_func_device(size_t count, const uint64_t* a, const uint64_t* b, uint32_t ctmod,
                               const uint64_t* f, uint64_t fmod, uint64_t* a_out, uint64_t* b_out, hipStream_t s);
    // the same with nt tables f[nt][ctmod]: ciphertext g bootstraps with table g % nt
    void bootstrap_func_tables(size_t count, const uint64_t* a, const uint64_t* b, uint32_t ctmod, const uint64_t* f,
                               uint32_t nt, uint64_t fmod, uint64_t* a_out, uint64_t* b_out, hipStream_t s);
    // EvalFunc: inputs / outputs mod q_in (= lut length, power of two)
    void eval_func_device(size_t count, const uint64_t* a, const uint64_t* b, uint64_t q_in, const uint64_t* lut,
                          uint64_t* a_out, uint64_t* b_out, hipStream_t s);
    // EvalFuncMultiOutputBatch (batch.cpp:141-174): nl LUTs luts[nl][q_in] on every input; output j of input
    // i at row i nl + j of a_out [count nl][n] / b_out [count nl].  The LUTs of one class (negacyclic /
    // periodic / arbitrary) share the class's LUT-independent first bootstrap, and their last bootstraps run
    // as one launch over count x nl ciphertexts
    void eval_func_multi_device(size_t count, const uint64_t* a, const uint64_t* b, uint64_t q_in, const uint64_t* luts,
                                uint32_t nl, uint64_t* a_out, uint64_t* b_out, hipStream_t s);
    // EvalFloor: inputs / outputs mod `mod`
    void eval_floor_device(size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod, uint32_t roundbits,
                           uint64_t* a_out, uint64_t* b_out, hipStream_t s);
    // EvalSign: inputs mod `mod` > q, outputs mod q
    void eval_sign_device(size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod, bool scheme_switch,
                          uint64_t* a_out, uint64_t* b_out, hipStream_t s);
    // EvalDecomp: a_out [parts][count][n], b_out [parts][count]
    uint32_t eval_decomp_parts(uint64_t mod) const;
    void eval_decomp_device(size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod, uint64_t* a_out,
                            uint64_t* b_out, hipStream_t s);
    // host-buffer versions (synchronous); op: 0 func (arg = q_in, lut), 1 floor (arg = mod, iarg =
    // roundbits), 2 sign (arg = mod, iarg = scheme_switch), 3 decomp (arg = mod), 4 bootstrap_func
    // (arg = ctmod, lut = f table, arg2 = fmod), 5 multi-output EvalFunc (arg = q_in, lut = luts[iarg][q_in];
    // outputs [count iarg] rows)
    void fb_host(int op, size_t count, const uint64_t* a, const uint64_t* b, uint64_t arg, uint64_t arg2,
                 uint32_t iarg, const uint64_t* lut, uint64_t* a_out, uint64_t* b_out);

    // host-buffer convenience entry points (synchronous)
    void eval_gate_host(int gate, size_t count, const uint64_t* a1, const uint64_t* b1, const uint64_t* a2,
                        const uint64_t* b2, uint64_t* a_out, uint64_t* b_out);
    void bootstrap_extended_host(int gate, size_t count, const uint64_t* a1, const uint64_t* b1,
                                 const uint64_t* a2, const uint64_t* b2, uint64_t* ext_a, uint64_t* ext_b);
    void keyswitch_host(size_t count, const uint64_t* a, const uint64_t* b, uint64_t* a_out, uint64_t* b_out);
    // extended = true returns ctExt ([count][N] mod Q) instead of the switched output
    void eval_gate_multi_host(int gate, size_t count, uint32_t k, const uint64_t* const* a, const uint64_t* const* b,
                              uint32_t p, uint64_t* a_out, uint64_t* b_out, bool extended);
    void refresh_host(size_t count, const uint64_t* a, const uint64_t* b, uint64_t* a_out, uint64_t* b_out);
    void eval_cmux_host(size_t count, const uint64_t* a0, const uint64_t* b0, const uint64_t* a1, const uint64_t* b1,
                        const uint64_t* a2, const uint64_t* b2, uint64_t* a_out, uint64_t* b_out);

private:
    // p: plaintext modulus of the bootstrapped ciphertext; multi: AND3..OR4/MAJORITY allowed
    GateArgs gate_args(int gate, size_t count, uint32_t p = 4, bool multi = false) const;
    // prep of g.count gates into the workspace slots [offset, offset + g.count)
    void prep_device(const GateArgs& g, const GateInputs& in, size_t offset, hipStream_t s);
    // blind rotation of workspace slots [0, g.count)
    void rotate_device(const GateArgs& g, hipStream_t s);
    void fb_floor(size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod, uint32_t roundbits, uint64_t* a_out,
                  uint64_t* b_out, uint64_t* w, hipStream_t s);
    uint64_t* fb_work(size_t count, int cts);
    void stage_inputs(size_t count, uint32_t k, const uint64_t* const* a, const uint64_t* const* b,
                      const uint64_t** da, const uint64_t** db);
    void ensure_work(size_t count);
    void ensure_host_stage(size_t count);
    void build_tables();
    void build_tables_wide();
    void build_loggen();
    // one ciphertext column switched to mod q (see eval_mixed_device): the flagged rows through
    // SwitchCTtoqn (negated at Q first when negate; b replaced by b_large when set_b), the others copied
    // (negated at q when negate); a_out [count][n] must not overlap the input
    void switch_column_device(size_t count, const uint64_t* a, const uint64_t* b, uint32_t stride, const uint8_t* large,
                              bool negate, bool set_b, uint64_t b_large, uint64_t* a_out, uint64_t* b_out, hipStream_t s);
    // ctExt of workspace slots [0, count) as u64 [count][N] / [count] into device buffers
    void ext_to_device(size_t count, uint64_t* a_out, uint64_t* b_out, hipStream_t s);
    // CMUX's two NAND levels (binfhe-base-scheme.cpp:176-182); a2n / b2n: NOT ct2 given explicitly
    // (nullptr: folded into the first NAND's input combination)
    void cmux_levels(size_t count, const uint64_t* a0, const uint64_t* b0, const uint64_t* a1, const uint64_t* b1,
                     const uint64_t* a2, const uint64_t* b2, const uint64_t* a2n, const uint64_t* b2n, uint64_t* a_out,
                     uint64_t* b_out, hipStream_t s);
    // grow-only device scratch (synchronises the context's streams before it grows)
    uint64_t* grow(uint64_t*& ptr, size_t& cap, size_t bytes);
    // KeySwitch + ModSwitch(qKS -> q_out) of workspace slots [0, count) (q_out = 0: none)
    void keyswitch_ext(size_t count, uint64_t q_out, uint64_t* a_out, uint64_t* b_out, hipStream_t s);
    // ctExt of workspace slots [0, count) to host u64 arrays
    void copy_ext_host(size_t count, uint64_t* ext_a, uint64_t* ext_b);

    Params p_;
    int device_;
    hipStream_t stream_ = nullptr;
    BootTables tabs_{};
    void* d_tables_ = nullptr;
    void* d_bsk_ = nullptr;
    void* d_autok_ = nullptr;   // LMKCDEY automorphism keys (inside the d_bsk_ allocation)
    int16_t* d_logGen_ = nullptr;
    uint32_t maxops_ = 0;
    uint16_t* d_ops_ = nullptr;
    uint32_t* d_nops_ = nullptr;
    uint16_t* d_ksk_ = nullptr;
    uint32_t* d_kspart_ = nullptr;   // row-split key-switch partials (ks_part)
    static constexpr size_t kKsPartWords = (size_t)1 << 25;  // 2^16 rows x 512 u32
    uint32_t* ks_part(size_t count);
    // GINX kernel choice: 0 by batch size, 1 one wave per gate (K1), 2 two waves per gate with the digit
    // exchange (K1s), 3 two waves per gate with K1w's one-word exchange (K1x).  K1s is slower than K1 at
    // every batch size (1024 gates 4.87 vs 4.37 ms: two barriers per index, the partner's digits read in
    // the MAC) and only FHE_HIP_GINX_KERNEL=split pins it; K1x runs batches of up to kXBatch gates.
    int ginx_kernel_ = 0;
    // GINX kernel of a gate launch (ginx_kernel_ pins, else by batch size): 1 K1, 2 K1s, 3 K1x, 4 K1q (four waves
    // per gate, up to one gate per CU; FHE_HIP_GINX_KERNEL=qsplit pins it)
    int ginx_choice(const GateArgs& g) const;
    // K1x runs batches of up to x_batch_ gates: one two-gate workgroup per CU (2 x the CU count, 512 on
    // MI355X).  Measured (tools/gate_time.py, STD128 AND, profiles/r06_k1x_ab2.txt): 512 gates 2.69 vs 4.16 ms
    // (K1), 768 gates 4.28 vs 4.18, 1024 gates 4.56 vs 4.24: once two of its waves share a SIMD they overlap
    // poorly, and the one-wave kernel wins.  Up to x_batch_ / 2 gates each gate has its own 128-thread workgroup
    // (a CU of its own: 1 gate 2.30 vs 2.64 ms, profiles/r06_k1x_lb_ab.txt); the LMKCDEY two-wave kernel likewise
    uint32_t x_batch_ = 512;
    // LMKCDEY kernel choice on the fast path: 0 by batch size, 1 the one-wave op-list kernel (K1 LMK), 2 two
    // waves per gate (K1m's two-digit form, k_blind_rotate_lmk3<2, ..>), 4 four waves per gate (K1m-4,
    // k_blind_rotate_lmk4x) -- FHE_HIP_LMK_KERNEL = wave | split | qsplit
    int lmk_kernel_ = 0;
    // the kernel of this LMKCDEY launch: 1, 2 (up to x_batch_ gates) or 4 (up to x_batch_ / 2); lmk_kernel_ pins
    int lmk_choice(const GateArgs& g) const;
    void* d_bsk2_ = nullptr;   // K1s / K1x / K1m-2 key layout (g3_: K1s's nd = 3 layout; n2k_: K1w's)
    void repack_ginx2();
    // digitsG = 4 GINX sets at N = 1024, Q < 2^27 (STD128_3, STD128Q, STD128_4, LPF_STD128, LPF_STD128Q):
    // gates on the split kernel with three digits per component (launch_blind_rotate_ginx3) over the
    // 32-bit tables tabs_, the rest of the 64-bit path unchanged.  FHE_HIP_GINX3=0 keeps them on the 64-bit accumulator (A/B, tests).
    bool g3_ = false;
    void pack_ginx3(const uint64_t* bsk);
    // GINX at N = 2048, Q < 2^27, digitsG = 4, q < 2N (STD256Q): gates on K1w (launch_blind_rotate_n2k)
    // over its own 32-bit tables, keys packed into d_bsk2_; the rest of the 64-bit path (prep, key
    // switch, functional bootstrapping) unchanged.  FHE_HIP_N2K=0 keeps them on K5 (A/B, tests).
    bool n2k_ = false;
    // the 32-bit key switch on the 64-bit path (ks32_set; g3_ sets always, FHE_HIP_KS32=0 keeps the
    // u64 row gathers of launch_keyswitch_wide for the others: A/B, tests)
    bool ks32_ = false;
    bool ks32w_ = false;
    uint32_t* d_ksk32_ = nullptr;  // ks32w_: u32 rows of ksk_width(n)
    BootTables tabs2k_{};
    void* d_tables2k_ = nullptr;
    void build_tables_n2k();
    void pack_n2k(const uint64_t* bsk);
    // cross-stream ordering (use_stream)
    hipStream_t last_stream_ = nullptr;
    hipEvent_t order_ev_ = nullptr;
    bool pending_ = false;
    // workspace; rot_count_ = ciphertexts the last blind rotation left in it
    size_t cap_ = 0;
    size_t rot_count_ = 0;
    uint16_t* d_idx_ = nullptr;
    uint32_t* d_tvb_ = nullptr;
    uint32_t* d_ext_a_ = nullptr;
    uint32_t* d_ext_b_ = nullptr;
    // CMUX: first-level NAND outputs [2 count][n] + [2 count] (ccap_: bytes)
    size_t ccap_ = 0;
    uint64_t* d_l1_ = nullptr;
    // mixed-modulus inputs: switched columns (eval_mixed_device) and the host entry point's staging
    size_t mixcap_ = 0, mixiocap_ = 0;
    uint64_t* d_mix_ = nullptr;
    uint64_t* d_mixio_ = nullptr;
    // functional bootstrapping: test-vector table [2N] u32 and ciphertext temporaries
    uint64_t* d_tvbuf_ = nullptr;   // BootstrapFunc tables: u32 words (u64 on the wide path), grown with their count
    size_t tvcap_ = 0;
    size_t fbcap_ = 0;
    uint64_t* d_fb_ = nullptr;
    // ExternalProduct: packed per-item keys and one-op lists (grown on demand)
    size_t epcap_ = 0;
    uint32_t* d_epk_ = nullptr;
    uint16_t* d_epops_ = nullptr;
    uint32_t* d_epn_ = nullptr;
    // staging for host entry points: up to 4 inputs + one ctExt-sized output
    size_t hcap_ = 0;
    uint64_t* d_io_ = nullptr;
    // large-precision family: u64 keys (Montgomery BSK, raw KSK A ++ B), tables, u64 ctExt
    bool wide_ = false;
    // the wide accumulator in 32-bit residues (bootstrap_wide.hip A32): Q < 2^30 and digitsG2 Q < 2^32;
    // d_bsk_ then holds u32 Montgomery words
    bool narrow_ = false;
    WideTables wtabs_{};
    // word w of the resident wide keys (u64, or u32 when narrow_)
    const void* wkey(size_t w) const {
        return narrow_ ? (const void*)(static_cast<const uint32_t*>(d_bsk_) + w)
                       : (const void*)(static_cast<const uint64_t*>(d_bsk_) + w);
    }
    void* d_wtables_ = nullptr;
    uint64_t* d_wksk_ = nullptr;
    uint64_t* d_wext_a_ = nullptr;
    uint64_t* d_wext_b_ = nullptr;
    // the key the wide kernel bootstraps with: the context's own baseG, or (timeOptimization) the
    // one EvalSign / EvalDecomp switched to (set_base); word offset into d_bsk_ and its digits
    Params cur_;
    size_t cur_off_ = 0;
    size_t cur_ksk_off_ = 0;   // word offset of the current base's switching key in d_wksk_
    void set_base(uint32_t bg);
    void dynamic_base(uint64_t mod);
    struct BaseGuard {  // Change_BaseG(curBase) when EvalSign / EvalDecomp end (:453, :518)
        Engine* e;
        ~BaseGuard() { e->set_base(e->p_.baseG); }
    };
};

}  // namespace fhe_amd
