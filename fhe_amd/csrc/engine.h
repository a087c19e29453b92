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
    bool ready() const { return d_bsk_ && d_ksk_; }

    // raw reference layouts (see include/fhe_hip.h)
    void load_bsk(const uint64_t* bsk, size_t words);
    void load_ksk(const uint64_t* A, size_t nA, const uint64_t* B, size_t nB);

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

    // host-buffer convenience entry points (synchronous)
    void eval_gate_host(int gate, size_t count, const uint64_t* a1, const uint64_t* b1, const uint64_t* a2,
                        const uint64_t* b2, uint64_t* a_out, uint64_t* b_out);
    void bootstrap_extended_host(int gate, size_t count, const uint64_t* a1, const uint64_t* b1,
                                 const uint64_t* a2, const uint64_t* b2, uint64_t* ext_a, uint64_t* ext_b);
    void keyswitch_host(size_t count, const uint64_t* a, const uint64_t* b, uint64_t* a_out, uint64_t* b_out);

private:
    GateArgs gate_args(int gate, size_t count) const;
    void ensure_work(size_t count);
    void ensure_host_stage(size_t count);
    void build_tables();

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
    uint16_t* d_scratch_ = nullptr;
    uint16_t* d_ksk_ = nullptr;
    // workspace
    size_t cap_ = 0;
    uint16_t* d_idx_ = nullptr;
    uint32_t* d_tvb_ = nullptr;
    uint32_t* d_ext_a_ = nullptr;
    uint32_t* d_ext_b_ = nullptr;
    // staging for host entry points
    size_t hcap_ = 0;
    uint64_t* d_io_ = nullptr;
};

}  // namespace fhe_amd
