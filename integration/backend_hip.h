// backend_hip.h -- lux::fhe::backend::Backend (src/binfhe/include/backend/backend.h:73-247 in the
// reference) implemented over the fhe_amd C-ABI (include/fhe_hip.h).  This is the reference-side
// half of the drop-in: a maintainer adds it to src/binfhe/lib/backend/ and links libfhe_amd.so.
// Only plain pointers and sizes cross into libfhe_amd; the reference's types stay on this side.
//
// Here it is built test-only by oracle/Makefile (oracle/_ref/libbackend_hip.so) against the
// reference's own headers and sources, and registered in the reference's BackendRegistry by the
// GPU tests (tests/test_backend.py through oracle/bh_driver.cpp).
#ifndef FHE_AMD_BACKEND_HIP_H
#define FHE_AMD_BACKEND_HIP_H

#include <mutex>
#include <string>
#include <vector>

#include "backend/backend.h"
#include "batch/binfhe-batch.h"
#include "binfhecontext.h"
#include "lwe-keyswitchkey.h"
#include "rlwe-ciphertext.h"
#include "fhe_hip.h"

namespace lux::fhe::backend {

// BackendType is {CPU, MLX, CUDA, AUTO} upstream (backend.h:31-36); the one-line enum addition
// `HIP` (value 4) is what INTEGRATION.md proposes.  Until then the registry is keyed by this value.
constexpr BackendType kBackendHIP = static_cast<BackendType>(4);

class BackendHIP : public Backend {
public:
    // one fhe_amd context on `device` for the parameter set a BinFHEContext was generated with
    BackendHIP(BINFHE_PARAMSET set, BINFHE_METHOD method, int device = 0);
    ~BackendHIP() override;
    BackendHIP(const BackendHIP&) = delete;
    BackendHIP& operator=(const BackendHIP&) = delete;

    // info (backend.h:81-87)
    BackendType Type() const override { return kBackendHIP; }
    std::string Name() const override;
    bool IsAvailable() const override;
    size_t MaxBatchSize() const override;
    size_t DeviceMemory() const override;

    // memory (backend.h:94-114): device buffers on this backend's GPU
    DeviceBuffer Allocate(size_t bytes) override;
    void Free(DeviceBuffer& buffer) override;
    void CopyToDevice(const void* host_ptr, DeviceBuffer& device_buffer, size_t bytes) override;
    void CopyToHost(const DeviceBuffer& device_buffer, void* host_ptr, size_t bytes) override;
    void Synchronize() override;

    // single ops (backend.h:131-165): batches of one
    void BlindRotate(const std::shared_ptr<RingGSWCryptoParams>& params, const LWECiphertext& ct,
                     const RingGSWACCKey& ek, RLWECiphertext& acc) override;
    void ExternalProduct(const std::shared_ptr<RingGSWCryptoParams>& params, const RingGSWEvalKey& rgsw,
                         const RLWECiphertext& rlwe, RLWECiphertext& result) override;
    void KeySwitch(const std::shared_ptr<LWECryptoParams>& params, const LWECiphertext& ct,
                   const LWESwitchingKey& ks, LWECiphertext& result) override;
    void ModSwitch(const std::shared_ptr<LWECryptoParams>& params, const LWECiphertext& ct,
                   LWECiphertext& result) override;

    // batch ops (backend.h:177-211): one device call per batch
    //   BlindRotateBatch    = EvalAcc of the method (accs in/out, EVALUATION); null accumulators
    //                         (what BootstrapBatch passes, batch.cpp:77-86) are initialised as
    //                         BinFHEScheme::Bootstrap's: BootstrapGateCore(AND, ct + q/4)
    //                         (binfhe-base-scheme.cpp:190-205, 525-583)
    //   ExternalProductBatch= AddToAccLMKCDEY / AddToAccDM (rgsw (x) rlwe)
    //   KeySwitchBatch      = LWEEncryptionScheme::KeySwitch (lwe-pke.cpp:348-372)
    //   ModSwitchBatch      = LWEEncryptionScheme::ModSwitch to the next modulus of SwitchCTtoqn:
    //                         Q -> qKS for ciphertexts mod Q, qKS -> q for ciphertexts mod qKS
    void BlindRotateBatch(const std::shared_ptr<RingGSWCryptoParams>& params, const std::vector<LWECiphertext>& cts,
                          const RingGSWACCKey& ek, std::vector<RLWECiphertext>& accs) override;
    void ExternalProductBatch(const std::shared_ptr<RingGSWCryptoParams>& params,
                              const std::vector<RingGSWEvalKey>& rgsws, const std::vector<RLWECiphertext>& rlwes,
                              std::vector<RLWECiphertext>& results) override;
    void KeySwitchBatch(const std::shared_ptr<LWECryptoParams>& params, const std::vector<LWECiphertext>& cts,
                        const LWESwitchingKey& ks, std::vector<LWECiphertext>& results) override;
    void ModSwitchBatch(const std::shared_ptr<LWECryptoParams>& params, const std::vector<LWECiphertext>& cts,
                        std::vector<LWECiphertext>& results) override;

    // packed formats (backend.h:223-246): the reference's packed.h byte formats, held in device memory
    DeviceBuffer PackBootstrappingKey(const RingGSWACCKey& ek) override;
    void UnpackBootstrappingKey(const DeviceBuffer& packed, RingGSWACCKey& ek) override;
    DeviceBuffer PackCiphertexts(const std::vector<LWECiphertext>& cts) override;
    void UnpackCiphertexts(const DeviceBuffer& packed, std::vector<LWECiphertext>& cts) override;

    // beyond the seam: the fused gate path, EvalBinGateBatch semantics (batch.cpp:176-210) -- prep,
    // blind rotation, extraction, ModSwitch, KeySwitch, ModSwitch in two device launches
    void EvalBinGateBatch(BINGATE gate, const RingGSWBTKey& keys, const std::vector<LWECiphertext>& ct1,
                          const std::vector<LWECiphertext>& ct2, std::vector<LWECiphertext>& out);

    // the reference's other batch callers on the GPU, one device pass per batch:
    //   EvalFuncBatch: BinFHEContext::EvalFunc (binfhe-base-scheme.cpp:241-332) on every ciphertext, at
    //                  its own modulus (ct->GetModulus(); ciphertexts of one modulus go in one pass)
    //   EvalCMUXBatch: EvalBinGate(CMUX, {ct0, ct1, ct2}) (binfhe-base-scheme.cpp:172-182) per row: three
    //                  NAND bootstraps in two dependent launches
    void EvalFuncBatch(const RingGSWBTKey& keys, const std::vector<LWECiphertext>& cts,
                       const std::vector<NativeInteger>& lut, std::vector<LWECiphertext>& out);
    //   EvalFuncMultiOutputBatch: EvalFunc(ct_i, luts[j]) for every pair (batch.cpp:141-174), output j of input
    //                  i at i * L + j; one device call per ciphertext modulus (fhe_hip_eval_func_multi_batch)
    void EvalFuncMultiOutputBatch(const RingGSWBTKey& keys, const std::vector<LWECiphertext>& cts,
                                  const std::vector<std::vector<NativeInteger>>& luts, std::vector<LWECiphertext>& out);
    //   RefreshBatch:  BinFHEContext::Bootstrap (BinFHEScheme::Bootstrap, binfhe-base-scheme.cpp:190-220) per
    //                  ciphertext, mod q or mod Q (switched first, :200-201), any plaintext modulus
    //   EvalBinGateBatch / EvalCMUXBatch take ciphertexts mod Q (dimension N) as well (:92-93, :180-182)
    void RefreshBatch(const RingGSWBTKey& keys, const std::vector<LWECiphertext>& cts, std::vector<LWECiphertext>& out);
    void EvalCMUXBatch(const RingGSWBTKey& keys, const std::vector<LWECiphertext>& ct0,
                       const std::vector<LWECiphertext>& ct1, const std::vector<LWECiphertext>& ct2,
                       std::vector<LWECiphertext>& out);

    fhe_hip_ctx* Context() const { return ctx_; }
    // destroys the device context now (the registry owns backends until static destruction, which
    // may run after the HIP runtime's own teardown); the backend is unavailable afterwards
    void Release();
    const fhe_hip_params& Params() const { return p_; }

private:
    void Check(int rc, const char* what) const;
    void CheckRGSW(const std::shared_ptr<RingGSWCryptoParams>& params) const;
    void CheckLWE(const std::shared_ptr<LWECryptoParams>& params) const;
    // keys are uploaded once and re-uploaded only when a different key object arrives
    void EnsureBSK(const RingGSWACCKey& ek);
    void EnsureKSK(const LWESwitchingKey& ks);
    std::vector<uint64_t> RawBSK(const RingGSWACCKey& ek) const;

    fhe_hip_ctx* ctx_ = nullptr;
    fhe_hip_params p_{};
    int device_ = 0;
    BINFHE_PARAMSET set_;
    BINFHE_METHOD method_;
    // the key objects resident on the device, held weakly: a key that was freed (and an unrelated
    // one allocated at its address) or replaced forces a reload; in-place edits of a live key object
    // are not detected (call PackBootstrappingKey to reload explicitly)
    std::weak_ptr<const void> bsk_id_;
    std::weak_ptr<const void> ksk_id_;
    std::mutex mu_;  // one context, one workspace: calls are serialized
};

// The routing INTEGRATION.md proposes for lux::fhe::EvalBinGateBatch (batch/batch.cpp:176-210): with a
// BackendHIP as the registry's default the whole batch goes through its fused gate path (two device
// launches) under the context's keys (cc.GetRefreshKey / GetSwitchKey); with any other default it is
// the reference's own OpenMP loop over cc.EvalBinGate.  Same BatchResult semantics as the reference
// (size mismatch, empty batch, exceptions caught into the result).
BatchResult EvalBinGateBatchHIP(BinFHEContext& cc, BINGATE gate, const std::vector<LWECiphertext>& ct1,
                                const std::vector<LWECiphertext>& ct2, std::vector<LWECiphertext>& ct_out,
                                uint32_t flags = 0);

// The same routing for the reference's other batch callers (batch/batch.cpp), each with the reference's
// BatchResult semantics and its OpenMP loop as the fallback when the default backend is not a BackendHIP:
//   EvalFuncBatchHIP            <- EvalFuncBatch (batch.cpp:106-139): ct_out[i] = cc.EvalFunc(ct_in[i], lut)
//   EvalFuncMultiOutputBatchHIP <- EvalFuncMultiOutputBatch (:141-174): ct_out[i * L + j] = EvalFunc(ct_in[i],
//                                  luts[j]); one GPU pass per LUT; processed = ct_in.size()
//   EvalCMUXBatchHIP            <- EvalCMUXBatch (:212-249): ct_out[i] = cc.EvalBinGate(CMUX, {ct_sel[i],
//                                  ct_true[i], ct_false[i]}), the vector order the reference passes
BatchResult EvalFuncBatchHIP(BinFHEContext& cc, const std::vector<LWECiphertext>& ct_in,
                             const std::vector<NativeInteger>& lut, std::vector<LWECiphertext>& ct_out,
                             uint32_t flags = 0);
BatchResult EvalFuncMultiOutputBatchHIP(BinFHEContext& cc, const std::vector<LWECiphertext>& ct_in,
                                        const std::vector<std::vector<NativeInteger>>& luts,
                                        std::vector<LWECiphertext>& ct_out, uint32_t flags = 0);
BatchResult EvalCMUXBatchHIP(BinFHEContext& cc, const std::vector<LWECiphertext>& ct_sel,
                             const std::vector<LWECiphertext>& ct_true, const std::vector<LWECiphertext>& ct_false,
                             std::vector<LWECiphertext>& ct_out, uint32_t flags = 0);

}  // namespace lux::fhe::backend

#endif
