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
 *     given HIP stream (NULL = the context's own stream);
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
/* Device memory (Backend::Allocate/Free/CopyToDevice/CopyToHost/Synchronize, */
/*   backend.h:94-114)                                                       */
/* ------------------------------------------------------------------------ */
int fhe_hip_alloc(int device, size_t bytes, void** d_ptr);
int fhe_hip_free(void* d_ptr);
int fhe_hip_copy_to_device(void* d_dst, const void* h_src, size_t bytes);
int fhe_hip_copy_to_host(void* h_dst, const void* d_src, size_t bytes);
int fhe_hip_synchronize(int device);
int fhe_hip_device_count(int* count);
/* message of the last error on this host thread */
const char* fhe_hip_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* FHE_HIP_H */
