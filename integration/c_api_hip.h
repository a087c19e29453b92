// c_api_hip.h -- batch entry points added next to the reference's public C API
// (/root/reference/include/lux/fhe/c_api.h) by integration/c_api_hip.cpp, the drop-in replacement of
// src/c_api/c_api.cpp whose bootstrapped operations run on the GPU through BackendHIP.
//
// The single-ciphertext functions of c_api.h keep their signatures and semantics (c_api.cpp:73-349); a
// gate on one pair is a batch of one.  These batch forms are what an FFI caller (Go cgo, ctypes) binds to
// amortise the device round trip over many gates: one GPU pass per call, outputs in input order, the
// same error convention (no exception crosses; LUX_FHE_ERR_GATE / _BOOTSTRAP on failure, nothing
// allocated then).
#ifndef FHE_AMD_C_API_HIP_H
#define FHE_AMD_C_API_HIP_H

#include "lux/fhe/c_api.h"

#ifdef __cplusplus
extern "C" {
#endif

// two-input gates of c_api.h (lux_fhe_and .. lux_fhe_xnor), as BINGATE values (binfhe-constants.h)
typedef enum {
    LUX_FHE_GATE_OR   = 0,
    LUX_FHE_GATE_AND  = 1,
    LUX_FHE_GATE_NOR  = 2,
    LUX_FHE_GATE_NAND = 3,
    LUX_FHE_GATE_XOR  = 4,
    LUX_FHE_GATE_XNOR = 5,
} LuxFheGate;

// result[i] = gate(a[i], b[i]) for i < count
LUX_FHE_API LuxFheError lux_fhe_gate_batch(LuxFheContext* ctx, const LuxFheBootstrapKey* bsk, LuxFheGate gate,
                                           const LuxFheCiphertext* const* a, const LuxFheCiphertext* const* b,
                                           size_t count, LuxFheCiphertext** result);
// result[i] = lux_fhe_mux(sel[i], a[i], b[i]): EvalBinGate(CMUX, {sel, a, b}) as c_api.cpp:249-261 passes it
LUX_FHE_API LuxFheError lux_fhe_mux_batch(LuxFheContext* ctx, const LuxFheBootstrapKey* bsk,
                                          const LuxFheCiphertext* const* sel, const LuxFheCiphertext* const* a,
                                          const LuxFheCiphertext* const* b, size_t count, LuxFheCiphertext** result);
// result[i] = lux_fhe_bootstrap(ct[i]) (BinFHEContext::Bootstrap)
LUX_FHE_API LuxFheError lux_fhe_bootstrap_batch(LuxFheContext* ctx, const LuxFheBootstrapKey* bsk,
                                                const LuxFheCiphertext* const* ct, size_t count,
                                                LuxFheCiphertext** result);

#ifdef __cplusplus
}
#endif

#endif
