// c_api_hip_types.h -- the opaque handles of include/lux/fhe/c_api.h as integration/c_api_hip.cpp defines
// them (the reference's c_api.cpp:20-42 plus the context's device backend).  Internal: shared with the
// test driver (oracle/bh_driver.cpp), which evaluates the reference's CPU path on the same context.
#ifndef FHE_AMD_C_API_HIP_TYPES_H
#define FHE_AMD_C_API_HIP_TYPES_H

#include <memory>

#include "backend_hip.h"
#include "binfhecontext.h"

struct LuxFheContext {
    lux::fhe::BinFHEContext cc;
    lux::fhe::BINFHE_PARAMSET set = lux::fhe::STD128_LMKCDEY;
    lux::fhe::BINFHE_METHOD method = lux::fhe::LMKCDEY;
    std::unique_ptr<lux::fhe::backend::BackendHIP> gpu;  // created with the first bootstrapped call
};
struct LuxFheSecretKey {
    lux::fhe::LWEPrivateKey sk;
};
struct LuxFhePublicKey {
    lux::fhe::LWEPublicKey pk;
};
struct LuxFheBootstrapKey {
    bool generated = false;
};
struct LuxFheCiphertext {
    lux::fhe::LWECiphertext ct;
};

#endif
