// c_api_hip.cpp -- the reference's public C API (include/lux/fhe/c_api.h:47-122) with every bootstrapped
// operation on the GPU.  A maintainer builds this file instead of src/c_api/c_api.cpp; FFI callers (the Go
// cgo bridge, ctypes) keep binding the same symbols.
//
//   context / keys / encryption / serialization   BinFHEContext on the CPU, as c_api.cpp:73-224, 291-349
//   lux_fhe_and .. xnor, lux_fhe_mux               BackendHIP::EvalBinGateBatch / EvalCMUXBatch, a batch of one
//   lux_fhe_bootstrap                               BackendHIP::RefreshBatch (BinFHEScheme::Bootstrap)
//   lux_fhe_gate_batch / mux_batch / bootstrap_batch (c_api_hip.h): the same over many ciphertexts
//
// Kept from the reference: the parameter mapping (c_api.cpp:44-68: LUX_FHE_PARAMS_STD128 is
// STD128_LMKCDEY, so the API's default path is the LMKCDEY accumulator), the error codes of each entry
// point, and that no exception crosses the boundary.  The device context is created with the bootstrap
// key (LUX_FHE_HIP_DEVICE selects the GPU, default 0); the keys are uploaded on the first gate and again
// only when BTKeyGen replaces them.
#include "c_api_hip.h"
#include "c_api_hip_types.h"

#include <cstdlib>
#include <cstring>
#include <memory>
#include <sstream>
#include <vector>

#include "backend_hip.h"
#include "binfhecontext.h"
#include "utils/serial.h"

using namespace lux::fhe;
using lux::fhe::backend::BackendHIP;

namespace {

// every entry point: run f, map any exception to the entry point's own error code
template <typename F>
LuxFheError guard(LuxFheError on_error, F&& f) {
    try {
        return f();
    }
    catch (...) {
        return on_error;
    }
}

BINFHE_PARAMSET paramset_of(LuxFheParams p) {
    static const BINFHE_PARAMSET sets[] = {TOY,           MEDIUM,          STD128_LMKCDEY, STD128Q_LMKCDEY,
                                           STD192_LMKCDEY, STD192Q_LMKCDEY, STD256_LMKCDEY, STD256Q_LMKCDEY};
    const int i = static_cast<int>(p);
    return i >= 0 && i < 8 ? sets[i] : STD128_LMKCDEY;
}

BINFHE_METHOD method_of(LuxFheMethod m) {
    return m == LUX_FHE_METHOD_AP ? AP : m == LUX_FHE_METHOD_GINX ? GINX : LMKCDEY;
}

BackendHIP& device(LuxFheContext* ctx) {
    if (!ctx->gpu) {
        const char* dev = std::getenv("LUX_FHE_HIP_DEVICE");
        ctx->gpu = std::make_unique<BackendHIP>(ctx->set, ctx->method, dev ? std::atoi(dev) : 0);
    }
    return *ctx->gpu;
}

RingGSWBTKey keys_of(LuxFheContext* ctx) {
    RingGSWBTKey k;
    k.BSkey = ctx->cc.GetRefreshKey();
    k.KSkey = ctx->cc.GetSwitchKey();
    return k;
}

std::vector<LWECiphertext> unwrap(const LuxFheCiphertext* const* v, size_t count) {
    std::vector<LWECiphertext> out(count);
    for (size_t i = 0; i < count; ++i) {
        if (!v[i])
            throw std::invalid_argument("null ciphertext");
        out[i] = v[i]->ct;
    }
    return out;
}

// results handed out only once all of them exist (nothing allocated on failure)
void wrap(const std::vector<LWECiphertext>& v, LuxFheCiphertext** out) {
    std::vector<std::unique_ptr<LuxFheCiphertext>> tmp(v.size());
    for (size_t i = 0; i < v.size(); ++i) {
        tmp[i]     = std::make_unique<LuxFheCiphertext>();
        tmp[i]->ct = v[i];
    }
    for (size_t i = 0; i < v.size(); ++i)
        out[i] = tmp[i].release();
}

LuxFheError gate_batch(LuxFheContext* ctx, const LuxFheBootstrapKey* bsk, BINGATE gate,
                       const LuxFheCiphertext* const* a, const LuxFheCiphertext* const* b, size_t count,
                       LuxFheCiphertext** result) {
    if (!ctx || !bsk || !result || (count && (!a || !b)))
        return LUX_FHE_ERR_NULL_PTR;
    if (!bsk->generated)
        return LUX_FHE_ERR_NOT_INIT;
    return guard(LUX_FHE_ERR_GATE, [&] {
        std::vector<LWECiphertext> out;
        device(ctx).EvalBinGateBatch(gate, keys_of(ctx), unwrap(a, count), unwrap(b, count), out);
        wrap(out, result);
        return LUX_FHE_OK;
    });
}

LuxFheError mux_batch(LuxFheContext* ctx, const LuxFheBootstrapKey* bsk, const LuxFheCiphertext* const* sel,
                      const LuxFheCiphertext* const* a, const LuxFheCiphertext* const* b, size_t count,
                      LuxFheCiphertext** result) {
    if (!ctx || !bsk || !result || (count && (!sel || !a || !b)))
        return LUX_FHE_ERR_NULL_PTR;
    if (!bsk->generated)
        return LUX_FHE_ERR_NOT_INIT;
    return guard(LUX_FHE_ERR_GATE, [&] {
        std::vector<LWECiphertext> out;
        device(ctx).EvalCMUXBatch(keys_of(ctx), unwrap(sel, count), unwrap(a, count), unwrap(b, count), out);
        wrap(out, result);
        return LUX_FHE_OK;
    });
}

LuxFheError bootstrap_batch(LuxFheContext* ctx, const LuxFheBootstrapKey* bsk, const LuxFheCiphertext* const* ct,
                            size_t count, LuxFheCiphertext** result) {
    if (!ctx || !bsk || !result || (count && !ct))
        return LUX_FHE_ERR_NULL_PTR;
    if (!bsk->generated)
        return LUX_FHE_ERR_NOT_INIT;
    return guard(LUX_FHE_ERR_BOOTSTRAP, [&] {
        std::vector<LWECiphertext> out;
        device(ctx).RefreshBatch(keys_of(ctx), unwrap(ct, count), out);
        wrap(out, result);
        return LUX_FHE_OK;
    });
}

template <typename T>
LuxFheError marshal(const T& obj, uint8_t** data, size_t* len) {
    return guard(LUX_FHE_ERR_SERIALIZE, [&] {
        std::ostringstream os;
        Serial::Serialize(obj, os, SerType::BINARY);
        const std::string s = os.str();
        auto buf            = std::make_unique<uint8_t[]>(s.size());
        std::memcpy(buf.get(), s.data(), s.size());
        *len  = s.size();
        *data = buf.release();
        return LUX_FHE_OK;
    });
}

template <typename T>
LuxFheError unmarshal(const uint8_t* data, size_t len, T& obj) {
    return guard(LUX_FHE_ERR_DESERIALIZE, [&] {
        std::istringstream is(std::string(reinterpret_cast<const char*>(data), len));
        Serial::Deserialize(obj, is, SerType::BINARY);
        return LUX_FHE_OK;
    });
}

}  // namespace

extern "C" {

// ---- context (c_api.h:97-116) ----
LuxFheError lux_fhe_context_new(LuxFheContext** ctx, LuxFheParams params, LuxFheMethod method) {
    if (!ctx)
        return LUX_FHE_ERR_NULL_PTR;
    return guard(LUX_FHE_ERR_ALLOC, [&] {
        auto c    = std::make_unique<LuxFheContext>();
        c->set    = paramset_of(params);
        c->method = method_of(method);
        c->cc.GenerateBinFHEContext(c->set, c->method);
        *ctx = c.release();
        return LUX_FHE_OK;
    });
}

void lux_fhe_context_free(LuxFheContext* ctx) {
    delete ctx;
}

uint32_t lux_fhe_context_n(const LuxFheContext* ctx) {
    return ctx ? const_cast<LuxFheContext*>(ctx)->cc.GetParams()->GetLWEParams()->Getn() : 0;
}

uint32_t lux_fhe_context_ring_dim(const LuxFheContext* ctx) {
    return ctx ? const_cast<LuxFheContext*>(ctx)->cc.GetParams()->GetRingGSWParams()->GetN() : 0;
}

uint64_t lux_fhe_context_modulus(const LuxFheContext* ctx) {
    return ctx ? const_cast<LuxFheContext*>(ctx)->cc.GetParams()->GetLWEParams()->Getq().ConvertToInt() : 0;
}

// ---- keys (c_api.h:122-147) ----
LuxFheError lux_fhe_keygen_secret(LuxFheContext* ctx, LuxFheSecretKey** sk) {
    if (!ctx || !sk)
        return LUX_FHE_ERR_NULL_PTR;
    return guard(LUX_FHE_ERR_KEYGEN, [&] {
        auto k = std::make_unique<LuxFheSecretKey>();
        k->sk  = ctx->cc.KeyGen();
        *sk    = k.release();
        return LUX_FHE_OK;
    });
}

LuxFheError lux_fhe_keygen_public(LuxFheContext* ctx, const LuxFheSecretKey* sk, LuxFhePublicKey** pk) {
    if (!ctx || !sk || !pk)
        return LUX_FHE_ERR_NULL_PTR;
    return guard(LUX_FHE_ERR_KEYGEN, [&] {
        auto k = std::make_unique<LuxFhePublicKey>();
        k->pk  = ctx->cc.PubKeyGen(sk->sk);
        *pk    = k.release();
        return LUX_FHE_OK;
    });
}

LuxFheError lux_fhe_keygen_bootstrap(LuxFheContext* ctx, const LuxFheSecretKey* sk, LuxFheBootstrapKey** bsk) {
    if (!ctx || !sk || !bsk)
        return LUX_FHE_ERR_NULL_PTR;
    return guard(LUX_FHE_ERR_KEYGEN, [&] {
        ctx->cc.BTKeyGen(sk->sk);  // new key objects: the device reloads them on the next gate
        auto k       = std::make_unique<LuxFheBootstrapKey>();
        k->generated = true;
        *bsk         = k.release();
        return LUX_FHE_OK;
    });
}

void lux_fhe_secretkey_free(LuxFheSecretKey* sk) {
    delete sk;
}
void lux_fhe_publickey_free(LuxFhePublicKey* pk) {
    delete pk;
}
void lux_fhe_bootstrapkey_free(LuxFheBootstrapKey* bsk) {
    delete bsk;
}

// ---- encryption (c_api.h:153-183): plaintext modulus 4, FRESH, as c_api.cpp:160-200 ----
LuxFheError lux_fhe_encrypt(LuxFheContext* ctx, const LuxFheSecretKey* sk, bool plaintext, LuxFheCiphertext** ct) {
    if (!ctx || !sk || !ct)
        return LUX_FHE_ERR_NULL_PTR;
    return guard(LUX_FHE_ERR_ENCRYPT, [&] {
        auto c = std::make_unique<LuxFheCiphertext>();
        c->ct  = ctx->cc.Encrypt(sk->sk, plaintext ? 1 : 0, FRESH, 4);
        *ct    = c.release();
        return LUX_FHE_OK;
    });
}

LuxFheError lux_fhe_encrypt_pk(LuxFheContext* ctx, const LuxFhePublicKey* pk, bool plaintext, LuxFheCiphertext** ct) {
    if (!ctx || !pk || !ct)
        return LUX_FHE_ERR_NULL_PTR;
    return guard(LUX_FHE_ERR_ENCRYPT, [&] {
        auto c = std::make_unique<LuxFheCiphertext>();
        c->ct  = ctx->cc.Encrypt(pk->pk, plaintext ? 1 : 0, FRESH, 4);
        *ct    = c.release();
        return LUX_FHE_OK;
    });
}

LuxFheError lux_fhe_decrypt(LuxFheContext* ctx, const LuxFheSecretKey* sk, const LuxFheCiphertext* ct, bool* plaintext) {
    if (!ctx || !sk || !ct || !plaintext)
        return LUX_FHE_ERR_NULL_PTR;
    return guard(LUX_FHE_ERR_DECRYPT, [&] {
        LWEPlaintext m = 0;
        ctx->cc.Decrypt(sk->sk, ct->ct, &m, 4);
        *plaintext = m == 1;
        return LUX_FHE_OK;
    });
}

void lux_fhe_ciphertext_free(LuxFheCiphertext* ct) {
    delete ct;
}

LuxFheError lux_fhe_ciphertext_clone(const LuxFheCiphertext* src, LuxFheCiphertext** dst) {
    if (!src || !dst)
        return LUX_FHE_ERR_NULL_PTR;
    return guard(LUX_FHE_ERR_ALLOC, [&] {
        auto c = std::make_unique<LuxFheCiphertext>();
        c->ct  = src->ct;  // shares the immutable ciphertext object, as the reference does
        *dst   = c.release();
        return LUX_FHE_OK;
    });
}

// ---- gates (c_api.h:189-263) ----
LuxFheError lux_fhe_not(LuxFheContext* ctx, const LuxFheCiphertext* ct, LuxFheCiphertext** result) {
    if (!ctx || !ct || !result)
        return LUX_FHE_ERR_NULL_PTR;
    return guard(LUX_FHE_ERR_GATE, [&] {  // no bootstrapping: stays on the CPU
        auto r = std::make_unique<LuxFheCiphertext>();
        r->ct  = ctx->cc.EvalNOT(ct->ct);
        *result = r.release();
        return LUX_FHE_OK;
    });
}

#define FHE_AMD_CAPI_GATE(name, G)                                                                          \
    LuxFheError lux_fhe_##name(LuxFheContext* ctx, const LuxFheBootstrapKey* bsk, const LuxFheCiphertext* a, \
                               const LuxFheCiphertext* b, LuxFheCiphertext** result) {                      \
        if (!a || !b)                                                                                       \
            return LUX_FHE_ERR_NULL_PTR;                                                                    \
        return gate_batch(ctx, bsk, G, &a, &b, 1, result);                                                  \
    }
FHE_AMD_CAPI_GATE(and, AND)
FHE_AMD_CAPI_GATE(or, OR)
FHE_AMD_CAPI_GATE(xor, XOR)
FHE_AMD_CAPI_GATE(nand, NAND)
FHE_AMD_CAPI_GATE(nor, NOR)
FHE_AMD_CAPI_GATE(xnor, XNOR)
#undef FHE_AMD_CAPI_GATE

LuxFheError lux_fhe_mux(LuxFheContext* ctx, const LuxFheBootstrapKey* bsk, const LuxFheCiphertext* sel,
                        const LuxFheCiphertext* a, const LuxFheCiphertext* b, LuxFheCiphertext** result) {
    if (!sel || !a || !b)
        return LUX_FHE_ERR_NULL_PTR;
    return mux_batch(ctx, bsk, &sel, &a, &b, 1, result);
}

LuxFheError lux_fhe_bootstrap(LuxFheContext* ctx, const LuxFheBootstrapKey* bsk, const LuxFheCiphertext* ct,
                              LuxFheCiphertext** result) {
    if (!ct)
        return LUX_FHE_ERR_NULL_PTR;
    return bootstrap_batch(ctx, bsk, &ct, 1, result);
}

LuxFheError lux_fhe_gate_batch(LuxFheContext* ctx, const LuxFheBootstrapKey* bsk, LuxFheGate gate,
                               const LuxFheCiphertext* const* a, const LuxFheCiphertext* const* b, size_t count,
                               LuxFheCiphertext** result) {
    if (gate < LUX_FHE_GATE_OR || gate > LUX_FHE_GATE_XNOR)
        return LUX_FHE_ERR_INVALID_PARAM;
    return gate_batch(ctx, bsk, static_cast<BINGATE>(gate), a, b, count, result);
}

LuxFheError lux_fhe_mux_batch(LuxFheContext* ctx, const LuxFheBootstrapKey* bsk, const LuxFheCiphertext* const* sel,
                              const LuxFheCiphertext* const* a, const LuxFheCiphertext* const* b, size_t count,
                              LuxFheCiphertext** result) {
    return mux_batch(ctx, bsk, sel, a, b, count, result);
}

LuxFheError lux_fhe_bootstrap_batch(LuxFheContext* ctx, const LuxFheBootstrapKey* bsk,
                                    const LuxFheCiphertext* const* ct, size_t count, LuxFheCiphertext** result) {
    return bootstrap_batch(ctx, bsk, ct, count, result);
}

// ---- serialization (c_api.h:269-299): cereal BINARY, as the reference ----
LuxFheError lux_fhe_secretkey_marshal(const LuxFheSecretKey* sk, uint8_t** data, size_t* len) {
    if (!sk || !data || !len)
        return LUX_FHE_ERR_NULL_PTR;
    return marshal(sk->sk, data, len);
}

LuxFheError lux_fhe_secretkey_unmarshal(LuxFheContext* ctx, const uint8_t* data, size_t len, LuxFheSecretKey** sk) {
    if (!ctx || !data || !sk)
        return LUX_FHE_ERR_NULL_PTR;
    auto k           = std::make_unique<LuxFheSecretKey>();
    const auto rc    = unmarshal(data, len, k->sk);
    if (rc == LUX_FHE_OK)
        *sk = k.release();
    return rc;
}

LuxFheError lux_fhe_ciphertext_marshal(const LuxFheCiphertext* ct, uint8_t** data, size_t* len) {
    if (!ct || !data || !len)
        return LUX_FHE_ERR_NULL_PTR;
    return marshal(ct->ct, data, len);
}

LuxFheError lux_fhe_ciphertext_unmarshal(LuxFheContext* ctx, const uint8_t* data, size_t len, LuxFheCiphertext** ct) {
    if (!ctx || !data || !ct)
        return LUX_FHE_ERR_NULL_PTR;
    auto c        = std::make_unique<LuxFheCiphertext>();
    const auto rc = unmarshal(data, len, c->ct);
    if (rc == LUX_FHE_OK)
        *ct = c.release();
    return rc;
}

void lux_fhe_bytes_free(uint8_t* data) {
    delete[] data;
}

// ---- utility (c_api.h:305-318) ----
const char* lux_fhe_version(void) {
    return "1.4.2";
}

const char* lux_fhe_strerror(LuxFheError err) {
    switch (err) {
        case LUX_FHE_OK: return "ok";
        case LUX_FHE_ERR_NULL_PTR: return "null pointer";
        case LUX_FHE_ERR_INVALID_PARAM: return "invalid parameter";
        case LUX_FHE_ERR_ALLOC: return "allocation failed";
        case LUX_FHE_ERR_KEYGEN: return "key generation failed";
        case LUX_FHE_ERR_ENCRYPT: return "encryption failed";
        case LUX_FHE_ERR_DECRYPT: return "decryption failed";
        case LUX_FHE_ERR_BOOTSTRAP: return "bootstrap failed";
        case LUX_FHE_ERR_GATE: return "gate evaluation failed";
        case LUX_FHE_ERR_SERIALIZE: return "serialization failed";
        case LUX_FHE_ERR_DESERIALIZE: return "deserialization failed";
        case LUX_FHE_ERR_NOT_INIT: return "not initialized";
    }
    return "unknown error";
}

// a HIP device is visible (the reference reports its compile-time GPU backends, c_api.cpp:343-349)
bool lux_fhe_has_gpu(void) {
    int n = 0;
    return fhe_hip_device_count(&n) == FHE_HIP_OK && n > 0;
}

}  // extern "C"
