// capi.cpp -- extern "C" boundary (include/fhe_hip.h).  No exception crosses it.
#include <hip/hip_runtime.h>

#include <string.h>

#include <exception>
#include <new>
#include <string>
#include <vector>
#include <algorithm>

#include "../../include/fhe_hip.h"
#include "engine.h"
#include "packed.h"
#include "cereal.h"
#include "multi.h"
#include "keygen.h"
#include "ntt.h"
#include "boot.h"

using namespace fhe_amd;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
int hip_fail(hipError_t e, const char* what) {
    return fail(FHE_HIP_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}
template <typename F>
int guarded(F&& f) {
    try {
        return f();
    } catch (const HipError& e) {
        return fail(FHE_HIP_ERR_DEVICE, e.what());
    } catch (const std::logic_error& e) {
        if (dynamic_cast<const std::invalid_argument*>(&e)) return fail(FHE_HIP_ERR_INVALID_PARAM, e.what());
        return fail(FHE_HIP_ERR_NOT_INIT, e.what());
    } catch (const std::bad_alloc&) {
        return fail(FHE_HIP_ERR_ALLOC, "host allocation failed");
    } catch (const std::exception& e) {
        return fail(FHE_HIP_ERR_INVALID_PARAM, e.what());
    } catch (...) {
        return fail(FHE_HIP_ERR_INVALID_PARAM, "unknown exception");
    }
}
}  // namespace

// A context's device scratch for its synchronous host-buffer calls (seam BlindRotate / ExternalProduct):
// grow-only, owned by the context, reused by every such call (each ends with a stream synchronize).
// Round 4 replaced a stream-ordered pool allocation (hipMallocAsync / hipFreeAsync per call): after a few
// such calls on one context, a block handed out again read back as zeros right after the kernel that
// wrote it had finished (tests/test_backend.py, std192_lmkcdey null accumulators).
struct fhe_hip_ctx {
    Engine eng;
    uint64_t* scr = nullptr;
    size_t scr_bytes = 0;
    fhe_hip_ctx(int ps, int m, int dev) : eng(ps, m, dev) {}
    ~fhe_hip_ctx() {
        if (scr) {
            (void)hipSetDevice(eng.device());
            (void)hipFree(scr);
        }
    }
    uint64_t* scratch(size_t bytes, hipStream_t s) {
        FHE_HIP_CHECK(hipSetDevice(eng.device()));
        if (bytes > scr_bytes) {
            FHE_HIP_CHECK(hipStreamSynchronize(s));
            if (scr) FHE_HIP_CHECK(hipFree(scr));
            scr = nullptr;
            scr_bytes = 0;
            FHE_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&scr), bytes));
            scr_bytes = bytes;
        }
        return scr;
    }
};

static void fill_params(const Params& p, fhe_hip_params* o) {
    o->paramset = p.paramset; o->method = p.method; o->n = p.n; o->N = p.N; o->q = p.q; o->qKS = p.qKS;
    o->kernel = Engine::kernel_kind(p);
    o->baseKS = p.baseKS; o->digitsKS = p.digitsKS; o->baseG = p.baseG; o->digitsG = p.digitsG;
    o->numAutoKeys = p.numAutoKeys; o->keyDist = p.keyDist; o->Q = p.Q; o->psi = p.psi;
    o->bsk_words = p.bsk_words(); o->ksk_rows = p.ksk_rows_all();
}

// The stream a context's call runs on: the caller's (or the context's own).  A context has one
// workspace, so a call on a different stream than the previous call first waits for that
// stream's work (Engine::use_stream): calls on one context are always ordered.
static hipStream_t ctx_stream(fhe_hip_ctx* ctx, void* stream) {
    return ctx->eng.use_stream(static_cast<hipStream_t>(stream));
}

// An asynchronous call's stream and its ordering point: the event a later call on another stream
// waits for is recorded when the call's scope ends, on every exit path (work may have been enqueued
// before an exception)
struct CallOrder {
    Engine& eng;
    hipStream_t s;
    CallOrder(fhe_hip_ctx* ctx, void* stream) : eng(ctx->eng), s(ctx_stream(ctx, stream)) {}
    ~CallOrder() {
        try {
            eng.end_call(s);
        } catch (...) {
        }
    }
    CallOrder(const CallOrder&) = delete;
    CallOrder& operator=(const CallOrder&) = delete;
};

struct fhe_hip_multi {
    MultiEngine eng;
    fhe_hip_multi(int ps, int m, const int* d, int n) : eng(ps, m, d, n) {}
};

struct fhe_hip_ntt_plan {
    NttPlan plan;
    hipStream_t stream = nullptr;
    uint64_t* d_buf    = nullptr;
    size_t cap         = 0;
};

extern "C" {

const char* fhe_hip_last_error(void) { return g_err.c_str(); }

int fhe_hip_device_count(int* count) {
    if (!count) return fail(FHE_HIP_ERR_NULL_PTR, "count is null");
    hipError_t e = hipGetDeviceCount(count);
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
    return FHE_HIP_OK;
}

int fhe_hip_alloc(int device, size_t bytes, void** d_ptr) {
    if (!d_ptr) return fail(FHE_HIP_ERR_NULL_PTR, "d_ptr is null");
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    e = hipMalloc(d_ptr, bytes);
    if (e != hipSuccess) return fail(FHE_HIP_ERR_ALLOC, std::string("hipMalloc: ") + hipGetErrorString(e));
    return FHE_HIP_OK;
}

int fhe_hip_free(void* d_ptr) {
    hipError_t e = hipFree(d_ptr);
    return e == hipSuccess ? FHE_HIP_OK : hip_fail(e, "hipFree");
}

int fhe_hip_copy_to_device(void* d_dst, const void* h_src, size_t bytes) {
    if (!d_dst || !h_src) return fail(FHE_HIP_ERR_NULL_PTR, "null pointer");
    hipError_t e = hipMemcpy(d_dst, h_src, bytes, hipMemcpyHostToDevice);
    return e == hipSuccess ? FHE_HIP_OK : hip_fail(e, "hipMemcpy H2D");
}

int fhe_hip_copy_to_host(void* h_dst, const void* d_src, size_t bytes) {
    if (!d_src || !h_dst) return fail(FHE_HIP_ERR_NULL_PTR, "null pointer");
    hipError_t e = hipMemcpy(h_dst, d_src, bytes, hipMemcpyDeviceToHost);
    return e == hipSuccess ? FHE_HIP_OK : hip_fail(e, "hipMemcpy D2H");
}

int fhe_hip_synchronize(int device) {
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    return e == hipSuccess ? FHE_HIP_OK : hip_fail(e, "hipDeviceSynchronize");
}

int fhe_hip_ntt_plan_create(uint64_t Q, uint64_t psi, uint32_t N, int device, fhe_hip_ntt_plan** out,
                            uint64_t* psi_out) {
    return guarded([&]() -> int {
        if (!out) return fail(FHE_HIP_ERR_NULL_PTR, "out is null");
        *out   = nullptr;
        auto* p = new fhe_hip_ntt_plan();
        hipError_t e = ntt_plan_init(p->plan, Q, psi, N, device);
        if (e == hipErrorInvalidValue) {
            delete p;
            return fail(FHE_HIP_ERR_INVALID_PARAM, "invalid NTT parameters (need N=1024, prime Q=1 mod 2N, Q<2^62, "
                                                   "psi a primitive 2N-th root)");
        }
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            ntt_plan_free(p->plan);
            delete p;
            return hip_fail(e, "ntt plan init");
        }
        if (psi_out) *psi_out = p->plan.psi;
        *out = p;
        return FHE_HIP_OK;
    });
}

void fhe_hip_ntt_plan_destroy(fhe_hip_ntt_plan* p) {
    if (!p) return;
    (void)hipSetDevice(p->plan.device);
    if (p->d_buf) (void)hipFree(p->d_buf);
    if (p->stream) (void)hipStreamDestroy(p->stream);
    ntt_plan_free(p->plan);
    delete p;
}

void* fhe_hip_ntt_plan_stream(fhe_hip_ntt_plan* p) { return p ? (void*)p->stream : nullptr; }

int fhe_hip_ntt_batch_device(fhe_hip_ntt_plan* p, const uint64_t* d_in, uint64_t* d_out, size_t count, int inverse,
                             void* stream) {
    if (!p || (!d_in && count) || (!d_out && count)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    if (count > 0xffffffffull) return fail(FHE_HIP_ERR_INVALID_PARAM, "count too large");
    hipError_t e = hipSetDevice(p->plan.device);
    if (e == hipSuccess)
        e = ntt1024_launch(p->plan, d_in, d_out, (uint32_t)count, inverse != 0,
                           stream ? (hipStream_t)stream : p->stream);
    return e == hipSuccess ? FHE_HIP_OK : hip_fail(e, "ntt launch");
}

int fhe_hip_ntt_batch(fhe_hip_ntt_plan* p, uint64_t* polys, size_t count, int inverse) {
    if (!p || (!polys && count)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    if (count == 0) return FHE_HIP_OK;
    hipError_t e = hipSetDevice(p->plan.device);
    const size_t bytes = count * p->plan.N * sizeof(uint64_t);
    if (e == hipSuccess && bytes > p->cap) {
        if (p->d_buf) (void)hipFree(p->d_buf);
        p->d_buf = nullptr;
        p->cap   = 0;
        e        = hipMalloc(&p->d_buf, bytes);
        if (e == hipSuccess) p->cap = bytes;
    }
    if (e == hipSuccess) e = hipMemcpyAsync(p->d_buf, polys, bytes, hipMemcpyHostToDevice, p->stream);
    if (e == hipSuccess) e = ntt1024_launch(p->plan, p->d_buf, p->d_buf, (uint32_t)count, inverse != 0, p->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(polys, p->d_buf, bytes, hipMemcpyDeviceToHost, p->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
    return e == hipSuccess ? FHE_HIP_OK : hip_fail(e, "ntt batch");
}

int fhe_hip_params_get(int paramset, int method, fhe_hip_params* out) {
    return guarded([&]() -> int {
        if (!out) return fail(FHE_HIP_ERR_NULL_PTR, "out is null");
        fill_params(make_params(paramset, method), out);
        return FHE_HIP_OK;
    });
}

int fhe_hip_create(int paramset, int method, int device, fhe_hip_ctx** out) {
    return guarded([&]() -> int {
        if (!out) return fail(FHE_HIP_ERR_NULL_PTR, "out is null");
        *out = nullptr;
        *out = new fhe_hip_ctx(paramset, method, device);
        return FHE_HIP_OK;
    });
}

void fhe_hip_destroy(fhe_hip_ctx* ctx) {
    try {
        delete ctx;
    } catch (...) {
    }
}

int fhe_hip_get_params(const fhe_hip_ctx* ctx, fhe_hip_params* out) {
    if (!ctx || !out) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    fill_params(ctx->eng.params(), out);
    out->kernel = ctx->eng.kernel();  // what this context runs (its own kernel flags, read at creation)
    return FHE_HIP_OK;
}

int fhe_hip_gate_kernel(const fhe_hip_ctx* ctx, size_t count, const char** name) {
    if (!ctx || !name) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        *name = ctx->eng.gate_kernel(count);
        return FHE_HIP_OK;
    });
}

void* fhe_hip_stream(fhe_hip_ctx* ctx) { return ctx ? (void*)ctx->eng.stream() : nullptr; }

int fhe_hip_load_bsk(fhe_hip_ctx* ctx, const uint64_t* bsk, size_t n_words) {
    if (!ctx || !bsk) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int { ctx->eng.load_bsk(bsk, n_words); return FHE_HIP_OK; });
}

int fhe_hip_load_ksk(fhe_hip_ctx* ctx, const uint64_t* A, size_t nA, const uint64_t* B, size_t nB) {
    if (!ctx || !A || !B) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int { ctx->eng.load_ksk(A, nA, B, nB); return FHE_HIP_OK; });
}

int fhe_hip_btkeygen_device(fhe_hip_ctx* ctx, const uint64_t* sk, size_t n, uint64_t seed, uint64_t* bsk,
                            uint64_t* kskA, uint64_t* kskB) {
    if (!ctx || !sk) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int { ctx->eng.keygen_device(sk, n, seed, bsk, kskA, kskB); return FHE_HIP_OK; });
}

static bool io_ok(size_t count, const void* a, const void* b, const void* c, const void* d, const void* e,
                  const void* f) {
    return count == 0 || (a && b && c && d && e && f);
}

// ---- packed transfer format (reference backend/packed.h) ----
int fhe_hip_pack_lwe_batch(uint32_t n, size_t count, const uint64_t* a, const uint64_t* b, uint32_t flags,
                           uint8_t* out, size_t capacity, size_t* size) {
    if (!size || (count && (!a || !b))) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        *size = packed_lwe_batch_size(n, count);
        if (!out) return FHE_HIP_OK;
        if (capacity < *size) return fail(FHE_HIP_ERR_INVALID_PARAM, "output buffer too small");
        pack_lwe_batch(n, count, a, b, flags, out);
        return FHE_HIP_OK;
    });
}

int fhe_hip_unpack_lwe_batch(const uint8_t* data, size_t size, uint32_t* n, size_t* count, uint64_t* a, uint64_t* b) {
    if (!data || !n || !count) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        unpack_lwe_batch(data, size, n, count, a, b);
        return FHE_HIP_OK;
    });
}

int fhe_hip_eval_bingate_packed(fhe_hip_ctx* ctx, int gate, const uint8_t* in1, size_t size1, const uint8_t* in2,
                                size_t size2, uint32_t out_flags, uint8_t* out, size_t capacity, size_t* size) {
    if (!ctx || !in1 || !in2 || !size) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        uint32_t n1, n2;
        size_t c1, c2;
        unpack_lwe_batch(in1, size1, &n1, &c1, nullptr, nullptr);
        unpack_lwe_batch(in2, size2, &n2, &c2, nullptr, nullptr);
        const uint32_t n = ctx->eng.params().n;
        if (n1 != n || n2 != n) return fail(FHE_HIP_ERR_INVALID_PARAM, "packed batch dimension != n");
        if (c1 != c2) return fail(FHE_HIP_ERR_INVALID_PARAM, "packed batches differ in size");
        *size = packed_lwe_batch_size(n, c1);
        if (!out) return FHE_HIP_OK;
        if (capacity < *size) return fail(FHE_HIP_ERR_INVALID_PARAM, "output buffer too small");
        std::vector<uint64_t> a1(c1 * n), b1(c1), a2(c1 * n), b2(c1), ao(c1 * n), bo(c1);
        unpack_lwe_batch(in1, size1, &n1, &c1, a1.data(), b1.data());
        unpack_lwe_batch(in2, size2, &n2, &c2, a2.data(), b2.data());
        ctx_stream(ctx, nullptr);
        ctx->eng.eval_gate_host(gate, c1, a1.data(), b1.data(), a2.data(), b2.data(), ao.data(), bo.data());
        pack_lwe_batch(n, c1, ao.data(), bo.data(), out_flags, out);
        return FHE_HIP_OK;
    });
}

int fhe_hip_pack_keys(int paramset, int method, const uint64_t* bsk, size_t bsk_words, const uint64_t* A,
                      const uint64_t* B, uint8_t* bsk_out, size_t bsk_cap, size_t* bsk_size, uint8_t* ksk_out,
                      size_t ksk_cap, size_t* ksk_size) {
    if (!bsk_size || !ksk_size) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        const Params p = make_params(paramset, method);
        *bsk_size = sizeof(PackedBskHdr) + p.bsk_words() * 8;
        *ksk_size = sizeof(PackedKskHdr) + p.ksk_rows_all() * ((size_t)p.n + 1) * 8;
        if (bsk_out) {
            if (!bsk || bsk_cap < *bsk_size) return fail(FHE_HIP_ERR_INVALID_PARAM, "bsk buffer missing or too small");
            auto v = pack_bsk(p, bsk, bsk_words);
            memcpy(bsk_out, v.data(), v.size());
        }
        if (ksk_out) {
            if (!A || !B || ksk_cap < *ksk_size) return fail(FHE_HIP_ERR_INVALID_PARAM, "ksk buffer missing or too small");
            auto v = pack_ksk(p, A, B);
            memcpy(ksk_out, v.data(), v.size());
        }
        return FHE_HIP_OK;
    });
}

int fhe_hip_load_keys_packed(fhe_hip_ctx* ctx, const uint8_t* bsk, size_t bsk_size, const uint8_t* ksk,
                             size_t ksk_size) {
    if (!ctx || !bsk || !ksk) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        const Params& p = ctx->eng.params();
        size_t words = 0;
        const uint64_t* raw = unpack_bsk(p, bsk, bsk_size, &words);
        const uint64_t *A = nullptr, *B = nullptr;
        unpack_ksk(p, ksk, ksk_size, &A, &B);
        ctx->eng.load_bsk(raw, words);
        ctx->eng.load_ksk(A, p.ksk_rows_all() * p.n, B, p.ksk_rows_all());
        return FHE_HIP_OK;
    });
}

static int emit_bytes(const std::string& v, uint8_t* out, size_t cap, size_t* size) {
    *size = v.size();
    if (out) {
        if (cap < v.size()) return fail(FHE_HIP_ERR_INVALID_PARAM, "output buffer too small");
        memcpy(out, v.data(), v.size());
    }
    return FHE_HIP_OK;
}

int fhe_hip_copy_keys(fhe_hip_ctx* dst, const fhe_hip_ctx* src) {
    if (!dst || !src) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    if (dst == src) return FHE_HIP_OK;
    return guarded([&]() -> int {
        dst->eng.copy_keys_from(src->eng);
        return FHE_HIP_OK;
    });
}

int fhe_hip_load_keys_cereal(fhe_hip_ctx* ctx, const uint8_t* refresh, size_t refresh_size, const uint8_t* sw,
                             size_t sw_size) {
    if (!ctx || !refresh || !sw) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        const Params& p = ctx->eng.params();
        std::vector<uint64_t> bsk, A, B;
        cereal_read_bsk(p, refresh, refresh_size, bsk);
        cereal_read_ksk(p, sw, sw_size, A, B);
        ctx->eng.load_bsk(bsk.data(), bsk.size());
        ctx->eng.load_ksk(A.data(), A.size(), B.data(), B.size());
        return FHE_HIP_OK;
    });
}

int fhe_hip_cereal_read_keys(int paramset, int method, const uint8_t* refresh, size_t refresh_size, const uint8_t* sw,
                             size_t sw_size, uint64_t* bsk, uint64_t* kskA, uint64_t* kskB) {
    if (!refresh || !sw || !bsk || !kskA || !kskB) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        const Params p = make_params(paramset, method);
        std::vector<uint64_t> b, A, B;
        cereal_read_bsk(p, refresh, refresh_size, b);
        cereal_read_ksk(p, sw, sw_size, A, B);
        std::copy(b.begin(), b.end(), bsk);
        std::copy(A.begin(), A.end(), kskA);
        std::copy(B.begin(), B.end(), kskB);
        return FHE_HIP_OK;
    });
}

int fhe_hip_cereal_write_keys(int paramset, int method, const uint64_t* bsk, size_t bsk_words, const uint64_t* kskA,
                              const uint64_t* kskB, uint8_t* refresh_out, size_t refresh_cap, size_t* refresh_size,
                              uint8_t* sw_out, size_t sw_cap, size_t* sw_size) {
    if (!bsk || !kskA || !kskB || !refresh_size || !sw_size) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        const Params p = make_params(paramset, method);
        if (bsk_words != p.bsk_words()) return fail(FHE_HIP_ERR_INVALID_PARAM, "bsk has wrong length");
        int rc = emit_bytes(cereal_write_bsk(p, bsk), refresh_out, refresh_cap, refresh_size);
        if (rc) return rc;
        return emit_bytes(cereal_write_ksk(p, kskA, kskB), sw_out, sw_cap, sw_size);
    });
}

int fhe_hip_cereal_read_lwe(const uint8_t* data, size_t size, int is_key, uint64_t* a, uint32_t cap_n, uint32_t* n,
                            uint64_t* b, uint64_t* mod) {
    if (!data || !n || !mod) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        CerealLwe v = cereal_read_lwe(data, size, is_key != 0);
        *n = (uint32_t)v.a.size();
        *mod = v.mod;
        if (b) *b = v.b;
        if (a) {
            if (cap_n < v.a.size()) return fail(FHE_HIP_ERR_INVALID_PARAM, "output buffer too small");
            std::copy(v.a.begin(), v.a.end(), a);
        }
        return FHE_HIP_OK;
    });
}

int fhe_hip_cereal_write_lwe(const uint64_t* a, uint32_t n, uint64_t b, uint64_t mod, int is_key, uint8_t* out,
                             size_t cap, size_t* size) {
    if ((!a && n) || !size) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int { return emit_bytes(cereal_write_lwe(a, n, b, mod, is_key != 0), out, cap, size); });
}

static void context_row(const uint8_t* data, size_t size, int& paramset, int& method) {
    if (!cereal_context_paramset(cereal_read_context(data, size), paramset, method))
        throw std::invalid_argument("cryptoContext archive: its parameters match no supported parameter set");
}

int fhe_hip_cereal_read_context(const uint8_t* data, size_t size, int* paramset, int* method, fhe_hip_params* out) {
    if (!data || !paramset || !method) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        context_row(data, size, *paramset, *method);
        if (out) fill_params(make_params(*paramset, *method), out);
        return FHE_HIP_OK;
    });
}

int fhe_hip_cereal_write_context(int paramset, int method, uint8_t* out, size_t cap, size_t* size) {
    if (!size) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        if (!is_large(paramset) && !method_compatible(paramset, method))
            return fail(FHE_HIP_ERR_INVALID_PARAM, "Specified BINFHE_METHOD and BINFHE_PARAMSET are incompatible");
        return emit_bytes(cereal_write_context(make_params(paramset, method)), out, cap, size);
    });
}

int fhe_hip_create_from_cereal(const uint8_t* data, size_t size, int device, fhe_hip_ctx** out) {
    if (!data || !out) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        *out = nullptr;
        int ps = 0, m = 0;
        context_row(data, size, ps, m);
        *out = new fhe_hip_ctx(ps, m, device);
        return FHE_HIP_OK;
    });
}

int fhe_hip_eval_bingate_batch(fhe_hip_ctx* ctx, int gate, size_t count, const uint64_t* a1, const uint64_t* b1,
                               const uint64_t* a2, const uint64_t* b2, uint64_t* a_out, uint64_t* b_out) {
    if (!ctx || !io_ok(count, a1, b1, a2, b2, a_out, b_out)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        ctx_stream(ctx, nullptr);
        ctx->eng.eval_gate_host(gate, count, a1, b1, a2, b2, a_out, b_out);
        return FHE_HIP_OK;
    });
}

int fhe_hip_eval_bingate_batch_device(fhe_hip_ctx* ctx, int gate, size_t count, const uint64_t* d_a1,
                                      const uint64_t* d_b1, const uint64_t* d_a2, const uint64_t* d_b2,
                                      uint64_t* d_a_out, uint64_t* d_b_out, void* stream) {
    if (!ctx || !io_ok(count, d_a1, d_b1, d_a2, d_b2, d_a_out, d_b_out))
        return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        const CallOrder order(ctx, stream);
        const hipStream_t s = order.s;
        ctx->eng.eval_gate_device(gate, count, d_a1, d_b1, d_a2, d_b2, d_a_out, d_b_out,
                                  s);
        return FHE_HIP_OK;
    });
}

int fhe_hip_blind_rotate_batch_device(fhe_hip_ctx* ctx, int gate, size_t count, const uint64_t* d_a1,
                                      const uint64_t* d_b1, const uint64_t* d_a2, const uint64_t* d_b2, void* stream) {
    if (!ctx || !io_ok(count, d_a1, d_b1, d_a2, d_b2, d_a1, d_b1)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        const CallOrder order(ctx, stream);
        const hipStream_t s = order.s;
        ctx->eng.bootstrap_device(gate, count, d_a1, d_b1, d_a2, d_b2, true,
                                  s);
        return FHE_HIP_OK;
    });
}

int fhe_hip_keyswitch_workspace_device(fhe_hip_ctx* ctx, size_t count, uint64_t* d_a_out, uint64_t* d_b_out,
                                       void* stream) {
    if (!ctx || (count && (!d_a_out || !d_b_out))) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        const CallOrder order(ctx, stream);
        const hipStream_t s = order.s;
        ctx->eng.keyswitch_workspace_device(count, d_a_out, d_b_out,
                                            s);
        return FHE_HIP_OK;
    });
}

int fhe_hip_eval_bingate_extended(fhe_hip_ctx* ctx, int gate, size_t count, const uint64_t* a1, const uint64_t* b1,
                                  const uint64_t* a2, const uint64_t* b2, uint64_t* ext_a, uint64_t* ext_b) {
    if (!ctx || !io_ok(count, a1, b1, a2, b2, ext_a, ext_b)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        ctx_stream(ctx, nullptr);
        ctx->eng.bootstrap_extended_host(gate, count, a1, b1, a2, b2, ext_a, ext_b);
        return FHE_HIP_OK;
    });
}

int fhe_hip_eval_gate_multi_batch(fhe_hip_ctx* ctx, int gate, uint32_t k, uint32_t ptmod, size_t count,
                                  const uint64_t* const* a_in, const uint64_t* const* b_in, uint64_t* a_out,
                                  uint64_t* b_out, int extended) {
    if (!ctx || (count && (!a_in || !b_in || !a_out || !b_out))) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    if (k < 2 || k > 4) return fail(FHE_HIP_ERR_INVALID_PARAM, "k must be 2..4");
    return guarded([&]() -> int {
        ctx_stream(ctx, nullptr);
        ctx->eng.eval_gate_multi_host(gate, count, k, a_in, b_in, ptmod, a_out, b_out, extended != 0);
        return FHE_HIP_OK;
    });
}

int fhe_hip_eval_gate_multi_batch_device(fhe_hip_ctx* ctx, int gate, uint32_t k, uint32_t ptmod, size_t count,
                                         const uint64_t* const* d_a_in, const uint64_t* const* d_b_in,
                                         uint64_t* d_a_out, uint64_t* d_b_out, void* stream) {
    if (!ctx || (count && (!d_a_in || !d_b_in || !d_a_out || !d_b_out)))
        return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    if (k < 2 || k > 4) return fail(FHE_HIP_ERR_INVALID_PARAM, "k must be 2..4");
    return guarded([&]() -> int {
        const CallOrder order(ctx, stream);
        const hipStream_t s = order.s;
        ctx->eng.eval_gate_multi_device(gate, count, k, d_a_in, d_b_in, ptmod, d_a_out, d_b_out,
                                        s);
        return FHE_HIP_OK;
    });
}

int fhe_hip_eval_cmux_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a0, const uint64_t* b0,
                            const uint64_t* a1, const uint64_t* b1, const uint64_t* a2, const uint64_t* b2,
                            uint64_t* a_out, uint64_t* b_out) {
    if (!ctx || !io_ok(count, a0, b0, a1, b1, a_out, b_out) || (count && (!a2 || !b2)))
        return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        ctx_stream(ctx, nullptr);
        ctx->eng.eval_cmux_host(count, a0, b0, a1, b1, a2, b2, a_out, b_out);
        return FHE_HIP_OK;
    });
}

int fhe_hip_eval_cmux_batch_device(fhe_hip_ctx* ctx, size_t count, const uint64_t* d_a0, const uint64_t* d_b0,
                                   const uint64_t* d_a1, const uint64_t* d_b1, const uint64_t* d_a2,
                                   const uint64_t* d_b2, uint64_t* d_a_out, uint64_t* d_b_out, void* stream) {
    if (!ctx || !io_ok(count, d_a0, d_b0, d_a1, d_b1, d_a_out, d_b_out) || (count && (!d_a2 || !d_b2)))
        return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        const CallOrder order(ctx, stream);
        const hipStream_t s = order.s;
        ctx->eng.eval_cmux_device(count, d_a0, d_b0, d_a1, d_b1, d_a2, d_b2, d_a_out, d_b_out,
                                  s);
        return FHE_HIP_OK;
    });
}

int fhe_hip_bootstrap_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b, uint64_t* a_out,
                            uint64_t* b_out) {
    if (!ctx || !io_ok(count, a, b, a_out, b_out, a, b)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        ctx_stream(ctx, nullptr);
        ctx->eng.refresh_host(count, a, b, a_out, b_out);
        return FHE_HIP_OK;
    });
}

int fhe_hip_bootstrap_batch_device(fhe_hip_ctx* ctx, size_t count, const uint64_t* d_a, const uint64_t* d_b,
                                   uint64_t* d_a_out, uint64_t* d_b_out, void* stream) {
    if (!ctx || !io_ok(count, d_a, d_b, d_a_out, d_b_out, d_a, d_b)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        const CallOrder order(ctx, stream);
        ctx->eng.refresh_device(count, d_a, d_b, d_a_out, d_b_out, order.s);
        return FHE_HIP_OK;
    });
}

int fhe_hip_switch_to_qn_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b, uint64_t* a_out,
                               uint64_t* b_out) {
    if (!ctx || !io_ok(count, a, b, a_out, b_out, a, b)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        ctx_stream(ctx, nullptr);
        ctx->eng.switch_to_qn_host(count, a, b, a_out, b_out);
        return FHE_HIP_OK;
    });
}

int fhe_hip_switch_to_qn_batch_device(fhe_hip_ctx* ctx, size_t count, const uint64_t* d_a, const uint64_t* d_b,
                                      uint64_t* d_a_out, uint64_t* d_b_out, void* stream) {
    if (!ctx || !io_ok(count, d_a, d_b, d_a_out, d_b_out, d_a, d_b)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        const CallOrder order(ctx, stream);
        ctx->eng.switch_to_qn_device(count, d_a, d_b, d_a_out, d_b_out, order.s);
        return FHE_HIP_OK;
    });
}

static bool mixed_args_ok(uint32_t k, size_t count, const uint64_t* const* a_in, const uint64_t* const* b_in,
                          const uint64_t* a_out, const uint64_t* b_out) {
    if (!count) return true;
    if (!a_in || !b_in || !a_out || !b_out) return false;
    for (uint32_t j = 0; j < k && j < 4; ++j)
        if (!a_in[j] || !b_in[j]) return false;
    return true;
}
// the column count of the mixed entry points: 1..4 (Bootstrap 1, 2-input gates 2, AND3 / OR3 / MAJORITY /
// CMUX 3, AND4 / OR4 4); reported apart from null pointers
#define FHE_MIXED_K_CHECK(k)                                                                          \
    if ((k) < 1 || (k) > 4) return fail(FHE_HIP_ERR_INVALID_PARAM, "k: 1 to 4 input columns")

int fhe_hip_eval_mixed_batch(fhe_hip_ctx* ctx, int op, uint32_t k, uint32_t ptmod, size_t count,
                             const uint64_t* const* a_in, const uint64_t* const* b_in, const uint8_t* const* large,
                             uint64_t* a_out, uint64_t* b_out, int extended) {
    FHE_MIXED_K_CHECK(k);
    if (!ctx || !mixed_args_ok(k, count, a_in, b_in, a_out, b_out)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        ctx_stream(ctx, nullptr);
        ctx->eng.eval_mixed_host(op, k, ptmod, count, a_in, b_in, large, a_out, b_out, extended != 0);
        return FHE_HIP_OK;
    });
}

int fhe_hip_eval_mixed_batch_device(fhe_hip_ctx* ctx, int op, uint32_t k, uint32_t ptmod, size_t count,
                                    const uint64_t* const* d_a_in, const uint64_t* const* d_b_in,
                                    const uint8_t* const* d_large, uint64_t* d_a_out, uint64_t* d_b_out, int extended,
                                    void* stream) {
    FHE_MIXED_K_CHECK(k);
    if (!ctx || !mixed_args_ok(k, count, d_a_in, d_b_in, d_a_out, d_b_out))
        return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        const CallOrder order(ctx, stream);
        ctx->eng.eval_mixed_device(op, k, ptmod, count, d_a_in, d_b_in, d_large, d_a_out, d_b_out, extended != 0,
                                   order.s);
        return FHE_HIP_OK;
    });
}

// ---- the Backend seam (backend.h:73-247) ----
int fhe_hip_blind_rotate_acc_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, uint64_t ctmod, uint64_t* acc) {
    if (!ctx || (count && (!a || !acc))) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    if (ctmod == 0 || ctmod > 0xffffffffull) return fail(FHE_HIP_ERR_INVALID_PARAM, "bad ciphertext modulus");
    return guarded([&]() -> int {
        if (count == 0) return FHE_HIP_OK;
        const Params& p = ctx->eng.params();
        const size_t aw = count * p.n, accw = count * 2 * (size_t)p.N;
        for (size_t i = 0; i < aw; ++i)
            if (a[i] >= ctmod) return fail(FHE_HIP_ERR_INVALID_PARAM, "a not reduced mod the ciphertext modulus");
        for (size_t i = 0; i < accw; ++i)
            if (acc[i] >= p.Q) return fail(FHE_HIP_ERR_INVALID_PARAM, "accumulator not reduced mod Q");
        hipStream_t s = ctx_stream(ctx, nullptr);
        uint64_t* d = ctx->scratch((aw + accw) * 8, s);
        FHE_HIP_CHECK(hipMemcpyAsync(d, a, aw * 8, hipMemcpyHostToDevice, s));
        FHE_HIP_CHECK(hipMemcpyAsync(d + aw, acc, accw * 8, hipMemcpyHostToDevice, s));
        ctx->eng.blind_rotate_acc_device(count, d, (uint32_t)ctmod, d + aw, s);
        FHE_HIP_CHECK(hipMemcpyAsync(acc, d + aw, accw * 8, hipMemcpyDeviceToHost, s));
        FHE_HIP_CHECK(hipStreamSynchronize(s));
        return FHE_HIP_OK;
    });
}

int fhe_hip_blind_rotate_acc_batch_device(fhe_hip_ctx* ctx, size_t count, const uint64_t* d_a, uint64_t ctmod,
                                          uint64_t* d_acc, void* stream) {
    if (!ctx || (count && (!d_a || !d_acc))) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    if (ctmod == 0 || ctmod > 0xffffffffull) return fail(FHE_HIP_ERR_INVALID_PARAM, "bad ciphertext modulus");
    return guarded([&]() -> int {
        const CallOrder order(ctx, stream);
        const hipStream_t s = order.s;
        ctx->eng.blind_rotate_acc_device(count, d_a, (uint32_t)ctmod, d_acc, s);
        return FHE_HIP_OK;
    });
}

int fhe_hip_blind_rotate_init_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b,
                                    uint64_t* acc) {
    if (!ctx || (count && (!a || !b || !acc))) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        if (count == 0) return FHE_HIP_OK;
        const Params& p = ctx->eng.params();
        const size_t aw = count * p.n, accw = count * 2 * (size_t)p.N;
        for (size_t i = 0; i < aw; ++i)
            if (a[i] >= p.q) return fail(FHE_HIP_ERR_INVALID_PARAM, "a not reduced mod q");
        for (size_t i = 0; i < count; ++i)
            if (b[i] >= p.q) return fail(FHE_HIP_ERR_INVALID_PARAM, "b not reduced mod q");
        hipStream_t s = ctx_stream(ctx, nullptr);
        uint64_t* d = ctx->scratch((aw + count + accw) * 8, s);
        FHE_HIP_CHECK(hipMemcpyAsync(d, a, aw * 8, hipMemcpyHostToDevice, s));
        FHE_HIP_CHECK(hipMemcpyAsync(d + aw, b, count * 8, hipMemcpyHostToDevice, s));
        ctx->eng.blind_rotate_init_device(count, d, d + aw, d + aw + count, s);
        FHE_HIP_CHECK(hipMemcpyAsync(acc, d + aw + count, accw * 8, hipMemcpyDeviceToHost, s));
        FHE_HIP_CHECK(hipStreamSynchronize(s));
        return FHE_HIP_OK;
    });
}

int fhe_hip_blind_rotate_init_batch_device(fhe_hip_ctx* ctx, size_t count, const uint64_t* d_a, const uint64_t* d_b,
                                           uint64_t* d_acc, void* stream) {
    if (!ctx || (count && (!d_a || !d_b || !d_acc))) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        const CallOrder order(ctx, stream);
        ctx->eng.blind_rotate_init_device(count, d_a, d_b, d_acc, order.s);
        return FHE_HIP_OK;
    });
}

int fhe_hip_external_product_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* rgsw, const uint64_t* rlwe,
                                   uint64_t* result) {
    if (!ctx || (count && (!rgsw || !rlwe || !result))) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        if (count == 0) return FHE_HIP_OK;
        const Params& p = ctx->eng.params();
        const size_t kw = count * (size_t)p.digitsG2 * 2 * p.N, rw = count * 2 * (size_t)p.N;
        for (size_t i = 0; i < kw; ++i)
            if (rgsw[i] >= p.Q) return fail(FHE_HIP_ERR_INVALID_PARAM, "RGSW key not reduced mod Q");
        for (size_t i = 0; i < rw; ++i)
            if (rlwe[i] >= p.Q) return fail(FHE_HIP_ERR_INVALID_PARAM, "RLWE ciphertext not reduced mod Q");
        hipStream_t s = ctx_stream(ctx, nullptr);
        uint64_t* d = ctx->scratch((kw + rw) * 8, s);
        FHE_HIP_CHECK(hipMemcpyAsync(d, rgsw, kw * 8, hipMemcpyHostToDevice, s));
        FHE_HIP_CHECK(hipMemcpyAsync(d + kw, rlwe, rw * 8, hipMemcpyHostToDevice, s));
        ctx->eng.external_product_device(count, d, d + kw, d + kw, s);
        FHE_HIP_CHECK(hipMemcpyAsync(result, d + kw, rw * 8, hipMemcpyDeviceToHost, s));
        FHE_HIP_CHECK(hipStreamSynchronize(s));
        return FHE_HIP_OK;
    });
}

int fhe_hip_external_product_batch_device(fhe_hip_ctx* ctx, size_t count, const uint64_t* d_rgsw,
                                          const uint64_t* d_rlwe, uint64_t* d_result, void* stream) {
    if (!ctx || (count && (!d_rgsw || !d_rlwe || !d_result))) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        const CallOrder order(ctx, stream);
        const hipStream_t s = order.s;
        ctx->eng.external_product_device(count, d_rgsw, d_rlwe, d_result, s);
        return FHE_HIP_OK;
    });
}

int fhe_hip_max_batch_size(fhe_hip_ctx* ctx, size_t* max_count) {
    if (!ctx || !max_count) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        *max_count = ctx->eng.max_batch();
        return FHE_HIP_OK;
    });
}

int fhe_hip_device_memory(int device, size_t* free_bytes, size_t* total_bytes) {
    if (!free_bytes && !total_bytes) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    size_t fr = 0, tot = 0;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipMemGetInfo(&fr, &tot);
    if (e != hipSuccess) return hip_fail(e, "hipMemGetInfo");
    if (free_bytes) *free_bytes = fr;
    if (total_bytes) *total_bytes = tot;
    return FHE_HIP_OK;
}

int fhe_hip_unpack_keys(int paramset, int method, const uint8_t* bsk_packed, size_t bsk_size, uint64_t* bsk,
                        size_t bsk_cap, const uint8_t* ksk_packed, size_t ksk_size, uint64_t* kskA, size_t kskA_cap,
                        uint64_t* kskB, size_t kskB_cap) {
    return guarded([&]() -> int {
        const Params p = make_params(paramset, method);
        if (bsk_packed && bsk) {
            size_t words = 0;
            const uint64_t* raw = unpack_bsk(p, bsk_packed, bsk_size, &words);
            if (bsk_cap < words) return fail(FHE_HIP_ERR_INVALID_PARAM, "bsk buffer too small");
            std::copy(raw, raw + words, bsk);
        }
        if (ksk_packed && kskA && kskB) {
            const uint64_t *A = nullptr, *B = nullptr;
            unpack_ksk(p, ksk_packed, ksk_size, &A, &B);
            const size_t rows = p.ksk_rows_all();
            if (kskA_cap < rows * p.n || kskB_cap < rows) return fail(FHE_HIP_ERR_INVALID_PARAM, "ksk buffers too small");
            std::copy(A, A + rows * p.n, kskA);
            std::copy(B, B + rows, kskB);
        }
        return FHE_HIP_OK;
    });
}

// ---- functional bootstrapping ----
int fhe_hip_eval_func_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b, uint64_t q_in,
                            const uint64_t* lut, size_t lut_len, uint64_t* a_out, uint64_t* b_out) {
    if (!ctx || !lut || !io_ok(count, a, b, a_out, b_out, a, b)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    if (lut_len != q_in) return fail(FHE_HIP_ERR_INVALID_PARAM, "LUT length must equal the ciphertext modulus");
    return guarded([&]() -> int {
        ctx_stream(ctx, nullptr);
        ctx->eng.fb_host(0, count, a, b, q_in, 0, 0, lut, a_out, b_out);
        return FHE_HIP_OK;
    });
}

int fhe_hip_eval_func_batch_device(fhe_hip_ctx* ctx, size_t count, const uint64_t* d_a, const uint64_t* d_b,
                                   uint64_t q_in, const uint64_t* lut, size_t lut_len, uint64_t* d_a_out,
                                   uint64_t* d_b_out, void* stream) {
    if (!ctx || !lut || !io_ok(count, d_a, d_b, d_a_out, d_b_out, d_a, d_b))
        return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    if (lut_len != q_in) return fail(FHE_HIP_ERR_INVALID_PARAM, "LUT length must equal the ciphertext modulus");
    return guarded([&]() -> int {
        const CallOrder order(ctx, stream);
        const hipStream_t s = order.s;
        ctx->eng.eval_func_device(count, d_a, d_b, q_in, lut, d_a_out, d_b_out,
                                  s);
        return FHE_HIP_OK;
    });
}

int fhe_hip_eval_func_multi_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b, uint64_t q_in,
                                  const uint64_t* luts, size_t lut_len, uint32_t num_luts, uint64_t* a_out,
                                  uint64_t* b_out) {
    if (!ctx || !luts || !io_ok(count, a, b, a_out, b_out, a, b)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    if (lut_len != q_in) return fail(FHE_HIP_ERR_INVALID_PARAM, "LUT length must equal the ciphertext modulus");
    if (num_luts == 0) return fail(FHE_HIP_ERR_INVALID_PARAM, "no LUTs");
    return guarded([&]() -> int {
        ctx_stream(ctx, nullptr);
        ctx->eng.fb_host(5, count, a, b, q_in, 0, num_luts, luts, a_out, b_out);
        return FHE_HIP_OK;
    });
}

int fhe_hip_eval_func_multi_batch_device(fhe_hip_ctx* ctx, size_t count, const uint64_t* d_a, const uint64_t* d_b,
                                         uint64_t q_in, const uint64_t* luts, size_t lut_len, uint32_t num_luts,
                                         uint64_t* d_a_out, uint64_t* d_b_out, void* stream) {
    if (!ctx || !luts || !io_ok(count, d_a, d_b, d_a_out, d_b_out, d_a, d_b))
        return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    if (lut_len != q_in) return fail(FHE_HIP_ERR_INVALID_PARAM, "LUT length must equal the ciphertext modulus");
    if (num_luts == 0) return fail(FHE_HIP_ERR_INVALID_PARAM, "no LUTs");
    return guarded([&]() -> int {
        const CallOrder order(ctx, stream);
        ctx->eng.eval_func_multi_device(count, d_a, d_b, q_in, luts, num_luts, d_a_out, d_b_out, order.s);
        return FHE_HIP_OK;
    });
}

int fhe_hip_eval_floor_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod,
                             uint32_t roundbits, uint64_t* a_out, uint64_t* b_out) {
    if (!ctx || !io_ok(count, a, b, a_out, b_out, a, b)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        ctx_stream(ctx, nullptr);
        ctx->eng.fb_host(1, count, a, b, mod, 0, roundbits, nullptr, a_out, b_out);
        return FHE_HIP_OK;
    });
}

int fhe_hip_eval_sign_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod,
                            int scheme_switch, uint64_t* a_out, uint64_t* b_out) {
    if (!ctx || !io_ok(count, a, b, a_out, b_out, a, b)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        ctx_stream(ctx, nullptr);
        ctx->eng.fb_host(2, count, a, b, mod, 0, scheme_switch ? 1u : 0u, nullptr, a_out, b_out);
        return FHE_HIP_OK;
    });
}

int fhe_hip_eval_decomp_parts(fhe_hip_ctx* ctx, uint64_t mod, uint32_t* parts) {
    if (!ctx || !parts) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        *parts = ctx->eng.eval_decomp_parts(mod);
        return FHE_HIP_OK;
    });
}

int fhe_hip_eval_decomp_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod,
                              uint64_t* a_out, uint64_t* b_out) {
    if (!ctx || !io_ok(count, a, b, a_out, b_out, a, b)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        ctx_stream(ctx, nullptr);
        ctx->eng.fb_host(3, count, a, b, mod, 0, 0, nullptr, a_out, b_out);
        return FHE_HIP_OK;
    });
}

int fhe_hip_bootstrap_func_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b,
                                 uint32_t ctmod, const uint64_t* f, uint64_t fmod, uint64_t* a_out, uint64_t* b_out) {
    if (!ctx || !f || !io_ok(count, a, b, a_out, b_out, a, b)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        ctx_stream(ctx, nullptr);
        ctx->eng.fb_host(4, count, a, b, ctmod, fmod, 0, f, a_out, b_out);
        return FHE_HIP_OK;
    });
}

int fhe_hip_keyswitch_batch(fhe_hip_ctx* ctx, size_t count, const uint64_t* a, const uint64_t* b, uint64_t* a_out,
                            uint64_t* b_out) {
    if (!ctx || !io_ok(count, a, b, a_out, b_out, a, b)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        ctx_stream(ctx, nullptr);
        ctx->eng.keyswitch_host(count, a, b, a_out, b_out);
        return FHE_HIP_OK;
    });
}

int fhe_hip_modswitch_batch(fhe_hip_ctx* ctx, uint64_t q_from, uint64_t q_to, uint32_t len, size_t count,
                            const uint64_t* a, const uint64_t* b, uint64_t* a_out, uint64_t* b_out) {
    if (!ctx || !io_ok(count, a, b, a_out, b_out, a, b)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    if (q_from == 0 || q_to == 0) return fail(FHE_HIP_ERR_INVALID_PARAM, "modswitch: zero modulus");
    return guarded([&]() -> int {
        if (count == 0) return FHE_HIP_OK;
        const size_t words = count * (size_t)len;
        for (size_t i = 0; i < words; ++i)
            if (a[i] >= q_from) return fail(FHE_HIP_ERR_INVALID_PARAM, "modswitch input not reduced");
        uint64_t* d = nullptr;
        FHE_HIP_CHECK(hipSetDevice(ctx->eng.device()));
        FHE_HIP_CHECK(hipMalloc(&d, (2 * words + 2 * count) * 8));
        hipStream_t s = ctx_stream(ctx, nullptr);
        hipError_t e = hipMemcpyAsync(d, a, words * 8, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(d + words, b, count * 8, hipMemcpyHostToDevice, s);
        if (e == hipSuccess)
            e = launch_modswitch(q_from, q_to, len, (uint32_t)count, d, d + words, d + words + count,
                                 d + 2 * words + count, s);
        if (e == hipSuccess) e = hipMemcpyAsync(a_out, d + words + count, words * 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipMemcpyAsync(b_out, d + 2 * words + count, count * 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        (void)hipFree(d);
        if (e != hipSuccess) return hip_fail(e, "modswitch");
        return FHE_HIP_OK;
    });
}

int fhe_hip_multi_create(int paramset, int method, const int* devices, int ndev, fhe_hip_multi** out) {
    if (!out || !devices) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        *out = nullptr;
        *out = new fhe_hip_multi(paramset, method, devices, ndev);
        return FHE_HIP_OK;
    });
}

void fhe_hip_multi_destroy(fhe_hip_multi* m) {
    try {
        delete m;
    } catch (...) {
    }
}

int fhe_hip_multi_load_keys(fhe_hip_multi* m, const uint64_t* bsk, size_t n_words, const uint64_t* A, size_t nA,
                            const uint64_t* B, size_t nB) {
    if (!m || !bsk || !A || !B) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int { m->eng.load_keys(bsk, n_words, A, nA, B, nB); return FHE_HIP_OK; });
}

int fhe_hip_multi_eval_bingate_batch(fhe_hip_multi* m, int gate, size_t count, const uint64_t* a1, const uint64_t* b1,
                                     const uint64_t* a2, const uint64_t* b2, uint64_t* a_out, uint64_t* b_out) {
    if (!m || !io_ok(count, a1, b1, a2, b2, a_out, b_out)) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        m->eng.eval_gate_host(gate, count, a1, b1, a2, b2, a_out, b_out);
        return FHE_HIP_OK;
    });
}

int fhe_hip_keygen_secret(int paramset, int method, uint64_t seed, uint64_t* sk) {
    if (!sk) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        Params p = make_params(paramset, method);
        std::vector<uint64_t> s;
        keygen_secret(p, seed, s);
        std::copy(s.begin(), s.end(), sk);
        return FHE_HIP_OK;
    });
}

int fhe_hip_keygen(int paramset, int method, uint64_t seed, uint64_t* sk, uint64_t* bsk, uint64_t* kskA,
                   uint64_t* kskB) {
    if (!sk || !bsk || !kskA || !kskB) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        Params p = make_params(paramset, method);
        KeySet ks;
        std::vector<uint64_t> s;
        keygen_secret(p, seed, s);
        keygen_bootstrap(p, s, seed, ks);
        std::copy(ks.sk.begin(), ks.sk.end(), sk);
        std::copy(ks.bsk.begin(), ks.bsk.end(), bsk);
        std::copy(ks.kskA.begin(), ks.kskA.end(), kskA);
        std::copy(ks.kskB.begin(), ks.kskB.end(), kskB);
        return FHE_HIP_OK;
    });
}

int fhe_hip_encrypt(int paramset, int method, const uint64_t* sk, const int* bits, size_t count, uint64_t seed,
                    uint64_t* a, uint64_t* b) {
    if (!sk || (count && (!bits || !a || !b))) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        encrypt(make_params(paramset, method), sk, bits, count, seed, a, b);
        return FHE_HIP_OK;
    });
}

int fhe_hip_decrypt(int paramset, int method, const uint64_t* sk, const uint64_t* a, const uint64_t* b, size_t count,
                    uint32_t len, uint64_t mod, int64_t* out) {
    if (!sk || (count && (!a || !b || !out))) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        Params p = make_params(paramset, method);
        if (len != p.n && len != p.N) return fail(FHE_HIP_ERR_INVALID_PARAM, "len must be n or N");
        for (size_t i = 0; i < count; ++i) out[i] = decrypt(p, sk, a + i * len, b[i], len, mod);
        return FHE_HIP_OK;
    });
}

int fhe_hip_encrypt_ptmod(int paramset, int method, const uint64_t* sk, const int* bits, size_t count, uint64_t seed,
                          uint32_t ptmod, uint64_t* a, uint64_t* b) {
    if (!sk || (count && (!bits || !a || !b))) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        encrypt(make_params(paramset, method), sk, bits, count, seed, a, b, ptmod);
        return FHE_HIP_OK;
    });
}

int fhe_hip_encrypt_mod(int paramset, int method, const uint64_t* sk, const int* bits, size_t count, uint64_t seed,
                        uint32_t ptmod, uint64_t mod, uint64_t* a, uint64_t* b) {
    if (!sk || (count && (!bits || !a || !b))) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        encrypt(make_params(paramset, method), sk, bits, count, seed, a, b, ptmod, mod);
        return FHE_HIP_OK;
    });
}

int fhe_hip_decrypt_ptmod(int paramset, int method, const uint64_t* sk, const uint64_t* a, const uint64_t* b,
                          size_t count, uint32_t len, uint64_t mod, uint32_t ptmod, int64_t* out) {
    if (!sk || (count && (!a || !b || !out))) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    if (ptmod < 2 || ptmod > mod) return fail(FHE_HIP_ERR_INVALID_PARAM, "plaintext modulus out of range");
    return guarded([&]() -> int {
        Params p = make_params(paramset, method);
        if (len != p.n && len != p.N) return fail(FHE_HIP_ERR_INVALID_PARAM, "len must be n or N");
        for (size_t i = 0; i < count; ++i) out[i] = decrypt(p, sk, a + i * len, b[i], len, mod, ptmod);
        return FHE_HIP_OK;
    });
}

int fhe_hip_keygen_ring_secret(int paramset, int method, uint64_t seed, uint64_t* skN) {
    if (!skN) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        Params p = make_params(paramset, method);
        std::vector<uint64_t> s;
        keygen_ring_secret(p, seed, s);
        for (uint32_t i = 0; i < p.N; ++i) skN[i] = s[i] > (p.Q >> 1) ? p.qKS - (p.Q - s[i]) % p.qKS : s[i] % p.qKS;
        return FHE_HIP_OK;
    });
}

int fhe_hip_encrypt_large(int paramset, int method, const uint64_t* skN, const int* bits, size_t count, uint64_t seed,
                          uint32_t ptmod, uint64_t* a, uint64_t* b) {
    if (!skN || (count && (!bits || !a || !b))) return fail(FHE_HIP_ERR_NULL_PTR, "null argument");
    return guarded([&]() -> int {
        Params p = make_params(paramset, method);
        encrypt(p, skN, bits, count, seed, a, b, ptmod, p.Q, p.N);
        return FHE_HIP_OK;
    });
}

}  // extern "C"
