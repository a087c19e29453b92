// capi.cpp -- extern "C" boundary (include/fhe_hip.h).  No exception crosses it.
#include <hip/hip_runtime.h>

#include <exception>
#include <new>
#include <string>

#include "../../include/fhe_hip.h"
#include "ntt.h"

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
    } catch (const std::bad_alloc&) {
        return fail(FHE_HIP_ERR_ALLOC, "host allocation failed");
    } catch (const std::exception& e) {
        return fail(FHE_HIP_ERR_INVALID_PARAM, e.what());
    } catch (...) {
        return fail(FHE_HIP_ERR_INVALID_PARAM, "unknown exception");
    }
}
}  // namespace

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

}  // extern "C"
