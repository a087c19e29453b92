// lwe.hip -- element-wise LWE ciphertext arithmetic between the bootstraps of the
// functional-bootstrapping compositions (EvalFunc / EvalFloor / EvalSign / EvalDecomp,
// binfhe-base-scheme.cpp:241-518).  HBM-bound streaming kernels over u64 arrays.
#include "boot.h"

#include <algorithm>

namespace fhe_amd {

namespace {
__global__ void k_lwe_reduce(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b, uint64_t* ao,
                             uint64_t* bo, uint64_t m, uint64_t total, size_t count) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x)
        ao[i] = a[i] % m;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x)
        bo[i] = b[i] % m;
}

__device__ __forceinline__ uint64_t sub_mod_u64(uint64_t x, uint64_t y, uint64_t m) {
    return x >= y ? x - y : x + m - y;
}

__global__ void k_lwe_sub(const uint64_t* xa, const uint64_t* xb, const uint64_t* ya, const uint64_t* yb, uint64_t* oa,
                          uint64_t* ob, uint64_t m, uint64_t total, size_t count) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x)
        oa[i] = sub_mod_u64(xa[i], ya[i], m);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x)
        ob[i] = sub_mod_u64(xb[i], yb[i], m);
}

__global__ void k_lwe_addb(uint64_t* b, uint64_t c, uint64_t m, size_t count) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t v = b[i] + c;
        b[i] = v >= m ? v - m : v;
    }
}

__global__ void k_narrow_u32(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b, uint32_t* __restrict__ ao,
                             uint32_t* __restrict__ bo, uint64_t total, size_t count) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x)
        ao[i] = (uint32_t)a[i];
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x)
        bo[i] = (uint32_t)b[i];
}

uint32_t grid_for(uint64_t work) { return (uint32_t)std::min<uint64_t>((work + 255) / 256, 8192); }
}  // namespace

hipError_t launch_lwe_reduce(const uint64_t* a, const uint64_t* b, uint64_t* ao, uint64_t* bo, uint64_t m,
                             uint32_t len, size_t count, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (m == 0) return hipErrorInvalidValue;
    const uint64_t total = (uint64_t)count * len;
    hipLaunchKernelGGL(k_lwe_reduce, dim3(grid_for(total)), dim3(256), 0, s, a, b, ao, bo, m, total, count);
    return hipGetLastError();
}

hipError_t launch_lwe_sub(const uint64_t* xa, const uint64_t* xb, const uint64_t* ya, const uint64_t* yb, uint64_t* oa,
                          uint64_t* ob, uint64_t m, uint32_t len, size_t count, hipStream_t s) {
    if (count == 0) return hipSuccess;
    const uint64_t total = (uint64_t)count * len;
    hipLaunchKernelGGL(k_lwe_sub, dim3(grid_for(total)), dim3(256), 0, s, xa, xb, ya, yb, oa, ob, m, total, count);
    return hipGetLastError();
}

hipError_t launch_lwe_addb(uint64_t* b, uint64_t c, uint64_t m, size_t count, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (c >= m) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_lwe_addb, dim3(grid_for(count)), dim3(256), 0, s, b, c, m, count);
    return hipGetLastError();
}

hipError_t launch_narrow_u32(const uint64_t* a, const uint64_t* b, uint32_t* ao, uint32_t* bo, uint32_t len, size_t count,
                             hipStream_t s) {
    if (count == 0) return hipSuccess;
    const uint64_t total = (uint64_t)count * len;
    hipLaunchKernelGGL(k_narrow_u32, dim3(grid_for(total)), dim3(256), 0, s, a, b, ao, bo, total, count);
    return hipGetLastError();
}

}  // namespace fhe_amd
