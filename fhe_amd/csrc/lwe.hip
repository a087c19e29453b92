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

__global__ void k_widen_u64(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b, uint64_t* __restrict__ ao,
                            uint64_t* __restrict__ bo, uint64_t total, size_t count) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x)
        ao[i] = a[i];
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x)
        bo[i] = b[i];
}

// RoundqQ as the reference writes it (lwe-pke.cpp:41-46): IEEE double, no contraction
__device__ __forceinline__ uint64_t round_qQ_ref(uint64_t v, uint64_t to, uint64_t from) {
#pragma clang fp contract(off)
    const double x = (double)v * (double)to / (double)from;
    return (uint64_t)floor(0.5 + x) % to;
}

// EvalNOT (binfhe-base-scheme.cpp:223-236) at modulus m: a -> m - a (a != 0), b -> m/4 - b mod m (ModSubFast)
__device__ __forceinline__ uint64_t not_a(uint64_t a, uint64_t m) { return a == 0 ? 0 : m - a; }
__device__ __forceinline__ uint64_t not_b(uint64_t b, uint64_t m) {
    const uint64_t c = m >> 2;
    return c < b ? c + m - b : c - b;
}

// row g of a column is mod Q when flagged (large == nullptr: every row)
__device__ __forceinline__ bool is_large_row(const uint8_t* large, uint64_t g) { return !large || large[g] != 0; }

template <typename W>
__global__ void k_switch_in(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b, uint32_t stride,
                            const uint8_t* __restrict__ large, uint64_t Q, uint64_t qKS, uint32_t N, size_t count,
                            int negate, W* __restrict__ ea, W* __restrict__ eb) {
    const uint64_t total = (uint64_t)count * N;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t g = i / N, x = i - g * N;
        uint64_t v = 0;
        if (is_large_row(large, g)) {
            const uint64_t y = a[g * stride + x];
            v = round_qQ_ref(negate ? not_a(y, Q) : y, qKS, Q);
        }
        ea[i] = (W)v;
    }
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < count; g += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t v = 0;
        if (is_large_row(large, g)) v = round_qQ_ref(negate ? not_b(b[g], Q) : b[g], qKS, Q);
        eb[g] = (W)v;
    }
}

__global__ void k_switch_out(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b, uint32_t stride,
                             const uint8_t* __restrict__ large, uint32_t n, uint64_t q, size_t count, int negate,
                             int set_b, uint64_t b_large, uint64_t* __restrict__ oa, uint64_t* __restrict__ ob) {
    const uint64_t total = (uint64_t)count * n;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t g = i / n, x = i - g * n;
        if (is_large_row(large, g)) continue;   // the key switch's output is already there
        const uint64_t y = a[g * stride + x];
        oa[i] = negate ? not_a(y, q) : y;
    }
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < count; g += (uint64_t)gridDim.x * blockDim.x) {
        if (is_large_row(large, g)) {
            if (set_b) ob[g] = b_large;
        } else {
            ob[g] = negate ? not_b(b[g], q) : b[g];
        }
    }
}

__global__ void k_lwe_repeat(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b, uint32_t n, size_t count,
                             uint32_t L, uint64_t* __restrict__ ao, uint64_t* __restrict__ bo) {
    const uint64_t total = (uint64_t)count * L * n;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t row = i / n, x = i - row * n;
        ao[i] = a[(row / L) * n + x];
    }
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < (uint64_t)count * L; r += (uint64_t)gridDim.x * blockDim.x)
        bo[r] = b[r / L];
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

hipError_t launch_lwe_repeat(const uint64_t* a, const uint64_t* b, uint32_t n, size_t count, uint32_t L, uint64_t* ao,
                             uint64_t* bo, hipStream_t s) {
    if (count == 0 || L == 0) return hipSuccess;
    hipLaunchKernelGGL(k_lwe_repeat, dim3(grid_for((uint64_t)count * L * n)), dim3(256), 0, s, a, b, n, count, L, ao, bo);
    return hipGetLastError();
}

hipError_t launch_widen_u64(const uint32_t* a, const uint32_t* b, uint64_t* ao, uint64_t* bo, uint32_t len, size_t count,
                            hipStream_t s) {
    if (count == 0) return hipSuccess;
    const uint64_t total = (uint64_t)count * len;
    hipLaunchKernelGGL(k_widen_u64, dim3(grid_for(total)), dim3(256), 0, s, a, b, ao, bo, total, count);
    return hipGetLastError();
}

hipError_t launch_switch_in(const uint64_t* a, const uint64_t* b, uint32_t stride, const uint8_t* large, uint64_t Q,
                            uint64_t qKS, uint32_t N, size_t count, bool negate, void* ext_a, void* ext_b, bool ext64,
                            hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (stride < N || Q == 0 || qKS == 0 || (!ext64 && qKS > (1ull << 32))) return hipErrorInvalidValue;
    const uint32_t grid = grid_for((uint64_t)count * N);
    if (ext64)
        hipLaunchKernelGGL(k_switch_in<uint64_t>, dim3(grid), dim3(256), 0, s, a, b, stride, large, Q, qKS, N, count,
                           negate ? 1 : 0, static_cast<uint64_t*>(ext_a), static_cast<uint64_t*>(ext_b));
    else
        hipLaunchKernelGGL(k_switch_in<uint32_t>, dim3(grid), dim3(256), 0, s, a, b, stride, large, Q, qKS, N, count,
                           negate ? 1 : 0, static_cast<uint32_t*>(ext_a), static_cast<uint32_t*>(ext_b));
    return hipGetLastError();
}

hipError_t launch_switch_out(const uint64_t* a, const uint64_t* b, uint32_t stride, const uint8_t* large, uint32_t n,
                             uint64_t q, size_t count, bool negate, bool set_b, uint64_t b_large, uint64_t* a_out,
                             uint64_t* b_out, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (stride < n || q == 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_switch_out, dim3(grid_for((uint64_t)count * n)), dim3(256), 0, s, a, b, stride, large, n, q,
                       count, negate ? 1 : 0, set_b ? 1 : 0, b_large, a_out, b_out);
    return hipGetLastError();
}

}  // namespace fhe_amd
