// FETCH_SIZE / WRITE_SIZE calibration: stream-read (and write) a known byte count with
// 4-, 8- and 16-byte-per-lane accesses; run under rocprofv3 --pmc FETCH_SIZE (or WRITE_SIZE)
// and compare the counter with the bytes printed here.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <typename V>
__global__ void k_read(const V* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const V v = p[i];
        acc ^= reinterpret_cast<const uint32_t*>(&v)[0];
    }
    if (acc == 0x12345678u) out[0] = acc;  // keep the loads alive
}
template <typename V>
__global__ void k_write(V* __restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        V v{};
        reinterpret_cast<uint32_t*>(&v)[0] = (uint32_t)i;
        p[i] = v;
    }
}

int main() {
    const size_t bytes = 512ull << 20;
    void* buf;
    uint32_t* out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    dim3 g(4096), b(256);
    hipLaunchKernelGGL(k_read<uint32_t>, g, b, 0, 0, (const uint32_t*)buf, bytes / 4, out);
    hipLaunchKernelGGL(k_read<uint2>, g, b, 0, 0, (const uint2*)buf, bytes / 8, out);
    hipLaunchKernelGGL(k_read<uint4>, g, b, 0, 0, (const uint4*)buf, bytes / 16, out);
    hipLaunchKernelGGL(k_write<uint32_t>, g, b, 0, 0, (uint32_t*)buf, bytes / 4);
    hipLaunchKernelGGL(k_write<uint2>, g, b, 0, 0, (uint2*)buf, bytes / 8);
    hipLaunchKernelGGL(k_write<uint4>, g, b, 0, 0, (uint4*)buf, bytes / 16);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("calib bytes per launch: %zu (%.1f KiB)\n", bytes, bytes / 1024.0);
    return 0;
}
