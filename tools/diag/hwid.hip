// Wave placement of a launch of `blocks` workgroups x 4 waves with `lds` bytes of LDS each (default: K1x's shape,
// 512 x 77,824 B, two per CU; `hwid 256 60416`: config 3 on K1), every wave records its HW_ID (SIMD, CU, SE,
// workgroup slot, wave slot) and a start timestamp.  usage: hwid [blocks] [lds bytes]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>
__global__ void k_hwid(uint32_t* out, uint64_t* t) {
    extern __shared__ uint32_t sm[];
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    sm[threadIdx.x] = hw;
    const uint64_t t0 = __builtin_readcyclecounter();
    for (int z = 0; z < 200; ++z) __builtin_amdgcn_s_sleep(127);
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        out[2 * w] = hw;
        out[2 * w + 1] = xcc;
        t[w] = t0;
    }
}
int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 512, lds = argc > 2 ? atoi(argv[2]) : 77824;
    const int threads = 256, waves = blocks * threads / 64;
    uint32_t* d; uint64_t* dt;
    hipMalloc(&d, waves * 8); hipMalloc(&dt, waves * 8);
    hipFuncSetAttribute((const void*)k_hwid, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(k_hwid, dim3(blocks), dim3(threads), lds, 0, d, dt);
    std::vector<uint32_t> h(waves * 2);
    hipMemcpy(h.data(), d, waves * 8, hipMemcpyDeviceToHost);
    std::map<std::tuple<int, int, int, int>, std::vector<int>> simd;  // (xcc, se, cu, simd) -> blocks
    for (int w = 0; w < waves; ++w) {
        const uint32_t hw = h[2 * w], x = h[2 * w + 1] & 15;
        const int wave = hw & 15, s = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7,
                  tg = (hw >> 16) & 15;
        if (w < 16 || (w >= 1024 && w < 1032))
            printf("wave %4d block %3d: xcc %d se %d sh %d cu %2d simd %d tg %2d slot %d\n", w, w / 4, x, se, sh, cu, s, tg, wave);
        simd[{(int)x, se * 2 + sh, cu, s}].push_back(w / 4);
    }
    std::map<int, int> hist;
    for (auto& kv : simd) hist[(int)kv.second.size()]++;
    printf("%d workgroups, %d B LDS: %zu SIMDs used\n", blocks, lds, simd.size());
    for (auto& kv : hist) printf("SIMDs holding %d waves: %d\n", kv.first, kv.second);
    int shown = 0;
    for (auto& kv : simd) {
        if (shown++ > 6) break;
        printf("xcc %d se/sh %d cu %d simd %d: blocks", std::get<0>(kv.first), std::get<1>(kv.first), std::get<2>(kv.first), std::get<3>(kv.first));
        for (int b : kv.second) printf(" %d", b);
        printf("\n");
    }
    return 0;
}
