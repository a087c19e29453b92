// ubench.hip -- measures gfx950 VALU throughput of the integer/fp ops the NTT
// and external product are built from (design input, not product code).
#include <hip/hip_runtime.h>
#include <stdio.h>

#define ITERS 2048
#define OP_KERNEL(NAME, ASM)                                                              \
    __global__ void NAME(unsigned* out, unsigned seed) {                                 \
        unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;          \
        unsigned a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed | 1;        \
        for (int i = 0; i < ITERS; ++i) {                                                 \
            asm volatile(ASM " %0, %0, %8\n\t" ASM " %1, %1, %8\n\t" ASM " %2, %2, %8\n\t"  \
                         ASM " %3, %3, %8\n\t" ASM " %4, %4, %8\n\t" ASM " %5, %5, %8\n\t"  \
                         ASM " %6, %6, %8\n\t" ASM " %7, %7, %8"                          \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5),   \
                           "+v"(a6), "+v"(a7)                                             \
                         : "v"(b));                                                       \
        }                                                                                 \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
    }

OP_KERNEL(k_add, "v_add_u32")
OP_KERNEL(k_mul_lo, "v_mul_lo_u32")
OP_KERNEL(k_mul_hi, "v_mul_hi_u32")
OP_KERNEL(k_mul24, "v_mul_u32_u24")
OP_KERNEL(k_mulhi24, "v_mul_hi_u32_u24")
OP_KERNEL(k_fmul, "v_mul_f32")
OP_KERNEL(k_mul_hi_i, "v_mul_hi_i32")
OP_KERNEL(k_bfe, "v_sub_u32")
OP_KERNEL(k_min, "v_min_u32")
OP_KERNEL(k_pkadd, "v_pk_add_u16")
OP_KERNEL(k_max, "v_max_u32")
OP_KERNEL(k_mini, "v_min_i32")
OP_KERNEL(k_xor, "v_xor_b32")
OP_KERNEL(k_lshl, "v_lshlrev_b32")
OP_KERNEL(k_subrev, "v_subrev_u32")
#define OP3_KERNEL(NAME, ASM)                                                             \
    __global__ void NAME(unsigned* out, unsigned seed) {                                 \
        unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;          \
        unsigned a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed | 1, c = seed * 5; \
        for (int i = 0; i < ITERS; ++i) {                                                 \
            asm volatile(ASM " %0, %0, %8, %9\n\t" ASM " %1, %1, %8, %9\n\t" ASM " %2, %2, %8, %9\n\t"  \
                         ASM " %3, %3, %8, %9\n\t" ASM " %4, %4, %8, %9\n\t" ASM " %5, %5, %8, %9\n\t"  \
                         ASM " %6, %6, %8, %9\n\t" ASM " %7, %7, %8, %9"                          \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5),   \
                           "+v"(a6), "+v"(a7)                                             \
                         : "v"(b), "v"(c) : "vcc");                                                \
        }                                                                                 \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
    }
OP3_KERNEL(k_add3, "v_add3_u32")
OP3_KERNEL(k_med3, "v_med3_u32")
OP3_KERNEL(k_min3, "v_min3_u32")
OP3_KERNEL(k_bfei, "v_bfe_i32")
OP3_KERNEL(k_lshladd, "v_lshl_add_u32")
OP3_KERNEL(k_andor, "v_and_or_b32")
OP3_KERNEL(k_xad, "v_xad_u32")
__global__ void k_cndmask(unsigned* out, unsigned seed) {
        unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
        unsigned a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed | 1;
        for (int i = 0; i < ITERS; ++i) {
            asm volatile("v_cmp_lt_u32 vcc, %0, %8\n\t v_cndmask_b32 %0, %0, %8, vcc\n\t v_cndmask_b32 %1, %1, %8, vcc\n\t v_cndmask_b32 %2, %2, %8, vcc\n\t"
                         "v_cndmask_b32 %3, %3, %8, vcc\n\t v_cndmask_b32 %4, %4, %8, vcc\n\t v_cndmask_b32 %5, %5, %8, vcc\n\t"
                         "v_cndmask_b32 %6, %6, %8, vcc\n\t v_cndmask_b32 %7, %7, %8, vcc"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "vcc");
        }
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_cmp(unsigned* out, unsigned seed) {
        unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
        unsigned b = seed | 1; unsigned long long s0=0,s1=0,s2=0,s3=0;
        for (int i = 0; i < ITERS; ++i) {
            asm volatile("v_cmp_lt_u32 %4, %0, %8\n\t v_cmp_lt_u32 %5, %1, %8\n\t v_cmp_lt_u32 %6, %2, %8\n\t v_cmp_lt_u32 %7, %3, %8\n\t"
                         "v_cmp_lt_u32 %4, %1, %8\n\t v_cmp_lt_u32 %5, %2, %8\n\t v_cmp_lt_u32 %6, %3, %8\n\t v_cmp_lt_u32 %7, %0, %8"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "=s"(s0), "=s"(s1), "=s"(s2), "=s"(s3) : "v"(b));
        }
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ (unsigned)(s0^s1^s2^s3);
}
__global__ void k_perm(unsigned* out, unsigned seed) {
        unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
        unsigned a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
        for (int i = 0; i < ITERS; ++i) {
            asm volatile("v_permlane32_swap_b32 %0, %1\n\t v_permlane32_swap_b32 %2, %3\n\t v_permlane32_swap_b32 %4, %5\n\t v_permlane32_swap_b32 %6, %7\n\t"
                         "v_permlane32_swap_b32 %1, %0\n\t v_permlane32_swap_b32 %3, %2\n\t v_permlane32_swap_b32 %5, %4\n\t v_permlane32_swap_b32 %7, %6"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
        }
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_subco(unsigned* out, unsigned seed) {
        unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
        unsigned a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed | 1;
        for (int i = 0; i < ITERS; ++i) {
            asm volatile("v_sub_co_u32 %0, vcc, %0, %8\n\t v_sub_co_u32 %1, vcc, %1, %8\n\t v_sub_co_u32 %2, vcc, %2, %8\n\t v_sub_co_u32 %3, vcc, %3, %8\n\t"
                         "v_sub_co_u32 %4, vcc, %4, %8\n\t v_sub_co_u32 %5, vcc, %5, %8\n\t v_sub_co_u32 %6, vcc, %6, %8\n\t v_sub_co_u32 %7, vcc, %7, %8"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "vcc");
        }
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k_mad64(unsigned long long* out, unsigned seed) {
    unsigned long long a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    unsigned long long a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    unsigned b = seed | 1, c = seed * 3;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_mad_u64_u32 %0, vcc, %8, %9, %0\n\t v_mad_u64_u32 %1, vcc, %8, %9, %1\n\t"
            "v_mad_u64_u32 %2, vcc, %8, %9, %2\n\t v_mad_u64_u32 %3, vcc, %8, %9, %3\n\t"
            "v_mad_u64_u32 %4, vcc, %8, %9, %4\n\t v_mad_u64_u32 %5, vcc, %8, %9, %5\n\t"
            "v_mad_u64_u32 %6, vcc, %8, %9, %6\n\t v_mad_u64_u32 %7, vcc, %8, %9, %7"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(b), "v"(c)
            : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k_fma64(double* out, unsigned seed) {
    double a0 = threadIdx.x + seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    double a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = 0.999, c = 1e-3;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_fma_f64 %0, %0, %8, %9\n\t v_fma_f64 %1, %1, %8, %9\n\t"
            "v_fma_f64 %2, %2, %8, %9\n\t v_fma_f64 %3, %3, %8, %9\n\t"
            "v_fma_f64 %4, %4, %8, %9\n\t v_fma_f64 %5, %5, %8, %9\n\t"
            "v_fma_f64 %6, %6, %8, %9\n\t v_fma_f64 %7, %7, %8, %9"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(b), "v"(c));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}


__global__ void k_madi64(unsigned long long* out, unsigned seed) {
    long long a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    long long a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    int b = seed | 1, c = seed * 3;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_mad_i64_i32 %0, vcc, %8, %9, %0\n\t v_mad_i64_i32 %1, vcc, %8, %9, %1\n\t"
            "v_mad_i64_i32 %2, vcc, %8, %9, %2\n\t v_mad_i64_i32 %3, vcc, %8, %9, %3\n\t"
            "v_mad_i64_i32 %4, vcc, %8, %9, %4\n\t v_mad_i64_i32 %5, vcc, %8, %9, %5\n\t"
            "v_mad_i64_i32 %6, vcc, %8, %9, %6\n\t v_mad_i64_i32 %7, vcc, %8, %9, %7"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(b), "v"(c)
            : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k_lshladd64(unsigned long long* out, unsigned seed) {
    unsigned long long a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    unsigned long long a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    unsigned long long b = seed | 1;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_lshl_add_u64 %0, %0, 1, %8\n\t v_lshl_add_u64 %1, %1, 1, %8\n\t"
            "v_lshl_add_u64 %2, %2, 1, %8\n\t v_lshl_add_u64 %3, %3, 1, %8\n\t"
            "v_lshl_add_u64 %4, %4, 1, %8\n\t v_lshl_add_u64 %5, %5, 1, %8\n\t"
            "v_lshl_add_u64 %6, %6, 1, %8\n\t v_lshl_add_u64 %7, %7, 1, %8"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(b));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ void k_lshl64(unsigned long long* out, unsigned seed) {
    unsigned long long a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    unsigned long long a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    unsigned b = (seed & 7) | 1;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_lshlrev_b64 %0, %8, %0\n\t v_lshlrev_b64 %1, %8, %1\n\t"
            "v_lshlrev_b64 %2, %8, %2\n\t v_lshlrev_b64 %3, %8, %3\n\t"
            "v_lshlrev_b64 %4, %8, %4\n\t v_lshlrev_b64 %5, %8, %5\n\t"
            "v_lshlrev_b64 %6, %8, %6\n\t v_lshlrev_b64 %7, %8, %7"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(b));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_lshladd64b(unsigned long long* out, unsigned seed) {
    unsigned long long a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    unsigned long long a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    unsigned long long b = seed | 1;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_lshl_add_u64 %0, %0, 0, %8\n\t v_lshl_add_u64 %1, %1, 0, %8\n\t"
            "v_lshl_add_u64 %2, %2, 0, %8\n\t v_lshl_add_u64 %3, %3, 0, %8\n\t"
            "v_lshl_add_u64 %4, %4, 0, %8\n\t v_lshl_add_u64 %5, %5, 0, %8\n\t"
            "v_lshl_add_u64 %6, %6, 0, %8\n\t v_lshl_add_u64 %7, %7, 0, %8"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(b));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_mov64(unsigned long long* out, unsigned seed) {
    unsigned long long a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    unsigned long long a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_mov_b64 %0, %1\n\t v_mov_b64 %1, %2\n\t v_mov_b64 %2, %3\n\t v_mov_b64 %3, %4\n\t"
            "v_mov_b64 %4, %5\n\t v_mov_b64 %5, %6\n\t v_mov_b64 %6, %7\n\t v_mov_b64 %7, %0"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <typename K, typename T>
static void run(const char* name, K kern, T* buf, int blocks, int threads) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, buf, 7u);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, buf, 7u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double ops = 5.0 * blocks * threads * ITERS * 8.0;
    // lane-ops per ns; per CU per clock at 2.4 GHz: ops / (256 * 2.4e9 * s)
    printf("%-18s %8.3f ms  %9.1f Glane-op/s  %6.2f lane-op/clk/CU (2.4GHz)\n", name, ms, ops / (ms * 1e6),
           ops / (ms * 1e-3) / (256 * 2.4e9));
}

int main() {
    const int blocks = 256 * 8, threads = 256;
    void* buf;
    hipMalloc(&buf, (size_t)blocks * threads * 8);
    run("v_add_u32", k_add, (unsigned*)buf, blocks, threads);
    run("v_mul_lo_u32", k_mul_lo, (unsigned*)buf, blocks, threads);
    run("v_mul_hi_u32", k_mul_hi, (unsigned*)buf, blocks, threads);
    run("v_mul_u32_u24", k_mul24, (unsigned*)buf, blocks, threads);
    run("v_mul_hi_u32_u24", k_mulhi24, (unsigned*)buf, blocks, threads);
    run("v_mul_f32", k_fmul, (unsigned*)buf, blocks, threads);
    run("v_mad_u64_u32", k_mad64, (unsigned long long*)buf, blocks, threads);
    run("v_fma_f64", k_fma64, (double*)buf, blocks, threads);
    run("v_mad_i64_i32", k_madi64, (unsigned long long*)buf, blocks, threads);
    run("v_lshl_add_u64", k_lshladd64, (unsigned long long*)buf, blocks, threads);
    run("v_lshl_add_u64(0)", k_lshladd64b, (unsigned long long*)buf, blocks, threads);
    run("v_lshlrev_b64", k_lshl64, (unsigned long long*)buf, blocks, threads);
    run("v_mov_b64", k_mov64, (unsigned long long*)buf, blocks, threads);
    run("v_mul_hi_i32", k_mul_hi_i, (unsigned*)buf, blocks, threads);
    run("v_sub_u32", k_bfe, (unsigned*)buf, blocks, threads);
    run("v_min_u32", k_min, (unsigned*)buf, blocks, threads);
    run("v_pk_add_u16", k_pkadd, (unsigned*)buf, blocks, threads);
    run("v_max_u32", k_max, (unsigned*)buf, blocks, threads);
    run("v_min_i32", k_mini, (unsigned*)buf, blocks, threads);
    run("v_xor_b32", k_xor, (unsigned*)buf, blocks, threads);
    run("v_lshlrev_b32", k_lshl, (unsigned*)buf, blocks, threads);
    run("v_subrev_u32", k_subrev, (unsigned*)buf, blocks, threads);
    run("v_add3_u32", k_add3, (unsigned*)buf, blocks, threads);
    run("v_med3_u32", k_med3, (unsigned*)buf, blocks, threads);
    run("v_min3_u32", k_min3, (unsigned*)buf, blocks, threads);
    run("v_bfe_i32", k_bfei, (unsigned*)buf, blocks, threads);
    run("v_lshl_add_u32", k_lshladd, (unsigned*)buf, blocks, threads);
    run("v_and_or_b32", k_andor, (unsigned*)buf, blocks, threads);
    run("v_xad_u32", k_xad, (unsigned*)buf, blocks, threads);
    run("v_cndmask_b32(+1cmp/8)", k_cndmask, (unsigned*)buf, blocks, threads);
    run("v_cmp_lt_u32", k_cmp, (unsigned*)buf, blocks, threads);
    run("v_permlane32_swap", k_perm, (unsigned*)buf, blocks, threads);
    run("v_sub_co_u32", k_subco, (unsigned*)buf, blocks, threads);

    hipFree(buf);
    return 0;
}
