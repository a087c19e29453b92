// arith.h -- modular arithmetic for the gfx950 kernels.
//
// All routines return canonical residues in [0, Q) given canonical inputs, so
// results are identical to the reference's NativeInteger ops
// (src/core/include/math/hal/intnat/ubintnat.h:751 ModAddFastEq, :924
// ModSubFastEq, :1464-1486 ModMulFastConst): exact modular arithmetic has one
// answer whatever the reduction algorithm.
//
// 32-bit path (Q < 2^31; both STD128 moduli are 27/28-bit): Shoup products with
// precomputed w' = floor(w * 2^32 / Q), and Montgomery (R = 2^32) for
// products of two variables.  64-bit path (Q < 2^62; the 60-bit
// poly-benchmark prime): Shoup with w' = floor(w * 2^64 / Q).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define FHE_DEV __device__ __forceinline__

// ---------------------------------------------------------------- 32-bit --
FHE_DEV uint32_t add_mod(uint32_t a, uint32_t b, uint32_t Q) {
    uint32_t s = a + b;
    uint32_t t = s - Q;
    return t < s ? t : s;  // unsigned min: s >= Q ? s - Q : s   (a, b < Q < 2^31)
}
FHE_DEV uint32_t sub_mod(uint32_t a, uint32_t b, uint32_t Q) {
    uint32_t d = a - b;
    uint32_t t = d + Q;
    return d < t ? d : t;  // a >= b ? d : d + Q
}
// reduce x in [0, 2Q) to [0, Q)
FHE_DEV uint32_t csub(uint32_t x, uint32_t Q) {
    uint32_t t = x - Q;
    return t < x ? t : x;
}
// Shoup: x * w mod Q with wp = floor(w * 2^32 / Q); x < 2^32, result in [0, Q)
FHE_DEV uint32_t mul_shoup(uint32_t x, uint32_t w, uint32_t wp, uint32_t Q) {
    uint32_t qt = __umulhi(x, wp);
    uint32_t r = x * w - qt * Q;  // in [0, 2Q)
    return csub(r, Q);
}
// Shoup without the final correction: result in [0, 2Q)
FHE_DEV uint32_t mul_shoup_lazy(uint32_t x, uint32_t w, uint32_t wp, uint32_t Q) {
    uint32_t qt = __umulhi(x, wp);
    return x * w - qt * Q;
}
// Montgomery reduction of a 64-bit t < Q * 2^32: returns t * 2^-32 mod Q in [0, Q).
// qinv = -Q^-1 mod 2^32.
FHE_DEV uint32_t mont_reduce(uint64_t t, uint32_t Q, uint32_t qinv) {
    uint32_t m = (uint32_t)t * qinv;
    uint64_t u = t + (uint64_t)m * Q;  // divisible by 2^32; < 2 * Q * 2^32 when t < Q * 2^32
    return csub((uint32_t)(u >> 32), Q);
}

// ---------------------------------------------------------------- 64-bit --
FHE_DEV uint64_t add_mod64(uint64_t a, uint64_t b, uint64_t Q) {
    uint64_t s = a + b;
    return s >= Q ? s - Q : s;
}
FHE_DEV uint64_t sub_mod64(uint64_t a, uint64_t b, uint64_t Q) {
    return a >= b ? a - b : a + Q - b;
}
FHE_DEV uint64_t mul_shoup64(uint64_t x, uint64_t w, uint64_t wp, uint64_t Q) {
    uint64_t qt = __umul64hi(x, wp);
    uint64_t r = x * w - qt * Q;
    return r >= Q ? r - Q : r;
}
