// ntt.hip -- batched negacyclic NTT / iNTT, N = 1024, for gfx950.
//
// Computes exactly the reference's
//   ChineseRemainderTransformFTTNat::ForwardTransformToBitReverseInPlace
//     (src/core/include/math/hal/intnat/transformnat-impl.h:647-672 -> :302-373)
//   ChineseRemainderTransformFTTNat::InverseTransformFromBitReverseInPlace
//     (transformnat-impl.h:707-735 -> :511-624)
// i.e. NativePoly::SwitchFormat (src/core/include/lattice/hal/default/poly-impl.h:420-440):
// forward output j (bit-reversed order) is a(psi^(2*brv(j)+1)); inverse is its exact inverse.
//
// Work decomposition (one polynomial per half-wave of 32 lanes, 32 coefficients
// per lane, PPB polynomials per workgroup):
//   index x = (h << 6) | (l << 1) | b0           ("layout A": lane l = x bits 5..1,
//                                                  register r = (h << 1) | b0)
//   "layout B" swaps register and lane:   lane = (h << 1) | b0, register = x bits 5..1.
// Forward: load A (16-byte loads: coefficient pairs) -> stages on bits 9..6 in
// registers (twiddles uniform across lanes: scalar loads) -> LDS transpose to B
// -> stages on bits 5..1 in registers (per-lane twiddles from the LDS-staged
// table) -> LDS transpose to A -> stage on bit 0 -> 16-byte stores.
// Inverse: the same in reverse order; the final stage folds N^-1 as the
// reference does (transformnat-impl.h:599-623).
// Global traffic = 8 B read + 8 B written per coefficient (u64 words, as the
// reference stores them); all arithmetic exact mod Q.
#include "arith.h"
#include "ntt.h"

namespace fhe_amd {

template <typename T>
struct ModT;

template <>
struct ModT<uint32_t> {
    using TW = uint2;  // (w, w' = floor(w 2^32 / Q))
    uint32_t Q;
    FHE_DEV uint32_t mul(uint32_t x, TW w) const { return mul_shoup(x, w.x, w.y, Q); }
    FHE_DEV uint32_t add(uint32_t a, uint32_t b) const { return add_mod(a, b, Q); }
    FHE_DEV uint32_t sub(uint32_t a, uint32_t b) const { return sub_mod(a, b, Q); }
};

template <>
struct ModT<uint64_t> {
    using TW = ulonglong2;  // (w, w' = floor(w 2^64 / Q))
    uint64_t Q;
    FHE_DEV uint64_t mul(uint64_t x, TW w) const { return mul_shoup64(x, w.x, w.y, Q); }
    FHE_DEV uint64_t add(uint64_t a, uint64_t b) const { return add_mod64(a, b, Q); }
    FHE_DEV uint64_t sub(uint64_t a, uint64_t b) const { return sub_mod64(a, b, Q); }
};

template <typename M, typename T>
FHE_DEV void bf_ct(T& x, T& y, typename M::TW w, const M& m) {
    T t = m.mul(y, w);
    y   = m.sub(x, t);
    x   = m.add(x, t);
}
template <typename M, typename T>
FHE_DEV void bf_gs(T& x, T& y, typename M::TW w, const M& m) {
    T t = m.sub(x, y);
    x   = m.add(x, y);
    y   = m.mul(t, w);
}

// 32x32 transpose of one half-wave's registers through its private LDS tile
// (row stride 33 words: conflict-free on both sides).
template <typename T>
FHE_DEV void half_transpose(T (&v)[32], T* tile, int l) {
#pragma unroll
    for (int r = 0; r < 32; ++r) tile[l * 33 + r] = v[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 32; ++r) v[r] = tile[r * 33 + l];
    __syncthreads();
}

template <typename T>
FHE_DEV void load_pair(const uint64_t* p, T& a, T& b) {
    ulonglong2 t = *reinterpret_cast<const ulonglong2*>(p);
    a = (T)t.x;
    b = (T)t.y;
}
template <typename T>
FHE_DEV void store_pair(uint64_t* p, T a, T b) {
    ulonglong2 t;
    t.x = (uint64_t)a;
    t.y = (uint64_t)b;
    *reinterpret_cast<ulonglong2*>(p) = t;
}

template <typename T, bool INV, int PPB>
__global__ void __launch_bounds__(PPB * 32)
    k_ntt1024(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, uint32_t count,
              const typename ModT<T>::TW* __restrict__ tab, T Q, typename ModT<T>::TW last_lo,
              typename ModT<T>::TW last_hi) {
    using M  = ModT<T>;
    using TW = typename M::TW;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    TW* s_tw = reinterpret_cast<TW*>(smem);                      // 1024 entries
    T* tiles = reinterpret_cast<T*>(smem + 1024 * sizeof(TW));   // PPB x 32 x 33
    const M m{Q};

    for (int i = threadIdx.x; i < 1024; i += PPB * 32) s_tw[i] = tab[i];

    const int l        = threadIdx.x & 31;
    const int hp       = threadIdx.x >> 5;
    const uint32_t ply = blockIdx.x * PPB + hp;
    const bool valid   = ply < count;
    T* tile            = tiles + hp * (32 * 33);
    const uint64_t* src = in + (size_t)(valid ? ply : 0) * 1024;
    uint64_t* dst       = out + (size_t)(valid ? ply : 0) * 1024;

    T v[32];
#pragma unroll
    for (int h = 0; h < 16; ++h) {
        if (valid) load_pair(src + (h << 6) + (l << 1), v[2 * h], v[2 * h + 1]);
        else v[2 * h] = v[2 * h + 1] = 0;
    }
    __syncthreads();  // s_tw ready

    if (!INV) {
        // stages on bits 9..6 (layout A): twiddle index depends on h only
#pragma unroll
        for (int b = 9; b >= 6; --b) {
            const int hb = b - 6;
#pragma unroll
            for (int h = 0; h < 16; ++h) {
                if (h & (1 << hb)) continue;
                const TW w = tab[(1 << (9 - b)) + (h >> (hb + 1))];
                bf_ct(v[(h << 1) | 0], v[((h | (1 << hb)) << 1) | 0], w, m);
                bf_ct(v[(h << 1) | 1], v[((h | (1 << hb)) << 1) | 1], w, m);
            }
        }
        half_transpose(v, tile, l);
        // layout B: lane = (h << 1) | b0, register r = x bits 5..1
        const int hl = l >> 1;
#pragma unroll
        for (int b = 5; b >= 1; --b) {
            const int rb = b - 1;
#pragma unroll
            for (int r = 0; r < 32; ++r) {
                if (r & (1 << rb)) continue;
                const TW w = s_tw[(1 << (9 - b)) + ((hl << (5 - b)) | (r >> b))];
                bf_ct(v[r], v[r | (1 << rb)], w, m);
            }
        }
        half_transpose(v, tile, l);
        // stage on bit 0 (layout A)
#pragma unroll
        for (int h = 0; h < 16; ++h) {
            const TW w = s_tw[512 + (h << 5) + l];
            bf_ct(v[2 * h], v[2 * h + 1], w, m);
        }
    } else {
        // stage on bit 0 (layout A), GS butterflies with the inverse table
#pragma unroll
        for (int h = 0; h < 16; ++h) {
            const TW w = s_tw[512 + (h << 5) + l];
            bf_gs(v[2 * h], v[2 * h + 1], w, m);
        }
        half_transpose(v, tile, l);
        const int hl = l >> 1;
#pragma unroll
        for (int b = 1; b <= 5; ++b) {
            const int rb = b - 1;
#pragma unroll
            for (int r = 0; r < 32; ++r) {
                if (r & (1 << rb)) continue;
                const TW w = s_tw[(1 << (9 - b)) + ((hl << (5 - b)) | (r >> b))];
                bf_gs(v[r], v[r | (1 << rb)], w, m);
            }
        }
        half_transpose(v, tile, l);
#pragma unroll
        for (int b = 6; b <= 8; ++b) {
            const int hb = b - 6;
#pragma unroll
            for (int h = 0; h < 16; ++h) {
                if (h & (1 << hb)) continue;
                const TW w = tab[(1 << (9 - b)) + (h >> (hb + 1))];
                bf_gs(v[(h << 1) | 0], v[((h | (1 << hb)) << 1) | 0], w, m);
                bf_gs(v[(h << 1) | 1], v[((h | (1 << hb)) << 1) | 1], w, m);
            }
        }
        // bit 9: lo' = (lo + hi) N^-1, hi' = (lo - hi) w1 N^-1
#pragma unroll
        for (int h = 0; h < 8; ++h) {
#pragma unroll
            for (int b0 = 0; b0 < 2; ++b0) {
                T& x = v[(h << 1) | b0];
                T& y = v[((h | 8) << 1) | b0];
                T s = m.add(x, y), d = m.sub(x, y);
                x   = m.mul(s, last_lo);
                y   = m.mul(d, last_hi);
            }
        }
    }
    if (valid) {
#pragma unroll
        for (int h = 0; h < 16; ++h) store_pair(dst + (h << 6) + (l << 1), v[2 * h], v[2 * h + 1]);
    }
}

template <typename T, int PPB>
static hipError_t launch(const NttPlan& p, const uint64_t* in, uint64_t* out, uint32_t count, bool inverse,
                         hipStream_t s) {
    using TW        = typename ModT<T>::TW;
    const size_t sm = 1024 * sizeof(TW) + (size_t)PPB * 32 * 33 * sizeof(T);
    dim3 grid((count + PPB - 1) / PPB), block(PPB * 32);
    const TW* tab = reinterpret_cast<const TW*>(inverse ? p.d_tab_inv : p.d_tab_fwd);
    TW lo, hi;
    if constexpr (sizeof(T) == 4) {
        lo = TW{(uint32_t)p.ninv, (uint32_t)p.ninv_pre};
        hi = TW{(uint32_t)p.w1ninv, (uint32_t)p.w1ninv_pre};
    } else {
        lo = TW{p.ninv, p.ninv_pre};
        hi = TW{p.w1ninv, p.w1ninv_pre};
    }
    if (count == 0) return hipSuccess;
    if (inverse)
        hipLaunchKernelGGL((k_ntt1024<T, true, PPB>), grid, block, sm, s, in, out, count, tab, (T)p.Q, lo, hi);
    else
        hipLaunchKernelGGL((k_ntt1024<T, false, PPB>), grid, block, sm, s, in, out, count, tab, (T)p.Q, lo, hi);
    return hipGetLastError();
}

hipError_t ntt1024_launch(const NttPlan& p, const uint64_t* in, uint64_t* out, uint32_t count, bool inverse,
                          hipStream_t s) {
    if (p.wide) return launch<uint64_t, 4>(p, in, out, count, inverse, s);
    return launch<uint32_t, 8>(p, in, out, count, inverse, s);
}

}  // namespace fhe_amd
