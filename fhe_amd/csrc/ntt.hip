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
// One polynomial per wave64 (16 coefficients per lane) in three register layouts, two LDS
// transposes per transform: k_ntt1024w (32-bit residues, Q < 2^30) and k_ntt1024w64 (64-bit, Q < 2^62;
// the Sol60 policy for the poly-benchmark prime 2^60 - 2^14 + 1).  Global traffic = 8 B read + 8 B
// written per coefficient (u64 words, as the reference stores them); all arithmetic exact mod Q.
#include "arith.h"
#include "ntt.h"

namespace fhe_amd {

template <typename T>
struct ModT;


// 32-bit path (Q < 2^30): Harvey-style lazy butterflies.  Forward values live in
// [0, 4Q), inverse values in [0, 2Q); one correction at the end gives [0, Q).
// Shoup's lazy product x*w - floor(x*w'/2^32)*Q is in [0, 2Q) for any x < 2^32.
template <>
struct ModT<uint32_t> {
    using TW = uint2;  // (w, w' = floor(w 2^32 / Q))
    uint32_t Q, Q2;
    FHE_DEV uint32_t lazy_mul(uint32_t x, TW w) const { return mul_shoup_lazy(x, w.x, w.y, Q); }
    // CT: (x, y) in [0,4Q)^2 -> (x + wy, x - wy) in [0,4Q)^2
    FHE_DEV void ct(uint32_t& x, uint32_t& y, TW w) const {
        x = csub(x, Q2);
        const uint32_t t = lazy_mul(y, w);
        y = x + Q2 - t;
        x = x + t;
    }
    // GS: (x, y) in [0,2Q)^2 -> (x + y, (x - y) w) in [0,2Q)^2
    FHE_DEV void gs(uint32_t& x, uint32_t& y, TW w) const {
        const uint32_t d = x + Q2 - y;
        x = csub(x + y, Q2);
        y = lazy_mul(d, w);
    }
    // last inverse stage with N^-1 folded: ((x + y) n^-1, (x - y) w1 n^-1) in [0,Q)
    FHE_DEV void gs_last(uint32_t& x, uint32_t& y, TW lo, TW hi) const {
        const uint32_t d = x + Q2 - y;
        x = csub(lazy_mul(x + y, lo), Q);
        y = csub(lazy_mul(d, hi), Q);
    }
    FHE_DEV uint32_t fwd_out(uint32_t x) const { return csub(csub(x, Q2), Q); }
};

// ---------------------------------------------------------------------------------------------
// One polynomial per wave64 (32-bit path, Q < 2^30): 16 coefficients per lane, so a 4096-poly
// batch is 4096 waves (4 per SIMD) instead of 2048 pairs, and the butterflies of the polynomials
// whose reads have landed overlap the reads and writes of the others.  Index x (10 bits):
//   layout A: lane L = x5..x0,              register r  = x9..x6      (coalesced 8-byte rows)
//   layout B: lane L = (x9..x6) << 2 | x1x0, register r' = x5..x2
//   layout C: lane L = x7..x2,              register r'' = (x9x8) << 2 | x1x0  (4 consecutive words)
// Forward: A (stages 9..6, uniform twiddles) -> T1 -> B (stages 5..2) -> T2 -> C (stages 1, 0)
// -> stores of 4 consecutive u64 per lane and x9x8.  Inverse: the mirror image, C -> B -> A.
// LDS word address of x in both transposes: x + 4 (x >> 6) (conflict-free for the dword accesses
// of A and B; C reads/writes 16-byte runs).
// ---------------------------------------------------------------------------------------------
namespace {
constexpr int kWTile = 1024 + 64;  // words per wave
FHE_DEV int wt(int x) { return x + ((x >> 6) << 2); }

// k_ntt1024w64: staggered wave priorities.  With equal priority the waves sharing a SIMD interleave,
// finish together and leave all their stores for the end of the pass; ranked (waves 4..7 of a
// workgroup above 0..3, two per SIMD each), the high pair finishes first and its stores overlap the
// low pair's arithmetic.  Round 3, interleaved A/B (profiles/archive/r03_ab_ntt_prio.txt): 20.8 / 20.6 ->
// 20.0 / 20.2 us per 60-bit forward / inverse pass; four levels (by grid half too) and the 32-bit
// kernel gain nothing.
FHE_DEV void ntt_stagger(int wv) {
    if (__builtin_amdgcn_readfirstlane(wv >> 2)) __builtin_amdgcn_s_setprio(1);
}

// arithmetic policies of k_ntt1024w: Shoup lazy (any Q < 2^30) or signed Montgomery (Q < 2^27:
// five VALU instructions per butterfly, no reductions in the forward transform)
struct NttK {
    uint32_t Q;
    uint2 lo, hi;                           // Shoup: (N^-1, pre), (w1 N^-1, pre)
    uint32_t qinvp, oneR, ninvR, w1ninvR;   // signed: Q^-1 mod 2^32, 2^32 mod Q, Montgomery N^-1, w1 N^-1
};
struct ShoupA {
    using TW = uint2;
    static constexpr bool kSigned = false;
    ModT<uint32_t> m;
    uint2 lo, hi;
    FHE_DEV explicit ShoupA(const NttK& k) : m{k.Q, 2 * k.Q}, lo(k.lo), hi(k.hi) {}
    FHE_DEV void refresh() {}
    FHE_DEV void ct(uint32_t& x, uint32_t& y, TW w) const { m.ct(x, y, w); }
    FHE_DEV void gs(uint32_t& x, uint32_t& y, TW w) const { m.gs(x, y, w); }
    FHE_DEV void gs_last(uint32_t& x, uint32_t& y) const { m.gs_last(x, y, lo, hi); }
    FHE_DEV uint32_t fwd_out(uint32_t x) const { return m.fwd_out(x); }
    FHE_DEV uint32_t red(uint32_t x) const { return x; }
    // two consecutive twiddles
    FHE_DEV static void tw2(const TW* p, TW& a, TW& b) {
        const uint4 q = *reinterpret_cast<const uint4*>(p);
        a = make_uint2(q.x, q.y);
        b = make_uint2(q.z, q.w);
    }
};
struct SignedA {
    using TW = uint32_t;
    static constexpr bool kSigned = true;
    uint32_t Q, qinvp, oneR, ninvR, w1R;
    int32_t nQ;
    FHE_DEV explicit SignedA(const NttK& k)
        : Q(k.Q), qinvp(k.qinvp), oneR(k.oneR), ninvR(k.ninvR), w1R(k.w1ninvR), nQ(-(int32_t)k.Q) {}
    // -Q defined inside the caller's loop body, so that its sign extension is not hoisted out of
    // the loop (a hoisted 64-bit constant turns each product below into a 64 x 64 multiply)
    FHE_DEV void refresh() { asm volatile("" : "+s"(nQ)); }
    // a b 2^-32 mod Q in (-Q, Q) for |a| < 2^31 (a read as signed), bR < Q
    FHE_DEV uint32_t mul(uint32_t a, uint32_t bR) const {
        const int64_t t  = (int64_t)(int32_t)a * (int32_t)bR;
        const int32_t mm = (int32_t)((uint32_t)t * qinvp);
        return (uint32_t)((t + (int64_t)mm * nQ) >> 32);
    }
    FHE_DEV uint32_t canon(uint32_t r) const { return min(r, r + Q); }  // (-Q, Q) -> [0, Q)
    FHE_DEV void ct(uint32_t& x, uint32_t& y, TW w) const {
        const uint32_t t = mul(y, w);
        y = x - t;
        x = x + t;
    }
    FHE_DEV void gs(uint32_t& x, uint32_t& y, TW w) const {
        const uint32_t t = x + y;
        y = mul(x - y, w);
        x = t;
    }
    FHE_DEV void gs_last(uint32_t& x, uint32_t& y) const {
        const uint32_t s = x + y, d = x - y;
        x = canon(mul(s, ninvR));
        y = canon(mul(d, w1R));
    }
    FHE_DEV uint32_t fwd_out(uint32_t x) const { return canon(mul(x, oneR)); }
    FHE_DEV uint32_t red(uint32_t x) const { return mul(x, oneR); }
    FHE_DEV static void tw2(const TW* p, TW& a, TW& b) {
        const uint2 q = *reinterpret_cast<const uint2*>(p);
        a = q.x;
        b = q.y;
    }
};

// signed inverse: |x| + |y| of every butterfly must stay < 2^31 = 16 Q (units of Q/10 below);
// before stage s (execution order: C bit 0, C bit 1, B bits 0..3, A bits 0..2, last) register r is
// reduced to (-Q, Q) when red[s][r].  Bounds are uniform over a register within a layout and
// become the maximum at a transpose.
struct InvPlanW {
    bool red[10][16];
};
constexpr InvPlanW make_inv_plan_w() {
    InvPlanW p{};
    int B[16] = {};
    for (int r = 0; r < 16; ++r) B[r] = 10;
    const int bits[10] = {0, 1, 0, 1, 2, 3, 0, 1, 2, 3};
    for (int st = 0; st < 10; ++st) {
        if (st == 2 || st == 6) {
            int U = 0;
            for (int r = 0; r < 16; ++r) U = B[r] > U ? B[r] : U;
            for (int r = 0; r < 16; ++r) B[r] = U;
        }
        const int bt = bits[st];
        for (int r = 0; r < 16; ++r) {
            if (r & (1 << bt)) continue;
            const int q = r | (1 << bt);
            while (B[r] + B[q] > 160) {
                const int e  = B[r] >= B[q] ? r : q;
                B[e]         = 10;
                p.red[st][e] = true;
            }
            B[r] = B[r] + B[q];
            B[q] = 10;
        }
    }
    return p;
}

// PF: a persistent wave's next polynomial is loaded during the current one (batches larger than the
// resident grid); without it every wave transforms at most one polynomial and loads nothing more
template <bool INV, class A, bool PF>
__global__ void __launch_bounds__(512)
    k_ntt1024w(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, uint32_t count,
               const typename A::TW* __restrict__ tab, NttK K) {
    using TW = typename A::TW;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    TW* s_tw        = reinterpret_cast<TW*>(smem);                            // 1024 entries
    uint32_t* tiles = reinterpret_cast<uint32_t*>(smem + 1024 * sizeof(TW));  // 8 x kWTile
    const A a0(K);
    constexpr InvPlanW P = make_inv_plan_w();
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) s_tw[i] = tab[i];

    const int L     = threadIdx.x & 63;
    const int wv    = threadIdx.x >> 6;
    uint32_t* tile  = tiles + wv * kWTile;
    const int G = L >> 2, j = L & 3;  // layout B lane fields
    const uint32_t W = gridDim.x * (blockDim.x >> 6);
    uint32_t poly    = blockIdx.x * (blockDim.x >> 6) + wv;
    auto rowp        = [&](uint32_t p) -> uint32_t { return p < count ? p : count - 1; };

    // raw loads, both directions in layout A: the low word of 16 u64 rows of 512 B (the values are
    // below 2^32)
    using Raw = uint4[8];
    auto load = [&](Raw& buf, uint32_t p) {
        const uint32_t* s32 = reinterpret_cast<const uint32_t*>(in + (size_t)rowp(p) * 1024);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            buf[r].x = s32[2 * ((2 * r) * 64 + L)];
            buf[r].y = s32[2 * ((2 * r + 1) * 64 + L)];
        }
    };
    auto step = [&](Raw& buf, uint32_t p) {
        A m = a0;
        m.refresh();
        uint32_t v[16];
        if (!INV) {
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                v[2 * r]     = buf[r].x;
                v[2 * r + 1] = buf[r].y;
            }
            // A: stages 9..6 on register bits 3..0 (r = x9..x6)
#pragma unroll
            for (int b = 9; b >= 6; --b) {
                const int rb = b - 6;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    if (r & (1 << rb)) continue;
                    m.ct(v[r], v[r | (1 << rb)], tab[(1 << (9 - b)) + (r >> (rb + 1))]);
                }
            }
            // T1: A -> B
#pragma unroll
            for (int r = 0; r < 16; ++r) tile[wt((r << 6) | L)] = v[r];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = tile[wt((G << 6) | (r << 2) | j)];
            // B: stages 5..2 on register bits 3..0 (r' = x5..x2)
#pragma unroll
            for (int b = 5; b >= 2; --b) {
                const int rb = b - 2;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    if (r & (1 << rb)) continue;
                    m.ct(v[r], v[r | (1 << rb)], s_tw[(1 << (9 - b)) + (G << (5 - b)) + (r >> (rb + 1))]);
                }
            }
            // T2: B -> C (16-byte runs)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int r = 0; r < 16; ++r) tile[wt((G << 6) | (r << 2) | j)] = v[r];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int hh = 0; hh < 4; ++hh) {
                const uint4 q = *reinterpret_cast<const uint4*>(tile + wt((hh << 8) | (L << 2)));
                v[4 * hh] = q.x; v[4 * hh + 1] = q.y; v[4 * hh + 2] = q.z; v[4 * hh + 3] = q.w;
            }
            // C: stage 1 (pairs j, j ^ 2) and stage 0 (j, j ^ 1)
#pragma unroll
            for (int hh = 0; hh < 4; ++hh) {
                const TW w1 = s_tw[256 + (hh << 6) + L];
                m.ct(v[4 * hh], v[4 * hh + 2], w1);
                m.ct(v[4 * hh + 1], v[4 * hh + 3], w1);
                TW w0a, w0b;
                A::tw2(s_tw + 512 + (hh << 7) + (L << 1), w0a, w0b);
                m.ct(v[4 * hh], v[4 * hh + 1], w0a);
                m.ct(v[4 * hh + 2], v[4 * hh + 3], w0b);
            }
            uint64_t* dst = out + (size_t)rowp(p) * 1024;
            // T3: C -> A, then coalesced 512-byte rows
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int hh = 0; hh < 4; ++hh)
                *reinterpret_cast<uint4*>(tile + wt((hh << 8) | (L << 2))) =
                    make_uint4(m.fwd_out(v[4 * hh]), m.fwd_out(v[4 * hh + 1]), m.fwd_out(v[4 * hh + 2]), m.fwd_out(v[4 * hh + 3]));
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int r = 0; r < 16; ++r) dst[(r << 6) + L] = (uint64_t)tile[wt((r << 6) | L)];
        } else {
            // T3^-1: A (coalesced rows) -> C
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                tile[wt(((2 * r) << 6) | L)]     = buf[r].x;
                tile[wt(((2 * r + 1) << 6) | L)] = buf[r].y;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int hh = 0; hh < 4; ++hh) {
                const uint4 q = *reinterpret_cast<const uint4*>(tile + wt((hh << 8) | (L << 2)));
                v[4 * hh] = q.x; v[4 * hh + 1] = q.y; v[4 * hh + 2] = q.z; v[4 * hh + 3] = q.w;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // C: stage 0 then stage 1 (GS); signed: planned reductions (InvPlanW)
            auto redp = [&](int st) {
                if (A::kSigned) {
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        if (P.red[st][r]) v[r] = m.red(v[r]);
                }
            };
            redp(0);
#pragma unroll
            for (int hh = 0; hh < 4; ++hh) {
                TW w0a, w0b;
                A::tw2(s_tw + 512 + (hh << 7) + (L << 1), w0a, w0b);
                m.gs(v[4 * hh], v[4 * hh + 1], w0a);
                m.gs(v[4 * hh + 2], v[4 * hh + 3], w0b);
            }
            redp(1);
#pragma unroll
            for (int hh = 0; hh < 4; ++hh) {
                const TW w1 = s_tw[256 + (hh << 6) + L];
                m.gs(v[4 * hh], v[4 * hh + 2], w1);
                m.gs(v[4 * hh + 1], v[4 * hh + 3], w1);
            }
            // T2^-1: C -> B
#pragma unroll
            for (int hh = 0; hh < 4; ++hh)
                *reinterpret_cast<uint4*>(tile + wt((hh << 8) | (L << 2))) = make_uint4(v[4 * hh], v[4 * hh + 1], v[4 * hh + 2], v[4 * hh + 3]);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = tile[wt((G << 6) | (r << 2) | j)];
            // B: stages 2..5
#pragma unroll
            for (int b = 2; b <= 5; ++b) {
                const int rb = b - 2;
                redp(b);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    if (r & (1 << rb)) continue;
                    m.gs(v[r], v[r | (1 << rb)], s_tw[(1 << (9 - b)) + (G << (5 - b)) + (r >> (rb + 1))]);
                }
            }
            // T1^-1: B -> A
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int r = 0; r < 16; ++r) tile[wt((G << 6) | (r << 2) | j)] = v[r];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = tile[wt((r << 6) | L)];
            // A: stages 6..8, then bit 9 with N^-1 folded (transformnat-impl.h:599-623)
#pragma unroll
            for (int b = 6; b <= 8; ++b) {
                const int rb = b - 6;
                redp(b);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    if (r & (1 << rb)) continue;
                    m.gs(v[r], v[r | (1 << rb)], tab[(1 << (9 - b)) + (r >> (rb + 1))]);
                }
            }
            redp(9);
#pragma unroll
            for (int r = 0; r < 8; ++r) m.gs_last(v[r], v[r | 8]);
            uint64_t* dst = out + (size_t)rowp(p) * 1024;
#pragma unroll
            for (int r = 0; r < 16; ++r) dst[(r << 6) + L] = (uint64_t)v[r];
        }
        // the next step's T1 / T2^-1 writes reuse the tile
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    Raw bufA, bufB;
    if (poly < count) load(bufA, poly);
    __syncthreads();  // s_tw ready
    if (!PF) {  // one polynomial per wave: no clamped prefetch of a row nobody transforms
        if (poly < count) step(bufA, poly);
        return;
    }
    for (; poly < count; poly += 2 * W) {
        load(bufB, poly + W);
        __builtin_amdgcn_sched_barrier(0);
        step(bufA, poly);
        if (poly + W >= count) break;
        load(bufA, poly + 2 * W);
        __builtin_amdgcn_sched_barrier(0);
        step(bufB, poly + W);
    }
}

// ---------------------------------------------------------------------------------------------
// One polynomial per wave64 for 64-bit moduli (2^30 <= Q < 2^62): the layouts A / B / C of
// k_ntt1024w with 16 u64 coefficients per lane.  The transposes move the low and the high words as
// two 32-bit planes through the same conflict-free tile (word address x + 4 (x >> 6)).  Two
// arithmetic policies:
//   Lazy64 (any Q < 2^62): Harvey-lazy butterflies (forward values in [0, 4Q), inverse in [0, 2Q))
//          around Shoup's lazy product x w - hi(x w') Q in [0, 2Q);
//   Sol60  (Q = 2^60 - (2^S - 1): the poly-benchmark prime LastPrime(60, 2048) = 2^60 - 2^14 + 1):
//          Shoup's quotient without its low partial product (short by at most 2, product in
//          [0, 4Q)), q Q = (q << 60) - (q << S) + q by shifts, no reduction inside a butterfly: values
//          grow below 16 Q < 2^64 and a compile-time plan (Plan64) folds x -> x mod 2^60 + (x >> 60) c
//          only where a bound would pass 16 Q.  6 multiplies per butterfly instead of 10.
// ---------------------------------------------------------------------------------------------
struct Lazy64 {
    static constexpr bool kPlanned = false;
    uint64_t Q, Q2;
    ulonglong2 lo, hi;  // (N^-1, pre), (w1 N^-1, pre)
    FHE_DEV static uint64_t csub(uint64_t x, uint64_t m) { return x >= m ? x - m : x; }
    FHE_DEV uint64_t lazy_mul(uint64_t x, ulonglong2 w) const {
        return x * w.x - __umul64hi(x, w.y) * Q;
    }
    FHE_DEV void ct(uint64_t& x, uint64_t& y, ulonglong2 w) const {
        x = csub(x, Q2);
        const uint64_t t = lazy_mul(y, w);
        y = x + Q2 - t;
        x = x + t;
    }
    FHE_DEV void gs(uint64_t& x, uint64_t& y, ulonglong2 w, int) const {
        const uint64_t d = x + Q2 - y;
        x = csub(x + y, Q2);
        y = lazy_mul(d, w);
    }
    FHE_DEV void gs_last(uint64_t& x, uint64_t& y, int) const {
        const uint64_t d = x + Q2 - y;
        x = csub(lazy_mul(x + y, lo), Q);
        y = csub(lazy_mul(d, hi), Q);
    }
    FHE_DEV uint64_t fwd_out(uint64_t x) const { return csub(csub(x, Q2), Q); }
    FHE_DEV uint64_t fold(uint64_t x) const { return x; }
};

struct Sol60 {
    static constexpr bool kPlanned = true;
    uint64_t Q;
    uint32_t S;         // c = 2^S - 1
    ulonglong2 lo, hi;  // (N^-1, pre), (w1 N^-1, pre)
    // y w mod Q in [0, 4Q) for any y < 2^64 (w < Q, w.y = floor(w 2^64 / Q))
    FHE_DEV uint64_t mul(uint64_t y, ulonglong2 w) const {
        const uint32_t yl = (uint32_t)y, yh = (uint32_t)(y >> 32);
        const uint32_t pl = (uint32_t)w.y, ph = (uint32_t)(w.y >> 32);
        // y w' / 2^64 = yh ph + (yl ph + yh pl) / 2^32 + yl pl / 2^64: the high words of the middle
        // products and yh ph; the dropped fractions are < 3
        const uint64_t q = (uint64_t)yh * ph + __umulhi(yl, ph) + __umulhi(yh, pl);  // floor(y w' / 2^64) - {0, 1, 2}
        const uint32_t wl = (uint32_t)w.x, wh = (uint32_t)(w.x >> 32);
        const uint64_t p  = (uint64_t)yl * wl;
        // y w - q Q = P + (q << S) - D (mod 2^64; the true value is in [0, 4Q)), with P = y w mod 2^64
        // (one 32 x 32 -> 64 product, two low products into its high word) and D = q + (q << 60)
        // (high word (q << 28) + (q >> 32)): three adds, one 64-bit shift, one 64-bit subtract
        const uint32_t ph32 = (uint32_t)(p >> 32) + yl * wh + yh * wl;
        const uint64_t E = ((((uint64_t)ph32) << 32) | (uint32_t)p) + (q << S);
        // E - D as one subtract with borrow (the compiler splits D into its words and folds the high
        // one into the product's addend: a move and a negation more per product)
        uint32_t rl, rh;
        asm("v_sub_co_u32 %0, vcc, %4, %2\n\t"
            "v_lshl_add_u32 %1, %2, 28, %3\n\t"
            "v_subb_co_u32 %1, vcc, %5, %1, vcc"
            : "=&v"(rl), "=&v"(rh)
            : "v"((uint32_t)q), "v"((uint32_t)(q >> 32)), "v"((uint32_t)E), "v"((uint32_t)(E >> 32))
            : "vcc");
        return ((uint64_t)rh << 32) | rl;
    }
    // any x < 2^64 -> x mod 2^60 + (x >> 60) c < Q + 16 c < 2Q (bound 2 in the plan)
    FHE_DEV uint64_t fold(uint64_t x) const {
        const uint32_t k = (uint32_t)(x >> 60);
        return (x & ((1ull << 60) - 1)) + (uint64_t)((k << S) - k);
    }
    FHE_DEV uint64_t canon(uint64_t x) const {
        const uint64_t f = fold(x);
        return f >= Q ? f - Q : f;
    }
    // (x, a) -> (x + t, a - t): the borrow chain of the subtract with the add between its halves
    // (no wait state; the compiler puts an s_nop between adjacent halves)
    FHE_DEV static void add_sub(uint64_t& x, uint64_t a, uint64_t t, uint64_t& d) {
        uint32_t dl, dh;
        uint64_t s;
        asm("v_sub_co_u32 %0, vcc, %3, %5\n\t"
            "v_lshl_add_u64 %2, %7, 0, %8\n\t"
            "v_subb_co_u32 %1, vcc, %4, %6, vcc"
            : "=&v"(dl), "=&v"(dh), "=&v"(s)
            : "v"((uint32_t)a), "v"((uint32_t)(a >> 32)), "v"((uint32_t)t), "v"((uint32_t)(t >> 32)), "v"(x), "v"(t)
            : "vcc");
        x = s;
        d = ((uint64_t)dh << 32) | dl;
    }
    FHE_DEV void ct(uint64_t& x, uint64_t& y, ulonglong2 w) const {
        const uint64_t t = mul(y, w);
        add_sub(x, x + 4 * Q, t, y);
    }
    // k: the plan's bound of y (y < k Q), so x - y + k Q >= 0
    FHE_DEV void gs(uint64_t& x, uint64_t& y, ulonglong2 w, int k) const {
        uint64_t d;
        add_sub(x, x + (uint64_t)k * Q, y, d);
        y = mul(d, w);
    }
    FHE_DEV void gs_last(uint64_t& x, uint64_t& y, int k) const {
        const uint64_t d = x + (uint64_t)k * Q - y;
        x = canon(mul(x + y, lo));
        y = canon(mul(d, hi));
    }
    FHE_DEV uint64_t fwd_out(uint64_t x) const { return canon(x); }
};

// Sol60's bound plan, per stage (execution order) and register: fold before the stage, and the
// GS offset multiple.  Bounds are in units of Q (canonical 1, fold output 2, products 4); every value
// stays below 16 Q.  In a layout every element of a register has the same bound; a transpose mixes
// all registers (the maximum carries over).
struct Plan64 {
    bool fold[10][16];
    int k[10][16];
    bool fold_out[16];
};
// stage st's register bit and whether a transpose precedes it
constexpr int kFwdBit[10] = {3, 2, 1, 0, 3, 2, 1, 0, 1, 0};   // A 9..6, B 5..2, C 1, 0
constexpr int kInvBit[10] = {0, 1, 0, 1, 2, 3, 0, 1, 2, 3};   // C 0, 1, B 2..5, A 6..8, last
constexpr Plan64 make_plan64(bool inv) {
    Plan64 p{};
    int B[16] = {};
    for (int r = 0; r < 16; ++r) B[r] = 1;
    for (int st = 0; st < 10; ++st) {
        if ((!inv && (st == 4 || st == 8)) || (inv && (st == 2 || st == 6))) {
            int U = 0;
            for (int r = 0; r < 16; ++r) U = B[r] > U ? B[r] : U;
            for (int r = 0; r < 16; ++r) B[r] = U;
        }
        const int bt = inv ? kInvBit[st] : kFwdBit[st];
        for (int r = 0; r < 16; ++r) {
            if (r & (1 << bt)) continue;
            const int q = r | (1 << bt);
            if (!inv) {            // CT: x' = x + t, y' = x + 4Q - t, t < 4Q
                if (B[r] + 4 > 16) {
                    p.fold[st][r] = true;
                    B[r] = 2;
                }
                B[r] += 4;
                B[q] = B[r];
            } else {               // GS: x' = x + y, y' = (x + kQ - y) w < 4Q
                while (B[r] + B[q] > 16) {
                    const int e = B[r] >= B[q] ? r : q;
                    p.fold[st][e] = true;
                    B[e] = 2;
                }
                p.k[st][r] = B[q];
                B[r] = st == 9 ? 1 : B[r] + B[q];
                B[q] = st == 9 ? 1 : 4;
            }
        }
    }
    return p;
}

FHE_DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
FHE_DEV uint32_t lo32(uint64_t x) { return (uint32_t)x; }
FHE_DEV uint32_t hi32(uint64_t x) { return (uint32_t)(x >> 32); }

#ifndef FHE_NTT64_PHASE
#define FHE_NTT64_PHASE 0  // A/B: load phasing of k_ntt1024w64's co-resident waves (units of 1024 cycles)
#endif
#ifndef FHE_NTT64_WPS
#define FHE_NTT64_WPS 4  // k_ntt1024w64: waves per SIMD (register budget and grid size)
#endif

// PF: a persistent wave's next polynomial is loaded during the current one (batches larger than
// the resident grid); without it a wave holds one polynomial's registers (no spills)
template <bool INV, class M, bool PF>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(FHE_NTT64_WPS)))
    k_ntt1024w64(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, uint32_t count,
                 const ulonglong2* __restrict__ tab, M m) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    ulonglong2* s_tw = reinterpret_cast<ulonglong2*>(smem);                            // 1024 entries
    uint32_t* tiles  = reinterpret_cast<uint32_t*>(smem + 1024 * sizeof(ulonglong2));  // 8 x kWTile
    constexpr Plan64 P = make_plan64(INV);

    const int L    = threadIdx.x & 63;
    const int wv   = threadIdx.x >> 6;
    uint32_t* tile = tiles + wv * kWTile;
    const int G = L >> 2, j = L & 3;  // layout B lane fields
    const uint32_t W = gridDim.x * (blockDim.x >> 6);
    uint32_t poly    = blockIdx.x * (blockDim.x >> 6) + wv;

    // A (word address (r << 6) | L) <-> B ((G << 6) | (r << 2) | j), one 32-bit plane at a time
    auto a_to_b = [&](uint64_t (&v)[16]) {
        uint32_t h[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) { tile[wt((r << 6) | L)] = lo32(v[r]); h[r] = hi32(v[r]); }
        wave_sync();
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = tile[wt((G << 6) | (r << 2) | j)];
        wave_sync();
#pragma unroll
        for (int r = 0; r < 16; ++r) tile[wt((r << 6) | L)] = h[r];
        wave_sync();
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] |= (uint64_t)tile[wt((G << 6) | (r << 2) | j)] << 32;
        wave_sync();
    };
    auto b_to_a = [&](uint64_t (&v)[16]) {
        uint32_t h[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) { tile[wt((G << 6) | (r << 2) | j)] = lo32(v[r]); h[r] = hi32(v[r]); }
        wave_sync();
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = tile[wt((r << 6) | L)];
        wave_sync();
#pragma unroll
        for (int r = 0; r < 16; ++r) tile[wt((G << 6) | (r << 2) | j)] = h[r];
        wave_sync();
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] |= (uint64_t)tile[wt((r << 6) | L)] << 32;
        wave_sync();
    };
    // B <-> C (C: 4 consecutive words (hh << 8) | (L << 2) .. + 3, 16-byte runs)
    auto b_to_c = [&](uint64_t (&v)[16]) {
        uint32_t h[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) { tile[wt((G << 6) | (r << 2) | j)] = lo32(v[r]); h[r] = hi32(v[r]); }
        wave_sync();
#pragma unroll
        for (int hh = 0; hh < 4; ++hh) {
            const uint4 q = *reinterpret_cast<const uint4*>(tile + wt((hh << 8) | (L << 2)));
            v[4 * hh] = q.x; v[4 * hh + 1] = q.y; v[4 * hh + 2] = q.z; v[4 * hh + 3] = q.w;
        }
        wave_sync();
#pragma unroll
        for (int r = 0; r < 16; ++r) tile[wt((G << 6) | (r << 2) | j)] = h[r];
        wave_sync();
#pragma unroll
        for (int hh = 0; hh < 4; ++hh) {
            const uint4 q = *reinterpret_cast<const uint4*>(tile + wt((hh << 8) | (L << 2)));
            v[4 * hh] |= (uint64_t)q.x << 32; v[4 * hh + 1] |= (uint64_t)q.y << 32;
            v[4 * hh + 2] |= (uint64_t)q.z << 32; v[4 * hh + 3] |= (uint64_t)q.w << 32;
        }
        wave_sync();
    };
    auto c_to_b = [&](uint64_t (&v)[16]) {
        uint32_t h[16];
#pragma unroll
        for (int hh = 0; hh < 4; ++hh) {
            *reinterpret_cast<uint4*>(tile + wt((hh << 8) | (L << 2))) =
                make_uint4(lo32(v[4 * hh]), lo32(v[4 * hh + 1]), lo32(v[4 * hh + 2]), lo32(v[4 * hh + 3]));
#pragma unroll
            for (int e = 0; e < 4; ++e) h[4 * hh + e] = hi32(v[4 * hh + e]);
        }
        wave_sync();
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = tile[wt((G << 6) | (r << 2) | j)];
        wave_sync();
#pragma unroll
        for (int hh = 0; hh < 4; ++hh)
            *reinterpret_cast<uint4*>(tile + wt((hh << 8) | (L << 2))) =
                make_uint4(h[4 * hh], h[4 * hh + 1], h[4 * hh + 2], h[4 * hh + 3]);
        wave_sync();
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] |= (uint64_t)tile[wt((G << 6) | (r << 2) | j)] << 32;
        wave_sync();
    };
    // fold plan of stage st (Sol60)
    auto plan = [&](uint64_t (&v)[16], int st) {
        if (M::kPlanned) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (P.fold[st][r]) v[r] = m.fold(v[r]);
        }
    };
    // Global I/O needs no third transpose: the forward transform reads rows in layout A and writes
    // layout C (4 consecutive u64 per lane and x9x8: 32-byte runs), the inverse reads C and writes A
    using Raw = uint64_t[16];
    auto load = [&](Raw& buf, uint32_t p) {
        const uint64_t* src = in + (size_t)p * 1024;
        if (!INV) {
#pragma unroll
            for (int r = 0; r < 16; ++r) buf[r] = src[(r << 6) + L];
        } else {
#pragma unroll
            for (int hh = 0; hh < 4; ++hh) {
                const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(src + (hh << 8) + (L << 2));
                const ulonglong2 b = *reinterpret_cast<const ulonglong2*>(src + (hh << 8) + (L << 2) + 2);
                buf[4 * hh] = a.x; buf[4 * hh + 1] = a.y; buf[4 * hh + 2] = b.x; buf[4 * hh + 3] = b.y;
            }
        }
    };
    // forward layout A: stages 9..6, uniform twiddles from the global table (no LDS)
    auto stage_a = [&](Raw& v) {
#pragma unroll
        for (int b = 9; b >= 6; --b) {
            const int rb = b - 6;
            plan(v, 9 - b);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                if (r & (1 << rb)) continue;
                m.ct(v[r], v[r | (1 << rb)], tab[(1 << (9 - b)) + (r >> (rb + 1))]);
            }
        }
    };
    // pre: the A stages already ran (the first polynomial, ahead of the LDS table's barrier)
    auto step = [&](Raw& v, uint32_t p, bool pre) {
        uint64_t* dst = out + (size_t)p * 1024;
        if (!INV) {
            if (!pre) stage_a(v);
            a_to_b(v);
#pragma unroll
            for (int b = 5; b >= 2; --b) {
                const int rb = b - 2;
                plan(v, 9 - b);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    if (r & (1 << rb)) continue;
                    m.ct(v[r], v[r | (1 << rb)], s_tw[(1 << (9 - b)) + (G << (5 - b)) + (r >> (rb + 1))]);
                }
            }
            b_to_c(v);
            plan(v, 8);
#pragma unroll
            for (int hh = 0; hh < 4; ++hh) {
                const ulonglong2 w1 = s_tw[256 + (hh << 6) + L];
                m.ct(v[4 * hh], v[4 * hh + 2], w1);
                m.ct(v[4 * hh + 1], v[4 * hh + 3], w1);
            }
            plan(v, 9);
#pragma unroll
            for (int hh = 0; hh < 4; ++hh) {
                m.ct(v[4 * hh], v[4 * hh + 1], s_tw[512 + (hh << 7) + (L << 1)]);
                m.ct(v[4 * hh + 2], v[4 * hh + 3], s_tw[512 + (hh << 7) + (L << 1) + 1]);
            }
#pragma unroll
            for (int hh = 0; hh < 4; ++hh) {
                *reinterpret_cast<ulonglong2*>(dst + (hh << 8) + (L << 2)) =
                    ulonglong2{m.fwd_out(v[4 * hh]), m.fwd_out(v[4 * hh + 1])};
                *reinterpret_cast<ulonglong2*>(dst + (hh << 8) + (L << 2) + 2) =
                    ulonglong2{m.fwd_out(v[4 * hh + 2]), m.fwd_out(v[4 * hh + 3])};
            }
        } else {
            plan(v, 0);
#pragma unroll
            for (int hh = 0; hh < 4; ++hh) {
                m.gs(v[4 * hh], v[4 * hh + 1], s_tw[512 + (hh << 7) + (L << 1)], P.k[0][0]);
                m.gs(v[4 * hh + 2], v[4 * hh + 3], s_tw[512 + (hh << 7) + (L << 1) + 1], P.k[0][2]);
            }
            plan(v, 1);
#pragma unroll
            for (int hh = 0; hh < 4; ++hh) {
                const ulonglong2 w1 = s_tw[256 + (hh << 6) + L];
                m.gs(v[4 * hh], v[4 * hh + 2], w1, P.k[1][0]);
                m.gs(v[4 * hh + 1], v[4 * hh + 3], w1, P.k[1][1]);
            }
            c_to_b(v);
#pragma unroll
            for (int b = 2; b <= 5; ++b) {
                const int rb = b - 2;
                plan(v, b);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    if (r & (1 << rb)) continue;
                    m.gs(v[r], v[r | (1 << rb)], s_tw[(1 << (9 - b)) + (G << (5 - b)) + (r >> (rb + 1))], P.k[b][r]);
                }
            }
            b_to_a(v);
#pragma unroll
            for (int b = 6; b <= 8; ++b) {
                const int rb = b - 6;
                plan(v, b);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    if (r & (1 << rb)) continue;
                    m.gs(v[r], v[r | (1 << rb)], tab[(1 << (9 - b)) + (r >> (rb + 1))], P.k[b][r]);
                }
            }
            plan(v, 9);
#pragma unroll
            for (int r = 0; r < 8; ++r) m.gs_last(v[r], v[r | 8], P.k[9][r]);
#pragma unroll
            for (int r = 0; r < 16; ++r) dst[(r << 6) + L] = v[r];
        }
    };
    // the first polynomial's rows, then the twiddle table; the forward transform runs its layout-A
    // stages (uniform twiddles, no LDS) on the rows as they land, before the table's barrier
    Raw bufA;
#if FHE_NTT64_PHASE
    {  // A/B: the four waves of a SIMD request their rows one after the other, FHE_NTT64_PHASE x 1024 cycles apart
        uint32_t hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        const uint32_t slot = ((hw >> 16) & 1) * 2 + (uint32_t)__builtin_amdgcn_readfirstlane(wv >> 2);
        for (uint32_t z = 0; z < slot * FHE_NTT64_PHASE; ++z) __builtin_amdgcn_s_sleep(16);
    }
#endif
    if (poly < count) load(bufA, poly);
    ntt_stagger(wv);
    const ulonglong2 tw0 = tab[threadIdx.x], tw1 = tab[threadIdx.x + 512];  // 512 threads (launch_wave64)
    const bool pre = !INV && poly < count;
    if (pre) stage_a(bufA);
    s_tw[threadIdx.x]       = tw0;
    s_tw[threadIdx.x + 512] = tw1;
    __syncthreads();  // s_tw ready
    if (!PF) {
        for (bool first = true; poly < count; poly += W, first = false) {
            step(bufA, poly, first && pre);
            if (poly + W < count) load(bufA, poly + W);
        }
        return;
    }
    Raw bufB;
    for (; poly < count; poly += 2 * W) {
        const bool more = poly + W < count;   // wave-uniform
        if (more) load(bufB, poly + W);
        __builtin_amdgcn_sched_barrier(0);
        step(bufA, poly, pre && poly < 2 * W);
        if (!more) break;
        if (poly + 2 * W < count) load(bufA, poly + 2 * W);
        __builtin_amdgcn_sched_barrier(0);
        step(bufB, poly + W, false);
    }
}
}  // namespace

#ifndef FHE_NTT_WWPS
#define FHE_NTT_WWPS 5   // k_ntt1024w: resident waves per SIMD the grid is sized for
#endif

static hipError_t launch_wave(const NttPlan& p, const uint64_t* in, uint64_t* out, uint32_t count, bool inverse,
                              hipStream_t s) {
    if (count == 0) return hipSuccess;
    const bool sg = p.d_tabm_fwd != nullptr;  // Q < 2^27: signed Montgomery
    // 8 waves (polynomials) per workgroup; twiddles (8 or 4 KB) + 8 tiles of 4.25 KB
    const size_t sm       = 1024 * (sg ? 4 : 8) + (size_t)8 * kWTile * 4;
    const uint32_t groups = (count + 7) / 8;
    const uint32_t cap    = (uint32_t)p.cus * 4 * FHE_NTT_WWPS / 8;
    dim3 grid(groups < cap ? groups : cap), block(512);
    NttK k{};
    k.Q  = (uint32_t)p.Q;
    k.lo = uint2{(uint32_t)p.ninv, (uint32_t)p.ninv_pre};
    k.hi = uint2{(uint32_t)p.w1ninv, (uint32_t)p.w1ninv_pre};
    k.qinvp = p.qinvp; k.oneR = p.oneR; k.ninvR = p.ninvR; k.w1ninvR = p.w1ninvR;
    const bool pf = count > grid.x * 8u;   // more polynomials than resident waves
#define FHE_NTT32_LAUNCH(AT, TT, TAB)                                                                           \
    {                                                                                                          \
        const TT* tab = reinterpret_cast<const TT*>(TAB);                                                      \
        if (pf) {                                                                                              \
            if (inverse) hipLaunchKernelGGL((k_ntt1024w<true, AT, true>), grid, block, sm, s, in, out, count, tab, k); \
            else hipLaunchKernelGGL((k_ntt1024w<false, AT, true>), grid, block, sm, s, in, out, count, tab, k); \
        } else {                                                                                               \
            if (inverse) hipLaunchKernelGGL((k_ntt1024w<true, AT, false>), grid, block, sm, s, in, out, count, tab, k); \
            else hipLaunchKernelGGL((k_ntt1024w<false, AT, false>), grid, block, sm, s, in, out, count, tab, k); \
        }                                                                                                      \
    }
    if (sg) FHE_NTT32_LAUNCH(SignedA, uint32_t, inverse ? p.d_tabm_inv : p.d_tabm_fwd)
    else FHE_NTT32_LAUNCH(ShoupA, uint2, inverse ? p.d_tab_inv : p.d_tab_fwd)
#undef FHE_NTT32_LAUNCH
    return hipGetLastError();
}

static hipError_t launch_wave64(const NttPlan& p, const uint64_t* in, uint64_t* out, uint32_t count, bool inverse,
                                hipStream_t s) {
    if (count == 0) return hipSuccess;
    // 8 waves (polynomials) per workgroup; 16 KB of twiddles + 8 tiles of 4.25 KB
    const size_t sm       = 1024 * sizeof(ulonglong2) + (size_t)8 * kWTile * 4;
    const uint32_t groups = (count + 7) / 8;
    const uint32_t cap    = (uint32_t)p.cus * 4 * FHE_NTT64_WPS / 8;
    dim3 grid(groups < cap ? groups : cap), block(512);
    const ulonglong2* tab = reinterpret_cast<const ulonglong2*>(inverse ? p.d_tab_inv : p.d_tab_fwd);
    const ulonglong2 lo{p.ninv, p.ninv_pre}, hi{p.w1ninv, p.w1ninv_pre};
    const bool pf = count > grid.x * 8u;   // more polynomials than resident waves
#define FHE_NTT64_LAUNCH(MT, PF_)                                                                              \
    if (inverse) hipLaunchKernelGGL((k_ntt1024w64<true, MT, PF_>), grid, block, sm, s, in, out, count, tab, m); \
    else hipLaunchKernelGGL((k_ntt1024w64<false, MT, PF_>), grid, block, sm, s, in, out, count, tab, m)
    if (p.sol_shift) {  // Q = 2^60 - (2^S - 1): Sol60
        const Sol60 m{p.Q, p.sol_shift, lo, hi};
        if (pf) { FHE_NTT64_LAUNCH(Sol60, true); } else { FHE_NTT64_LAUNCH(Sol60, false); }
    } else {
        const Lazy64 m{p.Q, 2 * p.Q, lo, hi};
        if (pf) { FHE_NTT64_LAUNCH(Lazy64, true); } else { FHE_NTT64_LAUNCH(Lazy64, false); }
    }
#undef FHE_NTT64_LAUNCH
    return hipGetLastError();
}

hipError_t ntt1024_launch(const NttPlan& p, const uint64_t* in, uint64_t* out, uint32_t count, bool inverse,
                          hipStream_t s) {
    if (p.wide) return launch_wave64(p, in, out, count, inverse, s);
    return launch_wave(p, in, out, count, inverse, s);
}

}  // namespace fhe_amd
