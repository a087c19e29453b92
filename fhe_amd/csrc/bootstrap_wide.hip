// bootstrap_wide.hip -- gate / functional bootstrapping of the large-precision family
// (boot_wide.h): 64-bit accumulator residues, N = 2048 (or 1024).
//
// One workgroup of N/4 threads per bootstrap.  Thread t owns the EVALUATION slots
// j = t + (N/4) r, r < 4, of both accumulator polynomials in registers; the transforms run
// radix-2 through one 2N-word LDS buffer (two polynomials at once).  Per accumulator index i
// (rgsw-acc-cggi.cpp:59-151), skipped when its monomial exponent is 0 (X^0 - 1 = 0):
//   1. both accumulators to COEF (inverse NTT, the N^-1 folded into the coefficient reads);
//   2. SignedDigitDecompose (rgsw-acc.cpp:54-91) kept as a running signed 64-bit state per
//      coefficient, one gadget level at a time: level L's two digit polynomials (from acc0 and
//      acc1) are written to LDS and forward-transformed;
//   3. every slot accumulates digit x key products for the 2 signs x 2 components in 128 bits
//      (keys stored in Montgomery form K 2^64 mod Q: one reduction per sum);
//   4. acc_c += S+_c (X^m - 1) + S-_c (X^-m - 1), the monomials EVAL(X^m) = psi^((2 brv(j)+1) m)
//      from one 2N-entry power table.
// Keys are read straight from HBM, coalesced (consecutive threads, consecutive slots).
// Two arithmetic policies share the code: A64 (64-bit residues, any Q < 2^62) and A32 (32-bit residues
// for Q < 2^30 with digitsG2 Q < 2^32: the N = 2048 STD256* / STD256Q* rows, SIGNED_MOD_TEST, TOY):
// Shoup products x w - hi(x w') Q in one 32 x 32 multiply pair, digit x key sums in 64 bits, one
// Montgomery (R = 2^32) reduction per sum -- a third of A64's multiplies and half its LDS words.
#include "boot_wide.h"

#include <algorithm>

// waves per SIMD the blind-rotation kernel is compiled for (VGPR budget 512 / waves)
#ifndef FHE_WIDE_WAVES
#define FHE_WIDE_WAVES 4
#endif
// the A32 instantiations: the gate kernel at 4 (113 VGPRs, 64 KB of LDS with its tables; with the
// monomial table through the caches and 6 waves it spills 14 VGPRs and runs 21-29% slower), the
// op-list kernel at 6 (80 VGPRs: +8% on STD256_LMKCDEY / STD256Q_3_LMKCDEY, profiles/archive/r03_bench_sets_narrow.txt)
#ifndef FHE_WIDE32_WAVES
#define FHE_WIDE32_WAVES 4
#endif
#ifndef FHE_WIDE32_OPS_WAVES
#define FHE_WIDE32_OPS_WAVES 6
#endif

namespace fhe_amd {

namespace {
#define WD __device__ __forceinline__

struct U128 {
    uint64_t lo, hi;
};

// RoundqQ(v, q, Q) = floor(0.5 + double(v) double(q) / double(Q)) mod q (lwe-pke.cpp:41-46), in
// IEEE double like the reference (no contraction: the product is divided before the add)
WD uint64_t round_qQ(uint64_t v, uint64_t q, uint64_t Q) {
#pragma clang fp contract(off)
    const double x = (double)v * (double)q / (double)Q;
    return (uint64_t)floor(0.5 + x) % q;
}

// 64-bit residues: Shoup products, 128-bit sums, Montgomery R = 2^64 (keys K 2^64 mod Q)
struct A64 {
    using T = uint64_t;
    using S = U128;
    using D = int64_t;   // SignedDigitDecompose state
    using UD = uint64_t;
    static constexpr int kWaves = FHE_WIDE_WAVES, kOpsWaves = FHE_WIDE_WAVES;
    static constexpr bool kLds = false;  // tables read through the caches (32 KB of LDS per gate already)
    const uint64_t *tab, *tabS, *tabI, *tabIS, *psiM;
    uint64_t Q, qinv, ninv, ninvS, oneM;
    WD explicit A64(const WideTables& t)
        : tab(t.tab), tabS(t.tabS), tabI(t.tabI), tabIS(t.tabIS), psiM(t.psiM), Q(t.Q), qinv(t.qinv), ninv(t.ninv),
          ninvS(t.ninvS), oneM(t.oneM) {}
    WD static S zero() { return U128{0, 0}; }
    WD static void mac(S& s, T a, T b) {
        const uint64_t lo = a * b, hi = __umul64hi(a, b);
        s.lo += lo;
        s.hi += hi + (s.lo < lo ? 1 : 0);
    }
    // t < Q 2^64  ->  t 2^-64 mod Q in [0, Q)
    WD T redc(const S& t) const {
        const uint64_t u = t.lo * qinv;
        const uint64_t r = t.hi + __umul64hi(u, Q) + (t.lo != 0 ? 1 : 0);
        return r >= Q ? r - Q : r;
    }
    // x w mod Q for w < Q, ws = floor(w 2^64 / Q), any 64-bit x
    WD T mul_shoup(T x, T w, T ws) const {
        const uint64_t r = x * w - __umul64hi(x, ws) * Q;
        return r >= Q ? r - Q : r;
    }
    WD T add(T a, T b) const {
        const T s = a + b;
        return s >= Q ? s - Q : s;
    }
    WD T sub(T a, T b) const { return a >= b ? a - b : a + Q - b; }
    // butterflies on canonical values
    WD void ct(T& x, T& y, T w, T ws) const {
        const T V = mul_shoup(y, w, ws);
        y = sub(x, V);
        x = add(x, V);
    }
    WD void gs(T& x, T& y, T w, T ws) const {
        const T U = x;
        x = add(U, y);
        y = mul_shoup(sub(U, y), w, ws);
    }
    WD T fwd_out(T x) const { return x; }
};
// 32-bit residues for Q < 2^30: the same operations one word wide (keys K 2^32 mod Q); the unreduced
// digit x key sums stay below digitsG2 Q^2 < Q 2^32 (Engine checks digitsG2 Q < 2^32), so one
// reduction lands in [0, 2Q)
struct A32 {
    using T = uint32_t;
    using S = uint64_t;
    using D = int32_t;   // |centred value| < Q/2 < 2^29: the decomposition in 32-bit words
    using UD = uint32_t;
    static constexpr int kWaves = FHE_WIDE32_WAVES, kOpsWaves = FHE_WIDE32_OPS_WAVES;
    // the twiddle (and monomial) tables staged in LDS once per gate: every transform pass reads its
    // twiddles right before use, so cached global reads left their latency exposed
    static constexpr bool kLds = true;
    const uint32_t *tab, *tabS, *tabI, *tabIS, *psiM;
    uint32_t Q, qinv, ninv, ninvS, oneM;
    WD explicit A32(const WideTables& t)
        : tab(t.tab32), tabS(t.tabS32), tabI(t.tabI32), tabIS(t.tabIS32), psiM(t.psiM32), Q(t.Q32), qinv(t.qinv32),
          ninv(t.ninv32), ninvS(t.ninvS32), oneM(t.oneM32) {}
    WD static S zero() { return 0; }
    WD static void mac(S& s, T a, T b) { s += (uint64_t)a * b; }
    WD T redc(S t) const {
        const uint32_t u = (uint32_t)t * qinv;
        const uint32_t r = (uint32_t)((t + (uint64_t)u * Q) >> 32);
        return r >= Q ? r - Q : r;
    }
    // x w mod Q for w < Q, ws = floor(w 2^32 / Q), any 32-bit x: x w - hi(x ws) Q in [0, 2Q)
    WD T mul_shoup(T x, T w, T ws) const {
        const uint32_t r = x * w - __umulhi(x, ws) * Q;
        return r >= Q ? r - Q : r;
    }
    WD T add(T a, T b) const {
        const T s = a + b;
        return s >= Q ? s - Q : s;
    }
    WD T sub(T a, T b) const { return a >= b ? a - b : a + Q - b; }
    // Harvey-lazy butterflies (4Q < 2^32): the forward transform keeps values in [0, 4Q) and ends
    // canonical (fwd_out), the inverse keeps [0, 2Q) (its readers reduce through mul_shoup)
    WD static T csub(T x, T m) { return x >= m ? x - m : x; }
    WD T lazy_mul(T x, T w, T ws) const { return x * w - __umulhi(x, ws) * Q; }  // [0, 2Q)
    WD void ct(T& x, T& y, T w, T ws) const {
        const T X = csub(x, 2 * Q);
        const T t = lazy_mul(y, w, ws);
        y = X + 2 * Q - t;
        x = X + t;
    }
    WD void gs(T& x, T& y, T w, T ws) const {
        const T U = x;
        x = csub(U + y, 2 * Q);
        y = lazy_mul(U + 2 * Q - y, w, ws);
    }
    WD T fwd_out(T x) const { return csub(csub(x, 2 * Q), Q); }
};

// Workgroup barrier for the accumulator kernels, whose threads share data through LDS only: a
// workgroup-scope fence on LDS ("local") waits for LDS accesses alone, so global loads issued before
// it (the A32 gate kernel's next-level keys) stay in flight across it; __syncthreads would drain them
WD void wg_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// A32 gate kernel: copy the tables into LDS and point the policy at them (+2.6% at STD256).
// Engine::build_tables_wide stores them contiguously (tab, tabS, tabI, tabIS: N words each, then
// psiM: 2N words); mono = false would leave the monomial table out
template <class A>
WD void stage_tables(A& a, typename A::T* st, int N, bool mono) {
    if constexpr (A::kLds) {
        const int words = (mono ? 6 : 4) * N;
        for (int i = threadIdx.x; i < words; i += blockDim.x) st[i] = a.tab[i];
        wg_sync();
        a.tab = st;
        a.tabS = st + N;
        a.tabI = st + 2 * N;
        a.tabIS = st + 3 * N;
        if (mono) a.psiM = st + 4 * N;
    }
}

// Orders one wave's LDS accesses (the next pass reads only what this wave wrote)
WD void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Merged Cooley-Tukey forward transform in place on NB polynomials at buf + p N (bit-reversed
// output, ForwardTransformToBitReverseInPlace transformnat-impl.h:302-373); all threads, synced.
template <int LOGN, int NB, class A>
WD void ntt_fwd(typename A::T* buf, const A& a) {
    constexpr int N = 1 << LOGN, T = N / 4;
#pragma unroll 1
    for (int s = 0; s < LOGN; ++s) {
        const int logt = LOGN - 1 - s, t = 1 << logt;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int b = (int)threadIdx.x + T * k;
            const int i = b >> logt;
            const int j = (i << (logt + 1)) | (b & (t - 1));
            const auto w = a.tab[(1 << s) + i], ws = a.tabS[(1 << s) + i];
#pragma unroll
            for (int p = 0; p < NB; ++p) {
                auto x = buf[p * N + j], y = buf[p * N + j + t];
                a.ct(x, y, w, ws);
                if (s == LOGN - 1) {
                    x = a.fwd_out(x);
                    y = a.fwd_out(y);
                }
                buf[p * N + j]     = x;
                buf[p * N + j + t] = y;
            }
        }
        wg_sync();
    }
}
// Gentleman-Sande inverse (InverseTransformFromBitReverseInPlace :511-624) WITHOUT the final
// N^-1 scaling (the readers apply it)
template <int LOGN, int NB, class A>
WD void ntt_inv(typename A::T* buf, const A& a) {
    constexpr int N = 1 << LOGN, T = N / 4;
#pragma unroll 1
    for (int s = 0; s < LOGN; ++s) {
        const int logt = s, t = 1 << logt, m = N >> (s + 1);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int b = (int)threadIdx.x + T * k;
            const int i = b >> logt;
            const int j = (i << (logt + 1)) | (b & (t - 1));
            const auto w = a.tabI[m + i], ws = a.tabIS[m + i];
#pragma unroll
            for (int p = 0; p < NB; ++p) {
                auto x = buf[p * N + j], y = buf[p * N + j + t];
                a.gs(x, y, w, ws);
                buf[p * N + j]     = x;
                buf[p * N + j + t] = y;
            }
        }
        wg_sync();
    }
}

// Radix-4 passes of the same transforms: each thread takes whole 4-element units through two
// stages between syncs, an odd last stage radix-2.  Wave w's 64 units of a pass whose butterfly
// blocks hold at most 64 units (forward distance t <= 128, inverse t <= 64; the last forward radix-2
// stage remapped) lie in elements [256 w, 256 w + 256) of each polynomial, so consecutive such
// passes synchronise the wave only; a workgroup barrier follows the passes that cross chunks and the
// last pass (N = 2048: 3 barriers per transform instead of 6).
template <int LOGN, int NB, class A>
WD void ntt_fwd4(typename A::T* buf, const A& a) {
    constexpr int N = 1 << LOGN;
    const int u = (int)threadIdx.x;  // one unit per thread per polynomial
#pragma unroll 1
    for (int s = 0; s + 1 < LOGN; s += 2) {
        const int logt = LOGN - 1 - s, t = 1 << logt, th = t >> 1, m = 1 << s;
        const int i = u >> (logt - 1), k = u & (th - 1);
        const int j0 = (i << (logt + 1)) + k;
        const auto w = a.tab[m + i], ws = a.tabS[m + i];
        const auto w1 = a.tab[2 * m + 2 * i], w1s = a.tabS[2 * m + 2 * i];
        const auto w2 = a.tab[2 * m + 2 * i + 1], w2s = a.tabS[2 * m + 2 * i + 1];
        const bool last = !(LOGN & 1) && s + 2 == LOGN;
#pragma unroll
        for (int p = 0; p < NB; ++p) {
            auto* b = buf + p * N + j0;
            auto x0 = b[0], x1 = b[th], x2 = b[t], x3 = b[t + th];
            a.ct(x0, x2, w, ws);
            a.ct(x1, x3, w, ws);
            a.ct(x0, x1, w1, w1s);
            a.ct(x2, x3, w2, w2s);
            if (last) {
                x0 = a.fwd_out(x0); x1 = a.fwd_out(x1); x2 = a.fwd_out(x2); x3 = a.fwd_out(x3);
            }
            b[0] = x0;
            b[th] = x1;
            b[t] = x2;
            b[t + th] = x3;
        }
        // this pass stayed in the wave's chunk (logt <= 7) and so does what follows: another radix-4
        // pass or the remapped radix-2 stage (not the end of the transform)
        const bool more4 = s + 3 < LOGN, r2next = (LOGN & 1) && s + 3 == LOGN;
        if (logt <= 7 && (more4 || r2next)) wave_sync();
        else wg_sync();
    }
    if (LOGN & 1) {  // last stage: t = 1, m = N / 2; wave w takes butterflies [128 w, 128 w + 128)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int bf = ((u >> 6) << 7) + (u & 63) + 64 * k;
            const auto w = a.tab[N / 2 + bf], ws = a.tabS[N / 2 + bf];
#pragma unroll
            for (int p = 0; p < NB; ++p) {
                auto* b = buf + p * N + 2 * bf;
                auto x = b[0], y = b[1];
                a.ct(x, y, w, ws);
                b[0] = a.fwd_out(x);
                b[1] = a.fwd_out(y);
            }
        }
        wg_sync();
    }
}
template <int LOGN, int NB, class A>
WD void ntt_inv4(typename A::T* buf, const A& a) {
    constexpr int N = 1 << LOGN, T = N / 4;
    const int u = (int)threadIdx.x;
#pragma unroll 1
    for (int s = 0; s + 1 < LOGN; s += 2) {
        const int t = 1 << s, m = N >> (s + 1);
        const int i = u >> s, k = u & (t - 1);
        const int e0 = (i << (s + 2)) + k;
        const auto wa = a.tabI[m + 2 * i], was = a.tabIS[m + 2 * i];
        const auto wb = a.tabI[m + 2 * i + 1], wbs = a.tabIS[m + 2 * i + 1];
        const auto w2 = a.tabI[(m >> 1) + i], w2s = a.tabIS[(m >> 1) + i];
#pragma unroll
        for (int p = 0; p < NB; ++p) {
            auto* b = buf + p * N + e0;
            auto x0 = b[0], x1 = b[t], x2 = b[2 * t], x3 = b[3 * t];
            a.gs(x0, x1, wa, was);
            a.gs(x2, x3, wb, wbs);
            a.gs(x0, x2, w2, w2s);
            a.gs(x1, x3, w2, w2s);
            b[0] = x0;
            b[t] = x1;
            b[2 * t] = x2;
            b[3 * t] = x3;
        }
        // within this wave's chunk while this pass and the next have t <= 64 (s + 2 <= 6)
        if (s + 2 <= 6 && s + 3 < LOGN) wave_sync();
        else wg_sync();
    }
    if (LOGN & 1) {  // last stage: t = N / 2, m = 1
        const auto w = a.tabI[1], ws = a.tabIS[1];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int j = u + T * k;
#pragma unroll
            for (int p = 0; p < NB; ++p) {
                auto* b = buf + p * N + j;
                auto x = b[0], y = b[N / 2];
                a.gs(x, y, w, ws);
                b[0] = x;
                b[N / 2] = y;
            }
        }
        wg_sync();
    }
}

#ifndef FHE_WIDE_R4
#define FHE_WIDE_R4 1
#endif
template <int LOGN, int NB, class A>
WD void fwd(typename A::T* buf, const A& a) {
    if (FHE_WIDE_R4) ntt_fwd4<LOGN, NB>(buf, a);
    else ntt_fwd<LOGN, NB>(buf, a);
}
template <int LOGN, int NB, class A>
WD void inv(typename A::T* buf, const A& a) {
    if (FHE_WIDE_R4) ntt_inv4<LOGN, NB>(buf, a);
    else ntt_inv<LOGN, NB>(buf, a);
}
}  // namespace

template <int LOGN, class A>
__global__ void __launch_bounds__((1 << LOGN) / 4, A::kWaves)
    k_blind_rotate_wide(WideArgs g, WideTables tb, const typename A::T* __restrict__ bsk,
                        const uint16_t* __restrict__ idx, const uint32_t* __restrict__ tvb, uint64_t* __restrict__ ext_a,
                        uint64_t* __restrict__ ext_b) {
    using T = typename A::T;
    using Sum = typename A::S;
    constexpr int N = 1 << LOGN, TH = N / 4, S = 4;
    __shared__ T buf[2 * N];
    __shared__ T stab[A::kLds ? 6 * N : 1];
    A a(tb);
    stage_tables(a, stab, N, true);
    const uint32_t gate = blockIdx.x, t = threadIdx.x;
    const T Q = a.Q, QHalf = Q >> 1;
    using D = typename A::D;
    using UD = typename A::UD;
    const uint32_t dG2 = (g.digitsG - 1) * 2, gb = g.gbits, sh = 8 * sizeof(D) - gb;

    // test vector (BootstrapGateCore binfhe-base-scheme.cpp:556-575 / BootstrapFuncCore :596-608):
    // acc1 = NTT(m), acc0 = 0
    T acc0[S], acc1[S];
    if (g.acc_io && !g.acc_tv) {  // the seam's accumulator (EvalAcc on a given acc)
        const uint64_t* src = g.acc_io + (size_t)gate * 2 * N;
#pragma unroll
        for (int r = 0; r < S; ++r) {
            acc0[r] = (T)src[t + TH * r];
            acc1[r] = (T)src[N + t + TH * r];
        }
    } else {
        const uint32_t b = tvb[gate], cm = g.ctmod - 1;
        // EvalFuncMultiOutput: table gate % tv_mod (GateArgs::tv_mod)
        const uint32_t tvo = g.tv_mod > 1 ? (gate % g.tv_mod) * g.ctmod : 0u;
#pragma unroll
        for (int r = 0; r < S; ++r) {
            const uint32_t x = t + TH * r;
            uint64_t v = 0;
            if (x % g.factor == 0) {
                const uint32_t bx = (b - x / g.factor) & cm;
                v = g.tv ? g.tv[tvo + bx] : (bx >= g.lb && bx < g.ub) ? g.lv : g.uv;
            }
            buf[x] = (T)v;
        }
        wg_sync();
        fwd<LOGN, 1>(buf, a);
#pragma unroll
        for (int r = 0; r < S; ++r) {
            acc0[r] = 0;
            acc1[r] = buf[t + TH * r];
        }
    }

    const uint16_t* gi = idx + (size_t)gate * g.n;
    const size_t key_stride = (size_t)2 * dG2 * 2 * N;  // [2 signs][dG2][2][N] per index
#pragma unroll 1
    for (uint32_t i = 0; i < g.n; ++i) {
        const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)gi[i]);
        if (m == 0) continue;  // AddToAccCGGI with X^0 - 1 = 0 leaves acc unchanged
        wg_sync();
#pragma unroll
        for (int r = 0; r < S; ++r) {
            buf[t + TH * r]     = acc0[r];
            buf[N + t + TH * r] = acc1[r];
        }
        wg_sync();
        inv<LOGN, 2>(buf, a);
        // SignedDigitDecompose state: centred value, lowest digit dropped
        D d[2][S];
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int r = 0; r < S; ++r) {
                const T v = a.mul_shoup(buf[p * N + t + TH * r], a.ninv, a.ninvS);
                D x = v < QHalf ? (D)v : (D)v - (D)Q;
                const D r0 = (D)((UD)x << sh) >> sh;
                d[p][r] = (x - r0) >> gb;
            }
        Sum acc[2][2][S];  // [sign][component][slot]
#pragma unroll
        for (int sg = 0; sg < 2; ++sg)
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int r = 0; r < S; ++r) acc[sg][c][r] = A::zero();
        const T* key = bsk + (size_t)i * key_stride;
#pragma unroll 1
        for (uint32_t L = 0; 2 * L < dG2; ++L) {
            // A32: this level's 32 key words per thread requested before its digit transform, so they
            // land during it (wg_sync's LDS-only barriers do not drain them): +1.2% on the N = 2048
            // GINX rows, 121 VGPRs (profiles/archive/r03_ab_wide.txt; the op-list kernel's EXT keys the same
            // way lose 1% at 6 waves per SIMD with spills, 7% at 5)
            constexpr bool kpf = sizeof(T) == 4;
            T kr[kpf ? 2 : 1][2][2][kpf ? S : 1];
            if (kpf) {
#pragma unroll
                for (int sg = 0; sg < 2; ++sg)
#pragma unroll
                    for (int c = 0; c < 2; ++c)
#pragma unroll
                        for (int w = 0; w < 2; ++w)
#pragma unroll
                            for (int r = 0; r < S; ++r)
                                kr[sg][c][w][r] = key[((size_t)(sg * dG2 + 2 * L + w) * 2 + c) * N + t + TH * r];
            }
            wg_sync();  // previous readers of buf are done
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int r = 0; r < S; ++r) {
                    const D x = d[p][r];
                    D r0 = (D)((UD)x << sh) >> sh;
                    d[p][r] = (x - r0) >> gb;
                    if (r0 < 0) r0 += (D)Q;
                    buf[p * N + t + TH * r] = (T)r0;
                }
            wg_sync();
            fwd<LOGN, 2>(buf, a);
#pragma unroll
            for (int r = 0; r < S; ++r) {
                const uint32_t j = t + TH * r;
                const T x0 = buf[j], x1 = buf[N + j];
#pragma unroll
                for (int sg = 0; sg < 2; ++sg)
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const T* k0 = key + ((size_t)(sg * dG2 + 2 * L) * 2 + c) * N;
                        A::mac(acc[sg][c][r], x0, kpf ? kr[sg][c][0][kpf ? r : 0] : k0[j]);
                        A::mac(acc[sg][c][r], x1, kpf ? kr[sg][c][1][kpf ? r : 0] : k0[2 * N + j]);  // row 2L + 1
                    }
            }
        }
        // acc_c += S+_c (X^m - 1) + S-_c (X^-m - 1)
        const uint32_t mneg = 2 * N - m, emask = 2 * N - 1;
#pragma unroll
        for (int r = 0; r < S; ++r) {
            const uint32_t j = t + TH * r;
            const uint32_t e = 2 * (__brev(j) >> (32 - LOGN)) + 1;
            const T mp = a.sub(a.psiM[(e * m) & emask], a.oneM);
            const T mn = a.sub(a.psiM[(e * mneg) & emask], a.oneM);
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                Sum z = A::zero();
                A::mac(z, a.redc(acc[0][c][r]), mp);
                A::mac(z, a.redc(acc[1][c][r]), mn);
                const T add = a.redc(z);
                if (c == 0) acc0[r] = a.add(acc0[r], add);
                else acc1[r] = a.add(acc1[r], add);
            }
        }
    }

    if (g.acc_io) {  // the seam: the accumulator itself (block-uniform branch)
        uint64_t* dst = g.acc_io + (size_t)gate * 2 * N;
#pragma unroll
        for (int r = 0; r < S; ++r) {
            dst[t + TH * r]     = acc0[r];
            dst[N + t + TH * r] = acc1[r];
        }
        return;
    }
    // extraction (binfhe-base-scheme.cpp:110-121, :616-626): Transpose(acc0) then COEF: coefficient
    // k of acc0(X^-1) is -a_(N-k) (k >= 1), a_0 for k = 0; b = b_const + acc1[0]
    wg_sync();
#pragma unroll
    for (int r = 0; r < S; ++r) {
        buf[t + TH * r]     = acc0[r];
        buf[N + t + TH * r] = acc1[r];
    }
    wg_sync();
    inv<LOGN, 2>(buf, a);
    uint64_t* oa = ext_a + (size_t)gate * N;
#pragma unroll
    for (int r = 0; r < S; ++r) {
        const uint32_t x = t + TH * r;
        const T c = a.mul_shoup(buf[x == 0 ? 0 : N - x], a.ninv, a.ninvS);
        const uint64_t v = (x == 0 || c == 0) ? c : Q - c;
        oa[x] = g.msb_out ? round_qQ(v, g.qKS, Q) : v;
    }
    if (t == 0) {
        const uint64_t bb = a.add((T)(g.b_const % Q), a.mul_shoup(buf[N], a.ninv, a.ninvS));
        ext_b[gate] = g.msb_out ? round_qQ(bb, g.qKS, Q) : bb;
    }
}

// ---------------------------------------------------------------------------
// LMKCDEY (rgsw-acc-lmkcdey.cpp:70-287) and DM (rgsw-acc-dm.cpp:62-145) on the wide accumulator:
// the per-gate op list of k_prep_lmk_w / k_prep_dm_w, in the work split of k_blind_rotate_wide.
//   EXT(i)  (AddToAccLMKCDEY / AddToAccDM): both accumulators to COEF, digitsG - 1 gadget levels of
//           both (rows 2L / 2L + 1 of ek[i]), acc_c <- sum_rows D x ek[i][row][c]  (acc replaced);
//   AUTO(t) (Automorphism, k = 5^t, or 2N - 5 for t = 0): acc <- sigma_k(acc) in EVAL (a slot
//           permutation), acc0' alone to COEF and decomposed, acc0 <- sum_L D_L x ak[t][L][0],
//           acc1 <- acc1' + sum_L D_L x ak[t][L][1].
// LMKCDEY starts with acc1 <- sigma_(2N-5)(acc1) (:99).  Keys in Montgomery form, one reduction per
// slot and component.
// ---------------------------------------------------------------------------
namespace {
// EVAL slot j holds the value at psi^(2 brv(j) + 1); sigma_k's slot j reads slot brv((e_j k mod 2N - 1) / 2)
template <int LOGN>
WD uint32_t auto_src(uint32_t j, uint32_t k) {
    constexpr uint32_t N = 1u << LOGN;
    const uint32_t e = 2 * (__brev(j) >> (32 - LOGN)) + 1;
    return __brev(((e * k) & (2 * N - 1)) >> 1) >> (32 - LOGN);
}
}  // namespace

template <int LOGN, bool DM, class A>
__global__ void __launch_bounds__((1 << LOGN) / 4, A::kOpsWaves)
    k_blind_rotate_wide_ops(WideArgs g, WideTables tb, const typename A::T* __restrict__ bsk,
                            const typename A::T* __restrict__ autok, const uint16_t* __restrict__ ops,
                            const uint32_t* __restrict__ nops, uint32_t maxops, const uint32_t* __restrict__ tvb,
                            uint64_t* __restrict__ ext_a, uint64_t* __restrict__ ext_b) {
    using T = typename A::T;
    using Sum = typename A::S;
    constexpr int N = 1 << LOGN, TH = N / 4, S = 4;
    __shared__ T buf[2 * N];
    const A a(tb);  // tables through the caches: staged in LDS (48 KB per gate) this kernel ran 8% slower
    const uint32_t gate = blockIdx.x, t = threadIdx.x;
    const T Q = a.Q, QHalf = Q >> 1;
    using D = typename A::D;
    using UD = typename A::UD;
    const uint32_t dA = g.digitsG - 1, dG2 = 2 * dA, gb = g.gbits, sh = 8 * sizeof(D) - gb;

    T acc0[S], acc1[S];
    if (g.acc_io && !g.acc_tv) {  // the seam's accumulator; LMKCDEY's acc1 <- sigma_(2N-5)(acc1) (:99)
        const uint64_t* src = g.acc_io + (size_t)gate * 2 * N;
#pragma unroll
        for (int r = 0; r < S; ++r) {
            acc0[r] = (T)src[t + TH * r];
            acc1[r] = (T)src[N + (DM ? t + TH * r : auto_src<LOGN>(t + TH * r, 2 * N - 5))];
        }
    } else {
        const uint32_t b = tvb[gate], cm = g.ctmod - 1;
        // EvalFuncMultiOutput: table gate % tv_mod (GateArgs::tv_mod)
        const uint32_t tvo = g.tv_mod > 1 ? (gate % g.tv_mod) * g.ctmod : 0u;
#pragma unroll
        for (int r = 0; r < S; ++r) {
            const uint32_t x = t + TH * r;
            uint64_t v = 0;
            if (x % g.factor == 0) {
                const uint32_t bx = (b - x / g.factor) & cm;
                v = g.tv ? g.tv[tvo + bx] : (bx >= g.lb && bx < g.ub) ? g.lv : g.uv;
            }
            buf[x] = (T)v;
        }
        wg_sync();
        fwd<LOGN, 1>(buf, a);
#pragma unroll
        for (int r = 0; r < S; ++r) {
            acc0[r] = 0;
            acc1[r] = buf[DM ? t + TH * r : auto_src<LOGN>(t + TH * r, 2 * N - 5)];
        }
    }
    // the decomposition of rgsw-acc.cpp:54-91 from the canonical COEF value at buf[p N + j]:
    // centred, the lowest digit dropped, one level per call of digit()
    auto start = [&](int p, uint32_t j) -> D {
        const T v = a.mul_shoup(buf[p * N + j], a.ninv, a.ninvS);
        const D x = v < QHalf ? (D)v : (D)v - (D)Q;
        const D r0 = (D)((UD)x << sh) >> sh;
        return (x - r0) >> gb;
    };
    auto digit = [&](D& d) -> T {
        D r0 = (D)((UD)d << sh) >> sh;
        d = (d - r0) >> gb;
        if (r0 < 0) r0 += (D)Q;
        return (T)r0;
    };
    const uint16_t* gops = ops + (size_t)gate * maxops;
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(nops[gate]);
#pragma unroll 1
    for (uint32_t it = 0; it < cnt; ++it) {
        const uint32_t op = __builtin_amdgcn_readfirstlane((uint32_t)gops[it]);
        Sum U[2][S];
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int r = 0; r < S; ++r) U[c][r] = A::zero();
        wg_sync();
        if (DM || !(op & 0x8000u)) {
#pragma unroll
            for (int r = 0; r < S; ++r) {
                buf[t + TH * r]     = acc0[r];
                buf[N + t + TH * r] = acc1[r];
            }
            wg_sync();
            inv<LOGN, 2>(buf, a);
            D d[2][S];
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int r = 0; r < S; ++r) d[p][r] = start(p, t + TH * r);
            const T* key = bsk + (size_t)op * dG2 * 2 * N;
#pragma unroll 1
            for (uint32_t L = 0; L < dA; ++L) {
                wg_sync();
#pragma unroll
                for (int p = 0; p < 2; ++p)
#pragma unroll
                    for (int r = 0; r < S; ++r) buf[p * N + t + TH * r] = digit(d[p][r]);
                wg_sync();
                fwd<LOGN, 2>(buf, a);
#pragma unroll
                for (int r = 0; r < S; ++r) {
                    const uint32_t j = t + TH * r;
                    const T x0 = buf[j], x1 = buf[N + j];
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        A::mac(U[c][r], x0, key[((size_t)(2 * L) * 2 + c) * N + j]);
                        A::mac(U[c][r], x1, key[((size_t)(2 * L + 1) * 2 + c) * N + j]);
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < S; ++r) {
                acc0[r] = a.redc(U[0][r]);
                acc1[r] = a.redc(U[1][r]);
            }
        } else {
            const uint32_t ta = op & 0x7fffu;
            uint32_t k = 2 * N - 5;
            if (ta) {
                k = 1;
                for (uint32_t z = 0; z < ta; ++z) k = (k * 5) & (2 * N - 1);
            }
#pragma unroll
            for (int r = 0; r < S; ++r) {
                buf[t + TH * r]     = acc0[r];
                buf[N + t + TH * r] = acc1[r];
            }
            wg_sync();
            T a0[S];
#pragma unroll
            for (int r = 0; r < S; ++r) {
                const uint32_t src = auto_src<LOGN>(t + TH * r, k);
                a0[r]   = buf[src];
                acc1[r] = buf[N + src];
            }
            wg_sync();
#pragma unroll
            for (int r = 0; r < S; ++r) buf[t + TH * r] = a0[r];
            wg_sync();
            inv<LOGN, 1>(buf, a);
            D d[S];
#pragma unroll
            for (int r = 0; r < S; ++r) d[r] = start(0, t + TH * r);
            const T* key = autok + (size_t)ta * dA * 2 * N;
#pragma unroll 1
            for (uint32_t L = 0; L < dA; ++L) {
                wg_sync();
#pragma unroll
                for (int r = 0; r < S; ++r) buf[t + TH * r] = digit(d[r]);
                wg_sync();
                fwd<LOGN, 1>(buf, a);
#pragma unroll
                for (int r = 0; r < S; ++r) {
                    const uint32_t j = t + TH * r;
                    const T x = buf[j];
#pragma unroll
                    for (int c = 0; c < 2; ++c) A::mac(U[c][r], x, key[((size_t)L * 2 + c) * N + j]);
                }
            }
#pragma unroll
            for (int r = 0; r < S; ++r) {
                acc0[r] = a.redc(U[0][r]);
                acc1[r] = a.add(acc1[r], a.redc(U[1][r]));
            }
        }
    }

    if (g.acc_io) {
        uint64_t* dst = g.acc_io + (size_t)gate * 2 * N;
#pragma unroll
        for (int r = 0; r < S; ++r) {
            dst[t + TH * r]     = acc0[r];
            dst[N + t + TH * r] = acc1[r];
        }
        return;
    }
    // extraction as k_blind_rotate_wide
    wg_sync();
#pragma unroll
    for (int r = 0; r < S; ++r) {
        buf[t + TH * r]     = acc0[r];
        buf[N + t + TH * r] = acc1[r];
    }
    wg_sync();
    inv<LOGN, 2>(buf, a);
    uint64_t* oa = ext_a + (size_t)gate * N;
#pragma unroll
    for (int r = 0; r < S; ++r) {
        const uint32_t x = t + TH * r;
        const T c = a.mul_shoup(buf[x == 0 ? 0 : N - x], a.ninv, a.ninvS);
        const uint64_t v = (x == 0 || c == 0) ? c : Q - c;
        oa[x] = g.msb_out ? round_qQ(v, g.qKS, Q) : v;
    }
    if (t == 0) {
        const uint64_t bb = a.add((T)(g.b_const % Q), a.mul_shoup(buf[N], a.ninv, a.ninvS));
        ext_b[gate] = g.msb_out ? round_qQ(bb, g.qKS, Q) : bb;
    }
}

static bool wide_args_ok(const WideArgs& g) {
    return (g.N == 512 || g.N == 1024 || g.N == 2048) && g.digitsG >= 2 && g.gbits >= 1 && g.gbits <= 62 &&
           g.factor != 0 && g.ctmod <= 2 * g.N && !(g.ctmod & (g.ctmod - 1));
}

template <class A>
static void launch_ops(const WideArgs& g, const WideTables& t, const void* bsk, const void* autok, const uint16_t* ops,
                       const uint32_t* nops, uint32_t maxops, const uint32_t* tvb, uint64_t* ext_a, uint64_t* ext_b,
                       bool dm, hipStream_t s) {
    using T = typename A::T;
    const T* kb = static_cast<const T*>(bsk);
    const T* ka = static_cast<const T*>(autok);
#define FHE_WIDE_OPS(LG, DM_)                                                                                     \
    hipLaunchKernelGGL((k_blind_rotate_wide_ops<LG, DM_, A>), dim3(g.count), dim3((1 << LG) / 4), 0, s, g, t, kb, \
                       ka, ops, nops, maxops, tvb, ext_a, ext_b)
    if (g.N == 2048) {
        if (dm) FHE_WIDE_OPS(11, true);
        else FHE_WIDE_OPS(11, false);
    } else if (g.N == 1024) {
        if (dm) FHE_WIDE_OPS(10, true);
        else FHE_WIDE_OPS(10, false);
    } else {  // TOY
        if (dm) FHE_WIDE_OPS(9, true);
        else FHE_WIDE_OPS(9, false);
    }
#undef FHE_WIDE_OPS
}

hipError_t launch_blind_rotate_wide_ops(const WideArgs& g, const WideTables& t, const void* bsk, const void* autok,
                                        const uint16_t* ops, const uint32_t* nops, uint32_t maxops, const uint32_t* tvb,
                                        uint64_t* ext_a, uint64_t* ext_b, bool dm, hipStream_t s) {
    if (g.count == 0) return hipSuccess;
    if (!wide_args_ok(g)) return hipErrorInvalidValue;
    if (t.narrow) launch_ops<A32>(g, t, bsk, autok, ops, nops, maxops, tvb, ext_a, ext_b, dm, s);
    else launch_ops<A64>(g, t, bsk, autok, ops, nops, maxops, tvb, ext_a, ext_b, dm, s);
    return hipGetLastError();
}

// ExternalProduct seam: raw RGSW rows (canonical mod Q) -> Montgomery form x R mod Q, the form
// k_blind_rotate_wide_ops reads its keys in: redc(x R2) with R2 = R^2 mod Q (x R2 < Q^2 < Q R)
__global__ void k_pack_rgsw_wide(const uint64_t* __restrict__ raw, size_t words, uint64_t Q, uint64_t qinv, uint64_t R2,
                                 uint64_t* __restrict__ out) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < words; i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t x = raw[i];
        const uint64_t lo = x * R2, u = lo * qinv;
        const uint64_t r = __umul64hi(x, R2) + __umul64hi(u, Q) + (lo != 0 ? 1 : 0);
        out[i] = r >= Q ? r - Q : r;
    }
}
__global__ void k_pack_rgsw_narrow(const uint64_t* __restrict__ raw, size_t words, uint32_t Q, uint32_t qinv,
                                   uint32_t R2, uint32_t* __restrict__ out) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < words; i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t t = (uint64_t)(uint32_t)raw[i] * R2;
        const uint32_t u = (uint32_t)t * qinv;
        const uint32_t r = (uint32_t)((t + (uint64_t)u * Q) >> 32);
        out[i] = r >= Q ? r - Q : r;
    }
}

hipError_t launch_pack_rgsw_wide(const uint64_t* raw, size_t words, const WideTables& t, void* out, hipStream_t s) {
    if (words == 0) return hipSuccess;
    const uint32_t blocks = (uint32_t)std::min<size_t>((words + 255) / 256, 8192);
    if (t.narrow)
        hipLaunchKernelGGL(k_pack_rgsw_narrow, dim3(blocks), dim3(256), 0, s, raw, words, t.Q32, t.qinv32, t.r2_32,
                           static_cast<uint32_t*>(out));
    else
        hipLaunchKernelGGL(k_pack_rgsw_wide, dim3(blocks), dim3(256), 0, s, raw, words, t.Q, t.qinv, t.r2,
                           static_cast<uint64_t*>(out));
    return hipGetLastError();
}

template <class A>
static void launch_gate(const WideArgs& g, const WideTables& t, const void* bsk, const uint16_t* idx,
                        const uint32_t* tvb, uint64_t* ext_a, uint64_t* ext_b, hipStream_t s) {
    const auto* kb = static_cast<const typename A::T*>(bsk);
    if (g.N == 2048)
        hipLaunchKernelGGL((k_blind_rotate_wide<11, A>), dim3(g.count), dim3(512), 0, s, g, t, kb, idx, tvb, ext_a, ext_b);
    else if (g.N == 1024)
        hipLaunchKernelGGL((k_blind_rotate_wide<10, A>), dim3(g.count), dim3(256), 0, s, g, t, kb, idx, tvb, ext_a, ext_b);
    else  // TOY
        hipLaunchKernelGGL((k_blind_rotate_wide<9, A>), dim3(g.count), dim3(128), 0, s, g, t, kb, idx, tvb, ext_a, ext_b);
}

hipError_t launch_blind_rotate_wide(const WideArgs& g, const WideTables& t, const void* bsk, const uint16_t* idx,
                                    const uint32_t* tvb, uint64_t* ext_a, uint64_t* ext_b, hipStream_t s) {
    if (g.count == 0) return hipSuccess;
    if (!wide_args_ok(g)) return hipErrorInvalidValue;
    if (t.narrow) launch_gate<A32>(g, t, bsk, idx, tvb, ext_a, ext_b, s);
    else launch_gate<A64>(g, t, bsk, idx, tvb, ext_a, ext_b, s);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// KeySwitch (lwe-pke.cpp:348-372) + ModSwitch(qKS -> q_out): one workgroup per ciphertext, thread t
// owns columns t + blockDim c of the n-wide A rows (u64, read coalesced) and thread 0 also the B
// column; the N digitsKS row values (each < qKS) sum below 2^64 unreduced, then mod qKS: a mask for
// qKS = 2^k, a remainder for the prime qKS of TOY / SIGNED_MOD_TEST (modKS = PRIME).  Digits of a_i
// in base baseKS: shifts for a power of two, remainders otherwise (STD256Q_3: 21, TOY: 25).
// ---------------------------------------------------------------------------
constexpr int kKsWideCols = 8;

__global__ void __launch_bounds__(256)
    k_keyswitch_wide(uint32_t n, uint32_t N, uint32_t baseKS, uint32_t logBase, uint32_t digitsKS, uint64_t qKS,
                     const uint64_t* __restrict__ A, const uint64_t* __restrict__ B, const uint64_t* __restrict__ ms_a,
                     const uint64_t* __restrict__ ms_b, uint64_t q_out, uint64_t* __restrict__ a_out,
                     uint64_t* __restrict__ b_out) {
    __shared__ uint64_t s_a[2048];
    const uint32_t gate = blockIdx.x, t = threadIdx.x, nt = blockDim.x;
    for (uint32_t i = t; i < N; i += nt) s_a[i] = ms_a[(size_t)gate * N + i];
    __syncthreads();
    const uint64_t mask = (1ull << logBase) - 1;
    uint64_t acc[kKsWideCols] = {};
    uint64_t accb = 0;
#pragma unroll 1
    for (uint32_t i = 0; i < N; ++i) {
        uint64_t ai = s_a[i];
#pragma unroll 1
        for (uint32_t j = 0; j < digitsKS; ++j) {
            uint64_t a0;
            if (logBase) {
                a0 = (ai >> (logBase * j)) & mask;
            } else {
                a0 = ai % baseKS;
                ai /= baseKS;
            }
            const uint64_t row = ((uint64_t)i * baseKS + a0) * digitsKS + j;
            const uint64_t* Ar = A + row * n;
#pragma unroll
            for (int c = 0; c < kKsWideCols; ++c) {
                const uint32_t k = t + nt * c;
                if (k < n) acc[c] += Ar[k];
            }
            if (t == 0) accb += B[row];
        }
    }
    const bool pow2 = (qKS & (qKS - 1)) == 0;
    const uint64_t qm = qKS - 1;
    auto sub_from = [&](uint64_t b, uint64_t sum) -> uint64_t {  // (b - sum) mod qKS, b < qKS
        if (pow2) return (b - sum) & qm;
        const uint64_t r = sum % qKS;
        return b >= r ? b - r : b + qKS - r;
    };
    uint64_t* oa = a_out + (size_t)gate * n;
#pragma unroll
    for (int c = 0; c < kKsWideCols; ++c) {
        const uint32_t k = t + nt * c;
        if (k < n) {
            const uint64_t v = sub_from(0, acc[c]);
            oa[k] = q_out ? round_qQ(v, q_out, qKS) : v;
        }
    }
    if (t == 0) {
        const uint64_t v = sub_from(ms_b[gate], accb);
        b_out[gate] = q_out ? round_qQ(v, q_out, qKS) : v;
    }
}

hipError_t launch_keyswitch_wide(size_t count, uint32_t n, uint32_t N, uint32_t baseKS, uint32_t digitsKS, uint64_t qKS,
                                 const uint64_t* A, const uint64_t* B, const uint64_t* ms_a, const uint64_t* ms_b,
                                 uint64_t q_out, uint64_t* a_out, uint64_t* b_out, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (N > 2048 || qKS < 2 || baseKS < 2 || count > 0x7fffffffull) return hipErrorInvalidValue;
    uint32_t logBase = 0;  // 0: baseKS is not a power of two
    if (!(baseKS & (baseKS - 1)))
        while ((1u << logBase) < baseKS) ++logBase;
    uint32_t nt = (n + 63) / 64 * 64;
    if (nt > 256) nt = 256;
    if ((size_t)nt * kKsWideCols < n) return hipErrorInvalidValue;
    // the digits must cover qKS and the unreduced column sums must fit 64 bits
    double cover = 1;
    for (uint32_t j = 0; j < digitsKS && cover < 1e30; ++j) cover *= baseKS;
    if (cover < (double)qKS) return hipErrorInvalidValue;
    if ((double)N * digitsKS * (double)qKS >= 18446744073709551616.0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_keyswitch_wide, dim3((uint32_t)count), dim3(nt), 0, s, n, N, baseKS, logBase, digitsKS, qKS,
                       A, B, ms_a, ms_b, q_out, a_out, b_out);
    return hipGetLastError();
}

}  // namespace fhe_amd
