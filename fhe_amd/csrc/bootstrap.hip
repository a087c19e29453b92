// bootstrap.hip -- fused TFHE gate bootstrap (GINX / CGGI) for gfx950.
//
// One wavefront per gate, for all n iterations of the accumulator loop
// (RingGSWAccumulatorCGGI::EvalAcc, src/binfhe/lib/rgsw-acc-cggi.cpp:59-68):
// the RLWE accumulator never leaves the CU.  Half-wave h (lanes 32h..32h+31)
// owns polynomial component h (acc0 / acc1) as 32 registers x 32 lanes:
//   layout A' (COEFFICIENT): lane l, register r  <->  coefficient x = (r << 5) | l
//   layout B' (EVALUATION):  lane l, register r  <->  NTT slot      x = (l << 5) | r
// (slot x is the reference's bit-reversed EVALUATION storage index).  A forward
// NTT runs 5 radix-2 stages in A' (twiddles uniform over the wave: scalar
// loads), one 32x32 LDS transpose, 5 stages in B' (per-lane twiddles from an
// LDS table laid out lane-major: conflict-free); the inverse runs backwards.
// Per iteration (AddToAccCGGI, rgsw-acc-cggi.cpp:102-151):
//   iNTT(acc0 | acc1) -> signed approximate decomposition (rgsw-acc.cpp:54-91)
//   -> NTT(D0 | D1), NTT(D2 | D3) -> per slot, all four digits gathered with
//   v_permlane32_swap -> S1 = sum_d D_d K+[d][h], S2 = sum_d D_d K-[d][h] as
//   64-bit v_mad_u64_u32 sums (keys in Montgomery form) -> one Montgomery
//   reduction each -> acc_h += S1 (X^a - 1) + S2 (X^-a - 1), the monomials
//   EVAL(X^m - 1) = omega_slot^m - 1 read from a 2N-entry LDS table instead of
//   the reference's 16 MiB table of 2N NTT'd polynomials
//   (rgsw-cryptoparameters.cpp:96-113).
// All arithmetic is exact mod Q: lazy residues (< 4Q) inside the NTTs, canonical
// [0, Q) at every point where the reference's values are observable (COEF acc
// before decomposition, EVAL acc between iterations, outputs).
#include "arith.h"
#include "boot.h"

#ifndef FHE_KEY_PF
#define FHE_KEY_PF 2     // key chunks (2 slots each) requested ahead of use in the CMUX loop
#endif
#ifndef FHE_WAVES_PER_EU
#define FHE_WAVES_PER_EU 2
#endif
#ifndef FHE_K1_PRIO
#define FHE_K1_PRIO 0     // A/B: K1's waves of odd workgroup slots on a CU at priority 1
#endif
#ifndef FHE_K1_STAGGER
#define FHE_K1_STAGGER 0  // A/B: odd workgroup slots start FHE_K1_STAGGER x 8128 cycles late
#endif

// Forward-transform bounds from the product itself (round 5): a signed Montgomery product is below
// |y| |w| 2^-32 + Q/2 < (Q / 2^32) |y| + Q/2, so a Cooley-Tukey stage takes a bound B to (1 + Q / 2^32) B + Q/2
// rather than B + Q.  From signed digits (B ~ 0): ten stages stay below 6.67 Q for Q < 2^28 (Q / 2^32 < 1/16),
// inside the 8 Q of 32-bit signed words, so FM 2 needs no reduction (the LMKCDEY accumulator bound grows from
// 2.0 Q to 2.2 Q: four digits < 6.67 Q times keys < Q, 26.7 Q^2 2^-32 + Q/2); and for Q < 2^29 (1/8) five
// stages stay below 3.21 Q < 4 Q, so K1w's QM 2 reduces after five stages and after nine (below 0.9 Q each
// time, 3.84 Q before the second) instead of after three, six and nine; for Q < 2^28 eleven stages stay below
// 7.59 Q < 8 Q, so K1w's QM 1 (STD256Q_LMKCDEY) drops its one reduction.  FHE_FWD_TIGHT=0: the round-4 points.
#ifndef FHE_FWD_TIGHT
#define FHE_FWD_TIGHT 1
#endif

namespace fhe_amd {

namespace {

constexpr int kTile = 32 * 33;  // one half-wave transpose tile (u32 words)
constexpr int kAccBoundLZ = 28; // GINX, Q < 2^27: |acc| < 2.8 Q between iterations (units of Q/10)

struct Mod {
    uint32_t Q, Q2, qinv;  // qinv = -Q^-1 mod 2^32
    uint32_t qinvp;        // Q^-1 mod 2^32 (signed Montgomery)
    int32_t nQ;            // -Q (signed Montgomery; see fresh_nq)
    uint32_t oneR;         // 2^32 mod Q: smont_mul(x, oneR) = x mod Q in (-Q, Q)
};
FHE_DEV Mod make_mod(const BootTables& T) { return Mod{T.Q, T.Q2, T.qinv, 0u - T.qinv, -(int32_t)T.Q, T.oneR}; }

// a * bR * 2^-32 mod Q, lazily: result < Q (1 + a / 2^32 * ...) < 2Q for a < 4Q, Q < 2^28
FHE_DEV uint32_t mont_mul(uint32_t a, uint32_t bR, const Mod& m) {
    uint64_t t  = (uint64_t)a * bR;
    uint32_t mm = (uint32_t)t * m.qinv;
    return (uint32_t)((t + (uint64_t)mm * m.Q) >> 32);
}
FHE_DEV uint32_t mont_red(uint64_t t, const Mod& m) {  // t < 16 Q^2 -> result < 2Q
    uint32_t mm = (uint32_t)t * m.qinv;
    return (uint32_t)((t + (uint64_t)mm * m.Q) >> 32);
}
// sum of four digit x key products as a non-negative 64-bit value for mont_red: unsigned digits
// (< 16Q) directly; signed digits (LZ, |d| < 10Q + 2^9, Q < 2^27) plus moff = 64 Q^2 (a multiple
// of Q above the most negative sum 4 (10Q + 2^9) Q)
template <bool LZ>
FHE_DEV uint64_t mac4(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3, uint32_t k0, uint32_t k1, uint32_t k2,
                      uint32_t k3, uint64_t moff) {
    if (LZ) {
        const int64_t s = (int64_t)(int32_t)d0 * (int32_t)k0 + (int64_t)(int32_t)d1 * (int32_t)k1 +
                          (int64_t)(int32_t)d2 * (int32_t)k2 + (int64_t)(int32_t)d3 * (int32_t)k3;
        return (uint64_t)(s + (int64_t)moff);
    }
    return (uint64_t)d0 * k0 + (uint64_t)d1 * k1 + (uint64_t)d2 * k2 + (uint64_t)d3 * k3;
}
// Cooley-Tukey (forward), lazy: t = y w < 2Q for any y < 2^32, so x, y < B in gives
// x + t, x + 2Q - t < B + 2Q out (no reduction; fwd_pass bounds the growth)
FHE_DEV void ct_bf(uint32_t& x, uint32_t& y, uint32_t wR, const Mod& m) {
    uint32_t t = mont_mul(y, wR, m);
    uint32_t s = x + m.Q2;
    y          = s - t;
    x          = x + t;
}
#ifndef FHE_DM_WAVES
#define FHE_DM_WAVES 3   // waves per SIMD of the AP/DM op-list kernel
#endif
#ifndef FHE_LMK_WAVES
#define FHE_LMK_WAVES 2  // waves per SIMD of the LMKCDEY op-list kernel
#endif
#ifndef FHE_LMK_OPAQUE
#define FHE_LMK_OPAQUE 0 // op-list kernel: per-lane addresses recomputed per op (register pressure)
#endif
#ifndef FHE_LMK_PRE
#define FHE_LMK_PRE 1    // op-list kernel: a pass's 31 per-lane twiddles requested together at its start
#endif
#ifndef FHE_LMK_AKPF
#define FHE_LMK_AKPF 1   // the same for the automorphism keys (4 slots x 2 rows)
#endif
#ifndef FHE_LMK_SWAP
#define FHE_LMK_SWAP 1   // LMKCDEY automorphism: the digits into the half-wave layout by v_permlane32_swap
#endif
#ifndef FHE_LMK_ABL
#define FHE_LMK_ABL 0    // timing-only ablations of the LMKCDEY op-list kernel (wrong results), bits: 1 every EXT op
                         // reads the keys of index 0, 2 every AUTO op those of key 0 (cache-resident: the data-
                         // dependent key traffic removed), 4 the automorphism gathers at linear positions, 8 no digit
                         // exchange between the half-waves in EXT
#endif
#ifndef FHE_LMK_KPF
#define FHE_LMK_KPF 1    // op-list kernel: key chunks (4 slots x 4 rows) requested ahead of their MAC
#endif
// v_mad_i64_i32 (a * b + c, 32 x 32 -> 64 signed) in plain C, with -Q re-materialised inside each
// loop body (fresh_nq) so that instruction selection sees a sign-extended 32-bit operand (hoisted,
// the compiler widens -Q into a 64-bit constant and the product becomes 5 instructions)
FHE_DEV int64_t mad_i64_i32(int32_t a, int32_t b, int64_t c) {
    return (int64_t)a * b + c;
}
// signed Montgomery (the Q < 2^27 path): a read as int32, bR < Q -> (a b 2^-32 mod Q) in (-Q, Q)
// for any |a| < 2^31: |a bR - mm Q| < 2^31 Q + 2^31 Q
FHE_DEV uint32_t smont_mul(uint32_t a, uint32_t bR, const Mod& m) {
    const int64_t t  = mad_i64_i32((int32_t)a, (int32_t)bR, 0);
    const int32_t mm = (int32_t)((uint32_t)t * m.qinvp);
    return (uint32_t)(mad_i64_i32(mm, m.nQ, t) >> 32);
}
// signed Montgomery reduction of a 64-bit t, |t| < 2^63 - 2^31 Q: t 2^-32 mod Q in (|t| 2^-32 +- Q/2)
FHE_DEV uint32_t smont_red(int64_t t, const Mod& m) {
    const int32_t mm = (int32_t)((uint32_t)t * m.qinvp);
    return (uint32_t)(mad_i64_i32(mm, m.nQ, t) >> 32);
}
// -Q as a value defined inside the current loop body (an empty asm the optimizer cannot hoist)
FHE_DEV Mod fresh_nq(Mod m) {
    asm volatile("" : "+s"(m.nQ));
    return m;
}
// signed Cooley-Tukey: |x|, |y| < B in, < B + Q out, two adds and no offset
FHE_DEV void ct_bf_s(uint32_t& x, uint32_t& y, uint32_t wR, const Mod& m) {
    const uint32_t t = smont_mul(y, wR, m);
    y                = x - t;
    x                = x + t;
}
// Gentleman-Sande (inverse): x, y < 2Q in, < 2Q out
FHE_DEV void gs_bf(uint32_t& x, uint32_t& y, uint32_t wR, const Mod& m) {
    uint32_t s = csub(x + y, m.Q2);
    uint32_t d = x + m.Q2 - y;
    x          = s;
    y          = mont_mul(d, wR, m);
}

// intra-wave LDS hand-off: orders this wave's LDS accesses around a layout change
FHE_DEV void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

FHE_DEV void transpose32(uint32_t (&v)[32], uint32_t* tile, int l) {
#pragma unroll
    for (int r = 0; r < 32; ++r) tile[l * 33 + r] = v[r];
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < 32; ++r) v[r] = tile[r * 33 + l];
    wave_lds_sync();
}

// offset of stage b's lane-major twiddle block: 32 * (2^(4-b) - 1)
constexpr int twb_off(int b) { return 32 * ((1 << (4 - b)) - 1); }
// PRE: the 31 per-lane twiddles of a pass's five B' stages requested together at its start
// (entry j of stage b is tw[twb_off(b) / 32 + j]) instead of one LDS round trip per stage pair
#define TWB(b, j) (PRE ? tw[twb_off(b) / 32 + (j)] : s_twB[twb_off(b) + (j) * 32 + l])
#define TW_PRELOAD                                                    \
    uint32_t tw[31];                                                  \
    if (PRE) {                                                        \
        _Pragma("unroll") for (int j = 0; j < 31; ++j) tw[j] = s_twB[j * 32 + l]; \
    }

// forward NTT: A' (COEF, inputs < Q) -> B' (EVAL), outputs < 14Q (< 2^32 for Q < 2^28):
// 5 stages (< 11Q), reduce to < 4Q at the transpose, 5 stages (< 14Q)
FHE_DEV void fwd_pass(uint32_t (&v)[32], uint32_t* tile, int l, const uint32_t* __restrict__ twA,
                      const uint32_t* s_twB, const Mod& m) {
#pragma unroll
    for (int b = 9; b >= 5; --b) {
        const int rb = b - 5;
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            if (r & (1 << rb)) continue;
            const uint32_t w = twA[(1 << (9 - b)) + (r >> (rb + 1))];
            ct_bf(v[r], v[r | (1 << rb)], w, m);
        }
    }
#pragma unroll
    for (int r = 0; r < 32; ++r) v[r] = csub(csub(v[r], 4 * m.Q2), m.Q2);  // < 11Q -> < 4Q
    transpose32(v, tile, l);
#pragma unroll
    for (int b = 4; b >= 0; --b) {
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            if (r & (1 << b)) continue;
            const uint32_t w = s_twB[twb_off(b) + (r >> (b + 1)) * 32 + l];
            ct_bf(v[r], v[r | (1 << b)], w, m);
        }
    }
}

// two forward NTTs at once (the digit polynomials D_h and D_{2+h}): each twiddle
// load feeds two butterflies and every stage has 32 independent butterflies.
// LZ (Q < 2^27): signed digits |d| <= 2^(g-1) and signed butterflies -- |v| grows by < Q per
// stage to < 10Q + 2^(g-1) < 2^31, no reduction anywhere.  Otherwise unsigned digits < 2Q grow by
// < 2Q per stage; < 12Q is reduced to < 6Q at the transpose (< 16Q out, Q < 2^28).
// FM (forward mode): 0 unsigned lazy (above), 1 signed without reduction (Q < 2^27), 2 signed for
// Q < 2^28: after 5 stages |v| < 5Q + 2^(g-1); the x inputs of the first B' stage (registers 0..15)
// are reduced to (-Q, Q), so the B' outputs stay < 6Q (a Cooley-Tukey output is bounded by |x| + Q)
template <int FM, bool PRE = false>
FHE_DEV void fwd_pass2(uint32_t (&v)[32], uint32_t (&u)[32], uint32_t* tile, int l,
                       const uint32_t* __restrict__ twA, const uint32_t* s_twB, const Mod& m) {
    constexpr bool LZ = FM != 0;
#pragma unroll
    for (int b = 9; b >= 5; --b) {
        const int rb = b - 5;
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            if (r & (1 << rb)) continue;
            const uint32_t w = twA[(1 << (9 - b)) + (r >> (rb + 1))];
            if (LZ) {
                ct_bf_s(v[r], v[r | (1 << rb)], w, m);
                ct_bf_s(u[r], u[r | (1 << rb)], w, m);
            } else {
                ct_bf(v[r], v[r | (1 << rb)], w, m);
                ct_bf(u[r], u[r | (1 << rb)], w, m);
            }
        }
    }
    if (!LZ) {
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            v[r] = csub(csub(v[r], 4 * m.Q2), m.Q2);
            u[r] = csub(csub(u[r], 4 * m.Q2), m.Q2);
        }
    }
    transpose32(v, tile, l);
    transpose32(u, tile, l);
    if (FM == 2 && !FHE_FWD_TIGHT) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            v[r] = smont_mul(v[r], m.oneR, m);
            u[r] = smont_mul(u[r], m.oneR, m);
        }
    }
    TW_PRELOAD
#pragma unroll
    for (int b = 4; b >= 0; --b) {
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            if (r & (1 << b)) continue;
            const uint32_t w = TWB(b, r >> (b + 1));
            if (LZ) {
                ct_bf_s(v[r], v[r | (1 << b)], w, m);
                ct_bf_s(u[r], u[r | (1 << b)], w, m);
            } else {
                ct_bf(v[r], v[r | (1 << b)], w, m);
                ct_bf(u[r], u[r | (1 << b)], w, m);
            }
        }
    }
}

// one signed forward pass (FM 1 or 2 as in fwd_pass2): the LMKCDEY automorphism step
template <int FM>
FHE_DEV void fwd_pass_s(uint32_t (&v)[32], uint32_t* tile, int l, const uint32_t* __restrict__ twA,
                        const uint32_t* s_twB, const Mod& m) {
#pragma unroll
    for (int b = 9; b >= 5; --b) {
        const int rb = b - 5;
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            if (r & (1 << rb)) continue;
            ct_bf_s(v[r], v[r | (1 << rb)], twA[(1 << (9 - b)) + (r >> (rb + 1))], m);
        }
    }
    transpose32(v, tile, l);
    if (FM == 2 && !FHE_FWD_TIGHT) {
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = smont_mul(v[r], m.oneR, m);
    }
#pragma unroll
    for (int b = 4; b >= 0; --b) {
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            if (r & (1 << b)) continue;
            ct_bf_s(v[r], v[r | (1 << b)], s_twB[twb_off(b) + (r >> (b + 1)) * 32 + l], m);
        }
    }
}

// inverse NTT of N^-1-scaled data (BootTables::w1R): B' (EVAL, inputs < 2Q) -> A' (COEF),
// outputs canonical [0, Q)
FHE_DEV void inv_pass(uint32_t (&v)[32], uint32_t* tile, int l, const uint32_t* __restrict__ twA,
                      const uint32_t* s_twB, uint32_t w1R, const Mod& m) {
#pragma unroll
    for (int b = 0; b <= 4; ++b) {
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            if (r & (1 << b)) continue;
            const uint32_t w = s_twB[twb_off(b) + (r >> (b + 1)) * 32 + l];
            gs_bf(v[r], v[r | (1 << b)], w, m);
        }
    }
    transpose32(v, tile, l);
#pragma unroll
    for (int b = 5; b <= 8; ++b) {
        const int rb = b - 5;
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            if (r & (1 << rb)) continue;
            const uint32_t w = twA[(1 << (9 - b)) + (r >> (rb + 1))];
            gs_bf(v[r], v[r | (1 << rb)], w, m);
        }
    }
    // bit 9 (transformnat-impl.h:599-623); its N^-1 factor is already in the data
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        uint32_t x = v[r], y = v[r | 16];
        v[r]      = csub(csub(x + y, m.Q2), m.Q);
        v[r | 16] = csub(mont_mul(x + m.Q2 - y, w1R, m), m.Q);
    }
}

// ---- signed inverse NTT (Q < 2^27) ------------------------------------------------------------
// Gentleman-Sande on signed residues: x' = x + y, y' = smont(x - y, w) in (-Q, Q): two adds and
// no reduction per butterfly.  Sums grow; |x +- y| must stay < 2^31 = 16Q, so elements whose
// bound would overflow are brought back to (-Q, Q) by one signed Montgomery product with 2^32 mod Q.
// Bounds are tracked per register at compile time (units of Q/10): in layout B' the register index
// is the slot's low 5 bits, so the bound of every element a register holds is the same.  At the
// transpose every register mixes, so the largest bound is carried into the A' stages.
struct InvPlanS {
    bool red1[5][32];  // reduce register r before B' stage b
    bool redT[32];     // ... before the transpose
    bool red2[4][32];  // ... before the A' stage on register bit rb
    bool red3[32];     // ... before the last stage (bit 9)
    int fin[16];       // last-stage sum x + y: |.| < 2^fin Q -> add 2^fin Q, then fin + 1 conditional subtractions
};
// LIM: the bound on |x| + |y| (units of Q/10) that keeps sums below 2^31: 16 Q for Q < 2^27,
// 8 Q for Q < 2^28
constexpr int lim_s(bool lz) { return lz ? 160 : 80; }
constexpr void plan_half(int (&B)[32], bool (&red)[5][32], int stages, int kLimS) {
    for (int b = 0; b < stages; ++b)
        for (int r = 0; r < 32; ++r) {
            if (r & (1 << b)) continue;
            const int s = r | (1 << b);
            while (B[r] + B[s] > kLimS) {
                const int e = B[r] >= B[s] ? r : s;
                B[e]         = 10;
                red[b][e]    = true;
            }
            B[r] = B[r] + B[s];
            B[s] = 10;
        }
}
template <int BIN, int kLimS>
constexpr InvPlanS make_inv_plan() {
    InvPlanS p{};
    int B[32] = {};
    for (int r = 0; r < 32; ++r) B[r] = BIN;
    plan_half(B, p.red1, 5, kLimS);
    int U = 0;
    for (int r = 0; r < 32; ++r) {
        if (B[r] > 20) {
            p.redT[r] = true;
            B[r]      = 10;
        }
        U = B[r] > U ? B[r] : U;
    }
    for (int r = 0; r < 32; ++r) B[r] = U;
    bool red2[5][32] = {};
    plan_half(B, red2, 4, kLimS);
    for (int b = 0; b < 4; ++b)
        for (int r = 0; r < 32; ++r) p.red2[b][r] = red2[b][r];
    for (int r = 0; r < 16; ++r) {
        while (B[r] + B[r | 16] > kLimS) {
            const int e = B[r] >= B[r | 16] ? r : (r | 16);
            B[e]        = 10;
            p.red3[e]   = true;
        }
        int f = 0;
        while ((10 << f) < B[r] + B[r | 16]) ++f;
        p.fin[r] = f;
    }
    return p;
}

// B' (EVAL, |inputs| < BIN Q / 10, signed) -> A' (COEF), canonical [0, Q) like inv_pass.
// LZ: Q < 2^27 (sums up to 16 Q), else Q < 2^28 (8 Q; the final 2^(fin+1) Q <= 16 Q < 2^32)
template <int BIN, bool LZ = true, bool PRE = false>
FHE_DEV void inv_pass_s(uint32_t (&v)[32], uint32_t* tile, int l, const uint32_t* __restrict__ twA,
                        const uint32_t* s_twB, uint32_t w1R, uint32_t oneR, const Mod& m) {
    constexpr InvPlanS P = make_inv_plan<BIN, lim_s(LZ)>();
    TW_PRELOAD
#pragma unroll
    for (int b = 0; b <= 4; ++b) {
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            if (r & (1 << b)) continue;
            const int s = r | (1 << b);
            if (P.red1[b][r]) v[r] = smont_mul(v[r], oneR, m);
            if (P.red1[b][s]) v[s] = smont_mul(v[s], oneR, m);
            const uint32_t w = TWB(b, r >> (b + 1));
            const uint32_t x = v[r], y = v[s];
            v[r]             = x + y;
            v[s]             = smont_mul(x - y, w, m);
        }
    }
#pragma unroll
    for (int r = 0; r < 32; ++r)
        if (P.redT[r]) v[r] = smont_mul(v[r], oneR, m);
    transpose32(v, tile, l);
#pragma unroll
    for (int b = 5; b <= 8; ++b) {
        const int rb = b - 5;
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            if (r & (1 << rb)) continue;
            const int s = r | (1 << rb);
            if (P.red2[rb][r]) v[r] = smont_mul(v[r], oneR, m);
            if (P.red2[rb][s]) v[s] = smont_mul(v[s], oneR, m);
            const uint32_t w = twA[(1 << (9 - b)) + (r >> (rb + 1))];
            const uint32_t x = v[r], y = v[s];
            v[r]             = x + y;
            v[s]             = smont_mul(x - y, w, m);
        }
    }
    // bit 9 (transformnat-impl.h:599-623); its N^-1 factor is already in the data.  Signed results
    // to [0, Q): the sum by adding 2^f Q and f + 1 conditional subtractions, the product (in
    // (-Q, Q)) by min(d, d + Q) on the unsigned words.
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        if (P.red3[r]) v[r] = smont_mul(v[r], oneR, m);
        if (P.red3[r | 16]) v[r | 16] = smont_mul(v[r | 16], oneR, m);
        const uint32_t x = v[r], y = v[r | 16];
        uint32_t s       = x + y + (m.Q << P.fin[r]);
#pragma unroll
        for (int f = P.fin[r]; f >= 0; --f) s = csub(s, m.Q << f);
        const uint32_t d = smont_mul(x - y, w1R, m);
        v[r]             = s;
        v[r | 16]        = min(d, d + m.Q);
    }
}

// the same register of the other half-wave (lane ^ 32), through the LDS crossbar (no VALU)
FHE_DEV uint32_t other_half(uint32_t x, int xaddr) { return (uint32_t)__builtin_amdgcn_ds_bpermute(xaddr, (int)x); }

// key vector load
FHE_DEV uint4 kload(const uint4* p, size_t i) { return p[i]; }
FHE_DEV uint32_t brv5(uint32_t x) { return __builtin_bitreverse32(x) >> 27; }

// SignedDigitDecompose (rgsw-acc.cpp:54-91) for digitsG = 3: centre x in [0, Q) to
// d in [-Q/2, Q/2), drop the lowest balanced base-2^g digit, return the next two.  The balanced
// digits of d are the plain base-2^g digits of d + C, C = 2^(g-1) (1 + 2^g + 2^2g), minus 2^(g-1)
// (the sequential sign-extend-and-subtract of the reference computes the same unique balanced
// representation; its last digit sign-extends the low g bits of the remainder, which is what the
// bit field gives too).  Digits come out as r + Q in [Q - 2^(g-1), Q + 2^(g-1)) (< 2Q: fwd_pass
// input bound).  Needs C + Q < 2^32 (g <= 10 with Q < 2^28; checked by Engine::gate_args).
// SG: the digits themselves, signed (field f -> f - 2^(g-1) is the sign-extension of f with its
// top bit flipped, so one XOR with M and a signed bit-field extract per digit).
struct Dec {
    uint32_t Q, Qh, C, CmQ, g, off, M;
};
FHE_DEV Dec make_dec(uint32_t Q, uint32_t g) {
    const uint32_t h = 1u << (g - 1), C = h * (1u + (1u << g) + (1u << (2 * g)));
    return Dec{Q, Q >> 1, C, C - Q, g, Q - h, (h << g) | (h << (2 * g))};
}
template <bool SG>
FHE_DEV void decompose2(uint32_t x, const Dec& c, uint32_t& dA, uint32_t& dB) {
    const uint32_t u = x >= c.Qh ? x + c.CmQ : x + c.C;  // d + C, d = x or x - Q
    if (SG) {
        const int32_t w = (int32_t)(u ^ c.M);
        dA              = (uint32_t)__builtin_amdgcn_sbfe(w, c.g, c.g);
        dB              = (uint32_t)__builtin_amdgcn_sbfe(w, 2 * c.g, c.g);
    } else {
        dA = __builtin_amdgcn_ubfe(u, c.g, c.g) + c.off;
        dB = __builtin_amdgcn_ubfe(u, 2 * c.g, c.g) + c.off;
    }
}

// ModSwitch RoundqQ (lwe-pke.cpp:41-46): floor(0.5 + v*to/from) mod to, in IEEE double in
// the reference.  For v*to < 2^53, v < from and odd `from` (or power-of-two from/to) the
// double expression never crosses a rounding boundary, so it equals the exact integer
// floor((2 v to + from) / (2 from)) (proof in DESIGN.md, exhaustively tested).
FHE_DEV uint32_t mod_switch(uint64_t v, uint64_t from, uint64_t to) {
    uint64_t r = (2 * v * to + from) / (2 * from);
    return (uint32_t)(r % to);
}

// accumulator I/O of the seam instantiations (GateArgs::acc_io): lane (h, l) register r holds
// EVAL slot (l << 5) | r of component h.  In: canonical u64 -> N^-1-scaled residue (the keys carry
// N^-1, BootTables::ninvR).  Out: any |acc| < 2^31 -> acc N mod Q, canonical u64.
FHE_DEV void acc_load(uint32_t (&acc)[32], const GateArgs& g, uint32_t gate, int h, int l, uint32_t ninvR,
                      const Mod& m) {
    const uint64_t* src = g.acc_io + ((size_t)gate * 2 + h) * g.N + ((uint32_t)l << 5);
#pragma unroll
    for (int r = 0; r < 32; ++r) acc[r] = csub(mont_mul((uint32_t)src[r], ninvR, m), m.Q);
}
FHE_DEV void acc_store(const uint32_t (&acc)[32], const GateArgs& g, uint32_t gate, int h, int l, uint32_t nR,
                       const Mod& m) {
    uint64_t* dst = g.acc_io + ((size_t)gate * 2 + h) * g.N + ((uint32_t)l << 5);
#pragma unroll
    for (int r = 0; r < 32; ++r) {
        const int32_t v = (int32_t)smont_mul(acc[r], nR, m);
        dst[r] = (uint64_t)(uint32_t)(v < 0 ? v + (int32_t)m.Q : v);
    }
}

}  // namespace

// ---------------------------------------------------------------------------
// prep: ct = combination of the inputs (GateInputs, boot.h) mod q, doubled for XOR/XNOR
// (binfhe-base-scheme.cpp:95-107, :146-150, :180-182); monomial exponent per i:
// ((q - a_i) mod q) * (2N / q) (rgsw-acc-cggi.cpp:62-66)
// ---------------------------------------------------------------------------
namespace {
FHE_DEV uint32_t combine(const GateInputs& in, const uint64_t* const* v, size_t t, uint32_t boff, uint32_t qm,
                         uint32_t dbl) {
    uint32_t s = boff;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (j < (int)in.k) {
            const uint32_t x = (uint32_t)v[j][t];
            s += ((in.neg_mask >> j) & 1) ? 0u - x : x;
        }
    }
    s &= qm;
    return dbl ? (2 * s) & qm : s;
}
}  // namespace

__global__ void k_prep_ginx(GateInputs in, GateArgs g, uint16_t* __restrict__ idx, uint32_t* __restrict__ tvb) {
    const uint64_t total = (uint64_t)g.count * g.n;
    const uint32_t qm = g.ctmod - 1, mbymod = 2 * g.N / g.ctmod;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t a = combine(in, in.a, t, 0, qm, g.xor_double);
        idx[t] = (uint16_t)(((g.ctmod - a) & qm) * mbymod);
    }
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < g.count; t += (uint64_t)gridDim.x * blockDim.x)
        tvb[t] = combine(in, in.b, t, in.boff, qm, g.xor_double);
}

// ---------------------------------------------------------------------------
// fused blind rotation, 4 gates (waves) per 256-thread workgroup
// ---------------------------------------------------------------------------
constexpr int kWaves = 4;
// LZ: the monomial table holds (plain, Montgomery) pairs
constexpr size_t boot_lds(bool full, bool lz) {
    return (size_t)(992 * 2 + (lz ? 2 : 1) * (full ? kMonoTableWords : kMonoHalfWords) + kWaves * 2 * kTile) * 4;
}

// MFULL: full-resolution monomial table (ciphertext modulus 2N, any exponent); otherwise the
// half-resolution table (even exponents: every gate), where slots r and r ^ 1 share a monomial
// and the compiler drops half of the table reads.
// ACCIO: Backend::BlindRotate seam -- the accumulator is read from and written back to g.acc_io
// (GateArgs) instead of the test vector / extraction (EvalAcc itself, rgsw-acc-cggi.cpp:59-68)
template <bool MFULL, bool LZ, bool ACCIO = false>
__global__ void __launch_bounds__(256, FHE_WAVES_PER_EU)
    k_blind_rotate_ginx(GateArgs g, BootTables T, const uint2* __restrict__ bsk, const uint16_t* __restrict__ idx,
                        const uint32_t* __restrict__ tvb, uint32_t* __restrict__ ext_a, uint32_t* __restrict__ ext_b,
                        const uint32_t* __restrict__ twAf, const uint32_t* __restrict__ twAi) {
    // twAf / twAi = T.twA_fwd / T.twA_inv as restrict const arguments: the uniform A'-stage
    // twiddles then come through the scalar cache (s_load) instead of vector loads
    extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
    uint32_t* s_twBf = sm;
    uint32_t* s_twBi = sm + 992;
    // the dynamic LDS size and the tile region follow the table (launch_blind_rotate_ginx)
    constexpr bool mfull = MFULL;
    constexpr int mwords = mfull ? kMonoTableWords : kMonoHalfWords;
    uint32_t* s_mono = sm + 1984;
    uint2* s_mono2   = reinterpret_cast<uint2*>(sm + 1984);  // LZ: (plain, Montgomery) pairs
    uint32_t* s_tile = sm + 1984 + (LZ ? 2 : 1) * mwords;
    for (int i = threadIdx.x; i < 992; i += 256) {
        s_twBf[i] = T.twB_fwd[i];
        s_twBi[i] = T.twB_inv[i];
    }
    {
        const uint32_t* src = mfull ? T.mono_full : T.mono;
        const uint32_t* srp = mfull ? T.monoP_full : T.monoP;
        for (int i = threadIdx.x; i < mwords; i += 256) {
            if (LZ) s_mono2[i] = make_uint2(srp[i], src[i]);
            else s_mono[i] = src[i];
        }
    }
    constexpr uint32_t msh = mfull ? 0u : 1u, emask = mfull ? 2047u : 1023u, umask = mfull ? 31u : 15u;
    constexpr uint32_t eper = mfull ? 4096u : 2048u;
    __syncthreads();

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, l = lane & 31;
    const uint32_t gate = blockIdx.x * kWaves + wave;
    if (gate >= g.count) return;  // no workgroup barrier below this point
    uint32_t* tileW = s_tile + wave * 2 * kTile;
    uint32_t* tile  = tileW + h * kTile;
    const Mod m0 = make_mod(T);
    const Mod& m  = m0;
#if FHE_K1_PRIO || FHE_K1_STAGGER
    uint32_t hwid;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    const uint32_t tgs = (hwid >> 16) & 15;  // the workgroup's slot on its CU
    if (FHE_K1_PRIO && (tgs & 1)) __builtin_amdgcn_s_setprio(1);
    if (tgs & 1)
        for (int z = 0; z < FHE_K1_STAGGER; ++z) __builtin_amdgcn_s_sleep(127);
#endif

    // test vector (BootstrapGateCore, binfhe-base-scheme.cpp:556-575): acc1 = NTT(m), acc0 = 0
    uint32_t acc[32];
    if (ACCIO && !g.acc_tv) {
        acc_load(acc, g, gate, h, l, T.ninvR, m);
    } else {
        const uint32_t b = tvb[gate], cm = g.ctmod - 1;
        // EvalFuncMultiOutput: table gate % tv_mod (GateArgs::tv_mod)
        const uint32_t tvo = g.tv_mod > 1 ? (gate % g.tv_mod) * g.ctmod : 0u;
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            const uint32_t x = (uint32_t)(r << 5) | l;
            uint32_t v       = 0;
            if (h == 1 && x % g.factor == 0) {
                const uint32_t bx = (b - x / g.factor) & cm;
                v                 = g.tv ? g.tv[tvo + bx] : (bx >= g.lb && bx < g.ub) ? g.lv : g.uv;
            }
            acc[r] = v;
        }
        fwd_pass(acc, tile, l, T.twA_fwd, s_twBf, m);
        // canonical, then scaled by N^-1 like everything the keys produce (BootTables::w1R)
#pragma unroll
        for (int r = 0; r < 32; ++r)
            acc[r] = csub(mont_mul(csub(csub(csub(acc[r], 4 * m.Q2), 2 * m.Q2), m.Q2), T.ninvR, m), m.Q);
    }

    const uint16_t* gidx = idx + (size_t)gate * g.n;
    const uint32_t lbase = 2 * brv5(l) + 1;
    const Dec dec        = make_dec(m.Q, g.gbits);
    const uint64_t moff  = 64ull * m.Q * m.Q;
    const uint32_t lofs  = (uint32_t)lane;
    const int xaddr      = (lane ^ 32) << 2;
    for (uint32_t i = 0; i < g.n; ++i) {
        const Mod m = fresh_nq(m0);
        const uint32_t a = __builtin_amdgcn_readfirstlane((uint32_t)gidx[i]);
        uint32_t dA[32], dB[32];
        // --- iNTT of a copy of acc -> canonical COEF (AddToAccCGGI :104-106)
#pragma unroll
        for (int r = 0; r < 32; ++r) dA[r] = acc[r];
        if (LZ) inv_pass_s<kAccBoundLZ, true, true>(dA, tile, l, twAi, s_twBi, T.w1R, T.oneR, m);
        else inv_pass(dA, tile, l, T.twA_inv, s_twBi, T.w1R, m);
        // --- SignedDigitDecompose (rgsw-acc.cpp:54-91): drop the lowest signed digit,
        //     keep the next two.  Half h decomposes acc_h: dA = D_h, dB = D_{2+h}.
#pragma unroll
        for (int r = 0; r < 32; ++r) decompose2<LZ>(dA[r], dec, dA[r], dB[r]);
        // --- NTT of the four digit polynomials (two per pass, one per half)
        fwd_pass2<LZ ? 1 : 0, true>(dA, dB, tile, l, twAf, s_twBf, m);
        // --- external product + CMUX, slot by slot.  Lane (h, l) owns slots
        //     l*32 + r of component h; its keys are 16-byte vectors (4 slots) laid
        //     out so that each load instruction reads 1 KiB contiguous.
        // monomial addressing: slot x = (l << 5) | r evaluates at psi^(2 brv(x) + 1), so X^a maps to
        // psi^e with e = a (2 brv(x) + 1) = a (2 brv5(l) + 1) + 64 (a brv5(r) mod 32)  (mod 2N):
        // a per-lane part plus a wave-uniform multiple of 64.  Half-resolution table (a = 2a'):
        // f = e / 2 = a' (2 brv5(l) + 1) + 64 ((a' brv5(r)) mod 16) (mod N), entry f at f + (f >> 5);
        // full table: e itself.  64 k in (half or full) index space moves a position by 66 k.
        const uint32_t as = a >> msh;
        const uint32_t el = (as * lbase) & emask;
        const uint32_t Pp = el + (el >> 5);                    // index el + 64k       -> Pp + 66k
        const uint32_t gl = eper - el;
        const uint32_t Pn = gl + (gl >> 5);                    // index eper - el - 64k -> Pn - 66k
        // one 16-byte vector per digit row and slot pair: (K+[2k], K+[2k+1], K-[2k], K-[2k+1])
        const uint4* kb4 = reinterpret_cast<const uint4*>(bsk) + (size_t)i * (4 * 16 * 64);
        uint4 kq[FHE_KEY_PF + 1][4];
#pragma unroll
        for (int k = 0; k < FHE_KEY_PF; ++k)
#pragma unroll
            for (int d = 0; d < 4; ++d) kq[k][d] = kload(kb4, (d * 16 + k) * 64 + lofs);
        // the other half's digits (ds_bpermute) and the monomial pairs of slot pair k + 1 are
        // requested before slot pair k is consumed (LDS latency off the critical path)
        uint32_t xo[2][4];
        uint2 mo[2][2][2];
        auto issue = [&](int k, int b) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int r      = 2 * k + e;
                xo[b][2 * e]     = other_half(dA[r], xaddr);
                xo[b][2 * e + 1] = other_half(dB[r], xaddr);
                const uint32_t u = __builtin_amdgcn_readfirstlane((as * (uint32_t)(__builtin_bitreverse32(r) >> 27)) & umask) * 66;
                if (e == 0 || mfull) {
                    mo[b][e][0] = s_mono2[Pp + u];
                    mo[b][e][1] = s_mono2[Pn - u];
                } else {  // half table: slots r, r ^ 1 share the monomial
                    mo[b][1][0] = mo[b][0][0];
                    mo[b][1][1] = mo[b][0][1];
                }
            }
        };
        issue(0, 0);
#pragma clang loop unroll(full)
        for (int k = 0; k < 16; ++k) {
            if (k + FHE_KEY_PF < 16) {
#pragma unroll
                for (int d = 0; d < 4; ++d) kq[(k + FHE_KEY_PF) % (FHE_KEY_PF + 1)][d] = kload(kb4, (d * 16 + k + FHE_KEY_PF) * 64 + lofs);
            }
            if (k + 1 < 16) issue(k + 1, (k + 1) & 1);
            asm volatile("" ::: "memory");
#define KP(d) make_uint2(kq[k % (FHE_KEY_PF + 1)][d].x, kq[k % (FHE_KEY_PF + 1)][d].y)
#define KN(d) make_uint2(kq[k % (FHE_KEY_PF + 1)][d].z, kq[k % (FHE_KEY_PF + 1)][d].w)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int r = 2 * k + e;
                // all four digits in every lane: D0/D1 = digit A of acc0/acc1, D2/D3 = digit B
                const uint32_t D0 = dA[r], D1 = xo[k & 1][2 * e], D2 = dB[r], D3 = xo[k & 1][2 * e + 1];
                // slot x = l*32 + r evaluates at psi^(2 brv(x) + 1), 2 brv(x) + 1 = 64 brv5(r) + 2 brv5(l) + 1
                const uint32_t u  = __builtin_amdgcn_readfirstlane((as * (uint32_t)(__builtin_bitreverse32(r) >> 27)) & umask) * 66;
                if (LZ) {
                    // S1, S2 = sum_d D_d K(+/-)_d unreduced (|.| < 40 Q^2 < 2^60, keys x 2^32); the monomial
                    // products S (X^m - 1) = lo(S) m + hi(S) (m 2^32) use the (plain, Montgomery) table pair,
                    // and acc is folded in as acc (2^32 mod Q): one signed Montgomery reduction per slot.
                    // |acc| < 2.75 Q in and out (S < 2^32 Q (2 + 1/8) + 2.75 Q^2).
                    const int64_t S1 = (int64_t)mac4<true>(D0, D1, D2, D3, e ? KP(0).y : KP(0).x, e ? KP(1).y : KP(1).x,
                                                           e ? KP(2).y : KP(2).x, e ? KP(3).y : KP(3).x, 0);
                    const int64_t S2 = (int64_t)mac4<true>(D0, D1, D2, D3, e ? KN(0).y : KN(0).x, e ? KN(1).y : KN(1).x,
                                                           e ? KN(2).y : KN(2).x, e ? KN(3).y : KN(3).x, 0);
                    const uint2 mp = mo[k & 1][e][0], mn = mo[k & 1][e][1];
                    int64_t S = (int64_t)((uint64_t)(uint32_t)S1 * mp.x) + (int64_t)(int32_t)(S1 >> 32) * (int32_t)mp.y;
                    S += (int64_t)((uint64_t)(uint32_t)S2 * mn.x) + (int64_t)(int32_t)(S2 >> 32) * (int32_t)mn.y;
                    S += (int64_t)(int32_t)acc[r] * (int32_t)T.oneR;
                    acc[r] = smont_red(S, m);
                } else {
                    const uint64_t S1 = mac4<LZ>(D0, D1, D2, D3, e ? KP(0).y : KP(0).x, e ? KP(1).y : KP(1).x,
                                                 e ? KP(2).y : KP(2).x, e ? KP(3).y : KP(3).x, moff);
                    const uint64_t S2 = mac4<LZ>(D0, D1, D2, D3, e ? KN(0).y : KN(0).x, e ? KN(1).y : KN(1).x,
                                                 e ? KN(2).y : KN(2).x, e ? KN(3).y : KN(3).x, moff);
                    const uint32_t t1 = mont_red(S1, m), t2 = mont_red(S2, m);
                    const uint64_t S  = (uint64_t)t1 * s_mono[Pp + u] + (uint64_t)t2 * s_mono[Pn - u];
                    // digits < 16Q (Q < 2^28): S1, S2 < 64 Q^2 -> t1, t2 < 5Q; S < 10Q^2 -> mont_red < 1.7Q;
                    // acc kept in [0, 2Q)
                    acc[r]            = csub(acc[r] + mont_red(S, m), m.Q2);
                }
            }
#undef KP
#undef KN
        }
    }

    if (ACCIO) {
        acc_store(acc, g, gate, h, l, T.nR, m);
        return;
    }
    // --- extraction (binfhe-base-scheme.cpp:110-121): acc0 <- Transpose(acc0) (automorphism
    // 2N-1), both to COEF; ctExt = (acc0 coefficients, (Q>>3)+1 + acc1[0]); then ModSwitch to qKS.
    // In COEF, Transpose maps coefficient k to -a_(N-k) (k >= 1), a_0 to itself.
    if (LZ) inv_pass_s<kAccBoundLZ>(acc, tile, l, T.twA_inv, s_twBi, T.w1R, T.oneR, m);
    else inv_pass(acc, tile, l, T.twA_inv, s_twBi, T.w1R, m);
    wave_lds_sync();
    if (h == 0) {
#pragma unroll
        for (int r = 0; r < 32; ++r) tileW[(r << 5) | l] = acc[r];
    } else if (l == 0) {
        tileW[1024] = acc[0];
    }
    wave_lds_sync();
    uint32_t* oa = ext_a + (size_t)gate * g.N;
#pragma unroll 4
    for (int t = 0; t < 16; ++t) {
        const uint32_t j = (uint32_t)lane + 64u * t;
        const uint32_t c = tileW[j == 0 ? 0 : g.N - j];
        const uint32_t v = (j == 0 || c == 0) ? c : m.Q - c;
        oa[j]            = g.msb_out ? mod_switch(v, m.Q, g.qKS) : v;
    }
    if (lane == 0) {
        const uint32_t bb = add_mod(g.b_const, tileW[1024], m.Q);
        ext_b[gate]       = g.msb_out ? mod_switch(bb, m.Q, g.qKS) : bb;
    }
}

hipError_t launch_prep_ginx(const GateArgs& g, const GateInputs& in, uint16_t* idx, uint32_t* tvb, hipStream_t s) {
    if (g.count == 0) return hipSuccess;
    if (in.k < 1 || in.k > 4) return hipErrorInvalidValue;
    const uint64_t total = (uint64_t)g.count * g.n;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(k_prep_ginx, dim3(blocks), dim3(256), 0, s, in, g, idx, tvb);
    return hipGetLastError();
}

hipError_t launch_blind_rotate_ginx(const GateArgs& g, const BootTables& t, const void* bsk, const uint16_t* idx,
                                    const uint32_t* tvb, uint32_t* ext_a, uint32_t* ext_b, hipStream_t s) {
    if (g.count == 0) return hipSuccess;
    const uint32_t blocks = (g.count + kWaves - 1) / kWaves;
    const uint2* k = reinterpret_cast<const uint2*>(bsk);
    const bool lz  = t.Q < (1u << 27);
    const bool full = g.ctmod == 2 * g.N;
#define FHE_LAUNCH_GINX(MF, LZ_, IO)                                                                        \
    hipLaunchKernelGGL((k_blind_rotate_ginx<MF, LZ_, IO>), dim3(blocks), dim3(256), boot_lds(MF, LZ_), s, g, t, k, \
                       idx, tvb, ext_a, ext_b, t.twA_fwd, t.twA_inv)
    if (g.acc_io) {
        if (full) { if (lz) FHE_LAUNCH_GINX(true, true, true); else FHE_LAUNCH_GINX(true, false, true); }
        else { if (lz) FHE_LAUNCH_GINX(false, true, true); else FHE_LAUNCH_GINX(false, false, true); }
    } else if (full) {
        if (lz) FHE_LAUNCH_GINX(true, true, false); else FHE_LAUNCH_GINX(true, false, false);
    } else {
        if (lz) FHE_LAUNCH_GINX(false, true, false); else FHE_LAUNCH_GINX(false, false, false);
    }
#undef FHE_LAUNCH_GINX
    return hipGetLastError();
}


// ===========================================================================
// LMKCDEY (RingGSWAccumulatorLMKCDEY::EvalAcc, src/binfhe/lib/rgsw-acc-lmkcdey.cpp:70-158)
// ===========================================================================
// Schedule ops, per gate, in the reference's exact order:
//   EXT(i)  (i < 0x8000): AddToAccLMKCDEY with (*ek)[0][0][i]            (:228-254)
//   AUTO(t) (0x8000 | t): Automorphism by 5^t (t >= 1) or by 2N-5 (t = 0)
//                         with (*ek)[0][1][t]                              (:257-287)
// k_prep_lmk_w builds them with a stable counting sort of the a_i into the
// logGen groups (permuteMap, :83-94) and replays the nSkips logic (:99-157).
namespace {
// EVAL-domain automorphism X -> X^k (poly-impl.h:350-356 / PrecomputeAutoMap, nbtheory2.cpp:264-275):
// out[slot brv(j)] = in[slot brv(((2j+1)k mod 2N) >> 1)].  Through the half-wave's LDS region
// (row stride 33: conflict-free writes).
// Output slot x = (l << 5) | r has j = brv10(x) = (brv5(r) << 5) | brv5(l), so
// (2j+1) k = (2 brv5(l) + 1) k + 64 brv5(r) k: one per-lane term plus a wave-uniform
// term per register (k is uniform), and no per-register index stays live across calls.
FHE_DEV void automorphism_eval(uint32_t (&v)[32], uint32_t* region, int l, uint32_t k) {
#pragma unroll
    for (int r = 0; r < 32; ++r) region[l * 33 + r] = v[r];
    wave_lds_sync();
    const uint32_t cl = (2 * (__builtin_bitreverse32((uint32_t)l) >> 27) + 1) * k;
#pragma unroll
    for (int r = 0; r < 32; ++r) {
        const uint32_t sr = ((__builtin_bitreverse32((uint32_t)r) >> 27) << 6) * k;  // uniform
        const uint32_t t  = ((cl + sr) & 2047) >> 1;
        const uint32_t sx = __builtin_bitreverse32(t) >> 22;   // source slot brv10(t)
        v[r]              = region[sx + (sx >> 5)];
    }
    wave_lds_sync();
}
// ---- LMKCDEY automorphism op, acc0' inverse-transformed across the whole wave ---------------------
// Only acc0' of an automorphism is decomposed, so instead of a half-wave pass per component (half 1
// transforming acc1' for nothing) the wave transforms acc0' alone with 16 coefficients per lane,
// in the three layouts of ntt.hip k_ntt1024w (x = EVAL slot or coefficient index):
//   C: lane L = x7..x2, register r = (x9x8) << 2 | x1x0;   B: lane = (x9..x6) << 2 | x1x0,
//   register = x5..x2;   A: lane = x5..x0, register = x9..x6.   LDS word of x: x + 4 (x >> 6).
FHE_DEV int wt64(int x) { return x + ((x >> 6) << 2); }
struct InvPlanWW {
    bool red[10][16];  // reduce register r before stage s (C bit 0, C bit 1, B bits 0..3, A bits 0..2, last)
    bool redT[2][16];  // ... before the C -> B / B -> A transpose
    int fin[8];        // last-stage sum: |x + y| < 2^fin Q
    int cost;          // 2 per reduction + 1 per final conditional subtraction (their issue-cycle ratio)
};
// a transpose mixes every register, so the largest bound reaches all of them: registers above the
// threshold TT[k] are reduced before transpose k (round 5; without it the A stages of the LMKCDEY
// automorphism's inverse took 36 reductions per lane, with it 16).  make_inv_plan_ww searches the thresholds.
template <int BIN, int LIM>
constexpr InvPlanWW inv_plan_ww_t(int T0, int T1) {
    InvPlanWW p{};
    int B[16] = {};
    for (int r = 0; r < 16; ++r) B[r] = BIN;
    const int bits[10] = {0, 1, 0, 1, 2, 3, 0, 1, 2, 3};
    int nred = 0;
    for (int st = 0; st < 10; ++st) {
        if (st == 2 || st == 6) {
            const int k = st == 2 ? 0 : 1, T = k ? T1 : T0;
            int U = 0;
            for (int r = 0; r < 16; ++r) {
                if (B[r] > T) {
                    B[r]         = 10;
                    p.redT[k][r] = true;
                    ++nred;
                }
                U = B[r] > U ? B[r] : U;
            }
            for (int r = 0; r < 16; ++r) B[r] = U;
        }
        const int bt = bits[st];
        for (int r = 0; r < 16; ++r) {
            if (r & (1 << bt)) continue;
            const int q = r | (1 << bt);
            while (B[r] + B[q] > LIM) {
                const int e  = B[r] >= B[q] ? r : q;
                B[e]         = 10;
                p.red[st][e] = true;
                ++nred;
            }
            if (st == 9) {
                int f = 0;
                while ((10 << f) < B[r] + B[q]) ++f;
                p.fin[r] = f;
            }
            B[r] = B[r] + B[q];
            B[q] = 10;
        }
    }
    p.cost = 2 * nred;
    for (int r = 0; r < 8; ++r) p.cost += p.fin[r] + 1;
    return p;
}
constexpr int kPlanT[8] = {10, 15, 20, 30, 40, 60, 80, 1 << 20};  // candidate thresholds (the last: none)
#ifndef FHE_PLAN_T
#define FHE_PLAN_T 1  // 0: no reductions before the transposes (the round-4 plans)
#endif
constexpr int kPlanTN = FHE_PLAN_T ? 8 : 0;
template <int BIN, int LIM>
constexpr InvPlanWW make_inv_plan_ww() {
    InvPlanWW best = inv_plan_ww_t<BIN, LIM>(kPlanT[7], kPlanT[7]);
    for (int a = 0; a < kPlanTN; ++a)
        for (int b = 0; b < kPlanTN; ++b) {
            const InvPlanWW p = inv_plan_ww_t<BIN, LIM>(kPlanT[a], kPlanT[b]);
            if (p.cost < best.cost) best = p;
        }
    return best;
}
// EVAL (layout C, |v| < BIN Q / 10) -> canonical COEF (layout A); the keys carry N^-1, so the last
// stage scales by TableI[1] only (as inv_pass_s).  tile: 1088 words of this wave; s_tabI: TableI.
template <int BIN, bool LZ>
FHE_DEV void inv_wave_s(uint32_t (&v)[16], uint32_t* tile, int L, const uint32_t* s_tabI, uint32_t w1R,
                        uint32_t oneR, const Mod& m) {
    constexpr InvPlanWW P = make_inv_plan_ww<BIN, lim_s(LZ)>();
    auto redp = [&](int st) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if (P.red[st][r]) v[r] = smont_mul(v[r], oneR, m);
    };
    auto redt = [&](int k) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if (P.redT[k][r]) v[r] = smont_mul(v[r], oneR, m);
    };
    auto gs = [&](uint32_t& x, uint32_t& y, uint32_t w) {
        const uint32_t t = x + y;
        y                = smont_mul(x - y, w, m);
        x                = t;
    };
    const int G = L >> 2, jj = L & 3;
    redp(0);
#pragma unroll
    for (int hh = 0; hh < 4; ++hh) {
        const uint2 w0 = *reinterpret_cast<const uint2*>(s_tabI + 512 + (hh << 7) + (L << 1));
        gs(v[4 * hh], v[4 * hh + 1], w0.x);
        gs(v[4 * hh + 2], v[4 * hh + 3], w0.y);
    }
    redp(1);
#pragma unroll
    for (int hh = 0; hh < 4; ++hh) {
        const uint32_t w1 = s_tabI[256 + (hh << 6) + L];
        gs(v[4 * hh], v[4 * hh + 2], w1);
        gs(v[4 * hh + 1], v[4 * hh + 3], w1);
    }
    // C -> B
    redt(0);
#pragma unroll
    for (int hh = 0; hh < 4; ++hh)
        *reinterpret_cast<uint4*>(tile + wt64((hh << 8) | (L << 2))) = make_uint4(v[4 * hh], v[4 * hh + 1], v[4 * hh + 2], v[4 * hh + 3]);
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = tile[wt64((G << 6) | (r << 2) | jj)];
    wave_lds_sync();
#pragma unroll
    for (int b = 2; b <= 5; ++b) {
        const int rb = b - 2;
        redp(b);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (r & (1 << rb)) continue;
            gs(v[r], v[r | (1 << rb)], s_tabI[(1 << (9 - b)) + (G << (5 - b)) + (r >> (rb + 1))]);
        }
    }
    // B -> A
    redt(1);
#pragma unroll
    for (int r = 0; r < 16; ++r) tile[wt64((G << 6) | (r << 2) | jj)] = v[r];
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = tile[wt64((r << 6) | L)];
    wave_lds_sync();
#pragma unroll
    for (int b = 6; b <= 8; ++b) {
        const int rb = b - 6;
        redp(b);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (r & (1 << rb)) continue;
            gs(v[r], v[r | (1 << rb)], s_tabI[(1 << (9 - b)) + (r >> (rb + 1))]);
        }
    }
    // bit 9 (transformnat-impl.h:599-623), canonical results as inv_pass_s
    redp(9);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const uint32_t x = v[r], y = v[r | 8];
        uint32_t s       = x + y + (m.Q << P.fin[r]);
#pragma unroll
        for (int f = P.fin[r]; f >= 0; --f) s = csub(s, m.Q << f);
        const uint32_t d = smont_mul(x - y, w1R, m);
        v[r]             = s;
        v[r | 8]         = min(d, d + m.Q);
    }
}
// automorphism X -> X^k of both components (as automorphism_eval: every half-wave gets its own
// component back in layout B'), plus acc0' gathered into layout C for inv_wave_s
FHE_DEV void automorphism_wide(uint32_t (&v)[32], uint32_t (&a0)[16], uint32_t* region, const uint32_t* region0,
                               int l, int L, uint32_t k) {
    // slot s = (l << 5) | r is stored at its exponent index brv10(s) = brv5(r) << 5 | brv5(l)
    // (EVAL slot s holds the value at psi^(2 brv10(s) + 1)); the slot that reads exponent
    // index t' gathers index ((2 t' + 1) k mod 2N) >> 1: one add, one bit-field extract, one
    // address add per value
    const uint32_t bl = __builtin_bitreverse32((uint32_t)l) >> 27;
#pragma unroll
    for (int r = 0; r < 32; ++r) region[(((__builtin_bitreverse32((uint32_t)r) >> 27) << 5) | bl)] = v[r];
    wave_lds_sync();
    const uint32_t cl = (2 * bl + 1) * k;
#pragma unroll
    for (int r = 0; r < 32; ++r) {
        const uint32_t sr = ((__builtin_bitreverse32((uint32_t)r) >> 27) << 6) * k;  // uniform
        // FHE_LMK_ABL bit 2 (timing only): every gather at a conflict-free linear position instead
        v[r]              = region[(FHE_LMK_ABL & 4) ? ((((cl + sr) >> 1) & 992) | (uint32_t)l) : (((cl + sr) >> 1) & 1023)];
    }
    const uint32_t cL = (((__builtin_bitreverse32((uint32_t)L) >> 26) << 3) + 1) * k;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t H = (uint32_t)r >> 2, j = (uint32_t)r & 3;
        const uint32_t su = ((((j & 1) << 1 | j >> 1) << 9) + (((H & 1) << 1 | H >> 1) << 1)) * k;  // uniform
        a0[r]             = region0[(FHE_LMK_ABL & 4) ? ((((cL + su) >> 1) & 960) | (uint32_t)L) : (((cL + su) >> 1) & 1023)];
    }
    wave_lds_sync();
}

}  // namespace

// |acc| between ops (units of Q/10): 2 Q, or 2.2 Q for Q >= 2^27 with FHE_FWD_TIGHT (see there)
template <bool LZ> constexpr int kLmkAcc = (!LZ && FHE_FWD_TIGHT) ? 22 : 20;
// DM: the AP/DM accumulator runs the same op loop with external products only (AddToAccDM ==
// AddToAccLMKCDEY, rgsw-acc-dm.cpp:119-145) and no initial automorphism of acc1.
// DM needs no automorphism path and fits 168 VGPRs: 3 waves per SIMD
// ACCIO: Backend::BlindRotate / ExternalProduct seam (GateArgs::acc_io), as in k_blind_rotate_ginx
template <bool DM, bool LZ, bool ACCIO = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DM ? FHE_DM_WAVES : FHE_LMK_WAVES)))
    k_blind_rotate_lmk(GateArgs g, BootTables T, const uint2* __restrict__ bsk, const uint2* __restrict__ autok,
                       const uint16_t* __restrict__ ops, const uint32_t* __restrict__ nops, uint32_t maxops,
                       const uint32_t* __restrict__ tvb, uint32_t* __restrict__ ext_a, uint32_t* __restrict__ ext_b) {
    extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
    uint32_t* s_twBf = sm;
    uint32_t* s_twBi = sm + 992;
    uint32_t* s_tile = sm + 1984;
    for (int i = threadIdx.x; i < 992; i += 256) {
        s_twBf[i] = T.twB_fwd[i];
        s_twBi[i] = T.twB_inv[i];
    }
    uint32_t* s_tabI = s_tile + kWaves * 2 * kTile;  // FHE_AUTO_WIDE: TableI (1024 words)
    if (!DM)
        for (int i = threadIdx.x; i < 1024; i += 256) s_tabI[i] = T.tabI[i];
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, l = lane & 31;
    const uint32_t gate = blockIdx.x * kWaves + wave;
    if (gate >= g.count) return;
    uint32_t* tileW = s_tile + wave * 2 * kTile;
    uint32_t* tile  = tileW + h * kTile;
    const Mod m0 = make_mod(T);
    const Mod& m  = m0;
    const uint32_t M = 2 * g.N;

    uint32_t acc[32];
    if (ACCIO && !g.acc_tv) {
        acc_load(acc, g, gate, h, l, T.ninvR, m);
        // acc1 <- acc1(X^(2N-5)) (:99) on half 1 only: X^1 (the identity) on half 0
        if (!DM) automorphism_eval(acc, tile, l, h ? M - 5 : 1u);
    } else {
        const uint32_t b = tvb[gate], cm = g.ctmod - 1;
        // EvalFuncMultiOutput: table gate % tv_mod (GateArgs::tv_mod)
        const uint32_t tvo = g.tv_mod > 1 ? (gate % g.tv_mod) * g.ctmod : 0u;
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            const uint32_t x = (uint32_t)(r << 5) | l;
            uint32_t v       = 0;
            if (h == 1 && x % g.factor == 0) {
                const uint32_t bx = (b - x / g.factor) & cm;
                v                 = g.tv ? g.tv[tvo + bx] : (bx >= g.lb && bx < g.ub) ? g.lv : g.uv;
            }
            acc[r] = v;
        }
        fwd_pass(acc, tile, l, T.twA_fwd, s_twBf, m);
        // canonical, then scaled by N^-1 like everything the keys produce (BootTables::w1R)
#pragma unroll
        for (int r = 0; r < 32; ++r)
            acc[r] = csub(mont_mul(csub(csub(csub(acc[r], 4 * m.Q2), 2 * m.Q2), m.Q2), T.ninvR, m), m.Q);
        // acc1 <- acc1(X^(2N-5))   (:99); applied to both halves, acc0 = 0 is invariant
        if (!DM) automorphism_eval(acc, tile, l, M - 5);
    }

    const Dec dec     = make_dec(m.Q, g.gbits);
    const uint16_t* gops = ops + (size_t)gate * maxops;
    const uint32_t cnt   = __builtin_amdgcn_readfirstlane(nops[gate]);  // uniform: a scalar loop
    // Signed residues throughout (Q < 2^28): acc in (-2Q, 2Q) between ops (one signed Montgomery
    // reduction of the digit x key sum), signed inverse NTT to canonical COEF, balanced digits as
    // signed words, signed forward NTT (FM 1 for Q < 2^27, FM 2 above).
    constexpr int FM = LZ ? 1 : 2;
    const uint32_t oneRh = h ? m0.oneR : 0u;  // automorphism: half 1 accumulates, half 0 is replaced
    const int xaddr      = (lane ^ 32) << 2;
    for (uint32_t it = 0; it < cnt; ++it) {
        const Mod m       = fresh_nq(m0);
        // the uniform twiddles re-read per op: hoisted out of the branchy loop they would hold
        // 62 VGPRs across it (spills)
        const uint32_t* twAf = T.twA_fwd;
        const uint32_t* twAi = T.twA_inv;
        asm volatile("" : "+s"(twAf), "+s"(twAi));
#if FHE_LMK_OPAQUE
        // the lane index and the wave's LDS regions made opaque per op as well: every per-lane address
        // of the op body is then derived inside it instead of being hoisted as a loop-invariant VGPR
        int l_o = l, lane_o = lane;
        uint32_t *tile_o = tile, *tileW_o = tileW;
        asm volatile("" : "+v"(l_o), "+v"(lane_o), "+v"(tile_o), "+v"(tileW_o));
        const int l = l_o, lane = lane_o, xaddr = (lane ^ 32) << 2;
        uint32_t* const tile  = tile_o;
        uint32_t* const tileW = tileW_o;
#endif
        const uint32_t op = __builtin_amdgcn_readfirstlane((uint32_t)gops[it]);
        uint32_t dA[32], dB[32];
        if (DM || !(op & 0x8000u)) {
            // ---- AddToAccLMKCDEY / AddToAccDM: acc <- sum_d D_d * ek[op][d]   (acc replaced)
            const uint4* kb4 = reinterpret_cast<const uint4*>(bsk) + (size_t)((FHE_LMK_ABL & 1) ? 0u : op) * (4 * 8 * 64);
            constexpr int KPF = FHE_LMK_KPF;
            uint4 kq[KPF + 1][4];
#pragma unroll
            for (int r = 0; r < 32; ++r) dA[r] = acc[r];
            inv_pass_s<kLmkAcc<LZ>, LZ, !DM && FHE_LMK_PRE>(dA, tile, l, twAi, s_twBi, T.w1R, m.oneR, m);
#pragma unroll
            for (int r = 0; r < 32; ++r) decompose2<true>(dA[r], dec, dA[r], dB[r]);
            fwd_pass2<FM, !DM && FHE_LMK_PRE>(dA, dB, tile, l, twAf, s_twBf, m);
            // one 16-byte vector per digit row and 4 slots (boot.h row_off)
#pragma unroll
            for (int p = 0; p < KPF; ++p)
#pragma unroll
                for (int d = 0; d < 4; ++d) kq[p][d] = kload(kb4, (d * 8 + p) * 64 + lane);
            // LMKCDEY: the other half's digits of slots 4(kk+1).. requested before 4kk.. are consumed
            constexpr bool PIPE = !DM;
            uint32_t xq[2][8];
            auto issue = [&](int kk, int b) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    xq[b][2 * e]     = other_half(dA[4 * kk + e], xaddr);
                    xq[b][2 * e + 1] = other_half(dB[4 * kk + e], xaddr);
                }
            };
            if (PIPE) issue(0, 0);
#pragma clang loop unroll(full)
            for (int kk = 0; kk < 8; ++kk) {
                if (kk + KPF < 8) {  // request slots 4(kk+KPF).. while 4kk.. are consumed
#pragma unroll
                    for (int d = 0; d < 4; ++d)
                        kq[(kk + KPF) % (KPF + 1)][d] = kload(kb4, (d * 8 + kk + KPF) * 64 + lane);
                }
                if (PIPE && kk + 1 < 8) issue(kk + 1, (kk + 1) & 1);
                asm volatile("" ::: "memory");
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = 4 * kk + e;
#define KC(d) (e == 0 ? kq[kk % (KPF + 1)][d].x : e == 1 ? kq[kk % (KPF + 1)][d].y : e == 2 ? kq[kk % (KPF + 1)][d].z : kq[kk % (KPF + 1)][d].w)
                    const uint32_t D0 = dA[r], D2 = dB[r];
                    const uint32_t D1 = (FHE_LMK_ABL & 8) ? dA[r] ^ 1u : PIPE ? xq[kk & 1][2 * e] : other_half(dA[r], xaddr);
                    const uint32_t D3 = (FHE_LMK_ABL & 8) ? dB[r] ^ 1u : PIPE ? xq[kk & 1][2 * e + 1] : other_half(dB[r], xaddr);
                    // |D| < 10Q + 2^8 (Q < 2^27) or 6Q (Q < 2^28; 6.67Q with FHE_FWD_TIGHT): |S| < 40 Q^2
                    // or 24 Q^2 (26.7 Q^2), so |S| 2^-32 + Q/2 < 2Q (2.2Q: kLmkAcc)
                    const int64_t S = (int64_t)mac4<true>(D0, D1, D2, D3, KC(0), KC(1), KC(2), KC(3), 0);
                    acc[r] = smont_red(S, m);
#undef KC
                }
            }
        } else {
            // ---- Automorphism(5^t or 2N-5, autokey[t])
            const uint32_t t = op & 0x7fffu;
            uint32_t kexp    = M - 5;
            if (t) {
                kexp = 1;
                for (uint32_t z = 0; z < t; ++z) kexp = (kexp * 5) & (M - 1);
            }
            asm volatile("" : "+s"(kexp));  // no reuse of the prologue's (2N - 5) index math (spills)
            {
                // acc0' across the wave: layout C -> canonical COEF layout A (16 per lane), its two
                // digits scattered into the two tiles in A' order (digit A for half 0, B for half 1)
                uint32_t a0[16];
                automorphism_wide(acc, a0, tile, tileW, l, lane, kexp);
                inv_wave_s<kLmkAcc<LZ>, LZ>(a0, tileW, lane, s_tabI, T.w1R, m.oneR, m);
#if FHE_LMK_SWAP
                // coefficient x = (r << 6) | lane goes to half-wave register (x >> 5), lane x & 31 of half 0
                // (digit A) and half 1 (digit B): one half exchange per register pair (v_permlane32_swap:
                // lanes 32..63 of x trade places with lanes 0..31 of y) instead of a pass through LDS
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    uint32_t x, y;
                    decompose2<true>(a0[r], dec, x, y);
                    const auto p = __builtin_amdgcn_permlane32_swap(x, y, false, false);
                    dA[2 * r]     = p[0];
                    dA[2 * r + 1] = p[1];
                }
#else
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    uint32_t x, y;
                    decompose2<true>(a0[r], dec, x, y);
                    const uint32_t c = ((uint32_t)r << 6) | (uint32_t)lane;
                    tileW[(c & 31) * 33 + (c >> 5)]         = x;
                    tileW[kTile + (c & 31) * 33 + (c >> 5)] = y;
                }
                wave_lds_sync();
#pragma unroll
                for (int r = 0; r < 32; ++r) dA[r] = tile[l * 33 + r];
                wave_lds_sync();
#endif
            }
            fwd_pass_s<FM>(dA, tile, l, twAf, s_twBf, m);  // half 0: EVAL digit A, half 1: EVAL digit B
            const uint4* kb4 = reinterpret_cast<const uint4*>(autok) + (size_t)((FHE_LMK_ABL & 2) ? 0u : t) * (2 * 8 * 64);
            constexpr int AKPF = FHE_LMK_AKPF;
            uint4 ka[AKPF + 1][2];
#pragma unroll
            for (int p = 0; p < AKPF; ++p) {
                ka[p][0] = kload(kb4, (0 * 8 + p) * 64 + lane);
                ka[p][1] = kload(kb4, (1 * 8 + p) * 64 + lane);
            }
            uint32_t xa[2][4];
            auto issue = [&](int kk, int b) {
#pragma unroll
                for (int e = 0; e < 4; ++e) xa[b][e] = other_half(dA[4 * kk + e], xaddr);
            };
            issue(0, 0);
#pragma clang loop unroll(full)
            for (int kk = 0; kk < 8; ++kk) {
                if (kk + AKPF < 8) {
                    ka[(kk + AKPF) % (AKPF + 1)][0] = kload(kb4, (0 * 8 + kk + AKPF) * 64 + lane);
                    ka[(kk + AKPF) % (AKPF + 1)][1] = kload(kb4, (1 * 8 + kk + AKPF) * 64 + lane);
                }
                if (kk + 1 < 8) issue(kk + 1, (kk + 1) & 1);
                asm volatile("" ::: "memory");
                const uint4 k0 = ka[kk % (AKPF + 1)][0], k1 = ka[kk % (AKPF + 1)][1];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = 4 * kk + e;
                    const uint32_t P0 = dA[r], P1 = xa[kk & 1][e];
                    const uint32_t c0 = e == 0 ? k0.x : e == 1 ? k0.y : e == 2 ? k0.z : k0.w;
                    const uint32_t c1 = e == 0 ? k1.x : e == 1 ? k1.y : e == 2 ? k1.z : k1.w;
                    // |S| < 2 (6Q) Q + 2Q Q -> |acc| < 14 Q^2 2^-32 + Q/2 < 2Q
                    int64_t S = (int64_t)(int32_t)P0 * (int32_t)c0 + (int64_t)(int32_t)P1 * (int32_t)c1;
                    S += (int64_t)(int32_t)acc[r] * (int32_t)oneRh;
                    acc[r] = smont_red(S, m);
                }
            }
        }
    }
    if (ACCIO) {
        acc_store(acc, g, gate, h, l, T.nR, m);
        return;
    }
    // extraction, identical to GINX
    inv_pass_s<kLmkAcc<LZ>, LZ>(acc, tile, l, T.twA_inv, s_twBi, T.w1R, m.oneR, m);
    wave_lds_sync();
    if (h == 0) {
#pragma unroll
        for (int r = 0; r < 32; ++r) tileW[(r << 5) | l] = acc[r];
    } else if (l == 0) {
        tileW[1024] = acc[0];
    }
    wave_lds_sync();
    uint32_t* oa = ext_a + (size_t)gate * g.N;
#pragma unroll 4
    for (int t = 0; t < 16; ++t) {
        const uint32_t j = (uint32_t)lane + 64u * t;
        const uint32_t c = tileW[j == 0 ? 0 : g.N - j];
        const uint32_t v = (j == 0 || c == 0) ? c : m.Q - c;
        oa[j]            = g.msb_out ? mod_switch(v, m.Q, g.qKS) : v;
    }
    if (lane == 0) {
        const uint32_t bb = add_mod(g.b_const, tileW[1024], m.Q);
        ext_b[gate]       = g.msb_out ? mod_switch(bb, m.Q, g.qKS) : bb;
    }
}

// ---------------------------------------------------------------------------
// Op-list preps, one wave per gate (a thread per gate serialises each gate's ~2000 steps on one
// lane with its scratch in global memory: 2.1 ms for 8192 LMKCDEY gates, 0.42 ms this way).
// ---------------------------------------------------------------------------
namespace {
FHE_DEV uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
FHE_DEV uint32_t lanes_below(uint64_t m, uint32_t lane) {
    return __builtin_popcountll(m & ((1ull << lane) - 1ull));
}
constexpr int kPrepWaves = 4;
}  // namespace

// LMKCDEY: the op schedule described at k_blind_rotate_lmk (rgsw-acc-lmkcdey.cpp:83-157).  Lanes compute the group position of every a_i and
// count them (LDS atomics), a wave scan gives the group starts, a chunked stable placement
// (rank among equal positions of lower lanes) writes every a_i's index straight to its op slot, whose
// offsets the nSkips logic gives in closed form per 64 positions (below).
// NMAX: the largest ring dimension and LWE dimension the LDS arrays hold (1024: the 32-bit sets;
// 2048: N = 2048 and n up to 2048 for the 64-bit accumulator)
template <int NMAX>
__global__ void __launch_bounds__(64 * kPrepWaves)
    k_prep_lmk_w(GateInputs in, GateArgs g, const int16_t* __restrict__ logGen, uint16_t* __restrict__ ops,
                 uint32_t* __restrict__ nops, uint32_t* __restrict__ tvb, uint32_t maxops, uint32_t numAutoKeys) {
    __shared__ uint32_t s_start[kPrepWaves][NMAX + 1];
    __shared__ uint16_t s_fill[kPrepWaves][NMAX];
    __shared__ uint16_t s_bkt[kPrepWaves][NMAX];
    __shared__ uint32_t s_part[kPrepWaves][64];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t gate = blockIdx.x * kPrepWaves + wv;
    if (gate >= g.count) return;  // wave-uniform; no workgroup barrier below
    const uint32_t N = g.N, M = 2 * N, Nh = N / 2, n = g.n, qm = g.ctmod - 1;
    uint32_t* start = s_start[wv];
    uint16_t* fill = s_fill[wv];
    uint16_t* bkt = s_bkt[wv];
    for (uint32_t p = lane; p < N; p += 64) start[p] = 0;
    wave_lds_sync();
    for (uint32_t i = lane; i < n; i += 64) {
        const uint32_t a    = combine(in, in.a, (size_t)gate * n + i, 0, qm, g.xor_double);
        const uint32_t aodd = ((M - a) & (M - 1)) | 1u;  // (0 - a_i) mod 2N, made odd
        const int32_t v     = logGen[aodd];
        const uint32_t p    = v == (int32_t)M ? Nh - 1                          // -1
                            : v < 0 ? Nh - 1 - (uint32_t)(-v)                    // -5^i
                                    : 2 * Nh - 1 - (uint32_t)v;                  // +5^i (v = 0 -> N-1)
        bkt[i] = (uint16_t)p;
        atomicAdd(&start[p], 1u);
    }
    wave_lds_sync();
    // exclusive scan of the N counts: 16 per lane, then across lanes
    const uint32_t per = N / 64;
    uint32_t loc = 0;
    for (uint32_t t = 0; t < per; ++t) loc += start[lane * per + t];
    s_part[wv][lane] = loc;
    wave_lds_sync();
    uint32_t run = 0;
    for (uint32_t j = 0; j < 64; ++j) run += j < lane ? s_part[wv][j] : 0u;
    wave_lds_sync();
    for (uint32_t t = 0; t < per; ++t) {
        const uint32_t c = start[lane * per + t];
        start[lane * per + t] = run;
        run += c;
    }
    if (lane == 0) start[N] = n;
    wave_lds_sync();
    // emission offsets (nSkips logic of rgsw-acc-lmkcdey.cpp:99-157), 64 positions at a time.  The ops
    // follow the group order 0..N-1 with AUTO ops between groups, so group p's items start at
    // start[p] + (AUTO ops before them).  Within a half the skip counter before position t is
    // (t - q) mod numAutoKeys after the last non-empty position q < t (that group leaves it at 1),
    // else (carry + t) mod numAutoKeys; a position emits at most a pre-group AUTO and a capping AUTO,
    // so two ballots give every lane its AUTO count below.
    uint16_t* o = ops + (size_t)gate * maxops;
    const uint32_t cap = numAutoKeys;
    uint32_t A = 0;  // AUTO ops emitted so far (wave-uniform)
    for (uint32_t half = 0; half < 2; ++half) {
        const uint32_t base = half ? Nh : 0u;
        uint32_t nS = 0;  // skip counter entering the chunk
        for (uint32_t tb = 0; tb < Nh - 1; tb += 64) {
            const uint32_t t = tb + lane, p = base + t;
            const bool ok = t < Nh - 1;
            const uint32_t s = ok ? start[p] : 0u, e = ok ? start[p + 1] : 0u;
            const bool ne = ok && e > s;
            const uint64_t lowm = (1ull << lane) - 1ull;
            const uint64_t mb = ballot(ne) & lowm;
            const uint32_t nsb = mb ? (lane - (63u - (uint32_t)__builtin_clzll(mb))) % cap : (nS + lane) % cap;
            const bool pre = ne && nsb != 0;
            const uint32_t aft = ne ? 1u : nsb + 1u;
            const bool capE = ok && (aft == cap || t == Nh - 2);  // t = Nh - 2: i == 1
            const uint64_t bp = ballot(pre), bc = ballot(capE);
            const uint32_t ab = A + __builtin_popcountll(bp & lowm) + __builtin_popcountll(bc & lowm);
            if (pre) o[s + ab] = (uint16_t)(0x8000u | nsb);
            if (ok) fill[p] = (uint16_t)(s + ab + (pre ? 1u : 0u));
            if (capE) o[e + ab + (pre ? 1u : 0u)] = (uint16_t)(0x8000u | aft);
            A += __builtin_popcountll(bp) + __builtin_popcountll(bc);
            const uint32_t cnt = (Nh - 1 - tb) < 64 ? Nh - 1 - tb : 64;
            nS = __builtin_amdgcn_readlane(capE ? 0u : aft, cnt - 1);
        }
        if (half == 0) {
            if (lane == 0) {
                fill[Nh - 1] = (uint16_t)(start[Nh - 1] + A);  // -1
                o[start[Nh] + A] = (uint16_t)0x8000u;          // automorphism by 2N - 5 with key 0
            }
            ++A;
        } else if (lane == 0) {
            fill[N - 1] = (uint16_t)(start[N - 1] + A);       // 0
        }
    }
    wave_lds_sync();
    // stable placement, 64 items at a time (increasing i within a group), straight into the op list
    for (uint32_t c = 0; c < n; c += 64) {
        const uint32_t i = c + lane;
        const bool valid = i < n;
        const uint32_t b = valid ? bkt[i] : 0xffffu;
        uint32_t rank = 0;
        bool last = true;
        const uint32_t m = n - c < 64 ? n - c : 64;
        for (uint32_t j = 0; j < m; ++j) {
            const uint32_t bj = bkt[c + j];
            rank += (bj == b && j < lane) ? 1u : 0u;
            last = last && !(bj == b && j > lane);
        }
        const uint32_t pos = valid ? fill[b] + rank : 0u;
        wave_lds_sync();
        if (valid) {
            o[pos] = (uint16_t)i;
            if (last) fill[b] = (uint16_t)(pos + 1);
        }
        wave_lds_sync();
    }
    const uint32_t k = n + A;
    if (lane == 0) {
        nops[gate] = k;
        tvb[gate]  = combine(in, in.b, gate, in.boff, qm, g.xor_double);
    }
}

// AP / DM: ops in (i, digit) order; per 64-item chunk each lane emits its 0..digitsR nonzero
// digits at the count of lower lanes' ops (ballots per digit slot)
__global__ void __launch_bounds__(64 * kPrepWaves)
    k_prep_dm_w(GateInputs in, GateArgs g, uint16_t* __restrict__ ops, uint32_t* __restrict__ nops,
                uint32_t* __restrict__ tvb, uint32_t maxops, uint32_t baseR, uint32_t digitsR) {
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t gate = blockIdx.x * kPrepWaves + wv;
    if (gate >= g.count) return;
    const uint32_t qm = g.q - 1, n = g.n;
    uint16_t* o = ops + (size_t)gate * maxops;
    uint32_t k = 0;
    for (uint32_t c = 0; c < n; c += 64) {
        const uint32_t i = c + lane;
        const uint32_t a = i < n ? (g.q - combine(in, in.a, (size_t)gate * n + i, 0, qm, g.xor_double)) & qm : 0u;
        uint32_t cnt = 0, aI = a;
        for (uint32_t d = 0; d < digitsR; ++d, aI /= baseR) cnt += (aI % baseR) ? 1u : 0u;
        uint32_t below = 0, total = 0;
        for (uint32_t t = 0; t < digitsR; ++t) {
            const uint64_t m = ballot(cnt > t);
            below += lanes_below(m, lane);
            total += __builtin_popcountll(m);
        }
        uint32_t w = k + below;
        aI = a;
        for (uint32_t d = 0; d < digitsR; ++d, aI /= baseR) {
            const uint32_t a0 = aI % baseR;
            if (a0) o[w++] = (uint16_t)((i * baseR + a0) * digitsR + d);
        }
        k += total;
    }
    if (lane == 0) {
        nops[gate] = k;
        tvb[gate]  = combine(in, in.b, gate, in.boff, qm, g.xor_double);
    }
}

hipError_t launch_prep_lmk(const GateArgs& g, const GateInputs& in, const int16_t* logGen,
                           uint16_t* ops, uint32_t* nops, uint32_t* tvb, uint32_t maxops, uint32_t numAutoKeys,
                           hipStream_t s) {
    if (g.count == 0) return hipSuccess;
    if (in.k < 1 || in.k > 4 || numAutoKeys == 0) return hipErrorInvalidValue;
    if (g.n > 2048 || (g.N != 512 && g.N != 1024 && g.N != 2048)) return hipErrorInvalidValue;  // LDS sizes
    if (g.n <= 1024 && g.N <= 1024)
        hipLaunchKernelGGL(k_prep_lmk_w<1024>, dim3((g.count + kPrepWaves - 1) / kPrepWaves), dim3(64 * kPrepWaves), 0,
                           s, in, g, logGen, ops, nops, tvb, maxops, numAutoKeys);
    else
        hipLaunchKernelGGL(k_prep_lmk_w<2048>, dim3((g.count + kPrepWaves - 1) / kPrepWaves), dim3(64 * kPrepWaves), 0,
                           s, in, g, logGen, ops, nops, tvb, maxops, numAutoKeys);
    return hipGetLastError();
}

hipError_t launch_blind_rotate_lmk(const GateArgs& g, const BootTables& t, const void* bsk, const void* autok,
                                   const uint16_t* ops, const uint32_t* nops, uint32_t maxops, const uint32_t* tvb,
                                   uint32_t* ext_a, uint32_t* ext_b, bool dm, hipStream_t s) {
    if (g.count == 0) return hipSuccess;
    const uint32_t blocks = (g.count + kWaves - 1) / kWaves;
    const size_t lds      = (size_t)(992 * 2 + kWaves * 2 * kTile + (!dm ? 1024 : 0)) * 4;
    const uint2* k  = reinterpret_cast<const uint2*>(bsk);
    const uint2* ak = reinterpret_cast<const uint2*>(autok);
    const bool lz   = t.Q < (1u << 27);
    if (t.Q >= (1u << 28)) return hipErrorInvalidValue;  // signed residue bounds
#define FHE_LAUNCH_LMK(DM_, LZ_, IO)                                                                          \
    hipLaunchKernelGGL((k_blind_rotate_lmk<DM_, LZ_, IO>), dim3(blocks), dim3(256), lds, s, g, t, k, ak, ops, nops, \
                       maxops, tvb, ext_a, ext_b)
    if (g.acc_io) {
        if (dm) { if (lz) FHE_LAUNCH_LMK(true, true, true); else FHE_LAUNCH_LMK(true, false, true); }
        else { if (lz) FHE_LAUNCH_LMK(false, true, true); else FHE_LAUNCH_LMK(false, false, true); }
    } else if (dm) {
        if (lz) FHE_LAUNCH_LMK(true, true, false); else FHE_LAUNCH_LMK(true, false, false);
    } else {
        if (lz) FHE_LAUNCH_LMK(false, true, false); else FHE_LAUNCH_LMK(false, false, false);
    }
#undef FHE_LAUNCH_LMK
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// AP/DM prep (rgsw-acc-dm.cpp:62-77): one thread per gate writes its op list
// ---------------------------------------------------------------------------
hipError_t launch_prep_dm(const GateArgs& g, const GateInputs& in, uint16_t* ops, uint32_t* nops, uint32_t* tvb,
                          uint32_t maxops, uint32_t baseR, uint32_t digitsR, hipStream_t s) {
    if (g.count == 0) return hipSuccess;
    if (in.k < 1 || in.k > 4 || (size_t)g.n * digitsR > maxops || (size_t)g.n * baseR * digitsR > 0x8000u)
        return hipErrorInvalidValue;
    if (digitsR > 8) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_prep_dm_w, dim3((g.count + kPrepWaves - 1) / kPrepWaves), dim3(64 * kPrepWaves), 0, s, in, g,
                       ops, nops, tvb, maxops, baseR, digitsR);
    return hipGetLastError();
}

// ===========================================================================
// GINX with two waves per gate: k_blind_rotate_ginx2<ND, OutT>
// ===========================================================================
// Wave c of a gate owns RLWE component c: 1024 values as 16 registers x 64 lanes, in the layouts of
// ntt.hip k_ntt1024w (x = coefficient or EVAL slot):
//   A (COEF): lane = x5..x0, register = x9..x6;   C (EVAL): lane = x7..x2, register = (x9x8) << 2 | x1x0.
// Per index (AddToAccCGGI, rgsw-acc-cggi.cpp:102-151), wave c: inverse NTT of acc_c (C -> B -> A,
// inv_wave_s), SignedDigitDecompose into its ND retained digits D_c, D_{2+c}, .. (rgsw-acc.cpp:54-91:
// digitsG - 1 of them, the lowest one dropped), all forward-transformed at once (A -> B -> C) and
// written to this wave's LDS region; one workgroup barrier; then per slot the MAC with its own ND
// digits and the partner wave's ND (read from the partner's region), the keys of component c, and the
// monomials: acc_c <- acc_c + S+ (w^a - 1) + S- (w^-a - 1), one signed Montgomery reduction per slot,
// as in k_blind_rotate_ginx.  Half the registers of the one-wave kernel per wave, twice the waves.
//   ND = 2 (digitsG = 3: STD128, MEDIUM ...): pinned by FHE_HIP_GINX_KERNEL=split (the one-wave kernel
//          is faster at every batch size, DESIGN K1), u32 ctExt for the 32-bit key switch;
//   ND = 3 (digitsG = 4 at N = 1024, Q < 2^27: STD128_3, STD128Q, and with q = 2N STD128_4, LPF_STD128,
//          LPF_STD128Q): the one-wave layout would need 96
//          digit registers per lane, so these sets ran on the 64-bit accumulator (bootstrap_wide.hip);
//          this instantiation runs them in 32-bit residues and writes the u64 ctExt of that path's
//          workspace, which its key switch (keyswitch_wide) reads unchanged.
// Bounds (Q < 2^27): signed digits |d| <= 2^(g-1) grow to < 10 Q + 2^(g-1) through the forward NTT;
// |S+-| < 2 ND (10 Q + 2^(g-1)) Q < 2^60; S < 2 (2^32 Q + 2 ND 0.32 Q^2) + 2.8 Q^2, so the reduced
// acc stays below 2.8 Q (kAccBoundLZ) for ND <= 3.
namespace {
#ifndef FHE_G2_GATES
#define FHE_G2_GATES 2
#endif
constexpr int kG2Gates = FHE_G2_GATES;  // gates per workgroup (2 waves each)
constexpr int kG2Tile  = 1088;  // one tile (1024 + 64 pad, wt64 addressing)
// words per wave: ND transpose tiles, which also hold the ND digit polynomials of the exchange
constexpr int g2_region(int nd) { return nd * kG2Tile; }
constexpr size_t g2_lds(int nd) { return (size_t)(1024 + 1024 + 2 * kMonoHalfWords + 2 * kG2Gates * g2_region(nd)) * 4; }

// key layout: boot.h g2_key_word / g2_row

// signed forward NTT of NP polynomials, layout A (|v| < B) -> C (|v| < B + 10 Q); polynomial p
// goes through the tile t + p kG2Tile, or with NT = 1 all of them through the one tile t in turn
// t1 (optional): the tiles of polynomials 1.. at t1, t1 + kG2Tile, .. instead of after t
template <int NP, int NT = NP>
FHE_DEV void fwd_wave_s(uint32_t (&v)[NP][16], uint32_t* t, int L, const uint32_t* __restrict__ twA,
                        const uint32_t* s_tab, const Mod& m, uint32_t* t1 = nullptr) {
    static_assert(NT == NP || NT == 1, "one tile per polynomial, or one tile for all");
    const int G = L >> 2, jj = L & 3;
    auto tp = [&](int p) { return p == 0 ? t : t1 ? t1 + (p - 1) * kG2Tile : t + p * kG2Tile; };
#pragma unroll
    for (int b = 9; b >= 6; --b) {
        const int rb = b - 6;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (r & (1 << rb)) continue;
            const uint32_t w = twA[(1 << (9 - b)) + (r >> (rb + 1))];
#pragma unroll
            for (int p = 0; p < NP; ++p) ct_bf_s(v[p][r], v[p][r | (1 << rb)], w, m);
        }
    }
    if (NT == 1 && NP > 1) {  // both transposes polynomial by polynomial through the one tile
#pragma unroll
        for (int p = 0; p < NP; ++p) {
#pragma unroll
            for (int r = 0; r < 16; ++r) t[wt64((r << 6) | L)] = v[p][r];
            wave_lds_sync();
#pragma unroll
            for (int r = 0; r < 16; ++r) v[p][r] = t[wt64((G << 6) | (r << 2) | jj)];
            wave_lds_sync();
        }
#pragma unroll
        for (int b = 5; b >= 2; --b) {
            const int rb = b - 2;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                if (r & (1 << rb)) continue;
                const uint32_t w = s_tab[(1 << (9 - b)) + (G << (5 - b)) + (r >> (rb + 1))];
#pragma unroll
                for (int p = 0; p < NP; ++p) ct_bf_s(v[p][r], v[p][r | (1 << rb)], w, m);
            }
        }
#pragma unroll
        for (int p = 0; p < NP; ++p) {
#pragma unroll
            for (int r = 0; r < 16; ++r) t[wt64((G << 6) | (r << 2) | jj)] = v[p][r];
            wave_lds_sync();
#pragma unroll
            for (int hh = 0; hh < 4; ++hh) {
                const uint4 q = *reinterpret_cast<const uint4*>(t + wt64((hh << 8) | (L << 2)));
                v[p][4 * hh] = q.x; v[p][4 * hh + 1] = q.y; v[p][4 * hh + 2] = q.z; v[p][4 * hh + 3] = q.w;
            }
            wave_lds_sync();
        }
#pragma unroll
        for (int hh = 0; hh < 4; ++hh) {
            const uint32_t w1 = s_tab[256 + (hh << 6) + L];
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                ct_bf_s(v[p][4 * hh], v[p][4 * hh + 2], w1, m);
                ct_bf_s(v[p][4 * hh + 1], v[p][4 * hh + 3], w1, m);
            }
            const uint2 w0 = *reinterpret_cast<const uint2*>(s_tab + 512 + (hh << 7) + (L << 1));
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                ct_bf_s(v[p][4 * hh], v[p][4 * hh + 1], w0.x, m);
                ct_bf_s(v[p][4 * hh + 2], v[p][4 * hh + 3], w0.y, m);
            }
        }
        return;
    }
    // A -> B
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
        for (int p = 0; p < NP; ++p) tp(p)[wt64((r << 6) | L)] = v[p][r];
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
        for (int p = 0; p < NP; ++p) v[p][r] = tp(p)[wt64((G << 6) | (r << 2) | jj)];
#pragma unroll
    for (int b = 5; b >= 2; --b) {
        const int rb = b - 2;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (r & (1 << rb)) continue;
            const uint32_t w = s_tab[(1 << (9 - b)) + (G << (5 - b)) + (r >> (rb + 1))];
#pragma unroll
            for (int p = 0; p < NP; ++p) ct_bf_s(v[p][r], v[p][r | (1 << rb)], w, m);
        }
    }
    // B -> C
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
        for (int p = 0; p < NP; ++p) tp(p)[wt64((G << 6) | (r << 2) | jj)] = v[p][r];
    wave_lds_sync();
#pragma unroll
    for (int hh = 0; hh < 4; ++hh)
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            const uint4 q = *reinterpret_cast<const uint4*>(tp(p) + wt64((hh << 8) | (L << 2)));
            v[p][4 * hh] = q.x; v[p][4 * hh + 1] = q.y; v[p][4 * hh + 2] = q.z; v[p][4 * hh + 3] = q.w;
        }
    wave_lds_sync();
#pragma unroll
    for (int hh = 0; hh < 4; ++hh) {
        const uint32_t w1 = s_tab[256 + (hh << 6) + L];
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            ct_bf_s(v[p][4 * hh], v[p][4 * hh + 2], w1, m);
            ct_bf_s(v[p][4 * hh + 1], v[p][4 * hh + 3], w1, m);
        }
        const uint2 w0 = *reinterpret_cast<const uint2*>(s_tab + 512 + (hh << 7) + (L << 1));
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            ct_bf_s(v[p][4 * hh], v[p][4 * hh + 1], w0.x, m);
            ct_bf_s(v[p][4 * hh + 2], v[p][4 * hh + 3], w0.y, m);
        }
    }
}

// SignedDigitDecompose (rgsw-acc.cpp:54-91) for digitsG = ND + 1, as decompose2 with SG: the
// balanced digits 1..ND of the centred value d are the signed bit fields j g of (d + C) ^ M,
// C = 2^(g-1) sum_{j <= ND} 2^(jg), M = 2^(g-1) sum_{1 <= j <= ND} 2^(jg) (needs (ND + 1) g <= 32 and
// C + Q < 2^32; Engine checks both)
struct DecN {
    uint32_t Qh, C, CmQ, g, M;
};
FHE_DEV DecN make_decn(uint32_t Q, uint32_t g, int nd) {
    const uint32_t h = 1u << (g - 1);
    uint32_t C = h, M = 0;
    for (int j = 1; j <= nd; ++j) {
        C += h << (j * g);
        M |= h << (j * g);
    }
    return DecN{Q >> 1, C, C - Q, g, M};
}
// accumulator I/O of the split kernels' seam instantiations: wave c holds component c in layout C, lane L
// register r <-> EVAL slot ((r >> 2) << 8) | (L << 2) | (r & 3); conventions as acc_load / acc_store
FHE_DEV uint32_t slot_c(int L, int r) { return ((uint32_t)(r >> 2) << 8) | ((uint32_t)L << 2) | (uint32_t)(r & 3); }
FHE_DEV void acc_load_c(uint32_t (&acc)[16], const GateArgs& g, uint32_t gate, int c, int L, uint32_t ninvR,
                        const Mod& m) {
    const uint64_t* src = g.acc_io + ((size_t)gate * 2 + c) * g.N;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = csub(mont_mul((uint32_t)src[slot_c(L, r)], ninvR, m), m.Q);
}
FHE_DEV void acc_store_c(const uint32_t (&acc)[16], const GateArgs& g, uint32_t gate, int c, int L, uint32_t nR,
                         const Mod& m) {
    uint64_t* dst = g.acc_io + ((size_t)gate * 2 + c) * g.N;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int32_t v = (int32_t)smont_mul(acc[r], nR, m);
        dst[slot_c(L, r)] = (uint64_t)(uint32_t)(v < 0 ? v + (int32_t)m.Q : v);
    }
}

template <int ND, int R>
FHE_DEV void decompose_n(uint32_t x, const DecN& c, uint32_t (&d)[ND][R], int r) {
    const uint32_t u = x >= c.Qh ? x + c.CmQ : x + c.C;  // d + C, d = x or x - Q
    const int32_t w  = (int32_t)(u ^ c.M);
#pragma unroll
    for (int j = 0; j < ND; ++j) d[j][r] = (uint32_t)__builtin_amdgcn_sbfe(w, (j + 1) * c.g, c.g);
}
}  // namespace

// MF: ciphertext modulus 2N (q = 2N sets: STD128_4, LPF_STD128, LPF_STD128Q): any exponent, the
// full-resolution table psi^e - 1 restricted to e in [0, 2N] (the same LDS footprint as the half table)
// ACCIO: the Backend::BlindRotate seam (GateArgs::acc_io), as in k_blind_rotate_ginx
template <int ND, bool MF, typename OutT, bool ACCIO = false>
__global__ void __launch_bounds__(128 * kG2Gates, 2)
    k_blind_rotate_ginx2(GateArgs g, BootTables T, const uint4* __restrict__ bsk2, const uint16_t* __restrict__ idx,
                         const uint32_t* __restrict__ tvb, OutT* __restrict__ ext_a, OutT* __restrict__ ext_b,
                         const uint32_t* __restrict__ twAf) {
    constexpr int kReg = g2_region(ND);
    constexpr int kRows = 2 * ND;  // digit rows per slot: own ND, partner ND
    extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
    uint32_t* s_tab  = sm;
    uint32_t* s_tabI = sm + 1024;
    uint2* s_mono2   = reinterpret_cast<uint2*>(sm + 2048);
    uint32_t* s_reg  = sm + 2048 + 2 * kMonoHalfWords;
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) {
        s_tab[i]  = T.tabF[i];
        s_tabI[i] = T.tabI[i];
    }
    for (int i = threadIdx.x; i < kMonoHalfWords; i += blockDim.x)
        s_mono2[i] = MF ? make_uint2(T.monoP_full[i], T.mono_full[i]) : make_uint2(T.monoP[i], T.mono[i]);

    const int wave = threadIdx.x >> 6, L = threadIdx.x & 63;
    const int c = wave & 1;  // RLWE component of this wave
    const uint32_t gslot = blockIdx.x * kG2Gates + (wave >> 1);
    const bool live = gslot < g.count;
    const uint32_t gate = live ? gslot : g.count - 1;   // spare waves shadow the last gate: every wave meets every barrier
    uint32_t* region  = s_reg + wave * kReg;
    uint32_t* partner = s_reg + (wave ^ 1) * kReg;
    uint32_t* t0 = region;
    const Mod m0 = make_mod(T);
    const Mod& m = m0;
    __syncthreads();

    // initial accumulator (BootstrapGateCore, binfhe-base-scheme.cpp:556-575): acc1 = NTT(m), acc0 = 0
    uint32_t acc[16];
    if (ACCIO && !g.acc_tv) {
        acc_load_c(acc, g, gate, c, L, T.ninvR, m);
    } else if (c == 1) {
        const uint32_t b = tvb[gate], cm = g.ctmod - 1;
        uint32_t tv[1][16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t x = ((uint32_t)r << 6) | (uint32_t)L;
            uint32_t v = 0;
            if (x % g.factor == 0) {
                const uint32_t bx = (b - x / g.factor) & cm;
                v = (bx >= g.lb && bx < g.ub) ? g.lv : g.uv;
            }
            tv[0][r] = v;
        }
        fwd_wave_s<1>(tv, t0, L, twAf, s_tab, m);
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = smont_mul(tv[0][r], T.ninvR, m);   // (-Q, Q), N^-1 scaled
    } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0;
    }

    const uint16_t* gidx = idx + (size_t)gate * g.n;
    const DecN dec = make_decn(m.Q, g.gbits, ND);
    // monomial index of slot x(L, r): f = a' (2 brv10(x) + 1) mod 2N in half-table units, split as a
    // per-lane part a' (8 brv6(L) + 1) and a per-register part a' (512 brv2(r & 3) + 2 brv2(r >> 2))
    const uint32_t lmul = 8 * (__builtin_bitreverse32((uint32_t)L) >> 26) + 1;
    const uint4* kc = bsk2 + (size_t)c * (kRows * 8 * 64) + L;
    for (uint32_t i = 0; i < g.n; ++i) {
        const Mod m = fresh_nq(m0);
        const uint32_t a  = __builtin_amdgcn_readfirstlane((uint32_t)gidx[i]);
        const uint32_t as = MF ? a : a >> 1;                // even exponents (ctmod = q < 2N) unless MF
        const uint4* kb   = kc + (size_t)i * (2 * kRows * 8 * 64);
        uint4 kq[2][kRows];
#pragma unroll
        for (int p = 0; p < kRows; ++p) kq[0][p] = kb[(p * 8 + 0) * 64];
        __syncthreads();   // the partner wave has read this wave's digits of the previous index
        uint32_t d[ND][16];
#pragma unroll
        for (int r = 0; r < 16; ++r) d[0][r] = acc[r];
        inv_wave_s<kAccBoundLZ, true>(d[0], t0, L, s_tabI, T.w1R, m.oneR, m);
#pragma unroll
        for (int r = 0; r < 16; ++r) decompose_n<ND>(d[0][r], dec, d, r);
        fwd_wave_s<ND>(d, t0, L, twAf, s_tab, m);
        wave_lds_sync();
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int j = 0; j < ND; ++j) region[j * 1024 + ((r << 6) | L)] = d[j][r];
        __syncthreads();   // both waves' digits are in LDS
        // MF: e = a (2 brv10(x) + 1) mod 2N = (el + ue) mod 2N, per-lane el and per-register ue
        const uint32_t fl = (as * lmul) & (MF ? 2047u : 1023u);
#pragma unroll
        for (int k2 = 0; k2 < 8; ++k2) {
            if (k2 + 1 < 8) {
#pragma unroll
                for (int p = 0; p < kRows; ++p) kq[(k2 + 1) & 1][p] = kb[(p * 8 + k2 + 1) * 64];
            }
            asm volatile("" ::: "memory");
            // registers r = 2 k2, 2 k2 + 1 differ in x bit 0: the same monomial (even exponents)
            const int r0 = 2 * k2;
            const uint32_t ur = __builtin_amdgcn_readfirstlane(
                (as * (512u * (__builtin_bitreverse32((uint32_t)(r0 & 3)) >> 30) +
                       2u * (__builtin_bitreverse32((uint32_t)(r0 >> 2)) >> 30))) & 1023u);
            const uint32_t f  = fl + ur;                  // < 2N
            const uint32_t fn = 2048u - f;                // -a: 2N - f
            uint2 mp, mn;
            if (!MF) {
                mp = s_mono2[f + (f >> 5)];
                mn = s_mono2[fn + (fn >> 5)];
            }
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int r = r0 + e;
                if (MF) {  // x bit 0 adds 1024 a to the exponent: registers r0, r0 + 1 differ for odd a
                    const uint32_t ue = __builtin_amdgcn_readfirstlane(
                        (as * (512u * (__builtin_bitreverse32((uint32_t)(r & 3)) >> 30) +
                               2u * (__builtin_bitreverse32((uint32_t)(r >> 2)) >> 30))) & 2047u);
                    const uint32_t ef = (fl + ue) & 2047u, en = 2048u - ef;
                    mp = s_mono2[ef + (ef >> 5)];
                    mn = s_mono2[en + (en >> 5)];
                }
                uint32_t pd[ND];
#pragma unroll
                for (int j = 0; j < ND; ++j) pd[j] = partner[j * 1024 + ((r << 6) | L)];
                const uint4* q = kq[k2 & 1];
                // digits x keys in row order (own digits, partner digits), unreduced 64-bit sums
                int64_t S1 = 0, S2 = 0;
#pragma unroll
                for (int p = 0; p < kRows; ++p) {
                    const int32_t dv = (int32_t)(p < ND ? d[p][r] : pd[p - ND]);
                    S1 += (int64_t)dv * (int32_t)(e ? q[p].y : q[p].x);
                    S2 += (int64_t)dv * (int32_t)(e ? q[p].w : q[p].z);
                }
                int64_t S = (int64_t)((uint64_t)(uint32_t)S1 * mp.x) + (int64_t)(int32_t)(S1 >> 32) * (int32_t)mp.y;
                S += (int64_t)((uint64_t)(uint32_t)S2 * mn.x) + (int64_t)(int32_t)(S2 >> 32) * (int32_t)mn.y;
                S += (int64_t)(int32_t)acc[r] * (int32_t)T.oneR;
                acc[r] = smont_red(S, m);
            }
        }
    }

    if (ACCIO) {   // every wave of the workgroup leaves here: no barrier is skipped by some only
        if (live) acc_store_c(acc, g, gate, c, L, T.nR, m);
        return;
    }
    // extraction (binfhe-base-scheme.cpp:110-121): canonical COEF in layout A; wave 0 writes the
    // transposed acc0 (coefficient k -> position N - k, negated), wave 1 the b term from acc1[0]
    __syncthreads();   // the partner wave's last MAC has read this wave's region
    inv_wave_s<kAccBoundLZ, true>(acc, t0, L, s_tabI, T.w1R, m.oneR, m);
    if (!live) return;
    if (c == 0) {
        OutT* oa = ext_a + (size_t)gate * g.N;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t x = ((uint32_t)r << 6) | (uint32_t)L;
            const uint32_t v = acc[r];
            const uint32_t o = (x == 0 || v == 0) ? v : m.Q - v;
            oa[(g.N - x) & (g.N - 1)] = (OutT)(g.msb_out ? mod_switch(o, m.Q, g.qKS) : o);
        }
    } else if (L == 0) {
        const uint32_t bb = add_mod(g.b_const, acc[0], m.Q);
        ext_b[gate] = (OutT)(g.msb_out ? mod_switch(bb, m.Q, g.qKS) : bb);
    }
}

// the resident GINX layout (ginx_u4_off, half-swapped rows) -> the k_blind_rotate_ginx2<2> layout
__global__ void k_repack_ginx2(const uint32_t* __restrict__ src, uint32_t n, uint32_t* __restrict__ dst) {
    const uint64_t words = (uint64_t)n * 16384;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < words; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = t >> 14;
        const uint32_t w = (uint32_t)(t & 16383);
        const uint32_t e4 = w & 3, L = (w >> 2) & 63, k2 = (w >> 8) & 7, p = (w >> 11) & 3, c = w >> 13;
        const uint32_t r = 2 * k2 + (e4 & 1), ks = e4 >> 1;
        const uint32_t x = ((r >> 2) << 8) | (L << 2) | (r & 3);          // EVAL slot
        const uint32_t row = g2_row(c, p, 2);
        const uint32_t lane = c * 32 + (x >> 5), kk = (x & 31) >> 1, e = x & 1;
        const uint32_t dpos = kBskHalfSwap ? row ^ c : row;
        dst[t] = src[i * 16384 + ginx_u4_off(ks, dpos, kk, lane, e)];
    }
}

bool ginx2_supported(const GateArgs& g, const BootTables& t) {
    return t.Q < (1u << 27) && g.N == 1024 && g.ctmod < 2 * g.N && g.tv == nullptr && g.acc_io == nullptr;
}

hipError_t launch_repack_ginx2(const void* bsk, uint32_t n, void* bsk2, hipStream_t s) {
    const uint64_t words = (uint64_t)n * 16384;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((words + 255) / 256, 16384);
    hipLaunchKernelGGL(k_repack_ginx2, dim3(blocks), dim3(256), 0, s, static_cast<const uint32_t*>(bsk), n,
                       static_cast<uint32_t*>(bsk2));
    return hipGetLastError();
}

hipError_t launch_blind_rotate_ginx2(const GateArgs& g, const BootTables& t, const void* bsk2, const uint16_t* idx,
                                     const uint32_t* tvb, uint32_t* ext_a, uint32_t* ext_b, hipStream_t s) {
    if (g.count == 0) return hipSuccess;
    if (!ginx2_supported(g, t)) return hipErrorInvalidValue;
    const uint32_t blocks = (g.count + kG2Gates - 1) / kG2Gates;
    hipLaunchKernelGGL((k_blind_rotate_ginx2<2, false, uint32_t>), dim3(blocks), dim3(128 * kG2Gates), g2_lds(2), s, g, t,
                       static_cast<const uint4*>(bsk2), idx, tvb, ext_a, ext_b, t.twA_fwd);
    return hipGetLastError();
}

bool ginx3_supported(const GateArgs& g, const BootTables& t) {
    return t.Q < (1u << 27) && g.N == 1024 && g.ctmod <= 2 * g.N && g.tv == nullptr && g.tv64 == nullptr &&
           g.gbits >= 2 && 4 * g.gbits <= 32 && g.qKS <= 65536;
}

hipError_t launch_blind_rotate_ginx3(const GateArgs& g, const BootTables& t, const void* bsk3, const uint16_t* idx,
                                     const uint32_t* tvb, uint64_t* ext_a, uint64_t* ext_b, hipStream_t s) {
    if (g.count == 0) return hipSuccess;
    if (!ginx3_supported(g, t)) return hipErrorInvalidValue;
    static const bool attr = [] {
        for (const void* k : {reinterpret_cast<const void*>(&k_blind_rotate_ginx2<3, false, uint64_t>),
                              reinterpret_cast<const void*>(&k_blind_rotate_ginx2<3, true, uint64_t>),
                              reinterpret_cast<const void*>(&k_blind_rotate_ginx2<3, false, uint64_t, true>),
                              reinterpret_cast<const void*>(&k_blind_rotate_ginx2<3, true, uint64_t, true>)})
            (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)g2_lds(3));
        return true;
    }();
    (void)attr;
    const uint32_t blocks = (g.count + kG2Gates - 1) / kG2Gates;
#define FHE_LAUNCH_G3(MF, IO)                                                                                    \
    hipLaunchKernelGGL((k_blind_rotate_ginx2<3, MF, uint64_t, IO>), dim3(blocks), dim3(128 * kG2Gates), g2_lds(3), s, \
                       g, t, static_cast<const uint4*>(bsk3), idx, tvb, ext_a, ext_b, t.twA_fwd)
    const bool mf = g.ctmod == 2 * g.N;
    if (g.acc_io) { if (mf) FHE_LAUNCH_G3(true, true); else FHE_LAUNCH_G3(false, true); }
    else if (mf) FHE_LAUNCH_G3(true, false);
    else FHE_LAUNCH_G3(false, false);
#undef FHE_LAUNCH_G3
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K1x: GINX at N = 1024 with two waves per gate and K1w's exchange (k_blind_rotate_ginx2x), the
// small-batch kernel: at 1024 STD128 gates (config 3) the one-wave kernel K1 has one wave per SIMD,
// which issues VALU in 68% of its cycles.  Wave c owns component c in layout C (16 registers x 64 lanes,
// as K1s).  Per index (AddToAccCGGI, rgsw-acc-cggi.cpp:102-151): inverse NTT of acc_c, SignedDigitDecompose
// into its 2 retained digits (rgsw-acc.cpp:54-91; digit rows c and 2 + c), forward NTT of both; then per
// slot its OWN digits times the key columns of BOTH components: the sum for component c, with the
// monomials and acc_c folded in, is reduced into acc_c; the other one is reduced to one word per slot and
// written to this wave's exchange buffer (i & 1); one workgroup barrier; the partner's word is added.  The
// transpose tile is private to the wave and the exchange buffers alternate, so one barrier per index
// suffices (K1s exchanges the digit polynomials: two barriers per index and the partner's digits read
// inside the MAC).  acc_c <- acc_c + S+_c (X^a - 1) + S-_c (X^-a - 1) as in K1; only the order of the
// modular additions differs, so the outputs are the same.
// Keys (launch_repack_ginx2x from the resident layout), per index i and wave c: [c][q < 4][k2 < 8][64][4]
// = (K+[r], K+[r+1], K-[r], K-[r+1]), r = 2 k2, slot x(L, r) of layout C; q = 2 j + o: digit row 2 j + c,
// column c (o = 0) or 1 - c (o = 1).
// Bounds (Q < 2^27): |D| < 10 Q + 2^(g-1) after the forward NTT; |S+-| < 2 (10 Q + 2^9) Q < 21 Q^2, so
// |hi(S)| < 0.66 Q; the own word is below 2 Q + 0.04 Q + A Q / 2^32 + Q / 2 < 2.54 Q + A / 32, the
// partner's below 2.54 Q: A < 5.3 Q between indices (the inverse plan's BIN, as K1w's kW2AccBound).
// ---------------------------------------------------------------------------
namespace {
#ifndef FHE_X_GATES
#define FHE_X_GATES 2   // gates per workgroup (two waves each)
#endif
#ifndef FHE_X_TILES
#define FHE_X_TILES 2   // transpose tiles of the forward NTT: 1 (the two digit polynomials in turn) or 2
#endif
#ifndef FHE_X_ABL
#define FHE_X_ABL 0     // timing-only ablations (wrong results): 1 no barrier, 2 no key loads
#endif
#if FHE_X_ABL == 2
#define XKEY(p, o) make_uint4((uint32_t)(o), (uint32_t)(o) ^ 5u, (uint32_t)(o) + 3u, (uint32_t)(size_t)(p))
#else
#define XKEY(p, o) (p)[o]
#endif
#ifndef FHE_X_MPF
#define FHE_X_MPF 0     // 1: the MAC's monomial pairs requested one slot pair ahead (measured slower,
                        // profiles/r06_lmk_attr.txt: 2.84 / 2.83 vs 2.74 / 2.71 ms at 512 gates)
#endif
#ifndef FHE_X_PRIO
#define FHE_X_PRIO 0    // A/B: waves of odd workgroup slots on a CU at priority 1
#endif
#ifndef FHE_X_STAGGER
#define FHE_X_STAGGER 0 // A/B: odd workgroup slots start FHE_X_STAGGER x 8128 cycles late (phase offset)
#endif
constexpr int kXGates = FHE_X_GATES;
constexpr int kXTiles = FHE_X_TILES;
// words per wave: a transpose tile and two exchange buffers (padded to tiles: with kXTiles = 2 the exchange
// buffer of index i is the forward transform's second tile before it takes the partner's words, see below)
constexpr int kXWave  = 3 * kG2Tile;
constexpr int kXAcc   = 53;                            // |acc| < 5.3 Q between indices (units of Q/10)
constexpr size_t x_lds(int gw = kXGates) { return (size_t)(1024 + 1024 + 2 * kMonoHalfWords + 2 * gw * kXWave) * 4; }
static_assert(x_lds() <= 160 * 1024, "LDS per workgroup");
static_assert(kXTiles == 1 || kXTiles == 2, "transpose tiles");
}  // namespace

// MF: ciphertext modulus 2N (BootstrapFunc of EvalFunc's arbitrary functions, seam calls at 2N): any exponent, the
// full-resolution table psi^e - 1 restricted to e in [0, 2N] (as K1s); ACCIO: the Backend::BlindRotate seam
// (GateArgs::acc_io), as K1 / K1s.  Test-vector tables (g.tv, BootstrapFuncCore) are read as K1 reads them.
// GW: gates per workgroup (kXGates; 1 for batches of up to one gate per CU, so that each gate has a CU to itself:
// with two per workgroup a lone gate shares its CU with the spare waves that shadow it)
template <bool MF, bool ACCIO, int GW = kXGates>
#ifndef FHE_X_LB
#define FHE_X_LB 0  // A/B: 1 = the launch bounds' minimum-blocks form for GW > 1 (round-6 first build)
#endif
#if FHE_X_LB
__global__ void __launch_bounds__(128 * GW, GW >= 4 ? 1 : 2)
#else
__global__ void __launch_bounds__(128 * GW) __attribute__((amdgpu_waves_per_eu(GW >= 4 ? 1 : 2, GW >= 4 ? 1 : 2)))
#endif
    k_blind_rotate_ginx2x(GateArgs g, BootTables T, const uint4* __restrict__ keys, const uint16_t* __restrict__ idx,
                          const uint32_t* __restrict__ tvb, uint32_t* __restrict__ ext_a, uint32_t* __restrict__ ext_b,
                          const uint32_t* __restrict__ twAf) {
    constexpr int ND = 2, kQ = 2 * ND;  // key vectors per slot pair: 2 digit rows x 2 columns
    extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
    uint32_t* s_tab  = sm;
    uint32_t* s_tabI = sm + 1024;
    uint2* s_mono2   = reinterpret_cast<uint2*>(sm + 2048);
    uint32_t* s_wave = sm + 2048 + 2 * kMonoHalfWords;
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) {
        s_tab[i]  = T.tabF[i];
        s_tabI[i] = T.tabI[i];
    }
    for (int i = threadIdx.x; i < kMonoHalfWords; i += blockDim.x)
        s_mono2[i] = MF ? make_uint2(T.monoP_full[i], T.mono_full[i]) : make_uint2(T.monoP[i], T.mono[i]);

    const int wave = threadIdx.x >> 6, L = threadIdx.x & 63;
    const int c = wave & 1;  // RLWE component of this wave
    const uint32_t gslot = blockIdx.x * GW + (wave >> 1);
    const bool live = gslot < g.count;
    const uint32_t gate = live ? gslot : g.count - 1;  // spare waves shadow the last gate: every wave meets every barrier
    uint32_t* tile = s_wave + wave * kXWave;
    uint32_t* xown = tile + kG2Tile;                                   // exchange buffers, this wave's ...
    const uint32_t* xpar = s_wave + (wave ^ 1) * kXWave + kG2Tile + L;  // ... and the partner's
    const Mod m0 = make_mod(T);
    const Mod& m = m0;
    __syncthreads();
#if FHE_X_PRIO || FHE_X_STAGGER
    uint32_t hwid;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    const uint32_t tgs = (hwid >> 16) & 15;  // the workgroup's slot on its CU
#endif
#if FHE_X_PRIO
    if (tgs & 1) __builtin_amdgcn_s_setprio(1);
#endif
#if FHE_X_STAGGER
    if (tgs & 1)
        for (int z = 0; z < FHE_X_STAGGER; ++z) __builtin_amdgcn_s_sleep(127);
#endif

    // initial accumulator (BootstrapGateCore, binfhe-base-scheme.cpp:556-575, or BootstrapFuncCore :596-608 from
    // the table g.tv): acc1 = NTT(m), acc0 = 0; the seam's accumulators from g.acc_io
    uint32_t acc[16];
    if (ACCIO && !g.acc_tv) {
        acc_load_c(acc, g, gate, c, L, T.ninvR, m);
    } else if (c == 1) {
        const uint32_t b = tvb[gate], cm = g.ctmod - 1;
        // EvalFuncMultiOutput: table gate % tv_mod (GateArgs::tv_mod)
        const uint32_t tvo = g.tv_mod > 1 ? (gate % g.tv_mod) * g.ctmod : 0u;
        uint32_t tv[1][16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t x = ((uint32_t)r << 6) | (uint32_t)L;
            uint32_t v = 0;
            if (x % g.factor == 0) {
                const uint32_t bx = (b - x / g.factor) & cm;
                v = g.tv ? g.tv[tvo + bx] : (bx >= g.lb && bx < g.ub) ? g.lv : g.uv;
            }
            tv[0][r] = v;
        }
        fwd_wave_s<1>(tv, tile, L, twAf, s_tab, m);
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = smont_mul(tv[0][r], T.ninvR, m);  // (-Q, Q), N^-1 scaled
    } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0;
    }

    const uint16_t* gidx = idx + (size_t)gate * g.n;
    const DecN dec = make_decn(m.Q, g.gbits, ND);
    // monomial index of slot x(L, r) in half-table units, as K1s: a per-lane part as' (8 brv6(L) + 1) and a
    // per-register part as' (512 brv2(r & 3) + 2 brv2(r >> 2)); registers 2 k2 and 2 k2 + 1 share it
    const uint32_t lmul = 8 * (__builtin_bitreverse32((uint32_t)L) >> 26) + 1;
    const uint4* kc = keys + (size_t)c * (kQ * 8 * 64) + L;
    for (uint32_t i = 0; i < g.n; ++i) {
        const Mod m = fresh_nq(m0);
        const uint32_t as = __builtin_amdgcn_readfirstlane((uint32_t)gidx[i]) >> (MF ? 0 : 1);  // even unless MF
        const uint4* kb = kc + (size_t)i * (2 * kQ * 8 * 64);
#if FHE_X_ABL == 2
        asm volatile("" : "+v"(kb));
#endif
        uint4 kq[2][kQ];
#pragma unroll
        for (int q = 0; q < kQ; ++q) kq[0][q] = XKEY(kb, (q * 8 + 0) * 64);
        uint32_t d[ND][16];
#pragma unroll
        for (int r = 0; r < 16; ++r) d[0][r] = acc[r];
        inv_wave_s<kXAcc, true>(d[0], tile, L, s_tabI, T.w1R, m.oneR, m);
#pragma unroll
        for (int r = 0; r < 16; ++r) decompose_n<ND>(d[0][r], dec, d, r);
        // the second digit polynomial's tile: this index's exchange buffer, whose last contents (index i - 2)
        // the partner read before it reached the barrier of index i - 1, which this wave has passed
        uint32_t* xb = xown + (i & 1) * kG2Tile;
        fwd_wave_s<ND, kXTiles>(d, tile, L, twAf, s_tab, m, xb);
        if (kXTiles == 2) wave_lds_sync();  // its last reads done before the partner words overwrite it
        const uint32_t fl = (as * lmul) & (MF ? 2047u : 1023u);
        uint32_t* xo = xb + L;
        // the monomial pair of slot pair k2: psi^(2f) - 1 and psi^(-2f) - 1 (MF: of register r0 = 2 k2,
        // psi^e - 1 and psi^(2N - e) - 1), requested one slot pair ahead of its use when FHE_X_MPF
        auto mono_r = [&](int r0, uint2& mp, uint2& mn) {
            const uint32_t ur = __builtin_amdgcn_readfirstlane(
                (as * (512u * (__builtin_bitreverse32((uint32_t)(r0 & 3)) >> 30) +
                       2u * (__builtin_bitreverse32((uint32_t)(r0 >> 2)) >> 30))) & (MF ? 2047u : 1023u));
            const uint32_t f  = MF ? (fl + ur) & 2047u : fl + ur;  // < 2N
            const uint32_t fn = 2048u - f;                        // -a: 2N - f
            mp = s_mono2[f + (f >> 5)];
            mn = s_mono2[fn + (fn >> 5)];
        };
        auto mono = [&](int k2, uint2& mp, uint2& mn) { mono_r(2 * k2, mp, mn); };
        uint2 mq[2][2];
#if FHE_X_MPF
        mono(0, mq[0][0], mq[0][1]);
#endif
#pragma unroll
        for (int k2 = 0; k2 < 8; ++k2) {
            if (k2 + 1 < 8) {
#pragma unroll
                for (int q = 0; q < kQ; ++q) kq[(k2 + 1) & 1][q] = XKEY(kb, (q * 8 + k2 + 1) * 64);
#if FHE_X_MPF
                mono(k2 + 1, mq[(k2 + 1) & 1][0], mq[(k2 + 1) & 1][1]);
#endif
            }
            asm volatile("" ::: "memory");
            const int r0 = 2 * k2;
#if !FHE_X_MPF
            mono(k2, mq[k2 & 1][0], mq[k2 & 1][1]);
#endif
            uint2 mp = mq[k2 & 1][0], mn = mq[k2 & 1][1];
            const uint4* q4 = kq[k2 & 1];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int r = r0 + e;
                // MF: x bit 0 adds 1024 a to the exponent: registers r0, r0 + 1 differ for odd a
                if (MF && e == 1) mono_r(r, mp, mn);
#pragma unroll
                for (int o = 0; o < 2; ++o) {  // o = 0: this wave's component, 1: the partner's
                    int64_t S1 = 0, S2 = 0;
#pragma unroll
                    for (int j = 0; j < ND; ++j) {
                        const uint4 kv = q4[2 * j + o];
                        S1 += (int64_t)(int32_t)d[j][r] * (int32_t)(e ? kv.y : kv.x);
                        S2 += (int64_t)(int32_t)d[j][r] * (int32_t)(e ? kv.w : kv.z);
                    }
                    int64_t S = (int64_t)((uint64_t)(uint32_t)S1 * mp.x) + (int64_t)(int32_t)(S1 >> 32) * (int32_t)mp.y;
                    S += (int64_t)((uint64_t)(uint32_t)S2 * mn.x) + (int64_t)(int32_t)(S2 >> 32) * (int32_t)mn.y;
                    if (o == 0) {
                        S += (int64_t)(int32_t)acc[r] * (int32_t)T.oneR;
                        acc[r] = smont_red(S, m);
                    } else {
                        xo[r << 6] = smont_red(S, m);
                    }
                }
            }
        }
        // both waves' partner words are in LDS (the buffer i & 1 is written again at index i + 2, after the
        // partner has passed the next barrier, i.e. after it read this one)
#if FHE_X_ABL != 1
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
#endif
        const uint32_t* xp = xpar + (i & 1) * kG2Tile;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] += xp[r << 6];
    }

    if (ACCIO) {  // after the last barrier: every wave of the workgroup leaves here
        if (live) acc_store_c(acc, g, gate, c, L, T.nR, m);
        return;
    }
    // extraction (binfhe-base-scheme.cpp:110-121): canonical COEF in layout A; wave 0 writes the transposed
    // acc0 (coefficient k -> position N - k, negated), wave 1 the b term from acc1[0] (tile private: no barrier)
    inv_wave_s<kXAcc, true>(acc, tile, L, s_tabI, T.w1R, m.oneR, m);
    if (!live) return;
    if (c == 0) {
        uint32_t* oa = ext_a + (size_t)gate * g.N;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t x = ((uint32_t)r << 6) | (uint32_t)L;
            const uint32_t v = acc[r];
            const uint32_t o = (x == 0 || v == 0) ? v : m.Q - v;
            oa[(g.N - x) & (g.N - 1)] = g.msb_out ? mod_switch(o, m.Q, g.qKS) : o;
        }
    } else if (L == 0) {
        const uint32_t bb = add_mod(g.b_const, acc[0], m.Q);
        ext_b[gate] = g.msb_out ? mod_switch(bb, m.Q, g.qKS) : bb;
    }
}

// the resident GINX layout (ginx_u4_off, half-swapped rows) -> the k_blind_rotate_ginx2x layout
__global__ void k_repack_ginx2x(const uint32_t* __restrict__ src, uint32_t n, uint32_t* __restrict__ dst) {
    const uint64_t words = (uint64_t)n * 16384;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < words; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = t >> 14;
        const uint32_t w = (uint32_t)(t & 16383);
        const uint32_t e4 = w & 3, L = (w >> 2) & 63, k2 = (w >> 8) & 7, q = (w >> 11) & 3, c = w >> 13;
        const uint32_t r = 2 * k2 + (e4 & 1), ks = e4 >> 1;
        const uint32_t x = ((r >> 2) << 8) | (L << 2) | (r & 3);  // EVAL slot
        const uint32_t row = 2 * (q >> 1) + c, col = c ^ (q & 1);
        const uint32_t lane = col * 32 + (x >> 5), kk = (x & 31) >> 1, e = x & 1;
        const uint32_t dpos = kBskHalfSwap ? row ^ col : row;
        dst[t] = src[i * 16384 + ginx_u4_off(ks, dpos, kk, lane, e)];
    }
}

hipError_t launch_repack_ginx2x(const void* bsk, uint32_t n, void* bskx, hipStream_t s) {
    const uint64_t words = (uint64_t)n * 16384;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((words + 255) / 256, 16384);
    hipLaunchKernelGGL(k_repack_ginx2x, dim3(blocks), dim3(256), 0, s, static_cast<const uint32_t*>(bsk), n,
                       static_cast<uint32_t*>(bskx));
    return hipGetLastError();
}

bool ginx2x_supported(const GateArgs& g, const BootTables& t) {
    return t.Q < (1u << 27) && g.N == 1024 && g.ctmod <= 2 * g.N && g.tv64 == nullptr && g.gbits >= 2 &&
           3 * g.gbits <= 32;
}

hipError_t launch_blind_rotate_ginx2x(const GateArgs& g, const BootTables& t, const void* bskx, const uint16_t* idx,
                                      const uint32_t* tvb, uint32_t* ext_a, uint32_t* ext_b, int gw, hipStream_t s) {
    if (g.count == 0) return hipSuccess;
    if (!ginx2x_supported(g, t) || gw < 1) return hipErrorInvalidValue;  // gw > 1: kXGates
    static const bool attr = [] {
        for (const void* k : {reinterpret_cast<const void*>(&k_blind_rotate_ginx2x<false, false>),
                              reinterpret_cast<const void*>(&k_blind_rotate_ginx2x<true, false>),
                              reinterpret_cast<const void*>(&k_blind_rotate_ginx2x<false, true>),
                              reinterpret_cast<const void*>(&k_blind_rotate_ginx2x<true, true>)})
            (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)x_lds());
        return true;
    }();
    (void)attr;
#define FHE_LAUNCH_X(MF_, IO, GW_)                                                                                  \
    hipLaunchKernelGGL((k_blind_rotate_ginx2x<MF_, IO, GW_>), dim3((g.count + GW_ - 1) / GW_), dim3(128 * GW_),       \
                       x_lds(GW_), s, g, t, static_cast<const uint4*>(bskx), idx, tvb, ext_a, ext_b, t.twA_fwd)
#define FHE_LAUNCH_X2(MF_, IO) \
    if (gw == 1) FHE_LAUNCH_X(MF_, IO, 1); else FHE_LAUNCH_X(MF_, IO, kXGates)
    const bool mf = g.ctmod == 2 * g.N;
    if (g.acc_io) { if (mf) { FHE_LAUNCH_X2(true, true); } else { FHE_LAUNCH_X2(false, true); } }
    else if (mf) { FHE_LAUNCH_X2(true, false); }
    else { FHE_LAUNCH_X2(false, false); }
#undef FHE_LAUNCH_X2
#undef FHE_LAUNCH_X
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K1q: GINX at N = 1024 with FOUR waves per gate (k_blind_rotate_ginx4x), the latency kernel for batches of up to
// one gate per CU.  Wave (c, j) = wave c + 2 j owns component c (layout C, as K1x) and its retained digit j (row
// 2 j + c).  Per index (AddToAccCGGI, rgsw-acc-cggi.cpp:102-151): the two waves of component c both inverse-
// transform acc_c (the same values in both), wave (c, j) keeps digit j only and forward-transforms that one
// polynomial, then multiplies it by the key columns of both components with the monomials: the word for its
// own component (wave (c, 0) folds acc_c in) and the word for the other one go to its exchange planes; one
// workgroup barrier; acc_c = own word + the sibling's (c, 1 - j) own-component word + both (1 - c, *) waves'
// other-component words.  Both waves of a component add the same four words (in another order), so they hold
// identical accumulators; only the order of the modular additions differs from K1, so the outputs are the same.
// Per wave and index: one inverse and one forward transform and half of K1x's MAC.
// Keys: K1x's layout (launch_repack_ginx2x); wave (c, j) reads q = 2 j + o of [i][c][q < 4][k2 < 8][64][4].
// Bounds (Q < 2^27): |S+-| < (10 Q + 2^9) Q, so each word is below 2^32 Q 2 / 2^32 + 0.02 Q + Q / 2 < 2.52 Q (the
// lo(S) x plain-monomial products dominate), + A / 32 for the word that folds acc in: A < 4 (2.52 Q) / (1 - 1/32)
// < 10.5 Q between indices (the inverse plan's BIN; 16 Q of signed headroom).
// ---------------------------------------------------------------------------
namespace {
#ifndef FHE_Q_X128
#define FHE_Q_X128 1  // the four words of a slot side by side: one ds_read_b128 instead of three b32 reads (0: A/B)
#endif
// words per wave: a transpose tile and [parity][o] exchange planes; with FHE_Q_X128 the tiles only, and a shared
// exchange area [parity][component][r][lane][4] (the word of wave (c', j') for component c at j' + 2 (c' != c),
// swizzled by lane bits 3..4 so that the 64 lanes' b32 writes hit distinct banks)
constexpr int kQWave = (FHE_Q_X128 ? 1 : 5) * kG2Tile;
constexpr int kQX    = FHE_Q_X128 ? 2 * 2 * 16 * 64 * 4 : 0;
constexpr int kQAcc  = 105;          // |acc| < 10.5 Q between indices (units of Q/10)
constexpr size_t q_lds() { return (size_t)(1024 + 1024 + 2 * kMonoHalfWords + 4 * kQWave + kQX) * 4; }
static_assert(q_lds() <= 160 * 1024, "LDS per workgroup");
}  // namespace

template <bool MF, bool ACCIO>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2)))
    k_blind_rotate_ginx4x(GateArgs g, BootTables T, const uint4* __restrict__ keys, const uint16_t* __restrict__ idx,
                          const uint32_t* __restrict__ tvb, uint32_t* __restrict__ ext_a, uint32_t* __restrict__ ext_b,
                          const uint32_t* __restrict__ twAf) {
    constexpr int ND = 2, kQ = 2 * ND;
    extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
    uint32_t* s_tab  = sm;
    uint32_t* s_tabI = sm + 1024;
    uint2* s_mono2   = reinterpret_cast<uint2*>(sm + 2048);
    uint32_t* s_wave = sm + 2048 + 2 * kMonoHalfWords;
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) {
        s_tab[i]  = T.tabF[i];
        s_tabI[i] = T.tabI[i];
    }
    for (int i = threadIdx.x; i < kMonoHalfWords; i += blockDim.x)
        s_mono2[i] = MF ? make_uint2(T.monoP_full[i], T.mono_full[i]) : make_uint2(T.monoP[i], T.mono[i]);

    const int wave = threadIdx.x >> 6, L = threadIdx.x & 63;
    const int c = wave & 1, j = wave >> 1;  // component c, digit j
    const uint32_t gate = blockIdx.x;
    uint32_t* tile = s_wave + wave * kQWave;
    uint32_t* xown = tile + kG2Tile;  // plane [p][o] at xown + (2 p + o) kG2Tile: this wave's word for component c ^ o
    const uint32_t* xsib = s_wave + (wave ^ 2) * kQWave + kG2Tile + L;            // (c, 1 - j), o = 0
    const uint32_t* xo0  = s_wave + (1 - c) * kQWave + 2 * kG2Tile + L;           // (1 - c, 0), o = 1
    const uint32_t* xo1  = s_wave + (3 - c) * kQWave + 2 * kG2Tile + L;           // (1 - c, 1), o = 1
    const Mod m0 = make_mod(T);
    const Mod& m = m0;
    __syncthreads();

    // initial accumulator as K1x: acc1 = NTT(m) (both waves of component 1), acc0 = 0, or the seam's
    uint32_t acc[16];
    if (ACCIO && !g.acc_tv) {
        acc_load_c(acc, g, gate, c, L, T.ninvR, m);
    } else if (c == 1) {
        const uint32_t b = tvb[gate], cm = g.ctmod - 1;
        const uint32_t tvo = g.tv_mod > 1 ? (gate % g.tv_mod) * g.ctmod : 0u;
        uint32_t tv[1][16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t x = ((uint32_t)r << 6) | (uint32_t)L;
            uint32_t v = 0;
            if (x % g.factor == 0) {
                const uint32_t bx = (b - x / g.factor) & cm;
                v = g.tv ? g.tv[tvo + bx] : (bx >= g.lb && bx < g.ub) ? g.lv : g.uv;
            }
            tv[0][r] = v;
        }
        fwd_wave_s<1>(tv, tile, L, twAf, s_tab, m);
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = smont_mul(tv[0][r], T.ninvR, m);
    } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0;
    }

    const uint16_t* gidx = idx + (size_t)gate * g.n;
    const DecN dec = make_decn(m.Q, g.gbits, ND);
    const uint32_t lmul = 8 * (__builtin_bitreverse32((uint32_t)L) >> 26) + 1;
    const uint4* kc = keys + (size_t)c * (kQ * 8 * 64) + (size_t)(2 * j) * (8 * 64) + L;
    const uint32_t oneRj = j == 0 ? T.oneR : 0u;  // wave (c, 0) folds acc_c into its own-component word
    for (uint32_t i = 0; i < g.n; ++i) {
        const Mod m = fresh_nq(m0);
        const uint32_t as = __builtin_amdgcn_readfirstlane((uint32_t)gidx[i]) >> (MF ? 0 : 1);
        const uint4* kb = kc + (size_t)i * (2 * kQ * 8 * 64);
        uint4 kq[2][2];
#pragma unroll
        for (int o = 0; o < 2; ++o) kq[0][o] = kb[(o * 8 + 0) * 64];
        uint32_t d[ND][16];
#pragma unroll
        for (int r = 0; r < 16; ++r) d[0][r] = acc[r];
        inv_wave_s<kQAcc, true>(d[0], tile, L, s_tabI, T.w1R, m.oneR, m);
#pragma unroll
        for (int r = 0; r < 16; ++r) decompose_n<ND>(d[0][r], dec, d, r);
        uint32_t dj[1][16];
#pragma unroll
        for (int r = 0; r < 16; ++r) dj[0][r] = j ? d[1][r] : d[0][r];
        fwd_wave_s<1>(dj, tile, L, twAf, s_tab, m);
        uint32_t* xb = xown + (i & 1) * (2 * kG2Tile) + L;
        uint32_t* xx = s_wave + 4 * kQWave + (i & 1) * (2 * 16 * 256) + L * 4;  // FHE_Q_X128
        const uint32_t sw = ((uint32_t)L >> 3) & 3u;
        const uint32_t fl = (as * lmul) & (MF ? 2047u : 1023u);
        auto mono_r = [&](int r0, uint2& mp, uint2& mn) {
            const uint32_t ur = __builtin_amdgcn_readfirstlane(
                (as * (512u * (__builtin_bitreverse32((uint32_t)(r0 & 3)) >> 30) +
                       2u * (__builtin_bitreverse32((uint32_t)(r0 >> 2)) >> 30))) & (MF ? 2047u : 1023u));
            const uint32_t f  = MF ? (fl + ur) & 2047u : fl + ur;
            const uint32_t fn = 2048u - f;
            mp = s_mono2[f + (f >> 5)];
            mn = s_mono2[fn + (fn >> 5)];
        };
#pragma unroll
        for (int k2 = 0; k2 < 8; ++k2) {
            if (k2 + 1 < 8) {
#pragma unroll
                for (int o = 0; o < 2; ++o) kq[(k2 + 1) & 1][o] = kb[(o * 8 + k2 + 1) * 64];
            }
            asm volatile("" ::: "memory");
            const int r0 = 2 * k2;
            uint2 mp, mn;
            mono_r(r0, mp, mn);
            const uint4* q4 = kq[k2 & 1];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int r = r0 + e;
                if (MF && e == 1) mono_r(r, mp, mn);
#pragma unroll
                for (int o = 0; o < 2; ++o) {  // o = 0: component c, 1: component 1 - c
                    const uint4 kv = q4[o];
                    const int64_t S1 = (int64_t)(int32_t)dj[0][r] * (int32_t)(e ? kv.y : kv.x);
                    const int64_t S2 = (int64_t)(int32_t)dj[0][r] * (int32_t)(e ? kv.w : kv.z);
                    int64_t S = (int64_t)((uint64_t)(uint32_t)S1 * mp.x) + (int64_t)(int32_t)(S1 >> 32) * (int32_t)mp.y;
                    S += (int64_t)((uint64_t)(uint32_t)S2 * mn.x) + (int64_t)(int32_t)(S2 >> 32) * (int32_t)mn.y;
                    if (o == 0) S += (int64_t)(int32_t)acc[r] * (int32_t)oneRj;
                    const uint32_t w = smont_red(S, m);
                    if (FHE_Q_X128) {
                        xx[((o ? 1 - c : c) * 16 + r) * 256 + (((uint32_t)(j + 2 * o)) ^ sw)] = w;
                    } else {
                        xb[o * kG2Tile + (r << 6)] = w;
                        if (o == 0) acc[r] = w;
                    }
                }
            }
        }
        // every wave's words are in LDS (plane parity i & 1 is written again at index i + 2, after the other
        // waves have passed the barrier of index i + 1, i.e. after they read it)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        if (FHE_Q_X128) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const uint4 q = *reinterpret_cast<const uint4*>(xx + (c * 16 + r) * 256);
                acc[r] = q.x + q.y + q.z + q.w;
            }
        } else {
            const uint32_t po = (i & 1) * (2 * kG2Tile);
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] += xsib[po + (r << 6)] + xo0[po + (r << 6)] + xo1[po + (r << 6)];
        }
    }

    if (ACCIO) {
        if (j == 0) acc_store_c(acc, g, gate, c, L, T.nR, m);
        return;
    }
    if (j != 0) return;  // the digit-1 waves hold the same accumulators
    inv_wave_s<kQAcc, true>(acc, tile, L, s_tabI, T.w1R, m.oneR, m);
    if (c == 0) {
        uint32_t* oa = ext_a + (size_t)gate * g.N;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t x = ((uint32_t)r << 6) | (uint32_t)L;
            const uint32_t v = acc[r];
            const uint32_t o = (x == 0 || v == 0) ? v : m.Q - v;
            oa[(g.N - x) & (g.N - 1)] = g.msb_out ? mod_switch(o, m.Q, g.qKS) : o;
        }
    } else if (L == 0) {
        const uint32_t bb = add_mod(g.b_const, acc[0], m.Q);
        ext_b[gate] = g.msb_out ? mod_switch(bb, m.Q, g.qKS) : bb;
    }
}

hipError_t launch_blind_rotate_ginx4x(const GateArgs& g, const BootTables& t, const void* bskx, const uint16_t* idx,
                                      const uint32_t* tvb, uint32_t* ext_a, uint32_t* ext_b, hipStream_t s) {
    if (g.count == 0) return hipSuccess;
    if (!ginx2x_supported(g, t)) return hipErrorInvalidValue;
    static const bool attr = [] {
        for (const void* k : {reinterpret_cast<const void*>(&k_blind_rotate_ginx4x<false, false>),
                              reinterpret_cast<const void*>(&k_blind_rotate_ginx4x<true, false>),
                              reinterpret_cast<const void*>(&k_blind_rotate_ginx4x<false, true>),
                              reinterpret_cast<const void*>(&k_blind_rotate_ginx4x<true, true>)})
            (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)q_lds());
        return true;
    }();
    (void)attr;
#define FHE_LAUNCH_Q(MF_, IO)                                                                                       \
    hipLaunchKernelGGL((k_blind_rotate_ginx4x<MF_, IO>), dim3(g.count), dim3(256), q_lds(), s, g, t,                 \
                       static_cast<const uint4*>(bskx), idx, tvb, ext_a, ext_b, t.twA_fwd)
    const bool mf = g.ctmod == 2 * g.N;
    if (g.acc_io) { if (mf) FHE_LAUNCH_Q(true, true); else FHE_LAUNCH_Q(false, true); }
    else if (mf) FHE_LAUNCH_Q(true, false);
    else FHE_LAUNCH_Q(false, false);
#undef FHE_LAUNCH_Q
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// LMKCDEY on the split layout: k_blind_rotate_lmk3 (RingGSWAccumulatorLMKCDEY::EvalAcc,
// rgsw-acc-lmkcdey.cpp:70-287) for the digitsG = 4 sets at N = 1024, Q < 2^27 (STD128_4_LMKCDEY,
// STD128Q_3_LMKCDEY, LPF_STD128Q_LMKCDEY), which otherwise run K5's op-list form.  One gate per
// 128-thread workgroup (op lists differ per gate, so a workgroup barrier may only join the two waves
// of one gate); wave c owns component c in layout C as k_blind_rotate_ginx2.  The op list of
// k_prep_lmk_w, per op:
//   EXT(i)  (AddToAccLMKCDEY, :228-254): both waves decompose their component into 3 digits and
//           forward-transform them, exchange through LDS, acc_c <- sum_{p<6} D_p ek[i][row p][c];
//   AUTO(t) (Automorphism, :257-287): both components permuted in EVAL through the wave's region;
//           wave 0 inverse-transforms acc0', decomposes it into 3 digits and forward-transforms
//           them; acc0 <- sum_d D_d ak[t][d][0], acc1 <- acc1' + sum_d D_d ak[t][d][1].
// Keys (Engine::pack_ginx3, u32 Montgomery with N^-1 folded in), one uint4 = 4 registers:
//   ek: [i][c][p < 6][k4 < 4][64 lanes] rows g2_row(c, p, 3);  ak: [t][c][d < 3][k4 < 4][64 lanes].
// Bounds (Q < 2^27): |D| < 10 Q + 2^6, |S| < 61 Q^2 < 2^60, acc < 61 Q / 32 + Q / 2 < 2.8 Q.
// Round 6, ND = 2 (digitsG = 3: STD128_LMKCDEY, STD128_3_LMKCDEY, STD128Q_LMKCDEY, LPF_STD128_LMKCDEY, MEDIUM),
// the small-batch form of the one-wave op-list kernel k_blind_rotate_lmk on its fast path (u32 ctExt, keys
// repacked on the device by k_repack_lmkx, test-vector tables g.tv): LZ = Q < 2^27, else Q < 2^28 with the
// 8 Q headroom (kL3Acc; the test vector centred before its forward transform: |v| <= Q/2 grows to < 7.6 Q).
// ---------------------------------------------------------------------------
namespace {
// words per wave: ND tiles / the ND digit polynomials / a permutation
constexpr int l3_reg(int nd) { return nd * kG2Tile; }
constexpr size_t l3_lds(int nd, int gw) { return (size_t)(1024 + 1024 + 2 * gw * l3_reg(nd) + 4 * gw) * 4; }
// |acc| between ops (units of Q/10): 2.8 Q for Q < 2^27 (above); for Q < 2^28 (ND = 2: STD128_LMKCDEY, MEDIUM)
// the forward transform takes signed digits to < 6.67 Q (FHE_FWD_TIGHT), so an EXT sum is below
// 4 (6.67 Q) Q = 26.7 Q^2 and the reduced acc below 26.7 Q / 16 + Q / 2 < 2.2 Q; an AUTO sum of acc1 is below
// 2.2 Q Q + 2 (6.67 Q) Q
template <bool LZ> constexpr int kL3Acc = LZ ? kAccBoundLZ : 22;
// EVAL automorphism X -> X^k (as automorphism_eval) on layout C through this wave's region:
// slot x(L, r) has brv10(x) = brv2(r & 3) << 8 | brv6(L) << 2 | brv2(r >> 2), so
// (2 brv10(x) + 1) k = k (8 brv6(L) + 1) + k (512 brv2(r & 3) + 2 brv2(r >> 2))
FHE_DEV void automorphism_c(uint32_t (&v)[16], uint32_t* region, int L, uint32_t k) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t x = ((uint32_t)(r >> 2) << 8) | ((uint32_t)L << 2) | (uint32_t)(r & 3);
        region[x + (x >> 5)] = v[r];
    }
    wave_lds_sync();
    const uint32_t cl = (8 * (__builtin_bitreverse32((uint32_t)L) >> 26) + 1) * k;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t sr = (512u * (__builtin_bitreverse32((uint32_t)(r & 3)) >> 30) +
                             2u * (__builtin_bitreverse32((uint32_t)(r >> 2)) >> 30)) * k;  // uniform
        const uint32_t t  = ((cl + sr) & 2047u) >> 1;
        const uint32_t sx = __builtin_bitreverse32(t) >> 22;  // source slot brv10(t)
        v[r] = region[sx + (sx >> 5)];
    }
    wave_lds_sync();
}
}  // namespace

// GW: gates per workgroup.  GW = 1 up to one gate per CU; GW = 2 up to two (round 6, STD128_LMKCDEY): four waves of
// one workgroup take the four SIMDs of a CU, where two 128-thread workgroups may share two of them (512 gates
// 5.2 ms against 3.7 at 64).  The two gates' op lists differ, so a workgroup barrier would run them in lockstep
// (every op as long as the slower of the two: 4.1 ms at 64 gates); the two waves of a gate meet instead at a
// pair of LDS counters (gate_sync): 4.3 ms at 512 gates
template <int ND, bool LZ, typename OutT, bool ACCIO, int GW>
__global__ void __launch_bounds__(128 * GW) __attribute__((amdgpu_waves_per_eu(2, 2)))
    k_blind_rotate_lmk3(GateArgs g, BootTables T, const uint4* __restrict__ ek, const uint4* __restrict__ ak,
                        const uint16_t* __restrict__ ops, const uint32_t* __restrict__ nops, uint32_t maxops,
                        const uint32_t* __restrict__ tvb, OutT* __restrict__ ext_a, OutT* __restrict__ ext_b,
                        const uint32_t* __restrict__ twAf) {
    constexpr int kRows = 2 * ND;
    constexpr int BIN = kL3Acc<LZ>;
    extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
    uint32_t* s_tab  = sm;
    uint32_t* s_tabI = sm + 1024;
    uint32_t* s_reg  = sm + 2048;
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) {
        s_tab[i]  = T.tabF[i];
        s_tabI[i] = T.tabI[i];
    }
    uint32_t* s_flag = s_reg + 2 * GW * l3_reg(ND);  // GW > 1: one counter per wave
    if (GW > 1 && threadIdx.x < 2 * GW) s_flag[threadIdx.x] = 0;
    const int wave = threadIdx.x >> 6, c = wave & 1, L = threadIdx.x & 63;  // wave c of a gate: RLWE component c
    const uint32_t gslot = blockIdx.x * GW + (wave >> 1);
    const bool live = gslot < g.count;
    const uint32_t gate = live ? gslot : g.count - 1;  // a spare gate's waves shadow the last gate's
    uint32_t* region  = s_reg + wave * l3_reg(ND);
    uint32_t* partner = s_reg + (wave ^ 1) * l3_reg(ND);
    uint32_t* t0 = region;
    const Mod m0 = make_mod(T);
    const Mod& m = m0;
    const uint32_t M = 2 * g.N;
    __syncthreads();
    if (GW > 1 && !live) return;  // (no workgroup barrier below when GW > 1)
    // the two waves of this gate meet: sync k publishes this wave's LDS writes and reads before it and waits for
    // the partner's sync k (LDS ordering only: key loads in flight stay in flight)
    uint32_t nsync = 0;
    auto gate_sync = [&]() {
        if (GW == 1) {
            __syncthreads();
            return;
        }
        ++nsync;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __hip_atomic_store(s_flag + wave, nsync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        while (__builtin_amdgcn_readfirstlane(
                   __hip_atomic_load(s_flag + (wave ^ 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < nsync)
            __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    };

    // BootstrapGateCore (binfhe-base-scheme.cpp:556-575): acc1 = NTT(m), acc0 = 0; then
    // acc1 <- acc1(X^(2N-5)) (:99; acc0 = 0 is invariant)
    uint32_t acc[16];
    if (ACCIO && !g.acc_tv) {
        acc_load_c(acc, g, gate, c, L, T.ninvR, m);
        if (c == 1) automorphism_c(acc, region, L, M - 5);   // acc1 <- acc1(X^(2N-5)) (:99)
    } else if (c == 1) {
        const uint32_t b = tvb[gate], cm = g.ctmod - 1;
        // BootstrapFuncCore's table g.tv (:596-608), EvalFuncMultiOutput: table gate % tv_mod (GateArgs::tv_mod)
        const uint32_t tvo = g.tv_mod > 1 ? (gate % g.tv_mod) * g.ctmod : 0u;
        uint32_t tv[1][16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t x = ((uint32_t)r << 6) | (uint32_t)L;
            uint32_t v = 0;
            if (x % g.factor == 0) {
                const uint32_t bx = (b - x / g.factor) & cm;
                v = g.tv ? g.tv[tvo + bx] : (bx >= g.lb && bx < g.ub) ? g.lv : g.uv;
            }
            if (!LZ) v = v > (m.Q >> 1) ? v - m.Q : v;  // centred: |v| <= Q/2 (8 Q headroom)
            tv[0][r] = v;
        }
        fwd_wave_s<1>(tv, t0, L, twAf, s_tab, m);
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = smont_mul(tv[0][r], T.ninvR, m);
        automorphism_c(acc, region, L, M - 5);
    } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0;
    }

    const DecN dec = make_decn(m.Q, g.gbits, ND);
    const uint16_t* gops = ops + (size_t)gate * maxops;
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(nops[gate]);
    const uint32_t oneR1 = c ? m0.oneR : 0u;  // automorphism: acc1 accumulates, acc0 is replaced
    for (uint32_t it = 0; it < cnt; ++it) {
        const Mod m = fresh_nq(m0);
        const uint32_t op = __builtin_amdgcn_readfirstlane((uint32_t)gops[it]);
        gate_sync();  // the partner wave has read this wave's region (previous op)
        uint32_t d[ND][16];
        if (!(op & 0x8000u)) {
            // ---- AddToAccLMKCDEY: acc_c <- sum_p D_p ek[op][g2_row(c, p)][c]   (acc replaced)
            const uint4* kb = ek + ((size_t)op * 2 + c) * (kRows * 4 * 64) + L;
            uint4 kq[2][kRows];
#pragma unroll
            for (int p = 0; p < kRows; ++p) kq[0][p] = kb[(p * 4 + 0) * 64];
#pragma unroll
            for (int r = 0; r < 16; ++r) d[0][r] = acc[r];
            inv_wave_s<BIN, LZ>(d[0], t0, L, s_tabI, T.w1R, m.oneR, m);
#pragma unroll
            for (int r = 0; r < 16; ++r) decompose_n<ND>(d[0][r], dec, d, r);
            fwd_wave_s<ND>(d, t0, L, twAf, s_tab, m);
            wave_lds_sync();
#pragma unroll
            for (int r = 0; r < 16; ++r)
#pragma unroll
                for (int j = 0; j < ND; ++j) region[j * 1024 + ((r << 6) | L)] = d[j][r];
            gate_sync();  // both waves' digits are in LDS
#pragma unroll
            for (int k4 = 0; k4 < 4; ++k4) {
                if (k4 + 1 < 4) {
#pragma unroll
                    for (int p = 0; p < kRows; ++p) kq[(k4 + 1) & 1][p] = kb[(p * 4 + k4 + 1) * 64];
                }
                asm volatile("" ::: "memory");
                const uint4* q = kq[k4 & 1];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = 4 * k4 + e;
                    int64_t S = 0;
#pragma unroll
                    for (int p = 0; p < kRows; ++p) {
                        const int32_t dv = (int32_t)(p < ND ? d[p][r] : partner[(p - ND) * 1024 + ((r << 6) | L)]);
                        const uint32_t kv = e == 0 ? q[p].x : e == 1 ? q[p].y : e == 2 ? q[p].z : q[p].w;
                        S += (int64_t)dv * (int32_t)kv;
                    }
                    acc[r] = smont_red(S, m);
                }
            }
        } else {
            // ---- Automorphism(5^t or 2N-5, ak[t])
            const uint32_t t = op & 0x7fffu;
            uint32_t kexp = M - 5;
            if (t) {
                kexp = 1;
                for (uint32_t z = 0; z < t; ++z) kexp = (kexp * 5) & (M - 1);
            }
            const uint4* kb = ak + ((size_t)t * 2 + c) * (ND * 4 * 64) + L;
            uint4 kq[2][ND];
#pragma unroll
            for (int p = 0; p < ND; ++p) kq[0][p] = kb[(p * 4 + 0) * 64];
            automorphism_c(acc, region, L, kexp);
            if (c == 0) {  // acc0' -> COEF -> 3 digits -> EVAL, to this wave's region
#pragma unroll
                for (int r = 0; r < 16; ++r) d[0][r] = acc[r];
                inv_wave_s<BIN, LZ>(d[0], t0, L, s_tabI, T.w1R, m.oneR, m);
#pragma unroll
                for (int r = 0; r < 16; ++r) decompose_n<ND>(d[0][r], dec, d, r);
                fwd_wave_s<ND>(d, t0, L, twAf, s_tab, m);
                wave_lds_sync();
#pragma unroll
                for (int r = 0; r < 16; ++r)
#pragma unroll
                    for (int j = 0; j < ND; ++j) region[j * 1024 + ((r << 6) | L)] = d[j][r];
            }
            gate_sync();  // acc0's digits are in wave 0's region
            const uint32_t* src = c == 0 ? region : partner;
#pragma unroll
            for (int k4 = 0; k4 < 4; ++k4) {
                if (k4 + 1 < 4) {
#pragma unroll
                    for (int p = 0; p < ND; ++p) kq[(k4 + 1) & 1][p] = kb[(p * 4 + k4 + 1) * 64];
                }
                asm volatile("" ::: "memory");
                const uint4* q = kq[k4 & 1];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = 4 * k4 + e;
                    int64_t S = (int64_t)(int32_t)acc[r] * (int32_t)oneR1;
#pragma unroll
                    for (int p = 0; p < ND; ++p) {
                        const int32_t dv = (int32_t)src[p * 1024 + ((r << 6) | L)];
                        const uint32_t kv = e == 0 ? q[p].x : e == 1 ? q[p].y : e == 2 ? q[p].z : q[p].w;
                        S += (int64_t)dv * (int32_t)kv;
                    }
                    acc[r] = smont_red(S, m);
                }
            }
        }
    }

    if (ACCIO) {
        if (live) acc_store_c(acc, g, gate, c, L, T.nR, m);
        return;
    }
    // extraction (binfhe-base-scheme.cpp:110-121), as k_blind_rotate_ginx2
    gate_sync();
    inv_wave_s<BIN, LZ>(acc, t0, L, s_tabI, T.w1R, m.oneR, m);
    if (!live) return;
    if (c == 0) {
        OutT* oa = ext_a + (size_t)gate * g.N;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t x = ((uint32_t)r << 6) | (uint32_t)L;
            const uint32_t v = acc[r];
            const uint32_t o = (x == 0 || v == 0) ? v : m.Q - v;
            oa[(g.N - x) & (g.N - 1)] = g.msb_out ? mod_switch(o, m.Q, g.qKS) : o;
        }
    } else if (L == 0) {
        const uint32_t bb = add_mod(g.b_const, acc[0], m.Q);
        ext_b[gate] = g.msb_out ? mod_switch(bb, m.Q, g.qKS) : bb;
    }
}

hipError_t launch_blind_rotate_lmk3(const GateArgs& g, const BootTables& t, const void* ek, const void* ak,
                                    const uint16_t* ops, const uint32_t* nops, uint32_t maxops, const uint32_t* tvb,
                                    uint64_t* ext_a, uint64_t* ext_b, hipStream_t s) {
    if (g.count == 0) return hipSuccess;
    if (!(t.Q < (1u << 27) && g.N == 1024 && g.tv == nullptr && g.tv64 == nullptr && g.gbits >= 2 &&
          4 * g.gbits <= 32 && g.qKS <= 65536))
        return hipErrorInvalidValue;
#define FHE_LAUNCH_L3(IO)                                                                                          \
    hipLaunchKernelGGL((k_blind_rotate_lmk3<3, true, uint64_t, IO, 1>), dim3(g.count), dim3(128), l3_lds(3, 1), s, g, t, \
                       static_cast<const uint4*>(ek), static_cast<const uint4*>(ak), ops, nops, maxops, tvb, ext_a,  \
                       ext_b, t.twA_fwd)
    if (g.acc_io) FHE_LAUNCH_L3(true);
    else FHE_LAUNCH_L3(false);
#undef FHE_LAUNCH_L3
    return hipGetLastError();
}

// the resident LMKCDEY layout (row_off, half-swapped rows: [n][4][16][64] uint2 ++ [nA + 1][2][16][64] uint2) ->
// k_blind_rotate_lmk3<2, ..>'s: ek [n][c][p < 4][k4 < 4][64][4] (rows g2_row(c, p, 2)) ++ ak [nA + 1][c][d < 2][k4][64][4]
__global__ void k_repack_lmkx(const uint32_t* __restrict__ src, uint32_t n, uint32_t nauto, uint32_t* __restrict__ dst) {
    const uint64_t ekw = (uint64_t)n * 8192, words = ekw + (uint64_t)nauto * 4096;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < words; t += (uint64_t)gridDim.x * blockDim.x) {
        const bool auto_key = t >= ekw;
        const uint64_t u = auto_key ? t - ekw : t;
        const uint64_t i = auto_key ? u >> 12 : u >> 13;
        const uint32_t w = (uint32_t)(u & (auto_key ? 4095 : 8191));
        const uint32_t e = w & 3, L = (w >> 2) & 63, k4 = (w >> 8) & 3;
        const uint32_t c = auto_key ? w >> 11 : w >> 12, p = auto_key ? (w >> 10) & 1 : (w >> 10) & 3;
        const uint32_t row = auto_key ? p : g2_row(c, p, 2);
        const uint32_t x = (k4 << 8) | (L << 2) | e;  // EVAL slot of layout C
        const uint32_t lane = c * 32 + (x >> 5), kk = (x & 31) >> 1, ee = x & 1;
        const uint32_t dpos = kBskHalfSwap ? row ^ c : row;
        const uint64_t base = auto_key ? ekw + i * 4096 : i * 8192;
        dst[t] = src[base + row_off(dpos, kk, lane, ee)];
    }
}

hipError_t launch_repack_lmkx(const void* bsk, uint32_t n, uint32_t nauto, void* bskx, hipStream_t s) {
    const uint64_t words = (uint64_t)n * 8192 + (uint64_t)nauto * 4096;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((words + 255) / 256, 16384);
    hipLaunchKernelGGL(k_repack_lmkx, dim3(blocks), dim3(256), 0, s, static_cast<const uint32_t*>(bsk), n, nauto,
                       static_cast<uint32_t*>(bskx));
    return hipGetLastError();
}

bool lmkx_supported(const GateArgs& g, const BootTables& t) {
    return t.Q < (1u << 28) && g.N == 1024 && g.tv64 == nullptr && g.gbits >= 2 && 3 * g.gbits <= 32;
}

hipError_t launch_blind_rotate_lmkx(const GateArgs& g, const BootTables& t, const void* ekx, uint32_t n,
                                    const uint16_t* ops, const uint32_t* nops, uint32_t maxops, const uint32_t* tvb,
                                    uint32_t* ext_a, uint32_t* ext_b, int gw, hipStream_t s) {
    if (g.count == 0) return hipSuccess;
    if (!lmkx_supported(g, t) || (gw != 1 && gw != 2)) return hipErrorInvalidValue;
    const uint4* ek = static_cast<const uint4*>(ekx);
    const uint4* ak = ek + (size_t)n * 2048;
#define FHE_LAUNCH_LX(LZ_, IO, GW_)                                                                                    \
    hipLaunchKernelGGL((k_blind_rotate_lmk3<2, LZ_, uint32_t, IO, GW_>), dim3((g.count + GW_ - 1) / GW_), dim3(128 * GW_), \
                       l3_lds(2, GW_), s, g, t, ek, ak, ops, nops, maxops, tvb, ext_a, ext_b, t.twA_fwd)
#define FHE_LAUNCH_LX2(LZ_, IO) \
    if (gw == 1) FHE_LAUNCH_LX(LZ_, IO, 1); else FHE_LAUNCH_LX(LZ_, IO, 2)
    const bool lz = t.Q < (1u << 27);
    if (g.acc_io) { if (lz) { FHE_LAUNCH_LX2(true, true); } else { FHE_LAUNCH_LX2(false, true); } }
    else if (lz) { FHE_LAUNCH_LX2(true, false); }
    else { FHE_LAUNCH_LX2(false, false); }
#undef FHE_LAUNCH_LX2
#undef FHE_LAUNCH_LX
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// K1m-4: LMKCDEY with FOUR waves per gate (k_blind_rotate_lmk4x), the latency kernel of the digitsG = 3 sets for
// batches of up to one gate per CU (K1q's split applied to the op list).  Wave (c, j) = wave c + 2 j owns component
// c (layout C) and retained digit j (row 2 j + c); one gate per 256-thread workgroup.  Per op of k_prep_lmk_w:
//   EXT(i)  (AddToAccLMKCDEY, rgsw-acc-lmkcdey.cpp:228-254): both waves of component c inverse-transform acc_c (the
//           same values), wave (c, j) forward-transforms digit j and multiplies it by ek[i][row 2 j + c] in both
//           columns: the column-c word and the column-(1 - c) word go to its exchange planes; one barrier;
//           acc_c = its column-c word + the sibling's + both (1 - c, *) waves' column-c words (acc replaced);
//   AUTO(t) (Automorphism, :257-287): every wave permutes its copy of acc_c; the component-0 waves transform
//           acc0' and multiply digit j by ak[t][row j] in both columns while the component-1 waves reduce
//           acc1' (one signed Montgomery product by 2^32 mod Q); one barrier; acc0 = the two column-0 words,
//           acc1 = acc1' + the two column-1 words.
// Keys: K1m's two-digit layout (k_repack_lmkx): row 2 j + c of column c at ek[i][c][p = j], of column 1 - c at
// ek[i][1 - c][p = 2 + j]; ak[t][c'][d = j] for column c'.
// Bounds: a word is one digit x key product reduced, < 6.67 Q^2 / 2^32 + Q/2 < 0.92 Q (Q < 2^28; < 0.68 Q for
// Q < 2^27), so acc < 3.7 Q after EXT and < 2.4 Q after AUTO (BIN 37; signed headroom 8 Q or 16 Q).
// ---------------------------------------------------------------------------
namespace {
#ifndef FHE_M4_X128
#define FHE_M4_X128 1  // K1q's shared exchange area: the four words of a slot side by side, one ds_read_b128 (0: A/B)
#endif
// words per wave: a transpose tile and [parity][o] exchange planes (FHE_M4_X128: the tile; the area after the tiles)
constexpr int kMWave = (FHE_M4_X128 ? 1 : 5) * kG2Tile;
constexpr int kMX    = FHE_M4_X128 ? 2 * 2 * 16 * 64 * 4 : 0;
constexpr int kMAcc  = 37;           // |acc| < 3.7 Q between ops (units of Q/10)
constexpr size_t m4_lds() { return (size_t)(1024 + 1024 + 4 * kMWave + kMX) * 4; }
static_assert(m4_lds() <= 160 * 1024, "LDS per workgroup");
}  // namespace

template <bool LZ, bool ACCIO>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2)))
    k_blind_rotate_lmk4x(GateArgs g, BootTables T, const uint4* __restrict__ ek, const uint4* __restrict__ ak,
                         const uint16_t* __restrict__ ops, const uint32_t* __restrict__ nops, uint32_t maxops,
                         const uint32_t* __restrict__ tvb, uint32_t* __restrict__ ext_a, uint32_t* __restrict__ ext_b,
                         const uint32_t* __restrict__ twAf) {
    constexpr int ND = 2;
    extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
    uint32_t* s_tab  = sm;
    uint32_t* s_tabI = sm + 1024;
    uint32_t* s_wave = sm + 2048;
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) {
        s_tab[i]  = T.tabF[i];
        s_tabI[i] = T.tabI[i];
    }
    const int wave = threadIdx.x >> 6, L = threadIdx.x & 63;
    const int c = wave & 1, j = wave >> 1;  // component c, digit j
    const uint32_t gate = blockIdx.x;
    uint32_t* tile = s_wave + wave * kMWave;
    uint32_t* xown = tile + kG2Tile + L;  // plane [p][o] at + (2 p + o) kG2Tile: this wave's word for column c ^ o
    uint32_t* xx_ = nullptr;              // FHE_M4_X128: this op's area, at this lane's four slots
    const uint32_t sw = ((uint32_t)L >> 3) & 3u;
    const uint32_t* xsib = s_wave + (wave ^ 2) * kMWave + kG2Tile + L;   // (c, 1 - j), o = 0
    const uint32_t* xo0  = s_wave + (1 - c) * kMWave + 2 * kG2Tile + L;  // (1 - c, 0), o = 1
    const uint32_t* xo1  = s_wave + (3 - c) * kMWave + 2 * kG2Tile + L;  // (1 - c, 1), o = 1
    const Mod m0 = make_mod(T);
    const Mod& m = m0;
    const uint32_t M = 2 * g.N;
    __syncthreads();
    auto barrier = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    };

    // BootstrapGateCore (binfhe-base-scheme.cpp:556-575) / BootstrapFuncCore's table: acc1 = NTT(m) in both
    // component-1 waves, acc0 = 0; then acc1 <- acc1(X^(2N-5)) (:99)
    uint32_t acc[16];
    if (ACCIO && !g.acc_tv) {
        acc_load_c(acc, g, gate, c, L, T.ninvR, m);
        if (c == 1) automorphism_c(acc, tile, L, M - 5);
    } else if (c == 1) {
        const uint32_t b = tvb[gate], cm = g.ctmod - 1;
        const uint32_t tvo = g.tv_mod > 1 ? (gate % g.tv_mod) * g.ctmod : 0u;
        uint32_t tv[1][16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t x = ((uint32_t)r << 6) | (uint32_t)L;
            uint32_t v = 0;
            if (x % g.factor == 0) {
                const uint32_t bx = (b - x / g.factor) & cm;
                v = g.tv ? g.tv[tvo + bx] : (bx >= g.lb && bx < g.ub) ? g.lv : g.uv;
            }
            if (!LZ) v = v > (m.Q >> 1) ? v - m.Q : v;  // centred: |v| <= Q/2 (8 Q headroom)
            tv[0][r] = v;
        }
        fwd_wave_s<1>(tv, tile, L, twAf, s_tab, m);
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = smont_mul(tv[0][r], T.ninvR, m);
        automorphism_c(acc, tile, L, M - 5);
    } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0;
    }

    const DecN dec = make_decn(m.Q, g.gbits, ND);
    const uint16_t* gops = ops + (size_t)gate * maxops;
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(nops[gate]);
    // digit j of acc (COEF, canonical) forward-transformed to EVAL
    auto digit = [&](uint32_t (&dj)[1][16], const Mod& m) {
        uint32_t d[ND][16];
#pragma unroll
        for (int r = 0; r < 16; ++r) d[0][r] = acc[r];
        inv_wave_s<kMAcc, LZ>(d[0], tile, L, s_tabI, T.w1R, m.oneR, m);
#pragma unroll
        for (int r = 0; r < 16; ++r) decompose_n<ND>(d[0][r], dec, d, r);
#pragma unroll
        for (int r = 0; r < 16; ++r) dj[0][r] = j ? d[1][r] : d[0][r];
        fwd_wave_s<1>(dj, tile, L, twAf, s_tab, m);
    };
    // the words of digit j against the key columns k0 (column c, or 0) and k1 (the other, or 1), to plane parity p
    auto words = [&](const uint32_t (&dj)[1][16], const uint4* k0, const uint4* k1, uint32_t* xb, const Mod& m) {
        uint4 kq[2][2];
        kq[0][0] = k0[0];
        kq[0][1] = k1[0];
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
            if (k4 + 1 < 4) {
                kq[(k4 + 1) & 1][0] = k0[(k4 + 1) * 64];
                kq[(k4 + 1) & 1][1] = k1[(k4 + 1) * 64];
            }
            asm volatile("" ::: "memory");
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int r = 4 * k4 + e;
#pragma unroll
                for (int o = 0; o < 2; ++o) {
                    const uint4 q = kq[k4 & 1][o];
                    const uint32_t kv = e == 0 ? q.x : e == 1 ? q.y : e == 2 ? q.z : q.w;
                    const uint32_t w = smont_red((int64_t)(int32_t)dj[0][r] * (int32_t)kv, m);
                    if (FHE_M4_X128) {  // component c ^ o, slot j + 2 o (swizzled)
                        xx_[(((uint32_t)(c ^ o)) * 16 + r) * 256 + (((uint32_t)(j + 2 * o)) ^ sw)] = w;
                    } else {
                        xb[o * kG2Tile + (r << 6)] = w;
                        if (o == 0) acc[r] = w;
                    }
                }
            }
        }
    };
    auto sum4 = [&](const uint32_t* xx) {  // FHE_M4_X128: acc_c = the four words of its slots
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint4 q = *reinterpret_cast<const uint4*>(xx + (c * 16 + r) * 256);
            acc[r] = q.x + q.y + q.z + q.w;
        }
    };
    for (uint32_t it = 0; it < cnt; ++it) {
        const Mod m = fresh_nq(m0);
        const uint32_t op = __builtin_amdgcn_readfirstlane((uint32_t)gops[it]);
        const uint32_t po = (it & 1) * (2 * kG2Tile);
        uint32_t* xb = xown + po;
        xx_ = s_wave + 4 * kMWave + (it & 1) * (2 * 16 * 256) + L * 4;
        uint32_t dj[1][16];
        if (!(op & 0x8000u)) {
            // ---- AddToAccLMKCDEY: acc_c <- sum over the four digits D ek[op][row][c]   (acc replaced)
            digit(dj, m);
            words(dj, ek + ((size_t)op * 2 + c) * (4 * 4 * 64) + (size_t)j * (4 * 64) + L,
                  ek + ((size_t)op * 2 + (1 - c)) * (4 * 4 * 64) + (size_t)(2 + j) * (4 * 64) + L, xb, m);
            barrier();
            if (FHE_M4_X128) {
                sum4(xx_);
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] += xsib[po + (r << 6)] + xo0[po + (r << 6)] + xo1[po + (r << 6)];
            }
        } else {
            // ---- Automorphism(5^t or 2N-5, ak[t])
            const uint32_t t = op & 0x7fffu;
            uint32_t kexp = M - 5;
            if (t) {
                kexp = 1;
                for (uint32_t z = 0; z < t; ++z) kexp = (kexp * 5) & (M - 1);
            }
            automorphism_c(acc, tile, L, kexp);
            if (c == 0) {  // acc0' -> digit j -> the column-0 and column-1 words
                digit(dj, m);
                words(dj, ak + ((size_t)t * 2 + 0) * (ND * 4 * 64) + (size_t)j * (4 * 64) + L,
                      ak + ((size_t)t * 2 + 1) * (ND * 4 * 64) + (size_t)j * (4 * 64) + L, xb, m);
            } else {       // acc1' reduced while component 0 transforms
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = smont_mul(acc[r], m.oneR, m);
                if (FHE_M4_X128) {  // acc1' (or 0) into slot j of component 1, 0 into slot 2 + j of component 0
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        xx_[(16 + r) * 256 + (((uint32_t)j) ^ sw)] = j == 0 ? acc[r] : 0u;
                        xx_[r * 256 + (((uint32_t)(2 + j)) ^ sw)] = 0u;
                    }
                }
            }
            barrier();
            if (FHE_M4_X128) {
                sum4(xx_);
            } else if (c == 0) {
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] += xsib[po + (r << 6)];
            } else {
                const uint32_t* w0 = s_wave + 0 * kMWave + 2 * kG2Tile + L + po;  // (0, 0), o = 1
                const uint32_t* w1 = s_wave + 2 * kMWave + 2 * kG2Tile + L + po;  // (0, 1), o = 1
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] += w0[r << 6] + w1[r << 6];
            }
        }
    }

    if (ACCIO) {
        if (j == 0) acc_store_c(acc, g, gate, c, L, T.nR, m);
        return;
    }
    if (j != 0) return;  // the digit-1 waves hold the same accumulators
    // extraction (binfhe-base-scheme.cpp:110-121), as k_blind_rotate_lmk3
    inv_wave_s<kMAcc, LZ>(acc, tile, L, s_tabI, T.w1R, m.oneR, m);
    if (c == 0) {
        uint32_t* oa = ext_a + (size_t)gate * g.N;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t x = ((uint32_t)r << 6) | (uint32_t)L;
            const uint32_t v = acc[r];
            const uint32_t o = (x == 0 || v == 0) ? v : m.Q - v;
            oa[(g.N - x) & (g.N - 1)] = g.msb_out ? mod_switch(o, m.Q, g.qKS) : o;
        }
    } else if (L == 0) {
        const uint32_t bb = add_mod(g.b_const, acc[0], m.Q);
        ext_b[gate] = g.msb_out ? mod_switch(bb, m.Q, g.qKS) : bb;
    }
}

hipError_t launch_blind_rotate_lmk4x(const GateArgs& g, const BootTables& t, const void* ekx, uint32_t n,
                                     const uint16_t* ops, const uint32_t* nops, uint32_t maxops, const uint32_t* tvb,
                                     uint32_t* ext_a, uint32_t* ext_b, hipStream_t s) {
    if (g.count == 0) return hipSuccess;
    if (!lmkx_supported(g, t)) return hipErrorInvalidValue;
    static const bool attr = [] {
        for (const void* k : {reinterpret_cast<const void*>(&k_blind_rotate_lmk4x<false, false>),
                              reinterpret_cast<const void*>(&k_blind_rotate_lmk4x<true, false>),
                              reinterpret_cast<const void*>(&k_blind_rotate_lmk4x<false, true>),
                              reinterpret_cast<const void*>(&k_blind_rotate_lmk4x<true, true>)})
            (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)m4_lds());
        return true;
    }();
    (void)attr;
    const uint4* ek = static_cast<const uint4*>(ekx);
    const uint4* ak = ek + (size_t)n * 2048;
#define FHE_LAUNCH_M4(LZ_, IO)                                                                                     \
    hipLaunchKernelGGL((k_blind_rotate_lmk4x<LZ_, IO>), dim3(g.count), dim3(256), m4_lds(), s, g, t, ek, ak, ops,  \
                       nops, maxops, tvb, ext_a, ext_b, t.twA_fwd)
    const bool lz = t.Q < (1u << 27);
    if (g.acc_io) { if (lz) FHE_LAUNCH_M4(true, true); else FHE_LAUNCH_M4(false, true); }
    else if (lz) FHE_LAUNCH_M4(true, false);
    else FHE_LAUNCH_M4(false, false);
#undef FHE_LAUNCH_M4
    return hipGetLastError();
}

// ===========================================================================
// K1w: GINX at N = 2048 with the accumulator in registers (k_blind_rotate_n2k<ND, ACCIO>) for the
// Q < 2^27 rows with even monomial exponents (ciphertext modulus q < 2N): STD256Q (digitsG = 4,
// ND = 3 retained digits), which otherwise run the one-gate-per-workgroup accumulator K5
// (bootstrap_wide.hip) with every butterfly through LDS.  As K1s, wave c of a gate owns RLWE
// component c, here as 32 registers x 64 lanes, through the three layouts (x: 11-bit coefficient
// or EVAL slot index)
//   A: lane = x5..x0, register = x10..x6      (COEF; forward stages on bits 10..6, uniform twiddles)
//   B: lane = (x10..x6) << 1 | x0, register = x5..x1   (stages on bits 5..1, per-lane twiddles)
//   C: lane = x6..x1, register = (x10..x7) << 1 | x0   (EVAL; the stage on bit 0)
// with one LDS tile per wave (word of x: x + 2 (x >> 6): A and B conflict-free, C moved as 8-byte
// pairs).  Per index i (AddToAccCGGI, rgsw-acc-cggi.cpp:102-151): wave c inverse-transforms acc_c
// (signed, its own reduction plan), decomposes it into its ND digits (SignedDigitDecompose,
// rgsw-acc.cpp:54-91; rows 2j + c of the RGSW keys) and forward-transforms them; it then multiplies
// its own digits by the key columns of BOTH components: the sum for its own component stays in its
// registers, the other one is reduced to a word per slot and handed to the partner through this
// wave's tile (8 KiB instead of the ND digit polynomials: four gates per CU fit in LDS), and after
// one barrier each wave adds the partner's word.  acc_c <- acc_c + S+_c (X^a - 1) + S-_c (X^-a - 1)
// exactly as in K1s; only the order of the modular additions differs.
// Keys (Engine::pack_n2k, u32 Montgomery with N^-1 folded in), per index and wave c:
//   [c][q < 2 ND][k2 < 16][64 lanes] uint4 = (K+[r], K+[r + 1], K-[r], K-[r + 1]), r = 2 k2, slot
//   x(L, r) of layout C; q = 2 j + o: digit row 2 j + c, column c (o = 0) or 1 - c (o = 1).
// Bounds (Q < 2^27): digits |d| <= 2^(g-1) grow to < 11 Q + 2^(g-1) in the forward transform;
// |S+-| < ND (11 Q + 2^(g-1)) Q; each reduced sum < 2.6 Q; acc < 5.3 Q after the exchange (the
// inverse plan's BIN).
// ===========================================================================
namespace {
#ifndef FHE_N2K_OPAQUE
#define FHE_N2K_OPAQUE 0
#endif
#ifndef FHE_N2K_KPF
#define FHE_N2K_KPF 1   // key chunks requested ahead of their MAC (0: on use)
#endif
constexpr int kW2Gates = 2;               // gates per workgroup (2 waves each)
constexpr int kW2Tile  = 2048 + 64;       // words of one wave's tile
constexpr int kW2Mono  = 2048 + 1 + 64;   // (plain, Montgomery) pairs psi^(2f) - 1, f in [0, 2048], entry f + (f >> 5)
constexpr int kW2AccBound = 53;           // |acc| < 5.3 Q between indices (units of Q/10)
constexpr size_t w2_lds() { return (size_t)(2048 + 2048 + 2 * kW2Mono + 2 * kW2Gates * kW2Tile) * 4; }
// LDS word of x: x + 2 (x >> 6) (wa2k / wb2k / wc2k below)
FHE_DEV uint32_t slot_2k(int L, int r) {
    return ((uint32_t)(r >> 1) << 7) | ((uint32_t)L << 1) | (uint32_t)(r & 1);
}

// signed forward NTT, layout A (|v| < B) -> C (|v| < B + 11 Q), NP polynomials through one tile
// (transposed one after the other); twA: Table[0..31] (uniform), s_tab: Table[0..2047] in LDS
// word of x in each layout as a per-lane base plus a per-register constant (so that every LDS access
// is base + immediate): A x = (r << 6) | L -> L + 66 r; B x = (G << 6) | (r << 1) | j -> 66 G + j + 2 r;
// C pair x = (rh << 7) | (L << 1) -> 2 L + 2 (L >> 5) + 132 rh
FHE_DEV int wa2k(int L) { return L; }
FHE_DEV int wb2k(int L) { return 66 * (L >> 1) + (L & 1); }
FHE_DEV int wc2k(int L) { return 2 * L + 2 * (L >> 5); }

// QM, the modulus class: 0: Q < 2^27 (16Q of signed headroom), no reduction; 1: Q < 2^28 (8Q): one signed
// Montgomery product by 2^32 mod Q after the five A stages (|v| < 5Q + 2^(g-1) -> < 0.82 Q), the six
// stages after it end below 6.82 Q; 2: Q < 2^29 (4Q): one after stages 3, 6 and 9 (< 3Q + 2^(g-1) ->
// < 0.875 Q, < 3.875 Q -> < 0.98 Q, < 3.98 Q -> < Q), the last two end below 3 Q
template <int NP>
FHE_DEV void red_2k(uint32_t (&v)[NP][32], const Mod& m) {
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int r = 0; r < 32; ++r) v[p][r] = smont_mul(v[p][r], m.oneR, m);
}

// one radix-2 stage over the 32 registers: A stages (b = 10..6) pair register bits b - 6 with the twiddles
// of twA; B stages (b = 5..1) pair register bits b - 1 with s_tab's, indexed by the lane pair G
template <int NP, bool B>
FHE_DEV void fwd_2k_stage(uint32_t (&v)[NP][32], int b, int G, const uint32_t* __restrict__ tw, const Mod& m) {
    const int rb = B ? b - 1 : b - 6;
#pragma unroll
    for (int r = 0; r < 32; ++r) {
        if (r & (1 << rb)) continue;
        const uint32_t w = B ? tw[(1 << (10 - b)) + (G << (5 - b)) + (r >> b)] : tw[(1 << (10 - b)) + (r >> (rb + 1))];
#pragma unroll
        for (int p = 0; p < NP; ++p) ct_bf_s(v[p][r], v[p][r | (1 << rb)], w, m);
    }
}

// v - rint(v / Q) Q in 32-bit registers (|v| < 2^31): the float quotient is off by under 2^-20, so the
// result is below 0.51 Q; no 64-bit temporaries (FRED: K1w GINX, whose 3-digit form spilled 104 VGPRs with
// smont_mul's and 30 with this; K1w-LMKCDEY keeps red_2k, measured 6% faster there)
template <int NP>
FHE_DEV void red_2k_f(uint32_t (&v)[NP][32], const Mod& m) {
    const float iq = 1.0f / (float)m.Q;
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            const int32_t x = (int32_t)v[p][r];
            const int32_t q = (int32_t)__builtin_rintf((float)x * iq);
            v[p][r]         = (uint32_t)(x - q * (int32_t)m.Q);
        }
}

template <int NP, int QM = 0, bool FRED = false>
FHE_DEV void fwd_2k_s(uint32_t (&v)[NP][32], uint32_t* t, int L, const uint32_t* __restrict__ twA,
                      const uint32_t* s_tab, const Mod& m) {
    // the stages are written out: a loop over them with the reductions inside was left rolled for NP = 3,
    // and a plain one for NP = 4 (the digit array in scratch)
    const int G = L >> 1;
    uint32_t* ta = t + wa2k(L);
    uint32_t* tb = t + wb2k(L);
    uint32_t* tc = t + wc2k(L);
    fwd_2k_stage<NP, false>(v, 10, G, twA, m);
    fwd_2k_stage<NP, false>(v, 9, G, twA, m);
    fwd_2k_stage<NP, false>(v, 8, G, twA, m);
    if (QM == 2 && !FHE_FWD_TIGHT) FRED ? red_2k_f<NP>(v, m) : red_2k<NP>(v, m);  // after stage 3
    fwd_2k_stage<NP, false>(v, 7, G, twA, m);
    fwd_2k_stage<NP, false>(v, 6, G, twA, m);
    if (QM == 1 && !FHE_FWD_TIGHT) red_2k<NP>(v, m);
    if (QM == 2 && FHE_FWD_TIGHT) FRED ? red_2k_f<NP>(v, m) : red_2k<NP>(v, m);  // after stage 5
#pragma unroll
    for (int p = 0; p < NP; ++p) {  // A -> B
#pragma unroll
        for (int r = 0; r < 32; ++r) ta[66 * r] = v[p][r];
        wave_lds_sync();
#pragma unroll
        for (int r = 0; r < 32; ++r) v[p][r] = tb[2 * r];
        wave_lds_sync();
    }
    fwd_2k_stage<NP, true>(v, 5, G, s_tab, m);
    if (QM == 2 && !FHE_FWD_TIGHT) FRED ? red_2k_f<NP>(v, m) : red_2k<NP>(v, m);  // after stage 6
    fwd_2k_stage<NP, true>(v, 4, G, s_tab, m);
    fwd_2k_stage<NP, true>(v, 3, G, s_tab, m);
    fwd_2k_stage<NP, true>(v, 2, G, s_tab, m);
    if (QM == 2) FRED ? red_2k_f<NP>(v, m) : red_2k<NP>(v, m);  // after stage 9
    fwd_2k_stage<NP, true>(v, 1, G, s_tab, m);
#pragma unroll
    for (int p = 0; p < NP; ++p) {  // B -> C
#pragma unroll
        for (int r = 0; r < 32; ++r) tb[2 * r] = v[p][r];
        wave_lds_sync();
#pragma unroll
        for (int rh = 0; rh < 16; ++rh) {
            const uint2 q = *reinterpret_cast<const uint2*>(tc + 132 * rh);
            v[p][2 * rh]     = q.x;
            v[p][2 * rh + 1] = q.y;
        }
        wave_lds_sync();
    }
#pragma unroll
    for (int rh = 0; rh < 16; ++rh) {
        const uint32_t w = s_tab[1024 + (rh << 6) + L];
#pragma unroll
        for (int p = 0; p < NP; ++p) ct_bf_s(v[p][2 * rh], v[p][2 * rh + 1], w, m);
    }
}

// the signed inverse's reduction plan (as InvPlanS / make_inv_plan_ww): stage st = 0 (C, register bit
// 0), 1..5 (B, register bits 0..4), 6..9 (A, register bits 0..3), 10 (the last, register bit 4); a
// transpose precedes stages 1 and 6
struct InvPlan2k {
    bool red[11][32];
    bool redT[2][32];  // before the C -> B / B -> A transpose (as InvPlanWW)
    int fin[16];
    int cost;
};
template <int BIN, int LIM>
constexpr InvPlan2k inv_plan_2k_t(int T0, int T1) {
    InvPlan2k p{};
    int B[32] = {};
    for (int r = 0; r < 32; ++r) B[r] = BIN;
    const int bits[11] = {0, 0, 1, 2, 3, 4, 0, 1, 2, 3, 4};
    int nred = 0;
    for (int st = 0; st < 11; ++st) {
        if (st == 1 || st == 6) {
            const int k = st == 1 ? 0 : 1, T = k ? T1 : T0;
            int U = 0;
            for (int r = 0; r < 32; ++r) {
                if (B[r] > T) {
                    B[r]         = 10;
                    p.redT[k][r] = true;
                    ++nred;
                }
                U = B[r] > U ? B[r] : U;
            }
            for (int r = 0; r < 32; ++r) B[r] = U;
        }
        const int bt = bits[st];
        for (int r = 0; r < 32; ++r) {
            if (r & (1 << bt)) continue;
            const int q = r | (1 << bt);
            while (B[r] + B[q] > LIM) {
                const int e = B[r] >= B[q] ? r : q;
                B[e]        = 10;
                p.red[st][e] = true;
                ++nred;
            }
            if (st == 10) {
                int f = 0;
                while ((10 << f) < B[r] + B[q]) ++f;
                p.fin[r] = f;
            }
            B[r] = B[r] + B[q];
            B[q] = 10;
        }
    }
    p.cost = 2 * nred;
    for (int r = 0; r < 16; ++r) p.cost += p.fin[r] + 1;
    return p;
}
template <int BIN, int LIM>
constexpr InvPlan2k make_inv_plan_2k() {
    InvPlan2k best = inv_plan_2k_t<BIN, LIM>(kPlanT[7], kPlanT[7]);
    for (int a = 0; a < kPlanTN; ++a)
        for (int b = 0; b < kPlanTN; ++b) {
            const InvPlan2k p = inv_plan_2k_t<BIN, LIM>(kPlanT[a], kPlanT[b]);
            if (p.cost < best.cost) best = p;
        }
    return best;
}
// signed inverse NTT, layout C (EVAL, |v| < BIN Q / 10) -> A (COEF), canonical [0, Q); the keys carry
// N^-1, so the last stage scales by TableI[1] only (w1R)
// LIM: the signed headroom in units of Q/10 (160: Q < 2^27; 80: Q < 2^28, where the last stage's
// x + y + (Q << fin) stays below 16 Q < 2^32)
template <int BIN, int LIM = 160>
FHE_DEV void inv_2k_s(uint32_t (&v)[32], uint32_t* t, int L, const uint32_t* __restrict__ twAi,
                      const uint32_t* s_tabI, uint32_t w1R, uint32_t oneR, const Mod& m) {
    constexpr InvPlan2k P = make_inv_plan_2k<BIN, LIM>();
    auto redp = [&](int st) {
#pragma unroll
        for (int r = 0; r < 32; ++r)
            if (P.red[st][r]) v[r] = smont_mul(v[r], oneR, m);
    };
    auto redt = [&](int k) {
#pragma unroll
        for (int r = 0; r < 32; ++r)
            if (P.redT[k][r]) v[r] = smont_mul(v[r], oneR, m);
    };
    auto gs = [&](uint32_t& x, uint32_t& y, uint32_t w) {
        const uint32_t s = x + y;
        y                = smont_mul(x - y, w, m);
        x                = s;
    };
    const int G = L >> 1;
    uint32_t* ta = t + wa2k(L);
    uint32_t* tb = t + wb2k(L);
    uint32_t* tc = t + wc2k(L);
    redp(0);
#pragma unroll
    for (int rh = 0; rh < 16; ++rh) gs(v[2 * rh], v[2 * rh + 1], s_tabI[1024 + (rh << 6) + L]);
    // C -> B
    redt(0);
#pragma unroll
    for (int rh = 0; rh < 16; ++rh)
        *reinterpret_cast<uint2*>(tc + 132 * rh) = make_uint2(v[2 * rh], v[2 * rh + 1]);
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < 32; ++r) v[r] = tb[2 * r];
    wave_lds_sync();
#pragma unroll
    for (int b = 1; b <= 5; ++b) {
        const int rb = b - 1;
        redp(b);
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            if (r & (1 << rb)) continue;
            gs(v[r], v[r | (1 << rb)], s_tabI[(1 << (10 - b)) + (G << (5 - b)) + (r >> b)]);
        }
    }
    // B -> A
    redt(1);
#pragma unroll
    for (int r = 0; r < 32; ++r) tb[2 * r] = v[r];
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < 32; ++r) v[r] = ta[66 * r];
    wave_lds_sync();
#pragma unroll
    for (int b = 6; b <= 9; ++b) {
        const int rb = b - 6;
        redp(b);
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            if (r & (1 << rb)) continue;
            gs(v[r], v[r | (1 << rb)], twAi[(1 << (10 - b)) + (r >> (rb + 1))]);
        }
    }
    // bit 10 (transformnat-impl.h:599-623), canonical results as inv_pass_s
    redp(10);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t x = v[r], y = v[r | 16];
        uint32_t s       = x + y + (m.Q << P.fin[r]);
#pragma unroll
        for (int f = P.fin[r]; f >= 0; --f) s = csub(s, m.Q << f);
        const uint32_t d = smont_mul(x - y, w1R, m);
        v[r]             = s;
        v[r | 16]        = min(d, d + m.Q);
    }
}
}  // namespace

// QM 2 (2^27 <= Q < 2^29, STD256 / STD256_3 with q = 2048): the forward transform reduced three times
// (fwd_2k_s), the monomial pairs centred to (-Q/2, Q/2] and the product's low word taken signed, so that
// |acc| < 2.6 Q (own wave: |lo mp.x| 2^-32 < Q/4 per column, |hi mp.y| 2^-32 < 3 ND Q^3 2^-65 < 0.07 Q,
// |acc oneR| 2^-32 < A/8, + Q/2; the partner's share without the acc term) fits the 4 Q plan
// FULL (q = 2N, STD256_4: odd monomial exponents): the table holds psi^g - 1 for g in [0, 2048] and
// psi^(g + 2048) - 1 = -(psi^g - 1) - 2 is formed on the fly, (-x - 2, -y - 2R) with 2R centred (|y'| < Q:
// |acc| < 2.93 Q, bound 30)
// QM 3 (round 5): the centred products of QM 2 for Q < 2^27 (STD256Q_3 / STD256Q_4: q = 2N, 4 digits), with QM 0's
// unreduced forward transform and 16 Q inverse plan: |D| < 11 Q + 2^(g-1), |S+-| < 44 Q^2, so each pair's hi part
// times a monomial half adds < 0.05 Q; own word < Q/2 (lo parts) + 0.09 Q + A/32 + Q/2, the partner's the same
// without A: A < 2.25 Q (bound 25)
template <int ND, int QM, bool FULL>
constexpr int kW2Bound = QM == 3 ? 25 : QM == 2 ? (FULL ? (ND == 4 ? 32 : 30) : 27) : kW2AccBound;
#ifndef FHE_N2K_QM3
#define FHE_N2K_QM3 1  // 4-digit K1w GINX at Q < 2^27 in the QM 3 class (0: QM 2, the round-4 form)
#endif
#ifndef FHE_N2K_ONEWAVE
#define FHE_N2K_ONEWAVE 0  // bit 0 / 1: the 4- / 3-digit K1w GINX forms at one wave per SIMD (512 registers)
#endif
template <int ND, bool ACCIO, int QM = 0, bool FULL = false>
__global__ void __launch_bounds__(128 * kW2Gates,
                                  (((FHE_N2K_ONEWAVE & 1) && ND == 4) || ((FHE_N2K_ONEWAVE & 2) && ND == 3)) ? 1 : 2)
    k_blind_rotate_n2k(GateArgs g, BootTables T, const uint4* __restrict__ keys, const uint16_t* __restrict__ idx,
                       const uint32_t* __restrict__ tvb, uint64_t* __restrict__ ext_a, uint64_t* __restrict__ ext_b,
                       const uint32_t* __restrict__ twAf, const uint32_t* __restrict__ twAi) {
    constexpr int kQ = 2 * ND;  // key vectors per slot pair: ND digit rows x 2 columns
    static_assert(!FULL || QM >= 2, "the full-resolution monomials need the centred (QM 2 / 3) products");
    constexpr int BIN = kW2Bound<ND, QM, FULL>, LIM = QM == 2 ? 40 : 160;
    constexpr int QF = QM == 3 ? 0 : QM;  // the forward transform's reduction class
    constexpr bool CEN = QM >= 2;         // centred monomial pairs and signed lo halves
    extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
    uint32_t* s_tab  = sm;
    uint32_t* s_tabI = sm + 2048;
    uint2* s_mono2   = reinterpret_cast<uint2*>(sm + 4096);
    uint32_t* s_tile = sm + 4096 + 2 * kW2Mono;
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) {
        s_tab[i]  = T.tabF[i];
        s_tabI[i] = T.tabI[i];
    }
    for (int i = threadIdx.x; i < kW2Mono; i += blockDim.x) {
        uint32_t mx = T.monoP[i], my = T.mono[i];
        if (CEN) {  // centred: (-Q/2, Q/2]
            mx = mx > T.Q / 2 ? mx - T.Q : mx;
            my = my > T.Q / 2 ? my - T.Q : my;
        }
        s_mono2[i] = make_uint2(mx, my);
    }

    const int wave = threadIdx.x >> 6, L = threadIdx.x & 63;
    const int c = wave & 1;  // RLWE component of this wave
    const uint32_t gslot = blockIdx.x * kW2Gates + (wave >> 1);
    const bool live = gslot < g.count;
    const uint32_t gate = live ? gslot : g.count - 1;  // spare waves shadow the last gate: every wave meets every barrier
    uint32_t* tile    = s_tile + wave * kW2Tile;
    uint32_t* partner = s_tile + (wave ^ 1) * kW2Tile;
    const Mod m0 = make_mod(T);
    const Mod& m = m0;
    __syncthreads();

    // initial accumulator (BootstrapGateCore, binfhe-base-scheme.cpp:556-575): acc1 = NTT(m), acc0 = 0
    uint32_t acc[32];
    if (ACCIO && !g.acc_tv) {
        const uint64_t* src = g.acc_io + ((size_t)gate * 2 + c) * g.N;
#pragma unroll
        for (int r = 0; r < 32; ++r) acc[r] = csub(mont_mul((uint32_t)src[slot_2k(L, r)], T.ninvR, m), m.Q);
    } else if (c == 1) {
        const uint32_t b = tvb[gate], cm = g.ctmod - 1;
        uint32_t tv[1][32];
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            const uint32_t x = ((uint32_t)r << 6) | (uint32_t)L;
            uint32_t v       = 0;
            if (x % g.factor == 0) {
                const uint32_t bx = (b - x / g.factor) & cm;
                v                 = (bx >= g.lb && bx < g.ub) ? g.lv : g.uv;
            }
            tv[0][r] = v;
        }
        fwd_2k_s<1, QF, true>(tv, tile, L, twAf, s_tab, m);
#pragma unroll
        for (int r = 0; r < 32; ++r) acc[r] = smont_mul(tv[0][r], T.ninvR, m);  // (-Q, Q), N^-1 scaled
    } else {
#pragma unroll
        for (int r = 0; r < 32; ++r) acc[r] = 0;
    }

    const uint16_t* gidx = idx + (size_t)gate * g.n;
    const DecN dec       = make_decn(m.Q, g.gbits, ND);
    // monomial of slot x(L, r): e = m (2 brv11(x) + 1) mod 2N, m = a 2N / ctmod even, in half units
    // f = e / 2 = as (32 brv6(L) + 1) + as 2 brv4(r >> 1) mod 2048 (bit 0 of x adds as 2048 = 0)
    // FULL: e = a (32 brv6(L) + 1) + a 2 brv4(r >> 1) + a 2048 (r & 1) mod 4096
    const uint32_t lmul = 32 * (__builtin_bitreverse32((uint32_t)L) >> 26) + 1;
    const uint4* kc     = keys + (size_t)c * (kQ * 16 * 64) + L;
    uint32_t two_r = 0;
    if (FULL) {
        two_r = 2 * T.oneR;
        two_r = two_r >= T.Q ? two_r - T.Q : two_r;
        two_r = two_r > T.Q / 2 ? two_r - T.Q : two_r;
    }
    // u or -u - (2, 2R) by a mask (0 or ~0): no control flow around the MAC
    auto negp = [&](uint2 u, uint32_t sm) {
        return make_uint2(((u.x ^ sm) - sm) - (2u & sm), ((u.y ^ sm) - sm) - (two_r & sm));
    };
    for (uint32_t i = 0; i < g.n; ++i) {
        const Mod m       = fresh_nq(m0);
        const uint32_t as = __builtin_amdgcn_readfirstlane((uint32_t)gidx[i]) >> (FULL ? 0 : 1);
        const uint4* kb   = kc + (size_t)i * (2 * kQ * 16 * 64);
        // the uniform twiddles re-read per index (hoisted, the 62 of them would sit in VGPRs across the loop)
        const uint32_t* twF = twAf;
        const uint32_t* twI = twAi;
        asm volatile("" : "+s"(twF), "+s"(twI));
#if FHE_N2K_OPAQUE
        // the lane index and this wave's tiles opaque per index: the per-lane LDS bases are re-derived
        // inside the body instead of being kept (spilled) across the loop
        int L_o = L;
        uint32_t *tile_o = tile, *partner_o = partner;
        asm volatile("" : "+v"(L_o), "+v"(tile_o), "+v"(partner_o));
        const int L = L_o;
        uint32_t* const tile    = tile_o;
        uint32_t* const partner = partner_o;
#endif
        constexpr int KB = ND == 4 ? 1 : FHE_N2K_KPF + 1;  // 4 digits: no registers for the key ring
        uint4 kq[KB][kQ];
        __syncthreads();  // the partner has read this wave's tile (previous index)
        uint32_t d[ND][32];
#pragma unroll
        for (int r = 0; r < 32; ++r) d[0][r] = acc[r];
        inv_2k_s<BIN, LIM>(d[0], tile, L, twI, s_tabI, T.w1R, m.oneR, m);
#pragma unroll
        for (int r = 0; r < 32; ++r) decompose_n<ND>(d[0][r], dec, d, r);
        fwd_2k_s<ND, QF, true>(d, tile, L, twF, s_tab, m);
        constexpr uint32_t EM = FULL ? 4095u : 2047u;
        const uint32_t fl = (as * lmul) & EM;
#pragma unroll
        for (int q = 0; q < kQ; ++q) kq[0][q] = kb[(q * 16 + 0) * 64];
#pragma unroll
        for (int k2 = 0; k2 < 16; ++k2) {
            if (KB == 2 && k2 + 1 < 16) {
#pragma unroll
                for (int q = 0; q < kQ; ++q) kq[(k2 + 1) % KB][q] = kb[(q * 16 + k2 + 1) * 64];
            } else if (KB == 1 && k2 > 0) {
#pragma unroll
                for (int q = 0; q < kQ; ++q) kq[0][q] = kb[(q * 16 + k2) * 64];
            }
            asm volatile("" ::: "memory");
            const uint32_t ur = __builtin_amdgcn_readfirstlane(
                (as * 2u * (__builtin_bitreverse32((uint32_t)k2) >> 28)) & EM);
            uint2 mp, mn;
            if (FULL) {
                const uint32_t e0 = (fl + ur) & 4095u, en = (4096u - e0) & 4095u;
                const uint32_t g0 = e0 & 2047u, gn = en & 2047u;
                const uint2 t0 = s_mono2[g0 + (g0 >> 5)], tn = s_mono2[gn + (gn >> 5)];
                mp = negp(t0, 0u - ((e0 >> 11) & 1u));
                mn = negp(tn, 0u - ((en >> 11) & 1u));
            } else {
                const uint32_t f = (fl + ur) & 2047u, fn = 2048u - f;
                mp = s_mono2[f + (f >> 5)];
                mn = s_mono2[fn + (fn >> 5)];
            }
            const uint4* q4 = kq[k2 % KB];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int r = 2 * k2 + e;
                if (FULL && e == 1) {  // odd a: slot r + 1 is 2048 a further
                    mp = negp(mp, 0u - (as & 1u));
                    mn = negp(mn, 0u - (as & 1u));
                }
#pragma unroll
                for (int o = 0; o < 2; ++o) {  // o = 0: this wave's component, 1: the partner's
                    int64_t S1 = 0, S2 = 0;
#pragma unroll
                    for (int j = 0; j < ND; ++j) {
                        const uint4 kv = q4[2 * j + o];
                        S1 += (int64_t)(int32_t)d[j][r] * (int32_t)(e ? kv.y : kv.x);
                        S2 += (int64_t)(int32_t)d[j][r] * (int32_t)(e ? kv.w : kv.z);
                    }
                    int64_t S;
                    if (CEN) {  // S1 = hi 2^32 + lo with lo signed
                        const int32_t l1 = (int32_t)S1, l2 = (int32_t)S2;
                        const int32_t h1 = (int32_t)((S1 - l1) >> 32), h2 = (int32_t)((S2 - l2) >> 32);
                        S = (int64_t)l1 * (int32_t)mp.x + (int64_t)h1 * (int32_t)mp.y;
                        S += (int64_t)l2 * (int32_t)mn.x + (int64_t)h2 * (int32_t)mn.y;
                    } else {
                        S = (int64_t)((uint64_t)(uint32_t)S1 * mp.x) + (int64_t)(int32_t)(S1 >> 32) * (int32_t)mp.y;
                        S += (int64_t)((uint64_t)(uint32_t)S2 * mn.x) + (int64_t)(int32_t)(S2 >> 32) * (int32_t)mn.y;
                    }
                    if (o == 0) {
                        S += (int64_t)(int32_t)acc[r] * (int32_t)T.oneR;
                        acc[r] = smont_red(S, m);
                    } else {
                        tile[(r << 6) | L] = smont_red(S, m);
                    }
                }
            }
        }
        __syncthreads();  // both waves' partner words are in LDS
#pragma unroll
        for (int r = 0; r < 32; ++r) acc[r] += partner[(r << 6) | L];
    }

    if (ACCIO) {  // every wave of the workgroup leaves here: no barrier is skipped by some only
        if (live) {
            uint64_t* dst = g.acc_io + ((size_t)gate * 2 + c) * g.N;
#pragma unroll
            for (int r = 0; r < 32; ++r) {
                const int32_t v = (int32_t)smont_mul(acc[r], T.nR, m);
                dst[slot_2k(L, r)] = (uint64_t)(uint32_t)(v < 0 ? v + (int32_t)m.Q : v);
            }
        }
        return;
    }
    // extraction (binfhe-base-scheme.cpp:110-121): canonical COEF in layout A; wave 0 writes the
    // transposed acc0 (coefficient k -> position N - k, negated), wave 1 the b term from acc1[0]
    __syncthreads();  // the partner has read this wave's tile
    inv_2k_s<BIN, LIM>(acc, tile, L, twAi, s_tabI, T.w1R, m.oneR, m);
    if (!live) return;
    if (c == 0) {
        uint64_t* oa = ext_a + (size_t)gate * g.N;
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            const uint32_t x = ((uint32_t)r << 6) | (uint32_t)L;
            const uint32_t v = acc[r];
            const uint32_t o = (x == 0 || v == 0) ? v : m.Q - v;
            oa[(g.N - x) & (g.N - 1)] = g.msb_out ? mod_switch(o, m.Q, g.qKS) : o;
        }
    } else if (L == 0) {
        const uint32_t bb = add_mod(g.b_const, acc[0], m.Q);
        ext_b[gate]       = g.msb_out ? mod_switch(bb, m.Q, g.qKS) : bb;
    }
}

bool n2k_supported(const GateArgs& g, const BootTables& t, int nd) {
    // The monomial table is full-resolution (psi^g - 1, the kernel negating past psi^2048) exactly when the set's
    // q = 2N, half-resolution (psi^(2f) - 1) otherwise (Engine::build_tables_n2k).  The full-resolution
    // instantiations (3 retained digits at 2^27 <= Q < 2^29, 4 digits) take any ciphertext modulus <= 2N; the
    // half-resolution ones need even exponents, ciphertext moduli below 2N (a seam call at 2N stays on K5).
    // 3 retained digits at Q < 2^29 (Q >= 2^27: QM 2), 2 retained digits at 2^27 <= Q < 2^29.
    const bool full = g.q == 2 * g.N;
    const bool qok = full ? (nd == 4 || (nd == 3 && t.Q >= (1u << 27))) : g.ctmod < 2 * g.N;
    const bool ndok = nd == 3 || (nd == 2 && t.Q >= (1u << 27)) || (nd == 4 && full);
    return t.Q < (1u << 29) && ndok && g.N == 2048 && qok && g.ctmod <= 2 * g.N &&
           g.tv == nullptr && g.tv64 == nullptr && g.gbits >= 2 && (uint32_t)(nd + 1) * g.gbits <= 32;
}

hipError_t launch_blind_rotate_n2k(const GateArgs& g, const BootTables& t, const void* keys, const uint16_t* idx,
                                   const uint32_t* tvb, uint64_t* ext_a, uint64_t* ext_b, int nd, hipStream_t s) {
    if (g.count == 0) return hipSuccess;
    if (!n2k_supported(g, t, nd)) return hipErrorInvalidValue;
    static const bool attr = [] {
        for (const void* k : {reinterpret_cast<const void*>(&k_blind_rotate_n2k<3, false>),
                              reinterpret_cast<const void*>(&k_blind_rotate_n2k<3, true>),
                              reinterpret_cast<const void*>(&k_blind_rotate_n2k<3, false, 2>),
                              reinterpret_cast<const void*>(&k_blind_rotate_n2k<3, true, 2>),
                              reinterpret_cast<const void*>(&k_blind_rotate_n2k<2, false, 2>),
                              reinterpret_cast<const void*>(&k_blind_rotate_n2k<2, true, 2>),
                              reinterpret_cast<const void*>(&k_blind_rotate_n2k<3, false, 2, true>),
                              reinterpret_cast<const void*>(&k_blind_rotate_n2k<3, true, 2, true>),
                              reinterpret_cast<const void*>(&k_blind_rotate_n2k<4, false, 2, true>),
                              reinterpret_cast<const void*>(&k_blind_rotate_n2k<4, true, 2, true>),
                              reinterpret_cast<const void*>(&k_blind_rotate_n2k<4, false, 3, true>),
                              reinterpret_cast<const void*>(&k_blind_rotate_n2k<4, true, 3, true>)})
            (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)w2_lds());
        return true;
    }();
    (void)attr;
    const uint32_t blocks = (g.count + kW2Gates - 1) / kW2Gates;
    const uint4* k = static_cast<const uint4*>(keys);
#define FHE_N2K(ND_, IO, QM_, ...)                                                                                 \
    hipLaunchKernelGGL((k_blind_rotate_n2k<ND_, IO, QM_, ##__VA_ARGS__>), dim3(blocks), dim3(128 * kW2Gates), w2_lds(), \
                       s, g, t, k, idx, tvb, ext_a, ext_b, t.twA_fwd, t.twA_inv)
    if (g.q == 2 * g.N) {  // full-resolution table: STD256_4 (29-bit Q, q = 2N); STD256Q_3 / STD256Q_4 (4 digits)
        if (nd == 4 && FHE_N2K_QM3 && t.Q < (1u << 27)) {  // STD256Q_3 / STD256Q_4: no forward reductions (QM 3)
            if (g.acc_io) FHE_N2K(4, true, 3, true); else FHE_N2K(4, false, 3, true);
        } else if (nd == 4) { if (g.acc_io) FHE_N2K(4, true, 2, true); else FHE_N2K(4, false, 2, true); }
        else if (g.acc_io) FHE_N2K(3, true, 2, true); else FHE_N2K(3, false, 2, true);
    } else if (t.Q < (1u << 27)) {  // STD256Q
        if (g.acc_io) FHE_N2K(3, true, 0); else FHE_N2K(3, false, 0);
    } else if (nd == 3) {  // STD256_3 (29-bit Q)
        if (g.acc_io) FHE_N2K(3, true, 2); else FHE_N2K(3, false, 2);
    } else {  // STD256 (29-bit Q, digitsG 3)
        if (g.acc_io) FHE_N2K(2, true, 2); else FHE_N2K(2, false, 2);
    }
#undef FHE_N2K
    return hipGetLastError();
}

// ===========================================================================
// K1w for LMKCDEY: k_blind_rotate_lmk2k<ACCIO> (RingGSWAccumulatorLMKCDEY::EvalAcc,
// rgsw-acc-lmkcdey.cpp:70-287) at N = 2048, Q < 2^27, digitsG = 4 (ND = 3 retained digits):
// STD256Q_LMKCDEY and STD256Q_3_LMKCDEY, which otherwise run K5's op-list form.  One gate per
// 128-thread workgroup (op lists differ per gate, so a barrier may only join the two waves of one
// gate); wave c owns component c in K1w's layout C.  Per op of k_prep_lmk_w's list:
//   EXT(i)  (AddToAccLMKCDEY, :228-254): each wave inverse-transforms its component, decomposes it into
//           its 3 digits (rows 2 j + c) and forward-transforms them, then multiplies them by both key
//           columns: the sum for its own component replaces acc_c, the other one is reduced to a word
//           per slot and handed over through this wave's tile (as K1w's GINX exchange).
//   AUTO(t) (Automorphism, :257-287): both components permuted in EVAL through the wave's tile; wave 0
//           inverse-transforms acc0', decomposes and forward-transforms it, acc0 <- sum_d D_d ak[t][d][0]
//           and hands sum_d D_d ak[t][d][1] to wave 1, which adds it to acc1'.
// Keys (Engine::pack_n2k, u32 Montgomery with N^-1 folded in), one uint4 = 4 consecutive registers:
//   ek: [i][c][q < 6][k4 < 8][64 lanes], q = 2 j + o: digit row 2 j + c, column c (o = 0) or 1 - c (o = 1);
//   ak: [t][q < 6][k4 < 8][64 lanes], q = 2 d + col.
// Bounds (Q < 2^27): |D| < 11 Q + 2^(g-1) after the forward transform, |S| < 3 (11 Q + 2^6) Q < 2^59,
// each reduced sum < 1.6 Q, acc < 3.2 Q after an exchange (the inverse plan's BIN = 33).
// ===========================================================================
namespace {
// |acc| between ops, units of Q/10: 2 (ND (11 Q + 2^(g-1)) Q 2^-32 + Q/2) for Q < 2^27; Q28 (ND = 2,
// 2^27 <= Q < 2^28, the forward transform reduced once): 2 (2 (6.82 Q) Q 2^-32 + Q/2) < 2.8 Q
// QM 2 (Q < 2^29, digits below 3 Q after the forward transform): 2 (ND 3 Q Q 2^-32 + Q/2) -> 33 (ND 3)
// FHE_FWD_TIGHT, Q28: no forward reduction, digits below 7.59 Q (see there): 2 (ND 7.59 Q Q 2^-32 + Q/2) -> 29 / 39
template <int ND, int QM>
constexpr int kL2AccBound = QM == 1 ? (FHE_FWD_TIGHT ? (ND == 3 ? 39 : 29) : (ND == 3 ? 36 : 28))
                                    : QM == 2 ? (ND == 3 ? 33 : 25) : 33;
constexpr size_t l2k_lds() { return (size_t)(2048 + 2048 + 2 * kW2Tile) * 4; }

// EVAL automorphism X -> X^k on layout C through this wave's tile (as automorphism_c at N = 1024):
// slot x(L, r) evaluates at psi^(2 brv11(x) + 1), 2 brv11(x) + 1 = 32 brv6(L) + 1 + 2048 (r & 1) +
// 2 brv4(r >> 1); the value at x moves from the slot y with 2 brv11(y) + 1 = k (2 brv11(x) + 1) mod 4N
FHE_DEV void automorphism_2k(uint32_t (&v)[32], uint32_t* t, int L, uint32_t k) {
    uint32_t* tc = t + wc2k(L);
#pragma unroll
    for (int rh = 0; rh < 16; ++rh) *reinterpret_cast<uint2*>(tc + 132 * rh) = make_uint2(v[2 * rh], v[2 * rh + 1]);
    wave_lds_sync();
    const uint32_t cl = (32u * (__builtin_bitreverse32((uint32_t)L) >> 26) + 1u) * k;
#pragma unroll
    for (int r = 0; r < 32; ++r) {
        const uint32_t sr = (2048u * (uint32_t)(r & 1) + 2u * (__builtin_bitreverse32((uint32_t)(r >> 1)) >> 28)) * k;
        const uint32_t e  = (cl + sr) & 4095u;                  // odd
        const uint32_t sx = __builtin_bitreverse32(e >> 1) >> 21;  // source slot brv11((e - 1) / 2)
        v[r] = t[sx + 2 * (sx >> 6)];
    }
    wave_lds_sync();
}

// acc_c <- (own sum), partner word <- (other sum) over ND digits and the 2 ND key vectors of kb
// (q = 2 j + o); keys one chunk of 4 registers ahead
template <int ND>
FHE_DEV void mac_2k(uint32_t (&acc)[32], const uint32_t (&d)[ND][32], const uint4* kb, uint32_t* tile, int L,
                    const Mod& m) {
    constexpr int kQ = 2 * ND;
    uint4 kq[2][kQ];
#pragma unroll
    for (int q = 0; q < kQ; ++q) kq[0][q] = kb[(q * 8 + 0) * 64];
#pragma unroll
    for (int k4 = 0; k4 < 8; ++k4) {
        if (k4 + 1 < 8) {
#pragma unroll
            for (int q = 0; q < kQ; ++q) kq[(k4 + 1) & 1][q] = kb[(q * 8 + k4 + 1) * 64];
        }
        asm volatile("" ::: "memory");
        const uint4* q4 = kq[k4 & 1];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = 4 * k4 + e;
#pragma unroll
            for (int o = 0; o < 2; ++o) {
                int64_t S = 0;
#pragma unroll
                for (int j = 0; j < ND; ++j) {
                    const uint4 kv   = q4[2 * j + o];
                    const uint32_t w = e == 0 ? kv.x : e == 1 ? kv.y : e == 2 ? kv.z : kv.w;
                    S += (int64_t)(int32_t)d[j][r] * (int32_t)w;
                }
                if (o == 0) acc[r] = smont_red(S, m);
                else tile[(r << 6) | L] = smont_red(S, m);
            }
        }
    }
}
}  // namespace

template <int ND, bool ACCIO, int QM = 0>
__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2, 2)))
    k_blind_rotate_lmk2k(GateArgs g, BootTables T, const uint4* __restrict__ ek, const uint4* __restrict__ ak,
                         const uint16_t* __restrict__ ops, const uint32_t* __restrict__ nops, uint32_t maxops,
                         const uint32_t* __restrict__ tvb, uint64_t* __restrict__ ext_a, uint64_t* __restrict__ ext_b,
                         const uint32_t* __restrict__ twAf, const uint32_t* __restrict__ twAi) {
    constexpr int kQ = 2 * ND;
    constexpr int BIN = kL2AccBound<ND, QM>, LIM = QM == 2 ? 40 : QM == 1 ? 80 : 160;
    extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
    uint32_t* s_tab  = sm;
    uint32_t* s_tabI = sm + 2048;
    uint32_t* s_tile = sm + 4096;
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) {
        s_tab[i]  = T.tabF[i];
        s_tabI[i] = T.tabI[i];
    }
    // wave c: RLWE component c.  (Giving component 0's role, the one the AUTO ops load, to the second
    // wave in half the workgroups was measured 1.7% slower: profiles/r04_lmk2k_swap_ab.txt)
    const int c = threadIdx.x >> 6, L = threadIdx.x & 63;
    const uint32_t gate = blockIdx.x;
    uint32_t* tile    = s_tile + c * kW2Tile;
    uint32_t* partner = s_tile + (c ^ 1) * kW2Tile;
    const Mod m0 = make_mod(T);
    const Mod& m = m0;
    const uint32_t M = 2 * g.N;
    __syncthreads();

    // BootstrapGateCore (binfhe-base-scheme.cpp:556-575): acc1 = NTT(m), acc0 = 0; then
    // acc1 <- acc1(X^(2N-5)) (rgsw-acc-lmkcdey.cpp:99; acc0 = 0 is invariant)
    uint32_t acc[32];
    if (ACCIO && !g.acc_tv) {
        const uint64_t* src = g.acc_io + ((size_t)gate * 2 + c) * g.N;
#pragma unroll
        for (int r = 0; r < 32; ++r) acc[r] = csub(mont_mul((uint32_t)src[slot_2k(L, r)], T.ninvR, m), m.Q);
        if (c == 1) automorphism_2k(acc, tile, L, M - 5);
    } else if (c == 1) {
        const uint32_t b = tvb[gate], cm = g.ctmod - 1;
        uint32_t tv[1][32];
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            const uint32_t x = ((uint32_t)r << 6) | (uint32_t)L;
            uint32_t v       = 0;
            if (x % g.factor == 0) {
                const uint32_t bx = (b - x / g.factor) & cm;
                v                 = (bx >= g.lb && bx < g.ub) ? g.lv : g.uv;
            }
            tv[0][r] = v;
        }
        fwd_2k_s<1, QM>(tv, tile, L, twAf, s_tab, m);
#pragma unroll
        for (int r = 0; r < 32; ++r) acc[r] = smont_mul(tv[0][r], T.ninvR, m);  // (-Q, Q), N^-1 scaled
        automorphism_2k(acc, tile, L, M - 5);
    } else {
#pragma unroll
        for (int r = 0; r < 32; ++r) acc[r] = 0;
    }

    const DecN dec       = make_decn(m.Q, g.gbits, ND);
    const uint16_t* gops = ops + (size_t)gate * maxops;
    const uint32_t cnt   = __builtin_amdgcn_readfirstlane(nops[gate]);
    for (uint32_t it = 0; it < cnt; ++it) {
        const Mod m       = fresh_nq(m0);
        const uint32_t op = __builtin_amdgcn_readfirstlane((uint32_t)gops[it]);
        const uint32_t* twF = twAf;
        const uint32_t* twI = twAi;
        asm volatile("" : "+s"(twF), "+s"(twI));
        __syncthreads();  // the partner has read this wave's tile (previous op)
        // ---- AddToAccLMKCDEY (op < 0x8000): acc_c <- sum over both components' digits of D ek[op][row][c];
        // ---- Automorphism(5^t or 2N - 5, ak[t]) (op = 0x8000 | t): acc0' -> COEF -> digits -> EVAL,
        // acc0 replaced, acc1's share to the tile.  One copy of the digit path serves both (the two copies
        // put the digit array of the 3-digit, 29-bit form in scratch)
        const bool isauto = op & 0x8000u;
        const uint32_t t  = op & 0x7fffu;
        if (isauto) {
            uint32_t kexp = M - 5;
            if (t) {
                kexp = 1;
                for (uint32_t z = 0; z < t; ++z) kexp = (kexp * 5u) & (M - 1);
            }
            automorphism_2k(acc, tile, L, kexp);
        }
        if (!isauto || c == 0) {
            uint32_t d[ND][32];
#pragma unroll
            for (int r = 0; r < 32; ++r) d[0][r] = acc[r];
            inv_2k_s<BIN, LIM>(d[0], tile, L, twI, s_tabI, T.w1R, m.oneR, m);
#pragma unroll
            for (int r = 0; r < 32; ++r) decompose_n<ND>(d[0][r], dec, d, r);
            fwd_2k_s<ND, QM>(d, tile, L, twF, s_tab, m);
            const uint4* key = isauto ? ak + (size_t)t * (kQ * 8 * 64) : ek + ((size_t)op * 2 + c) * (kQ * 8 * 64);
            mac_2k<ND>(acc, d, key + L, tile, L, m);
        }
        __syncthreads();  // the partner words (AddToAcc: both waves'; Automorphism: wave 0's share of acc1)
        if (!isauto) {
#pragma unroll
            for (int r = 0; r < 32; ++r) acc[r] += partner[(r << 6) | L];
        } else if (c == 1) {
#pragma unroll
            for (int r = 0; r < 32; ++r) {
                const int64_t S = (int64_t)(int32_t)acc[r] * (int32_t)m.oneR +
                                  (int64_t)(int32_t)partner[(r << 6) | L] * (int32_t)m.oneR;
                acc[r] = smont_red(S, m);
            }
        }
    }

    if (ACCIO) {
        uint64_t* dst = g.acc_io + ((size_t)gate * 2 + c) * g.N;
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            const int32_t v = (int32_t)smont_mul(acc[r], T.nR, m);
            dst[slot_2k(L, r)] = (uint64_t)(uint32_t)(v < 0 ? v + (int32_t)m.Q : v);
        }
        return;
    }
    // extraction (binfhe-base-scheme.cpp:110-121), as k_blind_rotate_n2k
    __syncthreads();  // the partner has read this wave's tile
    inv_2k_s<BIN, LIM>(acc, tile, L, twAi, s_tabI, T.w1R, m.oneR, m);
    if (c == 0) {
        uint64_t* oa = ext_a + (size_t)gate * g.N;
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            const uint32_t x = ((uint32_t)r << 6) | (uint32_t)L;
            const uint32_t v = acc[r];
            const uint32_t o = (x == 0 || v == 0) ? v : m.Q - v;
            oa[(g.N - x) & (g.N - 1)] = g.msb_out ? mod_switch(o, m.Q, g.qKS) : o;
        }
    } else if (L == 0) {
        const uint32_t bb = add_mod(g.b_const, acc[0], m.Q);
        ext_b[gate]       = g.msb_out ? mod_switch(bb, m.Q, g.qKS) : bb;
    }
}

bool lmk2k_supported(const GateArgs& g, const BootTables& t, int nd) {
    // 2 or 3 retained digits, Q < 2^29 (the forward transform reduced once at Q >= 2^27, three times at
    // Q >= 2^28); 4 digits (STD256Q_4_LMKCDEY) at Q < 2^27.  (The 4-digit form first ran at 1.07K gates/s
    // against 10.6K on K5, profiles/r04_ext_bench.txt: its digit array sat in scratch, the forward stage
    // loop left rolled; the stages are now written out.)
    const bool qok = nd == 4 ? t.Q < (1u << 27) : t.Q < (1u << 29);
    return qok && g.N == 2048 && g.tv == nullptr && g.tv64 == nullptr && g.gbits >= 2 && nd >= 2 && nd <= 4 &&
           (uint32_t)(nd + 1) * g.gbits <= 32;
}

hipError_t launch_blind_rotate_lmk2k(const GateArgs& g, const BootTables& t, const void* ek, const void* ak,
                                     const uint16_t* ops, const uint32_t* nops, uint32_t maxops, const uint32_t* tvb,
                                     uint64_t* ext_a, uint64_t* ext_b, int nd, hipStream_t s) {
    if (g.count == 0) return hipSuccess;
    if (!lmk2k_supported(g, t, nd)) return hipErrorInvalidValue;
    const uint4* e = static_cast<const uint4*>(ek);
    const uint4* a = static_cast<const uint4*>(ak);
#define FHE_L2K(ND_, IO, QM_)                                                                                      \
    hipLaunchKernelGGL((k_blind_rotate_lmk2k<ND_, IO, QM_>), dim3(g.count), dim3(128), l2k_lds(), s, g, t, e, a, ops,  \
                       nops, maxops, tvb, ext_a, ext_b, t.twA_fwd, t.twA_inv)
    const int qm = t.Q >= (1u << 28) ? 2 : t.Q >= (1u << 27) ? 1 : 0;  // the modulus class (fwd_2k_s)
    if (nd == 2) {  // STD256Q_LMKCDEY (28-bit Q)
        if (qm == 1) { if (g.acc_io) FHE_L2K(2, true, 1); else FHE_L2K(2, false, 1); }
        else if (qm == 2) { if (g.acc_io) FHE_L2K(2, true, 2); else FHE_L2K(2, false, 2); }
        else { if (g.acc_io) FHE_L2K(2, true, 0); else FHE_L2K(2, false, 0); }
    } else if (nd == 4) {  // STD256Q_4_LMKCDEY (digitsG 5)
        if (g.acc_io) FHE_L2K(4, true, 0); else FHE_L2K(4, false, 0);
    } else {  // STD256Q_3_LMKCDEY (26-bit); STD256_3 / _4_LMKCDEY (29-bit)
        if (qm == 0) { if (g.acc_io) FHE_L2K(3, true, 0); else FHE_L2K(3, false, 0); }
        else if (qm == 1) { if (g.acc_io) FHE_L2K(3, true, 1); else FHE_L2K(3, false, 1); }
        else { if (g.acc_io) FHE_L2K(3, true, 2); else FHE_L2K(3, false, 2); }
    }
#undef FHE_L2K
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// ExternalProduct seam (Backend::ExternalProduct[Batch], backend.h:141-146, 187-192): per-item
// RGSW keys in the reference's raw EVAL layout [dG2 = 4][2][N] packed into the op-list kernel's
// resident layout (the layout Engine::load_bsk writes), then one EXT op per item.
// ---------------------------------------------------------------------------
__global__ void k_pack_rgsw(const uint64_t* __restrict__ raw, uint32_t count, uint32_t N, uint32_t Q,
                            uint32_t ninv_mont, uint32_t* __restrict__ out) {
    // ninv_mont = N^-1 2^32 mod Q: out = raw N^-1 2^32 mod Q (Montgomery form of raw N^-1)
    const uint64_t words = (uint64_t)count * 4 * 2 * N;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < words; t += (uint64_t)gridDim.x * blockDim.x) {
        // t enumerates destination words of key g: (d, k, lane, e) in row_off order
        const uint64_t g = t / (8 * N), w = t % (8 * N);
        // (((d * 8 + k/2) * 64 + lane) * 4 + (k & 1) * 2 + e
        const uint32_t q4 = (uint32_t)(w >> 2), sub = (uint32_t)(w & 3);
        const uint32_t lane = q4 & 63, dk = q4 >> 6;
        const uint32_t d = dk >> 3, k = ((dk & 7) << 1) | (sub >> 1), e = sub & 1;
        const uint32_t h = lane >> 5, l = lane & 31;
        const uint32_t row = kBskHalfSwap ? d ^ h : d;
        const uint64_t src = raw[g * 8 * N + ((uint64_t)row * 2 + h) * N + l * 32 + 2 * k + e];
        out[g * 8 * N + row_off(d, k, lane, e)] = (uint32_t)((src % Q) * ninv_mont % Q);
    }
}

__global__ void k_single_ops(uint16_t* __restrict__ ops, uint32_t* __restrict__ nops, uint32_t count, uint32_t maxops) {
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < count; g += gridDim.x * blockDim.x) {
        ops[(size_t)g * maxops] = (uint16_t)g;
        nops[g] = 1;
    }
}

hipError_t launch_pack_rgsw(const uint64_t* raw, size_t count, uint32_t N, uint32_t Q, uint32_t ninv_mont,
                            uint32_t* out, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (N != 1024 || count > 0x7fffffffull) return hipErrorInvalidValue;
    const uint64_t words = (uint64_t)count * 8 * N;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((words + 255) / 256, 8192);
    hipLaunchKernelGGL(k_pack_rgsw, dim3(blocks), dim3(256), 0, s, raw, (uint32_t)count, N, Q, ninv_mont, out);
    return hipGetLastError();
}

hipError_t launch_single_ops(uint16_t* ops, uint32_t* nops, uint32_t count, uint32_t maxops, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (count > 0x8000u) return hipErrorInvalidValue;   // op codes: key index < 0x8000
    hipLaunchKernelGGL(k_single_ops, dim3((count + 255) / 256), dim3(256), 0, s, ops, nops, count, maxops);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// ModSwitch on u64 vectors (standalone entry point)
// ---------------------------------------------------------------------------
// RoundqQ exactly as the reference writes it (lwe-pke.cpp:41-46): IEEE double, the product divided
// before the add (no contraction).  Any moduli: the GPU's double divide is correctly rounded.
FHE_DEV uint64_t round_qQ_double(uint64_t v, uint64_t to, uint64_t from) {
#pragma clang fp contract(off)
    const double x = (double)v * (double)to / (double)from;
    return (uint64_t)floor(0.5 + x) % to;
}

__global__ void k_modswitch(uint64_t from, uint64_t to, uint32_t len, uint32_t count, const uint64_t* __restrict__ a,
                            const uint64_t* __restrict__ b, uint64_t* __restrict__ ao, uint64_t* __restrict__ bo) {
    const uint64_t total = (uint64_t)len * count;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x)
        ao[t] = round_qQ_double(a[t], to, from);
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < count; t += (uint64_t)gridDim.x * blockDim.x)
        bo[t] = round_qQ_double(b[t], to, from);
}

hipError_t launch_modswitch(uint64_t q_from, uint64_t q_to, uint32_t len, uint32_t count, const uint64_t* a,
                            const uint64_t* b, uint64_t* a_out, uint64_t* b_out, hipStream_t s) {
    if (count == 0) return hipSuccess;
    const uint64_t total = (uint64_t)len * count;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(k_modswitch, dim3(blocks), dim3(256), 0, s, q_from, q_to, len, count, a, b, a_out, b_out);
    return hipGetLastError();
}

}  // namespace fhe_amd
