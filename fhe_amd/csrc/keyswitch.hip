// keyswitch.hip -- LWE key switching (LWEEncryptionScheme::KeySwitch,
// src/binfhe/lib/lwe-pke.cpp:348-372) fused with the final ModSwitch(qKS -> q)
// (:254-261) of SwitchCTtoqn (:170-178).
//
// out = (0, b) - sum_{i<N, j<digitsKS} KSK[i][digit_j(a_i)][j]   (mod qKS)
// One workgroup per ciphertext; thread t owns columns 2t, 2t+1 of the
// (n+1)-wide rows (A row + B stored at column n, u16, padded to 512).  Each
// of the N*digitsKS row gathers is one fully coalesced 1 KiB read.  qKS is a
// power of two (2^14 in both STD128 sets), so the row sums are accumulated in
// plain u32 (3072 * 2^14 < 2^32) and reduced once.
#include "arith.h"
#include "boot.h"

#include <algorithm>
#include <type_traits>

namespace fhe_amd {

namespace {
// the reference's RoundqQ expression itself (lwe-pke.cpp:41-46): IEEE double, no contraction
FHE_DEV uint64_t round_qQ_ref(uint64_t v, uint64_t q, uint64_t Q) {
#pragma clang fp contract(off)
    const double x = (double)v * (double)q / (double)Q;
    return (uint64_t)floor(0.5 + x) % q;
}
// RoundqQ(v, q_out, qKS) = floor(0.5 + v q_out / qKS) mod q_out (lwe-pke.cpp:41-46).  qKS is a power
// of two, so while qKS q_out <= 2^52 every step of the double expression is exact (the product
// v q_out < 2^52, the division by 2^k, and the add of 0.5 to a value with < 2^52 units of 2^-k)
// and it equals the integer floor((2 v q_out + qKS) / (2 qKS)).  Larger q_out (BootstrapFunc's
// fmod can reach 2^40) take the reference's double expression itself.  q_out is uniform.
FHE_DEV uint64_t mod_switch_up(uint64_t v, uint32_t qKS, uint64_t q_out) {
    if ((unsigned __int128)qKS * q_out <= ((unsigned __int128)1 << 52))
        return ((2 * v * q_out + qKS) / (2 * (uint64_t)qKS)) % q_out;
    return round_qQ_ref(v, q_out, qKS);
}
}  // namespace

__global__ void __launch_bounds__(512)
    k_keyswitch(GateArgs g, uint32_t logBase, uint32_t digitsKS, const uint32_t* __restrict__ ksk,
                const uint32_t* __restrict__ ms_a, const uint32_t* __restrict__ ms_b, uint64_t q_out,
                uint64_t* __restrict__ a_out, uint64_t* __restrict__ b_out) {
    __shared__ uint32_t s_a[2048];
    const uint32_t gate = blockIdx.x, t = threadIdx.x;
    for (uint32_t i = t; i < g.N; i += blockDim.x) s_a[i] = ms_a[(size_t)gate * g.N + i];
    __syncthreads();
    const uint32_t base = 1u << logBase, mask = base - 1;
    const uint32_t rw = blockDim.x;   // u32 words per row = ksk_width(n) / 2
    uint32_t lo = 0, hi = 0;
#pragma unroll 4
    for (uint32_t i = 0; i < g.N; ++i) {
        const uint32_t ai = s_a[i];
        for (uint32_t j = 0; j < digitsKS; ++j) {
            const uint32_t dig = (ai >> (logBase * j)) & mask;
            const uint32_t row = (i * base + dig) * digitsKS + j;
            const uint32_t w   = ksk[(size_t)row * rw + t];
            lo += w & 0xffffu;
            hi += w >> 16;
        }
    }
    const uint32_t qm = g.qKS - 1;
    const uint32_t c0 = 2 * t, c1 = 2 * t + 1;
    const uint32_t b  = ms_b[gate];
    uint64_t v0 = ((c0 == g.n ? b : 0u) - lo) & qm;
    uint64_t v1 = ((c1 == g.n ? b : 0u) - hi) & qm;
    if (q_out) {  // ModSwitch qKS -> q_out
        v0 = mod_switch_up(v0, g.qKS, q_out);
        v1 = mod_switch_up(v1, g.qKS, q_out);
    }
    uint64_t* oa = a_out + (size_t)gate * g.n;
    if (c0 < g.n) oa[c0] = v0;
    else if (c0 == g.n) b_out[gate] = v0;
    if (c1 < g.n) oa[c1] = v1;
    else if (c1 == g.n) b_out[gate] = v1;
}

// ---------------------------------------------------------------------------
// Gate-tiled key switch: a workgroup handles G gates x 64 columns.  For each
// (i, j) the 32 candidate row slices KSK[i][0..31][j][cols] (32 x 128 B) are
// staged in LDS once and every gate (one thread) subtracts the slice its digit
// selects.  KSK gather traffic drops from 3 MB per gate to 12.6 MB per 256
// gates; accumulation is packed u16 (v_pk_sub_u16: mod 2^16, hence exact mod
// qKS = 2^14) with two columns per VGPR.  baseKS = 32 or 64 and digitsKS = 3 are
// compile-time (KsShape); at baseKS 32 a round covers 4 values of i (12 steps), so
// the gate's a_i come as one 16-byte load per round, prefetched two rounds
// ahead (a dependent a_i load per i was the kernel's critical path).
// Below 4096 gates the per-gate kernel above fills the chip better.
// ---------------------------------------------------------------------------
// two independent u16 subtractions (mod 2^16) in one VALU op
__device__ __forceinline__ uint32_t pk_sub_u16(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_pk_sub_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

#ifndef FHE_KS_COLS
#define FHE_KS_COLS 64  // 32: twice the workgroups, half the columns each (measured: 7% slower)
#endif
constexpr int kKsCols  = FHE_KS_COLS;           // columns per workgroup (packed u32 pairs)
#ifndef FHE_KS_B64
#define FHE_KS_B64 1
#endif
// LDS bytes per staged slice.  FHE_KS_B64: 136 B, read as 8-byte pieces: slice d's piece k sits in
// 8-byte bank slot (17 d + k) mod 32, distinct for all 32 slices, so the random per-gate slice
// choices never conflict (16-byte reads with a 144-B stride collide for slices d, d + 16).
// Tile shapes (G gates per workgroup, IPR values of i per round at baseKS = 32), by batch size
// (round 3, profiles/archive/r03_ab_keyswitch.txt, per launch at 65,536 / 8192 / 1024 gates):
//   G 256, IPR 4 (104 KB of LDS, one workgroup per CU):       6.64 ms / 0.82 ms / 125 + 11 us
//   G 512, IPR 4:                                              4.58 ms / 0.95 ms /  79 + 11 us
//   G 512, IPR 2 (52 KB: several workgroups per CU):           3.27 ms / 1.12 ms /  73 + 20 us
// and at 16,384 gates 1.70 ms (G 256, IPR 4) vs 1.23 ms (G 512, IPR 2); so the row split (below 4096
// gates) runs G 512 / IPR 4, kKsWideBatch gates and more G 512 / IPR 2, and the batches between them
// G 256 / IPR 4 (enough workgroups to fill the chip).
constexpr int kKsIPR = 4;                 // values of i per round (4: one uint4 of a_i) at baseKS = 32
#ifndef FHE_KS_WIDE_BATCH
#define FHE_KS_WIDE_BATCH 16384
#endif
constexpr uint32_t kKsWideBatch = FHE_KS_WIDE_BATCH;  // from here: G 512, IPR 2
constexpr int kKsSplitG = 512;
#ifndef FHE_KS_XCD
#define FHE_KS_XCD 0
#endif
#ifndef FHE_KS_G1024
#define FHE_KS_G1024 0  // A/B: 1024-thread workgroups with one gate per thread from 32,768 gates (baseKS 32)
#endif
#ifndef FHE_KS_GPT
#define FHE_KS_GPT 1  // gates per thread of the 512-thread tiles (1: 512-gate tiles)
#endif            // the row split's gate tile
// BASE = baseKS: 32 (STD128, STD128Q, LPF_STD128: 32 staged slices per step) or 64 (STD128_3/4,
// LPF_STD128Q, STD256Q_3_LMKCDEY: 64 slices, 2 values of i per round so that the double buffer keeps the
// same 104 KB; slices d and d + 32 share a bank slot, a 2-way conflict), both with KD = digitsKS = 3; or
// 16 with KD = 4 (STD256Q: baseKS 16, qKS 2^16; 2 values of i per round, 35 KB)
// W32: u32 rows and u32 column sums (exact mod any power-of-two qKS <= 2^32: STD192Q_4, STD256Q_4,
// STD256Q_4_LMKCDEY), one value of i per round, 264-byte slices (8-byte piece k of slice d in bank slot
// (d + k) mod 32)
// BASE 21 with KD = 4 (STD256Q_3: qKS 2^16): 21 staged slices, digits by division (ks_digit), 2 values of i per
// round (24 KB per buffer)
template <int BASE, int IPR, int KD = 3, bool W32 = false> struct KsShape {
    static constexpr int base  = BASE;
    static constexpr int eb    = W32 ? 4 : 2;                     // bytes per KSK element
    static constexpr int ipr   = W32 ? 1 : BASE == 32 ? IPR : 2;
    static constexpr int step  = ipr * KD;                        // (i, j) steps per round / LDS buffer / barrier
    static constexpr int rowb  = kKsCols * eb + (W32 || FHE_KS_B64 ? 8 : 16);  // LDS bytes per staged slice
    static constexpr int pps   = kKsCols * eb / 16;               // 16-byte parts per slice
    static constexpr int parts = base * pps;                      // 16-byte parts staged per step
};

// Row split (blockIdx.z, small batches): a workgroup sums the rounds [z R/S, (z+1) R/S) only and
// writes its packed partial sums to part [S][count][W/2]; k_keyswitch_reduce adds the S partials
// (mod 2^16 per column, as the sums themselves) and applies the epilogue.  Below 4096 gates the
// 256-gate tiles alone leave the chip idle; split S ways they fill it while every KSK slice is still
// staged once per gate tile (the per-gate kernel re-reads 3 MB of rows per ciphertext).
// GPT: gates per thread (u16 rows, no row split): a workgroup's tile is G GPT gates, so every staged KSK
// slice serves GPT times as many gates (KSK traffic / GPT); thread t owns gates t, t + G, ...
// digit j of a (base BASE, the reference's a0 = atmp % baseKS; atmp /= baseKS, lwe-pke.cpp:362-364): a bit
// field for a power-of-two base, a division by the constant BASE^j otherwise
template <int BASE>
FHE_DEV uint32_t ks_digit(uint32_t a, int j) {
    if ((BASE & (BASE - 1)) == 0) return (a >> (__builtin_ctz(BASE) * j)) & (BASE - 1);
    uint32_t p = 1;
    for (int k = 0; k < j; ++k) p *= BASE;
    return (a / p) % BASE;
}

// PRIME (with W32): a prime qKS (TOY, SIGNED_MOD_TEST: modKS = PRIME, qKS = Q < 2^28, baseKS 25): the column
// sums are kept in [0, qKS) by one conditional add per subtraction (min(d, d + qKS) on the unsigned words) instead of
// wrapping mod 2^32, and the epilogue adds b mod qKS
template <int G, bool SPLIT, int BASE, int IPR, int KD = 3, bool W32 = false, int GPT = 1, bool PRIME = false>
__global__ void __launch_bounds__(G)
    k_keyswitch_tiled(GateArgs g, const void* __restrict__ ksk, const uint32_t* __restrict__ ms_a,
                      const uint32_t* __restrict__ ms_b, uint64_t q_out, uint64_t* __restrict__ a_out,
                      uint64_t* __restrict__ b_out, uint32_t* __restrict__ part) {
    using S_ = KsShape<BASE, IPR, KD, W32>;
    constexpr int kKsDigits = KD;
    constexpr int kKsParts = S_::parts, kKsStep = S_::step, kIPR = S_::ipr, kBase = S_::base;
    constexpr int kRowB = S_::rowb, kPps = S_::pps, kEB = S_::eb;
    constexpr int kAcc = W32 ? kKsCols : kKsCols / 2;  // u32 sums, or packed u16 pairs
    static_assert(GPT == 1 || (!SPLIT && !W32 && FHE_KS_B64), "GPT > 1: the u16, single-pass form");
    static_assert(!PRIME || W32, "a prime qKS needs u32 sums");
    const uint32_t qks = g.qKS;
    static_assert(kKsParts % G == 0 || kKsParts < G, "staging split");
    constexpr int P = kKsParts >= G ? kKsParts / G : 1;  // parts per thread per step
    __shared__ __attribute__((aligned(16))) unsigned char s_buf[2][kKsStep][kBase * kRowB];
    const uint32_t t = threadIdx.x;
    // FHE_KS_XCD: workgroups are dispatched round-robin over the 8 XCDs by linear id, so with the
    // 8 column tiles of a 512-column KSK mapped to (linear id mod 8) every XCD stages one column
    // tile only and its workgroups share each staged slice through that XCD's L2
    uint32_t bx = blockIdx.x, by = blockIdx.y;
    if (FHE_KS_XCD && !SPLIT && gridDim.y == 8) {
        const uint32_t lin = blockIdx.x + blockIdx.y * gridDim.x;
        by = lin & 7u;
        bx = lin >> 3;
    }
    const uint32_t col0 = by * kKsCols;
    const uint32_t rounds = SPLIT ? g.N / kIPR / gridDim.z : g.N / kIPR;  // this workgroup's share
    const uint32_t r0 = SPLIT ? blockIdx.z * rounds : 0;
    using AV = typename std::conditional<kIPR == 4, uint4, typename std::conditional<kIPR == 2, uint2, uint32_t>::type>::type;
    static_assert(kIPR == 4 || kIPR == 2 || kIPR == 1, "a_i vector width");
    uint32_t gates[GPT];
    const AV* ga4[GPT];
#pragma unroll
    for (int u = 0; u < GPT; ++u) {
        gates[u] = (bx * GPT + u) * G + t;
        ga4[u]   = reinterpret_cast<const AV*>(ms_a + (size_t)(gates[u] < g.count ? gates[u] : 0) * g.N) + r0;
    }
    const uint32_t gate = gates[0];
    const bool valid = gate < g.count;

    // staging role: part x = t + G*r -> slice x / kPps, 16-byte part x % kPps
    auto slice_src = [&](uint32_t round, int q, int r) -> const uint4* {
        const uint32_t x = t + G * r, sd = x / kPps, sp = x % kPps;
        const uint32_t i = (r0 + round) * kIPR + q / kKsDigits, j = q % kKsDigits;
        const size_t row = ((size_t)i * kBase + sd) * kKsDigits + j;
        return reinterpret_cast<const uint4*>(static_cast<const unsigned char*>(ksk) +
                                              (row * ksk_width(g.n) + col0) * kEB) + sp;
    };
    auto slice_dst = [&](unsigned char* sb, int r) -> unsigned char* {
        const uint32_t x = t + G * r;
        return sb + (x / kPps) * kRowB + (x % kPps) * 16;
    };
    auto put = [&](unsigned char* dst, const uint4& v) {
        if (FHE_KS_B64) {  // 8-byte aligned only
            reinterpret_cast<uint2*>(dst)[0] = make_uint2(v.x, v.y);
            reinterpret_cast<uint2*>(dst)[1] = make_uint2(v.z, v.w);
        } else {
            *reinterpret_cast<uint4*>(dst) = v;
        }
    };

    uint32_t accs[GPT][kAcc];
#pragma unroll
    for (int u = 0; u < GPT; ++u)
#pragma unroll
        for (int k = 0; k < kAcc; ++k) accs[u][k] = 0;
    uint32_t (&acc)[kAcc] = accs[0];

    uint4 st[kKsStep][P];
    // threads past kKsParts (narrow column tiles) stage nothing: their slice index would run past
    // the KSK rows of this i
    const bool stager = kKsParts >= G || (int)t < kKsParts;
#pragma unroll
    for (int q = 0; q < kKsStep; ++q)
#pragma unroll
        for (int r = 0; r < P; ++r)
            if (stager) st[q][r] = *slice_src(0, q, r);
    AV a0[GPT], a1[GPT], a2[GPT];
#pragma unroll
    for (int u = 0; u < GPT; ++u) {
        a0[u] = ga4[u][0];
        a1[u] = ga4[u][rounds > 1 ? 1 : 0];
        a2[u] = ga4[u][rounds > 2 ? 2 : 0];
    }

    // one barrier per round: buffer buf is rewritten two rounds later, after every thread
    // has passed the next round's barrier (and so finished consuming it)
    for (uint32_t rd = 0, buf = 0; rd < rounds; ++rd, buf ^= 1) {
#pragma unroll
        for (int q = 0; q < kKsStep; ++q)
#pragma unroll
            for (int r = 0; r < P; ++r)
                if (stager) put(slice_dst(s_buf[buf][q], r), st[q][r]);
        __syncthreads();
        if (rd + 1 < rounds) {
#pragma unroll
            for (int q = 0; q < kKsStep; ++q)
#pragma unroll
                for (int r = 0; r < P; ++r)
                    if (stager) st[q][r] = *slice_src(rd + 1, q, r);
        }
        AV avs[GPT];
#pragma unroll
        for (int u = 0; u < GPT; ++u) {
            avs[u] = a0[u];
            a0[u]  = a1[u];
            a1[u]  = a2[u];
            if (rd + 3 < rounds) a2[u] = ga4[u][rd + 3];
        }
        if (GPT > 1) {
#pragma unroll
            for (int q = 0; q < kKsStep; ++q)
#pragma unroll
                for (int u = 0; u < GPT; ++u) {
                    const uint32_t* as = reinterpret_cast<const uint32_t*>(&avs[u]);
                    const uint32_t dig = ks_digit<kBase>(as[q / kKsDigits], q % kKsDigits);
                    const uint2* src = reinterpret_cast<const uint2*>(s_buf[buf][q] + dig * kRowB);
                    uint2 w[kKsCols / 4];
#pragma unroll
                    for (int k = 0; k < kKsCols / 4; ++k) {
                        w[k] = src[k];
                        asm volatile("" ::: "memory");
                    }
#pragma unroll
                    for (int k = 0; k < kKsCols / 4; ++k) {
                        accs[u][2 * k + 0] = pk_sub_u16(accs[u][2 * k + 0], w[k].x);
                        accs[u][2 * k + 1] = pk_sub_u16(accs[u][2 * k + 1], w[k].y);
                    }
                }
            continue;
        }
        const uint32_t* as = reinterpret_cast<const uint32_t*>(&avs[0]);
#pragma unroll
        for (int q = 0; q < kKsStep; ++q) {
            const uint32_t dig = ks_digit<kBase>(as[q / kKsDigits], q % kKsDigits);
            if (W32) {  // u32 columns: 32 8-byte pieces, one v_sub_u32 per column
                const uint2* src = reinterpret_cast<const uint2*>(s_buf[buf][q] + dig * kRowB);
                uint2 w[kKsCols / 2];
#pragma unroll
                for (int k = 0; k < kKsCols / 2; ++k) {
                    w[k] = src[k];
                    asm volatile("" ::: "memory");
                }
#pragma unroll
                for (int k = 0; k < kKsCols / 2; ++k) {
                    if (PRIME) {  // acc, w < qKS: acc - w in (-qKS, qKS), brought back to [0, qKS)
                        const uint32_t d0 = acc[2 * k + 0] - w[k].x, d1 = acc[2 * k + 1] - w[k].y;
                        acc[2 * k + 0] = min(d0, d0 + qks);
                        acc[2 * k + 1] = min(d1, d1 + qks);
                    } else {
                        acc[2 * k + 0] -= w[k].x;
                        acc[2 * k + 1] -= w[k].y;
                    }
                }
            } else if (FHE_KS_B64) {
                const uint2* src = reinterpret_cast<const uint2*>(s_buf[buf][q] + dig * kRowB);
                uint2 w[kKsCols / 4];
#pragma unroll
                for (int k = 0; k < kKsCols / 4; ++k) {
                    w[k] = src[k];
                    // no ds_read2_b64 merge: its 16-lane groups bank mod 32, where slices d and
                    // d + 16 collide again
                    asm volatile("" ::: "memory");
                }
#pragma unroll
                for (int k = 0; k < kKsCols / 4; ++k) {
                    acc[2 * k + 0] = pk_sub_u16(acc[2 * k + 0], w[k].x);
                    acc[2 * k + 1] = pk_sub_u16(acc[2 * k + 1], w[k].y);
                }
            } else {
                const uint4* src = reinterpret_cast<const uint4*>(s_buf[buf][q] + dig * kRowB);
#pragma unroll
                for (int k = 0; k < kKsCols / 8; ++k) {
                    const uint4 w = src[k];
                    acc[4 * k + 0] = pk_sub_u16(acc[4 * k + 0], w.x);
                    acc[4 * k + 1] = pk_sub_u16(acc[4 * k + 1], w.y);
                    acc[4 * k + 2] = pk_sub_u16(acc[4 * k + 2], w.z);
                    acc[4 * k + 3] = pk_sub_u16(acc[4 * k + 3], w.w);
                }
            }
        }
    }
    if (GPT > 1) {
        const uint32_t qm = g.qKS - 1;
#pragma unroll
        for (int u = 0; u < GPT; ++u) {
            if (gates[u] >= g.count) continue;
            const uint32_t b = ms_b[gates[u]];
            uint64_t* oa = a_out + (size_t)gates[u] * g.n;
#pragma unroll
            for (int k = 0; k < kKsCols / 2; ++k) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint32_t c = col0 + 2 * k + h;
                    const uint32_t neg = h ? (accs[u][k] >> 16) : (accs[u][k] & 0xffffu);
                    uint64_t v = ((c == g.n ? b : 0u) + neg) & qm;
                    if (q_out) v = mod_switch_up(v, g.qKS, q_out);
                    if (c < g.n) oa[c] = v;
                    else if (c == g.n) b_out[gates[u]] = v;
                }
            }
        }
        return;
    }
    if (!valid) return;
    if (SPLIT) {  // partial rows of ksk_width / 2 packed pairs, or ksk_width u32 sums (W32)
        const size_t hw = W32 ? ksk_width(g.n) : ksk_width(g.n) / 2;
        uint4* pp = reinterpret_cast<uint4*>(part + ((size_t)blockIdx.z * g.count + gate) * hw + (W32 ? col0 : col0 / 2));
#pragma unroll
        for (int k = 0; k < kAcc / 4; ++k)
            pp[k] = make_uint4(acc[4 * k], acc[4 * k + 1], acc[4 * k + 2], acc[4 * k + 3]);
        return;
    }
    const uint32_t qm = g.qKS - 1;
    const uint32_t b = ms_b[gate];
    uint64_t* oa = a_out + (size_t)gate * g.n;
    if (W32) {
#pragma unroll
        for (int k = 0; k < kKsCols; ++k) {
            const uint32_t c = col0 + k;
            uint64_t v;
            if (PRIME) {  // acc = -sum mod qKS in [0, qKS), b < qKS
                const uint32_t x = (c == g.n ? b : 0u) + acc[k];
                v = min(x, x - qks);
            } else {
                v = ((c == g.n ? b : 0u) + acc[k]) & qm;  // acc = -sum mod 2^32
            }
            if (q_out) v = mod_switch_up(v, g.qKS, q_out);
            if (c < g.n) oa[c] = v;
            else if (c == g.n) b_out[gate] = v;
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < kKsCols / 2; ++k) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t c = col0 + 2 * k + h;
            const uint32_t neg = h ? (acc[k] >> 16) : (acc[k] & 0xffffu);  // -sum mod 2^16
            uint64_t v = ((c == g.n ? b : 0u) + neg) & qm;
            if (q_out) v = mod_switch_up(v, g.qKS, q_out);  // ModSwitch qKS -> q_out
            if (c < g.n) oa[c] = v;
            else if (c == g.n) b_out[gate] = v;
        }
    }
}

// the S row-split partials of a gate, one packed column pair per thread and step (hw = W / 2 pairs, up
// to 640 at W = 1280, on at most 512 threads), then the epilogue
template <bool W32, bool PRIME = false>
__global__ void __launch_bounds__(512)
    k_keyswitch_reduce(GateArgs g, const uint32_t* __restrict__ part, uint32_t S, uint32_t hw,
                       const uint32_t* __restrict__ ms_b, uint64_t q_out, uint64_t* __restrict__ a_out,
                       uint64_t* __restrict__ b_out) {
    const uint32_t gate = blockIdx.x;
    const uint32_t qm = g.qKS - 1, qks = g.qKS;
    const uint32_t b = ms_b[gate];
    uint64_t* oa = a_out + (size_t)gate * g.n;
    if (W32) {  // hw = ksk_width u32 sums (mod 2^32; PRIME: partials in [0, qKS), summed mod qKS)
        for (uint32_t c = threadIdx.x; c < hw; c += blockDim.x) {
            uint32_t acc = 0;
            for (uint32_t z = 0; z < S; ++z) {
                acc += part[((size_t)z * g.count + gate) * hw + c];
                if (PRIME) acc = min(acc, acc - qks);
            }
            uint64_t v;
            if (PRIME) {
                const uint32_t x = (c == g.n ? b : 0u) + acc;
                v = min(x, x - qks);
            } else {
                v = ((c == g.n ? b : 0u) + acc) & qm;
            }
            if (q_out) v = mod_switch_up(v, g.qKS, q_out);
            if (c < g.n) oa[c] = v;
            else if (c == g.n) b_out[gate] = v;
        }
        return;
    }
    for (uint32_t t = threadIdx.x; t < hw; t += blockDim.x) {
        uint32_t acc = 0;
        for (uint32_t z = 0; z < S; ++z) {
            const uint32_t w = part[((size_t)z * g.count + gate) * hw + t];
            asm("v_pk_add_u16 %0, %1, %2" : "=v"(acc) : "v"(acc), "v"(w));
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t c = 2 * t + h;
            const uint32_t neg = h ? (acc >> 16) : (acc & 0xffffu);  // -sum mod 2^16
            uint64_t v = ((c == g.n ? b : 0u) + neg) & qm;
            if (q_out) v = mod_switch_up(v, g.qKS, q_out);
            if (c < g.n) oa[c] = v;
            else if (c == g.n) b_out[gate] = v;
        }
    }
}

// row-split factor of the tiled kernel for `count` gates: enough workgroups for 4 per CU, at
// least 8 rounds each, within the scratch the caller holds (part_words u32)
static uint32_t split_factor(size_t count, uint32_t n, uint32_t N, size_t part_words, uint32_t G) {
    const size_t tiles = ((count + G - 1) / G) * (ksk_width(n) / kKsCols);
    uint32_t S = 1;
    while (tiles * S < 1024 && N / kKsIPR / (2 * S) >= 8 && (size_t)2 * S * count * (ksk_width(n) / 2) <= part_words)
        S *= 2;
    return S;
}
// (the baseKS = 32 row split's gate tile)
uint32_t keyswitch_split(size_t count, uint32_t n, uint32_t N, size_t part_words) {
    return split_factor(count, n, N, part_words, kKsSplitG);
}

hipError_t launch_keyswitch(const GateArgs& g, uint32_t baseKS, uint32_t digitsKS, const uint16_t* ksk,
                            const uint32_t* ms_a, const uint32_t* ms_b, uint64_t q_out, uint64_t* a_out,
                            uint64_t* b_out, hipStream_t s, uint32_t* part, size_t part_words) {
    if (g.count == 0) return hipSuccess;
    const bool base21 = baseKS == 21 && digitsKS == 4;  // STD256Q_3: the tiled kernel only
    if ((baseKS & (baseKS - 1)) && !base21) return hipErrorInvalidValue;
    if (g.qKS & (g.qKS - 1) || g.qKS > 65536 || g.n >= 2048 || g.N > 2048) return hipErrorInvalidValue;
    const uint32_t W = ksk_width(g.n);
    const uint32_t logBase = base21 ? 0u : (uint32_t)__builtin_ctz(baseKS);
#ifndef FHE_KS_TILE
#define FHE_KS_TILE 0   // 0: choose by batch size; 1: per-gate kernel; 256: gate tile
#endif
    int tile = FHE_KS_TILE;
    // tiles need >= 16 x 8 workgroups to pay, or a row split (scratch) below 4096 gates
    if (tile == 0) tile = g.count >= 4096 || part ? 256 : 1;
    const bool shape3 = (logBase == 5 || logBase == 6) && digitsKS == 3, shape4 = logBase == 4 && digitsKS == 4;
    if (base21) tile = 256;
    if (tile > 1 && (!(shape3 || shape4 || base21) || g.N % kKsIPR)) tile = 1;
    if (base21 && tile == 1) return hipErrorInvalidValue;
    // the per-gate kernel: one thread per column pair, at most 512
    if (tile == 1 && W > 1024) return hipErrorInvalidValue;
    if (tile > 1) {
        // baseKS = 32: the tile shape by batch size (kKsIPR above); baseKS = 64: G 256
        const uint32_t Gs = logBase == 5 ? (uint32_t)kKsSplitG : 256u;
        const uint32_t S = part ? split_factor(g.count, g.n, g.N, part_words, Gs) : 1;
        const uint32_t G = S > 1 ? Gs : logBase == 5 && g.count >= kKsWideBatch ? 512u : 256u;
        const dim3 grid((g.count + G - 1) / G, W / kKsCols, S);
#define FHE_KS_LAUNCH(G_, SP, LB, IPR_, ...)                                                                      \
    hipLaunchKernelGGL((k_keyswitch_tiled<G_, SP, LB, IPR_, ##__VA_ARGS__>), grid, dim3(G_), 0, s, g, ksk, ms_a, ms_b, \
                       q_out, a_out, b_out, SP ? part : nullptr)
        if (base21) {
            if (S > 1) FHE_KS_LAUNCH(256, true, 21, 2, 4); else FHE_KS_LAUNCH(256, false, 21, 2, 4);
        } else if (shape4) {
            if (S > 1) FHE_KS_LAUNCH(256, true, 16, 2, 4); else FHE_KS_LAUNCH(256, false, 16, 2, 4);
        } else if (logBase == 5) {
            if (S > 1) FHE_KS_LAUNCH(kKsSplitG, true, 32, 4);
            else if (G == 512 && FHE_KS_GPT > 1) {  // GPT gates per thread: grid over G GPT-gate tiles
                const dim3 gg((g.count + 512 * FHE_KS_GPT - 1) / (512 * FHE_KS_GPT), W / kKsCols, 1);
                hipLaunchKernelGGL((k_keyswitch_tiled<512, false, 32, 2, 3, false, FHE_KS_GPT>), gg, dim3(512), 0, s, g,
                                   ksk, ms_a, ms_b, q_out, a_out, b_out, nullptr);
            } else if (G == 512 && FHE_KS_G1024 && g.count >= 32768) {  // 1024-gate tiles, one thread per gate
                const dim3 gg((g.count + 1023) / 1024, W / kKsCols, 1);
                hipLaunchKernelGGL((k_keyswitch_tiled<1024, false, 32, 2>), gg, dim3(1024), 0, s, g, ksk, ms_a, ms_b, q_out,
                                   a_out, b_out, nullptr);
            } else if (G == 512) FHE_KS_LAUNCH(512, false, 32, 2);
            else FHE_KS_LAUNCH(256, false, 32, 4);
        } else {
            if (S > 1) FHE_KS_LAUNCH(256, true, 64, 2); else FHE_KS_LAUNCH(256, false, 64, 2);
        }
#undef FHE_KS_LAUNCH
        if (S > 1) {
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(k_keyswitch_reduce<false>, dim3(g.count), dim3(std::min(W / 2, 512u)), 0, s, g, part, S,
                               W / 2, ms_b, q_out, a_out, b_out);
        }
    } else {
        hipLaunchKernelGGL(k_keyswitch, dim3(g.count), dim3(W / 2), 0, s, g, logBase, digitsKS,
                           reinterpret_cast<const uint32_t*>(ksk), ms_a, ms_b, q_out, a_out, b_out);
    }
    return hipGetLastError();
}

bool keyswitch_w32_shape(uint32_t baseKS, uint32_t digitsKS) {
    return (baseKS == 16 && (digitsKS == 5 || digitsKS == 6)) || (baseKS == 64 && digitsKS == 3) ||
           (baseKS == 25 && (digitsKS == 6 || digitsKS == 7));  // the prime-qKS rows (TOY, SIGNED_MOD_TEST)
}

// u32 rows (ksk_width(n) columns: A then B at column n), any power-of-two qKS <= 2^32, the shapes of
// keyswitch_w32_shape; row split below 4096 gates into part (u32 [S][count][W])
hipError_t launch_keyswitch_w32(const GateArgs& g, uint32_t baseKS, uint32_t digitsKS, const uint32_t* ksk,
                                const uint32_t* ms_a, const uint32_t* ms_b, uint64_t q_out, uint64_t* a_out,
                                uint64_t* b_out, hipStream_t s, uint32_t* part, size_t part_words) {
    if (g.count == 0) return hipSuccess;
    // baseKS 25: a prime qKS below 2^28 (sums kept mod qKS); otherwise a power of two (sums mod 2^32)
    const bool prime = baseKS == 25;
    if (!keyswitch_w32_shape(baseKS, digitsKS) || g.qKS < 2 || g.n >= 2048 || g.N > 2048 ||
        (prime ? (g.qKS >= (1u << 28) || !(g.qKS & 1)) : (g.qKS & (g.qKS - 1)) != 0))
        return hipErrorInvalidValue;
    const uint32_t W = ksk_width(g.n);
    if (prime) {  // 25 slices of 16 parts per step: 512-thread tiles (400 stagers), 92 KB of double buffer
        constexpr uint32_t GP = 512;
        uint32_t S = 1;
        if (part) {
            const size_t tiles = ((g.count + GP - 1) / GP) * (W / kKsCols);
            while (tiles * S < 1024 && g.N / (2 * S) >= 16 && (size_t)2 * S * g.count * W <= part_words) S *= 2;
        }
        const dim3 grid((g.count + GP - 1) / GP, W / kKsCols, S);
#define FHE_KSP_LAUNCH(SP, KD_)                                                                                     \
    hipLaunchKernelGGL((k_keyswitch_tiled<GP, SP, 25, 1, KD_, true, 1, true>), grid, dim3(GP), 0, s, g, ksk, ms_a, ms_b, \
                       q_out, a_out, b_out, SP ? part : nullptr)
        if (digitsKS == 6) { if (S > 1) FHE_KSP_LAUNCH(true, 6); else FHE_KSP_LAUNCH(false, 6); }
        else { if (S > 1) FHE_KSP_LAUNCH(true, 7); else FHE_KSP_LAUNCH(false, 7); }
#undef FHE_KSP_LAUNCH
        if (S > 1) {
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL((k_keyswitch_reduce<true, true>), dim3(g.count), dim3(512), 0, s, g, part, S, W, ms_b, q_out,
                               a_out, b_out);
        }
        return hipGetLastError();
    }
    constexpr uint32_t G = 256;
    uint32_t S = 1;
    if (part) {  // enough workgroups for 4 per CU, at least 16 rounds each, within the scratch
        const size_t tiles = ((g.count + G - 1) / G) * (W / kKsCols);
        while (tiles * S < 1024 && g.N / (2 * S) >= 16 && (size_t)2 * S * g.count * W <= part_words) S *= 2;
    }
    const dim3 grid((g.count + G - 1) / G, W / kKsCols, S);
#define FHE_KSW_LAUNCH(SP, LB, KD_)                                                                               \
    hipLaunchKernelGGL((k_keyswitch_tiled<G, SP, LB, 1, KD_, true>), grid, dim3(G), 0, s, g, ksk, ms_a, ms_b, q_out, \
                       a_out, b_out, SP ? part : nullptr)
    if (baseKS == 16 && digitsKS == 5) {
        if (S > 1) FHE_KSW_LAUNCH(true, 16, 5); else FHE_KSW_LAUNCH(false, 16, 5);
    } else if (baseKS == 16) {
        if (S > 1) FHE_KSW_LAUNCH(true, 16, 6); else FHE_KSW_LAUNCH(false, 16, 6);
    } else {
        if (S > 1) FHE_KSW_LAUNCH(true, 64, 3); else FHE_KSW_LAUNCH(false, 64, 3);
    }
#undef FHE_KSW_LAUNCH
    if (S > 1) {
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_keyswitch_reduce<true>, dim3(g.count), dim3(512), 0, s, g, part, S, W, ms_b, q_out, a_out,
                           b_out);
    }
    return hipGetLastError();
}

}  // namespace fhe_amd
