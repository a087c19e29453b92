/*
 * tfhe_oracle.c -- CPU restatement of the reference's TFHE gate-bootstrap path.
 * TEST INFRASTRUCTURE ONLY (see tfhe_oracle.h).  Plain C11 + OpenMP over gates.
 *
 * Each function follows the reference file:line cited next to it; u64
 * arithmetic with __uint128_t products, canonical residues in [0, Q).
 */
#include "tfhe_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;

static uint64_t mulmod(uint64_t a, uint64_t b, uint64_t m) { return (uint64_t)(((u128)a * b) % m); }
static uint64_t addmod(uint64_t a, uint64_t b, uint64_t m) { uint64_t s = a + b; return s >= m ? s - m : s; }
static uint64_t submod(uint64_t a, uint64_t b, uint64_t m) { return a >= b ? a - b : a + m - b; }
static uint64_t powmod(uint64_t b, uint64_t e, uint64_t m) {
    uint64_t r = 1 % m;
    b %= m;
    while (e) {
        if (e & 1) r = mulmod(r, b, m);
        b = mulmod(b, b, m);
        e >>= 1;
    }
    return r;
}
static uint32_t reverse_bits(uint32_t x, uint32_t bits) {  /* ReverseBits, nbtheory.h:135 */
    uint32_t r = 0;
    for (uint32_t i = 0; i < bits; ++i) r |= ((x >> i) & 1u) << (bits - 1 - i);
    return r;
}
static uint32_t ilog2(uint64_t x) { uint32_t r = 0; while (x > 1) { x >>= 1; ++r; } return r; }

/* deterministic Miller-Rabin for 64-bit (the reference's MillerRabinPrimalityTest
 * is probabilistic; for the primes used here both agree) */
static int is_prime(uint64_t n) {
    static const uint64_t bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    if (n < 2) return 0;
    for (int i = 0; i < 12; ++i) {
        if (n == bases[i]) return 1;
        if (n % bases[i] == 0) return 0;
    }
    uint64_t d = n - 1; int s = 0;
    while (!(d & 1)) { d >>= 1; ++s; }
    for (int i = 0; i < 12; ++i) {
        uint64_t x = powmod(bases[i], d, n);
        if (x == 1 || x == n - 1) continue;
        int ok = 0;
        for (int r = 1; r < s; ++r) {
            x = mulmod(x, x, n);
            if (x == n - 1) { ok = 1; break; }
        }
        if (!ok) return 0;
    }
    return 1;
}

/* LastPrime: nbtheory-impl.h:350-371 */
uint64_t tfo_last_prime(uint32_t bits, uint64_t m) {
    uint64_t q = (uint64_t)1 << bits;
    uint64_t r = q % m;
    uint64_t qn = q + 1 - r;
    if (r < 2) qn -= m;
    while (!is_prime(qn)) qn -= m;
    return qn;
}

/* RootOfUnity: nbtheory-impl.h:183-228 -- the minimal primitive m-th root
 * (minimum over all primitive roots, so independent of which generator). */
uint64_t tfo_root_of_unity(uint64_t m, uint64_t Q) {
    uint64_t phi = Q - 1, f[64]; int nf = 0; uint64_t t = phi;
    for (uint64_t p = 2; p * p <= t; ++p)
        if (t % p == 0) { f[nf++] = p; while (t % p == 0) t /= p; }
    if (t > 1) f[nf++] = t;
    uint64_t g = 2;
    for (;; ++g) {
        int ok = 1;
        for (int i = 0; i < nf; ++i) if (powmod(g, phi / f[i], Q) == 1) { ok = 0; break; }
        if (ok) break;
    }
    uint64_t r = powmod(g, phi / m, Q), best = 0, x = 1;
    for (uint64_t k = 1; k < m; ++k) {
        x = mulmod(x, r, Q);
        if ((k & 1) && x != 1 && (best == 0 || x < best)) best = x;  /* odd k = coprime to 2^k */
    }
    return best;
}

/* parameter rows: binfhecontext.cpp:113-159; digitsG rgsw-cryptoparameters.h:93-94;
 * digitsKS lwe-pke.cpp:354 */
int tfo_params_init(int paramset, int method, tfo_params* p) {
    uint32_t bits, cyc, n, q, qks, bks, bg, nauto;
    switch (paramset) {
        case TFO_TOY:            bits = 27; cyc = 1024; n = 64;  q = 512;  qks = 0;     bks = 25; bg = 512;  nauto = 9;  break;
        case TFO_STD128_AP:
        case TFO_STD128:         bits = 27; cyc = 2048; n = 503; q = 1024; qks = 16384; bks = 32; bg = 512;  nauto = 10; break;
        case TFO_STD128_LMKCDEY: bits = 28; cyc = 2048; n = 447; q = 2048; qks = 16384; bks = 32; bg = 1024; nauto = 10; break;
        default: return -1;
    }
    if (method != TFO_GINX && method != TFO_LMKCDEY && method != TFO_AP) return -2;
    memset(p, 0, sizeof(*p));
    p->paramset = paramset; p->method = method;
    p->n = n; p->N = cyc / 2; p->q = q;
    p->Q = tfo_last_prime(bits, cyc);
    p->qKS = qks ? qks : (uint32_t)p->Q;
    p->baseKS = bks;
    p->digitsKS = (uint32_t)ceil(log((double)p->qKS) / log((double)bks));
    p->baseG = bg; p->gBits = ilog2(bg);
    p->digitsG = (uint32_t)ceil(log((double)p->Q) / log((double)bg));
    p->numAutoKeys = nauto;
    p->psi = tfo_root_of_unity(cyc, p->Q);
    p->baseR = 32;                                              /* baseR column (binfhecontext.cpp:113-159) */
    p->digitsR = (uint32_t)ceil(log((double)q) / log((double)p->baseR));
    return 0;
}

/* ---- NTT (transformnat-impl.h) ------------------------------------------ */
typedef struct { uint32_t N, logN; uint64_t Q, Ninv; uint64_t *tab, *tabI; } ntt_tab;

/* PreCompute: transformnat-impl.h:777-831 (Table[brv(i)] = psi^i) */
static void ntt_tab_init(ntt_tab* t, uint32_t N, uint64_t Q, uint64_t psi) {
    t->N = N; t->logN = ilog2(N); t->Q = Q;
    t->tab = (uint64_t*)malloc(N * sizeof(uint64_t));
    t->tabI = (uint64_t*)malloc(N * sizeof(uint64_t));
    uint64_t psiI = powmod(psi, Q - 2, Q), x = 1, xi = 1;
    for (uint32_t i = 0; i < N; ++i) {
        uint32_t r = reverse_bits(i, t->logN);
        t->tab[r] = x; t->tabI[r] = xi;
        x = mulmod(x, psi, Q); xi = mulmod(xi, psiI, Q);
    }
    t->Ninv = powmod(N, Q - 2, Q);
}
static void ntt_tab_free(ntt_tab* t) { free(t->tab); free(t->tabI); }

/* ForwardTransformToBitReverseInPlace: transformnat-impl.h:302-373 (CT) */
static void ntt_fwd(const ntt_tab* T, uint64_t* a) {
    const uint64_t Q = T->Q; const uint32_t n = T->N;
    for (uint32_t m = 1, t = n >> 1; m < n; m <<= 1, t >>= 1)
        for (uint32_t i = 0; i < m; ++i) {
            uint64_t w = T->tab[m + i];
            for (uint32_t j = 2 * i * t; j < 2 * i * t + t; ++j) {
                uint64_t hi = mulmod(a[j + t], w, Q), lo = a[j];
                a[j] = addmod(lo, hi, Q);
                a[j + t] = submod(lo, hi, Q);
            }
        }
}
/* InverseTransformFromBitReverseInPlace: transformnat-impl.h:511-624 (GS, x N^-1) */
static void ntt_inv(const ntt_tab* T, uint64_t* a) {
    const uint64_t Q = T->Q; const uint32_t n = T->N;
    for (uint32_t m = n >> 1, t = 1; m >= 1; m >>= 1, t <<= 1)
        for (uint32_t i = 0; i < m; ++i) {
            uint64_t w = T->tabI[m + i];
            for (uint32_t j = 2 * i * t; j < 2 * i * t + t; ++j) {
                uint64_t lo = a[j], hi = a[j + t];
                a[j] = addmod(lo, hi, Q);
                a[j + t] = mulmod(submod(lo, hi, Q), w, Q);
            }
        }
    for (uint32_t i = 0; i < n; ++i) a[i] = mulmod(a[i], T->Ninv, Q);
}

int tfo_ntt_batch(uint64_t* polys, size_t count, uint32_t N, uint64_t Q, uint64_t psi, int inverse, int nthreads) {
    ntt_tab T; ntt_tab_init(&T, N, Q, psi);
    long long c;
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(static)
    for (c = 0; c < (long long)count; ++c) {
        if (inverse) ntt_inv(&T, polys + (size_t)c * N); else ntt_fwd(&T, polys + (size_t)c * N);
    }
    ntt_tab_free(&T);
    return 0;
}

/* ---- bootstrapping ------------------------------------------------------- */
typedef struct {
    const tfo_params* p;
    ntt_tab T;
    uint32_t dG2;
    uint64_t* gpow;       /* Gpow[i] = Bg^i mod Q, rgsw-cryptoparameters.cpp:69-74 */
    uint64_t* monomials;  /* [2N][N] EVAL(X^m - 1), rgsw-cryptoparameters.cpp:96-113 (GINX) */
    int32_t* logGen;      /* rgsw-cryptoparameters.cpp:115-127 (LMKCDEY) */
} boot_ctx;

static void boot_ctx_init(boot_ctx* c, const tfo_params* p) {
    memset(c, 0, sizeof(*c));
    c->p = p;
    ntt_tab_init(&c->T, p->N, p->Q, p->psi);
    c->dG2 = (p->digitsG - 1) * 2;
    c->gpow = (uint64_t*)malloc(p->digitsG * sizeof(uint64_t));
    uint64_t v = 1;
    for (uint32_t i = 0; i < p->digitsG; ++i) { c->gpow[i] = v; v = mulmod(v, p->baseG, p->Q); }
    const uint32_t N = p->N, M = 2 * N;
    if (p->method == TFO_GINX) {
        c->monomials = (uint64_t*)calloc((size_t)M * N, sizeof(uint64_t));
        for (uint32_t m = 0; m < M; ++m) {
            uint64_t* a = c->monomials + (size_t)m * N;
            a[0] = submod(a[0], 1, p->Q);
            if (m < N) a[m] = addmod(a[m], 1, p->Q);          /* X^m - 1 */
            else a[m - N] = submod(a[m - N], 1, p->Q);        /* -X^(m-N) - 1 */
            ntt_fwd(&c->T, a);
        }
    } else {
        c->logGen = (int32_t*)calloc(M, sizeof(int32_t));
        uint32_t g = 1;
        c->logGen[M - g] = (int32_t)M;
        for (uint32_t i = 1; i < N / 2; ++i) {
            g = (g * 5) % M;
            c->logGen[g] = (int32_t)i;
            c->logGen[M - g] = -(int32_t)i;
        }
    }
}
static void boot_ctx_free(boot_ctx* c) {
    ntt_tab_free(&c->T); free(c->gpow); free(c->monomials); free(c->logGen);
}

/* SignedDigitDecompose (two-poly form), rgsw-acc.cpp:54-91 */
static void decompose2(const boot_ctx* c, const uint64_t* in0, const uint64_t* in1, uint64_t* out /*[dG2][N]*/) {
    const tfo_params* p = c->p;
    const uint64_t QHalf = p->Q >> 1; const int64_t Qi = (int64_t)p->Q;
    const int64_t g = p->gBits, gm = 64 - g;
    memset(out, 0, (size_t)c->dG2 * p->N * sizeof(uint64_t));
    for (uint32_t k = 0; k < p->N; ++k) {
        int64_t d0 = in0[k] < QHalf ? (int64_t)in0[k] : (int64_t)in0[k] - Qi;
        int64_t d1 = in1[k] < QHalf ? (int64_t)in1[k] : (int64_t)in1[k] - Qi;
        int64_t r0 = (int64_t)((uint64_t)d0 << gm) >> gm; d0 = (d0 - r0) >> g;
        int64_t r1 = (int64_t)((uint64_t)d1 << gm) >> gm; d1 = (d1 - r1) >> g;
        for (uint32_t d = 0; d < c->dG2; d += 2) {
            r0 = (int64_t)((uint64_t)d0 << gm) >> gm; d0 = (d0 - r0) >> g;
            if (r0 < 0) r0 += Qi;
            out[(size_t)(d + 0) * p->N + k] += (uint64_t)r0;
            r1 = (int64_t)((uint64_t)d1 << gm) >> gm; d1 = (d1 - r1) >> g;
            if (r1 < 0) r1 += Qi;
            out[(size_t)(d + 1) * p->N + k] += (uint64_t)r1;
        }
    }
}
/* SignedDigitDecompose (single-poly form), rgsw-acc.cpp:94-119 */
static void decompose1(const boot_ctx* c, const uint64_t* in, uint64_t* out /*[digitsG-1][N]*/) {
    const tfo_params* p = c->p;
    const uint64_t QHalf = p->Q >> 1; const int64_t Qi = (int64_t)p->Q;
    const int64_t g = p->gBits, gm = 64 - g;
    memset(out, 0, (size_t)(p->digitsG - 1) * p->N * sizeof(uint64_t));
    for (uint32_t k = 0; k < p->N; ++k) {
        int64_t d0 = in[k] < QHalf ? (int64_t)in[k] : (int64_t)in[k] - Qi;
        int64_t r0 = (int64_t)((uint64_t)d0 << gm) >> gm; d0 = (d0 - r0) >> g;
        for (uint32_t d = 0; d < p->digitsG - 1; ++d) {
            r0 = (int64_t)((uint64_t)d0 << gm) >> gm; d0 = (d0 - r0) >> g;
            if (r0 < 0) r0 += Qi;
            out[(size_t)d * p->N + k] += (uint64_t)r0;
        }
    }
}

/* AutomorphismTransform(k) in EVALUATION (poly-impl.h:310-356, :366-376 with
 * PrecomputeAutoMap nbtheory2.cpp:264-275 -- both give the same permutation) */
static void automorphism(const tfo_params* p, uint32_t k, const uint64_t* in, uint64_t* out) {
    const uint32_t N = p->N, logN = ilog2(N), mask = N - 1;
    for (uint32_t j = 0; j < N; ++j) {
        uint32_t jk = (2 * j + 1) * k;
        out[reverse_bits(j, logN)] = in[reverse_bits((jk >> 1) & mask, logN)];
    }
}

/* AddToAccCGGI: rgsw-acc-cggi.cpp:102-151 */
static void add_to_acc_cggi(const boot_ctx* c, const uint64_t* ek1, const uint64_t* ek2, uint32_t a,
                            uint64_t* acc, uint64_t* work) {
    const tfo_params* p = c->p; const uint32_t N = p->N, dG2 = c->dG2; const uint64_t Q = p->Q;
    uint64_t* ct = work;                 /* 2N */
    uint64_t* dct = work + 2 * N;        /* dG2*N */
    memcpy(ct, acc, 2 * N * sizeof(uint64_t));
    ntt_inv(&c->T, ct); ntt_inv(&c->T, ct + N);
    decompose2(c, ct, ct + N, dct);
    for (uint32_t d = 0; d < dG2; ++d) ntt_fwd(&c->T, dct + (size_t)d * N);
    const uint32_t M = 2 * N;
    uint32_t ipos = a == M ? 0 : a;
    uint32_t ineg = a == 0 ? 0 : M - a;
    const uint64_t* mono = c->monomials + (size_t)ipos * N;
    const uint64_t* monoN = c->monomials + (size_t)ineg * N;
    for (int key = 0; key < 2; ++key) {
        const uint64_t* ek = key ? ek2 : ek1;   /* [dG2][2][N] */
        const uint64_t* mo = key ? monoN : mono;
        for (uint32_t comp = 0; comp < 2; ++comp)
            for (uint32_t j = 0; j < N; ++j) {
                uint64_t t = 0;
                for (uint32_t d = 0; d < dG2; ++d)
                    t = addmod(t, mulmod(dct[(size_t)d * N + j], ek[((size_t)d * 2 + comp) * N + j], Q), Q);
                acc[comp * N + j] = addmod(acc[comp * N + j], mulmod(t, mo[j], Q), Q);
            }
    }
}

/* AddToAccLMKCDEY: rgsw-acc-lmkcdey.cpp:228-254 (acc replaced) */
static void add_to_acc_lmk(const boot_ctx* c, const uint64_t* ek, uint64_t* acc, uint64_t* work) {
    const tfo_params* p = c->p; const uint32_t N = p->N, dG2 = c->dG2; const uint64_t Q = p->Q;
    uint64_t* ct = work; uint64_t* dct = work + 2 * N;
    memcpy(ct, acc, 2 * N * sizeof(uint64_t));
    ntt_inv(&c->T, ct); ntt_inv(&c->T, ct + N);
    decompose2(c, ct, ct + N, dct);
    for (uint32_t d = 0; d < dG2; ++d) ntt_fwd(&c->T, dct + (size_t)d * N);
    for (uint32_t comp = 0; comp < 2; ++comp)
        for (uint32_t j = 0; j < N; ++j) {
            uint64_t t = 0;
            for (uint32_t d = 0; d < dG2; ++d)
                t = addmod(t, mulmod(dct[(size_t)d * N + j], ek[((size_t)d * 2 + comp) * N + j], Q), Q);
            acc[comp * N + j] = t;
        }
}

/* EvalAcc DM (rgsw-acc-dm.cpp:62-77): for each i and base-baseR digit a0 of (q - a_i) mod q,
 * acc <- external product with key [i][a0][k] (AddToAccDM :119-145 == add_to_acc_lmk) */
static void eval_acc_dm(const boot_ctx* c, const uint64_t* bsk, const uint64_t* a, uint64_t* acc, uint64_t* work) {
    const tfo_params* p = c->p; const uint32_t N = p->N;
    const size_t rg = (size_t)c->dG2 * 2 * N;
    for (uint32_t i = 0; i < p->n; ++i) {
        uint64_t aI = (p->q - a[i] % p->q) % p->q;
        for (uint32_t k = 0; k < p->digitsR; ++k, aI /= p->baseR) {
            const uint64_t a0 = aI % p->baseR;
            if (a0) add_to_acc_lmk(c, bsk + (((size_t)i * p->baseR + a0) * p->digitsR + k) * rg, acc, work);
        }
    }
}

/* Automorphism: rgsw-acc-lmkcdey.cpp:257-287 */
static void lmk_automorphism(const boot_ctx* c, uint32_t k, const uint64_t* ak, uint64_t* acc, uint64_t* work) {
    const tfo_params* p = c->p; const uint32_t N = p->N, dG = p->digitsG - 1; const uint64_t Q = p->Q;
    uint64_t* tmp = work; uint64_t* cta = work + N; uint64_t* dcta = work + 2 * N;
    automorphism(p, k, acc + N, tmp);
    memcpy(acc + N, tmp, N * sizeof(uint64_t));
    automorphism(p, k, acc, cta);
    ntt_inv(&c->T, cta);
    decompose1(c, cta, dcta);
    for (uint32_t d = 0; d < dG; ++d) ntt_fwd(&c->T, dcta + (size_t)d * N);
    for (uint32_t j = 0; j < N; ++j) {
        uint64_t t0 = 0, t1 = acc[N + j];
        for (uint32_t d = 0; d < dG; ++d) {
            t0 = addmod(t0, mulmod(dcta[(size_t)d * N + j], ak[((size_t)d * 2 + 0) * N + j], Q), Q);
            t1 = addmod(t1, mulmod(dcta[(size_t)d * N + j], ak[((size_t)d * 2 + 1) * N + j], Q), Q);
        }
        acc[j] = t0; acc[N + j] = t1;
    }
}

static uint64_t gate_const(uint32_t q, int gate) {  /* rgsw-cryptoparameters.cpp:78-92 */
    switch (gate) {
        case 0: return 5ull * (q >> 3);  case 1: return 7ull * (q >> 3);
        case 2: return 1ull * (q >> 3);  case 3: return 3ull * (q >> 3);
        case 4: return 6ull * (q >> 3);  case 5: return 2ull * (q >> 3);
        case 6: return 7ull * (q >> 3);  case 7: return 11ull * (q / 12);
        case 8: return 7ull * (q / 12);  case 9: return 15ull * (q >> 4);
        case 10: return 9ull * (q >> 4); case 11: return 6ull * (q >> 3);
        case 12: return 2ull * (q >> 3);
        default: return 0;
    }
}

static uint64_t roundqQ(uint64_t v, uint64_t q, uint64_t Q) {  /* lwe-pke.cpp:41-46 */
    return (uint64_t)floor(0.5 + (double)v * (double)q / (double)Q) % q;
}

void tfo_modswitch(uint64_t q_from, uint64_t q_to, uint32_t len, size_t count, const uint64_t* a, const uint64_t* b,
                   uint64_t* a_out, uint64_t* b_out) {
    for (size_t g = 0; g < count; ++g) {
        for (uint32_t i = 0; i < len; ++i) a_out[g * len + i] = roundqQ(a[g * len + i], q_to, q_from);
        b_out[g] = roundqQ(b[g], q_to, q_from);
    }
}

static void keyswitch1(const tfo_params* p, const uint64_t* A, const uint64_t* B, const uint64_t* a, uint64_t b,
                       uint64_t* a_out, uint64_t* b_out) {
    const uint32_t n = p->n, N = p->N, bks = p->baseKS, dks = p->digitsKS; const uint64_t qk = p->qKS;
    for (uint32_t k = 0; k < n; ++k) a_out[k] = 0;
    for (uint32_t i = 0; i < N; ++i) {
        uint64_t at = a[i];
        for (uint32_t j = 0; j < dks; ++j) {
            uint64_t a0 = at % bks; at /= bks;
            size_t row = ((size_t)i * bks + a0) * dks + j;
            b = submod(b, B[row], qk);
            const uint64_t* r = A + row * n;
            for (uint32_t k = 0; k < n; ++k) a_out[k] = submod(a_out[k], r[k], qk);
        }
    }
    *b_out = b;
}

void tfo_keyswitch(const tfo_params* p, const uint64_t* kskA, const uint64_t* kskB, size_t count, const uint64_t* a,
                   const uint64_t* b, uint64_t* a_out, uint64_t* b_out) {
    for (size_t g = 0; g < count; ++g)
        keyswitch1(p, kskA, kskB, a + g * p->N, b[g], a_out + g * p->n, b_out + g);
}

/* EvalAcc GINX: rgsw-acc-cggi.cpp:59-68 */
/* ctmod: modulus of a (q for gates; BootstrapFunc may use 2q), rgsw-acc-cggi.cpp:61-66 */
static void eval_acc_cggi(const boot_ctx* c, const uint64_t* bsk, const uint64_t* a, uint64_t ctmod, uint64_t* acc,
                          uint64_t* work) {
    const tfo_params* p = c->p; const uint32_t N = p->N;
    const size_t rg = (size_t)c->dG2 * 2 * N;    /* one RGSW */
    const uint64_t MbyMod = 2 * N / ctmod;
    for (uint32_t i = 0; i < p->n; ++i) {
        uint64_t ai = (ctmod - a[i] % ctmod) % ctmod;
        add_to_acc_cggi(c, bsk + (size_t)i * 2 * rg, bsk + ((size_t)i * 2 + 1) * rg, (uint32_t)(ai * MbyMod), acc, work);
    }
}

/* EvalAcc LMKCDEY: rgsw-acc-lmkcdey.cpp:70-158 */
static void eval_acc_lmk(const boot_ctx* c, const uint64_t* bsk, const uint64_t* a, uint64_t* acc, uint64_t* work) {
    const tfo_params* p = c->p; const uint32_t N = p->N, M = 2 * N, Nh = N / 2, n = p->n;
    const size_t rg = (size_t)c->dG2 * 2 * N, ak = (size_t)(p->digitsG - 1) * 2 * N;
    const uint64_t* autok = bsk + (size_t)n * rg;
    /* permuteMap: index -> list of i in increasing order.  index in [-Nh, Nh] or M */
    int32_t* idx = (int32_t*)malloc(n * sizeof(int32_t));
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t aodd = (uint32_t)((M - a[i] % M) % M) | 1u;
        idx[i] = c->logGen[aodd];
    }
#define APPLY_GROUP(KEY)                                                                 \
    for (uint32_t j = 0; j < n; ++j)                                                     \
        if (idx[j] == (KEY)) add_to_acc_lmk(c, bsk + (size_t)j * rg, acc, work);
#define HAS_GROUP(KEY, OUT) do { OUT = 0; for (uint32_t j = 0; j < n; ++j) if (idx[j] == (KEY)) { OUT = 1; break; } } while (0)
    uint64_t* tmp = work;
    automorphism(p, M - 5, acc + N, tmp);
    memcpy(acc + N, tmp, N * sizeof(uint64_t));
    uint32_t nSkips = 0; int has;
    for (int32_t i = (int32_t)Nh - 1; i > 0; --i) {
        HAS_GROUP(-i, has);
        if (has) {
            if (nSkips != 0) {
                lmk_automorphism(c, (uint32_t)powmod(5, nSkips, M), autok + nSkips * ak, acc, work);
                nSkips = 0;
            }
            APPLY_GROUP(-i);
        }
        nSkips++;
        if (nSkips == p->numAutoKeys || i == 1) {
            lmk_automorphism(c, (uint32_t)powmod(5, nSkips, M), autok + nSkips * ak, acc, work);
            nSkips = 0;
        }
    }
    APPLY_GROUP((int32_t)M);
    lmk_automorphism(c, M - 5, autok, acc, work);
    for (int32_t i = (int32_t)Nh - 1; i > 0; --i) {
        HAS_GROUP(i, has);
        if (has) {
            if (nSkips != 0) {
                lmk_automorphism(c, (uint32_t)powmod(5, nSkips, M), autok + nSkips * ak, acc, work);
                nSkips = 0;
            }
            APPLY_GROUP(i);
        }
        nSkips++;
        if (nSkips == p->numAutoKeys || i == 1) {
            lmk_automorphism(c, (uint32_t)powmod(5, nSkips, M), autok + nSkips * ak, acc, work);
            nSkips = 0;
        }
    }
    APPLY_GROUP(0);
#undef APPLY_GROUP
#undef HAS_GROUP
    free(idx);
}

/* BootstrapGateCore (binfhe-base-scheme.cpp:525-583) on the combined ciphertext (a, b) mod q,
 * then Transpose/iNTT/b fix-up (:110-121 / :155-163) and SwitchCTtoqn (lwe-pke.cpp:170-178).
 * tv_p: plaintext modulus of the bootstrapped ct (test vector Q/(2p)+1, :555-556);
 * b_p: the b constant Q/(2 b_p)+1 (b_p = 4 for 2-input gates, :118; the ctvector p, :162). */
static void eval_core(const boot_ctx* c, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB, int gate,
                      const uint64_t* a, uint64_t b, uint64_t tv_p, uint64_t b_p, uint64_t* a_out, uint64_t* b_out,
                      int stage, uint64_t* work) {
    const tfo_params* p = c->p; const uint32_t n = p->n, N = p->N; const uint64_t q = p->q, Q = p->Q;
    const uint64_t qHalf = q >> 1;
    uint64_t q1 = gate_const((uint32_t)q, gate), q2 = (q1 + qHalf) % q;
    int swap = q1 >= q2;
    uint64_t lb = swap ? q2 : q1, ub = swap ? q1 : q2;
    uint64_t Q2p = Q / (tv_p * 2) + 1, Q2pNeg = Q - Q2p;
    uint64_t lv = swap ? Q2p : Q2pNeg, uv = swap ? Q2pNeg : Q2p;
    uint64_t* acc = work; work += 2 * N;
    memset(acc, 0, 2 * N * sizeof(uint64_t));
    const uint32_t factor = (uint32_t)(N / qHalf);
    uint64_t bb = b;
    for (uint32_t i = 0; i < N; i += factor) {
        acc[N + i] = (bb >= lb && bb < ub) ? lv : uv;
        bb = submod(bb, 1, q);
    }
    ntt_fwd(&c->T, acc + N);
    if (p->method == TFO_GINX) eval_acc_cggi(c, bsk, a, q, acc, work);
    else if (p->method == TFO_AP) eval_acc_dm(c, bsk, a, acc, work);
    else eval_acc_lmk(c, bsk, a, acc, work);
    /* Transpose acc0 (automorphism 2N-1), iNTT both */
    uint64_t* t0 = work;
    automorphism(p, 2 * N - 1, acc, t0);
    memcpy(acc, t0, N * sizeof(uint64_t));
    ntt_inv(&c->T, acc); ntt_inv(&c->T, acc + N);
    uint64_t bext = addmod(Q / (2 * b_p) + 1, acc[N], Q);
    if (stage == 1) {
        memcpy(a_out, acc, N * sizeof(uint64_t));
        *b_out = bext;
        return;
    }
    /* SwitchCTtoqn */
    uint64_t* ms = work; uint64_t bms;
    tfo_modswitch(Q, p->qKS, N, 1, acc, &bext, ms, &bms);
    uint64_t* ks = work + N; uint64_t bks;
    keyswitch1(p, kskA, kskB, ms, bms, ks, &bks);
    tfo_modswitch(p->qKS, q, n, 1, ks, &bks, a_out, b_out);
    (void)n;
}

/* EvalBinGate (binfhe-base-scheme.cpp:76-126) for one 2-input gate (inputs with p = 4). */
static void eval_gate1(const boot_ctx* c, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB, int gate,
                       const uint64_t* a1, uint64_t b1, const uint64_t* a2, uint64_t b2, uint64_t* a_out,
                       uint64_t* b_out, int stage, uint64_t* work) {
    const tfo_params* p = c->p; const uint32_t n = p->n, N = p->N; const uint64_t q = p->q;
    uint64_t* a = work; work += N;
    uint64_t b = (b1 + b2) % q;
    for (uint32_t i = 0; i < n; ++i) a[i] = (a1[i] + a2[i]) % q;
    if (gate == 4 || gate == 5 || gate == 11 || gate == 12) {  /* XOR/XNOR: 2(ct1+ct2) */
        for (uint32_t i = 0; i < n; ++i) a[i] = (2 * a[i]) % q;
        b = (2 * b) % q;
    }
    eval_core(c, bsk, kskA, kskB, gate, a, b, 4, 4, a_out, b_out, stage, work);
}

int tfo_eval_gate_batch(const tfo_params* p, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB, int gate,
                        size_t count, const uint64_t* a1, const uint64_t* b1, const uint64_t* a2, const uint64_t* b2,
                        uint64_t* a_out, uint64_t* b_out, int stage, int nthreads) {
    boot_ctx c; boot_ctx_init(&c, p);
    const uint32_t n = p->n, N = p->N, outLen = stage == 1 ? N : n;
    const size_t wlen = (size_t)N * (4 + 3 + 2 * c.dG2 + 4);
    long long g;
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(dynamic, 1)
    for (g = 0; g < (long long)count; ++g) {
        uint64_t* work = (uint64_t*)malloc(wlen * sizeof(uint64_t));
        eval_gate1(&c, bsk, kskA, kskB, gate, a1 + (size_t)g * n, b1[g], a2 + (size_t)g * n, b2[g],
                   a_out + (size_t)g * outLen, b_out + g, stage, work);
        free(work);
    }
    boot_ctx_free(&c);
    return 0;
}

/* EvalBinGate(gate, ctvector) for MAJORITY/AND3/OR3/AND4/OR4 (binfhe-base-scheme.cpp:129-171):
 * ct = sum of the k inputs mod q, bootstrapped with the inputs' plaintext modulus ptmod. */
int tfo_eval_gate_multi_batch(const tfo_params* p, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB,
                              int gate, uint32_t k, uint32_t ptmod, size_t count, const uint64_t* const* a_in,
                              const uint64_t* const* b_in, uint64_t* a_out, uint64_t* b_out, int stage, int nthreads) {
    if (k < 2 || k > 4 || gate < 6 || gate > 10) return -2;
    boot_ctx c; boot_ctx_init(&c, p);
    const uint32_t n = p->n, N = p->N, outLen = stage == 1 ? N : n;
    const uint64_t q = p->q;
    const size_t wlen = (size_t)N * (5 + 3 + 2 * c.dG2 + 4);
    long long g;
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(dynamic, 1)
    for (g = 0; g < (long long)count; ++g) {
        uint64_t* work = (uint64_t*)malloc(wlen * sizeof(uint64_t));
        uint64_t* a = work;
        uint64_t b = 0;
        for (uint32_t i = 0; i < n; ++i) a[i] = 0;
        for (uint32_t j = 0; j < k; ++j) {
            for (uint32_t i = 0; i < n; ++i) a[i] = (a[i] + a_in[j][(size_t)g * n + i]) % q;
            b = (b + b_in[j][g]) % q;
        }
        eval_core(&c, bsk, kskA, kskB, gate, a, b, ptmod, ptmod, a_out + (size_t)g * outLen, b_out + g, stage,
                  work + N);
        free(work);
    }
    boot_ctx_free(&c);
    return 0;
}

/* EvalBinGate(CMUX, {ct0, ct1, ct2}) = NAND(NAND(ct0, EvalNOT(ct2)), NAND(ct1, ct2))
 * (binfhe-base-scheme.cpp:172-182); EvalNOT: (q - a, q/4 - b) (:223-236). */
int tfo_eval_cmux_batch(const tfo_params* p, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB,
                        size_t count, const uint64_t* a0, const uint64_t* b0, const uint64_t* a1, const uint64_t* b1,
                        const uint64_t* a2, const uint64_t* b2, uint64_t* a_out, uint64_t* b_out, int nthreads) {
    const uint32_t n = p->n;
    const uint64_t q = p->q;
    uint64_t* na = (uint64_t*)malloc(count * n * sizeof(uint64_t));
    uint64_t* nb = (uint64_t*)malloc(count * sizeof(uint64_t));
    uint64_t* l1a = (uint64_t*)malloc(2 * count * n * sizeof(uint64_t));
    uint64_t* l1b = (uint64_t*)malloc(2 * count * sizeof(uint64_t));
    for (size_t i = 0; i < count * n; ++i) na[i] = a2[i] == 0 ? 0 : q - a2[i];
    for (size_t g = 0; g < count; ++g) nb[g] = ((q >> 2) + q - b2[g] % q) % q;
    tfo_eval_gate_batch(p, bsk, kskA, kskB, 3, count, a0, b0, na, nb, l1a, l1b, 0, nthreads);
    tfo_eval_gate_batch(p, bsk, kskA, kskB, 3, count, a1, b1, a2, b2, l1a + count * n, l1b + count, 0, nthreads);
    tfo_eval_gate_batch(p, bsk, kskA, kskB, 3, count, l1a, l1b, l1a + count * n, l1b + count, a_out, b_out, 0,
                        nthreads);
    free(na); free(nb); free(l1a); free(l1b);
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Functional bootstrapping (binfhe-base-scheme.cpp:241-521, 589-648)                          */
/* ------------------------------------------------------------------------------------------ */

/* BootstrapFunc for one ciphertext (a mod ctmod, b): BootstrapFuncCore (:592-614) with the test
 * vector m[j * 2N/ctmod] = tv[(b - j) mod ctmod] (tv[x] = (Q / fmod) f(x, ctmod, fmod)), EvalAcc,
 * Transpose / iNTT, ctExt = (acc0, acc1[0]), ModSwitch(qKS), KeySwitch, ModSwitch(fmod) (:617-642). */
static void bootstrap_func1(const boot_ctx* c, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB,
                            const uint64_t* a, uint64_t b, uint64_t ctmod, const uint64_t* tv, uint64_t fmod,
                            uint64_t* a_out, uint64_t* b_out, uint64_t* work) {
    const tfo_params* p = c->p; const uint32_t n = p->n, N = p->N; const uint64_t Q = p->Q;
    uint64_t* acc = work; work += 2 * N;
    memset(acc, 0, 2 * N * sizeof(uint64_t));
    const uint64_t factor = 2 * N / ctmod;
    b %= ctmod;
    for (uint64_t j = 0; j < (ctmod >> 1); ++j) acc[N + j * factor] = tv[(b + ctmod - j) % ctmod];
    ntt_fwd(&c->T, acc + N);
    if (p->method == TFO_GINX) eval_acc_cggi(c, bsk, a, ctmod, acc, work);
    else if (p->method == TFO_AP) eval_acc_dm(c, bsk, a, acc, work);
    else eval_acc_lmk(c, bsk, a, acc, work);
    uint64_t* t0 = work;
    automorphism(p, 2 * N - 1, acc, t0);
    memcpy(acc, t0, N * sizeof(uint64_t));
    ntt_inv(&c->T, acc); ntt_inv(&c->T, acc + N);
    uint64_t bext = acc[N];
    uint64_t* ms = work; uint64_t bms;
    tfo_modswitch(Q, p->qKS, N, 1, acc, &bext, ms, &bms);
    uint64_t* ks = work + N; uint64_t bks;
    keyswitch1(p, kskA, kskB, ms, bms, ks, &bks);
    tfo_modswitch(p->qKS, fmod, n, 1, ks, &bks, a_out, b_out);
    (void)Q;
}

int tfo_bootstrap_func_batch(const tfo_params* p, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB,
                             size_t count, const uint64_t* a, const uint64_t* b, uint64_t ctmod, const uint64_t* tv,
                             uint64_t fmod, uint64_t* a_out, uint64_t* b_out, int nthreads) {
    if (ctmod < 2 || (ctmod & (ctmod - 1)) || ctmod > 2ull * p->N) return -2;
    boot_ctx c; boot_ctx_init(&c, p);
    const uint32_t n = p->n, N = p->N;
    const size_t wlen = (size_t)N * (4 + 3 + 2 * c.dG2 + 4);
    long long g;
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(dynamic, 1)
    for (g = 0; g < (long long)count; ++g) {
        uint64_t* work = (uint64_t*)malloc(wlen * sizeof(uint64_t));
        bootstrap_func1(&c, bsk, kskA, kskB, a + (size_t)g * n, b[g], ctmod, tv, fmod, a_out + (size_t)g * n,
                        b_out + g, work);
        free(work);
    }
    boot_ctx_free(&c);
    return 0;
}

/* test-vector functions f(x, q = ctmod, Q = fmod) of the reference's lambdas */
enum { TV_LUT, TV_LUT_ANTI, TV_HALF, TV_FLOOR2, TV_SIGN, TV_SIGN_SS };
static void make_tv(const tfo_params* p, int kind, const uint64_t* lut, uint64_t lutlen, uint64_t q, uint64_t fmod,
                    uint64_t* tv) {
    const uint64_t scale = p->Q / fmod;
    for (uint64_t x = 0; x < q; ++x) {
        uint64_t f = 0;
        switch (kind) {
            case TV_LUT: f = lut[x]; break;                                             /* :254-256 */
            case TV_LUT_ANTI: f = x < (q >> 1) ? lut[x % lutlen] : fmod - lut[(x - q / 2) % lutlen]; break; /* :302-307, 324-329 */
            case TV_HALF: f = x < (q >> 1) ? fmod - (q >> 2) : (q >> 2); break;         /* f0 / f1 :285-290 */
            case TV_FLOOR2:                                                             /* f2 :361-368 */
                f = x < (q >> 2) ? fmod - (q >> 1) - x : (x < 3 * (q >> 2) ? x : fmod + (q >> 1) - x); break;
            case TV_SIGN: f = x < q / 2 ? fmod / 4 : fmod - fmod / 4; break;            /* f3 :413-416 */
            case TV_SIGN_SS: f = x < q / 2 ? fmod - fmod / 4 : fmod / 4; break;         /* :421-424 */
        }
        tv[x] = scale * f;
    }
}

static void lwe_addb(uint64_t* b, size_t count, uint64_t c, uint64_t m) {   /* EvalAddConstEq :230-232 */
    for (size_t g = 0; g < count; ++g) b[g] = (b[g] + c % m) % m;
}
static void lwe_subb(uint64_t* b, size_t count, uint64_t c, uint64_t m) {   /* EvalSubConstEq :244-246 */
    for (size_t g = 0; g < count; ++g) b[g] = (b[g] % m + m - c % m) % m;
}
static void lwe_reduce(const uint64_t* a, const uint64_t* b, uint64_t* ao, uint64_t* bo, size_t count, uint32_t n,
                       uint64_t m) {                                          /* SetModulus, lwe-ciphertext.h:116-120 */
    for (size_t i = 0; i < count * n; ++i) ao[i] = a[i] % m;
    for (size_t g = 0; g < count; ++g) bo[g] = b[g] % m;
}
/* out = x - y mod m (EvalSubEq :234-237 / EvalSubEq2 :239-242); out may alias x or y */
static void lwe_sub(const uint64_t* xa, const uint64_t* xb, const uint64_t* ya, const uint64_t* yb, uint64_t* oa,
                    uint64_t* ob, size_t count, uint32_t n, uint64_t m) {
    for (size_t i = 0; i < count * n; ++i) oa[i] = (xa[i] % m + m - ya[i] % m) % m;
    for (size_t g = 0; g < count; ++g) ob[g] = (xb[g] % m + m - yb[g] % m) % m;
}

static int lut_property(const uint64_t* lut, uint64_t len, uint64_t mod) {  /* checkInputFunction, binfhe-base-scheme.h:245-260 */
    uint64_t mid = len / 2;
    if (lut[0] == mod - lut[mid]) {
        for (uint64_t i = 1; i < mid; ++i) if (lut[i] != mod - lut[mid + i]) return 2;
        return 0;
    }
    if (lut[0] == lut[mid]) {
        for (uint64_t i = 1; i < mid; ++i) if (lut[i] != lut[mid + i]) return 2;
        return 1;
    }
    return 2;
}

#define BETA 128u  /* BinFHEContext::GetBeta, binfhecontext.h:445-447 */

/* EvalFunc (binfhe-base-scheme.cpp:241-337): inputs mod q_in (= LUT length), outputs mod q_in */
int tfo_eval_func_batch(const tfo_params* p, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB,
                        size_t count, const uint64_t* a, const uint64_t* b, uint64_t q_in, const uint64_t* lut,
                        uint64_t* a_out, uint64_t* b_out, int nthreads) {
    const uint32_t n = p->n;
    const int prop = lut_property(lut, q_in, q_in);
    uint64_t* tv = (uint64_t*)malloc(4 * (size_t)p->N * sizeof(uint64_t));
    uint64_t* ta = (uint64_t*)malloc(count * n * sizeof(uint64_t));
    uint64_t* tb = (uint64_t*)malloc(count * sizeof(uint64_t));
    uint64_t* ua = (uint64_t*)malloc(count * n * sizeof(uint64_t));
    uint64_t* ub = (uint64_t*)malloc(count * sizeof(uint64_t));
    int rc = 0;
    memcpy(ta, a, count * n * sizeof(uint64_t));
    memcpy(tb, b, count * sizeof(uint64_t));
    if (prop == 0) {                                   /* negacyclic: one bootstrap :253-259 */
        lwe_addb(tb, count, BETA, q_in);
        make_tv(p, TV_LUT, lut, q_in, q_in, q_in, tv);
        tfo_bootstrap_func_batch(p, bsk, kskA, kskB, count, ta, tb, q_in, tv, q_in, a_out, b_out, nthreads);
    } else if (prop == 2) {                            /* arbitrary :261-312 */
        if (q_in > p->N) { rc = -2; goto done; }
        const uint64_t dq = q_in << 1;
        /* ct1 = ct with a's modulus raised to dq (values unchanged); ct2 = ct1 + beta (mod dq) */
        memcpy(ua, ta, count * n * sizeof(uint64_t));
        memcpy(ub, tb, count * sizeof(uint64_t));
        lwe_addb(ub, count, BETA, dq);
        make_tv(p, TV_HALF, NULL, 0, dq, dq, tv);
        uint64_t* ca = (uint64_t*)malloc(count * n * sizeof(uint64_t));
        uint64_t* cb = (uint64_t*)malloc(count * sizeof(uint64_t));
        tfo_bootstrap_func_batch(p, bsk, kskA, kskB, count, ua, ub, dq, tv, dq, ca, cb, nthreads);  /* ct3 */
        lwe_sub(ta, tb, ca, cb, ca, cb, count, n, dq);  /* EvalSubEq2(ct1, ct3): ct3 = ct1 - ct3 */
        lwe_addb(cb, count, BETA, dq);
        lwe_subb(cb, count, q_in >> 1, dq);
        make_tv(p, TV_LUT_ANTI, lut, q_in, dq, dq, tv);   /* LUT2 = LUT || LUT */
        tfo_bootstrap_func_batch(p, bsk, kskA, kskB, count, ca, cb, dq, tv, dq, ua, ub, nthreads);  /* ct4 */
        lwe_reduce(ua, ub, a_out, b_out, count, n, q_in);   /* ct4->SetModulus(q) */
        free(ca); free(cb);
    } else {                                           /* periodic :315-337 */
        lwe_addb(tb, count, BETA, q_in);
        make_tv(p, TV_HALF, NULL, 0, q_in, q_in, tv);
        tfo_bootstrap_func_batch(p, bsk, kskA, kskB, count, ta, tb, q_in, tv, q_in, ua, ub, nthreads);  /* ct2 */
        lwe_sub(a, b, ua, ub, ua, ub, count, n, q_in);    /* EvalSubEq2(ct, ct2) */
        lwe_addb(ub, count, BETA, q_in);
        lwe_subb(ub, count, q_in >> 2, q_in);
        make_tv(p, TV_LUT_ANTI, lut, q_in, q_in, q_in, tv);
        tfo_bootstrap_func_batch(p, bsk, kskA, kskB, count, ua, ub, q_in, tv, q_in, a_out, b_out, nthreads);
    }
done:
    free(tv); free(ta); free(tb); free(ua); free(ub);
    return rc;
}

/* EvalFloor (:340-378): ct mod `mod` in and out; q' = q (roundbits = 0) or beta 2^(roundbits+1) */
static void eval_floor(const tfo_params* p, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB,
                       size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod, uint32_t roundbits,
                       uint64_t* a_out, uint64_t* b_out, int nthreads) {
    const uint32_t n = p->n;
    const uint64_t qq = roundbits == 0 ? p->q : (uint64_t)BETA << (roundbits + 1);
    uint64_t* tv = (uint64_t*)malloc(4 * (size_t)p->N * sizeof(uint64_t));
    uint64_t* ra = (uint64_t*)malloc(count * n * sizeof(uint64_t));
    uint64_t* rb = (uint64_t*)malloc(count * sizeof(uint64_t));
    uint64_t* sa = (uint64_t*)malloc(count * n * sizeof(uint64_t));
    uint64_t* sb = (uint64_t*)malloc(count * sizeof(uint64_t));
    memcpy(a_out, a, count * n * sizeof(uint64_t));   /* ct1 = ct + beta */
    memcpy(b_out, b, count * sizeof(uint64_t));
    lwe_addb(b_out, count, BETA, mod);
    lwe_reduce(a_out, b_out, ra, rb, count, n, qq);    /* ct1Modq */
    make_tv(p, TV_HALF, NULL, 0, qq, mod, tv);
    tfo_bootstrap_func_batch(p, bsk, kskA, kskB, count, ra, rb, qq, tv, mod, sa, sb, nthreads);   /* ct2 */
    lwe_sub(a_out, b_out, sa, sb, a_out, b_out, count, n, mod);                                   /* ct1 -= ct2 */
    lwe_reduce(a_out, b_out, ra, rb, count, n, qq);    /* ct2Modq */
    make_tv(p, TV_FLOOR2, NULL, 0, qq, mod, tv);
    tfo_bootstrap_func_batch(p, bsk, kskA, kskB, count, ra, rb, qq, tv, mod, sa, sb, nthreads);   /* ct3 */
    lwe_sub(a_out, b_out, sa, sb, a_out, b_out, count, n, mod);                                   /* ct1 -= ct3 */
    free(tv); free(ra); free(rb); free(sa); free(sb);
}

int tfo_eval_floor_batch(const tfo_params* p, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB,
                         size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod, uint32_t roundbits,
                         uint64_t* a_out, uint64_t* b_out, int nthreads) {
    eval_floor(p, bsk, kskA, kskB, count, a, b, mod, roundbits, a_out, b_out, nthreads);
    return 0;
}

/* EvalSign (:381-449) with one bootstrapping key (no dynamic base change): outputs mod q */
int tfo_eval_sign_batch(const tfo_params* p, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB,
                        size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod, int scheme_switch,
                        uint64_t* a_out, uint64_t* b_out, int nthreads) {
    const uint32_t n = p->n;
    const uint64_t q = p->q;
    if (mod <= q) return -2;
    uint64_t* ta = (uint64_t*)malloc(count * n * sizeof(uint64_t));
    uint64_t* tb = (uint64_t*)malloc(count * sizeof(uint64_t));
    uint64_t* fa = (uint64_t*)malloc(count * n * sizeof(uint64_t));
    uint64_t* fb = (uint64_t*)malloc(count * sizeof(uint64_t));
    uint64_t* tv = (uint64_t*)malloc(4 * (size_t)p->N * sizeof(uint64_t));
    memcpy(ta, a, count * n * sizeof(uint64_t));
    memcpy(tb, b, count * sizeof(uint64_t));
    while (mod > q) {
        eval_floor(p, bsk, kskA, kskB, count, ta, tb, mod, 0, fa, fb, nthreads);
        const uint64_t nmod = (mod << 1) * BETA / q;
        tfo_modswitch(mod, nmod, n, count, fa, fb, ta, tb);
        mod = nmod;
    }
    lwe_addb(tb, count, BETA, mod);
    make_tv(p, scheme_switch ? TV_SIGN_SS : TV_SIGN, NULL, 0, mod, q, tv);
    tfo_bootstrap_func_batch(p, bsk, kskA, kskB, count, ta, tb, mod, tv, q, a_out, b_out, nthreads);
    if (!scheme_switch) lwe_subb(b_out, count, q >> 2, q);
    free(ta); free(tb); free(fa); free(fb); free(tv);
    return 0;
}

/* number of ciphertexts EvalDecomp returns for an input modulus */
uint32_t tfo_eval_decomp_parts(const tfo_params* p, uint64_t mod) {
    uint32_t k = 1;
    while (mod > p->q) { ++k; mod = mod / p->q * 2 * BETA; }
    return k;
}

/* EvalDecomp (:452-518): parts k -> a_out [k][count][n], b_out [k][count]; part i < k-1 is mod q */
int tfo_eval_decomp_batch(const tfo_params* p, const uint64_t* bsk, const uint64_t* kskA, const uint64_t* kskB,
                          size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod, uint64_t* a_out,
                          uint64_t* b_out, int nthreads) {
    const uint32_t n = p->n;
    const uint64_t q = p->q;
    if (mod <= q) return -2;
    uint64_t* ta = (uint64_t*)malloc(count * n * sizeof(uint64_t));
    uint64_t* tb = (uint64_t*)malloc(count * sizeof(uint64_t));
    uint64_t* fa = (uint64_t*)malloc(count * n * sizeof(uint64_t));
    uint64_t* fb = (uint64_t*)malloc(count * sizeof(uint64_t));
    memcpy(ta, a, count * n * sizeof(uint64_t));
    memcpy(tb, b, count * sizeof(uint64_t));
    size_t part = 0;
    while (mod > q) {
        lwe_reduce(ta, tb, a_out + part * count * n, b_out + part * count, count, n, q);
        ++part;
        eval_floor(p, bsk, kskA, kskB, count, ta, tb, mod, 0, fa, fb, nthreads);
        const uint64_t nmod = mod / q * 2 * BETA;
        tfo_modswitch(mod, nmod, n, count, fa, fb, ta, tb);
        mod = nmod;
    }
    memcpy(a_out + part * count * n, ta, count * n * sizeof(uint64_t));
    memcpy(b_out + part * count, tb, count * sizeof(uint64_t));
    free(ta); free(tb); free(fa); free(fb);
    return 0;
}

/* Decrypt: lwe-pke.cpp:181-226 with plaintext modulus ptmod; SwitchModulus: mubintvecnat.cpp:109-122 */
int64_t tfo_decrypt_p(const uint64_t* sk, uint64_t skmod, const uint64_t* a, uint64_t b, uint32_t len, uint64_t mod,
                      uint32_t ptmod) {
    uint64_t inner = 0;
    for (uint32_t i = 0; i < len; ++i) {
        uint64_t s = sk[i], sm;
        if (s > (skmod >> 1)) {  /* negative value: (s - skmod) mod `mod` */
            int64_t v = ((int64_t)s - (int64_t)skmod) % (int64_t)mod;
            sm = (uint64_t)(v < 0 ? v + (int64_t)mod : v);
        } else {
            sm = s % mod;
        }
        inner = addmod(inner, mulmod(a[i], sm, mod), mod);
    }
    uint64_t r = submod(b % mod, inner, mod);
    r = addmod(r, mod / (2 * (uint64_t)ptmod), mod);
    return (int64_t)(((unsigned __int128)ptmod * r) / mod);
}

int64_t tfo_decrypt(const uint64_t* sk, uint64_t skmod, const uint64_t* a, uint64_t b, uint32_t len, uint64_t mod) {
    return tfo_decrypt_p(sk, skmod, a, b, len, mod, 4);
}
