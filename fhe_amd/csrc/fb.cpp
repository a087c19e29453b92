// fb.cpp -- functional bootstrapping on the device: BootstrapFunc and the
// EvalFunc / EvalFloor / EvalSign / EvalDecomp compositions of the reference
// (src/binfhe/lib/binfhe-base-scheme.cpp:241-521, 589-648) over batches of ciphertexts that
// stay in HBM.  Every bootstrap is the same prep + blind rotation + key switch launch sequence
// as the gates (bootstrap.hip, keyswitch.hip) with a test-vector table instead of the gate
// window; the LWE additions between bootstraps are element-wise kernels (lwe.hip).  The host
// code here only sequences launches and builds test-vector tables.
#include <algorithm>
#include <vector>

#include "engine.h"
#include "nt.h"

namespace fhe_amd {

namespace {
constexpr uint64_t kBeta = 128;  // BinFHEContext::GetBeta (binfhecontext.h:445-447)

bool pow2(uint64_t x) { return x && !(x & (x - 1)); }

// test-vector functions f(x, q = ctmod, Q = fmod) of the reference's lambdas
enum TvKind { TV_LUT, TV_LUT_ANTI, TV_HALF, TV_FLOOR2, TV_SIGN, TV_SIGN_SS };
std::vector<uint64_t> tv_values(TvKind kind, const uint64_t* lut, uint64_t lutlen, uint64_t q, uint64_t fmod) {
    std::vector<uint64_t> f(q);
    for (uint64_t x = 0; x < q; ++x) {
        switch (kind) {
            case TV_LUT: f[x] = lut[x]; break;                                                       // :254-256
            case TV_LUT_ANTI:                                                                        // :302-307, 324-329
                f[x] = x < (q >> 1) ? lut[x % lutlen] : fmod - lut[(x - q / 2) % lutlen];
                break;
            case TV_HALF: f[x] = x < (q >> 1) ? fmod - (q >> 2) : (q >> 2); break;                  // f0/f1 :285-290
            case TV_FLOOR2:                                                                          // f2 :361-368
                f[x] = x < (q >> 2) ? fmod - (q >> 1) - x : (x < 3 * (q >> 2) ? x : fmod + (q >> 1) - x);
                break;
            case TV_SIGN: f[x] = x < q / 2 ? fmod / 4 : fmod - fmod / 4; break;                      // f3 :413-416
            case TV_SIGN_SS: f[x] = x < q / 2 ? fmod - fmod / 4 : fmod / 4; break;                   // :421-424
        }
    }
    return f;
}

// checkInputFunction (binfhe-base-scheme.h:245-260): 0 negacyclic, 1 periodic, 2 arbitrary
int lut_property(const uint64_t* lut, uint64_t len, uint64_t mod) {
    const uint64_t mid = len / 2;
    if (lut[0] == mod - lut[mid]) {
        for (uint64_t i = 1; i < mid; ++i)
            if (lut[i] != mod - lut[mid + i]) return 2;
        return 0;
    }
    if (lut[0] == lut[mid]) {
        for (uint64_t i = 1; i < mid; ++i)
            if (lut[i] != lut[mid + i]) return 2;
        return 1;
    }
    return 2;
}
}  // namespace

uint64_t* Engine::fb_work(size_t count, int cts) {
    const size_t need = count * (size_t)cts;
    if (need > fbcap_) {
        FHE_HIP_CHECK(hipSetDevice(device_));
        FHE_HIP_CHECK(hipDeviceSynchronize());
        if (d_fb_) FHE_HIP_CHECK(hipFree(d_fb_));
        d_fb_ = nullptr;
        fbcap_ = 0;
        FHE_HIP_CHECK(hipMalloc(&d_fb_, need * ((size_t)p_.n + 1) * 8));
        fbcap_ = need;
    }
    return d_fb_;
}

void Engine::bootstrap_func_device(size_t count, const uint64_t* a, const uint64_t* b, uint32_t ctmod,
                                   const uint64_t* f, uint64_t fmod, uint64_t* a_out, uint64_t* b_out, hipStream_t s) {
    bootstrap_func_tables(count, a, b, ctmod, f, 1, fmod, a_out, b_out, s);
}

// BootstrapFunc (:617-642) with nt tables f[nt][ctmod]: ciphertext g bootstraps with table g % nt
// (GateArgs::tv_mod); outputs mod fmod
void Engine::bootstrap_func_tables(size_t count, const uint64_t* a, const uint64_t* b, uint32_t ctmod,
                                   const uint64_t* f, uint32_t nt, uint64_t fmod, uint64_t* a_out, uint64_t* b_out,
                                   hipStream_t s) {
    if (!ready()) throw std::logic_error("keys not loaded (load_bsk / load_ksk)");
    if (!pow2(ctmod) || ctmod < 4 || ctmod > 2 * p_.N) throw std::invalid_argument("ctmod must be a power of two <= 2N");
    if (fmod < 2 || fmod > (1ull << 40)) throw std::invalid_argument("fmod out of range");
    if (nt < 1 || nt > 4096) throw std::invalid_argument("BootstrapFunc: 1 to 4096 tables");
    if (count == 0) return;
    if (count > 0x7fffffffull) throw std::invalid_argument("batch too large");
    ensure_work(count);
    FHE_HIP_CHECK(hipSetDevice(device_));
    // BootstrapFuncCore (:596-608): m[j * 2N/ctmod] = (Q / fmod) f((b - j) mod ctmod)
    const size_t words = (size_t)nt * ctmod;
    std::vector<uint64_t> tv(words);
    const uint64_t scale = p_.Q / fmod;
    for (size_t x = 0; x < words; ++x) {
        if (f[x] > fmod) throw std::invalid_argument("BootstrapFunc: f(x) exceeds fmod");
        tv[x] = scale * f[x];  // <= Q
    }
    // the table region grows with the number of tables (grow: after the streams' earlier work that reads it)
    const size_t need = std::max<size_t>(words, 2 * (size_t)p_.N);
    // stream-ordered: the copy runs after every earlier launch on s that reads the table
    uint64_t* t = grow(d_tvbuf_, tvcap_, need * (wide_ ? 8 : 4));
    if (wide_) {
        FHE_HIP_CHECK(hipMemcpyAsync(t, tv.data(), words * 8, hipMemcpyHostToDevice, s));
    } else {
        std::vector<uint32_t> tv32(tv.begin(), tv.end());
        FHE_HIP_CHECK(hipMemcpyAsync(t, tv32.data(), words * 4, hipMemcpyHostToDevice, s));
    }
    GateArgs g{};
    g.count = (uint32_t)count;
    g.n = p_.n;
    g.N = p_.N;
    g.q = p_.q;
    g.qKS = p_.qKS;
    g.ctmod = ctmod;
    g.factor = 2 * p_.N / ctmod;
    g.tv = wide_ ? nullptr : reinterpret_cast<const uint32_t*>(t);
    g.tv64 = wide_ ? t : nullptr;
    g.tv_mod = nt;
    g.b_const = 0;  // ctExt = (acc0, acc1[0]) (:624-626)
    g.msb_out = 1;
    g.gbits = p_.gBits;
    GateInputs in{{a, nullptr, nullptr, nullptr}, {b, nullptr, nullptr, nullptr}, 1, 0, 0};
    prep_device(g, in, 0, s);
    rotate_device(g, s);
    keyswitch_ext(count, fmod, a_out, b_out, s);
}

// EvalFunc (:241-337)
void Engine::eval_func_device(size_t count, const uint64_t* a, const uint64_t* b, uint64_t q_in, const uint64_t* lut,
                              uint64_t* a_out, uint64_t* b_out, hipStream_t s) {
    if (!pow2(q_in) || q_in < 4 || q_in > 2 * p_.N) throw std::invalid_argument("EvalFunc: modulus must be a power of two <= 2N");
    if (count == 0) return;
    const size_t n = p_.n;
    uint64_t* w = fb_work(count, 3);
    uint64_t *ta = w, *tb = w + count * n;                       // ct1
    uint64_t *ua = tb + count, *ub = ua + count * n;             // ct2 / ct4
    uint64_t *ca = ub + count, *cb = ca + count * n;             // ct3
    FHE_HIP_CHECK(hipMemcpyAsync(ta, a, count * n * 8, hipMemcpyDeviceToDevice, s));
    FHE_HIP_CHECK(hipMemcpyAsync(tb, b, count * 8, hipMemcpyDeviceToDevice, s));
    const int prop = lut_property(lut, q_in, q_in);
    if (prop == 0) {  // negacyclic: one bootstrap (:253-259)
        FHE_HIP_CHECK(launch_lwe_addb(tb, kBeta % q_in, q_in, count, s));
        auto f = tv_values(TV_LUT, lut, q_in, q_in, q_in);
        bootstrap_func_device(count, ta, tb, (uint32_t)q_in, f.data(), q_in, a_out, b_out, s);
    } else if (prop == 2) {  // arbitrary (:261-312)
        if (q_in > p_.N)
            throw std::invalid_argument("ERROR: ciphertext modulus q needs to be <= ring dimension for arbitrary function evaluation");
        const uint64_t dq = q_in << 1;
        // ct1 = ct with a's modulus raised to dq (values unchanged); ct2 = ct1 + beta mod dq
        FHE_HIP_CHECK(hipMemcpyAsync(ua, ta, count * n * 8, hipMemcpyDeviceToDevice, s));
        FHE_HIP_CHECK(hipMemcpyAsync(ub, tb, count * 8, hipMemcpyDeviceToDevice, s));
        FHE_HIP_CHECK(launch_lwe_addb(ub, kBeta % dq, dq, count, s));
        auto f0 = tv_values(TV_HALF, nullptr, 0, dq, dq);
        bootstrap_func_device(count, ua, ub, (uint32_t)dq, f0.data(), dq, ca, cb, s);  // ct3
        FHE_HIP_CHECK(launch_lwe_sub(ta, tb, ca, cb, ca, cb, dq, (uint32_t)n, count, s));  // EvalSubEq2(ct1, ct3)
        FHE_HIP_CHECK(launch_lwe_addb(cb, kBeta % dq, dq, count, s));
        FHE_HIP_CHECK(launch_lwe_addb(cb, dq - (q_in >> 1), dq, count, s));              // - q/2
        auto f2 = tv_values(TV_LUT_ANTI, lut, q_in, dq, dq);                              // LUT2 = LUT || LUT
        bootstrap_func_device(count, ca, cb, (uint32_t)dq, f2.data(), dq, ua, ub, s);  // ct4
        FHE_HIP_CHECK(launch_lwe_reduce(ua, ub, a_out, b_out, q_in, (uint32_t)n, count, s));  // SetModulus(q)
    } else {  // periodic (:315-337)
        FHE_HIP_CHECK(launch_lwe_addb(tb, kBeta % q_in, q_in, count, s));
        auto f0 = tv_values(TV_HALF, nullptr, 0, q_in, q_in);
        bootstrap_func_device(count, ta, tb, (uint32_t)q_in, f0.data(), q_in, ua, ub, s);  // ct2
        FHE_HIP_CHECK(launch_lwe_sub(a, b, ua, ub, ua, ub, q_in, (uint32_t)n, count, s));   // EvalSubEq2(ct, ct2)
        FHE_HIP_CHECK(launch_lwe_addb(ub, kBeta % q_in, q_in, count, s));
        FHE_HIP_CHECK(launch_lwe_addb(ub, q_in - (q_in >> 2), q_in, count, s));            // - q/4
        auto f1 = tv_values(TV_LUT_ANTI, lut, q_in, q_in, q_in);
        bootstrap_func_device(count, ua, ub, (uint32_t)q_in, f1.data(), q_in, a_out, b_out, s);
    }
}

// EvalFuncMultiOutputBatch (batch.cpp:141-174): the reference runs EvalFunc(ct_i, lut_j) for every pair.
// EvalFunc's first bootstrap (periodic / arbitrary classes, :283-297, :315-323) does not depend on the LUT,
// so it runs once per input and class; the LUT-dependent last bootstrap of a class runs as one launch over
// count x (its LUTs) ciphertexts with a test-vector table per LUT (bootstrap_func_tables).  Every output is
// the value EvalFunc(ct_i, lut_j) computes: the same bootstraps on the same inputs.
void Engine::eval_func_multi_device(size_t count, const uint64_t* a, const uint64_t* b, uint64_t q_in,
                                    const uint64_t* luts, uint32_t nl, uint64_t* a_out, uint64_t* b_out,
                                    hipStream_t s) {
    if (!pow2(q_in) || q_in < 4 || q_in > 2 * p_.N) throw std::invalid_argument("EvalFunc: modulus must be a power of two <= 2N");
    if (nl == 0 || nl > 4096) throw std::invalid_argument("EvalFuncMultiOutput: 1 to 4096 LUTs");
    if (count == 0) return;
    if (count * nl > 0x7fffffffull) throw std::invalid_argument("batch too large");
    const size_t n = p_.n;
    std::vector<int> cls(nl);
    for (uint32_t j = 0; j < nl; ++j) cls[j] = lut_property(luts + (size_t)j * q_in, q_in, q_in);
    for (uint32_t j = 0; j < nl; ++j)
        if (cls[j] == 2 && q_in > p_.N)
            throw std::invalid_argument("ERROR: ciphertext modulus q needs to be <= ring dimension for arbitrary function evaluation");
    size_t maxg = 0;
    for (int c = 0; c < 3; ++c) maxg = std::max<size_t>(maxg, (size_t)std::count(cls.begin(), cls.end(), c));
    // temporaries (ciphertext slots of n + 1 words): t, u (count each), the repeated inputs and, when the
    // LUTs split into classes, the class's outputs (count x maxg each)
    const bool split = maxg < nl;
    uint64_t* w = fb_work(count, (int)(2 + maxg * (split ? 2 : 1)));
    uint64_t *ta = w, *tb = ta + count * n, *ua = tb + count, *ub = ua + count * n;
    uint64_t *ra = ub + count, *rb = ra + count * maxg * n;
    uint64_t *oa = rb + count * maxg, *ob = oa + count * maxg * n;
    for (int c = 0; c < 3; ++c) {
        std::vector<uint32_t> js;
        for (uint32_t j = 0; j < nl; ++j)
            if (cls[j] == c) js.push_back(j);
        if (js.empty()) continue;
        const uint32_t lg = (uint32_t)js.size();
        const uint64_t cm = c == 2 ? q_in << 1 : q_in;   // the last bootstrap's ciphertext modulus (:299-310)
        uint64_t* xa = split ? oa : a_out;
        uint64_t* xb = split ? ob : b_out;
        FHE_HIP_CHECK(hipMemcpyAsync(ta, a, count * n * 8, hipMemcpyDeviceToDevice, s));
        FHE_HIP_CHECK(hipMemcpyAsync(tb, b, count * 8, hipMemcpyDeviceToDevice, s));
        std::vector<uint64_t> f((size_t)lg * cm);
        if (c == 0) {  // negacyclic (:253-259): ct + beta, one bootstrap with the LUT itself
            FHE_HIP_CHECK(launch_lwe_addb(tb, kBeta % q_in, q_in, count, s));
            for (uint32_t k = 0; k < lg; ++k) {
                auto t = tv_values(TV_LUT, luts + (size_t)js[k] * q_in, q_in, q_in, q_in);
                std::copy(t.begin(), t.end(), f.begin() + (size_t)k * cm);
            }
            FHE_HIP_CHECK(launch_lwe_repeat(ta, tb, (uint32_t)n, count, lg, ra, rb, s));
            bootstrap_func_tables(count * lg, ra, rb, (uint32_t)q_in, f.data(), lg, q_in, xa, xb, s);
        } else if (c == 1) {  // periodic (:315-337)
            FHE_HIP_CHECK(launch_lwe_addb(tb, kBeta % q_in, q_in, count, s));
            auto f0 = tv_values(TV_HALF, nullptr, 0, q_in, q_in);
            bootstrap_func_device(count, ta, tb, (uint32_t)q_in, f0.data(), q_in, ua, ub, s);  // ct2, shared
            FHE_HIP_CHECK(launch_lwe_sub(a, b, ua, ub, ua, ub, q_in, (uint32_t)n, count, s));   // EvalSubEq2(ct, ct2)
            FHE_HIP_CHECK(launch_lwe_addb(ub, kBeta % q_in, q_in, count, s));
            FHE_HIP_CHECK(launch_lwe_addb(ub, q_in - (q_in >> 2), q_in, count, s));            // - q/4
            for (uint32_t k = 0; k < lg; ++k) {
                auto t = tv_values(TV_LUT_ANTI, luts + (size_t)js[k] * q_in, q_in, q_in, q_in);
                std::copy(t.begin(), t.end(), f.begin() + (size_t)k * cm);
            }
            FHE_HIP_CHECK(launch_lwe_repeat(ua, ub, (uint32_t)n, count, lg, ra, rb, s));
            bootstrap_func_tables(count * lg, ra, rb, (uint32_t)q_in, f.data(), lg, q_in, xa, xb, s);
        } else {  // arbitrary (:261-312)
            const uint64_t dq = cm;
            FHE_HIP_CHECK(hipMemcpyAsync(ua, ta, count * n * 8, hipMemcpyDeviceToDevice, s));
            FHE_HIP_CHECK(hipMemcpyAsync(ub, tb, count * 8, hipMemcpyDeviceToDevice, s));
            FHE_HIP_CHECK(launch_lwe_addb(ub, kBeta % dq, dq, count, s));
            auto f0 = tv_values(TV_HALF, nullptr, 0, dq, dq);
            bootstrap_func_device(count, ua, ub, (uint32_t)dq, f0.data(), dq, ua, ub, s);     // ct3, shared
            FHE_HIP_CHECK(launch_lwe_sub(ta, tb, ua, ub, ua, ub, dq, (uint32_t)n, count, s));  // EvalSubEq2(ct1, ct3)
            FHE_HIP_CHECK(launch_lwe_addb(ub, kBeta % dq, dq, count, s));
            FHE_HIP_CHECK(launch_lwe_addb(ub, dq - (q_in >> 1), dq, count, s));              // - q/2
            for (uint32_t k = 0; k < lg; ++k) {
                auto t = tv_values(TV_LUT_ANTI, luts + (size_t)js[k] * q_in, q_in, dq, dq);
                std::copy(t.begin(), t.end(), f.begin() + (size_t)k * cm);
            }
            FHE_HIP_CHECK(launch_lwe_repeat(ua, ub, (uint32_t)n, count, lg, ra, rb, s));
            bootstrap_func_tables(count * lg, ra, rb, (uint32_t)dq, f.data(), lg, dq, ra, rb, s);  // ct4
            FHE_HIP_CHECK(launch_lwe_reduce(ra, rb, xa, xb, q_in, (uint32_t)n, count * lg, s));   // SetModulus(q)
        }
        if (split)  // row i lg + k of the class -> row i nl + js[k]
            for (uint32_t k = 0; k < lg; ++k) {
                FHE_HIP_CHECK(hipMemcpy2DAsync(a_out + (size_t)js[k] * n, (size_t)nl * n * 8, oa + (size_t)k * n,
                                               (size_t)lg * n * 8, n * 8, count, hipMemcpyDeviceToDevice, s));
                FHE_HIP_CHECK(hipMemcpy2DAsync(b_out + js[k], (size_t)nl * 8, ob + k, (size_t)lg * 8, 8, count,
                                               hipMemcpyDeviceToDevice, s));
            }
    }
}

// EvalFloor (:340-378) with caller-provided temporaries w (2 ciphertext arrays)
void Engine::fb_floor(size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod, uint32_t roundbits,
                      uint64_t* a_out, uint64_t* b_out, uint64_t* w, hipStream_t s) {
    const size_t n = p_.n;
    const uint64_t qq = roundbits == 0 ? p_.q : kBeta << (roundbits + 1);
    if (!pow2(qq) || qq > 2 * p_.N || qq > mod) throw std::invalid_argument("EvalFloor: roundbits out of range");
    uint64_t *ra = w, *rb = w + count * n, *sa = rb + count, *sb = sa + count * n;
    if (a_out != a) FHE_HIP_CHECK(hipMemcpyAsync(a_out, a, count * n * 8, hipMemcpyDeviceToDevice, s));
    if (b_out != b) FHE_HIP_CHECK(hipMemcpyAsync(b_out, b, count * 8, hipMemcpyDeviceToDevice, s));
    FHE_HIP_CHECK(launch_lwe_addb(b_out, kBeta, mod, count, s));                                    // ct1 = ct + beta
    FHE_HIP_CHECK(launch_lwe_reduce(a_out, b_out, ra, rb, qq, (uint32_t)n, count, s));              // ct1Modq
    auto f1 = tv_values(TV_HALF, nullptr, 0, qq, mod);
    bootstrap_func_device(count, ra, rb, (uint32_t)qq, f1.data(), mod, sa, sb, s);                  // ct2
    FHE_HIP_CHECK(launch_lwe_sub(a_out, b_out, sa, sb, a_out, b_out, mod, (uint32_t)n, count, s));  // ct1 -= ct2
    FHE_HIP_CHECK(launch_lwe_reduce(a_out, b_out, ra, rb, qq, (uint32_t)n, count, s));              // ct2Modq
    auto f2 = tv_values(TV_FLOOR2, nullptr, 0, qq, mod);
    bootstrap_func_device(count, ra, rb, (uint32_t)qq, f2.data(), mod, sa, sb, s);                  // ct3
    FHE_HIP_CHECK(launch_lwe_sub(a_out, b_out, sa, sb, a_out, b_out, mod, (uint32_t)n, count, s));  // ct1 -= ct3
}

void Engine::eval_floor_device(size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod, uint32_t roundbits,
                               uint64_t* a_out, uint64_t* b_out, hipStream_t s) {
    if (!pow2(mod) || mod > (1ull << 31)) throw std::invalid_argument("EvalFloor: modulus must be a power of two <= 2^31");
    if (count == 0) return;
    fb_floor(count, a, b, mod, roundbits, a_out, b_out, fb_work(count, 2), s);
}

// timeOptimization (:409-431, :498-514): after each ModSwitch the running modulus picks the base,
// 2^27 up to 2^17, 2^18 up to 2^26, else unchanged (binLog = log2(mod): mod is a power of two)
void Engine::dynamic_base(uint64_t mod) {
    if (!p_.timeopt) return;
    const uint32_t binLog = 63 - __builtin_clzll(mod);
    if (binLog <= 17) set_base(1u << 27);
    else if (binLog <= 26) set_base(1u << 18);
}

// EvalSign (:381-449), outputs mod q; the bootstrapping key changes with the modulus under
// timeOptimization
void Engine::eval_sign_device(size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod, bool scheme_switch,
                              uint64_t* a_out, uint64_t* b_out, hipStream_t s) {
    const uint64_t q = p_.q;
    if (mod <= q) throw std::invalid_argument("ERROR: EvalSign is only for large precision. For small precision, please use bootstrapping directly");
    if (!pow2(mod) || mod > (1ull << 31)) throw std::invalid_argument("EvalSign: modulus must be a power of two <= 2^31");
    if (count == 0) return;
    const size_t n = p_.n;
    uint64_t* w = fb_work(count, 4);
    uint64_t *ta = w, *tb = w + count * n, *fa = tb + count, *fb = fa + count * n, *tmp = fb + count;
    FHE_HIP_CHECK(hipMemcpyAsync(ta, a, count * n * 8, hipMemcpyDeviceToDevice, s));
    FHE_HIP_CHECK(hipMemcpyAsync(tb, b, count * 8, hipMemcpyDeviceToDevice, s));
    BaseGuard restore{this};
    while (mod > q) {
        fb_floor(count, ta, tb, mod, 0, fa, fb, tmp, s);
        const uint64_t nmod = (mod << 1) * kBeta / q;
        FHE_HIP_CHECK(launch_modswitch(mod, nmod, (uint32_t)n, (uint32_t)count, fa, fb, ta, tb, s));
        mod = nmod;
        dynamic_base(mod);
    }
    FHE_HIP_CHECK(launch_lwe_addb(tb, kBeta % mod, mod, count, s));
    auto f3 = tv_values(scheme_switch ? TV_SIGN_SS : TV_SIGN, nullptr, 0, mod, q);
    bootstrap_func_device(count, ta, tb, (uint32_t)mod, f3.data(), q, a_out, b_out, s);
    if (!scheme_switch) FHE_HIP_CHECK(launch_lwe_addb(b_out, q - (q >> 2), q, count, s));  // - q/4
}

uint32_t Engine::eval_decomp_parts(uint64_t mod) const {
    uint32_t k = 1;
    while (mod > p_.q) {
        ++k;
        mod = mod / p_.q * 2 * kBeta;
    }
    return k;
}

// EvalDecomp (:452-518): part i < parts-1 is the running ciphertext reduced mod q; the last part
// is the final running ciphertext (its own modulus)
void Engine::eval_decomp_device(size_t count, const uint64_t* a, const uint64_t* b, uint64_t mod, uint64_t* a_out,
                                uint64_t* b_out, hipStream_t s) {
    const uint64_t q = p_.q;
    if (mod <= q) throw std::invalid_argument("ERROR: EvalDecomp is only for large precision. For small precision, please use bootstrapping directly");
    if (!pow2(mod) || mod > (1ull << 31)) throw std::invalid_argument("EvalDecomp: modulus must be a power of two <= 2^31");
    if (count == 0) return;
    const size_t n = p_.n;
    uint64_t* w = fb_work(count, 4);
    uint64_t *ta = w, *tb = w + count * n, *fa = tb + count, *fb = fa + count * n, *tmp = fb + count;
    FHE_HIP_CHECK(hipMemcpyAsync(ta, a, count * n * 8, hipMemcpyDeviceToDevice, s));
    FHE_HIP_CHECK(hipMemcpyAsync(tb, b, count * 8, hipMemcpyDeviceToDevice, s));
    size_t part = 0;
    BaseGuard restore{this};
    while (mod > q) {
        FHE_HIP_CHECK(launch_lwe_reduce(ta, tb, a_out + part * count * n, b_out + part * count, q, (uint32_t)n, count, s));
        ++part;
        fb_floor(count, ta, tb, mod, 0, fa, fb, tmp, s);
        const uint64_t nmod = mod / q * 2 * kBeta;
        FHE_HIP_CHECK(launch_modswitch(mod, nmod, (uint32_t)n, (uint32_t)count, fa, fb, ta, tb, s));
        mod = nmod;
        dynamic_base(mod);
    }
    FHE_HIP_CHECK(hipMemcpyAsync(a_out + part * count * n, ta, count * n * 8, hipMemcpyDeviceToDevice, s));
    FHE_HIP_CHECK(hipMemcpyAsync(b_out + part * count, tb, count * 8, hipMemcpyDeviceToDevice, s));
}

void Engine::fb_host(int op, size_t count, const uint64_t* a, const uint64_t* b, uint64_t arg, uint64_t arg2,
                     uint32_t iarg, const uint64_t* lut, uint64_t* a_out, uint64_t* b_out) {
    if (!ready()) throw std::logic_error("keys not loaded (load_bsk / load_ksk)");
    if (count == 0) return;
    const size_t n = p_.n;
    const size_t parts = op == 3 ? eval_decomp_parts(arg) : op == 5 ? iarg : 1;
    FHE_HIP_CHECK(hipSetDevice(device_));
    uint64_t* d = nullptr;
    FHE_HIP_CHECK(hipMalloc(&d, count * (n + 1) * (1 + parts) * 8));
    try {
        uint64_t *da = d, *db = d + count * n, *oa = db + count, *ob = oa + parts * count * n;
        FHE_HIP_CHECK(hipMemcpyAsync(da, a, count * n * 8, hipMemcpyHostToDevice, stream_));
        FHE_HIP_CHECK(hipMemcpyAsync(db, b, count * 8, hipMemcpyHostToDevice, stream_));
        switch (op) {
            case 0: eval_func_device(count, da, db, arg, lut, oa, ob, stream_); break;
            case 1: eval_floor_device(count, da, db, arg, iarg, oa, ob, stream_); break;
            case 2: eval_sign_device(count, da, db, arg, iarg != 0, oa, ob, stream_); break;
            case 3: eval_decomp_device(count, da, db, arg, oa, ob, stream_); break;
            case 4: bootstrap_func_device(count, da, db, (uint32_t)arg, lut, arg2, oa, ob, stream_); break;
            case 5: eval_func_multi_device(count, da, db, arg, lut, iarg, oa, ob, stream_); break;
            default: throw std::invalid_argument("unknown functional-bootstrapping op");
        }
        FHE_HIP_CHECK(hipMemcpyAsync(a_out, oa, parts * count * n * 8, hipMemcpyDeviceToHost, stream_));
        FHE_HIP_CHECK(hipMemcpyAsync(b_out, ob, parts * count * 8, hipMemcpyDeviceToHost, stream_));
        FHE_HIP_CHECK(hipStreamSynchronize(stream_));
    } catch (...) {
        (void)hipStreamSynchronize(stream_);
        (void)hipFree(d);
        throw;
    }
    FHE_HIP_CHECK(hipFree(d));
}

}  // namespace fhe_amd
