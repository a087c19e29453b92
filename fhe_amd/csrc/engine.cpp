// engine.cpp -- see engine.h.
#include "engine.h"

#include <algorithm>

#include "nt.h"

namespace fhe_amd {

namespace {
inline uint32_t to_mont(uint64_t x, uint64_t Q) { return (uint32_t)(((u128)(x % Q) << 32) % Q); }
inline uint32_t neg_inv32(uint32_t Q) {  // -Q^-1 mod 2^32 (Newton)
    uint32_t x = Q;                        // Q * Q = 1 mod 8
    for (int i = 0; i < 5; ++i) x *= 2 - Q * x;
    return (uint32_t)(0u - x);
}
}  // namespace

Engine::Engine(int paramset, int method, int device) : p_(make_params(paramset, method)), device_(device) {
    if (p_.N != 1024) throw std::invalid_argument("device path supports ring dimension N = 1024 (STD128 sets)");
    if (p_.Q >= (1ull << 28)) throw std::invalid_argument("device path needs Q < 2^28");
    if (p_.qKS & (p_.qKS - 1)) throw std::invalid_argument("device path needs a power-of-two qKS");
    if (p_.q & (p_.q - 1)) throw std::invalid_argument("device path needs a power-of-two q");
    if (p_.digitsG != 3) throw std::invalid_argument("device path expects digitsG = 3");
    if (p_.method == M_GINX && ((2 * p_.N / p_.q) & 1))
        throw std::invalid_argument("GINX device path needs an even 2N/q (monomial table)");
    FHE_HIP_CHECK(hipSetDevice(device_));
    FHE_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    build_tables();
    maxops_ = p_.N + p_.n + 128;
}

Engine::~Engine() {
    (void)hipSetDevice(device_);
    if (stream_) (void)hipStreamSynchronize(stream_);
    for (void* ptr : {(void*)d_tables_, d_bsk_, (void*)d_ksk_, (void*)d_idx_, (void*)d_tvb_, (void*)d_ext_a_,
                      (void*)d_ext_b_, (void*)d_io_, (void*)d_logGen_, (void*)d_ops_, (void*)d_nops_,
                      (void*)d_scratch_})
        if (ptr) (void)hipFree(ptr);
    if (stream_) (void)hipStreamDestroy(stream_);
}

void Engine::build_tables() {
    const uint64_t Q = p_.Q;
    HostNtt h;
    h.init(p_.N, Q, p_.psi);
    std::vector<uint32_t> t(32 + 32 + 992 + 992 + 2176, 0);
    uint32_t* twAf = t.data();
    uint32_t* twAi = twAf + 32;
    uint32_t* twBf = twAi + 32;
    uint32_t* twBi = twBf + 992;
    uint32_t* mono = twBi + 992;
    for (int i = 0; i < 32; ++i) {
        twAf[i] = to_mont(h.tab[i], Q);
        twAi[i] = to_mont(h.tabI[i], Q);
    }
    // lane-major tables of the stages on bits 4..0 (bootstrap.hip, twb_off)
    for (int b = 4; b >= 0; --b) {
        const int per = 1 << (4 - b), off = 32 * (per - 1);
        for (int k = 0; k < per; ++k)
            for (int l = 0; l < 32; ++l) {
                const size_t idx = (size_t)(1 << (9 - b)) + (size_t)l * per + k;
                twBf[off + k * 32 + l] = to_mont(h.tab[idx], Q);
                twBi[off + k * 32 + l] = to_mont(h.tabI[idx], Q);
            }
    }
    // EVAL(X^m - 1) at slot j = omega_j^m - 1 with omega_j = psi^(2 brv(j) + 1).  GINX exponents
    // are even (m = a_i * 2N/q), so the table holds psi^(2f) - 1 for f in [0, 2N], entry f at
    // f + (f >> 5) (bootstrap.hip, monomial addressing).
    {
        const uint64_t psi2 = mulmod(p_.psi, p_.psi, Q);
        uint64_t x = 1;
        for (uint32_t f = 0; f <= 2 * p_.N; ++f) {
            mono[f + (f >> 5)] = to_mont(submod(x, 1, Q), Q);
            x = mulmod(x, psi2, Q);
        }
    }
    if (p_.method == M_LMKCDEY) {  // rgsw-cryptoparameters.cpp:115-127
        const uint32_t M = 2 * p_.N;
        std::vector<int16_t> lg(M, 0);
        uint32_t gp = 1;
        lg[M - gp] = (int16_t)M;
        for (uint32_t i = 1; i < p_.N / 2; ++i) {
            gp = (gp * 5) % M;
            lg[gp] = (int16_t)i;
            lg[M - gp] = (int16_t)-(int32_t)i;
        }
        FHE_HIP_CHECK(hipMalloc(&d_logGen_, M * sizeof(int16_t)));
        FHE_HIP_CHECK(hipMemcpy(d_logGen_, lg.data(), M * sizeof(int16_t), hipMemcpyHostToDevice));
    }
    FHE_HIP_CHECK(hipMalloc(&d_tables_, t.size() * 4));
    FHE_HIP_CHECK(hipMemcpy(d_tables_, t.data(), t.size() * 4, hipMemcpyHostToDevice));
    const uint32_t* d = static_cast<const uint32_t*>(d_tables_);
    tabs_.twA_fwd = d;
    tabs_.twA_inv = d + 32;
    tabs_.twB_fwd = d + 64;
    tabs_.twB_inv = d + 64 + 992;
    tabs_.mono = d + 64 + 1984;  // 2176 words
    tabs_.Q = (uint32_t)Q;
    tabs_.Q2 = (uint32_t)(2 * Q);
    tabs_.qinv = neg_inv32((uint32_t)Q);
    tabs_.ninvR = to_mont(h.ninv, Q);
    tabs_.w1ninvR = to_mont(mulmod(h.tabI[1], h.ninv, Q), Q);
}

void Engine::load_bsk(const uint64_t* bsk, size_t words) {
    if (!bsk) throw std::invalid_argument("bsk is null");
    if (words != p_.bsk_words()) throw std::invalid_argument("bsk has wrong length");
    const uint32_t n = p_.n, N = p_.N, dG2 = p_.digitsG2;
    const uint64_t Q = p_.Q;
    if (dG2 != 4) throw std::invalid_argument("device path expects digitsG = 3");
    // device uint2 blocks [..][d][16][64 lanes]: lane = h*32 + l holds slots l*32 + 2k, +1 of
    // component h -- one 512-byte coalesced load per wave-instruction in the kernels.
    //   GINX   raw [n][2][dG2][2][N]                 -> [n][2][dG2][16][64]
    //   LMKCDEY raw [n][dG2][2][N] ++ [nA+1][2][2][N] -> [n][dG2][16][64] ++ [nA+1][2][16][64]
    const size_t nrgsw = p_.method == M_GINX ? (size_t)n * 2 : (size_t)n;  // RGSW keys of dG2 rows
    const size_t nauto = p_.method == M_GINX ? 0 : (size_t)p_.numAutoKeys + 1;
    const uint32_t dA = p_.digitsG - 1;
    std::vector<uint32_t> dev(nrgsw * dG2 * 2 * N + nauto * dA * 2 * N);
    auto pack = [&](const uint64_t* src_key, uint32_t rows, uint32_t* dst_key) {
        for (uint32_t d = 0; d < rows; ++d)
            for (uint32_t k = 0; k < 16; ++k)
                for (uint32_t lane = 0; lane < 64; ++lane) {
                    const uint32_t h = lane >> 5, l = lane & 31;
                    const size_t src = ((size_t)d * 2 + h) * N + l * 32 + 2 * k;
                    const size_t dst = (((size_t)d * 16 + k) * 64 + lane) * 2;
                    dst_key[dst] = to_mont(src_key[src] % Q, Q);
                    dst_key[dst + 1] = to_mont(src_key[src + 1] % Q, Q);
                }
    };
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)nrgsw; ++i)
        pack(bsk + (size_t)i * dG2 * 2 * N, dG2, dev.data() + (size_t)i * dG2 * 2 * N);
    const uint64_t* asrc = bsk + nrgsw * dG2 * 2 * N;
    uint32_t* adst = dev.data() + nrgsw * dG2 * 2 * N;
    for (size_t t = 0; t < nauto; ++t) pack(asrc + t * dA * 2 * N, dA, adst + t * dA * 2 * N);
    for (size_t i = 0; i < words; ++i)
        if (bsk[i] >= Q) throw std::invalid_argument("bsk coefficient not reduced mod Q");
    FHE_HIP_CHECK(hipSetDevice(device_));
    if (d_bsk_) FHE_HIP_CHECK(hipFree(d_bsk_));
    d_bsk_ = nullptr;
    FHE_HIP_CHECK(hipMalloc(&d_bsk_, dev.size() * 4));
    FHE_HIP_CHECK(hipMemcpy(d_bsk_, dev.data(), dev.size() * 4, hipMemcpyHostToDevice));
    d_autok_ = static_cast<uint32_t*>(d_bsk_) + nrgsw * dG2 * 2 * N;
}

void Engine::load_ksk(const uint64_t* A, size_t nA, const uint64_t* B, size_t nB) {
    if (!A || !B) throw std::invalid_argument("ksk is null");
    const size_t rows = p_.ksk_rows();
    if (nA != rows * p_.n || nB != rows) throw std::invalid_argument("ksk has wrong length");
    std::vector<uint16_t> dev(rows * 512, 0);
    bool bad = false;
#pragma omp parallel for schedule(static) reduction(|| : bad)
    for (int64_t r = 0; r < (int64_t)rows; ++r) {
        for (uint32_t k = 0; k < p_.n; ++k) {
            const uint64_t v = A[(size_t)r * p_.n + k];
            bad = bad || v >= p_.qKS;
            dev[(size_t)r * 512 + k] = (uint16_t)v;
        }
        bad = bad || B[r] >= p_.qKS;
        dev[(size_t)r * 512 + p_.n] = (uint16_t)B[r];
    }
    if (bad) throw std::invalid_argument("ksk value not reduced mod qKS");
    FHE_HIP_CHECK(hipSetDevice(device_));
    if (d_ksk_) FHE_HIP_CHECK(hipFree(d_ksk_));
    d_ksk_ = nullptr;
    FHE_HIP_CHECK(hipMalloc(&d_ksk_, dev.size() * 2));
    FHE_HIP_CHECK(hipMemcpy(d_ksk_, dev.data(), dev.size() * 2, hipMemcpyHostToDevice));
}

GateArgs Engine::gate_args(int gate, size_t count) const {
    switch (gate) {
        case G_OR: case G_AND: case G_NOR: case G_NAND: case G_XOR: case G_XNOR: case G_XOR_FAST: case G_XNOR_FAST:
            break;
        default:
            throw std::invalid_argument("EvalBinGate: only 2-input gates (OR AND NOR NAND XOR XNOR) are supported");
    }
    if (count > 0x7fffffffull) throw std::invalid_argument("batch too large");
    GateArgs g{};
    g.count = (uint32_t)count;
    g.n = p_.n;
    g.N = p_.N;
    g.q = p_.q;
    g.qKS = p_.qKS;
    // BootstrapGateCore window (binfhe-base-scheme.cpp:535-553), p = 4
    const uint64_t q = p_.q, qHalf = q >> 1, Q = p_.Q;
    const uint64_t q1 = p_.gate_const(gate), q2 = (q1 + qHalf) % q;
    const bool swap = q1 >= q2;
    g.lb = (uint32_t)(swap ? q2 : q1);
    g.ub = (uint32_t)(swap ? q1 : q2);
    const uint64_t Q2p = Q / 8 + 1, Q2pNeg = Q - Q2p;
    g.lv = (uint32_t)(swap ? Q2p : Q2pNeg);
    g.uv = (uint32_t)(swap ? Q2pNeg : Q2p);
    g.factor = (uint32_t)(p_.N / qHalf);
    g.b_const = (uint32_t)((Q >> 3) + 1);
    g.xor_double = (gate == G_XOR || gate == G_XNOR || gate == G_XOR_FAST || gate == G_XNOR_FAST) ? 1 : 0;
    g.msb_out = 1;
    g.gbits = p_.gBits;
    return g;
}

void Engine::ensure_work(size_t count) {
    if (count <= cap_) return;
    FHE_HIP_CHECK(hipSetDevice(device_));
    FHE_HIP_CHECK(hipStreamSynchronize(stream_));
    for (void* ptr : {(void*)d_idx_, (void*)d_tvb_, (void*)d_ext_a_, (void*)d_ext_b_})
        if (ptr) FHE_HIP_CHECK(hipFree(ptr));
    d_idx_ = nullptr; d_tvb_ = nullptr; d_ext_a_ = nullptr; d_ext_b_ = nullptr; cap_ = 0;
    FHE_HIP_CHECK(hipMalloc(&d_idx_, count * p_.n * sizeof(uint16_t)));
    FHE_HIP_CHECK(hipMalloc(&d_tvb_, count * sizeof(uint32_t)));
    FHE_HIP_CHECK(hipMalloc(&d_ext_a_, count * p_.N * sizeof(uint32_t)));
    FHE_HIP_CHECK(hipMalloc(&d_ext_b_, count * sizeof(uint32_t)));
    if (p_.method == M_LMKCDEY) {
        for (void* ptr : {(void*)d_ops_, (void*)d_nops_, (void*)d_scratch_})
            if (ptr) FHE_HIP_CHECK(hipFree(ptr));
        d_ops_ = nullptr; d_nops_ = nullptr; d_scratch_ = nullptr;
        FHE_HIP_CHECK(hipMalloc(&d_ops_, count * maxops_ * sizeof(uint16_t)));
        FHE_HIP_CHECK(hipMalloc(&d_nops_, count * sizeof(uint32_t)));
        FHE_HIP_CHECK(hipMalloc(&d_scratch_, count * (p_.N + p_.n) * sizeof(uint16_t)));
    }
    cap_ = count;
}

void Engine::ensure_host_stage(size_t count) {
    if (count <= hcap_) return;
    FHE_HIP_CHECK(hipSetDevice(device_));
    FHE_HIP_CHECK(hipStreamSynchronize(stream_));
    if (d_io_) FHE_HIP_CHECK(hipFree(d_io_));
    d_io_ = nullptr;
    hcap_ = 0;
    const size_t words = count * (2 * (size_t)p_.n + 2 + p_.N + 1);
    FHE_HIP_CHECK(hipMalloc(&d_io_, words * 8));
    hcap_ = count;
}

void Engine::bootstrap_device(int gate, size_t count, const uint64_t* a1, const uint64_t* b1, const uint64_t* a2,
                              const uint64_t* b2, bool modswitch, hipStream_t s) {
    if (!d_bsk_) throw std::logic_error("bootstrapping key not loaded");
    GateArgs g = gate_args(gate, count);
    g.msb_out = modswitch ? 1 : 0;
    if (count == 0) return;
    ensure_work(count);
    FHE_HIP_CHECK(hipSetDevice(device_));
    if (p_.method == M_GINX) {
        FHE_HIP_CHECK(launch_prep_ginx(g, a1, b1, a2, b2, d_idx_, d_tvb_, s));
        FHE_HIP_CHECK(launch_blind_rotate_ginx(g, tabs_, d_bsk_, d_idx_, d_tvb_, d_ext_a_, d_ext_b_, s));
    } else {
        FHE_HIP_CHECK(launch_prep_lmk(g, a1, b1, a2, b2, d_logGen_, d_scratch_, d_ops_, d_nops_, d_tvb_, maxops_,
                                      p_.numAutoKeys, s));
        FHE_HIP_CHECK(launch_blind_rotate_lmk(g, tabs_, d_bsk_, d_autok_, d_ops_, d_nops_, maxops_, d_tvb_, d_ext_a_,
                                              d_ext_b_, s));
    }
}

void Engine::keyswitch_workspace_device(size_t count, uint64_t* a_out, uint64_t* b_out, hipStream_t s) {
    if (!d_ksk_) throw std::logic_error("key-switching key not loaded");
    if (count == 0) return;
    if (count > cap_) throw std::logic_error("workspace holds fewer ciphertexts than requested");
    GateArgs g = gate_args(G_AND, count);
    FHE_HIP_CHECK(hipSetDevice(device_));
    FHE_HIP_CHECK(launch_keyswitch(g, p_.baseKS, p_.digitsKS, d_ksk_, d_ext_a_, d_ext_b_, p_.q, a_out, b_out, s));
}

void Engine::eval_gate_device(int gate, size_t count, const uint64_t* a1, const uint64_t* b1, const uint64_t* a2,
                              const uint64_t* b2, uint64_t* a_out, uint64_t* b_out, hipStream_t s) {
    if (!ready()) throw std::logic_error("keys not loaded (load_bsk / load_ksk)");
    if (count == 0) return;
    bootstrap_device(gate, count, a1, b1, a2, b2, true, s);
    keyswitch_workspace_device(count, a_out, b_out, s);
}

void Engine::eval_gate_host(int gate, size_t count, const uint64_t* a1, const uint64_t* b1, const uint64_t* a2,
                            const uint64_t* b2, uint64_t* a_out, uint64_t* b_out) {
    if (count == 0) return;
    ensure_host_stage(count);
    const size_t n = p_.n;
    uint64_t* da1 = d_io_;
    uint64_t* db1 = da1 + count * n;
    uint64_t* da2 = db1 + count;
    uint64_t* db2 = da2 + count * n;
    uint64_t* dao = db2 + count;
    uint64_t* dbo = dao + count * p_.N;
    FHE_HIP_CHECK(hipSetDevice(device_));
    FHE_HIP_CHECK(hipMemcpyAsync(da1, a1, count * n * 8, hipMemcpyHostToDevice, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(db1, b1, count * 8, hipMemcpyHostToDevice, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(da2, a2, count * n * 8, hipMemcpyHostToDevice, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(db2, b2, count * 8, hipMemcpyHostToDevice, stream_));
    eval_gate_device(gate, count, da1, db1, da2, db2, dao, dbo, stream_);
    FHE_HIP_CHECK(hipMemcpyAsync(a_out, dao, count * n * 8, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(b_out, dbo, count * 8, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipStreamSynchronize(stream_));
}

void Engine::bootstrap_extended_host(int gate, size_t count, const uint64_t* a1, const uint64_t* b1,
                                     const uint64_t* a2, const uint64_t* b2, uint64_t* ext_a, uint64_t* ext_b) {
    if (count == 0) return;
    ensure_host_stage(count);
    const size_t n = p_.n, N = p_.N;
    uint64_t* da1 = d_io_;
    uint64_t* db1 = da1 + count * n;
    uint64_t* da2 = db1 + count;
    uint64_t* db2 = da2 + count * n;
    FHE_HIP_CHECK(hipSetDevice(device_));
    FHE_HIP_CHECK(hipMemcpyAsync(da1, a1, count * n * 8, hipMemcpyHostToDevice, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(db1, b1, count * 8, hipMemcpyHostToDevice, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(da2, a2, count * n * 8, hipMemcpyHostToDevice, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(db2, b2, count * 8, hipMemcpyHostToDevice, stream_));
    bootstrap_device(gate, count, da1, db1, da2, db2, false, stream_);
    std::vector<uint32_t> ha(count * N), hb(count);
    FHE_HIP_CHECK(hipMemcpyAsync(ha.data(), d_ext_a_, count * N * 4, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(hb.data(), d_ext_b_, count * 4, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipStreamSynchronize(stream_));
    for (size_t i = 0; i < count * N; ++i) ext_a[i] = ha[i];
    for (size_t i = 0; i < count; ++i) ext_b[i] = hb[i];
}

void Engine::keyswitch_host(size_t count, const uint64_t* a, const uint64_t* b, uint64_t* a_out, uint64_t* b_out) {
    if (!d_ksk_) throw std::logic_error("key-switching key not loaded");
    if (count == 0) return;
    ensure_work(count);
    ensure_host_stage(count);
    const size_t N = p_.N;
    std::vector<uint32_t> ha(count * N), hb(count);
    for (size_t i = 0; i < count * N; ++i) {
        if (a[i] >= p_.qKS) throw std::invalid_argument("keyswitch input not reduced mod qKS");
        ha[i] = (uint32_t)a[i];
    }
    for (size_t i = 0; i < count; ++i) {
        if (b[i] >= p_.qKS) throw std::invalid_argument("keyswitch input not reduced mod qKS");
        hb[i] = (uint32_t)b[i];
    }
    uint64_t* dao = d_io_;
    uint64_t* dbo = dao + count * p_.n;
    FHE_HIP_CHECK(hipSetDevice(device_));
    FHE_HIP_CHECK(hipMemcpyAsync(d_ext_a_, ha.data(), count * N * 4, hipMemcpyHostToDevice, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(d_ext_b_, hb.data(), count * 4, hipMemcpyHostToDevice, stream_));
    GateArgs g = gate_args(G_AND, count);
    FHE_HIP_CHECK(launch_keyswitch(g, p_.baseKS, p_.digitsKS, d_ksk_, d_ext_a_, d_ext_b_, 0, dao, dbo, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(a_out, dao, count * p_.n * 8, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipMemcpyAsync(b_out, dbo, count * 8, hipMemcpyDeviceToHost, stream_));
    FHE_HIP_CHECK(hipStreamSynchronize(stream_));
}

}  // namespace fhe_amd
