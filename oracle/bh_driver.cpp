// bh_driver.cpp -- TEST INFRASTRUCTURE ONLY: extern "C" hooks that register our BackendHIP
// (integration/backend_hip.cpp) in the REFERENCE's own BackendRegistry (backend.cpp:241-305) and
// run each seam operation both through the registered backend (on the GPU) and through the
// reference's CPU path on the same objects, for tests/test_backend.py.  Linked with the reference
// sources into oracle/_ref/libbackend_hip.so by oracle/Makefile; never part of fhe_amd.
//
// Reference side of each comparison:
//   BlindRotateBatch     RingGSWAccumulator{CGGI,LMKCDEY,DM}::EvalAcc (rgsw-acc-cggi.cpp:59-68,
//                        rgsw-acc-lmkcdey.cpp:70-158, rgsw-acc-dm.cpp:62-77)
//   ExternalProductBatch AddToAccLMKCDEY (rgsw-acc-lmkcdey.cpp:228-254, private) restated with the
//                        public SignedDigitDecompose (rgsw-acc.cpp:54-91) and NativePoly products
//   KeySwitchBatch       LWEEncryptionScheme::KeySwitch (lwe-pke.cpp:348-372)
//   ModSwitchBatch       LWEEncryptionScheme::ModSwitch (lwe-pke.cpp:254-261)
//   EvalBinGateBatch     lux::fhe::EvalBinGateBatch (batch/batch.cpp:176-210), directly and routed
//                        through the registry (EvalBinGateBatchHIP)
//   null accumulators    BootstrapGateCore(AND, ct + q/4) (binfhe-base-scheme.cpp:190-205, 525-583),
//                        and lux::fhe::BootstrapBatch / KeySwitchBatch / ModSwitchBatch (batch.cpp:53-104,
//                        251-314) with BackendHIP as the registry's default
#include <execinfo.h>
#include <fcntl.h>
#include <omp.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <exception>
#include <string>
#include <vector>

#include "backend_hip.h"
#include "batch/binfhe-batch.h"
#include "c_api_hip.h"
#include "c_api_hip_types.h"
#include "rgsw-acc-cggi.h"
#include "rgsw-acc-dm.h"
#include "rgsw-acc-lmkcdey.h"

using namespace lux::fhe;
using namespace lux::fhe::backend;

extern "C" void* ref_ctx_context(void* h);  // ref_driver.cpp

namespace {
// test diagnostics: the native stack of the first thread that faults (FHE_SEGV_TRACE=1, tests/conftest.py)
std::atomic<int> g_fault{0};
void on_fault(int sig, siginfo_t* si, void*) {
    if (g_fault.exchange(1) == 0) {
        char msg[128];
        const int len = snprintf(msg, sizeof msg, "\n[segv-trace] signal %d at address %p, thread %ld\n", sig,
                                 si->si_addr, (long)syscall(SYS_gettid));
        (void)!write(2, msg, len);
        void* frames[64];
        const int n = backtrace(frames, 64);
        backtrace_symbols_fd(frames, n, 2);
        const int fd = open("/proc/self/maps", O_RDONLY);
        char buf[4096];
        for (ssize_t r; fd >= 0 && (r = read(fd, buf, sizeof buf)) > 0;)
            (void)!write(2, buf, r);
        signal(sig, SIG_DFL);  // returning re-executes the faulting access under the default action
        return;
    }
    for (;;)
        pause();
}

bool g_trace = false;
void step(const char* what) {
    if (g_trace)
        fprintf(stderr, "[bh] %s\n", what);
}
}  // namespace

extern "C" void bh_install_fault_trace() {
    void* warm[4];
    backtrace(warm, 4);  // loads the unwinder now, not inside the handler
    static char alt[1 << 16];
    stack_t ss{};
    ss.ss_sp   = alt;
    ss.ss_size = sizeof alt;
    sigaltstack(&ss, nullptr);
    g_trace = true;
    struct sigaction sa {};
    sa.sa_sigaction = on_fault;
    sa.sa_flags     = SA_SIGINFO | SA_ONSTACK;
    sigaction(SIGSEGV, &sa, nullptr);
    sigaction(SIGBUS, &sa, nullptr);
    sigaction(SIGABRT, &sa, nullptr);
}

namespace {

thread_local std::string g_err;
BackendHIP* g_be = nullptr;  // owned by the registry

template <typename F>
int guarded(F&& f) {
    try {
        f();
        return 0;
    }
    catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
    catch (...) {
        g_err = "unknown exception";
        return -1;
    }
}

BinFHEContext& CC(void* h) {
    return *static_cast<BinFHEContext*>(ref_ctx_context(h));
}

NativeVector vec_from(const uint64_t* p, uint32_t len, const NativeInteger& mod) {
    NativeVector v(len, mod);
    for (uint32_t i = 0; i < len; ++i)
        v[i] = NativeInteger(p[i]);
    return v;
}

NativePoly poly_from(const std::shared_ptr<ILNativeParams>& pp, const uint64_t* src, uint32_t N,
                     const NativeInteger& Q) {
    NativePoly poly(pp, Format::EVALUATION, true);
    poly.SetValues(vec_from(src, N, Q), Format::EVALUATION);
    return poly;
}

void poly_out(const NativePoly& p, uint64_t* dst) {
    const auto& v = p.GetValues();
    for (uint32_t i = 0; i < v.GetLength(); ++i)
        dst[i] = v[i].ConvertToInt();
}

RLWECiphertext rlwe_from(const std::shared_ptr<ILNativeParams>& pp, const uint64_t* src, uint32_t N,
                         const NativeInteger& Q) {
    std::vector<NativePoly> el{poly_from(pp, src, N, Q), poly_from(pp, src + N, N, Q)};
    return std::make_shared<RLWECiphertextImpl>(std::move(el));
}

void rlwe_out(const RLWECiphertext& c, uint64_t* dst, uint32_t N) {
    poly_out(c->GetElements()[0], dst);
    poly_out(c->GetElements()[1], dst + N);
}

std::vector<LWECiphertext> lwe_vec(const uint64_t* a, const uint64_t* b, size_t count, uint32_t len, uint64_t mod) {
    std::vector<LWECiphertext> v(count);
    for (size_t g = 0; g < count; ++g)
        v[g] = std::make_shared<LWECiphertextImpl>(vec_from(a + g * len, len, NativeInteger(mod)),
                                                   NativeInteger(b ? b[g] : 0));
    return v;
}

void lwe_out(const std::vector<LWECiphertext>& v, uint64_t* a, uint64_t* b) {
    for (size_t g = 0; g < v.size(); ++g) {
        const uint32_t len = v[g]->GetLength();
        for (uint32_t i = 0; i < len; ++i)
            a[g * len + i] = v[g]->GetA()[i].ConvertToInt();
        b[g] = v[g]->GetB().ConvertToInt();
    }
}

}  // namespace

extern "C" {

const char* bh_last_error() {
    return g_err.c_str();
}

// BackendRegistry::Instance().Register(BackendHIP) + SetDefault, for the context's parameter set
int bh_register(int paramset, int method, int device) {
    return guarded([&] {
        step("register: BackendHIP");
        auto be = std::make_unique<BackendHIP>(static_cast<BINFHE_PARAMSET>(paramset),
                                               static_cast<BINFHE_METHOD>(method), device);
        g_be = be.get();
        step("register: Register");
        BackendRegistry::Instance().Register(std::move(be));
        step("register: done");
        BackendRegistry::Instance().SetDefault(kBackendHIP);
        if (CurrentBackend() != g_be)
            throw std::runtime_error("registry does not return the registered backend");
    });
}

// releases the device context before static destruction; the default goes back to CPU
int bh_unregister() {
    return guarded([&] {
        if (g_be)
            g_be->Release();
        BackendRegistry::Instance().SetDefault(BackendType::CPU);
    });
}

// out: Type, IsAvailable, MaxBatchSize, DeviceMemory, registry IsAvailable(kBackendHIP); name
int bh_info(uint64_t* out, char* name, size_t cap) {
    return guarded([&] {
        Backend* be = BackendRegistry::Instance().Get(kBackendHIP);
        if (!be)
            throw std::runtime_error("not registered");
        out[0] = static_cast<uint64_t>(be->Type());
        out[1] = be->IsAvailable();
        out[2] = be->MaxBatchSize();
        out[3] = be->DeviceMemory();
        out[4] = BackendRegistry::Instance().IsAvailable(kBackendHIP);
        std::strncpy(name, be->Name().c_str(), cap - 1);
        name[cap - 1] = 0;
    });
}

// Allocate / CopyToDevice / CopyToHost / Synchronize / Free through CurrentBackend()
int bh_memory_roundtrip(const uint8_t* src, size_t bytes, uint8_t* back) {
    return guarded([&] {
        Backend* be   = CurrentBackend();
        DeviceBuffer d = be->Allocate(bytes);
        if (!d.IsValid() || !d.IsDevice())
            throw std::runtime_error("Allocate returned no device buffer");
        be->CopyToDevice(src, d, bytes);
        be->Synchronize();
        be->CopyToHost(d, back, bytes);
        be->Free(d);
        if (d.ptr)
            throw std::runtime_error("Free left the pointer set");
    });
}

// BlindRotateBatch through CurrentBackend() vs EvalAcc on the CPU; keys = the ones BTKeyLoad put in
// the reference context (ref_load_keys / ref_keygen)
int bh_blind_rotate(void* h, size_t count, const uint64_t* a, uint64_t ctmod, const uint64_t* acc_in,
                    uint64_t* acc_gpu, uint64_t* acc_ref, int nthreads) {
    return guarded([&] {
        BinFHEContext& cc = CC(h);
        auto rg           = cc.GetParams()->GetRingGSWParams();
        const uint32_t n = cc.GetParams()->GetLWEParams()->Getn(), N = rg->GetN();
        const NativeInteger Q = rg->GetQ();
        const auto pp         = rg->GetPolyParams();
        const auto& ek        = cc.GetRefreshKey();
        auto cts              = lwe_vec(a, nullptr, count, n, ctmod);
        std::vector<RLWECiphertext> accs(count);
        for (size_t g = 0; g < count; ++g)
            accs[g] = rlwe_from(pp, acc_in + g * 2 * N, N, Q);
        CurrentBackend()->BlindRotateBatch(rg, cts, ek, accs);
        for (size_t g = 0; g < count; ++g)
            rlwe_out(accs[g], acc_gpu + g * 2 * N, N);
        std::string err;
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : omp_get_max_threads()) schedule(dynamic)
        for (size_t g = 0; g < count; ++g) {
            try {
                auto acc = rlwe_from(pp, acc_in + g * 2 * N, N, Q);
                const NativeVector& av = cts[g]->GetA();
                switch (rg->GetMethod()) {
                    case GINX: RingGSWAccumulatorCGGI().EvalAcc(rg, ek, acc, av); break;
                    case LMKCDEY: RingGSWAccumulatorLMKCDEY().EvalAcc(rg, ek, acc, av); break;
                    default: RingGSWAccumulatorDM().EvalAcc(rg, ek, acc, av); break;
                }
                rlwe_out(acc, acc_ref + g * 2 * N, N);
            }
            catch (const std::exception& e) {
#pragma omp critical
                err = e.what();
            }
        }
        if (!err.empty())
            throw std::runtime_error(err);
    });
}

// ExternalProductBatch through CurrentBackend() vs AddToAccLMKCDEY restated with public pieces
int bh_external_product(void* h, size_t count, const uint64_t* rgsw, const uint64_t* rlwe, uint64_t* out_gpu,
                        uint64_t* out_ref) {
    return guarded([&] {
        BinFHEContext& cc = CC(h);
        auto rg           = cc.GetParams()->GetRingGSWParams();
        const uint32_t N = rg->GetN(), dG2 = 2 * (rg->GetDigitsG() - 1);
        const NativeInteger Q = rg->GetQ();
        const auto pp         = rg->GetPolyParams();
        const size_t kw       = (size_t)dG2 * 2 * N;
        std::vector<RingGSWEvalKey> keys(count);
        std::vector<RLWECiphertext> cts(count), res;
        for (size_t g = 0; g < count; ++g) {
            std::vector<std::vector<NativePoly>> el(dG2, std::vector<NativePoly>(2));
            for (uint32_t d = 0; d < dG2; ++d)
                for (uint32_t c = 0; c < 2; ++c)
                    el[d][c] = poly_from(pp, rgsw + g * kw + ((size_t)d * 2 + c) * N, N, Q);
            keys[g] = std::make_shared<RingGSWEvalKeyImpl>(el);
            cts[g]  = rlwe_from(pp, rlwe + g * 2 * N, N, Q);
        }
        CurrentBackend()->ExternalProductBatch(rg, keys, cts, res);
        for (size_t g = 0; g < count; ++g)
            rlwe_out(res[g], out_gpu + g * 2 * N, N);
        const RingGSWAccumulatorLMKCDEY scheme;
        for (size_t g = 0; g < count; ++g) {  // rgsw-acc-lmkcdey.cpp:228-254
            std::vector<NativePoly> ct(cts[g]->GetElements());
            ct[0].SetFormat(Format::COEFFICIENT);
            ct[1].SetFormat(Format::COEFFICIENT);
            std::vector<NativePoly> dct(dG2, NativePoly(pp, Format::COEFFICIENT, true));
            scheme.SignedDigitDecompose(rg, ct, dct);
            for (uint32_t d = 0; d < dG2; ++d)
                dct[d].SetFormat(Format::EVALUATION);
            const auto& ev = keys[g]->GetElements();
            NativePoly r0  = dct[0] * ev[0][0];
            for (uint32_t d = 1; d < dG2; ++d)
                r0 += dct[d] * ev[d][0];
            NativePoly r1 = dct[0] * ev[0][1];
            for (uint32_t d = 1; d < dG2; ++d)
                r1 += dct[d] * ev[d][1];
            poly_out(r0, out_ref + g * 2 * N);
            poly_out(r1, out_ref + g * 2 * N + N);
        }
    });
}

// KeySwitchBatch (inputs mod qKS, dimension N) vs LWEEncryptionScheme::KeySwitch
int bh_keyswitch(void* h, size_t count, const uint64_t* a, const uint64_t* b, uint64_t* ga, uint64_t* gb,
                 uint64_t* ra, uint64_t* rb) {
    return guarded([&] {
        BinFHEContext& cc = CC(h);
        auto lp           = cc.GetParams()->GetLWEParams();
        auto cts          = lwe_vec(a, b, count, lp->GetN(), lp->GetqKS().ConvertToInt());
        std::vector<LWECiphertext> out;
        CurrentBackend()->KeySwitchBatch(lp, cts, cc.GetSwitchKey(), out);
        lwe_out(out, ga, gb);
        std::vector<LWECiphertext> ref(count);
        const LWEEncryptionScheme lwe;
#pragma omp parallel for
        for (size_t g = 0; g < count; ++g)
            ref[g] = lwe.KeySwitch(lp, cc.GetSwitchKey(), cts[g]);
        lwe_out(ref, ra, rb);
    });
}

// ModSwitchBatch (inputs mod `mod` = Q or qKS) vs LWEEncryptionScheme::ModSwitch to the next modulus
int bh_modswitch(void* h, size_t count, uint32_t len, uint64_t mod, const uint64_t* a, const uint64_t* b,
                 uint64_t* ga, uint64_t* gb, uint64_t* ra, uint64_t* rb, uint64_t* mod_out) {
    return guarded([&] {
        BinFHEContext& cc = CC(h);
        auto lp           = cc.GetParams()->GetLWEParams();
        auto cts          = lwe_vec(a, b, count, len, mod);
        std::vector<LWECiphertext> out;
        CurrentBackend()->ModSwitchBatch(lp, cts, out);
        lwe_out(out, ga, gb);
        *mod_out = count ? out[0]->GetModulus().ConvertToInt() : 0;
        const NativeInteger to = mod == lp->GetQ().ConvertToInt() ? lp->GetqKS() : lp->Getq();
        const LWEEncryptionScheme lwe;
        std::vector<LWECiphertext> ref(count);
        for (size_t g = 0; g < count; ++g)
            ref[g] = lwe.ModSwitch(to, cts[g]);
        lwe_out(ref, ra, rb);
    });
}

// the backend's fused gate path vs the reference's EvalBinGateBatch (OpenMP over EvalBinGate)
int bh_eval_gates(void* h, int gate, size_t count, const uint64_t* a1, const uint64_t* b1, const uint64_t* a2,
                  const uint64_t* b2, uint64_t* ga, uint64_t* gb, uint64_t* ra, uint64_t* rb) {
    return guarded([&] {
        BinFHEContext& cc = CC(h);
        auto lp           = cc.GetParams()->GetLWEParams();
        const uint64_t q  = lp->Getq().ConvertToInt();
        auto c1 = lwe_vec(a1, b1, count, lp->Getn(), q), c2 = lwe_vec(a2, b2, count, lp->Getn(), q);
        RingGSWBTKey keys;
        keys.BSkey = cc.GetRefreshKey();
        keys.KSkey = cc.GetSwitchKey();
        std::vector<LWECiphertext> out, ref;
        g_be->EvalBinGateBatch(static_cast<BINGATE>(gate), keys, c1, c2, out);
        lwe_out(out, ga, gb);
        BatchResult r = EvalBinGateBatch(cc, static_cast<BINGATE>(gate), c1, c2, ref, 0);
        if (!r.success)
            throw std::runtime_error("reference EvalBinGateBatch: " + r.error);
        lwe_out(ref, ra, rb);
    });
}

// BlindRotateBatch with null accumulators -- the call BootstrapBatch makes (batch.cpp:77-86) --
// through CurrentBackend() vs the reference's BootstrapGateCore(AND, ct + q/4) (binfhe-base-scheme.cpp:
// 190-205, 525-583; private there, so its test-vector set-up :535-575 is restated here and EvalAcc is
// the reference's own).  The restatement is pinned by the reference's public Bootstrap: *flags bit 0 =
// the extraction of Bootstrap (:206-213) applied to the reference accumulator equals
// cc.Bootstrap(ct, true) for every ciphertext; bit 1 = lux::fhe::BootstrapBatch (batch.cpp:53-104) on
// the same ciphertexts with BackendHIP as the default returned success with every ciphertext processed
int bh_bootstrap_init(void* h, size_t count, const uint64_t* a, const uint64_t* b, uint64_t* acc_gpu,
                      uint64_t* acc_ref, int* flags) {
    return guarded([&] {
        BinFHEContext& cc = CC(h);
        auto rg           = cc.GetParams()->GetRingGSWParams();
        auto lp           = cc.GetParams()->GetLWEParams();
        const uint32_t n = lp->Getn(), N = rg->GetN();
        const NativeInteger Q = rg->GetQ(), q = lp->Getq();
        const auto pp         = rg->GetPolyParams();
        const auto& ek        = cc.GetRefreshKey();
        auto cts              = lwe_vec(a, b, count, n, q.ConvertToInt());
        std::vector<RLWECiphertext> accs(count);  // null, as BootstrapBatch passes them
        CurrentBackend()->BlindRotateBatch(rg, cts, ek, accs);
        for (size_t g = 0; g < count; ++g)
            rlwe_out(accs[g], acc_gpu + g * 2 * N, N);
        bool ext_ok = true;
        std::string err;
#pragma omp parallel for schedule(dynamic)
        for (size_t g = 0; g < count; ++g) {
            try {
                // ct + q/4 (EvalAddConstEq, :201), then BootstrapGateCore's window and test vector
                const uint32_t qHalf = q.ConvertToInt<uint32_t>() >> 1;
                NativeInteger bb    = NativeInteger(b[g]).ModAddFast(q >> 2, q);
                const NativeInteger q1 = rg->GetGateConst()[static_cast<size_t>(AND)];
                const NativeInteger q2 = q1.ModAddFast(NativeInteger(qHalf), q);
                const bool swap        = q1 >= q2;
                const NativeInteger lb = swap ? q2 : q1, ub = swap ? q1 : q2;
                const NativeInteger Q2p = Q / (cts[g]->GetptModulus() * 2) + 1, Q2pNeg = Q - Q2p;
                const NativeInteger lv = swap ? Q2p : Q2pNeg, uv = swap ? Q2pNeg : Q2p;
                NativeVector m(N, Q);
                for (uint32_t i = 0; i < N; i += N / qHalf) {
                    m[i] = (bb >= lb && bb < ub) ? lv : uv;
                    bb.ModSubFastEq(1, q);
                }
                std::vector<NativePoly> res(2);
                res[0] = NativePoly(pp, Format::EVALUATION, true);
                res[1] = NativePoly(pp, Format::COEFFICIENT, false);
                res[1].SetValues(std::move(m), Format::COEFFICIENT);
                res[1].SetFormat(Format::EVALUATION);
                auto acc = std::make_shared<RLWECiphertextImpl>(std::move(res));
                const NativeVector& av = cts[g]->GetA();
                switch (rg->GetMethod()) {
                    case GINX: RingGSWAccumulatorCGGI().EvalAcc(rg, ek, acc, av); break;
                    case LMKCDEY: RingGSWAccumulatorLMKCDEY().EvalAcc(rg, ek, acc, av); break;
                    default: RingGSWAccumulatorDM().EvalAcc(rg, ek, acc, av); break;
                }
                rlwe_out(acc, acc_ref + g * 2 * N, N);
                // Bootstrap's extraction (:206-213) vs the reference's own Bootstrap(ct, extended)
                auto el = acc->GetElements();
                el[0]   = el[0].Transpose();
                el[0].SetFormat(Format::COEFFICIENT);
                el[1].SetFormat(Format::COEFFICIENT);
                NativeInteger eb = Q / (cts[g]->GetptModulus() * 2) + 1;
                eb.ModAddFastEq(el[1][0], Q);
                const auto want = cc.Bootstrap(cts[g], true);
                const bool same = want->GetB() == eb && want->GetA() == el[0].GetValues();
                if (!same) {
#pragma omp critical
                    ext_ok = false;
                }
            }
            catch (const std::exception& e) {
#pragma omp critical
                err = e.what();
            }
        }
        if (!err.empty())
            throw std::runtime_error(err);
        std::vector<LWECiphertext> out;
        const BatchResult r = BootstrapBatch(cc, cts, out, 0);
        *flags = (ext_ok ? 1 : 0) | (r.success && r.processed == count && out.size() == count ? 2 : 0);
        if (!r.success)
            g_err = "BootstrapBatch: " + r.error;
    });
}

// the reference's own batch callers of the seam (batch.cpp:251-314) with BackendHIP as the default:
// KeySwitchBatch on (N, qKS) ciphertexts and ModSwitchBatch on (N, Q) ciphertexts, vs
// LWEEncryptionScheme::KeySwitch / ModSwitch(qKS, .) on the CPU; *ok = both BatchResults successful
int bh_batch_callers(void* h, size_t count, const uint64_t* ka, const uint64_t* kb, uint64_t* gka, uint64_t* gkb,
                     uint64_t* rka, uint64_t* rkb, const uint64_t* ma, const uint64_t* mb, uint64_t* gma, uint64_t* gmb,
                     uint64_t* rma, uint64_t* rmb, int* ok) {
    return guarded([&] {
        BinFHEContext& cc = CC(h);
        auto lp           = cc.GetParams()->GetLWEParams();
        const uint32_t N  = lp->GetN();
        auto kcts = lwe_vec(ka, kb, count, N, lp->GetqKS().ConvertToInt());
        auto mcts = lwe_vec(ma, mb, count, N, lp->GetQ().ConvertToInt());
        std::vector<LWECiphertext> ko, mo;
        const BatchResult r1 = KeySwitchBatch(cc, kcts, ko, 0);
        const BatchResult r2 = ModSwitchBatch(cc, mcts, mo, 0);
        *ok = r1.success && r2.success && r1.processed == count && r2.processed == count;
        if (!*ok)
            throw std::runtime_error("batch callers: " + r1.error + " / " + r2.error);
        lwe_out(ko, gka, gkb);
        lwe_out(mo, gma, gmb);
        const LWEEncryptionScheme lwe;
        std::vector<LWECiphertext> kr(count), mr(count);
#pragma omp parallel for
        for (size_t g = 0; g < count; ++g) {
            kr[g] = lwe.KeySwitch(lp, cc.GetSwitchKey(), kcts[g]);
            mr[g] = lwe.ModSwitch(lp->GetqKS(), mcts[g]);
        }
        lwe_out(kr, rka, rkb);
        lwe_out(mr, rma, rmb);
    });
}

// EvalBinGateBatch routed through the registry (EvalBinGateBatchHIP, integration/backend_hip.h) vs
// the reference's EvalBinGateBatch; *ok = the routed BatchResult reports success for every gate
int bh_eval_gates_routed(void* h, int gate, size_t count, const uint64_t* a1, const uint64_t* b1, const uint64_t* a2,
                         const uint64_t* b2, uint64_t* ga, uint64_t* gb, uint64_t* ra, uint64_t* rb, int* ok) {
    return guarded([&] {
        BinFHEContext& cc = CC(h);
        auto lp           = cc.GetParams()->GetLWEParams();
        const uint64_t q  = lp->Getq().ConvertToInt();
        auto c1 = lwe_vec(a1, b1, count, lp->Getn(), q), c2 = lwe_vec(a2, b2, count, lp->Getn(), q);
        std::vector<LWECiphertext> out, ref;
        step("routed: EvalBinGateBatchHIP");
        const BatchResult r = EvalBinGateBatchHIP(cc, static_cast<BINGATE>(gate), c1, c2, out, 0);
        *ok = r.success && r.processed == count;
        if (!r.success)
            throw std::runtime_error("EvalBinGateBatchHIP: " + r.error);
        lwe_out(out, ga, gb);
        step("routed: reference EvalBinGateBatch");
        const BatchResult rr = EvalBinGateBatch(cc, static_cast<BINGATE>(gate), c1, c2, ref, 0);
        step("routed: done");
        if (!rr.success)
            throw std::runtime_error("reference EvalBinGateBatch: " + rr.error);
        lwe_out(ref, ra, rb);
    });
}

// Ciphertexts mod Q through the routed callers (binfhe-base-scheme.cpp:92-93, 180-182, 200-201): k columns of
// count ciphertexts, rows of N words, large[j][g] != 0 marking a ciphertext mod Q (dimension N), 0 one mod q
// (its first n words), every input of plaintext modulus ptmod.  op < 6: EvalBinGateBatchHIP vs the reference's
// EvalBinGateBatch; op = 13 (CMUX, k = 3): EvalCMUXBatchHIP vs EvalCMUXBatch; op = -1 (k = 1):
// BackendHIP::RefreshBatch vs BinFHEContext::Bootstrap.  Outputs [count][n]; *ok = the routed call succeeded
int bh_eval_mixed_routed(void* h, int op, uint32_t k, uint32_t ptmod, size_t count, const uint64_t* const* a,
                         const uint64_t* const* b, const uint8_t* const* large, uint64_t* ga, uint64_t* gb,
                         uint64_t* ra, uint64_t* rb, int* ok) {
    return guarded([&] {
        BinFHEContext& cc = CC(h);
        auto lp           = cc.GetParams()->GetLWEParams();
        const uint32_t n = lp->Getn(), N = lp->GetN();
        const NativeInteger q = lp->Getq(), Q = lp->GetQ();
        std::vector<std::vector<LWECiphertext>> cols(k);
        for (uint32_t j = 0; j < k; ++j)
            for (size_t g = 0; g < count; ++g) {
                const bool lg = large[j][g] != 0;
                auto ct = std::make_shared<LWECiphertextImpl>(vec_from(a[j] + g * N, lg ? N : n, lg ? Q : q),
                                                              NativeInteger(b[j][g]));
                ct->SetptModulus(ptmod);
                cols[j].push_back(ct);
            }
        std::vector<LWECiphertext> out, ref(count);
        *ok = 0;
        if (op == -1) {
            RingGSWBTKey keys;
            keys.BSkey = cc.GetRefreshKey();
            keys.KSkey = cc.GetSwitchKey();
            g_be->RefreshBatch(keys, cols[0], out);
            *ok = out.size() == count;
            for (size_t g = 0; g < count; ++g)
                *ok = *ok && out[g]->GetptModulus() == ptmod;
#pragma omp parallel for
            for (size_t g = 0; g < count; ++g)
                ref[g] = cc.Bootstrap(cols[0][g]);
        }
        else if (op == CMUX) {
            const BatchResult r = EvalCMUXBatchHIP(cc, cols[0], cols[1], cols[2], out, 0);
            *ok = r.success && r.processed == count;
            if (!r.success)
                throw std::runtime_error("EvalCMUXBatchHIP: " + r.error);
            const BatchResult rr = EvalCMUXBatch(cc, cols[0], cols[1], cols[2], ref, 0);
            if (!rr.success)
                throw std::runtime_error("reference EvalCMUXBatch: " + rr.error);
        }
        else {
            const BatchResult r = EvalBinGateBatchHIP(cc, static_cast<BINGATE>(op), cols[0], cols[1], out, 0);
            *ok = r.success && r.processed == count;
            if (!r.success)
                throw std::runtime_error("EvalBinGateBatchHIP: " + r.error);
            const BatchResult rr = EvalBinGateBatch(cc, static_cast<BINGATE>(op), cols[0], cols[1], ref, 0);
            if (!rr.success)
                throw std::runtime_error("reference EvalBinGateBatch: " + rr.error);
        }
        lwe_out(out, ga, gb);
        lwe_out(ref, ra, rb);
    });
}

// PackCiphertexts -> UnpackCiphertexts and PackBootstrappingKey -> UnpackBootstrappingKey round trips
// through device memory; *ok bit 0: ciphertexts equal, bit 1: key equal to the context's refresh key
int bh_pack_roundtrip(void* h, size_t count, const uint64_t* a, const uint64_t* b, int* ok) {
    return guarded([&] {
        BinFHEContext& cc = CC(h);
        auto lp           = cc.GetParams()->GetLWEParams();
        Backend* be       = CurrentBackend();
        auto cts          = lwe_vec(a, b, count, lp->Getn(), lp->Getq().ConvertToInt());
        DeviceBuffer pc = be->PackCiphertexts(cts);
        std::vector<LWECiphertext> back;
        be->UnpackCiphertexts(pc, back);
        be->Free(pc);
        bool same = back.size() == cts.size();
        for (size_t g = 0; same && g < count; ++g)
            same = *back[g] == *cts[g];
        DeviceBuffer pk = be->PackBootstrappingKey(cc.GetRefreshKey());
        RingGSWACCKey ek;
        be->UnpackBootstrappingKey(pk, ek);
        be->Free(pk);
        *ok = (same ? 1 : 0) | (*ek == *cc.GetRefreshKey() ? 2 : 0);
    });
}

// EvalFuncBatchHIP (multi = 0) or EvalFuncMultiOutputBatchHIP (multi = 1) with BackendHIP as the default vs
// the reference's EvalFuncBatch / EvalFuncMultiOutputBatch (batch.cpp:106-174) on the same ciphertexts
// (mod ctmod).  luts [L][lut_len]; outputs [count][L][n] (multi) or, for multi = 0, [L][count][n] from one
// routed call per LUT.  *ok = every routed BatchResult reported success with processed = count
int bh_eval_func_routed(void* h, int multi, size_t count, const uint64_t* a, const uint64_t* b, uint64_t ctmod,
                        const uint64_t* luts, size_t L, size_t lut_len, uint64_t* ga, uint64_t* gb, uint64_t* ra,
                        uint64_t* rb, int* ok) {
    return guarded([&] {
        BinFHEContext& cc = CC(h);
        const uint32_t n  = cc.GetParams()->GetLWEParams()->Getn();
        auto cts          = lwe_vec(a, b, count, n, ctmod);
        std::vector<std::vector<NativeInteger>> tabs(L, std::vector<NativeInteger>(lut_len));
        for (size_t j = 0; j < L; ++j)
            for (size_t i = 0; i < lut_len; ++i)
                tabs[j][i] = NativeInteger(luts[j * lut_len + i]);
        *ok = 1;
        std::vector<LWECiphertext> out, ref;
        if (multi) {
            const BatchResult r = EvalFuncMultiOutputBatchHIP(cc, cts, tabs, out, 0);
            *ok = r.success && r.processed == count && out.size() == count * L;
            if (!r.success)
                throw std::runtime_error("EvalFuncMultiOutputBatchHIP: " + r.error);
            const BatchResult rr = EvalFuncMultiOutputBatch(cc, cts, tabs, ref, 0);
            if (!rr.success)
                throw std::runtime_error("reference EvalFuncMultiOutputBatch: " + rr.error);
            lwe_out(out, ga, gb);
            lwe_out(ref, ra, rb);
            return;
        }
        for (size_t j = 0; j < L; ++j) {
            const BatchResult r = EvalFuncBatchHIP(cc, cts, tabs[j], out, 0);
            *ok = *ok && r.success && r.processed == count && out.size() == count;
            if (!r.success)
                throw std::runtime_error("EvalFuncBatchHIP: " + r.error);
            const BatchResult rr = EvalFuncBatch(cc, cts, tabs[j], ref, 0);
            if (!rr.success)
                throw std::runtime_error("reference EvalFuncBatch: " + rr.error);
            lwe_out(out, ga + j * count * n, gb + j * count);
            lwe_out(ref, ra + j * count * n, rb + j * count);
        }
    });
}

// EvalCMUXBatchHIP (BackendHIP as the default) vs the reference's EvalCMUXBatch (batch.cpp:212-249): rows
// (sel, true, false) = (ct0, ct1, ct2)
int bh_eval_cmux_routed(void* h, size_t count, const uint64_t* a0, const uint64_t* b0, const uint64_t* a1,
                        const uint64_t* b1, const uint64_t* a2, const uint64_t* b2, uint64_t* ga, uint64_t* gb,
                        uint64_t* ra, uint64_t* rb, int* ok) {
    return guarded([&] {
        BinFHEContext& cc = CC(h);
        auto lp           = cc.GetParams()->GetLWEParams();
        const uint64_t q  = lp->Getq().ConvertToInt();
        const uint32_t n  = lp->Getn();
        auto c0 = lwe_vec(a0, b0, count, n, q), c1 = lwe_vec(a1, b1, count, n, q), c2 = lwe_vec(a2, b2, count, n, q);
        std::vector<LWECiphertext> out, ref;
        const BatchResult r = EvalCMUXBatchHIP(cc, c0, c1, c2, out, 0);
        *ok = r.success && r.processed == count;
        if (!r.success)
            throw std::runtime_error("EvalCMUXBatchHIP: " + r.error);
        const BatchResult rr = EvalCMUXBatch(cc, c0, c1, c2, ref, 0);
        if (!rr.success)
            throw std::runtime_error("reference EvalCMUXBatch: " + rr.error);
        lwe_out(out, ga, gb);
        lwe_out(ref, ra, rb);
    });
}

// BackendHIP::RefreshBatch vs the reference's BinFHEContext::Bootstrap on every ciphertext
int bh_refresh(void* h, size_t count, const uint64_t* a, const uint64_t* b, uint64_t* ga, uint64_t* gb, uint64_t* ra,
               uint64_t* rb) {
    return guarded([&] {
        BinFHEContext& cc = CC(h);
        auto lp           = cc.GetParams()->GetLWEParams();
        auto cts          = lwe_vec(a, b, count, lp->Getn(), lp->Getq().ConvertToInt());
        RingGSWBTKey keys;
        keys.BSkey = cc.GetRefreshKey();
        keys.KSkey = cc.GetSwitchKey();
        std::vector<LWECiphertext> out, ref(count);
        g_be->RefreshBatch(keys, cts, out);
#pragma omp parallel for
        for (size_t g = 0; g < count; ++g)
            ref[g] = cc.Bootstrap(cts[g]);
        lwe_out(out, ga, gb);
        lwe_out(ref, ra, rb);
    });
}

// ---- the C API (integration/c_api_hip.cpp): the reference's CPU evaluation on the same LuxFheContext ----
// gate < 6: cc.EvalBinGate(gate, a, b); gate = 6: cc.EvalBinGate(CMUX, {a, b, c}); gate = 7: cc.Bootstrap(a)
int capi_ref_eval(LuxFheContext* ctx, int gate, const LuxFheCiphertext* a, const LuxFheCiphertext* b,
                  const LuxFheCiphertext* c, LuxFheCiphertext** out) {
    return guarded([&] {
        auto r = std::make_unique<LuxFheCiphertext>();
        if (gate < 6)
            r->ct = ctx->cc.EvalBinGate(static_cast<BINGATE>(gate), a->ct, b->ct);
        else if (gate == 6)
            r->ct = ctx->cc.EvalBinGate(CMUX, std::vector<LWECiphertext>{a->ct, b->ct, c->ct});
        else
            r->ct = ctx->cc.Bootstrap(a->ct);
        *out = r.release();
    });
}

// the two ciphertexts are equal (LWECiphertextImpl::operator==: a and b), and the raw words of x
int capi_ct_equal(const LuxFheCiphertext* x, const LuxFheCiphertext* y) {
    return x && y && x->ct && y->ct && *x->ct == *y->ct;
}

// which backend the context's bootstrapped calls ran on: 1 = a BackendHIP exists for it
int capi_on_gpu(const LuxFheContext* ctx) {
    return ctx && ctx->gpu ? 1 : 0;
}

}  // extern "C"
