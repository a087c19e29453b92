// backend_hip.cpp -- see backend_hip.h.  Reference objects are flattened into the raw u64 layouts
// of include/fhe_hip.h on the host and handed to libfhe_amd; results come back the same way.
#include "backend_hip.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>

namespace lux::fhe::backend {

namespace {

// ceil(log_baseKS(qKS)), as LWEEncryptionScheme::KeySwitch computes digitsKS (lwe-pke.cpp:354)
uint32_t digits_ks(const fhe_hip_params& p) {
    uint32_t d = 0;
    for (uint64_t v = 1; v < p.qKS; v *= p.baseKS) ++d;
    return d;
}

NativeVector vec_from(const uint64_t* p, uint32_t len, const NativeInteger& mod) {
    NativeVector v(len, mod);
    for (uint32_t i = 0; i < len; ++i)
        v[i] = NativeInteger(p[i]);
    return v;
}

void poly_to(const NativePoly& poly, uint64_t* dst, uint32_t N) {
    if (poly.GetFormat() != Format::EVALUATION)
        throw std::invalid_argument("BackendHIP: polynomials must be in EVALUATION format");
    const auto& v = poly.GetValues();
    if (v.GetLength() != N)
        throw std::invalid_argument("BackendHIP: polynomial of the wrong ring dimension");
    for (uint32_t i = 0; i < N; ++i)
        dst[i] = v[i].ConvertToInt();
}

NativePoly poly_from(const std::shared_ptr<ILNativeParams>& pp, const uint64_t* src, uint32_t N,
                     const NativeInteger& Q) {
    NativePoly poly(pp, Format::EVALUATION, true);
    poly.SetValues(vec_from(src, N, Q), Format::EVALUATION);
    return poly;
}

void rgsw_to(const RingGSWEvalKey& k, uint32_t rows, uint64_t* dst, uint32_t N) {
    if (!k)
        throw std::invalid_argument("BackendHIP: null RingGSWEvalKey");
    const auto& el = k->GetElements();
    if (el.size() != rows)
        throw std::invalid_argument("BackendHIP: RingGSWEvalKey has the wrong number of rows");
    for (uint32_t r = 0; r < rows; ++r)
        for (uint32_t c = 0; c < 2; ++c)
            poly_to(el[r][c], dst + ((size_t)r * 2 + c) * N, N);
}

RingGSWEvalKey rgsw_from(const std::shared_ptr<ILNativeParams>& pp, const uint64_t* src, uint32_t rows, uint32_t N,
                         const NativeInteger& Q) {
    std::vector<std::vector<NativePoly>> el(rows, std::vector<NativePoly>(2));
    for (uint32_t r = 0; r < rows; ++r)
        for (uint32_t c = 0; c < 2; ++c)
            el[r][c] = poly_from(pp, src + ((size_t)r * 2 + c) * N, N, Q);
    return std::make_shared<RingGSWEvalKeyImpl>(el);
}

}  // namespace

BackendHIP::BackendHIP(BINFHE_PARAMSET set, BINFHE_METHOD method, int device)
    : device_(device), set_(set), method_(method) {
    Check(fhe_hip_create(static_cast<int>(set), static_cast<int>(method), device, &ctx_), "fhe_hip_create");
    Check(fhe_hip_get_params(ctx_, &p_), "fhe_hip_get_params");
}

BackendHIP::~BackendHIP() {
    Release();
}

void BackendHIP::Release() {
    std::lock_guard<std::mutex> lock(mu_);
    if (ctx_)
        fhe_hip_destroy(ctx_);
    ctx_ = nullptr;
    bsk_id_.reset();
    ksk_id_.reset();
}

void BackendHIP::Check(int rc, const char* what) const {
    if (rc == FHE_HIP_OK && !ctx_ && std::strcmp(what, "fhe_hip_create") != 0)
        throw std::runtime_error("BackendHIP: released");
    if (rc == FHE_HIP_OK)
        return;
    const std::string msg = std::string("BackendHIP: ") + what + ": " + fhe_hip_last_error();
    if (rc == FHE_HIP_ERR_INVALID_PARAM || rc == FHE_HIP_ERR_NULL_PTR)
        throw std::invalid_argument(msg);
    throw std::runtime_error(msg);
}

std::string BackendHIP::Name() const {
    return "HIP (fhe_amd, MI355X gfx950) device " + std::to_string(device_);
}

bool BackendHIP::IsAvailable() const {
    int n = 0;
    return ctx_ && fhe_hip_device_count(&n) == FHE_HIP_OK && device_ < n;
}

size_t BackendHIP::MaxBatchSize() const {
    size_t m = 0;
    Check(fhe_hip_max_batch_size(ctx_, &m), "MaxBatchSize");
    return m;
}

size_t BackendHIP::DeviceMemory() const {
    size_t total = 0;
    Check(fhe_hip_device_memory(device_, nullptr, &total), "DeviceMemory");
    return total;
}

// ---- memory --------------------------------------------------------------------------------------
DeviceBuffer BackendHIP::Allocate(size_t bytes) {
    DeviceBuffer b;
    Check(fhe_hip_alloc(device_, bytes, &b.ptr), "Allocate");
    b.size   = bytes;
    b.device = kBackendHIP;
    return b;
}

void BackendHIP::Free(DeviceBuffer& buffer) {
    if (buffer.ptr && buffer.device == kBackendHIP) {
        Check(fhe_hip_free(buffer.ptr), "Free");
        buffer.ptr  = nullptr;
        buffer.size = 0;
    }
}

void BackendHIP::CopyToDevice(const void* host_ptr, DeviceBuffer& buffer, size_t bytes) {
    if (!buffer.ptr || bytes > buffer.size)
        throw std::invalid_argument("BackendHIP::CopyToDevice: buffer too small");
    Check(fhe_hip_copy_to_device(buffer.ptr, host_ptr, bytes), "CopyToDevice");
}

void BackendHIP::CopyToHost(const DeviceBuffer& buffer, void* host_ptr, size_t bytes) {
    if (!buffer.ptr || bytes > buffer.size)
        throw std::invalid_argument("BackendHIP::CopyToHost: buffer too small");
    Check(fhe_hip_copy_to_host(host_ptr, buffer.ptr, bytes), "CopyToHost");
}

void BackendHIP::Synchronize() {
    Check(fhe_hip_synchronize(device_), "Synchronize");
}

// ---- parameter and key plumbing ------------------------------------------------------------------
void BackendHIP::CheckRGSW(const std::shared_ptr<RingGSWCryptoParams>& params) const {
    if (!params || params->GetN() != p_.N || params->GetQ().ConvertToInt() != p_.Q ||
        params->GetBaseG() != p_.baseG || params->GetDigitsG() != p_.digitsG || params->GetMethod() != method_)
        throw std::invalid_argument("BackendHIP: RingGSWCryptoParams differ from the backend's parameter set");
}

void BackendHIP::CheckLWE(const std::shared_ptr<LWECryptoParams>& params) const {
    if (!params || params->Getn() != p_.n || params->GetN() != p_.N || params->Getq().ConvertToInt() != p_.q ||
        params->GetQ().ConvertToInt() != p_.Q || params->GetqKS().ConvertToInt() != p_.qKS ||
        params->GetBaseKS() != p_.baseKS)
        throw std::invalid_argument("BackendHIP: LWECryptoParams differ from the backend's parameter set");
}

// raw layouts of include/fhe_hip.h: GINX [n][2][dG2][2][N]; LMKCDEY [n][dG2][2][N] ++
// [numAutoKeys+1][dG-1][2][N]; AP [n][baseR][digitsR][dG2][2][N] (j = 0 slots zero)
std::vector<uint64_t> BackendHIP::RawBSK(const RingGSWACCKey& ek) const {
    if (!ek)
        throw std::invalid_argument("BackendHIP: null bootstrapping key");
    const uint32_t n = p_.n, N = p_.N, dG2 = 2 * (p_.digitsG - 1);
    const size_t rgsw = (size_t)dG2 * 2 * N;
    std::vector<uint64_t> raw(p_.bsk_words, 0);
    if (method_ == GINX) {
        for (uint32_t i = 0; i < n; ++i)
            for (uint32_t s = 0; s < 2; ++s)
                rgsw_to((*ek)[0][s][i], dG2, raw.data() + ((size_t)i * 2 + s) * rgsw, N);
    }
    else if (method_ == LMKCDEY) {
        for (uint32_t i = 0; i < n; ++i)
            rgsw_to((*ek)[0][0][i], dG2, raw.data() + (size_t)i * rgsw, N);
        const size_t arow = (size_t)(p_.digitsG - 1) * 2 * N;
        for (uint32_t k = 0; k <= p_.numAutoKeys; ++k)
            rgsw_to((*ek)[0][1][k], p_.digitsG - 1, raw.data() + (size_t)n * rgsw + k * arow, N);
    }
    else {  // AP: (*ek)[i][j][k], RingGSWACCKeyImpl(n, baseR, digitsR) (rgsw-acc-dm.cpp:39-58)
        const size_t baseR = ek->GetElements()[0].size(), dR = ek->GetElements()[0][0].size();
        if ((size_t)n * baseR * dR * rgsw != raw.size())
            throw std::invalid_argument("BackendHIP: AP key has the wrong shape");
        for (uint32_t i = 0; i < n; ++i)
            for (size_t j = 1; j < baseR; ++j)
                for (size_t k = 0; k < dR; ++k)
                    rgsw_to((*ek)[i][j][k], dG2, raw.data() + ((i * baseR + j) * dR + k) * rgsw, N);
    }
    return raw;
}

namespace {
// the same live object as the one the weak reference was taken from (owner and address)
template <typename T>
bool same_key(const std::weak_ptr<const void>& w, const std::shared_ptr<T>& k) {
    const auto held = w.lock();
    return held && k && held.get() == static_cast<const void*>(k.get()) && !held.owner_before(k) &&
           !k.owner_before(held);
}
}  // namespace

void BackendHIP::EnsureBSK(const RingGSWACCKey& ek) {
    if (same_key(bsk_id_, ek))
        return;
    const auto raw = RawBSK(ek);
    Check(fhe_hip_load_bsk(ctx_, raw.data(), raw.size()), "load bootstrapping key");
    bsk_id_ = std::shared_ptr<const void>(ek);
}

void BackendHIP::EnsureKSK(const LWESwitchingKey& ks) {
    if (same_key(ksk_id_, ks))
        return;
    if (!ks)
        throw std::invalid_argument("BackendHIP: null switching key");
    const uint32_t n = p_.n, N = p_.N, dKS = digits_ks(p_);
    const auto& A = ks->GetElementsA();
    const auto& B = ks->GetElementsB();
    if (A.size() != N || A[0].size() != p_.baseKS || A[0][0].size() != dKS)
        throw std::invalid_argument("BackendHIP: switching key has the wrong shape");
    std::vector<uint64_t> rA(p_.ksk_rows * n), rB(p_.ksk_rows);
    for (uint32_t i = 0; i < N; ++i)
        for (uint32_t j = 0; j < p_.baseKS; ++j)
            for (uint32_t k = 0; k < dKS; ++k) {
                const size_t row = ((size_t)i * p_.baseKS + j) * dKS + k;
                const auto& v = A[i][j][k];
                for (uint32_t c = 0; c < n; ++c)
                    rA[row * n + c] = v[c].ConvertToInt();
                rB[row] = B[i][j][k].ConvertToInt();
            }
    Check(fhe_hip_load_ksk(ctx_, rA.data(), rA.size(), rB.data(), rB.size()), "load switching key");
    ksk_id_ = std::shared_ptr<const void>(ks);
}

// ---- single ops: batches of one --------------------------------------------------------------------
void BackendHIP::BlindRotate(const std::shared_ptr<RingGSWCryptoParams>& params, const LWECiphertext& ct,
                             const RingGSWACCKey& ek, RLWECiphertext& acc) {
    std::vector<RLWECiphertext> accs{acc};
    BlindRotateBatch(params, {ct}, ek, accs);
    acc = accs[0];
}

void BackendHIP::ExternalProduct(const std::shared_ptr<RingGSWCryptoParams>& params, const RingGSWEvalKey& rgsw,
                                 const RLWECiphertext& rlwe, RLWECiphertext& result) {
    std::vector<RLWECiphertext> out;
    ExternalProductBatch(params, {rgsw}, {rlwe}, out);
    result = out[0];
}

void BackendHIP::KeySwitch(const std::shared_ptr<LWECryptoParams>& params, const LWECiphertext& ct,
                           const LWESwitchingKey& ks, LWECiphertext& result) {
    std::vector<LWECiphertext> out;
    KeySwitchBatch(params, {ct}, ks, out);
    result = out[0];
}

void BackendHIP::ModSwitch(const std::shared_ptr<LWECryptoParams>& params, const LWECiphertext& ct,
                           LWECiphertext& result) {
    std::vector<LWECiphertext> out;
    ModSwitchBatch(params, {ct}, out);
    result = out[0];
}

// ---- batch ops ---------------------------------------------------------------------------------------
void BackendHIP::BlindRotateBatch(const std::shared_ptr<RingGSWCryptoParams>& params,
                                  const std::vector<LWECiphertext>& cts, const RingGSWACCKey& ek,
                                  std::vector<RLWECiphertext>& accs) {
    std::lock_guard<std::mutex> lock(mu_);
    CheckRGSW(params);
    const size_t B = cts.size();
    if (accs.size() != B)
        throw std::invalid_argument("BackendHIP::BlindRotateBatch: one accumulator per ciphertext");
    if (B == 0)
        return;
    EnsureBSK(ek);
    const uint32_t n = p_.n, N = p_.N;
    const uint64_t ctmod = cts[0]->GetModulus().ConvertToInt();
    // null accumulators (BootstrapBatch, batch.cpp:77-86): all of them or none
    const bool init = !accs[0];
    std::vector<uint64_t> a(B * n), b(init ? B : 0), acc(B * 2 * N);
    for (size_t g = 0; g < B; ++g) {
        const auto& v = cts[g]->GetA();
        if (v.GetLength() != n || cts[g]->GetModulus().ConvertToInt() != ctmod)
            throw std::invalid_argument("BackendHIP::BlindRotateBatch: ciphertexts of one dimension and modulus");
        for (uint32_t i = 0; i < n; ++i)
            a[g * n + i] = v[i].ConvertToInt();
        if (init) {
            if (accs[g])
                throw std::invalid_argument("BackendHIP::BlindRotateBatch: accumulators all given or all null");
            b[g] = cts[g]->GetB().ConvertToInt();
            continue;
        }
        if (!accs[g] || accs[g]->GetElements().size() != 2)
            throw std::invalid_argument("BackendHIP::BlindRotateBatch: accumulators must hold two polynomials");
        for (uint32_t c = 0; c < 2; ++c)
            poly_to(accs[g]->GetElements()[c], acc.data() + (g * 2 + c) * N, N);
    }
    if (init) {
        if (ctmod != p_.q)
            throw std::invalid_argument("BackendHIP::BlindRotateBatch: bootstrapped ciphertexts must be mod q");
        Check(fhe_hip_blind_rotate_init_batch(ctx_, B, a.data(), b.data(), acc.data()), "BlindRotateBatch");
    } else {
        Check(fhe_hip_blind_rotate_acc_batch(ctx_, B, a.data(), ctmod, acc.data()), "BlindRotateBatch");
    }
    const auto pp = params->GetPolyParams();
    const NativeInteger Q(p_.Q);
    for (size_t g = 0; g < B; ++g) {
        std::vector<NativePoly> el{poly_from(pp, acc.data() + g * 2 * N, N, Q),
                                   poly_from(pp, acc.data() + (g * 2 + 1) * N, N, Q)};
        accs[g] = std::make_shared<RLWECiphertextImpl>(std::move(el));
    }
}

void BackendHIP::ExternalProductBatch(const std::shared_ptr<RingGSWCryptoParams>& params,
                                      const std::vector<RingGSWEvalKey>& rgsws,
                                      const std::vector<RLWECiphertext>& rlwes, std::vector<RLWECiphertext>& results) {
    std::lock_guard<std::mutex> lock(mu_);
    CheckRGSW(params);
    if (rgsws.size() != rlwes.size())
        throw std::invalid_argument("Batch size mismatch in ExternalProductBatch");
    const size_t B = rlwes.size();
    results.resize(B);
    if (B == 0)
        return;
    const uint32_t N = p_.N, dG2 = 2 * (p_.digitsG - 1);
    const size_t kw = (size_t)dG2 * 2 * N;
    std::vector<uint64_t> k(B * kw), r(B * 2 * N), out(B * 2 * N);
    for (size_t g = 0; g < B; ++g) {
        rgsw_to(rgsws[g], dG2, k.data() + g * kw, N);
        if (!rlwes[g] || rlwes[g]->GetElements().size() != 2)
            throw std::invalid_argument("BackendHIP::ExternalProductBatch: RLWE ciphertexts hold two polynomials");
        for (uint32_t c = 0; c < 2; ++c)
            poly_to(rlwes[g]->GetElements()[c], r.data() + (g * 2 + c) * N, N);
    }
    Check(fhe_hip_external_product_batch(ctx_, B, k.data(), r.data(), out.data()), "ExternalProductBatch");
    const auto pp = params->GetPolyParams();
    const NativeInteger Q(p_.Q);
    for (size_t g = 0; g < B; ++g) {
        std::vector<NativePoly> el{poly_from(pp, out.data() + g * 2 * N, N, Q),
                                   poly_from(pp, out.data() + (g * 2 + 1) * N, N, Q)};
        results[g] = std::make_shared<RLWECiphertextImpl>(std::move(el));
    }
}

void BackendHIP::KeySwitchBatch(const std::shared_ptr<LWECryptoParams>& params, const std::vector<LWECiphertext>& cts,
                                const LWESwitchingKey& ks, std::vector<LWECiphertext>& results) {
    std::lock_guard<std::mutex> lock(mu_);
    CheckLWE(params);
    const size_t B = cts.size();
    results.resize(B);
    if (B == 0)
        return;
    EnsureKSK(ks);
    const uint32_t n = p_.n, N = p_.N;
    std::vector<uint64_t> a(B * N), b(B), ao(B * n), bo(B);
    for (size_t g = 0; g < B; ++g) {
        const auto& v = cts[g]->GetA();
        if (v.GetLength() != N)
            throw std::invalid_argument("BackendHIP::KeySwitchBatch: input ciphertexts have dimension N");
        for (uint32_t i = 0; i < N; ++i)
            a[g * N + i] = v[i].ConvertToInt();
        b[g] = cts[g]->GetB().ConvertToInt();
    }
    Check(fhe_hip_keyswitch_batch(ctx_, B, a.data(), b.data(), ao.data(), bo.data()), "KeySwitchBatch");
    const NativeInteger qKS(p_.qKS);
    for (size_t g = 0; g < B; ++g)
        results[g] = std::make_shared<LWECiphertextImpl>(vec_from(ao.data() + g * n, n, qKS), NativeInteger(bo[g]));
}

void BackendHIP::ModSwitchBatch(const std::shared_ptr<LWECryptoParams>& params, const std::vector<LWECiphertext>& cts,
                                std::vector<LWECiphertext>& results) {
    std::lock_guard<std::mutex> lock(mu_);
    CheckLWE(params);
    const size_t B = cts.size();
    results.resize(B);
    if (B == 0)
        return;
    const uint64_t from = cts[0]->GetModulus().ConvertToInt();
    const uint64_t to   = from == p_.Q ? p_.qKS : from == p_.qKS ? p_.q : 0;
    if (!to)
        throw std::invalid_argument("BackendHIP::ModSwitchBatch: ciphertexts must be mod Q or mod qKS");
    const uint32_t len = cts[0]->GetLength();
    std::vector<uint64_t> a(B * len), b(B), ao(B * len), bo(B);
    for (size_t g = 0; g < B; ++g) {
        const auto& v = cts[g]->GetA();
        if (v.GetLength() != len || cts[g]->GetModulus().ConvertToInt() != from)
            throw std::invalid_argument("BackendHIP::ModSwitchBatch: ciphertexts of one dimension and modulus");
        for (uint32_t i = 0; i < len; ++i)
            a[g * len + i] = v[i].ConvertToInt();
        b[g] = cts[g]->GetB().ConvertToInt();
    }
    Check(fhe_hip_modswitch_batch(ctx_, from, to, len, B, a.data(), b.data(), ao.data(), bo.data()),
          "ModSwitchBatch");
    const NativeInteger mto(to);
    for (size_t g = 0; g < B; ++g)
        results[g] = std::make_shared<LWECiphertextImpl>(vec_from(ao.data() + g * len, len, mto), NativeInteger(bo[g]));
}

// ---- packed formats ------------------------------------------------------------------------------------
DeviceBuffer BackendHIP::PackBootstrappingKey(const RingGSWACCKey& ek) {
    std::lock_guard<std::mutex> lock(mu_);
    const auto raw = RawBSK(ek);
    size_t bsize = 0, ksize = 0;
    Check(fhe_hip_pack_keys(set_, method_, raw.data(), raw.size(), nullptr, nullptr, nullptr, 0, &bsize, nullptr, 0,
                            &ksize),
          "pack_keys (size)");
    std::vector<uint8_t> bytes(bsize);
    Check(fhe_hip_pack_keys(set_, method_, raw.data(), raw.size(), nullptr, nullptr, bytes.data(), bytes.size(),
                            &bsize, nullptr, 0, &ksize),
          "PackBootstrappingKey");
    // resident for the blind rotations, and the packed bytes in device memory for the caller
    Check(fhe_hip_load_bsk(ctx_, raw.data(), raw.size()), "load bootstrapping key");
    bsk_id_ = std::shared_ptr<const void>(ek);
    DeviceBuffer buf;
    Check(fhe_hip_alloc(device_, bsize, &buf.ptr), "Allocate");
    buf.size   = bsize;
    buf.device = kBackendHIP;
    Check(fhe_hip_copy_to_device(buf.ptr, bytes.data(), bsize), "CopyToDevice");
    return buf;
}

void BackendHIP::UnpackBootstrappingKey(const DeviceBuffer& packed, RingGSWACCKey& ek) {
    std::vector<uint8_t> bytes(packed.size);
    Check(fhe_hip_copy_to_host(bytes.data(), packed.ptr, packed.size), "CopyToHost");
    std::vector<uint64_t> raw(p_.bsk_words);
    Check(fhe_hip_unpack_keys(set_, method_, bytes.data(), bytes.size(), raw.data(), raw.size(), nullptr, 0, nullptr, 0,
                              nullptr, 0),
          "UnpackBootstrappingKey");
    // rebuild with the key's own layout (rgsw-acc-cggi.cpp:39-57, rgsw-acc-lmkcdey.cpp:39-68,
    // rgsw-acc-dm.cpp:39-58); ring parameters from a context of the same set
    BinFHEContext cc;
    cc.GenerateBinFHEContext(set_, method_);
    const auto pp = cc.GetParams()->GetRingGSWParams()->GetPolyParams();
    const NativeInteger Q(p_.Q);
    const uint32_t n = p_.n, N = p_.N, dG2 = 2 * (p_.digitsG - 1);
    const size_t rgsw = (size_t)dG2 * 2 * N;
    if (method_ == GINX) {
        ek = std::make_shared<RingGSWACCKeyImpl>(1, 2, n);
        for (uint32_t i = 0; i < n; ++i)
            for (uint32_t s = 0; s < 2; ++s)
                (*ek)[0][s][i] = rgsw_from(pp, raw.data() + ((size_t)i * 2 + s) * rgsw, dG2, N, Q);
    }
    else if (method_ == LMKCDEY) {
        ek = std::make_shared<RingGSWACCKeyImpl>(1, 2, n);
        for (uint32_t i = 0; i < n; ++i)
            (*ek)[0][0][i] = rgsw_from(pp, raw.data() + (size_t)i * rgsw, dG2, N, Q);
        // (*ek)[0][1] keeps n slots with the first numAutoKeys + 1 used (rgsw-acc-lmkcdey.cpp:51-67)
        const size_t arow = (size_t)(p_.digitsG - 1) * 2 * N;
        for (uint32_t k = 0; k <= p_.numAutoKeys; ++k)
            (*ek)[0][1][k] = rgsw_from(pp, raw.data() + (size_t)n * rgsw + k * arow, p_.digitsG - 1, N, Q);
    }
    else {
        const auto rg     = cc.GetParams()->GetRingGSWParams();
        const size_t baseR = rg->GetBaseR(), dR = rg->GetDigitsR().size();
        ek = std::make_shared<RingGSWACCKeyImpl>(n, baseR, dR);
        for (uint32_t i = 0; i < n; ++i)
            for (size_t j = 1; j < baseR; ++j)
                for (size_t k = 0; k < dR; ++k)
                    (*ek)[i][j][k] = rgsw_from(pp, raw.data() + ((i * baseR + j) * dR + k) * rgsw, dG2, N, Q);
    }
}

DeviceBuffer BackendHIP::PackCiphertexts(const std::vector<LWECiphertext>& cts) {
    const size_t B  = cts.size();
    const uint32_t n = B ? cts[0]->GetLength() : p_.n;
    std::vector<uint64_t> a(B * n), b(B);
    for (size_t g = 0; g < B; ++g) {
        if (cts[g]->GetLength() != n)
            throw std::invalid_argument("BackendHIP::PackCiphertexts: ciphertexts of one dimension");
        const auto& v = cts[g]->GetA();
        for (uint32_t i = 0; i < n; ++i)
            a[g * n + i] = v[i].ConvertToInt();
        b[g] = cts[g]->GetB().ConvertToInt();
    }
    size_t size = 0;
    Check(fhe_hip_pack_lwe_batch(n, B, a.data(), b.data(), 0, nullptr, 0, &size), "pack (size)");
    std::vector<uint8_t> bytes(size);
    Check(fhe_hip_pack_lwe_batch(n, B, a.data(), b.data(), 0, bytes.data(), size, &size), "PackCiphertexts");
    DeviceBuffer buf;
    Check(fhe_hip_alloc(device_, size, &buf.ptr), "Allocate");
    buf.size   = size;
    buf.device = kBackendHIP;
    Check(fhe_hip_copy_to_device(buf.ptr, bytes.data(), size), "CopyToDevice");
    return buf;
}

// the packed LWE batch carries no modulus (PackLWEBatch writes q = 0, packed.cpp:174-176): the
// ciphertexts come back mod the parameter set's q
void BackendHIP::UnpackCiphertexts(const DeviceBuffer& packed, std::vector<LWECiphertext>& cts) {
    std::vector<uint8_t> bytes(packed.size);
    Check(fhe_hip_copy_to_host(bytes.data(), packed.ptr, packed.size), "CopyToHost");
    uint32_t n  = 0;
    size_t cnt = 0;
    Check(fhe_hip_unpack_lwe_batch(bytes.data(), bytes.size(), &n, &cnt, nullptr, nullptr), "UnpackCiphertexts");
    std::vector<uint64_t> a((size_t)cnt * n), b(cnt);
    Check(fhe_hip_unpack_lwe_batch(bytes.data(), bytes.size(), &n, &cnt, a.data(), b.data()), "UnpackCiphertexts");
    const NativeInteger q(p_.q);
    cts.resize(cnt);
    for (size_t g = 0; g < cnt; ++g)
        cts[g] = std::make_shared<LWECiphertextImpl>(vec_from(a.data() + g * n, n, q), NativeInteger(b[g]));
}

// ---- the fused gate path ---------------------------------------------------------------------------------
namespace {
// One input column in the C-ABI's mixed form (fhe_hip_eval_mixed_batch): the reference takes ciphertexts mod
// q (dimension n) or mod Q (dimension N: extended outputs, LARGE_DIM encryptions) and switches the latter
// first (binfhe-base-scheme.cpp:92-93, 150-152, 200).  Without any ciphertext mod Q the rows are n words;
// with one, every row is N words and large[g] marks the ciphertexts mod Q.
struct MixedColumn {
    std::vector<uint64_t> a, b;
    std::vector<uint8_t> large;
    bool any = false;
};
MixedColumn mixed_column(const std::vector<LWECiphertext>& v, const std::vector<size_t>& rows, uint32_t n, uint32_t N,
                         const NativeInteger& q, const NativeInteger& Q) {
    MixedColumn c;
    const size_t B = rows.size();
    c.large.assign(B, 0);
    for (size_t g = 0; g < B; ++g) {
        const auto& ct = v[rows[g]];
        if (!ct)
            throw std::invalid_argument("BackendHIP: null ciphertext");
        const bool lg = ct->GetModulus() == Q;
        if (lg ? ct->GetLength() != N : (ct->GetModulus() != q || ct->GetLength() != n))
            throw std::invalid_argument("BackendHIP: ciphertexts mod q of dimension n or mod Q of dimension N");
        c.large[g] = lg ? 1 : 0;
        c.any |= lg;
    }
    const uint32_t len = c.any ? N : n;
    c.a.assign(B * len, 0);
    c.b.resize(B);
    for (size_t g = 0; g < B; ++g) {
        const auto& ct = v[rows[g]];
        const auto& x  = ct->GetA();
        for (uint32_t i = 0; i < x.GetLength(); ++i)
            c.a[g * len + i] = x[i].ConvertToInt();
        c.b[g] = ct->GetB().ConvertToInt();
    }
    return c;
}
std::vector<size_t> all_rows(size_t B) {
    std::vector<size_t> r(B);
    for (size_t g = 0; g < B; ++g)
        r[g] = g;
    return r;
}
// fhe_hip_eval_mixed_batch over columns; outputs [B][n] mod q
void eval_mixed(fhe_hip_ctx* ctx, int op, uint32_t ptmod, std::vector<MixedColumn>& cols, size_t B, uint32_t n,
                std::vector<uint64_t>& ao, std::vector<uint64_t>& bo) {
    std::vector<const uint64_t*> pa, pb;
    std::vector<const uint8_t*> pl;
    for (auto& c : cols) {
        pa.push_back(c.a.data());
        pb.push_back(c.b.data());
        pl.push_back(c.any ? c.large.data() : nullptr);
    }
    ao.assign(B * n, 0);
    bo.assign(B, 0);
    const int rc = fhe_hip_eval_mixed_batch(ctx, op, (uint32_t)cols.size(), ptmod, B, pa.data(), pb.data(),
                                            pl.data(), ao.data(), bo.data(), 0);
    if (rc != FHE_HIP_OK) {  // BackendHIP::Check's mapping
        const std::string msg = std::string("BackendHIP: EvalBinGate (inputs mod Q): ") + fhe_hip_last_error();
        if (rc == FHE_HIP_ERR_INVALID_PARAM || rc == FHE_HIP_ERR_NULL_PTR)
            throw std::invalid_argument(msg);
        throw std::runtime_error(msg);
    }
}
}  // namespace

void BackendHIP::EvalBinGateBatch(BINGATE gate, const RingGSWBTKey& keys, const std::vector<LWECiphertext>& ct1,
                                  const std::vector<LWECiphertext>& ct2, std::vector<LWECiphertext>& out) {
    std::lock_guard<std::mutex> lock(mu_);
    if (ct1.size() != ct2.size())
        throw std::invalid_argument("Input size mismatch");
    const size_t B = ct1.size();
    out.resize(B);
    if (B == 0)
        return;
    for (size_t g = 0; g < B; ++g)
        if (ct1[g] == ct2[g])  // binfhe-base-scheme.cpp:85-86
            throw std::invalid_argument("Input ciphertexts should be independant");
    EnsureBSK(keys.BSkey);
    EnsureKSK(keys.KSkey);
    const uint32_t n = p_.n;
    const NativeInteger q(p_.q), Q(p_.Q);
    const auto rows = all_rows(B);
    std::vector<MixedColumn> cols{mixed_column(ct1, rows, n, p_.N, q, Q), mixed_column(ct2, rows, n, p_.N, q, Q)};
    std::vector<uint64_t> ao, bo;
    if (cols[0].any || cols[1].any) {  // SwitchCTtoqn of the inputs mod Q on the device first (:92-93)
        eval_mixed(ctx_, static_cast<int>(gate), 4, cols, B, n, ao, bo);
    } else {
        ao.assign(B * n, 0);
        bo.assign(B, 0);
        Check(fhe_hip_eval_bingate_batch(ctx_, static_cast<int>(gate), B, cols[0].a.data(), cols[0].b.data(),
                                         cols[1].a.data(), cols[1].b.data(), ao.data(), bo.data()),
              "EvalBinGateBatch");
    }
    for (size_t g = 0; g < B; ++g)
        out[g] = std::make_shared<LWECiphertextImpl>(vec_from(ao.data() + g * n, n, q), NativeInteger(bo[g]));
}

namespace {
// rows [first, first + count) of a ciphertext vector as the raw u64 arrays of the C-ABI
void flatten(const std::vector<LWECiphertext>& v, const std::vector<size_t>& rows, uint32_t n, uint64_t* a,
             uint64_t* b) {
    for (size_t g = 0; g < rows.size(); ++g) {
        const auto& ct = v[rows[g]];
        if (!ct)
            throw std::invalid_argument("BackendHIP: null ciphertext");
        const auto& x = ct->GetA();
        if (x.GetLength() != n)
            throw std::invalid_argument("BackendHIP: ciphertexts of dimension n");
        for (uint32_t i = 0; i < n; ++i)
            a[g * n + i] = x[i].ConvertToInt();
        b[g] = ct->GetB().ConvertToInt();
    }
}
}  // namespace

void BackendHIP::EvalFuncBatch(const RingGSWBTKey& keys, const std::vector<LWECiphertext>& cts,
                               const std::vector<NativeInteger>& lut, std::vector<LWECiphertext>& out) {
    std::lock_guard<std::mutex> lock(mu_);
    const size_t B = cts.size();
    out.resize(B);
    if (B == 0)
        return;
    EnsureBSK(keys.BSkey);
    EnsureKSK(keys.KSkey);
    std::vector<uint64_t> tab(lut.size());
    for (size_t i = 0; i < lut.size(); ++i)
        tab[i] = lut[i].ConvertToInt();
    // EvalFunc runs at each ciphertext's own modulus (binfhe-base-scheme.cpp:250): one pass per modulus
    std::vector<std::pair<uint64_t, size_t>> order(B);
    for (size_t g = 0; g < B; ++g) {
        if (!cts[g])
            throw std::invalid_argument("Ciphertext is empty");
        order[g] = {cts[g]->GetModulus().ConvertToInt(), g};
    }
    std::stable_sort(order.begin(), order.end(),
                     [](const auto& x, const auto& y) { return x.first < y.first; });
    const uint32_t n = p_.n;
    for (size_t s = 0; s < B;) {
        const uint64_t q = order[s].first;
        std::vector<size_t> rows;
        for (; s < B && order[s].first == q; ++s)
            rows.push_back(order[s].second);
        const size_t c = rows.size();
        std::vector<uint64_t> a(c * n), b(c), ao(c * n), bo(c);
        flatten(cts, rows, n, a.data(), b.data());
        Check(fhe_hip_eval_func_batch(ctx_, c, a.data(), b.data(), q, tab.data(), tab.size(), ao.data(), bo.data()),
              "EvalFuncBatch");
        const NativeInteger qn(q);
        for (size_t g = 0; g < c; ++g)
            out[rows[g]] = std::make_shared<LWECiphertextImpl>(vec_from(ao.data() + g * n, n, qn), NativeInteger(bo[g]));
    }
}

void BackendHIP::EvalFuncMultiOutputBatch(const RingGSWBTKey& keys, const std::vector<LWECiphertext>& cts,
                                          const std::vector<std::vector<NativeInteger>>& luts,
                                          std::vector<LWECiphertext>& out) {
    std::lock_guard<std::mutex> lock(mu_);
    const size_t B = cts.size(), L = luts.size();
    out.resize(B * L);
    if (B == 0 || L == 0)
        return;
    EnsureBSK(keys.BSkey);
    EnsureKSK(keys.KSkey);
    const size_t len = luts[0].size();
    std::vector<uint64_t> tab(L * len);
    for (size_t j = 0; j < L; ++j) {
        if (luts[j].size() != len)
            throw std::invalid_argument("EvalFuncMultiOutputBatch: LUTs of one length");
        for (size_t i = 0; i < len; ++i)
            tab[j * len + i] = luts[j][i].ConvertToInt();
    }
    // EvalFunc runs at each ciphertext's own modulus (binfhe-base-scheme.cpp:250): one call per modulus, all L
    // LUTs in it (output j of input i at i * L + j, batch.cpp:160-164)
    std::vector<std::pair<uint64_t, size_t>> order(B);
    for (size_t g = 0; g < B; ++g) {
        if (!cts[g])
            throw std::invalid_argument("Ciphertext is empty");
        order[g] = {cts[g]->GetModulus().ConvertToInt(), g};
    }
    std::stable_sort(order.begin(), order.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
    const uint32_t n = p_.n;
    for (size_t s0 = 0; s0 < B;) {
        const uint64_t q = order[s0].first;
        std::vector<size_t> rows;
        for (; s0 < B && order[s0].first == q; ++s0)
            rows.push_back(order[s0].second);
        const size_t c = rows.size();
        std::vector<uint64_t> a(c * n), b(c), ao(c * L * n), bo(c * L);
        flatten(cts, rows, n, a.data(), b.data());
        Check(fhe_hip_eval_func_multi_batch(ctx_, c, a.data(), b.data(), q, tab.data(), len, (uint32_t)L, ao.data(),
                                            bo.data()),
              "EvalFuncMultiOutputBatch");
        const NativeInteger qn(q);
        for (size_t g = 0; g < c; ++g)
            for (size_t j = 0; j < L; ++j)
                out[rows[g] * L + j] = std::make_shared<LWECiphertextImpl>(
                    vec_from(ao.data() + (g * L + j) * n, n, qn), NativeInteger(bo[g * L + j]));
    }
}

void BackendHIP::RefreshBatch(const RingGSWBTKey& keys, const std::vector<LWECiphertext>& cts,
                              std::vector<LWECiphertext>& out) {
    std::lock_guard<std::mutex> lock(mu_);
    const size_t B = cts.size();
    out.resize(B);
    if (B == 0)
        return;
    const NativeInteger q(p_.q), Q(p_.Q);
    // BinFHEScheme::Bootstrap (binfhe-base-scheme.cpp:190-220) per ciphertext of modulus q or Q (switched first,
    // :200, its constant Q >> 2 kept, :201); the extraction's b is Q/(2p) + 1 for the input's own plaintext
    // modulus p (:210), so one device call per distinct p
    std::vector<std::pair<uint64_t, size_t>> order(B);
    for (size_t g = 0; g < B; ++g) {
        if (!cts[g])
            throw std::invalid_argument("Ciphertext is empty");
        order[g] = {cts[g]->GetptModulus().ConvertToInt(), g};
    }
    std::stable_sort(order.begin(), order.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
    EnsureBSK(keys.BSkey);
    EnsureKSK(keys.KSkey);
    const uint32_t n = p_.n;
    for (size_t s0 = 0; s0 < B;) {
        const uint64_t p = order[s0].first;
        std::vector<size_t> rows;
        for (; s0 < B && order[s0].first == p; ++s0)
            rows.push_back(order[s0].second);
        if (p == 0 || p > 0xffffffffull)
            throw std::invalid_argument("BackendHIP::RefreshBatch: plaintext modulus");
        std::vector<MixedColumn> cols{mixed_column(cts, rows, n, p_.N, q, Q)};
        std::vector<uint64_t> ao, bo;
        eval_mixed(ctx_, FHE_HIP_OP_BOOTSTRAP, (uint32_t)p, cols, rows.size(), n, ao, bo);
        for (size_t g = 0; g < rows.size(); ++g) {
            out[rows[g]] = std::make_shared<LWECiphertextImpl>(vec_from(ao.data() + g * n, n, q), NativeInteger(bo[g]));
            out[rows[g]]->SetptModulus(NativeInteger(p));
        }
    }
}

void BackendHIP::EvalCMUXBatch(const RingGSWBTKey& keys, const std::vector<LWECiphertext>& ct0,
                               const std::vector<LWECiphertext>& ct1, const std::vector<LWECiphertext>& ct2,
                               std::vector<LWECiphertext>& out) {
    std::lock_guard<std::mutex> lock(mu_);
    const size_t B = ct0.size();
    if (ct1.size() != B || ct2.size() != B)
        throw std::invalid_argument("Input size mismatch");
    out.resize(B);
    if (B == 0)
        return;
    for (size_t g = 0; g < B; ++g)  // binfhe-base-scheme.cpp:136-143
        if (ct0[g] == ct1[g] || ct0[g] == ct2[g] || ct1[g] == ct2[g])
            throw std::invalid_argument("Input ciphertexts should be independent");
    EnsureBSK(keys.BSkey);
    EnsureKSK(keys.KSkey);
    const uint32_t n = p_.n;
    const auto rows  = all_rows(B);
    const NativeInteger q(p_.q), Q(p_.Q);
    std::vector<MixedColumn> cols{mixed_column(ct0, rows, n, p_.N, q, Q), mixed_column(ct1, rows, n, p_.N, q, Q),
                                  mixed_column(ct2, rows, n, p_.N, q, Q)};
    std::vector<uint64_t> ao(B * n), bo(B);
    if (cols[0].any || cols[1].any || cols[2].any)  // NAND's SwitchCTtoqn of inputs mod Q (:180-182, :92-93)
        eval_mixed(ctx_, static_cast<int>(CMUX), 4, cols, B, n, ao, bo);
    else
        Check(fhe_hip_eval_cmux_batch(ctx_, B, cols[0].a.data(), cols[0].b.data(), cols[1].a.data(), cols[1].b.data(),
                                      cols[2].a.data(), cols[2].b.data(), ao.data(), bo.data()),
              "EvalCMUXBatch");
    for (size_t g = 0; g < B; ++g)
        out[g] = std::make_shared<LWECiphertextImpl>(vec_from(ao.data() + g * n, n, q), NativeInteger(bo[g]));
}

namespace {
BackendHIP* default_hip() {
    return dynamic_cast<BackendHIP*>(BackendRegistry::Instance().GetDefault());
}
RingGSWBTKey context_keys(BinFHEContext& cc) {
    RingGSWBTKey keys;
    keys.BSkey = cc.GetRefreshKey();
    keys.KSkey = cc.GetSwitchKey();
    return keys;
}
// the reference's BatchResult convention: everything processed, or the whole batch failed with the message
template <typename F>
BatchResult batch_result(size_t count, F&& f) {
    try {
        f();
        return BatchResult{true, count, 0, ""};
    }
    catch (const std::exception& e) {
        return BatchResult{false, 0, count, e.what()};
    }
}
}  // namespace

BatchResult EvalFuncBatchHIP(BinFHEContext& cc, const std::vector<LWECiphertext>& ct_in,
                             const std::vector<NativeInteger>& lut, std::vector<LWECiphertext>& ct_out,
                             uint32_t flags) {
    auto* hip = default_hip();
    if (!hip)
        return lux::fhe::EvalFuncBatch(cc, ct_in, lut, ct_out, flags);
    if (ct_in.empty())
        return BatchResult{true, 0, 0, ""};
    return batch_result(ct_in.size(), [&] { hip->EvalFuncBatch(context_keys(cc), ct_in, lut, ct_out); });
}

BatchResult EvalFuncMultiOutputBatchHIP(BinFHEContext& cc, const std::vector<LWECiphertext>& ct_in,
                                        const std::vector<std::vector<NativeInteger>>& luts,
                                        std::vector<LWECiphertext>& ct_out, uint32_t flags) {
    auto* hip = default_hip();
    if (!hip)
        return lux::fhe::EvalFuncMultiOutputBatch(cc, ct_in, luts, ct_out, flags);
    if (ct_in.empty() || luts.empty())
        return BatchResult{true, 0, 0, ""};
    return batch_result(ct_in.size(), [&] { hip->EvalFuncMultiOutputBatch(context_keys(cc), ct_in, luts, ct_out); });
}

BatchResult EvalCMUXBatchHIP(BinFHEContext& cc, const std::vector<LWECiphertext>& ct_sel,
                             const std::vector<LWECiphertext>& ct_true, const std::vector<LWECiphertext>& ct_false,
                             std::vector<LWECiphertext>& ct_out, uint32_t flags) {
    auto* hip = default_hip();
    if (!hip)
        return lux::fhe::EvalCMUXBatch(cc, ct_sel, ct_true, ct_false, ct_out, flags);
    if (ct_sel.size() != ct_true.size() || ct_sel.size() != ct_false.size())
        return BatchResult{false, 0, ct_sel.size(), "Input size mismatch"};
    if (ct_sel.empty())
        return BatchResult{true, 0, 0, ""};
    return batch_result(ct_sel.size(),
                        [&] { hip->EvalCMUXBatch(context_keys(cc), ct_sel, ct_true, ct_false, ct_out); });
}

BatchResult EvalBinGateBatchHIP(BinFHEContext& cc, BINGATE gate, const std::vector<LWECiphertext>& ct1,
                                const std::vector<LWECiphertext>& ct2, std::vector<LWECiphertext>& ct_out,
                                uint32_t flags) {
    auto* hip = dynamic_cast<BackendHIP*>(BackendRegistry::Instance().GetDefault());
    if (!hip)
        return lux::fhe::EvalBinGateBatch(cc, gate, ct1, ct2, ct_out, flags);
    if (ct1.size() != ct2.size())
        return BatchResult{false, 0, ct1.size(), "Input size mismatch"};
    if (ct1.empty())
        return BatchResult{true, 0, 0, ""};
    try {
        RingGSWBTKey keys;
        keys.BSkey = cc.GetRefreshKey();
        keys.KSkey = cc.GetSwitchKey();
        hip->EvalBinGateBatch(gate, keys, ct1, ct2, ct_out);
        return BatchResult{true, ct1.size(), 0, ""};
    }
    catch (const std::exception& e) {
        return BatchResult{false, 0, ct1.size(), e.what()};
    }
}

}  // namespace lux::fhe::backend
