// cereal.cpp -- see cereal.h.
#include "cereal.h"

#include <cstring>
#include <map>
#include <stdexcept>

namespace fhe_amd {
namespace {

constexpr uint32_t kSameType = 0x40000000u;  // polymorphic id: dynamic type == static type
constexpr uint32_t kNewPtr = 0x80000000u;    // pointer id: first occurrence, object follows

// the classes that carry a version word (first occurrence per archive)
enum Cls { C_ACC, C_EVALKEY, C_POLY, C_VEC, C_INT, C_ILPARAMS, C_ELEMPARAMS, C_KSK, C_CT, C_SK, C_CTX, C_CPARAMS,
           C_LWEP, C_RGSWP, C_COUNT };

struct Reader {
    const uint8_t* p;
    const uint8_t* end;
    bool seen[C_COUNT] = {};
    std::map<uint32_t, uint64_t> params_q;  // pointer id of each ILParams -> its modulus

    Reader(const uint8_t* d, size_t n) : p(d), end(d + n) {
        if (!d || n < 1) throw std::invalid_argument("cereal: empty archive");
        if (u8() != 1) throw std::invalid_argument("cereal: not a little-endian PortableBinary archive");
    }
    void need(size_t n) const {
        if ((size_t)(end - p) < n) throw std::invalid_argument("cereal: archive truncated");
    }
    uint8_t u8() { need(1); return *p++; }
    uint32_t u32() { need(4); uint32_t v; std::memcpy(&v, p, 4); p += 4; return v; }
    uint64_t u64() { need(8); uint64_t v; std::memcpy(&v, p, 8); p += 8; return v; }
    void version(Cls c, uint32_t maxv) {
        if (seen[c]) return;
        seen[c] = true;
        if (u32() > maxv) throw std::invalid_argument("cereal: object version is from a later version of the library");
    }
    // polymorphic shared_ptr header; returns false for null, sets is_new
    bool ptr(bool& is_new, uint32_t& id) {
        const uint32_t pid = u32();
        if (pid == 0) return false;
        if (pid != kSameType) throw std::invalid_argument("cereal: unexpected polymorphic type");
        id = u32();
        is_new = (id & kNewPtr) != 0;
        id &= ~kNewPtr;
        return true;
    }
    uint64_t integer() { version(C_INT, 1); return u64(); }
    // NativeVector (mubintvecnat.h:656-665): size, u64 data, modulus
    uint64_t vec(uint64_t* out, size_t expect) {
        version(C_VEC, 1);
        const uint64_t n = u64();
        if (n != expect) throw std::invalid_argument("cereal: vector has the wrong length");
        need(n * 8);
        std::memcpy(out, p, n * 8);
        p += n * 8;
        return integer();
    }
    // NativePoly (poly.h:336-340): unique_ptr<NativeVector>, Format, shared_ptr<ILNativeParams>
    void poly(uint64_t* out, const Params& P) {
        version(C_POLY, 1);
        if (u32() != kSameType || u8() != 1) throw std::invalid_argument("cereal: polynomial without values");
        const uint64_t mod = vec(out, P.N);
        if (u32() != 0) throw std::invalid_argument("cereal: key polynomial not in EVALUATION format");
        bool is_new;
        uint32_t id;
        if (!ptr(is_new, id)) throw std::invalid_argument("cereal: polynomial without parameters");
        if (is_new) {
            // ILParamsImpl -> ElemParams (ilparams.h:139-142, elemparams.h:229-236)
            version(C_ILPARAMS, 1);
            version(C_ELEMPARAMS, 1);
            const uint32_t co = u32(), rd = u32();
            const uint64_t cm = integer(), ru = integer();
            integer();
            integer();
            if (co != 2 * P.N || rd != P.N || cm != P.Q || ru != P.psi)
                throw std::invalid_argument("cereal: ring parameters do not match the context");
            params_q[id] = cm;
        } else if (!params_q.count(id)) {
            throw std::invalid_argument("cereal: dangling parameter reference");
        }
        if (mod != P.Q) throw std::invalid_argument("cereal: polynomial modulus does not match Q");
        for (uint32_t j = 0; j < P.N; ++j)
            if (out[j] >= P.Q) throw std::invalid_argument("cereal: coefficient not reduced mod Q");
    }
    // shared_ptr<RingGSWEvalKeyImpl> (rgsw-evalkey.h:133-137): vector<vector<NativePoly>>
    bool evalkey(uint64_t* out, uint32_t rows, const Params& P) {
        bool is_new;
        uint32_t id;
        if (!ptr(is_new, id)) return false;
        if (!is_new) throw std::invalid_argument("cereal: shared RGSW keys are not supported");
        version(C_EVALKEY, 1);
        if (u64() != rows) throw std::invalid_argument("cereal: RGSW key has the wrong number of rows");
        for (uint32_t r = 0; r < rows; ++r) {
            if (u64() != 2) throw std::invalid_argument("cereal: RGSW row is not an RLWE pair");
            for (uint32_t c = 0; c < 2; ++c) poly(out + ((size_t)r * 2 + c) * P.N, P);
        }
        return true;
    }
    void top(Cls c) {
        bool is_new;
        uint32_t id;
        if (!ptr(is_new, id) || !is_new) throw std::invalid_argument("cereal: null object");
        version(c, 1);
    }
    void done() const {
        if (p != end) throw std::invalid_argument("cereal: trailing bytes after the object");
    }
};

struct Writer {
    std::string s;
    bool seen[C_COUNT] = {};
    uint32_t next_id = 1;
    uint32_t params_id = 0;

    Writer() { u8(1); }
    void u8(uint8_t v) { s.push_back((char)v); }
    void u32(uint32_t v) { s.append(reinterpret_cast<const char*>(&v), 4); }
    void u64(uint64_t v) { s.append(reinterpret_cast<const char*>(&v), 8); }
    // the reference writes cereal's default version 0 for classes without CEREAL_CLASS_VERSION
    // and SerializedVersion() = 1 for those with it (lattice.cpp:74-77, benative-math-impl.cpp:86-87)
    void version(Cls c) {
        if (seen[c]) return;
        seen[c] = true;
        const bool registered = c == C_POLY || c == C_VEC || c == C_INT || c == C_ILPARAMS || c == C_ELEMPARAMS;
        u32(registered ? 1 : 0);
    }
    void new_ptr() { u32(kSameType); u32(kNewPtr | next_id++); }
    void integer(uint64_t v) { version(C_INT); u64(v); }
    void vec(const uint64_t* v, size_t n, uint64_t mod) {
        version(C_VEC);
        u64(n);
        s.append(reinterpret_cast<const char*>(v), n * 8);
        integer(mod);
    }
    void poly(const uint64_t* v, const Params& P) {
        version(C_POLY);
        u32(kSameType);
        u8(1);
        vec(v, P.N, P.Q);
        u32(0);  // EVALUATION
        if (params_id) {
            u32(kSameType);
            u32(params_id);
            return;
        }
        params_id = next_id;
        new_ptr();
        version(C_ILPARAMS);
        version(C_ELEMPARAMS);
        u32(2 * P.N);
        u32(P.N);
        integer(P.Q);
        integer(P.psi);
        integer(0);
        integer(0);
    }
    void evalkey(const uint64_t* v, uint32_t rows, const Params& P) {
        new_ptr();
        version(C_EVALKEY);
        u64(rows);
        for (uint32_t r = 0; r < rows; ++r) {
            u64(2);
            for (uint32_t c = 0; c < 2; ++c) poly(v + ((size_t)r * 2 + c) * P.N, P);
        }
    }
};

// RingGSWACCKeyImpl dimensions and the raw-layout slot of each [i][j][k] (-1: null)
struct AccShape {
    uint32_t d1, d2, d3;
};
AccShape acc_shape(const Params& p) {
    if (p.method == M_AP) return {p.n, p.baseR, p.digitsR};  // RingGSWACCKeyImpl(n, baseR, digitsR)
    return {1, 2, p.n};                                       // RingGSWACCKeyImpl(1, 2, n)
}
// returns the raw word offset of element (i, j, k) and its row count, or false for a null slot
bool acc_slot(const Params& p, uint32_t i, uint32_t j, uint32_t k, size_t& off, uint32_t& rows) {
    const size_t rg = (size_t)p.digitsG2 * 2 * p.N;
    if (p.method == M_GINX) {  // [0][ks][i] -> raw [i][ks]
        off = ((size_t)k * 2 + j) * rg;
        rows = p.digitsG2;
        return true;
    }
    if (p.method == M_AP) {  // [i][j][k], j = 0 never generated (rgsw-acc-dm.cpp:39-58)
        off = (((size_t)i * p.baseR + j) * p.digitsR + k) * rg;
        rows = p.digitsG2;
        return j != 0;
    }
    if (j == 0) {  // LMKCDEY [0][0][i]: RGSW(X^{s_i})
        off = (size_t)k * rg;
        rows = p.digitsG2;
        return true;
    }
    // [0][1][k], k <= numAutoKeys: automorphism keys of digitsG - 1 rows
    rows = p.digitsG - 1;
    off = (size_t)p.n * rg + (size_t)k * rows * 2 * p.N;
    return k <= p.numAutoKeys;
}

}  // namespace

void cereal_read_bsk(const Params& p, const uint8_t* data, size_t size, std::vector<uint64_t>& bsk) {
    Reader r(data, size);
    r.top(C_ACC);
    const AccShape sh = acc_shape(p);
    bsk.assign(p.bsk_words(), 0);
    if (r.u64() != sh.d1) throw std::invalid_argument("cereal: refresh key does not match the parameter set");
    for (uint32_t i = 0; i < sh.d1; ++i) {
        if (r.u64() != sh.d2) throw std::invalid_argument("cereal: refresh key does not match the parameter set");
        for (uint32_t j = 0; j < sh.d2; ++j) {
            if (r.u64() != sh.d3) throw std::invalid_argument("cereal: refresh key does not match the parameter set");
            for (uint32_t k = 0; k < sh.d3; ++k) {
                size_t off;
                uint32_t rows;
                const bool want = acc_slot(p, i, j, k, off, rows);
                const bool got = want ? r.evalkey(bsk.data() + off, rows, p) : r.evalkey(nullptr, 0, p);
                if (want && !got) throw std::invalid_argument("cereal: refresh key is missing an RGSW key");
            }
        }
    }
    r.done();
}

void cereal_read_ksk(const Params& p, const uint8_t* data, size_t size, std::vector<uint64_t>& A,
                     std::vector<uint64_t>& B) {
    Reader r(data, size);
    r.top(C_KSK);
    const size_t rows = p.ksk_rows();
    A.assign(rows * p.n, 0);
    B.assign(rows, 0);
    // m_keyA [N][baseKS][digitsKS] NativeVector(n), m_keyB [N][baseKS][digitsKS] NativeInteger
    auto dims = [&](auto&& leaf) {
        if (r.u64() != p.N) throw std::invalid_argument("cereal: switching key does not match the parameter set");
        for (uint32_t i = 0; i < p.N; ++i) {
            if (r.u64() != p.baseKS) throw std::invalid_argument("cereal: switching key does not match the parameter set");
            for (uint32_t j = 0; j < p.baseKS; ++j) {
                if (r.u64() != p.digitsKS)
                    throw std::invalid_argument("cereal: switching key does not match the parameter set");
                for (uint32_t k = 0; k < p.digitsKS; ++k) leaf(((size_t)i * p.baseKS + j) * p.digitsKS + k);
            }
        }
    };
    dims([&](size_t row) {
        if (r.vec(A.data() + row * p.n, p.n) != p.qKS) throw std::invalid_argument("cereal: switching key modulus is not qKS");
    });
    dims([&](size_t row) { B[row] = r.integer(); });
    r.done();
    for (uint64_t v : A)
        if (v >= p.qKS) throw std::invalid_argument("cereal: switching key value not reduced mod qKS");
    for (uint64_t v : B)
        if (v >= p.qKS) throw std::invalid_argument("cereal: switching key value not reduced mod qKS");
}

std::string cereal_write_bsk(const Params& p, const uint64_t* bsk) {
    Writer w;
    w.new_ptr();
    w.version(C_ACC);
    const AccShape sh = acc_shape(p);
    w.u64(sh.d1);
    for (uint32_t i = 0; i < sh.d1; ++i) {
        w.u64(sh.d2);
        for (uint32_t j = 0; j < sh.d2; ++j) {
            w.u64(sh.d3);
            for (uint32_t k = 0; k < sh.d3; ++k) {
                size_t off;
                uint32_t rows;
                if (acc_slot(p, i, j, k, off, rows))
                    w.evalkey(bsk + off, rows, p);
                else
                    w.u32(0);  // null shared_ptr
            }
        }
    }
    return std::move(w.s);
}

std::string cereal_write_ksk(const Params& p, const uint64_t* A, const uint64_t* B) {
    Writer w;
    w.new_ptr();
    w.version(C_KSK);
    auto dims = [&](auto&& leaf) {
        w.u64(p.N);
        for (uint32_t i = 0; i < p.N; ++i) {
            w.u64(p.baseKS);
            for (uint32_t j = 0; j < p.baseKS; ++j) {
                w.u64(p.digitsKS);
                for (uint32_t k = 0; k < p.digitsKS; ++k) leaf(((size_t)i * p.baseKS + j) * p.digitsKS + k);
            }
        }
    };
    dims([&](size_t row) { w.vec(A + row * p.n, p.n, p.qKS); });
    dims([&](size_t row) { w.integer(B[row]); });
    return std::move(w.s);
}

CerealLwe cereal_read_lwe(const uint8_t* data, size_t size, bool is_key) {
    Reader r(data, size);
    r.top(is_key ? C_SK : C_CT);
    CerealLwe out;
    r.version(C_VEC, 1);
    const uint64_t n = r.u64();
    if (n > (1u << 20)) throw std::invalid_argument("cereal: implausible LWE dimension");
    r.need(n * 8);
    out.a.resize(n);
    std::memcpy(out.a.data(), r.p, n * 8);
    r.p += n * 8;
    out.mod = r.integer();
    if (!is_key) out.b = r.integer();
    r.done();
    return out;
}

std::string cereal_write_lwe(const uint64_t* a, uint32_t n, uint64_t b, uint64_t mod, bool is_key) {
    Writer w;
    w.new_ptr();
    w.version(is_key ? C_SK : C_CT);
    w.vec(a, n, mod);
    if (!is_key) w.integer(b);
    return std::move(w.s);
}

// ---- the cryptoContext archive ----------------------------------------------------------------------
namespace {
double f64_of(uint64_t bits) {
    double d;
    std::memcpy(&d, &bits, 8);
    return d;
}
uint64_t bits_of(double d) {
    uint64_t b;
    std::memcpy(&b, &d, 8);
    return b;
}
// lwe-cryptoparameters.h:66-86 / binfhecontext.cpp:161-167: both Gaussians of a row use STD_DEV
constexpr double kStdDev = 3.19;
}  // namespace

CerealContext cereal_read_context(const uint8_t* data, size_t size) {
    Reader r(data, size);
    CerealContext c;
    r.version(C_CTX, 1);           // BinFHEContext (the top-level object, by value)
    r.top(C_CPARAMS);              // "params": shared_ptr<BinFHECryptoParams>
    r.top(C_LWEP);                 // "lweparams"
    c.n = r.u32();
    c.N = r.u32();
    c.q = r.integer();
    c.Q = r.integer();
    c.qKS = r.integer();
    c.sigma = f64_of(r.u64());
    c.sigmaKS = f64_of(r.u64());
    c.baseKS = r.u32();
    r.top(C_RGSWP);                // "rgswparams"
    c.rN = r.u32();
    c.rQ = r.integer();
    c.rq = r.integer();
    c.baseR = r.u32();
    c.baseG = r.u32();
    c.method = r.u32();
    c.rsigma = f64_of(r.u64());
    c.digitsG = r.u32();
    bool is_new;                   // "bparams": shared_ptr<ILNativeParams>
    uint32_t id;
    if (!r.ptr(is_new, id) || !is_new) throw std::invalid_argument("cereal: context without ring parameters");
    r.version(C_ILPARAMS, 1);
    r.version(C_ELEMPARAMS, 1);
    c.order = r.u32();
    c.ringDim = r.u32();
    c.mod = r.integer();
    c.root = r.integer();
    c.bigMod = r.integer();
    c.bigRoot = r.integer();
    c.numAutoKeys = r.u32();
    r.done();
    if (c.rN != c.N || c.rQ != c.Q || c.rq != c.q || c.ringDim != c.N || c.order != 2 * c.N || c.mod != c.Q)
        throw std::invalid_argument("cereal: inconsistent context parameters");
    return c;
}

std::string cereal_write_context(const Params& p) {
    if (is_large(p.paramset)) throw std::invalid_argument("cereal: context archives of the standard rows only");
    Writer w;
    w.version(C_CTX);
    w.new_ptr();
    w.version(C_CPARAMS);
    w.new_ptr();
    w.version(C_LWEP);
    w.u32(p.n);
    w.u32(p.N);
    w.integer(p.q);
    w.integer(p.Q);
    w.integer(p.qKS);
    w.u64(bits_of(kStdDev));
    w.u64(bits_of(kStdDev));
    w.u32(p.baseKS);
    w.new_ptr();
    w.version(C_RGSWP);
    w.u32(p.N);
    w.integer(p.Q);
    w.integer(p.q);
    w.u32(p.baseR);
    w.u32(p.baseG);
    w.u32((uint32_t)p.method);
    w.u64(bits_of(kStdDev));
    w.u32(p.digitsG);
    w.new_ptr();
    w.version(C_ILPARAMS);
    w.version(C_ELEMPARAMS);
    w.u32(2 * p.N);
    w.u32(p.N);
    w.integer(p.Q);
    w.integer(p.psi);
    w.integer(0);
    w.integer(0);
    w.u32(p.numAutoKeys);
    return w.s;
}

bool cereal_context_paramset(const CerealContext& c, int& paramset, int& method) {
    for (int ps = 0; ps < paramset_rows(); ++ps) {
        if (!method_compatible(ps, (int)c.method)) continue;
        const Params p = make_params(ps, (int)c.method);
        if (p.n == c.n && p.N == c.N && p.q == c.q && p.Q == c.Q && p.qKS == c.qKS && p.baseKS == c.baseKS &&
            p.baseR == c.baseR && p.baseG == c.baseG && p.digitsG == c.digitsG && p.numAutoKeys == c.numAutoKeys &&
            p.psi == c.root && c.sigma == kStdDev && c.sigmaKS == kStdDev && c.rsigma == kStdDev) {
            paramset = ps;
            method = (int)c.method;
            return true;
        }
    }
    return false;
}

}  // namespace fhe_amd
