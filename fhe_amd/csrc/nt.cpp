// nt.cpp -- host number theory (see nt.h).
#include "nt.h"

namespace fhe_amd {

uint64_t powmod(uint64_t b, uint64_t e, uint64_t m) {
    uint64_t r = 1 % m;
    b %= m;
    while (e) {
        if (e & 1) r = mulmod(r, b, m);
        b = mulmod(b, b, m);
        e >>= 1;
    }
    return r;
}

bool is_prime(uint64_t n) {
    static const uint64_t bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    if (n < 2) return false;
    for (uint64_t b : bases) {
        if (n == b) return true;
        if (n % b == 0) return false;
    }
    uint64_t d = n - 1;
    int s = 0;
    while (!(d & 1)) { d >>= 1; ++s; }
    for (uint64_t b : bases) {
        uint64_t x = powmod(b, d, n);
        if (x == 1 || x == n - 1) continue;
        bool ok = false;
        for (int r = 1; r < s && !ok; ++r) {
            x = mulmod(x, x, n);
            ok = (x == n - 1);
        }
        if (!ok) return false;
    }
    return true;
}

uint64_t last_prime(uint32_t bits, uint64_t m) {
    uint64_t q = (uint64_t)1 << bits, r = q % m, qn = q + 1 - r;
    if (r < 2) qn -= m;
    while (!is_prime(qn)) qn -= m;
    return qn;
}

uint64_t root_of_unity(uint64_t m, uint64_t Q) {
    uint64_t phi = Q - 1, t = phi;
    std::vector<uint64_t> f;
    for (uint64_t p = 2; p * p <= t; ++p)
        if (t % p == 0) { f.push_back(p); while (t % p == 0) t /= p; }
    if (t > 1) f.push_back(t);
    uint64_t g = 2;
    for (;; ++g) {
        bool ok = true;
        for (uint64_t p : f) if (powmod(g, phi / p, Q) == 1) { ok = false; break; }
        if (ok) break;
    }
    uint64_t r = powmod(g, phi / m, Q), best = 0, x = 1;
    for (uint64_t k = 1; k < m; ++k) {
        x = mulmod(x, r, Q);
        if ((k & 1) && x != 1 && (best == 0 || x < best)) best = x;
    }
    return best;
}

void HostNtt::init(uint32_t N_, uint64_t Q_, uint64_t psi_) {
    N = N_; logN = ilog2(N); Q = Q_; psi = psi_;
    tab.assign(N, 0); tabI.assign(N, 0);
    uint64_t psiI = invmod(psi, Q), x = 1, xi = 1;
    for (uint32_t i = 0; i < N; ++i) {
        uint32_t r = reverse_bits(i, logN);
        tab[r] = x; tabI[r] = xi;
        x = mulmod(x, psi, Q); xi = mulmod(xi, psiI, Q);
    }
    ninv = invmod(N, Q);
}

void HostNtt::forward(uint64_t* a) const {
    for (uint32_t m = 1, t = N >> 1; m < N; m <<= 1, t >>= 1)
        for (uint32_t i = 0; i < m; ++i) {
            uint64_t w = tab[m + i];
            for (uint32_t j = 2 * i * t; j < 2 * i * t + t; ++j) {
                uint64_t hi = mulmod(a[j + t], w, Q), lo = a[j];
                a[j] = addmod(lo, hi, Q);
                a[j + t] = submod(lo, hi, Q);
            }
        }
}

void HostNtt::inverse(uint64_t* a) const {
    for (uint32_t m = N >> 1, t = 1; m >= 1; m >>= 1, t <<= 1)
        for (uint32_t i = 0; i < m; ++i) {
            uint64_t w = tabI[m + i];
            for (uint32_t j = 2 * i * t; j < 2 * i * t + t; ++j) {
                uint64_t lo = a[j], hi = a[j + t];
                a[j] = addmod(lo, hi, Q);
                a[j + t] = mulmod(submod(lo, hi, Q), w, Q);
            }
        }
    for (uint32_t i = 0; i < N; ++i) a[i] = mulmod(a[i], ninv, Q);
}

}  // namespace fhe_amd
