// multi.cpp -- single-process multi-device gate bootstrapping: one host thread and
// one HIP stream per device, contiguous shards of the batch, keys replicated,
// no inter-device traffic on the data path (the reference's EvalBinGateBatch
// OpenMP loop, src/binfhe/lib/batch/batch.cpp:176-210, spread over GPUs).
#include "multi.h"

#include <exception>
#include <thread>

namespace fhe_amd {

MultiEngine::MultiEngine(int paramset, int method, const int* devices, int ndev) {
    if (ndev <= 0 || !devices) throw std::invalid_argument("need at least one device");
    for (int i = 0; i < ndev; ++i) engines_.emplace_back(new Engine(paramset, method, devices[i]));
}

template <typename F>
static void for_each_parallel(size_t n, F&& f) {
    std::vector<std::thread> th;
    std::vector<std::exception_ptr> err(n);
    for (size_t i = 0; i < n; ++i)
        th.emplace_back([&, i] {
            try {
                f(i);
            } catch (...) {
                err[i] = std::current_exception();
            }
        });
    for (auto& t : th) t.join();
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
}

void MultiEngine::load_keys(const uint64_t* bsk, size_t nbsk, const uint64_t* A, size_t nA, const uint64_t* B,
                            size_t nB) {
    // packed once on the host into device 0's layouts, then fanned out device to device (xGMI peer copies
    // between GPUs) instead of every device repacking the host keys
    engines_[0]->load_bsk(bsk, nbsk);
    engines_[0]->load_ksk(A, nA, B, nB);
    for_each_parallel(engines_.size() - 1, [&](size_t i) { engines_[i + 1]->copy_keys_from(*engines_[0]); });
}

void MultiEngine::eval_gate_host(int gate, size_t count, const uint64_t* a1, const uint64_t* b1, const uint64_t* a2,
                                 const uint64_t* b2, uint64_t* a_out, uint64_t* b_out) {
    const size_t nd = engines_.size(), n = engines_[0]->params().n;
    for_each_parallel(nd, [&](size_t d) {
        const size_t base = count / nd, extra = count % nd;
        const size_t lo = d * base + std::min(d, extra), len = base + (d < extra ? 1 : 0);
        if (len == 0) return;
        engines_[d]->eval_gate_host(gate, len, a1 + lo * n, b1 + lo, a2 + lo * n, b2 + lo, a_out + lo * n, b_out + lo);
    });
}

}  // namespace fhe_amd
