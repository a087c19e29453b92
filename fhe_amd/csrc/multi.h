// multi.h -- see multi.cpp.
#pragma once
#include <memory>
#include <vector>

#include "engine.h"

namespace fhe_amd {

class MultiEngine {
public:
    MultiEngine(int paramset, int method, const int* devices, int ndev);
    size_t devices() const { return engines_.size(); }
    const Params& params() const { return engines_[0]->params(); }
    void load_keys(const uint64_t* bsk, size_t nbsk, const uint64_t* A, size_t nA, const uint64_t* B, size_t nB);
    void eval_gate_host(int gate, size_t count, const uint64_t* a1, const uint64_t* b1, const uint64_t* a2,
                        const uint64_t* b2, uint64_t* a_out, uint64_t* b_out);

private:
    std::vector<std::unique_ptr<Engine>> engines_;
};

}  // namespace fhe_amd
