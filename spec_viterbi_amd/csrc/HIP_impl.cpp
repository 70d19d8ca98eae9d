// C++ drop-in classes HIP_impl / HIP_spec_impl over the C ABI (svh.h).
#include "HIP_impl.h"

#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "HIP_spec_impl.h"
#include "svh.h"

namespace {

void check(int rc) {
    if (rc == SVH_OK) return;
    const std::string msg = svh_last_error();
    switch (rc) {
        case SVH_E_RANGE: throw std::out_of_range(msg);
        case SVH_E_INVALID: throw std::invalid_argument(msg);
        case SVH_E_STATE: throw std::logic_error(msg);
        default: throw std::runtime_error(msg);
    }
}

// FNV-1a over the model contents: identifies an HMM for the device-model cache.
struct Fingerprint {
    uint64_t h = 1469598103934665603ull;
    void add(const void* p, size_t n) {
        const auto* b = static_cast<const unsigned char*>(p);
        for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    }
    template <class T> void add_vec(const std::vector<T>& v) {
        const uint64_t sz = v.size();
        add(&sz, sizeof(sz));
        if (!v.empty()) add(v.data(), v.size() * sizeof(T));
    }
};

uint64_t fingerprint(const HMM& hmm) {
    Fingerprint f;
    f.add(&hmm.states_num, sizeof(hmm.states_num));
    f.add(&hmm.emit_num, sizeof(hmm.emit_num));
    f.add_vec(hmm.start_probabilities_cols);
    f.add_vec(hmm.start_probabilities);
    f.add_vec(hmm.trans_rows);
    f.add_vec(hmm.trans_cols);
    f.add_vec(hmm.trans_probs);
    for (const auto& e : hmm.emissions) f.add_vec(e);
    return f.h;
}

svh_model_t create_model(const HMM& hmm, int device) {
    const uint64_t n = hmm.states_num, S = hmm.emit_num;
    std::vector<float> emis(S * n);
    if (hmm.emissions.size() != S) throw std::invalid_argument("HMM emissions size != emit_num");
    for (uint64_t o = 0; o < S; ++o) {
        if (hmm.emissions[o].size() != n) throw std::invalid_argument("HMM emission row size != states_num");
        std::memcpy(emis.data() + o * n, hmm.emissions[o].data(), n * sizeof(float));
    }
    const uint64_t ns = std::min(hmm.start_probabilities.size(), hmm.start_probabilities_cols.size());
    const uint64_t nt = std::min({hmm.trans_rows.size(), hmm.trans_cols.size(), hmm.trans_probs.size()});
    svh_model_opts opts{};
    opts.device = device;
    svh_model_t m = nullptr;
    static_assert(sizeof(HMM::Index_t) == sizeof(uint64_t), "size_t indices");
    check(svh_model_create(n, S, ns, reinterpret_cast<const uint64_t*>(hmm.start_probabilities_cols.data()),
                           hmm.start_probabilities.data(), emis.data(), nt,
                           reinterpret_cast<const uint64_t*>(hmm.trans_rows.data()),
                           reinterpret_cast<const uint64_t*>(hmm.trans_cols.data()),
                           hmm.trans_probs.data(), &opts, &m));
    return m;
}

std::vector<HMM::Mod_prob_vec_t> run_batch(svh_model_t m, uint64_t n, uint32_t level,
                                           const HMM::Emit_seq_vec_t& seqs) {
    std::vector<uint64_t> offsets(seqs.size() + 1, 0);
    for (size_t q = 0; q < seqs.size(); ++q) offsets[q + 1] = offsets[q] + seqs[q].size();
    std::vector<uint64_t> symbols;
    symbols.reserve(offsets.back());
    for (const auto& s : seqs) symbols.insert(symbols.end(), s.begin(), s.end());
    std::vector<float> scores(seqs.size() * n);
    check(svh_viterbi(m, level, seqs.size(), offsets.data(), symbols.data(), scores.data(), nullptr,
                      nullptr));
    std::vector<HMM::Mod_prob_vec_t> out(seqs.size());
    for (size_t q = 0; q < seqs.size(); ++q)
        out[q].assign(scores.begin() + q * n, scores.begin() + (q + 1) * n);
    return out;
}

}  // namespace

// ---- HIP_impl ---------------------------------------------------------------------------------
struct HIP_impl::State {
    int device;
    std::mutex mu;
    uint64_t key = 0;
    const HMM* last = nullptr;
    svh_model_t model = nullptr;
    ~State() {
        if (model) svh_model_destroy(model);
    }
    // Device model for `hmm`, rebuilt only when the contents change.
    svh_model_t get(const HMM& hmm) {
        const uint64_t k = fingerprint(hmm);
        if (!model || k != key) {
            if (model) svh_model_destroy(model);
            model = nullptr;
            model = create_model(hmm, device);
            key = k;
        }
        last = &hmm;
        return model;
    }
};

HIP_impl::HIP_impl(int device) : st(std::make_unique<State>()) { st->device = device; }
HIP_impl::~HIP_impl() = default;

HMM::Mod_prob_vec_t HIP_impl::run_Viterbi(const HMM& hmm, const HMM::Emit_seq_t& seq) const {
    std::lock_guard<std::mutex> lock(st->mu);
    svh_model_t m = st->get(hmm);
    return std::move(run_batch(m, hmm.states_num, 0, HMM::Emit_seq_vec_t{seq})[0]);
}

std::vector<HMM::Mod_prob_vec_t> HIP_impl::run_Viterbi_batch(const HMM& hmm,
                                                            const HMM::Emit_seq_vec_t& seqs) const {
    std::lock_guard<std::mutex> lock(st->mu);
    if (seqs.empty()) return {};
    return run_batch(st->get(hmm), hmm.states_num, 0, seqs);
}

HMM::Index_vec_t HIP_impl::decode_path(const HMM& hmm, const HMM::Emit_seq_t& seq) const {
    std::lock_guard<std::mutex> lock(st->mu);
    svh_model_t m = st->get(hmm);
    const uint64_t offsets[2] = {0, seq.size()};
    std::vector<int32_t> path(seq.size());
    check(svh_viterbi(m, 0, 1, offsets, reinterpret_cast<const uint64_t*>(seq.data()), nullptr,
                      nullptr, path.data()));
    HMM::Index_vec_t out(path.size());
    for (size_t i = 0; i < path.size(); ++i)
        out[i] = path[i] < 0 ? static_cast<HMM::Index_t>(-1) : static_cast<HMM::Index_t>(path[i]);
    return out;
}

// ---- HIP_spec_impl ----------------------------------------------------------------------------
struct HIP_spec_impl::State {
    int device;
    std::mutex mu;
    svh_model_t model = nullptr;
    uint64_t n = 0;
    ~State() {
        if (model) svh_model_destroy(model);
    }
};

HIP_spec_impl::HIP_spec_impl(size_t level, int device)
    : Viterbi_spec_impl(level), st(std::make_unique<State>()) {
    st->device = device;
}

HIP_spec_impl::HIP_spec_impl(const HMM& hmm, size_t level, int device)
    : HIP_spec_impl(level, device) {
    spec_with(hmm);
}

HIP_spec_impl::~HIP_spec_impl() = default;

void HIP_spec_impl::spec_with(const HMM& hmm) {
    std::lock_guard<std::mutex> lock(st->mu);
    if (st->model) svh_model_destroy(st->model);
    st->model = nullptr;
    st->model = create_model(hmm, st->device);
    st->n = hmm.states_num;
    check(svh_spec_build(st->model, static_cast<uint32_t>(level), nullptr));
}

HMM::Mod_prob_vec_t HIP_spec_impl::run_Viterbi_spec(const HMM::Emit_seq_t& seq) const {
    auto r = run_Viterbi_spec_batch(HMM::Emit_seq_vec_t{seq});
    return std::move(r[0]);
}

std::vector<HMM::Mod_prob_vec_t> HIP_spec_impl::run_Viterbi_spec_batch(
    const HMM::Emit_seq_vec_t& seqs) const {
    std::lock_guard<std::mutex> lock(st->mu);
    if (!st->model) throw std::logic_error("run_Viterbi_spec before spec_with");
    if (seqs.empty()) return {};
    return run_batch(st->model, st->n, static_cast<uint32_t>(level), seqs);
}
