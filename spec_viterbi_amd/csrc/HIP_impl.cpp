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

// Host copy of the model contents the cached device model was built from.  run_Viterbi compares
// the HMM it is given against it field by field (memcmp: exact, no hash collisions, and about
// 20 us for 2405.chmm's 385 KB instead of a byte-serial hash chain), so the cache follows the
// HMM passed in, including one modified in place (reference semantics: GraphBLAS_impl.cpp:9-54
// rebuilds the model from the HMM on every call).
struct ModelKey {
    bool valid = false;
    HMM copy;
    // bit patterns: a float that changed in any bit (even -0.0 vs +0.0) rebuilds the model
    template <class T> static bool same_vec(const std::vector<T>& a, const std::vector<T>& b) {
        return a.size() == b.size() && (a.empty() || std::memcmp(a.data(), b.data(), a.size() * sizeof(T)) == 0);
    }
    bool matches(const HMM& h) const {
        if (!valid || h.states_num != copy.states_num || h.emit_num != copy.emit_num) return false;
        if (!same_vec(h.start_probabilities_cols, copy.start_probabilities_cols) ||
            !same_vec(h.start_probabilities, copy.start_probabilities) || !same_vec(h.trans_rows, copy.trans_rows) ||
            !same_vec(h.trans_cols, copy.trans_cols) || !same_vec(h.trans_probs, copy.trans_probs) ||
            h.emissions.size() != copy.emissions.size())
            return false;
        for (size_t o = 0; o < h.emissions.size(); ++o)
            if (!same_vec(h.emissions[o], copy.emissions[o])) return false;
        return true;
    }
    void set(const HMM& h) {
        copy = h;
        valid = true;
    }
};

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

// One sequence: its symbols are passed in place (HMM::Emit_t is the ABI's uint64_t) and the
// scores land straight in the result vector.
HMM::Mod_prob_vec_t run_one(svh_model_t m, uint64_t n, uint32_t level, const HMM::Emit_seq_t& seq) {
    static_assert(sizeof(HMM::Emit_t) == sizeof(uint64_t), "size_t symbols");
    const uint64_t offsets[2] = {0, seq.size()};
    HMM::Mod_prob_vec_t out(n);
    check(svh_viterbi(m, level, 1, offsets, reinterpret_cast<const uint64_t*>(seq.data()), out.data(), nullptr,
                      nullptr));
    return out;
}

std::vector<HMM::Mod_prob_vec_t> run_batch(svh_model_t m, uint64_t n, uint32_t level,
                                           const HMM::Emit_seq_vec_t& seqs) {
    // the sequences as they are (Emit_t is size_t = uint64_t): no flattened copy on this side
    static_assert(sizeof(HMM::Emit_t) == sizeof(uint64_t), "Emit_t must be 64-bit");
    std::vector<const uint64_t*> ptrs(seqs.size());
    std::vector<uint64_t> lens(seqs.size());
    for (size_t q = 0; q < seqs.size(); ++q) {
        ptrs[q] = reinterpret_cast<const uint64_t*>(seqs[q].data());
        lens[q] = seqs[q].size();
    }
    std::vector<float> scores(seqs.size() * n);
    check(svh_viterbi_seqs(m, level, seqs.size(), ptrs.data(), lens.data(), scores.data(), nullptr, nullptr));
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
    ModelKey key;
    svh_model_t model = nullptr;
    ~State() {
        if (model) svh_model_destroy(model);
    }
    // Device model for `hmm`, rebuilt only when the contents change.
    svh_model_t get(const HMM& hmm) {
        if (!model || !key.matches(hmm)) {
            if (model) svh_model_destroy(model);
            model = nullptr;
            key.valid = false;
            model = create_model(hmm, device);
            key.set(hmm);
        }
        return model;
    }
};

HIP_impl::HIP_impl(int device) : st(std::make_unique<State>()) { st->device = device; }
HIP_impl::~HIP_impl() = default;

HMM::Mod_prob_vec_t HIP_impl::run_Viterbi(const HMM& hmm, const HMM::Emit_seq_t& seq) const {
    std::lock_guard<std::mutex> lock(st->mu);
    return run_one(st->get(hmm), hmm.states_num, 0, seq);
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
    std::lock_guard<std::mutex> lock(st->mu);
    if (!st->model) throw std::logic_error("run_Viterbi_spec before spec_with");
    return run_one(st->model, st->n, static_cast<uint32_t>(level), seq);
}

std::vector<HMM::Mod_prob_vec_t> HIP_spec_impl::run_Viterbi_spec_batch(
    const HMM::Emit_seq_vec_t& seqs) const {
    std::lock_guard<std::mutex> lock(st->mu);
    if (!st->model) throw std::logic_error("run_Viterbi_spec before spec_with");
    if (seqs.empty()) return {};
    return run_batch(st->model, st->n, static_cast<uint32_t>(level), seqs);
}
