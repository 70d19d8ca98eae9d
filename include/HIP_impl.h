// MI355X (gfx950) backend for the reference's Viterbi_impl interface.
//
// Drops in beside GraphBLAS_impl (reference: Viterbi_impl/GraphBLAS_impl.h:5-9, implementation
// GraphBLAS_impl.cpp:4-93): same virtual, same result (final -log2 score per state, +inf for
// unreachable states, bit-identical to GraphBLAS_impl's association).  Unlike the reference,
// the model is uploaded to HBM once and cached, not rebuilt on every call: each call compares the
// HMM it is given field by field with a host copy of the one the cached model was built from
// (memcmp of every vector), so a different or modified HMM rebuilds it.
//
// Error behaviour: the reference leaves an empty sequence / out-of-range symbol undefined; here
// they throw std::invalid_argument / std::out_of_range.  HIP failures throw std::runtime_error.
#pragma once

#include <memory>

#include "Viterbi_impl.h"

class HIP_impl final : public Viterbi_impl {
  public:
    explicit HIP_impl(int device = -1);
    ~HIP_impl() override;
    HIP_impl(const HIP_impl&) = delete;
    HIP_impl& operator=(const HIP_impl&) = delete;

    [[nodiscard]] HMM::Mod_prob_vec_t run_Viterbi(const HMM& hmm,
                                                  const HMM::Emit_seq_t& seq) const override;

    // Extensions (not in the reference interface).
    // Many sequences in one launch (one persistent workgroup per sequence).
    [[nodiscard]] std::vector<HMM::Mod_prob_vec_t>
    run_Viterbi_batch(const HMM& hmm, const HMM::Emit_seq_vec_t& seqs) const;
    // Most likely state sequence (argmin backpointers, lowest index on ties).
    [[nodiscard]] HMM::Index_vec_t decode_path(const HMM& hmm, const HMM::Emit_seq_t& seq) const;

    struct State;

  private:
    std::unique_ptr<State> st;
};
