// Abstract specialised ("_spec") Viterbi backend.
//
// Identical declaration to the reference interface (reference: Viterbi_impl/Viterbi_spec_impl.h:6-24).
// spec_with(hmm) precomputes per-model state (for level L > 1 the products of every L-symbol
// chunk); run_Viterbi_spec(seq) then runs the chunked recurrence.
#pragma once

#include "HMM.h"

class Viterbi_spec_impl {
  public:
    Viterbi_spec_impl() = default;
    explicit Viterbi_spec_impl(size_t level) : level(level){};

    virtual void spec_with(const HMM& hmm) = 0;

    [[nodiscard]] virtual HMM::Mod_prob_vec_t
    run_Viterbi_spec(const HMM::Emit_seq_t& seq) const = 0;

    virtual ~Viterbi_spec_impl() = default;

    [[nodiscard]] size_t get_level() const { return level; }

  protected:
    // Number of consecutive observations folded into one precomputed product.
    size_t level;
};
