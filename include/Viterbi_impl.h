// Abstract non-specialised Viterbi backend.
//
// Identical declaration to the reference interface (reference: Viterbi_impl/Viterbi_impl.h:6-11)
// so HIP_impl (include/HIP_impl.h) drops in beside GraphBLAS_impl / CUSP_impl / cuASR_impl.
// run_Viterbi returns the final score vector (-log2 of the best path probability ending in each
// state), length hmm.states_num, +inf for unreachable states.
#pragma once

#include "HMM.h"

class Viterbi_impl {
  public:
    [[nodiscard]] virtual HMM::Mod_prob_vec_t run_Viterbi(const HMM& hmm,
                                                          const HMM::Emit_seq_t& seq) const = 0;
    virtual ~Viterbi_impl() = default;
};
