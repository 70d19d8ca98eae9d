// MI355X (gfx950) backend for the reference's Viterbi_spec_impl interface.
//
// Drops in beside GraphBLAS_spec_impl (reference: Viterbi_impl/GraphBLAS_spec_impl.h:8-30,
// implementation GraphBLAS_spec_impl.cpp).  spec_with(hmm) uploads the model and prepares level
// `level` (GraphBLAS_spec_impl.cpp:15-36, 146-181): level 2 evaluates each chunk's product on chip
// from the folded sparse matrices, nothing precomputed (the pipelined latency plan for MSV-shaped
// models with every score >= 0, spec2_kernel otherwise and for the rows the pipelined pass flags;
// DESIGN.md 5h, 5j); level >= 3 precomputes the emit_num^level dense products in HBM.
// run_Viterbi_spec(seq) runs the chunked recurrence (:50-97).  Results are bit-identical to
// GraphBLAS_spec_impl(level).
//
// Error behaviour: the reference throws std::out_of_range from unordered_map::at for an
// unknown symbol chunk (:74); here any out-of-range symbol throws std::out_of_range.
// run_Viterbi_spec before spec_with throws std::logic_error (undefined in the reference).
#pragma once

#include <memory>

#include "Viterbi_spec_impl.h"

class HIP_spec_impl final : public Viterbi_spec_impl {
  public:
    explicit HIP_spec_impl(size_t level, int device = -1);
    HIP_spec_impl(const HMM& hmm, size_t level, int device = -1);
    ~HIP_spec_impl() override;
    HIP_spec_impl(const HIP_spec_impl&) = delete;
    HIP_spec_impl& operator=(const HIP_spec_impl&) = delete;

    void spec_with(const HMM& hmm) override;

    [[nodiscard]] HMM::Mod_prob_vec_t run_Viterbi_spec(const HMM::Emit_seq_t& seq) const override;

    // Extension: many sequences in one pass.
    [[nodiscard]] std::vector<HMM::Mod_prob_vec_t>
    run_Viterbi_spec_batch(const HMM::Emit_seq_vec_t& seqs) const;

    struct State;

  private:
    std::unique_ptr<State> st;
};
