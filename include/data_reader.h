// Text readers for .chmm models and .ess observation files.
//
// Same declarations and behaviour as the reference readers (reference:
// Viterbi_impl/data_reader.h:8,11; formats documented at data_reader.cpp:7-15 and :81-91):
// every probability is parsed as fp32 and mapped through HMM::to_modified_prob; emissions are
// stored symbol-major; on a missing file or a bad sequence index the reader prints to stderr
// and returns an empty value.
#pragma once

#include "HMM.h"

#include <string>

// Read a .chmm file; probabilities are stored as -log2 (HMM::to_modified_prob).
HMM read_HMM(const std::string& HMM_file_name);

// Read all sequences of an .ess (emitted sequences) file.
HMM::Emit_seq_vec_t read_emit_seq(const std::string& emit_seq_file_name);
