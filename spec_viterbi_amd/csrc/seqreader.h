// Incremental .ess / FASTA sequence reader (host only, no HIP): the input side of the path
// (SURVEY.md 8(f) rank 3).  Used by stream.cpp (pipelined decoding) and the C ABI svh_reader_*;
// built alone under AddressSanitizer by tests/cpp/test_readers_asan.cpp.
#pragma once

#include <cstdint>
#include <fstream>
#include <string>
#include <vector>

#include "error.h"

namespace svh {

// Symbol of a residue under ess_files/fasta_to_ess.py:3-7 (20 amino acids, X -> 0); -1 if absent.
int fasta_symbol(unsigned char c);

// Incremental sequence reader.
//   ESS:   read_emit_seq semantics (Viterbi_impl/data_reader.cpp:93-134): count, then "index length"
//          and `length` symbols per sequence; an index out of order is an error (the reference
//          prints it and returns nothing).
//   FASTA: fasta_to_ess.py semantics: lines stripped of surrounding whitespace; a line starting
//          with '>' ends the current sequence (if it has residues); other lines append their
//          residues through the table above.  An empty line is an error (the script indexes
//          line[0]), so is a residue outside the table (the script's KeyError).
// Symbols are delivered as uint8 (the device format), so an .ess symbol must be < 256.
class SeqReader {
  public:
    SeqReader(const std::string& path, int format);  // format: SVH_FORMAT_*
    // Next chunk of whole sequences: at most max_seqs of them and at most max_symbols symbols in
    // total (a single longer sequence comes alone).  offsets gets nseq+1 entries from 0.
    // Returns false at the end of the input.
    bool next(uint64_t max_seqs, uint64_t max_symbols, std::vector<uint64_t>& offsets,
              std::vector<uint8_t>& symbols);
    bool is_fasta() const { return fasta_; }

  private:
    bool read_one(std::vector<uint8_t>& seq);
    bool read_one_ess(std::vector<uint8_t>& seq);
    bool read_one_fasta(std::vector<uint8_t>& seq);
    // buffered input
    int get();
    bool next_u64(uint64_t& x);
    bool next_line(std::string& line);

    std::string path_;
    std::ifstream in_;
    std::vector<char> buf_;
    size_t pos_ = 0, end_ = 0;
    bool fasta_ = false;
    // .ess state
    bool ess_started_ = false;
    uint64_t ess_count_ = 0, ess_index_ = 0;
    // FASTA state
    uint64_t line_no_ = 0;
    // one sequence read ahead that did not fit the previous chunk
    std::vector<uint8_t> pending_;
    bool has_pending_ = false;
};

}  // namespace svh
