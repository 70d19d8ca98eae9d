// Streaming ingestion: observation sequences read incrementally from .ess
// or FASTA files into batches, and a pipelined decoder that overlaps parsing, transfers and the
// Viterbi kernels.  Used by the C ABI (svh_reader_*, svh_decode_file in svh_api.cpp).
#pragma once

#include <cstdint>
#include <string>

#include "runtime.h"
#include "seqreader.h"

namespace svh {

// Result hand-off of decode_file: one call per chunk, in file order.  Non-zero return stops.
typedef int (*ResultFn)(void* user, uint64_t first_seq, uint64_t nseq, const uint64_t* offsets,
                        const float* scores, const int64_t* best_state, const int32_t* paths);

// Decode a whole file chunk by chunk: a host thread parses chunk k+1 while chunk k is uploaded
// and decoded on the model's stream; chunk k-1's results come back on a copy stream into pinned
// buffers and go to `fn` on the calling thread.  Two batches alternate, their device buffers
// grow only.  Returns the number of sequences decoded.
uint64_t decode_file(Model* model, const std::string& path, int format, uint32_t level, uint32_t flags,
                     uint64_t max_seqs, uint64_t max_symbols, ResultFn fn, void* user);

}  // namespace svh
