// Host side of the pipelined file decoder (stream.cpp decode_file): the parser thread's chunks of
// whole sequences and the bounded queue that hands them to the decoding thread.  No HIP: the
// sanitizer build (tests/cpp/test_host_asan.cpp) runs it under AddressSanitizer + UBSan.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <exception>
#include <mutex>
#include <vector>

#include "seqreader.h"

namespace svh {

struct Chunk {
    std::vector<uint64_t> offsets;  // nseq + 1 prefix offsets into symbols (from 0)
    std::vector<uint8_t> symbols;   // the device format (uint8)
    uint64_t first = 0;             // index of the chunk's first sequence in the file
};

// Bounded hand-off from the parser thread; an exception or the end closes it.
class ChunkQueue {
  public:
    explicit ChunkQueue(size_t cap) : cap_(cap) {}
    bool push(Chunk&& c);                // false: the consumer stopped
    void close(std::exception_ptr e);    // the producer's end (with its error, if any)
    bool pop(Chunk& c);                  // false at the end; rethrows the producer's error
    void stop();                         // the consumer's end: a blocked push returns false

  private:
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Chunk> q_;
    size_t cap_;
    bool closed_ = false, stop_ = false;
    std::exception_ptr err_;
};

// The parser thread's body: chunks of at most max_seqs sequences and max_symbols symbols (a single
// longer sequence alone) from `reader` into `queue` until the end of the file or a stop; the queue
// is closed with the reader's error, if any.
void produce_chunks(SeqReader& reader, ChunkQueue& queue, uint64_t max_seqs, uint64_t max_symbols);

}  // namespace svh
