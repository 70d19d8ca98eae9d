// Streaming ingestion and the pipelined file decoder (stream.h).
#include "stream.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <exception>
#include <memory>
#include <mutex>
#include <thread>

#include "chunker.h"
#include "svh.h"

namespace svh {

// ---------------------------------------------------------------------------------------------
// Pipelined decoder
// ---------------------------------------------------------------------------------------------
namespace {

struct Slot {
    std::unique_ptr<Batch> batch;
    Chunk chunk;
    hipEvent_t done = nullptr;
    Pinned<float> scores;
    Pinned<int64_t> best;
    Pinned<int32_t> paths;
};

}  // namespace

uint64_t decode_file(Model* model, const std::string& path, int format, uint32_t level, uint32_t flags,
                     uint64_t max_seqs, uint64_t max_symbols, ResultFn fn, void* user) {
    if (!fn) throw Error(SVH_E_INVALID, "null result callback");
    if (max_seqs == 0) throw Error(SVH_E_INVALID, "max_seqs must be > 0");
    const bool want_paths = (flags & SVH_BATCH_PATHS) != 0;
    auto reader = std::make_shared<SeqReader>(path, format);  // opens (errors surface here)

    ChunkQueue queue(2);
    std::thread producer([&queue, reader, max_seqs, max_symbols] { produce_chunks(*reader, queue, max_seqs, max_symbols); });

    DeviceGuard g(model->device);
    hipStream_t xs = nullptr;
    Slot slot[2];
    uint64_t decoded = 0;
    auto cleanup = [&] {
        queue.stop();
        if (producer.joinable()) producer.join();
        for (auto& s : slot)
            if (s.done) (void)hipEventDestroy(s.done);
        if (xs) (void)hipStreamDestroy(xs);
    };
    try {
        hip_check(hipStreamCreateWithFlags(&xs, hipStreamNonBlocking), "hipStreamCreate");
        for (auto& s : slot) hip_check(hipEventCreateWithFlags(&s.done, hipEventDisableTiming), "hipEventCreate");
        const uint64_t n = model->host.n;
        // copy slot k's results back on the copy stream and hand them over
        auto deliver = [&](Slot& s) -> bool {
            Batch& b = *s.batch;
            float* sc = s.scores.reserve((size_t)b.nseq * n);
            int64_t* be = s.best.reserve(b.nseq);
            int32_t* pa = want_paths ? s.paths.reserve(b.total) : nullptr;
            hip_check(hipStreamWaitEvent(xs, s.done, 0), "hipStreamWaitEvent");
            b.read_async(xs, sc, be, pa);
            hip_check(hipStreamSynchronize(xs), "results D2H");
            b.check_fault(xs);
            decoded += b.nseq;
            return fn(user, s.chunk.first, b.nseq, s.chunk.offsets.data(), sc, be, pa) == 0;
        };
        int prev = -1;
        bool go = true;
        for (uint64_t k = 0; go; ++k) {
            Slot& s = slot[k & 1];
            Chunk c;
            bool more;
            try {
                more = queue.pop(c);
            } catch (...) {  // a parse error: hand over what was decoded before it, then report
                if (prev >= 0) deliver(slot[prev]);
                throw;
            }
            if (!more) break;
            s.chunk = std::move(c);
            const uint64_t nseq = s.chunk.offsets.size() - 1;
            if (!s.batch)
                s.batch = std::make_unique<Batch>(model, nseq, s.chunk.offsets.data(), s.chunk.symbols.data(), flags);
            else
                s.batch->load(nseq, s.chunk.offsets.data(), nullptr, s.chunk.symbols.data(), model->stream);
            s.batch->run(level, model->stream);
            hip_check(hipEventRecord(s.done, model->stream), "hipEventRecord");
            if (prev >= 0) go = deliver(slot[prev]);  // overlaps this chunk's kernels
            prev = (int)(k & 1);
        }
        if (go && prev >= 0) deliver(slot[prev]);
        hip_check(hipStreamSynchronize(model->stream), "decode_file drain");
    } catch (...) {
        (void)hipStreamSynchronize(model->stream);
        cleanup();
        throw;
    }
    cleanup();
    return decoded;
}

}  // namespace svh
