// Host side of the pipelined file decoder (chunker.h).
#include "chunker.h"

namespace svh {

bool ChunkQueue::push(Chunk&& c) {
    std::unique_lock<std::mutex> l(mu_);
    cv_.wait(l, [&] { return q_.size() < cap_ || stop_; });
    if (stop_) return false;
    q_.push_back(std::move(c));
    cv_.notify_all();
    return true;
}

void ChunkQueue::close(std::exception_ptr e) {
    std::lock_guard<std::mutex> l(mu_);
    closed_ = true;
    err_ = e;
    cv_.notify_all();
}

bool ChunkQueue::pop(Chunk& c) {
    std::unique_lock<std::mutex> l(mu_);
    cv_.wait(l, [&] { return !q_.empty() || closed_; });
    if (!q_.empty()) {
        c = std::move(q_.front());
        q_.pop_front();
        cv_.notify_all();
        return true;
    }
    if (err_) std::rethrow_exception(err_);
    return false;
}

void ChunkQueue::stop() {
    std::lock_guard<std::mutex> l(mu_);
    stop_ = true;
    cv_.notify_all();
}

void produce_chunks(SeqReader& reader, ChunkQueue& queue, uint64_t max_seqs, uint64_t max_symbols) {
    try {
        uint64_t first = 0;
        while (true) {
            Chunk c;
            if (!reader.next(max_seqs, max_symbols, c.offsets, c.symbols)) break;
            c.first = first;
            first += c.offsets.size() - 1;
            if (!queue.push(std::move(c))) break;
        }
        queue.close(nullptr);
    } catch (...) {
        queue.close(std::current_exception());
    }
}

}  // namespace svh
