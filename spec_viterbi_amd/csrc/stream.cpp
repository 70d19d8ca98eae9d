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

#include "svh.h"

namespace svh {

namespace {

// ess_files/fasta_to_ess.py:3-7 (amino2num), X -> 0 ("X can be transformed into any aminoacid")
struct FastaTable {
    int8_t map[256];
    FastaTable() {
        std::memset(map, -1, sizeof(map));
        const char* order = "ACDEFGHIKLMNPQRSTVWY";
        for (int k = 0; k < 20; ++k) map[(unsigned char)order[k]] = (int8_t)k;
        map[(unsigned char)'X'] = 0;
    }
};
const FastaTable kFasta;

bool is_space(int c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }

bool ends_with(const std::string& s, const char* suf) {
    const size_t n = std::strlen(suf);
    if (s.size() < n) return false;
    for (size_t i = 0; i < n; ++i)
        if (std::tolower((unsigned char)s[s.size() - n + i]) != suf[i]) return false;
    return true;
}

}  // namespace

int fasta_symbol(unsigned char c) { return kFasta.map[c]; }

SeqReader::SeqReader(const std::string& path, int format) : path_(path), in_(path, std::ios::binary) {
    if (!in_) throw Error(SVH_E_IO, "cannot open " + path);
    buf_.resize(1 << 20);
    if (format == SVH_FORMAT_FASTA) {
        fasta_ = true;
    } else if (format == SVH_FORMAT_ESS) {
        fasta_ = false;
    } else if (format == SVH_FORMAT_AUTO) {
        if (ends_with(path, ".fasta") || ends_with(path, ".fa") || ends_with(path, ".faa") ||
            ends_with(path, ".fas")) {
            fasta_ = true;
        } else if (ends_with(path, ".ess")) {
            fasta_ = false;
        } else {  // content: FASTA starts with '>' (after whitespace)
            int c;
            while ((c = get()) != EOF && is_space(c)) {
            }
            fasta_ = c == '>';
            pos_ = 0;  // rewind the buffer (the first refill is still in it)
        }
    } else {
        throw Error(SVH_E_INVALID, "unknown sequence file format " + std::to_string(format));
    }
}

int SeqReader::get() {
    if (pos_ == end_) {
        in_.read(buf_.data(), (std::streamsize)buf_.size());
        end_ = (size_t)in_.gcount();
        pos_ = 0;
        if (end_ == 0) return EOF;
    }
    return (unsigned char)buf_[pos_++];
}

bool SeqReader::next_u64(uint64_t& x) {
    int c;
    while ((c = get()) != EOF && is_space(c)) {
    }
    if (c == EOF) return false;
    if (c < '0' || c > '9') throw Error(SVH_E_IO, path_ + ": expected an unsigned integer in the .ess file");
    uint64_t v = 0;
    while (c != EOF && c >= '0' && c <= '9') {
        if (v > (UINT64_MAX - 9) / 10) throw Error(SVH_E_RANGE, path_ + ": integer out of range");
        v = v * 10 + (uint64_t)(c - '0');
        c = get();
    }
    if (c != EOF && !is_space(c)) throw Error(SVH_E_IO, path_ + ": malformed integer in the .ess file");
    x = v;
    return true;
}

bool SeqReader::next_line(std::string& line) {
    line.clear();
    int c = get();
    if (c == EOF) return false;
    while (c != EOF && c != '\n') {
        line.push_back((char)c);
        c = get();
    }
    return true;
}

bool SeqReader::read_one_ess(std::vector<uint8_t>& seq) {
    if (!ess_started_) {
        ess_started_ = true;
        if (!next_u64(ess_count_)) ess_count_ = 0;  // empty file: no sequences
    }
    if (ess_index_ == ess_count_) return false;
    uint64_t idx = 0, len = 0;
    if (!next_u64(idx) || !next_u64(len))
        throw Error(SVH_E_IO, path_ + ": truncated .ess file (sequence " + std::to_string(ess_index_) + ")");
    if (idx != ess_index_)  // data_reader.cpp:112-119
        throw Error(SVH_E_IO, path_ + ": expected sequence number " + std::to_string(ess_index_) + ", but read " +
                                  std::to_string(idx));
    seq.resize(len);
    for (uint64_t k = 0; k < len; ++k) {
        uint64_t x;
        if (!next_u64(x)) throw Error(SVH_E_IO, path_ + ": truncated sequence " + std::to_string(idx));
        if (x > 255) throw Error(SVH_E_RANGE, path_ + ": symbol " + std::to_string(x) + " does not fit uint8");
        seq[k] = (uint8_t)x;
    }
    ++ess_index_;
    return true;
}

bool SeqReader::read_one_fasta(std::vector<uint8_t>& seq) {
    seq.clear();
    std::string line;
    while (next_line(line)) {
        ++line_no_;
        size_t a = 0, b = line.size();
        while (a < b && is_space((unsigned char)line[a])) ++a;
        while (b > a && is_space((unsigned char)line[b - 1])) --b;
        if (a == b)  // fasta_to_ess.py:27 reads line[0]
            throw Error(SVH_E_IO, path_ + ":" + std::to_string(line_no_) + ": empty line in FASTA input");
        if (line[a] == '>') {  // header: ends the current sequence if it has residues
            if (!seq.empty()) return true;
            continue;
        }
        for (size_t k = a; k < b; ++k) {
            const int sym = kFasta.map[(unsigned char)line[k]];
            if (sym < 0)
                throw Error(SVH_E_RANGE, path_ + ":" + std::to_string(line_no_) + ": residue '" +
                                             std::string(1, line[k]) + "' is not in fasta_to_ess.py's table");
            seq.push_back((uint8_t)sym);
        }
    }
    return !seq.empty();
}

bool SeqReader::read_one(std::vector<uint8_t>& seq) { return fasta_ ? read_one_fasta(seq) : read_one_ess(seq); }

bool SeqReader::next(uint64_t max_seqs, uint64_t max_symbols, std::vector<uint64_t>& offsets,
                     std::vector<uint8_t>& symbols) {
    if (max_seqs == 0) throw Error(SVH_E_INVALID, "max_seqs must be > 0");
    offsets.assign(1, 0);
    symbols.clear();
    while (offsets.size() - 1 < max_seqs) {
        if (!has_pending_) {
            if (!read_one(pending_)) break;
            has_pending_ = true;
        }
        if (offsets.size() > 1 && symbols.size() + pending_.size() > max_symbols) break;  // next chunk
        symbols.insert(symbols.end(), pending_.begin(), pending_.end());
        offsets.push_back(symbols.size());
        has_pending_ = false;
    }
    return offsets.size() > 1;
}

// ---------------------------------------------------------------------------------------------
// Pipelined decoder
// ---------------------------------------------------------------------------------------------
namespace {

struct Chunk {
    std::vector<uint64_t> offsets;
    std::vector<uint8_t> symbols;
    uint64_t first = 0;
};

// Bounded hand-off from the parser thread; an exception or the end closes it.
class ChunkQueue {
  public:
    explicit ChunkQueue(size_t cap) : cap_(cap) {}
    bool push(Chunk&& c) {  // false: the consumer stopped
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return q_.size() < cap_ || stop_; });
        if (stop_) return false;
        q_.push_back(std::move(c));
        cv_.notify_all();
        return true;
    }
    void close(std::exception_ptr e) {
        std::lock_guard<std::mutex> l(mu_);
        closed_ = true;
        err_ = e;
        cv_.notify_all();
    }
    bool pop(Chunk& c) {  // false at the end (rethrows the producer's error)
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
    void stop() {
        std::lock_guard<std::mutex> l(mu_);
        stop_ = true;
        cv_.notify_all();
    }

  private:
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Chunk> q_;
    size_t cap_;
    bool closed_ = false, stop_ = false;
    std::exception_ptr err_;
};

template <class T>
struct Pinned {
    T* p = nullptr;
    size_t n = 0;
    ~Pinned() {
        if (p) (void)hipHostFree(p);
    }
    T* reserve(size_t count) {
        if (count > n) {
            if (p) (void)hipHostFree(p);
            p = nullptr;
            hip_check(hipHostMalloc((void**)&p, std::max<size_t>(count, 1) * sizeof(T), hipHostMallocDefault),
                      "hipHostMalloc");
            n = count;
        }
        return p;
    }
};

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
    std::thread producer([&queue, reader, max_seqs, max_symbols] {
        try {
            uint64_t first = 0;
            while (true) {
                Chunk c;
                if (!reader->next(max_seqs, max_symbols, c.offsets, c.symbols)) break;
                c.first = first;
                first += c.offsets.size() - 1;
                if (!queue.push(std::move(c))) break;
            }
            queue.close(nullptr);
        } catch (...) {
            queue.close(std::current_exception());
        }
    });

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
            model->check_fault();
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
