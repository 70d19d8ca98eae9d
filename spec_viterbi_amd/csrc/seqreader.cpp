// Incremental .ess / FASTA reader (seqreader.h).
#include "seqreader.h"

#include <cctype>
#include <cstdio>
#include <cstring>

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

}  // namespace svh
