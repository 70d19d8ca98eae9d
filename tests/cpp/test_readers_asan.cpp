// Host readers under AddressSanitizer + UBSan (built by `make tests`, run by
// tests/test_readers_asan.py): every committed .chmm / .ess through read_HMM / read_emit_seq,
// every .ess and FASTA through the incremental SeqReader at several chunkings, and malformed
// inputs that must fail with the documented error codes -- never crash or touch memory out of
// bounds.  The counterpart of the reference's valgrind memcheck run (run_tests.sh:4-7).
//   usage: test_readers_asan <data dir> <fasta fixture> <scratch dir>
#include <cstdio>
#include <dirent.h>
#include <fstream>
#include <string>
#include <vector>

#include "data_reader.h"
#include "seqreader.h"
#include "svh.h"

namespace {

int failures = 0;

void check(bool ok, const std::string& what) {
    if (!ok) {
        std::fprintf(stderr, "FAIL: %s\n", what.c_str());
        ++failures;
    }
}

std::vector<std::string> list(const std::string& dir, const std::string& ext) {
    std::vector<std::string> out;
    if (DIR* d = opendir(dir.c_str())) {
        while (dirent* e = readdir(d)) {
            const std::string n = e->d_name;
            if (n.size() > ext.size() && n.compare(n.size() - ext.size(), ext.size(), ext) == 0) out.push_back(dir + "/" + n);
        }
        closedir(d);
    }
    return out;
}

// all sequences of a file through SeqReader in chunks of (max_seqs, max_symbols)
std::vector<std::vector<uint8_t>> stream_all(const std::string& path, int fmt, uint64_t ms, uint64_t mx) {
    svh::SeqReader r(path, fmt);
    std::vector<uint64_t> offs;
    std::vector<uint8_t> syms;
    std::vector<std::vector<uint8_t>> out;
    while (r.next(ms, mx, offs, syms))
        for (size_t q = 0; q + 1 < offs.size(); ++q) out.emplace_back(syms.begin() + offs[q], syms.begin() + offs[q + 1]);
    return out;
}

int error_code(const std::string& path, int fmt) {
    try {
        stream_all(path, fmt, 3, 100);
    } catch (const svh::Error& e) {
        return e.code;
    }
    return 0;
}

void write(const std::string& path, const std::string& text) { std::ofstream(path) << text; }

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    const std::string data = argv[1], fasta = argv[2], tmp = argv[3];
    const auto chmms = list(data + "/chmm_files", ".chmm");
    const auto esses = list(data + "/ess_files", ".ess");
    check(!chmms.empty() && !esses.empty(), "data files found");
    for (const auto& f : chmms) {
        const HMM h = read_HMM(f);
        check(h.states_num > 0 && h.emissions.size() == h.emit_num, "read_HMM " + f);
    }
    for (const auto& f : esses) {
        const auto ref = read_emit_seq(f);
        check(!ref.empty(), "read_emit_seq " + f);
        for (uint64_t ms : {1ull, 7ull, 4096ull}) {
            const auto got = stream_all(f, SVH_FORMAT_ESS, ms, 5000);
            bool same = got.size() == ref.size();
            for (size_t q = 0; same && q < got.size(); ++q) {
                same = got[q].size() == ref[q].size();
                for (size_t i = 0; same && i < got[q].size(); ++i) same = got[q][i] == ref[q][i];
            }
            check(same, "SeqReader .ess " + f);
        }
    }
    check(stream_all(fasta, SVH_FORMAT_AUTO, 4, 3000).size() == 16, "SeqReader FASTA fixture");
    // malformed inputs: documented errors, no crash
    write(tmp + "/empty_line.fasta", ">a\nAC\n\nDE\n");
    check(error_code(tmp + "/empty_line.fasta", SVH_FORMAT_FASTA) == SVH_E_IO, "FASTA empty line");
    write(tmp + "/bad_residue.fasta", ">a\nACDZ\n");
    check(error_code(tmp + "/bad_residue.fasta", SVH_FORMAT_FASTA) == SVH_E_RANGE, "FASTA residue");
    write(tmp + "/bad_index.ess", "2\n0 1\n3\n7 1\n3\n");
    check(error_code(tmp + "/bad_index.ess", SVH_FORMAT_ESS) == SVH_E_IO, ".ess index");
    write(tmp + "/truncated.ess", "3\n0 4\n1 2\n");
    check(error_code(tmp + "/truncated.ess", SVH_FORMAT_ESS) == SVH_E_IO, ".ess truncated");
    write(tmp + "/garbage.ess", "2\n0 x\n");
    check(error_code(tmp + "/garbage.ess", SVH_FORMAT_ESS) == SVH_E_IO, ".ess garbage");
    write(tmp + "/huge.ess", "1\n0 1\n99999999999999999999999\n");
    check(error_code(tmp + "/huge.ess", SVH_FORMAT_ESS) == SVH_E_RANGE, ".ess overflow");
    write(tmp + "/empty.ess", "");
    check(error_code(tmp + "/empty.ess", SVH_FORMAT_ESS) == 0, ".ess empty file");
    // the reference readers on malformed input: empty results, no crash
    check(read_emit_seq(tmp + "/bad_index.ess").empty(), "read_emit_seq bad index");
    write(tmp + "/trunc.chmm", "3\n2\n0 0.5\n");
    (void)read_HMM(tmp + "/trunc.chmm");
    (void)read_HMM(tmp + "/missing.chmm");
    std::printf("%s (%zu chmm, %zu ess)\n", failures ? "FAILED" : "ok", chmms.size(), esses.size());
    return failures ? 1 : 0;
}
