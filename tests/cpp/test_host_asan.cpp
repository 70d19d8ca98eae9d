// Host code of the engine under AddressSanitizer + UBSan (built by `make tests`, run by
// tests/test_readers_asan.py; no GPU is touched): the canonical host model and every plan builder
// of runtime.cpp (fused, band / chain, pipelined latency and wide, on-chip level 2) over every
// committed .chmm and over generated models with malformed and edge-case inputs, and the parser
// thread's chunk hand-off of the pipelined file decoder (chunker.cpp) over every .ess and the FASTA
// fixture, with a consumer thread, at several chunkings, including files that fail mid-way.  The
// counterpart of the reference running its whole test suite under valgrind memcheck
// (run_tests.sh:4-7, tests/CMakeLists.txt:4-5).
//   usage: test_host_asan <data dir> <fasta fixture> <scratch dir>
#include <cmath>
#include <cstdio>
#include <dirent.h>
#include <fstream>
#include <limits>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "chunker.h"
#include "data_reader.h"
#include "runtime.h"
#include "svh.h"

namespace {

int failures = 0;
int plans_built = 0;

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

struct Coo {  // a model in the C ABI's form (svh_model_create's arrays)
    uint64_t n = 0, S = 0;
    std::vector<uint64_t> scol, src, dst;
    std::vector<float> sval, emis, prob;
};

Coo from_hmm(const HMM& h) {
    Coo c;
    c.n = h.states_num;
    c.S = h.emit_num;
    c.scol.assign(h.start_probabilities_cols.begin(), h.start_probabilities_cols.end());
    c.sval.assign(h.start_probabilities.begin(), h.start_probabilities.end());
    for (const auto& row : h.emissions) c.emis.insert(c.emis.end(), row.begin(), row.end());
    c.src.assign(h.trans_rows.begin(), h.trans_rows.end());
    c.dst.assign(h.trans_cols.begin(), h.trans_cols.end());
    c.prob.assign(h.trans_probs.begin(), h.trans_probs.end());
    return c;
}

svh::HostModel host(const Coo& c) {
    return svh::build_host_model(c.n, c.S, c.scol.size(), c.scol.data(), c.sval.data(), c.emis.data(), c.src.size(),
                                 c.src.data(), c.dst.data(), c.prob.data());
}

int host_error(const Coo& c) {
    try {
        host(c);
    } catch (const svh::Error& e) {
        return e.code;
    }
    return 0;
}

// every plan builder over one model, with the invariants a launch relies on
void plans(const svh::HostModel& hm, const std::string& name) {
    const uint32_t n = hm.n;
    check(hm.rowptr.size() == n + 1 && hm.rowptr[n] == hm.col.size() && hm.col.size() == hm.val.size(), name + ": CSR");
    for (uint32_t c : hm.col) check(c < n, name + ": column in range");
    for (bool uni : {true, false}) {
        const svh::Plan p = svh::make_plan(hm, 0, uni);
        ++plans_built;
        if (p.fused) check(!p.emis_pad.empty() && !p.start_pad.empty(), name + ": fused tables");
    }
    for (bool chain : {true, false}) {
        const svh::BandPlan b = svh::make_band_plan(hm, 0, chain);
        ++plans_built;
        if (b.ok) check(b.lrow.size() > 0, name + ": band rows");
    }
    for (bool wide : {false, true}) {
        const svh::PipePlan p = svh::make_pipe_plan(hm, 0, 0, wide);
        ++plans_built;
        if (!p.ok) continue;
        check(p.P == p.nblk * 64 * p.SM && p.lrow.size() == p.P && p.start.size() == p.P, name + ": pipe sizes");
        check(p.e0.size() == (size_t)hm.S * p.P && p.hc.size() == (size_t)hm.S * 8, name + ": pipe tables");
        std::vector<uint8_t> seen(n, 0);
        for (uint32_t r : p.lrow)
            if (r != 0xFFFFFFFFu) {
                check(r < n && !seen[r], name + ": pipe position map");
                if (r < n) seen[r] = 1;
            }
        check(p.rowF >= 0 && (uint32_t)p.rowF < n && !seen[p.rowF], name + ": pipe feeder row");
        if (!wide) check(p.emax2 >= 0.0f, name + ": level-2 bound");
    }
    const svh::Spec2Plan s = svh::make_spec2_plan(hm);
    ++plans_built;
    if (s.ok) check(s.la.size() == s.lb.size() && s.lb.size() == s.lv.size() && s.hrow.size() >= 1, name + ": spec2 terms");
}

// MSV-shaped (N = 0, M_1..M_L, C = L + 1) or random models with edge cases
Coo generated(std::mt19937& rng, int kind) {
    std::uniform_real_distribution<float> u(0.0f, 8.0f);
    Coo c;
    const uint64_t L = 1 + rng() % 300;
    c.S = 1 + rng() % (kind == 3 ? 40 : 20);
    if (kind <= 1) {  // chain shape, with chain breaks, +inf terms and duplicates
        c.n = L + 2;
        for (uint64_t j = 1; j <= L; ++j) {
            c.src.push_back(0), c.dst.push_back(j), c.prob.push_back(u(rng));
            if (j < L && rng() % 17) c.src.push_back(j), c.dst.push_back(j + 1), c.prob.push_back(rng() % 9 ? u(rng) : INFINITY);
            c.src.push_back(j), c.dst.push_back(0), c.prob.push_back(1.0f);
            c.src.push_back(j), c.dst.push_back(L + 1), c.prob.push_back(2.0f);
            if (kind == 1 && rng() % 5 == 0) c.src.push_back(j), c.dst.push_back(j + 1 <= L ? j + 1 : 1), c.prob.push_back(u(rng));
        }
        c.src.push_back(0), c.dst.push_back(0), c.prob.push_back(0.5f);
        c.src.push_back(L + 1), c.dst.push_back(L + 1), c.prob.push_back(0.25f);
    } else {  // random out-degree, dense rows, self loops
        c.n = kind == 2 ? 1 + rng() % 3 : L;
        const uint64_t deg = 1 + rng() % 6;
        for (uint64_t a = 0; a < c.n; ++a)
            for (uint64_t k = 0; k < deg; ++k) c.src.push_back(a), c.dst.push_back(rng() % c.n), c.prob.push_back(u(rng));
        for (uint64_t b = 0; b < c.n && c.n > 4; ++b) c.src.push_back(b), c.dst.push_back(0), c.prob.push_back(u(rng));
    }
    c.emis.resize(c.S * c.n);
    for (float& e : c.emis) e = rng() % 13 ? u(rng) : INFINITY;
    c.scol = {0, rng() % c.n, 0};
    c.sval = {u(rng), u(rng), 99.0f};  // a duplicate start column: the first wins
    return c;
}

// the parser thread's hand-off with a consumer thread: the sequences, in file order
std::vector<std::vector<uint8_t>> chunked(const std::string& path, int fmt, uint64_t ms, uint64_t mx, size_t cap,
                                          int* err) {
    svh::SeqReader reader(path, fmt);
    svh::ChunkQueue queue(cap);
    std::thread producer([&] { svh::produce_chunks(reader, queue, ms, mx); });
    std::vector<std::vector<uint8_t>> out;
    uint64_t next_first = 0;
    *err = 0;
    try {
        svh::Chunk c;
        while (queue.pop(c)) {
            check(c.first == next_first, path + ": chunk order");
            check(!c.offsets.empty() && c.offsets.back() == c.symbols.size(), path + ": chunk offsets");
            for (size_t q = 0; q + 1 < c.offsets.size(); ++q)
                out.emplace_back(c.symbols.begin() + c.offsets[q], c.symbols.begin() + c.offsets[q + 1]);
            next_first += c.offsets.size() - 1;
        }
    } catch (const svh::Error& e) {
        *err = e.code;
    }
    queue.stop();
    producer.join();
    return out;
}

void write(const std::string& path, const std::string& text) { std::ofstream(path) << text; }

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s <data dir> <fasta fixture> <scratch dir>\n", argv[0]);
        return 2;
    }
    const std::string data = argv[1], fasta = argv[2], tmp = argv[3];

    // every committed model: host CSR and every plan
    const auto models = list(data + "/chmm_files", ".chmm");
    check(models.size() >= 20, "expected the reference's .chmm files");
    for (const auto& f : models) {
        const HMM h = read_HMM(f);
        plans(host(from_hmm(h)), f);
    }
    // generated models (chain shapes with breaks / +inf / duplicates, tiny and random ones)
    std::mt19937 rng(20261018);
    for (int i = 0; i < 240; ++i) {
        const Coo c = generated(rng, i % 4);
        plans(host(c), "generated #" + std::to_string(i));
    }
    // malformed inputs: the documented errors, never a crash or an out-of-bounds access
    {
        std::mt19937 r2(7);
        const Coo base = generated(r2, 0);
        Coo c = base;
        c.prob[0] = std::numeric_limits<float>::quiet_NaN();
        check(host_error(c) == SVH_E_INVALID, "NaN transition score");
        c = base;
        c.emis[3] = -INFINITY;
        check(host_error(c) == SVH_E_INVALID, "-inf emission score");
        c = base;
        c.dst[1] = c.n;
        check(host_error(c) == SVH_E_RANGE, "transition index out of range");
        c = base;
        c.scol[1] = c.n + 5;
        check(host_error(c) == SVH_E_RANGE, "start index out of range");
        c = base;
        c.S = 257;
        c.emis.resize(c.S * c.n, 1.0f);
        check(host_error(c) == SVH_E_UNSUPPORTED, "more than 256 symbols");
        c = base;
        c.n = 0;
        check(host_error(c) == SVH_E_INVALID, "no states");
        c = base;
        c.src.clear(), c.dst.clear(), c.prob.clear();
        plans(host(c), "no transitions");
        c = base;
        c.scol.clear(), c.sval.clear();
        plans(host(c), "no start states");
    }

    // the file decoder's chunk hand-off over every .ess and the FASTA fixture
    std::vector<std::pair<std::string, int>> files;
    for (const auto& f : list(data + "/ess_files", ".ess")) files.push_back({f, SVH_FORMAT_ESS});
    files.push_back({fasta, SVH_FORMAT_FASTA});
    for (const auto& [path, fmt] : files) {
        int err = 0;
        const auto whole = chunked(path, fmt, 1u << 30, 1ull << 40, 2, &err);
        check(err == 0 && !whole.empty(), path + ": whole file");
        for (auto [ms, mx, cap] : {std::tuple<uint64_t, uint64_t, size_t>{1, 1, 1}, {3, 100, 2}, {7, 5000, 1}, {64, 1u << 20, 4}}) {
            const auto got = chunked(path, fmt, ms, mx, cap, &err);
            check(err == 0 && got == whole, path + ": chunked " + std::to_string(ms) + "/" + std::to_string(mx));
        }
    }
    // a file that fails mid-way: the chunks before the error arrive, then the error
    write(tmp + "/bad.fasta", ">a\nACDE\n>b\nAC*D\n");
    {
        int err = 0;
        const auto got = chunked(tmp + "/bad.fasta", SVH_FORMAT_FASTA, 1, 1u << 20, 2, &err);
        check(err == SVH_E_RANGE && got.size() == 1, "FASTA error after one sequence");
    }
    write(tmp + "/bad.ess", "3\n0 4\n1 2\n");
    {
        int err = 0;
        chunked(tmp + "/bad.ess", SVH_FORMAT_ESS, 1, 1u << 20, 1, &err);
        check(err != 0, "truncated .ess");
    }
    // the consumer stopping early (a callback that returns non-zero): the producer unblocks
    for (const auto& [path, fmt] : files) {
        svh::SeqReader reader(path, fmt);
        svh::ChunkQueue queue(1);
        std::thread producer([&] { svh::produce_chunks(reader, queue, 1, 1u << 20); });
        svh::Chunk c;
        check(queue.pop(c), path + ": first chunk");
        queue.stop();
        producer.join();
    }
    std::printf("host asan: %zu models, %d plans built, %zu files chunked, %d failures\n", models.size(), plans_built,
                files.size(), failures);
    return failures ? 1 : 0;
}
