// The reference benchmark harness's call pattern over the drop-in classes HIP_impl / HIP_spec_impl.
//
// Reference: benchmark/bench_Viterbi.h:51-59 (a serial loop of single-sequence run_Viterbi calls
// over an .ess file, timed as a whole, median of helper::TIMES_TO_RUN = 10 runs,
// benchmark_helper.h:38-60), benchmark/bench_Viterbi_spec.h:69-80 (spec_with timed apart, then the
// same loop over run_Viterbi_spec, levels 1..2) and main.cpp:5-6 (the four datasets).  Every
// .chmm of the model folder is run, in ascending state count.
//
// Besides the reference's milliseconds (here with microsecond resolution) each cell reports the
// device time of the same single-sequence passes (one svh batch per sequence, HIP events around
// the launches) and the per-call host overhead of the drop-in path:
//     overhead_us = (loop time - sum of the per-sequence device times) / calls.
// One JSON object per line on stdout.
//
// usage: bench_harness [--data DIR] [--datasets a,b,..] [--models x.chmm,..] [--levels 0,1,2]
//                      [--reps N] [--min-states N] [--max-states N]
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dirent.h>
#include <functional>
#include <string>
#include <vector>

#include "HIP_impl.h"
#include "HIP_spec_impl.h"
#include "data_reader.h"
#include "svh.h"

namespace {

using Clock = std::chrono::steady_clock;

std::vector<std::string> split(const std::string& s) {
    std::vector<std::string> out;
    size_t a = 0;
    while (a <= s.size()) {
        const size_t b = s.find(',', a);
        const std::string t = s.substr(a, b == std::string::npos ? std::string::npos : b - a);
        if (!t.empty()) out.push_back(t);
        if (b == std::string::npos) break;
        a = b + 1;
    }
    return out;
}

double time_ms(const std::function<void()>& f) {
    const auto t0 = Clock::now();
    f();
    return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

// median of `reps` runs (benchmark_helper.h:38-60: sorted, middle element)
double median_ms(const std::function<void()>& f, int reps) {
    std::vector<double> t;
    for (int i = 0; i < reps; ++i) t.push_back(time_ms(f));
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

void check(int rc, const char* what) {
    if (rc != SVH_OK) {
        std::fprintf(stderr, "bench_harness: %s failed: %s\n", what, svh_last_error());
        std::exit(2);
    }
}

svh_model_t c_model(const HMM& hmm) {
    const uint64_t n = hmm.states_num, S = hmm.emit_num;
    std::vector<float> emis(S * n);
    for (uint64_t o = 0; o < S; ++o) std::memcpy(emis.data() + o * n, hmm.emissions[o].data(), n * 4);
    svh_model_t m = nullptr;
    check(svh_model_create(n, S, hmm.start_probabilities.size(),
                           reinterpret_cast<const uint64_t*>(hmm.start_probabilities_cols.data()),
                           hmm.start_probabilities.data(), emis.data(), hmm.trans_probs.size(),
                           reinterpret_cast<const uint64_t*>(hmm.trans_rows.data()),
                           reinterpret_cast<const uint64_t*>(hmm.trans_cols.data()), hmm.trans_probs.data(),
                           nullptr, &m),
          "svh_model_create");
    return m;
}

// Device time of the single-sequence passes the loop makes: one batch per sequence (created
// outside the timed part), each launch bracketed by the batch's HIP events; median of 3 sums.
double device_ms(svh_model_t m, const HMM::Emit_seq_vec_t& seqs, uint32_t level) {
    std::vector<svh_batch_t> bs;
    for (const auto& s : seqs) {
        const uint64_t off[2] = {0, s.size()};
        svh_batch_t b = nullptr;
        check(svh_batch_create(m, 1, off, reinterpret_cast<const uint64_t*>(s.data()), 0, &b), "svh_batch_create");
        bs.push_back(b);
    }
    std::vector<double> sums;
    for (int r = 0; r < 4; ++r) {
        double sum = 0;
        for (svh_batch_t b : bs) {
            check(svh_batch_run(b, level, nullptr), "svh_batch_run");
            float ms = 0;
            check(svh_batch_elapsed_ms(b, &ms), "svh_batch_elapsed_ms");
            sum += ms;
        }
        if (r > 0) sums.push_back(sum);  // the first round warms up
    }
    for (svh_batch_t b : bs) svh_batch_destroy(b);
    std::sort(sums.begin(), sums.end());
    return sums[sums.size() / 2];
}

struct Chmm {
    std::string name, path;
    HMM hmm;
};

}  // namespace

int main(int argc, char** argv) {
    std::string data = "data";
    std::vector<std::string> datasets = {"emit_3_3500_20", "emit_3_7000_20", "covid-19", "emit_50_3500_20"};
    std::vector<std::string> models;
    std::vector<int> levels = {0, 1, 2};
    int reps = 10;
    uint64_t min_states = 0, max_states = ~0ull;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i], v = argv[i + 1];
        if (k == "--data") data = v;
        else if (k == "--datasets") datasets = split(v);
        else if (k == "--models") models = split(v);
        else if (k == "--levels") {
            levels.clear();
            for (const auto& x : split(v)) levels.push_back(std::atoi(x.c_str()));
        } else if (k == "--reps") reps = std::max(1, std::atoi(v.c_str()));
        else if (k == "--min-states") min_states = std::strtoull(v.c_str(), nullptr, 10);
        else if (k == "--max-states") max_states = std::strtoull(v.c_str(), nullptr, 10);
        else {
            std::fprintf(stderr, "bench_harness: unknown option %s\n", k.c_str());
            return 2;
        }
    }
    // the model folder (bench_Viterbi.h:38-47: every .chmm of chmm_files)
    std::vector<Chmm> chmms;
    const std::string folder = data + "/chmm_files";
    if (DIR* d = opendir(folder.c_str())) {
        while (dirent* e = readdir(d)) {
            const std::string f = e->d_name;
            if (f.size() < 6 || f.substr(f.size() - 5) != ".chmm") continue;
            if (!models.empty() && std::find(models.begin(), models.end(), f) == models.end()) continue;
            chmms.push_back({f, folder + "/" + f, HMM()});
        }
        closedir(d);
    }
    for (auto& c : chmms) c.hmm = read_HMM(c.path);
    chmms.erase(std::remove_if(chmms.begin(), chmms.end(),
                               [&](const Chmm& c) {
                                   return c.hmm.states_num < min_states || c.hmm.states_num > max_states;
                               }),
                chmms.end());
    std::sort(chmms.begin(), chmms.end(), [](const Chmm& a, const Chmm& b) { return a.hmm.states_num < b.hmm.states_num; });
    if (chmms.empty()) {
        std::fprintf(stderr, "bench_harness: no models under %s\n", folder.c_str());
        return 2;
    }

    for (const auto& ds : datasets) {
        const auto seqs = read_emit_seq(data + "/ess_files/" + ds + ".ess");
        uint64_t obs = 0;
        for (const auto& s : seqs) obs += s.size();
        for (const auto& c : chmms) {
            const HMM& hmm = c.hmm;
            for (int level : levels) {
                double prep = 0, loop = 0, first = 0;
                if (level == 0) {
                    // bench_Viterbi.h:51-59 (the first loop also builds and caches the device model)
                    HIP_impl impl;
                    auto fn = [&] {
                        for (const auto& s : seqs) static_cast<void>(impl.run_Viterbi(hmm, s));
                    };
                    first = time_ms(fn);
                    loop = median_ms(fn, reps);
                } else {
                    // bench_Viterbi_spec.h:69-80
                    HIP_spec_impl impl(static_cast<size_t>(level));
                    prep = median_ms([&] { impl.spec_with(hmm); }, reps);
                    auto fn = [&] {
                        for (const auto& s : seqs) static_cast<void>(impl.run_Viterbi_spec(s));
                    };
                    first = time_ms(fn);
                    loop = median_ms(fn, reps);
                }
                svh_model_t m = c_model(hmm);
                if (level >= 2) check(svh_spec_build(m, (uint32_t)level, nullptr), "svh_spec_build");
                const double dev = device_ms(m, seqs, (uint32_t)level);
                svh_model_info info{};
                check(svh_model_get_info(m, &info), "svh_model_get_info");
                svh_model_destroy(m);
                const double calls = (double)seqs.size();
                std::printf(
                    "{\"dataset\": \"%s\", \"model\": \"%s\", \"states\": %llu, \"impl\": \"%s\", \"level\": %d, "
                    "\"calls\": %zu, \"observations\": %llu, \"reps\": %d, \"median_ms\": %.4f, \"first_ms\": %.4f, "
                    "\"prep_ms\": %.4f, \"device_ms\": %.4f, \"per_call_us\": %.2f, \"device_per_call_us\": %.2f, "
                    "\"overhead_us\": %.2f, \"M_state_updates_per_s\": %.1f, \"kernel\": %d}\n",
                    ds.c_str(), c.name.c_str(), (unsigned long long)hmm.states_num,
                    level == 0 ? "HIP_impl" : "HIP_spec_impl", level, seqs.size(), (unsigned long long)obs, reps, loop,
                    first, prep, dev, loop * 1e3 / calls, dev * 1e3 / calls, (loop - dev) * 1e3 / calls,
                    (double)hmm.states_num * (double)obs / (loop * 1e-3) / 1e6, info.kernel);
                std::fflush(stdout);
            }
        }
    }
    return 0;
}
