// Host runtime: model canonicalisation, fused-kernel planning, HBM residency, batches and the
// _spec product pipeline.  See DESIGN.md for the layouts.
#include "runtime.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <numeric>

namespace svh {

namespace {

constexpr float kInfH = std::numeric_limits<float>::infinity();

uint32_t round_up(uint32_t x, uint32_t m) { return (x + m - 1) / m * m; }

uint32_t float_bits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

}  // namespace

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) {
        throw Error(e == hipErrorOutOfMemory ? SVH_E_NOMEM : SVH_E_HIP,
                    std::string(what) + ": " + hipGetErrorString(e));
    }
}

DeviceGuard::DeviceGuard(int dev) {
    hip_check(hipGetDevice(&prev), "hipGetDevice");
    if (dev != prev) hip_check(hipSetDevice(dev), "hipSetDevice");
}
DeviceGuard::~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
}

DeviceBuffer& DeviceBuffer::operator=(DeviceBuffer&& o) noexcept {
    if (this != &o) {
        if (ptr) (void)hipFree(ptr);
        ptr = o.ptr;
        bytes = o.bytes;
        o.ptr = nullptr;
        o.bytes = 0;
    }
    return *this;
}
DeviceBuffer::~DeviceBuffer() {
    if (ptr) (void)hipFree(ptr);
}
void DeviceBuffer::alloc(size_t nbytes) {
    if (ptr) {
        (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
    if (nbytes == 0) nbytes = 16;
    hip_check(hipMalloc(&ptr, nbytes), "hipMalloc");
    bytes = nbytes;
}
void DeviceBuffer::reserve(size_t nbytes) {
    if (!ptr || nbytes > bytes) alloc(nbytes);
}
void DeviceBuffer::upload_async(const void* src, size_t nbytes, hipStream_t s) {
    reserve(nbytes);
    if (nbytes) hip_check(hipMemcpyAsync(ptr, src, nbytes, hipMemcpyHostToDevice, s), "hipMemcpyAsync H2D");
}
void DeviceBuffer::upload(const void* src, size_t nbytes, hipStream_t s) {
    alloc(nbytes);
    if (nbytes) hip_check(hipMemcpyAsync(ptr, src, nbytes, hipMemcpyHostToDevice, s), "hipMemcpyAsync H2D");
}

// ------------------------------------------------------------------------------------------
// Canonical host model.  Reference semantics (GraphBLAS_impl.cpp:9-45): the start column and
// T^T are built with GrB_Matrix_build(..., GrB_FIRST_FP32): duplicates keep the first tuple.
// ------------------------------------------------------------------------------------------
HostModel build_host_model(uint64_t n, uint64_t S, uint64_t nstart, const uint64_t* start_cols,
                           const float* start_vals, const float* emissions, uint64_t ntrans,
                           const uint64_t* src, const uint64_t* dst, const float* prob) {
    if (n == 0 || S == 0) throw Error(SVH_E_INVALID, "model needs states_num > 0 and emit_num > 0");
    if (n >= (1ull << 31)) throw Error(SVH_E_UNSUPPORTED, "states_num must be < 2^31");
    if (S > 256) throw Error(SVH_E_UNSUPPORTED, "emit_num must be <= 256 (uint8 symbols in HBM)");
    if (ntrans >= (1ull << 32)) throw Error(SVH_E_UNSUPPORTED, "trans_num must be < 2^32");
    if (!emissions || (nstart && (!start_cols || !start_vals)) || (ntrans && (!src || !dst || !prob)))
        throw Error(SVH_E_INVALID, "null model array");
    // Scores are -log2 p (HMM::to_modified_prob): finite or +inf.  A NaN or -inf (p = +inf)
    // would let fl(-inf + +inf) = NaN into the min, whose result the kernels (built with
    // -fno-honor-nans, so fminf is one v_min_f32) and GraphBLAS's GB_FMIN need not agree on.
    // The reference's reader never produces either for p in [0, 1]; reject them here.
    auto bad = [](float x) { return std::isnan(x) || x == -std::numeric_limits<float>::infinity(); };
    for (uint64_t i = 0; i < nstart; ++i)
        if (bad(start_vals[i])) throw Error(SVH_E_INVALID, "start score is NaN or -inf");
    for (uint64_t i = 0; i < S * n; ++i)
        if (bad(emissions[i])) throw Error(SVH_E_INVALID, "emission score is NaN or -inf");
    for (uint64_t e = 0; e < ntrans; ++e)
        if (bad(prob[e])) throw Error(SVH_E_INVALID, "transition score is NaN or -inf");
    HostModel h;
    h.n = (uint32_t)n;
    h.S = (uint32_t)S;
    h.start.assign(n, kInfH);
    std::vector<uint8_t> seen(n, 0);
    for (uint64_t i = 0; i < nstart; ++i) {
        const uint64_t c = start_cols[i];
        if (c >= n) throw Error(SVH_E_RANGE, "start state index out of range");
        if (!seen[c]) {
            h.start[c] = start_vals[i];
            seen[c] = 1;
        }
    }
    h.emis.assign(emissions, emissions + S * n);

    struct Tri { uint32_t dst, src, order; };
    std::vector<Tri> t(ntrans);
    for (uint64_t e = 0; e < ntrans; ++e) {
        if (src[e] >= n || dst[e] >= n) throw Error(SVH_E_RANGE, "transition state index out of range");
        t[e] = {(uint32_t)dst[e], (uint32_t)src[e], (uint32_t)e};
    }
    std::sort(t.begin(), t.end(), [](const Tri& a, const Tri& b) {
        if (a.dst != b.dst) return a.dst < b.dst;
        if (a.src != b.src) return a.src < b.src;
        return a.order < b.order;
    });
    h.rowptr.assign(n + 1, 0);
    h.col.reserve(ntrans);
    h.val.reserve(ntrans);
    for (uint64_t e = 0; e < ntrans; ++e) {
        if (e > 0 && t[e].dst == t[e - 1].dst && t[e].src == t[e - 1].src) continue;  // FIRST
        h.col.push_back(t[e].src);
        h.val.push_back(prob[t[e].order]);
        h.rowptr[t[e].dst + 1]++;
    }
    for (uint32_t j = 0; j < h.n; ++j) h.rowptr[j + 1] += h.rowptr[j];
    return h;
}

// ------------------------------------------------------------------------------------------
// Fused-kernel planning.
// ------------------------------------------------------------------------------------------
namespace {

struct HeavyAnalysis {
    bool ok = false;
    std::vector<uint32_t> heavy;  // row ids
};

// Uniform-heavy analysis: every heavy row = {dominant weight w_h over a non-heavy source set U
// shared by all heavy rows} + <= XM exception terms.
bool analyse_uniform(const HostModel& hm, const std::vector<int>& hidx,
                     const std::vector<uint32_t>& heavy, uint32_t XM, float* hw,
                     std::vector<std::pair<uint32_t, float>>* exc, std::vector<uint32_t>* U) {
    if (heavy.empty()) return false;
    std::vector<uint32_t> first_u;
    for (size_t h = 0; h < heavy.size(); ++h) {
        const uint32_t j = heavy[h];
        std::map<uint32_t, uint32_t> count;
        for (uint32_t p = hm.rowptr[j]; p < hm.rowptr[j + 1]; ++p)
            if (hidx[hm.col[p]] < 0) count[float_bits(hm.val[p])]++;
        uint32_t best_bits = float_bits(kInfH), best_cnt = 0;
        for (const auto& [bits, c] : count)
            if (c > best_cnt) {
                best_cnt = c;
                best_bits = bits;
            }
        std::memcpy(&hw[h], &best_bits, 4);
        std::vector<uint32_t> u;
        exc[h].clear();
        for (uint32_t p = hm.rowptr[j]; p < hm.rowptr[j + 1]; ++p) {
            const uint32_t k = hm.col[p];
            if (hidx[k] < 0 && best_cnt > 0 && float_bits(hm.val[p]) == best_bits) u.push_back(k);
            else exc[h].push_back({k, hm.val[p]});
        }
        if (exc[h].size() > XM) return false;
        if (h == 0) first_u = u;
        else if (u != first_u) return false;
    }
    *U = first_u;
    return true;
}

}  // namespace

Plan make_plan(const HostModel& hm, int max_threads, bool allow_uniform) {
    Plan plan;
    const uint32_t n = hm.n;
    if (max_threads <= 0) max_threads = kMaxFusedThreads;
    max_threads = std::min(max_threads, kMaxFusedThreads);
    std::vector<uint32_t> rowlen(n);
    for (uint32_t j = 0; j < n; ++j) rowlen[j] = hm.rowptr[j + 1] - hm.rowptr[j];

    for (int fam = 0; fam < kNumFamilies; ++fam) {
        const uint32_t R = family_rmax(fam), HM = family_hmax(fam), XM = family_xmax(fam);
        const int mode = family_mode(fam);
        if (mode == kHeavyUniform && !allow_uniform) continue;
        std::vector<uint32_t> heavy;
        for (uint32_t j = 0; j < n; ++j)
            if (rowlen[j] > R) heavy.push_back(j);
        if (heavy.size() > HM) continue;
        std::vector<int> hidx(n, -1);
        for (size_t h = 0; h < heavy.size(); ++h) hidx[heavy[h]] = (int)h;

        float hw[kMaxHeavy] = {kInfH, kInfH, kInfH, kInfH};
        std::vector<std::pair<uint32_t, float>> exc[kMaxHeavy];
        std::vector<uint32_t> U;
        if (mode == kHeavyUniform) {
            if (!analyse_uniform(hm, hidx, heavy, XM, hw, exc, &U)) continue;
        } else {
            // general: exceptions are the heavy sources of each heavy row
            for (size_t h = 0; h < heavy.size(); ++h) {
                const uint32_t j = heavy[h];
                for (uint32_t p = hm.rowptr[j]; p < hm.rowptr[j + 1]; ++p)
                    if (hidx[hm.col[p]] >= 0) exc[h].push_back({hm.col[p], hm.val[p]});
                if (exc[h].size() > XM) return plan;  // cannot happen: <= H <= HM <= XM
            }
        }

        // geometry: fewest slots per thread whose workgroup fits the cap and LDS
        uint32_t SM = 0, B = 0, vstride = 0;
        size_t lds = 0;
        for (int c = 0; c < kNumSlotChoices; ++c) {
            const uint32_t sm = kSlotChoices[c];
            uint32_t b = round_up((n + sm - 1) / sm, 64);
            if (b < 64) b = 64;
            if (b > (uint32_t)max_threads) continue;
            const uint32_t vs = round_up(sm * b + 1 + kMaxHeavy, 4);
            const size_t l = fused_lds_bytes_for((int)sm, b, vs);
            if (l > kMaxLdsBytes) continue;
            SM = sm;
            B = b;
            vstride = vs;
            lds = l;
            break;
        }
        if (SM == 0) return plan;  // too large for the fused kernel: generic fallback

        plan.fused = true;
        plan.family = fam;
        plan.B = B;
        plan.SM = SM;
        plan.R = R;
        plan.HM = HM;
        plan.XM = XM;
        plan.H = (uint32_t)heavy.size();
        plan.mode = mode;
        plan.estride = SM * B;
        plan.vstride = vstride;
        plan.lds_bytes = lds;
        const uint32_t est = plan.estride, scratch = est, hs0 = est + 1;
        auto lds_index = [&](uint32_t k) { return hidx[k] >= 0 ? hs0 + (uint32_t)hidx[k] : k; };

        for (uint32_t h = 0; h < kMaxHeavy; ++h) {
            plan.hrow[h] = h < plan.H ? (int)heavy[h] : 0;  // dummies: any valid state
            plan.hw[h] = (h < plan.H && mode == kHeavyUniform) ? hw[h] : kInfH;
            for (uint32_t x = 0; x < kMaxExc; ++x) {
                const bool ok = h < plan.H && x < exc[h].size();
                plan.xk[h][x] = ok ? lds_index(exc[h][x].first) : scratch;
                plan.xw[h][x] = ok ? exc[h][x].second : kInfH;
            }
        }
        // light rows
        plan.lcol.assign((size_t)SM * R * B, scratch);
        plan.lval.assign((size_t)SM * R * B, kInfH);
        for (uint32_t j = 0; j < n; ++j) {
            if (hidx[j] >= 0) continue;
            const uint32_t s = j / B, t = j % B;
            uint32_t r = 0;
            for (uint32_t p = hm.rowptr[j]; p < hm.rowptr[j + 1]; ++p, ++r) {
                const size_t idx = ((size_t)s * R + r) * B + t;
                plan.lcol[idx] = lds_index(hm.col[p]);
                plan.lval[idx] = hm.val[p];
            }
        }
        // heavy rows
        if (mode == kHeavyUniform) {
            plan.hmask.assign(est, kInfH);
            for (uint32_t k : U) plan.hmask[k] = 0.0f;
        } else {
            plan.hval.assign((size_t)HM * SM * B, kInfH);
            plan.hvalid.assign((size_t)HM * SM * B, 0);
            for (uint32_t h = 0; h < plan.H; ++h) {
                const uint32_t j = heavy[h];
                for (uint32_t p = hm.rowptr[j]; p < hm.rowptr[j + 1]; ++p) {
                    const uint32_t k = hm.col[p];
                    if (hidx[k] >= 0) continue;  // exception term
                    const size_t idx = ((size_t)h * SM + k / B) * B + k % B;
                    plan.hval[idx] = hm.val[p];
                    plan.hvalid[idx] = 1;
                }
            }
        }
        // emissions padded to estride, plus the DMA over-read tail
        const size_t ndma = (SM + 3) / 4;
        plan.emis_pad.assign((size_t)hm.S * est + ndma * B * 4 + 64, kInfH);
        for (uint32_t o = 0; o < hm.S; ++o)
            std::copy(hm.emis.begin() + (size_t)o * n, hm.emis.begin() + (size_t)(o + 1) * n,
                      plan.emis_pad.begin() + (size_t)o * est);
        plan.start_pad.assign(est + 16, kInfH);
        std::copy(hm.start.begin(), hm.start.end(), plan.start_pad.begin());
        return plan;
    }
    return plan;
}

// ------------------------------------------------------------------------------------------
// Chain ("band") planning: light rows in ascending row order at positions p; each light row's
// terms come from heavy rows and from position p-1 only; each heavy row's light sources are
// either all light rows with one shared weight, or none; heavy-row exceptions come from heavy
// rows only.  Every reference .chmm (MSV shape) qualifies.
// ------------------------------------------------------------------------------------------
namespace {

// Heavy rows of the chain plan: rows with in-degree > kBandHeavy + 1, plus (repeatedly) the first light row
// whose terms break the chain rule, while at most kBandHeavy rows are heavy.
bool band_heavy_rows(const HostModel& hm, std::vector<uint32_t>* heavy_out) {
    const uint32_t n = hm.n;
    std::vector<uint8_t> is_heavy(n, 0);
    uint32_t count = 0;
    for (uint32_t j = 0; j < n; ++j)
        if (hm.rowptr[j + 1] - hm.rowptr[j] > (uint32_t)kBandHeavy + 1) {  // > HA_max + 1 terms
            is_heavy[j] = 1;
            ++count;
        }
    while (count <= (uint32_t)kBandHeavy) {
        uint32_t prev = 0xFFFFFFFFu, bad = 0xFFFFFFFFu;
        for (uint32_t j = 0; j < n && bad == 0xFFFFFFFFu; ++j) {
            if (is_heavy[j]) continue;
            for (uint32_t e = hm.rowptr[j]; e < hm.rowptr[j + 1]; ++e) {
                const uint32_t k = hm.col[e];
                if (!is_heavy[k] && k != prev) {
                    bad = j;
                    break;
                }
            }
            prev = j;
        }
        if (bad == 0xFFFFFFFFu) {
            heavy_out->clear();
            for (uint32_t j = 0; j < n; ++j)
                if (is_heavy[j]) heavy_out->push_back(j);
            return true;
        }
        is_heavy[bad] = 1;
        ++count;
    }
    return false;
}

// Structure of a chain-shaped model (shared by the chain / band plans and the pipelined plan).
// Heavy rows are renumbered x = 0.. with the feeders of light rows first.
struct BandShape {
    bool ok = false;
    std::vector<uint32_t> heavy;               // heavy row ids, in renumbered order x
    std::vector<uint32_t> light;               // light row ids by position p
    uint32_t HA = 0;                           // heavy rows feeding light rows (x < HA)
    std::vector<float> bw;                     // [p] weight of the term from position p-1 (+inf: none)
    std::vector<uint8_t> bex;                  // [p] that term exists
    std::vector<std::vector<float>> aw;        // [x][p] weight of the term from heavy row x
    std::vector<std::vector<uint8_t>> aex;     // [x][p] that term exists
    float wh[kBandHeavy] = {kInfH, kInfH};     // shared weight of the light terms of heavy row x
    std::vector<std::pair<uint32_t, float>> exc[kBandHeavy];  // heavy row x's terms from heavy rows
    uint32_t hl_exist = 0, hx_exist = 0;       // BandModel::hl_exist / hx_exist
};

BandShape analyze_band(const HostModel& hm) {
    BandShape sh;
    const uint32_t n = hm.n;
    std::vector<uint32_t> heavy;
    if (!band_heavy_rows(hm, &heavy)) return sh;
    if (heavy.size() > (size_t)kBandHeavy || heavy.size() >= n) return sh;
    std::vector<int> hidx(n, -1);
    for (size_t h = 0; h < heavy.size(); ++h) hidx[heavy[h]] = (int)h;
    std::vector<uint32_t> light, pos(n, 0xFFFFFFFFu);
    for (uint32_t j = 0; j < n; ++j)
        if (hidx[j] < 0) {
            pos[j] = (uint32_t)light.size();
            light.push_back(j);
        }
    const uint32_t nL = (uint32_t)light.size();

    // light-row terms
    std::vector<float> bwp(nL, kInfH);
    std::vector<std::vector<float>> awp(heavy.size(), std::vector<float>(nL, kInfH));
    std::vector<uint8_t> feeds(heavy.size(), 0);
    std::vector<uint8_t> bex(nL, 0);                                            // term p-1 -> p exists
    std::vector<std::vector<uint8_t>> aex(heavy.size(), std::vector<uint8_t>(nL, 0));  // heavy -> p
    for (uint32_t p = 0; p < nL; ++p) {
        const uint32_t j = light[p];
        for (uint32_t e = hm.rowptr[j]; e < hm.rowptr[j + 1]; ++e) {
            const uint32_t k = hm.col[e];
            if (hidx[k] >= 0) {
                awp[hidx[k]][p] = hm.val[e];
                aex[hidx[k]][p] = 1;
                feeds[hidx[k]] = 1;
            } else if (p > 0 && pos[k] == p - 1) {
                bwp[p] = hm.val[e];
                bex[p] = 1;
            } else {
                return sh;
            }
        }
    }
    // heavy rows: feeders of light rows first (the kernel reads aw[h] against vh[h], h < HA)
    std::vector<uint32_t> order;
    for (size_t h = 0; h < heavy.size(); ++h)
        if (feeds[h]) order.push_back((uint32_t)h);
    const uint32_t HA = (uint32_t)order.size();
    for (size_t h = 0; h < heavy.size(); ++h)
        if (!feeds[h]) order.push_back((uint32_t)h);
    std::vector<int> newidx(heavy.size());
    for (size_t x = 0; x < order.size(); ++x) newidx[order[x]] = (int)x;

    for (size_t x = 0; x < order.size(); ++x) {
        const uint32_t j = heavy[order[x]];
        uint32_t nlight = 0;
        bool first = true, same = true;
        float w = kInfH;
        for (uint32_t e = hm.rowptr[j]; e < hm.rowptr[j + 1]; ++e) {
            const uint32_t k = hm.col[e];
            if (hidx[k] >= 0) {
                sh.exc[x].push_back({(uint32_t)newidx[hidx[k]], hm.val[e]});
            } else {
                ++nlight;
                if (first) w = hm.val[e];
                else same &= float_bits(hm.val[e]) == float_bits(w);
                first = false;
            }
        }
        if (sh.exc[x].size() > (size_t)kBandHeavy) return sh;  // cannot happen: one term per source
        if (nlight != 0 && (nlight != nL || !same)) return sh;
        sh.wh[x] = nlight ? w : kInfH;
        if (nlight) sh.hl_exist |= 1u << x;
        for (const auto& e : sh.exc[x]) sh.hx_exist |= 1u << (x * kBandHeavy + e.first);
    }
    for (size_t x = 0; x < order.size(); ++x) {
        sh.heavy.push_back(heavy[order[x]]);
        sh.aw.push_back(std::move(awp[order[x]]));
        sh.aex.push_back(std::move(aex[order[x]]));
    }
    sh.light = std::move(light);
    sh.HA = HA;
    sh.bw = std::move(bwp);
    sh.bex = std::move(bex);
    sh.ok = true;
    return sh;
}

}  // namespace

BandPlan make_band_plan(const HostModel& hm, int max_threads, bool chain, int ge_waves) {
    BandPlan bp;
    const uint32_t n = hm.n, S = hm.S;
    if (chain && S > (uint32_t)kChainMaxSym) return bp;
    if (max_threads <= 0) max_threads = chain ? kChainMaxThreads : kDefaultBandThreads;
    max_threads = std::min(max_threads, chain ? kChainMaxThreads : kMaxBandThreads);
    BandShape sh = analyze_band(hm);
    if (!sh.ok) return bp;
    const std::vector<uint32_t>& light = sh.light;
    const uint32_t nL = (uint32_t)light.size();
    const uint32_t HA = sh.HA;
    const float* wh = sh.wh;
    const auto& exc = sh.exc;
    bp.hl_exist = sh.hl_exist;
    bp.hx_exist = sh.hx_exist;

    uint32_t SM = 0, B = 0;
    bool ge = false;
    const char* ge_env = std::getenv("SVH_CHAIN_GE");  // diagnostic: waves
    const int gw = !chain ? 0 : ge_waves >= 0 ? ge_waves : (ge_env ? std::atoi(ge_env) : 0);
    if (gw > 0) {
        const uint32_t w = (uint32_t)gw;
        const uint32_t sm = (nL + 64 * w - 1) / (64 * w);
        if (chain_supported((int)sm, (int)w, (int)std::max<uint32_t>(HA, 1), true)) {
            SM = sm;
            B = 64 * w;
            ge = true;
        }
    } else if (chain) {
        // barrier-free kernel: fewest waves (1, 2, 4, 8) holding <= 5 positions per thread
        // (SVH_CHAIN_WAVES=<w>: diagnostic override of the wave count)
        const char* wv_env = std::getenv("SVH_CHAIN_WAVES");
        const uint32_t w_force = wv_env ? (uint32_t)std::atoi(wv_env) : 0;
        for (uint32_t w = w_force ? w_force : 1; w <= 8 && SM == 0; w *= 2) {
            if (64 * w > (uint32_t)max_threads) break;
            const uint32_t sm = (nL + 64 * w - 1) / (64 * w);
            if (sm <= 5 || w == 8 || 128 * w > (uint32_t)max_threads) {
                if (chain_supported((int)sm, (int)w, (int)std::max<uint32_t>(HA, 1), false)) {
                    SM = sm;
                    B = 64 * w;
                }
                break;
            }
        }
    } else {
        // barrier kernel: fewest slots per thread within the thread cap
        for (int c = 0; c < kNumBandSlotChoices; ++c) {
            const uint32_t sm = (uint32_t)kBandSlotChoices[c];
            const uint32_t b = std::max<uint32_t>(64, round_up((nL + sm - 1) / sm, 64));
            if (b > (uint32_t)max_threads) continue;
            SM = sm;
            B = b;
            break;
        }
    }
    if (SM == 0) return bp;
    const uint32_t cap = SM * B;
    const uint32_t erow = round_up(cap + kBandTail, 256);
    if (band_lds_bytes(erow) > kMaxLdsBytes) return bp;

    bp.ok = true;
    bp.chain = chain;
    bp.ge = ge;
    bp.B = B;
    bp.SM = SM;
    bp.HA = HA;
    bp.H = (uint32_t)sh.heavy.size();
    bp.nL = nL;
    bp.erow = erow;
    bp.lds_bytes = band_lds_bytes(erow);
    for (int x = 0; x < kBandHeavy; ++x) {
        const bool real = (size_t)x < sh.heavy.size();
        bp.hrow[x] = real ? (int)sh.heavy[x] : 0;
        bp.hvalid[x] = real ? 1 : 0;
        bp.hstart[x] = real ? hm.start[sh.heavy[x]] : kInfH;
    }
    // per-thread tables, lane-consecutive index s*B + t for position t*SM + s
    auto slot_of = [&](uint32_t p) { return (p % SM) * B + p / SM; };
    bp.lrow.assign(cap, 0xFFFFFFFFu);
    bp.start.assign(cap, kInfH);
    bp.bw.assign(cap, kInfH);
    bp.aw.assign((size_t)std::max<uint32_t>(HA, 1) * cap, kInfH);
    // decoded paths: per-position term flags (heavy feeder 0 only: the path variant has HA <= 1)
    // and the state -> position / heavy index map of the traceback
    bp.pflags.assign(cap, 0);
    bp.spos.assign(n, 0);
    for (uint32_t p = 0; p < nL; ++p) {
        const uint32_t x = slot_of(p);
        bp.lrow[x] = light[p];
        bp.start[x] = hm.start[light[p]];
        bp.bw[x] = sh.bw[p];
        for (uint32_t a = 0; a < HA; ++a) bp.aw[(size_t)a * cap + x] = sh.aw[a][p];
        uint8_t f = sh.bex[p] ? 1 : 0;
        if (HA >= 1 && sh.aex[0][p]) f |= 2;
        if (HA >= 1 && p > 0 && sh.heavy[0] < light[p - 1]) f |= 4;
        bp.pflags[x] = f;
        bp.ties_heavy = (p == 0 ? true : bp.ties_heavy) && (f & 2) && (!(f & 1) || (f & 4));
        bp.spos[light[p]] = (int32_t)p;
    }
    for (size_t x = 0; x < sh.heavy.size(); ++x) bp.spos[sh.heavy[x]] = -1 - (int32_t)x;
    // streamed-E chain kernel: [o][t][round_up(SM,4)]
    if (ge) {
        const uint32_t smp = (SM + 3) / 4 * 4;
        bp.erows_t.assign((size_t)S * B * smp, kInfH);
        for (uint32_t o = 0; o < S; ++o)
            for (uint32_t p = 0; p < nL; ++p)
                bp.erows_t[((size_t)o * B + p / SM) * smp + p % SM] = hm.emis[(size_t)o * n + light[p]];
    }
    // emission rows: permuted light part, then the folded heavy constants
    bp.erows.assign((size_t)S * erow, kInfH);
    for (uint32_t o = 0; o < S; ++o) {
        const float* E = hm.emis.data() + (size_t)o * n;
        float* row = bp.erows.data() + (size_t)o * erow;
        for (uint32_t p = 0; p < nL; ++p) row[slot_of(p)] = E[light[p]];
        float* tl = row + cap;
        for (int x = 0; x < kBandHeavy; ++x) {
            if (!bp.hvalid[x]) continue;
            const float eh = E[bp.hrow[x]];
            tl[kBandTailA + x] = eh + wh[x];  // fl(E_h + w_h): the shared uniform term
            for (const auto& [src, w] : exc[x]) tl[band_tail_x((int)x, (int)src)] = eh + w;  // heavy src -> h
            tl[kBandTailE + x] = eh;
        }
    }
    return bp;
}

void DeviceBandPlan::upload(const BandPlan& p, uint32_t n, uint32_t S, hipStream_t s) {
    plan = p;
    if (!p.ok) return;
    d_erows.upload(p.erows.data(), p.erows.size() * 4, s);
    d_start.upload(p.start.data(), p.start.size() * 4, s);
    d_aw.upload(p.aw.data(), p.aw.size() * 4, s);
    d_bw.upload(p.bw.data(), p.bw.size() * 4, s);
    d_lrow.upload(p.lrow.data(), p.lrow.size() * 4, s);
    if (p.ge) d_erows_t.upload(p.erows_t.data(), p.erows_t.size() * 4, s);
    d_pflags.upload(p.pflags.data(), p.pflags.size(), s);
    d_spos.upload(p.spos.data(), p.spos.size() * 4, s);
    std::memset(&view, 0, sizeof(view));
    view.erows = d_erows.as<float>();
    view.start = d_start.as<float>();
    view.aw = d_aw.as<float>();
    view.bw = d_bw.as<float>();
    view.lrow = d_lrow.as<uint32_t>();
    view.erows_t = p.ge ? d_erows_t.as<float>() : nullptr;
    view.ge = p.ge ? 1u : 0u;
    view.pflags = d_pflags.as<uint8_t>();
    view.spos = d_spos.as<int32_t>();
    view.hx_exist = p.hx_exist;
    view.hl_exist = p.hl_exist;
    view.ties_heavy = p.ties_heavy ? 1u : 0u;
    for (int h = 0; h < kBandHeavy; ++h) {
        view.hrow[h] = p.hrow[h];
        view.hvalid[h] = p.hvalid[h];
        view.hstart[h] = p.hstart[h];
    }
    view.n = n;
    view.S = S;
    view.B = p.B;
    view.SM = p.SM;
    view.erow = p.erow;
    view.H = p.H;
    const char* dbg = std::getenv("SVH_BAND_DEBUG");  // diagnostic ablations only
    view.dbg = dbg ? (uint32_t)std::atoi(dbg) : 0u;
    if (view.dbg & (4u | 128u)) {
        d_stamps.alloc((size_t)4096 * kMaxWaves * kBandStamps * 8);
        hip_check(hipMemsetAsync(d_stamps.ptr, 0, d_stamps.bytes, s), "stamps");
        view.stamps = d_stamps.as<unsigned long long>();
    }
}

// ------------------------------------------------------------------------------------------
// Pipelined chain plan (pipe.hip): chain-shaped models with exactly one heavy row F feeding the
// light rows, F's heavy-row terms from itself only, and the other heavy row S (if any) feeding
// no light row and not F.  Positions p (chain order) in blocks of 64*SM, one wave each.
// ------------------------------------------------------------------------------------------
PipePlan make_pipe_plan(const HostModel& hm, uint32_t sm, uint32_t waves, bool wide) {
    PipePlan pp;
    const uint32_t n = hm.n, S = hm.S;
    if (S > 32) return pp;
    const BandShape sh = analyze_band(hm);
    if (!sh.ok || sh.HA != 1) return pp;
    const uint32_t H = (uint32_t)sh.heavy.size();
    float xff = kInfH, xss = kInfH, xsf = kInfH;
    for (const auto& e : sh.exc[0]) {
        if (e.first != 0) return pp;  // F <- S: F would depend on S, which depends on every light row
        xff = e.second;
    }
    bool sx = false;
    if (H == 2) {
        for (const auto& e : sh.exc[1]) {
            if (e.first == 1) xss = e.second;
            else { xsf = e.second; sx = true; }
        }
    }
    if (const char* e = std::getenv(wide ? "SVH_PIPEW_SM" : "SVH_PIPE_SM")) sm = (uint32_t)std::atoi(e);
    if (const char* e = std::getenv(wide ? "SVH_PIPEW_WAVES" : "SVH_PIPE_WAVES")) waves = (uint32_t)std::atoi(e);
    // latency plan: 2 slots per lane, 4 waves per workgroup: one wave per SIMD at the headline
    // width (measured against 1 x 8, 1 x 4 and 2 x 8: DESIGN.md 5b); wide plan: 8 slots per
    // lane, 16 sequences per workgroup
    if (sm == 0) sm = wide ? 8 : 2;
    if (waves == 0) waves = wide ? 16 : 4;
    if (wide ? !pipew_supported((int)sm, (int)waves, sx) : !pipe_supported((int)sm, (int)waves, sx)) return pp;
    if (wide && pipew_lds_bytes(sm, waves, S, sx) > 160 * 1024) return pp;
    const uint32_t nL = (uint32_t)sh.light.size();
    const uint32_t bsz = 64 * sm;
    pp.wide = wide;
    pp.SM = sm;
    pp.W = waves;
    pp.nblk = (nL + bsz - 1) / bsz;
    pp.G = wide ? pp.nblk : (pp.nblk + waves - 1) / waves;
    pp.P = pp.nblk * bsz;
    pp.sx = sx;
    pp.rowF = (int)sh.heavy[0];
    pp.rowS = H == 2 ? (int)sh.heavy[1] : -1;
    pp.startF = hm.start[sh.heavy[0]];
    pp.startS = H == 2 ? hm.start[sh.heavy[1]] : kInfH;
    const uint32_t P = pp.P;
    const uint32_t nc = wide ? pipew_chunks(sm, sx) : 0;  // wide: 16-byte chunks per symbol and lane
    pp.tab.assign(wide ? (size_t)pp.nblk * S * nc * 64 * 4 : (size_t)pp.nblk * S * sm * 64 * 2, kInfH);
    pp.e0.assign((size_t)S * P, kInfH);
    pp.start.assign(P, kInfH);
    pp.lrow.assign(P, 0xFFFFFFFFu);
    for (uint32_t p = 0; p < nL; ++p) {
        const uint32_t j = sh.light[p], blk = p / bsz, lane = (p % bsz) / sm, s = p % sm;
        pp.start[p] = hm.start[j];
        pp.lrow[p] = j;
        for (uint32_t o = 0; o < S; ++o) {
            const float e = hm.emis[(size_t)o * n + j];
            pp.e0[(size_t)o * P + p] = e;
            const float eb = e + sh.bw[p];     // fl(E_o[p] + bw_p): the reference's first add of the chain term
            const float ea = e + sh.aw[0][p];  // fl(E_o[p] + aw_p): ... of F's term
            if (wide) {
                // chunks of 4 per lane: [eb_1 .. eb_{SM-1}, eb_0] then [ea_0 .. ea_{SM-1}]
                const uint32_t ib = s == 0 ? sm - 1 : s - 1, ia = sm + s;
                float* base = pp.tab.data() + (((size_t)blk * S + o) * nc) * 64 * 4;
                base[((ib / 4) * 64 + lane) * 4 + ib % 4] = eb;
                base[((ia / 4) * 64 + lane) * 4 + ia % 4] = ea;
            } else {
                float* t = pp.tab.data() + ((((size_t)blk * S + o) * sm + s) * 64 + lane) * 2;
                t[0] = eb;
                t[1] = ea;
            }
        }
    }
    // diagonal plan (diag.hip): position-major planes {ea, eb} per symbol over 64 nrng positions (the
    // light rows in chain order, then +inf dummies); position 0 has no chain term (bw_0 = +inf), which
    // the diagonals rely on when they wrap
    if (!wide && sm == 2) {
        pp.nrng = (nL + 63) / 64;
        const uint32_t NP = pp.nrng * 64;
        pp.dtab.assign((size_t)S * NP * 2, kInfH);
        for (uint32_t p = 0; p < nL; ++p)
            for (uint32_t o = 0; o < S; ++o) {
                const float e = hm.emis[(size_t)o * n + sh.light[p]];
                float* d = pp.dtab.data() + ((size_t)o * NP + p) * 2;
                d[0] = e + sh.aw[0][p];
                d[1] = e + sh.bw[p];
            }
        if (sh.bw[0] < kInfH) {  // cannot happen (analyze_band: p > 0), but the wrap depends on it
            pp.nrng = 0;
            pp.dtab.clear();
        }
    }
    // decoded paths: term flags per position (as BandPlan::pflags with heavy feeder F) and the
    // state -> position map (-1 F, -2 S)
    pp.pflags.assign(P, 0);
    pp.spos.assign(n, 0);
    pp.ties_heavy = nL > 0;
    for (uint32_t p = 0; p < nL; ++p) {
        uint8_t f = sh.bex[p] ? 1 : 0;
        if (sh.aex[0][p]) f |= 2;
        if (p > 0 && sh.heavy[0] < sh.light[p - 1]) f |= 4;
        pp.pflags[p] = f;
        pp.ties_heavy = pp.ties_heavy && (f & 2) && (!(f & 1) || (f & 4));
        pp.spos[sh.light[p]] = (int32_t)p;
    }
    for (uint32_t x = 0; x < H; ++x) pp.spos[sh.heavy[x]] = -1 - (int32_t)x;
    pp.hx_exist = sh.hx_exist;
    pp.hl_exist = sh.hl_exist;
    pp.hc.assign((size_t)S * 8, kInfH);
    auto wide_consts = [&](uint32_t o, const float* c) {  // wide: constants chunk(s) of every lane
        for (uint32_t blk = 0; blk < pp.nblk; ++blk)
            for (uint32_t lane = 0; lane < 64; ++lane) {
                float* base = pp.tab.data() + ((((size_t)blk * S + o) * nc + sm / 2) * 64 + lane) * 4;
                for (int k = 0; k < 4; ++k) base[k] = c[k];
                if (sx) {
                    float* b2 = base + 64 * 4;
                    b2[0] = c[4];
                    b2[1] = b2[2] = b2[3] = 0.0f;
                }
            }
    };
    for (uint32_t o = 0; o < S; ++o) {
        float* c = pp.hc.data() + (size_t)o * 8;
        const float eF = hm.emis[(size_t)o * n + sh.heavy[0]];
        const float eS = H == 2 ? hm.emis[(size_t)o * n + sh.heavy[1]] : kInfH;
        c[0] = eS + (H == 2 ? sh.wh[1] : kInfH);  // A_S
        c[1] = eF + sh.wh[0];  // A_F
        c[2] = eS + xss;       // X_SS
        c[3] = eF + xff;       // X_FF
        c[4] = eS + xsf;       // X_SF
        c[5] = eF;             // E_F (first observation)
        c[6] = eS;             // E_S
        c[7] = 0.0f;
        if (wide) wide_consts(o, c);
    }
    // level 2 (pipe_kernel.h step2): every score >= 0 (the margin bound), the largest finite ea
    bool nonneg = !wide;
    for (float v : hm.val) nonneg = nonneg && v >= 0.0f;
    for (float v : hm.emis) nonneg = nonneg && v >= 0.0f;
    for (float v : hm.start) nonneg = nonneg && v >= 0.0f;
    pp.emax2 = nonneg ? 0.0f : kInfH;
    if (nonneg)
        for (uint32_t p = 0; p < nL; ++p)
            for (uint32_t o = 0; o < S; ++o) {
                const float ea = hm.emis[(size_t)o * n + sh.light[p]] + sh.aw[0][p];
                if (ea < kInfH) pp.emax2 = std::max(pp.emax2, ea);
            }
    pp.ok = true;
    return pp;
}

void DevicePipePlan::upload(const PipePlan& p, uint32_t n, uint32_t S, hipStream_t s) {
    plan = p;
    if (!p.ok) return;
    d_tab.upload(p.tab.data(), p.tab.size() * 4, s);
    d_e0.upload(p.e0.data(), p.e0.size() * 4, s);
    d_start.upload(p.start.data(), p.start.size() * 4, s);
    d_lrow.upload(p.lrow.data(), p.lrow.size() * 4, s);
    d_hc.upload(p.hc.data(), p.hc.size() * 4, s);
    d_pflags.upload(p.pflags.data(), p.pflags.size(), s);
    d_spos.upload(p.spos.data(), p.spos.size() * 4, s);
    std::memset(&view, 0, sizeof(view));
    view.pflags = d_pflags.as<uint8_t>();
    view.spos = d_spos.as<int32_t>();
    view.hx_exist = p.hx_exist;
    view.hl_exist = p.hl_exist;
    view.ties_heavy = p.ties_heavy ? 1u : 0u;
    view.tab = d_tab.as<float2>();
    view.e0 = d_e0.as<float>();
    view.start = d_start.as<float>();
    view.lrow = d_lrow.as<uint32_t>();
    view.hc = d_hc.as<float>();
    view.rowF = p.rowF;
    view.rowS = p.rowS;
    view.startF = p.startF;
    view.startS = p.startS;
    view.n = n;
    view.S = S;
    view.P = p.P;
    view.nblk = p.nblk;
    view.SM = p.SM;
    view.W = p.W;
    view.G = p.G;
    view.sx = p.sx ? 1u : 0u;
    view.wide = p.wide ? 1u : 0u;
    view.rerun = !p.wide && pipe_rerun_fits(p.P, p.W) ? 1u : 0u;
    if (p.nrng && !p.dtab.empty() && diag_lds_bytes(diag_waves_for(4), S, p.P) <= 160 * 1024) {
        d_dtab.upload(p.dtab.data(), p.dtab.size() * 4, s);
        view.dtab = d_dtab.as<float2>();
        view.nrng = p.nrng;
    }
    view.emax2 = p.emax2;
    // the pair-table step wherever it applies: TM = 4 (indexed operands, packed feeder terms:
    // 0.255 ms on the headline against 0.263 / 0.268 / 0.277 for TM 2 / 3 / 1 and 0.334 for the
    // per-slot tables); SVH_PIPE_TM selects another mode (A/B and tests: 0 per-slot
    // tables, 1 pair tables by 64-bit moves, 2 indexed operands, 3 packed feeder terms, 4 both)
    view.tm = !p.wide && p.SM == 2 && (p.W == 4 || (p.W == 8 && pipe_tm_supported(-8))) && S <= kPairSymbols ? 4u : 0u;
    if (const char* e = std::getenv("SVH_PIPE_TM"); e) {
        const int t = std::atoi(e);
        if (t == 0 || (t >= 1 && t <= 4 && view.tm && pipe_tm_supported(t))) view.tm = (uint32_t)t;
    }
    if (const char* e = std::getenv("SVH_PIPE_DEBUG"); e && std::atoi(e)) {  // diagnostics only
        d_stamps.alloc((size_t)65536 * kPipeStamps * 8);
        hip_check(hipMemsetAsync(d_stamps.ptr, 0, d_stamps.bytes, s), "stamps");
        view.stamps = d_stamps.as<unsigned long long>();
        view.diag = (uint32_t)std::atoi(e) >> 1;
    }
}

void DevicePipePlan::report_stamps(uint32_t nseq) const {
    if (!view.stamps) return;
    const size_t waves = (size_t)nseq * plan.G * plan.W;
    if (waves > 65536 / kPipeStamps * kPipeStamps) return;
    std::vector<unsigned long long> h(waves * kPipeStamps);
    if (hipMemcpy(h.data(), view.stamps, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    double sum[kPipeStamps] = {}, mx[kPipeStamps] = {};
    for (size_t w = 0; w < waves; ++w)
        for (int k = 0; k < kPipeStamps; ++k) {
            sum[k] += (double)h[w * kPipeStamps + k];
            mx[k] = std::max(mx[k], (double)h[w * kPipeStamps + k]);
        }
    std::fprintf(stderr, "pipe stamps (avg / max per wave): loop %.0f/%.0f head %.0f/%.0f tail %.0f/%.0f "
                 "prev %.0f/%.0f next %.0f/%.0f gran %.0f/%.0f cons %.0f/%.0f iters %.0f slow-groups %.0f/%.0f\n",
                 sum[0] / waves, mx[0], sum[1] / waves, mx[1], sum[2] / waves, mx[2], sum[3] / waves, mx[3],
                 sum[4] / waves, mx[4], sum[5] / waves, mx[5], sum[6] / waves, mx[6], sum[7] / waves,
                 sum[14] / waves, mx[14]);
    {  // wall clock (100 MHz): per wave entry / sweep start / body end / sweep end, from the launch's first entry
        unsigned long long t0 = ~0ull, tend = 0;
        for (size_t w = 0; w < waves; ++w)
            if (h[w * kPipeStamps + 8]) {
                t0 = std::min(t0, h[w * kPipeStamps + 8]);
                tend = std::max(tend, h[w * kPipeStamps + 11]);
            }
        if (t0 != ~0ull) std::fprintf(stderr, "pipe wall (us from first entry): last sweep end %.2f\n", (tend - t0) * 0.01);
        // per sequence (tickets q*G .. q*G+G-1): each workgroup's latest entry, w0 start and latest end
        for (uint32_t q = 0; t0 != ~0ull && q < nseq; ++q) {
            std::fprintf(stderr, "  seq %u:", q);
            for (uint32_t g = 0; g < plan.G; ++g) {
                unsigned long long en = 0, st = 0, ed = 0, tb = 0;
                for (uint32_t w = 0; w < plan.W; ++w) {
                    const unsigned long long* r = h.data() + (((size_t)q * plan.G + g) * plan.W + w) * kPipeStamps;
                    if (!r[8]) continue;
                    en = std::max(en, r[8] - t0);
                    if (w == 0) st = r[9] - t0;
                    if (w == 0 && r[13]) tb = r[13] - t0;
                    ed = std::max(ed, r[11] - t0);
                }
                // placement of the workgroup's first wave: XCC and CU (HW_ID bits 11:8) / SE (14:13)
                // and its shader clock over the body: s_memtime cycles / s_memrealtime (100 MHz) span
                const unsigned long long* r0 = h.data() + (((size_t)q * plan.G + g) * plan.W) * kPipeStamps;
                const unsigned long long hw = r0[12];
                const double mhz = r0[10] > r0[9] ? (double)r0[0] / ((double)(r0[10] - r0[9]) * 0.01) : 0.0;
                std::fprintf(stderr, " [g%u in %.1f tab %.1f st %.1f end %.1f x%u s%u c%u %.0fMHz]", g, en * 0.01, tb * 0.01,
                             st * 0.01, ed * 0.01, (unsigned)(hw >> 32) & 0xFu, (unsigned)(hw >> 13) & 0x3u,
                             (unsigned)(hw >> 8) & 0xFu, mhz);
            }
            std::fprintf(stderr, "\n");
        }
        for (size_t w = 0; t0 != ~0ull && w < waves; ++w) {
            const unsigned long long* r = h.data() + w * kPipeStamps;
            if (!r[8] || w / plan.W >= 2 * plan.G) continue;  // the first two sequences' waves
            std::fprintf(stderr, "  wave %zu (seq-ticket %zu): entry %.2f start %.2f body_end %.2f end %.2f\n", w % plan.W,
                         w / plan.W, (r[8] - t0) * 0.01, (r[9] - t0) * 0.01, (r[10] - t0) * 0.01, (r[11] - t0) * 0.01);
        }
    }
    // the wait split by role: per (workgroup g, wave w) of a row, averaged over the batch's rows:
    // loop cycles, polls waiting for the previous wave's count (prev), for the next wave's count
    // (next, flow control), for granules (gran), for the consumer's progress word (cons), and the
    // groups whose boundary vector was re-read after a wait (slow)
    {
        std::fprintf(stderr, "pipe wait split by role (mean over %u rows): g w loop prev next gran cons slow\n", nseq);
        for (uint32_t g = 0; g < plan.G; ++g)
            for (uint32_t w = 0; w < plan.W; ++w) {
                double a[8] = {};
                uint32_t cnt = 0;
                for (uint32_t q = 0; q < nseq; ++q) {
                    const unsigned long long* r = h.data() + (((size_t)q * plan.G + g) * plan.W + w) * kPipeStamps;
                    if (!r[8]) continue;
                    ++cnt;
                    a[0] += (double)r[0];
                    for (int k = 3; k <= 6; ++k) a[k - 2] += (double)r[k];
                    a[5] += (double)r[14];
                }
                if (!cnt) continue;
                std::fprintf(stderr, "  role g%u w%u: %.0f %.1f %.1f %.1f %.1f %.1f\n", g, w, a[0] / cnt, a[1] / cnt,
                             a[2] / cnt, a[3] / cnt, a[4] / cnt, a[5] / cnt);
            }
    }
    // per-wave counters of sequence 0 and of the sequence whose sweep ends last
    uint32_t qlast = 0;
    unsigned long long elast = 0;
    for (uint32_t q = 0; q < nseq; ++q)
        for (size_t w = 0; w < (size_t)plan.G * plan.W; ++w)
            if (h[((size_t)q * plan.G * plan.W + w) * kPipeStamps + 11] > elast) {
                elast = h[((size_t)q * plan.G * plan.W + w) * kPipeStamps + 11];
                qlast = q;
            }
    for (uint32_t q : {0u, qlast}) {
        for (uint32_t g = 0; g < plan.G; ++g)
            for (uint32_t w = 0; w < plan.W; ++w) {
                const unsigned long long* r = h.data() + (((size_t)q * plan.G + g) * plan.W + w) * kPipeStamps;
                std::fprintf(stderr, "  seq %u g%u w%u: loop %llu head %llu tail %llu prev %llu next %llu gran %llu cons %llu slow %llu\n",
                             q, g, w, r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[14]);
            }
        if (qlast == 0) break;
    }
}

void PipeScratchBuffers::ensure(uint32_t rows, uint32_t G, hipStream_t s) {
    if (!d_ctr.ptr) {
        d_ctr.alloc(kCtrWords * 4);
        hip_check(hipMemsetAsync(d_ctr.ptr, 0, kCtrWords * 4, s), "pipe counters");
    }
    if (view.ctr && rows <= view.rows && G <= view.G) return;
    rows = std::max(rows, view.rows);
    G = std::max(G, view.G);
    auto zeroed = [&](DeviceBuffer& d, size_t bytes) {
        d.alloc(bytes);
        hip_check(hipMemsetAsync(d.ptr, 0, d.bytes, s), "pipe scratch");
    };
    zeroed(d_done, (size_t)rows * 128);  // (one 128-byte line per row: diag.hip SVH_DIAG_DONE_STRIDE)
    zeroed(d_part, (size_t)rows * G * 16);
    zeroed(d_gran, (size_t)rows * std::max<uint32_t>(G - 1, 1) * kPipeGRing * 8);
    zeroed(d_cons, (size_t)rows * G * 8);
    zeroed(d_viol, (size_t)rows * 4);
    zeroed(d_xcc, (size_t)rows * G * 4);
    view.ctr = d_ctr.as<uint32_t>();
    view.done = d_done.as<uint32_t>();
    view.part = d_part.as<uint64_t>();
    view.gran = d_gran.as<uint64_t>();
    view.cons = d_cons.as<uint32_t>();
    view.viol = d_viol.as<uint32_t>();
    view.xcc = d_xcc.as<uint32_t>();
    view.rows = rows;
    view.G = G;
}

void PipeScratchBuffers::note_launch(hipStream_t s) {
    if (launches > 0 && launches % kEpochSpan == 0) {
        hip_check(hipMemsetAsync(d_ctr.ptr, 0, d_ctr.bytes, s), "pipe epoch reset");
        hip_check(hipMemsetAsync(d_gran.ptr, 0, d_gran.bytes, s), "pipe epoch reset");
        hip_check(hipMemsetAsync(d_cons.ptr, 0, d_cons.bytes, s), "pipe epoch reset");
        hip_check(hipMemsetAsync(d_xcc.ptr, 0, d_xcc.bytes, s), "pipe epoch reset");
    }
    ++launches;
}

void DeviceBandPlan::report_stamps(uint32_t nseq) const {
    if (!(view.dbg & (4u | 128u)) || !view.stamps) return;
    std::vector<unsigned long long> h((size_t)nseq * kMaxWaves * kBandStamps);
    if (hipMemcpy(h.data(), view.stamps, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    double sum[kBandStamps] = {};
    uint32_t cnt = 0;
    for (uint32_t q = 0; q < nseq; ++q)
        for (uint32_t w = 0; w < std::max<uint32_t>(plan.B / 64, 1); ++w, ++cnt)
            for (int k = 0; k < kBandStamps; ++k) sum[k] += (double)h[((size_t)q * kMaxWaves + w) * kBandStamps + k];
    std::fprintf(stderr, "band stamps (avg cycles per wave over the launch):");
    for (int k = 0; k < kBandStamps; ++k) std::fprintf(stderr, " s%d=%.0f", k, sum[k] / cnt);
    std::fprintf(stderr, "\n");
}

// ------------------------------------------------------------------------------------------
// Model
// ------------------------------------------------------------------------------------------
void DevicePlan::upload(const Plan& p, hipStream_t s) {
    plan = p;
    if (!p.fused) return;
    d_emis.upload(p.emis_pad.data(), p.emis_pad.size() * 4, s);
    d_start.upload(p.start_pad.data(), p.start_pad.size() * 4, s);
    d_lcol.upload(p.lcol.data(), p.lcol.size() * 4, s);
    d_lval.upload(p.lval.data(), p.lval.size() * 4, s);
    d_hval.upload(p.hval.data(), p.hval.size() * 4, s);
    d_hvalid.upload(p.hvalid.data(), p.hvalid.size(), s);
    d_hmask.upload(p.hmask.data(), p.hmask.size() * 4, s);
    std::memset(&view, 0, sizeof(view));
    view.emis = d_emis.as<float>();
    view.start = d_start.as<float>();
    view.lcol = d_lcol.as<uint32_t>();
    view.lval = d_lval.as<float>();
    view.hval = d_hval.as<float>();
    view.hvalid = d_hvalid.as<uint8_t>();
    view.hmask = d_hmask.as<float>();
    for (int h = 0; h < kMaxHeavy; ++h) {
        view.hrow[h] = p.hrow[h];
        view.hw[h] = p.hw[h];
        for (int x = 0; x < kMaxExc; ++x) {
            view.xk[h][x] = p.xk[h][x];
            view.xw[h][x] = p.xw[h][x];
        }
    }
    view.H = p.H;
    view.slots = p.SM;
    view.estride = p.estride;
    view.vstride = p.vstride;
    view.B = p.B;
}

Model::Model(const HostModel& h, const svh_model_opts* opts) : host(h) {
    int dev = opts ? opts->device : -1;
    if (dev < 0) hip_check(hipGetDevice(&dev), "hipGetDevice");
    device = dev;
    kernel_pref = opts ? opts->kernel : SVH_KERNEL_AUTO;
    if (kernel_pref < SVH_KERNEL_AUTO || (kernel_pref > SVH_KERNEL_PIPE_WIDE && kernel_pref != SVH_KERNEL_DIAG))
        throw Error(SVH_E_INVALID, "kernel must be one of SVH_KERNEL_AUTO .. SVH_KERNEL_PIPE_WIDE or SVH_KERNEL_DIAG");
    if (opts && (opts->flags & ~SVH_MODEL_SPEC_DENSE))
        throw Error(SVH_E_INVALID, "unknown svh_model_opts.flags bits");
    spec_dense = opts && (opts->flags & SVH_MODEL_SPEC_DENSE);
    // 0 = each planner's default; the fused kernel caps at kMaxFusedThreads, the chain kernel at
    // kMaxBandThreads.
    const int max_threads = (opts && opts->max_threads > 0) ? opts->max_threads : 0;
    if (max_threads % 64 != 0 || max_threads > std::max(kMaxFusedThreads, kMaxBandThreads))
        throw Error(SVH_E_INVALID, "max_threads must be 0 or a multiple of 64 in [64, 1024]");
    DeviceGuard g(device);
    hip_check(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "hipStreamCreate");

    if (kernel_pref == SVH_KERNEL_AUTO || kernel_pref == SVH_KERNEL_BAND || kernel_pref == SVH_KERNEL_CHAIN ||
        kernel_pref == SVH_KERNEL_PIPE || kernel_pref == SVH_KERNEL_PIPE_WIDE || kernel_pref == SVH_KERNEL_DIAG) {
        BandPlan bpl;
        if (kernel_pref != SVH_KERNEL_BAND) bpl = make_band_plan(host, max_threads, true);
        if (!bpl.ok && kernel_pref != SVH_KERNEL_CHAIN) bpl = make_band_plan(host, max_threads, false);
        if (kernel_pref != SVH_KERNEL_AUTO && !bpl.ok)
            throw Error(SVH_E_UNSUPPORTED, "chain kernel requested but the model is not chain-shaped "
                                           "(or too large / too many symbols for it)");
        // pipelined plan (its fallback is the chain / band plan above); SVH_PIPE=0 disables it
        const char* pipe_env = std::getenv("SVH_PIPE");
        if (bpl.ok && !(pipe_env && std::atoi(pipe_env) == 0)) {
            const PipePlan ppl = make_pipe_plan(host);
            if (ppl.ok) pipe.upload(ppl, host.n, host.S, stream);
        }
        if (bpl.ok && pipe.plan.ok && !(std::getenv("SVH_PIPEW") && std::atoi(std::getenv("SVH_PIPEW")) == 0)) {
            const PipePlan wpl = make_pipe_plan(host, 0, 0, true);
            if (wpl.ok) {
                pipe_wide.upload(wpl, host.n, host.S, stream);
                int cus = 0;
                hip_check(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device), "CU count");
                pipe_wide.view.cus = (uint32_t)cus;
            }
        }
        if (((kernel_pref == SVH_KERNEL_PIPE || kernel_pref == SVH_KERNEL_DIAG) && !pipe.plan.ok) ||
            (kernel_pref == SVH_KERNEL_DIAG && !pipe.view.dtab) || (kernel_pref == SVH_KERNEL_PIPE_WIDE && !pipe_wide.plan.ok))
            throw Error(SVH_E_UNSUPPORTED, "pipelined kernel requested but the model does not qualify (chain shape "
                                           "with one heavy row feeding the light rows, emit_num <= 32)");
        band.upload(bpl, host.n, host.S, stream);
        // wide batches: the 8-wave E-in-VGPR geometry holds one workgroup per CU; 4 waves with
        // streamed E fit two, which doubles throughput once every CU is busy
        if (bpl.ok && bpl.chain && !bpl.ge && bpl.B >= 512) {
            BandPlan wide = make_band_plan(host, 0, true, 4);
            if (wide.ok) band_wide.upload(wide, host.n, host.S, stream);
        }
        int cus = 0;
        hip_check(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device), "CU count");
        cu_count = (uint32_t)cus;
        if (pipe.plan.ok) pipe.view.cus = cu_count;  // latency plan: the XCD-class mapping's residency test
        if (pipe.plan.ok) {
            // AUTO: scores-only batches take the latency plan while they give every CU at most two
            // of its workgroups (two waves per SIMD: the scores kernel's 232 VGPRs fit twice;
            // 2405 x 100 sequences 0.323 ms against 0.427 on the wide plan, 150 sequences 0.574
            // against 0.429, profiles/r05_s10); decoded-path batches while they give every CU at most
            // one (the path kernel's 290 registers fit once); wider batches run the wide pipelined plan
            // (DESIGN.md 5c), or the chain kernel where the model has none; SVH_PIPE_MAX_NSEQ
            // overrides the scores-only bound
            pipe_max_nseq = std::max<uint32_t>(1, 2 * cu_count / pipe.plan.G);
            pipe_max_nseq_paths = std::max<uint32_t>(1, cu_count / pipe.plan.G);
            if (const char* e = std::getenv("SVH_PIPE_MAX_NSEQ")) pipe_max_nseq = (uint32_t)std::atoi(e);
            // diagonal plan (diag.hip): the scores-only batches the latency plan would take (DESIGN.md
            // 5l); SVH_DIAG=0 disables it, SVH_DIAG_MAX_NSEQ overrides the bound
            if (pipe.view.dtab && !(std::getenv("SVH_DIAG") && std::atoi(std::getenv("SVH_DIAG")) == 0)) {
                // while its whole grid is resident at two workgroups per CU (its LDS allows two):
                // beyond that the latency plan's two-per-CU regime is faster (2405.chmm: 52 sequences;
                // at 64 the diagonal plan takes 0.296 ms against 0.303, at 90 0.363 against 0.313,
                // profiles/r06_diag/widths.log)
                const uint32_t w = diag_waves_for(4);
                diag_max_nseq = std::min<uint32_t>(pipe_max_nseq, w * (2 * cu_count / pipe.plan.nrng));
                if (const char* e = std::getenv("SVH_DIAG_MAX_NSEQ")) diag_max_nseq = (uint32_t)std::atoi(e);
            }
        }
        if (pipe_wide.plan.ok) {
            // AUTO: the wide pipelined plan for batches beyond the latency plan's range
            pipew_min_nseq = pipe_max_nseq + 1;
            if (const char* e = std::getenv("SVH_PIPEW_MIN_NSEQ")) pipew_min_nseq = (uint32_t)std::atoi(e);
        }
    }
    Plan fast = make_plan(host, max_threads, true);
    fast_plan.upload(fast, stream);
    if (fast.fused) {
        fast_plan.view.n = host.n;
        fast_plan.view.S = host.S;
    }
    if (fast.fused && fast.mode == kHeavyUniform) {
        Plan gen = make_plan(host, max_threads, false);
        paths_plan_storage.upload(gen, stream);
        if (gen.fused) {
            paths_plan_storage.view.n = host.n;
            paths_plan_storage.view.S = host.S;
        }
        paths_plan = &paths_plan_storage;
    } else {
        paths_plan = &fast_plan;
    }

    std::vector<uint32_t> row_of(host.nnz());
    for (uint32_t j = 0; j < host.n; ++j)
        for (uint32_t p = host.rowptr[j]; p < host.rowptr[j + 1]; ++p) row_of[p] = j;
    d_gemis.upload(host.emis.data(), host.emis.size() * 4, stream);
    d_gstart.upload(host.start.data(), host.start.size() * 4, stream);
    d_rowptr.upload(host.rowptr.data(), host.rowptr.size() * 4, stream);
    d_col.upload(host.col.data(), host.col.size() * 4, stream);
    d_val.upload(host.val.data(), host.val.size() * 4, stream);
    d_rowof.upload(row_of.data(), row_of.size() * 4, stream);
    hip_check(hipStreamSynchronize(stream), "model upload");
    if (kernel_pref == SVH_KERNEL_FUSED && !fast.fused)
        throw Error(SVH_E_UNSUPPORTED, "fused kernel requested but no fused family fits this model");
    if (!fast.fused && generic_lds_bytes(host.n) > kMaxLdsBytes)
        throw Error(SVH_E_UNSUPPORTED, "model too large for the on-chip score vector");
}

Model::~Model() {
    if (stream) {
        (void)hipStreamSynchronize(stream);
        (void)hipStreamDestroy(stream);
    }
}

CsrModel Model::csr_view() const {
    CsrModel c;
    c.emis = d_gemis.as<float>();
    c.start = d_gstart.as<float>();
    c.rowptr = d_rowptr.as<uint32_t>();
    c.col = d_col.as<uint32_t>();
    c.val = d_val.as<float>();
    c.row_of = d_rowof.as<uint32_t>();
    c.n = host.n;
    c.S = host.S;
    c.nnz = host.nnz();
    return c;
}

const DeviceBandPlan* Model::band_for(bool paths, uint32_t nseq) const {
    if (!band.plan.ok) return nullptr;
    if (kernel_pref != SVH_KERNEL_AUTO && kernel_pref != SVH_KERNEL_BAND && kernel_pref != SVH_KERNEL_CHAIN &&
        kernel_pref != SVH_KERNEL_PIPE && kernel_pref != SVH_KERNEL_PIPE_WIDE && kernel_pref != SVH_KERNEL_DIAG)
        // PIPE*, DIAG: the chain plan is their fallback (paths, the _spec tail)
        return nullptr;
    if (paths) return band.plan.paths_ok() ? &band : nullptr;  // decoded-path chain variant
    if (band_wide.plan.ok && nseq > cu_count) return &band_wide;
    return &band;
}

const DevicePipePlan* Model::pipe_for(uint32_t nseq) const {
    if (kernel_pref == SVH_KERNEL_PIPE) return pipe.plan.ok ? &pipe : nullptr;
    if (kernel_pref == SVH_KERNEL_PIPE_WIDE) return pipe_wide.plan.ok ? &pipe_wide : nullptr;
    if (kernel_pref != SVH_KERNEL_AUTO) return nullptr;
    if (pipe.plan.ok && nseq <= pipe_max_nseq) return &pipe;
    if (pipe_wide.plan.ok && nseq >= pipew_min_nseq) return &pipe_wide;
    return nullptr;
}

const DevicePipePlan* Model::diag_for(uint32_t nseq) const {
    if (!pipe.plan.ok || !pipe.view.dtab) return nullptr;
    if (kernel_pref == SVH_KERNEL_DIAG) return &pipe;
    if (kernel_pref != SVH_KERNEL_AUTO) return nullptr;
    return nseq <= diag_max_nseq ? &pipe : nullptr;
}

// Decoded paths: the latency plan's path variant for the batches its scores pass takes, the wide
// plan's beyond that (the chain kernel's path variant is the exact fallback of both, so the model
// needs its plan too); SVH_PIPEW_PATHS=0 sends wide path batches to the chain kernel (A/B).
const DevicePipePlan* Model::pipe_paths_for(uint32_t nseq) const {
    if (!band.plan.paths_ok()) return nullptr;
    const bool lat = pipe.plan.ok && pipe_paths_supported((int)pipe.plan.SM, (int)pipe.plan.W) &&
                     pipe.plan.P <= kPipeTbMaxP;
    static const bool wide_env = !(std::getenv("SVH_PIPEW_PATHS") && std::atoi(std::getenv("SVH_PIPEW_PATHS")) == 0);
    const bool wid = wide_env && pipe_wide.plan.ok && pipe_wide.plan.P <= kPipeTbMaxP &&
                     pipew_paths_supported((int)pipe_wide.plan.SM, host.S, pipe_wide.plan.sx);
    if (kernel_pref == SVH_KERNEL_PIPE) return lat ? &pipe : nullptr;
    if (kernel_pref == SVH_KERNEL_PIPE_WIDE) return wid ? &pipe_wide : nullptr;
    if (kernel_pref != SVH_KERNEL_AUTO) return nullptr;
    if (lat && nseq <= pipe_max_nseq_paths) return &pipe;
    if (wid && nseq > pipe_max_nseq_paths) return &pipe_wide;
    return nullptr;
}

bool Model::pipe_l2_on() const {
    return spec2_on && pipe.plan.ok && pipe_l2_supported(pipe.view) &&
           (kernel_pref == SVH_KERNEL_AUTO || kernel_pref == SVH_KERNEL_PIPE);
}

const DevicePlan* Model::plan_for(bool paths) const {
    if (kernel_pref == SVH_KERNEL_GENERIC) return nullptr;
    const DevicePlan* p = paths ? paths_plan : &fast_plan;
    return (p && p->plan.fused) ? p : nullptr;
}

// ------------------------------------------------------------------------------------------
// _spec level 2 on chip (spec2.hip).  Light rows (<= kSpec2LightMax terms) keep their terms in the
// registers of thread r % 1024, slot r / 1024; heavy rows' terms are spread over the threads in row
// order.  amax[h] bounds every finite a = fl(E_s[j] + T^T[j][p]) that meets heavy row p = hrow[h]
// in a chunk (the candidate pruning's bound); prune only when every score is >= 0.
// ------------------------------------------------------------------------------------------
Spec2Plan make_spec2_plan(const HostModel& hm) {
    Spec2Plan sp;
    const uint32_t n = hm.n, S = hm.S, T = kSpec2Threads;
    if (n == 0 || n > 65535 || n > 4 * T) return sp;
    std::vector<int32_t> hid(n, -1);
    uint32_t klmax = 1;
    std::vector<uint32_t> deg;
    for (uint32_t r = 0; r < n; ++r) {
        const uint32_t d = hm.rowptr[r + 1] - hm.rowptr[r];
        if (d > kSpec2LightMax) {
            hid[r] = (int32_t)sp.hrow.size();
            sp.hrow.push_back(r);
            deg.push_back(d);
        } else {
            klmax = std::max(klmax, d);
        }
    }
    const uint32_t H = (uint32_t)sp.hrow.size();
    if (H + 2 > T) return sp;
    // heavy terms per thread: the fewest (<= 8) whose padded rows fit the 1024 threads
    uint32_t nhs = 0;
    for (uint32_t c = 1; c <= 8 && !nhs; ++c) {
        uint64_t threads = 0;
        for (uint32_t d : deg) threads += (d + c - 1) / c;
        if (threads <= T) nhs = c;
    }
    if (H && !nhs) return sp;
    if (!nhs) nhs = 1;
    sp.nhs = nhs;
    sp.R = spec2_round_r((n + T - 1) / T);
    sp.KL = spec2_round_kl(klmax);
    sp.NHS = spec2_round_nhs(nhs);
    if (!sp.R || !sp.KL || !sp.NHS) return sp;
    std::vector<uint32_t> cpoff(H + 1, 0);  // candidate range of each heavy row (its padded term count)
    for (uint32_t h = 0; h < H; ++h) cpoff[h + 1] = cpoff[h] + (deg[h] + nhs - 1) / nhs * nhs;
    sp.NP = cpoff[H];
    const Spec2Lds L = spec2_lds_layout(n, sp.KL, sp.NP, H);
    if (L.bytes > kMaxLdsBytes || n * sp.KL + sp.NP >= (1u << 20)) return sp;
    sp.H = H;
    // the two words of a term whose column is m (spec2.hip): score address, pair list
    const uint32_t pad_a = L.v + n, pad_b = (H + 1) << 20;
    auto word_a = [&](uint32_t m) { return hid[m] < 0 ? L.v + m : (L.hacc + (uint32_t)hid[m]) | 0x80000000u; };
    auto word_b = [&](uint32_t m) {
        return hid[m] < 0 ? (m * sp.KL) | (H << 20) : (n * sp.KL + cpoff[hid[m]]) | ((uint32_t)hid[m] << 20);
    };
    sp.la.assign((size_t)sp.R * sp.KL * T, pad_a);
    sp.lb.assign((size_t)sp.R * sp.KL * T, pad_b);
    sp.lv.assign((size_t)sp.R * sp.KL * T, kInfH);
    for (uint32_t r = 0; r < n; ++r) {
        if (hid[r] >= 0) continue;
        const uint32_t s = r / T, t = r % T;
        for (uint32_t e = hm.rowptr[r], k = 0; e < hm.rowptr[r + 1]; ++e, ++k) {
            const size_t i = ((size_t)s * sp.KL + k) * T + t;
            sp.la[i] = word_a(hm.col[e]);
            sp.lb[i] = word_b(hm.col[e]);
            sp.lv[i] = hm.val[e];
        }
    }
    sp.thr.assign(T, H);
    sp.tcp.assign(T, 0);
    sp.ha.assign((size_t)T * sp.NHS, pad_a);
    sp.hb.assign((size_t)T * sp.NHS, pad_b);
    sp.hv.assign((size_t)T * sp.NHS, kInfH);
    uint32_t t = 0;
    for (uint32_t h = 0; h < H; ++h) {
        const uint32_t r = sp.hrow[h];
        for (uint32_t e = hm.rowptr[r], k = 0; e < hm.rowptr[r + 1]; ++e, ++k) {
            const uint32_t tt = t + k / nhs, hs = k % nhs;
            const size_t i = (size_t)tt * sp.NHS + hs;
            sp.ha[i] = word_a(hm.col[e]);
            sp.hb[i] = word_b(hm.col[e]);
            sp.hv[i] = hm.val[e];
        }
        const uint32_t nt = (deg[h] + nhs - 1) / nhs;
        for (uint32_t k = 0; k < nt; ++k) {
            sp.thr[t + k] = h;
            sp.tcp[t + k] = n * sp.KL + cpoff[h];
        }
        t += nt;
    }
    // a of the terms (j, p) with p heavy, over every symbol: fl(E_s[j] + T^T[j][p]) (float adds)
    sp.amax.assign(H, 0.0f);
    bool nonneg = true;
    for (uint32_t j = 0; j < n; ++j)
        for (uint32_t e = hm.rowptr[j]; e < hm.rowptr[j + 1]; ++e) {
            nonneg = nonneg && hm.val[e] >= 0.0f;
            const int32_t h = hid[hm.col[e]];
            if (h < 0) continue;
            for (uint32_t o = 0; o < S; ++o) {
                const float a = hm.emis[(size_t)o * n + j] + hm.val[e];
                if (a < kInfH) sp.amax[h] = std::max(sp.amax[h], a);
            }
        }
    for (float e : hm.emis) nonneg = nonneg && e >= 0.0f;
    for (float e : hm.start) nonneg = nonneg && e >= 0.0f;
    sp.prune = nonneg;
    if (H == 0) {  // no heavy rows: one padding entry each, so every upload has a source
        sp.hrow.push_back(0);
        sp.amax.push_back(0.0f);
    }
    sp.ok = true;
    return sp;
}

void DeviceSpec2Plan::upload(const Spec2Plan& p, const HostModel& hm, const float* d_emis, hipStream_t s) {
    plan = p;
    std::memset(&view, 0, sizeof(view));
    if (!p.ok) return;
    d_la.upload(p.la.data(), p.la.size() * 4, s);
    d_lb.upload(p.lb.data(), p.lb.size() * 4, s);
    d_lv.upload(p.lv.data(), p.lv.size() * 4, s);
    d_thr.upload(p.thr.data(), p.thr.size() * 4, s);
    d_tcp.upload(p.tcp.data(), p.tcp.size() * 4, s);
    d_ha.upload(p.ha.data(), p.ha.size() * 4, s);
    d_hb.upload(p.hb.data(), p.hb.size() * 4, s);
    d_hv.upload(p.hv.data(), p.hv.size() * 4, s);
    d_hrow.upload(p.hrow.data(), p.hrow.size() * 4, s);
    d_amax.upload(p.amax.data(), p.amax.size() * 4, s);
    view.emis = d_emis;
    view.la = d_la.as<uint32_t>();
    view.lb = d_lb.as<uint32_t>();
    view.lv = d_lv.as<float>();
    view.thr = d_thr.as<uint32_t>();
    view.tcp = d_tcp.as<uint32_t>();
    view.ha = d_ha.as<uint32_t>();
    view.hb = d_hb.as<uint32_t>();
    view.hv = d_hv.as<float>();
    view.hrow = d_hrow.as<uint32_t>();
    view.amax = d_amax.as<float>();
    view.n = hm.n;
    view.S = hm.S;
    view.H = p.H;
    view.NP = p.NP;
    view.R = p.R;
    view.KL = p.KL;
    view.NHS = p.NHS;
    view.nhs = p.nhs;
    view.prune = p.prune ? 1u : 0u;
    if (const char* e = std::getenv("SVH_SPEC2_DEBUG"); e && std::atoi(e)) {  // diagnostics only
        d_stamps.alloc((size_t)4096 * 16 * kSpec2Stamps * 8);
        hip_check(hipMemsetAsync(d_stamps.ptr, 0, d_stamps.bytes, s), "stamps");
        view.stamps = d_stamps.as<unsigned long long>();
    }
}

void DeviceSpec2Plan::report_stamps(uint32_t nseq) const {
    if (!view.stamps) return;
    nseq = std::min<uint32_t>(nseq, 4096);
    std::vector<unsigned long long> h((size_t)nseq * 16 * kSpec2Stamps);
    if (hipMemcpy(h.data(), view.stamps, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    double sum[kSpec2Stamps] = {};
    double chunks = 0;
    for (uint32_t q = 0; q < nseq; ++q)
        for (uint32_t w = 0; w < 16; ++w) {
            const unsigned long long* r = h.data() + ((size_t)q * 16 + w) * kSpec2Stamps;
            for (int k = 0; k < 7; ++k) sum[k] += (double)r[k];
            chunks += (double)r[7];
        }
    if (chunks <= 0) return;
    std::fprintf(stderr, "spec2 cycles per chunk and wave (s_memtime): phase1 %.0f bar1 %.0f phase1b %.0f bar2 %.0f "
                         "phase2 %.0f bar3 %.0f loop %.0f (%.0f chunks x waves)\n",
                 sum[0] / chunks, sum[1] / chunks, sum[2] / chunks, sum[3] / chunks, sum[4] / chunks, sum[5] / chunks,
                 sum[6] / chunks, chunks);
}

void Model::spec_build(uint32_t level, hipStream_t s) {
    std::lock_guard<std::mutex> lock(mu);
    DeviceGuard g(device);
    if (!s) s = stream;
    d_products = DeviceBuffer();
    spec_level = 0;
    spec2_on = false;
    if (level <= 1) {
        spec_level = level;
        return;
    }
    // level 2: the on-chip kernel when the model fits it (no products: the chunks are evaluated
    // from the folded sparse matrices, spec2.hip); SVH_SPEC_DENSE=1 streams the dense products (A/B)
    static const bool dense_env = std::getenv("SVH_SPEC_DENSE") && std::atoi(std::getenv("SVH_SPEC_DENSE")) == 1;
    if (level == 2 && !dense_env && !spec_dense) {
        if (!spec2.plan.ok) {
            const Spec2Plan sp = make_spec2_plan(host);
            if (sp.ok) {
                spec2.upload(sp, host, d_gemis.as<float>(), s);
                hip_check(hipStreamSynchronize(s), "spec2 plan upload");
            }
        }
        if (spec2.plan.ok) {
            spec2_on = true;
            spec_level = level;
            return;
        }
    }
    const CsrModel c = csr_view();
    if (host.n > 65535) throw Error(SVH_E_UNSUPPORTED, "_spec level >= 2 needs states_num <= 65535");
    pstride = (host.n + 3) & ~3u;
    const uint64_t mat = (uint64_t)host.n * pstride;
    uint64_t keys = host.S;
    for (uint32_t l = 2; l <= level; ++l) {
        keys *= host.S;
        if (keys / host.S > 65535 / ((host.S + 31) / 32))
            throw Error(SVH_E_UNSUPPORTED, "_spec level too high for the precompute grid");
    }
    const uint64_t final_bytes = keys * mat * 4;
    const uint64_t prev_bytes = (keys / host.S) * mat * 4;
    size_t free_b = 0, total_b = 0;
    hip_check(hipMemGetInfo(&free_b, &total_b), "hipMemGetInfo");
    if (final_bytes + prev_bytes + (64ull << 20) > free_b)
        throw Error(SVH_E_NOMEM, "_spec products need " + std::to_string(final_bytes + prev_bytes) +
                                     " bytes of HBM, " + std::to_string(free_b) + " free");
    d_mfold.alloc((size_t)host.nnz() * host.S * 4);
    hip_check(launch_spec_fold(c, d_mfold.as<float>(), s), "spec fold");
    DeviceBuffer prev;
    prev.alloc((size_t)host.S * mat * 4);
    hip_check(launch_spec_densify(c, d_mfold.as<float>(), prev.as<float>(), pstride, s), "spec densify");
    uint64_t kprev = host.S;
    for (uint32_t l = 2; l <= level; ++l) {
        DeviceBuffer next;
        next.alloc((size_t)(kprev * host.S * mat * 4));
        hip_check(launch_spec_extend(c, d_mfold.as<float>(), prev.as<float>(), kprev,
                                     next.as<float>(), pstride, s),
                  "spec extend");
        hip_check(hipStreamSynchronize(s), "spec extend");
        prev = std::move(next);
        kprev *= host.S;
    }
    d_products = std::move(prev);
    spec_level = level;
}

svh_model_info Model::info(uint32_t nseq, bool paths, uint32_t level) const {
    svh_model_info i;
    std::memset(&i, 0, sizeof(i));
    const bool steps = level <= 1 || spec_level < 2;  // level >= 2 runs only the tail on step kernels
    const DevicePlan* p = plan_for(paths && steps);
    const DeviceBandPlan* bpl = band_for(paths && steps, nseq);
    i.kernel = bpl ? (bpl->plan.chain ? SVH_KERNEL_CHAIN : SVH_KERNEL_BAND) : p ? SVH_KERNEL_FUSED : SVH_KERNEL_GENERIC;
    // the pipelined plan runs scores-only passes, the step-kernel tail of _spec level >= 2 and
    // (latency plan) decoded-path passes of small batches
    const DevicePipePlan* ppl = !nseq ? nullptr : !paths ? pipe_for(nseq) : steps ? pipe_paths_for(nseq) : nullptr;
    i.family = p ? p->plan.family : -1;
    i.threads = p ? (int32_t)p->plan.B : (int32_t)std::min<uint32_t>(1024, round_up(host.n, 64));
    i.slots = p ? (int32_t)p->plan.SM : 0;
    i.light_terms = p ? (int32_t)p->plan.R : 0;
    i.heavy_rows = p ? (int32_t)p->plan.H : 0;
    i.heavy_uniform = (p && p->plan.mode == kHeavyUniform) ? 1 : 0;
    i.device = device;
    i.n = host.n;
    i.S = host.S;
    i.nnz = host.nnz();
    i.lds_bytes = p ? p->plan.lds_bytes : generic_lds_bytes(host.n);
    if (bpl) {
        i.threads = (int32_t)bpl->plan.B;
        i.slots = (int32_t)bpl->plan.SM;
        i.light_terms = (int32_t)bpl->plan.HA + 1;
        i.heavy_rows = (int32_t)bpl->plan.H;
        i.heavy_uniform = 1;
        i.lds_bytes = bpl->plan.chain ? chain_lds_bytes() : bpl->plan.lds_bytes;
    }
    i.spec_level = spec_level;
    i.spec_bytes = d_products.bytes;
    const DevicePipePlan* pp1 = pipe_paths_for(1);
    i.paths_kernel = pp1 ? (pp1->plan.wide ? SVH_KERNEL_PIPE_WIDE : SVH_KERNEL_PIPE)
                     : band_for(true) ? SVH_KERNEL_CHAIN : plan_for(true) ? SVH_KERNEL_FUSED : SVH_KERNEL_GENERIC;
    i.wide_threads = band_wide.plan.ok && band_for(false) ? (int32_t)band_wide.plan.B : 0;
    i.wide_slots = band_wide.plan.ok && band_for(false) ? (int32_t)band_wide.plan.SM : 0;
    i.cu_count = cu_count;
    if (ppl) {
        uint32_t w = ppl->plan.wide ? pipew_waves_for(ppl->view, nseq) : ppl->plan.W;
        if (ppl->plan.wide && paths) w = std::min(w, pipew_paths_waves_max(ppl->plan.SM, host.S, ppl->plan.sx));
        i.kernel = ppl->plan.wide ? SVH_KERNEL_PIPE_WIDE : SVH_KERNEL_PIPE;
        i.threads = (int32_t)(64 * w);
        i.slots = (int32_t)ppl->plan.SM;
        i.lds_bytes = ppl->plan.wide ? pipew_lds_bytes(ppl->plan.SM, w, host.S, ppl->plan.sx, paths)
                                     : pipe_lds_bytes(ppl->plan.W, host.S);
    }
    if (pipe_wide.plan.ok) {
        i.pipew_slots = (int32_t)pipe_wide.plan.SM;
        i.pipew_waves = (int32_t)pipe_wide.plan.W;
        i.pipew_blocks = (int32_t)pipe_wide.plan.G;
        i.pipew_min_nseq = kernel_pref == SVH_KERNEL_PIPE_WIDE ? 0u
                           : kernel_pref == SVH_KERNEL_AUTO    ? pipew_min_nseq
                                                               : 0xFFFFFFFFu;
    }
    if (pipe.plan.ok) {
        i.pipe_slots = (int32_t)pipe.plan.SM;
        i.pipe_waves = (int32_t)pipe.plan.W;
        i.pipe_groups = (int32_t)pipe.plan.G;
        i.pipe_max_nseq = kernel_pref == SVH_KERNEL_PIPE ? 0xFFFFFFFFu : pipe_max_nseq;
        i.pipe_max_nseq_paths = kernel_pref == SVH_KERNEL_PIPE ? 0xFFFFFFFFu : pipe_max_nseq_paths;
    }
    if (!paths && steps && level <= 1 && nseq && diag_for(nseq)) {  // scores on the diagonal plan
        const uint32_t w = diag_waves_for(nseq);
        i.kernel = SVH_KERNEL_DIAG;
        i.threads = (int32_t)(64 * w);
        i.slots = 1;
        i.lds_bytes = diag_lds_bytes(w, host.S, pipe.plan.P);
    }
    if (pipe.view.dtab) {
        i.diag_ranges = (int32_t)pipe.plan.nrng;
        i.diag_max_nseq = kernel_pref == SVH_KERNEL_DIAG ? 0xFFFFFFFFu : kernel_pref == SVH_KERNEL_AUTO ? diag_max_nseq : 0u;
    }
    if (level == 2 && spec_level == 2 && nseq && pipe_l2_on()) {  // the chunks on the pipelined plan
        i.kernel = SVH_KERNEL_SPEC2_PIPE;
        i.threads = (int32_t)(64 * pipe.plan.W);
        i.slots = (int32_t)pipe.plan.SM;
        i.lds_bytes = pipe_lds_bytes(pipe.plan.W, host.S);
        i.spec_bytes = 0;
    } else if (level == 2 && spec_level == 2 && spec2_on && nseq) {  // the chunks run on chip (spec2.hip)
        const Spec2Plan& sp = spec2.plan;
        i.kernel = SVH_KERNEL_SPEC2;
        i.threads = (int32_t)kSpec2Threads;
        i.slots = 0;
        i.light_terms = (int32_t)sp.KL;
        i.heavy_rows = (int32_t)sp.H;
        i.lds_bytes = spec2_lds_layout(host.n, sp.KL, sp.NP, sp.H).bytes;
        i.spec_bytes = spec2.d_la.bytes + spec2.d_lb.bytes + spec2.d_lv.bytes + spec2.d_thr.bytes + spec2.d_tcp.bytes +
                       spec2.d_ha.bytes + spec2.d_hb.bytes + spec2.d_hv.bytes + spec2.d_hrow.bytes + spec2.d_amax.bytes;
    }
    return i;
}

// ------------------------------------------------------------------------------------------
// Batches
// ------------------------------------------------------------------------------------------
Batch::Batch(Model* m, uint64_t nseq_, const uint64_t* offs, const uint64_t* symbols, uint32_t flags)
    : model(m) {
    init(flags);
    load(nseq_, offs, symbols, nullptr, m->stream);
    hip_check(hipStreamSynchronize(m->stream), "batch upload");
}

Batch::Batch(Model* m, uint64_t nseq_, const uint64_t* offs, const uint8_t* symbols, uint32_t flags)
    : model(m) {
    init(flags);
    load(nseq_, offs, nullptr, symbols, m->stream);
    hip_check(hipStreamSynchronize(m->stream), "batch upload");
}

void Batch::init(uint32_t flags) {
    paths = (flags & SVH_BATCH_PATHS) != 0;
    chain_paths = paths && model->band_for(true) != nullptr;
    if (paths && !chain_paths && model->host.n >= kNoPred)
        throw Error(SVH_E_UNSUPPORTED, "paths need states_num < 65535 for models the chain kernel does not cover");
    timing = (flags & SVH_BATCH_NO_TIMING) == 0;
    DeviceGuard g(model->device);
    if (timing) {
        hip_check(hipEventCreate(&ev_start), "hipEventCreate");
        hip_check(hipEventCreate(&ev_stop), "hipEventCreate");
    }
}

// (Re)load the batch's sequences: host packing, then asynchronous uploads on `s` into device
// buffers that only ever grow (no hipFree / hipMalloc, hence no device-wide sync, once sized).
// The host staging arrays are members, so they outlive the copies until the next load.
void Batch::load(uint64_t nseq_, const uint64_t* offs, const uint64_t* sym64, const uint8_t* sym8,
                 hipStream_t s, const uint64_t* const* seqp) {
    if (nseq_ == 0) throw Error(SVH_E_INVALID, "empty batch");
    if (nseq_ > 0x7FFFFFFFull) throw Error(SVH_E_UNSUPPORTED, "too many sequences in one batch");
    if (!offs || (!sym64 && !sym8 && !seqp)) throw Error(SVH_E_INVALID, "null offsets/symbols");
    if (seqp)
        for (uint64_t q = 0; q < nseq_; ++q)
            if (!seqp[q] && offs[q + 1] > offs[q]) throw Error(SVH_E_INVALID, "null sequence pointer");
    const DeviceBandPlan* cpl = chain_paths ? model->band_for(true) : nullptr;
    nseq = (uint32_t)nseq_;
    const DevicePipePlan* ppl = chain_paths ? model->pipe_paths_for(nseq) : nullptr;
    pipe_paths = ppl != nullptr;
    offsets.assign(offs, offs + nseq + 1);
    lens.resize(nseq);
    h_symoff.resize(nseq);
    h_pathoff.resize(nseq);
    h_bpoff.resize(nseq);
    h_cmoff.resize(nseq);
    h_hroff.resize(nseq);
    h_ckoff.resize(nseq);
    h_pmoff.resize(pipe_paths ? nseq : 0);
    h_proff.resize(pipe_paths ? nseq : 0);
    h_pcoff.resize(pipe_paths ? nseq : 0);
    h_fcoff.resize(pipe_paths ? nseq : 0);
    uint64_t bytes = 0, bpn = 0, cmn = 0, hrn = 0, ckn = 0, pmn = 0, prn = 0, pcn = 0, fcn = 0;
    for (uint32_t q = 0; q < nseq; ++q) {
        if (offs[q + 1] < offs[q]) throw Error(SVH_E_INVALID, "offsets must be non-decreasing");
        const uint64_t len = offs[q + 1] - offs[q];
        if (len == 0)
            throw Error(SVH_E_INVALID, "empty observation sequence (reference: seq[0] is undefined)");
        if (len > 0xFFFFFF00ull) throw Error(SVH_E_UNSUPPORTED, "sequence too long");
        lens[q] = (uint32_t)len;
        h_symoff[q] = bytes;
        bytes += ((len + kSymPad + 4 + 15) / 16) * 16;
        if (cpl) {
            h_cmoff[q] = cmn;
            cmn += chain_mask_words(len, cpl->plan.B / 64, cpl->plan.SM);
            h_hroff[q] = hrn;
            hrn += chain_hrec_words(len);
            h_ckoff[q] = ckn;
            ckn += chain_ckpt_floats(len, cpl->plan.SM, cpl->plan.B);
            if (ppl) {
                h_pmoff[q] = pmn;
                pmn += pipe_mask_words(len, ppl->plan.nblk, ppl->plan.SM);
                h_proff[q] = prn;
                prn += pipe_prec_count(len, ppl->plan.nblk, pipe_prec_parts(ppl->plan.wide));
                h_pcoff[q] = pcn;
                pcn += pipe_ckpt_floats(len, ppl->plan.P);
                h_fcoff[q] = fcn;
                fcn += pipe_fck_floats(len);
            }
        } else if (paths) {
            h_bpoff[q] = bpn;
            bpn += (len - 1) * (uint64_t)model->host.n;
        }
        h_pathoff[q] = offs[q] - offs[0];
    }
    total = offs[nseq] - offs[0];
    DeviceGuard g(model->device);
    // Every input table of the batch -- symbols, then the per-sequence offset / begin / end
    // tables -- in one pinned staging arena and one asynchronous upload into one device arena
    // (separate pageable copies each cost a staging round trip; the symbols are converted from
    // the caller's uint64 straight into pinned memory).  The staging arena is reused by the next
    // load, which always follows the completion of this batch's previous run.
    struct Section {
        size_t off = 0, bytes = 0;
    };
    size_t in_bytes = 0;
    auto section = [&](size_t nb) {
        Section x;
        x.off = in_bytes;
        x.bytes = nb;
        in_bytes += (nb + 15) & ~(size_t)15;
        return x;
    };
    const Section s_sym = section(bytes), s_symoff = section((size_t)nseq * 8), s_begin = section((size_t)nseq * 4),
                  s_end = section((size_t)nseq * 4);
    const bool cp = paths && chain_paths, pp = cp && pipe_paths, fp = paths && !chain_paths;
    const Section s_path = section(paths ? (size_t)nseq * 8 : 0), s_cm = section(cp ? (size_t)nseq * 8 : 0),
                  s_hr = section(cp ? (size_t)nseq * 8 : 0), s_ck = section(cp ? (size_t)nseq * 8 : 0),
                  s_pm = section(pp ? (size_t)nseq * 8 : 0), s_pr = section(pp ? (size_t)nseq * 8 : 0),
                  s_pc = section(pp ? (size_t)nseq * 8 : 0), s_fc = section(pp ? (size_t)nseq * 8 : 0),
                  s_bp = section(fp ? (size_t)nseq * 8 : 0);
    static const bool trace = std::getenv("SVH_TRACE_ONESHOT") && std::atoi(std::getenv("SVH_TRACE_ONESHOT"));
    const auto tl0 = std::chrono::steady_clock::now();
    uint8_t* const hin = h_in.reserve(in_bytes);
    const uint64_t S = model->host.S;
    for (uint32_t q = 0; q < nseq; ++q) {
        uint8_t* dstp = hin + s_sym.off + h_symoff[q];
        const uint32_t L = lens[q];
        const uint64_t base = offs[q];
        // narrow into pinned staging; the range check is a branch-free OR the loop vectorises,
        // the error path re-scans for the offending symbol
        if (sym64 || seqp) {
            // (restrict: a uint8_t store may alias anything, which kept the loop byte-serial)
            const uint64_t* __restrict__ src = seqp ? seqp[q] : sym64 + base;
            uint8_t* __restrict__ d = dstp;
            uint64_t bad = 0;
            for (uint32_t i = 0; i < L; ++i) {
                const uint64_t x = src[i];
                bad |= x >= S ? 1u : 0u;
                d[i] = (uint8_t)x;
            }
            if (bad)
                for (uint32_t i = 0; i < L; ++i)
                    if (src[i] >= S)
                        throw Error(SVH_E_RANGE, "symbol " + std::to_string(src[i]) +
                                                     " out of range (emit_num " + std::to_string(S) + ")");
        } else {
            // the device format already: one memcpy, then a range check the compiler vectorises (a
            // byte loop that copies and checks ran at ~4 GB/s: 43 us for the headline's 175 KB)
            const uint8_t* __restrict__ src = sym8 + base;
            std::memcpy(dstp, src, L);
            uint8_t mx = 0;
            for (uint32_t i = 0; i < L; ++i) mx = src[i] > mx ? src[i] : mx;
            const uint32_t bad = mx >= S ? 1u : 0u;
            if (bad)
                for (uint32_t i = 0; i < L; ++i)
                    if (src[i] >= S)
                        throw Error(SVH_E_RANGE, "symbol " + std::to_string(src[i]) + " out of range (emit_num " +
                                                     std::to_string(S) + ")");
        }
        // zero padding after the sequence (kSymPad and the 16-byte round-up)
        const uint64_t end = q + 1 < nseq ? h_symoff[q + 1] : bytes;
        std::memset(dstp + L, 0, end - h_symoff[q] - L);
    }
    auto put = [&](const Section& x, const void* src) {
        if (x.bytes) std::memcpy(hin + x.off, src, x.bytes);
    };
    put(s_symoff, h_symoff.data());
    std::memset(hin + s_begin.off, 0, s_begin.bytes);
    put(s_end, lens.data());
    put(s_path, h_pathoff.data());
    put(s_cm, h_cmoff.data());
    put(s_hr, h_hroff.data());
    put(s_ck, h_ckoff.data());
    put(s_pm, h_pmoff.data());
    put(s_pr, h_proff.data());
    put(s_pc, h_pcoff.data());
    put(s_fc, h_fcoff.data());
    put(s_bp, h_bpoff.data());
    const auto tl1 = std::chrono::steady_clock::now();
    d_in.reserve(in_bytes);
    hip_check(hipMemcpyAsync(d_in.ptr, hin, in_bytes, hipMemcpyHostToDevice, s), "batch inputs H2D");
    if (trace) {
        const auto tl2 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "load trace (us): pack %.1f h2d-enqueue %.1f (%zu bytes)\n",
                     std::chrono::duration<double, std::micro>(tl1 - tl0).count(),
                     std::chrono::duration<double, std::micro>(tl2 - tl1).count(), in_bytes);
    }
    uint8_t* const din = d_in.as<uint8_t>();
    p_sym = din + s_sym.off;
    p_symoff = reinterpret_cast<uint64_t*>(din + s_symoff.off);
    p_begin = reinterpret_cast<uint32_t*>(din + s_begin.off);
    p_end = reinterpret_cast<uint32_t*>(din + s_end.off);
    auto u64p = [&](const Section& x) { return x.bytes ? reinterpret_cast<uint64_t*>(din + x.off) : nullptr; };
    p_pathoff = u64p(s_path);
    p_cmoff = u64p(s_cm);
    p_hroff = u64p(s_hr);
    p_ckoff = u64p(s_ck);
    p_pmoff = u64p(s_pm);
    p_proff = u64p(s_pr);
    p_pcoff = u64p(s_pc);
    p_fcoff = u64p(s_fc);
    p_bpoff = u64p(s_bp);
    // results: fault word | best states | scores, one device arena (read() copies it at once); a
    // grown arena starts with a clear fault word
    const size_t best_off = 16, score_off = best_off + (((size_t)nseq * 8 + 15) & ~(size_t)15);
    const size_t out_bytes = score_off + (size_t)nseq * model->host.n * 4;
    if (!d_out.ptr || out_bytes > d_out.bytes) {
        d_out.alloc(out_bytes);
        hip_check(hipMemsetAsync(d_out.ptr, 0, 16, s), "fault word");
    }
    p_fault = d_out.as<uint32_t>();
    p_best = reinterpret_cast<int64_t*>(d_out.as<uint8_t>() + best_off);
    p_scores = reinterpret_cast<float*>(d_out.as<uint8_t>() + score_off);
    if (cp) {
        d_cmask.reserve((size_t)std::max<uint64_t>(cmn, 1) * 4);
        d_hrec.reserve((size_t)std::max<uint64_t>(hrn, kRecWords) * 4);
        d_ckpt.reserve((size_t)std::max<uint64_t>(ckn, 1) * 4);
        if (pp) {
            d_pmask.reserve((size_t)std::max<uint64_t>(pmn, 1) * 4);
            d_prec.reserve((size_t)std::max<uint64_t>(prn, 1) * 8);
            d_pck.reserve((size_t)std::max<uint64_t>(pcn, 1) * 4);
            d_fck.reserve((size_t)std::max<uint64_t>(fcn, 1) * 4);
        }
    } else if (fp) {
        d_bp.reserve((size_t)std::max<uint64_t>(bpn, 1) * 2);
    }
    if (paths) d_paths.reserve((size_t)std::max<uint64_t>(total, 1) * 4);
    spec_ready_level = 0;
    ran = false;
    pipe_ran = false;
}

Batch::~Batch() {
    DeviceGuard g(model->device);
    if (ev_start) (void)hipEventDestroy(ev_start);
    if (ev_stop) (void)hipEventDestroy(ev_stop);
}

void Batch::run(uint32_t level, hipStream_t s) {
    std::lock_guard<std::mutex> lock(model->mu);
    DeviceGuard g(model->device);
    if (!s) s = model->stream;
    if (paths && level >= 2)
        throw Error(SVH_E_UNSUPPORTED, "decoded paths are defined for the per-observation recurrence (level <= 1)");
    if (level >= 2 && model->spec_level != level)
        throw Error(SVH_E_STATE, "run at _spec level " + std::to_string(level) +
                                     " needs svh_spec_build(" + std::to_string(level) + ") first");
    const CsrModel csr = model->csr_view();
    FusedBatch fb;
    std::memset(&fb, 0, sizeof(fb));
    fb.symbols = p_sym;
    fb.sym_off = p_symoff;
    fb.begin = p_begin;
    fb.end = p_end;
    fb.scores = p_scores;
    fb.best = p_best;
    fb.fault = p_fault;
    fb.nseq = nseq;
    if (paths && chain_paths) {
        fb.cmask = d_cmask.as<uint32_t>();
        fb.cmask_off = p_cmoff;
        fb.hrec = d_hrec.as<uint32_t>();
        fb.hrec_off = p_hroff;
        fb.ckpt = d_ckpt.as<float>();
        fb.ckpt_off = p_ckoff;
    } else if (paths) {
        fb.bp = d_bp.as<uint16_t>();
        fb.bp_off = p_bpoff;
    }
    pipe_ran = false;
    l2_ran = false;
    // (level >= 2: the chunks run elsewhere; the tail, rows resumed from the chunks' scores, runs on
    // the diagonal plan when it has one for this batch -- the scratch then covers both plans)
    const DevicePipePlan* dp = paths ? nullptr : model->diag_for(nseq);
    if (dp && level <= 1) {  // diagonal plan: scratch
        pipe.ensure(nseq, dp->plan.nrng, s);
        fb.pipe = &pipe.view;
        pipe_ran = true;
    } else if (const DevicePipePlan* pp = paths ? nullptr : model->pipe_for(nseq)) {  // pipelined plan: scratch
        pipe.ensure(nseq, std::max<uint32_t>(pp->plan.G, dp ? dp->plan.nrng : 0u), s);
        pipe.note_launch(s);
        fb.pipe = &pipe.view;
        pipe_ran = dp || model->band_for(false, nseq) != nullptr;  // launch_steps' condition
    } else if (dp) {
        pipe.ensure(nseq, dp->plan.nrng, s);
        fb.pipe = &pipe.view;
        pipe_ran = true;
    }
    auto launch_step_kernel = [&](const FusedBatch& b, bool want_paths) { model->launch_steps(b, want_paths, s); };

    last_stream = s;
    if (timing) hip_check(hipEventRecord(ev_start, s), "hipEventRecord");
    if (level <= 1 && pipe_paths) {
        // decoded paths on the pipelined plan: its path variant, the chain path variant for rows
        // whose speculation failed, the pipelined traceback (unflagged rows), the chain traceback
        // (flagged rows)
        const DevicePipePlan* ppl = model->pipe_paths_for(nseq);
        const DeviceBandPlan* bpl = model->band_for(true);
        if (!ppl || !bpl) throw Error(SVH_E_STATE, "batch planned for pipelined paths, model has no such plan");
        pipe.ensure(nseq, ppl->plan.G, s);
        pipe.note_launch(s);
        FusedBatch pb = fb;
        pb.cmask = d_pmask.as<uint32_t>();
        pb.cmask_off = p_pmoff;
        pb.ckpt = d_pck.as<float>();
        pb.ckpt_off = p_pcoff;
        pb.prec = d_prec.as<float2>();
        pb.prec_off = p_proff;
        pb.fck = d_fck.as<float>();
        pb.fck_off = p_fcoff;
        pb.pipe = &pipe.view;
        if (ppl->plan.wide) hip_check(launch_pipew(ppl->view, pb, pipe.view, s), "wide pipelined Viterbi kernel (paths)");
        else hip_check(launch_pipe(ppl->view, pb, pipe.view, s), "pipelined Viterbi kernel (paths)");
        FusedBatch cb = fb;  // chain buffers
        cb.run_mask = pipe.view.viol;
        hip_check(launch_chain(bpl->view, 1, cb, s), "chain Viterbi kernel (pipe paths fallback)");
        // SVH_PIPE_SKIP_TRACEBACK=1: diagnostic builds only (-DSVH_PIPE_DIAG; timing of the forward
        // kernels alone, e.g. of an ablation build whose path records are not stored; the paths read
        // back are wrong).  The production library has no such knob.
#ifdef SVH_PIPE_DIAG
        static const bool skip_tb = std::getenv("SVH_PIPE_SKIP_TRACEBACK") && std::atoi(std::getenv("SVH_PIPE_SKIP_TRACEBACK"));
#else
        constexpr bool skip_tb = false;
#endif
        if (!skip_tb) {
            hip_check(launch_pipe_traceback(ppl->view, pb, p_pathoff, d_paths.as<int32_t>(),
                                            pipe.view.viol, s),
                      "pipelined traceback kernel");
            hip_check(launch_chain_traceback(bpl->view, cb, p_pathoff, d_paths.as<int32_t>(), s),
                      "chain traceback kernel (pipe paths fallback)");
        }
        pipe_ran = true;
    } else if (level <= 1) {
        launch_step_kernel(fb, paths);
        if (paths && chain_paths)
            hip_check(launch_chain_traceback(model->band_for(true)->view, fb, p_pathoff,
                                             d_paths.as<int32_t>(), s),
                      "chain traceback kernel");
        else if (paths)
            hip_check(launch_traceback(fb, p_pathoff, d_paths.as<int32_t>(), model->host.n, s),
                      "traceback kernel");
    } else {
        const uint32_t n = model->host.n;
        const bool on_chip = level == 2 && model->spec2_on;
        // level 2 on the pipelined latency plan (pipe_l2.hip): every chunk of every row in one
        // launch into the second half of vbuf; rows whose speculation fails run again on spec2_kernel
        // from the first step's state (first half) into the second half; the tail reads row nseq + q
        const bool l2pipe = on_chip && model->pipe_l2_on();
        const uint32_t ready = level | (on_chip ? 0x100u : 0u) | (l2pipe ? 0x200u : 0u);
        if (spec_ready_level != ready) {
            std::vector<uint32_t> nch(nseq), tb(nseq), vrow(nseq);
            for (uint32_t q = 0; q < nseq; ++q) {
                nch[q] = (lens[q] - 1) / level;
                tb[q] = 1 + nch[q] * level;
                vrow[q] = l2pipe ? nseq + q : on_chip ? q : (nch[q] & 1u) * nseq + q;  // the row the chunks end in
            }
            if (l2pipe) d_l2viol.alloc((size_t)nseq * 4);
            d_nchunks.upload(nch.data(), nch.size() * 4, s);
            d_tbegin.upload(tb.data(), tb.size() * 4, s);
            d_vrow.upload(vrow.data(), vrow.size() * 4, s);
            d_vbuf.alloc((size_t)2 * nseq * n * 4);
            hip_check(hipStreamSynchronize(s), "spec batch setup");
            max_chunks = 0;
            for (uint32_t q = 0; q < nseq; ++q) max_chunks = std::max(max_chunks, nch[q]);
            spec_ready_level = ready;
        }
        float* vb = d_vbuf.as<float>();
        hip_check(launch_first_step(csr, fb.symbols, fb.sym_off, nseq, vb, s), "spec first step");
        if (l2pipe) {
            const DevicePipePlan& pl = model->pipe;
            pipe.ensure(nseq, pl.plan.G, s);
            pipe.note_launch(s);
            PipeScratch x2 = pipe.view;
            x2.viol = d_l2viol.as<uint32_t>();  // its own flags: the tail's pass rewrites pipe.view.viol
            FusedBatch lb = fb;
            lb.scores = vb + (size_t)nseq * n;
            lb.best = nullptr;
            lb.pipe = nullptr;
            hip_check(launch_pipe_l2(pl.view, lb, x2, s), "pipelined level-2 kernel");
            l2_ran = true;
        }
        if (on_chip) {  // every chunk of every sequence in one launch, v in place (row q)
            Spec2Batch sb;
            sb.symbols = fb.symbols;
            sb.sym_off = fb.sym_off;
            sb.len = p_end;
            sb.nchunks = d_nchunks.as<uint32_t>();
            sb.v = vb;
            sb.nseq = nseq;
            if (l2pipe) {  // only the rows the pipelined pass flagged, into the second half
                sb.run_mask = d_l2viol.as<uint32_t>();
                sb.v_out = vb + (size_t)nseq * n;
            }
            hip_check(launch_spec2(model->spec2.view, sb, s), "spec2 kernel");
            if (model->spec2.view.stamps) {
                hip_check(hipStreamSynchronize(s), "spec2 stamps");
                model->spec2.report_stamps(nseq);
            }
        }
        SpecChunkBatch cb;
        cb.symbols = fb.symbols;
        cb.sym_off = fb.sym_off;
        cb.nchunks = d_nchunks.as<uint32_t>();
        cb.nseq = nseq;
        cb.level = level;
        for (uint32_t c = 0; c < (on_chip ? 0u : max_chunks); ++c) {
            cb.chunk = c;
            cb.v_src = vb + (size_t)(c & 1u) * nseq * n;
            cb.v_dst = vb + (size_t)((c + 1) & 1u) * nseq * n;
            hip_check(launch_spec_chunk(csr, model->d_products.as<float>(), cb, model->pstride, s),
                      "spec chunk kernel");
        }
        FusedBatch tail = fb;
        tail.begin = d_tbegin.as<uint32_t>();
        tail.v_in = vb;
        tail.v_in_row = d_vrow.as<uint32_t>();
        tail.bp = nullptr;
        tail.bp_off = nullptr;
        launch_step_kernel(tail, false);
    }
    if (timing) hip_check(hipEventRecord(ev_stop, s), "hipEventRecord");
    ran = true;
}

// ------------------------------------------------------------------------------------------
// Time-parallel run (opt-in, scores within rounding of the serial run).
//   Sequence q of length L > 2*seg is cut into segments [b_k, e_k) of >= seg observations.
//   1a  every segment k >= 1 runs its first `probe` observations from the guess (all zeros),
//       segment 0 from the start column (exact) -> G
//   1b  the rest of every segment continues from G -> E1 (all segments of all sequences at
//       once: this is where the idle CUs go)
//   2   for k = 1, 2, ...: segment k's probe from the exact start (the corrected end of k-1)
//       -> X; if X - G is constant (within tol) the end is E1 + that constant, else the rest of
//       the segment runs from X (exact; counted in *fallbacks)
// The per-segment runs are ordinary step-kernel launches over a view of the batch (begin/end/
// v_in per row); only the check/correction and the finish are kernels of their own.
// ------------------------------------------------------------------------------------------
void Batch::run_time_parallel(uint32_t seg, uint32_t probe, float tol, hipStream_t s, uint64_t* fallbacks) {
    std::lock_guard<std::mutex> lock(model->mu);
    DeviceGuard g(model->device);
    if (!s) s = model->stream;
    if (paths) throw Error(SVH_E_UNSUPPORTED, "time-parallel runs compute scores only (no decoded paths)");
    if (seg < 2 || probe < 1 || probe >= seg)
        throw Error(SVH_E_INVALID, "time-parallel run needs seg >= 2 and 1 <= probe < seg");
    if (tol != tol) throw Error(SVH_E_INVALID, "tolerance is NaN");  // tol < 0: re-run every segment (exact)
    pipe_ran = false;  // this pass never uses the pipelined kernel (svh_batch_fallbacks reports 0)
    const uint32_t n = model->host.n;
    struct Seg {
        uint32_t q, k, b, e;
    };
    std::vector<Seg> segs;
    std::vector<uint32_t> nsegs(nseq), first_seg(nseq);
    uint32_t kmax = 1;
    for (uint32_t q = 0; q < nseq; ++q) {
        const uint32_t L = lens[q];
        // P equal segments of at least seg observations (the longest bounds the parallel phase)
        const uint32_t P = L > 2 * seg ? L / seg : 1;
        first_seg[q] = (uint32_t)segs.size();
        nsegs[q] = P;
        kmax = std::max(kmax, P);
        for (uint32_t k = 0; k < P; ++k)
            segs.push_back({q, k, (uint32_t)((uint64_t)k * L / P), (uint32_t)((uint64_t)(k + 1) * L / P)});
    }
    const uint32_t nv = (uint32_t)segs.size();
    // basis rows: the heavy rows of the model's band plan (none for other models).  Every segment
    // runs nb guesses: the light guess (zeros, basis rows +inf), then a unit vector per basis row.
    TpBasis basis{};
    if (const DeviceBandPlan* bpl = model->band_for(false))
        for (int x = 0; x < kBandHeavy; ++x)
            if (bpl->plan.hvalid[x]) basis.hrow[basis.H++] = bpl->plan.hrow[x];
    const uint32_t nb = 1 + basis.H;
    // device scratch (freed at return)
    DeviceBuffer d_zero, d_G, d_E1, d_X, d_P, d_S, d_Y, d_vbest, d_flag;
    std::vector<float> guess((size_t)nb * n, 0.0f);
    for (uint32_t b = 0; b < basis.H; ++b) {
        guess[basis.hrow[b]] = kInfH;
        std::fill(guess.begin() + (size_t)(b + 1) * n, guess.begin() + (size_t)(b + 2) * n, kInfH);
        guess[(size_t)(b + 1) * n + basis.hrow[b]] = 0.0f;
    }
    d_zero.upload_async(guess.data(), guess.size() * 4, s);
    d_G.reserve((size_t)nv * nb * n * 4);
    d_E1.reserve((size_t)nv * nb * n * 4);
    d_X.reserve((size_t)2 * nv * n * 4);
    d_P.reserve((size_t)2 * nseq * n * 4);
    d_S.reserve((size_t)nseq * n * 4);
    d_Y.reserve((size_t)nv * n * 4);
    d_vbest.reserve((size_t)2 * nv * nb * 8);
    uint32_t nflags = 0;
    DeviceBuffer d_fbeg, d_fend, d_arena;
    d_fbeg.reserve((size_t)nv * 4);
    d_fend.reserve((size_t)nv * 4);
    d_flag.reserve((size_t)nv * 4);
    // Every row table of the run (sequence offsets, begin / end / v_in rows, correction rows) is
    // packed into one host arena first and the device work recorded as operations on the arena's
    // device copy; then one upload and the operations back to back, so the timed region carries
    // no per-table allocation or copy (the launch sequence itself waits for nothing: the
    // fallbacks' begin / end come from the device).
    std::vector<uint8_t> arena;
    std::vector<std::function<void(const uint8_t*)>> ops;  // argument: the arena's device base
    constexpr size_t kNone = ~(size_t)0;
    auto put = [&](const void* p, size_t bytes) -> size_t {
        const size_t off = (arena.size() + 15) & ~(size_t)15;
        arena.resize(off + std::max<size_t>(bytes, 1));
        if (bytes) std::memcpy(arena.data() + off, p, bytes);
        return off;
    };
    auto table32 = [&](std::vector<uint32_t>& v) -> size_t {
        const size_t off = put(v.data(), v.size() * 4);
        v.clear();
        return off;
    };
    auto at32 = [](const uint8_t* base, size_t off) { return reinterpret_cast<const uint32_t*>(base + off); };
    std::vector<uint64_t> vsym;
    std::vector<uint32_t> vbeg, vend, vrow;
    // One launch of the step kernel over rows (begin, end, v_in row) of the batch's sequences;
    // begin/end may instead come from the device (fallbacks).
    auto launch_rows = [&](const float* v_in, float* out, const uint32_t* dbeg = nullptr,
                           const uint32_t* dend = nullptr) {
        const uint32_t rows = (uint32_t)vsym.size();
        if (rows == 0) return;
        const size_t osym = put(vsym.data(), (size_t)rows * 8);
        vsym.clear();
        const size_t ob = dbeg ? kNone : table32(vbeg);
        const size_t oe = dend ? kNone : table32(vend);
        const size_t orow = table32(vrow);
        vbeg.clear();
        vend.clear();
        const uint8_t* sym = p_sym;
        int64_t* vbest = d_vbest.as<int64_t>();
        uint32_t* fault = p_fault;
        Model* mdl = model;
        ops.push_back([=](const uint8_t* base) {
            FusedBatch fb;
            std::memset(&fb, 0, sizeof(fb));
            fb.symbols = sym;
            fb.sym_off = reinterpret_cast<const uint64_t*>(base + osym);
            fb.begin = dbeg ? dbeg : at32(base, ob);
            fb.end = dend ? dend : at32(base, oe);
            fb.v_in = v_in;
            fb.v_in_row = at32(base, orow);
            fb.scores = out;
            fb.best = vbest;
            fb.fault = fault;
            fb.nseq = rows;
            mdl->launch_steps(fb, false, s);
        });
    };
    // 1a: probes from the guesses, rows v * nb + b (segment 0: from the start column, and its
    // basis rows are unused zero-step copies)
    for (const Seg& x : segs) {
        for (uint32_t b = 0; b < nb; ++b) {
            const bool unused = x.k == 0 && b > 0;
            vsym.push_back(h_symoff[x.q]);
            vbeg.push_back(unused ? 1u : x.k == 0 ? 0u : x.b);
            vend.push_back(unused ? 1u : std::min(x.b + probe, x.e));
            vrow.push_back(b);
        }
    }
    launch_rows(d_zero.as<float>(), d_G.as<float>());
    // 1b: the rest of every segment (a zero-step row copies its start)
    for (uint32_t v = 0; v < nv; ++v) {
        const Seg& x = segs[v];
        for (uint32_t b = 0; b < nb; ++b) {
            const bool unused = x.k == 0 && b > 0;
            vsym.push_back(h_symoff[x.q]);
            vbeg.push_back(unused ? 1u : std::min(x.b + probe, x.e));
            vend.push_back(unused ? 1u : x.e);
            vrow.push_back(v * nb + b);
        }
    }
    launch_rows(d_G.as<float>(), d_E1.as<float>());
    float* const S_ = d_S.as<float>();
    float* const P_ = d_P.as<float>();
    float* const X_ = d_X.as<float>();
    float* const Y_ = d_Y.as<float>();
    const float* const G_ = d_G.as<float>();
    const float* const E1_ = d_E1.as<float>();
    // S[q] = end of segment 0 (exact)
    {
        std::vector<uint32_t> irow(nseq), orow(nseq);
        for (uint32_t q = 0; q < nseq; ++q) {
            irow[q] = first_seg[q] * nb;
            orow[q] = q;
        }
        const size_t di = table32(irow), dout = table32(orow);
        const uint32_t ns = nseq;
        ops.push_back([=](const uint8_t* base) {
            hip_check(launch_tp_copy_rows(E1_, at32(base, di), S_, at32(base, dout), ns, n, nullptr, s),
                      "time-parallel copy");
        });
    }
    // 2: segments 1, 2, ... in order, all sequences at once.  The correction kernel decides on
    // the device which segments are re-run: it writes each fallback row's (begin, end), a
    // converged segment's row has no steps, and only flagged rows are copied into S.
    uint32_t* const fbeg_ = d_fbeg.as<uint32_t>();
    uint32_t* const fend_ = d_fend.as<uint32_t>();
    for (uint32_t k = 1; k < kmax; ++k) {
        std::vector<uint32_t> act;  // virtual segment ids of segment k
        for (uint32_t q = 0; q < nseq; ++q)
            if (nsegs[q] > k) act.push_back(first_seg[q] + k);
        if (act.empty()) break;
        const uint32_t na = (uint32_t)act.size();
        // probes from the exact start S[q] -> X rows 0..na-1, and (with basis rows) from its light
        // part -> X rows na..2na-1
        {
            const uint32_t ns = nseq;
            ops.push_back([=](const uint8_t*) {
                hip_check(launch_tp_probe_starts(S_, P_, ns, n, basis, s), "time-parallel starts");
            });
        }
        std::vector<uint32_t> rx(na), rg(na), re(na), ro(na), rf(na), rp(na), rs(na);
        for (uint32_t part = 0; part < (basis.H ? 2u : 1u); ++part) {
            for (uint32_t a = 0; a < na; ++a) {
                const Seg& x = segs[act[a]];
                vsym.push_back(h_symoff[x.q]);
                vbeg.push_back(x.b);
                vend.push_back(std::min(x.b + probe, x.e));
                vrow.push_back(part * nseq + x.q);
                rx[a] = a;
                rg[a] = act[a] * nb;
                re[a] = act[a] * nb;
                ro[a] = x.q;
                rf[a] = x.b + probe >= x.e ? 1u : 0u;
                rp[a] = std::min(x.b + probe, x.e);
                rs[a] = x.e;
            }
        }
        launch_rows(P_, X_);
        std::vector<uint32_t> ya(na);
        for (uint32_t a = 0; a < na; ++a) ya[a] = a;
        const size_t o_rx = table32(rx), o_rg = table32(rg), o_re = table32(re), o_ro = table32(ro),
                     o_rf = table32(rf), o_rp = table32(rp), o_rs = table32(rs);
        uint32_t* const flag = d_flag.as<uint32_t>() + nflags;
        ops.push_back([=](const uint8_t* base) {
            const TpRows tr{at32(base, o_rx), at32(base, o_rg), at32(base, o_re), at32(base, o_ro),
                            at32(base, o_rf), at32(base, o_rp), at32(base, o_rs)};
            hip_check(launch_tp_correct(X_, G_, E1_, tr, na, basis.H ? na : 0, basis, S_, n, tol, flag, fbeg_,
                                        fend_, s),
                      "time-parallel correction");
        });
        // fallbacks: the rest of each flagged segment from X, exactly, into Y, then into S
        for (uint32_t a = 0; a < na; ++a) {
            const Seg& x = segs[act[a]];
            vsym.push_back(h_symoff[x.q]);
            vrow.push_back(a);
        }
        launch_rows(X_, Y_, fbeg_, fend_);
        const size_t o_ya = table32(ya);
        ops.push_back([=](const uint8_t* base) {
            hip_check(launch_tp_copy_rows(Y_, at32(base, o_ya), S_, at32(base, o_ro), na, n, flag, s),
                      "time-parallel copy");
        });
        nflags += na;
    }
    {
        int64_t* const best_ = p_best;
        float* const scores_ = p_scores;
        const uint32_t ns = nseq;
        ops.push_back([=](const uint8_t*) {
            hip_check(launch_tp_finish(S_, scores_, best_, ns, n, s), "time-parallel finish");
        });
    }
    d_arena.reserve(arena.size());
    last_stream = s;
    if (timing) hip_check(hipEventRecord(ev_start, s), "hipEventRecord");
    hip_check(hipMemcpyAsync(d_arena.ptr, arena.data(), arena.size(), hipMemcpyHostToDevice, s), "time-parallel rows");
    const uint8_t* const base = d_arena.as<uint8_t>();
    for (auto& op : ops) op(base);
    if (timing) hip_check(hipEventRecord(ev_stop, s), "hipEventRecord");
    std::vector<uint32_t> flags(nflags);
    if (nflags)
        hip_check(hipMemcpyAsync(flags.data(), d_flag.ptr, (size_t)nflags * 4, hipMemcpyDeviceToHost, s), "flags D2H");
    hip_check(hipStreamSynchronize(s), "time-parallel run");
    check_fault(s);
    uint64_t nfall = 0;
    for (uint32_t f : flags) nfall += f;
    if (fallbacks) *fallbacks = nfall;
    ran = true;
}

// Page-locked host memory (hipHostMalloc / hipHostRegister): the DMA engine can write it directly.
static bool is_pinned_host(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory reports an error on some runtimes: clear it
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

void Batch::read(hipStream_t s, float* scores, int64_t* best, int32_t* paths_out) {
    DeviceGuard g(model->device);
    if (!s) s = model->stream;
    if (!ran) throw Error(SVH_E_STATE, "svh_batch_read before svh_batch_run");
    if (paths_out && !paths) throw Error(SVH_E_STATE, "batch was created without SVH_BATCH_PATHS");
    // the fault word, best states and scores (one device arena: one copy) and the paths into
    // pinned staging on the run's stream, one synchronisation, then out to the caller (pageable
    // copies would each block on their own)
    const size_t sb = scores ? (size_t)nseq * model->host.n * 4 : 0, bb = best ? (size_t)nseq * 8 : 0;
    const size_t best_off = (size_t)(reinterpret_cast<uint8_t*>(p_best) - d_out.as<uint8_t>());
    const size_t score_off = (size_t)(reinterpret_cast<uint8_t*>(p_scores) - d_out.as<uint8_t>());
    const size_t pre = sb ? score_off + sb : bb ? best_off + bb : 16;
    const size_t pb = paths_out ? (size_t)total * 4 : 0, path_off = (pre + 15) & ~(size_t)15;
    uint8_t* st = h_out.reserve(path_off + pb);
    // One copy, one synchronisation, then out to the caller.  (Four pieces with an event each, the
    // host copying one out while the next moved, were slower: 83 vs 42 us for the headline's 482 KB,
    // profiles/r04_s8/e2e_split.json.)  Page-locked destinations (svh_host_alloc) take the scores
    // and paths straight from the DMA engine: no staging, no copy-out.
    const bool sd = sb && is_pinned_host(scores), pd = pb && is_pinned_host(paths_out);
    const size_t pre_st = sd ? (bb ? best_off + bb : 16) : pre;  // staged part of the arena
    hip_check(hipMemcpyAsync(st, d_out.ptr, pre_st, hipMemcpyDeviceToHost, s), "results D2H");
    if (sd) hip_check(hipMemcpyAsync(scores, p_scores, sb, hipMemcpyDeviceToHost, s), "scores D2H");
    if (pb)
        hip_check(hipMemcpyAsync(pd ? reinterpret_cast<uint8_t*>(paths_out) : st + path_off, d_paths.ptr, pb,
                                 hipMemcpyDeviceToHost, s),
                  "paths D2H");
    hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    {
        uint32_t f;
        std::memcpy(&f, st, sizeof(f));
        report_fault(f, s);
    }
    if (sb && !sd) std::memcpy(scores, st + score_off, sb);
    if (bb) std::memcpy(best, st + best_off, bb);
    if (pb && !pd) std::memcpy(paths_out, st + path_off, pb);
}

void Batch::read_async(hipStream_t s, float* scores, int64_t* best, int32_t* paths_out) {
    DeviceGuard g(model->device);
    if (!ran) throw Error(SVH_E_STATE, "read before run");
    if (paths_out && !paths) throw Error(SVH_E_STATE, "batch was created without SVH_BATCH_PATHS");
    if (scores)
        hip_check(hipMemcpyAsync(scores, p_scores, (size_t)nseq * model->host.n * 4, hipMemcpyDeviceToHost, s),
                  "scores D2H");
    if (best) hip_check(hipMemcpyAsync(best, p_best, (size_t)nseq * 8, hipMemcpyDeviceToHost, s), "best D2H");
    if (paths_out)
        hip_check(hipMemcpyAsync(paths_out, d_paths.ptr, (size_t)total * 4, hipMemcpyDeviceToHost, s), "paths D2H");
}

// One pass of the per-observation step kernel over a batch view (steps begin..end-1 of each row).
void Model::launch_steps(const FusedBatch& b, bool want_paths, hipStream_t s) const {
    const DevicePlan* dp = plan_for(want_paths);
    const DeviceBandPlan* bpl = band_for(want_paths, b.nseq);
    const DevicePipePlan* dpl = want_paths ? nullptr : diag_for(b.nseq);
    if (dpl && b.pipe && b.pipe->rows >= b.nseq && b.pipe->G >= dpl->plan.nrng) {
        // diagonal plan: rows whose speculation fails are re-run in the same launch
        hip_check(launch_diag(dpl->view, b, *b.pipe, s), "diagonal Viterbi kernel");
        return;
    }
    const DevicePipePlan* ppl = want_paths ? nullptr : pipe_for(b.nseq);
    if (ppl && bpl && b.pipe && b.pipe->rows >= b.nseq && b.pipe->G >= ppl->plan.G) {
        if (ppl->plan.wide) hip_check(launch_pipew(ppl->view, b, *b.pipe, s), "wide pipelined Viterbi kernel");
        else hip_check(launch_pipe(ppl->view, b, *b.pipe, s), "pipelined Viterbi kernel");
        if (ppl->view.stamps && !ppl->plan.wide) {
            hip_check(hipStreamSynchronize(s), "stamps");
            ppl->report_stamps(b.nseq);
        }
        // rows whose speculation failed: the latency plan re-runs them itself (PipeModel::rerun:
        // no second launch on the common path); otherwise they run again on the serial chain
        // kernel (the others exit);
        // SVH_PIPE_SKIP_FALLBACK=1: diagnostic builds only (-DSVH_PIPE_DIAG; timing without the
        // second launch; results of flagged rows would be wrong)
#ifdef SVH_PIPE_DIAG
        static const bool skip_fb = std::getenv("SVH_PIPE_SKIP_FALLBACK") && std::atoi(std::getenv("SVH_PIPE_SKIP_FALLBACK"));
        if (skip_fb) return;
#endif
        if (!ppl->plan.wide && ppl->view.rerun) return;
        FusedBatch fb = b;
        fb.run_mask = b.pipe->viol;
        fb.pipe = nullptr;
        const int ha = (int)std::max<uint32_t>(bpl->plan.HA, 1);
        if (bpl->plan.chain) hip_check(launch_chain(bpl->view, ha, fb, s), "chain Viterbi kernel (pipe fallback)");
        else hip_check(launch_band(bpl->view, ha, fb, s), "band Viterbi kernel (pipe fallback)");
        return;
    }
    if (bpl) {
        const int ha = (int)std::max<uint32_t>(bpl->plan.HA, 1);
        if (bpl->plan.chain) hip_check(launch_chain(bpl->view, ha, b, s), "chain Viterbi kernel");
        else hip_check(launch_band(bpl->view, ha, b, s), "band Viterbi kernel");
        if (bpl->view.dbg & (4u | 128u)) {
            hip_check(hipStreamSynchronize(s), "stamps");
            bpl->report_stamps(b.nseq);
        }
    } else if (dp) {
        hip_check(launch_fused(dp->view, b, dp->plan.family, want_paths, s), "fused Viterbi kernel");
    } else {
        const uint32_t threads = std::min<uint32_t>(1024, ((host.n + 63) / 64) * 64);
        hip_check(launch_generic(csr_view(), b, (int)threads, want_paths, s), "generic Viterbi kernel");
    }
}

void Batch::check_fault(hipStream_t s) {
    DeviceGuard g(model->device);
    if (!s) s = model->stream;
    uint32_t* f = reinterpret_cast<uint32_t*>(h_out.reserve(16));
    hip_check(hipMemcpyAsync(f, p_fault, sizeof(uint32_t), hipMemcpyDeviceToHost, s), "fault D2H");
    hip_check(hipStreamSynchronize(s), "fault D2H");
    report_fault(*f, s);
}

void Batch::report_fault(uint32_t f, hipStream_t s) {
    if (!f) return;
    // reported once: clear the word (ordered on the stream of the run that set it) so this batch's
    // later runs are judged on their own; other batches have words of their own
    hip_check(hipMemsetAsync(p_fault, 0, sizeof(uint32_t), s), "fault reset");
    if (f & (kFaultPipe | kFaultPipeWide))
        throw Error(SVH_E_HIP, "pipelined kernel: a bounded wait gave up (results invalid)");
    throw Error(SVH_E_HIP, "chain kernel: a bounded inter-wave wait gave up (results invalid)");
}

void Batch::inject_fault(hipStream_t s) {
    DeviceGuard g(model->device);
    if (!s) s = model->stream;
    if (!ran) throw Error(SVH_E_STATE, "no run recorded");
    hip_check(hipMemsetAsync(p_fault, 0x01, 1, s), "fault inject");  // kFaultPipe
}

uint64_t Batch::pipe_fallbacks(uint32_t* rows) {
    DeviceGuard g(model->device);
    if (!ran) throw Error(SVH_E_STATE, "no run recorded");
    if (rows) std::memset(rows, 0, (size_t)nseq * 4);
    if (!pipe_ran && !l2_ran) return 0;
    if (timing) hip_check(hipEventSynchronize(ev_stop), "hipEventSynchronize");
    else hip_check(hipStreamSynchronize(last_stream), "hipStreamSynchronize");
    std::vector<uint32_t> v(nseq, 0), v2(nseq, 0);
    if (pipe_ran) hip_check(hipMemcpy(v.data(), pipe.view.viol, (size_t)nseq * 4, hipMemcpyDeviceToHost), "fallback flags D2H");
    // level 2 on the pipelined plan: its rows re-run by spec2_kernel count too
    if (l2_ran) hip_check(hipMemcpy(v2.data(), d_l2viol.ptr, (size_t)nseq * 4, hipMemcpyDeviceToHost), "fallback flags D2H");
    uint64_t c = 0;
    for (uint32_t q = 0; q < nseq; ++q) {
        c += (v[q] | v2[q]) != 0;
        if (rows) rows[q] = (v[q] ? 1u : 0u) | (v2[q] ? 2u : 0u);
    }
    return c;
}

float Batch::step_floor_ms(hipStream_t s, uint32_t reps) {
    std::lock_guard<std::mutex> lock(model->mu);
    DeviceGuard g(model->device);
    if (!s) s = model->stream;
    const DevicePipePlan* pp = model->pipe_for(nseq);
    if (!pp || pp->plan.wide || pp->view.tm != 4 || pp->plan.W != 4 || !model->band_for(false, nseq))
        throw Error(SVH_E_UNSUPPORTED, "step floor: the batch's plan is not the pipelined latency plan (TM 4)");
    floor_scratch.ensure(nseq, pp->plan.G, s);
    const size_t n = model->host.n;
    d_floor_out.reserve(16 + (size_t)nseq * n * 4);
    FusedBatch fb;
    std::memset(&fb, 0, sizeof(fb));
    fb.symbols = p_sym;
    fb.sym_off = p_symoff;
    fb.begin = p_begin;
    fb.end = p_end;
    fb.fault = d_floor_out.as<uint32_t>();
    fb.scores = reinterpret_cast<float*>(d_floor_out.as<uint8_t>() + 16);
    fb.nseq = nseq;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hip_check(hipEventCreate(&e0), "hipEventCreate");
    hip_check(hipEventCreate(&e1), "hipEventCreate");
    float ms = 0;
    try {
        floor_scratch.note_launch(s);
        hip_check(launch_pipe(pp->view, fb, floor_scratch.view, s, true), "step-floor kernel (warm-up)");
        hip_check(hipEventRecord(e0, s), "hipEventRecord");
        for (uint32_t r = 0; r < reps; ++r) {
            floor_scratch.note_launch(s);
            hip_check(launch_pipe(pp->view, fb, floor_scratch.view, s, true), "step-floor kernel");
        }
        hip_check(hipEventRecord(e1, s), "hipEventRecord");
        hip_check(hipEventSynchronize(e1), "hipEventSynchronize");
        hip_check(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
    } catch (...) {
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        throw;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return ms / (float)reps;
}

float Batch::elapsed_ms() {
    DeviceGuard g(model->device);
    if (!ran) throw Error(SVH_E_STATE, "no run recorded");
    if (!timing) throw Error(SVH_E_STATE, "batch created with SVH_BATCH_NO_TIMING: no run events");
    hip_check(hipEventSynchronize(ev_stop), "hipEventSynchronize");
    float ms = 0;
    hip_check(hipEventElapsedTime(&ms, ev_start, ev_stop), "hipEventElapsedTime");
    return ms;
}

}  // namespace svh
