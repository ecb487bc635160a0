// sdfa_wave_model.cpp -- probe (not product): where the sparse AC-DFA
// product kernel (dfa_sparse_lds_kernel<4, 32, KR, 1, 0, 8, 2>) spends its
// dependent global loads on the lines stream, per lane step and per WAVE step
// (64 lanes in lock step: a wave step waits for its slowest lane's chain of
// dependent loads).  Simulates real segments (SEG bytes each, synchronizing
// 3-gram warm-ups as dfa_sync_lo) over the real 8-B-unit image.
//   g++ -O2 -std=c++17 -Ipatternmatching_amd/csrc -Iinclude scripts/sdfa_wave_model.cpp \
//       patternmatching_amd/csrc/pm_flatten.cpp patternmatching_amd/csrc/host/pm_dict.c -o /tmp/wave && \
//   /tmp/wave tests/golden/data/snort.dict
// Env: KR (LDS rows, default 64), HOT (1: the KR most-visited rows instead of
// the first KR), WAVES (default 64), SEG (default 4096), PF (1: a sequential
// next-block load at a block end is counted as prefetched).
#include "pm_flatten.h"
#include "pm_streamgen.h"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <string>
#include <vector>
extern "C" size_t pm_parse_line(const unsigned char* line, size_t n, unsigned char* out);

static int envi(const char* k, int d) { const char* v = getenv(k); return v ? atoi(v) : d; }

int main(int argc, char** argv) {
    std::vector<std::string> pats;
    for (int a = 1; a < argc; ++a) {
        std::ifstream f(argv[a]);
        std::string line;
        std::vector<unsigned char> buf(1 << 16);
        while (std::getline(f, line)) {
            size_t k = pm_parse_line((const unsigned char*)line.data(), line.size(), buf.data());
            if (k) pats.emplace_back((char*)buf.data(), k);
        }
    }
    {
        std::vector<std::string> u;
        std::map<std::string, int> m;
        for (auto& p : pats)
            if (!m.count(p)) { m[p] = 1; u.push_back(p); }
        pats = u;
    }
    PmGidMap g = pm_assign_gids(pats);
    DfaImage d = pm_build_dfa(pats, g);
    std::vector<uint32_t> B8, O8;
    if (!pm_pack_sparse8(d, B8, O8)) { printf("no 8-B units\n"); return 1; }
    const uint32_t F = d.sF;
    size_t maxlen = 0;
    for (auto& p : pats) maxlen = std::max(maxlen, p.size());
    std::vector<uint32_t> g3((1u << 24) / 32, 0u);
    for (auto& p : pats)
        for (size_t i = 0; i + 3 <= p.size(); ++i) {
            const uint32_t x = (uint8_t)p[i] | (uint32_t)(uint8_t)p[i + 1] << 8 | (uint32_t)(uint8_t)p[i + 2] << 16;
            g3[x >> 5] |= 1u << (x & 31);
        }
    std::vector<uint8_t> P;
    std::vector<uint32_t> O(1, 0);
    for (auto& p : pats) { P.insert(P.end(), p.begin(), p.end()); O.push_back(P.size()); }
    const int KR = envi("KR", 64), WAVES = envi("WAVES", 64), SEG = envi("SEG", 4096), PF = envi("PF", 0);
    const int HOT = envi("HOT", 0);
    const int BU = envi("BU", 8);  // record units per register block (8 = 64 B)
    printf("patterns %zu states %u rows F=%u units %zu maxlen %zu | KR %d HOT %d WAVES %d SEG %d PF %d\n",
           pats.size(), d.states, F, B8.size() / 2 - (size_t)F * 128, maxlen, KR, HOT, WAVES, SEG, PF);
    const int LANES = 64 * WAVES;
    const uint64_t WARM = maxlen - 1;
    // each lane's text: its segment (at lane * SPREAD) plus the warm-up window
    const uint64_t SPREAD = (1ull << 30) / LANES;
    auto text_at = [&](uint64_t pos) {
        static uint64_t cb = ~0ull;
        static std::vector<uint8_t> blk(PM_LINES_BLOCK);
        const uint64_t b = pos / PM_LINES_BLOCK;
        if (b != cb) { pm_lines_block(blk.data(), PM_LINES_BLOCK, b, P.data(), O.data(), pats.size(), 1); cb = b; }
        return blk[pos % PM_LINES_BLOCK];
    };
    std::vector<std::vector<uint8_t>> txt(LANES);
    std::vector<uint64_t> wst(LANES);  // warm-up steps per lane
    for (int L = 0; L < LANES; ++L) {
        const uint64_t lo = (uint64_t)L * SPREAD + WARM + 64;
        uint64_t wlo = lo - WARM;
        // dfa_sync_lo: the last absent 3-gram start in [wlo, lo - 3]
        for (int64_t q = (int64_t)lo - 3; q >= (int64_t)wlo; --q) {
            const uint32_t x = text_at(q) | (uint32_t)text_at(q + 1) << 8 | (uint32_t)text_at(q + 2) << 16;
            if (!(g3[x >> 5] >> (x & 31) & 1u)) { wlo = q; break; }
        }
        wst[L] = lo - wlo;
        for (uint64_t p = wlo; p < lo + SEG; ++p) txt[L].push_back(text_at(p));
    }
    // row visit counts (for HOT), from a first pass
    std::vector<uint64_t> rowvis(F, 0);
    auto step = [&](uint32_t s, uint32_t c, uint32_t& cb, int& lds, int& glob, int& depth, bool& blockload,
                    const std::vector<uint8_t>& inlds, bool count_rows) -> uint32_t {
        lds = glob = depth = 0;
        blockload = false;
        if (s < F) {
            if (count_rows) rowvis[s]++;
            if (inlds[s]) lds = 1; else { glob = 1; depth = 1; }
            return B8[(size_t)s * 256 + c];
        }
        const uint32_t rec = s - F, b = rec / BU;
        if (b != cb) { glob++; depth = 1; cb = b; blockload = true; }
        const uint32_t* U = B8.data() + (size_t)F * 256 + (size_t)rec * 2;
        const uint32_t key = c | 0x100u;
        const uint32_t y = U[0], x = U[1];
        if ((x & 0x1FFu) == key) return y;
        uint32_t w = (x >> 9) & 0x3FFFFFu;
        if (x >> 31) {
            if (((x >> 16) & 0x1FFu) == key) return U[2];
            w = U[3];
        }
        if (count_rows) rowvis[w]++;
        if (inlds[w]) lds++; else { glob++; depth++; }
        return B8[(size_t)w * 256 + c];
    };
    std::vector<uint8_t> inlds(F, 0);
    for (uint32_t r = 0; r < (uint32_t)KR && r < F; ++r) inlds[r] = 1;
    for (int pass = 0; pass < (HOT ? 2 : 1); ++pass) {
        if (pass == 1) {
            std::vector<uint32_t> ord(F);
            for (uint32_t r = 0; r < F; ++r) ord[r] = r;
            std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return rowvis[a] > rowvis[b]; });
            std::fill(inlds.begin(), inlds.end(), 0);
            for (int r = 0; r < KR && r < (int)F; ++r) inlds[ord[r]] = 1;
        }
        uint64_t lane_steps = 0, lane_lds = 0, lane_glob = 0, lane_d2 = 0, lane_blk = 0, lane_blk_seq = 0;
        uint64_t wave_steps = 0, wave_lat = 0, wave_any = 0, wave_d2 = 0, wave_loading_lanes = 0;
        for (int w = 0; w < WAVES; ++w) {
            uint64_t wmax = 0;
            for (int k = 0; k < 64; ++k) wmax = std::max(wmax, wst[w * 64 + k]);
            std::vector<uint32_t> s(64, 0), cb(64, 0xFFFFFFFFu), since(64, 0);
            for (uint64_t j = 0; j < wmax + SEG; ++j) {
                int maxd = 0, loading = 0;
                for (int k = 0; k < 64; ++k) {
                    const int L = w * 64 + k;
                    const int64_t idx = (int64_t)j - (int64_t)(wmax - wst[L]);  // right-aligned warm-ups
                    if (idx < 0) continue;
                    int lds, glob, depth;
                    bool bl;
                    const uint32_t prevb = cb[k];
                    const uint32_t v = step(s[k], txt[L][idx], cb[k], lds, glob, depth, bl, inlds, pass == 0);
                    if (bl && PF && prevb != 0xFFFFFFFFu && cb[k] == prevb + 1 && since[k] >= 2) {
                        // sequential block entered: prefetched at the previous block's entry
                        glob--; depth--;
                        lane_blk_seq++;
                    }
                    since[k] = bl ? 0 : since[k] + 1;
                    s[k] = v & PM_DFA_STATE_MASK;
                    lane_steps++; lane_lds += lds; lane_glob += glob; lane_d2 += depth >= 2; lane_blk += bl;
                    maxd = std::max(maxd, depth);
                    loading += glob > 0;
                }
                wave_steps++;
                wave_lat += maxd;
                wave_any += maxd > 0;
                wave_d2 += maxd >= 2;
                wave_loading_lanes += loading;
            }
        }
        // Decoupled lanes: each lane walks its own positions; a position whose
        // step needs a global load issues it and completes one wave step
        // later (two dependent loads: two wave steps later), and a lane does
        // at most K positions per wave step.  Wave steps of a wave = its
        // slowest lane's; every wave step then waits for one load latency.
        for (int K : {1, 2, 3, 4}) {
            uint64_t wsteps = 0, iters = 0;
            for (int w = 0; w < WAVES; ++w) {
                uint64_t worst = 0;
                for (int k = 0; k < 64; ++k) {
                    const int L = w * 64 + k;
                    uint32_t s = 0, cb = 0xFFFFFFFFu;
                    uint64_t steps = 0;
                    int done_in_step = 0;
                    for (size_t idx = 0; idx < txt[L].size(); ++idx) {
                        int lds, glob, depth;
                        bool bl;
                        const uint32_t v = step(s, txt[L][idx], cb, lds, glob, depth, bl, inlds, false);
                        s = v & PM_DFA_STATE_MASK;
                        if (depth > 0) {  // waits `depth` wave steps, then completes in the last
                            steps += depth;
                            done_in_step = 1;
                        } else if (++done_in_step > K) {
                            ++steps;
                            done_in_step = 1;
                        }
                    }
                    worst = std::max(worst, steps + 1);
                }
                wsteps += worst;
                iters += worst * K;
            }
            printf("      decoupled K=%d: wave steps per segment %.0f (iterations %.0f) vs lock step %.0f\n", K,
                   wsteps / (double)WAVES, iters / (double)WAVES, wave_steps / (double)WAVES);
        }
        printf("BU %d: TA lane-accesses per wave step %.1f (block %.1f + words %.1f)\n", BU,
               64.0 * ((lane_glob - lane_blk) + lane_blk * (BU / 2.0)) / lane_steps * (lane_steps / (double)wave_steps) / 64.0 * 64.0 / 64.0 * 1.0,
               64.0 * lane_blk * (BU / 2.0) / wave_steps, 64.0 * (lane_glob - lane_blk) / wave_steps);
        printf("%s lane steps %llu: LDS reads/step %.3f, global loads/step %.3f (block loads %.3f, %s%.3f), "
               "two dependent loads %.3f\n", pass ? "HOT " : "FIRST", (unsigned long long)lane_steps,
               lane_lds / (double)lane_steps, lane_glob / (double)lane_steps, lane_blk / (double)lane_steps,
               PF ? "prefetched " : "", lane_blk_seq / (double)lane_steps, lane_d2 / (double)lane_steps);
        printf("      wave steps %llu (per lane segment %.0f): waiting %.3f, two-deep %.3f, dependent loads per wave "
               "step %.3f, loading lanes per wave step %.1f\n", (unsigned long long)wave_steps,
               wave_steps / (double)WAVES, wave_any / (double)wave_steps, wave_d2 / (double)wave_steps,
               wave_lat / (double)wave_steps, wave_loading_lanes / (double)wave_steps);
    }
}
