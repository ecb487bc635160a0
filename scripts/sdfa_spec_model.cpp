// sdfa_spec_model.cpp -- probe (not product): dependent global-load latencies
// per WAVE step (64 lanes in lock step wait for their slowest lane) of the
// deep sparse AC-DFA kernel on the lines stream, for two designs:
//   cur   the product (dfa_sparse_stage16_kernel): 8-B record units in 32-B
//         register blocks; a record whose block the lane does not hold needs
//         the block, then at a slot miss its fallback row's word: two
//         dependent loads;
//   spec  the word that leads into a record also names the record's fallback
//         row (rows numbered by how many records fall back to them), so a
//         lane entering a record in a block it does not hold issues the block
//         and -- for records that are not a chain interior (no slot to the
//         next record) -- the fallback row's word at the next byte together:
//         one latency.  Records without slots whose output has an inline code
//         are folded into their fallback rows (the word into them names the
//         row and carries their output: the same Mealy machine).
// LDS rows: the first KR rows of each design's numbering (cur: shallowest;
// spec: most used as fallbacks).  Prints latencies per wave step and global
// requests per lane step (spec counts its unused speculative loads).
//   g++ -O2 -std=c++17 -Ipatternmatching_amd/csrc -Iinclude scripts/sdfa_spec_model.cpp \
//       patternmatching_amd/csrc/pm_flatten.cpp patternmatching_amd/csrc/host/pm_dict.c -o /tmp/spec && \
//   /tmp/spec tests/golden/data/snort.dict
#include "pm_flatten.h"
#include "pm_streamgen.h"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
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
    const uint32_t F = d.sF, S = d.states;
    const uint32_t* B = d.sblock.data();
    const uint32_t* REC = B + (size_t)F * 256;
    const int KR = envi("KR", 88), WAVES = envi("WAVES", 64), SEG = envi("SEG", 4096), SPECALL = envi("SPECALL", 0);
    const uint32_t WLIM = envi("WLIM", 2047);  // fallback rows the word can name (11 bits + a speculate bit)
    // BFS88 = 1: the first KR rows keep the trie's breadth-first order (the
    // shallowest states, as the 8-B form stages them), the rest by fallback
    // use; SPEC: 0 none, 1 non-chain records, 2 every new block; ASCII = 1:
    // the random ASCII stream instead of the lines stream
    const int BFS88 = envi("BFS88", 0), SPEC = envi("SPEC", 1), ASCII = envi("ASCII", 0);
    // cur: 8-B unit offsets, 32-B blocks
    std::vector<uint32_t> cur_blk(S, 0), new_blk(S, 0);
    {
        uint64_t u = 0;
        for (uint32_t v = F; v < S; ++v) {
            const bool two = REC[(size_t)(v - F) * 4] & 0x1000000u;
            if (two && (u & 3) == 3) ++u;
            cur_blk[v] = (uint32_t)(u / 4);
            u += two ? 2 : 1;
        }
    }
    // spec: fallback use ranks; folded slotless records; 4-B words, records
    // of 8 B (one slot) / 12 B (two), +4 B when the fallback's rank >= 4095
    std::vector<uint64_t> use(F, 0);
    for (uint32_t v = F; v < S; ++v) use[REC[(size_t)(v - F) * 4 + 3]]++;
    use[0] = ~0ull;  // the root stays row 0 (the warm-up's start)
    std::vector<uint32_t> ord(F), rank(F);
    for (uint32_t r = 0; r < F; ++r) ord[r] = r;
    if (BFS88) {
        for (uint32_t r = 0; r < F && r < (uint32_t)KR; ++r) use[r] = ~0ull - r;  // keep 0..KR-1 first, in order
    }
    std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return use[a] > use[b]; });
    for (uint32_t k = 0; k < F; ++k) rank[ord[k]] = k;
    std::vector<uint8_t> fold(S, 0), chain(S, 0);
    uint64_t nfold = 0, bytes = 0;
    {
        uint64_t u = 0;
        for (uint32_t v = F; v < S; ++v) {
            const uint32_t* r = REC + (size_t)(v - F) * 4;
            const bool s0 = r[0] & 0x100u, s1 = r[0] & 0x1000000u;
            const uint32_t t0 = r[1] & PM_DFA_STATE_MASK, t1 = r[2] & PM_DFA_STATE_MASK;
            chain[v] = (s0 && t0 == v + 1) || (s1 && t1 == v + 1);
            if (!s0 && d.sout[v] < PM_DFA_ESC) {
                fold[v] = 1, ++nfold;
                continue;
            }
            uint32_t b = s1 ? 16 : 8;  // 8-B granularity (20-bit ids): {out16 c0 c1, t0}, {t1, w}
            if (rank[r[3]] >= WLIM) b = 16;
            if (u / 32 != (u + b - 1) / 32) u = (u / 32 + 1) * 32;
            new_blk[v] = (uint32_t)(u / 32);
            u += b;
        }
        bytes = u;
    }
    printf("patterns %zu states %u rows %u records %u: spec layout %.2f MB of records, %llu slotless records "
           "folded | KR %d WAVES %d SEG %d%s\n", pats.size(), S, F, S - F, bytes / 1e6, (unsigned long long)nfold,
           KR, WAVES, SEG, SPECALL ? " (speculate at every new block)" : "");
    std::vector<uint8_t> P;
    std::vector<uint32_t> O(1, 0);
    for (auto& p : pats) { P.insert(P.end(), p.begin(), p.end()); O.push_back(P.size()); }
    const int LANES = 64 * WAVES;
    const uint64_t SPREAD = (1ull << 30) / LANES;
    std::vector<std::vector<uint8_t>> txt(LANES);
    {
        std::vector<uint8_t> blk(PM_LINES_BLOCK);
        for (int L = 0; L < LANES; ++L) {
            const uint64_t lo = (uint64_t)L * SPREAD;
            for (uint64_t p = lo; p < lo + 512 + SEG; ++p) {
                if (p % PM_LINES_BLOCK == 0 || p == lo)
                    pm_lines_block(blk.data(), PM_LINES_BLOCK, p / PM_LINES_BLOCK, P.data(), O.data(), pats.size(), 1);
                txt[L].push_back(ASCII ? pm_stream_byte(p, 1, 0) : blk[p % PM_LINES_BLOCK]);
            }
        }
    }
    for (int design = 0; design < 2; ++design) {
        uint64_t wave_steps = 0, wave_lat = 0, wave_d2 = 0, lane_steps = 0, req = 0, wasted = 0, d2 = 0;
        for (int w = 0; w < WAVES; ++w) {
            std::vector<uint32_t> s(64, 0), cb(64, ~0u);
            for (int j = 0; j < 512 + SEG; ++j) {
                const bool cnt = j >= 512;  // the first 512 steps: warm-up (states, blocks)
                int maxd = 0;
                for (int k = 0; k < 64; ++k) {
                    const int L = w * 64 + k;
                    const uint32_t c = txt[L][j], st = s[k];
                    int depth = 0;
                    uint32_t v;
                    if (st < F) {
                        const bool lds = design ? rank[st] < (uint32_t)KR : st < (uint32_t)KR;
                        depth = lds ? 0 : 1;
                        req += cnt && !lds;
                        v = B[(size_t)st * 256 + c];
                    } else {
                        const uint32_t* r = REC + (size_t)(st - F) * 4;
                        const uint32_t blkid = design ? new_blk[st] : cur_blk[st];
                        const bool nb = blkid != cb[k];
                        cb[k] = blkid;
                        const uint32_t key = c | 0x100u;
                        const bool hit0 = (r[0] & 0x1FF) == key, hit1 = ((r[0] >> 16) & 0x1FF) == key;
                        const uint32_t wr = r[3];
                        const bool wlds = design ? rank[wr] < (uint32_t)KR : wr < (uint32_t)KR;
                        const bool spec = design && SPEC && (SPECALL || SPEC == 2 || !chain[st]) && rank[wr] < WLIM && !wlds;
                        req += cnt && nb;
                        if (hit0 || hit1) {
                            v = hit0 ? r[1] : r[2];
                            depth = nb ? 1 : 0;
                            if (nb && spec) req += cnt, wasted += cnt;
                        } else {
                            v = B[(size_t)wr * 256 + c];
                            if (!wlds) req += cnt;
                            if (nb) depth = (spec || wlds) ? 1 : 2;
                            else depth = wlds ? 0 : 1;
                        }
                    }
                    uint32_t t = v & PM_DFA_STATE_MASK;
                    if (design && t >= F && fold[t]) t = REC[(size_t)(t - F) * 4 + 3];
                    s[k] = t;
                    if (cnt) {
                        lane_steps++;
                        d2 += depth == 2;
                        maxd = std::max(maxd, depth);
                    }
                }
                if (cnt) {
                    wave_steps++;
                    wave_lat += maxd;
                    wave_d2 += maxd == 2;
                }
            }
        }
        printf("%-4s latencies per wave step %.3f (two-deep wave steps %.3f, lane two-deep %.4f); global requests "
               "per lane step %.3f (unused speculative %.3f)\n", design ? "spec" : "cur", wave_lat / (double)wave_steps,
               wave_d2 / (double)wave_steps, d2 / (double)lane_steps, req / (double)lane_steps,
               wasted / (double)lane_steps);
    }
}
