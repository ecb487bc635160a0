// sdfa_u4_stats.cpp -- probe (not product): what a 4-B record unit could
// hold.  Classifies the sparse form's records (pm_flatten.h) statically and
// by visits on the lines stream (lanes of SEG bytes, as the deep kernel):
//   A  one slot, target = the next record in trie order, target's gid <= LIM
//   A+ one slot, target = the next record, gid > LIM
//   B  one slot, another target
//   C  no slot
//   D  two slots, one of them to the next record (gid <= LIM)
//   E  two slots, otherwise
// and the visit share of record steps whose slot hits / misses.
//   g++ -O2 -std=c++17 -Ipatternmatching_amd/csrc -Iinclude scripts/sdfa_u4_stats.cpp \
//       patternmatching_amd/csrc/pm_flatten.cpp patternmatching_amd/csrc/host/pm_dict.c -o /tmp/u4s && \
//   /tmp/u4s tests/golden/data/snort.dict
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
    const uint32_t LIM = envi("LIM", 248);
    PmGidMap g = pm_assign_gids(pats);
    DfaImage d = pm_build_dfa(pats, g);
    const uint32_t F = d.sF, S = d.states;
    const uint32_t* B = d.sblock.data();
    const uint32_t* REC = B + (size_t)F * 256;
    auto cls = [&](uint32_t v) -> int {
        const uint32_t* r = REC + (size_t)(v - F) * 4;
        const bool s0 = r[0] & 0x100u, s1 = r[0] & 0x1000000u;
        const uint32_t t0 = r[1] & PM_DFA_STATE_MASK, t1 = r[2] & PM_DFA_STATE_MASK;
        if (!s0) return 4;  // C
        if (!s1) {
            if (t0 == v + 1 && t0 < S && t0 >= F) return d.sout[t0] <= LIM ? 0 : 1;
            return 2;
        }
        if ((t0 == v + 1 && d.sout[t0] <= LIM) || (t1 == v + 1 && d.sout[t1] <= LIM)) return 5;
        return 6;
    };
    const char* names[7] = {"A one-slot next", "A+ next, gid>LIM", "B one-slot other", "-", "C no slot",
                            "D two-slot, one next", "E two-slot other"};
    uint64_t stat[7] = {};
    for (uint32_t v = F; v < S; ++v) stat[cls(v)]++;
    printf("patterns %zu states %u rows F=%u records %u  LIM %u\n", pats.size(), S, F, S - F, LIM);
    for (int k = 0; k < 7; ++k)
        if (k != 3) printf("  static %-22s %8llu (%.1f%%)\n", names[k], (unsigned long long)stat[k], 100.0 * stat[k] / (S - F));
    // sizes: A 4 B, A+ / B 8 B, C 4 B, D 8 B (u0 + the other target), E 12-16 B
    const double bytes = stat[0] * 4.0 + (stat[1] + stat[2]) * 8.0 + stat[4] * 4.0 + stat[5] * 12.0 + stat[6] * 16.0;
    printf("  U4 image (unpadded): %.2f MB (8-B units today: %.2f MB)\n", bytes / 1e6,
           ((stat[0] + stat[1] + stat[2] + stat[4]) * 8.0 + (stat[5] + stat[6]) * 16.0) / 1e6);
    // dynamic
    std::vector<uint8_t> P;
    std::vector<uint32_t> O(1, 0);
    for (auto& p : pats) { P.insert(P.end(), p.begin(), p.end()); O.push_back(P.size()); }
    const int LANES = envi("LANES", 4096), SEG = envi("SEG", 4096);
    const uint64_t SPREAD = (1ull << 30) / LANES;
    uint64_t dyn[7] = {}, hit[7] = {}, rows = 0, steps = 0, nz = 0, nzlim = 0;
    // two-deep steps (a record whose 32-B block of 8-B units is not the one
    // the lane holds, and whose slots miss): by how the state was entered
    // (0 row word, 1 record slot, 2 fallback row word) and the state's class
    uint64_t d2[3][7] = {}, ent[3] = {};
    std::map<uint32_t, uint64_t> d2w;
    std::vector<uint32_t> U8off(S, 0);
    {
        uint64_t u = 0;
        for (uint32_t v = F; v < S; ++v) {
            const bool two = REC[(size_t)(v - F) * 4] & 0x1000000u;
            if (two && (u & 3) == 3) ++u;
            U8off[v] = (uint32_t)u;
            u += two ? 2 : 1;
        }
    }
    std::vector<uint8_t> blk(PM_LINES_BLOCK);
    for (int L = 0; L < LANES; ++L) {
        uint32_t s = 0, cb = ~0u;
        int how = 0;
        const uint64_t lo = (uint64_t)L * SPREAD;
        for (uint64_t p = lo; p < lo + SEG; ++p) {
            if (p % PM_LINES_BLOCK == 0 || p == lo)
                pm_lines_block(blk.data(), PM_LINES_BLOCK, p / PM_LINES_BLOCK, P.data(), O.data(), pats.size(), 1);
            const uint32_t c = blk[p % PM_LINES_BLOCK];
            uint32_t v;
            const bool cnt = p - lo >= 400;
            if (s < F) {
                rows++;
                v = B[(size_t)s * 256 + c];
                how = 0;
            } else {
                const uint32_t* r = REC + (size_t)(s - F) * 4;
                const int k = cls(s);
                dyn[k]++;
                const uint32_t key = c | 0x100u;
                const bool nb = U8off[s] / 4 != cb;
                cb = U8off[s] / 4;
                if (cnt) ent[how]++;
                const int hw = how;
                if ((r[0] & 0x1FF) == key) v = r[1], hit[k]++, how = 1;
                else if (((r[0] >> 16) & 0x1FF) == key) v = r[2], hit[k]++, how = 1;
                else {
                    v = B[(size_t)r[3] * 256 + c];
                    how = 2;
                    if (nb && cnt && r[3] >= (uint32_t)envi("KR", 88)) d2[hw][k]++;
                    if (nb && cnt && r[3] >= (uint32_t)envi("KR", 88)) d2w[r[3]]++;
                }
            }
            s = v & PM_DFA_STATE_MASK;
            if (p - lo >= 400) {
                steps++;
                nz += d.sout[s] != 0;
                nzlim += d.sout[s] != 0 && d.sout[s] <= LIM;
            }
        }
    }
    // fallback rows of the records: distinct, and the share of records /
    // visits covered by the most used ones
    {
        std::vector<uint64_t> use(F, 0), vis(F, 0);
        for (uint32_t v = F; v < S; ++v) use[REC[(size_t)(v - F) * 4 + 3]]++;
        uint32_t distinct = 0;
        for (uint32_t r = 0; r < F; ++r) distinct += use[r] != 0;
        std::vector<uint32_t> ord(F);
        for (uint32_t r = 0; r < F; ++r) ord[r] = r;
        std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return use[a] > use[b]; });
        uint64_t tot = S - F, acc = 0;
        printf("  fallback rows used by records: %u distinct of %u rows;", distinct, F);
        for (uint32_t k = 0, lim = 256; k < F && lim <= 65536; ++k) {
            acc += use[ord[k]];
            if (k + 1 == lim) { printf(" top %u cover %.2f%%", lim, 100.0 * acc / tot); lim *= 4; }
        }
        printf("\n");
    }
    {
        const char* hn[3] = {"row word", "record slot", "fallback row"};
        for (int h = 0; h < 3; ++h) {
            uint64_t t = 0;
            for (int k = 0; k < 7; ++k) t += d2[h][k];
            printf("  two-deep steps entered by %-12s %.4f per step (of %.3f record steps entered so):", hn[h],
                   t / (double)steps, ent[h] / (double)steps);
            for (int k = 0; k < 7; ++k)
                if (d2[h][k]) printf(" %s %.4f", names[k], d2[h][k] / (double)steps);
            printf("\n");
        }
    }
    {
        std::vector<std::pair<uint64_t, uint32_t>> v;
        for (auto& kv : d2w) v.push_back({kv.second, kv.first});
        std::sort(v.rbegin(), v.rend());
        printf("  two-deep global fallbacks: %zu distinct rows; top:", v.size());
        for (size_t k = 0; k < v.size() && k < 12; ++k) printf(" %u:%.4f", v[k].second, v[k].first / (double)steps);
        printf("\n");
    }
    uint64_t recs = 0;
    for (int k = 0; k < 7; ++k) recs += dyn[k];
    printf("  lines stream, %d lanes x %d B: row steps %.1f%%, record steps %.1f%%; nonzero outputs %.1f%% of "
           "positions, %.1f%% of them gid <= LIM\n", LANES, SEG, 100.0 * rows / (rows + recs), 100.0 * recs / (rows + recs),
           100.0 * nz / steps, 100.0 * nzlim / std::max<uint64_t>(nz, 1));
    for (int k = 0; k < 7; ++k)
        if (k != 3)
            printf("  visits %-22s %6.1f%% of record steps (slot hit %.1f%%)\n", names[k], 100.0 * dyn[k] / recs,
                   100.0 * hit[k] / std::max<uint64_t>(dyn[k], 1));
}
