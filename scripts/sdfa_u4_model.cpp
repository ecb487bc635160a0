// sdfa_u4_model.cpp -- probe (not product): an LRU model of one XCD's 4 MiB L2
// (128-B lines) under the deep sparse AC-DFA kernel on the lines stream, for
// record layouts of different sizes.  32,768 chains per XCD (1,024 per CU, as
// dfa_sparse_stage16_kernel), each a 4 KiB segment of its own place in the
// stream; per 32-position block a chain touches its 32 text bytes and (ID=1)
// its 128 B of id lines; per step a row word (unless the row is one of the KR
// staged in LDS) or its record block (when the state leaves the block it
// holds) and, at a slot miss, the fallback row's word.
//   layout 8: the product's 8-B units (pm_pack_sparse8), BLK-byte blocks;
//   layout 4: 4-B units where a record allows (sdfa_u4_stats.cpp classes:
//             one slot to the next record, code < 4094, fallback among the
//             4,095 most used rows: 4 B; otherwise 8 / 12 / 16 B), records
//             kept inside aligned blocks.
// Env: LAYOUT (8), BLK (32), KR (88), HOTROWS (0: the first KR rows in LDS;
// 1: the KR rows most used as fallbacks), ID (1), CHAINS (32768), PER (1024).
//   g++ -O2 -std=c++17 -Ipatternmatching_amd/csrc -Iinclude scripts/sdfa_u4_model.cpp \
//       patternmatching_amd/csrc/pm_flatten.cpp patternmatching_amd/csrc/host/pm_dict.c -o /tmp/u4m && \
//   /tmp/u4m tests/golden/data/snort.dict
#include "pm_flatten.h"
#include "pm_streamgen.h"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <list>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>
extern "C" size_t pm_parse_line(const unsigned char* line, size_t n, unsigned char* out);
static int envi(const char* k, int d) { const char* v = getenv(k); return v ? atoi(v) : d; }
static int g_cat = 0;
static uint64_t g_cmiss[5], g_creq[5];
struct LRU {
    size_t cap;
    std::list<uint64_t> l;
    std::unordered_map<uint64_t, std::list<uint64_t>::iterator> m;
    uint64_t hit = 0, miss = 0;
    void touch(uint64_t k, bool count = true) {
        g_creq[g_cat] += count;
        auto it = m.find(k);
        if (it != m.end()) {
            hit += count;
            l.splice(l.begin(), l, it->second);
            return;
        }
        miss += count;
        g_cmiss[g_cat] += count;
        l.push_front(k);
        m[k] = l.begin();
        if (m.size() > cap) {
            m.erase(l.back());
            l.pop_back();
        }
    }
};

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
    const int LAYOUT = envi("LAYOUT", 8), BLK = envi("BLK", 32), KR = envi("KR", 88), HOT = envi("HOTROWS", 0);
    const int ID = envi("ID", 1);
    const size_t CHAINS = envi("CHAINS", 32768), PER = envi("PER", 1024);
    // fallback use per row (for the 4-B form's 12-bit row field and HOTROWS)
    std::vector<uint64_t> use(F, 0);
    for (uint32_t v = F; v < S; ++v) use[REC[(size_t)(v - F) * 4 + 3]]++;
    std::vector<uint32_t> ord(F);
    for (uint32_t r = 0; r < F; ++r) ord[r] = r;
    std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return use[a] > use[b]; });
    std::vector<uint32_t> rank(F);
    for (uint32_t k = 0; k < F; ++k) rank[ord[k]] = k;
    std::vector<uint8_t> inlds(F, 0);
    for (uint32_t k = 0; k < (uint32_t)KR && k < F; ++k) inlds[HOT ? ord[k] : k] = 1;
    // record byte offsets
    std::vector<uint64_t> off(S - F);
    uint64_t u = 0;
    auto place = [&](uint32_t v, uint32_t bytes) {
        if (u / BLK != (u + bytes - 1) / BLK) u = (u / BLK + 1) * BLK;  // never straddle a block
        off[v - F] = u;
        u += bytes;
    };
    uint64_t nshort = 0;
    for (uint32_t v = F; v < S; ++v) {
        const uint32_t* r = REC + (size_t)(v - F) * 4;
        const bool s0 = r[0] & 0x100u, s1 = r[0] & 0x1000000u;
        if (LAYOUT == 8) {
            place(v, s1 ? 16 : 8);
            continue;
        }
        const uint32_t t0 = r[1] & PM_DFA_STATE_MASK, t1 = r[2] & PM_DFA_STATE_MASK;
        const bool nx0 = s0 && t0 == v + 1 && d.sout[t0] < 4094, nx1 = s1 && t1 == v + 1 && d.sout[t1] < 4094;
        uint32_t bytes;
        if (s0 && !s1 && nx0 && rank[r[3]] < 4095) bytes = 4, ++nshort;
        else if (!s0) bytes = 8;
        else if (!s1) bytes = nx0 ? 8 : 12;
        else bytes = (nx0 || nx1) ? 12 : 16;
        place(v, bytes);
    }
    printf("states %u rows %u records %u: layout %d, %.2f MB of records (%llu 4-B short), blocks %d B, KR %d%s\n", S,
           F, S - F, LAYOUT, u / 1e6, (unsigned long long)nshort, BLK, KR, HOT ? " (hottest fallback rows)" : "");
    std::vector<uint8_t> P;
    std::vector<uint32_t> O(1, 0);
    for (auto& p : pats) { P.insert(P.end(), p.begin(), p.end()); O.push_back(P.size()); }
    const uint64_t RBASE = 1ull << 36, TBASE = 1ull << 40, IBASE = 1ull << 44;
    const size_t SEG = (1ull << 30) / CHAINS / 8;  // chains of one XCD are 1/8 of the launch's
    std::vector<uint8_t> t(CHAINS * PER);
    {
        std::vector<uint8_t> blk(PM_LINES_BLOCK);
        for (size_t L = 0; L < CHAINS; ++L) {
            const uint64_t lo = (uint64_t)L * SEG * 8;
            for (size_t j = 0; j < PER; j += PM_LINES_BLOCK) {
                pm_lines_block(blk.data(), PM_LINES_BLOCK, (lo + j) / PM_LINES_BLOCK, P.data(), O.data(), pats.size(), 1);
                memcpy(&t[L * PER + j], blk.data(), std::min<size_t>(PM_LINES_BLOCK, PER - j));
            }
        }
    }
    LRU l2{(4u << 20) / 128};
    std::vector<uint32_t> st(CHAINS, 0);
    std::vector<uint64_t> cb(CHAINS, ~0ull);
    const size_t WARM = 384;
    uint64_t loads = 0, steps = 0;
    for (size_t j = 0; j < PER; ++j) {
        const bool cnt = j >= WARM;
        for (size_t L = 0; L < CHAINS; ++L) {
            const uint64_t pos = (uint64_t)L * SEG * 8 + j;
            if (j % 32 == 0) {
                g_cat = 3;
                l2.touch((TBASE + pos) / 128, cnt);
                if (ID) {
                    g_cat = 4;
                    l2.touch((IBASE + pos * 4) / 128, cnt);
                }
            }
            const uint32_t s = st[L], c = t[L * PER + j];
            uint32_t v;
            steps += cnt;
            if (s < F) {
                g_cat = 0;
                if (!inlds[s]) l2.touch(((uint64_t)s * 1024 + c * 4) / 128, cnt), loads += cnt;
                v = B[(size_t)s * 256 + c];
            } else {
                const uint64_t o = off[s - F], b = o / BLK;
                if (b != cb[L]) {
                    g_cat = 1;
                    for (uint64_t q = b * BLK; q < b * BLK + BLK; q += 128) l2.touch((RBASE + q) / 128, cnt);
                    loads += cnt;
                    cb[L] = b;
                }
                const uint32_t* r = REC + (size_t)(s - F) * 4;
                const uint32_t key = c | 0x100u;
                if ((r[0] & 0x1FF) == key) v = r[1];
                else if (((r[0] >> 16) & 0x1FF) == key) v = r[2];
                else {
                    g_cat = 2;
                    if (!inlds[r[3]]) l2.touch(((uint64_t)r[3] * 1024 + c * 4) / 128, cnt), loads += cnt;
                    v = B[(size_t)r[3] * 256 + c];
                }
            }
            st[L] = v & PM_DFA_STATE_MASK;
        }
    }
    const double nb = (double)steps;
    printf("  per stream byte: L2 misses %.3f (rows %.3f, record blocks %.3f, fallback rows %.3f, text %.3f, ids %.3f)"
           "  table requests %.3f (rows %.3f, blocks %.3f, fallbacks %.3f)  hit rate %.3f\n",
           l2.miss / nb, g_cmiss[0] / nb, g_cmiss[1] / nb, g_cmiss[2] / nb, g_cmiss[3] / nb, g_cmiss[4] / nb,
           loads / nb, g_creq[0] / nb, g_creq[1] / nb, g_creq[2] / nb, l2.hit / (double)(l2.hit + l2.miss));
}
