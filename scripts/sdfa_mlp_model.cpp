// sdfa_mlp_model.cpp -- probe (not product): how the L2 misses of the sparse
// AC-DFA kernel on the lines stream depend on the number of chains in flight
// per XCD and on the records a lane keeps in registers.  An LRU model of one
// XCD's 4 MiB L2 (128-B lines) over the real sblock image: table steps, the
// lane's text loads (BLK bytes per block) and its id lines (write-allocate).
//   g++ -O2 -std=c++17 -Ipatternmatching_amd/csrc -Iinclude scripts/sdfa_mlp_model.cpp \
//       patternmatching_amd/csrc/pm_flatten.cpp patternmatching_amd/csrc/host/pm_dict.c -o /tmp/mlp && /tmp/mlp DICT...
#include "pm_flatten.h"
#include "pm_streamgen.h"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <fstream>
#include <list>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>
extern "C" size_t pm_parse_line(const unsigned char* line, size_t n, unsigned char* out);
static int g_cat = 0;
static uint64_t g_cmiss[4];
struct LRU {
    size_t cap;
    std::list<uint64_t> l;
    std::unordered_map<uint64_t, std::list<uint64_t>::iterator> m;
    uint64_t hit = 0, miss = 0;
    void touch(uint64_t k, bool count = true) {
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
    std::vector<uint8_t> P;
    std::vector<uint32_t> O(1, 0);
    for (auto& p : pats) { P.insert(P.end(), p.begin(), p.end()); O.push_back(P.size()); }
    printf("states %u rows %u (%.1f MB) records %.1f MB\n", S, F, F * 1024.0 / 1e6, (S - F) * 16.0 / 1e6);
    const uint64_t TBASE = 1ull << 40, IBASE = 1ull << 44;  // text / ids address spaces
    // byte permutation of the row slots: bytes by their frequency in the patterns
    std::vector<uint32_t> perm(256);
    {
        std::vector<std::pair<uint64_t, int>> fr(256);
        for (int c = 0; c < 256; ++c) fr[c] = {0, c};
        for (uint8_t c : P) fr[c].first++;
        fr['\n'].first += pats.size();
        std::sort(fr.begin(), fr.end(), [](auto a, auto b) { return a.first > b.first; });
        for (int r = 0; r < 256; ++r) perm[fr[r].second] = r;
    }
    const int RECB = getenv("RECB") ? atoi(getenv("RECB")) : 16;  // record bytes (8: an upper bound on 8-B unary records)
    for (int pm : {0})
    for (int regrec : {64 / RECB}) {
        for (size_t chains : {32768ul}) {
            memset(g_cmiss, 0, sizeof g_cmiss);
            const size_t per = 1024;  // bytes per chain
            const size_t SEG = 8192;                  // the real segment spacing (1 GiB / 131072 lanes)
            std::vector<uint8_t> t(chains * per);
            for (size_t L = 0; L < chains; ++L) {  // chain L's bytes come from its own place in the stream
                const uint64_t lo = (uint64_t)L * SEG * 8;
                std::vector<uint8_t> blk(PM_LINES_BLOCK);
                for (size_t j = 0; j < per; j += PM_LINES_BLOCK) {
                    const uint64_t b = (lo + j) / PM_LINES_BLOCK;
                    pm_lines_block(blk.data(), PM_LINES_BLOCK, b, P.data(), O.data(), pats.size(), 1);
                    memcpy(&t[L * per + j], blk.data(), std::min<size_t>(PM_LINES_BLOCK, per - j));
                }
            }
            LRU l2{32768};
            std::vector<uint32_t> st(chains, 0), cb(chains, 0xFFFFFFFFu);
            uint64_t tbl = 0, warmn = 0;
            const size_t WARM = 384;  // untimed warm-up steps (cache and states)
            for (size_t j = 0; j < per; ++j) {
                const bool cnt = j >= WARM;
                warmn += !cnt;
                for (size_t L = 0; L < chains; ++L) {
                    const uint64_t pos = (uint64_t)L * SEG * 8 + j;
                    g_cat = 3;
                    if (j % 32 == 0) {
                        l2.touch((TBASE + pos) / 128, cnt);        // 32 text bytes
                        l2.touch((IBASE + pos * 4) / 128, cnt);    // 128 B of ids
                    }
                    const uint32_t s = st[L], c = t[L * per + j];
                    uint32_t v;
                    const uint32_t pc = pm ? perm[c] : c;
                    if (s < F) {
                        g_cat = 0;
                        l2.touch(((uint64_t)s * 1024 + pc * 4) / 128, cnt);
                        tbl += cnt;
                        v = B[(size_t)s * 256 + c];
                    } else {
                        const uint64_t off = (uint64_t)F * 1024 + (uint64_t)(s - F) * RECB;
                        const uint32_t blk = (s - F) / regrec;
                        g_cat = 1;
                        if (blk != cb[L] || regrec == 1) {
                            l2.touch(off / 128, cnt);
                            tbl += cnt;
                            cb[L] = blk;
                        }
                        const uint32_t* r = B + (size_t)F * 256 + (size_t)(s - F) * 4;
                        const uint32_t key = c | 0x100u;
                        if ((r[0] & 0x1FF) == key) v = r[1];
                        else if (((r[0] >> 16) & 0x1FF) == key) v = r[2];
                        else {
                            g_cat = 2;
                            l2.touch(((uint64_t)r[3] * 1024 + pc * 4) / 128, cnt);
                            tbl += cnt;
                            v = B[(size_t)r[3] * 256 + c];
                        }
                    }
                    st[L] = v & PM_DFA_STATE_MASK;
                }
            }
            const double nb = (double)chains * (per - WARM);
            printf("perm %d rowmiss %.3f recmiss %.3f fbmiss %.3f streammiss %.3f | ", pm, g_cmiss[0] / nb, g_cmiss[1] / nb, g_cmiss[2] / nb, g_cmiss[3] / nb);
            printf("regrec %d chains/XCD %6zu (%4zu per CU): table loads/byte %.3f  L2 misses/byte %.3f  hit %.3f\n",
                   regrec, chains, chains / 32, tbl / nb, l2.miss / nb, l2.hit / (double)(l2.hit + l2.miss));
            fflush(stdout);
        }
    }
}
