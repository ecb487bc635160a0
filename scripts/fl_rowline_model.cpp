// fl_rowline_model.cpp -- probe (not product): the global lines the FL
// kernel (dfa_fl_kernel, pm_pack_sparse_fl's real image) touches on the
// lines stream, and an LRU model of one XCD's L2 over them, for the
// product's row layout and for rows whose columns are permuted by byte
// frequency in the dictionary (the bytes text uses most in a row's first
// 128-B lines).  LANES lanes (default 4,096 = one XCD's share scaled by
// 1/8) walk SEG bytes each from their own 1 GiB / LANES offset, in lock
// step; the L2 is scaled with them (L2KB, default 512 = 4 MiB / 8).
// Counts: row-word lines (rows past the KR in LDS), record lines (a new
// 16-B half or 32-B block), fallback-row lines at a record miss.
// Layouts (each line of output): the product image with its rows in BFS
// order (pm_pack_sparse_fl without a profile); rows with their columns
// permuted by byte frequency; unary-chain records in 4 B; deep records in
// 64-B / 128-B blocks; the LDS rows chosen by visits on a profile sample
// (MIX=1: MIXL of 512 lanes the dictionary's lines text, the rest random
// ASCII -- the packer's profile is 15:1; MIX=2 lines only; MIX=0 the
// evaluation text itself).  ASCII=1 / SHIP=<file>: evaluate on random
// ASCII / a tiled file instead of the lines stream.  COVER=1: instead, the
// share of non-root row requests LDS would serve holding whole rows, hot
// 128-B row lines, or rows' printable lines, chosen on the profile.
//   g++ -O2 -std=c++17 -Ipatternmatching_amd/csrc -Iinclude scripts/fl_rowline_model.cpp \
//       patternmatching_amd/csrc/pm_flatten.cpp patternmatching_amd/csrc/host/pm_dict.c -o /tmp/rowline && \
//   /tmp/rowline tests/golden/data/snort.dict
#include "pm_flatten.h"
#include "pm_streamgen.h"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <list>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>
extern "C" size_t pm_parse_line(const unsigned char* line, size_t n, unsigned char* out);
static int envi(const char* k, int d) { const char* v = getenv(k); return v ? atoi(v) : d; }

struct Lru {
    size_t cap;
    std::list<uint64_t> l;
    std::unordered_map<uint64_t, std::list<uint64_t>::iterator> m;
    uint64_t hit = 0, miss = 0;
    bool touch(uint64_t a) {
        auto it = m.find(a);
        if (it != m.end()) {
            l.splice(l.begin(), l, it->second);
            ++hit;
            return true;
        }
        ++miss;
        l.push_front(a);
        m[a] = l.begin();
        if (l.size() > cap) {
            m.erase(l.back());
            l.pop_back();
        }
        return false;
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
    FlImage fl;
    if (!pm_pack_sparse_fl(d, fl)) { printf("no FL form\n"); return 1; }
    const uint32_t F = fl.F;
    const int KR = envi("KR", 88), LANES = envi("LANES", 4096), SEG = envi("SEG", 4096), L2KB = envi("L2KB", 512);
    // byte frequency in the dictionary -> column order
    std::vector<uint64_t> freq(256, 0);
    for (auto& p : pats)
        for (unsigned char c : p) freq[c]++;
    std::vector<int> ord(256);
    for (int c = 0; c < 256; ++c) ord[c] = c;
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return freq[a] > freq[b]; });
    std::vector<uint32_t> perm(256);
    for (int k = 0; k < 256; ++k) perm[ord[k]] = k;
    // text
    std::vector<uint8_t> P;
    std::vector<uint32_t> O(1, 0);
    for (auto& p : pats) { P.insert(P.end(), p.begin(), p.end()); O.push_back(P.size()); }
    const uint64_t SPREAD = (1ull << 30) / LANES;
    const int WARM = 256;
    std::vector<std::vector<uint8_t>> txt(LANES);
    std::vector<uint8_t> ship;
    if (getenv("SHIP")) {  // the reference's shipped stream, tiled
        std::ifstream f(getenv("SHIP"), std::ios::binary);
        ship.assign(std::istreambuf_iterator<char>(f), {});
    }
    {
        std::vector<uint8_t> blk(PM_LINES_BLOCK);
        for (int L = 0; L < LANES; ++L) {
            const uint64_t lo = (uint64_t)L * SPREAD;
            for (uint64_t p = lo; p < lo + WARM + SEG; ++p) {
                if (p % PM_LINES_BLOCK == 0 || p == lo)
                    pm_lines_block(blk.data(), PM_LINES_BLOCK, p / PM_LINES_BLOCK, P.data(), O.data(), pats.size(), 1);
                txt[L].push_back(!ship.empty() ? ship[p % ship.size()]
                                 : envi("ASCII", 0) ? pm_stream_byte(p, 1, 0) : blk[p % PM_LINES_BLOCK]);
            }
        }
    }
    const uint32_t* B = fl.block.data();
    printf("rows %u granules %u deep_g %u | lanes %d seg %d L2 %d KiB, KR %d\n", F, fl.granules, fl.deep_g, LANES, SEG,
           L2KB, KR);
    // layout 2: records of one slot whose target is the next record (a
    // unary chain, word on c0 -> granule + 1) with a fallback rank < 2047
    // packed in 4 B instead of 8 (byte offsets below)
    std::vector<uint64_t> roff(fl.granules + 1, 0);
    {
        const uint32_t* R = B + (size_t)F * 256;
        uint64_t off = 0;
        uint32_t gr = 0;
        while (gr < fl.granules) {
            const uint32_t w0 = R[2 * (size_t)gr], w1 = R[2 * (size_t)gr + 1];
            const bool one = ((w0 >> 16) & 0xFFu) == (w0 >> 24);
            const uint32_t t = w1 & PM_DFA_STATE_MASK;
            const bool chain = one && t == F + gr + 1 && (w1 >> 20) < 2047;
            roff[gr] = off;
            off += chain ? 4 : 8;
            ++gr;
        }
        roff[fl.granules] = off;
        printf("compact chains: records %.2f MB -> %.2f MB\n", fl.granules * 8 / 1e6, off / 1e6);
    }
    // LDS row sets: the product's first KR rows, or (layouts 5, 6) the root
    // and the KR-1 rows visited most on a separate sample of the same text
    // (every row step and record-miss fallback counted)
    std::vector<uint8_t> inlds(F, 0);
    for (uint32_t r = 0; r < F && (int)r < KR; ++r) inlds[r] = 1;
    std::vector<uint8_t> inlds_v(F, 0);
    {
        std::vector<uint64_t> vis(F, 0);
        std::vector<uint32_t> w;
        // the profile sample (MIX=1, the product's choice): 256 lanes of
        // the dictionary's lines text and 256 of random printable ASCII,
        // 4 KiB each, from offsets the evaluation does not use; else a
        // quarter of the evaluation lanes themselves
        const int MIX = envi("MIX", 1);
        std::vector<std::vector<uint8_t>> smp;
        if (MIX) {
            std::vector<uint8_t> blk(PM_LINES_BLOCK);
            for (int L = 0; L < 512; ++L) {
                std::vector<uint8_t> t;
                const uint64_t lo = (1ull << 40) + (uint64_t)L * (1 << 20);
                for (uint64_t p = lo; p < lo + WARM + SEG; ++p) {
                    if (L < (MIX == 2 ? 512 : envi("MIXL", 256))) {
                        if (p % PM_LINES_BLOCK == 0 || p == lo)
                            pm_lines_block(blk.data(), PM_LINES_BLOCK, p / PM_LINES_BLOCK, P.data(), O.data(), pats.size(), 7);
                        t.push_back(blk[p % PM_LINES_BLOCK]);
                    } else {
                        t.push_back(pm_stream_byte(p, 7, 0));
                    }
                }
                smp.push_back(t);
            }
        } else {
            for (int L = 0; L < LANES; L += 4) smp.push_back(txt[L]);
        }
        w.assign(smp.size(), 0);
        for (int j = 0; j < WARM + SEG; ++j)
            for (size_t L = 0; L < smp.size(); ++L) {
                const uint32_t c = smp[L][j];
                const uint32_t s = w[L] & PM_DFA_STATE_MASK;
                if (s < F) { vis[s]++; w[L] = B[(size_t)s * 256 + c]; continue; }
                const uint32_t* U = B + (size_t)F * 256 + 2 * (size_t)(s - F);
                if (c == ((U[0] >> 16) & 0xFFu)) w[L] = U[1];
                else if (c == (U[0] >> 24)) w[L] = U[2];
                else {
                    const uint32_t fb = w[L] >> 20;
                    const uint32_t row = fb == PM_FL_FB_INREC ? U[3] : fb;
                    vis[row]++;
                    w[L] = B[(size_t)row * 256 + c];
                }
            }
        std::vector<uint32_t> ordr(F);
        for (uint32_t r = 0; r < F; ++r) ordr[r] = r;
        std::sort(ordr.begin(), ordr.end(), [&](uint32_t a, uint32_t b) { return vis[a] > vis[b]; });
        inlds_v[0] = 1;
        int k = 1;
        for (uint32_t r : ordr) {
            if (k >= KR) break;
            if (!inlds_v[r]) { inlds_v[r] = 1; ++k; }
        }
    }
    if (envi("COVER", 0)) {
        // row and fallback-row requests by (row, 128-B line), profile vs evaluation
        auto walk = [&](const std::vector<std::vector<uint8_t>>& T, std::unordered_map<uint64_t, uint64_t>& cnt) {
            std::vector<uint32_t> w(T.size(), 0);
            for (int j = 0; j < WARM + SEG; ++j)
                for (size_t L = 0; L < T.size(); ++L) {
                    const uint32_t c = T[L][j];
                    const uint32_t s = w[L] & PM_DFA_STATE_MASK;
                    uint32_t row = s;
                    if (s >= F) {
                        const uint32_t* U = B + (size_t)F * 256 + 2 * (size_t)(s - F);
                        if (c == ((U[0] >> 16) & 0xFFu)) { w[L] = U[1]; continue; }
                        if (c == (U[0] >> 24)) { w[L] = U[2]; continue; }
                        const uint32_t fb = w[L] >> 20;
                        row = fb == PM_FL_FB_INREC ? U[3] : fb;
                    }
                    if (row != 0 && j >= WARM) cnt[(uint64_t)row * 8 + (c >> 5)]++;
                    w[L] = B[(size_t)row * 256 + c];
                }
        };
        std::vector<std::vector<uint8_t>> prof;
        {
            std::vector<uint8_t> blk(PM_LINES_BLOCK);
            for (int L = 0; L < 512; ++L) {
                std::vector<uint8_t> t;
                const uint64_t lo = (1ull << 40) + (uint64_t)L * (1 << 20);
                for (uint64_t p = lo; p < lo + WARM + SEG; ++p) {
                    if (L < 480) {
                        if (p % PM_LINES_BLOCK == 0 || p == lo)
                            pm_lines_block(blk.data(), PM_LINES_BLOCK, p / PM_LINES_BLOCK, P.data(), O.data(), pats.size(), 7);
                        t.push_back(blk[p % PM_LINES_BLOCK]);
                    } else t.push_back(pm_stream_byte(p, 7, 0));
                }
                prof.push_back(t);
            }
        }
        std::unordered_map<uint64_t, uint64_t> pc, ec;
        walk(prof, pc);
        walk(txt, ec);
        uint64_t tot = 0;
        for (auto& x : ec) tot += x.second;
        // whole rows: top K by profile visits (sum over lines), lines: top N pairs
        std::unordered_map<uint32_t, uint64_t> rv;
        for (auto& x : pc) rv[(uint32_t)(x.first / 8)] += x.second;
        std::vector<std::pair<uint64_t, uint32_t>> rows;
        for (auto& x : rv) rows.push_back({x.second, x.first});
        std::sort(rows.rbegin(), rows.rend());
        std::vector<std::pair<uint64_t, uint64_t>> lns;
        for (auto& x : pc) lns.push_back({x.second, x.first});
        std::sort(lns.rbegin(), lns.rend());
        for (int K : {87, 150}) {
            std::unordered_map<uint32_t, int> in;
            for (int k = 0; k < K && k < (int)rows.size(); ++k) in[rows[k].second] = 1;
            uint64_t cov = 0;
            for (auto& x : ec) if (in.count((uint32_t)(x.first / 8))) cov += x.second;
            printf("whole rows %d (%d KiB): %.1f%% of non-root row requests\n", K, K, 100.0 * cov / tot);
        }
        for (int K : {234, 300}) {  // rows' printable lines only (bytes 32-127: 3 lines, 384 B a row)
            std::unordered_map<uint32_t, int> in;
            for (int k = 0; k < K && k < (int)rows.size(); ++k) in[rows[k].second] = 1;
            uint64_t cov = 0;
            for (auto& x : ec) {
                const uint32_t ln = (uint32_t)(x.first % 8);
                if (in.count((uint32_t)(x.first / 8)) && ln >= 1 && ln <= 3) cov += x.second;
            }
            printf("printable lines of %d rows (%d KiB): %.1f%% of non-root row requests\n", K, K * 3 / 8, 100.0 * cov / tot);
        }
        for (int N : {340, 680, 1200}) {
            std::unordered_map<uint64_t, int> in;
            for (int k = 0; k < N && k < (int)lns.size(); ++k) in[lns[k].second] = 1;
            uint64_t cov = 0;
            for (auto& x : ec) if (in.count(x.first)) cov += x.second;
            printf("row lines %d (%d KiB): %.1f%% of non-root row requests\n", N, N / 8, 100.0 * cov / tot);
        }
        return 0;
    }
    for (int layout = 0; layout < 8; ++layout) {
        const std::vector<uint8_t>& lds = layout == 5 ? inlds_v : inlds;
        Lru l2{(size_t)L2KB * 1024 / 128};
        uint64_t rowreq = 0, recreq = 0, fbreq = 0, steps = 0, rowmiss = 0, recmiss = 0, fbmiss = 0;
        std::unordered_map<uint64_t, uint64_t> lines;
        std::vector<uint32_t> w(LANES, 0), key(LANES, ~0u), ws(LANES, ~0u);
        auto col = [&](uint32_t c) { return layout == 1 ? perm[c] : c; };
        auto rowline = [&](uint32_t r, uint32_t c) { return ((uint64_t)r * 1024 + col(c) * 4) / 128; };
        for (int j = 0; j < WARM + SEG; ++j) {
            const bool cnt = j >= WARM;
            for (int L = 0; L < LANES; ++L) {
                const uint32_t c = txt[L][j];
                const uint32_t s = w[L] & PM_DFA_STATE_MASK;
                uint32_t nw;
                if (s < F) {
                    if (!lds[s]) {
                        const uint64_t a = rowline(s, c);
                        const bool h = l2.touch(a);
                        if (cnt) { ++rowreq; rowmiss += !h; lines[a]++; }
                    }
                    nw = B[(size_t)s * 256 + c];
                } else {
                    const uint32_t gr = s - F;
                    const bool deep = gr >= fl.deep_g;
                    // layouts 6 / 7: deep records in forward windows of 4 / 8
                    // halves (64 / 128 B) from the record's own half
                    if (layout >= 6 && deep) {
                        const uint32_t hh = gr >> 1, NH = layout == 6 ? 4 : 8;
                        if (!(ws[L] != ~0u && hh >= ws[L] && hh < ws[L] + NH)) {
                            ws[L] = hh;
                            key[L] = ~0u;
                            const uint64_t b0 = (uint64_t)hh * 16, b1 = b0 + NH * 16 - 1;
                            for (uint64_t ln = b0 / 128; ln <= b1 / 128; ++ln) {
                                const bool h = l2.touch((1ull << 40) + ln);
                                if (cnt) { ++recreq; recmiss += !h; lines[(1ull << 40) + ln]++; }
                            }
                        }
                    } else if (layout >= 6) ws[L] = ~0u;
                    if (!(layout >= 6 && deep)) {
                    // layouts 3 / 4: deep records in 64-B / 128-B blocks
                    const uint32_t k = deep ? (gr >> (layout == 3 ? 3 : layout == 4 ? 4 : 2)) | 0x80000000u : gr >> 1;
                    const uint64_t kk = layout == 2 ? roff[gr] / 32 : k;  // (layout 2: 32-B blocks by byte offset)
                    if (kk != key[L]) {
                        key[L] = (uint32_t)kk;
                        const uint64_t a = (1ull << 40) + (layout == 2 ? roff[gr] : (uint64_t)gr * 8) / 128;
                        const bool h = l2.touch(a);
                        if (cnt) { ++recreq; recmiss += !h; lines[a]++; }
                    }
                    }
                    const uint32_t* U = B + (size_t)F * 256 + 2 * (size_t)gr;
                    if (c == ((U[0] >> 16) & 0xFFu)) nw = U[1];
                    else if (c == (U[0] >> 24)) nw = U[2];
                    else {
                        const uint32_t fb = w[L] >> 20;
                        const uint32_t row = fb == PM_FL_FB_INREC ? U[3] : fb;
                        if (!lds[row]) {
                            const uint64_t a = rowline(row, c);
                            const bool h = l2.touch(a);
                            if (cnt) { ++fbreq; fbmiss += !h; lines[a]++; }
                        }
                        nw = B[(size_t)row * 256 + c];
                    }
                }
                w[L] = nw;
                if (cnt) ++steps;
            }
        }
        std::vector<uint64_t> h;
        for (auto& x : lines) h.push_back(x.second);
        std::sort(h.rbegin(), h.rend());
        uint64_t tot = 0;
        for (auto x : h) tot += x;
        uint64_t acc = 0;
        size_t n50 = 0, n90 = 0, n99 = 0;
        for (size_t k = 0; k < h.size(); ++k) {
            acc += h[k];
            if (!n50 && acc >= tot / 2) n50 = k + 1;
            if (!n90 && acc >= tot * 9 / 10) n90 = k + 1;
            if (!n99 && acc >= tot * 99 / 100) n99 = k + 1;
        }
        printf("%s: per step: row %.3f fallback %.3f record %.3f requests; L2 misses per step %.3f (row %.3f fb %.3f rec %.3f)\n"
               "   lines touched %zu (%.1f MB); 50/90/99%% of requests in %.2f / %.2f / %.2f MB\n",
               layout == 7 ? "deep 128-B forward windows" : layout == 6 ? "deep 64-B forward windows" : layout == 5 ? "LDS rows by visits" : layout == 4 ? "deep 128-B blocks" : layout == 3 ? "deep 64-B blocks" : layout == 2 ? "compact chains" : layout ? "permuted columns" : "product", (double)rowreq / steps, (double)fbreq / steps,
               (double)recreq / steps, (double)(rowmiss + fbmiss + recmiss) / steps, (double)rowmiss / steps,
               (double)fbmiss / steps, (double)recmiss / steps, h.size(), h.size() * 128 / 1e6, n50 * 128 / 1e6,
               n90 * 128 / 1e6, n99 * 128 / 1e6);
    }
    return 0;
}
