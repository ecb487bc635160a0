// sdfa_l2_model.cpp -- probe (not product): an LRU model of one XCD's 4 MiB L2 over
// 16,384 interleaved lanes scanning the lines stream through the sparse AC-DFA,
// for default-transition records of up to K = 2 / 12 / 28 slots (MEASUREMENTS.md §4).
//   g++ -O2 -std=c++17 -Ipatternmatching_amd/csrc -Iinclude scripts/sdfa_l2_model.cpp \
//       patternmatching_amd/csrc/pm_flatten.cpp patternmatching_amd/csrc/host/pm_dict.c -o /tmp/l2 && /tmp/l2 DICT...
#include "pm_flatten.h"
#include "pm_streamgen.h"
#include <algorithm>
#include <cstdio>
#include <fstream>
#include <list>
#include <map>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>
extern "C" size_t pm_parse_line(const unsigned char* line, size_t n, unsigned char* out);
struct LRU { size_t cap; std::list<uint64_t> l; std::unordered_map<uint64_t, std::list<uint64_t>::iterator> m; uint64_t hit = 0, miss = 0;
  void touch(uint64_t k) { auto it = m.find(k); if (it != m.end()) { ++hit; l.splice(l.begin(), l, it->second); return; } ++miss; l.push_front(k); m[k] = l.begin(); if (m.size() > cap) { m.erase(l.back()); l.pop_back(); } } };
int main(int argc, char** argv) {
    std::vector<std::string> pats;
    for (int a = 1; a < argc; ++a) {
        std::ifstream f(argv[a]); std::string line; std::vector<unsigned char> buf(1 << 16);
        while (std::getline(f, line)) { size_t k = pm_parse_line((const unsigned char*)line.data(), line.size(), buf.data()); if (k) pats.emplace_back((char*)buf.data(), k); }
    }
    { std::vector<std::string> u; std::map<std::string,int> m; for (auto& p : pats) if (!m.count(p)) { m[p]=1; u.push_back(p);} pats = u; }
    PmGidMap g = pm_assign_gids(pats);
    DfaImage d = pm_build_dfa(pats, g);
    const uint32_t S = d.states;
    auto nx = [&](uint32_t v, uint32_t c) { return d.next[(size_t)v * 256 + c] & 0xFFFFF; };
    std::vector<int> depth(S, -1); std::vector<uint32_t> q{0}; depth[0] = 0; std::vector<uint32_t> order;
    for (size_t h = 0; h < q.size(); ++h) { uint32_t v = q[h]; order.push_back(v); for (uint32_t c = 0; c < 256; ++c) { uint32_t u = nx(v, c); if (depth[u] < 0) { depth[u] = depth[v] + 1; q.push_back(u); } } }
    std::vector<uint32_t> fail(S, 0); std::vector<std::vector<uint8_t>> kids(S);
    for (uint32_t v : order) for (uint32_t c = 0; c < 256; ++c) { uint32_t u = nx(v, c); if (depth[u] == depth[v] + 1) { kids[v].push_back(c); fail[u] = depth[v] == 0 ? 0 : nx(fail[v], c); } }
    // lines stream, 16384 lanes x 512 bytes each (8 MiB)
    const size_t LANES = 16384, PER = 512, n = LANES * PER;
    std::vector<uint8_t> t(n);
    std::vector<uint8_t> P; std::vector<uint32_t> O(1, 0);
    for (auto& p : pats) { P.insert(P.end(), p.begin(), p.end()); O.push_back(P.size()); }
    for (uint64_t lo = 0, b = 0; lo < n; lo += PM_LINES_BLOCK, ++b) pm_lines_block(t.data() + lo, std::min<uint64_t>(n - lo, PM_LINES_BLOCK), b, P.data(), O.data(), pats.size(), 1);
    for (uint32_t K : {2u, 12u, 28u}) {
        std::vector<std::vector<uint8_t>> D(S); std::vector<char> isrow(S, 0); std::vector<uint32_t> fb(S, 0);
        for (uint32_t v : order) {
            if (v == 0) { isrow[v] = 1; continue; }
            std::set<uint8_t> s(kids[v].begin(), kids[v].end());
            if (!isrow[fail[v]]) s.insert(D[fail[v]].begin(), D[fail[v]].end());
            if (s.size() > K) isrow[v] = 1; else { D[v].assign(s.begin(), s.end()); fb[v] = isrow[fail[v]] ? fail[v] : fb[fail[v]]; }
        }
        // addresses: rows first (order of state id), then records in id order, size 16 B (<=2) or 64 B
        std::vector<uint64_t> addr(S); uint64_t a = 0; uint64_t rows = 0;
        for (uint32_t v = 0; v < S; ++v) if (isrow[v]) { addr[v] = a; a += 1024; ++rows; }
        uint64_t rowbytes = a;
        for (uint32_t v = 0; v < S; ++v) if (!isrow[v]) { addr[v] = a; a += D[v].size() <= 2 ? 16 : 64; }
        LRU l2{32768}; // 4 MiB of 128-B lines
        std::vector<uint32_t> st(LANES, 0);
        uint64_t loads = 0;
        for (size_t j = 0; j < PER; ++j) for (size_t L = 0; L < LANES; ++L) {
            uint32_t s = st[L], c = t[L * PER + j];
            if (isrow[s]) { l2.touch((addr[s] + c * 4) / 128); ++loads; }
            else { l2.touch(addr[s] / 128); ++loads; if (!std::binary_search(D[s].begin(), D[s].end(), (uint8_t)c)) { l2.touch((addr[fb[s]] + c * 4) / 128); ++loads; } }
            st[L] = nx(s, c);
        }
        printf("K=%2u rows %lu (%.1f MB) records %.1f MB: loads/byte %.3f, L2(4MB LRU) misses/byte %.3f, hit %.3f\n", K, rows, rowbytes / 1e6, (a - rowbytes) / 1e6, loads / (double)n, l2.miss / (double)n, l2.hit / (double)(l2.hit + l2.miss));
    }
}
