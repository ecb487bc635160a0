// pm_flatten.cpp -- see pm_flatten.h.
#include "pm_flatten.h"
#include "pm_streamgen.h"

#include <algorithm>
#include <array>
#include <cstdio>
#include <sys/stat.h>
#include <unistd.h>
#include <cstring>
#include <unordered_map>

namespace {

// A numbered byte trie: node 0 is the root, the children of a node are
// contiguous ids [cstart, cstart+ccount) sorted by edge byte, a parent's id
// is below its children's, and (build_trie) the first levels are in BFS
// order.
struct BfsTrie {
    uint32_t n = 0;
    std::vector<uint32_t> cstart, ccount, parent, gid, depth;
    std::vector<uint8_t> label;  // edge byte from the parent

    uint32_t child(uint32_t v, uint32_t c) const {
        uint32_t lo = cstart[v], hi = lo + ccount[v];
        while (lo < hi) {
            uint32_t mid = (lo + hi) >> 1;
            if (label[mid] < c) lo = mid + 1;
            else hi = mid;
        }
        return (lo < cstart[v] + ccount[v] && label[lo] == c) ? lo : 0;
    }
};

// dfs_depth: nodes of depth <= dfs_depth are numbered breadth-first (all
// of depth d before any of depth d+1); deeper ones get "children blocks in
// depth-first order": visiting a node allocates its children's contiguous
// block, then visits them first to last.  A unary chain's nodes are then
// consecutive ids, so a walk down it reads consecutive 16-B records (8 to a
// cache line) instead of one line per step.
BfsTrie build_trie(const std::vector<std::string>& pats, const PmGidMap& g, bool reversed,
                   uint32_t dfs_depth = UINT32_MAX) {
    // creation-order trie with a hash map of edges
    std::unordered_map<uint64_t, uint32_t> edge;
    size_t total = 0;
    for (const auto& p : pats) total += p.size();
    edge.reserve(total + 16);
    std::vector<uint32_t> gid(1, 0);
    uint32_t n = 1;
    for (size_t k = 0; k < pats.size(); ++k) {
        const std::string& p = pats[k];
        uint32_t cur = 0;
        for (size_t t = 0; t < p.size(); ++t) {
            uint8_t c = (uint8_t)(reversed ? p[p.size() - 1 - t] : p[t]);
            uint64_t key = ((uint64_t)cur << 8) | c;
            auto it = edge.find(key);
            if (it == edge.end()) {
                edge.emplace(key, n);
                gid.push_back(0);
                cur = n++;
            } else {
                cur = it->second;
            }
        }
        // a repeated byte string keeps the id added last, as ac_add_pattern
        // does (mpac.c:272 `cur->id = id`); the earlier gid has no node
        if (!p.empty()) gid[cur] = g.gid_of_index[k];
    }
    // children lists by creation id, sorted by byte
    std::vector<uint64_t> kids;  // (parent << 40) | (byte << 32) | child
    kids.reserve(edge.size());
    for (const auto& e : edge) kids.push_back(((e.first >> 8) << 40) | ((e.first & 0xFF) << 32) | e.second);
    std::sort(kids.begin(), kids.end());
    std::vector<uint32_t> kstart(n + 1, 0);
    for (uint64_t x : kids) kstart[(x >> 40) + 1]++;
    for (uint32_t v = 0; v < n; ++v) kstart[v + 1] += kstart[v];
    // renumbering: a node's fields are set when it is expanded (its
    // children block allocated)
    BfsTrie t;
    t.n = n;
    t.cstart.assign(n, 0);
    t.ccount.assign(n, 0);
    t.parent.assign(n, 0);
    t.gid.assign(n, 0);
    t.depth.assign(n, 0);
    t.label.assign(n, 0);
    std::vector<uint32_t> order;  // new id -> creation id
    order.reserve(n);
    order.push_back(0);
    auto expand = [&](uint32_t v) {
        const uint32_t old = order[v];
        t.gid[v] = gid[old];
        t.cstart[v] = (uint32_t)order.size();
        t.ccount[v] = kstart[old + 1] - kstart[old];
        for (uint32_t k = kstart[old]; k < kstart[old + 1]; ++k) {
            const uint32_t nv = (uint32_t)order.size();
            t.parent[nv] = v;
            t.label[nv] = (uint8_t)((kids[k] >> 32) & 0xFF);
            t.depth[nv] = t.depth[v] + 1;
            order.push_back((uint32_t)(kids[k] & 0xFFFFFFFFu));
        }
    };
    std::vector<uint32_t> deep;  // nodes at dfs_depth, in breadth-first order
    for (size_t h = 0; h < order.size(); ++h) {
        const uint32_t v = (uint32_t)h;
        if (t.depth[v] < dfs_depth) expand(v);
        else deep.push_back(v);
    }
    std::vector<uint32_t> stack;
    for (uint32_t r : deep) {
        stack.push_back(r);
        while (!stack.empty()) {
            const uint32_t v = stack.back();
            stack.pop_back();
            expand(v);
            for (uint32_t k = t.ccount[v]; k-- > 0;) stack.push_back(t.cstart[v] + k);  // first child on top
        }
    }
    return t;
}

// The LDS filters are a function of t12, t3h and rec: stage 1 holds every
// depth-3 key (every valid t3h entry); stage 2 the keys whose depth-3 node
// is a pattern (its best-so-far differs from the depth-2 answer, gids being
// unique per node) and every depth-4 suffix (the node's children: inline
// bytes or its record's bitmap).  The build derives them this way and a
// cached image must reproduce them exactly, so the filters can never drift
// from the tables or the hash functions.
std::vector<uint32_t> derive_filters(const RtImage& im) {
    std::vector<uint32_t> filt(RT_FILTER_WORDS + RT_F2_WORDS, 0);
    uint32_t* f2 = &filt[RT_FILTER_WORDS];
    for (size_t e = 0; e + 3 < im.t3h.size(); e += 4) {
        const uint32_t x = im.t3h[e], y = im.t3h[e + 1], z = im.t3h[e + 2], w = im.t3h[e + 3];
        if (!(x & RT_T3H_VALID)) continue;
        const uint32_t key = x & 0xFFFFFFu, kind = x >> 25;
        const uint32_t f = pm_rt_fhash(key);
        filt[pm_rt_filter_word(f)] |= pm_rt_filter_mask(f);
        if ((key >> 8) < im.t12.size() && y != (im.t12[key >> 8] & (RT_CONT16 - 1))) {
            const uint32_t g = pm_rt_p3hash(key);
            f2[pm_rt_p3word(g)] |= pm_rt_filter_mask(g);
        }
        auto s4 = [&](uint32_t c) {
            const uint32_t g = pm_rt_s4hash(c | (key << 8));
            f2[pm_rt_s4word(g)] |= pm_rt_filter_mask(g);
        };
        if (kind == 1) {
            for (uint32_t j = 0; j < (z >> 24) && j < RT_T3H_INLINE; ++j) s4((z >> (8 * j)) & 0xFFu);
        } else if (kind == 2) {
            const size_t r = (size_t)(w & ~RT_CONT32) * RT_REC_WORDS;
            if (r + RT_REC_WORDS > im.rec.size()) continue;
            const uint32_t* R = &im.rec[r];
            const uint32_t rk = R[0] >> 30;
            if (rk == RT_REC_KIDS) {
                for (uint32_t j = 0; j < ((R[0] >> 24) & 63u) && j < RT_REC_INLINE; ++j) s4((R[2 + j / 4] >> (8 * (j & 3))) & 0xFFu);
            } else if (rk == RT_REC_CHAIN) {
                s4(R[3] >> 24);
            } else if (rk == RT_REC_WIDE && (size_t)(R[2] + 1) * RT_WIDE_WORDS <= im.wide.size()) {
                const uint32_t* W = &im.wide[(size_t)R[2] * RT_WIDE_WORDS];
                for (uint32_t c = 0; c < 256; ++c)
                    if ((W[pm_rt_wide_word(c >> 5)] >> (c & 31)) & 1u) s4(c);
            }
        }
    }
    return filt;
}

}  // namespace

PmGidMap pm_assign_gids(const std::vector<std::string>& pats) {
    PmGidMap g;
    const size_t P = pats.size();
    g.gid_of_index.assign(P, 0);
    g.index_of_gid.assign(1, 0);
    g.index_of_gid.reserve(P + 1);
    // Patterns of <= 2 bytes first (the reverse trie's depth-2 answers are
    // 15-bit gids below RT_CONT16), then the rest by how often each is a
    // position's output, most often first: the coded DFA words carry gids <
    // DFA_ESC inline, and a larger one is an escape, looked up per position
    // (the sparse kernels' largest single cost on pattern-dense input).
    // The weight of pattern p: over the trie states whose output (the
    // longest pattern that is a suffix of the state's string, mpac.c:272's
    // rule) is p, the number of patterns below the state -- how often
    // pattern-dense text, which walks the patterns' own paths, visits them.
    // Share of the nonzero outputs that escape, 16 MiB of snort (lines
    // stream / shipped stream): add order 13.7% / 11.3%, by length 9.8% /
    // 6.1%, by this weight 5.1% / 1.4% (the best any order reaches on the
    // lines stream is 5.0%); random ASCII ~0 in every order.
    std::unordered_map<uint64_t, uint32_t> edge;
    size_t total = 0;
    for (const auto& p : pats) total += p.size();
    edge.reserve(total + 1);
    std::vector<uint32_t> parent(1, 0);
    std::vector<uint8_t> inbyte(1, 0);
    std::vector<uint16_t> depth(1, 0);
    std::vector<int64_t> term(1, -1);
    for (size_t k = 0; k < P; ++k) {
        uint32_t v = 0;
        for (unsigned char c : pats[k]) {
            const uint64_t key = (uint64_t)v << 8 | c;
            auto it = edge.find(key);
            if (it == edge.end()) {
                const uint32_t w = (uint32_t)parent.size();
                edge.emplace(key, w);
                parent.push_back(v);
                inbyte.push_back(c);
                depth.push_back((uint16_t)std::min<size_t>(depth[v] + 1, 65535));
                term.push_back(-1);
                v = w;
            } else {
                v = it->second;
            }
        }
        if (!pats[k].empty()) term[v] = (int64_t)k;  // a repeated pattern: the later one is the output
    }
    const uint32_t N = (uint32_t)parent.size();
    std::vector<uint64_t> sub(N, 0);  // patterns at or below each state (a child's id exceeds its parent's)
    for (uint32_t v = 0; v < N; ++v) sub[v] = term[v] >= 0;
    for (uint32_t v = N; v-- > 1;) sub[parent[v]] += sub[v];
    std::vector<uint32_t> bfs(N);
    for (uint32_t v = 0; v < N; ++v) bfs[v] = v;
    std::stable_sort(bfs.begin(), bfs.end(), [&](uint32_t a, uint32_t b) { return depth[a] < depth[b]; });
    std::vector<uint32_t> fail(N, 0);
    std::vector<int64_t> outp(N, -1);
    std::vector<uint64_t> weight(P, 0);
    for (uint32_t v : bfs) {
        if (v == 0) continue;
        const uint32_t p = parent[v];
        if (p != 0) {
            uint32_t f = fail[p];
            for (;;) {
                auto it = edge.find((uint64_t)f << 8 | inbyte[v]);
                if (it != edge.end()) {
                    fail[v] = it->second;
                    break;
                }
                if (f == 0) break;
                f = fail[f];
            }
        }
        outp[v] = term[v] >= 0 ? term[v] : outp[fail[v]];
        if (outp[v] >= 0) weight[(size_t)outp[v]] += sub[v];
    }
    std::vector<uint32_t> order(P);
    for (size_t k = 0; k < P; ++k) order[k] = (uint32_t)k;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        const bool sa = pats[a].size() <= 2, sb = pats[b].size() <= 2;
        if (sa != sb) return sa;
        if (sa) return false;  // add order among the short ones
        if (weight[a] != weight[b]) return weight[a] > weight[b];
        return pats[a].size() < pats[b].size();
    });
    for (uint32_t k : order) {
        g.gid_of_index[k] = (uint32_t)g.index_of_gid.size();
        g.index_of_gid.push_back(k);
    }
    return g;
}

RtImage pm_build_rt(const std::vector<std::string>& pats, const PmGidMap& g) {
    RtImage im;
    BfsTrie t = build_trie(pats, g, /*reversed=*/true, /*dfs_depth=*/3);
    im.nodes = t.n;
    // best pattern on the path root..v (deepest pattern node, inclusive)
    std::vector<uint32_t> best(t.n, 0);
    for (uint32_t v = 1; v < t.n; ++v) best[v] = t.gid[v] ? t.gid[v] : best[t.parent[v]];

    uint32_t n_short = 0;
    for (const auto& p : pats) n_short += p.size() <= 2;
    // depth-2 internal nodes, in BFS order, and the first depth-3 node
    std::vector<uint32_t> n2i(t.n, UINT32_MAX);
    uint32_t first_d3 = t.n;
    for (uint32_t v = 1; v < t.n; ++v) {
        if (t.depth[v] == 2 && t.ccount[v]) n2i[v] = im.n2int++;
        if (t.depth[v] >= 3 && first_d3 == t.n) first_d3 = v;
    }
    im.nrec = t.n - first_d3;
    uint32_t max_len = 0;
    for (const auto& p : pats) max_len = std::max<uint32_t>(max_len, (uint32_t)p.size());
    im.fits = n_short < RT_CONT16 && im.nrec < (1u << 23) && max_len <= 511;
    // (nwide < 2^14 is checked after the records are built)
    if (!im.fits) return im;

    im.t12.assign(RT_T1_BASE + 256, 0);
    for (uint32_t c0 = 0; c0 < 256; ++c0) {
        uint32_t n1 = t.child(0, c0);
        im.t12[RT_T1_BASE + c0] = (uint16_t)(n1 ? best[n1] : 0);
        for (uint32_t c1 = 0; c1 < 256; ++c1) {
            uint32_t v = 0;
            if (n1) {
                uint32_t n2 = t.child(n1, c1);
                if (!n2) v = best[n1];
                else v = (t.ccount[n2] ? RT_CONT16 : 0u) | best[n2];
            }
            im.t12[(c0 << 8) | c1] = (uint16_t)v;
        }
    }
    // depth-3 suffixes: filter bits + a two-choice cuckoo table (each key in
    // slot h1 or h2, so a lookup is two independent loads and no chain)
    uint32_t d3 = 0;
    for (uint32_t v = 1; v < t.n && t.depth[v] <= 2; ++v)
        if (t.depth[v] == 2) d3 += t.ccount[v];
    auto answer = [&](uint32_t v) { return t.ccount[v] ? (RT_CONT32 | (v - first_d3)) : best[v]; };
    std::vector<std::array<uint32_t, 4>> ents;
    ents.reserve(d3);
    for (uint32_t v = 1; v < t.n && t.depth[v] <= 2; ++v) {
        if (t.depth[v] != 2 || !t.ccount[v]) continue;
        const uint32_t c0 = t.label[t.parent[v]], c1 = t.label[v];
        for (uint32_t k = 0; k < t.ccount[v]; ++k) {
            const uint32_t n3 = t.cstart[v] + k;
            const uint32_t c2 = t.label[n3];
            const uint32_t key = c2 | (c1 << 8) | (c0 << 16);
            std::array<uint32_t, 4> e{};
            const uint32_t nch = t.ccount[n3];
            const uint32_t kind = nch == 0 ? 0u : (nch <= RT_T3H_INLINE ? 1u : 2u);
            e[0] = (kind << 25) | RT_T3H_VALID | key;
            e[1] = best[n3];
            if (kind == 1) {
                // up to three child bytes inline; the child's answer inline
                // for one child, else the first child's record (contiguous)
                e[2] = nch << 24;
                for (uint32_t j = 0; j < nch; ++j) e[2] |= (uint32_t)t.label[t.cstart[n3] + j] << (8 * j);
                e[3] = nch == 1 ? answer(t.cstart[n3]) : t.cstart[n3] - first_d3;
            } else if (kind == 2) {
                e[3] = RT_CONT32 | (n3 - first_d3);
            }
            ents.push_back(e);
        }
    }
    im.d3 = (uint32_t)ents.size();
    // load <= 1/4: few keys need their slot2 (the device probes slot1 first)
    for (im.t3h_bits = 4; (1u << im.t3h_bits) < 4 * im.d3; ++im.t3h_bits) {}
    for (;; ++im.t3h_bits) {  // load <= 1/2: two-choice cuckoo insertion virtually never fails; grow if it does
        const uint32_t bits = im.t3h_bits;
        im.t3h.assign((size_t)4 << bits, 0);
        bool ok = true;
        auto empty = [&](uint32_t sl) { return !(im.t3h[4 * (size_t)sl] & RT_T3H_VALID); };
        for (size_t q = 0; q < ents.size() && ok; ++q) {
            std::array<uint32_t, 4> cur = ents[q];
            const uint32_t k = cur[0] & 0xFFFFFFu;
            uint32_t slot = pm_rt_slot1(k, bits);
            if (!empty(slot) && empty(pm_rt_slot2(k, bits))) slot = pm_rt_slot2(k, bits);
            // cuckoo walk: take the slot, re-home its occupant in its other slot
            for (int kick = 0;; ++kick) {
                uint32_t* e = &im.t3h[4 * (size_t)slot];
                std::array<uint32_t, 4> ev;
                std::memcpy(ev.data(), e, 16);
                std::memcpy(e, cur.data(), 16);
                if (!(ev[0] & RT_T3H_VALID)) break;
                if (kick > 1000) { ok = false; break; }
                cur = ev;
                const uint32_t ke = cur[0] & 0xFFFFFFu;
                const uint32_t e1 = pm_rt_slot1(ke, bits), e2 = pm_rt_slot2(ke, bits);
                slot = slot == e1 ? e2 : e1;
            }
        }
        if (ok) break;
    }
    // 16-B node records (pm_flatten.h): children inline up to RT_REC_INLINE,
    // else a 64-B bitmap-rank entry in `wide`
    im.rec.assign((size_t)im.nrec * RT_REC_WORDS, 0);
    im.nwide = 0;
    for (uint32_t v = first_d3; v < t.n; ++v) {
        uint32_t* R = &im.rec[(size_t)(v - first_d3) * RT_REC_WORDS];
        const uint32_t nch = t.ccount[v], first = nch ? t.cstart[v] - first_d3 : 0;
        R[1] = best[v];
        if (nch == 0) {
            R[0] = RT_REC_LEAF << 30;
        } else if (nch == 1) {
            // the run below v: consecutive one-child records, no pattern inside
            uint32_t L = 1, w = t.cstart[v];
            uint64_t P = (uint64_t)t.label[w] << 56;
            while (L < RT_CHAIN_MAX && t.ccount[w] == 1 && t.cstart[w] == w + 1 && !t.gid[w]) {
                P |= (uint64_t)t.label[w + 1] << (8 * (7 - L));
                ++L;
                ++w;
            }
            R[0] = (RT_REC_CHAIN << 30) | (L << 24) | first;
            R[2] = (uint32_t)P;
            R[3] = (uint32_t)(P >> 32);
        } else if (nch <= RT_REC_INLINE) {
            R[0] = (RT_REC_KIDS << 30) | (nch << 24) | first;
            for (uint32_t j = 0; j < nch; ++j) R[2 + j / 4] |= (uint32_t)t.label[t.cstart[v] + j] << (8 * (j & 3));
        } else {
            R[0] = (RT_REC_WIDE << 30) | first;
            R[2] = im.nwide++;
            const size_t base = im.wide.size();
            im.wide.resize(base + RT_WIDE_WORDS, 0);
            uint32_t* W = &im.wide[base];
            for (uint32_t k = 0; k < nch; ++k) {
                const uint32_t c = t.label[t.cstart[v] + k];
                W[pm_rt_wide_word(c >> 5)] |= 1u << (c & 31);
            }
            uint32_t idx = first;
            for (int q = 0; q < 4; ++q) {  // quarter q: words 2q, 2q+1
                W[4 * q + 2] = idx;
                W[4 * q + 3] = best[v];
                idx += (uint32_t)__builtin_popcount(W[4 * q]) + (uint32_t)__builtin_popcount(W[4 * q + 1]);
            }
        }
    }
    if (im.nwide >= (1u << 14)) {  // a queued wide step holds the entry in 14 bits
        im.fits = false;
        return im;
    }
    im.filt = derive_filters(im);
    return im;
}

PmParents pm_build_parents(const std::vector<std::string>& pats, const PmGidMap& g) {
    // In the trie of the reversed patterns the nodes above a pattern's node
    // are its suffixes, so its parent is the deepest pattern strictly above.
    BfsTrie t = build_trie(pats, g, /*reversed=*/true, /*dfs_depth=*/3);
    std::vector<uint32_t> best(t.n, 0);
    PmParents r;
    r.parent.assign(g.index_of_gid.size(), 0);
    r.depth.assign(g.index_of_gid.size(), 0);
    for (uint32_t v = 1; v < t.n; ++v) {  // BFS order: parents first
        const uint32_t up = best[t.parent[v]];
        if (t.gid[v]) {
            r.parent[t.gid[v]] = up;
            r.depth[t.gid[v]] = 1 + (up ? r.depth[up] : 0);
        }
        best[v] = t.gid[v] ? t.gid[v] : up;
    }
    // a gid shadowed by a later duplicate has no trie node and never appears
    // in a scan: a root of its own (parent 0, depth 1) keeps the tables
    // acyclic and depth == 1 + depth[parent] for every gid
    for (size_t q = 1; q < r.depth.size(); ++q)
        if (!r.depth[q]) r.depth[q] = 1;
    return r;
}

// The sparse form (pm_flatten.h).  order: states by depth, so a state's
// failure (shallower) is decided before it.  The fallback of v is fail[v]
// when that keeps a row, else fail[v]'s own fallback; then delta(v, c) =
// next[v][c] = next[fallback][c] except at the bytes where the two rows
// differ, and v becomes a record when those are at most PM_SDFA_K.  That
// set needs no row scan: row(v) differs from row(fail[v]) exactly at v's
// goto bytes (a child is one level deeper than any state on the other row),
// and row(fail[v]) from the fallback's row at fail[v]'s own set, so
// D(v) = children(v) | D(fail[v]) when fail[v] is a record, children(v)
// when it keeps a row.
static void build_sparse(DfaImage& im, const BfsTrie& t, const std::vector<uint32_t>& fail,
                         const std::vector<uint32_t>& order) {
    const uint32_t S = im.states;
    std::vector<uint32_t> fb(S, UINT32_MAX);  // fallback (old numbering) of a record; UINT32_MAX = row
    std::vector<uint32_t> slots(S, 0);         // record x word: its D bytes, ascending
    for (uint32_t v : order) {
        if (v == 0 || t.ccount[v] > PM_SDFA_K) continue;
        const uint32_t u = fail[v];
        uint32_t d[PM_SDFA_K + 1], nd = 0;
        for (uint32_t k = 0; k < t.ccount[v]; ++k) d[nd++] = t.label[t.cstart[v] + k];
        if (fb[u] != UINT32_MAX)  // fail[v] is a record: add its bytes not already there
            for (uint32_t q = 0; q < PM_SDFA_K; ++q) {
                const uint32_t x = slots[u] >> (16 * q);
                if (!(x & 0x100u)) continue;
                const uint32_t c = x & 0xFFu;
                bool have = false;
                for (uint32_t k = 0; k < nd; ++k) have |= d[k] == c;
                if (have) continue;
                if (nd == PM_SDFA_K) {
                    nd = PM_SDFA_K + 1;
                    break;
                }
                d[nd++] = c;
            }
        if (nd > PM_SDFA_K) continue;
        std::sort(d, d + nd);
        uint32_t x = 0;
        for (uint32_t k = 0; k < nd; ++k) x |= (d[k] | 0x100u) << (16 * k);
        fb[v] = fb[u] == UINT32_MAX ? u : fb[u];
        slots[v] = x;
    }
    // new ids in the trie's own order (depth-first below PM_DFA_DFS_DEPTH):
    // the records of a unary run of states are then consecutive 16-B
    // entries, eight to a 128-B line, so a walk along a pattern re-reads the
    // line it just fetched instead of one new line per byte
    std::vector<uint32_t> nid(S);
    uint32_t F = 0;
    for (uint32_t v = 0; v < S; ++v)
        if (fb[v] == UINT32_MAX) nid[v] = F++;
    uint32_t r = F;
    for (uint32_t v = 0; v < S; ++v)
        if (fb[v] != UINT32_MAX) nid[v] = r++;
    auto remap = [&](uint32_t w) { return nid[w & PM_DFA_STATE_MASK] | (w & ~PM_DFA_STATE_MASK); };
    im.sF = F;
    im.sblock.assign((size_t)F * 256 + (size_t)(S - F) * PM_SDFA_REC_WORDS, 0);
    im.sout.assign(S, 0);
    for (uint32_t v = 0; v < S; ++v) {
        im.sout[nid[v]] = im.out[v];
        const uint32_t* a = &im.next[(size_t)v * 256];
        if (fb[v] == UINT32_MAX) {
            uint32_t* row = &im.sblock[(size_t)nid[v] * 256];
            for (uint32_t c = 0; c < 256; ++c) row[c] = remap(a[c]);
            continue;
        }
        uint32_t* R = &im.sblock[(size_t)F * 256 + (size_t)(nid[v] - F) * PM_SDFA_REC_WORDS];
        const uint32_t x = slots[v];
        R[0] = x;
        R[1] = (x & 0x100u) ? remap(a[x & 0xFFu]) : 0u;
        R[2] = (x & 0x1000000u) ? remap(a[(x >> 16) & 0xFFu]) : 0u;
        R[3] = nid[fb[v]];
    }
}

bool pm_pack_sparse8(const DfaImage& d, std::vector<uint32_t>& block8, std::vector<uint32_t>& out8) {
    const uint32_t F = d.sF, S = d.states;
    if (d.sblock.empty() || F < 1 || F >= (1u << 22)) return false;
    const uint32_t* rec = d.sblock.data() + (size_t)F * 256;
    std::vector<uint32_t> nid(S);
    for (uint32_t v = 0; v < F; ++v) nid[v] = v;
    uint64_t u = 0;  // next free unit
    for (uint32_t v = F; v < S; ++v) {
        const bool two = (rec[(size_t)(v - F) * 4] & 0x1000000u) != 0;
        if (two && (u & 3) == 3) ++u;  // keep both units in one aligned 32-B (so also 64-B) block
        nid[v] = F + (uint32_t)u;
        u += two ? 2 : 1;
        if (F + u > PM_DFA_STATE_MASK + 1) return false;
    }
    auto remap = [&](uint32_t w) { return nid[w & PM_DFA_STATE_MASK] | (w & ~PM_DFA_STATE_MASK); };
    block8.assign((size_t)F * 256 + 2 * u, 0);
    out8.assign(F + u, 0);
    for (size_t e = 0; e < (size_t)F * 256; ++e) block8[e] = remap(d.sblock[e]);
    for (uint32_t v = 0; v < S; ++v) out8[nid[v]] = d.sout[v];
    for (uint32_t v = F; v < S; ++v) {
        const uint32_t* R = rec + (size_t)(v - F) * 4;  // {x, y, z, w}
        uint32_t* U = &block8[(size_t)F * 256 + 2 * (size_t)(nid[v] - F)];
        const uint32_t y = (R[0] & 0x100u) ? remap(R[1]) : 0u;
        if (R[0] & 0x1000000u) {
            U[0] = y;
            U[1] = R[0] | 0x80000000u;
            U[2] = remap(R[2]);
            U[3] = R[3];
        } else {
            U[0] = y;
            U[1] = (R[0] & 0x1FFu) | R[3] << 9;
        }
    }
    return true;
}

std::vector<uint8_t> pm_fl_profile(const std::vector<std::string>& pats) {
    std::vector<uint8_t> P;
    std::vector<uint32_t> O(1, 0);
    for (const std::string& p : pats) {
        P.insert(P.end(), p.begin(), p.end());
        O.push_back((uint32_t)P.size());
    }
    std::vector<uint8_t> t(PM_FL_PROFILE_PIECES * PM_FL_PROFILE_PIECE);
    if (pats.empty()) return t;
    std::vector<uint8_t> blk(PM_LINES_BLOCK);
    for (size_t k = 0; k < PM_FL_PROFILE_PIECES; ++k) {
        uint8_t* dst = t.data() + k * PM_FL_PROFILE_PIECE;
        const uint64_t lo = (uint64_t)k << 30;  // far apart in either stream
        for (uint64_t p = lo; p < lo + PM_FL_PROFILE_PIECE; ++p) {
            if (k % 16 == 15) {
                dst[p - lo] = pm_stream_byte(p, 7, 0);
            } else {
                if (p % PM_LINES_BLOCK == 0 || p == lo)
                    pm_lines_block(blk.data(), PM_LINES_BLOCK, p / PM_LINES_BLOCK, P.data(), O.data(),
                                   (uint32_t)pats.size(), 7);
                dst[p - lo] = blk[p % PM_LINES_BLOCK];
            }
        }
    }
    return t;
}

bool pm_pack_sparse_fl(const DfaImage& d, FlImage& fl, const std::vector<uint8_t>* profile) {
    const uint32_t F = d.sF, S = d.states;
    fl = FlImage();
    if (d.sblock.empty() || F < 1 || F >= 65536) return false;
    const uint32_t* rec = d.sblock.data() + (size_t)F * 256;
    auto R = [&](uint32_t v) { return rec + (size_t)(v - F) * 4; };  // {x, y, z, w} of record v
    for (uint32_t v = 0; v < S; ++v)
        if (d.sout[v] >= 65536) return false;
    // rows: the first PM_FL_LDS_ROWS -- the rows the kernel stages in LDS
    // -- are the root and the rows the profile's walks step from most
    // (without a profile the trie's breadth-first order: the shallowest
    // states), then the others by fallback use, so the word's 12-bit field
    // names the most used ones
    std::vector<uint64_t> use(F, 0);
    for (uint32_t v = F; v < S; ++v) use[R(v)[3]]++;
    std::vector<uint32_t> ord(F), nrow(F);
    for (uint32_t r = 0; r < F; ++r) ord[r] = r;
    const uint32_t keep = std::min(F, PM_FL_LDS_ROWS);
    uint32_t kept = keep;  // rows whose order is fixed before the fallback-use sort
    if (profile && !profile->empty() && keep > 1) {
        // the rows the profile's walks step from (row states, and record
        // misses' fallback rows), one walk from the root per piece
        std::vector<uint64_t> vis(F, 0);
        const uint8_t* t = profile->data();
        const size_t pieces = std::max<size_t>(1, profile->size() / PM_FL_PROFILE_PIECE);
        for (size_t k = 0; k < pieces; ++k) {
            const size_t lo = k * PM_FL_PROFILE_PIECE, hi = std::min(profile->size(), lo + PM_FL_PROFILE_PIECE);
            uint32_t s = 0;
            for (size_t i = lo; i < hi; ++i) {
                const uint32_t c = t[i];
                uint32_t row = s;
                if (s >= F) {
                    const uint32_t* r = R(s);
                    if ((r[0] & 0x100u) && c == (r[0] & 0xFFu)) { s = r[1] & PM_DFA_STATE_MASK; continue; }
                    if ((r[0] & 0x1000000u) && c == ((r[0] >> 16) & 0xFFu)) { s = r[2] & PM_DFA_STATE_MASK; continue; }
                    row = r[3];
                }
                vis[row]++;
                s = d.sblock[(size_t)row * 256 + c] & PM_DFA_STATE_MASK;
            }
        }
        vis[0] = ~0ull;  // the root stays row 0 (the warm-ups' start)
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return vis[a] > vis[b]; });
        // the first PM_FL_COUNT_LDS_ROWS by visits (the count-only kernel
        // stages that many; the others the first PM_FL_LDS_ROWS of them)
        kept = std::min(F, PM_FL_COUNT_LDS_ROWS);
        std::sort(ord.begin() + kept, ord.end());  // (the rest: by fallback use, next)
    }
    std::stable_sort(ord.begin() + kept, ord.end(), [&](uint32_t a, uint32_t b) { return use[a] > use[b]; });
    for (uint32_t k = 0; k < F; ++k) nrow[ord[k]] = k;
    // trie depth of every state, breadth first from the root: a row's
    // entries hold its goto children, a record's slots are all of its own
    // (a goto child differs from the fallback's transition: it is deeper)
    std::vector<uint16_t> dep(S, 0xFFFFu);
    {
        std::vector<uint32_t> q(1, 0u);
        dep[0] = 0;
        for (size_t h = 0; h < q.size(); ++h) {
            const uint32_t v = q[h];
            auto visit = [&](uint32_t t) {
                if (dep[t] == 0xFFFFu) {
                    dep[t] = (uint16_t)std::min<uint32_t>(dep[v] + 1u, 0xFFFEu);
                    q.push_back(t);
                }
            };
            if (v < F) {
                for (uint32_t c = 0; c < 256; ++c) visit(d.sblock[(size_t)v * 256 + c] & PM_DFA_STATE_MASK);
            } else {
                const uint32_t* r = R(v);
                if (r[0] & 0x100u) visit(r[1] & PM_DFA_STATE_MASK);
                if (r[0] & 0x1000000u) visit(r[2] & PM_DFA_STATE_MASK);
            }
        }
    }
    // folded slotless records; granules of the others, shallow part first
    std::vector<uint8_t> fold(S, 0);
    std::vector<uint32_t> gid(S, 0);  // granule of a record
    uint64_t u = 0;
    for (int part = 0; part < 2; ++part) {
        if (part == 1) {
            u = (u + 7) & ~(uint64_t)7;  // the deep part starts a 64-B block (the kernel's: 32 or 64 B)
            fl.deep_g = (uint32_t)u;
        }
        for (uint32_t v = F; v < S; ++v) {
            if ((dep[v] >= PM_FL_DEEP_DEPTH) != (part == 1)) continue;
            const uint32_t* r = R(v);
            const bool s0 = r[0] & 0x100u, s1 = r[0] & 0x1000000u;
            if (!s0 && d.sout[v] < PM_DFA_ESC) {
                fold[v] = 1;
                ++fl.folded;
                continue;
            }
            const bool wide = s1 || nrow[r[3]] >= PM_FL_FB_INREC;
            if (wide && (u & 1)) ++u;  // 16 B at a 16-B boundary
            gid[v] = (uint32_t)u;
            u += wide ? 2 : 1;
            if (F + u > PM_DFA_STATE_MASK + 1) return false;
        }
    }
    fl.F = F;
    fl.granules = (uint32_t)u;
    // the word into old state t
    auto enc = [&](uint32_t t) -> uint32_t {
        if (t < F) return nrow[t] | std::min(d.sout[t], PM_DFA_ESC) << 20;
        const uint32_t* r = R(t);
        if (fold[t]) return nrow[r[3]] | d.sout[t] << 20;
        return (F + gid[t]) | std::min(nrow[r[3]], PM_FL_FB_INREC) << 20;
    };
    fl.block.assign((size_t)F * 256 + 2 * (size_t)u, 0);
    fl.rowout16.assign(F, 0);
    for (uint32_t r = 0; r < F; ++r) {
        fl.rowout16[nrow[r]] = (uint16_t)d.sout[r];
        const uint32_t* src = d.sblock.data() + (size_t)r * 256;
        uint32_t* dst = fl.block.data() + (size_t)nrow[r] * 256;
        for (uint32_t c = 0; c < 256; ++c) dst[c] = enc(src[c] & PM_DFA_STATE_MASK);
    }
    for (uint32_t v = F; v < S; ++v) {
        if (fold[v]) continue;
        const uint32_t* r = R(v);
        uint32_t* U = fl.block.data() + (size_t)F * 256 + 2 * (size_t)gid[v];
        const bool s0 = r[0] & 0x100u, s1 = r[0] & 0x1000000u;
        uint32_t c0, c1, t0, t1;
        if (!s0) {  // slotless (output escapes): one slot repeating the fallback's byte-0 transition
            c0 = c1 = 0;
            t0 = t1 = enc(d.sblock[(size_t)r[3] * 256] & PM_DFA_STATE_MASK);
        } else {
            c0 = r[0] & 0xFFu;
            c1 = s1 ? (r[0] >> 16) & 0xFFu : c0;
            t0 = enc(r[1] & PM_DFA_STATE_MASK);
            t1 = s1 ? enc(r[2] & PM_DFA_STATE_MASK) : t0;
        }
        U[0] = d.sout[v] | c0 << 16 | c1 << 24;
        U[1] = t0;
        if (s1 || nrow[r[3]] >= PM_FL_FB_INREC) {
            U[2] = t1;
            U[3] = nrow[r[3]];
        }
    }
    return true;
}

uint32_t pm_fl_output(const FlImage& fl, uint32_t w) {
    const uint32_t s = w & PM_DFA_STATE_MASK;
    if (s < fl.F) {
        const uint32_t f = w >> 20;
        return f < PM_DFA_ESC ? f : fl.rowout16[s];
    }
    return fl.block[(size_t)fl.F * 256 + 2 * (size_t)(s - fl.F)] & 0xFFFFu;
}

uint32_t pm_fl_host_step(const FlImage& fl, uint32_t w, uint8_t c, uint32_t* out_prev) {
    const uint32_t s = w & PM_DFA_STATE_MASK;
    if (out_prev) *out_prev = pm_fl_output(fl, w);
    if (s < fl.F) return fl.block[(size_t)s * 256 + c];
    const uint32_t* U = fl.block.data() + (size_t)fl.F * 256 + 2 * (size_t)(s - fl.F);
    if (c == ((U[0] >> 16) & 0xFFu)) return U[1];
    if (c == U[0] >> 24) return U[2];
    const uint32_t fb = w >> 20;
    const uint32_t row = fb == PM_FL_FB_INREC ? U[3] : fb;
    return fl.block[(size_t)row * 256 + c];
}

DfaImage pm_build_dfa(const std::vector<std::string>& pats, const PmGidMap& g) {
    DfaImage im;
    BfsTrie t = build_trie(pats, g, /*reversed=*/false, PM_DFA_DFS_DEPTH);
    const uint32_t S = t.n;
    im.states = S;
    im.next.assign((size_t)S * 256, 0);
    im.out.assign(S, 0);
    std::vector<uint32_t> fail(S, 0);
    // rows in breadth-first order (by depth), so fail[v] (shallower) has its
    // row before v's whatever the numbering below PM_DFA_DFS_DEPTH
    std::vector<uint32_t> by_depth(S), dstart;
    for (uint32_t v = 0; v < S; ++v) {
        if (t.depth[v] + 2 > dstart.size()) dstart.resize(t.depth[v] + 2, 0);
        dstart[t.depth[v] + 1]++;
    }
    for (size_t d = 1; d < dstart.size(); ++d) dstart[d] += dstart[d - 1];
    for (uint32_t v = 0; v < S; ++v) by_depth[dstart[t.depth[v]]++] = v;
    for (uint32_t v : by_depth) {
        uint32_t* row = &im.next[(size_t)v * 256];
        if (v) std::memcpy(row, &im.next[(size_t)fail[v] * 256], 256 * sizeof(uint32_t));
        for (uint32_t k = 0; k < t.ccount[v]; ++k) {
            uint32_t u = t.cstart[v] + k;
            uint32_t c = t.label[u];
            // failure of a child (mpac.c:172-180): the root's children fail to
            // the root; otherwise follow v's failure with the same byte.
            fail[u] = v ? im.next[(size_t)fail[v] * 256 + c] : 0;
            row[c] = u;
        }
        // suffix link / output (mpac.c:179, :318)
        im.out[v] = v == 0 ? 0 : (t.gid[v] ? t.gid[v] : im.out[fail[v]]);
    }
    // output-coded transitions (pm_flatten.h): target | code << 20
    if (pm_dfa_coded(S)) {
        for (uint32_t& x : im.next) x |= std::min(im.out[x], PM_DFA_ESC) << 20;
        build_sparse(im, t, fail, by_depth);
    }
    return im;
}

// ---- compiled-image cache --------------------------------------------------

namespace {

constexpr uint64_t IMG_MAGIC = 0x31474D494D500000ull;  // "\0\0PMIMG1"
constexpr uint32_t IMG_VERSION = 12;                    // bump when a table layout changes

uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 0x100000001B3ull;
    return h;
}

template <class T>
bool put(FILE* f, uint32_t tag, const std::vector<T>& v) {
    const uint32_t es = sizeof(T);
    const uint64_t n = v.size();
    return std::fwrite(&tag, 4, 1, f) == 1 && std::fwrite(&es, 4, 1, f) == 1 && std::fwrite(&n, 8, 1, f) == 1 &&
           (n == 0 || std::fwrite(v.data(), es, n, f) == n);
}

template <class T>
bool get(FILE* f, uint32_t tag, std::vector<T>& v) {
    uint32_t t = 0, es = 0;
    uint64_t n = 0;
    if (std::fread(&t, 4, 1, f) != 1 || std::fread(&es, 4, 1, f) != 1 || std::fread(&n, 8, 1, f) != 1) return false;
    if (t != tag || es != sizeof(T) || n > ((uint64_t)1 << 36) / es) return false;
    v.resize(n);
    return n == 0 || std::fread(v.data(), es, n, f) == n;
}

bool save(const std::string& path, uint64_t key, int kind, const PmImages& im) {
    const std::string tmp = path + ".tmp." + std::to_string((long)getpid());
    // the cache directory and its parents, as `mkdir -p` (existing ones are fine)
    for (size_t k = path.find('/', 1); k != std::string::npos; k = path.find('/', k + 1))
        (void)::mkdir(path.substr(0, k).c_str(), 0755);
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) return false;
    const uint32_t hdr[2] = {IMG_VERSION, (uint32_t)kind};
    const std::vector<uint32_t> scal = {im.rt.fits ? 1u : 0u, im.rt.t3h_bits, im.rt.n2int, im.rt.nrec, im.rt.nodes,
                                        im.rt.d3, im.dfa.states, im.rt.nwide, im.dfa.sF};
    bool ok = std::fwrite(&IMG_MAGIC, 8, 1, f) == 1 && std::fwrite(&key, 8, 1, f) == 1 && std::fwrite(hdr, 4, 2, f) == 2 &&
              put(f, 1, scal) && put(f, 2, im.rt.t12) && put(f, 3, im.rt.filt) && put(f, 4, im.rt.t3h) &&
              put(f, 5, im.rt.rec) && put(f, 6, im.dfa.next) && put(f, 7, im.dfa.out) && put(f, 8, im.par.parent) &&
              put(f, 9, im.par.depth) && put(f, 10, im.rt.wide) && put(f, 11, im.dfa.sblock) &&
              put(f, 12, im.dfa.sout);
    ok = (std::fclose(f) == 0) && ok;
    if (ok) ok = std::rename(tmp.c_str(), path.c_str()) == 0;
    if (!ok) std::remove(tmp.c_str());
    return ok;
}

bool load(const std::string& path, uint64_t key, int kind, PmImages& im) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    uint64_t magic = 0, k = 0;
    uint32_t hdr[2] = {0, 0};
    std::vector<uint32_t> scal;
    bool ok = std::fread(&magic, 8, 1, f) == 1 && std::fread(&k, 8, 1, f) == 1 && std::fread(hdr, 4, 2, f) == 2 &&
              magic == IMG_MAGIC && k == key && hdr[0] == IMG_VERSION && hdr[1] == (uint32_t)kind &&
              get(f, 1, scal) && scal.size() == 9 && get(f, 2, im.rt.t12) && get(f, 3, im.rt.filt) &&
              get(f, 4, im.rt.t3h) && get(f, 5, im.rt.rec) && get(f, 6, im.dfa.next) && get(f, 7, im.dfa.out) &&
              get(f, 8, im.par.parent) && get(f, 9, im.par.depth) && get(f, 10, im.rt.wide) &&
              get(f, 11, im.dfa.sblock) && get(f, 12, im.dfa.sout);
    char extra;
    ok = ok && std::fread(&extra, 1, 1, f) == 0;  // nothing after the last section
    std::fclose(f);
    if (!ok) return false;
    im.rt.fits = scal[0] != 0;
    im.rt.t3h_bits = scal[1];
    im.rt.n2int = scal[2];
    im.rt.nrec = scal[3];
    im.rt.nodes = scal[4];
    im.rt.d3 = scal[5];
    im.dfa.states = scal[6];
    im.rt.nwide = scal[7];
    im.dfa.sF = scal[8];
    // structural checks: the kernels index these tables without bounds
    if (kind == 1 && im.rt.fits &&
        (im.rt.t12.size() != RT_T1_BASE + 256 || im.rt.filt.size() != RT_FILTER_WORDS + RT_F2_WORDS ||
         im.rt.t3h_bits < 4 || im.rt.t3h_bits > 30 || im.rt.t3h.size() != ((size_t)4 << im.rt.t3h_bits) ||
         im.rt.rec.size() != (size_t)im.rt.nrec * RT_REC_WORDS ||
         im.rt.wide.size() != (size_t)im.rt.nwide * RT_WIDE_WORDS))
        return false;
    if (kind == 2 && (im.dfa.next.size() != (size_t)im.dfa.states * 256 || im.dfa.out.size() != im.dfa.states))
        return false;
    if (kind == 2 && pm_dfa_coded(im.dfa.states) &&
        (im.dfa.sF < 1 || im.dfa.sF > im.dfa.states || im.dfa.sout.size() != im.dfa.states ||
         im.dfa.sblock.size() != (size_t)im.dfa.sF * 256 + (size_t)(im.dfa.states - im.dfa.sF) * PM_SDFA_REC_WORDS))
        return false;
    return true;
}

// Values the kernels follow without bounds checks: table and record indices,
// gids (score_kernel indexes parent[] with them) and the parent chain (which
// score_kernel walks).  A file whose sizes validate but whose values do not
// is rejected too, so a damaged cache can neither fault the device nor hang
// a walk.
bool values_ok(const PmImages& im, int kind, size_t ngid) {
    if (ngid == 0 || im.par.parent.size() != ngid || im.par.depth.size() != ngid) return false;
    const uint32_t P = (uint32_t)(ngid - 1);
    const std::vector<uint32_t>& par = im.par.parent;
    const std::vector<uint32_t>& dep = im.par.depth;
    if (par[0] != 0 || dep[0] != 0) return false;
    // depth[g] == 1 + depth[parent[g]] for every g admits no cycle
    for (uint32_t g = 1; g <= P; ++g)
        if (par[g] > P || dep[g] != 1 + dep[par[g]]) return false;
    if (kind == 2) {
        for (uint32_t x : im.dfa.out)
            if (x > P) return false;
        const bool coded = pm_dfa_coded(im.dfa.states);
        for (uint32_t x : im.dfa.next) {
            const uint32_t t = coded ? x & PM_DFA_STATE_MASK : x;
            if (t >= im.dfa.states || (coded && (x >> 20) != std::min(im.dfa.out[t], PM_DFA_ESC))) return false;
        }
        if (!coded) return true;
        // sparse form: coded words consistent with sout, fallbacks are rows
        const DfaImage& d = im.dfa;
        auto word_ok = [&](uint32_t x) {
            const uint32_t t = x & PM_DFA_STATE_MASK;
            return t < d.states && (x >> 20) == std::min(d.sout[t], PM_DFA_ESC);
        };
        for (uint32_t x : d.sout)
            if (x > P) return false;
        const size_t nrow = (size_t)d.sF * 256;
        for (size_t e = 0; e < nrow; ++e)
            if (!word_ok(d.sblock[e])) return false;
        for (size_t e = nrow; e < d.sblock.size(); e += PM_SDFA_REC_WORDS) {
            const uint32_t* R = &d.sblock[e];
            if ((R[0] & ~0x01FF01FFu) || R[3] >= d.sF) return false;
            if ((R[0] & 0x100u) && !word_ok(R[1])) return false;
            if ((R[0] & 0x1000000u) && !word_ok(R[2])) return false;
        }
        return true;
    }
    const RtImage& rt = im.rt;
    if (!rt.fits) return true;
    if (rt.nrec >= (1u << 23) || rt.nwide >= (1u << 14)) return false;
    for (uint16_t x : rt.t12)
        if ((x & 0x7FFFu) > P) return false;
    for (size_t e = 0; e < rt.t3h.size(); e += 4) {
        const uint32_t x = rt.t3h[e], y = rt.t3h[e + 1], z = rt.t3h[e + 2], w = rt.t3h[e + 3];
        if (!(x & RT_T3H_VALID)) continue;
        const uint32_t k = x >> 25, nch = z >> 24, r = w & ~RT_CONT32;
        if (y > P || k > 2) return false;
        if (k == 1 && (nch < 1 || nch > RT_T3H_INLINE)) return false;
        if (k == 1 && nch > 1 && (uint64_t)w + nch > rt.nrec) return false;
        if (k == 1 && nch == 1 && ((w & RT_CONT32) ? r >= rt.nrec : w > P)) return false;
        if (k == 2 && (!(w & RT_CONT32) || r >= rt.nrec)) return false;
        // the entry sits in one of its key's two cuckoo slots (the device
        // probes only those)
        const uint32_t key = x & 0xFFFFFFu, sl = (uint32_t)(e / 4);
        if (sl != pm_rt_slot1(key, rt.t3h_bits) && sl != pm_rt_slot2(key, rt.t3h_bits)) return false;
    }
    // records: children strictly after their parent (BFS), so every walk
    // terminates; indices in range; wide entries' prefix counts consistent
    for (uint32_t n = 0; n < rt.nrec; ++n) {
        const uint32_t* R = &rt.rec[(size_t)n * RT_REC_WORDS];
        const uint32_t rk = R[0] >> 30, cnt = (R[0] >> 24) & 63u, first = R[0] & 0xFFFFFFu;
        if (R[1] > P) return false;
        if (rk == RT_REC_LEAF) continue;
        if (rk == RT_REC_KIDS) {
            if (cnt < 1 || cnt > RT_REC_INLINE || first <= n || (uint64_t)first + cnt > rt.nrec) return false;
            continue;
        }
        if (rk == RT_REC_CHAIN) {
            // the run the record describes is the one the records hold
            if (cnt < 1 || cnt > RT_CHAIN_MAX || first <= n || (uint64_t)first + cnt > rt.nrec) return false;
            const uint64_t Pb = (uint64_t)R[3] << 32 | R[2];
            for (uint32_t k = 1; k < cnt; ++k) {
                const uint32_t* C = &rt.rec[(size_t)(first + k - 1) * RT_REC_WORDS];
                if (C[0] >> 30 != RT_REC_CHAIN || (C[0] & 0xFFFFFFu) != first + k || C[1] != R[1] ||
                    (C[3] >> 24) != ((Pb >> (8 * (7 - k))) & 0xFFu))
                    return false;
            }
            continue;
        }
        if (rk != RT_REC_WIDE || R[2] >= rt.nwide || first <= n) return false;
        const uint32_t* W = &rt.wide[(size_t)R[2] * RT_WIDE_WORDS];
        uint64_t idx = first;
        for (int q = 0; q < 4; ++q) {
            if (W[4 * q + 2] != idx || W[4 * q + 3] != R[1]) return false;
            idx += (uint32_t)__builtin_popcount(W[4 * q]) + (uint32_t)__builtin_popcount(W[4 * q + 1]);
        }
        if (idx - first <= RT_REC_INLINE || idx > rt.nrec) return false;
    }
    // the LDS filters are exactly the ones the tables imply (no false
    // negatives can hide in a damaged or stale filter word)
    return rt.filt == derive_filters(rt);
}

}  // namespace

uint64_t pm_image_key(const std::vector<std::string>& pats, int kind) {
    uint64_t h = 0xCBF29CE484222325ull;
    const uint32_t v[2] = {IMG_VERSION, (uint32_t)kind};
    h = fnv1a(h, v, sizeof v);
    // layout constants and the hash functions themselves (their values on a
    // few keys): a change to either gives new keys, not a stale hit
    uint32_t lay[] = {RT_T1_BASE, RT_CONT16, RT_CONT32, (uint32_t)RT_REC_WORDS, RT_FILTER_WORDS, RT_F3_WORDS,
                      RT_F4_WORDS, RT_T3H_INLINE, RT_T3H_VALID, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                      RT_REC_INLINE, (uint32_t)RT_WIDE_WORDS, (uint32_t)PM_DFA_DFS_DEPTH, RT_CHAIN_MAX,
                      PM_SDFA_K, PM_SDFA_REC_WORDS};
    const uint32_t probe[2] = {0x00A1B2C3u, 0x00FFFFFFu};
    for (int q = 0; q < 2; ++q) {
        const uint32_t k = probe[q];
        uint32_t* o = &lay[9 + 7 * q];
        o[0] = pm_rt_fhash(k);
        o[1] = pm_rt_filter_mask(o[0]) ^ pm_rt_filter_word(o[0]);
        o[2] = pm_rt_p3hash(k) ^ pm_rt_p3word(pm_rt_p3hash(k));
        o[3] = pm_rt_s4hash(k << 8 | 0x5A) ^ pm_rt_s4word(pm_rt_s4hash(k << 8 | 0x5A));
        o[4] = pm_rt_slot1(k, 20);
        o[5] = pm_rt_slot2(k, 20);
        o[6] = pm_rt_hash(k);
    }
    h = fnv1a(h, lay, sizeof lay);
    for (const auto& p : pats) {
        const uint64_t n = p.size();
        h = fnv1a(h, &n, 8);
        h = fnv1a(h, p.data(), p.size());
    }
    return h;
}

PmImages pm_build_images_cached(const std::vector<std::string>& pats, const PmGidMap& g, int kind,
                                const std::string& dir, bool* hit) {
    PmImages im;
    *hit = false;
    std::string path;
    uint64_t key = 0;
    if (!dir.empty()) {
        key = pm_image_key(pats, kind);
        char name[64];
        std::snprintf(name, sizeof name, "/pm-%d-%016llx.img", kind, (unsigned long long)key);
        path = dir + name;
        if (load(path, key, kind, im) && values_ok(im, kind, g.index_of_gid.size())) {
            *hit = true;
            return im;
        }
        im = PmImages();
    }
    if (kind == 1) im.rt = pm_build_rt(pats, g);
    else im.dfa = pm_build_dfa(pats, g);
    im.par = pm_build_parents(pats, g);
    if (!dir.empty()) save(path, key, kind, im);  // best effort
    return im;
}
