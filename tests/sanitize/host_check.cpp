// host_check.cpp -- TEST-ONLY harness for tests/test_sanitize.py: the host
// code (pm_dict.c front end, pm_flatten.cpp flattener and image cache) built
// with -fsanitize=address,undefined.  It
//   * loads the dictionaries (PatternsTree.c:260-312 semantics) and checks
//     every pattern's parent is its longest proper suffix that is a pattern,
//     and that pm_build_parents agrees in gid space;
//   * feeds odd lines to the parser (parser.c:63-99 edge cases);
//   * builds both images through the cache twice (miss, then hit: the
//     loaded images must equal the built ones);
//   * walks the RT image the way pm_kernels.hip's rt_one / rt_from_d2 /
//     rt_deep do, every access bounds-checked (.at()), and the DFA image the
//     way dfa_scan_kernel / dfa_coded_kernel do, and requires the two answers to agree at
//     every position of the stream given plus a synthetic tail;
//   * checks the filters have no false negatives (a depth-3 node passes
//     stage 1; a position answered below depth 2 passes stage 2).
// Usage: host_check CACHE_DIR STREAM DICT...
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_set>
#include <vector>

#include "pm_flatten.h"
#include "pm_host.h"

namespace {

int g_fail = 0;
#define CHECK(c, ...)                                  \
    do {                                               \
        if (!(c)) {                                    \
            std::fprintf(stderr, "FAIL %s: ", #c);     \
            std::fprintf(stderr, __VA_ARGS__);         \
            std::fprintf(stderr, "\n");                \
            if (++g_fail > 20) std::exit(1);           \
        }                                              \
    } while (0)

struct Feed {
    std::vector<std::string> pats;
    std::vector<pm_pattern_id_t> ids;
};

void feed_add(void* obj, char* bytes, size_t len, pm_pattern_id_t id) {
    Feed* f = static_cast<Feed*>(obj);
    f->pats.emplace_back(bytes, len);
    f->ids.push_back(id);
}

uint32_t rt_deep(const RtImage& im, const std::vector<uint8_t>& text, uint32_t node, int64_t i, int64_t avail,
                 int64_t d) {
    for (;;) {
        const size_t R = (size_t)node * RT_REC_WORDS;
        const uint32_t x = im.rec.at(R), best = im.rec.at(R + 1);
        if (d >= avail) return best;
        const uint32_t kind = x >> 30, cnt = (x >> 24) & 63u, first = x & 0xFFFFFFu;
        const uint32_t c = text.at(i - d);
        if (kind == RT_REC_LEAF) return best;
        uint32_t next = 0;
        if (kind == RT_REC_CHAIN) {
            // the whole run at once, as the device tail does (pm_flatten.h)
            const uint64_t P = (uint64_t)im.rec.at(R + 3) << 32 | im.rec.at(R + 2);
            uint32_t m = 0;
            while (m < cnt && d + m < avail && text.at(i - d - m) == ((P >> (8 * (7 - m))) & 0xFFu)) ++m;
            if (m == 0) return best;
            if (m < cnt) {  // stopped inside the run: no pattern there, the answer is this record's
                const size_t Rm = (size_t)(first + m - 1) * RT_REC_WORDS;
                CHECK(im.rec.at(Rm + 1) == best, "chain best %u vs %u", im.rec.at(Rm + 1), best);
                return best;
            }
            CHECK(first + m - 1 > node && first + m - 1 < im.nrec, "chain %u -> %u", node, first + m - 1);
            node = first + m - 1;
            d += m;
            continue;
        } else if (kind == RT_REC_KIDS) {
            uint32_t j = 0;
            while (j < cnt && ((im.rec.at(R + 2 + j / 4) >> (8 * (j & 3))) & 0xFFu) != c) ++j;
            if (j == cnt) return best;
            next = first + j;
        } else {
            CHECK(kind == RT_REC_WIDE, "record kind %u", kind);
            const size_t Q = (size_t)im.rec.at(R + 2) * RT_WIDE_WORDS + 4 * (c >> 6);
            const uint32_t w = (c >> 5) & 1u, word = im.wide.at(Q + w), bit = c & 31u;
            CHECK(im.wide.at(Q + 3) == best, "wide best %u vs %u", im.wide.at(Q + 3), best);
            if (!((word >> bit) & 1u)) return best;
            next = im.wide.at(Q + 2) + (w ? (uint32_t)__builtin_popcount(im.wide.at(Q)) : 0u) +
                   (uint32_t)__builtin_popcount(word & ((1u << bit) - 1u));
            CHECK(im.wide.at(Q + 2) >= first, "wide index %u below first %u", im.wide.at(Q + 2), first);
        }
        CHECK(next > node && next < im.nrec, "record %u -> %u of %u", node, next, im.nrec);
        node = next;
        ++d;
    }
}

// Returns the answer; *deep = the walk went past depth 2 (the t3h entry exists).
uint32_t rt_one(const RtImage& im, const std::vector<uint8_t>& text, int64_t i, bool* deep, uint32_t* best2) {
    *deep = false;
    const int64_t avail = i + 1;
    const uint32_t c0 = text.at(i);
    if (avail == 1) return *best2 = im.t12.at(RT_T1_BASE + c0);
    const uint32_t c1 = text.at(i - 1);
    const uint32_t v = im.t12.at((c0 << 8) | c1);
    *best2 = v & 0x7FFFu;
    if (!(v & RT_CONT16) || avail == 2) return v & 0x7FFFu;
    const uint32_t key24 = text.at(i - 2) | (c1 << 8) | (c0 << 16);
    const uint32_t c3 = avail >= 4 ? text.at(i - 3) : 0u;
    const uint32_t want = RT_T3H_VALID | key24;
    size_t e = 4 * (size_t)pm_rt_slot1(key24, im.t3h_bits);
    if ((im.t3h.at(e) & 0x1FFFFFFu) != want) {
        e = 4 * (size_t)pm_rt_slot2(key24, im.t3h_bits);
        if ((im.t3h.at(e) & 0x1FFFFFFu) != want) return v & 0x7FFFu;
    }
    *deep = true;
    const uint32_t x = im.t3h.at(e), y = im.t3h.at(e + 1), z = im.t3h.at(e + 2), w = im.t3h.at(e + 3);
    const uint32_t kind = x >> 25;
    CHECK(kind <= 2, "t3h kind %u", kind);
    if (kind == 0 || avail < 4) return y;
    if (kind == 1) {
        const uint32_t nch = z >> 24;
        CHECK(nch >= 1 && nch <= RT_T3H_INLINE, "nch %u", nch);
        uint32_t k = 3;
        for (uint32_t j = 0; j < 3; ++j)
            if (c3 == ((z >> (8 * j)) & 0xFFu)) { k = j; break; }
        if (k >= nch) return y;
        if (nch > 1) return rt_deep(im, text, w + k, i, avail, 4);
        if (!(w & RT_CONT32)) return w;
        return rt_deep(im, text, w & 0x7FFFFFFFu, i, avail, 4);
    }
    return rt_deep(im, text, w & 0x7FFFFFFFu, i, avail, 3);
}

bool stage1(const RtImage& im, uint32_t key24) {
    const uint32_t f = pm_rt_fhash(key24);
    const uint32_t m = pm_rt_filter_mask(f);
    return (im.filt.at(pm_rt_filter_word(f)) & m) == m;
}

bool stage2(const RtImage& im, uint32_t key24, uint32_t c3) {
    const uint32_t g3 = pm_rt_p3hash(key24), m3 = pm_rt_filter_mask(g3);
    const uint32_t g4 = pm_rt_s4hash(c3 | (key24 << 8)), m4 = pm_rt_filter_mask(g4);
    return (im.filt.at(RT_FILTER_WORDS + pm_rt_p3word(g3)) & m3) == m3 ||
           (im.filt.at(RT_FILTER_WORDS + pm_rt_s4word(g4)) & m4) == m4;
}

void parser_edges() {
    const char* lines[] = {"", "|", "||", "|4", "|41|", "|4 1|", "|zz|", "a|41 42|b", "|41|42|", " |41|",
                           "\\x41", "|41 |", "| 41|", "||||", "abc\n"};
    unsigned char out[64];
    for (const char* l : lines) {
        const size_t n = std::strlen(l);
        const size_t r = pm_parse_line(reinterpret_cast<const unsigned char*>(l), n, out);
        CHECK(r <= n, "parse '%s' -> %zu", l, r);
    }
    // a long line of every byte value, and a line of NULs
    std::vector<unsigned char> big(70000), buf(70000);
    for (size_t i = 0; i < big.size(); ++i) big[i] = (unsigned char)(i * 131 + 7);
    CHECK(pm_parse_line(big.data(), big.size(), buf.data()) <= big.size(), "big line");
    std::vector<unsigned char> nul(100, 0);
    CHECK(pm_parse_line(nul.data(), nul.size(), buf.data()) <= nul.size(), "nul line");
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s CACHE_DIR STREAM DICT...\n", argv[0]);
        return 2;
    }
    const std::string cache = argv[1];
    parser_edges();

    char err[512] = {0};
    PmDict* d = pm_dict_load(const_cast<const char* const*>(argv + 3), (size_t)(argc - 3), err, sizeof err);
    if (!d) {
        std::fprintf(stderr, "dict load: %s\n", err);
        return 1;
    }
    Feed fd;
    pm_dict_feed(d, &fd, feed_add);
    CHECK(fd.pats.size() == d->n, "fed %zu of %zu", fd.pats.size(), d->n);

    // patterns tree: parent = longest proper suffix that is a pattern
    std::unordered_set<std::string> all(fd.pats.begin(), fd.pats.end());
    for (size_t k = 0; k < fd.pats.size(); ++k) {
        pm_pattern_id_t p = fd.ids[k];
        CHECK(p->index == k && p->len == fd.pats[k].size(), "pattern %zu", k);
        CHECK(std::memcmp(p->bytes, fd.pats[k].data(), p->len) == 0, "bytes of %zu", k);
        const std::string& s = fd.pats[k];
        size_t want = 0;
        for (size_t l = s.size() - 1; l > 0; --l)
            if (all.count(s.substr(s.size() - l))) { want = l; break; }
        if (!want) {
            CHECK(p->parent == nullptr, "pattern %zu has a parent", k);
        } else {
            CHECK(p->parent && p->parent->len == want, "parent of %zu", k);
            if (p->parent) {
                CHECK(std::memcmp(p->parent->bytes, p->bytes + p->len - want, want) == 0, "suffix of %zu", k);
                CHECK(pm_pattern_is_suffix(p->parent, p), "is_suffix %zu", k);
            }
        }
    }

    const PmGidMap g = pm_assign_gids(fd.pats);
    bool hit = false;
    PmImages rt1 = pm_build_images_cached(fd.pats, g, 1, cache, &hit);
    CHECK(!hit, "rt: first build hit the cache");
    PmImages rt2 = pm_build_images_cached(fd.pats, g, 1, cache, &hit);
    CHECK(hit, "rt: second build missed the cache");
    CHECK(rt1.rt.fits && rt2.rt.fits, "rt image does not fit");
    CHECK(rt1.rt.t12 == rt2.rt.t12 && rt1.rt.filt == rt2.rt.filt && rt1.rt.t3h == rt2.rt.t3h &&
              rt1.rt.rec == rt2.rt.rec && rt1.rt.wide == rt2.rt.wide && rt1.rt.t3h_bits == rt2.rt.t3h_bits && rt1.rt.nrec == rt2.rt.nrec,
          "rt: cached image differs");
    PmImages df1 = pm_build_images_cached(fd.pats, g, 2, cache, &hit);
    CHECK(!hit, "dfa: first build hit the cache");
    PmImages df2 = pm_build_images_cached(fd.pats, g, 2, cache, &hit);
    CHECK(hit, "dfa: second build missed the cache");
    CHECK(df1.dfa.next == df2.dfa.next && df1.dfa.out == df2.dfa.out, "dfa: cached image differs");
    CHECK(rt1.par.parent == df1.par.parent && rt1.par.depth == df1.par.depth, "parents differ");

    // parents in gid space agree with the dictionary's tree
    for (size_t k = 0; k < fd.pats.size(); ++k) {
        const uint32_t gk = g.gid_of_index.at(k);
        const PmPattern* par = fd.ids[k]->parent;
        const uint32_t want = par ? g.gid_of_index.at(par->index) : 0u;
        CHECK(rt1.par.parent.at(gk) == want, "gid parent of %zu", k);
        CHECK(rt1.par.depth.at(gk) == 1 + (want ? rt1.par.depth.at(want) : 0u), "depth of %zu", k);
    }

    // the stream plus a synthetic printable tail
    std::vector<uint8_t> text;
    if (FILE* f = std::fopen(argv[2], "rb")) {
        uint8_t buf[65536];
        size_t r;
        while ((r = std::fread(buf, 1, sizeof buf, f)) > 0) text.insert(text.end(), buf, buf + r);
        std::fclose(f);
    } else {
        std::fprintf(stderr, "cannot open %s\n", argv[2]);
        return 1;
    }
    uint32_t x = 2463534242u;
    for (int k = 0; k < 40000; ++k) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        text.push_back((uint8_t)(32 + x % 95));
    }

    const RtImage& im = rt2.rt;
    const DfaImage& dfa = df2.dfa;
    uint32_t s = 0;
    size_t nonnull = 0, deep = 0;
    for (int64_t i = 0; i < (int64_t)text.size(); ++i) {
        const uint32_t x = dfa.next.at((size_t)s * 256 + text[i]);
        s = pm_dfa_coded(dfa.states) ? x & PM_DFA_STATE_MASK : x;  // output-coded transitions
        CHECK(s < dfa.states, "state %u", s);
        const uint32_t want = dfa.out.at(s);
        CHECK(!pm_dfa_coded(dfa.states) || (x >> 20) == std::min(want, PM_DFA_ESC), "code %u out %u", x >> 20, want);
        bool dp = false;
        uint32_t best2 = 0;
        const uint32_t got = rt_one(im, text, i, &dp, &best2);
        CHECK(got == want, "position %lld: rt %u dfa %u", (long long)i, got, want);
        nonnull += want != 0;
        deep += dp;
        if (i >= 3) {
            const uint32_t key24 = text[i - 2] | (text[i - 1] << 8) | ((uint32_t)text[i] << 16);
            if (dp) CHECK(stage1(im, key24), "stage 1 false negative at %lld", (long long)i);
            if (got != best2) CHECK(stage2(im, key24, text[i - 3]), "stage 2 false negative at %lld", (long long)i);
        }
    }
    pm_dict_free(d);
    if (g_fail) return 1;
    std::printf("ok patterns=%zu positions=%zu nonnull=%zu deep=%zu states=%u records=%u\n",
                fd.pats.size(), text.size(), nonnull, deep, dfa.states, im.nrec);
    return 0;
}
