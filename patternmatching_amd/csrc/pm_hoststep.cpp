// pm_hoststep.cpp -- read_char's per-byte step on the host (pm_hoststep.h).
// The walk is the device's rt_one / rt_from_d2 / rt_deep
// (pm_kernels.hip) over the host copy of the same image; the DFA step is
// one transition of the flattened automaton (mpac.c:304-319 with the
// failure loop folded into the rows, pm_flatten.cpp).
#include "pm_hoststep.h"

namespace {

// The child of record R on byte c into node; 0 when the walk ends at R.
inline uint32_t rec_child(const RtImage& im, const uint32_t* R, uint32_t c, uint32_t& node) {
    const uint32_t kind = R[0] >> 30, first = R[0] & 0xFFFFFFu, cnt = (R[0] >> 24) & 63u;
    if (kind == RT_REC_LEAF) return 0;
    if (kind == RT_REC_CHAIN) {  // one byte of the run per step (the edge walker's form)
        if (c != (R[3] >> 24)) return 0;
        node = first;
        return 1;
    }
    if (kind == RT_REC_KIDS) {
        for (uint32_t j = 0; j < cnt && j < RT_REC_INLINE; ++j)
            if (((R[2 + j / 4] >> (8 * (j & 3))) & 0xFFu) == c) {
                node = first + j;
                return 1;
            }
        return 0;
    }
    // wide: quarter q = c >> 6 of its entry {word 2q, word 2q+1, index of word 2q, best}
    const uint32_t* Q = &im.wide[(size_t)R[2] * RT_WIDE_WORDS + 4 * (c >> 6)];
    const uint32_t odd = (c >> 5) & 1u, bit = c & 31u, word = odd ? Q[1] : Q[0];
    if (!((word >> bit) & 1u)) return 0;
    node = Q[2] + (odd ? (uint32_t)__builtin_popcount(Q[0]) : 0u) + (uint32_t)__builtin_popcount(word & ((1u << bit) - 1u));
    return 1;
}

// node = record reached after the newest d bytes
uint32_t rec_walk(const RtImage& im, const uint8_t* p, uint32_t node, size_t d, size_t avail) {
    for (;;) {
        const uint32_t* R = &im.rec[(size_t)node * RT_REC_WORDS];
        if (d >= avail) return R[1];
        if (!rec_child(im, R, p[-(ptrdiff_t)d], node)) return R[1];
        ++d;
    }
}

bool t3h_find(const RtImage& im, uint32_t key24, const uint32_t*& e) {
    const uint32_t want = RT_T3H_VALID | key24;
    for (uint32_t slot : {pm_rt_slot1(key24, im.t3h_bits), pm_rt_slot2(key24, im.t3h_bits)}) {
        e = &im.t3h[(size_t)slot * 4];
        if ((e[0] & 0x1FFFFFFu) == want) return true;
    }
    return false;
}

}  // namespace

uint32_t pm_rt_host_answer(const RtImage& im, const uint8_t* p, size_t avail) {
    if (avail < 3) {  // the stream's first bytes
        if (avail == 0) return 0;
        const uint32_t c0 = p[0];
        if (avail == 1) return im.t12[RT_T1_BASE + c0];
        return im.t12[(c0 << 8) | p[-1]] & 0x7FFFu;
    }
    const uint32_t c0 = p[0], c1 = p[-1];
    const uint32_t v = im.t12[(c0 << 8) | c1];
    const uint32_t best2 = v & 0x7FFFu;
    const uint32_t key24 = (uint32_t)p[-2] | (c1 << 8) | (c0 << 16);
    // the kernel's stage-1 Bloom filter (16 KiB, no false negatives), read
    // whether or not the depth-2 node continues: one rarely taken branch
    // (~2% of random text) instead of an unpredictable one per byte; a
    // position failing it has no depth-3 node on its walk
    const uint32_t f = pm_rt_fhash(key24), m1 = pm_rt_filter_mask(f);
    const uint32_t go = (v >> 15) & (uint32_t)((im.filt[pm_rt_filter_word(f)] & m1) == m1);
    if (__builtin_expect(!go, 1)) return best2;
    const uint32_t* f2 = &im.filt[RT_FILTER_WORDS];
    const uint32_t g3 = pm_rt_p3hash(key24), m3 = pm_rt_filter_mask(g3);
    const uint32_t key32 = (avail >= 4 ? (uint32_t)p[-3] : 0u) | (key24 << 8);
    const uint32_t g4 = pm_rt_s4hash(key32), m4 = pm_rt_filter_mask(g4);
    if ((f2[pm_rt_p3word(g3)] & m3) != m3 && (f2[pm_rt_s4word(g4)] & m4) != m4) return best2;
    const uint32_t* e;
    if (!t3h_find(im, key24, e)) return best2;
    const uint32_t kind = e[0] >> 25;
    if (kind == 0 || avail < 4) return e[1];
    if (kind == 1) {
        const uint32_t nch = e[2] >> 24, c3 = p[-3];
        uint32_t k = 0;
        while (k < nch && ((e[2] >> (8 * k)) & 0xFFu) != c3) ++k;
        if (k >= nch) return e[1];
        if (nch > 1) return rec_walk(im, p, e[3] + k, 4, avail);
        if (!(e[3] & RT_CONT32)) return e[3];
        return rec_walk(im, p, e[3] & ~RT_CONT32, 4, avail);
    }
    return rec_walk(im, p, e[3] & ~RT_CONT32, 3, avail);
}

uint32_t pm_dfa_host_step(const DfaImage& d, uint32_t& s, uint8_t c) {
    if (!d.sblock.empty()) {  // rows [0, F), 16-B records after them (pm_flatten.h)
        uint32_t x;
        if (s < d.sF) {
            x = d.sblock[(size_t)s * 256 + c];
        } else {
            const uint32_t* R = &d.sblock[(size_t)d.sF * 256 + (size_t)(s - d.sF) * PM_SDFA_REC_WORDS];
            const uint32_t key = c | 0x100u;
            x = (R[0] & 0x1FFu) == key ? R[1] : ((R[0] >> 16) & 0x1FFu) == key ? R[2] : d.sblock[(size_t)R[3] * 256 + c];
        }
        s = x & PM_DFA_STATE_MASK;
        const uint32_t code = x >> 20;
        return code != PM_DFA_ESC ? code : d.sout[s];
    }
    const uint32_t x = d.next[(size_t)s * 256 + c];
    if (pm_dfa_coded(d.states)) {
        s = x & PM_DFA_STATE_MASK;
        const uint32_t code = x >> 20;
        return code != PM_DFA_ESC ? code : d.out[s];
    }
    s = x;
    return d.out[s];
}

uint32_t pm_host_step(PmHostStep& h, PmHistRing& r, uint32_t max_len, uint8_t c) {
    if (h.kind == 1) {
        r.push(c);
        return pm_rt_host_answer(h.rt, r.newest(), r.avail());
    }
    if (h.kind != 2) {
        r.push(c);
        return 0;
    }
    if (!h.state_valid) {  // warm up from the root over the history (at most max_len-1 bytes)
        const size_t keep = max_len ? max_len - 1 : 0;
        const size_t w = r.avail() < keep ? r.avail() : keep;
        h.state = 0;
        const uint8_t* p = r.newest();
        for (size_t k = w; k > 0; --k) (void)pm_dfa_host_step(h.dfa, h.state, p[1 - (ptrdiff_t)k]);
        h.state_valid = true;
    }
    r.push(c);
    return pm_dfa_host_step(h.dfa, h.state, c);
}
