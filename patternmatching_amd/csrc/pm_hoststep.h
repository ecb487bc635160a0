// pm_hoststep.h -- the per-byte read_char step on the host (SURVEY.md §7
// step 4, §8b: "per-byte read_char stays available as a host DFA step").
//
// The reference's stream loop calls read_char once per byte
// (Core/src/measure.c:292-294) and, unmodified, has no batched path.  A GPU
// launch per byte would cost a full H2D / kernel / D2H round trip each, so
// read_char steps the object's own flattened images on the host instead --
// the same tables compile() uploads to HBM, not the oracle:
//
//   RT / auto kinds  the reverse-trie walk of the newest byte over the
//                    carried history (pm_kernels.hip rt_one):
//                    t12 for depth <= 2, the t3h entry, then node records.
//   AC kind          one transition of the output-coded DFA, sparse form
//                    when present (rows + default-transition records), else
//                    dense rows; the state is re-derived from the history
//                    after a read_block (warm-up of max_len-1 bytes from the
//                    root: exact by the shard rule).
//
// Both keep the history ring consistent with read_block, so read_char and
// read_block calls interleave exactly (mps.h:41-42, state carried).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "pm_flatten.h"

// The last stream bytes (at least max_len of them), newest at seen - 1.
struct PmHistRing {
    std::vector<uint8_t> b;
    uint64_t mask = 0;
    uint64_t seen = 0;  // bytes pushed since the last clear

    void init(uint32_t max_len) {
        size_t r = 16;
        while (r < (size_t)max_len + 1) r <<= 1;
        b.assign(r, 0);
        mask = r - 1;
        seen = 0;
    }
    void clear() { seen = 0; }
    size_t avail() const { return seen < b.size() ? (size_t)seen : b.size(); }
    void push(uint8_t c) { b[seen++ & mask] = c; }
    void append(const uint8_t* p, size_t n) {
        if (n > b.size()) {
            seen += n - b.size();
            p += n - b.size();
            n = b.size();
        }
        for (size_t k = 0; k < n; ++k) push(p[k]);
    }
    // byte d positions before the newest one (d < avail())
    uint8_t back(size_t d) const { return b[(seen - 1 - d) & mask]; }
    // the last h bytes (h <= avail()), oldest first
    void copy_last(uint8_t* dst, size_t h) const {
        for (size_t k = 0; k < h; ++k) dst[k] = b[(seen - h + k) & mask];
    }
};

// gid of the longest pattern ending at the newest byte of r (0 = none).
uint32_t pm_rt_host_answer(const RtImage& im, const PmHistRing& r);

// One DFA transition on byte c from state s (updated); returns the gid of
// the longest pattern ending at c.  State 0 is the root in both forms.
uint32_t pm_dfa_host_step(const DfaImage& d, uint32_t& s, uint8_t c);

// Host images kept for the step: the RT image, or the DFA (the sparse
// form's block only, when it exists).
struct PmHostStep {
    int kind = 0;  // 1 = RT walk, 2 = DFA step, 0 = nothing compiled
    RtImage rt;
    DfaImage dfa;
    uint32_t state = 0;
    bool state_valid = false;  // DFA: state matches the ring (false after read_block / reset)
    size_t bytes() const { return kind == 1 ? rt.bytes() : dfa.bytes() + dfa.sparse_bytes(); }
};

// read_char's step: push c, return the gid at it.
uint32_t pm_host_step(PmHostStep& h, PmHistRing& r, uint32_t max_len, uint8_t c);
