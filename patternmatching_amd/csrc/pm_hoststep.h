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
#include <cstring>
#include <vector>

#include "pm_flatten.h"

// The stream's last bytes (at least max_len of them) in one linear buffer:
// bytes are appended at `pos` and, when it fills, the last K bytes slide to
// the front (K >= max_len, the walk's reach), so a walk reads text[i - d] as
// p[-d] from a plain pointer -- as the kernel does -- instead of through
// ring indices (a ring cost 2x on the per-byte path).
struct PmHistRing {
    std::vector<uint8_t> b;
    size_t K = 16;    // bytes kept at a slide (power of two >= max_len)
    size_t pos = 0;   // bytes in b; the newest is b[pos - 1]
    uint64_t seen = 0;

    void init(uint32_t max_len) {
        K = 16;
        while (K < (size_t)max_len) K <<= 1;
        b.assign(K < 32768 ? 65536 : 2 * K, 0);
        pos = 0;
        seen = 0;
    }
    void clear() {
        pos = 0;
        seen = 0;
    }
    // bytes a walk may look back over, the newest included (>= min(seen, K))
    size_t avail() const { return pos; }
    const uint8_t* newest() const { return b.data() + pos - 1; }
    void slide() {
        std::memmove(b.data(), b.data() + pos - K, K);
        pos = K;
    }
    void push(uint8_t c) {
        if (pos == b.size()) slide();
        b[pos++] = c;
        ++seen;
    }
    void append(const uint8_t* p, size_t n) {
        seen += n;
        if (n >= K) {
            std::memcpy(b.data(), p + n - K, K);
            pos = K;
            return;
        }
        if (pos + n > b.size()) slide();
        std::memcpy(b.data() + pos, p, n);
        pos += n;
    }
    // byte d positions before the newest one (d < avail())
    uint8_t back(size_t d) const { return b[pos - 1 - d]; }
    // the last h bytes (h <= avail()), oldest first
    void copy_last(uint8_t* dst, size_t h) const { std::memcpy(dst, b.data() + pos - h, h); }
};

// gid of the longest pattern ending at p[0], the stream's newest byte, with
// avail bytes readable at p[0], p[-1], ... (0 = none).
uint32_t pm_rt_host_answer(const RtImage& im, const uint8_t* p, size_t avail);

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
