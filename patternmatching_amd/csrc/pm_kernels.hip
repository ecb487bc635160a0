// pm_kernels.hip -- gfx950 kernels of the stream scan (read_char batched).
//
// rt_scan_kernel  one wave per 1024 consecutive stream positions.  For each
//   position i it walks the reverse-suffix trie backwards over
//   text[i], text[i-1], ... and emits the gid of the deepest pattern node
//   met, which is exactly the id ac_read_char returns at i
//   (Core/src/mpac.c:304-319: the longest pattern that is a suffix of the
//   stream so far).  Positions are independent: no carried state, no
//   warm-up.  Per position:
//     depth <= 2   one u16 lookup in an LDS-resident 64K table keyed by the
//                  last two bytes (t12);
//     depth 3      only when t12 says the depth-2 node has children: a
//                  3-bit blocked Bloom filter in LDS over the 3-byte
//                  suffixes that exist (stage 1; ~1.9% of random-ASCII
//                  positions pass, no false negatives), then a second LDS
//                  filter over 3-byte patterns and 4-byte suffixes (stage 2);
//     queue        per wave, filled with DPP prefix offsets and drained by
//                  all 64 lanes at once: one probe of an L2-resident cuckoo
//                  table of depth-3 suffixes and, past depth 3, one 16-B
//                  node record per step;
//     spill/tail   what the queue cannot hold goes to a per-wave region,
//                  resolved after the chunk loop in two uniform phases
//                  (batched probes, then lock-step walks that take a run of
//                  one-child nodes per step from its chain record).
//   Each lane owns four groups of four consecutive positions at stride 256,
//   so every load instruction reads 256 contiguous bytes and every store
//   instruction writes 1 KiB of contiguous match ids; the next chunk's bytes
//   are loaded while the current one is resolved.
//
// dfa_coded_kernel / dfa_scan_kernel  the reference automaton itself,
//   flattened to a dense DFA whose transition words carry their target's
//   output (next[s*256+c] = target | code << 20; the uncoded form for
//   automata of 2^20 states or more); one lane per stream segment (two in
//   lock step when coded), started from the root max_len-1 bytes before the
//   segment (SURVEY.md §0.1 shard rule), so every segment is independent
//   and exact.
//
// dfa_sparse_kernel  the same automaton in its sparse form: full rows only
//   for states whose row differs from their fallback's in more than two
//   bytes, 16-B default-transition records for the rest (pm_flatten.h).  A
//   step is one 16-B load (a row's quad, or the record) plus, at a record
//   whose two bytes miss, one 4-B load of the fallback's row.  The plugin
//   times both forms and keeps the faster per input (pm_plugin.hip).
//   Product kernel of the form: dfa_sparse_lds_kernel without LDS rows --
//   each lane keeps the aligned block of 4 records holding its state in
//   registers -- at two 512-lane workgroups per CU.
#include <type_traits>

#include <algorithm>

#include "pm_kernels.h"
#include "pm_streamgen.h"

namespace {

// The chunk's answer stores (A/B builds: -DRT_PLAIN_STORES keeps the lines
// in L2 for the patches that follow a round later)
#ifdef RT_PLAIN_STORES
#define RT_OUT_STORE(v, p) (*(p) = (v))
#else
#define RT_OUT_STORE(v, p) __builtin_nontemporal_store((v), (p))
#endif
constexpr int RT_THREADS = 1024;
constexpr int RT_WAVES = RT_THREADS / 64;
constexpr int RT_T2_U16 = 65536;
constexpr int RT_FILTER_WORDS = 4096;  // must match pm_flatten.h
constexpr int RT_F3_WORDS = 256;        // stage-2 filter words, must match pm_flatten.h
constexpr int RT_F2_WORDS = 2048;
constexpr uint32_t RT_QCAP = 64;        // queue ring per wave (power of two, <= 64: one item per lane)
constexpr uint32_t RT_ROUND = 40;       // a round is issued once this many are queued
constexpr int RT_CHUNK = 1024;         // positions per wave iteration
constexpr uint32_t CONT16 = 0x8000u;
constexpr uint32_t CONT32 = 0x80000000u;
constexpr uint32_t T3H_VALID = 1u << 24;
constexpr uint32_t RT_POSMASK = (1u << 30) - 1;  // queue item: position - pos0
constexpr uint32_t RT_SLOT2 = 1u << 30;          // queue item: probe t3h slot2
constexpr uint32_t RT_REC_LEAF_K = 0, RT_REC_KIDS_K = 1, RT_REC_CHAIN_K = 2, RT_REC_WIDE_K = 3;  // record kinds, must match pm_flatten.h

__device__ __forceinline__ uint32_t rt_hash(uint32_t k) { return k * 0x9E3779B1u; }  // pm_rt_hash
// pm_rt_fhash of the low 24 bits of k (the operand's top byte is ignored):
// one full-rate v_mul_u32_u24 (written
// out: the compiler loses the 24-bit range through the byte extraction and
// would emit the quarter-rate v_mul_lo_u32)
__device__ __forceinline__ uint32_t rt_fhash(uint32_t k) {
    uint32_t h;
    asm("v_mul_u32_u24 %0, 0x9e3779, %1" : "=v"(h) : "v"(k));
    return h;
}
// the three filter bits of f (pm_rt_filter_mask) present in word w: shifts
// by bytes 0, 1, 2 of f (a shift uses bits 0-4 of its amount)
__device__ __forceinline__ uint32_t rt_fhit(uint32_t w, uint32_t f) {
    uint32_t a, b, c;  // written out: the compiler extracts the bytes with extra shifts
    asm("v_lshrrev_b32_e32 %0, %1, %2" : "=v"(a) : "v"(f), "v"(w));
    asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
        : "=v"(b) : "v"(f), "v"(w));
    asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD"
        : "=v"(c) : "v"(f), "v"(w));
    return a & b & c & 1u;
}

// Stage 2 of the filter for q = text[i-3..i] (pm_rt_p3hash / pm_rt_s4hash):
// nonzero when key24 = q >> 8 may be a 3-byte pattern or q a depth-4 suffix.
// Split in two so the LDS reads can be issued well before the test.
struct Stage2 {
    uint32_t g3, g4, w3, w4;
};
__device__ __forceinline__ Stage2 rt_stage2_load(const uint32_t* s_f2, uint32_t q) {
    Stage2 z;
    asm("v_mul_u32_u24 %0, 0x85ebca, %1" : "=v"(z.g3) : "v"(q >> 8));
    z.g4 = q * 0x9E3779B1u;
    z.w3 = s_f2[z.g3 >> 24];
    z.w4 = s_f2[RT_F3_WORDS + (((z.g4 >> 20) * 7u) >> 4)];
    return z;
}
__device__ __forceinline__ uint32_t rt_stage2_hit(const Stage2& z) { return rt_fhit(z.w3, z.g3) | rt_fhit(z.w4, z.g4); }

// Inclusive prefix sum over the 64 lanes: row_shr 1/2/4/8 within rows of 16,
// then row_bcast 15 / 31 across rows (lanes without a source add 0).
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

__device__ __forceinline__ uint32_t wave_prefix(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// One record step (pm_flatten.h 16-B records): R = the record of the node
// reached after text[i] .. text[i-d+1], c = text[i-d].  Returns the next
// record, or -1 when the walk ends here (answer R.y).  A wide node's child
// needs its `wide` entry W = {bitmap word, prefix} of word c >> 5.
template <class V4>
__device__ __forceinline__ uint32_t rec_kind(const V4& R) { return R.x >> 30; }
// inline children: index of byte c among the record's cnt child bytes, or cnt
// (the zero-byte test of payload ^ c*0x01010101: the lowest flagged byte is
// exact; later flags are masked off by j < cnt, and bytes are distinct)
template <class V4>
__device__ __forceinline__ uint32_t rec_kid_index(const V4& R, uint32_t c) {
    const uint32_t c4 = c * 0x01010101u;
    const uint32_t lo = R.z ^ c4, hi = R.w ^ c4;
    const uint32_t zl = (lo - 0x01010101u) & ~lo & 0x80808080u;
    const uint32_t zh = (hi - 0x01010101u) & ~hi & 0x80808080u;
    const uint32_t cnt = (R.x >> 24) & 63u;
    const uint32_t j = zl ? (uint32_t)__builtin_ctz(zl) >> 3 : zh ? 4u + ((uint32_t)__builtin_ctz(zh) >> 3) : 8u;
    return j < cnt ? j : cnt;
}

// A wide node's quarter Q = {word 2q, word 2q+1, child index of word 2q,
// best} for byte c (q = c >> 6): the child's record, or ~0u when c is not
// a child (the answer is then Q.w).
template <class V4>
__device__ __forceinline__ uint32_t wide_child(const V4& Q, uint32_t c) {
    const uint32_t odd = (c >> 5) & 1u, bit = c & 31u;
    const uint32_t word = odd ? Q.y : Q.x;
    if (!((word >> bit) & 1u)) return ~0u;
    return Q.z + (odd ? (uint32_t)__popc(Q.x) : 0u) + (uint32_t)__popc(word & ((1u << bit) - 1u));
}

// Record walk, one position (edge chunks): node = record reached after
// consuming text[i] .. text[i-d+1]; avail = bytes at or before i.
__device__ __forceinline__ uint32_t rt_deep(const uint8_t* __restrict__ text, const RtDev& t, uint32_t node, int64_t i,
                                            int64_t avail, int64_t d) {
    for (;;) {
        const uint4 R = t.rec[node];
        if (d >= avail) return R.y;
        const uint32_t c = text[i - d];
        const uint32_t kind = rec_kind(R), first = R.x & 0xFFFFFFu;
        if (kind == RT_REC_LEAF_K) return R.y;
        if (kind == RT_REC_CHAIN_K) {
            // the run's leading bytes that match, in one step (pm_flatten.h
            // RT_REC_CHAIN: b_k at byte 7 - k of w:z); bytes past the run or
            // the stream are read at an in-range position and not counted
            const uint32_t L = (R.x >> 24) & 63u;
            const uint32_t lim = avail - d < (int64_t)L ? (uint32_t)(avail - d) : L;  // >= 1
            uint64_t win = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t kk = (uint32_t)k < lim ? (uint32_t)k : lim - 1u;
                win |= (uint64_t)text[i - d - kk] << (8 * (7 - k));
            }
            const uint64_t dif = win ^ ((uint64_t)R.w << 32 | R.z);
            uint32_t m = dif ? (uint32_t)__builtin_clzll(dif) >> 3 : 8u;
            m = m < lim ? m : lim;
            // stopped inside the run: no pattern ends at its inner records,
            // so the answer is this record's (as the chunk loop's rounds take it)
            if (m < L) return R.y;
            node = first + m - 1u;
            d += m;
            continue;
        } else if (kind == RT_REC_KIDS_K) {
            const uint32_t j = rec_kid_index(R, c);
            if (j == ((R.x >> 24) & 63u)) return R.y;
            node = first + j;
        } else {
            const uint32_t ch = wide_child(t.wide[(size_t)R.z * 4 + (c >> 6)], c);
            if (ch == ~0u) return R.y;
            node = ch;
        }
        ++d;
    }
}

__device__ __forceinline__ uint32_t rt_slot1(uint32_t k, uint32_t bits) { return rt_hash(k) >> (32 - bits); }
__device__ __forceinline__ uint32_t rt_slot2(uint32_t k, uint32_t bits) { return (k * 0x85EBCA77u) >> (32 - bits); }

// The walk past depth 2 from key24 = text[i-2] | text[i-1] << 8 | text[i] << 16
// (a depth-2 node with children) with c3 = text[i-3] when avail >= 4;
// best2 = the answer if it stops at depth 2.  The t3h entry of key24 (slot1
// or slot2) decides depth 3 and, for nodes with at most three children,
// whether the walk goes on past depth 4.
__device__ __forceinline__ uint32_t rt_from_d2(const uint8_t* __restrict__ text, const RtDev& t, uint32_t key24,
                                               uint32_t c3, uint32_t best2, int64_t i, int64_t avail) {
    const uint32_t want = T3H_VALID | key24;
    uint4 e = t.t3h[rt_slot1(key24, t.t3h_bits)];
    if ((e.x & 0x1FFFFFFu) != want) {
        e = t.t3h[rt_slot2(key24, t.t3h_bits)];
        if ((e.x & 0x1FFFFFFu) != want) return best2;
    }
    const uint32_t kind = e.x >> 25;
    if (kind == 0 || avail < 4) return e.y;
    if (kind == 1) {
        const uint32_t nch = e.z >> 24;
        const uint32_t k = c3 == (e.z & 0xFFu) ? 0u : c3 == ((e.z >> 8) & 0xFFu) ? 1u : c3 == ((e.z >> 16) & 0xFFu) ? 2u : 3u;
        if (k >= nch) return e.y;
        if (nch > 1) return rt_deep(text, t, e.w + k, i, avail, 4);
        if (!(e.w & CONT32)) return e.w;
        return rt_deep(text, t, e.w & 0x7FFFFFFFu, i, avail, 4);
    }
    return rt_deep(text, t, e.w & 0x7FFFFFFFu, i, avail, 3);
}

// One position, every boundary case (stream start, short lookback).
__device__ uint32_t rt_one(const uint8_t* __restrict__ text, const uint16_t* s_t, const RtDev& t, int64_t i,
                           int64_t stream_start) {
    const int64_t avail = i - stream_start + 1;
    const uint32_t c0 = text[i];
    if (avail == 1) return t.t12[65536 + c0];
    const uint32_t c1 = text[i - 1];
    const uint32_t v = s_t[(c0 << 8) | c1];
    if (!(v & CONT16) || avail == 2) return v & 0x7FFFu;
    return rt_from_d2(text, t, text[i - 2] | (c1 << 8) | (c0 << 16), avail >= 4 ? text[i - 3] : 0u, v & 0x7FFFu, i,
                      avail);
}

// V (ablation, timing only; V=0 is the product kernel):
//   1 = loads + t12 lookups + stores (no filter, no queue)
//   2 = loads + stores only (streaming floor of this access pattern)
// OUTW: bytes per written id: 4 (u32 gids, read_block), 2 (u16 gids, when
// every gid < 65536), 0 (count only).
template <int OUTW>
__device__ __forceinline__ void put_id(void* out, int64_t k, uint32_t v) {
    if (OUTW == 4) reinterpret_cast<uint32_t*>(out)[k] = v;
    if (OUTW == 2) reinterpret_cast<uint16_t*>(out)[k] = (uint16_t)v;
}

// f(integral_constant<int, 0>) .. f(integral_constant<int, N-1>): a loop the
// compiler sees fully unrolled with constant indices (per-slot state stays
// in registers)
template <int I, int N, class F>
__device__ __forceinline__ void unroll_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        unroll_for<I + 1, N>(f);
    }
}

using tu32x2 = __attribute__((ext_vector_type(2))) unsigned int;
using tu32x4 = __attribute__((ext_vector_type(4))) unsigned int;

// The deep work of one wave's spilled candidates, after its chunk loop.
// Items sp[0, sn) are {text[i-3..i], position - pos0 | placeholder-nonzero
// << 31} (8 B).  Two phases, each uniform code:
//  1. probe: batches of 64 * RT_PROBE_G items, one per lane per group:
//     stage 2, the t3h slot1 probe (slot2 where slot1 holds another key).
//     A position that resolves there is written; one whose walk goes on
//     is compacted in place into a walk entry {record, position - pos0 |
//     (depth == 4) << 30 | placeholder-nonzero << 31}.
//  2. walk: RT_TAIL_SLOTS walks per lane in lock step, refilled from the
//     walk entries; each iteration issues one record (or wide quarter)
//     load and, when the next byte is not in the lane's 8 cached text
//     bytes, the aligned 8 bytes holding it.  A wave keeps 64 *
//     RT_TAIL_SLOTS dependent chains in flight with a short branch-free
//     body per step.
// Each position ends by writing its answer and settling the count against
// its placeholder.  (Measured and not kept: fetching the walk's first text
// bytes in phase 1, with 16-B entries, and writing the walk answers in
// position order from the entries afterwards -- both slower.)
constexpr int RT_PROBE_G = 4;
constexpr int RT_TAIL_SLOTS = 4;
constexpr uint32_t RT_D4 = 1u << 30;  // walk entry: starts at depth 4 (else 3)
enum : uint32_t { TS_EMPTY = 0, TS_ENTRY, TS_REC, TS_WIDE };

// One in-flight walk.  Offsets are u32 from pos0; pa / pb are the next
// iteration's load addresses, so issuing is two loads per slot whatever the
// state.
struct TailSlot {
    uint32_t st;          // TS_*
    uint32_t pos;         // position - pos0 | placeholder-nonzero << 31
    uint32_t av;          // bytes at or before the position, capped at 1024
    uint32_t node, dd;    // record, depth (bytes consumed)
    uint32_t c;           // TS_WIDE: the byte being decided; TS_ENTRY: entry parity
    uint32_t tlo, thi;    // cached text bytes [twa, twa + 8)
    int32_t twa;          // (4-aligned, may precede pos0)
    const tu32x4* pa;
    const tu32x2* pb;
    tu32x4 A;             // this iteration's 16-B load
    tu32x2 B;             // this iteration's 8-B load
};

template <int OUTW, bool kProbeOnly = false, int SLOTS = RT_TAIL_SLOTS>
__device__ __forceinline__ uint32_t rt_tail(const uint8_t* __restrict__ text, int64_t stream_start, int64_t pos0,
                                        void* __restrict__ out, const RtDev& t, const uint32_t* s_f2,
                                        uint32_t* sp, uint32_t sn, int lane, uint32_t& cnt) {
    const uint8_t* const tb = text + pos0;  // offsets are from pos0; pos0 % 16 == 0
    const int64_t ctx64 = pos0 - stream_start;  // context bytes before pos0
    const uint32_t ctx = ctx64 > 1024 ? 1024u : (uint32_t)ctx64;
    const tu32x4* const dummy4 = reinterpret_cast<const tu32x4*>(t.filt);
    const tu32x2* const dummy2 = reinterpret_cast<const tu32x2*>(t.filt);
    const tu32x4* const T3 = reinterpret_cast<const tu32x4*>(t.t3h);
    const tu32x4* const RC = reinterpret_cast<const tu32x4*>(t.rec);
    const tu32x4* const WD = reinterpret_cast<const tu32x4*>(t.wide);
    tu32x2* const items = reinterpret_cast<tu32x2*>(sp);

    // ---- phase 1: probes ------------------------------------------------
    uint32_t nwalk = 0;  // wave-uniform
    for (uint32_t base = 0; base < sn; base += 64 * RT_PROBE_G) {
        tu32x2 it[RT_PROBE_G];
        tu32x4 e[RT_PROBE_G];
        bool act[RT_PROBE_G];
        unroll_for<0, RT_PROBE_G>([&](auto g) __attribute__((always_inline)) {
            const uint32_t idx = base + 64 * g + lane;
            it[g] = idx < sn ? items[idx] : tu32x2{0u, 0u};
            act[g] = idx < sn && rt_stage2_hit(rt_stage2_load(s_f2, it[g].x)) != 0u;
        });
        unroll_for<0, RT_PROBE_G>([&](auto g) __attribute__((always_inline)) {
            e[g] = act[g] ? T3[rt_slot1(it[g].x >> 8, t.t3h_bits)] : *dummy4;
        });
        bool need2[RT_PROBE_G];
        bool any2 = false;
        unroll_for<0, RT_PROBE_G>([&](auto g) __attribute__((always_inline)) {
            const uint32_t want = T3H_VALID | (it[g].x >> 8);
            need2[g] = act[g] && (e[g].x & 0x1FFFFFFu) != want && (e[g].x & T3H_VALID);
            any2 |= need2[g];
        });
        if (__ballot(any2)) {  // wave-uniform
            unroll_for<0, RT_PROBE_G>([&](auto g) __attribute__((always_inline)) {
                if (need2[g]) e[g] = T3[rt_slot2(it[g].x >> 8, t.t3h_bits)];
            });
        }
        unroll_for<0, RT_PROBE_G>([&](auto g) __attribute__((always_inline)) {
            const tu32x4 E = e[g];
            const uint32_t key = it[g].x, pw = it[g].y, off = pw & RT_POSMASK;
            const bool match = act[g] && (E.x & 0x1FFFFFFu) == (T3H_VALID | (key >> 8));
            const uint32_t kind = E.x >> 25, nch = E.z >> 24, c3 = key & 0xFFu;
            const uint32_t j = c3 == (E.z & 0xFFu) ? 0u : c3 == ((E.z >> 8) & 0xFFu) ? 1u
                             : c3 == ((E.z >> 16) & 0xFFu) ? 2u : 3u;
            const bool deep4 = off + ctx >= 3;  // avail >= 4
            const bool inl = kind == 1 && j < nch && nch == 1 && !(E.w & CONT32);
            const bool walk = match && deep4 && ((kind == 1 && j < nch && !inl) || kind == 2);
            const uint32_t node = (kind == 2 || nch == 1) ? E.w & 0x7FFFFFFFu : E.w + j;
            const uint32_t ans = (deep4 && inl) ? E.w : E.y;
            if (match && !walk) {
                cnt += (uint32_t)(ans != 0u) - (pw >> 31);
                if (OUTW) put_id<OUTW>(out, (int64_t)off, ans);
            }
            // walk entries compacted in place: entry nwalk + k never passes
            // an item not yet read (every item of this batch is in registers)
            const uint64_t m = __ballot(walk);
            if (walk) items[nwalk + wave_prefix(m)] = tu32x2{node, (pw & ~RT_D4) | (kind == 1 ? RT_D4 : 0u)};
            nwalk += (uint32_t)__popcll(m);
        });
    }
    if (!nwalk || kProbeOnly) return nwalk;
    // the walk entries are stored (vmcnt 0) and this CU's L1 dropped
    // (phase 1 read the same lines before overwriting them) before they are
    // read
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");

    // ---- phase 2: walks -------------------------------------------------
    TailSlot S[SLOTS];
    unroll_for<0, SLOTS>([&](auto I) __attribute__((always_inline)) {
        TailSlot& z = S[I];
        z.st = TS_EMPTY;
        z.pos = z.av = z.node = z.dd = z.c = z.tlo = z.thi = 0;
        z.twa = 0;
        z.pa = dummy4;
        z.pb = dummy2;
        z.A = tu32x4{0u, 0u, 0u, 0u};
        z.B = tu32x2{0u, 0u};
    });
    uint32_t nxt = 0;  // wave-uniform: next unclaimed walk entry
    for (;;) {
        bool busy = false;
        unroll_for<0, SLOTS>([&](auto I) __attribute__((always_inline)) {
            TailSlot& z = S[I];
            const bool need = z.st == TS_EMPTY;
            const uint64_t m = __ballot(need);
            const uint32_t idx = nxt + wave_prefix(m);
            if (need && idx < nwalk) {
                z.st = TS_ENTRY;
                z.c = idx & 1u;  // the entry's half of the 16-B load
                z.pa = reinterpret_cast<const tu32x4*>(items + (idx & ~1u));
                z.pb = dummy2;
            }
            nxt += (uint32_t)__popcll(m);
            if (nxt > nwalk) nxt = nwalk;
            busy |= z.st != TS_EMPTY;
        });
        if (!__ballot(busy)) break;  // wave-uniform
        unroll_for<0, SLOTS>([&](auto I) __attribute__((always_inline)) {
            TailSlot& z = S[I];
            z.A = *z.pa;
            z.B = *z.pb;
        });
        // branch-free step: each state's outcome is computed and the slot's
        // own selected (divergent branches cost more: exec-mask bookkeeping
        // and register merges)
        unroll_for<0, SLOTS>([&](auto I) __attribute__((always_inline)) {
            TailSlot& z = S[I];
            const uint32_t st = z.st;
            const tu32x4 A = z.A;
            // TS_ENTRY: {record, position | d4 | ph}
            const uint32_t en = z.c ? A.z : A.x, ep = z.c ? A.w : A.y;
            // TS_REC: A is the record; B the aligned 8 text bytes holding
            // text[i-d] when they were not cached
            const uint32_t off = z.pos & RT_POSMASK;
            const int32_t rq = (int32_t)off - (int32_t)z.dd;
            const bool reload = rq < z.twa || rq >= z.twa + 8;
            const uint32_t rlo = reload ? z.B.x : z.tlo, rhi = reload ? z.B.y : z.thi;
            const int32_t rta = reload ? (rq & ~7) : z.twa;
            const uint32_t ro = (uint32_t)(rq - rta);
            const uint32_t c = ((ro & 4 ? rhi : rlo) >> (8 * (ro & 3))) & 0xFFu;
            const uint32_t rkind = rec_kind(A), first = A.x & 0xFFFFFFu;
            const uint32_t jr = rec_kid_index(A, c);
            const bool rend = z.dd >= z.av;
            const bool rnext = !rend && rkind == RT_REC_KIDS_K && jr != ((A.x >> 24) & 63u);
            const bool rwide = !rend && rkind == RT_REC_WIDE_K;
            // TS_REC at a CHAIN record: the run's bytes against text[i-d],
            // text[i-d-1], ... as far as the cached window, the run and the
            // stream allow, in one step (window byte ro to the top byte, then
            // the leading equal bytes of the two 64-bit words)
            const uint64_t win = ((uint64_t)rhi << 32 | rlo) << (8 * (7 - ro));
            const uint64_t dif = win ^ ((uint64_t)A.w << 32 | A.z);
            const uint32_t meq = dif ? (uint32_t)__builtin_clzll(dif) >> 3 : 8u;
            const uint32_t clen = (A.x >> 24) & 63u;
            const uint32_t cav = z.av > z.dd ? z.av - z.dd : 0u;
            const uint32_t clim = min(min(clen, ro + 1u), cav);
            const uint32_t cm = min(meq, clim);
            const bool cnext = rkind == RT_REC_CHAIN_K && cm >= 1u && (cm == clen || (cm == ro + 1u && cm < cav));
            // TS_WIDE: A is the quarter of the wide entry holding byte c
            const uint32_t wnode = wide_child(A, z.c);
            const bool wnext = wnode != ~0u;

            uint32_t nst = TS_EMPTY;
            bool fin = false;
            uint32_t ans = A.w;  // TS_WIDE: the node's best
            if (st == TS_ENTRY) {
                nst = TS_REC;
                z.node = en;
                z.dd = (ep & RT_D4) ? 4u : 3u;
                z.pos = ep & ~RT_D4;
                const uint32_t o = ep & RT_POSMASK;
                z.av = o + ctx + 1 > 1024u ? 1024u : o + ctx + 1;
                z.twa = INT32_MIN / 2;  // nothing cached
            }
            if (st == TS_REC) {
                nst = (rnext || cnext) ? TS_REC : rwide ? TS_WIDE : TS_EMPTY;
                fin = !rnext && !rwide && !cnext;
                ans = A.y;
                z.tlo = rlo;
                z.thi = rhi;
                z.twa = rta;
                z.node = cnext ? first + cm - 1u : first + jr;
                z.dd += rnext ? 1u : cnext ? cm : 0u;
                z.c = c;
            }
            if (st == TS_WIDE) {
                nst = wnext ? TS_REC : TS_EMPTY;
                fin = !wnext;
                z.node = wnode;
                z.dd += 1;
            }
            if (fin) {
                cnt += (uint32_t)(ans != 0u) - (z.pos >> 31);
                if (OUTW) put_id<OUTW>(out, (int64_t)(z.pos & RT_POSMASK), ans);
            }
            z.st = nst;
            // the next state's loads
            const int32_t nq = (int32_t)(z.pos & RT_POSMASK) - (int32_t)z.dd;
            const bool nreload = z.dd < z.av && (nq < z.twa || nq >= z.twa + 8);
            const tu32x4* pa = dummy4;
            const tu32x2* pb = dummy2;
            if (nst == TS_REC) {
                pa = RC + z.node;
                if (nreload) pb = reinterpret_cast<const tu32x2*>(tb + (nq & ~7));
            }
            if (nst == TS_WIDE) pa = WD + (size_t)A.z * 4 + (c >> 6);  // the quarter holding byte c
            z.pa = pa;
            z.pb = pb;
        });
    }
    return nwalk;
}

// EF: issue the prefetch of chunk c + 2 as soon as chunk c's bytes are in
// the window registers, ahead of the round and the stores (vmcnt retires in
// order, so a chunk's wait for its bytes then leaves two chunks of stores in
// flight instead of one).
template <int V, int OUTW, bool EF = false>
__global__ __launch_bounds__(RT_THREADS) void rt_scan_kernel(const uint8_t* __restrict__ text, int64_t stream_start,
                                                             int64_t pos0, int64_t n, void* __restrict__ out,
                                                             unsigned long long* __restrict__ count, RtDev t) {
    // One LDS block with fixed offsets, 16 + 128 + 8 + 8 KiB: all of the
    // CU's LDS.  The stage-1 filter sits at address 0, so a filter word's
    // address is the hash bits alone, and t12 at 16 KiB, which fits the
    // ds_read offset field: neither per-position address needs a base add.
    // Count only (V = 0, OUTW = 0) needs two bits of a depth-2 answer, not
    // the answer: whether it is nonzero (the position counts, however deep
    // its walk goes) and whether it is zero with a depth-2 node that has
    // children (the position is a candidate for the tail).  It keeps them
    // as one byte per key, t8 = nz | cand << 1 (64 KiB, derived from t12
    // while staging), at LDS address 0: the 16-bit key (text[i] << 8 |
    // text[i-1]) is the byte address, one ds_read_u8, no base add or mask.
    // V: 0 = the product kernel, 2 = its streaming floor (the chunk loop's
    // loads and stores, no lookups: bench.py's live floor; its ids are not
    // matches).  Round-4 and earlier ablation variants are in git history.
    static_assert(V == 0 || V == 2, "product kernel (0) or streaming floor (2)");
    constexpr bool kT8 = V == 0 && OUTW == 0;
    constexpr int kLdsWords = kT8 ? RT_T2_U16 / 4 + RT_F2_WORDS + 2 * RT_WAVES * RT_QCAP
                                  : RT_FILTER_WORDS + RT_T2_U16 / 2 + RT_F2_WORDS + 2 * RT_WAVES * RT_QCAP;
    __shared__ __attribute__((aligned(16))) uint32_t s_lds[kLdsWords];
    uint32_t* const s_f = s_lds;
    const uint8_t* const s_t8 = reinterpret_cast<const uint8_t*>(s_lds);
    // (count only: rt_one reads the depth-2 answers from global t12)
    const uint16_t* const s_t = kT8 ? t.t12 : reinterpret_cast<uint16_t*>(s_lds + RT_FILTER_WORDS);
    uint32_t* const s_f2 = s_lds + (kT8 ? RT_T2_U16 / 4 : RT_FILTER_WORDS + RT_T2_U16 / 2);
    uint32_t(*const s_qkey)[RT_QCAP] = reinterpret_cast<uint32_t(*)[RT_QCAP]>(s_f2 + RT_F2_WORDS);
    uint32_t(*const s_qpos)[RT_QCAP] = s_qkey + RT_WAVES;
    {
        const uint4* fsrc = reinterpret_cast<const uint4*>(t.filt);
        if (kT8) {
            const uint2* src = reinterpret_cast<const uint2*>(t.t12);  // 4 keys per thread step
            for (int k = threadIdx.x; k < RT_T2_U16 / 4; k += RT_THREADS) {
                const uint2 v = src[k];
                const uint32_t e[4] = {v.x & 0xFFFFu, v.x >> 16, v.y & 0xFFFFu, v.y >> 16};
                uint32_t w = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t nz = (e[q] & 0x7FFFu) != 0u, cand = !nz && (e[q] & CONT16);
                    w |= (nz | cand << 1) << (8 * q);
                }
                s_lds[k] = w;
            }
        } else {
            const uint4* src = reinterpret_cast<const uint4*>(t.t12);
            uint4* dst = reinterpret_cast<uint4*>(s_lds + RT_FILTER_WORDS);
            for (int k = threadIdx.x; k < RT_T2_U16 * 2 / 16; k += RT_THREADS) dst[k] = src[k];
            uint4* fdst = reinterpret_cast<uint4*>(s_f);
            for (int k = threadIdx.x; k < RT_FILTER_WORDS / 4; k += RT_THREADS) fdst[k] = fsrc[k];
        }
        uint4* f2dst = reinterpret_cast<uint4*>(s_f2);
        for (int k = threadIdx.x; k < RT_F2_WORDS / 4; k += RT_THREADS) f2dst[k] = fsrc[RT_FILTER_WORDS / 4 + k];
    }
    __syncthreads();

    constexpr bool kFilter = V == 0;
    // Stage 2 at push time: only its passers are queued, so rounds are ~3.3x
    // rarer and all their candidates probe.  Rounds in the chunk loop, or
    // every candidate to the spill region for the tail.  Side by side
    // (scripts/bench_variants.py; V = 8: push-time stage 2 with rounds, V =
    // 9: push-time stage 2, no rounds; snort / merged / shipped stream, ms):
    //   u32   issue-time 1.141 / 1.167 / 12.28   V8 1.135 / 1.149 / 11.52
    //         V9 1.178 / - / 11.26
    //   u16   issue-time 0.830 / 0.971 / 11.83   V8 0.838 / 0.970 / 10.57
    //         V9 0.809 / 1.012 / 10.71
    //   count issue-time 0.784 / 0.910 / 8.68    V8 0.807 / 0.944 / 8.05
    //         V9 0.768 / 0.882 / 8.00
    //         V10 (no rounds, stage 2 in the tail's batched probe phase)
    //         0.733 / 0.832 / 8.63 (V9 on the same box 0.763 / 0.879 / 7.95)
    // So the product: u32 = V8, count = V10, u16 = issue-time stage 2.
    // (Count only with stage 2 at push time too measured slower: 0.440 ->
    // 0.473 ms, profiles/r04/count_ablations.)
    constexpr bool kPushS2 = V == 0 && OUTW == 4;
    constexpr bool kRounds = !(V == 0 && OUTW == 0);
    // the stage-1 LDS filter; count-only without it (V = 0) queues every
    // zero-placeholder position under a depth-2 node with children (2.3%
    // of random-ASCII positions on snort) for the tail's batched stage 2
    constexpr bool kStage1 = !(V == 0 && OUTW == 0);
    const int lane = threadIdx.x & 63;
    // wave id through readfirstlane: the compiler then knows every per-chunk
    // quantity below is wave-uniform (scalar loop, no exec-mask loop)
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t* qkey = s_qkey[wid];
    uint32_t* qpos = s_qpos[wid];
    uint32_t cnt = 0;   // per lane
    uint32_t scnt = 0;  // per wave (scalar): the chunks' nonzero placeholders
    // chunk c is "fast" (main loop) when all of it is in range and it starts
    // >= 2 bytes into the stream: chunks [c_lo, c_hi)
    const int64_t nchunks = (n + RT_CHUNK - 1) / RT_CHUNK;
    const int64_t c_hi = n / RT_CHUNK;
    const int64_t c_lo = pos0 - stream_start >= 2 ? 0 : 1;
    // this wave's chunks: cbeg, cbeg + cstep, ... below cend
    const int64_t gw = (int64_t)blockIdx.x * RT_WAVES + wid;
    const int64_t nw = (int64_t)gridDim.x * RT_WAVES;
    const int64_t cbeg = c_lo + gw, cend = c_hi, cstep = nw;
    // this wave's spill region: the candidates of chunks whose queue room
    // ran out (dense deep matches), {text[i-3..i], position - pos0 |
    // placeholder-nonzero << 31}, resolved after the chunk loop (rt_tail).
    // At most one item per position of the wave's chunks, which is the
    // region's size.
    uint32_t* const sp = t.spill + 2 * gw * t.spill_stride;  // 8-B items
    uint32_t sn = 0;  // wave-uniform
    // out-of-range prefetches read this instead (any >= 1 KiB of table)
    const uint8_t* dummy = reinterpret_cast<const uint8_t*>(t.filt) + 4;
    using u32x2 = __attribute__((ext_vector_type(2))) unsigned int;
    using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

    // Resolve queue.  An item is a depth-3 candidate (qkey = the LE u32
    // text[i-3..i] = text[i-3] | key24 << 8) or a record step (qpos bit 31;
    // qkey = record | depth << 23); qpos = position - pos0 (30 bits) |
    // probe-slot2 << 30.  The match count is settled when a candidate
    // resolves or turns into record steps (its placeholder is the t12 entry
    // of its key, recomputed then).  A candidate probes t3h slot1 only: the
    // key there resolves it, and so does an empty slot1 (cuckoo entries are
    // only ever swapped, so a key whose slot1 is empty is absent); only a
    // slot1 holding another key sends it to slot2 next round.  A record step
    // (qkey = record | depth << 23) loads the 16-B record and the next
    // stream byte; at a wide record (more than RT_REC_INLINE children) the
    // item turns into a wide step (qpos bit 30; qkey = entry | byte << 14 |
    // depth << 22) that loads the one 16-B quarter of the entry deciding
    // the byte.  So a round has one scattered load per item.
    // Rounds are software-pipelined: issue() loads one set per item into the
    // round registers, and consume() uses them in the next chunk iteration,
    // so the load latency hides behind a chunk's store, push and LDS work.
    // Unfinished items go back to the queue for the next round.  The chunk
    // loop is unrolled by two with fixed A/B text windows, so no loaded
    // register is ever copied (a copy would wait for the load), and every
    // round issues the same two loads (idle lanes read a harmless address),
    // so the vmcnt the compiler computes is static: waiting for a chunk's
    // bytes or for a round never waits for the younger rounds, stores and
    // prefetches.
    // Ordering: items of chunk k are issued after chunk k's placeholder
    // store, and vmcnt retires in order, so a round's results imply the
    // stores of its items are complete at L2 before any patch overwrites one.
    struct Round {
        uint32_t n;     // items (wave-uniform)
        uint32_t keep;  // items that may survive the round (wave-uniform): ring room they hold
        uint32_t fk, fp;
        u32x2 tw;       // record steps: the aligned 8 text bytes holding text[i-d]
        uint32_t skip;  // stage 2 rejected the item: its answer is the placeholder
        u32x4 L0;
    };
    // The queue is a ring of RT_QCAP items per wave: head qh, count qn.  A
    // round takes all queued items once RT_ROUND are queued (idle chunks
    // issue an empty round: same loads, harmless addresses), so every round
    // runs all 64 lanes.
    uint32_t qh = 0, qn = 0;  // wave-uniform
    auto issue = [&](Round& r, uint32_t take) __attribute__((always_inline)) {
        __builtin_amdgcn_wave_barrier();
        const bool act = (uint32_t)lane < take;
        const uint32_t sl = (qh + lane) & (RT_QCAP - 1);
        r.fk = act ? qkey[sl] : 0u;
        r.fp = act ? qpos[sl] : 0u;
        const bool deep = r.fp >> 31;
        // stage 2 on first probes: only a 3-byte pattern or a depth-4 suffix
        // can change the placeholder, anything else needs no probe
        bool skip = false;
        if (!kPushS2 && take) {  // wave-uniform
            const bool first = act && !deep && !(r.fp & RT_SLOT2);
            if (first) skip = rt_stage2_hit(rt_stage2_load(s_f2, r.fk)) == 0u;
        }
        r.skip = skip;
        r.keep = (uint32_t)__popcll(__ballot(act && !skip));
        const uint32_t k = r.fk >> 8;
        const uint32_t node = r.fk & 0x7FFFFFu, d = r.fk >> 23;
        const bool wide = deep && (r.fp & RT_SLOT2);  // record step at a wide node: its quarter
        const int64_t i = pos0 + (int64_t)(r.fp & RT_POSMASK);
        const u32x4* T = reinterpret_cast<const u32x4*>(t.t3h);
        const u32x4* F = reinterpret_cast<const u32x4*>(t.filt);  // a harmless line
        const uint32_t slot = (r.fp & RT_SLOT2) ? rt_slot2(k, t.t3h_bits) : rt_slot1(k, t.t3h_bits);
        const u32x4* W = reinterpret_cast<const u32x4*>(t.wide) + (size_t)(r.fk & 0x3FFFu) * 4 + ((r.fk >> 20) & 3u);
        const u32x4* a0 = wide ? W : deep ? reinterpret_cast<const u32x4*>(t.rec) + node : ((act && !skip) ? T + slot : F);
        const uint8_t* a1 = (deep && !wide && (int64_t)d <= i - stream_start) ? text + ((i - d) & ~(int64_t)7) : dummy;
        r.L0 = *a0;
        r.tw = *reinterpret_cast<const u32x2*>(a1);
        r.n = take;
        qh += take;
        qn -= take;
    };
    auto consume = [&](Round& r) __attribute__((always_inline)) {
        // Nothing computed from the round may be hoisted above this point
        // (the compiler otherwise speculates it up to the loads and waits).
        // (Fenced copies: the round's own registers are never redefined.)
        u32x4 L0 = r.L0;
        u32x2 tw = r.tw;
        uint32_t fk = r.fk, fp = r.fp;
        asm volatile("" : "+v"(L0), "+v"(tw), "+v"(fk), "+v"(fp)::"memory");
        bool again = false, wstep = false;
        uint32_t nk = 0, np = 0;
        if ((uint32_t)lane < r.n && !r.skip) {
            const int64_t i = pos0 + (int64_t)(fp & RT_POSMASK);
            const int64_t avail = i - stream_start + 1;
            uint32_t v, ph0 = 0xFFFFFFFFu, node = 0, d = 0;  // ph0: the stored placeholder, when known
            bool reprobe = false;
            if (!(fp >> 31)) {
                const uint32_t k = fk >> 8, c3 = fk & 0xFFu;
                ph0 = s_t[k >> 8] & 0x7FFFu;
                const uint32_t want = T3H_VALID | k;
                const u32x4 e = L0;
                v = ph0;
                if ((e.x & 0x1FFFFFFu) != want && (e.x & T3H_VALID) && !(fp & RT_SLOT2)) {
                    reprobe = true;  // slot1 holds another key: try slot2
                    again = true;
                } else if ((e.x & 0x1FFFFFFu) == want) {
                    v = e.y;
                    const uint32_t kind = e.x >> 25;
                    if (avail >= 4 && kind == 1) {
                        const uint32_t nch = e.z >> 24;
                        const uint32_t j = c3 == (e.z & 0xFFu) ? 0u : c3 == ((e.z >> 8) & 0xFFu) ? 1u
                                         : c3 == ((e.z >> 16) & 0xFFu) ? 2u : 3u;
                        if (j < nch) {
                            if (nch == 1 && !(e.w & CONT32)) {
                                v = e.w;
                            } else {
                                again = true;
                                node = nch == 1 ? e.w & 0x7FFFFFFFu : e.w + j;
                                d = 4;
                            }
                        }
                    } else if (avail >= 4 && kind == 2) {
                        again = true;
                        node = e.w & 0x7FFFFFFFu;
                        d = 3;
                    }
                }
            } else if (fp & RT_SLOT2) {
                // wide step: L0 = the quarter of the node's wide entry
                // holding byte c; fk = entry | c << 14 | depth << 22
                const uint32_t ch = wide_child(L0, (fk >> 14) & 0xFFu);
                d = (fk >> 22) + 1;
                v = L0.w;
                if (ch != ~0u) {
                    node = ch;
                    again = true;
                }
            } else {
                // record step: {kind | count | first, best, child bytes}
                d = fk >> 23;
                const u32x4 R = L0;
                v = R.y;
                if ((int64_t)d < avail) {
                    const uint32_t kind = rec_kind(R);
                    const uint32_t ro = (uint32_t)(i - d) & 7u;  // text[i-d] in the 8-byte window
                    const uint32_t tc = (((ro & 4) ? tw.y : tw.x) >> (8 * (ro & 3))) & 0xFFu;
                    if (kind == RT_REC_CHAIN_K) {
                        // the run's bytes against text[i-d], text[i-d-1], ...
                        // as far as the window, the run and the stream allow
                        const uint64_t win = ((uint64_t)tw.y << 32 | tw.x) << (8 * (7 - ro));
                        const uint64_t dif = win ^ ((uint64_t)R.w << 32 | R.z);
                        const uint32_t meq = dif ? (uint32_t)__builtin_clzll(dif) >> 3 : 8u;
                        const uint32_t clen = (R.x >> 24) & 63u;
                        const uint32_t cav = (uint32_t)(avail - d);
                        const uint32_t cm = min(meq, min(min(clen, ro + 1u), cav));
                        if (cm >= 1u && (cm == clen || (cm == ro + 1u && cm < cav))) {
                            node = (R.x & 0xFFFFFFu) + cm - 1u;
                            d += cm;
                            again = true;
                        }
                    } else if (kind == RT_REC_KIDS_K) {
                        const uint32_t j = rec_kid_index(R, tc);
                        if (j != ((R.x >> 24) & 63u)) {
                            node = (R.x & 0xFFFFFFu) + j;
                            ++d;
                            again = true;
                        }
                    } else if (kind == RT_REC_WIDE_K) {
                        wstep = true;  // next round: the quarter of its entry holding tc
                        again = true;
                        node = R.z | (tc << 14);
                    }
                }
            }
            if (reprobe) {
                nk = fk;
                np = fp | RT_SLOT2;
            } else if (wstep) {
                nk = node | (d << 22);
                np = fp | RT_SLOT2;
            } else if (again) {
                nk = node | (d << 23);
                np = (fp & ~RT_SLOT2) | 0x80000000u;
                if (!(fp >> 31)) cnt -= (uint32_t)(ph0 != 0u);  // the placeholder leaves the count
            } else {
                cnt += (uint32_t)(v != 0u) - ((fp >> 31) ? 0u : (uint32_t)(ph0 != 0u));
                if (OUTW && v != ph0) put_id<OUTW>(out, i - pos0, v);
            }
        }
        __builtin_amdgcn_wave_barrier();
        const uint64_t m = __ballot(again);
        if (again) {
            const uint32_t sl = (qh + qn + wave_prefix(m)) & (RT_QCAP - 1);
            qkey[sl] = nk;
            qpos[sl] = np;
        }
        __builtin_amdgcn_wave_barrier();
        qn += (uint32_t)__popcll(m);
        r.n = 0;
        r.keep = 0;
    };
    // Text of chunk c: each lane loads its own aligned dword per group (256
    // B per instruction, two cache lines), plus one dword before the chunk
    // that all lanes load (one line); the three look-back bytes of a lane
    // come from its neighbour by DPP (chunk()).
    auto fetch = [&](uint32_t (&xr)[4], uint32_t& xp, int64_t c) __attribute__((always_inline)) {
        const uint8_t* base = c < cend ? text + pos0 + c * RT_CHUNK : dummy;
#pragma unroll
        for (int s = 0; s < 4; ++s)
            xr[s] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(base + 256 * s + 4 * lane));
        xp = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(base - 4));
    };
    auto stand_in_store = [&]() __attribute__((always_inline)) {
        if (OUTW == 4) {
            u32x4* o = reinterpret_cast<u32x4*>(t.scratch);
#pragma unroll
            for (int s = 0; s < 4; ++s) __builtin_nontemporal_store(u32x4{0u, 0u, 0u, 0u}, o + 64 * s + lane);
        }
        if (OUTW == 2) {
            u32x2* o = reinterpret_cast<u32x2*>(t.scratch);
#pragma unroll
            for (int s = 0; s < 4; ++s) __builtin_nontemporal_store(u32x2{0u, 0u}, o + 64 * s + lane);
        }
    };
    Round rr;
    rr.n = 0;
    rr.keep = 0;
    uint32_t xa[4], xb[4], pa, pb;
    int64_t ch = cbeg;
    // Drain the queue and resolve the spill region (the tail): after the
    // chunk loop, and inside it when the region could not take a chunk's
    // overflow -- the region is bounded (t.spill_stride items per wave,
    // pm_rt_spill_items), so deep input resolves it in several segments
    // while the loop's prefetched chunks stay in flight.  The test sits in
    // the push's ring-full branch, which random text never enters.
    const uint32_t scap = (uint32_t)t.spill_stride;
    auto resolve = [&]() __attribute__((always_inline)) {
        if (!kFilter) return;
        if (rr.n) consume(rr);
        while (qn) {  // wave-uniform; every round advances each item
            Round rs;
            issue(rs, qn);
            consume(rs);
        }
        // the auto kind's measure of deep matches: items the ring could not
        // hold; count-only queues nothing (every candidate goes to the
        // region), so there it is the positions the tail had to walk
        if (kRounds && t.spill_total && sn && lane == 0) atomicAdd(t.spill_total, (unsigned long long)sn);
        // every placeholder and spill store of this wave complete before
        // its walks patch or read them
        __builtin_amdgcn_s_waitcnt(0);
        {
            const uint32_t nwalk = rt_tail<OUTW>(text, stream_start, pos0, out, t, s_f2, sp, sn, lane, cnt);
            if (!kRounds && t.spill_total && nwalk && lane == 0)
                atomicAdd(t.spill_total, (unsigned long long)nwalk);
        }
        // the tail's stores and its reads of the region complete before the
        // region is refilled
        __builtin_amdgcn_s_waitcnt(0);
        sn = 0;
    };
    // One chunk: depth<=2 answers from LDS, filter, the previous chunk's
    // round consumed and a new one issued, the store, the push of this
    // chunk's candidates, the prefetch two chunks ahead.
    auto chunk = [&](uint32_t (&xr)[4], uint32_t& xp, int64_t c) __attribute__((always_inline)) {
        const int64_t pc = pos0 + c * RT_CHUNK;
        // 8-byte windows {previous dword, own dword}: wave_shr:1 hands each
        // lane its left neighbour's dword; lane 0 keeps `old`: the previous
        // group's lane-63 dword (wave_ror:1 of that group), or for group 0
        // the dword before the chunk
        u32x2 x[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const uint32_t fix = s == 0 ? xp : __builtin_amdgcn_update_dpp(0u, xr[s - 1], 0x13C, 0xf, 0xf, false);
            x[s].x = __builtin_amdgcn_update_dpp(fix, xr[s], 0x138, 0xf, 0xf, false);  // wave_shr:1
            x[s].y = xr[s];
        }
        if (EF) fetch(xr, xp, c + 2 * cstep);
        // position j = 4s + b of this lane is pc + 256s + 4*lane + b; its key
        // is the LE u24 ending at byte b of x[s].y (bytes i-2, i-1, i)
#define RT_RAW(j) ((uint32_t)((((uint64_t)x[(j) >> 2].y << 32) | x[(j) >> 2].x) >> (8 * (2 + ((j) & 3)))))
#define RT_KEY(j) (RT_RAW(j) & 0xFFFFFFu)
        uint32_t res[16];
        // bit j << CMS: position j goes past depth 2 (count only keeps two
        // bits per position, the candidate bit is the odd one)
        constexpr int CMS = kT8 ? 1 : 0;
        uint32_t cm = 0;
        if (kT8) {
            // count only: the 16 classes {nz, cand} of the lane's positions
            // side by side in one word, two bits each -- the key (text[i] <<
            // 8 | text[i-1], the byte address of the class) by one v_perm, the
            // class shifted into place by one v_lshl_or: two VALU per
            // position.  Nonzero answers (even bits) are counted per lane;
            // zero answers under a node with children (odd bits) are queued.
            // Against the class sum (5 VALU per position), side by side:
            // random ASCII 0.455 -> 0.432 ms, shipped 0.637 -> 0.600, lines
            // 0.879 -> 0.862 (profiles/r03/count_perm_staging_ab.txt).
            uint32_t f = 0;
            constexpr uint32_t kSel0 = 0x0C0C0000u;  // bytes 2, 3 = 0; byte 1 = text[i], byte 0 = text[i-1]
#define RT_T8KEY(j) \
    __builtin_amdgcn_perm(x[(j) >> 2].y, x[(j) >> 2].x, kSel0 | (4u + ((j) & 3)) << 8 | (3u + ((j) & 3)))
            // (measured and removed, round 4: a conflict-free 256-bit table
            // of the bytes that are 1-byte patterns read first, the class
            // table only for the other lanes -- by exec mask or with those
            // lanes on one broadcast address: exact, but 0.433 -> 0.647 /
            // 0.668 ms on ASCII, the 16 extra LDS reads per chunk cost more
            // than the conflicts they remove; profiles/r04/count_ablations.
            // Also measured and removed: a u16 class table whose zero
            // answers carry a filter of their depth-3 children's bytes (low
            // 3 bits of text[i-2]), candidates 2.1% -> 0.5% of random-ASCII
            // positions -- exact, but 0.444 -> 0.473 ms on ASCII, 0.600 ->
            // 0.659 shipped, 0.841 -> 0.834 lines: the classification, not
            // the candidates, is what count only waits for; count4_*.json)
#pragma unroll
            for (int j = 0; j < 16; ++j) f |= (uint32_t)s_t8[RT_T8KEY(j)] << (2 * j);
#undef RT_T8KEY
            cnt += (uint32_t)__popc(f & 0x55555555u);
            cm = f & 0xAAAAAAAAu;
        } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) res[j] = V == 2 ? RT_KEY(j) & 0xFFFFu : s_t[RT_KEY(j) >> 8];
        if (kFilter && kStage1) {
            uint32_t fw[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) fw[j] = s_f[rt_fhash(RT_RAW(j)) >> 20];  // the multiply reads 24 bits
#pragma unroll
            for (int j = 0; j < 16; ++j) cm |= ((res[j] >> 15) & rt_fhit(fw[j], rt_fhash(RT_RAW(j)))) << j;
        } else if (kFilter) {
#pragma unroll
            for (int j = 0; j < 16; ++j) cm |= (res[j] >> 15) << j;
        }
        if (kFilter) {
            // count-only: a nonzero depth-2 answer stays nonzero however deep
            // the walk goes (the answer is the deepest pattern on it), so only
            // positions whose placeholder is 0 can change the count
            if (OUTW == 0) {
                uint32_t zm = 0;
#pragma unroll
                for (int j = 0; j < 16; ++j) zm |= (uint32_t)((res[j] & 0x7FFFu) == 0u) << j;
                cm &= zm;
            }
        }
        // nonzero placeholders, counted on the scalar unit: one compare per
        // position into a lane mask, then s_bcnt1 (a per-lane sum, as count
        // only does, measured equal here: ids, 1.12-1.17 ms either way)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            res[j] &= 0x7FFFu;
            scnt += (uint32_t)__popcll(__ballot(res[j] != 0u));
        }
        }  // !kT8
#undef RT_KEY
#undef RT_RAW
        if (kFilter && kRounds) {
            if (rr.n) consume(rr);                // the round issued last chunk
            issue(rr, qn >= RT_ROUND ? qn : 0u);  // items of earlier chunks (stores issued)
        }
        // store the chunk: depth<=2 answers, queued positions patched later
        if (OUTW == 4) {
            u32x4* o = reinterpret_cast<u32x4*>(reinterpret_cast<uint32_t*>(out) + (pc - pos0));
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                u32x4 v = {res[4 * s], res[4 * s + 1], res[4 * s + 2], res[4 * s + 3]};
                RT_OUT_STORE(v, o + 64 * s + lane);
            }
        }
        if (OUTW == 2) {  // 512 contiguous bytes per store instruction
            u32x2* o = reinterpret_cast<u32x2*>(reinterpret_cast<uint16_t*>(out) + (pc - pos0));
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                u32x2 v = {res[4 * s] | (res[4 * s + 1] << 16), res[4 * s + 2] | (res[4 * s + 3] << 16)};
                RT_OUT_STORE(v, o + 64 * s + lane);
            }
        }
        asm volatile("" ::: "memory");  // the store stays ahead of any later probe
        if (kPushS2) {
            // stage 2 now, over the lane's own candidates: only its passers
            // are queued (a rejected one keeps its depth-2 placeholder)
            uint32_t mm = cm, keep = 0;
            while (mm) {
                const uint32_t bit = __builtin_ctz(mm), j = bit >> CMS;
                mm &= mm - 1;
                const uint32_t sg = j >> 2, b = j & 3;
                const u32x2 w01 = (sg & 1) ? x[1] : x[0], w23 = (sg & 1) ? x[3] : x[2];
                const u32x2 w = (sg & 2) ? w23 : w01;
                const uint32_t q32 = (uint32_t)((((uint64_t)w.y << 32) | w.x) >> (8 * (1 + b)));
                keep |= (rt_stage2_hit(rt_stage2_load(s_f2, q32)) != 0u) << bit;
            }
            cm = keep;
        }
        if (kFilter) {
            // lane count c = popc(cm); exclusive wave prefix by a DPP scan;
            // items written by a loop over the lane's own set bits
            const uint32_t c = __popc(cm);
            const uint32_t incl = wave_scan_incl(c);
            const uint32_t base = incl - c;
            const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
            uint32_t mm = cm;
            const uint32_t pbase = (uint32_t)(pc - pos0) + 4 * lane;
            if (kRounds && total <= RT_QCAP - qn - rr.keep) {
                // the whole chunk fits the ring (the in-flight round's
                // possible survivors keep their room); the window's bytes
                // i-3..i by one 64-bit shift
                uint32_t slot = qh + qn + base;
                while (mm) {
                    const uint32_t j = __builtin_ctz(mm) >> CMS;
                    mm &= mm - 1;
                    const uint32_t sg = j >> 2, b = j & 3;
                    const u32x2 w01 = (sg & 1) ? x[1] : x[0], w23 = (sg & 1) ? x[3] : x[2];
                    const u32x2 w = (sg & 2) ? w23 : w01;
                    const uint32_t sl = slot & (RT_QCAP - 1);
                    qkey[sl] = (uint32_t)((((uint64_t)w.y << 32) | w.x) >> (8 * (1 + b)));
                    qpos[sl] = pbase + 256 * sg + b;
                    ++slot;
                }
                qn += total;
            } else {
                // ring full (dense matches): the first `room` candidates
                // (in rank order) fill the ring, the rest go to the spill
                // region, walked after the chunk loop, with whether their
                // placeholder (t12 of the key) is nonzero
                uint32_t room = kRounds ? RT_QCAP - qn - rr.keep : 0u;
                // the region could overflow: resolve it first (the test
                // sits here, off the random-text path; in the chunk loop
                // itself it measured ~1.5% slower on ids, and an outer
                // loop of segments spilled 50 VGPRs in the u16 kernel)
                if (__builtin_expect(sn + (total - room) > scap, 0)) {
                    resolve();
                    room = kRounds ? min(RT_QCAP, total) : 0u;
                }
                uint32_t rank = base;
                while (mm) {
                    const uint32_t j = __builtin_ctz(mm) >> CMS;
                    mm &= mm - 1;
                    const uint32_t sg = j >> 2, b = j & 3;
                    const u32x2 w01 = (sg & 1) ? x[1] : x[0], w23 = (sg & 1) ? x[3] : x[2];
                    const u32x2 w = (sg & 2) ? w23 : w01;
                    const uint32_t q32 = (uint32_t)((((uint64_t)w.y << 32) | w.x) >> (8 * (1 + b)));
                    const uint32_t p = pbase + 256 * sg + b;
                    if (rank < room) {
                        const uint32_t sl = (qh + qn + rank) & (RT_QCAP - 1);
                        qkey[sl] = q32;
                        qpos[sl] = p;
                    } else {
                        // (count-only queues zero placeholders only)
                        const uint32_t ph = OUTW == 0 ? 0u : (uint32_t)((s_t[q32 >> 16] & 0x7FFFu) != 0u);
                        reinterpret_cast<u32x2*>(sp)[sn + rank - room] = u32x2{q32, p | (ph << 31)};
                    }
                    ++rank;
                }
                // (readfirstlane: keeps the counts scalar across the branch)
                sn = __builtin_amdgcn_readfirstlane(sn + total - room);
                qn = __builtin_amdgcn_readfirstlane(qn + room);
            }
        }
        if (!EF) fetch(xr, xp, c + 2 * cstep);
    };
    // Enter the loop with the memory-op pattern of the steady state (round,
    // store, prefetch; round, store, prefetch -- or with EF prefetch, round,
    // store) so the compiler's vmcnt is the steady-state one.
    Round r0;
    if (EF) fetch(xa, pa, ch);
    if (kFilter && kRounds) issue(r0, 0);
    stand_in_store();
    if (!EF) fetch(xa, pa, ch);
    if (EF) fetch(xb, pb, ch + cstep);
    if (kFilter && kRounds) issue(rr, 0);
    stand_in_store();
    if (!EF) fetch(xb, pb, ch + cstep);
    for (;;) {  // wave-uniform
        if (ch >= cend) break;
        chunk(xa, pa, ch);
        if (ch + cstep >= cend) break;
        chunk(xb, pb, ch + cstep);
        ch += 2 * cstep;
    }
    resolve();
    // the (at most two) chunks that touch the stream start or the tail: one
    // position per thread of the last workgroup (a chunk is 1024 positions),
    // so each costs one walk's latency, not sixteen
    if (blockIdx.x == gridDim.x - 1) {
#pragma unroll 1
        for (int e = 0; e < 2; ++e) {  // uniform
            int64_t c = -1;
            if (e == 0 && c_lo == 1) c = 0;
            if (e == 1 && c_hi < nchunks && !(c_lo == 1 && c_hi == 0)) c = c_hi;
            const int64_t p = pos0 + c * RT_CHUNK + threadIdx.x;
            if (c >= 0 && p < pos0 + n) {
                const uint32_t v = rt_one(text, s_t, t, p, stream_start);
                if (OUTW) put_id<OUTW>(out, p - pos0, v);
                cnt += v != 0u;
            }
        }
    }
    if (count) {
        for (int o = 32; o > 0; o >>= 1) cnt += __shfl_down(cnt, o);
        cnt += scnt;
        if (lane == 0 && cnt) atomicAdd(count, (unsigned long long)cnt);
    }
}

// Small launches (the reference's 100 KiB read_block chunks, measure.c:77):
// one thread per position, rt_one over the global tables -- no LDS tables to
// stage, no chunk loop, no queue; a launch costs about one walk's chain of
// dependent loads.  CONT positions (depth-2 node with children) count
// towards spill_total, the auto kind's deep-input signal.
// The deep-input signal of the auto kind (RtDev::spill_total) counts, like
// the chunked kernel's spilled items, the positions that pass both LDS
// filter stages -- the ones with a depth-3 probe to make -- not every
// position under a depth-2 node with children (the unfiltered
// count sent small launches to the DFA trials more often).
// (Measured and removed, round 4: staging each workgroup's text window in
// LDS first -- no faster at read_block's 100 KiB zero-copy calls, 40.6
// against 39.3 us per call, profiles/r04/host_path/small_call_variants_ab.json.)
constexpr int RT_SMALL_THREADS = 256;
template <int OUTW>
__global__ __launch_bounds__(RT_SMALL_THREADS) void rt_small_kernel(const uint8_t* __restrict__ text,
                                                                    int64_t stream_start, int64_t pos0, int64_t n,
                                                                    void* __restrict__ out,
                                                                    unsigned long long* __restrict__ count, RtDev t) {
    const int64_t k = (int64_t)blockIdx.x * RT_SMALL_THREADS + threadIdx.x;
    uint32_t v = 0, deep = 0;
    if (k < n) {
        const int64_t i = pos0 + k;
        v = rt_one(text, t.t12, t, i, stream_start);
        if (t.spill_total && i - stream_start >= 3 && (t.t12[(uint32_t)text[i] << 8 | text[i - 1]] & CONT16)) {
            const uint32_t q = (uint32_t)text[i - 3] | (uint32_t)text[i - 2] << 8 | (uint32_t)text[i - 1] << 16 |
                               (uint32_t)text[i] << 24;
            const uint32_t f = rt_fhash(q >> 8);
            if (rt_fhit(t.filt[f >> 20], f)) deep = rt_stage2_hit(rt_stage2_load(t.filt + RT_FILTER_WORDS, q));
        }
        if (OUTW) put_id<OUTW>(out, k, v);
    }
    const uint64_t nz = __ballot(v != 0u), dp = __ballot(deep != 0u);
    if ((threadIdx.x & 63) == 0) {
        if (count && nz) atomicAdd(count, (unsigned long long)__popcll(nz));
        if (t.spill_total && dp) atomicAdd(t.spill_total, (unsigned long long)__popcll(dp));
    }
}

// The resident small-call server (pm_kernels.h PmServeReq): the grid stays
// on the device between read_block calls, so a 100 KiB call (measure.c:77,
// 284) costs the link's round trips instead of a launch and a stream
// synchronization (~20 us of the ~35, profiles/r05/small_call/).
// Workgroup 0's first wave polls the request line (lanes 0-7 read its
// eight words: one 64-B read over the link; the host writes seq, the fields,
// then seq2, and a line is read whole, so seq2 == seq > seen is a complete
// new request) and forwards it to a 64-B line in device memory the other
// workgroups poll the same way.  A workgroup's share of the positions is 64-aligned; its
// text window -- the share plus the walk's look-back, RtDev::back + 1 bytes,
// 8-B aligned -- is copied from the pinned staging into LDS, and each lane
// walks its positions with rt_one from there.  The results go straight into
// the pinned result buffer; once every lane's stores have completed
// (s_waitcnt) and the barrier, the first lane writes seq's low 32 bits into
// done[wg].
// Coherence without fences: every access to host memory is an access at
// its coherence point (system-scope relaxed atomics: the sc0 sc1 bits), so
// nothing needs a cache invalidated or written back -- acquire / release
// fences here invalidate or write back the whole L2 per wave, taking the
// walk's tables out of L2 (measured: 74 us a 100 KiB call with them, against
// 31 us for a launch per call).
// Every exit is reached: a stop naming this grid's generation, or idle_ticks
// (100 MHz) with no request.  Idle waves sleep between polls (s_sleep).
constexpr int RT_SERVE_WIN = 16384;  // LDS bytes of a workgroup's text window
constexpr int RT_SERVE_POLLERS = 4;  // waves of workgroup 0 polling the host's line
#ifndef PM_SERVE_TRACE
#define PM_SERVE_TRACE 0  // ablation build: s_memrealtime stamps of workgroups 0 and 1 per request
#endif
// a 64-bit value the compiler then knows is wave-uniform (every branch on
// it scalar: the loop below has barriers, and a branch the compiler thinks
// divergent around them is structurized into a loop the waves never leave)
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {
    // (the builtin returns int: through uint32_t, or the low half sign-extends)
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
    return (uint64_t)hi << 32 | lo;
}
__device__ __forceinline__ uint64_t lane64(uint64_t x, int l) {  // lane l's x, wave-uniform
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)x, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(x >> 32), l);
    return (uint64_t)hi << 32 | lo;
}
template <class T>
__device__ __forceinline__ T sys_load(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <class T>
__device__ __forceinline__ void sys_store(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <class T>
__device__ __forceinline__ T dev_load(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void dev_store(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ __launch_bounds__(RT_SERVE_THREADS) void rt_serve_kernel(PmServeReq* req, uint64_t* fwd, uint32_t* done,
                                                                    uint64_t seen, uint64_t gen, int64_t idle_ticks,
                                                                    RtDev t) {
    __shared__ __attribute__((aligned(16))) uint8_t win[RT_SERVE_WIN];
    __shared__ uint64_t s_w[8];  // the request line
    __shared__ uint32_t s_state;  // this request: 0 polling, 1 found, 2 exit
    const uint64_t* const rq = reinterpret_cast<const uint64_t*>(req);
    const int tid = threadIdx.x;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t G = gridDim.x, wg = blockIdx.x;
    if (tid == 0) s_state = 0;
    __syncthreads();
    for (;;) {
        if (wg == 0 ? wid < RT_SERVE_POLLERS : wid == 0) {
            // Workgroup 0 polls the host's line with RT_SERVE_POLLERS waves
            // a quarter of a link round trip apart (a request is seen ~3/4 of
            // a round trip sooner than by one poller); the other workgroups
            // poll workgroup 0's copy of it in device memory with one wave.
            // One workgroup on the link: many pollers of one host line slow
            // the host's own reads of the results (128 of them 5x).
            for (int q = 0; q < wid; ++q) __builtin_amdgcn_s_sleep(24);  // (~0.6 us each)
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            uint64_t w = 0;
            uint32_t found = 0, quit = 0;
            const uint64_t* const src = wg == 0 ? rq : fwd;
            for (;;) {
                w = wg == 0 ? sys_load(src + (tid & 7)) : dev_load(src + (tid & 7));  // lanes 0-7: the line's words
                const uint64_t s2 = lane64(w, 7);
                if (s2 > seen && s2 == lane64(w, 0)) {
                    found = 1;
                    break;
                }
                if (lane64(w, 1) == gen || __builtin_amdgcn_s_memrealtime() - t0 > (uint64_t)idle_ticks) {
                    quit = 1;
                    break;
                }
                if (wg == 0 && __builtin_amdgcn_readfirstlane(
                                   __hip_atomic_load(&s_state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)))
                    break;  // another poller has decided
                __builtin_amdgcn_s_sleep(1);
            }
#if PM_SERVE_TRACE
            if ((tid & 63) == 0 && wg < 2 && found)
                sys_store(reinterpret_cast<uint64_t*>(done + G + 16) + 8 * wg, __builtin_amdgcn_s_memrealtime());
#endif
            if (found) {
                const int lane = tid & 63;
                uint32_t old = 1;
                if (lane == 0) old = __hip_atomic_exchange(&s_state, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (__builtin_amdgcn_readfirstlane(old) != 1) {  // the first poller to find it (the others skip)
                    if (lane < 8 && lane != 1) s_w[lane] = w;
                    if (wg == 0) {  // forward: the fields, then seq and seq2
                        if (lane >= 2 && lane < 7) dev_store(fwd + lane, w);
                        __builtin_amdgcn_s_waitcnt(0);
                        if (lane == 0 || lane == 7) dev_store(fwd + lane, w);
                    }
                }
            } else if (quit && (tid & 63) == 0) {
                uint32_t zero = 0;
                __hip_atomic_compare_exchange_strong(&s_state, &zero, 2u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        __syncthreads();
        if (__builtin_amdgcn_readfirstlane(s_state) == 2) {  // (uniform)
            if (wg == 0 && tid == 1) dev_store(fwd + 1, gen);  // the others exit too
            return;
        }
        __syncthreads();  // every thread has read s_state
        if (tid == 0) s_state = 0;  // (the next poll starts after the barriers below)
        const uint64_t v = rfl64(s_w[0]);
        seen = v;
        const uint8_t* const text = reinterpret_cast<const uint8_t*>(rfl64(s_w[2]));
        void* const out = reinterpret_cast<void*>(rfl64(s_w[3]));
        const int64_t ss = (int64_t)rfl64(s_w[4]), pos0 = (int64_t)rfl64(s_w[5]);
        const uint64_t nw = rfl64(s_w[6]);
        const int64_t n = (int64_t)(nw & ((1ull << 56) - 1));
        const bool w4 = (nw >> 56) == 4;
        const int64_t per = ((n + G - 1) / G + 63) & ~(int64_t)63;
        const int64_t a = wg * per < n ? wg * per : n, b = a + per < n ? a + per : n;
        if (a < b) {  // (uniform)
            const int64_t back = (int64_t)t.back + 4;  // rt_one reads text[i-3] and one byte past a leaf
            const int64_t lo = (pos0 + a - back > ss ? pos0 + a - back : ss) & ~(int64_t)7;
            const int64_t hi = (pos0 + b + 7) & ~(int64_t)7;  // the staging has 16 zero bytes after the block
            if (hi - lo <= RT_SERVE_WIN) {
                for (int64_t k = 8 * tid; k < hi - lo; k += 8 * RT_SERVE_THREADS)
                    *reinterpret_cast<uint64_t*>(win + k) = sys_load(reinterpret_cast<const uint64_t*>(text + lo + k));
                __syncthreads();
#if PM_SERVE_TRACE
                if (tid == 0 && wg < 2)
                    sys_store(reinterpret_cast<uint64_t*>(done + G + 16) + 8 * wg + 1, __builtin_amdgcn_s_memrealtime());
#endif
                for (int64_t k = a + tid; k < b; k += RT_SERVE_THREADS) {
                    const uint32_t r = rt_one(win, t.t12, t, pos0 + k - lo, ss - lo);
                    if (w4) reinterpret_cast<uint32_t*>(out)[k] = r;
                    else reinterpret_cast<uint16_t*>(out)[k] = (uint16_t)r;
                }
            } else {  // a look-back longer than the window: straight from the pinned staging
                for (int64_t k = a + tid; k < b; k += RT_SERVE_THREADS) {
                    const uint32_t r = rt_one(text, t.t12, t, pos0 + k, ss);
                    if (w4) reinterpret_cast<uint32_t*>(out)[k] = r;
                    else reinterpret_cast<uint16_t*>(out)[k] = (uint16_t)r;
                }
            }
        }
        // The results are ordinary stores: L2 merges them into whole lines,
        // which go over the link at the writeback (stores at the coherence
        // point go as partial lines, and the host then reads them at a
        // fraction of the rate).  Every wave's stores reach L2, then one
        // release per workgroup writes L2 back before the flag.
#if PM_SERVE_TRACE
        if (tid == 0 && wg < 2)
            sys_store(reinterpret_cast<uint64_t*>(done + G + 16) + 8 * wg + 2, __builtin_amdgcn_s_memrealtime());
#endif
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
#if PM_SERVE_TRACE
        if (tid == 0 && wg < 2)
            sys_store(reinterpret_cast<uint64_t*>(done + G + 16) + 8 * wg + 3, __builtin_amdgcn_s_memrealtime());
#endif
        if (tid == 0) __hip_atomic_store(done + wg, (uint32_t)v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
#if PM_SERVE_TRACE
        if (tid == 0 && wg < 2)
            sys_store(reinterpret_cast<uint64_t*>(done + G + 16) + 8 * wg + 4, __builtin_amdgcn_s_memrealtime());
#endif
    }
}

constexpr int DFA_THREADS = 256;

template <int OUTW>
__global__ __launch_bounds__(DFA_THREADS) void dfa_scan_kernel(const uint8_t* __restrict__ text, int64_t stream_start,
                                                               int64_t pos0, int64_t n, void* __restrict__ out,
                                                               unsigned long long* __restrict__ count, DfaDev t,
                                                               int64_t seg_len) {
    const int64_t nseg = (n + seg_len - 1) / seg_len;
    uint32_t cnt = 0;
    const int64_t stride = (int64_t)gridDim.x * DFA_THREADS;
    for (int64_t sg = (int64_t)blockIdx.x * DFA_THREADS + threadIdx.x; sg < nseg; sg += stride) {
        const int64_t lo = pos0 + sg * seg_len;
        const int64_t hi = (lo + seg_len < pos0 + n) ? lo + seg_len : pos0 + n;
        int64_t wlo = lo - t.warm;
        if (wlo < stream_start) wlo = stream_start;
        uint32_t s = 0;
        for (int64_t i = wlo; i < lo; ++i) s = t.next[(size_t)s * 256 + text[i]];
        int64_t i = lo;
        for (; i + 16 <= hi; i += 16) {
            const uint4 w = *reinterpret_cast<const uint4*>(text + i);
            const uint32_t W[4] = {w.x, w.y, w.z, w.w};
            uint32_t r[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                s = t.next[(size_t)s * 256 + ((W[j >> 2] >> (8 * (j & 3))) & 0xFFu)];
                r[j] = t.out[s];
            }
            if (OUTW == 4) {
                uint4* o = reinterpret_cast<uint4*>(reinterpret_cast<uint32_t*>(out) + (i - pos0));
                o[0] = make_uint4(r[0], r[1], r[2], r[3]);
                o[1] = make_uint4(r[4], r[5], r[6], r[7]);
                o[2] = make_uint4(r[8], r[9], r[10], r[11]);
                o[3] = make_uint4(r[12], r[13], r[14], r[15]);
            }
            if (OUTW == 2) {
                uint4* o = reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(out) + (i - pos0));
                o[0] = make_uint4(r[0] | r[1] << 16, r[2] | r[3] << 16, r[4] | r[5] << 16, r[6] | r[7] << 16);
                o[1] = make_uint4(r[8] | r[9] << 16, r[10] | r[11] << 16, r[12] | r[13] << 16, r[14] | r[15] << 16);
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) cnt += r[j] != 0u;
        }
        for (; i < hi; ++i) {
            s = t.next[(size_t)s * 256 + text[i]];
            const uint32_t v = t.out[s];
            if (OUTW) put_id<OUTW>(out, i - pos0, v);
            cnt += v != 0u;
        }
    }
    if (count) {
        for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off);
        if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(count, (unsigned long long)cnt);
    }
}

// Output-coded DFA (the image of a dictionary of < 2^20 states, pm_flatten.h):
// the transition word carries its target's output as a 12-bit code next to
// the 20-bit target state (4095 = look it up in out[]), so a step is one
// gather; CH segments per lane advance in lock step (CH gathers in flight
// per lane).  Escapes are looked up after each 16-step block, off the chain.
constexpr uint32_t DFA_STATE_MASK = 0xFFFFFu;  // must match pm_flatten.h
constexpr uint32_t DFA_ESC = 4095u;
constexpr uint32_t PM_FL_INREC = 4095u;  // must match pm_flatten.h PM_FL_FB_INREC
constexpr int FL_LDS_ROWS = 88;          // must match pm_flatten.h PM_FL_LDS_ROWS
// The count-only FL kernel has no staging rows: 156 rows fill the LDS (the
// root and the rows pm_pack_sparse_fl's profile visits most; must match
// pm_flatten.h PM_FL_COUNT_LDS_ROWS).
constexpr int FL_COUNT_LDS_ROWS = 156;

// The start of the last synchronizing 3-gram in [wlo, lo - 3], or wlo when
// there is none (DfaDev::gram3: no pattern holds it, so the state after it is
// the root's over its 3 bytes and a warm-up may start there instead of
// max_len - 1 bytes back); 16 candidates per round.
// Every load of a round is issued before any is used (the 18 bytes, then
// the 16 set words): two load latencies per round.  (With a branch per
// candidate the compiler had waited for each byte in turn: 48 latencies.)
__device__ __forceinline__ int64_t dfa_sync_lo(const uint8_t* __restrict__ text, int64_t lo, int64_t wlo,
                                               const uint32_t* __restrict__ gram3) {
    for (int64_t qh = lo - 3; qh >= wlo; qh -= 16) {
        uint32_t b[18];  // bytes qh - 15 .. qh + 2 (any before wlo read as text[wlo], then masked)
#pragma unroll
        for (int u = 0; u < 18; ++u) {
            const int64_t q = qh - 15 + u;
            b[u] = text[q < wlo ? wlo : q];
        }
        uint32_t g[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {  // the 3-gram at qh - u
            const uint32_t x = b[15 - u] | b[16 - u] << 8 | b[17 - u] << 16;
            g[u] = gram3[x >> 5] >> (x & 31);
        }
        uint32_t absent = 0;  // bit u: the 3-gram at qh - u is in no pattern
#pragma unroll
        for (int u = 0; u < 16; ++u) absent |= (uint32_t)(qh - u >= wlo && !(g[u] & 1u)) << u;
        if (absent) return qh - __builtin_ctz(absent);
    }
    return wlo;
}

template <int OUTW, int CH, int BLK = 16>
__global__ __launch_bounds__(DFA_THREADS) void dfa_coded_kernel(const uint8_t* __restrict__ text, int64_t stream_start,
                                                                int64_t pos0, int64_t n, void* __restrict__ out,
                                                                unsigned long long* __restrict__ count,
                                                                const uint32_t* __restrict__ nxt,
                                                                const uint32_t* __restrict__ outt, int64_t warm,
                                                                int64_t seg_len, const uint32_t* __restrict__ gram3) {
    const int64_t nseg = (n + seg_len - 1) / seg_len;
    const int64_t lanes = (int64_t)gridDim.x * DFA_THREADS;
    uint32_t cnt = 0;
    for (int64_t sg0 = (int64_t)blockIdx.x * DFA_THREADS + threadIdx.x; sg0 < nseg; sg0 += CH * lanes) {
        int64_t lo[CH], hi[CH];
        uint32_t s[CH];
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int64_t sg = sg0 + k * lanes;
            lo[k] = sg < nseg ? pos0 + sg * seg_len : pos0 + n;
            hi[k] = sg < nseg ? (lo[k] + seg_len < pos0 + n ? lo[k] + seg_len : pos0 + n) : pos0 + n;
            int64_t wlo = lo[k] - warm;
            if (wlo < stream_start) wlo = stream_start;
            if (gram3 && sg < nseg) wlo = dfa_sync_lo(text, lo[k], wlo, gram3);
            s[k] = 0;
            if (sg < nseg)
                for (int64_t i = wlo; i < lo[k]; ++i) s[k] = nxt[(size_t)s[k] * 256 + text[i]] & DFA_STATE_MASK;
        }
        const int64_t nblk = seg_len / BLK;
        for (int64_t b = 0; b < nblk; ++b) {
            bool act[CH];
            uint32_t W[CH][BLK / 4];
            bool any = false;
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                act[k] = lo[k] + BLK * b + BLK <= hi[k];
                any |= act[k];
#pragma unroll
                for (int q = 0; q < BLK / 16; ++q) {
                    const uint4 w = act[k] ? *reinterpret_cast<const uint4*>(text + lo[k] + BLK * b + 16 * q)
                                           : make_uint4(0, 0, 0, 0);
                    W[k][4 * q] = w.x; W[k][4 * q + 1] = w.y; W[k][4 * q + 2] = w.z; W[k][4 * q + 3] = w.w;
                }
            }
            if (!any) break;
            uint32_t code[CH][BLK], st[CH][BLK];
#pragma unroll
            for (int j = 0; j < BLK; ++j) {
#pragma unroll
                for (int k = 0; k < CH; ++k) {
                    const uint32_t c = (W[k][j >> 2] >> (8 * (j & 3))) & 0xFFu;
                    const uint32_t v = act[k] ? nxt[(size_t)s[k] * 256 + c] : 0u;
                    s[k] = act[k] ? v & DFA_STATE_MASK : s[k];
                    code[k][j] = v >> 20;
                    st[k][j] = s[k];
                }
            }
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                if (!act[k]) continue;
                uint32_t r[BLK];
#pragma unroll
                for (int j = 0; j < BLK; ++j)  // count only: an escape code is a nonzero id, no lookup
                    r[j] = OUTW && code[k][j] == DFA_ESC ? outt[st[k][j]] : code[k][j];
                const int64_t i = lo[k] + BLK * b;
                if (OUTW == 4) {
                    uint4* o = reinterpret_cast<uint4*>(reinterpret_cast<uint32_t*>(out) + (i - pos0));
#pragma unroll
                    for (int q = 0; q < BLK / 4; ++q) o[q] = make_uint4(r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]);
                }
                if (OUTW == 2) {
                    uint4* o = reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(out) + (i - pos0));
#pragma unroll
                    for (int q = 0; q < BLK / 8; ++q)
                        o[q] = make_uint4(r[8 * q] | r[8 * q + 1] << 16, r[8 * q + 2] | r[8 * q + 3] << 16,
                                          r[8 * q + 4] | r[8 * q + 5] << 16, r[8 * q + 6] | r[8 * q + 7] << 16);
                }
#pragma unroll
                for (int j = 0; j < BLK; ++j) cnt += r[j] != 0u;
            }
        }
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            for (int64_t i = lo[k] + BLK * ((hi[k] - lo[k]) / BLK); i < hi[k]; ++i) {
                s[k] = nxt[(size_t)s[k] * 256 + text[i]] & DFA_STATE_MASK;
                const uint32_t v = outt[s[k]];
                if (OUTW) put_id<OUTW>(out, i - pos0, v);
                cnt += v != 0u;
            }
        }
    }
    if (count) {
        for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off);
        if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(count, (unsigned long long)cnt);
    }
}

// The sparse (default-transition) form, pm_flatten.h: rows only for the
// states whose row differs from their fallback's in more than PM_SDFA_K
// bytes, 16-B records for the rest (8-B units in pm_pack_sparse8's
// repacking).  A step reads a row's word, or the state's record and, at a
// record whose slots miss the byte, the fallback row's word.  On deep
// inputs the states a stream visits are mostly records: their table is tens
// of MB instead of the dense rows' hundreds, so the loads stay in L2 / the
// Infinity Cache instead of going to HBM.  (The round-2 kernel that loaded
// each step's 16-B record or row quad, dfa_sparse_kernel, and its variants
// are in git history before round 5.)

// The sparse form with the transition tiles placed by the memory hierarchy
// (one segment per lane; DFA_LDS_THREADS lanes per workgroup, one
// workgroup per CU):
//  * rows: the first KR rows of the block -- the root and the shallowest
//    states, in the trie's breadth-first order -- are staged once per
//    workgroup into LDS (KR KiB); a row step or a record's fallback to one
//    of them is one ds_read_b32 instead of a scattered global load;
//  * records: a lane loads the aligned block of 4 records (64 B, one
//    quarter of a 128-B line) holding its state and keeps it in registers;
//    records are numbered depth-first, so a walk along a pattern's states
//    steps through the block without another load (on the lines stream
//    0.61 instead of 1.08 dependent global loads per byte, simulated).
// Every other step is the plain form's: a 4-B load of a row word, or at a
// record whose two slots miss the byte the fallback row's word.
constexpr int DFA_LDS_THREADS = 512;
__device__ __forceinline__ uint4 pick4(const uint4 (&R)[4], uint32_t k) {
    const uint4 a = (k & 1u) ? R[1] : R[0], b = (k & 1u) ? R[3] : R[2];
    return (k & 2u) ? b : a;
}

// RB: record bytes.  16: the 16-B form, 4 records per 64-B block.  8: the
// 8-B unit form (pm_pack_sparse8), 8 units per block: a one-slot record is
// one unit {y, x0 | w << 9}, a two-slot record two {y, x | 1 << 31}, {z, w}
// in the same block.
// BU (RB = 8): units per register block -- 8 (64 B, four 16-B loads) or 4
// (32 B, two loads; pm_pack_sparse8 keeps a two-unit record inside an
// aligned 32-B block)
// (measured and removed: the fallback rows' words read non-temporally, so
// row lines -- 64 B of which a step uses 4 -- would leave L2 to the
// records: lines 5.46 -> 8.80 ms; profiles/r04/gid_order/stage16_nt_rows_ab.json)
// Branch-free selects: (m & b) | (~m & a) is one v_bfi_b32.  (Written as
// ternaries, the compiler turned a record's word picks into exec-mask
// branches -- the first fallback-linked kernel had 2.2x the scalar and 1.5x
// the vector instructions of the 8-B-unit kernel per step and measured
// 13-30% slower.)
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) { return (m & b) | (~m & a); }
__device__ __forceinline__ uint32_t bmask(bool c) { return 0u - (uint32_t)c; }

template <int KR, int RB = 16, int BU = 8>
__device__ __forceinline__ uint32_t sdfa_lds_step(const uint8_t* __restrict__ base, uint32_t F,
                                                  const uint32_t* __restrict__ s_rows, uint32_t s, uint32_t c,
                                                  uint32_t& cb, uint4 (&R)[4]) {
    static_assert(BU == 8 || (BU == 4 && RB == 8), "4-unit blocks are 8-B units");
    const bool isrow = s < F;
    const uint32_t rec = s - F, b = rec >> (RB == 8 ? (BU == 8 ? 3 : 2) : 2);
    if (RB == 8) {
        // one guarded site per load, selects (v_bfi) elsewhere
        const bool lrow = KR && isrow && s < (uint32_t)KR;
        uint32_t rv = 0;
        if (isrow && !lrow) rv = *reinterpret_cast<const uint32_t*>(base + (s * 1024u + c * 4u));
        if (!isrow && b != cb) {
            const uint4* p = reinterpret_cast<const uint4*>(base + F * 1024u + b * (BU == 8 ? 64u : 32u));
            R[0] = p[0];
            R[1] = p[1];
            if (BU == 8) {
                R[2] = p[2];
                R[3] = p[3];
            }
            cb = b;
        }
        const uint32_t lw = KR ? s_rows[(bmask(lrow) & s) * 256u + c] : 0u;
        // unit e = {y, x} and the next unit {z, w2} (a two-unit record never
        // straddles an aligned 32-B block)
        const uint32_t e = rec & (BU - 1u);
        const uint32_t m1 = bmask(e & 1u), m2 = bmask(e & 2u);
        uint4 A = R[0], B = R[1];
        if (BU == 8) {
            const uint32_t m4 = bmask(e & 4u);
            A = make_uint4(bsel(m4, R[0].x, R[2].x), bsel(m4, R[0].y, R[2].y), bsel(m4, R[0].z, R[2].z),
                           bsel(m4, R[0].w, R[2].w));
            B = make_uint4(bsel(m4, R[1].x, R[3].x), bsel(m4, R[1].y, R[3].y), bsel(m4, R[1].z, R[3].z),
                           bsel(m4, R[1].w, R[3].w));
        }
        const uint32_t y = bsel(m2, bsel(m1, A.x, A.z), bsel(m1, B.x, B.z));
        const uint32_t x = bsel(m2, bsel(m1, A.y, A.w), bsel(m1, B.y, B.w));
        const uint32_t z = bsel(m2, bsel(m1, A.z, B.x), B.z);
        const uint32_t w2 = bsel(m2, bsel(m1, A.w, B.y), B.w);
        const uint32_t key = c | 0x100u;
        const bool two = x >> 31;
        const bool h0 = (x & 0x1FFu) == key, h1 = two && ((x >> 16) & 0x1FFu) == key;
        const uint32_t w = bsel(bmask(two), (x >> 9) & 0x3FFFFFu, w2);  // the fallback row
        uint32_t mv = 0;
        if (!isrow && !h0 && !h1) {
            if (KR && w < (uint32_t)KR) mv = s_rows[w * 256u + c];
            else mv = *reinterpret_cast<const uint32_t*>(base + (w * 1024u + c * 4u));
        }
        const uint32_t rrec = bsel(bmask(h0), bsel(bmask(h1), mv, z), y);
        return bsel(bmask(isrow), rrec, bsel(bmask(lrow), rv, lw));
    }
    uint32_t rv = 0;
    if (isrow) {
        if (KR && s < (uint32_t)KR) rv = s_rows[s * 256u + c];
        else rv = *reinterpret_cast<const uint32_t*>(base + (s * 1024u + c * 4u));
    } else if (b != cb) {
        const uint4* p = reinterpret_cast<const uint4*>(base + F * 1024u + b * 64u);
        R[0] = p[0];
        R[1] = p[1];
        R[2] = p[2];
        R[3] = p[3];
        cb = b;
    }
    if (isrow) return rv;
    const uint32_t key = c | 0x100u;
    const uint4 q = pick4(R, rec & 3u);
    if ((q.x & 0x1FFu) == key) return q.y;
    if (((q.x >> 16) & 0x1FFu) == key) return q.z;
    const uint32_t w = q.w;  // the fallback row
    if (KR && w < (uint32_t)KR) return s_rows[w * 256u + c];
    return *reinterpret_cast<const uint32_t*>(base + (w * 1024u + c * 4u));
}

// (two 512-lane workgroups per CU: 4 waves per SIMD, so at most 128 VGPRs)
template <int OUTW, int BLK, int KR, int CH = 1, int RB = 16, int TB = 1>
__global__ __launch_bounds__(DFA_LDS_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void dfa_sparse_lds_kernel(
    const uint8_t* __restrict__ text, int64_t stream_start, int64_t pos0, int64_t n, void* __restrict__ out,
    unsigned long long* __restrict__ count, const uint8_t* __restrict__ base, uint32_t F,
    const uint32_t* __restrict__ outt, int64_t warm, int64_t seg_len, const uint32_t* __restrict__ gram3) {
    __shared__ __attribute__((aligned(16))) uint32_t s_rows[KR ? KR * 256 : 1];
    if (KR) {
        const uint32_t nr = F < (uint32_t)KR ? F : (uint32_t)KR;
        const uint4* src = reinterpret_cast<const uint4*>(base);
        uint4* dst = reinterpret_cast<uint4*>(s_rows);
        for (uint32_t k = threadIdx.x; k < nr * 64u; k += DFA_LDS_THREADS) dst[k] = src[k];
        __syncthreads();
    }
    const int64_t nseg = (n + seg_len - 1) / seg_len;
    const int64_t lanes = (int64_t)gridDim.x * DFA_LDS_THREADS;
    uint32_t cnt = 0;
    uint32_t cb[CH];  // record block cached in R[k]
    uint4 R[CH][4];
#pragma unroll
    for (int k = 0; k < CH; ++k) {
        cb[k] = 0xFFFFFFFFu;
#pragma unroll
        for (int e = 0; e < 4; ++e) R[k][e] = make_uint4(0u, 0u, 0u, 0u);
    }
    // CH segments per lane in lock step (sg0 + k * lanes), their loads in flight together
    for (int64_t sg0 = (int64_t)blockIdx.x * DFA_LDS_THREADS + threadIdx.x; sg0 < nseg; sg0 += CH * lanes) {
        int64_t lo[CH], hi[CH], wlo[CH];
        uint32_t s[CH];
        int64_t wmax = 0;
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int64_t sg = sg0 + k * lanes;
            lo[k] = sg < nseg ? pos0 + sg * seg_len : pos0 + n;
            hi[k] = sg < nseg ? (lo[k] + seg_len < pos0 + n ? lo[k] + seg_len : pos0 + n) : pos0 + n;
            wlo[k] = lo[k] - warm < stream_start ? stream_start : lo[k] - warm;
            if (sg >= nseg) wlo[k] = lo[k];
            s[k] = 0;
            // start the warm-up at the last synchronizing 3-gram before lo
            if (gram3) wlo[k] = dfa_sync_lo(text, lo[k], wlo[k], gram3);
            wmax = lo[k] - wlo[k] > wmax ? lo[k] - wlo[k] : wmax;
        }
        // (every loop over the chains k is unrolled in the front end: R[k]
        // must never be indexed at run time, or the arrays go to scratch)
        for (int64_t j = wmax; j > 0; --j) {  // warm-up from the root, right-aligned
            unroll_for<0, CH>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                const bool on = lo[k] - j >= wlo[k];
                const uint32_t v = sdfa_lds_step<KR, RB>(base, F, s_rows, s[k], on ? text[lo[k] - j] : 0u, cb[k], R[k]);
                s[k] = on ? v & DFA_STATE_MASK : s[k];
            });
        }
        constexpr int NW = BLK / 4;
        const int64_t nblk = seg_len / BLK;
        // the text of TB consecutive blocks per load: with TB = 2 a lane's
        // 128-B line of text is fetched twice instead of four times (it is
        // evicted between blocks: 1,024 chains per CU step through the L2)
        for (int64_t b0 = 0; b0 < nblk; b0 += TB) {
            bool actt[TB][CH], anyt[TB];
            uint32_t WT[TB][CH][NW];
#pragma unroll
            for (int tt = 0; tt < TB; ++tt) {
                anyt[tt] = false;
#pragma unroll
                for (int k = 0; k < CH; ++k) {
                    actt[tt][k] = lo[k] + BLK * (b0 + tt) + BLK <= hi[k];
                    anyt[tt] |= actt[tt][k];
#pragma unroll
                    for (int q = 0; q < BLK / 16; ++q) {
                        const tu32x4 w = actt[tt][k]
                                             ? *reinterpret_cast<const tu32x4*>(text + lo[k] + BLK * (b0 + tt) + 16 * q)
                                             : tu32x4{0u, 0u, 0u, 0u};
                        WT[tt][k][4 * q] = w.x;
                        WT[tt][k][4 * q + 1] = w.y;
                        WT[tt][k][4 * q + 2] = w.z;
                        WT[tt][k][4 * q + 3] = w.w;
                    }
                }
            }
            if (!anyt[0]) break;
            unroll_for<0, TB>([&](auto tc) {
            constexpr int tt = decltype(tc)::value;
            if (tt > 0 && !anyt[tt]) return;
            const int64_t b = b0 + tt;
            const bool(&act)[CH] = actt[tt];
            const uint32_t(&W)[CH][NW] = WT[tt];
            // the coded words themselves (target | code << 20): one register
            // per position holds both the code and, for an escape, the state
            uint32_t vw[CH][BLK];
#pragma unroll
            for (int j = 0; j < BLK; ++j) {
                unroll_for<0, CH>([&](auto kc) {
                    constexpr int k = decltype(kc)::value;
                    const uint32_t v =
                        sdfa_lds_step<KR, RB>(base, F, s_rows, s[k], (W[k][j >> 2] >> (8 * (j & 3))) & 0xFFu, cb[k], R[k]);
                    s[k] = act[k] ? v & DFA_STATE_MASK : s[k];
                    vw[k][j] = v;
                });
            }
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                if (!act[k]) continue;
                uint32_t r[BLK];
                // (count only: an escape code is a nonzero id, no lookup)
#pragma unroll
                for (int j = 0; j < BLK; ++j)
                    r[j] = OUTW && (vw[k][j] >> 20) == DFA_ESC ? outt[vw[k][j] & DFA_STATE_MASK] : vw[k][j] >> 20;
                const int64_t i = lo[k] + BLK * b;
                if (OUTW == 4) {
                    uint4* o = reinterpret_cast<uint4*>(reinterpret_cast<uint32_t*>(out) + (i - pos0));
#pragma unroll
                    for (int q = 0; q < BLK / 4; ++q)
                        o[q] = make_uint4(r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]);
                }
                if (OUTW == 2) {
                    uint4* o = reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(out) + (i - pos0));
#pragma unroll
                    for (int q = 0; q < BLK / 8; ++q)
                        o[q] = make_uint4(r[8 * q] | r[8 * q + 1] << 16, r[8 * q + 2] | r[8 * q + 3] << 16,
                                          r[8 * q + 4] | r[8 * q + 5] << 16, r[8 * q + 6] | r[8 * q + 7] << 16);
                }
#pragma unroll
                for (int j = 0; j < BLK; ++j) cnt += r[j] != 0u;
            }
            });
        }
        // the segments' last (< BLK) positions; k a compile-time constant
        // (a runtime k would index R[k] dynamically: the array goes to scratch)
        unroll_for<0, CH>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            for (int64_t i = lo[k] + BLK * ((hi[k] - lo[k]) / BLK); i < hi[k]; ++i) {
                s[k] = sdfa_lds_step<KR, RB>(base, F, s_rows, s[k], text[i], cb[k], R[k]) & DFA_STATE_MASK;
                const uint32_t v = outt[s[k]];
                if (OUTW) put_id<OUTW>(out, i - pos0, v);
                cnt += v != 0u;
            }
        });
    }
    if (count) {
        for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off);
        if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(count, (unsigned long long)cnt);
    }
}

// A value every lane of the wave holds, in scalar registers.
__device__ __forceinline__ int64_t wave_uniform64(int64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
    return (int64_t)((uint64_t)hi << 32 | lo);
}

// ---- the fallback-linked (FL) form (pm_flatten.h, pm_pack_sparse_fl) -----
// The 8-B form's record holds its fallback row, so it has no room for the
// record's own output: record states whose output is past the inline code
// escape (a second pass over LDS and the global out8 table).  In the FL form
// the word that leads into a record names the record's fallback row (12
// bits; the rare fallbacks past that sit in the record), so a record
// carries its own 16-bit output and only row outputs past the code escape.
// (This was first built to let a lane load the block and the fallback row's
// word together -- the wave model, scripts/sdfa_spec_model.cpp, put that at
// 1.77 -> 1.22 dependent latencies per wave step -- but measured, the extra
// requests cost more than the latency saved on the lines stream: snort
// 5.09 ms/GiB without, 5.42 for non-chain records, 6.22 for every new
// block; profiles/r05/ab/fl_spec_ablation.jsonl.  The product does not
// speculate; the ablation build AB_HIPFLAGS=-DPM_FL_SPEC=2, scripts/
// build_ab.sh, loads the fallback word with every new record block.)
//
// One step from the word w that led to the lane's state (state w & MASK;
// for a record, the fallback row in bits 20-31) on byte c: returns the next
// word.  For a record state, own = its out16: the output of the position
// that produced w.
#ifndef PM_FL_SPEC
#define PM_FL_SPEC 0
#endif
static_assert(PM_FL_SPEC == 0 || PM_FL_SPEC == 2, "PM_FL_SPEC: 0 (product) or 2 (ablation)");
#ifndef PM_FL_COUNT_TB
#define PM_FL_COUNT_TB 2
#endif
// dfa_fl2_kernel's id staging: one ds_write_b32 per two positions (1) or
// one ds_write_b16 per position (0)
#ifndef PM_FL2_PACKED_STAGING
#define PM_FL2_PACKED_STAGING 1
#endif
// The FL kernels' text loads (ablation builds: -DPM_FL_TEXT_NT=1 loads the
// text non-temporally, so its lines are the first out of L2)
#if defined(PM_FL_TEXT_NT) && PM_FL_TEXT_NT
#define PM_FL_TEXT_LOAD(p) __builtin_nontemporal_load(p)
#else
#define PM_FL_TEXT_LOAD(p) (*(p))
#endif

// A lane holds the records around its state: for a shallow record (granule
// below GD, pm_flatten.h FlImage::deep_g) the 16-B half holding it, in
// R[0]; for a deep one the aligned block of NR 16-B halves (NR 2: 32 B, the
// default; 4: 64 B; 1: every record as a half, GD ignored -- DfaDev::flhold,
// the picks time all three).  The held key: the half's index, or the
// block's with the top bit set.
template <int NR>
struct FlHold {
    tu32x4 R[NR];
};

template <int NR>
__device__ __forceinline__ bool fl_deep(uint32_t g, uint32_t GD) {
    return NR > 1 && g >= GD;
}

template <int NR>
__device__ __forceinline__ uint32_t fl_key(uint32_t g, bool deep) {
    constexpr uint32_t DSHIFT = NR == 8 ? 4u : NR == 4 ? 3u : 2u;  // granules per deep block: 16, 8 or 4
    return deep ? (g >> DSHIFT) | 0x80000000u : g >> 1;
}

template <int NR>
__device__ __forceinline__ void fl_load(const uint8_t* __restrict__ base, uint32_t F, uint32_t g, bool deep,
                                        FlHold<NR>& H) {
    const tu32x4* p =
        reinterpret_cast<const tu32x4*>(base + F * 1024u + ((g >> 1) & (deep ? ~(uint32_t)(NR - 1) : ~0u)) * 16u);
    H.R[0] = p[0];
    if (deep) {
#pragma unroll
        for (int k = 1; k < NR; ++k) H.R[k] = p[k];
    }
}

__device__ __forceinline__ tu32x4 bsel4(uint32_t m, const tu32x4& a, const tu32x4& b) {
    return tu32x4{bsel(m, a.x, b.x), bsel(m, a.y, b.y), bsel(m, a.z, b.z), bsel(m, a.w, b.w)};
}

// The 16-B register holding granule g (a shallow half is always R[0]).
template <int NR>
__device__ __forceinline__ tu32x4 fl_reg(const FlHold<NR>& H, uint32_t g, bool deep) {
    if (NR == 1) return H.R[0];
    const uint32_t m2 = bmask(deep && (g & 2u));
    if (NR == 2) return bsel4(m2, H.R[0], H.R[NR - 1]);
    const uint32_t m4 = bmask(deep && (g & 4u));
    const tu32x4 a = bsel4(m4, bsel4(m2, H.R[0], H.R[1 % NR]), bsel4(m2, H.R[2 % NR], H.R[3 % NR]));
    if (NR == 4) return a;
    const uint32_t m8 = bmask(deep && (g & 8u));  // NR 8: 128-B blocks
    const tu32x4 b = bsel4(m4, bsel4(m2, H.R[4 % NR], H.R[5 % NR]), bsel4(m2, H.R[6 % NR], H.R[7 % NR]));
    return bsel4(m8, a, b);
}

template <int KR, int NR>
__device__ __forceinline__ uint32_t fl_step(const uint8_t* __restrict__ base, uint32_t F, uint32_t GD,
                                            const uint32_t* __restrict__ s_rows, uint32_t w, uint32_t c,
                                            uint32_t& cb, FlHold<NR>& H, uint32_t& own) {
    const uint32_t s = w & DFA_STATE_MASK;
    const bool isrow = s < F;
    const uint32_t g = s - F;
    const bool deep = fl_deep<NR>(g, GD);
    const uint32_t key = fl_key<NR>(g, deep);
    const uint32_t fb = w >> 20;
    const bool newblk = !isrow && key != cb;
    const bool pre = PM_FL_SPEC == 2 && newblk && fb != PM_FL_INREC && fb >= (uint32_t)KR;
    const bool lrow = isrow && s < (uint32_t)KR;
    // the global word: a row state's word (or, PM_FL_SPEC 2, a new
    // record's fallback word loaded with its block)
    uint32_t x = 0;
    if ((isrow && !lrow) || pre) x = *reinterpret_cast<const uint32_t*>(base + (bsel(bmask(isrow), fb, s) * 1024u + c * 4u));
    if (newblk) {
        fl_load(base, F, g, deep, H);
        cb = key;
    }
    const uint32_t lw = s_rows[(bmask(lrow) & s) * 256u + c];  // (row 0 for the other lanes: no branch)
    // words 2e .. 2e + 3 of what the lane holds, e the granule in it (a
    // 16-B record starts at an even granule)
    const tu32x4 RR = fl_reg(H, g, deep);
    const uint32_t m1 = bmask(g & 1u);
    const uint32_t w0 = bsel(m1, RR.x, RR.z), w1 = bsel(m1, RR.y, RR.w), w2 = RR.z, w3 = RR.w;
    own = w0 & 0xFFFFu;
    const bool h0 = c == ((w0 >> 16) & 0xFFu), h1 = c == (w0 >> 24);
    const uint32_t row = bsel(bmask(fb == PM_FL_INREC), fb, w3);
    // a record's miss: its fallback row's word
    uint32_t y = 0;
    if (!isrow && !h0 && !h1 && !pre) {
        if (KR && row < (uint32_t)KR) y = s_rows[row * 256u + c];
        else y = *reinterpret_cast<const uint32_t*>(base + (row * 1024u + c * 4u));
    }
    const uint32_t rec = bsel(bmask(h0), bsel(bmask(h1), bsel(bmask(pre), y, x), w2), w1);
    return bsel(bmask(isrow), rec, bsel(bmask(lrow), x, lw));
}

// The output of the position that produced w: a record's own out16 (what
// holds it loaded if the lane does not hold it -- the next step's load,
// made early), or a row word's code; *esc = the code escapes (the answer
// is then rowout16[w & MASK]).
template <int NR>
__device__ __forceinline__ uint32_t fl_output(const uint8_t* __restrict__ base, uint32_t F, uint32_t GD, uint32_t w,
                                              uint32_t& cb, FlHold<NR>& H, bool& esc) {
    const uint32_t s = w & DFA_STATE_MASK;
    esc = false;
    if (s < F) {
        esc = (w >> 20) == DFA_ESC;
        return w >> 20;
    }
    const uint32_t g = s - F;
    const bool deep = fl_deep<NR>(g, GD);
    const uint32_t key = fl_key<NR>(g, deep);
    if (key != cb) {
        fl_load(base, F, g, deep, H);
        cb = key;
    }
    const tu32x4 RR = fl_reg(H, g, deep);
    return ((g & 1u) ? RR.z : RR.x) & 0xFFFFu;
}

// The FL form's scan: ids staged in LDS (u16 staging rows of 17 dwords, so
// the 64 lanes of a step hit 64 banks; the rare row outputs past the inline
// code resolved in rounds, one load per lane per round), whole-line
// non-temporal stores (store instruction t writes the 128-B lines of chains
// CPI * t + lane / LPC), 1,024-lane workgroups, the KR profile-chosen rows
// in LDS, the FL step, and
// outputs one step late: a step writes the output of the position before it
// (the state it starts from holds it).  OUTW 4 / 2: u32 / u16 ids (a u16
// block of a chain is 64 B: four lanes' 16-B stores, 16 chains per store
// instruction); 0: the count alone, no staging rows, no escapes, no stores.
// NR: the 16-B halves a lane holds of a deep block (FlHold; each its own
// instance, so profiles tell the picks' trials from the default's launches).
template <int KR, int OUTW = 4, int NR = 2, int THREADS = 1024>
__global__ __launch_bounds__(THREADS) void dfa_fl_kernel(
    const uint8_t* __restrict__ text, int64_t stream_start, int64_t pos0, int64_t n, void* __restrict__ out,
    unsigned long long* __restrict__ count, const uint8_t* __restrict__ base, uint32_t F, uint32_t GD,
    const uint16_t* __restrict__ rowout16, int64_t warm, int64_t seg_len, const uint32_t* __restrict__ gram3) {
    static_assert(OUTW == 0 || OUTW == 2 || OUTW == 4, "u32 / u16 ids or the count");
    constexpr int BLK = 32, SROW = 17;
    constexpr bool kIds = OUTW != 0;
    __shared__ __attribute__((aligned(16))) uint32_t s_rows[KR * 256];
    __shared__ uint32_t s_ids[kIds ? THREADS * SROW : 1];
    {
        const uint32_t nr = F < (uint32_t)KR ? F : (uint32_t)KR;
        const uint4* src = reinterpret_cast<const uint4*>(base);
        uint4* dst = reinterpret_cast<uint4*>(s_rows);
        for (uint32_t k = threadIdx.x; k < nr * 64u; k += THREADS) dst[k] = src[k];
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    uint16_t* const my = reinterpret_cast<uint16_t*>(s_ids + (kIds ? threadIdx.x * SROW : 0));
    const uint32_t* const wrows = s_ids + (kIds ? (threadIdx.x - lane) * SROW : 0);  // the wave's rows
    const int64_t nseg = (n + seg_len - 1) / seg_len;
    const int64_t lanes = (int64_t)gridDim.x * THREADS;
    uint32_t cnt = 0, cb = 0xFFFFFFFFu, own = 0;
    FlHold<NR> H;
#pragma unroll
    for (int k = 0; k < NR; ++k) H.R[k] = tu32x4{0u, 0u, 0u, 0u};
    for (int64_t sg0 = (int64_t)blockIdx.x * THREADS + threadIdx.x; __ballot(sg0 < nseg); sg0 += lanes) {
        const bool has = sg0 < nseg;
        // the wave's segments are consecutive: a wave-uniform 64-bit base
        // (scalar registers) and 32-bit lane offsets for the text loads and
        // the stores
        const int64_t wseg = wave_uniform64(sg0 - lane);
        const uint32_t sl = (uint32_t)seg_len;
        const uint8_t* const tbase = text + pos0 + wseg * seg_len;
        const int64_t lo = has ? pos0 + sg0 * seg_len : pos0 + n;
        const int64_t hi = has ? (lo + seg_len < pos0 + n ? lo + seg_len : pos0 + n) : pos0 + n;
        int64_t wlo = !has ? lo : lo - warm < stream_start ? stream_start : lo - warm;
        if (gram3) wlo = dfa_sync_lo(text, lo, wlo, gram3);
        uint32_t w = 0;  // the root, reached by no word
        for (int64_t i = wlo; i < lo; ++i) w = fl_step<KR, NR>(base, F, GD, s_rows, w, text[i], cb, H, own);
        const int64_t nblk = seg_len / BLK;
        // two blocks' text per load (the count: PM_FL_COUNT_TB, an ablation
        // switch: 4 = a lane's whole 128-B text line at once)
        constexpr int TB = OUTW == 0 ? PM_FL_COUNT_TB : 2;
        for (int64_t b0 = 0; b0 < nblk; b0 += TB) {
            bool act[TB];
            uint32_t WT[TB][8];
#pragma unroll
            for (int tt = 0; tt < TB; ++tt) {
                act[tt] = lo + BLK * (b0 + tt) + BLK <= hi;
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const tu32x4* tp = reinterpret_cast<const tu32x4*>(
                        tbase + ((uint32_t)lane * sl + (uint32_t)(BLK * (b0 + tt) + 16 * q)));
                    const tu32x4 v = act[tt] ? PM_FL_TEXT_LOAD(tp) : tu32x4{0u, 0u, 0u, 0u};
                    WT[tt][4 * q] = v.x;
                    WT[tt][4 * q + 1] = v.y;
                    WT[tt][4 * q + 2] = v.z;
                    WT[tt][4 * q + 3] = v.w;
                }
            }
            if (!__ballot(act[0])) break;
            unroll_for<0, TB>([&](auto tc) {
                constexpr int tt = decltype(tc)::value;
                if (tt > 0 && !__ballot(act[tt])) return;
                const int64_t b = b0 + tt;
                uint32_t em = 0;
#pragma unroll
                for (int j = 0; j < BLK; ++j) {
                    const uint32_t wn = fl_step<KR, NR>(base, F, GD, s_rows, w, (WT[tt][j >> 2] >> (8 * (j & 3))) & 0xFFu, cb,
                                                    H, own);
                    if (j > 0) {  // the output of position j - 1, which produced w
                        const bool rec = (w & DFA_STATE_MASK) >= F;
                        const uint32_t code = w >> 20;
                        const bool esc = !rec && code == DFA_ESC;
                        const uint32_t id = rec ? own : code;
                        if (kIds) {
                            my[j - 1] = (uint16_t)(esc ? (w & DFA_STATE_MASK) : id);
                            em |= esc ? 1u << (j - 1) : 0u;
                        }
                        cnt += act[tt] && id != 0u;  // an escape is a nonzero id
                    }
                    w = act[tt] ? wn : w;
                }
                {  // position 31
                    bool esc;
                    const uint32_t id = fl_output(base, F, GD, w, cb, H, esc);
                    if (kIds) {
                        my[BLK - 1] = (uint16_t)(esc ? (w & DFA_STATE_MASK) : id);
                        em |= esc ? 1u << (BLK - 1) : 0u;
                    }
                    cnt += act[tt] && id != 0u;
                }
                if (!kIds) return;
                if (!act[tt]) em = 0;
                while (__ballot(em != 0)) {  // row outputs past the inline code: one per lane per round
                    if (em) {
                        const uint32_t j = __builtin_ctz(em);
                        em &= em - 1;
                        my[j] = rowout16[my[j]];
                    }
                }
                __builtin_amdgcn_wave_barrier();
                // Store instruction t writes chain cc = CPI * t + lane / LPC
                // (LPC lanes of 16 B each per chain block): whole lines.  The
                // lane's LDS and output offsets are laundered per block so
                // the compiler forms each store's addresses from one register
                // and an immediate / scalar step (hoisted out of the block
                // loop, eight of each spilled, and their reloads waited for
                // every store in flight)
                constexpr int LPC = OUTW == 4 ? 8 : 4, CPI = 64 / LPC, NST = 64 / CPI;
                const uint64_t am = __ballot(act[tt]);
                uint32_t lds_off = ((uint32_t)(lane / LPC) * SROW + (OUTW == 4 ? 2u : 4u) * (lane % LPC)) * 4u;
                uint32_t go = (uint32_t)(lane / LPC) * sl + (uint32_t)(16 / (OUTW ? OUTW : 4)) * (lane % LPC);
                asm volatile("" : "+v"(lds_off), "+v"(go));
                const uint64_t mine = am >> (lane / LPC);  // bit CPI * t: chain of store t active
                const bool full = am == ~0ull;
                const uint8_t* const lb = reinterpret_cast<const uint8_t*>(wrows) + lds_off;
                // every store's ids read first (one LDS wait per batch),
                // inactive chains too; two batches where the lane holds 64-B
                // blocks (registers)
                constexpr int NBAT = NR >= 4 ? 2 : 1, BST = NST / NBAT;
#pragma unroll
                for (int t0 = 0; t0 < NST; t0 += BST) {
                    tu32x4 vs[BST];
#pragma unroll
                    for (int t = t0; t < t0 + BST; ++t) {
                        const uint32_t* src = reinterpret_cast<const uint32_t*>(lb + t * CPI * SROW * 4);
                        if (OUTW == 4) {
                            const uint32_t w0 = src[0], w1 = src[1];
                            vs[t - t0] = tu32x4{w0 & 0xFFFFu, w0 >> 16, w1 & 0xFFFFu, w1 >> 16};
                        } else {
                            vs[t - t0] = tu32x4{src[0], src[1], src[2], src[3]};
                        }
                    }
#pragma unroll
                    for (int t = t0; t < t0 + BST; ++t) {
                        const tu32x4 v = vs[t - t0];
                        const int64_t step = (int64_t)(CPI * t) * seg_len + BLK * b;  // wave-uniform
                        tu32x4* o = OUTW == 4
                                        ? reinterpret_cast<tu32x4*>(reinterpret_cast<uint32_t*>(out) + wseg * seg_len + step + go)
                                        : reinterpret_cast<tu32x4*>(reinterpret_cast<uint16_t*>(out) + wseg * seg_len + step + go);
                        if (full || ((mine >> (CPI * t)) & 1u)) __builtin_nontemporal_store(v, o);
                    }
                }
                __builtin_amdgcn_wave_barrier();
            });
        }
        // the segment's last (< BLK) positions
        for (int64_t i = lo + BLK * ((hi - lo) / BLK); i < hi; ++i) {
            w = fl_step<KR, NR>(base, F, GD, s_rows, w, text[i], cb, H, own);
            bool esc;
            uint32_t id = fl_output(base, F, GD, w, cb, H, esc);
            if (kIds && esc) id = rowout16[w & DFA_STATE_MASK];
            if (OUTW == 4) reinterpret_cast<uint32_t*>(out)[i - pos0] = id;
            if (OUTW == 2) reinterpret_cast<uint16_t*>(out)[i - pos0] = (uint16_t)id;
            cnt += id != 0u;
        }
    }
    if (count) {
        for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off);
        if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(count, (unsigned long long)cnt);
    }
}

// ---- two chains per lane (round 6) ----------------------------------------
// A wave's step waits for the slowest of its 64 lanes' dependent loads (the
// record block a lane enters, then at a slot miss its fallback row's word):
// on pattern-dense text nearly every wave step has a lane that goes past L2,
// so dfa_fl_kernel runs at about one memory latency per wave step (~1.2 us
// per step on the lines stream, the SIMDs ~25% busy).  Here each lane walks
// two segments in lock step and issues the loads of both before it waits
// for either: two positions per lane per wave step for about one latency.
// The step is fl_step in three parts -- fl_issue (the row word, the record
// block, the LDS row word), fl_mid (on the block: the slot test, the
// record's output, the fallback row's word), fl_fin (the select) -- run
// chain A, chain B at each part.  Twice the staging rows (2 x 17 dwords a
// lane, 136 KiB) leave LDS for FL2_LDS_ROWS rows when ids are written; the
// count keeps FL_COUNT_LDS_ROWS.
// (ablation builds: -DPM_FL2_THREADS=768 -- 1,536 chains per CU, 56 rows,
// the registers for 64-B deep blocks)
#ifndef PM_FL2_THREADS
#define PM_FL2_THREADS 1024
#endif
constexpr int FL2_THREADS = PM_FL2_THREADS;
constexpr int FL2_LDS_ROWS = FL2_THREADS == 1024 ? 24 : 56;

struct FlPend {
    uint32_t s, c, fb, x, lw, r0, y, g;
    bool isrow, lrow, deep, miss;
};

template <int KR, int NR>
__device__ __forceinline__ void fl_issue(const uint8_t* __restrict__ base, uint32_t F, uint32_t GD,
                                         const uint32_t* __restrict__ s_rows, bool on, uint32_t w, uint32_t c,
                                         uint32_t& cb, FlHold<NR>& H, FlPend& P) {
    P.s = w & DFA_STATE_MASK;
    P.c = c;
    P.isrow = P.s < F;
    P.g = P.s - F;
    P.deep = fl_deep<NR>(P.g, GD);
    const uint32_t key = fl_key<NR>(P.g, P.deep);
    P.fb = w >> 20;
    const bool newblk = on && !P.isrow && key != cb;
    P.lrow = P.isrow && P.s < (uint32_t)KR;
    P.x = 0;
    if (on && P.isrow && !P.lrow) P.x = *reinterpret_cast<const uint32_t*>(base + (P.s * 1024u + c * 4u));
    if (newblk) {
        fl_load(base, F, P.g, P.deep, H);
        cb = key;
    }
    P.lw = s_rows[(bmask(P.lrow) & P.s) * 256u + c];  // (row 0 for the other lanes: no branch)
}

template <int KR, int NR>
__device__ __forceinline__ void fl_mid(const uint8_t* __restrict__ base, const uint32_t* __restrict__ s_rows, bool on,
                                       const FlHold<NR>& H, FlPend& P, uint32_t& own) {
    const tu32x4 RR = fl_reg(H, P.g, P.deep);
    const uint32_t m1 = bmask(P.g & 1u);
    const uint32_t w0 = bsel(m1, RR.x, RR.z), w1 = bsel(m1, RR.y, RR.w), w2 = RR.z, w3 = RR.w;
    own = w0 & 0xFFFFu;
    const uint32_t c = P.c;
    const bool h0 = c == ((w0 >> 16) & 0xFFu), h1 = c == (w0 >> 24);
    const uint32_t row = bsel(bmask(P.fb == PM_FL_INREC), P.fb, w3);
    P.miss = !P.isrow && !h0 && !h1;
    P.y = 0;
    if (on && P.miss) {
        if (KR && row < (uint32_t)KR) P.y = s_rows[row * 256u + c];
        else P.y = *reinterpret_cast<const uint32_t*>(base + (row * 1024u + c * 4u));
    }
    P.r0 = bsel(bmask(P.isrow), bsel(bmask(h0), bsel(bmask(h1), 0u, w2), w1), bsel(bmask(P.lrow), P.x, P.lw));
}

__device__ __forceinline__ uint32_t fl_fin(const FlPend& P) { return bsel(bmask(P.miss), P.r0, P.y); }

// fl_output in two parts: the block load of a record state (for both
// chains before either is used), then the output.
template <int NR>
__device__ __forceinline__ void fl_out_issue(const uint8_t* __restrict__ base, uint32_t F, uint32_t GD, uint32_t w,
                                             uint32_t& cb, FlHold<NR>& H) {
    const uint32_t s = w & DFA_STATE_MASK;
    if (s >= F) {
        const uint32_t g = s - F;
        const bool deep = fl_deep<NR>(g, GD);
        const uint32_t key = fl_key<NR>(g, deep);
        if (key != cb) {
            fl_load(base, F, g, deep, H);
            cb = key;
        }
    }
}
template <int NR>
__device__ __forceinline__ uint32_t fl_out_get(uint32_t F, uint32_t GD, uint32_t w, const FlHold<NR>& H, bool& esc) {
    const uint32_t s = w & DFA_STATE_MASK;
    esc = false;
    if (s < F) {
        esc = (w >> 20) == DFA_ESC;
        return w >> 20;
    }
    const uint32_t g = s - F;
    const tu32x4 RR = fl_reg(H, g, fl_deep<NR>(g, GD));
    return ((g & 1u) ? RR.z : RR.x) & 0xFFFFu;
}

// dfa_fl_kernel with two chains per lane (the segments of chain k of lane l
// in a wave: wave base + 64 k + l, so each chain set of a wave is 64
// consecutive segments and its stores are dfa_fl_kernel's whole lines).
template <int KR, int OUTW = 4, int NR = 1, int THREADS = 1024>
__global__ __launch_bounds__(THREADS) void dfa_fl2_kernel(
    const uint8_t* __restrict__ text, int64_t stream_start, int64_t pos0, int64_t n, void* __restrict__ out,
    unsigned long long* __restrict__ count, const uint8_t* __restrict__ base, uint32_t F, uint32_t GD,
    const uint16_t* __restrict__ rowout16, int64_t warm, int64_t seg_len, const uint32_t* __restrict__ gram3) {
    static_assert(OUTW == 0 || OUTW == 2 || OUTW == 4, "u32 / u16 ids or the count");
    constexpr int BLK = 32, SROW = 17, CH = 2;
    constexpr bool kIds = OUTW != 0;
    __shared__ __attribute__((aligned(16))) uint32_t s_rows[KR * 256];
    __shared__ uint32_t s_ids[kIds ? CH * THREADS * SROW : 1];
    {
        const uint32_t nr = F < (uint32_t)KR ? F : (uint32_t)KR;
        const uint4* src = reinterpret_cast<const uint4*>(base);
        uint4* dst = reinterpret_cast<uint4*>(s_rows);
        for (uint32_t k = threadIdx.x; k < nr * 64u; k += THREADS) dst[k] = src[k];
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint16_t* my[CH];
    const uint32_t* wrows[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k) {
        my[k] = reinterpret_cast<uint16_t*>(s_ids + (kIds ? k * THREADS * SROW + threadIdx.x * SROW : 0));
        wrows[k] = s_ids + (kIds ? k * THREADS * SROW + (threadIdx.x - lane) * SROW : 0);
    }
    const int64_t nseg = (n + seg_len - 1) / seg_len;
    const int64_t nwaves = (int64_t)gridDim.x * (THREADS / 64);
    const uint32_t sl = (uint32_t)seg_len;
    uint32_t cnt = 0, cb[CH], own[CH], w[CH];
    uint32_t held16[CH] = {0u, 0u};  // PM_FL2_PACKED_STAGING: the even position of a pair
    FlHold<NR> H[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k) {
        cb[k] = 0xFFFFFFFFu;
        own[k] = 0;
#pragma unroll
        for (int r = 0; r < NR; ++r) H[k].R[r] = tu32x4{0u, 0u, 0u, 0u};
    }
    for (int64_t wv = (int64_t)blockIdx.x * (THREADS / 64) + wid; wv * 64 * CH < nseg; wv += nwaves) {  // uniform
        const int64_t wseg = wv * 64 * CH;
        // len: the chain's segment length (0: no segment); the warm-up is
        // the wn bytes before the segment
        uint32_t len[CH], wn[CH];
        const uint8_t* wp[CH];
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int64_t sg = wseg + 64 * k + lane;
            const bool has = sg < nseg;
            const int64_t lo = has ? pos0 + sg * seg_len : pos0 + n;
            const int64_t hi = has ? (lo + seg_len < pos0 + n ? lo + seg_len : pos0 + n) : pos0 + n;
            int64_t wlo = !has ? lo : lo - warm < stream_start ? stream_start : lo - warm;
            if (gram3) wlo = dfa_sync_lo(text, lo, wlo, gram3);
            len[k] = (uint32_t)(hi - lo);
            wn[k] = (uint32_t)(lo - wlo);
            wp[k] = text + wlo;
            w[k] = 0;  // the root, reached by no word
        }
        // the warm-ups, both chains in lock step
        for (uint32_t t = 0; __ballot(t < wn[0] || t < wn[1]); ++t) {
            bool on[CH];
            uint32_t cc[CH];
            FlPend P[CH];
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                on[k] = t < wn[k];
                cc[k] = on[k] ? wp[k][t] : 0u;
            }
#pragma unroll
            for (int k = 0; k < CH; ++k) fl_issue<KR, NR>(base, F, GD, s_rows, on[k], w[k], cc[k], cb[k], H[k], P[k]);
#pragma unroll
            for (int k = 0; k < CH; ++k) fl_mid<KR, NR>(base, s_rows, on[k], H[k], P[k], own[k]);
#pragma unroll
            for (int k = 0; k < CH; ++k) w[k] = on[k] ? fl_fin(P[k]) : w[k];
        }
        const int64_t nblk = seg_len / BLK;
        for (int64_t b = 0; b < nblk; ++b) {
            bool act[CH];
            uint32_t WT[CH][8];
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                act[k] = (uint32_t)(BLK * b + BLK) <= len[k];
                const uint8_t* const tb = text + pos0 + (wseg + 64 * k) * seg_len;  // wave-uniform
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const tu32x4* tp =
                        reinterpret_cast<const tu32x4*>(tb + ((uint32_t)lane * sl + (uint32_t)(BLK * b + 16 * q)));
                    const tu32x4 v = act[k] ? PM_FL_TEXT_LOAD(tp) : tu32x4{0u, 0u, 0u, 0u};
                    WT[k][4 * q] = v.x;
                    WT[k][4 * q + 1] = v.y;
                    WT[k][4 * q + 2] = v.z;
                    WT[k][4 * q + 3] = v.w;
                }
            }
            if (!__ballot(act[0] || act[1])) break;
            uint32_t em[CH] = {0u, 0u};
            // four positions per iteration, not unrolled further: the
            // dword of each chain's text in use is WT[k][0], shifted down
            // after each iteration (a fully unrolled block kept too much
            // live and spilled)
#pragma unroll 1
            for (uint32_t q = 0; q < BLK / 4; ++q) {
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const uint32_t j = 4 * q + jj;
                    FlPend P[CH];
#pragma unroll
                    for (int k = 0; k < CH; ++k)
                        fl_issue<KR, NR>(base, F, GD, s_rows, act[k], w[k], (WT[k][0] >> (8 * jj)) & 0xFFu, cb[k], H[k],
                                         P[k]);
#pragma unroll
                    for (int k = 0; k < CH; ++k) fl_mid<KR, NR>(base, s_rows, act[k], H[k], P[k], own[k]);
#pragma unroll
                    for (int k = 0; k < CH; ++k) {
                        const uint32_t wn = fl_fin(P[k]);
                        if (jj > 0 || q > 0) {  // the output of position j - 1, which produced w
                            const bool rec = (w[k] & DFA_STATE_MASK) >= F;
                            const uint32_t code = w[k] >> 20;
                            const bool esc = !rec && code == DFA_ESC;
                            const uint32_t id = rec ? own[k] : code;
                            if (kIds) {
                                const uint32_t v16 = esc ? (w[k] & DFA_STATE_MASK) : id;
#if PM_FL2_PACKED_STAGING
                                // two positions per staging write: position
                                // j - 1 even (jj 1, 3) is held, odd (jj 2, 0)
                                // writes the pair's dword
                                if (jj & 1) held16[k] = v16;
                                else reinterpret_cast<uint32_t*>(my[k])[(j - 1) >> 1] = held16[k] | v16 << 16;
#else
                                my[k][j - 1] = (uint16_t)v16;
#endif
                                em[k] |= esc ? 1u << (j - 1) : 0u;
                            }
                            cnt += act[k] && id != 0u;  // an escape is a nonzero id
                        }
                        w[k] = act[k] ? wn : w[k];
                    }
                }
#pragma unroll
                for (int k = 0; k < CH; ++k)
#pragma unroll
                    for (int i = 0; i < 7; ++i) WT[k][i] = WT[k][i + 1];
            }
            // position 31 of both chains
#pragma unroll
            for (int k = 0; k < CH; ++k) fl_out_issue<NR>(base, F, GD, w[k], cb[k], H[k]);
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                bool esc;
                const uint32_t id = fl_out_get<NR>(F, GD, w[k], H[k], esc);
                if (kIds) {
#if PM_FL2_PACKED_STAGING
                    reinterpret_cast<uint32_t*>(my[k])[(BLK - 1) >> 1] =
                        held16[k] | (esc ? (w[k] & DFA_STATE_MASK) : id) << 16;
#else
                    my[k][BLK - 1] = (uint16_t)(esc ? (w[k] & DFA_STATE_MASK) : id);
#endif
                    em[k] |= esc ? 1u << (BLK - 1) : 0u;
                }
                cnt += act[k] && id != 0u;
            }
            if (!kIds) continue;
#pragma unroll
            for (int k = 0; k < CH; ++k)
                if (!act[k]) em[k] = 0;
            while (__ballot(em[0] != 0 || em[1] != 0)) {  // row outputs past the inline code
#pragma unroll
                for (int k = 0; k < CH; ++k)
                    if (em[k]) {
                        const uint32_t j = __builtin_ctz(em[k]);
                        em[k] &= em[k] - 1;
                        my[k][j] = rowout16[my[k][j]];
                    }
            }
            __builtin_amdgcn_wave_barrier();
            // each chain set's block as dfa_fl_kernel stores it: whole lines
            constexpr int LPC = OUTW == 4 ? 8 : 4, CPI = 64 / LPC, NST = 64 / CPI, BST = 2;
#pragma unroll
            for (int k = 0; k < CH; ++k) {
                const uint64_t am = __ballot(act[k]);
                uint32_t lds_off = ((uint32_t)(lane / LPC) * SROW + (OUTW == 4 ? 2u : 4u) * (lane % LPC)) * 4u;
                uint32_t go = (uint32_t)(lane / LPC) * sl + (uint32_t)(16 / (OUTW ? OUTW : 4)) * (lane % LPC);
                asm volatile("" : "+v"(lds_off), "+v"(go));
                const uint64_t mine = am >> (lane / LPC);
                const bool full = am == ~0ull;
                const uint8_t* const lb = reinterpret_cast<const uint8_t*>(wrows[k]) + lds_off;
#pragma unroll
                for (int t0 = 0; t0 < NST; t0 += BST) {
                    tu32x4 vs[BST];
#pragma unroll
                    for (int t = t0; t < t0 + BST; ++t) {
                        const uint32_t* src = reinterpret_cast<const uint32_t*>(lb + t * CPI * SROW * 4);
                        if (OUTW == 4) {
                            const uint32_t w0 = src[0], w1 = src[1];
                            vs[t - t0] = tu32x4{w0 & 0xFFFFu, w0 >> 16, w1 & 0xFFFFu, w1 >> 16};
                        } else {
                            vs[t - t0] = tu32x4{src[0], src[1], src[2], src[3]};
                        }
                    }
#pragma unroll
                    for (int t = t0; t < t0 + BST; ++t) {
                        const tu32x4 v = vs[t - t0];
                        const int64_t step = (wseg + 64 * k + CPI * t) * seg_len + BLK * b;  // wave-uniform
                        tu32x4* o = OUTW == 4
                                        ? reinterpret_cast<tu32x4*>(reinterpret_cast<uint32_t*>(out) + step + go)
                                        : reinterpret_cast<tu32x4*>(reinterpret_cast<uint16_t*>(out) + step + go);
                        if (full || ((mine >> (CPI * t)) & 1u)) __builtin_nontemporal_store(v, o);
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        // the segments' last (< BLK) positions
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int64_t lo = pos0 + (wseg + 64 * k + lane) * seg_len;
            for (int64_t i = lo + BLK * (len[k] / BLK); i < lo + len[k]; ++i) {
                w[k] = fl_step<KR, NR>(base, F, GD, s_rows, w[k], text[i], cb[k], H[k], own[k]);
                bool esc;
                uint32_t id = fl_output(base, F, GD, w[k], cb[k], H[k], esc);
                if (kIds && esc) id = rowout16[w[k] & DFA_STATE_MASK];
                if (OUTW == 4) reinterpret_cast<uint32_t*>(out)[i - pos0] = id;
                if (OUTW == 2) reinterpret_cast<uint16_t*>(out)[i - pos0] = (uint16_t)id;
                cnt += id != 0u;
            }
        }
    }
    if (count) {
        for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off);
        if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(count, (unsigned long long)cnt);
    }
}

// The gather ceiling (pm_launch_gather_probe): the FL kernel's lanes
// without its logic -- each lane's next index is a hash of the word it
// loaded, so the loads are dependent and uniform over the table.
__global__ __launch_bounds__(1024) void gather_probe_kernel(const uint32_t* __restrict__ tab, uint32_t words,
                                                            int steps, uint32_t* __restrict__ sink) {
    const uint32_t lane = blockIdx.x * 1024u + threadIdx.x;
    uint32_t idx = __umulhi(lane * 0x9E3779B1u, words), acc = 0;
    for (int j = 0; j < steps; ++j) {
        const uint32_t v = tab[idx];
        acc += v;
        idx = __umulhi((v ^ (lane + (uint32_t)j)) * 0x9E3779B1u, words);
    }
    if (acc == 0x9E3779B1u && idx == 1u) sink[0] = acc;  // (all but never; keeps the chain live)
}

// Accuracy of one id stream against a reference one (Core/src/measure.c:
// 174-190 with is_pattern_suffix, PatternsTree.c:485-494), one position per
// lane-element: equal -> success; algo on real's parent chain -> partial;
// algo none -> false negative; else false positive.  all_matches adds
// depth[real] (patterns ending at the position).  counts[0..4] += success,
// partial, false_neg, false_pos, all_matches.  HBM-bound: 8 B per position.
__device__ __forceinline__ void score_one(uint32_t a, uint32_t r, const uint32_t* __restrict__ parent,
                                          const uint32_t* __restrict__ depth, uint32_t (&c)[5]) {
    if (a == r) {
        ++c[0];
    } else if (a) {
        uint32_t cur = r;
        while (cur && cur != a) cur = parent[cur];
        ++c[cur ? 1 : 3];
    } else {
        ++c[2];
    }
    if (r) c[4] += depth[r];
}

constexpr int SCORE_THREADS = 256;

// V pairs of 16-B loads per thread before scoring them (1 GiB: V=1 1.78 ms, V=2 1.69 ms).
constexpr int SCORE_V = 2;
template <int V>
__global__ __launch_bounds__(SCORE_THREADS) void score_kernel(const uint32_t* __restrict__ algo,
                                                              const uint32_t* __restrict__ real, int64_t n,
                                                              const uint32_t* __restrict__ parent,
                                                              const uint32_t* __restrict__ depth,
                                                              unsigned long long* __restrict__ counts) {
    uint32_t c[5] = {0, 0, 0, 0, 0};
    const int64_t nv = n / 4;
    const int64_t stride = (int64_t)gridDim.x * SCORE_THREADS;
    using v4 = __attribute__((ext_vector_type(4))) unsigned int;
    const v4* A = reinterpret_cast<const v4*>(algo);
    const v4* R = reinterpret_cast<const v4*>(real);
    for (int64_t k = (int64_t)blockIdx.x * SCORE_THREADS + threadIdx.x; k < nv; k += V * stride) {
        v4 a[V], r[V];
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const int64_t kj = k + j * stride;
            a[j] = kj < nv ? __builtin_nontemporal_load(A + kj) : v4{0, 0, 0, 0};
            r[j] = kj < nv ? __builtin_nontemporal_load(R + kj) : v4{0, 0, 0, 0};
        }
#pragma unroll
        for (int j = 0; j < V; ++j) {
            if (k + j * stride >= nv) break;
            score_one(a[j].x, r[j].x, parent, depth, c);
            score_one(a[j].y, r[j].y, parent, depth, c);
            score_one(a[j].z, r[j].z, parent, depth, c);
            score_one(a[j].w, r[j].w, parent, depth, c);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) score_one(algo[4 * nv + threadIdx.x], real[4 * nv + threadIdx.x], parent, depth, c);
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        unsigned long long v = c[q];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o);
        if ((threadIdx.x & 63) == 0 && v) atomicAdd(counts + q, v);
    }
}

// Per-pattern occurrence counts: every pattern on the suffix chain of
// real[i] occurs at i (all-matches expansion).  Gids [lo, lo + cnt) are
// counted in an LDS histogram per workgroup (cnt <= HIST_WINDOW), flushed to
// the u64 global histogram (nonzero counters only) at the end.
constexpr int HIST_THREADS = 1024;
constexpr uint32_t HIST_WINDOW = 38912;  // 152 KiB of u32 counters
constexpr int HIST_V = 4;  // 16-B answer loads per thread per step (snort 1 GiB: V=1/2/4/8 2.07/1.49/1.29/1.30 ms; one chain at a time 3.66)

// Each thread takes V 16-B loads of answers (4V positions) and walks their 4V
// suffix chains together, so the dependent parent[] gathers of one step are
// all in flight at once (one chain after another left them latency-bound).
// Measured and not kept (round 2): a "has parent" bit per gid so that only
// the ~5% of chains that go on gather parent[] — kept in bit 31 of the
// counter and read back by the add, 3.40 ms against 1.28 (an LDS add that
// returns its value waits; one that does not is fire-and-forget), or in an
// LDS bitmap beside the counters, 1.30-1.32 against 1.28 (the gathers of
// the ~3,000 gids a stream hits are L1 hits).
template <int V>
__global__ __launch_bounds__(HIST_THREADS) void hist_kernel(const uint32_t* __restrict__ real, int64_t n,
                                                            const uint32_t* __restrict__ parent, uint32_t lo,
                                                            uint32_t cnt, unsigned long long* __restrict__ hist) {
    __shared__ uint32_t s_h[HIST_WINDOW];
    for (uint32_t k = threadIdx.x; k < cnt; k += HIST_THREADS) s_h[k] = 0;
    __syncthreads();
    using v4 = __attribute__((ext_vector_type(4))) unsigned int;
    const int64_t nv = n / 4;
    const int64_t stride = (int64_t)gridDim.x * HIST_THREADS;
    for (int64_t k = (int64_t)blockIdx.x * HIST_THREADS + threadIdx.x; k < nv; k += V * stride) {
        uint32_t g[4 * V];
#pragma unroll
        for (int j = 0; j < V; ++j) {
            const int64_t kj = k + j * stride;
            const v4 r = kj < nv ? __builtin_nontemporal_load(reinterpret_cast<const v4*>(real) + kj) : v4{0, 0, 0, 0};
            g[4 * j] = r.x;
            g[4 * j + 1] = r.y;
            g[4 * j + 2] = r.z;
            g[4 * j + 3] = r.w;
        }
        for (;;) {
            uint32_t any = 0;
#pragma unroll
            for (int i = 0; i < 4 * V; ++i) any |= g[i];
            if (!any) break;
#pragma unroll
            for (int i = 0; i < 4 * V; ++i)
                if (g[i] - lo < cnt) atomicAdd(&s_h[g[i] - lo], 1u);
#pragma unroll
            for (int i = 0; i < 4 * V; ++i) g[i] = g[i] ? parent[g[i]] : 0u;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        for (uint32_t g = real[4 * nv + threadIdx.x]; g; g = parent[g])
            if (g - lo < cnt) atomicAdd(&s_h[g - lo], 1u);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < cnt; k += HIST_THREADS)
        if (s_h[k]) atomicAdd(hist + lo + k, (unsigned long long)s_h[k]);
}

__global__ void gen_lines_kernel(uint8_t* __restrict__ dst, uint64_t n, const uint8_t* __restrict__ pats,
                                 const uint32_t* __restrict__ offs, uint32_t npats, uint64_t seed) {
    const uint64_t nb = (n + PM_LINES_BLOCK - 1) / PM_LINES_BLOCK;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += stride) {
        const uint64_t lo = b * PM_LINES_BLOCK;
        pm_lines_block(dst + lo, n - lo < PM_LINES_BLOCK ? n - lo : PM_LINES_BLOCK, b, pats, offs, npats, seed);
    }
}

__global__ void gen_stream_kernel(uint8_t* __restrict__ dst, uint64_t off, uint64_t n, uint64_t seed, int mode) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride)
        dst[k] = pm_stream_byte(off + k, seed, mode);
}

}  // namespace

// Workgroups of an RT launch over n positions (persistent: one 1024-lane
// workgroup per CU, LDS-bound) and the spill items its waves may need.
// Workgroups: one per CU for large launches; a small launch gives each
// wave at least 8 chunks, but keeps a quarter of the CUs (each workgroup
// stages 80-160 KiB of tables into LDS, a fixed cost that swamps one or two
// chunks per wave).  Side by side on et (ms, profiles/r03/rt_grid_sweep.json):
//   4 MiB: 32 / 64 / 128 / 256 workgroups 0.036 / 0.027 / 0.035 / 0.059
//   16 MiB:                              0.101 / 0.058 / 0.049 / 0.067
//   64 MiB:                              0.366 / 0.193 / 0.116 / 0.104
static int64_t rt_blocks(int64_t n, int num_cu) {
    const int64_t nchunks = (n + RT_CHUNK - 1) / RT_CHUNK;
    const int64_t one_each = (nchunks + RT_WAVES - 1) / RT_WAVES;     // one chunk per wave
    const int64_t eight_each = (nchunks + 8 * RT_WAVES - 1) / (8 * RT_WAVES);
    const int64_t floor_b = one_each < num_cu / 4 ? one_each : num_cu / 4;
    int64_t b = eight_each > floor_b ? eight_each : floor_b;
    if (b > num_cu) b = num_cu;
    return b < 1 ? 1 : b;
}
// Spill items per wave region: one per position of the wave's main-loop
// chunks, capped at RT_SPILL_WAVE_CAP (the kernel resolves a full region
// and goes on, rt_scan_kernel): 128 KiB per wave, 512 MiB for a 1 GiB launch
// on 256 CUs instead of 8 B per position (8 GiB).  Side by side on the
// deep streams (1 GiB snort, dense / count, profiles/r03/spill_cap_ab.txt)
// caps of 16 / 32 / 64 / 128 chunks and the unbounded region measured
// equal (shipped 11.33-11.37 ms, lines 15.68-15.86 ms; random ASCII equal).
// RtDev::spill_cap_chunks lowers it per object (tests: small launches then
// resolve full regions many times).
// The scratch is sized for RT_SPILL_CAP_CHUNKS, but a launch resolves its
// region at a smaller default fill (round 6, scripts/rt_spillcap_ab.py,
// profiles/r06/spillcap/): a region that fills is resolved inside the
// chunk loop, where the other waves' streaming hides its probes, instead of
// once after it, when every wave of the CU waits at the same time.  Count
// only at 4 chunks: random ASCII 0.434 -> 0.411 ms (the shipped stream
// equal, the lines stream +2.5%, which the auto kind gives to the DFA);
// ids at 2 chunks: the shipped stream 11.39 -> 10.07 ms, the lines stream
// 15.93 -> 13.90, random ASCII equal.
constexpr int64_t RT_SPILL_CAP_CHUNKS = 16;
constexpr int64_t RT_SPILL_FILL_COUNT = 4, RT_SPILL_FILL_IDS = 2;
static int64_t rt_wave_cap(int64_t cap_chunks, int outw = -1) {
    const int64_t dflt = outw < 0 ? RT_SPILL_CAP_CHUNKS : outw == 0 ? RT_SPILL_FILL_COUNT : RT_SPILL_FILL_IDS;
    return (cap_chunks >= 1 && cap_chunks < RT_SPILL_CAP_CHUNKS ? cap_chunks : dflt) * RT_CHUNK;
}
static int64_t rt_spill_stride(int64_t n, int64_t blocks, int64_t wave_cap) {
    const int64_t nw = blocks * RT_WAVES;
    const int64_t natural = ((n / RT_CHUNK + nw - 1) / nw) * RT_CHUNK;
    return natural < wave_cap ? natural : wave_cap;
}

hipError_t pm_launch_gather_probe(const uint32_t* table, uint32_t words, int steps, uint32_t* sink, int num_cu,
                                  hipStream_t s) {
    if (!table || words == 0 || steps <= 0 || num_cu <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(gather_probe_kernel, dim3((unsigned)num_cu), dim3(1024), 0, s, table, words, steps, sink);
    return hipGetLastError();
}

int64_t pm_rt_spill_items(int64_t n, int num_cu, int64_t cap_chunks) {
    constexpr int64_t PIECE = (int64_t)RT_POSMASK + 1;
    const int64_t m = n > PIECE ? PIECE : n;
    const int64_t blocks = rt_blocks(m, num_cu);
    return blocks * RT_WAVES * rt_spill_stride(m, blocks, rt_wave_cap(cap_chunks));
}

static hipError_t launch_rt_impl(bool floor, const uint8_t* text, int64_t stream_start, int64_t pos0, int64_t n,
                                 void* out, int outw, unsigned long long* count, const RtDev& t0, int num_cu,
                                 hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (!out) outw = 0;
    if (outw != 0 && outw != 2 && outw != 4) return hipErrorInvalidValue;
    // queued positions are kept as 30-bit offsets from pos0: split huge scans
    constexpr int64_t PIECE = (int64_t)RT_POSMASK + 1;
    if (n > PIECE) {
        for (int64_t off = 0; off < n; off += PIECE) {
            const int64_t m = n - off < PIECE ? n - off : PIECE;
            void* o = outw ? reinterpret_cast<uint8_t*>(out) + off * outw : nullptr;
            hipError_t e = launch_rt_impl(floor, text, stream_start, pos0 + off, m, o, outw, count, t0, num_cu, s);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    const int64_t small_max = t0.small_max >= 0 ? t0.small_max : RT_SMALL_MAX;
    if (!floor && n <= small_max) {  // small launch: one thread per position
        const dim3 gs((unsigned)((n + RT_SMALL_THREADS - 1) / RT_SMALL_THREADS)), bs(RT_SMALL_THREADS);
        if (outw == 4) hipLaunchKernelGGL((rt_small_kernel<4>), gs, bs, 0, s, text, stream_start, pos0, n, out, count, t0);
        else if (outw == 2) hipLaunchKernelGGL((rt_small_kernel<2>), gs, bs, 0, s, text, stream_start, pos0, n, out, count, t0);
        else hipLaunchKernelGGL((rt_small_kernel<0>), gs, bs, 0, s, text, stream_start, pos0, n, out, count, t0);
        return hipGetLastError();
    }
    const int64_t blocks = rt_blocks(n, num_cu);
    RtDev t = t0;
    t.spill_stride = rt_spill_stride(n, blocks, rt_wave_cap(t0.spill_cap_chunks, out ? outw : 0));
    // The caller sizes the scratch (pm_rt_spill_items); a launch whose
    // scratch holds less than the stride clamps it to whole chunks, at least
    // one (the kernel resolves a full region and goes on, so any stride of
    // >= one chunk is exact).
    const int64_t fit = t.spill_cap / (blocks * RT_WAVES) / RT_CHUNK * RT_CHUNK;
    if (t.spill_stride > fit) {
        if (fit < RT_CHUNK) return hipErrorInvalidValue;  // scratch smaller than one chunk per wave
        t.spill_stride = fit;
    }
    const dim3 g((unsigned)blocks), b(RT_THREADS);
    // early prefetch (EF) for u16 ids and count only (0.864 -> 0.847 ms,
    // 0.565 -> 0.547); u32 ids would spill (1.166 -> 1.216)
    if (floor) {
        if (outw == 4) hipLaunchKernelGGL((rt_scan_kernel<2, 4>), g, b, 0, s, text, stream_start, pos0, n, out, count, t);
        else if (outw == 2) hipLaunchKernelGGL((rt_scan_kernel<2, 2>), g, b, 0, s, text, stream_start, pos0, n, out, count, t);
        else hipLaunchKernelGGL((rt_scan_kernel<2, 0>), g, b, 0, s, text, stream_start, pos0, n, out, count, t);
    } else if (outw == 4) {
        hipLaunchKernelGGL((rt_scan_kernel<0, 4>), g, b, 0, s, text, stream_start, pos0, n, out, count, t);
    } else if (outw == 2) {
        hipLaunchKernelGGL((rt_scan_kernel<0, 2, true>), g, b, 0, s, text, stream_start, pos0, n, out, count, t);
    } else {
        hipLaunchKernelGGL((rt_scan_kernel<0, 0, true>), g, b, 0, s, text, stream_start, pos0, n, out, count, t);
    }
    return hipGetLastError();
}

hipError_t pm_launch_rt(const uint8_t* text, int64_t stream_start, int64_t pos0, int64_t n, void* out, int outw,
                        unsigned long long* count, const RtDev& t, int num_cu, hipStream_t s) {
    return launch_rt_impl(false, text, stream_start, pos0, n, out, outw, count, t, num_cu, s);
}

hipError_t pm_launch_rt_serve(PmServeReq* req, uint64_t* fwd, uint32_t* done, int blocks, uint64_t seen,
                              uint64_t gen, int64_t idle_ticks, const RtDev& t, hipStream_t s) {
    if (blocks <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(rt_serve_kernel, dim3((unsigned)blocks), dim3(RT_SERVE_THREADS), 0, s, req, fwd, done, seen,
                       gen, idle_ticks, t);
    return hipGetLastError();
}

hipError_t pm_launch_rt_floor(const uint8_t* text, int64_t n, void* out, int outw, const RtDev& t, int num_cu,
                              hipStream_t s) {
    return launch_rt_impl(true, text, 0, 0, n, out, outw, nullptr, t, num_cu, s);
}

// ---- DFA launches ----------------------------------------------------------
// Dense rows (dfa_coded_kernel): 512 lanes per CU, two chains per lane in
// lock step (two gathers in flight), 32-position blocks with ids (one whole
// 128-B line of u32 ids per lane and chain: shipped stream 4.32 -> 3.84 ms,
// ASCII 6.58 -> 5.93, lines 20.5 -> 19.8; u16 5.23 -> 4.30 / 6.40 -> 5.58 /
// 19.8 -> 19.3; profiles/r02/dfa_dense_block_sweep.txt), 1,024 lanes per CU
// for count only once warm-ups start at a synchronizing 3-gram (shipped
// 3.28 -> 2.47 ms, ASCII 4.04 -> 4.10; profiles/r03/dfa_sync_lanes.txt).
// More lanes measured slower: the gathers then touch more distinct table
// lines than the caches hold.  The uncoded kernel (automata of 2^20 states
// or more): one chain per lane.
constexpr int DFA_LANES_PER_CU = 512, DFA_COUNT_LANES_PER_CU = 1024, DFA_CHAINS = 2, DFA_DENSE_BLK = 32;
#ifndef PM_DFA_SMALL_SEG
#define PM_DFA_SMALL_SEG 32  // shortest segment of a launch below 1 Mi positions (64: round 5)
#endif
// The sparse form: 1,024 lanes per CU (two 512-lane lock-step workgroups,
// or one 1,024-lane staged workgroup), one chain per lane, 32-position
// blocks (MEASUREMENTS.md §4, profiles/r03/sdfa_lanes_*.txt, sdfa_occupancy_sweep.txt:
// past 1,024 lanes per CU every stream slows down).
constexpr int SDFA_LANES_PER_CU = 1024, SDFA_BLK = 32;
// Shortest segment: a launch of fewer segments than lanes is latency-bound
// (each lane's chain of warm-up + segment steps is the launch time), so
// short launches take short segments, n / 65536 clamped to [64, 512] bytes
// (against the round-1 fixed 2 KiB: 100 KiB 0.34 -> 0.07 ms, 1 MiB 0.62 ->
// 0.07, 16 MiB 0.76-0.86 -> 0.28-0.37, 64 MiB 1.06-1.43 -> 0.59-0.73;
// scripts/dfa_seg_sweep.py, profiles/r02/dfa_segment_sweep.txt).
//
// Product kernels of the sparse form (DfaDev::sparse_kernel 0; side by side
// histories in MEASUREMENTS.md): the fallback-linked form (dfa_fl_kernel,
// PM_SK_FL) at every width -- u32 / u16 ids staged in LDS, or the count
// alone -- where the object has it (< 65,536 rows and gids); else the
// lock-step kernel over 8-B units (PM_SK_LOCK8), and without 8-B units (ids
// past 2^20) the lock-step kernel over the 16-B records (PM_SK_LOCK16).
// A forced kernel (DfaDev::sparse_kernel; tests, A/B timing) runs where the
// object has its image; other launches take the product choice
// (pm_dfa_sparse_choice reports which ran, pm_hip_sparse_kernel_last).
int pm_dfa_sparse_choice(const DfaDev& t, int outw) {
    (void)outw;  // every sparse kernel writes every width
    if (!(t.coded && t.sbase && t.form != 1)) return 0;
    const int sk = t.sparse_kernel;
    const bool ok = sk == PM_SK_FL ? t.flbase != nullptr : sk == PM_SK_LOCK8 ? t.sbase8 != nullptr : sk == PM_SK_LOCK16;
    if (ok) return sk;
    if (t.flbase) return PM_SK_FL;
    return t.sbase8 ? PM_SK_LOCK8 : PM_SK_LOCK16;
}

hipError_t pm_launch_dfa(const uint8_t* text, int64_t stream_start, int64_t pos0, int64_t n, void* out, int outw,
                         unsigned long long* count, const DfaDev& t, int num_cu, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (!out) outw = 0;
    if (outw != 0 && outw != 2 && outw != 4) return hipErrorInvalidValue;
    const uint32_t* g3 = t.sync ? t.gram3 : nullptr;  // warm-ups from synchronizing 3-grams
    const int sk = pm_dfa_sparse_choice(t, outw);
    const bool sparse = sk != 0;
    // segments: one per lane and chain, none shorter than short_seg, whole
    // blocks
    const bool fl2 = sk == PM_SK_FL && t.flchains == 2;  // dfa_fl2_kernel: two chains per lane
    const int64_t ch = !t.coded ? 1 : sparse ? (fl2 ? 2 : 1) : DFA_CHAINS;
    const int lanes_cu = sparse ? (fl2 ? FL2_THREADS : SDFA_LANES_PER_CU)
                                : t.coded && outw == 0 ? DFA_COUNT_LANES_PER_CU : DFA_LANES_PER_CU;
    const int64_t lanes = (int64_t)num_cu * lanes_cu;
    int64_t seg = (n + lanes * ch - 1) / (lanes * ch);
    // (launches below 1 Mi positions -- read_block's 100 KiB calls -- take
    // 32-position segments: twice the lanes, half the dependent steps each)
    const int64_t short_seg = std::min<int64_t>(512, std::max<int64_t>(n < (1 << 20) ? PM_DFA_SMALL_SEG : 64, n >> 16));
    if (seg < short_seg) seg = short_seg;
    const int64_t align = sparse ? SDFA_BLK : t.coded && outw != 0 ? DFA_DENSE_BLK : 16;
    seg = (seg + align - 1) / align * align;
    const int64_t nseg = (n + seg - 1) / seg;
    if (sparse) {
        // persistent workgroups (LDS staged once each), at most one lane per
        // segment and SDFA_LANES_PER_CU lanes per CU
        const int wgt = sk == PM_SK_FL ? (fl2 ? FL2_THREADS : 1024) : DFA_LDS_THREADS;
        int64_t wg = (nseg + wgt * ch - 1) / (wgt * ch);
        const int64_t cap = lanes / wgt;
        if (wg > cap) wg = cap;
        if (wg < 1) wg = 1;
        const dim3 gs((unsigned)wg), bs(wgt);
        switch (sk) {
            case PM_SK_FL:
#define PM_FL_LAUNCH(KR_, W_, NR_)                                                                                  \
    hipLaunchKernelGGL((dfa_fl_kernel<KR_, W_, NR_>), gs, bs, 0, s, text, stream_start, pos0, n, out, count, t.flbase, \
                       t.flF, t.flGD, t.flrowout16, t.warm, seg, g3)
#define PM_FL_WIDTHS(NR_)                                       \
    do {                                                        \
        if (outw == 4) PM_FL_LAUNCH(FL_LDS_ROWS, 4, NR_);       \
        else if (outw == 2) PM_FL_LAUNCH(FL_LDS_ROWS, 2, NR_);  \
        else PM_FL_LAUNCH(FL_COUNT_LDS_ROWS, 0, NR_);           \
    } while (0)
                if (fl2) {  // two chains per lane (NR 1 or 2: the registers of two holds)
#define PM_FL2_LAUNCH(KR_, W_, NR_)                                                                              \
    hipLaunchKernelGGL((dfa_fl2_kernel<KR_, W_, NR_, FL2_THREADS>), gs, bs, 0, s, text, stream_start, pos0, n, out, count, \
                       t.flbase, t.flF, t.flGD, t.flrowout16, t.warm, seg, g3)
                    if (t.flhold == 1) {
                        if (outw == 4) PM_FL2_LAUNCH(FL2_LDS_ROWS, 4, 1);
                        else if (outw == 2) PM_FL2_LAUNCH(FL2_LDS_ROWS, 2, 1);
                        else PM_FL2_LAUNCH(FL_COUNT_LDS_ROWS, 0, 1);
                    } else if (FL2_THREADS < 1024 && t.flhold == 4) {
                        if constexpr (FL2_THREADS < 1024) {  // (the registers for 64-B blocks)
                            if (outw == 4) PM_FL2_LAUNCH(FL2_LDS_ROWS, 4, 4);
                            else if (outw == 2) PM_FL2_LAUNCH(FL2_LDS_ROWS, 2, 4);
                            else PM_FL2_LAUNCH(FL_COUNT_LDS_ROWS, 0, 4);
                        }
                    } else {
                        if (outw == 4) PM_FL2_LAUNCH(FL2_LDS_ROWS, 4, 2);
                        else if (outw == 2) PM_FL2_LAUNCH(FL2_LDS_ROWS, 2, 2);
                        else PM_FL2_LAUNCH(FL_COUNT_LDS_ROWS, 0, 2);
                    }
#undef PM_FL2_LAUNCH
                    break;
                }
                if (t.flhold == 1) PM_FL_WIDTHS(1);  // every record as a 16-B half
                else if (t.flhold == 4) PM_FL_WIDTHS(4);  // 64-B deep blocks
                else PM_FL_WIDTHS(2);
#undef PM_FL_WIDTHS
#undef PM_FL_LAUNCH
                break;
            case PM_SK_LOCK8:  // 8-B units, two blocks' text per load; LDS rows for ids only
                if (outw == 4)
                    hipLaunchKernelGGL((dfa_sparse_lds_kernel<4, 32, 64, 1, 8, 2>), gs, bs, 0, s, text, stream_start,
                                       pos0, n, out, count, t.sbase8, t.sF, t.sout8, t.warm, seg, g3);
                else if (outw == 2)
                    hipLaunchKernelGGL((dfa_sparse_lds_kernel<2, 32, 64, 1, 8, 2>), gs, bs, 0, s, text, stream_start,
                                       pos0, n, out, count, t.sbase8, t.sF, t.sout8, t.warm, seg, g3);
                else
                    hipLaunchKernelGGL((dfa_sparse_lds_kernel<0, 32, 0, 1, 8, 2>), gs, bs, 0, s, text, stream_start,
                                       pos0, n, out, count, t.sbase8, t.sF, t.sout8, t.warm, seg, g3);
                break;
            default:  // PM_SK_LOCK16: the 16-B records, register record blocks (no warm-up shortcut)
                if (outw == 4)
                    hipLaunchKernelGGL((dfa_sparse_lds_kernel<4, 32, 0, 1, 16, 1>), gs, bs, 0, s, text, stream_start,
                                       pos0, n, out, count, t.sbase, t.sF, t.sout, t.warm, seg, (const uint32_t*)nullptr);
                else if (outw == 2)
                    hipLaunchKernelGGL((dfa_sparse_lds_kernel<2, 32, 0, 1, 16, 1>), gs, bs, 0, s, text, stream_start,
                                       pos0, n, out, count, t.sbase, t.sF, t.sout, t.warm, seg, (const uint32_t*)nullptr);
                else
                    hipLaunchKernelGGL((dfa_sparse_lds_kernel<0, 32, 0, 1, 16, 1>), gs, bs, 0, s, text, stream_start,
                                       pos0, n, out, count, t.sbase, t.sF, t.sout, t.warm, seg, (const uint32_t*)nullptr);
        }
        return hipGetLastError();
    }
    int64_t blocks = (nseg + DFA_THREADS * ch - 1) / (DFA_THREADS * ch);
    if (blocks < 1) blocks = 1;
    const dim3 g((unsigned)blocks), b(DFA_THREADS);
    if (t.coded) {
        if (outw == 4)
            hipLaunchKernelGGL((dfa_coded_kernel<4, 2, 32>), g, b, 0, s, text, stream_start, pos0, n, out, count, t.next,
                               t.out, t.warm, seg, g3);
        else if (outw == 2)
            hipLaunchKernelGGL((dfa_coded_kernel<2, 2, 32>), g, b, 0, s, text, stream_start, pos0, n, out, count, t.next,
                               t.out, t.warm, seg, g3);
        else
            hipLaunchKernelGGL((dfa_coded_kernel<0, 2>), g, b, 0, s, text, stream_start, pos0, n, out, count, t.next,
                               t.out, t.warm, seg, g3);
        return hipGetLastError();
    }
    if (outw == 4)
        hipLaunchKernelGGL(dfa_scan_kernel<4>, g, b, 0, s, text, stream_start, pos0, n, out, count, t, seg);
    else if (outw == 2)
        hipLaunchKernelGGL(dfa_scan_kernel<2>, g, b, 0, s, text, stream_start, pos0, n, out, count, t, seg);
    else
        hipLaunchKernelGGL(dfa_scan_kernel<0>, g, b, 0, s, text, stream_start, pos0, n, out, count, t, seg);
    return hipGetLastError();
}

hipError_t pm_launch_score(const uint32_t* algo, const uint32_t* real, int64_t n, const uint32_t* parent,
                          const uint32_t* depth, unsigned long long* counts, int num_cu, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int64_t blocks = (n / 4 + SCORE_THREADS - 1) / SCORE_THREADS;
    if (blocks > (int64_t)num_cu * 8) blocks = (int64_t)num_cu * 8;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(score_kernel<SCORE_V>, dim3((unsigned)blocks), dim3(SCORE_THREADS), 0, s, algo, real, n, parent,
                       depth, counts);
    return hipGetLastError();
}

hipError_t pm_launch_pattern_counts(const uint32_t* real, int64_t n, const uint32_t* parent, uint32_t n_gids,
                                   unsigned long long* hist, int num_cu, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int64_t blocks = (n / 4 + HIST_THREADS - 1) / HIST_THREADS;
    if (blocks > num_cu) blocks = num_cu;  // one workgroup per CU (LDS-bound)
    if (blocks < 1) blocks = 1;
    for (uint32_t lo = 1; lo < n_gids; lo += HIST_WINDOW) {
        const uint32_t cnt = n_gids - lo < HIST_WINDOW ? n_gids - lo : HIST_WINDOW;
        hipLaunchKernelGGL(hist_kernel<HIST_V>, dim3((unsigned)blocks), dim3(HIST_THREADS), 0, s, real, n, parent,
                           lo, cnt, hist);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t pm_launch_gen_lines(uint8_t* dst, uint64_t n, const uint8_t* pats, const uint32_t* offs, uint32_t npats,
                               uint64_t seed, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (npats == 0) return hipErrorInvalidValue;
    const uint64_t nb = (n + PM_LINES_BLOCK - 1) / PM_LINES_BLOCK;
    uint64_t blocks = (nb + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(gen_lines_kernel, dim3((unsigned)blocks), dim3(256), 0, s, dst, n, pats, offs, npats, seed);
    return hipGetLastError();
}

hipError_t pm_launch_gen(uint8_t* dst, uint64_t offset, uint64_t n, uint64_t seed, int mode, hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(gen_stream_kernel, dim3((unsigned)blocks), dim3(256), 0, s, dst, offset, n, seed, mode);
    return hipGetLastError();
}
