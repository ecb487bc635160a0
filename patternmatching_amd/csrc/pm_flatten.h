// pm_flatten.h -- host flattener: unique patterns -> HBM table images.
//
// Two images, one per kernel (DESIGN.md §3 gives the byte layouts):
//
//  RtImage  reverse-suffix trie of the patterns (every pattern inserted
//           last byte first).  Walking it backwards from stream position i
//           visits exactly the patterns that end at i; the deepest pattern
//           node on the walk is the answer of read_char at i (the reference's
//           "longest pattern ending here", mps.h:41-42 / mpac.c:318).
//             t12   u16[65536 + 256]  depth<=2 in one lookup (first 64K
//                                     LDS-resident): best pattern so far, bit
//                                     15 set when the depth-2 node has children
//             filt  u32[RT_FILTER_WORDS + RT_F2_WORDS], LDS-resident:
//                   stage 1: blocked Bloom filter (3 bits per key) of the
//                     3-byte suffixes that are depth-3 nodes (every
//                     position under a depth-2 node with children tests it);
//                   stage 2 (only queued stage-1 candidates test it): the
//                     3-byte suffixes that are patterns (RT_F3_WORDS) and
//                     the 4-byte suffixes that are depth-4 nodes
//                     (RT_F4_WORDS).  A position failing stage 2 has no
//                     pattern at depth >= 3 on its walk, so its answer is
//                     the depth-2 one and it needs no probe.
//                   No false negatives in either stage.
//             t3h   u32x4[2^k]        open-addressing table of those suffixes
//                                     (two-choice cuckoo, load <= 1/4), one 16-B entry per
//                                     depth-3 node n3 that decides depth 4 too:
//                                       x = kind << 25 | valid << 24 | key24
//                                           (kind 0: n3 has no children,
//                                            1: one to three children,
//                                            2: more)
//                                       y = best pattern on the path to n3
//                                       z = kind 1: child bytes (byte k =
//                                           child k, sorted) | count << 24
//                                       w = kind 1, one child: the child's
//                                           answer (gid, or RT_CONT32 | its
//                                           record); several: the record of
//                                           the first child (children are
//                                           contiguous);
//                                           kind 2: RT_CONT32 | n3's record
//             rec   u32x4[nrec]       16-B records for nodes of depth >= 3
//                                     (BFS to depth 3, then depth-first
//                                     child blocks; children contiguous):
//                                       x = kind << 30 | count << 24 | first
//                                           (kind RT_REC_LEAF: no children;
//                                            RT_REC_CHAIN: one child, and
//                                            count = the bytes of its run in
//                                            z, w (below, RT_REC_CHAIN);
//                                            RT_REC_KIDS: count <= 8 children,
//                                            their bytes in z, w (byte j =
//                                            child j, sorted), child j at
//                                            record first + j;
//                                            RT_REC_WIDE: more children, z =
//                                            its `wide` entry)
//                                       y = best pattern on the path to the node
//             wide  u32[nwide * 16]   per wide node, 4 quarters of 16 B; quarter
//                                     q = {bitmap word 2q, bitmap word 2q+1,
//                                     first + children before word 2q, best}:
//                                     one 16-B load decides a byte (child of
//                                     byte c at that index + rank of c in the
//                                     quarter's words)
//  DfaImage the Aho-Corasick automaton of Core/src/mpac.c (goto + BFS
//           failure links + suffix/output links, :147-210) flattened into a
//           dense DFA: next[s*256 + c] and out[s] (gid of the longest pattern
//           that is a suffix of state s, 0 if none), states numbered
//           breadth-first to PM_DFA_DFS_DEPTH, depth-first below;
//           below 2^20 states next also carries the target's output code
//           (pm_dfa_coded, below).
//
// Pattern ids: gid 1..P, short patterns (length <= 2) first so that every
// depth<=2 answer fits the 15-bit payload of a t12 entry.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

struct PmGidMap {
    std::vector<uint32_t> index_of_gid;  // [0] unused; gid -> pattern index (add order)
    std::vector<uint32_t> gid_of_index;  // pattern index -> gid
};

struct RtImage {
    // encodings fit: fewer than 32768 patterns of length <= 2 (u16 t12),
    // records < 2^23 and patterns < 512 bytes (a queued record step holds
    // record | depth << 23)
    bool fits = false;
    std::vector<uint16_t> t12;
    std::vector<uint32_t> filt;
    std::vector<uint32_t> t3h;  // 4 words per entry
    std::vector<uint32_t> rec;   // 4 words per node of depth >= 3
    std::vector<uint32_t> wide;  // RT_WIDE_WORDS per node with > RT_REC_INLINE children
    uint32_t t3h_bits = 0;
    uint32_t n2int = 0, nrec = 0, nodes = 0, d3 = 0, nwide = 0;
    size_t bytes() const {
        return t12.size() * 2 + filt.size() * 4 + t3h.size() * 4 + rec.size() * 4 + wide.size() * 4;
    }
};

// With fewer than 2^20 states (every reference dictionary: merged has
// 716,744) a transition word also carries its target's output: target |
// min(out[target], PM_DFA_ESC) << 20, so a DFA step is one gather and only
// PM_DFA_ESC (gid >= 4095) needs out[].
constexpr uint32_t PM_DFA_STATE_MASK = 0xFFFFFu;
constexpr uint32_t PM_DFA_ESC = 4095u;
inline bool pm_dfa_coded(uint32_t states) { return states <= PM_DFA_STATE_MASK; }

// Sparse (default-transition) form of the same automaton, built only when
// it is output-coded.  A state whose dense row differs from the row of its
// fallback -- the first state with a full row on its failure chain -- in at
// most PM_SDFA_K bytes keeps a 16-B record instead of a 1 KiB row:
//   x = (c0 | 0x100) | (c1 | 0x100) << 16 (a missing slot is 0), y / z =
//   the coded transitions on c0 / c1, w = the fallback's state (< F).
// States are renumbered: full rows [0, F) (the root is 0), records [F, S),
// both in the trie's order (depth-first below PM_DFA_DFS_DEPTH, so a unary
// run of records is consecutive), and every coded word carries the new
// numbering.  The
// device keeps one block `rows (F * 1 KiB) | records ((S - F) * 16 B)`, so a
// step is one 16-B load at offset s * 1024 + (c & ~3) * 4 (row) or F * 1024
// + (s - F) * 16 (record), plus, at a record whose slots miss the byte, one
// 4-B load of row w.  out is indexed by the new numbering.
constexpr uint32_t PM_SDFA_K = 2;
constexpr uint32_t PM_SDFA_REC_WORDS = 4;

struct DfaImage {
    std::vector<uint32_t> next;  // states * 256 (output-coded when pm_dfa_coded(states))
    std::vector<uint32_t> out;   // states
    uint32_t states = 0;
    // sparse form (pm_dfa_coded(states) only; empty otherwise)
    std::vector<uint32_t> sblock;  // F * 256 row words, then (states - F) * 4 record words
    std::vector<uint32_t> sout;    // states, new numbering
    uint32_t sF = 0;
    size_t bytes() const { return next.size() * 4 + out.size() * 4; }
    size_t sparse_bytes() const { return sblock.size() * 4 + sout.size() * 4; }
};

// Pattern suffix relation in gid space (the reference's patterns tree,
// PatternsTree.c:180-217 / 388-397: a pattern's parent is its longest proper
// suffix that is a pattern): parent[g] (0 = none) and depth[g] = the number
// of patterns on g's parent chain including g = how many patterns end at a
// position whose answer is g.  parent[0] = depth[0] = 0.
struct PmParents {
    std::vector<uint32_t> parent, depth;
};

// Patterns are given in add_pattern order.  The host front end de-duplicates
// (PatternsTree.c:193-196), but a plugin caller may repeat a byte string: as
// in ac_add_pattern (mpac.c:272) the id added last wins.
PmGidMap pm_assign_gids(const std::vector<std::string>& pats);
RtImage pm_build_rt(const std::vector<std::string>& pats, const PmGidMap& g);
DfaImage pm_build_dfa(const std::vector<std::string>& pats, const PmGidMap& g);
PmParents pm_build_parents(const std::vector<std::string>& pats, const PmGidMap& g);

// The sparse form with 8-B record units (a device layout, built from the
// 16-B form at compile time; not cached): rows [0, F) as before, then the
// records in the same order, each at a unit offset u with state id F + u:
//   zero or one slot (75% of snort's records): one unit {y, x0 | w << 9},
//     x0 = c0 | 0x100 (0: no slot), w = the fallback row;
//   two slots: two units {y, x | 1 << 31}, {z, w} (x as in the 16-B
//     form), never straddling an aligned 32-B block of 4 units (so neither
//     a 64-B block of 8; a padding unit before it when it would).
// Every coded word's target is renumbered; out8 is indexed by the new ids
// (padding ids 0).  A walk along a pattern's unary run reads twice as many
// states per line as with 16-B records.  False when the new ids do not fit
// the coded word's 20-bit target field.
bool pm_pack_sparse8(const DfaImage& d, std::vector<uint32_t>& block8, std::vector<uint32_t>& out8);

// The fallback-linked ("FL") form of the same automaton (round 5; a device
// layout built from the 16-B form at compile, not cached).  In the 8-B form
// a record's fallback row is inside the record, so a lane that enters a
// record in a block it does not hold waits for the block and then, at a
// slot miss, for the fallback row's word: two dependent loads, and with 64
// lanes in lock step nearly every wave step waits for some lane's pair.
// Here the word that leads INTO a record names its fallback row, so a
// record needs no room for it and carries its own output instead.
//   Rows [0, F): the first PM_FL_LDS_ROWS are staged in LDS by the kernel
//   (the root and, with a profile, the rows its walks visit most, else the
//   shallowest states), the rest are renumbered by how many records fall
//   back to them, so the fallback rows records use most have the smallest
//   ids.
//   Records: in the trie's order, at 8-B granules (state id = F + granule):
//     word0 = out16 | c0 << 16 | c1 << 24   out16 = the record's OWN output
//             (gid < 65536); c1 == c0 for one slot (a slotless record that
//             cannot be folded, below, takes one slot repeating its
//             fallback's transition on byte 0)
//     word1 = the word on c0
//     16-B records (two slots, or a fallback outside the word's range):
//     word2 = the word on c1 (word1 again for one slot), word3 = the
//             fallback row; 16-B aligned.
//   A word (in rows and records): target | f << 20 with
//     target a row: f = min(output of the target, PM_DFA_ESC) (escapes:
//       FlImage::rowout16[target]);
//     target a record: f = its fallback row when that is below
//       PM_FL_FB_INREC, else PM_FL_FB_INREC (the fallback is word3).
//   The output of a position whose state is a record is that record's out16
//   (read with the record at the next step); of a row state, the word's f.
//   A slotless record whose output has an inline code is folded: every word
//   into it names its fallback row instead (with its output as the code) --
//   the same transitions, the same outputs.
// False when it does not apply: 65,536 patterns or rows or more, or ids past
// the 20-bit target field.
constexpr uint32_t PM_FL_FB_INREC = 4095;  // the 12-bit field's top value
constexpr uint32_t PM_FL_LDS_ROWS = 88;  // rows the kernel stages in LDS (dfa_fl_kernel<88>)
constexpr uint32_t PM_FL_COUNT_LDS_ROWS = 156;  // ... its count-only instance (no staging rows)
// Records of trie depth < PM_FL_DEEP_DEPTH come first (the kernel loads
// them as 16-B halves: a walk rarely stays), then, from granule deep_g (a
// multiple of 8), the deeper ones (loaded as aligned 32-B blocks: a walk
// that got this deep is usually on a pattern's unary run, whose records
// follow each other).  Within each part, the trie's order.
#ifndef PM_FL_DEEP_DEPTH
#define PM_FL_DEEP_DEPTH 4
#endif
struct FlImage {
    std::vector<uint32_t> block;     // F * 256 row words, then 2 words per granule
    std::vector<uint16_t> rowout16;  // output of each row (escapes)
    uint32_t F = 0, granules = 0, folded = 0;
    uint32_t deep_g = 0;             // first granule of the deep records
};
// The profile text of the LDS-row choice: PM_FL_PROFILE_PIECES pieces of
// PM_FL_PROFILE_PIECE bytes, walked from the root each; 15 of 16 are the
// dictionary's own lines text (pm_streamgen.h pm_lines_block, seed 7: its
// patterns drawn at random, '\n' after each), 1 of 16 random printable
// ASCII (pm_stream_byte mode 0).  A function of the pattern list alone.
constexpr size_t PM_FL_PROFILE_PIECES = 64, PM_FL_PROFILE_PIECE = 32 << 10;
std::vector<uint8_t> pm_fl_profile(const std::vector<std::string>& pats);
// With a profile, the LDS rows (the first PM_FL_LDS_ROWS) are the root and
// the rows the profile's walks step from most -- row states and record
// fallbacks -- instead of the root and the shallowest (scripts/
// fl_rowline_model.cpp, snort: lines 0.209 -> 0.188 row and fallback
// requests per step, random ASCII 0.477 -> 0.319).
bool pm_pack_sparse_fl(const DfaImage& d, FlImage& fl, const std::vector<uint8_t>* profile = nullptr);
// One FL step from state s with the word w that led to it (w = 0 at the
// root) on byte c: returns the next word.  *out_prev = the output of the
// position whose step produced w (s's own output when s is a record; w's
// code -- or the escaped row output -- when a row).  Host reference of the
// device kernel (tests; pm_flat_host_scan mode 2).
uint32_t pm_fl_host_step(const FlImage& fl, uint32_t w, uint8_t c, uint32_t* out_prev);
uint32_t pm_fl_output(const FlImage& fl, uint32_t w);  // the output of the position whose step produced w

// Compiled-image cache: the flattened tables of a
// dictionary, on disk, keyed by a hash of the patterns in add order and the
// image kind.  pm_image_key hashes (format version, kind, the layout
// constants and hash functions below, every pattern's length and bytes).  Files are written to a temporary name and renamed, so
// a reader never sees a partial file; anything that does not validate
// (magic, key, kind, section sizes, every index and gid, the cuckoo slots,
// and filters equal to the ones the tables imply) is ignored and rebuilt.
struct PmImages {
    RtImage rt;
    DfaImage dfa;
    PmParents par;
};
uint64_t pm_image_key(const std::vector<std::string>& pats, int kind);
// Build (kind 1 = RT, 2 = DFA; parents always), through the cache directory
// when dir is non-empty.  *hit tells whether the file was used.
PmImages pm_build_images_cached(const std::vector<std::string>& pats, const PmGidMap& g, int kind,
                                const std::string& dir, bool* hit);

constexpr uint32_t RT_T1_BASE = 65536;   // t12[65536 + c]: lookback of exactly one byte
constexpr uint32_t RT_CONT16 = 0x8000u;  // t12: depth-2 node has children (low 15 bits: best so far)
constexpr uint32_t RT_CONT32 = 0x80000000u;  // t3: continue at record (low 31 bits)
constexpr int RT_REC_WORDS = 4;
constexpr uint32_t RT_REC_LEAF = 0, RT_REC_KIDS = 1, RT_REC_CHAIN = 2, RT_REC_WIDE = 3;  // record kinds (x >> 30)
// A one-child node's record is a CHAIN: x = kind | L << 24 | first, y = best,
// and (w << 32 | z) holds the bytes b_0 .. b_{L-1} of its run at bytes 7 ..
// 8-L (b_0, the child's byte, in the top byte of w).  The run: the child is
// record `first`, and for k = 1 .. L-1 record first+k-1 has one child,
// record first+k, reached by b_k, and no pattern ends at it.  A walk may
// consume the m <= L leading bytes that match in one step: it is then at
// record first+m-1, and if it stops there (m < L) the answer is y.
constexpr uint32_t RT_CHAIN_MAX = 8;
constexpr uint32_t RT_REC_INLINE = 8;  // children held inline in a record
constexpr int RT_WIDE_WORDS = 16;
// DFA state numbering: breadth-first to this depth, then children blocks in
// depth-first order (build_trie), so a pattern's deep states are neighbours
// (the dense rows do not care, 1 KiB each; the sparse form's 16-B records do)
#ifndef PM_DFA_DFS_DEPTH
#define PM_DFA_DFS_DEPTH 2u
#endif
inline uint32_t pm_rt_wide_word(uint32_t w) { return 4 * (w >> 1) + (w & 1); }  // bitmap word w in an entry
constexpr uint32_t RT_FILTER_WORDS = 4096;  // stage 1: 16 KiB of LDS
constexpr uint32_t RT_F3_WORDS = 256;       // stage 2, 3-byte patterns: 1 KiB
constexpr uint32_t RT_F4_WORDS = 1792;      // stage 2, depth-4 suffixes: 7 KiB
constexpr uint32_t RT_F2_WORDS = RT_F3_WORDS + RT_F4_WORDS;

// Hashes (host and device must agree).  key24 = text[i-2] | text[i-1] << 8
// | text[i] << 16 (the little-endian u24 ending at i, so the t12 index is
// key24 >> 8).  Filter: f = key24 * 0x9E3779 (mod 2^32; one full-rate 24-bit
// multiply on the device), word f >> 20, bits f, f >> 8 and f >> 16 (& 31:
// byte fields, so the device shifts take them by SDWA byte select).  t3h: a key sits in slot pm_rt_slot1 (h >> (32 -
// t3h_bits), h = key24 * 0x9E3779B1) or pm_rt_slot2.
inline uint32_t pm_rt_hash(uint32_t k) { return k * 0x9E3779B1u; }
inline uint32_t pm_rt_fhash(uint32_t k) { return k * 0x9E3779u; }
inline uint32_t pm_rt_filter_word(uint32_t f) { return f >> 20; }
inline uint32_t pm_rt_filter_mask(uint32_t f) {
    return (1u << (f & 31)) | (1u << ((f >> 8) & 31)) | (1u << ((f >> 16) & 31));
}
// Stage 2 (word indices relative to the stage-2 block, same bit mask):
// 3-byte patterns g = key24 * 0x85EBCA, word g >> 24; depth-4 suffixes
// g = key32 * 0x9E3779B1 with key32 = text[i-3] | key24 << 8, word
// RT_F3_WORDS + ((g >> 20) * 7 >> 4).
inline uint32_t pm_rt_p3hash(uint32_t key24) { return key24 * 0x85EBCAu; }
inline uint32_t pm_rt_p3word(uint32_t g) { return g >> 24; }
inline uint32_t pm_rt_s4hash(uint32_t key32) { return key32 * 0x9E3779B1u; }
inline uint32_t pm_rt_s4word(uint32_t g) { return RT_F3_WORDS + (((g >> 20) * 7u) >> 4); }
constexpr uint32_t RT_T3H_VALID = 1u << 24;
inline uint32_t pm_rt_slot1(uint32_t k, uint32_t bits) { return pm_rt_hash(k) >> (32 - bits); }
inline uint32_t pm_rt_slot2(uint32_t k, uint32_t bits) { return (k * 0x85EBCA77u) >> (32 - bits); }
constexpr uint32_t RT_T3H_INLINE = 3;  // child bytes held in a t3h entry
