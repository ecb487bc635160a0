// pm_flatten.h -- host flattener: unique patterns -> HBM table images.
//
// Two images, one per kernel (DESIGN.md §3 gives the byte layouts):
//
//  RtImage  reverse-suffix trie of the patterns (every pattern inserted
//           last byte first).  Walking it backwards from stream position i
//           visits exactly the patterns that end at i; the deepest pattern
//           node on the walk is the answer of read_char at i (the reference's
//           "longest pattern ending here", mps.h:41-42 / mpac.c:318).
//             t12   u16[65536 + 256]  depth<=2 in one lookup (LDS-resident)
//             t3    u32[n2int * 256]  depth-3 step from internal depth-2 nodes
//             b2    u32[n2int]        best pattern on the path to a depth-2 node
//             rec   u32[nrec * 12]    48-B records for nodes of depth >= 3:
//                                     child bitmap[8], child base, best, 8 u8
//                                     prefix popcounts
//  DfaImage the Aho-Corasick automaton of Core/src/mpac.c (goto + BFS
//           failure links + suffix/output links, :147-210) flattened into a
//           dense DFA: next[s*256 + c] and out[s] (gid of the longest pattern
//           that is a suffix of state s, 0 if none), states BFS-numbered.
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
    bool fits = false;   // u16 t12 encoding possible (short patterns and n2int < 32768)
    std::vector<uint16_t> t12;
    std::vector<uint32_t> t3;
    std::vector<uint32_t> b2;
    std::vector<uint32_t> rec;
    uint32_t n2int = 0, nrec = 0, nodes = 0;
    size_t bytes() const {
        return t12.size() * 2 + t3.size() * 4 + b2.size() * 4 + rec.size() * 4;
    }
};

struct DfaImage {
    std::vector<uint32_t> next;  // states * 256
    std::vector<uint32_t> out;   // states
    uint32_t states = 0;
    size_t bytes() const { return next.size() * 4 + out.size() * 4; }
};

// Patterns are given in add_pattern order; duplicates are not expected (the
// host front end de-duplicates) but are tolerated: the first one wins.
PmGidMap pm_assign_gids(const std::vector<std::string>& pats);
RtImage pm_build_rt(const std::vector<std::string>& pats, const PmGidMap& g);
DfaImage pm_build_dfa(const std::vector<std::string>& pats, const PmGidMap& g);

constexpr uint32_t RT_T1_BASE = 65536;   // t12[65536 + c]: lookback of exactly one byte
constexpr uint32_t RT_CONT16 = 0x8000u;  // t12: continue at internal depth-2 node (low 15 bits)
constexpr uint32_t RT_CONT32 = 0x80000000u;  // t3: continue at record (low 31 bits)
constexpr int RT_REC_WORDS = 12;
