// pm_kernels.h -- launchers of the gfx950 scan kernels (pm_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

constexpr size_t RT_SCRATCH_BYTES = 4096;

struct RtDev {
    const uint16_t* t12;   // 65536 + 256 u16; the first 64K staged into LDS per workgroup
    const uint32_t* filt;  // RT_FILTER_WORDS + RT_F2_WORDS u32, staged into LDS per workgroup
    const uint4* t3h;      // 2^t3h_bits entries (pm_flatten.h)
    const uint4* rec;      // nrec 16-B node records
    const uint4* wide;     // 4 quarters {word 2q, word 2q+1, child index, best} per wide node
    uint32_t* scratch;     // RT_SCRATCH_BYTES the kernel may overwrite (stand-in stores)
    uint32_t* spill;       // spill_cap 8-B items: per-wave regions of overflow candidates (scratch)
    int64_t spill_cap;     // items
    int64_t spill_stride;  // items per wave region, set per launch
    unsigned long long* spill_total;  // when set: += items spilled (the auto kernel choice)
    uint32_t t3h_bits;
    uint32_t back;         // max pattern length - 1: the bytes a walk may read before its position
};

// Spill items (8 B each) an RT launch over n positions needs in
// RtDev::spill: one per position of each wave's chunks.  Launches of any n reuse one buffer of
// this size for n' <= n.
int64_t pm_rt_spill_items(int64_t n, int num_cu);
// Tests: the spill region's bound per wave in chunks (>= 1; 0 restores the
// default), so small launches resolve full regions many times.
void pm_rt_set_spill_cap(int chunks);
void pm_rt_set_max_blocks(int b);  // timing sweeps: RT workgroups per launch (0 = one per CU)
void pm_rt_set_small_stage(int on);  // timing: rt_small_kernel stages its text window in LDS (default 0)
void pm_rt_set_small_max(int64_t n);  // launches of <= n positions use rt_small_kernel (0 = never, < 0 = default)

struct DfaDev {
    const uint32_t* next;  // states * 256 (output-coded when coded, pm_flatten.h)
    const uint32_t* out;   // states
    int64_t warm;          // max pattern length - 1
    int coded;             // pm_dfa_coded(states)
    const uint8_t* sbase;  // sparse form (coded only): rows | records block, pm_flatten.h
    const uint32_t* sout;  // states, the sparse numbering
    uint32_t sF;           // states with full rows
    const uint8_t* sbase8;  // the same with 8-B record units (pm_pack_sparse8), or null
    const uint32_t* sout8;  // its ids' outputs
    const uint16_t* sout8h; // the same as u16 when every gid < 65536 (else null)
    // 2^24-bit set of the 3-byte strings occurring in some pattern (bit
    // t[q] | t[q+1] << 8 | t[q+2] << 16), or null.  A 3-gram outside it is
    // synchronizing: the state after it is the root's over those 3 bytes
    // (every longer suffix would hold the 3-gram), so a segment's warm-up
    // can start at the last one before the segment instead of max_len - 1
    // bytes back.
    const uint32_t* gram3;
    int form;              // 0 = the default (pm_dfa_set_sparse), 1 = dense rows, 2 = sparse
};

// Positions [pos0, pos0+n) of text; bytes back to stream_start are context.
// pos0 % 16 == 0.  out: n ids of outw bytes each (4 = u32 gids, 2 = u16
// gids, valid when every gid < 65536), or null; count (u64) may be null.
hipError_t pm_launch_rt(const uint8_t* text, int64_t stream_start, int64_t pos0, int64_t n, void* out, int outw,
                        unsigned long long* count, const RtDev& t, int num_cu, hipStream_t s);
// ablation variants of the RT kernel (timing only; see pm_kernels.hip)
hipError_t pm_launch_rt_variant(int variant, const uint8_t* text, int64_t stream_start, int64_t pos0, int64_t n,
                                void* out, int outw, unsigned long long* count, const RtDev& t, int num_cu,
                                hipStream_t s);
hipError_t pm_launch_dfa(const uint8_t* text, int64_t stream_start, int64_t pos0, int64_t n, void* out, int outw,
                         unsigned long long* count, const DfaDev& t, int num_cu, hipStream_t s);
// launch shape of the DFA kernel (timing sweeps): lanes per CU; <= 0
// restores the default
void pm_dfa_set_shape(int lanes_per_cu);
void pm_dfa_set_chains(int chains);
void pm_dfa_set_min_seg(int min_seg);
// Timing sweeps: force the form of coded automata (1 = sparse, 0 = dense
// rows) for launches whose DfaDev::form is 0; < 0 = no forced form (the
// default form is then the sparse one).
void pm_dfa_set_sparse(int sparse);
bool pm_dfa_forced_form();
void pm_dfa_set_variant(int v);  // timing experiments of the sparse kernel (u32 ids, one chain)
void pm_dfa_set_block(int blk);  // sparse form, one chain: positions per block (16 or 32)
// sparse form's kernel (timing; pm_hip_debug_dfa_lds)
void pm_dfa_set_lds(int v);
void pm_dfa_set_sync(int on);  // warm-ups from synchronizing 3-grams (timing; default on)
bool pm_dfa_default_sparse();  // the form a launch with DfaDev::form 0 runs
// counts[0..4] += success, partial, false_neg, false_pos, all_matches of algo
// against real (n u32 gids each, 16-B aligned); parent/depth: PmParents.
hipError_t pm_launch_score(const uint32_t* algo, const uint32_t* real, int64_t n, const uint32_t* parent,
                          const uint32_t* depth, unsigned long long* counts, int num_cu, hipStream_t s);
// hist[g] (u64, g in 1..n_gids-1) += occurrences of pattern g in the stream
// whose dense answers are real: the suffix chain of every answer.
hipError_t pm_launch_pattern_counts(const uint32_t* real, int64_t n, const uint32_t* parent, uint32_t n_gids,
                                   unsigned long long* hist, int num_cu, hipStream_t s);
hipError_t pm_launch_gen(uint8_t* dst, uint64_t offset, uint64_t n, uint64_t seed, int mode, hipStream_t s);
hipError_t pm_launch_gen_lines(uint8_t* dst, uint64_t n, const uint8_t* pats, const uint32_t* offs, uint32_t npats,
                               uint64_t seed, hipStream_t s);
