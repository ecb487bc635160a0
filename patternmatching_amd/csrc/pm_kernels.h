// pm_kernels.h -- launchers of the gfx950 scan kernels (pm_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

constexpr size_t RT_SCRATCH_BYTES = 4096;
// RT launches of at most this many positions take the one-thread-per-
// position kernel, which needs no spill scratch (RtDev::small_max
// overrides it per object: 0 = never).
constexpr int64_t RT_SMALL_MAX = (int64_t)256 << 10;

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
    // per-object options (pm_hip_set_option): launches of at most small_max
    // positions run the one-thread-per-position kernel (-1: the default,
    // 256 Ki; 0: never); the spill region per wave in 1,024-position chunks
    // (0: the default 16; smaller: tests resolve full regions many times)
    int64_t small_max = -1;
    int64_t spill_cap_chunks = 0;
};

// Spill items (8 B each) an RT launch over n positions needs in
// RtDev::spill: one per position of each wave's chunks, up to the per-wave
// cap (RtDev::spill_cap_chunks).  Launches of any n reuse one buffer of
// this size for n' <= n.
int64_t pm_rt_spill_items(int64_t n, int num_cu, int64_t cap_chunks);

// Kernels of the sparse DFA form (DfaDev::sparse_kernel; pm_kernels.hip
// pm_dfa_sparse_choice is the product choice).  The u32- and u16-staged
// 8-B-unit kernels of round 4 were retired in round 6 (no default path
// picked them once the FL form existed; MEASUREMENTS.md keeps their numbers).
enum PmSparseKernel {
    PM_SK_PRODUCT = 0,
    PM_SK_FL = 1,      // dfa_fl_kernel: the fallback-linked form (every width)
    PM_SK_LOCK8 = 2,   // dfa_sparse_lds_kernel over 8-B units, lock step (automata without the FL form)
    PM_SK_LOCK16 = 3,  // dfa_sparse_lds_kernel over the 16-B records, lock step (ids past the 8-B units' 2^20)
};

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
    // 2^24-bit set of the 3-byte strings occurring in some pattern (bit
    // t[q] | t[q+1] << 8 | t[q+2] << 16), or null.  A 3-gram outside it is
    // synchronizing: the state after it is the root's over those 3 bytes
    // (every longer suffix would hold the 3-gram), so a segment's warm-up
    // can start at the last one before the segment instead of max_len - 1
    // bytes back.
    const uint32_t* gram3;
    int form;              // 0 = the default (the sparse form when there is one), 1 = dense rows, 2 = sparse
    int sync = 1;          // warm-ups from the last synchronizing 3-gram (0: max_len - 1 bytes back)
    int sparse_kernel = PM_SK_PRODUCT;
    // the fallback-linked form (pm_pack_sparse_fl), or null: the product
    // kernel of the sparse form for u32 ids
    const uint8_t* flbase;
    const uint16_t* flrowout16;
    uint32_t flF;
    uint32_t flGD;  // first deep granule (pm_flatten.h FlImage::deep_g)
    uint32_t flwords;  // 4-B words of the FL image (rows, then records)
    // 16-B registers a lane holds of a deep record's block: 2 (32-B blocks,
    // the default), 4 (64-B blocks) or 1 (every record as a 16-B half,
    // flGD ignored); the auto / ac picks time all three
    int flhold = 2;
    // chains per lane of the FL kernel: 1 = dfa_fl_kernel, 2 = dfa_fl2_kernel
    // (two segments per lane in lock step; record holds of NR 1 or 2)
    int flchains = 1;
};

// Positions [pos0, pos0+n) of text; bytes back to stream_start are context.
// pos0 % 16 == 0.  out: n ids of outw bytes each (4 = u32 gids, 2 = u16
// gids, valid when every gid < 65536), or null; count (u64) may be null.
hipError_t pm_launch_rt(const uint8_t* text, int64_t stream_start, int64_t pos0, int64_t n, void* out, int outw,
                        unsigned long long* count, const RtDev& t, int num_cu, hipStream_t s);
// The RT kernel's streaming floor (rt_scan_kernel<2>: the chunk loop's loads
// and stores, no lookups; its ids are not matches) over text[0, n).
hipError_t pm_launch_rt_floor(const uint8_t* text, int64_t n, void* out, int outw, const RtDev& t, int num_cu,
                              hipStream_t s);
// The gather ceiling of a table of `words` 4-B words (bench.py's live bound
// for the DFA legs): the sparse kernel's launch shape (1,024 lanes per CU),
// each lane chasing `steps` dependent 4-B loads at hashed indices; *sink is
// never written in practice.
hipError_t pm_launch_gather_probe(const uint32_t* table, uint32_t words, int steps, uint32_t* sink, int num_cu,
                                  hipStream_t s);
// The DFA form DfaDev::form names (0: the sparse one when the automaton has
// it), and for the sparse form DfaDev::sparse_kernel (0: the product choice).
hipError_t pm_launch_dfa(const uint8_t* text, int64_t stream_start, int64_t pos0, int64_t n, void* out, int outw,
                         unsigned long long* count, const DfaDev& t, int num_cu, hipStream_t s);
// The sparse kernel (PmSparseKernel) a launch of this width runs, 0 when
// it runs dense rows: the forced DfaDev::sparse_kernel where the object
// and width allow it, else the product choice.
int pm_dfa_sparse_choice(const DfaDev& t, int outw);
// counts[0..4] += success, partial, false_neg, false_pos, all_matches of algo
// against real (n u32 gids each, 16-B aligned); parent/depth: PmParents.
hipError_t pm_launch_score(const uint32_t* algo, const uint32_t* real, int64_t n, const uint32_t* parent,
                          const uint32_t* depth, unsigned long long* counts, int num_cu, hipStream_t s);
// hist[g] (u64, g in 1..n_gids-1) += occurrences of pattern g in the stream
// whose dense answers are real: the suffix chain of every answer.
hipError_t pm_launch_pattern_counts(const uint32_t* real, int64_t n, const uint32_t* parent, uint32_t n_gids,
                                   unsigned long long* hist, int num_cu, hipStream_t s);
// The resident small-call server (rt_serve_kernel): a grid that stays on the
// device between read_block calls and takes each call from a request line
// in host memory instead of a launch.  PmServeReq (one 64-B line) and the
// done flags live in coherent (fine-grained) pinned host memory.  A call:
// the host writes seq, the fields, then seq2 = seq; workgroup 0 polls the
// line (one 64-B read over the link) and copies it to device memory for the
// others; a workgroup takes a request when seq2 is new and equals seq, scans its share of [pos0, pos0 + n) (text and out are
// pinned host buffers) and then writes seq's low 32 bits into done[its
// index].  A workgroup exits when stop equals its grid's generation or when
// no request came for idle_ticks of the 100 MHz real-time counter.
struct alignas(64) PmServeReq {
    uint64_t seq;   // written first ...
    uint64_t stop;  // = the generation of a grid that is to exit
    const uint8_t* text;
    void* out;
    int64_t stream_start, pos0;
    uint64_t n_outw;  // n | out width (4: u32 gids, 2: u16) << 56
    uint64_t seq2;  // ... and last
};
constexpr int RT_SERVE_THREADS = 1024;
// Launch the server grid (`blocks` workgroups) on s: requests after `seen`
// are its work; gen identifies it for stop.  done has `blocks` u32 flags.
// fwd: 64 B of device memory (workgroup 0's copy of the request line).
hipError_t pm_launch_rt_serve(PmServeReq* req, uint64_t* fwd, uint32_t* done, int blocks, uint64_t seen,
                              uint64_t gen, int64_t idle_ticks, const RtDev& t, hipStream_t s);
hipError_t pm_launch_gen(uint8_t* dst, uint64_t offset, uint64_t n, uint64_t seed, int mode, hipStream_t s);
hipError_t pm_launch_gen_lines(uint8_t* dst, uint64_t n, const uint8_t* pats, const uint32_t* offs, uint32_t npats,
                               uint64_t seed, hipStream_t s);
