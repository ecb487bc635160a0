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
//     depth 3      only when t12 says the depth-2 node has children: a 2-bit
//                  blocked Bloom filter in LDS over the 3-byte suffixes that
//                  exist; a filter hit (about 1.5 % of positions on random
//                  text, no false negatives) is queued;
//     queue        per wave, filled with ballot/mbcnt prefix offsets and
//                  drained by all 64 lanes at once: one probe of an
//                  L2-resident hash table of depth-3 suffixes and, past depth
//                  3, one 48-B bitmap-rank record per step.
//   Each lane owns four groups of four consecutive positions at stride 256,
//   so every load instruction reads 256 contiguous bytes and every store
//   instruction writes 1 KiB of contiguous match ids; the next chunk's bytes
//   are loaded while the current one is resolved.
//
// dfa_scan_kernel the reference automaton itself, flattened to a dense DFA
//   (next[s*256+c], out[s]); one lane per stream segment, started from the
//   root max_len-1 bytes before the segment (SURVEY.md §0.1 shard rule), so
//   every segment is independent and exact.
#include "pm_kernels.h"
#include "pm_streamgen.h"

namespace {

constexpr int RT_THREADS = 1024;
constexpr int RT_WAVES = RT_THREADS / 64;
constexpr int RT_T2_U16 = 65536;
constexpr int RT_FILTER_WORDS = 6144;  // must match pm_flatten.h
constexpr int RT_QCAP = 64;            // queue items per wave (one per lane per round)
constexpr uint32_t RT_QFLUSH = 40;     // resolve once this many are queued
constexpr int RT_CHUNK = 1024;         // positions per wave iteration
constexpr uint32_t CONT16 = 0x8000u;
constexpr uint32_t CONT32 = 0x80000000u;
constexpr uint32_t T3H_VALID = 1u << 24;

__device__ __forceinline__ uint32_t rt_hash(uint32_t k) { return k * 0x9E3779B1u; }  // pm_rt_hash
__device__ __forceinline__ uint32_t rt_fmask(uint32_t h) { return (1u << ((h >> 4) & 31)) | (1u << ((h >> 9) & 31)); }

__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

__device__ __forceinline__ uint32_t wave_prefix(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Record walk.  `node` is a record reached after consuming text[i] ..
// text[i-d+1]; avail = bytes that exist at or before i.
// Each step loads the whole record and the next byte together.
__device__ __forceinline__ uint32_t rt_deep(const uint8_t* __restrict__ text, const uint32_t* __restrict__ rec,
                                            uint32_t node, int64_t i, int64_t avail, int64_t d) {
    for (;;) {
        const uint32_t* R = rec + (size_t)node * 12;
        const uint4 meta = *reinterpret_cast<const uint4*>(R + 8);  // {base, best, prefix}
        if (d >= avail) return meta.y;
        const uint32_t c = text[i - d];
        const uint32_t w = c >> 5, bit = c & 31u;
        const uint32_t word = R[w];
        if (!((word >> bit) & 1u)) return meta.y;
        const uint32_t pre = ((w < 4 ? meta.z : meta.w) >> (8 * (w & 3))) & 0xFFu;
        node = meta.x + pre + __popc(word & ((1u << bit) - 1u));
        ++d;
    }
}

// The walk past depth 2 from key24 = text[i-2] | text[i-1] << 8 | text[i] << 16
// (a depth-2 node with children) with c3 = text[i-3] when avail >= 4;
// best2 = the answer if it stops at depth 2.  One probe of t3h decides
// depth 3 and, for nodes with at most one child, depth 4.
__device__ __forceinline__ uint32_t rt_from_d2(const uint8_t* __restrict__ text, const RtDev& t, uint32_t key24,
                                               uint32_t c3, uint32_t best2, int64_t i, int64_t avail) {
    const uint32_t mask = (1u << t.t3h_bits) - 1u;
    uint32_t slot = rt_hash(key24) >> (32 - t.t3h_bits);
    uint4 e;
    for (;;) {
        e = t.t3h[slot];
        if (!(e.x & T3H_VALID)) return best2;
        if ((e.x & 0xFFFFFFu) == key24) break;
        slot = (slot + 1) & mask;
    }
    const uint32_t kind = e.x >> 25;
    if (kind == 0 || avail < 4) return e.y;
    if (kind == 1) {
        if (c3 != e.z) return e.y;
        if (!(e.w & CONT32)) return e.w;
        return rt_deep(text, t.rec, e.w & 0x7FFFFFFFu, i, avail, 4);
    }
    return rt_deep(text, t.rec, e.w & 0x7FFFFFFFu, i, avail, 3);
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
//   9 = product kernel with s_memtime stamps per phase (diagnostic: count
//       receives 8 u64 cycle sums: lds+filter, push, resolve, pull, store,
//       rounds, chunks, total)
template <int V>
__global__ __launch_bounds__(RT_THREADS) void rt_scan_kernel(const uint8_t* __restrict__ text, int64_t stream_start,
                                                             int64_t pos0, int64_t n, uint32_t* __restrict__ out,
                                                             unsigned long long* __restrict__ count, RtDev t) {
    __shared__ __attribute__((aligned(16))) uint16_t s_t[RT_T2_U16];
    __shared__ __attribute__((aligned(16))) uint32_t s_f[RT_FILTER_WORDS];
    __shared__ uint32_t s_qkey[RT_WAVES][RT_QCAP];  // key24 | text[i-3] << 24
    __shared__ uint32_t s_qpos[RT_WAVES][RT_QCAP];  // position - pos0
    {
        const uint4* src = reinterpret_cast<const uint4*>(t.t12);
        uint4* dst = reinterpret_cast<uint4*>(s_t);
        for (int k = threadIdx.x; k < RT_T2_U16 * 2 / 16; k += RT_THREADS) dst[k] = src[k];
        const uint4* fsrc = reinterpret_cast<const uint4*>(t.filt);
        uint4* fdst = reinterpret_cast<uint4*>(s_f);
        for (int k = threadIdx.x; k < RT_FILTER_WORDS / 4; k += RT_THREADS) fdst[k] = fsrc[k];
    }
    __syncthreads();

    const int lane = threadIdx.x & 63;
    // wave id through readfirstlane: the compiler then knows every per-chunk
    // quantity below is wave-uniform (scalar loop, no exec-mask loop)
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t* qkey = s_qkey[wid];
    uint32_t* qpos = s_qpos[wid];
    uint32_t cnt = 0;
    uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tA = 0, tB = 0;
    if (V == 9) tA = stamp();
    const int64_t nchunks = (n + RT_CHUNK - 1) / RT_CHUNK;
    const int64_t stride = (int64_t)gridDim.x * RT_WAVES;
    // a chunk is "fast" when all of it (and the 4 bytes before it) is in range
    // and it starts >= 2 bytes into the stream
    auto is_fast = [&](int64_t c) {
        const int64_t pc = pos0 + c * RT_CHUNK;
        return c < nchunks && pc + RT_CHUNK <= pos0 + n && pc - stream_start >= 2;
    };
    using u32x2 = __attribute__((ext_vector_type(2))) unsigned int;
    using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;
    // Queued positions carry over chunks; a round resolves the queue once it
    // holds RT_QFLUSH items (or is full), so one round's latency is shared by
    // several chunks.  Each chunk is stored before its positions can be
    // resolved: a round's probes are issued after those stores and waited
    // for, and vmcnt counts loads and stores in one in-order queue, so every
    // store is complete at L2 before a patch overwrites one of its
    // placeholders (a line this CU wrote a few chunks ago, still in L2).
    uint32_t qn = 0;  // items queued (wave-uniform)
    auto flush = [&]() {
        __builtin_amdgcn_wave_barrier();
        if (V == 9) { const uint64_t u = stamp(); ph[1] += u - tB; tB = u; ph[5] += 1; }
        if ((uint32_t)lane < qn) {
            const uint32_t qk = qkey[lane];
            const uint32_t k = qk & 0xFFFFFFu;
            const int64_t i = pos0 + (int64_t)qpos[lane];
            const uint32_t best2 = s_t[k >> 8] & 0x7FFFu;
            const uint32_t v = rt_from_d2(text, t, k, qk >> 24, best2, i, i - stream_start + 1);
            cnt += (uint32_t)(v != 0u) - (uint32_t)(best2 != 0u);
            if (out && v != best2) out[i - pos0] = v;
        }
        __builtin_amdgcn_wave_barrier();
        if (V == 9) { const uint64_t u = stamp(); ph[2] += u - tB; tB = u; }
        qn = 0;
    };
    // text is prefetched two chunks ahead; streamed bytes and ids are non-temporal
    int64_t ch = (int64_t)blockIdx.x * RT_WAVES + wid;
    u32x2 nx[4] = {}, nnx[4] = {};
    bool nfast = is_fast(ch), nnfast = is_fast(ch + stride);
    if (nfast) {
        const uint8_t* src = text + pos0 + ch * RT_CHUNK + 4 * lane - 4;
#pragma unroll
        for (int s = 0; s < 4; ++s) nx[s] = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(src + 256 * s));
    }
    if (nnfast) {
        const uint8_t* src = text + pos0 + (ch + stride) * RT_CHUNK + 4 * lane - 4;
#pragma unroll
        for (int s = 0; s < 4; ++s) nnx[s] = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(src + 256 * s));
    }
    for (; ch < nchunks; ch += stride) {  // wave-uniform
        const int64_t pc = pos0 + ch * RT_CHUNK;
        const bool fast = nfast;
        const u32x2 x[4] = {nx[0], nx[1], nx[2], nx[3]};
#pragma unroll
        for (int s = 0; s < 4; ++s) nx[s] = nnx[s];
        nfast = nnfast;
        nnfast = is_fast(ch + 2 * stride);
        if (nnfast) {  // prefetch two chunks ahead
            const uint8_t* src = text + pc + 2 * stride * RT_CHUNK + 4 * lane - 4;
#pragma unroll
            for (int s = 0; s < 4; ++s) nnx[s] = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(src + 256 * s));
        }
        if (!fast) continue;  // stream start / tail: handled after the loop
        if (V == 9) { tB = stamp(); ph[6] += 1; }
        // position j = 4s + b of this lane is pc + 256s + 4*lane + b; its key
        // is the LE u24 ending at byte b of x[s].y (bytes i-2, i-1, i)
#define RT_KEY(j) ((uint32_t)((((uint64_t)x[(j) >> 2].y << 32) | x[(j) >> 2].x) >> (8 * (2 + ((j) & 3)))) & 0xFFFFFFu)
        uint32_t r[16];
        uint32_t cm = 0;  // bit j: position j goes past depth 2
#pragma unroll
        for (int j = 0; j < 16; ++j) r[j] = V == 2 ? RT_KEY(j) & 0xFFFFu : s_t[RT_KEY(j) >> 8];
        if (V == 0 || V == 9) {
            uint32_t fw[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) fw[j] = s_f[__umulhi(rt_hash(RT_KEY(j)), (uint32_t)RT_FILTER_WORDS)];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t m = rt_fmask(rt_hash(RT_KEY(j)));
                cm |= (((r[j] >> 15) & 1u) & (uint32_t)((fw[j] & m) == m)) << j;
            }
        }
#undef RT_KEY
#pragma unroll
        for (int j = 0; j < 16; ++j) r[j] &= 0x7FFFu;
        if (V == 9) { const uint64_t u = stamp(); ph[0] += u - tB; tB = u; }
        // store the chunk: depth<=2 answers, queued positions patched by flush()
        if (out) {
            uint4* o = reinterpret_cast<uint4*>(out + (pc - pos0));
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                u32x4 v = {r[4 * s], r[4 * s + 1], r[4 * s + 2], r[4 * s + 3]};
                __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(o + 64 * s + lane));
            }
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) cnt += r[j] != 0u;
        asm volatile("" ::: "memory");  // the store stays ahead of any later probe
        if (V == 9) { const uint64_t u = stamp(); ph[4] += u - tB; tB = u; }
        if (V == 0 || V == 9) {
            // lane count c = popc(cm); exclusive wave prefix from five ballots
            // (one per bit of c); items written by a loop over own set bits
            const uint32_t c = __popc(cm);
            uint32_t base = 0, total = 0;
#pragma unroll
            for (int b = 0; b < 5; ++b) {
                const uint64_t mb = __ballot((c >> b) & 1u);
                base += wave_prefix(mb) << b;
                total += (uint32_t)__popcll(mb) << b;
            }
            for (uint32_t done = 0;;) {  // wave-uniform
                uint32_t mm = cm, rank = base;
                while (mm) {
                    const uint32_t j = __builtin_ctz(mm);
                    mm &= mm - 1;
                    const uint32_t slot = qn + rank - done;
                    if (rank >= done && slot < RT_QCAP) {
                        const uint32_t sg = j >> 2, b = j & 3;
                        const uint32_t lo = sg == 0 ? x[0].x : sg == 1 ? x[1].x : sg == 2 ? x[2].x : x[3].x;
                        const uint32_t hi = sg == 0 ? x[0].y : sg == 1 ? x[1].y : sg == 2 ? x[2].y : x[3].y;
                        const uint64_t win = ((uint64_t)hi << 32) | lo;
                        qkey[slot] = ((uint32_t)(win >> (8 * (2 + b))) & 0xFFFFFFu) |
                                     (((uint32_t)(win >> (8 * (1 + b))) & 0xFFu) << 24);
                        qpos[slot] = (uint32_t)(pc - pos0) + 256 * sg + 4 * lane + b;
                    }
                    ++rank;
                }
                const uint32_t took = (total - done < RT_QCAP - qn) ? total - done : RT_QCAP - qn;
                qn += took;
                done += took;
                if (qn < RT_QFLUSH && done == total) break;
                flush();
                if (done == total) break;
            }
        }
    }
    if (V == 0 || V == 9) {
        if (qn) flush();
    }
    if (V == 9) {
        ph[7] = stamp() - tA;
        if (lane == 0 && count)
            for (int k = 0; k < 8; ++k) atomicAdd(count + k, (unsigned long long)ph[k]);
        return;
    }
    // the (at most two) chunks that touch the stream start or the tail, one
    // position at a time; kept out of the main loop to keep it lean
    for (int64_t c = (int64_t)blockIdx.x * RT_WAVES + wid; c < nchunks; c += stride) {
        if (is_fast(c)) continue;
        const int64_t pc = pos0 + c * RT_CHUNK;
#pragma unroll 1
        for (int s = 0; s < 4; ++s) {
            const int64_t p = pc + 256 * s + 4 * lane;
#pragma unroll 1
            for (int b = 0; b < 4; ++b) {
                if (p + b < pos0 + n) {
                    const uint32_t v = rt_one(text, s_t, t, p + b, stream_start);
                    if (out) out[p + b - pos0] = v;
                    cnt += v != 0u;
                }
            }
        }
    }
    if (count) {
        for (int o = 32; o > 0; o >>= 1) cnt += __shfl_down(cnt, o);
        if (lane == 0 && cnt) atomicAdd(count, (unsigned long long)cnt);
    }
}

constexpr int DFA_THREADS = 256;

__global__ __launch_bounds__(DFA_THREADS) void dfa_scan_kernel(const uint8_t* __restrict__ text, int64_t stream_start,
                                                               int64_t pos0, int64_t n, uint32_t* __restrict__ out,
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
            if (out) {
                uint4* o = reinterpret_cast<uint4*>(out + (i - pos0));
                o[0] = make_uint4(r[0], r[1], r[2], r[3]);
                o[1] = make_uint4(r[4], r[5], r[6], r[7]);
                o[2] = make_uint4(r[8], r[9], r[10], r[11]);
                o[3] = make_uint4(r[12], r[13], r[14], r[15]);
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) cnt += r[j] != 0u;
        }
        for (; i < hi; ++i) {
            s = t.next[(size_t)s * 256 + text[i]];
            const uint32_t v = t.out[s];
            if (out) out[i - pos0] = v;
            cnt += v != 0u;
        }
    }
    if (count) {
        for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off);
        if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(count, (unsigned long long)cnt);
    }
}

__global__ void gen_stream_kernel(uint8_t* __restrict__ dst, uint64_t off, uint64_t n, uint64_t seed, int mode) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride)
        dst[k] = pm_stream_byte(off + k, seed, mode);
}

}  // namespace

static hipError_t launch_rt_impl(int variant, const uint8_t* text, int64_t stream_start, int64_t pos0, int64_t n,
                                 uint32_t* out, unsigned long long* count, const RtDev& t, int num_cu, hipStream_t s,
                                 int blocks_override) {
    if (n <= 0) return hipSuccess;
    // queued positions are kept as u32 offsets from pos0: split huge scans
    constexpr int64_t PIECE = (int64_t)1 << 31;
    if (n > PIECE) {
        for (int64_t off = 0; off < n; off += PIECE) {
            const int64_t m = n - off < PIECE ? n - off : PIECE;
            hipError_t e = launch_rt_impl(variant, text, stream_start, pos0 + off, m, out ? out + off : nullptr,
                                          count, t, num_cu, s, blocks_override);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    const int64_t nchunks = (n + RT_CHUNK - 1) / RT_CHUNK;
    int64_t blocks = (nchunks + RT_WAVES - 1) / RT_WAVES;
    if (blocks > num_cu) blocks = num_cu;  // persistent: one 1024-lane workgroup per CU (LDS-bound)
    if (blocks_override > 0) blocks = blocks_override;
    const dim3 g((unsigned)blocks), b(RT_THREADS);
    switch (variant) {
        case 1: hipLaunchKernelGGL(rt_scan_kernel<1>, g, b, 0, s, text, stream_start, pos0, n, out, count, t); break;
        case 2: hipLaunchKernelGGL(rt_scan_kernel<2>, g, b, 0, s, text, stream_start, pos0, n, out, count, t); break;
        case 9: hipLaunchKernelGGL(rt_scan_kernel<9>, g, b, 0, s, text, stream_start, pos0, n, out, count, t); break;
        default: hipLaunchKernelGGL(rt_scan_kernel<0>, g, b, 0, s, text, stream_start, pos0, n, out, count, t);
    }
    return hipGetLastError();
}

hipError_t pm_launch_rt(const uint8_t* text, int64_t stream_start, int64_t pos0, int64_t n, uint32_t* out,
                        unsigned long long* count, const RtDev& t, int num_cu, hipStream_t s) {
    return launch_rt_impl(0, text, stream_start, pos0, n, out, count, t, num_cu, s, 0);
}

hipError_t pm_launch_rt_variant(int variant, const uint8_t* text, int64_t stream_start, int64_t pos0, int64_t n,
                                uint32_t* out, unsigned long long* count, const RtDev& t, int num_cu, hipStream_t s,
                                int blocks_override) {
    return launch_rt_impl(variant, text, stream_start, pos0, n, out, count, t, num_cu, s, blocks_override);
}

hipError_t pm_launch_dfa(const uint8_t* text, int64_t stream_start, int64_t pos0, int64_t n, uint32_t* out,
                         unsigned long long* count, const DfaDev& t, int num_cu, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    // enough segments for ~8 waves per CU, each at least 2 KiB so the
    // max_len-1 warm-up stays a small fraction
    const int64_t lanes = (int64_t)num_cu * 512;
    int64_t seg = (n + lanes - 1) / lanes;
    if (seg < 2048) seg = 2048;
    seg = (seg + 15) & ~(int64_t)15;
    const int64_t nseg = (n + seg - 1) / seg;
    int64_t blocks = (nseg + DFA_THREADS - 1) / DFA_THREADS;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(dfa_scan_kernel, dim3((unsigned)blocks), dim3(DFA_THREADS), 0, s, text, stream_start, pos0, n,
                       out, count, t, seg);
    return hipGetLastError();
}

hipError_t pm_launch_gen(uint8_t* dst, uint64_t offset, uint64_t n, uint64_t seed, int mode, hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(gen_stream_kernel, dim3((unsigned)blocks), dim3(256), 0, s, dst, offset, n, seed, mode);
    return hipGetLastError();
}
