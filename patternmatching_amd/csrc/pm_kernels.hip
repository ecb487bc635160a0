// pm_kernels.hip -- gfx950 kernels of the stream scan (read_char batched).
//
// rt_scan_kernel  one lane per 16 consecutive stream positions.  For each
//   position i it walks the reverse-suffix trie backwards over
//   text[i], text[i-1], ... and emits the gid of the deepest pattern node
//   met, which is exactly the id ac_read_char returns at i
//   (Core/src/mpac.c:304-319: the longest pattern that is a suffix of the
//   stream so far).  Depth <= 2 is one u16 lookup in an LDS-resident 64K
//   table keyed by the two last bytes; depth 3 is one u32 load from an
//   L2-resident table; deeper walks (about 1 % of positions on random text)
//   follow 48-B bitmap-rank records.  Positions are independent: no carried
//   state, no warm-up, fully coalesced 16-B loads and 64-B stores per lane.
//
// dfa_scan_kernel the reference automaton itself, flattened to a dense DFA
//   (next[s*256+c], out[s]); one lane per stream segment, started from the
//   root max_len-1 bytes before the segment (SURVEY.md §0.1 shard rule), so
//   every segment is independent and exact.
#include "pm_kernels.h"
#include "pm_streamgen.h"

namespace {

constexpr int RT_THREADS = 1024;
constexpr int RT_LDS_U16 = 65536 + 256;
constexpr uint32_t CONT16 = 0x8000u;
constexpr uint32_t CONT32 = 0x80000000u;

// Depth >= 3 walk.  `node` is a record reached after consuming
// text[i], text[i-1], text[i-2]; avail = bytes that exist at or before i.
__device__ __forceinline__ uint32_t rt_deep(const uint8_t* __restrict__ text, const uint32_t* __restrict__ rec,
                                            uint32_t node, int64_t i, int64_t avail) {
    int64_t d = 3;
    for (;;) {
        const uint32_t* R = rec + (size_t)node * 12;
        const uint4 meta = *reinterpret_cast<const uint4*>(R + 8);  // base, best, prefix[0..3], prefix[4..7]
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

// One position, every boundary case (stream start, short lookback).
__device__ uint32_t rt_one(const uint8_t* __restrict__ text, const uint16_t* s_t, const RtDev& t, int64_t i,
                           int64_t stream_start) {
    const int64_t avail = i - stream_start + 1;
    const uint32_t c0 = text[i];
    if (avail == 1) return s_t[65536 + c0];
    const uint32_t v = s_t[(c0 << 8) | text[i - 1]];
    if (!(v & CONT16)) return v;
    const uint32_t n2 = v & 0x7FFFu;
    if (avail == 2) return t.b2[n2];
    const uint32_t r = t.t3[(size_t)n2 * 256 + text[i - 2]];
    if (!(r & CONT32)) return r;
    return rt_deep(text, t.rec, r & 0x7FFFFFFFu, i, avail);
}

__global__ __launch_bounds__(RT_THREADS) void rt_scan_kernel(const uint8_t* __restrict__ text, int64_t stream_start,
                                                             int64_t pos0, int64_t n, uint32_t* __restrict__ out,
                                                             unsigned long long* __restrict__ count, RtDev t) {
    __shared__ __attribute__((aligned(16))) uint16_t s_t[RT_LDS_U16];
    {
        const uint4* src = reinterpret_cast<const uint4*>(t.t12);
        uint4* dst = reinterpret_cast<uint4*>(s_t);
        for (int k = threadIdx.x; k < RT_LDS_U16 * 2 / 16; k += RT_THREADS) dst[k] = src[k];
    }
    __syncthreads();

    uint32_t cnt = 0;
    const int64_t ngroups = (n + 15) >> 4;
    const int64_t stride = (int64_t)gridDim.x * RT_THREADS;
    for (int64_t g = (int64_t)blockIdx.x * RT_THREADS + threadIdx.x; g < ngroups; g += stride) {
        const int64_t p = pos0 + (g << 4);
        const int64_t rem = n - (g << 4);
        if (rem >= 16 && p - stream_start >= 2) {
            const uint4 w = *reinterpret_cast<const uint4*>(text + p);
            const uint32_t prev = *reinterpret_cast<const uint32_t*>(text + p - 4);
            const uint32_t W[5] = {prev, w.x, w.y, w.z, w.w};  // bytes p-4 .. p+15
            uint32_t r[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                // key = text[i] << 8 | text[i-1] = the LE u16 at window offset j+3
                const int o = j + 3;
                uint32_t key;
                if ((o & 3) != 3) key = (W[o >> 2] >> (8 * (o & 3))) & 0xFFFFu;
                else key = __builtin_amdgcn_alignbyte(W[(o >> 2) + 1], W[o >> 2], 3) & 0xFFFFu;
                r[j] = s_t[key];
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                if (r[j] & CONT16) {
                    const int o2 = j + 2;  // text[i-2]
                    const uint32_t c2 = (W[o2 >> 2] >> (8 * (o2 & 3))) & 0xFFu;
                    r[j] = t.t3[(size_t)(r[j] & 0x7FFFu) * 256 + c2];
                }
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                if (r[j] & CONT32) r[j] = rt_deep(text, t.rec, r[j] & 0x7FFFFFFFu, p + j, p + j - stream_start + 1);
            }
            if (out) {
                uint4* o = reinterpret_cast<uint4*>(out + (p - pos0));
                o[0] = make_uint4(r[0], r[1], r[2], r[3]);
                o[1] = make_uint4(r[4], r[5], r[6], r[7]);
                o[2] = make_uint4(r[8], r[9], r[10], r[11]);
                o[3] = make_uint4(r[12], r[13], r[14], r[15]);
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) cnt += r[j] != 0u;
        } else {
            const int64_t m = rem < 16 ? rem : 16;
            for (int64_t j = 0; j < m; ++j) {
                const uint32_t v = rt_one(text, s_t, t, p + j, stream_start);
                if (out) out[p - pos0 + j] = v;
                cnt += v != 0u;
            }
        }
    }
    if (count) {
        for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off);
        if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(count, (unsigned long long)cnt);
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

hipError_t pm_launch_rt(const uint8_t* text, int64_t stream_start, int64_t pos0, int64_t n, uint32_t* out,
                        unsigned long long* count, const RtDev& t, int num_cu, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t ngroups = (n + 15) >> 4;
    int64_t blocks = (ngroups + RT_THREADS - 1) / RT_THREADS;
    if (blocks > num_cu) blocks = num_cu;  // persistent: one 1024-lane workgroup per CU (LDS-bound)
    hipLaunchKernelGGL(rt_scan_kernel, dim3((unsigned)blocks), dim3(RT_THREADS), 0, s, text, stream_start, pos0, n,
                       out, count, t);
    return hipGetLastError();
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
