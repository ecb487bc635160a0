// Chained-gather rate with and without a concurrent stream (VERDICT r04
// item 1: does the deep kernel's 1 B read + 4 B write per position evict its
// table from the Infinity Cache?).  The deep kernel's shape without its DFA
// logic: one 1024-lane workgroup per CU (16 waves), one chain per lane, each
// lane owning a 4 KiB segment of a 1 GiB stream; per 32-position block a lane
//   STREAM=1: loads its 32 text bytes (two 16-B loads), makes 32 chained 4-B
//             gathers (each index = previous load ^ a text byte), and stores
//             the 32 results as 128 B (eight 16-B stores, non-temporal or
//             plain);
//   STREAM=0: the same 32 chained gathers, text bytes from registers, no
//             stores;
//   STREAM=2: the loads and stores alone (the stream floor, no gathers).
// Prints ms per 1 GiB launch and G gathers/s for each table size.
//   hipcc --offload-arch=gfx950 -O3 scripts/gather_stream_probe.hip -o /tmp/gsp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

template <int STREAM, bool NT>
__global__ __launch_bounds__(1024) void probe(const unsigned* __restrict__ tab, unsigned words,
                                              const unsigned char* __restrict__ text, unsigned* __restrict__ out,
                                              long long seg, unsigned* __restrict__ sink) {
    const long long lane = (long long)blockIdx.x * 1024 + threadIdx.x;
    const unsigned char* t = text + lane * seg;
    unsigned* o = out + lane * seg;
    unsigned idx = __umulhi((unsigned)lane * 0x9E3779B1u, words), acc = 0;
    for (long long b = 0; b < seg; b += 32) {
        unsigned w[8];
        if (STREAM) {
            const u32x4 a = *reinterpret_cast<const u32x4*>(t + b);
            const u32x4 c = *reinterpret_cast<const u32x4*>(t + b + 16);
            w[0] = a.x, w[1] = a.y, w[2] = a.z, w[3] = a.w, w[4] = c.x, w[5] = c.y, w[6] = c.z, w[7] = c.w;
        } else {
#pragma unroll
            for (int q = 0; q < 8; ++q) w[q] = (unsigned)(b + q) * 0x01010101u;
        }
        unsigned r[32];
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const unsigned c = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            if (STREAM == 2) {
                r[j] = c;
            } else {
                idx = __umulhi(tab[idx] ^ (c * 0x9E3779B1u), words);  // uniform in [0, words)
                r[j] = idx;
            }
        }
        if (STREAM) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const u32x4 v = {r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]};
                u32x4* p = reinterpret_cast<u32x4*>(o + b + 4 * q);
                if (NT) __builtin_nontemporal_store(v, p);
                else *p = v;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 32; ++j) acc += r[j];
        }
    }
    if (acc == 0x12345678u) sink[0] = acc ^ idx;
}

template <int STREAM, bool NT>
float run(const unsigned* tab, unsigned words, const unsigned char* text, unsigned* out, long long seg, int ncu,
          unsigned* sink) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL((probe<STREAM, NT>), dim3(ncu), dim3(1024), 0, 0, tab, words, text, out, seg, sink);
    CK(hipGetLastError());
    const int reps = 5;
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((probe<STREAM, NT>), dim3(ncu), dim3(1024), 0, 0, tab, words, text, out, seg, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const long long n = 1ll << 30;
    const long long seg = n / ((long long)ncu * 1024);  // 4 KiB on 256 CUs
    const unsigned max_words = 1u << 27;                // 512 MiB
    std::vector<unsigned> h(max_words);
    unsigned x = 12345;
    for (unsigned i = 0; i < max_words; ++i) {
        x ^= x << 13, x ^= x >> 17, x ^= x << 5;
        h[i] = x;
    }
    unsigned *tab, *sink, *out;
    unsigned char* text;
    CK(hipMalloc(&tab, (size_t)max_words * 4));
    CK(hipMalloc(&sink, 4));
    CK(hipMalloc(&text, (size_t)n));
    CK(hipMalloc(&out, (size_t)n * 4));
    CK(hipMemcpy(tab, h.data(), (size_t)max_words * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(text, h.data(), (size_t)max_words * 4, hipMemcpyHostToDevice));  // 512 MiB of random bytes
    CK(hipMemcpy(text + (n >> 1), h.data(), (size_t)max_words * 4, hipMemcpyHostToDevice));
    const double gathers = (double)ncu * 1024 * seg;
    std::printf("%d CUs, 1024 lanes per CU, one chain per lane, %lld B segments, 1 GiB stream\n", ncu, seg);
    const float fl = run<2, true>(tab, 1u << 10, text, out, seg, ncu, sink);
    const float fp = run<2, false>(tab, 1u << 10, text, out, seg, ncu, sink);
    std::printf("stream floor (1 B read + 4 B nt / plain store per position, no gathers): %.3f / %.3f ms\n", fl, fp);
    for (unsigned words : {1u << 19, 1u << 22, 46u << 18, 70u << 18, 1u << 25, 1u << 27}) {
        // 46u << 18 words = 46 MiB (snort's sparse image), 70 MiB (merged's)
        const float g0 = run<0, true>(tab, words, text, out, seg, ncu, sink);
        const float g1 = run<1, true>(tab, words, text, out, seg, ncu, sink);
        const float g2 = run<1, false>(tab, words, text, out, seg, ncu, sink);
        std::printf("table %7.1f MiB  gathers alone %7.3f ms (%6.1f G/s) | + stream nt %7.3f ms (%6.1f G/s) | + stream plain %7.3f ms (%6.1f G/s)\n",
                    words * 4.0 / (1 << 20), g0, gathers / (g0 * 1e6), g1, gathers / (g1 * 1e6), g2,
                    gathers / (g2 * 1e6));
        std::fflush(stdout);
    }
    return 0;
}
