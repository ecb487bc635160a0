// bw_probe4.hip -- what separates the rt_scan_kernel streaming floor
// (variant 2) from the plain read-1-write-4 loop of bw_probe3: the probe's
// loop (prefetch 2 chunks ahead, 16-B nt stores) plus, one at a time, the
// kernel's extras: XP the broadcast dword before each chunk, LDS a 160 KiB
// workgroup LDS block staged from global memory at the start, BAL 16
// ballot + popcount steps per chunk, RND varying (random-text) input.
// Timing tool only.
//   hipcc --offload-arch=gfx950 -O3 -o bw_probe4 bw_probe4.hip && ./bw_probe4
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

template <bool XP, bool LDS, bool BAL>
__global__ __launch_bounds__(1024) void rw(const uint8_t* in, uint32_t* out, int64_t n, const uint32_t* table,
                                           unsigned long long* sink) {
    __shared__ uint32_t s_tab[LDS ? 40960 : 1];
    if (LDS) {
        for (int k = threadIdx.x; k < 40960; k += 1024) s_tab[k] = table[k];
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int64_t nchunk = n / 1024;
    const int64_t wave = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
    const int64_t nw = (int64_t)gridDim.x * 16;
    constexpr int D = 2;
    uint32_t ring[D + 1][4], pre[D + 1];
    uint32_t acc = 0, sc = 0;
    auto fetch = [&](uint32_t (&x)[4], uint32_t& p, int64_t c) {
        const uint8_t* src = in + (c < nchunk ? c : 0) * 1024 + 4 * lane;
#pragma unroll
        for (int s = 0; s < 4; ++s) x[s] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(src + 256 * s));
        if (XP) p = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(in + (c < nchunk ? c : 0) * 1024 + 60));
    };
#pragma unroll
    for (int d = 0; d < D; ++d) fetch(ring[d], pre[d], wave + d * nw);
    for (int64_t c = wave; c < nchunk; c += (D + 1) * nw) {
#pragma unroll
        for (int u = 0; u <= D; ++u) {
            const int64_t cc = c + u * nw;
            fetch(ring[(u + D) % (D + 1)], pre[(u + D) % (D + 1)], cc + D * nw);
            if (cc < nchunk) {
                uint32_t* o = out + cc * 1024;
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const uint32_t x = ring[u][s] ^ (XP ? pre[u] : 0u);
                    uint32_t v0 = x & 0xFFu, v1 = (x >> 8) & 0xFFu, v2 = (x >> 16) & 0xFFu, v3 = x >> 24;
                    if (LDS) v0 = s_tab[x & 0x7FFFu];
                    if (BAL) {
                        sc += (uint32_t)__popcll(__ballot(v0 != 0u)) + (uint32_t)__popcll(__ballot(v1 != 0u)) +
                              (uint32_t)__popcll(__ballot(v2 != 0u)) + (uint32_t)__popcll(__ballot(v3 != 0u));
                    }
                    const u32x4 v = {v0, v1, v2, v3};
                    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(o + 256 * s) + lane);
                    acc += x;
                }
            }
        }
    }
    if (acc == 0x12345678u || sc == 0x12345678u) atomicAdd(sink, 1ull);
}

__global__ void fill(uint8_t* p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 31)) * 0xBF58476D1CE4E5B9ull;
        p[i] = (uint8_t)(0x20 + (((z >> 32) & 0xFF) * 95 >> 8));
    }
}

int main() {
    const int64_t n = (int64_t)1 << 30;
    uint8_t *in, *in_rnd;
    uint32_t *out, *table;
    unsigned long long* sink;
    CK(hipMalloc(&in, n + 64));
    CK(hipMalloc(&in_rnd, n + 64));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&table, 40960 * 4));
    CK(hipMalloc(&sink, 8));
    CK(hipMemset(in, 7, n + 64));
    CK(hipMemset(table, 1, 40960 * 4));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, in_rnd, n + 64);
    CK(hipMemset(out, 0, n * 4));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cu = p.multiProcessorCount;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](const char* name, auto launch) {
        for (int w = 0; w < 2; ++w) launch();
        CK(hipEventRecord(a));
        const int R = 10;
        for (int r = 0; r < R; ++r) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= R;
        std::printf("{\"case\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", name, ms, 5.0 * n / (ms * 1e-3) / 1e12);
        std::fflush(stdout);
        return 0;
    };
#define RW(XP, LDS, BAL, SRC, NAME)                                                                              \
    timeit(NAME, [&] { hipLaunchKernelGGL((rw<XP, LDS, BAL>), dim3(cu), dim3(1024), 0, 0, SRC, out, n, table, sink); });
    for (int rep = 0; rep < 2; ++rep) {
        RW(false, false, false, in, "base")
        RW(false, false, false, in_rnd, "base+RND")
        RW(true, false, false, in_rnd, "XP+RND")
        RW(false, true, false, in_rnd, "LDS+RND")
        RW(false, false, true, in_rnd, "BAL+RND")
        RW(true, true, true, in_rnd, "all+RND")
    }
    return 0;
}
