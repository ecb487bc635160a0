// bw_probe3.hip -- the dense scan's memory shape (read 1 B, write 4 B per
// position, 1 KiB-of-input chunks grid-stride per wave, dword text loads,
// 16-B non-temporal id stores, one 1024-thread workgroup per CU) with the
// text prefetched D chunks ahead in a register ring: is the streaming floor
// bound by how far ahead the reads are issued?  Timing tool only.
//   hipcc --offload-arch=gfx950 -O3 -o bw_probe3 bw_probe3.hip && ./bw_probe3
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

// D: chunks in flight ahead of the one being stored (D + 1 register sets)
template <int D, bool NT_ST>
__global__ __launch_bounds__(1024) void rw(const uint8_t* in, uint32_t* out, int64_t n, unsigned long long* sink) {
    const int lane = threadIdx.x & 63;
    const int64_t nchunk = n / 1024;
    const int64_t wave = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
    const int64_t nw = (int64_t)gridDim.x * 16;
    uint32_t ring[D + 1][4];
    uint32_t acc = 0;
    auto fetch = [&](uint32_t (&x)[4], int64_t c) {
        const uint8_t* src = in + (c < nchunk ? c : 0) * 1024 + 4 * lane;
#pragma unroll
        for (int s = 0; s < 4; ++s) x[s] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(src + 256 * s));
    };
#pragma unroll
    for (int d = 0; d < D; ++d) fetch(ring[d], wave + d * nw);
    for (int64_t c = wave; c < nchunk; c += (D + 1) * nw) {
#pragma unroll
        for (int u = 0; u <= D; ++u) {  // fully unrolled ring: slot u holds chunk c + u * nw
            const int64_t cc = c + u * nw;
            fetch(ring[(u + D) % (D + 1)], cc + D * nw);
            if (cc < nchunk) {
                uint32_t* o = out + cc * 1024;
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const uint32_t x = ring[u][s];
                    const u32x4 v = {x & 0xFFu, (x >> 8) & 0xFFu, (x >> 16) & 0xFFu, x >> 24};
                    u32x4* p = reinterpret_cast<u32x4*>(o + 256 * s) + lane;
                    if (NT_ST) __builtin_nontemporal_store(v, p);
                    else *p = v;
                    acc += x;
                }
            }
        }
    }
    if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}

int main() {
    const int64_t n = (int64_t)1 << 30;
    uint8_t* in;
    uint32_t* out;
    unsigned long long* sink;
    CK(hipMalloc(&in, n + 64));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&sink, 8));
    CK(hipMemset(in, 7, n + 64));
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
#define RW(D, NT)                                                                                   \
    timeit("prefetch=" #D " nt_store=" #NT, [&] {                                                   \
        hipLaunchKernelGGL((rw<D, NT>), dim3(cu), dim3(1024), 0, 0, in, out, n, sink);             \
    });
    for (int rep = 0; rep < 2; ++rep) {
        RW(0, true)
        RW(1, true)
        RW(2, true)
        RW(3, true)
        RW(5, true)
        RW(7, true)
        RW(2, false)
        RW(5, false)
    }
    return 0;
}
