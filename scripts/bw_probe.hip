// bw_probe.hip -- HBM streaming microbenchmark for the dense scan's memory
// shape (read 1 B, write 4 B per stream position), to find the store form
// and launch shape that reach the chip's copy rate.  Timing tool only.
//   hipcc --offload-arch=gfx950 -O3 -o bw_probe bw_probe.hip && ./bw_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

using u32x2 = __attribute__((ext_vector_type(2))) unsigned int;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

// write-only: each wave stores CH KiB chunks, chunks strided over the grid
template <bool NT>
__global__ __launch_bounds__(1024) void wr(uint32_t* out, int64_t n_u32, int persist) {
    const int lane = threadIdx.x & 63;
    const int64_t nchunk = n_u32 / 1024;  // 4 KiB per wave-chunk
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int64_t stride = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t c = wave; c < nchunk; c += stride) {
        u32x4* o = reinterpret_cast<u32x4*>(out + c * 1024);
        u32x4 v = {(uint32_t)c, 1u, 2u, 3u};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if (NT) __builtin_nontemporal_store(v, o + 64 * s + lane);
            else o[64 * s + lane] = v;
        }
        if (!persist) break;
    }
}

// the scan's shape: read 1 KiB (8 B windows), write 4 KiB per wave-chunk
template <bool NT>
__global__ __launch_bounds__(1024) void rw(const uint8_t* in, uint32_t* out, int64_t n, unsigned long long* sink) {
    const int lane = threadIdx.x & 63;
    const int64_t nchunk = n / 1024;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int64_t stride = (int64_t)gridDim.x * (blockDim.x / 64);
    uint32_t acc = 0;
    for (int64_t c = wave; c < nchunk; c += stride) {
        const uint8_t* src = in + c * 1024 + 4 * lane;
        u32x2 x[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) x[s] = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(src + 256 * s));
        u32x4* o = reinterpret_cast<u32x4*>(out + c * 1024);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            u32x4 v = {x[s].x & 0xFFFF, x[s].x >> 16, x[s].y & 0xFFFF, x[s].y >> 16};
            if (NT) __builtin_nontemporal_store(v, o + 64 * s + lane);
            else o[64 * s + lane] = v;
            acc += x[s].x;
        }
    }
    if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}

int main() {
    const int64_t n = (int64_t)1 << 30;  // stream positions
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
    auto timeit = [&](const char* name, double bytes, auto launch) {
        for (int w = 0; w < 2; ++w) launch();
        CK(hipEventRecord(a));
        const int R = 10;
        for (int r = 0; r < R; ++r) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= R;
        std::printf("{\"case\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", name, ms, bytes / (ms * 1e-3) / 1e12);
        return 0;
    };
    const double wbytes = 4.0 * n, rwbytes = 5.0 * n;
    for (int blocks : {cu, 2 * cu, 4 * cu}) {
        char nm[96];
        std::snprintf(nm, sizeof nm, "write 4GiB plain persistent blocks=%d", blocks);
        timeit(nm, wbytes, [&] { hipLaunchKernelGGL(wr<false>, dim3(blocks), dim3(1024), 0, 0, out, n, 1); });
        std::snprintf(nm, sizeof nm, "write 4GiB nt persistent blocks=%d", blocks);
        timeit(nm, wbytes, [&] { hipLaunchKernelGGL(wr<true>, dim3(blocks), dim3(1024), 0, 0, out, n, 1); });
    }
    timeit("write 4GiB plain one-chunk-per-wave", wbytes,
           [&] { hipLaunchKernelGGL(wr<false>, dim3((unsigned)(n / 1024 / 16)), dim3(1024), 0, 0, out, n, 0); });
    for (int blocks : {cu, 2 * cu}) {
        char nm[96];
        std::snprintf(nm, sizeof nm, "read1+write4 plain blocks=%d", blocks);
        timeit(nm, rwbytes, [&] { hipLaunchKernelGGL(rw<false>, dim3(blocks), dim3(1024), 0, 0, in, out, n, sink); });
        std::snprintf(nm, sizeof nm, "read1+write4 nt blocks=%d", blocks);
        timeit(nm, rwbytes, [&] { hipLaunchKernelGGL(rw<true>, dim3(blocks), dim3(1024), 0, 0, in, out, n, sink); });
    }
    timeit("hipMemsetD32 4GiB", wbytes, [&] { (void)hipMemsetD32Async((hipDeviceptr_t)out, 0, n, 0); });
    timeit("hipMemcpy DtoD 2GiB (4GiB traffic)", wbytes, [&] {
        (void)hipMemcpyAsync(out + n / 2, out, n * 2, hipMemcpyDeviceToDevice, 0);
    });
    return 0;
}
