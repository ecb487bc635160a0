// bw_probe2.hip -- more store forms for the dense scan's memory shape
// (read 1 B, write 4 B per position): per-wave contiguous spans vs
// grid-stride chunks, plain / nt / sc1 stores, 1-4 workgroups per CU, and
// pure write / pure read rates.  Timing tool only.
//   hipcc --offload-arch=gfx950 -O3 -o bw_probe2 bw_probe2.hip && ./bw_probe2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)
using u32x2 = __attribute__((ext_vector_type(2))) unsigned int;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

// ST: 0 plain, 1 nt, 2 sc1 (buffer store, glc/slc bits)
template <int ST>
__device__ __forceinline__ void st16(uint32_t* base, int byteoff, u32x4 v) {
    if (ST == 0) *reinterpret_cast<u32x4*>(reinterpret_cast<char*>(base) + byteoff) = v;
    if (ST == 1) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(reinterpret_cast<char*>(base) + byteoff));
    if (ST == 2) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, byteoff, 0, 16);
    }
}

// MAP: 0 grid-stride 1 KiB-of-input chunks per wave; 1 contiguous span per wave;
//      2 grid-stride, chunk index swizzled so 8 consecutive chunks share a block's XCD slot
template <int ST, int MAP, int UNR>
__global__ __launch_bounds__(1024) void rw(const uint8_t* in, uint32_t* out, int64_t n, unsigned long long* sink) {
    const int lane = threadIdx.x & 63;
    const int wpb = blockDim.x / 64;
    const int64_t nchunk = n / 1024;
    const int64_t wave = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6);
    const int64_t nw = (int64_t)gridDim.x * wpb;
    uint32_t acc = 0;
    int64_t c0, cs, cend;
    if (MAP == 1) {
        const int64_t per = (nchunk + nw - 1) / nw;
        c0 = wave * per; cs = 1; cend = c0 + per < nchunk ? c0 + per : nchunk;
    } else {
        c0 = wave; cs = nw; cend = nchunk;
    }
    for (int64_t c = c0; c < cend; c += cs * UNR) {
        u32x2 x[UNR][4];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const int64_t cc = c + u * cs < cend ? c + u * cs : c;
            const uint8_t* src = in + cc * 1024 + 4 * lane;
#pragma unroll
            for (int s = 0; s < 4; ++s) x[u][s] = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(src + 256 * s));
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            if (c + u * cs >= cend) break;
            uint32_t* o = out + (c + u * cs) * 1024;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                u32x4 v = {x[u][s].x & 0xFFFF, x[u][s].x >> 16, x[u][s].y & 0xFFFF, x[u][s].y >> 16};
                st16<ST>(o, 1024 * s + 16 * lane, v);
                acc += x[u][s].x;
            }
        }
    }
    if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}

template <int ST>
__global__ __launch_bounds__(1024) void wr(uint32_t* out, int64_t n_u32) {
    const int lane = threadIdx.x & 63;
    const int64_t nchunk = n_u32 / 1024;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int64_t stride = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t c = wave; c < nchunk; c += stride) {
        u32x4 v = {(uint32_t)c, 1u, 2u, 3u};
#pragma unroll
        for (int s = 0; s < 4; ++s) st16<ST>(out + c * 1024, 1024 * s + 16 * lane, v);
    }
}

__global__ __launch_bounds__(1024) void rd(const uint8_t* in, int64_t n, unsigned long long* sink) {
    const int lane = threadIdx.x & 63;
    const int64_t nchunk = n / 4096;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int64_t stride = (int64_t)gridDim.x * (blockDim.x / 64);
    uint32_t acc = 0;
    for (int64_t c = wave; c < nchunk; c += stride) {
        u32x4 x[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) x[s] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in + c * 4096 + 1024 * s + 16 * lane));
#pragma unroll
        for (int s = 0; s < 4; ++s) acc += x[s].x ^ x[s].w;
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
        std::fflush(stdout);
        return 0;
    };
    const double rw_b = 5.0 * n;
    char nm[128];
#define RW(ST, MAP, UNR, BLK, THR)                                                                        \
    std::snprintf(nm, sizeof nm, "rw st=%d map=%d unr=%d blocks=%d threads=%d", ST, MAP, UNR, BLK, THR); \
    timeit(nm, rw_b, [&] { hipLaunchKernelGGL((rw<ST, MAP, UNR>), dim3(BLK), dim3(THR), 0, 0, in, out, n, sink); });
    RW(1, 0, 1, cu, 1024)
    RW(0, 0, 1, cu, 1024)
    RW(2, 0, 1, cu, 1024)
    RW(1, 0, 2, cu, 1024)
    RW(0, 0, 2, cu, 1024)
    RW(1, 1, 1, cu, 1024)
    RW(0, 1, 1, cu, 1024)
    RW(1, 1, 2, cu, 1024)
    RW(1, 0, 1, 2 * cu, 512)
    RW(1, 0, 1, 4 * cu, 256)
    RW(1, 0, 1, 8 * cu, 256)
    RW(0, 0, 1, 8 * cu, 256)
    RW(1, 0, 2, 2 * cu, 1024)
    RW(1, 0, 1, (int)(n / 1024 / 16), 1024)
    for (int blocks : {cu, 4 * cu}) {
        std::snprintf(nm, sizeof nm, "write4GiB plain blocks=%d", blocks);
        timeit(nm, 4.0 * n, [&] { hipLaunchKernelGGL(wr<0>, dim3(blocks), dim3(1024), 0, 0, out, n); });
        std::snprintf(nm, sizeof nm, "write4GiB nt blocks=%d", blocks);
        timeit(nm, 4.0 * n, [&] { hipLaunchKernelGGL(wr<1>, dim3(blocks), dim3(1024), 0, 0, out, n); });
        std::snprintf(nm, sizeof nm, "write4GiB sc1 blocks=%d", blocks);
        timeit(nm, 4.0 * n, [&] { hipLaunchKernelGGL(wr<2>, dim3(blocks), dim3(1024), 0, 0, out, n); });
        std::snprintf(nm, sizeof nm, "read4GiB nt blocks=%d", blocks);
        timeit(nm, 4.0 * n, [&] { hipLaunchKernelGGL(rd, dim3(blocks), dim3(1024), 0, 0, reinterpret_cast<const uint8_t*>(out), 4 * n, sink); });
    }
    timeit("hipMemsetD32 4GiB", 4.0 * n, [&] { (void)hipMemsetD32Async((hipDeviceptr_t)out, 0, n, 0); });
    timeit("hipMemcpy DtoD 2GiB (4GiB traffic)", 4.0 * n, [&] {
        (void)hipMemcpyAsync(out + n / 2, out, n * 2, hipMemcpyDeviceToDevice, 0);
    });
    return 0;
}
