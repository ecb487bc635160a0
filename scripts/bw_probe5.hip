// bw_probe5.hip -- probe (not product): the headline scan's memory shape
// (read 1 B, write a 4-B id per position; 1 KiB-of-input chunks grid-stride
// per wave, one 1024-thread workgroup per CU, text two chunks ahead,
// non-temporal 16-B id stores) with the text loaded as
//   dword:  each lane one dword per 256-B group, four loads per chunk (the
//           product kernel's shape: 256 contiguous bytes per instruction);
//   x4nat:  each lane the 16 contiguous bytes of positions 16L..16L+15, one
//           load per chunk (1 KiB per instruction), ids stored as four
//           16-B stores per lane at a 64-B lane stride (the natural layout);
//   x4lds:  the same 16-B loads, ids re-laid through LDS so every store
//           instruction writes 1 KiB contiguous (as dword);
// plus write-only and read-only references.  Timing tool only.
//   hipcc --offload-arch=gfx950 -O3 -o bw_probe5 bw_probe5.hip && ./bw_probe5
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

enum { DWORD = 0, X4NAT = 1, X4LDS = 2, WRITE_ONLY = 3, READ_ONLY = 4 };

template <int MODE>
__global__ __launch_bounds__(1024) void rw(const uint8_t* in, uint32_t* out, int64_t n, unsigned long long* sink) {
    __shared__ u32x4 s_x[MODE == X4LDS ? 1024 * 4 : 1];
    const int lane = threadIdx.x & 63;
    const int64_t nchunk = n / 1024;
    const int64_t wave = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
    const int64_t nw = (int64_t)gridDim.x * 16;
    u32x4 ring[3];
    uint32_t acc = 0;
    auto fetch = [&](u32x4& x, int64_t c) {
        const uint8_t* src = in + (c < nchunk ? c : 0) * 1024;
        if (MODE == DWORD || MODE == WRITE_ONLY) {
            if (MODE == WRITE_ONLY) { x = u32x4{(uint32_t)c, 1u, 2u, 3u}; return; }
#pragma unroll
            for (int s = 0; s < 4; ++s) x[s] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(src + 256 * s + 4 * lane));
        } else {
            x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + lane);
        }
    };
    fetch(ring[0], wave);
    fetch(ring[1], wave + nw);
    for (int64_t c = wave; c < nchunk; c += 3 * nw) {
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int64_t cc = c + u * nw;
            fetch(ring[(u + 2) % 3], cc + 2 * nw);
            if (cc >= nchunk) continue;
            const u32x4 x = ring[u];
            uint32_t* o = out + cc * 1024;
            if (MODE == READ_ONLY) {
                acc += x.x ^ x.y ^ x.z ^ x.w;
                continue;
            }
            if (MODE == DWORD || MODE == WRITE_ONLY) {
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const uint32_t w = x[s];
                    const u32x4 v = {w & 0xFFu, (w >> 8) & 0xFFu, (w >> 16) & 0xFFu, w >> 24};
                    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(o + 256 * s) + lane);
                }
            } else if (MODE == X4NAT) {
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const uint32_t w = x[s];
                    const u32x4 v = {w & 0xFFu, (w >> 8) & 0xFFu, (w >> 16) & 0xFFu, w >> 24};
                    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(o + 16 * lane) + s);
                }
            } else {  // X4LDS: ids of positions 16L + 4s .. to LDS, read back as positions 256s + 4L ..
                u32x4* my = s_x + (threadIdx.x >> 6) * 256;
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const uint32_t w = x[s];
                    my[4 * lane + s] = u32x4{w & 0xFFu, (w >> 8) & 0xFFu, (w >> 16) & 0xFFu, w >> 24};
                }
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    __builtin_nontemporal_store(my[64 * s + lane], reinterpret_cast<u32x4*>(o + 256 * s) + lane);
                __builtin_amdgcn_wave_barrier();
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
    auto timeit = [&](const char* name, double bytes_per_pos, auto launch) {
        for (int w = 0; w < 2; ++w) launch();
        CK(hipEventRecord(a));
        const int R = 10;
        for (int r = 0; r < R; ++r) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= R;
        std::printf("{\"case\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", name, ms, bytes_per_pos * n / (ms * 1e-3) / 1e12);
        std::fflush(stdout);
        return 0;
    };
#define RW(M, BPP) timeit(#M, BPP, [&] { hipLaunchKernelGGL((rw<M>), dim3(cu), dim3(1024), 0, 0, in, out, n, sink); });
    for (int rep = 0; rep < 3; ++rep) {
        RW(DWORD, 5.0)
        RW(X4NAT, 5.0)
        RW(X4LDS, 5.0)
        RW(WRITE_ONLY, 4.0)
        RW(READ_ONLY, 1.0)
    }
    return 0;
}
