// Scattered-load rate probe (MEASUREMENTS.md §4: what bounds the DFA kernel and
// the RT tail).  Every lane runs `chains` independent pointer chases through
// a table of random u32 indices (each load's address depends on the previous
// load of its chain), `steps` loads per chain; prints loads/s for each
// table size, load form and width.
//   hipcc --offload-arch=gfx950 -O3 scripts/gather_probe.hip -o /tmp/gather_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e = (x);                                                   \
        if (e != hipSuccess) {                                                \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            std::exit(1);                                                     \
        }                                                                     \
    } while (0)

using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

// FORM 0 plain, 1 nontemporal, 2 sc1 (agent-scope relaxed: bypasses L1)
template <int FORM>
__device__ __forceinline__ unsigned ld1(const unsigned* p) {
    if (FORM == 1) return __builtin_nontemporal_load(p);
    if (FORM == 2) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return *p;
}

template <int FORM, int WIDE, int CH>
__global__ __launch_bounds__(256) void chase(const unsigned* __restrict__ tab, unsigned mask, int steps,
                                             unsigned* __restrict__ sink) {
    const unsigned tid = blockIdx.x * 256u + threadIdx.x;
    unsigned idx[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) idx[c] = ((tid * CH + c) * 0x9E3779B1u) & mask;
    unsigned acc = 0;
    for (int s = 0; s < steps; ++s) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            if (WIDE) {
                const u32x4 v = *reinterpret_cast<const u32x4*>(tab + (idx[c] & ~3u));
                idx[c] = (v.x ^ v.y ^ v.z ^ v.w) & mask;
            } else {
                idx[c] = ld1<FORM>(tab + idx[c]) & mask;  // stay inside the table
            }
        }
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) acc ^= idx[c];
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int FORM, int WIDE, int CH>
double run(const unsigned* tab, unsigned words, int blocks, int steps, unsigned* sink) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL((chase<FORM, WIDE, CH>), dim3(blocks), dim3(256), 0, 0, tab, words - 1, steps, sink);
    CK(hipEventRecord(a));
    const int reps = 3;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((chase<FORM, WIDE, CH>), dim3(blocks), dim3(256), 0, 0, tab, words - 1, steps, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double loads = (double)blocks * 256 * CH * steps * reps;
    return loads / (ms * 1e-3) / 1e9;
}

int main() {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const unsigned max_words = 1u << 27;  // 512 MiB
    std::vector<unsigned> h(max_words);
    unsigned x = 12345;
    for (unsigned i = 0; i < max_words; ++i) {
        x ^= x << 13, x ^= x >> 17, x ^= x << 5;
        h[i] = x;
    }
    unsigned *tab, *sink;
    CK(hipMalloc(&tab, (size_t)max_words * 4));
    CK(hipMalloc(&sink, 4));
    CK(hipMemcpy(tab, h.data(), (size_t)max_words * 4, hipMemcpyHostToDevice));
    const int steps = 256;
    for (int wpc : {8, 16}) {  // waves per CU
        const int blocks = ncu * wpc / 4;
        for (unsigned words : {1u << 12, 1u << 15, 1u << 19, 1u << 22, 1u << 27}) {
            std::printf("waves/CU %2d table %8.3f MiB  G loads/s:  4B plain ch1 %6.1f ch4 %6.1f | nt ch4 %6.1f | sc1 ch4 %6.1f | 16B ch4 %6.1f\n",
                        wpc, words * 4.0 / (1 << 20), run<0, 0, 1>(tab, words, blocks, steps, sink),
                        run<0, 0, 4>(tab, words, blocks, steps, sink), run<1, 0, 4>(tab, words, blocks, steps, sink),
                        run<2, 0, 4>(tab, words, blocks, steps, sink), run<0, 1, 4>(tab, words, blocks, steps, sink));
            std::fflush(stdout);
        }
    }
    return 0;
}
