// pm_streamgen.h -- synthetic stream generator (host and device), the
// product's implementation of the stream specification in DESIGN.md §5:
//   word(k) = splitmix64((seed << 40) | k),  k = i / 8
//   raw(i)  = (word(i/8) >> (8 * (i % 8))) & 0xFF
//   mode 0 "ascii": 0x20 + ((raw * 95) >> 8)   mode 1 "bytes": raw
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define PM_HD __host__ __device__
#else
#define PM_HD
#endif

PM_HD inline uint64_t pm_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

PM_HD inline uint8_t pm_stream_byte(uint64_t i, uint64_t seed, int mode) {
    uint64_t w = pm_splitmix64((seed << 40) | (i >> 3));
    uint32_t b = (uint32_t)(w >> (8 * (i & 7))) & 0xFFu;
    return (uint8_t)(mode == 0 ? 0x20u + ((b * 95u) >> 8) : b);
}
