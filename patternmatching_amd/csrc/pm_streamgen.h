// pm_streamgen.h -- synthetic stream generator (host and device), the
// product's implementation of the stream specification in DESIGN.md §6:
//   word(k) = splitmix64((seed << 40) | k),  k = i / 8
//   raw(i)  = (word(i/8) >> (8 * (i % 8))) & 0xFF
//   mode 0 "ascii": 0x20 + ((raw * 95) >> 8)   mode 1 "bytes": raw
// and the "lines" stream (dense deep matches without the period of a tiled
// file): blocks of PM_LINES_BLOCK bytes, block b filled with dictionary
// patterns drawn by splitmix64((seed << 40) ^ (b << 20) ^ k), k = 0, 1, ...,
// each followed by '\n', the last one cut at the block end.
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

constexpr uint64_t PM_LINES_BLOCK = 1024;

// Block b of the lines stream (len <= PM_LINES_BLOCK bytes) into dst.
// pats: the patterns' bytes back to back; offs[p] .. offs[p+1]: pattern p.
PM_HD inline void pm_lines_block(uint8_t* dst, uint64_t len, uint64_t b, const uint8_t* pats, const uint32_t* offs,
                                 uint32_t npats, uint64_t seed) {
    uint64_t pos = 0;
    for (uint64_t k = 0; pos < len; ++k) {
        const uint32_t p = (uint32_t)(pm_splitmix64((seed << 40) ^ (b << 20) ^ k) % npats);
        for (uint32_t j = offs[p]; j < offs[p + 1] && pos < len; ++j) dst[pos++] = pats[j];
        if (pos < len) dst[pos++] = '\n';
    }
}
