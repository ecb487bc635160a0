/*
 * streamgen.h -- TEST INFRASTRUCTURE ONLY (oracle side).
 *
 * The synthetic-stream specification shared by the oracle, the reference
 * driver and the golden fixtures.  The product carries its own
 * implementation of the same specification (patternmatching_amd/csrc/
 * pm_streamgen.h, host and device); tests check the two agree byte for byte.
 *
 *   word(k)  = splitmix64((seed << 40) | k)        k = i / 8
 *   raw(i)   = (word(i/8) >> (8 * (i % 8))) & 0xFF
 *   mode 0 "ascii": 0x20 + ((raw * 95) >> 8)       printable 0x20..0x7E
 *   mode 1 "bytes": raw                             all 256 values
 */
#ifndef ORACLE_STREAMGEN_H
#define ORACLE_STREAMGEN_H
#include <stddef.h>
#include <stdint.h>

static inline uint64_t oracle_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

static inline void oracle_gen_stream(unsigned char* dst, size_t off, size_t n, uint64_t seed, int mode) {
    for (size_t j = 0; j < n; ++j) {
        size_t i = off + j;
        uint64_t w = oracle_splitmix64((seed << 40) | (uint64_t)(i >> 3));
        unsigned b = (unsigned)(w >> (8 * (i & 7))) & 0xFFu;
        dst[j] = (unsigned char)(mode == 0 ? 0x20u + ((b * 95u) >> 8) : b);
    }
}
#endif
