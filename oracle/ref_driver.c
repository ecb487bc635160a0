/*
 * ref_driver.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A small driver of our own that links the REFERENCE's unmodified C objects
 * (compiled from /root/reference/Core/src by oracle/Makefile into
 * oracle/_ref/, never copied) to produce golden vectors and to time the
 * reference's own per-byte Aho-Corasick loop as the CPU baseline.
 *
 * It uses only the reference's public entry points:
 *   mps_table_setup()                  Core/src/mps.c:120-124
 *   patterns_tree_build(conf,obj,cb)   Core/src/PatternsTree.c:469-475
 *                                      (its return value is garbage, unused)
 *   mps_table[MPS_AC].create/add_pattern/compile/read_char/reset/total_mem
 *                                      Core/src/mpac.c:358-367
 *   parse_pattern_from_line            Core/src/parser.c:63-99
 * A pattern_id_t is a PatternsTreeNode* whose pattern_id holds
 * (file_number, line_number) (PatternsTree.h:25-28, :104).
 *
 * Modes:
 *   dense  OUT STREAM DICT...     u32 (file<<24 | line) per position, 0 = none
 *   gen    OUT SEED MODE NBYTES   write a synthetic stream (oracle/streamgen.h)
 *   digest SEED MODE NBYTES DICT... stream generated in memory; prints JSON with
 *                                 nonnull count, FNV-1a-64 of the dense u32
 *                                 codes and the first 1000 (pos, code) records
 *   stats  DICT...                unique patterns, AC states, max length
 *   parse  DICT                   per accepted line: "line hexbytes"
 *   time   SEED MODE NBYTES DICT... time the reference read_char loop (1 core)
 *   timefile STREAM DICT...       the same over a stream file (e.g. a lines sample)
 *   parents OUT DICT...           the patterns tree (PatternsTree.h:90-94): per
 *                                 pattern in add order, u32 code and u32 code of
 *                                 its PatternsTreeNode->parent (0 = the root)
 *   suffix OUT SEED NPAIRS DICT...  is_pattern_suffix (PatternsTree.c:485-494)
 *                                 on sampled pairs: u32 code(first), code(second),
 *                                 result; half the firsts are on the second's
 *                                 parent chain, 1/16 are NULL
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "conf.h"
#include "mps.h"
#include "mpac.h"
#include "parser.h"
#include "PatternsTree.h"
#include "streamgen.h"

static size_t n_added = 0;
static void* ac_obj = NULL;
static pattern_id_t* added = NULL;  /* ids in add order (the tree's nodes) */
static size_t added_cap = 0;

static void add_cb(void* obj, char* pat, size_t len, pattern_id_t id) {
    (void)obj;
    if (n_added == added_cap) {
        added_cap = added_cap ? 2 * added_cap : 4096;
        added = (pattern_id_t*)realloc(added, added_cap * sizeof(pattern_id_t));
    }
    added[n_added] = id;
    ++n_added;
    mps_table[MPS_AC].add_pattern(ac_obj, pat, len, id);
}

static Conf* build(char** dicts, int n) {
    Conf* conf = (Conf*)calloc(1, sizeof(Conf));
    conf->dictionary_files = dicts;
    conf->n_dictionary_files = (size_t)n;
    mps_table_setup();
    ac_obj = mps_table[MPS_AC].create();
    (void)patterns_tree_build(conf, NULL, add_cb);
    mps_table[MPS_AC].compile(ac_obj);
    mps_table[MPS_AC].reset(ac_obj);
    return conf;
}

static inline uint32_t code_of(pattern_id_t id) {
    if (id == NULL) return 0;
    PatternsTreeNode* n = (PatternsTreeNode*)id;
    if (n->parent == NULL) return 0; /* the root: null internal id {-1,-1} (PatternsTree.c:69, 247) */
    return (uint32_t)((n->pattern_id.file_number << 24) | n->pattern_id.line_number);
}

static unsigned char* read_file(const char* path, size_t* n) {
    FILE* f = fopen(path, "rb");
    if (!f) { perror(path); exit(1); }
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char* b = (unsigned char*)malloc(sz > 0 ? (size_t)sz : 1);
    if (sz > 0 && fread(b, 1, (size_t)sz, f) != (size_t)sz) { perror(path); exit(1); }
    fclose(f);
    *n = (size_t)sz;
    return b;
}

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

int main(int argc, char** argv) {
    if (argc < 3) { fprintf(stderr, "usage: see header\n"); return 2; }
    const char* mode = argv[1];
    if (!strcmp(mode, "dense") && argc >= 5) {
        build(argv + 4, argc - 4);
        size_t n;
        unsigned char* s = read_file(argv[3], &n);
        uint32_t* out = (uint32_t*)malloc((n ? n : 1) * 4);
        pattern_id_t (*rc)(void*, char) = mps_table[MPS_AC].read_char;
        for (size_t j = 0; j < n; ++j) out[j] = code_of(rc(ac_obj, (char)s[j]));
        FILE* f = fopen(argv[2], "wb");
        fwrite(out, 4, n, f);
        fclose(f);
        return 0;
    }
    if (!strcmp(mode, "gen") && argc == 6) {
        uint64_t seed = strtoull(argv[3], 0, 0);
        int m = atoi(argv[4]);
        size_t n = strtoull(argv[5], 0, 0);
        unsigned char* b = (unsigned char*)malloc(n ? n : 1);
        oracle_gen_stream(b, 0, n, seed, m);
        FILE* f = fopen(argv[2], "wb");
        fwrite(b, 1, n, f);
        fclose(f);
        return 0;
    }
    if (!strcmp(mode, "digest") && argc >= 6) {
        uint64_t seed = strtoull(argv[2], 0, 0);
        int m = atoi(argv[3]);
        size_t n = strtoull(argv[4], 0, 0);
        build(argv + 5, argc - 5);
        unsigned char* b = (unsigned char*)malloc(n ? n : 1);
        oracle_gen_stream(b, 0, n, seed, m);
        pattern_id_t (*rc)(void*, char) = mps_table[MPS_AC].read_char;
        uint64_t h = 1469598103934665603ULL, nonnull = 0;
        int shown = 0;
        printf("{\"seed\": %llu, \"mode\": %d, \"n\": %zu, \"first\": [", (unsigned long long)seed, m, n);
        for (size_t j = 0; j < n; ++j) {
            uint32_t c = code_of(rc(ac_obj, (char)b[j]));
            for (int k = 0; k < 4; ++k) { h ^= (c >> (8 * k)) & 0xFF; h *= 1099511628211ULL; }
            if (c) {
                ++nonnull;
                if (shown < 1000) { printf("%s[%zu, %u]", shown ? ", " : "", j, c); ++shown; }
            }
        }
        printf("], \"nonnull\": %llu, \"fnv1a64\": \"%016llx\"}\n", (unsigned long long)nonnull,
               (unsigned long long)h);
        return 0;
    }
    if (!strcmp(mode, "stats")) {
        Conf* conf = build(argv + 2, argc - 2);
        size_t mem = mps_table[MPS_AC].total_mem(ac_obj);
        /* mpac.c:328-332: sizeof(AC) + n_states * sizeof(State) */
        printf("{\"unique\": %zu, \"ac_total_mem\": %zu, \"max_len\": %zu}\n", n_added, mem, conf->max_pat_len);
        return 0;
    }
    if (!strcmp(mode, "parse") && argc == 3) {
        FILE* fp = fopen(argv[2], "r");
        if (!fp) { perror(argv[2]); return 1; }
        char* line = NULL;
        size_t cap = 0, ln = 0;
        ssize_t got;
        while ((got = getline(&line, &cap, fp)) != -1) {
            char* pat = NULL;
            ++ln;
            if (line[got - 1] == '\n') --got;
            size_t len = parse_pattern_from_line(line, (size_t)got, &pat);
            if (len) {
                printf("%zu ", ln);
                for (size_t k = 0; k < len; ++k) printf("%02x", (unsigned char)pat[k]);
                printf("\n");
            }
            if (pat) free(pat);
        }
        return 0;
    }
    if (!strcmp(mode, "time") && argc >= 6) {
        uint64_t seed = strtoull(argv[2], 0, 0);
        int m = atoi(argv[3]);
        size_t n = strtoull(argv[4], 0, 0);
        double tb = now();
        build(argv + 5, argc - 5);
        double build_s = now() - tb;
        unsigned char* b = (unsigned char*)malloc(n ? n : 1);
        oracle_gen_stream(b, 0, n, seed, m);
        pattern_id_t (*rc)(void*, char) = mps_table[MPS_AC].read_char;
        uint64_t nonnull = 0;
        double t0 = now();
        for (size_t j = 0; j < n; ++j) nonnull += rc(ac_obj, (char)b[j]) != NULL;
        double dt = now() - t0;
        printf("{\"bytes\": %zu, \"seconds\": %.6f, \"MBps\": %.3f, \"nonnull\": %llu, \"build_s\": %.3f}\n",
               n, dt, n / dt / 1e6, (unsigned long long)nonnull, build_s);
        return 0;
    }
    if (!strcmp(mode, "timefile") && argc >= 4) {
        size_t n;
        unsigned char* b = read_file(argv[2], &n);
        double tb = now();
        build(argv + 3, argc - 3);
        double build_s = now() - tb;
        pattern_id_t (*rc)(void*, char) = mps_table[MPS_AC].read_char;
        uint64_t nonnull = 0;
        double t0 = now();
        for (size_t j = 0; j < n; ++j) nonnull += rc(ac_obj, (char)b[j]) != NULL;
        double dt = now() - t0;
        printf("{\"bytes\": %zu, \"seconds\": %.6f, \"MBps\": %.3f, \"nonnull\": %llu, \"build_s\": %.3f}\n",
               n, dt, n / dt / 1e6, (unsigned long long)nonnull, build_s);
        return 0;
    }
    if (!strcmp(mode, "parents") && argc >= 4) {
        build(argv + 3, argc - 3);
        FILE* f = fopen(argv[2], "wb");
        if (!f) { perror(argv[2]); return 1; }
        for (size_t k = 0; k < n_added; ++k) {
            PatternsTreeNode* nd = (PatternsTreeNode*)added[k];
            uint32_t rec[2] = {code_of(added[k]), code_of(nd->parent)};
            fwrite(rec, 4, 2, f);
        }
        fclose(f);
        return 0;
    }
    if (!strcmp(mode, "suffix") && argc >= 6) {
        uint64_t seed = strtoull(argv[3], 0, 0);
        size_t npairs = strtoull(argv[4], 0, 0);
        build(argv + 5, argc - 5);
        FILE* f = fopen(argv[2], "wb");
        if (!f) { perror(argv[2]); return 1; }
        for (size_t k = 0; k < npairs && n_added; ++k) {
            uint64_t r = oracle_splitmix64((seed << 32) ^ k);
            pattern_id_t second = added[r % n_added];
            pattern_id_t first;
            if (((r >> 40) & 15) == 0) {
                first = NULL;
            } else if ((r >> 44) & 1) { /* a node on second's parent chain, below the root */
                size_t depth = 0;
                for (PatternsTreeNode* c = (PatternsTreeNode*)second; c->parent; c = c->parent) ++depth;
                size_t up = (size_t)((r >> 48) % depth);
                PatternsTreeNode* c = (PatternsTreeNode*)second;
                while (up--) c = c->parent;
                first = c;
            } else {
                first = added[(r >> 20) % n_added];
            }
            uint32_t rec[3] = {code_of(first), code_of(second), (uint32_t)is_pattern_suffix(first, second)};
            fwrite(rec, 4, 3, f);
        }
        fclose(f);
        return 0;
    }
    fprintf(stderr, "bad arguments\n");
    return 2;
}
