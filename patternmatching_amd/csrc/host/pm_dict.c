/*
 * pm_dict.c -- dictionary parsing, de-duplication and the pattern-id model.
 *
 * Behaviour follows the reference:
 *   pm_parse_line        Core/src/parser.c:63-99
 *   pm_dict_load         Core/src/PatternsTree.c:260-312
 *   de-duplication       Core/src/PatternsTree.c:193-196 (first (file,line) wins)
 *   parent links         Core/src/PatternsTree.c:1-33 ("patterns tree": a node's
 *                        parent is its longest proper suffix that is a pattern)
 *   pm_pattern_is_suffix Core/src/PatternsTree.c:485-494
 *   pm_success_rate_add  Core/src/measure.c:174-190
 *
 * The reference builds the patterns tree as a linked suffix tree and walks
 * it recursively; here the same information is a flat array of PmPattern
 * records with a parent pointer, built with one hash set.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <errno.h>
#include "pm_host.h"

static int hexval(int ch) {
    if (ch >= '0' && ch <= '9') return ch - '0';
    if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
    if (ch >= 'A' && ch <= 'F') return ch - 'A' + 10;
    return -1;
}

/*
 * Rules (parser.c:63-99): literal bytes pass through; '|' opens a hex block
 * in which each byte is <spaces> nibble <spaces> nibble; any other
 * character where a nibble is expected -- including the closing '|' after
 * a space -- rejects the whole line, as does a block left open.  The
 * reference may look at line[n] (the stripped '\n' or NUL); that byte is
 * modelled as 0, which is neither a space nor a nibble.
 */
size_t pm_parse_line(const unsigned char* line, size_t n, unsigned char* out) {
    size_t len = 0, pos = 0;
    if (n == 0) return 0;
    while (pos < n) {
        if (line[pos] != '|') {
            out[len++] = line[pos++];
            continue;
        }
        ++pos;
        while (pos < n && line[pos] != '|') {
            int hi, lo;
            while (pos < n && line[pos] == ' ') ++pos;
            hi = pos < n ? hexval(line[pos]) : -1;
            ++pos;
            while (pos < n && line[pos] == ' ') ++pos;
            lo = pos < n ? hexval(line[pos]) : -1;
            ++pos;
            if (hi < 0 || lo < 0) return 0;
            out[len++] = (unsigned char)((hi << 4) | lo);
        }
        if (pos >= n) return 0; /* block never closed */
        ++pos;
    }
    return len;
}

/* ------------------------------------------------------------- hash set */

static uint64_t hash_bytes(const unsigned char* p, size_t n) {
    uint64_t h = 0xcbf29ce484222325ULL;
    for (size_t i = 0; i < n; ++i) { h ^= p[i]; h *= 0x100000001b3ULL; }
    return h ^ (h >> 29);
}

static int64_t find_slot(const PmDict* d, const unsigned char* p, size_t len, uint64_t* slot_out) {
    uint64_t mask = d->nslots - 1, h = hash_bytes(p, len) & mask;
    while (d->slots[h] >= 0) {
        const struct PmPattern* q = &d->pats[d->slots[h]];
        if (q->len == len && memcmp(q->bytes, p, len) == 0) { *slot_out = h; return d->slots[h]; }
        h = (h + 1) & mask;
    }
    *slot_out = h;
    return -1;
}

static void rehash(PmDict* d) {
    size_t ns = d->nslots ? d->nslots * 2 : (size_t)1 << 16;
    free(d->slots);
    d->slots = (int64_t*)malloc(ns * sizeof(int64_t));
    if (!d->slots) { perror("pm: out of memory"); exit(EXIT_FAILURE); }
    for (size_t i = 0; i < ns; ++i) d->slots[i] = -1;
    d->nslots = ns;
    for (size_t i = 0; i < d->n; ++i) {
        uint64_t s;
        find_slot(d, d->pats[i].bytes, d->pats[i].len, &s);
        d->slots[s] = (int64_t)i;
    }
}

PmDict* pm_dict_new(void) {
    PmDict* d = (PmDict*)calloc(1, sizeof(PmDict));
    if (!d) { perror("pm: out of memory"); exit(EXIT_FAILURE); }
    rehash(d);
    return d;
}

int pm_dict_add(PmDict* d, const unsigned char* bytes, size_t len, uint32_t file, uint32_t line) {
    uint64_t s;
    if (len == 0) return 0;
    if (2 * (d->n + 1) > d->nslots) rehash(d);
    if (find_slot(d, bytes, len, &s) >= 0) return 0; /* PatternsTree.c:193-196 */
    if (d->n == d->cap) {
        /* pattern records must not move once handed out as ids: grow only
         * before pm_dict_finalize/pm_dict_feed */
        d->cap = d->cap ? d->cap * 2 : 4096;
        d->pats = (struct PmPattern*)realloc(d->pats, d->cap * sizeof(struct PmPattern));
        if (!d->pats) { perror("pm: out of memory"); exit(EXIT_FAILURE); }
    }
    struct PmPattern* p = &d->pats[d->n];
    p->bytes = (unsigned char*)malloc(len);
    if (!p->bytes) { perror("pm: out of memory"); exit(EXIT_FAILURE); }
    memcpy(p->bytes, bytes, len);
    p->len = (uint32_t)len;
    p->file = file;
    p->line = line;
    p->index = (uint32_t)d->n;
    p->parent = NULL;
    d->slots[s] = (int64_t)d->n;
    d->n++;
    if (len > d->max_len) d->max_len = len;
    return 1;
}

static int load_one(PmDict* d, const char* path, uint32_t file_index, char* err, size_t errlen) {
    FILE* fp = fopen(path, "rb");
    if (!fp) {
        snprintf(err, errlen, "failed to open dictionary file %s: %s", path, strerror(errno));
        return -1;
    }
    char* line = NULL;
    size_t cap = 0, pcap = 0;
    unsigned char* pat = NULL;
    ssize_t got;
    uint32_t line_num = 0;
    while ((got = getline(&line, &cap, fp)) != -1) {
        size_t n = (size_t)got, len;
        ++line_num;
        d->lines_total++;
        if (line[n - 1] == '\n') --n; /* PatternsTree.c:277 */
        if (n + 1 > pcap) {
            pcap = 2 * (n + 1);
            pat = (unsigned char*)realloc(pat, pcap);
        }
        len = pm_parse_line((const unsigned char*)line, n, pat);
        if (len) pm_dict_add(d, pat, len, file_index, line_num);
        else if (n) d->lines_rejected++;
    }
    free(pat);
    free(line);
    fclose(fp);
    return 0;
}

void pm_dict_finalize(PmDict* d) {
    /* parent = longest proper suffix that is a pattern: try suffixes from
     * the longest down; the first hit is the parent. */
    for (size_t i = 0; i < d->n; ++i) {
        struct PmPattern* p = &d->pats[i];
        p->parent = NULL;
        for (uint32_t k = 1; k < p->len; ++k) {
            uint64_t s;
            int64_t hit = find_slot(d, p->bytes + k, p->len - k, &s);
            if (hit >= 0) { p->parent = &d->pats[hit]; break; }
        }
    }
}

PmDict* pm_dict_load(const char* const* paths, size_t n_paths, char* err, size_t errlen) {
    PmDict* d = pm_dict_new();
    for (size_t f = 0; f < n_paths; ++f) {
        if (load_one(d, paths[f], (uint32_t)f, err, errlen) != 0) {
            pm_dict_free(d);
            return NULL;
        }
    }
    pm_dict_finalize(d);
    return d;
}

void pm_dict_feed(PmDict* d, void* obj, void (*add)(void*, char*, size_t, pm_pattern_id_t)) {
    char* scratch = (char*)malloc(d->max_len ? d->max_len : 1);
    for (size_t i = 0; i < d->n; ++i) {
        memcpy(scratch, d->pats[i].bytes, d->pats[i].len);
        add(obj, scratch, d->pats[i].len, &d->pats[i]);
    }
    free(scratch);
}

void pm_dict_free(PmDict* d) {
    if (!d) return;
    for (size_t i = 0; i < d->n; ++i) free(d->pats[i].bytes);
    free(d->pats);
    free(d->slots);
    free(d);
}

/* PatternsTree.c:485-494: walk parents of `second`; equality counts. */
int pm_pattern_is_suffix(pm_pattern_id_t first, pm_pattern_id_t second) {
    if (first == NULL) return 0;
    for (const struct PmPattern* cur = second; cur; cur = cur->parent)
        if (cur == first) return 1;
    return 0;
}

uint32_t pm_pattern_code(pm_pattern_id_t id) {
    return id ? (id->file << 24) | id->line : 0;
}

/* measure.c:174-190 */
void pm_success_rate_add(PmSuccessRate* sr, const pm_pattern_id_t* algo, const pm_pattern_id_t* real,
                         size_t n) {
    for (size_t i = 0; i < n; ++i) {
        if (real[i] == algo[i]) sr->success++;
        else if (pm_pattern_is_suffix(algo[i], real[i])) sr->partial_suc++;
        else if (algo[i] == PM_NULL_PATTERN_ID) sr->false_neg++;
        else sr->false_pos++;
    }
}
