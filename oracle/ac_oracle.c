/*
 * ac_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's exact per-byte matcher (Aho-Corasick),
 * used as the parity oracle by tests/, by __graft_entry__.smoke() and as the
 * "port" CPU baseline leg of bench.py.  Nothing in the product
 * (patternmatching_amd/) links, loads or calls this file.
 *
 * Parity pinning: checked against golden vectors produced by the reference
 * itself (oracle/_ref/ref_driver built from /root/reference/Core/src by
 * oracle/Makefile) -- see tests/golden/ and tests/test_oracle_golden.py.
 *
 * What it restates (reference file:line):
 *   - dictionary line parser ............ Core/src/parser.c:25 (skip_spaces),
 *                                          :36-46 (get_binary_val), :63-99
 *   - line reading (getline, 1-based line numbers, one trailing '\n'
 *     stripped) ......................... Core/src/PatternsTree.c:260-291
 *   - de-duplication, first (file,line) wins
 *                                          Core/src/PatternsTree.c:193-196
 *   - AC trie insert .................... Core/src/mpac.c:257-273
 *   - BFS failure + suffix ("output") links
 *                                          Core/src/mpac.c:172-210
 *   - read_char (failure while-loop, stay at root, return id of suffix link)
 *                                          Core/src/mpac.c:304-319
 *   - reset per stream file ............. Core/src/mpac.c:339-342,
 *                                          Core/src/measure.c:274-275
 *
 * Differences that cannot change the output: children are u32 (the
 * reference uses size_t), states are numbered in creation order (the
 * reference renumbers in DFS order, mpac.c:147-161), and the pattern id is
 * an index into a (file,line) table rather than a PatternsTreeNode pointer.
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <time.h>

/* ------------------------------------------------------------------ parser */

static int oracle_hexval(int ch) { /* parser.c:36-46 */
    if (ch >= '0' && ch <= '9') return ch - '0';
    if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
    if (ch >= 'A' && ch <= 'F') return ch - 'A' + 10;
    return -1;
}

/*
 * parser.c:63-99.  `line` holds n bytes; the reference may read line[n]
 * (the stripped '\n' or getline's NUL), which is neither a space nor a hex
 * digit -- at() models it as 0.  Returns the pattern length, 0 when the line
 * is rejected or empty.  `out` needs room for n bytes.
 */
size_t oracle_parse_line(const unsigned char* line, size_t n, unsigned char* out) {
#define at(k) ((k) < n ? (int)line[(k)] : 0)
    size_t len = 0, pos = 0;
    if (n == 0) return 0;
    while (pos < n) {
        if (line[pos] == '|') {
            ++pos;
            while (pos < n && line[pos] != '|') {
                int hi, lo;
                while (at(pos) == ' ') ++pos;
                hi = oracle_hexval(at(pos));
                ++pos;
                while (at(pos) == ' ') ++pos;
                lo = oracle_hexval(at(pos));
                ++pos;
                if (hi < 0 || lo < 0) return 0;
                out[len++] = (unsigned char)(hi * 16 + lo);
            }
            if (pos >= n) return 0;
            ++pos;
        } else {
            out[len++] = line[pos++];
        }
    }
    return len;
#undef at
}

/* --------------------------------------------------------- pattern table */

typedef struct {
    unsigned char* bytes;
    uint32_t len;
    uint32_t file;
    uint32_t line;
} OPattern;

typedef struct {
    OPattern* v;
    size_t n, cap;
    /* open-addressing set of indices into v, keyed by the bytes */
    int64_t* slots;
    size_t nslots;
    size_t max_len;
} OPatternSet;

static uint64_t fnv1a(const unsigned char* p, size_t n) {
    uint64_t h = 1469598103934665603ULL;
    for (size_t i = 0; i < n; ++i) { h ^= p[i]; h *= 1099511628211ULL; }
    return h;
}

static void pset_grow(OPatternSet* s) {
    size_t ns = s->nslots ? s->nslots * 2 : 1 << 16;
    int64_t* sl = (int64_t*)malloc(ns * sizeof(int64_t));
    for (size_t i = 0; i < ns; ++i) sl[i] = -1;
    for (size_t i = 0; i < s->n; ++i) {
        uint64_t h = fnv1a(s->v[i].bytes, s->v[i].len) & (ns - 1);
        while (sl[h] >= 0) h = (h + 1) & (ns - 1);
        sl[h] = (int64_t)i;
    }
    free(s->slots);
    s->slots = sl;
    s->nslots = ns;
}

/* PatternsTree.c:193-196: an identical byte string already present wins. */
static void pset_add(OPatternSet* s, const unsigned char* p, size_t len, uint32_t file, uint32_t line) {
    if (2 * (s->n + 1) > s->nslots) pset_grow(s);
    uint64_t h = fnv1a(p, len) & (s->nslots - 1);
    while (s->slots[h] >= 0) {
        OPattern* q = &s->v[s->slots[h]];
        if (q->len == len && memcmp(q->bytes, p, len) == 0) return;
        h = (h + 1) & (s->nslots - 1);
    }
    if (s->n == s->cap) {
        s->cap = s->cap ? s->cap * 2 : 1024;
        s->v = (OPattern*)realloc(s->v, s->cap * sizeof(OPattern));
    }
    OPattern* q = &s->v[s->n];
    q->bytes = (unsigned char*)malloc(len);
    memcpy(q->bytes, p, len);
    q->len = (uint32_t)len;
    q->file = file;
    q->line = line;
    s->slots[h] = (int64_t)s->n;
    s->n++;
    if (len > s->max_len) s->max_len = len;
}

/* PatternsTree.c:260-291: getline loop, 1-based numbering, strip one '\n'. */
static int pset_fill_file(OPatternSet* s, const char* path, uint32_t file_index) {
    FILE* fp = fopen(path, "rb");
    if (!fp) return -1;
    char* line = NULL;
    size_t cap = 0;
    ssize_t got;
    uint32_t line_num = 0;
    unsigned char* pat = NULL;
    size_t pat_cap = 0;
    while ((got = getline(&line, &cap, fp)) != -1) {
        ++line_num;
        size_t n = (size_t)got;
        if (line[n - 1] == '\n') --n;
        if (n + 1 > pat_cap) { pat_cap = n + 1; pat = (unsigned char*)realloc(pat, pat_cap); }
        size_t len = oracle_parse_line((const unsigned char*)line, n, pat);
        if (len) pset_add(s, pat, len, file_index, line_num);
    }
    free(pat);
    free(line);
    fclose(fp);
    return 0;
}

/* ------------------------------------------------------------ automaton */

typedef struct {
    uint32_t children[256]; /* mpac.c:43-48 (size_t there) */
    uint32_t failure;
    uint32_t suffix_link;
    uint32_t id;            /* pattern index + 1, 0 = null_pattern_id */
} OState;

typedef struct OracleAC {
    OPatternSet pats;
    OState* st;
    size_t n_states, cap_states;
    uint32_t cur;            /* mpac.c:53 current_state */
} OracleAC;

static uint32_t ac_new_state(OracleAC* ac) {
    if (ac->n_states == ac->cap_states) {
        ac->cap_states = ac->cap_states ? ac->cap_states * 2 : 4096;
        ac->st = (OState*)realloc(ac->st, ac->cap_states * sizeof(OState));
        if (!ac->st) { fprintf(stderr, "oracle: out of memory\n"); exit(1); }
    }
    memset(&ac->st[ac->n_states], 0, sizeof(OState));
    return (uint32_t)ac->n_states++;
}

/* mpac.c:257-273 */
static void ac_insert(OracleAC* ac, const unsigned char* p, size_t len, uint32_t id) {
    uint32_t cur = 0;
    size_t i = 0;
    while (i < len && ac->st[cur].children[p[i]]) cur = ac->st[cur].children[p[i++]];
    for (; i < len; ++i) {
        uint32_t nx = ac_new_state(ac);
        ac->st[cur].children[p[i]] = nx;
        cur = nx;
    }
    ac->st[cur].id = id;
}

/* mpac.c:172-210: BFS; failure of depth-1 states is the root; suffix link is
 * the state itself when it carries an id, else the failure's suffix link. */
static void ac_links(OracleAC* ac) {
    OState* s = ac->st;
    uint32_t* q = (uint32_t*)malloc(ac->n_states * sizeof(uint32_t));
    size_t qh = 0, qt = 0;
    s[0].failure = 0;
    s[0].suffix_link = 0;
    for (int c = 0; c < 256; ++c) {
        uint32_t ch = s[0].children[c];
        if (ch) {
            q[qt++] = ch;
            s[ch].failure = 0;
            s[ch].suffix_link = s[ch].id ? ch : 0;
        }
    }
    while (qh < qt) {
        uint32_t cur = q[qh++];
        for (int c = 0; c < 256; ++c) {
            uint32_t ch = s[cur].children[c];
            if (!ch) continue;
            uint32_t fs = s[cur].failure;
            while (!s[fs].children[c] && fs) fs = s[fs].failure;
            s[ch].failure = s[fs].children[c];
            s[ch].suffix_link = s[ch].id ? ch : s[s[ch].failure].suffix_link;
            q[qt++] = ch;
        }
    }
    free(q);
}

OracleAC* oracle_ac_build(const char** dict_paths, int n_dicts) {
    OracleAC* ac = (OracleAC*)calloc(1, sizeof(OracleAC));
    for (int f = 0; f < n_dicts; ++f) {
        if (pset_fill_file(&ac->pats, dict_paths[f], (uint32_t)f) != 0) {
            fprintf(stderr, "oracle: cannot open dictionary %s\n", dict_paths[f]);
            free(ac);
            return NULL;
        }
    }
    ac_new_state(ac); /* root */
    for (size_t i = 0; i < ac->pats.n; ++i)
        ac_insert(ac, ac->pats.v[i].bytes, ac->pats.v[i].len, (uint32_t)(i + 1));
    ac_links(ac);
    ac->cur = 0;
    return ac;
}

size_t oracle_ac_n_states(const OracleAC* ac) { return ac->n_states; }
size_t oracle_ac_n_patterns(const OracleAC* ac) { return ac->pats.n; }
size_t oracle_ac_max_len(const OracleAC* ac) { return ac->pats.max_len; }
void oracle_ac_reset(OracleAC* ac) { ac->cur = 0; }

/* Pattern table access: idx is 0-based in first-occurrence order. */
uint32_t oracle_ac_pattern(const OracleAC* ac, size_t idx, uint32_t* file, uint32_t* line,
                           unsigned char* buf, uint32_t buf_cap) {
    const OPattern* p = &ac->pats.v[idx];
    if (file) *file = p->file;
    if (line) *line = p->line;
    if (buf) memcpy(buf, p->bytes, p->len < buf_cap ? p->len : buf_cap);
    return p->len;
}

/* mpac.c:304-319 */
static inline uint32_t ac_step(const OState* s, uint32_t* curp, unsigned char uc) {
    uint32_t cur = *curp;
    while (!s[cur].children[uc] && cur) cur = s[cur].failure;
    if (s[cur].children[uc]) cur = s[cur].children[uc];
    *curp = cur;
    return s[s[cur].suffix_link].id;
}

/* The reference's per-byte read_char, reached through a function pointer as
 * in measure.c:292-294.  Returns pattern index + 1, 0 for null. */
uint32_t oracle_ac_read_char(void* obj, char c) {
    OracleAC* ac = (OracleAC*)obj;
    return ac_step(ac->st, &ac->cur, (unsigned char)c);
}

static inline uint32_t code_of(const OracleAC* ac, uint32_t id) {
    if (!id) return 0;
    const OPattern* p = &ac->pats.v[id - 1];
    return (p->file << 24) | p->line;
}

/* Dense output: per position (file << 24 | line) of the longest pattern
 * ending there, or 0.  State carries across calls (like read_char). */
void oracle_ac_scan(OracleAC* ac, const unsigned char* buf, size_t n, uint32_t* out_code) {
    for (size_t j = 0; j < n; ++j) out_code[j] = code_of(ac, ac_step(ac->st, &ac->cur, buf[j]));
}

/* Same, but the 1-based pattern index (first-occurrence order) instead of a code. */
void oracle_ac_scan_idx(OracleAC* ac, const unsigned char* buf, size_t n, uint32_t* out_idx) {
    for (size_t j = 0; j < n; ++j) out_idx[j] = ac_step(ac->st, &ac->cur, buf[j]);
}

/* ---------------------------------------------------- CPU baseline timing */

typedef struct {
    const OracleAC* ac;
    const unsigned char* buf;
    size_t lo, hi, warm_lo; /* scan [warm_lo, hi), count only [lo, hi) */
    uint64_t nonnull;
} ShardArg;

static void* shard_run(void* p) {
    ShardArg* a = (ShardArg*)p;
    uint32_t (*read_char)(void*, char) = oracle_ac_read_char; /* measure.c:292-294 */
    OracleAC local = *a->ac;                                  /* private cursor, shared table */
    local.cur = 0;
    uint64_t cnt = 0;
    for (size_t j = a->warm_lo; j < a->lo; ++j) read_char(&local, (char)a->buf[j]);
    for (size_t j = a->lo; j < a->hi; ++j) cnt += read_char(&local, (char)a->buf[j]) != 0;
    a->nonnull = cnt;
    return NULL;
}

/*
 * Time the per-byte loop over buf[0..n) with `threads` threads, each taking a
 * contiguous shard and warming up max_len-1 bytes early (SURVEY.md §0.1
 * "Shard exactness").  Returns seconds (CLOCK_MONOTONIC); *nonnull gets the
 * number of positions with a match.
 */
double oracle_ac_time_scan(const OracleAC* ac, const unsigned char* buf, size_t n, int threads,
                           uint64_t* nonnull) {
    if (threads < 1) threads = 1;
    size_t warm = ac->pats.max_len ? ac->pats.max_len - 1 : 0;
    ShardArg* args = (ShardArg*)calloc((size_t)threads, sizeof(ShardArg));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    for (int t = 0; t < threads; ++t) {
        args[t].ac = ac;
        args[t].buf = buf;
        args[t].lo = n * (size_t)t / (size_t)threads;
        args[t].hi = n * (size_t)(t + 1) / (size_t)threads;
        args[t].warm_lo = args[t].lo > warm ? args[t].lo - warm : 0;
    }
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, shard_run, &args[t]);
    uint64_t total = 0;
    for (int t = 0; t < threads; ++t) { pthread_join(th[t], NULL); total += args[t].nonnull; }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (nonnull) *nonnull = total;
    free(args);
    free(th);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

void oracle_ac_free(OracleAC* ac) {
    if (!ac) return;
    for (size_t i = 0; i < ac->pats.n; ++i) free(ac->pats.v[i].bytes);
    free(ac->pats.v);
    free(ac->pats.slots);
    free(ac->st);
    free(ac);
}

/* FNV-1a-64 of a byte buffer (the golden digests of oracle/ref_driver.c). */
uint64_t oracle_fnv1a64(const unsigned char* p, size_t n) {
    uint64_t h = 1469598103934665603ULL;
    for (size_t i = 0; i < n; ++i) { h ^= p[i]; h *= 1099511628211ULL; }
    return h;
}
