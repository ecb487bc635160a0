/*
 * pm_host.h -- host-side front end of the matcher (plain C, in libpm.so and
 * the `pm` CLI).  It replaces the reference's layers L2/L5/L6
 * (SURVEY.md §1):
 *
 *   pm_parse_line         parser.c:63-99 (get_binary_val :36-46,
 *                         skip_spaces :25), byte-exact rules of SURVEY §8a A11
 *   pm_dict_load          PatternsTree.c:260-312 (getline loop, 1-based line
 *                         numbers, one trailing '\n' stripped, first
 *                         occurrence of a byte string wins :193-196)
 *   pm_dict_feed          PatternsTree.c:378-403 (callback feed of every
 *                         unique pattern) via mps.c:64-77
 *   PmPattern.parent      the patterns tree as an array: longest proper
 *                         suffix that is itself a pattern (PatternsTree.c:1-33)
 *   pm_pattern_is_suffix  PatternsTree.c:485-494
 *   pm_success_rate_add   measure.c:174-190
 *   pm_measure_*          measure.c:241-332 stream loop and
 *                         measure.c:339-408 CSV writer
 *   pm_parse_args         parser.c:104-161 (-d -s -o -v) plus -a -B -g -m
 */
#ifndef PM_HOST_H
#define PM_HOST_H

#include <stddef.h>
#include <stdint.h>
#include "pm_mps.h"

#ifdef __cplusplus
extern "C" {
#endif

/* A unique dictionary pattern.  pm_pattern_id_t points at one of these. */
struct PmPattern {
    uint32_t file;             /* 0-based index of its -d file (first occurrence) */
    uint32_t line;             /* 1-based line number (first occurrence) */
    uint32_t len;
    uint32_t index;            /* 0-based, first-occurrence order */
    struct PmPattern* parent;  /* longest proper suffix that is a pattern, or NULL */
    unsigned char* bytes;
};

typedef struct PmDict {
    struct PmPattern* pats;
    size_t n;
    size_t max_len;
    size_t lines_total;
    size_t lines_rejected;     /* non-empty lines the parser rejected */
    /* private */
    size_t cap;
    int64_t* slots;
    size_t nslots;
} PmDict;

/* Returns the pattern length; 0 = rejected or empty.  out: room for n bytes. */
size_t pm_parse_line(const unsigned char* line, size_t n, unsigned char* out);

/* Load dictionaries in -d order.  NULL on failure (message in err). */
PmDict* pm_dict_load(const char* const* paths, size_t n_paths, char* err, size_t errlen);
/* Add a pattern from memory (file/line are caller-chosen ids). Returns 1 if new. */
int pm_dict_add(PmDict* d, const unsigned char* bytes, size_t len, uint32_t file, uint32_t line);
PmDict* pm_dict_new(void);
/* Compute parent links (call once after the last add). */
void pm_dict_finalize(PmDict* d);
/* Feed every unique pattern to add(obj, bytes, len, id) in first-occurrence
 * order.  bytes points into a scratch buffer (borrowed, like the reference's
 * PatternsTree.c:393-400). */
void pm_dict_feed(PmDict* d, void* obj, void (*add)(void*, char*, size_t, pm_pattern_id_t));
void pm_dict_free(PmDict* d);

int pm_pattern_is_suffix(pm_pattern_id_t first, pm_pattern_id_t second);
/* (file << 24) | line, the golden-fixture code; 0 for NULL. */
uint32_t pm_pattern_code(pm_pattern_id_t id);

typedef struct {
    uint64_t success, partial_suc, false_neg, false_pos;
} PmSuccessRate;

void pm_success_rate_add(PmSuccessRate* sr, const pm_pattern_id_t* algo, const pm_pattern_id_t* real,
                         size_t n);

/* ---- stream driver (measure.c) -------------------------------------- */
typedef struct {
    char** dict_files;
    size_t n_dict_files;
    char** stream_files;
    size_t n_stream_files;
    char* output_file;
    char* matches_file;        /* -m: dump per-position codes of the first algorithm */
    int verbose;
    int algo_mask;             /* bit k = run pm_mps_table[k]; default all */
    size_t chunk_bytes;        /* -B, default 64 MiB */
    int device;                /* -g */
} PmConf;

typedef struct {
    double wall_seconds;       /* read_block/read_char calls, CLOCK_MONOTONIC */
    double device_seconds;     /* kernel time reported by the plugin (0 if n/a, < 0 if not measured) */
    uint64_t bytes;
    uint64_t nonnull;
    size_t total_mem;
    PmSuccessRate sr;
    int out_width;             /* id bytes per position the device scans wrote (pm_hip_last_out_width) */
} PmInstanceStats;

/* Returns 0 on success; prints usage and returns nonzero on bad input. */
int pm_parse_args(int argc, char** argv, PmConf* conf);
void pm_conf_free(PmConf* conf);
/* Runs every selected algorithm over every stream file, scoring each against
 * the reliable instance (PM_MPS_HIP_AC).  stats has PM_MPS_SIZE entries. */
int pm_measure_all(PmConf* conf, PmDict* dict, PmInstanceStats* stats);
int pm_write_stats(const PmConf* conf, const PmInstanceStats* stats);

#ifdef __cplusplus
}
#endif
#endif /* PM_HOST_H */
