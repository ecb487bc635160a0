/*
 * pm_measure.c -- stream driver, accuracy scoring and CSV report.
 *
 * Mirrors Core/src/measure.c:
 *   measure_single_instance_stats  measure.c:241-311  -> measure_one()
 *     reset per stream file (:274-275), chunked read (:284) with matcher
 *     state carried across chunks, timed matcher loop (:290-297), the
 *     reliable instance's untimed pass (:300-302) and scoring (:303)
 *   measure_instances_stats        measure.c:324-332  -> pm_measure_all()
 *   write_stats_to_file            measure.c:339-408  -> pm_write_stats()
 *   parse_arguments                parser.c:104-161   -> pm_parse_args()
 *
 * Changes, each deliberate:
 *   - the per-byte loop becomes one read_block call per chunk when the
 *     plugin has it (both GPU plugins do); chunks default to 16 MiB instead
 *     of 100 KiB (a GPU launch needs a large batch; state still carries);
 *   - clock() (process CPU time) becomes CLOCK_MONOTONIC wall time, plus
 *     the plugin's own hipEvent device time; perf_event columns become GPU
 *     columns (device seconds, GB/s, non-null positions, bytes);
 *   - the reliable instance is the GPU Aho-Corasick DFA (PM_MPS_HIP_AC);
 *   - the CSV is opened O_TRUNC with mode 0644 (measure.c:348 uses no mode);
 *   - the dictionary/stream name arrays hold pointers (parser.c:124-125
 *     allocates n bytes for n pointers);
 *   - -a selects algorithms (the reference always runs every one).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include "pm_host.h"
#include "pm_hip.h"

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void usage(const char* prog) {
    fprintf(stderr, "Usage: %s [OPTION]...\n", prog);
    fprintf(stderr, "options:\n");
    fprintf(stderr, "  -d FILE               use FILE as one of the dictionary files (can be used many times).\n");
    fprintf(stderr, "  -s FILE               use FILE as one of the stream files (can be used many times).\n");
    fprintf(stderr, "  -o FILE               set FILE to be the output file.\n");
    fprintf(stderr, "  -v                    set verbose to true (print more information)\n");
    fprintf(stderr, "  -a LIST               algorithms: rt, ac, auto or all (comma separated; default all)\n");
    fprintf(stderr, "  -B BYTES              stream chunk per read_block call (default 16777216)\n");
    fprintf(stderr, "  -g DEVICE             HIP device index (default 0)\n");
    fprintf(stderr, "  -m FILE               dump per-position (file<<24|line) u32 codes of the first algorithm\n");
}

static char* dupstr(const char* s) {
    char* r = (char*)malloc(strlen(s) + 1);
    strcpy(r, s);
    return r;
}

int pm_parse_args(int argc, char** argv, PmConf* conf) {
    int opt;
    size_t n_dict = 0, n_stream = 0, n_out = 0;
    memset(conf, 0, sizeof(*conf));
    conf->algo_mask = (1 << PM_MPS_SIZE) - 1;
    conf->chunk_bytes = (size_t)16 << 20;
    opterr = 0;
    optind = 1;
    while ((opt = getopt(argc, argv, "d:s:o:va:B:g:m:")) != -1) {
        if (opt == 'd') ++n_dict;
        else if (opt == 's') ++n_stream;
        else if (opt == 'o') ++n_out;
    }
    if (n_out > 1) {
        fprintf(stderr, "Error: have more than one output file\n\n");
        usage(argv[0]);
        return 1;
    }
    conf->dict_files = (char**)calloc(n_dict + 1, sizeof(char*));
    conf->stream_files = (char**)calloc(n_stream + 1, sizeof(char*));
    optind = 1;
    while ((opt = getopt(argc, argv, "d:s:o:va:B:g:m:")) != -1) {
        switch (opt) {
        case 'd': conf->dict_files[conf->n_dict_files++] = dupstr(optarg); break;
        case 's': conf->stream_files[conf->n_stream_files++] = dupstr(optarg); break;
        case 'o': conf->output_file = dupstr(optarg); break;
        case 'm': conf->matches_file = dupstr(optarg); break;
        case 'v': conf->verbose = 1; break;
        case 'B': conf->chunk_bytes = strtoull(optarg, NULL, 0); break;
        case 'g': conf->device = atoi(optarg); break;
        case 'a': {
            int mask = 0;
            char* s = dupstr(optarg);
            for (char* tok = strtok(s, ","); tok; tok = strtok(NULL, ",")) {
                if (!strcmp(tok, "all")) mask |= (1 << PM_MPS_SIZE) - 1;
                else if (!strcmp(tok, "rt")) mask |= 1 << PM_MPS_HIP_RT;
                else if (!strcmp(tok, "ac")) mask |= 1 << PM_MPS_HIP_AC;
                else if (!strcmp(tok, "auto")) mask |= 1 << PM_MPS_HIP_AUTO;
                else {
                    fprintf(stderr, "Unknown algorithm %s.\n\n", tok);
                    free(s);
                    usage(argv[0]);
                    return 1;
                }
            }
            free(s);
            conf->algo_mask = mask;
            break;
        }
        case '?':
            if (optopt == 'd' || optopt == 's' || optopt == 'o' || optopt == 'a' || optopt == 'B' ||
                optopt == 'g' || optopt == 'm')
                fprintf(stderr, "Option -%c must have argument.\n\n", optopt);
            else
                fprintf(stderr, "Unknown option -%c.\n\n", optopt);
            usage(argv[0]);
            return 1;
        default:
            usage(argv[0]);
            return 1;
        }
    }
    if (conf->chunk_bytes < 16) conf->chunk_bytes = 16;
    if (!conf->n_dict_files) {
        fprintf(stderr, "Error: no dictionary file (-d)\n\n");
        usage(argv[0]);
        return 1;
    }
    return 0;
}

void pm_conf_free(PmConf* conf) {
    for (size_t i = 0; i < conf->n_dict_files; ++i) free(conf->dict_files[i]);
    for (size_t i = 0; i < conf->n_stream_files; ++i) free(conf->stream_files[i]);
    free(conf->dict_files);
    free(conf->stream_files);
    free(conf->output_file);
    free(conf->matches_file);
}

static void feed_cb(void* obj, char* pat, size_t len, pm_pattern_id_t id) {
    PmMpsInstance* inst = (PmMpsInstance*)obj;
    pm_mps_table[inst->algo].add_pattern(inst->obj, pat, len, id);
}

static void run_block(const PmMpsElem* e, void* obj, const char* buf, size_t n, pm_pattern_id_t* out) {
    if (e->read_block) {
        e->read_block(obj, buf, n, out);
    } else {
        pm_pattern_id_t (*rc)(void*, char) = e->read_char; /* measure.c:292-294 */
        for (size_t j = 0; j < n; ++j) out[j] = rc(obj, buf[j]);
    }
}

int pm_measure_all(PmConf* conf, PmDict* dict, PmInstanceStats* stats) {
    PmMpsInstance inst[PM_MPS_SIZE];
    PmMpsInstance reliable = {NULL, PM_MPS_HIP_AC};
    size_t chunk = conf->chunk_bytes;
    char* buf = (char*)malloc(chunk);
    pm_pattern_id_t* algo_res = (pm_pattern_id_t*)malloc(chunk * sizeof(pm_pattern_id_t));
    pm_pattern_id_t* real_res = (pm_pattern_id_t*)malloc(chunk * sizeof(pm_pattern_id_t));
    uint32_t* codes = conf->matches_file ? (uint32_t*)malloc(chunk * sizeof(uint32_t)) : NULL;
    FILE* mf = NULL;
    int first_algo = -1;
    if (!buf || !algo_res || !real_res || (conf->matches_file && !codes)) {
        fprintf(stderr, "pm: cannot allocate %zu-byte stream buffers\n", chunk);
        return 1;
    }
    if (conf->matches_file) {
        mf = fopen(conf->matches_file, "wb");
        if (!mf) { fprintf(stderr, "pm: cannot open %s: %s\n", conf->matches_file, strerror(errno)); return 1; }
    }
    memset(stats, 0, PM_MPS_SIZE * sizeof(PmInstanceStats));

    /* init_mps (mps.c:44-54, 64-77, 84-96): create, feed, compile */
    for (int a = 0; a < PM_MPS_SIZE; ++a) {
        inst[a].algo = a;
        inst[a].obj = NULL;
        if (!(conf->algo_mask & (1 << a))) continue;
        if (first_algo < 0) first_algo = a;
        inst[a].obj = pm_mps_table[a].create();
        /* the device-time columns: time every read_block launch, small ones too */
        (void)pm_hip_set_option(inst[a].obj, "host_events", 1);
        pm_dict_feed(dict, &inst[a], feed_cb);
        pm_mps_table[a].compile(inst[a].obj);
    }
    if (inst[PM_MPS_HIP_AC].obj) {
        reliable.obj = inst[PM_MPS_HIP_AC].obj;
    } else {
        reliable.obj = pm_mps_table[PM_MPS_HIP_AC].create();
        pm_dict_feed(dict, &reliable, feed_cb);
        pm_mps_table[PM_MPS_HIP_AC].compile(reliable.obj);
    }

    for (int a = 0; a < PM_MPS_SIZE; ++a) {
        const PmMpsElem* e = &pm_mps_table[a];
        PmInstanceStats* st = &stats[a];
        if (!inst[a].obj) continue;
        if (conf->verbose) { printf("Measuring algorithm %s...", e->name); fflush(stdout); }
        for (size_t f = 0; f < conf->n_stream_files; ++f) {
            int fd = open(conf->stream_files[f], O_RDONLY);
            if (fd == -1) {
                fprintf(stderr, "can't open stream file %s: %s\n", conf->stream_files[f], strerror(errno));
                exit(EXIT_FAILURE);
            }
            e->reset(inst[a].obj); /* measure.c:274-275 */
            if (reliable.obj != inst[a].obj) pm_mps_table[reliable.algo].reset(reliable.obj);
            for (;;) {
                size_t got = 0;
                while (got < chunk) { /* fill the chunk (read() may return short) */
                    ssize_t r = read(fd, buf + got, chunk - got);
                    if (r < 0) {
                        fprintf(stderr, "can't read from stream file %s: %s\n", conf->stream_files[f],
                                strerror(errno));
                        exit(EXIT_FAILURE);
                    }
                    if (r == 0) break;
                    got += (size_t)r;
                }
                if (got == 0) break;
                double t0 = now_s();
                run_block(e, inst[a].obj, buf, got, algo_res);
                st->wall_seconds += now_s() - t0;
                st->bytes += got;
                if (reliable.obj != inst[a].obj) {
                    run_block(&pm_mps_table[reliable.algo], reliable.obj, buf, got, real_res);
                    pm_success_rate_add(&st->sr, algo_res, real_res, got);
                } else {
                    st->sr.success += got; /* the reliable instance scores itself */
                }
                for (size_t j = 0; j < got; ++j) st->nonnull += algo_res[j] != PM_NULL_PATTERN_ID;
                if (mf && a == first_algo) {
                    for (size_t j = 0; j < got; ++j) codes[j] = pm_pattern_code(algo_res[j]);
                    fwrite(codes, sizeof(uint32_t), got, mf);
                }
                if (got < chunk) break;
            }
            close(fd);
            {
                /* < 0: some launches were not timed ("host_events" off) --
                 * the device columns are then unmeasured */
                const double ds = pm_hip_device_seconds(inst[a].obj);
                if (ds < 0 || st->device_seconds < 0) st->device_seconds = -1.0;
                else st->device_seconds += ds;
            }
            st->out_width = pm_hip_last_out_width(inst[a].obj);
        }
        st->total_mem = e->total_mem(inst[a].obj);
        if (conf->verbose) printf("Done\n");
    }
    if (mf) fclose(mf);
    free(buf);
    free(algo_res);
    free(real_res);
    free(codes);
    return 0;
}

static void put(int fd, const char* s) {
    size_t n = strlen(s);
    while (n) {
        ssize_t w = write(fd, s, n);
        if (w <= 0) return;
        s += w;
        n -= (size_t)w;
    }
}

int pm_write_stats(const PmConf* conf, const PmInstanceStats* stats) {
    int fd = STDOUT_FILENO;
    char buf[512];
    if (conf->output_file) {
        if (conf->verbose) printf("opening file %s to write results\n", conf->output_file);
        fd = open(conf->output_file, O_WRONLY | O_CREAT | O_TRUNC, 0644);
        if (fd == -1) {
            fprintf(stderr, "failed to open results file %s: %s\n", conf->output_file, strerror(errno));
            return 1;
        }
    }
    put(fd, "Algorithm,Time (in secs),Total Memory Used,False Positive Rate,False Negative Rate,"
            "Partial Success Rate,Device Time (in secs),Device GB/s,Non-null Positions,Bytes,"
            "Device Roofline Fraction,GPU");
    for (int a = 0; a < PM_MPS_SIZE; ++a) {
        const PmInstanceStats* s = &stats[a];
        if (!(conf->algo_mask & (1 << a))) continue;
        uint64_t sum = s->sr.success + s->sr.false_pos + s->sr.false_neg + s->sr.partial_suc;
        long double den = sum ? (long double)sum : 1.0L;
        /* roofline: the algorithmic bytes per position the device scans
         * moved (1 read + the id width they wrote: u16 gids for pattern-id
         * output of dictionaries under 65,536 patterns, else u32) over the
         * device time, against the HBM peak bench.py uses too */
        const double dev_gbs = s->device_seconds > 0 ? (double)s->bytes / s->device_seconds / 1e9 : 0.0;
        const double per_pos = 1.0 + (s->out_width ? s->out_width : 4);
        /* device columns: empty when the device time was not measured */
        char dt[32] = "", dg[32] = "", df[32] = "";
        if (s->device_seconds >= 0) {
            snprintf(dt, sizeof(dt), "%.6f", s->device_seconds);
            snprintf(dg, sizeof(dg), "%.3f", dev_gbs);
            snprintf(df, sizeof(df), "%.6g", dev_gbs * per_pos / PM_HBM_PEAK_GBS);
        }
        snprintf(buf, sizeof(buf), "\n%s,%.6f,%zu,%.6Lf,%.6Lf,%.6Lf,%s,%s,%llu,%llu,%s,%d", pm_mps_table[a].name,
                 s->wall_seconds, s->total_mem, (long double)s->sr.false_pos / den,
                 (long double)s->sr.false_neg / den, (long double)s->sr.partial_suc / den, dt, dg,
                 (unsigned long long)s->nonnull, (unsigned long long)s->bytes, df, conf->device);
        put(fd, buf);
    }
    put(fd, "\n");
    if (fd != STDOUT_FILENO) close(fd);
    return 0;
}
