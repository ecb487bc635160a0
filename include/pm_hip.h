/*
 * pm_hip.h -- C-ABI of the MI355X (gfx950) matcher library libpm.so.
 *
 * Two groups of entry points:
 *
 * 1. The plugin functions behind pm_mps_table (include/pm_mps.h).  Each one
 *    replaces the reference function named beside it, with the same
 *    argument meaning and the same "no error channel" behaviour: a HIP
 *    failure prints a message and exits(1), like FatalExit()
 *    (/root/reference/Core/src/util.h:37-39).
 *
 *      reference (Core/src/)            this library
 *      mpac.c:236  ac_create            pm_hip_rt_create / pm_hip_ac_create
 *      mpac.c:257  ac_add_pattern       pm_hip_add_pattern
 *      mpac.c:282  ac_compile           pm_hip_compile
 *      mpac.c:304  ac_read_char         pm_hip_read_char
 *      (none)                           pm_hip_read_block (batched read_char)
 *      mpac.c:328  ac_total_mem         pm_hip_total_mem
 *      mpac.c:339  ac_reset             pm_hip_reset
 *      mpac.c:349  ac_free              pm_hip_free
 *      mpac.c:358  mps_ac_register      pm_mps_hip_rt_register / pm_mps_hip_ac_register
 *
 *    The same functions serve both algorithms; the object created decides
 *    which kernel runs.
 *
 * 2. Device-resident batch entry points for callers that keep the stream in
 *    HBM (bench.py, the multi-GPU driver).  They return 0 on success and a
 *    negative code on failure (message via pm_hip_last_error()).
 *
 * Pattern ids inside the library are "gids": 1..n_patterns, 0 = no match.
 * pm_hip_gid_index maps a gid back to the 0-based add_pattern call order.
 */
#ifndef PM_HIP_H
#define PM_HIP_H

#include <stddef.h>
#include <stdint.h>
#include "pm_mps.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- 1. plugin ABI (MpsElem members) ---------------------------------- */
void* pm_hip_rt_create(void);
void* pm_hip_ac_create(void);
/* Both kernels; each launch picks one: the RT kernel, unless the last RT
 * launch spilled more than 10% of its positions (dense deep matches), when
 * the next 64 launches run the AC-DFA kernel.  reset()
 * forgets the choice. */
void* pm_hip_auto_create(void);
void pm_hip_add_pattern(void* obj, char* pat, size_t len, pm_pattern_id_t id);
void pm_hip_compile(void* obj);
pm_pattern_id_t pm_hip_read_char(void* obj, char c);
void pm_hip_read_block(void* obj, const char* buf, size_t n, pm_pattern_id_t* out);
size_t pm_hip_total_mem(void* obj);
void pm_hip_reset(void* obj);
void pm_hip_free(void* obj);

void pm_mps_hip_rt_register(PmMpsElem* slot);
void pm_mps_hip_ac_register(PmMpsElem* slot);
void pm_mps_hip_auto_register(PmMpsElem* slot);

/* ---- 2. batch / introspection ----------------------------------------- */

/* Same as pm_hip_read_block but writes gids (u32, 0 = none) instead of
 * pattern ids; state carries across calls exactly like read_block. */
int pm_hip_read_block_gid(void* obj, const uint8_t* buf, size_t n, uint32_t* out_gid);

/*
 * Scan positions [pos0, pos0+n) of the device buffer d_text.
 *   stream_start  index in d_text of the stream's first byte (<= pos0);
 *                 bytes in [stream_start, pos0) are context: they are looked
 *                 back at but produce no output.  Context of
 *                 pm_hip_max_pattern_len()-1 bytes makes the result exact for
 *                 a position anywhere in a longer stream.
 *   pos0          must be a multiple of 16; d_text 16-byte aligned and
 *                 readable up to round_up(pos0+n, 16).
 *   d_out         n u32 gids (16-byte aligned), or NULL for count-only.
 *   d_count       device u64, incremented by the number of non-null
 *                 positions (may be NULL).
 *   hip_stream    hipStream_t to launch on (NULL = default stream).
 * Asynchronous: returns after the launch.
 */
int pm_hip_scan_device(void* obj, const uint8_t* d_text, int64_t stream_start, int64_t pos0,
                       int64_t n, uint32_t* d_out, unsigned long long* d_count, void* hip_stream);
/* The same with u16 gids (n * 2 bytes, 16-byte aligned): the compact id
 * stream for dictionaries of fewer than 65536 patterns (every reference
 * dictionary; the merged snort + ET set has 55,580).  Returns -4 when the
 * dictionary is larger. */
int pm_hip_scan_device16(void* obj, const uint8_t* d_text, int64_t stream_start, int64_t pos0,
                         int64_t n, uint16_t* d_out, unsigned long long* d_count, void* hip_stream);

/* Accuracy of one dense u32 gid stream against a reference one, on the
 * device (the scoring of Core/src/measure.c:174-190 with is_pattern_suffix,
 * PatternsTree.c:485-494): per position, equal -> success; d_algo's pattern
 * a proper suffix (ancestor) of d_real's -> partial; d_algo none -> false
 * negative; else false positive.  Also all-matches: the number of patterns
 * ending at each position of d_real (its suffix chain), summed.  Both
 * arrays come from objects compiled from the same patterns in the same add
 * order (RT and AC objects then share gids).  d_counts (5 device u64) +=
 * {success, partial, false_neg, false_pos, all_matches}.  16-B aligned.
 * Asynchronous. */
int pm_hip_score_device(void* obj, const uint32_t* d_algo, const uint32_t* d_real, int64_t n,
                        unsigned long long* d_counts, void* hip_stream);
/* Per-pattern occurrence counts of a dense u32 gid stream (all-matches
 * expansion: each position counts its answer and every pattern on the
 * answer's suffix chain).  d_hist: n_patterns + 1 device u64, indexed by gid
 * (pm_hip_gid_index maps a gid to its add order), accumulated.  Asynchronous. */
int pm_hip_pattern_counts_device(void* obj, const uint32_t* d_ids, int64_t n, unsigned long long* d_hist,
                                 void* hip_stream);
/* ac / auto kinds: keep the kernel picked for pm_hip_scan_device launches
 * (pm_hip_auto_create) for at least the next `launches` launches, so a timed
 * region never re-measures.  Returns the held kernel (1 = reverse trie,
 * 2 = AC dense rows, 3 = AC rows + records, 4 = the same with every record
 * loaded as a 16-B half, 5 = the same with deep records' 64-B blocks,
 * 6 = the same with every record as a 16-B half and two segments per lane), 0
 * when the object has no choice
 * to make (rt kind, or a single DFA form), -1 while the pick is still being
 * measured (launch more, synchronize, and ask again). */
int pm_hip_hold_choice(void* obj, int launches);
/* Before a scan_device launch is captured into a HIP graph (hipStreamBeginCapture,
 * torch.cuda.graph): allocates the scratch captured launches of the rt / auto
 * kinds use (the reverse-trie kernel's spill regions, sized for a launch of
 * any length: 512 MiB on 256 CUs), since nothing may be allocated while a
 * stream captures.  Without it a captured scan_device that would run the
 * chunked reverse-trie kernel (more than 256 Ki positions, the "rt_small_max"
 * option) returns -5 and launches nothing; smaller launches, and launches of
 * an auto object holding a DFA form, need none.  Direct launches allocate
 * their own scratch per stream (pm_hip_scratch_bytes).  0 on success. */
int pm_hip_prepare_capture(void* obj);
/* Device scratch the object holds beside its tables (pm_hip_table_bytes):
 * the capture scratch, the per-stream scratch of direct scan_device
 * launches and the read_block pipeline's staging.  Bytes. */
size_t pm_hip_scratch_bytes(void* obj);
/* Compiled-image cache: compile() keeps the flattened tables of each
 * dictionary in DIR (pm-<kind>-<hash>.img, keyed by the patterns in add order)
 * and reuses them; without a call here, $PM_IMAGE_CACHE names the directory
 * (unset = no cache).  A file that does not validate is rebuilt. */
void pm_hip_set_image_cache(void* obj, const char* dir);
/* 1 when the last compile() loaded its tables from the cache. */
int pm_hip_image_cache_hit(void* obj);
/* Start-up cost of the last compile(): *compile_ms = the whole call (gid
 * numbering, flattening or the cache read, the uploads), *upload_ms = its
 * host-to-device table copies (pm_hip_table_bytes bytes).  Wall time, ms.
 * 0, or -1 before compile().  (No reference counterpart: the reference's
 * init_mps, mps.c:109-113, is untimed.) */
int pm_hip_compile_stats(void* obj, double* compile_ms, double* upload_ms);
/* The patterns-tree parent of a gid (longest proper suffix pattern, 0 = none);
 * UINT32_MAX when out of range. */
uint32_t pm_hip_parent_gid(void* obj, uint32_t gid);

/* Device-side synthetic stream, identical to pm_gen_stream_host(). */
int pm_hip_gen_stream_device(uint8_t* d_dst, uint64_t offset, uint64_t n, uint64_t seed, int mode,
                             void* hip_stream);
void pm_gen_stream_host(uint8_t* dst, uint64_t offset, uint64_t n, uint64_t seed, int mode);
/* The "lines" stream: 1 KiB blocks of the object's patterns
 * drawn at random (splitmix64), each followed by '\n' -- dense deep matches
 * without the period of a tiled file.  Device and host give the same bytes. */
int pm_hip_gen_lines_device(void* obj, uint8_t* d_dst, uint64_t n, uint64_t seed, void* hip_stream);
void pm_gen_lines_host(void* obj, uint8_t* dst, uint64_t n, uint64_t seed);
/* The same bytes from a loaded dictionary (its patterns in first-occurrence
 * order, as pm_dict_feed adds them), without a matcher object or a device. */
struct PmDict;
void pm_gen_lines_dict(const struct PmDict* d, uint8_t* dst, uint64_t n, uint64_t seed);

uint32_t pm_hip_n_patterns(void* obj);
uint32_t pm_hip_max_pattern_len(void* obj);
/* gid (1..n) -> 0-based add_pattern order; returns UINT32_MAX if out of range */
uint32_t pm_hip_gid_index(void* obj, uint32_t gid);
/* Which kernel a compiled object runs: 1 = reverse trie, 2 = AC DFA,
 * 3 = auto (both, picked per launch). */
int pm_hip_kernel_kind(void* obj);
/* The kernel of the object's last launch: 1 = reverse trie, 2 = AC DFA
 * (0 before any). */
int pm_hip_kernel_last(void* obj);
/* DFA form of the last launch: 1 = dense rows, 2 = rows + 16-B records
 * (pm_flatten.h), 0 = the RT kernel ran. */
int pm_hip_dfa_form_last(void* obj);
/* The sparse form's kernel of the last launch that ran it ("sparse_kernel"
 * option numbering: 1 fallback-linked, 2 lock-step 8-B units, 3 lock-step
 * 16-B records; 0 before any). */
int pm_hip_sparse_kernel_last(void* obj);
/* Seconds of device time of the scan kernels issued through read_block
 * since the last reset (hipEvent based); -1 when some of those launches were
 * not timed (the "host_events" option off): the device time is then
 * unmeasured, not zero. */
double pm_hip_device_seconds(void* obj);
/* Bytes per position the last read_block's device scans wrote: 2 (u16 gids,
 * dictionaries of < 65,536 patterns, pattern-id output) or 4; 0 before any. */
int pm_hip_last_out_width(void* obj);
/* The HBM roofline every report prices against: MI355X HBM3E peak, GB/s
 * (MI355X_MICROARCH.md), shared by the CLI's CSV and bench.py. */
#define PM_HBM_PEAK_GBS 8000.0
double pm_hip_hbm_peak_gbs(void);
/* Bytes of flattened tables per kind, for DESIGN/bench reporting. */
size_t pm_hip_table_bytes(void* obj);
const char* pm_hip_last_error(void);
/* Returns the number of HIP devices (0 when none); never exits. */
int pm_hip_device_count(void);
/* hipSetDevice for C callers (the CLI's -g); 0 on success. */
int pm_hip_set_device(int device);

/* Per-object options (set before or after compile(); they change which
 * product kernel or host path the object's launches take, never a result).
 * Returns 0, or -1 for an unknown name or a value out of range.
 *   "dfa_form"        ac / auto kinds: 0 = timed choice between the DFA's
 *                     dense rows and sparse form (default), 1 = dense rows,
 *                     2 = sparse form (the pick measures again)
 *   "sparse_kernel"   the sparse form's kernel: 0 = the product choice
 *                     (default: the fallback-linked form where the object
 *                     has it), 1 = fallback-linked form, 2 = lock-step 8-B
 *                     units, 3 = lock-step 16-B records.  A forced kernel
 *                     whose image the object lacks (the FL form needs fewer
 *                     than 65,536 rows and gids, the 8-B units ids below
 *                     2^20) is not an error: the launch runs the product
 *                     choice, and pm_hip_sparse_kernel_last reports which
 *                     kernel ran
 *   "fl_hold"         the fallback-linked kernel's record loads outside the
 *                     picks' trials: 2 = deep records' 32-B blocks (0, the
 *                     default), 4 = 64-B blocks, 1 = every record as a 16-B
 *                     half (the ac / auto picks time 1 and 4, and 1 with two
 *                     chains per lane)
 *   "fl_chains"       segments per lane of the fallback-linked kernel
 *                     outside the picks' trials: 1 (0, the default) or 2
 *                     (dfa_fl2_kernel; with fl_hold 1 or 2)
 *   "dfa_sync"        1 = DFA warm-ups start at the last synchronizing 3-gram
 *                     (default), 0 = max_len - 1 bytes back
 *   "rt_small_max"    reverse-trie launches of at most this many positions
 *                     run one thread per position (-1 = default 256 Ki,
 *                     0 = never)
 *   "spill_cap_chunks" the reverse-trie spill region per wave, 1,024-position
 *                     chunks (1..16; 0 = the default fill: 4 for the count,
 *                     2 with ids -- a full region is resolved where the
 *                     other waves' streaming hides it)
 *   "host_spin" / "host_gid16" / "host_events" / "host_pool"
 *                     read_block's host path (-1 = the environment's
 *                     default, 0 / 1; csrc/pm_plugin.hip HostOpts).
 *                     host_events (default off): small read_block calls
 *                     (<= 256 Ki positions) record timing events for
 *                     pm_hip_device_seconds; the CLI turns it on
 *   "host_serve"      rt objects, and auto objects while their pick holds
 *                     the reverse trie: small read_block calls go to a resident
 *                     server grid polling a doorbell in host memory instead
 *                     of a launch per call (-1 = PM_HOST_SERVE, default 1;
 *                     0 = a launch per call).  Calls timed by host_events
 *                     take the launch path.  DESIGN.md §3
 *   "serve_idle_us"   the server grid exits after this long without a call
 *                     (-1 = PM_HOST_SERVE_IDLE_US, default 2,000; >= 10);
 *                     the next call launches it again */
int pm_hip_set_option(void* obj, const char* name, int64_t value);
/* The resident server of an rt / auto object (the "host_serve" option): grids
 * launched and requests served since the object was made.  0. */
int pm_hip_serve_stats(void* obj, uint64_t* launches, uint64_t* calls);
/* The reverse-trie kernel's streaming floor on this GPU: the same chunk
 * loop's loads and stores with no lookups (its d_out values are not match
 * ids) over d_text[0, n).  bench.py's live floor.  0 on success. */
int pm_hip_streaming_floor_device(void* obj, const uint8_t* d_text, int64_t n, void* d_out, int out_width,
                                  void* hip_stream);
/* The gather ceiling of the object's sparse DFA image (the fallback-linked
 * form; ac / auto kinds): one 1,024-lane workgroup per CU, each lane making
 * `steps` dependent 4-B loads at hashed, uniform indices over the image --
 * the deep kernel's loads without its logic, over its own table.  bench.py
 * times it beside the DFA legs: steps * 1,024 * CUs loads per launch.
 * d_sink: one device u32 (not written in practice).  0, -2 without the
 * image, -3 on a launch error. */
int pm_hip_gather_ceiling_device(void* obj, int steps, uint32_t* d_sink, void* hip_stream);
/* The read_block host path's breakdown since the last call -- out5 =
 * {staging s, enqueue s, wait s, result copy / map s, calls} -- then reset
 * and turn the accounting on (on != 0) or off.  Process-wide accounting;
 * changes no result. */
void pm_hip_host_profile(int on, double* out5);

/* ---- 3. host-only table images (no device; used by the CPU test suite
 *         to check the flattener, and by DESIGN.md sizing) ------------ */
/* kind 1 = reverse-trie image, 2 = AC dense-DFA image */
void* pm_flat_build(const char* const* pats, const uint32_t* lens, size_t n, int kind);
/* The same through the compiled-image cache in cache_dir (NULL = none). */
void* pm_flat_build_cached(const char* const* pats, const uint32_t* lens, size_t n, int kind, const char* cache_dir);
int pm_flat_cache_hit(void* handle);
int pm_flat_fits(void* handle);
/* States with full rows in the sparse DFA form (0 when it has none). */
uint32_t pm_flat_dfa_sparse_rows(void* handle);
/* name: "t12" "filt" "t3h" "rec" "next" "out" "sblock" "sout" "index_of_gid" "parent" "depth";
 * returns element count */
size_t pm_flat_array(void* handle, const char* name, const void** data, size_t* elem_size);
/* read_char's host step (the per-byte path, csrc/pm_hoststep.h) over a
 * whole text from the stream start: the reverse-trie walk (RT image) or
 * the DFA step (its sparse form; dense rows when dense_rows != 0 or it has
 * none).  out_gid: n gids.  Returns 0, or -1 when the RT image does not fit. */
int pm_flat_host_scan(void* handle, const uint8_t* text, size_t n, uint32_t* out_gid, int dense_rows);
void pm_flat_free(void* handle);

#ifdef __cplusplus
}
#endif
#endif /* PM_HIP_H */
