// pm_plugin.hip -- the GPU matcher objects behind the plugin ABI
// (include/pm_hip.h, include/pm_mps.h).
//
// Object life cycle = the reference's (Core/src/mps.h:29-69):
// create -> add_pattern x P (bytes borrowed: copied here) -> compile (flatten
// + upload to HBM) -> per stream file: reset, then read_char / read_block
// with state carried across calls -> total_mem -> free.
//
// The carried state is not an automaton state: for the reverse-trie kernel
// it is the last max_len-1 stream bytes (every position only looks back
// that far), and the DFA kernel re-derives its state from the same bytes
// (warm-up).  read_block therefore stages [history | new bytes] in device
// memory and scans the new positions with the history as context.
//
// Errors: the ABI has no error channel; every HIP failure prints and exits
// (util.h:37-39 FatalExit semantics).  There is no CPU fallback: without a
// HIP device, create() fails loudly.
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <unistd.h>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "pm_flatten.h"
#include "pm_hip.h"
#include "pm_host.h"
#include "pm_hoststep.h"
#include "pm_kernels.h"
#include "pm_streamgen.h"

#ifndef PM_NT_IDS
#define PM_NT_IDS 1  // read_block's id map with non-temporal stores (0: plain stores)
#endif

namespace {

thread_local char g_err[512] = "";

[[noreturn]] void fatal(const char* what, hipError_t e) {
    std::fprintf(stderr, "pm_hip: %s failed: %s\n", what, hipGetErrorString(e));
    std::fflush(stderr);
    std::exit(EXIT_FAILURE);
}

#define PM_CHECK(call)                            \
    do {                                          \
        hipError_t e_ = (call);                   \
        if (e_ != hipSuccess) fatal(#call, e_);   \
    } while (0)

enum Kind { KIND_RT = 1, KIND_AC = 2, KIND_AUTO = 3 };

// KIND_AUTO holds both images and picks a kernel per launch: the RT kernel
// reports how many candidates it spilled (its queue overflowed: dense deep
// matches -- DESIGN.md §5; a count-only launch, which queues nothing,
// reports the positions its tail walked) and its time; when a launch
// reported more than AUTO_SPILL_FRAC of its positions, the next launches
// try the AC-DFA kernel in each of its forms (dense rows, then rows +
// records, pm_flatten.h), AUTO_TRIAL launches each, the last one timed (the
// first pays cold caches), and whichever of the measured kernels took least
// per position runs the next AUTO_HOLD launches; then RT measures again.
// (Deep input is where the DFA can win: on the tiled shipped stream the
// dense form is 2.2x RT, on the non-periodic lines stream the sparse form
// is 1.4x RT and 2x the dense form.)  KIND_AC runs the same trials of its
// two forms without the RT launch.  Counts and times come back through
// pinned memory and events, waited for at the next launch (see launch()).
// reset() (a new stream) clears it.
constexpr double AUTO_SPILL_FRAC = 0.10;
constexpr int AUTO_TRIAL = 2;
constexpr int AUTO_HOLD = 64;
// A choice that the next measurement confirms is held twice as long (up to
// AUTO_HOLD << AUTO_STREAK_MAX launches): on a long deep stream each
// measurement costs an RT launch and the DFA trials -- on the lines stream
// ~3x and ~1-3.5x the held kernel's time -- so a fixed hold of 64 launches
// spent ~20% of the time measuring.  reset() (a new stream) starts over.
// Launches below AUTO_SMALL_LAUNCH positions (read_block's 100 KiB chunks,
// measure.c:77) double only up to AUTO_STREAK_MAX_SMALL: 512 launches of
// 100 KiB are 50 MiB before the next measurement instead of 400 MiB, so a
// stream that turns from ASCII to deep lines is re-measured soon.
constexpr int AUTO_STREAK_MAX = 6;
constexpr int AUTO_STREAK_MAX_SMALL = 3;
constexpr int64_t AUTO_SMALL_LAUNCH = 4ll << 20;
// CAND_SPARSE16: the sparse form's fallback-linked kernel holding every
// record as a 16-B half (DfaDev::flhold 1, FlImage::deep_g ignored): faster
// where walks rarely stay in a record's block (snort, the tiled shipped
// stream 3.48 -> 3.24 ms, ASCII 2.90 -> 2.78), slower on the lines stream
// (4.99 -> 5.42).  CAND_SPARSE64: the same kernel holding deep records'
// 64-B blocks (flhold 4): faster where walks run down long chains (snort
// lines 4.99 -> 4.87, merged lines 5.43 -> 5.13), slower elsewhere (shipped
// 3.64, ASCII 3.07).  profiles/r05/ab/fl_hold_1_2_4.jsonl; all three timed
// beside the other forms.
// CAND_FL2: the same form, two chains per lane (dfa_fl2_kernel, records as
// 16-B halves): faster where the walks' table lines stay in L2 (snort, the
// tiled shipped stream 3.23 -> 2.54 ms, count 2.64 -> 1.96), slower where
// they come from further out (lines 4.87 -> 6.31; ASCII 2.78 -> 3.30);
// profiles/r06/fl2/.
enum Cand {
    CAND_RT = 0,
    CAND_DENSE = 1,
    CAND_SPARSE = 2,
    CAND_SPARSE16 = 3,
    CAND_SPARSE64 = 4,
    CAND_FL2 = 5,
    NCAND = 6
};

struct AutoPick {
    unsigned long long* d_spill = nullptr;  // device counter of the last measured RT launch
    unsigned long long* h_spill = nullptr;  // pinned copy
    hipEvent_t ev = nullptr;                // the copy has landed
    hipEvent_t t0[NCAND] = {}, t1[NCAND] = {};  // timing of each candidate's measured launch
    bool pending = false;     // a measured RT launch (spill count + time) in flight
    bool timing = false;      // the DFA trials are launched, their times in flight
    int queue[NCAND] = {};    // DFA forms to try, in order
    int nq = 0, qi = 0;       // forms queued / started
    int trial = 0;            // launches left of the form being tried (the last one timed)
    int64_t n_of[NCAND] = {};
    double ns[NCAND] = {};    // measured ns per position (0 = not measured this round)
    int hold = 0;             // launches left on the chosen candidate
    int chosen = CAND_RT;
    int prev = -1;            // the choice the previous measurement made
    int streak = 0;           // measurements in a row that made the same choice
    int last = 0;             // KIND_RT / KIND_AC of the last launch
    int last_form = 0;        // DFA form of the last launch: 1 dense rows, 2 sparse (0: RT)
};

// read_block pipeline blocks (positions): the upload, kernel and download of
// block k overlap the host finishing block k-1.  Gid output
// is downloaded straight into the caller's array (no host work per block);
// pattern-id output is mapped on the host, so smaller blocks overlap more
// of that mapping with the transfers.
constexpr size_t PIPE_GID_POSITIONS = (size_t)16 << 20;
constexpr size_t PIPE_ID_POSITIONS = (size_t)8 << 20;
// Blocks up to this size go through the pinned staging buffers both ways
// (one host memcpy each side, one DMA each way) instead of the runtime's
// own staging of pageable memory, whose fixed cost per copy dominates a
// small call such as the reference's 100 KiB chunks (measure.c:284):
// +10-18% there; at 1 MiB the single-threaded 4 MiB result copy made the
// gid path 37% slower (profiles/r02/host_path_small_staging_ab.txt).
constexpr size_t PIPE_SMALL_POSITIONS = (size_t)256 << 10;

// One pipeline slot: pinned host and device staging for one block and its
// own stream, so two blocks are in flight.
struct PipeSlot {
    uint8_t* d_stage = nullptr;
    uint32_t* d_res = nullptr;
    uint8_t* h_stage = nullptr;
    uint32_t* h_res = nullptr;
    size_t cap = 0;  // positions
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    uint32_t* spill = nullptr;  // RT deep-walk scratch of this slot's launches
    int64_t spill_cap = 0;
    AutoPick pick;
    bool busy = false;
    bool staged = false;    // small block: results land in h_res, copied out by finish
    bool served = false;    // ... by the object's resident server, in its own h_res
    bool timed = false;     // ev0 / ev1 bracket the launch (device seconds)
    int w = 4;              // bytes per result position in h_res / d_res
    size_t off = 0, m = 0;  // block = positions [off, off + m) of the call
};

// RT scratch of the scan_device launches on one stream.  Launches on one
// stream are ordered, so they share it; launches on different streams may
// run at once, so each stream has its own (two launches sharing one wrote
// each other's spill items).  Past PM_STREAM_SCRATCH streams the least
// recently used one is handed over, behind an event wait on its last launch.
constexpr size_t PM_STREAM_SCRATCH = 4;
struct StreamSpill {
    hipStream_t s = nullptr;
    uint32_t* buf = nullptr;
    int64_t cap = 0;
    hipEvent_t done = nullptr;  // recorded after each launch on s
    uint64_t used = 0;
};

// Host-path options of an object (pm_hip_set_option; -1 = the environment's
// default, read once):
//   host_spin    wait for a read_block slot by polling the stream instead of
//                hipStreamSynchronize (PM_HOST_SPIN, default 0: no faster)
//   host_gid16   small read_block_gid calls bring u16 gids over the link and
//                widen them on the host when every gid < 65,536
//                (PM_HOST_GID16; default 1 for calls the resident server
//                takes, 0 for launched ones: there the link wait shrinks
//                3 us and the widening cost 5 us more than the copy, round 4)
//   host_events  small calls bracket their launch with timing events for
//                pm_hip_device_seconds (PM_HOST_SMALL_EVENTS, default 0:
//                the two events cost 7 us of a 43-us 100 KiB call,
//                profiles/r05/small_call/; without them device_seconds is -1
//                after a small call, and the CLI, which reports device time,
//                turns them on for its objects)
//   host_pool    small calls copy / map their results on the process's host
//                pool (1, default) or on the calling thread alone (0)
// (Measured and removed, round 5: small calls replayed from captured HIP
// graphs -- 100 KiB gids 43.3 -> 51.2 us per call, a replayed zero-copy
// launch + wait 24.0 -> 38.0 us; profiles/r05/small_call/.)
//   host_serve   small read_block calls of an rt object, or of an auto object
//                while its pick holds the RT kernel (the one-thread-per-
//                position walk's sizes, RtDev::small_max) go to its resident
//                server grid (Server below) instead of a launch each
//                (PM_HOST_SERVE, default 1)
struct HostOpts {
    int spin = -1, gid16 = -1, events = -1, pool = -1, serve = -1;
};

// The resident small-call server of an rt / auto object (pm_kernels.h PmServeReq,
// rt_serve_kernel): the request line and the grid's done flags in coherent
// pinned host memory, coherent staging and result buffers of its own, and
// its own stream.  A call posts a request and
// spins on the done flags; a grid that has exited (idle for
// PM_HOST_SERVE_IDLE_US, default 2,000 us, or stopped) is launched again --
// also in the middle of a wait, when the grid ended just as the request came
// (it then redoes the request: the writes are the same).  serve_stop() asks
// the grid to exit without waiting (before launches that want the whole
// device); pm_hip_free and the process's exit wait for it.
struct Server {
    PmServeReq* req = nullptr;  // then, 64 B on, `blocks` u32 done flags
    uint32_t* done = nullptr;
    uint64_t* fwd = nullptr;    // device memory: workgroup 0's copy of the request line
    uint8_t* h_stage = nullptr;
    uint32_t* h_res = nullptr;
    size_t cap = 0;  // positions
    hipStream_t s = nullptr;
    hipEvent_t ev = nullptr;  // recorded after the grid: complete once it exited
    int blocks = 0;
    uint64_t seq = 0, gen = 0;
    bool live = false;  // a grid was launched and not yet told to stop
    uint64_t launches = 0, calls = 0;
    int64_t idle_us = -1;  // option "serve_idle_us" (-1: PM_HOST_SERVE_IDLE_US, default 2,000)
    bool failed = false;   // its buffers could not be made: the object's calls launch
};
struct PmHip {
    int kind_req = KIND_RT;
    int kind = 0;
    int device = 0;
    int num_cu = 0;
    bool compiled = false;
    std::vector<std::string> pats;
    std::vector<pm_pattern_id_t> ids;
    uint32_t max_len = 0;
    PmGidMap gids;
    // device tables
    RtDev rt{};
    DfaDev dfa{};
    const uint32_t* d_parent = nullptr;  // PmParents, gid space (scoring)
    const uint32_t* d_depth = nullptr;
    std::vector<uint32_t> parent;
    std::string cache_dir;   // compiled-image cache (else $PM_IMAGE_CACHE)
    bool cache_hit = false;
    std::vector<void*> allocs;
    size_t table_bytes = 0;
    // start-up cost of the last compile() (pm_hip_compile_stats): wall
    // seconds of the whole call and of its host-to-device table copies
    double compile_s = 0.0, upload_s = 0.0;
    uint32_t* spill = nullptr;  // RT deep-walk scratch of captured scan_device launches (graphs)
    int64_t spill_cap = 0;
    std::vector<StreamSpill> sspill;  // ... and of direct ones, per stream (stream_spill)
    uint64_t sspill_tick = 0;
    // streaming: the carried history (the last stream bytes, at least
    // max_len of them) and a two-slot pipeline (scan_host)
    PmHistRing hist;
    PmHostStep host;  // read_char's per-byte step over host copies of the images (pm_hoststep.h)
    std::vector<pm_pattern_id_t> id_of_gid;  // [0] = PM_NULL_PATTERN_ID
    PipeSlot slot[2];
    double dev_seconds = 0.0;
    AutoPick pick;        // scan_device launches (read_block slots have their own)
    // the lines stream generator's copy of the patterns (pm_hip_gen_lines_*)
    std::vector<uint8_t> lines_pats;
    std::vector<uint32_t> lines_offs;
    uint8_t* d_lines_pats = nullptr;
    uint32_t* d_lines_offs = nullptr;
    int last_kernel = 0;  // KIND_RT / KIND_AC of the last launch
    int last_out_width = 0;  // bytes per position the last read_block's scans wrote (2 or 4)
    int last_form = 0;    // its DFA form (1 dense rows, 2 sparse; 0 for RT)
    // per-object options (pm_hip_set_option; the kernel-side ones live in
    // rt / dfa): the host path's, and the DFA form (0 = timed choice, 1 =
    // dense rows, 2 = sparse)
    HostOpts hopt;
    Server srv;
    int dfa_form = 0;
    uint64_t untimed_calls = 0;  // read_block launches since reset without timing events
    int last_sparse_kernel = 0;  // PmSparseKernel of the last sparse-form launch (0: none yet)
};

// Drop the pick's choice and measurements (a measurement still in flight
// belongs to the old stream: wait for it and drop it).
void forget_pick(AutoPick& a) {
    if (a.pending) (void)hipEventSynchronize(a.ev);
    if (a.timing) (void)hipEventSynchronize(a.t1[a.queue[a.nq - 1]]);
    a.pending = a.timing = false;
    a.nq = a.qi = a.trial = 0;
    a.hold = 0;
    a.prev = -1;
    a.streak = 0;
}

void free_pick(AutoPick& a) {
    if (a.d_spill) (void)hipFree(a.d_spill);
    if (a.h_spill) (void)hipHostFree(a.h_spill);
    if (a.ev) (void)hipEventDestroy(a.ev);
    for (int c = 0; c < NCAND; ++c)
        for (hipEvent_t e : {a.t0[c], a.t1[c]})
            if (e) (void)hipEventDestroy(e);
    a = AutoPick();
}

// The measurement resources of a kind that picks per launch (KIND_AUTO /
// KIND_AC): made when the object or slot is set up, never at a launch, so a
// launch under stream capture (which may not allocate) finds them.
void init_pick(AutoPick& a, int kind, bool has_sparse) {
    if (a.ev || (kind != KIND_AUTO && kind != KIND_AC)) return;
    if (kind == KIND_AC) a.chosen = has_sparse ? CAND_SPARSE : CAND_DENSE;  // no RT image
    PM_CHECK(hipMalloc(&a.d_spill, sizeof(unsigned long long)));
    PM_CHECK(hipHostMalloc(&a.h_spill, sizeof(unsigned long long), hipHostMallocDefault));
    PM_CHECK(hipEventCreateWithFlags(&a.ev, hipEventDisableTiming));
    for (int c = 0; c < NCAND; ++c) {
        PM_CHECK(hipEventCreate(&a.t0[c]));
        PM_CHECK(hipEventCreate(&a.t1[c]));
    }
}

void* dalloc_copy(PmHip* o, const void* src, size_t bytes) {
    void* p = nullptr;
    PM_CHECK(hipMalloc(&p, bytes ? bytes : 16));
    const auto t0 = std::chrono::steady_clock::now();
    if (bytes) PM_CHECK(hipMemcpy(p, src, bytes, hipMemcpyHostToDevice));
    o->upload_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    o->allocs.push_back(p);
    o->table_bytes += bytes;
    return p;
}

PmHip* create(int kind) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        std::fprintf(stderr, "pm_hip: no HIP device; this matcher has no CPU fallback\n");
        std::exit(EXIT_FAILURE);
    }
    PmHip* o = new PmHip();
    o->kind_req = kind;
    PM_CHECK(hipGetDevice(&o->device));
    hipDeviceProp_t prop;
    PM_CHECK(hipGetDeviceProperties(&prop, o->device));
    o->num_cu = prop.multiProcessorCount;
    return o;
}

void free_slot(PipeSlot& q) {
    if (q.d_stage) {
        (void)hipFree(q.d_stage);
        (void)hipFree(q.d_res);
        (void)hipHostFree(q.h_stage);
        (void)hipHostFree(q.h_res);
    }
    if (q.spill) (void)hipFree(q.spill);
    free_pick(q.pick);
    q.d_stage = nullptr;
    q.spill = nullptr;
    q.spill_cap = 0;
    q.cap = 0;
}

// The RT kernel's spill regions (pm_kernels.h): 8-B items, one per position
// of each wave's chunks up to a bound per wave (the kernel resolves a full
// region and goes on), so a launch of any size needs at most
// pm_rt_spill_items(INT64_MAX) items: 512 MiB on 256 CUs.  compile()
// allocates that for captured scan_device launches, which may not allocate;
// a stream's scratch (stream_spill) grows to its largest launch (a hipFree
// synchronizes the device, once per size step); read_block slots size theirs
// to their block.  Scratch, not part of the automaton's total_mem.
void ensure_spill(PmHip* o, uint32_t*& buf, int64_t& cap, int64_t n) {
    if (o->kind != KIND_RT && o->kind != KIND_AUTO) return;
    const int64_t need = pm_rt_spill_items(n, o->num_cu, o->rt.spill_cap_chunks);
    if (need <= cap) return;
    if (buf) PM_CHECK(hipFree(buf));
    buf = nullptr;
    PM_CHECK(hipMalloc(&buf, (size_t)need * 2 * sizeof(uint32_t)));  // 8-B items
    cap = need;
}

// The scratch of a direct (not captured) scan_device launch of n positions
// on stream s; nullptr for a kind without the RT kernel.
StreamSpill* stream_spill(PmHip* o, hipStream_t s, int64_t n) {
    if (o->kind != KIND_RT && o->kind != KIND_AUTO) return nullptr;
    StreamSpill* e = nullptr;
    for (StreamSpill& x : o->sspill)
        if (x.s == s) e = &x;
    if (!e && o->sspill.size() < PM_STREAM_SCRATCH) {
        o->sspill.emplace_back();
        e = &o->sspill.back();
        e->s = s;
        PM_CHECK(hipEventCreateWithFlags(&e->done, hipEventDisableTiming));
    }
    if (!e) {  // hand over the least recently used one, after its last launch
        e = &o->sspill[0];
        for (StreamSpill& x : o->sspill)
            if (x.used < e->used) e = &x;
        PM_CHECK(hipStreamWaitEvent(s, e->done, 0));
        e->s = s;
    }
    e->used = ++o->sspill_tick;
    ensure_spill(o, e->buf, e->cap, n);
    return e;
}

void ensure_slot(PmHip* o, PipeSlot& q, size_t positions) {
    if (!q.stream) {
        PM_CHECK(hipStreamCreateWithFlags(&q.stream, hipStreamNonBlocking));
        PM_CHECK(hipEventCreate(&q.ev0));
        PM_CHECK(hipEventCreate(&q.ev1));
    }
    init_pick(q.pick, o->kind, o->dfa.sbase != nullptr);
    if (positions <= q.cap) return;
    free_slot(q);
    const size_t cap = std::max(positions, (size_t)1 << 16);
    const size_t stage_bytes = cap + o->max_len + 64;
    PM_CHECK(hipMalloc(&q.d_stage, stage_bytes));
    PM_CHECK(hipMalloc(&q.d_res, cap * sizeof(uint32_t)));
    PM_CHECK(hipHostMalloc(&q.h_stage, stage_bytes, hipHostMallocDefault));
    PM_CHECK(hipHostMalloc(&q.h_res, cap * sizeof(uint32_t), hipHostMallocDefault));
    ensure_spill(o, q.spill, q.spill_cap, (int64_t)cap);
    init_pick(q.pick, o->kind, o->dfa.sbase != nullptr);
    q.cap = cap;
}

// Zero-copy small read_block calls (PM_HOST_ZC, a bit mask, default 3):
// 1 = the kernel writes its results straight into the pinned result buffer,
// 2 = it reads the pinned staging buffer instead of a device copy.  At the
// reference's 100 KiB chunks (measure.c:77), per call, rt / ac gids: 65.6 /
// 93.9 us with copies (0), 55.1 / 84.4 with 1, 48.2 / 76.5 with 3
// (scripts/host_profile.py, profiles/r04/host_path).
int host_zero_copy() {
    static const int z = [] {
        const char* e = std::getenv("PM_HOST_ZC");
        return e ? (int)std::strtol(e, nullptr, 10) & 3 : 3;
    }();
    return z;
}

int env_int(const char* k, int d) {
    const char* e = std::getenv(k);
    return e ? (int)std::strtol(e, nullptr, 10) : d;
}

bool opt_or_env(int v, const char* env, int d) {
    if (v >= 0) return v != 0;
    return env_int(env, d) != 0;
}

// Host threads for the copy/map work around the pipeline (PM_HOST_THREADS,
// default min(8, the job's core share)).
unsigned core_share() {
    static const unsigned c = [] {
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        const int omp = env_int("OMP_NUM_THREADS", 0);  // the job's share on a shared host
        return omp > 0 ? std::min(hw, (unsigned)omp) : hw;
    }();
    return c;
}
unsigned host_threads() {
    static const unsigned t = [] {
        const char* e = std::getenv("PM_HOST_THREADS");
        long v = e ? std::strtol(e, nullptr, 10) : 0;
        if (v <= 0) v = std::min(8u, core_share());
        return (unsigned)std::min(v, 64L);
    }();
    return t;
}

// A small persistent pool for the result copy / id map of small read_block
// calls (the reference's 100 KiB chunks, measure.c:77), whose ~10-27 us of
// single-threaded host work is a quarter to a half of the call: a thread
// per piece per call would cost more than the piece.  Workers spin on a
// ticket for up to PM_HOST_POOL_SPIN_US (default 200; 0 when the job's core
// share is below 8, so the spin never competes with the job's own threads)
// microseconds after their last piece -- so back-to-back calls find them
// awake -- then sleep on a condition variable.  A job is one generation of
// the ticket (gen << 40 | pieces << 20 | next piece); a worker runs a piece
// only after claiming it by CAS in that generation, so the job's function
// stays valid while it runs (the caller waits for every piece before
// returning).  PM_HOST_POOL = the workers (default 3, at most the core share
// minus one; 0 = no pool).  The pool is a static object: its destructor (at
// exit or when the library is unloaded) wakes the workers and joins them --
// in the process that started them only.  A child forked after the pool
// started holds std::thread objects whose threads do not exist in it (and
// maybe a mutex some worker held at the fork), so there the destructor
// touches neither the lock nor the threads: it detaches them.
class HostPool {
public:
    explicit HostPool(unsigned workers) : owner_(getpid()) {
        spin_us_ = std::max(0, env_int("PM_HOST_POOL_SPIN_US", core_share() >= 8 ? 200 : 0));
        for (unsigned i = 0; i < workers; ++i) th_.emplace_back([this] { loop(); });
    }
    ~HostPool() {
        if (getpid() != owner_) {
            for (std::thread& t : th_) t.detach();
            return;
        }
        {
            std::lock_guard<std::mutex> l(m_);
            stop_.store(true, std::memory_order_seq_cst);
            cv_.notify_all();
        }
        for (std::thread& t : th_) t.join();
    }
    unsigned workers() const { return (unsigned)th_.size(); }
    // f(k) for k in [0, pieces) on the workers and the caller; returns when all are done
    void run(unsigned pieces, const std::function<void(unsigned)>& f) {
        std::lock_guard<std::mutex> g(submit_);
        fn_.store(&f, std::memory_order_relaxed);
        pending_.store(pieces, std::memory_order_relaxed);
        const uint64_t gen = (ticket_.load(std::memory_order_relaxed) >> 40) + 1;
        ticket_.store(gen << 40 | (uint64_t)pieces << 20, std::memory_order_seq_cst);
        if (sleepers_.load(std::memory_order_seq_cst)) {
            std::lock_guard<std::mutex> l(m_);
            cv_.notify_all();
        }
        work(gen);
        while (pending_.load(std::memory_order_acquire)) {}
    }

private:
    bool claim(uint64_t gen, unsigned& k) {
        uint64_t v = ticket_.load(std::memory_order_acquire);
        for (;;) {
            if ((v >> 40) != gen || (v & 0xFFFFFu) >= ((v >> 20) & 0xFFFFFu)) return false;
            if (ticket_.compare_exchange_weak(v, v + 1, std::memory_order_acq_rel)) {
                k = (unsigned)(v & 0xFFFFFu);
                return true;
            }
        }
    }
    void work(uint64_t gen) {
        unsigned k;
        while (claim(gen, k)) {
            (*fn_.load(std::memory_order_relaxed))(k);
            pending_.fetch_sub(1, std::memory_order_release);
        }
    }
    void loop() {
        uint64_t seen = 0;
        while (!stop_.load(std::memory_order_acquire)) {
            const auto t0 = std::chrono::steady_clock::now();
            uint64_t g;
            unsigned spins = 0;
            while ((g = ticket_.load(std::memory_order_acquire) >> 40) == seen) {
                if (stop_.load(std::memory_order_acquire)) return;
                if ((++spins & 1023u) == 0 &&
                    std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us_)) {
                    std::unique_lock<std::mutex> l(m_);
                    sleepers_.fetch_add(1, std::memory_order_seq_cst);
                    cv_.wait(l, [&] {
                        return stop_.load(std::memory_order_seq_cst) ||
                               (ticket_.load(std::memory_order_seq_cst) >> 40) != seen;
                    });
                    sleepers_.fetch_sub(1, std::memory_order_relaxed);
                }
            }
            seen = g;
            work(g);
        }
    }
    std::atomic<uint64_t> ticket_{0};
    std::atomic<unsigned> pending_{0}, sleepers_{0};
    std::atomic<bool> stop_{false};
    std::atomic<const std::function<void(unsigned)>*> fn_{nullptr};
    std::mutex submit_, m_;
    std::condition_variable cv_;
    long spin_us_ = 200;
    const pid_t owner_;  // the process that started the workers
    std::vector<std::thread> th_;
};

HostPool* host_pool() {
    static HostPool pool((unsigned)std::max(
        0, std::min({env_int("PM_HOST_POOL", 3), 15, (int)core_share() - 1})));
    return pool.workers() ? &pool : nullptr;
}

// f(lo, hi) over [0, n) of a small block: pieces on the pool, or the caller alone.
template <class F>
void small_par(bool use_pool, size_t n, const F& f) {
    HostPool* p = use_pool && n >= ((size_t)16 << 10) ? host_pool() : nullptr;
    const unsigned pieces = p ? std::min<unsigned>(p->workers() + 1, (unsigned)(n >> 14)) : 1u;
    if (pieces <= 1) {
        f((size_t)0, n);
        return;
    }
    const size_t step = (n + pieces - 1) / pieces;
    p->run(pieces, [&](unsigned k) {
        const size_t lo = std::min(n, (size_t)k * step), hi = std::min(n, lo + step);
        if (lo < hi) f(lo, hi);
    });
}

// f(lo, hi) over [0, n) split across host threads, pieces of at least grain.
template <class F>
void par_range(size_t n, size_t grain, const F& f) {
    const size_t parts = std::min<size_t>(host_threads(), std::max<size_t>(1, n / grain));
    if (parts <= 1) {
        f((size_t)0, n);
        return;
    }
    const size_t step = (n + parts - 1) / parts;
    std::vector<std::thread> th;
    th.reserve(parts - 1);
    for (size_t k = 1; k < parts; ++k) {
        const size_t lo = std::min(n, k * step), hi = std::min(n, lo + step);
        th.emplace_back([&f, lo, hi] { f(lo, hi); });
    }
    f((size_t)0, std::min(n, step));
    for (auto& t : th) t.join();
}

// Servers with a grid that may still run: at the process's exit each is
// told to stop and waited for (the handler is registered after the HIP
// runtime's own, so it runs before them), so no grid outlives the process.
std::mutex g_srv_m;
std::vector<Server*> g_srv;
void serve_exit_all() {
    std::lock_guard<std::mutex> l(g_srv_m);
    for (Server* v : g_srv) {
        __atomic_store_n(&v->req->stop, v->gen, __ATOMIC_SEQ_CST);
        (void)hipStreamSynchronize(v->s);
    }
    g_srv.clear();
}

bool serve_on(const PmHip* o) {
    return (o->kind == KIND_RT || o->kind == KIND_AUTO) && opt_or_env(o->hopt.serve, "PM_HOST_SERVE", 1);
}

// Ask the grid to exit (no wait).
void serve_stop(PmHip* o) {
    Server& v = o->srv;
    if (!v.live) return;
    __atomic_store_n(&v.req->stop, v.gen, __ATOMIC_SEQ_CST);
    v.live = false;
}

void serve_free(PmHip* o) {
    Server& v = o->srv;
    if (!v.req) return;
    const int64_t idle_us = v.idle_us;
    serve_stop(o);
    (void)hipStreamSynchronize(v.s);
    {
        std::lock_guard<std::mutex> l(g_srv_m);
        g_srv.erase(std::remove(g_srv.begin(), g_srv.end(), &v), g_srv.end());
    }
    (void)hipHostFree(v.req);
    (void)hipHostFree(v.h_stage);
    (void)hipHostFree(v.h_res);
    (void)hipFree(v.fwd);
    (void)hipEventDestroy(v.ev);
    (void)hipStreamDestroy(v.s);
    v = Server();
    v.idle_us = idle_us;
}

void serve_launch(PmHip* o, uint64_t seen) {
    Server& v = o->srv;
    ++v.gen;
    static const int64_t env_idle = std::max(10, env_int("PM_HOST_SERVE_IDLE_US", 2000));
    const int64_t idle_us = v.idle_us >= 0 ? v.idle_us : env_idle;
    RtDev t = o->rt;
    PM_CHECK(pm_launch_rt_serve(v.req, v.fwd, v.done, v.blocks, seen, v.gen, idle_us * 100, t, v.s));
    PM_CHECK(hipEventRecord(v.ev, v.s));
    v.live = true;
    ++v.launches;
}

// The server's buffers (first call): staging for [context | block | 16 zero
// bytes] of a block of up to PIPE_SMALL_POSITIONS positions, u32 results.
bool serve_ready(PmHip* o) {
    Server& v = o->srv;
    if (v.req) return true;
    if (v.failed) return false;
    v.blocks = std::max(1, o->num_cu / 4);
    if (const char* e = std::getenv("PM_SERVE_BLOCKS")) v.blocks = std::max(1, std::min(o->num_cu, std::atoi(e)));
    v.cap = PIPE_SMALL_POSITIONS;
    const unsigned coh = hipHostMallocCoherent | hipHostMallocMapped;
    const size_t req_bytes = 64 + sizeof(uint32_t) * (size_t)v.blocks + 64 + 256;  // (+ the trace build's stamps)
    // (staging and results in ordinary pinned memory: the grid reads and
    // writes them at the coherence point anyway, and the host reads coherent
    // memory at a third of the rate -- 400 KB of results 24.8 against 9.1 us)
    bool ok = hipHostMalloc(&v.req, req_bytes, coh) == hipSuccess;
    ok = ok && hipHostMalloc(&v.h_stage, v.cap + o->max_len + 64, hipHostMallocDefault) == hipSuccess;
    ok = ok && hipHostMalloc(&v.h_res, v.cap * sizeof(uint32_t), hipHostMallocDefault) == hipSuccess;
    ok = ok && hipMalloc(&v.fwd, 64) == hipSuccess && hipMemset(v.fwd, 0, 64) == hipSuccess;
    ok = ok && hipStreamCreateWithFlags(&v.s, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&v.ev, hipEventDisableTiming) == hipSuccess;
    if (!ok) {  // no server for this object: its calls launch, as without one
        (void)hipGetLastError();
        if (v.req) (void)hipHostFree(v.req);
        if (v.h_stage) (void)hipHostFree(v.h_stage);
        if (v.h_res) (void)hipHostFree(v.h_res);
        if (v.fwd) (void)hipFree(v.fwd);
        if (v.s) (void)hipStreamDestroy(v.s);
        const int64_t idle_us = v.idle_us;
        v = Server();
        v.idle_us = idle_us;
        v.failed = true;
        return false;
    }
    std::memset(v.req, 0, req_bytes);
    v.done = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(v.req) + 64);
    static const bool registered = [] { return std::atexit(serve_exit_all) == 0; }();
    (void)registered;
    std::lock_guard<std::mutex> l(g_srv_m);
    g_srv.push_back(&v);
    return true;
}

// Post the request: positions [pos0, pos0 + n) of the server's staging
// (context back to stream_start), results of outw bytes into its h_res.
void serve_post(PmHip* o, int64_t stream_start, int64_t pos0, int64_t n, int outw) {
    Server& v = o->srv;
    PmServeReq* r = v.req;
    const uint64_t s = ++v.seq;
    ++v.calls;
    // seq, the fields, seq2 (x86 stores are seen in order; the device reads
    // the line whole and takes it when seq2 == seq)
    __atomic_store_n(&r->seq, s, __ATOMIC_SEQ_CST);
    r->text = v.h_stage;
    r->out = v.h_res;
    r->stream_start = stream_start;
    r->pos0 = pos0;
    r->n_outw = (uint64_t)n | (uint64_t)outw << 56;
    __atomic_store_n(&r->seq2, s, __ATOMIC_SEQ_CST);  // after the staging and the fields
    // a grid that exited (idle) or was stopped: a new one, which takes s
    if (!v.live || hipEventQuery(v.ev) == hipSuccess) serve_launch(o, s - 1);
}

// Wait for every workgroup's done flag of the last request.
void serve_wait(PmHip* o) {
    Server& v = o->srv;
    const uint32_t want = (uint32_t)v.seq;
    int w = 0;
    const auto t0 = std::chrono::steady_clock::now();
#ifdef PM_SERVE_TRACE
    // the first stamp of workgroup 0 (written when it sees the request): its arrival
    static uint64_t last0 = 0;
    const volatile uint64_t* tr0 = reinterpret_cast<const uint64_t*>(v.done + v.blocks + 16);
    while (*tr0 == last0 && std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(100)) {}
    last0 = *tr0;
    const double ack_us = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e6;
#endif
    for (uint64_t spin = 1;; ++spin) {
        while (w < v.blocks && __atomic_load_n(&v.done[w], __ATOMIC_ACQUIRE) == want) ++w;
        if (w == v.blocks) {
#ifdef PM_SERVE_TRACE
            const uint64_t* tr = reinterpret_cast<const uint64_t*>(v.done + v.blocks + 16);
            std::fprintf(stderr, "serve trace (10 ns): wg0 detect->window %lld walk %lld waitcnt+bar %lld flag %lld | "
                         "wg1 detect-wg0 %lld ->window %lld walk %lld bar %lld flag %lld | host: wg0's detect stamp "
                         "seen %.2f us, last flag %.2f us\n",
                         (long long)(tr[1] - tr[0]), (long long)(tr[2] - tr[1]), (long long)(tr[3] - tr[2]),
                         (long long)(tr[4] - tr[3]), (long long)(tr[8] - tr[0]), (long long)(tr[9] - tr[8]),
                         (long long)(tr[10] - tr[9]), (long long)(tr[11] - tr[10]), (long long)(tr[12] - tr[11]), ack_us,
                         std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e6);
#endif
            return;
        }
        if ((spin & 1023) == 0) {
            const hipError_t e = hipEventQuery(v.ev);
            if (e == hipSuccess) {  // the grid ended before it saw the request
                serve_launch(o, v.seq - 1);
            } else if (e != hipErrorNotReady) {
                fatal("resident server grid", e);
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
                std::fprintf(stderr, "pm_hip: resident server: no answer in 60 s (%d of %d workgroups done)\n", w,
                             v.blocks);
                std::exit(EXIT_FAILURE);
            }
        }
    }
}

hipError_t launch_cand(PmHip* o, AutoPick& ap, int c, const uint8_t* text, int64_t stream_start, int64_t pos0,
                       int64_t n, void* out, int outw, unsigned long long* count, hipStream_t s, const RtDev& t) {
    ap.last = c == CAND_RT ? KIND_RT : KIND_AC;
    ap.last_form = c == CAND_RT ? 0 : c == CAND_DENSE ? 1 : 2;
    if (c == CAND_RT) return pm_launch_rt(text, stream_start, pos0, n, out, outw, count, t, o->num_cu, s);
    DfaDev d = o->dfa;
    d.form = c == CAND_DENSE ? 1 : 2;
    if (c == CAND_SPARSE16) d.flhold = 1;
    if (c == CAND_SPARSE64) d.flhold = 4;
    if (c == CAND_FL2) {
        d.flhold = 1;
        d.flchains = 2;
    }
    o->last_sparse_kernel = pm_dfa_sparse_choice(d, out ? outw : 0);
    return pm_launch_dfa(text, stream_start, pos0, n, out, outw, count, d, o->num_cu, s);
}

// The DFA forms to try, in order (dense rows, then rows + records; only the
// object's forced form when it has one).
void start_trials(const PmHip* o, AutoPick& ap) {
    // (the last one queued also runs while the trials' times are in flight:
    // a caller far ahead of the device launches it until they land, so the
    // usual winner on deep input goes last)
    ap.nq = 0;
    const bool fl = o->dfa.flbase && o->dfa_form != 1 &&
                    (o->dfa.sparse_kernel == PM_SK_PRODUCT || o->dfa.sparse_kernel == PM_SK_FL);
    if (o->dfa_form != 2 || !o->dfa.sbase) ap.queue[ap.nq++] = CAND_DENSE;
    if (fl) ap.queue[ap.nq++] = CAND_SPARSE16;
    if (fl) ap.queue[ap.nq++] = CAND_FL2;
    // (with the FL form the 32-B-block policy is not a candidate: it was the
    // best on no stream measured -- snort / merged lines, the shipped stream,
    // ASCII; profiles/r05/ab/fl_hold_1_2_4.jsonl -- and each candidate costs
    // two launches per measurement)
    if (o->dfa.sbase && o->dfa_form != 1 && !fl) ap.queue[ap.nq++] = CAND_SPARSE;
    if (fl) ap.queue[ap.nq++] = CAND_SPARSE64;
    ap.qi = 0;
    ap.trial = 0;
}

// The hold after a measurement chose ap.chosen (AUTO_STREAK_MAX; for small
// launches AUTO_STREAK_MAX_SMALL).
int confirm_hold(AutoPick& ap) {
    const int cap = ap.n_of[ap.chosen] < AUTO_SMALL_LAUNCH ? AUTO_STREAK_MAX_SMALL : AUTO_STREAK_MAX;
    ap.streak = ap.chosen == ap.prev ? std::min(ap.streak + 1, cap) : 0;
    ap.prev = ap.chosen;
    return AUTO_HOLD << ap.streak;
}

// Fold in whatever measurement has landed (KIND_AUTO / KIND_AC, see
// AUTO_SPILL_FRAC).
void resolve_pick(const PmHip* o, AutoPick& ap) {
    if (!ap.ev) return;
    auto elapsed_ns = [&](int c) {
        float ms = 0.f;
        return hipEventElapsedTime(&ms, ap.t0[c], ap.t1[c]) == hipSuccess && ap.n_of[c] > 0
                   ? ms * 1e6 / (double)ap.n_of[c]
                   : 0.0;
    };
    if (ap.pending && hipEventQuery(ap.ev) == hipSuccess) {
        ap.pending = false;
        ap.ns[CAND_RT] = elapsed_ns(CAND_RT);
        if ((double)*ap.h_spill > AUTO_SPILL_FRAC * (double)ap.n_of[CAND_RT]) {
            start_trials(o, ap);
        } else {  // shallow: RT holds
            ap.chosen = CAND_RT;
            ap.hold = confirm_hold(ap);
        }
    }
    auto trials_done = [&]() {  // every trial's end event (they may sit on different streams)
        for (int k = 0; k < ap.nq; ++k)
            if (hipEventQuery(ap.t1[ap.queue[k]]) != hipSuccess) return false;
        return true;
    };
    if (ap.timing && trials_done()) {
        ap.timing = false;
        int best = o->kind == KIND_AUTO ? CAND_RT : ap.queue[0];
        double best_ns = o->kind == KIND_AUTO ? ap.ns[CAND_RT] : 0.0;
        for (int k = 0; k < ap.nq; ++k) {
            const int c = ap.queue[k];
            ap.ns[c] = elapsed_ns(c);
            if (ap.ns[c] > 0.0 && (best_ns <= 0.0 || ap.ns[c] < best_ns)) {
                best = c;
                best_ns = ap.ns[c];
            }
        }
        ap.chosen = best;
        ap.hold = confirm_hold(ap);
        ap.nq = ap.qi = 0;
    }
}

hipError_t launch(PmHip* o, const uint8_t* text, int64_t stream_start, int64_t pos0, int64_t n, void* out, int outw,
                  unsigned long long* count, hipStream_t s, uint32_t* spill, int64_t spill_cap, AutoPick& ap) {
    RtDev t = o->rt;
    t.spill = spill;
    t.spill_cap = spill_cap;
    if (o->kind == KIND_RT) return pm_launch_rt(text, stream_start, pos0, n, out, outw, count, t, o->num_cu, s);
    // one DFA form only (an uncoded automaton), or the object's forced form
    if (o->kind == KIND_AC && (!o->dfa.sbase || o->dfa_form)) {
        ap.last = KIND_AC;
        DfaDev d = o->dfa;
        d.form = o->dfa.sbase ? (o->dfa_form ? o->dfa_form : 2) : 1;
        ap.last_form = d.form == 2 ? 2 : 1;
        o->last_sparse_kernel = pm_dfa_sparse_choice(d, out ? outw : 0);
        return pm_launch_dfa(text, stream_start, pos0, n, out, outw, count, d, o->num_cu, s);
    }
    // KIND_AUTO / KIND_AC (see AUTO_SPILL_FRAC): RT launches are measured
    // (spill count and time); a deep one (or, for KIND_AC, the end of a
    // hold) starts timed trials of the DFA forms; the fastest per position
    // then runs AUTO_HOLD launches.
    // Measurements are polled, never waited for: scan_device stays an
    // asynchronous launch on the caller's stream.  Until a measurement has
    // landed the current choice keeps running (a burst of launches queued
    // ahead of the device adapts once it catches up; bench.py synchronizes
    // its untimed pick launches, pm_hip_hold_choice).  The read_block
    // pipeline has synchronized the slot already, so there it lands at the
    // next call.  Under stream capture nothing is measured (no events, no
    // copies, nothing allocated -- the pick's resources are made with the
    // object, init_pick): the current choice runs.
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone)
        return launch_cand(o, ap, ap.chosen, text, stream_start, pos0, n, out, outw, count, s, t);
    init_pick(ap, o->kind, o->dfa.sbase != nullptr);
    resolve_pick(o, ap);
    if (ap.hold > 0) {  // hold the chosen kernel
        --ap.hold;
        return launch_cand(o, ap, ap.chosen, text, stream_start, pos0, n, out, outw, count, s, t);
    }
    if (o->kind == KIND_AC && !ap.timing && ap.qi >= ap.nq) start_trials(o, ap);
    if (!ap.timing && ap.qi < ap.nq) {  // DFA trials: AUTO_TRIAL launches per form, the last one timed
        const int c = ap.queue[ap.qi];
        if (ap.trial == 0) ap.trial = AUTO_TRIAL;
        if (--ap.trial > 0) return launch_cand(o, ap, c, text, stream_start, pos0, n, out, outw, count, s, t);
        hipError_t e = hipEventRecord(ap.t0[c], s);
        if (e == hipSuccess) e = launch_cand(o, ap, c, text, stream_start, pos0, n, out, outw, count, s, t);
        if (e == hipSuccess) e = hipEventRecord(ap.t1[c], s);
        ap.n_of[c] = n;
        if (++ap.qi == ap.nq) ap.timing = e == hipSuccess;
        return e;
    }
    // a measurement still in flight: keep running the current choice
    if (ap.timing || ap.pending)
        return launch_cand(o, ap, ap.timing ? ap.queue[ap.nq - 1] : ap.chosen, text, stream_start, pos0, n, out, outw,
                           count, s, t);
    ap.last = KIND_RT;
    ap.last_form = 0;
    t.spill_total = ap.d_spill;
    hipError_t e = hipMemsetAsync(ap.d_spill, 0, sizeof(unsigned long long), s);
    if (e == hipSuccess) e = hipEventRecord(ap.t0[CAND_RT], s);
    if (e == hipSuccess) e = pm_launch_rt(text, stream_start, pos0, n, out, outw, count, t, o->num_cu, s);
    if (e == hipSuccess) e = hipEventRecord(ap.t1[CAND_RT], s);
    if (e == hipSuccess) e = hipMemcpyAsync(ap.h_spill, ap.d_spill, sizeof(unsigned long long), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipEventRecord(ap.ev, s);
    ap.pending = e == hipSuccess;
    ap.n_of[CAND_RT] = n;
    return e;
}

// Scan n new bytes after the carried history.  Results go to out_gid (gids)
// or out_ids (the caller's pattern ids, PM_NULL_PATTERN_ID for none) -- one
// of the two is non-null.  Blocks alternate between two slots (streams):
// block k's bytes are uploaded straight from the caller's buffer behind its
// context -- the last max_len-1 stream bytes before it (carried history,
// then the caller's own buffer), staged in pinned memory -- scanned, and the
// gids downloaded straight into out_gid, or into pinned memory from which
// the host maps them to pattern ids (threads) while block k+1 is in flight.
// For pattern ids, dictionaries of < 65,536 patterns (every reference
// dictionary) come back as u16 gids (half the PCIe bytes) for the host
// threads to map: +12% (RT) / +28% (AC).  Gids for the caller stay u32 and
// direct: widening u16 on the host measured 2-5% slower.  Rates: MEASUREMENTS.md §5.
// Host-path breakdown (pm_hip_host_profile): seconds spent staging
// the input, enqueueing the copies and the launch, waiting for the slot,
// and copying / mapping the results; calls.
double g_hprof[5] = {0, 0, 0, 0, 0};
bool g_hprof_on = false;
inline double hp_now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void scan_host(PmHip* o, const uint8_t* buf, size_t n, uint32_t* out_gid, pm_pattern_id_t* out_ids) {
    if (!o->compiled) {
        std::fprintf(stderr, "pm_hip: read before compile\n");
        std::exit(EXIT_FAILURE);
    }
    PM_CHECK(hipSetDevice(o->device));
    const size_t keep = o->max_len ? o->max_len - 1 : 0;
    const size_t pipe = out_gid ? PIPE_GID_POSITIONS : PIPE_ID_POSITIONS;
    const bool fits16 = o->gids.index_of_gid.size() <= 65536;
    const bool narrow = !out_gid && fits16;  // u16 gids over PCIe
    o->last_out_width = narrow ? 2 : 4;
    double t_mark = g_hprof_on ? hp_now() : 0.0;
    auto lap = [&](int k) {
        if (!g_hprof_on) return;
        const double t = hp_now();
        g_hprof[k] += t - t_mark;
        t_mark = t;
    };
    if (g_hprof_on) g_hprof[4] += 1;
    const bool pool = o->hopt.pool != 0;  // (the pool's size: PM_HOST_POOL)
    const bool gid16 = opt_or_env(o->hopt.gid16, "PM_HOST_GID16", 0);
    // (served calls: u16 gids over the link by default -- 100 KiB gids 29.0
    // -> 25.4 us, the host pool's widening under the halved link time;
    // profiles/r06/serve/)
    const bool gid16_served = opt_or_env(o->hopt.gid16, "PM_HOST_GID16", 1);
    const bool events = opt_or_env(o->hopt.events, "PM_HOST_SMALL_EVENTS", 0);
    auto finish = [&](PipeSlot& q) {
        lap(1);
        if (q.served) {
            serve_wait(o);
        } else if (opt_or_env(o->hopt.spin, "PM_HOST_SPIN", 0)) {
            hipError_t e;
            while ((e = hipStreamQuery(q.stream)) == hipErrorNotReady) {}
            PM_CHECK(e);
        } else {
            PM_CHECK(hipStreamSynchronize(q.stream));
        }
        lap(2);
        if (q.timed) {
            float ms = 0.f;
            PM_CHECK(hipEventElapsedTime(&ms, q.ev0, q.ev1));
            o->dev_seconds += ms * 1e-3;
        }
        const pm_pattern_id_t* map = o->id_of_gid.data();
        const uint32_t* const hres = q.served ? o->srv.h_res : q.h_res;
        if (out_gid && q.staged && q.w == 2) {  // widen
            const uint16_t* g = reinterpret_cast<const uint16_t*>(hres);
            uint32_t* dst = out_gid + q.off;
            small_par(pool, q.m, [&](size_t lo, size_t hi) {
                for (size_t j = lo; j < hi; ++j) dst[j] = g[j];
            });
        } else if (!out_gid) {
            pm_pattern_id_t* dst = out_ids + q.off;
            auto map_ids = [&](size_t lo, size_t hi) {
                if (narrow && PM_NT_IDS) {
                    // non-temporal 8-B stores: no read for ownership of the
                    // caller's lines (800 KB for a 100 KiB call)
                    const uint16_t* g = reinterpret_cast<const uint16_t*>(hres);
                    long long* d = reinterpret_cast<long long*>(dst);
                    for (size_t j = lo; j < hi; ++j) _mm_stream_si64(d + j, (long long)(uintptr_t)map[g[j]]);
                    _mm_sfence();
                } else if (narrow) {
                    const uint16_t* g = reinterpret_cast<const uint16_t*>(hres);
                    for (size_t j = lo; j < hi; ++j) dst[j] = map[g[j]];
                } else {
                    const uint32_t* g = hres;
                    for (size_t j = lo; j < hi; ++j) dst[j] = map[g[j]];
                }
            };
            if (q.staged) small_par(pool, q.m, map_ids);
            else par_range(q.m, (size_t)1 << 18, map_ids);
        } else if (q.staged) {
            small_par(pool, q.m, [&](size_t lo, size_t hi) {
                std::memcpy(out_gid + q.off + lo, hres + lo, (hi - lo) * sizeof(uint32_t));
            });
        }
        q.busy = false;
        lap(3);
    };
    size_t done = 0;
    for (int k = 0; done < n; ++k) {
        PipeSlot& q = o->slot[k & 1];
        if (q.busy) finish(q);
        const size_t m = std::min(pipe, n - done);
        ensure_slot(o, q, m);
        q.staged = m <= PIPE_SMALL_POSITIONS;
        // small blocks of an rt / auto object: the resident server (its own
        // staging and results), unless the call is to be timed
        q.served = q.staged && !events && host_zero_copy() == 3 && serve_on(o) &&
                   (int64_t)m <= (o->rt.small_max >= 0 ? o->rt.small_max : RT_SMALL_MAX);
        if (q.served) q.served = serve_ready(o);
        if (q.served && o->kind == KIND_AUTO) {
            // an auto object's calls are served while its pick holds the RT
            // kernel; its measurements (an RT launch, the DFA trials) launch
            init_pick(q.pick, o->kind, o->dfa.sbase != nullptr);
            resolve_pick(o, q.pick);
            q.served = q.pick.hold > 0 && q.pick.chosen == CAND_RT && !q.pick.timing && !q.pick.pending;
            if (q.served) {
                --q.pick.hold;
                q.pick.last = KIND_RT;
                q.pick.last_form = 0;
            }
        }
        // a launched block wants the device to itself: the grid exits (an
        // auto object holding a DFA form on deep input: 126 against 95 us a
        // 100 KiB call with the grid left resident, profiles/r06/serve/)
        if (!q.served) serve_stop(o);
        uint8_t* const hstage = q.served ? o->srv.h_stage : q.h_stage;
        // context: the last `keep` bytes of (history | buf[0, done))
        const size_t h = std::min(keep, o->hist.avail() + done);
        const size_t ctx = (h + 15) & ~(size_t)15;  // new bytes start 16-aligned
        uint8_t* st = hstage + ctx - h;
        if (done >= h) {
            std::memcpy(st, buf + done - h, h);
        } else {
            const size_t from_hist = h - done;
            o->hist.copy_last(st, from_hist);
            std::memcpy(st + from_hist, buf, done);
        }
        // small blocks, zero-copy (host_zero_copy()): the kernel reads the
        // pinned staging (2) / writes the pinned results (1) over the link
        const bool zc_in = q.staged && (host_zero_copy() & 2), zc_out = q.staged && (host_zero_copy() & 1);
        if (q.staged) {  // [context | bytes | 16 zero bytes] in one DMA from pinned memory
            std::memcpy(hstage + ctx, buf + done, m);
            std::memset(hstage + ctx + m, 0, 16);
            lap(0);
            if (!zc_in) PM_CHECK(hipMemcpyAsync(q.d_stage, q.h_stage, ctx + m + 16, hipMemcpyHostToDevice, q.stream));
        } else {
            std::memset(q.h_stage + ctx, 0, 16);
            if (ctx) PM_CHECK(hipMemcpyAsync(q.d_stage, q.h_stage, ctx, hipMemcpyHostToDevice, q.stream));
            PM_CHECK(hipMemcpyAsync(q.d_stage + ctx, buf + done, m, hipMemcpyHostToDevice, q.stream));
            PM_CHECK(hipMemcpyAsync(q.d_stage + ctx + m, q.h_stage + ctx, 16, hipMemcpyHostToDevice, q.stream));
        }
        q.w = narrow || (out_gid && q.staged && fits16 && (q.served ? gid16_served : gid16)) ? 2 : 4;
        q.timed = !q.staged || events;
        if (!q.timed) o->untimed_calls++;
        if (q.served) {
            serve_post(o, (int64_t)(ctx - h), (int64_t)ctx, (int64_t)m, q.w);
            o->last_kernel = KIND_RT;
            o->last_form = 0;
            o->last_out_width = q.w;
            q.busy = true;
            q.off = done;
            q.m = m;
            done += m;
            continue;
        }
        if (q.timed) PM_CHECK(hipEventRecord(q.ev0, q.stream));
        const uint8_t* text = zc_in ? q.h_stage : q.d_stage;
        void* res = zc_out ? q.h_res : q.d_res;
        PM_CHECK(launch(o, text, (int64_t)(ctx - h), (int64_t)ctx, (int64_t)m, res, q.w, nullptr, q.stream, q.spill,
                        q.spill_cap, q.pick));
        o->last_kernel = q.pick.last ? q.pick.last : o->kind;
        o->last_form = q.pick.last_form;
        o->last_out_width = q.w;
        if (q.timed) PM_CHECK(hipEventRecord(q.ev1, q.stream));
        if (zc_out)
            ;  // the results are in h_res once the stream is done
        else if (q.w == 2)
            PM_CHECK(hipMemcpyAsync(q.h_res, q.d_res, m * sizeof(uint16_t), hipMemcpyDeviceToHost, q.stream));
        else
            PM_CHECK(hipMemcpyAsync(out_gid && !q.staged ? out_gid + done : q.h_res, q.d_res, m * sizeof(uint32_t),
                                    hipMemcpyDeviceToHost, q.stream));
        q.busy = true;
        q.off = done;
        q.m = m;
        done += m;
    }
    // oldest block first
    for (int k = 0; k < 2; ++k) {
        PipeSlot& a = o->slot[0], &b = o->slot[1];
        PipeSlot& q = (a.busy && (!b.busy || a.off < b.off)) ? a : b;
        if (q.busy) finish(q);
    }
    // carry the stream's last bytes; the host DFA step re-derives its state
    o->hist.append(buf, n);
    o->host.state_valid = false;
}

PmHip* as(void* obj) { return static_cast<PmHip*>(obj); }

}  // namespace

extern "C" {

int pm_hip_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int pm_hip_set_device(int dev) { return hipSetDevice(dev) == hipSuccess ? 0 : -1; }

const char* pm_hip_last_error(void) { return g_err; }

void* pm_hip_rt_create(void) { return create(KIND_RT); }
void* pm_hip_ac_create(void) { return create(KIND_AC); }
void* pm_hip_auto_create(void) { return create(KIND_AUTO); }

void pm_hip_add_pattern(void* obj, char* pat, size_t len, pm_pattern_id_t id) {
    PmHip* o = as(obj);
    if (o->compiled) {
        std::fprintf(stderr, "pm_hip: add_pattern after compile\n");
        std::exit(EXIT_FAILURE);
    }
    if (len == 0) return;
    o->pats.emplace_back(pat, len);  // borrowed bytes (PatternsTree.c:393-400): copy
    o->ids.push_back(id);
    o->max_len = std::max(o->max_len, (uint32_t)len);
}

void pm_hip_compile(void* obj) {
    PmHip* o = as(obj);
    const auto tc0 = std::chrono::steady_clock::now();
    o->upload_s = 0.0;
    PM_CHECK(hipSetDevice(o->device));
    serve_free(o);  // a server grid of an earlier compile reads the old tables
    o->gids = pm_assign_gids(o->pats);
    o->kind = o->kind_req;
    // flattened tables, through the on-disk image cache when configured
    const char* env = std::getenv("PM_IMAGE_CACHE");
    const std::string dir = !o->cache_dir.empty() ? o->cache_dir : (env ? env : "");
    bool hit = false;
    const int first = o->kind == KIND_AC ? KIND_AC : KIND_RT;  // AUTO: the RT image, then the DFA's
    PmImages im = pm_build_images_cached(o->pats, o->gids, first, dir, &hit);
    if (first == KIND_RT && !im.rt.fits) {
        std::fprintf(stderr, "pm_hip: dictionary exceeds the reverse-trie u16 encoding; using the DFA kernel\n");
        o->kind = KIND_AC;
        im = pm_build_images_cached(o->pats, o->gids, KIND_AC, dir, &hit);
    }
    o->cache_hit = hit;
    if (o->kind == KIND_RT || o->kind == KIND_AUTO) {
        o->rt.t12 = (const uint16_t*)dalloc_copy(o, im.rt.t12.data(), im.rt.t12.size() * 2);
        o->rt.filt = (const uint32_t*)dalloc_copy(o, im.rt.filt.data(), im.rt.filt.size() * 4);
        o->rt.t3h = (const uint4*)dalloc_copy(o, im.rt.t3h.data(), im.rt.t3h.size() * 4);
        o->rt.t3h_bits = im.rt.t3h_bits;
        o->rt.back = o->max_len ? o->max_len - 1 : 0;
        o->rt.rec = (const uint4*)dalloc_copy(o, im.rt.rec.data(), im.rt.rec.size() * 4);
        o->rt.wide = (const uint4*)dalloc_copy(o, im.rt.wide.data(), im.rt.wide.size() * 4);
        const std::vector<uint8_t> zero(RT_SCRATCH_BYTES, 0);
        o->rt.scratch = (uint32_t*)dalloc_copy(o, zero.data(), zero.size());
    }
    if (o->kind == KIND_AUTO) {
        bool hit2 = false;
        PmImages d = pm_build_images_cached(o->pats, o->gids, KIND_AC, dir, &hit2);
        o->cache_hit = hit && hit2;
        im.dfa = std::move(d.dfa);
    }
    if (o->kind == KIND_AC || o->kind == KIND_AUTO) {
        o->dfa.next = (const uint32_t*)dalloc_copy(o, im.dfa.next.data(), im.dfa.next.size() * 4);
        o->dfa.out = (const uint32_t*)dalloc_copy(o, im.dfa.out.data(), im.dfa.out.size() * 4);
        o->dfa.warm = o->max_len ? (int64_t)o->max_len - 1 : 0;
        if (o->dfa.warm > 3) {  // the synchronizing 3-grams (DfaDev::gram3)
            std::vector<uint32_t> g3((1u << 24) / 32, 0u);
            for (const std::string& pt : o->pats)
                for (size_t i = 0; i + 3 <= pt.size(); ++i) {
                    const uint32_t x = (uint8_t)pt[i] | (uint32_t)(uint8_t)pt[i + 1] << 8 |
                                       (uint32_t)(uint8_t)pt[i + 2] << 16;
                    g3[x >> 5] |= 1u << (x & 31);
                }
            o->dfa.gram3 = (const uint32_t*)dalloc_copy(o, g3.data(), g3.size() * 4);
        }
        o->dfa.coded = pm_dfa_coded(im.dfa.states) ? 1 : 0;
        if (!im.dfa.sblock.empty()) {
            // (+64 zero bytes: the LDS kernel reads records in aligned
            // blocks of four, the last one past the table's end)
            im.dfa.sblock.resize(im.dfa.sblock.size() + 16, 0u);
            o->dfa.sbase = (const uint8_t*)dalloc_copy(o, im.dfa.sblock.data(), im.dfa.sblock.size() * 4);
            im.dfa.sblock.resize(im.dfa.sblock.size() - 16);
            o->dfa.sout = (const uint32_t*)dalloc_copy(o, im.dfa.sout.data(), im.dfa.sout.size() * 4);
            o->dfa.sF = im.dfa.sF;
            std::vector<uint32_t> b8, o8;  // the 8-B record units (pm_pack_sparse8)
            if (pm_pack_sparse8(im.dfa, b8, o8)) {
                b8.resize(b8.size() + 16, 0u);  // the last aligned 64-B block
                o->dfa.sbase8 = (const uint8_t*)dalloc_copy(o, b8.data(), b8.size() * 4);
                o->dfa.sout8 = (const uint32_t*)dalloc_copy(o, o8.data(), o8.size() * 4);
            }
            FlImage fl;  // the fallback-linked form (pm_pack_sparse_fl)
            const std::vector<uint8_t> prof = pm_fl_profile(o->pats);  // the LDS rows' profile
            if (pm_pack_sparse_fl(im.dfa, fl, &prof)) {
                fl.block.resize(fl.block.size() + 32, 0u);  // the last aligned 128-B block
                o->dfa.flbase = (const uint8_t*)dalloc_copy(o, fl.block.data(), fl.block.size() * 4);
                o->dfa.flrowout16 = (const uint16_t*)dalloc_copy(o, fl.rowout16.data(), fl.rowout16.size() * 2);
                o->dfa.flF = fl.F;
                o->dfa.flGD = fl.deep_g;
                o->dfa.flwords = (uint32_t)(fl.block.size() - 32);
            }
        }
    }
    // read_char's host step keeps the RT image (rt / auto), or the DFA's
    // sparse block (dense rows when it has none) for the ac kind
    o->host = PmHostStep();
    if (o->kind == KIND_RT || o->kind == KIND_AUTO) {
        o->host.kind = 1;
        o->host.rt = std::move(im.rt);
    } else {
        o->host.kind = 2;
        DfaImage& h = o->host.dfa;
        h.states = im.dfa.states;
        if (!im.dfa.sblock.empty()) {
            h.sblock = std::move(im.dfa.sblock);
            h.sout = std::move(im.dfa.sout);
            h.sF = im.dfa.sF;
        } else {
            h.next = std::move(im.dfa.next);
            h.out = std::move(im.dfa.out);
        }
    }
    o->hist.init(o->max_len);
    init_pick(o->pick, o->kind, o->dfa.sbase != nullptr);
    o->d_parent = (const uint32_t*)dalloc_copy(o, im.par.parent.data(), im.par.parent.size() * 4);
    o->d_depth = (const uint32_t*)dalloc_copy(o, im.par.depth.data(), im.par.depth.size() * 4);
    o->parent = std::move(im.par.parent);
    o->id_of_gid.assign(o->gids.index_of_gid.size(), PM_NULL_PATTERN_ID);
    for (size_t g = 1; g < o->gids.index_of_gid.size(); ++g) o->id_of_gid[g] = o->ids[o->gids.index_of_gid[g]];
    o->compiled = true;
    o->compile_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - tc0).count();
}

void pm_hip_host_profile(int on, double* out5) {
    if (out5)
        for (int k = 0; k < 5; ++k) out5[k] = g_hprof[k];
    for (double& x : g_hprof) x = 0.0;
    g_hprof_on = on != 0;
}

int pm_hip_read_block_gid(void* obj, const uint8_t* buf, size_t n, uint32_t* out_gid) {
    scan_host(as(obj), buf, n, out_gid, nullptr);
    return 0;
}

void pm_hip_read_block(void* obj, const char* buf, size_t n, pm_pattern_id_t* out) {
    scan_host(as(obj), reinterpret_cast<const uint8_t*>(buf), n, nullptr, out);
}

// The per-byte entry point of the reference ABI (mpac.c:304-319 contract,
// called per byte by measure.c:292-294).  One byte is far too little work for
// a launch, so it steps the host copy of the object's own flattened image
// (pm_hoststep.h): the reverse-trie walk over the carried history (rt /
// auto), or one transition of the flattened DFA (ac).  The history is the
// one read_block carries, so the two interleave exactly.
pm_pattern_id_t pm_hip_read_char(void* obj, char c) {
    PmHip* o = as(obj);
    if (!o->compiled) {
        std::fprintf(stderr, "pm_hip: read before compile\n");
        std::exit(EXIT_FAILURE);
    }
    return o->id_of_gid[pm_host_step(o->host, o->hist, o->max_len, (uint8_t)c)];
}

// Device tables + the host copy read_char steps + the object (the
// reference's total_mem counts the automaton the object holds, mpac.c:328).
size_t pm_hip_total_mem(void* obj) {
    PmHip* o = as(obj);
    return sizeof(PmHip) + o->table_bytes + o->host.bytes();
}

void pm_hip_reset(void* obj) {
    PmHip* o = as(obj);
    o->hist.clear();
    o->host.state_valid = false;
    o->dev_seconds = 0.0;
    o->untimed_calls = 0;
    // a new stream: the auto kernel choice is measured again, for read_block
    // slots and scan_device launches alike
    forget_pick(o->pick);
    for (PipeSlot& q : o->slot) forget_pick(q.pick);
}

void pm_hip_free(void* obj) {
    PmHip* o = as(obj);
    (void)hipSetDevice(o->device);
    serve_free(o);  // before the tables it reads
    for (void* p : o->allocs) (void)hipFree(p);
    if (o->spill) (void)hipFree(o->spill);
    for (StreamSpill& x : o->sspill) {
        if (x.buf) (void)hipFree(x.buf);
        if (x.done) (void)hipEventDestroy(x.done);
    }
    if (o->d_lines_pats) (void)hipFree(o->d_lines_pats);
    if (o->d_lines_offs) (void)hipFree(o->d_lines_offs);
    free_pick(o->pick);
    for (PipeSlot& q : o->slot) {
        free_slot(q);
        if (q.ev0) (void)hipEventDestroy(q.ev0);
        if (q.ev1) (void)hipEventDestroy(q.ev1);
        if (q.stream) (void)hipStreamDestroy(q.stream);
    }
    delete o;
}

static void fill_slot(PmMpsElem* slot, const char* name, void* (*create_fn)(void)) {
    slot->name = const_cast<char*>(name);
    slot->create = create_fn;
    slot->add_pattern = pm_hip_add_pattern;
    slot->compile = pm_hip_compile;
    slot->read_char = pm_hip_read_char;
    slot->total_mem = pm_hip_total_mem;
    slot->reset = pm_hip_reset;
    slot->free = pm_hip_free;
    slot->read_block = pm_hip_read_block;
}

void pm_mps_hip_rt_register(PmMpsElem* slot) { fill_slot(slot, "HIP Reverse-Trie", pm_hip_rt_create); }
void pm_mps_hip_ac_register(PmMpsElem* slot) { fill_slot(slot, "HIP Aho-Corasick DFA", pm_hip_ac_create); }
void pm_mps_hip_auto_register(PmMpsElem* slot) { fill_slot(slot, "HIP Auto (RT / AC per launch)", pm_hip_auto_create); }

static int scan_device(void* obj, const uint8_t* d_text, int64_t stream_start, int64_t pos0, int64_t n, void* d_out,
                       int outw, unsigned long long* d_count, void* hip_stream) {
    PmHip* o = as(obj);
    if (!o->compiled) { std::snprintf(g_err, sizeof(g_err), "not compiled"); return -1; }
    if (pos0 % 16 || stream_start > pos0 || stream_start < 0 || n < 0 || ((uintptr_t)d_text & 15) ||
        ((uintptr_t)d_out & 15)) {
        std::snprintf(g_err, sizeof(g_err), "bad arguments (pos0 %% 16, stream_start <= pos0, 16-B alignment)");
        return -2;
    }
    if (outw == 2 && d_out && o->gids.index_of_gid.size() > 65536) {
        std::snprintf(g_err, sizeof(g_err), "u16 ids need fewer than 65536 patterns (have %zu)",
                      o->gids.index_of_gid.size() - 1);
        return -4;
    }
    hipError_t e = hipSetDevice(o->device);
    serve_stop(o);  // a device launch wants the whole device
    if (e == hipSuccess) {
        // a captured launch keeps the compile-time scratch (a graph owns the
        // pointers it was captured with: replays of graphs of one object run
        // one at a time, as any graph's scratch); a direct one its stream's
        const hipStream_t s = (hipStream_t)hip_stream;
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        e = hipStreamIsCapturing(s, &cs);
        StreamSpill* sp = e == hipSuccess && cs == hipStreamCaptureStatusNone ? stream_spill(o, s, n) : nullptr;
        // Only the chunked RT kernel uses the scratch: a captured launch the
        // one-thread-per-position kernel takes (n <= the small-launch
        // bound), or one of an auto object whose held choice is a DFA form,
        // needs no prepare_capture.
        const int64_t small_max = o->rt.small_max >= 0 ? o->rt.small_max : RT_SMALL_MAX;
        const bool rt_next = o->kind == KIND_RT || (o->kind == KIND_AUTO && o->pick.chosen == CAND_RT);
        if (e == hipSuccess && cs != hipStreamCaptureStatusNone && !o->spill && rt_next && n > small_max) {
            // nothing launched: the capture stays valid for the caller to end
            std::snprintf(g_err, sizeof(g_err),
                          "scan_device under stream capture needs pm_hip_prepare_capture(obj) first (the RT "
                          "kernel's scratch cannot be allocated while a stream captures)");
            return -5;
        }
        if (e == hipSuccess)
            e = launch(o, d_text, stream_start, pos0, n, d_out, outw, d_count, s, sp ? sp->buf : o->spill,
                       sp ? sp->cap : o->spill_cap, o->pick);
        if (e == hipSuccess && sp) e = hipEventRecord(sp->done, s);
        o->last_kernel = o->pick.last ? o->pick.last : o->kind;
        o->last_form = o->pick.last_form;
    }
    if (e != hipSuccess) {
        std::snprintf(g_err, sizeof(g_err), "launch: %s", hipGetErrorString(e));
        return -3;
    }
    return 0;
}

int pm_hip_scan_device(void* obj, const uint8_t* d_text, int64_t stream_start, int64_t pos0, int64_t n,
                       uint32_t* d_out, unsigned long long* d_count, void* hip_stream) {
    return scan_device(obj, d_text, stream_start, pos0, n, d_out, 4, d_count, hip_stream);
}

int pm_hip_scan_device16(void* obj, const uint8_t* d_text, int64_t stream_start, int64_t pos0, int64_t n,
                         uint16_t* d_out, unsigned long long* d_count, void* hip_stream) {
    return scan_device(obj, d_text, stream_start, pos0, n, d_out, 2, d_count, hip_stream);
}

int pm_hip_score_device(void* obj, const uint32_t* d_algo, const uint32_t* d_real, int64_t n,
                        unsigned long long* d_counts, void* hip_stream) {
    PmHip* o = as(obj);
    if (!o->compiled) { std::snprintf(g_err, sizeof(g_err), "not compiled"); return -1; }
    if (n < 0 || !d_counts || ((uintptr_t)d_algo & 15) || ((uintptr_t)d_real & 15)) {
        std::snprintf(g_err, sizeof(g_err), "bad arguments (n >= 0, counts, 16-B alignment)");
        return -2;
    }
    hipError_t e = hipSetDevice(o->device);
    if (e == hipSuccess)
        e = pm_launch_score(d_algo, d_real, n, o->d_parent, o->d_depth, d_counts, o->num_cu, (hipStream_t)hip_stream);
    if (e != hipSuccess) {
        std::snprintf(g_err, sizeof(g_err), "score launch: %s", hipGetErrorString(e));
        return -3;
    }
    return 0;
}

int pm_hip_pattern_counts_device(void* obj, const uint32_t* d_ids, int64_t n, unsigned long long* d_hist,
                                 void* hip_stream) {
    PmHip* o = as(obj);
    if (!o->compiled) { std::snprintf(g_err, sizeof(g_err), "not compiled"); return -1; }
    if (n < 0 || !d_hist || ((uintptr_t)d_ids & 15)) {
        std::snprintf(g_err, sizeof(g_err), "bad arguments (n >= 0, hist, 16-B alignment)");
        return -2;
    }
    hipError_t e = hipSetDevice(o->device);
    if (e == hipSuccess)
        e = pm_launch_pattern_counts(d_ids, n, o->d_parent, (uint32_t)o->parent.size(), d_hist, o->num_cu,
                                     (hipStream_t)hip_stream);
    if (e != hipSuccess) {
        std::snprintf(g_err, sizeof(g_err), "pattern counts launch: %s", hipGetErrorString(e));
        return -3;
    }
    return 0;
}

int pm_hip_prepare_capture(void* obj) {
    PmHip* o = as(obj);
    if (!o->compiled) { std::snprintf(g_err, sizeof(g_err), "not compiled"); return -1; }
    if (hipSetDevice(o->device) != hipSuccess) { std::snprintf(g_err, sizeof(g_err), "set device"); return -3; }
    ensure_spill(o, o->spill, o->spill_cap, INT64_MAX);  // the bound for any scan_device launch
    init_pick(o->pick, o->kind, o->dfa.sbase != nullptr);
    return 0;
}

size_t pm_hip_scratch_bytes(void* obj) {
    PmHip* o = as(obj);
    size_t b = (size_t)o->spill_cap * 8;
    for (const StreamSpill& x : o->sspill) b += (size_t)x.cap * 8;
    for (const PipeSlot& q : o->slot)
        b += (size_t)q.spill_cap * 8 + (q.d_stage ? q.cap * sizeof(uint32_t) + q.cap + o->max_len + 64 : 0);
    return b;
}

int pm_hip_hold_choice(void* obj, int launches) {
    PmHip* o = as(obj);
    if (o->kind == KIND_RT || (o->kind == KIND_AC && (!o->dfa.sbase || o->dfa_form))) return 0;
    AutoPick& ap = o->pick;
    resolve_pick(o, ap);
    if (ap.pending || ap.timing || ap.hold <= 0) return -1;
    ap.hold = std::max(ap.hold, launches);
    return 1 + ap.chosen;
}

void pm_hip_set_image_cache(void* obj, const char* dir) { as(obj)->cache_dir = dir ? dir : ""; }

int pm_hip_serve_stats(void* obj, uint64_t* launches, uint64_t* calls) {
    const PmHip* o = as(obj);
    if (launches) *launches = o->srv.launches;
    if (calls) *calls = o->srv.calls;
    return 0;
}

int pm_hip_image_cache_hit(void* obj) { return as(obj)->cache_hit ? 1 : 0; }

int pm_hip_compile_stats(void* obj, double* compile_ms, double* upload_ms) {
    const PmHip* o = as(obj);
    if (!o->compiled) return -1;
    if (compile_ms) *compile_ms = o->compile_s * 1e3;
    if (upload_ms) *upload_ms = o->upload_s * 1e3;
    return 0;
}

uint32_t pm_hip_parent_gid(void* obj, uint32_t gid) {
    PmHip* o = as(obj);
    if (!o->compiled || gid >= o->parent.size()) return UINT32_MAX;
    return o->parent[gid];
}

// Timing-only ablation launches of the RT kernel (bench_variants.py).
int pm_hip_streaming_floor_device(void* obj, const uint8_t* d_text, int64_t n, void* d_out, int out_width,
                                  void* hip_stream) {
    PmHip* o = as(obj);
    if (o->kind != KIND_RT && o->kind != KIND_AUTO) return -1;
    ensure_spill(o, o->spill, o->spill_cap, n);
    RtDev t = o->rt;
    t.spill = o->spill;
    t.spill_cap = o->spill_cap;
    hipError_t e = pm_launch_rt_floor(d_text, n, d_out, out_width, t, o->num_cu, (hipStream_t)hip_stream);
    return e == hipSuccess ? 0 : -3;
}

int pm_hip_gather_ceiling_device(void* obj, int steps, uint32_t* d_sink, void* hip_stream) {
    PmHip* o = as(obj);
    if (!o->compiled || !o->dfa.flbase) return -2;
    hipError_t e = hipSetDevice(o->device);
    if (e == hipSuccess)
        e = pm_launch_gather_probe(reinterpret_cast<const uint32_t*>(o->dfa.flbase), o->dfa.flwords, steps, d_sink,
                                   o->num_cu, (hipStream_t)hip_stream);
    if (e != hipSuccess) {
        std::snprintf(g_err, sizeof(g_err), "gather_ceiling: %s", hipGetErrorString(e));
        return -3;
    }
    return 0;
}

int pm_hip_set_option(void* obj, const char* name, int64_t value) {
    PmHip* o = as(obj);
    if (!name) return -1;
    const std::string k(name);
    auto flag = [&](int& dst) {  // -1 = the environment's default, 0 / 1
        if (value < -1 || value > 1) return -1;
        dst = (int)value;
        return 0;
    };
    if (k == "dfa_form") {
        if (value < 0 || value > 2) return -1;
        o->dfa_form = (int)value;
        forget_pick(o->pick);  // the choice is measured again
        for (PipeSlot& q : o->slot) forget_pick(q.pick);
        return 0;
    }
    if (k == "sparse_kernel") {
        if (value < PM_SK_PRODUCT || value > PM_SK_LOCK16) return -1;
        o->dfa.sparse_kernel = (int)value;
        return 0;
    }
    if (k == "fl_hold") {
        if (value != 0 && value != 1 && value != 2 && value != 4) return -1;
        o->dfa.flhold = value ? (int)value : 2;
        return 0;
    }
    if (k == "fl_chains") {
        if (value < 0 || value > 2) return -1;
        o->dfa.flchains = value ? (int)value : 1;
        return 0;
    }
    if (k == "dfa_sync") {
        if (value < 0 || value > 1) return -1;
        o->dfa.sync = (int)value;
        return 0;
    }
    if (k == "rt_small_max") {
        if (value < -1) return -1;
        o->rt.small_max = value;
        return 0;
    }
    if (k == "spill_cap_chunks") {
        if (value < 0 || value > 16) return -1;
        o->rt.spill_cap_chunks = value;
        return 0;
    }
    if (k == "host_spin") return flag(o->hopt.spin);
    if (k == "host_gid16") return flag(o->hopt.gid16);
    if (k == "host_events") return flag(o->hopt.events);
    if (k == "host_pool") return flag(o->hopt.pool);
    if (k == "serve_idle_us") {  // the server grid's idle life (>= 10 us; -1 = the default)
        if (value != -1 && (value < 10 || value > 10000000)) return -1;
        o->srv.idle_us = value;
        serve_stop(o);  // the next call launches a grid with it
        return 0;
    }
    if (k == "host_serve") {
        if (value == 0) serve_stop(o);
        return flag(o->hopt.serve);
    }
    return -1;
}

int pm_hip_gen_stream_device(uint8_t* d_dst, uint64_t offset, uint64_t n, uint64_t seed, int mode,
                             void* hip_stream) {
    hipError_t e = pm_launch_gen(d_dst, offset, n, seed, mode, (hipStream_t)hip_stream);
    if (e != hipSuccess) {
        std::snprintf(g_err, sizeof(g_err), "gen: %s", hipGetErrorString(e));
        return -3;
    }
    return 0;
}

static void lines_table(PmHip* o) {
    if (!o->lines_offs.empty()) return;
    o->lines_offs.push_back(0);
    for (const std::string& p : o->pats) {
        o->lines_pats.insert(o->lines_pats.end(), p.begin(), p.end());
        o->lines_offs.push_back((uint32_t)o->lines_pats.size());
    }
    if (o->lines_pats.empty()) o->lines_pats.push_back(0);
}

int pm_hip_gen_lines_device(void* obj, uint8_t* d_dst, uint64_t n, uint64_t seed, void* hip_stream) {
    PmHip* o = as(obj);
    if (o->pats.empty()) {
        std::snprintf(g_err, sizeof(g_err), "gen_lines: no patterns");
        return -2;
    }
    lines_table(o);
    hipError_t e = hipSetDevice(o->device);  // the object's device, like every other entry point
    if (e == hipSuccess && !o->d_lines_pats) {
        e = hipMalloc(&o->d_lines_pats, o->lines_pats.size());
        if (e == hipSuccess) e = hipMalloc(&o->d_lines_offs, o->lines_offs.size() * sizeof(uint32_t));
        if (e == hipSuccess)
            e = hipMemcpy(o->d_lines_pats, o->lines_pats.data(), o->lines_pats.size(), hipMemcpyHostToDevice);
        if (e == hipSuccess)
            e = hipMemcpy(o->d_lines_offs, o->lines_offs.data(), o->lines_offs.size() * sizeof(uint32_t),
                          hipMemcpyHostToDevice);
        if (e != hipSuccess) {  // leave no half-made tables behind
            if (o->d_lines_pats) (void)hipFree(o->d_lines_pats);
            if (o->d_lines_offs) (void)hipFree(o->d_lines_offs);
            o->d_lines_pats = nullptr;
            o->d_lines_offs = nullptr;
        }
    }
    if (e == hipSuccess)
        e = pm_launch_gen_lines(d_dst, n, o->d_lines_pats, o->d_lines_offs, (uint32_t)o->pats.size(), seed,
                                (hipStream_t)hip_stream);
    if (e != hipSuccess) {
        std::snprintf(g_err, sizeof(g_err), "gen_lines: %s", hipGetErrorString(e));
        return -3;
    }
    return 0;
}

void pm_gen_lines_host(void* obj, uint8_t* dst, uint64_t n, uint64_t seed) {
    PmHip* o = as(obj);
    if (o->pats.empty()) return;
    lines_table(o);
    for (uint64_t lo = 0, b = 0; lo < n; lo += PM_LINES_BLOCK, ++b)
        pm_lines_block(dst + lo, n - lo < PM_LINES_BLOCK ? n - lo : PM_LINES_BLOCK, b, o->lines_pats.data(),
                       o->lines_offs.data(), (uint32_t)o->pats.size(), seed);
}

// The lines stream of a dictionary's patterns (first-occurrence order, the
// order pm_dict_feed gives a matcher), with no matcher object: the CPU
// baseline's deep-input sample (bench.py), generated before any GPU call.
void pm_gen_lines_dict(const PmDict* d, uint8_t* dst, uint64_t n, uint64_t seed) {
    if (!d || d->n == 0) return;
    std::vector<uint8_t> pats;
    std::vector<uint32_t> offs(1, 0);
    for (size_t k = 0; k < d->n; ++k) {
        pats.insert(pats.end(), d->pats[k].bytes, d->pats[k].bytes + d->pats[k].len);
        offs.push_back((uint32_t)pats.size());
    }
    for (uint64_t lo = 0, b = 0; lo < n; lo += PM_LINES_BLOCK, ++b)
        pm_lines_block(dst + lo, n - lo < PM_LINES_BLOCK ? n - lo : PM_LINES_BLOCK, b, pats.data(), offs.data(),
                       (uint32_t)d->n, seed);
}

void pm_gen_stream_host(uint8_t* dst, uint64_t offset, uint64_t n, uint64_t seed, int mode) {
    for (uint64_t k = 0; k < n; ++k) dst[k] = pm_stream_byte(offset + k, seed, mode);
}

uint32_t pm_hip_n_patterns(void* obj) { return (uint32_t)as(obj)->pats.size(); }
uint32_t pm_hip_max_pattern_len(void* obj) { return as(obj)->max_len; }
uint32_t pm_hip_gid_index(void* obj, uint32_t gid) {
    PmHip* o = as(obj);
    if (gid == 0 || gid >= o->gids.index_of_gid.size()) return UINT32_MAX;
    return o->gids.index_of_gid[gid];
}
int pm_hip_kernel_kind(void* obj) { return as(obj)->kind; }
int pm_hip_kernel_last(void* obj) { return as(obj)->last_kernel; }
int pm_hip_dfa_form_last(void* obj) { return as(obj)->last_form; }
int pm_hip_sparse_kernel_last(void* obj) { return as(obj)->last_sparse_kernel; }
double pm_hip_device_seconds(void* obj) {
    const PmHip* o = as(obj);
    return o->untimed_calls ? -1.0 : o->dev_seconds;
}
int pm_hip_last_out_width(void* obj) { return as(obj)->last_out_width; }
double pm_hip_hbm_peak_gbs(void) { return PM_HBM_PEAK_GBS; }
size_t pm_hip_table_bytes(void* obj) { return as(obj)->table_bytes; }

}  // extern "C"

// ---- host-only table export (tests validate the flattened images on CPU) --
namespace {
struct PmFlatHandle {
    PmGidMap g;
    RtImage rt;
    DfaImage dfa;
    PmParents par;
    std::vector<uint32_t> block8, out8;  // pm_pack_sparse8 of the DFA's sparse form
    FlImage fl;                          // pm_pack_sparse_fl of it
    std::vector<uint32_t> flinfo;        // pm_flat_array "flinfo"
    bool has_fl = false;
    int kind = 0;
    bool hit = false;
};
}  // namespace

extern "C" {

void* pm_flat_build_cached(const char* const* pats, const uint32_t* lens, size_t n, int kind, const char* cache_dir) {
    std::vector<std::string> v;
    v.reserve(n);
    for (size_t i = 0; i < n; ++i) v.emplace_back(pats[i], lens[i]);
    PmFlatHandle* h = new PmFlatHandle();
    h->kind = kind;
    h->g = pm_assign_gids(v);
    PmImages im = pm_build_images_cached(v, h->g, kind, cache_dir ? cache_dir : "", &h->hit);
    h->rt = std::move(im.rt);
    h->dfa = std::move(im.dfa);
    h->par = std::move(im.par);
    if (!pm_pack_sparse8(h->dfa, h->block8, h->out8)) h->block8.clear(), h->out8.clear();
    const std::vector<uint8_t> prof = pm_fl_profile(v);  // as compile() does
    h->has_fl = pm_pack_sparse_fl(h->dfa, h->fl, &prof);
    return h;
}

void* pm_flat_build(const char* const* pats, const uint32_t* lens, size_t n, int kind) {
    return pm_flat_build_cached(pats, lens, n, kind, nullptr);
}

int pm_flat_cache_hit(void* handle) { return static_cast<PmFlatHandle*>(handle)->hit ? 1 : 0; }

uint32_t pm_flat_dfa_sparse_rows(void* handle) { return static_cast<PmFlatHandle*>(handle)->dfa.sF; }

int pm_flat_fits(void* handle) { return static_cast<PmFlatHandle*>(handle)->rt.fits ? 1 : 0; }

size_t pm_flat_array(void* handle, const char* name, const void** data, size_t* elem_size) {
    PmFlatHandle* h = static_cast<PmFlatHandle*>(handle);
    auto ret = [&](const auto& vec) {
        *data = vec.data();
        *elem_size = sizeof(vec[0]);
        return vec.size();
    };
    std::string s(name);
    if (s == "t12") return ret(h->rt.t12);
    if (s == "filt") return ret(h->rt.filt);
    if (s == "t3h") return ret(h->rt.t3h);
    if (s == "rec") return ret(h->rt.rec);
    if (s == "wide") return ret(h->rt.wide);
    if (s == "next") return ret(h->dfa.next);
    if (s == "out") return ret(h->dfa.out);
    if (s == "sblock") return ret(h->dfa.sblock);
    if (s == "sout") return ret(h->dfa.sout);
    if (s == "sblock8") return ret(h->block8);
    if (s == "sout8") return ret(h->out8);
    if (s == "flblock") return ret(h->fl.block);
    if (s == "flrowout16") return ret(h->fl.rowout16);
    if (s == "flinfo") {  // {F, granules, folded records, first deep granule}
        h->flinfo = {h->fl.F, h->fl.granules, h->fl.folded, h->fl.deep_g};
        return ret(h->flinfo);
    }
    if (s == "index_of_gid") return ret(h->g.index_of_gid);
    if (s == "parent") return ret(h->par.parent);
    if (s == "depth") return ret(h->par.depth);
    *data = nullptr;
    *elem_size = 0;
    return 0;
}

// read_char's host step (pm_hoststep.h) over a whole text from the stream
// start: the RT walk (kind 1), or the DFA step (kind 2; its sparse form, or
// dense rows when dense_rows is 1 or it has no sparse form; dense_rows 2:
// the fallback-linked form's host reference, pm_fl_host_step).  CPU tests.
int pm_flat_host_scan(void* handle, const uint8_t* text, size_t n, uint32_t* out_gid, int dense_rows) {
    PmFlatHandle* h = static_cast<PmFlatHandle*>(handle);
    if (h->kind == 2 && dense_rows == 2) {
        if (!h->has_fl) return -1;
        uint32_t w = 0;
        for (size_t k = 0; k < n; ++k) {
            w = pm_fl_host_step(h->fl, w, text[k], nullptr);
            out_gid[k] = pm_fl_output(h->fl, w);
        }
        return 0;
    }
    PmHostStep st;
    uint32_t max_len = 0;
    if (h->kind == 1) {
        if (!h->rt.fits) return -1;
        st.kind = 1;
        st.rt = h->rt;
        max_len = 512;  // RtImage::fits bounds patterns below 512 bytes
    } else {
        st.kind = 2;
        st.dfa.states = h->dfa.states;
        if (!dense_rows && !h->dfa.sblock.empty()) {
            st.dfa.sblock = h->dfa.sblock;
            st.dfa.sout = h->dfa.sout;
            st.dfa.sF = h->dfa.sF;
        } else {
            st.dfa.next = h->dfa.next;
            st.dfa.out = h->dfa.out;
        }
    }
    PmHistRing r;
    r.init(max_len);
    for (size_t k = 0; k < n; ++k) out_gid[k] = pm_host_step(st, r, max_len, text[k]);
    return 0;
}

void pm_flat_free(void* handle) { delete static_cast<PmFlatHandle*>(handle); }

}  // extern "C"
