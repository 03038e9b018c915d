// common.hpp -- error plumbing, device buffers and small device helpers shared by
// the npge_amd HIP translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/npge_amd.h"

namespace npgx {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string& msg);

// Waits for a stream by polling (hipStreamQuery) instead of the runtime's
// blocking wait: the host thread is dedicated to the pipeline, and a blocking
// wait costs an interrupt and a thread wake-up (tens of microseconds) at each
// of the block build's many short host<->device round trips.
hipError_t stream_wait(hipStream_t s);

#define NPGX_HIP(call)                                                                \
    do {                                                                              \
        hipError_t e_ = (call);                                                       \
        if (e_ != hipSuccess)                                                         \
            throw ::npgx::Error(NPGX_ERR_HIP, std::string(#call) + ": " +             \
                                                  hipGetErrorString(e_));             \
    } while (0)

#define NPGX_REQUIRE(cond, code, msg)                     \
    do {                                                  \
        if (!(cond)) throw ::npgx::Error((code), (msg));  \
    } while (0)

// Runs f, converts exceptions into a status code + thread-local message.
template <class F>
int guard(F&& f) {
    try {
        f();
        return NPGX_OK;
    } catch (const Error& e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return NPGX_ERR_ARG;
    } catch (...) {
        set_last_error("unknown error");
        return NPGX_ERR_ARG;
    }
}

// Device (kind 0) and pinned host (kind 1) allocations, optionally through a
// cache of freed buffers (NPGX_BUF_CACHE=1; seqset.hip: size classes, one
// device synchronisation before freed buffers are reused, reused device
// buffers zeroed).  buf_alloc sets *got to the bytes actually held (what
// buf_free takes back).
void* buf_alloc(int kind, size_t bytes, size_t* got);
void buf_free(int kind, void* p, size_t got);

// Growable device buffer (capacity kept across runs so repeated steps do not
// re-allocate).
template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t cap = 0;
    size_t held = 0;  // bytes of the allocation
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) buf_free(0, p, held);
        p = nullptr;
        cap = 0;
        held = 0;
    }
    T* ensure(size_t n) {
        if (n == 0) n = 1;
        if (n > cap) {
            release();
            p = (T*)buf_alloc(0, n * sizeof(T), &held);
            cap = n;
        }
        return p;
    }
    // ensure() with 1.5x headroom for buffers whose size varies from call to call
    T* grow(size_t n) { return ensure(n > cap ? std::max(n, cap + cap / 2) : n); }
    void swap(DevBuf& o) {
        std::swap(p, o.p);
        std::swap(cap, o.cap);
        std::swap(held, o.held);
    }
};

// Pinned host buffer that only grows.
template <class T>
struct PinnedBuf {
    T* p = nullptr;
    size_t cap = 0;
    size_t held = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    ~PinnedBuf() {
        if (p) buf_free(1, p, held);
    }
    T* ensure(size_t n) {
        if (n == 0) n = 1;
        if (n > cap) {
            if (p) buf_free(1, p, held);
            p = nullptr;
            cap = std::max(n, cap + cap / 2);
            p = (T*)buf_alloc(1, cap * sizeof(T), &held);
        }
        return p;
    }
};

// Pinned host staging for async copies (bump allocated; when full, the stream
// is synchronised so every earlier copy from it has completed).
struct PinnedArena {
    char* p = nullptr;
    size_t cap = 0, used = 0, held = 0;
    PinnedArena() = default;
    PinnedArena(const PinnedArena&) = delete;
    PinnedArena& operator=(const PinnedArena&) = delete;
    ~PinnedArena() {
        if (p) buf_free(1, p, held);
    }
    char* take(size_t n, hipStream_t st) {
        n = (n + 63) & ~(size_t)63;
        if (used + n > cap) {
            NPGX_HIP(stream_wait(st));
            used = 0;
            if (n > cap) {
                if (p) buf_free(1, p, held);
                p = nullptr;
                cap = std::max<size_t>(std::max<size_t>(n, 2 * cap), (size_t)1 << 22);
                p = (char*)buf_alloc(1, cap, &held);
            }
        }
        char* r = p + used;
        used += n;
        return r;
    }
    void reset() { used = 0; }  // only with no copy from it in flight
};

// Stage timer: pairs of HIP events on one stream.
struct StageTimer {
    struct Rec {
        std::string name;
        hipEvent_t a, b;
        double bytes;
        int64_t units;
    };
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;
    size_t used = 0;
    ~StageTimer() {
        for (auto e : pool) (void)hipEventDestroy(e);
    }
    hipEvent_t get() {
        if (used == pool.size()) {
            hipEvent_t e;
            NPGX_HIP(hipEventCreate(&e));
            pool.push_back(e);
        }
        return pool[used++];
    }
    void reset() {
        recs.clear();
        used = 0;
    }
    // Every event record is a marker packet in the queue that costs the GPU a
    // few microseconds between the kernels around it (C3: 1.6 ms a step with
    // every launch timed).  NPGX_TIMERS: 0 = none; 1 (default) = the launches
    // the benches' rooflines read (k_align_jobs, k_align_wide, k_general_align,
    // by name); 2 = every launch
    // (the diagnostics in tools/ set it).
    static int level_from_env() {
        const char* e = getenv("NPGX_TIMERS");
        if (!e || !*e) return 1;
        return e[0] == '0' ? 0 : e[0] == '2' ? 2 : 1;
    }
    static bool key_launch(const char* name) {
        return strcmp(name, "align_jobs") == 0 || strcmp(name, "align_jobs_retry") == 0 ||
               strcmp(name, "align_wide") == 0 || strcmp(name, "general_align") == 0;
    }
    int level = level_from_env();
    static constexpr size_t NONE = ~(size_t)0;
    size_t begin(const char* name, hipStream_t s, double bytes, int64_t units) {
        if (level == 0 || (level == 1 && !key_launch(name))) return NONE;
        Rec r{name, get(), get(), bytes, units};
        NPGX_HIP(hipEventRecord(r.a, s));
        recs.push_back(r);
        return recs.size() - 1;
    }
    void end(size_t i, hipStream_t s) {
        if (i != NONE) NPGX_HIP(hipEventRecord(recs[i].b, s));
    }
    int copy_out(npgx_kernel_time* out, int32_t cap, int32_t* n) const {
        int32_t k = 0;
        for (const Rec& r : recs) {
            if (k >= cap) break;
            float ms = 0.f;
            // (the end marker may still be in the queue when the caller waited on
            // the work itself, not on the marker: wait for it)
            if (hipEventSynchronize(r.b) != hipSuccess || hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) ms = -1.f;
            snprintf(out[k].name, sizeof(out[k].name), "%s", r.name.c_str());
            out[k].ms = ms;
            out[k].bytes = r.bytes;
            out[k].units = r.units;
            k++;
        }
        *n = (int32_t)recs.size();
        return NPGX_OK;
    }
};

// Step timeline: one HIP event at each stage boundary of a step on one stream;
// the interval ending at a marker is booked to that marker's stage, so the
// stages sum to the step's GPU-timeline span (device time plus the idle time
// the host leaves between them).  Off unless a caller turns it on: every
// marker is a queue packet that costs the GPU a few microseconds (bench.py
// runs one extra, untimed step with it).
struct StageClock {
    bool on = false;
    bool live = false;  // between start() and collect()
    std::vector<std::pair<hipEvent_t, int>> marks;
    std::vector<hipEvent_t> pool;
    ~StageClock() {
        for (auto e : pool) (void)hipEventDestroy(e);
    }
    void start(hipStream_t s) {
        marks.clear();
        live = on;
        mark(s, -1);
    }
    void mark(hipStream_t s, int stage) {
        if (!live) return;
        if (marks.size() == pool.size()) {
            hipEvent_t e;
            NPGX_HIP(hipEventCreate(&e));
            pool.push_back(e);
        }
        hipEvent_t e = pool[marks.size()];
        NPGX_HIP(hipEventRecord(e, s));
        marks.emplace_back(e, stage);
    }
    // out[stage] += ms of every interval; the caller has waited for the work
    void collect(double* out, int nstages) {
        if (!live) return;
        live = false;
        for (size_t i = 1; i < marks.size(); i++) {
            float ms = 0.f;
            NPGX_HIP(hipEventSynchronize(marks[i].first));
            NPGX_HIP(hipEventElapsedTime(&ms, marks[i - 1].first, marks[i].first));
            const int k = marks[i].second;
            if (k >= 0 && k < nstages) out[k] += ms;
        }
        marks.clear();
    }
};

int current_device_checked();

// Makes `device` current for the guard's scope and restores the calling
// thread's previous device on every exit path (a collective callback must not
// move the caller's later HIP work to the communicator's device).
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(device) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

// Small persistent host thread pool for the block bookkeeping that is
// independent per block (hashing).  run(n, f) calls f(i) for i < n on the
// workers and the calling thread and returns when all are done.
class HostPool {
  public:
    explicit HostPool(int threads);
    ~HostPool();
    HostPool(const HostPool&) = delete;
    HostPool& operator=(const HostPool&) = delete;
    void run(size_t n, const std::function<void(size_t)>& f);
    int size() const { return (int)workers_.size() + 1; }

  private:
    void loop();
    std::vector<std::thread> workers_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(size_t)>* f_ = nullptr;
    size_t n_ = 0;
    std::atomic<size_t> next_{0};
    int active_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// f(i) for i < n; with at least 2^20 units of work in all, on a persistent
// pool of up to OMP_NUM_THREADS (else 16) host threads (seqset.hip), each
// taking the next index; the first exception is rethrown
void heavy_for(size_t n, int64_t work, const std::function<void(size_t)>& f);

// similar_aligner.hip: batched align_seqs (results in the aligner's host buffers)
void align_batch(npgx_aligner* al, const char* rows, const int64_t* row_off,
                 const int32_t* job_row_start, int32_t n_jobs);
// device-resident batch: results stay in the aligner's scratch
struct AlignResult {
    std::vector<int32_t> len;          // alignment length per job
    std::vector<int32_t> cap;          // row stride of the job's output
    std::vector<int32_t> n;            // non-empty rows per job
    std::vector<const char*> bptr;     // device address of the job's first output row
    std::vector<int64_t> row_ne;       // batch row -> index among its job's non-empty rows (-1: empty)
};
// job j's gapped rows on the device: row k at p + k * stride, len columns
struct JobRows {
    const char* p;
    int32_t stride, len;
};
// align_device without a host wait (the device ExtendLoopFast): the jobs that
// overflow the first attempt re-run at the proven bound in the same stream
// (their list made on the device), and every job's result goes to `out`
// (device, one JobRows per job); `err` (device) is set when a job overflows
// both attempts.  No job may have more than 64 non-empty rows (k_align_wide
// is host-driven); AlignResult is left empty.
// a sequence of an AnchorFinder run, by rank (anchor_finder.hip)
struct SeqMeta {
    int64_t size;
    int64_t word_off;
    int64_t n_off;
    uint64_t order_off;   // sum of sizes of lower-ranked eligible sequences
};

// The last AnchorFinder run's sorted FoundFragment keys on the device, when
// the run deferred its host result (af_set_defer): key = group index <<
// key_bits | 2 * order_off(rank) + position (the reverse strand's positions
// after the direct ones), the first `keep` keys kept (max-anchor-fragments)
struct AfDevKeys {
    const uint64_t* keys;
    int64_t keep;
    int key_bits, k;
    int32_t R;              // eligible sequences (the ranks with meta)
    const SeqMeta* meta;    // by rank
    const int32_t* by_rank; // rank -> input index
};
void af_set_defer(npgx_af* af, bool on);
bool af_device_keys(npgx_af* af, AfDevKeys* out);  // false: no deferred result pending

struct AlignAsync {
    JobRows* out;
    int32_t* err;
    uint32_t* epoch;  // (device) the launches' highest word-table epoch; hand it back with aligner_note_epoch
    // optional, uniform jobs (the device ExtendLoopFast's flank batches):
    // job j is ujobs[j].x rows of ujobs[j].y > 0 letters each, its rows
    // consecutive in the device arrays d_row_off / d_row_len (the caller's
    // plan wrote them); the host row arrays of align_device are then unused
    const int2* ujobs = nullptr;
    const int64_t* d_row_off = nullptr;
    const int32_t* d_row_len = nullptr;
};
// the highest word-table epoch an async call reached (read from AlignAsync::epoch
// after the caller's wait): the next call's tables start above it
void aligner_note_epoch(npgx_aligner* al, uint32_t epoch);
void aligner_set_long_head(npgx_aligner* al, int32_t long_head);
int32_t aligner_long_head(const npgx_aligner* al);
void align_device(npgx_aligner* al, const char* d_rows, const int64_t* row_off, const int32_t* row_len,
                  const int32_t* job_row_start, int32_t n_jobs, AlignResult& res, const AlignAsync* as = nullptr);
// wide_aligner.hip: align_seqs for problems of more than 64 non-empty rows (one
// workgroup per problem); results stay in the WideBufs (row r at ptr + r * cap)
struct WideJobIn {
    int64_t row0;  // first of the problem's non-empty rows in ne_off / ne_len
    int32_t n, pad;
};
struct WideBufs;
WideBufs* wide_create();
void wide_free(WideBufs* w);
void align_wide(WideBufs* w, hipStream_t st, const char* d_rows, const int64_t* ne_off, const int32_t* ne_len,
                int64_t n_ne, const std::vector<WideJobIn>& in, const int params[5], int aligner_type,
                std::vector<int32_t>& len, std::vector<int32_t>& cap, std::vector<const char*>& ptr,
                double* wait_ms = nullptr);
void aligner_timer_reset(npgx_aligner* al);
const std::vector<int64_t>& aligner_job_stats(const npgx_aligner* al);
bool aligner_wants_stats(const npgx_aligner* al);
void aligner_host_ms(npgx_aligner* al, double* prep, double* wait);  // read and clear
hipStream_t aligner_stream(const npgx_aligner* al);
const char* aligner_result(const npgx_aligner* al, const int64_t** row_off);
std::string genome_of(const std::string& name);
// a sequence set over text already on the device: sequence i is
// [off[i], off[i+1]) of d_text and of host_text (ATGCN only), named names[i]
npgx_seqset* seqset_from_device(const char* host_text, const char* d_text, const std::vector<int64_t>& off,
                                const std::vector<std::string>& names);
void pack_device(npgx_seqset* s, const unsigned char* d_ascii, const std::vector<int64_t>& ascii);

}  // namespace npgx

// ----------------------------------------------------------------- sequence set
inline uint64_t npgx_next_uid() {
    static std::atomic<uint64_t> n{0};
    return ++n;
}

struct npgx_seqset {
    uint64_t uid = npgx_next_uid();  // unique per set made (device caches key on it, not on the address)
    int device = 0;
    int32_t n = 0;
    std::vector<std::string> names;
    std::vector<std::string> data;       // after to_atgcn (input order)
    std::vector<int32_t> rank_of;        // input index -> rank
    std::vector<int32_t> by_rank;        // rank -> input index
    // device layout, in rank order
    std::vector<int64_t> word_off;       // first uint64 word of rank r (32 bases/word)
    std::vector<int64_t> n_off;          // first uint64 word of the N bitmap of rank r
    int64_t total_words = 0, total_nwords = 0;
    npgx::DevBuf<uint64_t> words, nmask;
    double ms_host = 0, ms_upload = 0;   // npgx_seqset_create: host to_atgcn / H2D + k_pack
};
