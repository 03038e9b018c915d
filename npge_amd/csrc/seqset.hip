// seqset.hip -- device-resident 2-bit sequence storage.
//
// Replaces the CompactLowNSequence storage (src/model/Sequence.cpp:525-600: 4 nt
// per byte, A0 T1 G2 C3, LSB first, plus a sorted vector of N positions) with an
// HBM layout built for coalesced window loads:
//   * words: uint64, 32 bases per word, base i of a sequence at bits 2*(i%32) of
//     word off+i/32 -- byte-for-byte the reference's packing, widened to 64 bits;
//     every sequence starts on a word boundary and is followed by one zero word so
//     a window load may always read word w+1.
//   * nmask: uint64, bit i%64 of word noff+i/64 set iff base i is N (N's 2-bit code
//     is 0, as in CompactLowNSequence::set_item :587-591).
// Sequences are stored in processing (rank) order: size desc, name asc, input
// index asc (the pinned form of SeqI.hpp:54).
#include <algorithm>
#include <chrono>
#include <cstring>
#include <mutex>
#include <thread>
#include <memory>
#include <map>
#include <numeric>
#include <tuple>

#include "common.hpp"

namespace npgx {

static thread_local std::string g_last_error;
void set_last_error(const std::string& m) { g_last_error = m; }

int current_device_checked() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        throw Error(NPGX_ERR_NODEV, "no HIP device available");
    int d = 0;
    NPGX_HIP(hipGetDevice(&d));
    return d;
}

// Sequence::to_atgcn (Sequence.cpp:151-179) as a 256-entry table:
// 0 = drop, else the output letter.
static const unsigned char* atgcn_table() {
    static unsigned char t[256];
    static std::once_flag once;
    std::call_once(once, [] {
        memset(t, 0, sizeof(t));
        const char* keep = "ATGCN";
        for (const char* c = keep; *c; c++) {
            t[(unsigned char)*c] = (unsigned char)*c;
            t[(unsigned char)tolower(*c)] = (unsigned char)*c;
        }
        const char* iupac = "RYMKWSBVHD";
        for (const char* c = iupac; *c; c++) {
            t[(unsigned char)*c] = 'N';
            t[(unsigned char)tolower(*c)] = 'N';
        }
    });
    return t;
}

std::string to_atgcn(const char* s, int64_t len) {
    const unsigned char* t = atgcn_table();
    std::string out;
    out.resize((size_t)len);
    int64_t k = 0;
    for (int64_t i = 0; i < len; i++) {
        unsigned char c = t[(unsigned char)s[i]];
        if (c) out[(size_t)k++] = (char)c;
    }
    out.resize((size_t)k);
    return out;
}

// One thread packs 32 bases of ASCII (already ATGCN) into one word; one wave's
// 64 words also yield 32 N-bitmap words via pairs of lanes.
__global__ void k_pack(const unsigned char* __restrict__ ascii, const int64_t* __restrict__ seq_word_off,
                       const int64_t* __restrict__ seq_ascii_off, const int64_t* __restrict__ seq_n_off,
                       const int64_t* __restrict__ seq_size, int32_t n_seqs,
                       int64_t total_words, uint64_t* __restrict__ words, uint64_t* __restrict__ nmask) {
    int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= total_words) return;
    int32_t r = 0, hi = n_seqs - 1;  // the sequence holding word w (word offsets ascend)
    while (r < hi) {
        const int32_t mid = (r + hi + 1) >> 1;
        if (seq_word_off[mid] <= w) r = mid;
        else hi = mid - 1;
    }
    int64_t local = w - seq_word_off[r];           // word index within the sequence
    int64_t base0 = local * 32;
    int64_t size = seq_size[r];
    const unsigned char* src = ascii + seq_ascii_off[r] + base0;
    uint64_t v = 0;
    uint32_t nbits = 0;
#pragma unroll 8
    for (int j = 0; j < 32; j++) {
        unsigned char c = (base0 + j < size) ? src[j] : 'A';
        uint64_t code = (c == 'T') ? 1 : (c == 'G') ? 2 : (c == 'C') ? 3 : 0;
        v |= code << (2 * j);
        nbits |= (uint32_t)(c == 'N') << j;
    }
    words[w] = v;  // the trailing pad word of each sequence packs to 0
    // N bitmap: word local/2 of the sequence gets bits from two packed words
    int64_t nw = seq_n_off[r] + local / 2;
    if (local % 2 == 0) {
        // lower half written by the even word; the odd word ORs its half in.
        atomicOr((unsigned long long*)&nmask[nw], (unsigned long long)nbits);
    } else {
        atomicOr((unsigned long long*)&nmask[nw], (unsigned long long)nbits << 32);
    }
}

}  // namespace npgx

namespace npgx {

void heavy_for(size_t n, int64_t work, const std::function<void(size_t)>& f) {
    static HostPool* pool = [] {
        int cap = 16;
        if (const char* e = getenv("OMP_NUM_THREADS")) cap = std::max(1, atoi(e));
        return new HostPool(std::min<int>(cap, (int)std::max(1u, std::thread::hardware_concurrency())));
    }();
    static std::mutex busy;
    std::unique_lock<std::mutex> lk(busy, std::try_to_lock);
    if (work < (1 << 20) || n < 2 || pool->size() < 2 || !lk.owns_lock()) {  // small, or the pool is in use
        for (size_t i = 0; i < n; i++) f(i);
        return;
    }
    std::exception_ptr err;
    std::mutex m;
    std::atomic<bool> failed{false};
    pool->run(n, [&](size_t i) {
        if (failed.load(std::memory_order_relaxed)) return;
        try {
            f(i);
        } catch (...) {
            std::lock_guard<std::mutex> g(m);
            if (!err) err = std::current_exception();
            failed = true;
        }
    });
    if (err) std::rethrow_exception(err);
}

// Poll the stream (a blocking hipStreamSynchronize costs tens of us of wake-up
// on every short wait of the block build).  When several host threads wait at
// once (the pair-sharded job runs a dozen block sets on one GPU) a waiter
// that has polled for a while sleeps between polls instead: a dozen threads
// spinning on hipStreamQuery took the runtime's locks and the host cores from
// the threads with work to do.
hipError_t stream_wait(hipStream_t s) {
    static std::atomic<int> waiters{0};
    waiters.fetch_add(1, std::memory_order_relaxed);
    hipError_t e;
    int polls = 0;
    while ((e = hipStreamQuery(s)) == hipErrorNotReady) {
        if (++polls > 64 && waiters.load(std::memory_order_relaxed) > 1)
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        else
            __builtin_ia32_pause();
    }
    waiters.fetch_sub(1, std::memory_order_relaxed);
    return e;
}

// ---- buffer cache behind DevBuf / PinnedBuf / PinnedArena (common.hpp)
//
// hipFree and hipHostFree synchronise the whole device and unmap; hipMalloc /
// hipHostMalloc map (and pin) again.  Pipes that build and drop whole block
// sets per step (AnchorLoopFast's consensus set, the pair job's per-pair sets)
// paid ~170 frees and a dozen pinned allocations a step for that.  Freed
// buffers are kept instead, by (kind, device, size class): a freed buffer
// first waits in `pend` (kernels or copies may still use it); the first
// allocation that would reuse one synchronises the device once, zeroes the
// pending device buffers (a fresh allocation reads as zeros) and makes them
// all reusable.  Size classes: 4 KiB, then 8 steps an octave.  At most
// 24 GiB of device and 4 GiB of pinned memory are kept; above that buffers
// are freed as before.  The cache is never torn down (no runtime calls at
// process exit).  Opt-in (NPGX_BUF_CACHE=1): the whole GPU suite passes with
// it, but its gain measured within run-to-run noise (C3 + AnchorLoopFast
// 173.8 against 180.1 ms a step, C3 and the pair job unchanged;
// gpurun_out/r05av), so the default keeps the runtime's own allocations.
namespace {
struct BufCache {
    using Key = std::tuple<int, int, size_t>;  // kind (0 device, 1 pinned host), device, class bytes
    std::mutex mu;
    std::multimap<Key, void*> ready;
    std::vector<std::pair<Key, void*>> pend;
    size_t held[2] = {0, 0};
    const bool on = getenv("NPGX_BUF_CACHE") && atoi(getenv("NPGX_BUF_CACHE")) != 0;
};
BufCache& buf_cache() {
    static BufCache* c = new BufCache;  // (leaked on purpose)
    return *c;
}
constexpr size_t BUF_CACHE_MAX[2] = {24ull << 30, 4ull << 30};

void raw_free(int kind, void* p) {
    if (kind == 0)
        (void)hipFree(p);
    else
        (void)hipHostFree(p);
}
hipError_t raw_alloc(int kind, void** p, size_t bytes) {
    return kind == 0 ? hipMalloc(p, bytes) : hipHostMalloc(p, bytes, hipHostMallocDefault);
}
// the pending buffers of device dev (-1: the pinned host buffers) become
// reusable once that device (every device, for pinned buffers, which any
// device's copies may still read) has finished its work (caller holds the lock)
void buf_flush(BufCache& c, int dev) {
    bool any = false;
    for (const auto& e : c.pend) any |= std::get<1>(e.first) == dev;
    if (!any) return;
    if (dev >= 0) {
        DeviceGuard g(dev);
        NPGX_HIP(hipDeviceSynchronize());
    } else {
        int nd = 0;
        NPGX_HIP(hipGetDeviceCount(&nd));
        for (int d = 0; d < nd; d++) {
            DeviceGuard g(d);
            NPGX_HIP(hipDeviceSynchronize());
        }
    }
    DeviceGuard g(dev >= 0 ? dev : 0);  // (the zeroing below runs on the buffers' own device)
    bool zeroed = false;
    std::vector<std::pair<BufCache::Key, void*>> keep;
    for (const auto& e : c.pend) {
        if (std::get<1>(e.first) != dev) {
            keep.push_back(e);
            continue;
        }
        if (std::get<0>(e.first) == 0) {
            NPGX_HIP(hipMemsetAsync(e.second, 0, std::get<2>(e.first), nullptr));
            zeroed = true;
        }
        c.ready.emplace(e.first, e.second);
    }
    c.pend.swap(keep);
    if (zeroed) NPGX_HIP(hipStreamSynchronize(nullptr));
}
}  // namespace

size_t buf_class(size_t bytes) {
    if (bytes <= 4096) return 4096;
    const int k = 63 - __builtin_clzll((unsigned long long)bytes);
    const size_t step = (size_t)1 << (k - 3);
    return (bytes + step - 1) / step * step;
}

void* buf_alloc(int kind, size_t bytes, size_t* got) {
    BufCache& c = buf_cache();
    const size_t cls = c.on ? buf_class(bytes) : bytes;  // (off: the exact size, as before)
    *got = cls;
    int dev = -1;  // pinned host buffers are filed under -1: any device may use them
    if (kind == 0) NPGX_HIP(hipGetDevice(&dev));
    void* p = nullptr;
    if (c.on) {
        std::lock_guard<std::mutex> lk(c.mu);
        const BufCache::Key key{kind, dev, cls};
        auto it = c.ready.find(key);
        if (it == c.ready.end()) {
            bool pending = false;
            for (const auto& e : c.pend) pending |= e.first == key;
            if (pending) {
                buf_flush(c, dev);
                it = c.ready.find(key);
            }
        }
        if (it != c.ready.end()) {
            p = it->second;
            c.ready.erase(it);
            c.held[kind] -= cls;
            return p;
        }
    }
    hipError_t e = raw_alloc(kind, &p, cls);
    if (e != hipSuccess && c.on) {  // out of memory: give the cache back to the runtime, then retry once
        (void)hipGetLastError();
        std::lock_guard<std::mutex> lk(c.mu);
        buf_flush(c, dev);
        if (kind == 0) NPGX_HIP(hipSetDevice(dev));
        for (auto it = c.ready.begin(); it != c.ready.end();) {
            if (std::get<0>(it->first) == kind && std::get<1>(it->first) == dev) {
                raw_free(kind, it->second);
                c.held[kind] -= std::get<2>(it->first);
                it = c.ready.erase(it);
            } else {
                ++it;
            }
        }
        e = raw_alloc(kind, &p, cls);
    }
    NPGX_HIP(e);
    return p;
}

void buf_free(int kind, void* p, size_t cls) {
    if (!p) return;
    BufCache& c = buf_cache();
    // filed under the device that owns the allocation, not the calling
    // thread's current device (a set freed from another device's thread)
    int dev = -1;
    bool known = kind == 1;
    if (c.on && kind == 0) {
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, p) == hipSuccess && a.device >= 0) {
            dev = a.device;
            known = true;
        } else {
            (void)hipGetLastError();
        }
    }
    if (c.on && known) {
        std::lock_guard<std::mutex> lk(c.mu);
        if (c.held[kind] + cls <= BUF_CACHE_MAX[kind]) {
            c.pend.emplace_back(BufCache::Key{kind, dev, cls}, p);
            c.held[kind] += cls;
            return;
        }
    }
    raw_free(kind, p);
}

// Rank (size desc, name asc, input index asc), layout and the packed words /
// N bitmap of s, whose sequence i (s->data[i], ATGCN only) also sits on the
// device at d_ascii + ascii[i].
void pack_device(npgx_seqset* s, const unsigned char* d_ascii, const std::vector<int64_t>& ascii) {
    const int32_t n = s->n;
    s->by_rank.resize(n);
    std::iota(s->by_rank.begin(), s->by_rank.end(), 0);
    std::sort(s->by_rank.begin(), s->by_rank.end(), [&](int32_t a, int32_t b) {
        if (s->data[a].size() != s->data[b].size()) return s->data[a].size() > s->data[b].size();
        if (s->names[a] != s->names[b]) return s->names[a] < s->names[b];
        return a < b;
    });
    s->rank_of.assign(n, 0);
    for (int32_t r = 0; r < n; r++) s->rank_of[s->by_rank[r]] = r;
    s->word_off.resize(n);
    s->n_off.resize(n);
    std::vector<int64_t> ascii_off(n), size_r(n);
    int64_t wo = 0, no = 0;
    for (int32_t r = 0; r < n; r++) {
        const int32_t i = s->by_rank[r];
        const int64_t sz = (int64_t)s->data[i].size();
        int64_t nw = (sz + 31) / 32 + 1;  // + zero pad word
        if (nw % 2) nw += 1;              // keep N-word pairing aligned
        s->word_off[r] = wo;
        s->n_off[r] = no;
        ascii_off[r] = ascii[i];
        size_r[r] = sz;
        wo += nw;
        no += nw / 2;
    }
    s->total_words = wo;
    s->total_nwords = no;
    s->words.ensure((size_t)wo);
    s->nmask.ensure((size_t)no);
    if (wo == 0) return;
    // the four per-rank tables in one upload
    std::vector<int64_t> tab(4 * (size_t)n);
    std::copy(s->word_off.begin(), s->word_off.end(), tab.begin());
    std::copy(ascii_off.begin(), ascii_off.end(), tab.begin() + n);
    std::copy(s->n_off.begin(), s->n_off.end(), tab.begin() + 2 * (size_t)n);
    std::copy(size_r.begin(), size_r.end(), tab.begin() + 3 * (size_t)n);
    DevBuf<int64_t> d_tab;
    d_tab.ensure(tab.size());
    NPGX_HIP(hipMemcpy(d_tab.p, tab.data(), tab.size() * 8, hipMemcpyHostToDevice));
    NPGX_HIP(hipMemset(s->nmask.p, 0, (size_t)no * 8));
    const int threads = 256;
    const int64_t blocks = (wo + threads - 1) / threads;
    hipLaunchKernelGGL(k_pack, dim3((unsigned)blocks), dim3(threads), 0, 0, d_ascii, d_tab.p, d_tab.p + n,
                       d_tab.p + 2 * n, d_tab.p + 3 * n, n, wo, s->words.p, s->nmask.p);
    NPGX_HIP(hipGetLastError());
    NPGX_HIP(hipDeviceSynchronize());
}

npgx_seqset* seqset_from_device(const char* host_text, const char* d_text, const std::vector<int64_t>& off,
                                const std::vector<std::string>& names) {
    const int32_t n = (int32_t)off.size() - 1;
    NPGX_REQUIRE(names.size() == (size_t)n, NPGX_ERR_ARG, "one name per sequence");
    std::unique_ptr<npgx_seqset> s(new npgx_seqset);
    s->device = current_device_checked();
    s->n = n;
    s->names = names;
    s->data.resize(n);
    heavy_for((size_t)n, off[n], [&](size_t i) { s->data[i].assign(host_text + off[i], (size_t)(off[i + 1] - off[i])); });
    pack_device(s.get(), (const unsigned char*)d_text, off);
    return s.release();
}

HostPool::HostPool(int threads) {
    for (int i = 1; i < threads; i++) workers_.emplace_back([this] { loop(); });
}

HostPool::~HostPool() {
    {
        std::lock_guard<std::mutex> g(m_);
        stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
}

void HostPool::loop() {
    uint64_t seen = 0;
    while (true) {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        const std::function<void(size_t)>* f = f_;
        const size_t n = n_;
        g.unlock();
        for (size_t i; (i = next_.fetch_add(1)) < n;) (*f)(i);
        g.lock();
        if (--active_ == 0) done_.notify_all();
    }
}

void HostPool::run(size_t n, const std::function<void(size_t)>& f) {
    if (workers_.empty() || n < 2) {
        for (size_t i = 0; i < n; i++) f(i);
        return;
    }
    {
        std::lock_guard<std::mutex> g(m_);
        f_ = &f;
        n_ = n;
        next_ = 0;
        active_ = (int)workers_.size();
        gen_++;
    }
    cv_.notify_all();
    for (size_t i; (i = next_.fetch_add(1)) < n;) f(i);
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [&] { return active_ == 0; });
}

}  // namespace npgx

using namespace npgx;

extern "C" {

const char* npgx_last_error(void) { return g_last_error.c_str(); }
const char* npgx_version(void) { return "npge_amd 0.1 (gfx950)"; }

int npgx_device_count(int32_t* n) {
    return guard([&] {
        int c = 0;
        if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
        *n = c;
    });
}

int npgx_set_device(int32_t device) {
    return guard([&] { NPGX_HIP(hipSetDevice(device)); });
}

int npgx_memcpy(void* dst, const void* src, int64_t bytes) {
    return guard([&] {
        NPGX_REQUIRE(bytes >= 0 && (bytes == 0 || (dst && src)), NPGX_ERR_ARG, "npgx_memcpy: bad arguments");
        if (bytes) NPGX_HIP(hipMemcpy(dst, src, (size_t)bytes, hipMemcpyDefault));
    });
}

int npgx_seqset_create(const char* const* seqs, const int64_t* lens, const char* const* names,
                       int32_t n, npgx_seqset** out) {
    return guard([&] {
        NPGX_REQUIRE(out && n >= 0 && (n == 0 || (seqs && lens)), NPGX_ERR_ARG,
                     "npgx_seqset_create: bad arguments");
        int dev = current_device_checked();
        std::unique_ptr<npgx_seqset> s(new npgx_seqset);
        s->device = dev;
        s->n = n;
        s->names.resize(n);
        s->data.resize(n);
        int64_t total = 0;
        for (int32_t i = 0; i < n; i++) {
            NPGX_REQUIRE(lens[i] >= 0, NPGX_ERR_ARG, "negative sequence length");
            s->names[i] = names && names[i] ? names[i] : "";
            total += lens[i];
        }
        const auto t0 = std::chrono::steady_clock::now();
        heavy_for((size_t)n, total, [&](size_t i) { s->data[i] = to_atgcn(seqs[i], lens[i]); });
        const auto t1 = std::chrono::steady_clock::now();
        s->ms_host = std::chrono::duration<double, std::milli>(t1 - t0).count();
        // the ASCII text on the device in input order (one DMA from pinned
        // staging kept across calls), then packed by k_pack
        std::vector<int64_t> ascii(n + 1, 0);
        for (int32_t i = 0; i < n; i++) ascii[i + 1] = ascii[i] + (int64_t)s->data[i].size();
        DevBuf<unsigned char> d_ascii;
        d_ascii.ensure((size_t)std::max<int64_t>(ascii[n], 1));
        // sets up to 256 MiB share one pinned staging buffer (kept, so repeated
        // creations skip the pinning; creations of such sets serialize on it);
        // larger ones pin a buffer of their own for the call, so the largest
        // set ever uploaded does not stay pinned in host memory
        static constexpr int64_t SHARED_STAGING_MAX = 256ll << 20;
        auto stage_copy = [&](char* st) {
            heavy_for((size_t)n, ascii[n], [&](size_t i) { memcpy(st + ascii[i], s->data[i].data(), s->data[i].size()); });
            NPGX_HIP(hipMemcpy(d_ascii.p, st, (size_t)ascii[n], hipMemcpyHostToDevice));
        };
        if (ascii[n] > SHARED_STAGING_MAX) {
            PinnedBuf<char> own;
            stage_copy(own.ensure((size_t)ascii[n]));
        } else if (ascii[n] > 0) {
            static std::mutex mu;
            static PinnedBuf<char> staging;
            std::lock_guard<std::mutex> lk(mu);
            stage_copy(staging.ensure((size_t)ascii[n]));
        }
        pack_device(s.get(), d_ascii.p, ascii);
        s->ms_upload = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
        *out = s.release();
    });
}

int npgx_seqset_timings(const npgx_seqset* s, double* ms_host, double* ms_upload) {
    return guard([&] {
        NPGX_REQUIRE(s && ms_host && ms_upload, NPGX_ERR_ARG, "null argument");
        *ms_host = s->ms_host;
        *ms_upload = s->ms_upload;
    });
}

int npgx_seqset_count(const npgx_seqset* s, int32_t* n) {
    return guard([&] {
        NPGX_REQUIRE(s && n, NPGX_ERR_ARG, "null argument");
        *n = s->n;
    });
}

int npgx_seqset_size(const npgx_seqset* s, int32_t index, int64_t* size) {
    return guard([&] {
        NPGX_REQUIRE(s && size && index >= 0 && index < s->n, NPGX_ERR_ARG, "bad index");
        *size = (int64_t)s->data[index].size();
    });
}

int npgx_seqset_rank(const npgx_seqset* s, int32_t index, int32_t* rank) {
    return guard([&] {
        NPGX_REQUIRE(s && rank && index >= 0 && index < s->n, NPGX_ERR_ARG, "bad index");
        *rank = s->rank_of[index];
    });
}

int npgx_seqset_text(const npgx_seqset* s, int32_t index, int64_t start, int64_t len, char* out) {
    return guard([&] {
        NPGX_REQUIRE(s && out && index >= 0 && index < s->n, NPGX_ERR_ARG, "bad index");
        const std::string& d = s->data[index];
        NPGX_REQUIRE(start >= 0 && len >= 0 && start + len <= (int64_t)d.size(), NPGX_ERR_RANGE,
                     "range outside sequence");
        memcpy(out, d.data() + start, (size_t)len);
    });
}

int npgx_seqset_device_bytes(const npgx_seqset* s, int64_t* bytes) {
    return guard([&] {
        NPGX_REQUIRE(s && bytes, NPGX_ERR_ARG, "null argument");
        *bytes = (s->total_words + s->total_nwords) * 8;
    });
}

void npgx_seqset_free(npgx_seqset* s) { delete s; }

}  // extern "C"
