// anchor_finder.hip -- MI355X-native AnchorFinder (src/algo/AnchorFinder.cpp:37-406).
//
// The reference runs two sequential rolling-hash passes per sequence: a Bloom
// "seen before" pass collecting hashes (BloomTask, :152-197) and an exact
// membership pass emitting FoundFragments (FragmentTask, :283-326), followed by a
// sort / truncate / group step (:356-391).  Its Bloom pass is order-dependent
// (a window is "found" when all k_b bits were already set by earlier windows).
// Here the same result is computed data-parallel:
//
//   k_bloom_first   first[bit] = min over admitted windows of order(window)
//                   (atomicMin; admitted = valid, hash not in the used set)
//   k_found_collect found(p) = admitted(p) && all first[bit_i(p)] < order(p)
//                   -- exactly "all bits were set by an earlier window";
//                   collected(p) = found(p) && !(similar && found(p-1));
//                   workgroup compaction of collected hashes (one atomic per WG)
//   sort + unique   H = sorted unique collected hashes (rocPRIM radix sort)
//   k_table_insert  open-addressing table hash -> index in H
//   k_ff_count      count[idx(h)]++ for every valid window whose hash is in H
//   exclusive scan  offsets; cut G = #groups starting before max-anchor-fragments
//   k_ff_scatter    windows of the first G groups -> (idx << B) | key2, where
//                   key2 = 2*order_off(rank) + pos (+size if reverse) orders by
//                   (rank, direct before reverse, pos) -- FoundFragment's order
//   radix sort      over the candidate keys, truncate, group on the host.
//
// Windows are read straight from the 2-bit packed words: the window [p, p+k) is
// bits [2p, 2p+2k) of the sequence's bit stream, which IS make_hash's value
// (make_hash.hpp:29-42, LSB = first base); the reverse hash is the 2-bit-group
// reversal of its complement (complement.cpp:24-50).
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>

#include <chrono>

#include "common.hpp"

namespace npgx {

std::string genome_of(const std::string& name);
uint64_t estimate_length(const npgx_seqset* s);
int64_t optimal_bits(uint64_t members, double error_prob);
int optimal_hashes(uint64_t members, uint64_t bits);
void glibc_rand(uint32_t seed, int n, uint64_t* out);

static constexpr int WG = 256;         // windows per workgroup (4 waves)
static constexpr int MAX_KB = 32;
static constexpr int FKB = 4;          // hash functions with the batched-load path (fp 0.1 -> 3)

struct Chunk {
    int32_t seq;
    int32_t pad;
    int64_t pos;
};

struct AfArgs {
    const SeqMeta* meta;
    const Chunk* chunks;
    const uint64_t* words;
    const uint64_t* nmask;
    const uint64_t* used;
    int64_t n_used;
    uint64_t kmask;
    uint64_t mmagic;      // floor((2^64-1)/m)
    uint32_t nbits_mask;  // (1<<k)-1 over the N bitmap
    uint32_t m;
    int32_t k;
    int32_t kb;
    int32_t similar;
    int32_t nseg;         // found_collect's output segments (see k_seg_compact)
    int64_t chunk_base;   // global index of chunks[0] (an epoch's first chunk)
    int64_t seg_cap;      // entries per output segment
    uint8_t* wmask;       // per window (chunk index * WG + thread): k_bloom_first_f's P test for
                          // k_found_collect_f (bit 7 admitted, bit i: bit i in P); null: not used
    uint64_t params[MAX_KB];
};

// membership table hash -> index in H: key and value side by side in one
// 16-byte slot, so a lookup that finds its key reads one cache line (four
// slots a 64-byte line; linear probing stays in it mostly)
struct __attribute__((aligned(16))) TableSlot {
    uint64_t key;
    uint32_t val;
    uint32_t pad;
};

struct TableArgs {
    const TableSlot* slots;
    const uint32_t* occ;  // one bit per slot: occupied (cap / 8 bytes, cache-resident)
    uint32_t mask;
    int32_t shift;
};

static constexpr uint64_t EMPTY_KEY = ~0ull;  // never a canonical hash (min(dir, rev))

// ------------------------------------------------------------------ device helpers
__device__ __forceinline__ uint64_t revcomp(uint64_t d, int k) {
    uint64_t x = d ^ 0x5555555555555555ull;  // complement_letter(x) = x ^ 1 per base
    x = __builtin_bitreverse64(x);
    x = ((x >> 1) & 0x5555555555555555ull) | ((x & 0x5555555555555555ull) << 1);
    return x >> (64 - 2 * k);
}

// Loads window p of sequence s.  Returns false for windows containing N.
__device__ __forceinline__ bool load_window(const AfArgs& a, const SeqMeta& s, int64_t p,
                                            uint64_t& dir) {
    const int64_t w = s.word_off + (p >> 5);
    const int sh = (int)(p & 31) * 2;
    const uint64_t lo = a.words[w], hi = a.words[w + 1];
    uint64_t d = sh ? ((lo >> sh) | (hi << (64 - sh))) : lo;
    dir = d & a.kmask;
    const int64_t nw = s.n_off + (p >> 6);
    const int nsh = (int)(p & 63);
    const uint64_t nlo = a.nmask[nw], nhi = a.nmask[nw + 1];
    const uint64_t nb = nsh ? ((nlo >> nsh) | (nhi << (64 - nsh))) : nlo;
    return ((uint32_t)nb & a.nbits_mask) == 0;
}

__device__ __forceinline__ uint32_t bloom_index(uint64_t x, uint32_t m, uint64_t magic) {
    // exact x % m for 64-bit x, 32-bit m: q_est in {q-1, q}
    const uint64_t q = __umul64hi(x, magic);
    uint64_t r = x - q * (uint64_t)m;
    return (uint32_t)(r >= m ? r - m : r);
}

__device__ __forceinline__ bool in_sorted(const uint64_t* v, int64_t n, uint64_t h) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (v[mid] < h) lo = mid + 1;
        else hi = mid;
    }
    return lo < n && v[lo] == h;
}

// most windows are not in H (C3: 85 %): with linear probing a key whose
// home slot is empty is absent, and the occupancy bit of the home slot comes
// from a bit array that stays in cache, so those windows never touch the
// table's lines.  (Round 6 measured two alternatives slower: a fingerprint
// byte per slot, `profiles/r06s_af_fingerprints_ab.txt`, and a second bit
// array under another hash, r06v: C5 AnchorFinder +4.5 ms.)
__device__ __forceinline__ int64_t table_find(const TableArgs& t, uint64_t h) {
    uint32_t s = (uint32_t)((h * 0x9E3779B97F4A7C15ull) >> t.shift) & t.mask;
    if (!((t.occ[s >> 5] >> (s & 31)) & 1u)) return -1;
    while (true) {
        const uint4 v = *(const uint4*)(t.slots + s);  // key and value in one 16-byte load
        const uint64_t key = ((uint64_t)v.y << 32) | v.x;
        if (key == h) return (int64_t)v.z;
        if (key == EMPTY_KEY) return -1;
        s = (s + 1) & t.mask;
    }
}

// valid && not used: the windows the reference admits to the Bloom filter
// (AnchorFinder.cpp:170-182).
__device__ __forceinline__ bool admitted(const AfArgs& a, const SeqMeta& s, int64_t p,
                                         uint64_t& h, uint64_t& dir) {
    if (p < 0 || p + a.k > s.size) return false;
    if (!load_window(a, s, p, dir)) return false;
    const uint64_t rev = revcomp(dir, a.k);
    h = dir < rev ? dir : rev;
    if (a.n_used && in_sorted(a.used, a.n_used, h)) return false;
    return true;
}

__device__ __forceinline__ bool found_at(const AfArgs& a, const SeqMeta& s, int64_t p,
                                         const uint32_t* __restrict__ first, uint64_t& h) {
    uint64_t dir;
    if (!admitted(a, s, p, h, dir)) return false;
    const uint32_t ord = (uint32_t)(s.order_off + (uint64_t)p);
    bool f = true;
    for (int i = 0; i < a.kb; i++) {
        const uint32_t idx = bloom_index(h ^ a.params[i], a.m, a.mmagic);
        f &= first[idx] < ord;
    }
    return f;
}

// ------------------------------------------------------------------ kernels
// Appends h to out for every thread with col set, one atomic on the shared
// counter per workgroup: with one per wave the counter's serialized atomics
// bounded found/collect (most waves collect a window)
__device__ __forceinline__ void wg_append(bool col, uint64_t h, uint64_t* __restrict__ out,
                                          unsigned long long* __restrict__ n_out) {
    __shared__ uint32_t wcnt[WG / 64];
    __shared__ unsigned long long wbase;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const unsigned long long mask = __ballot(col);
    if (lane == 0) wcnt[wv] = (uint32_t)__popcll(mask);
    __syncthreads();
    if (t == 0) {
        uint32_t tot = 0;
        for (int i = 0; i < WG / 64; i++) {
            const uint32_t c = wcnt[i];
            wcnt[i] = tot;
            tot += c;
        }
        wbase = tot ? atomicAdd(n_out, (unsigned long long)tot) : 0ull;
    }
    __syncthreads();
    if (col) out[wbase + wcnt[wv] + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull))] = h;
}

// ---- epoch-filtered Bloom pass (one GPU).  The windows run in epochs of
// consecutive chunks (order ascending); P is the Bloom bit array of every
// window of the earlier epochs.  A bit in P was first set in an earlier epoch,
// whose windows all atomicMin'ed it then, so first[bit] is already exact and
// below the order of any window of this epoch: such bits need neither the
// atomic nor the read of first[] -- the result equals the unfiltered pass.
__device__ __forceinline__ bool bit_in(const uint32_t* __restrict__ P, uint32_t idx) {
    return (P[idx >> 5] >> (idx & 31)) & 1u;
}

// With a.wmask (kb <= FKB) the P test of every window is kept for
// k_found_collect_f of the same epoch (P does not change in between): one
// coalesced byte per window instead of kb random P loads there again (P is
// m/8 bytes: 45 MB at C5, past the L2s, where random loads run at about 55 G/s).
__device__ __forceinline__ void bloom_first_body(const AfArgs& a, uint32_t* first, const uint32_t* P, int64_t bid) {
    const Chunk c = a.chunks[bid];
    const SeqMeta s = a.meta[c.seq];
    const int64_t p = c.pos + threadIdx.x;
    uint64_t h, dir;
    uint8_t* wm = a.wmask ? a.wmask + (a.chunk_base + bid) * WG + threadIdx.x : nullptr;
    if (!admitted(a, s, p, h, dir)) {
        if (wm) *wm = 0;
        return;
    }
    const uint32_t ord = (uint32_t)(s.order_off + (uint64_t)p);
    if (a.kb <= FKB) {
        uint32_t idx[FKB], pw[FKB];
#pragma unroll
        for (int i = 0; i < FKB; i++)
            if (i < a.kb) {
                idx[i] = bloom_index(h ^ a.params[i], a.m, a.mmagic);
                pw[i] = P[idx[i] >> 5];
            }
        uint32_t v = 0x80u;
#pragma unroll
        for (int i = 0; i < FKB; i++)
            if (i < a.kb) {
                const uint32_t in = (pw[i] >> (idx[i] & 31)) & 1u;
                v |= in << i;
                if (!in) atomicMin(&first[idx[i]], ord);
            }
        if (wm) *wm = (uint8_t)v;
        return;
    }
    for (int i = 0; i < a.kb; i++) {
        const uint32_t idx = bloom_index(h ^ a.params[i], a.m, a.mmagic);
        if (!bit_in(P, idx)) atomicMin(&first[idx], ord);
    }
}
__global__ __launch_bounds__(WG) void k_bloom_first_f(AfArgs a, uint32_t* __restrict__ first,
                                                      const uint32_t* __restrict__ P) {
    bloom_first_body(a, first, P, blockIdx.x);
}

// found/collect of one epoch, reading P (bits of the earlier epochs) and
// adding this epoch's bits to Pn (copied to P before the next epoch)
// Sharded mode (P0 != null): P0 holds the bits set by the lower ranks'
// windows and first[] the orders of this rank's own (for the bits outside
// P0), so the exact test of a window of this range uses both; the range's
// first window, whose predecessor lies on another rank, is not collected here
// but reported in bfirst[0..1] (found, hash), and the found state of the
// range's last window goes to blast[0]: the host settles the boundary after
// one small exchange.
__device__ __forceinline__ bool found_at_p(const AfArgs& a, const SeqMeta& s, int64_t p,
                                           const uint32_t* __restrict__ first, const uint32_t* __restrict__ P,
                                           uint64_t& h) {
    uint64_t dir;
    if (!admitted(a, s, p, h, dir)) return false;
    const uint32_t ord = (uint32_t)(s.order_off + (uint64_t)p);
    bool f = true;
    for (int i = 0; i < a.kb; i++) {
        const uint32_t idx = bloom_index(h ^ a.params[i], a.m, a.mmagic);
        f &= bit_in(P, idx) || first[idx] < ord;
    }
    return f;
}

__device__ __forceinline__ void found_collect_body(const AfArgs& a, const uint32_t* first, const uint32_t* P,
                                                   uint32_t* Pn,  // (may be P: the host's Pw)
                                                   uint64_t* out, unsigned long long* n_out, const uint32_t* P0,
                                                   unsigned long long* bfirst, unsigned long long* blast,
                                                   int64_t bid, int64_t nblk) {
    __shared__ uint8_t fs[WG];
    const Chunk c = a.chunks[bid];
    const SeqMeta s = a.meta[c.seq];
    const int t = threadIdx.x;
    const int64_t p = c.pos + t;
    uint64_t h = 0;
    bool f = false;
    if (a.wmask) {
        // k_bloom_first_f's admission and P test (kb <= FKB): the first[]
        // entries of the bits outside P are the only random loads left
        const uint32_t v = a.wmask[(a.chunk_base + bid) * WG + t];
        if (v & 0x80u) {
            const int64_t w = s.word_off + (p >> 5);
            const int sh = (int)(p & 31) * 2;
            const uint64_t lo = a.words[w], hi = a.words[w + 1];
            const uint64_t dir = (sh ? ((lo >> sh) | (hi << (64 - sh))) : lo) & a.kmask;
            const uint64_t rev = revcomp(dir, a.k);
            h = dir < rev ? dir : rev;
            const uint32_t ord = (uint32_t)(s.order_off + (uint64_t)p);
            f = true;
            uint32_t idx[FKB], fv[FKB];
#pragma unroll
            for (int i = 0; i < FKB; i++)
                if (i < a.kb && !((v >> i) & 1u)) {
                    idx[i] = bloom_index(h ^ a.params[i], a.m, a.mmagic);
                    fv[i] = first[idx[i]];
                }
#pragma unroll
            for (int i = 0; i < FKB; i++)
                if (i < a.kb && !((v >> i) & 1u)) {
                    f &= fv[i] < ord;
                    if (Pn && fv[i] == ord) atomicOr(&Pn[idx[i] >> 5], 1u << (idx[i] & 31));
                }
        }
    } else {
        uint64_t dir;
        if (admitted(a, s, p, h, dir)) {
            const uint32_t ord = (uint32_t)(s.order_off + (uint64_t)p);
            f = true;
            if (a.kb <= FKB) {
                // all P words, then the needed first[] entries, then the new
                // bits: independent loads issued together
                uint32_t idx[FKB], pw[FKB], fv[FKB];
#pragma unroll
                for (int i = 0; i < FKB; i++)
                    if (i < a.kb) {
                        idx[i] = bloom_index(h ^ a.params[i], a.m, a.mmagic);
                        pw[i] = P[idx[i] >> 5];
                    }
#pragma unroll
                for (int i = 0; i < FKB; i++)
                    if (i < a.kb) {
                        pw[i] = (pw[i] >> (idx[i] & 31)) & 1u;  // set by an earlier epoch
                        fv[i] = pw[i] ? 0u : first[idx[i]];
                    }
                // a bit new in this epoch goes into Pn once, by its first
                // setter (first[] holds that window's order)
#pragma unroll
                for (int i = 0; i < FKB; i++)
                    if (i < a.kb && !pw[i]) {
                        f &= fv[i] < ord;
                        if (Pn && fv[i] == ord) atomicOr(&Pn[idx[i] >> 5], 1u << (idx[i] & 31));
                    }
            } else {
                for (int i = 0; i < a.kb; i++) {
                    const uint32_t idx = bloom_index(h ^ a.params[i], a.m, a.mmagic);
                    const uint32_t bit = 1u << (idx & 31);
                    if (P[idx >> 5] & bit) continue;   // set by an earlier epoch
                    f &= first[idx] < ord;
                    if (Pn && !(Pn[idx >> 5] & bit)) atomicOr(&Pn[idx >> 5], bit);
                }
            }
        }
    }
    fs[t] = f;
    __syncthreads();
    bool prev;
    bool col;
    if (t > 0) {
        prev = fs[t - 1];
        col = f && !(a.similar && prev);
    } else if (!P0) {
        // p-1 may belong to an earlier epoch (P then holds bits set after it):
        // the exact test on first[] alone
        uint64_t hp;
        prev = found_at(a, s, p - 1, first, hp);
        col = f && !(a.similar && prev);
    } else if (bfirst && bid == 0 && p > 0) {  // the predecessor is on another rank
        bfirst[0] = f ? 1ull : 0ull;
        bfirst[1] = h;
        col = false;
    } else {
        uint64_t hp;
        prev = found_at_p(a, s, p - 1, first, P0, hp);
        col = f && !(a.similar && prev);
    }
    if (blast && bid == nblk - 1) {  // the range's last window
        const int64_t last = min((int64_t)WG, s.size - a.k + 1 - c.pos) - 1;
        if (t == last) blast[0] = f ? 1ull : 0ull;
    }
    // one of nseg output segments (by global chunk index), each with its own
    // counter on its own 128-byte line: the workgroups' append atomics spread
    // over nseg addresses instead of queueing on one (k_seg_compact packs them)
    const int64_t seg = (a.chunk_base + bid) % a.nseg;
    wg_append(col, h, out + seg * a.seg_cap, n_out + seg * 16);
}
__global__ __launch_bounds__(WG) void k_found_collect_f(AfArgs a, const uint32_t* __restrict__ first,
                                                        const uint32_t* P, uint32_t* Pn,
                                                        uint64_t* __restrict__ out,
                                                        unsigned long long* __restrict__ n_out,
                                                        const uint32_t* __restrict__ P0,
                                                        unsigned long long* __restrict__ bfirst,
                                                        unsigned long long* __restrict__ blast) {
    found_collect_body(a, first, P, Pn, out, n_out, P0, bfirst, blast, blockIdx.x, gridDim.x);
}
// One launch for epoch e's found/collect (the first nc workgroups) and epoch
// e+1's first-setter pass (the rest), with the window masks (P is only read
// by the first-setter role and only written, by first setters, in the
// other): a bit the collect role adds to P while the other role runs is
// either seen there (its first[] is already exact and below every order of
// epoch e+1) or not (the atomicMin changes nothing, and the mask sends the
// window to first[], which says the same); and the atomicMins of epoch e+1
// cannot lower an entry below the order of a window of epoch e that set it.
// Two launches an epoch become one.
__global__ __launch_bounds__(WG) void k_bloom_epoch_f(AfArgs ac, AfArgs ab, int64_t nc, uint32_t* first,
                                                      uint32_t* P, uint64_t* __restrict__ out,
                                                      unsigned long long* __restrict__ n_out,
                                                      const uint32_t* __restrict__ P0,
                                                      unsigned long long* __restrict__ bfirst) {
    if ((int64_t)blockIdx.x < nc) found_collect_body(ac, first, P, P, out, n_out, P0, bfirst, nullptr, blockIdx.x, nc);
    else bloom_first_body(ab, first, P, (int64_t)blockIdx.x - nc);
}

// the segments of found_collect's output, packed in segment order into out;
// *total = their sum.  One workgroup per segment (nseg <= 256).
__global__ __launch_bounds__(256) void k_seg_compact(const uint64_t* __restrict__ hseg,
                                                     const unsigned long long* __restrict__ ctr, int nseg,
                                                     int64_t seg_cap, uint64_t* __restrict__ out,
                                                     unsigned long long* __restrict__ total) {
    __shared__ unsigned long long part[256];
    const int j = blockIdx.x, t = threadIdx.x;
    part[t] = t < j ? ctr[t * 16] : 0ull;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (t < w) part[t] += part[t + w];
        __syncthreads();
    }
    const unsigned long long off = part[0];
    const unsigned long long n = ctr[j * 16];
    for (unsigned long long i = t; i < n; i += 256) out[off + i] = hseg[(int64_t)j * seg_cap + (int64_t)i];
    if (j == nseg - 1 && t == 0) *total = off + n;
}

// Up to 8 buffers set to a 32-bit pattern in ONE launch (the run's resets:
// first[], the bit arrays, the counters; the table's slots and counts), instead
// of one fill dispatch each.  blockIdx.y = buffer; 16-byte stores where the
// buffer is 16-byte aligned and a multiple of 4 words.
struct FillOp {
    uint32_t* p;
    int64_t n;  // 32-bit words
    uint32_t v;
};
struct FillArgs {
    FillOp op[8];
};
__global__ __launch_bounds__(256) void k_fill_multi(FillArgs f) {
    const FillOp o = f.op[blockIdx.y];
    const int64_t stride = (int64_t)gridDim.x * 256;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (((uintptr_t)o.p & 15) == 0 && (o.n & 3) == 0) {
        uint4* q = (uint4*)o.p;
        const uint4 v = make_uint4(o.v, o.v, o.v, o.v);
        for (int64_t i = t; i < o.n / 4; i += stride) q[i] = v;
    } else {
        for (int64_t i = t; i < o.n; i += stride) o.p[i] = o.v;
    }
}

struct Fills {
    FillArgs a{};
    int n = 0;
    void add(void* p, int64_t bytes, uint32_t v) {
        if (bytes <= 0) return;
        NPGX_REQUIRE(n < (int)(sizeof(a.op) / sizeof(a.op[0])), NPGX_ERR_STATE,
                     "k_fill_multi: more resets than one launch holds (launch() before adding more)");
        a.op[n++] = FillOp{(uint32_t*)p, bytes / 4, v};
    }
    void launch(hipStream_t st) {
        if (n == 0) return;
        int64_t most = 0;
        for (int i = 0; i < n; i++) most = std::max(most, a.op[i].n);
        const unsigned gx = (unsigned)std::min<int64_t>(2048, std::max<int64_t>(1, (most / 4 + 255) / 256));
        hipLaunchKernelGGL(k_fill_multi, dim3(gx, (unsigned)n), dim3(256), 0, st, a);
        n = 0;
    }
};

// this rank's Bloom bit array: the bits its admitted windows set
__global__ __launch_bounds__(WG) void k_bloom_bits(AfArgs a, uint32_t* __restrict__ bits) {
    const Chunk c = a.chunks[blockIdx.x];
    const SeqMeta s = a.meta[c.seq];
    const int64_t p = c.pos + threadIdx.x;
    uint64_t h, dir;
    if (!admitted(a, s, p, h, dir)) return;
    for (int i = 0; i < a.kb; i++) {
        const uint32_t idx = bloom_index(h ^ a.params[i], a.m, a.mmagic);
        const uint32_t bit = 1u << (idx & 31);
        if (!(bits[idx >> 5] & bit)) atomicOr(&bits[idx >> 5], bit);
    }
}

// P = OR of the bit arrays of the ranks below `rank` (gathered in rank order)
__global__ void k_prefix_or(const unsigned long long* __restrict__ g, int64_t words, int rank,
                            unsigned long long* __restrict__ P) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= words) return;
    unsigned long long v = 0;
    for (int q = 0; q < rank; q++) v |= g[(int64_t)q * words + w];
    P[w] = v;
}

__global__ void k_table_insert(const uint64_t* __restrict__ hs, int64_t n, TableSlot* slots, uint32_t* occ,
                               uint32_t mask, int shift) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t h = hs[i];
    uint32_t s = (uint32_t)((h * 0x9E3779B97F4A7C15ull) >> shift) & mask;
    while (true) {
        const unsigned long long prev =
            atomicCAS((unsigned long long*)&slots[s].key, (unsigned long long)EMPTY_KEY,
                      (unsigned long long)h);
        if (prev == EMPTY_KEY) {
            slots[s].val = (uint32_t)i;
            slots[s].pad = 0u;
            atomicOr(&occ[s >> 5], 1u << (s & 31));
            return;
        }
        s = (s + 1) & mask;
    }
}

// FoundFragment counts per hash index (atomics on counts[]).  (Round 5 tried
// the counts in the membership table's slots, the cache line the key compare
// just read: no faster at C3 / C5, profiles/r05j_af_slot_counts.txt; removed.)
__global__ __launch_bounds__(WG) void k_ff_count(AfArgs a, TableArgs t, uint32_t* __restrict__ counts) {
    const Chunk c = a.chunks[blockIdx.x];
    const SeqMeta s = a.meta[c.seq];
    const int64_t p = c.pos + threadIdx.x;
    if (p + a.k > s.size) return;
    uint64_t dir;
    if (!load_window(a, s, p, dir)) return;
    const uint64_t rev = revcomp(dir, a.k);
    const uint64_t h = dir < rev ? dir : rev;
    const int64_t idx = table_find(t, h);
    if (idx >= 0) atomicAdd(&counts[idx], 1u);
}

__global__ void k_find_cut(const uint32_t* __restrict__ offsets, const uint32_t* __restrict__ counts,
                           int64_t nH, uint64_t max_frag, uint64_t* __restrict__ out /*G, C, total*/) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint64_t total = nH ? (uint64_t)offsets[nH - 1] + counts[nH - 1] : 0;
    int64_t lo = 0, hi = nH;  // first g with offsets[g] >= max_frag
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if ((uint64_t)offsets[mid] < max_frag) lo = mid + 1;
        else hi = mid;
    }
    out[0] = (uint64_t)lo;
    out[1] = lo < nH ? (uint64_t)offsets[lo] : total;
    out[2] = total;
}

__global__ __launch_bounds__(WG) void k_ff_scatter(AfArgs a, TableArgs t, const uint64_t* __restrict__ H,
                                                   uint64_t G, const uint32_t* __restrict__ offsets,
                                                   uint32_t* __restrict__ cursor, int key_bits,
                                                   uint64_t* __restrict__ cand) {
    const Chunk c = a.chunks[blockIdx.x];
    const SeqMeta s = a.meta[c.seq];
    const int64_t p = c.pos + threadIdx.x;
    if (p + a.k > s.size) return;
    uint64_t dir;
    if (!load_window(a, s, p, dir)) return;
    const uint64_t rev = revcomp(dir, a.k);
    const uint64_t h = dir < rev ? dir : rev;
    if (h > H[G - 1]) return;  // groups beyond the cut (H is sorted)
    const int64_t idx = table_find(t, h);
    if (idx < 0) return;
    // FoundFragment pos (AnchorFinder.cpp:295-301): + size for the reverse strand;
    // a palindrome (dir == rev) counts as direct (:308).
    const uint64_t pos2 = (uint64_t)p + (h == dir ? 0ull : (uint64_t)s.size);
    const uint64_t key2 = 2ull * s.order_off + pos2;
    const uint32_t slot = offsets[idx] + atomicAdd(&cursor[idx], 1u);
    cand[slot] = ((uint64_t)idx << key_bits) | key2;
}

// uint32 <-> order-preserving int32 (x ^ 2^31), so a signed MIN collective over
// ranks is the unsigned MIN of first-setter orders (0xFFFFFFFF = "never set").
__global__ void k_flip_sign(uint32_t* __restrict__ v, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] ^= 0x80000000u;
}

// this rank's candidates in the kept groups: local offset of group G
__global__ void k_local_cut(const uint32_t* __restrict__ offsets, const uint32_t* __restrict__ counts,
                            int64_t nH, uint64_t G, uint64_t* __restrict__ out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    out[3] = G < (uint64_t)nH ? (uint64_t)offsets[G]
                              : (nH ? (uint64_t)offsets[nH - 1] + counts[nH - 1] : 0ull);
}

// ------------------------------------------------------------------ host helpers
static int bits_for(uint64_t v) {  // bits needed to represent values < v
    int b = 0;
    while (b < 64 && (v > (1ull << b))) b++;
    return b;
}

}  // namespace npgx

using namespace npgx;

struct npgx_af {
    npgx_af_options opt;
    std::vector<uint64_t> explicit_params;
    int device = 0;
    hipStream_t stream = nullptr;
    std::vector<uint64_t> used;       // sorted (AnchorFinderImpl::used_hashes_)
    bool used_dirty = true;
    DevBuf<uint64_t> d_used;
    DevBuf<SeqMeta> d_meta;
    std::vector<SeqMeta> layout_meta;  // d_meta / d_chunks hold this layout (chunks follow from it and k)
    int layout_k = 0;
    int64_t layout_n = -1;
    std::vector<Chunk> layout_chunks;  // host copy of d_chunks
    int64_t layout_c0 = -1, layout_c1 = -1, layout_local = 0;  // this rank's chunk range and its windows
    DevBuf<Chunk> d_chunks;
    DevBuf<uint32_t> first;
    DevBuf<uint32_t> bloom_bits;  // P of the epoch-filtered pass
    DevBuf<uint64_t> hraw, hsorted, huniq;
    DevBuf<uint64_t> hseg;                 // found_collect's segmented output (packed into hraw)
    DevBuf<unsigned long long> segctr;     // its per-segment counters, 16 apart
    DevBuf<uint8_t> wmask;                 // per window: bloom_first's P test for found_collect
    DevBuf<unsigned long long> counters;  // [0] = n_raw, [1] = n_unique
    DevBuf<TableSlot> tslots;
    DevBuf<uint32_t> tocc;
    DevBuf<uint32_t> counts, offsets, cursor;
    DevBuf<uint32_t> counts_local, offsets_local;  // sharded runs: this rank's windows
    DevBuf<uint64_t> gathered;                     // sharded runs: all ranks' hashes / keys
    DevBuf<uint64_t> cut;  // G, C, total
    DevBuf<uint64_t> cand, cand_sorted;
    DevBuf<unsigned char> temp;
    uint64_t* h_pinned = nullptr;  // small host staging
    PinnedBuf<uint64_t> pinned_dl;  // FoundFragment keys + H downloads
    npgx_af_stats stats{};
    bool has_result = false;
    std::vector<int64_t> r_block_start;
    std::vector<int32_t> r_seq;
    std::vector<int64_t> r_min, r_max;
    std::vector<int8_t> r_ori;
    StageTimer timer;
    std::vector<uint64_t> host_keys, host_H;
    std::vector<size_t> h_group_key;  // grouping: first key of each kept group
    // Deferred host result (af_set_defer): the sorted FoundFragment keys of
    // the last run stay on the device for a caller that builds its blocks
    // there (DraftPangenome -> the device ExtendLoopFast); the host grouping
    // (fragmenttg_postprocess, AnchorFinder.cpp:356-391) runs when a result,
    // the used-hash set or the statistics are asked for, or before the next run
    bool defer_host = false;
    bool pending = false;       // the last run's keys are not grouped on the host yet
    bool pending_used = false;  // ... nor their used hashes added (cleared by npgx_af_clear_used)
    int64_t p_keep = 0;
    uint64_t p_G = 0;
    int p_key_bits = 0, p_k = 0;
    int32_t p_R = 0;
    std::vector<SeqMeta> p_meta;
    std::vector<int32_t> p_by_rank;
    DevBuf<int32_t> d_by_rank;   // rank -> input index (the device's key -> fragment conversion)

    void ensure_temp(size_t bytes) { temp.ensure(bytes); }
};

namespace npgx {

// Sequence.cpp:193-202
std::string genome_of(const std::string& name) {
    std::vector<std::string> parts;
    size_t start = 0;
    while (true) {
        size_t p = name.find('&', start);
        if (p == std::string::npos) {
            parts.push_back(name.substr(start));
            break;
        }
        parts.push_back(name.substr(start, p - start));
        start = p + 1;
    }
    if (parts.size() == 3 && (parts[2] == "c" || parts[2] == "l")) return parts[0];
    return "";
}

// AnchorFinder.cpp:81-97 (over ALL sequences of the block set)
uint64_t estimate_length(const npgx_seqset* s) {
    std::map<std::string, uint64_t> gtl;
    uint64_t max_length = 0;
    for (int32_t i = 0; i < s->n; i++) {
        uint64_t& g = gtl[genome_of(s->names[i])];
        g += s->data[i].size();
        max_length = std::max(max_length, g);
    }
    if (gtl.size() == 1) return max_length;  // consensuses
    return max_length / 2 * 3;
}

static const double LN2 = 0.69314718055994530942;

// BloomFilter.cpp:147-156 -- the reference stores the result in an int; sizes
// that would overflow it are rejected instead of reproducing the UB.
int64_t optimal_bits(uint64_t members, double error_prob) {
    double v = double(members) * (-std::log(error_prob) / (LN2 * LN2)) + 0.5;
    if (!(v < 2147483647.0)) return -1;
    int r = (int)v;
    if (r % 2 == 0) r += 1;
    if (r < 1) r = 1;
    return r;
}

// BloomFilter.cpp:158-164
int optimal_hashes(uint64_t members, uint64_t bits) {
    if (members == 0) return 1;  // +inf -> INT_MIN on x86 -> clamped to 1
    int r = (int)std::round(LN2 * double(bits) / double(members));
    if (r < 1) r = 1;
    return r;
}

// glibc TYPE_3 random(): r[i] = r[i-31] + r[i-3], output r[i+344] >> 1
void glibc_rand(uint32_t seed, int n, uint64_t* out) {
    std::vector<uint32_t> r(34 + 310 + (size_t)n);
    int32_t s0 = (int32_t)seed;
    if (s0 == 0) s0 = 1;
    r[0] = (uint32_t)s0;
    for (int i = 1; i < 31; i++) {
        int64_t v = (16807ll * (int32_t)r[i - 1]) % 2147483647ll;
        if (v < 0) v += 2147483647ll;
        r[i] = (uint32_t)v;
    }
    for (int i = 31; i < 34; i++) r[i] = r[i - 31];
    for (size_t i = 34; i < r.size(); i++) r[i] = r[i - 31] + r[i - 3];
    for (int i = 0; i < n; i++) out[i] = (uint64_t)(r[344 + (size_t)i] >> 1);
}

static void comm_check(int rc, const char* what) {
    if (rc != 0) throw Error(NPGX_ERR_ARG, std::string("collective callback failed: ") + what);
}

static void af_group_host(npgx_af* af, const std::vector<uint64_t>& keys, const std::vector<uint64_t>& Hh,
                          int key_bits, int32_t R, const SeqMeta* meta, const int32_t* by_rank, int k,
                          bool add_used);
static void af_materialize(npgx_af* af);

static void af_run(npgx_af* af, const npgx_seqset* ss, const npgx_comm* comm) {
    static const bool hdbg = getenv("NPGX_AF_DEBUG") != nullptr;  // host phase times to stderr
    const auto th0 = std::chrono::steady_clock::now();
    auto hms = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th0).count(); };
    double h_prep = 0, h_dl = 0;
    NPGX_REQUIRE(ss->device == af->device, NPGX_ERR_ARG, "sequence set and finder on different devices");
    NPGX_HIP(hipSetDevice(af->device));
    hipStream_t st = af->stream;
    const int k = af->opt.anchor_size;
    af_materialize(af);  // (the used set the last run added to)
    af->timer.reset();
    af->has_result = false;
    npgx_af_stats& S = af->stats;
    memset(&S, 0, sizeof(S));

    // --- Bloom sizing (BloomTG::initialize_bloom AnchorFinder.cpp:120-131)
    uint64_t members = estimate_length(ss);
    if (k * 2 < 64) members = std::min<uint64_t>(members, 1ull << (2 * k));
    const double fp = double(af->opt.anchor_fp_x1e4) / 10000.0;  // Decimal::to_d
    const int64_t m = optimal_bits(members, fp);
    NPGX_REQUIRE(m > 0, NPGX_ERR_RANGE, "Bloom filter size overflows the reference's int");
    const int kb = optimal_hashes(members, (uint64_t)m);
    NPGX_REQUIRE(kb <= MAX_KB, NPGX_ERR_RANGE, "too many Bloom hash functions");
    AfArgs A;
    memset(&A, 0, sizeof(A));
    if (!af->explicit_params.empty()) {
        NPGX_REQUIRE((int)af->explicit_params.size() >= kb, NPGX_ERR_ARG,
                     "explicit Bloom parameter vector shorter than the hash count");
        for (int i = 0; i < kb; i++) A.params[i] = af->explicit_params[i];
    } else {
        glibc_rand(af->opt.bloom_seed, kb, A.params);
    }
    S.members = (int64_t)members;
    S.bloom_bits = m;
    S.bloom_hashes = kb;
    for (int i = 0; i < kb; i++) S.bloom_params[i] = A.params[i];

    // --- eligible sequences (size >= k) are a prefix of the rank order
    int32_t R = 0;
    while (R < ss->n && (int64_t)ss->data[ss->by_rank[R]].size() >= k) R++;
    std::vector<SeqMeta> meta(R > 0 ? R : 1);
    uint64_t order = 0;
    int64_t n_windows = 0;
    for (int32_t r = 0; r < R; r++) {
        const int64_t size = (int64_t)ss->data[ss->by_rank[r]].size();
        meta[r] = SeqMeta{size, ss->word_off[r], ss->n_off[r], order};
        order += (uint64_t)size;
        n_windows += size - k + 1;
    }
    // the window layout depends only on the sequence set and k: built and
    // uploaded once per (set, k) and reused by later runs of this handle
    const bool same_layout = af->layout_k == k && af->layout_meta.size() == meta.size() &&
                             memcmp(af->layout_meta.data(), meta.data(), meta.size() * sizeof(SeqMeta)) == 0;
    std::vector<Chunk>& chunks = af->layout_chunks;
    if (!same_layout) {
        chunks.clear();
        for (int32_t r = 0; r < R; r++)
            for (int64_t p = 0; p < meta[r].size - k + 1; p += WG) chunks.push_back(Chunk{r, 0, p});
    }
    // window orders are 32-bit (first[] holds one per Bloom bit): a run over
    // more bases is refused, never wrapped.  NPGX_AF_MAX_BASES lowers the
    // limit (tests exercise the refusal without a 4 Gbp input).
    static const uint64_t max_bases = [] {
        const char* e = getenv("NPGX_AF_MAX_BASES");
        const uint64_t v = e ? strtoull(e, nullptr, 10) : 0;
        return v > 0 && v < 0xFFFFFFFEull ? v : 0xFFFFFFFEull;
    }();
    NPGX_REQUIRE(order < max_bases, NPGX_ERR_RANGE, "more than 2^32-2 bases in one run (32-bit window orders)");
    S.n_windows = n_windows;
    S.n_used = (int64_t)af->used.size();

    // persistent used hashes on the device
    if (af->used_dirty) {
        af->d_used.ensure(af->used.size());
        if (!af->used.empty())
            NPGX_HIP(hipMemcpyAsync(af->d_used.p, af->used.data(), af->used.size() * 8,
                                    hipMemcpyHostToDevice, st));
        af->used_dirty = false;
    }
    const int64_t nchunks_all = (int64_t)chunks.size();
    // sharded run: this rank scans the contiguous chunk range [c0, c1)
    const int world = comm ? comm->world : 1;
    const int rank = comm ? comm->rank : 0;
    const int64_t c0 = nchunks_all * rank / world, c1 = nchunks_all * (rank + 1) / world;
    const int64_t nchunks = c1 - c0;
    if (comm) NPGX_REQUIRE(n_windows < (1ll << 31), NPGX_ERR_RANGE,
                           "sharded run: FoundFragment counts must fit int32");
    if (!same_layout || af->layout_c0 != c0 || af->layout_c1 != c1) {
        int64_t lw = 0;
        for (int64_t c = c0; c < c1; c++) lw += std::min<int64_t>(WG, meta[chunks[c].seq].size - k + 1 - chunks[c].pos);
        af->layout_local = lw;
        af->layout_c0 = c0;
        af->layout_c1 = c1;
    }
    const int64_t local_windows = af->layout_local;
    if (nchunks_all == 0) {
        af->r_block_start.assign(1, 0);
        af->r_seq.clear();
        af->r_min.clear();
        af->r_max.clear();
        af->r_ori.clear();
        af->has_result = true;
        return;
    }
    if (!same_layout) {
        af->d_meta.ensure(meta.size());
        af->d_chunks.ensure(chunks.size());
        NPGX_HIP(hipMemcpyAsync(af->d_meta.p, meta.data(), meta.size() * sizeof(SeqMeta),
                                hipMemcpyHostToDevice, st));
        NPGX_HIP(hipMemcpyAsync(af->d_chunks.p, chunks.data(), chunks.size() * sizeof(Chunk),
                                hipMemcpyHostToDevice, st));
        NPGX_HIP(stream_wait(st));  // the host vectors are pageable and local
        af->layout_meta = meta;
        af->layout_k = k;
        af->layout_n = (int64_t)chunks.size();
    }

    A.meta = af->d_meta.p;
    A.chunks = af->d_chunks.p + c0;
    A.words = ss->words.p;
    A.nmask = ss->nmask.p;
    A.used = af->d_used.p;
    A.n_used = (int64_t)af->used.size();
    A.k = k;
    A.kb = kb;
    A.kmask = (k == 32) ? ~0ull : ((1ull << (2 * k)) - 1);
    A.nbits_mask = (k == 32) ? 0xFFFFFFFFu : ((1u << k) - 1);
    A.m = (uint32_t)m;
    A.mmagic = ~0ull / (uint64_t)m;
    A.similar = af->opt.anchor_similar ? 1 : 0;

    const dim3 grid((unsigned)std::max<int64_t>(nchunks, 1)), block(WG);
    h_prep = hms();
    const bool run_local = nchunks > 0;  // ranks without windows still join every collective
    uint64_t* hp = af->h_pinned;

    // --- pass 1: Bloom first-setter + found/collect
    af->first.ensure((size_t)m);
    af->counters.ensure(8);  // [0] collected, [1] unique, [4..6] sharded boundary
    Fills fills;  // the run's resets, one launch (k_fill_multi)
    fills.add(af->counters.p, 4 * sizeof(unsigned long long), 0u);
    af->hraw.ensure((size_t)local_windows + 1);
    // found_collect appends into nseg segments (global chunk index mod nseg),
    // each with room for all windows of its chunks
    A.nseg = (int32_t)std::max<int64_t>(1, std::min<int64_t>(256, nchunks));
    A.seg_cap = (nchunks + A.nseg - 1) / A.nseg * WG;
    A.chunk_base = 0;
    af->hseg.ensure((size_t)(A.nseg * A.seg_cap));
    af->segctr.ensure((size_t)A.nseg * 16);
    fills.add(af->segctr.p, (int64_t)A.nseg * 16 * 8, 0u);
    if (kb <= FKB && nchunks > 0) {  // every byte is written by k_bloom_first_f before it is read
        af->wmask.ensure((size_t)nchunks * WG);
        A.wmask = af->wmask.p;
    }
    size_t ti = 0;
    // bit arrays (uint32 words, W each): P (bits set before this epoch) | Pn
    // (through this one) | this rank's bits | P0 (the lower ranks' bits)
    const int64_t w64 = ((int64_t)m + 63) / 64, W = 2 * w64;
    af->bloom_bits.ensure((size_t)(4 * W));
    uint32_t* P = af->bloom_bits.p;
    uint32_t* Pn = P + W;
    uint32_t* mine = P + 2 * W;
    uint32_t* P0 = nullptr;
    unsigned long long* bfirst = comm ? af->counters.p + 4 : nullptr;
    unsigned long long* blast = comm ? af->counters.p + 6 : nullptr;
    ti = af->timer.begin("bloom_first", st, local_windows * (0.375 + 8.0 * kb), local_windows);
    fills.add(af->first.p, m * 4, 0xFFFFFFFFu);
    if (comm) {
        fills.add(af->counters.p + 4, 3 * 8, 0u);
        fills.add(mine, W * 4, 0u);
    } else {
        fills.add(P, 2 * W * 4, 0u);
    }
    fills.launch(st);
    NPGX_HIP(hipGetLastError());
    af->timer.end(ti, st);
    if (comm) {
        // exchange 1: every rank's Bloom bit array (m / 8 bytes); this rank
        // keeps the OR of the lower ranks' (P0), whose windows all precede
        // its own: a window here is found iff each of its bits is in P0 or was
        // set by an earlier window of this rank (first[] over the bits outside
        // P0) -- the reference's sequential test exactly.  P and Pn start at P0.
        P0 = P + 3 * W;
        ti = af->timer.begin("bloom_bits_exchange", st, (double)m / 8 * world, m);
        if (run_local) hipLaunchKernelGGL(k_bloom_bits, grid, block, 0, st, A, mine);
        NPGX_HIP(hipGetLastError());
        std::vector<int64_t> cnt(world, w64);
        af->gathered.grow((size_t)(w64 * world));
        NPGX_HIP(stream_wait(st));
        comm_check(comm->allgatherv_u64(comm->user, (const uint64_t*)mine, cnt.data(), af->gathered.p),
                   "allgatherv(Bloom bits)");
        hipLaunchKernelGGL(k_prefix_or, dim3((unsigned)((w64 + 255) / 256)), dim3(256), 0, st,
                           (const unsigned long long*)af->gathered.p, w64, rank, (unsigned long long*)P0);
        NPGX_HIP(hipGetLastError());
        NPGX_HIP(hipMemcpyAsync(P, P0, (size_t)W * 4, hipMemcpyDeviceToDevice, st));
        NPGX_HIP(hipMemcpyAsync(Pn, P0, (size_t)W * 4, hipMemcpyDeviceToDevice, st));
        af->timer.end(ti, st);
    }
    if (af->opt.bloom_epochs != 1 && run_local) {
        // epochs of consecutive chunks (SeqMeta order); bits set by earlier
        // epochs (or lower ranks) skip the atomics and the first[] reads.
        // Automatic count: one epoch per 2 M windows, at most 24 (each epoch
        // costs two launches and a copy of the m/8-byte bit array; past ~20
        // epochs the filtering gains nothing more: C5 sweep)
        const int auto_epochs = (int)std::min<int64_t>(24, std::max<int64_t>(1, local_windows / (2 << 20)));
        // With the window masks (kb <= FKB) k_found_collect_f never reads P
        // and only a bit's first setter adds it: the epoch's new bits go
        // straight into P (a reader of P in the same launch would need the
        // bits of the earlier epochs only, but there is none), and the copy
        // of the m/8-byte array after each epoch goes (C3: 24 x 5 us)
        uint32_t* Pw = A.wmask ? P : Pn;
        const int64_t per = std::max<int64_t>(
            1, (int64_t)std::ceil(double(nchunks) / std::max(1, af->opt.bloom_epochs > 0 ? af->opt.bloom_epochs
                                                                                          : auto_epochs)));
        static const bool fuse_env = !(getenv("NPGX_AF_EPOCH_FUSE") && getenv("NPGX_AF_EPOCH_FUSE")[0] == '0');
        const bool fuse = fuse_env && Pw == P && af->timer.level < 2;  // (NPGX_TIMERS=2 times each pass)
        auto epoch_args = [&](int64_t e0) {
            AfArgs E = A;
            E.chunks = A.chunks + e0;
            E.chunk_base = e0;
            return E;
        };
        if (fuse) {  // k_bloom_epoch_f: collect of epoch e with the first-setter pass of e + 1
            hipLaunchKernelGGL(k_bloom_first_f, dim3((unsigned)std::min(per, nchunks)), block, 0, st, epoch_args(0),
                               af->first.p, P);
            for (int64_t e0 = 0; e0 < nchunks; e0 += per) {
                const int64_t ne = std::min(per, nchunks - e0), e1 = e0 + ne;
                if (e1 < nchunks) {
                    const int64_t nn = std::min(per, nchunks - e1);
                    hipLaunchKernelGGL(k_bloom_epoch_f, dim3((unsigned)(ne + nn)), block, 0, st, epoch_args(e0),
                                       epoch_args(e1), ne, af->first.p, P, af->hseg.p, af->segctr.p, P0,
                                       e0 == 0 ? bfirst : nullptr);
                } else {
                    hipLaunchKernelGGL(k_found_collect_f, dim3((unsigned)ne), block, 0, st, epoch_args(e0), af->first.p,
                                       P, nullptr, af->hseg.p, af->segctr.p, P0, e0 == 0 ? bfirst : nullptr, blast);
                }
                NPGX_HIP(hipGetLastError());
            }
        }
        for (int64_t e0 = 0; e0 < nchunks && !fuse; e0 += per) {
            const int64_t ne = std::min(per, nchunks - e0);
            const AfArgs E = epoch_args(e0);
            const dim3 eg((unsigned)ne);
            ti = af->timer.begin("bloom_first", st, 0.0, 0);
            hipLaunchKernelGGL(k_bloom_first_f, eg, block, 0, st, E, af->first.p, P);
            NPGX_HIP(hipGetLastError());
            af->timer.end(ti, st);
            ti = af->timer.begin("found_collect", st, local_windows * (0.375 + 4.0 * kb) * double(ne) / nchunks, 0);
            const bool more = e0 + ne < nchunks;
            hipLaunchKernelGGL(k_found_collect_f, eg, block, 0, st, E, af->first.p, P, more ? Pw : nullptr,
                               af->hseg.p, af->segctr.p, P0, e0 == 0 ? bfirst : nullptr,
                               more ? nullptr : blast);
            NPGX_HIP(hipGetLastError());
            af->timer.end(ti, st);
            if (more && Pw != P) NPGX_HIP(hipMemcpyAsync(P, Pn, (size_t)W * 4, hipMemcpyDeviceToDevice, st));
        }
    } else if (run_local) {
        ti = af->timer.begin("bloom_first", st, 0.0, 0);
        hipLaunchKernelGGL(k_bloom_first_f, grid, block, 0, st, A, af->first.p, P);
        NPGX_HIP(hipGetLastError());
        af->timer.end(ti, st);
        ti = af->timer.begin("found_collect", st, local_windows * (0.375 + 4.0 * kb), local_windows);
        hipLaunchKernelGGL(k_found_collect_f, grid, block, 0, st, A, af->first.p, P, nullptr, af->hseg.p,
                           af->segctr.p, P0, bfirst, blast);
        NPGX_HIP(hipGetLastError());
        af->timer.end(ti, st);
    }
    if (run_local) {  // the collected hashes packed into hraw, their count into counters[0]
        ti = af->timer.begin("collect_pack", st, 0.0, 0);
        hipLaunchKernelGGL(k_seg_compact, dim3((unsigned)A.nseg), dim3(256), 0, st, af->hseg.p, af->segctr.p,
                           A.nseg, A.seg_cap, af->hraw.p, af->counters.p);
        NPGX_HIP(hipGetLastError());
        af->timer.end(ti, st);
    }
    if (comm) {
        NPGX_HIP(hipMemcpyAsync(hp, af->counters.p, 8 * 8, hipMemcpyDeviceToHost, st));
        NPGX_HIP(stream_wait(st));
        // exchange 2: every rank's last window (order, found): the similar
        // rule (AnchorFinder.cpp:185-192) for this range's first window
        int64_t mine_last = -1;
        uint64_t first_order = 0;
        bool pred_elsewhere = false;
        if (run_local) {
            const Chunk& cf = chunks[c0];
            const Chunk& cl = chunks[c1 - 1];
            const int64_t last_p = std::min<int64_t>(WG, meta[cl.seq].size - k + 1 - cl.pos) - 1 + cl.pos;
            mine_last = (int64_t)(((meta[cl.seq].order_off + (uint64_t)last_p) << 1) | (hp[6] & 1ull));
            first_order = meta[cf.seq].order_off + (uint64_t)cf.pos;
            pred_elsewhere = cf.pos > 0;
        }
        std::vector<int64_t> lasts(world);
        comm_check(comm->allgather_i64(comm->user, mine_last, lasts.data()), "allgather(boundary windows)");
        if (pred_elsewhere && (hp[4] & 1ull)) {
            bool prev = false, seen = false;
            for (int q = 0; q < world; q++)
                if (lasts[q] >= 0 && (uint64_t)(lasts[q] >> 1) + 1 == first_order) {
                    prev = (lasts[q] & 1) != 0;
                    seen = true;
                }
            NPGX_REQUIRE(seen, NPGX_ERR_STATE, "sharded run: the boundary window's rank is missing");
            if (!(af->opt.anchor_similar && prev)) {  // collected after all: appended
                const uint64_t h0 = hp[5];
                const uint64_t n1 = hp[0] + 1;
                NPGX_HIP(hipMemcpyAsync(af->hraw.p + hp[0], &h0, 8, hipMemcpyHostToDevice, st));
                NPGX_HIP(hipMemcpyAsync(af->counters.p, &n1, 8, hipMemcpyHostToDevice, st));
                NPGX_HIP(stream_wait(st));
            }
        }
    }
    NPGX_HIP(hipMemcpyAsync(hp, af->counters.p, 8, hipMemcpyDeviceToHost, st));
    NPGX_HIP(stream_wait(st));
    const int64_t n_raw = (int64_t)hp[0];
    S.n_collected_raw = n_raw;

    // --- bloomtg_postprocess (AnchorFinder.cpp:213-218): sort + unique
    const unsigned h_end_bit = (unsigned)std::min(64, 2 * k);
    auto sort_unique = [&](const uint64_t* in, int64_t n) -> int64_t {
        if (n <= 0) return 0;
        af->hsorted.ensure((size_t)n);
        af->huniq.ensure((size_t)n);
        size_t b1 = 0, b2 = 0;
        NPGX_HIP(rocprim::radix_sort_keys(nullptr, b1, in, af->hsorted.p, (size_t)n, 0u, h_end_bit, st));
        NPGX_HIP(rocprim::unique(nullptr, b2, af->hsorted.p, af->huniq.p, af->counters.p + 1,
                                 (size_t)n, rocprim::equal_to<uint64_t>(), st));
        af->ensure_temp(std::max(b1, b2));
        size_t t = af->timer.begin("sort_unique_H", st, n * 8.0 * 4, n);
        NPGX_HIP(rocprim::radix_sort_keys(af->temp.p, b1, in, af->hsorted.p, (size_t)n, 0u, h_end_bit, st));
        NPGX_HIP(rocprim::unique(af->temp.p, b2, af->hsorted.p, af->huniq.p, af->counters.p + 1,
                                 (size_t)n, rocprim::equal_to<uint64_t>(), st));
        af->timer.end(t, st);
        NPGX_HIP(hipMemcpyAsync(hp, af->counters.p + 1, 8, hipMemcpyDeviceToHost, st));
        NPGX_HIP(stream_wait(st));
        return (int64_t)hp[0];
    };
    std::vector<int64_t> rc(world);
    // all-gather of this rank's n values from `src` into af->gathered; returns the total
    auto gather_u64 = [&](const uint64_t* src, int64_t n, const char* what) -> int64_t {
        comm_check(comm->allgather_i64(comm->user, n, rc.data()), what);
        int64_t tot = 0;
        for (int64_t v : rc) tot += v;
        af->gathered.grow((size_t)std::max<int64_t>(tot, 1));
        NPGX_HIP(stream_wait(st));
        if (tot > 0) comm_check(comm->allgatherv_u64(comm->user, src, rc.data(), af->gathered.p), what);
        return tot;
    };
    int64_t nH = sort_unique(af->hraw.p, n_raw);
    if (comm) {
        // exchange 2: every rank's unique collected hashes -> the global H
        const int64_t tot = gather_u64(af->huniq.p, nH, "allgatherv(collected hashes)");
        nH = sort_unique(af->gathered.p, tot);
    }
    S.n_collected = nH;

    std::vector<uint64_t>& keys = af->host_keys;
    std::vector<uint64_t>& Hh = af->host_H;
    keys.clear();
    Hh.clear();
    uint64_t G = 0;
    int key_bits = bits_for(2ull * order);
    if (nH > 0) {
        // --- membership table
        uint64_t cap = 1024;
        // at least 4 slots per hash (NPGX_AF_TABLE_SLOTS overrides): a
        // non-member window reads a slot line only when its home slot is
        // taken -- C3 ff_count 0.82 -> 0.63 ms from 2 to 4 slots, C5
        // 6.9 -> 6.1 ms (`profiles/r03y_table_slots.txt`)
        static const uint64_t spf = getenv("NPGX_AF_TABLE_SLOTS") ? std::max(2, atoi(getenv("NPGX_AF_TABLE_SLOTS"))) : 4;
        while (cap < spf * (uint64_t)nH) cap <<= 1;
        NPGX_REQUIRE(cap <= (1ull << 31), NPGX_ERR_RANGE, "hash set too large");
        int log2cap = 0;
        while ((1ull << log2cap) < cap) log2cap++;
        af->tslots.ensure(cap);
        af->tocc.ensure((size_t)(cap + 31) / 32);
        TableArgs T{af->tslots.p, af->tocc.p, (uint32_t)(cap - 1), 64 - log2cap};
        ti = af->timer.begin("table_insert", st, nH * 8.0 + nH * 12.0, nH);
        af->counts.ensure((size_t)nH);
        af->offsets.ensure((size_t)nH);
        af->cursor.ensure((size_t)nH);
        fills.add(af->tslots.p, (int64_t)(cap * sizeof(TableSlot)), 0xFFFFFFFFu);
        fills.add(af->tocc.p, (int64_t)(cap + 31) / 32 * 4, 0u);
        fills.add(af->counts.p, nH * 4, 0u);
        fills.add(af->cursor.p, nH * 4, 0u);
        fills.launch(st);
        NPGX_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_table_insert, dim3((unsigned)((nH + 255) / 256)), dim3(256), 0, st,
                           af->huniq.p, nH, af->tslots.p, af->tocc.p, (uint32_t)(cap - 1),
                           64 - log2cap);
        NPGX_HIP(hipGetLastError());
        af->timer.end(ti, st);

        // --- pass 2a: FoundFragment counts per hash
        ti = af->timer.begin("ff_count", st, local_windows * (0.375 + 12.0), local_windows);
        if (run_local) hipLaunchKernelGGL(k_ff_count, grid, block, 0, st, A, T, af->counts.p);
        NPGX_HIP(hipGetLastError());
        af->timer.end(ti, st);
        if (comm) {
            // exchange 3: global FoundFragment count per hash; keep this rank's own
            af->counts_local.ensure((size_t)nH);
            af->offsets_local.ensure((size_t)nH);
            NPGX_HIP(hipMemcpyAsync(af->counts_local.p, af->counts.p, (size_t)nH * 4,
                                    hipMemcpyDeviceToDevice, st));
            NPGX_HIP(stream_wait(st));
            comm_check(comm->allreduce_i32(comm->user, (int32_t*)af->counts.p, nH, NPGX_OP_SUM),
                       "allreduce(counts, SUM)");
        }
        size_t b3 = 0;
        NPGX_HIP(rocprim::exclusive_scan(nullptr, b3, af->counts.p, af->offsets.p, 0u, (size_t)nH,
                                         rocprim::plus<uint32_t>(), st));
        af->ensure_temp(b3);
        ti = af->timer.begin("scan_cut", st, nH * 8.0, nH);
        NPGX_HIP(rocprim::exclusive_scan(af->temp.p, b3, af->counts.p, af->offsets.p, 0u,
                                         (size_t)nH, rocprim::plus<uint32_t>(), st));
        af->cut.ensure(4);
        hipLaunchKernelGGL(k_find_cut, dim3(1), dim3(64), 0, st, af->offsets.p, af->counts.p, nH,
                           (uint64_t)af->opt.max_anchor_fragments, af->cut.p);
        NPGX_HIP(hipGetLastError());
        af->timer.end(ti, st);
        NPGX_HIP(hipMemcpyAsync(hp, af->cut.p, 3 * 8, hipMemcpyDeviceToHost, st));
        NPGX_HIP(stream_wait(st));
        G = hp[0];
        const uint64_t C = hp[1];
        S.n_found_frags = (int64_t)hp[2];
        S.n_kept_groups = (int64_t)G;
        if (G > 0 && C > 0) {
            const int idx_bits = bits_for(G);
            NPGX_REQUIRE(idx_bits + key_bits <= 64, NPGX_ERR_RANGE,
                         "FoundFragment sort key does not fit 64 bits");
            // sharded: this rank scatters its own windows by its own offsets
            uint64_t C_local = C;
            const uint32_t* scatter_off = af->offsets.p;
            if (comm) {
                NPGX_HIP(rocprim::exclusive_scan(af->temp.p, b3, af->counts_local.p, af->offsets_local.p,
                                                 0u, (size_t)nH, rocprim::plus<uint32_t>(), st));
                hipLaunchKernelGGL(k_local_cut, dim3(1), dim3(64), 0, st, af->offsets_local.p,
                                   af->counts_local.p, nH, G, af->cut.p);
                NPGX_HIP(hipGetLastError());
                NPGX_HIP(hipMemcpyAsync(hp, af->cut.p + 3, 8, hipMemcpyDeviceToHost, st));
                NPGX_HIP(stream_wait(st));
                C_local = hp[0];
                scatter_off = af->offsets_local.p;
            }
            af->cand.ensure(std::max<uint64_t>(C_local, 1));
            af->cand_sorted.ensure(C);
            ti = af->timer.begin("ff_scatter", st, local_windows * 0.375 + C_local * 24.0, local_windows);
            if (run_local && C_local > 0)
                hipLaunchKernelGGL(k_ff_scatter, grid, block, 0, st, A, T, af->huniq.p, G, scatter_off,
                                   af->cursor.p, key_bits, af->cand.p);
            NPGX_HIP(hipGetLastError());
            af->timer.end(ti, st);
            const uint64_t* sort_in = af->cand.p;
            if (comm) {
                // exchange 4: all ranks' FoundFragment keys of the kept groups
                const int64_t tot = gather_u64(af->cand.p, (int64_t)C_local, "allgatherv(FoundFragments)");
                NPGX_REQUIRE((uint64_t)tot == C, NPGX_ERR_STATE, "sharded FoundFragment count mismatch");
                sort_in = af->gathered.p;
            }
            size_t b4 = 0;
            const unsigned end_bit = (unsigned)(idx_bits + key_bits);
            NPGX_HIP(rocprim::radix_sort_keys(nullptr, b4, sort_in, af->cand_sorted.p, (size_t)C, 0u,
                                              end_bit, st));
            af->ensure_temp(b4);
            ti = af->timer.begin("ff_sort", st, C * 32.0, (int64_t)C);
            NPGX_HIP(rocprim::radix_sort_keys(af->temp.p, b4, sort_in, af->cand_sorted.p, (size_t)C,
                                              0u, end_bit, st));
            af->timer.end(ti, st);
            const uint64_t keep = std::min<uint64_t>(C, (uint64_t)af->opt.max_anchor_fragments);
            if (af->defer_host && !comm && keep > 0) {  // the keys stay on the device (af_device_keys)
                af->pending = true;
                af->pending_used = true;
                af->p_keep = (int64_t)keep;
                af->p_G = G;
                af->p_key_bits = key_bits;
                af->p_k = k;
                af->p_R = R;
                af->p_meta.assign(meta.begin(), meta.begin() + R);
                af->p_by_rank.assign(ss->by_rank.begin(), ss->by_rank.begin() + R);
                af->d_by_rank.ensure((size_t)std::max<int32_t>(R, 1));
                int32_t* hb = (int32_t*)af->pinned_dl.ensure((size_t)R / 2 + 2);
                memcpy(hb, af->p_by_rank.data(), (size_t)R * 4);
                NPGX_HIP(hipMemcpyAsync(af->d_by_rank.p, hb, (size_t)R * 4, hipMemcpyHostToDevice, st));
                NPGX_HIP(stream_wait(st));
                S.n_blocks = S.n_fragments = -1;  // (af_materialize)
                af->has_result = true;
                return;
            }
            keys.resize(keep);
            Hh.resize(G);
            af->pinned_dl.ensure((keep + G) * 8);
            uint64_t* pk = af->pinned_dl.p;
            NPGX_HIP(hipMemcpyAsync(pk, af->cand_sorted.p, keep * 8, hipMemcpyDeviceToHost, st));
            NPGX_HIP(hipMemcpyAsync(pk + keep, af->huniq.p, G * 8, hipMemcpyDeviceToHost, st));
            NPGX_HIP(stream_wait(st));
            memcpy(keys.data(), pk, keep * 8);
            memcpy(Hh.data(), pk + keep, G * 8);
        }
    }

    h_dl = hms();
    af_group_host(af, keys, Hh, key_bits, R, meta.data(), ss->by_rank.data(), k, true);
    if (hdbg)
        fprintf(stderr, "af host: prep %.3f ms, results downloaded at %.3f ms, grouping %.3f ms (%zu keys, %lld blocks)\n",
                h_prep, h_dl, hms() - h_dl, keys.size(), (long long)S.n_blocks);
}

// fragmenttg_postprocess (AnchorFinder.cpp:356-391) on the truncated key list
// (keys sorted, H the kept hashes): the groups, the used-hash quirk (add_used)
// and the host result
static void af_group_host(npgx_af* af, const std::vector<uint64_t>& keys, const std::vector<uint64_t>& Hh,
                          int key_bits, int32_t R, const SeqMeta* meta, const int32_t* by_rank, int k,
                          bool add_used) {
    npgx_af_stats& S = af->stats;
    std::vector<uint64_t> prefix2(R);
    for (int32_t r = 0; r < R; r++) prefix2[r] = 2ull * meta[r].order_off;
    const uint64_t key_mask = key_bits >= 64 ? ~0ull : ((1ull << key_bits) - 1);
    const bool sort_used = !af->used.empty();
    // pass 1 (sequential, cheap): the groups, the used-hash quirk and the
    // output offsets of the groups of two or more fragments
    const size_t nk = keys.size();
    std::vector<size_t>& gk = af->h_group_key;  // first key of each kept group
    gk.clear();
    af->r_block_start.clear();
    int64_t nout = 0;
    bool first_group = true;
    for (size_t i = 0; i < nk;) {
        const uint64_t idx = keys[i] >> key_bits;
        size_t j = i + 1;
        while (j < nk && (keys[j] >> key_bits) == idx) j++;
        if (!first_group && add_used) af->used.push_back(Hh[idx]);  // quirk: not the first group
        first_group = false;
        if (j - i >= 2) {
            af->r_block_start.push_back(nout);
            gk.push_back(i);
            nout += (int64_t)(j - i);
        }
        i = j;
    }
    af->r_block_start.push_back(nout);
    af->r_seq.resize((size_t)nout);
    af->r_min.resize((size_t)nout);
    af->r_max.resize((size_t)nout);
    af->r_ori.resize((size_t)nout);
    // pass 2: the fragments (FoundFragment::make_fragment :240-246), groups on
    // host threads; a group's keys ascend, so its sequence rank only moves forward
    const size_t ng = gk.size(), per = 256;  // groups per task: few tasks on the pool's shared counter
    heavy_for((ng + per - 1) / per, nout * 16, [&](size_t t) {
      for (size_t g = t * per; g < std::min(ng, (t + 1) * per); g++) {
        size_t q = gk[g];
        int32_t r = 0;
        for (int64_t o = af->r_block_start[g]; o < af->r_block_start[g + 1]; o++, q++) {
            const uint64_t key2 = keys[q] & key_mask;
            if (r + 1 < R && prefix2[(size_t)r + 1] <= key2)
                r = (int32_t)(std::upper_bound(prefix2.begin() + r + 1, prefix2.end(), key2) - prefix2.begin()) - 1;
            const uint64_t pos2 = key2 - prefix2[(size_t)r];
            const uint64_t size = (uint64_t)meta[(size_t)r].size;
            const bool direct = pos2 < size;
            const int64_t mn = (int64_t)(direct ? pos2 : pos2 - size);
            af->r_seq[(size_t)o] = by_rank[(size_t)r];
            af->r_min[(size_t)o] = mn;
            af->r_max[(size_t)o] = mn + k - 1;
            af->r_ori[(size_t)o] = direct ? 1 : -1;
        }
      }
    });
    if (sort_used) std::sort(af->used.begin(), af->used.end());
    if (af->used.size() != (size_t)S.n_used) af->used_dirty = true;
    S.n_blocks = (int64_t)af->r_block_start.size() - 1;
    S.n_fragments = (int64_t)af->r_seq.size();
    S.n_used = (int64_t)af->used.size();
    af->has_result = true;
}

// the deferred host result of the last run (see npgx_af.defer_host)
static void af_materialize(npgx_af* af) {
    if (!af->pending) return;
    af->pending = false;
    hipStream_t st = af->stream;
    NPGX_HIP(hipSetDevice(af->device));
    std::vector<uint64_t>& keys = af->host_keys;
    std::vector<uint64_t>& Hh = af->host_H;
    keys.resize((size_t)af->p_keep);
    Hh.resize((size_t)af->p_G);
    af->pinned_dl.ensure((size_t)(af->p_keep + af->p_G) * 8 + 8);
    uint64_t* pk = af->pinned_dl.p;
    if (af->p_keep) NPGX_HIP(hipMemcpyAsync(pk, af->cand_sorted.p, (size_t)af->p_keep * 8, hipMemcpyDeviceToHost, st));
    if (af->p_G) NPGX_HIP(hipMemcpyAsync(pk + af->p_keep, af->huniq.p, (size_t)af->p_G * 8, hipMemcpyDeviceToHost, st));
    NPGX_HIP(stream_wait(st));
    memcpy(keys.data(), pk, (size_t)af->p_keep * 8);
    memcpy(Hh.data(), pk + af->p_keep, (size_t)af->p_G * 8);
    af_group_host(af, keys, Hh, af->p_key_bits, af->p_R, af->p_meta.data(), af->p_by_rank.data(), af->p_k,
                  af->pending_used);
}

void af_set_defer(npgx_af* af, bool on) { af->defer_host = on; }

bool af_device_keys(npgx_af* af, AfDevKeys* o) {
    if (!af->pending) return false;
    o->keys = af->cand_sorted.p;
    o->keep = af->p_keep;
    o->key_bits = af->p_key_bits;
    o->k = af->p_k;
    o->R = af->p_R;
    o->meta = af->d_meta.p;
    o->by_rank = af->d_by_rank.p;
    return true;
}

}  // namespace npgx

extern "C" {

void npgx_af_default_options(npgx_af_options* o) {
    if (!o) return;
    memset(o, 0, sizeof(*o));
    o->anchor_size = 20;            // ANCHOR_SIZE
    o->anchor_similar = 1;
    o->anchor_fp_x1e4 = 1000;       // ANCHOR_FP 0.1
    o->max_anchor_fragments = 100000;  // MAX_ANCHOR_FRAGMENTS
    o->bloom_seed = 1;
}

int npgx_af_create(const npgx_af_options* o, npgx_af** out) {
    return guard([&] {
        NPGX_REQUIRE(o && out, NPGX_ERR_ARG, "null argument");
        // option rules (AnchorFinder.cpp:49-51)
        NPGX_REQUIRE(o->anchor_size > 0, NPGX_ERR_ARG, "Option rule failed: anchor-size > 0");
        NPGX_REQUIRE(o->anchor_size <= 32, NPGX_ERR_ARG, "Option rule failed: anchor-size <= 32");
        NPGX_REQUIRE(o->anchor_fp_x1e4 > 0 && o->anchor_fp_x1e4 < 10000, NPGX_ERR_ARG,
                     "anchor-fp must be in (0, 1)");
        NPGX_REQUIRE(o->max_anchor_fragments >= 0, NPGX_ERR_ARG, "max-anchor-fragments < 0");
        NPGX_REQUIRE(o->n_bloom_params >= 0 && o->n_bloom_params <= MAX_KB, NPGX_ERR_ARG,
                     "n_bloom_params out of range");
        NPGX_REQUIRE(o->bloom_epochs >= 0, NPGX_ERR_ARG, "bloom_epochs < 0");
        int dev = current_device_checked();
        auto* af = new npgx_af;
        af->opt = *o;
        af->opt.bloom_params = nullptr;
        if (o->n_bloom_params > 0)
            af->explicit_params.assign(o->bloom_params, o->bloom_params + o->n_bloom_params);
        af->device = dev;
        if (hipStreamCreateWithFlags(&af->stream, hipStreamNonBlocking) != hipSuccess ||
            hipHostMalloc((void**)&af->h_pinned, 64) != hipSuccess) {
            delete af;
            throw Error(NPGX_ERR_HIP, "stream / pinned allocation failed");
        }
        *out = af;
    });
}

int npgx_af_run(npgx_af* af, const npgx_seqset* s) {
    return guard([&] {
        NPGX_REQUIRE(af && s, NPGX_ERR_ARG, "null argument");
        af_run(af, s, nullptr);
    });
}

int npgx_af_run_sharded(npgx_af* af, const npgx_seqset* s, const npgx_comm* comm) {
    return guard([&] {
        NPGX_REQUIRE(af && s && comm, NPGX_ERR_ARG, "null argument");
        NPGX_REQUIRE(comm->world >= 1 && comm->rank >= 0 && comm->rank < comm->world, NPGX_ERR_ARG,
                     "bad rank / world");
        NPGX_REQUIRE(comm->allreduce_i32 && comm->allgather_i64 && comm->allgatherv_u64, NPGX_ERR_ARG,
                     "missing collective callback");
        af_run(af, s, comm->world > 1 ? comm : nullptr);
    });
}

int npgx_af_stats_get(const npgx_af* af, npgx_af_stats* out) {
    return guard([&] {
        NPGX_REQUIRE(af && out, NPGX_ERR_ARG, "null argument");
        af_materialize(const_cast<npgx_af*>(af));
        *out = af->stats;
    });
}

int npgx_af_result_counts(const npgx_af* af, int64_t* nb, int64_t* nf) {
    return guard([&] {
        NPGX_REQUIRE(af && nb && nf, NPGX_ERR_ARG, "null argument");
        NPGX_REQUIRE(af->has_result, NPGX_ERR_STATE, "no AnchorFinder result yet");
        af_materialize(const_cast<npgx_af*>(af));
        *nb = (int64_t)af->r_block_start.size() - 1;
        *nf = (int64_t)af->r_seq.size();
    });
}

int npgx_af_result_copy(const npgx_af* af, int64_t* block_start, int32_t* seq, int64_t* min_pos,
                        int64_t* max_pos, int8_t* ori) {
    return guard([&] {
        NPGX_REQUIRE(af, NPGX_ERR_ARG, "null argument");
        NPGX_REQUIRE(af->has_result, NPGX_ERR_STATE, "no AnchorFinder result yet");
        af_materialize(const_cast<npgx_af*>(af));
        const size_t nf = af->r_seq.size();
        if (block_start) memcpy(block_start, af->r_block_start.data(), af->r_block_start.size() * 8);
        if (seq) memcpy(seq, af->r_seq.data(), nf * 4);
        if (min_pos) memcpy(min_pos, af->r_min.data(), nf * 8);
        if (max_pos) memcpy(max_pos, af->r_max.data(), nf * 8);
        if (ori) memcpy(ori, af->r_ori.data(), nf);
    });
}

int npgx_af_used_hashes(const npgx_af* af, uint64_t* out, int64_t cap, int64_t* n) {
    return guard([&] {
        NPGX_REQUIRE(af && n, NPGX_ERR_ARG, "null argument");
        af_materialize(const_cast<npgx_af*>(af));
        *n = (int64_t)af->used.size();
        if (out) memcpy(out, af->used.data(), (size_t)std::min<int64_t>(cap, *n) * 8);
    });
}

int npgx_af_clear_used(npgx_af* af) {
    return guard([&] {
        NPGX_REQUIRE(af, NPGX_ERR_ARG, "null argument");
        af->used.clear();
        af->pending_used = false;  // (a deferred result's used hashes go with the rest)
        af->used_dirty = true;
    });
}

int npgx_af_kernel_times(const npgx_af* af, npgx_kernel_time* out, int32_t cap, int32_t* n) {
    return guard([&] {
        NPGX_REQUIRE(af && n && (out || cap == 0), NPGX_ERR_ARG, "null argument");
        af->timer.copy_out(out, cap, n);
    });
}

void npgx_af_free(npgx_af* af) {
    if (!af) return;
    (void)hipSetDevice(af->device);
    if (af->stream) (void)hipStreamDestroy(af->stream);
    if (af->h_pinned) (void)hipHostFree(af->h_pinned);
    delete af;
}

}  // extern "C"
