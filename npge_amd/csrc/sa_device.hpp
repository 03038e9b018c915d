// sa_device.hpp -- wave-level building blocks of the greedy multiple aligner
// (SimilarAligner, src/algo/SimilarAligner.cpp:41-485) on CDNA4.
//
// One wavefront owns one alignment problem.  Two lane layouts alternate:
//   * rows mode: lane i owns row i (n <= 64) -- pos and the view live in lane
//     i's registers; column tests (is_equal :101-115) are ballots.  Used for the
//     branchy steps: try_gap, try_aligned, the bookkeeping of append_end.
//   * columns mode: lane j owns column pos+j of EVERY row; a 64-column chunk is
//     read and written with coalesced byte accesses, one row at a time.  Used for
//     the common case -- runs of identical columns and single mismatches
//     (process_cols :355-358 with try_mismatch :122-134) -- and for bulk copies.
// A row is read through a View (char(q) = p[d*q], q < len), so the reversed
// sub-problems the reference builds with substr + std::reverse
// (append_aligned :274-293) are views, not copies.  The recursion
// append_aligned -> process_seqs runs on an explicit per-wave stack; a child
// writes right after the parent's cursor and is reversed in place on return.
//
// Past-the-end reads (find_best_gap :191-217 may read beyond a row): char(len)
// is '\0' like std::string; char(q > len) is a per-row sentinel equal to
// nothing (same convention as the oracle).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#ifdef NPGX_SA_PROFILE
#define SA_T0(x) const long long x = clock64()
#define SA_ACC(k, x) prof[k] += clock64() - x
#else
#define SA_T0(x)
#define SA_ACC(k, x)
#endif

namespace npgx {
namespace sa {

struct View {
    const char* p;  // address of char 0
    int len;
    int d;          // +1 forward, -1 reversed
};

struct Params {
    int mc, gc, ac, min_length;
    int wf;  // FindLowSimilar weight factor (FindLowSimilar.cpp:56-60)
    int lh;  // try_aligned: shifts searched incrementally before the prefix search (0: never switch)
    int lm;  // ... the prefix search's first prefix (shifts)
    int llds = 1;  // the prefix search's first prefixes in the LDS word table when they fit (NPGX_LONG_LDS)
};

// Per-wave scratch (global memory), sized by the host for the batch.
struct Slot {
    unsigned long long* tkeys;  // try_aligned word table: (epoch << 48 | word)
    unsigned long long* tmask;  // row masks
    uint32_t* tdone;            // row-parallel search: the word's last first sighting
    uint32_t tcap_log2;
    unsigned long long* lkeys;  // the same table in LDS (tried first)
    unsigned long long* lmask;
    uint32_t* ldone;
    uint32_t ltab_log2;
    unsigned long long* lwords;  // LDS [row][64]: one chunk's words (vector try_aligned);
                                 // more rows: [shift][row] words of the first 2048/n shifts
    int hist_cap;                // > 0: lwords holds HIST_SHIFTS x 64 words of history
    const char** st_p;          // append_aligned stack, 64 lanes per level
    int* st_len;
    int* st_pos;
    int* st_col;
    int st_depth_max;
    int4* regions;              // FindLowSimilar regions (start, stop, good, weight)
    unsigned char* good_col;
};

static constexpr int VEC_ROWS = 8;
#ifndef SA_FAST_ROWS  // (4 measured no faster at C3 / R3 / C2 and 2 % slower on the pair job, r05e / r05n)
#define SA_FAST_ROWS 1
#endif
static constexpr int FR = SA_FAST_ROWS;  // fast_run: rows loaded per batch
typedef __attribute__((address_space(3))) unsigned long long LdsU64;  // LDS-qualified word-table entry
typedef __attribute__((address_space(3))) uint32_t LdsU32;
static constexpr int HIST_SHIFTS = 32;  // words per lane kept for the first-sighting scan  // try_aligned with lanes = shifts up to this many rows

struct WaveCtx {
    int lane;
    int n;
    unsigned long long rowmask;
    bool act;
};

__device__ __forceinline__ unsigned long long ballot(bool b) { return __ballot(b); }

__device__ __forceinline__ int vch(const View& v, int q, int lane) {
    if ((unsigned)q < (unsigned)v.len) return (unsigned char)v.p[(ptrdiff_t)v.d * q];
    return q == v.len ? 0 : 0x100 + lane;  // q < 0 only on idle lanes (rows >= n)
}

__device__ __forceinline__ bool all_eq(const WaveCtx& w, int c) {
    const int c0 = __builtin_amdgcn_readlane(c, 0);
    return (ballot(!w.act || c == c0) & w.rowmask) == w.rowmask;
}

__device__ __forceinline__ bool any_lane(const WaveCtx& w, bool b) {
    return (ballot(w.act && b) & w.rowmask) != 0;
}

// Wave reductions with DPP row shifts and row broadcasts (a few VALU cycles
// each) instead of ds_bpermute round trips; every lane gets the result.
// Called with all 64 lanes active.
template <class Op>
__device__ __forceinline__ int dpp_reduce(int v, int id, Op op) {
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x118, 0xf, 0xf, false));  // row_shr:8
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ int wave_max(int v) {
    return dpp_reduce(v, (int)0x80000000, [](int a, int b) { return max(a, b); });
}
__device__ __forceinline__ int wave_min(int v) {
    return dpp_reduce(v, 0x7fffffff, [](int a, int b) { return min(a, b); });
}
__device__ __forceinline__ int wave_sum(int v) {
    return dpp_reduce(v, 0, [](int a, int b) { return a + b; });
}
__device__ __forceinline__ unsigned long long shfl64(unsigned long long v, int src) {
    const unsigned lo = (unsigned)__shfl((int)(unsigned)v, src);
    const unsigned hi = (unsigned)__shfl((int)(unsigned)(v >> 32), src);
    return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ const char* shfl_ptr(const char* p, int src) {
    return (const char*)shfl64((unsigned long long)p, src);
}
// lane k's value for a wave-uniform k: v_readlane instead of ds_bpermute
__device__ __forceinline__ int bcast(int v, int k) { return __builtin_amdgcn_readlane(v, k); }
__device__ __forceinline__ unsigned long long bcast64(unsigned long long v, int k) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, k);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), k);
    return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ const char* bcast_ptr(const char* p, int k) {
    return (const char*)bcast64((unsigned long long)p, k);
}

// number of trailing one bits
__device__ __forceinline__ int ctz_ones(unsigned long long m) {
    return m == ~0ull ? 64 : __ffsll((long long)~m) - 1;
}

// ------------------------------------------------------------ columns-mode helpers
// Buffers hold row r at base + r*cap.  All lanes take part; rows loop uniformly.

// rows [0,n): dst[d0 + j] = src[s0 + j] for j < len.  (row, 64-column chunk)
// pairs four at a time: four loads in flight per lane instead of one.
__device__ __forceinline__ void cm_copy(const WaveCtx& w, const char* src, char* dst, int cap, int s0, int d0,
                                        int len) {
    const int nch = (len + 63) >> 6, np = w.n * nch;
    for (int p0 = 0; p0 < np; p0 += 4) {
        char t[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int p = p0 + u, r = p / max(nch, 1), j = (p - r * nch) * 64 + w.lane;
            t[u] = (p < np && j < len) ? src[(size_t)r * cap + s0 + j] : 0;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int p = p0 + u, r = p / max(nch, 1), j = (p - r * nch) * 64 + w.lane;
            if (p < np && j < len) dst[(size_t)r * cap + d0 + j] = t[u];
        }
    }
    __syncthreads();
}

// rows [0,n): dst[d0 + j] = src[len - 1 - j] for j < len (a reversed copy;
// src and dst rows of stride cap, (row, 64-column chunk) pairs four at a time)
__device__ __forceinline__ void cm_copy_rev(const WaveCtx& w, const char* src, char* dst, int cap, int d0, int len) {
    const int nch = (len + 63) >> 6, np = w.n * nch;
    for (int p0 = 0; p0 < np; p0 += 4) {
        char t[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int p = p0 + u, r = p / max(nch, 1), j = (p - r * nch) * 64 + w.lane;
            t[u] = (p < np && j < len) ? src[(size_t)r * cap + len - 1 - j] : 0;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int p = p0 + u, r = p / max(nch, 1), j = (p - r * nch) * 64 + w.lane;
            if (p < np && j < len) dst[(size_t)r * cap + d0 + j] = t[u];
        }
    }
    __syncthreads();
}

// reverse columns [c0, c1) of every row in place (pairs four at a time)
__device__ __forceinline__ void cm_reverse(const WaveCtx& w, char* base, int cap, int c0, int c1) {
    const int half = (c1 - c0) >> 1;
    const int nch = (half + 63) >> 6, np = w.n * nch;
    for (int p0 = 0; p0 < np; p0 += 4) {
        char x[4], y[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int p = p0 + u, r = p / max(nch, 1), j = (p - r * nch) * 64 + w.lane;
            const bool in = p < np && j < half;
            char* row = base + (size_t)r * cap;
            x[u] = in ? row[c0 + j] : 0;
            y[u] = in ? row[c1 - 1 - j] : 0;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int p = p0 + u, r = p / max(nch, 1), j = (p - r * nch) * 64 + w.lane;
            if (p < np && j < half) {
                char* row = base + (size_t)r * cap;
                row[c0 + j] = y[u];
                row[c1 - 1 - j] = x[u];
            }
        }
    }
    __syncthreads();
}

__device__ __forceinline__ unsigned long long Proc_code3(int c) {
    return c == 'A' ? 1 : c == 'C' ? 2 : c == 'G' ? 3 : c == 'N' ? 4 : c == 'T' ? 5 : 6;
}

// find_best_word over 64 shifts at once for up to VEC_ROWS rows: lanes are
// shifts.  Row i's word at shift s is complete when every row k has had it
// at some shift <= s: within the chunk by a broadcast compare against row
// k's 64 words, before the chunk through the global word table, which
// receives each finished chunk's words (row bits, epoch-tagged).  The
// first shift with a complete word wins; among the rows complete there the
// highest one names the word (the reference overwrites best_word row by
// row), and every row's shift is its first sighting of that word.
struct VecOut {
    int found, my_shift, shifts;
    uint32_t epoch;
#ifdef NPGX_SA_PROFILE
    long long t_words, t_cmp;
    int chunks;
#endif
};

// (a free function of scalars: the caller's Proc stays in registers)
__device__ __noinline__ VecOut find_word_vec(const char* vp, int vlen, int vd, int pos, int lane, int n, int ac,
                                             int max_shift, unsigned long long* W, unsigned long long* tkeys,
                                             unsigned long long* tmask, uint32_t tcap_log2, uint32_t epoch) {
    // the arguments are wave-uniform: make that visible (scalar loop control)
    n = __builtin_amdgcn_readfirstlane(n);
    ac = __builtin_amdgcn_readfirstlane(ac);
    max_shift = __builtin_amdgcn_readfirstlane(max_shift);
    tcap_log2 = (uint32_t)__builtin_amdgcn_readfirstlane((int)tcap_log2);
    epoch = (uint32_t)__builtin_amdgcn_readfirstlane((int)epoch);
    W = (unsigned long long*)bcast_ptr((const char*)W, 0);
    VecOut out{};
    out.epoch = epoch;
    const View v{vp, vlen, vd};
    const bool act = lane < n;
    int my_shift = 0;
    const unsigned long long wmask = (ac >= 16) ? ((1ull << 48) - 1) : ((1ull << (3 * ac)) - 1);
    const unsigned long long EPM = ~((1ull << 48) - 1);
    const uint32_t tcap = 1u << tcap_log2;
    unsigned long long ep = 0;
    uint32_t inserted = 0;  // keys this call claimed in the global table
    for (int S0 = 0; S0 < max_shift; S0 += 64) {
        const int s = S0 + lane;
        const bool valid = s < max_shift;
        const int last = __builtin_amdgcn_readfirstlane(min(63, max_shift - 1 - S0));
#ifdef NPGX_SA_PROFILE
        out.chunks++;
        const long long tw0 = clock64();
#endif
        for (int k = 0; k < n; k++) {
            // codes of chars q0 .. q0+127 (two coalesced loads), words by shuffles
            const char* pk = bcast_ptr(v.p, k);
            const int lk = bcast(v.len, k), dk = bcast(v.d, k);
            const int q0 = bcast(pos, k) + S0;
            const int qa = q0 + lane, qb = q0 + 64 + lane;
            const int ca = qa < lk ? (int)Proc_code3((unsigned char)pk[(ptrdiff_t)dk * qa]) : 6;
            const int cb = qb < lk ? (int)Proc_code3((unsigned char)pk[(ptrdiff_t)dk * qb]) : 6;
            const int packed = ca | (cb << 8);
            unsigned long long x = 0;
            for (int j = 0; j < ac; j++) {
                const int src = lane + j;
                const int got = __shfl(packed, src & 63);
                x = (x << 3) | (unsigned long long)(src < 64 ? (got & 0xFF) : (got >> 8));
            }
            W[k * 64 + lane] = valid ? (x & wmask) : 0ull;
        }
        __syncthreads();
#ifdef NPGX_SA_PROFILE
        out.t_words += clock64() - tw0;
        const long long tc0 = clock64();
#endif
        const unsigned long long vmask = ballot(valid);
        int f_best = 64, i_best = -1;
        if (n <= 4 && ac <= 10) {
            // LDS table of the chunk's words (rows 4..7 of W): key = word + 1,
            // and per row the first shift holding it (byte k, 0xFF = absent).
            // Rows insert one after the other, so a row's byte is the only one
            // changing during its pass and a 32-bit atomicMin of the whole
            // byte vector is that byte's minimum.  Then lane s of row i knows
            // for every row k whether wi occurs in row k at a shift <= s.
            uint32_t* T32 = (uint32_t*)(W + 4 * 64);  // 256 entries x (key, shifts)
            for (int e = lane; e < 256; e += 64) {
                T32[2 * e] = 0u;
                T32[2 * e + 1] = 0xFFFFFFFFu;
            }
            __syncthreads();
            for (int k = 0; k < n; k++) {
                if (valid) {
                    const uint32_t key = (uint32_t)W[k * 64 + lane] + 1u;
                    uint32_t e = (key * 0x9E3779B1u) >> 24;
                    for (int probe = 0; probe < 256; probe++) {
                        const uint32_t o = atomicCAS(&T32[2 * e], 0u, key);
                        if (o == 0u || o == key) break;
                        e = (e + 1) & 255u;
                    }
                    const uint32_t cur = T32[2 * e + 1];
                    atomicMin(&T32[2 * e + 1], (cur & ~(0xFFu << (8 * k))) | ((uint32_t)lane << (8 * k)));
                }
                __syncthreads();
            }
            for (int i = 0; i < n; i++) {
                const unsigned long long wi = W[i * 64 + lane];
                unsigned old = 0;  // rows that had wi before this chunk
                if (S0 > 0 && valid) {
                    const unsigned long long key = ep | wi;
                    uint32_t slot = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - tcap_log2));
                    while (true) {
                        const unsigned long long k = tkeys[slot];
                        if (k == key) {
                            const unsigned long long m = tmask[slot];
                            old = (m & EPM) == ep ? (unsigned)(m & 0xFFu) : 0u;
                            break;
                        }
                        if ((k & EPM) != ep) break;
                        slot = (slot + 1) & (tcap - 1);
                    }
                }
                bool ok = valid;
                if (valid) {
                    const uint32_t key = (uint32_t)wi + 1u;
                    uint32_t e = (key * 0x9E3779B1u) >> 24;
                    for (int probe = 0; probe < 256 && T32[2 * e] != key; probe++) e = (e + 1) & 255u;
                    const uint32_t sh = T32[2 * e + 1];
                    for (int k = 0; k < n; k++)
                        if (k != i) ok &= ((old >> k) & 1u) || ((sh >> (8 * k)) & 0xFFu) <= (uint32_t)lane;
                }
                const unsigned long long comp = ballot(ok);
                if (comp) {
                    const int f = __ffsll((long long)comp) - 1;
                    if (f <= f_best) {  // ties: the higher row names the word
                        f_best = f;
                        i_best = i;
                    }
                }
            }
            __syncthreads();
        } else
        for (int i = 0; i < n; i++) {
            const unsigned long long wi = W[i * 64 + lane];
            unsigned old = 0;  // rows that had wi before this chunk
            if (S0 > 0 && valid) {
                const unsigned long long key = ep | wi;
                uint32_t slot = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - tcap_log2));
                while (true) {
                    const unsigned long long k = tkeys[slot];
                    if (k == key) {
                        const unsigned long long m = tmask[slot];
                        old = (m & EPM) == ep ? (unsigned)(m & 0xFFu) : 0u;
                        break;
                    }
                    if ((k & EPM) != ep) break;
                    slot = (slot + 1) & (tcap - 1);
                }
            }
            unsigned long long comp = vmask;
            for (int k = 0; k < n; k++) {
                if (k == i) continue;
                unsigned long long found = ballot((old >> k) & 1u);
                const unsigned long long wk = W[k * 64 + lane];
                const unsigned lo = (unsigned)wk, hi = (unsigned)(wk >> 32);
                if (ac <= 10) {  // 30-bit words: one readlane and a 32-bit compare per shift
                    const unsigned wi32 = (unsigned)wi;
                    int t = 0;
                    for (; t + 3 <= last; t += 4) {
                        const unsigned x0 = (unsigned)__builtin_amdgcn_readlane((int)lo, t);
                        const unsigned x1 = (unsigned)__builtin_amdgcn_readlane((int)lo, t + 1);
                        const unsigned x2 = (unsigned)__builtin_amdgcn_readlane((int)lo, t + 2);
                        const unsigned x3 = (unsigned)__builtin_amdgcn_readlane((int)lo, t + 3);
                        found |= (ballot(wi32 == x0) & (~0ull << t)) | (ballot(wi32 == x1) & (~0ull << (t + 1))) |
                                 (ballot(wi32 == x2) & (~0ull << (t + 2))) |
                                 (ballot(wi32 == x3) & (~0ull << (t + 3)));
                    }
                    for (; t <= last; t++)
                        found |= ballot(wi32 == (unsigned)__builtin_amdgcn_readlane((int)lo, t)) & (~0ull << t);
                } else {
                    for (int t = 0; t <= last; t++) {
                        const unsigned long long x =
                            ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)hi, t) << 32) |
                            (unsigned)__builtin_amdgcn_readlane((int)lo, t);
                        found |= ballot(wi == x) & (~0ull << t);
                    }
                }
                comp &= found;
            }
            if (comp) {
                const int f = __ffsll((long long)comp) - 1;
                if (f <= f_best) {  // ties: the higher row names the word
                    f_best = f;
                    i_best = i;
                }
            }
        }
#ifdef NPGX_SA_PROFILE
        out.t_cmp += clock64() - tc0;
#endif
        if (i_best >= 0) {
            out.shifts += f_best + 1;
            const unsigned long long best = W[i_best * 64 + f_best];
            bool one = true;
            for (int k = 0; k < n; k++) one &= W[k * 64 + f_best] == best;
            if (one) {  // words.size() == 1: every row at this shift
                my_shift = S0 + f_best;
            } else if (S0 == 0) {
                for (int k = 0; k < n; k++) {
                    const unsigned long long m =
                        ballot(W[k * 64 + lane] == best) & (f_best == 63 ? ~0ull : ((2ull << f_best) - 1));
                    if (lane == k) my_shift = __ffsll((long long)m) - 1;
                }
            } else {  // first sighting may lie in an earlier chunk: scan the row
                const int sb = S0 + f_best;
                my_shift = -1;
                if (act) {
                    unsigned long long x = 0;
                    for (int j = 0; j < ac - 1; j++) x = (x << 3) | Proc_code3(vch(v, pos + j, lane));
                    for (int t = 0; t <= sb; t++) {
                        x = ((x << 3) | Proc_code3(vch(v, pos + t + ac - 1, lane))) & wmask;
                        if (x == best) {
                            my_shift = t;
                            break;
                        }
                    }
                }
            }
            __syncthreads();
            out.found = 1;
            out.my_shift = my_shift;
            return out;
        }
        out.shifts += last + 1;
        if (S0 + 64 >= max_shift) break;
        // remember this chunk's words for the next chunks (the table is kept
        // at most half full: a call that would pass that gives up, -1)
        if (inserted + 64u * (uint32_t)n > (tcap >> 1)) {
            __syncthreads();
            out.found = -1;
            return out;
        }
        if (S0 == 0) {
            uint32_t ep32 = out.epoch + 1;
            if (ep32 >= 0xFFFF) {
                for (uint32_t i = lane; i < tcap; i += 64) {
                    tkeys[i] = 0ull;
                    tmask[i] = 0ull;
                }
                __threadfence();
                ep32 = 1;
            }
            out.epoch = ep32;
            ep = (unsigned long long)ep32 << 48;
        }
        for (int k = 0; k < n; k++) {
            if (!valid) continue;
            const unsigned long long key = ep | W[k * 64 + lane];
            uint32_t slot = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - tcap_log2));
            bool claimed = false;
            while (true) {
                const unsigned long long kk =
                    __hip_atomic_load(&tkeys[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (kk == key) break;
                if ((kk & EPM) != ep) {
                    if (atomicCAS(&tkeys[slot], kk, key) == kk) {
                        claimed = true;
                        break;
                    }
                    continue;
                }
                slot = (slot + 1) & (tcap - 1);
            }
            inserted += (uint32_t)__popcll(ballot(claimed));
            const unsigned long long bit = 1ull << k;
            unsigned long long m = __hip_atomic_load(&tmask[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            while (true) {
                if ((m & EPM) == ep) {
                    atomicOr(&tmask[slot], bit);
                    break;
                }
                const unsigned long long prev = atomicCAS(&tmask[slot], m, ep | bit);
                if (prev == m) break;
                m = prev;
            }
        }
        __threadfence();
        __syncthreads();
    }
    __syncthreads();
    return out;
}

// ------------------------------------------------------------ long word searches
// try_aligned (:295-308) when the first complete word lies far away (rows
// unrelated over hundreds or thousands of bases: inversions, insertions).
// The incremental searches above take the shifts one after the other, each
// paying a round of word-table atomics (a shift cost ~2800 cycles on the
// repeat-rich R3 set).  Past their first shifts this search answers the
// same question for a whole prefix of shifts [0, M) and doubles M until the
// answer lies inside:
//   T(w)  = max over rows k of first_k(w): the shift at which the reference's
//           ff[w] becomes complete (every row has sighted w);
//   S*    = min over w of T(w): the shift at which try_aligned stops;
//   best  = word_i(S*) of the highest row i whose word is complete at S*
//           (find_best_word overwrites best_word row by row);
//   shift = first_k(best) per row, or S* for every row when all rows hold
//           the same word at S* (words.size() == 1).
// A complete word is one of row 0's words, so the table holds row 0's words
// of [0, M) only (at most M keys, not n x M), each with a state packed into
// 64 bits: epoch (16) | rows that have sighted it (16) | ~T (32).  Rows
// 1..n-1 then pass over [0, M) in order; row k's sighting at s of a word rows
// 0..k-1 all have sighted raises it to k+1 rows with T = max(T, s) by
// atomicMax -- the packing makes the higher row count win and, among equal
// counts, the smaller T: the row's FIRST sighting.  A step takes 512 shifts
// (8 per lane) in increasing order and reads every state before any of its
// atomics, so a word raised by an earlier step of the pass is never raised
// again.  A row pass that raises nothing ends the prefix (S* >= M); the
// last row's smallest T is S*.
static constexpr int LW_STEP = 512;
typedef __attribute__((address_space(3))) unsigned char LdsU8;

struct LongOut {
    int found, my_shift, shifts;  // found: 1, 0 (no shift works), -1 (the table cannot take a prefix)
    uint32_t epoch;
    int M;                        // found == -1: the prefix the table could not take
};

// codes of chars q0 .. q0 + 575 of a row into LDS (7 past the row's end)
__device__ __forceinline__ void lw_codes(const char* p, int len, int d, int q0, int lane, LdsU8* buf) {
#pragma unroll
    for (int j = 0; j < 9; j++) {
        const int q = q0 + j * 64 + lane;
        buf[j * 64 + lane] = q < len ? (unsigned char)Proc_code3((unsigned char)p[(ptrdiff_t)d * q]) : 7;
    }
}

// words at shifts base + 8*lane + u, u < 8, from the codes of chars base + ...
__device__ __forceinline__ void lw_words(const LdsU8* buf, int lane, int ac, unsigned long long wmask,
                                         unsigned long long (&wd)[8]) {
    const int sb = 8 * lane;
    unsigned long long x = 0;
    for (int t = 0; t < ac - 1; t++) x = (x << 3) | buf[sb + t];
#pragma unroll
    for (int u = 0; u < 8; u++) {
        x = ((x << 3) | buf[sb + ac - 1 + u]) & wmask;
        wd[u] = x;
    }
}

// T: the table in global memory (unsigned long long) or in LDS (LdsU64: the
// prefixes that fit the workgroup's LDS word table -- no HBM traffic, LDS
// atomics); a call on the LDS table that meets a prefix too long for it
// returns found -1 with that prefix in M, and the caller goes on from there
// on the global table (every prefix's pass starts from scratch: the same answer)
template <class TT>
#ifdef SA_LONG_INLINE  // (A/B builds: inlined instead of called)
__device__ __forceinline__
#else
__device__ __noinline__
#endif
LongOut find_word_long(const char* vp, int vlen, int vd, int pos, int lane, int n, int ac,
                                               int max_shift, int M0, unsigned long long* W,
                                               TT* tkeys, TT* tmask,
                                               uint32_t tcap_log2, uint32_t epoch) {
    n = __builtin_amdgcn_readfirstlane(n);
    ac = __builtin_amdgcn_readfirstlane(ac);
    max_shift = __builtin_amdgcn_readfirstlane(max_shift);
    M0 = __builtin_amdgcn_readfirstlane(M0);
    tcap_log2 = (uint32_t)__builtin_amdgcn_readfirstlane((int)tcap_log2);
    epoch = (uint32_t)__builtin_amdgcn_readfirstlane((int)epoch);
    LdsU8* buf = (LdsU8*)W;
    LongOut out{0, 0, max_shift, epoch, 0};
    const bool act = lane < n;
    const View v{vp, vlen, vd};
    const unsigned long long wmask = (ac >= 16) ? ((1ull << 48) - 1) : ((1ull << (3 * ac)) - 1);
    const unsigned long long EPM = ~((1ull << 48) - 1);
    const uint32_t tcap = 1u << tcap_log2;
    const uint32_t INV = 0xFFFFFFFFu;
    int S = -1;
    unsigned long long ep = 0;
    for (int M = max(M0, LW_STEP);; M *= 2) {
        const int Mp = min(M, max_shift);
        if (2u * (uint32_t)Mp > tcap) {
            out.found = -1;
            out.M = M;
            return out;
        }
        uint32_t ep32 = out.epoch + 1;
        if (ep32 >= 0xFFFF) {  // epoch wrap: clear the table
            for (uint32_t i = lane; i < tcap; i += 64) {
                tkeys[i] = 0ull;
                tmask[i] = 0ull;
            }
            __threadfence();
            ep32 = 1;
        }
        out.epoch = ep32;
        ep = (unsigned long long)ep32 << 48;
        bool alive = true;
        int tmin = 0x7fffffff;
        for (int k = 0; k < n && alive; k++) {
            const char* pk = bcast_ptr(vp, k);
            const int lk = bcast(vlen, k), dk = bcast(vd, k), qk = bcast(pos, k);
            int any = 0;
            for (int base = 0; base < Mp; base += LW_STEP) {
                if (k == n - 1 && base > tmin) break;  // later shifts cannot lower the last row's T
                __syncthreads();
                lw_codes(pk, lk, dk, qk + base, lane, buf);
                __syncthreads();
                unsigned long long wd[8];
                lw_words(buf, lane, ac, wmask, wd);
                uint32_t slot[8];
                bool valid[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    valid[u] = base + 8 * lane + u < Mp;
                    slot[u] = (uint32_t)(((ep | wd[u]) * 0x9E3779B97F4A7C15ull) >> (64 - tcap_log2));
                }
                if (k == 0) {  // row 0: insert (claim the key, reset a new key's state)
                    bool claimed[8];
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        claimed[u] = false;
                        if (!valid[u]) continue;
                        const unsigned long long key = ep | wd[u];
                        while (true) {
                            unsigned long long kk =
                                __hip_atomic_load(&tkeys[slot[u]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            if (kk == key) break;
                            if ((kk & EPM) != ep) {
                                if (__hip_atomic_compare_exchange_strong(&tkeys[slot[u]], &kk, key, __ATOMIC_RELAXED,
                                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                                    claimed[u] = true;
                                    break;
                                }
                                if (kk == key) break;
                                continue;
                            }
                            slot[u] = (slot[u] + 1) & (tcap - 1);
                        }
                    }
#pragma unroll
                    for (int u = 0; u < 8; u++)
                        if (claimed[u]) __hip_atomic_store(&tmask[slot[u]], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __threadfence();
#pragma unroll
                    for (int u = 0; u < 8; u++)
                        if (valid[u])
                            __hip_atomic_fetch_max(&tmask[slot[u]],
                                                   ep | (1ull << 32) | (unsigned long long)(INV - (uint32_t)(base + 8 * lane + u)),
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    any = 1;
                } else {  // rows 1..n-1: raise the words rows 0..k-1 all have
                    unsigned long long kk[8];
#pragma unroll
                    for (int u = 0; u < 8; u++)
                        kk[u] = valid[u] ? __hip_atomic_load(&tkeys[slot[u]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                         : 0ull;
                    bool hit[8];
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        const unsigned long long key = ep | wd[u];
                        while (valid[u] && kk[u] != key && (kk[u] & EPM) == ep) {
                            slot[u] = (slot[u] + 1) & (tcap - 1);
                            kk[u] = __hip_atomic_load(&tkeys[slot[u]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        }
                        hit[u] = valid[u] && kk[u] == key;
                    }
                    unsigned long long st[8];
#pragma unroll
                    for (int u = 0; u < 8; u++)
                        st[u] = hit[u] ? __hip_atomic_load(&tmask[slot[u]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                       : 0ull;
                    const unsigned long long want = ep | ((unsigned long long)k << 32);
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        if (!hit[u] || (st[u] & ~0xFFFFFFFFull) != want) continue;
                        const int s = base + 8 * lane + u;
                        const int T = (int)(INV - (uint32_t)st[u]);
                        const int t = max(T, s);
                        __hip_atomic_fetch_max(&tmask[slot[u]],
                                               ep | ((unsigned long long)(k + 1) << 32) | (unsigned long long)(INV - (uint32_t)t),
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        any = 1;
                        if (k == n - 1) tmin = min(tmin, t);
                    }
                    if (k == n - 1) tmin = wave_min(tmin);
                }
            }
            __threadfence();  // this row's raises before the next row's reads
            alive = ballot(any != 0) != 0ull;
        }
        if (alive) {
            S = tmin;
            break;
        }
        if (Mp >= max_shift) {
            __syncthreads();
            return out;  // no shift works
        }
    }
    // the word: the highest row whose word at S* is complete
    unsigned long long wi = 0;
    if (act)
        for (int t = 0; t < ac; t++) wi = (wi << 3) | Proc_code3(vch(v, pos + S + t, lane));
    bool complete = false;
    if (act) {
        const unsigned long long key = ep | wi;
        uint32_t sl = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - tcap_log2));
        while (true) {
            const unsigned long long kk = __hip_atomic_load(&tkeys[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (kk == key) {
                const unsigned long long st = __hip_atomic_load(&tmask[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                complete = (st & ~0xFFFFFFFFull) == (ep | ((unsigned long long)n << 32)) &&
                           (int)(INV - (uint32_t)st) <= S;
                break;
            }
            if ((kk & EPM) != ep) break;
            sl = (sl + 1) & (tcap - 1);
        }
    }
    const unsigned long long cm = ballot(complete);
    const int ib = cm ? 63 - __clzll((long long)cm) : 0;
    const unsigned long long best = bcast64(wi, ib);
    int my_shift = S;
    if ((ballot(act && wi != best)) != 0ull) {
        // first sightings of the word: each row's shifts [0, S] in steps
        for (int k = 0; k < n; k++) {
            const char* pk = bcast_ptr(vp, k);
            const int lk = bcast(vlen, k), dk = bcast(vd, k), qk = bcast(pos, k);
            int f = 0x7fffffff;
            for (int base = 0; base <= S && f == 0x7fffffff; base += LW_STEP) {
                __syncthreads();
                lw_codes(pk, lk, dk, qk + base, lane, buf);
                __syncthreads();
                unsigned long long wd[8];
                lw_words(buf, lane, ac, wmask, wd);
                int g = 0x7fffffff;
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int s = base + 8 * lane + u;
                    if (s <= S && wd[u] == best) g = min(g, s);
                }
                f = wave_min(g);
            }
            if (lane == k) my_shift = f;
        }
    }
    __syncthreads();
    out.found = 1;
    out.my_shift = my_shift;
    out.shifts = S + 1;
    return out;
}


// ---------------------------------------------------------------- process_seqs
// LONG: try_aligned may switch to the prefix search (find_word_long).  Its
// call costs the kernels that can make it 664 bytes of scratch a lane against
// 312 (the registers live across the call): under many concurrent streams
// (the pair job) that scratch throttled the aligner by a fifth, so the
// kernels come in both forms and an aligner with long_head 0 launches the
// ones without the call.
template <bool LONG>
struct ProcT {
    WaveCtx w;
    Params P;
    Slot S;
    char* ob;        // output base (row r at ob + r*cap)
    int cap;
    View v;          // this lane's row (rows mode)
    int pos;         // this lane's cursor
    int col;         // output cursor (all rows equal length between steps)
    bool ovf;
    bool rovf;       // ... because the output room ran out (not a table or the stack)
    uint32_t epoch;   // global word-table epoch (carried from one Proc to the next)
    uint32_t lepoch;  // LDS word-table epoch
    int n_aligned_calls, n_shifts, n_gaps, n_fast;
    // Segment of a split job (similar_aligner.hip, "Long jobs"): the top-level
    // walk stops when its state (every row's pos) equals one of the sync
    // states tg[t*n + row], t in [tm, tK) -- process_cols is memoryless in
    // pos, so the walk from that state on is the next segment's.
    const int* tg;
    int tK, tm;      // targets, the next one tested (wave-uniform)
    int tv;          // this row's position in target tm (relative to the view)
    int tbase;       // this row's view start in the full row (targets are full-row positions)
    bool chk;        // the top-level frame is running: test the targets
    bool stop;       // a target was reached (pos == target tm)
#ifdef NPGX_SA_PROFILE
    // fast_run, equal/mismatch steps, try_gap, try_aligned, vector words,
    // vector compares, chunks, calls, append_end, child return (reverse)
    long long prof[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#endif

    __device__ __forceinline__ ProcT(const WaveCtx& w_, const Params& P_, const Slot& S_, char* ob_, int cap_,
                                    uint32_t ep, uint32_t lep)
        : w(w_), P(P_), S(S_), ob(ob_), cap(cap_), pos(0), col(0), ovf(false), rovf(false), epoch(ep), lepoch(lep),
          n_aligned_calls(0), n_shifts(0), n_gaps(0), n_fast(0), tg(nullptr), tK(0), tm(0), tv(0), tbase(0),
          chk(false), stop(false) {}

    // targets t in [t0, tK) of a segment (row-major, n per target; positions
    // in the full rows, the view of this row starting at `base`)
    __device__ __forceinline__ void set_targets(const int* targets, int t0, int nt, int base) {
        tg = targets;
        tm = t0;
        tK = nt;
        tbase = base;
        tv = (tm < tK && w.act) ? tg[tm * w.n + w.lane] - tbase : 0;
    }

    // Every row advances by c columns from pos (states pos, pos+1, .., pos+c):
    // the d with pos + d == target tm, or -1.  A target some row has passed
    // can no longer be reached (pos only grows): the next one is tested.
    __device__ __forceinline__ int target_hit(int c) {
        while (tm < tK) {
            const int d = w.act ? tv - pos : 0;
            if (any_lane(w, d < 0)) {
                tm++;
                if (tm < tK && w.act) tv = tg[tm * w.n + w.lane] - tbase;
                continue;
            }
            const int d0 = __builtin_amdgcn_readlane(d, 0);
            if (d0 <= c && all_eq(w, d)) return d0;
            return -1;
        }
        return -1;
    }

    __device__ __forceinline__ void put(int c, char x) {
        if (c < cap) ob[(size_t)w.lane * cap + c] = x;
        else ovf = rovf = true;
    }
    __device__ __forceinline__ int ch(int q) const { return vch(v, q, w.lane); }
    __device__ __forceinline__ bool is_stop(int shift) const { return any_lane(w, pos + shift >= v.len); }

    // append_cols :67-77 (rows mode, a few columns)
    __device__ __forceinline__ void append_cols(int cols) {
        if (w.act)
            for (int j = 0; j < cols; j++) put(col + j, (char)ch(pos + j));
        if (chk) {
            const int d = target_hit(cols);
            if (d >= 0) {  // the columns past the target are not kept
                pos += w.act ? d : 0;
                col += d;
                stop = true;
                return;
            }
        }
        pos += w.act ? cols : 0;
        col += cols;
    }

    // every row's [pos, pos+t) then '-' up to m columns (columns mode);
    // append_gaps :79-89 is the padding.  Advances pos by t and col by m.
    __device__ __forceinline__ void write_tails(int t, int m) {
        if (col + m > cap) {
            ovf = rovf = true;
            return;
        }
        __syncthreads();
        for (int r = 0; r < w.n; r++) {
            const char* pr = bcast_ptr(v.p, r);
            const int dr = bcast(v.d, r), qr = bcast(pos, r), tr = bcast(t, r);
            char* o = ob + (size_t)r * cap + col;
            for (int j = w.lane; j < m; j += 64) o[j] = j < tr ? pr[(ptrdiff_t)dr * (qr + j)] : '-';
        }
        __syncthreads();
        pos += w.act ? t : 0;
        col += m;
    }
    // append_all :91-99
    __device__ __forceinline__ void append_all() {
        int t = w.act ? v.len - pos : 0;
        if (t < 0) t = 0;
        write_tails(t, wave_max(t));
    }

    // Columns mode: consume the columns process_cols takes with is_equal /
    // try_mismatch.  Returns 0: the next column needs a rows-mode step,
    // 1: a row ended (is_stop(0) -> append_all), 2: a segment target reached.
    __device__ __forceinline__ int fast_run() {
        __syncthreads();
        while (true) {
            if (col + 64 > cap) return 0;  // near capacity: rows mode guards the writes
            unsigned long long em, vm;
            {
                const int j = w.lane;
                const char* p0 = bcast_ptr(v.p, 0);
                const int d0 = bcast(v.d, 0), l0 = bcast(v.len, 0), q0 = bcast(pos, 0);
                bool valid = q0 + j < l0;
                const char c0 = valid ? p0[(ptrdiff_t)d0 * (q0 + j)] : 0;
                ob[col + j] = c0;  // speculative: columns past the consumed ones are rewritten later
                bool eq = true;
                // FR rows' loads in flight before their stores: a store the
                // compiler cannot prove apart from the next row's load would
                // otherwise hold every load back a full latency (the rows never
                // alias the output: they are the job's input, a stage or C)
                for (int r0 = 1; r0 < w.n; r0 += FR) {
                    char cb[FR];
#pragma unroll
                    for (int u = 0; u < FR; u++) {
                        const int r = r0 + u;
                        cb[u] = 0;
                        if (r < w.n) {
                            const char* pr = bcast_ptr(v.p, r);
                            const int dr = bcast(v.d, r), lr = bcast(v.len, r), qr = bcast(pos, r);
                            const bool vr = qr + j < lr;
                            cb[u] = vr ? pr[(ptrdiff_t)dr * (qr + j)] : 0;
                            valid &= vr;
                        }
                    }
#pragma unroll
                    for (int u = 0; u < FR; u++) {
                        const int r = r0 + u;
                        if (r < w.n) {
                            ob[(size_t)r * cap + col + j] = cb[u];
                            eq &= cb[u] == c0;
                        }
                    }
                }
                vm = ballot(valid);
                em = ballot(valid && eq);
            }
            n_fast++;
            int k = 0;
            int ret = -1;  // -1: chunk consumed / restart, 0: rows step, 1: stop
            while (true) {
                const unsigned long long m = k == 0 ? em : ((em >> k) | (~0ull << (64 - k)));
                k += ctz_ones(m);
                if (k >= 64) {
                    k = 64;
                    break;
                }
                if (!((vm >> k) & 1ull)) {  // a row ends at column k
                    ret = 1;
                    break;
                }
                if (k + P.mc < 64) {  // try_mismatch: columns k+1..k+mc equal
                    const unsigned long long need =
                        P.mc == 0 ? 0ull : (((1ull << P.mc) - 1ull) << (k + 1));
                    if ((em & need) == need) {
                        k += P.mc + 1;
                        if (k >= 64) {
                            k = 64;
                            break;
                        }
                        continue;
                    }
                    ret = 0;
                    break;
                }
                break;  // the mismatch window crosses the chunk: restart the chunk at k
            }
            if (chk) {  // (the consumed columns advance every row by one)
                const int d = target_hit(k);
                if (d >= 0) {
                    pos += w.act ? d : 0;
                    col += d;
                    stop = true;
                    __syncthreads();
                    return 2;
                }
            }
            pos += w.act ? k : 0;
            col += k;
            if (ret >= 0) {
                __syncthreads();
                return ret;
            }
            if (k == 0) {
                __syncthreads();
                return 0;
            }
        }
    }

    // is_equal(pos + off, shift, cols), off = 1 for lanes in `shifted`
    __device__ __forceinline__ bool is_equal_sh(unsigned long long shifted, int shift, int cols) const {
        const int base = pos + (int)((shifted >> w.lane) & 1ull) + shift;
        for (int j = 0; j < cols; j++)
            if (!all_eq(w, ch(base + j))) return false;
        return true;
    }
    // apply_gap :165-174
    __device__ __forceinline__ void apply_gap(unsigned long long shifted, int g) {
        const bool s = w.act && ((shifted >> w.lane) & 1ull);
        if (w.act) put(col, s ? (char)ch(pos) : '-');
        pos += s ? 1 : 0;
        col += 1;  // at least one row is shifted (else the column was equal)
        append_cols(g);
    }
    // try_gap :219-235 + find_all_gaps :176-189 + find_best_gap :191-217.
    // Variant k belongs to letter k of the std::set<char> order A < C < G < N < T;
    // `alive` keeps that order (front() = lowest alive letter).
    __device__ __forceinline__ bool try_gap() {
        if (is_stop(P.gc)) return false;
        n_gaps++;
        const int c_here = ch(pos), c_next = ch(pos + 1);
        unsigned long long v0 = 0, v1 = 0, v2 = 0, v3 = 0, v4 = 0;
        int alive = 0;
#pragma unroll
        for (int k = 0; k < 5; k++) {
            const int c = k == 0 ? 'A' : k == 1 ? 'C' : k == 2 ? 'G' : k == 3 ? 'N' : 'T';
            if (!any_lane(w, c_here == c)) continue;
            const bool mt = c_here == c, mn = c_next == c;
            if (any_lane(w, mt == mn)) continue;
            const unsigned long long sh = ballot(w.act && mn) & w.rowmask;
            if (!is_equal_sh(sh, 0, P.gc)) continue;
            alive |= 1 << k;
            if (k == 0) v0 = sh;
            else if (k == 1) v1 = sh;
            else if (k == 2) v2 = sh;
            else if (k == 3) v3 = sh;
            else v4 = sh;
        }
        if (!alive) return false;
        auto var = [&](int k) { return k == 0 ? v0 : k == 1 ? v1 : k == 2 ? v2 : k == 3 ? v3 : v4; };
        if (__popc(alive) == 1) {
            apply_gap(var(__ffs(alive) - 1), P.gc);
            return true;
        }
        for (int g = P.gc + 1;; g++) {
            int next = 0;
#pragma unroll
            for (int k = 0; k < 5; k++)
                if ((alive >> k) & 1)
                    if (is_equal_sh(var(k), g - 1, 1)) next |= 1 << k;  // columns < g-1 known equal
            if (!next) {
                apply_gap(var(__ffs(alive) - 1), g - 1);
                return true;
            }
            if (__popc(next) == 1) {
                apply_gap(var(__ffs(next) - 1), g);
                return true;
            }
            alive = next;
        }
    }

    __device__ static __forceinline__ unsigned long long code3(int c) {
        return c == 'A' ? 1 : c == 'C' ? 2 : c == 'G' ? 3 : c == 'N' ? 4 : c == 'T' ? 5 : 6;
    }

    // try_aligned :295-308 + find_best_word :246-272.  The word table lives in
    // LDS; a call that inserts more than half of its entries is re-run on the
    // global table (same result, the table only records first sightings).
    __device__ __forceinline__ bool try_aligned(int& my_shift) {
        const int mt = wave_min(w.act ? v.len - pos : 0x7fffffff);
        const int max_shift = mt - P.ac;
        if (max_shift <= 0) return false;
        n_aligned_calls++;
        // the first P.lh shifts incrementally (most searches end there), then
        // whole prefixes (find_word_long)
        const bool lng = LONG && P.lh > 0 && w.n >= 2 && max_shift > P.lh;
        const int head = lng ? P.lh : max_shift;
        if (w.n <= VEC_ROWS) {
            const VecOut r = find_word_vec(v.p, v.len, v.d, pos, w.lane, w.n, P.ac, head, S.lwords, S.tkeys,
                                           S.tmask, S.tcap_log2, epoch);
            epoch = r.epoch;
            n_shifts += r.shifts;
#ifdef NPGX_SA_PROFILE
            prof[4] += r.t_words;
            prof[5] += r.t_cmp;
            prof[6] += r.chunks;
            prof[7] += 1;
#endif
            if (r.found > 0) my_shift = r.my_shift;
            if (r.found < 0) table_full();
            if (r.found != 0 || !lng) return r.found > 0;
        } else {
            const int r = find_word<LdsU64, LdsU32>(my_shift, head, (LdsU64*)S.lkeys, (LdsU64*)S.lmask,
                                                    (LdsU32*)S.ldone, S.ltab_log2, lepoch, 1 << (S.ltab_log2 - 1));
            if (r == 1 || (r == 0 && !lng)) return r == 1;
            if (r < 0) {
                const int g = find_word<unsigned long long, uint32_t>(my_shift, head, S.tkeys, S.tmask, S.tdone,
                                                                      S.tcap_log2, epoch, (1 << (S.tcap_log2 - 1)) - 64);
                if (g < 0) table_full();
                if (g != 0 || !lng) return g == 1;
            }
        }
        LongOut L;
        L.found = -1;
        L.M = P.lm;
        if (P.llds && S.ltab_log2 > 0 && 2u * (uint32_t)min(max(P.lm, LW_STEP), max_shift) <= (1u << S.ltab_log2)) {
            // the first prefixes in the LDS word table
            L = find_word_long<LdsU64>(v.p, v.len, v.d, pos, w.lane, w.n, P.ac, max_shift, P.lm, S.lwords,
                                       (LdsU64*)S.lkeys, (LdsU64*)S.lmask, S.ltab_log2, lepoch);
            lepoch = L.epoch;
        }
        if (L.found == -1) {  // (the LDS table took none, or not the prefix L.M)
            L = find_word_long<unsigned long long>(v.p, v.len, v.d, pos, w.lane, w.n, P.ac, max_shift, L.M, S.lwords,
                                                   S.tkeys, S.tmask, S.tcap_log2, epoch);
            epoch = L.epoch;
        }
        n_shifts += L.shifts - head;
        if (L.found > 0) my_shift = L.my_shift;
        if (L.found >= 0) return L.found > 0;
        // a prefix the table cannot take: every shift incrementally
        const int g = find_word<unsigned long long, uint32_t>(my_shift, max_shift, S.tkeys, S.tmask, S.tdone,
                                                              S.tcap_log2, epoch, (1 << (S.tcap_log2 - 1)) - 64);
        if (g < 0) table_full();
        return g == 1;
    }

    // The slot's global word table cannot take this call's words (the host
    // sized it below the job's bound): the walk ends here and the job is
    // reported as overflowed, to be re-run with a table of the full bound.
    __device__ __forceinline__ void table_full() {
        ovf = true;
        stop = true;
    }

    // 1: found (my_shift set), 0: no shift works, -1: more than `limit` inserts
    // T = unsigned long long (global table) or LdsU64 (the LDS table: ds_* atomics)
    // Rows in parallel, J = 64/n shifts per step: lane = j*n + r holds row r's
    // word at shift s0+j.  Per word the table keeps the rows that have had it
    // (mask) and the largest first-sighting shift (done): at shift s the word
    // is complete iff mask is full and done <= s, which is what the reference
    // sees after inserting the words of shifts 0..s.  A row's first sighting
    // within a step is its lowest j with the word (shuffle compares).
    template <class T, class U>
    __device__ __forceinline__ int find_word(int& my_shift, int max_shift, T* tkeys, T* tmask, U* tdone,
                                             uint32_t tlog, uint32_t& ep_ref, int limit) {
        uint32_t ep32 = ep_ref + 1;
        const uint32_t tcap = 1u << tlog;
        if (ep32 >= 0xFFFF) {  // epoch wrap: clear the table
            for (uint32_t i = w.lane; i < tcap; i += 64) {
                tkeys[i] = 0ull;
                tmask[i] = 0ull;
            }
            __threadfence();
            ep32 = 1;
        }
        ep_ref = ep32;
        const unsigned long long ep = (unsigned long long)ep32 << 48;
        const int ac = P.ac;
        const unsigned long long wmask = (ac >= 16) ? ((1ull << 48) - 1) : ((1ull << (3 * ac)) - 1);
        const int n = w.n;
        // a step inserts up to 64 keys: keep them well inside the table
        const int J = tcap >= 256 ? 64 / n : 1;
        const int r = w.lane % n, j = w.lane / n;
        const bool act = j < J;
        const View vr{shfl_ptr(v.p, r), __shfl(v.len, r), __shfl(v.d, r)};
        const int pr = __shfl(pos, r);
        // this call's words of the first `hist` shifts, [shift][row] in LDS:
        // the first sighting of the chosen word is then a scan of LDS
        LdsU64* hw = (LdsU64*)S.lwords;
        const int hist = S.hist_cap > 0 ? S.hist_cap * 64 / n : 0;
        unsigned long long word = 0;
        int nxt = pr + j + ac - 1;  // next char of this lane's word
        if (act) {
            int c[15];
#pragma unroll
            for (int t = 0; t < 15; t++) c[t] = t < ac - 1 ? vch(vr, pr + j + t, r) : 0;  // independent loads
#pragma unroll
            for (int t = 0; t < 15; t++)
                if (t < ac - 1) word = (word << 3) | code3(c[t]);
        }
        int inserted = 0;
        // the chars a step adds are loaded one step ahead: the table atomics
        // between steps would otherwise keep every step waiting on its loads
        int cn[8];
#pragma unroll
        for (int t = 0; t < 8; t++) cn[t] = (act && t < 1) ? vch(vr, nxt + t, r) : 0;
        for (int s0 = 0; s0 < max_shift; s0 += J) {
            const int s = s0 + j;
            const bool valid = act && s < max_shift;
            const int add = s0 == 0 ? 1 : J;  // chars entering this lane's word
            if (act) {
#pragma unroll
                for (int t = 0; t < 8; t++)
                    if (t < add) word = (word << 3) | code3(cn[t]);
                word &= wmask;
                for (int t = 8; t < add; t++) word = ((word << 3) | code3(vch(vr, nxt + t, r))) & wmask;
                nxt += add;
                if (s0 + J < max_shift) {
#pragma unroll
                    for (int t = 0; t < 8; t++) cn[t] = t < J ? vch(vr, nxt + t, r) : 0;
                }
            }
            if (valid && s < hist) hw[s * n + r] = word;
            // every lane inserts its word: claim (or find) the key, reset the
            // row mask and done of a new key, then record first sightings
            const unsigned long long key = ep | word;
            uint32_t slot = 0;
            bool claimed = false;
            if (valid) {
                slot = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - tlog));
                while (true) {
                    unsigned long long k = __hip_atomic_load(&tkeys[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (k == key) break;
                    if ((k & ~((1ull << 48) - 1)) != ep) {  // stale or empty: claim
                        if (__hip_atomic_compare_exchange_strong(&tkeys[slot], &k, key, __ATOMIC_RELAXED,
                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                            claimed = true;
                            break;
                        }
                        if (k == key) break;  // another lane claimed the same word
                        continue;
                    }
                    slot = (slot + 1) & (tcap - 1);
                }
            }
            if (claimed) {
                __hip_atomic_store(&tmask[slot], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&tdone[slot], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            bool first = valid;  // the row's lowest j with this word in this step
            for (int jj = 1; jj < J; jj++) {
                const unsigned long long o = shfl64(word, max(w.lane - jj * n, 0));
                if (jj <= j && o == word) first = false;
            }
            __syncthreads();
            if (first) {
                const unsigned long long old =
                    __hip_atomic_fetch_or(&tmask[slot], 1ull << r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (!((old >> r) & 1ull))
                    __hip_atomic_fetch_max(&tdone[slot], (uint32_t)s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __syncthreads();
            bool complete = false;
            if (valid)
                complete = __hip_atomic_load(&tmask[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == w.rowmask &&
                           (int)__hip_atomic_load(&tdone[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= s;
            inserted += __popcll(ballot(claimed));
            const unsigned long long cm = ballot(complete);
            n_shifts += min(J, max_shift - s0);
            if (cm) {
                // the first complete shift (lowest j), its highest complete row names the word
                const int jm = (__ffsll((long long)cm) - 1) / n;
                const unsigned long long rows = (cm >> (jm * n)) & w.rowmask;
                const int rb = 63 - __clzll((long long)rows);
                const unsigned long long best = bcast64(word, jm * n + rb);
                const int sb = s0 + jm;
                const unsigned long long same = ballot(act && j == jm && word == bcast64(word, jm * n));
                if (((same >> (jm * n)) & w.rowmask) == w.rowmask) {  // words.size() == 1
                    my_shift = sb;
                } else {
                    my_shift = -1;
                    if (sb < hist) {
                        if (w.act)
                            for (int t = 0; t <= sb; t++)
                                if (hw[t * n + w.lane] == best) {
                                    my_shift = t;
                                    break;
                                }
                    } else {
                        // rescan the rows J shifts per step in the same lane layout
                        unsigned long long x = 0;
                        if (act)
                            for (int q = 0; q < ac - 1; q++) x = (x << 3) | code3(vch(vr, pr + j + q, r));
                        int at = pr + j + ac - 1, fs = -1;
                        unsigned long long found = 0;  // rows with a first sighting
                        for (int t0 = 0; t0 <= sb && (found & w.rowmask) != w.rowmask; t0 += J) {
                            const int add = t0 == 0 ? 1 : J;
                            if (act)
                                for (int t = 0; t < add; t++) x = ((x << 3) | code3(vch(vr, at + t, r))) & wmask;
                            at += add;
                            const bool hit = act && t0 + j <= sb && x == best;
                            const unsigned long long hm = ballot(hit);
                            // lowest j of each row not found before
                            if (hit && fs < 0 && !((found >> r) & 1ull)) {
                                bool lowest = true;
                                for (int jj = 1; jj <= j; jj++) lowest &= !((hm >> (w.lane - jj * n)) & 1ull);
                                if (lowest) fs = t0 + j;
                            }
                            for (int q = 0; q < J; q++) found |= (hm >> (q * n)) & w.rowmask;
                        }
                        // lane r of the Proc layout takes row r's shift from lane (r, j)
                        int got = -1;
                        for (int q = 0; q < J; q++) {
                            const int o = __shfl(fs, q * n + (w.lane < n ? w.lane : 0));
                            if (got < 0 && o >= 0) got = o;
                        }
                        if (w.act) my_shift = got;
                    }
                }
                return 1;
            }
            if (inserted > limit) return -1;
        }
        return 0;
    }

    // append_end :323-342 -- the end walk tests 63 end offsets per pass.
    // Offset t from the row ends: E(t) = column len_i-1-t identical over rows,
    // V(t) = every pos_i < len_i-1-t; walk while (V&&E)(t) || (V&&E)(t+1).
    __device__ __forceinline__ void append_end() {
        int t = 0;
        while (true) {
            const int j = w.lane;
            const char* p0 = bcast_ptr(v.p, 0);
            const int d0 = bcast(v.d, 0), q0 = bcast(pos, 0), l0 = bcast(v.len, 0);
            const int cp0 = l0 - 1 - (t + j);
            const int c0 = cp0 >= 0 ? (unsigned char)p0[(ptrdiff_t)d0 * cp0] : -1;
            bool E = true, V = q0 < cp0;
            for (int r = 1; r < w.n; r++) {
                const char* pr = bcast_ptr(v.p, r);
                const int dr = bcast(v.d, r), lr = bcast(v.len, r), qr = bcast(pos, r);
                const int cp = lr - 1 - (t + j);
                const int c = cp >= 0 ? (unsigned char)pr[(ptrdiff_t)dr * cp] : -2;
                E &= c == c0;
                V &= qr < cp;
            }
            const unsigned long long a = ballot(E && V);
            const unsigned long long cond = (a | (a >> 1)) | (1ull << 63);  // bit 63 needs the next chunk
            const int run = ctz_ones(cond);
            if (run < 63) {
                t += run;
                break;
            }
            t += 63;
        }
        int cols = w.act ? (v.len - 1 - t) - pos : 0;
        if (cols < 0) cols = 0;
        write_tails(cols, wave_max(cols));  // append_chars to end_pos, append_gaps
        append_all();
    }

    // One step of process_cols (SimilarAligner.cpp:351-368): a columns-mode run,
    // then one rows-mode step.  Returns 0 = keep stepping, 1 = frame finished,
    // 2 = descend into a child (sh = this row's shift); a segment target
    // reached (stop) shows as 0 or 1.
    __device__ __forceinline__ int step(int& sh) {
        SA_T0(t0);
        const int fr = fast_run();
        SA_ACC(0, t0);
        if (fr == 2) return 1;
        if (fr == 1) {
            append_all();  // is_stop(0)
            return 1;
        }
        if (is_stop(0)) {
            append_all();
            return 1;
        }
        SA_T0(t1);
        if (all_eq(w, ch(pos))) {
            append_cols(1);
            SA_ACC(1, t1);
            return 0;
        }
        if (!is_stop(P.mc) && is_equal_sh(0ull, 1, P.mc)) {  // try_mismatch
            append_cols(P.mc + 1);
            SA_ACC(1, t1);
            return 0;
        }
        SA_ACC(1, t1);
        SA_T0(t2);
        const bool gap = try_gap();
        SA_ACC(2, t2);
        if (gap) return 0;
        sh = 0;
        SA_T0(t3);
        const bool al = try_aligned(sh);
        SA_ACC(3, t3);
        if (stop) return 1;  // table_full
        if (al) {
            if (!any_lane(w, sh > 0)) {  // every prefix empty: the child adds nothing
                append_cols(P.ac);
                return 0;
            }
            return 2;
        }
        SA_T0(t4);
        append_end();
        SA_ACC(8, t4);
        return 1;
    }

    // process_seqs on view v0 from output column col0; returns the length.
    __device__ __forceinline__ int run(const View& v0, int col0) {
        v = v0;
        pos = 0;
        col = col0;
        int depth = 0;
        bool fresh = true;
        stop = false;
        chk = tm < tK;
        while (true) {
            int r;
            if (fresh && any_lane(w, v.len == 0)) {  // process_cols :345-350
                append_all();
                r = 1;
            } else {
                int sh = 0;
                r = step(sh);
                if (stop) return col - col0;  // (depth 0: only the top-level frame tests targets)
                if (r == 2) {
                    chk = false;
                    if (depth >= S.st_depth_max) {  // excluded by the host's sizing
                        ovf = true;
                        return col - col0;
                    }
                    const size_t o = (size_t)depth * 64 + w.lane;
                    S.st_p[o] = v.p;
                    S.st_len[o] = v.len | (v.d < 0 ? (int)0x80000000 : 0);
                    S.st_pos[o] = pos;
                    if (w.lane == 0) S.st_col[depth] = col;
                    depth++;
                    View c;  // reversed prefixes [pos, pos+sh) (append_aligned :274-293)
                    c.p = v.p + (ptrdiff_t)v.d * (pos + sh - 1);
                    c.d = -v.d;
                    c.len = w.act ? sh : 0;
                    v = c;
                    pos = 0;
                    fresh = true;
                    continue;
                }
            }
            fresh = false;
            if (r == 0) continue;
            if (depth == 0) return col - col0;
            SA_T0(t5);
            depth--;
            const int child_len = v.len;  // = this row's shift in the parent
            const size_t o = (size_t)depth * 64 + w.lane;
            const int c0 = bcast(S.st_col[depth], 0);
            v.p = S.st_p[o];
            const int l = S.st_len[o];
            v.len = l & 0x7fffffff;
            v.d = (l & (int)0x80000000) ? -1 : 1;
            pos = S.st_pos[o];
            if (col > cap) {
                ovf = rovf = true;
            } else {
                __syncthreads();
                cm_reverse(w, ob, cap, c0, col);
            }
            pos += w.act ? child_len : 0;
            chk = depth == 0 && tm < tK;
            append_cols(P.ac);
            SA_ACC(9, t5);
            if (stop) return col - col0;
        }
    }
};

}  // namespace sa
}  // namespace npgx
