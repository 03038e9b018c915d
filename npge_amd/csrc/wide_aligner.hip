// wide_aligner.hip -- align_seqs (aligner-type "similar" or "dummy") for
// alignment problems of more than 64 non-empty rows: repeat families and the
// consensus blocks of AnchorLoopFast, which the reference aligns like any other
// block (SimilarAligner.cpp:41-501, AbstractAligner.cpp:104-143).
//
// The batched aligner (similar_aligner.hip) puts one row on each lane of a
// wave; a wider problem gets one 256-thread workgroup here, rows dealt out
// over the threads (row i on thread i mod 256), every decision of the
// reference's column loop taken by a workgroup vote (barrier and/or/min/max).
// Such jobs are rare (RemoveNonStem keeps DraftPangenome's blocks at one
// fragment per genome), so this path is written for exactness first:
//   * process_seqs (:344-369) is one step machine over an explicit stack of
//     frames: append_aligned (:274-293) pushes the reversed prefixes as a
//     child frame and, when it ends, the child's rows are appended reversed;
//   * a frame's rows are views (base, start, length, direction) into the batch
//     rows or into gap-filtered copies, so reversing is free;
//   * try_aligned's "first shift at which each row saw a word" (:246-272) is a
//     pair table (word, row) plus a word table counting the rows that saw the
//     word, both global open-addressing tables cleared through their used lists;
//   * fix_bad_regions (:428-459, FindLowSimilar.cpp:62-130) and realing_end
//     (:461-484) re-run the step machine on gap-filtered reversed copies;
//   * remove_gaps (AbstractAligner.cpp:89-102) compacts the columns into the
//     job's output (row r at out + r * cap).
// Past-the-end reads follow the oracle's documented convention (position len
// reads 0, later positions 0x100 + row), as the batched aligner does.
// A job whose output, arena or tables outgrow their first sizes is re-run
// with larger ones (status 1); a frame stack deeper than DMAX or more than
// MAXV gap variants is refused (NPGX_ERR_RANGE).
#include <chrono>
#include <cstring>

#include <deque>

#include "common.hpp"

namespace npgx {
namespace wide {

constexpr int WT = 256;    // threads per job
constexpr int DMAX = 96;   // frames (nested process_seqs calls)
constexpr int MAXV = 8;    // gap variants (distinct letters at the cursor)
constexpr unsigned long long EMPTY = ~0ull;

struct RowV {              // a frame's row: a view of [start, start + len) of base
    const char* base;
    int32_t start, len, pos, pad;
};

struct WJob {
    int64_t row0;          // first entry in row_off / row_len (non-empty rows)
    int64_t out;           // byte offset of the n x cap output
    int64_t arena;         // byte offset of the job's arena
    int64_t arena_bytes;
    int64_t tab;           // first entry of the job's pair / word tables (tcap = 1 << tlog2 each)
    int32_t n, cap;
    uint32_t tlog2, pad;
};

struct WArgs {
    const char* rows;
    const int64_t* row_off;
    const int32_t* row_len;
    const WJob* jobs;
    unsigned char* out;
    unsigned char* arena;
    unsigned long long* pt;   // pair table (word << 16 | row), tcap per job
    unsigned long long* wk;   // word table keys, tcap per job
    uint32_t* wc;             // word table counts
    uint32_t* used;           // used lists: pairs then words, tcap/2 each per job
    int32_t* len_out;
    int32_t* status;          // 0 ok, 1 re-run larger, 2 refused
    int mc, gc, ac, min_length, wf, aligner_type;
    int lh, lm;               // try_aligned: incremental shifts before the prefix search (0: never), its first prefix
};

struct Frame {
    char* out;
    RowV* rv;
    int64_t save_top;
    int32_t cap, col, dir, pad;
};

struct Ctx {
    Frame fr[DMAX];
    unsigned long long best;
    unsigned long long r64;
    int r32;
    int abort;
    uint32_t n_pu, n_wu;      // used-list lengths
    uint32_t chars[8];
    int live[MAXV];
    int nlive;
    int head;
};

__device__ __forceinline__ int lds_min(Ctx& C, int v) {
    __syncthreads();
    if (threadIdx.x == 0) C.r32 = 0x7fffffff;
    __syncthreads();
    atomicMin(&C.r32, v);
    __syncthreads();
    return C.r32;
}
__device__ __forceinline__ int lds_max(Ctx& C, int v) {
    __syncthreads();
    if (threadIdx.x == 0) C.r32 = -0x7fffffff;
    __syncthreads();
    atomicMax(&C.r32, v);
    __syncthreads();
    return C.r32;
}
__device__ __forceinline__ long long lds_sum(Ctx& C, long long v) {
    __syncthreads();
    if (threadIdx.x == 0) C.r64 = 0;
    __syncthreads();
    if (v) atomicAdd(&C.r64, (unsigned long long)v);
    __syncthreads();
    return (long long)C.r64;
}
__device__ __forceinline__ unsigned long long lds_min64(Ctx& C, unsigned long long v) {
    __syncthreads();
    if (threadIdx.x == 0) C.r64 = ~0ull;
    __syncthreads();
    atomicMin(&C.r64, v);
    __syncthreads();
    return C.r64;
}

__device__ __forceinline__ unsigned long long aload(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t aload(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the view's letter at p (p < len)
__device__ __forceinline__ char raw(const RowV& v, int dir, int p) {
    if (p < 0 || p >= v.len) return 0;
    return v.base[dir ? v.start + v.len - 1 - p : v.start + p];
}
// SimilarAligner's character read with the past-the-end convention
__device__ __forceinline__ int at(const RowV& v, int dir, int i, int p) {
    if (p < v.len) return p < 0 ? -1 : (unsigned char)v.base[dir ? v.start + v.len - 1 - p : v.start + p];
    if (p == v.len) return 0;
    return 0x100 + i;
}
// aligned_check letters from p, 3 bits each (A 1, C 3, T 4, N 6, G 7)
__device__ __forceinline__ unsigned long long word_at(const RowV& v, int dir, int p, int ac) {
    unsigned long long w = 0;
    for (int j = 0; j < ac; j++) w = (w << 3) | (unsigned long long)(raw(v, dir, p + j) & 7);
    return w;
}
__device__ __forceinline__ uint32_t slot_of(unsigned long long k, uint32_t log2) {
    return (uint32_t)((k * 0x9E3779B97F4A7C15ull) >> (64 - log2));
}

struct Job {
    WArgs a;
    Ctx* C;
    int n;
    unsigned char* arena;
    int64_t top, lim;
    unsigned char* var;       // MAXV x n gap-variant offsets (0: pos, 1: pos + 1)
    unsigned long long *pt, *wk;
    uint32_t *wc, *pu, *wu;
    uint32_t tcap, tlog2;

    // bump allocation from the arena (uniform: every thread computes the same)
    __device__ unsigned char* alloc(int64_t bytes) {
        bytes = (bytes + 255) & ~255ll;
        if (top + bytes > lim) {
            if (threadIdx.x == 0) C->abort = 1;
            return nullptr;
        }
        unsigned char* p = arena + top;
        top += bytes;
        return p;
    }
    __device__ bool failed() {
        __syncthreads();
        return C->abort != 0;
    }
    __device__ void fail(int code) {  // uniform caller
        if (threadIdx.x == 0) C->abort = max(C->abort, code);
        __syncthreads();
    }

    // ---- column operations on frame F (col: its output cursor, uniform)
    __device__ bool room(const Frame& F, int col, int64_t k) {
        if ((int64_t)col + k <= F.cap) return true;
        fail(1);
        return false;
    }
    __device__ void append_cols(Frame& F, int& col, int k) {  // :67-77
        if (!room(F, col, k)) return;
        for (int i = threadIdx.x; i < n; i += WT) {
            RowV v = F.rv[i];
            char* o = F.out + (int64_t)i * F.cap + col;
            for (int j = 0; j < k; j++) o[j] = raw(v, F.dir, v.pos + j);
            F.rv[i].pos = v.pos + k;
        }
        col += k;
    }
    // each row appends its remaining letters (up to `to` = len) then gaps to
    // the widest: append_chars / append_all + append_gaps (:79-99, :136-143)
    __device__ void append_upto(Frame& F, int& col, int back) {
        int w = 0;
        for (int i = threadIdx.x; i < n; i += WT) {
            const RowV v = F.rv[i];
            w = max(w, v.len - back - v.pos);
        }
        w = lds_max(*C, w);
        if (w <= 0) return;
        if (!room(F, col, w)) return;
        for (int i = threadIdx.x; i < n; i += WT) {
            RowV v = F.rv[i];
            const int e = v.len - back;
            char* o = F.out + (int64_t)i * F.cap + col;
            int j = 0;
            for (; v.pos + j < e; j++) o[j] = raw(v, F.dir, v.pos + j);
            for (int q = j; q < w; q++) o[q] = '-';
            F.rv[i].pos = e;
        }
        col += w;
    }
    // consecutive columns from the cursor where every row equals row 0 (<= maxk)
    __device__ int equal_run(const Frame& F, int maxk) {
        const RowV v0 = F.rv[0];
        int r = maxk;
        for (int i = threadIdx.x; i < n; i += WT) {
            const RowV v = F.rv[i];
            int j = 0;
            while (j < r && raw(v, F.dir, v.pos + j) == raw(v0, F.dir, v0.pos + j)) j++;
            r = j;
        }
        return lds_min(*C, r);
    }
    // is_equal over rows at pos + off + var offset, columns [c0, c1) (:101-115)
    __device__ bool cols_equal(const Frame& F, int off, const unsigned char* vr, int c0, int c1) {
        const RowV v0 = F.rv[0];
        const int p0 = v0.pos + off + (vr ? vr[0] : 0);
        bool ok = true;
        for (int i = threadIdx.x; i < n && ok; i += WT) {
            const RowV v = F.rv[i];
            const int p = v.pos + off + (vr ? vr[i] : 0);
            for (int j = c0; j < c1; j++)
                if (at(v, F.dir, i, p + j) != at(v0, F.dir, 0, p0 + j)) {
                    ok = false;
                    break;
                }
        }
        return __syncthreads_and(ok);
    }
    __device__ void apply_gap(Frame& F, int& col, const unsigned char* vr, int g) {  // :165-174
        if (!room(F, col, 1 + (int64_t)g)) return;
        int any = 0;
        for (int i = threadIdx.x; i < n; i += WT) {
            RowV v = F.rv[i];
            char* o = F.out + (int64_t)i * F.cap + col;
            if (vr[i]) {
                *o = raw(v, F.dir, v.pos);
                F.rv[i].pos = v.pos + 1;
                any = 1;
            } else {
                *o = '-';
            }
        }
        if (__syncthreads_or(any)) col += 1;
        append_cols(F, col, g);
    }
    // try_gap (:219-235) with find_all_gaps / find_best_gap (:176-217); tail > gc
    __device__ bool try_gap(Frame& F, int& col) {
        const int gc = a.gc;
        if (threadIdx.x < 8) C->chars[threadIdx.x] = 0;
        __syncthreads();
        for (int i = threadIdx.x; i < n; i += WT) {
            const RowV v = F.rv[i];
            const int c = (unsigned char)raw(v, F.dir, v.pos);
            atomicOr(&C->chars[c >> 5], 1u << (c & 31));
        }
        __syncthreads();
        int nv = 0;
        for (int c = 0; c < 256; c++) {  // std::set<char>: ascending
            if (!((C->chars[c >> 5] >> (c & 31)) & 1)) continue;
            if (nv == MAXV) {
                fail(2);
                return false;
            }
            unsigned char* vr = var + (int64_t)nv * n;
            int bad = 0;
            for (int i = threadIdx.x; i < n; i += WT) {
                const RowV v = F.rv[i];
                const bool mt = at(v, F.dir, i, v.pos) == c, mn = at(v, F.dir, i, v.pos + 1) == c;
                bad |= mt == mn;
                vr[i] = mt ? 0 : 1;
            }
            if (__syncthreads_or(bad)) continue;
            if (cols_equal(F, 0, vr, 0, gc)) nv++;
        }
        if (nv == 0) return false;
        if (nv == 1) {
            apply_gap(F, col, var, gc);
            return true;
        }
        if (threadIdx.x == 0) {
            for (int v = 0; v < nv; v++) C->live[v] = v;
            C->nlive = nv;
        }
        __syncthreads();
        for (int g = gc + 1;; g++) {
            const int nl = C->nlive;
            int keep[MAXV], nk = 0;
            for (int q = 0; q < nl; q++) {
                const int v = C->live[q];
                if (cols_equal(F, 0, var + (int64_t)v * n, g - 1, g)) keep[nk++] = v;
            }
            if (nk == 0) {
                apply_gap(F, col, var + (int64_t)C->live[0] * n, g - 1);
                return true;
            }
            if (nk == 1) {
                apply_gap(F, col, var + (int64_t)keep[0] * n, g);
                return true;
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                for (int q = 0; q < nk; q++) C->live[q] = keep[q];
                C->nlive = nk;
            }
            __syncthreads();
        }
    }

    // ---- try_aligned (:246-308): returns true after pushing the child frame
    __device__ void clear_tables() {
        __syncthreads();
        const uint32_t np = min(C->n_pu, tcap / 2), nw = min(C->n_wu, tcap / 2);
        for (uint32_t q = threadIdx.x; q < np; q += WT) pt[pu[q]] = EMPTY;
        for (uint32_t q = threadIdx.x; q < nw; q += WT) {
            wk[wu[q]] = EMPTY;
            wc[wu[q]] = 0;
            pt[wu[q]] = EMPTY;  // (the prefix search keeps a word's state at its key's slot)
        }
        __threadfence();
        __syncthreads();
        if (threadIdx.x == 0) C->n_pu = C->n_wu = 0;
        __syncthreads();
    }
    __device__ uint32_t word_slot(unsigned long long w, bool insert) {
        const uint32_t lg = tlog2, mask = tcap - 1;
        uint32_t h = slot_of(w, lg);
        while (true) {
            unsigned long long k = aload(wk + h);
            if (k == w) return h;
            if (k == EMPTY) {
                if (!insert) return ~0u;
                k = atomicCAS(wk + h, EMPTY, w);
                if (k == EMPTY) {
                    const uint32_t q = atomicAdd(&C->n_wu, 1u);
                    if (q < tcap / 2) wu[q] = h;
                    return h;
                }
                if (k == w) return h;
            }
            h = (h + 1) & mask;
        }
    }
    __device__ bool pair_insert(unsigned long long key) {  // true: new pair
        const uint32_t mask = tcap - 1;
        uint32_t h = slot_of(key, tlog2);
        while (true) {
            const unsigned long long k = atomicCAS(pt + h, EMPTY, key);
            if (k == EMPTY) {
                const uint32_t q = atomicAdd(&C->n_pu, 1u);
                if (q < tcap / 2) pu[q] = h;
                return true;
            }
            if (k == key) return false;
            h = (h + 1) & mask;
        }
    }
    // try_aligned past the first lh shifts (the batched aligner's
    // find_word_long, sa_device.hpp, for a workgroup): for a prefix [0, M)
    // of shifts, T(w) = the shift at which the last row first sights word w
    // and S* = min T(w) is where the shift-by-shift loop stops.  A complete
    // word is one of row 0's words, so the word table holds row 0's words of
    // the prefix, each with a state at its key's slot in pt packed as
    // (~rows that have sighted it) << 32 | T, lowered by atomicMin (more rows,
    // then the earlier sighting, win).  Rows 1..n-1 pass over the prefix in
    // order, 4 x WT shifts a step, every state read before any of the step's
    // atomics: row k raises only words all of rows 0..k-1 have sighted, at
    // its first sighting.  No complete word: the prefix doubles (from lm) up
    // to max_shift.  At S* the loop's own tests follow (one word in every
    // row; else the word of the highest row complete at S*) and every row's
    // first sighting of it.
    __device__ static unsigned long long pstate(uint32_t rows, uint32_t t) {
        return ((unsigned long long)(0xFFFFFFFFu - rows) << 32) | t;
    }
    __device__ bool prefix_search(Frame& F, int max_shift) {
        const int ac = a.ac;
        bool found = false;
        for (int M = min(max(a.lm, a.lh + 1), max_shift);; M = min(2 * M, max_shift)) {
            if ((uint32_t)M > tcap / 2) {  // row 0's words would not fit: a larger table (status 1)
                fail(1);
                break;
            }
            __syncthreads();
            {
                const RowV v0 = F.rv[0];
                for (int s = threadIdx.x; s < M; s += WT) {
                    const uint32_t h = word_slot(word_at(v0, F.dir, v0.pos + s, ac), true);
                    atomicMin(pt + h, pstate(1, (uint32_t)s));
                }
            }
            __threadfence();
            __syncthreads();
            for (int k = 1; k < n; k++) {
                const RowV v = F.rv[k];
                int raised = 0;  // a row that raises no word ends the pass: none can be complete
                for (int s0 = 0; s0 < M; s0 += 4 * WT) {
                    uint32_t hs[4];
                    unsigned long long nv[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const int s = s0 + u * WT + (int)threadIdx.x;
                        hs[u] = ~0u;
                        if (s < M) {
                            const uint32_t h = word_slot(word_at(v, F.dir, v.pos + s, ac), false);
                            if (h != ~0u) {
                                const unsigned long long st = aload(pt + h);
                                if (0xFFFFFFFFu - (uint32_t)(st >> 32) == (uint32_t)k) {
                                    hs[u] = h;
                                    nv[u] = pstate((uint32_t)k + 1, max((uint32_t)st, (uint32_t)s));
                                }
                            }
                        }
                    }
                    __syncthreads();  // every state of the step read before its atomics
#pragma unroll
                    for (int u = 0; u < 4; u++)
                        if (hs[u] != ~0u) {
                            atomicMin(pt + hs[u], nv[u]);
                            raised = 1;
                        }
                    __threadfence();
                    __syncthreads();
                }
                if (!__syncthreads_or(raised)) break;
            }
            // S*: the smallest T of a word all n rows have sighted
            int tmin = 0x7fffffff;
            {
                const RowV v0 = F.rv[0];
                for (int s = threadIdx.x; s < M; s += WT) {
                    const uint32_t h = word_slot(word_at(v0, F.dir, v0.pos + s, ac), false);
                    const unsigned long long st = h != ~0u ? aload(pt + h) : EMPTY;
                    if (0xFFFFFFFFu - (uint32_t)(st >> 32) == (uint32_t)n) tmin = min(tmin, (int)(uint32_t)st);
                }
            }
            const int S = lds_min(*C, tmin);
            if (S < M) {
                const RowV v0 = F.rv[0];
                const unsigned long long w0 = word_at(v0, F.dir, v0.pos + S, ac);
                bool same = true;
                int cand = -1;
                for (int i = threadIdx.x; i < n; i += WT) {
                    const RowV v = F.rv[i];
                    const unsigned long long w = word_at(v, F.dir, v.pos + S, ac);
                    same &= w == w0;
                    const uint32_t h = word_slot(w, false);
                    const unsigned long long st = h != ~0u ? aload(pt + h) : EMPTY;
                    if (0xFFFFFFFFu - (uint32_t)(st >> 32) == (uint32_t)n && (int)(uint32_t)st <= S) cand = i;
                }
                if (__syncthreads_and(same)) {
                    for (int i = threadIdx.x; i < n; i += WT) F.rv[i].pad = S;
                } else {
                    cand = lds_max(*C, cand);  // (>= 0: the row that sighted S*'s word last holds it at S*)
                    if (threadIdx.x == (unsigned)(cand % WT)) {
                        const RowV v = F.rv[cand];
                        C->best = word_at(v, F.dir, v.pos + S, ac);
                    }
                    __syncthreads();
                    const unsigned long long best = C->best;
                    for (int i = threadIdx.x; i < n; i += WT) {
                        const RowV v = F.rv[i];
                        int s = 0;
                        while (s < S && word_at(v, F.dir, v.pos + s, ac) != best) s++;
                        F.rv[i].pad = s;
                    }
                }
                found = true;
            }
            clear_tables();
            if (found || failed() || M >= max_shift) break;
        }
        __syncthreads();
        return found;
    }

    __device__ bool try_aligned(Frame& F, int tail, int& d, int col) {
        if (failed()) return false;
        const int ac = a.ac;
        const int max_shift = tail - ac;
        if (max_shift <= 0) return false;
        bool found = false;
        int shift = 0;
        // the first lh shifts incrementally (most searches end there), then
        // whole prefixes (prefix_search)
        const bool lng = a.lh > 0 && max_shift > a.lh;
        const int head = lng ? a.lh : max_shift;
        // per shift: the rows' words inserted (the first RPT x WT rows' words
        // kept in registers for the count test), one barrier, the count test
        // with the last completing row's index raised in LDS, one barrier
        constexpr int RPT = 4;
        for (; shift < head; shift++) {
            __syncthreads();
            if (C->n_pu + (uint32_t)n > tcap / 2 || C->n_wu + (uint32_t)n > tcap / 2) {
                fail(1);
                break;
            }
            if (threadIdx.x == 0) C->r32 = -0x7fffffff;
            const RowV v0 = F.rv[0];
            const unsigned long long w0 = word_at(v0, F.dir, v0.pos + shift, ac);
            bool same = true;
            unsigned long long wr[RPT];
#pragma unroll
            for (int u = 0; u < RPT; u++) {
                const int i = (int)threadIdx.x + u * WT;
                wr[u] = 0;
                if (i < n) {
                    const RowV v = F.rv[i];
                    wr[u] = word_at(v, F.dir, v.pos + shift, ac);
                    same &= wr[u] == w0;
                    if (pair_insert((wr[u] << 16) | (unsigned long long)i)) atomicAdd(wc + word_slot(wr[u], true), 1u);
                }
            }
            for (int i = threadIdx.x + RPT * WT; i < n; i += WT) {
                const RowV v = F.rv[i];
                const unsigned long long w = word_at(v, F.dir, v.pos + shift, ac);
                same &= w == w0;
                if (pair_insert((w << 16) | (unsigned long long)i)) atomicAdd(wc + word_slot(w, true), 1u);
            }
            __threadfence();
            __syncthreads();
            int cand = -1;
#pragma unroll
            for (int u = 0; u < RPT; u++) {
                const int i = (int)threadIdx.x + u * WT;
                if (i < n && aload(wc + word_slot(wr[u], false)) == (uint32_t)n) cand = i;
            }
            for (int i = threadIdx.x + RPT * WT; i < n; i += WT) {
                const RowV v = F.rv[i];
                if (aload(wc + word_slot(word_at(v, F.dir, v.pos + shift, ac), false)) == (uint32_t)n) cand = i;
            }
            if (cand >= 0) atomicMax(&C->r32, cand);  // the last row completing a word wins
            if (__syncthreads_and(same)) {  // one word: every row at this shift
                for (int i = threadIdx.x; i < n; i += WT) F.rv[i].pad = shift;
                found = true;
                break;
            }
            cand = C->r32;
            if (cand >= 0) {
                if (threadIdx.x == (unsigned)(cand % WT)) {
                    const RowV v = F.rv[cand];
                    C->best = word_at(v, F.dir, v.pos + shift, ac);
                }
                __syncthreads();
                const unsigned long long best = C->best;
                for (int i = threadIdx.x; i < n; i += WT) {
                    const RowV v = F.rv[i];
                    int s = 0;
                    while (s < shift && word_at(v, F.dir, v.pos + s, ac) != best) s++;
                    F.rv[i].pad = s;
                }
                found = true;
                break;
            }
        }
        clear_tables();
        if (!found && lng && !failed()) found = prefix_search(F, max_shift);
        if (!found || failed()) return false;
        // append_aligned: the reversed prefixes [pos, pos + shift_i) as a child frame
        long long sum = 0;
        for (int i = threadIdx.x; i < n; i += WT) sum += F.rv[i].pad;
        sum = lds_sum(*C, sum);
        if (d + 1 >= DMAX) {
            fail(2);
            return false;
        }
        const int64_t save = top;
        const int ccap = (int)((sum + 16 + 15) & ~15ll);
        RowV* rv = (RowV*)alloc((int64_t)n * sizeof(RowV));
        char* out = (char*)alloc((int64_t)n * ccap);
        if (!rv || !out) {
            __syncthreads();
            return false;
        }
        for (int i = threadIdx.x; i < n; i += WT) {
            const RowV v = F.rv[i];
            RowV c;
            c.base = v.base;
            c.len = v.pad;
            c.start = F.dir ? v.start + v.len - v.pos - v.pad : v.start + v.pos;
            c.pos = 0;
            c.pad = 0;
            rv[i] = c;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            C->fr[d].col = col;
            Frame& c = C->fr[d + 1];
            c.out = out;
            c.rv = rv;
            c.save_top = save;
            c.cap = ccap;
            c.col = 0;
            c.dir = !F.dir;
        }
        __syncthreads();
        d++;
        return true;
    }

    // process_seqs on frame d0 (and the frames it pushes) to completion
    __device__ void run(int d0) {
        int d = d0;
        __syncthreads();
        int col = C->fr[d].col;
        while (true) {
            __syncthreads();
            if (C->abort) return;
            Frame F = C->fr[d];
            bool finish = false;
            int tail = 0x7fffffff;
            for (int i = threadIdx.x; i < n; i += WT) {
                const RowV v = F.rv[i];
                tail = min(tail, v.len - v.pos);
            }
            tail = lds_min(*C, tail);
            if (tail <= 0) {  // is_stop (:58-65) -> append_all
                append_upto(F, col, 0);
                finish = true;
            } else {
                const int k = equal_run(F, min(tail, 64));
                if (k > 0) {
                    append_cols(F, col, k);
                } else if (tail > a.mc && cols_equal(F, 1, nullptr, 0, a.mc)) {  // try_mismatch
                    append_cols(F, col, a.mc + 1);
                } else if (tail > a.gc && try_gap(F, col)) {
                } else if (try_aligned(F, tail, d, col)) {
                    col = 0;
                    continue;
                } else {
                    if (failed()) return;
                    end_of(F, col);
                    finish = true;
                }
            }
            if (!finish) continue;
            if (failed()) return;
            if (d == d0) {
                if (threadIdx.x == 0) C->fr[d].col = col;
                __syncthreads();
                return;
            }
            // the child ends: its rows, reversed, after the parent's columns
            const Frame P = C->fr[d - 1];
            int pcol = P.col;
            const int Lc = col;
            if (!room(P, pcol, (int64_t)Lc + a.ac)) return;
            for (int i = threadIdx.x; i < n; i += WT) {
                const char* s = F.out + (int64_t)i * F.cap;
                char* o = P.out + (int64_t)i * P.cap + pcol;
                for (int q = 0; q < Lc; q++) o[q] = s[Lc - 1 - q];
                P.rv[i].pos += F.rv[i].len;
            }
            pcol += Lc;
            top = F.save_top;
            d--;
            Frame PP = C->fr[d];
            append_cols(PP, pcol, a.ac);
            col = pcol;
            __syncthreads();
            if (threadIdx.x == 0) C->fr[d].col = col;
        }
    }
    __device__ void end_of(Frame& F, int& col) {
        int k = 0;
        while (true) {
            bool c1 = true, c2 = true;
            const RowV v0 = F.rv[0];
            for (int i = threadIdx.x; i < n; i += WT) {
                const RowV v = F.rv[i];
                const int e = v.len - 1 - k;
                c1 &= v.pos < e && at(v, F.dir, i, e) == at(v0, F.dir, 0, v0.len - 1 - k);
                c2 &= v.pos < e - 1 && at(v, F.dir, i, e - 1) == at(v0, F.dir, 0, v0.len - 2 - k);
            }
            const bool a1 = __syncthreads_and(c1), a2 = __syncthreads_and(c2);
            if (!a1 && !a2) break;
            k++;
        }
        append_upto(F, col, k + 1);  // append_chars to end_pos, append_gaps
        append_upto(F, col, 0);      // append_all
    }
};


// gap-filtered copies of columns [c0, c1) of the n x cap rows R as the
// reversed rows of frame d (the input of a re-alignment, :444-447, :470-474)
__device__ bool push_filtered(Job& J, int d, const char* R, int cap, int c0, int c1) {
    const int n = J.n, w = c1 - c0;
    const int64_t save = J.top;
    char* M = (char*)J.alloc((int64_t)n * max(w, 1));
    RowV* rv = (RowV*)J.alloc((int64_t)n * sizeof(RowV));
    if (!M || !rv) return false;
    long long sum = 0;
    for (int i = threadIdx.x; i < n; i += WT) {
        const char* r = R + (int64_t)i * cap;
        char* m = M + (int64_t)i * w;
        int k = 0;
        for (int c = c0; c < c1; c++)
            if (r[c] != '-') m[k++] = r[c];
        RowV v;
        v.base = m;
        v.start = 0;
        v.len = k;
        v.pos = 0;
        v.pad = 0;
        rv[i] = v;
        sum += k;
    }
    sum = lds_sum(*J.C, sum);
    const int ocap = (int)((sum + 16 + 15) & ~15ll);
    char* O = (char*)J.alloc((int64_t)n * ocap);
    if (!O) return false;
    if (threadIdx.x == 0) {
        Frame& F = J.C->fr[d];
        F.out = O;
        F.rv = rv;
        F.save_top = save;
        F.cap = ocap;
        F.col = 0;
        F.dir = 1;
    }
    __syncthreads();
    return true;
}

// columns c < L of the n x cap rows R where every row equals row 0 (score_of, :416-426)
__device__ int score_of(Job& J, const char* R, int cap, int c0, int c1) {
    int s = 0;
    for (int c = c0 + (int)threadIdx.x; c < c1; c += WT) {
        const char x = R[c];
        bool eq = true;
        for (int i = 1; i < J.n && eq; i++) eq = R[(int64_t)i * cap + c] == x;
        s += eq;
    }
    return (int)lds_sum(*J.C, s);
}

// appends frame d's rows reversed into the n x cap rows R at column at
__device__ void put_reversed(Job& J, const Frame& F, char* R, int cap, int at) {
    const int L = F.col;
    for (int64_t q = threadIdx.x; q < (int64_t)J.n * L; q += WT) {
        const int i = (int)(q / L), c = (int)(q - (int64_t)i * L);
        R[(int64_t)i * cap + at + c] = F.out[(int64_t)i * F.cap + L - 1 - c];
    }
}

__device__ void copy_cols(Job& J, const char* S, char* D, int cap, int s0, int d0, int w) {
    for (int64_t q = threadIdx.x; q < (int64_t)J.n * w; q += WT) {
        const int i = (int)(q / w), c = (int)(q - (int64_t)i * w);
        D[(int64_t)i * cap + d0 + c] = S[(int64_t)i * cap + s0 + c];
    }
}

__global__ __launch_bounds__(WT) void k_align_wide(WArgs a) {
    __shared__ Ctx C;
    const WJob W = a.jobs[blockIdx.x];
    const int n = W.n, cap = W.cap;
    char* out = (char*)a.out + W.out;
    if (threadIdx.x == 0) {
        C.abort = 0;
        C.n_pu = C.n_wu = 0;
    }
    __syncthreads();
    if (a.aligner_type == 1) {  // DummyAligner: rows padded with gaps (DummyAligner.cpp:18-26)
        int mx = 0;
        for (int i = threadIdx.x; i < n; i += WT) mx = max(mx, a.row_len[W.row0 + i]);
        mx = lds_max(C, mx);
        if (mx > cap) {
            if (threadIdx.x == 0) a.status[blockIdx.x] = 1;
            return;
        }
        for (int64_t q = threadIdx.x; q < (int64_t)n * mx; q += WT) {
            const int i = (int)(q / mx), c = (int)(q - (int64_t)i * mx);
            const int len = a.row_len[W.row0 + i];
            out[(int64_t)i * cap + c] = c < len ? a.rows[a.row_off[W.row0 + i] + c] : '-';
        }
        if (threadIdx.x == 0) {
            a.len_out[blockIdx.x] = mx;
            a.status[blockIdx.x] = 0;
        }
        return;
    }
    Job J;
    J.a = a;
    J.C = &C;
    J.n = n;
    J.arena = a.arena + W.arena;
    J.top = 0;
    J.lim = W.arena_bytes;
    J.tlog2 = W.tlog2;
    J.tcap = 1u << W.tlog2;
    J.pt = a.pt + W.tab;
    J.wk = a.wk + W.tab;
    J.wc = a.wc + W.tab;
    J.pu = a.used + W.tab;
    J.wu = J.pu + J.tcap / 2;
    J.var = J.alloc((int64_t)MAXV * n);
    char* A = (char*)J.alloc((int64_t)n * cap);
    char* B = (char*)J.alloc((int64_t)n * cap);
    RowV* rv = (RowV*)J.alloc((int64_t)n * sizeof(RowV));
    int status = 0, L = 0;
    if (!J.var || !A || !B || !rv) {
        status = 1;
    } else {
        // process_seqs on the job's rows -> A
        for (int i = threadIdx.x; i < n; i += WT) {
            RowV v;
            v.base = a.rows + a.row_off[W.row0 + i];
            v.start = 0;
            v.len = a.row_len[W.row0 + i];
            v.pos = 0;
            v.pad = 0;
            rv[i] = v;
        }
        if (threadIdx.x == 0) {
            Frame& F = C.fr[0];
            F.out = A;
            F.rv = rv;
            F.save_top = J.top;
            F.cap = cap;
            F.col = 0;
            F.dir = 0;
        }
        __syncthreads();
        J.run(0);
        const int LA = C.fr[0].col;
        // fix_bad_regions (:428-459): identical columns, regions, re-alignment
        unsigned char* good = J.failed() ? nullptr : J.alloc(LA + 1);
        int* rg = good ? (int*)J.alloc(6ll * 4 * (LA + 1)) : nullptr;
        int LB = 0;
        if (good && rg) {
            int *rs = rg, *re = rs + (LA + 1), *rgd = re + (LA + 1), *rw = rgd + (LA + 1), *rp = rw + (LA + 1),
                *rn = rp + (LA + 1);
            for (int c = threadIdx.x; c < LA; c += WT) {
                const char x = A[c];
                bool eq = true;
                for (int i = 1; i < n && eq; i++) eq = A[(int64_t)i * cap + c] == x;
                good[c] = eq;
            }
            __syncthreads();
            if (threadIdx.x == 0) {  // make_regions (FindLowSimilar.cpp:62-80)
                int R = 0;
                for (int c = 0; c < LA; c++) {
                    if (R > 0 && rgd[R - 1] == good[c]) {
                        re[R - 1] = c;
                    } else {
                        rs[R] = re[R] = c;
                        rgd[R] = good[c];
                        R++;
                    }
                }
                for (int r = 0; r < R; r++) {
                    const int len = re[r] - rs[r] + 1;
                    rw[r] = rgd[r] ? len : len * a.wf;
                    rp[r] = r - 1;
                    rn[r] = r + 1 < R ? r + 1 : -1;
                }
                C.r32 = R;
                C.head = R ? 0 : -1;
            }
            __syncthreads();
            const int R = C.r32;
            int live = R;
            // reduce_regions (:121-130): merge the lightest (first on ties) while < min_length
            while (live >= 2) {
                unsigned long long m = ~0ull;
                for (int r = threadIdx.x; r < R; r += WT)
                    if (rw[r] >= 0) m = min(m, ((unsigned long long)(uint32_t)rw[r] << 32) | (uint32_t)r);
                m = lds_min64(C, m);
                const int mi = (int)(m & 0xffffffffu), mw = (int)(m >> 32);
                if (mw >= a.min_length) break;
                if (threadIdx.x == 0) {
                    const int p = rp[mi], q = rn[mi];
                    int w = rw[mi];
                    if (p >= 0) {
                        rs[mi] = rs[p];
                        w += rw[p];
                        rw[p] = -1;
                        rp[mi] = rp[p];
                        if (rp[p] >= 0) rn[rp[p]] = mi; else C.head = mi;
                    }
                    if (q >= 0) {
                        re[mi] = re[q];
                        w += rw[q];
                        rw[q] = -1;
                        rn[mi] = rn[q];
                        if (rn[q] >= 0) rp[rn[q]] = mi;
                    }
                    rw[mi] = w;
                    rgd[mi] = !rgd[mi];
                }
                __syncthreads();
                int cnt = 0;
                for (int r = threadIdx.x; r < R; r += WT) cnt += rw[r] >= 0;
                live = (int)lds_sum(C, cnt);
            }
            __syncthreads();
            for (int r = C.head; r >= 0 && status == 0; r = rn[r]) {
                const int s0 = rs[r], s1 = re[r] + 1, w = s1 - s0;
                if (LB + w > cap) {
                    status = 1;
                    break;
                }
                if (rgd[r]) {
                    copy_cols(J, A, B, cap, s0, LB, w);
                    LB += w;
                    continue;
                }
                const int before = score_of(J, A, cap, s0, s1);
                const int64_t save = J.top;
                if (!push_filtered(J, 1, A, cap, s0, s1)) {
                    status = 1;
                    break;
                }
                J.run(1);
                if (J.failed()) {
                    status = C.abort;
                    break;
                }
                const Frame F = C.fr[1];
                const int after = score_of(J, F.out, F.cap, 0, F.col);
                if (after > before) {
                    if (LB + F.col > cap) {
                        status = 1;
                        break;
                    }
                    put_reversed(J, F, B, cap, LB);
                    LB += F.col;
                } else {
                    copy_cols(J, A, B, cap, s0, LB, w);
                    LB += w;
                }
                J.top = save;
                __syncthreads();
            }
        } else {
            status = max(C.abort, 1);
        }
        // realing_end (:461-484) on B
        if (status == 0 && LB >= 2) {
            const int pre = max(1, LB - a.ac);
            if (!push_filtered(J, 1, B, cap, pre, LB)) {
                status = 1;
            } else {
                J.run(1);
                if (J.failed()) {
                    status = C.abort;
                } else {
                    const Frame F = C.fr[1];
                    if (pre + F.col > cap) {
                        status = 1;
                    } else {
                        __syncthreads();
                        put_reversed(J, F, B, cap, pre);
                        LB = pre + F.col;
                    }
                }
            }
        }
        // remove_gaps (AbstractAligner.cpp:89-102): B -> out, pure-gap columns dropped
        if (status == 0) {
            __syncthreads();
            __shared__ int wsum[WT / 64];
            const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
            for (int c0 = 0; c0 < LB; c0 += WT) {
                const int c = c0 + (int)threadIdx.x;
                bool keep = false;
                if (c < LB)
                    for (int i = 0; i < n && !keep; i++) keep = B[(int64_t)i * cap + c] != '-';
                const unsigned long long m = __ballot(keep);
                if (lane == 0) wsum[wv] = __popcll(m);
                __syncthreads();
                int base = L;
                for (int q = 0; q < wv; q++) base += wsum[q];
                const int tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
                if (keep) {
                    const int dst = base + __popcll(m & ((1ull << lane) - 1));
                    for (int i = 0; i < n; i++) out[(int64_t)i * cap + dst] = B[(int64_t)i * cap + c];
                }
                L += tot;
                __syncthreads();
            }
        }
    }
    if (threadIdx.x == 0) {
        a.len_out[blockIdx.x] = L;
        a.status[blockIdx.x] = status;
    }
}

}  // namespace wide

struct WideBufs {
    DevBuf<wide::WJob> jobs;
    std::deque<DevBuf<unsigned char>> outs;  // one output buffer per launch of a call (kept until the next call)
    DevBuf<unsigned char> arena;
    DevBuf<unsigned long long> pt, wk;
    DevBuf<uint32_t> wc, used;
    DevBuf<int32_t> len, status;
    DevBuf<int64_t> row_off;
    DevBuf<int32_t> row_len;
};

WideBufs* wide_create() { return new WideBufs(); }
void wide_free(WideBufs* w) { delete w; }

void align_wide(WideBufs* W, hipStream_t st, const char* d_rows, const int64_t* ne_off, const int32_t* ne_len,
                int64_t n_ne, const std::vector<WideJobIn>& in, const int params[5], int aligner_type,
                std::vector<int32_t>& len, std::vector<int32_t>& cap, std::vector<const char*>& ptr,
                double* wait_ms) {
    using namespace wide;
    const size_t nj = in.size();
    len.assign(nj, 0);
    cap.assign(nj, 0);
    ptr.assign(nj, nullptr);
    if (!nj) return;
    NPGX_REQUIRE(params[2] >= 1 && params[2] <= 16, NPGX_ERR_RANGE, "aligned-check must be 1..16");
    W->row_off.ensure(n_ne);
    W->row_len.ensure(n_ne);
    NPGX_HIP(hipMemcpyAsync(W->row_off.p, ne_off, n_ne * 8, hipMemcpyHostToDevice, st));
    NPGX_HIP(hipMemcpyAsync(W->row_len.p, ne_len, n_ne * 4, hipMemcpyHostToDevice, st));
    // Every job runs until it fits: each attempt gives a failing job more
    // columns (2x the longest row, 4x, 16x, then the proven bound: the sum of
    // its rows), larger pair / word tables and a larger arena.  One
    // try_aligned call inserts at most n x (min tail - aligned_check) pairs
    // and as many words before its tables are cleared (SimilarAligner.cpp:
    // 246-308), so tables of 2 (n (longest - ac) + n) entries cannot overflow:
    // a job's tables stop growing there.  The arena (recursion frames) keeps
    // doubling.  Jobs of one attempt launch in waves whose scratch fits the
    // budget (NPGX_WIDE_BUDGET_MB, default 8 GiB); a job that alone needs more
    // than the budget is refused with NPGX_ERR_RANGE, never cut short.
    static const int64_t budget = [] {
        const char* e = getenv("NPGX_WIDE_BUDGET_MB");
        return (e ? std::max<int64_t>(atoll(e), 64) : 8192) << 20;
    }();
    struct Size {
        int64_t sum, mx;
        uint32_t lg_need;
    };
    std::vector<Size> sz(nj);
    for (size_t q = 0; q < nj; q++) {
        const WideJobIn& I = in[q];
        NPGX_REQUIRE(I.n < 65536, NPGX_ERR_RANGE, "more than 65535 rows in one alignment");
        int64_t sum = 0, mx = 0;
        for (int i = 0; i < I.n; i++) {
            sum += ne_len[I.row0 + i];
            mx = std::max<int64_t>(mx, ne_len[I.row0 + i]);
        }
        NPGX_REQUIRE(sum < (1ll << 30), NPGX_ERR_RANGE, "alignment problem too large");
        const int64_t need = 2 * ((int64_t)I.n * std::max<int64_t>(mx - params[2], 0) + I.n) + 2;
        uint32_t lg = 12;
        while (((int64_t)1 << lg) < need) lg++;
        sz[q] = Size{sum, mx, lg};
    }
    std::vector<size_t> todo(nj);
    for (size_t q = 0; q < nj; q++) todo[q] = q;
    size_t launch = 0;
    for (int attempt = 0; !todo.empty(); attempt++) {
        NPGX_REQUIRE(attempt < 24, NPGX_ERR_RANGE, "wide alignment: no progress after 24 attempts");
        std::vector<WJob> jobs(todo.size());
        std::vector<int64_t> cost(todo.size());
        for (size_t t = 0; t < todo.size(); t++) {
            const WideJobIn& I = in[todo[t]];
            const Size& Z = sz[todo[t]];
            // columns: 2 x the longest row first, then 4x, 16x, the proven bound (the sum)
            const int64_t grow[4] = {2, 4, 16, 1ll << 40};
            int64_t c = aligner_type == 1 ? Z.mx : std::min<int64_t>(Z.sum, grow[std::min(attempt, 3)] * Z.mx + 64);
            c = (std::max<int64_t>(c, 1) + 15) & ~15ll;
            WJob& J = jobs[t];
            J.row0 = I.row0;
            J.n = I.n;
            J.cap = (int32_t)c;
            J.arena_bytes = aligner_type == 1 ? 0
                            : ((4 * (int64_t)I.n * c + 32 * c + (int64_t)I.n * (MAXV + 4 * sizeof(RowV)) + (1 << 16))
                               << std::min(attempt, 20));
            // tables: room for 256 shifts of every row first, x4 per attempt, at most the proven size
            uint32_t lg = 12;
            while ((1u << lg) < 512u * (uint32_t)I.n && lg < 22) lg++;
            J.tlog2 = aligner_type == 1 ? 0 : std::min<uint32_t>(lg + 2 * (uint32_t)attempt, Z.lg_need);
            const int64_t tab_bytes = aligner_type == 1 ? 0 : ((int64_t)1 << J.tlog2) * 24;
            cost[t] = (((int64_t)I.n * c + 255) & ~255ll) + ((J.arena_bytes + 255) & ~255ll) + tab_bytes;
            NPGX_REQUIRE(cost[t] <= budget, NPGX_ERR_RANGE,
                         "wide alignment problem needs more scratch than NPGX_WIDE_BUDGET_MB allows");
        }
        std::vector<size_t> again;
        for (size_t w0 = 0; w0 < todo.size();) {  // one wave: the jobs [w0, w1)
            size_t w1 = w0;
            int64_t used = 0;
            while (w1 < todo.size() && (w1 == w0 || used + cost[w1] <= budget)) used += cost[w1++];
            int64_t out_bytes = 0, arena_bytes = 0, tab = 0;
            for (size_t t = w0; t < w1; t++) {
                WJob& J = jobs[t];
                J.out = out_bytes;
                out_bytes += ((int64_t)J.n * J.cap + 255) & ~255ll;
                J.arena = arena_bytes;
                arena_bytes += (J.arena_bytes + 255) & ~255ll;
                J.tab = tab;
                tab += aligner_type == 1 ? 0 : (int64_t)1 << J.tlog2;
            }
            const size_t nw = w1 - w0;
            W->jobs.ensure(nw);
            if (W->outs.size() <= launch) W->outs.emplace_back();
            DevBuf<unsigned char>& ob = W->outs[launch++];
            ob.ensure(std::max<int64_t>(out_bytes, 1));
            W->arena.ensure(std::max<int64_t>(arena_bytes, 1));
            const size_t tabn = (size_t)std::max<int64_t>(tab, 1);
            if (W->pt.cap < tabn) {  // a fresh pool is cleared once; the kernel leaves it cleared
                W->pt.ensure(tabn);
                W->wk.ensure(tabn);
                NPGX_HIP(hipMemsetAsync(W->pt.p, 0xff, W->pt.cap * 8, st));
                NPGX_HIP(hipMemsetAsync(W->wk.p, 0xff, W->wk.cap * 8, st));
                W->wc.ensure(tabn);
                NPGX_HIP(hipMemsetAsync(W->wc.p, 0, W->wc.cap * 4, st));
                W->used.ensure(tabn);
            }
            W->len.ensure(nw);
            W->status.ensure(nw);
            NPGX_HIP(hipMemcpyAsync(W->jobs.p, jobs.data() + w0, nw * sizeof(WJob), hipMemcpyHostToDevice, st));
            WArgs A;
            A.rows = d_rows;
            A.row_off = W->row_off.p;
            A.row_len = W->row_len.p;
            A.jobs = W->jobs.p;
            A.out = ob.p;
            A.arena = W->arena.p;
            A.pt = W->pt.p;
            A.wk = W->wk.p;
            A.wc = W->wc.p;
            A.used = W->used.p;
            A.len_out = W->len.p;
            A.status = W->status.p;
            A.mc = params[0];
            A.gc = params[1];
            A.ac = params[2];
            A.min_length = params[3];
            A.wf = params[4];
            A.aligner_type = aligner_type;
            // try_aligned's prefix search after the first WIDE_LONG_HEAD shifts
            // (NPGX_WIDE_LONG_HEAD; 0: shift by shift only, the round-4 search)
            const char* wl = getenv("NPGX_WIDE_LONG_HEAD");  // (read per batch: tests switch it)
            const int wlh = wl && *wl ? std::max(0, atoi(wl)) : 4;
            A.lh = wlh;
            const char* wm = getenv("NPGX_WIDE_LONG_M");  // the first prefix (doubling from there)
            A.lm = wm && *wm ? std::max(1, atoi(wm)) : 512;
            hipLaunchKernelGGL(k_align_wide, dim3((unsigned)nw), dim3(WT), 0, st, A);
            NPGX_HIP(hipGetLastError());
            std::vector<int32_t> L(nw), S(nw);
            // (the wait for the launch: the copies into pageable memory wait too)
            const auto tw = std::chrono::steady_clock::now();
            NPGX_HIP(stream_wait(st));
            NPGX_HIP(hipMemcpy(L.data(), W->len.p, nw * 4, hipMemcpyDeviceToHost));
            NPGX_HIP(hipMemcpy(S.data(), W->status.p, nw * 4, hipMemcpyDeviceToHost));
            if (wait_ms)
                *wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw).count();
            for (size_t t = w0; t < w1; t++) {
                NPGX_REQUIRE(S[t - w0] != 2, NPGX_ERR_RANGE,
                             "wide alignment: more than 96 nested re-alignments or 8 gap variants");
                if (S[t - w0] != 0) {
                    again.push_back(todo[t]);
                    continue;
                }
                len[todo[t]] = L[t - w0];
                cap[todo[t]] = jobs[t].cap;
                ptr[todo[t]] = (const char*)(ob.p + jobs[t].out);
            }
            w0 = w1;
        }
        todo.swap(again);
    }
}

}  // namespace npgx
