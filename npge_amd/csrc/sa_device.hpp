// sa_device.hpp -- wave-level building blocks of the greedy multiple aligner
// (SimilarAligner, src/algo/SimilarAligner.cpp:41-485) on CDNA4.
//
// One wavefront owns one alignment problem; lane i owns row i (n <= 64 rows).
// A row is read through a View (char(q) = p[d*q] for q < len), so the reversed
// sub-problems the reference creates with substr + std::reverse
// (append_aligned :274-293) are views on the parent's rows, not copies.
// Column tests (is_equal :101-115) are wave ballots.  The reference's recursion
// (append_aligned -> process_seqs) runs on an explicit per-wave stack; a child
// writes its output right after the parent's cursor and is reversed in place
// when it returns.
//
// Past-the-end reads (find_best_gap :191-217 may read beyond a row): char(len)
// is '\0' like std::string; char(q > len) is a per-row sentinel that equals
// nothing (same convention as the oracle).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace npgx {
namespace sa {

struct View {
    const char* p;  // address of char 0
    int len;
    int d;          // +1 forward, -1 reversed
};

struct Params {
    int mc, gc, ac, min_length;
    int wf;                 // FindLowSimilar weight factor (FindLowSimilar.cpp:56-60)
};

// Per-wave scratch (global memory), sized by the host for the batch.
struct Slot {
    unsigned long long* tkeys;   // try_aligned word table: (epoch << 48 | word)
    unsigned long long* tmask;   // row masks
    uint32_t tcap_log2;
    uint32_t epoch;
    // append_aligned stack: per level 64 lanes x {p, len|dneg<<31, pos} + uniform col
    const char** st_p;
    int* st_len;
    int* st_pos;
    int* st_col;
    int st_depth_max;
    // FindLowSimilar regions (start, stop, good, weight)
    int4* regions;
    unsigned char* good_col;
};

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

// all active lanes agree on c
__device__ __forceinline__ bool all_eq(const WaveCtx& w, int c) {
    const int c0 = __shfl(c, 0);
    return (ballot(!w.act || c == c0) & w.rowmask) == w.rowmask;
}

__device__ __forceinline__ bool any_lane(const WaveCtx& w, bool b) {
    return (ballot(w.act && b) & w.rowmask) != 0;
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ unsigned long long shfl64(unsigned long long v, int src) {
    const unsigned lo = (unsigned)__shfl((int)(unsigned)v, src);
    const unsigned hi = (unsigned)__shfl((int)(unsigned)(v >> 32), src);
    return ((unsigned long long)hi << 32) | lo;
}

// Output buffer of one problem: row i at base + i*cap.
struct Out {
    char* base;
    int cap;
};

struct Frame {
    View v;
    int pos;
};

// ---------------------------------------------------------------- process_seqs
// State of one process_seqs call tree (SimilarAligner.cpp:396-405) with the
// append_aligned recursion flattened onto Slot's stack.
struct Proc {
    const WaveCtx& w;
    const Params& P;
    Slot& S;
    Out out;
    View v;
    int pos;
    int col;        // output cursor (all rows equal length between steps)
    bool ovf;       // lane-local overflow

    __device__ Proc(const WaveCtx& w_, const Params& P_, Slot& S_, Out o)
        : w(w_), P(P_), S(S_), out(o), pos(0), col(0), ovf(false) {}

    __device__ __forceinline__ void put(int c, char ch) {
        if (c < out.cap) out.base[(size_t)w.lane * out.cap + c] = ch;
        else ovf = true;
    }
    __device__ __forceinline__ int ch(int q) const { return vch(v, q, w.lane); }

    // is_stop :58-65
    __device__ bool is_stop(int shift) const { return any_lane(w, pos + shift >= v.len); }

    // append_cols :67-77
    __device__ void append_cols(int cols) {
        if (w.act)
            for (int j = 0; j < cols; j++) put(col + j, (char)ch(pos + j));
        pos += w.act ? cols : 0;
        col += cols;
    }
    // append_all :91-99 (tail of every row, then append_gaps :79-89)
    __device__ void append_all() {
        int t = w.act ? v.len - pos : 0;
        if (t < 0) t = 0;
        const int m = wave_max(t);
        if (w.act) {
            for (int j = 0; j < t; j++) put(col + j, (char)ch(pos + j));
            for (int j = t; j < m; j++) put(col + j, '-');
            pos += t;
        }
        col += m;
    }
    // is_equal(pos + off, shift, cols) where off = 1 for lanes in `shifted`
    __device__ bool is_equal_sh(unsigned long long shifted, int shift, int cols) const {
        const int base = pos + (int)((shifted >> w.lane) & 1ull) + shift;
        for (int j = 0; j < cols; j++)
            if (!all_eq(w, ch(base + j))) return false;
        return true;
    }
    // apply_gap :165-174
    __device__ void apply_gap(unsigned long long shifted, int g) {
        const bool s = w.act && ((shifted >> w.lane) & 1ull);
        if (w.act) put(col, s ? (char)ch(pos) : '-');
        pos += s ? 1 : 0;
        col += 1;  // at least one row is shifted (else the column was equal)
        append_cols(g);
    }
    // try_gap :219-235 with find_all_gaps :176-189 and find_best_gap :191-217
    __device__ bool try_gap() {
        if (is_stop(P.gc)) return false;
        unsigned long long var[5];
        int nv = 0;
        const int c_here = ch(pos);
        const int c_next = ch(pos + 1);
        // std::set<char> order: 'A' < 'C' < 'G' < 'N' < 'T'
        const char order[5] = {'A', 'C', 'G', 'N', 'T'};
        for (int k = 0; k < 5; k++) {
            const int c = order[k];
            if (!any_lane(w, c_here == c)) continue;
            const bool mt = c_here == c, mn = c_next == c;
            if (any_lane(w, mt == mn)) continue;
            const unsigned long long shifted = ballot(w.act && mn) & w.rowmask;
            if (is_equal_sh(shifted, 0, P.gc)) var[nv++] = shifted;
        }
        if (nv == 0) return false;
        if (nv == 1) {
            apply_gap(var[0], P.gc);
            return true;
        }
        for (int g = P.gc + 1;; g++) {
            unsigned long long nx[5];
            int nn = 0;
            for (int k = 0; k < nv; k++)  // columns < g-1 are known equal
                if (is_equal_sh(var[k], g - 1, 1)) nx[nn++] = var[k];
            if (nn == 0) {
                apply_gap(var[0], g - 1);
                return true;
            }
            if (nn == 1) {
                apply_gap(nx[0], g);
                return true;
            }
            for (int k = 0; k < nn; k++) var[k] = nx[k];
            nv = nn;
        }
    }

    // word code of a letter (injective on ATGCN)
    __device__ static __forceinline__ unsigned long long code3(int c) {
        return c == 'A' ? 1 : c == 'C' ? 2 : c == 'G' ? 3 : c == 'N' ? 4 : c == 'T' ? 5 : 6;
    }

    // try_aligned :295-308 + find_best_word :246-272.  Returns true and the
    // per-lane shift (first shift at which the row shows the chosen word).
    __device__ bool try_aligned(int& my_shift) {
        const int mt = wave_min(w.act ? v.len - pos : 0x7fffffff);
        const int max_shift = mt - P.ac;
        if (max_shift <= 0) return false;
        // fresh epoch of the word table
        S.epoch += 1;
        const uint32_t tcap = 1u << S.tcap_log2;
        if (S.epoch >= 0xFFFF) {
            for (uint32_t i = w.lane; i < tcap; i += 64) {
                S.tkeys[i] = 0ull;
                S.tmask[i] = 0ull;
            }
            __threadfence();
            S.epoch = 1;
        }
        const unsigned long long ep = (unsigned long long)S.epoch << 48;
        const unsigned long long wmask = (P.ac >= 16) ? ((1ull << 48) - 1) : ((1ull << (3 * P.ac)) - 1);
        unsigned long long word = 0;
        if (w.act)
            for (int j = 0; j < P.ac - 1; j++) word = (word << 3) | code3(ch(pos + j));
        for (int s = 0; s < max_shift; s++) {
            if (w.act) word = ((word << 3) | code3(ch(pos + s + P.ac - 1))) & wmask;
            // group lanes by word
            unsigned long long remaining = w.rowmask, gm = 0;
            int leader = 0;
            while (remaining) {
                const int l = __ffsll((long long)remaining) - 1;
                const unsigned long long wl = shfl64(word, l);
                const unsigned long long m = ballot(w.act && word == wl) & w.rowmask;
                if ((m >> w.lane) & 1ull) {
                    gm = m;
                    leader = l;
                }
                remaining &= ~m;
            }
            // leaders update the table (one lane per distinct word: no mask races)
            bool complete = false;
            if (w.act && leader == w.lane) {
                const unsigned long long key = ep | word;
                uint32_t slot = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - S.tcap_log2));
                unsigned long long newm;
                while (true) {
                    const unsigned long long k =
                        __hip_atomic_load(&S.tkeys[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (k == key) {
                        newm = atomicOr(&S.tmask[slot], gm) | gm;
                        break;
                    }
                    if ((k & ~((1ull << 48) - 1)) != ep) {  // stale or empty: claim it
                        if (atomicCAS(&S.tkeys[slot], k, key) == k) {
                            atomicExch(&S.tmask[slot], gm);
                            newm = gm;
                            break;
                        }
                        continue;
                    }
                    slot = (slot + 1) & (tcap - 1);
                }
                complete = (newm == w.rowmask);
            }
            const bool comp_i = __shfl(complete ? 1 : 0, leader) != 0;
            const unsigned long long cm = ballot(w.act && comp_i) & w.rowmask;
            if (cm) {
                const int bl = 63 - __clzll((long long)cm);
                const unsigned long long best = shfl64(word, bl);
                const unsigned long long g0 = shfl64(gm, 0);
                if (g0 == w.rowmask) {  // words.size() == 1: every row at this shift
                    my_shift = s;
                } else {
                    // first shift at which this row produced the best word
                    my_shift = -1;
                    if (w.act) {
                        unsigned long long x = 0;
                        for (int j = 0; j < P.ac - 1; j++) x = (x << 3) | code3(ch(pos + j));
                        for (int t = 0; t <= s; t++) {
                            x = ((x << 3) | code3(ch(pos + t + P.ac - 1))) & wmask;
                            if (x == best) {
                                my_shift = t;
                                break;
                            }
                        }
                    }
                }
                return true;
            }
        }
        return false;
    }

    // append_end :323-342
    __device__ void append_end() {
        int e = v.len - 1;
        while (true) {
            bool c1 = !any_lane(w, !(pos < e)) && all_eq(w, ch(e));
            if (!c1) {
                bool c2 = !any_lane(w, !(pos < e - 1)) && all_eq(w, ch(e - 1));
                if (!c2) break;
            }
            e -= 1;
        }
        int cols = w.act ? e - pos : 0;
        const int m = wave_max(cols);
        if (w.act) {
            for (int j = 0; j < cols; j++) put(col + j, (char)ch(pos + j));
            for (int j = cols; j < m; j++) put(col + j, '-');
            pos += cols;
        }
        col += m;
        append_all();
    }

    // reverse the output columns [c0, c1) of every row in place
    __device__ void reverse_cols(int c0, int c1) {
        if (!w.act) return;
        if (c1 > out.cap) {
            ovf = true;
            return;
        }
        char* r = out.base + (size_t)w.lane * out.cap;
        for (int a = c0, b = c1 - 1; a < b; a++, b--) {
            const char t = r[a];
            r[a] = r[b];
            r[b] = t;
        }
    }

    // One step of process_cols (SimilarAligner.cpp:351-368).  Returns 0 = keep
    // stepping, 1 = frame finished, 2 = descend into a child (sh = shift).
    __device__ int step(int& sh) {
        if (is_stop(0)) {
            append_all();
            return 1;
        }
        if (all_eq(w, ch(pos))) {
            append_cols(1);
            return 0;
        }
        if (!is_stop(P.mc) && is_equal_sh(0ull, 1, P.mc)) {  // try_mismatch :122-134
            append_cols(P.mc + 1);
            return 0;
        }
        if (try_gap()) return 0;
        sh = 0;
        if (try_aligned(sh)) {
            if (!any_lane(w, sh > 0)) {  // every prefix empty: the child adds nothing
                append_cols(P.ac);
                return 0;
            }
            return 2;
        }
        append_end();
        return 1;
    }

    // process_seqs on view v0 writing from output column col0; returns the
    // alignment length.  append_aligned's recursion runs on S's stack.
    __device__ int run(const View& v0, int col0) {
        v = v0;
        pos = 0;
        col = col0;
        int depth = 0;
        bool fresh = true;
        while (true) {
            int r;
            if (fresh && any_lane(w, v.len == 0)) {  // process_cols :345-350
                append_all();
                r = 1;
            } else {
                int sh = 0;
                r = step(sh);
                if (r == 2) {
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
            // frame finished
            if (depth == 0) return col - col0;
            depth--;
            const int child_len = v.len;  // = this row's shift in the parent
            const size_t o = (size_t)depth * 64 + w.lane;
            const int c0 = __shfl(S.st_col[depth], 0);
            v.p = S.st_p[o];
            const int l = S.st_len[o];
            v.len = l & 0x7fffffff;
            v.d = (l & (int)0x80000000) ? -1 : 1;
            pos = S.st_pos[o];
            reverse_cols(c0, col);
            pos += w.act ? child_len : 0;
            append_cols(P.ac);
        }
    }
};

}  // namespace sa
}  // namespace npgx
