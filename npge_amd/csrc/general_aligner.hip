// general_aligner.hip -- MI355X-native batched GeneralAligner: banded min-cost
// Needleman-Wunsch with a gap frame and an error stop rule
// (src/util/GeneralAligner.hpp:28-414, NPG-explorer 0.5.8), on nucleotide
// contents whose substitution is 0 for equal non-N letters and
// mismatch_penalty otherwise (FragmentDistance.cpp:18-21, "see PairAligner").
//
// One wave per pair, anti-diagonal wavefront over the band:
//   * the band |col - row| <= gap_range has D = 2*gap_range + 1 diagonals; lane
//     j owns diagonals q = 2j and 2j+1 (q = col - row + gap_range), so 64 lanes
//     cover gap_range <= 63;
//   * step s processes anti-diagonal row + col = s: the cells of one
//     anti-diagonal are independent (their diag / left / up predecessors lie on
//     anti-diagonals s-2, s-1, s-1), and on step s exactly the diagonals with
//     q = s + gap_range (mod 2) are live -- one cell per lane per step;
//   * left and up neighbours come from the lanes on either side (one shuffle
//     each), the diagonal predecessor from the lane's own register;
//   * frame cells (row -1 / col -1, make_frame :388-407) are the registers'
//     initial values, band-edge cells (limit_range :377-386) read BAD_VALUE;
//   * the traceback direction (2 bits per cell, MATCH > COL_INC > ROW_INC as
//     :140-142) accumulates 16 steps per lane in a register and goes to HBM as
//     one coalesced 256-byte store per 16 steps;
//   * each row's first minimum column (:137-139) is an LDS ds_min_u64 of
//     (score << 32 | col) in a 256-row ring; rows complete one per step at
//     most (at step row + max_col(row)), where the max_errors stop rule
//     (:144-147) is evaluated wave-uniformly;
//   * cut_tail (:240-255) and export_alignment (:262-282) walk back
//     wave-uniformly: each 16-step block of directions is one coalesced load,
//     a cell's 2 bits come from v_readlane, and the ops go out 64 at a time.
// Scores are exact int32 arithmetic: at(prev) < at(cur) along a traced path is
// exactly "the step cost is positive", which is what cut_tail needs.
#include <algorithm>
#include <climits>
#include <cstring>
#include <type_traits>

#include "common.hpp"

namespace npgx {
namespace ga {

static constexpr int BAD_VALUE = 1000000;   // GeneralAligner.hpp:24
static constexpr int RING = 256;            // open rows (<= gap_range + 2 at a time)
#ifdef NPGX_SA_PROFILE
static constexpr int RES = 8;  // + cycles of the forward pass and of the traceback
#else
static constexpr int RES = 5;
#endif
enum { MATCH = 0, ROW_INC = 1, COL_INC = 2 };

struct Pair {
    int64_t a_off, b_off;   // into the letters of the batch
    int64_t track_off;      // uint32 words
    int64_t out_end;        // ops are written backwards, ending here
    int32_t la, lb;
};

struct GaArgs {
    const char* a;
    const char* b;
    const Pair* pairs;
    uint32_t* track;
    int8_t* ops;
    int32_t* res;           // per pair: first_last, second_last, score, status, n_ops
    int32_t gr, max_errors, gp, mm, cut_tail, pad;
};

struct Geo {  // GeneralAligner::side / max_row / min_col / max_col (:300-316)
    int rows, cols, gr;
    __device__ int side() const { return min(min(rows, cols) + gr, max(rows, cols)); }
    __device__ int max_row() const { return min(rows, side()) - 1; }
    __device__ int max_col(int r) const { return min(cols - 1, min(side() - 1, r + gr)); }
};

__device__ __forceinline__ int sub(const char* a, const char* b, int r, int c, int mm) {
    const char x = a[r];
    return (x == b[c] && x != 'N') ? 0 : mm;
}

// wave-wide lane shifts by one (DPP wave_shr:1 / wave_shl:1, gfx9 family);
// the lane shifted in from outside the wave gets `edge`
__device__ __forceinline__ int from_lane_below(int v, int edge) {  // lane l gets lane l-1's v
    return __builtin_amdgcn_update_dpp(edge, v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ int from_lane_above(int v, int edge) {  // lane l gets lane l+1's v
    return __builtin_amdgcn_update_dpp(edge, v, 0x130, 0xF, 0xF, false);
}

static constexpr int LWIN = 256;  // LDS window of each sequence (bytes, a ring)
static constexpr int REFILL = 32; // steps per window refill / mismatch-mask batch

// high bit of each byte set iff that byte of x is zero (exact)
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
    return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}

// 16 substitution flags (1 = mismatch or N) of the cells (r0+k, c0+k),
// k < 16, from the LDS windows: dword loads, byte-aligned by v_alignbyte,
// byte-parallel compares (FragmentDistance.cpp:18-21 semantics)
__device__ __forceinline__ uint32_t mism16(const uint32_t* wa, const uint32_t* wb, int r0, int c0) {
    const int ia = r0 >> 2, sa = r0 & 3, ib = c0 >> 2, sb = c0 & 3;
    uint32_t A[5], B[5];
#pragma unroll
    for (int i = 0; i < 5; i++) {
        A[i] = wa[(ia + i) & (LWIN / 4 - 1)];
        B[i] = wb[(ib + i) & (LWIN / 4 - 1)];
    }
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t x = __builtin_amdgcn_alignbyte(A[i + 1], A[i], sa);
        const uint32_t y = __builtin_amdgcn_alignbyte(B[i + 1], B[i], sb);
        const uint32_t good = zero_bytes(x ^ y) & ~zero_bytes(x ^ 0x4E4E4E4Eu);  // equal, not N
        const uint32_t bad = (~good >> 7) & 0x01010101u;
        m |= ((bad * 0x01020408u) >> 24) << (4 * i);
    }
    return m;
}

struct Fwd {  // per-wave state of the forward pass
    int H0, H1;
    uint32_t acc;
    int r_row, r_col, r_score, next_row;
    bool pend;
    unsigned long long pend_key;
    int end_v;
    int loaded;
    uint32_t pa[8], pb[8];  // next 32 letters of each sequence (scalar loads, one refill ahead)
};

__global__ __launch_bounds__(64) void k_general_align(GaArgs A) {
    __shared__ unsigned long long ring[RING];
    __shared__ uint32_t wa32[LWIN / 4], wb32[LWIN / 4];
    char* wa = (char*)wa32;
    char* wb = (char*)wb32;
    const int lane = threadIdx.x;
    const Pair P = A.pairs[blockIdx.x];
    const char* a = A.a + P.a_off;
    const char* b = A.b + P.b_off;
    uint32_t* track = A.track + P.track_off;
    const int G = A.gr, gp = A.gp, mm = A.mm;
    const Geo g{P.la, P.lb, G};
    const int max_row = g.max_row();
    int32_t* out = A.res + (int64_t)blockIdx.x * RES;
    if (P.la == 0 || P.lb == 0) {  // find_aln handles these without the aligner (:612-615)
        if (lane == 0) {
            out[0] = -1;
            out[1] = -1;
            out[2] = 0;
            out[3] = -2;
            out[4] = 0;
        }
        return;
    }
    for (int i = lane; i < RING; i += 64) ring[i] = ~0ull;
    // letters: the first 128 of each sequence, then 32 more per refill from
    // scalar loads issued one refill ahead (lgkmcnt: they never wait behind the
    // traceback stores).  Pair letters start 16-byte aligned with 64 bytes of
    // slack after the batch, so whole dwords can be read past the end.
    const uint32_t* __restrict__ a32 = (const uint32_t*)a;
    const uint32_t* __restrict__ b32 = (const uint32_t*)b;
    for (int i = lane; i < 128; i += 64) {
        wa[i] = i < P.la ? a[i] : 0;
        wb[i] = i < P.lb ? b[i] : 0;
    }
    Fwd F;
    F.loaded = 128;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        F.pa[i] = a32[32 + i];
        F.pb[i] = b32[32 + i];
    }
    __syncthreads();

    // registers: the last value on each owned diagonal (frame value at start)
    const int q0 = 2 * lane, q1 = 2 * lane + 1;
    F.H0 = q0 <= 2 * G + 1 ? abs(q0 - G) * gp : BAD_VALUE;
    F.H1 = q1 <= 2 * G + 1 ? abs(q1 - G) * gp : BAD_VALUE;
    F.acc = 0;
    F.r_row = -1;
    F.r_col = -1;
    F.r_score = 0;
    F.next_row = 0;
    F.pend = false;
    F.pend_key = 0;
    F.end_v = BAD_VALUE;
    const int s_end = max_row >= 0 ? max_row + g.max_col(max_row) : -1;
    const int end_c = max_row >= 0 ? g.max_col(max_row) : -1;
    const bool stop_rule = A.max_errors != -1;

    // keeps the windows ahead of the steps [s, s + REFILL)
    auto window = [&](int s) {
        const int need = (s + REFILL + G + 2) / 2 + 2;
        bool wrote = false;
        while (F.loaded < need + 32) {
            uint32_t xa = F.pa[0], xb = F.pb[0];
#pragma unroll
            for (int i = 1; i < 8; i++) {
                xa = (lane & 7) == i ? F.pa[i] : xa;
                xb = (lane & 7) == i ? F.pb[i] : xb;
            }
            const int at = ((F.loaded >> 2) + (lane & 7)) & (LWIN / 4 - 1);
            if (lane < 8) wa32[at] = xa;
            else if (lane < 16) wb32[at] = xb;
            F.loaded += 32;
#pragma unroll
            for (int i = 0; i < 8; i++) {
                F.pa[i] = a32[(F.loaded >> 2) + i];
                F.pb[i] = b32[(F.loaded >> 2) + i];
            }
            wrote = true;
        }
        if (wrote) __syncthreads();
    };
    // stop test of the row completed on the previous step (:144-147); true = stop
    auto pending = [&]() -> bool {
        if (!F.pend) return false;
        F.pend = false;
        const int best = (int)(F.pend_key >> 32);
        if (best > A.max_errors) return true;
        F.r_row = F.next_row - 1;
        F.r_col = (int)(F.pend_key & 0xFFFFFFFFull);
        F.r_score = best;
        return false;
    };
    // row minima and the row that completes on step s (rows complete in order,
    // <= 1 per step); its minimum is tested at the top of the next step
    auto rows = [&](int s, bool live, int r, int c, int v) {
        if (live) atomicMin(&ring[r & (RING - 1)], ((unsigned long long)(unsigned)v << 32) | (unsigned)c);
        if (F.next_row <= max_row && F.next_row + g.max_col(F.next_row) == s) {
            F.pend_key = ring[F.next_row & (RING - 1)];
            if (lane == 0) ring[F.next_row & (RING - 1)] = ~0ull;  // LDS ops stay in order
            F.pend = true;
            F.next_row++;
        }
    };
    auto put_code = [&](int s, uint32_t code) {
        F.acc |= code << (2 * (s & 15));
        if ((s & 15) == 15) {
            track[(int64_t)(s >> 4) * 64 + lane] = F.acc;
            F.acc = 0;
        }
    };

    // the general step: frame, band edges and matrix ends (the first
    // gap_range + 2 anti-diagonals and the last ones)
    auto slow_step = [&](int s) {
        const int p = (s + G) & 1;
        const int q = 2 * lane + p;
        const int d = q - G;
        const int r = (s - d) >> 1, c = (s + d) >> 1;
        const int up_nb = from_lane_above(F.H0, BAD_VALUE);   // q+1 when p = 1
        const int left_nb = from_lane_below(F.H1, BAD_VALUE); // q-1 when p = 0
        const int Hd = p ? F.H1 : F.H0;
        int v = Hd;
        uint32_t code = 0;
        bool live = false;
        if (r >= 0 && c >= 0) {
            if (q > 2 * G || r > max_row || c > g.max_col(r)) {
                v = BAD_VALUE;
            } else {
                const int left = p ? F.H0 : (lane ? left_nb : (c == 0 ? (r + 1) * gp : BAD_VALUE));
                const int up = p ? up_nb : F.H1;
                const char x = wa[r & (LWIN - 1)];
                const int match = Hd + ((x == wb[c & (LWIN - 1)] && x != 'N') ? 0 : mm);
                const int gap1 = left + gp;
                const int gap2 = up + gp;
                v = min(match, min(gap1, gap2));
                code = v == match ? MATCH : v == gap1 ? COL_INC : ROW_INC;
                live = true;
                if (r == max_row && c == end_c) F.end_v = v;
            }
            if (p) F.H1 = v;
            else F.H0 = v;
        }
        put_code(s, code);
        if (stop_rule) rows(s, live, r, c, v);
    };

    // interior anti-diagonals: every band cell of the step is inside the
    // matrix and off the frame, so the step is branch-free
    const int L = min(max_row, min(g.cols - 1, g.side() - 1));
    const int f0 = G + 2;
    int f1 = min(s_end + 1, 2 * L - G);
    f1 = f1 < f0 + 2 ? f0 : f0 + ((f1 - f0) & ~1);  // whole step pairs (or none)
    const int lo0 = q0 > 2 * G ? BAD_VALUE : INT_MIN;  // out-of-band diagonals stay BAD
    const int lo1 = q1 > 2 * G ? BAD_VALUE : INT_MIN;

    int s = 0;
    bool stopped = false;
#ifdef NPGX_SA_PROFILE
    const long long t_start = clock64();
#endif
    for (; s < min(f0, s_end + 1); s++) {
        if ((stopped = pending())) break;
        if ((s & (REFILL - 1)) == 0) window(s);
        slow_step(s);
    }
    // pairs (s, s+1): step s on the lane's diagonal qa = 2j + P, step s+1 on
    // qb = 2j + 1 - P, P = (f0 + gap_range) & 1 for every pair
    auto fast = [&](auto PC) {
        constexpr int P = decltype(PC)::value;
        const int qa = 2 * lane + P, qb = 2 * lane + (1 - P);
        const int da = qa - G, db = qb - G;
        const int lo_a = P ? lo1 : lo0, lo_b = P ? lo0 : lo1;
        int ha = P ? F.H1 : F.H0;
        int hb = P ? F.H0 : F.H1;
        uint32_t ma = 0, mb = 0;
        int k = 16;
        for (; s < f1; s += 2, k++) {
            if (k == 16) {  // the next 16 pairs' substitution flags
                window(s);
                ma = mism16(wa32, wb32, (s - da) >> 1, (s + da) >> 1);
                mb = mism16(wa32, wb32, (s + 1 - db) >> 1, (s + 1 + db) >> 1);
                k = 0;
            }
            if (stop_rule && (stopped = pending())) break;
            {  // step s
                const int left = P == 0 ? from_lane_below(hb, BAD_VALUE) : hb;
                const int up = P == 0 ? hb : from_lane_above(hb, BAD_VALUE);
                const int match = ha + (int)((ma >> k) & 1u) * mm;
                const int gap1 = left + gp, gap2 = up + gp;
                const int v = min(match, min(gap1, gap2));
                put_code(s, v == match ? MATCH : v == gap1 ? COL_INC : ROW_INC);
                ha = max(v, lo_a);
                if (stop_rule) rows(s, qa <= 2 * G, (s - da) >> 1, (s + da) >> 1, ha);
            }
            if (stop_rule && (stopped = pending())) {
                s += 1;  // step s is done
                break;
            }
            {  // step s+1
                const int left = P == 0 ? ha : from_lane_below(ha, BAD_VALUE);
                const int up = P == 0 ? from_lane_above(ha, BAD_VALUE) : ha;
                const int match = hb + (int)((mb >> k) & 1u) * mm;
                const int gap1 = left + gp, gap2 = up + gp;
                const int v = min(match, min(gap1, gap2));
                put_code(s + 1, v == match ? MATCH : v == gap1 ? COL_INC : ROW_INC);
                hb = max(v, lo_b);
                if (stop_rule) rows(s + 1, qb <= 2 * G, (s + 1 - db) >> 1, (s + 1 + db) >> 1, hb);
            }
        }
        F.H0 = P ? hb : ha;
        F.H1 = P ? ha : hb;
    };
    if (!stopped && s == f0 && f1 > f0) {
        if ((f0 + G) & 1) fast(std::integral_constant<int, 1>{});
        else fast(std::integral_constant<int, 0>{});
    }
    const int s_tail = s;
    for (; s <= s_end && !stopped; s++) {
        if ((stopped = pending())) break;
        if ((s & (REFILL - 1)) == 0 || s == s_tail) window(s);
        slow_step(s);
    }
    if (!stopped && F.pend) pending();  // the last row's test
    {  // the last computed step's 16-step block, unless it was just stored
        const int last = s - 1;
        if (last >= 0 && (last & 15) != 15) track[(int64_t)(last >> 4) * 64 + lane] = F.acc;
    }
    int r_row = F.r_row, r_col = F.r_col, r_score = F.r_score;
    const int end_v = F.end_v;
    __threadfence();
    __syncthreads();
#ifdef NPGX_SA_PROFILE
    const long long t_fwd = clock64();
#endif

    int status = 0;
    int end_row = r_row, end_col = r_col, score = r_score;
    int forced_row = 0, forced_col = 0;  // max_errors == -1 completion (:151-172)
    if (!stop_rule) {
        end_row = max_row;
        end_col = end_c;
        const int last_row = g.rows - 1, last_col = g.cols - 1;
        if (end_row == last_row) {
            forced_col = last_col - end_col;
        } else if (end_col == last_col) {
            forced_row = last_row - end_row;
        } else {
            status = -1;  // "row and column are not last"
        }
        // at() of the completion cell: computed in the band, or BAD_VALUE for a
        // forced end (cells the reference never computes either)
        score = (forced_row || forced_col || end_row < 0)
                    ? BAD_VALUE
                    : __builtin_amdgcn_readlane(end_v, (end_col - end_row + G) >> 1);
    }
    if (status != 0) {
        if (lane == 0) {
            out[0] = -1;
            out[1] = -1;
            out[2] = 0;
            out[3] = status;
            out[4] = 0;
        }
        return;
    }

    // traceback reader: 16-step blocks of directions, one coalesced load each,
    // in batches of 4 blocks with the next batch down loaded one batch ahead
    // (a single wait per batch); a cell's 2 bits by readlane
    int batch = INT_MIN;
    uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, n0 = 0, n1 = 0, n2 = 0, n3 = 0;
    const int n_blk = s_end >= 0 ? (s_end >> 4) + 1 : 0;  // blocks of this pair's track region
    auto load4 = [&](int bt, uint32_t& x0, uint32_t& x1, uint32_t& x2, uint32_t& x3) {
        const int b0 = 4 * bt;  // only blocks inside the region are read
        x0 = (b0 >= 0 && b0 < n_blk) ? track[(int64_t)b0 * 64 + lane] : 0u;
        x1 = (b0 + 1 >= 0 && b0 + 1 < n_blk) ? track[(int64_t)(b0 + 1) * 64 + lane] : 0u;
        x2 = (b0 + 2 >= 0 && b0 + 2 < n_blk) ? track[(int64_t)(b0 + 2) * 64 + lane] : 0u;
        x3 = (b0 + 3 >= 0 && b0 + 3 < n_blk) ? track[(int64_t)(b0 + 3) * 64 + lane] : 0u;
    };
    auto code_at = [&](int r, int c) -> int {
        if (r < 0 && c < 0) return -1;
        if (r < 0) return COL_INC;   // make_frame :399-406
        if (c < 0) return ROW_INC;   // :391-398
        const int ss = r + c;
        const int nb = ss >> 4, bt = nb >> 2;
        if (bt != batch) {
            if (bt == batch - 1) {
                c0 = n0;
                c1 = n1;
                c2 = n2;
                c3 = n3;
            } else {
                load4(bt, c0, c1, c2, c3);
            }
            load4(bt - 1, n0, n1, n2, n3);
            batch = bt;
        }
        const int i = nb & 3;
        const uint32_t w = i == 0 ? c0 : i == 1 ? c1 : i == 2 ? c2 : c3;
        const int owner = (c - r + G) >> 1;
        const uint32_t word = (uint32_t)__builtin_amdgcn_readlane((int)w, owner);
        return (int)((word >> (2 * (ss & 15))) & 3u);
    };
    auto go_prev = [&](int code, int& r, int& c) {
        if (code == MATCH || code == ROW_INC) r -= 1;
        if (code == MATCH || code == COL_INC) c -= 1;
    };
    if (A.cut_tail) {  // cut_tail (:240-255), max_errors != -1 only
        while (end_row >= 0 || end_col >= 0) {
            const int code = code_at(end_row, end_col);
            const int cost = (end_row >= 0 && end_col >= 0) ? (code == MATCH ? sub(a, b, end_row, end_col, mm) : gp)
                                                            : gp;
            if (cost <= 0) break;
            score -= cost;
            go_prev(code, end_row, end_col);
        }
    }
    // export_alignment (:262-282), backwards from out_end
    int8_t* o = A.ops + P.out_end;
    int n = 0;
    int8_t obuf = 0;
    auto emit = [&](int code) {
        if ((n & 63) == lane) obuf = (int8_t)code;
        n++;
        if ((n & 63) == 0) {
            o[-(int64_t)(n - 64 + lane) - 1] = obuf;
        }
    };
    for (int i = 0; i < forced_col; i++) emit(COL_INC);
    for (int i = 0; i < forced_row; i++) emit(ROW_INC);
    {
        int r = end_row, c = end_col;
        while (r >= 0 || c >= 0) {
            const int code = code_at(r, c);
            emit(code);
            go_prev(code, r, c);
        }
    }
    if ((n & 63) && lane < (n & 63)) o[-(int64_t)((n & ~63) + lane) - 1] = obuf;
    if (lane == 0) {
        out[0] = end_row + forced_row;
        out[1] = end_col + forced_col;
        out[2] = score;
        out[3] = 0;
        out[4] = n;
#ifdef NPGX_SA_PROFILE
        out[5] = (int32_t)((t_fwd - t_start) >> 4);
        out[6] = (int32_t)((clock64() - t_fwd) >> 4);
        out[7] = s_end + 1;
#endif
    }
}

}  // namespace ga
}  // namespace npgx

using namespace npgx;
using namespace npgx::ga;

struct npgx_dp {
    npgx_dp_options opt;
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf<char> d_a, d_b;
    DevBuf<Pair> d_pairs;
    DevBuf<uint32_t> d_track;
    DevBuf<int8_t> d_ops;
    DevBuf<int32_t> d_res;
    PinnedArena pinned;
    StageTimer timer;
    bool has_result = false;
    std::vector<int32_t> res;        // RES per pair
    std::vector<int64_t> op_off;     // n_pairs + 1
    std::vector<int8_t> ops;         // forward order
    int64_t cells = 0;
};

namespace npgx {
namespace ga {

static int64_t band_steps(int la, int lb, int gr) {  // anti-diagonals of the band
    const int side = std::min(std::min(la, lb) + gr, std::max(la, lb));
    const int max_row = std::min(la, side) - 1;
    if (max_row < 0) return 0;
    const int mc = std::min(lb - 1, std::min(side - 1, max_row + gr));
    return (int64_t)max_row + mc + 1;
}

static int64_t band_cells(int la, int lb, int gr) {
    const int side = std::min(std::min(la, lb) + gr, std::max(la, lb));
    const int max_row = std::min(la, side) - 1;
    int64_t n = 0;
    for (int r = 0; r <= max_row; r++) {
        const int c0 = std::max(0, r - gr), c1 = std::min(lb - 1, std::min(side - 1, r + gr));
        if (c1 >= c0) n += c1 - c0 + 1;
    }
    return n;
}

static void dp_run(npgx_dp* D, const char* first, const int64_t* first_off, const char* second,
                   const int64_t* second_off, int32_t n) {
    NPGX_HIP(hipSetDevice(D->device));
    hipStream_t st = D->stream;
    D->timer.reset();
    D->has_result = false;
    const npgx_dp_options& o = D->opt;
    NPGX_REQUIRE(n >= 0, NPGX_ERR_ARG, "n_pairs < 0");
    // device layout: every pair's letters start 16-byte aligned (the kernel
    // reads them as dwords with scalar loads), 64 bytes of slack at the end
    std::vector<Pair> pairs((size_t)n);
    D->op_off.assign((size_t)n + 1, 0);
    int64_t tw = 0, oc = 0, pa = 0, pb = 0;
    D->cells = 0;
    for (int32_t i = 0; i < n; i++) {
        const int64_t la = first_off[i + 1] - first_off[i], lb = second_off[i + 1] - second_off[i];
        NPGX_REQUIRE(la >= 0 && lb >= 0 && la < (1 << 30) && lb < (1 << 30), NPGX_ERR_RANGE,
                     "sequence length out of range");
        Pair& P = pairs[(size_t)i];
        P.a_off = pa;
        P.b_off = pb;
        pa += (la + 15) & ~15ll;
        pb += (lb + 15) & ~15ll;
        P.la = (int32_t)la;
        P.lb = (int32_t)lb;
        P.track_off = tw;
        tw += (band_steps(P.la, P.lb, o.gap_range) + 15) / 16 * 64;
        oc += la + lb;
        P.out_end = oc;
        D->cells += band_cells(P.la, P.lb, o.gap_range);
    }
    const int64_t abytes = pa + 64, bbytes = pb + 64;
    NPGX_REQUIRE(tw < (1ll << 36), NPGX_ERR_RANGE, "traceback store over 256 GiB");
    D->d_a.grow((size_t)abytes);
    D->d_b.grow((size_t)bbytes);
    D->d_pairs.grow((size_t)std::max(n, 1));
    D->d_track.grow((size_t)std::max<int64_t>(tw, 1));
    D->d_ops.grow((size_t)std::max<int64_t>(oc, 1));
    D->d_res.grow((size_t)std::max(n, 1) * RES);
    auto put = [&](void* d, const void* h, size_t bytes) {
        if (!bytes) return;
        char* p = D->pinned.take(bytes, st);
        memcpy(p, h, bytes);
        NPGX_HIP(hipMemcpyAsync(d, p, bytes, hipMemcpyHostToDevice, st));
    };
    auto put_letters = [&](char* d, const char* src, const int64_t* off, int64_t bytes, bool first_seq) {
        char* p = D->pinned.take((size_t)bytes, st);
        memset(p + bytes - 64, 0, 64);
        for (int32_t i = 0; i < n; i++) {
            const int64_t len = off[i + 1] - off[i];
            const int64_t at = first_seq ? pairs[(size_t)i].a_off : pairs[(size_t)i].b_off;
            memcpy(p + at, src + off[i], (size_t)len);
            memset(p + at + len, 0, (size_t)(((len + 15) & ~15ll) - len));
        }
        NPGX_HIP(hipMemcpyAsync(d, p, (size_t)bytes, hipMemcpyHostToDevice, st));
    };
    put_letters(D->d_a.p, first, first_off, abytes, true);
    put_letters(D->d_b.p, second, second_off, bbytes, false);
    put(D->d_pairs.p, pairs.data(), pairs.size() * sizeof(Pair));
    if (n) {
        GaArgs A{D->d_a.p, D->d_b.p, D->d_pairs.p, D->d_track.p, D->d_ops.p, D->d_res.p,
                 o.gap_range, o.max_errors, o.gap_penalty, o.mismatch_penalty, o.cut_tail, 0};
        // algorithmic bytes: letters in, 2 bits per band cell out, ops out
        const double bytes = double(oc) + 0.25 * double(D->cells) + double(oc);
        size_t ti = D->timer.begin("general_align", st, bytes, D->cells);
        hipLaunchKernelGGL(k_general_align, dim3((unsigned)n), dim3(64), 0, st, A);
        NPGX_HIP(hipGetLastError());
        D->timer.end(ti, st);
    }
    D->res.assign((size_t)n * RES, 0);
    std::vector<int8_t> raw((size_t)oc);
    if (n) {
        NPGX_HIP(hipMemcpyAsync(D->res.data(), D->d_res.p, (size_t)n * RES * 4, hipMemcpyDeviceToHost, st));
        if (oc) NPGX_HIP(hipMemcpyAsync(raw.data(), D->d_ops.p, (size_t)oc, hipMemcpyDeviceToHost, st));
    }
    NPGX_HIP(stream_wait(st));
    D->pinned.reset();
    D->ops.clear();
    for (int32_t i = 0; i < n; i++) {
        const int32_t k = D->res[(size_t)i * RES + 4];
        const int64_t end = pairs[(size_t)i].out_end;
        D->ops.insert(D->ops.end(), raw.begin() + (end - k), raw.begin() + end);
        D->op_off[(size_t)i + 1] = (int64_t)D->ops.size();
    }
    D->has_result = true;
}

}  // namespace ga
}  // namespace npgx

extern "C" {

void npgx_dp_default_options(npgx_dp_options* o) {
    if (!o) return;
    memset(o, 0, sizeof(*o));
    // GeneralAligner::GeneralAligner (:39-41) and the nucleotide substitution
    o->gap_range = 1;
    o->max_errors = 0;
    o->gap_penalty = 1;
    o->mismatch_penalty = 1;
    o->cut_tail = 0;
}

int npgx_dp_create(const npgx_dp_options* o, npgx_dp** out) {
    return guard([&] {
        NPGX_REQUIRE(o && out, NPGX_ERR_ARG, "null argument");
        NPGX_REQUIRE(o->gap_range >= 0 && o->gap_range <= 63, NPGX_ERR_RANGE,
                     "gap_range must be in [0, 63] (one wave covers 2*gap_range+1 diagonals)");
        NPGX_REQUIRE(o->max_errors >= -1, NPGX_ERR_ARG, "max_errors < -1");
        NPGX_REQUIRE(o->gap_penalty >= 0 && o->mismatch_penalty >= 0, NPGX_ERR_ARG,
                     "penalties must be >= 0");
        NPGX_REQUIRE(!(o->cut_tail && o->max_errors == -1), NPGX_ERR_ARG,
                     "cut_tail needs max_errors >= 0 (the completed cells have no scores)");
        int dev = current_device_checked();
        auto* D = new npgx_dp;
        D->opt = *o;
        D->device = dev;
        if (hipStreamCreateWithFlags(&D->stream, hipStreamNonBlocking) != hipSuccess) {
            delete D;
            throw Error(NPGX_ERR_HIP, "stream creation failed");
        }
        *out = D;
    });
}

int npgx_dp_align_batch(npgx_dp* D, const char* first, const int64_t* first_off, const char* second,
                        const int64_t* second_off, int32_t n_pairs) {
    return guard([&] {
        NPGX_REQUIRE(D && first_off && second_off && (n_pairs == 0 || (first && second)), NPGX_ERR_ARG,
                     "null argument");
        dp_run(D, first, first_off, second, second_off, n_pairs);
    });
}

int npgx_dp_result_counts(const npgx_dp* D, int64_t* n_pairs, int64_t* total_ops) {
    return guard([&] {
        NPGX_REQUIRE(D && n_pairs && total_ops, NPGX_ERR_ARG, "null argument");
        NPGX_REQUIRE(D->has_result, NPGX_ERR_STATE, "no GeneralAligner result yet");
        *n_pairs = (int64_t)D->op_off.size() - 1;
        *total_ops = (int64_t)D->ops.size();
    });
}

int npgx_dp_result_copy(const npgx_dp* D, int32_t* first_last, int32_t* second_last, int32_t* score,
                        int32_t* status, int64_t* op_off, int8_t* ops) {
    return guard([&] {
        NPGX_REQUIRE(D, NPGX_ERR_ARG, "null argument");
        NPGX_REQUIRE(D->has_result, NPGX_ERR_STATE, "no GeneralAligner result yet");
        const size_t n = D->op_off.size() - 1;
        for (size_t i = 0; i < n; i++) {
            if (first_last) first_last[i] = D->res[i * RES + 0];
            if (second_last) second_last[i] = D->res[i * RES + 1];
            if (score) score[i] = D->res[i * RES + 2];
            if (status) status[i] = D->res[i * RES + 3];
        }
        if (op_off) memcpy(op_off, D->op_off.data(), D->op_off.size() * 8);
        if (ops && !D->ops.empty()) memcpy(ops, D->ops.data(), D->ops.size());
    });
}

int npgx_dp_phase_cycles(const npgx_dp* D, int64_t* fwd, int64_t* back, int64_t* steps) {
    return guard([&] {
        NPGX_REQUIRE(D && fwd && back && steps, NPGX_ERR_ARG, "null argument");
        NPGX_REQUIRE(D->has_result, NPGX_ERR_STATE, "no GeneralAligner result yet");
#ifdef NPGX_SA_PROFILE
        *fwd = *back = *steps = 0;
        for (size_t i = 0; i + RES <= D->res.size(); i += RES) {
            *fwd += 16ll * D->res[i + 5];
            *back += 16ll * D->res[i + 6];
            *steps += D->res[i + 7];
        }
#else
        throw Error(NPGX_ERR_STATE, "phase cycles need the diagnostic build (NPGX_PROFILE=1)");
#endif
    });
}

int npgx_dp_kernel_times(const npgx_dp* D, npgx_kernel_time* out, int32_t cap, int32_t* n) {
    return guard([&] {
        NPGX_REQUIRE(D && n && (out || cap == 0), NPGX_ERR_ARG, "null argument");
        D->timer.copy_out(out, cap, n);
    });
}

void npgx_dp_free(npgx_dp* D) {
    if (!D) return;
    (void)hipSetDevice(D->device);
    if (D->stream) (void)hipStreamDestroy(D->stream);
    delete D;
}

}  // extern "C"
