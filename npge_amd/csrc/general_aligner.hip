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
#include <cstring>

#include "common.hpp"

namespace npgx {
namespace ga {

static constexpr int BAD_VALUE = 1000000;   // GeneralAligner.hpp:24
static constexpr int RING = 256;            // open rows (<= gap_range + 2 at a time)
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

__global__ __launch_bounds__(64) void k_general_align(GaArgs A) {
    __shared__ unsigned long long ring[RING];
    const int lane = threadIdx.x;
    const Pair P = A.pairs[blockIdx.x];
    const char* a = A.a + P.a_off;
    const char* b = A.b + P.b_off;
    uint32_t* track = A.track + P.track_off;
    const int G = A.gr, gp = A.gp, mm = A.mm;
    const Geo g{P.la, P.lb, G};
    const int max_row = g.max_row();
    if (P.la == 0 || P.lb == 0) {  // find_aln handles these without the aligner (:612-615)
        if (lane == 0) {
            int32_t* out = A.res + (int64_t)blockIdx.x * 5;
            out[0] = -1;
            out[1] = -1;
            out[2] = 0;
            out[3] = -2;
            out[4] = 0;
        }
        return;
    }
    for (int i = lane; i < RING; i += 64) ring[i] = ~0ull;
    __syncthreads();

    // registers: the last value on each owned diagonal (frame value at start)
    const int q0 = 2 * lane, q1 = 2 * lane + 1;
    int H0 = q0 <= 2 * G + 1 ? abs(q0 - G) * gp : BAD_VALUE;
    int H1 = q1 <= 2 * G + 1 ? abs(q1 - G) * gp : BAD_VALUE;
    int r_row = -1, r_col = -1, r_score = 0;
    int next_row = 0;
    uint32_t acc = 0;
    const int s_end = max_row >= 0 ? max_row + g.max_col(max_row) : -1;
    int s = 0;
    for (; s <= s_end; s++) {
        const int p = (s + G) & 1;
        const int q = 2 * lane + p;
        const int d = q - G;
        const int r = (s - d) >> 1, c = (s + d) >> 1;
        const int up_nb = __shfl_down(H0, 1);   // lane+1's even diagonal = q+1 when p = 1
        const int left_nb = __shfl_up(H1, 1);   // lane-1's odd diagonal = q-1 when p = 0
        const int Hd = p ? H1 : H0;
        int v = Hd;
        uint32_t code = 0;
        bool live = false;
        if (r >= 0 && c >= 0) {
            if (q > 2 * G || r > max_row || c > g.max_col(r)) {
                v = BAD_VALUE;
            } else {
                int left = p ? H0 : (lane ? left_nb : (c == 0 ? (r + 1) * gp : BAD_VALUE));
                int up = p ? (lane < 63 ? up_nb : BAD_VALUE) : H1;
                const int match = Hd + sub(a, b, r, c, mm);
                const int gap1 = left + gp;
                const int gap2 = up + gp;
                v = min(match, min(gap1, gap2));
                code = v == match ? MATCH : v == gap1 ? COL_INC : ROW_INC;
                live = true;
            }
            if (p) H1 = v;
            else H0 = v;
        }
        acc |= code << (2 * (s & 15));
        if ((s & 15) == 15) {
            track[(int64_t)(s >> 4) * 64 + lane] = acc;
            acc = 0;
        }
        if (live) atomicMin(&ring[r & (RING - 1)], ((unsigned long long)(unsigned)v << 32) | (unsigned)c);
        // the row that completes on this step (rows complete in order, <= 1 per step)
        if (next_row <= max_row && next_row + g.max_col(next_row) == s) {
            const unsigned long long key = ring[next_row & (RING - 1)];
            __syncthreads();  // single wave: orders the read before the reset
            if (lane == 0) ring[next_row & (RING - 1)] = ~0ull;
            const int best = (int)(key >> 32);
            if (A.max_errors != -1 && best > A.max_errors) break;
            r_row = next_row;
            r_col = (int)(key & 0xFFFFFFFFull);
            r_score = best;
            next_row++;
        }
    }
    {  // the last step's 16-step block, unless it was just stored
        const int last = min(s, s_end);
        if (last >= 0 && (last & 15) != 15) track[(int64_t)(last >> 4) * 64 + lane] = acc;
    }
    __threadfence();
    __syncthreads();

    int32_t* out = A.res + (int64_t)blockIdx.x * 5;
    int status = 0;
    int end_row = r_row, end_col = r_col, score = r_score;
    int forced_row = 0, forced_col = 0;  // max_errors == -1 completion (:151-172)
    if (A.max_errors == -1) {
        end_row = max_row;
        end_col = max_row >= 0 ? g.max_col(max_row) : min(g.cols - 1, min(g.side() - 1, G - 1));
        const int last_row = g.rows - 1, last_col = g.cols - 1;
        if (end_row == last_row) {
            forced_col = last_col - end_col;
        } else if (end_col == last_col) {
            forced_row = last_row - end_row;
        } else {
            status = -1;  // "row and column are not last"
        }
        score = 0;
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

    // traceback reader: one coalesced load per 16-step block, 2 bits by readlane
    int blk = -1;
    uint32_t w = 0;
    auto code_at = [&](int r, int c) -> int {
        if (r < 0 && c < 0) return -1;
        if (r < 0) return COL_INC;   // make_frame :399-406
        if (c < 0) return ROW_INC;   // :391-398
        const int ss = r + c;
        if ((ss >> 4) != blk) {
            blk = ss >> 4;
            w = track[(int64_t)blk * 64 + lane];
        }
        const int owner = (c - r + G) >> 1;
        const uint32_t word = (uint32_t)__builtin_amdgcn_readlane((int)w, owner);
        return (int)((word >> (2 * (ss & 15))) & 3u);
    };
    auto step_cost = [&](int code, int r, int c) -> int {
        return code == MATCH ? sub(a, b, r, c, mm) : gp;
    };
    auto go_prev = [&](int code, int& r, int& c) {
        if (code == MATCH || code == ROW_INC) r -= 1;
        if (code == MATCH || code == COL_INC) c -= 1;
    };
    if (A.max_errors == -1) {
        // the in-band score of the completion cell, or BAD_VALUE for a forced end
        // (those cells are never computed by the reference either)
        if (forced_row || forced_col || end_row < 0) score = BAD_VALUE;
        else {  // replay the path's costs from the start (exact: at() = sum of step costs)
            int r = end_row, c = end_col, acc_s = 0;
            while (r >= 0 || c >= 0) {
                const int code = code_at(r, c);
                acc_s += (r >= 0 && c >= 0) ? step_cost(code, r, c) : gp;
                go_prev(code, r, c);
            }
            score = acc_s;
        }
    }
    if (A.cut_tail && end_row >= -1) {  // cut_tail (:240-255), max_errors != -1 only
        while (end_row >= 0 || end_col >= 0) {
            const int code = code_at(end_row, end_col);
            const int cost = (end_row >= 0 && end_col >= 0) ? step_cost(code, end_row, end_col) : gp;
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
    std::vector<int32_t> res;        // 5 per pair
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
    const int64_t a0 = n ? first_off[0] : 0, b0 = n ? second_off[0] : 0;
    const int64_t abytes = n ? first_off[n] - a0 : 0, bbytes = n ? second_off[n] - b0 : 0;
    std::vector<Pair> pairs((size_t)n);
    D->op_off.assign((size_t)n + 1, 0);
    int64_t tw = 0, oc = 0;
    D->cells = 0;
    for (int32_t i = 0; i < n; i++) {
        const int64_t la = first_off[i + 1] - first_off[i], lb = second_off[i + 1] - second_off[i];
        NPGX_REQUIRE(la >= 0 && lb >= 0 && la < (1 << 30) && lb < (1 << 30), NPGX_ERR_RANGE,
                     "sequence length out of range");
        Pair& P = pairs[(size_t)i];
        P.a_off = first_off[i] - a0;
        P.b_off = second_off[i] - b0;
        P.la = (int32_t)la;
        P.lb = (int32_t)lb;
        P.track_off = tw;
        tw += (band_steps(P.la, P.lb, o.gap_range) + 15) / 16 * 64;
        oc += la + lb;
        P.out_end = oc;
        D->cells += band_cells(P.la, P.lb, o.gap_range);
    }
    NPGX_REQUIRE(tw < (1ll << 36), NPGX_ERR_RANGE, "traceback store over 256 GiB");
    D->d_a.grow((size_t)std::max<int64_t>(abytes, 1));
    D->d_b.grow((size_t)std::max<int64_t>(bbytes, 1));
    D->d_pairs.grow((size_t)std::max(n, 1));
    D->d_track.grow((size_t)std::max<int64_t>(tw, 1));
    D->d_ops.grow((size_t)std::max<int64_t>(oc, 1));
    D->d_res.grow((size_t)std::max(n, 1) * 5);
    auto put = [&](void* d, const void* h, size_t bytes) {
        if (!bytes) return;
        char* p = D->pinned.take(bytes, st);
        memcpy(p, h, bytes);
        NPGX_HIP(hipMemcpyAsync(d, p, bytes, hipMemcpyHostToDevice, st));
    };
    put(D->d_a.p, first + a0, (size_t)abytes);
    put(D->d_b.p, second + b0, (size_t)bbytes);
    put(D->d_pairs.p, pairs.data(), pairs.size() * sizeof(Pair));
    if (n) {
        GaArgs A{D->d_a.p, D->d_b.p, D->d_pairs.p, D->d_track.p, D->d_ops.p, D->d_res.p,
                 o.gap_range, o.max_errors, o.gap_penalty, o.mismatch_penalty, o.cut_tail, 0};
        // algorithmic bytes: letters in, 2 bits per band cell out, ops out
        const double bytes = double(abytes + bbytes) + 0.25 * double(D->cells) + double(oc);
        size_t ti = D->timer.begin("general_align", st, bytes, D->cells);
        hipLaunchKernelGGL(k_general_align, dim3((unsigned)n), dim3(64), 0, st, A);
        NPGX_HIP(hipGetLastError());
        D->timer.end(ti, st);
    }
    D->res.assign((size_t)n * 5, 0);
    std::vector<int8_t> raw((size_t)oc);
    if (n) {
        NPGX_HIP(hipMemcpyAsync(D->res.data(), D->d_res.p, (size_t)n * 5 * 4, hipMemcpyDeviceToHost, st));
        if (oc) NPGX_HIP(hipMemcpyAsync(raw.data(), D->d_ops.p, (size_t)oc, hipMemcpyDeviceToHost, st));
    }
    NPGX_HIP(hipStreamSynchronize(st));
    D->pinned.reset();
    D->ops.clear();
    for (int32_t i = 0; i < n; i++) {
        const int32_t k = D->res[(size_t)i * 5 + 4];
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
            if (first_last) first_last[i] = D->res[i * 5 + 0];
            if (second_last) second_last[i] = D->res[i * 5 + 1];
            if (score) score[i] = D->res[i * 5 + 2];
            if (status) status[i] = D->res[i * 5 + 3];
        }
        if (op_off) memcpy(op_off, D->op_off.data(), D->op_off.size() * 8);
        if (ops && !D->ops.empty()) memcpy(ops, D->ops.data(), D->ops.size());
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
