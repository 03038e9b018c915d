// general_aligner.cpp -- CPU restatement of GeneralAligner (banded min-cost
// Needleman-Wunsch with a gap frame and an error stop rule) on nucleotide
// contents.  TEST INFRASTRUCTURE ONLY (the checker of npgx_dp_*).
//
// Follows src/util/GeneralAligner.hpp (NPG-explorer 0.5.8):
//   align()            :113-173   row loop, band [min_col, max_col], min/left/up
//                                 with MATCH > COL_INC > ROW_INC tie order,
//                                 first-minimum column per row, max_errors stop,
//                                 max_errors == -1 completion to the last cell
//   cut_tail()         :240-255   walk back while the previous cell scores lower
//   export_alignment() :262-282   traceback to (-1, -1)
//   side/max_row/min_col/max_col :300-316, limit_range :377-386, make_frame :388-407
// The nucleotide contents' substitution is the one FragmentDistance.cpp:18-21
// keeps for PairAligner: 0 if a == b and a != 'N', else 1 (here a parameter).
// The reference has no test of GeneralAligner: the restatement is pinned by
// textbook edit-distance known answers (tests/test_oracle_dp.py); band, stop
// rule and tie-breaking follow the code above ("parity unpinned" beyond that).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

namespace orc_ga {

enum { MATCH = 0, ROW_INC = 1, COL_INC = 2 };  // GeneralAligner::Track (+1 / -1 renamed)
static const int BAD_VALUE = 1000000;          // :24

struct GA {
    const char* a;
    const char* b;
    int rows, cols, gr, max_errors, gp, mm;
    // The reference keeps the whole (rows+1) x (cols+1) matrix; here only the
    // diagonal band |c - r| <= gr + 1 is stored densely (every cell align()
    // computes or limit_range() marks) and the few other cells it touches --
    // the frame, max_errors == -1's completion run -- live in a map whose
    // default is the matrix's initial value (BAD_VALUE, MATCH).  Same values,
    // so 100 kb pairs fit in memory.
    struct Cell {
        int s = BAD_VALUE, t = MATCH;
    };
    std::vector<Cell> band;
    std::unordered_map<int64_t, Cell> off;

    int bw() const { return 2 * gr + 3; }
    Cell& cell(int r, int c) {
        const int d = c - r;
        if (d >= -(gr + 1) && d <= gr + 1) return band[(size_t)(r + 1) * bw() + (d + gr + 1)];
        return off[(int64_t)(r + 1) * (cols + 1) + (c + 1)];
    }
    int& at(int r, int c) { return cell(r, c).s; }
    int& tr(int r, int c) { return cell(r, c).t; }
    bool in(int r, int c) const { return -1 <= r && r < rows && -1 <= c && c < cols; }
    int side() const { return std::min(std::min(rows, cols) + gr, std::max(rows, cols)); }
    int max_row() const { return std::min(rows, side()) - 1; }
    int min_col(int r) const { return std::max(0, r - gr); }
    int max_col(int r) const { return std::min(cols - 1, std::min(side() - 1, r + gr)); }
    int sub(int r, int c) const { return (a[r] == b[c] && a[r] != 'N') ? 0 : mm; }

    void go_prev(int& r, int& c) {
        const int t = tr(r, c);
        if (t == MATCH || t == ROW_INC) r -= 1;
        if (t == MATCH || t == COL_INC) c -= 1;
    }

    // returns false where the reference throws "row and column are not last"
    bool align(int& r_row, int& r_col) {
        band.assign((size_t)(rows + 1) * bw(), Cell());
        off.clear();
        for (int r = -1; r < rows; r++)  // limit_range
            for (int o = -1; o <= 1; o += 2) {
                const int c = r + o * (gr + 1);
                if (in(r, c)) at(r, c) = BAD_VALUE;
            }
        at(-1, -1) = 0;  // make_frame
        for (int r = 0; r < rows; r++) {
            at(r, -1) = (r + 1) * gp;
            tr(r, -1) = ROW_INC;
        }
        for (int c = 0; c < cols; c++) {
            at(-1, c) = (c + 1) * gp;
            tr(-1, c) = COL_INC;
        }
        r_row = r_col = -1;
        for (int r = 0; r <= max_row(); r++) {
            const int c0 = min_col(r), c1 = max_col(r);
            int best = c0;
            for (int c = c0; c <= c1; c++) {
                const int match = at(r - 1, c - 1) + sub(r, c);
                const int gap1 = at(r, c - 1) + gp;
                const int gap2 = at(r - 1, c) + gp;
                const int s = std::min(match, std::min(gap1, gap2));
                at(r, c) = s;
                if (s < at(r, best)) best = c;
                tr(r, c) = s == match ? MATCH : s == gap1 ? COL_INC : ROW_INC;
            }
            if (max_errors != -1 && at(r, best) > max_errors) break;
            r_row = r;
            r_col = best;
        }
        if (max_errors == -1) {
            r_col = max_col(max_row());
            const int last_row = rows - 1, last_col = cols - 1;
            if (r_row == last_row) {
                while (r_col < last_col) tr(r_row, ++r_col) = COL_INC;
            } else if (r_col == last_col) {
                while (r_row < last_row) tr(++r_row, r_col) = ROW_INC;
            } else {
                return false;
            }
        }
        return true;
    }

    void cut_tail(int& r_row, int& r_col) {
        while (true) {
            int pr = r_row, pc = r_col;
            go_prev(pr, pc);
            if (in(pr, pc) && at(pr, pc) < at(r_row, r_col)) {
                r_row = pr;
                r_col = pc;
            } else {
                break;
            }
        }
    }

    int export_ops(int r, int c, int8_t* ops) {  // forward order
        int n = 0;
        while (r != -1 || c != -1) {
            ops[n++] = (int8_t)tr(r, c);
            go_prev(r, c);
        }
        std::reverse(ops, ops + n);
        return n;
    }
};

}  // namespace orc_ga

extern "C" {

// One pair.  ops needs la + lb entries.  Returns 0, -1 for the reference's
// "row and column are not last" exception, -2 for an empty sequence.
int orc_ga_align(const char* a, int la, const char* b, int lb, int gap_range, int max_errors,
                 int gap_penalty, int mismatch_penalty, int cut_tail, int* first_last,
                 int* second_last, int* score, int8_t* ops, int* n_ops) {
    *n_ops = 0;
    *first_last = *second_last = -1;
    *score = 0;
    if (la == 0 || lb == 0) return -2;  // outside the reference's contract (find_aln :612-615)
    orc_ga::GA g{a, b, la, lb, gap_range, max_errors, gap_penalty, mismatch_penalty, {}, {}};
    int r = -1, c = -1;
    if (!g.align(r, c)) return -1;
    if (cut_tail && r >= 0) g.cut_tail(r, c);
    *first_last = r;
    *second_last = c;
    *score = g.at(r, c);
    *n_ops = g.export_ops(r, c, ops);
    return 0;
}

}  // extern "C"
