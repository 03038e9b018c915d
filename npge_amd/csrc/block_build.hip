// block_build.hip -- the block build around the anchors: the Processor/BlockSet
// surface of the DraftPangenome path (src/algo/lua_lib.lua:1569-1621).
//
// Blocks live on the host as fragments + gapped rows; every alignment problem of
// a processor pass is gathered into ONE batch for the GPU aligner
// (similar_aligner.hip): FragmentsExtender aligns the right and the left flank
// of every block in the same launch.  The bookkeeping between the batches
// (FixEnds' frame scan, OverlaplessUnion's greedy admission, MoveUnchanged's
// hash set, Filter's slice search) is sequential per block and runs in host C++.
//
// Pinned conventions (the reference breaks these ties by pointer order):
//   OverlaplessUnion admits blocks by (size desc, alignment length desc,
//   name desc), then by the smallest fragment (Fragment::operator< with the
//   sequence's input index for Sequence*), then by the sorted fragment list.
#include <algorithm>
#include <chrono>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <tuple>

#include "common.hpp"

namespace npgx {
namespace bb {

struct Frag {
    int32_t seq;
    int32_t ori;
    int64_t min, max;
    int64_t len() const { return max - min + 1; }
    int64_t begin() const { return ori == 1 ? min : max; }
};

struct Block {
    std::vector<Frag> f;
    std::vector<std::string> rows;  // empty = no alignment
    std::string name;
    bool has_rows() const { return !rows.empty(); }
    int64_t aln_len() const {
        if (f.empty()) return 0;
        return has_rows() ? (int64_t)rows[0].size() : f[0].len();
    }
};

static inline char compl_char(char c) {
    switch (c) {
        case 'A': return 'T';
        case 'T': return 'A';
        case 'G': return 'C';
        case 'C': return 'G';
        default: return c;
    }
}

// text of [begin, begin + ori*len) read in orientation ori (Sequence::substr)
static std::string seq_text(const std::string& s, int64_t begin, int64_t len, int ori) {
    std::string r((size_t)len, ' ');
    if (ori == 1) {
        memcpy(&r[0], s.data() + begin, (size_t)len);
    } else {
        for (int64_t i = 0; i < len; i++) r[(size_t)i] = compl_char(s[(size_t)(begin - i)]);
    }
    return r;
}

static void revcomp_inplace(std::string& s) {  // complement(std::string&) keeps '-'
    std::reverse(s.begin(), s.end());
    for (char& c : s) c = compl_char(c);
}

}  // namespace bb
}  // namespace npgx

using namespace npgx;
using namespace npgx::bb;

struct npgx_blockset {
    const npgx_seqset* ss = nullptr;
    npgx_bb_options opt;
    std::vector<Block> blocks;
    npgx_aligner* aligner = nullptr;
    npgx_aligner* dummy = nullptr;
    npgx_bb_stats stats{};
    StageTimer timer;        // only host-visible timings are kept here
    std::vector<npgx_kernel_time> ktimes;
    std::vector<int64_t> job_stats;  // aligner per-job statistics of the last apply
    const std::string& text(int32_t seq) const { return ss->data[(size_t)seq]; }
};

namespace npgx {
namespace bb {

using Clock = std::chrono::steady_clock;
static double ms_since(Clock::time_point t) {
    return std::chrono::duration<double, std::milli>(Clock::now() - t).count();
}

static void collect_kernel_times(npgx_blockset* B) {
    npgx_kernel_time kt[16];
    int32_t n = 0;
    if (npgx_align_kernel_times(B->aligner, kt, 16, &n) == NPGX_OK)
        for (int32_t i = 0; i < std::min<int32_t>(n, 16); i++) B->ktimes.push_back(kt[i]);
    int64_t nj = 0;
    if (npgx_align_job_stats(B->aligner, nullptr, 0, &nj) == NPGX_OK && nj > 0) {
        const size_t o = B->job_stats.size();
        B->job_stats.resize(o + (size_t)nj * 8);
        npgx_align_job_stats(B->aligner, B->job_stats.data() + o, nj, &nj);
    }
}

// Fragment::id (Fragment.cpp:173-183)
static std::string frag_id(const npgx_blockset* B, const Frag& f, bool inverse) {
    const int ori = inverse ? -f.ori : f.ori;
    int64_t a = ori == 1 ? f.min : f.max;
    int64_t b = ori == 1 ? f.max : f.min;
    if (a == b && ori == -1) b = -1;
    return B->ss->names[(size_t)f.seq] + "_" + std::to_string(a) + "_" + std::to_string(b);
}

// block_hash (block_hash.cpp:29-55)
static uint64_t block_hash(const npgx_blockset* B, const Block& b) {
    std::vector<std::string> d, v;
    d.reserve(b.f.size());
    v.reserve(b.f.size());
    for (const Frag& f : b.f) {
        d.push_back(frag_id(B, f, false));
        v.push_back(frag_id(B, f, true));
    }
    std::sort(d.begin(), d.end());
    std::sort(v.begin(), v.end());
    const std::vector<std::string>& ids = d < v ? d : v;
    std::string j;
    for (size_t i = 0; i < ids.size(); i++) {
        if (i) j.push_back(' ');
        j += ids[i];
    }
    j.resize((j.size() + 15) / 16 * 16, ' ');
    uint64_t a = 1;
    for (size_t i = 0; i < j.size(); i += 16) {
        uint64_t x, y;
        memcpy(&x, j.data() + i, 8);
        memcpy(&y, j.data() + i + 8, 8);
        a = a * x;
        a ^= y;
    }
    return a;
}

static uint64_t blockset_hash(const npgx_blockset* B) {
    uint64_t h = 0;
    for (const Block& b : B->blocks)
        if (b.f.size() > 1) h ^= block_hash(B, b);
    return h;
}

// ---------------------------------------------------------------- RemoveNonStem
static void remove_non_stem(npgx_blockset* B) {
    std::vector<std::string> genome((size_t)B->ss->n);
    std::set<std::string> all;
    for (int32_t i = 0; i < B->ss->n; i++) {
        genome[(size_t)i] = genome_of(B->ss->names[(size_t)i]);
        NPGX_REQUIRE(!genome[(size_t)i].empty(), NPGX_ERR_ARG,
                     "Genome undefined: " + B->ss->names[(size_t)i]);
        all.insert(genome[(size_t)i]);
    }
    std::vector<Block> keep;
    for (Block& b : B->blocks) {
        std::set<std::string> g;
        bool ok = true;
        for (const Frag& f : b.f)
            if (!g.insert(genome[(size_t)f.seq]).second) {  // --exact
                ok = false;
                break;
            }
        if (ok && g.size() != all.size()) ok = false;  // g is a subset of all
        if (ok) keep.push_back(std::move(b));
    }
    B->blocks.swap(keep);
}

// ---------------------------------------------------------------- refine_alignment
// refine_alignment.cpp:15-190 (used by align_block after the dummy aligner)
struct Refiner {
    std::vector<std::string>& a;
    explicit Refiner(std::vector<std::string>& rows) : a(rows) {}
    void props(int i, int j, char c, bool& gap, bool& other, int& matches) const {
        gap = other = false;
        matches = 0;
        for (int k = 0; k < (int)a.size(); k++) {
            if (k == i) continue;
            const char x = a[(size_t)k][(size_t)j];
            if (x == '-') gap = true;
            else if (x == c) matches++;
            else other = true;
        }
    }
    bool try_move(int i, int from, int to) {
        std::string& r = a[(size_t)i];
        const char c = r[(size_t)from], t = r[(size_t)to];
        if ((c == '-') == (t == '-')) return false;
        bool fg, fo, tg, to_;
        int fm, tm;
        props(i, from, c, fg, fo, fm);
        props(i, to, c, tg, to_, tm);
        if (tm == 0 || !fo || (to_ && fm)) return false;
        std::swap(r[(size_t)from], r[(size_t)to]);
        return true;
    }
    bool equal_col(int j) const {
        for (size_t k = 1; k < a.size(); k++)
            if (a[k][(size_t)j] != a[0][(size_t)j]) return false;
        return true;
    }
    bool movable(int i, int first, int last) {
        const int l = (int)a[0].size();
        const std::string& r = a[(size_t)i];
        if (r[(size_t)first] == '-') {
            if (first > 0 && try_move(i, first - 1, last)) return true;
            if (last < l - 1 && try_move(i, last + 1, first)) return true;
            return false;
        }
        if (last < l - 1 && try_move(i, first, last + 1)) return true;
        if (first > 0 && try_move(i, last, first - 1)) return true;
        for (int j = first + 1; j <= last - 1; j++) {
            if (equal_col(j)) continue;
            if (last < l - 1 && try_move(i, j, last + 1)) return true;
            if (first > 0 && try_move(i, j, first - 1)) return true;
        }
        return false;
    }
    bool move_chars() {
        bool any = false;
        const int length = (int)a[0].size();
        for (int i = 0; i < (int)a.size(); i++) {
            std::string& r = a[(size_t)i];
            char rep = r[0];
            int first = 0, last = 0;
            for (int j = 1; j < length; j++) {
                if (r[(size_t)j] == rep) {
                    last = j;
                    continue;
                }
                any |= movable(i, first, last);
                rep = r[(size_t)j];
                first = last = j;
                while (first > 0 && r[(size_t)first - 1] == rep) first--;
            }
            any |= movable(i, first, last);
        }
        return any;
    }
    void drop_pure_gaps() {
        const size_t L = a[0].size();
        std::vector<std::string> n(a.size());
        for (size_t j = 0; j < L; j++) {
            bool pure = true;
            for (auto& r : a)
                if (r[j] != '-') {
                    pure = false;
                    break;
                }
            if (!pure)
                for (size_t k = 0; k < a.size(); k++) n[k].push_back(a[k][j]);
        }
        a.swap(n);
    }
    void run() {
        if (a.empty()) return;
        while (move_chars()) drop_pure_gaps();
        drop_pure_gaps();
    }
};

// ---------------------------------------------------------------- DummyAligner
// AbstractAligner::align_block with DummyAligner (AbstractAligner.cpp:51-69,145-177)
static void dummy_align(npgx_blockset* B) {
    for (Block& b : B->blocks) {
        if (b.f.empty()) continue;
        if (b.f.size() == 1) {
            if (b.has_rows() && (int64_t)b.rows[0].size() == b.f[0].len()) continue;
            b.rows.assign(1, seq_text(B->text(b.f[0].seq), b.f[0].begin(), b.f[0].len(), b.f[0].ori));
            continue;
        }
        if (b.has_rows()) {
            bool same = true;
            for (auto& r : b.rows) same &= r.size() == b.rows[0].size();
            if (same) continue;
        }
        std::vector<std::string> rows;
        size_t ml = 0;
        for (const Frag& f : b.f) {
            rows.push_back(seq_text(B->text(f.seq), f.begin(), f.len(), f.ori));
            ml = std::max(ml, rows.back().size());
        }
        for (auto& r : rows) r.resize(ml, '-');
        Refiner(rows).drop_pure_gaps();  // AbstractAligner remove_gaps
        Refiner(rows).run();
        b.rows.swap(rows);
    }
}

// ---------------------------------------------------------------- FragmentsExtender
// FragmentsExtender.cpp:34-119, all blocks in one GPU batch (2 jobs per block)
struct FlankJob {
    size_t block;
    bool left;
};

static int max_right_shift(const npgx_blockset* B, const Frag& f, int ori) {
    if (ori == 1) return (int)((int64_t)B->text(f.seq).size() - 1 - f.max);
    return (int)f.min;
}

static void fragments_extender(npgx_blockset* B, const std::vector<size_t>& which) {
    const int64_t portion = B->opt.extend_portion_x1e4;
    auto tg = Clock::now();
    std::vector<FlankJob> jobs;
    std::string rows;
    std::vector<int64_t> row_off(1, 0);
    std::vector<int32_t> job_start(1, 0);
    std::vector<std::vector<std::string>> central(which.size());
    for (size_t w = 0; w < which.size(); w++) {
        Block& b = B->blocks[which[w]];
        if (b.f.size() < 2 || !b.has_rows()) continue;
        central[w] = b.rows;
        const int64_t L = b.aln_len();
        const int64_t portion_length = portion * L / 10000;  // (Decimal(portion) * L).to_i()
        const int E = (int)std::max<int64_t>(B->opt.extend_length, portion_length);
        for (int side = 0; side < 2; side++) {
            // side 0: right; side 1: left == right of the inverted block (Block::inverse)
            int sh = E;
            for (const Frag& f : b.f) sh = std::min(sh, max_right_shift(B, f, side ? -f.ori : f.ori));
            if (sh <= 0) continue;
            for (Frag& f : b.f) {
                const int o = side ? -f.ori : f.ori;
                const int64_t begin = o == 1 ? f.min : f.max;
                rows += seq_text(B->text(f.seq), begin + o * f.len(), sh, o);
                row_off.push_back((int64_t)rows.size());
                if (o == 1) f.max += sh;  // shift_end
                else f.min -= sh;
            }
            jobs.push_back(FlankJob{w, side == 1});
            job_start.push_back((int32_t)(row_off.size() - 1));
        }
    }
    // align every flank of every block in one batch
    B->stats.ms_stage[3] += ms_since(tg);
    auto t0 = Clock::now();
    if (!jobs.empty()) {
        align_batch(B->aligner, rows.data(), row_off.data(), job_start.data(), (int32_t)jobs.size());
        collect_kernel_times(B);
        B->stats.aligned_residues += (int64_t)rows.size();
        B->stats.align_jobs += (int64_t)jobs.size();
    }
    B->stats.ms_align += ms_since(t0);
    B->stats.ms_stage[4] += ms_since(t0);
    auto ts = Clock::now();
    const int64_t* ooff = nullptr;
    const char* out = jobs.empty() ? nullptr : aligner_result(B->aligner, &ooff);
    // stitch: revcomp(left) + central + right (FragmentsExtender.cpp:108-118)
    std::vector<std::vector<std::string>> lr(which.size() * 2);
    for (size_t j = 0; j < jobs.size(); j++) {
        auto& dst = lr[jobs[j].block * 2 + (jobs[j].left ? 1 : 0)];
        for (int32_t r = job_start[j]; r < job_start[j + 1]; r++)
            dst.emplace_back(out + ooff[r], (size_t)(ooff[r + 1] - ooff[r]));
    }
    for (size_t w = 0; w < which.size(); w++) {
        Block& b = B->blocks[which[w]];
        if (central[w].empty()) continue;
        auto& R = lr[w * 2];
        auto& Lf = lr[w * 2 + 1];
        for (size_t i = 0; i < b.f.size(); i++) {
            std::string row;
            if (!Lf.empty()) {
                row = Lf[i];
                revcomp_inplace(row);
            }
            row += central[w][i];
            if (!R.empty()) row += R[i];
            b.rows[i].swap(row);
        }
    }
    B->stats.ms_stage[5] += ms_since(ts);
}

// ---------------------------------------------------------------- FixEnds
// GoodAlnFinder::find_start (FixEnds.cpp:36-115) over the identity flags of one
// direction; window sums come from a prefix sum (same integers as the
// reference's circular buffer).
static int64_t find_start(const std::vector<int>& pre, const std::vector<char>& good, bool rev,
                          int64_t L, int mf, int min_good, int sub_frame) {
    if (L < mf) return L;
    auto g = [&](int64_t c) { return (int)good[(size_t)(rev ? L - 1 - c : c)]; };
    auto W = [&](int64_t s) {  // sum of good over [s, s+mf)
        if (!rev) return pre[(size_t)(s + mf)] - pre[(size_t)s];
        return pre[(size_t)(L - s)] - pre[(size_t)(L - s - mf)];
    };
    int64_t s = 0;
    auto first_good = [&](int64_t& st) {
        while (true) {
            if (W(st) >= min_good && g(st)) return true;
            st += 1;
            if (st + mf - 1 >= L) return false;
        }
    };
    if (!first_good(s)) return L;
    int best = W(s);
    int64_t best_s = s;
    while (true) {
        s += 1;
        if (s + mf - 1 >= L) break;
        const bool ok = first_good(s);
        if (!ok || s - best_s > sub_frame) break;
        if (W(s) > best) {
            best = W(s);
            best_s = s;
        }
    }
    return best_s;
}

// Block::slice (Block.cpp:238-284): letters of columns [start, stop]
static bool slice_block(const npgx_blockset* B, const Block& b, int64_t start, int64_t stop, Block& out) {
    out.f.clear();
    out.rows.clear();
    out.name.clear();
    for (size_t i = 0; i < b.f.size(); i++) {
        const Frag& f = b.f[i];
        const std::string& r = b.rows[i];
        int64_t before = 0, cnt = 0;
        for (int64_t c = 0; c < start; c++) before += r[(size_t)c] != '-';
        for (int64_t c = start; c <= stop; c++) cnt += r[(size_t)c] != '-';
        if (!cnt) continue;
        const int64_t s0 = f.begin() + f.ori * before;
        const int64_t s1 = f.begin() + f.ori * (before + cnt - 1);
        Frag nf{f.seq, s0 <= s1 ? 1 : -1, std::min(s0, s1), std::max(s0, s1)};
        std::string nr = r.substr((size_t)start, (size_t)(stop - start + 1));
        if (nf.ori != f.ori)  // set_begin_last turns a 1-letter ori -1 fragment into ori +1
            for (char& c : nr)
                if (c != '-') c = B->text(f.seq)[(size_t)nf.min];
        out.f.push_back(nf);
        out.rows.push_back(std::move(nr));
    }
    return true;
}

static void fix_ends(npgx_blockset* B, std::vector<Block>& blocks) {
    const int mf = B->opt.min_fragment;
    const int64_t mi = B->opt.min_identity_x1e4;
    const int min_good = (int)(mi * mf / 10000);           // (min_identity * min_fragment).to_i()
    const int sub_frame = (int)((10000 - mi) * mf / 10000);  // ((1 - min_identity) * ...).to_i()
    std::vector<Block> out;
    out.reserve(blocks.size());
    std::vector<char> good;
    std::vector<int> pre;
    for (Block& b : blocks) {
        if (!b.has_rows()) {
            out.push_back(std::move(b));
            continue;
        }
        const int64_t L = b.aln_len();
        good.assign((size_t)L, 0);
        for (int64_t c = 0; c < L; c++) {  // is_ident_nogap (block_stat.cpp:156-169)
            const char x = b.rows[0][(size_t)c];
            bool ok = x != '-';
            for (size_t i = 1; ok && i < b.rows.size(); i++) ok = b.rows[i][(size_t)c] == x;
            good[(size_t)c] = ok;
        }
        pre.assign((size_t)L + 1, 0);
        for (int64_t c = 0; c < L; c++) pre[(size_t)c + 1] = pre[(size_t)c] + good[(size_t)c];
        const int64_t sd = find_start(pre, good, false, L, mf, min_good, sub_frame);
        const int64_t sr = find_start(pre, good, true, L, mf, min_good, sub_frame);
        if (sd == 0 && sr == 0) {
            out.push_back(std::move(b));
            continue;
        }
        const int64_t stop = L - sr - 1;
        if (stop - sd + 1 >= mf) {
            Block s;
            slice_block(B, b, sd, stop, s);
            out.push_back(std::move(s));
        }
    }
    blocks.swap(out);
}

// ---------------------------------------------------------------- OverlaplessUnion
static bool frag_less(const Frag& a, const Frag& b) {  // Fragment::operator< (Fragment.cpp:214-222)
    return std::tie(a.min, a.max, a.ori, a.seq) < std::tie(b.min, b.max, b.ori, b.seq);
}
struct OuKey {
    int64_t size, len;
    const std::string* name;
    Frag minf;
    std::vector<std::tuple<int64_t, int64_t, int32_t, int32_t>> all;
};
static OuKey ou_key(const Block& b) {
    OuKey k;
    k.size = (int64_t)b.f.size();
    k.len = b.aln_len();
    k.name = &b.name;
    k.minf = b.f.empty() ? Frag{0, 0, 0, 0} : b.f[0];
    for (const Frag& f : b.f) {
        if (frag_less(f, k.minf)) k.minf = f;
        k.all.emplace_back(f.min, f.max, f.ori, f.seq);
    }
    std::sort(k.all.begin(), k.all.end());
    return k;
}
static bool ou_before(const OuKey& a, const OuKey& b) {
    if (a.size != b.size) return a.size > b.size;
    if (a.len != b.len) return a.len > b.len;
    if (*a.name != *b.name) return *a.name > *b.name;
    if (frag_less(a.minf, b.minf)) return true;
    if (frag_less(b.minf, a.minf)) return false;
    return a.all < b.all;
}

// SetFc (FragmentCollection.hpp:273-307): per sequence, fragments ordered by
// Fragment::operator<; a fragment overlaps if its lower_bound or predecessor does
struct FragCmp {
    bool operator()(const Frag& a, const Frag& b) const { return frag_less(a, b); }
};
struct Overlaps {
    std::vector<std::multiset<Frag, FragCmp>> by_seq;
    explicit Overlaps(int n) : by_seq((size_t)n) {}
    static bool common(const Frag& a, const Frag& b) {
        return std::max(a.min, b.min) <= std::min(a.max, b.max);
    }
    bool has(const Frag& f) const {
        const auto& s = by_seq[(size_t)f.seq];
        if (s.empty()) return false;
        auto it = s.lower_bound(f);
        if (it != s.end() && common(*it, f)) return true;
        if (it != s.begin() && common(*std::prev(it), f)) return true;
        return false;
    }
    bool block(const Block& b) const {
        for (const Frag& f : b.f)
            if (has(f)) return true;
        return false;
    }
    void add(const Block& b) {
        for (const Frag& f : b.f) by_seq[(size_t)f.seq].insert(f);
    }
};

static void overlapless_union(npgx_blockset* B, std::vector<Block>& blocks) {
    std::vector<OuKey> keys;
    keys.reserve(blocks.size());
    for (const Block& b : blocks) keys.push_back(ou_key(b));
    std::vector<size_t> order(blocks.size());
    for (size_t i = 0; i < order.size(); i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(),
                     [&](size_t a, size_t b) { return ou_before(keys[a], keys[b]); });
    Overlaps idx(B->ss->n);
    std::vector<Block> ol;
    for (size_t i : order) {
        if (idx.block(blocks[i])) continue;
        idx.add(blocks[i]);
        ol.push_back(std::move(blocks[i]));
    }
    blocks.swap(ol);
}

// ---------------------------------------------------------------- ExtendLoopFast
static void extend_loop_fast(npgx_blockset* B) {
    std::set<uint64_t> states;
    states.insert(blockset_hash(B));
    std::vector<uint64_t> seen;  // MoveUnchanged::hashes_ (sorted)
    for (int it = 0; it < B->opt.max_iterations || B->opt.max_iterations == -1; it++) {
        B->stats.iterations++;
        auto t0 = Clock::now();
        // MoveUnchanged target=unchanged other=target
        std::vector<Block> unchanged, work;
        std::vector<uint64_t> fresh;
        for (Block& b : B->blocks) {
            const uint64_t h = block_hash(B, b);
            if (std::binary_search(seen.begin(), seen.end(), h)) {
                unchanged.push_back(std::move(b));
            } else {
                fresh.push_back(h);
                work.push_back(std::move(b));
            }
        }
        seen.insert(seen.end(), fresh.begin(), fresh.end());
        std::sort(seen.begin(), seen.end());
        seen.erase(std::unique(seen.begin(), seen.end()), seen.end());
        B->stats.ms_host += ms_since(t0);
        B->stats.ms_stage[2] += ms_since(t0);
        // ExtendAndFix: FragmentsExtender --extend-length-portion:=0.5, then FixEnds
        B->blocks.swap(work);
        std::vector<size_t> all(B->blocks.size());
        for (size_t i = 0; i < all.size(); i++) all[i] = i;
        fragments_extender(B, all);
        t0 = Clock::now();
        fix_ends(B, B->blocks);
        B->stats.ms_stage[6] += ms_since(t0);
        // Move target=target other=unchanged; OverlaplessUnion --ou-move; Clear; Move
        auto t1 = Clock::now();
        for (Block& b : unchanged) B->blocks.push_back(std::move(b));
        overlapless_union(B, B->blocks);
        B->stats.ms_stage[7] += ms_since(t1);
        auto t2 = Clock::now();
        const uint64_t h = blockset_hash(B);
        B->stats.ms_stage[8] += ms_since(t2);
        B->stats.ms_host += ms_since(t0);
        if (states.count(h)) break;
        states.insert(h);
    }
}

// ---------------------------------------------------------------- Filter
static const int MAX_SCORE = 100;
// goodColumns.cpp:50-149 (the reference's table, generated by its documented
// formula floor(100 * (1 - log2(g+1)/g)), g = 0 -> -100)
static const int LOG_SCORE[1000] = {
#include "log_score.inc"
};
static int log_score(int64_t g) { return LOG_SCORE[g]; }

static std::vector<int> good_columns(const std::vector<std::string>& rows, int64_t L, int mi, int ml) {
    std::vector<int> sc((size_t)L, 0);
    int64_t run = 0;
    auto flush = [&](int64_t end) {  // mapGap
        int64_t start = end - run, length = run;
        if (length >= 1000) length = 999;
        int s = log_score(length);
        s = s == MAX_SCORE ? s : s * mi / MAX_SCORE;
        if (length >= ml) s = -100 * MAX_SCORE;
        for (int64_t i = start; i < end; i++) sc[(size_t)i] = s;
        run = 0;
    };
    for (int64_t c = 0; c < L; c++) {
        const char x = rows[0][(size_t)c];
        bool same = true, gap = false;
        int letters = 0;
        bool A = false, T = false, G = false, C = false, N = false;
        for (const auto& r : rows) {
            const char y = r[(size_t)c];
            same &= y == x;
            gap |= y == '-';
            A |= y == 'A';
            T |= y == 'T';
            G |= y == 'G';
            C |= y == 'C';
            N |= y == 'N';
        }
        letters = A + T + G + C;
        if (same && x != '-' && x != 'N') sc[(size_t)c] = MAX_SCORE;  // isColumnGood
        if (gap && letters == 1 && !N) run++;                        // isColumnIdentGap
        else if (run > 0) flush(c);
    }
    if (run > 0) flush(L);
    return sc;
}

typedef std::pair<int64_t, int64_t> Span;

// goodSlices.cpp:17-245
struct Slicer {
    const std::vector<int>& sc;
    std::vector<int64_t> sum, gapless;
    int64_t frame, end, frame_score, end_score, L, min_len;
    int mi;
    Slicer(const std::vector<int>& s, int64_t fl, int64_t el, int mi_, int64_t ml) : sc(s) {
        L = (int64_t)s.size();
        frame = std::min(fl, L);
        end = el;
        frame_score = frame * mi_;
        end_score = el * mi_;
        min_len = ml;
        mi = mi_;
        sum.assign((size_t)L + 1, 0);
        gapless.assign((size_t)L + 1, 0);
        for (int64_t i = 0; i < L; i++) {
            sum[(size_t)i + 1] = sum[(size_t)i] + s[(size_t)i];
            gapless[(size_t)i + 1] =
                gapless[(size_t)i] + (s[(size_t)i] == MAX_SCORE ? MAX_SCORE : std::min(s[(size_t)i], 0));
        }
    }
    int64_t score(int64_t a, int64_t b) const { return sum[(size_t)b + 1] - sum[(size_t)a]; }
    int64_t gscore(int64_t a, int64_t b) const { return gapless[(size_t)b + 1] - gapless[(size_t)a]; }
    bool left_ok(int64_t a) const { return sc[(size_t)a] == MAX_SCORE && gscore(a, a + end - 1) >= end_score; }
    bool right_ok(int64_t b) const { return sc[(size_t)b] == MAX_SCORE && gscore(b - end + 1, b) >= end_score; }
    static int64_t len(const Span& s) { return s.second - s.first + 1; }
    bool valid(const Span& s) const { return len(s) >= min_len && s.first >= 0 && s.second < L; }
    Span strip(Span s) const {
        if (!valid(s)) return s;
        while (!left_ok(s.first) && s.first + end - 1 < s.second) s.first++;
        while (!right_ok(s.second) && s.first + end - 1 < s.second) s.second--;
        return s;
    }
    bool ends_ok(const Span& s) const {
        if (!left_ok(s.first) || !right_ok(s.second)) return false;
        if (len(s) >= frame) return true;
        return score(s.first, s.second) >= (int64_t)mi * len(s);
    }
    std::vector<Span> run() const {
        if (min_len > L || min_len <= 0 || frame > L || frame <= 0 || end > min_len || end < 0) return {};
        std::vector<Span> joined;
        bool prev = false;
        for (int64_t i = 0; i + frame <= L; i++) {
            const bool cur = score(i, i + frame - 1) >= frame_score;
            if (cur && prev) joined.back().second++;
            else if (cur) joined.push_back(Span(i, i + frame - 1));
            prev = cur;
        }
        std::vector<Span> cand, res;
        for (const Span& s : joined) {
            Span t = strip(s);
            if (valid(t)) cand.push_back(t);
        }
        while (!cand.empty()) {
            Span best = cand[0];
            for (const Span& s : cand)
                if (len(s) > len(best)) best = s;
            if (!(valid(best) && ends_ok(best))) break;
            res.push_back(best);
            std::vector<Span> next;
            for (const Span& s : cand) {
                const bool ov = (best.first <= s.first && s.first <= best.second) ||
                                (s.first <= best.first && best.first <= s.second);
                if (!ov) {
                    next.push_back(s);
                    continue;
                }
                Span t = s;
                if (best.first <= s.first && s.first <= best.second) t.first = best.second + 1;
                if (best.first <= s.second && s.second <= best.second) t.second = best.first - 1;
                t = strip(t);
                if (valid(t) && ends_ok(t)) next.push_back(t);
            }
            cand.swap(next);
        }
        return res;
    }
};

static int min_ident_count(int64_t mi) {  // Filter.cpp:112-120
    int64_t v = mi * 100;                 // (min_identity * 100) x 1e4
    return (int)(v / 10000 + (v % 10000 ? 1 : 0));
}

static std::vector<Span> good_subblocks(const npgx_blockset* B, const Block& b) {
    const int mi = min_ident_count(B->opt.min_identity_x1e4);
    std::vector<int> sc = good_columns(b.rows, b.aln_len(), mi, B->opt.min_fragment);
    return Slicer(sc, B->opt.frame_length, B->opt.min_end, mi, B->opt.min_fragment).run();
}

static bool frag_valid(const npgx_blockset* B, const Frag& f) {
    return f.min <= f.max && f.max < (int64_t)B->text(f.seq).size();
}

static bool filter_good(const npgx_blockset* B, const Block& b) {  // Filter.cpp:143-174
    const int64_t L = b.aln_len();
    if (L < B->opt.min_fragment) return false;
    for (const Frag& f : b.f)
        if (!frag_valid(B, f)) return false;
    if ((int64_t)b.f.size() < B->opt.min_block) return false;
    if (B->opt.max_block != -1 && (int64_t)b.f.size() > B->opt.max_block) return false;
    if (b.has_rows() && B->opt.min_identity_x1e4 > 500) {
        std::vector<Span> s = good_subblocks(B, b);
        if (!(s.size() == 1 && s[0] == Span(0, L - 1))) return false;
    }
    return true;
}

static void filter_subblocks(const npgx_blockset* B, const Block& b, std::vector<Block>& out) {
    if ((int64_t)b.f.size() < B->opt.min_block || !b.has_rows() || b.aln_len() < B->opt.min_fragment)
        return;
    for (const Span& s : good_subblocks(B, b)) {
        Block x;
        slice_block(B, b, s.first, s.second, x);
        out.push_back(std::move(x));
    }
}

static void filter(npgx_blockset* B) {  // Filter::process_block_impl (Filter.cpp:208-248)
    std::vector<Block> out;
    for (Block& b : B->blocks) {
        if (filter_good(B, b)) {
            out.push_back(std::move(b));
            continue;
        }
        std::vector<Block> sub;
        if (B->opt.find_subblocks) filter_subblocks(B, b, sub);
        if (!sub.empty()) {
            for (auto& x : sub) out.push_back(std::move(x));
            continue;
        }
        Block k = b;
        k.f.clear();
        k.rows.clear();
        for (size_t i = 0; i < b.f.size(); i++)
            if (frag_valid(B, b.f[i])) {
                k.f.push_back(b.f[i]);
                if (b.has_rows()) k.rows.push_back(b.rows[i]);
            }
        if (k.f.size() != b.f.size()) {
            if (filter_good(B, k)) {
                out.push_back(std::move(k));
                continue;
            }
            if (B->opt.find_subblocks) filter_subblocks(B, k, out);
        }
    }
    B->blocks.swap(out);
}

static void add_anchors(npgx_blockset* B, const npgx_af* af) {
    int64_t nb = 0, nf = 0;
    if (npgx_af_result_counts(af, &nb, &nf) != NPGX_OK) throw Error(NPGX_ERR_STATE, npgx_last_error());
    std::vector<int64_t> bs((size_t)nb + 1), mn((size_t)nf), mx((size_t)nf);
    std::vector<int32_t> seq((size_t)nf);
    std::vector<int8_t> ori((size_t)nf);
    if (npgx_af_result_copy(af, bs.data(), seq.data(), mn.data(), mx.data(), ori.data()) != NPGX_OK)
        throw Error(NPGX_ERR_STATE, npgx_last_error());
    for (int64_t b = 0; b < nb; b++) {
        Block blk;
        for (int64_t i = bs[(size_t)b]; i < bs[(size_t)b + 1]; i++)
            blk.f.push_back(Frag{seq[(size_t)i], ori[(size_t)i], mn[(size_t)i], mx[(size_t)i]});
        B->blocks.push_back(std::move(blk));
    }
}

static void apply(npgx_blockset* B, const std::string& p, npgx_af* af) {
    B->ktimes.clear();
    B->job_stats.clear();
    if (p == "RemoveNonStem") return remove_non_stem(B);
    if (p == "DummyAligner") return dummy_align(B);
    if (p == "FragmentsExtender") {
        std::vector<size_t> all(B->blocks.size());
        for (size_t i = 0; i < all.size(); i++) all[i] = i;
        return fragments_extender(B, all);
    }
    if (p == "FixEnds") return fix_ends(B, B->blocks);
    if (p == "ExtendLoopFast") return extend_loop_fast(B);
    if (p == "Filter") return filter(B);
    if (p == "OverlaplessUnion") return overlapless_union(B, B->blocks);
    if (p == "DraftPangenome") {
        NPGX_REQUIRE(af, NPGX_ERR_ARG, "DraftPangenome needs an AnchorFinder handle");
        B->stats = npgx_bb_stats{};
        auto ta = Clock::now();
        if (npgx_af_run(af, B->ss) != NPGX_OK) throw Error(NPGX_ERR_HIP, npgx_last_error());
        B->blocks.clear();
        add_anchors(B, af);
        B->stats.ms_stage[0] = ms_since(ta);
        B->stats.anchor_blocks = (int64_t)B->blocks.size();
        auto tb = Clock::now();
        remove_non_stem(B);
        B->stats.stem_blocks = (int64_t)B->blocks.size();
        dummy_align(B);
        B->stats.ms_stage[1] = ms_since(tb);
        extend_loop_fast(B);
        auto t0 = Clock::now();
        filter(B);
        B->stats.ms_stage[9] = ms_since(t0);
        B->stats.ms_host += ms_since(t0);
        return;
    }
    throw Error(NPGX_ERR_ARG, "unknown processor: " + p);
}

}  // namespace bb
}  // namespace npgx

extern "C" {

void npgx_bb_default_options(npgx_bb_options* o) {
    if (!o) return;
    memset(o, 0, sizeof(*o));
    o->extend_length = 100;          // MIN_LENGTH
    o->max_iterations = 10;          // DraftPangenome: extender:set_max_iterations(10)
    o->extend_portion_x1e4 = 5000;   // ExtendAndFix --extend-length-portion:=0.5
    o->min_fragment = 100;           // MIN_LENGTH
    o->frame_length = 100;           // FRAME_LENGTH
    o->min_end = 10;                 // MIN_END
    o->min_block = 2;
    o->max_block = -1;
    o->find_subblocks = 1;
    o->min_identity_x1e4 = 9000;     // MIN_IDENTITY
    npgx_align_default_options(&o->align);
}

int npgx_blockset_create(const npgx_seqset* s, const npgx_bb_options* o, npgx_blockset** out) {
    return guard([&] {
        NPGX_REQUIRE(s && o && out, NPGX_ERR_ARG, "null argument");
        auto* B = new npgx_blockset;
        B->ss = s;
        B->opt = *o;
        npgx_align_options ao = o->align;
        ao.aligner_type = 0;
        int rc = npgx_aligner_create(&ao, &B->aligner);
        if (rc != NPGX_OK) {
            delete B;
            throw Error(rc, npgx_last_error());
        }
        *out = B;
    });
}

int npgx_blockset_set_blocks(npgx_blockset* B, int64_t nb, const int64_t* bs, const int32_t* seq,
                             const int64_t* mn, const int64_t* mx, const int8_t* ori,
                             const int64_t* row_off, const char* rows) {
    return guard([&] {
        NPGX_REQUIRE(B && (nb == 0 || (bs && seq && mn && mx && ori)), NPGX_ERR_ARG, "null argument");
        B->blocks.clear();
        for (int64_t b = 0; b < nb; b++) {
            Block blk;
            for (int64_t i = bs[b]; i < bs[b + 1]; i++) {
                NPGX_REQUIRE(seq[i] >= 0 && seq[i] < B->ss->n, NPGX_ERR_ARG, "bad sequence index");
                NPGX_REQUIRE(ori[i] == 1 || ori[i] == -1, NPGX_ERR_ARG, "ori must be +-1");
                blk.f.push_back(Frag{seq[i], ori[i], mn[i], mx[i]});
                if (row_off) blk.rows.emplace_back(rows + row_off[i], (size_t)(row_off[i + 1] - row_off[i]));
            }
            B->blocks.push_back(std::move(blk));
        }
    });
}

int npgx_blockset_add_anchors(npgx_blockset* B, const npgx_af* af) {
    return guard([&] {
        NPGX_REQUIRE(B && af, NPGX_ERR_ARG, "null argument");
        add_anchors(B, af);
    });
}

int npgx_blockset_apply(npgx_blockset* B, const char* processor, npgx_af* af) {
    return guard([&] {
        NPGX_REQUIRE(B && processor, NPGX_ERR_ARG, "null argument");
        apply(B, processor, af);
    });
}

int npgx_blockset_counts(const npgx_blockset* B, int64_t* nb, int64_t* nf, int64_t* rb) {
    return guard([&] {
        NPGX_REQUIRE(B && nb && nf && rb, NPGX_ERR_ARG, "null argument");
        int64_t f = 0, r = 0;
        for (const Block& b : B->blocks) {
            f += (int64_t)b.f.size();
            for (const auto& x : b.rows) r += (int64_t)x.size();
        }
        *nb = (int64_t)B->blocks.size();
        *nf = f;
        *rb = r;
    });
}

int npgx_blockset_copy(const npgx_blockset* B, int64_t* bs, int32_t* seq, int64_t* mn, int64_t* mx,
                       int8_t* ori, int64_t* row_off, char* rows) {
    return guard([&] {
        NPGX_REQUIRE(B, NPGX_ERR_ARG, "null argument");
        int64_t k = 0, ro = 0;
        size_t b = 0;
        for (; b < B->blocks.size(); b++) {
            const Block& blk = B->blocks[b];
            if (bs) bs[b] = k;
            for (size_t i = 0; i < blk.f.size(); i++, k++) {
                if (seq) seq[k] = blk.f[i].seq;
                if (mn) mn[k] = blk.f[i].min;
                if (mx) mx[k] = blk.f[i].max;
                if (ori) ori[k] = (int8_t)blk.f[i].ori;
                if (row_off) row_off[k] = ro;
                if (blk.has_rows()) {
                    if (rows) memcpy(rows + ro, blk.rows[i].data(), blk.rows[i].size());
                    ro += (int64_t)blk.rows[i].size();
                }
            }
        }
        if (bs) bs[b] = k;
        if (row_off) row_off[k] = ro;
    });
}

int npgx_blockset_hash(const npgx_blockset* B, uint64_t* h) {
    return guard([&] {
        NPGX_REQUIRE(B && h, NPGX_ERR_ARG, "null argument");
        *h = blockset_hash(B);
    });
}

int npgx_blockset_stats(const npgx_blockset* B, npgx_bb_stats* out) {
    return guard([&] {
        NPGX_REQUIRE(B && out, NPGX_ERR_ARG, "null argument");
        *out = B->stats;
    });
}

int npgx_blockset_kernel_times(const npgx_blockset* B, npgx_kernel_time* out, int32_t cap, int32_t* n) {
    return guard([&] {
        NPGX_REQUIRE(B && n && (out || cap == 0), NPGX_ERR_ARG, "null argument");
        int32_t k = 0;
        for (const auto& t : B->ktimes) {
            if (k >= cap) break;
            out[k++] = t;
        }
        *n = (int32_t)B->ktimes.size();
    });
}

int npgx_blockset_job_stats(const npgx_blockset* B, int64_t* out, int64_t cap, int64_t* n) {
    return guard([&] {
        NPGX_REQUIRE(B && n, NPGX_ERR_ARG, "null argument");
        *n = (int64_t)B->job_stats.size() / 8;
        if (out) memcpy(out, B->job_stats.data(), (size_t)std::min<int64_t>(cap, *n) * 64);
    });
}

void npgx_blockset_free(npgx_blockset* B) {
    if (!B) return;
    if (B->aligner) npgx_aligner_free(B->aligner);
    delete B;
}

}  // extern "C"
