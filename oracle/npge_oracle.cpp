// npge_oracle.cpp -- CPU restatement of NPG-explorer's anchor-finding and greedy
// multiple-alignment hot path.  TEST INFRASTRUCTURE ONLY: this file is the
// parity checker for the HIP product in npge_amd/.  Only tests/, the smoke()
// entry and bench.py's cpu_baseline leg may load it.  The product never links it.
//
// Every function cites the reference file:line it restates (paths relative to
// the NPG-explorer 0.5.8 tree).  It is a sequential, 1-worker restatement that
// follows the reference control flow literally (it is NOT the data-parallel
// reformulation the GPU uses), so agreement between the two is a real check.
//
// Determinism conventions (the reference itself is time-seeded / pointer-ordered,
// SURVEY.md §0.2-0.3):
//   * Bloom hash parameters come from an explicit glibc-rand() seed or an explicit
//     parameter vector instead of srand(make_seed()) (BloomFilter.cpp:55-63).
//   * Sequences are ranked by (size desc, name asc, input index asc) where the
//     reference uses an unstable std::sort by size (SeqI.hpp:54).
//   * FoundFragment order uses that rank where the reference compares Sequence*
//     (AnchorFinder.cpp:234-238).
//   * SimilarAligner reads one past the end of a row (std::string's '\0') and,
//     in find_best_gap, possibly further (UB).  Here: s[size] == '\0' as in C++11,
//     and s[p > size] is a per-row sentinel that equals nothing (counted in
//     g_past_end_reads so tests can see whether an input exercised it).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>

typedef uint64_t hash_t;
typedef std::vector<std::string> Strings;

namespace orc {

// ---------------------------------------------------------------- letters
// char_to_size.hpp:24-36 (A=0 T=1 G=2 C=3 N=4), complement_letter :54-57
static inline size_t char_to_size(char c) {
    if (c == 'A') return 0;
    if (c == 'T') return 1;
    if (c == 'G') return 2;
    if (c == 'C') return 3;
    return 4;
}
// complement.hpp:19-32 -- complement of a single char, non-ATGC unchanged
static inline char complement_char(char c) {
    char C = (char)toupper((unsigned char)c);
    if (C == 'A') return 'T';
    if (C == 'T') return 'A';
    if (C == 'G') return 'C';
    if (C == 'C') return 'G';
    return c;
}
// complement.cpp:16-21 -- reverse complement of a string
static void complement_str(std::string& s) {
    for (char& c : s) c = complement_char(c);
    std::reverse(s.begin(), s.end());
}

// Sequence.cpp:151-179 -- uppercase, keep ATGCN, IUPAC -> N, drop the rest
static std::string to_atgcn(const std::string& in) {
    std::string out;
    out.reserve(in.size());
    for (char c0 : in) {
        char c = (char)toupper((unsigned char)c0);
        if (c == 'A' || c == 'T' || c == 'G' || c == 'C' || c == 'N') {
            out += c;
        } else if (c == 'R' || c == 'Y' || c == 'M' || c == 'K' || c == 'W' ||
                   c == 'S' || c == 'B' || c == 'V' || c == 'H' || c == 'D') {
            out += 'N';
        }
    }
    return out;
}

// ---------------------------------------------------------------- hashing
const int MAX_ANCHOR_SIZE = 32;  // make_hash.hpp:19
static inline size_t shift_in_hash(int pos) { return (pos * 2) % 64; }  // :25-27

// make_hash.hpp:29-42 (+ FChar :44-60): ori=-1 walks backwards and complements
// every letter except N.
static hash_t make_hash(const char* start, int length, int ori) {
    hash_t result = 0;
    for (int j = 0; j < length; j++) {
        char c = (ori == 1) ? start[j] : start[-j];
        size_t s = char_to_size(c) & 3;
        if (ori == -1 && c != 'N') s ^= 1;
        result ^= hash_t(s) << shift_in_hash(j);
    }
    return result;
}

// make_hash.hpp:88-108
static hash_t reuse_hash(hash_t old_hash, int length, char remove_char,
                         char add_char, bool forward) {
    hash_t remove = char_to_size(remove_char) & 3;
    old_hash ^= remove << shift_in_hash(forward ? 0 : length - 1);
    int occupied = std::min(2 * length, 64);
    if (forward) {
        old_hash = (old_hash >> 2) | ((old_hash & 3) << (occupied - 2));
    } else {
        old_hash = (old_hash << 2) | ((old_hash >> (occupied - 2)) & 3);
    }
    hash_t add = char_to_size(add_char) & 3;
    old_hash ^= add << shift_in_hash(forward ? length - 1 : 0);
    return old_hash;
}

// complement.cpp:24-50
static hash_t complement_hash(hash_t hash, int letters_number) {
    hash_t result = 0;
    int digits = std::min(letters_number, MAX_ANCHOR_SIZE);
    size_t r = (letters_number / MAX_ANCHOR_SIZE) % 2;
    size_t xor_swap_pos = letters_number % MAX_ANCHOR_SIZE;
    size_t smal_xor = r ^ 1;
    size_t great_xor = r;
    for (int i = 0; i < digits; i++) {
        int dest = (letters_number - 1 - i) % MAX_ANCHOR_SIZE;
        hash_t last_2_bits = hash & 0x03;
        if ((size_t)i < xor_swap_pos) last_2_bits ^= smal_xor;
        else last_2_bits ^= great_xor;
        result ^= last_2_bits << (2 * dest);
        hash = hash >> 2;
    }
    return result;
}

// ---------------------------------------------------------------- glibc rand
// glibc random_r.c TYPE_3 (degree 31, separation 3), the generator behind
// std::srand/std::rand used by BloomFilter::set_hashes (BloomFilter.cpp:55-63).
// Not part of /root/reference; restated from glibc's published algorithm.
struct GlibcRand {
    std::vector<int32_t> r;
    size_t i;
    explicit GlibcRand(uint32_t seed) {
        r.resize(34);
        int32_t s = (int32_t)seed;
        if (s == 0) s = 1;
        r[0] = s;
        for (int k = 1; k < 31; k++) {
            int32_t hi = r[k - 1] / 127773;
            int32_t lo = r[k - 1] % 127773;
            int32_t word = 16807 * lo - 2836 * hi;
            if (word < 0) word += 2147483647;
            r[k] = word;
        }
        for (int k = 31; k < 34; k++) r[k] = r[k - 31];
        i = 34;
        for (int k = 0; k < 310; k++) next_raw();
    }
    uint32_t next_raw() {
        int32_t v = (int32_t)((uint32_t)r[i - 31] + (uint32_t)r[i - 3]);
        r.push_back(v);
        i++;
        return (uint32_t)v;
    }
    int32_t next() { return (int32_t)(next_raw() >> 1); }
};

// ---------------------------------------------------------------- Bloom filter
static const double LN_TWO = 0.69314718055994530942;  // boost ln_two<double>

// BloomFilter.cpp:147-156 (int result; overflow beyond INT_MAX is rejected)
static int64_t optimal_bits(uint64_t members, double error_prob) {
    double v = double(members) * (-std::log(error_prob) / (LN_TWO * LN_TWO)) + 0.5;
    if (v >= 2147483647.0) return -1;
    int result = (int)v;
    if (result % 2 == 0) result += 1;
    if (result < 1) result = 1;
    return result;
}
// BloomFilter.cpp:158-164 (members == 0 gives +inf -> INT_MIN on x86 -> 1)
static int optimal_hashes(uint64_t members, uint64_t bits) {
    if (members == 0) return 1;
    int result = (int)std::round(LN_TWO * double(bits) / double(members));
    if (result < 1) result = 1;
    return result;
}

struct Bloom {
    std::vector<bool> bits;
    std::vector<hash_t> params;
    // BloomFilter.cpp:166-170
    size_t make_index(size_t i, hash_t h) const {
        return (h ^ params[i]) % hash_t(bits.size());
    }
    // BloomFilter.cpp:65-76
    bool test_and_add(hash_t h) {
        bool result = true;
        for (size_t i = 0; i < params.size(); i++) {
            size_t idx = make_index(i, h);
            if (!bits[idx]) result = false;
            bits[idx] = true;
        }
        return result;
    }
};

// ---------------------------------------------------------------- AnchorFinder
struct Seq {
    std::string name;
    std::string data;  // after to_atgcn
    int index;         // input order
};

// Sequence.cpp:193-202
static std::string genome_of(const std::string& name) {
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

// AnchorFinder.cpp:81-97
static uint64_t estimate_length(const std::vector<Seq>& seqs) {
    std::map<std::string, uint64_t> gtl;
    uint64_t max_length = 0;
    for (const Seq& s : seqs) {
        uint64_t& g = gtl[genome_of(s.name)];
        g += s.data.size();
        max_length = std::max(max_length, g);
    }
    if (gtl.size() == 1) return max_length;
    return max_length / 2 * 3;
}

struct FoundFragment {  // AnchorFinder.cpp:222-247 (Sequence* -> rank)
    hash_t hash;
    int rank;
    uint64_t pos;  // if ori = -1, pos = size + min_pos
    bool operator<(const FoundFragment& o) const {
        if (hash != o.hash) return hash < o.hash;
        if (rank != o.rank) return rank < o.rank;
        return pos < o.pos;
    }
};

struct AnchorResult {
    // fragments in output order; block boundaries in block_start
    std::vector<int> frag_seq;  // input index of the sequence
    std::vector<int64_t> frag_min, frag_max;
    std::vector<int> frag_ori;
    std::vector<int64_t> block_start;  // size n_blocks+1
    std::vector<hash_t> block_hash;
    // stats
    int64_t members = 0, bits = 0;
    int hashes = 0;
    std::vector<hash_t> params;
    int64_t n_collected = 0;   // |H| after sort+unique
    int64_t n_found_frags = 0; // before truncation
};

struct AnchorFinder {
    int anchor = 20;
    int64_t fp_x1e4 = 1000;     // Decimal("0.1")
    bool similar = true;
    int64_t max_anchor_fragments = 100000;
    uint32_t seed = 1;
    std::vector<hash_t> explicit_params;  // overrides seed when non-empty
    std::vector<hash_t> used_hashes;      // AnchorFinder.cpp:30-35 (persistent)

    // AnchorFinder.cpp:393-406
    int run(std::vector<Seq>& all, AnchorResult& out) {
        // SeqBase::make_seqs SeqI.hpp:45-57 (ties pinned by name, then index)
        std::vector<const Seq*> seqs;
        for (const Seq& s : all)
            if ((int64_t)s.data.size() >= anchor) seqs.push_back(&s);
        std::sort(seqs.begin(), seqs.end(), [](const Seq* a, const Seq* b) {
            if (a->data.size() != b->data.size()) return a->data.size() > b->data.size();
            if (a->name != b->name) return a->name < b->name;
            return a->index < b->index;
        });
        // BloomTG::initialize_bloom AnchorFinder.cpp:120-131
        uint64_t length_sum = estimate_length(all);
        if (anchor * 2 < 64) {
            uint64_t all_anchors = uint64_t(1) << (anchor * 2);
            if (all_anchors < length_sum) length_sum = all_anchors;
        }
        double error_prob = double(fp_x1e4) / 10000.0;  // Decimal::to_d
        int64_t m = optimal_bits(length_sum, error_prob);
        if (m < 0) return -1;
        int kb = optimal_hashes(length_sum, (uint64_t)m);
        Bloom bloom;
        bloom.bits.assign((size_t)m, false);
        if (!explicit_params.empty()) {
            bloom.params = explicit_params;
            bloom.params.resize(kb, 0);
            if ((int)explicit_params.size() < kb) return -2;
        } else {
            GlibcRand rnd(seed);
            for (int i = 0; i < kb; i++) bloom.params.push_back((hash_t)rnd.next());
        }
        out.members = (int64_t)length_sum;
        out.bits = m;
        out.hashes = kb;
        out.params = bloom.params;

        auto used = [&](hash_t h) {
            return std::binary_search(used_hashes.begin(), used_hashes.end(), h);
        };

        // pass 1: BloomTask AnchorFinder.cpp:152-197 (one worker, rank order)
        std::vector<hash_t> hashes;
        for (size_t r = 0; r < seqs.size(); r++) {
            const std::string& s = seqs[r]->data;
            const int k = anchor;
            // SeqI::init_state SeqI.hpp:86-96
            int ns = 0;
            for (int i = 0; i < k; i++) ns += (s[i] == 'N');
            hash_t dir = make_hash(s.c_str(), k, 1);
            hash_t rev = make_hash(s.c_str() + k - 1, k, -1);
            bool prev = false;
            auto test_and_add = [&]() {
                bool found = false;
                if (ns == 0) {
                    hash_t h = std::min(dir, rev);
                    if (!used(h)) {
                        found = bloom.test_and_add(h);
                        if (found && (!prev || !similar)) hashes.push_back(h);
                    }
                }
                prev = found;
            };
            test_and_add();
            size_t n = s.size() - k;
            for (size_t i = 0; i < n; i++) {
                // SeqI::next_hash SeqI.hpp:105-119
                char rm = s[i], ad = s[i + k];
                if (rm == 'N') ns -= 1;
                if (ad == 'N') ns += 1;
                dir = reuse_hash(dir, k, rm, ad, true);
                rev = reuse_hash(rev, k, complement_char(rm), complement_char(ad), false);
                test_and_add();
            }
        }
        // bloomtg_postprocess AnchorFinder.cpp:213-218
        std::sort(hashes.begin(), hashes.end());
        hashes.erase(std::unique(hashes.begin(), hashes.end()), hashes.end());
        out.n_collected = (int64_t)hashes.size();

        // pass 2: FragmentTask AnchorFinder.cpp:283-326
        std::vector<FoundFragment> ffs;
        for (size_t r = 0; r < seqs.size(); r++) {
            const std::string& s = seqs[r]->data;
            const int k = anchor;
            int ns = 0;
            for (int i = 0; i < k; i++) ns += (s[i] == 'N');
            hash_t dir = make_hash(s.c_str(), k, 1);
            hash_t rev = make_hash(s.c_str() + k - 1, k, -1);
            uint64_t pos = 0;
            auto test_and_push = [&]() {
                if (ns == 0) {
                    hash_t h = std::min(dir, rev);
                    if (std::binary_search(hashes.begin(), hashes.end(), h)) {
                        bool direct = (h == dir);
                        uint64_t p = pos + (direct ? 0 : s.size());
                        ffs.push_back(FoundFragment{h, (int)r, p});
                    }
                }
            };
            test_and_push();
            size_t n = s.size() - k;
            for (size_t i = 0; i < n; i++) {
                char rm = s[i], ad = s[i + k];
                pos += 1;
                if (rm == 'N') ns -= 1;
                if (ad == 'N') ns += 1;
                dir = reuse_hash(dir, k, rm, ad, true);
                rev = reuse_hash(rev, k, complement_char(rm), complement_char(ad), false);
                test_and_push();
            }
        }
        out.n_found_frags = (int64_t)ffs.size();
        // fragmenttg_postprocess AnchorFinder.cpp:356-391
        std::sort(ffs.begin(), ffs.end());
        if ((int64_t)ffs.size() > max_anchor_fragments) ffs.resize((size_t)max_anchor_fragments);
        bool sort_used = !used_hashes.empty();
        const FoundFragment* prev = nullptr;
        bool in_block = false;
        auto emit = [&](const FoundFragment& ff) {
            const Seq* sq = seqs[ff.rank];
            uint64_t size = sq->data.size();
            bool direct = ff.pos < size;   // FoundFragment::make_fragment :240-246
            uint64_t min_pos = direct ? ff.pos : ff.pos - size;
            out.frag_seq.push_back(sq->index);
            out.frag_min.push_back((int64_t)min_pos);
            out.frag_max.push_back((int64_t)(min_pos + anchor - 1));
            out.frag_ori.push_back(direct ? 1 : -1);
        };
        for (const FoundFragment& ff : ffs) {
            if (prev == nullptr) {
                prev = &ff;
            } else if (prev->hash == ff.hash) {
                if (!in_block) {
                    in_block = true;
                    out.block_start.push_back((int64_t)out.frag_seq.size());
                    out.block_hash.push_back(ff.hash);
                    emit(*prev);
                }
                emit(ff);
            } else {
                prev = &ff;
                in_block = false;
                used_hashes.push_back(ff.hash);
            }
        }
        out.block_start.push_back((int64_t)out.frag_seq.size());
        if (sort_used) std::sort(used_hashes.begin(), used_hashes.end());
        return 0;
    }
};

// ---------------------------------------------------------------- Decimal
// util/Decimal.hpp:25-213 (int64 x 1e4 fixed point) -- only what the path uses
struct Decimal {
    int64_t impl;
    static Decimal raw(int64_t v) { Decimal d; d.impl = v; return d; }
    int64_t to_i() const { return impl >= 0 ? impl / 10000 : -(-impl / 10000); }
    int64_t fraction() const { return (impl < 0 ? -impl : impl) % 10000; }
    int64_t round() const {
        if (fraction() < 5000) return to_i();
        int64_t r = to_i();
        r += (r < 0) ? -1 : 1;
        return r;
    }
    Decimal operator-(const Decimal& o) const { return raw(impl - o.impl); }
    Decimal operator*(const Decimal& o) const { return raw(impl * o.impl / 10000); }
    Decimal operator/(const Decimal& o) const { return raw(impl * 10000 / o.impl); }
};

// ---------------------------------------------------------------- FindLowSimilar
struct Region { int start, stop, good, weight; int length() const { return stop - start + 1; } };
typedef std::vector<Region> Regions;

// FindLowSimilar.cpp:48-54
static void set_weight(Region& r, int wf) { r.weight = r.good ? r.length() : r.length() * wf; }
// FindLowSimilar.cpp:56-60
static int get_weight_factor(int64_t min_identity_x1e4) {
    int64_t mi = std::min<int64_t>(min_identity_x1e4, 9900);
    Decimal one = Decimal::raw(10000);
    return (int)(one / (one - Decimal::raw(mi))).round();
}
// FindLowSimilar.cpp:62-80
static Regions make_regions(const std::vector<bool>& good_col, int wf) {
    Regions result;
    for (size_t i = 0; i < good_col.size(); i++) {
        if (!result.empty() && result.back().good == (int)good_col[i]) {
            result.back().stop = (int)i;
            set_weight(result.back(), wf);
        } else {
            Region r{(int)i, (int)i, (int)good_col[i], 0};
            set_weight(r, wf);
            result.push_back(r);
        }
    }
    return result;
}
// FindLowSimilar.cpp:82-92
static int find_min_region(const Regions& regions) {
    int min_index = 0;
    int min_weight = regions[0].weight;
    for (size_t i = 0; i < regions.size(); i++) {
        if (regions[i].weight < min_weight) {
            min_index = (int)i;
            min_weight = regions[i].weight;
        }
    }
    return min_index;
}
// FindLowSimilar.cpp:94-119
static Regions merge_region(const Regions& regions, int index) {
    Region region = regions[index];
    Region nr = region;
    if (index > 0) {
        nr.start = regions[index - 1].start;
        nr.weight += regions[index - 1].weight;
    }
    if (index < (int)regions.size() - 1) {
        nr.stop = regions[index + 1].stop;
        nr.weight += regions[index + 1].weight;
    }
    nr.good = region.good == 0 ? 1 : 0;
    Regions result;
    for (int i = 0; i < (int)regions.size(); i++) {
        if (i == index) result.push_back(nr);
        else if (i != index - 1 && i != index + 1) result.push_back(regions[i]);
    }
    return result;
}
// FindLowSimilar.cpp:121-130
static void reduce_regions(Regions& regions, int min_length) {
    while (regions.size() >= 2) {
        int mi = find_min_region(regions);
        if (regions[mi].weight >= min_length) break;
        regions = merge_region(regions, mi);
    }
}

// ---------------------------------------------------------------- SimilarAligner
static int64_t g_past_end_reads = 0;

struct Alignment {  // SimilarAligner.cpp:28-39
    const Strings& seqs;
    Strings aligned;
    std::vector<int> pos;
    int size;
    explicit Alignment(const Strings& s) : seqs(s), size((int)s.size()) {
        aligned.resize(size);
        pos.resize(size);
    }
};

struct SimilarAlignerImpl {  // SimilarAligner.cpp:41-485
    int mismatch_check = 1, gap_check = 2, aligned_check = 10, min_length = 100;
    int64_t min_identity_x1e4 = 9000;

    // character read with the documented past-the-end convention
    static int at(const Alignment& aln, int i, int p) {
        const std::string& s = aln.seqs[i];
        if (p < (int)s.size()) return (unsigned char)s[p];
        if (p == (int)s.size()) return 0;
        g_past_end_reads++;
        return 0x100 + i;
    }
    bool is_stop(const Alignment& aln, int shift = 0) const {  // :58-65
        for (int i = 0; i < aln.size; i++)
            if (aln.pos[i] + shift >= (int)aln.seqs[i].size()) return true;
        return false;
    }
    void append_cols(Alignment& aln, int cols = 1) const {  // :67-77
        for (int i = 0; i < aln.size; i++)
            for (int j = 0; j < cols; j++) {
                aln.aligned[i] += aln.seqs[i][aln.pos[i]];
                aln.pos[i] += 1;
            }
    }
    void append_gaps(Alignment& aln) const {  // :79-89
        size_t max_l = 0;
        for (int i = 0; i < aln.size; i++) max_l = std::max(max_l, aln.aligned[i].size());
        for (int i = 0; i < aln.size; i++) aln.aligned[i].resize(max_l, '-');
    }
    void append_all(Alignment& aln) const {  // :91-99
        for (int i = 0; i < aln.size; i++) {
            std::string tail = aln.seqs[i].substr(aln.pos[i]);
            aln.aligned[i] += tail;
            aln.pos[i] += (int)tail.size();
        }
        append_gaps(aln);
    }
    bool is_equal(const std::vector<int>& pos, const Alignment& aln, int shift = 0,
                  int cols = 1) const {  // :101-115
        for (int j = 0; j < cols; j++) {
            int c = at(aln, 0, pos[0] + shift + j);
            for (int i = 1; i < aln.size; i++)
                if (at(aln, i, pos[i] + shift + j) != c) return false;
        }
        return true;
    }
    bool is_equal(const Alignment& aln, int shift = 0, int cols = 1) const {
        return is_equal(aln.pos, aln, shift, cols);
    }
    bool try_mismatch(Alignment& aln) const {  // :122-134
        if (!is_stop(aln, mismatch_check) && is_equal(aln, 1, mismatch_check)) {
            append_cols(aln, mismatch_check + 1);
            return true;
        }
        return false;
    }
    void append_chars(Alignment& aln, int i, int cols = 1) const {  // :136-143
        for (int j = 0; j < cols; j++) {
            aln.aligned[i] += aln.seqs[i][aln.pos[i]];
            aln.pos[i] += 1;
        }
    }
    bool make_gap_shift(std::vector<int>& equal_pos, char c, const Alignment& aln) const {
        // :145-163
        equal_pos.resize(aln.size);
        for (int i = 0; i < aln.size; i++) {
            int p = aln.pos[i];
            bool match_this = at(aln, i, p) == (unsigned char)c;
            bool match_next = at(aln, i, p + 1) == (unsigned char)c;
            if (match_this == match_next) return false;
            equal_pos[i] = match_this ? p : p + 1;
        }
        return is_equal(equal_pos, aln, 0, gap_check);
    }
    void apply_gap(Alignment& aln, const std::vector<int>& equal_pos, int gc) const {
        // :165-174
        for (int i = 0; i < aln.size; i++)
            if (equal_pos[i] == aln.pos[i] + 1) append_chars(aln, i);
        append_gaps(aln);
        append_cols(aln, gc);
    }
    void find_all_gaps(std::vector<std::vector<int>>& variants, const Alignment& aln) const {
        // :176-189 -- std::set<char> iterates in ascending char order
        std::set<char> chars;
        for (int i = 0; i < aln.size; i++) chars.insert(aln.seqs[i][aln.pos[i]]);
        for (char c : chars) {
            std::vector<int> ep;
            if (make_gap_shift(ep, c, aln)) variants.push_back(ep);
        }
    }
    void find_best_gap(std::vector<std::vector<int>>& variants, Alignment& aln) const {
        // :191-217
        for (int gc = gap_check + 1;; gc += 1) {
            std::vector<std::vector<int>> next;
            for (const auto& ep : variants)
                if (is_equal(ep, aln, 0, gc)) next.push_back(ep);
            if (next.empty()) {
                apply_gap(aln, variants.front(), gc - 1);
                return;
            } else if (next.size() == 1) {
                apply_gap(aln, next.front(), gc);
                return;
            }
            variants.swap(next);
        }
    }
    bool try_gap(Alignment& aln) const {  // :219-235
        if (is_stop(aln, gap_check)) return false;
        std::vector<std::vector<int>> variants;
        find_all_gaps(variants, aln);
        if (variants.empty()) return false;
        if (variants.size() == 1) {
            apply_gap(aln, variants.front(), gap_check);
            return true;
        }
        find_best_gap(variants, aln);
        return true;
    }
    int min_tail(const Alignment& aln) const {  // :237-244
        int mt = (int)aln.seqs[0].size() - aln.pos[0];
        for (int i = 1; i < aln.size; i++)
            mt = std::min(mt, (int)aln.seqs[i].size() - aln.pos[i]);
        return mt;
    }
    typedef std::map<int, int> Seq2Pos;
    typedef std::map<std::string, Seq2Pos> Found;
    std::string find_best_word(const Alignment& aln, Found& ff, int shift) const {
        // :246-272
        std::set<std::string> words;
        std::string best_word;
        for (int i = 0; i < aln.size; i++) {
            std::string word = aln.seqs[i].substr(aln.pos[i] + shift, aligned_check);
            words.insert(word);
            Seq2Pos& s2p = ff[word];
            if (s2p.find(i) == s2p.end()) s2p[i] = shift;
            if ((int)s2p.size() == aln.size) best_word = word;
        }
        if (words.size() == 1) {
            best_word = *words.begin();
            for (int i = 0; i < aln.size; i++) ff[best_word][i] = shift;
        }
        return best_word;
    }
    void append_aligned(Alignment& aln, const Seq2Pos& s2p) const {  // :274-293
        Strings tmp((size_t)aln.size);
        for (int i = 0; i < aln.size; i++) {
            tmp[i] = aln.seqs[i].substr(aln.pos[i], s2p.find(i)->second);
            std::reverse(tmp[i].begin(), tmp[i].end());
        }
        process_seqs(tmp);
        for (int i = 0; i < aln.size; i++) {
            std::reverse(tmp[i].begin(), tmp[i].end());
            aln.aligned[i] += tmp[i];
            aln.pos[i] += s2p.find(i)->second;
        }
    }
    bool try_aligned(Alignment& aln) const {  // :295-308
        Found ff;
        int max_shift = min_tail(aln) - aligned_check;
        for (int shift = 0; shift < max_shift; shift++) {
            std::string best = find_best_word(aln, ff, shift);
            if (!best.empty()) {
                append_aligned(aln, ff[best]);
                append_cols(aln, aligned_check);
                return true;
            }
        }
        return false;
    }
    static bool pos_less(const std::vector<int>& a, const std::vector<int>& b, int shift = 0) {
        for (size_t i = 0; i < a.size(); i++)  // :310-320
            if (a[i] >= b[i] + shift) return false;
        return true;
    }
    void append_end(Alignment& aln) const {  // :323-342
        std::vector<int> end_pos((size_t)aln.size);
        for (int i = 0; i < aln.size; i++) end_pos[i] = (int)aln.seqs[i].size() - 1;
        while ((pos_less(aln.pos, end_pos) && is_equal(end_pos, aln)) ||
               (pos_less(aln.pos, end_pos, -1) && is_equal(end_pos, aln, -1))) {
            for (int i = 0; i < aln.size; i++) end_pos[i] -= 1;
        }
        for (int i = 0; i < aln.size; i++) append_chars(aln, i, end_pos[i] - aln.pos[i]);
        append_gaps(aln);
        append_all(aln);
    }
    void process_cols(Alignment& aln) const {  // :344-369
        for (int i = 0; i < aln.size; i++)
            if (aln.seqs[i].empty()) {
                append_all(aln);
                return;
            }
        while (true) {
            if (is_stop(aln)) {
                append_all(aln);
                return;
            } else if (is_equal(aln)) {
                append_cols(aln);
            } else if (try_mismatch(aln)) {
            } else if (try_gap(aln)) {
            } else if (try_aligned(aln)) {
            } else {
                append_end(aln);
                return;
            }
        }
    }
    void process_seqs(Strings& seqs) const {  // :396-405
        Alignment aln(seqs);
        process_cols(aln);
        seqs.swap(aln.aligned);
    }
    static void filter_out_gaps(Strings& a) {  // :379-386
        for (auto& s : a) s.erase(std::remove(s.begin(), s.end(), '-'), s.end());
    }
    static void reverse_strings(Strings& a) {  // :388-394
        for (auto& s : a) std::reverse(s.begin(), s.end());
    }
    int score_of(const Strings& rows) const {  // :416-426
        Alignment aln(rows);
        int score = 0;
        int length = (int)rows[0].size();
        for (int j = 0; j < length; j++)
            if (is_equal(aln, j)) score += 1;
        return score;
    }
    void fix_bad_regions(Strings& aligned) const {  // :428-459
        Alignment aln(aligned);
        int length = (int)aligned[0].size();
        std::vector<bool> good_col((size_t)length);
        for (int j = 0; j < length; j++) good_col[j] = is_equal(aln, j);
        int wf = get_weight_factor(min_identity_x1e4);
        Regions regions = make_regions(good_col, wf);
        reduce_regions(regions, min_length);
        Strings na((size_t)aln.size);
        for (const Region& r : regions) {
            if (r.good) {
                for (int i = 0; i < aln.size; i++) na[i] += aligned[i].substr(r.start, r.length());
            } else {
                Strings seqs((size_t)aln.size);
                for (int i = 0; i < aln.size; i++) seqs[i] = aligned[i].substr(r.start, r.length());
                int before = score_of(seqs);
                filter_out_gaps(seqs);
                reverse_strings(seqs);
                process_seqs(seqs);
                int after = score_of(seqs);
                if (after > before) {
                    reverse_strings(seqs);
                    for (int i = 0; i < aln.size; i++) na[i] += seqs[i];
                } else {
                    for (int i = 0; i < aln.size; i++)
                        na[i] += aligned[i].substr(r.start, r.length());
                }
            }
        }
        aligned.swap(na);
    }
    void realing_end(Strings& aligned) const {  // :461-484
        int size = (int)aligned.size();
        int length = (int)aligned[0].size();
        if (length < 2) return;
        int prefix_length = length - aligned_check;
        if (prefix_length < 1) prefix_length = 1;
        Strings tails((size_t)size);
        for (int i = 0; i < size; i++) {
            tails[i] = aligned[i].substr(prefix_length);
            aligned[i].resize(prefix_length);
        }
        filter_out_gaps(tails);
        reverse_strings(tails);
        process_seqs(tails);
        reverse_strings(tails);
        for (int i = 0; i < size; i++) aligned[i] += tails[i];
    }
    // SimilarAligner::similar_aligner SimilarAligner.cpp:487-501
    void similar_aligner(Strings& seqs) const {
        if (seqs.empty()) return;
        process_seqs(seqs);
        fix_bad_regions(seqs);
        realing_end(seqs);
    }
};

// AbstractAligner.cpp:71-102
static void remove_gaps(Strings& seqs) {
    int length = (int)seqs[0].size();
    int dest = 0;
    for (int src = 0; src < length; src++) {
        bool pure = true;
        for (auto& s : seqs)
            if (s[src] != '-') { pure = false; break; }
        if (!pure) {
            if (dest != src)
                for (auto& s : seqs) s[dest] = s[src];
            dest += 1;
        }
    }
    for (auto& s : seqs) s.resize(dest);
}

// AbstractAligner::align_seqs AbstractAligner.cpp:104-143; aligner: 0 = similar,
// 1 = dummy (DummyAligner.cpp:18-26).  MetaAligner's double wrapping
// (MetaAligner.cpp:76-84) is idempotent and not repeated here.
static void align_seqs(Strings& seqs, int aligner, const SimilarAlignerImpl& im) {
    if (seqs.empty()) return;
    std::vector<int> idx, empties;
    Strings ne;
    for (int i = 0; i < (int)seqs.size(); i++) {
        if (seqs[i].empty()) empties.push_back(i);
        else {
            idx.push_back(i);
            ne.push_back(std::string());
            ne.back().swap(seqs[i]);
        }
    }
    if (ne.empty()) return;
    if (aligner == 0) {
        im.similar_aligner(ne);
    } else {
        size_t ml = ne[0].size();
        for (auto& s : ne) ml = std::max(ml, s.size());
        for (auto& s : ne) s.resize(ml, '-');
    }
    size_t length = ne[0].size();
    for (size_t i = 0; i < idx.size(); i++) seqs[idx[i]].swap(ne[i]);
    for (int i : empties) seqs[i].resize(length, '-');
    for (auto& s : seqs)
        for (char& c : s) c = (char)toupper((unsigned char)c);
    remove_gaps(seqs);
}

// ---------------------------------------------------------------- refine_alignment
// refine_alignment.cpp:15-190
struct PosProps {
    bool gap = false, other = false;
    int matches = 0;
    PosProps(const Strings& a, int i, int j, char c) {
        for (int i1 = 0; i1 < (int)a.size(); i1++) {
            if (i1 == i) continue;
            char c1 = a[i1][j];
            if (c1 == '-') gap = true;
            else if (c1 == c) matches += 1;
            else other = true;
        }
    }
};
static bool can_move(const Strings& a, int i, int from, int to) {
    const std::string& row = a[i];
    char c = row[from], to_c = row[to];
    if ((c == '-') == (to_c == '-')) return false;
    PosProps fp(a, i, from, c), tp(a, i, to, c);
    if (tp.matches == 0) return false;
    if (!fp.other) return false;
    if (tp.other && fp.matches) return false;
    return true;
}
static bool try_move(Strings& a, int i, int from, int to) {
    bool r = can_move(a, i, from, to);
    if (r) std::swap(a[i][from], a[i][to]);
    return r;
}
static bool col_equal(const Strings& a, int j) {
    char c = a[0][j];
    for (size_t i = 1; i < a.size(); i++)
        if (a[i][j] != c) return false;
    return true;
}
static bool check_movable(Strings& a, int i, int first, int last) {
    int l = (int)a[0].size();
    const std::string& row = a[i];
    if (row[first] == '-') {
        if (first > 0 && try_move(a, i, first - 1, last)) return true;
        if (last < l - 1 && try_move(a, i, last + 1, first)) return true;
    } else {
        if (last < l - 1 && try_move(a, i, first, last + 1)) return true;
        if (first > 0 && try_move(a, i, last, first - 1)) return true;
        for (int j = first + 1; j <= last - 1; j++) {
            if (!col_equal(a, j)) {
                if (last < l - 1 && try_move(a, i, j, last + 1)) return true;
                if (first > 0 && try_move(a, i, j, first - 1)) return true;
            }
        }
    }
    return false;
}
static bool move_chars(Strings& a) {
    bool result = false;
    int size = (int)a.size();
    int length = (int)a[0].size();
    for (int i = 0; i < size; i++) {
        std::string& row = a[i];
        char repeated = row[0];
        int first = 0, last = 0;
        for (int j = 1; j < length; j++) {
            char c = row[j];
            if (c == repeated) {
                last = j;
            } else {
                result |= check_movable(a, i, first, last);
                repeated = row[j];
                first = j;
                last = j;
                while (first > 0 && row[first - 1] == repeated) first -= 1;
            }
        }
        result |= check_movable(a, i, first, last);
    }
    return result;
}
static void remove_pure_gaps(Strings& a) {
    int size = (int)a.size();
    int length = (int)a[0].size();
    Strings na((size_t)size);
    for (int j = 0; j < length; j++) {
        bool pure = true;
        for (int i = 0; i < size; i++)
            if (a[i][j] != '-') { pure = false; break; }
        if (!pure)
            for (int i = 0; i < size; i++) na[i] += a[i][j];
    }
    a.swap(na);
}
static void refine_alignment(Strings& a) {
    if (a.empty()) return;
    while (move_chars(a)) remove_pure_gaps(a);
    remove_pure_gaps(a);
}

}  // namespace orc

// ============================================================================
// C ABI used by oracle/oracle.py (ctypes).
// ============================================================================
extern "C" {

void orc_glibc_rand(uint32_t seed, int n, int32_t* out) {
    orc::GlibcRand r(seed);
    for (int i = 0; i < n; i++) out[i] = r.next();
}

uint64_t orc_make_hash(const char* s, int length, int ori) {
    return orc::make_hash(s, length, ori);
}
uint64_t orc_reuse_hash(uint64_t h, int length, char rm, char ad, int forward) {
    return orc::reuse_hash(h, length, rm, ad, forward != 0);
}
uint64_t orc_complement_hash(uint64_t h, int k) { return orc::complement_hash(h, k); }
int64_t orc_optimal_bits(uint64_t members, double p) { return orc::optimal_bits(members, p); }
int orc_optimal_hashes(uint64_t members, uint64_t bits) {
    return orc::optimal_hashes(members, bits);
}
int orc_weight_factor(int64_t min_identity_x1e4) {
    return orc::get_weight_factor(min_identity_x1e4);
}

// to_atgcn into caller buffer (capacity >= len); returns new length
int64_t orc_to_atgcn(const char* in, int64_t len, char* out) {
    std::string s = orc::to_atgcn(std::string(in, (size_t)len));
    memcpy(out, s.data(), s.size());
    return (int64_t)s.size();
}

// --- AnchorFinder -----------------------------------------------------------
struct orc_af {
    orc::AnchorFinder af;
    orc::AnchorResult res;
};

orc_af* orc_af_create(int anchor, int64_t fp_x1e4, int similar,
                      int64_t max_fragments, uint32_t seed) {
    orc_af* h = new orc_af;
    h->af.anchor = anchor;
    h->af.fp_x1e4 = fp_x1e4;
    h->af.similar = similar != 0;
    h->af.max_anchor_fragments = max_fragments;
    h->af.seed = seed;
    return h;
}
void orc_af_set_params(orc_af* h, const uint64_t* params, int n) {
    h->af.explicit_params.assign(params, params + n);
}
void orc_af_free(orc_af* h) { delete h; }

// Runs one AnchorFinder pass; returns 0 on success.
int orc_af_run(orc_af* h, int nseq, const char* const* seqs, const int64_t* lens,
               const char* const* names) {
    std::vector<orc::Seq> all((size_t)nseq);
    for (int i = 0; i < nseq; i++) {
        all[i].name = names[i];
        all[i].data = orc::to_atgcn(std::string(seqs[i], (size_t)lens[i]));
        all[i].index = i;
    }
    h->res = orc::AnchorResult();
    return h->af.run(all, h->res);
}
// stats: [members, bits, hashes, n_collected, n_found_frags, n_blocks, n_frags, n_used]
void orc_af_stats(const orc_af* h, int64_t* st) {
    st[0] = h->res.members;
    st[1] = h->res.bits;
    st[2] = h->res.hashes;
    st[3] = h->res.n_collected;
    st[4] = h->res.n_found_frags;
    st[5] = (int64_t)h->res.block_start.size() - 1;
    st[6] = (int64_t)h->res.frag_seq.size();
    st[7] = (int64_t)h->af.used_hashes.size();
}
void orc_af_params(const orc_af* h, uint64_t* out) {
    for (size_t i = 0; i < h->res.params.size(); i++) out[i] = h->res.params[i];
}
void orc_af_fragments(const orc_af* h, int32_t* seq, int64_t* mn, int64_t* mx, int32_t* ori,
                      int64_t* block_start) {
    const orc::AnchorResult& r = h->res;
    for (size_t i = 0; i < r.frag_seq.size(); i++) {
        seq[i] = r.frag_seq[i];
        mn[i] = r.frag_min[i];
        mx[i] = r.frag_max[i];
        ori[i] = r.frag_ori[i];
    }
    for (size_t i = 0; i < r.block_start.size(); i++) block_start[i] = r.block_start[i];
}
void orc_af_used(const orc_af* h, uint64_t* out) {
    for (size_t i = 0; i < h->af.used_hashes.size(); i++) out[i] = h->af.used_hashes[i];
}

// --- aligners -----------------------------------------------------------------
// rows: concatenated input rows, lens[i]; params: [mismatch, gap, aligned,
// min_length, min_identity_x1e4]; mode: 0 = similar_aligner only,
// 1 = AbstractAligner::align_seqs(similar), 2 = align_seqs(dummy),
// 3 = similar_aligner + refine_alignment, 4 = refine_alignment only,
// 5 = AbstractAligner::align_block (align_seqs + refine_alignment).
// Output written to out (capacity out_cap): rows back-to-back, each of length
// *out_len.  Returns 0, or -1 when out_cap is too small (then *out_len is set).
int orc_align(int nrows, const char* rows, const int64_t* lens, const int32_t* params,
              int mode, char* out, int64_t out_cap, int64_t* out_len,
              int64_t* past_end_reads) {
    Strings seqs((size_t)nrows);
    int64_t off = 0;
    for (int i = 0; i < nrows; i++) {
        seqs[i].assign(rows + off, (size_t)lens[i]);
        off += lens[i];
    }
    orc::SimilarAlignerImpl im;
    im.mismatch_check = params[0];
    im.gap_check = params[1];
    im.aligned_check = params[2];
    im.min_length = params[3];
    im.min_identity_x1e4 = params[4];
    orc::g_past_end_reads = 0;
    switch (mode) {
        case 0: im.similar_aligner(seqs); break;
        case 1: orc::align_seqs(seqs, 0, im); break;
        case 2: orc::align_seqs(seqs, 1, im); break;
        case 3: im.similar_aligner(seqs); orc::refine_alignment(seqs); break;
        case 4: orc::refine_alignment(seqs); break;
        case 5: orc::align_seqs(seqs, 0, im); orc::refine_alignment(seqs); break;
        default: return -2;
    }
    if (past_end_reads) *past_end_reads = orc::g_past_end_reads;
    int64_t L = seqs.empty() ? 0 : (int64_t)seqs[0].size();
    for (auto& s : seqs)
        if ((int64_t)s.size() != L) return -3;
    *out_len = L;
    if (L * nrows > out_cap) return -1;
    for (int i = 0; i < nrows; i++) memcpy(out + (int64_t)i * L, seqs[i].data(), (size_t)L);
    return 0;
}

}  // extern "C"
