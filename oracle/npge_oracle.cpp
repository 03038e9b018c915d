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
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>
#include <tuple>
#include <stdexcept>
#include <string>
#include <thread>
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

// BlocksJobs (BlocksJobs.cpp:38-240) over `workers` threads: fn(i, tid) for every
// block index i, blocks claimed `chunk` at a time from a shared counter.  Callers
// write per-index results, so the output does not depend on the thread count.
template <class F>
static void for_blocks(size_t n, int workers, F fn, size_t chunk = 16) {
    if (workers <= 1 || n < 2) {
        for (size_t i = 0; i < n; i++) fn(i, 0);
        return;
    }
    std::atomic<size_t> next(0);
    std::vector<std::thread> pool;
    for (int t = 0; t < std::min<int>(workers, (int)((n + chunk - 1) / chunk)); t++)
        pool.emplace_back([&, t] {
            for (;;) {
                size_t a = next.fetch_add(chunk);
                if (a >= n) break;
                for (size_t i = a; i < std::min(n, a + chunk); i++) fn(i, t);
            }
        });
    for (auto& th : pool) th.join();
}

struct AnchorFinder {
    int anchor = 20;
    int64_t fp_x1e4 = 1000;     // Decimal("0.1")
    bool similar = true;
    int64_t max_anchor_fragments = 100000;
    uint32_t seed = 1;
    std::vector<hash_t> explicit_params;  // overrides seed when non-empty
    std::vector<hash_t> used_hashes;      // AnchorFinder.cpp:30-35 (persistent)
    int workers = 1;                      // FragmentTG threads of pass 2 (one sequence per task)

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
        std::vector<std::vector<FoundFragment>> per_seq(seqs.size());
        for_blocks(seqs.size(), workers, [&](size_t r, int) {
            std::vector<FoundFragment>& ffs = per_seq[r];
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
        }, 1);
        std::vector<FoundFragment> ffs;
        for (auto& v : per_seq) ffs.insert(ffs.end(), v.begin(), v.end());
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


// ============================================================================
// Block-set model and the DraftPangenome block build (lua_lib.lua:1569-1621)
// ============================================================================
struct BSeq {
    std::string name, data, genome;
    int index;
};

// A fragment with an optional gapped row.  Letters of the row are always the
// fragment's own text in its orientation (Fragment::print_contents,
// Fragment.cpp:344-372).
struct BFrag {
    int seq;
    int64_t min, max;
    int ori;
    std::string row;  // empty = no row
    bool has_row = false;
    int64_t length() const { return max - min + 1; }
    int64_t begin() const { return ori == 1 ? min : max; }
    int64_t last() const { return ori == 1 ? max : min; }
};

// Block::Block() names a new block "00000000" (Block.cpp:29-34); ConSeq names
// each consensus sequence after its block (Sequence.cpp:318-320), so the
// consensus fragment ids -- and block_hash over them -- carry that name
static const char* const NULL_BLOCK_NAME = "00000000";

struct BBlock {
    std::vector<BFrag> f;
    std::string name = NULL_BLOCK_NAME;
    int64_t aln_len() const {
        if (f.empty()) return 0;
        return f[0].has_row ? (int64_t)f[0].row.size() : f[0].length();
    }
};

struct BlockSetO {
    std::vector<BSeq>* seqs;
    std::vector<BBlock> blocks;
};

// Sequence::substr_impl (Sequence.cpp:310-325): ori -1 walks down and complements
static std::string seq_substr(const BSeq& s, int64_t index, int64_t length, int ori) {
    std::string r;
    r.reserve((size_t)length);
    for (int64_t i = 0; i < length; i++) {
        char c = s.data[(size_t)index];
        if (ori == -1) c = complement_char(c);
        r += c;
        index += ori;
    }
    return r;
}

static std::string frag_text(const std::vector<BSeq>& seqs, const BFrag& f) {
    return seq_substr(seqs[f.seq], f.begin(), f.length(), f.ori);
}

// Fragment::str() with gap '-' (row) or plain text
static std::string frag_str(const std::vector<BSeq>& seqs, const BFrag& f) {
    if (f.has_row) return f.row;
    return frag_text(seqs, f);
}

// Fragment::id (Fragment.cpp:173-183)
static std::string frag_id(const std::vector<BSeq>& seqs, const BFrag& f, bool inv = false) {
    int ori = inv ? -f.ori : f.ori;
    int64_t a = ori == 1 ? f.min : f.max, b = ori == 1 ? f.max : f.min;
    if (a == b && ori == -1) b = -1;
    return seqs[f.seq].name + "_" + std::to_string(a) + "_" + std::to_string(b);
}

// block_hash (block_hash.cpp:29-55)
static uint64_t block_hash(const std::vector<BSeq>& seqs, const BBlock& b) {
    std::vector<std::string> d, v;
    for (const BFrag& f : b.f) {
        d.push_back(frag_id(seqs, f));
        v.push_back(frag_id(seqs, f, true));
    }
    std::sort(d.begin(), d.end());
    std::sort(v.begin(), v.end());
    const std::vector<std::string>& ids = (d < v) ? d : v;
    std::string joint;
    for (size_t i = 0; i < ids.size(); i++) {
        if (i) joint += ' ';
        joint += ids[i];
    }
    size_t ns = (joint.size() + 15) / 16 * 16;
    joint.resize(ns, ' ');
    uint64_t a = 1;
    for (size_t i = 0; i < ns / 16; i++) {
        uint64_t v0, v1;
        memcpy(&v0, joint.data() + 16 * i, 8);
        memcpy(&v1, joint.data() + 16 * i + 8, 8);
        a *= v0;
        a ^= v1;
    }
    return a;
}

// blockset_hash (block_hash.cpp:112-130): XOR over blocks of size > 1
static uint64_t blockset_hash(const BlockSetO& bs) {
    uint64_t h = 0;
    for (const BBlock& b : bs.blocks)
        if (b.f.size() > 1) h ^= block_hash(*bs.seqs, b);
    return h;
}

// ---------------------------------------------------------------- aligners as processors
// AbstractAligner::alignment_needed + align_block (AbstractAligner.cpp:51-69,145-177)
static void align_block(const std::vector<BSeq>& seqs, BBlock& b, int aligner,
                        const SimilarAlignerImpl& im) {
    if (b.f.empty()) return;
    if (b.f.size() == 1) {
        BFrag& f = b.f[0];
        if (f.has_row && (int64_t)f.row.size() == f.length()) return;
        f.row = frag_text(seqs, f);
        f.has_row = true;
        return;
    }
    if (b.f[0].has_row) {
        size_t L = b.f[0].row.size();
        bool all = true;
        for (const BFrag& f : b.f)
            if (!f.has_row || f.row.size() != L) { all = false; break; }
        if (all) return;
    }
    Strings rows;
    for (const BFrag& f : b.f) rows.push_back(frag_text(seqs, f));  // str(gap = 0)
    align_seqs(rows, aligner, im);
    refine_alignment(rows);
    for (size_t i = 0; i < b.f.size(); i++) {
        b.f[i].row = rows[i];
        b.f[i].has_row = true;
    }
}

// ---------------------------------------------------------------- FragmentsExtender
// FragmentsExtender.cpp:34-119
static int max_right_shift(const std::vector<BSeq>& seqs, const BFrag& f) {
    if (f.ori == 1) return (int)seqs[f.seq].data.size() - 1 - (int)f.max;
    return (int)f.min;
}

static void extend_right(const std::vector<BSeq>& seqs, BBlock& b, std::vector<std::string>& out,
                         int extend_length, const SimilarAlignerImpl& im, int64_t* aligned) {
    int rl = max_right_shift(seqs, b.f[0]);
    for (const BFrag& f : b.f) rl = std::min(rl, max_right_shift(seqs, f));
    rl = std::min(rl, extend_length);
    out.assign(b.f.size(), std::string());
    if (rl == 0) return;
    Strings rows;
    for (BFrag& f : b.f) {
        int64_t start = f.length();
        // Fragment::substr(start, stop) -> seq substr from frag_to_seq(start)
        int64_t sp = f.begin() + f.ori * start;
        rows.push_back(seq_substr(seqs[f.seq], sp, rl, f.ori));
        if (f.ori == 1) f.max += rl;  // shift_end
        else f.min -= rl;
    }
    if (aligned) for (auto& r : rows) *aligned += (int64_t)r.size();
    align_seqs(rows, 0, im);
    for (size_t i = 0; i < rows.size(); i++) out[i].swap(rows[i]);
}

static void fragments_extender(const std::vector<BSeq>& seqs, BBlock& b, int extend_length_opt,
                               int64_t portion_x1e4, const SimilarAlignerImpl& im,
                               int64_t* aligned) {
    if (b.f.size() < 2 || !b.f[0].has_row) return;
    std::vector<std::string> central;
    for (const BFrag& f : b.f) central.push_back(frag_str(seqs, f));
    int64_t length = b.aln_len();
    // (portion * length).to_i() with Decimal arithmetic
    int64_t portion_length = (portion_x1e4 * (length * 10000) / 10000) / 10000;
    int extend_length = (int)std::max<int64_t>(extend_length_opt, portion_length);
    std::vector<std::string> right, left;
    extend_right(seqs, b, right, extend_length, im, aligned);
    for (BFrag& f : b.f) f.ori = -f.ori;  // Block::inverse(false)
    extend_right(seqs, b, left, extend_length, im, aligned);
    for (BFrag& f : b.f) f.ori = -f.ori;
    for (size_t i = 0; i < b.f.size(); i++) {
        std::string l = left[i];
        complement_str(l);
        b.f[i].row = l + central[i] + right[i];
        b.f[i].has_row = true;
    }
}

// ---------------------------------------------------------------- FixEnds
// is_ident_nogap (block_stat.cpp:156-169) on gapped rows
static bool is_ident_nogap(const BBlock& b, int64_t col, bool reversed) {
    char seen = 0;
    const int64_t L = b.aln_len();
    for (const BFrag& f : b.f) {
        char c = f.row[(size_t)(reversed ? L - 1 - col : col)];
        if (c == '-') return false;
        if (reversed) c = complement_char(c);
        if (seen == 0) seen = c;
        else if (c != seen) return false;
    }
    return true;
}

// GoodAlnFinder (FixEnds.cpp:36-115)
struct GoodAlnFinder {
    const BBlock* block;
    bool reversed;
    std::vector<char> good_col;
    int64_t length;
    int min_fragment;
    int min_good, sub_frame, good;
    int64_t start, stop;
    void init_frame() {
        good_col.assign((size_t)min_fragment, 0);
        good = 0;
        for (int i = 0; i < min_fragment; i++) {
            bool g = is_ident_nogap(*block, i, reversed);
            good += g;
            good_col[i] = g;
        }
        start = 0;
        stop = min_fragment - 1;
    }
    void shift() {
        bool g = is_ident_nogap(*block, stop, reversed);
        char& c = good_col[(size_t)(stop % min_fragment)];
        good -= c;
        good += g;
        c = g;
    }
    bool start_is_good() const { return good_col[(size_t)(start % min_fragment)]; }
    bool find_first_good_frame() {
        while (true) {
            if (good >= min_good && start_is_good()) return true;
            start += 1;
            stop += 1;
            if (stop >= length) return false;
            shift();
        }
    }
    int64_t find_start() {
        if (length < min_fragment) return length;
        init_frame();
        if (!find_first_good_frame()) return length;
        int best_score = good;
        int64_t best_start = start;
        while (true) {
            start += 1;
            stop += 1;
            if (stop >= length) break;
            shift();
            bool ok = find_first_good_frame();
            if (!ok || start - best_start > sub_frame) break;
            if (good > best_score) {
                best_score = good;
                best_start = start;
            }
        }
        return best_start;
    }
};

// Block::slice with rows (Block.cpp:238-284): the letters of columns
// [start, stop]; fragments with no letter there are dropped.
static BBlock block_slice(const std::vector<BSeq>& seqs, const BBlock& b, int64_t start, int64_t stop) {
    BBlock r;
    for (const BFrag& f : b.f) {
        int64_t before = 0, cnt = 0;
        for (int64_t c = 0; c < start; c++) before += f.row[(size_t)c] != '-';
        for (int64_t c = start; c <= stop; c++) cnt += f.row[(size_t)c] != '-';
        if (cnt == 0) continue;
        int64_t s_start = f.begin() + f.ori * before;
        int64_t s_stop = f.begin() + f.ori * (before + cnt - 1);
        BFrag nf;
        nf.seq = f.seq;
        if (s_start <= s_stop) {  // Fragment::set_begin_last (Fragment.cpp:111-121)
            nf.min = s_start;
            nf.max = s_stop;
            nf.ori = 1;
        } else {
            nf.min = s_stop;
            nf.max = s_start;
            nf.ori = -1;
        }
        nf.row = f.row.substr((size_t)start, (size_t)(stop - start + 1));
        nf.has_row = true;
        if (nf.ori != f.ori) {
            // single letter of an ori -1 fragment: set_begin_last makes it ori +1 and
            // the row then shows the forward letter
            for (char& c : nf.row)
                if (c != '-') c = seqs[f.seq].data[(size_t)nf.min];
        }
        r.f.push_back(nf);
    }
    return r;
}

// FixEnds::process_block_impl (FixEnds.cpp:117-144): returns 0 keep, 1 replace, 2 drop
static int fix_ends(const std::vector<BSeq>& seqs, const BBlock& b, int min_fragment,
                    int64_t min_identity_x1e4, BBlock& out) {
    GoodAlnFinder g;
    g.block = &b;
    g.length = b.aln_len();
    g.min_fragment = min_fragment;
    // (min_identity * min_fragment).to_i(), ((1 - min_identity) * min_fragment).to_i()
    g.min_good = (int)((min_identity_x1e4 * ((int64_t)min_fragment * 10000) / 10000) / 10000);
    g.sub_frame = (int)(((10000 - min_identity_x1e4) * ((int64_t)min_fragment * 10000) / 10000) / 10000);
    g.reversed = false;
    int64_t sd = g.find_start();
    g.reversed = true;
    int64_t sr = g.find_start();
    if (sd == 0 && sr == 0) return 0;
    int64_t stop_direct = g.length - sr - 1;
    int64_t slice_length = stop_direct - sd + 1;
    if (slice_length >= min_fragment) {
        out = block_slice(seqs, b, sd, stop_direct);
        return 1;
    }
    return 2;
}

// ---------------------------------------------------------------- Filter
// ---------------------------------------------------------------- Rest
// Rest::run_impl (Rest.cpp:43-72) with add_f (:31-41): per sequence, the
// fragments sorted (VectorFc::prepare, Fragment::operator<: min, then max),
// a one-fragment block for the stretch before the first, between consecutive
// ones and after the last (a sequence without fragments: all of it)
static void rest(const std::vector<BSeq>& seqs, std::vector<BBlock>& blocks) {
    std::vector<std::vector<std::pair<int64_t, int64_t>>> fr(seqs.size());
    for (const BBlock& b : blocks)
        for (const BFrag& f : b.f) fr[(size_t)f.seq].push_back({f.min, f.max});
    std::vector<BBlock> add;
    auto add_f = [&](int s, int64_t mn, int64_t mx) {
        mn = std::max<int64_t>(0, mn);
        mx = std::min<int64_t>((int64_t)seqs[(size_t)s].data.size() - 1, mx);
        if (mn > mx) return;
        BBlock b;
        BFrag f;
        f.seq = s;
        f.min = mn;
        f.max = mx;
        f.ori = 1;
        b.f.push_back(f);
        add.push_back(b);
    };
    for (size_t s = 0; s < seqs.size(); s++) {
        auto& ff = fr[s];
        const int64_t size = (int64_t)seqs[s].data.size();
        if (ff.empty()) {
            add_f((int)s, 0, size - 1);
            continue;
        }
        std::sort(ff.begin(), ff.end());
        add_f((int)s, 0, ff[0].first - 1);
        for (size_t i = 1; i < ff.size(); i++) add_f((int)s, ff[i - 1].second + 1, ff[i].first - 1);
        add_f((int)s, ff.back().second + 1, size - 1);
    }
    for (auto& b : add) blocks.push_back(b);
}

// ---------------------------------------------------------------- ConSeq / DeConSeq
// A gapped row as the reference's AlignmentRow sees it: column -> fragment
// position (-1 = gap) and back (AlignmentRow.hpp:40-120).
struct RowMap {
    std::vector<int64_t> a2f, f2a;
    explicit RowMap(const std::string& row) : a2f(row.size(), -1) {
        for (size_t c = 0; c < row.size(); c++)
            if (row[c] != '-') {
                a2f[c] = (int64_t)f2a.size();
                f2a.push_back((int64_t)c);
            }
    }
    int64_t length() const { return (int64_t)a2f.size(); }
    int64_t map_to_fragment(int64_t col) const { return col >= 0 && col < length() ? a2f[(size_t)col] : -1; }
    int64_t map_to_alignment(int64_t pos) const {
        return pos >= 0 && pos < (int64_t)f2a.size() ? f2a[(size_t)pos] : -1;
    }
    // AlignmentRow::nearest_in_fragment_impl (AlignmentRow.cpp:101-112): left first
    int64_t nearest_in_fragment(int64_t col) const {
        for (int64_t d = 0; d <= length(); d++)
            for (int o = -1; o <= 1; o += 2) {
                const int64_t p = map_to_fragment(col + o * d);
                if (p != -1) return p;
            }
        return -1;
    }
};

// the row string of fragment f (letters = f's text in its orientation) for
// the fragment positions bound at columns: bound[col] = position or -1
static std::string row_from_binding(const std::vector<BSeq>& seqs, const BFrag& f,
                                    const std::vector<int64_t>& bound) {
    const std::string t = frag_text(seqs, f);
    std::string r(bound.size(), '-');
    for (size_t c = 0; c < bound.size(); c++)
        if (bound[c] >= 0) {
            if ((size_t)bound[c] >= t.size()) throw std::runtime_error("row binds a position past the fragment");
            r[c] = t[(size_t)bound[c]];
        }
    return r;
}

// Block::alignment_length (Block.cpp:133-139)
static int64_t block_alignment_length(const BBlock& b) {
    int64_t r = 0;
    for (const BFrag& f : b.f) r = std::max<int64_t>(r, f.has_row ? (int64_t)f.row.size() : f.length());
    return r;
}

// Block::consensus (Block.cpp:147-185): unaligned -> the first longest
// fragment's text; aligned -> consensus_char per column: counts of the letters
// (test_column, block_stat.cpp:188-210, char_to_size index < LETTERS_NUMBER = 5,
// i.e. A T G C N), the first letter in that order with the highest count
// (a column without letters: every count is 0 = the maximum -> 'A')
static std::string consensus(const std::vector<BSeq>& seqs, const BBlock& b) {
    if (b.f.empty()) return std::string();
    if (!b.f[0].has_row) {
        const BFrag* longest = &b.f[0];
        for (const BFrag& f : b.f)
            if (f.length() > longest->length()) longest = &f;
        return frag_text(seqs, *longest);
    }
    const int64_t L = block_alignment_length(b);
    std::string out((size_t)L, ' ');
    for (int64_t c = 0; c < L; c++) {
        int freq[5] = {0, 0, 0, 0, 0};
        for (const BFrag& f : b.f) {
            const char x = c < (int64_t)f.row.size() ? f.row[(size_t)c] : '-';  // alignment_at: 0 = gap
            if (x != '-') {
                const size_t li = char_to_size(x);
                if (li < 5) freq[li]++;
            }
        }
        int mx = 0;
        for (int l = 0; l < 5; l++) mx = std::max(mx, freq[l]);
        int l = 0;
        while (freq[l] != mx) l++;
        out[(size_t)c] = "ATGCN"[l];
    }
    return out;
}

// ConSeq::process_block_impl (ConSeq.cpp:37-50): one fragment -> the fragment
// itself (FragmentSequence), two or more -> Block::consensus
static std::string conseq_text(const std::vector<BSeq>& seqs, const BBlock& b) {
    if (b.f.size() == 1) return frag_text(seqs, b.f[0]);
    return consensus(seqs, b);
}

// proportion.hpp:16-23
static int64_t proportion(int64_t part1, int64_t total1, int64_t total2) {
    if (total1 == 0) return 0;
    const double percentage = double(part1) / double(total1);
    return (int64_t)(int)(percentage * (double)total2 + 0.00000001);
}

// fragment_pos (convert_position.cpp:44-67)
static int64_t fragment_pos(const BFrag& f, int64_t block_pos, int64_t block_length) {
    if (f.has_row) {
        int64_t r = RowMap(f.row).nearest_in_fragment(block_pos);
        if (r == -1) r = block_pos < block_length / 2 ? 0 : f.length();
        return r;
    }
    return proportion(block_pos, block_length, f.length());
}

// Fragment::set_begin_last (Fragment.cpp:117-127)
static void set_begin_last(BFrag& f, int64_t b, int64_t l) {
    if (b <= l) {
        f.min = b;
        f.max = l;
        f.ori = 1;
    } else {
        f.min = l;
        f.max = b;
        f.ori = -1;
    }
}

// Block::slice (Block.cpp:238-289) with AlignmentRow::slice (AlignmentRow.cpp:153-171)
static BBlock block_slice_full(const std::vector<BSeq>& seqs, const BBlock& b, int64_t start, int64_t stop,
                               bool alignment) {
    const int64_t bl = block_alignment_length(b);
    const int64_t mn = std::min(start, stop), mx = std::max(start, stop);
    const int ori = mn == start ? 1 : -1;
    BBlock r;
    for (const BFrag& f : b.f) {
        int64_t fs = fragment_pos(f, start, bl), fe = fragment_pos(f, stop, bl);
        if (f.has_row) {
            const RowMap m(f.row);
            const int64_t a = m.map_to_alignment(fs);
            if (a < mn || a > mx) fs += ori;
            const int64_t z = m.map_to_alignment(fe);
            if (z < mn || z > mx) fe -= ori;
        }
        if ((fe - fs) * ori < 0) continue;  // empty sub-fragment
        BFrag nf;
        nf.seq = f.seq;
        set_begin_last(nf, f.begin() + f.ori * fs, f.begin() + f.ori * fe);  // frag_to_seq
        if (alignment) {
            nf.has_row = true;
            if (f.has_row) {
                const RowMap m(f.row);
                std::vector<int64_t> bound((size_t)(mx - mn + 1), -1);
                int64_t fp = 0;
                for (int64_t c = 0; c < (int64_t)bound.size(); c++)
                    if (m.map_to_fragment(start + c * ori) != -1) bound[(size_t)c] = fp++;
                nf.row = row_from_binding(seqs, nf, bound);
            } else {
                nf.row = frag_text(seqs, nf);  // CompactAlignmentRow(new_fragment->str())
            }
        }
        r.f.push_back(nf);
    }
    return r;
}

// deconseq_row (DeConSeq.cpp:27-46): column i of the consensus fragment's row
// -> its fragment position -> the position bound there in the sliced row
static void deconseq_row(const std::vector<BSeq>& seqs, const BFrag& cons, BFrag& f) {
    const RowMap row(cons.row), tmp(f.row);
    std::vector<int64_t> bound((size_t)row.length(), -1);
    for (int64_t i = 0; i < row.length(); i++) {
        const int64_t tp = row.map_to_fragment(i);
        if (tp != -1) {
            const int64_t np = tmp.map_to_fragment(tp);
            if (np != -1) bound[(size_t)i] = np;
        }
    }
    f.row = row_from_binding(seqs, f, bound);
}

// DeConSeq::deconseq_block (DeConSeq.cpp:48-74): every fragment of a block
// over consensus sequences (sequence i = source block i) becomes the slice of
// that source block at the fragment's columns
static BBlock deconseq_block(const std::vector<BSeq>& seqs, const std::vector<BBlock>& source,
                             const BBlock& cb) {
    BBlock nb;
    nb.name = cb.name;
    for (const BFrag& cf : cb.f) {
        const BBlock& sb = source.at((size_t)cf.seq);
        BBlock t = block_slice_full(seqs, sb, cf.begin(), cf.last(), cf.has_row);
        for (BFrag& f : t.f) {
            if (f.has_row) deconseq_row(seqs, cf, f);
            nb.f.push_back(f);
        }
    }
    return nb;
}

static const int MAX_COLUMN_SCORE = 100;
static const int LOG_SCORE[1000] = {
#include "log_score.inc"
};

// goodColumns.cpp:10-31
static bool isColumnGood(const Strings& rows, int64_t i) {
    char first = rows[0][(size_t)i];
    bool ok = true;
    for (const auto& r : rows) ok &= r[(size_t)i] == first;
    return ok && first != '-' && first != 'N';
}
static bool isColumnIdentGap(const Strings& rows, int64_t i) {
    bool gap = false;
    int A = 0, T = 0, G = 0, C = 0, N = 0;
    for (const auto& r : rows) {
        char l = r[(size_t)i];
        gap |= l == '-';
        A |= l == 'A';
        T |= l == 'T';
        G |= l == 'G';
        C |= l == 'C';
        N |= l == 'N';
    }
    return gap && (A + T + G + C == 1) && !N;
}
// goodColumns.cpp:150-209
static void mapGap(std::vector<int>& sc, int64_t start, int64_t length, int min_identity, int min_length) {
    int64_t end = start + length;
    if (length >= 1000) length = 999;
    int score = LOG_SCORE[length];
    score = (score == MAX_COLUMN_SCORE) ? score : (score * min_identity / MAX_COLUMN_SCORE);
    if (length >= min_length) score = -100 * MAX_COLUMN_SCORE;
    for (int64_t i = start; i < end; i++) sc[(size_t)i] = score;
}
static std::vector<int> goodColumns(const Strings& rows, int64_t length, int min_identity, int min_length) {
    if (min_length == -1) min_length = (int)length;
    if (min_identity == -1) min_identity = MAX_COLUMN_SCORE;
    std::vector<int> sc((size_t)length, 0);
    int64_t gap_length = 0;
    for (int64_t i = 0; i < length; i++) {
        bool good = isColumnGood(rows, i);
        bool ig = isColumnIdentGap(rows, i);
        if (good) sc[(size_t)i] = MAX_COLUMN_SCORE;
        if (ig) gap_length += 1;
        else if (gap_length > 0) {
            mapGap(sc, i - gap_length, gap_length, min_identity, min_length);
            gap_length = 0;
        }
    }
    if (gap_length > 0) mapGap(sc, length - gap_length, gap_length, min_identity, min_length);
    return sc;
}

typedef std::pair<int64_t, int64_t> SS;
// goodSlices.cpp:17-245
struct GoodSlicer {
    std::vector<int> score;
    std::vector<int64_t> ssum, gsum;
    int64_t frame_length, end_length, frame_score, end_score, block_length, min_length;
    int min_identity;
    GoodSlicer(const std::vector<int>& sc, int64_t fl, int64_t el, int mi, int64_t ml) : score(sc) {
        block_length = (int64_t)sc.size();
        frame_length = std::min(fl, block_length);
        end_length = el;
        frame_score = frame_length * mi;
        end_score = el * mi;
        min_length = ml;
        min_identity = mi;
        ssum.assign((size_t)block_length + 1, 0);
        gsum.assign((size_t)block_length + 1, 0);
        for (int64_t i = 0; i < block_length; i++) {
            ssum[i + 1] = ssum[i] + sc[i];
            int v = (sc[i] == MAX_COLUMN_SCORE) ? MAX_COLUMN_SCORE : std::min(sc[i], 0);
            gsum[i + 1] = gsum[i] + v;
        }
    }
    int64_t countScore(int64_t a, int64_t b) const { return ssum[b + 1] - ssum[a]; }
    int64_t countGapless(int64_t a, int64_t b) const { return gsum[b + 1] - gsum[a]; }
    bool goodSlice(int64_t start) const { return countScore(start, start + frame_length - 1) >= frame_score; }
    bool goodLeftEnd(int64_t start) const {
        return score[start] == MAX_COLUMN_SCORE && countGapless(start, start + end_length - 1) >= end_score;
    }
    bool goodRightEnd(int64_t stop) const {
        return score[stop] == MAX_COLUMN_SCORE && countGapless(stop - end_length + 1, stop) >= end_score;
    }
    static int64_t len(const SS& s) { return s.second - s.first + 1; }
    static bool overlaps(const SS& a, const SS& o) {
        if (o.first <= a.first && a.first <= o.second) return true;
        if (a.first <= o.first && o.first <= a.second) return true;
        return false;
    }
    static SS exclude(const SS& a, const SS& o) {
        int64_t s1 = a.first, e1 = a.second;
        if (o.first <= a.first && a.first <= o.second) s1 = o.second + 1;
        if (o.first <= a.second && a.second <= o.second) e1 = o.first - 1;
        return SS(s1, e1);
    }
    bool valid(const SS& s) const { return len(s) >= min_length && s.first >= 0 && s.second < block_length; }
    SS strip(const SS& s) const {
        if (!valid(s)) return s;
        int64_t a = s.first, b = s.second;
        while (!goodLeftEnd(a) && a + end_length - 1 < b) a++;
        while (!goodRightEnd(b) && a + end_length - 1 < b) b--;
        return SS(a, b);
    }
    bool goodFrame(const SS& s) const {
        if (len(s) >= frame_length) return true;
        return countScore(s.first, s.second) >= (int64_t)min_identity * len(s);
    }
    bool goodEnds(const SS& s) const { return goodLeftEnd(s.first) && goodRightEnd(s.second) && goodFrame(s); }
    std::vector<SS> joinedSlices() const {
        std::vector<SS> s0;
        bool prev = false;
        for (int64_t i = 0; i <= block_length - frame_length; i++) {
            bool cur = goodSlice(i);
            if (cur) {
                if (prev) s0.back().second += 1;
                else s0.push_back(SS(i, i + frame_length - 1));
            }
            prev = cur;
        }
        std::vector<SS> out;
        for (const SS& s : s0) {
            SS t = strip(s);
            if (valid(t)) out.push_back(t);
        }
        return out;
    }
    std::vector<SS> calculate() const {
        if (min_length > block_length || min_length <= 0) return {};
        if (frame_length > block_length || frame_length <= 0) return {};
        if (end_length > min_length || end_length < 0) return {};
        std::vector<SS> slices = joinedSlices(), result;
        while (!slices.empty()) {
            SS sel = slices.front();
            for (const SS& s : slices)
                if (len(s) > len(sel)) sel = s;
            if (valid(sel) && goodEnds(sel)) {
                result.push_back(sel);
                std::vector<SS> n;
                for (const SS& s : slices) {
                    if (!overlaps(s, sel)) n.push_back(s);
                    else {
                        SS t = strip(exclude(s, sel));
                        if (valid(t) && goodEnds(t)) n.push_back(t);
                    }
                }
                slices.swap(n);
            } else {
                break;
            }
        }
        return result;
    }
};

struct FilterOpts {
    int min_fragment = 100, min_block = 2, max_block = -1, frame_length = 100, min_end = 10;
    int64_t min_identity_x1e4 = 9000;
    bool find_subblocks = true;
};

static int min_ident_count(int64_t mi) {  // Filter.cpp:112-120
    int64_t v = mi * 100 * 10000 / 10000;  // Decimal * 100
    int r = (int)(v / 10000);
    if (v % 10000) r += 1;
    return r;
}

static std::vector<SS> good_subblocks(const std::vector<BSeq>& seqs, const BBlock& b, const FilterOpts& o) {
    Strings rows;
    for (const BFrag& f : b.f) rows.push_back(frag_str(seqs, f));
    int64_t length = b.aln_len();
    int mi = min_ident_count(o.min_identity_x1e4);
    std::vector<int> sc = goodColumns(rows, length, mi, o.min_fragment);
    GoodSlicer gs(sc, o.frame_length, o.min_end, mi, o.min_fragment);
    return gs.calculate();
}

static bool frag_valid(const std::vector<BSeq>& seqs, const BFrag& f) {
    return f.min <= f.max && f.max < (int64_t)seqs[f.seq].data.size();
}

// Filter::is_good_block (Filter.cpp:143-174)
static bool filter_is_good(const std::vector<BSeq>& seqs, const BBlock& b, const FilterOpts& o) {
    int64_t L = b.aln_len();
    if (L < o.min_fragment) return false;
    for (const BFrag& f : b.f)
        if (!frag_valid(seqs, f)) return false;
    if ((int)b.f.size() < o.min_block) return false;
    if (o.max_block != -1 && (int)b.f.size() > o.max_block) return false;
    bool all_rows = true;
    for (const BFrag& f : b.f) all_rows &= f.has_row;
    if (all_rows && o.min_identity_x1e4 > 500) {
        std::vector<SS> sl = good_subblocks(seqs, b, o);
        if (!(sl.size() == 1 && sl[0] == SS(0, L - 1))) return false;
    }
    return true;
}

// Filter::find_good_subblocks (Filter.cpp:176-196)
static void filter_subblocks(const std::vector<BSeq>& seqs, const BBlock& b, const FilterOpts& o,
                             std::vector<BBlock>& out) {
    if ((int)b.f.size() < o.min_block) return;
    for (const BFrag& f : b.f)
        if (!f.has_row) return;
    if (b.aln_len() < o.min_fragment) return;
    for (const SS& s : good_subblocks(seqs, b, o)) out.push_back(block_slice(seqs, b, s.first, s.second));
}

// Filter::process_block_impl (Filter.cpp:208-248): 0 keep, 1 replaced by out, 2 drop
static int filter_block(const std::vector<BSeq>& seqs, BBlock& b, const FilterOpts& o,
                        std::vector<BBlock>& out) {
    if (filter_is_good(seqs, b, o)) return 0;
    std::vector<BBlock> sub;
    if (o.find_subblocks) filter_subblocks(seqs, b, o, sub);
    if (!sub.empty()) {
        for (auto& x : sub) out.push_back(x);
        return 1;
    }
    std::vector<BFrag> kept;
    for (const BFrag& f : b.f)
        if (frag_valid(seqs, f)) kept.push_back(f);
    if (kept.size() != b.f.size()) {
        b.f = kept;
        if (filter_is_good(seqs, b, o)) return 0;
        if (o.find_subblocks) filter_subblocks(seqs, b, o, out);
        return out.empty() ? 2 : 1;
    }
    return 2;
}

// ---------------------------------------------------------------- MoveGaps / CutGaps
// The row checks of MoveGaps / CutGaps (MoveGaps.cpp:37-44, CutGaps.cpp:66-74)
static int64_t checked_rows_length(const BBlock& b) {
    const int64_t length = block_alignment_length(b);
    for (const BFrag& f : b.f)
        if (!f.has_row || (int64_t)f.row.size() != length)
            throw std::logic_error("No alignment row is set, or its length differs from the block's");
    return length;
}

// AlignmentRow::map_to_fragment(col) != -1 on a gapped row (out of range: -1)
static bool letter_at(const std::string& row, int64_t col) {
    return col >= 0 && col < (int64_t)row.size() && row[(size_t)col] != '-';
}

// MoveGaps::move_gaps (MoveGaps.cpp:30-103): a terminal run of at most
// max_tail letters separated from the rest by a gap run (ending before the
// middle column) moves inside when tail / gap <= max_tail_to_gap (Decimal:
// tail * 10^4 / gap, truncated).  Returns whether a row changed.
static bool move_gaps(BBlock& b, int max_tail, int64_t max_tail_to_gap_x1e4) {
    const int64_t length = checked_rows_length(b);
    bool result = false;
    for (BFrag& f : b.f) {
        std::pair<int64_t, int64_t> moves[3] = {{0, 0}, {0, 0}, {0, 0}};  // index ori + 1
        for (int ori = -1; ori <= 1; ori += 2) {
            const int64_t begin = ori == 1 ? 0 : length - 1;
            int64_t tail = 0, i;
            for (i = 0; i < max_tail + 1; i++) {
                if (letter_at(f.row, begin + i * ori)) tail += 1;
                else break;
            }
            if (0 < tail && tail <= max_tail) {
                int64_t gap = 0;
                const int64_t max_pos = length / 2;
                for (; i < max_pos; i++) {
                    if (!letter_at(f.row, begin + i * ori)) gap += 1;
                    else break;
                }
                if (i < max_pos && gap != 0 && tail * 10000 / gap <= max_tail_to_gap_x1e4)
                    moves[ori + 1] = std::make_pair(tail, gap);
            }
        }
        if (moves[0].first != 0 || moves[2].first != 0) {
            result = true;
            std::string& data = f.row;
            for (int ori = -1; ori <= 1; ori += 2) {
                const int64_t begin = ori == 1 ? 0 : length - 1;
                const int64_t tail = moves[ori + 1].first, gap = moves[ori + 1].second;
                if (!tail) continue;
                for (int64_t i = tail - 1; i >= 0; i--) data[(size_t)(begin + (gap + i) * ori)] = data[(size_t)(begin + i * ori)];
                for (int64_t i = 0; i < gap; i++) data[(size_t)(begin + i * ori)] = '-';
            }
        }
    }
    return result;
}

// CutGaps' slice_fragment (CutGaps.cpp:26-61): the row's columns [from, to];
// the coordinates move by the letters cut (set_begin_pos / set_last_pos keep
// the orientation); no letter there -> the fragment leaves the block
static bool cut_fragment(BFrag& f, int64_t from, int64_t to) {
    const RowMap m(f.row);
    int64_t fr_from = -1, fr_to = -1;
    for (int64_t i = from; i <= to && fr_from == -1; i++) fr_from = m.map_to_fragment(i);
    if (fr_from == -1) return false;
    for (int64_t i = to; i >= from && fr_to == -1; i--) fr_to = m.map_to_fragment(i);
    const int64_t begin = f.begin() + fr_from * f.ori, last = f.begin() + fr_to * f.ori;
    f.row = f.row.substr((size_t)from, (size_t)(to - from + 1));
    if (f.ori == 1) {
        f.min = begin;
        f.max = last;
    } else {
        f.max = begin;
        f.min = last;
    }
    return true;
}

// CutGaps::cut_gaps (CutGaps.cpp:63-159): strict -- the first and the last
// gapless column; permissive -- the longest terminal gaps over the rows
static bool cut_gaps(BBlock& b, bool strict) {
    const int64_t length = checked_rows_length(b);
    int64_t from = 0, to = length - 1;
    if (strict) {
        auto gapless = [&](int64_t c) {
            for (const BFrag& f : b.f)
                if (!letter_at(f.row, c)) return false;
            return true;
        };
        for (; from <= to; from++)
            if (gapless(from)) break;
        for (; to >= from; to--)
            if (gapless(to)) break;
    } else {
        for (const BFrag& f : b.f)
            for (int ori = -1; ori <= 1; ori += 2) {
                const int64_t begin = ori == 1 ? 0 : length - 1;
                for (int64_t i = 0; i < length; i++) {
                    const int64_t al = begin + i * ori;
                    if (letter_at(f.row, al)) {
                        if (ori == 1 && al > from) from = al;
                        else if (ori == -1 && al < to) to = al;
                        break;
                    }
                }
            }
    }
    if (from == 0 && to == length - 1) return false;
    if (to < from) {
        b.f.clear();
        return true;
    }
    std::vector<BFrag> kept;
    for (BFrag& f : b.f)
        if (cut_fragment(f, from, to)) kept.push_back(std::move(f));
    b.f.swap(kept);
    return true;
}

// ---------------------------------------------------------------- SelfOverlapsResolver
// has_self_overlaps (hit.cpp:51-66): fragments sorted by (sequence, Fragment
// operator<) -- Sequence* pinned to the sequence index -- and neighbours
// tested for common positions
static bool has_self_overlaps(const BBlock& b) {
    if (b.f.empty()) return false;
    std::vector<const BFrag*> v;
    for (const BFrag& f : b.f) v.push_back(&f);
    std::sort(v.begin(), v.end(), [](const BFrag* x, const BFrag* y) {
        if (x->seq != y->seq) return x->seq < y->seq;
        if (x->min != y->min) return x->min < y->min;
        if (x->max != y->max) return x->max < y->max;
        return x->ori < y->ori;
    });
    for (size_t i = 0; i + 1 < v.size(); i++)
        if (v[i]->seq == v[i + 1]->seq && std::max(v[i]->min, v[i + 1]->min) <= std::min(v[i]->max, v[i + 1]->max))
            return true;
    return false;
}

// fix_self_overlaps (hit.cpp:68-91): the block's columns cut back from the
// end, one at a time, until no two fragments overlap; every fragment is
// replaced by a row-less one from its begin to the position of that column
// (fragment_pos, convert_position.cpp:44-67), one-letter ones dropped
static void fix_self_overlaps(BBlock& b) {
    if (!has_self_overlaps(b)) return;
    const BBlock copy = b;
    const int64_t block_length = block_alignment_length(copy);
    for (int64_t length = block_length - 1; length >= 0; length--) {
        b.f.clear();
        for (const BFrag& f : copy.f) {
            const int64_t seq_last = f.begin() + f.ori * fragment_pos(f, length, block_length);  // frag_to_seq
            const int64_t seq_begin = f.begin();
            if (seq_last != seq_begin) {
                BFrag nf;
                nf.seq = f.seq;
                set_begin_last(nf, seq_begin, seq_last);
                b.f.push_back(nf);
            }
        }
        if (!has_self_overlaps(b)) break;
    }
    if (has_self_overlaps(b)) throw std::logic_error("fix_self_overlaps left an overlap");
}

// ---------------------------------------------------------------- ExtendLoopFast driver
struct PipelineOpts {
    SimilarAlignerImpl im;
    int extend_length = 100;            // MIN_LENGTH
    int64_t portion_x1e4 = 0;           // FragmentsExtender --extend-length-portion (FragmentsExtender.cpp:28-30: 0.0)
    int fix_min_fragment = 100;
    int64_t fix_min_identity_x1e4 = 9000;
    int max_iterations = 10;
    FilterOpts filter;
    bool do_filter = true;
    int workers = 1;  // BlocksJobs workers (the reference's --workers); 1 = reference-exact sequential run
    int max_tail = 3;                       // MoveGaps max-tail (MAX_TAIL, CMakeLists.txt:89)
    int64_t max_tail_to_gap_x1e4 = 10000;   // MoveGaps max-tail-to-gap (MAX_TAIL_TO_GAP 1.0, CMakeLists.txt:90)
};

// Filter (Filter.cpp:208-248) over every block of the set
static void filter_all(const std::vector<BSeq>& seqs, std::vector<BBlock>& blocks, const FilterOpts& fo,
                       int workers) {
    std::vector<std::vector<BBlock>> subs(blocks.size());
    std::vector<int> res(blocks.size());
    for_blocks(blocks.size(), workers, [&](size_t i, int) { res[i] = filter_block(seqs, blocks[i], fo, subs[i]); });
    std::vector<BBlock> out;
    for (size_t i = 0; i < blocks.size(); i++) {
        if (res[i] == 0) out.push_back(std::move(blocks[i]));
        else if (res[i] == 1)
            for (auto& x : subs[i]) out.push_back(std::move(x));
    }
    blocks.swap(out);
}

// Align (Align.cpp:36-52): MetaAligner, SelfOverlapsResolver, MetaAligner,
// then AlignLoop = Pipe{MoveGaps, CutGaps, Filter} with set_max_iterations(-1)
// (Pipe.cpp:60-78: the block-set hash before the loop and after every lap;
// a lap ending on a seen hash ends the loop).  lite: LiteAlign (Align.cpp:17-30):
// MetaAligner, then Pipe{MoveGaps, CutGaps} to the same fixpoint.
static void align_pipe(BlockSetO& bs, const PipelineOpts& o, bool lite) {
    const std::vector<BSeq>& seqs = *bs.seqs;
    auto meta = [&] {
        for_blocks(bs.blocks.size(), o.workers, [&](size_t i, int) { align_block(seqs, bs.blocks[i], 0, o.im); });
    };
    meta();
    if (!lite) {
        for (BBlock& b : bs.blocks) fix_self_overlaps(b);
        meta();
    }
    std::set<uint64_t> seen;
    seen.insert(blockset_hash(bs));
    while (true) {
        for (BBlock& b : bs.blocks) move_gaps(b, o.max_tail, o.max_tail_to_gap_x1e4);
        for (BBlock& b : bs.blocks) cut_gaps(b, false);
        if (!lite) filter_all(seqs, bs.blocks, o.filter, o.workers);
        const uint64_t h = blockset_hash(bs);
        if (seen.count(h)) break;
        seen.insert(h);
    }
}


// RemoveNonStem --exact (RemoveNonStem.cpp:29-45)
static void remove_non_stem(BlockSetO& bs, bool exact) {
    std::set<std::string> genomes;
    for (const BSeq& s : *bs.seqs) genomes.insert(s.genome);
    std::vector<BBlock> keep;
    for (BBlock& b : bs.blocks) {
        std::set<std::string> g;
        bool ok = true;
        for (const BFrag& f : b.f) {
            const std::string& gn = (*bs.seqs)[f.seq].genome;
            if (exact && g.count(gn)) { ok = false; break; }
            g.insert(gn);
        }
        if (ok)
            for (const std::string& gn : genomes)
                if (!g.count(gn)) { ok = false; break; }
        if (ok) keep.push_back(std::move(b));
    }
    bs.blocks.swap(keep);
}

// pinned order for OverlaplessUnion (OverlaplessUnion.cpp:25-32 + block_less ties)
static bool frag_less(const BFrag& a, const BFrag& b) {  // Fragment::operator< (seq* -> index)
    if (a.min != b.min) return a.min < b.min;
    if (a.max != b.max) return a.max < b.max;
    if (a.ori != b.ori) return a.ori < b.ori;
    return a.seq < b.seq;
}
static const BFrag& min_frag(const BBlock& b) {
    size_t k = 0;
    for (size_t i = 1; i < b.f.size(); i++)
        if (frag_less(b.f[i], b.f[k])) k = i;
    return b.f[k];
}
static bool ou_before(const BBlock& a, const BBlock& b) {
    if (a.f.size() != b.f.size()) return a.f.size() > b.f.size();
    if (a.aln_len() != b.aln_len()) return a.aln_len() > b.aln_len();
    if (a.name != b.name) return a.name > b.name;
    if (a.f.empty()) return false;
    const BFrag& x = min_frag(a);
    const BFrag& y = min_frag(b);
    if (frag_less(x, y)) return true;
    if (frag_less(y, x)) return false;
    // final pin: sorted fragment lists
    std::vector<std::tuple<int64_t, int64_t, int, int>> fa, fb;
    for (const BFrag& f : a.f) fa.emplace_back(f.min, f.max, f.ori, f.seq);
    for (const BFrag& f : b.f) fb.emplace_back(f.min, f.max, f.ori, f.seq);
    std::sort(fa.begin(), fa.end());
    std::sort(fb.begin(), fb.end());
    return fa < fb;
}

// SetFc::has_overlap (FragmentCollection.hpp:273-297): neighbours in a
// per-sequence set ordered by Fragment::operator<
struct FragSetCmp {
    bool operator()(const BFrag& a, const BFrag& b) const { return frag_less(a, b); }
};
struct OverlapIndex {
    std::map<int, std::multiset<BFrag, FragSetCmp>> m;
    static bool common(const BFrag& a, const BFrag& b) {
        return a.seq == b.seq && std::max(a.min, b.min) <= std::min(a.max, b.max);
    }
    bool has_overlap(const BFrag& f) const {
        auto it = m.find(f.seq);
        if (it == m.end() || it->second.empty()) return false;
        auto i2 = it->second.lower_bound(f);
        if (i2 != it->second.end() && common(*i2, f)) return true;
        if (i2 != it->second.begin()) {
            --i2;
            if (common(*i2, f)) return true;
        }
        return false;
    }
    bool block_has_overlap(const BBlock& b) const {
        for (const BFrag& f : b.f)
            if (has_overlap(f)) return true;
        return false;
    }
    void add(const BBlock& b) {
        for (const BFrag& f : b.f) m[f.seq].insert(f);
    }
};

struct PipelineStats {
    int iterations = 0;
    int64_t aligned_residues = 0;   // flank residues sent to the aligner
    int64_t anchor_blocks = 0, stem_blocks = 0;
};

// ExtendLoopFast (lua_lib.lua:697-709) under Pipe::run_impl (Pipe.cpp:60-78)
// OverlaplessUnion --ou-move into an empty target (OverlaplessUnion.cpp:55-77):
// blocks in ou_before order (ties: input order), admitted greedily if no
// fragment overlaps an admitted one
static void overlapless_union(std::vector<BBlock>& blocks) {
    std::vector<size_t> order(blocks.size());
    for (size_t i = 0; i < order.size(); i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return ou_before(blocks[a], blocks[b]); });
    OverlapIndex idx;
    std::vector<BBlock> ol;
    for (size_t i : order) {
        if (!idx.block_has_overlap(blocks[i])) {
            idx.add(blocks[i]);
            ol.push_back(std::move(blocks[i]));
        }
    }
    blocks.swap(ol);
}

static void extend_loop_fast(BlockSetO& bs, const PipelineOpts& o, PipelineStats& st) {
    const std::vector<BSeq>& seqs = *bs.seqs;
    std::set<uint64_t> seen_states;
    seen_states.insert(blockset_hash(bs));
    std::vector<uint64_t> mu_hashes;  // MoveUnchanged::hashes_ (sorted)
    for (int it = 0; it < o.max_iterations || o.max_iterations == -1; it++) {
        st.iterations++;
        // MoveUnchanged target=unchanged other=target
        std::vector<BBlock> unchanged, work;
        std::vector<uint64_t> fresh;
        for (BBlock& b : bs.blocks) {
            uint64_t h = block_hash(seqs, b);
            if (std::binary_search(mu_hashes.begin(), mu_hashes.end(), h)) unchanged.push_back(std::move(b));
            else {
                fresh.push_back(h);
                work.push_back(std::move(b));
            }
        }
        for (uint64_t h : fresh) mu_hashes.push_back(h);
        std::sort(mu_hashes.begin(), mu_hashes.end());
        mu_hashes.erase(std::unique(mu_hashes.begin(), mu_hashes.end()), mu_hashes.end());
        // ExtendAndFix: FragmentsExtender --extend-length-portion:=0.5, FixEnds
        // (lua_lib.lua:690-695; ":=" fixes the value whatever the options)
        const int64_t extend_and_fix_portion = 5000;
        std::vector<int64_t> aligned((size_t)std::max(o.workers, 1), 0);
        std::vector<BBlock> outs(work.size());
        std::vector<int> res(work.size(), 0);
        for_blocks(work.size(), o.workers, [&](size_t i, int t) {
            BBlock& b = work[i];
            fragments_extender(seqs, b, o.extend_length, extend_and_fix_portion, o.im, &aligned[(size_t)t]);
            if (b.f.empty() || !b.f[0].has_row) return;  // FixEnds asserts alignment; anchors have rows
            res[i] = fix_ends(seqs, b, o.fix_min_fragment, o.fix_min_identity_x1e4, outs[i]);
        });
        for (int64_t a : aligned) st.aligned_residues += a;
        std::vector<BBlock> fixed;
        for (size_t i = 0; i < work.size(); i++) {
            if (res[i] == 0) fixed.push_back(std::move(work[i]));
            else if (res[i] == 1) fixed.push_back(std::move(outs[i]));
        }
        // Move target=target other=unchanged
        for (BBlock& b : unchanged) fixed.push_back(std::move(b));
        // OverlaplessUnion target=ol other=target --ou-move:=1
        const size_t n_ou = fixed.size();
        overlapless_union(fixed);
        // Clear target; Move target=target other=ol; Clear ol
        bs.blocks.swap(fixed);
        uint64_t h = blockset_hash(bs);
        static const bool dbg = getenv("ORACLE_ELF_DEBUG") != nullptr;  // (diagnostic: per-iteration state)
        if (dbg)
            fprintf(stderr, "elf it %d: ou_in %zu kept %zu state %016llx\n", it, n_ou, bs.blocks.size(),
                    (unsigned long long)h);
        if (seen_states.count(h)) break;
        seen_states.insert(h);
    }
}

// DraftPangenome without the random genome subset (ngenomes = all):
// AnchorFinder -> RemoveNonStem --exact -> DummyAligner -> ExtendLoopFast(10) -> Filter
static void draft_pangenome(std::vector<BSeq>& seqs, AnchorFinder& af, const PipelineOpts& o,
                            BlockSetO& bs, PipelineStats& st) {
    std::vector<Seq> all(seqs.size());
    for (size_t i = 0; i < seqs.size(); i++) {
        all[i].name = seqs[i].name;
        all[i].data = seqs[i].data;
        all[i].index = (int)i;
    }
    AnchorResult ar;
    af.run(all, ar);
    bs.seqs = &seqs;
    bs.blocks.clear();
    for (size_t b = 0; b + 1 < ar.block_start.size(); b++) {
        BBlock blk;
        for (int64_t i = ar.block_start[b]; i < ar.block_start[b + 1]; i++) {
            BFrag f;
            f.seq = ar.frag_seq[i];
            f.min = ar.frag_min[i];
            f.max = ar.frag_max[i];
            f.ori = ar.frag_ori[i];
            blk.f.push_back(f);
        }
        bs.blocks.push_back(blk);
    }
    st.anchor_blocks = (int64_t)bs.blocks.size();
    remove_non_stem(bs, true);
    st.stem_blocks = (int64_t)bs.blocks.size();
    for_blocks(bs.blocks.size(), o.workers,
               [&](size_t i, int) { align_block(seqs, bs.blocks[i], 1, o.im); });  // DummyAligner
    extend_loop_fast(bs, o, st);
    if (o.do_filter) filter_all(seqs, bs.blocks, o.filter, o.workers);
}


// ================================================================ AnchorLoop
// The AnchorLoop pipe (lua_lib.lua:711-737) and the processors only it uses:
// UniqueNames, RemoveWithSameName, SplitExtendable, ExtendLoop with
// AddingLoopBySize.

// block_less (block_hash.cpp:190-215): size, alignment length, the smallest
// fragment (Fragment::operator<, the Sequence* compare pinned to the index)
static bool block_less_ref(const BBlock& a, const BBlock& b) {
    if (a.f.size() != b.f.size()) return a.f.size() < b.f.size();
    if (a.f.empty()) return false;
    if (a.aln_len() != b.aln_len()) return a.aln_len() < b.aln_len();
    return frag_less(min_frag(a), min_frag(b));
}

// block_name (block_hash.cpp:132-177): u (one fragment), r (two fragments of
// one genome), s (one per genome), h; then size "x" alignment length
static std::string block_name(const std::vector<BSeq>& seqs, const BBlock& b, int genomes) {
    bool repeats = false;
    std::set<std::string> g;
    for (const BFrag& f : b.f) {
        if (!g.insert(seqs[(size_t)f.seq].genome).second) {
            repeats = true;
            break;
        }
    }
    const char type = b.f.size() == 1 ? 'u' : repeats ? 'r' : (int)b.f.size() == genomes ? 's' : 'h';
    return std::string(1, type) + std::to_string(b.f.size()) + "x" + std::to_string(b.aln_len());
}

// rand_name(8) (rand_name.cpp:34-46: 8 hex digits, a letter first) drawn from
// the clock-seeded rand(); here the k-th name "a" + 7 hex digits of k
static std::string det_seq_name(uint64_t k) {
    static const char* const hex = "0123456789abcdef";
    std::string r = "a0000000";
    for (int i = 7; i >= 1; i--, k >>= 4) r[(size_t)i] = hex[k & 15];
    return r;
}

// UniqueNames (UniqueNames.cpp:23-67): blocks with the null or an empty name
// get their canonical name, then repeated names get "n1", "n2", ... in
// block_greater order (ties: set order); sequences with an empty or a repeated
// name get a fresh one
static void unique_names(std::vector<BSeq>& seqs, std::vector<BBlock>& blocks) {
    std::set<std::string> all_genomes;
    for (const BSeq& s : seqs) all_genomes.insert(s.genome);
    const int genomes = (int)all_genomes.size();
    for (BBlock& b : blocks)
        if (b.name == NULL_BLOCK_NAME || b.name.empty()) b.name = block_name(seqs, b, genomes);
    std::vector<size_t> order(blocks.size());
    for (size_t i = 0; i < order.size(); i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(),
                     [&](size_t a, size_t b) { return block_less_ref(blocks[b], blocks[a]); });
    std::set<std::string> names;
    std::map<std::string, int> last_n;
    for (size_t i : order) {
        BBlock& b = blocks[i];
        if (names.count(b.name)) {
            const std::string orig = b.name;
            int& k = last_n[orig];
            do {
                k += 1;
                b.name = orig + "n" + std::to_string(k);
            } while (names.count(b.name));
        }
        names.insert(b.name);
    }
    std::set<std::string> snames;
    uint64_t next = 0;
    for (BSeq& s : seqs) {
        while (s.name.empty() || snames.count(s.name)) s.name = det_seq_name(next++);
        snames.insert(s.name);
    }
}

// SplitExtendable::process_block_impl with find_extendable / try_extend
// (SplitExtendable.cpp:46-84): the fragments of each block (std::set<Fragment*>,
// pointer order; here block order) are taken off one by one; the first is
// paired with each later one, the pair extended by FragmentsExtender::extend
// (the child's defaults: extend-length MIN_LENGTH, portion 0) and cut by
// Filter::find_good_subblocks; the first pair with good subblocks gives them
// and loses its second fragment too
static void split_extendable(const std::vector<BSeq>& seqs, const std::vector<BBlock>& blocks,
                             const PipelineOpts& o, std::vector<BBlock>& out) {
    for (const BBlock& blk : blocks) {
        std::vector<BFrag> ff(blk.f.begin(), blk.f.end());
        while (ff.size() >= 2) {
            const BFrag a = ff[0];
            ff.erase(ff.begin());
            for (size_t j = 0; j < ff.size(); j++) {
                BBlock pb;
                pb.f.push_back(a);
                pb.f.push_back(ff[j]);
                fragments_extender(seqs, pb, o.extend_length, 0, o.im, nullptr);
                std::vector<BBlock> gb;
                filter_subblocks(seqs, pb, o.filter, gb);
                if (!gb.empty()) {
                    for (auto& x : gb) out.push_back(std::move(x));
                    ff.erase(ff.begin() + (std::ptrdiff_t)j);
                    break;
                }
            }
        }
    }
}

// SetFc::find_overlaps (FragmentCollection.hpp:319-364): the common part of f
// with every fragment of the collection on f's sequence
static void find_overlaps(const OverlapIndex& idx, const BFrag& f, std::vector<std::pair<int64_t, int64_t>>& out) {
    out.clear();
    auto it = idx.m.find(f.seq);
    if (it == idx.m.end()) return;
    for (const BFrag& g : it->second) {
        const int64_t a = std::max(g.min, f.min), b = std::min(g.max, f.max);
        if (a <= b) out.emplace_back(a, b);
    }
}

// SmthUnion (TrySmth.cpp:35-155): `other`'s blocks by BlockLengthLess (size,
// alignment length, name, all descending; std::sort ties pinned to
// OverlaplessUnion's order) go to `target` when they overlap neither target
// nor the subblocks made so far; a block overlapping a subblock becomes one;
// a block overlapping only target is cut at the columns its overlaps cover
// and its remaining column runs (Block::slice) become subblocks.  `other`
// ends holding the subblocks.
static void smth_union(const std::vector<BSeq>& seqs, std::vector<BBlock>& target, std::vector<BBlock>& other) {
    OverlapIndex s2f, sub_idx;
    for (const BBlock& b : target) s2f.add(b);
    std::vector<size_t> order(other.size());
    for (size_t i = 0; i < order.size(); i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return ou_before(other[a], other[b]); });
    std::vector<BBlock> subblocks;
    std::vector<std::pair<int64_t, int64_t>> ovl;
    for (size_t i : order) {
        BBlock& b = other[i];
        if (sub_idx.block_has_overlap(b)) {
            sub_idx.add(b);
            subblocks.push_back(std::move(b));
        } else if (!s2f.block_has_overlap(b)) {
            s2f.add(b);
            target.push_back(std::move(b));
        } else {
            const int64_t L = b.aln_len();
            std::vector<char> good((size_t)L, 1);
            for (const BFrag& f : b.f) {
                if (!f.has_row) throw std::logic_error("SmthUnion: block without alignment");
                find_overlaps(s2f, f, ovl);
                if (ovl.empty()) continue;
                const RowMap rm(f.row);
                for (const auto& ol : ovl) {
                    // mark_bad (TrySmth.cpp:106-125): seq_to_frag, block_pos
                    const int64_t fa = (ol.first - f.begin()) * f.ori, fb = (ol.second - f.begin()) * f.ori;
                    const int64_t ba = rm.map_to_alignment(fa), bb = rm.map_to_alignment(fb);
                    if (ba < 0 || bb < 0) throw std::logic_error("SmthUnion: overlap outside the row");
                    for (int64_t c = std::min(ba, bb); c <= std::max(ba, bb); c++) good[(size_t)c] = 0;
                }
            }
            // add_subblocks (TrySmth.cpp:127-147)
            int64_t first = -1;
            for (int64_t c = 0; c <= L; c++) {
                const bool g = c < L && good[(size_t)c];
                if (g && first == -1) first = c;
                if (!g && first != -1) {
                    BBlock sb = block_slice(seqs, b, first, c - 1);
                    sub_idx.add(sb);
                    subblocks.push_back(std::move(sb));
                    first = -1;
                }
            }
        }
    }
    other.swap(subblocks);
}

// AddingLoopBySize (TrySmth.cpp:157-178): while other has blocks, Align them
// and SmthUnion them into target
static void adding_loop_by_size(std::vector<BSeq>& seqs, std::vector<BBlock>& target, std::vector<BBlock>& other,
                                const PipelineOpts& o) {
    for (int guard = 0; !other.empty(); guard++) {
        if (guard > 100000) throw std::logic_error("AddingLoopBySize does not converge");
        BlockSetO t{&seqs, {}};
        t.blocks.swap(other);
        align_pipe(t, o, false);
        other.swap(t.blocks);
        smth_union(seqs, target, other);
        static const bool dbg = getenv("ORACLE_AL_DEBUG") != nullptr;
        if (dbg) fprintf(stderr, "  adding loop %d: target %zu other %zu\n", guard, target.size(), other.size());
    }
}

// ExtendLoop (lua_lib.lua:677-688) under Pipe::run_impl (Pipe.cpp:60-78) with
// set_max_iterations(-1): MoveUnchanged target=unchanged other=target;
// ExtendAndAlign (FragmentsExtender --extend-length-portion:=0.5, Align);
// Move target=target other=unchanged; AddingLoopBySize target=ol
// other=target; Clear target; Move target=target other=ol; Clear ol
static void extend_loop(BlockSetO& bs, const PipelineOpts& o, PipelineStats& st) {
    std::vector<BSeq>& seqs = *bs.seqs;
    std::set<uint64_t> seen_states;
    seen_states.insert(blockset_hash(bs));
    std::vector<uint64_t> mu_hashes;
    for (int it = 0;; it++) {
        if (it > 100000) throw std::logic_error("ExtendLoop does not converge");
        st.iterations++;
        std::vector<BBlock> unchanged;
        BlockSetO work{&seqs, {}};
        std::vector<uint64_t> fresh;
        for (BBlock& b : bs.blocks) {
            const uint64_t h = block_hash(seqs, b);
            if (std::binary_search(mu_hashes.begin(), mu_hashes.end(), h)) unchanged.push_back(std::move(b));
            else {
                fresh.push_back(h);
                work.blocks.push_back(std::move(b));
            }
        }
        for (uint64_t h : fresh) mu_hashes.push_back(h);
        std::sort(mu_hashes.begin(), mu_hashes.end());
        mu_hashes.erase(std::unique(mu_hashes.begin(), mu_hashes.end()), mu_hashes.end());
        for (BBlock& b : work.blocks)
            fragments_extender(seqs, b, o.extend_length, 5000, o.im, &st.aligned_residues);
        align_pipe(work, o, false);
        for (BBlock& b : unchanged) work.blocks.push_back(std::move(b));
        std::vector<BBlock> ol;
        adding_loop_by_size(seqs, ol, work.blocks, o);
        bs.blocks.swap(ol);
        const uint64_t h = blockset_hash(bs);
        static const bool dbg = getenv("ORACLE_AL_DEBUG") != nullptr;
        if (dbg) fprintf(stderr, "extend_loop it %d: %zu blocks\n", it, bs.blocks.size());
        if (seen_states.count(h)) break;
        seen_states.insert(h);
    }
}

// consensus_order: ConSeq's block order (the std::set<Block*> pointer order,
// BlockSet.hpp:30) pinned to the blocks' sorted fragment coordinates
static void consensus_sort(std::vector<BBlock>& blocks) {
    auto key = [](const BBlock& b) {
        std::vector<std::tuple<int, int64_t, int64_t, int>> k;
        for (const BFrag& f : b.f) k.emplace_back(f.seq, f.min, f.max, f.ori);
        std::sort(k.begin(), k.end());
        return k;
    };
    std::vector<std::pair<std::vector<std::tuple<int, int64_t, int64_t, int>>, size_t>> ks(blocks.size());
    for (size_t i = 0; i < blocks.size(); i++) ks[i] = {key(blocks[i]), i};
    std::sort(ks.begin(), ks.end());
    std::vector<BBlock> out;
    out.reserve(blocks.size());
    for (auto& k : ks) out.push_back(std::move(blocks[k.second]));
    blocks.swap(out);
}

struct AnchorLoopStats {
    int64_t cons_seqs = 0, cons_anchors = 0, anchors_left = 0, split_blocks = 0, cons_blocks = 0,
            dec_blocks = 0, cons_iterations = 0, dec_iterations = 0;
};

// AnchorLoop (lua_lib.lua:711-737), a fresh pipe (its processors' memories
// empty): Filter; Rest target=target other=target; ConSeq target=cons
// other=target; AnchorFinder target=cons; MoveUnchanged target=null other=cons
// (nothing seen yet); Clear null; DummyAligner target=cons; UniqueNames
// target=cons; Union target=anchors other=cons; ExtendAndAlign target=cons;
// RemoveWithSameName target=anchors other=cons; SplitExtendable other=anchors
// target=cons; RemoveNames target=cons --remove-seqs-names:=0; DeConSeq
// target=deconseq other=cons; ExtendLoop target=cons; ExtendLoop
// target=deconseq; DeConSeq target=target other=cons; Align; Move
// target=target other=deconseq; Clear cons, anchors, deconseq.
static void anchor_loop(std::vector<BSeq>& seqs, BlockSetO& bs, const AnchorFinder& af_opts,
                        const PipelineOpts& o, PipelineStats& st, AnchorLoopStats& al) {
    static const bool dbg = getenv("ORACLE_AL_DEBUG") != nullptr;  // (diagnostic: phase sizes)
    auto note = [&](const char* what, size_t n) {
        if (dbg) fprintf(stderr, "anchor_loop %s: %zu\n", what, n);
    };
    filter_all(seqs, bs.blocks, o.filter, o.workers);
    rest(seqs, bs.blocks);
    consensus_sort(bs.blocks);
    std::vector<BSeq> cseqs(bs.blocks.size());
    std::vector<Seq> cin(bs.blocks.size());
    for (size_t i = 0; i < bs.blocks.size(); i++) {
        cseqs[i].name = bs.blocks[i].name;  // Sequence::set_block (Sequence.cpp:318-320)
        cseqs[i].data = conseq_text(seqs, bs.blocks[i]);
        cseqs[i].genome = genome_of(cseqs[i].name);
        cseqs[i].index = (int)i;
        cin[i].name = cseqs[i].name;
        cin[i].data = cseqs[i].data;
        cin[i].index = (int)i;
    }
    al.cons_seqs = (int64_t)cseqs.size();
    BlockSetO cons{&cseqs, {}};
    {
        AnchorFinder caf;
        caf.anchor = af_opts.anchor;
        caf.fp_x1e4 = af_opts.fp_x1e4;
        caf.similar = af_opts.similar;
        caf.max_anchor_fragments = af_opts.max_anchor_fragments;
        caf.seed = af_opts.seed;
        caf.explicit_params = af_opts.explicit_params;
        AnchorResult ar;
        if (caf.run(cin, ar) != 0) throw std::logic_error("AnchorFinder on the consensus sequences failed");
        for (size_t b = 0; b + 1 < ar.block_start.size(); b++) {
            BBlock blk;
            for (int64_t i = ar.block_start[b]; i < ar.block_start[b + 1]; i++) {
                BFrag f;
                f.seq = ar.frag_seq[(size_t)i];
                f.min = ar.frag_min[(size_t)i];
                f.max = ar.frag_max[(size_t)i];
                f.ori = ar.frag_ori[(size_t)i];
                blk.f.push_back(f);
            }
            cons.blocks.push_back(blk);
        }
    }
    al.cons_anchors = (int64_t)cons.blocks.size();
    for (BBlock& b : cons.blocks) align_block(cseqs, b, 1, o.im);  // DummyAligner
    unique_names(cseqs, cons.blocks);
    std::vector<BBlock> anchors = cons.blocks;  // Union (Block::clone keeps names and rows)
    for (BBlock& b : cons.blocks) fragments_extender(cseqs, b, o.extend_length, 5000, o.im, &st.aligned_residues);
    align_pipe(cons, o, false);
    {  // RemoveWithSameName target=anchors other=cons (RemoveWithSameName.cpp:28-58)
        std::set<std::string> names;
        for (const BBlock& b : cons.blocks) names.insert(b.name);
        std::vector<BBlock> keep;
        for (BBlock& b : anchors)
            if (!names.count(b.name)) keep.push_back(std::move(b));
        anchors.swap(keep);
    }
    al.anchors_left = (int64_t)anchors.size();
    note("anchors left", anchors.size());
    {
        std::vector<BBlock> gb;
        split_extendable(cseqs, anchors, o, gb);
        al.split_blocks = (int64_t)gb.size();
        for (auto& x : gb) cons.blocks.push_back(std::move(x));
    }
    for (BBlock& b : cons.blocks) b.name.clear();  // RemoveNames --remove-seqs-names:=0 (RemoveNames.cpp:26-35)
    BlockSetO dec{&seqs, {}};
    for (const BBlock& cb : cons.blocks) dec.blocks.push_back(deconseq_block(seqs, bs.blocks, cb));
    PipelineStats sc, sd;
    note("split done, cons blocks", cons.blocks.size());
    extend_loop(cons, o, sc);
    note("cons ExtendLoop done", cons.blocks.size());
    extend_loop(dec, o, sd);
    note("deconseq ExtendLoop done", dec.blocks.size());
    st.aligned_residues += sc.aligned_residues + sd.aligned_residues;
    al.cons_iterations = sc.iterations;
    al.dec_iterations = sd.iterations;
    al.cons_blocks = (int64_t)cons.blocks.size();
    al.dec_blocks = (int64_t)dec.blocks.size();
    {
        std::vector<BBlock> add;
        for (const BBlock& cb : cons.blocks) add.push_back(deconseq_block(seqs, bs.blocks, cb));
        for (auto& b : add) bs.blocks.push_back(std::move(b));
    }
    align_pipe(bs, o, false);
    for (auto& b : dec.blocks) bs.blocks.push_back(std::move(b));
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

// --- block-set processors and the DraftPangenome pipeline ----------------------
struct orc_bs {
    std::vector<orc::BSeq> seqs;
    orc::BlockSetO bs;
    orc::PipelineStats st;
    orc::AnchorFinder af;
    orc::PipelineOpts po;
    orc::AnchorLoopStats al;
};

// params (int64): [0] extend_length, [1] portion_x1e4, [2] fix_min_fragment,
// [3] fix_min_identity_x1e4, [4] max_iterations, [5] filter.min_fragment,
// [6] filter.min_block, [7] filter.frame_length, [8] filter.min_end,
// [9] filter.min_identity_x1e4, [10] filter.find_subblocks, [11] do_filter,
// [12..16] aligner (mismatch, gap, aligned, min_length, min_identity_x1e4),
// [17] anchor_size, [18] anchor_fp_x1e4, [19] max_anchor_fragments, [20] seed,
// [21] filter.max_block
orc_bs* orc_bs_create(int nseq, const char* const* seqs, const int64_t* lens,
                      const char* const* names, const int64_t* prm) {
    orc_bs* h = new orc_bs;
    h->seqs.resize((size_t)nseq);
    for (int i = 0; i < nseq; i++) {
        h->seqs[i].name = names[i];
        h->seqs[i].data = orc::to_atgcn(std::string(seqs[i], (size_t)lens[i]));
        h->seqs[i].genome = orc::genome_of(names[i]);
        h->seqs[i].index = i;
    }
    h->bs.seqs = &h->seqs;
    orc::PipelineOpts& o = h->po;
    o.extend_length = (int)prm[0];
    o.portion_x1e4 = prm[1];
    o.fix_min_fragment = (int)prm[2];
    o.fix_min_identity_x1e4 = prm[3];
    o.max_iterations = (int)prm[4];
    o.filter.min_fragment = (int)prm[5];
    o.filter.min_block = (int)prm[6];
    o.filter.frame_length = (int)prm[7];
    o.filter.min_end = (int)prm[8];
    o.filter.min_identity_x1e4 = prm[9];
    o.filter.find_subblocks = prm[10] != 0;
    o.do_filter = prm[11] != 0;
    o.im.mismatch_check = (int)prm[12];
    o.im.gap_check = (int)prm[13];
    o.im.aligned_check = (int)prm[14];
    o.im.min_length = (int)prm[15];
    o.im.min_identity_x1e4 = prm[16];
    h->af.anchor = (int)prm[17];
    h->af.fp_x1e4 = prm[18];
    h->af.max_anchor_fragments = prm[19];
    h->af.seed = (uint32_t)prm[20];
    o.filter.max_block = (int)prm[21];
    return h;
}
void orc_bs_free(orc_bs* h) { delete h; }

// replace the block set: fragments in block order; rows optional (row_len[i] < 0: none)
void orc_bs_set_blocks(orc_bs* h, int64_t nb, const int64_t* block_start, const int32_t* seq,
                       const int64_t* mn, const int64_t* mx, const int32_t* ori,
                       const int64_t* row_off, const int64_t* row_len, const char* rows) {
    h->bs.blocks.clear();
    for (int64_t b = 0; b < nb; b++) {
        orc::BBlock blk;
        for (int64_t i = block_start[b]; i < block_start[b + 1]; i++) {
            orc::BFrag f;
            f.seq = seq[i];
            f.min = mn[i];
            f.max = mx[i];
            f.ori = ori[i];
            if (row_len && row_len[i] >= 0) {
                f.row.assign(rows + row_off[i], (size_t)row_len[i]);
                f.has_row = true;
            }
            blk.f.push_back(f);
        }
        h->bs.blocks.push_back(blk);
    }
}

// Worker count for DraftPangenome: BlocksJobs for the per-block stages, FragmentTG
// (one sequence per task) for AnchorFinder's pass 2; the Bloom pass stays
// sequential (racy in the reference when threaded); results identical for every count
void orc_bs_set_workers(orc_bs* h, int workers) { h->af.workers = h->po.workers = workers < 1 ? 1 : workers; }

// op: 0 FragmentsExtender, 1 FixEnds, 2 Filter, 3 ExtendLoopFast, 4 DummyAligner,
// 5 RemoveNonStem --exact, 6 DraftPangenome (AnchorFinder on all sequences first),
// 7 MetaAligner(similar) align_block, 8 Filter::find_good_subblocks, 9 Rest,
// 10 OverlaplessUnion --ou-move, 11 MoveGaps, 12 CutGaps, 13 CutGaps --cut-strict,
// 14 SelfOverlapsResolver, 15 Align, 16 LiteAlign, 17 AnchorLoop (a fresh pipe;
// its consensus AnchorFinder takes this set's AnchorFinder options),
// 18 ExtendLoop, 19 AddingLoopBySize into an empty target
static int bs_apply(orc_bs* h, int op);
// op codes: see bs_apply; exceptions (the reference's ASSERTs) -> -2
int orc_bs_apply(orc_bs* h, int op) {
    try {
        return bs_apply(h, op);
    } catch (const std::exception&) {
        return -2;
    }
}

static int bs_apply(orc_bs* h, int op) {
    const std::vector<orc::BSeq>& seqs = h->seqs;
    orc::PipelineOpts& o = h->po;
    std::vector<orc::BBlock> out;
    switch (op) {
        case 0:
            for (auto& b : h->bs.blocks)
                orc::fragments_extender(seqs, b, o.extend_length, o.portion_x1e4, o.im,
                                        &h->st.aligned_residues);
            return 0;
        case 1:
            for (auto& b : h->bs.blocks) {
                orc::BBlock x;
                int r = orc::fix_ends(seqs, b, o.fix_min_fragment, o.fix_min_identity_x1e4, x);
                if (r == 0) out.push_back(b);
                else if (r == 1) out.push_back(x);
            }
            h->bs.blocks.swap(out);
            return 0;
        case 2:
            for (auto& b : h->bs.blocks) {
                std::vector<orc::BBlock> sub;
                int r = orc::filter_block(seqs, b, o.filter, sub);
                if (r == 0) out.push_back(b);
                else if (r == 1)
                    for (auto& x : sub) out.push_back(x);
            }
            h->bs.blocks.swap(out);
            return 0;
        case 3:
            orc::extend_loop_fast(h->bs, o, h->st);
            return 0;
        case 4:
            for (auto& b : h->bs.blocks) orc::align_block(seqs, b, 1, o.im);
            return 0;
        case 5:
            orc::remove_non_stem(h->bs, true);
            return 0;
        case 6:
            orc::draft_pangenome(h->seqs, h->af, o, h->bs, h->st);
            return 0;
        case 7:
            for (auto& b : h->bs.blocks) orc::align_block(seqs, b, 0, o.im);
            return 0;
        case 9:
            orc::rest(seqs, h->bs.blocks);
            return 0;
        case 10:
            orc::overlapless_union(h->bs.blocks);
            return 0;
        case 8:  // Filter::find_good_subblocks only
            for (auto& b : h->bs.blocks) orc::filter_subblocks(seqs, b, o.filter, out);
            h->bs.blocks.swap(out);
            return 0;
        case 11:
            for (auto& b : h->bs.blocks) orc::move_gaps(b, o.max_tail, o.max_tail_to_gap_x1e4);
            return 0;
        case 12:
        case 13:
            for (auto& b : h->bs.blocks) orc::cut_gaps(b, op == 13);
            return 0;
        case 14:
            for (auto& b : h->bs.blocks) orc::fix_self_overlaps(b);
            return 0;
        case 15:
        case 16:
            orc::align_pipe(h->bs, o, op == 16);
            return 0;
        case 17:
            h->al = orc::AnchorLoopStats{};
            orc::anchor_loop(h->seqs, h->bs, h->af, o, h->st, h->al);
            return 0;
        case 18:
            orc::extend_loop(h->bs, o, h->st);
            return 0;
        case 19: {
            std::vector<orc::BBlock> target;
            orc::adding_loop_by_size(h->seqs, target, h->bs.blocks, o);
            h->bs.blocks.swap(target);
            return 0;
        }
    }
    return -1;
}

// MoveGaps options: max-tail, max-tail-to-gap (x 1e4)
void orc_bs_set_gap_opts(orc_bs* h, int max_tail, int64_t max_tail_to_gap_x1e4) {
    h->po.max_tail = max_tail;
    h->po.max_tail_to_gap_x1e4 = max_tail_to_gap_x1e4;
}

// [n_blocks, n_fragments, row_bytes, iterations, aligned_residues, anchor_blocks, stem_blocks]
void orc_bs_counts(const orc_bs* h, int64_t* c) {
    int64_t nf = 0, rb = 0;
    for (const auto& b : h->bs.blocks) {
        nf += (int64_t)b.f.size();
        for (const auto& f : b.f) rb += (int64_t)f.row.size();
    }
    c[0] = (int64_t)h->bs.blocks.size();
    c[1] = nf;
    c[2] = rb;
    c[3] = h->st.iterations;
    c[4] = h->st.aligned_residues;
    c[5] = h->st.anchor_blocks;
    c[6] = h->st.stem_blocks;
}

void orc_bs_copy(const orc_bs* h, int64_t* block_start, int32_t* seq, int64_t* mn, int64_t* mx,
                 int32_t* ori, int64_t* row_off, int64_t* row_len, char* rows) {
    int64_t k = 0, ro = 0;
    size_t b = 0;
    for (; b < h->bs.blocks.size(); b++) {
        block_start[b] = k;
        for (const auto& f : h->bs.blocks[b].f) {
            seq[k] = f.seq;
            mn[k] = f.min;
            mx[k] = f.max;
            ori[k] = f.ori;
            row_off[k] = ro;
            row_len[k] = f.has_row ? (int64_t)f.row.size() : -1;
            memcpy(rows + ro, f.row.data(), f.row.size());
            ro += (int64_t)f.row.size();
            k++;
        }
    }
    block_start[b] = k;
}

uint64_t orc_bs_hash(const orc_bs* h) { return orc::blockset_hash(h->bs); }

// the last AnchorLoop's counts: [consensus sequences, consensus anchor blocks,
// anchors left for SplitExtendable, its blocks, consensus blocks after
// ExtendLoop, deconseq blocks after ExtendLoop, the two ExtendLoop iterations]
void orc_bs_anchor_loop_stats(const orc_bs* h, int64_t* c) {
    const orc::AnchorLoopStats& a = h->al;
    const int64_t v[8] = {a.cons_seqs, a.cons_anchors, a.anchors_left, a.split_blocks,
                          a.cons_blocks, a.dec_blocks, a.cons_iterations, a.dec_iterations};
    memcpy(c, v, sizeof(v));
}

// goodSlices (goodSlices.cpp:247-255) over n column scores: the slices'
// (start, stop) pairs into out (at most max_out); returns their count
int orc_good_slices(const int32_t* scores, int n, int frame_length, int end_length, int min_identity, int min_length,
                    int64_t* out, int max_out) {
    const std::vector<int> sc(scores, scores + n);
    const std::vector<orc::SS> r = orc::GoodSlicer(sc, frame_length, end_length, min_identity, min_length).calculate();
    for (size_t i = 0; i < r.size() && (int)i < max_out; i++) {
        out[2 * i] = r[i].first;
        out[2 * i + 1] = r[i].second;
    }
    return (int)r.size();
}

// goodColumns (goodColumns.cpp:177-209) of nrows rows of `length` chars each
int orc_good_columns(int nrows, const char* rows, int length, int min_identity, int min_length, int32_t* out) {
    Strings r((size_t)nrows);
    for (int i = 0; i < nrows; i++) r[(size_t)i].assign(rows + (size_t)i * (size_t)length, (size_t)length);
    const std::vector<int> s = orc::goodColumns(r, length, min_identity, min_length);
    for (int i = 0; i < length; i++) out[i] = s[(size_t)i];
    return 0;
}

// ConSeq: the text of the sequence each block becomes (in block order), two
// calls: total size (out == NULL), then the bytes and n_blocks + 1 offsets
int64_t orc_bs_conseq(const orc_bs* h, char* out, int64_t* off) {
    int64_t t = 0;
    for (size_t b = 0; b < h->bs.blocks.size(); b++) {
        const std::string s = orc::conseq_text(h->seqs, h->bs.blocks[b]);
        if (off) off[b] = t;
        if (out) memcpy(out + t, s.data(), s.size());
        t += (int64_t)s.size();
    }
    if (off) off[h->bs.blocks.size()] = t;
    return t;
}

// DeConSeq: the blocks of `cons` (over the sequences orc_bs_conseq made from
// `source`'s blocks) mapped onto source's sequences, appended to target's
// blocks (target and source share their sequences); -1 on a mismatch
int orc_bs_deconseq(orc_bs* target, const orc_bs* source, const orc_bs* cons) {
    if (cons->seqs.size() != source->bs.blocks.size()) return -1;
    std::vector<orc::BBlock> out;
    for (const auto& cb : cons->bs.blocks) {
        for (const auto& cf : cb.f)
            if (cf.seq < 0 || (size_t)cf.seq >= source->bs.blocks.size()) return -1;
        try {
            orc::BBlock nb = orc::deconseq_block(source->seqs, source->bs.blocks, cb);
            out.push_back(nb);  // empty ones too (DeConSeq.cpp:94-99 inserts every new block)
        } catch (const std::exception&) {
            return -2;
        }
    }
    for (auto& b : out) target->bs.blocks.push_back(b);
    return 0;
}

}  // extern "C"
