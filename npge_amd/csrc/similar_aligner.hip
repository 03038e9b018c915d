// similar_aligner.hip -- batched AbstractAligner::align_seqs with aligner-type
// "similar" (SimilarAligner::similar_aligner, src/algo/SimilarAligner.cpp:487-501)
// or "dummy" (DummyAligner.cpp:18-26) on MI355X.
//
// Blocks are independent ("Blocks should not interfere", BlocksJobs.hpp:49-53),
// so a batch of alignment problems (one per block) is the batch axis: a
// persistent grid of single-wave workgroups pulls jobs from an atomic counter
// (heaviest first).  Inside a job, lanes are rows.  Phases per job:
//   1. process_seqs on the input rows           -> A   (sa_device.hpp)
//   2. fix_bad_regions (:428-459) A -> B: column-parallel good-column scan,
//      FindLowSimilar::make_regions/reduce_regions (FindLowSimilar.cpp:62-130),
//      re-alignment of every bad region (gap-filtered, reversed) kept only if
//      its identical-column score grows
//   3. realing_end (:461-484) on B
//   4. AbstractAligner::remove_gaps (AbstractAligner.cpp:89-102)
// Empty rows are removed before and re-added as all-gap rows after
// (AbstractAligner.cpp:104-143).  Output columns are bounded by the sum of the
// row lengths (every column holds a letter); a job first gets a tighter
// capacity and is re-run at the full bound if it overflows.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>

#include "common.hpp"
#include "sa_device.hpp"

// waves of k_align_jobs / k_align_sub per SIMD, chosen per launch: 2 gives
// each wave 256 registers and no scratch spills (4: 128 registers, 648 bytes
// of scratch a lane with the prefix search's call) -- C3 / C2 align -3 to -5
// %, R3 and the pair job level (profiles/r06c_ab_waves_per_eu.txt); a launch
// with more tasks than 2 waves a SIMD hold (SA_WAVES_MANY_AT) takes the
// 4-wave form: C5's first launches (tens of thousands of 8-row jobs) ran
// 30 ms a step slower with 2 (profiles/r06t_c5_waves_twins_anchor_ab.txt)
#ifndef SA_WAVES_PER_EU
#define SA_WAVES_PER_EU 2
#endif
#ifndef SA_WAVES_MANY
#define SA_WAVES_MANY 4
#endif
static constexpr int SA_WAVES_MANY_AT = 256 * 4 * SA_WAVES_PER_EU;

namespace npgx {

using namespace sa;

static const int64_t LDS_PER_CU = 160 * 1024;  // gfx950: a workgroup may use all of it

struct SaJob {
    int64_t row0;       // first non-empty row (index into row_off / row_len)
    int64_t scratch;    // byte offset of this job's A|B|C scratch
    int32_t n;          // non-empty rows (<= 64)
    int32_t cap;        // column capacity of A, B and C rows
    int64_t reg_off;    // first entry of the job's region list (deferred fix_bad_regions)
    int32_t reg_cap;    // entries available there
    int32_t pad;
};

// One bad region of a deferred job, re-aligned as a job of its own
// (fix_bad_regions :428-459): rows = the region's gap-filtered reversed
// segments, written by the parent into its C at column x.
struct SaSub {
    int32_t job, x;
    int32_t out_cap, pad;
    int64_t out_off;    // byte offset in the sub-job output pool (n rows x out_cap)
};

// Long jobs are split into segments at sync states (see "Long jobs" at
// k_split_find): segment k runs process_seqs from state k to the first later
// state its walk passes through exactly.
struct SaSplit {
    int32_t job;
    int32_t K;          // segments (K - 1 sync states)
    int64_t tgt;        // first int of its sync states (K - 1 states x n rows)
    int32_t seg0;       // its first segment task
    int32_t win;        // half-width of the sync word search window
    int32_t sub;        // -1: the job's own rows; -2: a twin (the job's rows reversed, see
                        // "Twins"); else the job's sub-job (a bad region) of this index
    int32_t twin;       // job splits: 1 + index of the job's twin split, 0: none
    int64_t post;       // >= 0: byte offset of k_split_post's global work area (chains too long for LDS)
};

// split-state counters (device): the job splits are planned on the host, the
// sub-job splits by k_plan_subs
enum { SC_SPLITS, SC_SEGS, SC_TGT, SC_FIND, SC_QSEG, SC_QSUB, SC_POOL_LO, SC_POOL_HI, SC_N };

struct SaSeg {
    int32_t split;      // index into splits
    int32_t k;          // segment index
    int32_t cap;        // output columns
    int32_t pad;
    int64_t out;        // byte offset of its n x cap output rows in seg_pool
};

struct SaArgs {
    const char* rows;
    const int64_t* row_off;
    const int32_t* row_len;
    const SaJob* jobs;
    const int32_t* order;      // job processing order (heaviest first)
    int32_t n_jobs;
    const int32_t* n_jobs_dev; // non-null: the job count is on the device (the re-run of align_device's async mode)
    int32_t aligner_type;      // 0 similar, 1 dummy
    unsigned char* scratch;
    int32_t* job_len;
    int32_t* job_status;       // 0 ok (rows in B), 2 ok (rows in A), 1 capacity overflow
    int64_t* job_stats;        // per job: cycles, columns, aligned calls, shifts, gaps, regions, rows
    unsigned int* next_job;
    // per-slot scratch
    unsigned long long* tkeys;
    unsigned long long* tmask;
    uint32_t* tdone;           // row-parallel search: completion shift of a word
    uint32_t tcap_log2;
    uint32_t* slot_epoch;      // out: highest word-table epoch reached (one word)
    uint32_t epoch_base;       // every slot's first epoch
    const char** st_p;
    int* st_len;
    int* st_pos;
    int* st_col;
    int32_t st_depth_max;
    int4* regions;
    unsigned char* good_col;
    int32_t slot_cols;         // regions / good_col entries per slot
    int32_t stage_bytes;       // LDS bytes for a job's rows (after the word table)
    int32_t hist_cap;          // > 0: LDS word history of the row-parallel search
    int32_t words_bytes;       // LDS bytes of the chunk words / code history
    uint32_t ltab_log2;        // LDS word-table entries (log2)
    Params P;
    // deferred fix_bad_regions (attempt 0): regions and sub-jobs
    int32_t defer;             // > 0: defer the bad regions of alignments of at least this many columns
    int32_t defer_rows;        // ... and at least this many rows
    int4* job_regions;         // per job: x, y, good (1) or -(sub+1), identical columns before
    int32_t* job_nreg;         // regions per deferred job
    SaSub* subs;
    int2* sub_res;             // per sub-job: columns (-1: overflow), identical columns after
    unsigned long long* alloc; // [0] pool bytes taken, [1] sub-jobs issued
    unsigned int* counters;    // [0] next sub-job, [1] deferred jobs, [2] next deferred job,
                               // [3] sub-jobs re-run in place, [4] next retried sub-job, [5] retried sub-jobs
    unsigned char* pool;       // per sub-job: 64 row lengths (int32), then n rows x out_cap
    int64_t pool_cap;
    int64_t max_sub;
    int32_t* fin;              // the deferred jobs
    // split long jobs (order[] entries < 0 are segment tasks -(t+1))
    const SaSplit* splits;
    const SaSeg* segs;
    int32_t* targets;          // sync states (k_split_find)
    int4* seg_res;             // per segment: next segment (K: ran to the end, -1: idle), columns, overflow
    int64_t* seg_wall;         // per segment: wall clock at start and end (job statistics)
    int64_t* sub_wall;         // per whole sub-job: wall clock at start and end (job statistics)
    unsigned char* seg_pool;
    // sub-job splits (k_plan_subs): capacities of the arrays above and the
    // sub-job queue (segment tasks first, then whole sub-jobs)
    unsigned int* sctr;
    int32_t* qseg;
    int32_t* qsub;
    const int32_t* rq;         // k_align_sub's retry launch: the failed sub-jobs (count in counters[5])
    int2* ftasks;
    unsigned char* post_area;  // k_split_post's global work areas (SaSplit.post)
    int4* chain;               // per job split, from its seg0: the chain (segment, columns, first column)
    int4* chain_hdr;           // per job split: chain length, columns, failed
    unsigned long long* chain_bits;  // per job split without a post area: identical-column bits
    const int64_t* bits_off;   // ... their first word
    const int32_t* part0;      // per job split: its first k_chain_copy workgroup (n_splits + 1 entries)
    int32_t split_len;         // segment length for a job of 16 rows (0: no splitting)
    // twins (split jobs' reversed rows, walked beside the jobs): the reversed
    // copies, at twin_off[row] for the rows of jobs with a twin
    const char* twin_rows;
    const int64_t* twin_off;
    // unsplit twins (order[] entries >= UTWIN_BASE, see "Unsplit twins" at
    // align_device): per job the twin's output offset in utw_pool (-1: none),
    // its state (0 running, 1 done, 2 overflowed) and its columns
    const int64_t* utw_off;
    int32_t* utw_state;
    int32_t* utw_len;
    unsigned char* utw_pool;
    int32_t cap_splits, cap_segs;
    int64_t cap_tgt, cap_find, cap_pool;
};

// number of columns c in [c0, c1) identical over all rows (score_of :416-426)
__device__ int count_equal_cols(const WaveCtx& w, const char* buf, int cap, int c0, int c1,
                                unsigned char* flags) {
    int cnt = 0;
    for (int b = c0; b < c1; b += 256) {  // four 64-column chunks per step: four loads in flight
        char x[4];
        bool eq[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int c = b + u * 64 + w.lane;
            eq[u] = c < c1;
            x[u] = eq[u] ? buf[c] : 0;
        }
        for (int r = 1; r < w.n; r++) {
            char y[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int c = b + u * 64 + w.lane;
                y[u] = c < c1 ? buf[(size_t)r * cap + c] : 0;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) eq[u] &= y[u] == x[u];
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int c = b + u * 64 + w.lane;
            if (c < c1) {
                cnt += eq[u];
                if (flags) flags[c] = eq[u];
            }
        }
    }
    return wave_sum(cnt);
}

// gap-filtered, reversed copy of every row's segment [s0, s1) into C (row r
// at C + r*cstride; columns mode, ballot compaction); returns this lane's row
// as a view
__device__ View filter_reverse(const WaveCtx& w, const char* src, int cap, char* C, int cstride, int s0, int s1) {
    int my_len = 0;
    for (int r = 0; r < w.n; r++) {
        const char* a = src + (size_t)r * cap;
        char* c = C + (size_t)r * cstride;
        int k = 0;
        for (int base = s1 - 1; base >= s0; base -= 64) {
            const int idx = base - w.lane;
            const bool in = idx >= s0;
            const char x = in ? a[idx] : '-';
            const bool keep = in && x != '-';
            const unsigned long long m = ballot(keep);
            if (keep) c[k + __popcll(m & ((1ull << w.lane) - 1ull))] = x;
            k += __popcll(m);
        }
        if (w.lane == r) my_len = k;
    }
    __syncthreads();
    View v{C + (size_t)w.lane * cstride, w.act ? my_len : 0, 1};
    return v;
}

// segment [s0, s1) of every row, gap-filtered and reversed, into LDS when it fits
__device__ View stage_segment(const WaveCtx& w, const char* src, int cap, char* C, char* stage, int stage_bytes,
                              int s0, int s1) {
    const int len = s1 - s0;
    if ((int64_t)w.n * len <= stage_bytes) return filter_reverse(w, src, cap, stage, len, s0, s1);
    return filter_reverse(w, src, cap, C, cap, s0, s1);
}

// FindLowSimilar::make_regions (:62-80) from good_col[0..L)
__device__ int make_regions(const WaveCtx& w, const unsigned char* good, int L, int wf, int4* reg) {
    int R = 0;
    for (int base = 0; base < L; base += 64) {
        const int j = base + w.lane;
        const bool in = j < L;
        const int g = in ? good[j] : 0;
        const int gp = (in && j > 0) ? good[j - 1] : -1;
        const bool b = in && (j == 0 || g != gp);
        const unsigned long long bm = ballot(b);
        const int idx = R + __popcll(bm & ((1ull << w.lane) - 1ull));
        if (b) reg[idx] = make_int4(j, 0, g, 0);
        R += __popcll(bm);
    }
    __syncthreads();
    for (int i = w.lane; i < R; i += 64) {
        int4 r = reg[i];
        const int stop = (i + 1 < R) ? reg[i + 1].x - 1 : L - 1;
        const int len = stop - r.x + 1;
        r.y = stop;
        r.w = r.z ? len : len * wf;  // Region::set_weight :48-54
        reg[i] = r;
    }
    __syncthreads();
    return R;
}

// FindLowSimilar::reduce_regions (:121-130) with find_min_region (:82-92) and
// merge_region (:94-119)
__device__ int reduce_regions(const WaveCtx& w, int4* reg, int R, int min_length) {
    while (R >= 2) {
        int bw = 0x7fffffff, bi = 0x7fffffff;
        for (int i = w.lane; i < R; i += 64) {
            const int wt = reg[i].w;
            if (wt < bw) {
                bw = wt;
                bi = i;
            }
        }
        // first index of the minimum weight
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const int ow = __shfl_xor(bw, o), oi = __shfl_xor(bi, o);
            if (ow < bw || (ow == bw && oi < bi)) {
                bw = ow;
                bi = oi;
            }
        }
        if (bw >= min_length) break;
        const int mi = bi;
        int4 nr = reg[mi];
        const int good = nr.z;
        int first = mi, last = mi;
        if (mi > 0) {
            const int4 p = reg[mi - 1];
            nr.x = p.x;
            nr.w += p.w;
            first = mi - 1;
        }
        if (mi < R - 1) {
            const int4 q = reg[mi + 1];
            nr.y = q.y;
            nr.w += q.w;
            last = mi + 1;
        }
        nr.z = good == 0 ? 1 : 0;
        __syncthreads();
        if (w.lane == 0) reg[first] = nr;
        const int shiftn = last - first;
        if (shiftn > 0) {
            for (int base = last + 1; base < R; base += 64) {
                const int i = base + w.lane;
                int4 x;
                if (i < R) x = reg[i];
                __syncthreads();
                if (i < R) reg[i - shiftn] = x;
                __syncthreads();
            }
        }
        R -= shiftn;
        __syncthreads();
    }
    return R;
}

// make_regions + reduce_regions with the regions in registers (lane i holds
// region i) for alignments of at most 4096 columns and 64 initial regions;
// good-column masks in registers too (lane c holds columns [64c, 64c+64)).
// Returns the region count, or -1 when the alignment is outside that range.
__device__ int regions_in_registers(const WaveCtx& w, const char* A, int cap, int L, int wf, int min_length,
                                    int4& rg, unsigned long long& gm, int* tmp) {
    if (L > 64 * 64) return -1;
    const int lane = w.lane;
    const int nch = (L + 63) >> 6;
    gm = 0;
    for (int ch = 0; ch < nch; ch++) {  // count_equal_cols flags (:416-426)
        const int c = ch * 64 + lane;
        bool eq = false;
        if (c < L) {
            const char x = A[c];
            eq = true;
            for (int r = 1; r < w.n; r++) eq &= A[(size_t)r * cap + c] == x;
        }
        const unsigned long long m = ballot(eq);
        if (lane == ch) gm = m;
    }
    const unsigned long long prev = __shfl((long long)gm, lane > 0 ? lane - 1 : 0);
    const unsigned long long valid =
        lane < nch - 1 ? ~0ull : lane == nch - 1 ? ((L & 63) ? ((1ull << (L & 63)) - 1) : ~0ull) : 0ull;
    unsigned long long starts = (gm ^ ((gm << 1) | (lane > 0 ? prev >> 63 : (gm & 1ull)))) & valid;
    if (lane == 0 && L > 0) starts |= 1ull;  // a region starts at column 0
    const int cnt = __popcll(starts);
    int pre = cnt;  // inclusive scan over lanes
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(pre, o);
        if (lane >= o) pre += t;
    }
    const int R = bcast(pre, 63);
    if (R > 64) return -1;
    int idx = pre - cnt;
    for (unsigned long long m = starts; m; m &= m - 1) tmp[idx++] = lane * 64 + __ffsll((long long)m) - 1;
    __syncthreads();
    const int st = lane < R ? tmp[lane] : 0;
    const int nx = lane + 1 < R ? tmp[lane + 1] : L;
    __syncthreads();
    const int good = (int)((((unsigned long long)__shfl((long long)gm, st >> 6)) >> (st & 63)) & 1ull);
    rg = make_int4(st, nx - 1, good, good ? nx - st : (nx - st) * wf);  // Region::set_weight :48-54
    int n = R;
    while (n >= 2) {  // reduce_regions (:121-130)
        const int wv = lane < n ? rg.w : 0x7fffffff;
        const int bw = wave_min(wv);
        if (bw >= min_length) break;
        const int mi = __ffsll((long long)ballot(lane < n && rg.w == bw)) - 1;  // first minimum
        int4 nr = make_int4(bcast(rg.x, mi), bcast(rg.y, mi), bcast(rg.z, mi), bcast(rg.w, mi));
        const int px = bcast(rg.x, mi > 0 ? mi - 1 : 0), pw = bcast(rg.w, mi > 0 ? mi - 1 : 0);
        const int qy = bcast(rg.y, mi + 1 < 64 ? mi + 1 : 63), qw = bcast(rg.w, mi + 1 < 64 ? mi + 1 : 63);
        int first = mi, last = mi;
        if (mi > 0) {
            nr.x = px;
            nr.w += pw;
            first = mi - 1;
        }
        if (mi < n - 1) {
            nr.y = qy;
            nr.w += qw;
            last = mi + 1;
        }
        nr.z = nr.z == 0 ? 1 : 0;
        const int shiftn = last - first;
        const int src = lane + shiftn < 64 ? lane + shiftn : 63;
        const int4 moved = make_int4(__shfl(rg.x, src), __shfl(rg.y, src), __shfl(rg.z, src), __shfl(rg.w, src));
        if (lane == first) rg = nr;
        else if (lane > first) rg = moved;
        n -= shiftn;
    }
    return n;
}

typedef __attribute__((address_space(3))) int LdsInt;

// count_equal_cols flags (:416-426) + make_regions (:62-80) + reduce_regions
// (:121-130) for long alignments, in LDS (the job's row stage, free after
// process_seqs): identical-column flags as one bit per column, regions as
// arrays with prev/next links; a merge rewrites the surviving region and
// unlinks the others (no shifting); the minimum is a wave-parallel scan (alive
// entries keep their order, so the lowest index is the reference's first
// minimum).  The survivors go to `out` in order with .w = the number of
// identical columns in the region (score_of before re-alignment); returns
// their count, or -1 when the LDS area is too small.
typedef __attribute__((address_space(3))) unsigned long long LdsU64w;

template <bool WG>
__device__ __forceinline__ void wave_or_wg_sync() {
    if (WG) {
        __syncthreads();
    } else {  // one wave's LDS accesses in program order across its lanes
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
}

// make_regions + reduce_regions from the identical-column bits gm[0, nw) in
// LDS, the arrays after them (area_bytes in all, gm included); WG: the
// workgroup is this one wave (barriers), else a wave of a larger workgroup
// working alone (wave-level ordering of its LDS accesses)
template <bool WG>
__device__ int regions_from_bits(const WaveCtx& w, LdsU64w* gm, int nw, int L, int wf, int min_length,
                                 int area_bytes, int4* out) {
    const int lane = w.lane;
    LdsU64w* sm = gm + nw;  // region-start bits
    int R0 = 0;
    for (int q = lane; q < nw; q += 64) {
        const unsigned long long g = gm[q];
        const unsigned long long valid = (q < nw - 1 || (L & 63) == 0) ? ~0ull : ((1ull << (L & 63)) - 1);
        unsigned long long st = (g ^ ((g << 1) | (q > 0 ? (gm[q - 1] >> 63) : (g & 1ull)))) & valid;
        if (q == 0) st |= 1ull;
        sm[q] = st;
        R0 += __popcll(st);
    }
    R0 = wave_sum(R0);
    wave_or_wg_sync<WG>();
    // per region 12 bytes: start (-1: merged away), weight | good << 31, and
    // next | prev << 16 (0xFFFF: none); a region ends where the next alive starts
    const long long need = (long long)nw * 16 + (long long)R0 * 12;
    if (need > area_bytes || R0 >= 0xFFFF) return -1;
    LdsInt* rx = (LdsInt*)(sm + nw);
    LdsInt* rw = rx + R0;
    LdsInt* lk = rx + 2 * R0;
    int k = 0;
    for (int q0 = 0; q0 < nw; q0 += 64) {  // region starts in order: word prefix counts
        const int q = q0 + lane;
        unsigned long long st = q < nw ? sm[q] : 0ull;
        const int c = __popcll(st);
        int pre = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(pre, o);
            if (lane >= o) pre += t;
        }
        int i = k + pre - c;
        for (; st; st &= st - 1) {
            const int j = q * 64 + __ffsll((long long)st) - 1;
            rx[i] = j;
            rw[i] = (int)((gm[q] >> (j & 63)) & 1ull) << 31;  // good flag; weight below
            i++;
        }
        k += bcast(pre, 63);
    }
    wave_or_wg_sync<WG>();
    for (int i = lane; i < R0; i += 64) {
        const int len = (i + 1 < R0 ? rx[i + 1] : L) - rx[i];
        const int good = (int)((unsigned)rw[i] >> 31);
        rw[i] = (good << 31) | (good ? len : len * wf);  // Region::set_weight :48-54
        lk[i] = (i + 1 < R0 ? i + 1 : 0xFFFF) | ((i > 0 ? i - 1 : 0xFFFF) << 16);
    }
    wave_or_wg_sync<WG>();
    const int WM = 0x7fffffff;
    int R = R0;
    // one merge of the minimum region mi with its alive neighbours (merge_region :94-119)
    auto merge = [&](int mi, int& hp_out, int& hq_out, int& p_out, int& q_out) {
        const int l = lk[mi];
        const int p = (l >> 16) & 0xFFFF, q = l & 0xFFFF;
        const bool hp = p != 0xFFFF, hq = q != 0xFFFF;
        const int keep = hp ? p : mi;
        const int nwt = (rw[mi] & WM) + (hp ? rw[p] & WM : 0) + (hq ? rw[q] & WM : 0);
        const int z = ((unsigned)rw[mi] >> 31) ? 0 : 1;
        const int after = hq ? lk[q] & 0xFFFF : q;
        const int keep_prev = (lk[keep] >> 16) & 0xFFFF;
        wave_or_wg_sync<WG>();
        if (lane == 0) {
            if (hp) rx[mi] = -1;
            if (hq) rx[q] = -1;
            rw[keep] = (z << 31) | nwt;
            lk[keep] = after | (keep_prev << 16);
            if (after != 0xFFFF) lk[after] = (lk[after] & 0xFFFF) | (keep << 16);
        }
        wave_or_wg_sync<WG>();
        hp_out = hp;
        hq_out = hq;
        p_out = p;
        q_out = q;
    };
    const int nb = (R0 + 63) >> 6;
    if (nb <= 256) {
        // minimum of every 64-entry block in registers (lane l: blocks l + 64k):
        // a step reads the block minima, merges, and rescans only the blocks
        // whose entries changed
        int bm[4], bi[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            bm[k] = WM;
            bi[k] = WM;
        }
        auto rescan = [&](int b) {
            const int i = b * 64 + lane;
            const bool alive = i < R0 && rx[i] >= 0;
            const int wt = alive ? rw[i] & WM : WM;
            const int mw = wave_min(wt);
            const unsigned long long m = ballot(alive && wt == mw);
            const int first = m ? b * 64 + __ffsll((long long)m) - 1 : WM;
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (lane == (b & 63) && k == (b >> 6)) {
                    bm[k] = m ? mw : WM;
                    bi[k] = first;
                }
        };
        for (int b = 0; b < nb; b++) rescan(b);
        while (R >= 2) {
            const int bw = wave_min(min(min(bm[0], bm[1]), min(bm[2], bm[3])));
            if (bw >= min_length) break;
            // first minimum: lowest block, i.e. lowest k, then lowest lane
            int mi = WM;
#pragma unroll
            for (int k = 3; k >= 0; k--) {
                const unsigned long long m = ballot(bm[k] == bw);
                if (m) mi = bcast(bi[k], __ffsll((long long)m) - 1);
            }
            int hp, hq, p, q;
            merge(mi, hp, hq, p, q);
            R -= hp + hq;
            const int b0 = mi >> 6, b1 = hp ? p >> 6 : b0, b2 = hq ? q >> 6 : b0;
            rescan(b0);
            if (b1 != b0) rescan(b1);
            if (b2 != b0 && b2 != b1) rescan(b2);
        }
    } else {
        while (R >= 2) {
            int bw = WM, bi = WM;
            for (int i = lane; i < R0; i += 64) {
                const int wt = rw[i] & WM;
                if (rx[i] >= 0 && wt < bw) {
                    bw = wt;
                    bi = i;
                }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const int ow = __shfl_xor(bw, o), oi = __shfl_xor(bi, o);
                if (ow < bw || (ow == bw && oi < bi)) {
                    bw = ow;
                    bi = oi;
                }
            }
            if (bw >= min_length) break;
            int hp, hq, p, q;
            merge(bi, hp, hq, p, q);
            R -= hp + hq;
        }
    }
    // survivors in order, with their identical-column counts
    k = 0;
    for (int base = 0; base < R0; base += 64) {
        const int i = base + lane;
        const bool alive = i < R0 && rx[i] >= 0;
        int4 rg = make_int4(0, 0, 0, 0);
        if (alive) {
            const int nxt = lk[i] & 0xFFFF;
            rg = make_int4(rx[i], (nxt != 0xFFFF ? rx[nxt] : L) - 1, (int)((unsigned)rw[i] >> 31), 0);
            int cnt = 0;
            for (int q = rg.x >> 6; q <= (rg.y >> 6); q++) {
                const int lo = q == (rg.x >> 6) ? (rg.x & 63) : 0, hi = q == (rg.y >> 6) ? (rg.y & 63) : 63;
                cnt += __popcll(gm[q] & ((hi == 63 ? ~0ull : ((1ull << (hi + 1)) - 1)) & (~0ull << lo)));
            }
            rg.w = cnt;
        }
        const unsigned long long m = ballot(alive);
        if (alive) out[k + __popcll(m & ((1ull << lane) - 1ull))] = rg;
        k += __popcll(m);
    }
    wave_or_wg_sync<WG>();
    return R;
}


__device__ int regions_in_lds(const WaveCtx& w, const char* A, int cap, int L, int wf, int min_length,
                              char* area_g, int area_bytes, int4* out) {
    const int lane = w.lane;
    const int nw = (L + 63) >> 6;
    if ((long long)nw * 16 > area_bytes) return -1;
    LdsU64w* gm = (LdsU64w*)area_g;  // identical-column bits
    for (int b = 0; b < nw; b += 4) {
        bool eq[4];
        char x[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int c = (b + u) * 64 + lane;
            eq[u] = c < L;
            x[u] = eq[u] ? A[c] : 0;
        }
        for (int r = 1; r < w.n; r++) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int c = (b + u) * 64 + lane;
                eq[u] &= (c < L ? A[(size_t)r * cap + c] : 0) == x[u];
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const unsigned long long m = ballot(eq[u]);
            if (lane == 0 && b + u < nw) gm[b + u] = m;
        }
    }
    __syncthreads();
    return regions_from_bits<true>(w, gm, nw, L, wf, min_length, area_bytes, out);
}

// AbstractAligner.cpp:89-102: drop columns that are '-' in every row
__device__ int remove_pure_gap_cols(const WaveCtx& w, char* buf, int cap, int L) {
    int dest = 0;
    for (int b = 0; b < L; b += 256) {
        // keep flags of four chunks: row 0 first (four loads in flight), the
        // other rows only where row 0 has a gap
        bool keep[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int c = b + u * 64 + w.lane;
            keep[u] = c < L && buf[c] != '-';
        }
        for (int r = 1; r < w.n; r++) {
            bool need = false;
#pragma unroll
            for (int u = 0; u < 4; u++) need |= (b + u * 64 + w.lane < L) && !keep[u];
            if (!any_lane(WaveCtx{w.lane, w.n, ~0ull, true}, need)) break;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int c = b + u * 64 + w.lane;
                if (c < L && !keep[u]) keep[u] = buf[(size_t)r * cap + c] != '-';
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int base = b + u * 64;
            if (base >= L) break;
            const int c = base + w.lane;
            const unsigned long long km = ballot(keep[u]);
            if (km == ((base + 64 <= L) ? ~0ull : ((1ull << (L - base)) - 1ull)) && dest == base) {
                dest += __popcll(km);  // nothing removed so far
                continue;
            }
            __syncthreads();
            // move kept columns of this chunk left (row by row, lanes = columns)
            const int to = dest + __popcll(km & ((1ull << w.lane) - 1ull));
            for (int r = 0; r < w.n; r++) {
                char x = 0;
                if (keep[u]) x = buf[(size_t)r * cap + c];
                __syncthreads();
                if (keep[u]) buf[(size_t)r * cap + to] = x;
                __syncthreads();
            }
            dest += __popcll(km);
        }
    }
    return dest;
}

// take n units of a bounded counter; -1 when they do not fit (the counter
// still advances: later requests fail too, nothing is handed out twice)
__device__ __forceinline__ long long reserve(unsigned long long* ctr, unsigned long long n, unsigned long long cap) {
    const unsigned long long old = atomicAdd(ctr, n);
    return old + n > cap ? -1 : (long long)old;
}

__device__ __forceinline__ int sub_out_cap(int cap, int width) { return min(cap, (2 * width + 64 + 15) & ~15); }

__device__ __forceinline__ int64_t sub_bytes(int n, int out_cap) {
    return (256 + (int64_t)n * out_cap + 255) & ~255ll;
}

// fix_bad_regions (:428-459), deferred: the regions go to the job's list with
// each bad region's identical columns, every bad region's gap-filtered
// reversed rows to C at its own columns, and the bad regions become sub-jobs
// realigned GPU-wide by k_align_sub; k_align_finish assembles the job.
// Returns false (nothing deferred: realign inline) when the lists or the
// sub-job pool are full.
// (DeferOut instead of SaArgs: no copy of the kernel arguments to the stack)
struct DeferOut {  // the SaArgs fields defer_regions writes
    int4* job_regions;
    int32_t* job_nreg;
    SaSub* subs;
    unsigned long long* alloc;
    unsigned int* counters;
    unsigned char* pool;
    int64_t pool_cap, max_sub;
    int32_t* fin;
};

__device__ __forceinline__ bool defer_regions(const DeferOut a, int n, int j, int64_t reg_off, int reg_cap,
                                           const char* A, char* C, int cap, int R, bool fast, bool counted,
                                           int4 rreg, unsigned long long gmask, const int4* regions,
                                           const unsigned char* good_col) {
    WaveCtx w;
    const int lane = threadIdx.x;
    w.lane = lane;
    w.n = n;
    w.rowmask = (n >= 64) ? ~0ull : ((1ull << n) - 1ull);
    w.act = lane < n;
    if (R > reg_cap) return false;
    int4* jr = a.job_regions + reg_off;
    int nbad = 0;
    int64_t need = 0;
    for (int ri = 0; ri < R; ri++) {
        const int4 rg = fast ? make_int4(bcast(rreg.x, ri), bcast(rreg.y, ri), bcast(rreg.z, ri),
                                         bcast(rreg.w, ri))
                             : regions[ri];
        int before = 0;
        if (!rg.z) {
            if (fast) {
                const int lo = lane * 64, hi = lo + 63;
                if (lo <= rg.y && hi >= rg.x) {
                    const int a0 = max(rg.x, lo) - lo, a1 = min(rg.y, hi) - lo;
                    before = __popcll(gmask & ((a1 == 63 ? ~0ull : ((1ull << (a1 + 1)) - 1)) & (~0ull << a0)));
                }
                before = wave_sum(before);
            } else if (counted) {
                before = rg.w;
            } else {
                for (int c = rg.x + lane; c <= rg.y; c += 64) before += good_col[c];
                before = wave_sum(before);
            }
            nbad++;
            need += sub_bytes(w.n, sub_out_cap(cap, rg.y - rg.x + 1));
        }
        if (lane == 0) jr[ri] = make_int4(rg.x, rg.y, rg.z ? 1 : 0, before);
    }
    if (nbad == 0) return false;
    long long base = 0, s0 = 0;
    if (lane == 0) {
        base = reserve(&a.alloc[0], (unsigned long long)need, (unsigned long long)a.pool_cap);
        if (base >= 0) s0 = (long long)atomicAdd(&a.alloc[1], (unsigned long long)nbad);  // max_sub bounds every job's bad regions
    }
    base = (long long)bcast64((unsigned long long)base, 0);
    s0 = (long long)bcast64((unsigned long long)s0, 0);
    __syncthreads();
    if (base < 0) return false;
    int64_t off = base;
    int k = 0;
    for (int ri = 0; ri < R; ri++) {
        const int4 rg = jr[ri];
        if (rg.z) continue;
        const int out_cap = sub_out_cap(cap, rg.y - rg.x + 1);
        const View cv = filter_reverse(w, A, cap, C + rg.x, cap, rg.x, rg.y + 1);
        const long long sub = s0 + k++;
        if (w.act) ((int*)(a.pool + off))[lane] = cv.len;
        if (lane == 0) {
            SaSub d;
            d.job = j;
            d.x = rg.x;
            d.out_cap = out_cap;
            d.pad = 0;
            d.out_off = off;
            a.subs[sub] = d;
            jr[ri] = make_int4(rg.x, rg.y, -(int)(sub + 1), rg.w);
        }
        off += sub_bytes(w.n, out_cap);
    }
    if (lane == 0) {
        a.job_nreg[j] = R;
        a.fin[atomicAdd(&a.counters[1], 1u)] = j;
    }
    __syncthreads();
    return true;
}

// first word-table epoch of a follow-up kernel: above every epoch the
// previous launches used
__device__ __forceinline__ uint32_t next_epoch(const SaArgs& a) {
    return max(a.epoch_base, atomicMax(a.slot_epoch, 0u) + 1u);
}

// slot setup shared by the three aligner kernels (same LDS layout)
struct SlotEnv {
    Slot S;
    char* stage;
};

__device__ __forceinline__ SlotEnv slot_env(const SaArgs& a, unsigned long long* lds_u64) {
    SlotEnv e;
    Slot& S = e.S;
    const int lane = threadIdx.x;
    const uint32_t ltab = 1u << a.ltab_log2;
    S.lkeys = lds_u64;
    S.lmask = lds_u64 + ltab;
    S.ldone = (uint32_t*)(lds_u64 + 2 * ltab);
    S.ltab_log2 = a.ltab_log2;
    S.lwords = lds_u64 + 2 * ltab + (ltab + 1) / 2;
    S.hist_cap = a.hist_cap;
    for (uint32_t i = lane; i < ltab; i += 64) lds_u64[i] = 0ull;
    __syncthreads();
    e.stage = (char*)S.lwords + a.words_bytes;
    const size_t slot = blockIdx.x;
    const size_t tcap = (size_t)1 << a.tcap_log2;
    S.tkeys = a.tkeys + slot * tcap;
    S.tmask = a.tmask + slot * tcap;
    S.tdone = a.tdone + slot * tcap;
    S.tcap_log2 = a.tcap_log2;
    const size_t stn = (size_t)a.st_depth_max * 64;
    S.st_p = a.st_p + slot * stn;
    S.st_len = a.st_len + slot * stn;
    S.st_pos = a.st_pos + slot * stn;
    S.st_col = a.st_col + slot * a.st_depth_max;
    S.st_depth_max = a.st_depth_max;
    S.regions = a.regions + slot * (size_t)a.slot_cols;
    S.good_col = a.good_col + slot * (size_t)a.slot_cols;
    return e;
}

// rows of a view set into LDS when they fit (every char(q) then an LDS read)
__device__ __forceinline__ void stage_rows(View& v0, int n, char* stage, int stage_bytes) {
    const int lane = threadIdx.x;
    int off = 0, tot = 0;
    for (int r = 0; r < n; r++) {
        const int lr = bcast(v0.len, r);
        if (lane == r) off = tot;
        tot += lr;
    }
    if (tot > stage_bytes) return;
    for (int r = 0; r < n; r++) {
        const char* src = bcast_ptr(v0.p, r);
        const int lr = bcast(v0.len, r), o = bcast(off, r);
        for (int base = 0; base < lr; base += 64 * 8) {
            char x[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int q = base + u * 64 + lane;
                x[u] = q < lr ? src[q] : 0;
            }
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int q = base + u * 64 + lane;
                if (q < lr) stage[o + q] = x[u];
            }
        }
    }
    __syncthreads();
    if (lane < n) v0.p = stage + off;
}

// realing_end (:461-484) re-aligns the reversed, gap-free last aligned_check
// columns; when each of them holds one letter in every row the greedy
// process_seqs rebuilds exactly those columns, so the pass is skipped
__device__ __forceinline__ bool tail_identical(const WaveCtx& w, const char* B, int cap, int c0, int c1) {
    for (int j = c0; j < c1; j++) {
        const int c = w.act ? (unsigned char)B[(size_t)w.lane * cap + j] : 0;
        if (any_lane(w, c == '-') || !all_eq(w, c)) return false;
    }
    return true;
}

// realing_end (:461-484) on B; returns the length (remove_gaps has nothing to
// remove from the similar aligner's columns, see k_align_jobs)
template <class PR>
__device__ int finish_tail(PR& pr, const WaveCtx& w, char* B, char* C, int cap, int L, char* stage,
                           int stage_bytes, int ac, bool& ovf) {
    pr.ob = B;
    int prefix = L - ac;
    if (prefix < 1) prefix = 1;
    if (!ovf && L >= 2 && !tail_identical(w, B, cap, prefix, L)) {
        const View tv = stage_segment(w, B, cap, C, stage, stage_bytes, prefix, L);
        const int Lt = pr.run(tv, prefix);
        if (any_lane(w, pr.ovf)) ovf = true;
        else {
            cm_reverse(w, B, cap, prefix, prefix + Lt);
            L = prefix + Lt;
        }
    }
    __syncthreads();
    return L;
}

// Width of region ri of a deferred job in B: a good region or a bad one whose
// re-alignment did not gain keeps its columns of A, else the re-alignment's
// columns; -1: the re-alignment overflowed
__device__ __forceinline__ int fin_width(const SaArgs& a, int4 rg) {
    const int len = rg.y - rg.x + 1;
    if (rg.z > 0) return len;
    const int2 res = a.sub_res[-rg.z - 1];
    if (res.x < 0) return -1;
    return res.y > rg.w ? res.x : len;  // more identical columns: the re-alignment (score_of :445-455)
}

// k_align_sub: every bad region of every deferred job, one wave each; with a
// plan (k_plan_subs) the segments of the split sub-jobs first, then the other
// sub-jobs
template <bool LONG, int W>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(W))) void k_align_sub(SaArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long lds_u64[];
    const int lane = threadIdx.x;
    SlotEnv e = slot_env(a, lds_u64);
    uint32_t epoch = next_epoch(a), lepoch = 0;
    const unsigned int n_sub = (unsigned int)a.alloc[1];
    // retry launch (a.rq): the sub-jobs whose split chain failed or that
    // overflowed, each whole in a room of its rows' total length
    const bool retry = a.rq != nullptr;
    const bool planned = !retry && a.sctr != nullptr;
    const unsigned int nseg = planned ? a.sctr[SC_QSEG] : 0u;
    const unsigned int nq = retry ? (unsigned int)min((int64_t)a.counters[5], a.max_sub)
                                  : planned ? nseg + a.sctr[SC_QSUB] : n_sub;
    while (true) {
        unsigned int qn = 0;
        if (lane == 0) qn = atomicAdd(&a.counters[retry ? 4 : 0], 1u);
        qn = bcast(qn, 0);
        if (qn >= nq) break;
        const bool seg = qn < nseg;
        const int seg_t = seg ? a.qseg[qn] : -1;
        SaSeg sg{};
        SaSplit sp{};
        int sn;
        if (seg) {
            sg = a.segs[seg_t];
            sp = a.splits[sg.split];
            sn = sp.sub;
        } else {
            sn = retry ? a.rq[qn] : planned ? a.qsub[qn - nseg] : (int)qn;
        }
        const SaSub d = a.subs[sn];
        const SaJob job = a.jobs[d.job];
        const int n = job.n, cap = job.cap;
        WaveCtx w;
        w.lane = lane;
        w.n = n;
        w.rowmask = (n >= 64) ? ~0ull : ((1ull << n) - 1ull);
        w.act = lane < n;
        char* C = (char*)(a.scratch + job.scratch) + 2ll * n * cap;
        const int* T = seg ? a.targets + sp.tgt : nullptr;  // sync state k >= 1 at T[(k-1)*n + row]
        const int start = (seg && sg.k > 0 && w.act) ? T[(sg.k - 1) * n + lane] : 0;
        const bool idle = seg && any_lane(w, start < 0);
        View v{nullptr, 0, 1};
        if (w.act && !idle) {
            v.p = C + (size_t)lane * cap + d.x + start;
            v.len = ((const int*)(a.pool + d.out_off))[lane] - start;
        }
        char* out = seg ? (char*)(a.seg_pool + sg.out) : (char*)(a.pool + d.out_off + 256);
        int ocap = d.out_cap;  // (a re-run below moves the output)
        if (retry) {  // a new room at the proven bound, from the pool
            const int tot = wave_sum(w.act ? v.len : 0);
            const int room = min(cap, (tot + 15) & ~15);
            long long off2 = -1;
            if (lane == 0) off2 = reserve(&a.alloc[0], (unsigned long long)sub_bytes(n, room),
                                          (unsigned long long)a.pool_cap);
            off2 = (long long)bcast64((unsigned long long)off2, 0);
            if (off2 < 0) {  // pool full: the job re-runs whole, as before
                if (lane == 0) a.sub_res[sn] = make_int2(-1, 0);
                __syncthreads();
                continue;
            }
            if (w.act) ((int*)(a.pool + off2))[lane] = ((const int*)(a.pool + d.out_off))[lane];
            if (lane == 0) {
                SaSub d2 = d;
                d2.out_off = off2;
                d2.out_cap = room;
                a.subs[sn] = d2;
            }
            out = (char*)(a.pool + off2 + 256);
            ocap = room;
        }
        const unsigned long long w_start = wall_clock64();
        ProcT<LONG> pr(w, a.P, e.S, out, seg ? sg.cap : ocap, epoch, lepoch);
        int Lc = 0;
        bool ovf = false;
        if (!idle) {
            stage_rows(v, n, e.stage, a.stage_bytes);
            if (seg) pr.set_targets(T, sg.k, sp.K - 1, start);
            Lc = pr.run(v, 0);
            ovf = any_lane(w, pr.ovf);
        }
        __syncthreads();
        // a bad region whose re-alignment outgrew 2 x width + 64 columns (rows
        // with unrelated insertions: R3): again at once in a room of its rows'
        // total length (the proven bound) from the pool, instead of the whole
        // job re-running at attempt 1
        if (!seg && !idle && ovf && any_lane(w, pr.rovf) && !any_lane(w, pr.ovf && !pr.rovf)) {
            const int tot = wave_sum(w.act ? v.len : 0);
            const int room = min(cap, (tot + 15) & ~15);
            long long off2 = -1;
            if (room > d.out_cap) {
                if (lane == 0) off2 = reserve(&a.alloc[0], (unsigned long long)sub_bytes(n, room),
                                              (unsigned long long)a.pool_cap);
                off2 = (long long)bcast64((unsigned long long)off2, 0);
            }
            if (off2 >= 0) {
                if (w.act) ((int*)(a.pool + off2))[lane] = ((const int*)(a.pool + d.out_off))[lane];
                if (lane == 0) {
                    SaSub d2 = d;
                    d2.out_off = off2;
                    d2.out_cap = room;
                    a.subs[sn] = d2;
                }
                out = (char*)(a.pool + off2 + 256);
                ocap = room;
                ProcT<LONG> pr2(w, a.P, e.S, out, room, pr.epoch, pr.lepoch);
                Lc = pr2.run(v, 0);
                ovf = any_lane(w, pr2.ovf);
                pr.epoch = pr2.epoch;
                pr.lepoch = pr2.lepoch;
                if (lane == 0 && a.counters) atomicAdd(&a.counters[3], 1u);  // (sub-jobs re-run)
            }
            __syncthreads();
        }
        if (lane == 0 && a.job_stats) {  // (statistics wanted: the critical path of the launch)
            int64_t* wl = seg ? a.seg_wall + 2 * (size_t)seg_t : (a.sub_wall ? a.sub_wall + 2 * (size_t)sn : nullptr);
            if (wl) {
                wl[0] = (int64_t)w_start;
                wl[1] = (int64_t)wall_clock64();
            }
        }
        if (seg) {
            if (lane == 0)
                a.seg_res[seg_t] = idle ? make_int4(-1, 0, 0, 0)
                                        : make_int4(pr.stop ? pr.tm + 1 : sp.K, Lc, ovf ? 1 : 0, 0);
        } else {
            const int after = ovf ? 0 : count_equal_cols(w, out, ocap, 0, Lc, nullptr);
            if (lane == 0) a.sub_res[sn] = make_int2(ovf ? -1 : Lc, after);
        }
        epoch = pr.epoch;
        lepoch = pr.lepoch;
        __syncthreads();
    }
    if (lane == 0) atomicMax(a.slot_epoch, epoch);
}

// the sub-jobs to retry: failed (columns -1) after their segments' chain or
// their own run, whole ones only (a twin's stays with its job)
__global__ void k_sub_retry_list(SaArgs a) {
    const unsigned int n_sub = (unsigned int)a.alloc[1];
    for (unsigned int sn = blockIdx.x * blockDim.x + threadIdx.x; sn < n_sub; sn += gridDim.x * blockDim.x)
        if (a.sub_res[sn].x < 0 && a.subs[sn].pad >= 0) {
            const unsigned int q = atomicAdd(&a.counters[5], 1u);  // (< n_sub <= max_sub, rq's size)
            if ((int64_t)q < a.max_sub) ((int32_t*)a.rq)[q] = (int32_t)sn;
        }
}

// k_align_finish: realing_end on the deferred jobs' B (= good regions of A +
// the better of each bad region and its re-alignment, k_fin_copy)
template <bool LONG>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void k_align_finish(SaArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long lds_u64[];
    const int lane = threadIdx.x;
    SlotEnv e = slot_env(a, lds_u64);
    uint32_t epoch = next_epoch(a), lepoch = 0;
    const unsigned int n_fin = a.counters[1];
    while (true) {
        unsigned int fn = 0;
        if (lane == 0) fn = atomicAdd(&a.counters[2], 1u);
        fn = bcast(fn, 0);
        if (fn >= n_fin) break;
        const int j = a.fin[fn];
        const SaJob job = a.jobs[j];
        const int n = job.n, cap = job.cap;
        WaveCtx w;
        w.lane = lane;
        w.n = n;
        w.rowmask = (n >= 64) ? ~0ull : ((1ull << n) - 1ull);
        w.act = lane < n;
        char* A = (char*)(a.scratch + job.scratch);
        char* B = A + (size_t)n * cap;
        char* C = B + (size_t)n * cap;
        const int R = a.job_nreg[j];
        const int4* jr = a.job_regions + job.reg_off;
        // B was assembled by k_fin_copy: its length, or an overflow
        int colB = 0, bad = 0;
        for (int ri = lane; ri < R; ri += 64) {
            const int wd = fin_width(a, jr[ri]);
            bad |= wd < 0;
            colB += max(wd, 0);
        }
        colB = wave_sum(colB);
        bool ovf = ballot(bad) != 0 || colB > cap;
        // an overflowed job's length field holds why (negative; NPGX_RETRY_DEBUG)
        const int why = ballot(bad) != 0 ? -10 : colB > cap ? -11 : -12;
        ProcT<LONG> pr(w, a.P, e.S, B, cap, epoch, lepoch);
        const int L = finish_tail(pr, w, B, C, cap, colB, e.stage, a.stage_bytes, a.P.ac, ovf);
        if (lane == 0) {
            a.job_len[j] = ovf ? why : L;
            a.job_status[j] = ovf ? 1 : 0;
        }
        epoch = pr.epoch;
        lepoch = pr.lepoch;
        __syncthreads();
    }
    if (lane == 0) atomicMax(a.slot_epoch, epoch);
}

// ------------------------------------------------------------------ Long jobs
// A wave walks a job's columns one dependent step after another, so a launch
// lasts as long as its longest job (C3: 46 jobs of up to 20k columns and 17
// rows, 14 ms on one wave).  process_cols (SimilarAligner.cpp:344-369) is
// memoryless in the row cursors: every decision reads the rows forward from
// pos (is_equal, try_mismatch, try_gap, try_aligned's min_tail, append_end's
// row ends), so the walk from a state (pos_0 .. pos_n-1) -- and its output
// columns -- is process_seqs of the row suffixes from that state.  A long job
// is therefore cut at K-1 sync states chosen where the rows surely align (the
// middle of a 32-mer that occurs exactly once in a window of every row around
// the same fraction of the rows), and segment k runs process_seqs of the
// suffixes from state k until its top-level walk is exactly at a later state
// m (then the walk from there is segment m's) or ends.  The job's alignment is
// the chain 0 -> m1 -> m2 .. -> end of the segments' columns: bit-exact by
// construction whether or not the speculation holds (a segment whose walk
// passes a state without landing on it just continues to the next one).
// Only uniform advances of the top-level frame are tested (fast_run chunks and
// append_cols); a state inside a multi-column step is still exact because the
// rest of such a step is identical columns (try_mismatch's mc columns,
// apply_gap's gc, the aligned word after a child), which process_cols from
// the state appends one by one.
static constexpr int SPLIT_W = 12;       // sync word length (the reference's aligned_check is 10)
static constexpr int SPLIT_C = 128;      // candidate words per sync state (two per lane)
static constexpr int SPLIT_RMAX = 1024;  // largest search half-width
static constexpr int SPLIT_SPAN = 2 * SPLIT_RMAX + SPLIT_C + 1;  // word positions per row window
static constexpr int SPLIT_CT = 256;     // LDS table of the candidate words
static constexpr int SPLIT_KMAX = 1024;  // segments per job at most
static constexpr int32_t UTWIN_BASE = 1 << 30;  // order[] entries >= this: the twin of unsplit job (entry - UTWIN_BASE)
#ifndef SA_SPLIT_WAVES
#define SA_SPLIT_WAVES 8  // (4 -> 8: C3 align -0.2 ms, R3 -0.2 ms; profiles/r06l_aligner_param_sweep.txt)
#endif
static constexpr int SPLIT_WAVES = SA_SPLIT_WAVES;  // waves per sync state (rows dealt out)
static constexpr int SPLIT_CH = ((SPLIT_SPAN + SPLIT_W + 63) / 64) * 64;  // window chars per wave
static constexpr size_t SPLIT_LDS = (size_t)SPLIT_CT * 8 + (size_t)SPLIT_C * 4 +
                                    (size_t)SPLIT_WAVES * SPLIT_C * 8 + (size_t)64 * SPLIT_C * 2 +
                                    (size_t)SPLIT_WAVES * SPLIT_CH + 64;

// segment length of a job of n rows: per-column cost grows with the rows, so
// few-row jobs take longer segments (the sync state search costs the same)
__host__ __device__ __forceinline__ int split_len_for(int split, int n) {
    const int f = n >= 16 ? 1 : 16 / (n > 0 ? n : 1);
    return split * (f > 8 ? 8 : f);
}

// output columns of segment k of K (longest row mx, search half-width win):
// room for a walk that misses up to about eight sync states in a row (the
// speculation then still chains; past that its job re-runs whole), never
// more than the suffix bound or `limit`
__host__ __device__ __forceinline__ int seg_cap_for(int mx, int k, int K, int win, int64_t limit, bool full = false) {
    const int64_t rest = mx - (int64_t)mx * k / K + win;
    const int64_t reach = 8ll * (mx / K + 1) + 2ll * win;
    const int64_t lim = (full || rest < reach) ? rest : reach;  // full: the rest of the longest row, twice
    const int64_t c = (2 * lim + 64 + 15) & ~15ll;
    return (int)(c < limit ? c : limit);
}

// row `lane` of a split problem: the job's input row, or the gap-filtered
// reversed bad-region row of one of its sub-jobs (in the job's C)
__device__ __forceinline__ void split_row(const SaArgs& a, const SaSplit& sp, const SaJob& job, int lane,
                                          const char*& p, int& len) {
    if (sp.sub == -2) {  // a twin: the job's row reversed
        p = a.twin_rows + a.twin_off[job.row0 + lane];
        len = a.row_len[job.row0 + lane];
    } else if (sp.sub < 0) {
        p = a.rows + a.row_off[job.row0 + lane];
        len = a.row_len[job.row0 + lane];
    } else {
        const SaSub d = a.subs[sp.sub];
        p = (const char*)(a.scratch + job.scratch) + (2 * (size_t)job.n + lane) * job.cap + d.x;
        len = ((const int*)(a.pool + d.out_off))[lane];
    }
}

__device__ __forceinline__ uint32_t base2(uint32_t c) {  // A C G T -> 0..3, anything else 4
    return c == 'A' ? 0u : c == 'C' ? 1u : c == 'G' ? 2u : c == 'T' ? 3u : 4u;
}

// Sync state t of split problem s (the start of segment t+1), one workgroup
// each (tasks[b] = (s, t)).  Candidates: row 0's 12-mers at x0 .. x0+127, x0
// the fraction (t+1)/K of row 0, in a small LDS hash table.  The rows are
// dealt out to the waves: every 12-mer of a row's window around the same
// fraction is looked up there (a rolling word per lane over a stretch of the
// window) and counted per candidate, and a candidate survives when it occurs
// exactly once in every row's window.  The state is the middle of the longest
// run of surviving consecutive candidates, W/2 into its word -- inside an
// identical stretch of at least 12 columns, which the walk crosses column by
// column when it is in step there.  None survives: -1 in every row (segment
// t+1 idles).
__global__ __launch_bounds__(64 * SPLIT_WAVES) void k_split_find(SaArgs a, const int2* tasks, int n_tasks,
                                                                 int task0) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_w[];
    uint32_t* ckey = lds_w;                              // candidate word + 1 (0: empty)
    uint32_t* cid = ckey + SPLIT_CT;                     // its candidate index
    uint32_t* cok = cid + SPLIT_CT;                      // candidate still alive
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t* cnt = cok + SPLIT_C + wid * 2 * SPLIT_C;   // this wave's row: occurrences per candidate
    uint32_t* cpos = cnt + SPLIT_C;                      // ... and the window offset of one
    uint16_t* P = (uint16_t*)(cok + SPLIT_C + SPLIT_WAVES * 2 * SPLIT_C);  // [row][candidate] offsets
    unsigned char* ch = (unsigned char*)(P + 64 * SPLIT_C) + wid * SPLIT_CH;  // this wave's window
    if (n_tasks < 0) n_tasks = (int)min(a.sctr[SC_FIND], (unsigned int)a.cap_find);  // the sub-job pass
    const uint32_t WM = (1u << (2 * SPLIT_W)) - 1u;
    constexpr int PER = SPLIT_CH / 64;
    for (int b = task0 + blockIdx.x; b < n_tasks; b += gridDim.x) {
        const int2 tk = tasks[b];
        if (tk.x < 0) continue;  // (a sub-job k_plan_subs could not split)
        const SaSplit sp = a.splits[tk.x];
        const SaJob job = a.jobs[sp.job];
        const int n = job.n, t = tk.y, R = min(sp.win, SPLIT_RMAX);
        const int span = 2 * R + SPLIT_C + 1;
        const int S = (span + 63) / 64;  // window positions per lane (a contiguous stretch)
        // window chars of row i into registers, then into this wave's LDS window
        unsigned char nx[PER];
        auto load_row = [&](int i, int& lo) {
            const char* ri;
            int li;
            split_row(a, sp, job, i, ri, li);
            lo = (int)((int64_t)li * (t + 1) / sp.K) - R;
#pragma unroll
            for (int u = 0; u < PER; u++) {
                const int q = u * 64 + lane, p = lo + q;
                nx[u] = (q < span + SPLIT_W - 1 && p >= 0 && p < li) ? (unsigned char)ri[p] : 0;
            }
        };
        auto stage = [&]() {
#pragma unroll
            for (int u = 0; u < PER; u++) ch[u * 64 + lane] = nx[u];
        };
        __syncthreads();
        for (int e = threadIdx.x; e < SPLIT_CT; e += 64 * SPLIT_WAVES) ckey[e] = 0u;
        __syncthreads();
        if (wid == 0) {  // the candidates: row 0 at window offsets R + c, into the table
            int lo0;
            load_row(0, lo0);
            stage();
            wave_or_wg_sync<false>();
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int q = R + lane + 64 * h;
                uint32_t x = 0, bad = 0;
                for (int j = 0; j < SPLIT_W; j++) {
                    const uint32_t c = base2(ch[q + j]);
                    bad |= c >> 2;
                    x = (x << 2) | (c & 3u);
                }
                x &= WM;
                bool ok = bad == 0 && lo0 >= 0;
                if (ok) {
                    const uint32_t key = x + 1u;
                    uint32_t e = (x * 2654435761u) >> 24;
                    while (true) {
                        const uint32_t old = atomicCAS(&ckey[e], 0u, key);
                        if (old == 0u) {
                            cid[e] = (uint32_t)(lane + 64 * h);
                            break;
                        }
                        if (old == key) {  // a repeated candidate word: both fail on row 0's count
                            ok = false;
                            break;
                        }
                        e = (e + 1) & (SPLIT_CT - 1);
                    }
                }
                cok[lane + 64 * h] = ok;
            }
        }
        __syncthreads();
        int lo_next = 0;
        if (wid < n) load_row(wid, lo_next);
        for (int i = wid; i < n; i += SPLIT_WAVES) {
            const int lo = lo_next;
            wave_or_wg_sync<false>();
            stage();
            for (int e = lane; e < SPLIT_C; e += 64) cnt[e] = 0u;
            wave_or_wg_sync<false>();
            if (i + SPLIT_WAVES < n) load_row(i + SPLIT_WAVES, lo_next);
            (void)lo;
            // this lane's stretch of window words, rolling
            const int q0 = lane * S, q1 = min(span, q0 + S);
            if (q0 < q1) {
                uint32_t x = 0;
                int nb = 0;
                for (int j = 0; j < SPLIT_W - 1; j++) {
                    const uint32_t c = base2(ch[q0 + j]);
                    nb += (int)(c >> 2);
                    x = (x << 2) | (c & 3u);
                }
                for (int q = q0; q < q1; q++) {
                    const uint32_t cin = base2(ch[q + SPLIT_W - 1]);
                    nb += (int)(cin >> 2);
                    x = ((x << 2) | (cin & 3u)) & WM;
                    if (nb == 0) {
                        uint32_t e = (x * 2654435761u) >> 24;
                        const uint32_t key = x + 1u;
                        while (true) {
                            const uint32_t k = ckey[e];
                            if (k == key) {
                                const uint32_t c = cid[e];
                                atomicAdd(&cnt[c], 1u);
                                cpos[c] = (uint32_t)q;
                                break;
                            }
                            if (k == 0u) break;
                            e = (e + 1) & (SPLIT_CT - 1);
                        }
                    }
                    nb -= (int)(base2(ch[q]) >> 2);  // char q leaves the next word
                }
            }
            wave_or_wg_sync<false>();
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int c = lane + 64 * h;
                if (cnt[c] == 1u) P[i * SPLIT_C + c] = (uint16_t)cpos[c];
                else cok[c] = 0u;
            }
        }
        __syncthreads();
        if (wid == 0) {
            // the longest run of surviving consecutive candidates, its middle
            const unsigned long long m0 = ballot(cok[lane] != 0u), m1 = ballot(cok[lane + 64] != 0u);
            int best = -1, blen = 0, run = 0;
            for (int c = 0; c < SPLIT_C; c++) {  // (wave-uniform scan of the two masks)
                const bool o = c < 64 ? ((m0 >> c) & 1ull) : ((m1 >> (c - 64)) & 1ull);
                run = o ? run + 1 : 0;
                if (run > blen) {
                    blen = run;
                    best = c - (run - 1) / 2;
                }
            }
            int* out = a.targets + sp.tgt + (int64_t)t * n;
            if (lane < n) {
                int v = -1;
                if (best >= 0) {
                    const char* ri;
                    int li;
                    split_row(a, sp, job, lane, ri, li);
                    const int lo = (int)((int64_t)li * (t + 1) / sp.K) - R;
                    v = lo + (int)P[lane * SPLIT_C + best] + SPLIT_W / 2;
                }
                out[lane] = v;
            }
        }
    }  // tasks
}

// ---------------------------------------------------- split jobs after their segments
static constexpr int POST_THREADS = 256;
// k_split_post's workgroup: FindLowSimilar's region rounds over a whole-genome
// chain (tens of thousands of regions in global memory) are bound by the
// elements each thread walks per round
static constexpr int REG_THREADS = 1024;
static constexpr int FIN_PARTS = 64;  // workgroups assembling one deferred job's B
static constexpr size_t POST_LDS = 144 * 1024;

__device__ __forceinline__ long long wave_sum64(long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (long long)shfl64((unsigned long long)v, threadIdx.x % 64 ^ o);
    return v;
}

// exclusive prefix sum over the POST_THREADS threads of the workgroup (every
// thread calls it); *total = the sum of all
__device__ __forceinline__ int block_scan_excl(int v, int* total, int* scratch4) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(inc, o);
        if (lane >= o) inc += t;
    }
    if (lane == 63) scratch4[wid] = inc;
    __syncthreads();
    int before = 0, all = 0;
    const int nwv = (int)blockDim.x >> 6;  // (POST_THREADS or REG_THREADS)
    for (int q = 0; q < nwv; q++) {
        const int s = scratch4[q];
        before += q < wid ? s : 0;
        all += s;
    }
    __syncthreads();
    *total = all;
    return before + inc - v;
}

// FindLowSimilar::make_regions (:62-80) + reduce_regions (:121-130) by the
// whole workgroup, from the identical-column bits gm[0, nw): the reference
// merges the first minimum-weight region with its neighbours until every
// weight reaches min_length.  A region whose (weight, index) is below that of
// every region within two places is merged by the reference before anything
// touches its neighbours (merged weights only grow, and nothing within two
// places can become the minimum first), and two such regions are at least
// three places apart: so every round merges all of them at once, with the
// reference's result.  Survivors to out[] as (start, stop, good, identical
// columns); returns their count, or -1 when the area (LDS, or the global
// work area of a chain too long for LDS: G, I plain pointers) is too small or
// more than out_cap survive.
template <class G, class I>
__device__ int regions_block(G* gm, int nw, int L, int wf, int min_length, long long area_bytes, int4* out,
                             int out_cap, int* scratch4) {
    const int tid = threadIdx.x;
    // region starts: where the identical bit flips (and column 0)
    int cnt = 0;
    for (int q = tid; q < nw; q += (int)blockDim.x) {
        const unsigned long long g = gm[q];
        const unsigned long long valid = (q < nw - 1 || (L & 63) == 0) ? ~0ull : ((1ull << (L & 63)) - 1);
        unsigned long long st = (g ^ ((g << 1) | (q > 0 ? (gm[q - 1] >> 63) : (g & 1ull)))) & valid;
        if (q == 0) st |= 1ull;
        cnt += __popcll(st);
    }
    int R = 0;
    block_scan_excl(cnt, &R, scratch4);
    // two copies of the region arrays (a round reads one, writes the other)
    const long long need = (long long)nw * 8 + (long long)R * 17 + 64;
    if (need > area_bytes) return -1;
    I* rx = (I*)(gm + nw);
    I* rw = rx + R;  // weight | good << 31
    I* qx = rw + R;
    I* qw = qx + R;
    unsigned char* mf = (unsigned char*)(qw + R);  // this round's merging regions
    // starts in order: words dealt out in contiguous runs per thread
    {
        const int per = (nw + (int)blockDim.x - 1) / (int)blockDim.x;
        const int q0 = min(nw, tid * per), q1 = min(nw, q0 + per);
        int c = 0;
        for (int q = q0; q < q1; q++) {
            const unsigned long long g = gm[q];
            const unsigned long long valid = (q < nw - 1 || (L & 63) == 0) ? ~0ull : ((1ull << (L & 63)) - 1);
            unsigned long long st = (g ^ ((g << 1) | (q > 0 ? (gm[q - 1] >> 63) : (g & 1ull)))) & valid;
            if (q == 0) st |= 1ull;
            c += __popcll(st);
        }
        int tot = 0;
        int i = block_scan_excl(c, &tot, scratch4);
        for (int q = q0; q < q1; q++) {
            const unsigned long long g = gm[q];
            const unsigned long long valid = (q < nw - 1 || (L & 63) == 0) ? ~0ull : ((1ull << (L & 63)) - 1);
            unsigned long long st = (g ^ ((g << 1) | (q > 0 ? (gm[q - 1] >> 63) : (g & 1ull)))) & valid;
            if (q == 0) st |= 1ull;
            for (; st; st &= st - 1) {
                const int col = q * 64 + __ffsll((long long)st) - 1;
                rx[i] = col;
                rw[i] = (int)((g >> (col & 63)) & 1ull) << 31;
                i++;
            }
        }
    }
    __syncthreads();
    const int WM = 0x7fffffff;
    for (int i = tid; i < R; i += (int)blockDim.x) {  // Region::set_weight :48-54
        const int len = (i + 1 < R ? rx[i + 1] : L) - rx[i];
        const int good = (int)((unsigned)rw[i] >> 31);
        rw[i] = (good << 31) | (good ? len : len * wf);
    }
    __syncthreads();
    __shared__ int s_any;
    while (R >= 2) {
        if (tid == 0) s_any = 0;
        __syncthreads();
        int any = 0;
        for (int i = tid; i < R; i += (int)blockDim.x) {
            const int wi = rw[i] & WM;
            bool m = wi < min_length;
            for (int d = -2; d <= 2 && m; d++) {
                const int k = i + d;
                if (d == 0 || k < 0 || k >= R) continue;
                const int wk = rw[k] & WM;
                m = wi < wk || (wi == wk && i < k);
            }
            mf[i] = m;
            any |= m;
        }
        if (any) s_any = 1;
        __syncthreads();
        if (!s_any) break;
        // merge (merge_region :94-119) and compact into the other copy: every
        // thread a contiguous run of regions, one scan for the new places
        const int C = (R + (int)blockDim.x - 1) / (int)blockDim.x;
        const int i0 = min(R, tid * C), i1 = min(R, i0 + C);
        int kept = 0;
        for (int i = i0; i < i1; i++) kept += !((i > 0 && mf[i - 1]) || (i + 1 < R && mf[i + 1]));
        int tot = 0;
        int at = block_scan_excl(kept, &tot, scratch4);
        for (int i = i0; i < i1; i++) {
            if ((i > 0 && mf[i - 1]) || (i + 1 < R && mf[i + 1])) continue;  // merged into a neighbour
            int nx = rx[i], nwt = rw[i];
            if (mf[i]) {
                int wsum = nwt & WM;
                if (i > 0) {
                    nx = rx[i - 1];
                    wsum += rw[i - 1] & WM;
                }
                if (i + 1 < R) wsum += rw[i + 1] & WM;
                nwt = ((((unsigned)nwt >> 31) ? 0 : 1) << 31) | wsum;
            }
            qx[at] = nx;
            qw[at] = nwt;
            at++;
        }
        __syncthreads();
        I* t = rx;
        rx = qx;
        qx = t;
        t = rw;
        rw = qw;
        qw = t;
        R = tot;
    }
    if (R > out_cap) return -1;
    // survivors with their identical columns (score_of before re-alignment)
    for (int i = tid; i < R; i += (int)blockDim.x) {
        const int x = rx[i], y = (i + 1 < R ? rx[i + 1] : L) - 1;
        const int good = (int)((unsigned)rw[i] >> 31);
        int c = 0;
        if (!good)
            for (int q = x >> 6; q <= (y >> 6); q++) {
                const int lo = q == (x >> 6) ? (x & 63) : 0, hi = q == (y >> 6) ? (y & 63) : 63;
                c += __popcll(gm[q] & ((hi == 63 ? ~0ull : ((1ull << (hi + 1)) - 1)) & (~0ull << lo)));
            }
        out[i] = make_int4(x, y, good, c);
    }
    __syncthreads();
    return R;
}

// After k_align_jobs, per split job: k_split_chain follows its segments'
// chain (0 -> m1 -> m2 .. -> end), k_chain_copy copies the chain into the
// job's A with the identical-column bits (count_equal_cols :416-426), many
// workgroups per job, and k_split_post (one workgroup per job) derives
// FindLowSimilar's regions from those bits (make_regions + reduce_regions, in
// LDS, or in the split's global work area when too long) and defers
// fix_bad_regions: every bad region is queued as a sub-job for k_align_sub
// (its rows gap-filtered and reversed into C by k_sub_rows); k_fin_copy /
// k_align_finish assemble B and run realing_end.  A chain that overflowed or
// does not fit marks the job for the whole-job re-run (status 1).
static constexpr int CHAIN_PART = 8192;  // output columns per k_chain_copy workgroup

__device__ __forceinline__ unsigned long long* split_bits(const SaArgs& a, const SaSplit& sp, int s) {
    return sp.post >= 0 ? (unsigned long long*)(a.post_area + sp.post) : a.chain_bits + a.bits_off[s];
}

// rows 1..n-1 of four columns (a dword at src + r * scap each) handed to
// put(r, x) after the loads of eight rows are in flight (a put's stores
// cannot be proven apart from the next rows' loads, so load-store-load
// would pay one memory round trip per row); returns the OR of every row's
// XOR with row 0's dword x0 (zero bytes: identical columns)
template <class Put>
__device__ __forceinline__ uint32_t rows_dwords(const char* src, size_t scap, int n, uint32_t x0, Put put) {
    uint32_t diff = 0;
    for (int r0 = 1; r0 < n; r0 += 8) {
        uint32_t x[8];
#pragma unroll
        for (int u = 0; u < 8; u++) x[u] = r0 + u < n ? *(const uint32_t*)(src + (size_t)(r0 + u) * scap) : x0;
#pragma unroll
        for (int u = 0; u < 8; u++) {
            if (r0 + u >= n) break;
            diff |= x[u] ^ x0;
            put(r0 + u, x[u]);
        }
    }
    return diff;
}

// one workgroup per job split: the segment results in parallel into LDS, the
// walk along the chain by one thread, the chain and its identical-column bit
// words (cleared) to global memory
__global__ __launch_bounds__(POST_THREADS) void k_split_chain(SaArgs a) {
    __shared__ int nx[SPLIT_KMAX], nc[SPLIT_KMAX];
    __shared__ int s_np, s_L0, s_fail;
    const int tid = threadIdx.x, si = blockIdx.x;
    const SaSplit sp = a.splits[si];
    const SaJob job = a.jobs[sp.job];
    for (int k = tid; k < sp.K; k += POST_THREADS) {
        const int4 r = a.seg_res[sp.seg0 + k];
        nx[k] = r.x;
        nc[k] = r.z ? -1 : r.y;
    }
    __syncthreads();
    if (tid == 0) {
        int k = 0, col = 0, np = 0, fail = 0;
        int4* ch = a.chain + sp.seg0;
        while (k < sp.K) {
            const int nxt = nx[k], cols = nc[k];
            if (nxt <= k || cols < 0 || col + cols > job.cap) {  // (an idle segment is never on the chain)
                fail = nxt <= k ? 1 : cols < 0 ? 2 : 3;  // (NPGX_RETRY_DEBUG: job_len -201 / -202 / -203)
                break;
            }
            ch[np] = make_int4(sp.seg0 + k, cols, col, 0);
            np++;
            col += cols;
            k = nxt;
        }
        s_np = np;
        s_L0 = col;
        s_fail = fail;
        a.chain_hdr[si] = make_int4(np, col, fail, 0);
    }
    __syncthreads();
    if (s_fail) return;
    unsigned long long* gb = split_bits(a, sp, si);
    const int nw = (s_L0 + 63) >> 6;
    for (int q = tid; q < nw; q += POST_THREADS) gb[q] = 0ull;
}

// workgroup b: output columns [c0, c0 + CHAIN_PART) of one job split's chain
// into A, four columns per thread (rows read as dwords), the identical
// columns' bits OR-ed into the split's bit words
__global__ __launch_bounds__(POST_THREADS) void k_chain_copy(SaArgs a, int n_splits) {
    const int b = blockIdx.x, tid = threadIdx.x;
    int lo = 0, hi = n_splits - 1;  // the split whose parts hold b
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.part0[mid] <= b) lo = mid;
        else hi = mid - 1;
    }
    const int si = lo;
    const int4 hd = a.chain_hdr[si];
    const int c0 = (b - a.part0[si]) * CHAIN_PART, c1 = min(hd.y, c0 + CHAIN_PART);
    if (hd.z || c0 >= c1) return;
    const SaSplit sp = a.splits[si];
    const SaJob job = a.jobs[sp.job];
    const int n = job.n, cap = job.cap;
    char* A = (char*)(a.scratch + job.scratch);
    unsigned long long* gb = split_bits(a, sp, si);
    const int4* ch = a.chain + sp.seg0;
    int e0 = 0, eh = hd.x - 1;  // the chain element holding column c0
    while (e0 < eh) {
        const int mid = (e0 + eh + 1) >> 1;
        if (ch[mid].z <= c0) e0 = mid;
        else eh = mid - 1;
    }
    for (int e = e0; e < hd.x; e++) {
        const int4 el = ch[e];
        const int d0 = el.z, cols = el.y;
        if (d0 >= c1) break;
        const SaSeg g = a.segs[el.x];
        const char* src = (const char*)(a.seg_pool + g.out);
        const int cs = (max(c0 - d0, 0)) & ~3, ce = min(c1 - d0, cols);
        for (int c = cs + 4 * tid; c < ce; c += 4 * POST_THREADS) {
            const uint32_t x0 = *(const uint32_t*)(src + c);  // (rows of 16-aligned length: in bounds)
            int lo_b = 0, hi_b = min(4, ce - c);  // this part's columns only
            if (d0 + c < c0) lo_b = c0 - (d0 + c);
            char* d = A + d0 + c;
            const uint32_t diff = rows_dwords(src + c, (size_t)g.cap, n, x0, [&](int r, uint32_t x) {
                char* dr = A + (size_t)r * cap + d0 + c;
                for (int q = lo_b; q < hi_b; q++) dr[q] = (char)(x >> (8 * q));
            });
            for (int q = lo_b; q < hi_b; q++) d[q] = (char)(x0 >> (8 * q));
            unsigned long long m0 = 0, m1 = 0;
            const int col0 = d0 + c, w0 = col0 >> 6;
            for (int q = lo_b; q < hi_b; q++)
                if (!((diff >> (8 * q)) & 0xFFu)) {
                    const int col = col0 + q;
                    if ((col >> 6) == w0) m0 |= 1ull << (col & 63);
                    else m1 |= 1ull << (col & 63);
                }
            if (m0) atomicOr(&gb[w0], m0);
            if (m1) atomicOr(&gb[w0 + 1], m1);
        }
    }
}

struct PostShared {
    int np, L0, fail, R, scan[REG_THREADS / 64];
};

template <class G, class I>
__device__ void split_post_body(const SaArgs& a, const SaSplit& sp, G* gm, long long area_bytes, PostShared& ps);

__global__ __launch_bounds__(REG_THREADS) void k_split_post(SaArgs a, int lds_bytes) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long lds_p[];
    __shared__ PostShared ps;
    const int tid = threadIdx.x, si = blockIdx.x;
    const SaSplit sp = a.splits[si];
    const SaJob job = a.jobs[sp.job];
    const int4 hd = a.chain_hdr[si];
    if (tid == 0) {
        ps.np = hd.x;
        ps.L0 = hd.y;
        ps.fail = hd.z;
        ps.R = 0;
    }
    const int nw = (hd.y + 63) >> 6;
    if (sp.post >= 0 && !hd.z) {  // the bits are already in the split's global work area
        __syncthreads();
        split_post_body<unsigned long long, int>(a, sp, (unsigned long long*)(a.post_area + sp.post),
                                                 (long long)nw * 8 + ((long long)job.cap + 1) * 17 + 64, ps);
        return;
    }
    LdsU64w* gm = (LdsU64w*)lds_p;
    if (!hd.z && (long long)nw * 16 <= lds_bytes) {
        const unsigned long long* gb = a.chain_bits + a.bits_off[si];
        for (int q = tid; q < nw; q += (int)blockDim.x) gm[q] = gb[q];
    }
    __syncthreads();
    split_post_body<LdsU64w, LdsInt>(a, sp, gm, lds_bytes, ps);
}

template <class G, class I>
__device__ void split_post_body(const SaArgs& a, const SaSplit& sp, G* gm, long long area_bytes, PostShared& ps) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int j = sp.job;
    const SaJob job = a.jobs[j];
    const int n = job.n, cap = job.cap;
    char* A = (char*)(a.scratch + job.scratch);
    char* C = A + 2 * (size_t)n * cap;
    const int L0 = ps.L0, nw = (L0 + 63) >> 6;
    if (ps.fail || (long long)nw * 16 > area_bytes) {
        if (tid == 0) {
            a.job_len[j] = ps.fail ? -(200 + ps.fail) : -21;
            a.job_status[j] = 1;
        }
        return;
    }
    int4* jr = a.job_regions + job.reg_off;
    const int R = regions_block<G, I>(gm, nw, L0, a.P.wf, a.P.min_length, area_bytes, jr, job.reg_cap, ps.scan);
    if (R < 0 || R > job.reg_cap) {
        if (tid == 0) {
            a.job_len[j] = -22;
            a.job_status[j] = 1;
        }
        return;
    }
    // every bad region a sub-job: pool bytes and sub-job ids in region order
    if (wid == 0) {
        long long need = 0;
        int nbad = 0;
        for (int ri = lane; ri < R; ri += 64) {
            const int4 rg = jr[ri];
            if (!rg.z) {
                nbad++;
                need += sub_bytes(n, sub_out_cap(cap, rg.y - rg.x + 1));
            }
        }
        nbad = wave_sum(nbad);
        need = wave_sum64(need);
        long long base = 0, s0 = 0;
        if (lane == 0 && nbad) {
            base = reserve(&a.alloc[0], (unsigned long long)need, (unsigned long long)a.pool_cap);
            if (base >= 0) s0 = (long long)atomicAdd(&a.alloc[1], (unsigned long long)nbad);
        }
        base = (long long)bcast64((unsigned long long)base, 0);
        s0 = (long long)bcast64((unsigned long long)s0, 0);
        if (base < 0) {
            if (lane == 0) ps.R = -1;
        } else {
            long long off = base;
            int sub = (int)s0;
            for (int c0 = 0; c0 < R; c0 += 64) {
                const int ri = c0 + lane;
                const int4 rg = ri < R ? jr[ri] : make_int4(0, 0, 1, 0);
                const bool bad = ri < R && !rg.z;
                const int oc = bad ? sub_out_cap(cap, rg.y - rg.x + 1) : 0;
                const long long by = bad ? sub_bytes(n, oc) : 0;
                long long pb = by;  // inclusive scans over the chunk
                int pc = bad ? 1 : 0;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const long long tb = (long long)shfl64((unsigned long long)pb, max(lane - o, 0));
                    const int tc = __shfl(pc, max(lane - o, 0));
                    if (lane >= o) {
                        pb += tb;
                        pc += tc;
                    }
                }
                if (bad) {
                    const int sn = sub + pc - 1;
                    SaSub d;
                    d.job = j;
                    d.x = rg.x;
                    d.out_cap = oc;
                    d.pad = rg.y - rg.x + 1;  // > 0: its rows are k_sub_rows' to write
                    d.out_off = off + pb - by;
                    if (sp.twin > 0 && rg.x == 0 && rg.y == L0 - 1) {
                        // the whole job is one bad region: its rows gap-filtered
                        // and reversed are the job's input rows reversed, whose
                        // walk the twin has done (k_twin_post takes it over;
                        // a negative width keeps k_sub_rows / k_plan_subs off)
                        d.pad = -d.pad;
                        ((SaSplit*)a.splits)[sp.twin - 1].sub = sn;
                    }
                    a.subs[sn] = d;
                    jr[ri] = make_int4(rg.x, rg.y, -(sn + 1), rg.w);
                }
                off += (long long)shfl64((unsigned long long)pb, 63);
                sub += __shfl(pc, 63);
            }
        }
    }
    __syncthreads();
    if (ps.R < 0) {  // sub-job pool full
        if (tid == 0) {
            a.job_len[j] = -23;
            a.job_status[j] = 1;
        }
        return;
    }
    if (tid == 0) {
        a.job_nreg[j] = R;
        a.fin[atomicAdd(&a.counters[1], 1u)] = j;
        a.job_len[j] = L0;
        a.job_status[j] = 3;
    }
}

// The rows of the bad regions k_split_post queued (SaSub.pad = the region's
// width): columns [x, x + width) of every row of the job's A, gap-filtered
// and reversed into C at column x (fix_bad_regions :443-447), the lengths
// into the sub-job's pool header; one wave per (sub-job, row) for the rows
// the batch's jobs have (`rows`, not 64 row slots: each slot reread the
// sub-job and job records -- 11 ms at C5's 8-row jobs)
__global__ __launch_bounds__(256) void k_sub_rows(SaArgs a, int rows) {
    const unsigned long long n_pairs = a.alloc[1] * (unsigned long long)rows;
    const int lane = threadIdx.x & 63;
    for (unsigned long long p = blockIdx.x * 4ull + (threadIdx.x >> 6); p < n_pairs; p += gridDim.x * 4ull) {
        const SaSub d = a.subs[p / rows];
        if (d.pad <= 0) continue;
        const SaJob job = a.jobs[d.job];
        const int r = (int)(p % rows);
        if (r < job.n) {
            const char* src = (const char*)(a.scratch + job.scratch) + (size_t)r * job.cap;
            char* dst = (char*)(a.scratch + job.scratch) + (2 * (size_t)job.n + r) * job.cap + d.x;
            int k = 0;
            // 1024 columns per step (16 a lane, from the top down): the lane's
            // letters counted, a wave prefix sum places them (long bad regions --
            // tens of thousands of columns at C5 -- took one step per 64 columns)
            for (int top = d.x + d.pad - 1; top >= d.x; top -= 1024) {
                const int hi = top - 16 * lane;  // this lane's columns hi, hi-1, .., hi-15
                char x[16];
                int cnt = 0;
    #pragma unroll
                for (int u = 0; u < 16; u++) {
                    const int idx = hi - u;
                    x[u] = idx >= d.x ? src[idx] : '-';
                    cnt += x[u] != '-';
                }
                int pre = cnt;  // inclusive prefix over the lanes
    #pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int t = __shfl_up(pre, o);
                    if (lane >= o) pre += t;
                }
                int at = k + pre - cnt;
    #pragma unroll
                for (int u = 0; u < 16; u++)
                    if (x[u] != '-') dst[at++] = x[u];
                k += __shfl(pre, 63);
            }
            if (lane == 0) ((int*)(a.pool + d.out_off))[r] = k;
        }
    }
}

// One thread per sub-job (after k_align_jobs and k_split_post created them):
// a sub-job whose longest row spans at least two segments is split like the
// long jobs -- its sync states by k_split_find, its segments ahead of the
// whole sub-jobs in k_align_sub's queue, its chain by k_sub_post.  The split
// arrays are bounded; a sub-job that does not fit them runs whole.
__global__ __launch_bounds__(256) void k_plan_subs(SaArgs a) {
    const unsigned int n_sub = (unsigned int)a.alloc[1];
    unsigned long long* pool_ctr = (unsigned long long*)(a.sctr + SC_POOL_LO);
    for (unsigned int sn = blockIdx.x * blockDim.x + threadIdx.x; sn < n_sub; sn += gridDim.x * blockDim.x) {
        const SaSub d = a.subs[sn];
        if (d.pad < 0) continue;  // a twin's walk is this sub-job's re-alignment (k_twin_post)
        const SaJob job = a.jobs[d.job];
        const int n = job.n;
        const int* lens = (const int*)(a.pool + d.out_off);
        int mx = 0;
        for (int i = 0; i < n; i++) mx = max(mx, lens[i]);
        const int K = (a.split_len > 0 && n >= 2) ? min(SPLIT_KMAX, mx / split_len_for(a.split_len, n)) : 1;
        bool ok = K >= 2 && mx >= 4 * SPLIT_W;
        if (ok) {
            const int win = min(SPLIT_RMAX, 64 + mx / 128);
            auto seg_cap = [&](int k) { return seg_cap_for(mx, k, K, win, d.out_cap); };
            int64_t bytes = 0;
            for (int k = 0; k < K; k++) bytes += ((int64_t)n * seg_cap(k) + 255) & ~255ll;
            const unsigned long long p0 = atomicAdd(pool_ctr, (unsigned long long)bytes);
            const unsigned int s0 = atomicAdd(&a.sctr[SC_SEGS], (unsigned int)K);
            const unsigned int t0 = atomicAdd(&a.sctr[SC_TGT], (unsigned int)((K - 1) * n));
            const unsigned int f0 = atomicAdd(&a.sctr[SC_FIND], (unsigned int)(K - 1));
            const unsigned int si = atomicAdd(&a.sctr[SC_SPLITS], 1u);
            ok = p0 + bytes <= (unsigned long long)a.cap_pool && s0 + K <= (unsigned int)a.cap_segs &&
                 (int64_t)t0 + (int64_t)(K - 1) * n <= a.cap_tgt && (int64_t)f0 + K - 1 <= a.cap_find &&
                 si < (unsigned int)a.cap_splits;
            for (int t = 0; t + 1 < K; t++)  // (allocated find tasks are written either way)
                if ((int64_t)f0 + t < a.cap_find) a.ftasks[f0 + t] = ok ? make_int2((int)si, t) : make_int2(-1, -1);
            if (si < (unsigned int)a.cap_splits) {
                SaSplit sp;
                sp.job = d.job;
                sp.K = ok ? K : 0;
                sp.tgt = t0;
                sp.seg0 = (int32_t)s0;
                sp.win = win;
                sp.sub = (int32_t)sn;
                sp.twin = 0;
                sp.post = -1;
                ((SaSplit*)a.splits)[si] = sp;
            }
            if (ok) {
                int64_t off = (int64_t)p0;
                const unsigned int q0 = atomicAdd(&a.sctr[SC_QSEG], (unsigned int)K);
                for (int k = 0; k < K; k++) {
                    SaSeg g;
                    g.split = (int32_t)si;
                    g.k = k;
                    g.cap = seg_cap(k);
                    g.pad = 0;
                    g.out = off;
                    off += ((int64_t)n * g.cap + 255) & ~255ll;
                    ((SaSeg*)a.segs)[s0 + k] = g;
                    a.qseg[q0 + k] = (int32_t)(s0 + k);
                }
            }
        }
        if (!ok) a.qsub[atomicAdd(&a.sctr[SC_QSUB], 1u)] = (int32_t)sn;
    }
}

// One workgroup per split sub-job (split index from `first`): the chain of its
// segments into the sub-job's output (rows of out_cap) and its identical
// columns (score_of after the re-alignment) -- what k_align_sub writes for a
// whole sub-job; a chain that overflowed or does not fit: (-1, 0).
// Twins (k_twin_post, `last` >= 0: the twin splits [first, last)): a twin
// whose job k_split_post found to be one bad region (sp.sub >= 0) chains into
// that sub-job's output; when its chain fails the sub-job goes back to the
// ordinary path (its width restored: k_sub_rows, k_plan_subs, k_align_sub).
__global__ __launch_bounds__(POST_THREADS) void k_sub_post(SaArgs a, int first, int last_twin) {
    __shared__ int pk[SPLIT_KMAX], pcols[SPLIT_KMAX], pdst[SPLIT_KMAX];
    __shared__ int s_np, s_L, s_fail, s_scan[POST_THREADS / 64];
    const int tid = threadIdx.x;
    const bool twins = last_twin >= 0;
    const int last = twins ? last_twin : (int)min(a.sctr[SC_SPLITS], (unsigned int)a.cap_splits);
    for (int si = first + blockIdx.x; si < last; si += gridDim.x) {
        const SaSplit sp = a.splits[si];
        if (sp.K < 2 || sp.sub < 0) continue;  // (a twin its job did not need)
        const SaSub d = a.subs[sp.sub];
        const int n = a.jobs[d.job].n;
        __syncthreads();
        if (tid == 0) {
            int k = 0, col = 0, np = 0, fail = 0;
            while (k < sp.K) {
                const int4 r = a.seg_res[sp.seg0 + k];
                if (r.x <= k || r.z || col + r.y > d.out_cap) {
                    fail = 1;
                    break;
                }
                pk[np] = sp.seg0 + k;
                pcols[np] = r.y;
                pdst[np] = col;
                np++;
                col += r.y;
                k = r.x;
            }
            s_np = np;
            s_L = col;
            s_fail = fail;
        }
        __syncthreads();
        if (s_fail) {
            if (tid == 0) {
                if (twins) a.subs[sp.sub].pad = -d.pad;  // the ordinary re-alignment after all
                else a.sub_res[sp.sub] = make_int2(-1, 0);
            }
            continue;
        }
        char* out = (char*)(a.pool + d.out_off + 256);
        int same = 0;
        for (int p = 0; p < s_np; p++) {
            const SaSeg g = a.segs[pk[p]];
            const char* src = (const char*)(a.seg_pool + g.out);
            const int cols = pcols[p], d0 = pdst[p];
            for (int c = 4 * tid; c < cols; c += 4 * POST_THREADS) {
                const int nb = min(4, cols - c);
                const uint32_t x0 = *(const uint32_t*)(src + c);
                const uint32_t diff = rows_dwords(src + c, (size_t)g.cap, n, x0, [&](int r, uint32_t x) {
                    char* dr = out + (size_t)r * d.out_cap + d0 + c;
                    for (int b = 0; b < nb; b++) dr[b] = (char)(x >> (8 * b));
                });
                for (int b = 0; b < nb; b++) out[d0 + c + b] = (char)(x0 >> (8 * b));
                for (int b = 0; b < nb; b++) same += !((diff >> (8 * b)) & 0xFFu);
            }
        }
        int tot = 0;
        block_scan_excl(same, &tot, s_scan);
        if (tid == 0) a.sub_res[sp.sub] = make_int2(s_L, tot);
    }
}

// k_fin_prefix: per deferred job (one workgroup of REG_THREADS each), the
// output offset of every region in B (g_dst[reg_off + j ..], R + 1 values;
// the last = B's length, or -1 when a re-alignment overflowed or B would
// not fit) -- once, for all of k_fin_copy's parts (each part scanned every
// region itself: serial in the region count of whole-genome jobs)
__global__ __launch_bounds__(REG_THREADS) void k_fin_prefix(SaArgs a, int* g_dst) {
    __shared__ int scan[REG_THREADS / 64];
    __shared__ int s_bad;
    const int fn = blockIdx.x;
    if (fn >= (int)a.counters[1]) return;
    const int tid = threadIdx.x;
    const int j = a.fin[fn];
    const SaJob job = a.jobs[j];
    const int R = a.job_nreg[j];
    const int4* jr = a.job_regions + job.reg_off;
    int* dst = g_dst + job.reg_off + j;
    if (tid == 0) {
        dst[0] = 0;
        s_bad = 0;
    }
    int carry = 0, bad = 0;
    for (int c0 = 0; c0 < R; c0 += REG_THREADS) {
        const int ri = c0 + tid;
        const int wd = ri < R ? fin_width(a, jr[ri]) : 0;
        bad |= wd < 0;
        int tot = 0;
        const int pre = block_scan_excl(max(wd, 0), &tot, scan);
        if (ri < R) dst[ri + 1] = carry + pre + max(wd, 0);
        carry += tot;
    }
    if (bad) s_bad = 1;
    __syncthreads();
    if (tid == 0) dst[R] = (s_bad || carry > job.cap) ? -1 : carry;  // k_align_finish marks the overflow
}

// k_fin_copy: B of every deferred job, FIN_PARTS workgroups per job, each a
// share of B's columns (the region offsets from k_fin_prefix, into LDS when
// they fit)
__global__ __launch_bounds__(POST_THREADS) void k_fin_copy(SaArgs a, int lds_ints, int* g_dst) {
    extern __shared__ __attribute__((aligned(16))) int dst_l[];
    const int fn = blockIdx.x / FIN_PARTS, part = blockIdx.x % FIN_PARTS;
    if (fn >= (int)a.counters[1]) return;
    const int tid = threadIdx.x;
    const int j = a.fin[fn];
    const SaJob job = a.jobs[j];
    const int n = job.n, cap = job.cap;
    const char* A = (const char*)(a.scratch + job.scratch);
    char* B = (char*)A + (size_t)n * cap;
    const int R = a.job_nreg[j];
    const int4* jr = a.job_regions + job.reg_off;
    const int* gd = g_dst + job.reg_off + j;
    const int tot = gd[R];
    if (tot <= 0) return;
    const int* dst = gd;
    if (R + 1 <= lds_ints) {
        for (int i = tid; i <= R; i += POST_THREADS) dst_l[i] = gd[i];
        __syncthreads();
        dst = dst_l;
    }
    const int c0 = (int)((int64_t)tot * part / FIN_PARTS), c1 = (int)((int64_t)tot * (part + 1) / FIN_PARTS);
    for (int c = c0 + tid; c < c1; c += POST_THREADS) {
        int lo = 0, hi = R - 1;  // the region ri with dst[ri] <= c < dst[ri+1]
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (dst[mid] <= c) lo = mid;
            else hi = mid - 1;
        }
        const int4 rg = jr[lo];
        const int off = c - dst[lo];
        bool from_sub = false;
        const char* sp = A + rg.x + off;
        size_t stride = (size_t)cap;
        if (rg.z <= 0) {
            const int2 res = a.sub_res[-rg.z - 1];
            if (res.y > rg.w) {  // the re-alignment, reversed back
                const SaSub d = a.subs[-rg.z - 1];
                sp = (const char*)(a.pool + d.out_off + 256) + (res.x - 1 - off);
                stride = (size_t)d.out_cap;
                from_sub = true;
            }
        }
        (void)from_sub;
        int r = 0;
        for (; r + 4 <= n; r += 4) {
            const char x0 = sp[(size_t)r * stride], x1 = sp[(size_t)(r + 1) * stride];
            const char x2 = sp[(size_t)(r + 2) * stride], x3 = sp[(size_t)(r + 3) * stride];
            B[(size_t)r * cap + c] = x0;
            B[(size_t)(r + 1) * cap + c] = x1;
            B[(size_t)(r + 2) * cap + c] = x2;
            B[(size_t)(r + 3) * cap + c] = x3;
        }
        for (; r < n; r++) B[(size_t)r * cap + c] = sp[(size_t)r * stride];
    }
}

template <bool LONG, int W>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(W))) void k_align_jobs(SaArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long lds_u64[];
    const int lane = threadIdx.x;
    SlotEnv e = slot_env(a, lds_u64);
    Slot& S = e.S;
    char* stage = e.stage;
    uint32_t lepoch = 0;
    // above every epoch an earlier launch of this batch reached (slot_epoch is
    // zeroed before a batch's first launch)
    uint32_t epoch = next_epoch(a);
    const unsigned int n_jobs = a.n_jobs_dev ? (unsigned)*a.n_jobs_dev : (unsigned)a.n_jobs;

    while (true) {
        unsigned int jn = 0;
        if (lane == 0) jn = atomicAdd(a.next_job, 1u);
        jn = bcast(jn, 0);
        if (jn >= n_jobs) break;
        const int oj = a.order[jn];
        if (oj >= UTWIN_BASE) {
            // the twin of unsplit job tj: process_seqs of the job's rows
            // reversed -- what fix_bad_regions re-aligns when the job's whole
            // alignment is one bad region -- into its own output, beside the
            // job's forward walk.  Twins come first in the queue, so every
            // job that waits for its twin finds it running or done.
            const int tj = oj - UTWIN_BASE;
            const SaJob job = a.jobs[tj];
            WaveCtx w;
            w.lane = lane;
            w.n = job.n;
            w.rowmask = (job.n >= 64) ? ~0ull : ((1ull << job.n) - 1ull);
            w.act = lane < job.n;
            View v{nullptr, 0, 1};
            if (w.act) {
                v.p = a.rows + a.row_off[job.row0 + lane];
                v.len = a.row_len[job.row0 + lane];
            }
            {  // the rows into LDS when they fit (as the job's own walk does)
                int off = 0, tot = 0;
                for (int r = 0; r < job.n; r++) {
                    const int lr = bcast(v.len, r);
                    if (lane == r) off = tot;
                    tot += lr;
                }
                if (tot <= a.stage_bytes) {
                    for (int r = 0; r < job.n; r++) {
                        const char* src = bcast_ptr(v.p, r);
                        const int lr = bcast(v.len, r), o = bcast(off, r);
                        for (int q = lane; q < lr; q += 64) stage[o + q] = src[q];
                    }
                    __syncthreads();
                    if (w.act) v.p = stage + off;
                }
            }
            if (w.act) {  // char(q) = row[len - 1 - q]
                v.p += v.len - 1;
                v.d = -1;
            }
            ProcT<LONG> pr(w, a.P, S, (char*)(a.utw_pool + a.utw_off[tj]), job.cap, epoch, lepoch);
            const int Lc = pr.run(v, 0);
            const bool tovf = any_lane(w, pr.ovf);
            epoch = pr.epoch;
            lepoch = pr.lepoch;
            __threadfence();  // the rows before the state
            if (lane == 0) {
                a.utw_len[tj] = Lc;
                __hip_atomic_store(&a.utw_state[tj], tovf ? 2 : 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            }
            __syncthreads();
            continue;
        }
        // oj < 0: segment task -oj-1 of a split job -- process_seqs of the row
        // suffixes from its sync state into its own output; the wave that
        // finishes the job's last segment goes on with the chained result in A
        const bool chained = oj < 0;
        const int seg_t = -oj - 1;
        SaSeg sg{};
        SaSplit sp{};
        if (chained) {
            sg = a.segs[seg_t];
            sp = a.splits[sg.split];
        }
        const int j = chained ? sp.job : oj;
        const SaJob job = a.jobs[j];
        const int n = job.n;
        if (n == 0) {
            if (lane == 0) {
                a.job_len[j] = 0;
                a.job_status[j] = 0;
            }
            continue;
        }
        const long long t_job = clock64();
        const unsigned long long w_job = wall_clock64();  // constant-rate clock, for timelines
        long long t_ph[3] = {0, 0, 0}, st_prof[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        long long t_regions = 0;
        int st_regions0 = 0;
        int st_calls = 0, st_shifts = 0, st_gaps = 0, st_regions = 0, st_fast = 0;
        WaveCtx w;
        w.lane = lane;
        w.n = n;
        w.rowmask = (n >= 64) ? ~0ull : ((1ull << n) - 1ull);
        w.act = lane < n;
        const int cap = job.cap;
        char* const gA = (char*)(a.scratch + job.scratch);  // the job's global A|B|C
        char* A = gA;
        char* B = A + (size_t)n * cap;
        char* C = B + (size_t)n * cap;
        int sb = a.stage_bytes;  // stage bytes free for segments / region arrays
        bool lds_abc = false;
        const int* T = chained ? a.targets + sp.tgt : nullptr;  // sync state k >= 1 at T[(k-1)*n + row]
        const int start = (chained && sg.k > 0 && w.act) ? T[(sg.k - 1) * n + lane] : 0;
        const bool idle = chained && any_lane(w, start < 0);  // no sync state found
        View v0{nullptr, 0, 1};
        if (w.act) {
            v0.p = (chained && sp.sub == -2 ? a.twin_rows + a.twin_off[job.row0 + lane]
                                            : a.rows + a.row_off[job.row0 + lane]) + start;
            v0.len = a.row_len[job.row0 + lane] - start;
        }
        if (a.aligner_type == 0 && !idle) {
            // the rows into LDS when they fit: every char(q) of the greedy walk
            // is then an LDS read instead of a global one
            int off = 0, tot = 0;
            for (int r = 0; r < n; r++) {
                const int lr = bcast(v0.len, r);
                if (lane == r) off = tot;
                tot += lr;
            }
            // short jobs (no deferred sub-jobs) also keep A|B|C in LDS, at the
            // end of the stage: the walk's writes and fix_bad_regions /
            // realing_end / remove_gaps then never leave the CU; the result is
            // copied to the global A or B at the end
            const int abc = 3 * n * cap;
            const bool may_defer = a.defer != 0 && cap >= a.defer && n >= a.defer_rows;
            if (!chained && !may_defer && ((tot + 15) & ~15) + abc <= a.stage_bytes) {
                lds_abc = true;
                sb = (a.stage_bytes - abc) & ~15;
                A = stage + sb;
                B = A + (size_t)n * cap;
                C = B + (size_t)n * cap;
            }
            if (tot <= sb) {
                // four rows at a time, so that their loads are in flight
                // together (one row at a time cost a global round trip per
                // row before the walk could start)
                for (int r0 = 0; r0 < n; r0 += 4) {
                    const char* s4[4];
                    int l4[4], o4[4], lmax = 0;
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const int r = min(r0 + k, n - 1);
                        s4[k] = bcast_ptr(v0.p, r);
                        l4[k] = r0 + k < n ? bcast(v0.len, r) : 0;
                        o4[k] = bcast(off, r);
                        lmax = max(lmax, l4[k]);
                    }
                    for (int base = 0; base < lmax; base += 64 * 4) {
                        char x[4][4];
#pragma unroll
                        for (int k = 0; k < 4; k++)
#pragma unroll
                            for (int u = 0; u < 4; u++) {
                                const int q = base + u * 64 + lane;
                                x[k][u] = q < l4[k] ? s4[k][q] : 0;
                            }
#pragma unroll
                        for (int k = 0; k < 4; k++)
#pragma unroll
                            for (int u = 0; u < 4; u++) {
                                const int q = base + u * 64 + lane;
                                if (q < l4[k]) stage[o4[k] + q] = x[k][u];
                            }
                    }
                }
                __syncthreads();
                if (w.act) v0.p = stage + off;
            }
        }
        bool deferred = false, ovf = false;
        int L = 0;
        if (a.aligner_type == 1) {
            // DummyAligner: pad to the longest row
            const int m = wave_max(v0.len);
            if (m > cap) ovf = true;
            else if (w.act) {
                char* b = B + (size_t)lane * cap;
                for (int q = 0; q < v0.len; q++) b[q] = v0.p[q];
                for (int q = v0.len; q < m; q++) b[q] = '-';
            }
            L = m;
        } else {
            // 1. process_seqs
            // one Proc for every process_seqs call of the job (state is per call)
            ProcT<LONG> pr(w, a.P, S, chained ? (char*)(a.seg_pool + sg.out) : A, chained ? sg.cap : cap, epoch, lepoch);
            long long t0 = clock64();
            int L0 = 0;
            if (!idle) {
                if (chained) pr.set_targets(T, sg.k, sp.K - 1, start);
                L0 = pr.run(v0, 0);
                ovf = any_lane(w, pr.ovf);
            }
            if (chained) {  // the segment's result; k_split_post chains the job's segments
                if (lane == 0) {
                    a.seg_res[seg_t] = idle ? make_int4(-1, 0, 0, 0)
                                            : make_int4(pr.stop ? pr.tm + 1 : sp.K, L0, ovf ? 1 : 0, 0);
                    if (a.job_stats) {
                        a.seg_wall[2 * seg_t] = (int64_t)w_job;
                        a.seg_wall[2 * seg_t + 1] = (int64_t)wall_clock64();
                    }
                }
                epoch = pr.epoch;
                lepoch = pr.lepoch;
                continue;
            }
            t_ph[0] = clock64() - t0;
            t0 = clock64();

            __syncthreads();
            if (!ovf) {
                // 2. fix_bad_regions
                int4 rreg = make_int4(0, 0, 0, 0);
                unsigned long long gmask = 0;
                const long long t_reg0 = clock64();
                // 64 ints of scratch: the row stage (its rows are dead after
                // process_seqs) when it has room, else the slot's global area
                int* rtmp = sb >= 256 ? (int*)stage : (int*)S.good_col;
                int R = regions_in_registers(w, A, cap, L0, a.P.wf, a.P.min_length, rreg, gmask, rtmp);
                const bool fast = R >= 0;
                bool counted = false;  // S.regions[].w holds each region's identical columns
                if (!fast) {
                    R = regions_in_lds(w, A, cap, L0, a.P.wf, a.P.min_length, stage, sb, S.regions);
                    counted = R >= 0;
                    if (R < 0) {
                        count_equal_cols(w, A, cap, 0, L0, S.good_col);
                        __syncthreads();
                        R = make_regions(w, S.good_col, L0, a.P.wf, S.regions);
                        st_regions0 = R;
                        R = reduce_regions(w, S.regions, R, a.P.min_length);
                    }
                }
                t_regions = clock64() - t_reg0;
                st_regions = R;
                int colB = 0;
                // the whole alignment one bad region and a twin walked the
                // reversed rows: its result is the re-alignment
                bool tw_ok = false;
                if (a.utw_state && R == 1 && a.utw_off[j] >= 0) tw_ok = !(fast ? bcast(rreg.z, 0) : S.regions[0].z);
                if (a.defer && L0 >= a.defer && n >= a.defer_rows && !(fast && R == 1 && bcast(rreg.z, 0)) && !tw_ok)
                    deferred = defer_regions(DeferOut{a.job_regions, a.job_nreg, a.subs, a.alloc, a.counters,
                                                      a.pool, a.pool_cap, a.max_sub, a.fin},
                                             n, j, job.reg_off, job.reg_cap, A, C, cap, R, fast, counted, rreg,
                                             gmask, S.regions, S.good_col);
                if (deferred) {
                    L = L0;
                    R = 0;
                } else if (fast && R == 1 && bcast(rreg.z, 0)) {  // one good region: the alignment stays in A
                    B = A;
                    colB = L0;
                    R = 0;
                }
                pr.ob = B;
                for (int ri = 0; ri < R && !ovf; ri++) {
                    const int4 rg = fast ? make_int4(bcast(rreg.x, ri), bcast(rreg.y, ri), bcast(rreg.z, ri),
                                                     bcast(rreg.w, ri))
                                         : S.regions[ri];
                    const int len = rg.y - rg.x + 1;
                    if (colB + len > cap) {
                        ovf = true;
                        break;
                    }
                    if (rg.z) {
                        cm_copy(w, A, B, cap, rg.x, colB, len);
                        colB += len;
                        continue;
                    }
                    int before = 0;
                    if (fast) {
                        const int lo = lane * 64, hi = lo + 63;
                        if (lo <= rg.y && hi >= rg.x) {
                            const int a0 = max(rg.x, lo) - lo, a1 = min(rg.y, hi) - lo;
                            const unsigned long long m =
                                (a1 == 63 ? ~0ull : ((1ull << (a1 + 1)) - 1)) & (~0ull << a0);
                            before = __popcll(gmask & m);
                        }
                        before = wave_sum(before);
                    } else if (counted) {
                        before = rg.w;
                    } else {
                        for (int c = rg.x + lane; c <= rg.y; c += 64) before += S.good_col[c];
                        before = wave_sum(before);
                    }
                    if (tw_ok) {  // (R == 1: the region is every column, colB = 0)
                        int ts;
                        while ((ts = __hip_atomic_load(&a.utw_state[j], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) == 0)
                            __builtin_amdgcn_s_sleep(8);
                        if (ts != 1) {  // the twin overflowed where this walk would have
                            ovf = true;
                            break;
                        }
                        const int Lc = __hip_atomic_load(&a.utw_len[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const char* tw = (const char*)(a.utw_pool + a.utw_off[j]);
                        const int after = count_equal_cols(w, tw, cap, 0, Lc, nullptr);
                        __syncthreads();
                        if (after > before) {
                            cm_copy_rev(w, tw, B, cap, colB, Lc);
                            colB += Lc;
                        } else {
                            cm_copy(w, A, B, cap, rg.x, colB, len);
                            colB += len;
                        }
                        __syncthreads();
                        continue;
                    }
                    const View cv = stage_segment(w, A, cap, C, stage, sb, rg.x, rg.y + 1);
                    const int Lc = pr.run(cv, colB);
                    if (any_lane(w, pr.ovf)) {
                        ovf = true;
                        break;
                    }
                    __syncthreads();
                    const int after = count_equal_cols(w, B, cap, colB, colB + Lc, nullptr);
                    __syncthreads();
                    if (after > before) {
                        cm_reverse(w, B, cap, colB, colB + Lc);
                        colB += Lc;
                    } else {
                        cm_copy(w, A, B, cap, rg.x, colB, len);
                        colB += len;
                    }
                    __syncthreads();
                }
                // 3. realing_end
                t_ph[1] = clock64() - t0;
                t0 = clock64();
                if (!deferred) L = colB;
                int prefix = L - a.P.ac;
                if (prefix < 1) prefix = 1;
                if (!deferred && !ovf && L >= 2 && !tail_identical(w, B, cap, prefix, L)) {
                    const View tv = stage_segment(w, B, cap, C, stage, sb, prefix, L);
                    const int Lt = pr.run(tv, prefix);
                    if (any_lane(w, pr.ovf)) ovf = true;
                    else {
                        cm_reverse(w, B, cap, prefix, prefix + Lt);
                        L = prefix + Lt;
                    }
                }
                t_ph[2] = clock64() - t0;
            }
#ifdef NPGX_SA_PROFILE
            for (int q = 0; q < 10; q++) st_prof[q] = pr.prof[q];
#endif
            st_calls = pr.n_aligned_calls;
            st_shifts = pr.n_shifts;
            st_gaps = pr.n_gaps;
            st_fast = pr.n_fast;
            epoch = pr.epoch;
            lepoch = pr.lepoch;
        }
        __syncthreads();
        // 4. remove pure-gap columns (AbstractAligner::remove_gaps): the
        // similar aligner's alignments have none -- every column of
        // process_seqs holds a letter (append_cols, apply_gap's shifted rows,
        // the longest tail of append_all / append_end), and fix_bad_regions /
        // realing_end only concatenate such columns -- so only the dummy
        // aligner (whose input rows may hold gaps) needs the pass
        if (!ovf && !deferred && a.aligner_type == 1) L = remove_pure_gap_cols(w, B, cap, L);
        if (lds_abc && !ovf) {  // the result to where the host reads it (A for status 2, else B)
            __syncthreads();
            char* dst = gA + (B == A ? 0 : (size_t)n * cap);
            for (int r = 0; r < n; r++)
                for (int c = lane; c < L; c += 64) dst[(size_t)r * cap + c] = B[(size_t)r * cap + c];
            __syncthreads();
        }
        if (lane == 0) {
            a.job_len[j] = ovf ? -30 : L;
            a.job_status[j] = ovf ? 1 : deferred ? 3 : (B == A ? 2 : 0);  // 2: the rows are in A, 3: deferred
        }
        if (lane == 0 && a.job_stats) {  // only when the statistics are wanted
            int64_t* js = a.job_stats + (size_t)j * NPGX_JOB_STATS;
            const int64_t w0 = (int64_t)w_job;
            js[0] = clock64() - t_job;
            js[1] = L;
            js[2] = st_calls;
            js[3] = st_shifts;
            js[4] = st_gaps;
            js[5] = st_regions;
            js[6] = n;
            js[7] = (int64_t)(st_fast);
            js[8] = t_ph[0];
            js[9] = t_ph[1];
            js[10] = t_ph[2];
            js[11] = w0;
            for (int q = 0; q < 10; q++) js[12 + q] = st_prof[q];
            js[22] = t_regions;
            js[23] = (int64_t)wall_clock64();
        }
        __syncthreads();
    }
    if (lane == 0) atomicMax(a.slot_epoch, epoch);  // the launch's highest epoch
}

// the reversed copies of the twin jobs' rows (list: their rows' indices)
__global__ void k_twin_rows(const char* __restrict__ rows, const int64_t* __restrict__ row_off,
                            const int32_t* __restrict__ row_len, const int32_t* __restrict__ list, int n,
                            const int64_t* __restrict__ twin_off, char* __restrict__ out) {
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        const int r = list[i];
        const char* src = rows + row_off[r];
        const int L = row_len[r];
        char* d = out + twin_off[r];
        for (int c = threadIdx.x; c < L; c += blockDim.x) d[c] = src[L - 1 - c];
    }
}

struct GatherRow {
    int64_t out_off;    // output byte offset
    int64_t src;        // device address of the aligned row (0: empty row -> gaps)
    int32_t len;        // job alignment length
    int32_t pad;
};

__global__ void k_gather_rows(const GatherRow* rows, int64_t n, char* out) {
    const int64_t r = blockIdx.x;
    if (r >= n) return;
    const GatherRow g = rows[r];
    char* d = out + g.out_off;
    if (g.src == 0) {
        for (int c = threadIdx.x; c < g.len; c += blockDim.x) d[c] = '-';
    } else {
        const char* s = (const char*)(uintptr_t)g.src;
        for (int c = threadIdx.x; c < g.len; c += blockDim.x) d[c] = s[c];
    }
}

// A batch's small host->device arrays and zeroed counters in one upload: the
// arrays are staged back to back after a table of these ops, copied in one
// hipMemcpy and scattered by one launch (instead of ~10 copies and 4 fills,
// each a serialized dispatch of ~8 us, per aligner batch)
struct ScatterOp {
    void* dst;
    int64_t src;    // byte offset in the blob; < 0: zero fill
    int64_t bytes;
};

__global__ void k_scatter(const unsigned char* __restrict__ blob, int n_ops) {
    const ScatterOp op = ((const ScatterOp*)blob)[blockIdx.x];
    const int64_t t = (int64_t)blockIdx.y * blockDim.x + threadIdx.x, step = (int64_t)gridDim.y * blockDim.x;
    if (op.bytes % 4 == 0 && ((uintptr_t)op.dst & 3) == 0) {
        uint32_t* d = (uint32_t*)op.dst;
        const uint32_t* sp = (const uint32_t*)(blob + (op.src < 0 ? 0 : op.src));
        for (int64_t i = t; i < op.bytes / 4; i += step) d[i] = op.src < 0 ? 0u : sp[i];
    } else {
        unsigned char* d = (unsigned char*)op.dst;
        for (int64_t i = t; i < op.bytes; i += step) d[i] = op.src < 0 ? 0 : blob[op.src + i];
    }
}

// align_device's async mode: the jobs the first attempt overflowed (status
// 1) listed for the re-run at the proven bound
__global__ void k_retry_list(const int32_t* __restrict__ status, int32_t n, int32_t* __restrict__ order,
                             int32_t* __restrict__ count, uint8_t* __restrict__ retried) {
    const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const bool r = status[j] == 1;
    retried[j] = r;
    if (r) order[atomicAdd(count, 1)] = j;
}
// ... and every job's rows (B of its A|B|C scratch, or A for status 2) from
// the attempt that finished it
__global__ void k_job_rows(const SaJob* __restrict__ jobs0, const SaJob* __restrict__ jobs1,
                           const uint8_t* __restrict__ retried, const int32_t* __restrict__ status,
                           const int32_t* __restrict__ len, int32_t n, const unsigned char* scratch0,
                           const unsigned char* scratch1, JobRows* __restrict__ out, int32_t* __restrict__ err) {
    const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const bool r = retried[j];
    const SaJob J = r ? jobs1[j] : jobs0[j];
    const int32_t st = status[j];
    if (st != 0 && st != 2) atomicOr(err, 1);
    out[j] = JobRows{(const char*)((r ? scratch1 : scratch0) + J.scratch + (st == 2 ? 0 : (int64_t)J.n * J.cap)),
                     J.cap, len[j]};
}

int weight_factor(int64_t min_identity_x1e4) {
    // FindLowSimilar::get_weight_factor with Decimal arithmetic (Decimal.hpp)
    int64_t mi = std::min<int64_t>(min_identity_x1e4, 9900);
    const int64_t one = 10000;
    const int64_t q = one * 10000 / (one - mi);          // Decimal division
    const int64_t ip = q / 10000, fr = q % 10000;       // q > 0
    return (int)(fr < 5000 ? ip : ip + 1);               // Decimal::round
}

}  // namespace npgx

using namespace npgx;

struct npgx_aligner {
    npgx_align_options opt;
    int device = 0;
    hipStream_t stream = nullptr;
    // align_device's host arrays (kept for their capacity)
    std::vector<npgx::SaJob> h_jobs;
    std::vector<int64_t> h_ne_off;
    std::vector<int32_t> h_ne_len, h_order, h_jlen, h_jstat;
    std::vector<double> h_cost;
    std::vector<int32_t> h_jsum;
    std::vector<uint8_t> h_cls;
    DevBuf<char> d_rows;
    DevBuf<int64_t> d_row_off;
    DevBuf<int32_t> d_row_len;
    DevBuf<SaJob> d_jobs;
    // per job: length | status, then the launch's highest word-table epoch --
    // one array, so the results come back in one copy
    DevBuf<int32_t> d_order, d_job_out;
    DevBuf<int64_t> d_job_stats;
    std::vector<int64_t> job_stats;
    DevBuf<unsigned int> d_next;
    DevBuf<unsigned char> d_scratch, d_scratch2;
    double host_ms[2] = {0, 0};  // align_device: host preparation, kernel wait
    PinnedArena pinned;          // staging of the batch's host<->device copies
    DevBuf<unsigned long long> tkeys, tmask;
    DevBuf<uint32_t> tdone;
    size_t tcap_alloc = 0;
    uint32_t epoch_base = 1;  // first word-table epoch of the next launch
    DevBuf<const char*> st_p;
    DevBuf<int> st_len, st_pos, st_col;
    DevBuf<int4> regions;
    DevBuf<unsigned char> good_col;
    DevBuf<GatherRow> d_gather;
    DevBuf<char> d_out;
    // deferred fix_bad_regions (first attempt)
    // NPGX_ALIGN_DEFER=<columns>: alignments at least this long hand their bad
    // regions to k_align_sub (0: every bad region realigned inside its job)
    // deferred bad regions (sub-jobs of their own): alignments of at least
    // this many columns and rows -- with long jobs split into segments the
    // unsplit many-row jobs of a few hundred columns became a launch's tail
    // (their bad regions re-aligned one after the other by one wave): C3
    // align 19.3 -> 18.6 ms at 500 vs 8000 columns (tools/gpu_defer_sweep.sh);
    // 3-row ones only pay the extra launches (defer_rows)
    int defer = 500;
    int defer_rows = 4;
    DevBuf<int4> d_job_regions;
    DevBuf<int32_t> d_job_nreg, d_fin;
    DevBuf<SaSub> d_subs;
    DevBuf<int2> d_sub_res;
    DevBuf<unsigned long long> d_alloc;
    DevBuf<unsigned int> d_counters;
    DevBuf<unsigned char> d_pool;
    // long jobs split into segments (k_split_find, run_segment): jobs of at
    // least two rows are cut every `split` columns of their longest row
    // (NPGX_ALIGN_SPLIT; 0: never)
    int split = 384;
    // try_aligned's word search: the first `long_head` shifts incrementally,
    // then whole prefixes from `long_m` shifts on (find_word_long,
    // sa_device.hpp; NPGX_LONG_HEAD / NPGX_LONG_M; long_head 0: incremental
    // only, the round-4 search)
    int long_head = 128;
    int long_m = 512;
    int long_lds = 1;  // NPGX_LONG_LDS=0: the prefix search on the global word table only (A/B)
    int64_t waves_many_at = SA_WAVES_MANY_AT;  // NPGX_SA_MANY_AT: tasks past which a launch takes 4 waves a SIMD (A/B)
    // split jobs whose segment rooms for the whole row suffixes take at most
    // this many bytes get them (NPGX_SEG_FULL_MB; 0: the 8-sync-state rooms).
    // R3: the segment overflows (reason 202) go with them; the sub-job
    // overflows that were left (reason 10, gpurun_out/r05m) re-run in the
    // sub-job retry launch
    int64_t seg_full_bytes = 64ll << 20;
    // twins of the split jobs (NPGX_TWINS: 0 never -- the default: measured at
    // C3 and C5 the whole-job bad region they serve is rare among split jobs
    // and their segments slow the launch -- 1 always, -1 in launches with few
    // tasks): see "Twins" at align_device
    int twins = 0;
    // unsplit twins (see "Unsplit twins" at align_device): jobs of at least
    // utw_rows rows (0: none; NPGX_UTWINS), while the launch stays within
    // utw_max_tasks tasks (NPGX_UTWIN_TASKS)
    // (C3 kernel traces, gpurun_out/r06e: with twins in a launch of 1020
    // jobs its k_align_jobs went 363 -> 547 us -- twice the waves, half the
    // LDS each -- while launches of 154-386 jobs gained up to a fifth: twins
    // only while the launch keeps to about one wave per SIMD)
    int utw_rows = 3;
    int utw_max_tasks = 512;
    std::vector<int64_t> h_utw_off;
    std::vector<int32_t> h_utw_q;
    DevBuf<unsigned char> d_utw_pool;
    DevBuf<int64_t> d_utw_off;
    DevBuf<int32_t> d_utw_st;
    std::vector<int64_t> h_twin_off;
    std::vector<int32_t> h_twin_list;
    DevBuf<char> d_twin;
    DevBuf<int64_t> d_twin_off;
    DevBuf<int32_t> d_twin_list;
    // bytes the per-slot scratch of one launch may take (NPGX_SLOT_BUDGET_MB;
    // default 16 GiB: allocating much more costs seconds on first use)
    int64_t slot_budget = 0;
    std::vector<SaSplit> h_splits;
    std::vector<SaSeg> h_segs;
    std::vector<int2> h_ftasks;
    std::vector<int32_t> h_queue, h_jmax;
    DevBuf<SaSplit> d_splits;
    DevBuf<unsigned char> d_post;  // k_split_post's global work areas
    DevBuf<int4> d_chain, d_chain_hdr;
    DevBuf<unsigned long long> d_chain_bits;
    DevBuf<int64_t> d_bits_off;
    DevBuf<int32_t> d_part0;
    std::vector<int64_t> h_bits_off;
    std::vector<int32_t> h_part0;
    DevBuf<SaSeg> d_segs;
    DevBuf<int2> d_ftasks;
    DevBuf<int32_t> d_targets;
    DevBuf<int4> d_seg_res;
    DevBuf<int64_t> d_seg_wall;
    DevBuf<int64_t> d_sub_wall;
    DevBuf<int32_t> d_qseg, d_qsub;
    DevBuf<unsigned int> d_sctr;
    DevBuf<unsigned char> d_seg_pool;
    DevBuf<int> d_reg_dst;  // k_fin_copy's region offsets when they do not fit its LDS
    DevBuf<int32_t> d_rq;   // k_align_sub's retry launch: failed sub-jobs
    // last result
    std::vector<char> out;
    std::vector<int64_t> out_off;
    std::vector<int64_t> job_len;
    bool has_result = false;
    bool want_stats = false;  // per-job statistics copied back (NPGX_JOB_STATS=1)
    StageTimer timer;
    WideBufs* wide = nullptr;  // problems of more than 64 rows (wide_aligner.hip)
    // the batch's small uploads and zeroed counters, scattered by one launch
    std::vector<npgx::ScatterOp> h_ops;
    std::vector<unsigned char> h_blob;
    DevBuf<unsigned char> d_blob;
    // async mode (AlignAsync): the re-run's jobs, list, counters, flags
    std::vector<npgx::SaJob> h_jobs1;
    DevBuf<SaJob> d_jobs1;
    DevBuf<int32_t> d_order1, d_ctr1;
    DevBuf<uint8_t> d_retried;
};

namespace npgx {

// Device-resident batch: row r of the batch is d_rows[row_off[r] .. +row_len[r])
// (host arrays describing device memory).  Results stay on the device: job j's
// non-empty row k is at res.bptr[j] + k*res.cap[j] for res.len[j] columns.
void align_device(npgx_aligner* al, const char* d_rows, const int64_t* row_off, const int32_t* row_len,
                  const int32_t* job_row_start, int32_t n_jobs, AlignResult& res, const AlignAsync* as) {
    NPGX_HIP(hipSetDevice(al->device));

    auto tp = std::chrono::steady_clock::now();
    auto ms = [](std::chrono::steady_clock::time_point t) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    };
    hipStream_t st = al->stream;
    const npgx_align_options& o = al->opt;
    NPGX_REQUIRE(n_jobs >= 0, NPGX_ERR_ARG, "n_jobs < 0");
    const int2* uj = as ? as->ujobs : nullptr;  // uniform jobs: no host row arrays
    const int64_t r_base = (n_jobs && !uj) ? job_row_start[0] : 0;
    const int64_t n_rows = (n_jobs && !uj) ? (int64_t)job_row_start[n_jobs] - r_base : 0;
    // host arrays kept in the handle across calls (capacity reused)
    std::vector<SaJob>& jobs = al->h_jobs;
    std::vector<int64_t>& ne_off = al->h_ne_off;
    std::vector<int32_t>& ne_len = al->h_ne_len;
    jobs.resize(n_jobs);
    ne_off.clear();
    ne_len.clear();
    if (!uj) res.row_ne.assign((size_t)std::max<int64_t>(n_rows, 1), -1);
    int64_t u_rows = 0;  // (uniform jobs: rows so far)
    std::vector<double>& cost = al->h_cost;
    cost.resize(n_jobs);
    std::vector<int32_t>& jsum = al->h_jsum;  // residues per job
    jsum.resize(n_jobs);
    std::vector<int32_t>& jmax = al->h_jmax;  // longest row per job
    jmax.resize(n_jobs);
    int64_t scratch = 0, n_reg = 0, n_sub_max = 0;
    int max_n = 1, max_len = 1, max_cap = 1;
    std::vector<WideJobIn> wide_in;
    std::vector<int32_t> wide_idx;
    const int wf = weight_factor(o.min_identity_x1e4);
    // after reduce_regions every region but a lone one weighs >= min_length:
    // at least this many columns wide
    const int min_width = std::max(1, std::min(o.min_length, (o.min_length + wf - 1) / std::max(wf, 1)));
    for (int32_t j = 0; j < n_jobs; j++) {
        SaJob& J = jobs[j];
        int n = 0;
        int64_t sum = 0;
        int mx = 0;
        if (uj) {
            const int2 q = uj[j];
            NPGX_REQUIRE(q.x >= 0 && q.x <= 64 && q.y > 0 && q.y < (1 << 30), NPGX_ERR_RANGE, "uniform job out of range");
            J.row0 = u_rows;
            u_rows += q.x;
            n = q.x;
            sum = (int64_t)q.x * q.y;
            mx = q.x ? q.y : 0;
        }
        const int64_t r0 = uj ? 0 : job_row_start[j], r1 = uj ? 0 : job_row_start[j + 1];
        NPGX_REQUIRE(r1 >= r0, NPGX_ERR_ARG, "job_row_start not monotone");
        if (!uj) J.row0 = (int64_t)ne_len.size();
        for (int64_t r = r0; r < r1; r++) {
            const int64_t len = row_len[r];
            NPGX_REQUIRE(len >= 0 && len < (1ll << 30), NPGX_ERR_RANGE, "row length out of range");
            if (len == 0) continue;
            res.row_ne[(size_t)(r - r_base)] = (int64_t)ne_len.size() - J.row0;
            ne_off.push_back(row_off[r]);
            ne_len.push_back((int32_t)len);
            n++;
            sum += len;
            mx = std::max<int>(mx, (int)len);
        }
        J.n = n;
        if (n > 64) {  // a wide problem: one workgroup of its own (wide_aligner.hip)
            wide_in.push_back(WideJobIn{J.row0, n, 0});
            wide_idx.push_back(j);
            J.cap = 0;
            J.scratch = 0;
            J.reg_off = 0;
            J.reg_cap = 0;
            J.pad = 0;
            cost[j] = 0;
            jsum[j] = (int32_t)std::min<int64_t>(sum, INT32_MAX);
            jmax[j] = mx;
            continue;
        }
        // first attempt: 2*max+64 columns (the proven bound is the sum of lengths)
        int64_t cap = std::min<int64_t>(sum, 2ll * mx + 64);
        if (o.aligner_type == 1) cap = mx;
        J.cap = (int32_t)((std::max<int64_t>(cap, 1) + 15) & ~15ll);
        J.scratch = scratch;
        scratch += (3ll * n * J.cap + 255) & ~255ll;
        J.reg_off = n_reg;
        J.reg_cap = n > 1 ? std::min(J.cap + 1, J.cap / min_width + 2) : 0;
        J.pad = 0;
        n_reg += J.reg_cap;
        n_sub_max += (J.reg_cap + 1) / 2;
        cost[j] = double(n) * double(sum);
        jsum[j] = (int32_t)std::min<int64_t>(sum, INT32_MAX);
        jmax[j] = mx;
        max_n = std::max(max_n, n);
        max_len = std::max(max_len, mx);
        max_cap = std::max<int>(max_cap, J.cap);
    }
    static const bool pdbg = getenv("NPGX_PREP_DEBUG") != nullptr;  // host phase times to stderr
    double pt[12] = {0};
    auto pt0 = tp;  // (phase 0: the per-job loop above)
    auto pmark = [&](int i) {
        if (!pdbg) return;
        pt[i] += ms(pt0);
        pt0 = std::chrono::steady_clock::now();
    };
    pmark(0);
    // heaviest first (rows x residues), by power-of-two cost classes: the order
    // only balances the load, results do not depend on it
    std::vector<int32_t>& order = al->h_order;
    order.resize(n_jobs);
    {
        int cnt[65] = {0};
        std::vector<uint8_t>& cls = al->h_cls;
        cls.resize(n_jobs);
        for (int32_t j = 0; j < n_jobs; j++) {
            const uint64_t c = (uint64_t)cost[j];
            cls[j] = (uint8_t)(c ? 64 - __builtin_clzll(c) : 0);  // 0..64
            cnt[cls[j]]++;
        }
        int at[65];
        int acc = 0;
        for (int c = 64; c >= 0; c--) {
            at[c] = acc;
            acc += cnt[c];
        }
        for (int32_t j = 0; j < n_jobs; j++) order[at[cls[j]]++] = j;
        if (!wide_idx.empty()) {  // the wide problems are not in the batched queue
            std::vector<uint8_t> is_wide(n_jobs, 0);
            for (int32_t j : wide_idx) is_wide[j] = 1;
            order.erase(std::remove_if(order.begin(), order.end(), [&](int32_t j) { return is_wide[j] != 0; }),
                        order.end());
        }
    }

    pmark(1);
    al->d_row_off.ensure(ne_off.size());
    al->d_row_len.ensure(ne_len.size());
    al->d_jobs.ensure(jobs.size());
    al->d_order.ensure(order.size());
    al->d_job_out.ensure(2 * jobs.size() + 1);
    int32_t* const d_job_len = al->d_job_out.p;
    int32_t* const d_job_status = d_job_len + jobs.size();
    uint32_t* const d_slot_epoch = (uint32_t*)(d_job_status + jobs.size());
    al->d_job_stats.ensure(jobs.size() * NPGX_JOB_STATS);
    al->job_stats.assign(al->want_stats ? jobs.size() * NPGX_JOB_STATS : 0, 0);
    al->d_next.ensure(1);
    // uploads and zeroings are collected and issued together by flush() before
    // the next launch (one copy + one k_scatter)
    al->h_ops.clear();
    al->h_blob.clear();
    auto put = [&](void* d, const void* h, size_t bytes) {
        if (!bytes) return;
        const size_t at = (al->h_blob.size() + 15) & ~(size_t)15;
        al->h_blob.resize(at + bytes);
        memcpy(al->h_blob.data() + at, h, bytes);
        al->h_ops.push_back(ScatterOp{d, (int64_t)at, (int64_t)bytes});
    };
    auto zero = [&](void* d, size_t bytes) { al->h_ops.push_back(ScatterOp{d, -1, (int64_t)bytes}); };
    // k_align_jobs / k_align_sub in the form of the set (long head or not) and
    // of the launch's waves a SIMD
    typedef void (*SaKernel)(SaArgs);
    auto launch_sa = [&](SaKernel lf, SaKernel sf, SaKernel lm, SaKernel sm, int wv, size_t g, size_t lds,
                         const SaArgs& X) {
        const bool lh = al->long_head > 0, many = wv == SA_WAVES_MANY;
        hipLaunchKernelGGL(lh ? (many ? lm : lf) : (many ? sm : sf), dim3((unsigned)g), dim3(64), lds, st, X);
    };
    auto flush = [&]() {
        if (al->h_ops.empty()) return;
        const size_t nop = al->h_ops.size(), head = (nop * sizeof(ScatterOp) + 15) & ~(size_t)15;
        for (ScatterOp& op : al->h_ops)
            if (op.src >= 0) op.src += (int64_t)head;
        const size_t total = head + al->h_blob.size();
        char* p = al->pinned.take(total, st);
        memcpy(p, al->h_ops.data(), nop * sizeof(ScatterOp));
        memcpy(p + head, al->h_blob.data(), al->h_blob.size());
        al->d_blob.ensure(total);
        NPGX_HIP(hipMemcpyAsync(al->d_blob.p, p, total, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_scatter, dim3((unsigned)nop, 16), dim3(256), 0, st, al->d_blob.p, (int)nop);
        NPGX_HIP(hipGetLastError());
        al->h_ops.clear();
        al->h_blob.clear();
    };
    if (!uj) {
        put(al->d_row_off.p, ne_off.data(), ne_off.size() * 8);
        put(al->d_row_len.p, ne_len.data(), ne_len.size() * 4);
    }
    const int64_t* const d_roff = uj ? as->d_row_off : al->d_row_off.p;
    const int32_t* const d_rlen = uj ? as->d_row_len : al->d_row_len.p;
    // row i of job j's letters (host)
    auto row_len_at = [&](int32_t j, int i) -> int32_t { return uj ? uj[j].y : ne_len[jobs[j].row0 + i]; };
    Params P{o.mismatch_check, o.gap_check, o.aligned_check, o.min_length, wf, al->long_head, al->long_m, al->long_lds};

    std::vector<int32_t>& jlen = al->h_jlen;
    std::vector<int32_t>& jstat = al->h_jstat;
    jlen.resize(n_jobs);
    jstat.resize(n_jobs);
    std::vector<int64_t> jst(al->want_stats ? (size_t)n_jobs * NPGX_JOB_STATS : 0);
    res.len.assign(n_jobs, 0);
    res.cap.assign(n_jobs, 0);
    res.n.assign(n_jobs, 0);
    res.bptr.assign(n_jobs, nullptr);
    for (int32_t j = 0; j < n_jobs; j++) res.n[j] = jobs[j].n;
    std::vector<int32_t> todo = order;
    // async mode: the re-run at the proven bound is planned now for every job
    // (the device picks the ones that overflow), and the first attempt's
    // buffers are sized to hold it too (nothing may be reallocated under the
    // kernels in flight)
    int64_t scratch1 = 0;
    uint32_t tlog1 = 10;
    int depth1 = 4, cols1 = 256;
    size_t slots1 = 1;
    if (as) {
        NPGX_REQUIRE(wide_idx.empty(), NPGX_ERR_ARG, "align_device async: problems of more than 64 rows");
        std::vector<SaJob>& j1 = al->h_jobs1;
        j1 = jobs;
        int mn = 1, ml = 1, mc = 1;
        for (int32_t j : order) {
            SaJob& J = j1[j];
            int64_t sum = 0;
            for (int i = 0; i < J.n; i++) sum += row_len_at(j, i);
            J.cap = (int32_t)((std::max<int64_t>(sum, 1) + 15) & ~15ll);
            J.scratch = scratch1;
            scratch1 += (3ll * J.n * J.cap + 255) & ~255ll;
            mn = std::max(mn, J.n);
            ml = std::max(ml, jmax[j]);
            mc = std::max(mc, J.cap);
        }
        while ((1ull << tlog1) < 2ull * (uint64_t)mn * (uint64_t)(ml + 1) + 64) tlog1++;
        depth1 = ml / std::max(1, o.aligned_check + 1) + 4;
        cols1 = std::max(256, mc + 1);
        const int64_t per1 = (20ll << tlog1) + 1028ll * depth1 + 17ll * cols1;
        slots1 = (size_t)std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>((int64_t)order.size(), 256),
                                                                 std::max<int64_t>(al->slot_budget, 1ll << 22) / per1));
        al->d_scratch2.grow((size_t)std::max<int64_t>(scratch1, 256));
        al->d_jobs1.ensure(jobs.size());
        al->d_order1.ensure(std::max<size_t>(jobs.size(), 1));
        al->d_ctr1.ensure(2);
        al->d_retried.ensure(std::max<size_t>(jobs.size(), 1));
    }
    // NPGX_RETRY_DEBUG: the re-run jobs (rows, longest row, residues, first
    // room, split or not, final length) to stderr
    static const bool rdbg = getenv("NPGX_RETRY_DEBUG") != nullptr;
    std::vector<int32_t> dbg_cap0;
    std::vector<uint8_t> dbg_split;
    std::vector<int32_t> dbg_why;  // attempt 0's overflow reason (-job_len)
    for (int attempt = 0; attempt < 2 && !todo.empty(); attempt++) {
        DevBuf<unsigned char>& scr = attempt == 0 ? al->d_scratch : al->d_scratch2;
        if (attempt == 1 && rdbg) {
            dbg_cap0.assign(n_jobs, 0);
            for (int32_t j : todo) dbg_cap0[j] = jobs[j].cap;
        }
        if (attempt == 1) {  // re-run overflowed jobs at the proven bound, in a second scratch
            scratch = 0;
            max_cap = 1;
            max_n = 1;
            max_len = 1;
            for (int32_t j : todo) {
                SaJob& J = jobs[j];
                max_n = std::max(max_n, J.n);
                max_len = std::max(max_len, jmax[j]);
                int64_t sum = 0;
                for (int i = 0; i < J.n; i++) sum += row_len_at(j, i);
                J.cap = (int32_t)((std::max<int64_t>(sum, 1) + 15) & ~15ll);
                J.scratch = scratch;
                scratch += (3ll * J.n * J.cap + 255) & ~255ll;
                max_cap = std::max<int>(max_cap, J.cap);
            }
        }
        pmark(2);
        // the work queue: the segments of the split jobs (heaviest first), then
        // the other jobs
        std::vector<SaSplit>& splits = al->h_splits;
        std::vector<SaSeg>& segs = al->h_segs;
        std::vector<int2>& ftasks = al->h_ftasks;
        std::vector<int32_t>& queue = al->h_queue;
        splits.clear();
        segs.clear();
        ftasks.clear();
        queue.clear();
        int64_t n_tgt = 0, seg_bytes = 0, post_bytes = 0, bits_words = 0;
        std::vector<int64_t>& bits_off = al->h_bits_off;
        std::vector<int32_t>& part0 = al->h_part0;
        bits_off.clear();
        part0.assign(1, 0);
        if (attempt == 0 && o.aligner_type == 0 && al->split > 0) {
            for (int32_t j : todo) {
                const SaJob& J = jobs[j];
                const int mx = jmax[j];
                const int K = std::min(SPLIT_KMAX, mx / split_len_for(al->split, J.n));
                if (J.n < 2 || K < 2 || mx < 4 * SPLIT_W) continue;
                SaSplit sp;
                sp.job = j;
                sp.K = K;
                sp.tgt = n_tgt;
                sp.seg0 = (int32_t)segs.size();
                sp.win = std::min(SPLIT_RMAX, 64 + mx / 128);
                sp.sub = -1;
                sp.twin = 0;
                sp.post = -1;
                {  // a chain that may outgrow k_split_post's LDS: a global work area
                    const int64_t need = (((int64_t)J.cap + 63) / 64) * 8 + 17ll * (J.cap + 1) + 64;
                    if (need > (int64_t)POST_LDS) {
                        sp.post = post_bytes;
                        post_bytes += (need + 255) & ~255ll;
                    }
                    bits_off.push_back(bits_words);  // (unused with a post area)
                    if (sp.post < 0) bits_words += J.cap / 64 + 1;
                    part0.push_back(part0.back() + (J.cap + CHAIN_PART - 1) / CHAIN_PART);
                }
                n_tgt += (int64_t)(K - 1) * J.n;
                // rooms for the whole rest of the rows when that stays within
                // seg_full_bytes for the job: a walk that misses the later
                // sync states (repeat insertions: R3) then still finishes its
                // segment instead of overflowing and re-running the job whole
                int64_t full_bytes = 0;
                for (int k = 0; k < K; k++) full_bytes += (int64_t)J.n * seg_cap_for(mx, k, K, sp.win, J.cap, true);
                const bool full = full_bytes <= al->seg_full_bytes;
                for (int k = 0; k < K; k++) {
                    SaSeg g;
                    g.split = (int32_t)splits.size();
                    g.k = k;
                    g.cap = seg_cap_for(mx, k, K, sp.win, J.cap, full);
                    g.pad = 0;
                    g.out = seg_bytes;
                    seg_bytes += ((int64_t)J.n * g.cap + 255) & ~255ll;
                    queue.push_back(-(int32_t)segs.size() - 1);
                    segs.push_back(g);
                }
                for (int t = 0; t + 1 < K; t++) ftasks.push_back(make_int2((int)splits.size(), t));
                splits.push_back(sp);
            }
        }
        // Twins.  fix_bad_regions (SimilarAligner.cpp:428-459) re-aligns a bad
        // region's rows gap-filtered and reversed; when the whole alignment is
        // one bad region -- most many-row alignments (at 17 rows and 0.8 %
        // divergence fewer than 90 % of the columns are identical) -- those
        // rows are the job's input rows reversed, known before the walk.  In a
        // launch with few tasks (the last ExtendLoopFast iterations: tens of
        // long jobs on a GPU of thousands of wave slots) every split job gets
        // a twin split over its reversed rows whose segments run in the same
        // k_align_jobs launch; k_split_post hands a whole-job bad region to
        // the twin (k_twin_post chains it), so the re-alignment no longer
        // follows the forward walk.  The walk is the same process_seqs either
        // way (bit-exact); a twin whose chain fails leaves its sub-job to the
        // ordinary path, an unneeded twin costs only idle slots.
        const int n_js = (int)splits.size();
        bool twins = false;
        if (attempt == 0 && n_js > 0 && al->twins != 0) {
            const int64_t unsplit = (int64_t)todo.size() - n_js;
            twins = al->twins > 0 || 2 * (int64_t)segs.size() + unsplit <= 2048;
        }
        int64_t twin_bytes = 0;
        if (twins) {
            al->h_twin_off.assign(uj ? (size_t)u_rows : ne_len.size(), 0);
            al->h_twin_list.clear();
            for (int si = 0; si < n_js; si++) {
                SaSplit tw = splits[si];
                const SaJob& J = jobs[tw.job];
                for (int i = 0; i < J.n; i++) {
                    al->h_twin_off[J.row0 + i] = twin_bytes;
                    al->h_twin_list.push_back((int32_t)(J.row0 + i));
                    twin_bytes += row_len_at(tw.job, i);
                }
                const int ti = (int)splits.size();
                tw.sub = -2;
                tw.twin = 0;
                tw.tgt = n_tgt;
                tw.seg0 = (int32_t)segs.size();
                tw.post = -1;
                n_tgt += (int64_t)(tw.K - 1) * J.n;
                for (int k = 0; k < tw.K; k++) {
                    SaSeg g;
                    g.split = ti;
                    g.k = k;
                    g.cap = seg_cap_for(jmax[tw.job], k, tw.K, tw.win, J.cap);
                    g.pad = 0;
                    g.out = seg_bytes;
                    seg_bytes += ((int64_t)J.n * g.cap + 255) & ~255ll;
                    queue.push_back(-(int32_t)segs.size() - 1);
                    segs.push_back(g);
                }
                for (int t = 0; t + 1 < tw.K; t++) ftasks.push_back(make_int2(ti, t));
                splits[si].twin = ti + 1;
                splits.push_back(tw);
            }
        }
        if (rdbg && attempt == 0) {
            dbg_split.assign(n_jobs, 0);
            for (const SaSplit& sp : splits) dbg_split[sp.job] = 1;
        }
        if (splits.empty()) {
            queue = todo;
        } else {
            std::vector<uint8_t> is_split(n_jobs, 0);
            for (const SaSplit& sp : splits) is_split[sp.job] = 1;
            for (int32_t j : todo)
                if (!is_split[j]) queue.push_back(j);
        }
        // Unsplit twins.  Most many-row alignments are one bad region as a
        // whole (C3: 90 % of the 17-row flank jobs of the first iterations),
        // and fix_bad_regions (SimilarAligner.cpp:428-459) then re-aligns the
        // job's rows reversed after its forward walk: half of a launch's
        // critical path.  Every unsplit job of at least utw_rows rows gets a
        // twin task that walks its rows reversed in the same launch
        // (k_align_jobs, ahead of the jobs in the queue); a job that finds
        // itself one bad region takes the twin's result, any other leaves it
        // unused.  The walk is the same process_seqs (bit-exact).  Twins are
        // added while the launch stays within utw_max_tasks tasks.
        int64_t utw_bytes = 0;
        int n_utw = 0;
        std::vector<int64_t>& uoff = al->h_utw_off;
        if (attempt == 0 && o.aligner_type == 0 && al->utw_rows > 0) {
            std::vector<int32_t>& tq = al->h_utw_q;
            tq.clear();
            uoff.assign((size_t)n_jobs, -1);
            // up to utw_max_tasks tasks, and in any launch the heaviest jobs'
            // twins that fill the last 256-task step: the LDS share of every
            // workgroup (one per 256 tasks and CU) stays what it was
            const int64_t q = (int64_t)queue.size();
            const int64_t room = std::max<int64_t>((int64_t)al->utw_max_tasks - q, (q + 255) / 256 * 256 - q);
            for (int32_t q : queue) {
                if ((int64_t)tq.size() >= room) break;
                if (q < 0 || jobs[q].n < al->utw_rows) continue;
                uoff[(size_t)q] = utw_bytes;
                utw_bytes += ((int64_t)jobs[q].n * jobs[q].cap + 255) & ~255ll;
                tq.push_back(UTWIN_BASE + q);
            }
            n_utw = (int)tq.size();
            if (n_utw) queue.insert(queue.begin(), tq.begin(), tq.end());
        }
        const int nj = (int)queue.size();
        scr.grow((size_t)std::max<int64_t>(scratch, 256));  // (1.5x headroom: batches grow loop by loop)
        put(al->d_jobs.p, jobs.data(), jobs.size() * sizeof(SaJob));
        al->d_order.grow(queue.size());
        put(al->d_order.p, queue.data(), queue.size() * 4);
        zero(al->d_next.p, 4);
        pmark(3);
        // per-slot scratch: the word table (20 B an entry), the append_aligned
        // stack (1028 B a level) and the regions of unsplit jobs (17 B a
        // column), for wv waves on each of the 4 SIMDs of the 256
        // CUs.  The largest job's bounds set the sizes (a call inserts at most
        // rows x (length + 1) words and nests at most length / (aligned_check
        // + 1) deep).  When that many slots at those sizes pass the budget,
        // attempt 0 caps the table and the stack -- a call that would need more
        // ends its walk and marks the job overflowed (Proc::table_full, the
        // depth check in Proc::run) -- and attempt 1 runs fewer slots at the
        // full bounds: the giant alignments of whole-genome blocks
        // (AnchorLoopFast at C4) then cost memory only where they run.
        int64_t cols_need = 256;  // good_col doubles as 64 ints of scratch
        for (int32_t q : queue)
            if (q >= 0 && q < UTWIN_BASE) cols_need = std::max<int64_t>(cols_need, (int64_t)jobs[q].cap + 1);
        uint32_t tlog = 10;
        while ((1ull << tlog) < 2ull * (uint64_t)max_n * (uint64_t)(max_len + 1) + 64) tlog++;
        int depth = max_len / std::max(1, o.aligned_check + 1) + 4;
        auto per_slot = [&](uint32_t tl, int dp) { return (20ll << tl) + 1028ll * dp + 17ll * cols_need; };
        const int wv = nj > al->waves_many_at ? SA_WAVES_MANY : SA_WAVES_PER_EU;  // this launch's waves a SIMD
        size_t slots = (size_t)std::max(1, std::min(nj, 256 * 4 * wv));
        const int64_t mem_budget = std::max<int64_t>(al->slot_budget, 1ll << 22);
        if (attempt == 0)
            while ((int64_t)slots * per_slot(tlog, depth) > mem_budget && (tlog > 16 || depth > 512)) {
                if (tlog > 16 && (20ll << tlog) >= 1028ll * depth) tlog--;
                else depth = std::max(512, depth / 2);
            }
        slots = std::max<size_t>(1, std::min<size_t>(slots, (size_t)(mem_budget / per_slot(tlog, depth))));
        const size_t tcap = (size_t)1 << tlog;
        // Word tables: epochs only grow from launch to launch (every slot starts
        // at the last launch's highest epoch + 1), so entries left by earlier
        // launches never match, whatever the slot layout; the tables are
        // cleared only when they grow or the 16-bit epochs run out.
        const size_t tneed = as ? std::max(slots * tcap, slots1 * ((size_t)1 << tlog1)) : slots * tcap;
        if (tneed > al->tcap_alloc || al->epoch_base > 0xF000) {
            al->tkeys.grow(tneed);
            al->tmask.grow(tneed);
            al->tdone.grow(tneed);  // reset when a key is claimed
            NPGX_HIP(hipMemsetAsync(al->tkeys.p, 0, al->tkeys.cap * 8, st));
            NPGX_HIP(hipMemsetAsync(al->tmask.p, 0, al->tmask.cap * 8, st));  // epoch-tagged masks (vector search)
            al->tcap_alloc = std::min({al->tkeys.cap, al->tmask.cap, al->tdone.cap});  // cleared headroom counts
            al->epoch_base = 1;
        }
        zero(d_slot_epoch, 4);
        const size_t sneed = as ? std::max(slots * depth, slots1 * depth1) : slots * depth;
        al->st_p.grow(sneed * 64);
        al->st_len.grow(sneed * 64);
        al->st_pos.grow(sneed * 64);
        al->st_col.grow(sneed);
        const int slot_cols = (int)cols_need;
        const size_t cneed = as ? std::max(slots * (size_t)slot_cols, slots1 * (size_t)cols1) : slots * (size_t)slot_cols;
        al->regions.grow(cneed);
        al->good_col.grow(cneed);

        pmark(4);
        SaArgs A;
        A.rows = d_rows;
        A.row_off = d_roff;
        A.row_len = d_rlen;
        A.jobs = al->d_jobs.p;
        A.order = al->d_order.p;
        A.n_jobs = nj;
        A.n_jobs_dev = nullptr;
        A.aligner_type = o.aligner_type;
        A.scratch = scr.p;
        A.job_len = d_job_len;
        A.job_status = d_job_status;
        A.job_stats = al->want_stats ? al->d_job_stats.p : nullptr;
        A.next_job = al->d_next.p;
        A.tkeys = al->tkeys.p;
        A.tmask = al->tmask.p;
        A.tdone = al->tdone.p;
        A.tcap_log2 = tlog;
        A.slot_epoch = d_slot_epoch;
        A.epoch_base = al->epoch_base;
        A.st_p = al->st_p.p;
        A.st_len = al->st_len.p;
        A.st_pos = al->st_pos.p;
        A.st_col = al->st_col.p;
        A.st_depth_max = depth;
        A.regions = al->regions.p;
        A.good_col = al->good_col.p;
        A.slot_cols = slot_cols;
        A.P = P;
        bool defer = attempt == 0 && al->defer > 0 && o.aligner_type == 0 && n_reg > 0 && max_cap >= al->defer;
        if (defer) {  // some job long enough and with enough rows
            defer = false;
            for (int32_t j : todo) defer |= jobs[j].cap >= al->defer && jobs[j].n >= al->defer_rows;
        }
        A.defer = defer ? al->defer : 0;
        A.defer_rows = al->defer_rows;
        // deferred bad regions: of the long jobs (defer) and of every split job
        const bool deferring = defer || !splits.empty();
        if (deferring) {
            al->d_job_regions.grow((size_t)n_reg);
            al->d_job_nreg.grow(jobs.size());
            al->d_fin.grow(jobs.size());
            const int64_t max_sub = n_sub_max;
            al->d_subs.grow((size_t)max_sub);
            al->d_sub_res.grow((size_t)max_sub);
            al->d_alloc.ensure(2);
            al->d_counters.ensure(8);
            // sub-job outputs: about what the jobs' own scratch holds
            al->d_pool.grow((size_t)scratch + (16u << 20));
            zero(al->d_alloc.p, 16);
            zero(al->d_counters.p, 32);
            A.job_regions = al->d_job_regions.p;
            A.job_nreg = al->d_job_nreg.p;
            A.subs = al->d_subs.p;
            A.sub_res = al->d_sub_res.p;
            A.alloc = al->d_alloc.p;
            A.counters = al->d_counters.p;
            A.pool = al->d_pool.p;
            A.pool_cap = (int64_t)al->d_pool.cap;
            A.max_sub = max_sub;
            A.fin = al->d_fin.p;
        } else {
            A.job_regions = nullptr;
            A.job_nreg = nullptr;
            A.subs = nullptr;
            A.sub_res = nullptr;
            A.alloc = nullptr;
            A.counters = nullptr;
            A.pool = nullptr;
            A.pool_cap = 0;
            A.max_sub = 0;
            A.fin = nullptr;
        }
        pmark(5);
        // LDS: word table (20 B/entry) + the largest job's rows.  A workgroup may
        // take all 160 KiB of a CU's LDS; when the batch has more jobs than
        // workgroups can be resident at that size the stage shrinks, and the
        // jobs that no longer fit read their rows from global memory.
        // LDS per workgroup: the 64-shift chunk words (vector search, up to
        // VEC_ROWS rows), the word table of the row-parallel search (more rows:
        // up to half of what is left) and the stage for the job's rows.  The
        // budget shrinks as more workgroups must be resident per CU.
        int64_t max_rows = 0;
        for (int32_t j : todo) max_rows = std::max<int64_t>(max_rows, jsum[j]);
        static const int64_t per_cu_max = getenv("NPGX_SA_PER_CU_MAX") ? std::max(1, atoi(getenv("NPGX_SA_PER_CU_MAX")))
                                                                       : 4 * SA_WAVES_MANY;  // (A/B: LDS per slot)
        const int64_t per_cu = std::min<int64_t>(std::min<int64_t>(4 * wv, per_cu_max),
                                                 std::max<int64_t>(1, ((int64_t)nj + 255) / 256));
        const int64_t budget = LDS_PER_CU / per_cu;
        // word history of the row-parallel search (HIST_SHIFTS x 64 words) when
        // the budget allows
        const int64_t hist_bytes = 64 * HIST_SHIFTS * 8;
        A.hist_cap = (max_n > VEC_ROWS && hist_bytes * 4 <= budget) ? HIST_SHIFTS : 0;
        const int64_t words_bytes = std::max<int64_t>(64 * VEC_ROWS * 8, A.hist_cap ? hist_bytes : 0);
        A.words_bytes = (int32_t)words_bytes;
        A.ltab_log2 = 0;
        if (max_n > VEC_ROWS)
            while (A.ltab_log2 < 12 && (20ll << (A.ltab_log2 + 1)) <= (budget - words_bytes) / 2) A.ltab_log2++;
        // key, row mask and completion shift per entry
        const int64_t ltab = 1ll << A.ltab_log2;
        const int table_bytes = (int)(16 * ltab + 8 * ((ltab + 1) / 2) + words_bytes);
        const int64_t stage_cap = std::max<int64_t>(0, budget - table_bytes);
        // short jobs keep A|B|C in the stage too (k_align_jobs): size the stage
        // for the largest such job within the budget
        int64_t max_need = (max_rows + 15) & ~15ll;
        for (int32_t j : todo) {
            if (A.defer != 0 && jobs[j].cap >= A.defer && jobs[j].n >= A.defer_rows) continue;
            const int64_t need = (((int64_t)jsum[j] + 15) & ~15ll) + 3ll * jobs[j].n * jobs[j].cap;
            if (need <= stage_cap) max_need = std::max(max_need, need);
        }
        A.stage_bytes = o.aligner_type == 0 ? (int32_t)std::min<int64_t>(max_need, stage_cap & ~15ll) : 0;
        const size_t lds_bytes = (size_t)table_bytes + (size_t)A.stage_bytes;
        NPGX_REQUIRE(A.stage_bytes >= 0 && lds_bytes <= (size_t)LDS_PER_CU, NPGX_ERR_STATE, "LDS budget");
        A.splits = nullptr;
        A.segs = nullptr;
        A.targets = nullptr;
        A.seg_res = nullptr;
        A.seg_wall = nullptr;
        A.sub_wall = nullptr;
        A.seg_pool = nullptr;
        A.sctr = nullptr;
        A.qseg = nullptr;
        A.qsub = nullptr;
        A.rq = nullptr;
        A.ftasks = nullptr;
        A.split_len = o.aligner_type == 0 ? al->split : 0;
        A.twin_rows = nullptr;
        A.twin_off = nullptr;
        A.utw_off = nullptr;
        A.utw_state = nullptr;
        A.utw_len = nullptr;
        A.utw_pool = nullptr;
        if (n_utw) {
            al->d_utw_pool.grow((size_t)std::max<int64_t>(utw_bytes, 256));
            al->d_utw_off.grow((size_t)n_jobs);
            al->d_utw_st.grow(2 * (size_t)n_jobs);
            put(al->d_utw_off.p, uoff.data(), (size_t)n_jobs * 8);
            zero(al->d_utw_st.p, 2 * (size_t)n_jobs * 4);
            A.utw_off = al->d_utw_off.p;
            A.utw_state = al->d_utw_st.p;
            A.utw_len = al->d_utw_st.p + n_jobs;
            A.utw_pool = al->d_utw_pool.p;
        }
        A.post_area = nullptr;
        if (post_bytes > 0) {
            al->d_post.grow((size_t)post_bytes);
            A.post_area = al->d_post.p;
        }
        A.chain = nullptr;
        A.chain_hdr = nullptr;
        A.chain_bits = nullptr;
        A.bits_off = nullptr;
        A.part0 = nullptr;
        if (!splits.empty()) {
            al->d_chain.grow(segs.size());
            al->d_chain_hdr.grow(splits.size());
            al->d_chain_bits.grow((size_t)std::max<int64_t>(bits_words, 1));
            al->d_bits_off.grow(bits_off.size());
            al->d_part0.grow(part0.size());
            put(al->d_bits_off.p, bits_off.data(), bits_off.size() * 8);
            put(al->d_part0.p, part0.data(), part0.size() * 4);
            A.chain = al->d_chain.p;
            A.chain_hdr = al->d_chain_hdr.p;
            A.chain_bits = al->d_chain_bits.p;
            A.bits_off = al->d_bits_off.p;
            A.part0 = al->d_part0.p;
        }
        A.cap_splits = A.cap_segs = 0;
        A.cap_tgt = A.cap_find = A.cap_pool = 0;
        const int n_job_splits = (int)splits.size(), n_job_find = (int)ftasks.size();
        const bool split_subs = deferring && A.split_len > 0;
        if (!splits.empty() || split_subs) {
            // the job splits (host plan) and room for the sub-job splits (k_plan_subs)
            A.cap_splits = n_job_splits + (split_subs ? (int32_t)std::min<int64_t>(n_sub_max, 1 << 20) : 0);
            A.cap_segs = (int32_t)segs.size() + (split_subs ? (1 << 17) : 0);
            A.cap_tgt = n_tgt + (split_subs ? (1ll << 22) : 0);
            A.cap_find = n_job_find + (split_subs ? (1ll << 17) : 0);
            A.cap_pool = seg_bytes + (split_subs ? std::max<int64_t>(256ll << 20, 4 * (int64_t)(scratch + (16 << 20))) : 0);
            al->d_splits.grow((size_t)std::max(1, A.cap_splits));
            al->d_segs.grow((size_t)std::max(1, A.cap_segs));
            al->d_ftasks.grow((size_t)std::max<int64_t>(1, A.cap_find));
            al->d_targets.grow((size_t)std::max<int64_t>(1, A.cap_tgt));
            al->d_seg_res.grow((size_t)std::max(1, A.cap_segs));
            al->d_seg_wall.grow(2 * (size_t)std::max(1, A.cap_segs));
            al->d_seg_pool.grow((size_t)std::max<int64_t>(256, A.cap_pool));
            al->d_qseg.grow((size_t)std::max(1, A.cap_segs));
            al->d_qsub.grow((size_t)std::max<int64_t>(1, n_sub_max));
            al->d_sctr.ensure(SC_N);
            if (!splits.empty()) {
                put(al->d_splits.p, splits.data(), splits.size() * sizeof(SaSplit));
                put(al->d_segs.p, segs.data(), segs.size() * sizeof(SaSeg));
                put(al->d_ftasks.p, ftasks.data(), ftasks.size() * sizeof(int2));
            }
            const uint32_t sc[SC_N] = {(uint32_t)n_job_splits, (uint32_t)segs.size(), (uint32_t)n_tgt,
                                       (uint32_t)n_job_find, 0u, 0u, (uint32_t)seg_bytes,
                                       (uint32_t)((uint64_t)seg_bytes >> 32)};
            put(al->d_sctr.p, sc, sizeof(sc));
            A.splits = al->d_splits.p;
            A.segs = al->d_segs.p;
            A.targets = al->d_targets.p;
            A.seg_res = al->d_seg_res.p;
            A.seg_wall = al->d_seg_wall.p;
            if (al->want_stats && deferring) {
                al->d_sub_wall.grow(2 * (size_t)std::max<int64_t>(1, n_sub_max));
                NPGX_HIP(hipMemsetAsync(al->d_sub_wall.p, 0, 2 * (size_t)std::max<int64_t>(1, n_sub_max) * 8, st));
                A.sub_wall = al->d_sub_wall.p;
            }
            A.seg_pool = al->d_seg_pool.p;
            A.sctr = al->d_sctr.p;
            A.qseg = al->d_qseg.p;
            A.qsub = al->d_qsub.p;
            A.ftasks = al->d_ftasks.p;
            if (twins) {
                al->d_twin.grow((size_t)std::max<int64_t>(twin_bytes, 1));
                al->d_twin_off.grow(al->h_twin_off.size());
                al->d_twin_list.grow(al->h_twin_list.size());
                put(al->d_twin_off.p, al->h_twin_off.data(), al->h_twin_off.size() * 8);
                put(al->d_twin_list.p, al->h_twin_list.data(), al->h_twin_list.size() * 4);
                A.twin_rows = al->d_twin.p;
                A.twin_off = al->d_twin_off.p;
            }
            flush();
            if (twins) {
                hipLaunchKernelGGL(k_twin_rows, dim3((unsigned)std::min<size_t>(al->h_twin_list.size(), 4096)),
                                   dim3(256), 0, st, d_rows, d_roff, d_rlen, al->d_twin_list.p,
                                   (int)al->h_twin_list.size(), al->d_twin_off.p, al->d_twin.p);
                NPGX_HIP(hipGetLastError());
            }
            if (n_job_find > 0) {
                size_t tf = al->timer.begin("align_split", st, 0.0, (int64_t)n_job_find);
                hipLaunchKernelGGL(k_split_find, dim3((unsigned)n_job_find), dim3(64 * SPLIT_WAVES), SPLIT_LDS, st, A,
                                   al->d_ftasks.p, n_job_find, 0);
                NPGX_HIP(hipGetLastError());
                al->timer.end(tf, st);
            }
        }
        pmark(6);
        int64_t residues = 0;
        for (int32_t j : todo) residues += jsum[j];
        if (as) {
            put(al->d_jobs1.p, al->h_jobs1.data(), al->h_jobs1.size() * sizeof(SaJob));
            zero(al->d_ctr1.p, 8);
        }
        flush();
        size_t ti = al->timer.begin(attempt == 0 ? "align_jobs" : "align_jobs_retry", st,
                                    double(residues) * 2.0, residues);
        launch_sa(k_align_jobs<true, SA_WAVES_PER_EU>, k_align_jobs<false, SA_WAVES_PER_EU>,
                  k_align_jobs<true, SA_WAVES_MANY>, k_align_jobs<false, SA_WAVES_MANY>, wv, slots, lds_bytes, A);
        NPGX_HIP(hipGetLastError());
        al->timer.end(ti, st);
        pmark(7);
        if (!splits.empty()) {  // the split jobs: chain, regions, deferred bad regions
            // (the job splits only: the twins [n_js, splits.size()) are chained by k_twin_post)
            ti = al->timer.begin("align_split_chain", st, 0.0, (int64_t)n_js);
            hipLaunchKernelGGL(k_split_chain, dim3((unsigned)n_js), dim3(POST_THREADS), 0, st, A);
            NPGX_HIP(hipGetLastError());
            hipLaunchKernelGGL(k_chain_copy, dim3((unsigned)part0.back()), dim3(POST_THREADS), 0, st, A, n_js);
            NPGX_HIP(hipGetLastError());
            al->timer.end(ti, st);
            ti = al->timer.begin("align_split_post", st, 0.0, (int64_t)n_js);
            hipLaunchKernelGGL(k_split_post, dim3((unsigned)n_js), dim3(REG_THREADS), POST_LDS, st, A,
                               (int)POST_LDS);
            NPGX_HIP(hipGetLastError());
            if (twins) {  // k_twin_post: the twins whose jobs are one bad region
                const int n_tw = (int)splits.size() - n_js;
                hipLaunchKernelGGL(k_sub_post, dim3((unsigned)std::min(n_tw, 512)), dim3(POST_THREADS), 0, st, A, n_js,
                                   (int)splits.size());
                NPGX_HIP(hipGetLastError());
            }
            al->timer.end(ti, st);
        }
        if (deferring) {  // the deferred bad regions, then their jobs (no-ops when nothing was deferred)
            // jobs that may have deferred: the split ones and the long ones
            int64_t n_fin = (int64_t)n_js;
            int64_t max_rc = 1;
            {
                std::vector<uint8_t> is_split(n_jobs, 0);
                for (const SaSplit& sp : splits) is_split[sp.job] = 1;
                for (int32_t j : todo) {
                    const bool may = is_split[j] || (defer && jobs[j].cap >= al->defer && jobs[j].n >= al->defer_rows);
                    if (!may) continue;
                    n_fin += is_split[j] ? 0 : 1;
                    max_rc = std::max<int64_t>(max_rc, jobs[j].reg_cap + 1);
                }
            }
            const int lds_ints = (int)std::min<int64_t>(max_rc, 32768);
            al->d_reg_dst.grow((size_t)n_reg + jobs.size());
            if (!splits.empty()) {  // the rows of the split jobs' bad regions
                ti = al->timer.begin("align_sub_rows", st, 0.0, 0);
                hipLaunchKernelGGL(k_sub_rows, dim3(1024), dim3(256), 0, st, A, max_n);
                NPGX_HIP(hipGetLastError());
                al->timer.end(ti, st);
            }
            if (split_subs) {  // the long sub-jobs: plan, sync states
                ti = al->timer.begin("align_sub_split", st, 0.0, 0);
                hipLaunchKernelGGL(k_plan_subs, dim3(256), dim3(256), 0, st, A);
                NPGX_HIP(hipGetLastError());
                hipLaunchKernelGGL(k_split_find, dim3(2048), dim3(64 * SPLIT_WAVES), SPLIT_LDS, st, A, al->d_ftasks.p, -1,
                                   n_job_find);
                NPGX_HIP(hipGetLastError());
                al->timer.end(ti, st);
            }
            ti = al->timer.begin("align_sub", st, 0.0, 0);
            launch_sa(k_align_sub<true, SA_WAVES_PER_EU>, k_align_sub<false, SA_WAVES_PER_EU>,
                      k_align_sub<true, SA_WAVES_MANY>, k_align_sub<false, SA_WAVES_MANY>, wv, slots, lds_bytes, A);
            NPGX_HIP(hipGetLastError());
            al->timer.end(ti, st);
            if (split_subs) {  // the split sub-jobs' chains
                ti = al->timer.begin("align_sub_post", st, 0.0, 0);
                hipLaunchKernelGGL(k_sub_post, dim3(512), dim3(POST_THREADS), 0, st, A, n_job_splits, -1);
                NPGX_HIP(hipGetLastError());
                al->timer.end(ti, st);
                // the failed sub-jobs again, whole, at their proven bound (one
                // launch, usually empty): a split sub-job whose chain broke or
                // overflowed no longer sends its job to attempt 1 whole
                // 
                al->d_rq.grow((size_t)std::max<int64_t>(n_sub_max, 1));
                SaArgs A2 = A;
                A2.rq = al->d_rq.p;
                ti = al->timer.begin("align_sub_retry", st, 0.0, 0);
                hipLaunchKernelGGL(k_sub_retry_list, dim3(256), dim3(256), 0, st, A2);
                launch_sa(k_align_sub<true, SA_WAVES_PER_EU>, k_align_sub<false, SA_WAVES_PER_EU>,
                          k_align_sub<true, SA_WAVES_MANY>, k_align_sub<false, SA_WAVES_MANY>, wv, slots, lds_bytes, A2);
                NPGX_HIP(hipGetLastError());
                al->timer.end(ti, st);
            }
            if (n_fin > 0) {
                ti = al->timer.begin("align_fin_copy", st, 0.0, 0);
                hipLaunchKernelGGL(k_fin_prefix, dim3((unsigned)n_fin), dim3(REG_THREADS), 0, st, A, al->d_reg_dst.p);
                NPGX_HIP(hipGetLastError());
                hipLaunchKernelGGL(k_fin_copy, dim3((unsigned)(n_fin * FIN_PARTS)), dim3(POST_THREADS),
                                   (size_t)lds_ints * 4, st, A, lds_ints, al->d_reg_dst.p);
                NPGX_HIP(hipGetLastError());
                al->timer.end(ti, st);
            }
            ti = al->timer.begin("align_finish", st, 0.0, 0);
            if (al->long_head > 0) hipLaunchKernelGGL(k_align_finish<true>, dim3((unsigned)slots), dim3(64), lds_bytes, st, A);
            else hipLaunchKernelGGL(k_align_finish<false>, dim3((unsigned)slots), dim3(64), lds_bytes, st, A);
            NPGX_HIP(hipGetLastError());
            al->timer.end(ti, st);
        }
        if (!splits.empty() && getenv("NPGX_SPLIT_DEBUG")) {  // diagnostic: sync states and segment results
            std::vector<int32_t> tg((size_t)n_tgt);
            std::vector<int4> sr(segs.size());
            NPGX_HIP(hipMemcpyAsync(tg.data(), al->d_targets.p, tg.size() * 4, hipMemcpyDeviceToHost, st));
            NPGX_HIP(hipMemcpyAsync(sr.data(), al->d_seg_res.p, sr.size() * 16, hipMemcpyDeviceToHost, st));
            NPGX_HIP(hipStreamSynchronize(st));
            for (const SaSplit& sp : splits) {
                const int n = jobs[sp.job].n;
                int valid = 0, ovf = 0, hits = 0;
                for (int k = 1; k < sp.K; k++) valid += tg[sp.tgt + (int64_t)(k - 1) * n] >= 0;
                std::string chain;
                for (int k = 0; k < sp.K; k++) {
                    const int4 r = sr[sp.seg0 + k];
                    ovf += r.z;
                    hits += r.x >= 0 && r.x < sp.K;
                }
                for (int k = 0, guard = 0; k < sp.K && k >= 0 && guard < 1000; guard++) {
                    const int4 r = sr[sp.seg0 + k];
                    chain += std::to_string(k) + "(" + std::to_string(r.y) + (r.z ? "!" : "") + ")>";
                    if (r.x <= k) break;
                    k = r.x;
                }
                fprintf(stderr, "split job %d n=%d K=%d maxlen=%d valid_states=%d hits=%d ovf=%d chain %s\n", sp.job,
                        n, sp.K, jmax[sp.job], valid, hits, ovf, chain.c_str());
            }
            if (al->want_stats) {  // the slowest segments (wall clock at 100 MHz)
                std::vector<int64_t> sw(2 * segs.size());
                NPGX_HIP(hipMemcpy(sw.data(), al->d_seg_wall.p, sw.size() * 8, hipMemcpyDeviceToHost));
                std::vector<std::pair<int64_t, int>> d;
                for (size_t q = 0; q < segs.size(); q++) d.push_back({sw[2 * q + 1] - sw[2 * q], (int)q});
                std::sort(d.rbegin(), d.rend());
                for (size_t q = 0; q < std::min<size_t>(5, d.size()); q++) {
                    const int4 r = sr[(size_t)d[q].second];
                    fprintf(stderr, "slow segment %d: %.1f us, %d cols, next %d (K %d), n %d\n", d[q].second,
                            d[q].first / 100.0, r.y, r.x, splits[segs[(size_t)d[q].second].split].K,
                            jobs[splits[segs[(size_t)d[q].second].split].job].n);
                }
                // the launch's critical path: when the segments and the whole jobs end
                std::vector<int64_t> js((size_t)n_jobs * NPGX_JOB_STATS);
                NPGX_HIP(hipMemcpy(js.data(), al->d_job_stats.p, js.size() * 8, hipMemcpyDeviceToHost));
                int64_t t0 = INT64_MAX, se = 0, je = 0, jd = 0;
                int jslow = -1;
                for (size_t q = 0; q < segs.size(); q++) {
                    t0 = std::min(t0, sw[2 * q]);
                    se = std::max(se, sw[2 * q + 1]);
                }
                std::vector<uint8_t> was_split(n_jobs, 0);
                for (const SaSplit& sp2 : splits) was_split[sp2.job] = 1;
                for (int32_t j : todo) {
                    const int64_t* r = js.data() + (size_t)j * NPGX_JOB_STATS;
                    if (was_split[j] || r[11] <= 0 || r[23] <= 0) continue;
                    t0 = std::min(t0, r[11]);
                    je = std::max(je, r[23]);
                    if (r[23] - r[11] > jd) {
                        jd = r[23] - r[11];
                        jslow = j;
                    }
                }
                if (t0 != INT64_MAX)
                    fprintf(stderr, "launch: segments end at %.1f us, whole jobs at %.1f us; slowest whole job %d: "
                            "%.1f us, %lld cols, %d rows (process_seqs %.1f us, regions+realign %.1f us)\n",
                            (se - t0) / 100.0, (je - t0) / 100.0, jslow, jd / 100.0,
                            jslow >= 0 ? (long long)js[(size_t)jslow * NPGX_JOB_STATS + 1] : 0ll,
                            jslow >= 0 ? jobs[jslow].n : 0,
                            jslow >= 0 ? js[(size_t)jslow * NPGX_JOB_STATS + 8] / 2400.0 : 0.0,
                            jslow >= 0 ? js[(size_t)jslow * NPGX_JOB_STATS + 9] / 2400.0 : 0.0);
            }
            if (deferring) {  // sub-jobs: count and widths
                unsigned long long al2[2];
                NPGX_HIP(hipMemcpy(al2, al->d_alloc.p, 16, hipMemcpyDeviceToHost));
                std::vector<SaSub> sb((size_t)al2[1]);
                std::vector<int2> rs((size_t)al2[1]);
                if (!sb.empty()) {
                    NPGX_HIP(hipMemcpy(sb.data(), al->d_subs.p, sb.size() * sizeof(SaSub), hipMemcpyDeviceToHost));
                    NPGX_HIP(hipMemcpy(rs.data(), al->d_sub_res.p, rs.size() * 8, hipMemcpyDeviceToHost));
                }
                if (al->want_stats && A.sub_wall && !sb.empty()) {  // the sub-job launch's critical path
                    std::vector<int64_t> sw2(2 * sb.size());
                    NPGX_HIP(hipMemcpy(sw2.data(), al->d_sub_wall.p, sw2.size() * 8, hipMemcpyDeviceToHost));
                    unsigned int sc2[SC_N];
                    NPGX_HIP(hipMemcpy(sc2, al->d_sctr.p, sizeof(sc2), hipMemcpyDeviceToHost));
                    std::vector<int64_t> segw(2 * (size_t)std::max(1, A.cap_segs));
                    NPGX_HIP(hipMemcpy(segw.data(), al->d_seg_wall.p, segw.size() * 8, hipMemcpyDeviceToHost));
                    int64_t t0 = INT64_MAX, wend = 0, send = 0, wmax = 0;
                    int wslow = -1;
                    for (size_t q = 0; q < sb.size(); q++)
                        if (sw2[2 * q] > 0) {
                            t0 = std::min(t0, sw2[2 * q]);
                            wend = std::max(wend, sw2[2 * q + 1]);
                            if (sw2[2 * q + 1] - sw2[2 * q] > wmax) {
                                wmax = sw2[2 * q + 1] - sw2[2 * q];
                                wslow = (int)q;
                            }
                        }
                    for (unsigned int q = (unsigned int)segs.size(); q < std::min(sc2[SC_SEGS], (unsigned)A.cap_segs); q++)
                        if (segw[2 * q] > 0) {
                            t0 = std::min(t0, segw[2 * q]);
                            send = std::max(send, segw[2 * q + 1]);
                        }
                    if (t0 != INT64_MAX)
                        fprintf(stderr, "sub launch: %u sub segments end at %.1f us, whole subs at %.1f us; slowest whole "
                                "sub %d: %.1f us, %d cols, %d rows\n", sc2[SC_SEGS] - (unsigned)segs.size(),
                                send ? (send - t0) / 100.0 : 0.0, (wend - t0) / 100.0, wslow, wmax / 100.0,
                                wslow >= 0 ? rs[(size_t)wslow].x : 0, wslow >= 0 ? jobs[sb[(size_t)wslow].job].n : 0);
                }
                std::vector<int> wd;
                for (const int2& r : rs) wd.push_back(r.x);
                std::sort(wd.begin(), wd.end());
                long long tot = 0;
                for (int x : wd) tot += x;
                fprintf(stderr, "subs %zu total_cols %lld p50 %d p90 %d p99 %d max %d\n", wd.size(), tot,
                        wd.empty() ? 0 : wd[wd.size() / 2], wd.empty() ? 0 : wd[wd.size() * 9 / 10],
                        wd.empty() ? 0 : wd[wd.size() * 99 / 100], wd.empty() ? 0 : wd.back());
            }
        }
        pmark(8);
        if (as) {
            // the overflowed jobs again at the proven bound (no splits, no
            // deferred regions: attempt 1 of the synchronous path), then every
            // job's rows
            const unsigned jg = (unsigned)std::max<int64_t>(1, ((int64_t)n_jobs + 255) / 256);
            hipLaunchKernelGGL(k_retry_list, dim3(jg), dim3(256), 0, st, d_job_status, n_jobs, al->d_order1.p,
                               al->d_ctr1.p, al->d_retried.p);
            SaArgs A1 = A;
            A1.jobs = al->d_jobs1.p;
            A1.order = al->d_order1.p;
            A1.n_jobs = 0;
            A1.n_jobs_dev = al->d_ctr1.p;
            A1.next_job = (unsigned int*)(al->d_ctr1.p + 1);
            A1.scratch = al->d_scratch2.p;
            A1.tcap_log2 = tlog1;
            A1.st_depth_max = depth1;
            A1.slot_cols = cols1;
            A1.defer = 0;
            A1.job_regions = nullptr;
            A1.job_nreg = nullptr;
            A1.subs = nullptr;
            A1.sub_res = nullptr;
            A1.alloc = nullptr;
            A1.counters = nullptr;
            A1.pool = nullptr;
            A1.pool_cap = 0;
            A1.max_sub = 0;
            A1.fin = nullptr;
            A1.splits = nullptr;
            A1.segs = nullptr;
            A1.targets = nullptr;
            A1.seg_res = nullptr;
            A1.seg_wall = nullptr;
            A1.sub_wall = nullptr;
            A1.seg_pool = nullptr;
            A1.sctr = nullptr;
            A1.qseg = nullptr;
            A1.qsub = nullptr;
            A1.ftasks = nullptr;
            A1.post_area = nullptr;
            A1.chain = nullptr;
            A1.chain_hdr = nullptr;
            A1.chain_bits = nullptr;
            A1.bits_off = nullptr;
            A1.part0 = nullptr;
            A1.split_len = 0;
            A1.twin_rows = nullptr;
            A1.twin_off = nullptr;
            A1.utw_off = nullptr;
            A1.utw_state = nullptr;
            A1.utw_len = nullptr;
            A1.utw_pool = nullptr;
            A1.cap_splits = A1.cap_segs = 0;
            A1.cap_tgt = A1.cap_find = A1.cap_pool = 0;
            size_t tr = al->timer.begin("align_jobs_retry", st, 0.0, 0);
            if (al->long_head > 0)
                hipLaunchKernelGGL((k_align_jobs<true, SA_WAVES_PER_EU>), dim3((unsigned)slots1), dim3(64), lds_bytes, st, A1);
            else
                hipLaunchKernelGGL((k_align_jobs<false, SA_WAVES_PER_EU>), dim3((unsigned)slots1), dim3(64), lds_bytes, st, A1);
            al->timer.end(tr, st);
            hipLaunchKernelGGL(k_job_rows, dim3(jg), dim3(256), 0, st, al->d_jobs.p, al->d_jobs1.p, al->d_retried.p,
                               d_job_status, d_job_len, n_jobs, scr.p, al->d_scratch2.p, as->out, as->err);
            NPGX_HIP(hipGetLastError());
            NPGX_HIP(hipMemcpyAsync(as->epoch, d_slot_epoch, 4, hipMemcpyDeviceToDevice, st));
            res.len.clear();
            res.cap.clear();
            res.bptr.clear();
            al->host_ms[0] += ms(tp);
            pmark(8);
            if (pdbg)
                fprintf(stderr, "align_device async %d jobs: prep %.3f order %.3f puts %.3f split_plan %.3f slots %.3f "
                        "args %.3f lds+split %.3f launch %.3f post %.3f ms\n", n_jobs, pt[0], pt[1], pt[2], pt[3],
                        pt[4], pt[5], pt[6], pt[7], pt[8]);
            return;
        }
        int32_t* pl = (int32_t*)al->pinned.take((size_t)n_jobs * 8 + 8, st);
        NPGX_HIP(hipMemcpyAsync(pl, d_job_len, ((size_t)n_jobs * 2 + 1) * 4, hipMemcpyDeviceToHost, st));
        al->host_ms[0] += ms(tp);
        tp = std::chrono::steady_clock::now();
        NPGX_HIP(stream_wait(st));
        al->host_ms[1] += ms(tp);
        tp = std::chrono::steady_clock::now();
        // (after the wait: a copy into pageable memory would wait for the
        // kernels itself and book their time as host preparation)
        if (al->want_stats)
            NPGX_HIP(hipMemcpy(jst.data(), al->d_job_stats.p, jst.size() * 8, hipMemcpyDeviceToHost));
        memcpy(jlen.data(), pl, n_jobs * 4);
        memcpy(jstat.data(), pl + n_jobs, n_jobs * 4);
        al->epoch_base = std::max(al->epoch_base, (uint32_t)pl[2 * n_jobs] + 1);
        al->pinned.reset();
        pmark(9);
        std::vector<int32_t> again;
        for (int32_t j : todo) {
            NPGX_REQUIRE(jstat[j] >= 0 && jstat[j] <= 2, NPGX_ERR_STATE, "alignment job left unfinished");
            if (jstat[j] == 1) {
                again.push_back(j);
                if (rdbg && attempt == 0) {
                    dbg_why.resize(n_jobs, 0);
                    dbg_why[j] = jlen[j];
                }
                continue;
            }
            if (al->want_stats)
                for (int q = 0; q < NPGX_JOB_STATS; q++)
                    al->job_stats[(size_t)j * NPGX_JOB_STATS + q] = jst[(size_t)j * NPGX_JOB_STATS + q];
            res.len[j] = jlen[j];
            res.cap[j] = jobs[j].cap;
            // B of the job (rows [n, 2n) of its A|B|C scratch), or A (status 2)
            res.bptr[j] = (const char*)(scr.p + jobs[j].scratch + (jstat[j] == 2 ? 0 : (int64_t)jobs[j].n * jobs[j].cap));
        }
        if (attempt == 1 && !again.empty())
            throw Error(NPGX_ERR_RANGE, "alignment exceeded the proven column bound");
        if (attempt == 1 && rdbg)
            for (int32_t j : todo)
                fprintf(stderr, "retry job %d: rows %d longest %d residues %d room0 %d split %d length %d why %d\n", j,
                        jobs[j].n, jmax[j], jsum[j], dbg_cap0[j], j < (int32_t)dbg_split.size() ? dbg_split[j] : -1,
                        jlen[j], j < (int32_t)dbg_why.size() ? -dbg_why[j] : 0);
        todo.swap(again);
    }
    if (!wide_idx.empty()) {
        if (!al->wide) al->wide = wide_create();
        const int params[5] = {o.mismatch_check, o.gap_check, o.aligned_check, o.min_length, wf};
        std::vector<int32_t> wl, wc;
        std::vector<const char*> wp;
        auto ti = al->timer.begin("align_wide", st, 0.0, 0);
        double wide_wait = 0;  // booked as kernel wait, not host preparation
        align_wide(al->wide, st, d_rows, ne_off.data(), ne_len.data(), (int64_t)ne_len.size(), wide_in, params,
                   o.aligner_type, wl, wc, wp, &wide_wait);
        al->timer.end(ti, st);
        al->host_ms[1] += wide_wait;
        tp += std::chrono::duration_cast<std::chrono::steady_clock::duration>(
            std::chrono::duration<double, std::milli>(wide_wait));
        for (size_t q = 0; q < wide_idx.size(); q++) {
            res.len[wide_idx[q]] = wl[q];
            res.cap[wide_idx[q]] = wc[q];
            res.bptr[wide_idx[q]] = wp[q];
        }
    }
    al->host_ms[0] += ms(tp);
    pmark(10);
    if (pdbg)
        fprintf(stderr, "align_device %d jobs: prep %.3f order %.3f puts %.3f split_plan %.3f slots %.3f args %.3f "
                "lds+split %.3f launch %.3f post %.3f wait %.3f results %.3f ms\n", n_jobs, pt[0], pt[1], pt[2],
                pt[3], pt[4], pt[5], pt[6], pt[7], pt[8], pt[9], pt[10]);
}

void align_batch(npgx_aligner* al, const char* rows, const int64_t* row_off,
                 const int32_t* job_row_start, int32_t n_jobs) {
    NPGX_HIP(hipSetDevice(al->device));
    hipStream_t st = al->stream;
    al->timer.reset();
    al->has_result = false;
    NPGX_REQUIRE(n_jobs >= 0, NPGX_ERR_ARG, "n_jobs < 0");
    const int64_t r_base = n_jobs ? job_row_start[0] : 0;
    const int64_t n_rows = n_jobs ? (int64_t)job_row_start[n_jobs] - r_base : 0;
    // host rows -> device (validated for the similar aligner)
    const int64_t b0 = n_rows ? row_off[r_base] : 0;
    const int64_t bytes = n_rows ? row_off[r_base + n_rows] - b0 : 0;
    std::vector<int64_t> roff((size_t)n_rows + 1);
    std::vector<int32_t> rlen((size_t)std::max<int64_t>(n_rows, 1));
    for (int64_t r = 0; r < n_rows; r++) {
        roff[(size_t)r] = row_off[r_base + r] - b0;
        const int64_t len = row_off[r_base + r + 1] - row_off[r_base + r];
        NPGX_REQUIRE(len >= 0 && len < (1ll << 30), NPGX_ERR_RANGE, "row length out of range");
        rlen[(size_t)r] = (int32_t)len;
    }
    if (al->opt.aligner_type == 0)
        for (int64_t q = 0; q < bytes; q++) {
            const char c = rows[b0 + q];
            NPGX_REQUIRE(c == 'A' || c == 'C' || c == 'G' || c == 'T' || c == 'N', NPGX_ERR_ARG,
                         "similar aligner rows must be upper-case ATGCN");
        }
    al->d_rows.ensure((size_t)std::max<int64_t>(bytes, 1));
    if (bytes) NPGX_HIP(hipMemcpyAsync(al->d_rows.p, rows + b0, (size_t)bytes, hipMemcpyHostToDevice, st));
    std::vector<int32_t> js((size_t)n_jobs + 1);
    for (int32_t j = 0; j <= n_jobs; j++) js[(size_t)j] = (int32_t)(job_row_start[j] - r_base);
    AlignResult res;
    align_device(al, al->d_rows.p, roff.data(), rlen.data(), js.data(), n_jobs, res);
    // gather every row (empty rows become all-gap rows), one D2H copy
    std::vector<GatherRow> g((size_t)n_rows);
    int64_t tot = 0;
    al->out_off.assign((size_t)n_rows + 1, 0);
    al->job_len.assign(n_jobs, 0);
    for (int32_t j = 0; j < n_jobs; j++) {
        al->job_len[j] = res.len[j];
        for (int32_t r = js[j]; r < js[j + 1]; r++) {
            GatherRow& x = g[(size_t)r];
            x.len = res.len[j];
            x.pad = 0;
            x.out_off = tot;
            const int64_t k = res.row_ne[(size_t)r];
            x.src = k < 0 ? 0 : (int64_t)(uintptr_t)(res.bptr[j] + k * res.cap[j]);
            al->out_off[(size_t)r] = tot;
            tot += x.len;
        }
    }
    al->out_off[(size_t)n_rows] = tot;
    al->out.resize((size_t)std::max<int64_t>(tot, 1));
    if (n_rows && tot) {
        al->d_gather.ensure(g.size());
        al->d_out.ensure((size_t)tot);
        NPGX_HIP(hipMemcpyAsync(al->d_gather.p, g.data(), g.size() * sizeof(GatherRow),
                                hipMemcpyHostToDevice, st));
        size_t tg = al->timer.begin("gather_rows", st, double(tot) * 2.0, tot);
        hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)g.size()), dim3(64), 0, st, al->d_gather.p,
                           (int64_t)g.size(), al->d_out.p);
        NPGX_HIP(hipGetLastError());
        al->timer.end(tg, st);
        NPGX_HIP(hipMemcpyAsync(al->out.data(), al->d_out.p, (size_t)tot, hipMemcpyDeviceToHost, st));
        NPGX_HIP(stream_wait(st));
    }
    al->has_result = true;
}

void aligner_timer_reset(npgx_aligner* al) { al->timer.reset(); }
void aligner_note_epoch(npgx_aligner* al, uint32_t epoch) { al->epoch_base = std::max(al->epoch_base, epoch + 1); }
void aligner_set_long_head(npgx_aligner* al, int32_t long_head) { al->long_head = std::max(0, long_head); }
int32_t aligner_long_head(const npgx_aligner* al) { return al->long_head; }
const std::vector<int64_t>& aligner_job_stats(const npgx_aligner* al) { return al->job_stats; }
bool aligner_wants_stats(const npgx_aligner* al) { return al->want_stats; }
void aligner_host_ms(npgx_aligner* al, double* prep, double* wait) {
    *prep = al->host_ms[0];
    *wait = al->host_ms[1];
    al->host_ms[0] = al->host_ms[1] = 0;
}
hipStream_t aligner_stream(const npgx_aligner* al) { return al->stream; }

const char* aligner_result(const npgx_aligner* al, const int64_t** row_off) {
    *row_off = al->out_off.data();
    return al->out.data();
}

}  // namespace npgx

extern "C" {

void npgx_align_default_options(npgx_align_options* o) {
    if (!o) return;
    memset(o, 0, sizeof(*o));
    o->mismatch_check = 1;        // MISMATCH_CHECK
    o->gap_check = 2;             // GAP_CHECK
    o->aligned_check = 10;        // ALIGNED_CHECK
    o->min_length = 100;          // MIN_LENGTH
    o->min_identity_x1e4 = 9000;  // MIN_IDENTITY 0.9
    o->aligner_type = 0;
    o->refine = 0;
}

int npgx_aligner_create(const npgx_align_options* o, npgx_aligner** out) {
    return guard([&] {
        NPGX_REQUIRE(o && out, NPGX_ERR_ARG, "null argument");
        NPGX_REQUIRE(o->mismatch_check >= 0 && o->gap_check >= 1 && o->aligned_check >= 1 &&
                         o->aligned_check <= 16 && o->min_length >= 0,
                     NPGX_ERR_ARG, "aligner option out of range");
        NPGX_REQUIRE(o->aligner_type == 0 || o->aligner_type == 1, NPGX_ERR_ARG, "unknown aligner type");
        NPGX_REQUIRE(o->refine == 0, NPGX_ERR_ARG, "refine_alignment is not available yet");
        int dev = current_device_checked();
        auto* a = new npgx_aligner;
        a->opt = *o;
        a->device = dev;
        const char* js = getenv("NPGX_JOB_STATS");
        a->want_stats = js && js[0] == '1';
        const char* df = getenv("NPGX_ALIGN_DEFER");
        if (df && *df) a->defer = std::max(0, atoi(df));
        const char* dr = getenv("NPGX_ALIGN_DEFER_ROWS");
        if (dr && *dr) a->defer_rows = std::max(0, atoi(dr));
        const char* sp = getenv("NPGX_ALIGN_SPLIT");
        if (sp && *sp) a->split = std::max(0, atoi(sp));
        const char* lh = getenv("NPGX_LONG_HEAD");
        if (lh && *lh) a->long_head = std::max(0, atoi(lh));
        const char* ll = getenv("NPGX_LONG_LDS");
        if (ll && *ll) a->long_lds = atoi(ll) != 0;
        const char* wm = getenv("NPGX_SA_MANY_AT");
        if (wm && *wm) a->waves_many_at = std::max(0ll, atoll(wm));
        const char* lm = getenv("NPGX_LONG_M");
        if (lm && *lm) a->long_m = std::max(64, atoi(lm));
        const char* sf = getenv("NPGX_SEG_FULL_MB");
        if (sf && *sf) a->seg_full_bytes = (int64_t)std::max(0, atoi(sf)) << 20;
        const char* tw = getenv("NPGX_TWINS");
        if (tw && *tw) a->twins = atoi(tw) > 0 ? 1 : (atoi(tw) == 0 ? 0 : -1);
        const char* ut = getenv("NPGX_UTWINS");
        if (ut && *ut) a->utw_rows = std::max(0, atoi(ut));
        const char* utt = getenv("NPGX_UTWIN_TASKS");
        if (utt && *utt) a->utw_max_tasks = std::max(0, atoi(utt));
        const char* sb = getenv("NPGX_SLOT_BUDGET_MB");
        if (sb && *sb) {
            a->slot_budget = (int64_t)std::max(1, atoi(sb)) << 20;
        } else {
            a->slot_budget = 16ll << 30;
        }
        if (hipStreamCreateWithFlags(&a->stream, hipStreamNonBlocking) != hipSuccess) {
            delete a;
            throw Error(NPGX_ERR_HIP, "stream creation failed");
        }
        // dynamic LDS of each kernel at most (k_split_post and k_fin_copy also
        // have static LDS)
        const std::pair<const void*, int> kernels[12] = {
            {(const void*)k_align_jobs<true, SA_WAVES_PER_EU>, (int)LDS_PER_CU},
            {(const void*)k_align_sub<true, SA_WAVES_PER_EU>, (int)LDS_PER_CU},
            {(const void*)k_align_jobs<false, SA_WAVES_PER_EU>, (int)LDS_PER_CU},
            {(const void*)k_align_sub<false, SA_WAVES_PER_EU>, (int)LDS_PER_CU},
            {(const void*)k_align_jobs<true, SA_WAVES_MANY>, (int)LDS_PER_CU},
            {(const void*)k_align_sub<true, SA_WAVES_MANY>, (int)LDS_PER_CU},
            {(const void*)k_align_jobs<false, SA_WAVES_MANY>, (int)LDS_PER_CU},
            {(const void*)k_align_sub<false, SA_WAVES_MANY>, (int)LDS_PER_CU},
            {(const void*)k_align_finish<true>, (int)LDS_PER_CU}, {(const void*)k_align_finish<false>, (int)LDS_PER_CU},
            {(const void*)k_split_post, (int)POST_LDS},          {(const void*)k_fin_copy, 32768 * 4}};
        bool lds_ok = true;
        for (const auto& k : kernels)
            lds_ok = lds_ok && hipFuncSetAttribute(k.first, hipFuncAttributeMaxDynamicSharedMemorySize, k.second) ==
                                   hipSuccess;
        if (!lds_ok) {
            (void)hipStreamDestroy(a->stream);
            delete a;
            throw Error(NPGX_ERR_HIP, "cannot enable 160 KiB of LDS for the aligner");
        }
        *out = a;
    });
}

int npgx_align_batch(npgx_aligner* a, const char* rows, const int64_t* row_off,
                     const int32_t* job_row_start, int32_t n_jobs) {
    return guard([&] {
        NPGX_REQUIRE(a && (n_jobs == 0 || (rows && row_off && job_row_start)), NPGX_ERR_ARG,
                     "null argument");
        align_batch(a, rows, row_off, job_row_start, n_jobs);
    });
}

int npgx_align_result_sizes(const npgx_aligner* a, int64_t* total_bytes) {
    return guard([&] {
        NPGX_REQUIRE(a && total_bytes, NPGX_ERR_ARG, "null argument");
        NPGX_REQUIRE(a->has_result, NPGX_ERR_STATE, "no alignment result yet");
        *total_bytes = a->out_off.empty() ? 0 : a->out_off.back();
    });
}

int npgx_align_result_copy(const npgx_aligner* a, char* out, int64_t* out_off, int64_t* job_len) {
    return guard([&] {
        NPGX_REQUIRE(a, NPGX_ERR_ARG, "null argument");
        NPGX_REQUIRE(a->has_result, NPGX_ERR_STATE, "no alignment result yet");
        if (out && !a->out_off.empty()) memcpy(out, a->out.data(), (size_t)a->out_off.back());
        if (out_off) memcpy(out_off, a->out_off.data(), a->out_off.size() * 8);
        if (job_len) memcpy(job_len, a->job_len.data(), a->job_len.size() * 8);
    });
}

int npgx_align_job_stats(const npgx_aligner* a, int64_t* out, int64_t cap, int64_t* n) {
    return guard([&] {
        NPGX_REQUIRE(a && n, NPGX_ERR_ARG, "null argument");
        NPGX_REQUIRE(a->has_result, NPGX_ERR_STATE, "no alignment result yet");
        *n = (int64_t)a->job_stats.size() / NPGX_JOB_STATS;
        if (out) memcpy(out, a->job_stats.data(), (size_t)std::min<int64_t>(cap, *n) * NPGX_JOB_STATS * 8);
    });
}

int npgx_align_kernel_times(const npgx_aligner* a, npgx_kernel_time* out, int32_t cap, int32_t* n) {
    return guard([&] {
        NPGX_REQUIRE(a && n && (out || cap == 0), NPGX_ERR_ARG, "null argument");
        a->timer.copy_out(out, cap, n);
    });
}

void npgx_aligner_free(npgx_aligner* a) {
    if (!a) return;
    (void)hipSetDevice(a->device);
    if (a->stream) (void)hipStreamDestroy(a->stream);
    wide_free(a->wide);
    delete a;
}

}  // extern "C"
