/*
 * npge_amd.h -- C ABI of the MI355X-native anchor-finding / greedy-MSA engine
 * for NPG-explorer's block-construction hot path.
 *
 * Plain pointers and sizes only.  Every handle owns one hipStream_t and lives on
 * the device that was current (npgx_set_device) when it was created; handles
 * are not thread-safe.  The caller owns inputs; the library owns outputs until
 * the matching *_free.  All functions return NPGX_OK (0) or a negative code;
 * npgx_last_error() returns the thread-local message of the last failure.
 *
 * Reference interfaces replaced (paths in NPG-explorer 0.5.8):
 *   npgx_seqset_*   Sequence storage + SeqBase::make_seqs ranking
 *                   (src/model/Sequence.cpp:151-179,525-600; src/algo/SeqI.hpp:45-57)
 *   npgx_af_*       Processor "AnchorFinder" (src/algo/AnchorFinder.hpp:33-53,
 *                   AnchorFinder.cpp:37-53 options, :393-406 run_impl)
 *   npgx_blockset_* Processor/BlockSet surface of the block build (below)
 *   npgx_align_*    AbstractAligner::align_seqs + SimilarAligner::similar_aligner
 *                   (src/algo/AbstractAligner.cpp:104-143,
 *                   src/algo/SimilarAligner.cpp:487-501), MetaAligner
 *                   "aligner-type" similar|dummy (src/algo/MetaAligner.cpp:22-84)
 */
#ifndef NPGE_AMD_H_
#define NPGE_AMD_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NPGX_OK 0
#define NPGX_ERR_ARG (-1)      /* bad argument / option rule violated */
#define NPGX_ERR_HIP (-2)      /* HIP runtime failure */
#define NPGX_ERR_NODEV (-3)    /* no usable GPU */
#define NPGX_ERR_RANGE (-4)    /* input outside supported sizes */
#define NPGX_ERR_STATE (-5)    /* result requested before a run */

typedef struct npgx_seqset npgx_seqset;
typedef struct npgx_af npgx_af;
typedef struct npgx_aligner npgx_aligner;

/* ------------------------------------------------------------------ runtime */
const char* npgx_last_error(void);
const char* npgx_version(void);
int npgx_device_count(int32_t* n);
int npgx_set_device(int32_t device);

/* Per-kernel timing of the last run of a handle (HIP events on the handle's
 * stream).  bytes = algorithmic bytes of that launch. */
typedef struct {
    char name[32];
    double ms;
    double bytes;
    int64_t units;   /* windows / residues processed by the launch */
} npgx_kernel_time;

/* ------------------------------------------------------------------ sequences
 * Creates a device-resident, 2-bit packed (A0 T1 G2 C3, LSB first) sequence set
 * with an N bitmap.  Input strings go through Sequence::to_atgcn
 * (uppercase, IUPAC -> N, other characters dropped).  Sequences are ranked by
 * (size desc, name asc, input index asc) -- the pinned form of the reference's
 * unstable size sort (SeqI.hpp:54).  names may be NULL (empty names).
 * Thread-safe; creations of sets up to 256 MiB of text share one pinned
 * staging buffer and run their upload one at a time. */
int npgx_seqset_create(const char* const* seqs, const int64_t* lens,
                       const char* const* names, int32_t n, npgx_seqset** out);
int npgx_seqset_count(const npgx_seqset* s, int32_t* n);
/* wall ms of npgx_seqset_create: the host's to_atgcn (the CPU side's input
 * conversion, excluded from throughput) and the upload proper -- one DMA of
 * the ASCII text from pinned staging plus k_pack (H2D included
 * on the GPU side) */
int npgx_seqset_timings(const npgx_seqset* s, double* ms_host, double* ms_upload);
/* size after to_atgcn of input sequence `index` */
int npgx_seqset_size(const npgx_seqset* s, int32_t index, int64_t* size);
/* rank of input sequence `index` in the processing order */
int npgx_seqset_rank(const npgx_seqset* s, int32_t index, int32_t* rank);
/* copies the ATGCN text of [start, start+len) of sequence `index` into out */
int npgx_seqset_text(const npgx_seqset* s, int32_t index, int64_t start, int64_t len,
                     char* out);
/* total device bytes held (packed words + N bitmap) */
int npgx_seqset_device_bytes(const npgx_seqset* s, int64_t* bytes);
void npgx_seqset_free(npgx_seqset* s);

/* ------------------------------------------------------------------ AnchorFinder
 * Options mirror AnchorFinder's (AnchorFinder.cpp:37-53, CMakeLists.txt:41-45):
 *   anchor-size (1..32, default 20), anchor-fp (Decimal, default 0.1 -> 1000),
 *   anchor-similar (default 1), max-anchor-fragments (default 100000).
 * The Bloom hash parameters are glibc rand() after srand(bloom_seed) -- the
 * reference draws them after srand(make_seed()) (BloomFilter.cpp:55-63) -- or the
 * explicit vector bloom_params[0..n_bloom_params) when n_bloom_params > 0. */
typedef struct {
    int32_t anchor_size;
    int32_t anchor_similar;
    int64_t anchor_fp_x1e4;
    int64_t max_anchor_fragments;
    uint32_t bloom_seed;
    int32_t n_bloom_params;
    const uint64_t* bloom_params;
    /* one-GPU Bloom pass in epochs of consecutive windows (a bit array of the
     * earlier epochs filters atomics and reads; same result): 0 = automatic
     * (about 2M windows per epoch), 1 = a single pass, k = k epochs */
    int32_t bloom_epochs;
    int32_t pad0;
} npgx_af_options;

void npgx_af_default_options(npgx_af_options* o);

typedef struct {
    int64_t members;        /* estimate_length (AnchorFinder.cpp:81-97) after 4^k cap */
    int64_t bloom_bits;     /* optimal_bits (BloomFilter.cpp:147-156) */
    int32_t bloom_hashes;   /* optimal_hashes (BloomFilter.cpp:158-164) */
    int32_t pad0;
    uint64_t bloom_params[32];
    int64_t n_windows;      /* windows scanned per pass (sum of size-k+1) */
    int64_t n_collected_raw;/* collected windows (before sort/unique) */
    int64_t n_collected;    /* |H| after sort + unique */
    int64_t n_found_frags;  /* FoundFragments before truncation */
    int64_t n_kept_groups;  /* hash groups materialised before truncation */
    int64_t n_blocks;
    int64_t n_fragments;
    int64_t n_used;         /* size of the persistent used-hash set */
} npgx_af_stats;

/* The handle owns the persistent used-hash set (AnchorFinder.cpp:30-35): runs on
 * the same handle skip hashes recorded by earlier runs, like the reference's
 * processor instance cached by MetaProcessor (MetaProcessor.cpp:32-38). */
int npgx_af_create(const npgx_af_options* o, npgx_af** out);
int npgx_af_run(npgx_af* af, const npgx_seqset* s);
int npgx_af_stats_get(const npgx_af* af, npgx_af_stats* out);
/* Result of the last run, in reference order: blocks in FoundFragment (hash)
 * order, fragments inside a block by (sequence rank, direct before reverse,
 * position).  seq[] holds the INPUT index of the sequence; ori is +1/-1. */
int npgx_af_result_counts(const npgx_af* af, int64_t* n_blocks, int64_t* n_fragments);
int npgx_af_result_copy(const npgx_af* af, int64_t* block_start /* n_blocks+1 */,
                        int32_t* seq, int64_t* min_pos, int64_t* max_pos, int8_t* ori);
int npgx_af_used_hashes(const npgx_af* af, uint64_t* out, int64_t cap, int64_t* n);
int npgx_af_clear_used(npgx_af* af);
int npgx_af_kernel_times(const npgx_af* af, npgx_kernel_time* out, int32_t cap, int32_t* n);
void npgx_af_free(npgx_af* af);

/* ------------------------------------------------------------------ multi-GPU
 * Exact sharding of ONE AnchorFinder run over `world` ranks (one process per
 * GPU).  The windows of the run are split into contiguous
 * ranges, one per rank; the result equals npgx_af_run on one GPU bit for bit.
 * The exchange steps go through caller-supplied collectives (the host binds
 * them to torch.distributed -- RCCL over xGMI on MI355X, gloo in tests):
 *   1. the Bloom bit arrays (m / 8 bytes per rank): all-gather; each rank
 *      ORs the lower ranks' arrays, whose windows all precede its own, and
 *      tests its windows against that OR and its own first-setter orders (the
 *      reference's sequential "bits set by an earlier window", BloomFilter.cpp
 *      :65-76, AnchorFinder.cpp:170-197); then every rank's last window
 *      (order, found): all-gather of one value (the `similar` rule across a
 *      rank boundary, :185-192);
 *   2. the collected hashes (bloomtg_postprocess :213-218): all-gather;
 *   3. FoundFragment counts per hash (truncation :356-391): SUM;
 *   4. the FoundFragment keys of the kept groups: all-gather.
 * Every rank ends with the whole result and the same used-hash set.
 * Callbacks return 0 on success; buffers named dev live in device memory of
 * the handle's device, the library's stream is idle when a callback runs, and
 * the callback must have finished its writes when it returns.  Every rank
 * must call npgx_af_run_sharded with the same inputs and options. */
#define NPGX_OP_SUM 0
#define NPGX_OP_MIN 1
typedef struct {
    int32_t rank;
    int32_t world;
    void* user;
    /* in-place element-wise reduction of n int32 values (op NPGX_OP_SUM/MIN) */
    int (*allreduce_i32)(void* user, int32_t* dev, int64_t n, int32_t op);
    /* out[r] = value of rank r (host memory, world entries) */
    int (*allgather_i64)(void* user, int64_t value, int64_t* out);
    /* concatenation in rank order of counts[r] uint64 values from each rank
     * into dev_out (capacity sum(counts)); counts is host memory */
    int (*allgatherv_u64)(void* user, const uint64_t* dev_in, const int64_t* counts,
                          uint64_t* dev_out);
} npgx_comm;

int npgx_af_run_sharded(npgx_af* af, const npgx_seqset* s, const npgx_comm* comm);

/* A library-owned npgx_comm over RCCL (xGMI), one process per GPU: rank 0
 * makes the unique id (NPGX_RCCL_ID_BYTES bytes) and the launcher hands it to
 * every rank before each calls npgx_rccl_comm_create on its own device.  The
 * collectives run on the communicator's stream with device buffers in and out
 * (ncclAllReduce, ncclAllGather, grouped ncclBroadcast for the variable
 * all-gather).  Free with npgx_rccl_comm_free after every handle using it. */
#define NPGX_RCCL_ID_BYTES 128
int npgx_rccl_unique_id(void* out);
int npgx_rccl_comm_create(const void* unique_id, int32_t rank, int32_t world, int32_t device,
                          npgx_comm** out);
void npgx_rccl_comm_free(npgx_comm* comm);
/* the rank count RCCL itself reports for a communicator made by
 * npgx_rccl_comm_create (ncclCommCount); bench.py puts it in its line */
int npgx_rccl_comm_count(const npgx_comm* comm, int32_t* n);
/* Runs every collective of comm on small device buffers and checks the
 * results (a start-up check of a multi-GPU run; collective on all ranks). */
int npgx_comm_check(const npgx_comm* comm);

/* Copies bytes between any two of host/device memory (hipMemcpyDefault);
 * for host-side collective adapters. */
int npgx_memcpy(void* dst, const void* src, int64_t bytes);

/* ------------------------------------------------------------------ aligner
 * Batched AbstractAligner::align_seqs with aligner-type "similar"
 * (SimilarAligner) or "dummy" (DummyAligner).  A batch holds n_jobs independent
 * alignment problems (one per block); job j owns rows
 * [job_row_start[j], job_row_start[j+1]) and row r is the text
 * rows[row_off[r] .. row_off[r+1]).  Similar-aligner rows must be upper-case
 * ATGCN (the sequences' to_atgcn alphabet); dummy rows may hold anything.
 * Options (SimilarAligner.cpp:503-516, CMakeLists.txt:35-37,55-60): */
typedef struct {
    int32_t mismatch_check;     /* default 1 */
    int32_t gap_check;          /* default 2 */
    int32_t aligned_check;      /* default 10 */
    int32_t min_length;         /* default 100 */
    int64_t min_identity_x1e4;  /* default 9000 (Decimal 0.9) */
    int32_t aligner_type;       /* 0 = similar, 1 = dummy */
    int32_t refine;             /* 1 = also refine_alignment (align_block) */
} npgx_align_options;

void npgx_align_default_options(npgx_align_options* o);
int npgx_aligner_create(const npgx_align_options* o, npgx_aligner** out);
int npgx_align_batch(npgx_aligner* a, const char* rows, const int64_t* row_off,
                     const int32_t* job_row_start, int32_t n_jobs);
/* Output of the last batch: job j's aligned rows all have length out_len[j];
 * row r's gapped text is out[out_off[r] .. out_off[r] + out_len[job(r)]). */
int npgx_align_result_sizes(const npgx_aligner* a, int64_t* total_bytes);
int npgx_align_result_copy(const npgx_aligner* a, char* out, int64_t* out_off,
                           int64_t* job_len);
int npgx_align_kernel_times(const npgx_aligner* a, npgx_kernel_time* out, int32_t cap,
                            int32_t* n);
/* per job of the last batch, NPGX_JOB_STATS int64: 0 device cycles,
 * 1 alignment columns, 2 try_aligned calls, 3 shifts scanned, 4 try_gap calls,
 * 5 FindLowSimilar regions, 6 non-empty rows, 7 columns-mode chunks; cycles
 * of 8 process_seqs, 9 fix_bad_regions, 10 realing_end; 11 wall_clock64() at
 * the job's start (constant-rate device clock, 23 at its end); and,
 * in a library built with NPGX_SA_PROFILE, cycles inside process_seqs of
 * 12 columns-mode runs, 13 rows-mode equal/mismatch steps, 14 try_gap,
 * 15 try_aligned, 16 vector word building, 17 vector word compares,
 * 18 vector chunks, 19 vector calls, 20 append_end, 21 returns from
 * append_aligned (0 otherwise); 22 cycles of the region search */
#define NPGX_JOB_STATS 24
int npgx_align_job_stats(const npgx_aligner* a, int64_t* out, int64_t cap, int64_t* n);
void npgx_aligner_free(npgx_aligner* a);

/* refine_alignment (replaces refine_alignment(Strings&), src/algo/refine_alignment.cpp:
 * 182-190, the step AbstractAligner::align_block runs after align_seqs) for a
 * batch of alignments on the GPU: alignment j = rows [job_row_start[j],
 * job_row_start[j+1]), row r = rows[row_off[r] .. row_off[r+1]), the rows of
 * one alignment of equal length and consecutive in `rows`.  The refined rows
 * go to out at the same offsets; only their first out_len[j] characters are
 * valid (pure-gap columns are removed). */
int npgx_refine_batch(const char* rows, const int64_t* row_off, const int32_t* job_row_start, int32_t n_jobs,
                      char* out, int32_t* out_len);


/* ------------------------------------------------------------------ block sets
 * A block set over a sequence set: blocks of fragments (sequence input index,
 * min_pos, max_pos, ori) with optional gapped rows ('-' = gap).  Processors run
 * in place.  Names and semantics follow the reference processors:
 *   "RemoveNonStem"      RemoveNonStem --exact (src/algo/RemoveNonStem.cpp:29-45)
 *   "DummyAligner"       AbstractAligner::align_block with DummyAligner
 *                        (AbstractAligner.cpp:51-69, DummyAligner.cpp:18-26)
 *   "MetaAligner"        align_block with aligner-type similar: the blocks
 *                        alignment_needed selects aligned on the GPU, then
 *                        refine_alignment (AbstractAligner.cpp:51-69,145-177,
 *                        refine_alignment.cpp:15-190)
 *   "Align"              Align (src/algo/Align.cpp:36-52): MetaAligner,
 *                        SelfOverlapsResolver, MetaAligner, then the loop
 *                        {MoveGaps, CutGaps, Filter} until the block set repeats
 *   "LiteAlign"          LiteAlign (Align.cpp:17-30): MetaAligner, then the
 *                        loop {MoveGaps, CutGaps}
 *   "MoveGaps"           MoveGaps (src/algo/MoveGaps.cpp:30-103); options
 *                        --max-tail=N --max-tail-to-gap=D
 *   "CutGaps"            CutGaps (src/algo/CutGaps.cpp:136-159); option
 *                        --cut-strict=0|1
 *   "SelfOverlapsResolver" fix_self_overlaps (src/algo/hit.cpp:68-91)
 *   "Rest"               Rest target=X other=X (src/algo/Rest.cpp:40-77)
 *   "OverlaplessUnion"   OverlaplessUnion --ou-move into an empty target
 *                        (src/algo/OverlaplessUnion.cpp:54-80)
 *   "AnchorLoopFast"     the AnchorLoopFast pipe (lua_lib.lua:741-758), af =
 *                        its AnchorFinder
 *   "AnchorLoop"         the AnchorLoop pipe (lua_lib.lua:711-737) as a fresh
 *                        pipe, af = its AnchorFinder: ConSeq, AnchorFinder,
 *                        DummyAligner, UniqueNames (UniqueNames.cpp:23-67),
 *                        ExtendAndAlign, RemoveWithSameName
 *                        (RemoveWithSameName.cpp:28-58), SplitExtendable
 *                        (SplitExtendable.cpp:46-84), RemoveNames, DeConSeq,
 *                        ExtendLoop on both sets, DeConSeq, Align
 *   "ExtendLoop"         Pipe ExtendLoop (lua_lib.lua:677-688) to its fixpoint
 *   "AddingLoopBySize"   AddingLoopBySize (src/algo/TrySmth.cpp:157-178) of all
 *                        blocks into an empty target (SmthUnion, :35-155)
 *   "FragmentsExtender"  FragmentsExtender (src/algo/FragmentsExtender.cpp:87-119)
 *   "FixEnds"            FixEnds (src/algo/FixEnds.cpp:117-144)
 *   "ExtendLoopFast"     Pipe ExtendLoopFast (src/algo/lua_lib.lua:697-709,
 *                        src/algo/Pipe.cpp:60-78)
 *   "Filter"             Filter (src/algo/Filter.cpp:208-248)
 *   "DraftPangenome"     AnchorFinder -> RemoveNonStem -> DummyAligner ->
 *                        ExtendLoopFast -> Filter (lua_lib.lua:1569-1621) */
typedef struct npgx_blockset npgx_blockset;

typedef struct {
    int32_t extend_length;          /* FragmentsExtender extend-length (MIN_LENGTH 100) */
    int32_t max_iterations;         /* ExtendLoopFast iterations (DraftPangenome: 10) */
    int64_t extend_portion_x1e4;    /* FragmentsExtender extend-length-portion: default 0
                                     * (FragmentsExtender.cpp:28-30); ExtendAndFix /
                                     * ExtendAndAlign (inside ExtendLoopFast, AnchorLoopFast)
                                     * pass 0.5 themselves, whatever this holds */
    int32_t min_fragment;           /* FixEnds / Filter min-fragment (MIN_LENGTH) */
    int32_t frame_length;           /* Filter frame-length (FRAME_LENGTH 100) */
    int32_t min_end;                /* Filter min-end (MIN_END 10) */
    int32_t min_block;              /* Filter min-block (2) */
    int32_t max_block;              /* Filter max-block (-1) */
    int32_t find_subblocks;         /* Filter find-subblocks (1) */
    int64_t min_identity_x1e4;      /* FixEnds / Filter min-identity (MIN_IDENTITY 0.9) */
    npgx_align_options align;       /* aligner used by FragmentsExtender */
    int32_t max_tail;               /* MoveGaps max-tail (MAX_TAIL 3) */
    int64_t max_tail_to_gap_x1e4;   /* MoveGaps max-tail-to-gap (MAX_TAIL_TO_GAP 1.0) */
} npgx_bb_options;

typedef struct {
    int64_t iterations;             /* ExtendLoopFast iterations run */
    int64_t aligned_residues;       /* flank residues sent to the aligner */
    int64_t align_jobs;             /* alignment problems solved */
    int64_t anchor_blocks;
    int64_t stem_blocks;
    double ms_align;                /* wall ms inside the GPU aligner */
    double ms_host;                 /* wall ms of host bookkeeping */
    /* wall ms per stage of the last apply: 0 AnchorFinder, 1 RemoveNonStem +
     * DummyAligner, 2 MoveUnchanged, 3 flank gather, 4 align batch, 5 stitch,
     * 6 FixEnds, 7 OverlaplessUnion, 8 blockset hash, 9 Filter,
     * 10 aligner host preparation, 11 the host's waits on the device (the
     * aligner's kernels in the host loop; each iteration's GPU work in the
     * device loop, whose other entries are then enqueue times), 12 FixEnds
     * device part, 13 FixEnds slicing, 14 OverlaplessUnion order,
     * 15 OverlaplessUnion admission */
    double ms_stage[16];
    /* 0 blocks after ExtendLoopFast, 1 blocks passing Filter whole, 2 blocks
     * sent to goodSlices, 3 blocks after Filter, 4 blocks into OverlaplessUnion
     * (all iterations), 5 of them rejected, 6 block hashes computed (host), 7
     * ExtendLoopFast on the device: OverlaplessUnion runs handed to the host
     * (AnchorLoop: AddingLoopBySize rounds) */
    int64_t counters[8];
    /* AnchorLoopFast: 0 consensus sequences, 1 anchor blocks on them, 2
     * consensus blocks after the pipe's ExtendLoopFast, 3 blocks DeConSeq
     * added, 4 the consensus ExtendLoopFast's iterations, 5 consensus blocks
     * MoveUnchanged dropped.  AnchorLoop: 0 consensus sequences, 1 anchor
     * blocks on them, 2 anchors left for SplitExtendable, 3 its blocks, 4
     * consensus blocks after ExtendLoop, 5 deconseq blocks after ExtendLoop,
     * 6 / 7 the two ExtendLoop's iterations (AnchorLoop: counters[7] =
     * AddingLoopBySize rounds, ms_loop = 0 Filter..AnchorFinder, 1
     * DummyAligner..RemoveWithSameName, 2 SplitExtendable, 3 DeConSeq, 4 / 5
     * the two ExtendLoops, 6 DeConSeq, 7 Align) */
    int64_t loop[8];
    /* AnchorLoopFast wall ms: 0 Filter + Rest + order, 1 ConSeq, 2 AnchorFinder
     * on the consensus sequences, 3 MoveUnchanged + DummyAligner, 4
     * ExtendAndAlign (FragmentsExtender + Align), 5 ExtendLoopFast, 6 DeConSeq,
     * 7 the closing Align (the consensus pipe's stages add into ms_stage) */
    double ms_loop[8];
    /* DraftPangenome's GPU timeline with the "stage-clock" tuning on (else 0):
     * ms between HIP events recorded on the set's stream at the stage
     * boundaries, so the entries sum to the step's span on the GPU (kernels
     * plus the idle time the host leaves between them): 0 AnchorFinder (its
     * kernels, grouping, anchor blocks), 1 RemoveNonStem + DummyAligner, 2
     * ExtendLoopFast table upload, 3 per iteration: block_hash, Pipe state,
     * MoveUnchanged, flank plan + its download and the host's batch arrays,
     * 4 flank decode, 5 aligner (k_align_jobs and its re-runs / sub-jobs),
     * 6 stitch, 7 FixEnds + slicing, 8 OverlaplessUnion, 9 the blocks'
     * download, 10 Filter, 11 ExtendLoopFast on the host (host loop only) */
    double ms_gpu[12];
    /* ExtendLoopFast iterations the device loop ran (ms_align and ms_stage 3-8
     * are then host enqueue times: the GPU time is in ms_gpu) */
    int64_t device_iterations;
    /* ... of which the aligner ran synchronously because the asynchronous
     * form's planned memory passed its budget (NPGX_ASYNC_BUDGET_MB) or a
     * problem had more than 64 rows */
    int64_t device_sync_iterations;
} npgx_bb_stats;

void npgx_bb_default_options(npgx_bb_options* o);
int npgx_blockset_create(const npgx_seqset* s, const npgx_bb_options* o, npgx_blockset** out);
/* as npgx_blockset_create, but the new set borrows lender's aligner (its device
 * scratch and HIP stream) instead of making one: the two sets must not run at
 * the same time (one host thread), and lender must outlive the new set.  The
 * pair-sharded job (npge_amd/pairs.py) runs its pairs this way, one lender per
 * worker thread.  No reference counterpart: a device-memory sharing hint. */
int npgx_blockset_create_sharing(const npgx_seqset* s, const npgx_bb_options* o, npgx_blockset* lender,
                                 npgx_blockset** out);
/* tuning hooks with no reference counterpart (results never change):
 *   "long-head"  the set's aligner searches that many shifts incrementally
 *                before the prefix search (default 128); 0 = incremental only,
 *                and the aligner then launches its kernels without the prefix
 *                search's call (less scratch: the form for many concurrent
 *                streams, e.g. the pair job).  Sets sharing the aligner share it.
 *   "elf-device" ExtendLoopFast on the device (1), on the host (0) or the
 *                default (-1, the device where its rules allow); sets made by
 *                npgx_blockset_create_sharing inherit the lender's, and so do
 *                the sets a pipe makes internally (AnchorLoopFast's and
 *                AnchorLoop's consensus sets).
 *   "stage-clock" 1: DraftPangenome records HIP events at its stage
 *                boundaries and fills npgx_bb_stats.ms_gpu (each marker costs
 *                the GPU a few microseconds: diagnostics only); 0: off (default).
 * NPGX_ERR_ARG for an unknown key or a value out of range. */
int npgx_blockset_tune(npgx_blockset* b, const char* key, int64_t value);
/* replace the blocks; row_off == NULL: no rows, else row i = rows[row_off[i]..row_off[i+1])
 * (a block whose rows are all empty is unaligned) */
int npgx_blockset_set_blocks(npgx_blockset* b, int64_t n_blocks, const int64_t* block_start,
                             const int32_t* seq, const int64_t* min_pos, const int64_t* max_pos,
                             const int8_t* ori, const int64_t* row_off, const char* rows);
/* append the blocks found by the last npgx_af_run of af */
/* Multi-GPU block build: with a comm of world > 1, DraftPangenome
 * runs npgx_af_run_sharded and every FragmentsExtender batch aligns this rank's
 * share of the jobs (longest-processing-time assignment on rows x residues)
 * and all-gathers the gapped rows; the rest of the build runs identically on
 * every rank, so every rank ends with the one-GPU block set.  The comm must
 * outlive the handle's runs; NULL (or world 1) returns to one GPU. */
int npgx_blockset_set_comm(npgx_blockset* b, const npgx_comm* comm);
int npgx_blockset_add_anchors(npgx_blockset* b, const npgx_af* af);
/* run a processor by its reference name (see above); DraftPangenome uses af */
int npgx_blockset_apply(npgx_blockset* b, const char* processor, npgx_af* af);
int npgx_blockset_counts(const npgx_blockset* b, int64_t* n_blocks, int64_t* n_fragments,
                         int64_t* row_bytes);
int npgx_blockset_copy(const npgx_blockset* b, int64_t* block_start, int32_t* seq,
                       int64_t* min_pos, int64_t* max_pos, int8_t* ori, int64_t* row_off,
                       char* rows);
/* A 64-bit digest of every gapped row, each bound to its fragment, computed on
 * the device (no row crosses PCIe); it pins the gap columns the way
 * npgx_blockset_hash pins the coordinates (rows as RawWrite writes them,
 * src/algo/RawWrite.cpp:40-59).  With sm(x) = splitmix64's output function of
 * x + 0x9E3779B97F4A7C15 and, per fragment with a row (seq = input index),
 *   key = sm(sm(sm(2 * seq + (ori > 0)) + min) + max),
 *   digest = sum over those rows of [ sm(key + len)
 *            + sum over columns c of sm(key ^ (c << 8 | row[c])) ]  (mod 2^64).
 * Independent of the block order; blocks without rows add nothing.  No
 * reference counterpart (tests/helpers.py restates it in numpy). */
int npgx_blockset_rows_digest(npgx_blockset* b, uint64_t* digest);
/* blockset_hash (src/model/block_hash.cpp:112-130) */
int npgx_blockset_hash(const npgx_blockset* b, uint64_t* hash);
/* ConSeq (replaces ConSeq::process_block_impl, src/algo/ConSeq.cpp:37-50):
 * the text of the sequence each block becomes, in block order -- one
 * fragment: its text (FragmentSequence); aligned: Block::consensus
 * (Block.cpp:147-185, per column the most frequent of A T G C N, first in
 * that order on ties, 'A' for a column without letters), computed on the
 * GPU; unaligned: the first longest fragment's text.  Call with out == NULL
 * for *n_blocks and *total, then with out (total bytes) and out_off
 * (n_blocks + 1 offsets). */
int npgx_blockset_conseq(npgx_blockset* b, char* out, int64_t* out_off, int64_t* n_blocks,
                         int64_t* total);
/* DeConSeq (replaces DeConSeq::deconseq_block / deconseq_row,
 * src/algo/DeConSeq.cpp:27-96): every block of `cons` -- a block set over
 * the sequences npgx_blockset_conseq made of `source`'s blocks (sequence i =
 * source block i, source unchanged since) -- becomes a block over source's
 * sequences: each fragment is Block::slice (Block.cpp:238-289) of its source
 * block at the fragment's consensus columns, aligned fragments compose their
 * rows.  The new blocks are appended to `target`, whose sequences equal
 * source's (target may be source).  NPGX_ERR_STATE when cons does not
 * match source. */
int npgx_blockset_deconseq(npgx_blockset* target, npgx_blockset* source, npgx_blockset* cons);
int npgx_blockset_stats(const npgx_blockset* b, npgx_bb_stats* out);
int npgx_blockset_kernel_times(const npgx_blockset* b, npgx_kernel_time* out, int32_t cap,
                               int32_t* n);
/* aligner per-job statistics of every batch of the last apply
 * (NPGX_JOB_STATS int64 per job, layout of npgx_align_job_stats) */
int npgx_blockset_job_stats(const npgx_blockset* b, int64_t* out, int64_t cap, int64_t* n);
/* AnchorLoopFast keeps MoveUnchanged's memory across runs on one block set
 * (the hashes of the consensus blocks earlier runs saw, MoveUnchanged.cpp:
 * 37-67, the lua pipe object's state, lua_lib.lua:741-758); this drops it, so
 * the next AnchorLoopFast acts as a freshly made pipe. */
int npgx_blockset_reset_loop(npgx_blockset* b);
void npgx_blockset_free(npgx_blockset* b);

/* ------------------------------------------------------------------ banded DP
 * GeneralAligner (src/util/GeneralAligner.hpp:28-414): banded min-cost
 * Needleman-Wunsch with gap frame 2*gap_range+1 and the max_errors stop rule
 * ("find the end of good alignment"), align() then optionally cut_tail() and
 * export_alignment(), on nucleotide contents: substitution 0 for equal non-N
 * letters, mismatch_penalty otherwise (FragmentDistance.cpp:18-21).  A batch
 * of independent pairs per call; one wave per pair on the GPU (anti-diagonal
 * wavefront).  Defaults = GeneralAligner's constructor (:39-41): gap_range 1,
 * max_errors 0, gap_penalty 1; mismatch_penalty 1.  gap_range <= 63.  Local
 * mode (find_aln, used by BSA only) is not provided. */
typedef struct npgx_dp npgx_dp;
typedef struct {
    int32_t gap_range;
    int32_t max_errors;        /* -1: no limit (the alignment is completed to the last cell) */
    int32_t gap_penalty;
    int32_t mismatch_penalty;
    int32_t cut_tail;          /* strip the bad tail (cut_tail :240-255); needs max_errors >= 0 */
} npgx_dp_options;
void npgx_dp_default_options(npgx_dp_options* o);
int npgx_dp_create(const npgx_dp_options* o, npgx_dp** out);
/* pair i = first[first_off[i] .. first_off[i+1]) against second[second_off[i] ..) */
int npgx_dp_align_batch(npgx_dp* dp, const char* first, const int64_t* first_off,
                        const char* second, const int64_t* second_off, int32_t n_pairs);
int npgx_dp_result_counts(const npgx_dp* dp, int64_t* n_pairs, int64_t* total_ops);
/* Per pair: last aligned position in first / second (-1: none), score = at()
 * of that cell (1000000 = BAD_VALUE for a completed end outside the band),
 * status (0; -1 "row and column are not last"; -2 empty input), and the
 * alignment as ops[op_off[i] .. op_off[i+1]) in order: 0 = both letters
 * (MATCH), 1 = first only (ROW_INC), 2 = second only (COL_INC). */
int npgx_dp_result_copy(const npgx_dp* dp, int32_t* first_last, int32_t* second_last,
                        int32_t* score, int32_t* status, int64_t* op_off /* n+1 */, int8_t* ops);
int npgx_dp_kernel_times(const npgx_dp* dp, npgx_kernel_time* out, int32_t cap, int32_t* n);
/* diagnostic build only (NPGX_PROFILE=1): summed per-wave cycles of the
 * forward pass and of the traceback, and the anti-diagonal steps, of the
 * last batch */
int npgx_dp_phase_cycles(const npgx_dp* dp, int64_t* fwd, int64_t* back, int64_t* steps);
void npgx_dp_free(npgx_dp* dp);

/* ---- diagnostics (host only, no device needed) ---- */
/* goodSlices (goodSlices.cpp:247-255) over n column scores as Filter runs it
 * (replaces GoodSlicer::calculate): the slices' (start, stop) pairs into out
 * (at most max_out pairs); returns their count, -1 on bad arguments. */
int npgx_diag_good_slices(const int32_t* scores, int32_t n, int32_t frame_length, int32_t end_length,
                          int32_t min_identity, int32_t min_length, int64_t* out, int32_t max_out);

#ifdef __cplusplus
}
#endif

#endif /* NPGE_AMD_H_ */
