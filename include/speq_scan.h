/*
 * speq_scan.h — C ABI of libspeq_scan.so, the MI355X-native SPeQ scan path.
 *
 * This is the drop-in boundary for the reference's hot path.
 * The reference has no FFI; its seam is the SeqAn3 library call pair
 *
 *   seqan3::fm_index{collection}            /root/reference/src/fm_indexer.cpp:36
 *   search(windows, fm_index, cfg)          /root/reference/src/fm_scanner.cpp:208 (+12 more sites)
 *
 * followed by the per-window tally `do_a_count` (fm_scanner.cpp:153-196, :426-471, :665-708, :916-962),
 * the per-thread reduction (fm_scanner.cpp:224-233 …) and the reference-uniqueness pass
 * `_async_count_unique_kmers_per_group` (fm_scanner.cpp:1476-1576).  The functions below replace that
 * seam AND the tally, so per-window hit lists never materialise: the GPU returns the counters directly.
 *
 * Conventions
 *  - Every function returns 0 on success, a negative SPEQ_E_* code on failure; the message of the last
 *    failure on the calling thread is returned by speq_last_error() (mirrors the reference's exceptions,
 *    e.g. std::logic_error at fm_scanner.cpp:69, which the C++ CLI re-raises).
 *  - Plain pointers and sizes only.  "d_" pointers are device (HBM) pointers of the device the handle was
 *    opened on; "stream" is a hipStream_t passed as void* (NULL = the default stream).
 *  - An index is immutable after build/load; a device replica may be used concurrently from many host
 *    threads (the reference copies the index per worker thread, fm_scanner.cpp:145 — we do not need to).
 *  - Product paths run on the GPU only.  There is no CPU fallback: a call that needs a device fails
 *    with SPEQ_E_DEVICE when none is present.
 */
#ifndef SPEQ_SCAN_H
#define SPEQ_SCAN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPEQ_ABI_VERSION 7

enum {
    SPEQ_OK = 0,
    SPEQ_E_ARG = -1,      /* invalid argument (shape, range, null pointer) */
    SPEQ_E_IO = -2,       /* file could not be read / written / has a bad format */
    SPEQ_E_DEVICE = -3,   /* no GPU, HIP runtime failure, or kernel launch failure */
    SPEQ_E_GROUPS = -4,   /* groupings do not cover every reference record */
    SPEQ_E_NOMEM = -5,
    SPEQ_E_RETRY = -6     /* speq_scan_fastq_shard, cut = 1: the parallel cut does not fit this file; counters and
                             EM histogram are cleared, scan again with cut = 0 (every rank) */
};

/* Scan modes: fm_scanner.cpp:5-32 picks "local" (Phred-weighted) when --fixed-accuracy == 0. */
enum { SPEQ_MODE_GLOBAL = 0, SPEQ_MODE_LOCAL = 1 };

typedef struct speq_index speq_index;            /* host-side FM-index (immutable) */
typedef struct speq_device_index speq_device_index; /* replica of an index in one GPU's HBM */

typedef struct {
    uint32_t prefix_q;   /* length of the q-mer interval lookup table (0 = none, max 13) */
    uint32_t threads;    /* host threads for the build (0 = all) */
    uint32_t pair_steps; /* 1: add the 16 two-symbol occ planes (LF over two bases per gather pair) */
    uint32_t label_table;/* 1: add the per-SA-position {group, run distance} table (one-load classification);
                            2: auto (only when the collection has >= 4 M symbols) */
    uint32_t gpu_build;  /* 1: build the suffix array and planes on GPU `device` (prefix doubling on radix sorts);
                            0: host SA-IS. Both produce identical indexes. */
    int32_t device;      /* GPU ordinal for gpu_build */
    uint32_t triple_steps; /* 1: also add the 64 three-symbol occ planes (LF over three bases per gather pair;
                              10.7 bytes per text symbol); requires pair_steps; 2: auto (on while the planes fit
                              32-bit buffer offsets, ~400 M symbols) */
} speq_build_opts;

/* Per-scan parameters (reference: cmd_arguments in include/arg_parse.h:10-28). */
typedef struct {
    uint32_t k;              /* --kmer (reference default 70)                               */
    uint32_t phred_cutoff;   /* --phred-cutoff; a window passes iff min(Q) > cutoff (:162) */
    uint32_t paired;         /* 1: records 2i and 2i+1 are mates; ambiguity per pair (:709-729) */
    uint32_t mode;           /* SPEQ_MODE_GLOBAL (integer U[g]) or SPEQ_MODE_LOCAL (also fp64 W[g]) */
} speq_scan_params;

/* Counter vector layout (u64): [0] = T (passing windows, fm_scanner.cpp:164),
 *                              [1] = ambiguous reads/pairs (:183-190, :213),
 *                              [2 .. 2+G) = U[g] (windows unique to group g, :180).
 * Local mode additionally fills a fp64 vector W[G] (:454-455). */
#define SPEQ_COUNTS_LEN(G) ((size_t)(G) + 2u)

/* ---- library ---- */
const char* speq_last_error(void);
int speq_abi_version(void);
/* Number of visible GPUs (0 when none); never fails. */
int speq_device_count(void);

/* ---- index build / persistence (replaces seqan3::fm_index{…}, fm_indexer.cpp:8-52) ----
 * seq          : concatenated ASCII sequences of the R reference records (FASTA order)
 * rec_offsets  : R+1 offsets into seq
 * group_of_rec : group id of each record (file_to_map's group_scaffolds, file_to_map.cpp:20-119);
 *                n_group_entries may exceed R (extra entries are ignored like the zip at
 *                fm_scanner.cpp:1494) but every record r < R must have 0 <= group < n_groups.
 * The indexed collection is [fwd_0, rc_0, fwd_1, rc_1, …] as built at fm_indexer.cpp:25-33. */
int speq_index_build(const char* seq, const uint64_t* rec_offsets, uint32_t n_records,
                     const int32_t* group_of_rec, uint32_t n_group_entries, uint32_t n_groups,
                     const speq_build_opts* opts, speq_index** out);
/* user_header: opaque bytes stored in front of the index (the CLI stores the reference's
 * {ref path, ref mtime, groups mtime, names, group_scaffolds, counts}, fm_indexer.cpp:39-50). */
int speq_index_save(const speq_index* idx, const char* path, const void* user_header, uint64_t header_len);
/* Loads an index; *user_header (may be NULL) receives a malloc'ed copy of the stored header that the
 * caller frees with speq_free(). */
int speq_index_load(const char* path, speq_index** out, void** user_header, uint64_t* header_len);
/* Reads only the user header of an index file (for the staleness check at fm_indexer.cpp:68-97). */
int speq_index_read_header(const char* path, void** user_header, uint64_t* header_len);
void speq_index_free(speq_index* idx);
void speq_free(void* p);

typedef struct {
    uint64_t n;            /* FM text length (all texts + separators + terminator) */
    uint32_t n_texts;      /* 2R */
    uint32_t n_records;    /* R */
    uint32_t n_groups;     /* G */
    uint32_t prefix_q;
    uint32_t pair_steps;   /* 1 when the two-symbol occ planes are present */
    uint32_t label_table;  /* 1 when the per-position label table is present */
    uint64_t n_runs;       /* runs of equal group label along the suffix array */
    uint64_t device_bytes; /* bytes a device replica occupies in HBM */
    uint32_t triple_steps; /* 1 when the three-symbol occ planes are present */
} speq_index_info;
int speq_index_get_info(const speq_index* idx, speq_index_info* info);

/* Read-only views of the host arrays (for tests and tools; layout documented in DESIGN.md §3).
 * name: "text", "sa", "occ", "occ2", "occ3", "runs", "run_label", "lab", "prefix", "prefix_q1", "prefix_q2", "C",
 *       "text_start", "text_group". */
int speq_index_array(const speq_index* idx, const char* name, const void** ptr, uint64_t* bytes);

/* ---- device replica ---- */
/* Optional, before the index is even loaded (any thread): prepares GPU `device` for this process's first scan — its
 * context, the scan's GPU code (otherwise loaded at the first use of each kernel file, inside the first scan; the
 * GPU index builder's code is left to its first use) and `streams` (0-16) ready streams that speq_device_open and the FASTQ pipelines then take instead of creating
 * them (3-10 ms each). New in the MI355X build: the reference loads a host index (fm_scanner.cpp:45-58). */
int speq_device_warmup(int device, uint32_t streams);
int speq_device_open(const speq_index* idx, int device, speq_device_index** out);
int speq_device_close(speq_device_index* d);

/* ---- the hot path: scan reads already resident in HBM ----
 * Replaces search() + do_a_count() for every window of every read (fm_scanner.cpp:149-214 and the
 * paired/local variants).  Counters are ADDED to d_counts (u64[G+2]) and, in local mode, to d_weights
 * (f64[G]); the caller zeroes them.  d_seq/d_qual: ASCII bases and Phred+33 qualities, d_offsets:
 * n_reads+1 u64 offsets into both.  With params->paired the records are mate pairs (2i, 2i+1) and
 * n_reads must be even.  Asynchronous on `stream`. */
int speq_scan_reads_device(speq_device_index* d, const uint8_t* d_seq, const uint8_t* d_qual,
                           const uint64_t* d_offsets, uint64_t n_reads, const speq_scan_params* params,
                           uint64_t* d_counts, double* d_weights, void* stream);

/* Diagnostic twin of speq_scan_reads_device (not the hot path; bench.py's roofline model): the same scan and
 * results, run by an instrumented instantiation of the anchor-and-extend kernel that also counts the work it did.
 * stats (host, u64[SPEQ_AX_STATS_N], overwritten; synchronous): [0] loop iterations per wave, [1] anchor-bucket loads
 * (64 B each), [2] run iterations (lanes), [3]/[4] iterations in which a wave issued bucket/granule loads, [5] windows
 * classified by runs, [6] deferred windows, [7] deferred windows past the Bloom filter, [8] phase-2 bucket loads,
 * [9] phase-2 candidate verifications (ceil(k / 32) + 1 16-B granules each), [10] staged 16-base chunks (16 B of
 * bases + 16 B of qualities), [11] staged read segments, [12] single quality bytes loaded, [13] windows tallied by
 * runs, [14] 16-B granules loaded by runs, [15] lane refills (per wave), [16..19] phase-1 wave iterations
 * with 1-4, 5-16, 17-32, 33-64 busy lanes, [20..24] shader-clock cycles (s_memtime) summed over waves: in refills
 * (staging), phase-1 lookup iterations, phase-1 run iterations, phase 2 (deferred windows), and the whole loop,
 * [25] deferred-window passes (per wave), [26] cycles of the Bloom-filter part of phase 2, [27] phase-2 probe rounds
 * of the filter's survivors (per wave), [28] / [29] cycles of refills before their staging loads / in their staging
 * batches, [30] the longest wave's loop cycles (a maximum), [31] waves, [32..36] loop cycles summed over the waves of
 * blocks 0-255, 256-511, 512-767, 768-1023 and 1024 on. Fails with SPEQ_E_ARG when the scan does not use that kernel. */
#define SPEQ_AX_STATS_N 37
int speq_scan_reads_device_stats(speq_device_index* d, const uint8_t* d_seq, const uint8_t* d_qual,
                                 const uint64_t* d_offsets, uint64_t n_reads, const speq_scan_params* params,
                                 uint64_t* d_counts, double* d_weights, uint64_t* stats);

/* Host-buffer convenience used by the CLI: stages the reads to HBM in batches, runs the kernel and
 * returns the totals (counts: u64[G+2]; weights: f64[G] or NULL). Synchronous. */
int speq_scan_reads(speq_device_index* d, const uint8_t* seq, const uint8_t* qual, const uint64_t* offsets,
                    uint64_t n_reads, const speq_scan_params* params, uint64_t* counts, double* weights);

/* ---- reference-uniqueness pass (replaces _async_count_unique_kmers_per_group, fm_scanner.cpp:1476-1576)
 * For every window of every text (fwd and rc of each record): Tot_ref[g] += 1, and U_ref[g] += 1 iff
 * every occurrence lies in a text of group g.  Outputs are host arrays of G u64 (overwritten). */
int speq_ref_unique(speq_device_index* d, uint32_t k, uint64_t* u_ref, uint64_t* tot_ref);
/* Same on device buffers (added to d_u_ref/d_tot_ref), asynchronous. */
int speq_ref_unique_device(speq_device_index* d, uint32_t k, uint64_t* d_u_ref, uint64_t* d_tot_ref,
                           void* stream);

/* ---- multi-GPU: one all-reduce of the counter vector (replaces the future.get() sums, fm_scanner.cpp:224-233).
 * A communicator (void* comm) runs over one of two transports: RCCL (ncclAllReduce over xGMI; one rank per GPU) or
 * host sockets (loopback TCP: a reduce at rank 0 in rank order and a broadcast; ranks may share a GPU). Every
 * speq_allreduce_* / speq_em_allreduce call below takes either. ---- */
enum { SPEQ_COMM_AUTO = 0, SPEQ_COMM_RCCL = 1, SPEQ_COMM_HOST = 2 };
/* RCCL communicator from an id that rank 0 made with speq_comm_unique_id and handed to the others out of band
 * (bench.py: torch.distributed); binds to the calling thread's current GPU. */
int speq_comm_unique_id(void* id_out /* 128 bytes */);
int speq_comm_init(int nranks, int rank, const void* id /* 128 bytes */, void** comm_out);
/* Rendezvous + communicator in one call (the CLI's one-process-per-GPU mode). Rank 0 listens on 127.0.0.1 and
 * publishes {nonce, port} in the file rendezvous_path (replacing a stale one); the other ranks poll that file, connect
 * and present the nonce (a stale file of a dead run is skipped: its port refuses or its nonce does not match), all
 * within timeout_s. transport: SPEQ_COMM_RCCL, SPEQ_COMM_HOST, or SPEQ_COMM_AUTO = RCCL when every rank's `device`
 * is a different GPU (PCI bus id), else host sockets (RCCL refuses two ranks on one GPU). The RCCL communicator is
 * created on GPU `device` (set and restored around ncclCommInitRank); device may be -1 with SPEQ_COMM_HOST. */
int speq_comm_connect(int nranks, int rank, int device, const char* rendezvous_path, int transport, int timeout_s,
                      void** comm_out);
/* SPEQ_COMM_RCCL or SPEQ_COMM_HOST (the transport a communicator runs on); SPEQ_E_ARG for NULL. */
int speq_comm_transport(void* comm);
int speq_comm_destroy(void* comm);
int speq_allreduce_u64(void* comm, uint64_t* d_buf, uint64_t count, void* stream);
int speq_allreduce_f64(void* comm, double* d_buf, uint64_t count, void* stream);

/* ---- EM refinement (reference: fm_scanner.cpp:1069-1453 and the loops at :248-279) ----
 * The reference re-reads and re-searches all reads in every EM iteration. Here ONE scan records, for every passing
 * window whose occurrences span >= 2 groups, its SA interval (a window's EM weight depends only on the per-group
 * occurrence counts of its k-mer; the per-window factor temp_acc/qavg cancels), and every iteration is a sweep
 * over that histogram:
 *   speq_em_create -> speq_em_scan_reads[_device] (any number of batches; also returns the normal counters)
 *   -> speq_em_finalize -> speq_em_step per iteration.
 * The speq_index and the device replica must outlive the histogram. */
typedef struct speq_em speq_em;
int speq_em_create(const speq_index* idx, speq_device_index* d, speq_em** out);
int speq_em_scan_reads(speq_em* em, const uint8_t* seq, const uint8_t* qual, const uint64_t* offsets,
                       uint64_t n_reads, const speq_scan_params* params, uint64_t* counts, double* weights);
int speq_em_scan_reads_device(speq_em* em, const uint8_t* d_seq, const uint8_t* d_qual, const uint64_t* d_offsets,
                              uint64_t n_reads, const speq_scan_params* params, uint64_t* d_counts,
                              double* d_weights, void* stream);
/* Downloads the histogram and builds one row per distinct interval {multiplicity, (group, count)...}; rows of equal
 * content are then merged (multiplicities summed). `threads` is kept for the ABI: the rows are built on the
 * library's worker pool (at most 16 threads), as the EM steps are. */
int speq_em_finalize(speq_em* em, uint32_t threads);
/* Distinct intervals recorded, their (group, count) entries, and the windows (sum of multiplicities); before merging. */
int speq_em_info(const speq_em* em, uint64_t* n_intervals, uint64_t* n_entries, uint64_t* n_windows);
/* next[g] = sum over passing windows with hits of (c_g p_g / n_g) / sum_j (c_j p_j / n_j) (windows with a
 * non-positive sum skipped), given percent[G], group_counts[G] (the "(count)" of each groupings line) and
 * unique[G] (the U[g] counters of the same scan, i.e. its single-group windows). */
int speq_em_step(const speq_em* em, const double* percent, const int32_t* group_counts, const uint64_t* unique,
                 double* next);
void speq_em_free(speq_em* em);

/* ---- streaming scan: pinned host slots, H2D on a copy stream overlapped with the kernel ----
 * Replaces the reference's single-producer async_input_buffer feeding T-1 search workers
 * (fm_scanner.cpp:138-141, :219-222; paired :651-655). A pipeline owns n_slots pinned host buffers, each with a
 * device twin; a producer thread acquires a free slot, writes whole records into it (ASCII bases, Phred+33
 * qualities, offsets[0] = 0 .. offsets[n]), and submits it: the slot is copied to HBM on a copy stream while the
 * kernel of the previous slot runs on a compute stream. Any number of producer threads may acquire/submit
 * concurrently. Counters accumulate on the device; finish returns them (and resets them to zero).
 * em may be NULL; when given, the scan also records its EM histogram (the pipeline must use em's device). */
typedef struct speq_pipeline speq_pipeline;
typedef struct {
    uint8_t* seq;          /* capacity cap_bytes */
    uint8_t* qual;         /* capacity cap_bytes */
    uint64_t* offsets;     /* capacity cap_records + 1 */
    uint64_t cap_bytes;
    uint64_t cap_records;
    int32_t slot;          /* pass back to speq_pipeline_submit */
} speq_slot;
int speq_pipeline_create(speq_device_index* d, const speq_scan_params* params, speq_em* em, uint64_t slot_bytes,
                         uint64_t slot_records, uint32_t n_slots, speq_pipeline** out);
/* Blocks until a slot is free (its previous copy and kernel have completed). */
int speq_pipeline_acquire(speq_pipeline* pl, speq_slot* out);
/* Grows a slot's capacity (host and device) before it is filled; contents are not preserved. */
int speq_pipeline_reserve(speq_pipeline* pl, speq_slot* slot, uint64_t bytes, uint64_t records);
/* Enqueues the copy + scan of n_records records of an acquired slot (n_records may be 0: releases the slot). */
int speq_pipeline_submit(speq_pipeline* pl, int32_t slot, uint64_t n_records);
/* Waits for every submitted slot; counts u64[G+2] (and weights f64[G] in local mode) receive the totals since
 * the last finish. */
int speq_pipeline_finish(speq_pipeline* pl, uint64_t* counts, double* weights);
void speq_pipeline_free(speq_pipeline* pl);

/* Scan of FASTQ files (plain or gzip; paired when path2 != NULL: records i of both files are mates) through a
 * pipeline: one reader thread per file decompresses and cuts record-aligned blocks, `threads` parser threads fill
 * pinned slots. FASTQ grammar of the reference's reader (multi-line sequence/quality accepted; a FASTA file is
 * rejected: qualities are required). counts/weights as speq_scan_reads; stats may be NULL. */
typedef struct {
    uint64_t records;      /* records scanned (both mates) */
    uint64_t bases;
    uint64_t batches;      /* slots submitted */
    double seconds;        /* wall time of the call */
} speq_stream_stats;
int speq_scan_fastq(speq_device_index* d, const char* path1, const char* path2, const speq_scan_params* params,
                    speq_em* em, uint32_t threads, uint64_t* counts, double* weights, speq_stream_stats* stats);
/* Optional, ahead of speq_scan_fastq on GPU `device` with `threads` parsers (e.g. while the index loads): allocates
 * the stream's pinned and device slot buffers now (otherwise the parser threads' first slots allocate them: up to
 * 66 ms of page-locking at the start of a `speq scan` run); the next stream's slots of that device take them. */
int speq_stream_reserve(int device, uint32_t threads, uint32_t paired);
/* The same reader and parsers without a device (host only; for tests and tools): record and base counts, and an
 * order-independent digest = sum over records of mix64(FNV-1a-64 over (len, (base << 8 | qual) per position)). */
int speq_fastq_checksum(const char* path1, const char* path2, uint32_t threads, uint64_t* records, uint64_t* bases,
                        uint64_t* digest);

/* ---- several GPUs in one process ----
 * Reads shard across the GPUs of a node, the index is replicated (one speq_device_index per GPU, opened from the
 * same speq_index), and the only exchange is a sum of the counters. The reference sums its per-thread vectors after
 * future.get() (fm_scanner.cpp:224-233, :1544-1557); here one host thread owns every replica, so the G + 2 counter
 * words of each replica are added on the host, and the EM histograms (n words per replica) are added on the first
 * replica's GPU (peer copy over xGMI + an add kernel). For one process per GPU use speq_allreduce_* (RCCL).
 * Replicas may share a GPU (logical shards; results are the same). */
/* speq_scan_fastq over n_devices replicas: record-aligned blocks are dealt to the replicas in turn. ems is NULL or
 * holds one histogram per replica (ems[i] created on ds[i]); fold them with speq_em_merge before speq_em_finalize. */
int speq_scan_fastq_multi(speq_device_index* const* ds, speq_em* const* ems, uint32_t n_devices, const char* path1,
                          const char* path2, const speq_scan_params* params, uint32_t threads, uint64_t* counts,
                          double* weights, speq_stream_stats* stats);
/* speq_ref_unique with replica i scanning the i-th equal slice of the reference windows (the .dat pass sharded the
 * same way as the reads; fm_scanner.cpp:1476-1560). */
int speq_ref_unique_multi(speq_device_index* const* ds, uint32_t n_devices, uint32_t k, uint64_t* u_ref,
                          uint64_t* tot_ref);
/* dst += src for two unfinalized EM histograms of replicas of one index (any GPUs of this process). src's device
 * arrays are released: afterwards src accepts only speq_em_free. */
int speq_em_merge(speq_em* dst, speq_em* src);

/* ---- one process per GPU (RANK / WORLD_SIZE of a launcher such as torchrun; `speq scan` runs this way when
 * WORLD_SIZE > 1). Every rank opens its own replica, scans ITS share of the input, and the exchange is RCCL:
 * speq_allreduce_u64/_f64 of the counters, speq_em_allreduce of the EM histogram. This replaces the reference's
 * future.get() sums (fm_scanner.cpp:224-233) across processes instead of threads. ---- */
/* speq_scan_fastq over shard `shard` of `n_shards`: the input is cut into record-aligned blocks exactly as on every
 * other rank and this rank scans the blocks b with b % n_shards == shard (counts, weights, em and stats cover those
 * only). cut: -1 = parallel cut, falling back to the sequential cutter on this rank alone (n_shards = 1 only);
 * 1 = parallel cut only, failing with SPEQ_E_RETRY (counters, weights, em cleared) when the file does not fit it —
 * the ranks then agree (an all-reduce of the flag) and all scan again with cut = 0 (sequential cutter). */
int speq_scan_fastq_shard(speq_device_index* d, speq_em* em, const char* path1, const char* path2,
                          const speq_scan_params* params, uint32_t threads, uint32_t shard, uint32_t n_shards, int cut,
                          uint64_t* counts, double* weights, speq_stream_stats* stats);
/* speq_fastq_checksum over one shard (same blocks as speq_scan_fastq_shard; cut 0 or 1, SPEQ_E_RETRY as there). */
int speq_fastq_checksum_shard(const char* path1, const char* path2, uint32_t threads, uint32_t shard,
                              uint32_t n_shards, int cut, uint64_t* records, uint64_t* bases, uint64_t* digest);
/* The .dat pass over shard `shard` of `n_shards` equal slices of the reference windows (host outputs, this
 * shard's partial sums; fm_scanner.cpp:1476-1560). */
int speq_ref_unique_shard(speq_device_index* d, uint32_t k, uint32_t shard, uint32_t n_shards, uint64_t* u_ref,
                          uint64_t* tot_ref);
/* Sums an unfinalized EM histogram over the ranks of comm (multiplicities added, interval ends by max: a position
 * that starts a multi-group interval on any rank starts the same interval everywhere), enqueued on stream and
 * synchronized. Every rank then holds the whole job's histogram (speq_em_finalize / speq_em_step as usual). */
int speq_em_allreduce(speq_em* em, void* comm, void* stream);
/* In-place sum over the ranks of comm of `count` u64 (is_f64 = 0) or f64 (is_f64 = 1) words in HOST memory (blocking;
 * RCCL communicators stage it through GPU `device`): the CLI's counters, weights, .dat sums, statistics and flags. */
int speq_allreduce_host(void* comm, int device, void* buf, uint64_t count, int is_f64);

/* ---- groupings file (speq::file_to_map, /root/reference/src/file_to_map.cpp:20-119) ----
 * Same grammar "Name(count): i, j-k, …"; parse errors of single tokens are collected (the reference prints
 * them to std::cerr) and returned by speq_groupings_errors(). A missing "(count)" fails with SPEQ_E_ARG
 * (std::invalid_argument from std::stoi at file_to_map.cpp:43). */
typedef struct speq_groupings speq_groupings;
int speq_groupings_parse(const char* path, speq_groupings** out);
uint32_t speq_groupings_n_groups(const speq_groupings* g);
const char* speq_groupings_name(const speq_groupings* g, uint32_t i);
int32_t speq_groupings_count(const speq_groupings* g, uint32_t i);
uint32_t speq_groupings_n_entries(const speq_groupings* g);
const int32_t* speq_groupings_scaffolds(const speq_groupings* g);
const char* speq_groupings_errors(const speq_groupings* g);
void speq_groupings_free(speq_groupings* g);

/* ---- launch tuning (performance only; results never depend on it) ----
 * "blocks_per_cu": cap resident 256-thread workgroups per CU (0 = no cap; the kernel's LDS is padded);
 *                  default by plane footprint: <= 16 MB none, <= 256 MB (Infinity Cache) 4, larger 3;
 * "grid_blocks"  : upper bound of the grid (default 16384 below 4 M symbols, else 8192);
 * "ilp"          : k-mer windows each lane searches concurrently, 1 or 2 (default 2 for indexes of < 4 M
 *                  symbols, else 1); "ilp_local" the same for Phred-weighted scans (default 1);
 * "prefix_level" : q-mer table used by scans: -1 (default) picks, per k, the longest of q, q-1, q-2 that leaves a
 *                  multiple of the widest LF step; 0..2 forces table q - level (results never change);
 * "sparse_prefix": 0 (default) dense q-mer tables; 1 a presence bitvector with ranks + the present intervals
 *                  (less memory, one more dependent load per window); -1 sparse when < 1/8 of the codes occur;
 * "fastq_gpu_parse": 1 (default) speq_scan_fastq parses blocks of simple four-line records on the GPU (raw text
 *                  to HBM); 0 parses every block on host threads. Results are identical;
 * "kmer_table"   : 1 (default) scans of k <= 31 look each N-free window up in the replica's k-mer interval table
 *                  for k (built by the first scan with that k, or by speq_device_prepare); 0 searches every window
 *                  with LF steps. Results are identical;
 * "kt_compact"   : 1 (default) 8-B-slot tables for k <= 23 (0: 16-B slots); "kt_load8": their load factor in percent
 *                  (default 35); "kt_slots": 16-B slots per distinct k-mer of the wide form (default 2). These apply to
 *                  tables built afterwards;
 * "ilp_kt"       : windows per lane of table scans, 1 or 2 (pipelined kernel), 4 (k_scan); 0 (default) = 1 for
 *                  compact tables (k <= 23), 2 for 16-B-slot tables;
 *                  "kt_pipeline": 1 (default) the software-pipelined table kernel k_scan_kt, 0 k_scan;
 *                  "blocks_per_cu_kt": blocks_per_cu of table scans (default 0: no cap);
 * "stream_lanes" : compute streams of a pipeline created afterwards (speq_pipeline_create, speq_scan_fastq, host
 *                  scans), 1..8 (default 3): consecutive batches are parsed and scanned on them in turn, so the
 *                  short launches of different batches overlap on the CUs;
 * anchor-and-extend scans (k <= 128): "ax_scan" 1 (default) / 0 (other kernels), "ax_load" anchor-table load factor in
 *                  percent for tables built afterwards, "grid_blocks_ax" grid cap, "blocks_per_cu_ax" resident blocks
 *                  per CU (0: as registers/LDS allow), "ax_generations" grid = 1..16 times the resident blocks
 *                  (default 1: one persistent generation), "ax_mproof" m-mer absence proofs of the windows around a
 *                  mismatch (1 default: known and unknown mismatches, 2: known ones only, 0: off; results are the
 *                  same); "last_kernel" (read only) the kernel of the last scan. */
int speq_device_set_tuning(speq_device_index* d, const char* key, int64_t value);
int speq_device_get_tuning(const speq_device_index* d, const char* key, int64_t* value);

/* ---- k-mer interval table (the q-mer table of the FM-index taken to q = k) ----
 * For a scan length k <= 31 the replica keeps a hash table of every distinct N-free k-mer of the reference texts
 * with its SA interval start and its classification (one group, or the interval width when its occurrences span
 * >= 2 groups), computed once per distinct k-mer by FM backward search; a scan then resolves each window with one
 * 64-B bucket load instead of a chain of LF steps (an absent k-mer does not occur). Built on the replica's GPU by
 * the first scan with k, or here ahead of time; blocking. Outputs may be NULL; all zero when tables are off
 * (tuning "kmer_table" = 0), k > 31, or the table would not fit the free HBM (those scans use LF steps). Replaces no reference call; the reference
 * searches each window from scratch (fm_scanner.cpp:208). */
int speq_device_prepare(speq_device_index* d, uint32_t k, uint64_t* distinct_kmers, uint64_t* table_bytes,
                        double* build_ms);

/* ---- kernel timing (HIP events on the launch stream; bench/roofline support) ----
 * Returns the summed elapsed milliseconds of the scan kernels launched by speq_scan_reads_device on
 * this handle since the last reset, and the number of launches.  Enabled by speq_timing_enable(d, 1). */
int speq_timing_enable(speq_device_index* d, int on);
int speq_timing_read(speq_device_index* d, double* total_ms, uint64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* SPEQ_SCAN_H */
