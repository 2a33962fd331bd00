/*
 * ghostm_hip.h — C ABI of the MI355X (gfx950) search/align plugin.
 *
 * Part 1 is the reference GPU plugin surface, symbol for symbol: GHOSTM 2.0's
 * aligner.cpp binds exactly these ten functions (reference aligner_gpu.h:33-114,
 * called from aligner.cpp:77-93, 110, 123-124, 356-361, 529-531, 211). A build of
 * the reference host that links libghostm_hip.so instead of aligner_gpu.o runs
 * its `-D <device>` path on this implementation unchanged.
 *
 * Part 2 extends the surface where the reference ABI cannot express the whole
 * hot path: a whole-query-set candidate count (needed to
 * reproduce the CPU path's batching exactly), a device traceback, error strings
 * instead of exit(), and a session API that runs the complete `aln` pipeline
 * (seed -> score -> merge -> traceback -> E-value) with inputs resident in HBM.
 *
 * Conventions: plain pointers and sizes, no C++ or torch types. Host arrays are
 * owned by the caller; copies are synchronous unless stated. Int returns: 0 = OK,
 * non-zero = error (message via GhostmGetLastError). One device per process.
 */
#ifndef GHOSTM_HIP_H_
#define GHOSTM_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- Part 1: reference plugin surface ------------------------ */

/* replaces aligner_gpu.h:37 InitGpu (aligner_gpu.cu:588) — reset module state */
int InitGpu(void);

/* replaces aligner_gpu.h:39-47 (aligner_gpu.cu:506) — device bytes the search
 * needs for the given maxima (counts this build's buffers, not the reference's) */
size_t GetNeededGPUMemorySize(uint32_t seed, uint32_t shift_size,
                              uint32_t max_list_length, uint32_t max_query_length,
                              uint32_t max_number_queries, uint32_t max_db_length);

/* replaces aligner_gpu.h:49-57 (aligner_gpu.cu:560) — 1 if it does not fit */
int CheckGpuMemory(uint32_t seed, uint32_t shift_size, uint32_t max_list_length,
                   uint32_t max_query_length, uint32_t max_number_queries,
                   uint32_t max_db_length);

/* replaces aligner_gpu.h:59-64 (aligner_gpu.cu:620) — bind device, upload the
 * 32x32 score matrix M[db_code*32 + query_code], size candidate buffers */
int SetOptionGpu(uint32_t max_list_length, int score_matrix[], int device);

/* replaces aligner_gpu.h:66 (aligner_gpu.cu:646) */
void printGpuInfo(int device);

/* replaces aligner_gpu.h:68-73 (aligner_gpu.cu:654) — upload a query chunk of
 * number_sequences fixed-width records of sequence_length codes */
int SetQueryGpu(uint8_t sequences[], uint32_t number_sequences, uint32_t sequence_length);

/* replaces aligner_gpu.h:75-83 (aligner_gpu.cu:691) — upload a DB chunk and its
 * k-mer index (keys_count = CSR offsets, positions = ascending per key) */
int SetDbGpu(uint8_t sequences[], uint32_t sequences_legnth, uint32_t keys_count[],
             uint32_t keys_count_length, uint32_t positions[], uint32_t positions_length);

/* replaces aligner_gpu.h:85-97 (aligner_gpu.cu:759) — seed search for the queries
 * from start_query_id on. Batches queries with the reference GPU rule (stop before
 * the running candidate total reaches max_number_alignments). Fills
 * alignment_count_list[0..q] (prefix counts) and starts[] (candidate DB starts,
 * ascending per query); returns q = number of queries in the batch. The starts
 * stay resident on the device for the next CalculateScoreGpu. */
uint32_t SearchNextGpu(uint32_t query_sequence_length, uint32_t number_query_sequences,
                       uint32_t seed, uint32_t threshold, uint32_t shift_size,
                       uint32_t log_region_size, uint32_t max_number_alignments,
                       uint32_t start_query_id, uint32_t *alignment_count_list,
                       uint32_t *starts);

/* replaces aligner_gpu.h:99-110 (aligner_gpu.cu:971) — Gotoh local score + end of
 * every candidate of the last SearchNextGpu batch */
void CalculateScoreGpu(uint32_t db_length, uint32_t query_sequence_length,
                       uint32_t number_alignment_list, uint32_t scores[], uint32_t ends[],
                       uint32_t base_search_length, uint32_t offset, int open_gap,
                       int extend_gap);

/* replaces aligner_gpu.h:112 (aligner_gpu.cu:1029) */
int FreeGpu(void);

/* ---------------- Part 2: extensions -------------------------------------- */

/* Last error message of this thread's most recent failing call ("" if none). */
const char *GhostmGetLastError(void);

/* Build identity (kernel variant names, arch), for logs. */
const char *GhostmBuildInfo(void);

/* Device blocks a destroyed session released stay cached for the next session
 * (at most GHOSTM_DEV_POOL_MB, default 8192 MB). An allocation that runs out of
 * memory empties the cache and retries once. GhostmDevicePoolTrim frees every
 * cached block now (for a caller that shares the device with other allocators)
 * and returns the bytes freed; GhostmDevicePoolInfo reports the cached bytes and
 * how many allocations were retried after emptying the cache. No reference
 * counterpart (the reference allocates per Aligner, aligner_gpu.cu). */
uint64_t GhostmDevicePoolTrim(void);
int GhostmDevicePoolInfo(uint64_t *cached_bytes, uint64_t *oom_retries);

/* Candidate count of EVERY query of the resident chunk (no batching), K1 count
 * pass; counts[number_query_sequences]. Lets a host reproduce the CPU path's
 * batch cuts exactly (reference aligner.cpp:511-514). */
int CountCandidatesGpu(uint32_t query_sequence_length, uint32_t number_query_sequences,
                       uint32_t seed, uint32_t threshold, uint32_t shift_size,
                       uint32_t log_region_size, uint32_t counts[]);

/* Reverse-DP traceback (reference aligner.cpp:771-949) of nhits hits on the
 * resident query/DB chunk: per hit (query_id, db_end) -> db_start (absolute),
 * aln_len, aln_match, seq_id = match/len (float). base_search_length is the
 * reference's L + 2*e*2*R window. */
int TraceBackGpu(uint32_t nhits, const uint32_t query_ids[], const uint32_t db_ends[],
                 uint32_t query_sequence_length, uint32_t base_search_length,
                 int open_gap, int extend_gap, uint32_t db_starts[], uint32_t aln_lens[],
                 uint32_t aln_matches[], float seq_ids[]);

/* The `db` formatter's k-mer index of one DB chunk, built on the GPU
 * (replaces DBCreator::ConstructIndex, db_creator.cpp:167-241).
 * seq[len] = the chunk's END-separated residues (.seq); seed = the index seed mask
 * (db -k k -> 2^k - 1); kcl = 32^weight(seed) + 1. Fills keys_count[kcl] (CSR
 * offsets) and positions[*npos] (ascending per key; the array must hold len
 * entries) byte-identical to the CPU formatter's .ind. device_ms (optional)
 * receives the device time of the build (HIP events, after the upload). */
int GhostmBuildIndexGpu(const uint8_t *seq, uint32_t len, uint32_t seed, uint32_t kcl,
                        uint32_t *keys_count, uint32_t *positions, uint32_t *npos, int device,
                        float *device_ms);

/* The `qry` formatter's per-residue work on the GPU (replaces QueryCreator's
 * coding, query_creator.cpp:388-423, and six-frame translation, :242-324;
 * SURVEY.md §8 f2). raw[raw_len] = the chunk's records' letters concatenated
 * (no newlines); record r is raw[offsets[r] .. + lengths[r]). dna_len = 0:
 * protein, records[n * width] = each record's residue codes, cut at or X-padded
 * to width. dna_len > 0: DNA reads cut/padded to dna_len letters (the reference
 * uses the chunk's first read length), records[6n * width] = per read the
 * frames +0 +1 +2 and the reverse complement's +0 +1 +2 with stop codons
 * masked to '*' until the next ATG, each cut/X-padded to width. Byte-identical
 * to the CPU formatter's .seq. device_ms (optional) = the kernel time. */
int GhostmFormatQueriesGpu(const uint8_t *raw, uint64_t raw_len, const uint64_t *offsets,
                           const uint32_t *lengths, uint32_t n, uint32_t width, uint32_t dna_len,
                           uint8_t *records, int device, float *device_ms);

/* General Karlin-Altschul parameters. The reference `aln` knows
 * only two gapped parameter sets (statistics.cpp:134-146); its vendored routines
 * compute ungapped ones for any matrix. GhostmKarlinUngapped restates
 * Statistics::CalculateUngappedIdealKarlinParameters (statistics.cpp:100-112,
 * Robinson & Robinson background) with BlastKarlinBlkCalc (karlin.cpp:16-32) on
 * a 32x32 matrix M[db_code*32 + query_code]; the floats are bit-identical to the
 * reference's. `aln` uses them for E-values of matrix/gap combinations outside
 * the table when GHOSTM_KARLIN=ungapped is set (otherwise the reference's error). */
int GhostmKarlinUngapped(const int score_matrix[], float *lambda, float *K, float *H);

/* The 32x32 matrix `aln -M path` scores with (ScoreMatrixReader::Read,
 * score_matrix_reader.cpp:44-113: built-in BLOSUM62 when the path cannot be
 * opened), row-major M[db_code*32 + query_code]; the input GhostmKarlinUngapped takes. */
int GhostmReadScoreMatrix(const char *path, int score_matrix[]);

/* BlastComputeLengthAdjustment (karlin.cpp:393-476): the edge-effect length
 * adjustment; returns 0 when the iteration converged, 1 otherwise, as the
 * reference. */
int GhostmLengthAdjustment(float K, float logK, float alpha_d_lambda, float beta, int query_length,
                           uint32_t db_length, int db_num_seqs, int *length_adjustment);

/* One resolved hit, the record gathered across ranks (32 bytes). Coordinates are
 * subject-relative, as printed minus one. */
typedef struct GhostmHit {
  uint32_t query_id;   /* global query index over all chunks */
  uint32_t db_id;      /* global subject index over all DB chunks */
  uint32_t score;
  uint32_t db_start;
  uint32_t db_end;
  uint32_t aln_len;
  uint32_t aln_match;
  float seq_id;
} GhostmHit;

/* Stage timings / work counters of the last GhostmSessionRun. */
typedef struct GhostmStats {
  double seconds_total;      /* whole run, host wall clock */
  double seconds_seed;       /* K1 count + write passes (device time) */
  double seconds_score;      /* K2 (device time) */
  double seconds_traceback;  /* K3 (device time) */
  double seconds_merge;      /* host Merge (sort/dedup/select) */
  double seconds_output;     /* host E-value + text formatting */
  uint64_t queries;
  uint64_t query_residues;   /* sum over queries of non-X prefix length */
  uint64_t candidates;
  uint64_t score_cells;      /* sum over candidates of L x window columns W (END columns included: the
                                reference's CalculateScore loop visits them, aligner.cpp:576-660) */
  uint64_t tracebacks;       /* hits traced back (K3), new selections only */
  uint64_t traceback_cells;
  uint64_t hits;
  uint64_t batches;
  uint64_t score_launches;
  uint64_t seed_bytes;       /* algorithmic bytes of the K1 passes */
  uint64_t score_launches_packed; /* K2 launches that ran a packed 16-bit kernel */
  uint64_t score_launches_half;   /* ... of which the f16 encoding */
  uint64_t traceback_launches;
  uint64_t traceback_launches_key; /* K3 launches that ran the key formulation */
  uint64_t seed_runs_hash;        /* K1 runs whose slot pass used the hash-count kernel */
  uint64_t score_rechecks;        /* guarded f16 K2 candidates re-scored exactly in int16 */
  uint64_t traceback_launches_scan; /* K3 launches preceded by the scores-only scan (K3a) */
  uint64_t traceback_scan_cells;    /* K3a: sum over hits of L x reverse-window columns */
  uint64_t merge_launches;          /* K4 launches */
  uint64_t merge_launches_wave;     /* ... that ran one wave per name group (k_merge_wave) */
  uint64_t score_launches_framed;   /* f16 K2 launches of the column-framed kernel (k_score16f) */
  uint64_t seed_queries_class[4];   /* K1 queries per size class by list entries (3 = global merge) */
  uint64_t seed_queries_wide;       /* K1 queries with more candidates than a slot (offset pass) */
  uint64_t segments;                /* device-merge segments (K2 -> K4 -> K3 rounds) */
  uint64_t seed_runs_filter;        /* K1 runs whose classes 0/1 used the presence-filtered table */
  uint64_t seed_filter_overflows;   /* ... queries whose filter queue overflowed (redone unfiltered) */
  uint64_t score_launches_swar;     /* framed K2 launches over 16-bit integer patterns (k_score16f<S, true>) */
  uint64_t traceback_launches_scan_swar; /* K3a scans over 16-bit integer patterns (k_tb_scan<..., true>) */
  uint64_t seed_list_entries;       /* K1: sum over queries of the k-mer position-list lengths */
  uint64_t score_launches_unit;     /* framed integer-pattern K2 launches with unit-pair profile words (k_score16f<S, true, true>) */
  uint64_t traceback_launches_strips; /* K3 key DPs run by strip class (each hit on the strips up to its first maximal cell) */
  double seconds_traceback_scan;    /* of seconds_traceback: the scan phase (k_tb_prep, k_tb_pairs, the sorts,
                                       k_tb_scan); the rest is the key DP (k_traceback_key) */
  uint64_t score_launches_pair;     /* K2 launches of sparse segments run by the pair-table kernel (k_score_pair) */
  uint64_t seed_table_full;         /* K1 queries whose LDS bin table reached its probe bound (redone by the
                                       table-free merge kernel) */
  uint64_t seed_compact_redo;       /* K1 compactions re-run by the host (queue overflow, candidate buffers grown) */
  uint64_t score_launches_sparse;   /* K2 launches of sparse segments run by the 16-row profile kernel (k_score16f<16, true>,
                                       seven query profiles per block) */
  uint64_t traceback_launches_keyframe; /* K3 key DPs run with the column-framed E chain (k_traceback_key FRAME) */
  uint64_t score_launches_levels;   /* K2 launches of the 16-bit-row integer-pattern kernel with restart levels
                                       (k_score16f<S, true, false, true>) */
} GhostmStats;

/* Session: parse `aln` options exactly like the reference (getopt string
 * "b:d:D:e:E:G:i:l:M:o:r:s:t:S:L:y:v", aligner.cpp:225-345; argv[0] is ignored),
 * load every query and DB chunk and make them resident on the device given by
 * -D (default 0). Returns NULL on error. */
void *GhostmSessionCreate(int argc, char **argv);

/* Multi-GPU (the reference has no multi-GPU path, common.h:37):
 * one process per GPU, each opening a shard session. The query set selected by
 * -i/-S/-L is cut into `world` contiguous ranges of about equal residues, only
 * at name-group starts (a DNA read's six frames stay together: the reference
 * merges a group into one result list, aligner.cpp:697-700), and this session
 * searches range `rank` on the device given by -D. Hit records keep global
 * query indices, and the shards' outputs concatenated in rank order are the
 * unsharded output byte for byte; the data-path collective is the caller's
 * gather of GhostmSessionDeviceHits records (RCCL over xGMI). Returns NULL on
 * error. world = 1 is GhostmSessionCreate.
 *
 * Batch cuts: the reference's output depends on where its batch loop cuts a
 * query chunk (aligner.cpp:131-171, 511-514: carried result lists are re-sorted
 * every batch, a batch may split a name group, a chunk whose first query alone
 * exceeds -l ends early). A shard therefore replays the UNSHARDED run's batches
 * on its own queries (a batch that misses them is a pass over its carried
 * lists only). This batch plan is made at creation from the whole chunk's
 * candidate counts: GhostmSessionCreateShard reads every query of the set and
 * counts them all itself (K1 once, no communication); see
 * GhostmSessionCreateShardEx for the rank-local form. Every run re-derives its
 * counts and fails if they differ from the plan's. */
void *GhostmSessionCreateShard(int argc, char **argv, int rank, int world);

/* The collective GhostmSessionCreateShardEx calls (on the creating thread, the
 * same calls in the same order on every rank): an all-gather. Each rank passes
 * send_bytes bytes; recv receives every rank's buffer concatenated in rank
 * order, recv_bytes[r] bytes from rank r (known to all ranks). 0 = success. */
typedef int (*GhostmAllGatherFn)(void *ctx, const void *send, uint64_t send_bytes, void *recv,
                                 const uint64_t *recv_bytes);

/* GhostmSessionCreateShard for one process per GPU with a communicator: the
 * rank reads only the .seq rows and .nam lines of its own range (every rank
 * still derives the cut from all queries' residue counts and name-group
 * starts), counts only its own queries, and the ranks agree on the batch plan
 * with one all-gather of their candidate totals per (query chunk, DB chunk),
 * plus one of the per-query counts when some chunk needs more than one batch.
 * allgather == NULL is GhostmSessionCreateShard. */
void *GhostmSessionCreateShardEx(int argc, char **argv, int rank, int world, GhostmAllGatherFn allgather,
                                 void *ctx);

/* The query range [begin, end) of a shard session, as indices over the
 * selected chunks' queries (0, UINT64_MAX for an unsharded session). */
int GhostmSessionShardRange(void *session, uint64_t *begin, uint64_t *end);

/* The most hit records one run of this session can return: its name groups x
 * max(-b, 1) (each group keeps at most -b hits, reference aligner.cpp:742-760;
 * -b is read with atoi as aligner.cpp:251 does). A caller sizes its
 * GhostmSessionDeviceHits destination, or a fixed-capacity gather buffer, from
 * it. Returns UINT64_MAX for a null session. */
uint64_t GhostmSessionHitCapacity(void *session);

/* The shard rule on its own (host only, no device): cuts[0..world] over n
 * queries of the given weights; a cut falls only where group_start[i] != 0 and
 * is the first such i at or after the previous cut with
 * sum(weights[0..i)) * world >= sum(weights) * r. */
int GhostmShardCuts(uint64_t n, const uint32_t weights[], const uint8_t group_start[], int world,
                    uint64_t cuts[]);

/* Run the whole search with the CPU path's semantics (batch cuts, merge order,
 * tie rules) on the device. Results replace those of any previous run. */
int GhostmSessionRun(void *session);

/* GhostmSessionRun that also writes the -o file while the search runs: each
 * segment's text is written, in output order, as soon as it is formatted (the
 * reference writes after each query chunk, aligner.cpp:211). The file equals
 * what GhostmSessionWrite writes; GhostmSessionWrite is then a no-op. */
int GhostmSessionRunToFile(void *session);

/* Formatted output of the last run (reference WriteOutput/V1/V2 text). With
 * buf == NULL returns the byte count; otherwise copies min(cap, size) bytes. */
size_t GhostmSessionOutput(void *session, char *buf, size_t cap);

/* Write the formatted output of the last run to the -o file. */
int GhostmSessionWrite(void *session);

/* Hit records of the last run in output order; same NULL/cap convention. */
size_t GhostmSessionHits(void *session, GhostmHit *hits, size_t cap);

/* The same records resident on the session's GPU, for a device-to-device
 * gather across ranks: copies min(n, cap) records to dst_device
 * (device memory on the session's GPU; NULL only counts) and returns n, or
 * (size_t)-1 on error. */
size_t GhostmSessionDeviceHits(void *session, void *dst_device, size_t cap);

int GhostmSessionStats(void *session, GhostmStats *stats);

/* The same with the caller's struct size: GhostmStats only ever grows by
 * fields appended at its end, so a caller built against an older header
 * passes its sizeof and gets exactly the fields it knows (min(size, the
 * library's sizeof) bytes are written). Returns the library's sizeof, or 0 on
 * a null argument. */
size_t GhostmSessionStatsSized(void *session, GhostmStats *stats, size_t size);

void GhostmSessionDestroy(void *session);

/* `ghostm aln ...` end to end (create + run + write + destroy). Exit status like
 * the reference CLI: errors are printed and 0 is still returned (main.cpp:116-121). */
int GhostmAlignMain(int argc, char **argv);

#ifdef __cplusplus
}
#endif

#endif /* GHOSTM_HIP_H_ */
