/*
 * nwk.h -- C-ABI of the MI355X all-pairs Needleman-Wunsch engine.
 *
 * Drop-in boundary for the reference's hot path (paths relative to the
 * reference repository yangxvlin/multiple-sequence-alignment-openMP-openMPI):
 *
 *   nwk_get_minimum_penalties  replaces  std::string getMinimumPenalties(
 *        std::string *genes, int k, int pxy, int pgap, int *penalties)
 *        seqalign-mpi-skeleton.cpp:13,117-175 / submit/xuliny-seqalkway.cpp:232-364
 *   nwk_align_pairs            replaces  the per-rank worker loop
 *        do_MPI_task(rank) + do_task(...)  submit/xuliny-seqalkway.cpp:369-417,183-227
 *        (one call aligns a shard of canonical pair ids and returns the
 *        per-pair result record {penalty, problemhash} of Packet, sub:126-130)
 *   nwk_get_minimum_penalty    replaces  int getMinimumPenalty(std::string x,
 *        std::string y, int pxy, int pgap, int *xans, int *yans)
 *        seqalign-mpi-skeleton.cpp:14,186-280 (+ the trim at skel:135-154)
 *   nwk_chain_hash             replaces  the hash chain at skel:159 / sub:334-337
 *   nwk_sha512_hex             replaces  sw::sha512::calculate, sha512.hh:159-164
 *
 * Conventions: plain pointers and sizes, caller-owned buffers, no exceptions
 * across the ABI.  Every function returns NWK_OK (0) or a negative NWK_E*
 * code; nwk_last_error() gives a thread-local message.  A context owns one
 * HIP device, its pooled HBM workspace and its streams; a context is not
 * re-entrant (one host thread per context), separate contexts may run
 * concurrently on different devices.
 *
 * Canonical pair order (skel:122-123): for i = 1..k-1, for j = 0..i-1, pair
 * id p = i*(i-1)/2 + j; genes[i] gives the DP rows (x), genes[j] the columns
 * (y).  There is no CPU fallback: every DP cell is computed by the HIP
 * kernels; a call without a usable device fails with NWK_EDEVICE.
 */
#ifndef NWK_H
#define NWK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NWK_OK 0
#define NWK_EINVAL (-1)   /* bad argument */
#define NWK_ENOMEM (-2)   /* host or device allocation failed */
#define NWK_EDEVICE (-3)  /* no HIP device / HIP runtime error */
#define NWK_EKERNEL (-4)  /* kernel reported a fault (hand-off timeout) */
#define NWK_ECOMM (-5)    /* RCCL error */

#define NWK_HASH_RAW 64   /* bytes of a raw SHA-512 digest */
#define NWK_HASH_HEX 129  /* 128 lowercase hex chars + NUL */

typedef struct nwk_ctx nwk_ctx;

typedef struct nwk_opts {
  int32_t device;            /* HIP device ordinal for nwk_ctx_create (default 0) */
  int32_t ngpus;             /* nwk_get_minimum_penalties: devices to shard over (0 = 1) */
  int32_t bits;              /* DP storage width 4/8/16/32; 0 = narrowest exact width */
  int32_t host_threads;      /* SHA-512 / finalize threads; 0 = min(16, cores) */
  int64_t workspace_bytes;   /* HBM budget per device; 0 = 92% of free memory */
  int32_t verbose;           /* 1 = per-call statistics on stderr */
  int32_t finalize;          /* pair finalize (rows, penalty, SHA-512): 0 auto, 1 host, 2 device (nw_rows + nw_hash
                                after each fill launch), 3 device fused into the nw_align_bits / nw_align_strip /
                                nw_align_col launch: each pair's record reaches the host as soon as it is hashed
                                (nwk_align_pairs_poll).  Auto fuses nw_align_col batches of >= 8,192 pairs in a
                                chained call, and streams nw_align_col pairs to host threads during the launch where
                                the host keeps up with the fill */
  int32_t linear_space;      /* linear-space traceback: 0 = only for pairs whose matrix exceeds
                                the HBM budget, -1 = never, G > 0 = every pair, G bands per recompute group */
  int32_t kernel;            /* linear fill kernel: 0 auto (where admissible -- pxy >= 0, pgap 1 or 2, <= 4
                                symbols -- nw_align_col, unless the job is more than 3 rounds of wave slots of
                                2048-row bands and has pairs longer than 16k, then nw_align_bits as band tasks or,
                                for jobs of many pairs per wave slot, one rolling strip per pair, nw_align_strip;
                                elsewhere the integer kernels), 1 nw_align, 2 nw_align_pk,
                                3 nw_align_pk2, 4 nw_align_bits band tasks, 5 nw_align_strip wherever admissible
                                (n / 64 in [63, 200] for pgap 2, [63, 500] for pgap 1), 6 nw_align_col (bit-parallel
                                columns, nw_align_bits' domain; a kernel where it is not exact -- W > 4, mixed-sign K,
                                pgap > 2 -- falls back), 7 nw_align_gotoh for the affine calls (bit-sliced Gotoh
                                planes; instantiated scorings only, else nw_align_pka / nw_align_affine).  Affine
                                calls under 0 take nw_align_gotoh where instantiated and <= 4 symbols, else
                                nw_align_pka where its int16 window holds, else nw_align_affine; 1 pins
                                nw_align_affine, 2 / 3 nw_align_pka */
  int32_t collective;        /* nwk_get_minimum_penalties: 1 = take the sharded RCCL all-gather path even when
                                ngpus == 1 (one communicator of one rank; tests the collective on a 1-GPU box) */
  int32_t task_order;        /* nw_align_bits band tasks: 0 auto (band-major above one round of wave slots), 1 pair-major
                                (pairs finish in the order given -- ascending ids stream out first, for
                                nwk_align_pairs_poll), 2 band-major */
} nwk_opts;

typedef struct nwk_stats {
  double fill_ms;            /* device time of the fill kernels incl. their fused traceback (HIP events) */
  double traceback_ms;       /* device time after the fill launches: segment gather + device finalize */
  double total_ms;           /* wall time of the call */
  double cells;              /* sum of m*n over the pairs of the call */
  int64_t matrix_bytes;      /* HBM bytes of the stored DP matrices */
  int32_t batches;           /* workspace batches used */
  int32_t bits;              /* storage width used */
  int32_t mode;              /* 0 = profile, 1 = compare, 2 = literal, 3 = affine, 4 = packed profile, 5 = packed band
                                pairs, 7 = packed affine band pairs, 8 = bit-sliced planes (nw_align_bits), 9 =
                                bit-sliced strips (nw_align_strip), 10 = bit-parallel columns (nw_align_col), 11 =
                                bit-sliced affine planes (nw_align_gotoh) */
  int32_t fill_launches;     /* fill-kernel launches in the call */
  int32_t device_finalized;  /* batches whose pairs were finalized on the device */
  int32_t linear_space_pairs; /* pairs aligned with the linear-space traceback */
  int32_t window_retries;    /* windowed storage: pairs re-run wider (path left the window) */
  int32_t window;            /* storage window W in columns of the call's first pairs (0 = full storage) */
  int32_t guard_checked;     /* pairs whose walked path's cost was checked against the fill's own dp[m][n] */
  int32_t guard_reruns;      /* pairs re-run because their walked path's cost differed from it (skel:274) */
} nwk_stats;

/* Defaults for nwk_opts (device 0, auto everything). */
void nwk_opts_default(nwk_opts *opts);

/* Thread-local description of the last error. */
const char *nwk_last_error(void);

/* Number of visible HIP devices (0 when none). */
int nwk_device_count(void);

int nwk_ctx_create(const nwk_opts *opts, nwk_ctx **out);
void nwk_ctx_destroy(nwk_ctx *ctx);

/*
 * Uploads the k sequences (concatenated in seqs, offsets[k+1]) to the
 * context's device; replaces the previous set.  Bytes are compared as raw
 * bytes (case-sensitive), exactly like std::string::operator[] in skel:215.
 */
int nwk_set_sequences(nwk_ctx *ctx, const uint8_t *seqs, const int64_t *offsets, int32_t k);

/*
 * The per-rank worker (sub:369-417): aligns pair_ids[0..npairs) of the
 * current sequence set.  penalties[npairs] and problem_hash[npairs*64] (raw
 * SHA-512 of sha512hex(align1) ++ sha512hex(align2), skel:155-157) are
 * written in the order of pair_ids.
 */
int nwk_align_pairs(nwk_ctx *ctx, const int64_t *pair_ids, int64_t npairs, int32_t pxy,
                    int32_t pgap, int32_t *penalties, uint8_t *problem_hash);

/*
 * nwk_align_pairs in two halves: _begin launches the call on a host thread of
 * the context and returns at once; _end waits for it and writes penalties[n]
 * and problem_hash[n*64] (order of pair_ids).  Between the two the context
 * must not be used (one call in flight).  A rank overlaps its exchange and the
 * chain of one chunk of its shard with the alignment of the next this way.
 */
int nwk_align_pairs_begin(nwk_ctx *ctx, const int64_t *pair_ids, int64_t npairs, int32_t pxy, int32_t pgap);
int nwk_align_pairs_end(nwk_ctx *ctx, int32_t *penalties, uint8_t *problem_hash);
/*
 * While a _begin call is in flight: copies the results of pair_ids[from ..
 * *upto) -- the longest run from `from` whose results are final -- into
 * penalties[] / problem_hash[] (indexed like pair_ids) and sets *upto.  With
 * the bits kernels' fused device finalize, each pair's record streams to the
 * host as soon as its traceback is done, so a rank can exchange (and rank 0
 * chain) a prefix of its shard while the rest still aligns -- the reference
 * collects results as they arrive, sub:305-331.  Returns the call's error once
 * it has ended without every result.
 */
int nwk_align_pairs_poll(nwk_ctx *ctx, int64_t from, int32_t *penalties, uint8_t *problem_hash, int64_t *upto);

/*
 * getMinimumPenalties on a context (skel:117-175, sub:232-364): aligns all
 * P = k(k-1)/2 pairs of the current sequence set, fills penalties[P] (and
 * problem_hash[P*64] unless NULL) in canonical order and writes the chained
 * answer hash (skel:159) into hash_hex[129].  The chain runs on the host
 * while later workspace batches are still on the GPU.
 */
int nwk_align_all(nwk_ctx *ctx, int32_t pxy, int32_t pgap, int32_t *penalties,
                  uint8_t *problem_hash, char *hash_hex);

/* Statistics of the context's last nwk_align_pairs call, or of its last nwk_msa call
 * (fill_ms = the nw_profile launches incl. their walks, cells = the merges' DP cells,
 * fill_launches = batches = guide-tree levels, mode 6, traceback_ms 0). */
int nwk_last_stats(const nwk_ctx *ctx, nwk_stats *out);

/*
 * getMinimumPenalties (skel:117-175): aligns all k(k-1)/2 pairs, fills
 * penalties[P] in canonical order and writes the chained answer hash into
 * hash_hex[129] ("" when P == 0).  With opts->ngpus = G > 1 the pairs are
 * cell-cost sharded over devices 0..G-1 (one host thread each) and the
 * 72-byte result records are collected with one ncclAllGather over xGMI.
 * opts may be NULL (defaults).
 */
int nwk_get_minimum_penalties(const uint8_t *seqs, const int64_t *offsets, int32_t k,
                              int32_t pxy, int32_t pgap, int32_t *penalties, char *hash_hex,
                              const nwk_opts *opts);

/*
 * getMinimumPenalty + trim (skel:186-280, 135-154) for one pair: a1/a2 get
 * the trimmed alignment rows (capacity m+n bytes each, not NUL-terminated),
 * *alen their length, *penalty = dp[m][n].
 */
int nwk_get_minimum_penalty(nwk_ctx *ctx, const uint8_t *x, int32_t m, const uint8_t *y,
                            int32_t n, int32_t pxy, int32_t pgap, uint8_t *a1, uint8_t *a2,
                            int32_t *alen, int32_t *penalty);

/*
 * Affine-gap variant (SURVEY.md §8 a9 -- no reference counterpart; the build
 * defines it, see oracle/nw_oracle.c nwo_pair_affine):
 *   E = min(E[i][j-1] + ge, H[i][j-1] + go + ge), F = min(F[i-1][j] + ge, H[i-1][j] + go + ge),
 *   H = x_i == y_j ? H[i-1][j-1] : min(H[i-1][j-1] + pxy, F, E),
 *   H[i][0] = go + i*ge, H[0][j] = go + j*ge, H[0][0] = 0.
 * Traceback DIAG > UP > LEFT as the reference, a gap closing (returning to
 * H) whenever its open term ties; prefix, trim and hashes as the linear path.
 * With go = 0, ge = pgap every result equals the linear entry point's.
 * Requires pxy, go, ge >= 0 (NWK_EINVAL otherwise).
 */
int nwk_align_pairs_affine(nwk_ctx *ctx, const int64_t *pair_ids, int64_t npairs, int32_t pxy,
                           int32_t go, int32_t ge, int32_t *penalties, uint8_t *problem_hash);
int nwk_get_minimum_penalty_affine(nwk_ctx *ctx, const uint8_t *x, int32_t m, const uint8_t *y,
                                   int32_t n, int32_t pxy, int32_t go, int32_t ge, uint8_t *a1,
                                   uint8_t *a2, int32_t *alen, int32_t *penalty);
int nwk_align_all_affine(nwk_ctx *ctx, int32_t pxy, int32_t go, int32_t ge, int32_t *penalties,
                         uint8_t *problem_hash, char *hash_hex);
int nwk_get_minimum_penalties_affine(const uint8_t *seqs, const int64_t *offsets, int32_t k,
                                     int32_t pxy, int32_t go, int32_t ge, int32_t *penalties,
                                     char *hash_hex, const nwk_opts *opts);

/*
 * Progressive sum-of-pairs MSA of the context's sequences (SURVEY.md §8 f3 --
 * the reference stops at the pairwise penalties, skel:117-175, so the build
 * defines it; oracle/msa_oracle.c nwo_msa is the restatement it must equal):
 * UPGMA guide tree on `penalties` (the P pairwise penalties in canonical order,
 * e.g. from nwk_align_all with the same pxy, pgap), then one profile-profile
 * Needleman-Wunsch per merge under SoP costs (c(a,a) = 0, c(a,b) = pxy,
 * c(a,'_') = pgap, c('_','_') = 0), traceback DIAG > UP > LEFT; merges of
 * independent subtrees run in one launch.  Writes the k aligned rows (row r
 * at rows + r*cap, '_' = gap), the MSA length and its SoP score.  For k = 2
 * the rows are the reference's alignment of pair (1, 0).
 * Requires pxy, pgap >= 0, no '_' in the input and at most 5 distinct bytes
 * (NWK_EINVAL otherwise); cap >= the MSA length (<= the summed lengths).
 */
int nwk_msa(nwk_ctx *ctx, int32_t pxy, int32_t pgap, const int32_t *penalties, uint8_t *rows,
            int64_t cap, int64_t *len, int64_t *sop);

/*
 * Deterministic cell-cost shard of the P pairs of a sequence set over world
 * ranks (LPT on m*n, ties by pair id).  Writes this rank's pair ids
 * (ascending) to out_ids (capacity P) and their count to *out_n.
 */
int nwk_shard_pairs(const int64_t *offsets, int32_t k, int32_t rank, int32_t world,
                    int64_t *out_ids, int64_t *out_n);

/*
 * Host finalize of one traced pair (the step after the GPU traceback): the
 * prefix fill (skel:263-272), trim (skel:135-154), penalty (the cost of the
 * traced path, = dp[m][n]) and problemhash (skel:155-157).  moves[0..nmoves)
 * is the traceback in walk order from (m, n): 'D' diagonal, 'U' up (x_i
 * against '_'), 'L' left ('_' against y_j); the walk must end on row 0 or
 * column 0 (NWK_EINVAL otherwise).  a1/a2 need m+n bytes each; problem_hash
 * gets the 64 raw bytes.  No device is needed.
 */
int nwk_finalize_moves(const uint8_t *x, int32_t m, const uint8_t *y, int32_t n, int32_t pxy,
                       int32_t pgap, const uint8_t *moves, int64_t nmoves, uint8_t *a1, uint8_t *a2,
                       int32_t *alen, int32_t *penalty, uint8_t *problem_hash);

/* Chain (skel:159): acc = sha512hex(acc ++ hex(problem_hash[p])), p = 0..P-1. */
int nwk_chain_hash(const uint8_t *problem_hash, int64_t P, char *hash_hex);

/*
 * Streaming chain of skel:159 over P pairs, fed in any order as results
 * arrive (sub:305-337 collects results out of order, then chains): a worker
 * thread advances the chain over the ready prefix of canonical ids while the
 * caller works.  feed: n records {pair id, penalty, raw problem hash}, each id
 * once (penalties may be NULL); finish: waits for the last link and writes
 * hash_hex[129] and, unless NULL, penalties[P] and problem_hash[P*64] in
 * canonical order (NWK_EINVAL if some pair was never fed).
 */
typedef struct nwk_chain nwk_chain;
int nwk_chain_create(int64_t P, nwk_chain **out);
int nwk_chain_feed(nwk_chain *ch, const int64_t *pair_ids, const int32_t *penalties,
                   const uint8_t *problem_hash, int64_t n);
int nwk_chain_finish(nwk_chain *ch, char *hash_hex, int32_t *penalties, uint8_t *problem_hash);
void nwk_chain_destroy(nwk_chain *ch);

/* sw::sha512::calculate equivalent: lowercase hex digest of data[0..len). */
void nwk_sha512_hex(const uint8_t *data, int64_t len, char *out_hex);

/* ---- Multi-process collectives over RCCL (one process per GPU) ----------
 * Replaces the reference's MPI exchange for the sharded path (sub:249-266
 * broadcasts, sub:296-331 task / result messages): each rank process aligns
 * its shard on its own device and the fixed-size result records travel by
 * ncclAllGather over xGMI.  The communicator lives in this library, so a rank
 * process binds exactly one HIP runtime and one RCCL (no second copy brought
 * in by a Python framework).  Rank 0 makes the id (NWK_COMM_ID_BYTES opaque
 * bytes) and hands it to the other ranks out of band; nwk_comm_create is
 * collective over all ranks.  Buffers are host memory; the library stages them
 * through device memory on its own stream, and every call returns after the
 * collective has completed. */
#define NWK_COMM_ID_BYTES 128
typedef struct nwk_comm nwk_comm;
int nwk_comm_unique_id(uint8_t *id);
int nwk_comm_create(int32_t device, const uint8_t *id, int32_t world, int32_t rank, nwk_comm **out);
/* recv (world x bytes) = every rank's send block (bytes), in rank order */
int nwk_comm_all_gather(nwk_comm *comm, const void *send, int64_t bytes, void *recv);
/* vals[0..n) = the maximum over ranks, element-wise (also a barrier) */
int nwk_comm_all_reduce_max_f64(nwk_comm *comm, double *vals, int64_t n);
void nwk_comm_destroy(nwk_comm *comm);
/* hipDeviceSynchronize on the device (the bench's timed-region brackets) */
int nwk_device_synchronize(int32_t device);

#ifdef __cplusplus
}
#endif
#endif /* NWK_H */
