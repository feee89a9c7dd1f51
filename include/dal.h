/*
 * dal.h -- C ABI of the MI355X-native active-learning query-selection path.
 *
 * Drop-in boundary for the hot path of dv66/Distributed-Active-Learning
 * (final_thesis/uncertainty_sampling.py, density_weighting.py,
 * cosine_similarity.py, similarity.py).  The reference calls Spark MLlib over
 * Py4J for every operation below; each entry point names the reference call
 * site it replaces.  A maintainer binds these with ctypes;
 * the in-tree binding is distributed-active-learning_amd/dal/_lib.py.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Every pointer is DEVICE memory owned by
 *    the caller (the library never allocates); ``stream`` is a hipStream_t
 *    (NULL = default stream) and every call is asynchronous and
 *    stream-ordered.  No global mutable state: calls are re-entrant.
 *  - Return value: DAL_OK (0) or a negative dal_status (argument / shape /
 *    launch errors, detected on the host before or at launch).
 *    Data-dependent conditions found by a kernel (zero-norm row, candidate
 *    overflow) are OR-ed into the caller's device word ``dev_status``
 *    (DAL_FLAG_*), which the caller reads after synchronising.
 *  - Pool rows are fp32, row-major with leading dimension ``ldx`` (floats).
 *  - Normalised pool buffer ``u``: [n_pad][d_pad] fp32, rows padded with zero
 *    rows to dal_pad_rows(n), features padded with zeros to
 *    dal_pad_features(d).  Zero rows/features contribute exactly 0.
 *  - Density accumulator: int64 fixed point, value = acc * 2^-32
 *    (DAL_FIXED_SCALE).  Integer adds are associative, so the density is
 *    bit-identical for any launch geometry and any number of GPUs.
 *  - Sort keys: uint64, smaller = better (dal_score_key() order); NaN scores
 *    map to DAL_KEY_NAN (last), rows that are not candidates to DAL_KEY_NONE.
 *    Ties are broken by the lower global row index.
 */
#ifndef DAL_H
#define DAL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* dal_stream_t; /* hipStream_t */
typedef void* dal_event_t;  /* hipEvent_t */

enum dal_status {
  DAL_OK = 0,
  DAL_ERR_ARG = -1,         /* null pointer / bad enum */
  DAL_ERR_SHAPE = -2,       /* size, padding or alignment contract violated */
  DAL_ERR_UNSUPPORTED = -3, /* e.g. tree deeper than DAL_MAX_TREE_DEPTH */
  DAL_ERR_HIP = -4,         /* HIP launch / attribute failure */
  DAL_ERR_CAPACITY = -5     /* k or candidate count above the kernel capacity */
};

/* bits OR-ed into *dev_status by kernels */
#define DAL_FLAG_ZERO_NORM 1      /* a pool row has ||x|| == 0 (cosine undefined) */
#define DAL_FLAG_CAND_OVERFLOW 2  /* re-rank candidate set exceeded capacity */
#define DAL_FLAG_RF_SPLITS 4      /* a feature produced more than num_splits + 1 thresholds */
#define DAL_FLAG_SAMPLE_MISS 8    /* fast top-k level 1 over capacity: re-run with level1_passes = 0 */

/* per-row flags (uint8 per pool row) */
#define DAL_ROW_CANDIDATE 1 /* row is in the unlabeled set and may be selected */
#define DAL_ROW_EXCLUDED 2  /* row is in E: dropped from density as i and as j */

#define DAL_DENSITY_NONE 0
#define DAL_DENSITY_FIXED 1
#define DAL_DENSITY_EXACT 2

#define DAL_ASCENDING 0
#define DAL_DESCENDING 1

#define DAL_KEY_NAN 0xFFFFFFFFFFFFFFFEull
#define DAL_KEY_NONE 0xFFFFFFFFFFFFFFFFull
#define DAL_FIXED_SCALE 4294967296.0 /* 2^32 */
#define DAL_ROW_GRANULE 512
#define DAL_CANON_CHUNK 256
#define DAL_MAX_TREE_DEPTH 16
#define DAL_SORT_CAP 8192          /* max pairs the single-block sort handles */
#define DAL_SORT_CAP_PAYLOAD 4096  /* ... when it also carries an fp64 payload */
#define DAL_RF_MAX_SPLITS 255          /* thresholds per feature (bins fit a uint8) */
#define DAL_RF_MAX_SPLIT_SAMPLE 16384  /* rows one threshold search sorts in LDS */
#define DAL_RF_MAX_DEPTH 10            /* deepest tree dal_rf_train grows */
#define DAL_RF_SPLIT_LDS_BYTES 163840  /* m * (num_splits + 2) * 8 must fit (one node's histogram, LDS) */

const char* dal_status_string(int status);
int dal_abi_version(void);
int64_t dal_pad_rows(int64_t n);
int64_t dal_pad_features(int64_t d);
/* Rigorous bound |d_gemm - d_canonical| <= dal_density_error_bound(n_cols)
 * for the fp32-MFMA density ("Density error bound"). */
double dal_density_error_bound(int64_t n_cols);

/* ---- (a1) row L2 normalisation --------------------------------------
 * Replaces density_weighting.py:66 / cosine_similarity.py:28 /
 * similarity.py:28  ``data.map(lambda _: _/np.linalg.norm(_))``.
 * norm64[i] = sqrt(sum_d x_id^2) in fp64 (sequential over d, no FMA);
 * u[i][d] = (float)(x_id / norm64[i]); rows with DAL_ROW_EXCLUDED and rows
 * n..n_pad-1 are written as zeros (E is dropped as j: density_weighting.py:95-100).
 * row_flags may be NULL.  A zero row sets DAL_FLAG_ZERO_NORM. */
int dal_normalize_rows(const float* x, int64_t n, int64_t d, int64_t ldx,
                       const uint8_t* row_flags, int64_t n_pad, int64_t d_pad,
                       float* u, double* norm64, int32_t* dev_status, dal_stream_t stream);

/* OR ``bits`` into flags[idx[t] - row_base] for every index of this shard
 * (0 <= idx - row_base < n): builds DAL_ROW_CANDIDATE from an unlabeled index
 * list without a host round trip. */
int dal_mark_rows(const int64_t* idx, int64_t count, int64_t row_base, int64_t n, int bits,
                  uint8_t* flags, dal_stream_t stream);
/* dal_mark_rows that also writes to *in_range (device int32, zeroed by the
 * call) how many of the count indices fall inside this shard -- the
 * candidate count of a shard given global candidates, with no extra pass
 * (ABI v4). */
int dal_mark_rows_count(const int64_t* idx, int64_t count, int64_t row_base, int64_t n, int bits,
                        uint8_t* flags, int32_t* in_range, dal_stream_t stream);

/* ---- canonical fp64 column sum (re-rank side of the density) -----------
 * partials[c][f] = sum over rows c*256 .. c*256+255 (< n, not EXCLUDED) of
 * x_rf / norm64[r], sequential in row order; rows of a shard start at a
 * multiple of 256.  dal_canon_colsum_reduce sums partials sequentially over c. */
int dal_canon_colsum_partials(const float* x, int64_t n, int64_t d, int64_t ldx,
                              const double* norm64, const uint8_t* row_flags,
                              double* partials, dal_stream_t stream);
int dal_canon_colsum_reduce(const double* partials, int64_t n_chunks, int64_t d,
                            double* colsum, dal_stream_t stream);
/* Separable canonical density (the exact identity sum_j <u_i,u_j> = <u_i, s>):
 * density[i] = sum_f (x_if / norm64[i]) * colsum[f], sequential, no FMA --
 * bit-identical to the re-rank and the oracle; NaN for EXCLUDED rows.
 * O(N*D), HBM-bound; the opt-in alternative to dal_gram_rowsum. */
int dal_density_separable(const float* x, int64_t n, int64_t d, int64_t ldx,
                          const double* norm64, const double* colsum, const uint8_t* row_flags,
                          double* density, dal_stream_t stream);

/* ---- (a2-a4) fused cosine Gram row-sum -------------------------------
 * Replaces density_weighting.py:67-75 (IndexedRowMatrix -> BlockMatrix
 * U.multiply(UT) -> toCoordinateMatrix().entries), :95-100 (L0 exclusion) and
 * :157-161 (groupByKey sum):  acc[i] += sum_j <u_rows[i], u_cols[j]> * 2^32.
 * Tiled fp32 MFMA (v_mfma_f32_32x32x2_f32) with the row-sum fused into the
 * accumulators; S is never materialised.  acc must be zeroed by the caller
 * (the call accumulates, so it can be issued once per column shard).
 * n_rows_pad % 256 == 0, n_cols_pad % 512 == 0, d_pad from dal_pad_features,
 * ld >= d_pad (floats).  grid_blocks <= 0 selects one block per CU. */
int dal_gram_rowsum(const float* u_rows, int64_t n_rows_pad, const float* u_cols,
                    int64_t n_cols_pad, int64_t d_pad, int64_t ld, int64_t* acc,
                    int grid_blocks, dal_stream_t stream);

/* ---- (a2-a4) the same row-sum on fp16 MFMA: symmetric + compensated -------
 * Same replaced reference lines as dal_gram_rowsum, at the fp16 matrix-core
 * rate.  dal_split_f16 writes each normalised fp32 row u (from
 * dal_normalize_rows, ld >= d_pad) at scale 2^12 as H = fp16(2^12 u),
 * L = fp16(2^12 u - H) (RNE) in the layout [n_pad][d_pad / KS][KS H halves |
 * KS L halves], KS = 128 if d_pad % 128 == 0, 32 if d_pad == 32, else 64
 * (dal_split_f16_halves(n_pad, d_pad) halves in all). */
int64_t dal_split_f16_halves(int64_t n_pad, int64_t d_pad);
int dal_split_f16(const float* u, int64_t n_pad, int64_t d_pad, int64_t ld, uint16_t* out,
                  dal_stream_t stream);
/* dal_normalize_rows + dal_split_f16 (one fused kernel) + optionally
 * dal_canon_colsum_partials, same bits (the fp32 unit rows never reach HBM): norm64[i] =
 * canonical ||x_i||, the split operand of the unit rows (E rows, zero-norm
 * rows and padding rows -> zeros) and, if partials != NULL, the canonical
 * column-sum partials [ceil(n / DAL_CANON_CHUNK)][d]; acc_zero (nullable,
 * int64 [n_pad]: the density accumulator the Gram adds into) is zeroed by the
 * same kernel (ABI v3).  n_pad % 512 == 0. */
int dal_prep_split(const float* x, int64_t n, int64_t d, int64_t ldx, const uint8_t* row_flags,
                   int64_t n_pad, int64_t d_pad, uint16_t* out, double* norm64, double* partials,
                   int64_t* acc_zero, int32_t* dev_status, dal_stream_t stream);
/* Symmetric (SYRK-style), compensated Gram row-sum (ABI v5; row sums only
 * since ABI v8).  S = U U^T is symmetric: rows are grouped in 512-row super
 * blocks (pairs of 256-row blocks) and each unordered pair {P, Q} is
 * multiplied once.  P takes Q iff Q == P, or Q > P and P+Q even, or Q < P and
 * P+Q odd (global indices, so the bits do not depend on the sharding).  The
 * taker's side is H only: per 32 features two v_mfma_f32_16x16x32_f16 (H.H,
 * H.L) form the row sums of <H_i, H_j + L_j> over the taken pairs (-> acc
 * rows of P).  dal_gram_sym_residual adds everything else in closed form:
 * the taker's remainder <L_i, H_j + L_j> and the pair's column sums for Q's
 * rows (sum over the P taking Q of <u~_j, sum_{i in P} u~_i>) -- acc holds the
 * density only after BOTH (any order; integer adds), and each call writes
 * only the acc rows of ITS row blocks (no cross-GPU density sum).  rows: the
 * operand of global 256-row blocks [row_block0, row_block0 + n_row_blocks)
 * (even counts); cols: the operand whose first block is global block
 * col_block0; column blocks [j_lo, j_hi) minus [skip_lo, skip_hi) are
 * processed (j_hi <= nb_active = pad512(N_total) / 256), so a caller can
 * split the columns over several calls.  acc is indexed by GLOBAL row
 * (>= nb_active * 256 entries, zeroed by the caller).  Chains are folded to
 * multiples of 2^-32 and added exactly (int64): the bits do not depend on the
 * grid, the column split or the GPU count.  Rigorous bound on |d -
 * d_canonical| of the completed density: dal_density_error_bound_sym_d. */
int dal_gram_rowsum_sym(const uint16_t* rows, int64_t row_block0, int64_t n_row_blocks,
                        const uint16_t* cols, int64_t col_block0, int64_t j_lo, int64_t j_hi,
                        int64_t nb_active, int64_t d_pad, int64_t* acc, int grid_blocks,
                        dal_stream_t stream);
int dal_gram_rowsum_sym_skip(const uint16_t* rows, int64_t row_block0, int64_t n_row_blocks,
                             const uint16_t* cols, int64_t col_block0, int64_t j_lo, int64_t j_hi,
                             int64_t skip_lo, int64_t skip_hi, int64_t nb_active, int64_t d_pad,
                             int64_t* acc, int grid_blocks, dal_stream_t stream);
/* The closed-form part of dal_gram_rowsum_sym's density for the rows of
 * global blocks [row_block0, row_block0 + n_row_blocks) (even), ADDED into acc
 * (global row index): acc[r] += rint(2^32 * (<L_r, R_B> + <H_r + L_r, C_B>)),
 * B = r's super block, R_B = sum over the super blocks B takes of their
 * (H + L) row sums (the taker side's remainder), C_B = the same sum over the
 * other super blocks that take B (their pairs' column sums for B's rows;
 * sigma~ since ABI v8) -- exact int64 sums in units of 2^-24, fp64 dots in a
 * fixed order.  ops: the
 * operand of EVERY active row (nb_active * 256 rows: the gathered operand on
 * several GPUs).  Three launches, O(N * D); workspace from
 * dal_gram_sym_residual_workspace_bytes (256-byte aligned). */
size_t dal_gram_sym_residual_workspace_bytes(int64_t nb_active, int64_t n_row_blocks, int64_t d_pad);
int dal_gram_sym_residual(const uint16_t* ops, int64_t nb_active, int64_t row_block0, int64_t n_row_blocks,
                          int64_t d_pad, int64_t* acc, void* ws, size_t ws_bytes, dal_stream_t stream);
double dal_density_error_bound_sym(int64_t n_cols);
/* The same bound for the kernel that runs features padded to d_pad (ABI v8):
 * the row-side chain length depends on the slice width KS (1,024 products at
 * KS 32, 2,048 at KS 64 / 128); dal_density_error_bound_sym(n) ==
 * dal_density_error_bound_sym_d(n, 0) is the longest chain's, valid for any
 * d_pad. */
double dal_density_error_bound_sym_d(int64_t n_cols, int64_t d_pad);

/* ---- (a5-a10) forest votes + uncertainty / density-weighted score ------
 * Replaces uncertainty_sampling.py:88-98 / density_weighting.py:136-167:
 * T x DecisionTreeModel.predict, groupByKey vote sum, the LUT score and the
 * e*d product.  Forest in complete-heap SoA layout (dal/forest.py):
 *   inner[t][h] = {feature (int32), threshold bits (fp32, rounded toward -inf
 *   from fp64 so that x32 <= t32  <=>  x <= t64)}, h < 2^depth - 1,
 *   leaf[t][l] in {0,1}, l < 2^depth.  x[f] <= thr -> child 2h+1, else 2h+2.
 * lut: fp64[T+1].  density_kind 0 (density NULL) -> uncertainty mode:
 * score = lut[v]; else score = lut[v] * d^beta (NaN for EXCLUDED rows) with
 * d = ((int64*)density)[i] * 2^-32 (kind DAL_DENSITY_FIXED, the GEMM
 * accumulator; interval scores) or d = ((double*)density)[i] (kind
 * DAL_DENSITY_EXACT, canonical fp64; exact scores, keys_hi == keys).
 * keys[i] = dal score key for ``order`` (DAL_KEY_NONE when not CANDIDATE).
 * In density mode the GEMM density is approximate, so each score is an
 * interval [score - err_i, score + err_i], err_i = |lut[v]| * density_err
 * (beta = 1; the d^beta image of the interval otherwise): keys[i] is the
 * PESSIMISTIC end's key and keys_hi[i] (nullable) the OPTIMISTIC end's key;
 * exact scores (lut[v] == 0 or NaN) have keys[i] == keys_hi[i]. */
int dal_forest_score(const float* x, int64_t n, int64_t d, int64_t ldx,
                     const int32_t* inner, const uint8_t* leaf, int32_t n_trees, int32_t depth,
                     const double* lut, const void* density, int density_kind, double density_err,
                     const uint8_t* row_flags, double beta, int order,
                     int32_t* votes, double* scores, uint64_t* keys, uint64_t* keys_hi,
                     dal_stream_t stream);

/* ---- (a5-a10) the same over the pool's blocked feature-major copy (ABI v9)
 * dal_pool_blocked writes the pool as tiles of 64 rows, feature-major inside
 * a tile: xb[(t * d + f) * 64 + r] = x[t * 64 + r][f], rows past n zero
 * (dal_pool_blocked_floats(n, d) floats; a per-pool copy, built once -- the
 * pool is constant across AL iterations).  dal_forest_score_blocked gives
 * dal_forest_score's outputs bit for bit; when dal_forest_blocked_rows(d,
 * n_trees, depth) is non-zero (the forest's node count bounds its distinct
 * features at <= 256, and a tile of those plus the forest fits 96 KiB of LDS)
 * it reads only the features the forest tests -- each tile's listed features
 * as 256-B runs (config 4, T = 10: ~116 of 256 features) -- else it runs
 * dal_forest_score's row-major kernel on x.  xb must be 16-B aligned.
 * Every inner node's feature must lie in [0, d) (the forest is device data, so
 * the library does not read it back to check; dal.forest.Forest.check_features
 * does before upload).  For an invalid forest the outputs are unspecified and
 * the two entry points differ: the blocked kernel clamps a feature into
 * [0, d - 1], the row-major kernel does not. */
int dal_forest_blocked_rows(int64_t d, int32_t n_trees, int32_t depth);
int64_t dal_pool_blocked_floats(int64_t n, int64_t d);
int dal_pool_blocked(const float* x, int64_t n, int64_t d, int64_t ldx, float* xb, dal_stream_t stream);
/* The prepared forest (ABI v10): the blocked kernel's per-block forest setup
 * (the distinct tested features, every node's feature remapped to its slot in
 * that list, the leaves) done ONCE per (forest, d) into a caller-owned device
 * buffer of dal_forest_prep_bytes(d, n_trees, depth) bytes (16-B aligned; 0
 * when dal_forest_blocked_rows is 0).  Pass it as ``fprep`` to
 * dal_forest_score_blocked / dal_dw_step / dal_dw_plan_create with the same
 * forest (inner, leaf, n_trees, depth) and d: each block of the score kernel
 * then copies it into LDS instead of rebuilding it; the outputs are the same
 * bits.  A stale fprep (another forest) gives that forest's votes: re-prepare
 * after the forest changes (stream-ordered: one launch, one block).  Reads the
 * forest arrays; a node feature outside [0, d) is clamped (as the unprepared
 * blocked kernel does) and counted in the buffer's second int32 word. */
size_t dal_forest_prep_bytes(int64_t d, int32_t n_trees, int32_t depth);
int dal_forest_prepare(const int32_t* inner, const uint8_t* leaf, int32_t n_trees, int32_t depth, int64_t d,
                       void* fprep, size_t fprep_bytes, dal_stream_t stream);
int dal_forest_score_blocked(const float* x, const float* xb, const void* fprep, int64_t n, int64_t d,
                             int64_t ldx, const int32_t* inner, const uint8_t* leaf, int32_t n_trees,
                             int32_t depth, const double* lut, const void* density, int density_kind,
                             double density_err, const uint8_t* row_flags, double beta, int order,
                             int32_t* votes, double* scores, uint64_t* keys, uint64_t* keys_hi,
                             dal_stream_t stream);

/* ---- (a11) top-k: sortBy(score).take(k) --------------------------------
 * Replaces uncertainty_sampling.py:106,109 / density_weighting.py:168,172.
 * The k smallest keys, ties -> lower index; out_idx = idx_base + row, sorted
 * by (key, index).  1 <= k <= min(n, DAL_SORT_CAP).  Exact radix select
 * (8 x 8-bit digit histograms) + ordered compaction + one-block bitonic sort. */
size_t dal_topk_workspace_bytes(int64_t n, int64_t k);
int dal_topk(const uint64_t* keys, int64_t n, int64_t k, int64_t idx_base, void* ws,
             size_t ws_bytes, int64_t* out_idx, uint64_t* out_keys, dal_stream_t stream);

/* ---- density-weighted selection with exact fp64 re-rank ----------------
 * Given the interval keys written by dal_forest_score (density mode,
 * DAL_DESCENDING): K = k-th smallest pessimistic key; candidates = every row
 * whose optimistic key is < K (or == K with a non-point interval) plus the
 * first k point-interval rows == K, in row order -- a superset of the
 * canonical top-k (at most ``cap`` of them).  Each candidate's canonical fp64
 * score  lut[v] * (sum_f (x_if / norm64[i]) * colsum[f])^beta  (sequential,
 * no FMA) is recomputed and an exact top-k over the candidates returns the k
 * best by (score desc, NaN last, index asc): bit-exact with the fp64 oracle.
 * out_scores are canonical fp64 scores, out_keys (nullable) their keys.  More
 * than ``cap`` candidates sets DAL_FLAG_CAND_OVERFLOW (retry with a larger cap).
 * colsum_ready (nullable): an event recorded after ``colsum`` was written on
 * another stream; the call makes ``stream`` wait for it just before the
 * re-rank (the radix select and compaction run without it), so a cold step's
 * canonical column sum overlaps the candidate search.
 * level1_passes > 0 (1..5; cap <= DAL_SORT_CAP_PAYLOAD): the fast level 1
 * (ABI v6) -- the pool is cut into <= 4096 row groups, tau = the k-th smallest
 * group-minimum pessimistic key (k keys of the pool, so tau >= K), and the
 * candidates are every row whose optimistic key is <= tau, found by scanning
 * only the groups whose minimum optimistic key is <= tau: a superset of the
 * exact candidates in two launches (group minima; tau + append with the
 * in-place canonical re-rank + the final sort by the block that finishes
 * last).  More than cap candidates sets DAL_FLAG_SAMPLE_MISS: re-run with
 * level1_passes = 0.  The selection is the same either way. */
size_t dal_dw_select_workspace_bytes(int64_t n, int64_t k, int64_t cap);
int dal_dw_select(const uint64_t* keys_lo, const uint64_t* keys_hi, const int32_t* votes,
                  const uint8_t* row_flags, int64_t n, int64_t k, int64_t idx_base,
                  const double* lut, double beta, const float* x, int64_t d, int64_t ldx,
                  const double* norm64, const double* colsum, int64_t cap, int32_t level1_passes, void* ws,
                  size_t ws_bytes, int64_t* out_idx, double* out_scores, uint64_t* out_keys,
                  int32_t* dev_status, dal_event_t colsum_ready, dal_stream_t stream);

/* ---- one density-weighted iteration in one call (a5-a11) ----------------
 * The body of density_weighting.py:133-176 for a cached density: equivalent to
 * dal_forest_score(x, ..., density_fixed, DAL_DENSITY_FIXED, density_err,
 * row_flags, beta, DAL_DESCENDING, votes, scores, keys_lo, keys_hi) followed by
 * dal_dw_select(keys_lo, keys_hi, votes, row_flags, n, k, idx_base, lut, beta,
 * x, d, ldx, norm64, colsum, cap, level1_passes, ...) -- same outputs, same
 * bits -- with the fast level 1 fused when level1_passes > 0 (and cap <=
 * DAL_SORT_CAP_PAYLOAD): the score kernel folds each block's minimum keys
 * into the row groups itself, and ONE more launch derives tau, appends the
 * candidates with their canonical scores and sorts them (capacity check:
 * DAL_FLAG_SAMPLE_MISS; the level-1 words are cleared for the next call).
 * step_flags:
 *   DAL_STEP_RESET_STATUS  *dev_status is zeroed at the start of the step (on
 *                          the device: a replayed hipGraph needs no memset node);
 *   DAL_STEP_WS_CLEAN      the workspace header is zero on entry (a previous
 *                          dal_dw_step left it so, or the caller zeroed the
 *                          workspace once): no zeroing launch.  The header is
 *                          left zero on exit whenever this flag is given.
 *   DAL_STEP_KEEP_GROUPS   (ABI v8; MEASUREMENT flag, fast level 1) the row-group
 *                          minima the step folded are left in the workspace
 *                          instead of cleared, so that DAL_STEP_SELECT_ONLY
 *                          calls can re-run the selection.  The workspace is
 *                          then NOT clean for a full step: the next call on it
 *                          MUST be DAL_STEP_SELECT_ONLY, and the sequence ends
 *                          with a SELECT_ONLY call without KEEP_GROUPS (which
 *                          clears the minima) before any full step uses the
 *                          workspace with DAL_STEP_WS_CLEAN again.
 *   DAL_STEP_SELECT_ONLY   (ABI v8; MEASUREMENT flag; with DAL_STEP_WS_CLEAN, fast
 *                          level 1, no DAL_STEP_RESET_STATUS) only the selection
 *                          launch: it re-reads the votes, keys and group minima
 *                          that the previous call with DAL_STEP_KEEP_GROUPS left
 *                          on the same buffers and workspace (the same
 *                          arguments), and gives the same outputs.  bench.py
 *                          times the fused step's selection launch on its own
 *                          with these two flags (time_step_select); the product
 *                          path never sets them.
 * xb (ABI v9; nullable): the pool's blocked copy (dal_pool_blocked) -- the
 * score kernel is then dal_forest_score_blocked's; fprep (ABI v10; nullable,
 * with xb): the forest prepared by dal_forest_prepare.
 * Workspace: dal_dw_step_workspace_bytes (== dal_dw_select's). */
#define DAL_STEP_RESET_STATUS 1u
#define DAL_STEP_WS_CLEAN 2u
#define DAL_STEP_KEEP_GROUPS 4u
#define DAL_STEP_SELECT_ONLY 8u
size_t dal_dw_step_workspace_bytes(int64_t n, int64_t k, int64_t cap);
int dal_dw_step(const float* x, const float* xb, const void* fprep, int64_t n, int64_t d, int64_t ldx,
                const int32_t* inner,
                const uint8_t* leaf,
                int32_t n_trees, int32_t depth, const double* lut, const int64_t* density_fixed,
                double density_err, const uint8_t* row_flags, double beta, int64_t idx_base,
                const double* norm64, const double* colsum, int64_t k, int64_t cap, int32_t level1_passes,
                uint32_t step_flags, void* ws, size_t ws_bytes, int32_t* votes, double* scores,
                uint64_t* keys_lo, uint64_t* keys_hi, int64_t* out_idx, double* out_scores,
                uint64_t* out_keys, int32_t* dev_status, dal_event_t colsum_ready, dal_stream_t stream);

/* ---- warm-step plan: a replayed dal_dw_step with a one-call host side -----
 * dal_dw_plan_create captures dal_dw_step (DAL_STEP_RESET_STATUS |
 * DAL_STEP_WS_CLEAN, no colsum event) over the given caller-owned buffers as a
 * hipGraph (the workspace is zeroed once, synchronously on ``stream``).
 * ``flags`` is the step's row-flag scratch: runs with the exact level 1
 * (level1_passes = 0) rebuild it from ``base_flags`` (the pool's EXCLUDED
 * bits) and the unlabeled list; with the fast level 1 the re-rank derives its
 * candidates' flags from the step's row stamps and ``flags`` is not written
 * (ABI v7); the
 * selection lands in out_pair[0..k) (indices) and out_pair[k..2k) (fp64
 * score bits).  dal_dw_plan_run(plan, unl, n_unl, out_idx, out_scores,
 * status, stream): flags <- base_flags, mark unl as DAL_ROW_CANDIDATE, replay
 * (the graph's last kernel also writes the selection to out_idx / out_scores
 * -- nullable, k each -- and the final status word to host-mapped memory),
 * wait for that word (a bounded spin, then a stream sync) and return the
 * status in *status -- the
 * density_weighting.py:133-176 iteration in one call.  Buffers must outlive
 * the plan; dal_dw_plan_destroy frees it.  xb (ABI v9) and fprep (ABI v10;
 * both nullable): as dal_dw_step's -- the plan reads fprep at its captured
 * address on every replay, so a new forest is re-prepared into the same
 * buffer before the next run. */
typedef struct dal_dw_plan dal_dw_plan_t;
int dal_dw_plan_create(const float* x, const float* xb, const void* fprep, int64_t n, int64_t d, int64_t ldx,
                       const int32_t* inner,
                       const uint8_t* leaf, int32_t n_trees, int32_t depth, const double* lut,
                       const int64_t* density_fixed, double density_err, const uint8_t* base_flags,
                       uint8_t* flags, double beta, int64_t idx_base, const double* norm64,
                       const double* colsum, int64_t k, int64_t cap, int32_t level1_passes, void* ws,
                       size_t ws_bytes, int32_t* votes, double* scores, uint64_t* keys_lo, uint64_t* keys_hi,
                       int64_t* out_pair, uint64_t* out_keys, int32_t* dev_status, dal_stream_t stream,
                       dal_dw_plan_t** plan);
int dal_dw_plan_run(dal_dw_plan_t* plan, const int64_t* unl, int64_t n_unl, int64_t* out_idx,
                    double* out_scores, int32_t* status, dal_stream_t stream);
/* The plan's replay WITHOUT the host wait (ABI v5): refreshes the row marks,
 * launches the graph on ``stream`` and returns.  The outputs stay in the
 * buffers given at creation (out_keys, out_pair = selected indices | score
 * bits, dev_status) -- e.g. one packed row [keys k | indices k | score bits
 * k | status] that a multi-GPU caller all-gathers and merges stream-ordered,
 * reading the status once after the merge. */
int dal_dw_plan_launch(dal_dw_plan_t* plan, const int64_t* unl, int64_t n_unl, dal_stream_t stream);
void dal_dw_plan_destroy(dal_dw_plan_t* plan);

/* ---- (a12, config 5) max-cosine to a labeled set -----------------------
 * Restates similarity.py:26-43 (columnSimilarities of the normalised pool) as
 * m_i = max_{l in L} cos(x_i, x_l) over a bf16 pool (row-major [n][d],
 * d in {64,128,256}) and a bf16 labeled table [m_pad][d] whose rows beyond the
 * real m carry inv_lab = NaN (ignored).  bf16 MFMA (v_mfma_f32_32x32x16_bf16),
 * fp32 accumulate, row-max epilogue; the n x m matrix is never stored.
 * m_pad % dal_maxcos_label_rows_granule(d) == 0, m_pad <= 4096.  inv_pool
 * (nullable): per-row 1/||x_i||; NULL computes it in-kernel (the diagonal of
 * the register-resident row fragments' own Gram, fp32 sums of exact products).
 * |m_gpu - m_canonical| <= dal_maxcos_error_bound(d) (Cauchy-Schwarz). */
int64_t dal_maxcos_label_rows_granule(int64_t d);
double dal_maxcos_error_bound(int64_t d);
int dal_inv_norms_bf16(const uint16_t* x, int64_t n, int64_t n_pad, int64_t d, int64_t ld,
                       float* inv, int32_t* dev_status, dal_stream_t stream);
/* Canonical fp64 unit rows (sequential fp64 norm, then divide) of n bf16
 * rows: u[i * d + f] (feature_major = 0) or u[f * n + i] (feature_major = 1). */
int dal_canon_unit_rows_bf16(const uint16_t* x, int64_t n, int64_t d, int64_t ld, int feature_major,
                             double* u, dal_stream_t stream);
/* out_arg (nullable): the arg-max l (position in the labeled table, first l
 * among equal values) of every row.  A row whose two largest fp32 cosines are
 * within 2 x dal_maxcos_error_bound(d) of each other cannot be ordered from
 * the fp32 values: it gets -1 - l, and dal_maxcos_argmax_resolve replaces
 * every such entry by the canonical fp64 arg-max (similarity.py:34-38,
 * columnSimilarities' exact cosines; ties -> first l).  Every other entry is
 * already the canonical arg-max. */
int dal_max_cosine(const uint16_t* pool, int64_t n, int64_t d, const uint16_t* lab, int64_t m_pad,
                   const float* inv_lab, const float* inv_pool, float* out_max, int32_t* out_arg,
                   int32_t* dev_status, dal_stream_t stream);
/* Max-cosine WITHOUT the arg-max on a folded labeled operand (ABI v7; the
 * diversity selection's values): lab_unit = dal_unit_rows_f16's fp16 table
 * 2^15 x_l / ||x_l|| [m_pad][d] (no per-column scaling left in the kernel:
 * the epilogue is a bare running max).  Each pool row is rescaled by a power
 * of two and converted to fp16 in registers; v_mfma_f32_16x16x32_f16.
 * |m_gpu - m_canonical| <= dal_maxcos_unit_error_bound(d) (~2^-11: the fp16
 * rounding of the unit rows; the selection stays exact through the fp64
 * re-rank).  Rows whose largest |x_if| is zero or a bf16 subnormal flag
 * DAL_FLAG_ZERO_NORM, as in dal_max_cosine. */
int dal_unit_rows_f16(const uint16_t* x, int64_t m, int64_t m_pad, int64_t d, int64_t ld, uint16_t* out,
                      int32_t* dev_status, dal_stream_t stream);
double dal_maxcos_unit_error_bound(int64_t d);
int dal_max_cosine_unit(const uint16_t* pool, int64_t n, int64_t d, const uint16_t* lab_unit, int64_t m_pad,
                        float* out_max, int32_t* dev_status, dal_stream_t stream);
/* Canonical fp64 arg-max (oracle max_cosine_canonical: sequential norm and
 * dot products, no FMA, first l on ties) of every row with out_arg < 0;
 * ulab = canonical fp64 unit rows of the m labeled rows, feature-major [d][m]
 * (dal_canon_unit_rows_bf16 with feature_major = 1); d <= 256. */
int dal_maxcos_argmax_resolve(const uint16_t* pool, int64_t n, int64_t d, int64_t ld, const double* ulab,
                              int64_t m, int32_t* out_arg, dal_stream_t stream);
/* Interval keys [v - err, v + err] of fp32 values (pessimistic -> keys_lo). */
int dal_interval_keys_f32(const float* values, int64_t n, double err, const uint8_t* row_flags,
                          int order, uint64_t* keys_lo, uint64_t* keys_hi, dal_stream_t stream);
/* Diversity selection: the k rows with the smallest canonical fp64 max-cosine
 * (ties -> lower index), from interval keys of dal_max_cosine's output;
 * ulab = canonical fp64 unit rows of the m labeled rows, feature-major
 * [d][m] (dal_canon_unit_rows_bf16 with feature_major = 1); d <= 256.  Same candidate/re-rank contract
 * as dal_dw_select, including level1_passes (0 = exact radix level 1; 1-5 =
 * the fast group-minimum level 1, DAL_FLAG_SAMPLE_MISS when its candidates
 * overflow cap <= 4096). */
size_t dal_maxcos_select_workspace_bytes(int64_t n, int64_t k, int64_t cap);
int dal_maxcos_select(const uint64_t* keys_lo, const uint64_t* keys_hi, int64_t n, int64_t k,
                      int64_t idx_base, const uint16_t* pool, int64_t d, int64_t ld,
                      const double* ulab, int64_t m, int64_t cap, int32_t level1_passes, void* ws,
                      size_t ws_bytes,
                      int64_t* out_idx, double* out_scores, uint64_t* out_keys,
                      int32_t* dev_status, dal_stream_t stream);

/* ---- multi-GPU merge ----------------------------------------------------
 * Sort n (key, idx) pairs (e.g. the all-gathered per-GPU top-k lists) by
 * (key, idx) and keep the first k.  n <= DAL_SORT_CAP.  ``payload`` (nullable)
 * is permuted alongside (then n <= DAL_SORT_CAP_PAYLOAD). */
int dal_sort_pairs(const uint64_t* keys, const int64_t* idx, const double* payload, int64_t n,
                   int64_t k, uint64_t* out_keys, int64_t* out_idx, double* out_payload,
                   dal_stream_t stream);

/* dal_topk_merge: the same merge read straight from one all-gather's output.
 * packed [n_ranks][width] int64 rows = a rank's k keys | k global indices |
 * k fp64 score bit patterns (| its status word at 3k when status_or is
 * given).  Writes the k best by (key, rank-major position) -- ties resolve
 * by global row index -- to out_idx / out_scores, and the OR of the status
 * words to *status_or (nullable), the winners' keys to out_keys (nullable;
 * DAL_KEY_NONE marks padding that won only because fewer than k candidates
 * exist).  n_ranks * k <= DAL_SORT_CAP.  One launch and no workspace (ws may
 * be NULL; dal_topk_merge_workspace_bytes returns 0) when n_ranks * k <=
 * DAL_SORT_CAP_PAYLOAD and n_ranks <= 32: the rows are read in place by the
 * one-block sort, ordered by (key, global index) -- the same order, as ranks
 * hold ascending row ranges; otherwise three launches (unpack, sort, gather).
 * Replaces the sortBy(...).take(k) of density_weighting.py:168,172 across
 * shards (the Spark range-partition sort over all executors). */
size_t dal_topk_merge_workspace_bytes(int64_t n_ranks, int64_t k);
int dal_topk_merge(const int64_t* packed, int64_t n_ranks, int64_t width, int64_t k, void* ws, size_t ws_bytes,
                   int64_t* out_idx, double* out_scores, uint64_t* out_keys, int32_t* status_or,
                   dal_stream_t stream);

/* ---- pool ingest (host-side parser) -------------------------------------
 * Replaces uncertainty_sampling.py:37-42 / density_weighting.py:45-53,59-65
 * (sc.textFile -> split -> LabeledPoint(0 if int(_[-1]) == -1 else 1,
 * np.array(_[:-1]).astype(float)), take(n_samples)).  HOST pointers (the one
 * exception to the device-pointer convention): ``text`` is a byte range of
 * whitespace-separated rows, label last; blank lines are skipped.
 * dal_text_shape: rows (at most max_rows if >= 0) and fields per row.
 * dal_parse_labeled_text: x [rows][cols-1] fp32 = (float)strtod(field) (the
 * bits of np.float64 parsing narrowed to fp32), labels [rows] (label_map 0:
 * -1 -> 0, else 1; 1: as is); x may be pinned memory handed straight to an
 * async H2D copy.  DAL_ERR_SHAPE: ragged rows; DAL_ERR_ARG: a bad field. */
int dal_text_shape(const char* text, size_t len, int64_t max_rows, int64_t* rows, int64_t* cols);
int dal_parse_labeled_text(const char* text, size_t len, int64_t rows, int64_t cols, int label_map, float* x,
                           int64_t* labels, int n_threads);

/* ---- GPU random-forest training ---------------------
 * Replaces RandomForest.trainClassifier(train, numClasses=2,
 * categoricalFeaturesInfo={}, numTrees=T, featureSubsetStrategy="auto",
 * impurity='gini', maxDepth=4, maxBins=32) (uncertainty_sampling.py:71-76,
 * density_weighting.py:119-124; Spark 2.1 MLlib, continuous features, binary
 * labels).  The training rows x [n][ldx] fp32 are the labeled set.
 *
 * dal_rf_find_splits: findSplitsForContinuousFeature per feature over the
 * sample rows (sample_rows nullable = rows 0..n_sample-1; n_sample <=
 * DAL_RF_MAX_SPLIT_SAMPLE): thresholds [d][DAL_RF_MAX_SPLITS] fp32 (ascending),
 * n_splits [d].  num_splits = min(maxBins, n) - 1.  A feature that would emit
 * more than num_splits + 1 thresholds sets DAL_FLAG_RF_SPLITS in *dev_status.
 *
 * dal_rf_train: grows T trees level by level on the given bagging weights
 * [T][n] (integer Poisson counts; 0 = row not drawn) and per-node feature
 * subsets [T][2^max_depth - 1][m] (heap order, evaluation order; MLlib draws
 * both from JVM RNGs, so they are inputs).  Gini gain in fp64 in MLlib's
 * operation order, first maximum over subset order then split index; a node
 * is a leaf when gain <= 0 (or no valid split) or at max_depth; a child is
 * created as a leaf when pure.  Output in dal_forest_score's heap layout:
 * out_inner [T][2^D - 1][2] = (feature, fp32 threshold bits), (0, +inf) below
 * a leaf; out_leaf [T][2^D] = class (first maximum of the weighted counts),
 * a shallow leaf's class repeated over its subtree.  ws: 256-B aligned,
 * dal_rf_train_workspace_bytes(...) bytes. */
int dal_rf_find_splits(const float* x, int64_t n, int64_t d, int64_t ldx, const int64_t* sample_rows,
                       int64_t n_sample, int32_t num_splits, float* thresholds, int32_t* n_splits,
                       int32_t* dev_status, dal_stream_t stream);
size_t dal_rf_train_workspace_bytes(int64_t n, int64_t d, int32_t n_trees, int32_t max_depth, int32_t m,
                                    int32_t num_splits);
int dal_rf_train(const float* x, int64_t n, int64_t d, int64_t ldx, const uint8_t* labels,
                 const float* thresholds, const int32_t* n_splits, int32_t num_splits, const int32_t* weights,
                 const int32_t* feature_subsets, int32_t m, int32_t n_trees, int32_t max_depth,
                 int32_t min_instances, double min_info_gain, int32_t* out_inner, uint8_t* out_leaf, void* ws,
                 size_t ws_bytes, dal_stream_t stream);

/* ---- standalone similarity kernels --------------------------------------
 * cosine_similarity.py:42-45: every entry of U.U^T (fp32 MFMA), written to
 * out[n_pad][n_pad] (fp32).  similarity.py:38 (columnSimilarities, i<j) is
 * the strict upper triangle of the same matrix. */
int dal_gram_entries(const float* u, int64_t n_pad, int64_t d_pad, int64_t ld, float* out,
                     dal_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* DAL_H */
