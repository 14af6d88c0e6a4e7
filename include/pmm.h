/*
 * pmm.h -- C ABI of the MI355X-native similarity-search engine (libpmm.so).
 *
 * Drop-in boundary for the reference's `.pmm.topk` / `.pmm.matmul` hot path
 * (NivekNey/polars-matmul v0.1.4).  The reference binds its Rust numerics to
 * Python through pyo3 (src/lib.rs:15-62); the numerics themselves are
 * src/matmul.rs:295-519, src/metrics.rs:38-393 and src/topk.rs:1-75.  Every
 * entry point below names the reference function it replaces.  Plain pointers
 * and sizes only: no torch / Arrow / Polars types cross this boundary.
 *
 * Conventions
 *   - Matrices are row-major.  Q is m x d (queries), C is n x d (corpus).
 *   - Return value: PMM_OK (0) or a PMM_ERR_* code; the message of the last
 *     failure on the calling thread is available from pmm_last_error().
 *   - Thread safety: every entry point may be called concurrently from
 *     different threads (each thread owns its HIP stream and scratch).  The
 *     reference runs two `.pmm` expressions concurrently inside one Polars
 *     plan (tests/test_polars_matmul.py:551-572).
 *   - Result order per query row: best first (descending score for cosine /
 *     dot, ascending distance for euclidean); equal scores break to the lower
 *     corpus index; NaN scores rank last.  The reference leaves the order of
 *     equal scores unspecified (src/topk.rs:55-59, partial_cmp -> Equal).
 */
#ifndef PMM_H_
#define PMM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PMM_OK 0
#define PMM_ERR_ARG 1         /* invalid argument (sizes, pointers, metric) */
#define PMM_ERR_HIP 2         /* HIP runtime error (message has the HIP text) */
#define PMM_ERR_UNSUPPORTED 3 /* combination not supported by this build */
#define PMM_ERR_NODEVICE 4    /* no gfx950 device visible */

/* Metric ids; src/metrics.rs:10-18 `enum Metric`. */
#define PMM_METRIC_COSINE 0
#define PMM_METRIC_DOT 1
#define PMM_METRIC_EUCLIDEAN 2

/* Arithmetic the top-k GEMM runs in (f32 inputs).  F32 = exact f32 MFMA
 * (v_mfma_f32_32x32x2_f32), the reference's precision.  BF16 = inputs rounded
 * to bf16 (round to nearest even) on device, products accumulated in f32
 * (v_mfma_f32_16x16x32_bf16), norms of the rounded rows in f32: the result is
 * the top-k of the bf16-rounded embeddings (BASELINE configs[3]).  The bf16
 * MFMA kernels take d <= 768, k <= 960 and n < 2^27; beyond (configs[4]'s
 * d = 1024, larger k) the rounded rows are widened to f32 exactly and
 * searched by the f32 path: the same bar (exact top-k of the rounded rows up
 * to f32 accumulation order) at the f32 MFMA rate. */
#define PMM_COMPUTE_F32 0
#define PMM_COMPUTE_BF16 1

const char *pmm_version(void);

/* Message of the last failing call on this thread ("" if none). */
const char *pmm_last_error(void);

/* Replaces Metric::from_str (src/metrics.rs:20-27): case-insensitive
 * "cosine" | "dot" | "euclidean" | "l2".  Unknown names return PMM_ERR_ARG with
 * pmm_last_error() = "Unknown metric: '<s>'. Supported: cosine, dot, euclidean"
 * (the reference's text, src/metrics.rs:25). */
int pmm_metric_from_str(const char *s, int *metric);

/* Replaces Metric::higher_is_better (src/metrics.rs:30-35). */
int pmm_metric_higher_is_better(int metric);

int pmm_device_count(int *count);
/* Free and total HBM of the device this thread's host calls run on
 * (hipMemGetInfo); the corpus cache sizes itself by it.  No reference
 * counterpart (the reference has no device memory). */
int pmm_device_memory(size_t *free_bytes, size_t *total_bytes);
/* Selects the HIP device that later HOST-buffer calls on this thread run on
 * (pmm_topk_f32*, pmm_topk_f64, pmm_matmul_*, pmm_corpus_create_f32,
 * pmm_device_memory); they restore the caller's current device on return.
 * Device-pointer entry points (*_device) ignore it and run on the caller's
 * current HIP device (hipSetDevice), where their pointers live. */
int pmm_set_device(int device);

/* Multi-GPU through the drop-in boundary (no reference
 * counterpart -- the reference is single-process, src/lib.rs:33-55).  With a
 * list of n >= 2 devices, pmm_topk_f32 / pmm_topk_f32_ex (k <= 1024) and
 * corpora created afterwards by pmm_corpus_create_f32 row-shard the corpus
 * over the list, one contiguous shard per entry (sizes differ by <= 1; at most
 * n shards).  Every device runs the fused top-k on its shard with global
 * indices, the per-shard [2][m][k] lists are copied peer to peer (xGMI) to
 * ids[0] and k-way merged there: the result equals the one-device result bit
 * with f32 compute (PMM_COMPUTE_F32): a shard's list is the exact top-k of
 * its rows under the total order (score, then lower index), so the merged
 * list equals the one-device result bit for bit.  With PMM_COMPUTE_BF16 the
 * result is the exact top-k of the bf16-rounded rows up to f32 accumulation
 * order, as on one device; the shard size can change which bf16 kernel and
 * threshold seed run, so near-ties may resolve differently than on one device
 * (tests assert > 99% index agreement).  A device may be listed more than once
 * (one shard per entry).  A one-entry list moves every host call to that
 * device.  The f64 entries (pmm_topk_f64, pmm_corpus_create_f64 /
 * pmm_topk_f64_corpus; any k) shard the same way: each device runs the f64
 * top-k on its shard (k_g = min(k, shard rows), padded with empty slots), the
 * [m][k] (index, f64 score) lists meet on ids[0] and are k-way merged there,
 * bit-equal to one device (indices and f64 scores).  Work that is not sharded
 * (f32 k > 1024, pmm_matmul_*) runs on ids[0].  Process-wide; n = 0 (or ids = NULL) returns to one device
 * (pmm_set_device's).
 * VERIFIED ON ONE GPU ONLY: the one-GPU test box lists device 0 repeatedly,
 * which plans all shards onto one stream; the distinct-device branch
 * (concurrent devices, cross-device event waits, peer copies over xGMI) has
 * not run on a multi-GPU node yet (tests/test_gpu_parity.py
 * test_set_devices_distinct_gpus runs it where >= 2 GPUs are visible). */
int pmm_set_devices(const int *ids, int n);
/* The current device list: *n entries, the first min(cap, *n) copied to ids. */
int pmm_get_devices(int *ids, int cap, int *n);
/* Diagnostics (no reference counterpart; no HIP call, runs without a GPU):
 * the memory plan the sharded search uses for G shards of an n-row corpus
 * over devs[0..G-1] (shard g = rows [n g / G, n (g + 1) / G)).  One plan per
 * DISTINCT device: plan_of[g] = the plan running shard g, *n_plans plans with
 * plan_dev[j] its device and plan_bytes[j] its device-memory bytes (queries,
 * host_rows ? uploaded shard rows : nothing, per-shard [2][m][k] lists at
 * list_offsets[g] inside the plan, one workspace; the root plan, plan_of[0],
 * also the gathered [G][2][m][k] lists and the merged output).  All output
 * arrays hold G entries. */
int pmm_shard_plan(const int *devs, int G, int64_t m, int64_t n, int64_t d, int64_t k, int metric, int compute,
                   int host_rows, int *plan_of, int *plan_dev, uint64_t *plan_bytes, uint64_t *list_offsets,
                   int *n_plans);

/* ---------------------------------------------------------------------------
 * Host-buffer entry points (what `_topk` / `_matmul` call; src/lib.rs:15-55).
 * Inputs are borrowed for the duration of the call and copied to HBM; outputs
 * are caller-allocated host buffers.
 * ------------------------------------------------------------------------- */

/* Replaces compute_topk_indices_scores, f32 branch (src/matmul.rs:429-448):
 * compute_similarity_matrix_f32 (src/metrics.rs:314-365) +
 * select_topk_with_scores_f32 (src/topk.rs:42-75), fused so the m x n score
 * matrix is never materialised.  k is clipped to n (src/matmul.rs:443) by the
 * caller; out_idx / out_score hold m*k entries.  Scores are f32 here; the
 * Python layer widens them to f64 as src/matmul.rs:447 does. */
int pmm_topk_f32(const float *q, int64_t m, const float *c, int64_t n, int64_t d, int64_t k,
                 int metric, uint32_t *out_idx, float *out_score);

/* Same with an explicit compute mode (PMM_COMPUTE_F32 / PMM_COMPUTE_BF16). */
int pmm_topk_f32_ex(const float *q, int64_t m, const float *c, int64_t n, int64_t d, int64_t k,
                    int metric, int compute, uint32_t *out_idx, float *out_score);

/* Replaces compute_topk_indices_scores, f64 branch (src/matmul.rs:449-468):
 * compute_similarity_matrix (src/metrics.rs:258-311) +
 * select_topk_with_scores (src/topk.rs:6-39). */
int pmm_topk_f64(const double *q, int64_t m, const double *c, int64_t n, int64_t d, int64_t k,
                 int metric, uint32_t *out_idx, double *out_score);

/* The same f64 top-k on device rows (row strides >= roundup(d, 16), zero-
 * padded, 16-byte-aligned bases) on the caller's stream; out_idx / out_score
 * are device buffers of m*k entries, indices offset by index_base.  k <=
 * 1024 and an m x n score matrix of 256 MB or more: fused (f64 MFMA GEMM whose
 * epilogue appends each element that beats its row's running k-th to a
 * candidate buffer, the corpus scanned in growing column chunks with the k-th
 * raised between chunks: no m x n matrix), else (or when a row's buffer
 * overflows) the materialised GEMM + row select.  The fused scan
 * synchronises the stream before returning (its overflow check); the
 * materialised path returns with the work queued on the stream. */
int pmm_topk_f64_device(const double *q, int64_t ldq, int64_t m, const double *c, int64_t ldc, int64_t n,
                        int64_t d, int64_t k, int metric, uint32_t index_base, uint32_t *out_idx,
                        double *out_score, void *stream);

/* Replaces matmul_slice_f32 / matmul_f32 (src/metrics.rs:160-202, :204-255):
 * out (m x n, row-major) = Q * C^T. */
int pmm_matmul_f32(const float *q, int64_t m, const float *c, int64_t n, int64_t d, float *out);

/* Page-locked host memory for results (hipHostMalloc, portable to every
 * device).  `.pmm.matmul` returns an m x n matrix (40 MB at the reference
 * benchmark's size): written into a fresh pageable buffer, the call pays that
 * buffer's page faults and the runtime's staging; into a page-locked one the
 * D2H copy runs at link rate.  The Python layer keeps a pool of these and
 * hands them to Arrow as foreign buffers (the reference moves its result Vec
 * into the Series the same way, src/matmul.rs:116-124).  No reference
 * counterpart of the allocation itself. */
int pmm_host_alloc(size_t bytes, void **out);
int pmm_host_free(void *p);

/* Replaces matmul_slice_f64 / matmul_f64 (src/metrics.rs:111-157, :40-97). */
int pmm_matmul_f64(const double *q, int64_t m, const double *c, int64_t n, int64_t d,
                   double *out);

/* ---------------------------------------------------------------------------
 * Device-resident entry points: inputs already in HBM, work enqueued on the
 * caller's HIP stream (NULL = the HIP default stream, as in the HIP API), no
 * host synchronisation.
 * Used by the benchmark and the multi-GPU (corpus-sharded) path.
 * ------------------------------------------------------------------------- */

/* Scratch bytes pmm_topk_f32_device (compute F32) or pmm_topk_bf16_device
 * (compute BF16) needs for this problem. */
size_t pmm_topk_workspace_bytes(int64_t m, int64_t n, int64_t d, int64_t k, int metric,
                                int compute);

/* Algorithmic bytes of the last fused top-k's merge pass (merge_kernel) for
 * this problem and workspace, read after the call completed: the split
 * counts, the candidates the GEMM left, the shared thresholds and the m x k
 * output.  Measurement only (the HBM-roofline line of the reduction,
 * SURVEY 8d); synchronous. */
int pmm_topk_merge_bytes(const void *workspace, int64_t m, int64_t n, int64_t d, int64_t k,
                         int metric, int compute, uint64_t *bytes);

/* Fused top-k over device buffers.  d is the logical dimension; ldq / ldc are
 * row strides in elements, multiples of 4 and >= roundup(d, 32), with columns
 * d..roundup(d, 32)-1 zero-filled and 16-byte-aligned bases (pmm_topk_f32 pads
 * host inputs itself).  Norms use exactly d elements in the reference's order
 * (ndarray unrolled_dot).  index_base is added to every
 * returned corpus index (global index of corpus row 0 of this shard).  For
 * k <= 1024, k may exceed n (a small shard): slots past n are empty (index
 * 0xFFFFFFFF, score NaN).  workspace may be NULL (a per-thread cached buffer
 * is used). */
int pmm_topk_f32_device(const float *q, int64_t ldq, int64_t m, const float *c, int64_t ldc,
                        int64_t n, int64_t d, int64_t k, int metric, int compute,
                        uint32_t index_base, uint32_t *out_idx, float *out_score,
                        void *workspace, size_t workspace_bytes, void *stream);

/* The bf16 compute path over device-resident bf16 rows (bit patterns, e.g. a
 * torch.bfloat16 tensor): d is the logical dimension; ldq / ldc >=
 * roundup(d, 128), multiples of 8, columns past d zero-filled, 16-byte-aligned
 * bases (any d and k: past the bf16 kernels' limits, the widened f32 path of
 * PMM_COMPUTE_BF16).  Scores are f32; k may exceed n as in
 * pmm_topk_f32_device. */
int pmm_topk_bf16_device(const uint16_t *q, int64_t ldq, int64_t m, const uint16_t *c,
                         int64_t ldc, int64_t n, int64_t d, int64_t k, int metric,
                         uint32_t index_base, uint32_t *out_idx, float *out_score,
                         void *workspace, size_t workspace_bytes, void *stream);

/* Row norms over device rows, the first stage of the metric pipeline:
 * replaces compute_norms_f32 / compute_squared_norms_f32
 * (src/metrics.rs:382-393; f64: compute_norms / compute_squared_norms,
 * :368-379).  out[r] = sqrt(row.row) (squared = 0, cosine) or row.row
 * (squared = 1, euclidean), accumulated in ndarray's unrolled_dot order
 * over exactly d elements with no FMA contraction -- the values the fused
 * top-k kernels use.  a has `rows` rows of stride ld elements (ld >= d). */
int pmm_norms_f32_device(const float *a, int64_t ld, int64_t rows, int64_t d, int squared,
                         float *out, void *stream);
int pmm_norms_f64_device(const double *a, int64_t ld, int64_t rows, int64_t d, int squared,
                         double *out, void *stream);

/* k-way merge of per-shard top-k lists: idx/score are [m][lists][k_in] (the
 * lists in any order; idx 0xFFFFFFFF marks an empty slot).  Writes the best k_out of each row to out_idx/out_score
 * [m][k_out].  This is the merge step after the RCCL gather of the
 * corpus-sharded path (no reference counterpart: the reference is
 * single-process). */
int pmm_merge_topk_device(const uint32_t *idx, const float *score, int64_t m, int64_t lists,
                          int64_t k_in, int64_t k_out, int metric, uint32_t *out_idx,
                          float *out_score, void *stream);

/* The same merge over any list layout: entry i of list s of row r is
 * idx[r * row_stride + s * list_stride + i] (and the same offset in score).
 * pmm_merge_topk_device is (lists * k_in, k_in).  The sharded path gathers
 * each rank's [idx plane | score plane] (2 x m x k_in 32-bit words) straight
 * into a [ranks][2][m][k_in] buffer with ONE collective and merges it in
 * place: idx = buffer, score = buffer + m * k_in, row_stride = k_in,
 * list_stride = 2 * m * k_in (no re-layout copy). */
int pmm_merge_topk_strided_device(const uint32_t *idx, const float *score, int64_t m,
                                  int64_t lists, int64_t k_in, int64_t row_stride,
                                  int64_t list_stride, int64_t k_out, int metric,
                                  uint32_t *out_idx, float *out_score, void *stream);

/* The same merge of lists that are each best-first under the total order
 * (score, then lower index; empty slots last) -- as every pmm_topk_* and merge
 * output is.  A row's answer is then a prefix of each list: the kernel reads
 * the first 256 / lists entries of each and reads on only for a row whose
 * prefixes cannot hold its k_out best (lists <= 64, k_out <= 256; otherwise
 * the general merge).  Unsorted input gives unspecified results.  The
 * sharded paths (in-process and RCCL) merge with this entry. */
int pmm_merge_sorted_topk_strided_device(const uint32_t *idx, const float *score, int64_t m,
                                         int64_t lists, int64_t k_in, int64_t row_stride,
                                         int64_t list_stride, int64_t k_out, int metric,
                                         uint32_t *out_idx, float *out_score, void *stream);

/* ---------------------------------------------------------------------------
 * Device-resident corpus: upload a corpus once and run many top-k calls
 * against it (Polars' map_batches may call `_topk` repeatedly with the same
 * corpus Series: python/polars_matmul/__init__.py:115-119).  The handle keeps
 * the padded rows in HBM and the norms of every metric (src/metrics.rs:368-393,
 * computed once at creation).  A handle may be used from several threads
 * concurrently; it is bound to the device current at creation, or sharded over
 * the device list (pmm_set_devices) in effect then.  Its row type is fixed at
 * creation: an f32 handle serves pmm_topk_f32_corpus (the reference's f32
 * branch, src/matmul.rs:429-448), an f64 handle pmm_topk_f64_corpus (the f64
 * branch, src/matmul.rs:449-468 -- what Polars' default Float64 columns take).
 * ------------------------------------------------------------------------- */
typedef struct pmm_corpus pmm_corpus;

#define PMM_DTYPE_F32 0
#define PMM_DTYPE_F64 1

int pmm_corpus_create_f32(const float *c, int64_t n, int64_t d, pmm_corpus **out);
/* An f64 corpus: rows kept in f64 (stride roundup(d, 16), zero-padded) with
 * their f64 norms of both metrics; with pmm_set_devices in effect, row-sharded
 * over the list like an f32 corpus (pmm_topk_f64_corpus merges the shards). */
int pmm_corpus_create_f64(const double *c, int64_t n, int64_t d, pmm_corpus **out);
/* PMM_DTYPE_F32 or PMM_DTYPE_F64. */
int pmm_corpus_dtype(const pmm_corpus *corpus, int *dtype);
int pmm_corpus_destroy(pmm_corpus *corpus);
int pmm_corpus_info(const pmm_corpus *corpus, int64_t *n, int64_t *d, int *device);
/* Number of device shards of a corpus handle (1, or the device list's length
 * capped at n when pmm_set_devices was in effect at creation). */
int pmm_corpus_shards(const pmm_corpus *corpus, int *shards);

/* pmm_topk_f32 against a device-resident corpus (host queries in, host
 * results out; 0 <= k <= n). */
int pmm_topk_f32_corpus(const pmm_corpus *corpus, const float *q, int64_t m, int64_t k,
                        int metric, uint32_t *out_idx, float *out_score);

/* pmm_topk_f64 against an f64 corpus handle (host queries in, host results
 * out; 0 <= k <= n; any k: the fused scan for k <= 1024 and a large score
 * matrix, else the materialised path, as pmm_topk_f64_device).  The results
 * equal pmm_topk_f64's bit for bit: the handle's norms are the ones every
 * call would compute, by the same kernel.  An f32 handle: PMM_ERR_ARG (and
 * pmm_topk_f32_corpus refuses an f64 handle the same way). */
int pmm_topk_f64_corpus(const pmm_corpus *corpus, const double *q, int64_t m, int64_t k,
                        int metric, uint32_t *out_idx, double *out_score);

/* Per-kernel timing on the launch stream (hipEvents around each launch).
 * enable=1 starts recording; pmm_timing_read returns the summed milliseconds
 * and launch count of kernels whose name contains `kernel` since the last
 * reset (it synchronises the recorded events). */
int pmm_timing_enable(int enable);
int pmm_timing_reset(void);
int pmm_timing_read(const char *kernel, double *total_ms, int64_t *launches);

#ifdef __cplusplus
}
#endif

#endif /* PMM_H_ */
