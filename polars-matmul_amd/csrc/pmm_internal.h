// pmm_internal.h -- launch-side interface between the host orchestration
// (pmm_capi.hip) and the gfx950 kernels (pmm_kernels.hip).  Not installed.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace pmm {

// Benchmarking-only phase removal (PMM_ABLATE / PMM_MERGE_ABLATE: results are
// wrong by design).  Compiled in only by the lab build (`make lab` ->
// libpmm_lab.so, -DPMM_LAB); in the shipped libpmm.so the variables are never
// read and every ablation branch folds away at compile time.
#ifdef PMM_LAB
#define PMM_ABL(x) (x)
#else
#define PMM_ABL(x) 0
#endif

constexpr int kMetricCosine = 0;
constexpr int kMetricDot = 1;
constexpr int kMetricEuclidean = 2;

// Fused top-k path limits.  k above kFusedMaxK goes through the materialise +
// row-select path (kernels below), which also serves f64.
constexpr int kFusedMaxK = 1024;
// Row-select (materialised scores) keeps up to kRowSelMaxP entries per row in
// LDS; larger k uses the full-row global sort.
constexpr int kRowSelMaxP = 4096;

// Arguments of the f32 MFMA GEMM kernel (top-k and store modes).
struct GemmF32Args {
  const float *q;       // M x ldq
  const float *c;       // N x ldc
  const uint16_t *qb;   // bf16 compute path: M x ldq bf16 (bit patterns)
  const uint16_t *cb;   // bf16 compute path: N x ldc bf16
  const float *qn;      // cosine: L2 norms of Q rows; euclidean: squared norms
  const float *cn;      // same for C rows
  const float *cpre;    // pre-filter column factor: cosine 1/||c|| (0 if zero-norm),
                        // euclidean ||c||^2 * (1 - 2^-18)
  int64_t ldq, ldc;
  int M, N, D;          // D % 32 == 0
  int k, capg;          // top-k and candidate-buffer capacity (power of two)
  int ctrig;            // compaction trigger: a row's buffer is compacted to its best k
                        // once it holds more than ctrig entries (k < ctrig <= capg - 64)
  int metric;
  int QB, S, tps, ntiles, units;  // work decomposition (see plan_units)
  unsigned *counter;              // work-queue head, zeroed per call
  unsigned long long *cand;       // [M*S][capg] candidate composites
  unsigned *cnt;                  // [M*S] candidate counts
  unsigned long long *gthr;       // [M] shared per-row threshold, zeroed per call
  unsigned long long *wq;         // per-wave survivor queue [grid][NW][32 * BN]
  int qcap;                       // f32 kernel: survivor-queue entries per wave in LDS
                                  // (set by launch_gemm_f32; past them, wq)
  float *out;                     // store mode: out[M][ldo]
  int64_t ldo;
  int store_metric;               // store mode: 1 = metric-transformed score, 0 = raw dot
  int ablate;                     // benchmarking only (PMM_ABLATE): 1 = skip the epilogue
  int nst;                        // bf16 kernel: LDS ring slots (3 or 4)
  int round_sync;                 // bf16 kernel: align workgroups at unit rounds (speed only)
  int sync_timeout;               // bf16 kernel: round-barrier spin limit (100 MHz ticks)
  int pf;                         // bf16 kernel: corpus-fragment prefetch depth (1 or 2 substeps)
  int defer;                      // bf16 kernel: hold each K-step's last MFMA group past the barrier
  int qb_full;                    // wave-specialised bf16 kernel: query blocks processed whole
                                  // (phase A; a multiple of the grid), the rest as split units
  unsigned long long *stats;      // PMM_STATS only: [queued, flagged groups, tiles, compactions]
  // fire-and-forget bf16 kernel (pmm_bf16_ff_kernel.h): per-(unit, wave)
  // survivor regions of ffcap items (raw dot | row << 58 | column << 32) and
  // their counts (a count above ffcap: the region overflowed)
  unsigned long long *ffreg;
  unsigned *ffcnt;
  int ffcap;
};

struct MergeArgs {
  // loader 0: candidate segments from the fused kernel
  const unsigned long long *cand;
  const unsigned *cnt;
  const unsigned long long *gthr;
  int capg;
  // loader 1: gathered (idx, score) lists; entry i of list s of row r is at
  // in_idx[r * row_stride + s * list_stride + i] (same offsets in in_score):
  // [M][S][k_in] is (S * k_in, k_in); the RCCL gather's [S][2][M][k_in]
  // (idx plane, score plane per rank) is (k_in, 2 * M * k_in)
  const uint32_t *in_idx;
  const float *in_score;
  int k_in;
  int64_t row_stride, list_stride;
  int M, S, k_out, P, metric;
  uint32_t index_base;
  uint32_t *out_idx;
  float *out_score;
  int ablate;  // benchmarking only (PMM_MERGE_ABLATE): 1 = no selection/sort, 2 = no candidate loads
  int no_rank;  // set by launch_merge: bitonic sort instead of rank counting (many rows)
  int flags;    // set by launch_merge: kMergeReverse, kMergePipelined, kMergeSplitRow
  int sorted;   // loader 1: every input list is best-first (the prefix fast path)
};
constexpr int kMergeReverse = 1;    // rows last to first (split rows, the heavy ones, start first)
constexpr int kMergePipelined = 2;  // next candidate batch's loads in flight while one is taken
constexpr int kMergeSplitRow = 4;   // a block of 4 waves per row, each merging a quarter of its lists

struct RowSelArgs {
  const void *scores;   // [rows][lds] f32 or f64, already metric-transformed
  int64_t lds;
  int rows, N, k, P, metric, is_f64;
  uint32_t index_base;  // added to every output index
  uint32_t *out_idx;    // [rows][k]
  void *out_score;      // [rows][k] f32 or f64
};

// ---- launchers (pmm_kernels.hip) ----
// (also zeroes zero_bytes at zero, a multiple of 16 at a 16-byte address)
hipError_t launch_norms_pair_f32(const float *q, int64_t m, int64_t ldq, float *qout, const float *c,
                                 int64_t n, int64_t ldc, float *cout, float *cinv, int64_t d, int squared,
                                 hipStream_t s, void *zero = nullptr, size_t zero_bytes = 0);
hipError_t launch_norms_f32(const float *a, int64_t rows, int64_t d, int64_t ld, int squared,
                            float *out, float *inv, hipStream_t s);
hipError_t launch_norms_f64(const double *a, int64_t rows, int64_t d, int64_t ld, int squared,
                            double *out, hipStream_t s);
// Tile-shape variant of the f32 GEMM (see pmm_kernels.hip): 0 = 128x128,
// 1 = 128x256, 2 = 256x128 (2 waves/SIMD), 3 = 256x256 (2 waves/SIMD),
// 4 = 128x64, 5 = 128x64 column-split (2 waves/SIMD, fused top-k only).
// mode 0 = fused top-k, 1 = store.  grid = number of persistent workgroups.
hipError_t launch_gemm_f32(const GemmF32Args &a, int variant, int mode, int grid, hipStream_t s);
int gemm_f32_bm(int variant);   // query rows per workgroup
int gemm_f32_bn(int variant);   // corpus columns per tile
int gemm_f32_nw(int variant);   // waves per workgroup
int gemm_f32_segs(int variant); // candidate segments per (row, corpus split): 2 for the column split
size_t gemm_f32_lds_bytes(int variant, int mode, int capg);
hipError_t launch_merge(const MergeArgs &a, int loader, hipStream_t s);
// Threshold seeding: gthr[row] = (k-th best composite of the row's ns
// materialised scores S[row][0..ns)) - 1, one wave per row; ns <= kSeedMaxNs.
constexpr int kSeedMaxNs = 1024;
// The fused top-k's prologue with threshold seeding in one launch: the seed
// (the sample's scores as fmaf chains, bit-identical to the fused kernel's,
// with its own norms; writes every row's gthr), the query norms (and the
// corpus norms when corpus_norms), and zeroing [z0, +z0_bytes) and [z1,
// +z1_bytes).  Padded dp <= kSeedDotsMaxD.
constexpr int kSeedDotsMaxD = 2048;
hipError_t launch_seeded_prologue(const float *q, int64_t ldq, int m, const float *c, int64_t ldc, int64_t n,
                                  int d, int dp, int ns, int k, int metric, float *qn, float *cn, bool corpus_norms,
                                  unsigned long long *gthr, void *z0, size_t z0_bytes, void *z1, size_t z1_bytes,
                                  hipStream_t s);
hipError_t launch_seed_select(const float *S, int64_t lds, int m, int ns, int k, int metric,
                              unsigned long long *gthr, hipStream_t s);
// ---- bf16 compute path (pmm_bf16.hip) ----
// Fused top-k on bf16 operands: 128 query rows x 128 corpus columns per
// workgroup tile, 4 waves (1 per SIMD), query rows register-resident.
constexpr int kBf16BM = 128, kBf16BN = 128, kBf16NW = 4;
constexpr int kBf16MaxD = 768;  // padded D (multiple of kBf16DAlign) limit: registers
constexpr int kBf16DAlign = 128;
constexpr int kBf16MaxCapg = 1024;  // LDS budget for the compaction scratch (k <= 960)
hipError_t launch_gemm_bf16(const GemmF32Args &a, int grid, hipStream_t s);
size_t gemm_bf16_lds_bytes(int capg, int nst);
// Wave-specialised bf16 kernel (pmm_bf16_ws_kernel.h): 128 query rows x 64
// corpus columns per tile, 4 MFMA waves + 4 epilogue waves.  Used when its
// LDS (compaction scratch included) fits: capg <= kBf16WsMaxCapg.
constexpr int kBf16WsBN = 64;
constexpr int kBf16WsMaxCapg = 512;
size_t gemm_bf16_ws_lds_bytes(int capg, int D);  // D = padded dimension
hipError_t launch_gemm_bf16_ws(const GemmF32Args &a, int grid, hipStream_t s);
// bf16 threshold seed (pmm_bf16_ws_kernel.h): S[row][0..ns) = the scores of
// corpus rows 0..ns-1 exactly as the wave-specialised kernel computes them
hipError_t launch_seed_bf16_ws(const GemmF32Args &a, float *S, int ns, hipStream_t s);
// 256-query-row bf16 kernel on v_mfma_f32_16x16x32_bf16 with survivors stored
// fire-and-forget against a static guessed threshold (pmm_bf16_ff_kernel.h):
// 64 rows x D per wave, 32-column corpus tiles.  N < 2^26.
constexpr int kBf16FfBM = 256, kBf16FfBN = 32;
size_t gemm_bf16_ff_lds_bytes(int D);  // D = padded dimension; 0 if unsupported
hipError_t launch_gemm_bf16_ff(const GemmF32Args &a, int grid, hipStream_t s);
// Exact re-score and bucketing of the ff kernel's survivor regions into the
// per-(row, split) candidate lists of merge_kernel: one workgroup per (query
// block, wave); rows whose lists overflowed, whose region overflowed or that
// kept fewer than k candidates at or above their threshold go to fb_rows
// (*fb_count of them) for a re-run.
hipError_t launch_ff_gather_rows(const uint16_t *q, int64_t ldq, const int *rows, int r, uint16_t *dst,
                                 hipStream_t s);
hipError_t launch_ff_scatter_lists(const uint32_t *oi, const float *os, const int *rows, int r, int k,
                                   uint32_t *out_idx, float *out_score, hipStream_t s);
hipError_t launch_ff_bucket(const GemmF32Args &a, unsigned *fb_count, int *fb_rows, hipStream_t s);
// f32 rows -> bf16 (round to nearest even) with row stride ldd, columns
// d..ldd-1 zero-filled.
hipError_t launch_f32_to_bf16(const float *src, int64_t rows, int64_t d, int64_t lds, uint16_t *dst,
                              int64_t ldd, hipStream_t s);
// bf16 rows -> f32 rows (exact), columns d..ldd-1 zero-filled
hipError_t launch_bf16_to_f32(const uint16_t *src, int64_t rows, int64_t d, int64_t lds, float *dst, int64_t ldd,
                              hipStream_t s);
hipError_t launch_norms_bf16(const uint16_t *a, int64_t rows, int64_t d, int64_t ld, int squared,
                             float *out, float *inv, hipStream_t s);
size_t merge_lds_bytes_per_wave(int P);
hipError_t launch_gemm_f64_store(const double *q, int64_t ldq, const double *c, int64_t ldc,
                                 const double *qn, const double *cn, int M, int N, int D,
                                 int metric, int store_metric, double *out, int64_t ldo,
                                 hipStream_t s);
hipError_t launch_rowselect(const RowSelArgs &a, hipStream_t s);
// ---- fused f64 top-k (pmm_f64.hip) ----
struct Ent;
struct F64TopkArgs {
  const double *q;           // this launch's rows (row stride ldq)
  const double *c;           // the whole corpus (row stride ldc)
  const double *qn, *cn;     // cosine: norms, euclidean: squared norms (qn: this launch's rows)
  int64_t ldq, ldc;
  int M, D;                  // rows; padded K (multiple of 16)
  int col0, ncol;            // corpus columns [col0, col0 + ncol) of this chunk
  int metric;
  const unsigned long long *tkey;  // [M] row threshold: the k-th entry (key, index); (0, ~0) = accept all
  const uint32_t *tidx;
  unsigned *cnt;             // [M] buffer counts
  Ent *cand;                 // [M][cap] candidate buffers
  int cap;
  int accept_all;            // first chunk (ncol <= cap): every element at slot = its chunk column
};
struct F64SelArgs {
  Ent *cand;
  unsigned *cnt;
  int cap, M, k, P;          // P: LDS entries per wave, a power of two >= cap
  int mode;                  // 0: keep the best k + raise the thresholds; 1: write the final lists
  unsigned long long *tkey;
  uint32_t *tidx;
  int metric;
  uint32_t index_base;
  uint32_t *out_idx;
  double *out_score;
  unsigned *overflow;        // set when a row's count exceeded cap (entries were dropped)
};
// k-way merge of G (<= 64) sorted f64 top-k lists per row: entry i of list g
// of row r at gi / gs[g * list_stride + r * k + i]
struct F64MergeArgs {
  const uint32_t *gi;
  const double *gs;
  int64_t list_stride;
  int M, G, k, metric;
  uint32_t *out_idx;    // [M][k]
  double *out_score;
};
hipError_t launch_f64_merge(const F64MergeArgs &a, hipStream_t s);
hipError_t launch_gemm_f64_topk(const F64TopkArgs &a, hipStream_t s);
hipError_t launch_f64_select(const F64SelArgs &a, hipStream_t s);
hipError_t launch_f64_reset(unsigned long long *tkey, uint32_t *tidx, unsigned *cnt, int m, unsigned cnt0,
                            hipStream_t s);
// full-row sort fallback for very large k
hipError_t launch_rowsort_global(const void *scores, int64_t lds, int rows, int N, int is_f64,
                                 int metric, void *keys_ws, int P2, int k, uint32_t index_base,
                                 uint32_t *out_idx,
                                 void *out_score, hipStream_t s);

}  // namespace pmm
