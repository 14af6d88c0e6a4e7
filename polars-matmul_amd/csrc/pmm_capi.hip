// pmm_capi.hip -- C ABI (include/pmm.h) and host orchestration.
//
// Host side of the hot path that the reference implements in
// src/matmul.rs:295-519 (dispatch, extraction, k clipping, error texts) and
// src/lib.rs:15-55 (the FFI boundary).  Here it owns: per-thread HIP stream
// and scratch arena, upload/padding of host inputs, the work decomposition of
// the fused kernel, and the launch sequence norms -> fused GEMM+top-k ->
// merge.  All device work of one call is enqueued on one stream; host calls
// synchronise that stream once at the end.
#include "pmm_internal.h"
#include "../../include/pmm.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

using namespace pmm;

namespace {

constexpr const char *kVersion = "0.1.4+mi355x.r1";
constexpr size_t kMaterialiseBudget = size_t(2) << 30;  // bytes of score chunk (f64/large-k/matmul)

thread_local std::string t_err;

int fail(int code, const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  t_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail(PMM_ERR_HIP, "HIP error %s at %s:%d (%s)", hipGetErrorString(e_),      \
                  __FILE__, __LINE__, #expr);                                           \
  } while (0)

struct DeviceInfo {
  bool probed = false;
  bool ok = false;
  int cus = 256;
  std::string arch;
};
constexpr int kMaxDevices = 64;
std::mutex g_dev_mu;
DeviceInfo g_dev[kMaxDevices];  // fixed storage: readers index it without the lock

// Corpus sharding over several devices for the host entry points
// (pmm_set_devices): process-wide, empty = one device.
std::mutex g_devs_mu;
std::vector<int> g_devs;

struct TimingRec {
  const char *name;
  hipEvent_t a, b;
  int dev;
};

// Per-thread, per-device scratch arena.  Host entry points use it on the
// thread's own stream and synchronise before returning; device entry points
// called with workspace = NULL use it on the CALLER's stream and return
// without synchronising.  `ev` is recorded behind the last device-API use, and
// a use on a different stream first waits for it, so two streams never work
// in the same bytes at once.
struct ArenaSlot {
  void *p = nullptr;
  size_t bytes = 0;
  hipEvent_t ev = nullptr;
  hipStream_t last = nullptr;
  bool used = false;
};

struct ThreadCtx {
  int device = -1;                   // pmm_set_device's choice for host calls (-1: current)
  std::vector<hipStream_t> streams;  // per device, created lazily, never destroyed
  std::vector<hipStream_t> copy_streams;  // per device: host uploads overlapped with compute
  std::vector<ArenaSlot> arena;      // per device
  bool timing = false;
  std::vector<TimingRec> recs;
  // events of read timing records, per device, reused (an event creation per
  // timed launch is host time comparable to a small problem's whole step)
  std::vector<std::vector<hipEvent_t>> free_events;
};
thread_local ThreadCtx t_ctx;

hipEvent_t timing_event(int dev) {
  if ((int)t_ctx.free_events.size() <= dev) t_ctx.free_events.resize(dev + 1);
  auto &v = t_ctx.free_events[dev];
  hipEvent_t e = nullptr;
  if (!v.empty()) {
    e = v.back();
    v.pop_back();
  } else {
    (void)hipEventCreate(&e);
  }
  return e;
}

// Restores the caller's current HIP device when a host entry point switched it.
struct DevScope {
  int prev = -1;
  ~DevScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// Probes device `dev` once (gfx950 or a PMM_ERR_NODEVICE failure).
int probe_device(int dev) {
  if (dev < 0 || dev >= kMaxDevices) return fail(PMM_ERR_NODEVICE, "HIP device %d out of range", dev);
  std::lock_guard<std::mutex> lk(g_dev_mu);
  DeviceInfo &di = g_dev[dev];
  if (!di.probed) {
    hipDeviceProp_t p;
    hipError_t e = hipGetDeviceProperties(&p, dev);
    if (e != hipSuccess) return fail(PMM_ERR_NODEVICE, "no HIP device %d: %s", dev, hipGetErrorString(e));
    di.probed = true;
    di.arch = p.gcnArchName;
    di.cus = p.multiProcessorCount > 0 ? p.multiProcessorCount : 256;
    di.ok = di.arch.rfind("gfx950", 0) == 0;
  }
  if (!di.ok)
    return fail(PMM_ERR_NODEVICE, "libpmm is built for gfx950 (MI355X); HIP device %d is %s", dev,
                di.arch.c_str());
  return PMM_OK;
}

// Device-pointer entry points (scope == NULL) run on the caller's current
// device and leave it alone.  Host entry points pass a scope: they run on
// `want` (a corpus handle's device), else on pmm_set_device's choice for this
// thread, else on the current device, and restore the current device on return.
int ensure_device(int *dev_out, DevScope *scope = nullptr, int want = -1) {
  int cur = 0;
  HIP_TRY(hipGetDevice(&cur));
  int dev = cur;
  if (scope) dev = want >= 0 ? want : (t_ctx.device >= 0 ? t_ctx.device : cur);
  if (int rc = probe_device(dev)) return rc;
  if (dev != cur) {
    HIP_TRY(hipSetDevice(dev));
    scope->prev = cur;
  }
  *dev_out = dev;
  return PMM_OK;
}

int thread_stream(int dev, hipStream_t *s, bool copy = false) {
  std::vector<hipStream_t> &v = copy ? t_ctx.copy_streams : t_ctx.streams;
  if ((int)v.size() <= dev) v.resize(dev + 1, nullptr);
  if (!v[dev]) HIP_TRY(hipStreamCreateWithFlags(&v[dev], hipStreamNonBlocking));
  *s = v[dev];
  return PMM_OK;
}

// Grow-only per-thread, per-device scratch (see ArenaSlot).  A use on another
// stream than the last device-API use waits for that use's event; growing
// waits for both, so in-flight work never sees its buffer freed.
int arena(int dev, hipStream_t s, size_t bytes, void **p) {
  if ((int)t_ctx.arena.size() <= dev) t_ctx.arena.resize(dev + 1);
  ArenaSlot &a = t_ctx.arena[dev];
  if (!a.ev) HIP_TRY(hipEventCreateWithFlags(&a.ev, hipEventDisableTiming));
  if (a.used && a.last != s) HIP_TRY(hipStreamWaitEvent(s, a.ev, 0));
  if (a.bytes < bytes) {
    if (a.p) {
      if (a.used) HIP_TRY(hipEventSynchronize(a.ev));
      HIP_TRY(hipStreamSynchronize(s));
      HIP_TRY(hipFree(a.p));
      a.p = nullptr;
      a.bytes = 0;
    }
    size_t want = bytes + bytes / 8;
    HIP_TRY(hipMalloc(&a.p, want));
    a.bytes = want;
  }
  *p = a.p;
  return PMM_OK;
}

// Marks the end of a device-API use of the arena on stream s (no host sync).
int arena_record(int dev, hipStream_t s) {
  ArenaSlot &a = t_ctx.arena[dev];
  HIP_TRY(hipEventRecord(a.ev, s));
  a.last = s;
  a.used = true;
  return PMM_OK;
}

size_t al256(size_t x) { return (x + 255) & ~size_t(255); }
int next_pow2(int x, int lo = 64) {
  int p = lo;
  while (p < x) p <<= 1;
  return p;
}
int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

struct Timed {
  hipStream_t s;
  TimingRec rec{};
  bool on;
  Timed(const char *name, hipStream_t st) : s(st), on(t_ctx.timing) {
    if (on) {
      rec.name = name;
      (void)hipGetDevice(&rec.dev);
      rec.a = timing_event(rec.dev);
      rec.b = timing_event(rec.dev);
      (void)hipEventRecord(rec.a, s);
    }
  }
  ~Timed() {
    if (on) {
      (void)hipEventRecord(rec.b, s);
      t_ctx.recs.push_back(rec);
    }
  }
};

// ---------------------------------------------------------------------------
// Work decomposition of the persistent GEMM: units = QB query blocks x S
// corpus splits of tps tiles.  Minimise rounds * (tps + overhead) over all tps
// so the last round of units fills the chip, subject to the candidate-buffer
// memory budget (M * S * capg * 8 bytes).
// ---------------------------------------------------------------------------
struct Plan {
  int variant = 0;
  int QB = 0, T = 0, tps = 0, S = 0, units = 0, grid = 0, capg = 0, P = 0, qb_full = 0;
  int ctrig = 0;  // compaction trigger (GemmF32Args::ctrig)
  int segs = 0;   // candidate segments per row (S, or 2 S for the column-split f32 variant)
  size_t off_counter = 0, off_gthr = 0, off_cnt = 0, off_cand = 0, off_qn = 0, off_cn = 0;
  size_t off_wq = 0;
  // fire-and-forget bf16 kernel (variant -6): guess sample size and rank,
  // region capacity; survivor counts, regions, the re-run row list
  int ff_ns = 0, ff_j = 0, ffcap = 0;
  size_t off_ffcnt = 0, off_ffreg = 0, off_fb = 0;
  size_t total = 0;
};
// set while a call re-runs the rows the fire-and-forget kernel could not
// prove exact (they go to the wave-specialised kernel)
thread_local bool t_no_ff = false;

void plan_units(int64_t m, int64_t n, int bm, int bn, int cus, double unit_overhead, int64_t max_S,
                Plan &p, bool whole_blocks = false) {
  p.QB = (int)cdiv(m, bm);
  p.T = (int)cdiv(n, bn);
  double best = 1e300;
  int best_tps = p.T;
  for (int tps = 1; tps <= p.T; tps++) {
    const int64_t S = cdiv(p.T, tps);
    if (S > max_S) continue;
    if (tps > 1 && cdiv(p.T, tps - 1) == S) continue;  // same S, fewer tiles: dominated
    const int64_t units = (int64_t)p.QB * S;
    // whole_blocks (wave-specialised bf16 kernel): floor(QB / grid) * grid
    // query blocks run whole, split by split, the rest as split units
    const int64_t grid = std::min<int64_t>(units, cus);
    const int64_t rounds = whole_blocks && p.QB >= grid
                               ? (p.QB / grid) * S + cdiv((p.QB % grid) * S, grid)
                               : cdiv(units, cus);
    const double cost = (double)rounds * (tps + unit_overhead) + 1e-4 * (double)S;
    if (cost < best) {
      best = cost;
      best_tps = tps;
    }
  }
  p.tps = best_tps;
  p.S = (int)cdiv(p.T, p.tps);
  p.units = p.QB * p.S;
  p.grid = (int)std::min<int64_t>(p.units, cus);
  p.qb_full = (whole_blocks && p.QB >= p.grid) ? (p.QB / p.grid) * p.grid : 0;
}

// Tile-shape variant: PMM_GEMM_VARIANT overrides; otherwise the preferred
// order below, skipping variants whose LDS (staging + per-wave scratch) does
// not fit in the CU's 160 KiB.
// Small problems (fewer than 4 x CUs 256 x 256 tiles: the reference's own
// 1000 x 10000 benchmark size) fill the chip better with 128 x 128 tiles.
int choose_variant(int mode, int capg, int64_t m = 1 << 30, int64_t n = 1 << 30, int cus = 256) {
  // (read per call, so a test can force each variant in turn)
  const char *ev = getenv("PMM_GEMM_VARIANT");
  const int env = ev ? atoi(ev) : -1;
  if (env >= 0 && env < 6 && (env != 5 || mode == 0) && gemm_f32_lds_bytes(env, mode, capg) <= 160 * 1024)
    return env;
  if (cdiv(m, 256) * cdiv(n, 256) < 4 * (int64_t)cus && gemm_f32_lds_bytes(0, mode, capg) <= 160 * 1024) {
    // 128 x 128 tiles, or for the fused top-k 128 x 64 (variant 4) when its
    // finer units give a shorter makespan: per unit, tps tiles of bn / 128
    // (128-column tile times, the thin tile's extra overhead at 12%) plus
    // half a tile of unit start.  c1: 3 tiles per unit on 216 CUs, or 5 thin
    // tiles on 256 -> fused kernel 82 -> 76 us, c2 80 -> 74-75
    // (profiles/r3_c1/variant4_ab.txt).
    if (mode == 0 && gemm_f32_lds_bytes(4, mode, capg) <= 160 * 1024) {
      auto makespan = [&](int v) {
        Plan q;
        plan_units(m, n, gemm_f32_bm(v), gemm_f32_bn(v), cus, 0.5, 1 << 20, q);
        const double tile = gemm_f32_bn(v) / 128.0 * (v == 4 ? 1.12 : 1.0);
        return (double)cdiv(q.units, cus) * (q.tps * tile + 0.5);
      };
      if (makespan(4) < makespan(0)) return 4;
    }
    return 0;
  }
  // measured on c3 (100k x 1M x 768 cosine k=100): v3 136.9, v2 133.1, v1 120.5 TFLOP/s
  static const int order[4] = {3, 2, 0, 1};
  for (int v : order)
    if (gemm_f32_lds_bytes(v, mode, capg) <= 160 * 1024) return v;
  return 0;
}

// bf16 kernel choice: the wave-specialised kernel (pmm_bf16_ws_kernel.h)
// whenever its LDS carve holds the compaction scratch (k <= 448);
// PMM_BF16_WS=0 forces the one-wave-per-SIMD kernel (pmm_bf16_kernel.h).
// Read per call, so tests can exercise both.
bool bf16_ws_enabled(int capg, int64_t d) {
  const char *e = getenv("PMM_BF16_WS");
  if (e && atoi(e) == 0) return false;
  const int dp = (int)(cdiv(d, kBf16DAlign) * kBf16DAlign);
  return capg <= kBf16WsMaxCapg && gemm_bf16_ws_lds_bytes(capg, dp) <= 160 * 1024;
}



// compute = PMM_COMPUTE_F32: the f32 kernel (variant chosen by LDS fit);
// PMM_COMPUTE_BF16: the wave-specialised bf16 kernel (variant -2, 128 x 64
// tiles, 8 waves) or the 4-wave one (variant -1, 128 x 128 tiles).
// Fire-and-forget 256-row bf16 kernel (pmm_bf16_ff_kernel.h): PMM_BF16_FF=1
// (read per call).  Needs a corpus long enough for its guessed threshold: a
// sample of ns_g <= n / 16 rows whose j-th best leaves about n j / ns_g >= 4 k
// scores per row, N < 2^26, and a padded D the kernel's registers hold.
int ff_guess_j() {
  const char *e = getenv("PMM_FF_J");
  return e ? std::max(1, atoi(e)) : 5;
}
int64_t ff_guess_ns(int64_t n) { return std::min<int64_t>(2048, (n / 16) / 32 * 32); }
// The kernel is not part of the product library (it measured slower than the
// wave-specialised kernel): it is compiled into
// libpmm_ff.so (`make ff`, -DPMM_WITH_FF), which the GPU tests load beside
// libpmm.so as the shipped kernel's bit-exact cross-check.
bool bf16_ff_enabled(int64_t k, int64_t n, int64_t d) {
#ifndef PMM_WITH_FF
  (void)k, (void)n, (void)d;
  return false;
#else
  const char *e = getenv("PMM_BF16_FF");
  const int mode = e ? atoi(e) : 0;  // 2 (tests): whenever the kernel can run, however bad the guess
  if (mode == 0) return false;
  const int dp = (int)(cdiv(d, kBf16DAlign) * kBf16DAlign);
  const int64_t ns = ff_guess_ns(n);
  const bool guess_ok = (double)n * ff_guess_j() / (double)ns >= 4.0 * (double)k;
  return ns >= 256 && ns >= ff_guess_j() && (guess_ok || mode == 2) && k + 64 <= 8192 && n < (1 << 26) &&
         gemm_bf16_ff_lds_bytes(dp) > 0 && gemm_bf16_ff_lds_bytes(dp) <= 160 * 1024;
#endif
}

int plan_topk(int64_t m, int64_t n, int64_t d, int64_t k, int metric, int cus, Plan &p,
              int compute = PMM_COMPUTE_F32) {
  // testing knob: plan for fewer workgroups (small problems then take the
  // whole-query-block schedule that only full-size runs reach otherwise);
  // read per call so a test can set and clear it
  if (const char *ce = getenv("PMM_CUS")) {
    const int c = atoi(ce);
    if (c > 0 && c < cus) cus = c;
  }
  // Candidate buffer capacity per (row, split): a compaction keeps k, so a
  // bigger buffer compacts less often but prunes with an older threshold.
  // With selection-based compaction (wave_kth_u64, capg <= 512) 1.5x the
  // power of two measured best (c4 155 -> 151 ms, c3 1082 -> 1077 ms);
  // beyond 512 the compaction sorts, which needs a power of two.
  p.capg = next_pow2((int)k + 64, 128);
  if (p.capg * 3 / 2 <= 512) p.capg = p.capg * 3 / 2;
  {
    // experiment knob: candidate buffer capacity (>= k + 64, multiple of 8)
    const int cap_env = getenv("PMM_CAPG") ? atoi(getenv("PMM_CAPG")) : 0;  // (per call)
    if (cap_env > 0 && k + 64 <= 512) p.capg = std::max<int>(((int)k + 64 + 7) / 8 * 8, std::min(cap_env, 512) / 8 * 8);
  }
  const bool bf16 = compute == PMM_COMPUTE_BF16;
  const bool ffk = bf16 && !t_no_ff && bf16_ff_enabled(k, n, d);
  const bool ws = bf16 && !ffk && bf16_ws_enabled(p.capg, d);
  // the wave-specialised kernel on 16x16x32: twice the power of two (512 at
  // k = 100) compacts less often; c4 alternated twice on one box: 131.0 /
  // 130.5 vs 132.0 / 131.5 ms per launch (256: 135.4 / 135.0;
  // profiles/r4_ws16/capg_ab.txt)
  if (ws && !getenv("PMM_CAPG") && 2 * next_pow2((int)k + 64, 128) <= kBf16WsMaxCapg &&
      bf16_ws_enabled(2 * next_pow2((int)k + 64, 128), d))
    p.capg = 2 * next_pow2((int)k + 64, 128);
  p.variant = bf16 ? (ffk ? -6 : ws ? -2 : -1) : choose_variant(0, p.capg, m, n, cus);
  const int bm = bf16 ? (ffk ? kBf16FfBM : kBf16BM) : gemm_f32_bm(p.variant);
  const int bn = bf16 ? (ffk ? kBf16FfBN : ws ? kBf16WsBN : kBf16BN) : gemm_f32_bn(p.variant);
  const size_t per_S = (size_t)m * p.capg * 8 + (size_t)m * 4;
  const size_t cand_budget = size_t(8) << 30;
  int64_t max_S = std::max<int64_t>(1, (int64_t)(cand_budget / std::max<size_t>(per_S, 1)));
  // a bf16 unit starts by loading its 128 query rows into registers (about
  // two tiles' worth of time): longer splits amortise it
  // Wave-specialised kernel: floor(QB / grid) * grid query blocks run whole
  // (one workgroup carries a block's row state across all splits: 46% fewer
  // survivors at c4), the rest as split units.  Measured 9% slower with the
  // LDS-sort compaction (the longer-lived buffers compact twice as often);
  // with selection-based compaction 2% faster at c4 (149.5 -> 146.8 ms) and
  // the merge reads one segment per row.  PMM_BF16_WHOLE=0: split units only.
  const char *we = getenv("PMM_BF16_WHOLE");
  const char *fe = getenv("PMM_F32_WHOLE");
  // f32 kernel: the same split of units (PMM_F32_WHOLE=0: split units only).
  // At c3 the GEMM time is unchanged (1076 ms either way) and the merge reads
  // 0.89 GB instead of 2.17 GB (0.40 vs 0.65 ms).
  const bool whole = bf16 ? (ws && !ffk && !(we && atoi(we) == 0)) : !(fe && atoi(fe) == 0);
  // unit overhead in tiles: loading the unit's query rows into registers
  // (Two 128 x 128 f32 workgroups per CU -- 196 registers and 74 KiB of LDS
  // let them co-reside -- planned for 512 slots measured slower at c1: 0.129
  // vs 0.118 ms, profiles/r3_c1/wpc_variant_ab.txt.)
  plan_units(m, n, bm, bn, cus, bf16 ? (ffk ? 8.0 : ws ? 4.0 : 2.0) : 0.5, max_S, p, whole);
  if (ffk) {
    // expected survivors of the guessed threshold per row, n j / ns, and per
    // (row, split); a row's count varies with the sample's j-th (a Gamma(j)
    // quantile: 3x the mean is rare), a region's (64 rows) much less
    p.ff_ns = (int)ff_guess_ns(n);
    p.ff_j = ff_guess_j();
    const double e_row = (double)n * p.ff_j / p.ff_ns;
    const double e_rs = e_row * std::min<double>(1.0, (double)p.tps * bn / (double)n);
    p.capg = (int)std::max<int64_t>(k + 64, ((int64_t)(3.0 * e_rs) + 64 + 63) / 64 * 64);
    // (the seed's sample of ns scores per row lives in the candidate lists)
    p.capg = (int)std::max<int64_t>(p.capg, cdiv((int64_t)p.ff_ns, 2 * p.S));
    p.ffcap = (int)(((int64_t)(1.5 * 64.0 * e_rs) + 256 + 63) / 64 * 64);
    if (const char *ce = getenv("PMM_FF_CAP")) p.ffcap = std::max(64, atoi(ce));  // (tests: force overflows)
  }
  // Compaction trigger: a row's buffer is compacted (its k-th selected, the
  // row threshold raised to it) once it holds more than ctrig entries.  A
  // drain round adds at most 64 per row, so ctrig <= capg - 64.
  p.ctrig = p.capg - 64;
  if (const char *te = getenv("PMM_CTRIG")) {  // (experiment knob, per call)
    const int t = atoi(te);
    if (t > 0) p.ctrig = std::max<int>((int)k + 8, std::min(t, p.capg - 64));
  }
  // merge_kernel's per-row LDS capacity: at least 512, so a row's candidate
  // lists rarely need a compaction before the final one (c1: ~400 survivors
  // of the seed threshold per row; P = 128 compacted ~6 times, 23 us)
  p.P = std::min(8192, std::max(512, next_pow2(2 * (int)k + 64, 128)));
  size_t off = 0;
  p.off_counter = off;
  off += 256;
  p.off_gthr = off;
  off = al256(off + (size_t)m * 8);
  p.segs = p.S * (bf16 ? 1 : gemm_f32_segs(p.variant));
  p.off_cnt = off;
  off = al256(off + (size_t)m * p.segs * 4);
  p.off_cand = off;
  off = al256(off + (size_t)m * p.segs * p.capg * 8);
  p.off_qn = off;  // [norms m | inverse norms m]
  off = al256(off + (metric != kMetricDot ? (size_t)m * 8 : 0));
  p.off_cn = off;  // [norms n | inverse norms n]
  off = al256(off + (metric != kMetricDot ? (size_t)n * 8 : 0));
  p.off_wq = off;  // f32 kernel: per-wave survivor queues, grid x waves x (32 x BN) u64
  off = al256(off + (bf16 ? 0 : (size_t)p.grid * gemm_f32_nw(p.variant) * 32 * bn * 8));
  if (ffk) {
    p.off_ffcnt = off;  // [units][4 waves]
    off = al256(off + (size_t)p.units * 4 * 4);
    p.off_ffreg = off;  // [units][4 waves][ffcap]
    off = al256(off + (size_t)p.units * 4 * p.ffcap * 8);
    p.off_fb = off;  // [count | rows m]
    off = al256(off + 16 + (size_t)m * 4);
  }
  p.total = off;
  (void)d;
  return PMM_OK;
}

// Materialised path (k > kFusedMaxK, f32): rows per chunk and workspace.
struct MatPlan {
  int64_t rows = 0;
  int P = 0, P2 = 0;
  bool global_sort = false;
  size_t off_counter = 0, off_qn = 0, off_cn = 0, off_scores = 0, off_keys = 0, total = 0;
};

void plan_materialise(int64_t m, int64_t n, int64_t k, size_t elem, MatPlan &p) {
  p.P = next_pow2(2 * (int)std::min<int64_t>(k, 1 << 20) + 64, 128);
  p.global_sort = (k > (kRowSelMaxP - 64) / 2) || p.P > kRowSelMaxP;
  p.P2 = p.global_sort ? next_pow2((int)n, 2) : 0;
  size_t per_row = (size_t)n * elem + (p.global_sort ? (size_t)p.P2 * 16 : 0);
  p.rows = std::max<int64_t>(1, std::min<int64_t>(m, (int64_t)(kMaterialiseBudget / per_row)));
  size_t off = 0;
  p.off_counter = off;
  off += 256;
  p.off_qn = off;
  off = al256(off + (size_t)m * elem);
  p.off_cn = off;
  off = al256(off + (size_t)n * elem);
  p.off_scores = off;
  off = al256(off + (size_t)p.rows * n * elem);
  p.off_keys = off;
  off = al256(off + (p.global_sort ? (size_t)p.rows * p.P2 * 16 : 0));
  p.total = off;
}

// Page-locks a caller's host output buffer for the duration of a call so the
// D2H copy of an m x n result runs at full link rate instead of through the
// runtime's pageable staging (PMM_PIN_OUTPUT=0 disables; a failed
// registration just leaves the copy pageable).
struct HostPin {
  void *p = nullptr;
  HostPin(void *ptr, size_t bytes) {
    static const bool on = !(getenv("PMM_PIN_OUTPUT") && atoi(getenv("PMM_PIN_OUTPUT")) == 0);
    // already page-locked (pmm_host_alloc's buffers, or the caller's): nothing to do
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, ptr) == hipSuccess && at.type == hipMemoryTypeHost) return;
    (void)hipGetLastError();
    if (on && bytes >= (size_t(8) << 20) && hipHostRegister(ptr, bytes, hipHostRegisterDefault) == hipSuccess)
      p = ptr;
    else
      (void)hipGetLastError();
  }
  ~HostPin() {
    if (p) (void)hipHostUnregister(p);
  }
};

int check_metric(int metric) {
  if (metric != kMetricCosine && metric != kMetricDot && metric != kMetricEuclidean)
    return fail(PMM_ERR_ARG, "invalid metric id %d", metric);
  return PMM_OK;
}

// Store-mode GEMM over rows [0, rows) of q into out (ldo), raw or transformed.
// counter_zeroed: the caller's fill already zeroed *counter (no extra launch).
int gemm_store_f32(const float *q, int64_t ldq, int64_t rows, const float *c, int64_t ldc, int64_t n,
                   int64_t d, int metric, int store_metric, const float *qn, const float *cn,
                   float *out, int64_t ldo, unsigned *counter, int cus, hipStream_t s,
                   const char *label = nullptr, bool counter_zeroed = false) {
  Plan p;
  p.variant = choose_variant(1, 0, rows, n, cus);
  plan_units(rows, n, gemm_f32_bm(p.variant), gemm_f32_bn(p.variant), cus, 0.1, 1 << 20, p);
  GemmF32Args a{};
  a.q = q;
  a.c = c;
  a.qn = qn;
  a.cn = cn;
  a.ldq = ldq;
  a.ldc = ldc;
  a.M = (int)rows;
  a.N = (int)n;
  a.D = (int)d;
  a.k = 0;
  a.capg = 0;
  a.metric = metric;
  a.QB = p.QB;
  a.S = p.S;
  a.tps = p.tps;
  a.ntiles = p.T;
  a.units = p.units;
  a.counter = counter;
  a.out = out;
  a.ldo = ldo;
  a.store_metric = store_metric;
  if (!counter_zeroed) HIP_TRY(hipMemsetAsync(counter, 0, 4, s));
  Timed t(label ? label : (store_metric ? "gemm_f32_scores" : "gemm_f32_matmul"), s);
  HIP_TRY(launch_gemm_f32(a, p.variant, 1, p.grid, s));
  return PMM_OK;
}

// One fused top-k pass (gemm_f32_kernel + merge_kernel) over a planned
// workspace whose work counter and shared thresholds are already set.
struct FusedF32 {
  const float *q;
  int64_t ldq, m;
  const float *c;
  int64_t ldc, n, dp, k;
  int metric;
  const float *qn, *cn, *cpre;
};
hipError_t run_fused_f32(const FusedF32 &f, const Plan &p, char *w, uint32_t index_base,
                         uint32_t *out_idx, float *out_score, const char *gemm_label,
                         const char *merge_label, hipStream_t s) {
  // whole query blocks first (see gemm_f32_kernel's unit decode)
  const int64_t units = p.qb_full ? p.qb_full + (int64_t)(p.QB - p.qb_full) * p.S : p.units;
  // the caller has zeroed [w, w + p.off_cand): counter, thresholds, counts
  GemmF32Args a{};
  a.q = f.q;
  a.c = f.c;
  a.qn = f.qn;
  a.cn = f.cn;
  a.cpre = f.cpre;
  a.ldq = f.ldq;
  a.ldc = f.ldc;
  a.M = (int)f.m;
  a.N = (int)f.n;
  a.D = (int)f.dp;
  a.k = (int)f.k;
  a.capg = p.capg;
  a.ctrig = p.ctrig;
  a.metric = f.metric;
  a.QB = p.QB;
  a.tps = p.tps;
  a.ntiles = p.T;
  a.units = (int)units;
  a.qb_full = p.qb_full;
  a.S = p.segs;  // (the kernel indexes candidate segments with it)
  a.counter = (unsigned *)(w + p.off_counter);
#ifdef PMM_LAB
  {
    static const int ablate = getenv("PMM_ABLATE") ? atoi(getenv("PMM_ABLATE")) : 0;
    a.ablate = ablate;
  }
#endif
  a.cand = (unsigned long long *)(w + p.off_cand);
  a.wq = (unsigned long long *)(w + p.off_wq);
  a.cnt = (unsigned *)(w + p.off_cnt);
  a.gthr = (unsigned long long *)(w + p.off_gthr);
#ifdef PMM_LAB
  // per-phase cycle counters of the f32 kernel (make lab LAB=-DPMM_F32_STATS,
  // PMM_STATS=1): summed over waves, printed per call
  static const bool f32_stats = getenv("PMM_STATS") != nullptr;
  static unsigned long long *f32_stats_buf = nullptr;
  if (f32_stats) {
    if (!f32_stats_buf) {
      hipError_t e = hipMalloc(&f32_stats_buf, 128);
      if (e != hipSuccess) return e;
    }
    hipError_t e = hipMemsetAsync(f32_stats_buf, 0, 128, s);
    if (e != hipSuccess) return e;
    a.stats = f32_stats_buf;
  }
#endif
  {
    Timed t(gemm_label, s);
    hipError_t e = launch_gemm_f32(a, p.variant, 0, p.grid, s);
    if (e != hipSuccess) return e;
  }
#ifdef PMM_LAB
  if (f32_stats) {
    unsigned long long h[16];
    hipError_t e = hipMemcpyAsync(h, f32_stats_buf, 128, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    fprintf(stderr,
            "[pmm stats] gemm_f32 variant %d: units %d, S %d, tps %d, grid %d; wave cycles (sum): total %.4g, "
            "unit setup %.4g, K loops %.4g (barriers %.4g), epilogues %.4g (pre-filter + queueing %.4g, "
            "compactions %.4g; CNL flags + prefix sum %.4g); wave-tiles %llu, queued survivors %llu\n",
            p.variant, p.units, p.S, p.tps, p.grid, (double)h[0], (double)h[4], (double)h[2], (double)h[1],
            (double)h[3], (double)h[6], (double)h[7], (double)h[9], h[5], h[8]);
    a.stats = nullptr;
  }
#endif
  MergeArgs ma{};
  ma.cand = a.cand;
  ma.cnt = a.cnt;
  ma.gthr = a.gthr;
  ma.capg = p.capg;
  ma.M = (int)f.m;
  ma.S = p.segs;
  ma.k_out = (int)f.k;
  ma.P = p.P;
  ma.metric = f.metric;
  ma.index_base = index_base;
  ma.out_idx = out_idx;
  ma.out_score = out_score;
#ifdef PMM_LAB
  {
    static const int ablate = getenv("PMM_MERGE_ABLATE") ? atoi(getenv("PMM_MERGE_ABLATE")) : 0;
    ma.ablate = ablate;
  }
#endif
  Timed t(merge_label, s);
  return launch_merge(ma, 0, s);
}

// c_norms: optional precomputed corpus norms for `metric` laid out as
// [n norms | n pre-filter factors] (a pmm_corpus handle's cache); NULL =
// compute them in this call.
// keep_gthr: the workspace's shared per-row thresholds already hold a lower
// bound of the rows' k-th best from earlier corpus chunks (see
// topk_f32_host_chunked); they are kept instead of zeroed, so this chunk
// only returns what can still enter the top-k (possibly fewer than k per row:
// the rest are empty slots, which the chunk merge skips).
int topk_f32_device_impl(const float *q, int64_t ldq, int64_t m, const float *c, int64_t ldc,
                         int64_t n, int64_t d, int64_t k, int metric, uint32_t index_base,
                         uint32_t *out_idx, float *out_score, void *ws, size_t ws_bytes,
                         hipStream_t s, int dev, const float *c_norms = nullptr,
                         bool keep_gthr = false) {
  // d is the logical dimension (norms follow ndarray's order over exactly d
  // elements); the GEMM runs over dp = roundup(d, 32), the rows being
  // zero-padded up to dp.
  const int cus = g_dev[dev].cus;
  const int64_t dp = cdiv(d, 32) * 32;
  if (k <= kFusedMaxK) {
    Plan p;
    plan_topk(m, n, dp, k, metric, cus, p);
    const bool own = !ws;
    if (!ws) {
      int rc = arena(dev, s, p.total, &ws);
      if (rc) return rc;
    } else if (ws_bytes < p.total) {
      return fail(PMM_ERR_ARG, "workspace too small: %zu < %zu bytes", ws_bytes, p.total);
    }
    char *w = (char *)ws;
    float *qn = (float *)(w + p.off_qn), *cn = (float *)(w + p.off_cn);
    if (c_norms) cn = const_cast<float *>(c_norms);
    // Threshold seeding.  When every unit spans few corpus tiles (small
    // problems: the reference's own benchmark size), a unit starts cold: its
    // first tile's scores nearly all survive the pre-filter and are re-scored
    // exactly, appended and compacted, which took most of the kernel's time.
    // Instead, the scores of the first ns corpus rows are computed first --
    // by seed_dots_kernel as fmaf chains in natural K order (bit-identical to
    // the main pass's MFMA chain and epilogue arithmetic), or, past its
    // limits or with PMM_SEED_GEMM=1, by the MFMA main loop in store mode into
    // the still unused candidate buffers -- and one wave per row selects the
    // k-th best composite of that sample: (that key - 1) is an exact lower
    // bound of the row's final k-th best and seeds the shared threshold.
    // Sample size max(256, 8k): at c1 128 / 256 / 512 / 1024 rows measured
    // 0.170 / 0.163 / 0.174 / 0.192 ms per call (tools/experiments/gpu_seedns.sh).
    int64_t ns = std::min<int64_t>(n, next_pow2((int)std::max<int64_t>(256, 8 * k), 256));
    if (const char *ne = getenv("PMM_SEED_NS")) ns = std::min<int64_t>(n, std::max<int64_t>(atoll(ne), k));
    const char *se = getenv("PMM_SEED");
    // (only when most query blocks run as split units: a block run whole
    // carries its threshold across the corpus and gains nothing from the
    // seed, which costs m * ns * d fmaf on the vector units -- at a c3 shard
    // of 8, 100k x 125k x 768 with 256 of 391 blocks whole, 9.3 ms for no
    // GEMM time saved; tools/experiments/shard_shapes.py, profiles/r4_shards/)
    const bool mostly_split = 2 * (int64_t)p.qb_full < (int64_t)p.QB;
    bool seed = (se ? atoi(se) != 0
                    : ((int64_t)p.tps * gemm_f32_bn(p.variant) < 8192 && n >= 4 * ns && mostly_split)) &&
                ns >= k && ns < n && ns <= kSeedMaxNs && !keep_gthr &&
                (size_t)m * ns * 4 <= p.off_qn - p.off_cand;
    FusedF32 f{q, ldq, m, c, ldc, n, dp, k, metric, qn, cn, cn + n};
    // Seeded small problems: one prologue launch (seed + norms + fills).
    const bool one_prologue = seed && dp <= kSeedDotsMaxD && ldq % 4 == 0 && ldc % 4 == 0 &&
                              !(((uintptr_t)q | (uintptr_t)c | (uintptr_t)w) & 15) && p.off_gthr % 16 == 0 &&
                              p.off_cnt % 16 == 0 && p.off_cand % 16 == 0 && !getenv("PMM_SEED_GEMM");
    if (one_prologue) {
      Timed t("gemm_f32_seed", s);
      HIP_TRY(launch_seeded_prologue(q, ldq, (int)m, c, ldc, n, (int)d, (int)dp, (int)ns, (int)k, metric, qn, cn,
                                     !c_norms, (unsigned long long *)(w + p.off_gthr), w, p.off_gthr,
                                     w + p.off_cnt, p.off_cand - p.off_cnt, s));
    } else {
      // one fill zeroes the work counters (the main pass's and the seed store
      // pass's), thresholds and buffer counts [0, off_cand); with the norms
      // pair kernel the fill rides in the same launch
      const bool fill_in_norms =
          metric != kMetricDot && !c_norms && !keep_gthr && p.off_cand % 16 == 0 && ((uintptr_t)w & 15) == 0;
      if (keep_gthr) {
        HIP_TRY(hipMemsetAsync(w + p.off_counter, 0, p.off_gthr - p.off_counter, s));
        HIP_TRY(hipMemsetAsync(w + p.off_cnt, 0, p.off_cand - p.off_cnt, s));
      } else if (!fill_in_norms) {
        HIP_TRY(hipMemsetAsync(w, 0, p.off_cand, s));
      }
      if (metric != kMetricDot) {
        const int sq = metric == kMetricEuclidean;
        Timed t("norms_f32", s);
        if (c_norms) HIP_TRY(launch_norms_f32(q, m, d, ldq, sq, qn, nullptr, s));
        else HIP_TRY(launch_norms_pair_f32(q, m, ldq, qn, c, n, ldc, cn, cn + n, d, sq, s,
                                           fill_in_norms ? w : nullptr, fill_in_norms ? p.off_cand : 0));
      }
      if (seed) {
        // PMM_SEED_GEMM=1 or outside the one-launch limits: the sample's
        // scores from the fused kernel's main loop in store mode, then a
        // select launch
        float *sample = (float *)(w + p.off_cand);
        int rc = gemm_store_f32(q, ldq, m, c, ldc, ns, dp, metric, 1, qn, cn, sample, ns,
                                (unsigned *)(w + p.off_counter) + 16, cus, s, "gemm_f32_seed", true);
        if (rc) return rc;
        Timed t("seed_select", s);
        HIP_TRY(launch_seed_select(sample, ns, (int)m, (int)ns, (int)k, metric,
                                   (unsigned long long *)(w + p.off_gthr), s));
      }
    }
    HIP_TRY(run_fused_f32(f, p, w, index_base, out_idx, out_score, "gemm_f32_topk", "merge_topk", s));
    return own ? arena_record(dev, s) : PMM_OK;
  }
  // k beyond the fused path: materialise score chunks, row-select them.
  MatPlan p;
  plan_materialise(m, n, k, 4, p);
  const bool own = !ws;
  if (!ws) {
    int rc = arena(dev, s, p.total, &ws);
    if (rc) return rc;
  } else if (ws_bytes < p.total) {
    return fail(PMM_ERR_ARG, "workspace too small: %zu < %zu bytes", ws_bytes, p.total);
  }
  char *w = (char *)ws;
  float *qn = (float *)(w + p.off_qn), *cn = (float *)(w + p.off_cn);
  float *sc = (float *)(w + p.off_scores);
  if (c_norms) cn = const_cast<float *>(c_norms);
  if (metric != kMetricDot) {
    const int sq = metric == kMetricEuclidean;
    HIP_TRY(launch_norms_f32(q, m, d, ldq, sq, qn, nullptr, s));
    if (!c_norms) HIP_TRY(launch_norms_f32(c, n, d, ldc, sq, cn, nullptr, s));
  }
  for (int64_t r0 = 0; r0 < m; r0 += p.rows) {
    const int64_t rows = std::min<int64_t>(p.rows, m - r0);
    int rc = gemm_store_f32(q + r0 * ldq, ldq, rows, c, ldc, n, dp, metric, 1, qn + r0, cn, sc, n,
                            (unsigned *)(w + p.off_counter), cus, s);
    if (rc) return rc;
    if (!p.global_sort) {
      RowSelArgs ra{};
      ra.scores = sc;
      ra.lds = n;
      ra.rows = (int)rows;
      ra.N = (int)n;
      ra.k = (int)k;
      ra.P = p.P;
      ra.metric = metric;
      ra.is_f64 = 0;
      ra.index_base = index_base;
      ra.out_idx = out_idx + r0 * k;
      ra.out_score = out_score + r0 * k;
      HIP_TRY(launch_rowselect(ra, s));
    } else {
      HIP_TRY(launch_rowsort_global(sc, n, (int)rows, (int)n, 0, metric, w + p.off_keys, p.P2,
                                    (int)k, index_base, out_idx + r0 * k, out_score + r0 * k, s));
    }
  }
  return own ? arena_record(dev, s) : PMM_OK;
}

// bf16 compute path over device bf16 rows (row strides ldq / ldc >=
// roundup(d, 128), zero-padded); d is the logical dimension.
//
// The bf16 MFMA kernels hold a wave's 32 query rows x padded D in registers
// (D <= 768), their candidate buffers take k <= 960 and pack the column into
// 27 bits.  Outside that (configs[4]'s D = 1024, larger k, n >= 2^27) the
// bf16 operands are widened to f32 -- exactly: a bf16 value is an f32 with
// its low 16 bits zero -- and searched by the f32 path.  The result is the
// exact top-k of the bf16-rounded rows with f32 products and a k-ordered f32
// sum (the f32 path's bit-exact chain), so it meets the bf16 bar; the f32
// MFMA runs at 1/16 of the bf16 rate, which the bench line of such a shape
// states.
bool bf16_native(int64_t d, int64_t k, int64_t n) {
  return cdiv(d, kBf16DAlign) * kBf16DAlign <= kBf16MaxD && n < (int64_t(1) << 27) &&
         next_pow2((int)std::min<int64_t>(k, 1 << 20) + 64, 128) <= kBf16MaxCapg;
}

size_t f32_topk_ws_bytes(int64_t m, int64_t n, int64_t dp, int64_t k, int metric, int cus) {
  if (k <= kFusedMaxK) {
    Plan p;
    plan_topk(m, n, dp, k, metric, cus, p);
    return p.total;
  }
  MatPlan p;
  plan_materialise(m, n, k, 4, p);
  return p.total;
}

// workspace of the widened path: the f32 rows, then the f32 search's own
size_t bf16_widened_bytes(int64_t m, int64_t n, int64_t d, int64_t k, int metric, int cus) {
  const int64_t dp = cdiv(d, 32) * 32;
  return al256((size_t)m * dp * 4) + al256((size_t)n * dp * 4) + f32_topk_ws_bytes(m, n, dp, k, metric, cus);
}

int ff_rerun(const uint16_t *q, int64_t ldq, int64_t m, const uint16_t *c, int64_t ldc, int64_t n, int64_t d,
             int64_t k, int metric, uint32_t index_base, uint32_t *out_idx, float *out_score, const unsigned *fb,
             hipStream_t s, int dev);

int topk_bf16_device_impl(const uint16_t *q, int64_t ldq, int64_t m, const uint16_t *c,
                          int64_t ldc, int64_t n, int64_t d, int64_t k, int metric,
                          uint32_t index_base, uint32_t *out_idx, float *out_score, void *ws,
                          size_t ws_bytes, hipStream_t s, int dev) {
  const int cus = g_dev[dev].cus;
  if (!bf16_native(d, k, n)) {
    // widened to f32 and searched by the f32 path (see bf16_native)
    const int64_t dp32 = cdiv(d, 32) * 32;
    const size_t oc = al256((size_t)m * dp32 * 4), ow = oc + al256((size_t)n * dp32 * 4);
    const size_t wsf = f32_topk_ws_bytes(m, n, dp32, k, metric, cus);
    const bool own = !ws;
    if (!ws) {
      int rc = arena(dev, s, ow + wsf, &ws);
      if (rc) return rc;
    } else if (ws_bytes < ow + wsf) {
      return fail(PMM_ERR_ARG, "workspace too small: %zu < %zu bytes", ws_bytes, ow + wsf);
    }
    char *w = (char *)ws;
    {
      Timed t("bf16_widen", s);
      HIP_TRY(launch_bf16_to_f32(q, m, d, ldq, (float *)w, dp32, s));
      HIP_TRY(launch_bf16_to_f32(c, n, d, ldc, (float *)(w + oc), dp32, s));
    }
    int rc = topk_f32_device_impl((const float *)w, dp32, m, (const float *)(w + oc), dp32, n, d, k, metric,
                                  index_base, out_idx, out_score, w + ow, wsf, s, dev);
    if (rc) return rc;
    return own ? arena_record(dev, s) : PMM_OK;
  }
  const int64_t dp = cdiv(d, kBf16DAlign) * kBf16DAlign;
  Plan p;
  plan_topk(m, n, dp, k, metric, cus, p, PMM_COMPUTE_BF16);
  const bool own = !ws;
  if (!ws) {
    int rc = arena(dev, s, p.total, &ws);
    if (rc) return rc;
  } else if (ws_bytes < p.total) {
    return fail(PMM_ERR_ARG, "workspace too small: %zu < %zu bytes", ws_bytes, p.total);
  }
  char *w = (char *)ws;
  float *qn = (float *)(w + p.off_qn), *cn = (float *)(w + p.off_cn);
  HIP_TRY(hipMemsetAsync(w, 0, p.off_gthr + (size_t)m * 8, s));
  if (p.qb_full) HIP_TRY(hipMemsetAsync(w + p.off_cnt, 0, (size_t)m * p.S * 4, s));
  if (metric != kMetricDot) {
    const int sq = metric == kMetricEuclidean;
    Timed t("norms_bf16", s);
    HIP_TRY(launch_norms_bf16(q, m, d, ldq, sq, qn, nullptr, s));
    HIP_TRY(launch_norms_bf16(c, n, d, ldc, sq, cn, cn + n, s));
  }
  GemmF32Args a{};
  a.qb = q;
  a.cb = c;
  a.qn = qn;
  a.cn = cn;
  a.cpre = cn + n;
  a.ldq = ldq;
  a.ldc = ldc;
  a.M = (int)m;
  a.N = (int)n;
  a.D = (int)dp;
  a.k = (int)k;
  a.capg = p.capg;
  a.ctrig = p.ctrig;
  a.metric = metric;
  a.QB = p.QB;
  a.S = p.S;
  a.tps = p.tps;
  a.ntiles = p.T;
  a.units = p.units;
  a.counter = (unsigned *)(w + p.off_counter);
#ifdef PMM_LAB
  {
    static const int ablate = getenv("PMM_ABLATE") ? atoi(getenv("PMM_ABLATE")) : 0;
    a.ablate = ablate;
  }
#endif
  a.cand = (unsigned long long *)(w + p.off_cand);
  a.wq = (unsigned long long *)(w + p.off_wq);
  a.cnt = (unsigned *)(w + p.off_cnt);
  a.gthr = (unsigned long long *)(w + p.off_gthr);
  {
    a.nst = 3;  // LDS ring slots of the bf16 kernel
    a.pf = 1;
    static const int defer_env = getenv("PMM_BF16_DEFER") ? atoi(getenv("PMM_BF16_DEFER")) : 1;
    a.defer = defer_env;
    a.qb_full = p.qb_full;
    static const int sync_env = getenv("PMM_BF16_SYNC") ? atoi(getenv("PMM_BF16_SYNC")) : 1;
    a.round_sync = sync_env;
    // round-barrier spin limit: workgroups of one round finish up to a few ms
    // apart (uneven epilogues); a workgroup that times out stops syncing
    static const int tmo_env =
        getenv("PMM_BF16_SYNC_TIMEOUT_US") ? atoi(getenv("PMM_BF16_SYNC_TIMEOUT_US")) : 20000;
    a.sync_timeout = tmo_env * 100;
#ifdef PMM_LAB
    static const bool stats = getenv("PMM_STATS") != nullptr;
#else
    constexpr bool stats = false;  // (per-phase cycle counters: lab build only)
#endif
    static unsigned long long *stats_buf = nullptr;
    if (stats) {
      if (!stats_buf) HIP_TRY(hipMalloc(&stats_buf, 128));
      HIP_TRY(hipMemsetAsync(stats_buf, 0, 128, s));
      a.stats = stats_buf;
    }
    {
      // Threshold seed (wave-specialised kernel): unseeded, every row starts
      // at "accept all" and its threshold only rises at compactions (every
      // ~220 appends), so a row queues and re-scores ~2k survivors over a 1M
      // corpus.  The k-th best of the first ns columns -- scored bit for bit
      // as the main pass scores them -- minus 1 is an exact lower bound of
      // the row's final k-th best: the main pass starts from it.
      const int seed_env = getenv("PMM_BF16_SEED") ? atoi(getenv("PMM_BF16_SEED")) : 1;  // (read per call: tests toggle it)
      int64_t ns = kSeedMaxNs;
      if (const char *ne = getenv("PMM_SEED_NS")) ns = std::max<int64_t>(32, std::min<int64_t>(atoll(ne), 4096) / 32 * 32);
      if (seed_env && p.variant == -2 && 4 * k <= ns && n >= 8 * ns &&
          (size_t)m * ns * 4 <= p.off_qn - p.off_cand) {
        float *sample = (float *)(w + p.off_cand);
        Timed t("seed_bf16", s);
        HIP_TRY(launch_seed_bf16_ws(a, sample, (int)ns, s));
        HIP_TRY(launch_seed_select(sample, ns, (int)m, (int)ns, (int)k, metric, a.gthr, s));
      }
    }
    if (p.variant == -6) {
#ifdef PMM_WITH_FF
      // fire-and-forget 256-row kernel: the guessed threshold (the j-th best
      // of an exact ns-row sample, minus 1), the pass, the exact re-score and
      // bucketing into the candidate lists; rows it cannot prove exact are
      // re-run below
      float *sample = (float *)(w + p.off_cand);
      {
        Timed t("seed_bf16", s);
        HIP_TRY(launch_seed_bf16_ws(a, sample, p.ff_ns, s));
        HIP_TRY(launch_seed_select(sample, p.ff_ns, (int)m, p.ff_ns, p.ff_j, metric, a.gthr, s));
      }
      a.qb_full = 0;
      a.ffreg = (unsigned long long *)(w + p.off_ffreg);
      a.ffcnt = (unsigned *)(w + p.off_ffcnt);
      a.ffcap = p.ffcap;
      {
        Timed t("gemm_bf16_topk/ff", s);
        HIP_TRY(launch_gemm_bf16_ff(a, p.grid, s));
      }
      HIP_TRY(hipMemsetAsync(w + p.off_fb, 0, 16, s));
      {
        Timed t("ff_bucket", s);
        HIP_TRY(launch_ff_bucket(a, (unsigned *)(w + p.off_fb), (int *)(w + p.off_fb + 16), s));
      }
#endif
    } else {
      // (the suffix names the kernel; pmm_timing_read matches substrings)
      Timed t(p.variant == -2 ? "gemm_bf16_topk/ws" : "gemm_bf16_topk/one-wave", s);
      HIP_TRY(p.variant == -2 ? launch_gemm_bf16_ws(a, p.grid, s) : launch_gemm_bf16(a, p.grid, s));
    }
    if (stats) {
      unsigned long long h[16];
      HIP_TRY(hipMemcpyAsync(h, stats_buf, 128, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
      if (p.variant == -2)
        fprintf(stderr,
                "[pmm stats] gemm_bf16_ws: units %d, S %d, tps %d, sync timeouts %llu, survivors "
                "%llu; MFMA-wave cycles %.3g; epilogue-wave cycles: DMA issue %.3g, epilogue "
                "%.3g, vmcnt waits %.3g, barriers %.3g of %.3g; compactions %.3g (%llu rows), "
                "survivor queueing %.3g, drains %.3g\n",
                p.units, p.S, p.tps, h[2], h[0], (double)h[1], (double)h[3], (double)h[4],
                (double)h[5], (double)h[6], (double)h[7], (double)h[8], h[9], (double)h[10],
                (double)h[11]);
      else
      fprintf(stderr,
              "[pmm stats] gemm_bf16: queued %llu, LDS-queue tiles %llu, sync timeouts %llu, "
              "compactions %llu, units %d, S %d, tps %d; wave cycles: K-loop %.3g, extract %.3g, "
              "pass 2 %.3g\n",
              h[0], h[1], h[2], h[3], p.units, p.S, p.tps, (double)h[4], (double)h[5], (double)h[6]);
    }
  }
  MergeArgs ma{};
  ma.cand = a.cand;
  ma.cnt = a.cnt;
  ma.gthr = a.gthr;
  ma.capg = p.capg;
  ma.M = (int)m;
  ma.S = p.S;
  ma.k_out = (int)k;
  ma.P = p.P;
  ma.metric = metric;
  ma.index_base = index_base;
  ma.out_idx = out_idx;
  ma.out_score = out_score;
  {
    Timed t("merge_topk", s);
    HIP_TRY(launch_merge(ma, 0, s));
  }
#ifdef PMM_WITH_FF
  if (p.variant == -6) {
    int rc = ff_rerun(q, ldq, m, c, ldc, n, d, k, metric, index_base, out_idx, out_score,
                      (const unsigned *)(w + p.off_fb), s, dev);
    if (rc) return rc;
  }
#endif
  return own ? arena_record(dev, s) : PMM_OK;
}

#ifdef PMM_WITH_FF
// The fire-and-forget kernel's rows that it could not prove exact (fewer than
// k candidates at or above the guessed threshold, or a dropped survivor):
// their query rows are gathered and re-run on the wave-specialised kernel
// against the whole corpus, and their lists replace the merge's.  Reads the
// row count back (a stream synchronisation) and allocates the re-run's
// buffers itself (hipMalloc, outside the caller's workspace): test-library
// behaviour only (libpmm_ff.so), never in libpmm.so.  Rare: the guess leaves
// about n j / ns scores per row against the k needed.
int ff_rerun(const uint16_t *q, int64_t ldq, int64_t m, const uint16_t *c, int64_t ldc, int64_t n, int64_t d,
             int64_t k, int metric, uint32_t index_base, uint32_t *out_idx, float *out_score, const unsigned *fb,
             hipStream_t s, int dev) {
  unsigned nfb = 0;
  HIP_TRY(hipMemcpyAsync(&nfb, fb, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (getenv("PMM_FF_DEBUG")) fprintf(stderr, "[pmm ff] re-run rows %u of %lld\n", nfb, (long long)m);
  if (nfb == 0) return PMM_OK;
  // one allocation: the gathered rows, their lists, the re-run's workspace;
  // the row list stays on the device (gather and scatter kernels read it)
  const int64_t r = nfb;
  const int *rows = (const int *)(fb + 4);
  const bool prev = t_no_ff;
  t_no_ff = true;
  const int64_t dp = cdiv(d, kBf16DAlign) * kBf16DAlign;
  const size_t wb = pmm_topk_workspace_bytes(r, n, dp, k, metric, PMM_COMPUTE_BF16);
  const size_t o_i = al256((size_t)r * ldq * 2), o_s = o_i + al256((size_t)r * k * 4),
               o_w = o_s + al256((size_t)r * k * 4);
  char *buf = nullptr;
  hipError_t e = hipMalloc(&buf, o_w + wb);
  int rc = PMM_OK;
  if (e == hipSuccess) e = launch_ff_gather_rows(q, ldq, rows, (int)r, (uint16_t *)buf, s);
  if (e == hipSuccess)
    rc = topk_bf16_device_impl((const uint16_t *)buf, ldq, r, c, ldc, n, d, k, metric, index_base,
                               (uint32_t *)(buf + o_i), (float *)(buf + o_s), buf + o_w, wb, s, dev);
  if (e == hipSuccess && rc == PMM_OK)
    e = launch_ff_scatter_lists((const uint32_t *)(buf + o_i), (const float *)(buf + o_s), rows, (int)r, (int)k,
                                out_idx, out_score, s);
  t_no_ff = prev;
  if (buf) {
    const hipError_t e2 = hipStreamSynchronize(s);  // (before the buffer is freed)
    (void)hipFree(buf);
    if (e == hipSuccess) e = e2;
  }
  if (e != hipSuccess) return fail(PMM_ERR_HIP, "ff re-run: %s", hipGetErrorString(e));
  return rc;
}
#endif  // PMM_WITH_FF

// Upload a host matrix rows x d into a device buffer with row stride dp,
// zero-padding columns d..dp-1.
int upload_padded(void *dst, const void *src, int64_t rows, int64_t d, int64_t dp, size_t elem,
                  hipStream_t s) {
  if (rows <= 0) return PMM_OK;
  Timed t("h2d", s);  // bench.py's end-to-end breakdown (pmm_timing_*)
  if (dp == d) {
    HIP_TRY(hipMemcpyAsync(dst, src, (size_t)rows * d * elem, hipMemcpyHostToDevice, s));
  } else {
    HIP_TRY(hipMemsetAsync(dst, 0, (size_t)rows * dp * elem, s));
    HIP_TRY(hipMemcpy2DAsync(dst, (size_t)dp * elem, src, (size_t)d * elem, (size_t)d * elem,
                             (size_t)rows, hipMemcpyHostToDevice, s));
  }
  return PMM_OK;
}

int validate_sizes(int64_t m, int64_t n, int64_t d, int64_t k, bool topk, bool allow_k_gt_n = false) {
  if (m < 0 || n < 0 || d < 0) return fail(PMM_ERR_ARG, "negative size (m=%lld n=%lld d=%lld)",
                                           (long long)m, (long long)n, (long long)d);
  if (m > INT32_MAX || n > (int64_t)UINT32_MAX - 1 || n > INT32_MAX)
    return fail(PMM_ERR_ARG, "size out of range (m=%lld n=%lld)", (long long)m, (long long)n);
  if (topk) {
    if (k < 0) return fail(PMM_ERR_ARG, "k must be >= 0 (got %lld)", (long long)k);
    if (k > n && !allow_k_gt_n)
      return fail(PMM_ERR_ARG, "k (%lld) must be <= n (%lld): clip k to n first", (long long)k,
                  (long long)n);
  }
  return PMM_OK;
}

// A non-empty call needs every buffer it names (the reference never passes
// null; a binding that does gets an error instead of a fault).
template <typename... P>
int need_buffers(P... p) {
  return ((p != nullptr) && ...) ? PMM_OK : fail(PMM_ERR_ARG, "null argument");
}

// Host-buffer f32 top-k over a large corpus with the upload overlapped with
// compute.  The corpus is cut into chunks: a small first one (uploaded, with
// the queries, before any compute) and CHUNKS-1 equal ones.  Chunk i + 1 is
// copied on the thread's copy stream while chunk i's fused top-k runs on the
// compute stream; each chunk's list carries global indices (index_base) into
// a [chunks][2][m][k] buffer (index plane, score plane), merged in place at
// the end -- the sharded path's merge, on one device.  The shared per-row
// thresholds carry from chunk to chunk (keep_gthr): a chunk's k-th composite
// is a lower bound of the global k-th, so later chunks start pruned and the
// result equals the one-launch result bit for bit.
constexpr size_t kChunkedMinBytes = size_t(256) << 20;  // corpus bytes from which uploads overlap
constexpr int kChunks = 4;

int topk_f32_host_chunked(const float *q, int64_t m, const float *c, int64_t n, int64_t d, int64_t k,
                          int metric, uint32_t *out_idx, float *out_score, int dev, hipStream_t s) {
  const int64_t dp = cdiv(d, 32) * 32;
  int64_t bnd[kChunks + 1];
  bnd[0] = 0;
  bnd[1] = std::max<int64_t>(k, n / 16);
  for (int i = 2; i <= kChunks; i++) bnd[i] = bnd[1] + (n - bnd[1]) * (i - 1) / (kChunks - 1);
  size_t ws_need = 0;
  for (int i = 0; i < kChunks; i++)
    ws_need = std::max(ws_need, pmm_topk_workspace_bytes(m, bnd[i + 1] - bnd[i], dp, k, metric, PMM_COMPUTE_F32));
  const size_t lists = (size_t)kChunks * 2 * m * k * 4;
  size_t off_q = 0, off_c = al256((size_t)m * dp * 4), off_l = off_c + al256((size_t)n * dp * 4);
  size_t off_i = off_l + al256(lists), off_s = off_i + al256((size_t)m * k * 4);
  size_t off_w = off_s + al256((size_t)m * k * 4);
  hipStream_t cs;
  int rc;
  if ((rc = thread_stream(dev, &cs, true))) return rc;
  void *base;
  if ((rc = arena(dev, s, off_w + ws_need, &base))) return rc;
  char *b = (char *)base;
  uint32_t *li = (uint32_t *)(b + off_l);
  hipEvent_t ev[kChunks + 1] = {};
  // One exit for every failure after the copy stream may have work queued:
  // the copy stream writes into the arena, so it is drained before the arena
  // can be reused or grown (freed) by a later call, and the events are freed.
  auto finish = [&](int code) {
    if (code != PMM_OK) {
      (void)hipStreamSynchronize(cs);
      (void)hipStreamSynchronize(s);
    }
    for (auto &e : ev)
      if (e) (void)hipEventDestroy(e);
    return code;
  };
#define CHUNK_TRY(expr)                                                                   \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return finish(fail(PMM_ERR_HIP, "HIP error %s at %s:%d (%s)", hipGetErrorString(e_), \
                         __FILE__, __LINE__, #expr));                                     \
  } while (0)
  for (auto &e : ev) CHUNK_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  // the copy stream must not overwrite the arena before earlier compute on
  // the compute stream is done with it
  hipEvent_t ready = ev[kChunks];
  CHUNK_TRY(hipEventRecord(ready, s));
  CHUNK_TRY(hipStreamWaitEvent(cs, ready, 0));
  if ((rc = upload_padded(b + off_q, q, m, d, dp, 4, cs))) return finish(rc);
  for (int i = 0; i < kChunks; i++) {
    const int64_t lo = bnd[i], rows = bnd[i + 1] - bnd[i];
    // a pageable copy returns once staged: chunk i + 1 is copied while the
    // device computes chunk i
    if ((rc = upload_padded(b + off_c + (size_t)lo * dp * 4, c + lo * d, rows, d, dp, 4, cs))) return finish(rc);
    CHUNK_TRY(hipEventRecord(ev[i], cs));
    CHUNK_TRY(hipStreamWaitEvent(s, ev[i], 0));
    rc = topk_f32_device_impl((const float *)(b + off_q), dp, m, (const float *)(b + off_c) + lo * dp, dp,
                              rows, d, k, metric, (uint32_t)lo, li + (size_t)i * 2 * m * k,
                              (float *)(li + (size_t)i * 2 * m * k + (size_t)m * k), b + off_w, ws_need, s,
                              dev, nullptr, i > 0);
    if (rc) return finish(rc);
  }
  MergeArgs ma{};
  ma.in_idx = li;
  ma.in_score = (const float *)(li + (size_t)m * k);
  ma.k_in = (int)k;
  ma.row_stride = k;
  ma.list_stride = 2 * m * k;
  ma.M = (int)m;
  ma.S = kChunks;
  ma.sorted = 1;  // each chunk's lists are a top-k output: best first
  ma.k_out = (int)k;
  ma.P = std::min(8192, next_pow2(2 * (int)k + 64, 128));
  ma.metric = metric;
  ma.out_idx = (uint32_t *)(b + off_i);
  ma.out_score = (float *)(b + off_s);
  {
    Timed t("merge_chunks", s);
    CHUNK_TRY(launch_merge(ma, 1, s));
  }
  {
    Timed t("d2h", s);
    CHUNK_TRY(hipMemcpyAsync(out_idx, b + off_i, (size_t)m * k * 4, hipMemcpyDeviceToHost, s));
    CHUNK_TRY(hipMemcpyAsync(out_score, b + off_s, (size_t)m * k * 4, hipMemcpyDeviceToHost, s));
  }
  CHUNK_TRY(hipStreamSynchronize(s));
#undef CHUNK_TRY
  return finish(PMM_OK);
}

// ---------------------------------------------------------------------------
// Corpus-sharded top-k over several devices from ONE host thread (the
// drop-in boundary's multi-GPU path; pmm_set_devices).  SURVEY 8e's plan in
// one process: the corpus is row-sharded (contiguous, sizes differ by <= 1),
// every device gets the queries, runs the fused top-k on its shard with
// index_base = the shard's first global row into a [2][m][k] block (index
// plane, score plane), the blocks are copied peer-to-peer (xGMI) into the
// root device's [G][2][m][k] buffer and k-way merged there in place
// (merge_kernel, the same strided loader the RCCL-gathered lists use).  All
// devices work concurrently: every launch is asynchronous on the device's own
// stream of this thread; the root waits on per-shard events.  Each shard's
// list is the exact top-k of its rows under the total order, so the merged
// list equals the one-device result bit for bit.
// ---------------------------------------------------------------------------
struct ShardSrc {
  int dev;
  int64_t lo, rows;
  const float *host;       // host corpus rows [lo, lo + rows), row stride d, or
  const float *dev_rows;   // resident padded rows (stride dp) of a corpus handle
  const float *dev_norms;  // with dev_rows: the handle's norms of this metric ([rows | rows factors])
};

std::mutex g_peer_mu;
bool g_peer_tried[kMaxDevices][kMaxDevices];

// Lets `dev` read `peer`'s memory directly (xGMI) when the platform allows;
// a peer copy works either way, so failures are ignored.
void enable_peer(int dev, int peer) {
  if (dev == peer) return;
  std::lock_guard<std::mutex> lk(g_peer_mu);
  if (g_peer_tried[dev][peer]) return;
  g_peer_tried[dev][peer] = true;
  int can = 0;
  if (hipDeviceCanAccessPeer(&can, dev, peer) == hipSuccess && can) (void)hipDeviceEnablePeerAccess(peer, 0);
  (void)hipGetLastError();
}

// Memory plan of topk_sharded (pure: no HIP call, so the CPU tests check it
// through pmm_shard_plan).  One DevPlan per DISTINCT device of the list: that
// device's queries once, one workspace (its shards run in stream order), and
// per shard the uploaded rows (host shards only) and its [2][m][k] list; the
// root plan (the first shard's device) also holds the gathered [G][2][m][k]
// lists and the merged output.
struct DevPlan {
  int dev;
  hipStream_t s = nullptr;
  char *base = nullptr;
  size_t off_q = 0, off_qb = 0, off_ws = 0, ws_bytes = 0, total = 0;
};
struct ShardLayout {
  std::vector<DevPlan> dps;
  std::vector<int> plan_of;  // shard -> index into dps
  std::vector<size_t> off_c, off_cb, off_list;
  size_t off_gather = 0, off_out = 0;  // in the root plan
};

int device_cus(int dev) {
  std::lock_guard<std::mutex> lk(g_dev_mu);
  return (dev >= 0 && dev < kMaxDevices && g_dev[dev].probed) ? g_dev[dev].cus : 256;
}

void plan_sharded(const std::vector<ShardSrc> &sh, int64_t m, int64_t d, int64_t k, int metric, int compute,
                  ShardLayout &L) {
  const int G = (int)sh.size();
  const bool bf16 = compute == PMM_COMPUTE_BF16;
  const int64_t dp = bf16 ? cdiv(d, kBf16DAlign) * kBf16DAlign : cdiv(d, 32) * 32;
  const size_t list_bytes = (size_t)2 * m * k * 4;
  L.dps.clear();
  L.plan_of.assign(G, 0);
  L.off_c.assign(G, 0);
  L.off_cb.assign(G, 0);
  L.off_list.assign(G, 0);
  for (int g = 0; g < G; g++) {
    int j = 0;
    while (j < (int)L.dps.size() && L.dps[j].dev != sh[g].dev) j++;
    if (j == (int)L.dps.size()) {
      DevPlan p;
      p.dev = sh[g].dev;
      L.dps.push_back(p);
    }
    L.plan_of[g] = j;
  }
  for (auto &p : L.dps) {
    size_t off = 0;
    p.off_q = off;  // f32: padded rows; bf16: f32 staging rows (stride d)
    off = al256(off + (size_t)m * (bf16 ? d : dp) * 4);
    p.off_qb = off;  // bf16 rows
    off = al256(off + (bf16 ? (size_t)m * dp * 2 : 0));
    for (int g = 0; g < G; g++) {
      if (sh[g].dev != p.dev) continue;
      size_t need;
      if (bf16 && !bf16_native(d, k, sh[g].rows)) {
        need = bf16_widened_bytes(m, sh[g].rows, d, k, metric, device_cus(p.dev));
      } else {
        Plan tp;
        plan_topk(m, sh[g].rows, dp, k, metric, device_cus(p.dev), tp, compute);
        need = tp.total;
      }
      p.ws_bytes = std::max(p.ws_bytes, need);
      L.off_c[g] = off;
      if (sh[g].host) off = al256(off + (size_t)sh[g].rows * (bf16 ? d : dp) * 4);
      L.off_cb[g] = off;
      if (bf16) off = al256(off + (size_t)sh[g].rows * dp * 2);
      L.off_list[g] = off;
      off = al256(off + list_bytes);
    }
    p.off_ws = off;
    off = al256(off + p.ws_bytes);
    p.total = off;
  }
  DevPlan &rp = L.dps[L.plan_of[0]];
  L.off_gather = rp.total;
  L.off_out = al256(L.off_gather + (size_t)G * list_bytes);
  rp.total = al256(L.off_out + list_bytes);
}

int topk_sharded(const float *q, int64_t m, int64_t d, int64_t k, int metric, int compute,
                 const std::vector<ShardSrc> &sh, uint32_t *out_idx, float *out_score) {
  const int G = (int)sh.size();
  int cur = 0;
  HIP_TRY(hipGetDevice(&cur));
  struct Restore {
    int d;
    ~Restore() { (void)hipSetDevice(d); }
  } restore{cur};
  const bool bf16 = compute == PMM_COMPUTE_BF16;
  const int64_t dp = bf16 ? cdiv(d, kBf16DAlign) * kBf16DAlign : cdiv(d, 32) * 32;
  const int root = sh[0].dev;
  const size_t list_bytes = (size_t)2 * m * k * 4;
  for (const ShardSrc &x : sh)
    if (int rc = probe_device(x.dev)) return rc;
  ShardLayout L;
  plan_sharded(sh, m, d, k, metric, compute, L);
  std::vector<DevPlan> &dps = L.dps;
  const std::vector<int> &plan_of = L.plan_of;
  const std::vector<size_t> &off_c = L.off_c, &off_cb = L.off_cb, &off_list = L.off_list;
  DevPlan &rp = dps[plan_of[0]];
  const size_t off_gather = L.off_gather, off_out = L.off_out;
  for (auto &p : dps) {
    HIP_TRY(hipSetDevice(p.dev));
    if (int rc = thread_stream(p.dev, &p.s)) return rc;
    void *b;
    if (int rc = arena(p.dev, p.s, p.total, &b)) return rc;
    p.base = (char *)b;
  }
  std::vector<hipEvent_t> ev(G, nullptr);
  auto finish = [&](int code) {
    if (code != PMM_OK)
      for (auto &p : dps) {
        (void)hipSetDevice(p.dev);
        (void)hipStreamSynchronize(p.s);
      }
    for (int g = 0; g < G; g++)
      if (ev[g]) {
        (void)hipSetDevice(sh[g].dev);
        (void)hipEventDestroy(ev[g]);
      }
    return code;
  };
#define SH_TRY(expr)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return finish(fail(PMM_ERR_HIP, "HIP error %s at %s:%d (%s)", hipGetErrorString(e_), \
                         __FILE__, __LINE__, #expr));                                     \
  } while (0)
#define SH_RC(expr)                   \
  do {                                \
    int rc_ = (expr);                 \
    if (rc_ != PMM_OK) return finish(rc_); \
  } while (0)
  // queries to every device
  for (auto &p : dps) {
    SH_TRY(hipSetDevice(p.dev));
    if (bf16) {
      SH_TRY(hipMemcpyAsync(p.base + p.off_q, q, (size_t)m * d * 4, hipMemcpyHostToDevice, p.s));
      SH_TRY(launch_f32_to_bf16((const float *)(p.base + p.off_q), m, d, d, (uint16_t *)(p.base + p.off_qb), dp,
                                p.s));
    } else {
      SH_RC(upload_padded(p.base + p.off_q, q, m, d, dp, 4, p.s));
    }
  }
  // per shard: rows, fused top-k with global indices, completion event
  for (int g = 0; g < G; g++) {
    DevPlan &p = dps[plan_of[g]];
    const ShardSrc &x = sh[g];
    SH_TRY(hipSetDevice(p.dev));
    SH_TRY(hipEventCreateWithFlags(&ev[g], hipEventDisableTiming));
    uint32_t *li = (uint32_t *)(p.base + off_list[g]);
    float *ls = (float *)(li + (size_t)m * k);
    if (bf16) {
      SH_TRY(hipMemcpyAsync(p.base + off_c[g], x.host, (size_t)x.rows * d * 4, hipMemcpyHostToDevice, p.s));
      SH_TRY(launch_f32_to_bf16((const float *)(p.base + off_c[g]), x.rows, d, d,
                                (uint16_t *)(p.base + off_cb[g]), dp, p.s));
      SH_RC(topk_bf16_device_impl((const uint16_t *)(p.base + p.off_qb), dp, m,
                                  (const uint16_t *)(p.base + off_cb[g]), dp, x.rows, d, k, metric,
                                  (uint32_t)x.lo, li, ls, p.base + p.off_ws, p.ws_bytes, p.s, p.dev));
    } else {
      const float *c = x.dev_rows;
      if (x.host) {
        SH_RC(upload_padded(p.base + off_c[g], x.host, x.rows, d, dp, 4, p.s));
        c = (const float *)(p.base + off_c[g]);
      }
      SH_RC(topk_f32_device_impl((const float *)(p.base + p.off_q), dp, m, c, dp, x.rows, d, k, metric,
                                 (uint32_t)x.lo, li, ls, p.base + p.off_ws, p.ws_bytes, p.s, p.dev,
                                 x.host ? nullptr : x.dev_norms));
    }
    SH_TRY(hipEventRecord(ev[g], p.s));
  }
  // gather into the root (peer copies over xGMI), merge, download
  SH_TRY(hipSetDevice(root));
  char *gb = rp.base + off_gather;
  for (int g = 0; g < G; g++) {
    enable_peer(root, sh[g].dev);
    SH_TRY(hipStreamWaitEvent(rp.s, ev[g], 0));
    SH_TRY(hipMemcpyPeerAsync(gb + (size_t)g * list_bytes, root, dps[plan_of[g]].base + off_list[g], sh[g].dev,
                              list_bytes, rp.s));
  }
  MergeArgs ma{};
  ma.in_idx = (const uint32_t *)gb;
  ma.in_score = (const float *)((const uint32_t *)gb + (size_t)m * k);
  ma.k_in = (int)k;
  ma.row_stride = k;
  ma.list_stride = 2 * m * k;
  ma.M = (int)m;
  ma.S = G;
  ma.sorted = 1;  // each shard's lists are a top-k output: best first
  ma.k_out = (int)k;
  ma.P = std::min(8192, next_pow2(2 * (int)k + 64, 128));
  ma.metric = metric;
  ma.out_idx = (uint32_t *)(rp.base + off_out);
  ma.out_score = (float *)(ma.out_idx + (size_t)m * k);
  {
    Timed t("merge_devices", rp.s);
    SH_TRY(launch_merge(ma, 1, rp.s));
  }
  SH_TRY(hipMemcpyAsync(out_idx, ma.out_idx, (size_t)m * k * 4, hipMemcpyDeviceToHost, rp.s));
  SH_TRY(hipMemcpyAsync(out_score, ma.out_score, (size_t)m * k * 4, hipMemcpyDeviceToHost, rp.s));
  SH_TRY(hipStreamSynchronize(rp.s));
#undef SH_TRY
#undef SH_RC
  return finish(PMM_OK);
}

// ---------------------------------------------------------------------------
// f64 top-k (src/matmul.rs:449-468 -> src/metrics.rs:258-311 + src/topk.rs:6-39)
// on device rows of stride >= roundup(d, 16), zero-padded.  k <= kFusedMaxK:
// the fused chunked scan of pmm_f64.hip (no M x N matrix); a row whose buffer
// overflowed (adversarial data: every chunk beats the last) or k above the
// fused limit: the materialised path (f64 GEMM store + row select), which also
// serves as the PMM_F64_FUSED=0 reference.
// ---------------------------------------------------------------------------
struct F64Plan {
  int cap = 0, P = 0;
  int64_t mc = 0;  // query rows per pass (candidate-buffer budget)
  size_t off_qn = 0, off_cn = 0, off_tkey = 0, off_tidx = 0, off_cnt = 0, off_cand = 0, off_flag = 0,
         off_mat = 0, total = 0;
};
constexpr size_t kF64CandBudget = size_t(1) << 30;

void plan_f64(int64_t m, int64_t n, int64_t k, F64Plan &p) {
  p.cap = std::min(4096, std::max(1024, next_pow2(4 * (int)std::min<int64_t>(k, kFusedMaxK) + 256)));
  p.P = p.cap;
  p.mc = std::max<int64_t>(1, std::min<int64_t>(m, (int64_t)(kF64CandBudget / ((size_t)p.cap * 16))));
  size_t off = 0;
  p.off_flag = off;
  off += 256;
  p.off_qn = off;
  off = al256(off + (size_t)m * 8);
  p.off_cn = off;
  off = al256(off + (size_t)n * 8);
  p.off_tkey = off;
  off = al256(off + (size_t)p.mc * 8);
  p.off_tidx = off;
  off = al256(off + (size_t)p.mc * 4);
  p.off_cnt = off;
  off = al256(off + (size_t)p.mc * 4);
  p.off_cand = off;
  off = al256(off + (size_t)p.mc * p.cap * 16);
  p.total = off;
}


// Fused scan or materialised scores, by the size of the M x N f64 score
// matrix the materialised path writes and re-reads (device API, cosine,
// k = 10, D = 256; profiles/r4_f64/f64_sizes.jsonl): 1000 x 10000 (80 MB)
// materialised 0.239 ms vs fused 0.348 (its chunk launches, selects and
// overflow check); 1000 x 100000 (0.8 GB) 2.02 vs 1.40; 4096 x 1M (33 GB)
// 209 vs 47.6.  The threshold sits between the first two.  PMM_F64_FUSED=1
// / 0 forces either (read per call: tests compare both paths).
constexpr double kF64FusedMinMatrixBytes = 256.0 * 1024.0 * 1024.0;
bool f64_fused_enabled(int64_t m, int64_t n) {
  const char *e = getenv("PMM_F64_FUSED");
  if (e && *e) return atoi(e) != 0;
  return (double)m * (double)n * 8.0 > kF64FusedMinMatrixBytes;
}

// Which path a call takes, decided once per call (the workspace is sized for
// it and the device code follows it, whatever PMM_F64_FUSED says meanwhile).
bool f64_use_fused(int64_t m, int64_t n, int64_t k) { return k <= kFusedMaxK && f64_fused_enabled(m, n); }

// Workspace of one f64 top-k call: the materialised path's alone when the call
// takes it; the fused scan's and the materialised path's (its overflow
// fallback reuses the workspace) otherwise.  (Sizing every call for both held
// up to 1 GiB of candidate buffers next to a small score matrix.)
size_t f64_workspace_bytes(int64_t m, int64_t n, int64_t k, bool fused) {
  MatPlan mp;
  plan_materialise(m, n, k, 8, mp);
  if (!fused) return mp.total;
  F64Plan p;
  plan_f64(m, n, k, p);
  return std::max(p.total, mp.total);
}

// cn_pre: the corpus rows' norms of this metric already on the device (a
// corpus handle's, computed at creation by the same kernel), else nullptr.
int topk_f64_materialised(const double *dq, int64_t ldq, int64_t m, const double *dc, int64_t ldc, int64_t n,
                          int64_t d, int64_t k, int metric, uint32_t index_base, uint32_t *oi, double *os,
                          char *w, hipStream_t s, const double *cn_pre = nullptr) {
  MatPlan p;
  plan_materialise(m, n, k, 8, p);
  double *qn = (double *)(w + p.off_qn), *cn = (double *)(w + p.off_cn);
  double *sc = (double *)(w + p.off_scores);
  if (metric != kMetricDot) {
    const int sq = metric == kMetricEuclidean;
    HIP_TRY(launch_norms_f64(dq, m, d, ldq, sq, qn, s));
    if (cn_pre) cn = (double *)cn_pre;
    else HIP_TRY(launch_norms_f64(dc, n, d, ldc, sq, cn, s));
  }
  const int64_t dp = cdiv(d, 16) * 16;
  for (int64_t r0 = 0; r0 < m; r0 += p.rows) {
    const int64_t rows = std::min<int64_t>(p.rows, m - r0);
    {
      Timed t("gemm_f64_scores", s);
      HIP_TRY(launch_gemm_f64_store(dq + r0 * ldq, ldq, dc, ldc, qn + r0, cn, (int)rows, (int)n, (int)dp, metric,
                                    1, sc, n, s));
    }
    if (!p.global_sort) {
      RowSelArgs ra{};
      ra.scores = sc;
      ra.lds = n;
      ra.rows = (int)rows;
      ra.N = (int)n;
      ra.k = (int)k;
      ra.P = p.P;
      ra.metric = metric;
      ra.is_f64 = 1;
      ra.index_base = index_base;
      ra.out_idx = oi + r0 * k;
      ra.out_score = os + r0 * k;
      Timed t("select_f64_rows", s);
      HIP_TRY(launch_rowselect(ra, s));
    } else {
      HIP_TRY(launch_rowsort_global(sc, n, (int)rows, (int)n, 1, metric, w + p.off_keys, p.P2, (int)k, index_base,
                                    oi + r0 * k, os + r0 * k, s));
    }
  }
  return PMM_OK;
}

// flag_copy (the sharded path): instead of waiting here for the fused scan's
// overflow flag, enqueue a copy of it to flag_copy (device memory) and return;
// the caller checks it once every device has finished and re-runs an
// overflowed shard with topk_f64_materialised.
int topk_f64_device_impl(const double *dq, int64_t ldq, int64_t m, const double *dc, int64_t ldc, int64_t n,
                         int64_t d, int64_t k, int metric, uint32_t index_base, uint32_t *oi, double *os, char *w,
                         hipStream_t s, bool fused, const double *cn_pre = nullptr, unsigned *flag_copy = nullptr) {
  if (!fused)
    return topk_f64_materialised(dq, ldq, m, dc, ldc, n, d, k, metric, index_base, oi, os, w, s, cn_pre);
  F64Plan p;
  plan_f64(m, n, k, p);
  const int64_t dp = cdiv(d, 16) * 16;
  double *qn = (double *)(w + p.off_qn), *cn = (double *)(w + p.off_cn);
  unsigned *flag = (unsigned *)(w + p.off_flag);
  if (metric != kMetricDot) {
    const int sq = metric == kMetricEuclidean;
    Timed t("norms_f64", s);
    HIP_TRY(launch_norms_f64(dq, m, d, ldq, sq, qn, s));
    if (cn_pre) cn = (double *)cn_pre;
    else HIP_TRY(launch_norms_f64(dc, n, d, ldc, sq, cn, s));
  }
  // chunk schedule: the first chunk fills half a buffer (accept-all), later
  // chunks are g times the columns seen.  After `seen` columns the threshold
  // is the k-th best of them, so a chunk of g * seen columns from the same
  // distribution leaves ~g * X survivors in a row, X ~ Gamma(k) (the k-th
  // order statistic's quantile times seen).  Its spread is k^-1/2 of its mean
  // whatever `seen` is, so g is sized for the tail, not the mean: with
  // P(X > k + t) <= exp(-t^2 / (2 (k + t))) and t = 23 + sqrt(529 + 46 k)
  // (a per-row, per-chunk tail of e^-23 ~ 1e-10), g (k + t) <= cap - k keeps
  // every row inside its buffer.  (g = (cap/2 - k) / k, sized for the mean,
  // overflowed some row of nearly every call at 4096 x 1M: the whole call
  // then re-ran materialised, 257 vs 209 ms; profiles/r4_f64/.)  Adversarial
  // orders still overflow and fall back below.
  const int64_t s0 = std::min<int64_t>(n, p.cap / 2);
  const double tail = 23.0 + std::sqrt(529.0 + 46.0 * (double)k);
  const int64_t g = std::max<int64_t>(1, (int64_t)((double)(p.cap - k) / ((double)k + tail)));
  HIP_TRY(hipMemsetAsync(flag, 0, 4, s));
  for (int64_t r0 = 0; r0 < m; r0 += p.mc) {
    const int rows = (int)std::min<int64_t>(p.mc, m - r0);
    unsigned long long *tkey = (unsigned long long *)(w + p.off_tkey);
    uint32_t *tidx = (uint32_t *)(w + p.off_tidx);
    unsigned *cnt = (unsigned *)(w + p.off_cnt);
    Ent *cand = (Ent *)(w + p.off_cand);
    HIP_TRY(launch_f64_reset(tkey, tidx, cnt, rows, (unsigned)s0, s));
    F64TopkArgs a{};
    a.q = dq + r0 * ldq;
    a.c = dc;
    a.qn = qn + r0;
    a.cn = cn;
    a.ldq = ldq;
    a.ldc = ldc;
    a.M = rows;
    a.D = (int)dp;
    a.metric = metric;
    a.tkey = tkey;
    a.tidx = tidx;
    a.cnt = cnt;
    a.cand = cand;
    a.cap = p.cap;
    F64SelArgs sa{};
    sa.cand = cand;
    sa.cnt = cnt;
    sa.cap = p.cap;
    sa.M = rows;
    sa.k = (int)k;
    sa.P = p.P;
    sa.tkey = tkey;
    sa.tidx = tidx;
    sa.metric = metric;
    sa.index_base = index_base;
    sa.out_idx = oi + r0 * k;
    sa.out_score = os + r0 * k;
    sa.overflow = flag;
    int64_t seen = 0, chunk = s0;
    while (seen < n) {
      const int64_t cc = std::min<int64_t>(chunk, n - seen);
      a.col0 = (int)seen;
      a.ncol = (int)cc;
      a.accept_all = seen == 0;  // (s0 <= cap / 2)
      {
        Timed t("gemm_f64_topk", s);
        HIP_TRY(launch_gemm_f64_topk(a, s));
      }
      seen += cc;
      sa.mode = seen < n ? 0 : 1;
      {
        Timed t("select_f64", s);
        HIP_TRY(launch_f64_select(sa, s));
      }
      chunk = seen * g;
    }
  }
  if (flag_copy) {
    HIP_TRY(hipMemcpyAsync(flag_copy, flag, 4, hipMemcpyDeviceToDevice, s));
    return PMM_OK;
  }
  // an overflowed row dropped candidates: redo the call on the materialised path
  unsigned of = 0;
  HIP_TRY(hipMemcpyAsync(&of, flag, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (of) return topk_f64_materialised(dq, ldq, m, dc, ldc, n, d, k, metric, index_base, oi, os, w, s, cn_pre);
  return PMM_OK;
}

// ---------------------------------------------------------------------------
// Corpus-sharded f64 top-k (the drop-in path of Polars' default Float64
// columns under pmm_set_devices): the f32 path's plan (topk_sharded) with the
// f64 top-k per shard.  Every device gets the queries once; each shard runs
// topk_f64_device_impl on its rows with index_base = its first global row,
// k_g = min(k, rows) (a shorter list is padded with empty slots); the fused
// scans' overflow flags are read only after every device has finished (an
// overflowed shard re-runs materialised, as one device would); the [m][k]
// lists meet in the root's [G][m][k] planes by peer copies and
// f64_kway_merge_kernel merges them.  A shard's list is the exact top-k of
// its rows under the f64 total order, so the merged list equals the
// one-device result bit for bit (indices and f64 scores).
// ---------------------------------------------------------------------------
struct ShardSrc64 {
  int dev;
  int64_t lo, rows;
  const double *host;       // host rows [lo, lo + rows), row stride d, or
  const double *dev_rows;   // a corpus handle's resident padded rows (stride dp)
  const double *dev_norms;  // with dev_rows: the handle's norms of this metric (nullptr for dot)
};

int topk_sharded_f64(const double *q, int64_t m, int64_t d, int64_t k, int metric, const std::vector<ShardSrc64> &sh,
                     uint32_t *out_idx, double *out_score) {
  const int G = (int)sh.size();
  int cur = 0;
  HIP_TRY(hipGetDevice(&cur));
  struct Restore {
    int d;
    ~Restore() { (void)hipSetDevice(d); }
  } restore{cur};
  const int64_t dp = cdiv(d, 16) * 16;
  const int root = sh[0].dev;
  for (const ShardSrc64 &x : sh)
    if (int rc = probe_device(x.dev)) return rc;
  struct Dev64 {
    int dev;
    hipStream_t s = nullptr;
    char *base = nullptr;
    size_t off_q = 0, off_ws = 0, ws_bytes = 0, off_flags = 0, total = 0;
  };
  std::vector<Dev64> dps;
  std::vector<int> plan_of(G), slot(G);
  std::vector<int64_t> kg(G);
  std::vector<bool> fused(G);
  std::vector<size_t> off_c(G), off_tmp(G), off_li(G), off_ls(G);
  for (int g = 0; g < G; g++) {
    int j = 0;
    while (j < (int)dps.size() && dps[j].dev != sh[g].dev) j++;
    if (j == (int)dps.size()) dps.push_back(Dev64{sh[g].dev});
    plan_of[g] = j;
    kg[g] = std::min<int64_t>(k, sh[g].rows);
    fused[g] = f64_use_fused(m, sh[g].rows, kg[g]);
  }
  for (int j = 0; j < (int)dps.size(); j++) {
    Dev64 &p = dps[j];
    size_t off = 0;
    p.off_q = off;
    off = al256(off + (size_t)m * dp * 8);
    int ns = 0;
    for (int g = 0; g < G; g++) {
      if (plan_of[g] != j) continue;
      slot[g] = ns++;
      p.ws_bytes = std::max(p.ws_bytes, f64_workspace_bytes(m, sh[g].rows, kg[g], fused[g]));
      off_c[g] = off;
      if (sh[g].host) off = al256(off + (size_t)sh[g].rows * dp * 8);
      off_tmp[g] = off;
      if (kg[g] < k) off = al256(off + (size_t)m * kg[g] * 12);
      off_li[g] = off;
      off = al256(off + (size_t)m * k * 4);
      off_ls[g] = off;
      off = al256(off + (size_t)m * k * 8);
    }
    p.off_flags = off;
    off = al256(off + (size_t)ns * 4);
    p.off_ws = off;
    off = al256(off + p.ws_bytes);
    p.total = off;
  }
  Dev64 &rp = dps[plan_of[0]];
  const size_t off_gi = rp.total, off_gs = al256(off_gi + (size_t)G * m * k * 4);
  const size_t off_oi = al256(off_gs + (size_t)G * m * k * 8), off_os = al256(off_oi + (size_t)m * k * 4);
  rp.total = al256(off_os + (size_t)m * k * 8);
  for (auto &p : dps) {
    HIP_TRY(hipSetDevice(p.dev));
    if (int rc = thread_stream(p.dev, &p.s)) return rc;
    void *b;
    if (int rc = arena(p.dev, p.s, p.total, &b)) return rc;
    p.base = (char *)b;
  }
  std::vector<hipEvent_t> ev(G, nullptr);
  auto finish = [&](int code) {
    if (code != PMM_OK)
      for (auto &p : dps) {
        (void)hipSetDevice(p.dev);
        (void)hipStreamSynchronize(p.s);
      }
    for (int g = 0; g < G; g++)
      if (ev[g]) {
        (void)hipSetDevice(sh[g].dev);
        (void)hipEventDestroy(ev[g]);
      }
    return code;
  };
#define SH_TRY(expr)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return finish(fail(PMM_ERR_HIP, "HIP error %s at %s:%d (%s)", hipGetErrorString(e_), \
                         __FILE__, __LINE__, #expr));                                     \
  } while (0)
#define SH_RC(expr)                        \
  do {                                     \
    int rc_ = (expr);                      \
    if (rc_ != PMM_OK) return finish(rc_); \
  } while (0)
  for (auto &p : dps) {
    SH_TRY(hipSetDevice(p.dev));
    SH_RC(upload_padded(p.base + p.off_q, q, m, d, dp, 8, p.s));
  }
  // per shard: rows, f64 top-k with global indices (every device at once:
  // the overflow flags are copied, not waited for)
  auto run_shard = [&](int g, bool materialised) -> int {
    Dev64 &p = dps[plan_of[g]];
    const ShardSrc64 &x = sh[g];
    const double *c = x.dev_rows;
    if (x.host) c = (const double *)(p.base + off_c[g]);
    uint32_t *li = (uint32_t *)(p.base + off_li[g]);
    double *ls = (double *)(p.base + off_ls[g]);
    uint32_t *oi = li;
    double *os = ls;
    if (kg[g] < k) {
      // a shard shorter than k: its kg best into a compact list, then into
      // the [m][k] rows behind empty slots (idx 0xFFFFFFFF, score NaN)
      oi = (uint32_t *)(p.base + off_tmp[g]);
      os = (double *)(oi + (size_t)m * kg[g]);
      HIP_TRY(hipMemsetAsync(li, 0xFF, (size_t)m * k * 4, p.s));
      HIP_TRY(hipMemsetAsync(ls, 0xFF, (size_t)m * k * 8, p.s));  // (all-ones f64: a NaN)
    }
    unsigned *flag = (unsigned *)(p.base + p.off_flags) + slot[g];
    int rc = materialised ? topk_f64_materialised((const double *)(p.base + p.off_q), dp, m, c, dp, x.rows, d,
                                                  kg[g], metric, (uint32_t)x.lo, oi, os, p.base + p.off_ws, p.s,
                                                  x.dev_norms)
                          : topk_f64_device_impl((const double *)(p.base + p.off_q), dp, m, c, dp, x.rows, d, kg[g],
                                                 metric, (uint32_t)x.lo, oi, os, p.base + p.off_ws, p.s, fused[g],
                                                 x.dev_norms, fused[g] ? flag : nullptr);
    if (rc) return rc;
    if (kg[g] < k) {
      HIP_TRY(hipMemcpy2DAsync(li, (size_t)k * 4, oi, (size_t)kg[g] * 4, (size_t)kg[g] * 4, (size_t)m,
                               hipMemcpyDeviceToDevice, p.s));
      HIP_TRY(hipMemcpy2DAsync(ls, (size_t)k * 8, os, (size_t)kg[g] * 8, (size_t)kg[g] * 8, (size_t)m,
                               hipMemcpyDeviceToDevice, p.s));
    }
    return PMM_OK;
  };
  for (int g = 0; g < G; g++) {
    Dev64 &p = dps[plan_of[g]];
    SH_TRY(hipSetDevice(p.dev));
    if (sh[g].host) SH_RC(upload_padded(p.base + off_c[g], sh[g].host, sh[g].rows, d, dp, 8, p.s));
    SH_TRY(hipMemsetAsync((unsigned *)(p.base + p.off_flags) + slot[g], 0, 4, p.s));
    SH_RC(run_shard(g, false));
  }
  // overflow flags, once every device is done: an overflowed shard re-runs
  // on the materialised path (its rows, its workspace)
  for (auto &p : dps) {
    SH_TRY(hipSetDevice(p.dev));
    SH_TRY(hipStreamSynchronize(p.s));
  }
  for (int g = 0; g < G; g++) {
    Dev64 &p = dps[plan_of[g]];
    SH_TRY(hipSetDevice(p.dev));
    if (fused[g]) {
      unsigned of = 0;
      SH_TRY(hipMemcpy(&of, (unsigned *)(p.base + p.off_flags) + slot[g], 4, hipMemcpyDeviceToHost));
      if (of) SH_RC(run_shard(g, true));
    }
    SH_TRY(hipEventCreateWithFlags(&ev[g], hipEventDisableTiming));
    SH_TRY(hipEventRecord(ev[g], p.s));
  }
  // gather into the root (peer copies over xGMI), merge, download
  SH_TRY(hipSetDevice(root));
  uint32_t *gi = (uint32_t *)(rp.base + off_gi);
  double *gs = (double *)(rp.base + off_gs);
  for (int g = 0; g < G; g++) {
    enable_peer(root, sh[g].dev);
    SH_TRY(hipStreamWaitEvent(rp.s, ev[g], 0));
    const char *pb = dps[plan_of[g]].base;
    SH_TRY(hipMemcpyPeerAsync(gi + (size_t)g * m * k, root, pb + off_li[g], sh[g].dev, (size_t)m * k * 4, rp.s));
    SH_TRY(hipMemcpyPeerAsync(gs + (size_t)g * m * k, root, pb + off_ls[g], sh[g].dev, (size_t)m * k * 8, rp.s));
  }
  F64MergeArgs ma{};
  ma.gi = gi;
  ma.gs = gs;
  ma.list_stride = m * k;
  ma.M = (int)m;
  ma.G = G;
  ma.k = (int)k;
  ma.metric = metric;
  ma.out_idx = (uint32_t *)(rp.base + off_oi);
  ma.out_score = (double *)(rp.base + off_os);
  {
    Timed t("merge_devices_f64", rp.s);
    SH_TRY(launch_f64_merge(ma, rp.s));
  }
  SH_TRY(hipMemcpyAsync(out_idx, ma.out_idx, (size_t)m * k * 4, hipMemcpyDeviceToHost, rp.s));
  SH_TRY(hipMemcpyAsync(out_score, ma.out_score, (size_t)m * k * 8, hipMemcpyDeviceToHost, rp.s));
  SH_TRY(hipStreamSynchronize(rp.s));
#undef SH_TRY
#undef SH_RC
  return finish(PMM_OK);
}

std::vector<int> devices_snapshot() {
  std::lock_guard<std::mutex> lk(g_devs_mu);
  return g_devs;
}

// The device host entry points run on when a device list is set: its first
// entry (the root, which also merges a sharded search), else -1 (the thread's
// pmm_set_device choice or the current device).  A one-entry list therefore
// moves all host work to that device; work that is not sharded (f32 k > 1024,
// .pmm.matmul) runs on the root of a longer list.
int list_root() {
  std::lock_guard<std::mutex> lk(g_devs_mu);
  return g_devs.empty() ? -1 : g_devs[0];
}

// shard g of n rows over G shards: rows [n g / G, n (g + 1) / G)
int64_t shard_lo(int64_t n, int G, int g) { return n * g / G; }

}  // namespace

// Device-resident corpus (pmm_corpus_*): padded f32 rows in HBM plus the
// norms / pre-filter factors of every metric, computed once at creation.
// With a device list set (pmm_set_devices) the rows are sharded over the
// devices at creation, one contiguous shard each.
// A Float64 corpus (pmm_corpus_create_f64; Polars' default float columns
// take the reference's f64 branch, src/matmul.rs:449-468) keeps its rows in
// f64 with the f64 norms of both metrics, sharded over a device list the same
// way (round 6).
struct CorpusShard {
  int device = 0;
  int64_t lo = 0, n = 0;       // rows [lo, lo + n) of the corpus
  float *data = nullptr;       // f32: n x dp
  float *norms = nullptr;      // f32: [cosine: n norms | n 1/norm][euclid: n sq | n sq*(1-2^-18)]
  double *data64 = nullptr;    // f64: n x dp
  double *norms64 = nullptr;   // f64: [cosine: n norms][euclid: n sq]
};
struct pmm_corpus {
  int64_t n = 0, d = 0, dp = 0;
  int dtype = PMM_DTYPE_F32;
  std::vector<CorpusShard> shards;
};

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

const char *pmm_version(void) { return kVersion; }

const char *pmm_last_error(void) { return t_err.c_str(); }

int pmm_metric_from_str(const char *s, int *metric) {
  if (!s || !metric) return fail(PMM_ERR_ARG, "null argument");
  std::string l(s);
  for (auto &ch : l) ch = (char)tolower((unsigned char)ch);
  if (l == "cosine") *metric = PMM_METRIC_COSINE;
  else if (l == "dot") *metric = PMM_METRIC_DOT;
  else if (l == "euclidean" || l == "l2") *metric = PMM_METRIC_EUCLIDEAN;
  else return fail(PMM_ERR_ARG, "Unknown metric: '%s'. Supported: cosine, dot, euclidean", s);
  return PMM_OK;
}

int pmm_metric_higher_is_better(int metric) { return metric != PMM_METRIC_EUCLIDEAN; }

int pmm_device_count(int *count) {
  if (!count) return fail(PMM_ERR_ARG, "null argument");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  *count = n;
  return PMM_OK;
}

int pmm_device_memory(size_t *free_bytes, size_t *total_bytes) {
  if (!free_bytes || !total_bytes) return fail(PMM_ERR_ARG, "null argument");
  int dev, rc;
  DevScope scope;
  if ((rc = ensure_device(&dev, &scope, list_root()))) return rc;
  HIP_TRY(hipMemGetInfo(free_bytes, total_bytes));
  return PMM_OK;
}

int pmm_set_device(int device) {
  int n = 0;
  pmm_device_count(&n);
  if (device < 0 || device >= n) return fail(PMM_ERR_NODEVICE, "no HIP device %d (%d visible)", device, n);
  HIP_TRY(hipSetDevice(device));
  t_ctx.device = device;
  return PMM_OK;
}

int pmm_host_alloc(size_t bytes, void **out) {
  if (!out) return fail(PMM_ERR_ARG, "null argument");
  *out = nullptr;
  if (bytes == 0) return PMM_OK;
  HIP_TRY(hipHostMalloc(out, bytes, hipHostMallocPortable));
  return PMM_OK;
}

int pmm_host_free(void *p) {
  if (p) HIP_TRY(hipHostFree(p));
  return PMM_OK;
}

int pmm_set_devices(const int *ids, int n) {
  if (n < 0 || (n > 0 && !ids)) return fail(PMM_ERR_ARG, "bad device list (n=%d)", n);
  int count = 0;
  pmm_device_count(&count);
  for (int i = 0; i < n; i++)
    if (ids[i] < 0 || ids[i] >= count || ids[i] >= kMaxDevices)
      return fail(PMM_ERR_NODEVICE, "no HIP device %d (%d visible)", ids[i], count);
  for (int i = 0; i < n; i++)
    if (int rc = probe_device(ids[i])) return rc;
  std::lock_guard<std::mutex> lk(g_devs_mu);
  g_devs.assign(ids, ids + n);
  return PMM_OK;
}

int pmm_shard_plan(const int *devs, int G, int64_t m, int64_t n, int64_t d, int64_t k, int metric, int compute,
                   int host_rows, int *plan_of, int *plan_dev, uint64_t *plan_bytes, uint64_t *list_offsets,
                   int *n_plans) {
  if (!devs || G < 1 || !plan_of || !plan_dev || !plan_bytes || !list_offsets || !n_plans)
    return fail(PMM_ERR_ARG, "null argument or empty device list");
  if (m < 1 || n < G || d < 1 || k < 1 || k > kFusedMaxK)
    return fail(PMM_ERR_ARG, "bad sizes (m=%lld n=%lld G=%d d=%lld k=%lld)", (long long)m, (long long)n, G,
                (long long)d, (long long)k);
  static const float kHostTag = 0.0f;  // any non-null host pointer: rows are uploaded
  std::vector<ShardSrc> sh(G);
  for (int g = 0; g < G; g++) {
    const int64_t lo = shard_lo(n, G, g), hi = shard_lo(n, G, g + 1);
    sh[g] = ShardSrc{devs[g], lo, hi - lo, host_rows ? &kHostTag : nullptr, nullptr, nullptr};
  }
  ShardLayout L;
  plan_sharded(sh, m, d, k, metric, compute, L);
  *n_plans = (int)L.dps.size();
  for (int j = 0; j < (int)L.dps.size(); j++) {
    plan_dev[j] = L.dps[j].dev;
    plan_bytes[j] = L.dps[j].total;
  }
  for (int g = 0; g < G; g++) {
    plan_of[g] = L.plan_of[g];
    list_offsets[g] = L.off_list[g];
  }
  return PMM_OK;
}

int pmm_get_devices(int *ids, int cap, int *n) {
  if (!n || cap < 0 || (cap > 0 && !ids)) return fail(PMM_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> lk(g_devs_mu);
  *n = (int)g_devs.size();
  for (int i = 0; i < (int)g_devs.size() && i < cap; i++) ids[i] = g_devs[i];
  return PMM_OK;
}

size_t pmm_topk_workspace_bytes(int64_t m, int64_t n, int64_t d, int64_t k, int metric,
                                int compute) {
  int cus = 256;
  int dev = 0;
  if (hipGetDevice(&dev) == hipSuccess) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    if (dev >= 0 && dev < kMaxDevices && g_dev[dev].probed) cus = g_dev[dev].cus;
  }
  if (compute == PMM_COMPUTE_BF16) {
    if (!bf16_native(d, k, n)) return bf16_widened_bytes(m, n, d, k, metric, cus);
    Plan p;
    plan_topk(m, n, d, k, metric, cus, p, PMM_COMPUTE_BF16);
    return p.total;
  }
  if (k <= kFusedMaxK) {
    Plan p;
    plan_topk(m, n, d, k, metric, cus, p);
    return p.total;
  }
  MatPlan p;
  plan_materialise(m, n, k, 4, p);
  return p.total;
}

int pmm_topk_merge_bytes(const void *workspace, int64_t m, int64_t n, int64_t d, int64_t k,
                         int metric, int compute, uint64_t *bytes) {
  if (!bytes) return fail(PMM_ERR_ARG, "null output");
  *bytes = 0;
  if (m <= 0 || k <= 0) return PMM_OK;
  if (compute != PMM_COMPUTE_BF16 && k > kFusedMaxK)
    return fail(PMM_ERR_UNSUPPORTED, "no merge pass on the materialised path (k > %d)", kFusedMaxK);
  int dev;
  int rc = ensure_device(&dev);
  if (rc) return rc;
  int cus = 256;
  {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    if (dev >= 0 && dev < kMaxDevices && g_dev[dev].probed) cus = g_dev[dev].cus;
  }
  Plan p;
  plan_topk(m, n, d, k, metric, cus, p, compute);
  // the merge reads every row's split counts and shared threshold, the
  // candidates the GEMM left, and writes the m x k (index, score) lists
  std::vector<unsigned> cnt((size_t)m * p.segs);
  HIP_TRY(hipMemcpy(cnt.data(), (const char *)workspace + p.off_cnt, cnt.size() * 4,
                    hipMemcpyDeviceToHost));
  uint64_t cands = 0;
  for (unsigned c : cnt) cands += std::min<unsigned>(c, (unsigned)p.capg);
  *bytes = (uint64_t)m * p.segs * 4 + cands * 8 + (uint64_t)m * 8 + (uint64_t)m * k * 8;
  return PMM_OK;
}

int pmm_topk_f32_device(const float *q, int64_t ldq, int64_t m, const float *c, int64_t ldc,
                        int64_t n, int64_t d, int64_t k, int metric, int compute,
                        uint32_t index_base, uint32_t *out_idx, float *out_score, void *workspace,
                        size_t workspace_bytes, void *stream) {
  // a corpus shard may hold fewer than k rows: the fused path pads with empty
  // slots (index 0xFFFFFFFF, score NaN), which the shard merge skips
  int rc = validate_sizes(m, n, d, k, true, k <= kFusedMaxK);
  if (rc) return rc;
  if ((rc = check_metric(metric))) return rc;
  if (compute == PMM_COMPUTE_BF16)
    return fail(PMM_ERR_UNSUPPORTED,
                "device f32 inputs with bf16 compute: convert to bf16 and call pmm_topk_bf16_device");
  if (compute != PMM_COMPUTE_F32)
    return fail(PMM_ERR_UNSUPPORTED, "unknown compute mode %d", compute);
  if (m == 0 || k == 0) return PMM_OK;
  if (n == 0) return fail(PMM_ERR_ARG, "Empty series");
  if ((rc = need_buffers(q, c, out_idx, out_score))) return rc;
  const int64_t dp = cdiv(d, 32) * 32;
  if (d == 0 || ldq % 4 != 0 || ldc % 4 != 0 || ldq < dp || ldc < dp || ((uintptr_t)q & 15) ||
      ((uintptr_t)c & 15))
    return fail(PMM_ERR_ARG,
                "device inputs need row strides >= roundup(d, 32) (zero-padded), multiples of 4, "
                "16-byte-aligned bases (d=%lld ldq=%lld ldc=%lld)",
                (long long)d, (long long)ldq, (long long)ldc);
  int dev;
  if ((rc = ensure_device(&dev))) return rc;
  hipStream_t s = (hipStream_t)stream;  // NULL = the HIP default stream
  return topk_f32_device_impl(q, ldq, m, c, ldc, n, d, k, metric, index_base, out_idx, out_score,
                              workspace, workspace_bytes, s, dev);
}

int pmm_topk_f32_ex(const float *q, int64_t m, const float *c, int64_t n, int64_t d, int64_t k,
                    int metric, int compute, uint32_t *out_idx, float *out_score) {
  int rc = validate_sizes(m, n, d, k, true);
  if (rc) return rc;
  if ((rc = check_metric(metric))) return rc;
  if (compute != PMM_COMPUTE_F32 && compute != PMM_COMPUTE_BF16)
    return fail(PMM_ERR_UNSUPPORTED, "unknown compute mode %d", compute);
  if (m == 0 || k == 0) return PMM_OK;
  if (n == 0) return fail(PMM_ERR_ARG, "Empty series");
  if (d == 0) return fail(PMM_ERR_ARG, "Zero-dimensional vectors");
  if ((rc = need_buffers(q, c, out_idx, out_score))) return rc;
  {
    // a device list (pmm_set_devices): the corpus row-sharded over it, one
    // shard per listed device (at most n shards), results merged on the first
    const std::vector<int> devs = devices_snapshot();
    if (devs.size() > 1 && k <= kFusedMaxK) {
      const int G = (int)std::min<int64_t>((int64_t)devs.size(), n);
      std::vector<ShardSrc> sh(G);
      for (int g = 0; g < G; g++) {
        const int64_t lo = shard_lo(n, G, g), hi = shard_lo(n, G, g + 1);
        sh[g] = ShardSrc{devs[g], lo, hi - lo, c + lo * d, nullptr, nullptr};
      }
      return topk_sharded(q, m, d, k, metric, compute, sh, out_idx, out_score);
    }
  }
  int dev;
  DevScope scope;
  if ((rc = ensure_device(&dev, &scope, list_root()))) return rc;
  hipStream_t s;
  if ((rc = thread_stream(dev, &s))) return rc;
  if (compute == PMM_COMPUTE_BF16) {
    // f32 rows uploaded as they are, rounded to zero-padded bf16 rows on device
    const int64_t db = cdiv(d, kBf16DAlign) * kBf16DAlign;
    size_t ws_need = pmm_topk_workspace_bytes(m, n, db, k, metric, compute);
    size_t off_qf = 0, off_cf = al256((size_t)m * d * 4);
    size_t off_qb = off_cf + al256((size_t)n * d * 4), off_cb = off_qb + al256((size_t)m * db * 2);
    size_t off_i = off_cb + al256((size_t)n * db * 2), off_s = off_i + al256((size_t)m * k * 4);
    size_t off_w = off_s + al256((size_t)m * k * 4);
    void *base;
    if ((rc = arena(dev, s, off_w + ws_need, &base))) return rc;
    char *b = (char *)base;
    HIP_TRY(hipMemcpyAsync(b + off_qf, q, (size_t)m * d * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(b + off_cf, c, (size_t)n * d * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(launch_f32_to_bf16((const float *)(b + off_qf), m, d, d, (uint16_t *)(b + off_qb), db, s));
    HIP_TRY(launch_f32_to_bf16((const float *)(b + off_cf), n, d, d, (uint16_t *)(b + off_cb), db, s));
    rc = topk_bf16_device_impl((const uint16_t *)(b + off_qb), db, m, (const uint16_t *)(b + off_cb),
                               db, n, d, k, metric, 0u, (uint32_t *)(b + off_i),
                               (float *)(b + off_s), b + off_w, ws_need, s, dev);
    if (rc) return rc;
    {
      Timed t("d2h", s);
      HIP_TRY(hipMemcpyAsync(out_idx, b + off_i, (size_t)m * k * 4, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipMemcpyAsync(out_score, b + off_s, (size_t)m * k * 4, hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    return PMM_OK;
  }
  const int64_t dp = cdiv(d, 32) * 32;
  {
    const char *ce = getenv("PMM_CHUNKED_UPLOAD");  // 0: one upload, then one launch
    if (k <= kFusedMaxK && (size_t)n * dp * 4 >= kChunkedMinBytes && n >= 64 * k && !(ce && atoi(ce) == 0))
      return topk_f32_host_chunked(q, m, c, n, d, k, metric, out_idx, out_score, dev, s);
  }
  size_t ws_need = pmm_topk_workspace_bytes(m, n, dp, k, metric, compute);
  size_t off_q = 0, off_c = al256((size_t)m * dp * 4), off_i = off_c + al256((size_t)n * dp * 4);
  size_t off_s = off_i + al256((size_t)m * k * 4), off_w = off_s + al256((size_t)m * k * 4);
  void *base;
  if ((rc = arena(dev, s, off_w + ws_need, &base))) return rc;
  char *b = (char *)base;
  if ((rc = upload_padded(b + off_q, q, m, d, dp, 4, s))) return rc;
  if ((rc = upload_padded(b + off_c, c, n, d, dp, 4, s))) return rc;
  rc = topk_f32_device_impl((const float *)(b + off_q), dp, m, (const float *)(b + off_c), dp, n,
                            d, k, metric, 0u, (uint32_t *)(b + off_i), (float *)(b + off_s),
                            b + off_w, ws_need, s, dev);
  if (rc) return rc;
  {
    Timed t("d2h", s);
    HIP_TRY(hipMemcpyAsync(out_idx, b + off_i, (size_t)m * k * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(out_score, b + off_s, (size_t)m * k * 4, hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(hipStreamSynchronize(s));
  return PMM_OK;
}

int pmm_topk_bf16_device(const uint16_t *q, int64_t ldq, int64_t m, const uint16_t *c,
                         int64_t ldc, int64_t n, int64_t d, int64_t k, int metric,
                         uint32_t index_base, uint32_t *out_idx, float *out_score,
                         void *workspace, size_t workspace_bytes, void *stream) {
  // (k > n only where the fused path pads short lists, as for f32)
  int rc = validate_sizes(m, n, d, k, true, k <= kFusedMaxK);
  if (rc) return rc;
  if ((rc = check_metric(metric))) return rc;
  if (m == 0 || k == 0) return PMM_OK;
  if (n == 0) return fail(PMM_ERR_ARG, "Empty series");
  if (d == 0) return fail(PMM_ERR_ARG, "Zero-dimensional vectors");
  if ((rc = need_buffers(q, c, out_idx, out_score))) return rc;
  const int64_t dp = cdiv(d, kBf16DAlign) * kBf16DAlign;
  if (ldq % 8 != 0 || ldc % 8 != 0 || ldq < dp || ldc < dp || ((uintptr_t)q & 15) ||
      ((uintptr_t)c & 15))
    return fail(PMM_ERR_ARG,
                "bf16 device inputs need row strides >= roundup(d, 128) (zero-padded), multiples "
                "of 8, 16-byte-aligned bases (d=%lld ldq=%lld ldc=%lld)",
                (long long)d, (long long)ldq, (long long)ldc);
  int dev;
  if ((rc = ensure_device(&dev))) return rc;
  hipStream_t s = (hipStream_t)stream;  // NULL = the HIP default stream
  return topk_bf16_device_impl(q, ldq, m, c, ldc, n, d, k, metric, index_base, out_idx, out_score,
                               workspace, workspace_bytes, s, dev);
}

int pmm_topk_f32(const float *q, int64_t m, const float *c, int64_t n, int64_t d, int64_t k,
                 int metric, uint32_t *out_idx, float *out_score) {
  return pmm_topk_f32_ex(q, m, c, n, d, k, metric, PMM_COMPUTE_F32, out_idx, out_score);
}

int pmm_topk_f64(const double *q, int64_t m, const double *c, int64_t n, int64_t d, int64_t k,
                 int metric, uint32_t *out_idx, double *out_score) {
  int rc = validate_sizes(m, n, d, k, true);
  if (rc) return rc;
  if ((rc = check_metric(metric))) return rc;
  if (m == 0 || k == 0) return PMM_OK;
  if (n == 0) return fail(PMM_ERR_ARG, "Empty series");
  if (d == 0) return fail(PMM_ERR_ARG, "Zero-dimensional vectors");
  if ((rc = need_buffers(q, c, out_idx, out_score))) return rc;
  {
    // a device list (pmm_set_devices): the corpus row-sharded over it, as the
    // f32 path does (topk_sharded_f64)
    const std::vector<int> devs = devices_snapshot();
    if (devs.size() > 1 && n > 1) {
      const int G = (int)std::min<int64_t>((int64_t)devs.size(), n);
      std::vector<ShardSrc64> sh(G);
      for (int g = 0; g < G; g++) {
        const int64_t lo = shard_lo(n, G, g), hi = shard_lo(n, G, g + 1);
        sh[g] = ShardSrc64{devs[g], lo, hi - lo, c + lo * d, nullptr, nullptr};
      }
      return topk_sharded_f64(q, m, d, k, metric, sh, out_idx, out_score);
    }
  }
  int dev;
  DevScope scope;
  if ((rc = ensure_device(&dev, &scope, list_root()))) return rc;
  hipStream_t s;
  if ((rc = thread_stream(dev, &s))) return rc;
  const int64_t dp = cdiv(d, 16) * 16;
  size_t off_q = 0, off_c = al256((size_t)m * dp * 8), off_i = off_c + al256((size_t)n * dp * 8);
  size_t off_s = off_i + al256((size_t)m * k * 4), off_w = off_s + al256((size_t)m * k * 8);
  void *base;
  const bool fused = f64_use_fused(m, n, k);
  if ((rc = arena(dev, s, off_w + f64_workspace_bytes(m, n, k, fused), &base))) return rc;
  char *b = (char *)base;
  const double *dq = (const double *)(b + off_q), *dc = (const double *)(b + off_c);
  if ((rc = upload_padded(b + off_q, q, m, d, dp, 8, s))) return rc;
  if ((rc = upload_padded(b + off_c, c, n, d, dp, 8, s))) return rc;
  uint32_t *oi = (uint32_t *)(b + off_i);
  double *os = (double *)(b + off_s);
  if ((rc = topk_f64_device_impl(dq, dp, m, dc, dp, n, d, k, metric, 0u, oi, os, b + off_w, s, fused))) return rc;
  {
    Timed t("d2h", s);
    HIP_TRY(hipMemcpyAsync(out_idx, oi, (size_t)m * k * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(out_score, os, (size_t)m * k * 8, hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(hipStreamSynchronize(s));
  return PMM_OK;
}

int pmm_topk_f64_device(const double *q, int64_t ldq, int64_t m, const double *c, int64_t ldc, int64_t n,
                        int64_t d, int64_t k, int metric, uint32_t index_base, uint32_t *out_idx,
                        double *out_score, void *stream) {
  int rc = validate_sizes(m, n, d, k, true);
  if (rc) return rc;
  if ((rc = check_metric(metric))) return rc;
  if (m == 0 || k == 0) return PMM_OK;
  if (n == 0) return fail(PMM_ERR_ARG, "Empty series");
  if ((rc = need_buffers(q, c, out_idx, out_score))) return rc;
  const int64_t dp = cdiv(d, 16) * 16;
  if (d == 0 || ldq < dp || ldc < dp || ((uintptr_t)q & 15) || ((uintptr_t)c & 15))
    return fail(PMM_ERR_ARG,
                "device f64 inputs need row strides >= roundup(d, 16) (zero-padded) and 16-byte-aligned "
                "bases (d=%lld ldq=%lld ldc=%lld)",
                (long long)d, (long long)ldq, (long long)ldc);
  int dev;
  if ((rc = ensure_device(&dev))) return rc;
  hipStream_t s = (hipStream_t)stream;
  void *w;
  const bool fused = f64_use_fused(m, n, k);
  if ((rc = arena(dev, s, f64_workspace_bytes(m, n, k, fused), &w))) return rc;
  rc = topk_f64_device_impl(q, ldq, m, c, ldc, n, d, k, metric, index_base, out_idx, out_score, (char *)w, s, fused);
  if (rc) return rc;
  return arena_record(dev, s);
}

int pmm_matmul_f32(const float *q, int64_t m, const float *c, int64_t n, int64_t d, float *out) {
  int rc = validate_sizes(m, n, d, 0, false);
  if (rc) return rc;
  if (m == 0 || n == 0) return PMM_OK;
  if ((rc = need_buffers(q, c, out))) return rc;
  int dev;
  DevScope scope;
  if ((rc = ensure_device(&dev, &scope, list_root()))) return rc;
  hipStream_t s;
  if ((rc = thread_stream(dev, &s))) return rc;
  const int64_t dp = cdiv(std::max<int64_t>(d, 1), 32) * 32;
  const int64_t rows_chunk =
      std::max<int64_t>(1, std::min<int64_t>(m, (int64_t)(kMaterialiseBudget / ((size_t)n * 4))));
  size_t off_q = 0, off_c = al256((size_t)m * dp * 4), off_o = off_c + al256((size_t)n * dp * 4);
  size_t off_cnt = off_o + al256((size_t)rows_chunk * n * 4);
  void *base;
  if ((rc = arena(dev, s, off_cnt + 256, &base))) return rc;
  char *b = (char *)base;
  if ((rc = upload_padded(b + off_q, q, m, d, dp, 4, s))) return rc;
  if ((rc = upload_padded(b + off_c, c, n, d, dp, 4, s))) return rc;
  const float *dq = (const float *)(b + off_q), *dc = (const float *)(b + off_c);
  float *dout = (float *)(b + off_o);
  HostPin pin(out, (size_t)m * n * 4);
  for (int64_t r0 = 0; r0 < m; r0 += rows_chunk) {
    const int64_t rows = std::min<int64_t>(rows_chunk, m - r0);
    rc = gemm_store_f32(dq + r0 * dp, dp, rows, dc, dp, n, dp, kMetricDot, 0, nullptr, nullptr,
                        dout, n, (unsigned *)(b + off_cnt), g_dev[dev].cus, s);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(out + r0 * n, dout, (size_t)rows * n * 4, hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(hipStreamSynchronize(s));
  return PMM_OK;
}

int pmm_matmul_f64(const double *q, int64_t m, const double *c, int64_t n, int64_t d,
                   double *out) {
  int rc = validate_sizes(m, n, d, 0, false);
  if (rc) return rc;
  if (m == 0 || n == 0) return PMM_OK;
  if ((rc = need_buffers(q, c, out))) return rc;
  int dev;
  DevScope scope;
  if ((rc = ensure_device(&dev, &scope, list_root()))) return rc;
  hipStream_t s;
  if ((rc = thread_stream(dev, &s))) return rc;
  const int64_t dp = cdiv(std::max<int64_t>(d, 1), 16) * 16;
  const int64_t rows_chunk =
      std::max<int64_t>(1, std::min<int64_t>(m, (int64_t)(kMaterialiseBudget / ((size_t)n * 8))));
  size_t off_q = 0, off_c = al256((size_t)m * dp * 8), off_o = off_c + al256((size_t)n * dp * 8);
  void *base;
  if ((rc = arena(dev, s, off_o + al256((size_t)rows_chunk * n * 8), &base))) return rc;
  char *b = (char *)base;
  if ((rc = upload_padded(b + off_q, q, m, d, dp, 8, s))) return rc;
  if ((rc = upload_padded(b + off_c, c, n, d, dp, 8, s))) return rc;
  const double *dq = (const double *)(b + off_q), *dc = (const double *)(b + off_c);
  double *dout = (double *)(b + off_o);
  HostPin pin(out, (size_t)m * n * 8);
  for (int64_t r0 = 0; r0 < m; r0 += rows_chunk) {
    const int64_t rows = std::min<int64_t>(rows_chunk, m - r0);
    {
      Timed t("gemm_f64_matmul", s);
      HIP_TRY(launch_gemm_f64_store(dq + r0 * dp, dp, dc, dp, nullptr, nullptr, (int)rows, (int)n,
                                    (int)dp, kMetricDot, 0, dout, n, s));
    }
    HIP_TRY(hipMemcpyAsync(out + r0 * n, dout, (size_t)rows * n * 8, hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(hipStreamSynchronize(s));
  return PMM_OK;
}

int pmm_norms_f32_device(const float *a, int64_t ld, int64_t rows, int64_t d, int squared,
                         float *out, void *stream) {
  if (rows < 0 || d < 0 || ld < d) return fail(PMM_ERR_ARG, "bad norm sizes (rows=%lld d=%lld ld=%lld)",
                                                (long long)rows, (long long)d, (long long)ld);
  if (rows == 0) return PMM_OK;
  int dev, rc;
  if ((rc = ensure_device(&dev))) return rc;
  HIP_TRY(launch_norms_f32(a, rows, d, ld, squared ? 1 : 0, out, nullptr, (hipStream_t)stream));
  return PMM_OK;
}

int pmm_norms_f64_device(const double *a, int64_t ld, int64_t rows, int64_t d, int squared,
                         double *out, void *stream) {
  if (rows < 0 || d < 0 || ld < d) return fail(PMM_ERR_ARG, "bad norm sizes (rows=%lld d=%lld ld=%lld)",
                                                (long long)rows, (long long)d, (long long)ld);
  if (rows == 0) return PMM_OK;
  int dev, rc;
  if ((rc = ensure_device(&dev))) return rc;
  HIP_TRY(launch_norms_f64(a, rows, d, ld, squared ? 1 : 0, out, (hipStream_t)stream));
  return PMM_OK;
}

int pmm_merge_topk_device(const uint32_t *idx, const float *score, int64_t m, int64_t lists,
                          int64_t k_in, int64_t k_out, int metric, uint32_t *out_idx,
                          float *out_score, void *stream) {
  return pmm_merge_topk_strided_device(idx, score, m, lists, k_in, lists * k_in, k_in, k_out, metric,
                                       out_idx, out_score, stream);
}

static int merge_strided(const uint32_t *idx, const float *score, int64_t m, int64_t lists, int64_t k_in,
                         int64_t row_stride, int64_t list_stride, int64_t k_out, int metric, uint32_t *out_idx,
                         float *out_score, void *stream, bool sorted);

int pmm_merge_topk_strided_device(const uint32_t *idx, const float *score, int64_t m,
                                  int64_t lists, int64_t k_in, int64_t row_stride,
                                  int64_t list_stride, int64_t k_out, int metric,
                                  uint32_t *out_idx, float *out_score, void *stream) {
  return merge_strided(idx, score, m, lists, k_in, row_stride, list_stride, k_out, metric, out_idx, out_score,
                       stream, false);
}

int pmm_merge_sorted_topk_strided_device(const uint32_t *idx, const float *score, int64_t m,
                                         int64_t lists, int64_t k_in, int64_t row_stride,
                                         int64_t list_stride, int64_t k_out, int metric,
                                         uint32_t *out_idx, float *out_score, void *stream) {
  return merge_strided(idx, score, m, lists, k_in, row_stride, list_stride, k_out, metric, out_idx, out_score,
                       stream, true);
}

static int merge_strided(const uint32_t *idx, const float *score, int64_t m, int64_t lists, int64_t k_in,
                         int64_t row_stride, int64_t list_stride, int64_t k_out, int metric, uint32_t *out_idx,
                         float *out_score, void *stream, bool sorted) {
  int rc;
  if ((rc = check_metric(metric))) return rc;
  if (m < 0 || lists < 1 || k_in < 0 || k_out < 0 || k_out > lists * k_in || row_stride < 0 ||
      list_stride < 0)
    return fail(PMM_ERR_ARG, "bad merge sizes (m=%lld lists=%lld k_in=%lld k_out=%lld)",
                (long long)m, (long long)lists, (long long)k_in, (long long)k_out);
  if (k_out > kFusedMaxK) return fail(PMM_ERR_UNSUPPORTED, "merge k_out > %d", kFusedMaxK);
  if (m == 0 || k_out == 0) return PMM_OK;
  int dev;
  if ((rc = ensure_device(&dev))) return rc;
  hipStream_t s = (hipStream_t)stream;  // NULL = the HIP default stream
  MergeArgs ma{};
  ma.in_idx = idx;
  ma.in_score = score;
  ma.k_in = (int)k_in;
  ma.row_stride = row_stride;
  ma.list_stride = list_stride;
  ma.M = (int)m;
  ma.S = (int)lists;
  ma.sorted = sorted ? 1 : 0;
  ma.k_out = (int)k_out;
  ma.P = std::min(8192, next_pow2(2 * (int)k_out + 64, 128));
  ma.metric = metric;
  ma.out_idx = out_idx;
  ma.out_score = out_score;
  Timed t("merge_shards", s);
  HIP_TRY(launch_merge(ma, 1, s));
  return PMM_OK;
}

int pmm_corpus_create_f32(const float *c, int64_t n, int64_t d, pmm_corpus **out) {
  if (!out) return fail(PMM_ERR_ARG, "null argument");
  *out = nullptr;
  int rc = validate_sizes(0, n, d, 0, false);
  if (rc) return rc;
  if (n == 0) return fail(PMM_ERR_ARG, "Empty series");
  if (d == 0) return fail(PMM_ERR_ARG, "Zero-dimensional vectors");
  if (!c) return fail(PMM_ERR_ARG, "null argument");
  int dev;
  DevScope scope;
  if ((rc = ensure_device(&dev, &scope, list_root()))) return rc;
  std::vector<int> devs = devices_snapshot();
  if (devs.size() <= 1) devs.assign(1, dev);
  const int G = (int)std::min<int64_t>((int64_t)devs.size(), n);
  pmm_corpus *h = new pmm_corpus();
  h->n = n;
  h->d = d;
  h->dp = cdiv(d, 32) * 32;
  h->shards.resize(G);
  for (int g = 0; g < G; g++) {
    CorpusShard &x = h->shards[g];
    x.device = devs[g];
    x.lo = shard_lo(n, G, g);
    x.n = shard_lo(n, G, g + 1) - x.lo;
  }
  for (int g = 0; g < G; g++) {
    CorpusShard &x = h->shards[g];
    hipStream_t s;
    hipError_t e = hipSetDevice(x.device);
    if (e == hipSuccess && (rc = thread_stream(x.device, &s))) {
      pmm_corpus_destroy(h);
      return rc;
    }
    if (e == hipSuccess) e = hipMalloc(&x.data, (size_t)x.n * h->dp * 4);
    if (e == hipSuccess) e = hipMalloc(&x.norms, (size_t)x.n * 4 * 4);
    if (e != hipSuccess) {
      pmm_corpus_destroy(h);
      return fail(PMM_ERR_HIP, "corpus allocation failed on device %d: %s", x.device, hipGetErrorString(e));
    }
    if ((rc = upload_padded(x.data, c + x.lo * d, x.n, d, h->dp, 4, s))) {
      pmm_corpus_destroy(h);
      return rc;
    }
    hipError_t e1 = launch_norms_f32(x.data, x.n, d, h->dp, 0, x.norms, x.norms + x.n, s);
    hipError_t e2 = launch_norms_f32(x.data, x.n, d, h->dp, 1, x.norms + 2 * x.n, x.norms + 3 * x.n, s);
    hipError_t e3 = hipStreamSynchronize(s);
    if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess) {
      pmm_corpus_destroy(h);
      return fail(PMM_ERR_HIP, "corpus norms failed");
    }
  }
  (void)hipSetDevice(dev);
  *out = h;
  return PMM_OK;
}

int pmm_corpus_destroy(pmm_corpus *h) {
  if (!h) return PMM_OK;
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (auto &x : h->shards) {
    if (!x.data && !x.norms && !x.data64 && !x.norms64) continue;
    (void)hipSetDevice(x.device);
    (void)hipDeviceSynchronize();
    if (x.data) (void)hipFree(x.data);
    if (x.norms) (void)hipFree(x.norms);
    if (x.data64) (void)hipFree(x.data64);
    if (x.norms64) (void)hipFree(x.norms64);
  }
  (void)hipSetDevice(cur);
  delete h;
  return PMM_OK;
}

int pmm_corpus_info(const pmm_corpus *h, int64_t *n, int64_t *d, int *device) {
  if (!h) return fail(PMM_ERR_ARG, "null corpus");
  if (n) *n = h->n;
  if (d) *d = h->d;
  if (device) *device = h->shards.empty() ? -1 : h->shards[0].device;
  return PMM_OK;
}

int pmm_corpus_shards(const pmm_corpus *h, int *shards) {
  if (!h || !shards) return fail(PMM_ERR_ARG, "null argument");
  *shards = (int)h->shards.size();
  return PMM_OK;
}

int pmm_corpus_dtype(const pmm_corpus *h, int *dtype) {
  if (!h || !dtype) return fail(PMM_ERR_ARG, "null argument");
  *dtype = h->dtype;
  return PMM_OK;
}

int pmm_corpus_create_f64(const double *c, int64_t n, int64_t d, pmm_corpus **out) {
  if (!out) return fail(PMM_ERR_ARG, "null argument");
  *out = nullptr;
  int rc = validate_sizes(0, n, d, 0, false);
  if (rc) return rc;
  if (n == 0) return fail(PMM_ERR_ARG, "Empty series");
  if (d == 0) return fail(PMM_ERR_ARG, "Zero-dimensional vectors");
  if (!c) return fail(PMM_ERR_ARG, "null argument");
  int dev;
  DevScope scope;
  if ((rc = ensure_device(&dev, &scope, list_root()))) return rc;
  // with a device list the rows are sharded over it, as pmm_corpus_create_f32
  // does (one contiguous shard per listed device, at most n)
  std::vector<int> devs = devices_snapshot();
  if (devs.size() <= 1) devs.assign(1, dev);
  const int G = (int)std::min<int64_t>((int64_t)devs.size(), n);
  pmm_corpus *h = new pmm_corpus();
  h->n = n;
  h->d = d;
  h->dp = cdiv(d, 16) * 16;  // the f64 kernels' K step (pmm_topk_f64_device's stride rule)
  h->dtype = PMM_DTYPE_F64;
  h->shards.resize(G);
  for (int g = 0; g < G; g++) {
    CorpusShard &x = h->shards[g];
    x.device = devs[g];
    x.lo = shard_lo(n, G, g);
    x.n = shard_lo(n, G, g + 1) - x.lo;
  }
  for (int g = 0; g < G; g++) {
    CorpusShard &x = h->shards[g];
    hipStream_t s;
    hipError_t e = hipSetDevice(x.device);
    if (e == hipSuccess && (rc = thread_stream(x.device, &s))) {
      pmm_corpus_destroy(h);
      return rc;
    }
    if (e == hipSuccess) e = hipMalloc(&x.data64, (size_t)x.n * h->dp * 8);
    if (e == hipSuccess) e = hipMalloc(&x.norms64, (size_t)x.n * 2 * 8);
    if (e != hipSuccess) {
      pmm_corpus_destroy(h);
      return fail(PMM_ERR_HIP, "corpus allocation failed on device %d: %s", x.device, hipGetErrorString(e));
    }
    if ((rc = upload_padded(x.data64, c + x.lo * d, x.n, d, h->dp, 8, s))) {
      pmm_corpus_destroy(h);
      return rc;
    }
    // the norms every f64 call would compute (src/metrics.rs:368-379), by the
    // same kernel on the same padded rows: bit-identical to the per-call ones
    hipError_t e1 = launch_norms_f64(x.data64, x.n, d, h->dp, 0, x.norms64, s);
    hipError_t e2 = launch_norms_f64(x.data64, x.n, d, h->dp, 1, x.norms64 + x.n, s);
    hipError_t e3 = hipStreamSynchronize(s);
    if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess) {
      pmm_corpus_destroy(h);
      return fail(PMM_ERR_HIP, "corpus norms failed");
    }
  }
  (void)hipSetDevice(dev);
  *out = h;
  return PMM_OK;
}

int pmm_topk_f64_corpus(const pmm_corpus *h, const double *q, int64_t m, int64_t k, int metric,
                        uint32_t *out_idx, double *out_score) {
  if (!h) return fail(PMM_ERR_ARG, "null corpus");
  if (h->dtype != PMM_DTYPE_F64)
    return fail(PMM_ERR_ARG, "the corpus handle holds f32 rows: use pmm_topk_f32_corpus");
  int rc = validate_sizes(m, h->n, h->d, k, true);
  if (rc) return rc;
  if ((rc = check_metric(metric))) return rc;
  if (m == 0 || k == 0) return PMM_OK;
  if ((rc = need_buffers(q, out_idx, out_score))) return rc;
  if (h->shards.size() > 1) {
    std::vector<ShardSrc64> sh(h->shards.size());
    for (size_t g = 0; g < sh.size(); g++) {
      const CorpusShard &x = h->shards[g];
      const double *cn = metric == kMetricCosine ? x.norms64 : metric == kMetricEuclidean ? x.norms64 + x.n : nullptr;
      sh[g] = ShardSrc64{x.device, x.lo, x.n, nullptr, x.data64, cn};
    }
    return topk_sharded_f64(q, m, h->d, k, metric, sh, out_idx, out_score);
  }
  const CorpusShard &x = h->shards[0];
  int dev;
  DevScope scope;
  if ((rc = ensure_device(&dev, &scope, x.device))) return rc;
  hipStream_t s;
  if ((rc = thread_stream(dev, &s))) return rc;
  const int64_t dp = h->dp, n = h->n;
  const bool fused = f64_use_fused(m, n, k);
  size_t off_q = 0, off_i = al256((size_t)m * dp * 8);
  size_t off_s = off_i + al256((size_t)m * k * 4), off_w = off_s + al256((size_t)m * k * 8);
  void *base;
  if ((rc = arena(dev, s, off_w + f64_workspace_bytes(m, n, k, fused), &base))) return rc;
  char *b = (char *)base;
  if ((rc = upload_padded(b + off_q, q, m, h->d, dp, 8, s))) return rc;
  const double *cn = metric == kMetricCosine ? x.norms64 : metric == kMetricEuclidean ? x.norms64 + n : nullptr;
  uint32_t *oi = (uint32_t *)(b + off_i);
  double *os = (double *)(b + off_s);
  rc = topk_f64_device_impl((const double *)(b + off_q), dp, m, x.data64, dp, n, h->d, k, metric, 0u, oi, os,
                            b + off_w, s, fused, cn);
  if (rc) return rc;
  {
    Timed t("d2h", s);
    HIP_TRY(hipMemcpyAsync(out_idx, oi, (size_t)m * k * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(out_score, os, (size_t)m * k * 8, hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(hipStreamSynchronize(s));
  return PMM_OK;
}

int pmm_topk_f32_corpus(const pmm_corpus *h, const float *q, int64_t m, int64_t k, int metric,
                        uint32_t *out_idx, float *out_score) {
  if (!h) return fail(PMM_ERR_ARG, "null corpus");
  if (h->dtype != PMM_DTYPE_F32)
    return fail(PMM_ERR_ARG, "the corpus handle holds f64 rows: use pmm_topk_f64_corpus");
  int rc = validate_sizes(m, h->n, h->d, k, true);
  if (rc) return rc;
  if ((rc = check_metric(metric))) return rc;
  if (m == 0 || k == 0) return PMM_OK;
  if ((rc = need_buffers(q, out_idx, out_score))) return rc;
  // which of a shard's norm arrays this metric reads (none for dot)
  auto shard_norms = [&](const CorpusShard &x) -> const float * {
    return metric == kMetricCosine ? x.norms : metric == kMetricEuclidean ? x.norms + 2 * x.n : nullptr;
  };
  if (h->shards.size() > 1 && k <= kFusedMaxK) {
    std::vector<ShardSrc> sh(h->shards.size());
    for (size_t g = 0; g < sh.size(); g++) {
      const CorpusShard &x = h->shards[g];
      sh[g] = ShardSrc{x.device, x.lo, x.n, nullptr, x.data, shard_norms(x)};
    }
    return topk_sharded(q, m, h->d, k, metric, PMM_COMPUTE_F32, sh, out_idx, out_score);
  }
  if (h->shards.size() > 1)
    return fail(PMM_ERR_UNSUPPORTED, "a device-sharded corpus supports k <= %d (got %lld)", kFusedMaxK,
                (long long)k);
  const CorpusShard &x = h->shards[0];
  int dev;
  DevScope scope;
  if ((rc = ensure_device(&dev, &scope, x.device))) return rc;
  hipStream_t s;
  if ((rc = thread_stream(dev, &s))) return rc;
  const int64_t dp = h->dp;
  size_t ws_need = pmm_topk_workspace_bytes(m, h->n, dp, k, metric, PMM_COMPUTE_F32);
  size_t off_q = 0, off_i = al256((size_t)m * dp * 4);
  size_t off_s = off_i + al256((size_t)m * k * 4), off_w = off_s + al256((size_t)m * k * 4);
  void *base;
  if ((rc = arena(dev, s, off_w + ws_need, &base))) return rc;
  char *b = (char *)base;
  if ((rc = upload_padded(b + off_q, q, m, h->d, dp, 4, s))) return rc;
  rc = topk_f32_device_impl((const float *)(b + off_q), dp, m, x.data, dp, h->n, h->d, k, metric,
                            0u, (uint32_t *)(b + off_i), (float *)(b + off_s), b + off_w, ws_need,
                            s, dev, shard_norms(x));
  if (rc) return rc;
  {
    Timed t("d2h", s);
    HIP_TRY(hipMemcpyAsync(out_idx, b + off_i, (size_t)m * k * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(out_score, b + off_s, (size_t)m * k * 4, hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(hipStreamSynchronize(s));
  return PMM_OK;
}

int pmm_timing_enable(int enable) {
  t_ctx.timing = enable != 0;
  return PMM_OK;
}

int pmm_timing_reset(void) {
  for (auto &r : t_ctx.recs) {
    (void)hipEventSynchronize(r.b);
    if ((int)t_ctx.free_events.size() <= r.dev) t_ctx.free_events.resize(r.dev + 1);
    t_ctx.free_events[r.dev].push_back(r.a);
    t_ctx.free_events[r.dev].push_back(r.b);
  }
  t_ctx.recs.clear();
  return PMM_OK;
}

int pmm_timing_read(const char *kernel, double *total_ms, int64_t *launches) {
  double tot = 0.0;
  int64_t cnt = 0;
  for (auto &r : t_ctx.recs) {
    if (kernel && !strstr(r.name, kernel)) continue;
    HIP_TRY(hipEventSynchronize(r.b));
    float ms = 0.0f;
    HIP_TRY(hipEventElapsedTime(&ms, r.a, r.b));
    tot += ms;
    cnt++;
  }
  if (total_ms) *total_ms = tot;
  if (launches) *launches = cnt;
  return PMM_OK;
}

}  // extern "C"
