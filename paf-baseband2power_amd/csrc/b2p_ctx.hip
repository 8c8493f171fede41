// C ABI of the integrator (include/b2p.h): context, streams, staging, timing.
//
// Replaces the empty host driver of the reference (baseband2power.cu:1-16)
// and its error convention (cudautil.cuh:29-66: print + exit(-1)) with
// status codes.  All HIP calls go through CK() which records the HIP error
// text in the context and returns B2P_EHIP.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "b2p.h"
#include "b2p_internal.h"
#include "b2p_plan.h"

using namespace b2p;

namespace {

constexpr uint32_t kMaxOut = 8192;      // LDS: 64 KiB of uint64 sums
constexpr uint32_t kTimingRing = 4096;  // event pairs kept before a drain

thread_local char g_err[256];  // errors before a context exists

static_assert(B2P_MAX_BLOCKS == kMaxBlk, "b2p.h and the kernels agree on blocks per launch");

struct EvPair {
  hipEvent_t a, b;
  uint64_t bytes;
  int kind;  // 0 integrate, 1 finalize
};

// Host memory registered through b2p_register_host, process-wide (HIP's
// registration is): which context registered each range, so that b2p_close
// releases what its context registered and a register that overlaps a live
// registration is refused up front.  A range left registered after its
// owner freed it is the hazard: HIP would keep serving copies of that
// address from the stale pinned mapping ("Host memory").
struct HostReg {
  const char *base;
  size_t bytes;
  const b2p_ctx *owner;
};
std::mutex g_reg_mu;
std::vector<HostReg> g_regs;

}  // namespace

struct b2p_ctx {
  b2p_geom_t g;
  int device = 0;
  int mode = kI8;
  KernelChoice kc{};
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;
  // launch geometry
  uint32_t VW = 0, IV = 0, FV = 0, CP = 0;
  uint32_t B = 0, Bpad = 0, S = 0, NC = 0, G = 0;
  uint32_t nchan = 0, nout = 0, nrep = 0;
  uint64_t frame_bytes = 0, block_bytes = 0;
  // two replica sets: integration k sums into set k&1.  Its finalize is
  // deferred and carried by ONE extra workgroup of the next integrate launch
  // (which sums into the other set), so no finalize launch and no
  // cross-stream dependency sits between two integrations; b2p_sync /
  // b2p_finish flush a finalize that found no launch to ride on.
  unsigned long long *d_rep = nullptr;
  uint32_t *d_ticket = nullptr;  // arrival counters of the in-launch finalize [2]
  float *d_out = nullptr;
  int cur = 0;                   // replica set of the running integration
  struct {
    int valid;
    unsigned long long *rep;     // its first replica set
    uint32_t nblk;               // integrations (consecutive sets / outputs)
    float *dev_out;              // where the kernel writes the spectrum
    float *host_out;             // non-null: D2H copy after it
    int raw;                     // 1: exact uint64 sums instead of fp32
  } pend = {0, nullptr, 1, nullptr, nullptr, 0};
  // b2p_integrate_n: two banks of kMaxBlk replica sets (launch k sums into
  // bank k&1 while it finalizes the other), allocated on first use
  unsigned long long *d_mrep = nullptr;
  float *d_mout = nullptr;  // host-output staging, kMaxBlk spectra
  int mbank = 0;
  uint32_t interleave = 0;
  int fuse = 0;  // b2p_integrate: finalize in the last workgroup (1) or a
                 // separate launch (0, measured faster: DESIGN.md)
  // host-buffer staging (double buffered)
  uint8_t *d_stage[2] = {nullptr, nullptr};
  uint64_t stage_bytes = 0;
  hipEvent_t ev_copied[2] = {nullptr, nullptr};
  hipEvent_t ev_consumed[2] = {nullptr, nullptr};
  uint32_t stage_next = 0;
  int staging_ready = 0;        // both buffers, their events and the copy stream exist
  uint64_t samples = 0;
  unsigned long long *d_dbg = nullptr;  // B2P_DEBUG builds: out-of-bounds records (b2p_kernels.hip)
  // timing: 1 = per-launch dispatch-packet events, 2 = one event pair
  // around a region of launches (no per-launch packets)
  int timing = 0;
  hipEvent_t region_a = nullptr, region_b = nullptr;
  uint64_t region_launches = 0, region_bytes = 0, region_finalizes = 0;
  int region_closed = 0;  // closing event recorded, not read yet (read by drain_timing)
  // region opened, its first event not recorded yet: it is recorded by the
  // region's first enqueue, so the caller's own time between opening the
  // region and its first call is not GPU time (region_mark)
  int region_open = 0;
  std::vector<EvPair> pending;
  std::vector<hipEvent_t> ev_pool;
  b2p_stats_t stats{};
  // b2p_fence tickets: event ring
  hipEvent_t fence_ev[8] = {};
  uint64_t fence_next = 0;
  // sticky failure: a call failed after part of its work was enqueued
  // (b2p_push's host-span loop), so the running sums are unknown; only
  // b2p_close is meaningful afterwards (B2P_EFAILED)
  int failed = 0;
  b2p_tuning_t tun{};           // launch variant (b2p_open_tuned); defaults otherwise
#ifdef B2P_TEST_HOOKS
  long inject_push_fail = -1;  // test build only: b2p_test_inject_push_fail
  long dbg_shrink = 0;         // debug + test build only: b2p_test_debug_shrink_bound
#endif
  char err[256] = {0};
};

static int set_err(b2p_ctx_t *c, int code, const char *fmt, ...) {
  char *dst = c ? c->err : g_err;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(dst, 256, fmt, ap);
  va_end(ap);
  return code;
}

// entry guard of every call that touches a context's stream or sums; the
// first failure's text stays in c->err
#define LIVE(c)                                 \
  do {                                          \
    if ((c) && (c)->failed) return B2P_EFAILED; \
  } while (0)

#define CK(c, call)                                                            \
  do {                                                                         \
    hipError_t e_ = (call);                                                    \
    if (e_ != hipSuccess)                                                      \
      return set_err((c), B2P_EHIP, "%s failed at %s:%d: %s", #call, __FILE__, \
                     __LINE__, hipGetErrorString(e_));                         \
  } while (0)

static uint64_t word_bytes(const b2p_geom_t *g) {
  return (uint64_t)g->npol * g->ndim * (g->nbit / 8);
}

extern "C" {

int b2p_abi_version(void) { return B2P_ABI_VERSION; }

const char *b2p_strerror(int code) {
  switch (code) {
    case B2P_OK: return "ok";
    case B2P_EINVAL: return "invalid argument or unsupported geometry";
    case B2P_ERAGGED: return "span is not a whole number of frames";
    case B2P_EOVERFLOW: return "push exceeds nsamp_int of the integration";
    case B2P_EPARTIAL: return "integration finished with != nsamp_int samples";
    case B2P_ENODEV: return "no such HIP device";
    case B2P_EHIP: return "HIP runtime error";
    case B2P_ENOMEM: return "out of memory";
    case B2P_EALIGN: return "buffer not 16-byte aligned";
    case B2P_EFAILED: return "context failed part-way through an earlier call; close it";
    case B2P_ETIMEDOUT: return "collective did not complete within the group's time limit";
  }
  return "unknown error";
}

const char *b2p_last_error(const b2p_ctx_t *c) { return c ? c->err : g_err; }

int b2p_geom_bmf(b2p_geom_t *g) {
  if (!g) return B2P_EINVAL;
  memset(g, 0, sizeof(*g));
  g->nbit = 16;          // BMF payload: 16-bit complex, big-endian
  g->big_endian = 1;
  g->nchunk = 48;        // NCHK_NIC (capture.h:20, conf:5)
  g->nsamp_df = 128;     // NSAMP_DF (conf:2); 7168 B = 128 x 7 x 8 (capture.h:28)
  g->nchan_chunk = 7;
  g->npol = 2;           // NPOL_SAMP (conf:3)
  g->ndim = 2;           // NDIM_POL (conf:4)
  g->npol_out = 1;       // header_baseband2power.txt:41 NPOL 1
  g->nsamp_int = 1u << 20;  // README.md:2, 1024 x 1024
  g->mean = 0;
  return B2P_OK;
}

uint64_t b2p_frame_bytes(const b2p_geom_t *g) {
  return g ? (uint64_t)g->nchunk * g->nsamp_df * g->nchan_chunk * word_bytes(g) : 0;
}

uint64_t b2p_block_bytes(const b2p_geom_t *g) {
  if (!g || !g->nsamp_df) return 0;
  return g->nsamp_int / g->nsamp_df * b2p_frame_bytes(g);
}

int b2p_geom_check(const b2p_geom_t *g) {
  if (!g) return B2P_EINVAL;
  if (g->nbit != 8 && g->nbit != 16) return B2P_EINVAL;
  if (g->nbit == 8 && g->big_endian) return B2P_EINVAL;
  if (g->npol != 2 || g->ndim != 2) return B2P_EINVAL;
  if (g->npol_out != 1 && g->npol_out != 2) return B2P_EINVAL;
  if (!g->nchunk || !g->nsamp_df || !g->nchan_chunk) return B2P_EINVAL;
  if (g->reserved) return B2P_EINVAL;
  if (!g->nsamp_int || g->nsamp_int % g->nsamp_df) return B2P_EINVAL;
  const uint64_t chunk_bytes = (uint64_t)g->nsamp_df * g->nchan_chunk * word_bytes(g);
  if (chunk_bytes % 16) return B2P_EINVAL;
  const uint64_t nout = (uint64_t)g->nchunk * g->nchan_chunk * g->npol_out;
  if (nout > kMaxOut) return B2P_EINVAL;
  if (chunk_bytes / 16 * g->nchunk > 0xffffffffull) return B2P_EINVAL;
  return B2P_OK;
}

int b2p_device_count(int *count) {
  if (!count) return B2P_EINVAL;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return set_err(nullptr, B2P_ENODEV, "hipGetDeviceCount: %s", hipGetErrorString(e));
  }
  *count = n;
  return B2P_OK;
}

// The workgroup shape (b2p_plan.h plan_shape, shared with the CPU address
// model of tests/c/plan_model.cpp).
static int plan_launch(b2p_ctx_t *c, int ncu) {
  const b2p_geom_t *g = &c->g;
  const ShapeKnobs k{c->tun.max_threads, c->tun.threads, c->tun.wg_per_cu, c->tun.row_groups, c->tun.replicas};
  Shape sh;
  char msg[160];
  if (plan_shape(g->nbit, g->nchunk, g->nsamp_df, g->nchan_chunk, k, ncu, &sh, msg, sizeof msg) != 0)
    return set_err(c, B2P_EINVAL, "%s", msg);
  c->VW = sh.VW;
  c->IV = sh.IV;
  c->FV = sh.FV;
  c->CP = sh.CP;
  c->B = sh.B;
  c->Bpad = sh.Bpad;
  c->S = sh.S;
  c->NC = sh.NC;
  c->G = sh.G;
  c->nrep = sh.nrep;
  return B2P_OK;
}

void b2p_tuning_init(b2p_tuning_t *t) {
  if (!t) return;
  memset(t, 0, sizeof *t);
  t->size = sizeof *t;
  t->nontemporal = t->interleave = t->fuse = -1;
}

// every value a tuning may carry; anything else is refused, not clamped
static const char *tuning_problem(const b2p_tuning_t *t) {
  if (t->size != sizeof *t) return "b2p_tuning_t.size does not match this library";
  if (t->max_threads && (t->max_threads < 64 || t->max_threads > 1024)) return "max_threads";
  if (t->threads && (t->threads < 64 || t->threads > 1024 || t->threads % 64)) return "threads";
  if (t->wg_per_cu && (t->wg_per_cu < 1 || t->wg_per_cu > 32)) return "wg_per_cu";
  if (t->row_groups < 0) return "row_groups";
  if (t->replicas && (t->replicas < 1 || t->replicas > 1024)) return "replicas";
  if (t->unroll && t->unroll != 4 && t->unroll != 8 && t->unroll != 16) return "unroll";
  if (t->nontemporal < -1 || t->nontemporal > 1) return "nontemporal";
  if (t->interleave < -1 || t->interleave > 1) return "interleave";
  if (t->fuse < -1 || t->fuse > 1) return "fuse";
  if (t->stage_mib && (t->stage_mib < 1 || t->stage_mib > 16384)) return "stage_mib";
  if (t->assemble_grid < 0) return "assemble_grid";
  return nullptr;
}

int b2p_device_pci_bus_id(int device, char *buf, int len) {
  if (!buf || len < 13 || device < 0) return B2P_EINVAL;
  hipError_t e = hipDeviceGetPCIBusId(buf, len, device);
  if (e != hipSuccess) {
    buf[0] = 0;
    return set_err(nullptr, B2P_ENODEV, "hipDeviceGetPCIBusId(%d): %s", device, hipGetErrorString(e));
  }
  return B2P_OK;
}

int b2p_open(b2p_ctx_t **out, const b2p_geom_t *g, int device) {
  return b2p_open_tuned(out, g, device, nullptr);
}

int b2p_open_tuned(b2p_ctx_t **out, const b2p_geom_t *g, int device, const b2p_tuning_t *tun) {
  if (!out || !g) return set_err(nullptr, B2P_EINVAL, "null argument");
  *out = nullptr;
  if (b2p_geom_check(g) != B2P_OK) return set_err(nullptr, B2P_EINVAL, "unsupported geometry");
  b2p_tuning_t t;
  b2p_tuning_init(&t);
  if (tun) {
    if (const char *bad = tuning_problem(tun)) return set_err(nullptr, B2P_EINVAL, "tuning: %s", bad);
    t = *tun;
  }
  if (device < 0) return set_err(nullptr, B2P_ENODEV, "device index %d < 0", device);
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0)
    return set_err(nullptr, B2P_ENODEV, "no HIP device (%s)", hipGetErrorString(e));
  if (n == 1) device = 0;  // paf_baseband2power.cu:89-90
  if (device >= n) return set_err(nullptr, B2P_ENODEV, "device %d of %d", device, n);

  b2p_ctx_t *c = new (std::nothrow) b2p_ctx_t();
  if (!c) return set_err(nullptr, B2P_ENOMEM, "context allocation");
  c->g = *g;
  c->tun = t;
  c->device = device;
  c->mode = g->nbit == 8 ? kI8 : (g->big_endian ? kI16BE : kI16LE);
  c->nchan = g->nchunk * g->nchan_chunk;
  c->nout = c->nchan * g->npol_out;
  c->frame_bytes = b2p_frame_bytes(g);
  c->kc.mode = c->mode;
  c->kc.npol_out = (int)g->npol_out;
  // measured defaults (tools/tune.py, DESIGN.md "launch shape"): 28-32 KiB
  // of loads in flight per CU -- 4 rows per lane; int8 512 threads with
  // contiguous row slices, int16 (BMF) 448 threads with interleaved rows --
  // one workgroup per CU, non-temporal loads (the row order is chosen after
  // the launch shape, below)
  c->kc.unroll = t.unroll ? t.unroll : 4;
  c->kc.nt = t.nontemporal != 0;
  c->fuse = t.fuse > 0;
  c->block_bytes = b2p_block_bytes(g);
  int rc;
  int ncu = 256;
  auto fail = [&](int code) {
    if (code != B2P_OK) {
      snprintf(g_err, sizeof g_err, "%s", c->err);
      b2p_close(c);
    }
    return code;
  };
  if (hipSetDevice(device) != hipSuccess) return fail(set_err(c, B2P_ENODEV, "hipSetDevice(%d)", device));
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu <= 0)
    ncu = 256;
  if ((rc = plan_launch(c, ncu)) != B2P_OK) return fail(rc);
  // rows: contiguous slices for a one-column int8 row (configs[1..4]);
  // interleaved for int16 and for rows over several workgroup columns, whose
  // columns then walk the same rows together (int8 TFTFP 32x8: 6.51 -> 6.95
  // TB/s, int8 336 ch 6.80 -> 6.96; profiles/r03_tune_interleave.jsonl)
  c->interleave = t.interleave >= 0 ? (uint32_t)t.interleave : (g->nbit == 16 || c->NC > 1 ? 1u : 0u);
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess)
    return fail(set_err(c, B2P_EHIP, "hipStreamCreate"));
  c->stream = c->own_stream;
  // fence events up front: the first event a process creates can take tens
  // of ms, which must not land on the first integration of a pipeline
  for (auto &e : c->fence_ev)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
      return fail(set_err(c, B2P_EHIP, "hipEventCreate"));
  // the timing region's pair too, so opening the first region costs nothing
  if (hipEventCreate(&c->region_a) != hipSuccess || hipEventCreate(&c->region_b) != hipSuccess)
    return fail(set_err(c, B2P_EHIP, "hipEventCreate"));
  // two replica sets, then the two 4-B tickets (zeroed together; every
  // finalize leaves its set and ticket zero again)
  const size_t set_words = (size_t)c->nrep * c->nout;
  const size_t rep_bytes = 2 * set_words * sizeof(unsigned long long) + 16;
  if (hipMalloc(&c->d_rep, rep_bytes) != hipSuccess) return fail(set_err(c, B2P_ENOMEM, "hipMalloc replicas"));
  c->d_ticket = (uint32_t *)(c->d_rep + 2 * set_words);

  // sized for uint64 sums too (b2p_finish_partial_async to host)
  if (hipMalloc(&c->d_out, (size_t)c->nout * sizeof(unsigned long long)) != hipSuccess)
    return fail(set_err(c, B2P_ENOMEM, "hipMalloc out"));
#ifdef B2P_DEBUG
  if (hipMalloc(&c->d_dbg, 8 * sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(c->d_dbg, 0, 8 * sizeof(unsigned long long)) != hipSuccess)
    return fail(set_err(c, B2P_ENOMEM, "hipMalloc debug record"));
#endif
  if (hipMemsetAsync(c->d_rep, 0, rep_bytes, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return fail(set_err(c, B2P_EHIP, "zero replicas"));
  // load the code object now: a process's first kernel launch costs tens of
  // ms (40 ms measured in paf_baseband2power), which belongs to start-up,
  // not to the first integration
  if (launch_warm(c->stream) != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess)
    return fail(set_err(c, B2P_EHIP, "warm-up launch"));

  *out = c;
  return B2P_OK;
}

static void drain_timing(b2p_ctx_t *c) {
  if (c->region_closed) {  // a closed mode-2 region: its elapsed time
    float ms = 0.f;
    if (hipEventSynchronize(c->region_b) == hipSuccess &&
        hipEventElapsedTime(&ms, c->region_a, c->region_b) == hipSuccess) {
      c->stats.launches += c->region_launches;
      c->stats.bytes += c->region_bytes;
      c->stats.finalizes += c->region_finalizes;
      c->stats.kernel_ms += ms;  // the whole region, gaps and finalizes included
    }
    c->region_launches = c->region_bytes = c->region_finalizes = 0;
    c->region_closed = 0;
  }
  for (auto &p : c->pending) {
    float ms = 0.f;
    if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      if (p.kind == 0) {
        c->stats.launches++;
        c->stats.bytes += p.bytes;
        c->stats.kernel_ms += ms;
      } else {
        c->stats.finalizes++;
        c->stats.finalize_ms += ms;
      }
    }
    c->ev_pool.push_back(p.a);
    c->ev_pool.push_back(p.b);
  }
  c->pending.clear();
}

int b2p_close(b2p_ctx_t *c) {
  if (!c) return B2P_EINVAL;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
  drain_timing(c);
  {  // what this context registered and the caller did not release
    std::lock_guard<std::mutex> lk(g_reg_mu);
    for (auto it = g_regs.begin(); it != g_regs.end();) {
      if (it->owner == c) {
        (void)hipHostUnregister(const_cast<char *>(it->base));
        it = g_regs.erase(it);
      } else {
        ++it;
      }
    }
  }
  for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
  for (int i = 0; i < 2; ++i) {
    if (c->d_stage[i]) (void)hipFree(c->d_stage[i]);
    if (c->ev_copied[i]) (void)hipEventDestroy(c->ev_copied[i]);
    if (c->ev_consumed[i]) (void)hipEventDestroy(c->ev_consumed[i]);
  }
  if (c->d_rep) (void)hipFree(c->d_rep);
  if (c->d_out) (void)hipFree(c->d_out);
  if (c->d_mrep) (void)hipFree(c->d_mrep);
  if (c->d_mout) (void)hipFree(c->d_mout);
  if (c->d_dbg) (void)hipFree(c->d_dbg);
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  for (auto e : c->fence_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->region_a) (void)hipEventDestroy(c->region_a);
  if (c->region_b) (void)hipEventDestroy(c->region_b);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
  return B2P_OK;
}

int b2p_get_info(const b2p_ctx_t *c, b2p_info_t *info) {
  if (!c || !info) return B2P_EINVAL;
  info->nchan = c->nchan;
  info->nout = c->nout;
  info->frame_bytes = c->frame_bytes;
  info->block_bytes = c->block_bytes;
  info->threads = c->B;
  info->columns = c->NC;
  info->row_groups = c->G;
  info->row_vectors = c->S;
  info->replicas = c->nrep;
  info->device = (uint32_t)c->device;
  info->unroll = (uint32_t)c->kc.unroll;
  info->nontemporal = c->kc.nt ? 1u : 0u;
  return B2P_OK;
}

int b2p_set_stream(b2p_ctx_t *c, void *s) {
  if (!c) return B2P_EINVAL;
  LIVE(c);
  CK(c, hipSetDevice(c->device));
  CK(c, hipStreamSynchronize(c->stream));
  c->stream = s ? (hipStream_t)s : c->own_stream;
  return B2P_OK;
}

// pages a host range touches: [first, last] page numbers (pinning is per page)
static void page_span(const char *p, size_t n, uintptr_t *lo, uintptr_t *hi) {
  const uintptr_t pg = 4096;
  *lo = reinterpret_cast<uintptr_t>(p) / pg;
  *hi = (reinterpret_cast<uintptr_t>(p) + n - 1) / pg;
}

int b2p_register_host(b2p_ctx_t *c, void *base, size_t bytes) {
  if (!c || !base || !bytes) return B2P_EINVAL;
  const char *b = static_cast<const char *>(base);
  std::lock_guard<std::mutex> lk(g_reg_mu);
  uintptr_t lo, hi;
  page_span(b, bytes, &lo, &hi);
  for (const HostReg &r : g_regs) {  // a page may be pinned by one registration only
    uintptr_t rlo, rhi;
    page_span(r.base, r.bytes, &rlo, &rhi);
    if (lo <= rhi && rlo <= hi)
      return set_err(c, B2P_EINVAL, "host range %p+%zu shares pages with the registered range %p+%zu", base,
                     bytes, (const void *)r.base, r.bytes);
  }
  CK(c, hipSetDevice(c->device));
  CK(c, hipHostRegister(base, bytes, hipHostRegisterDefault));
  g_regs.push_back(HostReg{b, bytes, c});
  return B2P_OK;
}

static int flush_pending(b2p_ctx_t *c);

// Release a registration once no copy of this context can still read or
// write the range: a deferred finalize (b2p_finish_async into host memory
// that no launch has carried yet) is enqueued first, then the context's
// streams are drained (a host finish may still be landing in the range; a
// failed push's copies were drained by b2p_push).  Found by the ABI state
// machine (tests/test_gpu_api_model.py): without the flush, a spectrum
// finished into the range was copied only at the next sync -- after the
// caller had unregistered, and possibly freed, it.  Work the caller
// enqueued on other contexts or streams that touches the range must be
// complete before this call.
// The drain runs without g_reg_mu: it waits on this context's streams only,
// and holding the process-wide lock across it stalled every other
// context's register / unregister (and, in the debug build, its host pushes,
// dbg_check_host_range) for as long (advisor, round 5).  The range stays in
// g_regs until it is unregistered, so no overlapping registration can slip
// in meanwhile.
static int drain_for_unregister(b2p_ctx_t *c) {
  if (!c->failed && c->pend.valid) {
    const int rf = flush_pending(c);
    if (rf != B2P_OK) return rf;
  }
  if (c->stream) CK(c, hipStreamSynchronize(c->stream));
  if (c->copy_stream) CK(c, hipStreamSynchronize(c->copy_stream));
  return B2P_OK;
}

int b2p_unregister_host(b2p_ctx_t *c, void *base) {
  if (!c || !base) return B2P_EINVAL;
  CK(c, hipSetDevice(c->device));
  const int rc = drain_for_unregister(c);
  if (rc != B2P_OK) return rc;
  const char *b = static_cast<const char *>(base);
  std::lock_guard<std::mutex> lk(g_reg_mu);
  auto it = std::find_if(g_regs.begin(), g_regs.end(), [b](const HostReg &r) { return r.base == b; });
  if (it == g_regs.end()) return set_err(c, B2P_EINVAL, "host range %p is not registered", base);
  CK(c, hipHostUnregister(const_cast<char *>(b)));
  g_regs.erase(it);
  return B2P_OK;
}

static hipEvent_t pool_event(b2p_ctx_t *c) {
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// The opening event of a timing region, recorded in front of the region's
// first piece of GPU work.
static int region_mark(b2p_ctx_t *c) {
  if (c->region_open) {
    CK(c, hipEventRecord(c->region_a, c->stream));
    c->region_open = 0;
  }
  return B2P_OK;
}

static size_t pend_bytes(const b2p_ctx_t *c) {
  return (size_t)c->pend.nblk * c->nout * (c->pend.raw ? sizeof(unsigned long long) : sizeof(float));
}

static int flush_pending(b2p_ctx_t *c);

#ifdef B2P_DEBUG
// Debug build: read the kernels' out-of-bounds record (b2p_kernels.hip
// dbg_record) once the stream is idle; a record fails the call with the
// access that would have been made, and the context.
static int dbg_check(b2p_ctx_t *c) {
  CK(c, hipStreamSynchronize(c->stream));
  unsigned long long r[5] = {0, 0, 0, 0, 0};
  CK(c, hipMemcpy(r, c->d_dbg, sizeof r, hipMemcpyDeviceToHost));
  if (r[0] == 0) return B2P_OK;
  c->failed = 1;
  return set_err(c, B2P_EHIP,
                 "B2P_DEBUG: %llu out-of-bounds %s; first: index %llu of %llu, workgroup %llu thread %llu", r[0],
                 r[1] == 1 ? "span loads" : "output slots", r[2], r[3], r[4] >> 32, r[4] & 0xffffffffull);
}
#endif

// Enqueue one integrate launch over a device span (frame-aligned).  With
// fused_out set, the launch also emits the integration (last workgroup).
static int enqueue_span(b2p_ctx_t *c, const void *dev, uint64_t nbytes, float *fused_out,
                        const void *const *blocks = nullptr, uint32_t nblk = 1) {
  IntegrateArgs a;
  a.data = (const uint4 *)dev;
  a.nvec = nbytes / 16;
  a.S = c->S;
  a.B = c->B;
  a.NC = c->NC;
  a.G = c->G;
  a.IV = c->IV;
  a.FV = c->FV;
  a.nchunk = c->g.nchunk;
  a.nchan_chunk = c->g.nchan_chunk;
  a.nout = c->nout;
  a.nrep = c->nrep;
  a.interleave = c->interleave;
  a.rep = c->d_rep + (size_t)c->cur * c->nrep * c->nout;
  a.nblk = 1;
  a.set_words = (uint64_t)c->nrep * c->nout;
  if (blocks) {  // b2p_integrate_n: nblk whole integrations, this bank's sets
    a.rep = c->d_mrep + (size_t)c->mbank * kMaxBlk * a.set_words;
    a.nblk = nblk;
    for (uint32_t b = 0; b < nblk; ++b) a.blk[b] = (const uint4 *)blocks[b];
  }
  a.out = fused_out;
  a.dbg = c->d_dbg;
  a.dbg_bound = a.nvec;
#if defined(B2P_DEBUG) && defined(B2P_TEST_HOOKS)
  if (c->dbg_shrink) a.dbg_bound = a.nvec > (uint64_t)c->dbg_shrink ? a.nvec - (uint64_t)c->dbg_shrink : 0;
#endif
#ifdef B2P_DEBUG
  // the launch invariants the kernel's indexing assumes
  {
    const unsigned long long *r0 = c->d_rep, *r1 = c->d_rep + 2 * (size_t)c->nrep * c->nout;
    if (blocks) r0 = c->d_mrep, r1 = c->d_mrep + 2 * (size_t)kMaxBlk * c->nrep * c->nout;
    const unsigned long long *a0 = a.rep, *a1 = a.rep + (size_t)a.nblk * a.set_words;
    if (nbytes % c->frame_bytes || nbytes % 16 || (uint64_t)c->NC * c->B > c->S || a0 < r0 || a1 > r1 ||
        (size_t)c->nout * sizeof(unsigned long long) > 65536 || !c->d_dbg)
      return set_err(c, B2P_EINVAL,
                     "B2P_DEBUG: launch invariants: span %llu B (frame %llu), NC %u x B %u vs S %u, replicas "
                     "[%p,%p) in [%p,%p)",
                     (unsigned long long)nbytes, (unsigned long long)c->frame_bytes, c->NC, c->B, c->S,
                     (const void *)a0, (const void *)a1, (const void *)r0, (const void *)r1);
  }
#endif
  a.ticket = c->d_ticket + c->cur;
  a.mean = c->g.mean;
  a.nsamp = (double)c->g.nsamp_int;
  uint32_t grid = c->NC * c->G;
  a.nwork = grid;
  // the previous integration's finalize rides on this launch (extra block)
  a.fin_rep = nullptr;
  a.fin_out = nullptr;
  a.fin_raw = 0;
  a.fin_nblk = 0;
  // A deferred finalize rides on this launch in its own extra workgroup,
  // which runs at no fixed point against the workgroup that emits a fused
  // integration.  If both would write the same output (a caller reusing an
  // output buffer before b2p_sync), the older spectrum could land last: run
  // the deferred one first, on its own (found by tests/test_gpu_api_model.py).
  if (fused_out && c->pend.valid) {
    const char *f0 = reinterpret_cast<const char *>(fused_out), *f1 = f0 + (size_t)c->nout * sizeof(float);
    const char *p0 = reinterpret_cast<const char *>(c->pend.dev_out), *p1 = p0 + pend_bytes(c);
    if (f0 < p1 && p0 < f1) {
      int rf = flush_pending(c);
      if (rf != B2P_OK) return rf;
    }
  }
  const bool carry = c->pend.valid;
  if (carry) {
    a.fin_rep = c->pend.rep;
    a.fin_out = c->pend.dev_out;
    a.fin_raw = (uint32_t)c->pend.raw;
    a.fin_nblk = c->pend.nblk;
    grid += 1;
  }
  EvPair p{nullptr, nullptr, nbytes, 0};
  p.bytes = nbytes * a.nblk;
  if (c->timing == 2) {
    if (int rm = region_mark(c)) return rm;
    c->region_launches++;
    c->region_bytes += nbytes * a.nblk;
  } else if (c->timing) {
    if (c->pending.size() >= kTimingRing) drain_timing(c);
    p.a = pool_event(c);
    p.b = pool_event(c);
    if (!p.a || !p.b) return set_err(c, B2P_EHIP, "hipEventCreate");
  }
  CK(c, launch_integrate(a, c->kc, c->Bpad, grid, c->stream, p.a, p.b));
  if (c->timing == 1) c->pending.push_back(p);
  if (carry) {
    if (c->pend.host_out)
      CK(c, hipMemcpyAsync(c->pend.host_out, c->pend.dev_out, pend_bytes(c), hipMemcpyDeviceToHost,
                           c->stream));
    c->pend.valid = 0;
  }
  return B2P_OK;
}

// A deferred finalize with no integrate launch to ride on: run it alone.
static int flush_pending(b2p_ctx_t *c) {
  if (!c->pend.valid) return B2P_OK;
  FinalizeArgs f;
  f.rep = c->pend.rep;
  f.nblk = c->pend.nblk;
  f.nrep = c->nrep;
  f.nout = c->nout;
  f.out = c->pend.dev_out;
  f.mean = c->g.mean;
  f.nsamp = (double)c->g.nsamp_int;
  f.raw = (uint32_t)c->pend.raw;
  EvPair p{nullptr, nullptr, 0, 1};
  if (c->timing == 2) {
    if (int rm = region_mark(c)) return rm;
    c->region_finalizes++;
  } else if (c->timing) {
    if (c->pending.size() >= kTimingRing) drain_timing(c);
    p.a = pool_event(c);
    p.b = pool_event(c);
    if (!p.a || !p.b) return set_err(c, B2P_EHIP, "hipEventCreate");
  }
  CK(c, launch_finalize(f, c->stream, p.a, p.b));
  if (c->timing == 1) c->pending.push_back(p);
  if (c->pend.host_out)
    CK(c, hipMemcpyAsync(c->pend.host_out, c->pend.dev_out, pend_bytes(c), hipMemcpyDeviceToHost,
                         c->stream));
  c->pend.valid = 0;
  return B2P_OK;
}

// The staging pair, its events and the copy stream: all or nothing (a
// half-made set would hand push_host a null buffer or stream).
static void release_staging(b2p_ctx_t *c) {
  for (int i = 0; i < 2; ++i) {
    if (c->d_stage[i]) (void)hipFree(c->d_stage[i]);
    if (c->ev_copied[i]) (void)hipEventDestroy(c->ev_copied[i]);
    if (c->ev_consumed[i]) (void)hipEventDestroy(c->ev_consumed[i]);
    c->d_stage[i] = nullptr;
    c->ev_copied[i] = c->ev_consumed[i] = nullptr;
  }
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  c->copy_stream = nullptr;
}

static int make_staging(b2p_ctx_t *c) {
  const uint64_t want = (uint64_t)(c->tun.stage_mib ? c->tun.stage_mib : 256) << 20;
  const uint64_t sb = stage_bytes_for(want, c->frame_bytes);
  c->stage_bytes = sb;
  for (int i = 0; i < 2; ++i) {
    if (hipMalloc(&c->d_stage[i], sb) != hipSuccess) {
      c->d_stage[i] = nullptr;
      return set_err(c, B2P_ENOMEM, "hipMalloc staging");
    }
    CK(c, hipEventCreateWithFlags(&c->ev_copied[i], hipEventDisableTiming));
    CK(c, hipEventCreateWithFlags(&c->ev_consumed[i], hipEventDisableTiming));
  }
  CK(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
  for (int i = 0; i < 2; ++i) CK(c, hipEventRecord(c->ev_consumed[i], c->stream));
  return B2P_OK;
}

static int ensure_staging(b2p_ctx_t *c) {
  if (c->staging_ready) return B2P_OK;
  const int rc = make_staging(c);
  if (rc != B2P_OK) {
    (void)hipStreamSynchronize(c->stream);  // the consumed-event records
    release_staging(c);
    return rc;
  }
  c->staging_ready = 1;
  return B2P_OK;
}

#ifdef B2P_DEBUG
// Debug build: the invariants push_host relies on, checked per chunk; a
// violation fails the push with its text instead of reaching the GPU.
#define DBG_REQUIRE(c, cond, ...)                                                           \
  do {                                                                                       \
    if (!(cond)) return set_err((c), B2P_EINVAL, "B2P_DEBUG: " __VA_ARGS__);                 \
  } while (0)

// A host range inside a registration must end inside it: a copy that ran
// past the registered pages would read memory HIP never mapped.
static int dbg_check_host_range(b2p_ctx_t *c, const uint8_t *h, uint64_t n) {
  std::lock_guard<std::mutex> lk(g_reg_mu);
  const char *p = reinterpret_cast<const char *>(h);
  for (const HostReg &r : g_regs)
    if (p >= r.base && p < r.base + r.bytes)
      DBG_REQUIRE(c, p + n <= r.base + r.bytes, "host chunk %p+%llu runs past its registration %p+%zu",
                  (const void *)p, (unsigned long long)n, (const void *)r.base, r.bytes);
  return B2P_OK;
}
#endif

// A host span through the two staging buffers: chunk k is copied on the
// copy stream while chunk k-1 is integrated.  Returns once every copy has
// landed (the caller may release the span).  A failure after the first
// chunk leaves part of the span summed, and copies from the span may still
// be in flight: b2p_push drains them before it returns.
static int push_host(b2p_ctx_t *c, const uint8_t *h, uint64_t nbytes) {
  if (int rm = region_mark(c)) return rm;  // the region holds the copies as well
  int last = -1;
  long k = 0;
  for (uint64_t off = 0; off < nbytes; off += c->stage_bytes, ++k) {
    const uint64_t n = stage_chunk(nbytes, c->stage_bytes, off);
    const int i = (int)(c->stage_next++ & 1);
#ifdef B2P_DEBUG
    DBG_REQUIRE(c, c->staging_ready && c->d_stage[i] && c->copy_stream && c->ev_copied[i] && c->ev_consumed[i],
                "staging set incomplete at chunk %ld", k);
    DBG_REQUIRE(c, n > 0 && n <= c->stage_bytes && n % c->frame_bytes == 0 && off + n <= nbytes,
                "chunk %ld: %llu B at %llu of a %llu-B span, staging %llu B, frame %llu B", k,
                (unsigned long long)n, (unsigned long long)off, (unsigned long long)nbytes,
                (unsigned long long)c->stage_bytes, (unsigned long long)c->frame_bytes);
    if (int rd = dbg_check_host_range(c, h + off, n)) return rd;
#endif
#ifdef B2P_TEST_HOOKS
    if (k == c->inject_push_fail)
      return set_err(c, B2P_EHIP, "injected failure at staging chunk %ld (test build)", k);
#endif
    // the staging buffer is free once chunk k-2's launch is done: usually
    // long since (a chunk copies in ~4.7 ms, integrates in ~40 us), and then
    // the copy queue gets no cross-stream wait at all
    const hipError_t q = hipEventQuery(c->ev_consumed[i]);
    if (q == hipErrorNotReady)
      CK(c, hipStreamWaitEvent(c->copy_stream, c->ev_consumed[i], 0));
    else
      CK(c, q);
    CK(c, hipMemcpyAsync(c->d_stage[i], h + off, n, hipMemcpyHostToDevice, c->copy_stream));
    CK(c, hipEventRecord(c->ev_copied[i], c->copy_stream));
    CK(c, hipStreamWaitEvent(c->stream, c->ev_copied[i], 0));
    int rc = enqueue_span(c, c->d_stage[i], n, nullptr);
    if (rc != B2P_OK) return rc;
    CK(c, hipEventRecord(c->ev_consumed[i], c->stream));
    last = i;
  }
  if (last >= 0) CK(c, hipEventSynchronize(c->ev_copied[last]));
  return B2P_OK;
}

int b2p_push(b2p_ctx_t *c, const void *buf, size_t nbytes, int is_device) {
  if (!c) return B2P_EINVAL;
  LIVE(c);
  if (nbytes == 0) return B2P_OK;
  if (!buf) return set_err(c, B2P_EINVAL, "null buffer");
  if (nbytes % c->frame_bytes)
    return set_err(c, B2P_ERAGGED, "%zu bytes is not a multiple of the %llu-byte frame", nbytes,
                   (unsigned long long)c->frame_bytes);
  const uint64_t samples = nbytes / c->frame_bytes * c->g.nsamp_df;
  if (c->samples + samples > c->g.nsamp_int)
    return set_err(c, B2P_EOVERFLOW, "push of %llu samples overflows the %llu-sample integration",
                   (unsigned long long)samples, (unsigned long long)c->g.nsamp_int);
  CK(c, hipSetDevice(c->device));
  int rc;
  if (is_device && (uintptr_t)buf % 16) return set_err(c, B2P_EALIGN, "device span not 16-B aligned");
  if (is_device) {
    if ((rc = enqueue_span(c, buf, nbytes, nullptr)) != B2P_OK) return rc;
  } else {
    if ((rc = ensure_staging(c)) != B2P_OK) return rc;
    rc = push_host(c, (const uint8_t *)buf, nbytes);
    if (rc != B2P_OK) {
      // part of the span may already be summed: the integration is unknown.
      // Copies from the span may still be in flight: drain them, so that the
      // caller can release (unregister, free, close its DADA block) the span
      // as soon as this returns -- a copy still reading memory its owner
      // has released is a GPU page fault
      (void)hipStreamSynchronize(c->copy_stream);
      (void)hipStreamSynchronize(c->stream);
      c->failed = 1;
      return rc;
    }
#ifdef B2P_DEBUG
    if ((rc = dbg_check(c)) != B2P_OK) return rc;
#endif
  }
  c->samples += samples;
  return B2P_OK;
}

uint64_t b2p_samples_pending(const b2p_ctx_t *c) { return c ? c->samples : 0; }

}  // extern "C"

void *b2p_internal_stream(b2p_ctx_t *c) { return c ? (void *)c->stream : nullptr; }

void *b2p_internal_fence_event(b2p_ctx_t *c, uint64_t ticket) {
  if (!c || ticket >= c->fence_next || c->fence_next - ticket > 8) return nullptr;
  return (void *)c->fence_ev[ticket % 8];
}

int b2p_internal_flush(b2p_ctx_t *c) {
  if (!c) return B2P_EINVAL;
  LIVE(c);  // a group collective over a failed member reports it
  CK(c, hipSetDevice(c->device));
  return flush_pending(c);
}

extern "C" {

static int finish_common(b2p_ctx_t *c, void *out, int out_is_device, int raw) {
  if (!c || !out) return B2P_EINVAL;
  LIVE(c);
  CK(c, hipSetDevice(c->device));
  int rc = flush_pending(c);  // two finishes in a row: the first runs alone
  if (rc != B2P_OK) return rc;
  // defer: the next integrate launch (or b2p_sync) emits this integration
  c->pend.valid = 1;
  c->pend.rep = c->d_rep + (size_t)c->cur * c->nrep * c->nout;
  c->pend.nblk = 1;
  c->pend.raw = raw;
  c->pend.dev_out = out_is_device ? (float *)out : c->d_out;
  c->pend.host_out = out_is_device ? nullptr : (float *)out;
  c->cur ^= 1;
  const uint64_t got = c->samples;
  c->samples = 0;
  if (got != c->g.nsamp_int)
    return set_err(c, B2P_EPARTIAL, "integration had %llu of %llu samples", (unsigned long long)got,
                   (unsigned long long)c->g.nsamp_int);
  return B2P_OK;
}

int b2p_finish_async(b2p_ctx_t *c, float *out, int out_is_device) {
  return finish_common(c, out, out_is_device, 0);
}

int b2p_finish_partial_async(b2p_ctx_t *c, uint64_t *sums, int sums_is_device) {
  return finish_common(c, sums, sums_is_device, 1);
}

int b2p_finalize_sums(b2p_ctx_t *c, const uint64_t *sums, uint64_t nspec, uint64_t nsamp_total,
                      float *out) {
  if (!c || !sums || !out) return B2P_EINVAL;
  LIVE(c);
  CK(c, hipSetDevice(c->device));
  int rc = flush_pending(c);  // sums this context still owes come first
  if (rc != B2P_OK) return rc;
  ConvertArgs a;
  a.sums = (const unsigned long long *)sums;
  a.out = out;
  a.n = nspec * c->nout;
  a.mean = c->g.mean;
  a.nsamp = (double)(nsamp_total ? nsamp_total : c->g.nsamp_int);
  if ((rc = region_mark(c)) != B2P_OK) return rc;
  CK(c, launch_convert(a, c->stream));
  return B2P_OK;
}

int b2p_fence(b2p_ctx_t *c, uint64_t *ticket) {
  if (!c || !ticket) return B2P_EINVAL;
  LIVE(c);
  CK(c, hipSetDevice(c->device));
  const int slot = (int)(c->fence_next % 8);
  if (!c->fence_ev[slot]) CK(c, hipEventCreateWithFlags(&c->fence_ev[slot], hipEventDisableTiming));
  CK(c, hipEventRecord(c->fence_ev[slot], c->stream));
  *ticket = c->fence_next++;
  return B2P_OK;
}

int b2p_fence_wait(b2p_ctx_t *c, uint64_t ticket) {
  if (!c || ticket >= c->fence_next) return B2P_EINVAL;
  LIVE(c);
  CK(c, hipSetDevice(c->device));
  if (c->fence_next - ticket > 8) {  // its event was recorded again since
    CK(c, hipStreamSynchronize(c->stream));
    return B2P_OK;
  }
  CK(c, hipEventSynchronize(c->fence_ev[ticket % 8]));
  return B2P_OK;
}

int b2p_fence_done(b2p_ctx_t *c, uint64_t ticket) {
  if (!c || ticket >= c->fence_next) return B2P_EINVAL;
  LIVE(c);
  CK(c, hipSetDevice(c->device));
  if (c->fence_next - ticket > 8) {  // its event was recorded again since: ask the stream
    const hipError_t e = hipStreamQuery(c->stream);
    if (e == hipErrorNotReady) return 0;
    CK(c, e);
    return 1;
  }
  const hipError_t e = hipEventQuery(c->fence_ev[ticket % 8]);
  if (e == hipErrorNotReady) return 0;
  CK(c, e);
  return 1;
}

int b2p_flush(b2p_ctx_t *c) {
  if (!c) return B2P_EINVAL;
  LIVE(c);
  CK(c, hipSetDevice(c->device));
  return flush_pending(c);
}

int b2p_sync(b2p_ctx_t *c) {
  if (!c) return B2P_EINVAL;
  LIVE(c);
  CK(c, hipSetDevice(c->device));
  int rc = flush_pending(c);
  if (rc != B2P_OK) return rc;
  CK(c, hipStreamSynchronize(c->stream));
#ifdef B2P_DEBUG
  if ((rc = dbg_check(c)) != B2P_OK) return rc;
#endif
  return B2P_OK;
}

int b2p_finish(b2p_ctx_t *c, float *out) {
  int rc = b2p_finish_async(c, out, 0);
  if (rc != B2P_OK && rc != B2P_EPARTIAL) return rc;
  int rs = b2p_sync(c);
  return rs != B2P_OK ? rs : rc;
}

int b2p_integrate(b2p_ctx_t *c, const void *buf, size_t nbytes, int is_device, float *out,
                  int out_is_device) {
  if (!c || !out) return B2P_EINVAL;
  LIVE(c);
  if (c->samples != 0) return set_err(c, B2P_EINVAL, "b2p_integrate with a push pending");
  if (nbytes != c->block_bytes)
    return set_err(c, nbytes % c->frame_bytes ? B2P_ERAGGED : B2P_EINVAL,
                   "b2p_integrate needs exactly one integration (%llu B), got %zu",
                   (unsigned long long)c->block_bytes, nbytes);
  if (!is_device || !c->fuse) {  // staged / plain push, then the finalize kernel
    int rc = b2p_push(c, buf, nbytes, is_device);
    if (rc != B2P_OK) return rc;
    return b2p_finish_async(c, out, out_is_device);
  }
  if (!buf) return set_err(c, B2P_EINVAL, "null buffer");
  if ((uintptr_t)buf % 16) return set_err(c, B2P_EALIGN, "device span not 16-B aligned");
  CK(c, hipSetDevice(c->device));
  // a deferred finalize that lands in d_out (host output of an earlier
  // finish_async) must not ride on a launch that writes d_out itself
  if (!out_is_device && c->pend.valid && c->pend.dev_out == c->d_out) {
    int rf = flush_pending(c);
    if (rf != B2P_OK) return rf;
  }
  // the launch finalizes its own set in its last workgroup; a deferred
  // finalize of the previous integration rides on it as well
  int rc = enqueue_span(c, buf, nbytes, out_is_device ? out : c->d_out);
  if (rc != B2P_OK) return rc;
  if (!out_is_device)
    CK(c, hipMemcpyAsync(out, c->d_out, (size_t)c->nout * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  c->cur ^= 1;
  return B2P_OK;
}

int b2p_integrate_n(b2p_ctx_t *c, const void *const *bufs, uint32_t nblk, float *out, int out_is_device) {
  if (!c || !bufs || !out || nblk < 1 || nblk > kMaxBlk) return B2P_EINVAL;
  LIVE(c);
  if (c->samples != 0) return set_err(c, B2P_EINVAL, "b2p_integrate_n with a push pending");
  for (uint32_t b = 0; b < nblk; ++b) {
    if (!bufs[b]) return set_err(c, B2P_EINVAL, "null block %u", b);
    if ((uintptr_t)bufs[b] % 16) return set_err(c, B2P_EALIGN, "block %u not 16-B aligned", b);
  }
  CK(c, hipSetDevice(c->device));
  if (!c->d_mrep) {
    const size_t words = 2 * (size_t)kMaxBlk * c->nrep * c->nout;
    if (hipMalloc(&c->d_mrep, words * sizeof(unsigned long long)) != hipSuccess)
      return set_err(c, B2P_ENOMEM, "hipMalloc multi-block replicas");
    CK(c, hipMemsetAsync(c->d_mrep, 0, words * sizeof(unsigned long long), c->stream));
  }
  // host output: one staging row per block (d_out holds one spectrum)
  float *dev_out = out;
  if (!out_is_device) {
    if (!c->d_mout) {
      if (hipMalloc(&c->d_mout, (size_t)kMaxBlk * c->nout * sizeof(unsigned long long)) != hipSuccess)
        return set_err(c, B2P_ENOMEM, "hipMalloc multi-block output");
    }
    dev_out = c->d_mout;
  }
  // the previous launch's finalize rides on this one, as for b2p_integrate
  int rc = enqueue_span(c, bufs[0], c->block_bytes, nullptr, bufs, nblk);
  if (rc != B2P_OK) return rc;
  c->pend.valid = 1;
  c->pend.rep = c->d_mrep + (size_t)c->mbank * kMaxBlk * c->nrep * c->nout;
  c->pend.nblk = nblk;
  c->pend.raw = 0;
  c->pend.dev_out = dev_out;
  c->pend.host_out = out_is_device ? nullptr : out;
  c->mbank ^= 1;
  return B2P_OK;
}

uint32_t b2p_blocks_per_launch(uint64_t block_bytes) {
  const uint64_t n = block_bytes ? B2P_BATCH_BYTES / block_bytes : 1;
  return n < 1 ? 1 : n > kMaxBlk ? (uint32_t)kMaxBlk : (uint32_t)n;
}

int b2p_set_timing(b2p_ctx_t *c, int mode) {
  if (!c || mode < 0 || mode > 2) return B2P_EINVAL;
  LIVE(c);
  CK(c, hipSetDevice(c->device));
  if (c->timing == 2 && mode != 2) {  // close the region, last finalize included
    int rc = flush_pending(c);
    if (rc == B2P_OK) rc = region_mark(c);  // an empty region
    if (rc != B2P_OK) return rc;
    // no host wait: work enqueued next (a collective) follows the region on
    // the stream at once; b2p_get_stats reads the time
    CK(c, hipEventRecord(c->region_b, c->stream));
    c->region_closed = 1;
  }
  if (mode == 2 && c->timing != 2) {  // open a region
    drain_timing(c);  // an earlier region still unread
    if (!c->region_a) CK(c, hipEventCreate(&c->region_a));
    if (!c->region_b) CK(c, hipEventCreate(&c->region_b));
    c->region_open = 1;  // region_a goes in front of the region's first launch
  }
  c->timing = mode;
  return B2P_OK;
}

int b2p_get_stats(b2p_ctx_t *c, b2p_stats_t *s) {
  if (!c || !s) return B2P_EINVAL;
  CK(c, hipSetDevice(c->device));
  drain_timing(c);
  *s = c->stats;
  return B2P_OK;
}

int b2p_reset_stats(b2p_ctx_t *c) {
  if (!c) return B2P_EINVAL;
  drain_timing(c);
  memset(&c->stats, 0, sizeof c->stats);
  return B2P_OK;
}

int b2p_fill_synthetic(b2p_ctx_t *c, void *dev, size_t nbytes, uint64_t seed, uint32_t subband,
                       uint64_t block, uint64_t elem0) {
  if (!c || !dev) return B2P_EINVAL;
  if (nbytes % 16 || (uintptr_t)dev % 16) return set_err(c, B2P_EALIGN, "fill needs 16-B multiples");
  CK(c, hipSetDevice(c->device));
  FillArgs f;
  const uint64_t k_sub = splitmix64_host(seed ^ (0xD1B54A32D192ED03ULL * ((uint64_t)subband + 1)));
  f.key = splitmix64_host(k_sub ^ (0x8CB92BA72F3D8DD7ULL * (block + 1)));
  f.elem0 = elem0;
  f.elem_bytes = c->g.nbit / 8;
  f.big_endian = c->g.big_endian;
  f.comp = c->g.npol * c->g.ndim;
  f.nchan_chunk = c->g.nchan_chunk;
  f.wpc = (uint64_t)c->g.nsamp_df * c->g.nchan_chunk;
  f.wpf = f.wpc * c->g.nchunk;
  f.nchan = c->nchan;
  f.amp = c->g.nbit == 8 ? 35 : 3464;
  CK(c, launch_fill((uint4 *)dev, nbytes / 16, f, c->stream));
  return B2P_OK;
}

int b2p_assemble(b2p_ctx_t *c, const void *dfs, uint64_t ndf, uint32_t df_bytes,
                 const uint8_t *chunk_of_df, uint64_t ref_idf, uint64_t ref_sec, void *block,
                 uint64_t block_ndf, uint32_t nchunk, unsigned long long *counts) {
  if (!c || (ndf && (!dfs || !chunk_of_df)) || !block || !counts) return B2P_EINVAL;
  LIVE(c);
  // chunk byte 255 always marks "no chunk" (paf_capture), so at most 255
  if (df_bytes != 7232 || !nchunk || nchunk > 255 || !block_ndf)
    return set_err(c, B2P_EINVAL, "b2p_assemble: 7232-B frames, 1..255 chunks");
  if ((uintptr_t)dfs % 16 || (uintptr_t)block % 16)
    return set_err(c, B2P_EALIGN, "b2p_assemble: 16-B aligned buffers");
  CK(c, hipSetDevice(c->device));
  AssembleArgs a;
  a.dfs = (const unsigned char *)dfs;
  a.ndf = ndf;
  a.df_bytes = df_bytes;
  a.hdr_bytes = 64;
  a.chunk_of_df = chunk_of_df;
  a.ref_idf = ref_idf;
  a.ref_sec = ref_sec;
  a.block = (unsigned char *)block;
  a.block_ndf = block_ndf;
  a.nchunk = nchunk;
  a.counts = counts;
  if (int rm = region_mark(c)) return rm;  // a timing region may open with an assembly
  CK(c, launch_assemble(a, (uint32_t)c->tun.assemble_grid, c->stream));
  return B2P_OK;
}

int b2p_dev_alloc(b2p_ctx_t *c, void **dev, size_t bytes) {
  if (!c || !dev) return B2P_EINVAL;
  CK(c, hipSetDevice(c->device));
  if (hipMalloc(dev, bytes ? bytes : 16) != hipSuccess) return set_err(c, B2P_ENOMEM, "hipMalloc %zu", bytes);
  return B2P_OK;
}

int b2p_dev_free(b2p_ctx_t *c, void *dev) {
  if (!c) return B2P_EINVAL;
  CK(c, hipSetDevice(c->device));
  CK(c, hipStreamSynchronize(c->stream));
  if (dev) CK(c, hipFree(dev));
  return B2P_OK;
}

int b2p_memset(b2p_ctx_t *c, void *dev, int value, size_t bytes) {
  if (!c || (!dev && bytes)) return B2P_EINVAL;
  if (!bytes) return B2P_OK;
  CK(c, hipSetDevice(c->device));
  if (int rm = region_mark(c)) return rm;
  CK(c, hipMemsetAsync(dev, value, bytes, c->stream));
  return B2P_OK;
}

int b2p_memcpy(b2p_ctx_t *c, void *dst, const void *src, size_t bytes, int kind) {
  if (!c || !dst || !src) return B2P_EINVAL;
  hipMemcpyKind k = kind == 1 ? hipMemcpyHostToDevice
                              : (kind == 2 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice);
  if (kind < 1 || kind > 3) return B2P_EINVAL;
  CK(c, hipSetDevice(c->device));
  CK(c, hipStreamSynchronize(c->stream));
  CK(c, hipMemcpy(dst, src, bytes, k));
  return B2P_OK;
}

#ifdef B2P_TEST_HOOKS
// Test build only (lib/hooks/libpafb2p.so, -DB2P_TEST_HOOKS): the next
// host-span push fails at staging chunk `chunk` after the earlier chunks were
// enqueued, as a HIP error would.  The release library has no such entry.
int b2p_test_inject_push_fail(b2p_ctx_t *c, long chunk) {
  if (!c) return B2P_EINVAL;
  c->inject_push_fail = chunk;
  return B2P_OK;
}
#endif

#ifdef B2P_DEBUG
// Debug build only (lib/debug/libpafb2p.so, -DB2P_DEBUG): 1.
int b2p_debug_build(void) { return 1; }
#ifdef B2P_TEST_HOOKS
// Debug + test build: the bound the kernels check span loads against is
// lowered by `vectors` on later launches, so the last rows of a span read
// as out-of-bounds loads -- the detector is exercised without any access
// outside real memory (tests/debug_build_checks.py).
int b2p_test_debug_shrink_bound(b2p_ctx_t *c, long vectors) {
  if (!c || vectors < 0) return B2P_EINVAL;
  c->dbg_shrink = vectors;
  return B2P_OK;
}
#endif
#endif

}  // extern "C"
