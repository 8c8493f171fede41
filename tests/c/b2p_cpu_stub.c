/* tests/c/b2p_cpu_stub.c -- TEST DOUBLE, never part of a product library.
 *
 * A CPU stand-in for the include/b2p.h entry points that the stage
 * (csrc/host/paf_baseband2power.c) calls, so that the stage's host threads
 * -- worker (-n N, host rings), worker_split (-t N), worker_gather_dev and
 * run_device_pipelined (GPU-resident rings, reached in a test build with
 * -DB2P_TEST_HOST_RING_AS_DEVICE) -- run under ThreadSanitizer on a machine
 * without a GPU (tests/test_sanitizers.py).  The product's libpafb2p.so is
 * HIP only and has no CPU path; this file is linked
 * into sanitizer test executables only.
 *
 * Semantics kept: exact uint64 sums per output, one RNE rounding to fp32
 * (mean: (double)sum / nsamp_int), npol_out 1 or 2, partial-integration and
 * ragged-push codes, member-major gathers, summed time-split partials.
 * Layouts: int8 and little-endian int16 only (B2P_EINVAL otherwise).  Every
 * call has finished when it returns, so fences, flushes, syncs and group
 * waits are no-ops, and "device" memory is host memory.  A context is used
 * by one thread, as the ABI says; group calls read member buffers that the
 * stage orders with its own barriers. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "b2p.h"

struct b2p_ctx {
  b2p_geom_t g;
  uint64_t nchan, nout, frame_bytes, block_bytes, pending;
  uint64_t *acc;
  uint64_t tickets;
  int device;
};

struct b2p_group {
  b2p_ctx_t *m[64];
  int n;
};

static const char *k_err[] = {"ok", "invalid argument", "ragged push", "overflow", "partial integration",
                              "no device", "HIP error", "out of memory", "misaligned", "failed",
                              "timed out"};

const char *b2p_strerror(int code) { return code <= 0 && code >= -10 ? k_err[-code] : "unknown"; }
const char *b2p_last_error(const b2p_ctx_t *ctx) { (void)ctx; return "b2p_cpu_stub"; }
const char *b2p_group_last_error(const b2p_group_t *grp) { (void)grp; return "b2p_cpu_stub"; }

int b2p_geom_bmf(b2p_geom_t *g) {
  memset(g, 0, sizeof *g);
  *g = (b2p_geom_t){16, 1, 48, 128, 7, 2, 2, 1, 1u << 20, 0, 0};
  return B2P_OK;
}

static uint64_t word_bytes(const b2p_geom_t *g) { return (uint64_t)g->npol * g->ndim * (g->nbit / 8); }

uint64_t b2p_frame_bytes(const b2p_geom_t *g) {
  return (uint64_t)g->nchunk * g->nsamp_df * g->nchan_chunk * word_bytes(g);
}

int b2p_geom_check(const b2p_geom_t *g) {
  if (!g || (g->nbit != 8 && g->nbit != 16) || g->big_endian || g->npol != 2 || g->ndim != 2 ||
      (g->npol_out != 1 && g->npol_out != 2) || !g->nchunk || !g->nsamp_df || !g->nchan_chunk ||
      !g->nsamp_int || g->nsamp_int % g->nsamp_df || g->reserved)
    return B2P_EINVAL;
  return B2P_OK;
}

int b2p_device_count(int *count) {
  *count = 1;
  return B2P_OK;
}

int b2p_device_pci_bus_id(int device, char *buf, int len) {
  snprintf(buf, (size_t)len, "0000:00:%02x.0", device & 0xff);
  return B2P_OK;
}

uint32_t b2p_blocks_per_launch(uint64_t block_bytes) {
  uint64_t n = block_bytes ? B2P_BATCH_BYTES / block_bytes : 1;
  return (uint32_t)(n < 1 ? 1 : n > B2P_MAX_BLOCKS ? B2P_MAX_BLOCKS : n);
}

int b2p_open(b2p_ctx_t **ctx, const b2p_geom_t *g, int device) {
  if (!ctx || device < 0 || b2p_geom_check(g)) return B2P_EINVAL;
  b2p_ctx_t *c = calloc(1, sizeof *c);
  if (!c) return B2P_ENOMEM;
  c->g = *g;
  c->nchan = (uint64_t)g->nchunk * g->nchan_chunk;
  c->nout = c->nchan * g->npol_out;
  c->frame_bytes = b2p_frame_bytes(g);
  c->block_bytes = c->frame_bytes * (g->nsamp_int / g->nsamp_df);
  c->acc = calloc(c->nout, sizeof *c->acc);
  c->device = 0;
  if (!c->acc) {
    free(c);
    return B2P_ENOMEM;
  }
  *ctx = c;
  return B2P_OK;
}

int b2p_close(b2p_ctx_t *ctx) {
  if (ctx) free(ctx->acc);
  free(ctx);
  return B2P_OK;
}

int b2p_get_info(const b2p_ctx_t *ctx, b2p_info_t *info) {
  memset(info, 0, sizeof *info);
  info->nchan = (uint32_t)ctx->nchan;
  info->nout = (uint32_t)ctx->nout;
  info->frame_bytes = ctx->frame_bytes;
  info->block_bytes = ctx->block_bytes;
  info->device = (uint32_t)ctx->device;
  return B2P_OK;
}

int b2p_register_host(b2p_ctx_t *ctx, void *base, size_t bytes) {
  (void)ctx, (void)base, (void)bytes;
  return B2P_OK;
}
int b2p_unregister_host(b2p_ctx_t *ctx, void *base) {
  (void)ctx, (void)base;
  return B2P_OK;
}

int b2p_dev_alloc(b2p_ctx_t *ctx, void **dev, size_t bytes) {
  (void)ctx;
  *dev = aligned_alloc(64, (bytes + 63) / 64 * 64);
  return *dev ? B2P_OK : B2P_ENOMEM;
}
int b2p_dev_free(b2p_ctx_t *ctx, void *dev) {
  (void)ctx;
  free(dev);
  return B2P_OK;
}
int b2p_memcpy(b2p_ctx_t *ctx, void *dst, const void *src, size_t bytes, int kind) {
  (void)ctx, (void)kind;
  memcpy(dst, src, bytes);
  return B2P_OK;
}

/* [frame][chunk][samp][chan][pol][re,im] -> acc[chan*npol_out + pol?] */
int b2p_push(b2p_ctx_t *ctx, const void *buf, size_t nbytes, int is_device) {
  (void)is_device;
  const b2p_geom_t *g = &ctx->g;
  if (nbytes % ctx->frame_bytes) return B2P_ERAGGED;
  const uint64_t frames = nbytes / ctx->frame_bytes;
  if (ctx->pending + frames * g->nsamp_df > g->nsamp_int) return B2P_EOVERFLOW;
  const int8_t *b8 = buf;
  const int16_t *b16 = buf;
  uint64_t i = 0;
  for (uint64_t f = 0; f < frames; f++)
    for (uint32_t c = 0; c < g->nchunk; c++)
      for (uint32_t s = 0; s < g->nsamp_df; s++)
        for (uint32_t ch = 0; ch < g->nchan_chunk; ch++)
          for (uint32_t p = 0; p < 2; p++, i += 2) {
            const int64_t re = g->nbit == 8 ? b8[i] : b16[i], im = g->nbit == 8 ? b8[i + 1] : b16[i + 1];
            const uint64_t o = ((uint64_t)c * g->nchan_chunk + ch) * g->npol_out + (g->npol_out == 2 ? p : 0);
            ctx->acc[o] += (uint64_t)(re * re + im * im);
          }
  ctx->pending += frames * g->nsamp_df;
  return B2P_OK;
}

static float to_fp32(const b2p_ctx_t *ctx, uint64_t sum, uint64_t nsamp) {
  return ctx->g.mean ? (float)((double)sum / (double)nsamp) : (float)(double)sum;
}

int b2p_finish_async(b2p_ctx_t *ctx, float *out, int out_is_device) {
  (void)out_is_device;
  for (uint64_t o = 0; o < ctx->nout; o++) out[o] = to_fp32(ctx, ctx->acc[o], ctx->g.nsamp_int);
  const int rc = ctx->pending == ctx->g.nsamp_int ? B2P_OK : B2P_EPARTIAL;
  memset(ctx->acc, 0, ctx->nout * sizeof *ctx->acc);
  ctx->pending = 0;
  return rc;
}

int b2p_finish_partial_async(b2p_ctx_t *ctx, uint64_t *sums, int sums_is_device) {
  (void)sums_is_device;
  memcpy(sums, ctx->acc, ctx->nout * sizeof *sums);
  const int rc = ctx->pending == ctx->g.nsamp_int ? B2P_OK : B2P_EPARTIAL;
  memset(ctx->acc, 0, ctx->nout * sizeof *ctx->acc);
  ctx->pending = 0;
  return rc;
}

int b2p_finalize_sums(b2p_ctx_t *ctx, const uint64_t *sums, uint64_t nspec, uint64_t nsamp_total,
                      float *out) {
  const uint64_t n = nsamp_total ? nsamp_total : ctx->g.nsamp_int;
  for (uint64_t i = 0; i < nspec * ctx->nout; i++) out[i] = to_fp32(ctx, sums[i], n);
  return B2P_OK;
}

int b2p_integrate(b2p_ctx_t *ctx, const void *buf, size_t nbytes, int is_device, float *out,
                  int out_is_device) {
  if (ctx->pending || nbytes != ctx->block_bytes) return B2P_EINVAL;
  int rc = b2p_push(ctx, buf, nbytes, is_device);
  return rc == B2P_OK ? b2p_finish_async(ctx, out, out_is_device) : rc;
}

int b2p_integrate_n(b2p_ctx_t *ctx, const void *const *bufs, uint32_t nblk, float *out, int out_is_device) {
  if (!nblk || nblk > B2P_MAX_BLOCKS) return B2P_EINVAL;
  for (uint32_t b = 0; b < nblk; b++) {
    int rc = b2p_integrate(ctx, bufs[b], ctx->block_bytes, 1, out + (size_t)b * ctx->nout, out_is_device);
    if (rc != B2P_OK) return rc;
  }
  return B2P_OK;
}

int b2p_fence(b2p_ctx_t *ctx, uint64_t *ticket) {
  *ticket = ++ctx->tickets;
  return B2P_OK;
}
int b2p_fence_wait(b2p_ctx_t *ctx, uint64_t ticket) {
  (void)ctx, (void)ticket;
  return B2P_OK;
}
int b2p_fence_done(b2p_ctx_t *ctx, uint64_t ticket) {
  (void)ctx, (void)ticket;
  return 1;
}
int b2p_flush(b2p_ctx_t *ctx) {
  (void)ctx;
  return B2P_OK;
}
int b2p_sync(b2p_ctx_t *ctx) {
  (void)ctx;
  return B2P_OK;
}

int b2p_group_open_timed(b2p_group_t **grp, b2p_ctx_t *const *ctxs, int n, int mode, int timeout_ms) {
  (void)mode;
  if (n < 1 || n > 64 || timeout_ms <= 0) return B2P_EINVAL;
  for (int r = 1; r < n; r++)
    if (ctxs[r]->nout != ctxs[0]->nout) return B2P_EINVAL;
  b2p_group_t *g = calloc(1, sizeof *g);
  if (!g) return B2P_ENOMEM;
  memcpy(g->m, ctxs, (size_t)n * sizeof *ctxs);
  g->n = n;
  *grp = g;
  return B2P_OK;
}

int b2p_group_close(b2p_group_t *grp) {
  free(grp);
  return B2P_OK;
}

int b2p_group_gather(b2p_group_t *grp, float *const *spectra, float *root_out) {
  const uint64_t nout = grp->m[0]->nout;
  for (int r = 0; r < grp->n; r++) memcpy(root_out + (size_t)r * nout, spectra[r], nout * sizeof(float));
  return B2P_OK;
}

int b2p_group_gather_async(b2p_group_t *grp, float *const *spectra, uint32_t nspec, float *root_out,
                           const uint64_t *tickets, float *host_out, uint64_t *gticket) {
  (void)tickets;
  const size_t per = (size_t)nspec * grp->m[0]->nout;
  for (int r = 0; r < grp->n; r++) memcpy(root_out + (size_t)r * per, spectra[r], per * sizeof(float));
  if (host_out) memcpy(host_out, root_out, (size_t)grp->n * per * sizeof(float));
  *gticket = 1;
  return B2P_OK;
}

int b2p_group_wait(b2p_group_t *grp, uint64_t gticket) {
  (void)grp, (void)gticket;
  return B2P_OK;
}
int b2p_group_done(b2p_group_t *grp, uint64_t gticket) {
  (void)grp, (void)gticket;
  return 1;
}

int b2p_group_reduce(b2p_group_t *grp, uint64_t *const *sums, uint64_t count, uint64_t *root_sum) {
  for (uint64_t i = 0; i < count; i++) {
    uint64_t t = 0;
    for (int r = 0; r < grp->n; r++) t += sums[r][i];
    root_sum[i] = t;
  }
  return B2P_OK;
}

int b2p_group_sync(b2p_group_t *grp) {
  (void)grp;
  return B2P_OK;
}
