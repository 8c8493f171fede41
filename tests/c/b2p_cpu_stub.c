/* tests/c/b2p_cpu_stub.c -- TEST DOUBLE, never part of a product library.
 *
 * A CPU stand-in for the include/b2p.h entry points that the stage
 * (csrc/host/paf_baseband2power.c) calls, so that the stage's host threads
 * -- worker (-n N, host rings), worker_split (-t N), worker_gather_dev and
 * run_device_pipelined (GPU-resident rings, reached in a test build with
 * -DB2P_TEST_HOST_RING_AS_DEVICE) -- run under ThreadSanitizer on a machine
 * without a GPU (tests/test_sanitizers.py, tests/test_stage_stub_random.py).
 * The product's libpafb2p.so is HIP only and has no CPU path (DESIGN.md
 * section 1); this file is linked into test executables only.
 *
 * Semantics kept: exact uint64 sums per output, one RNE rounding to fp32
 * (mean: (double)sum / nsamp_int), npol_out 1 or 2, partial-integration and
 * ragged-push codes, member-major gathers, summed time-split partials.
 * Layouts: int8, little-endian int16 and BMF's big-endian int16 (each 8-B
 * word BSWAP_64-decoded, cudautil.cuh:118-125: X in bytes 4-7, Y in 0-3).
 * For paf_dfdb and paf_capture (tests/test_frames_stub.py) also
 * b2p_memset and b2p_assemble, on the context's queue like the rest: a frame
 * is placed where capture.c:540 puts it, its index from libpafdada's
 * b2p_df_index (capture.c:562-568), with the library's counts. 
 *
 * The stream model.  Every context owns a queue standing for its HIP stream
 * and every group one for its own gather streams (b2p_group_gather_async).
 * Work is enqueued as the library enqueues it and keeps the library's
 * deferrals: b2p_finish_async / b2p_integrate_n leave a pending finalize
 * that the next launch, b2p_flush or b2p_sync enqueues (b2p_ctx.hip
 * finish_common, enqueue_span's carried finalize); a device span is READ
 * WHEN ITS SUM RUNS, not when it is pushed; a host span is copied before
 * b2p_push returns, as push_host's staging does.  Fences are tickets over the
 * queue with the library's ring of 8 events, and the library's ticket
 * contracts are enforced with its codes: a fence wait on a ticket not yet
 * issued, a gather behind a member ticket that is not one of its last 8, a
 * group wait on a gather not yet issued are B2P_EINVAL (b2p_fence_wait,
 * b2p_internal_fence_event, b2p_group_wait).
 *
 * B2P_STUB_NDEV=N (environment, default 1): N devices, so a stage with
 * members on distinct devices takes the RCCL group path; a group opened in
 * RCCL mode (mode 0) with two members on one device is refused, as RCCL
 * refuses it ("Duplicate GPU detected"), naming the call.
 *
 * B2P_STUB_FAIL=name:n[,name:n...] (environment): the n-th call (1-based,
 * process-wide) of entry point `name` fails with B2P_EHIP as a HIP error
 * would, so the stage's failure paths run: every member stops, the output
 * transfer ends, the ERR line reaches stderr, nothing hangs.
 *
 * B2P_STUB_DELAY_US=D (environment): each queue runs on a thread of its own
 * and sleeps 0..D us before every piece of work, so the stage's fences,
 * held blocks and gathers are exercised against work that completes late --
 * a block released to its writer before the sum that reads it has run is
 * summed after the writer refilled it, and its spectrum is wrong.  Unset or
 * 0: work runs when it is enqueued (every call finished on return). */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "b2p.h"
#include "b2p_df.h"

enum { OP_SUM, OP_SUMN, OP_FIN, OP_CONV, OP_COPY, OP_WAIT, OP_REDUCE, OP_FREE, OP_SET, OP_ASM };

typedef struct queue queue_t;

typedef struct op {
  int kind;
  uint64_t seq;
  struct op *next;
  const b2p_geom_t *g;
  const void *src[B2P_MAX_BLOCKS]; /* SUM: one span; SUMN: nblk blocks; COPY: src[0] */
  uint64_t nbytes;                 /* SUM / COPY bytes */
  uint32_t nblk;
  uint64_t *acc;                   /* SUM / SUMN / FIN: accumulator set(s), nout each */
  uint64_t nout;
  void *dst;                       /* FIN / CONV / COPY / REDUCE destination */
  int raw;                         /* FIN: uint64 sums out instead of fp32 */
  const uint64_t *sums;            /* CONV input */
  uint64_t nsamp;                  /* FIN / CONV: samples of one integration */
  void *owned;                     /* freed once the op ran (a host span's staging copy) */
  queue_t *other;                  /* WAIT: until other->done >= wait_seq */
  uint64_t wait_seq;
  uint64_t *const *parts;          /* REDUCE inputs (count each) */
  int nparts;
  int value;                       /* SET: the byte */
  const uint8_t *chunks;           /* ASM: chunk of each frame (src[0]: the frames, nbytes: their count) */
  uint64_t ref_idf, ref_sec, block_ndf;
  uint32_t nchunk;
  unsigned long long *counts;      /* ASM: nchunk + 3, accumulated */
} op_t;

struct queue {
  pthread_mutex_t mu;
  pthread_cond_t cv;
  op_t *head, *tail;
  uint64_t enq, done;
  pthread_t th;
  int async, stop;
  unsigned delay_us, seed;
};

static pthread_mutex_t g_inj_mu = PTHREAD_MUTEX_INITIALIZER;
static struct {
  char name[48];
  int n, calls;
} g_inj[8];
static int g_ninj = -1;

/* 1 when this call of `name` is the one B2P_STUB_FAIL names */
static int inject(const char *name) {
  int hit = 0;
  pthread_mutex_lock(&g_inj_mu);
  if (g_ninj < 0) {
    g_ninj = 0;
    const char *e = getenv("B2P_STUB_FAIL");
    char buf[256];
    snprintf(buf, sizeof buf, "%s", e ? e : "");
    for (char *save = NULL, *t = strtok_r(buf, ",", &save); t && g_ninj < 8; t = strtok_r(NULL, ",", &save)) {
      char *colon = strchr(t, ':');
      if (!colon) continue;
      *colon = 0;
      snprintf(g_inj[g_ninj].name, sizeof g_inj[g_ninj].name, "%s", t);
      g_inj[g_ninj].n = atoi(colon + 1);
      g_ninj++;
    }
  }
  for (int i = 0; i < g_ninj; i++)
    if (!strcmp(g_inj[i].name, name) && ++g_inj[i].calls == g_inj[i].n) hit = 1;
  pthread_mutex_unlock(&g_inj_mu);
  return hit;
}

#define INJECT(name)                                                        \
  do {                                                                      \
    if (inject(name)) {                                                     \
      fprintf(stderr, "b2p_cpu_stub: injected failure of %s\n", name);     \
      return B2P_EHIP;                                                      \
    }                                                                       \
  } while (0)

static unsigned stub_delay_us(void) {
  const char *e = getenv("B2P_STUB_DELAY_US");
  return e ? (unsigned)strtoul(e, NULL, 10) : 0;
}

static float to_fp32(const b2p_geom_t *g, uint64_t sum, uint64_t nsamp) {
  return g->mean ? (float)((double)sum / (double)nsamp) : (float)(double)sum;
}

static uint64_t word_bytes(const b2p_geom_t *g) { return (uint64_t)g->npol * g->ndim * (g->nbit / 8); }

uint64_t b2p_frame_bytes(const b2p_geom_t *g) {
  return (uint64_t)g->nchunk * g->nsamp_df * g->nchan_chunk * word_bytes(g);
}

/* component k of pol p's (re, im) pair at element i (one component per int) */
static int64_t comp(const b2p_geom_t *g, const void *buf, uint64_t i) {
  if (g->nbit == 8) return ((const int8_t *)buf)[i];
  if (!g->big_endian) return ((const int16_t *)buf)[i];
  /* BSWAP_64 of the word holding element i: lane k of the swapped word is
   * the big-endian int16 at bytes 6-2k, 7-2k of the raw word */
  const uint8_t *w = (const uint8_t *)buf + (i / 4) * 8;
  const unsigned k = (unsigned)(i % 4);
  return (int16_t)(uint16_t)((w[6 - 2 * k] << 8) | w[7 - 2 * k]);
}

/* [frame][chunk][samp][chan][pol][re,im] -> acc[chan*npol_out + pol?] */
static void sum_span(const b2p_geom_t *g, const void *buf, uint64_t nbytes, uint64_t *acc) {
  const uint64_t frames = nbytes / b2p_frame_bytes(g);
  uint64_t i = 0;
  for (uint64_t f = 0; f < frames; f++)
    for (uint32_t c = 0; c < g->nchunk; c++)
      for (uint32_t s = 0; s < g->nsamp_df; s++)
        for (uint32_t ch = 0; ch < g->nchan_chunk; ch++)
          for (uint32_t p = 0; p < 2; p++, i += 2) {
            const int64_t re = comp(g, buf, i), im = comp(g, buf, i + 1);
            const uint64_t o = ((uint64_t)c * g->nchan_chunk + ch) * g->npol_out + (g->npol_out == 2 ? p : 0);
            acc[o] += (uint64_t)(re * re + im * im);
          }
}

static void run_op(op_t *o) {
  switch (o->kind) {
    case OP_SUM: sum_span(o->g, o->src[0], o->nbytes, o->acc); break;
    case OP_SUMN:
      for (uint32_t b = 0; b < o->nblk; b++) sum_span(o->g, o->src[b], o->nbytes, o->acc + (size_t)b * o->nout);
      break;
    case OP_FIN: /* replicas -> output, then re-zeroed for the set's next use */
      for (uint64_t i = 0; i < (uint64_t)o->nblk * o->nout; i++) {
        if (o->raw)
          ((uint64_t *)o->dst)[i] = o->acc[i];
        else
          ((float *)o->dst)[i] = to_fp32(o->g, o->acc[i], o->nsamp);
        o->acc[i] = 0;
      }
      break;
    case OP_CONV:
      for (uint64_t i = 0; i < o->nout; i++) ((float *)o->dst)[i] = to_fp32(o->g, o->sums[i], o->nsamp);
      break;
    case OP_COPY: memcpy(o->dst, o->src[0], o->nbytes); break;
    case OP_WAIT:
      pthread_mutex_lock(&o->other->mu);
      while (o->other->done < o->wait_seq) pthread_cond_wait(&o->other->cv, &o->other->mu);
      pthread_mutex_unlock(&o->other->mu);
      break;
    case OP_REDUCE:
      for (uint64_t i = 0; i < o->nout; i++) {
        uint64_t t = 0;
        for (int r = 0; r < o->nparts; r++) t += o->parts[r][i];
        ((uint64_t *)o->dst)[i] = t;
      }
      break;
    case OP_FREE: break;
    case OP_SET: memset(o->dst, o->value, o->nbytes); break;
    case OP_ASM: {
      b2p_df_hdr_t ref = {0};
      ref.idf = o->ref_idf;
      ref.sec = o->ref_sec;
      for (uint64_t d = 0; d < o->nbytes; d++) {
        const uint8_t *df = (const uint8_t *)o->src[0] + d * B2P_DF_BYTES;
        b2p_df_hdr_t h;
        b2p_df_decode(df, &h);
        const int64_t idf = b2p_df_index(&h, &ref);
        const uint32_t ch = o->chunks[d];
        if (ch >= o->nchunk) {
          o->counts[o->nchunk + 2]++;
        } else if (idf < 0) {
          o->counts[o->nchunk]++;
        } else if ((uint64_t)idf >= o->block_ndf) {
          o->counts[o->nchunk + 1]++;
        } else {
          memcpy((uint8_t *)o->dst + ((uint64_t)idf * o->nchunk + ch) * B2P_DF_PAYLOAD_BYTES,
                 df + B2P_DF_HDR_BYTES, B2P_DF_PAYLOAD_BYTES);
          o->counts[ch]++;
        }
      }
      break;
    }
  }
  free(o->owned);
}

static void *queue_main(void *arg) {
  queue_t *q = arg;
  pthread_mutex_lock(&q->mu);
  for (;;) {
    while (!q->head && !q->stop) pthread_cond_wait(&q->cv, &q->mu);
    if (!q->head) break;
    op_t *o = q->head;
    pthread_mutex_unlock(&q->mu);
    if (q->delay_us) {
      const unsigned us = rand_r(&q->seed) % (q->delay_us + 1);
      nanosleep(&(struct timespec){us / 1000000, (long)(us % 1000000) * 1000}, NULL);
    }
    run_op(o);
    pthread_mutex_lock(&q->mu);
    q->head = o->next;
    if (!q->head) q->tail = NULL;
    q->done = o->seq;
    free(o);
    pthread_cond_broadcast(&q->cv);
  }
  pthread_mutex_unlock(&q->mu);
  return NULL;
}

static int queue_init(queue_t *q, unsigned seed) {
  memset(q, 0, sizeof *q);
  pthread_mutex_init(&q->mu, NULL);
  pthread_cond_init(&q->cv, NULL);
  q->delay_us = stub_delay_us();
  q->seed = seed;
  q->async = q->delay_us > 0;
  if (q->async && pthread_create(&q->th, NULL, queue_main, q) != 0) return B2P_ENOMEM;
  return B2P_OK;
}

static uint64_t enqueue(queue_t *q, op_t *o) {
  pthread_mutex_lock(&q->mu);
  o->seq = ++q->enq;
  const uint64_t seq = o->seq;
  if (!q->async) { /* run now, outside the lock (a WAIT takes another queue's): done as issued */
    pthread_mutex_unlock(&q->mu);
    run_op(o);
    free(o);
    pthread_mutex_lock(&q->mu);
    if (q->done < seq) q->done = seq;
    pthread_cond_broadcast(&q->cv);
  } else {
    o->next = NULL;
    if (q->tail)
      q->tail->next = o;
    else
      q->head = o;
    q->tail = o;
    pthread_cond_broadcast(&q->cv);
  }
  pthread_mutex_unlock(&q->mu);
  return seq;
}

static void queue_wait(queue_t *q, uint64_t seq) {
  pthread_mutex_lock(&q->mu);
  while (q->done < seq) pthread_cond_wait(&q->cv, &q->mu);
  pthread_mutex_unlock(&q->mu);
}

static uint64_t queue_pos(queue_t *q) {
  pthread_mutex_lock(&q->mu);
  const uint64_t e = q->enq;
  pthread_mutex_unlock(&q->mu);
  return e;
}

static int queue_reached(queue_t *q, uint64_t seq) {
  pthread_mutex_lock(&q->mu);
  const int d = q->done >= seq;
  pthread_mutex_unlock(&q->mu);
  return d;
}

static void queue_fini(queue_t *q) {
  queue_wait(q, queue_pos(q));
  if (q->async) {
    pthread_mutex_lock(&q->mu);
    q->stop = 1;
    pthread_cond_broadcast(&q->cv);
    pthread_mutex_unlock(&q->mu);
    pthread_join(q->th, NULL);
  }
  pthread_cond_destroy(&q->cv);
  pthread_mutex_destroy(&q->mu);
}

static op_t *new_op(int kind) {
  op_t *o = calloc(1, sizeof *o);
  if (!o) abort(); /* test double: out of memory ends the test run loudly */
  o->kind = kind;
  return o;
}

/* ---- contexts ---------------------------------------------------------- */

struct b2p_ctx {
  b2p_geom_t g;
  uint64_t nchan, nout, frame_bytes, block_bytes;
  uint64_t samples;  /* pushed into the open integration (host-side count, as the library keeps it) */
  uint64_t *rep[2];  /* accumulator sets of single integrations, alternating (c->cur) */
  uint64_t *mrep[2]; /* b2p_integrate_n banks: B2P_MAX_BLOCKS sets each (c->mbank) */
  int cur, mbank, device;
  struct {
    int valid, raw;
    uint64_t *acc;
    uint32_t nblk;
    void *out;
  } pend; /* a finalize not yet enqueued (b2p_ctx.hip pend) */
  uint64_t fence_next, fence_seq[8];
  queue_t q;
};

struct b2p_group {
  b2p_ctx_t *m[64];
  int n, mode;
  queue_t q; /* the group's own gather streams */
  uint64_t gnext, gseq[8];
};

static const char *k_err[] = {"ok", "invalid argument", "ragged push", "overflow", "partial integration",
                              "no device", "HIP error", "out of memory", "misaligned", "failed",
                              "timed out"};

const char *b2p_strerror(int code) { return code <= 0 && code >= -10 ? k_err[-code] : "unknown"; }
const char *b2p_last_error(const b2p_ctx_t *ctx) { (void)ctx; return "b2p_cpu_stub"; }
const char *b2p_group_last_error(const b2p_group_t *grp);

int b2p_geom_bmf(b2p_geom_t *g) {
  memset(g, 0, sizeof *g);
  *g = (b2p_geom_t){16, 1, 48, 128, 7, 2, 2, 1, 1u << 20, 0, 0};
  return B2P_OK;
}

int b2p_geom_check(const b2p_geom_t *g) {
  if (!g || (g->nbit != 8 && g->nbit != 16) || g->big_endian > 1 || (g->big_endian && g->nbit != 16) ||
      g->npol != 2 || g->ndim != 2 ||
      (g->npol_out != 1 && g->npol_out != 2) || !g->nchunk || !g->nsamp_df || !g->nchan_chunk ||
      !g->nsamp_int || g->nsamp_int % g->nsamp_df || g->reserved)
    return B2P_EINVAL;
  return B2P_OK;
}

static int stub_ndev(void) {
  const char *e = getenv("B2P_STUB_NDEV");
  const int n = e ? atoi(e) : 1;
  return n > 0 ? n : 1;
}

static const char *g_group_err = "b2p_cpu_stub";

int b2p_device_count(int *count) {
  *count = stub_ndev();
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
  static unsigned nopen;
  if (!ctx || b2p_geom_check(g)) return B2P_EINVAL;
  if (device < 0 || device >= stub_ndev()) return B2P_ENODEV;
  b2p_ctx_t *c = calloc(1, sizeof *c);
  if (!c) return B2P_ENOMEM;
  c->g = *g;
  c->device = device;
  c->nchan = (uint64_t)g->nchunk * g->nchan_chunk;
  c->nout = c->nchan * g->npol_out;
  c->frame_bytes = b2p_frame_bytes(g);
  c->block_bytes = c->frame_bytes * (g->nsamp_int / g->nsamp_df);
  for (int i = 0; i < 2; i++) {
    c->rep[i] = calloc(c->nout, sizeof(uint64_t));
    c->mrep[i] = calloc((size_t)B2P_MAX_BLOCKS * c->nout, sizeof(uint64_t));
  }
  if (!c->rep[0] || !c->rep[1] || !c->mrep[0] || !c->mrep[1] ||
      queue_init(&c->q, 0x9e3779b9u * (__atomic_add_fetch(&nopen, 1, __ATOMIC_RELAXED))) != B2P_OK) {
    for (int i = 0; i < 2; i++) free(c->rep[i]), free(c->mrep[i]);
    free(c);
    return B2P_ENOMEM;
  }
  *ctx = c;
  return B2P_OK;
}

int b2p_close(b2p_ctx_t *c) {
  if (!c) return B2P_OK;
  queue_fini(&c->q);
  for (int i = 0; i < 2; i++) free(c->rep[i]), free(c->mrep[i]);
  free(c);
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

int b2p_unregister_host(b2p_ctx_t *c, void *base) { /* drains the context first, as the library does */
  (void)base;
  if (!c) return B2P_EINVAL;
  queue_wait(&c->q, queue_pos(&c->q));
  return B2P_OK;
}

int b2p_dev_alloc(b2p_ctx_t *ctx, void **dev, size_t bytes) {
  (void)ctx;
  *dev = aligned_alloc(64, (bytes + 63) / 64 * 64);
  return *dev ? B2P_OK : B2P_ENOMEM;
}

int b2p_dev_free(b2p_ctx_t *c, void *dev) { /* after the stream, as hipStreamSynchronize + hipFree */
  if (!c) return B2P_EINVAL;
  queue_wait(&c->q, queue_pos(&c->q));
  free(dev);
  return B2P_OK;
}

int b2p_memcpy(b2p_ctx_t *c, void *dst, const void *src, size_t bytes, int kind) {
  INJECT("b2p_memcpy");
  if (!c || !dst || !src || kind < 1 || kind > 3) return B2P_EINVAL;
  queue_wait(&c->q, queue_pos(&c->q)); /* the library syncs the stream, then copies */
  memcpy(dst, src, bytes);
  return B2P_OK;
}

int b2p_memset(b2p_ctx_t *c, void *dev, int value, size_t bytes) {
  INJECT("b2p_memset");
  if (!c || (!dev && bytes)) return B2P_EINVAL;
  op_t *o = new_op(OP_SET);
  o->dst = dev;
  o->value = value;
  o->nbytes = bytes;
  enqueue(&c->q, o);
  return B2P_OK;
}

/* not modelled: the synthetic generator (paf_dfdb -R, bench.py) runs on the
 * GPU only (tests/test_gpu_device_ring.py) */
int b2p_fill_synthetic(b2p_ctx_t *c, void *dev, size_t nbytes, uint64_t seed, uint32_t subband, uint64_t block,
                       uint64_t elem0) {
  (void)c, (void)dev, (void)nbytes, (void)seed, (void)subband, (void)block, (void)elem0;
  return B2P_EINVAL;
}

int b2p_assemble(b2p_ctx_t *c, const void *dfs, uint64_t ndf, uint32_t df_bytes, const uint8_t *chunk_of_df,
                 uint64_t ref_idf, uint64_t ref_sec, void *block, uint64_t block_ndf, uint32_t nchunk,
                 unsigned long long *counts) {
  INJECT("b2p_assemble");
  if (!c || (ndf && (!dfs || !chunk_of_df)) || !block || !counts || df_bytes != B2P_DF_BYTES || !nchunk ||
      nchunk > 255)
    return B2P_EINVAL;
  op_t *o = new_op(OP_ASM);
  o->src[0] = dfs; /* read when the assembly runs, as the kernel reads device memory */
  o->nbytes = ndf;
  o->chunks = chunk_of_df;
  o->ref_idf = ref_idf;
  o->ref_sec = ref_sec;
  o->dst = block;
  o->block_ndf = block_ndf;
  o->nchunk = nchunk;
  o->counts = counts;
  enqueue(&c->q, o);
  return B2P_OK;
}

static void flush_pending(b2p_ctx_t *c) {
  if (!c->pend.valid) return;
  op_t *o = new_op(OP_FIN);
  o->g = &c->g;
  o->acc = c->pend.acc;
  o->nblk = c->pend.nblk;
  o->nout = c->nout;
  o->dst = c->pend.out;
  o->raw = c->pend.raw;
  o->nsamp = c->g.nsamp_int;
  enqueue(&c->q, o);
  c->pend.valid = 0;
}

int b2p_push(b2p_ctx_t *c, const void *buf, size_t nbytes, int is_device) {
  if (!c) return B2P_EINVAL;
  INJECT("b2p_push");
  if (nbytes == 0) return B2P_OK;
  if (!buf) return B2P_EINVAL;
  if (nbytes % c->frame_bytes) return B2P_ERAGGED;
  const uint64_t samples = nbytes / c->frame_bytes * c->g.nsamp_df;
  if (c->samples + samples > c->g.nsamp_int) return B2P_EOVERFLOW;
  if (is_device && (uintptr_t)buf % 16) return B2P_EALIGN;
  flush_pending(c); /* the previous integration's finalize rides ahead of this launch */
  op_t *o = new_op(OP_SUM);
  o->g = &c->g;
  o->nbytes = nbytes;
  o->acc = c->rep[c->cur];
  if (is_device) {
    o->src[0] = buf; /* read when the sum runs */
  } else {            /* staged: the span is copied before b2p_push returns */
    o->owned = malloc(nbytes);
    if (!o->owned) abort();
    memcpy(o->owned, buf, nbytes);
    o->src[0] = o->owned;
  }
  enqueue(&c->q, o);
  c->samples += samples;
  return B2P_OK;
}

static int finish_common(b2p_ctx_t *c, void *out, int raw) {
  if (!c || !out) return B2P_EINVAL;
  flush_pending(c); /* two finishes in a row: the first runs alone */
  c->pend.valid = 1;
  c->pend.raw = raw;
  c->pend.acc = c->rep[c->cur];
  c->pend.nblk = 1;
  c->pend.out = out;
  c->cur ^= 1;
  const uint64_t got = c->samples;
  c->samples = 0;
  return got == c->g.nsamp_int ? B2P_OK : B2P_EPARTIAL;
}

int b2p_finish_async(b2p_ctx_t *c, float *out, int out_is_device) {
  INJECT("b2p_finish_async");
  (void)out_is_device;
  return finish_common(c, out, 0);
}

int b2p_finish_partial_async(b2p_ctx_t *c, uint64_t *sums, int sums_is_device) {
  INJECT("b2p_finish_partial_async");
  (void)sums_is_device;
  return finish_common(c, sums, 1);
}

int b2p_finalize_sums(b2p_ctx_t *c, const uint64_t *sums, uint64_t nspec, uint64_t nsamp_total, float *out) {
  INJECT("b2p_finalize_sums");
  if (!c || !sums || !out) return B2P_EINVAL;
  flush_pending(c);
  op_t *o = new_op(OP_CONV);
  o->g = &c->g;
  o->sums = sums;
  o->nout = nspec * c->nout;
  o->dst = out;
  o->nsamp = nsamp_total ? nsamp_total : c->g.nsamp_int;
  enqueue(&c->q, o);
  return B2P_OK;
}

int b2p_integrate(b2p_ctx_t *c, const void *buf, size_t nbytes, int is_device, float *out, int out_is_device) {
  if (!c || !out) return B2P_EINVAL;
  INJECT("b2p_integrate");
  if (c->samples) return B2P_EINVAL; /* "b2p_integrate with a push pending" */
  if (nbytes != c->block_bytes) return nbytes % c->frame_bytes ? B2P_ERAGGED : B2P_EINVAL;
  int rc = b2p_push(c, buf, nbytes, is_device);
  return rc == B2P_OK ? b2p_finish_async(c, out, out_is_device) : rc;
}

int b2p_integrate_n(b2p_ctx_t *c, const void *const *bufs, uint32_t nblk, float *out, int out_is_device) {
  (void)out_is_device;
  INJECT("b2p_integrate_n");
  if (!c || !bufs || !out || !nblk || nblk > B2P_MAX_BLOCKS) return B2P_EINVAL;
  if (c->samples) return B2P_EINVAL;
  for (uint32_t b = 0; b < nblk; b++)
    if (!bufs[b] || (uintptr_t)bufs[b] % 16) return bufs[b] ? B2P_EALIGN : B2P_EINVAL;
  flush_pending(c);
  op_t *o = new_op(OP_SUMN);
  o->g = &c->g;
  o->nblk = nblk;
  o->nbytes = c->block_bytes;
  o->nout = c->nout;
  o->acc = c->mrep[c->mbank];
  for (uint32_t b = 0; b < nblk; b++) o->src[b] = bufs[b];
  enqueue(&c->q, o);
  c->pend.valid = 1;
  c->pend.raw = 0;
  c->pend.acc = c->mrep[c->mbank];
  c->pend.nblk = nblk;
  c->pend.out = out;
  c->mbank ^= 1;
  return B2P_OK;
}

int b2p_fence(b2p_ctx_t *c, uint64_t *ticket) {
  INJECT("b2p_fence");
  if (!c || !ticket) return B2P_EINVAL;
  c->fence_seq[c->fence_next % 8] = queue_pos(&c->q);
  *ticket = c->fence_next++;
  return B2P_OK;
}

int b2p_fence_wait(b2p_ctx_t *c, uint64_t ticket) {
  INJECT("b2p_fence_wait");
  if (!c || ticket >= c->fence_next) return B2P_EINVAL;
  queue_wait(&c->q, c->fence_next - ticket > 8 ? queue_pos(&c->q) : c->fence_seq[ticket % 8]);
  return B2P_OK;
}

int b2p_fence_done(b2p_ctx_t *c, uint64_t ticket) {
  INJECT("b2p_fence_done");
  if (!c || ticket >= c->fence_next) return B2P_EINVAL;
  return queue_reached(&c->q, c->fence_next - ticket > 8 ? queue_pos(&c->q) : c->fence_seq[ticket % 8]);
}

int b2p_flush(b2p_ctx_t *c) {
  INJECT("b2p_flush");
  if (!c) return B2P_EINVAL;
  flush_pending(c);
  return B2P_OK;
}

int b2p_sync(b2p_ctx_t *c) {
  if (!c) return B2P_EINVAL;
  INJECT("b2p_sync");
  flush_pending(c);
  queue_wait(&c->q, queue_pos(&c->q));
  return B2P_OK;
}

/* ---- groups: copies gathered on the group's own queue -------------------- */

const char *b2p_group_last_error(const b2p_group_t *grp) {
  (void)grp;
  return g_group_err;
}

int b2p_group_open_timed(b2p_group_t **grp, b2p_ctx_t *const *ctxs, int n, int mode, int timeout_ms) {
  if (n < 1 || n > 64 || timeout_ms <= 0 || (mode != 0 && mode != 1)) return B2P_EINVAL;
  for (int r = 1; r < n; r++)
    if (ctxs[r]->nout != ctxs[0]->nout) return B2P_EINVAL;
  for (int r = 0; mode == 0 && r < n; r++)
    for (int q = 0; q < r; q++)
      if (ctxs[q]->device == ctxs[r]->device) {
        g_group_err = "ncclCommInitRankConfig: Duplicate GPU detected (b2p_cpu_stub: RCCL members share a device)";
        return B2P_EHIP;
      }
  b2p_group_t *g = calloc(1, sizeof *g);
  if (!g) return B2P_ENOMEM;
  memcpy(g->m, ctxs, (size_t)n * sizeof *ctxs);
  g->n = n;
  g->mode = mode;
  if (queue_init(&g->q, 0x51ed27u) != B2P_OK) {
    free(g);
    return B2P_ENOMEM;
  }
  *grp = g;
  return B2P_OK;
}

int b2p_group_close(b2p_group_t *g) {
  if (!g) return B2P_OK;
  queue_fini(&g->q);
  free(g);
  return B2P_OK;
}

static void wait_behind(b2p_group_t *g, queue_t *member, uint64_t seq) {
  op_t *o = new_op(OP_WAIT);
  o->other = member;
  o->wait_seq = seq;
  enqueue(&g->q, o);
}

static void copy_on(b2p_group_t *g, void *dst, const void *src, uint64_t n) {
  op_t *o = new_op(OP_COPY);
  o->dst = dst;
  o->src[0] = src;
  o->nbytes = n;
  enqueue(&g->q, o);
}

/* behind everything each member has enqueued, its deferred finalize included */
int b2p_group_gather(b2p_group_t *g, float *const *spectra, float *root_out) {
  INJECT("b2p_group_gather");
  if (!g || !spectra || !root_out) return B2P_EINVAL;
  const uint64_t nout = g->m[0]->nout;
  for (int r = 0; r < g->n; r++) {
    flush_pending(g->m[r]);
    wait_behind(g, &g->m[r]->q, queue_pos(&g->m[r]->q));
  }
  for (int r = 0; r < g->n; r++) copy_on(g, root_out + (size_t)r * nout, spectra[r], nout * sizeof(float));
  return B2P_OK;
}

int b2p_group_gather_async(b2p_group_t *g, float *const *spectra, uint32_t nspec, float *root_out,
                           const uint64_t *tickets, float *host_out, uint64_t *gticket) {
  INJECT("b2p_group_gather_async");
  if (!g || !spectra || !root_out || !tickets || !gticket || nspec < 1) return B2P_EINVAL;
  if (g->gnext >= 8) queue_wait(&g->q, g->gseq[(g->gnext - 8) % 8]); /* its event slot is reused */
  for (int r = 0; r < g->n; r++) { /* b2p_internal_fence_event: one of the member's last 8 tickets */
    const b2p_ctx_t *c = g->m[r];
    if (tickets[r] >= c->fence_next || c->fence_next - tickets[r] > 8) {
      fprintf(stderr, "b2p_cpu_stub: gather behind member %d ticket %llu, its fences at %llu\n", r,
              (unsigned long long)tickets[r], (unsigned long long)c->fence_next);
      return B2P_EINVAL;
    }
    wait_behind(g, &g->m[r]->q, c->fence_seq[tickets[r] % 8]);
  }
  const size_t per = (size_t)nspec * g->m[0]->nout;
  for (int r = 0; r < g->n; r++) copy_on(g, root_out + (size_t)r * per, spectra[r], per * sizeof(float));
  if (host_out) copy_on(g, host_out, root_out, (size_t)g->n * per * sizeof(float));
  g->gseq[g->gnext % 8] = queue_pos(&g->q);
  *gticket = g->gnext++;
  return B2P_OK;
}

int b2p_group_wait(b2p_group_t *g, uint64_t gticket) {
  INJECT("b2p_group_wait");
  if (!g || gticket >= g->gnext) return B2P_EINVAL;
  if (g->gnext - gticket > 8) return B2P_OK;
  queue_wait(&g->q, g->gseq[gticket % 8]);
  return B2P_OK;
}

int b2p_group_done(b2p_group_t *g, uint64_t gticket) {
  INJECT("b2p_group_done");
  if (!g || gticket >= g->gnext) return B2P_EINVAL;
  if (g->gnext - gticket > 8) return 1;
  return queue_reached(&g->q, g->gseq[gticket % 8]);
}

int b2p_group_reduce(b2p_group_t *g, uint64_t *const *sums, uint64_t count, uint64_t *root_sum) {
  INJECT("b2p_group_reduce");
  if (!g || !sums || !root_sum || !count) return B2P_EINVAL;
  for (int r = 0; r < g->n; r++) {
    flush_pending(g->m[r]);
    wait_behind(g, &g->m[r]->q, queue_pos(&g->m[r]->q));
  }
  op_t *o = new_op(OP_REDUCE);
  uint64_t **parts = malloc((size_t)g->n * sizeof *parts);
  if (!parts) abort();
  memcpy(parts, sums, (size_t)g->n * sizeof *parts);
  o->owned = parts;
  o->parts = parts;
  o->nparts = g->n;
  o->nout = count;
  o->dst = root_sum;
  enqueue(&g->q, o);
  /* the root's later work (b2p_finalize_sums) is ordered behind the reduce
   * on the root's stream, as ncclReduce on member 0's stream orders it */
  op_t *w = new_op(OP_WAIT);
  w->other = &g->q;
  w->wait_seq = queue_pos(&g->q);
  enqueue(&g->m[0]->q, w);
  return B2P_OK;
}

int b2p_group_sync(b2p_group_t *g) {
  INJECT("b2p_group_sync");
  if (!g) return B2P_EINVAL;
  queue_wait(&g->q, queue_pos(&g->q));
  for (int r = 0; r < g->n; r++) queue_wait(&g->m[r]->q, queue_pos(&g->m[r]->q));
  return B2P_OK;
}
