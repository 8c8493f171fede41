/*
 * paf_baseband2power -- the baseband->power stage of the PAF pipeline, on
 * MI355X.  Same command line as the reference (paf_baseband2power.cu:17-28,
 * getopt at :40-71) and the same log file and device-index rule (:75-90);
 * the body the reference never wrote (SURVEY.md 3.3 "required"):
 *
 *   attach key_in (lock_read) - read its header - attach key_out (lock_write)
 *   - write the output header - for every input block: push it through the
 *   C ABI of include/b2p.h (H2D overlapped with the gfx950 kernel), release
 *   it, emit one fp32 spectrum into the output ring - until end of data.
 *
 * One input ring block is one integration (the ring is sized so:
 * paf-baseband2power.py:67 / conf:9, NDF 8192 x 48 x 7168 B = 1024x1024
 * samples).  A short final block (EOD) is skipped and logged.
 *
 * -n N (extension): N sub-bands in one process, sub-band r on
 * ring key_in + 0x10*r and GPU d + r, one host thread + one stream each; the
 * N spectra of every integration are gathered to GPU d over RCCL
 * (b2p_group_gather) and written as one N*NCHAN block to key_out.  On
 * GPU-resident rings the members integrate their queued blocks in rounds of
 * one launch each, launches kept in flight, gathered on the group's own
 * streams (worker_gather_dev).
 *
 * DADA library: built by default against libpafdada (include/b2p_dada.h).
 * With -DB2P_PSRDADA it includes PSRDADA's own headers and calls only the
 * PSRDADA subset the reference's hosts use, touching
 * no DADA struct but dada_hdu_t's data_block / header_block, so it links
 * against the real libpsrdada; GPU-resident rings, launches
 * in flight over held blocks and pinning every ring block up front
 * (libpafdada extensions) are then off, and blocks are pinned when first
 * seen.
 */
#include <dlfcn.h>
#include <errno.h>
#include <getopt.h>
#include <inttypes.h>
#include <pthread.h>
#include <signal.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "b2p.h"
#ifdef B2P_PSRDADA
#include "ascii_header.h"
#include "dada_def.h"
#include "dada_hdu.h"
#include "futils.h"
#include "ipcio.h"
#include "multilog.h"
#define DEVICE_RINGS 0
#else
#include "b2p_dada.h"
#define DEVICE_RINGS 1
#endif

/* why the last device-ring call of this thread failed ("" for host rings) */
#if DEVICE_RINGS
#define RING_WHY() dada_device_error()
#else
#define RING_WHY() ""
#endif

#define MSTR_LEN 512 /* paf_baseband2power.cuh:4 */
#define TSAMP_BMF_US (27.0 / 32.0) /* README.md:2 */
#define MAX_SUB 64
#define MAX_PIN 64 /* ring blocks pinned per input ring */
#define kWarm 8 /* outputs before the steady-state clock starts (FINISH line) */

typedef struct conf_t { /* baseband2power.cuh:18-23, plus options */
  int device_id;
  char dir[MSTR_LEN];
  key_t key_in, key_out;
  char layout[64];
  int npol_out;
  int mean;
  int nsub;
  int nsplit; /* > 1: one ring's integration split by time over nsplit GPUs */
  int gather;  /* -G: 0 auto (RCCL unless members share a GPU), 1 RCCL, 2 copies */
  int coll_timeout_s; /* -T: RCCL set-up / collective time limit */
  int sync;  /* -S: one block per launch, waited for (the unpipelined baseline) */
  int trace; /* -V: log every launch / round */
  double writer_grace_s; /* -W: a transfer left open by a writer that went away ends the run after this */
} conf_t;

typedef struct sub_t { /* one sub-band: ring + GPU context + worker thread */
  int r;
  key_t key;
  int device;
  dada_hdu_t *in;
  char *hdr;         /* the input ring's header block, copied */
  uint64_t hdr_size;
  b2p_ctx_t *ctx;
  b2p_geom_t g;
  double tsamp_us;
  float *spec_dev; /* this sub-band's spectrum (device) */
  uint64_t *part_dev; /* time split: this member's exact partial sums (device) */
  uint64_t rbufsz;
  int locked;
  int ondev; /* input blocks are in GPU memory (dada_db -g) */
  char *pinned[MAX_PIN]; /* host ring blocks registered for DMA (dada_cuda_dbregister role) */
  int npinned;
} sub_t;

static void usage(void) {
  fprintf(stdout,
          "paf_baseband2power - To detect baseband data with original channels and average the "
          "detected data in time\n"
          "\n"
          "Usage: paf_baseband2power [options]\n"
          " -a  Hexacdecimal shared memory key for incoming ring buffer\n"
          " -b  Hexacdecimal shared memory key for outcoming ring buffer\n"
          " -c  The name of the directory in which we will record the data\n"
          " -d  The index of GPU\n"
          " -f  Input layout: bmf | int8:NCHAN | int16:NCHAN[:be] | header (default: header "
          "keys if they describe 8/16-bit baseband, else bmf)\n"
          " -p  Output pols: 1 = |X|^2+|Y|^2 (default), 2 = X and Y\n"
          " -m  Write the time average instead of the sum\n"
          " -n  Number of sub-bands (rings key_in + 0x10*r, GPUs d + r), gathered to GPU d\n"
          " -t  Split each integration of the one input ring by time over N GPUs (d + r);\n"
          "     exact partial sums are reduced on GPU d (host ring: N PCIe links in parallel)\n"
          " -G  Transport for -n / -t: rccl | copy (default: RCCL unless members share a GPU);\n"
          "     -n 1 -G rccl gathers the one sub-band through a one-member RCCL group\n"
          " -T  Time limit in s for the RCCL set-up and each collective (default 60); past it\n"
          "     the communicators are aborted and the stage exits with an error\n"
          " -S  GPU-resident rings: one block per launch, each waited for before the next\n"
          "     (no launches in flight, no batching of queued blocks; a diagnostic baseline)\n"
          " -V  Log every integrate launch / gathered round\n"
          " -W  Seconds an input transfer may stay open with no writer attached and nothing\n"
          "     to read before the run ends with an error (a writer that died mid-transfer;\n"
          "     default 0: wait for a writer to take the transfer on, as PSRDADA allows)\n"
          " -h  show help\n");
}

/* SIGINT / SIGTERM: stop between blocks and end the output transfer
 * cleanly (unlock_write writes its end of data, so the sink finishes).
 * Ring waits in progress give up (dada_interrupt_waits); worker threads
 * blocked in one are woken with SIGUSR2 by the main thread. */
static atomic_int g_stop; /* lock-free: set by the signal handler, read by every thread */
/* a member's input ring failed under it (next_block): every other member
 * waiting on its own ring is woken the same way, so the run ends instead of
 * waiting for blocks that are not coming */
static atomic_int g_abort; /* written by a worker, read by every thread */

static void on_stop(int sig) {
  (void)sig;
  g_stop = 1;
#if DEVICE_RINGS
  dada_interrupt_waits();
#endif
}

static void on_wake(int sig) { (void)sig; }

static void install_stop_handlers(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sigemptyset(&sa.sa_mask);
  sa.sa_handler = on_stop; /* no SA_RESTART: a blocked semop returns EINTR */
  sigaction(SIGINT, &sa, NULL);
  sigaction(SIGTERM, &sa, NULL);
  sa.sa_handler = on_wake;
  sigaction(SIGUSR2, &sa, NULL);
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + (double)t.tv_nsec * 1e-9;
}

/* layout from -f, else from the input header, else BMF-native */
static int pick_geometry(const conf_t *conf, const char *hdr, uint64_t rbufsz, b2p_geom_t *g,
                         double *tsamp_us, multilog_t *log) {
  b2p_geom_bmf(g);
  *tsamp_us = TSAMP_BMF_US;
  int nbit = 0, nchan = 0, npol = 0, ndim = 0;
  int hdr_ok = hdr && ascii_header_get(hdr, "NBIT", "%d", &nbit) == 1 &&
               ascii_header_get(hdr, "NCHAN", "%d", &nchan) == 1 && (nbit == 8 || nbit == 16);
  if (hdr_ok) {
    if (ascii_header_get(hdr, "NPOL", "%d", &npol) != 1) npol = 2;
    if (ascii_header_get(hdr, "NDIM", "%d", &ndim) != 1) ndim = 2;
  }
  const char *lay = conf->layout;
  if (!strcmp(lay, "bmf") || (!lay[0] && !hdr_ok)) {
    /* BMF-native constants (capture.h:20,28; conf:2-5) */
    if (!lay[0])
      multilog(log, LOG_INFO, "input header has no 8/16-bit baseband layout (NBIT %d): "
               "using BMF-native 48x7 chan int16 BE TFTFP", nbit);
  } else if (!strncmp(lay, "int8:", 5) || !strncmp(lay, "int16:", 6)) {
    int bits = lay[3] == '8' ? 8 : 16;
    const char *p = strchr(lay, ':') + 1;
    g->nbit = (uint32_t)bits;
    g->nchunk = 1;
    g->nchan_chunk = (uint32_t)atoi(p);
    g->big_endian = (bits == 16 && strstr(p, ":be")) ? 1 : 0;
    g->nsamp_df = 1;
  } else if (!strcmp(lay, "header") || (!lay[0] && hdr_ok)) {
    if (!hdr_ok) {
      multilog(log, LOG_ERR, "-f header: input header lacks NBIT 8/16 and NCHAN");
      return -1;
    }
    int nchunk = 1, nsamp_df = 1, ncc = nchan;
    char order[16] = "LE";
    ascii_header_get(hdr, "NCHUNK", "%d", &nchunk);
    ascii_header_get(hdr, "NSAMP_DF", "%d", &nsamp_df);
    ascii_header_get(hdr, "NCHAN_CHUNK", "%d", &ncc);
    ascii_header_get(hdr, "BYTE_ORDER", "%15s", order);
    if (nchunk < 1 || ncc * nchunk != nchan) {
      multilog(log, LOG_ERR, "NCHUNK %d x NCHAN_CHUNK %d != NCHAN %d", nchunk, ncc, nchan);
      return -1;
    }
    g->nbit = (uint32_t)nbit;
    g->nchunk = (uint32_t)nchunk;
    g->nchan_chunk = (uint32_t)ncc;
    g->nsamp_df = (uint32_t)nsamp_df;
    g->npol = (uint32_t)npol;
    g->ndim = (uint32_t)ndim;
    g->big_endian = (order[0] == 'B' || order[0] == 'b') ? 1 : 0;
    double ts = 0;
    if (ascii_header_get(hdr, "TSAMP", "%lf", &ts) == 1 && ts > 0) *tsamp_us = ts;
  } else {
    multilog(log, LOG_ERR, "unknown layout '%s'", lay);
    return -1;
  }
  g->npol_out = (uint32_t)conf->npol_out;
  g->mean = (uint32_t)conf->mean;
  /* one ring block = one integration */
  uint64_t fb = b2p_frame_bytes(g);
  if (!fb || rbufsz % fb) {
    multilog(log, LOG_ERR, "ring block of %" PRIu64 " B is not a whole number of %" PRIu64
             "-B frames", rbufsz, fb);
    return -1;
  }
  g->nsamp_int = rbufsz / fb * g->nsamp_df;
  if (b2p_geom_check(g) != B2P_OK) {
    multilog(log, LOG_ERR, "unsupported input layout");
    return -1;
  }
  return 0;
}

/* data block of a ring as the ipcbuf_t PSRDADA puts first in ipcio_t */
static ipcbuf_t *data_buf(dada_hdu_t *h) { return (ipcbuf_t *)h->data_block; }

/* Reader side of the header ring, in PSRDADA calls: take the next header
 * block, copy it, release it. */
static int read_header(dada_hdu_t *h, char **hdr, uint64_t *size) {
  uint64_t n = 0;
  char *p = ipcbuf_get_next_read(h->header_block, &n);
  if (!p) return -1;
  const uint64_t hsz = ipcbuf_get_bufsz(h->header_block);
  *hdr = calloc(1, hsz + 1);
  if (!*hdr) return -1;
  memcpy(*hdr, p, n < hsz ? n : hsz);
  *size = hsz;
  return ipcbuf_mark_cleared(h->header_block) < 0 ? -1 : 0;
}

/* ring location of an input ring's blocks: -1 host, else the HIP device */
static int ring_device(dada_hdu_t *h, int member_device) {
#if DEVICE_RINGS && defined(B2P_TEST_HOST_RING_AS_DEVICE)
  /* test build only (tests/test_sanitizers.py): host rings take the
   * GPU-resident paths, driven by the CPU test double tests/c/b2p_cpu_stub.c,
   * so their threads run under ThreadSanitizer on a machine with no GPU;
   * each ring counts as living on its member's device */
  (void)h;
  return member_device;
#elif DEVICE_RINGS
  (void)member_device;
  return ipcbuf_get_device(data_buf(h));
#else
  (void)h, (void)member_device;
  return -1;
#endif
}

/* Register a host ring block for DMA once, the first time it is seen (the
 * default build registers every block up front, so this finds them all). */
static void pin_block(sub_t *s, char *blk, multilog_t *log) {
  if (s->ondev || !blk) return;
  for (int i = 0; i < s->npinned; i++)
    if (s->pinned[i] == blk) return;
  if (s->npinned == MAX_PIN) return; /* unpinned blocks still work, at pageable rate */
  if (b2p_register_host(s->ctx, blk, s->rbufsz) != B2P_OK) {
    multilog(log, LOG_INFO, "register block: %s", b2p_last_error(s->ctx));
    return;
  }
  s->pinned[s->npinned++] = blk;
}

/* A failed run also names its errors on stderr (the reference's errors go
 * there, paf_baseband2power.cu:51-52): this run's ERR lines of the log. */
static void echo_errors(FILE *fp, long from, const char *fname) {
  char line[1200];
  fflush(fp);
  if (from < 0 || fseek(fp, from, SEEK_SET) != 0) return;
  while (fgets(line, sizeof line, fp))
    if (strstr(line, "] ERR: ")) fprintf(stderr, "paf_baseband2power: %s", line);
  fprintf(stderr, "paf_baseband2power: FAILED, log %s\n", fname);
}

/* next input block, or NULL at the end of the transfer (checked with
 * ipcbuf_eod first, so a reader never waits on a ring whose transfer
 * ended).  A read that fails instead -- the ring's semaphores removed under
 * the stage (EIDRM), not an end of data nor a stop signal -- sets *failed
 * (the caller reports it and fails the run: it is not an end of data). */
static char *next_block(dada_hdu_t *h, uint64_t *bytes, int *failed) {
  uint64_t bid = 0;
  *failed = 0;
  if (ipcbuf_eod(data_buf(h))) return NULL;
  errno = 0;
  char *p = ipcio_open_block_read(h->data_block, bytes, &bid);
  *failed = !p && errno && !g_stop && !g_abort ? errno : 0;
  if (*failed) {
    g_abort = 1;
#if DEVICE_RINGS
    dada_interrupt_waits(); /* the main thread then signals the members still waiting */
#endif
  }
  return p;
}

/* have[] of a member whose read failed (next_block): the round stops, and
 * the run fails */
#define HAVE_READ_FAILED (-2)

#if DEVICE_RINGS
/* -W S: the stage notices a writer that went away mid-transfer.  An input
 * transfer that is open, with no writer holding the ring and no block
 * waiting for this reader, for S seconds in a row, means the writer died
 * (the kernel undid its write lock) and no other writer took the transfer
 * on -- PSRDADA lets one, hence the grace period.  The run then ends as on
 * a failed read: an ERR line, every member woken, exit 1.  Only shared ring
 * state is read here (semaphores, the sync segment), never a member's
 * ipcbuf_t fields that its thread changes. */
typedef struct watch_t {
  struct shared_t *sh;
  dada_hdu_t *ring[MAX_SUB];
  key_t key[MAX_SUB];
  int nring;
  double grace_s;
  pthread_t main_th;
  atomic_int stop;
} watch_t;
#endif

/* ---- the integration loop, one thread per sub-band ---------------------- */

typedef struct shared_t {
  conf_t *conf;
  sub_t *sub;
  int nsub;
  multilog_t *log;
  dada_hdu_t *out;
  b2p_group_t *grp;
  float *root_dev;  /* nsub*nout on sub[0]'s device (x bmax when gathering batches) */
  float *spec_host; /* nsub*nout, pinned (x bmax when gathering batches) */
  float *stage;     /* gathered batches: one output block reordered member by member */
  uint64_t nout, obytes;
  pthread_barrier_t bar;
  int have[MAX_SUB]; /* this round: 1 whole block, 0 partial, -1 end of data */
  /* gathered batches (device rings): blocks each member has queued, whole
   * blocks it took, and whether its batch ended at a partial block */
  int avail[MAX_SUB], got[MAX_SUB], partial[MAX_SUB];
  uint32_t bmax;
  int depth;      /* read depth: two batches held */
  int gather_dev; /* every sub-band on a GPU-resident ring: worker_gather_dev */
  uint64_t tick[MAX_SUB]; /* each member's fence after its latest launch */
  uint64_t tick2[MAX_SUB]; /* ... after finishing its batch at once (nothing queued) */
  int idle[MAX_SUB];       /* nothing queued behind this round's batch */
  /* Any thread may raise `failed`, and a worker reads it at the top of its
   * next round while the root may still be writing it after the round's last
   * barrier: atomic (seq_cst), so those reads and writes are not a data race.
   * Whether a round stops is never decided from a read that can meet a write
   * in the same barrier phase: the per-member flags below are raised between
   * barriers and folded into `failed` by the root after the next one. */
  atomic_int failed;
  int mfail[MAX_SUB]; /* worker / worker_split: this member failed this round */
  uint64_t nblocks, nskipped;
  int end_lost; /* -n N: the integration lost when the first sub-band's transfer ended is counted (once) */
  uint64_t nlaunches; /* device ring: integrate launches, several queued blocks each at most */
  uint32_t max_batch;
  double t_first, t_last; /* first integration started, last output written */
  double t_warm;          /* output kWarm written: start of the steady-state span */
  /* time split (-t): the block every member takes its share of */
  char *blk;
  uint64_t blk_bytes, share_bytes, nsamp_full;
  uint64_t *root_sum; /* on member 0's device */
  /* spectra go through the group's gather (-n N > 1, or -n 1 -G rccl: one
   * RCCL member, the collective path exercised on one GPU) */
  int grouped;
} shared_t;

typedef struct worker_t {
  shared_t *sh;
  int r;
} worker_t;

static int write_output(shared_t *sh, const float *spec) {
  uint64_t bid;
  char *o = ipcio_open_block_write(sh->out->data_block, &bid);
  if (!o) {
    multilog(sh->log, LOG_ERR, "output block %" PRIu64 ": ipcio_open_block_write failed (%s)", sh->nblocks,
             strerror(errno));
    return -1;
  }
  memcpy(o, spec, sh->obytes);
  if (ipcio_close_block_write(sh->out->data_block, sh->obytes) < 0) {
    multilog(sh->log, LOG_ERR, "output block %" PRIu64 ": ipcio_close_block_write failed (%s)", sh->nblocks,
             strerror(errno));
    return -1;
  }
  sh->nblocks++;
  sh->t_last = now_s();
  if (sh->nblocks == kWarm) sh->t_warm = sh->t_last;
  return 0;
}

#if DEVICE_RINGS
static void *watch_writers(void *arg) {
  watch_t *w = (watch_t *)arg;
  double since[MAX_SUB];
  for (int r = 0; r < w->nring; r++) since[r] = -1;
  while (!w->stop && !g_stop && !g_abort) {
    const double t = now_s();
    for (int r = 0; r < w->nring; r++) {
      ipcbuf_t *db = data_buf(w->ring[r]);
      const int open = ipcbuf_get_transfer_open(db), conn = ipcbuf_get_writer_conn(db);
      const uint64_t waiting = ipcbuf_get_nfull_iread(db, db->iread);
      if (open != 1 || conn != 0 || waiting) {
        since[r] = -1;
      } else if (since[r] < 0) {
        since[r] = t;
      } else if (t - since[r] >= w->grace_s) {
        multilog(w->sh->log, LOG_ERR, "input ring %x: its writer went away without ending the transfer "
                 "(open, no writer, nothing to read for %.1f s)", (unsigned)w->key[r], t - since[r]);
        w->sh->failed = 1;
        g_abort = 1;
        dada_interrupt_waits();
        pthread_kill(w->main_th, SIGUSR2); /* the main thread may be the reader (run_device_pipelined) */
        return NULL;
      }
    }
    usleep(50000);
  }
  return NULL;
}
#endif

static void *worker(void *arg) {
  worker_t *w = (worker_t *)arg;
  shared_t *sh = w->sh;
  sub_t *s = &sh->sub[w->r];
  double t_prev = 0; /* the previous output's time */
  for (;;) {
    uint64_t bytes = 0;
    const double t_ask = now_s();
    int rfail = 0;
    char *blk = g_stop || g_abort ? NULL : next_block(s->in, &bytes, &rfail);
    const double t_got = now_s();
    if (rfail)
      multilog(sh->log, LOG_ERR, "sub-band %d: reading input ring %x failed (%s)", w->r, (unsigned)s->key,
               strerror(rfail));
    /* a 0-byte block only carries the end of data (PSRDADA's ipcio_close
     * after a full block): it ends the loop like a NULL one */
    sh->have[w->r] = rfail ? HAVE_READ_FAILED : !blk || !bytes ? -1 : (bytes == s->rbufsz ? 1 : 0);
    pthread_barrier_wait(&sh->bar); /* all sub-bands agree on this round */
    int stop = sh->failed, skip = 0;
    for (int r = 0; r < sh->nsub; r++) {
      if (sh->have[r] < 0) stop = 1;
      if (sh->have[r] == 0) skip = 1;
    }
    if (stop || skip) {
      if (blk) ipcio_close_block_read(s->in->data_block, bytes);
      int whole = 0; /* a member had a whole block for a round another member's end of data stops */
      for (int r = 0; r < sh->nsub; r++) {
        whole |= sh->have[r] == 1;
        if (w->r == 0 && sh->have[r] == HAVE_READ_FAILED) sh->failed = 1; /* stop is decided already */
      }
      if (w->r == 0 && skip && !stop) {
        sh->nskipped++;
        if (sh->nsub > 1) sh->end_lost = 1;
        multilog(sh->log, LOG_INFO, "partial integration skipped (a sub-band block held %" PRIu64
                 " of %" PRIu64 " B)", bytes, s->rbufsz);
      } else if (w->r == 0 && stop && whole && !sh->end_lost && !sh->failed && !g_stop) {
        sh->nskipped++;
        sh->end_lost = 1;
        multilog(sh->log, LOG_INFO, "partial integration skipped (a sub-band's transfer ended)");
      }
      pthread_barrier_wait(&sh->bar);
      if (stop) break;
      continue;
    }
    const double t0 = now_s();
    if (w->r == 0 && sh->t_first == 0) sh->t_first = t0;
    double t_copied = 0;
    int rc;
    if (s->ondev) {
      /* the block is already in HBM: one integrate launch reads it in place;
       * it must be done with the block before the block goes back to the ring */
      rc = b2p_integrate(s->ctx, blk, bytes, 1, !sh->grouped ? sh->spec_host : s->spec_dev,
                         !sh->grouped ? 0 : 1);
      if (rc == B2P_OK) rc = b2p_sync(s->ctx);
      ipcio_close_block_read(s->in->data_block, bytes);
    } else {
      pin_block(s, blk, sh->log);
      rc = b2p_push(s->ctx, blk, bytes, 0); /* returns once the block is copied */
      t_copied = now_s();
      ipcio_close_block_read(s->in->data_block, bytes);
      if (rc == B2P_OK) rc = b2p_finish_async(s->ctx, !sh->grouped ? sh->spec_host : s->spec_dev,
                                              !sh->grouped ? 0 : 1);
      if (rc == B2P_OK && !sh->grouped) rc = b2p_sync(s->ctx);
    }
    if (rc != B2P_OK)
      multilog(sh->log, LOG_ERR, "sub-band %d: %s (%s)", w->r, b2p_strerror(rc), b2p_last_error(s->ctx));
    sh->mfail[w->r] = rc != B2P_OK;
    pthread_barrier_wait(&sh->bar); /* every spectrum of this round is enqueued */
    if (w->r == 0)
      for (int r = 0; r < sh->nsub; r++)
        if (sh->mfail[r]) sh->failed = 1;
    if (w->r == 0 && !sh->failed) {
      if (sh->grouped) {
        float *specs[MAX_SUB];
        for (int r = 0; r < sh->nsub; r++) specs[r] = sh->sub[r].spec_dev;
        rc = b2p_group_gather(sh->grp, specs, sh->root_dev);
        if (rc == B2P_OK) rc = b2p_group_sync(sh->grp);
        if (rc == B2P_OK) rc = b2p_memcpy(s->ctx, sh->spec_host, sh->root_dev, sh->obytes, 2);
        if (rc != B2P_OK) {
          multilog(sh->log, LOG_ERR, "gather: %s", b2p_group_last_error(sh->grp));
          sh->failed = 1;
        }
      }
      if (!sh->failed) {
        if (write_output(sh, sh->spec_host) < 0) {
          sh->failed = 1;
        } else {
          const double dt = sh->t_last - t0;
          multilog(sh->log, LOG_INFO, "integration %" PRIu64 ": %.3f ms, %.2f GB/s per sub-band, "
                   "%.1f Msamples/s in all (asked for the block %.3f ms after the previous output, "
                   "waited for it %.3f ms, integrating from %.3f ms after it%s%.3f ms)", sh->nblocks, dt * 1e3,
                   (double)bytes / dt / 1e9,
                   (double)sh->nsub * (double)(sh->nout / s->g.npol_out) * s->g.npol *
                       (double)s->g.nsamp_int / dt / 1e6,
                   t_prev > 0 ? (t_ask - t_prev) * 1e3 : 0.0, (t_got - t_ask) * 1e3,
                   t_prev > 0 ? (t0 - t_prev) * 1e3 : 0.0, t_copied > 0 ? ", copied in " : ", integrated in ",
                   ((t_copied > 0 ? t_copied : sh->t_last) - t0) * 1e3);
        }
      }
    }
    if (w->r == 0) t_prev = sh->t_last; /* written by the root only (write_output) */
    pthread_barrier_wait(&sh->bar);
    if (sh->failed) break;
  }
  return NULL;
}

#if DEVICE_RINGS
/* nsub > 1 sub-bands on GPU-resident rings, gathered, launches kept in
 * flight.  Round k: every member takes the same number m_k of whole blocks
 * -- the next block plus what it has queued, the fewest any member has, up
 * to sh->bmax (b2p_blocks_per_launch) -- and integrates them in one launch,
 * which also finalizes its batch k-1 (carried).  Only then does it wait for
 * batch k-1's kernel and release those blocks, so its GPU never waits on the
 * host between rounds.  The root gathers batch k-1 of every member in one
 * collective on the group's own streams behind the members' fences
 * (b2p_group_gather_async) and writes batch k-2's output blocks.  Outputs
 * trail by two rounds while blocks are queued; when no member has one
 * queued behind its batch (a real-time stream between blocks, m = 1) the
 * round finishes at once and its spectra go out a kernel after the blocks.  One block per round
 * with a sync, a gather and the outputs inside it held two sub-bands
 * sharing one GPU to 4.45 TB/s (tools/bench_ring.py --nsub 2).  A member
 * whose transfer ends (a partial block) ends the batch at the blocks every
 * member has whole; the rest are released unintegrated and counted as one
 * skipped integration. */
typedef struct {
  uint64_t slot;   /* batch index */
  uint32_t m;      /* integrations per member */
  uint64_t gticket;
} gathered_t;

static int root_write_batch(shared_t *sh, const gathered_t *b, size_t nfl) {
  int rc = b2p_group_wait(sh->grp, b->gticket);
  if (rc != B2P_OK) {
    multilog(sh->log, LOG_ERR, "gather: %s", b2p_group_last_error(sh->grp));
    return -1;
  }
  const float *host = sh->spec_host + (b->slot % 3) * (size_t)sh->bmax * (sh->obytes / sizeof(float));
  for (uint32_t j = 0; j < b->m; j++) { /* member-major -> one output block per integration */
    for (int q = 0; q < sh->nsub; q++)
      memcpy(sh->stage + (size_t)q * nfl, host + ((size_t)q * b->m + j) * nfl, nfl * sizeof(float));
    if (write_output(sh, sh->stage) < 0) return -1;
  }
  return 0;
}

static int root_gather_batch(shared_t *sh, uint64_t slot, uint32_t m, size_t nfl, const uint64_t *tickets,
                             gathered_t *out) {
  float *specs[MAX_SUB];
  const size_t per = (size_t)sh->bmax * nfl;
  for (int q = 0; q < sh->nsub; q++) specs[q] = sh->sub[q].spec_dev + (slot % 3) * per;
  const size_t rs = (size_t)sh->bmax * (sh->obytes / sizeof(float));
  out->slot = slot;
  out->m = m;
  int rc = b2p_group_gather_async(sh->grp, specs, m, sh->root_dev + (slot % 3) * rs, tickets,
                                  sh->spec_host + (slot % 3) * rs, &out->gticket);
  if (rc != B2P_OK) multilog(sh->log, LOG_ERR, "gather: %s", b2p_group_last_error(sh->grp));
  return rc == B2P_OK ? 0 : -1;
}

static void *worker_gather_dev(void *arg) {
  worker_t *w = (worker_t *)arg;
  shared_t *sh = w->sh;
  const int r = w->r;
  sub_t *s = &sh->sub[r];
  ipcio_t *in = s->in->data_block;
  const size_t nfl = sh->obytes / sizeof(float) / (size_t)sh->nsub; /* floats per member spectrum */
  const uint32_t B = sh->bmax;
  const int depth = sh->depth;
  if (ipcbuf_set_read_depth(&in->buf, depth) < 0) {
    multilog(sh->log, LOG_ERR, "sub-band %d: read depth %d refused", r, depth);
    sh->failed = 1;
  }
  uint64_t t_held = 0; /* fence after the launch that reads the held blocks */
  int held = 0;        /* blocks of the previous batch, still held */
  uint32_t m_prev = 0; /* batch k-1's integrations, if its gather is still to come */
  gathered_t gq[3];  /* root: gathers issued, not yet written (oldest first) */
  int ngq = 0;
  for (uint64_t k = 0;; k++) {
    const void *blks[B2P_MAX_BLOCKS];
    uint64_t bytes = 0, bid = 0;
    int rfail = 0;
    char *blk = g_stop || g_abort || sh->failed ? NULL : next_block(s->in, &bytes, &rfail);
    int taken = blk ? 1 : 0, avail = 0;
    if (rfail)
      multilog(sh->log, LOG_ERR, "sub-band %d: reading input ring %x failed (%s)", r, (unsigned)s->key,
               strerror(rfail));
    sh->have[r] = rfail ? HAVE_READ_FAILED : !blk || !bytes ? -1 : (bytes == s->rbufsz ? 1 : 0);
    if (sh->have[r] == 1) {
      blks[0] = blk;
      const uint64_t q = ipcbuf_get_nfull_iread(&in->buf, in->buf.iread);
      uint64_t cap = B < (uint32_t)(depth - held) ? B : (uint32_t)(depth - held);
      avail = (int)(1 + q < cap ? 1 + q : cap);
    }
    sh->avail[r] = avail;
    pthread_barrier_wait(&sh->bar); /* B1: every member knows what it holds */
    int stop = sh->failed, skip = 0, n = (int)B;
    for (int q = 0; q < sh->nsub; q++) {
      if (sh->have[q] < 0) stop = 1;
      if (sh->have[q] == 0) skip = 1;
      if (sh->avail[q] < n) n = sh->avail[q];
    }
    int m = stop || skip ? 0 : 1, part = 0;
    for (int j = 1; m && j < n; j++) { /* queued: no wait */
      uint64_t b = 0;
      char *p = ipcio_open_block_read(in, &b, &bid);
      if (!p) break;
      taken++;
      if (b != s->rbufsz) { /* this sub-band's transfer ends here */
        part = b != 0;
        break;
      }
      blks[m++] = p;
    }
    sh->got[r] = m;
    sh->partial[r] = part;
    pthread_barrier_wait(&sh->bar); /* B2: every member's batch is known */
    uint32_t mm = (uint32_t)m;
    for (int q = 0; q < sh->nsub; q++)
      if ((uint32_t)sh->got[q] < mm) mm = (uint32_t)sh->got[q];
    if (r == 0 && mm && sh->t_first == 0) sh->t_first = now_s();
    int rc = B2P_OK;
    uint64_t t = 0;
    float *slot = s->spec_dev + (k % 3) * (size_t)B * nfl;
    if (mm) { /* batch k; its launch also finalizes batch k-1 */
      rc = mm == 1 ? b2p_integrate(s->ctx, blks[0], s->rbufsz, 1, slot, 1)
                   : b2p_integrate_n(s->ctx, blks, mm, slot, 1);
      if (rc == B2P_OK) rc = b2p_fence(s->ctx, &t);
    } else if (m_prev) { /* no launch to carry batch k-1's finalize: enqueue it */
      rc = b2p_sync(s->ctx);
      if (rc == B2P_OK) rc = b2p_fence(s->ctx, &t);
    }
    if (rc == B2P_OK && held) rc = b2p_fence_wait(s->ctx, t_held); /* batch k-1's kernel is done */
    for (; held; held--) ipcio_close_block_read(in, 0); /* its blocks go back, oldest first */
    held = taken;
    if (mm) t_held = t;
    if (!mm)
      for (; held; held--) ipcio_close_block_read(in, 0); /* nothing launched on these */
    if (rc != B2P_OK) {
      multilog(sh->log, LOG_ERR, "sub-band %d: %s (%s)", r, b2p_strerror(rc), b2p_last_error(s->ctx));
      sh->failed = 1;
    }
    sh->tick[r] = t;
    sh->idle[r] = mm && !g_stop && ipcbuf_get_nfull_iread(&in->buf, in->buf.iread) == 0;
    pthread_barrier_wait(&sh->bar); /* B3: every member launched batch k, tickets published */
    int drain = mm && !stop; /* nobody has a block queued: finish batch k now */
    for (int q = 0; q < sh->nsub; q++) drain &= sh->idle[q];
    if (r == 0) {
      /* an integration is lost when a member's transfer ended while another
       * had a whole block for it: taken in this round's queued loop (got >
       * mm), or as the round's first block (have 1 in a stop round).  The
       * first such round counts one skipped integration, however the
       * writers' timing split the blocks between the two rounds */
      int lost = skip && !stop;
      for (int q = 0; q < sh->nsub; q++) {
        lost |= (uint32_t)sh->got[q] > mm || sh->partial[q] || (stop && sh->have[q] == 1);
        if (stop && sh->have[q] == HAVE_READ_FAILED) sh->failed = 1; /* the members break below */
      }
      if (lost && !sh->end_lost) {
        sh->end_lost = 1;
        sh->nskipped++;
        multilog(sh->log, LOG_INFO, "partial integration skipped (a sub-band's transfer ended)");
      }
      /* batch k-1's gather, behind every member's fence of this round.  In a
       * drain round the members go on to flush and fence batch k at once, so
       * the root issues it after B3b instead: a gather reads each member's
       * fence ring (b2p_group_gather_async), which b2p_fence writes -- found
       * by ThreadSanitizer on the asynchronous CPU double (b2p_cpu_stub.c) */
      if (!drain && !sh->failed && m_prev && root_gather_batch(sh, k - 1, m_prev, nfl, sh->tick, &gq[ngq++]) < 0)
        sh->failed = 1;
      if (mm) {
        sh->nlaunches++;
        if (mm > sh->max_batch) sh->max_batch = mm;
        if (sh->conf->trace || sh->nlaunches % 64 == 1)
          multilog(sh->log, LOG_INFO, "round %" PRIu64 ": %u integration(s) per sub-band, %.3f ms since the "
                   "first", sh->nlaunches, mm, (now_s() - sh->t_first) * 1e3);
      }
    }
    /* every member breaks on the same round: stop was decided at B1 (a
     * failure raised after B3 stops the next round, at its B1) */
    if (stop) break;
    if (drain) { /* a real-time stream between blocks: batch k's spectra go out as soon as they can */
      uint64_t t2 = 0;
      rc = b2p_flush(s->ctx); /* its finalize now, as a kernel of its own (no wait) */
      if (rc == B2P_OK) rc = b2p_fence(s->ctx, &t2);
      if (rc != B2P_OK) {
        multilog(sh->log, LOG_ERR, "sub-band %d: %s (%s)", r, b2p_strerror(rc), b2p_last_error(s->ctx));
        sh->failed = 1;
      }
      sh->tick2[r] = t2;
      pthread_barrier_wait(&sh->bar); /* B3b: every member's batch k is finalized on its stream */
      if (r == 0 && !sh->failed) {
        if (m_prev && root_gather_batch(sh, k - 1, m_prev, nfl, sh->tick, &gq[ngq++]) < 0) sh->failed = 1;
        const int i0 = ngq;
        if (!sh->failed && root_gather_batch(sh, k, mm, nfl, sh->tick2, &gq[ngq++]) < 0) sh->failed = 1;
        /* write everything once batch k's gather is done, unless every
         * member's next block arrives first (then the rounds go on in flight) */
        while (!sh->failed && !g_stop) {
          int queued = 1;
          for (int q = 0; q < sh->nsub && queued; q++) {
            ipcbuf_t *qb = &sh->sub[q].in->data_block->buf;
            queued = ipcbuf_get_nfull_iread(qb, qb->iread) > 0;
          }
          if (queued) break;
          const int d = b2p_group_done(sh->grp, gq[i0].gticket);
          if (d < 0) {
            multilog(sh->log, LOG_ERR, "gather: %s", b2p_group_last_error(sh->grp));
            sh->failed = 1;
          } else if (d) {
            for (int i = 0; i < ngq && !sh->failed; i++)
              if (root_write_batch(sh, &gq[i], nfl) < 0) sh->failed = 1;
            ngq = 0;
            break;
          } else {
            nanosleep(&(struct timespec){0, 20000}, NULL);
          }
        }
      }
      m_prev = 0; /* batch k is gathered; its blocks are released next round, after t_held */
      if (r == 0)
        while (ngq > 2 && !sh->failed) { /* keep at most the two newest gathers pending */
          if (root_write_batch(sh, &gq[0], nfl) < 0) sh->failed = 1;
          gq[0] = gq[1];
          gq[1] = gq[2];
          ngq--;
        }
      continue;
    }
    if (r == 0) /* batch k-2 is home: its gather waited for launch k-1 */
      while (ngq > 1 && !sh->failed) {
        if (root_write_batch(sh, &gq[0], nfl) < 0) sh->failed = 1;
        gq[0] = gq[1];
        ngq--;
      }
    m_prev = mm;
  }
  /* stopped: batch k-1 was finalized and gathered above (m = 0 in a stop
   * round); release what is held, write what is gathered */
  for (; held; held--) ipcio_close_block_read(in, 0);
  if (r == 0)
    for (int i = 0; i < ngq && !sh->failed; i++)
      if (root_write_batch(sh, &gq[i], nfl) < 0) sh->failed = 1;
  return NULL;
}

/* One sub-band on a GPU-resident ring, launches kept in flight.  Batch k's
 * launch is enqueued before batch k-1's blocks are released, so the GPU
 * never waits on the host between launches; batch k-1 goes back to the ring
 * once its launch has finished (b2p_fence).  A batch is the next block plus
 * every further full block already queued in the ring (ipcbuf_get_nfull:
 * no wait), up to b2p_blocks_per_launch (a launch of >= 4 GiB), in ONE launch
 * (b2p_integrate_n): a consumer that has fallen behind catches up without
 * paying a launch per block.  Spectra are finalized by the next launch and
 * copied home behind it, so outputs trail by one batch -- unless nothing is
 * queued behind a batch (a real-time stream between blocks): then the batch
 * is finished at once and its spectra go out a kernel after their block. */

typedef struct {
  uint64_t first; /* index of its first integration */
  uint32_t n;     /* blocks (integrations) */
  uint64_t ticket;
} batch_t;

static void run_device_pipelined(shared_t *sh) {
  sub_t *s = &sh->sub[0];
  ipcio_t *in = s->in->data_block;
  const uint64_t nbufs = ipcbuf_get_nbufs(&in->buf);
  /* blocks held: the batch in flight and the one being gathered */
  const int depth = (int)(nbufs < 2 * B2P_MAX_BLOCKS ? nbufs : 2 * B2P_MAX_BLOCKS);
  /* per launch: b2p_blocks_per_launch (>= 4 GiB read), within the depth */
  const uint32_t want = b2p_blocks_per_launch(s->rbufsz);
  const uint32_t bmax = depth > 1 ? ((uint32_t)depth - 1 < want ? (uint32_t)depth - 1 : want) : 1;
  const size_t sb = (sh->obytes * bmax + 4095) / 4096 * 4096;
  float *spec = aligned_alloc(4096, 3 * sb); /* spectra of batches k-2, k-1, k */
  if (!spec || ipcbuf_set_read_depth(&in->buf, depth < 2 ? 2 : depth) < 0) {
    multilog(sh->log, LOG_ERR, "%s", !spec ? "cannot allocate the output spectra" : "read depth refused");
    free(spec);
    sh->failed = 1;
    return;
  }
  b2p_register_host(s->ctx, spec, 3 * sb);
#define SPEC(k) ((float *)((char *)spec + ((k) % 3) * sb))
  batch_t bat[3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  uint64_t k = 0, next = 0; /* batches launched; integrations launched */
  uint64_t written = 0;    /* batches whose spectra went out */
  int held = 0;            /* blocks of batch k-1 still held */
  for (;;) {
    const void *blks[B2P_MAX_BLOCKS];
    uint64_t bytes = 0, bid = 0;
    char *blk = NULL;
    if (!g_stop && !g_abort && !ipcbuf_eod(&in->buf)) {
      errno = 0;
      blk = ipcio_open_block_read(in, &bytes, &bid);
      if (!blk && errno && !g_stop && !g_abort) { /* not an end of data: the ring failed under the stage */
        multilog(sh->log, LOG_ERR, "reading input ring %x failed (%s)", (unsigned)s->key, strerror(errno));
        sh->failed = 1;
      }
    }
    uint32_t n = 0;
    while (blk && bytes == s->rbufsz) { /* gather this batch */
      blks[n++] = blk;
      blk = NULL;
      if (n == bmax || held + (int)n >= depth || g_stop || ipcbuf_get_nfull_iread(&in->buf, in->buf.iread) == 0)
        break;
      blk = ipcio_open_block_read(in, &bytes, &bid); /* already queued: no wait */
    }
    batch_t *b = &bat[k % 3];
    int rc = B2P_OK;
    if (n) {
      const double t0 = now_s();
      if (sh->t_first == 0) sh->t_first = t0;
      *b = (batch_t){next, n, 0};
      rc = n == 1 ? b2p_integrate(s->ctx, blks[0], s->rbufsz, 1, SPEC(k), 0)
                  : b2p_integrate_n(s->ctx, blks, n, SPEC(k), 0);
      if (rc == B2P_OK) rc = b2p_fence(s->ctx, &b->ticket);
      if (rc == B2P_OK && held) {
        rc = b2p_fence_wait(s->ctx, bat[(k - 1) % 3].ticket); /* batch k-1 is done */
        for (; rc == B2P_OK && held; held--) ipcio_close_block_read(in, 0); /* its blocks go back */
        for (; rc == B2P_OK && written + 2 <= k; written++) /* batch k-2 is home */
          for (uint32_t j = 0; rc == B2P_OK && j < bat[written % 3].n; j++)
            if (write_output(sh, SPEC(written) + (size_t)j * (sh->obytes / 4)) < 0) rc = B2P_EHIP;
      }
      held += (int)n; /* this batch's blocks, launched or not */
      if (rc == B2P_OK) {
        next += n;
        k++;
        sh->nlaunches = k;
        if (n > sh->max_batch) sh->max_batch = n;
        if (sh->conf->trace || k % 64 == 1)
          multilog(sh->log, LOG_INFO, "launch %" PRIu64 ": %u integration(s) from %" PRIu64 ", %.3f ms in "
                   "the loop body, %.3f ms since the first", k, n, b->first + 1, (now_s() - t0) * 1e3,
                   (now_s() - sh->t_first) * 1e3);
      } else {
        multilog(sh->log, LOG_ERR, "integrate: %s (%s)", b2p_strerror(rc), b2p_last_error(s->ctx));
        sh->failed = 1;
      }
      /* nothing queued behind this batch 0.2 ms after its launch (a
       * real-time stream between blocks): its finalize is enqueued now, as
       * a kernel of its own, and
       * the batch is finished as soon as its kernel ends -- its spectra go
       * out then, not a block later -- unless a block arrives first, which
       * keeps the launches in flight */
      if (rc == B2P_OK && !blk && !g_stop) { /* a producer ahead refills the slot just released */
        const double t_idle = now_s();
        while (!g_stop && ipcbuf_get_nfull_iread(&in->buf, in->buf.iread) == 0 && now_s() - t_idle < 2e-4)
          nanosleep(&(struct timespec){0, 10000}, NULL);
      }
      if (rc == B2P_OK && !blk && !g_stop && ipcbuf_get_nfull_iread(&in->buf, in->buf.iread) == 0) {
        uint64_t tf = 0;
        rc = b2p_flush(s->ctx);
        if (rc == B2P_OK) rc = b2p_fence(s->ctx, &tf);
        while (rc == B2P_OK && !g_stop && ipcbuf_get_nfull_iread(&in->buf, in->buf.iread) == 0) {
          const int d = b2p_fence_done(s->ctx, tf);
          if (d < 0) {
            rc = d;
          } else if (d) { /* batch k done: its blocks go back, every spectrum out */
            for (; held; held--) ipcio_close_block_read(in, 0);
            for (; rc == B2P_OK && written < k; written++)
              for (uint32_t j = 0; rc == B2P_OK && j < bat[written % 3].n; j++)
                if (write_output(sh, SPEC(written) + (size_t)j * (sh->obytes / 4)) < 0) rc = B2P_EHIP;
            break;
          } else {
            nanosleep(&(struct timespec){0, 20000}, NULL);
          }
        }
        if (rc != B2P_OK) {
          multilog(sh->log, LOG_ERR, "integrate: %s (%s)", b2p_strerror(rc), b2p_last_error(s->ctx));
          sh->failed = 1;
        }
      }
      if (rc == B2P_OK && !blk && !g_stop) continue; /* the next block decides */
    }
    /* end of data, a partial block, a stop or a failure: drain the pipeline */
    if (b2p_sync(s->ctx) != B2P_OK) {
      multilog(sh->log, LOG_ERR, "drain: %s", b2p_last_error(s->ctx));
      sh->failed = 1;
    }
    for (; held; held--) ipcio_close_block_read(in, 0);
    for (; !sh->failed && written < k; written++)
      for (uint32_t j = 0; !sh->failed && j < bat[written % 3].n; j++)
        if (write_output(sh, SPEC(written) + (size_t)j * (sh->obytes / 4)) < 0) sh->failed = 1;
    if (blk) {
      ipcio_close_block_read(in, bytes);
      if (bytes) { /* a 0-byte block only carries the end of data */
        sh->nskipped++;
        multilog(sh->log, LOG_INFO, "partial integration skipped (a block held %" PRIu64 " of %" PRIu64
                 " B)", bytes, s->rbufsz);
      }
    }
    if (!blk || sh->failed) break;
  }
#undef SPEC
  b2p_unregister_host(s->ctx, spec);
  free(spec);
}
#endif

/* -t N: member r integrates bytes [r*share, (r+1)*share) of every block of
 * the one input ring; member 0 reduces the exact partial sums (RCCL
 * ncclReduce, b2p_group_reduce) and rounds once (second mode) */
static void *worker_split(void *arg) {
  worker_t *w = (worker_t *)arg;
  shared_t *sh = w->sh;
  sub_t *s = &sh->sub[w->r];
  sub_t *s0 = &sh->sub[0];
  for (;;) {
    if (w->r == 0) {
      sh->blk_bytes = 0;
      int rfail = 0;
      sh->blk = g_stop || g_abort ? NULL : next_block(s0->in, &sh->blk_bytes, &rfail);
      pin_block(s0, sh->blk, sh->log);
      if (rfail)
        multilog(sh->log, LOG_ERR, "reading input ring %x failed (%s)", (unsigned)s0->key, strerror(rfail));
      sh->have[0] = rfail ? HAVE_READ_FAILED
                          : !sh->blk || !sh->blk_bytes ? -1 : (sh->blk_bytes == s0->rbufsz ? 1 : 0);
    }
    pthread_barrier_wait(&sh->bar);
    if (sh->have[0] <= 0 || sh->failed) {
      if (w->r == 0 && sh->have[0] == HAVE_READ_FAILED) sh->failed = 1; /* the round stops either way */
      if (w->r == 0 && sh->blk) {
        ipcio_close_block_read(s0->in->data_block, sh->blk_bytes);
        if (sh->have[0] == 0 && !sh->failed) {
          sh->nskipped++;
          multilog(sh->log, LOG_INFO, "partial integration skipped (block held %" PRIu64 " of %" PRIu64
                   " B)", sh->blk_bytes, s0->rbufsz);
        }
      }
      const int stop = sh->have[0] < 0 || sh->failed;
      pthread_barrier_wait(&sh->bar);
      if (stop) break;
      continue;
    }
    const double t0 = now_s();
    if (w->r == 0 && sh->t_first == 0) sh->t_first = t0;
    int rc = b2p_push(s->ctx, sh->blk + (uint64_t)w->r * sh->share_bytes, sh->share_bytes, 0);
    if (rc == B2P_OK) rc = b2p_finish_partial_async(s->ctx, s->part_dev, 1);
    if (rc != B2P_OK)
      multilog(sh->log, LOG_ERR, "member %d: %s (%s)", w->r, b2p_strerror(rc), b2p_last_error(s->ctx));
    sh->mfail[w->r] = rc != B2P_OK;
    pthread_barrier_wait(&sh->bar); /* every share has left the host block */
    if (w->r == 0) {
      for (int r = 0; r < sh->nsub; r++)
        if (sh->mfail[r]) sh->failed = 1;
      ipcio_close_block_read(s0->in->data_block, sh->blk_bytes);
      if (!sh->failed) {
        uint64_t *parts[MAX_SUB];
        for (int r = 0; r < sh->nsub; r++) parts[r] = sh->sub[r].part_dev;
        rc = b2p_group_reduce(sh->grp, parts, sh->nout, sh->root_sum);
        if (rc == B2P_OK) rc = b2p_group_sync(sh->grp); /* bounded by -T */
        if (rc == B2P_OK)
          rc = b2p_finalize_sums(s0->ctx, sh->root_sum, 1, sh->nsamp_full, s0->spec_dev);
        if (rc == B2P_OK) rc = b2p_memcpy(s0->ctx, sh->spec_host, s0->spec_dev, sh->obytes, 2);
        if (rc != B2P_OK) {
          multilog(sh->log, LOG_ERR, "reduce: %s / %s", b2p_group_last_error(sh->grp),
                   b2p_last_error(s0->ctx));
          sh->failed = 1;
        }
      }
      if (!sh->failed) {
        if (write_output(sh, sh->spec_host) < 0) {
          sh->failed = 1;
        } else {
          const double dt = sh->t_last - t0;
          multilog(sh->log, LOG_INFO, "integration %" PRIu64 ": %.3f ms, %.2f GB/s over %d GPUs",
                   sh->nblocks, dt * 1e3, (double)sh->blk_bytes / dt / 1e9, sh->nsub);
        }
      }
    }
    pthread_barrier_wait(&sh->bar);
    if (sh->failed) break;
  }
  return NULL;
}

/* RCCL refuses two members on one GPU, so members sharing one use peer
 * copies unless -G rccl insists (which then fails at set-up, reported) */
static int group_mode(const conf_t *conf, int dup_dev, multilog_t *log) {
  if (conf->gather == 1) {
    if (dup_dev) multilog(log, LOG_WARNING, "-G rccl with members sharing a GPU: RCCL will refuse it");
    return 0;
  }
  if (conf->gather == 2) return 1;
  return dup_dev ? 1 : 0;
}

int main(int argc, char *argv[]) {
  int arg;
  conf_t conf;
  memset(&conf, 0, sizeof conf);
  conf.npol_out = 1;
  conf.nsub = 1;
  conf.nsplit = 1;
  conf.coll_timeout_s = 60;
  strcpy(conf.dir, ".");
  int have_in = 0, have_out = 0;

  while ((arg = getopt(argc, argv, "a:b:c:d:f:p:n:t:G:T:W:mSVh")) != -1) {
    switch (arg) {
      case 'h':
        usage();
        return EXIT_FAILURE;
      case 'a':
        if (sscanf(optarg, "%x", (unsigned *)&conf.key_in) != 1) {
          fprintf(stderr, "Could not parse key from %s\n", optarg);
          return EXIT_FAILURE;
        }
        have_in = 1;
        break;
      case 'b':
        if (sscanf(optarg, "%x", (unsigned *)&conf.key_out) != 1) {
          fprintf(stderr, "Could not parse key from %s\n", optarg);
          return EXIT_FAILURE;
        }
        have_out = 1;
        break;
      case 'c': snprintf(conf.dir, sizeof conf.dir, "%s", optarg); break;
      case 'd': sscanf(optarg, "%d", &conf.device_id); break;
      case 'f': snprintf(conf.layout, sizeof conf.layout, "%s", optarg); break;
      case 'p': conf.npol_out = atoi(optarg); break;
      case 'n': conf.nsub = atoi(optarg); break;
      case 't': conf.nsplit = atoi(optarg); break;
      case 'm': conf.mean = 1; break;
      case 'S': conf.sync = 1; break;
      case 'V': conf.trace = 1; break;
      case 'G':
        if (!strcmp(optarg, "rccl")) conf.gather = 1;
        else if (!strcmp(optarg, "copy")) conf.gather = 2;
        else {
          fprintf(stderr, "-G takes rccl or copy, not %s\n", optarg);
          return EXIT_FAILURE;
        }
        break;
      case 'T': conf.coll_timeout_s = atoi(optarg); break;
      case 'W':
        if (sscanf(optarg, "%lf", &conf.writer_grace_s) != 1 || conf.writer_grace_s < 0) {
          fprintf(stderr, "-W takes seconds >= 0, not %s\n", optarg);
          return EXIT_FAILURE;
        }
#if !DEVICE_RINGS
        if (conf.writer_grace_s > 0) {
          fprintf(stderr, "-W needs libpafdada's writer queries (not in PSRDADA)\n");
          return EXIT_FAILURE;
        }
#endif
        break;
      default: usage(); return EXIT_FAILURE;
    }
  }
  if (!have_in || !have_out || conf.nsub < 1 || conf.nsub > MAX_SUB || conf.nsplit < 1 ||
      conf.nsplit > MAX_SUB || (conf.nsub > 1 && conf.nsplit > 1) || conf.coll_timeout_s < 1 ||
      conf.coll_timeout_s > 86400) {
    usage();
    return EXIT_FAILURE;
  }

  /* log interface (paf_baseband2power.cu:74-84) */
  char log_fname[MSTR_LEN + 64];
  snprintf(log_fname, sizeof log_fname, "%s/paf_baseband2power.log", conf.dir);
  FILE *fp_log = fopen(log_fname, "ab+");
  if (!fp_log) {
    fprintf(stderr, "Can not open log file %s\n", log_fname);
    return EXIT_FAILURE;
  }
  fseek(fp_log, 0, SEEK_END);
  const long log_start = ftell(fp_log); /* this run's lines start here */
  multilog_t *log = multilog_open("paf_baseband2power", 0);
  multilog_add(log, fp_log);
  multilog(log, LOG_INFO, "START PAF_PROCESS");
  install_stop_handlers();

  /* only one visible GPU => index 0 (paf_baseband2power.cu:86-90) */
  int ndev = 0;
  if (b2p_device_count(&ndev) != B2P_OK || ndev < 1) {
    multilog(log, LOG_ERR, "no HIP device: %s", b2p_last_error(NULL));
    fprintf(stderr, "no HIP device\n");
    return EXIT_FAILURE;
  }
  if (ndev == 1) conf.device_id = 0;

  int status = EXIT_FAILURE, out_locked = 0;
  shared_t sh;
  memset(&sh, 0, sizeof sh);
  sh.conf = &conf;
  sh.nsub = conf.nsub;
  sh.log = log;
  sub_t sub[MAX_SUB];
  memset(sub, 0, sizeof sub);
  sh.sub = sub;
  dada_hdu_t *out = dada_hdu_create(log);
  dada_hdu_set_key(out, conf.key_out);
  sh.out = out;
  int dup_dev = 0;

  const int split = conf.nsplit > 1;
  const int nmem = split ? conf.nsplit : conf.nsub;
  sh.nsub = nmem;
  sh.grouped = !split && (conf.nsub > 1 || conf.gather == 1);
  for (int r = 0; r < nmem; r++) {
    sub_t *s = &sub[r];
    s->r = r;
    s->key = conf.key_in + 0x10 * r;
    s->device = ndev == 1 ? 0 : (conf.device_id + r) % ndev;
    if (r && s->device == sub[0].device) dup_dev = 1;
    if (split && r > 0) { /* members share ring 0; each takes a time share */
      s->g = sub[0].g;
      s->rbufsz = sub[0].rbufsz;
      s->tsamp_us = sub[0].tsamp_us;
      int rc = b2p_open(&s->ctx, &s->g, s->device);
      if (rc != B2P_OK) {
        multilog(log, LOG_ERR, "b2p_open: %s (%s)", b2p_strerror(rc), b2p_last_error(NULL));
        goto done;
      }
      continue;
    }
    s->in = dada_hdu_create(log);
    dada_hdu_set_key(s->in, s->key);
    if (dada_hdu_connect(s->in) < 0 || dada_hdu_lock_read(s->in) < 0) {
      multilog(log, LOG_ERR, "cannot attach/lock input ring %x %s", (unsigned)s->key, RING_WHY());
      goto done;
    }
    s->locked = 1;
    if (read_header(s->in, &s->hdr, &s->hdr_size) < 0) {
      multilog(log, LOG_ERR, "no header on input ring %x", (unsigned)s->key);
      goto done;
    }
    s->rbufsz = ipcbuf_get_bufsz(data_buf(s->in));
    if (pick_geometry(&conf, s->hdr, s->rbufsz, &s->g, &s->tsamp_us, log) < 0) goto done;
    if (split) { /* every member's context integrates one time share */
      const uint64_t frames = s->g.nsamp_int / s->g.nsamp_df;
      if (frames % (uint64_t)conf.nsplit) {
        multilog(log, LOG_ERR, "%" PRIu64 " frames per block do not split into %d equal shares", frames,
                 conf.nsplit);
        goto done;
      }
      sh.nsamp_full = s->g.nsamp_int;
      s->g.nsamp_int /= (uint64_t)conf.nsplit;
      sh.share_bytes = s->rbufsz / (uint64_t)conf.nsplit;
    }
    if (r && memcmp(&s->g, &sub[0].g, sizeof s->g)) {
      multilog(log, LOG_ERR, "sub-band %d layout differs from sub-band 0", r);
      goto done;
    }
    int rc = b2p_open(&s->ctx, &s->g, s->device);
    if (rc != B2P_OK) {
      multilog(log, LOG_ERR, "b2p_open: %s (%s)", b2p_strerror(rc), b2p_last_error(NULL));
      goto done;
    }
    const int ring_dev = ring_device(s->in, s->device);
    s->ondev = ring_dev >= 0;
    if (s->ondev && split) {
      multilog(log, LOG_ERR, "-t splits host rings (one PCIe link per GPU); ring %x is on a GPU",
               (unsigned)s->key);
      goto done;
    }
    if (s->ondev) {
      b2p_info_t ci;
      b2p_get_info(s->ctx, &ci);
      if ((int)ci.device != ring_dev) {
        multilog(log, LOG_ERR, "input ring %x lives on GPU %d, this sub-band runs on GPU %d",
                 (unsigned)s->key, ring_dev, (int)ci.device);
        goto done;
      }
      multilog(log, LOG_INFO, "input ring %x is GPU-resident (device %d): no H2D copy",
               (unsigned)s->key, ring_dev);
    }
#if DEVICE_RINGS
    /* pin the input ring's blocks for DMA up front (dada_cuda_dbregister
     * role), so no first-use registration lands on an integration */
    for (uint64_t i = 0; !s->ondev && i < ipcbuf_get_nbufs(data_buf(s->in)); i++)
      pin_block(s, ipcbuf_get_buffer(data_buf(s->in), i), log);
#endif
  }
  b2p_info_t info;
  b2p_get_info(sub[0].ctx, &info);
  sh.nout = info.nout;
  { /* the bounds-checked debug build of libpafb2p (LD_LIBRARY_PATH=lib/debug:
     * the launcher's -e, in the role cuda-memcheck has in the reference,
     * paf-baseband2power.py:89-90) exports b2p_debug_build */
    int (*dbg)(void) = NULL;
    *(void **)&dbg = dlsym(RTLD_DEFAULT, "b2p_debug_build");
    if (dbg && dbg())
      multilog(log, LOG_INFO, "libpafb2p: debug build, every span load and output slot bounds-checked");
  }
  for (int r = 0; r < nmem && nmem > 1; r++) { /* which physical GPU each member drives */
    b2p_info_t mi;
    char bus[32] = "?";
    b2p_get_info(sub[r].ctx, &mi);
    b2p_device_pci_bus_id((int)mi.device, bus, (int)sizeof bus);
    multilog(log, LOG_INFO, "member %d: GPU %u (PCI %s)", r, mi.device, bus);
  }
  sh.obytes = (uint64_t)conf.nsub * info.nout * sizeof(float);
  if (split)
    multilog(log, LOG_INFO, "time split: each integration of ring %x over %d GPUs, %" PRIu64
             " B per share, exact partials reduced on GPU %d", (unsigned)conf.key_in, conf.nsplit,
             sh.share_bytes, sub[0].device);
  multilog(log, LOG_INFO,
           "%d sub-band(s): nbit %u %s, %u chunks x %u chans x %u samp/DF, %u outputs each, "
           "%" PRIu64 " samples per integration, first GPU %d",
           conf.nsub, sub[0].g.nbit, sub[0].g.big_endian ? "BE" : "LE", sub[0].g.nchunk,
           sub[0].g.nchan_chunk, sub[0].g.nsamp_df, info.nout, sub[0].g.nsamp_int, (int)info.device);

  if (dada_hdu_connect(out) < 0 || dada_hdu_lock_write(out) < 0) {
    multilog(log, LOG_ERR, "cannot attach/lock output ring %x", (unsigned)conf.key_out);
    goto done;
  }
  out_locked = 1;
  if (ipcbuf_get_bufsz(data_buf(out)) != sh.obytes) {
    /* same check as diskdb.cu:36-42, for the output ring (py:77-79) */
    multilog(log, LOG_ERR, "output ring block %" PRIu64 " B != NSUB x NCHAN x NPOL x 4 = %" PRIu64 " B",
             ipcbuf_get_bufsz(data_buf(out)), sh.obytes);
    goto done;
  }

  /* output header: NBIT 32, NDIM 1, NPOL, NCHAN (header_baseband2power.txt:36-42) */
  {
    char *ohdr = ipcbuf_get_next_write(out->header_block);
    uint64_t ohsz = ipcbuf_get_bufsz(out->header_block);
    if (!ohdr) {
      multilog(log, LOG_ERR, "output header block: ipcbuf_get_next_write failed (%s)", strerror(errno));
      goto done;
    }
    memset(ohdr, 0, ohsz);
    memcpy(ohdr, sub[0].hdr, sub[0].hdr_size < ohsz ? sub[0].hdr_size : ohsz);
    ohdr[ohsz - 1] = 0;
    const uint64_t nsamp_out = split ? sh.nsamp_full : sub[0].g.nsamp_int;
    const double tsamp_out = sub[0].tsamp_us * (double)nsamp_out;
    double tmpl = 0;
    if (ascii_header_get(ohdr, "TSAMP", "%lf", &tmpl) == 1 && tmpl != tsamp_out)
      multilog(log, LOG_INFO, "TSAMP %.6g us in the input header replaced by %.6f us "
               "(= %.6f us x %" PRIu64 ")", tmpl, tsamp_out, sub[0].tsamp_us, nsamp_out);
    ascii_header_set(ohdr, "NBIT", "%d", 32);
    ascii_header_set(ohdr, "NDIM", "%d", 1);
    ascii_header_set(ohdr, "NPOL", "%u", sub[0].g.npol_out);
    ascii_header_set(ohdr, "NCHAN", "%u", (uint32_t)conf.nsub * info.nchan);
    ascii_header_set(ohdr, "TSAMP", "%.6f", tsamp_out);
    ascii_header_set(ohdr, "BYTES_PER_SECOND", "%.6f", (double)sh.obytes / (tsamp_out * 1e-6));
    ascii_header_set(ohdr, "NSAMP_INT", "%" PRIu64, nsamp_out);
    ascii_header_set(ohdr, "POWER_MODE", "%s", sub[0].g.mean ? "MEAN" : "SUM");
    if (conf.nsub > 1) ascii_header_set(ohdr, "NSUBBAND", "%d", conf.nsub);
    if (split) ascii_header_set(ohdr, "NSPLIT", "%d", conf.nsplit);
#ifndef B2P_PSRDADA /* input-layout keys (libpafdada extension; kept with PSRDADA) */
    ascii_header_del(ohdr, "NCHUNK");
    ascii_header_del(ohdr, "NCHAN_CHUNK");
    ascii_header_del(ohdr, "NSAMP_DF");
    ascii_header_del(ohdr, "BYTE_ORDER");
#endif
    if (ipcbuf_mark_filled(out->header_block, ohsz) < 0) {
      multilog(log, LOG_ERR, "output header block: ipcbuf_mark_filled failed (%s)", strerror(errno));
      goto done;
    }
  }

  sh.bmax = 1;
#if DEVICE_RINGS
  if (sh.grouped && !conf.sync) { /* gathered batches (worker_gather_dev) */
    int all_dev = 1;
    uint64_t nb = UINT64_MAX;
    for (int r = 0; r < conf.nsub; r++) {
      all_dev &= sub[r].ondev;
      const uint64_t x = ipcbuf_get_nbufs(&sub[r].in->data_block->buf);
      if (x < nb) nb = x;
    }
    const uint32_t want = b2p_blocks_per_launch(sub[0].rbufsz);
    /* two batches held: B <= nbufs - 1, depth = min(nbufs, 2B) */
    sh.gather_dev = all_dev && nb >= 2;
    if (sh.gather_dev) {
      sh.bmax = nb - 1 < want ? (uint32_t)(nb - 1) : want;
      sh.depth = (int)(nb < 2 * sh.bmax ? nb : 2 * sh.bmax);
      if (sh.depth < 2) sh.depth = 2;
    }
  }
#endif
  {
    const size_t hb = ((sh.gather_dev ? 3 : 1) * sh.bmax * sh.obytes + 4095) / 4096 * 4096;
    sh.spec_host = aligned_alloc(4096, hb);
    sh.stage = malloc(sh.obytes);
    if (!sh.spec_host || !sh.stage) {
      multilog(log, LOG_ERR, "cannot allocate %zu B of output staging", hb);
      goto done;
    }
    if (b2p_register_host(sub[0].ctx, sh.spec_host, hb) != B2P_OK) /* the copies still work, unpinned */
      multilog(log, LOG_WARNING, "output staging not pinned: %s", b2p_last_error(sub[0].ctx));
  }
  if (split) {
    for (int r = 0; r < nmem; r++)
      if (b2p_dev_alloc(sub[r].ctx, (void **)&sub[r].part_dev, info.nout * sizeof(uint64_t)) != B2P_OK) {
        multilog(log, LOG_ERR, "member %d: b2p_dev_alloc: %s", r, b2p_last_error(sub[r].ctx));
        goto done;
      }
    if (b2p_dev_alloc(sub[0].ctx, (void **)&sub[0].spec_dev, info.nout * sizeof(float)) != B2P_OK ||
        b2p_dev_alloc(sub[0].ctx, (void **)&sh.root_sum, info.nout * sizeof(uint64_t)) != B2P_OK) {
      multilog(log, LOG_ERR, "b2p_dev_alloc: %s", b2p_last_error(sub[0].ctx));
      goto done;
    }
    b2p_ctx_t *ctxs[MAX_SUB];
    for (int r = 0; r < nmem; r++) ctxs[r] = sub[r].ctx;
    const int mode = group_mode(&conf, dup_dev, log);
    int rc = b2p_group_open_timed(&sh.grp, ctxs, nmem, mode, conf.coll_timeout_s * 1000);
    if (rc != B2P_OK) {
      multilog(log, LOG_ERR, "b2p_group_open: %s: %s", b2p_strerror(rc), b2p_group_last_error(NULL));
      fprintf(stderr, "paf_baseband2power: b2p_group_open: %s: %s\n", b2p_strerror(rc),
              b2p_group_last_error(NULL));
      goto done;
    }
    multilog(log, LOG_INFO, "reduce of %d time shares to GPU %d via %s", nmem, sub[0].device,
             mode ? "peer copies (shared device)" : "RCCL ncclReduce");
  } else if (sh.grouped) {
    for (int r = 0; r < conf.nsub; r++)
      if (b2p_dev_alloc(sub[r].ctx, (void **)&sub[r].spec_dev, 3 * sh.bmax * info.nout * sizeof(float)) !=
          B2P_OK) {
        multilog(log, LOG_ERR, "sub-band %d: b2p_dev_alloc: %s", r, b2p_last_error(sub[r].ctx));
        goto done;
      }
    if (b2p_dev_alloc(sub[0].ctx, (void **)&sh.root_dev, 3 * sh.bmax * sh.obytes) != B2P_OK) {
      multilog(log, LOG_ERR, "b2p_dev_alloc: %s", b2p_last_error(sub[0].ctx));
      goto done;
    }
    b2p_ctx_t *ctxs[MAX_SUB];
    for (int r = 0; r < conf.nsub; r++) ctxs[r] = sub[r].ctx;
    const int mode = group_mode(&conf, dup_dev, log);
    int rc = b2p_group_open_timed(&sh.grp, ctxs, conf.nsub, mode, conf.coll_timeout_s * 1000);
    if (rc != B2P_OK) {
      multilog(log, LOG_ERR, "b2p_group_open: %s: %s", b2p_strerror(rc), b2p_group_last_error(NULL));
      fprintf(stderr, "paf_baseband2power: b2p_group_open: %s: %s\n", b2p_strerror(rc),
              b2p_group_last_error(NULL));
      goto done;
    }
    multilog(log, LOG_INFO, "gather of %d sub-bands to GPU %d via %s%s", conf.nsub, sub[0].device,
             mode ? "peer copies (shared device)" : "RCCL ncclGather",
             sh.gather_dev ? ", queued blocks in rounds of up to b2p_blocks_per_launch" : "");
  }

#if DEVICE_RINGS
  watch_t watch = {0};
  pthread_t watch_th;
  int watching = 0;
  if (conf.writer_grace_s > 0) {
    watch.sh = &sh;
    watch.nring = split ? 1 : nmem;
    for (int r = 0; r < watch.nring; r++) {
      watch.ring[r] = sub[r].in;
      watch.key[r] = sub[r].key;
    }
    watch.grace_s = conf.writer_grace_s;
    watch.main_th = pthread_self();
    watching = pthread_create(&watch_th, NULL, watch_writers, &watch) == 0;
    if (!watching) multilog(log, LOG_WARNING, "-W: cannot start the writer watch; running without it");
  }
#endif
  {
#if DEVICE_RINGS
    if (!split && nmem == 1 && !sh.grouped && sub[0].ondev && !conf.sync) {
      multilog(log, LOG_INFO, "GPU-resident input: two launches in flight, queued blocks integrated "
               "together (up to %d per launch)", B2P_MAX_BLOCKS);
      run_device_pipelined(&sh);
      goto joined;
    }
#endif
    pthread_barrier_init(&sh.bar, NULL, (unsigned)nmem);
    pthread_t th[MAX_SUB];
    worker_t wk[MAX_SUB];
    for (int r = 0; r < nmem; r++) {
      wk[r].sh = &sh;
      wk[r].r = r;
#if DEVICE_RINGS
      void *(*fn)(void *) = split ? worker_split : sh.gather_dev ? worker_gather_dev : worker;
#else
      void *(*fn)(void *) = split ? worker_split : worker;
#endif
      pthread_create(&th[r], NULL, fn, &wk[r]);
    }
    /* join by polling, so a stop request can wake workers that wait on a ring */
    int joined[MAX_SUB] = {0}, left = nmem;
    while (left) {
      for (int r = 0; r < nmem; r++)
        if (!joined[r] && pthread_tryjoin_np(th[r], NULL) == 0) {
          joined[r] = 1;
          left--;
        }
      if (g_stop || g_abort)
        for (int r = 0; r < nmem; r++)
          if (!joined[r]) pthread_kill(th[r], SIGUSR2);
      if (left) usleep(20000);
    }
    pthread_barrier_destroy(&sh.bar);
  }
#if DEVICE_RINGS
joined:
  if (watching) {
    watch.stop = 1;
    pthread_join(watch_th, NULL);
  }
#endif
  status = sh.failed ? EXIT_FAILURE : EXIT_SUCCESS;

done:
  if (out_locked) dada_hdu_unlock_write(out); /* ends the output transfer (EOD) */
  if (sh.grp) b2p_group_close(sh.grp);
  for (int r = 0; r < sh.nsub; r++) {
    sub_t *s = &sub[r];
    if (s->ctx) {
      if (s->part_dev) b2p_dev_free(s->ctx, s->part_dev);
      if (r == 0 && sh.root_sum) b2p_dev_free(s->ctx, sh.root_sum);
      for (int i = 0; i < s->npinned; i++) b2p_unregister_host(s->ctx, s->pinned[i]);
      if (r == 0 && sh.spec_host) b2p_unregister_host(s->ctx, sh.spec_host);
      if (s->spec_dev) b2p_dev_free(s->ctx, s->spec_dev);
      if (r == 0 && sh.root_dev) b2p_dev_free(s->ctx, sh.root_dev);
      b2p_close(s->ctx);
    }
    if (s->locked) dada_hdu_unlock_read(s->in);
    if (s->in) dada_hdu_destroy(s->in);
    free(s->hdr);
  }
  free(sh.spec_host);
  free(sh.stage);
  dada_hdu_destroy(out);
  if (g_stop) multilog(log, LOG_INFO, "stopped by a signal between blocks; output transfer ended");
  if (sh.nlaunches)
    multilog(log, LOG_INFO, "%" PRIu64 " integrate %s for %" PRIu64 " integrations%s, up to %u queued "
             "blocks per launch", sh.nlaunches, sh.gather_dev ? "rounds" : "launches", sh.nblocks,
             sh.gather_dev ? " per sub-band" : "", sh.max_batch);
  multilog(log, LOG_INFO, "FINISH PAF_PROCESS: %" PRIu64 " integrations, %" PRIu64 " skipped, %s, "
           "%.6f s from the first integration to the last output, %.6f s for the last %" PRIu64,
           sh.nblocks, sh.nskipped, status == EXIT_SUCCESS ? "ok" : "FAILED",
           sh.t_last > sh.t_first ? sh.t_last - sh.t_first : 0.0,
           sh.nblocks > kWarm ? sh.t_last - sh.t_warm : 0.0,
           sh.nblocks > kWarm ? sh.nblocks - kWarm : (uint64_t)0);
  multilog_close(log);
  if (status != EXIT_SUCCESS) echo_errors(fp_log, log_start, log_fname);
  fclose(fp_log);
  return status;
}
