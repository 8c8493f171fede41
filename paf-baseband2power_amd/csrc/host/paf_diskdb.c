/*
 * paf_diskdb -- read a DADA data file into a ring buffer.
 * Command line of paf_diskdb.cu:10-22 (getopt "a:b:c:d:e:h", :30-62) and the
 * behaviour of diskdb.cu:
 *   init_diskdb (:12-72)  open file, attach + lock-write the ring, check the
 *                         4096-B header block, SOD on/off, skip the file's own
 *                         4096-B header;
 *   do_diskdb   (:74-124) the TEMPLATE header file (-d) goes into the header
 *                         ring; the payload is copied in ring-block-sized
 *                         reads until EOF; the short (possibly empty) last
 *                         block ends the transfer (EOD);
 *   destroy_diskdb (:126-134).
 * Differences: a failing init stops the program (the reference ignored the
 * return value, paf_diskdb.cu:65), -l names a log file (the reference's
 * conf.log was never initialised, paf_diskdb.cu:28), and -T N reads each
 * block with N threads, each pread()ing its own contiguous slice (default
 * 8).  One fread of the block (diskdb.cu:103-121) copies page-cached data at
 * ~10 GB/s on one core and bounds the whole file -> ring -> GPU chain
 * (DESIGN.md section 7); the slices are filled in parallel and the block is
 * closed once all of them have landed, so readers see the same bytes.
 * SIGINT / SIGTERM stop it as the end of the file would: the blocks read so
 * far are delivered, the one being read is dropped (the end-of-data block
 * takes its place), the transfer ends and it exits 0, so the stage
 * downstream finishes normally (the reference's diskdb had no handler;
 * killed, it left the transfer open and its reader waiting).
 *
 * -DB2P_PSRDADA builds it against PSRDADA's own headers and the PSRDADA
 * subset the reference calls, as the reference is
 * built; GPU-resident rings (a libpafdada extension) are then off.
 */
#include <errno.h>
#include <fcntl.h>
#include <getopt.h>
#include <inttypes.h>
#include <pthread.h>
#include <signal.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#ifdef B2P_PSRDADA
#include "ascii_header.h"
#include "dada_def.h"
#include "dada_hdu.h"
#include "futils.h"
#include "ipcio.h"
#include "multilog.h"
#else
#include "b2p_dada.h"
#endif

#define MSTR_LEN 512
#define DADA_HDR_SIZE 4096 /* diskdb.cuh:17 */
#define MAX_READERS 64

typedef struct conf_t { /* diskdb.cuh:19-30 */
  key_t key;
  int sod;
  char fname[2 * MSTR_LEN + 2], hfname[MSTR_LEN];
  int fd;
  int nthread;       /* -T: parallel readers per block */
  int seekable;      /* a regular file (pread slices); else a pipe / FIFO / terminal, read in order */
  dada_hdu_t *hdu;
  multilog_t *log;
  size_t hdrsz;
  size_t rbufsz;
} conf_t;

static void usage(void) {
  fprintf(stdout,
          "paf_diskdb - read dada data file into shared memory \n"
          "\n"
          "Usage: paf_diskdb [options]\n"
          " -a Hexadecimal shared memory key for capture \n"
          " -b Directory with data file \n"
          " -c The name of data file    \n"
          " -d The name of header file  \n"
          " -e Enable start-of-data or not \n"
          " -l Log file (default: stderr) \n"
          " -T Reader threads per block (default 8) \n"
          " -h Show help    \n");
}

static int init_diskdb(conf_t *conf) {
  conf->fd = open(conf->fname, O_RDONLY);
  struct stat st;
  if (conf->fd < 0 || fstat(conf->fd, &st) < 0) {
    fprintf(stderr, "Can not open file: %s\n", conf->fname);
    return EXIT_FAILURE;
  }
  /* the file's own header is skipped (diskdb.cu:69): a regular file's
   * reads start past it; a stream (a FIFO or a pipe) has it read
   * and dropped.  Either way the payload is read until end of file, not up
   * to a size taken at open (a file still growing is read to its end, as
   * the reference's fread loop did) */
  conf->seekable = S_ISREG(st.st_mode);
  if (!conf->seekable) {
    char skip[DADA_HDR_SIZE];
    size_t got = 0;
    while (got < sizeof skip) {
      const ssize_t k = read(conf->fd, skip + got, sizeof skip - got);
      if (k < 0 && errno == EINTR) continue;
      if (k <= 0) break;
      got += (size_t)k;
    }
  }
  conf->hdu = dada_hdu_create(conf->log);
  dada_hdu_set_key(conf->hdu, conf->key);
  if (dada_hdu_connect(conf->hdu) < 0) {
    multilog(conf->log, LOG_ERR, "could not connect to hdu");
#ifdef B2P_PSRDADA
    fprintf(stderr, "Can not connect to hdu %x\n", (unsigned)conf->key);
#else
    fprintf(stderr, "Can not connect to hdu %x %s\n", (unsigned)conf->key, dada_device_error());
#endif
    return EXIT_FAILURE;
  }
  ipcbuf_t *db = (ipcbuf_t *)conf->hdu->data_block; /* diskdb.cu:33 */
  conf->rbufsz = ipcbuf_get_bufsz(db);
  conf->hdrsz = ipcbuf_get_bufsz(conf->hdu->header_block);
  if (conf->hdrsz != DADA_HDR_SIZE) {
    multilog(conf->log, LOG_ERR, "header buffer size mismatch");
    fprintf(stderr, "Buffer size mismatch (%zu != %d)\n", conf->hdrsz, DADA_HDR_SIZE);
    return EXIT_FAILURE;
  }
  if (dada_hdu_lock_write(conf->hdu) < 0) {
    multilog(conf->log, LOG_ERR, "open_hdu: could not lock write");
    fprintf(stderr, "Error locking HDU\n");
    return EXIT_FAILURE;
  }
  if (conf->sod ? ipcbuf_enable_sod(db, 0, 0) < 0 : ipcbuf_disable_sod(db) < 0) {
    fprintf(stderr, "Can not write data before start\n");
    return EXIT_FAILURE;
  }
  return EXIT_SUCCESS;
}

/* set by SIGINT / SIGTERM; a read blocked on a stream returns at once (no
 * SA_RESTART), a wait for a free ring block finishes first */
static atomic_int g_stop; /* lock-free: set by the signal handler, read by every thread */
static void on_stop(int sig) {
  (void)sig;
  g_stop = 1;
}

typedef struct slice_t {
  int fd;
  char *dst;
  uint64_t off; /* file offset */
  size_t len;
  size_t got;
  int err;
} slice_t;

static void *read_slice(void *arg) {
  slice_t *s = arg;
  s->got = 0;
  s->err = 0;
  while (s->got < s->len) {
    const ssize_t k = pread(s->fd, s->dst + s->got, s->len - s->got, (off_t)(s->off + s->got));
    if (k < 0) {
      if (errno == EINTR && !g_stop) continue;
      s->err = errno;
      break;
    }
    if (k == 0) break; /* the file shrank under us: the block ends here */
    s->got += (size_t)k;
  }
  return NULL;
}

typedef struct span_t {
  char *p;
  size_t len;
} span_t;

/* map every page of a span writable in this process (its first write would
 * otherwise fault page by page inside the data path) */
static void *populate_span(void *arg) {
  span_t *s = arg;
  const uintptr_t pg = (uintptr_t)sysconf(_SC_PAGESIZE);
  const uintptr_t a = (uintptr_t)s->p / pg * pg, e = ((uintptr_t)s->p + s->len + pg - 1) / pg * pg;
#ifdef MADV_POPULATE_WRITE
  if (madvise((void *)a, e - a, MADV_POPULATE_WRITE) == 0) return NULL;
#endif
  /* older kernels: rewrite one byte of each page with itself (every block
   * is still free: the ring's reader sees none of it before it is filled) */
  for (uintptr_t q = a < (uintptr_t)s->p ? a + pg : a; q < e && q < (uintptr_t)s->p + s->len; q += pg) {
    volatile char *c = (volatile char *)q;
    *c = *c;
  }
  return NULL;
}

/* Before the first block: the ring's blocks mapped writable in this process,
 * nthread spans at a time, so that no page fault lands in the data path.
 * On the GPU box's host (profiles/r04_diskdb_readers_paging.jsonl) this took
 * 0.16-0.19 s for a ring of 2 x 1 GiB made with dada_db -p, and 0.33-0.68 s
 * for one that was not (its pages are allocated here); the reads after it
 * ran at 65-92 GB/s with 8-16 threads against 18-22 GB/s with one. */
static void populate_ring(const conf_t *conf) {
  ipcbuf_t *db = (ipcbuf_t *)conf->hdu->data_block;
#ifndef B2P_PSRDADA
  if (ipcbuf_get_device(db) >= 0) return; /* device blocks: nothing mapped here */
#endif
  const uint64_t nbufs = ipcbuf_get_nbufs(db);
  const size_t per = (conf->rbufsz + (size_t)conf->nthread - 1) / (size_t)conf->nthread;
  for (uint64_t b = 0; b < nbufs; b++) {
    span_t sp[MAX_READERS];
    pthread_t th[MAX_READERS];
    int ns = 0, started = 0;
    for (size_t at = 0; at < conf->rbufsz; at += per)
      sp[ns++] = (span_t){db->buffer[b] + at, at + per < conf->rbufsz ? per : conf->rbufsz - at};
    for (int i = 1; i < ns; i++)
      if (pthread_create(&th[i], NULL, populate_span, &sp[i]) == 0) started = i;
      else break;
    populate_span(&sp[0]);
    for (int i = 1; i <= started; i++) pthread_join(th[i], NULL);
    for (int i = started + 1; i < ns; i++) populate_span(&sp[i]);
  }
}

/* up to n bytes of a stream, in order, until end of file */
static int64_t read_stream(int fd, char *dst, size_t n) {
  size_t got = 0;
  while (got < n) {
    const ssize_t k = read(fd, dst + got, n - got);
    if (k < 0) {
      if (errno == EINTR && !g_stop) continue;
      return -1;
    }
    if (k == 0) break;
    got += (size_t)k;
  }
  return (int64_t)got;
}

/* up to n bytes of the payload from offset off into dst, in nthread
 * contiguous slices (whole 2 MiB pieces, so a thread's copy stays on whole
 * pages); returns the bytes read before the first short slice (the end of
 * the file as it stands), or -1.  A stream is read in order instead. */
static int64_t read_block(const conf_t *conf, char *dst, uint64_t off, size_t n) {
  if (!conf->seekable) return read_stream(conf->fd, dst, n);
  slice_t sl[MAX_READERS];
  pthread_t th[MAX_READERS];
  const size_t piece = 2u << 20;
  size_t per = (n + (size_t)conf->nthread - 1) / (size_t)conf->nthread;
  per = (per + piece - 1) / piece * piece;
  int ns = 0;
  for (size_t at = 0; at < n || ns == 0; at += per) {
    sl[ns] = (slice_t){conf->fd, dst + at, DADA_HDR_SIZE + off + at, at + per < n ? per : n - at, 0, 0};
    ns++;
    if (at + per >= n) break;
  }
  int started = 1;
  for (int i = 1; i < ns; i++)
    if (pthread_create(&th[i], NULL, read_slice, &sl[i]) == 0)
      started++;
    else
      break;
  read_slice(&sl[0]);
  for (int i = 1; i < started; i++) pthread_join(th[i], NULL);
  for (int i = started; i < ns; i++) read_slice(&sl[i]); /* no thread for it: read here */
  uint64_t total = 0;
  for (int i = 0; i < ns; i++) {
    if (sl[i].err) {
      errno = sl[i].err;
      return -1;
    }
    total += sl[i].got;
    if (sl[i].got < sl[i].len) break;
  }
  return (int64_t)total;
}

static int do_diskdb(conf_t *conf) {
  char *hdrbuf = ipcbuf_get_next_write(conf->hdu->header_block);
  if (!hdrbuf || fileread(conf->hfname, hdrbuf, DADA_HDR_SIZE) < 0) {
    multilog(conf->log, LOG_ERR, "cannot read header from %s", conf->hfname);
    fprintf(stderr, "Error reading header file %s\n", conf->hfname);
    return EXIT_FAILURE;
  }
  if (ipcbuf_mark_filled(conf->hdu->header_block, DADA_HDR_SIZE) < 0) {
    multilog(conf->log, LOG_ERR, "Could not mark filled header block");
    return EXIT_FAILURE;
  }
  struct timespec t0, t1, tp;
  clock_gettime(CLOCK_MONOTONIC, &tp);
  populate_ring(conf);
  clock_gettime(CLOCK_MONOTONIC, &t0);
  const double populate_s = (double)(t0.tv_sec - tp.tv_sec) + (double)(t0.tv_nsec - tp.tv_nsec) * 1e-9;
  uint64_t block_id, total = 0, nblk = 0;
  char *stage = NULL;
#ifndef B2P_PSRDADA
  /* a GPU-resident ring (dada_db -g) takes each block through host staging */
  ipcbuf_t *db = (ipcbuf_t *)conf->hdu->data_block;
  if (ipcbuf_get_device(db) >= 0 && !(stage = malloc(conf->rbufsz))) {
    multilog(conf->log, LOG_ERR, "cannot allocate %zu B of staging", conf->rbufsz);
    return EXIT_FAILURE;
  }
#endif
  /* ring-block-sized reads until end of file; the short (or empty) last
   * block ends the transfer, as fread's did (diskdb.cu:103-121) */
  double wait_s = 0, read_s = 0, first_s = 0; /* first_s: the first pass over the ring's blocks */
  const uint64_t nbufs = ipcbuf_get_nbufs((ipcbuf_t *)conf->hdu->data_block);
  int stopped = 0;
  for (uint64_t off = 0;;) {
    struct timespec a, b, c;
    if (g_stop) { /* before a block is opened: the transfer ends after the last one */
      stopped = 1;
      break;
    }
    clock_gettime(CLOCK_MONOTONIC, &a);
    char *curbuf = ipcio_open_block_write(conf->hdu->data_block, &block_id);
    if (!curbuf) {
      multilog(conf->log, LOG_ERR, "no block to write in ring %x (block %" PRIu64 ")", (unsigned)conf->key, nblk);
      free(stage);
      return EXIT_FAILURE;
    }
    clock_gettime(CLOCK_MONOTONIC, &b);
    const int64_t got = read_block(conf, stage ? stage : curbuf, off, conf->rbufsz);
    clock_gettime(CLOCK_MONOTONIC, &c);
    wait_s += (double)(b.tv_sec - a.tv_sec) + (double)(b.tv_nsec - a.tv_nsec) * 1e-9;
    const double rs = (double)(c.tv_sec - b.tv_sec) + (double)(c.tv_nsec - b.tv_nsec) * 1e-9;
    read_s += rs;
    if (nblk < nbufs) first_s += rs;
    if (g_stop) { /* the block being read is dropped: the end of the transfer takes its place */
      stopped = 1;
      break;
    }
    if (got < 0) {
      multilog(conf->log, LOG_ERR, "read of %s at %" PRIu64 " failed: %s", conf->fname, off, strerror(errno));
      ipcio_close_block_write(conf->hdu->data_block, 0);
      free(stage);
      return EXIT_FAILURE;
    }
    const size_t n = (size_t)got;
#ifndef B2P_PSRDADA
    if (stage && ipcbuf_copy_in(db, curbuf, stage, n) < 0) {
      multilog(conf->log, LOG_ERR, "copy into device block failed: %s", dada_device_error());
      ipcio_close_block_write(conf->hdu->data_block, 0); /* the 0-byte end of data, not a half-copied block */
      free(stage);
      return EXIT_FAILURE;
    }
#endif
    ipcio_close_block_write(conf->hdu->data_block, n);
    total += n;
    off += n;
    nblk++;
    if (n < conf->rbufsz) break; /* the short block already ended the transfer */
  }
  free(stage);
  if (stopped)
    multilog(conf->log, LOG_INFO, "stopped by a signal after %" PRIu64 " blocks: ending the transfer", nblk);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  double el = (double)(t1.tv_sec - t0.tv_sec) + (double)(t1.tv_nsec - t0.tv_nsec) * 1e-9;
  multilog(conf->log, LOG_INFO,
           "diskdb: %" PRIu64 " B in %" PRIu64 " blocks, %.3f s (%.2f GB/s), %d reader%s; %.3f s reading "
           "(%.2f GB/s; %.3f s of it in the first pass over the %" PRIu64 " ring blocks), %.3f s waiting for a "
           "free block; %.3f s mapping the ring's blocks before the first",
           total, nblk, el, el > 0 ? (double)total / el / 1e9 : 0.0, conf->nthread, conf->nthread == 1 ? "" : "s",
           read_s, read_s > 0 ? (double)total / read_s / 1e9 : 0.0, first_s, nbufs, wait_s, populate_s);
  return EXIT_SUCCESS;
}

static int destroy_diskdb(conf_t *conf) {
  if (conf->hdu) {
    dada_hdu_unlock_write(conf->hdu);
    dada_hdu_disconnect(conf->hdu);
    dada_hdu_destroy(conf->hdu);
  }
  if (conf->fd >= 0) close(conf->fd);
  return EXIT_SUCCESS;
}

int main(int argc, char **argv) {
  int arg;
  char fdir[MSTR_LEN] = ".", fname[MSTR_LEN] = "", logname[MSTR_LEN] = "";
  conf_t conf;
  memset(&conf, 0, sizeof conf);
  conf.fd = -1;
  conf.nthread = 8;
  int have_key = 0;
  while ((arg = getopt(argc, argv, "a:b:c:d:e:l:T:h")) != -1) {
    switch (arg) {
      case 'h':
        usage();
        return EXIT_FAILURE;
      case 'a':
        if (sscanf(optarg, "%x", (unsigned *)&conf.key) != 1) {
          fprintf(stderr, "Could not parse key from %s\n", optarg);
          return EXIT_FAILURE;
        }
        have_key = 1;
        break;
      case 'b': snprintf(fdir, sizeof fdir, "%s", optarg); break;
      case 'c': snprintf(fname, sizeof fname, "%s", optarg); break;
      case 'd': snprintf(conf.hfname, sizeof conf.hfname, "%s", optarg); break;
      case 'e': sscanf(optarg, "%d", &conf.sod); break;
      case 'l': snprintf(logname, sizeof logname, "%s", optarg); break;
      case 'T':
        conf.nthread = atoi(optarg);
        if (conf.nthread < 1 || conf.nthread > MAX_READERS) {
          fprintf(stderr, "-T takes 1..%d reader threads\n", MAX_READERS);
          return EXIT_FAILURE;
        }
        break;
      default: usage(); return EXIT_FAILURE;
    }
  }
  if (!have_key || !fname[0] || !conf.hfname[0]) {
    usage();
    return EXIT_FAILURE;
  }
  snprintf(conf.fname, sizeof conf.fname, "%s/%s", fdir, fname);
  conf.log = multilog_open("paf_diskdb", 0);
  FILE *lf = logname[0] ? fopen(logname, "ab") : NULL;
  multilog_add(conf.log, lf ? lf : stderr);

  {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sigemptyset(&sa.sa_mask);
    sa.sa_handler = on_stop; /* no SA_RESTART: a read blocked on a stream returns EINTR */
    sigaction(SIGINT, &sa, NULL);
    sigaction(SIGTERM, &sa, NULL);
  }
  int rc = init_diskdb(&conf);
  if (rc == EXIT_SUCCESS) rc = do_diskdb(&conf);
  destroy_diskdb(&conf);
  multilog_close(conf.log);
  if (lf) fclose(lf);
  return rc;
}
