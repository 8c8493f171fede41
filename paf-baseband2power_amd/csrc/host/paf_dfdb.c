/*
 * paf_dfdb -- GPU-side producer for a GPU-resident input ring
 * (SURVEY.md 8f ranks 2 and 3).
 *
 * The reference's capture threads copy each received data frame into the
 * host ring block at (idf*NCHK_NIC + chunk)*7168 (capture.c:536-541), and
 * the GPU stage would then copy the whole block to the device.  Here raw
 * frames (a paf_dfgen stream file stands in for the sockets) go to HBM in
 * batches and b2p_assemble scatters them straight into a ring block that
 * lives in GPU memory (dada_db -g), which paf_baseband2power integrates in
 * place: the payload crosses PCIe once, as frames.
 *
 *   paf_dfdb -a key -b header_file -c df_file -k chunk_file [-n nchunk]
 *            [-x ref_idf] [-s ref_sec] [-d device] [-Z] [-e dir]
 *     Frames are read in batches of one block's worth.  The host decodes
 *     every frame's header as the batch arrives and records which blocks
 *     the batch touches; block b is assembled from every batch that holds
 *     frames of it, once a batch that lies wholly past block b+1 has been
 *     read (so a frame may arrive up to about one block early or late, as
 *     the reference's temp buffer allows, capture.c:525-531).  A frame that
 *     arrives later than that -- for a block already written, or more than
 *     one block behind the newest block seen -- is dropped, as the capture
 *     drops it, and so a lagging source cannot hold the read-ahead back until
 *     the batch slots overflow.  Blocks
 *     follow the frames' timestamps, not the batch count, so a lossy stream
 *     (fewer frames than blocks x frames per block) still yields every
 *     block it has frames for.  A frame more than 2 blocks past the latest
 *     block seen so far is taken as corrupt and left out; the reference's
 *     capture stops at such a frame (capture.c:491-508), and here a stream
 *     whose frames jump that far ends its blocks at the jump as well.  The
 *     block is zeroed first unless -Z (the reference leaves lost frames'
 *     slots stale).
 *
 *   paf_dfdb -a key -b header_file -R nblocks [-f layout] [-r seed] [-u subband] [-d device]
 *     Replay: fill each ring block once with the synthetic generator (block
 *     i of sub-band `subband`, the stream bench.py and the tests regenerate), then
 *     hand the ring's blocks out nblocks times without rewriting them -- a
 *     consumer-side throughput test of a GPU-resident ring (or, for
 *     comparison, of a host ring, whose consumer copies each block H2D).  layout:
 *     bmf (default), int8:NCHAN, int16:NCHAN[:be].
 */
#include <getopt.h>
#include <inttypes.h>
#include <signal.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "b2p.h"
#include "b2p_dada.h"
#include "b2p_df.h"

/* the GPU holding ring db's blocks, -1 for a host ring */
static int ring_device_of(ipcbuf_t *db) {
#if defined(B2P_TEST_HOST_RING_AS_DEVICE)
  /* test build only (tests/test_frames_stub.py): a host ring takes the
   * GPU-resident path, driven by the CPU test double tests/c/b2p_cpu_stub.c,
   * so this host runs under ThreadSanitizer on a machine with no GPU */
  (void)db;
  return 0;
#else
  return ipcbuf_get_device(db);
#endif
}

#define HDR_SIZE DADA_DEFAULT_HEADER_SIZE

/* SIGINT / SIGTERM: the block being assembled is finished and delivered,
 * then the transfer ends and paf_dfdb exits 0 (as paf_capture stops), so
 * the stage downstream finishes normally */
static atomic_int g_stop; /* lock-free: set by the signal handler, read by every thread */
static void on_stop(int sig) {
  (void)sig;
  g_stop = 1;
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

static int parse_layout(const char *lay, b2p_geom_t *g) {
  b2p_geom_bmf(g);
  if (!strcmp(lay, "bmf")) return 0;
  if (strncmp(lay, "int8:", 5) && strncmp(lay, "int16:", 6)) return -1;
  const int bits = lay[3] == '8' ? 8 : 16;
  const char *p = strchr(lay, ':') + 1;
  g->nbit = (uint32_t)bits;
  g->nchunk = 1;
  g->nsamp_df = 1;
  g->nchan_chunk = (uint32_t)atoi(p);
  g->big_endian = (bits == 16 && strstr(p, ":be")) ? 1 : 0;
  return g->nchan_chunk ? 0 : -1;
}

#define NSLOT 6 /* batches held on the GPU at once */

typedef struct batch_t {
  void *frames;  /* device: n x 7232 B */
  void *chunks;  /* device: n chunk indices */
  uint64_t n;
  int64_t lo, hi; /* blocks (from the first reference) its frames fall in; hi < 0: none */
} batch_t;

/* next batch of up to cap frames from the stream files, via host staging;
 * the headers are decoded on the host for the blocks the batch touches,
 * leaving out frames before block 0 and past block `limit` (corrupt) */
static int load_batch(b2p_ctx_t *ctx, FILE *fd, FILE *fc, batch_t *b, uint64_t cap, unsigned char *hf,
                      unsigned char *hc, const b2p_df_hdr_t *ref0, uint64_t block_ndf, int64_t late_before,
                      int64_t limit) {
  const size_t got = fread(hf, B2P_DF_BYTES, cap, fd);
  b->n = got;
  b->lo = INT64_MAX;
  b->hi = -1;
  if (!got) return 0;
  if (fread(hc, 1, got, fc) != got) {
    fprintf(stderr, "paf_dfdb: chunk file shorter than the frame file\n");
    return -1;
  }
  for (size_t i = 0; i < got; i++) {
    b2p_df_hdr_t h;
    b2p_df_decode(hf + i * B2P_DF_BYTES, &h);
    const int64_t rel = b2p_df_index(&h, ref0);
    if (rel < 0) continue;
    const int64_t k = rel / (int64_t)block_ndf;
    /* late: a block already written, or more than one block behind the
     * newest seen -- the capture drops such a frame (capture.c:464-531), so
     * it neither places it nor lets it hold the read-ahead back */
    if (k < late_before || k > limit) continue;
    if (k < b->lo) b->lo = k;
    if (k > b->hi) b->hi = k;
  }
  if (b2p_memcpy(ctx, b->frames, hf, got * B2P_DF_BYTES, 1) != B2P_OK ||
      b2p_memcpy(ctx, b->chunks, hc, got, 1) != B2P_OK) {
    fprintf(stderr, "paf_dfdb: uploading %zu frames: %s\n", got, b2p_last_error(ctx));
    return -1;
  }
  return 0;
}

int main(int argc, char **argv) {
  key_t key = 0;
  const char *hfile = NULL, *dfile = NULL, *cfile = NULL, *layout = "bmf", *logdir = NULL;
  uint64_t ref_idf = 0, ref_sec = 0, seed = 20181105, replay = 0;
  uint32_t subband = 0;
  int nchunk = 48, device = 0, nozero = 0, arg, have_key = 0;
  while ((arg = getopt(argc, argv, "a:b:c:k:n:x:s:d:ZR:f:r:u:e:h")) != -1) {
    switch (arg) {
      case 'a': have_key = sscanf(optarg, "%x", (unsigned *)&key) == 1; break;
      case 'b': hfile = optarg; break;
      case 'c': dfile = optarg; break;
      case 'k': cfile = optarg; break;
      case 'n': nchunk = atoi(optarg); break;
      case 'x': ref_idf = strtoull(optarg, NULL, 10); break;
      case 's': ref_sec = strtoull(optarg, NULL, 10); break;
      case 'd': device = atoi(optarg); break;
      case 'Z': nozero = 1; break;
      case 'R': replay = strtoull(optarg, NULL, 10); break;
      case 'f': layout = optarg; break;
      case 'r': seed = strtoull(optarg, NULL, 10); break;
      case 'u': subband = (uint32_t)strtoul(optarg, NULL, 10); break;
      case 'e': logdir = optarg; break;
      default:
        fprintf(stdout,
                "paf_dfdb -a key -b header -c frames.df -k chunks.u8 [-n nchunk] [-x ref_idf] "
                "[-s ref_sec] [-d dev] [-Z]\n"
                "paf_dfdb -a key -b header -R nblocks [-f bmf|int8:N|int16:N[:be]] [-r seed] [-u subband] "
                "[-d dev]\n");
        return EXIT_FAILURE;
    }
  }
  if (!have_key || !hfile || (!replay && (!dfile || !cfile)) || nchunk < 1 || nchunk > 256) {
    fprintf(stderr, "paf_dfdb: -a, -b and either -c/-k or -R are required (-h for usage)\n");
    return EXIT_FAILURE;
  }
  {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sigemptyset(&sa.sa_mask);
    sa.sa_handler = on_stop;
    sa.sa_flags = SA_RESTART; /* reads and waits carry on; the loops look at g_stop per block */
    sigaction(SIGINT, &sa, NULL);
    sigaction(SIGTERM, &sa, NULL);
  }
  multilog_t *log = multilog_open("paf_dfdb", 0);
  multilog_add(log, stderr);
  FILE *logf = NULL;
  if (logdir) {
    char p[4096];
    snprintf(p, sizeof p, "%s/paf_dfdb.log", logdir);
    if ((logf = fopen(p, "w"))) multilog_add(log, logf);
  }
  int status = EXIT_FAILURE;
  dada_hdu_t *hdu = dada_hdu_create(log);
  dada_hdu_set_key(hdu, key);
  b2p_ctx_t *ctx = NULL;
  FILE *fd = NULL, *fc = NULL;
  unsigned char *hf = NULL, *hc = NULL;
  batch_t bt[NSLOT] = {{0}};
  unsigned long long *d_cnt = NULL;
  void *stage = NULL; /* replay into a host ring: blocks generated on the GPU, copied down */
  int locked = 0;
  if (dada_hdu_connect(hdu) < 0 || dada_hdu_lock_write(hdu) < 0) {
    multilog(log, LOG_ERR, "cannot attach/lock ring %x for writing %s", (unsigned)key, dada_device_error());
    goto done;
  }
  locked = 1;
  ipcbuf_t *db = &hdu->data_block->buf;
  const uint64_t bufsz = ipcbuf_get_bufsz(db), nbufs = ipcbuf_get_nbufs(db);
  const int ondev = ring_device_of(db) >= 0;
  if (!ondev && !replay) {
    multilog(log, LOG_ERR, "ring %x is not GPU-resident (create it with dada_db -g)", (unsigned)key);
    goto done;
  }
  if (ondev) device = ring_device_of(db);

  b2p_geom_t g;
  if (replay) {
    if (parse_layout(layout, &g) < 0) {
      multilog(log, LOG_ERR, "unknown layout '%s'", layout);
      goto done;
    }
  } else {
    b2p_geom_bmf(&g);
    g.nchunk = (uint32_t)nchunk;
  }
  const uint64_t fb = b2p_frame_bytes(&g);
  if (!fb || bufsz % fb) {
    multilog(log, LOG_ERR, "ring block %" PRIu64 " B is not a whole number of %" PRIu64 "-B frames",
             bufsz, fb);
    goto done;
  }
  g.nsamp_int = bufsz / fb * g.nsamp_df;
  int rc = b2p_open(&ctx, &g, device);
  if (rc != B2P_OK) {
    multilog(log, LOG_ERR, "b2p_open: %s (%s)", b2p_strerror(rc), b2p_last_error(NULL));
    goto done;
  }

  /* header ring first (diskdb.cu:75-92 role) */
  char *hb = ipcbuf_get_next_write(hdu->header_block);
  if (!hb || fileread(hfile, hb, HDR_SIZE) < 0 || ipcbuf_mark_filled(hdu->header_block, HDR_SIZE) < 0) {
    multilog(log, LOG_ERR, "cannot pass header %s", hfile);
    goto done;
  }
  const double t0 = now_s();
  uint64_t nblk = 0;
  if (replay) {
    if (!ondev && b2p_dev_alloc(ctx, &stage, bufsz) != B2P_OK) {
      multilog(log, LOG_ERR, "staging block of %" PRIu64 " B: %s", bufsz, b2p_last_error(ctx));
      goto done;
    }
    for (uint64_t i = 0; i < replay && !g_stop; i++) {
      uint64_t bid;
      char *blk = ipcio_open_block_write(hdu->data_block, &bid);
      if (!blk) {
        multilog(log, LOG_ERR, "no block to write in ring %x", (unsigned)key);
        goto done;
      }
      if (i < nbufs) { /* first pass: synthetic block i, then re-used as is */
        if (b2p_fill_synthetic(ctx, ondev ? (void *)blk : stage, bufsz, seed, subband, i, 0) != B2P_OK ||
            b2p_sync(ctx) != B2P_OK || (!ondev && b2p_memcpy(ctx, blk, stage, bufsz, 2) != B2P_OK)) {
          multilog(log, LOG_ERR, "fill: %s", b2p_last_error(ctx));
          goto done;
        }
      }
      ipcio_close_block_write(hdu->data_block, bufsz);
      nblk++;
    }
  } else {
    const uint64_t block_ndf = bufsz / ((uint64_t)nchunk * B2P_DF_PAYLOAD_BYTES);
    const uint64_t cap = block_ndf * (uint64_t)nchunk; /* frames per batch */
    if (!(fd = fopen(dfile, "rb")) || !(fc = fopen(cfile, "rb"))) {
      multilog(log, LOG_ERR, "cannot open %s / %s", dfile, cfile);
      goto done;
    }
    hf = malloc(cap * B2P_DF_BYTES);
    hc = malloc(cap);
    if (!hf || !hc) {
      multilog(log, LOG_ERR, "cannot allocate %" PRIu64 " frames of host staging", cap);
      goto done;
    }
    b2p_register_host(ctx, hf, cap * B2P_DF_BYTES); /* pinned: full PCIe rate */
    for (int k = 0; k < NSLOT; k++)
      if (b2p_dev_alloc(ctx, &bt[k].frames, cap * B2P_DF_BYTES) != B2P_OK ||
          b2p_dev_alloc(ctx, &bt[k].chunks, cap) != B2P_OK) {
        multilog(log, LOG_ERR, "device batch %d: %s", k, b2p_last_error(ctx));
        goto done;
      }
    if (b2p_dev_alloc(ctx, (void **)&d_cnt, (nchunk + 3) * sizeof(unsigned long long)) != B2P_OK) {
      multilog(log, LOG_ERR, "device counters: %s", b2p_last_error(ctx));
      goto done;
    }
    const b2p_df_hdr_t ref0 = {1, ref_idf, ref_sec, 0, 0, 0.0};
    b2p_df_hdr_t ref = ref0;
    /* live batches: slots head, head+1, ... (mod NSLOT), oldest first */
    int head = 0, live = 0, eof = 0;
    int64_t seen_hi = 0; /* latest block any accepted frame fell in */
    uint64_t placed_all = 0, sent_all = 0, dropped = 0;
    for (int64_t b = 0; !g_stop; b++) {
      /* read on until a batch lies wholly past block b+1: no later frame is
       * for block b any more */
      while (!eof) {
        if (live) {
          const batch_t *nw = &bt[(head + live - 1) % NSLOT];
          if (nw->hi >= 0 && nw->lo > b + 1) break;
        }
        if (live == NSLOT) { /* out of slots: the oldest batch goes */
          if (bt[head].hi >= b) dropped += bt[head].n;
          head = (head + 1) % NSLOT;
          live--;
        }
        batch_t *x = &bt[(head + live) % NSLOT];
        if (load_batch(ctx, fd, fc, x, cap, hf, hc, &ref0, block_ndf, b > seen_hi - 1 ? b : seen_hi - 1,
                       seen_hi + 2) < 0) {
          multilog(log, LOG_ERR, "reading the frame stream failed before block %" PRId64, b);
          goto done;
        }
        if (!x->n) {
          eof = 1;
          break;
        }
        sent_all += x->n;
        if (x->hi > seen_hi) seen_hi = x->hi;
        live++;
      }
      int any = 0;
      for (int j = 0; j < live; j++) any |= bt[(head + j) % NSLOT].hi >= b;
      if (!any) break; /* no frame of block b or later is left */
      uint64_t bid;
      char *blk = ipcio_open_block_write(hdu->data_block, &bid);
      if (!blk) {
        multilog(log, LOG_ERR, "no block to write in ring %x", (unsigned)key);
        goto done;
      }
      /* a failure from here on leaves the open block unfilled: the end of
       * the transfer (dada_hdu_unlock_write) marks it as the 0-byte
       * end-of-data block, so no reader integrates a half-assembled block */
      if ((!nozero && b2p_memset(ctx, blk, 0, bufsz) != B2P_OK) ||
          b2p_memset(ctx, d_cnt, 0, (nchunk + 3) * sizeof(unsigned long long)) != B2P_OK) {
        multilog(log, LOG_ERR, "block %" PRId64 ": clearing: %s", b, b2p_last_error(ctx));
        goto done;
      }
      for (int j = 0; j < live; j++) {
        batch_t *x = &bt[(head + j) % NSLOT];
        if (x->hi < b || x->lo > b) continue;
        if (b2p_assemble(ctx, x->frames, x->n, B2P_DF_BYTES, x->chunks, ref.idf, ref.sec, blk,
                         block_ndf, (uint32_t)nchunk, d_cnt) != B2P_OK) {
          multilog(log, LOG_ERR, "assemble: %s", b2p_last_error(ctx));
          goto done;
        }
      }
      unsigned long long cnt[256 + 3];
      if (b2p_sync(ctx) != B2P_OK ||
          b2p_memcpy(ctx, cnt, d_cnt, (nchunk + 3) * sizeof(unsigned long long), 2) != B2P_OK) {
        multilog(log, LOG_ERR, "block %" PRId64 ": assembly: %s", b, b2p_last_error(ctx));
        goto done;
      }
      uint64_t placed = 0;
      for (int c = 0; c < nchunk; c++) placed += cnt[c];
      placed_all += placed;
      ipcio_close_block_write(hdu->data_block, bufsz);
      nblk++;
      multilog(log, LOG_INFO, "block %" PRId64 ": %" PRIu64 " of %" PRIu64 " frames placed (%.3f%% lost), "
               "%llu with a bad chunk", b, placed, cap, 100.0 * (double)(cap - placed) / (double)cap,
               cnt[nchunk + 2]);
      b2p_df_ref_advance(&ref, block_ndf);
      /* batches whose frames all fell in blocks <= b are done with */
      while (live && bt[head].hi <= b) {
        head = (head + 1) % NSLOT;
        live--;
      }
    }
    if (dropped)
      multilog(log, LOG_WARNING, "%" PRIu64 " frames of batches dropped for want of slots (arrival "
               "more than %d blocks out of order)", dropped, NSLOT - 2);
    multilog(log, LOG_INFO, "%" PRIu64 " frames read, %" PRIu64 " placed", sent_all, placed_all);
  }
  if (g_stop) multilog(log, LOG_INFO, "stopped by a signal after %" PRIu64 " blocks: ending the transfer", nblk);
  const double el = now_s() - t0;
  multilog(log, LOG_INFO, "dfdb: %" PRIu64 " blocks of %" PRIu64 " B in %.3f s (%.2f GB/s of blocks)",
           nblk, bufsz, el, el > 0 ? (double)nblk * bufsz / el / 1e9 : 0.0);
  status = EXIT_SUCCESS;

done:
  /* the context first: closing it drains its stream, so no clear or
   * assembly a failure left in flight still writes into a ring block once
   * the ring is detached (its IPC mapping closed) */
  if (ctx) {
    for (int k = 0; k < NSLOT; k++) {
      if (bt[k].frames) b2p_dev_free(ctx, bt[k].frames);
      if (bt[k].chunks) b2p_dev_free(ctx, bt[k].chunks);
    }
    if (d_cnt) b2p_dev_free(ctx, d_cnt);
    if (stage) b2p_dev_free(ctx, stage);
    if (hf) b2p_unregister_host(ctx, hf);
    b2p_close(ctx);
  }
  if (locked) dada_hdu_unlock_write(hdu); /* ends the transfer (EOD) */
  dada_hdu_destroy(hdu);
  free(hf);
  free(hc);
  if (fd) fclose(fd);
  if (fc) fclose(fc);
  multilog_close(log);
  if (logf) fclose(logf);
  return status;
}
