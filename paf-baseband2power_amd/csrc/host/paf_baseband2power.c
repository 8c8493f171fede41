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
 */
#include <getopt.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "b2p.h"
#include "b2p_dada.h"

#define MSTR_LEN 512 /* paf_baseband2power.cuh:4 */
#define TSAMP_BMF_US (27.0 / 32.0) /* README.md:2 */

typedef struct conf_t { /* baseband2power.cuh:18-23, plus layout options */
  int device_id;
  char dir[MSTR_LEN];
  key_t key_in, key_out;
  char layout[64];
  int npol_out;
  int mean;
} conf_t;

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
          " -h  show help\n");
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
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

int main(int argc, char *argv[]) {
  int arg;
  conf_t conf;
  memset(&conf, 0, sizeof conf);
  conf.npol_out = 1;
  strcpy(conf.dir, ".");
  int have_in = 0, have_out = 0;

  while ((arg = getopt(argc, argv, "a:b:c:d:f:p:mh")) != -1) {
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
      case 'c':
        snprintf(conf.dir, sizeof conf.dir, "%s", optarg);
        break;
      case 'd':
        sscanf(optarg, "%d", &conf.device_id);
        break;
      case 'f':
        snprintf(conf.layout, sizeof conf.layout, "%s", optarg);
        break;
      case 'p':
        conf.npol_out = atoi(optarg);
        break;
      case 'm':
        conf.mean = 1;
        break;
      default:
        usage();
        return EXIT_FAILURE;
    }
  }
  if (!have_in || !have_out) {
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
  multilog_t *log = multilog_open("paf_baseband2power", 0);
  multilog_add(log, fp_log);
  multilog(log, LOG_INFO, "START PAF_PROCESS");

  /* only one visible GPU => index 0 (paf_baseband2power.cu:86-90) */
  int ndev = 0;
  if (b2p_device_count(&ndev) != B2P_OK || ndev < 1) {
    multilog(log, LOG_ERR, "no HIP device: %s", b2p_last_error(NULL));
    fprintf(stderr, "no HIP device\n");
    return EXIT_FAILURE;
  }
  if (ndev == 1) conf.device_id = 0;

  int status = EXIT_FAILURE;
  b2p_ctx_t *ctx = NULL;
  float *spec = NULL;
  dada_hdu_t *in = dada_hdu_create(log), *out = dada_hdu_create(log);
  dada_hdu_set_key(in, conf.key_in);
  dada_hdu_set_key(out, conf.key_out);
  int in_locked = 0, out_locked = 0;
  uint64_t nblocks = 0, nskipped = 0;

  if (dada_hdu_connect(in) < 0 || dada_hdu_lock_read(in) < 0) {
    multilog(log, LOG_ERR, "cannot attach/lock input ring %x", conf.key_in);
    goto done;
  }
  in_locked = 1;
  if (dada_hdu_open_read(in) < 0) {
    multilog(log, LOG_ERR, "no header on input ring");
    goto done;
  }
  const uint64_t rbufsz = ipcbuf_get_bufsz(&in->data_block->buf);
  b2p_geom_t g;
  double tsamp_us = TSAMP_BMF_US;
  if (pick_geometry(&conf, in->header, rbufsz, &g, &tsamp_us, log) < 0) goto done;

  int rc = b2p_open(&ctx, &g, conf.device_id);
  if (rc != B2P_OK) {
    multilog(log, LOG_ERR, "b2p_open: %s (%s)", b2p_strerror(rc), b2p_last_error(NULL));
    goto done;
  }
  b2p_info_t info;
  b2p_get_info(ctx, &info);
  multilog(log, LOG_INFO,
           "layout nbit %u %s, %u chunks x %u chans x %u samp/DF, %u outputs, %" PRIu64
           " samples per integration, GPU %d",
           g.nbit, g.big_endian ? "BE" : "LE", g.nchunk, g.nchan_chunk, g.nsamp_df, info.nout,
           g.nsamp_int, (int)info.device);
  /* pin the input ring's blocks for DMA (dada_cuda_dbregister role) */
  for (uint64_t i = 0; i < ipcbuf_get_nbufs(&in->data_block->buf); i++) {
    rc = b2p_register_host(ctx, ipcbuf_get_buffer(&in->data_block->buf, i), rbufsz);
    if (rc != B2P_OK) multilog(log, LOG_INFO, "register block %" PRIu64 ": %s", i, b2p_last_error(ctx));
  }

  if (dada_hdu_connect(out) < 0 || dada_hdu_lock_write(out) < 0) {
    multilog(log, LOG_ERR, "cannot attach/lock output ring %x", conf.key_out);
    goto done;
  }
  out_locked = 1;
  const uint64_t obytes = (uint64_t)info.nout * sizeof(float);
  if (ipcbuf_get_bufsz(&out->data_block->buf) != obytes) {
    /* same check as diskdb.cu:36-42, for the output ring (py:77-79) */
    multilog(log, LOG_ERR, "output ring block %" PRIu64 " B != NCHAN x NPOL x 4 = %" PRIu64 " B",
             ipcbuf_get_bufsz(&out->data_block->buf), obytes);
    goto done;
  }

  /* output header: NBIT 32, NDIM 1, NPOL, NCHAN (header_baseband2power.txt:36-42) */
  {
    char *ohdr = ipcbuf_get_next_write(out->header_block);
    uint64_t ohsz = ipcbuf_get_bufsz(out->header_block);
    if (!ohdr) goto done;
    memset(ohdr, 0, ohsz);
    memcpy(ohdr, in->header, in->header_size < ohsz ? in->header_size : ohsz);
    ohdr[ohsz - 1] = 0;
    const double tsamp_out = tsamp_us * (double)g.nsamp_int;
    double tmpl = 0;
    if (ascii_header_get(ohdr, "TSAMP", "%lf", &tmpl) == 1 && tmpl != tsamp_out)
      multilog(log, LOG_INFO, "TSAMP %.6g us in the input header replaced by %.6f us "
               "(= %.6f us x %" PRIu64 ")", tmpl, tsamp_out, tsamp_us, g.nsamp_int);
    ascii_header_set(ohdr, "NBIT", "%d", 32);
    ascii_header_set(ohdr, "NDIM", "%d", 1);
    ascii_header_set(ohdr, "NPOL", "%u", g.npol_out);
    ascii_header_set(ohdr, "NCHAN", "%u", info.nchan);
    ascii_header_set(ohdr, "TSAMP", "%.6f", tsamp_out);
    ascii_header_set(ohdr, "BYTES_PER_SECOND", "%.6f", obytes / (tsamp_out * 1e-6));
    ascii_header_set(ohdr, "NSAMP_INT", "%" PRIu64, g.nsamp_int);
    ascii_header_set(ohdr, "POWER_MODE", "%s", g.mean ? "MEAN" : "SUM");
    ascii_header_del(ohdr, "NCHUNK");
    ascii_header_del(ohdr, "NCHAN_CHUNK");
    ascii_header_del(ohdr, "NSAMP_DF");
    ascii_header_del(ohdr, "BYTE_ORDER");
    if (ipcbuf_mark_filled(out->header_block, ohsz) < 0) goto done;
  }

  spec = aligned_alloc(4096, (obytes + 4095) / 4096 * 4096);
  if (!spec) goto done;
  b2p_register_host(ctx, spec, (obytes + 4095) / 4096 * 4096);

  for (;;) {
    uint64_t bytes = 0, bid = 0;
    char *blk = ipcio_open_block_read(in->data_block, &bytes, &bid);
    if (!blk) break; /* end of data */
    if (bytes != rbufsz) {
      multilog(log, LOG_INFO, "partial integration skipped: block %" PRIu64 " holds %" PRIu64
               " of %" PRIu64 " B", bid, bytes, rbufsz);
      ipcio_close_block_read(in->data_block, bytes);
      nskipped++;
      continue;
    }
    const double t0 = now_s();
    rc = b2p_push(ctx, blk, bytes, 0); /* returns once the block is copied */
    ipcio_close_block_read(in->data_block, bytes);
    if (rc != B2P_OK) {
      multilog(log, LOG_ERR, "b2p_push: %s (%s)", b2p_strerror(rc), b2p_last_error(ctx));
      goto done;
    }
    rc = b2p_finish(ctx, spec);
    if (rc != B2P_OK) {
      multilog(log, LOG_ERR, "b2p_finish: %s (%s)", b2p_strerror(rc), b2p_last_error(ctx));
      goto done;
    }
    char *o = ipcio_open_block_write(out->data_block, &bid);
    if (!o) goto done;
    memcpy(o, spec, obytes);
    ipcio_close_block_write(out->data_block, obytes);
    const double dt = now_s() - t0;
    nblocks++;
    multilog(log, LOG_INFO, "integration %" PRIu64 ": %.3f ms, %.2f GB/s, %.1f Msamples/s",
             nblocks, dt * 1e3, bytes / dt / 1e9,
             (double)info.nchan * g.npol * g.nsamp_int / dt / 1e6);
  }
  status = EXIT_SUCCESS;

done:
  if (out_locked) dada_hdu_unlock_write(out); /* ends the output transfer (EOD) */
  if (in_locked) dada_hdu_unlock_read(in);
  if (ctx) {
    for (uint64_t i = 0; in->data_block && i < ipcbuf_get_nbufs(&in->data_block->buf); i++)
      b2p_unregister_host(ctx, ipcbuf_get_buffer(&in->data_block->buf, i));
    if (spec) b2p_unregister_host(ctx, spec);
    b2p_close(ctx);
  }
  free(spec);
  dada_hdu_destroy(in);
  dada_hdu_destroy(out);
  multilog(log, LOG_INFO, "FINISH PAF_PROCESS: %" PRIu64 " integrations, %" PRIu64 " skipped, %s",
           nblocks, nskipped, status == EXIT_SUCCESS ? "ok" : "FAILED");
  multilog_close(log);
  fclose(fp_log);
  return status;
}
