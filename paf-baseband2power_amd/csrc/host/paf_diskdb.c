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
 * return value, paf_diskdb.cu:65), and -l names a log file (the reference's
 * conf.log was never initialised, paf_diskdb.cu:28).
 *
 * -DB2P_PSRDADA builds it against PSRDADA's own headers and the PSRDADA
 * subset the reference calls, as the reference is
 * built; GPU-resident rings (a libpafdada extension) are then off.
 */
#include <getopt.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

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

typedef struct conf_t { /* diskdb.cuh:19-30 */
  key_t key;
  int sod;
  char fname[2 * MSTR_LEN + 2], hfname[MSTR_LEN];
  FILE *fp;
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
          " -h Show help    \n");
}

static int init_diskdb(conf_t *conf) {
  conf->fp = fopen(conf->fname, "r");
  if (!conf->fp) {
    fprintf(stderr, "Can not open file: %s\n", conf->fname);
    return EXIT_FAILURE;
  }
  conf->hdu = dada_hdu_create(conf->log);
  dada_hdu_set_key(conf->hdu, conf->key);
  if (dada_hdu_connect(conf->hdu) < 0) {
    multilog(conf->log, LOG_ERR, "could not connect to hdu");
    fprintf(stderr, "Can not connect to hdu %x\n", (unsigned)conf->key);
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
  fseek(conf->fp, DADA_HDR_SIZE, SEEK_SET);
  return EXIT_SUCCESS;
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
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
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
  while (!feof(conf->fp)) {
    char *curbuf = ipcio_open_block_write(conf->hdu->data_block, &block_id);
    if (!curbuf) {
      free(stage);
      return EXIT_FAILURE;
    }
    size_t n = fread(stage ? stage : curbuf, 1, conf->rbufsz, conf->fp);
#ifndef B2P_PSRDADA
    if (stage && ipcbuf_copy_in(db, curbuf, stage, n) < 0) {
      multilog(conf->log, LOG_ERR, "copy into device block failed");
      free(stage);
      return EXIT_FAILURE;
    }
#endif
    ipcio_close_block_write(conf->hdu->data_block, n);
    total += n;
    nblk++;
    if (n < conf->rbufsz) break; /* the short block already ended the transfer */
  }
  free(stage);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  double el = (double)(t1.tv_sec - t0.tv_sec) + (double)(t1.tv_nsec - t0.tv_nsec) * 1e-9;
  multilog(conf->log, LOG_INFO, "diskdb: %" PRIu64 " B in %" PRIu64 " blocks, %.3f s (%.2f GB/s)",
           total, nblk, el, el > 0 ? (double)total / el / 1e9 : 0.0);
  return EXIT_SUCCESS;
}

static int destroy_diskdb(conf_t *conf) {
  if (conf->hdu) {
    dada_hdu_unlock_write(conf->hdu);
    dada_hdu_disconnect(conf->hdu);
    dada_hdu_destroy(conf->hdu);
  }
  if (conf->fp) fclose(conf->fp);
  return EXIT_SUCCESS;
}

int main(int argc, char **argv) {
  int arg;
  char fdir[MSTR_LEN] = ".", fname[MSTR_LEN] = "", logname[MSTR_LEN] = "";
  conf_t conf;
  memset(&conf, 0, sizeof conf);
  int have_key = 0;
  while ((arg = getopt(argc, argv, "a:b:c:d:e:l:h")) != -1) {
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

  int rc = init_diskdb(&conf);
  if (rc == EXIT_SUCCESS) rc = do_diskdb(&conf);
  destroy_diskdb(&conf);
  multilog_close(conf.log);
  if (lf) fclose(lf);
  return rc;
}
