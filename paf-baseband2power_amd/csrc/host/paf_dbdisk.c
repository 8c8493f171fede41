/*
 * paf_dbdisk -- write a DADA ring to disk (the sink stage the reference runs
 * as PSRDADA's `dada_dbdisk -b cpu -k key -D dir -W`, paf-baseband2power.py
 * :94-95).  Attaches as a reader, waits for the header, writes
 * "<dir>/<UTC_START>_<OBS_OFFSET>.000000.dada" = 4096-B header + every data
 * block until end of data.
 *   -k key   -D dir   -b cpu (accepted, ignored)   -W (accepted: overwrite)
 *   -o file  explicit output path (instead of the DADA naming rule)
 */
#include <getopt.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "b2p_dada.h"

static void usage(void) {
  fprintf(stdout,
          "paf_dbdisk - write a DADA ring buffer to a file\n"
          "Usage: paf_dbdisk -k key -D dir [-o file] [-W] [-b cpu]\n");
}

int main(int argc, char **argv) {
  key_t key = 0xdada;
  char dir[512] = ".", ofile[1024] = "";
  int arg;
  while ((arg = getopt(argc, argv, "k:D:o:b:Wsh")) != -1) {
    switch (arg) {
      case 'k':
        if (sscanf(optarg, "%x", (unsigned *)&key) != 1) {
          fprintf(stderr, "Could not parse key from %s\n", optarg);
          return EXIT_FAILURE;
        }
        break;
      case 'D': snprintf(dir, sizeof dir, "%s", optarg); break;
      case 'o': snprintf(ofile, sizeof ofile, "%s", optarg); break;
      case 'b': case 'W': case 's': break;
      default: usage(); return EXIT_FAILURE;
    }
  }
  multilog_t *log = multilog_open("paf_dbdisk", 0);
  multilog_add(log, stderr);
  dada_hdu_t *hdu = dada_hdu_create(log);
  dada_hdu_set_key(hdu, key);
  if (dada_hdu_connect(hdu) < 0 || dada_hdu_lock_read(hdu) < 0) {
    fprintf(stderr, "paf_dbdisk: cannot attach/lock ring %x\n", (unsigned)key);
    return EXIT_FAILURE;
  }
  if (dada_hdu_open_read(hdu) < 0) {
    fprintf(stderr, "paf_dbdisk: no header\n");
    return EXIT_FAILURE;
  }
  if (!ofile[0]) {
    char utc[128] = "unset";
    uint64_t off = 0;
    ascii_header_get(hdu->header, "UTC_START", "%127s", utc);
    ascii_header_get(hdu->header, "OBS_OFFSET", "%" SCNu64, &off);
    snprintf(ofile, sizeof ofile, "%s/%s_%016" PRIu64 ".000000.dada", dir, utc, off);
  }
  FILE *fp = fopen(ofile, "wb");
  if (!fp) {
    fprintf(stderr, "paf_dbdisk: cannot open %s\n", ofile);
    return EXIT_FAILURE;
  }
  int rc = EXIT_SUCCESS;
  if (fwrite(hdu->header, 1, hdu->header_size, fp) != hdu->header_size) rc = EXIT_FAILURE;
  uint64_t total = 0, nblk = 0;
  ipcbuf_t *db = &hdu->data_block->buf;
  char *stage = NULL; /* a GPU-resident ring's blocks come back through host */
  if (ipcbuf_get_device(db) >= 0 && !(stage = malloc(ipcbuf_get_bufsz(db)))) rc = EXIT_FAILURE;
  for (; rc == EXIT_SUCCESS;) {
    uint64_t bytes = 0, bid = 0;
    char *b = ipcio_open_block_read(hdu->data_block, &bytes, &bid);
    if (!b) break;
    if (stage && ipcbuf_copy_out(db, stage, b, bytes) < 0) rc = EXIT_FAILURE;
    if (bytes && fwrite(stage ? stage : b, 1, bytes, fp) != bytes) rc = EXIT_FAILURE;
    ipcio_close_block_read(hdu->data_block, bytes);
    total += bytes;
    if (bytes) nblk++; /* a 0-byte block only carries the end of data */
  }
  free(stage);
  fclose(fp);
  multilog(log, LOG_INFO, "dbdisk: %s: %" PRIu64 " B in %" PRIu64 " blocks", ofile, total, nblk);
  dada_hdu_unlock_read(hdu);
  dada_hdu_destroy(hdu);
  multilog_close(log);
  return rc;
}
