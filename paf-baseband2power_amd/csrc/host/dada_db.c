/*
 * dada_db -- create or destroy a ring pair (data at key, header at key+1),
 * the tool the reference's launcher calls (paf-baseband2power.py:114-115
 * "dada_db -l -p -k KEY -b BUFSZ -n NBUFS -r NREADERS", :129-130 "-d").
 *   -k key -b bufsz -n nbufs -r nreaders [-l] [-p] [-g dev]   create
 *   -k key -d                                                  destroy
 * -l locks the segments in RAM (SHM_LOCK, as PSRDADA's dada_db -l; it
 * needs CAP_IPC_LOCK or a large enough RLIMIT_MEMLOCK, and the ring is
 * removed again if that fails) and -p touches every host block's pages.  -g dev puts the data blocks in that GPU's memory (PSRDADA's
 * device rings): a holder process keeps them until -d.
 */
#include <getopt.h>
#include <inttypes.h>
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "b2p_dada.h"

int main(int argc, char **argv) {
  key_t key = 0xdada;
  uint64_t bufsz = 524288, nbufs = 4, hdr_nbufs = 8, hdr_bufsz = DADA_DEFAULT_HEADER_SIZE;
  unsigned nread = 1;
  int destroy = 0, page = 0, lock = 0, device = -1, arg;
  while ((arg = getopt(argc, argv, "k:b:n:r:dlpH:g:h")) != -1) {
    switch (arg) {
      case 'k':
        if (sscanf(optarg, "%x", (unsigned *)&key) != 1) {
          fprintf(stderr, "dada_db: could not parse key from %s\n", optarg);
          return EXIT_FAILURE;
        }
        break;
      case 'b': bufsz = strtoull(optarg, NULL, 10); break;
      case 'n': nbufs = strtoull(optarg, NULL, 10); break;
      case 'r': nread = (unsigned)atoi(optarg); break;
      case 'H': hdr_bufsz = strtoull(optarg, NULL, 10); break;
      case 'd': destroy = 1; break;
      case 'l': lock = 1; break;
      case 'p': page = 1; break;
      case 'g': device = atoi(optarg); break;
      default:
        fprintf(stdout, "dada_db -k key -b bufsz -n nbufs -r nreaders [-l -p] [-g device] | -k key -d\n");
        return EXIT_FAILURE;
    }
  }
  if (destroy) {
    if (dada_db_destroy(key) < 0) {
      if (errno == EBUSY) /* a device ring's holder still serves attached processes */
        fprintf(stderr, "dada_db: ring %x removed, %s\n", (unsigned)key, dada_device_error());
      else
        fprintf(stderr, "dada_db: nothing (complete) to destroy at key %x\n", (unsigned)key);
      return EXIT_FAILURE;
    }
    return EXIT_SUCCESS;
  }
  if (dada_db_create_work(key, nbufs, bufsz, nread, hdr_nbufs, hdr_bufsz, device) < 0) {
    perror("dada_db: create");
    return EXIT_FAILURE;
  }
  int rc = EXIT_SUCCESS;
  for (int r = 0; (page || lock) && r < 2; r++) { /* data ring, then header ring */
    ipcbuf_t b = IPCBUF_INIT;
    if (r == 0 && device >= 0) continue; /* device blocks: zeroed by their holder, not lockable */
    if (ipcbuf_connect(&b, key + r) < 0) continue;
    if (page) ipcbuf_page(&b);
    if (lock && ipcbuf_lock(&b) < 0) {
      /* PSRDADA's ipcbuf_lock needs CAP_IPC_LOCK or a large RLIMIT_MEMLOCK */
      perror("dada_db: -l: cannot lock the ring in RAM");
      rc = EXIT_FAILURE;
    }
    ipcbuf_disconnect(&b);
  }
  if (rc != EXIT_SUCCESS) {
    dada_db_destroy(key);
    return rc;
  }
  fprintf(stdout, "dada_db: key %x: %" PRIu64 " x %" PRIu64 " B, %u reader(s)%s\n", (unsigned)key,
          nbufs, bufsz, nread, device >= 0 ? " on the GPU" : "");
  return EXIT_SUCCESS;
}
