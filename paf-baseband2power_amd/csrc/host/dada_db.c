/*
 * dada_db -- create or destroy a ring pair (data at key, header at key+1),
 * the tool the reference's launcher calls (paf-baseband2power.py:114-115
 * "dada_db -l -p -k KEY -b BUFSZ -n NBUFS -r NREADERS", :129-130 "-d").
 *   -k key -b bufsz -n nbufs -r nreaders [-l] [-p] [-g dev]   create
 *   -k key -d                                                  destroy
 * -l (lock in RAM) and -p (page in) are accepted; pages are touched when
 * -p is given.  -g dev puts the data blocks in that GPU's memory (PSRDADA's
 * device rings): a holder process keeps them until -d.
 */
#include <getopt.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "b2p_dada.h"

int main(int argc, char **argv) {
  key_t key = 0xdada;
  uint64_t bufsz = 524288, nbufs = 4, hdr_nbufs = 8, hdr_bufsz = DADA_DEFAULT_HEADER_SIZE;
  unsigned nread = 1;
  int destroy = 0, page = 0, device = -1, arg;
  while ((arg = getopt(argc, argv, "k:b:n:r:dlpH:g:h")) != -1) {
    switch (arg) {
      case 'k':
        if (sscanf(optarg, "%x", (unsigned *)&key) != 1) return EXIT_FAILURE;
        break;
      case 'b': bufsz = strtoull(optarg, NULL, 10); break;
      case 'n': nbufs = strtoull(optarg, NULL, 10); break;
      case 'r': nread = (unsigned)atoi(optarg); break;
      case 'H': hdr_bufsz = strtoull(optarg, NULL, 10); break;
      case 'd': destroy = 1; break;
      case 'l': break;
      case 'p': page = 1; break;
      case 'g': device = atoi(optarg); break;
      default:
        fprintf(stdout, "dada_db -k key -b bufsz -n nbufs -r nreaders [-l -p] [-g device] | -k key -d\n");
        return EXIT_FAILURE;
    }
  }
  if (destroy) {
    if (dada_db_destroy(key) < 0) {
      fprintf(stderr, "dada_db: nothing (complete) to destroy at key %x\n", (unsigned)key);
      return EXIT_FAILURE;
    }
    return EXIT_SUCCESS;
  }
  if (dada_db_create_work(key, nbufs, bufsz, nread, hdr_nbufs, hdr_bufsz, device) < 0) {
    perror("dada_db: create");
    return EXIT_FAILURE;
  }
  if (page && device < 0) { /* device blocks are zeroed by their holder */
    ipcbuf_t b = IPCBUF_INIT;
    if (ipcbuf_connect(&b, key) == 0) {
      for (uint64_t i = 0; i < nbufs; i++) memset(ipcbuf_get_buffer(&b, i), 0, bufsz);
      ipcbuf_disconnect(&b);
    }
  }
  fprintf(stdout, "dada_db: key %x: %" PRIu64 " x %" PRIu64 " B, %u reader(s)%s\n", (unsigned)key,
          nbufs, bufsz, nread, device >= 0 ? " on the GPU" : "");
  return EXIT_SUCCESS;
}
