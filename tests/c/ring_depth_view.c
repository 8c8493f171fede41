/* A read depth survives a view on the same handle (libpafdada extension;
 * tests/test_sanitizers.py builds it with ASan+UBSan).
 *
 * libpafdada keeps a process's read depth in ipcbuf_t.viewbuf, which a
 * viewer also uses for its block position.  The handle here sets depth 2,
 * views the ring's first block (its view position becomes 1), closes the
 * view, then locks for reading: it must hold two blocks at once -- with the
 * depth in the low byte it read as depth 1 (its old view position) and the
 * second open returned nothing.  Sequential, one process, two attachments
 * (a writer and the handle under test).  Exit 0 and "errors 0" when well. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "b2p_dada.h"

#define BUFSZ 64
static int errors;
#define FAIL(...)                           \
  do {                                      \
    fprintf(stderr, "line %d: ", __LINE__); \
    fprintf(stderr, __VA_ARGS__);           \
    fputc('\n', stderr);                    \
    errors++;                               \
  } while (0)

static void write_block(ipcio_t *w, char fill) {
  uint64_t id = 0;
  char *p = ipcio_open_block_write(w, &id);
  if (!p) {
    FAIL("open_block_write");
    return;
  }
  memset(p, fill, BUFSZ);
  if (ipcio_close_block_write(w, BUFSZ) < 0) FAIL("close_block_write");
}

int main(int argc, char **argv) {
  const key_t key = argc > 1 ? (key_t)strtol(argv[1], NULL, 16) : 0x7e80 + (getpid() % 64) * 2;
  dada_db_destroy(key);
  if (dada_db_create(key, 4, BUFSZ, 1, 4, 4096)) {
    perror("create");
    return 2;
  }
  ipcio_t w = IPCIO_INIT, h = IPCIO_INIT;
  if (ipcio_connect(&w, key) < 0 || ipcio_open(&w, 'W') < 0) FAIL("writer attach");
  write_block(&w, 'a');
  if (ipcio_connect(&h, key) < 0 || ipcbuf_set_read_depth(&h.buf, 2) < 0 || ipcio_open(&h, 'r') < 0)
    FAIL("viewer attach");
  uint64_t sz = 0, id = 0;
  char *p = ipcio_open_block_read(&h, &sz, &id);
  if (!p || sz != BUFSZ || p[0] != 'a') FAIL("view of block 0: %p %lu", (void *)p, (unsigned long)sz);
  if (p) ipcio_close_block_read(&h, sz);
  if (ipcio_close(&h) < 0) FAIL("close view");
  write_block(&w, 'b');
  write_block(&w, 'c');
  if (ipcio_open(&h, 'R') < 0) FAIL("read lock after the view");
  char *b0 = ipcio_open_block_read(&h, &sz, &id);
  if (!b0 || b0[0] != 'a') FAIL("first held block");
  char *b1 = ipcio_open_block_read(&h, &sz, &id); /* depth 2: a second block while the first is held */
  if (!b1 || b1[0] != 'b') FAIL("second held block (read depth lost to the view position?)");
  if (b0 && ipcio_close_block_read(&h, 0) < 0) FAIL("release 0");
  if (b1 && ipcio_close_block_read(&h, 0) < 0) FAIL("release 1");
  if (ipcio_close(&w) < 0) FAIL("writer close"); /* end of data */
  for (;;) { /* drain to the end of data */
    char *q = ipcio_open_block_read(&h, &sz, &id);
    if (!q) break;
    ipcio_close_block_read(&h, sz);
    if (ipcbuf_eod(&h.buf)) break;
  }
  ipcio_close(&h);
  ipcio_disconnect(&h);
  ipcio_disconnect(&w);
  dada_db_destroy(key);
  printf("errors %d\n", errors);
  return errors ? 1 : 0;
}
