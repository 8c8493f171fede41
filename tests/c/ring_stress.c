/* Host-side stress of the DADA layer (include/b2p_dada.h) for sanitizer
 * builds: one writer thread, two reader threads (one holding a single block,
 * one holding two with the read-depth extension), many small blocks through
 * a 3-block ring, a short final block (EOD), header get/set/del round trips.
 * Exit 0 = every block arrived intact in order at every reader. */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "b2p_dada.h"

#define NBLK 200
#define BUFSZ 4096

static key_t key;
static int errors;
#define FAIL() __atomic_add_fetch(&errors, 1, __ATOMIC_RELAXED)

static void fill(char *p, int i, uint64_t n) {
  for (uint64_t k = 0; k < n; k++) p[k] = (char)((i * 131 + k * 7) & 0xff);
}

static void *writer(void *arg) {
  (void)arg;
  dada_hdu_t *h = dada_hdu_create(NULL);
  dada_hdu_set_key(h, key);
  if (dada_hdu_connect(h) || dada_hdu_lock_write(h)) { FAIL(); return NULL; }
  char *hb = ipcbuf_get_next_write(h->header_block);
  memset(hb, 0, ipcbuf_get_bufsz(h->header_block));
  strcpy(hb, "HDR_SIZE 4096\nNCHAN 336 # chans\n");
  ascii_header_set(hb, "NBIT", "%d", 32);
  ascii_header_set(hb, "NCHAN", "%d", 1024);
  ipcbuf_mark_filled(h->header_block, ipcbuf_get_bufsz(h->header_block));
  for (int i = 0; i < NBLK; i++) {
    uint64_t id;
    char *p = ipcio_open_block_write(h->data_block, &id);
    uint64_t n = i == NBLK - 1 ? BUFSZ / 2 : BUFSZ;
    fill(p, i, n);
    ipcio_close_block_write(h->data_block, n);
  }
  dada_hdu_unlock_write(h);
  dada_hdu_destroy(h);
  return NULL;
}

static void *reader(void *arg) {
  const int depth = (int)(intptr_t)arg;
  dada_hdu_t *h = dada_hdu_create(NULL);
  dada_hdu_set_key(h, key);
  if (dada_hdu_connect(h) || dada_hdu_lock_read(h) || dada_hdu_open_read(h)) { FAIL(); return NULL; }
  if (depth > 1 && ipcbuf_set_read_depth(&h->data_block->buf, depth)) FAIL();
  int nchan = 0, nbit = 0;
  if (ascii_header_get(h->header, "NCHAN", "%d", &nchan) != 1 || nchan != 1024) FAIL();
  if (ascii_header_get(h->header, "NBIT", "%d", &nbit) != 1 || nbit != 32) FAIL();
  char *want = malloc(BUFSZ);
  int i = 0, held = 0;
  for (;; i++) {
    uint64_t n, id;
    char *p = ipcio_open_block_read(h->data_block, &n, &id);
    if (!p) break;
    fill(want, i, n);
    if (memcmp(p, want, n) || (i < NBLK - 1 && n != BUFSZ)) FAIL();
    if (++held == depth) { /* release the oldest, keep the rest */
      ipcio_close_block_read(h->data_block, n);
      held--;
    }
  }
  while (held-- > 0) ipcio_close_block_read(h->data_block, 0);
  if (i != NBLK || !ipcbuf_eod(&h->data_block->buf)) FAIL();
  free(want);
  dada_hdu_unlock_read(h);
  dada_hdu_destroy(h);
  return NULL;
}

int main(int argc, char **argv) {
  key = argc > 1 ? (key_t)strtol(argv[1], NULL, 16) : 0x7e00 + (getpid() % 256) * 2;
  dada_db_destroy(key);
  if (dada_db_create(key, 3, BUFSZ, 2, 4, 4096)) { perror("create"); return 2; }
  pthread_t w, r1, r2;
  pthread_create(&r1, NULL, reader, (void *)(intptr_t)1);
  pthread_create(&r2, NULL, reader, (void *)(intptr_t)2);
  pthread_create(&w, NULL, writer, NULL);
  pthread_join(w, NULL);
  pthread_join(r1, NULL);
  pthread_join(r2, NULL);
  /* header edge cases */
  char hdr[4096] = "A 1\nKEY  old   # keep me\nB 2";
  ascii_header_set(hdr, "KEY", "%s", "a-much-longer-value");
  ascii_header_set(hdr, "NEW", "%d", 7);
  ascii_header_del(hdr, "A");
  char v[64] = "";
  if (ascii_header_get(hdr, "KEY", "%63s", v) != 1 || strcmp(v, "a-much-longer-value")) FAIL();
  if (!strstr(hdr, "# keep me") || ascii_header_get(hdr, "A", "%63s", v) != -1) FAIL();
  dada_db_destroy(key);
  printf("errors %d\n", errors);
  return errors ? 1 : 0;
}
