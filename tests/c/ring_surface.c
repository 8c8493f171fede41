/* Sanitizer driver for the rest of libpafdada's PSRDADA surface (round 3's
 * additions), threads in one process, each with its own attachment of the
 * ring (tests/test_sanitizers.py builds it with ASan+UBSan and with TSan):
 *
 *   writer    round 0: ipcio 'w' -- bytes written before the start of data
 *             stay invisible, ipcio_start names a stream byte mid-block,
 *             ipcio_stop ends the transfer and keeps the lock, three times,
 *             then ipcio_close; ipcbuf_reset (writer) once both readers have
 *             everything; round 1: two 'W' transfers with ipcio_write, the
 *             second spanning the block where round 0's second transfer
 *             ended (a reset must not leave that end behind) and watched by
 *             a viewer; ipcbuf_hard_reset from a fresh attachment while
 *             nobody reads; round 2: one transfer of whole blocks
 *             (open/close_block_write) ended by a short block.
 *   reader 1  read depth 1, ipcio_read in odd-sized pieces, ipcio_tell and
 *             ipcio_seek (back within the block, then forward by reading).
 *   reader 2  read depth 2 set BEFORE the read lock, holding two blocks at
 *             a time with ipcio_open_block_read / close_block_read.
 *   viewer    ipcio 'r' attached during round 1's second transfer: follows
 *             the writer, takes nothing, stops at the end of data.
 * Every reader checks every transfer byte for byte against the stream the
 * writer published (start and end byte per transfer).  Exit 0 and
 * "errors 0" when all is well. */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "b2p_dada.h"

#define BUFSZ 256
#define NBUFS 4
#define NROUND 3
static const int kXfers[NROUND] = {3, 2, 1};

static key_t key;
static int errors;
#define FAIL(...)                                       \
  do {                                                  \
    fprintf(stderr, "line %d: ", __LINE__);             \
    fprintf(stderr, __VA_ARGS__);                       \
    fputc('\n', stderr);                                \
    __atomic_add_fetch(&errors, 1, __ATOMIC_RELAXED);   \
  } while (0)

/* the writer's published transfers: [start, end) stream bytes of each */
static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t cv = PTHREAD_COND_INITIALIZER;
static uint64_t xs[NROUND][4], xe[NROUND][4];
static int viewer_go, viewer_done, viewer_blocks;
static pthread_barrier_t bar; /* writer, 2 readers, viewer: between rounds 1 and 2 */

static char byte_at(int round, uint64_t p) { return (char)((p * 131 + (p >> 8) * 7 + (uint64_t)round * 29) & 0xff); }

static void fill(char *dst, int round, uint64_t p, uint64_t n) {
  for (uint64_t i = 0; i < n; i++) dst[i] = byte_at(round, p + i);
}

static void check(const char *who, int round, int t, const char *got, uint64_t n) {
  pthread_mutex_lock(&mu);
  const uint64_t s = xs[round][t], e = xe[round][t];
  pthread_mutex_unlock(&mu);
  if (n != e - s) {
    FAIL("%s: round %d transfer %d: %lu bytes, want %lu", who, round, t, (unsigned long)n, (unsigned long)(e - s));
    return;
  }
  for (uint64_t i = 0; i < n; i++)
    if (got[i] != byte_at(round, s + i)) {
      FAIL("%s: round %d transfer %d: byte %lu differs", who, round, t, (unsigned long)i);
      return;
    }
}

static void publish(uint64_t *slot, uint64_t v) {
  pthread_mutex_lock(&mu);
  *slot = v;
  pthread_mutex_unlock(&mu);
}

/* ipcio_write of n stream bytes from absolute position *pos, in 29-B pieces */
static void write_stream(ipcio_t *w, int round, uint64_t *pos, uint64_t n) {
  char piece[29];
  while (n) {
    const uint64_t k = n < sizeof piece ? n : sizeof piece;
    fill(piece, round, *pos, k);
    if (ipcio_write(w, piece, k) != (ssize_t)k) {
      FAIL("ipcio_write");
      return;
    }
    *pos += k;
    n -= k;
  }
}

static void *writer(void *arg) {
  (void)arg;
  ipcio_t w = IPCIO_INIT;
  if (ipcio_connect(&w, key) < 0) {
    FAIL("writer connect");
    return NULL;
  }
  /* round 0: deferred start of data */
  if (ipcio_open(&w, 'w') < 0) FAIL("ipcio_open w");
  uint64_t pos = 0;
  for (int t = 0; t < kXfers[0]; t++) {
    write_stream(&w, 0, &pos, 2 * BUFSZ + 60 + 17 * (uint64_t)t); /* invisible to the readers */
    const uint64_t start = pos - 20; /* mid-block, inside what this phase wrote */
    publish(&xs[0][t], start);
    if (ipcio_start(&w, start) < 0) FAIL("ipcio_start %d", t);
    write_stream(&w, 0, &pos, 5 * BUFSZ + 33 * (uint64_t)t + 7);
    publish(&xe[0][t], pos);
    if (t + 1 < kXfers[0] ? ipcio_stop(&w) < 0 : ipcio_close(&w) < 0) FAIL("stop/close %d", t);
  }
  /* writer reset: waits until both readers cleared and acknowledged it all */
  if (ipcio_open(&w, 'W') < 0 || ipcbuf_reset(&w.buf) < 0) FAIL("writer reset");
  if (ipcbuf_get_write_count(&w.buf) != 0) FAIL("w_buf after reset");
  /* round 1: two 'W' transfers; the viewer watches the second */
  pos = 0;
  publish(&xs[1][0], pos);
  write_stream(&w, 1, &pos, 2 * BUFSZ + 100);
  publish(&xe[1][0], pos);
  if (ipcio_close(&w) < 0) FAIL("close r1 t0");
  if (ipcio_open(&w, 'W') < 0) FAIL("open r1 t1");
  pos = ipcbuf_get_write_count(&w.buf) * BUFSZ; /* the transfer starts at the next block */
  publish(&xs[1][1], pos);
  write_stream(&w, 1, &pos, 3 * BUFSZ);
  pthread_mutex_lock(&mu);
  viewer_go = 1;
  pthread_cond_broadcast(&cv);
  pthread_mutex_unlock(&mu);
  for (int k = 0; k < 14; k++) { /* slow enough for the viewer's 0.1-s polls to see blocks */
    write_stream(&w, 1, &pos, BUFSZ);
    usleep(15000);
  }
  write_stream(&w, 1, &pos, 45);
  publish(&xe[1][1], pos);
  if (ipcio_close(&w) < 0) FAIL("close r1 t1");
  pthread_barrier_wait(&bar); /* readers and viewer are done with round 1 */
  {
    ipcbuf_t hb = IPCBUF_INIT;
    if (ipcbuf_connect(&hb, key) < 0 || ipcbuf_hard_reset(&hb) < 0) FAIL("hard reset");
    ipcbuf_disconnect(&hb);
  }
  pthread_barrier_wait(&bar);
  /* round 2: whole blocks, a short one ends it */
  if (ipcio_open(&w, 'W') < 0) FAIL("open r2");
  publish(&xs[2][0], 0);
  uint64_t p2 = 0;
  for (int i = 0; i < 5; i++) {
    uint64_t id;
    char *b = ipcio_open_block_write(&w, &id);
    if (!b) {
      FAIL("open_block_write");
      break;
    }
    const uint64_t n = i == 4 ? BUFSZ / 3 : BUFSZ;
    fill(b, 2, p2, n);
    p2 += n;
    if (i == 4) publish(&xe[2][0], p2);
    if (ipcio_close_block_write(&w, n) < 0) FAIL("close_block_write");
  }
  if (ipcio_close(&w) < 0) FAIL("close r2");
  ipcio_disconnect(&w);
  return NULL;
}

/* reader 1: byte stream, tell / seek */
static void *reader_stream(void *arg) {
  (void)arg;
  ipcio_t r = IPCIO_INIT;
  if (ipcio_connect(&r, key) < 0 || ipcio_open(&r, 'R') < 0) {
    FAIL("reader 1 attach");
    return NULL;
  }
  char *got = malloc(64 * BUFSZ);
  for (int round = 0; round < NROUND; round++) {
    for (int t = 0; t < kXfers[round]; t++) {
      const uint64_t t0 = ipcio_tell(&r);
      uint64_t n = (uint64_t)ipcio_read(&r, got, 10);
      if (n != 10) FAIL("reader 1 first read");
      if (ipcio_tell(&r) != t0 + 10) FAIL("reader 1 tell %lu -> %lu", (unsigned long)t0, (unsigned long)ipcio_tell(&r));
      const uint64_t back = r.bytes < 4 ? r.bytes : 4; /* back, within the current block */
      if (back) {
        char again[4];
        if (ipcio_seek(&r, -(int64_t)back, SEEK_CUR) != (int64_t)(t0 + 10 - back)) FAIL("reader 1 seek back");
        if (ipcio_read(&r, again, back) != (ssize_t)back || memcmp(again, got + 10 - back, back))
          FAIL("reader 1 re-read after seek");
      }
      if (round == 0 && t == 0) { /* forward: bytes read and dropped */
        if (ipcio_seek(&r, (int64_t)(t0 + 60), SEEK_SET) != (int64_t)(t0 + 60)) FAIL("reader 1 seek forward");
        pthread_mutex_lock(&mu);
        fill(got + 10, 0, xs[0][0] + 10, 50); /* what was dropped */
        pthread_mutex_unlock(&mu);
        n = 60;
      }
      for (;;) {
        const ssize_t k = ipcio_read(&r, got + n, 37);
        if (k < 0) {
          FAIL("reader 1 read");
          break;
        }
        n += (uint64_t)k;
        if (k < 37) break;
      }
      check("reader 1", round, t, got, n);
      if (!ipcbuf_eod(&r.buf)) FAIL("reader 1: no end of data");
      ipcbuf_reset(&r.buf);
    }
    if (round == 1) {
      pthread_barrier_wait(&bar);
      pthread_barrier_wait(&bar);
    }
  }
  free(got);
  ipcio_close(&r);
  ipcio_disconnect(&r);
  return NULL;
}

/* reader 2: depth 2 (set before the lock), two blocks held at a time */
static void *reader_blocks(void *arg) {
  (void)arg;
  ipcio_t r = IPCIO_INIT;
  if (ipcio_connect(&r, key) < 0 || ipcbuf_set_read_depth(&r.buf, 2) < 0 || ipcio_open(&r, 'R') < 0) {
    FAIL("reader 2 attach");
    return NULL;
  }
  char *got = malloc(64 * BUFSZ);
  for (int round = 0; round < NROUND; round++) {
    for (int t = 0; t < kXfers[round]; t++) {
      uint64_t n = 0;
      int held = 0, maxheld = 0;
      for (;;) {
        uint64_t sz = 0, id = 0;
        char *p = ipcio_open_block_read(&r, &sz, &id);
        if (!p) break;
        memcpy(got + n, p, sz);
        n += sz;
        if (++held > maxheld) maxheld = held;
        if (held == 2) {
          if (ipcio_close_block_read(&r, sz) < 0) FAIL("reader 2 close");
          held--;
        }
      }
      while (held-- > 0)
        if (ipcio_close_block_read(&r, 0) < 0) FAIL("reader 2 release");
      check("reader 2", round, t, got, n);
      if (maxheld != 2 && n > BUFSZ) FAIL("reader 2 never held two blocks");
      if (!ipcbuf_eod(&r.buf)) FAIL("reader 2: no end of data");
      ipcbuf_reset(&r.buf);
    }
    if (round == 1) {
      pthread_barrier_wait(&bar);
      pthread_barrier_wait(&bar);
    }
  }
  free(got);
  ipcio_close(&r);
  ipcio_disconnect(&r);
  return NULL;
}

static void *viewer(void *arg) {
  (void)arg;
  pthread_mutex_lock(&mu);
  while (!viewer_go) pthread_cond_wait(&cv, &mu);
  pthread_mutex_unlock(&mu);
  ipcio_t v = IPCIO_INIT;
  if (ipcio_connect(&v, key) < 0 || ipcio_open(&v, 'r') < 0) {
    FAIL("viewer attach");
  } else {
    int n = 0;
    for (;;) {
      uint64_t sz = 0, id = 0;
      char *p = ipcio_open_block_read(&v, &sz, &id);
      if (!p) break;
      if (sz > BUFSZ) FAIL("viewer block of %lu B", (unsigned long)sz);
      volatile char c = sz ? p[sz - 1] : 0; /* touch what it was given */
      (void)c;
      ipcio_close_block_read(&v, sz);
      n++;
      if (ipcbuf_eod(&v.buf)) break;
    }
    if (!ipcbuf_eod(&v.buf)) FAIL("viewer did not stop at the end of data");
    if (ipcio_close(&v) < 0) FAIL("viewer close");
    ipcio_disconnect(&v);
    pthread_mutex_lock(&mu);
    viewer_blocks = n;
    viewer_done = 1;
    pthread_mutex_unlock(&mu);
  }
  pthread_barrier_wait(&bar);
  pthread_barrier_wait(&bar);
  return NULL;
}

int main(int argc, char **argv) {
  key = argc > 1 ? (key_t)strtol(argv[1], NULL, 16) : 0x7f00 + (getpid() % 256) * 2;
  dada_db_destroy(key);
  if (dada_db_create(key, NBUFS, BUFSZ, 2, 4, 4096)) {
    perror("create");
    return 2;
  }
  pthread_barrier_init(&bar, NULL, 4);
  pthread_t th[4];
  pthread_create(&th[0], NULL, reader_stream, NULL);
  pthread_create(&th[1], NULL, reader_blocks, NULL);
  pthread_create(&th[2], NULL, viewer, NULL);
  pthread_create(&th[3], NULL, writer, NULL);
  for (int i = 0; i < 4; i++) pthread_join(th[i], NULL);
  pthread_barrier_destroy(&bar);
  if (!viewer_done || viewer_blocks < 2) FAIL("viewer saw %d block(s)", viewer_blocks);
  dada_db_destroy(key);
  printf("viewer blocks %d\nerrors %d\n", viewer_blocks, errors);
  return errors ? 1 : 0;
}
