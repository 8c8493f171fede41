/* pread_probe -- how fast can a page-cached file be read into memory with
 * N threads (diagnostic for paf_diskdb -T; not the product).
 *   pread_probe FILE BLOCK_BYTES [shm]
 * Reads FILE (after a 4096-B header) in BLOCK_BYTES blocks into one reused
 * buffer (malloc'd, or a SysV shared-memory segment like a DADA block),
 * each block split into N contiguous slices read in parallel, for N = 1, 2,
 * 4, 8, 16; prints one JSON line per N. */
#include <fcntl.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ipc.h>
#include <sys/shm.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

typedef struct {
  int fd;
  char *dst;
  off_t off;
  size_t len;
} job_t;

static void *rd(void *a) {
  job_t *j = a;
  size_t got = 0;
  while (got < j->len) {
    ssize_t k = pread(j->fd, j->dst + got, j->len - got, j->off + (off_t)got);
    if (k <= 0) break;
    got += (size_t)k;
  }
  return NULL;
}

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(int argc, char **argv) {
  if (argc < 3) return 2;
  int fd = open(argv[1], O_RDONLY);
  struct stat st;
  if (fd < 0 || fstat(fd, &st) < 0) return 1;
  const size_t bs = strtoull(argv[2], NULL, 10);
  const int shm = argc > 3 && !strcmp(argv[3], "shm");
  char *buf;
  if (shm) {
    int id = shmget(IPC_PRIVATE, bs, IPC_CREAT | 0600);
    buf = id >= 0 ? shmat(id, NULL, 0) : (void *)-1;
    if (id >= 0) shmctl(id, IPC_RMID, NULL);
    if (buf == (void *)-1) return 1;
  } else {
    buf = malloc(bs);
  }
  memset(buf, 1, bs);
  const uint64_t payload = (uint64_t)st.st_size - 4096, nblk = payload / bs;
  const int ns[] = {1, 2, 4, 8, 16};
  for (int r = 0; r < 2; r++)
    for (unsigned t = 0; t < sizeof ns / sizeof ns[0]; t++) {
      const int n = ns[t];
      const double t0 = now();
      for (uint64_t b = 0; b < nblk; b++) {
        pthread_t th[16];
        job_t j[16];
        const size_t per = (bs + n - 1) / n;
        for (int i = 0; i < n; i++) {
          const size_t at = (size_t)i * per, len = at < bs ? (bs - at < per ? bs - at : per) : 0;
          j[i] = (job_t){fd, buf + at, (off_t)(4096 + b * bs + at), len};
          pthread_create(&th[i], NULL, rd, &j[i]);
        }
        for (int i = 0; i < n; i++) pthread_join(th[i], NULL);
      }
      const double el = now() - t0;
      printf("{\"threads\": %d, \"rep\": %d, \"dest\": \"%s\", \"bytes\": %llu, \"s\": %.4f, \"GBps\": %.2f}\n", n, r,
             shm ? "sysv_shm" : "malloc", (unsigned long long)(nblk * bs), el, nblk * bs / el / 1e9);
      fflush(stdout);
    }
  return 0;
}
