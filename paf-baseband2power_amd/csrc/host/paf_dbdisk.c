/*
 * paf_dbdisk -- write a DADA ring to disk (the sink stage the reference runs
 * as PSRDADA's `dada_dbdisk -b cpu -k key -D dir -W`, paf-baseband2power.py
 * :94-95).  Attaches as a reader, waits for the header, writes
 * "<dir>/<UTC_START>_<OBS_OFFSET>.000000.dada" = 4096-B header + every data
 * block until end of data.
 *   -k key   -D dir   -b core (bind to that CPU core)   -W (overwrite an
 *   existing file; without it an existing file is an error, as in
 *   dada_dbdisk)   -s (single transfer: the only mode here -- the sink
 *   exits after the first end of data, where dada_dbdisk without -s waits
 *   for the next transfer)
 *   -o file  explicit output path (instead of the DADA naming rule)
 * SIGINT / SIGTERM: the block being written is finished, the file closed,
 * exit 0 (a wait for the next block gives up at once).
 */
#include <errno.h>
#include <fcntl.h>
#include <getopt.h>
#include <sched.h>
#include <signal.h>
#include <inttypes.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <unistd.h>

#include "b2p_dada.h"

static atomic_int g_stop; /* lock-free: set by the signal handler, read by every thread */
static void on_stop(int sig) {
  (void)sig;
  g_stop = 1;
  dada_interrupt_waits(); /* a reader waiting for its next block gives up */
}

/* every byte of buf to fd (a block reaches the file when it leaves the ring,
 * as in dada_dbdisk: no stdio buffer holding small spectra back) */
static int write_all(int fd, const char *buf, uint64_t n) {
  while (n) {
    const ssize_t w = write(fd, buf, n > (1u << 30) ? (1u << 30) : (size_t)n);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) return -1;
    buf += w;
    n -= (uint64_t)w;
  }
  return 0;
}

static void usage(void) {
  fprintf(stdout,
          "paf_dbdisk - write a DADA ring buffer to a file\n"
          "Usage: paf_dbdisk -k key -D dir [-o file] [-W] [-b core] [-s]\n");
}

int main(int argc, char **argv) {
  key_t key = 0xdada;
  char dir[512] = ".", ofile[1024] = "";
  int arg, overwrite = 0, core = -1;
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
      case 'b':
        if (sscanf(optarg, "%d", &core) != 1 || core < 0) {
          fprintf(stderr, "paf_dbdisk: -b takes a CPU core number, not %s\n", optarg);
          return EXIT_FAILURE;
        }
        break;
      case 'W': overwrite = 1; break;
      case 's': break; /* single transfer: always */
      default: usage(); return EXIT_FAILURE;
    }
  }
  if (ofile[0] && !overwrite && access(ofile, F_OK) == 0) { /* an explicit name: refused up front */
    fprintf(stderr, "paf_dbdisk: %s exists; -W overwrites\n", ofile);
    return EXIT_FAILURE;
  }
  {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sigemptyset(&sa.sa_mask);
    sa.sa_handler = on_stop;
    sa.sa_flags = SA_RESTART; /* a write in progress completes */
    sigaction(SIGINT, &sa, NULL);
    sigaction(SIGTERM, &sa, NULL);
  }
  multilog_t *log = multilog_open("paf_dbdisk", 0);
  multilog_add(log, stderr);
  if (core >= 0) {
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(core, &set);
    if (sched_setaffinity(0, sizeof set, &set) < 0)
      multilog(log, LOG_WARNING, "cannot bind to core %d (%s); running unbound", core, strerror(errno));
  }
  dada_hdu_t *hdu = dada_hdu_create(log);
  dada_hdu_set_key(hdu, key);
  if (dada_hdu_connect(hdu) < 0 || dada_hdu_lock_read(hdu) < 0) {
    fprintf(stderr, "paf_dbdisk: cannot attach/lock ring %x %s\n", (unsigned)key, dada_device_error());
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
  const int fd = open(ofile, O_WRONLY | O_CREAT | (overwrite ? O_TRUNC : O_EXCL), 0644);
  if (fd < 0) {
    fprintf(stderr, "paf_dbdisk: cannot open %s (%s)%s\n", ofile, strerror(errno),
            errno == EEXIST ? "; -W overwrites" : "");
    return EXIT_FAILURE;
  }
  int rc = EXIT_SUCCESS;
  if (write_all(fd, hdu->header, hdu->header_size) < 0) rc = EXIT_FAILURE;
  uint64_t total = 0, nblk = 0;
  ipcbuf_t *db = &hdu->data_block->buf;
  char *stage = NULL; /* a GPU-resident ring's blocks come back through host */
  if (ipcbuf_get_device(db) >= 0 && !(stage = malloc(ipcbuf_get_bufsz(db)))) rc = EXIT_FAILURE;
  for (; rc == EXIT_SUCCESS && !g_stop;) {
    uint64_t bytes = 0, bid = 0;
    char *b = ipcio_open_block_read(hdu->data_block, &bytes, &bid);
    if (!b) break;
    if (stage && ipcbuf_copy_out(db, stage, b, bytes) < 0) {
      multilog(log, LOG_ERR, "dbdisk: block %" PRIu64 " from the GPU: %s", nblk, dada_device_error());
      rc = EXIT_FAILURE;
    } else if (bytes && write_all(fd, stage ? stage : b, bytes) < 0) {
      multilog(log, LOG_ERR, "dbdisk: writing %s failed (%s)", ofile, strerror(errno));
      rc = EXIT_FAILURE;
    }
    ipcio_close_block_read(hdu->data_block, bytes);
    total += bytes;
    if (bytes) nblk++; /* a 0-byte block only carries the end of data */
  }
  free(stage);
  if (g_stop) multilog(log, LOG_INFO, "dbdisk: stopped by a signal after %" PRIu64 " blocks", nblk);
  if (close(fd) < 0) rc = EXIT_FAILURE;
  multilog(log, LOG_INFO, "dbdisk: %s: %" PRIu64 " B in %" PRIu64 " blocks", ofile, total, nblk);
  dada_hdu_unlock_read(hdu);
  dada_hdu_destroy(hdu);
  multilog_close(log);
  return rc;
}
