/*
 * dada_ring.c -- PSRDADA rings (ipcbuf / ipcio / dada_hdu) on SysV IPC.
 *
 * The reference links PSRDADA and uses its writer half (diskdb.cu:24-124,
 * capture.c:586-642, sync.c:101-109); the reader half its baseband2power
 * stage needed was never written.  This is a
 * fresh implementation of that library's ring protocol, as its code in the
 * reference's own binaries runs it (debug info + disassembly, recorded in
 * tests/golden/psrdada_abi.json; the addresses below are paf_diskdb's):
 * the same shared segments, keys and semaphores (dada_internal.h), and the
 * same writer / reader state machine, so a ring is shared with processes
 * linked against libpsrdada itself (dada_db, dada_dbdisk, ...).
 *
 *  writer  lock_write (WRITE lock) -> [enable_sod] -> get_next_write (waits
 *          CLEAR of every reader for a block still counted in count[]) ->
 *          mark_filled (FULL of every reader +1; a short block, or any block
 *          after enable_eod, ends the transfer: EODACK, e_buf / e_byte /
 *          eod[xfer]) -> unlock_write
 *  reader  lock_read (READ slot + the free reader slot with the lowest
 *          r_bufs) -> get_next_read (FULL -1; the first block of a transfer
 *          starts at s_buf / s_byte and acknowledges SODACK) -> mark_cleared
 *          (CLEAR +1; the end-of-data block acknowledges EODACK and stops the
 *          reader: ipcbuf_eod) -> unlock_read
 *
 * Extensions (not in PSRDADA, invisible on the wire): a reader may hold
 * several blocks (ipcbuf_set_read_depth), ring waits can be interrupted
 * from a signal handler (dada_interrupt_waits), and device rings keep their
 * blocks in a holder process (dada_device.c).
 */
#include <errno.h>
#include <inttypes.h>
#include <signal.h>
#include <stdarg.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ipc.h>
#include <sys/sem.h>
#include <sys/shm.h>
#include <time.h>
#include <unistd.h>

#include "b2p_dada.h"
#include "dada_internal.h"

/* set by dada_interrupt_waits (a signal handler, or any thread): interrupted waits fail */
static atomic_int g_interrupt; /* lock-free: set from a signal handler or another thread */

void dada_interrupt_waits(void) { g_interrupt = 1; }

/* ipc_semop (@0x4088a0) with EINTR retry until dada_interrupt_waits;
 * flags e.g. SEM_UNDO | IPC_NOWAIT */
static int sem_op(int semid, int num, int op, int flags) {
  struct sembuf sb;
  sb.sem_num = (unsigned short)num;
  sb.sem_op = (short)op;
  sb.sem_flg = (short)flags;
  for (;;) {
    if (semop(semid, &sb, 1) == 0) return 0;
    if (errno != EINTR || (g_interrupt && op < 0)) return -1;
  }
}

/* the exported one: a single semop, 0 or -1 */
int ipc_semop(int semid, short num, short op, short flag) {
  struct sembuf sb = {(unsigned short)num, op, flag};
  return semop(semid, &sb, 1) < 0 ? -1 : 0;
}

/* ipc_alloc (@0x408800): attach (creating with IPC_CREAT in flag) a segment */
void *ipc_alloc(key_t key, size_t size, int flag, int *shmid) {
  const int id = shmget(key, size, flag);
  if (id < 0) {
    fprintf(stderr, "ipc_alloc: shmget (key=%x, size=%zu, flag=%x) %s\n", (unsigned)key, size, (unsigned)flag,
            strerror(errno));
    return NULL;
  }
  void *p = shmat(id, NULL, 0);
  if (p == (void *)-1) {
    fprintf(stderr, "ipc_alloc: shmat (shmid=%d) %s\n", id, strerror(errno));
    return NULL;
  }
  if (shmid) *shmid = id;
  return p;
}

/* ------------------------------------------------------------------ */
/* multilog                                                            */

struct multilog {
  char name[128];
  int use_syslog;
  int nfp;
  FILE *fp[8];
};

multilog_t *multilog_open(const char *program_name, char use_syslog) {
  multilog_t *m = calloc(1, sizeof(*m));
  if (!m) return NULL;
  snprintf(m->name, sizeof m->name, "%s", program_name ? program_name : "");
  m->use_syslog = use_syslog;
  if (use_syslog) openlog(m->name, LOG_CONS | LOG_PID, LOG_USER);
  return m;
}

int multilog_add(multilog_t *m, FILE *fptr) {
  if (!m || !fptr || m->nfp >= 8) return -1;
  m->fp[m->nfp++] = fptr;
  return 0;
}

/* one line as multilog (@0x402ad0) writes it: "[%Y-%m-%d-%H:%M:%S] ", "ERR: "
 * for LOG_ERR or "WARN: " for LOG_WARNING, the message.  Departure: a
 * message without a trailing newline gets one */
static int log_line(FILE *fp, int priority, const char *msg) {
  char ts[64];
  time_t now = time(NULL);
  struct tm tmv;
  strftime(ts, sizeof ts, "%Y-%m-%d-%H:%M:%S", localtime_r(&now, &tmv));
  const char *tag = priority == LOG_ERR ? "ERR: " : priority == LOG_WARNING ? "WARN: " : "";
  const int rc = fprintf(fp, "[%s] %s%s%s", ts, tag, msg, (msg[0] && msg[strlen(msg) - 1] == '\n') ? "" : "\n");
  fflush(fp);
  return rc < 0 ? -1 : 0;
}

int multilog(multilog_t *m, int priority, const char *format, ...) {
  if (!m) return -1;
  char msg[1024];
  va_list ap;
  va_start(ap, format);
  vsnprintf(msg, sizeof msg, format, ap);
  va_end(ap);
  for (int i = 0; i < m->nfp; i++) log_line(m->fp[i], priority, msg);
  if (m->use_syslog) syslog(priority, "%s", msg);
  return 0;
}

/* multilog_fprintf (@0x402dd0): the same line to one stream */
int multilog_fprintf(FILE *stream, int priority, const char *format, ...) {
  if (!stream) return -1;
  char msg[1024];
  va_list ap;
  va_start(ap, format);
  vsnprintf(msg, sizeof msg, format, ap);
  va_end(ap);
  if (log_line(stream, priority, msg) < 0) perror("multilog: error vfprintf");
  return 0;
}

int multilog_close(multilog_t *m) {
  if (!m) return -1;
  for (int i = 0; i < m->nfp; i++) fflush(m->fp[i]);
  if (m->use_syslog) closelog();
  free(m);
  return 0;
}

/* ------------------------------------------------------------------ */
/* ipcbuf: segments                                                     */

/* shmkey[] follows count[] at 520 + nbufs: possibly unaligned, so it is
 * read and written by value */
static key_t shmkey_get(const ipcbuf_t *id, uint64_t i) {
  key_t k;
  memcpy(&k, (const char *)id->shmkey + i * sizeof(key_t), sizeof k);
  return k;
}

static void shmkey_set(ipcbuf_t *id, uint64_t i, key_t k) {
  memcpy((char *)id->shmkey + i * sizeof(key_t), &k, sizeof k);
}

/* ipcsync_get (@0x402fe0): the sync segment, count[] and shmkey[] after it */
static int sync_get(ipcbuf_t *id, key_t key, uint64_t nbufs, int flag) {
  id->syncid = shmget(key, nbufs ? sync_size(nbufs) : sizeof(ipcsync_t), flag);
  if (id->syncid < 0) return -1;
  void *p = shmat(id->syncid, NULL, 0);
  if (p == (void *)-1) {
    id->syncid = -1;
    return -1;
  }
  id->sync = p;
  if (!nbufs) nbufs = id->sync->nbufs;
  id->count = (char *)(id->sync + 1);
  id->shmkey = (key_t *)(id->count + nbufs);
  id->state = ST_DISCON;
  id->viewbuf = 0;
  return 0;
}

static size_t seg_size(int shmid) {
  struct shmid_ds ds;
  return shmctl(shmid, IPC_STAT, &ds) == 0 ? ds.shm_segsz : 0;
}

/* ipcbuf_get (@0x403090): the semaphore sets and the blocks; kc is the
 * connect set's key (semkey_connect, published last by a creator) */
static int ring_get(ipcbuf_t *id, key_t kc, int flag) {
  ipcsync_t *s = id->sync;
  const uint64_t n = s->nbufs;
  id->semid_connect = semget(kc, NSEM_CONNECT, flag);
  if (id->semid_connect < 0) return -1;
  id->semid_data = malloc((s->n_readers ? s->n_readers : 1) * sizeof(int));
  id->buffer = calloc(n, sizeof(char *));
  id->shm_addr = calloc(n, sizeof(void *));
  id->shmid = malloc(n * sizeof(int));
  if (!id->semid_data || !id->buffer || !id->shm_addr || !id->shmid) return -1;
  for (unsigned r = 0; r < s->n_readers; r++) id->semid_data[r] = -1;
  for (unsigned r = 0; r < s->n_readers; r++) {
    id->semid_data[r] = semget(s->semkey_data[r], NSEM_DATA, flag);
    if (id->semid_data[r] < 0) return -1;
  }
  for (uint64_t i = 0; i < n; i++) id->shmid[i] = -1;
  for (uint64_t i = 0; i < n; i++) {
    const int dev = s->on_device_id >= 0;
    /* a device ring's segment holds the handle (block 0: and the holder) */
    const size_t sz = !dev ? s->bufsz : (flag & IPC_CREAT) ? (i ? DEV_HANDLE_BYTES : sizeof(dev_seg_t)) : 0;
    id->shmid[i] = shmget(shmkey_get(id, i), sz, flag);
    if (id->shmid[i] < 0) return -1;
    if (dev && i == 0 && !(flag & IPC_CREAT) && seg_size(id->shmid[0]) < sizeof(dev_seg_t)) {
      errno = ENODEV; /* a device ring without a libpafdada holder (e.g. PSRDADA's CUDA one) */
      return -1;
    }
    void *p = shmat(id->shmid[i], NULL, 0);
    if (p == (void *)-1) return -1;
    id->shm_addr[i] = p;
    if (!dev) id->buffer[i] = p;
  }
  return 0;
}

/* the exported ipcbuf_get, on an attached sync segment; n_readers is not
 * used (nor is it by the binary's) */
int ipcbuf_get(ipcbuf_t *id, int flag, int n_readers) {
  (void)n_readers;
  if (!id || !id->sync) return -1;
  return ring_get(id, id->sync->semkey_connect, flag);
}

static void free_local(ipcbuf_t *id) {
  if (id->shm_addr && id->sync) {
    if (id->sync->on_device_id >= 0 && id->buffer) dev_close_blocks(id);
    for (uint64_t i = 0; i < id->sync->nbufs; i++)
      if (id->shm_addr[i]) shmdt(id->shm_addr[i]);
  }
  free(id->buffer);
  free(id->shm_addr);
  free(id->shmid);
  free(id->semid_data);
  id->buffer = NULL;
  id->shm_addr = NULL;
  id->shmid = NULL;
  id->semid_data = NULL;
}

/* remove every segment and semaphore set a (possibly half-built) ring has */
static void remove_ipc(ipcbuf_t *id) {
  ipcsync_t *s = id->sync;
  if (s->on_device_id >= 0 && id->shm_addr && id->shm_addr[0]) {
    /* this process's own handles first, then its attachment to block 0's
     * segment, which the holder would count as an importer (the ordering
     * rule, dada_internal.h) */
    if (id->buffer) dev_close_blocks(id);
    shmdt(id->shm_addr[0]);
    id->shm_addr[0] = NULL;
    if (id->shmid) dev_stop_holder(id->shmid[0]);
  }
  for (uint64_t i = 0; id->shmid && i < s->nbufs; i++)
    if (id->shmid[i] >= 0) shmctl(id->shmid[i], IPC_RMID, NULL);
  for (unsigned r = 0; id->semid_data && r < s->n_readers; r++)
    if (id->semid_data[r] >= 0) semctl(id->semid_data[r], 0, IPC_RMID);
  if (id->semid_connect >= 0) semctl(id->semid_connect, 0, IPC_RMID);
}

static int ring_create(ipcbuf_t *id, key_t key, uint64_t nbufs, uint64_t bufsz, unsigned n_readers,
                       int device, int open_device) {
  const ipcbuf_t init = IPCBUF_INIT;
  *id = init;
  if (!nbufs || !bufsz || n_readers > IPCBUF_READERS || nbufs > 0x7fff) {
    errno = EINVAL;
    return -1;
  }
  if (sync_get(id, key, nbufs, IPC_CREAT | IPC_EXCL | 0666) < 0) return -1;
  ipcsync_t *s = id->sync;
  memset(s, 0, sync_size(nbufs));
  s->nbufs = nbufs;
  s->bufsz = bufsz;
  s->n_readers = n_readers;
  s->on_device_id = device;
  for (int x = 0; x < IPCBUF_XFERS; x++) s->eod[x] = 1; /* @0x403434 */
  for (int r = 0; r < IPCBUF_READERS; r++) s->semkey_data[r] = key_data(key, r);
  for (uint64_t i = 0; i < nbufs; i++) shmkey_set(id, i, key_block(key, i));
  /* semkey_connect is published last (below): a connector that finds the
   * segment before the ring is complete sees 0 there and backs off */
  const key_t kc = key_connect(key);
  int ok = ring_get(id, kc, IPC_CREAT | IPC_EXCL | 0666) == 0;
  /* @0x403528-0x4035b1: WRITE 1, READ n_readers; per reader SODACK 8,
   * EODACK 8, READER_CONN 1 */
  if (ok) ok = sem_op(id->semid_connect, SEM_WRITE, 1, 0) == 0;
  if (ok && n_readers) ok = sem_op(id->semid_connect, SEM_READ, (int)n_readers, 0) == 0;
  for (unsigned r = 0; ok && r < n_readers; r++)
    ok = sem_op(id->semid_data[r], SEM_SODACK, IPCBUF_XFERS, 0) == 0 &&
         sem_op(id->semid_data[r], SEM_EODACK, IPCBUF_XFERS, 0) == 0 &&
         sem_op(id->semid_data[r], SEM_READER_CONN, 1, 0) == 0;
  if (ok && device >= 0) ok = dev_create_blocks(id, device) == 0 && (!open_device || dev_open_blocks(id) == 0);
  if (!ok) {
    const int e = errno;
    remove_ipc(id);
    free_local(id);
    shmdt(s);
    shmctl(id->syncid, IPC_RMID, NULL);
    *id = init;
    errno = e;
    return -1;
  }
  __atomic_store_n(&s->semkey_connect, kc, __ATOMIC_RELEASE);
  id->state = ST_VIEWER;
  return 0;
}

int ipcbuf_create(ipcbuf_t *id, key_t key, uint64_t nbufs, uint64_t bufsz, unsigned n_readers) {
  return ipcbuf_create_work(id, key, nbufs, bufsz, n_readers, -1);
}

int ipcbuf_create_work(ipcbuf_t *id, key_t key, uint64_t nbufs, uint64_t bufsz, unsigned n_readers,
                       int device_id) {
  if (!id) return -1;
  return ring_create(id, key, nbufs, bufsz, n_readers, device_id < 0 ? -1 : device_id, 1);
}

int ipcbuf_connect(ipcbuf_t *id, key_t key) {
  if (!id) return -1;
  const ipcbuf_t init = IPCBUF_INIT;
  *id = init;
  if (sync_get(id, key, 0, 0666) < 0) return -1;
  if (__atomic_load_n(&id->sync->semkey_connect, __ATOMIC_ACQUIRE) == 0) { /* still being built */
    ipcbuf_disconnect(id);
    errno = EAGAIN;
    return -1;
  }
  if (ring_get(id, id->sync->semkey_connect, 0666) < 0 ||
      (id->sync->on_device_id >= 0 && dev_open_blocks(id) < 0)) {
    const int e = errno;
    ipcbuf_disconnect(id);
    errno = e;
    return -1;
  }
  id->state = ST_VIEWER;
  return 0;
}

/* ipcbuf_disconnect (@0x403780): detach; a lock still held stays with the
 * process until it exits (SEM_UNDO) */
int ipcbuf_disconnect(ipcbuf_t *id) {
  if (!id) return -1;
  free_local(id);
  if (id->sync) shmdt(id->sync);
  id->sync = NULL;
  id->count = NULL;
  id->shmkey = NULL;
  id->state = ST_DISCON;
  id->iread = -1;
  return 0;
}

int ipcbuf_destroy(ipcbuf_t *id) {
  if (!id || !id->sync) return -1;
  const int syncid = id->syncid;
  remove_ipc(id);
  ipcbuf_disconnect(id);
  shmctl(syncid, IPC_RMID, NULL);
  id->syncid = -1;
  id->semid_connect = -1;
  return 0;
}

/* ------------------------------------------------------------------ */
/* ipcbuf: writer                                                       */

char ipcbuf_is_writer(ipcbuf_t *id) { return id && id->state >= ST_WRITER && id->state <= ST_WCHANGE; }
char ipcbuf_is_writing(ipcbuf_t *id) { return id && id->state == ST_WRITING; }
char ipcbuf_is_reader(ipcbuf_t *id) { return id && id->state >= ST_READER && id->state <= ST_RSTOP; }

int ipcbuf_lock_write(ipcbuf_t *id) {  /* @0x403b00 */
  if (!id || id->state != ST_VIEWER) return -1;
  if (sem_op(id->semid_connect, SEM_WRITE, -1, SEM_UNDO) < 0) return -1;
  id->state = id->sync->w_state ? ST_WRITING : ST_WCHANGE;
  id->xfer = id->sync->w_xfer % IPCBUF_XFERS;
  return 0;
}

int ipcbuf_unlock_write(ipcbuf_t *id) {  /* @0x403b90 */
  if (!ipcbuf_is_writer(id)) return -1;
  if (sem_op(id->semid_connect, SEM_WRITE, 1, SEM_UNDO) < 0) return -1;
  id->state = ST_VIEWER;
  return 0;
}

/* the earliest block a start of data may name: the last transfer's end
 * (soclock_buf) while it is still in the ring, else the oldest block left */
uint64_t ipcbuf_get_sod_minbuf(ipcbuf_t *id) {  /* @0x403ca0 */
  const ipcsync_t *s = id->sync;
  return s->w_buf - id->soclock_buf < s->nbufs ? id->soclock_buf : s->w_buf + 1 - s->nbufs;
}

int ipcbuf_enable_sod(ipcbuf_t *id, uint64_t start_buf, uint64_t start_byte) {  /* @0x403cd0 */
  if (!id || !(id->state == ST_WRITER || id->state == ST_WCHANGE)) return -1;
  ipcsync_t *s = id->sync;
  if (start_buf > s->w_buf || start_buf < ipcbuf_get_sod_minbuf(id) || start_byte > s->bufsz) return -1;
  for (unsigned r = 0; r < s->n_readers; r++) /* every reader has acknowledged a start slot */
    if (sem_op(id->semid_data[r], SEM_SODACK, -1, 0) < 0) return -1;
  const uint64_t x = s->w_xfer % IPCBUF_XFERS;
  id->xfer = x;
  s->s_buf[x] = start_buf;
  s->s_byte[x] = start_byte;
  if (s->w_buf == 0)
    s->eod[x] = 0;
  else
    for (uint64_t b = start_buf; b < s->w_buf; b++) id->count[b % s->nbufs]++;
  const uint64_t new_bufs = s->w_buf - start_buf;
  id->state = ST_WRITING;
  s->w_state = ST_WRITING;
  for (unsigned r = 0; new_bufs && r < s->n_readers; r++)
    if (sem_op(id->semid_data[r], SEM_FULL, (int)(short)new_bufs, 0) < 0) return -1;
  return 0;
}

int ipcbuf_disable_sod(ipcbuf_t *id) {  /* @0x403c60 */
  if (!id || id->state != ST_WCHANGE) return -1;
  id->state = ST_WRITER;
  return 0;
}

int ipcbuf_enable_eod(ipcbuf_t *id) {  /* @0x403c20 */
  if (!id || id->state != ST_WRITING) return -1;
  id->state = ST_WCHANGE;
  return 0;
}

char *ipcbuf_get_next_write(ipcbuf_t *id) {  /* @0x403f20 */
  if (!ipcbuf_is_writer(id)) return NULL;
  ipcsync_t *s = id->sync;
  if (id->state == ST_WCHANGE && ipcbuf_enable_sod(id, s->w_buf, 0) < 0) return NULL;
  const uint64_t b = s->w_buf % s->nbufs;
  while (id->count[b]) { /* every reader has cleared the block's last fill */
    for (unsigned r = 0; r < s->n_readers; r++)
      if (sem_op(id->semid_data[r], SEM_CLEAR, -1, 0) < 0) return NULL;
    id->count[b]--;
  }
  return id->buffer[b];
}

/* ipcbuf_zero_next_write (@0x404060): zero the block after the one being
 * written, once it is free, polling every 10 ms.  Departure: "free" is
 * decided from count[] and every reader's CLEAR (the fills still pending in
 * this block and the current one all cleared); libpsrdada only waits for
 * every CLEAR to be non-zero, which never happens on a fresh ring and does
 * not say which block was cleared */
int ipcbuf_zero_next_write(ipcbuf_t *id) {
  if (!ipcbuf_is_writer(id)) {
    fprintf(stderr, "ipcbuf_get_next_write: process is not writer\n");
    return -1;
  }
  ipcsync_t *s = id->sync;
  const uint64_t cur = s->w_buf % s->nbufs, next = (s->w_buf + 1) % s->nbufs;
  for (;;) {
    const int need = id->count[next] ? id->count[next] + (next != cur ? id->count[cur] : 0) : 0;
    int ok = 1;
    for (unsigned r = 0; ok && r < s->n_readers && need; r++) {
      const int v = semctl(id->semid_data[r], SEM_CLEAR, GETVAL);
      if (v < 0) return -1;
      ok = v >= need;
    }
    if (ok) break;
    if (g_interrupt) return -1;
    nanosleep(&(struct timespec){0, 10000000}, NULL);
  }
  if (s->on_device_id >= 0) return dev_zero(id->buffer[next], s->bufsz);
  memset(id->buffer[next], 0, s->bufsz);
  return 0;
}

int ipcbuf_mark_filled(ipcbuf_t *id, uint64_t nbytes) {  /* @0x404170 */
  if (!ipcbuf_is_writer(id)) return -1;
  ipcsync_t *s = id->sync;
  if (nbytes > s->bufsz) return -1;
  if (id->state == ST_WRITER) { /* start of data disabled: invisible to readers */
    s->w_buf++;
    return 0;
  }
  if (id->state == ST_WCHANGE || nbytes < s->bufsz) { /* this block ends the transfer */
    for (unsigned r = 0; r < s->n_readers; r++)
      if (sem_op(id->semid_data[r], SEM_EODACK, -1, 0) < 0) return -1;
    s->e_buf[id->xfer] = s->w_buf;
    s->e_byte[id->xfer] = nbytes;
    s->eod[id->xfer] = 1;
    s->w_xfer++;
    id->xfer = s->w_xfer % IPCBUF_XFERS;
    id->state = ST_WRITER;
    s->w_state = 0;
  }
  id->count[s->w_buf % s->nbufs]++;
  s->w_buf++;
  for (unsigned r = 0; r < s->n_readers; r++)
    if (sem_op(id->semid_data[r], SEM_FULL, 1, 0) < 0) return -1;
  return 0;
}

/* ------------------------------------------------------------------ */
/* ipcbuf: reader                                                       */

/* read depth (extension), kept in viewbuf, which PSRDADA leaves unused for
 * a reader: bits 56-63 hold this process's read depth, set only through
 * ipcbuf_set_read_depth and kept by every other call; the low bits hold a
 * reader's blocks held (8-15) and end-of-data block held (16), or a
 * viewer's block position (0-55, view_next).  So a handle that views and
 * then reads keeps the depth it was given, never its old view position. */
#define VB_DEPTH_SHIFT 56
#define VB_LOW_MASK ((UINT64_C(1) << VB_DEPTH_SHIFT) - 1)
static int rd_depth(const ipcbuf_t *id) {
  const int d = (int)(id->viewbuf >> VB_DEPTH_SHIFT);
  return d ? d : 1;
}
static int rd_open(const ipcbuf_t *id) { return (int)((id->viewbuf >> 8) & 0xff); }
static int rd_eod_held(const ipcbuf_t *id) { return (int)((id->viewbuf >> 16) & 1); }
static void rd_set(ipcbuf_t *id, int open, int eod_held) {
  id->viewbuf = (id->viewbuf & ~VB_LOW_MASK) | ((uint64_t)open << 8) | ((uint64_t)(eod_held != 0) << 16);
}
/* a viewer's block position */
static uint64_t vw_pos(const ipcbuf_t *id) { return id->viewbuf & VB_LOW_MASK; }
static void vw_set(ipcbuf_t *id, uint64_t pos) { id->viewbuf = (id->viewbuf & ~VB_LOW_MASK) | (pos & VB_LOW_MASK); }

/* before or after ipcbuf_lock_read: lock_read / unlock_read keep the depth */
int ipcbuf_set_read_depth(ipcbuf_t *id, int depth) {
  if (!id || !id->sync || depth < 1 || depth > 255 || (uint64_t)depth > id->sync->nbufs) return -1;
  id->viewbuf = (id->viewbuf & VB_LOW_MASK) | ((uint64_t)depth << VB_DEPTH_SHIFT);
  return 0;
}

uint64_t ipcbuf_view_position(const ipcbuf_t *id) { return id ? vw_pos(id) : 0; }

int ipcbuf_lock_read(ipcbuf_t *id) {  /* @0x404360 */
  if (!id || id->state != ST_VIEWER || id->iread != -1) return -1;
  if (sem_op(id->semid_connect, SEM_READ, -1, SEM_UNDO) < 0) return -1;
  ipcsync_t *s = id->sync;
  const unsigned n = s->n_readers;
  int order[IPCBUF_READERS], used[IPCBUF_READERS] = {0};
  for (unsigned k = 0; k < n; k++) { /* reader slots by r_bufs, lowest first */
    uint64_t best = UINT64_MAX;
    order[k] = -1;
    for (unsigned i = 0; i < n; i++)
      if (!used[i] && (order[k] < 0 || s->r_bufs[i] < best)) best = s->r_bufs[i], order[k] = (int)i;
    used[order[k]] = 1;
  }
  for (unsigned k = 0; k < n && id->iread < 0; k++) {
    if (sem_op(id->semid_data[order[k]], SEM_READER_CONN, -1, IPC_NOWAIT | SEM_UNDO) == 0)
      id->iread = order[k];
    else if (errno != EAGAIN)
      break;
  }
  if (id->iread < 0) {
    sem_op(id->semid_connect, SEM_READ, 1, SEM_UNDO);
    return -1;
  }
  id->state = s->r_states[id->iread] ? ST_READING : ST_READER;
  id->xfer = s->r_xfers[id->iread] % IPCBUF_XFERS;
  id->viewbuf &= ~VB_LOW_MASK; /* a read depth set before the lock stays (blocks held: none) */
  return 0;
}

int ipcbuf_unlock_read(ipcbuf_t *id) {  /* @0x4045f0 */
  if (!ipcbuf_is_reader(id) || id->iread < 0 || (unsigned)id->iread >= id->sync->n_readers) return -1;
  if (sem_op(id->semid_data[id->iread], SEM_READER_CONN, 1, SEM_UNDO) < 0) return -1;
  if (sem_op(id->semid_connect, SEM_READ, 1, SEM_UNDO) < 0) return -1;
  id->state = ST_VIEWER;
  id->iread = -1;
  id->viewbuf &= ~VB_LOW_MASK; /* the read depth stays for the next lock_read */
  return 0;
}

int ipcbuf_eod(ipcbuf_t *id) { return id && (id->state == ST_RSTOP || id->state == ST_VSTOP); }
int ipcbuf_sod(ipcbuf_t *id) { return id && (id->state == ST_READING || id->state == ST_WRITING); }

/* A viewer (ipcio_open 'r': no lock, takes nothing) follows the writer:
 * its first block is the newest one written (or its transfer's start), then
 * each next one as it is written, polled every 0.1 s, skipping ahead when
 * the writer laps it; it stops (VSTOP, ipcbuf_eod) once reader 0 is at the
 * transfer's end-of-data block.  Departures: the view that stops returns a
 * 0-byte block (libpsrdada returns the unwritten block at the view
 * position), and a block's size is that block's own (libpsrdada sizes it by
 * reader 0's position). */
static char *view_next(ipcbuf_t *id, uint64_t *bytes) {
  ipcsync_t *s = id->sync;
  uint64_t start = 0;
  if (id->state == ST_VIEWER) {
    id->xfer = s->r_xfers[0] % IPCBUF_XFERS;
    id->state = ST_VIEWING;
    vw_set(id, s->s_buf[id->xfer]);
    if (s->w_buf > vw_pos(id) + 1)
      vw_set(id, s->w_buf - 1);
    else
      start = s->s_byte[id->xfer];
  }
  while (s->w_buf <= vw_pos(id)) {
    if (s->eod[id->xfer] && s->r_bufs[0] && s->r_bufs[0] == s->e_buf[id->xfer]) {
      id->state = ST_VSTOP;
      if (bytes) *bytes = 0;
      return id->buffer[vw_pos(id) % s->nbufs];
    }
    if (g_interrupt) return NULL;
    nanosleep(&(struct timespec){0, 100000000}, NULL);
  }
  if (vw_pos(id) + s->nbufs < s->w_buf) vw_set(id, s->w_buf - s->nbufs + 1);
  const uint64_t b = vw_pos(id);
  vw_set(id, b + 1);
  const int last = s->eod[id->xfer] && s->e_buf[id->xfer] == b;
  if (bytes) *bytes = (last ? s->e_byte[id->xfer] : s->bufsz) - start;
  return id->buffer[b % s->nbufs] + start;
}

/* ipcbuf_get_next_read_work (@0x404710); flag goes to the reader's FULL and
 * SODACK semops */
char *ipcbuf_get_next_read_work(ipcbuf_t *id, uint64_t *bytes, int flag) {
  if (!id || !id->sync || ipcbuf_eod(id)) return NULL;
  if (id->state == ST_VIEWER || id->state == ST_VIEWING) return view_next(id, bytes);
  if (!ipcbuf_is_reader(id)) return NULL;
  ipcsync_t *s = id->sync;
  const int r = id->iread, open = rd_open(id);
  if (open >= rd_depth(id) || (open && rd_eod_held(id))) return NULL;
  if (sem_op(id->semid_data[r], SEM_FULL, -1, flag) < 0) return NULL;
  uint64_t start = 0;
  if (id->state == ST_READER) { /* first block of a transfer */
    id->xfer = s->r_xfers[r] % IPCBUF_XFERS;
    id->state = ST_READING;
    s->r_states[r] = ST_READING;
    s->r_bufs[r] = s->s_buf[id->xfer];
    start = s->s_byte[id->xfer];
    if (sem_op(id->semid_data[r], SEM_SODACK, 1, flag) < 0) return NULL;
  }
  const uint64_t b = s->r_bufs[r] + (uint64_t)open;
  const int last = s->eod[id->xfer] && s->e_buf[id->xfer] == b;
  if (bytes) *bytes = (last ? s->e_byte[id->xfer] : s->bufsz) - start;
  rd_set(id, open + 1, last);
  return id->buffer[b % s->nbufs] + start;
}

char *ipcbuf_get_next_read(ipcbuf_t *id, uint64_t *bytes) { return ipcbuf_get_next_read_work(id, bytes, 0); }

/* @0x4049d0: the binary passes 0x1000 (SEM_UNDO), so it waits as
 * ipcbuf_get_next_read does */
char *ipcbuf_get_next_readable(ipcbuf_t *id, uint64_t *bytes) {
  return ipcbuf_get_next_read_work(id, bytes, SEM_UNDO);
}

int ipcbuf_mark_cleared(ipcbuf_t *id) {  /* @0x404b80: the oldest block held */
  if (!id || id->state != ST_READING) return -1;
  ipcsync_t *s = id->sync;
  const int r = id->iread, open = rd_open(id);
  if (sem_op(id->semid_data[r], SEM_CLEAR, 1, 0) < 0) return -1;
  if (s->eod[id->xfer] && s->r_bufs[r] == s->e_buf[id->xfer]) { /* end of this transfer */
    id->state = ST_RSTOP;
    s->r_states[r] = 0;
    s->r_xfers[r]++;
    id->xfer = s->r_xfers[r] % IPCBUF_XFERS;
    rd_set(id, 0, 0);
    return sem_op(id->semid_data[r], SEM_EODACK, 1, 0);
  }
  s->r_bufs[r]++;
  rd_set(id, open ? open - 1 : 0, rd_eod_held(id));
  return 0;
}

/* Every transfer slot as ring_create leaves it: end of data set, no start
 * or end block recorded.  A reset that kept the old e_buf[x] / e_byte[x]
 * would leave transfer x >= 1 of the next sequence (whose eod[x] is already
 * set, enable_sod clears it only for a transfer starting at block 0) ending
 * early at a stale block number.  Departure: the resets of the libpsrdada
 * the reference links rewrite eod[] only (tests/golden/psrdada_abi.json,
 * "resets"), so there a second transfer after a reset that spans an old
 * e_buf ends there; here the slots go back to their created state. */
static void clear_xfers(ipcsync_t *s) {
  for (int x = 0; x < IPCBUF_XFERS; x++) {
    s->eod[x] = 1;
    s->s_buf[x] = s->s_byte[x] = 0;
    s->e_buf[x] = s->e_byte[x] = 0;
  }
}

/* ipcbuf_reset (@0x404ca0).  A reader at end of data gets ready for the
 * next transfer.  A writer takes the ring back to its created state once
 * every reader has cleared every block and acknowledged every transfer
 * (CLEARs for count[], SODACK and EODACK down by 8 and back up); a ring
 * never written to is left as it is. */
int ipcbuf_reset(ipcbuf_t *id) {
  if (!id) return -1;
  if (id->state == ST_RSTOP) {
    id->state = ST_READER;
    return 0;
  }
  if (!ipcbuf_is_writer(id)) return -1;
  ipcsync_t *s = id->sync;
  if (!s->w_buf) return 0;
  for (uint64_t b = 0; b < s->nbufs; b++)
    for (; id->count[b]; id->count[b]--)
      for (unsigned r = 0; r < s->n_readers; r++)
        if (sem_op(id->semid_data[r], SEM_CLEAR, -1, 0) < 0) return -1;
  for (unsigned r = 0; r < s->n_readers; r++) {
    if (sem_op(id->semid_data[r], SEM_SODACK, -IPCBUF_XFERS, 0) < 0 ||
        sem_op(id->semid_data[r], SEM_EODACK, -IPCBUF_XFERS, 0) < 0 ||
        sem_op(id->semid_data[r], SEM_SODACK, IPCBUF_XFERS, 0) < 0 ||
        sem_op(id->semid_data[r], SEM_EODACK, IPCBUF_XFERS, 0) < 0)
      return -1;
    s->r_bufs[r] = 0;
    s->r_xfers[r] = 0;
  }
  s->w_buf = 0;
  s->w_xfer = 0;
  clear_xfers(s);
  return 0;
}

/* ipcbuf_hard_reset (@0x404f70): the same end state without waiting for
 * anyone -- FULL and CLEAR of every reader set to 0.  Departure: count[] is
 * zeroed too (libpsrdada leaves it, and the next writer then waits for
 * CLEARs that were just discarded) */
int ipcbuf_hard_reset(ipcbuf_t *id) {
  if (!id || !id->sync) return -1;
  ipcsync_t *s = id->sync;
  s->w_buf = 0;
  s->w_xfer = 0;
  clear_xfers(s);
  memset(id->count, 0, s->nbufs);
  for (unsigned r = 0; r < s->n_readers; r++) {
    s->r_bufs[r] = 0;
    s->r_xfers[r] = 0;
    if (semctl(id->semid_data[r], SEM_FULL, SETVAL, 0) < 0 || semctl(id->semid_data[r], SEM_CLEAR, SETVAL, 0) < 0) {
      perror("ipcbuf_hard_reset: semctl (IPCBUF_FULL, SETVAL)");
      return -1;
    }
  }
  return 0;
}

/* ------------------------------------------------------------------ */
/* ipcbuf: queries                                                      */

uint64_t ipcbuf_get_bufsz(ipcbuf_t *id) { return id && id->sync ? id->sync->bufsz : 0; }
uint64_t ipcbuf_get_nbufs(ipcbuf_t *id) { return id && id->sync ? id->sync->nbufs : 0; }
int ipcbuf_get_nreaders(ipcbuf_t *id) { return id && id->sync ? (int)id->sync->n_readers : 0; }
uint64_t ipcbuf_get_write_count(ipcbuf_t *id) { return id && id->sync ? id->sync->w_buf : 0; }
uint64_t ipcbuf_get_write_index(ipcbuf_t *id) {
  return id && id->sync ? id->sync->w_buf % id->sync->nbufs : 0;
}
uint64_t ipcbuf_get_read_count(ipcbuf_t *id) {
  return id && id->sync ? id->sync->r_bufs[id->iread < 0 ? 0 : id->iread] : 0;
}
uint64_t ipcbuf_get_read_count_iread(ipcbuf_t *id, unsigned iread) {
  return id && id->sync && iread < IPCBUF_READERS ? id->sync->r_bufs[iread] : 0;
}
uint64_t ipcbuf_get_read_index(ipcbuf_t *id) {
  return id && id->sync ? ipcbuf_get_read_count(id) % id->sync->nbufs : 0;
}
char *ipcbuf_get_buffer(ipcbuf_t *id, uint64_t i) {
  return id && id->buffer && id->sync && i < id->sync->nbufs ? id->buffer[i] : NULL;
}
int ipcbuf_get_device(ipcbuf_t *id) { return id && id->sync ? id->sync->on_device_id : -1; }

int ipcbuf_copy_in(ipcbuf_t *id, char *block, const void *src, uint64_t n) {
  if (!id || !id->sync || (!block && n) || (!src && n)) return -1;
  if (id->sync->on_device_id >= 0) return dev_copy(block, src, n, 1);
  memcpy(block, src, n);
  return 0;
}

int ipcbuf_copy_out(ipcbuf_t *id, void *dst, const char *block, uint64_t n) {
  if (!id || !id->sync || (!block && n) || (!dst && n)) return -1;
  if (id->sync->on_device_id >= 0) return dev_copy(dst, block, n, 0);
  memcpy(dst, block, n);
  return 0;
}

/* ipcbuf_lock / _unlock (@0x405050 / @0x405100): pin the sync segment and
 * every host block in RAM (shmctl SHM_LOCK), as dada_db -l does */
static int lock_segments(ipcbuf_t *id, int cmd) {
  if (!id || !id->sync || id->syncid < 0 || !id->shmid) return -1;
  if (shmctl(id->syncid, cmd, NULL) < 0) return -1;
  for (uint64_t i = 0; id->sync->on_device_id < 0 && i < id->sync->nbufs; i++)
    if (shmctl(id->shmid[i], cmd, NULL) < 0) return -1;
  return 0;
}

int ipcbuf_lock(ipcbuf_t *id) { return lock_segments(id, SHM_LOCK); }
int ipcbuf_unlock(ipcbuf_t *id) { return lock_segments(id, SHM_UNLOCK); }

/* ipcbuf_page (@0x4051b0): touch (zero) every block so its pages exist */
int ipcbuf_page(ipcbuf_t *id) {
  if (!id || !id->sync || !id->buffer) return -1;
  if (id->sync->on_device_id >= 0) return 0; /* device blocks are zeroed by their holder */
  for (uint64_t i = 0; i < id->sync->nbufs; i++) memset(id->buffer[i], 0, id->sync->bufsz);
  return 0;
}

/* ------------------------------------------------------------------ */
/* ipcio                                                                */

void ipcio_init(ipcio_t *ipc) {  /* @0x4057f0 */
  ipc->bytes = 0;
  ipc->rdwrt = 0;
  ipc->curbuf = NULL;
  ipc->marked_filled = 0;
  ipc->sod_pending = 0;
  ipc->sod_buf = 0;
  ipc->sod_byte = 0;
}

int ipcio_connect(ipcio_t *ipc, key_t key) {
  if (!ipc || ipcbuf_connect(&ipc->buf, key) < 0) return -1;
  ipcio_init(ipc);
  return 0;
}

int ipcio_disconnect(ipcio_t *ipc) {
  if (!ipc || ipcbuf_disconnect(&ipc->buf) < 0) return -1;
  ipcio_init(ipc);
  return 0;
}

int ipcio_create_work(ipcio_t *ipc, key_t key, uint64_t nbufs, uint64_t bufsz, unsigned num_read,
                      int device_id) {  /* @0x405830 */
  if (!ipc || ipcbuf_create_work(&ipc->buf, key, nbufs, bufsz, num_read, device_id) < 0) {
    fprintf(stderr, "ipcio_create: ipcbuf_create error\n");
    return -1;
  }
  ipcio_init(ipc);
  return 0;
}

int ipcio_create(ipcio_t *ipc, key_t key, uint64_t nbufs, uint64_t bufsz, unsigned num_read) {
  return ipcio_create_work(ipc, key, nbufs, bufsz, num_read, -1);
}

int ipcio_destroy(ipcio_t *ipc) {  /* @0x405990 */
  if (!ipc) return -1;
  ipcio_init(ipc);
  return ipcbuf_destroy(&ipc->buf);
}

/* 'W' writer, 'w' writer with the start of data deferred (ipcio_start),
 * 'R' reader, 'r' viewer (no lock: follows the writer, takes nothing) */
int ipcio_open(ipcio_t *ipc, char rdwrt) {  /* @0x4059d0 */
  if (!ipc) return -1;
  if (rdwrt != 'W' && rdwrt != 'w' && rdwrt != 'R' && rdwrt != 'r') {
    fprintf(stderr, "ipcio_open: invalid rdwrt = '%c'\n", rdwrt);
    return -1;
  }
  ipc->rdwrt = 0;
  ipc->bytes = 0;
  ipc->curbuf = NULL;
  if (rdwrt == 'W' || rdwrt == 'w') {
    if (ipcbuf_lock_write(&ipc->buf) < 0) return -1;
    if (rdwrt == 'w' && ipcbuf_disable_sod(&ipc->buf) < 0) return -1;
  } else if (rdwrt == 'R') {
    if (ipcbuf_lock_read(&ipc->buf) < 0) return -1;
  }
  ipc->rdwrt = rdwrt;
  return 0;
}

int ipcio_is_open(ipcio_t *ipc) {
  return ipc && (ipc->rdwrt == 'R' || ipc->rdwrt == 'r' || ipc->rdwrt == 'W' || ipc->rdwrt == 'w');
}

int ipcio_check_pending_sod(ipcio_t *ipc) {  /* @0x405b20 */
  if (!ipc->sod_pending || ipcbuf_get_write_count(&ipc->buf) <= ipc->sod_buf) return 0;
  if (ipcbuf_enable_sod(&ipc->buf, ipc->sod_buf, ipc->sod_byte) < 0) return -1;
  ipc->sod_pending = 0;
  return 0;
}

/* The slot of the 0-byte end-of-data block ipcio_close marks: taken as
 * get_next_write takes one (every reader's CLEAR for its last fill), but
 * waiting at most EOD_WAIT_S per reader, so a writer whose readers have gone
 * still ends its transfer -- then without the wait, as libpsrdada always
 * does (CLEARs taken in this round are given back first). */
#define EOD_WAIT_S 60
static int take_eod_slot(ipcbuf_t *id) {
  ipcsync_t *s = id->sync;
  const uint64_t b = s->w_buf % s->nbufs;
  while (id->count[b]) {
    for (unsigned r = 0; r < s->n_readers; r++) {
      struct sembuf sb = {SEM_CLEAR, -1, 0};
      struct timespec t = {EOD_WAIT_S, 0};
      while (semtimedop(id->semid_data[r], &sb, 1, &t) != 0) {
        if (errno == EINTR && !g_interrupt) continue;
        for (unsigned q = 0; q < r; q++) sem_op(id->semid_data[q], SEM_CLEAR, 1, 0);
        return errno == EAGAIN ? 0 : -1; /* EAGAIN: timed out */
      }
    }
    id->count[b]--;
  }
  return 0;
}

/* ipcio_stop_close (@0x405c10).  A writer with a transfer open ends it --
 * the block being written, or a 0-byte block after a full one, carries the
 * end of data -- and stays locked in 'w' mode (ipcio_start opens the next
 * transfer); with unlock it also resets w_buf to the last transfer's end
 * and unlocks.  A reader unlocks.  Departures, none visible to a reader:
 *  - the 0-byte block is taken like any other (get_next_write: the
 *    readers' CLEAR for its slot's last fill first).  libpsrdada marks it
 *    without that wait, so count[] runs one fill behind and the writer's
 *    next transfer can reuse a block a slow reader has not cleared yet
 *    (tests/test_dada.py::test_ring_transfers_property found it);
 *  - a writer that locked and wrote no block at all ends an empty transfer
 *    on close (a 0-byte end-of-data block) where libpsrdada would leave its
 *    readers waiting for data that never comes;
 *  - a viewer closes (back to VIEWER; libpsrdada refuses 'r' here). */
int ipcio_stop_close(ipcio_t *ipc, char unlock) {
  if (!ipc) return -1;
  ipcbuf_t *b = &ipc->buf;
  if (ipc->rdwrt == 'W') {
    if (unlock && b->state == ST_WCHANGE && !b->sync->w_state && ipcbuf_enable_sod(b, b->sync->w_buf, 0) < 0)
      return -1;
    if (ipcbuf_is_writing(b)) {
      if ((!ipc->curbuf || ipc->marked_filled) && take_eod_slot(b) < 0) return -1;
      if (ipcbuf_enable_eod(b) < 0 || ipcbuf_mark_filled(b, ipc->bytes) < 0 || ipcio_check_pending_sod(ipc) < 0)
        return -1;
      ipc->marked_filled = 1;
      if (ipc->bytes == ipcbuf_get_bufsz(&ipc->buf)) ipc->curbuf = NULL;
    }
    ipc->rdwrt = 'w';
    if (!unlock) return 0;
  }
  if (ipc->rdwrt == 'w') {
    ipcsync_t *s = ipc->buf.sync;
    if (s->w_xfer) s->w_buf = s->e_buf[(s->w_xfer - 1) % IPCBUF_XFERS] + 1;
    if (ipcbuf_unlock_write(&ipc->buf) < 0) return -1;
    ipc->rdwrt = 0;
    return 0;
  }
  if (ipc->rdwrt == 'R') {
    if (ipcbuf_unlock_read(&ipc->buf) < 0) return -1;
    ipc->rdwrt = 0;
    return 0;
  }
  if (ipc->rdwrt == 'r') {
    b->state = ST_VIEWER;
    ipc->rdwrt = 0;
    ipc->curbuf = NULL;
    ipc->bytes = 0;
    return 0;
  }
  fprintf(stderr, "ipcio_close: invalid ipcio_t\n");
  return -1;
}

int ipcio_close(ipcio_t *ipc) { return ipcio_stop_close(ipc, 1); }  /* @0x405e10 */

/* ipcio_stop (@0x405dd0): end the transfer, keep the writer lock */
int ipcio_stop(ipcio_t *ipc) {
  if (!ipc || ipc->rdwrt != 'W') {
    fprintf(stderr, "ipcio_stop: not writing!\n");
    return -1;
  }
  return ipcio_stop_close(ipc, 0);
}

/* ipcio_start (@0x405b90): a 'w' writer starts a transfer at byte `byte`
 * of its stream (block byte / bufsz, byte % bufsz into it), as soon as that
 * block has been written */
int ipcio_start(ipcio_t *ipc, uint64_t byte) {
  if (!ipc || ipc->rdwrt != 'w') {
    fprintf(stderr, "ipcio_start: invalid ipcio_t (%c)\n", ipc ? ipc->rdwrt : '?');
    return -1;
  }
  const uint64_t bufsz = ipcbuf_get_bufsz(&ipc->buf);
  ipc->sod_pending = 1;
  ipc->rdwrt = 'W';
  ipc->sod_buf = byte / bufsz;
  ipc->sod_byte = byte % bufsz;
  return ipcio_check_pending_sod(ipc);
}

char *ipcio_open_block_write(ipcio_t *ipc, uint64_t *block_id) {  /* @0x406340 */
  if (!ipc || ipc->bytes || ipc->curbuf || ipc->rdwrt != 'W') return NULL;
  ipc->curbuf = ipcbuf_get_next_write(&ipc->buf);
  if (!ipc->curbuf) return NULL;
  if (block_id) *block_id = ipcbuf_get_write_index(&ipc->buf);
  ipc->marked_filled = 0;
  ipc->bytes = 0;
  return ipc->curbuf;
}

ssize_t ipcio_update_block_write(ipcio_t *ipc, uint64_t bytes) {  /* @0x406490 */
  if (!ipc || ipc->bytes || !ipc->curbuf || ipc->rdwrt != 'W' || bytes > ipcbuf_get_bufsz(&ipc->buf))
    return -1;
  ipc->bytes += bytes;
  return 0;
}

ssize_t ipcio_close_block_write(ipcio_t *ipc, uint64_t bytes) {  /* @0x406580 */
  if (ipcio_update_block_write(ipc, bytes) < 0) return -1;
  if (ipc->marked_filled) return 0;
  if (ipcbuf_mark_filled(&ipc->buf, ipc->bytes) < 0) return -2;
  if (ipcio_check_pending_sod(ipc) < 0) return -3;
  ipc->marked_filled = 1;
  ipc->curbuf = NULL;
  ipc->bytes = 0;
  return 0;
}

char *ipcio_open_block_read(ipcio_t *ipc, uint64_t *curbufsz, uint64_t *block_id) {  /* @0x4060b0 */
  if (!ipc || ipc->bytes || (ipc->rdwrt != 'R' && ipc->rdwrt != 'r')) return NULL;
  ipcbuf_t *id = &ipc->buf;
  const int reader = ipc->rdwrt == 'R';
  if (ipc->curbuf && (!reader || rd_depth(id) <= 1)) return NULL; /* one block at a time (PSRDADA) */
  if (ipcbuf_eod(id)) return NULL;
  uint64_t sz = 0;
  char *p = ipcbuf_get_next_read(id, &sz);
  if (!p) return NULL;
  ipc->curbuf = p;
  ipc->curbufsz = sz;
  if (block_id)
    *block_id = (reader ? id->sync->r_bufs[id->iread] + (uint64_t)rd_open(id) - 1 : vw_pos(id) - 1) %
                id->sync->nbufs;
  if (curbufsz) *curbufsz = sz;
  ipc->bytes = 0;
  return p;
}

/* the block is released once `bytes` add up to its size (PSRDADA); a
 * reader holding several blocks (read depth > 1) releases the oldest */
ssize_t ipcio_close_block_read(ipcio_t *ipc, uint64_t bytes) {  /* @0x406200 */
  if (ipc && ipc->rdwrt == 'r' && ipc->curbuf) { /* a viewer: nothing to release (libpsrdada refuses) */
    ipc->curbuf = NULL;
    ipc->bytes = 0;
    return 0;
  }
  if (!ipc || ipc->rdwrt != 'R' || !ipc->curbuf) return -1;
  ipcbuf_t *id = &ipc->buf;
  if (rd_depth(id) > 1) {
    if (ipcbuf_mark_cleared(id) < 0) return -1;
    if (!rd_open(id)) ipc->curbuf = NULL;
    ipc->bytes = 0;
    return 0;
  }
  if (ipc->bytes) return -1;
  if (bytes != ipc->curbufsz) {
    ipc->bytes += bytes;
    if (ipc->bytes != ipc->curbufsz) return 0;
  }
  if (ipcbuf_mark_cleared(id) < 0) return -1;
  ipc->curbuf = NULL;
  ipc->bytes = 0;
  return 0;
}

/* ipcio_write (@0x405e40): a byte stream over the blocks */
ssize_t ipcio_write(ipcio_t *ipc, char *ptr, size_t bytes) {
  if (!ipc || (ipc->rdwrt != 'W' && ipc->rdwrt != 'w')) return -1;
  const uint64_t bufsz = ipcbuf_get_bufsz(&ipc->buf);
  size_t left = bytes;
  while (left) {
    if (ipc->bytes == bufsz) { /* the current block is full */
      if (!ipc->marked_filled) {
        if (ipcbuf_mark_filled(&ipc->buf, ipc->bytes) < 0 || ipcio_check_pending_sod(ipc) < 0) return -1;
      }
      ipc->curbuf = NULL;
      ipc->bytes = 0;
      ipc->marked_filled = 1;
    }
    if (!ipc->curbuf) {
      ipc->curbuf = ipcbuf_get_next_write(&ipc->buf);
      if (!ipc->curbuf) return -1;
      ipc->marked_filled = 0;
      ipc->bytes = 0;
    }
    uint64_t n = bufsz - ipc->bytes;
    if (n > left) n = left;
    if (ipcbuf_copy_in(&ipc->buf, ipc->curbuf + ipc->bytes, ptr, n) < 0) return -1;
    ipc->bytes += n;
    ptr += n;
    left -= n;
  }
  return (ssize_t)bytes;
}

/* ipcio_read (@0x406660): fewer bytes than asked at the end of data */
ssize_t ipcio_read(ipcio_t *ipc, char *ptr, size_t bytes) {
  if (!ipc || (ipc->rdwrt != 'R' && ipc->rdwrt != 'r')) return -1;
  size_t left = bytes;
  while (left && !ipcbuf_eod(&ipc->buf)) {
    if (!ipc->curbuf) {
      ipc->curbuf = ipcbuf_get_next_read(&ipc->buf, &ipc->curbufsz);
      if (!ipc->curbuf) return -1;
      ipc->bytes = 0;
    }
    uint64_t n = ipc->curbufsz - ipc->bytes;
    if (n > left) n = left;
    if (ptr) {
      if (ipcbuf_copy_out(&ipc->buf, ptr, ipc->curbuf + ipc->bytes, n) < 0) return -1;
      ptr += n;
    }
    ipc->bytes += n;
    left -= n;
    if (ipc->bytes == ipc->curbufsz) {
      if (ipc->rdwrt == 'R' && ipcbuf_mark_cleared(&ipc->buf) < 0) return -1;
      ipc->curbuf = NULL;
      ipc->bytes = 0;
    }
  }
  return (ssize_t)(bytes - left);
}

/* ------------------------------------------------------------------ */
/* dada_hdu                                                             */

dada_hdu_t *dada_hdu_create(multilog_t *log) {  /* @0x407490 */
  dada_hdu_t *h = calloc(1, sizeof(*h));
  if (!h) return NULL;
  h->log = log;
  h->data_block_key = 0xdada; /* PSRDADA's default key */
  h->header_block_key = 0xdadb;
  return h;
}

void dada_hdu_set_key(dada_hdu_t *h, key_t key) {
  if (!h) return;
  h->data_block_key = key;
  h->header_block_key = key + 1; /* header key = key+1 */
}

int dada_hdu_connect(dada_hdu_t *h) {  /* @0x407500: header ring first */
  if (!h || h->data_block) return -1;
  const ipcbuf_t hb = IPCBUF_INIT;
  const ipcio_t io = IPCIO_INIT;
  h->header_block = malloc(sizeof(ipcbuf_t));
  h->data_block = malloc(sizeof(ipcio_t));
  if (h->header_block) *h->header_block = hb;
  if (h->data_block) *h->data_block = io;
  const char *what = NULL;
  if (!h->header_block || !h->data_block)
    what = "out of memory";
  else if (ipcbuf_connect(h->header_block, h->header_block_key) < 0)
    what = "no header ring at key";
  else if (ipcio_connect(h->data_block, h->data_block_key) < 0)
    what = "no data ring at key";
  if (!what) return 0;
  if (h->log) multilog(h->log, LOG_ERR, "dada_hdu_connect: %s %x", what, (unsigned)h->data_block_key);
  if (h->header_block && h->header_block->sync) ipcbuf_disconnect(h->header_block);
  free(h->header_block);
  free(h->data_block);
  h->header_block = NULL;
  h->data_block = NULL;
  return -1;
}

int dada_hdu_disconnect(dada_hdu_t *h) {
  if (!h || !h->data_block) return -1;
  ipcio_disconnect(h->data_block);
  ipcbuf_disconnect(h->header_block);
  free(h->header_block);
  free(h->data_block);
  h->header_block = NULL;
  h->data_block = NULL;
  return 0;
}

void dada_hdu_destroy(dada_hdu_t *h) {
  if (!h) return;
  if (h->data_block) dada_hdu_disconnect(h);
  free(h->header);
  free(h);
}

int dada_hdu_lock_write_spec(dada_hdu_t *h, char mode) {  /* @0x407970 */
  if (!h || !h->data_block) return -1;
  if (ipcbuf_lock_write(h->header_block) < 0) return -1;
  if (ipcio_open(h->data_block, mode) < 0) {
    ipcbuf_unlock_write(h->header_block);
    return -1;
  }
  return 0;
}

int dada_hdu_lock_write(dada_hdu_t *h) { return dada_hdu_lock_write_spec(h, 'W'); }

int dada_hdu_unlock_write(dada_hdu_t *h) {  /* @0x407a20 */
  if (!h || !h->data_block) return -1;
  int rc = 0;
  if (ipcio_is_open(h->data_block) && ipcio_close(h->data_block) < 0) rc = -1;
  if (ipcbuf_unlock_write(h->header_block) < 0) rc = -1;
  return rc;
}

int dada_hdu_lock_read(dada_hdu_t *h) {  /* @0x407810 */
  if (!h || !h->data_block) return -1;
  if (ipcbuf_lock_read(h->header_block) < 0) return -1;
  if (ipcio_open(h->data_block, 'R') < 0) {
    ipcbuf_unlock_read(h->header_block);
    return -1;
  }
  return 0;
}

int dada_hdu_unlock_read(dada_hdu_t *h) {  /* @0x4078b0 */
  if (!h || !h->data_block) return -1;
  int rc = ipcio_is_open(h->data_block) && ipcio_close(h->data_block) < 0 ? -1 : 0;
  if (h->header) { /* the header block dada_hdu_open took goes back now */
    free(h->header);
    h->header = NULL;
    if (h->header_block->state == ST_READING) ipcbuf_mark_cleared(h->header_block);
  }
  if (ipcbuf_unlock_read(h->header_block) < 0) rc = -1;
  return rc;
}

/* dada_hdu_open (@0x407bc0): the next header block, empty end-of-data
 * header blocks skipped; kept (not cleared) until dada_hdu_unlock_read */
int dada_hdu_open(dada_hdu_t *h) {
  if (!h || !h->header_block || h->header) return -1;
  ipcbuf_t *hb = h->header_block;
  uint64_t size = 0;
  char *p = NULL;
  while (!size) {
    p = ipcbuf_get_next_read(hb, &size);
    if (!p) {
      if (h->log) multilog(h->log, LOG_ERR, "dada_hdu_open: could not get next header block");
      return -1;
    }
    if (!size) {
      if (hb->state == ST_READING) ipcbuf_mark_cleared(hb);
      if (!ipcbuf_eod(hb)) {
        if (h->log) multilog(h->log, LOG_ERR, "dada_hdu_open: empty header block");
        return -1;
      }
      ipcbuf_reset(hb);
    }
  }
  size = ipcbuf_get_bufsz(hb);
  uint64_t hdr_size = 0;
  if (ascii_header_get(p, "HDR_SIZE", "%" SCNu64, &hdr_size) != 1 || hdr_size == 0) hdr_size = size;
  if (hdr_size > size) {
    if (h->log) multilog(h->log, LOG_ERR, "dada_hdu_open: HDR_SIZE %" PRIu64 " > block %" PRIu64,
                         hdr_size, size);
    return -1;
  }
  h->header = malloc(hdr_size + 1);
  if (!h->header) return -1;
  memcpy(h->header, p, hdr_size);
  h->header[hdr_size] = 0;
  h->header_size = hdr_size;
  return 0;
}

int dada_hdu_open_read(dada_hdu_t *h) { return dada_hdu_open(h); }

/* dada_hdu_open_view / _close_view (@0x407ac0 / @0x407b40): view the data
 * ring (ipcio 'r'); the header ring is not touched */
int dada_hdu_open_view(dada_hdu_t *h) {
  if (!h || !h->data_block) {
    fprintf(stderr, "dada_hdu_open_view: not connected\n");
    return -1;
  }
  if (ipcio_open(h->data_block, 'r') < 0) {
    if (h->log) multilog(h->log, LOG_ERR, "Could not open Data Block for viewing\n");
    return -1;
  }
  return 0;
}

int dada_hdu_close_view(dada_hdu_t *h) {
  if (!h || !h->data_block) {
    fprintf(stderr, "dada_hdu_close_view: not connected\n");
    return -1;
  }
  if (ipcio_close(h->data_block) < 0) {
    if (h->log) multilog(h->log, LOG_ERR, "Could not close Data Block view\n");
    return -1;
  }
  return 0;
}

/* dada_hdu_db_addresses / _hb_addresses (@0x407e50 / @0x407e80): the block
 * address list of the data / header ring, with its geometry */
char **dada_hdu_db_addresses(dada_hdu_t *h, uint64_t *nbufs, uint64_t *bufsz) {
  if (!h || !h->data_block) return NULL;
  ipcbuf_t *b = &h->data_block->buf;
  if (nbufs) *nbufs = ipcbuf_get_nbufs(b);
  if (bufsz) *bufsz = ipcbuf_get_bufsz(b);
  return b->buffer;
}

char **dada_hdu_hb_addresses(dada_hdu_t *h, uint64_t *nbufs, uint64_t *bufsz) {
  if (!h || !h->header_block) return NULL;
  ipcbuf_t *b = h->header_block;
  if (nbufs) *nbufs = ipcbuf_get_nbufs(b);
  if (bufsz) *bufsz = ipcbuf_get_bufsz(b);
  return b->buffer;
}

/* ------------------------------------------------------------------ */
/* ring pairs (the dada_db tool)                                        */

int dada_db_create(key_t key, uint64_t nbufs, uint64_t bufsz, unsigned n_readers, uint64_t hdr_nbufs,
                   uint64_t hdr_bufsz) {
  return dada_db_create_work(key, nbufs, bufsz, n_readers, hdr_nbufs, hdr_bufsz, -1);
}

/* the creator does not open a device ring's blocks: they are opened only by
 * the processes that use them */
int dada_db_create_work(key_t key, uint64_t nbufs, uint64_t bufsz, unsigned n_readers,
                        uint64_t hdr_nbufs, uint64_t hdr_bufsz, int device_id) {
  ipcbuf_t d, hb;
  if (ring_create(&d, key, nbufs, bufsz, n_readers, device_id < 0 ? -1 : device_id, 0) < 0) return -1;
  ipcbuf_disconnect(&d);
  if (ring_create(&hb, key + 1, hdr_nbufs, hdr_bufsz, n_readers, -1, 1) < 0) {
    const int e = errno;
    dada_db_destroy(key);
    errno = e;
    return -1;
  }
  ipcbuf_disconnect(&hb);
  return 0;
}

/* removes one ring without opening its blocks (a device ring's holder is
 * stopped instead) */
static int ring_remove(key_t key) {
  ipcbuf_t id = IPCBUF_INIT;
  if (sync_get(&id, key, 0, 0) < 0) {
    /* no sync segment: remove what a creation that died half-way may have
     * left at the ring's keys (semaphores, blocks 0, 1, ... while present),
     * so the key can be used again; still "nothing to destroy" */
    for (int r = -1; r < IPCBUF_READERS; r++) {
      const int sem = semget(r < 0 ? key_connect(key) : key_data(key, r), 0, 0);
      if (sem >= 0) semctl(sem, 0, IPC_RMID);
    }
    for (uint64_t i = 0; i < 0x7fff; i++) {
      const int sid = shmget(key_block(key, i), 0, 0);
      if (sid < 0) break;
      shmctl(sid, IPC_RMID, NULL);
    }
    return -1;
  }
  ipcsync_t *s = id.sync;
  int rc = 0, busy = 0;
  if (s->semkey_connect == 0) rc = -1; /* not a (complete) ring */
  if (s->on_device_id >= 0) {
    const int sid = shmget(shmkey_get(&id, 0), 0, 0);
    if (sid >= 0 && seg_size(sid) >= sizeof(dev_seg_t) && dev_stop_holder(sid) < 0) {
      rc = -1;
      busy = errno == EBUSY; /* kept through the removals below */
    }
  }
  for (uint64_t i = 0; i < s->nbufs; i++) {
    const int sid = shmget(shmkey_get(&id, i), 0, 0);
    if (sid >= 0) shmctl(sid, IPC_RMID, NULL);
  }
  for (unsigned r = 0; r < s->n_readers && r < IPCBUF_READERS; r++) {
    const int sem = semget(s->semkey_data[r], 0, 0);
    if (sem >= 0) semctl(sem, 0, IPC_RMID);
  }
  const int sem = semget(key_connect(key), 0, 0);
  if (sem >= 0) semctl(sem, 0, IPC_RMID);
  shmdt(s);
  shmctl(id.syncid, IPC_RMID, NULL);
  if (busy) errno = EBUSY; /* the holder still serves importers: not "nothing to destroy" */
  return rc;
}

int dada_db_destroy(key_t key) {
  const int a = ring_remove(key);
  const int e = errno; /* EBUSY: the data ring's holder still serves importers */
  const int b = ring_remove(key + 1);
  if (a != 0) errno = e;
  return a == 0 && b == 0 ? 0 : -1;
}

int dada_device_ring_info(key_t key, dada_device_info_t *info) {
  if (!info) {
    errno = EINVAL;
    return -1;
  }
  memset(info, 0, sizeof *info);
  ipcbuf_t id = IPCBUF_INIT;
  if (sync_get(&id, key, 0, 0) < 0) return -1;
  const int dev = id.sync->on_device_id;
  const key_t k0 = shmkey_get(&id, 0);
  shmdt(id.sync);
  if (dev < 0) {
    errno = ENODEV; /* a host ring */
    return -1;
  }
  const int sid = shmget(k0, 0, 0);
  dev_seg_t v;
  if (sid < 0 || seg_size(sid) < sizeof(dev_seg_t) || dev_look_seg0(sid, &v) < 0) {
    errno = ENOENT;
    return -1;
  }
  info->device = dev;
  info->holder_pid = v.holder_pid;
  info->holder_state = v.holder_state;
  info->importers = v.importers;
  info->export_retries = v.export_retries;
  info->primer_refused = v.primer_refused;
  return 0;
}

long fileread(const char *filename, char *buffer, unsigned bufsz) {
  if (!filename || !buffer || !bufsz) return -1;
  FILE *fp = fopen(filename, "r");
  if (!fp) return -1;
  memset(buffer, 0, bufsz);
  size_t n = fread(buffer, 1, bufsz - 1, fp);
  fclose(fp);
  return (long)n;
}
