/*
 * dada_ring.c -- SysV shared-memory rings with the PSRDADA ipcbuf / ipcio /
 * dada_hdu call surface (include/b2p_dada.h).
 *
 * The reference links PSRDADA and uses its writer half (diskdb.cu:24-124,
 * capture.c:586-642, sync.c:101-109); the reader half its baseband2power
 * stage needed was never written.  Semantics
 * kept from PSRDADA: data ring at key, header ring at key+1; one writer,
 * several readers, each sees every block; a block marked filled with fewer
 * than bufsz bytes ends the transfer; a writer that stops
 * on a full block ends it with an empty block (ipcbuf_enable_eod).
 */
#include <errno.h>
#include <signal.h>
#include <stdarg.h>
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

/* set by dada_interrupt_waits (a signal handler): interrupted waits fail */
static volatile sig_atomic_t g_interrupt;

void dada_interrupt_waits(void) { g_interrupt = 1; }

/* semop with EINTR retry (until dada_interrupt_waits); flags e.g.
 * SEM_UNDO | IPC_NOWAIT */
static int sem_do(int semid, int num, int op, int flags) {
  struct sembuf sb;
  sb.sem_num = (unsigned short)num;
  sb.sem_op = (short)op;
  sb.sem_flg = (short)flags;
  for (;;) {
    if (semop(semid, &sb, 1) == 0) return 0;
    if (errno != EINTR || (g_interrupt && op < 0)) return -1;
  }
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

int multilog(multilog_t *m, int priority, const char *format, ...) {
  if (!m) return -1;
  char msg[1024];
  va_list ap;
  va_start(ap, format);
  vsnprintf(msg, sizeof msg, format, ap);
  va_end(ap);
  char ts[64];
  time_t now = time(NULL);
  struct tm tmv;
  strftime(ts, sizeof ts, "%Y-%m-%d-%H:%M:%S", localtime_r(&now, &tmv));
  for (int i = 0; i < m->nfp; i++) {
    fprintf(m->fp[i], "[%s] %s%s%s", ts, priority <= LOG_ERR ? "ERR " : "", msg,
            (msg[0] && msg[strlen(msg) - 1] == '\n') ? "" : "\n");
    fflush(m->fp[i]);
  }
  if (m->use_syslog) syslog(priority, "%s", msg);
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
/* ipcbuf                                                               */

/* Build the sync segment, the semaphores and the blocks: SysV segments for
 * a host ring, device memory held by a holder process for a device ring
 * (dada_device.c).  The magic is written last, so a connector never sees a
 * half-built ring. */
static int ring_create(key_t key, uint64_t nbufs, uint64_t bufsz, unsigned n_readers, int device) {
  if (!nbufs || !bufsz || n_readers > IPCBUF_READERS || nbufs > 32767) return -1;
  int syncid = shmget(key, sync_size(nbufs), IPC_CREAT | IPC_EXCL | 0666);
  if (syncid < 0) return -1;
  ipcsync_t *s = shmat(syncid, NULL, 0);
  if (s == (void *)-1) {
    shmctl(syncid, IPC_RMID, NULL);
    return -1;
  }
  memset(s, 0, sync_size(nbufs));
  s->nbufs = nbufs;
  for (uint64_t i = 0; i < nbufs; i++) sync_shmids(s)[i] = -1;
  s->bufsz = bufsz;
  s->n_readers = n_readers;
  s->on_device_id = -1;
  s->semid = semget(IPC_PRIVATE, NSEMS, IPC_CREAT | 0666);
  int ok = s->semid >= 0;
  if (ok) {
    unsigned short v[NSEMS];
    memset(v, 0, sizeof v);
    v[SEM_CLEAR] = (unsigned short)nbufs;
    v[SEM_WLOCK] = 1;
    for (int r = 0; r < IPCBUF_READERS; r++) v[SEM_RLOCK(r)] = 1;
    union semun_u {
      int val;
      struct semid_ds *buf;
      unsigned short *array;
    } arg;
    arg.array = v;
    ok = semctl(s->semid, 0, SETALL, arg) == 0;
  }
  if (ok && device >= 0) {
    ok = dev_create_blocks(syncid, s, device) == 0;
  } else {
    for (uint64_t i = 0; ok && i < nbufs; i++) {
      int sid = shmget(IPC_PRIVATE, bufsz, IPC_CREAT | 0666);
      sync_shmids(s)[i] = sid;
      if (sid < 0) ok = 0;
    }
  }
  if (!ok) {
    const int e = errno;
    for (uint64_t i = 0; i < nbufs; i++)
      if (sync_shmids(s)[i] >= 0) shmctl(sync_shmids(s)[i], IPC_RMID, NULL);
    if (s->semid >= 0) semctl(s->semid, 0, IPC_RMID);
    shmdt(s);
    shmctl(syncid, IPC_RMID, NULL);
    errno = e;
    return -1;
  }
  s->version = SYNC_VERSION;
  __atomic_store_n(&s->magic, SYNC_MAGIC, __ATOMIC_RELEASE);
  shmdt(s);
  return 0;
}

int ipcbuf_create(ipcbuf_t *id, key_t key, uint64_t nbufs, uint64_t bufsz, unsigned n_readers) {
  return ipcbuf_create_work(id, key, nbufs, bufsz, n_readers, -1);
}

int ipcbuf_create_work(ipcbuf_t *id, key_t key, uint64_t nbufs, uint64_t bufsz, unsigned n_readers,
                       int device_id) {
  if (!id || ring_create(key, nbufs, bufsz, n_readers, device_id) < 0) return -1;
  return ipcbuf_connect(id, key);
}

int ipcbuf_connect(ipcbuf_t *id, key_t key) {
  if (!id) return -1;
  ipcbuf_t init = IPCBUF_INIT;
  *id = init;
  id->key = key;
  id->syncid = shmget(key, 0, 0);
  if (id->syncid < 0) return -1;
  id->sync = shmat(id->syncid, NULL, 0);
  if (id->sync == (void *)-1) {
    id->sync = NULL;
    return -1;
  }
  if (__atomic_load_n(&id->sync->magic, __ATOMIC_ACQUIRE) != SYNC_MAGIC ||
      id->sync->version != SYNC_VERSION) {
    shmdt(id->sync);
    id->sync = NULL;
    errno = EINVAL;
    return -1;
  }
  id->nbufs = id->sync->nbufs;
  id->bufsz = id->sync->bufsz;
  id->semid = id->sync->semid;
  id->buffer = calloc(id->nbufs, sizeof(char *));
  if (!id->buffer) return -1;
  if (id->sync->on_device_id >= 0) {
    if (dev_open_blocks(id) < 0) {
      ipcbuf_disconnect(id);
      return -1;
    }
  } else {
    for (uint64_t i = 0; i < id->nbufs; i++) {
      void *p = shmat(sync_shmids(id->sync)[i], NULL, 0);
      if (p == (void *)-1) {
        ipcbuf_disconnect(id);
        return -1;
      }
      id->buffer[i] = p;
    }
  }
  id->state = 1;
  return 0;
}

int ipcbuf_disconnect(ipcbuf_t *id) {
  if (!id) return -1;
  if (id->state == 2) ipcbuf_unlock_write(id);
  if (id->state == 3) ipcbuf_unlock_read(id);
  if (id->buffer) {
    if (id->sync && id->sync->on_device_id >= 0) {
      dev_close_blocks(id);
    } else {
      for (uint64_t i = 0; i < id->nbufs; i++)
        if (id->buffer[i]) shmdt(id->buffer[i]);
    }
    free(id->buffer);
    id->buffer = NULL;
  }
  if (id->sync) shmdt(id->sync);
  id->sync = NULL;
  id->state = 0;
  return 0;
}

int ipcbuf_destroy(ipcbuf_t *id) {
  if (!id || !id->sync) return -1;
  int semid = id->semid, syncid = id->syncid;
  uint64_t n = id->nbufs;
  int32_t *ids = malloc(n * sizeof(int32_t));
  if (!ids) return -1;
  memcpy(ids, sync_shmids(id->sync), n * sizeof(int32_t));
  ipcsync_t *s = shmat(syncid, NULL, 0); /* outlives the disconnect below */
  ipcbuf_disconnect(id);
  if (s != (void *)-1) {
    if (s->on_device_id >= 0) dev_stop_holder(s);
    shmdt(s);
  }
  for (uint64_t i = 0; i < n; i++)
    if (ids[i] >= 0) shmctl(ids[i], IPC_RMID, NULL);
  free(ids);
  semctl(semid, 0, IPC_RMID);
  shmctl(syncid, IPC_RMID, NULL);
  return 0;
}

int ipcbuf_lock_write(ipcbuf_t *id) {
  if (!id || id->state != 1) return -1;
  if (sem_do(id->semid, SEM_WLOCK, -1, SEM_UNDO | IPC_NOWAIT) < 0) return -1;
  id->state = 2;
  id->xfer_count = id->sync->w_count;
  id->wrote_eod = 0;
  return 0;
}

int ipcbuf_unlock_write(ipcbuf_t *id) {
  if (!id || id->state != 2) return -1;
  sem_do(id->semid, SEM_WLOCK, 1, SEM_UNDO);
  id->state = 1;
  return 0;
}

int ipcbuf_lock_read(ipcbuf_t *id) {
  if (!id || id->state != 1) return -1;
  for (uint32_t r = 0; r < id->sync->n_readers; r++) {
    if (sem_do(id->semid, SEM_RLOCK(r), -1, SEM_UNDO | IPC_NOWAIT) == 0) {
      id->iread = (int)r;
      id->state = 3;
      id->xfer_count = id->sync->r_count[r];
      id->eod_seen = 0; /* the next transfer starts after the last EOD taken */
      return 0;
    }
  }
  return -1;
}

int ipcbuf_unlock_read(ipcbuf_t *id) {
  if (!id || id->state != 3) return -1;
  sem_do(id->semid, SEM_RLOCK(id->iread), 1, SEM_UNDO);
  id->iread = -1;
  id->state = 1;
  return 0;
}

char *ipcbuf_get_next_write(ipcbuf_t *id) {
  if (!id || id->state != 2 || id->cur_open) return NULL;
  if (sem_do(id->semid, SEM_CLEAR, -1, 0) < 0) return NULL;
  id->cur_index = id->sync->w_count % id->nbufs;
  id->cur_open = 1;
  return id->buffer[id->cur_index];
}

int ipcbuf_mark_filled(ipcbuf_t *id, uint64_t nbytes) {
  if (!id || id->state != 2 || !id->cur_open || nbytes > id->bufsz) return -1;
  ipcsync_t *s = id->sync;
  sync_nbytes(s)[id->cur_index] = nbytes;
  sync_eod(s)[id->cur_index] = nbytes < id->bufsz; /* short block = EOD */
  if (nbytes < id->bufsz) id->wrote_eod = 1;
  __atomic_store_n(&s->w_count, s->w_count + 1, __ATOMIC_RELEASE);
  id->cur_open = 0;
  id->xfer_count++;
  for (uint32_t r = 0; r < s->n_readers; r++)
    if (sem_do(id->semid, SEM_FULL(r), 1, 0) < 0) return -1;
  return 0;
}

int ipcbuf_enable_eod(ipcbuf_t *id) {
  if (!id || id->state != 2) return -1;
  if (id->wrote_eod) return 0; /* this session's transfer already ended */
  if (!ipcbuf_get_next_write(id)) return -1;
  return ipcbuf_mark_filled(id, 0);
}

int ipcbuf_set_read_depth(ipcbuf_t *id, int depth) {
  if (!id || depth < 1 || (uint64_t)depth > id->nbufs) return -1;
  id->read_depth = depth;
  return 0;
}

char *ipcbuf_get_next_read(ipcbuf_t *id, uint64_t *bytes) {
  if (!id || id->state != 3) return NULL;
  if (id->cur_open >= (id->read_depth > 1 ? id->read_depth : 1)) return NULL;
  if (id->eod_seen) return NULL; /* this transfer is over */
  if (sem_do(id->semid, SEM_FULL(id->iread), -1, 0) < 0) return NULL;
  id->cur_index = (id->sync->r_count[id->iread] + (uint64_t)id->cur_open) % id->nbufs;
  id->cur_open++;
  if (sync_eod(id->sync)[id->cur_index]) id->eod_seen = 1;
  if (bytes) *bytes = sync_nbytes(id->sync)[id->cur_index];
  return id->buffer[id->cur_index];
}

static int clear_oldest(ipcbuf_t *id) {
  ipcsync_t *s = id->sync;
  const uint64_t idx = s->r_count[id->iread] % id->nbufs;
  s->r_count[id->iread]++;
  id->cur_open--;
  id->xfer_count++;
  if (__atomic_add_fetch(&sync_clear(s)[idx], 1, __ATOMIC_ACQ_REL) == s->n_readers) {
    __atomic_store_n(&sync_clear(s)[idx], 0, __ATOMIC_RELEASE);
    if (sem_do(id->semid, SEM_CLEAR, 1, 0) < 0) return -1;
  }
  return 0;
}

int ipcbuf_mark_cleared(ipcbuf_t *id) {
  if (!id || id->state != 3 || id->cur_open < 1) return -1;
  if (clear_oldest(id) < 0) return -1;
  /* an empty EOD block taken behind open ones goes once it is the oldest */
  if (id->eod_pending && id->cur_open == 1) {
    id->eod_pending = 0;
    return clear_oldest(id);
  }
  return 0;
}

int ipcbuf_enable_sod(ipcbuf_t *id, uint64_t start_buf, uint64_t start_byte) {
  if (!id || !id->sync) return -1;
  id->sync->sod = 1;
  id->sync->s_buf = start_buf;
  id->sync->s_byte = start_byte;
  return 0;
}

int ipcbuf_disable_sod(ipcbuf_t *id) {
  if (!id || !id->sync) return -1;
  id->sync->sod = 0;
  return 0;
}

int ipcbuf_sod(ipcbuf_t *id) { return id && id->sync ? id->sync->sod : 0; }

int ipcbuf_eod(ipcbuf_t *id) {
  if (!id || !id->sync || id->iread < 0) return 0;
  return id->eod_seen;
}

uint64_t ipcbuf_get_bufsz(ipcbuf_t *id) { return id ? id->bufsz : 0; }
uint64_t ipcbuf_get_nbufs(ipcbuf_t *id) { return id ? id->nbufs : 0; }
uint64_t ipcbuf_get_nreaders(ipcbuf_t *id) { return id && id->sync ? id->sync->n_readers : 0; }
char *ipcbuf_get_buffer(ipcbuf_t *id, uint64_t i) {
  return id && id->buffer && i < id->nbufs ? id->buffer[i] : NULL;
}
int ipcbuf_get_device(ipcbuf_t *id) { return id && id->sync ? id->sync->on_device_id : -1; }

int ipcbuf_copy_in(ipcbuf_t *id, char *block, const void *src, uint64_t n) {
  if (!id || !id->sync || (!block && n) || (!src && n)) return -1;
  if (id->sync->on_device_id >= 0) return dev_copy(block, src, n);
  memcpy(block, src, n);
  return 0;
}

int ipcbuf_copy_out(ipcbuf_t *id, void *dst, const char *block, uint64_t n) {
  if (!id || !id->sync || (!block && n) || (!dst && n)) return -1;
  if (id->sync->on_device_id >= 0) return dev_copy(dst, block, n);
  memcpy(dst, block, n);
  return 0;
}

uint64_t ipcbuf_get_write_count(ipcbuf_t *id) { return id && id->sync ? id->sync->w_count : 0; }
uint64_t ipcbuf_get_read_count(ipcbuf_t *id, int iread) {
  return id && id->sync && iread >= 0 && iread < IPCBUF_READERS ? id->sync->r_count[iread] : 0;
}

/* ------------------------------------------------------------------ */
/* ipcio                                                                */

int ipcio_open(ipcio_t *ipc, char rdwrt) {
  if (!ipc) return -1;
  ipc->rdwrt = rdwrt;
  ipc->curbuf = NULL;
  ipc->curbufsz = 0;
  return rdwrt == 'W' ? ipcbuf_lock_write(&ipc->buf) : ipcbuf_lock_read(&ipc->buf);
}

int ipcio_close(ipcio_t *ipc) {
  if (!ipc) return -1;
  if (ipc->buf.state == 2) return ipcbuf_enable_eod(&ipc->buf);
  return 0;
}

char *ipcio_open_block_write(ipcio_t *ipc, uint64_t *block_id) {
  if (!ipc) return NULL;
  char *p = ipcbuf_get_next_write(&ipc->buf);
  if (p && block_id) *block_id = ipc->buf.cur_index;
  ipc->curbuf = p;
  ipc->curbufsz = ipc->buf.bufsz;
  return p;
}

int ipcio_close_block_write(ipcio_t *ipc, uint64_t bytes) {
  if (!ipc) return -1;
  ipc->curbuf = NULL;
  return ipcbuf_mark_filled(&ipc->buf, bytes);
}

char *ipcio_open_block_read(ipcio_t *ipc, uint64_t *curbufsz, uint64_t *block_id) {
  if (!ipc) return NULL;
  uint64_t bytes = 0;
  char *p = ipcbuf_get_next_read(&ipc->buf, &bytes);
  if (!p) return NULL;
  if (bytes == 0 && ipcbuf_eod(&ipc->buf)) { /* empty EOD marker block */
    if (ipc->buf.cur_open == 1)
      ipcbuf_mark_cleared(&ipc->buf);
    else
      ipc->buf.eod_pending = 1; /* released after the blocks still open */
    return NULL;
  }
  if (curbufsz) *curbufsz = bytes;
  if (block_id) *block_id = ipc->buf.cur_index;
  ipc->curbuf = p;
  ipc->curbufsz = bytes;
  return p;
}

ssize_t ipcio_close_block_read(ipcio_t *ipc, uint64_t bytes) {
  (void)bytes;
  if (!ipc) return -1;
  ipc->curbuf = NULL;
  return ipcbuf_mark_cleared(&ipc->buf);
}

/* ------------------------------------------------------------------ */
/* dada_hdu                                                             */

dada_hdu_t *dada_hdu_create(multilog_t *log) {
  dada_hdu_t *h = calloc(1, sizeof(*h));
  if (!h) return NULL;
  h->log = log;
  h->data_block_key = 0xdada;  /* PSRDADA default key */
  h->header_block_key = 0xdadb;
  return h;
}

void dada_hdu_set_key(dada_hdu_t *h, key_t key) {
  if (!h) return;
  h->data_block_key = key;
  h->header_block_key = key + 1; /* header key = key+1 */
}

int dada_hdu_connect(dada_hdu_t *h) {
  if (!h) return -1;
  ipcio_t io = IPCIO_INIT;
  ipcbuf_t hb = IPCBUF_INIT;
  h->data_block = malloc(sizeof(ipcio_t));
  h->header_block = malloc(sizeof(ipcbuf_t));
  if (!h->data_block || !h->header_block) return -1;
  *h->data_block = io;
  *h->header_block = hb;
  if (ipcbuf_connect(&h->data_block->buf, h->data_block_key) < 0) {
    if (h->log) multilog(h->log, LOG_ERR, "dada_hdu_connect: no data ring at key %x", h->data_block_key);
    return -1;
  }
  if (ipcbuf_connect(h->header_block, h->header_block_key) < 0) {
    if (h->log) multilog(h->log, LOG_ERR, "dada_hdu_connect: no header ring at key %x", h->header_block_key);
    ipcbuf_disconnect(&h->data_block->buf);
    return -1;
  }
  return 0;
}

int dada_hdu_disconnect(dada_hdu_t *h) {
  if (!h) return -1;
  if (h->data_block) {
    ipcbuf_disconnect(&h->data_block->buf);
    free(h->data_block);
    h->data_block = NULL;
  }
  if (h->header_block) {
    ipcbuf_disconnect(h->header_block);
    free(h->header_block);
    h->header_block = NULL;
  }
  return 0;
}

void dada_hdu_destroy(dada_hdu_t *h) {
  if (!h) return;
  if (h->data_block || h->header_block) dada_hdu_disconnect(h);
  free(h->header);
  free(h);
}

int dada_hdu_lock_write(dada_hdu_t *h) {
  if (!h || !h->data_block) return -1;
  if (ipcbuf_lock_write(h->header_block) < 0) return -1;
  if (ipcio_open(h->data_block, 'W') < 0) {
    ipcbuf_unlock_write(h->header_block);
    return -1;
  }
  return 0;
}

int dada_hdu_unlock_write(dada_hdu_t *h) {
  if (!h || !h->data_block) return -1;
  if (h->data_block->curbuf) ipcio_close_block_write(h->data_block, 0);
  ipcio_close(h->data_block);
  ipcbuf_unlock_write(&h->data_block->buf);
  ipcbuf_unlock_write(h->header_block);
  return 0;
}

int dada_hdu_lock_read(dada_hdu_t *h) {
  if (!h || !h->data_block) return -1;
  if (ipcbuf_lock_read(h->header_block) < 0) return -1;
  if (ipcio_open(h->data_block, 'R') < 0) {
    ipcbuf_unlock_read(h->header_block);
    return -1;
  }
  return 0;
}

int dada_hdu_unlock_read(dada_hdu_t *h) {
  if (!h || !h->data_block) return -1;
  ipcbuf_unlock_read(&h->data_block->buf);
  ipcbuf_unlock_read(h->header_block);
  return 0;
}

int dada_hdu_open_read(dada_hdu_t *h) {
  if (!h || !h->header_block) return -1;
  uint64_t bytes = 0;
  char *p = ipcbuf_get_next_read(h->header_block, &bytes);
  if (!p) return -1;
  uint64_t hsz = ipcbuf_get_bufsz(h->header_block);
  if (!h->header) {
    h->header = calloc(1, hsz + 1);
    if (!h->header) return -1;
  }
  h->header_size = hsz;
  memcpy(h->header, p, bytes < hsz ? bytes : hsz);
  h->header[hsz] = 0;
  return ipcbuf_mark_cleared(h->header_block);
}

int dada_db_create(key_t key, uint64_t nbufs, uint64_t bufsz, unsigned n_readers, uint64_t hdr_nbufs,
                   uint64_t hdr_bufsz) {
  return dada_db_create_work(key, nbufs, bufsz, n_readers, hdr_nbufs, hdr_bufsz, -1);
}

/* the creator does not attach: a device ring's blocks are opened only by
 * the processes that use them */
int dada_db_create_work(key_t key, uint64_t nbufs, uint64_t bufsz, unsigned n_readers,
                        uint64_t hdr_nbufs, uint64_t hdr_bufsz, int device_id) {
  if (ring_create(key, nbufs, bufsz, n_readers, device_id) < 0) return -1;
  if (ring_create(key + 1, hdr_nbufs, hdr_bufsz, n_readers, -1) < 0) {
    const int e = errno;
    dada_db_destroy(key);
    errno = e;
    return -1;
  }
  return 0;
}

/* removes one ring without attaching its blocks (a device ring's holder is
 * stopped instead) */
static int ring_remove(key_t key) {
  int syncid = shmget(key, 0, 0);
  if (syncid < 0) return -1;
  ipcsync_t *s = shmat(syncid, NULL, 0);
  if (s == (void *)-1) return -1;
  int rc = 0;
  if (s->magic == SYNC_MAGIC && s->version == SYNC_VERSION) {
    if (s->on_device_id >= 0) rc = dev_stop_holder(s);
    for (uint64_t i = 0; i < s->nbufs; i++)
      if (sync_shmids(s)[i] >= 0) shmctl(sync_shmids(s)[i], IPC_RMID, NULL);
    semctl(s->semid, 0, IPC_RMID);
  } else {
    rc = -1;
  }
  shmdt(s);
  shmctl(syncid, IPC_RMID, NULL);
  return rc;
}

int dada_db_destroy(key_t key) {
  const int a = ring_remove(key), b = ring_remove(key + 1);
  return a == 0 && b == 0 ? 0 : -1;
}

int fileread(const char *filename, char *buffer, unsigned bufsz) {
  if (!filename || !buffer || !bufsz) return -1;
  FILE *fp = fopen(filename, "r");
  if (!fp) return -1;
  memset(buffer, 0, bufsz);
  size_t n = fread(buffer, 1, bufsz - 1, fp);
  fclose(fp);
  return (int)n;
}
