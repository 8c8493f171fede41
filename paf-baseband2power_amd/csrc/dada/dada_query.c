/*
 * dada_query.c -- the rest of the PSRDADA ring API the reference's binaries
 * link (tests/golden/psrdada_abi.json): semaphore counts, transfer
 * positions ("tell"), the stream-level ipcio queries and seek.  Restated
 * from the same disassembly as dada_ring.c (addresses are paf_diskdb's);
 * where libpsrdada reads a field that looks unintended the restatement
 * reads the same one, so a caller sees the same numbers under either
 * library.
 */
#include <stdio.h>
#include <sys/ipc.h>
#include <sys/sem.h>

#include "b2p_dada.h"
#include "dada_internal.h"

/* ---- semaphore counts: FULL / CLEAR / SODACK / EODACK / READER_CONN ----
 * iread >= 0: that reader's set.  iread < 0: reader 0's for a process that
 * is not a reader; for a reader, every reader's set is read and the last
 * one's value returned (as the binary does, @0x4053d0) */
static long sem_count(ipcbuf_t *id, int iread, int num) {
  if (!id || !id->sync || !id->semid_data || !id->sync->n_readers) return 0;
  const unsigned n = id->sync->n_readers;
  if (iread >= 0) return (unsigned)iread < n ? semctl(id->semid_data[iread], num, GETVAL) : 0;
  if (id->iread == -1) return semctl(id->semid_data[0], num, GETVAL);
  long v = 0;
  for (unsigned r = 0; r < n; r++) v = semctl(id->semid_data[r], num, GETVAL);
  return v;
}

uint64_t ipcbuf_get_nfull_iread(ipcbuf_t *id, int iread) { return (uint64_t)sem_count(id, iread, SEM_FULL); }
uint64_t ipcbuf_get_nfull(ipcbuf_t *id) { return ipcbuf_get_nfull_iread(id, -1); }
uint64_t ipcbuf_get_nclear_iread(ipcbuf_t *id, int iread) { return (uint64_t)sem_count(id, iread, SEM_CLEAR); }
uint64_t ipcbuf_get_nclear(ipcbuf_t *id) { return ipcbuf_get_nclear_iread(id, -1); }
uint64_t ipcbuf_get_sodack_iread(ipcbuf_t *id, int iread) { return (uint64_t)sem_count(id, iread, SEM_SODACK); }
uint64_t ipcbuf_get_sodack(ipcbuf_t *id) { return ipcbuf_get_sodack_iread(id, -1); }
uint64_t ipcbuf_get_eodack_iread(ipcbuf_t *id, int iread) { return (uint64_t)sem_count(id, iread, SEM_EODACK); }
uint64_t ipcbuf_get_eodack(ipcbuf_t *id) { return ipcbuf_get_eodack_iread(id, -1); }
int ipcbuf_get_reader_conn_iread(ipcbuf_t *id, int iread) { return (int)sem_count(id, iread, SEM_READER_CONN); }
int ipcbuf_get_reader_conn(ipcbuf_t *id) { return ipcbuf_get_reader_conn_iread(id, -1); }

/* free reader slots (the connect set's READ count, @0x405780) */
/* ---- extensions (not in PSRDADA): a reader watching its writer ----
 * A writer holds the write lock (SEM_WRITE, taken with SEM_UNDO) for the
 * whole of its transfer, and the sync segment's w_state is ST_WRITING from
 * the start of data until the end-of-data block is marked filled.  A writer
 * that dies mid-transfer releases the lock (the kernel undoes it) but leaves
 * the transfer open: a reader sees an open transfer with no writer. */
int ipcbuf_get_writer_conn(ipcbuf_t *id) {
  if (!id || id->semid_connect < 0) return -1;
  const int v = semctl(id->semid_connect, SEM_WRITE, GETVAL);
  return v < 0 ? -1 : v == 0;
}

int ipcbuf_get_transfer_open(ipcbuf_t *id) {
  if (!id || !id->sync) return -1;
  return __atomic_load_n(&id->sync->w_state, __ATOMIC_ACQUIRE) != 0;
}

int ipcbuf_get_read_semaphore_count(ipcbuf_t *id) {
  return id && id->semid_connect >= 0 ? semctl(id->semid_connect, SEM_READ, GETVAL) : -1;
}

/* ---- positions within this process's transfer (id->xfer) ---- */

/* bytes of the transfer before block bufnum (@0x4049e0) */
uint64_t ipcbuf_tell(ipcbuf_t *id, uint64_t bufnum) {
  const ipcsync_t *s = id->sync;
  const uint64_t x = id->xfer;
  return bufnum > s->s_buf[x] ? (bufnum - s->s_buf[x]) * s->bufsz - s->s_byte[x] : 0;
}

/* bytes written into the open transfer (@0x404a10); -1 if not a writer */
int64_t ipcbuf_tell_write(ipcbuf_t *id) {
  if (!id || ipcbuf_eod(id) || !ipcbuf_is_writer(id)) return -1;
  return (int64_t)ipcbuf_tell(id, id->sync->w_buf);
}

/* bytes before the reader's (or viewer's) current block (@0x404aa0) */
int64_t ipcbuf_tell_read(ipcbuf_t *id) {
  if (!id || ipcbuf_eod(id)) return -1;
  if (id->state == ST_READING) return (int64_t)ipcbuf_tell(id, id->sync->r_bufs[id->iread]);
  if (id->state == ST_VIEWING) return (int64_t)ipcbuf_tell(id, ipcbuf_view_position(id));
  return 0;
}

/* bytes of this process's transfer so far: e_byte once it has ended
 * (@0x405280) */
uint64_t ipcbuf_get_write_byte_xfer(ipcbuf_t *id) {
  const ipcsync_t *s = id->sync;
  const uint64_t x = id->xfer;
  if (s->eod[x]) return s->e_byte[x];
  return ipcbuf_tell(id, s->w_buf);
}

/* w_buf while the writer is in this process's transfer, else e_byte of it
 * -- the field the binary reads (@0x4052e0) */
uint64_t ipcbuf_get_write_count_xfer(ipcbuf_t *id) {
  const ipcsync_t *s = id->sync;
  return s->w_xfer == id->xfer ? s->w_buf : s->e_byte[id->xfer];
}

/* soclock_buf = the block after the last transfer's end (0 before any),
 * the earliest start a deferred transfer may name (@0x4057a0) */
uint64_t ipcbuf_set_soclock_buf(ipcbuf_t *id) {
  const ipcsync_t *s = id->sync;
  id->soclock_buf = s->w_xfer ? s->e_buf[(s->w_xfer - 1) % IPCBUF_XFERS] + 1 : 0;
  return id->soclock_buf;
}

/* ---- ipcio ---- */

/* byte position in the transfer (@0x4068d0); 0 after a complaint if this
 * is not an open reader/viewer/writer */
uint64_t ipcio_tell(ipcio_t *ipc) {
  const char m = ipc->rdwrt & ~0x20;
  int64_t t = -1;
  if (m == 'R')
    t = ipcbuf_tell_read(&ipc->buf);
  else if (m == 'W')
    t = ipcbuf_tell_write(&ipc->buf);
  if (t < 0) {
    fprintf(stderr, "ipcio_tell: failed ipcbuf_tell mode=%c current=%li\n", ipc->rdwrt, (long)t);
    return 0;
  }
  return (uint64_t)t + ipc->bytes;
}

/* ipcio_seek (@0x406930): forward by reading (readers and viewers), back
 * only within the current block; whence SEEK_SET or SEEK_CUR */
int64_t ipcio_seek(ipcio_t *ipc, int64_t offset, int whence) {
  const uint64_t current = ipcio_tell(ipc);
  uint64_t target = (uint64_t)offset;
  if (whence == SEEK_CUR) target += ipcio_tell(ipc);
  if (current < target) {
    if (ipcio_read(ipc, NULL, target - current) < 0) {
      fprintf(stderr, "ipcio_seek: empty read %li bytes error\n", (long)(target - current));
      return -1;
    }
  } else if (current > target) {
    const uint64_t back = current - target;
    if (back > ipc->bytes) {
      fprintf(stderr, "ipcio_seek: %lu > max backwards %lu\n", (unsigned long)back, (unsigned long)ipc->bytes);
      return -1;
    }
    ipc->bytes -= back;
  }
  return (int64_t)ipcio_tell(ipc);
}

/* bytes of blocks not full for this process's reader (@0x406a00) */
int64_t ipcio_space_left(ipcio_t *ipc) {
  ipcbuf_t *b = &ipc->buf;
  return (int64_t)((ipcbuf_get_nbufs(b) - ipcbuf_get_nfull(b)) * ipcbuf_get_bufsz(b));
}

float ipcio_percent_full(ipcio_t *ipc) {  /* @0x406a40: a fraction, despite the name */
  ipcbuf_t *b = &ipc->buf;
  return (float)ipcbuf_get_nfull(b) / (float)ipcbuf_get_nbufs(b);
}

uint64_t ipcio_get_soclock_byte(ipcio_t *ipc) {  /* @0x406ad0 */
  return ipcbuf_get_bufsz(&ipc->buf) * ipc->buf.soclock_buf;
}

uint64_t ipcio_get_start_minimum(ipcio_t *ipc) {  /* @0x405af0 */
  return ipcbuf_get_bufsz(&ipc->buf) * ipcbuf_get_sod_minbuf(&ipc->buf);
}

int ipcio_zero_next_block(ipcio_t *ipc) {  /* @0x406450 */
  if (!ipc || ipc->rdwrt != 'W') {
    fprintf(stderr, "ipcio_open_block_write: ipc -> rdwrt != W\n");
    return -1;
  }
  return ipcbuf_zero_next_write(&ipc->buf);
}

/* ---- dada_hdu: see dada_ring.c; ascii_header: see ascii_header.c ---- */
