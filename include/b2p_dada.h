/*
 * include/b2p_dada.h -- the DADA ring-buffer / header / log surface the
 * reference's hosts are written against, re-implemented on SysV IPC.
 *
 * The reference links PSRDADA statically and
 * calls this subset: dada_hdu_*, ipcbuf_*, ipcio_*, ascii_header_*,
 * multilog*, fileread (diskdb.cu:24-130, capture.c:590-781,
 * paf_baseband2power.cu:82-84).  Same names, argument meaning and return
 * conventions (0 / pointer on success, -1 / NULL on error), so a host that
 * compiles against libpsrdada compiles against this and vice versa
 * (INTEGRATION.md).  Also provides the READER half the reference never
 * wrote (lock_read, open_block_read, ...; SURVEY.md Appendix A last item).
 *
 * Ring model (one writer, up to 8 readers):
 *  - a data ring at `key` and a header ring at `key+1` (dada_hdu_set_key,
 *    SURVEY.md 3.1); each ring = a small sync segment at its key plus one
 *    shared-memory segment per block (ids kept in the sync segment), and one
 *    semaphore set (clear / full-per-reader / lock semaphores);
 *  - a block filled with fewer than bufsz bytes ends the transfer (EOD),
 *    exactly as PSRDADA's ipcbuf_mark_filled does.  The EOD
 *    mark is kept per block, so a ring carries any number of transfers: a
 *    reader stops at its transfer's EOD block and takes the next transfer
 *    (header, then data) after unlock_read + lock_read;
 *  - wire compatibility with libpsrdada's own segment layout is NOT claimed:
 *    processes on both sides of a ring must use this library.
 */
#ifndef B2P_DADA_H
#define B2P_DADA_H

#include <stdint.h>
#include <stdio.h>
#include <sys/types.h>
#include <syslog.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DADA_DEFAULT_HEADER_SIZE 4096 /* HDR_SIZE, header_baseband2power.txt:3 */
#define IPCBUF_READERS 8

/* ---- multilog (paf_baseband2power.cu:82-84) ---- */
typedef struct multilog multilog_t;
multilog_t *multilog_open(const char *program_name, char syslog);
int multilog_add(multilog_t *log, FILE *fptr);
int multilog(multilog_t *log, int priority, const char *format, ...)
    __attribute__((format(printf, 3, 4)));
int multilog_close(multilog_t *log);

/* ---- ipcbuf: one ring of shared-memory blocks ---- */
typedef struct ipcsync ipcsync_t; /* shared state (opaque) */
typedef struct ipcbuf {
  int state;              /* 0 disconnected, 1 connected, 2 writer, 3 reader */
  key_t key;
  int syncid;             /* shm id of the sync segment */
  int semid;              /* semaphore set id */
  ipcsync_t *sync;
  char **buffer;          /* attached block addresses */
  uint64_t nbufs, bufsz;
  int iread;              /* reader slot, -1 if not a reader */
  uint64_t xfer_count;    /* blocks taken by this process */
  int cur_open;           /* blocks open (writer: 0/1; reader: up to read_depth) */
  uint64_t cur_index;     /* the block opened last */
  int read_depth;         /* reader: blocks it may hold at once (0 = 1, PSRDADA) */
  int eod_pending;        /* reader: the empty EOD block waits behind open ones */
  int eod_seen;           /* reader: took this transfer's EOD block (reset by lock_read) */
  int wrote_eod;          /* writer: this session ended its transfer (reset by lock_write) */
} ipcbuf_t;
#define IPCBUF_INIT {0, 0, -1, -1, NULL, NULL, 0, 0, -1, 0, 0, 0, 0, 0, 0, 0}

int ipcbuf_create(ipcbuf_t *id, key_t key, uint64_t nbufs, uint64_t bufsz, unsigned n_readers);
/* device_id >= 0: blocks in that GPU's memory, owned by a holder process and
 * shared through HIP IPC handles (PSRDADA ipcbuf_create_work; the sync
 * segment's on_device_id).  -1: SysV shared memory. */
int ipcbuf_create_work(ipcbuf_t *id, key_t key, uint64_t nbufs, uint64_t bufsz,
                       unsigned n_readers, int device_id);
int ipcbuf_connect(ipcbuf_t *id, key_t key);
int ipcbuf_disconnect(ipcbuf_t *id);
int ipcbuf_destroy(ipcbuf_t *id);
int ipcbuf_lock_write(ipcbuf_t *id);
int ipcbuf_unlock_write(ipcbuf_t *id);
int ipcbuf_lock_read(ipcbuf_t *id);
int ipcbuf_unlock_read(ipcbuf_t *id);
char *ipcbuf_get_next_write(ipcbuf_t *id);
int ipcbuf_mark_filled(ipcbuf_t *id, uint64_t nbytes);
char *ipcbuf_get_next_read(ipcbuf_t *id, uint64_t *bytes);
int ipcbuf_mark_cleared(ipcbuf_t *id); /* releases the OLDEST block this reader holds */
/* Extension (not in PSRDADA): let a reader hold up to `depth` blocks at once,
 * so a GPU consumer can launch on block k+1 before block k's kernel has
 * finished with it.  ipcbuf_get_next_read / ipcio_open_block_read take the
 * next block; ipcbuf_mark_cleared / ipcio_close_block_read release the oldest. */
int ipcbuf_set_read_depth(ipcbuf_t *id, int depth);
int ipcbuf_enable_sod(ipcbuf_t *id, uint64_t start_buf, uint64_t start_byte);
int ipcbuf_disable_sod(ipcbuf_t *id);
int ipcbuf_enable_eod(ipcbuf_t *id); /* end the transfer with an empty block */
int ipcbuf_eod(ipcbuf_t *id);        /* 1 once this reader has reached EOD */
int ipcbuf_sod(ipcbuf_t *id);
uint64_t ipcbuf_get_bufsz(ipcbuf_t *id);
uint64_t ipcbuf_get_nbufs(ipcbuf_t *id);
uint64_t ipcbuf_get_nreaders(ipcbuf_t *id);
/* address of block i (for device registration; PSRDADA's
 * dada_cuda_dbregister walks the same list) */
char *ipcbuf_get_buffer(ipcbuf_t *id, uint64_t i);
/* blocks written / cleared so far (monitoring, dada_dbmonitor role) */
uint64_t ipcbuf_get_write_count(ipcbuf_t *id);
/* -1 for a host ring; else the HIP device holding the blocks, whose
 * addresses (ipcbuf_get_next_read/write, ipcio_open_block_*) are device
 * pointers valid in this process.  Writers finish their kernels before
 * ipcbuf_mark_filled; readers finish theirs before ipcbuf_mark_cleared. */
int ipcbuf_get_device(ipcbuf_t *id);
/* copy host or device memory into / out of a block of either kind
 * (memcpy, or a synchronous hipMemcpy for a device ring) */
int ipcbuf_copy_in(ipcbuf_t *id, char *block, const void *src, uint64_t n);
int ipcbuf_copy_out(ipcbuf_t *id, void *dst, const char *block, uint64_t n);
uint64_t ipcbuf_get_read_count(ipcbuf_t *id, int iread);
/* Extension: make every ring wait of this process (a reader waiting for a
 * block, a writer waiting for a free one) give up -- the call fails, e.g.
 * ipcio_open_block_read returns NULL -- instead of resuming, once a signal
 * has interrupted it.  Async-signal-safe: meant for a SIGINT/SIGTERM
 * handler, so a stage stops between blocks and ends its output transfer
 * (unlock_write) cleanly instead of dying mid-ring. */
void dada_interrupt_waits(void);

/* ---- ipcio: block-level streaming over an ipcbuf ---- */
typedef struct ipcio {
  ipcbuf_t buf;
  char *curbuf;
  uint64_t curbufsz;
  int rdwrt; /* 'R' or 'W' */
} ipcio_t;
#define IPCIO_INIT {IPCBUF_INIT, NULL, 0, 0}

int ipcio_open(ipcio_t *ipc, char rdwrt);
int ipcio_close(ipcio_t *ipc); /* writer: ends the transfer (EOD) */
char *ipcio_open_block_write(ipcio_t *ipc, uint64_t *block_id);
int ipcio_close_block_write(ipcio_t *ipc, uint64_t bytes);
/* NULL at end of data (writer signalled EOD and every block was read) */
char *ipcio_open_block_read(ipcio_t *ipc, uint64_t *curbufsz, uint64_t *block_id);
ssize_t ipcio_close_block_read(ipcio_t *ipc, uint64_t bytes); /* PSRDADA's type */

/* ---- dada_hdu: data ring at key + header ring at key+1 ---- */
typedef struct dada_hdu {
  multilog_t *log;
  ipcio_t *data_block;
  ipcbuf_t *header_block;
  char *header;
  uint64_t header_size;
  key_t data_block_key;
  key_t header_block_key;
} dada_hdu_t;

dada_hdu_t *dada_hdu_create(multilog_t *log);
void dada_hdu_set_key(dada_hdu_t *hdu, key_t key);
int dada_hdu_connect(dada_hdu_t *hdu);
int dada_hdu_disconnect(dada_hdu_t *hdu);
void dada_hdu_destroy(dada_hdu_t *hdu);
int dada_hdu_lock_write(dada_hdu_t *hdu);
int dada_hdu_unlock_write(dada_hdu_t *hdu);
int dada_hdu_lock_read(dada_hdu_t *hdu);
int dada_hdu_unlock_read(dada_hdu_t *hdu);
/* reader: wait for the next header block and copy it into hdu->header */
int dada_hdu_open_read(dada_hdu_t *hdu);

/* ring creation / removal (the dada_db tool, paf-baseband2power.py:114-115,
 * :129-130).  Header ring: hdr_nbufs blocks of hdr_bufsz bytes. */
int dada_db_create(key_t key, uint64_t nbufs, uint64_t bufsz, unsigned n_readers,
                   uint64_t hdr_nbufs, uint64_t hdr_bufsz);
/* as dada_db_create, data blocks on HIP device device_id (-1: host); the
 * header ring stays in host memory.  Removes both rings and stops the
 * holder when destroyed. */
int dada_db_create_work(key_t key, uint64_t nbufs, uint64_t bufsz, unsigned n_readers,
                        uint64_t hdr_nbufs, uint64_t hdr_bufsz, int device_id);
int dada_db_destroy(key_t key);

/* ---- ASCII header (ascii_header_set at capture.c:758-778) ---- */
/* returns the number of items scanned (>= 1), or -1 if the key is absent */
int ascii_header_get(const char *header, const char *keyword, const char *format, void *result);
/* replaces the value of an existing key or appends "KEY value"; 0 / -1 */
int ascii_header_set(char *header, const char *keyword, const char *format, ...)
    __attribute__((format(printf, 3, 4)));
int ascii_header_del(char *header, const char *keyword);

/* read up to bufsz bytes of a file into buffer, NUL-terminated (futils) */
int fileread(const char *filename, char *buffer, unsigned bufsz); /* bytes read, -1 on error */

#ifdef __cplusplus
}
#endif
#endif /* B2P_DADA_H */
