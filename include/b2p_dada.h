/*
 * include/b2p_dada.h -- the DADA ring-buffer / header / log surface the
 * reference's hosts are written against, re-implemented on SysV IPC.
 *
 * The reference links PSRDADA statically and
 * calls this subset: dada_hdu_*, ipcbuf_*, ipcio_*, ascii_header_*,
 * multilog*, fileread (diskdb.cu:24-130, capture.c:590-781,
 * paf_baseband2power.cu:82-84).  Same names, prototypes, struct layouts and
 * return conventions as that libpsrdada (its debug info, recorded in
 * tests/golden/psrdada_abi.json by tools/psrdada_dwarf.py), so a host
 * compiled against either library's headers links against the other.
 * Also the READER half the reference never wrote (lock_read,
 * open_block_read, ...; SURVEY.md Appendix A last item).
 *
 * Rings are PSRDADA rings on the wire (csrc/dada/dada_internal.h): the same
 * sync segment, key schedule, semaphore sets and writer/reader protocol, so
 * libpafdada and libpsrdada processes share a ring (one writer, up to 8
 * readers; data ring at `key`, header ring at `key+1`; a block marked filled
 * with fewer than bufsz bytes, or the 0-byte block ipcio_close appends after
 * a full one, ends the transfer; up to 8 transfers in flight).
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
/* one "[date-time] ERR: message" line to a stream, as multilog writes it */
int multilog_fprintf(FILE *stream, int priority, const char *format, ...)
    __attribute__((format(printf, 3, 4)));

/* ---- SysV helpers (ipcutil) ---- */
void *ipc_alloc(key_t key, size_t size, int flag, int *shmid); /* shmget + shmat, NULL on error */
int ipc_semop(int semid, short int num, short int op, short int flag); /* one semop, 0 / -1 */

/* ---- ipcbuf: one ring of shared-memory blocks ---- */
typedef struct ipcsync ipcsync_t; /* the shared sync segment (dada_internal.h) */
typedef struct {                  /* PSRDADA's ipcbuf_t, 104 B */
  int state;                      /* DISCON 0, VIEWER 1, WRITER 2, WRITING 3, WCHANGE 4,
                                     READER 5, READING 6, RSTOP 7 (end of data),
                                     VIEWING 8, VSTOP 9 */
  int syncid;
  int semid_connect;
  int *semid_data;
  int *shmid;
  ipcsync_t *sync;
  char **buffer;                  /* block addresses in this process */
  void **shm_addr;
  char *count;                    /* in the sync segment: fills not yet cleared, per block */
  key_t *shmkey;                  /* in the sync segment */
  uint64_t viewbuf;
  uint64_t xfer;
  uint64_t soclock_buf;
  int iread;                      /* reader slot, -1 if not a reader */
} ipcbuf_t;
#define IPCBUF_INIT {0, -1, -1, NULL, NULL, NULL, NULL, NULL, NULL, NULL, 0, 0, 0, -1}

int ipcbuf_create(ipcbuf_t *id, key_t key, uint64_t nbufs, uint64_t bufsz, unsigned n_readers);
/* device_id >= 0: blocks in that GPU's memory, owned by a holder process and
 * shared through HIP IPC handles (PSRDADA's ipcbuf_create_work and
 * on_device_id).  -1: SysV shared memory. */
int ipcbuf_create_work(ipcbuf_t *id, key_t key, uint64_t nbufs, uint64_t bufsz,
                       unsigned n_readers, int device_id);
int ipcbuf_connect(ipcbuf_t *id, key_t key);
int ipcbuf_disconnect(ipcbuf_t *id);
int ipcbuf_destroy(ipcbuf_t *id);
/* the semaphore sets and blocks of a ring whose sync segment is attached
 * (a step of ipcbuf_connect; n_readers is not used) */
int ipcbuf_get(ipcbuf_t *id, int flag, int n_readers);
int ipcbuf_lock_write(ipcbuf_t *id);  /* waits for the writer lock */
int ipcbuf_unlock_write(ipcbuf_t *id);
int ipcbuf_lock_read(ipcbuf_t *id);   /* waits for a free reader slot */
int ipcbuf_unlock_read(ipcbuf_t *id);
char *ipcbuf_get_next_write(ipcbuf_t *id);
int ipcbuf_mark_filled(ipcbuf_t *id, uint64_t nbytes);
/* a reader takes its next block; a viewer (ipcio_open 'r') is given the
 * next block the writer fills, without taking it */
char *ipcbuf_get_next_read(ipcbuf_t *id, uint64_t *bytes);
char *ipcbuf_get_next_read_work(ipcbuf_t *id, uint64_t *bytes, int flag); /* flag: semop flags */
char *ipcbuf_get_next_readable(ipcbuf_t *id, uint64_t *bytes);
int ipcbuf_mark_cleared(ipcbuf_t *id); /* releases the OLDEST block this reader holds */
/* Extension (not in PSRDADA): let a reader hold up to `depth` blocks at once,
 * so a GPU consumer can launch on block k+1 before block k's kernel has
 * finished with it.  ipcbuf_get_next_read / ipcio_open_block_read take the
 * next block; ipcbuf_mark_cleared / ipcio_close_block_read release the
 * oldest.  The shared state moves exactly as for a reader taking the blocks
 * one at a time, so writers and other readers see a plain PSRDADA reader. */
int ipcbuf_set_read_depth(ipcbuf_t *id, int depth);
int ipcbuf_enable_sod(ipcbuf_t *id, uint64_t start_buf, uint64_t start_byte);
int ipcbuf_disable_sod(ipcbuf_t *id);
int ipcbuf_enable_eod(ipcbuf_t *id); /* the next mark_filled ends the transfer */
int ipcbuf_eod(ipcbuf_t *id);        /* 1 once this reader has cleared its transfer's EOD block */
int ipcbuf_sod(ipcbuf_t *id);
/* reader at EOD: ready for the next transfer.  writer: once every block is
 * cleared and every transfer acknowledged, the ring is as created */
int ipcbuf_reset(ipcbuf_t *id);
int ipcbuf_hard_reset(ipcbuf_t *id); /* the same, without waiting for anyone */
int ipcbuf_zero_next_write(ipcbuf_t *id); /* writer: zero the block after this one once free */
int ipcbuf_lock(ipcbuf_t *id);       /* pin the segments in RAM (SHM_LOCK; dada_db -l) */
int ipcbuf_unlock(ipcbuf_t *id);
int ipcbuf_page(ipcbuf_t *id);       /* zero every host block (dada_db -p) */
char ipcbuf_is_writer(ipcbuf_t *id);
char ipcbuf_is_writing(ipcbuf_t *id);
char ipcbuf_is_reader(ipcbuf_t *id);
uint64_t ipcbuf_get_bufsz(ipcbuf_t *id);
uint64_t ipcbuf_get_nbufs(ipcbuf_t *id);
int ipcbuf_get_nreaders(ipcbuf_t *id);
uint64_t ipcbuf_get_write_count(ipcbuf_t *id); /* blocks filled so far */
uint64_t ipcbuf_get_write_index(ipcbuf_t *id);
uint64_t ipcbuf_get_read_count(ipcbuf_t *id);  /* this reader's (slot 0's) blocks cleared */
uint64_t ipcbuf_get_read_count_iread(ipcbuf_t *id, unsigned iread);
uint64_t ipcbuf_get_read_index(ipcbuf_t *id);
/* semaphore counts of reader iread (iread < 0: see dada_query.c) */
uint64_t ipcbuf_get_nfull(ipcbuf_t *id);   /* blocks filled, not yet taken */
uint64_t ipcbuf_get_nfull_iread(ipcbuf_t *id, int iread);
uint64_t ipcbuf_get_nclear(ipcbuf_t *id);  /* blocks cleared, not yet reused */
uint64_t ipcbuf_get_nclear_iread(ipcbuf_t *id, int iread);
uint64_t ipcbuf_get_sodack(ipcbuf_t *id);
uint64_t ipcbuf_get_sodack_iread(ipcbuf_t *id, int iread);
uint64_t ipcbuf_get_eodack(ipcbuf_t *id);
uint64_t ipcbuf_get_eodack_iread(ipcbuf_t *id, int iread);
int ipcbuf_get_reader_conn(ipcbuf_t *id);
int ipcbuf_get_reader_conn_iread(ipcbuf_t *id, int iread);
int ipcbuf_get_read_semaphore_count(ipcbuf_t *id); /* free reader slots */
/* Extensions (not in PSRDADA), for a reader watching its writer: 1 if a
 * writer holds the ring's write lock, 0 if none, -1 on error; 1 while a
 * transfer is open (its start of data written, its end-of-data block not
 * yet), 0 if not, -1 on error.  A writer that died mid-transfer shows as an
 * open transfer with no writer (its lock is undone by the kernel); a new
 * writer may still take the lock and go on with that transfer. */
int ipcbuf_get_writer_conn(ipcbuf_t *id);
int ipcbuf_get_transfer_open(ipcbuf_t *id);
/* byte positions in this process's transfer */
uint64_t ipcbuf_tell(ipcbuf_t *id, uint64_t bufnum);
int64_t ipcbuf_tell_write(ipcbuf_t *id);
int64_t ipcbuf_tell_read(ipcbuf_t *id);
uint64_t ipcbuf_get_write_byte_xfer(ipcbuf_t *id);
uint64_t ipcbuf_get_write_count_xfer(ipcbuf_t *id);
uint64_t ipcbuf_get_sod_minbuf(ipcbuf_t *id);  /* earliest block a start of data may name */
uint64_t ipcbuf_set_soclock_buf(ipcbuf_t *id); /* = the block after the last transfer's end */
/* address of block i (for device registration; PSRDADA's
 * dada_cuda_dbregister walks the same list) -- extension */
char *ipcbuf_get_buffer(ipcbuf_t *id, uint64_t i);
/* -1 for a host ring; else the HIP device holding the blocks, whose
 * addresses (ipcbuf_get_next_read/write, ipcio_open_block_*) are device
 * pointers valid in this process.  Writers finish their kernels before
 * ipcbuf_mark_filled; readers finish theirs before ipcbuf_mark_cleared. */
int ipcbuf_get_device(ipcbuf_t *id);
/* extension: copy host or device memory into / out of a block of either
 * kind (memcpy, or a synchronous hipMemcpy for a device ring) */
int ipcbuf_copy_in(ipcbuf_t *id, char *block, const void *src, uint64_t n);
int ipcbuf_copy_out(ipcbuf_t *id, void *dst, const char *block, uint64_t n);
/* extension: why this thread's last device-ring call failed (hipMemcpy,
 * hipIpcOpenMemHandle ...: the HIP call, its error string and code); ""
 * when none has */
const char *dada_device_error(void);
/* Extension: make every ring wait of this process (a reader waiting for a
 * block, a writer waiting for a free one) give up -- the call fails, e.g.
 * ipcio_open_block_read returns NULL -- instead of resuming, once a signal
 * has interrupted it.  Async-signal-safe: meant for a SIGINT/SIGTERM
 * handler, so a stage stops between blocks and ends its output transfer
 * (unlock_write) cleanly instead of dying mid-ring; also callable from any
 * thread (the flag is a lock-free atomic), e.g. when one input ring failed
 * and the threads waiting on the others must be woken. */
void dada_interrupt_waits(void);

/* ---- ipcio: block-level streaming over an ipcbuf ---- */
typedef struct { /* PSRDADA's ipcio_t, 152 B */
  ipcbuf_t buf;
  char *curbuf;
  uint64_t curbufsz;
  uint64_t bytes;
  char rdwrt; /* 'R', 'r' (viewer), 'W', 'w' (writer, start of data deferred) or 0 */
  char marked_filled;
  char sod_pending;
  uint64_t sod_buf;
  uint64_t sod_byte;
} ipcio_t;
#define IPCIO_INIT {IPCBUF_INIT, NULL, 0, 0, 0, 0, 0, 0, 0}

void ipcio_init(ipcio_t *ipc);
int ipcio_create(ipcio_t *ipc, key_t key, uint64_t nbufs, uint64_t bufsz, unsigned num_read);
int ipcio_create_work(ipcio_t *ipc, key_t key, uint64_t nbufs, uint64_t bufsz, unsigned num_read,
                      int device_id);
int ipcio_destroy(ipcio_t *ipc);
int ipcio_connect(ipcio_t *ipc, key_t key);
int ipcio_disconnect(ipcio_t *ipc);
/* 'W' writer, 'w' writer with the start of data deferred, 'R' reader, 'r' viewer */
int ipcio_open(ipcio_t *ipc, char rdwrt);
int ipcio_is_open(ipcio_t *ipc);
int ipcio_close(ipcio_t *ipc); /* writer: ends the open transfer (EOD) and unlocks */
int ipcio_stop(ipcio_t *ipc);  /* writer: ends the open transfer, keeps the lock ('w') */
int ipcio_stop_close(ipcio_t *ipc, char unlock);
int ipcio_start(ipcio_t *ipc, uint64_t byte); /* 'w' writer: a transfer from stream byte `byte` */
int ipcio_check_pending_sod(ipcio_t *ipc);
uint64_t ipcio_tell(ipcio_t *ipc);
int64_t ipcio_seek(ipcio_t *ipc, int64_t offset, int whence);
int64_t ipcio_space_left(ipcio_t *ipc);
float ipcio_percent_full(ipcio_t *ipc); /* nfull / nbufs */
uint64_t ipcio_get_soclock_byte(ipcio_t *ipc);
uint64_t ipcio_get_start_minimum(ipcio_t *ipc);
int ipcio_zero_next_block(ipcio_t *ipc);
char *ipcio_open_block_write(ipcio_t *ipc, uint64_t *block_id);
ssize_t ipcio_update_block_write(ipcio_t *ipc, uint64_t bytes);
ssize_t ipcio_close_block_write(ipcio_t *ipc, uint64_t bytes);
/* NULL once the reader is at end of data; the block that ends a transfer
 * may hold 0 bytes (the writer's ipcio_close after a full block) */
char *ipcio_open_block_read(ipcio_t *ipc, uint64_t *curbufsz, uint64_t *block_id);
ssize_t ipcio_close_block_read(ipcio_t *ipc, uint64_t bytes);
ssize_t ipcio_write(ipcio_t *ipc, char *ptr, size_t bytes);
ssize_t ipcio_read(ipcio_t *ipc, char *ptr, size_t bytes); /* < bytes at end of data */

/* ---- dada_hdu: data ring at key + header ring at key+1 ---- */
typedef struct dada_hdu { /* PSRDADA's dada_hdu_t, 48 B */
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
int dada_hdu_lock_write_spec(dada_hdu_t *hdu, char writemode); /* 'W', or 'w' (ipcio_start later) */
int dada_hdu_unlock_write(dada_hdu_t *hdu);
int dada_hdu_lock_read(dada_hdu_t *hdu);
int dada_hdu_unlock_read(dada_hdu_t *hdu); /* releases the header block dada_hdu_open took */
/* reader: wait for the next header block and copy it into hdu->header
 * (PSRDADA's dada_hdu_open; dada_hdu_open_read is the same call) */
int dada_hdu_open(dada_hdu_t *hdu);
int dada_hdu_open_read(dada_hdu_t *hdu);
int dada_hdu_open_view(dada_hdu_t *hdu);  /* view the data ring (ipcio 'r') */
int dada_hdu_close_view(dada_hdu_t *hdu);
char **dada_hdu_db_addresses(dada_hdu_t *hdu, uint64_t *nbufs, uint64_t *bufsz);
char **dada_hdu_hb_addresses(dada_hdu_t *hdu, uint64_t *nbufs, uint64_t *bufsz);

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

/* Extension: the holder of a GPU-resident ring, read from block 0's segment
 * without opening any block (dada_db -g; SURVEY.md 8f rank 3 -- PSRDADA's
 * ipc_alloc_cuda has no holder to ask).  export_retries counts ring blocks
 * whose HIP IPC export was refused once and exported after a retry (0 on a
 * healthy ring; the GPU tests assert it for every ring they make);
 * primer_refused is 1 when the holder's first allocation -- a 2 MiB primer
 * no block uses -- was refused export (counted, harmless).  0, or -1 with
 * errno ENOENT (no ring / no holder record) or ENODEV (a host ring). */
typedef struct {
  int device;
  int holder_pid;
  int holder_state; /* 0 starting, 1 serving, 2 gone (blocks freed) */
  int importers;    /* processes with the blocks open, as the holder last counted */
  int export_retries;
  int primer_refused;
} dada_device_info_t;
int dada_device_ring_info(key_t key, dada_device_info_t *info);

/* ---- ASCII header (ascii_header_set at capture.c:758-778) ---- */
/* returns the number of items scanned (>= 1), or -1 if the key is absent */
int ascii_header_get(const char *header, const char *keyword, const char *format, ...)
    __attribute__((format(scanf, 3, 4)));
/* replaces the value of an existing key or appends "KEY value"; 0 / -1 */
int ascii_header_set(char *header, const char *keyword, const char *format, ...)
    __attribute__((format(printf, 3, 4)));
int ascii_header_del(char *header, const char *keyword);
char *ascii_header_find(const char *header, const char *keyword); /* the keyword, or NULL */
size_t ascii_header_get_size(char *filename); /* HDR_SIZE of a DADA file, (size_t)-1 on error */
size_t ascii_header_get_size_fd(int fd);

/* read up to bufsz bytes of a file into buffer, NUL-terminated (futils) */
long fileread(const char *filename, char *buffer, unsigned bufsz); /* bytes read, -1 on error */

#ifdef __cplusplus
}
#endif
#endif /* B2P_DADA_H */
