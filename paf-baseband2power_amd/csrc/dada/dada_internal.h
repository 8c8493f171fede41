/* dada_internal.h -- PSRDADA's shared ring layout, as libpafdada writes it
 * (private to dada_ring.c, dada_device.c).
 *
 * Everything here is the wire format of the reference's statically linked
 * libpsrdada, read off its debug info and disassembly
 * (tools/psrdada_dwarf.py -> tests/golden/psrdada_abi.json, SURVEY.md
 * Appendix A), so a ring made by either library is used by the other:
 *
 *  - sync segment at `key`: ipcsync_t (520 B) + char count[nbufs] + key_t
 *    shmkey[nbufs]  (ipcsync_get @0x402fe0: size 0x208 + 5*nbufs);
 *  - semaphores: a 2-set at key + 0x10000 (WRITE lock, READ slots) and one
 *    5-set per reader at key + 0x10000*(2+r) (SODACK, EODACK, FULL, CLEAR,
 *    READER_CONN)  (ipcbuf_create_work @0x40344a-0x403598);
 *  - block i: a segment at key + 0x10000*(10+i) of bufsz bytes, or, for a
 *    device ring (on_device_id >= 0), of a 64-B IPC memory handle
 *    (ipc_alloc_cuda @0x407ede).
 */
#ifndef B2P_DADA_INTERNAL_H
#define B2P_DADA_INTERNAL_H

#include <stddef.h>
#include <stdint.h>

#include "b2p_dada.h"

#define IPCBUF_XFERS 8

/* ipcbuf_t.state (ipcbuf_lock_write @0x403b25, ipcbuf_lock_read @0x4044e5,
 * ipcbuf_mark_cleared @0x404bf6, ipcbuf_eod @0x405247) */
enum {
  ST_DISCON = 0,
  ST_VIEWER = 1,
  ST_WRITER = 2,  /* locked, start of data disabled */
  ST_WRITING = 3, /* a transfer is open */
  ST_WCHANGE = 4, /* the next write starts / the next mark_filled ends a transfer */
  ST_READER = 5,
  ST_READING = 6,
  ST_RSTOP = 7, /* this reader reached its transfer's end of data */
  ST_VIEWING = 8,
  ST_VSTOP = 9
};

/* semaphore numbers */
enum { SEM_WRITE = 0, SEM_READ = 1, NSEM_CONNECT = 2 };
enum { SEM_SODACK = 0, SEM_EODACK = 1, SEM_FULL = 2, SEM_CLEAR = 3, SEM_READER_CONN = 4, NSEM_DATA = 5 };

#define KEY_STEP 0x10000
static inline key_t key_connect(key_t k) { return k + KEY_STEP; }
static inline key_t key_data(key_t k, int r) { return k + KEY_STEP * (2 + r); }
static inline key_t key_block(key_t k, uint64_t i) { return k + KEY_STEP * (10 + (key_t)i); }

/* the shared sync segment: PSRDADA's ipcsync_t, byte for byte */
struct ipcsync {
  key_t semkey_connect;
  key_t semkey_data[IPCBUF_READERS];
  uint64_t nbufs;
  uint64_t bufsz;
  uint64_t w_buf;  /* blocks marked filled so far */
  int w_state;     /* 0, or ST_WRITING while a transfer is open */
  uint64_t w_xfer; /* transfers ended so far */
  uint64_t r_bufs[IPCBUF_READERS];
  int r_states[IPCBUF_READERS];
  uint64_t r_xfers[IPCBUF_READERS];
  unsigned n_readers;
  uint64_t s_buf[IPCBUF_XFERS]; /* start of data of transfer x % 8: block, byte */
  uint64_t s_byte[IPCBUF_XFERS];
  char eod[IPCBUF_XFERS];
  uint64_t e_buf[IPCBUF_XFERS]; /* end of data of transfer x % 8: block, byte */
  uint64_t e_byte[IPCBUF_XFERS];
  int on_device_id;
};

_Static_assert(sizeof(struct ipcsync) == 520, "ipcsync_t is 520 B (psrdada_abi.json)");
_Static_assert(offsetof(struct ipcsync, nbufs) == 40, "ipcsync_t.nbufs");
_Static_assert(offsetof(struct ipcsync, w_xfer) == 72, "ipcsync_t.w_xfer");
_Static_assert(offsetof(struct ipcsync, r_states) == 144, "ipcsync_t.r_states");
_Static_assert(offsetof(struct ipcsync, n_readers) == 240, "ipcsync_t.n_readers");
_Static_assert(offsetof(struct ipcsync, eod) == 376, "ipcsync_t.eod");
_Static_assert(offsetof(struct ipcsync, on_device_id) == 512, "ipcsync_t.on_device_id");
_Static_assert(sizeof(ipcbuf_t) == 104 && offsetof(ipcbuf_t, iread) == 96, "ipcbuf_t");
_Static_assert(sizeof(ipcio_t) == 152 && offsetof(ipcio_t, sod_byte) == 144, "ipcio_t");
_Static_assert(sizeof(dada_hdu_t) == 48 && offsetof(dada_hdu_t, header_block_key) == 44, "dada_hdu_t");

static inline size_t sync_size(uint64_t nbufs) { return sizeof(ipcsync_t) + 5 * (size_t)nbufs; }

/* a device ring's block segment: the 64-B HIP IPC handle PSRDADA's layout
 * reserves for it; block 0's segment carries the holder process after it
 * (a libpafdada extension: the segment is larger, the handle unchanged).
 *
 * Ordering rule of a device ring (dada_device.c): every process that opened
 * the blocks' IPC handles stays attached to block 0's segment until it has
 * closed them (free_local: dev_close_blocks, then shmdt), and the holder
 * frees the blocks only once no such process is attached -- counted by the
 * kernel as shm_nattch of block 0's segment, less the holder itself.  A
 * killed importer detaches when it dies, so the count needs no cooperation
 * to come down; and nothing else stays attached: a destroyer attaches only
 * for a moment per look at the holder's state (dev_stop_holder), so a
 * destroyer that dies mid-wait leaves nothing behind, and a look that
 * meets the holder's count makes it wait one more tick, never free early.
 *
 * The holder also records how its IPC exports went (dada_device_ring_info):
 * export_retries -- ring blocks whose first export was refused and that
 * were exported after a retry (0 expected; a test asserts it); and
 * primer_refused -- its first allocation, the 2 MiB primer no block uses,
 * was refused (the refusal that probes saw on first allocations, counted,
 * allowed). */
#define DEV_HANDLE_BYTES 64
typedef struct {
  unsigned char handle[DEV_HANDLE_BYTES];
  int32_t holder_pid;
  int32_t holder_state;   /* 0 starting, 1 serving, 2 gone */
  int32_t importers;      /* last count the holder saw (diagnostics) */
  int32_t export_retries; /* ring blocks exported only after a retry */
  int32_t primer_refused; /* 1: the primer allocation's export was refused */
  int32_t reserved;
} dev_seg_t;

/* dada_device.c: HIP reached through dlopen, so libpafdada loads without ROCm */
/* a viewer's block position (dada_ring.c: the low bits of viewbuf) */
uint64_t ipcbuf_view_position(const ipcbuf_t *id);

int dev_create_blocks(ipcbuf_t *id, int device); /* fork the holder, fill the handles */
/* stop the holder of the ring whose block 0 is segment seg0_id and wait
 * (<= 10 s) until it has freed the blocks; -1 with errno EBUSY (text in
 * dada_device_error) while importers stay attached -- the holder then frees
 * the blocks when the last one detaches */
int dev_stop_holder(int seg0_id);
/* copy block 0's segment, attached read-only for the copy only; -1 once the
 * segment is gone */
int dev_look_seg0(int seg0_id, dev_seg_t *out);
int dev_open_blocks(ipcbuf_t *id);
void dev_close_blocks(ipcbuf_t *id);
int dev_copy(void *dst, const void *src, uint64_t n, int into_block); /* hipMemcpyDefault; into_block: finished on return */
int dev_zero(void *dst, uint64_t n);                  /* hipMemset, synchronised */

#endif
