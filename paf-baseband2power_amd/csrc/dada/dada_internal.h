/* dada_internal.h -- shared layout of the ring's sync segment (private to
 * libpafdada: dada_ring.c, dada_device.c). */
#ifndef B2P_DADA_INTERNAL_H
#define B2P_DADA_INTERNAL_H

#include <stdint.h>

#include "b2p_dada.h"

#define SYNC_MAGIC 0x50414642u /* "PAFB" */
#define SYNC_VERSION 3u
#define DEV_HANDLE_BYTES 64 /* HIP_IPC_HANDLE_SIZE, hip_runtime_api.h */

/* semaphore set layout */
#define SEM_CLEAR 0
#define SEM_WLOCK 1
#define SEM_FULL(r) (2 + (r))
#define SEM_RLOCK(r) (2 + IPCBUF_READERS + (r))
#define NSEMS (2 + 2 * IPCBUF_READERS)

struct ipcsync {
  uint32_t magic, version;
  uint64_t nbufs, bufsz;
  uint32_t n_readers;
  int32_t semid;
  uint64_t w_count;                  /* blocks filled so far            */
  uint64_t r_count[IPCBUF_READERS];  /* blocks cleared by each reader   */
  int32_t sod;
  int32_t pad;
  uint64_t s_buf, s_byte;
  int32_t on_device_id;              /* -1: blocks are SysV shm; else a HIP device */
  int32_t holder_pid;                /* device rings: process owning the blocks */
  int32_t holder_state;              /* 0 starting, 1 serving, 2 gone    */
  int32_t pad2;
  /* followed by: int32 shmid[nbufs]; uint32 clear_cnt[nbufs];
   *              uint32 eod[nbufs] (1: the block ends its transfer);
   *              uint64 nbytes[nbufs] (8-aligned);
   *              uint8 handle[nbufs][DEV_HANDLE_BYTES] (device rings)    */
};

static inline int32_t *sync_shmids(ipcsync_t *s) { return (int32_t *)(s + 1); }
static inline uint32_t *sync_clear(ipcsync_t *s) { return (uint32_t *)(sync_shmids(s) + s->nbufs); }
static inline uint32_t *sync_eod(ipcsync_t *s) { return sync_clear(s) + s->nbufs; }
static inline uint64_t *sync_nbytes(ipcsync_t *s) {
  uintptr_t p = (uintptr_t)(sync_eod(s) + s->nbufs);
  return (uint64_t *)((p + 7) & ~(uintptr_t)7);
}
static inline unsigned char *sync_handles(ipcsync_t *s) {
  return (unsigned char *)(sync_nbytes(s) + s->nbufs);
}
static inline size_t sync_size(uint64_t nbufs) {
  return sizeof(ipcsync_t) + nbufs * (sizeof(int32_t) + 2 * sizeof(uint32_t)) + 8 +
         nbufs * sizeof(uint64_t) + nbufs * DEV_HANDLE_BYTES;
}

/* dada_device.c: HIP reached through dlopen, so libpafdada loads without ROCm */
int dev_create_blocks(int syncid, ipcsync_t *s, int device); /* fork the holder */
int dev_stop_holder(ipcsync_t *s);
int dev_open_blocks(ipcbuf_t *id);
void dev_close_blocks(ipcbuf_t *id);
int dev_copy(void *dst, const void *src, uint64_t n); /* hipMemcpyDefault */

#endif
