/* declarations only -- see README.txt.  ipcbuf_t as laid out in the
 * reference's libpsrdada (its DWARF: tests/golden/psrdada_abi.json, 104 B). */
#ifndef __DADA_IPCBUF_H
#define __DADA_IPCBUF_H
#include <stdint.h>
#include <sys/types.h>
typedef struct ipcsync_t ipcsync_t;
typedef struct {
  int state;
  int syncid;
  int semid_connect;
  int *semid_data;
  int *shmid;
  ipcsync_t *sync;
  char **buffer;
  void **shm_addr;
  char *count;
  key_t *shmkey;
  uint64_t viewbuf;
  uint64_t xfer;
  uint64_t soclock_buf;
  int iread;
} ipcbuf_t;
char *ipcbuf_get_next_write(ipcbuf_t *id);
int ipcbuf_mark_filled(ipcbuf_t *id, uint64_t nbytes);
char *ipcbuf_get_next_read(ipcbuf_t *id, uint64_t *bytes);
int ipcbuf_mark_cleared(ipcbuf_t *id);
int ipcbuf_enable_sod(ipcbuf_t *id, uint64_t start_buf, uint64_t start_byte);
int ipcbuf_disable_sod(ipcbuf_t *id);
int ipcbuf_eod(ipcbuf_t *id);
uint64_t ipcbuf_get_bufsz(ipcbuf_t *id);
uint64_t ipcbuf_get_nbufs(ipcbuf_t *id);
#endif
