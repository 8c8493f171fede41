/* declarations only -- see README.txt.  ipcio_t per the reference's DWARF
 * (152 B): the ipcbuf_t comes first, so (ipcbuf_t *)ipcio is valid. */
#ifndef __DADA_IPCIO_H
#define __DADA_IPCIO_H
#include <sys/types.h>
#include "ipcbuf.h"
typedef struct {
  ipcbuf_t buf;
  char *curbuf;
  uint64_t curbufsz;
  uint64_t bytes;
  char rdwrt;
  char marked_filled;
  char sod_pending;
  uint64_t sod_buf;
  uint64_t sod_byte;
} ipcio_t;
char *ipcio_open_block_write(ipcio_t *ipc, uint64_t *block_id);
ssize_t ipcio_close_block_write(ipcio_t *ipc, uint64_t bytes);
char *ipcio_open_block_read(ipcio_t *ipc, uint64_t *curbufsz, uint64_t *block_id);
ssize_t ipcio_close_block_read(ipcio_t *ipc, uint64_t bytes);
#endif
