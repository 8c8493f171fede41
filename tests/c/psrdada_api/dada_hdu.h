/* declarations only -- see README.txt.  dada_hdu per SURVEY.md Appendix A
 * (48 B; header key = key + 1). */
#ifndef __DADA_HDU_H
#define __DADA_HDU_H
#include "ipcio.h"
#include "multilog.h"
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
void dada_hdu_destroy(dada_hdu_t *hdu);
int dada_hdu_connect(dada_hdu_t *hdu);
int dada_hdu_disconnect(dada_hdu_t *hdu);
int dada_hdu_lock_read(dada_hdu_t *hdu);
int dada_hdu_unlock_read(dada_hdu_t *hdu);
int dada_hdu_lock_write(dada_hdu_t *hdu);
int dada_hdu_unlock_write(dada_hdu_t *hdu);
#endif
