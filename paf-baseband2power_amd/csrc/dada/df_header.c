/*
 * df_header.c -- BMF data-frame header arithmetic (include/b2p_df.h).
 * Restates hdr.c:10-28 (decode), capture.c:562-584 (frame index, chunk from
 * IP) and sync.c:119-125 (reference advance); the encoder is new (the
 * reference only receives frames); capture.c:791-843 (start time of a
 * capture: UTC_START, PICOSECONDS).  Decode is pinned by tests against the
 * reference's own hdr.c (tests/golden/hdr_pin.npz).
 */
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

#include "b2p_df.h"

static uint64_t load_be64(const unsigned char *p) {
  uint64_t v = 0;
  for (int k = 0; k < 8; k++) v = (v << 8) | p[k];
  return v;
}

static void store_be64(unsigned char *p, uint64_t v) {
  for (int k = 7; k >= 0; k--) {
    p[k] = (unsigned char)(v & 0xff);
    v >>= 8;
  }
}

void b2p_df_decode(const void *df, b2p_df_hdr_t *h) {
  const unsigned char *p = (const unsigned char *)df;
  const uint64_t w0 = load_be64(p), w1 = load_be64(p + 8), w2 = load_be64(p + 16);
  h->idf = w0 & 0x00000000ffffffffULL;
  h->sec = (w0 & 0x3fffffff00000000ULL) >> 32;
  h->valid = (int)((w0 & 0x8000000000000000ULL) >> 63);
  h->epoch = (int)((w1 & 0x00000000fc000000ULL) >> 26);
  h->freq = (double)((w2 & 0x00000000ffff0000ULL) >> 16);
  h->beam = (int)(w2 & 0x000000000000ffffULL);
}

void b2p_df_encode(const b2p_df_hdr_t *h, void *df) {
  unsigned char *p = (unsigned char *)df;
  memset(p, 0, B2P_DF_HDR_BYTES);
  const uint64_t w0 = (h->idf & 0xffffffffULL) | ((h->sec & 0x3fffffffULL) << 32) |
                      ((uint64_t)(h->valid & 1) << 63);
  const uint64_t w1 = ((uint64_t)(h->epoch & 0x3f)) << 26;
  const uint64_t freq = h->freq > 0 ? (uint64_t)h->freq : 0;
  const uint64_t w2 = ((uint64_t)(h->beam & 0xffff)) | ((freq & 0xffffULL) << 16);
  store_be64(p, w0);
  store_be64(p + 8, w1);
  store_be64(p + 16, w2);
}

int64_t b2p_df_index(const b2p_df_hdr_t *h, const b2p_df_hdr_t *ref) {
  /* the C of capture.c:566, evaluated in the same types */
  return (int64_t)h->idf + (int64_t)(h->sec - ref->sec) / B2P_DF_TSAMP_SEC - (int64_t)ref->idf;
}

void b2p_df_ref_advance(b2p_df_hdr_t *ref, uint64_t ndf) {
  ref->idf += ndf;
  while (ref->idf >= B2P_DF_PER_PERIOD) { /* sync.c:121-125, for any ndf */
    ref->sec += B2P_DF_PERIOD_SEC;
    ref->idf -= B2P_DF_PER_PERIOD;
  }
}

int b2p_df_chunk_from_ip(uint32_t s_addr) {
  const unsigned char *ip = (const unsigned char *)&s_addr;
  return (int)(ip[2] - 1) * B2P_DF_NCHK_BMF + (int)ceil((double)(ip[3] / 2.0)) - 1;
}

int b2p_df_epoch_days(const char *epoch_file, int epoch, double *days) {
  FILE *fp = epoch_file ? fopen(epoch_file, "r") : NULL;
  if (!fp) return -1; /* capture.c:798-805 */
  char line[512];
  int found = 0;
  while (!found && fgets(line, sizeof line, fp)) {
    if (line[0] == '#') continue; /* capture.c:810 */
    int e;
    double d;
    if (sscanf(line, "%d %lf", &e, &d) == 2 && e == epoch) { /* capture.c:811-813 */
      *days = d;
      found = 1;
    }
  }
  fclose(fp);
  return found ? 0 : -2;
}

int b2p_df_start_time(const b2p_df_hdr_t *start, double days, char *utc_start, size_t len,
                      uint64_t *picoseconds) {
  if (!start || !utc_start || len < 20 || !picoseconds) return -1;
  const double sec_prd = (double)start->idf * B2P_DF_TSAMP_SEC;                     /* :819 */
  const time_t t = (time_t)(B2P_DF_SECDAY * days + (double)start->sec + floor(sec_prd)); /* :820 */
  struct tm tm;
  if (!gmtime_r(&t, &tm) || strftime(utc_start, len, B2P_DF_TIMESTR, &tm) == 0) return -1; /* :821 */
  const double micro = 1.0E6 * (sec_prd - floor(sec_prd));                        /* :824 */
  *picoseconds = (uint64_t)(1E6 * round(micro));                                  /* :825 */
  return 0;
}
