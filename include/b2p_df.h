/*
 * include/b2p_df.h -- PAF BMF data-frame (DF) headers: decode, encode and
 * placement arithmetic of the capture side.
 *
 * A DF is 7232 B: a 64-B header followed by a 7168-B payload of
 * [128 samples][7 channels][2 pols][re,im] int16 big-endian
 * (capture.h:27-29).  The header's first three 64-bit words are big-endian
 * (hdr.c:10-28):
 *   word0: idf bits 0-31, sec bits 32-61, valid bit 63
 *   word1: epoch bits 26-31
 *   word2: beam bits 0-15, freq (integer MHz) bits 16-31
 * Capture places a DF's payload in a ring block at
 *   (idf_rel * NCHK_NIC + ifreq) * 7168          (capture.c:527-547)
 * with idf_rel from the header relative to a reference DF (capture.c:562-568)
 * and ifreq from the sender's IP address (capture.c:571-584).  The GPU
 * scatter that builds whole blocks from a raw DF stream is b2p_assemble()
 * in include/b2p.h.  Plain C, host side (libpafdada.so).
 */
#ifndef B2P_DF_H
#define B2P_DF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define B2P_DF_HDR_BYTES 64          /* HDR_SIZE, capture.h:29 */
#define B2P_DF_PAYLOAD_BYTES 7168    /* DT_SIZE,  capture.h:28 */
#define B2P_DF_BYTES 7232            /* DF_SIZE,  capture.h:27 */
#define B2P_DF_PER_PERIOD 250000     /* NDF_PRD,  capture.h:32 */
#define B2P_DF_PERIOD_SEC 27         /* PRD_SEC,  capture.h:31 */
#define B2P_DF_TSAMP_SEC 1.08E-4     /* TDF_SEC,  capture.h:30 */
#define B2P_DF_NCHK_BMF 6            /* NCHK_BMF, capture.h:21 */
#define B2P_DF_SECDAY 86400.0        /* SECDAY,   capture.h:43 */
#define B2P_DF_TIMESTR "%Y-%m-%d-%H:%M:%S" /* DADA_TIMESTR, capture.h:15 */

/* same members as hdr_t (hdr.h:6-14) */
typedef struct b2p_df_hdr {
  int valid;     /* 1: the DF is valid                                  */
  uint64_t idf;  /* DF number inside the current 27-s period            */
  uint64_t sec;  /* seconds from the reference epoch at period start    */
  int epoch;     /* half-years since 2000-01-01                         */
  int beam;      /* beam id                                              */
  double freq;   /* frequency of the chunk's first channel, integer MHz */
} b2p_df_hdr_t;

/* hdr_keys (hdr.c:10-28): decode the first 24 bytes of a DF header */
void b2p_df_decode(const void *df, b2p_df_hdr_t *hdr);
/* inverse of b2p_df_decode: writes the 64-B header (unused bits zero);
 * fields are masked to their widths (freq truncated to an integer) */
void b2p_df_encode(const b2p_df_hdr_t *hdr, void *df);
/* acquire_idf (capture.c:562-568), same double arithmetic:
 * (int64)hdr.idf + (int64)(hdr.sec - ref.sec) / TDF_SEC - (int64)ref.idf */
int64_t b2p_df_index(const b2p_df_hdr_t *hdr, const b2p_df_hdr_t *ref);
/* the block switch of sync.c:119-125: the reference moves on by ndf DFs,
 * wrapping into the next 27-s period */
void b2p_df_ref_advance(b2p_df_hdr_t *ref, uint64_t ndf);
/* acquire_ifreq (capture.c:571-584): chunk index from the sender's IPv4
 * address, as stored in sockaddr_in.sin_addr.s_addr (network byte order):
 * (octet3 - 1) * NCHK_BMF + ceil(octet4 / 2) - 1 */
int b2p_df_chunk_from_ip(uint32_t s_addr);

/* ---- start time of a capture (acquire_start_time, capture.c:791-843) ----
 * The epoch file maps a header epoch to a day number: lines "EPOCH DAYS
 * [anything]", '#' lines skipped (capture.c:808-815).  Returns 0 and sets
 * *days, -1 if the file cannot be opened (capture.c:798-805), -2 if no line
 * names `epoch` (the reference then silently used the last line read; here
 * that is an error). */
int b2p_df_epoch_days(const char *epoch_file, int epoch, double *days);
/* UTC_START and PICOSECONDS of the frame `start`, the same double
 * arithmetic as capture.c:819-825:
 *   sec_prd     = idf * TDF_SEC
 *   t           = (time_t)(SECDAY * days + sec + floor(sec_prd))
 *   utc_start   = strftime(DADA_TIMESTR, gmtime(t))
 *   picoseconds = 1e6 * round(1e6 * (sec_prd - floor(sec_prd)))
 * utc_start needs >= 20 bytes.  Returns 0, or -1 if the time does not
 * convert. */
int b2p_df_start_time(const b2p_df_hdr_t *start, double days, char *utc_start, size_t len,
                      uint64_t *picoseconds);

#ifdef __cplusplus
}
#endif
#endif /* B2P_DF_H */
