/*
 * oracle/b2p_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the baseband->power integrate path of
 * xinpingdeng/paf-baseband2power.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this code; the product library
 * (paf-baseband2power_amd/) never links or calls it.
 *
 * PARITY STATUS: partially pinned.  The reference's hot path is an empty stub
 * (kernel.cu:1-7, baseband2power.cu:1-16, paf_baseband2power.cu:32-93) and the
 * reference ships no golden vectors, known-answer tests or fixtures
 * (SURVEY.md section 8c).  The accumulate semantics below are therefore a
 * restatement of the reference's *specification*:
 *   - input layout TFTFP, payload only:  capture.c:222, capture.c:527,540;
 *     geometry capture.h:20,28 and paf-baseband2power.conf:2-5,9
 *   - big-endian 64-bit word unpack:     cudautil.cuh:118-125 (BSWAP_64),
 *     same primitive as bswap_64 in hdr.c:15-24.  This primitive IS pinned:
 *     tests/golden/hdr_pin.npz holds outputs of the reference's own hdr.c,
 *     compiled from /root/reference by oracle/Makefile (target ref).
 *   - detect + time-integrate 1024x1024 samples: README.md:2,
 *     paf_baseband2power.cu:20
 *   - output one fp32 per channel, pols summed: header_baseband2power.txt:39-42,
 *     paf-baseband2power.py:77-79
 * The accumulate is an exact integer sum (uint64) rounded once to fp32 (RNE).
 */
#ifndef B2P_ORACLE_H
#define B2P_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same field order and meaning as b2p_geom_t (include/b2p.h), restated here
 * so the oracle does not depend on product headers. */
typedef struct orc_geom {
  uint32_t nbit;        /* 8 or 16 bits per real component                    */
  uint32_t big_endian;  /* 1: int16 BE words decoded via BSWAP_64 (BMF)       */
  uint32_t nchunk;      /* frequency chunks per frame  (capture.h:20 -> 48)   */
  uint32_t nsamp_df;    /* samples per chunk per frame (conf:2 -> 128)        */
  uint32_t nchan_chunk; /* channels per chunk          (7168/128/8 -> 7)      */
  uint32_t npol;        /* polarisations               (conf:3 -> 2)          */
  uint32_t ndim;        /* 2 = complex                 (conf:4 -> 2)          */
  uint32_t npol_out;    /* 1: X+Y summed (header NPOL 1); 2: X and Y          */
  uint64_t nsamp_int;   /* samples per integration (README.md:2 -> 1<<20)     */
  uint32_t mean;        /* 0: sum, 1: sum / nsamp_int                         */
  uint32_t reserved;
} orc_geom_t;

/* bytes of one (time, channel) word: npol * ndim * nbit/8 */
size_t orc_word_bytes(const orc_geom_t *g);
/* bytes of one frame: nchunk * nsamp_df * nchan_chunk * word */
size_t orc_frame_bytes(const orc_geom_t *g);
/* total channels = nchunk * nchan_chunk ; output values = nchan * npol_out */
uint32_t orc_nchan(const orc_geom_t *g);
uint32_t orc_nout(const orc_geom_t *g);

/* Decode one big-endian 64-bit BMF word into 4 int16 lanes, lane k = bits
 * [16k, 16k+16) of BSWAP_64(word) (cudautil.cuh:118-125).  Build convention
 * (SURVEY 8a a4): lane0 = X.re, lane1 = X.im, lane2 = Y.re, lane3 = Y.im. */
void orc_bmf_lanes(const uint8_t word[8], int16_t lanes[4]);

/* Exact accumulate of nbytes (a whole number of frames) into acc[nout].
 * Returns 0, or -1 on a ragged/invalid input. Single thread. */
int orc_integrate(const orc_geom_t *g, const uint8_t *buf, size_t nbytes,
                  uint64_t *acc);
/* Same, split over nthreads OpenMP threads (frames partitioned). */
int orc_integrate_mt(const orc_geom_t *g, const uint8_t *buf, size_t nbytes,
                     uint64_t *acc, int nthreads);

/* fp32 output: RNE(sum) or RNE((double)sum / nsamp_int) */
void orc_finalize(const orc_geom_t *g, const uint64_t *acc, float *out);

/* Counter-based synthetic baseband (SURVEY 8d "Value distribution"):
 * element e (memory order, one real component) of block `block` of sub-band
 * `subband` is a function of (seed, subband, block, e) only.  elem0 is the
 * element index of buf[0] within the block. */
void orc_fill_synthetic(const orc_geom_t *g, uint8_t *buf, size_t nbytes,
                        uint64_t seed, uint32_t subband, uint64_t block,
                        uint64_t elem0);

uint64_t orc_splitmix64(uint64_t x);

/* ---- data frames (capture side) -------------------- */
typedef struct orc_df_hdr { /* hdr_t, hdr.h:6-14 */
  int valid;
  uint64_t idf, sec;
  int epoch, beam;
  double freq;
} orc_df_hdr_t;
/* hdr_keys, hdr.c:10-28 (bswap_64 of the first three words) */
void orc_df_decode(const uint8_t *df, orc_df_hdr_t *h);
/* acquire_idf, capture.c:562-568 */
int64_t orc_df_index(const orc_df_hdr_t *h, uint64_t ref_idf, uint64_t ref_sec);
/* capture.c:527-547 placement of ndf frames (df_bytes each, 64-B header),
 * in arrival order, into a payload-only block; counts[nchunk + 3] as
 * b2p_assemble (include/b2p.h) */
void orc_assemble(const uint8_t *dfs, uint64_t ndf, uint32_t df_bytes, const uint8_t *chunk_of_df,
                  uint64_t ref_idf, uint64_t ref_sec, uint8_t *block, uint64_t block_ndf,
                  uint32_t nchunk, uint64_t *counts);

#ifdef __cplusplus
}
#endif
#endif
