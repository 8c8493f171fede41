/*
 * oracle/b2p_oracle.c -- TEST INFRASTRUCTURE ONLY (see b2p_oracle.h header
 * for the parity status and the reference lines each rule follows).
 *
 * Deliberately written as plain nested loops over the TFTFP indices so a
 * reader can check it against capture.c:540 line by line:
 *     cbuf_loc = (idf * NCHK_NIC + ifreq) * pkt_size        (capture.c:540)
 * i.e. block = [frame idf][chunk ifreq][7168-B payload], and the payload is
 * [sample 128][chan 7][pol 2][re,im] int16 big-endian (capture.h:28,
 * paf-baseband2power.conf:2-5).
 */
#include "b2p_oracle.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

size_t orc_word_bytes(const orc_geom_t *g) {
  return (size_t)g->npol * g->ndim * (g->nbit / 8);
}
size_t orc_frame_bytes(const orc_geom_t *g) {
  return (size_t)g->nchunk * g->nsamp_df * g->nchan_chunk * orc_word_bytes(g);
}
uint32_t orc_nchan(const orc_geom_t *g) { return g->nchunk * g->nchan_chunk; }
uint32_t orc_nout(const orc_geom_t *g) { return orc_nchan(g) * g->npol_out; }

static int geom_ok(const orc_geom_t *g) {
  if (g->nbit != 8 && g->nbit != 16) return 0;
  if (g->nbit == 8 && g->big_endian) return 0;
  if (g->npol != 2 || g->ndim != 2) return 0;
  if (g->npol_out != 1 && g->npol_out != 2) return 0;
  if (!g->nchunk || !g->nsamp_df || !g->nchan_chunk) return 0;
  return 1;
}

/* BSWAP_64 (cudautil.cuh:118-125): byte k of the swapped value is byte 7-k
 * of the word as stored; reading the swapped value as a little-endian
 * uint64, lane k = bits [16k, 16k+16). */
static uint64_t bswap64_restated(uint64_t x) {
  uint64_t r = 0;
  for (int k = 0; k < 8; k++) r |= ((x >> (8 * k)) & 0xffu) << (8 * (7 - k));
  return r;
}

void orc_bmf_lanes(const uint8_t word[8], int16_t lanes[4]) {
  uint64_t w = 0;
  for (int k = 0; k < 8; k++) w |= (uint64_t)word[k] << (8 * k); /* host LE */
  uint64_t s = bswap64_restated(w);
  for (int k = 0; k < 4; k++) lanes[k] = (int16_t)(uint16_t)(s >> (16 * k));
}

/* components of one word, in the order X.re, X.im, Y.re, Y.im */
static void decode_word(const orc_geom_t *g, const uint8_t *p, int32_t c[4]) {
  if (g->nbit == 8) {
    for (int k = 0; k < 4; k++) c[k] = (int8_t)p[k];
  } else if (g->big_endian) {
    int16_t l[4];
    orc_bmf_lanes(p, l);
    for (int k = 0; k < 4; k++) c[k] = l[k];
  } else {
    for (int k = 0; k < 4; k++)
      c[k] = (int16_t)(uint16_t)(p[2 * k] | (p[2 * k + 1] << 8));
  }
}

static void integrate_frames(const orc_geom_t *g, const uint8_t *buf,
                             uint64_t f0, uint64_t f1, uint64_t *acc) {
  const size_t wb = orc_word_bytes(g);
  for (uint64_t f = f0; f < f1; f++)
    for (uint32_t ck = 0; ck < g->nchunk; ck++)
      for (uint32_t s = 0; s < g->nsamp_df; s++)
        for (uint32_t k = 0; k < g->nchan_chunk; k++) {
          uint64_t word =
              ((f * g->nchunk + ck) * g->nsamp_df + s) * g->nchan_chunk + k;
          int32_t c[4];
          decode_word(g, buf + word * wb, c);
          uint64_t px = (uint64_t)((int64_t)c[0] * c[0] + (int64_t)c[1] * c[1]);
          uint64_t py = (uint64_t)((int64_t)c[2] * c[2] + (int64_t)c[3] * c[3]);
          uint32_t ch = ck * g->nchan_chunk + k;
          if (g->npol_out == 1) {
            acc[ch] += px + py;
          } else {
            acc[2 * ch] += px;
            acc[2 * ch + 1] += py;
          }
        }
}

int orc_integrate(const orc_geom_t *g, const uint8_t *buf, size_t nbytes,
                  uint64_t *acc) {
  if (!geom_ok(g)) return -1;
  size_t fb = orc_frame_bytes(g);
  if (nbytes % fb) return -1;
  integrate_frames(g, buf, 0, nbytes / fb, acc);
  return 0;
}

int orc_integrate_mt(const orc_geom_t *g, const uint8_t *buf, size_t nbytes,
                     uint64_t *acc, int nthreads) {
  if (!geom_ok(g)) return -1;
  size_t fb = orc_frame_bytes(g);
  if (nbytes % fb) return -1;
  uint64_t nf = nbytes / fb;
  uint32_t nout = orc_nout(g);
  if (nthreads < 1) nthreads = 1;
  uint64_t *part = calloc((size_t)nthreads * nout, sizeof(uint64_t));
  if (!part) return -1;
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads)
#endif
  {
    int t = 0, nt = 1;
#ifdef _OPENMP
    t = omp_get_thread_num();
    nt = omp_get_num_threads();
#endif
    uint64_t f0 = nf * t / nt, f1 = nf * (t + 1) / nt;
    integrate_frames(g, buf, f0, f1, part + (size_t)t * nout);
  }
  for (int t = 0; t < nthreads; t++)
    for (uint32_t j = 0; j < nout; j++) acc[j] += part[(size_t)t * nout + j];
  free(part);
  return 0;
}

void orc_finalize(const orc_geom_t *g, const uint64_t *acc, float *out) {
  uint32_t nout = orc_nout(g);
  for (uint32_t j = 0; j < nout; j++) {
    if (g->mean)
      out[j] = (float)((double)acc[j] / (double)g->nsamp_int);
    else
      out[j] = (float)acc[j]; /* one round-to-nearest-even */
  }
}

/* ---------------------------------------------------------------------- */
/* synthetic baseband: SplitMix64 counter generator, integer-only Gaussian */

uint64_t orc_splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

void orc_fill_synthetic(const orc_geom_t *g, uint8_t *buf, size_t nbytes,
                        uint64_t seed, uint32_t subband, uint64_t block,
                        uint64_t elem0) {
  const uint64_t k_sub =
      orc_splitmix64(seed ^ (0xD1B54A32D192ED03ULL * ((uint64_t)subband + 1)));
  const uint64_t key =
      orc_splitmix64(k_sub ^ (0x8CB92BA72F3D8DD7ULL * (block + 1)));
  const uint32_t eb = g->nbit / 8;
  const uint64_t nelem = nbytes / eb;
  const uint64_t comp = (uint64_t)g->npol * g->ndim;
  const uint64_t wpc = (uint64_t)g->nsamp_df * g->nchan_chunk;
  const uint64_t wpf = wpc * g->nchunk;
  const uint32_t nchan = orc_nchan(g);
  const int64_t amp = g->nbit == 8 ? 35 : 3464; /* sigma ~ 20 / ~ 2000 */
  const int64_t lo = g->nbit == 8 ? -128 : -32768;
  const int64_t hi = g->nbit == 8 ? 127 : 32767;
#ifdef _OPENMP
#pragma omp parallel for schedule(static) if (nelem > (1u << 22))
#endif
  for (uint64_t i = 0; i < nelem; i++) {
    uint64_t e = elem0 + i;
    uint64_t r = orc_splitmix64(key + e);
    int64_t gs = (int64_t)(r & 0xffff) + (int64_t)((r >> 16) & 0xffff) +
                 (int64_t)((r >> 32) & 0xffff) + (int64_t)(r >> 48) - 131070;
    uint64_t wf = (e / comp) % wpf;
    uint32_t ch = (uint32_t)((wf / wpc) * g->nchan_chunk + wf % g->nchan_chunk);
    int64_t a = (ch == 0 || ch == 7 || ch == nchan - 1) ? 2 * amp : amp;
    int64_t v = (gs * a) >> 16;
    if (v < lo) v = lo;
    if (v > hi) v = hi;
    if (eb == 1) {
      buf[i] = (uint8_t)(int8_t)v;
    } else {
      uint16_t u = (uint16_t)(int16_t)v;
      if (g->big_endian) {
        buf[2 * i] = (uint8_t)(u >> 8);
        buf[2 * i + 1] = (uint8_t)u;
      } else {
        buf[2 * i] = (uint8_t)u;
        buf[2 * i + 1] = (uint8_t)(u >> 8);
      }
    }
  }
}

/* ---------------------------------------------------------------------- */
/* data frames: hdr.c:10-28, capture.c:527-568                              */

static uint64_t be64_at(const uint8_t *p) {
  uint64_t w = 0;
  for (int k = 0; k < 8; k++) w |= (uint64_t)p[k] << (8 * k); /* host LE load */
  return bswap64_restated(w);                                 /* bswap_64 */
}

void orc_df_decode(const uint8_t *df, orc_df_hdr_t *h) {
  uint64_t w = be64_at(df);
  h->idf = w & 0x00000000ffffffffULL;
  h->sec = (w & 0x3fffffff00000000ULL) >> 32;
  h->valid = (int)((w & 0x8000000000000000ULL) >> 63);
  w = be64_at(df + 8);
  h->epoch = (int)((w & 0x00000000fc000000ULL) >> 26);
  w = be64_at(df + 16);
  h->freq = (double)((w & 0x00000000ffff0000ULL) >> 16);
  h->beam = (int)(w & 0x000000000000ffffULL);
}

int64_t orc_df_index(const orc_df_hdr_t *h, uint64_t ref_idf, uint64_t ref_sec) {
  return (int64_t)h->idf + (int64_t)(h->sec - ref_sec) / 1.08E-4 - (int64_t)ref_idf;
}

void orc_assemble(const uint8_t *dfs, uint64_t ndf, uint32_t df_bytes, const uint8_t *chunk_of_df,
                  uint64_t ref_idf, uint64_t ref_sec, uint8_t *block, uint64_t block_ndf,
                  uint32_t nchunk, uint64_t *counts) {
  for (uint64_t d = 0; d < ndf; d++) {
    const uint8_t *df = dfs + d * df_bytes;
    orc_df_hdr_t h;
    orc_df_decode(df, &h);
    const int64_t idf = orc_df_index(&h, ref_idf, ref_sec);
    const uint32_t ifreq = chunk_of_df[d];
    if (ifreq >= nchunk) { counts[nchunk + 2]++; continue; }
    if (idf < 0) { counts[nchunk]++; continue; }
    if ((uint64_t)idf >= block_ndf) { counts[nchunk + 1]++; continue; }
    memcpy(block + ((uint64_t)idf * nchunk + ifreq) * 7168u, df + 64, 7168); /* capture.c:540-542 */
    counts[ifreq]++;
  }
}
