/*
 * oracle/b2p_cpu_port.c -- the tuned CPU port of the integrate path, used
 * ONLY as bench.py's cpu_baseline (SURVEY.md 8(d) "CPU baseline": -O3,
 * vectorised, OpenMP over time tiles).  It is not the checker: tests assert
 * that it equals the oracle (b2p_oracle.c) bit for bit, and nothing in the
 * product library links or calls it.
 *
 * Same arithmetic as the oracle -- the reference's specification of the path
 * (README.md:2, capture.c:540 TFTFP layout, cudautil.cuh:118-125 BSWAP_64,
 * header_baseband2power.txt:39-42) -- organised for a CPU:
 *
 *   - The chunk's [samp][chan] words repeat with period nchan_chunk, so a
 *     chunk is read as whole periods of P = lcm(nchan_chunk, words per
 *     vector) words; every vector lane then sees the same (channel, pol) in
 *     every period and keeps its own accumulator (no gathers, no shuffles).
 *   - Detect: components widened to int16, then one pmaddwd per vector
 *     gives re^2 + im^2 per (word, pol) lane (vpdpwssd with AVX-512 VNNI,
 *     which also does the add).  BMF int16 BE words are byte-swapped per
 *     16-bit lane first (vpshufb); after BSWAP_64 the lanes read
 *     [Y.im, Y.re, X.im, X.re] in memory order, so the pol of a lane flips.
 *   - Accumulate: int8 in 32-bit lanes (<= 2^15 per add, flushed to 64 bits
 *     every 32768 adds); int16 lanes can reach 2^31 per add, so they are
 *     widened to 64 bits on every add.  All exact, so the sums equal the
 *     oracle's uint64 sums.
 *   - Threads: frames are split into equal contiguous tiles, one per OpenMP
 *     thread (the same static split that first-touched the block), each cut
 *     into ~4 MiB pieces.  A thread takes its own tile's pieces in order,
 *     then takes pieces left in its neighbours' tiles: on a host shared with
 *     other jobs a thread that is preempted for a while no longer holds the
 *     whole pass back (one slow thread set the pass time with plain static
 *     tiles).  Sums are exact integers, so who adds a piece cannot change a
 *     bit.
 *
 * ISA chosen at run time (__builtin_cpu_supports): avx512vnni > avx512bw >
 * avx2 > scalar; cpp_integrate's `isa` argument forces one for tests.
 */
#include <immintrin.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "b2p_oracle.h"

enum { ISA_AUTO = 0, ISA_SCALAR = 1, ISA_AVX2 = 2, ISA_AVX512 = 3, ISA_VNNI = 4 };

static const char *kIsaName[] = {"auto", "scalar", "avx2", "avx512bw", "avx512vnni"};

typedef struct plan {
  uint32_t wb;     /* bytes per word (4 int8, 8 int16)          */
  uint32_t vw;     /* words per vector                          */
  uint32_t P;      /* period in words, multiple of vw and nchan_chunk */
  uint32_t nper;   /* periods per chunk                         */
  uint32_t lanes;  /* accumulator lanes per chunk = 2 P         */
  uint64_t cw;     /* words per chunk                           */
} plan_t;

static uint64_t gcd64(uint64_t a, uint64_t b) {
  while (b) {
    uint64_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}

/* 0 if the vector path applies at this vector width */
static int make_plan(const orc_geom_t *g, uint32_t vbytes, plan_t *p) {
  p->wb = g->nbit / 8 * 4;
  p->vw = vbytes / p->wb;
  p->cw = (uint64_t)g->nsamp_df * g->nchan_chunk;
  const uint64_t P = (uint64_t)g->nchan_chunk / gcd64(g->nchan_chunk, p->vw) * p->vw;
  if (P > 4096 || p->cw % P) return -1;
  p->P = (uint32_t)P;
  p->nper = (uint32_t)(p->cw / P);
  p->lanes = 2 * p->P;
  if (g->nbit == 8 && p->nper > 32768) return -1;
  return 0;
}

/* lane i of a chunk's accumulators -> output index */
static void fold(const orc_geom_t *g, const plan_t *p, const uint64_t *acc64, uint64_t *out) {
  const uint32_t be = g->nbit == 16 && g->big_endian;
  for (uint32_t ck = 0; ck < g->nchunk; ck++)
    for (uint32_t i = 0; i < p->lanes; i++) {
      const uint32_t ch = ck * g->nchan_chunk + (i / 2) % g->nchan_chunk;
      const uint32_t pol = (i & 1) ^ be;
      out[g->npol_out == 1 ? ch : 2 * ch + pol] += acc64[(uint64_t)ck * p->lanes + i];
    }
}

/* ---- scalar (any layout) ------------------------------------------------ */
static void run_scalar(const orc_geom_t *g, const uint8_t *buf, uint64_t f0, uint64_t f1,
                       uint64_t *out) {
  const uint64_t wb = g->nbit / 8 * 4, cw = (uint64_t)g->nsamp_df * g->nchan_chunk;
  for (uint64_t f = f0; f < f1; f++)
    for (uint32_t ck = 0; ck < g->nchunk; ck++) {
      const uint8_t *c = buf + (f * g->nchunk + ck) * cw * wb;
      for (uint64_t w = 0; w < cw; w++) {
        const uint8_t *q = c + w * wb;
        int64_t v[4];
        for (int k = 0; k < 4; k++) {
          if (g->nbit == 8) v[k] = (int8_t)q[k];
          else if (g->big_endian) v[k] = (int16_t)(uint16_t)((q[2 * k] << 8) | q[2 * k + 1]);
          else v[k] = (int16_t)(uint16_t)(q[2 * k] | (q[2 * k + 1] << 8));
        }
        /* BE: memory order [Y.im, Y.re, X.im, X.re] after BSWAP_64 */
        const uint64_t a = (uint64_t)(v[0] * v[0] + v[1] * v[1]);
        const uint64_t b = (uint64_t)(v[2] * v[2] + v[3] * v[3]);
        const uint64_t px = g->nbit == 16 && g->big_endian ? b : a;
        const uint64_t py = g->nbit == 16 && g->big_endian ? a : b;
        const uint32_t ch = ck * g->nchan_chunk + (uint32_t)(w % g->nchan_chunk);
        if (g->npol_out == 1) {
          out[ch] += px + py;
        } else {
          out[2 * ch] += px;
          out[2 * ch + 1] += py;
        }
      }
    }
}

/* ---- vector bodies ------------------------------------------------------- */
/* int8: acc32[lanes per chunk x nchunk], flushed into acc64 */
#define INT8_BODY(VEC, LOAD, WIDEN_LO, WIDEN_HI, DOT, ZERO, STORE, LOADA, HALF)               \
  {                                                                                      \
    const uint32_t nv = p->P / p->vw;                                                    \
    uint64_t adds = 0;                                                                   \
    for (uint64_t f = f0; f < f1; f++) {                                                 \
      if (adds + p->nper > 32768) {                                                      \
        for (uint64_t i = 0; i < (uint64_t)p->lanes * g->nchunk; i++) {                  \
          acc64[i] += (uint64_t)(uint32_t)acc32[i];                                      \
          acc32[i] = 0;                                                                  \
        }                                                                                \
        adds = 0;                                                                        \
      }                                                                                  \
      adds += p->nper;                                                                   \
      for (uint32_t ck = 0; ck < g->nchunk; ck++) {                                      \
        const uint8_t *c = buf + (f * g->nchunk + ck) * p->cw * 4;                       \
        int32_t *a = acc32 + (uint64_t)ck * p->lanes;                                    \
        for (uint32_t per = 0; per < p->nper; per++) {                                   \
          const uint8_t *q = c + (uint64_t)per * p->P * 4;                               \
          for (uint32_t v = 0; v < nv; v++) {                                            \
            VEC x = LOAD(q + (uint64_t)v * p->vw * 4);                                   \
            VEC lo = WIDEN_LO(x), hi = WIDEN_HI(x);                                      \
            VEC s0 = LOADA(a + 2 * v * HALF), s1 = LOADA(a + (2 * v + 1) * HALF);        \
            STORE(a + 2 * v * HALF, DOT(s0, lo));                                        \
            STORE(a + (2 * v + 1) * HALF, DOT(s1, hi));                                  \
          }                                                                              \
        }                                                                                \
      }                                                                                  \
    }                                                                                    \
    for (uint64_t i = 0; i < (uint64_t)p->lanes * g->nchunk; i++) {                      \
      acc64[i] += (uint64_t)(uint32_t)acc32[i];                                          \
      acc32[i] = 0; /* the next call (another piece) starts from zero */                 \
    }                                                                                    \
    (void)ZERO;                                                                          \
  }

/* AVX-512 */
#define L512(ptr) _mm512_loadu_si512((const void *)(ptr))
#define LA512(ptr) _mm512_load_si512((const void *)(ptr))
#define S512(ptr, v) _mm512_store_si512((void *)(ptr), (v))
#define W512LO(x) _mm512_cvtepi8_epi16(_mm512_castsi512_si256(x))
#define W512HI(x) _mm512_cvtepi8_epi16(_mm512_extracti64x4_epi64((x), 1))
#define DOT512(s, v) _mm512_add_epi32((s), _mm512_madd_epi16((v), (v)))
#define DOTVNNI(s, v) _mm512_dpwssd_epi32((s), (v), (v))

__attribute__((target("avx512f,avx512bw"))) static void i8_avx512(
    const orc_geom_t *g, const plan_t *p, const uint8_t *buf, uint64_t f0, uint64_t f1,
    int32_t *acc32, uint64_t *acc64) INT8_BODY(__m512i, L512, W512LO, W512HI, DOT512, 0, S512, LA512, 16)

__attribute__((target("avx512f,avx512bw,avx512vnni"))) static void i8_vnni(
    const orc_geom_t *g, const plan_t *p, const uint8_t *buf, uint64_t f0, uint64_t f1,
    int32_t *acc32, uint64_t *acc64) INT8_BODY(__m512i, L512, W512LO, W512HI, DOTVNNI, 0, S512, LA512, 16)

/* AVX2 */
#define L256(ptr) _mm256_loadu_si256((const __m256i *)(ptr))
#define LA256(ptr) _mm256_load_si256((const __m256i *)(ptr))
#define S256(ptr, v) _mm256_store_si256((__m256i *)(ptr), (v))
#define W256LO(x) _mm256_cvtepi8_epi16(_mm256_castsi256_si128(x))
#define W256HI(x) _mm256_cvtepi8_epi16(_mm256_extracti128_si256((x), 1))
#define DOT256(s, v) _mm256_add_epi32((s), _mm256_madd_epi16((v), (v)))

__attribute__((target("avx2"))) static void i8_avx2(const orc_geom_t *g, const plan_t *p,
                                                     const uint8_t *buf, uint64_t f0, uint64_t f1,
                                                     int32_t *acc32, uint64_t *acc64)
    INT8_BODY(__m256i, L256, W256LO, W256HI, DOT256, 0, S256, LA256, 8)

/* int16: every pmaddwd lane (<= 2^31, read as uint32) widened into 64 bits */
__attribute__((target("avx512f,avx512bw"))) static void i16_avx512(
    const orc_geom_t *g, const plan_t *p, const uint8_t *buf, uint64_t f0, uint64_t f1,
    uint64_t *acc64) {
  const uint32_t nv = p->P / p->vw;
  const __m512i swap = _mm512_set4_epi32(0x0e0f0c0d, 0x0a0b0809, 0x06070405, 0x02030001);
  const int be = g->big_endian;
  for (uint64_t f = f0; f < f1; f++)
    for (uint32_t ck = 0; ck < g->nchunk; ck++) {
      const uint8_t *c = buf + (f * g->nchunk + ck) * p->cw * 8;
      uint64_t *a = acc64 + (uint64_t)ck * p->lanes;
      for (uint32_t per = 0; per < p->nper; per++) {
        const uint8_t *q = c + (uint64_t)per * p->P * 8;
        for (uint32_t v = 0; v < nv; v++) {
          __m512i x = L512(q + (uint64_t)v * 64);
          if (be) x = _mm512_shuffle_epi8(x, swap);
          const __m512i m = _mm512_madd_epi16(x, x);
          const __m512i lo = _mm512_cvtepu32_epi64(_mm512_castsi512_si256(m));
          const __m512i hi = _mm512_cvtepu32_epi64(_mm512_extracti64x4_epi64(m, 1));
          S512(a + 16 * v, _mm512_add_epi64(LA512(a + 16 * v), lo));
          S512(a + 16 * v + 8, _mm512_add_epi64(LA512(a + 16 * v + 8), hi));
        }
      }
    }
}

__attribute__((target("avx2"))) static void i16_avx2(const orc_geom_t *g, const plan_t *p,
                                                      const uint8_t *buf, uint64_t f0, uint64_t f1,
                                                      uint64_t *acc64) {
  const uint32_t nv = p->P / p->vw;
  const __m256i swap = _mm256_set_epi8(14, 15, 12, 13, 10, 11, 8, 9, 6, 7, 4, 5, 2, 3, 0, 1,
                                       14, 15, 12, 13, 10, 11, 8, 9, 6, 7, 4, 5, 2, 3, 0, 1);
  const int be = g->big_endian;
  for (uint64_t f = f0; f < f1; f++)
    for (uint32_t ck = 0; ck < g->nchunk; ck++) {
      const uint8_t *c = buf + (f * g->nchunk + ck) * p->cw * 8;
      uint64_t *a = acc64 + (uint64_t)ck * p->lanes;
      for (uint32_t per = 0; per < p->nper; per++) {
        const uint8_t *q = c + (uint64_t)per * p->P * 8;
        for (uint32_t v = 0; v < nv; v++) {
          __m256i x = L256(q + (uint64_t)v * 32);
          if (be) x = _mm256_shuffle_epi8(x, swap);
          const __m256i m = _mm256_madd_epi16(x, x);
          const __m256i lo = _mm256_cvtepu32_epi64(_mm256_castsi256_si128(m));
          const __m256i hi = _mm256_cvtepu32_epi64(_mm256_extracti128_si256(m, 1));
          S256(a + 8 * v, _mm256_add_epi64(LA256(a + 8 * v), lo));
          S256(a + 8 * v + 4, _mm256_add_epi64(LA256(a + 8 * v + 4), hi));
        }
      }
    }
}

/* ---- dispatch ------------------------------------------------------------ */
static int best_isa(void) {
  __builtin_cpu_init();
  if (__builtin_cpu_supports("avx512vnni") && __builtin_cpu_supports("avx512bw")) return ISA_VNNI;
  if (__builtin_cpu_supports("avx512bw")) return ISA_AVX512;
  if (__builtin_cpu_supports("avx2")) return ISA_AVX2;
  return ISA_SCALAR;
}

/* The ISA `want` resolves to (ISA_AUTO: the best this CPU has; a forced ISA
 * the CPU lacks resolves to scalar), as a name. */
const char *cpp_isa_name(int want) {
  int best = best_isa();
  int isa = want == ISA_AUTO ? best : (want <= best ? want : ISA_SCALAR);
  return kIsaName[isa];
}

/* Exact accumulate of nbytes (whole frames) into acc[nout], like
 * orc_integrate_mt; returns 0, or -1 on ragged/unsupported input. */
int cpp_integrate(const orc_geom_t *g, const uint8_t *buf, size_t nbytes, uint64_t *acc,
                  int nthreads, int want) {
  if (!g || (g->nbit != 8 && g->nbit != 16) || g->npol != 2 || g->ndim != 2 ||
      (g->npol_out != 1 && g->npol_out != 2) || !g->nchunk || !g->nsamp_df || !g->nchan_chunk)
    return -1;
  const size_t fb = orc_frame_bytes(g);
  if (!fb || nbytes % fb) return -1;
  const uint64_t nf = nbytes / fb;
  const uint32_t nout = orc_nout(g);
  int best = best_isa();
  int isa = want == ISA_AUTO ? best : (want <= best ? want : ISA_SCALAR);
  plan_t p;
  if (isa != ISA_SCALAR && make_plan(g, isa == ISA_AVX2 ? 32 : 64, &p) != 0) isa = ISA_SCALAR;
  if (nthreads < 1) nthreads = 1;
  uint64_t *part = calloc((size_t)nthreads * nout, sizeof(uint64_t));
  if (!part) return -1;
  /* pieces of ~4 MiB of whole frames; next[t * 8]: the next unclaimed piece
   * of thread t's tile (one cache line per counter) */
  const uint64_t pf = fb >= (4u << 20) ? 1 : (4u << 20) / fb;
  uint64_t *next = calloc((size_t)nthreads * 8, sizeof(uint64_t));
  if (!next) {
    free(part);
    return -1;
  }
  int bad = 0;
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads) reduction(| : bad)
#endif
  {
    int t = 0, nt = 1;
#ifdef _OPENMP
    t = omp_get_thread_num();
    nt = omp_get_num_threads();
#endif
    uint64_t *out = part + (size_t)t * nout;
    const size_t nl = isa == ISA_SCALAR ? 0 : (size_t)p.lanes * g->nchunk;
    uint64_t *acc64 = nl ? aligned_alloc(64, (nl * 8 + 63) / 64 * 64) : NULL;
    int32_t *acc32 = nl && g->nbit == 8 ? aligned_alloc(64, (nl * 4 + 63) / 64 * 64) : NULL;
    if (nl && (!acc64 || (g->nbit == 8 && !acc32))) {
      bad = 1;
    } else {
      if (acc64) memset(acc64, 0, nl * 8);
      if (acc32) memset(acc32, 0, nl * 4);
      /* own tile first, then the neighbours' tiles in thread order */
      for (int k = 0; k < nt; k++) {
        const int v = (t + k) % nt;
        const uint64_t v0 = nf * v / nt, v1 = nf * (v + 1) / nt;
        const uint64_t npieces = (v1 - v0 + pf - 1) / pf;
        for (;;) {
          const uint64_t i = __atomic_fetch_add(&next[(size_t)v * 8], 1, __ATOMIC_RELAXED);
          if (i >= npieces) break;
          const uint64_t f0 = v0 + i * pf, f1 = f0 + pf < v1 ? f0 + pf : v1;
          if (isa == ISA_SCALAR) {
            run_scalar(g, buf, f0, f1, out);
          } else if (g->nbit == 8) {
            if (isa == ISA_VNNI) i8_vnni(g, &p, buf, f0, f1, acc32, acc64);
            else if (isa == ISA_AVX512) i8_avx512(g, &p, buf, f0, f1, acc32, acc64);
            else i8_avx2(g, &p, buf, f0, f1, acc32, acc64);
          } else {
            if (isa == ISA_AVX2) i16_avx2(g, &p, buf, f0, f1, acc64);
            else i16_avx512(g, &p, buf, f0, f1, acc64);
          }
        }
      }
      if (acc64) fold(g, &p, acc64, out);
    }
    free(acc64);
    free(acc32);
  }
  free(next);
  if (!bad)
    for (int t = 0; t < nthreads; t++)
      for (uint32_t j = 0; j < nout; j++) acc[j] += part[(size_t)t * nout + j];
  free(part);
  return bad ? -1 : 0;
}
