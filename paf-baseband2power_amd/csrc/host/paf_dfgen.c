/*
 * paf_dfgen -- synthetic BMF capture stream: turn a payload-only TFTFP DADA
 * file (what paf_diskdb reads) into the raw data-frame stream a beamformer
 * sends: 7232-B frames = 64-B header (include/b2p_df.h, the inverse of
 * hdr.c:10-28) + 7168-B payload, one per (frame, chunk), in arrival order.
 *
 *   paf_dfgen -i in.dada -o out.df -n NCHK [-x ref_idf] [-s ref_sec]
 *             [-b beam] [-e epoch] [-f freq0_MHz] [-r seed] [-l lost_per_mille]
 *             [-c chunks.u8] [-w window]
 * Frame k*NCHK + c carries chunk c and DF number ref_idf + k, wrapping into
 * the next 27-s period (sync.c:119-125); -r shuffles the arrival order
 * (within consecutive windows of -w frames, default the whole file), -l
 * drops frames; -c writes the per-frame chunk index (what capture derives
 * from the sender's IP, capture.c:571-584).
 */
#include <getopt.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "b2p_df.h"

static uint64_t rng_state;
static uint64_t rnd(void) { /* splitmix64 */
  uint64_t z = (rng_state += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

int main(int argc, char **argv) {
  const char *in = NULL, *out = NULL, *chunks = NULL;
  uint64_t ref_idf = 0, ref_sec = 0, seed = 0;
  int nchk = 48, beam = 0, epoch = 0, lost = 0, arg;
  uint64_t window = 0;
  double freq0 = 1300.0;
  while ((arg = getopt(argc, argv, "i:o:n:x:s:b:e:f:r:l:c:w:h")) != -1) {
    switch (arg) {
      case 'i': in = optarg; break;
      case 'o': out = optarg; break;
      case 'n': nchk = atoi(optarg); break;
      case 'x': ref_idf = strtoull(optarg, NULL, 10); break;
      case 's': ref_sec = strtoull(optarg, NULL, 10); break;
      case 'b': beam = atoi(optarg); break;
      case 'e': epoch = atoi(optarg); break;
      case 'f': freq0 = atof(optarg); break;
      case 'r': seed = strtoull(optarg, NULL, 10); break;
      case 'l': lost = atoi(optarg); break;
      case 'c': chunks = optarg; break;
      case 'w': window = strtoull(optarg, NULL, 10); break;
      default:
        fprintf(stdout, "paf_dfgen -i in.dada -o out.df -n NCHK [-x idf] [-s sec] [-b beam] "
                        "[-e epoch] [-f freq0] [-r seed] [-l lost_per_mille] [-c chunks.u8] [-w window]\n");
        return EXIT_FAILURE;
    }
  }
  if (!in || !out || nchk < 1 || nchk > 255) {
    fprintf(stderr, "paf_dfgen: -i, -o and 1 <= -n <= 255 are required\n");
    return EXIT_FAILURE;
  }
  FILE *fi = fopen(in, "rb");
  if (!fi) { perror(in); return EXIT_FAILURE; }
  fseek(fi, 0, SEEK_END);
  long long fsz = ftell(fi);
  if (fsz < 4096) { fprintf(stderr, "paf_dfgen: %s shorter than a DADA header\n", in); return EXIT_FAILURE; }
  const uint64_t pay = (uint64_t)fsz - 4096;
  if (pay % ((uint64_t)nchk * B2P_DF_PAYLOAD_BYTES)) {
    fprintf(stderr, "paf_dfgen: payload is not a whole number of %d-chunk frames\n", nchk);
    return EXIT_FAILURE;
  }
  const uint64_t n = pay / B2P_DF_PAYLOAD_BYTES;
  unsigned char *data = malloc(pay);
  uint64_t *order = malloc(n * sizeof(uint64_t));
  if (!data || !order) { fprintf(stderr, "paf_dfgen: out of memory\n"); return EXIT_FAILURE; }
  fseek(fi, 4096, SEEK_SET); /* diskdb.cu:69: skip the file's own header */
  if (fread(data, 1, pay, fi) != pay) { fprintf(stderr, "paf_dfgen: short read\n"); return EXIT_FAILURE; }
  fclose(fi);
  for (uint64_t k = 0; k < n; k++) order[k] = k;
  if (seed) { /* Fisher-Yates arrival order, window by window */
    rng_state = seed;
    const uint64_t w = window ? window : n;
    for (uint64_t w0 = 0; w0 < n; w0 += w) {
      const uint64_t m = n - w0 < w ? n - w0 : w;
      for (uint64_t k = m - 1; k > 0; k--) {
        uint64_t j = rnd() % (k + 1), t = order[w0 + k];
        order[w0 + k] = order[w0 + j];
        order[w0 + j] = t;
      }
    }
  }
  FILE *fo = fopen(out, "wb");
  FILE *fc = chunks ? fopen(chunks, "wb") : NULL;
  if (!fo || (chunks && !fc)) { perror("paf_dfgen: output"); return EXIT_FAILURE; }
  rng_state = seed ^ 0x5DEECE66DULL;
  unsigned char df[B2P_DF_BYTES];
  uint64_t written = 0;
  for (uint64_t q = 0; q < n; q++) {
    const uint64_t k = order[q];
    if (lost && (int)(rnd() % 1000) < lost) continue;
    const uint64_t t = k / nchk, c = k % nchk;
    b2p_df_hdr_t h = {1, ref_idf, ref_sec, epoch, beam, freq0 + (double)c};
    b2p_df_ref_advance(&h, t);
    b2p_df_encode(&h, df);
    memcpy(df + B2P_DF_HDR_BYTES, data + k * B2P_DF_PAYLOAD_BYTES, B2P_DF_PAYLOAD_BYTES);
    if (fwrite(df, 1, sizeof df, fo) != sizeof df) { perror("write"); return EXIT_FAILURE; }
    if (fc) fputc((int)c, fc);
    written++;
  }
  fclose(fo);
  if (fc) fclose(fc);
  fprintf(stderr, "paf_dfgen: %" PRIu64 " of %" PRIu64 " frames written\n", written, n);
  free(data);
  free(order);
  return EXIT_SUCCESS;
}
