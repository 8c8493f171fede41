// CPU address model of the integrate path under ASan+UBSan (test only).
//
// Compiles the library's own index arithmetic (csrc/b2p_plan.h: the launch
// shape, a lane's channels, a workgroup's rows, the ragged row, the staging
// chunks) on the host and replays random cases through it exactly as
// b2p_push / push_host / b2p_integrate_kernel would:
//
//   * a random layout b2p_geom_check accepts, a random CU count and knobs;
//   * the integration cut into random host spans, each span its own malloc
//     of exactly its size (the caller's buffer);
//   * each span copied in staging chunks (stage_chunk) into two staging
//     buffers of exactly stage_bytes (malloc'd, so ASan sees their ends);
//   * each chunk "launched": every (workgroup, lane) of the grid reads the
//     vectors the kernel's indexing names, from the staging buffer, with a
//     per-vector read count.
//
// Checked per chunk: every load in bounds (ASan would also trap it), every
// vector read exactly once, every output slot < nout; per integration: the
// detected sums equal the C oracle's (orc_integrate) exactly.
//
//   plan_model CASES SEED     -> "plan model: N cases ok (...)" and exit 0
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "b2p_oracle.h"
#include "b2p_plan.h"

using namespace b2p;

static uint64_t rng_state;
static uint64_t rnd() { return rng_state = orc_splitmix64(rng_state); }
static uint64_t rnd_in(uint64_t lo, uint64_t hi) { return lo + rnd() % (hi - lo + 1); }

static int failures = 0;
#define REQUIRE(cond, ...)                     \
  do {                                         \
    if (!(cond)) {                             \
      fprintf(stderr, "FAIL %s: ", #cond);     \
      fprintf(stderr, __VA_ARGS__);            \
      fprintf(stderr, "\n");                   \
      failures++;                              \
      return -1;                               \
    }                                          \
  } while (0)

struct Case {
  orc_geom_t g;
  Shape sh;
  uint32_t interleave;
  uint64_t frame, block, stage;
};

// the detect of one 16-B vector's words into acc (the kernel's Acc8/Acc16)
static void detect(const Case &k, const uint8_t *v, const uint32_t *ch, uint64_t *acc) {
  const uint32_t npo = k.g.npol_out;
  for (uint32_t w = 0; w < k.sh.VW; ++w) {
    int64_t xr, xi, yr, yi;
    if (k.g.nbit == 8) {
      const int8_t *b = reinterpret_cast<const int8_t *>(v + 4 * w);
      xr = b[0], xi = b[1], yr = b[2], yi = b[3];
    } else if (k.g.big_endian) {
      int16_t l[4];
      orc_bmf_lanes(v + 8 * w, l);
      xr = l[0], xi = l[1], yr = l[2], yi = l[3];
    } else {
      int16_t l[4];
      memcpy(l, v + 8 * w, 8);
      xr = l[0], xi = l[1], yr = l[2], yi = l[3];
    }
    const uint64_t px = (uint64_t)(xr * xr + xi * xi), py = (uint64_t)(yr * yr + yi * yi);
    if (npo == 1) {
      acc[ch[w]] += px + py;
    } else {
      acc[ch[w] * 2] += px;
      acc[ch[w] * 2 + 1] += py;
    }
  }
}

template <int VW>
static int lane_chans(const Case &k, uint32_t pos, uint32_t *ch) {
  lane_channels<VW>(pos, k.g.nchunk, k.sh.FV, k.sh.IV, k.g.nchan_chunk, ch);
  return 0;
}

// one launch over a staging buffer of nvec valid vectors (exactly `cap`
// bytes allocated)
static int launch(const Case &k, const uint8_t *stage, uint64_t nvec, uint64_t *acc, std::vector<uint8_t> &seen) {
  const Shape &s = k.sh;
  const uint32_t nout = k.g.nchunk * k.g.nchan_chunk * k.g.npol_out;
  seen.assign(nvec, 0);
  const uint64_t full = nvec / s.S;
  for (uint32_t blk = 0; blk < s.NC * s.G; ++blk) {
    const uint32_t col = blk % s.NC, grp = blk / s.NC;
    for (uint32_t t = 0; t < s.B; ++t) {
      const uint32_t pos = col * s.B + t;
      REQUIRE(pos < s.S, "lane position %u of a %u-vector row", pos, s.S);
      uint32_t ch[4];
      if (s.VW == 4)
        lane_chans<4>(k, pos, ch);
      else
        lane_chans<2>(k, pos, ch);
      for (uint32_t w = 0; w < s.VW; ++w)
        REQUIRE(ch[w] * k.g.npol_out + k.g.npol_out - 1 < nout, "channel %u of %u outputs", ch[w], nout);
      uint64_t start, step, count;
      group_rows(full, grp, s.G, k.interleave, &start, &step, &count);
      for (uint64_t i = 0; i < count; ++i) {
        const uint64_t idx = (start + i * step) * s.S + pos;
        REQUIRE(idx < nvec, "load %llu of %llu (group %u lane %u)", (unsigned long long)idx,
                (unsigned long long)nvec, grp, t);
        seen[idx]++;
        detect(k, stage + idx * 16, ch, acc);
      }
      if (takes_ragged_row(grp, s.G, full, s.S, pos, nvec)) {
        const uint64_t idx = full * s.S + pos;
        REQUIRE(idx < nvec, "ragged load %llu of %llu", (unsigned long long)idx, (unsigned long long)nvec);
        seen[idx]++;
        detect(k, stage + idx * 16, ch, acc);
      }
    }
  }
  for (uint64_t v = 0; v < nvec; ++v)
    REQUIRE(seen[v] == 1, "vector %llu of %llu read %u times", (unsigned long long)v, (unsigned long long)nvec,
            seen[v]);
  return 0;
}

static int draw_case(Case &k) {
  memset(&k.g, 0, sizeof k.g);
  orc_geom_t &g = k.g;
  g.nbit = rnd_in(0, 1) ? 8 : 16;
  g.big_endian = g.nbit == 16 ? (uint32_t)rnd_in(0, 1) : 0;
  g.npol = g.ndim = 2;
  g.nchunk = (uint32_t)rnd_in(1, 64);
  g.nchan_chunk = (uint32_t)rnd_in(1, 96);
  const uint32_t word = 4 * g.nbit / 8;
  uint32_t base = 1;
  while ((base * g.nchan_chunk * word) % 16) base *= 2;
  g.nsamp_df = base * (uint32_t)rnd_in(1, 4);
  g.npol_out = (uint32_t)rnd_in(1, 2);
  if (g.nchunk * g.nchan_chunk * g.npol_out > 8192) g.nchunk = 8192 / (g.nchan_chunk * g.npol_out);
  k.frame = orc_frame_bytes(&g);
  const uint64_t max_frames = (2u << 20) / k.frame ? (2u << 20) / k.frame : 1;
  const uint64_t nframes = rnd_in(1, max_frames);
  g.nsamp_int = nframes * g.nsamp_df;
  k.block = nframes * k.frame;
  ShapeKnobs knobs{0, 0, 0, 0, 0};
  if (rnd_in(0, 3) == 0) knobs.row_groups = (int)rnd_in(1, 9);
  if (rnd_in(0, 5) == 0) knobs.max_threads = (int)(64 * rnd_in(1, 16));
  static const int cus[] = {1, 4, 32, 80, 256};
  char err[160];
  if (plan_shape(g.nbit, g.nchunk, g.nsamp_df, g.nchan_chunk, knobs, cus[rnd_in(0, 4)], &k.sh, err, sizeof err))
    return 1;  // refused by the planner (b2p_open would return B2P_EINVAL)
  // the library's row ownership rule (b2p_open): interleaved for int16 and
  // for rows over several columns; a tuning may force either
  k.interleave = rnd_in(0, 4) == 0 ? (uint32_t)rnd_in(0, 1) : (g.nbit == 16 || k.sh.NC > 1 ? 1u : 0u);
  // staging of 1 .. nframes+2 frames (stage_bytes_for keeps whole frames)
  k.stage = stage_bytes_for(rnd_in(0, (nframes + 2) * k.frame), k.frame);
  return 0;
}

int main(int argc, char **argv) {
  const long ncase = argc > 1 ? atol(argv[1]) : 200;
  rng_state = argc > 2 ? strtoull(argv[2], nullptr, 0) : 20181105;
  long done = 0, refused = 0, chunks = 0, pushes = 0;
  std::vector<uint8_t> seen;
  for (long c = 0; c < ncase && !failures; ++c) {
    Case k;
    if (draw_case(k)) {
      refused++;
      continue;
    }
    const uint32_t nout = k.g.nchunk * k.g.nchan_chunk * k.g.npol_out;
    std::vector<uint8_t> blockbuf(k.block);
    orc_fill_synthetic(&k.g, blockbuf.data(), k.block, 20181105, (uint32_t)c, 0, 0);
    std::vector<uint64_t> acc(nout, 0), want(nout, 0);
    // random cuts into pushes (frame-aligned host spans)
    const uint64_t nframes = k.block / k.frame;
    std::vector<uint64_t> cuts = {0};
    const int ncut = (int)rnd_in(0, 3);
    for (int i = 0; i < ncut && nframes > 1; ++i) cuts.push_back(rnd_in(1, nframes - 1));
    cuts.push_back(nframes);
    std::sort(cuts.begin(), cuts.end());
    // the two staging buffers, exactly stage bytes each
    uint8_t *stage[2] = {static_cast<uint8_t *>(malloc(k.stage)), static_cast<uint8_t *>(malloc(k.stage))};
    uint32_t stage_next = 0;
    for (size_t p = 0; p + 1 < cuts.size() && !failures; ++p) {
      const uint64_t nbytes = (cuts[p + 1] - cuts[p]) * k.frame;
      if (!nbytes) continue;
      uint8_t *span = static_cast<uint8_t *>(malloc(nbytes));  // the caller's buffer, exact size
      memcpy(span, blockbuf.data() + cuts[p] * k.frame, nbytes);
      pushes++;
      for (uint64_t off = 0; off < nbytes && !failures; off += k.stage) {
        const uint64_t n = stage_chunk(nbytes, k.stage, off);
        const int i = (int)(stage_next++ & 1);
        if (n == 0 || n > k.stage || n % k.frame || off + n > nbytes) {
          fprintf(stderr, "FAIL chunk %llu at %llu of %llu (stage %llu)\n", (unsigned long long)n,
                  (unsigned long long)off, (unsigned long long)nbytes, (unsigned long long)k.stage);
          failures++;
          break;
        }
        memcpy(stage[i], span + off, n);
        if (launch(k, stage[i], n / 16, acc.data(), seen)) {
          fprintf(stderr, "  case %ld: nbit %u be %u nchunk %u ncc %u nsamp_df %u npol_out %u frames %llu; "
                  "B %u S %u NC %u G %u interleave %u; chunk %llu B\n", c, k.g.nbit, k.g.big_endian,
                  k.g.nchunk, k.g.nchan_chunk, k.g.nsamp_df, k.g.npol_out, (unsigned long long)nframes,
                  k.sh.B, k.sh.S, k.sh.NC, k.sh.G, k.interleave, (unsigned long long)n);
          break;
        }
        chunks++;
      }
      free(span);
    }
    free(stage[0]);
    free(stage[1]);
    if (failures) break;
    if (orc_integrate(&k.g, blockbuf.data(), k.block, want.data()) != 0) {
      fprintf(stderr, "FAIL oracle refused case %ld\n", c);
      failures++;
      break;
    }
    for (uint32_t o = 0; o < nout; ++o)
      if (acc[o] != want[o]) {
        fprintf(stderr, "FAIL case %ld output %u: %llu != oracle %llu\n", c, o, (unsigned long long)acc[o],
                (unsigned long long)want[o]);
        failures++;
        break;
      }
    done++;
  }
  if (failures) return 1;
  printf("plan model: %ld cases ok (%ld refused by the planner, %ld pushes, %ld staging chunks)\n", done, refused,
         pushes, chunks);
  return 0;
}
