// Index arithmetic of the integrate path, shared by the HIP library and a
// CPU address model.
//
// Everything that decides WHICH bytes a launch reads lives here:
//  * the launch shape (plan_shape: workgroup width B, row S, columns NC, row
//    groups G) -- called by b2p_open (b2p_ctx.hip);
//  * a lane's channels and its workgroup's rows (lane_channels, group_rows,
//    takes_ragged_row) -- called by b2p_integrate_kernel (b2p_kernels.hip);
//  * the host-span staging chunks (stage_bytes_for, stage_chunk) -- called
//    by push_host (b2p_ctx.hip).
// tests/c/plan_model.cpp compiles this same header on the CPU under
// ASan+UBSan, replays random layouts, staging sizes and push cuts through it
// with exact-size allocations, and checks that every vector of every span
// is read exactly once and lands on the oracle's spectrum
// (tests/test_sanitizers.py::test_staging_and_addressing_model_under_asan).
// Plain integers only: no HIP types, so a host compiler takes it as is.
#pragma once

#include <stdint.h>
#include <stdio.h>

#if defined(__HIP__)
#define B2P_HD __host__ __device__ __forceinline__
#else
#define B2P_HD inline
#endif

namespace b2p {

B2P_HD uint32_t gcd_u32(uint32_t a, uint32_t b) {
  while (b) {
    uint32_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}

// ---- launch shape ----------------------------------------------------------
struct Shape {
  uint32_t VW;    // words per 16-B vector (4 int8, 2 int16)
  uint32_t IV;    // vectors per chunk
  uint32_t FV;    // vectors per frame
  uint32_t CP;    // channel period in vectors
  uint32_t B;     // active threads per workgroup
  uint32_t Bpad;  // B rounded up to whole waves
  uint32_t S;     // vectors per row
  uint32_t NC;    // workgroups across a row
  uint32_t G;     // row groups
  uint32_t nrep;  // accumulator replicas
};

// the b2p_tuning_t fields the shape depends on (0 = measured default)
struct ShapeKnobs {
  int max_threads, threads, wg_per_cu, row_groups, replicas;
};

// Choose the workgroup shape (DESIGN.md "integrate kernel / launch shape").
// Returns 0, or -1 with a message in err.
inline int plan_shape(uint32_t nbit, uint32_t nchunk, uint32_t nsamp_df, uint32_t nchan_chunk,
                      const ShapeKnobs &t, int ncu, Shape *c, char *err, size_t errlen) {
  const uint32_t wb = 4 * nbit / 8;  // npol 2 x ndim 2
  c->VW = 16 / wb;
  c->IV = nsamp_df * nchan_chunk / c->VW;
  c->FV = nchunk * c->IV;
  const uint32_t P = nchan_chunk / gcd_u32(nchan_chunk, c->VW);
  c->CP = nchunk == 1 ? P : c->FV;
  uint32_t maxT = nbit == 8 ? 512 : 448;
  if (t.max_threads) maxT = (uint32_t)t.max_threads;
  const uint32_t L = c->CP / gcd_u32(c->CP, 64) * 64;  // lcm(CP, 64)
  uint32_t colB = 0;  // whole-wave divisor of L for a row split into columns
  if (c->CP <= maxT && L > maxT && nchunk == 1)
    for (uint32_t b = maxT / 64 * 64; b >= 256 && !colB; b -= 64)
      if (L % b == 0) colB = b;
  if (c->CP <= maxT && !colB) {
    c->B = L <= maxT ? (maxT / L) * L : (maxT / c->CP) * c->CP;
    c->S = c->B;
    c->NC = 1;
  } else if (colB) {
    // the channel period fits a workgroup but not in whole waves (e.g. 336
    // int8 channels = 84 vectors): a row of lcm(period, 64) vectors split
    // into whole-wave columns keeps every lane on fixed channels without a
    // partial wave (504 threads measured 6.3 TB/s, tools/perf_matrix.py)
    c->B = colB;
    c->S = L;
    c->NC = L / colB;
  } else {
    // the frame is split into NC = CP / B columns: the largest whole-wave B
    // (multiple of 64) that divides the frame -- partial waves straddle
    // 1-KiB lines and measured 10-15 % slower (BMF: 168 or 336 threads)
    uint32_t best = 0;
    for (uint32_t b = maxT / 64 * 64; b >= 64; b -= 64)
      if (c->CP % b == 0) {
        best = b;
        break;
      }
    // a power-of-two frame (TFTFP 8x8 int16: 4096 vectors) divides into 256
    // under the int16 cap; 512-thread columns, one per CU, measured 2-4 %
    // faster there (8 KiB contiguous per row and workgroup), while BMF keeps
    // 448 (512 measured 2.7 % slower; profiles/archive/r03_tune_frame_split.jsonl)
    if (!t.max_threads && best && best <= 256 && maxT < 512 && c->CP % 512 == 0) best = 512;
    if (t.threads) {  // tuning: an exact whole-wave divisor of the frame
      if (c->CP % (uint32_t)t.threads) {
        snprintf(err, errlen, "tuning threads %d does not divide the %u-vector frame", t.threads, c->CP);
        return -1;
      }
      best = (uint32_t)t.threads;
    }
    if (best) {
      c->B = best;
      c->S = c->CP;
      c->NC = c->CP / c->B;
    } else {
      // no whole-wave divisor (e.g. 61 chunks x 11 vectors): rows of
      // lcm(frame, 64) vectors, split into whole-wave columns (64 always
      // divides), so every lane still keeps its channels
      const uint64_t rowv = (uint64_t)c->CP / gcd_u32(c->CP, 64) * 64;
      if (rowv > 0x7fffffffull) {
        snprintf(err, errlen, "frame of %u vectors too large", c->CP);
        return -1;
      }
      uint32_t b = maxT / 64 * 64;
      while (b > 64 && rowv % b) b -= 64;
      c->B = b;
      c->S = (uint32_t)rowv;
      c->NC = (uint32_t)(rowv / b);
    }
  }
  c->Bpad = (c->B + 63) / 64 * 64;
  // one workgroup per CU: with ~32 KiB of loads in flight per CU more
  // resident waves only cost bandwidth (tools/tune.py sweep)
  // ... counted as ~8 waves: a narrower workgroup (a frame that only
  // divides into 256-thread columns) gets two per CU
  uint32_t per_cu = 512 / c->Bpad;
  if (per_cu < 1) per_cu = 1;
  if (t.wg_per_cu) per_cu = (uint32_t)t.wg_per_cu;
  const uint32_t target = (uint32_t)ncu * per_cu;
  c->G = (target + c->NC / 2) / c->NC;
  if (c->G < 1) c->G = 1;
  if (t.row_groups) c->G = (uint32_t)t.row_groups;  // e.g. long per-lane runs in tests
  c->nrep = t.replicas ? (uint32_t)t.replicas : 16;
  return 0;
}

// ---- what one lane of one workgroup reads ----------------------------------
// Channels of the VW word slots of the lane at vector position pos of a row
// (fixed for the whole launch).  A row may hold several frames: fold first.
template <int VW>
B2P_HD void lane_channels(uint32_t pos, uint32_t nchunk, uint32_t FV, uint32_t IV, uint32_t nchan_chunk,
                          uint32_t ch[VW]) {
  const uint32_t fpos = nchunk == 1 ? pos : pos % FV;
  const uint32_t chunk = nchunk == 1 ? 0u : fpos / IV;
  const uint32_t q = nchunk == 1 ? pos : fpos % IV;
#pragma unroll
  for (int w = 0; w < VW; ++w) ch[w] = chunk * nchan_chunk + (q * VW + w) % nchan_chunk;
}

// The rows of row group grp among the `full` whole rows of a span:
// start + i * step, i < count.  interleave 1: rows grp, grp+G, ...;
// interleave 0: a contiguous slice.
B2P_HD void group_rows(uint64_t full, uint32_t grp, uint32_t G, uint32_t interleave, uint64_t *start,
                       uint64_t *step, uint64_t *count) {
  if (interleave) {
    *start = grp;
    *step = G;
    *count = full > grp ? (full - grp + G - 1) / G : 0;
  } else {
    *start = (uint64_t)grp * full / G;
    *step = 1;
    *count = (uint64_t)(grp + 1) * full / G - *start;
  }
}

// The ragged last row (a span that is not a whole number of rows): the last
// group of every column reads vector full*S + pos when it exists.
B2P_HD bool takes_ragged_row(uint32_t grp, uint32_t G, uint64_t full, uint32_t S, uint32_t pos, uint64_t nvec) {
  return grp == G - 1 && full * S + pos < nvec;
}

// ---- host-span staging -----------------------------------------------------
// A staging buffer holds a whole number of frames (at least one).
inline uint64_t stage_bytes_for(uint64_t want, uint64_t frame_bytes) {
  const uint64_t sb = want / frame_bytes * frame_bytes;
  return sb ? sb : frame_bytes;
}

// Bytes of the staging chunk that starts at byte off of an nbytes span.
inline uint64_t stage_chunk(uint64_t nbytes, uint64_t stage_bytes, uint64_t off) {
  return nbytes - off < stage_bytes ? nbytes - off : stage_bytes;
}

}  // namespace b2p
