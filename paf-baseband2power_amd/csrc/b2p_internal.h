// Internal interface between the C-ABI context (b2p_ctx.hip) and the gfx950
// kernels (b2p_kernels.hip).  Not installed; include/b2p.h is the boundary.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace b2p {

// ring blocks one launch may integrate back to back (b2p_integrate_n)
constexpr uint32_t kMaxBlk = 8;

enum Mode : int { kI8 = 0, kI16LE = 1, kI16BE = 2 };

// One launch of the detect+integrate kernel over one pushed span.
// The span is viewed as rows of S 16-B vectors; workgroup (col, grp) owns
// the vectors [col*B, col*B+B) of every row in its row range, so each thread
// sees the same channels in every row and keeps its partial sums in
// registers (DESIGN.md "integrate kernel").
struct IntegrateArgs {
  const uint4 *data;            // span base, 16-B aligned, frame-aligned
  uint64_t nvec;                // 16-B vectors in the span
  uint32_t S;                   // vectors per row
  uint32_t B;                   // active threads per workgroup
  uint32_t NC;                  // workgroups across a row (S / B, or 1)
  uint32_t G;                   // row groups
  uint32_t IV;                  // vectors per chunk (nsamp_df*nchan_chunk/VW)
  uint32_t FV;                  // vectors per frame (nchunk*IV)
  uint32_t nchunk;
  uint32_t nchan_chunk;
  uint32_t nout;                // nchan * npol_out
  uint32_t nrep;                // accumulator replicas
  uint32_t interleave;          // 1: group g owns rows g, g+G, ...; 0: a slice
  unsigned long long *rep;      // [nrep][nout] exact sums
  // in-launch finalize (null out: the finalize kernel runs later instead)
  float *out;                   // nout fp32, written by the last workgroup
  uint32_t *ticket;             // arrival counter, 0 between launches
  uint32_t mean;
  double nsamp;
  // deferred finalize of the previous integration, done by the LAST
  // workgroup of this launch (grid = NC*G + 1) when fin_out is set
  unsigned long long *fin_rep;  // its replica set (re-zeroed)
  float *fin_out;
  uint32_t fin_raw;             // 1: fin_out receives the exact uint64 sums
  uint32_t nwork;               // streaming workgroups (NC*G)
  // several whole integrations in one launch (b2p_integrate_n): block b is
  // read from blk[b] and sums into rep + b * set_words; the carried
  // finalize then covers fin_nblk sets into fin_out + b * nout
  uint32_t nblk;                // 1: the single span at data
  uint32_t fin_nblk;
  uint64_t set_words;           // nrep * nout
  const uint4 *blk[kMaxBlk];
  // debug build only (B2P_DEBUG): where out-of-bounds accesses are recorded
  // (b2p_kernels.hip dbg_record); null and unused in the release library
  unsigned long long *dbg;
  uint64_t dbg_bound;           // the bound loads are checked against (nvec)
};

struct FinalizeArgs {
  unsigned long long *rep;      // zeroed as it is read
  uint32_t nrep;
  uint32_t nout;
  float *out;
  uint32_t mean;
  double nsamp;
  uint32_t raw;                 // 1: out receives the exact uint64 sums
  uint32_t nblk;                // sets (grid.y): set b at rep + b * nrep * nout -> out + b * nout
};

// fp32 from exact sums that were reduced elsewhere (b2p_finalize_sums)
struct ConvertArgs {
  const unsigned long long *sums;
  float *out;
  uint64_t n;
  uint32_t mean;
  double nsamp;
};

// dst[i] = sum over r < nrows of src[r*count + i] (b2p_group_reduce, mode 1)
struct SumRowsArgs {
  const unsigned long long *src;
  unsigned long long *dst;
  uint64_t count;
  uint32_t nrows;
};

struct FillArgs {
  uint64_t key;                 // splitmix key of (seed, subband, block)
  uint64_t elem0;
  uint32_t elem_bytes;          // 1 or 2
  uint32_t big_endian;
  uint32_t comp;                // npol*ndim
  uint32_t nchan_chunk;
  uint64_t wpc;                 // words per chunk (nsamp_df*nchan_chunk)
  uint64_t wpf;                 // words per frame
  uint32_t nchan;
  int32_t amp;
};

// TFTFP assembly of a raw data-frame stream (b2p_assemble)
struct AssembleArgs {
  const unsigned char *dfs;     // ndf frames of df_bytes (header + payload)
  uint64_t ndf;
  uint32_t df_bytes;            // 7232
  uint32_t hdr_bytes;           // 64
  const uint8_t *chunk_of_df;   // per frame: chunk (ifreq) index
  uint64_t ref_idf, ref_sec;    // reference frame of the block
  unsigned char *block;         // block_ndf x nchunk x 7168 B
  uint64_t block_ndf;
  uint32_t nchunk;
  unsigned long long *counts;   // nchunk placed, then before / after / bad chunk
};
hipError_t launch_assemble(const AssembleArgs &a, uint32_t grid_cap, hipStream_t s);
hipError_t launch_convert(const ConvertArgs &a, hipStream_t s);
hipError_t launch_warm(hipStream_t s);
hipError_t launch_sum_rows(const SumRowsArgs &a, hipStream_t s);

// which instantiation of the integrate kernel runs
struct KernelChoice {
  int mode;       // Mode
  int npol_out;   // 1 or 2
  int unroll;     // 4, 8 or 16 rows in flight per lane
  bool nt;        // non-temporal loads
};

// ev0/ev1 may be null; when set they time the dispatch (hipExtLaunchKernel)
hipError_t launch_integrate(const IntegrateArgs &a, const KernelChoice &k,
                            uint32_t block_threads, uint32_t grid, hipStream_t s,
                            hipEvent_t ev0, hipEvent_t ev1);
hipError_t occupancy_integrate(const KernelChoice &k, uint32_t threads,
                               size_t lds_bytes, int *blocks_per_cu);
hipError_t launch_finalize(const FinalizeArgs &a, hipStream_t s, hipEvent_t ev0,
                           hipEvent_t ev1);
hipError_t launch_fill(uint4 *dst, uint64_t nvec, const FillArgs &f,
                       hipStream_t s);
uint64_t splitmix64_host(uint64_t x);

}  // namespace b2p

// library-internal hooks for b2p_group.hip (not part of include/b2p.h)
struct b2p_ctx;
void *b2p_internal_stream(struct b2p_ctx *ctx);  // the context's current stream
int b2p_internal_flush(struct b2p_ctx *ctx);     // enqueue a deferred finalize
// the event b2p_fence recorded for `ticket` (one of the last 8), or null
void *b2p_internal_fence_event(struct b2p_ctx *ctx, uint64_t ticket);
