// gfx950 kernels of the baseband->power integrator.
//
// Replaces the empty kernel module of the reference (kernel.cu:1-7,
// kernel.cuh:1-9): unpack -> |X|^2 + |Y|^2 -> 1024x1024-sample time sum
// (README.md:2, paf_baseband2power.cu:20).
//
// The path is a streaming map-reduce at ~1-2 integer ops per byte, bound by
// HBM read bandwidth (DESIGN.md "roofline"), so the kernel is built around
// the load stream, not arithmetic:
//  * every lane issues 16-B global_load_dwordx4 and a wave covers 1 KiB of
//    contiguous baseband per instruction;
//  * a lane keeps the same 16-B position inside a row for the whole launch,
//    so its channels are loop-invariant and its partial sums live in
//    registers (no LDS traffic in the stream);
//  * int8 words [X.re X.im Y.re Y.im] are detected with ONE v_dot4c_i32_i8
//    per word (dot(w, w) = |X|^2 + |Y|^2), accumulated exactly in 32 bits and
//    widened to 64 bits every 32768 rows;
//  * int16 big-endian BMF words are byte-swapped per 16-bit lane with one
//    v_perm_b32 per dword (the BSWAP_64 of cudautil.cuh:118-125, applied to
//    the halves) and detected with v_dot2c_i32_i16, summed in 64 bits;
//  * per-workgroup reduction through LDS 64-bit atomics, then one 64-bit
//    global atomic per touched output into one of nrep replicas (exact
//    integers: the result does not depend on arrival order).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "b2p_internal.h"
#include "b2p_plan.h"

namespace b2p {

typedef short short2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// rows a lane may accumulate in 32 bits before widening: a row adds at most
// 4*128^2 = 2^16 per int8 word, so 2^15 rows stay below 2^31.
constexpr uint32_t kFlushRows = 32768;

__device__ __forceinline__ uint32_t pol_power16(uint32_t d, bool be) {
  if (be) d = __builtin_amdgcn_perm(d, d, 0x02030001u);  // swap bytes in each half
  short2_t s = __builtin_bit_cast(short2_t, d);
  // re^2 + im^2 <= 2^31: exact as uint32 (the int32 result may read -2^31)
  return (uint32_t)__builtin_amdgcn_sdot2(s, s, 0, false);
}

template <int MODE, int NPO>
struct Acc;

// ---- int8: 4 words per 16-B vector --------------------------------------
template <int NPO>
struct Acc8 {
  unsigned long long tot[4][NPO];
  uint32_t s[4][NPO];
  __device__ __forceinline__ void zero_all() {
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int p = 0; p < NPO; ++p) tot[w][p] = 0, s[w][p] = 0;
  }
  __device__ __forceinline__ void add(const u32x4 v) {
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      if (NPO == 1) {
        s[w][0] = (uint32_t)__builtin_amdgcn_sdot4((int)d[w], (int)d[w], (int)s[w][0], false);
      } else {
        // s[w][0] = |X|^2 (bytes 0,1), s[w][1] = |X|^2 + |Y|^2
        s[w][0] = (uint32_t)__builtin_amdgcn_sdot4((int)(d[w] & 0xffffu), (int)d[w],
                                                  (int)s[w][0], false);
        s[w][1] = (uint32_t)__builtin_amdgcn_sdot4((int)d[w], (int)d[w], (int)s[w][1], false);
      }
    }
  }
  __device__ __forceinline__ void flush() {
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      if (NPO == 1) {
        tot[w][0] += s[w][0];
      } else {
        tot[w][0] += s[w][0];
        tot[w][1] += s[w][1] - s[w][0];  // |Y|^2, exact mod 2^32
      }
#pragma unroll
      for (int p = 0; p < NPO; ++p) s[w][p] = 0;
    }
  }
  __device__ __forceinline__ unsigned long long get(int w, int p) const { return tot[w][p]; }
};

// ---- int16: 2 words (4 dwords) per 16-B vector -----------------------------
template <bool BE, int NPO>
struct Acc16 {
  unsigned long long tot[2][NPO];
  __device__ __forceinline__ void zero_all() {
#pragma unroll
    for (int w = 0; w < 2; ++w)
#pragma unroll
      for (int p = 0; p < NPO; ++p) tot[w][p] = 0;
  }
  __device__ __forceinline__ void add(const u32x4 v) {
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      // BE (BSWAP_64 convention): bytes 4-7 hold X (lanes 0,1), bytes 0-3 Y.
      // LE: bytes 0-3 hold X, 4-7 Y.
      const uint32_t p0 = pol_power16(d[2 * w], BE);
      const uint32_t p1 = pol_power16(d[2 * w + 1], BE);
      const uint32_t px = BE ? p1 : p0, py = BE ? p0 : p1;
      if (NPO == 1) {
        tot[w][0] += (unsigned long long)px + py;
      } else {
        tot[w][0] += px;
        tot[w][1] += py;
      }
    }
  }
  __device__ __forceinline__ void flush() {}
  __device__ __forceinline__ unsigned long long get(int w, int p) const { return tot[w][p]; }
};

template <int NPO> struct Acc<kI8, NPO> : Acc8<NPO> { static constexpr int VW = 4; };
template <int NPO> struct Acc<kI16LE, NPO> : Acc16<false, NPO> { static constexpr int VW = 2; };
template <int NPO> struct Acc<kI16BE, NPO> : Acc16<true, NPO> { static constexpr int VW = 2; };

template <bool NT>
__device__ __forceinline__ u32x4 stream_load(const u32x4 *p) {
  if (NT) return __builtin_nontemporal_load(p);  // read-once stream: nt cache policy
  return *p;
}

#ifdef B2P_DEBUG
// Debug build (make B2P_DEBUG=1 -> lib/debug/libpafb2p.so): every access the
// launch would make outside its span or its outputs is recorded in a.dbg
// instead of being made -- [0] count, [1] kind (1 load, 2 output slot),
// [2] offending index, [3] its bound, [4] workgroup << 32 | thread -- and the
// host turns a non-zero count into an error naming the access (b2p_ctx.hip
// dbg_check).  Plain vector-memory atomics and stores.
__device__ __noinline__ void dbg_record(unsigned long long *dbg, uint64_t kind, uint64_t idx, uint64_t bound) {
  if (atomicAdd(&dbg[0], 1ull) == 0) {
    dbg[1] = kind;
    dbg[2] = idx;
    dbg[3] = bound;
    dbg[4] = ((unsigned long long)blockIdx.x << 32) | threadIdx.x;
  }
}
#endif

// A load of the span: in a debug build, checked against the span's nvec
// vectors (an out-of-span load is recorded and not made).
template <bool NT>
__device__ __forceinline__ u32x4 checked_load(const IntegrateArgs &a, const u32x4 *data, const u32x4 *p) {
#ifdef B2P_DEBUG
  const uint64_t idx = (uint64_t)(p - data);
  if (idx >= a.dbg_bound) {
    dbg_record(a.dbg, 1, idx, a.dbg_bound);
    return u32x4{0u, 0u, 0u, 0u};
  }
#else
  (void)a, (void)data;
#endif
  return stream_load<NT>(p);
}

__device__ __forceinline__ float to_output(unsigned long long tot, uint32_t mean, double nsamp) {
  // tot < 2^53: the double is exact, the float conversion is the one RNE
  const double d = (double)tot;
  return mean ? (float)(d / nsamp) : (float)d;
}

// UNROLL rows are loaded before any is consumed (UNROLL x 1 KiB in flight
// per wave); NT selects the non-temporal load policy.  Both are tuning
// variants (b2p_tuning_t unroll / nontemporal) measured on the box, see DESIGN.md.
//
// Row mapping (a.interleave): 0 = row group g owns a contiguous slice of the
// rows; 1 = group g owns rows g, g+G, g+2G, ... so that the whole grid
// sweeps the span front to back together (the probe in tools/hbm_probe.hip
// reads faster that way).  Either way a lane's channels never change.
//
// MULTI: the launch carries several queued blocks (b2p_integrate_n, a.nblk >
// 1) rather than one.  The two shapes are separate instantiations so that a
// rocprofv3 summary lists them as separate kernels (bench.py times both).
template <int MODE, int NPO, int UNROLL, bool NT, bool MULTI>
__global__ void __launch_bounds__(1024)
b2p_integrate_kernel(IntegrateArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds[];
  __shared__ uint32_t s_last;
  using A = Acc<MODE, NPO>;
  constexpr int VW = A::VW;
  const uint32_t t = threadIdx.x;
  for (uint32_t j = t; j < a.nout; j += blockDim.x) lds[j] = 0;

  if (a.fin_out && blockIdx.x == gridDim.x - 1) {
    // the previous launch's finalize (its sets were completed by the
    // previous launch on this stream; this launch sums into other sets):
    // one set per integration it carried
    const uint32_t nwords = a.nrep * a.nout;
    for (uint32_t b = 0; b < a.fin_nblk; ++b) {
      unsigned long long *fr = a.fin_rep + (uint64_t)b * a.set_words;
      if (b) {
        __syncthreads();
        for (uint32_t j = t; j < a.nout; j += blockDim.x) lds[j] = 0;
      }
      __syncthreads();
      for (uint32_t k = t; k < nwords; k += blockDim.x) {
        const unsigned long long x = fr[k];
        if (x) atomicAdd(&lds[k % a.nout], x);
        fr[k] = 0;
      }
      __syncthreads();
      if (a.fin_raw)
        for (uint32_t j = t; j < a.nout; j += blockDim.x)
          reinterpret_cast<unsigned long long *>(a.fin_out)[(uint64_t)b * a.nout + j] = lds[j];
      else
        for (uint32_t j = t; j < a.nout; j += blockDim.x)
          a.fin_out[(uint64_t)b * a.nout + j] = to_output(lds[j], a.mean, a.nsamp);
    }
    return;
  }
  const uint32_t col = blockIdx.x % a.NC;
  const uint32_t grp = blockIdx.x / a.NC;
  const bool active = t < a.B;
  const uint32_t pos = col * a.B + t;  // vector position inside a row

  // channels of this lane's VW word slots (fixed for the whole launch)
  uint32_t ch[VW];
  lane_channels<VW>(pos, a.nchunk, a.FV, a.IV, a.nchan_chunk, ch);

  const uint64_t full = a.nvec / a.S;  // rows with every vector valid
  // this group's rows: rstart + i * rstep, i < rcount
  uint64_t rstart, rstep, rcount;
  group_rows(full, grp, a.G, a.interleave, &rstart, &rstep, &rcount);
  // one integration per block: the rows of block b stream through the same
  // lanes (same channels), then the workgroup's sums go to block b's set
  const uint32_t nblk = MULTI ? a.nblk : 1u;
  for (uint32_t b = 0; b < nblk; ++b) {
  const u32x4 *data = reinterpret_cast<const u32x4 *>(MULTI ? a.blk[b] : a.data);
  A acc;
  acc.zero_all();
  if (b) {  // LDS of the previous block was drained into its set
    __syncthreads();
    for (uint32_t j = t; j < a.nout; j += blockDim.x) lds[j] = 0;
  }
  if (active) {
    // row offsets are wave-uniform (scalar); the lane offset is invariant
    const u32x4 *p = data + rstart * a.S + pos;
    const uint64_t stepv = rstep * a.S;
    uint64_t i = 0;
    while (i < rcount) {
      const uint64_t iend = (rcount - i > kFlushRows) ? i + kFlushRows : rcount;
      for (; i + UNROLL <= iend; i += UNROLL) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = checked_load<NT>(a, data, p + u * stepv);
        p += UNROLL * stepv;
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc.add(v[u]);
      }
      for (; i < iend; ++i, p += stepv) acc.add(checked_load<NT>(a, data, p));
      acc.flush();
    }
    // ragged last row (span not a whole number of rows): the last group of
    // every column takes it, its lanes keep their channels
    if (takes_ragged_row(grp, a.G, full, a.S, pos, a.nvec)) {
      acc.add(checked_load<false>(a, data, data + full * a.S + pos));
      acc.flush();
    }
  }
  __syncthreads();
  if (active) {
#pragma unroll
    for (int w = 0; w < VW; ++w)
#pragma unroll
      for (int p = 0; p < NPO; ++p) {
        const unsigned long long x = acc.get(w, p);
#ifdef B2P_DEBUG
        if (ch[w] * NPO + p >= a.nout) {
          dbg_record(a.dbg, 2, ch[w] * NPO + p, a.nout);
          continue;
        }
#endif
        if (x) atomicAdd(&lds[ch[w] * NPO + p], x);
      }
  }
  __syncthreads();
  unsigned long long *rep = a.rep + (uint64_t)b * a.set_words + (uint64_t)(blockIdx.x % a.nrep) * a.nout;
  for (uint32_t j = t; j < a.nout; j += blockDim.x) {
    const unsigned long long x = lds[j];
    if (x) atomicAdd(&rep[j], x);
  }
  }  // blocks
  if (!a.out) return;

  // ---- in-launch finalize by the last workgroup to arrive ----------------
  // (cdna_hip_programming.md Guideline 16 / MI355X_MICROARCH.md "Valid
  // forms"): every wave drains its replica atomics, the workgroup meets at a
  // barrier, one lane releases at agent scope and takes a ticket; the
  // workgroup holding the last ticket acquires and reads the replicas with
  // agent-scope (L1-bypassing) loads.  Integer sums: arrival order is moot.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t ticket =
        __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = ticket == a.nwork - 1;  // the carried-finalize block takes no ticket
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!s_last) return;
  // every (replica, output) word read by its own lane -- all loads in flight
  // at once -- and folded per output through LDS
  for (uint32_t j = t; j < a.nout; j += blockDim.x) lds[j] = 0;
  __syncthreads();
  const uint32_t nwords = a.nrep * a.nout;
  for (uint32_t k = t; k < nwords; k += blockDim.x) {
    const unsigned long long x =
        __hip_atomic_load(a.rep + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (x) atomicAdd(&lds[k % a.nout], x);
    a.rep[k] = 0;
  }
  __syncthreads();
  for (uint32_t j = t; j < a.nout; j += blockDim.x) a.out[j] = to_output(lds[j], a.mean, a.nsamp);
  if (t == 0) __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sum the replicas, emit fp32 with one RNE rounding, zero the replicas.
// 256 threads = 4 waves per 64 outputs; wave w sums replicas w, w+4, ...
__global__ void __launch_bounds__(256) b2p_finalize_kernel(FinalizeArgs a) {
  __shared__ unsigned long long part[4][64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t j = blockIdx.x * 64 + lane;
  unsigned long long *set = a.rep + (uint64_t)blockIdx.y * a.nrep * a.nout;  // integration y
  float *out = a.out + (uint64_t)blockIdx.y * a.nout * (a.raw ? 2 : 1);
  unsigned long long s = 0;
  if (j < a.nout) {
    for (uint32_t r = w; r < a.nrep; r += 4) {
      unsigned long long *p = set + (uint64_t)r * a.nout + j;
      s += *p;
      *p = 0;
    }
  }
  part[w][lane] = s;
  __syncthreads();
  if (w == 0 && j < a.nout) {
    const unsigned long long tot = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
    if (a.raw)
      reinterpret_cast<unsigned long long *>(out)[j] = tot;
    else
      out[j] = to_output(tot, a.mean, a.nsamp);
  }
}

__global__ void __launch_bounds__(256) b2p_convert_kernel(ConvertArgs a) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n;
       i += (uint64_t)gridDim.x * blockDim.x)
    a.out[i] = to_output(a.sums[i], a.mean, a.nsamp);
}

__global__ void __launch_bounds__(256) b2p_sum_rows_kernel(SumRowsArgs a) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.count;
       i += (uint64_t)gridDim.x * blockDim.x) {
    unsigned long long s = 0;
    for (uint32_t r = 0; r < a.nrows; ++r) s += a.src[(uint64_t)r * a.count + i];
    a.dst[i] = s;
  }
}

// ---- synthetic baseband (same generator as oracle/b2p_oracle.c) -----------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__device__ __forceinline__ int32_t synth_value(const FillArgs &f, uint64_t e) {
  const uint64_t r = splitmix64(f.key + e);
  const int64_t gs = (int64_t)(r & 0xffff) + (int64_t)((r >> 16) & 0xffff) +
                     (int64_t)((r >> 32) & 0xffff) + (int64_t)(r >> 48) - 131070;
  const uint64_t wf = (e / f.comp) % f.wpf;
  const uint32_t ch = (uint32_t)((wf / f.wpc) * f.nchan_chunk + wf % f.nchan_chunk);
  const int64_t amp = (ch == 0 || ch == 7 || ch == f.nchan - 1) ? 2 * f.amp : f.amp;
  int64_t v = (gs * amp) >> 16;
  const int64_t lo = f.elem_bytes == 1 ? -128 : -32768, hi = f.elem_bytes == 1 ? 127 : 32767;
  v = v < lo ? lo : (v > hi ? hi : v);
  return (int32_t)v;
}

__global__ void __launch_bounds__(256) b2p_fill_kernel(uint4 *dst, uint64_t nvec, FillArgs f) {
  for (uint64_t vi = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; vi < nvec;
       vi += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t d[4];
    if (f.elem_bytes == 1) {
      const uint64_t e0 = f.elem0 + vi * 16;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        uint32_t x = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b)
          x |= ((uint32_t)(uint8_t)(int8_t)synth_value(f, e0 + 4 * k + b)) << (8 * b);
        d[k] = x;
      }
    } else {
      const uint64_t e0 = f.elem0 + vi * 8;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        uint32_t x = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          uint32_t u = (uint16_t)(int16_t)synth_value(f, e0 + 2 * k + h);
          if (f.big_endian) u = ((u & 0xff) << 8) | (u >> 8);
          x |= u << (16 * h);
        }
        d[k] = x;
      }
    }
    dst[vi] = make_uint4(d[0], d[1], d[2], d[3]);
  }
}

// ---- TFTFP assembly of a raw DF stream (capture.c:527-547) ------------------
// One wave per data frame: every lane reads the (broadcast) 24-B header and
// computes the frame index itself (capture.c:566, same double arithmetic),
// so no barrier is needed; the 7168-B payload moves as 7 x 1 KiB wave loads
// and stores to (idf * nchunk + chunk) * 7168.  Per-chunk counts go through
// LDS and leave with one atomic per counter per workgroup.
__device__ __forceinline__ uint32_t asm_slot(const AssembleArgs &a, uint64_t d, int64_t &rel) {
  const unsigned char *df = a.dfs + d * (uint64_t)a.df_bytes;
  const uint64_t w0 = __builtin_bswap64(*(const uint64_t *)df);  // hdr.c:15-18
  const uint64_t idf = w0 & 0x00000000ffffffffULL;
  const uint64_t sec = (w0 & 0x3fffffff00000000ULL) >> 32;
  rel = (int64_t)idf + (int64_t)(sec - a.ref_sec) / 1.08E-4 - (int64_t)a.ref_idf;
  const uint32_t chunk = a.chunk_of_df[d];
  if (chunk >= a.nchunk) return a.nchunk + 2;
  if (rel < 0) return a.nchunk;
  if ((uint64_t)rel >= a.block_ndf) return a.nchunk + 1;
  return chunk;
}

__global__ void __launch_bounds__(256) b2p_assemble_kernel(AssembleArgs a) {
  __shared__ unsigned long long cnt[256 + 3];
  const uint32_t ncnt = a.nchunk + 3;
  for (uint32_t j = threadIdx.x; j < ncnt; j += blockDim.x) cnt[j] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t d = wave; d < a.ndf; d += nwaves) {
    // the payload loads do not wait for the header: every frame in the
    // buffer is read (nontemporal: read once), the header only decides where
    // (or whether) it lands
    const u32x4 *src = reinterpret_cast<const u32x4 *>(a.dfs + d * (uint64_t)a.df_bytes + a.hdr_bytes);
    u32x4 v[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) v[k] = __builtin_nontemporal_load(src + k * 64 + lane);
    int64_t rel;
    const uint32_t slot = asm_slot(a, d, rel);  // wave-uniform
    if (lane == 0) atomicAdd(&cnt[slot], 1ull);
    if (slot >= a.nchunk) continue;
    const uint32_t chunk = a.chunk_of_df[d];
    u32x4 *dst = reinterpret_cast<u32x4 *>(a.block + ((uint64_t)rel * a.nchunk + chunk) * 7168ull);
#pragma unroll
    for (int k = 0; k < 7; ++k) __builtin_nontemporal_store(v[k], dst + k * 64 + lane);
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < ncnt; j += blockDim.x)
    if (cnt[j]) atomicAdd(&a.counts[j], cnt[j]);
}

// Nontemporal loads and stores, payload loads issued before the header is
// decoded, one frame per wave per iteration, 8192 workgroups of 4 waves: the
// winner of the round-1 sweep over load/store policy, frames per iteration,
// header-first ordering and grid (profiles/r01_assemble_sweep.txt).
// grid_cap (b2p_tuning_t.assemble_grid) overrides the workgroup cap.
hipError_t launch_assemble(const AssembleArgs &a, uint32_t grid_cap, hipStream_t s) {
  if (a.nchunk > 256) return hipErrorInvalidValue;
  uint64_t blocks = (a.ndf + 3) / 4;  // 4 waves per workgroup
  const uint64_t cap = grid_cap ? grid_cap : 8192;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(b2p_assemble_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

// ---- launchers --------------------------------------------------------------
typedef void (*IntegrateFn)(IntegrateArgs);

template <int MODE, int NPO, bool MULTI>
static IntegrateFn pick_t(int unroll, bool nt) {
  switch (unroll * 2 + (nt ? 1 : 0)) {
    case 4 * 2 + 0: return b2p_integrate_kernel<MODE, NPO, 4, false, MULTI>;
    case 4 * 2 + 1: return b2p_integrate_kernel<MODE, NPO, 4, true, MULTI>;
    case 16 * 2 + 0: return b2p_integrate_kernel<MODE, NPO, 16, false, MULTI>;
    case 16 * 2 + 1: return b2p_integrate_kernel<MODE, NPO, 16, true, MULTI>;
    case 8 * 2 + 0: return b2p_integrate_kernel<MODE, NPO, 8, false, MULTI>;
    default: return b2p_integrate_kernel<MODE, NPO, 8, true, MULTI>;
  }
}

template <bool MULTI>
static IntegrateFn pick_m(int mode, int npol_out, int unroll, bool nt) {
  switch (mode * 2 + (npol_out - 1)) {
    case kI8 * 2 + 0: return pick_t<kI8, 1, MULTI>(unroll, nt);
    case kI8 * 2 + 1: return pick_t<kI8, 2, MULTI>(unroll, nt);
    case kI16LE * 2 + 0: return pick_t<kI16LE, 1, MULTI>(unroll, nt);
    case kI16LE * 2 + 1: return pick_t<kI16LE, 2, MULTI>(unroll, nt);
    case kI16BE * 2 + 0: return pick_t<kI16BE, 1, MULTI>(unroll, nt);
    case kI16BE * 2 + 1: return pick_t<kI16BE, 2, MULTI>(unroll, nt);
  }
  return nullptr;
}

static IntegrateFn pick(int mode, int npol_out, int unroll, bool nt, bool multi) {
  return multi ? pick_m<true>(mode, npol_out, unroll, nt) : pick_m<false>(mode, npol_out, unroll, nt);
}

hipError_t launch_integrate(const IntegrateArgs &a, const KernelChoice &k, uint32_t threads,
                            uint32_t grid, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
  // a.blk is read only by the MULTI instantiation, a.data only by the other
  IntegrateFn f = pick(k.mode, k.npol_out, k.unroll, k.nt, a.nblk > 1);
  if (!f) return hipErrorInvalidValue;
  const size_t lds = (size_t)a.nout * sizeof(unsigned long long);
  IntegrateArgs arg = a;
  void *args[] = {&arg};
  // start/stop events ride on the dispatch packet itself (no marker packets
  // between kernels), so timing does not perturb the back-to-back stream
  return hipExtLaunchKernel(reinterpret_cast<const void *>(f), dim3(grid), dim3(threads), args,
                            lds, s, ev0, ev1, 0);
}

hipError_t occupancy_integrate(const KernelChoice &k, uint32_t threads, size_t lds, int *blocks) {
  IntegrateFn f = pick(k.mode, k.npol_out, k.unroll, k.nt, false);  // both shapes: the same resources
  if (!f) return hipErrorInvalidValue;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, reinterpret_cast<const void *>(f),
                                                      (int)threads, lds);
}

hipError_t launch_finalize(const FinalizeArgs &a, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
  const uint32_t grid = (a.nout + 63) / 64;
  FinalizeArgs arg = a;
  void *args[] = {&arg};
  return hipExtLaunchKernel(reinterpret_cast<const void *>(b2p_finalize_kernel),
                            dim3(grid, a.nblk ? a.nblk : 1), dim3(256), args, 0, s, ev0, ev1, 0);
}

// Launched once by b2p_open: loading this translation unit's code object
// is what makes a process's first launch slow (tens of ms), and an empty
// kernel of its own keeps that launch out of the integrate kernel's
// rocprofv3 statistics.
__global__ void b2p_warm_kernel() {}

hipError_t launch_warm(hipStream_t s) {
  hipLaunchKernelGGL(b2p_warm_kernel, dim3(1), dim3(64), 0, s);
  return hipGetLastError();
}

hipError_t launch_convert(const ConvertArgs &a, hipStream_t s) {
  uint64_t blocks = (a.n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(b2p_convert_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_sum_rows(const SumRowsArgs &a, hipStream_t s) {
  uint64_t blocks = (a.count + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(b2p_sum_rows_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_fill(uint4 *dst, uint64_t nvec, const FillArgs &f, hipStream_t s) {
  uint64_t blocks = (nvec + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(b2p_fill_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, dst, nvec, f);
  return hipGetLastError();
}

uint64_t splitmix64_host(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

}  // namespace b2p
