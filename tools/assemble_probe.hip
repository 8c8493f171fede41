// assemble_probe -- can frame assembly (b2p_assemble_kernel) move its bytes
// faster?  Diagnostic only (not the product).  Every variant copies the
// 7168-B payload of each 7232-B frame of a BMF block (393216 frames,
// 2.84 GB read + 2.82 GB written) to the slot a precomputed index gives, as
// the product kernel does after decoding the header.  Arrival orders:
// time-major with the 48 chunks of each time step shuffled (capture), or
// contiguous (slot = frame: a plain copy of the same shape).
// Variants (one frame per wave unless noted, 256-thread workgroups):
//   nt         nontemporal loads and stores (the product kernel)
//   plain_st   nontemporal loads, plain stores
//   sc1_st     nontemporal loads, write-through stores (sc1: drop from L2)
//   sc01_st    nontemporal loads, sc0 sc1 stores (system scope)
//   nt2        two frames per wave in flight (14 loads, then 14 stores)
//   nt_512     512-thread workgroups
//   pipe       software pipelined: frame i+1's loads issued before frame
//              i's stores
//   sw*        small grids (256-1024 workgroups): the whole grid sweeps the
//              stream front to back with few frames in flight per CU
// Prints one JSON line per variant: median GB/s of (read + write) bytes.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr unsigned kDF = 7232, kHDR = 64, kPAY = 7168;

template <int POL>
__device__ __forceinline__ void store16(u32x4 *p, u32x4 v) {
  if (POL == 0) {
    __builtin_nontemporal_store(v, p);
  } else if (POL == 1) {
    *p = v;
  } else if (POL == 2) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  } else {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  }
}

// FPW frames per wave per iteration; POL store policy; PIPE: loads of the
// next frame before the stores of this one (FPW 1 only)
template <int FPW, int POL, bool PIPE>
__global__ void __launch_bounds__(512) copy_kernel(const unsigned char *dfs, unsigned char *blk,
                                                   const unsigned *slot, unsigned long long ndf) {
  const unsigned lane = threadIdx.x & 63;
  const unsigned long long wave = ((unsigned long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const unsigned long long nwaves = ((unsigned long long)gridDim.x * blockDim.x) >> 6;
  if (PIPE) {
    unsigned long long d = wave;
    if (d >= ndf) return;
    u32x4 v[7];
    const u32x4 *src = reinterpret_cast<const u32x4 *>(dfs + d * kDF + kHDR);
#pragma unroll
    for (int k = 0; k < 7; ++k) v[k] = __builtin_nontemporal_load(src + k * 64 + lane);
    for (;;) {
      const unsigned long long dn = d + nwaves;
      u32x4 w[7];
      if (dn < ndf) {
        const u32x4 *s2 = reinterpret_cast<const u32x4 *>(dfs + dn * kDF + kHDR);
#pragma unroll
        for (int k = 0; k < 7; ++k) w[k] = __builtin_nontemporal_load(s2 + k * 64 + lane);
      }
      u32x4 *dst = reinterpret_cast<u32x4 *>(blk + (unsigned long long)slot[d] * kPAY);
#pragma unroll
      for (int k = 0; k < 7; ++k) store16<POL>(dst + k * 64 + lane, v[k]);
      if (dn >= ndf) break;
      for (int k = 0; k < 7; ++k) v[k] = w[k];  // register moves: no unroll pragma needed
      d = dn;
    }
    return;
  }
  for (unsigned long long d0 = wave * FPW; d0 < ndf; d0 += nwaves * FPW) {
    u32x4 v[FPW][7];
#pragma unroll
    for (int f = 0; f < FPW; ++f) {
      const unsigned long long d = d0 + f < ndf ? d0 + f : d0;
      const u32x4 *src = reinterpret_cast<const u32x4 *>(dfs + d * kDF + kHDR);
#pragma unroll
      for (int k = 0; k < 7; ++k) v[f][k] = __builtin_nontemporal_load(src + k * 64 + lane);
    }
#pragma unroll
    for (int f = 0; f < FPW; ++f) {
      if (d0 + f < ndf) {
        u32x4 *dst = reinterpret_cast<u32x4 *>(blk + (unsigned long long)slot[d0 + f] * kPAY);
#pragma unroll
        for (int k = 0; k < 7; ++k) store16<POL>(dst + k * 64 + lane, v[f][k]);
      }
    }
  }
}

typedef void (*Kern)(const unsigned char *, unsigned char *, const unsigned *, unsigned long long);

struct Variant {
  const char *name;
  Kern k;
  unsigned threads, grid;
};

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const unsigned long long ndf = 393216, nchunk = 48;
  unsigned char *dfs, *blk;
  unsigned *slot_tm, *slot_lin;
  CK(hipMalloc(&dfs, ndf * kDF));
  CK(hipMalloc(&blk, ndf * kPAY));
  CK(hipMalloc(&slot_tm, ndf * 4));
  CK(hipMalloc(&slot_lin, ndf * 4));
  CK(hipMemset(dfs, 7, ndf * kDF));
  std::vector<unsigned> s(ndf);
  std::mt19937 rng(20181105);
  for (unsigned long long t = 0; t < ndf / nchunk; ++t) {
    std::vector<unsigned> c(nchunk);
    for (unsigned i = 0; i < nchunk; ++i) c[i] = i;
    std::shuffle(c.begin(), c.end(), rng);
    for (unsigned i = 0; i < nchunk; ++i) s[t * nchunk + i] = (unsigned)(t * nchunk + c[i]);
  }
  CK(hipMemcpy(slot_tm, s.data(), ndf * 4, hipMemcpyHostToDevice));
  for (unsigned long long i = 0; i < ndf; ++i) s[i] = (unsigned)i;
  CK(hipMemcpy(slot_lin, s.data(), ndf * 4, hipMemcpyHostToDevice));

  const Variant vs[] = {
      {"nt", copy_kernel<1, 0, false>, 256, 8192},
      {"nt_g4096", copy_kernel<1, 0, false>, 256, 4096},
      {"nt_g16384", copy_kernel<1, 0, false>, 256, 16384},
      {"plain_st", copy_kernel<1, 1, false>, 256, 8192},
      {"sc1_st", copy_kernel<1, 2, false>, 256, 8192},
      {"sc01_st", copy_kernel<1, 3, false>, 256, 8192},
      {"nt2", copy_kernel<2, 0, false>, 256, 8192},
      {"nt_512", copy_kernel<1, 0, false>, 512, 4096},
      {"pipe", copy_kernel<1, 0, true>, 256, 2048},
      {"pipe_g4096", copy_kernel<1, 0, true>, 256, 4096},
      {"pipe_sc1", copy_kernel<1, 2, true>, 256, 2048},
      // sweeps with few frames in flight per CU (the read_pattern_probe
      // copy_sweep_u4 shape: ~32 KiB in flight per CU, grid front to back)
      {"sw_g256_t512", copy_kernel<1, 0, false>, 512, 256},
      {"sw_g512_t512", copy_kernel<1, 0, false>, 512, 512},
      {"sw_g512_t256", copy_kernel<1, 0, false>, 256, 512},
      {"sw_g1024_t256", copy_kernel<1, 0, false>, 256, 1024},
      {"sw2_g256_t512", copy_kernel<2, 0, false>, 512, 256},
      {"sw2_g512_t256", copy_kernel<2, 0, false>, 256, 512},
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = (double)ndf * (kDF + kPAY);
  for (int order = 0; order < 2; ++order) {
    const unsigned *slot = order == 0 ? slot_tm : slot_lin;
    for (const Variant &v : vs) {
      for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(v.k, dim3(v.grid), dim3(v.threads), 0, 0, dfs, blk, slot, ndf);
      CK(hipDeviceSynchronize());
      std::vector<double> gbs;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(v.k, dim3(v.grid), dim3(v.threads), 0, 0, dfs, blk, slot, ndf);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        gbs.push_back(bytes / (ms * 1e-3) / 1e9);
      }
      std::sort(gbs.begin(), gbs.end());
      printf("{\"variant\": \"%s\", \"order\": \"%s\", \"threads\": %u, \"grid\": %u, \"median_GBps\": %.1f, "
             "\"best_GBps\": %.1f, \"median_us\": %.1f}\n",
             v.name, order == 0 ? "time-major, chunks shuffled" : "contiguous (plain copy)", v.threads,
             v.grid, gbs[gbs.size() / 2], gbs.back(), bytes / (gbs[gbs.size() / 2] * 1e9) * 1e6);
      fflush(stdout);
    }
  }
  // references: the runtime's device-to-device copy of the payload bytes
  // (contiguous, no frame headers), and the same frame copy with a 7168-B
  // source stride (no 64-B header gap between payloads)
  {
    std::vector<double> gbs;
    for (int r = 0; r < reps + 2; ++r) {
      CK(hipEventRecord(e0, 0));
      CK(hipMemcpyAsync(blk, dfs, ndf * kPAY, hipMemcpyDeviceToDevice, 0));
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 2) gbs.push_back(2.0 * ndf * kPAY / (ms * 1e-3) / 1e9);
    }
    std::sort(gbs.begin(), gbs.end());
    printf("{\"variant\": \"hipMemcpy D2D\", \"order\": \"contiguous payload bytes\", \"median_GBps\": %.1f, "
           "\"best_GBps\": %.1f}\n", gbs[gbs.size() / 2], gbs.back());
  }
  return 0;
}
