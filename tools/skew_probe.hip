// skew_probe -- where does a 1-GiB streaming launch lose time?  Diagnostic
// only (not the product): the integrate kernel's load pattern (512 threads x
// 4 rows of 16-B nt loads, one workgroup per CU) with per-workgroup start /
// end stamps (s_memrealtime, 100 MHz), for
//   static    contiguous row slices (the shipped mapping)
//   dynamic   64-row chunks handed out by one device-scope atomic counter
//   xcd       dynamic, one counter per XCD group (blockIdx % 8)
// Prints launch time, mean/min/max workgroup busy span and the tail
// (last end - median end) as JSON.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned long long rt() { return __builtin_amdgcn_s_memrealtime(); }

template <int MODE>
__global__ void __launch_bounds__(512) stream_kernel(const u32x4 *data, unsigned long long nrows,
                                                     unsigned S, unsigned long long *ctr,
                                                     unsigned long long base, unsigned chunk,
                                                     unsigned long long *stamps, unsigned *sink) {
  __shared__ unsigned long long s_idx;
  const unsigned t = threadIdx.x;
  unsigned long long t0 = rt();
  unsigned acc = 0;
  auto rows = [&](unsigned long long r0, unsigned long long r1) {
    const u32x4 *p = data + r0 * S + t;
    unsigned long long r = r0;
    for (; r + 4 <= r1; r += 4, p += 4 * S) {
      u32x4 v0 = __builtin_nontemporal_load(p), v1 = __builtin_nontemporal_load(p + S);
      u32x4 v2 = __builtin_nontemporal_load(p + 2 * S), v3 = __builtin_nontemporal_load(p + 3 * S);
      acc = __builtin_amdgcn_sdot4(v0.x, v0.y, acc, false) ^ __builtin_amdgcn_sdot4(v1.z, v2.w, v3.x, false);
    }
    for (; r < r1; ++r, p += S) acc ^= __builtin_nontemporal_load(p).x;
  };
  if (MODE == 0) {
    const unsigned long long r0 = (unsigned long long)blockIdx.x * nrows / gridDim.x;
    const unsigned long long r1 = (unsigned long long)(blockIdx.x + 1) * nrows / gridDim.x;
    rows(r0, r1);
  } else if (MODE == 3) {
    // hybrid: static slices over the first (1 - 1/16) of the rows, then the
    // last 1/16 handed out in `chunk`-row pieces to whoever finishes first
    const unsigned long long head = nrows - nrows / 16;
    const unsigned long long r0 = (unsigned long long)blockIdx.x * head / gridDim.x;
    const unsigned long long r1 = (unsigned long long)(blockIdx.x + 1) * head / gridDim.x;
    rows(r0, r1);
    const unsigned long long nch = (nrows - head + chunk - 1) / chunk;
    for (;;) {
      if (t == 0) s_idx = atomicAdd(ctr, 1ull);
      __syncthreads();
      const unsigned long long k = s_idx - base;
      __syncthreads();
      if (k >= nch) break;
      const unsigned long long a0 = head + k * chunk;
      rows(a0, a0 + chunk < nrows ? a0 + chunk : nrows);
    }
  } else {
    unsigned long long *c = MODE == 1 ? ctr : ctr + 8 * (blockIdx.x % 8);  // 64-B apart
    const unsigned long long nch = (nrows + chunk - 1) / chunk;
    // MODE 2: XCD group x owns chunks x, x+8, ... (its own counter)
    for (;;) {
      if (t == 0) s_idx = atomicAdd(c, 1ull);
      __syncthreads();
      const unsigned long long k = s_idx - base;
      __syncthreads();
      const unsigned long long ch = MODE == 1 ? k : k * 8 + (blockIdx.x % 8);
      if (ch >= nch) break;
      const unsigned long long r0 = ch * chunk;
      rows(r0, r0 + chunk < nrows ? r0 + chunk : nrows);
    }
  }
  __syncthreads();
  if (t == 0) {
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = rt();
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main() {
  const size_t bytes = 1ull << 30;
  const unsigned S = 512;  // vectors per row = one 512-thread workgroup
  const unsigned long long nrows = bytes / 16 / S;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = ncu;
  u32x4 *bufs[4];
  for (int i = 0; i < 4; ++i) {
    CK(hipMalloc(&bufs[i], bytes));
    CK(hipMemset(bufs[i], i + 1, bytes));
  }
  unsigned long long *ctr, *stamps;
  unsigned *sink;
  CK(hipMalloc(&ctr, 1024));  // ctr[0]: dynamic; ctr[8 + 8x]: XCD group x
  CK(hipMemset(ctr, 0, 1024));
  CK(hipMalloc(&stamps, 16 * grid));
  CK(hipMalloc(&sink, 4));
  std::vector<unsigned long long> h(2 * grid);
  unsigned long long base[4] = {0, 0, 0, 0};
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const char *names[4] = {"static", "dynamic", "xcd", "hybrid"};
  printf("{\"grid\": %d, \"rows\": %llu, \"results\": [\n", grid, nrows);
  for (int rep = 0; rep < 3; ++rep)
    for (int mode = 0; mode < 4; ++mode)
      for (unsigned chunk : {8u, 32u, 128u}) {
        if (mode == 0 && chunk != 32) continue;
        if ((mode == 1 || mode == 2) && chunk == 8) continue;
        float best = 1e9, ms = 0;
        double span_mean = 0, span_min = 1e18, span_max = 0, tail = 0;
        for (int it = 0; it < 8; ++it) {
          CK(hipEventRecord(a, 0));
          if (mode == 0)
            hipLaunchKernelGGL(stream_kernel<0>, grid, 512, 0, 0, bufs[it % 4], nrows, S, ctr, 0ull, chunk, stamps, sink);
          else if (mode == 1)
            hipLaunchKernelGGL(stream_kernel<1>, grid, 512, 0, 0, bufs[it % 4], nrows, S, ctr, base[1], chunk, stamps, sink);
          else if (mode == 2)
            hipLaunchKernelGGL(stream_kernel<2>, grid, 512, 0, 0, bufs[it % 4], nrows, S, ctr + 8, base[2], chunk, stamps, sink);
          else
            hipLaunchKernelGGL(stream_kernel<3>, grid, 512, 0, 0, bufs[it % 4], nrows, S, ctr + 120, base[3], chunk, stamps, sink);
          CK(hipEventRecord(b, 0));
          CK(hipEventSynchronize(b));
          CK(hipEventElapsedTime(&ms, a, b));
          const unsigned long long nch = (nrows + chunk - 1) / chunk;
          if (mode == 1) base[1] += nch + grid;
          if (mode == 3) base[3] += (nrows / 16 + chunk - 1) / chunk + grid;
          if (mode == 2) {  // each XCD-group counter: its chunks + its blocks; keep counters in step
            // group x gets ceil((nch - x)/8) chunks and grid/8 blocks; use a fresh
            // zeroed counter set instead of tracking 8 bases
            CK(hipMemset(ctr + 8, 0, 8 * 8 * 8));
          }
          if (ms < best) best = ms;
          CK(hipMemcpy(h.data(), stamps, 16 * grid, hipMemcpyDeviceToHost));
          std::vector<double> ends, starts;
          for (int i = 0; i < grid; ++i) { starts.push_back(h[2 * i]); ends.push_back(h[2 * i + 1]); }
          double s0 = *std::min_element(starts.begin(), starts.end());
          std::vector<double> se = ends;
          std::sort(se.begin(), se.end());
          double sm = 0, smin = 1e18, smax = 0;
          for (int i = 0; i < grid; ++i) { double sp = (ends[i] - starts[i]) / 100.0; sm += sp; smin = std::min(smin, sp); smax = std::max(smax, sp); }
          span_mean = sm / grid; span_min = smin; span_max = smax;
          tail = (se.back() - se[grid / 2]) / 100.0;
          (void)s0;
        }
        printf(" {\"mode\": \"%s\", \"chunk\": %u, \"rep\": %d, \"best_us\": %.1f, \"GBps\": %.1f, "
               "\"span_mean_us\": %.1f, \"span_min_us\": %.1f, \"span_max_us\": %.1f, \"tail_us\": %.1f},\n",
               names[mode], chunk, rep, best * 1e3, bytes / (best * 1e-3) / 1e9, span_mean, span_min,
               span_max, tail);
      }
  printf(" {}]}\n");
  return 0;
}
