// overlap_probe -- can back-to-back streaming launches hide their tails?
// Diagnostic only (not the product).  The integrate kernel's load pattern
// (512 threads x 4 rows of 16-B nt loads, static contiguous row slices, one
// workgroup per CU) launched K times over rotating 1-GiB buffers:
//   streams 1   every launch on one stream: launch k+1 starts after the
//               last workgroup of launch k ends (tail skew + boundary)
//   streams 2/3 launches alternate over 2 or 3 streams, so launch k+1's
//               workgroups may take CUs that launch k has released
// and a dynamic-LDS pad that caps residency at one workgroup per CU (so
// launch k+1 does not double up on busy CUs but fills freed ones).
// Prints per-variant GB/s and the mean overlap between consecutive launches
// (last end of k - first start of k+1, from s_memrealtime stamps) as JSON.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned long long rt() { return __builtin_amdgcn_s_memrealtime(); }

__global__ void __launch_bounds__(512) stream_kernel(const u32x4 *data, unsigned long long nrows,
                                                     unsigned S, unsigned long long *stamps,
                                                     unsigned *sink) {
  extern __shared__ unsigned pad[];
  const unsigned t = threadIdx.x;
  const unsigned long long t0 = rt();
  unsigned acc = 0;
  const unsigned long long r0 = (unsigned long long)blockIdx.x * nrows / gridDim.x;
  const unsigned long long r1 = (unsigned long long)(blockIdx.x + 1) * nrows / gridDim.x;
  const u32x4 *p = data + r0 * S + t;
  unsigned long long r = r0;
  for (; r + 4 <= r1; r += 4, p += 4 * S) {
    u32x4 v0 = __builtin_nontemporal_load(p), v1 = __builtin_nontemporal_load(p + S);
    u32x4 v2 = __builtin_nontemporal_load(p + 2 * S), v3 = __builtin_nontemporal_load(p + 3 * S);
    acc += __builtin_amdgcn_sdot4(v0.x, v0.x, 0, false) + __builtin_amdgcn_sdot4(v0.y, v0.y, 0, false) +
           __builtin_amdgcn_sdot4(v0.z, v0.z, 0, false) + __builtin_amdgcn_sdot4(v0.w, v0.w, 0, false);
    acc += __builtin_amdgcn_sdot4(v1.x, v1.x, 0, false) + __builtin_amdgcn_sdot4(v1.y, v1.y, 0, false) +
           __builtin_amdgcn_sdot4(v1.z, v1.z, 0, false) + __builtin_amdgcn_sdot4(v1.w, v1.w, 0, false);
    acc += __builtin_amdgcn_sdot4(v2.x, v2.x, 0, false) + __builtin_amdgcn_sdot4(v2.y, v2.y, 0, false) +
           __builtin_amdgcn_sdot4(v2.z, v2.z, 0, false) + __builtin_amdgcn_sdot4(v2.w, v2.w, 0, false);
    acc += __builtin_amdgcn_sdot4(v3.x, v3.x, 0, false) + __builtin_amdgcn_sdot4(v3.y, v3.y, 0, false) +
           __builtin_amdgcn_sdot4(v3.z, v3.z, 0, false) + __builtin_amdgcn_sdot4(v3.w, v3.w, 0, false);
  }
  for (; r < r1; ++r, p += S) acc ^= __builtin_nontemporal_load(p).x;
  if (t == 0) pad[0] = acc;
  __syncthreads();
  if (t == 0) {
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = rt();
  }
  if (pad[0] == 0x9e3779b9u) sink[0] = acc;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main(int argc, char **argv) {
  const size_t bytes = 1ull << 30;
  const unsigned S = 512;
  const unsigned long long nrows = bytes / 16 / S;
  const int K = argc > 1 ? atoi(argv[1]) : 40;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  u32x4 *bufs[4];
  for (int i = 0; i < 4; ++i) {
    CK(hipMalloc(&bufs[i], bytes));
    CK(hipMemset(bufs[i], i + 1, bytes));
  }
  CK(hipFuncSetAttribute((const void *)stream_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  unsigned long long *stamps;
  unsigned *sink;
  CK(hipMalloc(&stamps, (size_t)16 * 2 * ncu * K));
  CK(hipMalloc(&sink, 4));
  hipStream_t st[3];
  for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b, ev[3];
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (auto &x : ev) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
  std::vector<unsigned long long> h((size_t)2 * 2 * ncu * K);

  struct V { int nstreams; unsigned lds_kib; int grid_mul; };
  const V all_vars[] = {{1, 0, 1}, {1, 96, 1}, {2, 0, 1}, {2, 96, 1}, {3, 96, 1}, {2, 64, 1},
                        {1, 0, 2}, {2, 96, 2}};
  // "dist": one stream only, plus the distribution of per-launch spans
  const bool dist = argc > 2 && argv[2][0] == 'd';
  const int nvars = dist ? 1 : (int)(sizeof all_vars / sizeof all_vars[0]);
  const V *vars = all_vars;
  printf("{\"cu\": %d, \"launches\": %d, \"bytes_per_launch\": %zu, \"results\": [\n", ncu, K, bytes);
  for (int rep = 0; rep < 3; ++rep)
    for (int vi = 0; vi < nvars; ++vi) {
      const V &v = vars[vi];
      const int grid = ncu * v.grid_mul;
      const size_t lds = (size_t)v.lds_kib * 1024 + 16;
      // warm
      for (int k = 0; k < 4; ++k)
        hipLaunchKernelGGL(stream_kernel, grid, 512, lds, st[0], bufs[k % 4], nrows, S, stamps, sink);
      CK(hipStreamSynchronize(st[0]));
      CK(hipEventRecord(a, st[0]));
      for (int s = 1; s < v.nstreams; ++s) CK(hipStreamWaitEvent(st[s], a, 0));
      for (int k = 0; k < K; ++k)
        hipLaunchKernelGGL(stream_kernel, grid, 512, lds, st[k % v.nstreams], bufs[k % 4], nrows, S,
                           stamps + (size_t)2 * grid * k, sink);
      for (int s = 1; s < v.nstreams; ++s) {
        CK(hipEventRecord(ev[s], st[s]));
        CK(hipStreamWaitEvent(st[0], ev[s], 0));
      }
      CK(hipEventRecord(b, st[0]));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      CK(hipMemcpy(h.data(), stamps, (size_t)16 * grid * K, hipMemcpyDeviceToHost));
      // overlap of consecutive launches (positive: k+1 started before k ended)
      double ov = 0, span = 0;
      for (int k = 0; k + 1 < K; ++k) {
        unsigned long long end_k = 0, start_n = ~0ull;
        for (int i = 0; i < grid; ++i) {
          end_k = std::max(end_k, h[(size_t)2 * grid * k + 2 * i + 1]);
          start_n = std::min(start_n, h[(size_t)2 * grid * (k + 1) + 2 * i]);
        }
        ov += ((double)end_k - (double)start_n) / 100.0;
      }
      std::vector<double> spans;
      for (int k = 0; k < K; ++k) {
        unsigned long long s0 = ~0ull, e0 = 0;
        for (int i = 0; i < grid; ++i) {
          s0 = std::min(s0, h[(size_t)2 * grid * k + 2 * i]);
          e0 = std::max(e0, h[(size_t)2 * grid * k + 2 * i + 1]);
        }
        span += (e0 - s0) / 100.0;
        spans.push_back((e0 - s0) / 100.0);
      }
      if (dist) {
        std::vector<double> so = spans;
        std::sort(so.begin(), so.end());
        printf(" {\"span_us_min\": %.2f, \"p10\": %.2f, \"median\": %.2f, \"p90\": %.2f, \"max\": %.2f, "
               "\"over_153\": %d, \"spans\": [", so[0], so[K / 10], so[K / 2], so[K * 9 / 10], so[K - 1],
               (int)std::count_if(so.begin(), so.end(), [](double x) { return x > 153.0; }));
        for (int k = 0; k < K; ++k) printf("%s%.1f", k ? ", " : "", spans[k]);
        printf("]},\n");
      }
      printf(" {\"streams\": %d, \"lds_kib\": %u, \"grid\": %d, \"rep\": %d, \"us_per_launch\": %.2f, "
             "\"GBps\": %.1f, \"launch_span_us\": %.2f, \"overlap_us\": %.2f},\n",
             v.nstreams, v.lds_kib, grid, rep, ms * 1e3 / K, (double)bytes * K / (ms * 1e-3) / 1e9,
             span / K, ov / (K - 1));
      fflush(stdout);
    }
  printf(" {}]}\n");
  return 0;
}
