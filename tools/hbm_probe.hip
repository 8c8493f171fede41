// hbm_probe -- measured HBM read ceiling on this box (not part of the
// product).  Streams N GiB of distinct buffers (rotating, > Infinity Cache)
// with 16-B loads per lane and a trivial reduction, for several grid shapes
// and both cache policies, timed with hipEvents.  The best figure is the
// practical read roofline the integrate kernel is compared against in
// DESIGN.md (the spec peak, 8 TB/s, stays the roofline "peak" in bench.py).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT, int UNROLL>
__global__ void __launch_bounds__(1024) read_kernel(const u32x4 *p, size_t n, unsigned *sink) {
  unsigned acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
      v[u] = NT ? __builtin_nontemporal_load(p + i + u * stride) : p[i + u * stride];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < n; i += stride) {
    u32x4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;  // keeps the loads live
}

// copy ceiling (read + write), the bound of b2p_assemble
template <bool NTL, bool NTS, int UNROLL>
__global__ void __launch_bounds__(1024) copy_kernel(const u32x4 *p, u32x4 *q, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
      v[u] = NTL ? __builtin_nontemporal_load(p + i + u * stride) : p[i + u * stride];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if (NTS) __builtin_nontemporal_store(v[u], q + i + u * stride);
      else q[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) q[i] = p[i];
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <bool NT, int U>
static double run(u32x4 **bufs, int nbuf, size_t n, int grid, int block, unsigned *sink, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < nbuf; ++w) hipLaunchKernelGGL((read_kernel<NT, U>), grid, block, 0, 0, bufs[w], n, sink);
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((read_kernel<NT, U>), grid, block, 0, 0, bufs[r % nbuf], n, sink);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return (double)n * 16 * reps / (ms * 1e-3) / 1e9;
}

int main(int argc, char **argv) {
  const size_t bytes = (argc > 1 ? strtoull(argv[1], 0, 10) : 1024) << 20;
  const int nbuf = 4, reps = 40;
  const size_t n = bytes / 16;
  u32x4 *bufs[nbuf];
  unsigned *sink;
  for (int i = 0; i < nbuf; ++i) {
    CK(hipMalloc(&bufs[i], bytes));
    CK(hipMemset(bufs[i], i + 1, bytes));
  }
  CK(hipMalloc(&sink, 4));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  printf("{\"bytes_per_launch\": %zu, \"results\": [\n", bytes);
  const int blocks[] = {256, 512, 1024};
  const int per_cu[] = {1, 2, 4, 8};
  int first = 1;
  for (int bi = 0; bi < 3; ++bi)
    for (int pi = 0; pi < 4; ++pi) {
      const int block = blocks[bi], grid = ncu * per_cu[pi];
      if (block * per_cu[pi] > 2048) continue;
      double g0 = run<false, 8>(bufs, nbuf, n, grid, block, sink, reps);
      double g1 = run<true, 8>(bufs, nbuf, n, grid, block, sink, reps);
      double g2 = run<true, 16>(bufs, nbuf, n, grid, block, sink, reps);
      double g3 = run<false, 4>(bufs, nbuf, n, grid, block, sink, reps);
      printf("%s {\"block\": %d, \"grid\": %d, \"plain_u8\": %.1f, \"nt_u8\": %.1f, \"nt_u16\": %.1f, \"plain_u4\": %.1f}",
             first ? "" : ",\n", block, grid, g0, g1, g2, g3);
      first = 0;
    }
  printf("\n], \"copy\": [\n");
  first = 1;
  for (int bi = 0; bi < 2; ++bi)
    for (int pi = 0; pi < 4; ++pi) {
      const int block = blocks[bi], grid = ncu * per_cu[pi] * 2;
      double c[4];
      for (int m = 0; m < 4; ++m) {
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        for (int r = -2; r < reps; ++r) {
          if (r == 0) CK(hipEventRecord(a, 0));
          const u32x4 *src = bufs[(r + 4) % 2];
          u32x4 *dst = bufs[2 + (r + 4) % 2];
          switch (m) {
            case 0: hipLaunchKernelGGL((copy_kernel<false, false, 4>), grid, block, 0, 0, src, dst, n); break;
            case 1: hipLaunchKernelGGL((copy_kernel<true, true, 4>), grid, block, 0, 0, src, dst, n); break;
            case 2: hipLaunchKernelGGL((copy_kernel<true, false, 8>), grid, block, 0, 0, src, dst, n); break;
            default: CK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, 0));
          }
        }
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        c[m] = 2.0 * bytes * reps / (ms * 1e-3) / 1e9;
      }
      printf("%s {\"block\": %d, \"grid\": %d, \"copy_plain_u4\": %.1f, \"copy_nt_u4\": %.1f, "
             "\"copy_ntload_u8\": %.1f, \"hipMemcpyD2D\": %.1f}",
             first ? "" : ",\n", block, grid, c[0], c[1], c[2], c[3]);
      first = 0;
    }
  printf("\n]}\n");
  return 0;
}
