// read_pattern_probe -- which read pattern streams HBM fastest?  Diagnostic
// only (not the product).  Every variant reads the same rotating 1-GiB
// buffers with 16-B nontemporal loads, 512-thread workgroups, one per CU,
// and folds the data with v_dot4 (as the integrate kernel does):
//   slice      workgroup g owns a contiguous 1/G of the buffer, read as
//              rows of 8 KiB (512 lanes x 16 B), U rows in flight (the
//              integrate kernel's int8 mapping; U = 2, 4, 8)
//   xcd        slice, but the 32 workgroups of one XCD (blockIdx % 8) own
//              adjacent slices, so each XCD streams one contiguous 1/8
//   wave       each wave owns a contiguous 1/(8G): 8x more, shorter streams
//   lane64     slice, but a lane reads 64 contiguous bytes (4 loads) of a
//              32-KiB row instead of 16 B of 4 rows
// Also copy variants (read + write, the bound of b2p_assemble).
// Prints GB/s per variant and repetition as JSON.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned fold(u32x4 v) {
  return __builtin_amdgcn_sdot4(v.x, v.x, 0, false) + __builtin_amdgcn_sdot4(v.y, v.y, 0, false) +
         __builtin_amdgcn_sdot4(v.z, v.z, 0, false) + __builtin_amdgcn_sdot4(v.w, v.w, 0, false);
}

// MODE 0 slice, 1 xcd, 2 wave, 3 lane64
template <int MODE, int U>
__global__ void __launch_bounds__(512) read_kernel(const u32x4 *data, unsigned long long nvec,
                                                   unsigned *sink) {
  const unsigned t = threadIdx.x;
  unsigned acc = 0;
  if (MODE == 2) {
    const unsigned long long nw = (unsigned long long)gridDim.x * 8;
    const unsigned long long w = (unsigned long long)blockIdx.x * 8 + (t >> 6);
    const unsigned long long rows = nvec / 64;  // 1-KiB wave rows
    const unsigned long long r0 = w * rows / nw, r1 = (w + 1) * rows / nw;
    const u32x4 *p = data + r0 * 64 + (t & 63);
    unsigned long long r = r0;
    for (; r + U <= r1; r += U, p += U * 64) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + u * 64);
#pragma unroll
      for (int u = 0; u < U; ++u) acc += fold(v[u]);
    }
    for (; r < r1; ++r, p += 64) acc += fold(__builtin_nontemporal_load(p));
  } else {
    unsigned g = blockIdx.x;
    if (MODE == 1) g = (blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8;
    const unsigned S = MODE == 3 ? 2048 : 512;  // vectors per row
    const unsigned long long rows = nvec / S;
    const unsigned long long r0 = (unsigned long long)g * rows / gridDim.x;
    const unsigned long long r1 = (unsigned long long)(g + 1) * rows / gridDim.x;
    if (MODE == 3) {
      const u32x4 *p = data + r0 * S + t * 4;
      for (unsigned long long r = r0; r < r1; ++r, p += S) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(p + u);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += fold(v[u]);
      }
    } else {
      const u32x4 *p = data + r0 * S + t;
      unsigned long long r = r0;
      for (; r + U <= r1; r += U, p += U * S) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + u * S);
#pragma unroll
        for (int u = 0; u < U; ++u) acc += fold(v[u]);
      }
      for (; r < r1; ++r, p += S) acc += fold(__builtin_nontemporal_load(p));
    }
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

// copy variants (the bound of b2p_assemble): MODE 0 slice (a workgroup
// copies a contiguous 1/G in 8-KiB rows, U in flight), 1 sweep (row r of
// every workgroup is r*G + g: the whole grid moves front to back together)
template <int MODE, int U>
__global__ void __launch_bounds__(512) copy_kernel(const u32x4 *src, u32x4 *dst, unsigned long long nvec) {
  const unsigned t = threadIdx.x, S = 512;
  const unsigned long long rows = nvec / S, G = gridDim.x, g = blockIdx.x;
  unsigned long long r0, r1, step;
  if (MODE == 0) {
    r0 = g * rows / G, r1 = (g + 1) * rows / G, step = 1;
  } else {
    r0 = g, r1 = rows, step = G;
  }
  unsigned long long r = r0;
  for (; r + (U - 1) * step < r1; r += U * step) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(src + (r + u * step) * S + t);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(v[u], dst + (r + u * step) * S + t);
  }
  for (; r < r1; r += step) __builtin_nontemporal_store(__builtin_nontemporal_load(src + r * S + t), dst + r * S + t);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef void (*Fn)(const u32x4 *, unsigned long long, unsigned *);

int main(int argc, char **argv) {
  const size_t bytes = 1ull << 30;
  const unsigned long long nvec = bytes / 16;
  const int K = argc > 1 ? atoi(argv[1]) : 40;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  u32x4 *bufs[4];
  for (int i = 0; i < 4; ++i) {
    CK(hipMalloc(&bufs[i], bytes));
    CK(hipMemset(bufs[i], i + 1, bytes));
  }
  unsigned *sink;
  CK(hipMalloc(&sink, 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  struct V { const char *name; Fn f; };
  const V vars[] = {{"slice_u4", read_kernel<0, 4>}, {"slice_u2", read_kernel<0, 2>},
                    {"slice_u8", read_kernel<0, 8>}, {"xcd_u4", read_kernel<1, 4>},
                    {"wave_u4", read_kernel<2, 4>},  {"wave_u8", read_kernel<2, 8>},
                    {"lane64", read_kernel<3, 4>}};
  printf("{\"cu\": %d, \"launches\": %d, \"bytes_per_launch\": %zu, \"results\": [\n", ncu, K, bytes);
  for (int rep = 0; rep < 3; ++rep)
    for (const V &v : vars) {
      for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(v.f, ncu, 512, 0, 0, bufs[k % 4], nvec, sink);
      CK(hipStreamSynchronize(0));
      CK(hipEventRecord(a, 0));
      for (int k = 0; k < K; ++k) hipLaunchKernelGGL(v.f, ncu, 512, 0, 0, bufs[k % 4], nvec, sink);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      printf(" {\"variant\": \"%s\", \"rep\": %d, \"us_per_launch\": %.2f, \"GBps\": %.1f},\n", v.name, rep,
             ms * 1e3 / K, (double)bytes * K / (ms * 1e-3) / 1e9);
      fflush(stdout);
    }
  // copies: 1 GiB -> 1 GiB over rotating buffer pairs, grid = 1 or 2 per CU
  struct CV { const char *name; void (*f)(const u32x4 *, u32x4 *, unsigned long long); int per_cu; };
  const CV cvars[] = {{"copy_slice_u4", copy_kernel<0, 4>, 1}, {"copy_slice_u2", copy_kernel<0, 2>, 1},
                      {"copy_slice_u4_x2", copy_kernel<0, 4>, 2}, {"copy_sweep_u4", copy_kernel<1, 4>, 1},
                      {"copy_sweep_u2_x2", copy_kernel<1, 2>, 2}};
  for (int rep = 0; rep < 3; ++rep)
    for (const CV &v : cvars) {
      const int grid = ncu * v.per_cu;
      for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(v.f, grid, 512, 0, 0, bufs[k % 4], bufs[(k + 1) % 4], nvec);
      CK(hipStreamSynchronize(0));
      CK(hipEventRecord(a, 0));
      for (int k = 0; k < K; ++k) hipLaunchKernelGGL(v.f, grid, 512, 0, 0, bufs[k % 4], bufs[(k + 2) % 4], nvec);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      printf(" {\"variant\": \"%s\", \"rep\": %d, \"us_per_launch\": %.2f, \"GBps_read_plus_write\": %.1f},\n",
             v.name, rep, ms * 1e3 / K, 2.0 * bytes * K / (ms * 1e-3) / 1e9);
      fflush(stdout);
    }
  printf(" {}]}\n");
  return 0;
}
