// h2d_probe -- the box's host-to-device copy ceiling (diagnostic only, not
// the product): the bound of configs[2] (a pinned capture buffer fed to the
// GPU, bench.py --config c3).  Copies a pinned 4-GiB host buffer to HBM in
// chunks of 64/256/1024 MiB on one or two streams, timed with hipEvents.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main() {
  const size_t total = 4ull << 30;
  void *h, *d;
  CK(hipHostMalloc(&h, total, hipHostMallocDefault));
  CK(hipMalloc(&d, total));
  for (size_t i = 0; i < total; i += 4096) ((char *)h)[i] = (char)i;
  hipStream_t st[2];
  for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b, e1;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
  printf("{\"bytes\": %zu, \"results\": [\n", total);
  for (int rep = 0; rep < 3; ++rep)
    for (size_t chunk_mib : {64, 256, 1024})
      for (int ns = 1; ns <= 2; ++ns) {
        const size_t chunk = chunk_mib << 20;
        CK(hipMemcpy(d, h, chunk, hipMemcpyHostToDevice));  // warm
        CK(hipEventRecord(a, st[0]));
        if (ns > 1) CK(hipStreamWaitEvent(st[1], a, 0));
        size_t k = 0;
        for (size_t off = 0; off < total; off += chunk, ++k)
          CK(hipMemcpyAsync((char *)d + off, (char *)h + off, chunk, hipMemcpyHostToDevice, st[k % ns]));
        if (ns > 1) {
          CK(hipEventRecord(e1, st[1]));
          CK(hipStreamWaitEvent(st[0], e1, 0));
        }
        CK(hipEventRecord(b, st[0]));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        printf(" {\"rep\": %d, \"chunk_MiB\": %zu, \"streams\": %d, \"GBps\": %.2f},\n", rep, chunk_mib, ns,
               total / (ms * 1e-3) / 1e9);
        fflush(stdout);
      }
  printf(" {}]}\n");
  CK(hipHostFree(h));
  CK(hipFree(d));
  return 0;
}
