// h2d_probe -- the box's host-to-device copy ceiling (diagnostic only, not
// the product): the bound of configs[2] (a pinned capture buffer fed to the
// GPU, bench.py --config c3).  Copies a pinned 4-GiB host buffer to HBM in
// chunks of 64/256/1024 MiB on one or two streams, timed with hipEvents.
// Then the same 4 GiB as a host DADA ring holds it: a SysV shared-memory
// segment (or a plain allocation) pinned with hipHostRegister, which is what
// paf_baseband2power's host-ring path copies from (pin_block).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/ipc.h>
#include <sys/shm.h>

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
  // the host-ring sources, 256 MiB chunks on one stream
  for (int src = 0; src < 2; ++src) {
    void *r = nullptr;
    int shmid = -1;
    if (src == 0) {
      shmid = shmget(IPC_PRIVATE, total, IPC_CREAT | 0600);
      if (shmid < 0) { perror("shmget"); continue; }
      r = shmat(shmid, nullptr, 0);
      shmctl(shmid, IPC_RMID, nullptr);  // removed once detached
      if (r == (void *)-1) { perror("shmat"); continue; }
    } else {
      r = aligned_alloc(4096, total);
      if (!r) continue;
    }
    for (size_t i = 0; i < total; i += 4096) ((char *)r)[i] = (char)i;
    CK(hipHostRegister(r, total, hipHostRegisterDefault));
    for (int rep = 0; rep < 3; ++rep) {
      const size_t chunk = 256ull << 20;
      CK(hipMemcpy(d, r, chunk, hipMemcpyHostToDevice));
      CK(hipEventRecord(a, st[0]));
      for (size_t off = 0; off < total; off += chunk)
        CK(hipMemcpyAsync((char *)d + off, (char *)r + off, chunk, hipMemcpyHostToDevice, st[0]));
      CK(hipEventRecord(b, st[0]));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      printf(" {\"rep\": %d, \"source\": \"%s\", \"chunk_MiB\": 256, \"streams\": 1, \"GBps\": %.2f},\n", rep,
             src == 0 ? "SysV shm + hipHostRegister (host DADA ring)" : "aligned_alloc + hipHostRegister",
             total / (ms * 1e-3) / 1e9);
      fflush(stdout);
    }
    CK(hipHostUnregister(r));
    if (src == 0) shmdt(r); else free(r);
  }
  printf(" {}]}\n");
  CK(hipHostFree(h));
  CK(hipFree(d));
  return 0;
}
