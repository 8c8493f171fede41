/* tests/c/fake_hip.c -- TEST DOUBLE, never part of a product library.
 *
 * A host-memory stand-in for the eleven HIP runtime calls libpafdada reaches
 * through dlopen("libamdhip64.so.7") (csrc/dada/dada_device.c hip_load), so
 * the device-ring holder's lifecycle -- exports, the export record in block
 * 0's segment, the ordering rule, dada_db -d -- runs in the CPU suite
 * (tests/test_device_holder_cpu.py).  The test builds this file as
 * <tmp>/libamdhip64.so.7 and puts <tmp> first on LD_LIBRARY_PATH of the
 * processes it starts; nothing else ever loads it.
 *
 * FAKE_HIP_REFUSE=i,j,...  refuse the i-th, j-th ... hipIpcGetMemHandle call
 *                          of the process (0-based) with "invalid argument",
 *                          as the runtime refused first allocations (DESIGN.md
 *                          7b).  The holder's call 0 is its primer's.
 * FAKE_HIP_LOG=path        append "free <ptr>" per hipFree, "export <n>" per
 *                          export try, so a test sees when the holder frees.
 * FAKE_HIP_MEMCPY_FAIL=n   the n-th hipMemcpy of the process (1-based) fails,
 *                          as a copy into a block would on a HIP error. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

typedef struct {
  char reserved[64];
} fake_ipc_handle_t;

static char g_mapped[1 << 16]; /* what an imported handle points at */
static int g_nexport;

static void fake_log(const char *fmt, const void *p, long n) {
  const char *path = getenv("FAKE_HIP_LOG");
  if (!path) return;
  FILE *f = fopen(path, "a");
  if (!f) return;
  fprintf(f, fmt, p, n, (int)getpid());
  fclose(f);
}

static int refused(int call) {
  const char *e = getenv("FAKE_HIP_REFUSE");
  if (!e || !*e) return 0;
  char buf[256];
  snprintf(buf, sizeof buf, "%s", e);
  for (char *t = strtok(buf, ","); t; t = strtok(NULL, ","))
    if (atoi(t) == call) return 1;
  return 0;
}

int hipSetDevice(int d) { return d < 0; }
int hipMalloc(void **p, size_t n) { return posix_memalign(p, 4096, n ? n : 1) ? 2 : 0; }
int hipFree(void *p) {
  fake_log("free %p %ld pid %d\n", p, 0);
  free(p);
  return 0;
}
int hipMemset(void *p, int v, size_t n) {
  memset(p, v, n);
  return 0;
}
int hipIpcGetMemHandle(fake_ipc_handle_t *h, void *p) {
  const int call = g_nexport++;
  fake_log("export %p %ld pid %d\n", p, call);
  if (refused(call)) return 1; /* hipErrorInvalidValue */
  memset(h, 0, sizeof *h);
  memcpy(h->reserved, "FAKEHIP", 7);
  memcpy(h->reserved + 8, &p, sizeof p);
  return 0;
}
int hipIpcOpenMemHandle(void **p, fake_ipc_handle_t h, unsigned flags) {
  (void)flags;
  if (memcmp(h.reserved, "FAKEHIP", 7)) return 1;
  *p = g_mapped;
  return 0;
}
int hipIpcCloseMemHandle(void *p) { return p == g_mapped ? 0 : 1; }
int hipMemcpy(void *d, const void *s, size_t n, int kind) {
  static int calls;
  (void)d, (void)s, (void)n, (void)kind;
  const char *e = getenv("FAKE_HIP_MEMCPY_FAIL");
  if (e && ++calls == atoi(e)) return 2; /* hipErrorOutOfMemory-like: any failure */
  return 0; /* imported blocks are not backed here */
}
int hipDeviceSynchronize(void) { return 0; }
const char *hipGetErrorString(int e) { return e == 1 ? "invalid argument (fake_hip)" : "fake_hip error"; }
int hipMemGetAddressRange(void **base, size_t *size, void *p) {
  *base = p;
  *size = 0;
  return 0;
}
