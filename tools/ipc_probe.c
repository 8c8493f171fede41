/* tools/ipc_probe.c -- measurement tool: when does the HIP runtime refuse an
 * IPC export (hipIpcGetMemHandle "invalid argument"), and does an import
 * ever fail?  DESIGN.md 7b: round 5's device-ring holders saw the refusal on
 * their FIRST allocation only (~1 ring in 100), sticky to that allocation.
 * Each run of this program is one fresh process (the holder's situation);
 * tools/ipc_probe.sh runs it hundreds of times per variant.
 *
 *   ipc_probe export VARIANT   one JSON line: every allocation's export result
 *     first     hipSetDevice, then 2 MiB hipMalloc + hipMemset + export, x3
 *               (the pre-primer holder: the first allocation is a ring block)
 *     delay     as first, after 500 ms of sleep following hipSetDevice
 *               (is it the time since start, or the first allocation?)
 *     order     allocate A then B (both memset), export B first, then A
 *               (is it the first allocation, or the first export call?)
 *     nomemset  as first without the hipMemset (does touching it matter?)
 *   ipc_probe import KEY       connect to the device ring at KEY (libpafdada:
 *               every block's handle opened), disconnect; one JSON line
 *
 * Build: make -C paf-baseband2power_amd bin/ipc_probe (links libamdhip64 and
 * libpafdada). */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "b2p_dada.h"

static double t0;

static double now_ms(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec * 1e3 + (double)t.tv_nsec * 1e-6;
}

static void emit(const char *variant, const char *what, int idx, hipError_t rc, double at) {
  printf("%s{\"alloc\": \"%s\", \"index\": %d, \"rc\": %d, \"err\": \"%s\", \"ms\": %.1f}", idx ? ", " : "", what,
         idx, (int)rc, rc == hipSuccess ? "" : hipGetErrorString(rc), at);
  (void)variant;
}

static int export_variant(const char *v) {
  const size_t sz = 2u << 20;
  hipError_t rc = hipSetDevice(0);
  const double t_init = now_ms() - t0;
  if (rc != hipSuccess) {
    printf("{\"variant\": \"%s\", \"setdevice\": \"%s\"}\n", v, hipGetErrorString(rc));
    return 1;
  }
  if (!strcmp(v, "delay")) usleep(500000);
  printf("{\"variant\": \"%s\", \"pid\": %d, \"init_ms\": %.1f, \"exports\": [", v, (int)getpid(), t_init);
  hipIpcMemHandle_t h;
  if (!strcmp(v, "order")) {
    void *a = NULL, *b = NULL;
    if (hipMalloc(&a, sz) != hipSuccess || hipMalloc(&b, sz) != hipSuccess) return 1;
    (void)hipMemset(a, 0, sz);
    (void)hipMemset(b, 0, sz);
    (void)hipDeviceSynchronize();
    rc = hipIpcGetMemHandle(&h, b);
    emit(v, "B (second allocation, first export)", 0, rc, now_ms() - t0);
    rc = hipIpcGetMemHandle(&h, a);
    emit(v, "A (first allocation, second export)", 1, rc, now_ms() - t0);
    (void)hipFree(a);
    (void)hipFree(b);
  } else {
    void *p[3] = {NULL, NULL, NULL};
    for (int i = 0; i < 3; i++) {
      if (hipMalloc(&p[i], sz) != hipSuccess) return 1;
      if (strcmp(v, "nomemset")) {
        (void)hipMemset(p[i], 0, sz);
        (void)hipDeviceSynchronize();
      }
      rc = hipIpcGetMemHandle(&h, p[i]);
      char what[32];
      snprintf(what, sizeof what, "allocation %d", i);
      emit(v, what, i, rc, now_ms() - t0);
    }
    for (int i = 0; i < 3; i++) (void)hipFree(p[i]);
  }
  printf("]}\n");
  return 0;
}

static int import_ring(const char *keyhex) {
  unsigned key = 0;
  if (sscanf(keyhex, "%x", &key) != 1) return 2;
  dada_hdu_t *h = dada_hdu_create(NULL);
  dada_hdu_set_key(h, (key_t)key);
  const double a = now_ms();
  const int rc = dada_hdu_connect(h);
  const double b = now_ms();
  printf("{\"import\": \"%x\", \"pid\": %d, \"rc\": %d, \"why\": \"%s\", \"connect_ms\": %.1f, \"start_ms\": %.1f}\n",
         key, (int)getpid(), rc, rc ? dada_device_error() : "", b - a, a - t0);
  if (rc == 0) dada_hdu_disconnect(h);
  dada_hdu_destroy(h);
  return rc ? 1 : 0;
}

int main(int argc, char **argv) {
  t0 = now_ms();
  if (argc == 3 && !strcmp(argv[1], "export")) return export_variant(argv[2]);
  if (argc == 3 && !strcmp(argv[1], "import")) return import_ring(argv[2]);
  fprintf(stderr, "usage: ipc_probe export first|delay|order|nomemset | ipc_probe import KEY\n");
  return 2;
}
