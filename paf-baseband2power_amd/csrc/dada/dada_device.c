/*
 * dada_device.c -- GPU-resident ring blocks.
 *
 * PSRDADA keeps a device ring's blocks in GPU memory: on_device_id in the
 * sync segment names the device, and block i's shared segment (key + 0x10000
 * * (10+i)) holds a 64-B IPC memory handle instead of the data
 * (`ipc_alloc_cuda` in the reference's linked libpsrdada, @0x407ec0).  Here
 * the handles are HIP ones, and:
 *
 *  - a holder process (double-forked from the creator, so it outlives it)
 *    allocates the blocks with hipMalloc, publishes each block's handle in
 *    its segment, and keeps the memory alive until the ring is destroyed
 *    (SIGTERM) or its sync segment disappears (and, when DADA_HOLDER_IDLE_S
 *    is set, after that many seconds with no process attached but itself --
 *    a guard against rings orphaned by a killed run).  Its pid and state
 *    follow the handle in block 0's segment (dev_seg_t);
 *  - every process that connects opens the handles (hipIpcOpenMemHandle),
 *    so ipcbuf_get_next_read/write hand out device pointers;
 *  - producers and consumers order their kernels against the ring with
 *    their own stream synchronisation: a writer's kernels are complete
 *    before ipcbuf_mark_filled, a reader's before ipcbuf_mark_cleared.
 *
 * The creator forks: call dada_db_create_work from a single-threaded program
 * (the dada_db tool does; paf_b2p.dada runs that tool rather than forking a
 * threaded Python process).
 *
 * HIP is reached through dlopen of libamdhip64.so.7, so libpafdada still
 * loads (and host rings still work) on machines without ROCm; in a process
 * that already mapped a HIP runtime (torch, libpafb2p) the same one is used.
 */
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ipc.h>
#include <sys/shm.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include "dada_internal.h"

typedef struct {
  char reserved[DEV_HANDLE_BYTES];
} ipc_handle_t; /* hipIpcMemHandle_t, hip_runtime_api.h:688-690 */

static struct {
  int loaded;
  int (*set_device)(int);
  int (*malloc_)(void **, size_t);
  int (*free_)(void *);
  int (*memset_)(void *, int, size_t);
  int (*get_handle)(ipc_handle_t *, void *);
  int (*open_handle)(void **, ipc_handle_t, unsigned);
  int (*close_handle)(void *);
  int (*memcpy_)(void *, const void *, size_t, int);
  int (*sync)(void);
  const char *(*err_str)(int);
  int (*addr_range)(void **, size_t *, void *); /* hipMemGetAddressRange (diagnostics) */
} hip;

static int hip_load(void) {
  if (hip.loaded) return hip.loaded > 0 ? 0 : -1;
  void *h = dlopen("libamdhip64.so.7", RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
  if (!h) h = dlopen("libamdhip64.so.7", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("/opt/rocm/lib/libamdhip64.so.7", RTLD_NOW | RTLD_GLOBAL);
  if (!h) {
    hip.loaded = -1;
    return -1;
  }
#define SYM(field, name) *(void **)(&hip.field) = dlsym(h, name)
  SYM(set_device, "hipSetDevice");
  SYM(malloc_, "hipMalloc");
  SYM(free_, "hipFree");
  SYM(memset_, "hipMemset");
  SYM(get_handle, "hipIpcGetMemHandle");
  SYM(open_handle, "hipIpcOpenMemHandle");
  SYM(close_handle, "hipIpcCloseMemHandle");
  SYM(memcpy_, "hipMemcpy");
  SYM(sync, "hipDeviceSynchronize");
  SYM(err_str, "hipGetErrorString");
  SYM(addr_range, "hipMemGetAddressRange");
#undef SYM
  hip.loaded = (hip.set_device && hip.malloc_ && hip.free_ && hip.memset_ && hip.get_handle &&
                hip.open_handle && hip.close_handle && hip.memcpy_ && hip.sync && hip.err_str)
                   ? 1
                   : -1;
  return hip.loaded > 0 ? 0 : -1;
}

/* this thread's last device-ring failure (dada_device_error) */
static __thread char dev_err[200];

const char *dada_device_error(void) { return dev_err; }

static void dev_fail(const char *what, int code) {
  snprintf(dev_err, sizeof dev_err, "%s: %s (%d)", what, code >= 0 && hip.err_str ? hip.err_str(code) : "unavailable",
           code);
}

static void report(int fd, const char *what, int code) {
  char msg[240];
  int n = snprintf(msg, sizeof msg, "E%s: %s", what,
                   code >= 0 && hip.err_str ? hip.err_str(code) : "unavailable");
  if (n > 0) (void)!write(fd, msg, (size_t)n < sizeof msg ? (size_t)n : sizeof msg - 1);
}

#define DEV_ALLOC_ALIGN (2ull << 20)
#define DEV_EXPORT_TRIES 4

/* processes attached to block 0's segment besides the holder: the importers
 * (dada_internal.h).  A destroyer's momentary look (dev_stop_holder) can only
 * add to the count, so a race makes the holder wait a tick longer, never
 * free blocks an importer still has open. */
static long importers_attached(int seg0_id) {
  struct shmid_ds ds;
  if (shmctl(seg0_id, IPC_STAT, &ds) < 0) return 0; /* gone: nobody can be attached */
  const long n = (long)ds.shm_nattch - 1;
  return n > 0 ? n : 0;
}

/* the holder: owns the blocks until it is told to stop (SIGTERM/SIGINT/
 * SIGHUP), the ring is removed, or DADA_HOLDER_IDLE_S seconds pass with no
 * importer -- and in every case only once no importer is attached (the
 * ordering rule in dada_internal.h), so no process can still have a block
 * mapped when it is freed */
static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + (double)t.tv_nsec * 1e-9;
}

static void holder(ipcbuf_t *id, int device, int wfd) {
  const double t_start = now_s();
  int rc;
  const uint64_t n = id->sync->nbufs, bufsz = id->sync->bufsz;
  dev_seg_t *seg0 = id->shm_addr[0];
  const int seg0_id = id->shmid[0];
  void **blk = calloc(n, sizeof(void *));
  if (!blk) {
    report(wfd, "calloc", -1);
    _exit(1);
  }
  if (hip_load() < 0) {
    report(wfd, "dlopen libamdhip64.so.7", -1);
    _exit(1);
  }
  if ((rc = hip.set_device(device)) != 0) {
    report(wfd, "hipSetDevice", rc);
    _exit(1);
  }
  /* each block its own allocation of whole 2 MiB pages: HIP serves small
   * requests (a 29 952-B block did) from a shared sub-allocated chunk, and
   * hipIpcGetMemHandle refuses a pointer inside one ("invalid argument").
   * An export that still fails is retried with a fresh allocation (the
   * failed one kept aside so hipMalloc cannot hand it back), up to
   * DEV_EXPORT_TRIES times per block; the first failure's call, error and
   * hipMemGetAddressRange of the pointer are reported with the retry count
   * (the R message), so a retry is never silent. */
  const uint64_t alloc = (bufsz + DEV_ALLOC_ALIGN - 1) / DEV_ALLOC_ALIGN * DEV_ALLOC_ALIGN;
  void *spare[DEV_EXPORT_TRIES * 4];
  int nspare = 0, retries = 0;
  char first[240] = "";
  /* The primer: round 5's probes (profiles/r05_devring_leak*.jsonl) found the
   * export refusal only ever on a holder's FIRST device allocation (block
   * 0, ~210 ms after start), about 1 ring in 100, sticky to that allocation
   * (refused again 20 ms later) while a fresh one exported.  So the holder
   * makes its first allocation a 2 MiB primer that no ring block uses,
   * tries to export it, and keeps it until exit; whether the primer's
   * export was refused is reported with the retries (the "P" count). */
  void *primer = NULL;
  int primer_refused = 0;
  /* DADA_HOLDER_NO_PRIMER=1: diagnostics only (tools/devring_probe.py
   * noprimer): the first allocation is block 0 again, as before round 5 */
  const char *no_primer = getenv("DADA_HOLDER_NO_PRIMER");
  if (no_primer && no_primer[0] == '1') {
    /* no primer */
  } else if (hip.malloc_(&primer, DEV_ALLOC_ALIGN) == 0) {
    ipc_handle_t ph;
    primer_refused = hip.memset_(primer, 0, DEV_ALLOC_ALIGN) == 0 && hip.get_handle(&ph, primer) != 0;
  } else {
    primer = NULL;
  }
  for (uint64_t i = 0; i < n; i++) {
    ipc_handle_t h;
    const char *what = "hipMalloc";
    for (int t = 0;; t++) {
      blk[i] = NULL;
      what = "hipMalloc";
      if ((rc = hip.malloc_(&blk[i], alloc)) == 0 && (what = "hipMemset", rc = hip.memset_(blk[i], 0, alloc)) == 0 &&
          (what = "hipIpcGetMemHandle", rc = hip.get_handle(&h, blk[i])) == 0)
        break;
      if (rc != 0 && blk[i] && !strcmp(what, "hipIpcGetMemHandle")) {
        /* the same pointer once more after a pause: tells a transient
         * export failure from one that sticks to the allocation */
        struct timespec pause = {0, 20 * 1000 * 1000};
        nanosleep(&pause, NULL);
        const int again = hip.get_handle(&h, blk[i]);
        if (!first[0]) {
          void *base = NULL;
          size_t size = 0;
          const int ar = hip.addr_range ? hip.addr_range(&base, &size, blk[i]) : -1;
          snprintf(first, sizeof first,
                   "%s: %s (%d) on block %llu of %llu B, range %s%+lld %llu B, %.0f ms after start; "
                   "same pointer 20 ms later: %s",
                   what, hip.err_str(rc), rc, (unsigned long long)i, (unsigned long long)alloc,
                   ar == 0 ? "base" : "?", ar == 0 ? (long long)((char *)blk[i] - (char *)base) : 0LL,
                   (unsigned long long)size, (now_s() - t_start) * 1e3, again == 0 ? "exported" : hip.err_str(again));
        }
        if (again == 0) {
          retries++;
          break;
        }
      }
      if (!first[0]) {
        void *base = NULL;
        size_t size = 0;
        const int ar = blk[i] && hip.addr_range ? hip.addr_range(&base, &size, blk[i]) : -1;
        snprintf(first, sizeof first, "%s: %s (%d) on block %llu of %llu B, range %s%+lld %llu B", what,
                 hip.err_str(rc), rc, (unsigned long long)i, (unsigned long long)alloc, ar == 0 ? "base" : "?",
                 ar == 0 ? (long long)((char *)blk[i] - (char *)base) : 0LL, (unsigned long long)size);
      }
      if (t + 1 >= DEV_EXPORT_TRIES || !blk[i] || nspare == (int)(sizeof spare / sizeof spare[0])) {
        char w[160];
        snprintf(w, sizeof w, "%s (block %llu of %llu, %llu B, try %d)", what, (unsigned long long)i,
                 (unsigned long long)n, (unsigned long long)alloc, t + 1);
        report(wfd, w, rc);
        for (uint64_t j = 0; j <= i; j++)
          if (blk[j]) hip.free_(blk[j]);
        for (int j = 0; j < nspare; j++) hip.free_(spare[j]);
        _exit(1);
      }
      spare[nspare++] = blk[i];
      retries++;
      struct timespec pause = {0, 20 * 1000 * 1000};
      nanosleep(&pause, NULL);
    }
    memcpy(id->shm_addr[i], &h, DEV_HANDLE_BYTES);
  }
  for (int j = 0; j < nspare; j++) hip.free_(spare[j]);
  hip.sync();
  seg0->holder_pid = (int32_t)getpid();
  seg0->export_retries = retries;
  seg0->primer_refused = primer_refused;
  __atomic_store_n(&seg0->holder_state, 1, __ATOMIC_RELEASE);
  char ready[300];
  /* 'R' + export retries of ring blocks, 'P' + 1 if the primer's export was refused */
  const int nr = snprintf(ready, sizeof ready, "R%d P%d %s", retries, primer_refused, first);
  (void)!write(wfd, ready, (size_t)nr < sizeof ready ? (size_t)nr : sizeof ready - 1);
  close(wfd);

  sigset_t set;
  sigemptyset(&set);
  sigaddset(&set, SIGTERM);
  sigaddset(&set, SIGINT);
  sigaddset(&set, SIGHUP);
  const char *idle_env = getenv("DADA_HOLDER_IDLE_S");
  const long idle_max = idle_env ? atol(idle_env) : 0;
  long idle = 0;
  int stopping = 0;
  for (;;) {
    /* 1-s ticks while serving; 10-ms ticks while draining the importers */
    struct timespec tick = {stopping ? 0 : 1, stopping ? 10 * 1000 * 1000 : 0};
    if (sigtimedwait(&set, NULL, &tick) > 0) stopping = 1;
    struct shmid_ds ds;
    if (shmctl(id->syncid, IPC_STAT, &ds) < 0 || (ds.shm_perm.mode & SHM_DEST)) stopping = 1; /* ring removed */
    const long others = importers_attached(seg0_id);
    __atomic_store_n(&seg0->importers, (int32_t)others, __ATOMIC_RELEASE);
    if (!stopping) {
      idle = others == 0 ? idle + 1 : 0;
      if (idle_max > 0 && idle >= idle_max) stopping = 1;
    }
    if (stopping && others == 0) break;
  }
  for (uint64_t i = 0; i < n; i++) hip.free_(blk[i]);
  if (primer) hip.free_(primer);
  __atomic_store_n(&seg0->holder_state, 2, __ATOMIC_RELEASE);
  _exit(0);
}

int dev_create_blocks(ipcbuf_t *id, int device) {
  int fds[2];
  if (pipe(fds) < 0) return -1;
  /* block the stop signals before forking: the holder takes them with
   * sigtimedwait and never runs a handler */
  sigset_t set, old;
  sigemptyset(&set);
  sigaddset(&set, SIGTERM);
  sigaddset(&set, SIGINT);
  sigaddset(&set, SIGHUP);
  pthread_sigmask(SIG_BLOCK, &set, &old);
  pid_t mid = fork();
  if (mid == 0) {
    close(fds[0]);
    setsid();
    pid_t h = fork();
    if (h != 0) _exit(h < 0 ? 1 : 0);
    /* the holder: detached, stdio on /dev/null so no caller waits on it */
    int dn = open("/dev/null", O_RDWR);
    if (dn >= 0) {
      dup2(dn, 0);
      dup2(dn, 1);
      dup2(dn, 2);
      if (dn > 2) close(dn);
    }
    holder(id, device, fds[1]);
  }
  pthread_sigmask(SIG_SETMASK, &old, NULL);
  close(fds[1]);
  if (mid < 0) {
    close(fds[0]);
    return -1;
  }
  int st = 0;
  while (waitpid(mid, &st, 0) < 0 && errno == EINTR) {
  }
  char msg[200] = {0};
  ssize_t got;
  do {
    got = read(fds[0], msg, sizeof msg - 1);
  } while (got < 0 && errno == EINTR);
  close(fds[0]);
  if (got >= 1 && msg[0] == 'R') {
    const int retries = atoi(msg + 1);
    const char *pp = strstr(msg, " P");
    const int primer_refused = pp ? atoi(pp + 2) : 0;
    if (retries > 0) {
      const char *why = pp ? strchr(pp + 1, ' ') : NULL;
      fprintf(stderr, "dada device ring: %d IPC export retr%s in the holder (first: %s)\n", retries,
              retries == 1 ? "y" : "ies", why ? why + 1 : "?");
    }
    if (primer_refused) /* diagnostics only: no ring block is affected */
      fprintf(stderr, "dada device ring: the holder's primer allocation was not exportable\n");
    return 0;
  }
  fprintf(stderr, "dada device ring: holder failed: %s\n", got > 1 ? msg + 1 : "no reply");
  errno = ENODEV;
  return -1;
}

/* one look at block 0's segment, attached only for the look (the holder
 * counts attachments as importers): 0, or -1 once the segment is gone */
int dev_look_seg0(int seg0_id, dev_seg_t *out) {
  const dev_seg_t *seg0 = shmat(seg0_id, NULL, SHM_RDONLY);
  if (seg0 == (void *)-1) return -1;
  memcpy(out->handle, seg0->handle, sizeof out->handle);
  out->holder_pid = seg0->holder_pid;
  out->holder_state = __atomic_load_n(&seg0->holder_state, __ATOMIC_ACQUIRE);
  out->importers = __atomic_load_n(&seg0->importers, __ATOMIC_ACQUIRE);
  out->export_retries = seg0->export_retries;
  out->primer_refused = seg0->primer_refused;
  shmdt(seg0);
  return 0;
}

/* until process pid has exited (gone, or a zombie whose resources -- its GPU
 * context among them -- are released), at most ms milliseconds */
static void wait_exited(pid_t pid, int ms) {
  char path[64], st[256];
  snprintf(path, sizeof path, "/proc/%d/stat", (int)pid);
  for (int t = 0; t < ms; t += 5) {
    if (kill(pid, 0) < 0 && errno == ESRCH) return;
    FILE *f = fopen(path, "r");
    if (!f) return;
    const size_t n = fread(st, 1, sizeof st - 1, f);
    fclose(f);
    st[n] = 0;
    const char *q = strrchr(st, ')'); /* "pid (comm) S ..." */
    if (q && q[1] == ' ' && (q[2] == 'Z' || q[2] == 'X')) return;
    nanosleep(&(struct timespec){0, 5 * 1000 * 1000}, NULL);
  }
}

int dev_stop_holder(int seg0_id) {
  dev_seg_t v;
  if (dev_look_seg0(seg0_id, &v) < 0 || v.holder_pid <= 0 || v.holder_state != 1) return 0;
  if (kill(v.holder_pid, SIGTERM) < 0) return errno == ESRCH ? 0 : -1;
  /* the holder frees the blocks once no importer is attached; this process
   * looks every 10 ms and stays attached for no longer than each look, so
   * dying while it waits (Ctrl-C on dada_db -d, a test timeout) leaves the
   * holder's count as it was */
  const pid_t pid = v.holder_pid;
  for (int i = 0; i < 1000; i++) { /* <= 10 s */
    struct timespec t = {0, 10 * 1000 * 1000};
    nanosleep(&t, NULL);
    if (dev_look_seg0(seg0_id, &v) < 0 || v.holder_state == 2) {
      /* and until the holder's process has ended: a holder that starts
       * while the previous one's GPU context is still being torn down can
       * have its first allocation refused IPC export (DESIGN.md 7b,
       * profiles/r06_devring_*.jsonl) */
      wait_exited(pid, 3000);
      return 0;
    }
  }
  snprintf(dev_err, sizeof dev_err,
           "device ring holder %d: %d process(es) still have the blocks open; it frees them when they detach",
           v.holder_pid, v.importers);
  errno = EBUSY;
  return -1;
}

int dev_open_blocks(ipcbuf_t *id) {
  const dev_seg_t *seg0 = id->shm_addr[0];
  int rc;
  if (__atomic_load_n(&seg0->holder_state, __ATOMIC_ACQUIRE) != 1) {
    snprintf(dev_err, sizeof dev_err, "device ring: no live holder (state %d)",
             __atomic_load_n(&seg0->holder_state, __ATOMIC_ACQUIRE));
    errno = ENODEV;
    return -1;
  }
  if (hip_load() < 0) {
    dev_fail("dlopen libamdhip64.so.7", -1);
    errno = ENODEV;
    return -1;
  }
  if ((rc = hip.set_device(id->sync->on_device_id)) != 0) {
    dev_fail("hipSetDevice", rc);
    errno = ENODEV;
    return -1;
  }
  for (uint64_t i = 0; i < id->sync->nbufs; i++) {
    ipc_handle_t h;
    void *p = NULL;
    memcpy(&h, id->shm_addr[i], DEV_HANDLE_BYTES);
    if ((rc = hip.open_handle(&p, h, 1 /* hipIpcMemLazyEnablePeerAccess */)) != 0) {
      char w[80];
      snprintf(w, sizeof w, "hipIpcOpenMemHandle (block %llu of %llu)", (unsigned long long)i,
               (unsigned long long)id->sync->nbufs);
      dev_fail(w, rc);
      for (uint64_t j = 0; j < i; j++) { /* none of them stays open */
        hip.close_handle(id->buffer[j]);
        id->buffer[j] = NULL;
      }
      errno = ENODEV;
      return -1;
    }
    id->buffer[i] = p;
  }
  return 0;
}

void dev_close_blocks(ipcbuf_t *id) {
  if (hip_load() < 0) return;
  for (uint64_t i = 0; i < id->sync->nbufs; i++)
    if (id->buffer[i]) {
      const int rc = hip.close_handle(id->buffer[i]);
      if (rc != 0) { /* kept for dada_device_error(); the block is dropped either way */
        char w[80];
        snprintf(w, sizeof w, "hipIpcCloseMemHandle (block %llu)", (unsigned long long)i);
        dev_fail(w, rc);
      }
      id->buffer[i] = NULL;
    }
}

int dev_copy(void *dst, const void *src, uint64_t n, int into_block) {
  if (!n) return 0;
  if (hip_load() < 0) {
    dev_fail("dlopen libamdhip64.so.7", -1);
    return -1;
  }
  int rc = hip.memcpy_(dst, src, n, 4 /* hipMemcpyDefault */);
  /* into a block: the bytes are in HBM before the caller marks it filled
   * (hipMemcpy does not promise completion for a pageable source) */
  if (rc == 0 && into_block) rc = hip.sync();
  if (rc != 0) {
    char w[96];
    snprintf(w, sizeof w, "hipMemcpy of %llu B (%p <- %p)", (unsigned long long)n, dst, src);
    dev_fail(w, rc);
    return -1;
  }
  return 0;
}

/* zero n bytes of a device block, finished on return (ipc_zero_buffer_cuda) */
int dev_zero(void *dst, uint64_t n) {
  if (!n) return 0;
  if (hip_load() < 0) {
    dev_fail("dlopen libamdhip64.so.7", -1);
    return -1;
  }
  int rc = hip.memset_(dst, 0, n);
  if (rc == 0) rc = hip.sync();
  if (rc != 0) {
    dev_fail("hipMemset", rc);
    return -1;
  }
  return 0;
}
