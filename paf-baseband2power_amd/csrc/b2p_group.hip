// Multi-GPU collectives of the integrator (include/b2p.h "b2p_group").
//
// sub-bands shard with no exchange during the integrate; the
// collective is the final gather of each sub-band's spectrum to the root
// device -- RCCL over xGMI (ncclCommInitAll + ncclGather,
// /opt/rocm/include/rccl/rccl.h:236,745).  The second mode splits ONE
// sub-band's integration across members by time; their exact uint64 partial
// sums meet in an ncclReduce(ncclUint64, ncclSum) at the root, so the result
// is bit-identical to one GPU's.  Both are issued on each context's own
// stream, ordered behind that context's finalize.  Mode 1 replaces
// RCCL with peer copies for rigs where several contexts share one device
// (RCCL refuses duplicate devices in a communicator).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <vector>

#include "b2p.h"
#include "b2p_internal.h"

struct b2p_group {
  int n = 0;
  int mode = 0;  // 0 RCCL, 1 device copies
  std::vector<b2p_ctx_t *> ctx;
  std::vector<int> dev;
  std::vector<hipStream_t> stream;
  std::vector<ncclComm_t> comm;
  std::vector<hipEvent_t> done;  // mode 1: member r's spectrum is final
  // b2p_group_gather_async: the group's own streams (not the members'), and
  // one event per issued gather (ring of 8), waited on by b2p_group_wait
  std::vector<hipStream_t> gstream;
  hipEvent_t gev[8] = {};
  uint64_t gnext = 0;
  unsigned long long *scratch = nullptr;  // mode 1 reduce: rows gathered on the root
  uint64_t scratch_count = 0;
  uint32_t nout = 0;
  int timeout_ms = 60000;
  int dead = 0;  // communicators aborted (time limit or RCCL error): close only
  char err[256] = {0};
};

namespace {
thread_local char g_gerr[256];
int gerr(b2p_group_t *g, int code, const char *what, const char *detail) {
  snprintf(g ? g->err : g_gerr, 256, "%s: %s", what, detail ? detail : "");
  return code;
}
double now_s() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

// Abort every communicator: after a time limit or an asynchronous RCCL
// error nothing else may be issued on them (rccl.h:266-271).
void abort_comms(b2p_group_t *g) {
  for (auto &c : g->comm)
    if (c) {
      ncclCommAbort(c);
      c = nullptr;
    }
  g->dead = 1;
}

// Poll the non-blocking communicators until none is ncclInProgress, an
// asynchronous error shows, or the deadline passes (then abort).
int settle_comms(b2p_group_t *g, double deadline, const char *what) {
  for (;;) {
    bool pending = false;
    for (int r = 0; r < (int)g->comm.size(); ++r) {
      ncclResult_t st = ncclSuccess;
      ncclResult_t q = ncclCommGetAsyncError(g->comm[r], &st);
      if (q != ncclSuccess) st = q;
      if (st == ncclInProgress) {
        pending = true;
      } else if (st != ncclSuccess) {
        char d[160];
        snprintf(d, sizeof d, "member %d (device %d): %s", r, g->dev[r], ncclGetErrorString(st));
        abort_comms(g);
        return gerr(g, B2P_EHIP, what, d);
      }
    }
    if (!pending) return B2P_OK;
    if (now_s() > deadline) {
      char d[96];
      snprintf(d, sizeof d, "not complete after %d ms; communicators aborted", g->timeout_ms);
      abort_comms(g);
      return gerr(g, B2P_ETIMEDOUT, what, d);
    }
    usleep(200);
  }
}

// The collective's work on every member stream, with the group's deadline.
int wait_streams(b2p_group_t *g, const char *what) {
  const double deadline = now_s() + 1e-3 * g->timeout_ms;
  for (;;) {
    bool busy = false;
    for (int r = 0; r < g->n; ++r) {
      (void)hipSetDevice(g->dev[r]);
      hipError_t e = hipStreamQuery(g->stream[r]);
      if (e == hipErrorNotReady) {
        busy = true;
      } else if (e != hipSuccess) {
        if (!g->comm.empty()) abort_comms(g);
        g->dead = 1;
        return gerr(g, B2P_EHIP, what, hipGetErrorString(e));
      }
    }
    if (!g->comm.empty()) {  // an RCCL failure shows here before the stream idles
      ncclResult_t st = ncclSuccess;
      for (int r = 0; r < (int)g->comm.size() && st == ncclSuccess; ++r) {
        ncclResult_t q = ncclCommGetAsyncError(g->comm[r], &st);
        if (q != ncclSuccess) st = q;
        if (st == ncclInProgress) st = ncclSuccess;
      }
      if (st != ncclSuccess) {
        abort_comms(g);
        return gerr(g, B2P_EHIP, what, ncclGetErrorString(st));
      }
    }
    if (!busy) return B2P_OK;
    if (now_s() > deadline) {
      char d[96];
      snprintf(d, sizeof d, "not complete after %d ms; communicators aborted", g->timeout_ms);
      if (!g->comm.empty()) abort_comms(g);
      g->dead = 1;
      return gerr(g, B2P_ETIMEDOUT, what, d);
    }
    usleep(50);
  }
}

}  // namespace

extern "C" {

int b2p_group_open(b2p_group_t **out, b2p_ctx_t *const *ctxs, int n, int mode) {
  return b2p_group_open_timed(out, ctxs, n, mode, 60000);
}

int b2p_group_open_timed(b2p_group_t **out, b2p_ctx_t *const *ctxs, int n, int mode, int timeout_ms) {
  if (!out || !ctxs || n < 1 || (mode != 0 && mode != 1) || timeout_ms <= 0) return B2P_EINVAL;
  *out = nullptr;
  b2p_group_t *g = new (std::nothrow) b2p_group_t();
  if (!g) return B2P_ENOMEM;
  g->n = n;
  g->mode = mode;
  g->timeout_ms = timeout_ms;
  for (int r = 0; r < n; ++r) {
    b2p_info_t info;
    if (!ctxs[r] || b2p_get_info(ctxs[r], &info) != B2P_OK) {
      delete g;
      return gerr(nullptr, B2P_EINVAL, "b2p_group_open", "null context");
    }
    if (r == 0) g->nout = info.nout;
    if (info.nout != g->nout) {
      delete g;
      return gerr(nullptr, B2P_EINVAL, "b2p_group_open", "members differ in nout");
    }
    g->ctx.push_back(ctxs[r]);
    g->dev.push_back((int)info.device);
    g->stream.push_back((hipStream_t)b2p_internal_stream(ctxs[r]));
  }
  if (mode == 0) {
    // ncclCommInitAll's work (rccl.h:236), made non-blocking so that a
    // set-up that never completes ends at the time limit instead of hanging
    // the process: one unique id, every rank initialised inside one group
    // call, then polled
    const double deadline = now_s() + 1e-3 * timeout_ms;
    ncclUniqueId id;
    ncclResult_t nr = ncclGetUniqueId(&id);
    if (nr != ncclSuccess) {
      int rc = gerr(nullptr, B2P_EHIP, "ncclGetUniqueId", ncclGetErrorString(nr));
      delete g;
      return rc;
    }
    g->comm.assign(n, nullptr);
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    nr = ncclGroupStart();
    for (int r = 0; r < n && (nr == ncclSuccess || nr == ncclInProgress); ++r) {
      (void)hipSetDevice(g->dev[r]);
      nr = ncclCommInitRankConfig(&g->comm[r], n, id, r, &cfg);
    }
    ncclResult_t ne = ncclGroupEnd();
    if (nr == ncclSuccess || nr == ncclInProgress) nr = ne;
    int rc = B2P_OK;
    if (nr != ncclSuccess && nr != ncclInProgress) {
      char d[160];
      snprintf(d, sizeof d, "%s (%d members)", ncclGetErrorString(nr), n);
      rc = gerr(g, B2P_EHIP, "ncclCommInitRankConfig", d);
      abort_comms(g);
    } else {
      rc = settle_comms(g, deadline, "RCCL communicator set-up");
    }
    if (rc != B2P_OK) {
      snprintf(g_gerr, sizeof g_gerr, "%s", g->err);
      g->comm.clear();
      delete g;
      return rc;
    }
  } else {
    g->done.resize(n, nullptr);
    for (int r = 0; r < n; ++r) {
      (void)hipSetDevice(g->dev[r]);
      if (hipEventCreateWithFlags(&g->done[r], hipEventDisableTiming) != hipSuccess) {
        b2p_group_close(g);
        return gerr(nullptr, B2P_EHIP, "b2p_group_open", "hipEventCreate");
      }
    }
  }
  *out = g;
  return B2P_OK;
}

int b2p_group_gather(b2p_group_t *g, float *const *spectra, float *root_out) {
  return b2p_group_gather_n(g, spectra, 1, root_out);
}

// nspec consecutive spectra per member in one collective: root_out holds
// member r's nspec x nout floats at r * nspec * nout (member-major)
int b2p_group_gather_n(b2p_group_t *g, float *const *spectra, uint32_t nspec, float *root_out) {
  if (!g || !spectra || !root_out || nspec < 1) return B2P_EINVAL;
  if (g->dead) return gerr(g, B2P_ETIMEDOUT, "b2p_group_gather", "group aborted earlier; close it");
  // every member's deferred finalize must be enqueued before the gather
  for (int r = 0; r < g->n; ++r) {
    int rc = b2p_internal_flush(g->ctx[r]);
    if (rc != B2P_OK) return gerr(g, rc, "flush", b2p_last_error(g->ctx[r]));
  }
  const size_t count = (size_t)g->nout * nspec, bytes = count * sizeof(float);
  if (g->mode == 0) {
    ncclResult_t nr = ncclGroupStart();
    for (int r = 0; r < g->n && nr == ncclSuccess; ++r) {
      (void)hipSetDevice(g->dev[r]);
      nr = ncclGather(spectra[r], r == 0 ? root_out : nullptr, count, ncclFloat32, 0, g->comm[r],
                      g->stream[r]);
    }
    ncclResult_t ne = ncclGroupEnd();
    if ((nr != ncclSuccess && nr != ncclInProgress) || (ne != ncclSuccess && ne != ncclInProgress))
      return gerr(g, B2P_EHIP, "ncclGather", ncclGetErrorString(nr != ncclSuccess ? nr : ne));
    return settle_comms(g, now_s() + 1e-3 * g->timeout_ms, "ncclGather enqueue");
  }
  for (int r = 0; r < g->n; ++r) {
    (void)hipSetDevice(g->dev[r]);
    if (hipEventRecord(g->done[r], g->stream[r]) != hipSuccess)
      return gerr(g, B2P_EHIP, "hipEventRecord", "");
  }
  (void)hipSetDevice(g->dev[0]);
  for (int r = 0; r < g->n; ++r) {
    if (hipStreamWaitEvent(g->stream[0], g->done[r], 0) != hipSuccess ||
        hipMemcpyPeerAsync(root_out + (size_t)r * count, g->dev[0], spectra[r], g->dev[r], bytes,
                           g->stream[0]) != hipSuccess)
      return gerr(g, B2P_EHIP, "hipMemcpyPeerAsync", "");
  }
  return B2P_OK;
}

// Gather behind the members' fences, on streams of the group's own: the
// members' next launches are not held behind the collective, and their
// pending finalizes are left to ride those launches.
int b2p_group_gather_async(b2p_group_t *g, float *const *spectra, uint32_t nspec, float *root_out,
                           const uint64_t *tickets, float *host_out, uint64_t *gticket) {
  if (!g || !spectra || !root_out || !tickets || !gticket || nspec < 1) return B2P_EINVAL;
  if (g->dead) return gerr(g, B2P_ETIMEDOUT, "b2p_group_gather_async", "group aborted earlier; close it");
  if (g->gnext >= 8) {  // gather gnext - 8's event is recorded again: it must have completed,
    // waited for like b2p_group_wait (bounded by the group's limit, the
    // communicators aborted past it), never in an unbounded event sync
    int rc = b2p_group_wait(g, g->gnext - 8);
    if (rc != B2P_OK) return rc;
  }
  if (g->gstream.empty()) {
    g->gstream.assign(g->n, nullptr);
    for (int r = 0; r < g->n; ++r) {
      (void)hipSetDevice(g->dev[r]);
      if (hipStreamCreateWithFlags(&g->gstream[r], hipStreamNonBlocking) != hipSuccess)
        return gerr(g, B2P_EHIP, "hipStreamCreate", "");
    }
  }
  for (int r = 0; r < g->n; ++r) {
    hipEvent_t e = (hipEvent_t)b2p_internal_fence_event(g->ctx[r], tickets[r]);
    if (!e) return gerr(g, B2P_EINVAL, "b2p_group_gather_async", "a member's ticket is not one of its last 8");
    (void)hipSetDevice(g->dev[r]);
    // mode 1 copies on the root's group stream: it waits for every member
    if (hipStreamWaitEvent(g->gstream[g->mode == 0 ? r : 0], e, 0) != hipSuccess)
      return gerr(g, B2P_EHIP, "hipStreamWaitEvent", "");
  }
  const size_t count = (size_t)g->nout * nspec, bytes = count * sizeof(float);
  if (g->mode == 0) {
    ncclResult_t nr = ncclGroupStart();
    for (int r = 0; r < g->n && nr == ncclSuccess; ++r) {
      (void)hipSetDevice(g->dev[r]);
      nr = ncclGather(spectra[r], r == 0 ? root_out : nullptr, count, ncclFloat32, 0, g->comm[r],
                      g->gstream[r]);
    }
    ncclResult_t ne = ncclGroupEnd();
    if ((nr != ncclSuccess && nr != ncclInProgress) || (ne != ncclSuccess && ne != ncclInProgress))
      return gerr(g, B2P_EHIP, "ncclGather", ncclGetErrorString(nr != ncclSuccess ? nr : ne));
    int rc = settle_comms(g, now_s() + 1e-3 * g->timeout_ms, "ncclGather enqueue");
    if (rc != B2P_OK) return rc;
  } else {
    (void)hipSetDevice(g->dev[0]);
    for (int r = 0; r < g->n; ++r)
      if (hipMemcpyPeerAsync(root_out + (size_t)r * count, g->dev[0], spectra[r], g->dev[r], bytes,
                             g->gstream[0]) != hipSuccess)
        return gerr(g, B2P_EHIP, "hipMemcpyPeerAsync", "");
  }
  (void)hipSetDevice(g->dev[0]);
  if (host_out && hipMemcpyAsync(host_out, root_out, bytes * g->n, hipMemcpyDeviceToHost, g->gstream[0]) !=
                      hipSuccess)
    return gerr(g, B2P_EHIP, "hipMemcpyAsync", "");
  const int slot = (int)(g->gnext % 8);
  if (!g->gev[slot] && hipEventCreateWithFlags(&g->gev[slot], hipEventDisableTiming) != hipSuccess)
    return gerr(g, B2P_EHIP, "hipEventCreate", "");
  if (hipEventRecord(g->gev[slot], g->gstream[0]) != hipSuccess) return gerr(g, B2P_EHIP, "hipEventRecord", "");
  *gticket = g->gnext++;
  return B2P_OK;
}

// Has one b2p_group_gather_async finished?  1 / 0, no wait
int b2p_group_done(b2p_group_t *g, uint64_t gticket) {
  if (!g || gticket >= g->gnext) return B2P_EINVAL;
  if (g->dead) return gerr(g, B2P_ETIMEDOUT, "b2p_group_done", "group aborted earlier; close it");
  if (g->gnext - gticket > 8) return 1;
  (void)hipSetDevice(g->dev[0]);
  const hipError_t e = hipEventQuery(g->gev[gticket % 8]);
  if (e == hipErrorNotReady) return 0;
  if (e != hipSuccess) return gerr(g, B2P_EHIP, "b2p_group_done", hipGetErrorString(e));
  return 1;
}

// Wait for one b2p_group_gather_async (polled against the group's limit)
int b2p_group_wait(b2p_group_t *g, uint64_t gticket) {
  if (!g || gticket >= g->gnext) return B2P_EINVAL;
  if (g->dead) return gerr(g, B2P_ETIMEDOUT, "b2p_group_wait", "group aborted earlier; close it");
  if (g->gnext - gticket > 8) return B2P_OK;  // a later gather's event has been waited on since
  (void)hipSetDevice(g->dev[0]);
  const double deadline = now_s() + 1e-3 * g->timeout_ms;
  for (;;) {
    hipError_t e = hipEventQuery(g->gev[gticket % 8]);
    if (e == hipSuccess) return B2P_OK;
    if (e != hipErrorNotReady) {
      if (!g->comm.empty()) abort_comms(g);
      g->dead = 1;
      return gerr(g, B2P_EHIP, "b2p_group_wait", hipGetErrorString(e));
    }
    if (!g->comm.empty()) {
      ncclResult_t st = ncclSuccess;
      for (int r = 0; r < (int)g->comm.size() && st == ncclSuccess; ++r) {
        ncclResult_t q = ncclCommGetAsyncError(g->comm[r], &st);
        if (q != ncclSuccess) st = q;
        if (st == ncclInProgress) st = ncclSuccess;
      }
      if (st != ncclSuccess) {
        abort_comms(g);
        return gerr(g, B2P_EHIP, "b2p_group_wait", ncclGetErrorString(st));
      }
    }
    if (now_s() > deadline) {
      char d[96];
      snprintf(d, sizeof d, "gather not complete after %d ms; communicators aborted", g->timeout_ms);
      if (!g->comm.empty()) abort_comms(g);
      g->dead = 1;
      return gerr(g, B2P_ETIMEDOUT, "b2p_group_wait", d);
    }
    usleep(20);
  }
}

int b2p_group_reduce(b2p_group_t *g, uint64_t *const *sums, uint64_t count, uint64_t *root_sum) {
  if (!g || !sums || !root_sum || !count) return B2P_EINVAL;
  if (g->dead) return gerr(g, B2P_ETIMEDOUT, "b2p_group_reduce", "group aborted earlier; close it");
  for (int r = 0; r < g->n; ++r) {
    int rc = b2p_internal_flush(g->ctx[r]);
    if (rc != B2P_OK) return gerr(g, rc, "flush", b2p_last_error(g->ctx[r]));
  }
  if (g->mode == 0) {  // exact: integer sums, any order
    ncclResult_t nr = ncclGroupStart();
    for (int r = 0; r < g->n && nr == ncclSuccess; ++r) {
      (void)hipSetDevice(g->dev[r]);
      nr = ncclReduce(sums[r], r == 0 ? root_sum : nullptr, count, ncclUint64, ncclSum, 0, g->comm[r],
                      g->stream[r]);
    }
    ncclResult_t ne = ncclGroupEnd();
    if ((nr != ncclSuccess && nr != ncclInProgress) || (ne != ncclSuccess && ne != ncclInProgress))
      return gerr(g, B2P_EHIP, "ncclReduce", ncclGetErrorString(nr != ncclSuccess ? nr : ne));
    return settle_comms(g, now_s() + 1e-3 * g->timeout_ms, "ncclReduce enqueue");
  }
  // mode 1: rows copied to the root, summed there
  (void)hipSetDevice(g->dev[0]);
  if (g->scratch_count < count * (uint64_t)g->n) {
    if (g->scratch) (void)hipFree(g->scratch);
    g->scratch = nullptr;
    g->scratch_count = 0;
    if (hipMalloc(&g->scratch, count * (uint64_t)g->n * sizeof(unsigned long long)) != hipSuccess)
      return gerr(g, B2P_ENOMEM, "b2p_group_reduce", "hipMalloc");
    g->scratch_count = count * (uint64_t)g->n;
  }
  for (int r = 0; r < g->n; ++r) {
    (void)hipSetDevice(g->dev[r]);
    if (hipEventRecord(g->done[r], g->stream[r]) != hipSuccess)
      return gerr(g, B2P_EHIP, "hipEventRecord", "");
  }
  (void)hipSetDevice(g->dev[0]);
  const size_t bytes = count * sizeof(unsigned long long);
  for (int r = 0; r < g->n; ++r) {
    if (hipStreamWaitEvent(g->stream[0], g->done[r], 0) != hipSuccess ||
        hipMemcpyPeerAsync(g->scratch + (size_t)r * count, g->dev[0], sums[r], g->dev[r], bytes,
                           g->stream[0]) != hipSuccess)
      return gerr(g, B2P_EHIP, "hipMemcpyPeerAsync", "");
  }
  b2p::SumRowsArgs a;
  a.src = g->scratch;
  a.dst = (unsigned long long *)root_sum;
  a.count = count;
  a.nrows = (uint32_t)g->n;
  if (b2p::launch_sum_rows(a, g->stream[0]) != hipSuccess) return gerr(g, B2P_EHIP, "sum_rows", "");
  return B2P_OK;
}

int b2p_group_sync(b2p_group_t *g) {
  if (!g) return B2P_EINVAL;
  if (g->dead) return gerr(g, B2P_ETIMEDOUT, "b2p_group_sync", "group aborted earlier; close it");
  // enqueue every member's deferred finalize, then wait -- polled against
  // the group's deadline rather than hipStreamSynchronize, so a collective
  // that never completes is reported instead of hanging the caller
  for (int r = 0; r < g->n; ++r) {
    int rc = b2p_internal_flush(g->ctx[r]);
    if (rc != B2P_OK) return gerr(g, rc, "flush", b2p_last_error(g->ctx[r]));
  }
  return wait_streams(g, "b2p_group_sync");
}

const char *b2p_group_last_error(const b2p_group_t *g) { return g ? g->err : g_gerr; }

int b2p_group_close(b2p_group_t *g) {
  if (!g) return B2P_EINVAL;
  // non-blocking communicators: finalize (polled, bounded), then destroy;
  // past the limit they are aborted instead
  if (!g->dead && !g->comm.empty()) {
    for (auto c : g->comm)
      if (c) ncclCommFinalize(c);
    if (settle_comms(g, now_s() + 1e-3 * g->timeout_ms, "ncclCommFinalize") == B2P_OK)
      for (auto c : g->comm)
        if (c) ncclCommDestroy(c);
  }
  if (g->scratch) {
    (void)hipSetDevice(g->dev[0]);
    (void)hipFree(g->scratch);
  }
  for (size_t r = 0; r < g->done.size(); ++r)
    if (g->done[r]) {
      (void)hipSetDevice(g->dev[r]);
      (void)hipEventDestroy(g->done[r]);
    }
  for (size_t r = 0; r < g->gstream.size(); ++r)
    if (g->gstream[r]) {
      (void)hipSetDevice(g->dev[r]);
      (void)hipStreamSynchronize(g->gstream[r]);
      (void)hipStreamDestroy(g->gstream[r]);
    }
  (void)hipSetDevice(g->dev[0]);
  for (auto e : g->gev)
    if (e) (void)hipEventDestroy(e);
  delete g;
  return B2P_OK;
}

}  // extern "C"
