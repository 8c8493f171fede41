// tests/c/group_rccl_stub.cpp -- TEST DOUBLE + driver, CPU only.
//
// csrc/b2p_group.hip (the multi-GPU gather / reduce behind include/b2p.h) has
// run with one RCCL member on the test box's single GPU; more than one RCCL
// rank cannot run there.  This file links b2p_group.hip's object against
// stand-ins for every RCCL and HIP runtime function it calls, plus fake
// member contexts, and checks the argument plumbing of n = 8 members:
//   - member r initialises communicator rank r of n, on member r's device,
//     non-blocking, all inside one ncclGroupStart/End, with one unique id;
//   - ncclGroupEnd / ncclCommGetAsyncError answering ncclInProgress is polled
//     to completion, not treated as a failure; an asynchronous error aborts
//     every communicator (B2P_EHIP); one that never settles times out
//     (B2P_ETIMEDOUT, communicators aborted) within the group's limit;
//   - gathers: member r sends on its own (or the group's own) stream from its
//     own device; only rank 0 passes root_out; root_out is member-major
//     (r * nspec * nout), for b2p_group_gather, _gather_n and _gather_async;
//   - gather_async waits on each member's fence event; its 9th gather reuses
//     the oldest event slot and that wait is bounded (B2P_ETIMEDOUT, aborted)
//     instead of blocking forever (round-3 ADVICE);
//   - ncclReduce(ncclUint64, ncclSum) of the time-split partials to rank 0.
// Exit 0 and "group stub: all checks passed" on success.
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <vector>

#include "b2p.h"

static int g_fail = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
      g_fail++;                                                    \
    }                                                              \
  } while (0)

// ---- fake member contexts (b2p_get_info and the library-internal hooks) ----
struct b2p_ctx {
  int device;
  uint32_t nout;
  hipStream_t stream;
  hipEvent_t fence[16];
};
struct ihipStream_t {
  int id;
  int device;
};
struct ihipEvent_t {
  int id;
  int not_ready;  // hipEventQuery answers hipErrorNotReady while > 0 (-1: forever)
};

extern "C" int b2p_get_info(const b2p_ctx_t *ctx, b2p_info_t *info) {
  memset(info, 0, sizeof *info);
  info->nout = ctx->nout;
  info->device = (uint32_t)ctx->device;
  return B2P_OK;
}
extern "C" const char *b2p_last_error(const b2p_ctx_t *) { return "stub"; }
void *b2p_internal_stream(struct b2p_ctx *ctx) { return ctx->stream; }
int b2p_internal_flush(struct b2p_ctx *) { return B2P_OK; }
void *b2p_internal_fence_event(struct b2p_ctx *ctx, uint64_t ticket) { return ticket < 16 ? ctx->fence[ticket] : nullptr; }
namespace b2p {
struct SumRowsArgs {
  const unsigned long long *src;
  unsigned long long *dst;
  uint64_t count;
  uint32_t nrows;
};
hipError_t launch_sum_rows(const SumRowsArgs &a, hipStream_t) {
  for (uint64_t i = 0; i < a.count; i++) {
    unsigned long long t = 0;
    for (uint32_t r = 0; r < a.nrows; r++) t += a.src[(uint64_t)r * a.count + i];
    a.dst[i] = t;
  }
  return hipSuccess;
}
}  // namespace b2p

// ---- HIP runtime stand-ins: host memory, every copy done at once ----------
static int g_dev = -1;  // hipSetDevice
static std::vector<ihipStream_t *> g_streams;
static std::vector<ihipEvent_t *> g_events;
struct Wait {
  hipStream_t s;
  hipEvent_t e;
  int dev;
};
static std::vector<Wait> g_waits;

extern "C" {
hipError_t hipSetDevice(int d) {
  g_dev = d;
  return hipSuccess;
}
const char *hipGetErrorString(hipError_t) { return "stub hip error"; }
hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned int) {
  *s = new ihipStream_t{(int)g_streams.size() + 100, g_dev};
  g_streams.push_back(*s);
  return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t) { return hipSuccess; }
hipError_t hipStreamQuery(hipStream_t) { return hipSuccess; }
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned int) {
  g_waits.push_back({s, e, g_dev});
  return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned) {
  *e = new ihipEvent_t{(int)g_events.size(), 0};
  g_events.push_back(*e);
  return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t) { return hipSuccess; }
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
hipError_t hipEventSynchronize(hipEvent_t) {  // an unbounded wait: never used by the group
  fprintf(stderr, "hipEventSynchronize called (unbounded wait)\n");
  g_fail++;
  return hipSuccess;
}
hipError_t hipEventQuery(hipEvent_t e) {
  if (e->not_ready < 0) return hipErrorNotReady;
  if (e->not_ready > 0) {
    e->not_ready--;
    return hipErrorNotReady;
  }
  return hipSuccess;
}
hipError_t hipMalloc(void **p, size_t n) {
  *p = malloc(n ? n : 1);
  return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void *p) {
  free(p);
  return hipSuccess;
}
hipError_t hipMemcpyAsync(void *dst, const void *src, size_t n, hipMemcpyKind, hipStream_t) {
  memcpy(dst, src, n);
  return hipSuccess;
}
hipError_t hipMemcpyPeerAsync(void *dst, int, const void *src, int, size_t n, hipStream_t) {
  memcpy(dst, src, n);
  return hipSuccess;
}
}

// ---- RCCL stand-ins ---------------------------------------------------------
struct ncclComm {
  int rank, nranks, dev;
  int polls;      // ncclCommGetAsyncError answers ncclInProgress this many more times (-1: forever)
  int aborted, destroyed, finalized;
  ncclResult_t async_err;
};
static std::vector<ncclComm *> g_comms;
static int g_in_group = 0, g_group_calls = 0, g_init_in_group = 0, g_end_in_progress = 1;
static char g_id[128];
static int g_init_polls = 3, g_init_err_rank = -1;
struct Coll {  // one ncclGather / ncclReduce call, executed at ncclGroupEnd
  int reduce;
  const void *send;
  void *recv;
  size_t count;
  int rank, dev, root;
  ncclDataType_t type;
  hipStream_t stream;
};
static std::vector<Coll> g_pending, g_log;

extern "C" {
const char *ncclGetErrorString(ncclResult_t) { return "stub nccl error"; }
ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
  for (int i = 0; i < 128; i++) g_id[i] = (char)(i * 7 + 1);
  memcpy(id->internal, g_id, sizeof g_id);
  return ncclSuccess;
}
ncclResult_t ncclGroupStart() {
  g_in_group++;
  return ncclSuccess;
}
ncclResult_t ncclGroupEnd() {
  g_in_group--;
  g_group_calls++;
  for (const Coll &c : g_pending) {  // the collective's data movement, on host memory
    void *rbuf = nullptr;
    for (const Coll &d : g_pending)
      if (d.rank == c.root) rbuf = d.recv;
    if (!rbuf) continue;
    const size_t esz = c.type == ncclUint64 ? 8 : 4;
    if (!c.reduce) {
      memcpy((char *)rbuf + (size_t)c.rank * c.count * esz, c.send, c.count * esz);
    } else if (c.rank == c.root) {
      for (size_t i = 0; i < c.count; i++) {
        uint64_t t = 0;
        for (const Coll &d : g_pending) t += ((const uint64_t *)d.send)[i];
        ((uint64_t *)rbuf)[i] = t;
      }
    }
  }
  g_pending.clear();
  if (g_end_in_progress) return ncclInProgress;  // non-blocking communicators: polled later
  return ncclSuccess;
}
ncclResult_t ncclCommInitRankConfig(ncclComm_t *comm, int nranks, ncclUniqueId id, int rank, ncclConfig_t *cfg) {
  CHECK(g_in_group == 1);
  CHECK(cfg && cfg->blocking == 0);
  CHECK(memcmp(id.internal, g_id, sizeof g_id) == 0);
  if (g_in_group == 1) g_init_in_group++;
  ncclComm *c = new ncclComm{rank, nranks, g_dev, g_init_polls, 0, 0, 0,
                             rank == g_init_err_rank ? ncclSystemError : ncclSuccess};
  g_comms.push_back(c);
  *comm = c;
  return ncclInProgress;
}
ncclResult_t ncclCommGetAsyncError(ncclComm_t c, ncclResult_t *err) {
  if (c->polls != 0) {
    if (c->polls > 0) c->polls--;
    *err = ncclInProgress;
    return ncclSuccess;
  }
  *err = c->async_err;
  return ncclSuccess;
}
ncclResult_t ncclCommAbort(ncclComm_t c) {
  c->aborted = 1;
  return ncclSuccess;
}
ncclResult_t ncclCommFinalize(ncclComm_t c) {
  c->finalized = 1;
  return ncclSuccess;
}
ncclResult_t ncclCommDestroy(ncclComm_t c) {
  c->destroyed = 1;
  return ncclSuccess;
}
ncclResult_t ncclGather(const void *send, void *recv, size_t count, ncclDataType_t type, int root, ncclComm_t comm,
                        hipStream_t stream) {
  CHECK(g_in_group == 1);
  Coll c{0, send, recv, count, comm->rank, g_dev, root, type, stream};
  g_pending.push_back(c);
  g_log.push_back(c);
  return ncclSuccess;
}
ncclResult_t ncclReduce(const void *send, void *recv, size_t count, ncclDataType_t type, ncclRedOp_t op, int root,
                        ncclComm_t comm, hipStream_t stream) {
  CHECK(g_in_group == 1);
  CHECK(op == ncclSum && type == ncclUint64);
  Coll c{1, send, recv, count, comm->rank, g_dev, root, type, stream};
  g_pending.push_back(c);
  g_log.push_back(c);
  return ncclSuccess;
}
}

// ---- the checks ---------------------------------------------------------------
static const int N = 8;
static const int kDev[N] = {3, 0, 5, 1, 7, 2, 6, 4};  // member r on device kDev[r]
static const uint32_t NOUT = 16;

static double now_s() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

static void make_members(b2p_ctx *m, b2p_ctx_t **ptrs) {
  for (int r = 0; r < N; r++) {
    m[r].device = kDev[r];
    m[r].nout = NOUT;
    m[r].stream = new ihipStream_t{r, kDev[r]};
    for (int t = 0; t < 16; t++) m[r].fence[t] = new ihipEvent_t{1000 + r * 16 + t, 0};
    ptrs[r] = &m[r];
  }
}

static void reset_stub() {
  g_comms.clear();
  g_log.clear();
  g_pending.clear();
  g_waits.clear();
  g_init_in_group = 0;
}

int main() {
  b2p_ctx members[N];
  b2p_ctx_t *ctx[N];
  make_members(members, ctx);

  // 1. set-up: rank order = member order, devices, non-blocking, one group, polled
  reset_stub();
  g_init_polls = 3;
  b2p_group_t *grp = nullptr;
  int rc = b2p_group_open_timed(&grp, ctx, N, 0, 5000);
  CHECK(rc == B2P_OK);
  CHECK((int)g_comms.size() == N && g_init_in_group == N);
  for (int r = 0; r < (int)g_comms.size(); r++) {
    CHECK(g_comms[r]->rank == r && g_comms[r]->nranks == N && g_comms[r]->dev == kDev[r]);
    CHECK(g_comms[r]->polls == 0 && !g_comms[r]->aborted);  // every in-progress answer was polled through
  }

  // 2. gather of one spectrum per member: member-major at the root
  std::vector<std::vector<float>> spec(N, std::vector<float>(NOUT * 8));
  for (int r = 0; r < N; r++)
    for (uint32_t i = 0; i < NOUT * 8; i++) spec[r][i] = (float)(r * 1000 + i);
  float *sp[N];
  for (int r = 0; r < N; r++) sp[r] = spec[r].data();
  std::vector<float> root(N * NOUT * 8, -1.f);
  g_log.clear();
  CHECK(b2p_group_gather(grp, sp, root.data()) == B2P_OK);
  CHECK((int)g_log.size() == N);
  for (int r = 0; r < (int)g_log.size(); r++) {
    const Coll &c = g_log[r];
    CHECK(!c.reduce && c.rank == r && c.root == 0 && c.count == NOUT && c.type == ncclFloat32);
    CHECK(c.dev == kDev[r] && c.stream == members[r].stream && c.send == sp[r]);
    CHECK(r == 0 ? c.recv == root.data() : c.recv == nullptr);
  }
  for (int r = 0; r < N; r++)
    for (uint32_t i = 0; i < NOUT; i++) CHECK(root[r * NOUT + i] == spec[r][i]);

  // 3. gather_n: nspec spectra per member, member-major (r * nspec * nout)
  const uint32_t nspec = 3;
  std::fill(root.begin(), root.end(), -1.f);
  g_log.clear();
  CHECK(b2p_group_gather_n(grp, sp, nspec, root.data()) == B2P_OK);
  for (const Coll &c : g_log) CHECK(c.count == (size_t)nspec * NOUT);
  for (int r = 0; r < N; r++)
    for (uint32_t i = 0; i < nspec * NOUT; i++) CHECK(root[(size_t)r * nspec * NOUT + i] == spec[r][i]);

  // 4. gather_async: behind each member's fence event, on the group's own
  //    streams, host copy of the whole root_out, tickets in order
  uint64_t tickets[N], gt = 0;
  std::vector<float> host(N * NOUT * 8);
  for (int k = 0; k < 8; k++) {
    for (int r = 0; r < N; r++) tickets[r] = (uint64_t)k;
    g_waits.clear();
    g_log.clear();
    std::fill(root.begin(), root.end(), -1.f);
    CHECK(b2p_group_gather_async(grp, sp, 2, root.data(), tickets, host.data(), &gt) == B2P_OK);
    CHECK(gt == (uint64_t)k);
    CHECK((int)g_waits.size() == N);
    for (int r = 0; r < (int)g_waits.size(); r++) {
      CHECK(g_waits[r].e == members[r].fence[k] && g_waits[r].dev == kDev[r]);
      CHECK(g_waits[r].s != members[r].stream && g_waits[r].s->device == kDev[r]);  // the group's stream
    }
    for (int r = 0; r < (int)g_log.size(); r++) CHECK(g_log[r].stream == g_waits[r].s && g_log[r].dev == kDev[r]);
    for (int r = 0; r < N; r++)
      for (uint32_t i = 0; i < 2 * NOUT; i++) {
        CHECK(root[(size_t)r * 2 * NOUT + i] == spec[r][i]);
        CHECK(host[(size_t)r * 2 * NOUT + i] == spec[r][i]);
      }
    CHECK(b2p_group_done(grp, gt) == 1 && b2p_group_wait(grp, gt) == B2P_OK);
  }

  // 5. time-split reduce: exact uint64 sums at rank 0
  std::vector<std::vector<uint64_t>> part(N, std::vector<uint64_t>(NOUT));
  uint64_t *pp[N];
  for (int r = 0; r < N; r++) {
    for (uint32_t i = 0; i < NOUT; i++) part[r][i] = (1ull << 50) + (uint64_t)r * 977 + i;
    pp[r] = part[r].data();
  }
  std::vector<uint64_t> tot(NOUT, 0);
  g_log.clear();
  CHECK(b2p_group_reduce(grp, pp, NOUT, tot.data()) == B2P_OK);
  for (int r = 0; r < (int)g_log.size(); r++) CHECK(g_log[r].reduce && (r == 0 ? g_log[r].recv == tot.data() : !g_log[r].recv));
  for (uint32_t i = 0; i < NOUT; i++) CHECK(tot[i] == 8 * (1ull << 50) + 977ull * 28 + 8 * i);

  // 6. the 9th gather_async reuses gather 1's event slot: if that gather
  //    never finishes, the call must end at the group's limit, aborted
  CHECK(b2p_group_close(grp) == B2P_OK);
  reset_stub();
  g_init_polls = 0;
  CHECK(b2p_group_open_timed(&grp, ctx, N, 0, 300) == B2P_OK);
  for (int k = 0; k < 8; k++) {
    for (int r = 0; r < N; r++) tickets[r] = (uint64_t)k;
    CHECK(b2p_group_gather_async(grp, sp, 1, root.data(), tickets, nullptr, &gt) == B2P_OK);
  }
  for (ihipEvent_t *e : g_events) e->not_ready = -1;  // nothing completes any more
  CHECK(b2p_group_done(grp, 0) == 0);
  for (int r = 0; r < N; r++) tickets[r] = 8;
  double t0 = now_s();
  rc = b2p_group_gather_async(grp, sp, 1, root.data(), tickets, nullptr, &gt);
  double dt = now_s() - t0;
  CHECK(rc == B2P_ETIMEDOUT);
  CHECK(dt >= 0.25 && dt < 5.0);
  for (ncclComm *c : g_comms) CHECK(c->aborted);
  CHECK(strstr(b2p_group_last_error(grp), "gather not complete") != nullptr);
  CHECK(b2p_group_gather(grp, sp, root.data()) == B2P_ETIMEDOUT);  // the group only closes now
  CHECK(b2p_group_close(grp) == B2P_OK);
  for (ihipEvent_t *e : g_events) e->not_ready = 0;

  // 7. an asynchronous error during set-up: every communicator aborted, EHIP
  reset_stub();
  g_init_polls = 2;
  g_init_err_rank = 5;
  grp = nullptr;
  CHECK(b2p_group_open_timed(&grp, ctx, N, 0, 5000) == B2P_EHIP && grp == nullptr);
  for (ncclComm *c : g_comms) CHECK(c->aborted);
  CHECK(strstr(b2p_group_last_error(nullptr), "member 5") != nullptr);
  g_init_err_rank = -1;

  // 8. a set-up that never settles: B2P_ETIMEDOUT at the limit, aborted
  reset_stub();
  g_init_polls = -1;
  t0 = now_s();
  CHECK(b2p_group_open_timed(&grp, ctx, N, 0, 200) == B2P_ETIMEDOUT && grp == nullptr);
  dt = now_s() - t0;
  CHECK(dt >= 0.2 && dt < 5.0);
  for (ncclComm *c : g_comms) CHECK(c->aborted);
  CHECK(strstr(b2p_group_last_error(nullptr), "not complete") != nullptr);

  // 9. a blocking-style ncclGroupEnd (ncclSuccess) works the same
  reset_stub();
  g_init_polls = 0;
  g_end_in_progress = 0;
  CHECK(b2p_group_open_timed(&grp, ctx, N, 0, 5000) == B2P_OK);
  CHECK(b2p_group_gather(grp, sp, root.data()) == B2P_OK);
  CHECK(b2p_group_close(grp) == B2P_OK);
  for (ncclComm *c : g_comms) CHECK(c->finalized && c->destroyed && !c->aborted);

  if (g_fail) {
    fprintf(stderr, "group stub: %d check(s) failed\n", g_fail);
    return 1;
  }
  printf("group stub: all checks passed (n = %d, %d group calls)\n", N, g_group_calls);
  return 0;
}
