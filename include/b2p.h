/*
 * include/b2p.h -- C ABI of the MI355X baseband->power integrator.
 *
 * This is the drop-in boundary for the reference's hot path.  The reference
 * (xinpingdeng/paf-baseband2power) declares the path but leaves it empty:
 *   - paf_baseband2power.cu:32-93  main(): CLI, log, cudaGetDeviceCount, exit
 *   - baseband2power.cuh:18-23     conf_t {device_id, dir, key_in, key_out}
 *   - baseband2power.cu:1-16       host driver (includes only)
 *   - kernel.cu:1-7, kernel.cuh    GPU kernel module (includes only)
 *   - cudautil.cuh:10-66           CudaSafeCall -> exit(-1) error convention
 *   - cudautil.cuh:118-125         BSWAP_64 unpack primitive
 * Every entry point below names the reference item it replaces.  The C host
 * (paf-baseband2power_amd/csrc/host/paf_baseband2power.c) calls only this
 * header; hipcc-built code lives behind it (libpafb2p.so).
 *
 * Conventions: plain C types only, no exceptions, never exit(); every call
 * returns B2P_OK (0) or a negative B2P_E* code (b2p_strerror()).  The caller
 * owns every buffer.  A context is not thread-safe; use one per device /
 * sub-band (contexts are independent).
 */
#ifndef B2P_H
#define B2P_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define B2P_ABI_VERSION 2

/* status codes (replace CudaSafeCall's exit(-1), cudautil.cuh:29-41) */
#define B2P_OK 0
#define B2P_EINVAL (-1)       /* bad argument or unsupported geometry          */
#define B2P_ERAGGED (-2)      /* nbytes is not a whole number of frames        */
#define B2P_EOVERFLOW (-3)    /* push would exceed nsamp_int of the integration */
#define B2P_EPARTIAL (-4)     /* finish with != nsamp_int samples (output written) */
#define B2P_ENODEV (-5)       /* no HIP device / device index out of range     */
#define B2P_EHIP (-6)         /* HIP runtime error; text in b2p_last_error()    */
#define B2P_ENOMEM (-7)       /* device or host allocation failed              */
#define B2P_EALIGN (-8)       /* buffer not 16-byte aligned                    */
#define B2P_EFAILED (-9)      /* an earlier call failed after part of its work
                                 was enqueued, so the running sums are unknown;
                                 every later call that enqueues work or emits a
                                 result (push, integrate, finish*, sync, fence*,
                                 finalize_sums, assemble, set_stream,
                                 set_timing) returns this until b2p_close;
                                 cleanup (dev_free, unregister_host, close) and
                                 b2p_last_error (the first failure) still work */
#define B2P_ETIMEDOUT (-10)   /* a group's communicator setup or collective did
                                 not complete within the group's time limit;
                                 the communicators were aborted and the group
                                 only accepts b2p_group_close from then on */

/*
 * Layout of one input ring block:
 *   [frame][chunk nchunk][samp nsamp_df][chan nchan_chunk][pol npol][dim ndim]
 * This is the TFTFP order of capture.c:540 ("cbuf_loc = (idf*NCHK_NIC +
 * ifreq)*pkt_size"), payload only (capture.c:222).  Global channel =
 * chunk*nchan_chunk + chan.  BMF-native: nbit 16, big_endian 1, nchunk 48,
 * nsamp_df 128, nchan_chunk 7 (capture.h:20,28; paf-baseband2power.conf:2-5).
 * The 256/1024-channel int8 configs use nchunk 1, nsamp_df 1.
 *
 * Supported: nbit 8 (big_endian 0) or 16; npol 2; ndim 2; npol_out 1 or 2;
 * chunk bytes (nsamp_df*nchan_chunk*word) a multiple of 16;
 * nchan*npol_out <= 8192; nsamp_int a multiple of nsamp_df.
 *
 * Word decode (16-bit BE, cudautil.cuh:118-125): lane k = bits [16k,16k+16)
 * of BSWAP_64(word); lane0 X.re, lane1 X.im, lane2 Y.re, lane3 Y.im.
 * Otherwise components are stored X.re, X.im, Y.re, Y.im.
 *
 * Output (header_baseband2power.txt:39-42, paf-baseband2power.py:77-79):
 * one fp32 per channel (npol_out 1: |X|^2+|Y|^2), or per channel and pol
 * ([chan][pol], npol_out 2).  Value = RNE_fp32(exact integer sum), or
 * RNE_fp32((double)sum / nsamp_int) with mean = 1 ("average", :20).
 */
typedef struct b2p_geom {
  uint32_t nbit;
  uint32_t big_endian;
  uint32_t nchunk;
  uint32_t nsamp_df;
  uint32_t nchan_chunk;
  uint32_t npol;
  uint32_t ndim;
  uint32_t npol_out;
  uint64_t nsamp_int;   /* samples per integration, README.md:2 -> 1024*1024 */
  uint32_t mean;
  uint32_t reserved;    /* must be 0 */
} b2p_geom_t;

/* Launch/geometry facts of an open context. */
typedef struct b2p_info {
  uint32_t nchan;        /* nchunk*nchan_chunk                     */
  uint32_t nout;         /* nchan*npol_out fp32 outputs             */
  uint64_t frame_bytes;  /* push granule                            */
  uint64_t block_bytes;  /* one integration = nsamp_int samples     */
  uint32_t threads;      /* active threads per workgroup            */
  uint32_t columns;      /* workgroups across one row               */
  uint32_t row_groups;   /* workgroups along time                   */
  uint32_t row_vectors;  /* 16-B vectors per row                    */
  uint32_t replicas;     /* accumulator replicas                    */
  uint32_t device;
  uint32_t unroll;       /* rows in flight per lane                 */
  uint32_t nontemporal;  /* 1 if the stream uses nt loads           */
} b2p_info_t;

/* Kernel timing collected with HIP events on the context's stream. */
typedef struct b2p_stats {
  uint64_t launches;      /* integrate-kernel launches timed        */
  uint64_t bytes;         /* algorithmic bytes read by them         */
  double kernel_ms;       /* summed kernel time (ms)                */
  double finalize_ms;     /* summed finalize-kernel time (ms)       */
  uint64_t finalizes;
} b2p_stats_t;

typedef struct b2p_ctx b2p_ctx_t;

/* ---- geometry helpers (no device needed) ---- */
/* BMF-native defaults: 48 chunks x 7 chans int16 BE, 1<<20 samples.
 * Replaces the constants of capture.h:20,28 and paf-baseband2power.conf. */
int b2p_geom_bmf(b2p_geom_t *g);
/* 0 if supported, else B2P_EINVAL */
int b2p_geom_check(const b2p_geom_t *g);
uint64_t b2p_frame_bytes(const b2p_geom_t *g);
uint64_t b2p_block_bytes(const b2p_geom_t *g);
const char *b2p_strerror(int code);
int b2p_abi_version(void);

/* ---- devices (paf_baseband2power.cu:86-90) ---- */
int b2p_device_count(int *count);

/* PCI bus id of a device ("0000:75:00.0"), for logs and multi-GPU run
 * records: which physical GPU a member or rank actually used. */
int b2p_device_pci_bus_id(int device, char *buf, int len);

/* ---- launch tuning (tools/tune.py) ----
 * The release defaults are the measured ones and no
 * environment variable changes them; a tuning sweep passes its variant
 * explicitly.  Every field at 0 / -1 (b2p_tuning_init) means "default".
 * Unsupported values are refused with B2P_EINVAL, not clamped. */
typedef struct b2p_tuning {
  uint32_t size;          /* sizeof(b2p_tuning_t)                           */
  int32_t max_threads;    /* 0, or 64..1024: cap on threads per workgroup   */
  int32_t threads;        /* 0, or a whole-wave divisor of the frame's 16-B
                             vectors (frame-split layouts only)             */
  int32_t wg_per_cu;      /* 0, or 1..32 workgroups per CU                  */
  int32_t row_groups;     /* 0, or >= 1 workgroups along time               */
  int32_t replicas;       /* 0, or 1..1024 accumulator replicas             */
  int32_t unroll;         /* 0, or 4 | 8 | 16 rows in flight per lane       */
  int32_t nontemporal;    /* -1, or 0 | 1: non-temporal loads               */
  int32_t interleave;     /* -1, or 0 | 1: interleaved row ownership        */
  int32_t fuse;           /* -1, or 0 | 1: b2p_integrate finalizes in its
                             own last workgroup                             */
  int32_t stage_mib;      /* 0, or 1..16384: host-span staging buffer size  */
  int32_t assemble_grid;  /* 0, or >= 1: b2p_assemble workgroup cap         */
} b2p_tuning_t;
void b2p_tuning_init(b2p_tuning_t *t);

/* ---- context lifecycle ----
 * b2p_open replaces the intended init of baseband2power.cu (empty) and the
 * device selection at paf_baseband2power.cu:87-90: device < 0 is an error;
 * if exactly one device is visible, index 0 is used whatever was asked (the
 * reference's docker fallback). */
int b2p_open(b2p_ctx_t **ctx, const b2p_geom_t *g, int device);
/* b2p_open with an explicit launch variant (t may be NULL = defaults) */
int b2p_open_tuned(b2p_ctx_t **ctx, const b2p_geom_t *g, int device, const b2p_tuning_t *t);
int b2p_close(b2p_ctx_t *ctx);
int b2p_get_info(const b2p_ctx_t *ctx, b2p_info_t *info);
const char *b2p_last_error(const b2p_ctx_t *ctx); /* ctx may be NULL */
/* Run on the caller's HIP stream (e.g. a framework's current stream);
 * NULL restores the context's own stream. */
int b2p_set_stream(b2p_ctx_t *ctx, void *hip_stream);

/* ---- host memory (role of PSRDADA dada_cuda_dbregister; dada_cuda.h is
 * included at baseband2power.cuh:9) ----
 * Lifetime rules (a copy that reads or writes host memory its owner has
 * released is a GPU page fault that kills the process's HIP context):
 *  - register: B2P_EINVAL if the range shares a (4 KiB) page with a range
 *    still registered through any context of the process (pinning is per
 *    page);
 *  - the memory must stay allocated while registered;
 *  - unregister: first drains the context's streams (a b2p_finish_async into
 *    the range may still be landing); work the caller enqueued elsewhere on
 *    the range must be complete; any context may release a range; a base
 *    that is not registered is B2P_EINVAL;
 *  - b2p_close releases every range its context registered and the caller
 *    left registered. */
int b2p_register_host(b2p_ctx_t *ctx, void *base, size_t bytes);
int b2p_unregister_host(b2p_ctx_t *ctx, void *base);

/* ---- the hot path (the intended body of kernel.cu) ----
 * Accumulate nbytes (a whole number of frames) of baseband into the
 * context's running integration: unpack -> |X|^2+|Y|^2 -> exact time sum.
 * is_device = 1: buf is device memory (16-B aligned), the kernel reads it in
 *   place; returns once enqueued.
 * is_device = 0: buf is host memory (register it for full PCIe rate); it is
 *   copied in frame-aligned chunks on a copy stream overlapped with the
 *   kernel, and b2p_push returns once every byte has been copied, so the
 *   caller may release / close the DADA block.  If a host-span push fails
 *   after its first chunk was enqueued, the context is marked failed
 *   (B2P_EFAILED from then on, see above); its copies from buf are drained
 *   before it returns, so buf may be released on every return. */
int b2p_push(b2p_ctx_t *ctx, const void *buf, size_t nbytes, int is_device);
/* Emit the integration: out[nout] (host memory), blocking.  Returns B2P_OK
 * if exactly nsamp_int samples were pushed, B2P_EPARTIAL otherwise (the
 * output is still written).  Resets the integration. */
int b2p_finish(b2p_ctx_t *ctx, float *out);
/* Same, enqueued: out is device memory (out_is_device = 1) or pinned host
 * memory; valid after b2p_sync(). */
int b2p_finish_async(b2p_ctx_t *ctx, float *out, int out_is_device);
/* As b2p_finish_async, but emits the integration's exact uint64 sums
 * (nout values) instead of fp32: the partial of one member of a time-split
 * integration (b2p_group_reduce), or for callers that reduce sums
 * themselves.  Replaces the finalize of the reference's unwritten
 * kernel.cu:1-7 for that mode. */
int b2p_finish_partial_async(b2p_ctx_t *ctx, uint64_t *sums, int sums_is_device);
/* fp32 from reduced exact sums: nspec x nout uint64 on this context's device
 * -> out (device), one RNE rounding each; with mean set, divided by
 * nsamp_total (0: this context's nsamp_int).  Stream-ordered. */
int b2p_finalize_sums(b2p_ctx_t *ctx, const uint64_t *sums, uint64_t nspec, uint64_t nsamp_total,
                      float *out);
/* Host fences on the context's stream, for consumers that keep several ring
 * blocks in flight: b2p_fence returns a ticket covering everything enqueued
 * so far (a deferred finalize stays deferred); b2p_fence_wait blocks until
 * that work has finished.  The last 8 tickets wait precisely; an older one
 * waits for the whole stream. */
int b2p_fence(b2p_ctx_t *ctx, uint64_t *ticket);
int b2p_fence_wait(b2p_ctx_t *ctx, uint64_t ticket);
/* 1 once the work behind `ticket` has finished, 0 while it runs (no wait) */
int b2p_fence_done(b2p_ctx_t *ctx, uint64_t ticket);
/* Enqueue a deferred finalize now (b2p_finish_async / b2p_integrate leave
 * it to ride the next launch) without waiting: for a consumer that has no
 * next block yet and wants the spectrum out as soon as its kernel ends. */
int b2p_flush(b2p_ctx_t *ctx);
int b2p_sync(b2p_ctx_t *ctx);
/* One whole integration in one call: push exactly block_bytes and emit it,
 * enqueued (out valid after b2p_sync()).  For a device span this is ONE
 * kernel launch -- the last workgroup to finish writes the spectrum -- so
 * no separate finalize launch; a host span falls back to b2p_push +
 * b2p_finish_async.  Requires no pending push.  Same output bits as the
 * push/finish pair. */
int b2p_integrate(b2p_ctx_t *ctx, const void *buf, size_t nbytes, int is_device, float *out,
                  int out_is_device);
/* Several whole integrations in ONE kernel launch: bufs[b] (device, 16-B
 * aligned, block_bytes each; b < nblk <= B2P_MAX_BLOCKS) is integration b,
 * its spectrum out + b * nout (device, or host memory valid after
 * b2p_sync()).  For a consumer that finds several ring blocks queued: the
 * launch's fixed cost (dispatch ramp and tail, ~2 us) is paid once, not
 * nblk times, which matters for short integrations (a 256 MiB block reads in
 * ~40 us).  Same output bits as nblk b2p_integrate calls; the finalize is
 * deferred as for b2p_finish_async.  Requires no pending push.  Every
 * layout runs in one launch (frame-split TFTFP 8x8: 6.8 -> 7.2 TB/s at 8
 * per launch; BMF equal). */
#define B2P_MAX_BLOCKS 8
/* How many queued blocks a consumer should hand one b2p_integrate_n: enough
 * that a launch reads at least B2P_BATCH_BYTES (4 GiB), so its fixed ramp
 * and tail (~2-3 us) cost under 0.5 %; 1..B2P_MAX_BLOCKS.  Measured on
 * MI355X: 1 GiB blocks 0.890 -> 0.900 of 8 TB/s at 4 per launch, 4 GiB
 * blocks gain nothing. */
#define B2P_BATCH_BYTES (4ull << 30)
uint32_t b2p_blocks_per_launch(uint64_t block_bytes);
int b2p_integrate_n(b2p_ctx_t *ctx, const void *const *bufs, uint32_t nblk, float *out,
                    int out_is_device);
/* Number of samples pushed into the current integration. */
uint64_t b2p_samples_pending(const b2p_ctx_t *ctx);

/* ---- multi-GPU gather ----
 * N contexts in one process, one per GPU / sub-band (one host thread, one
 * stream, one ring each).  Sub-bands never exchange data while they
 * integrate; b2p_group_gather collects each member's finished spectrum
 * (nout fp32 in that member's device memory) into root_out (n*nout fp32,
 * sub-band-major, device memory of ctxs[0]) with RCCL over xGMI:
 * ncclCommInitAll + ncclGather (rccl.h:236,745), enqueued on every member's
 * stream behind its finalize; valid on ctxs[0] after b2p_group_sync().
 * mode 0 = RCCL; mode 1 = peer copies (test rigs where members share a
 * device, which RCCL refuses).  All members need the same nout.  A member's
 * spectra / sums buffer must not be rewritten before b2p_group_sync()
 * (mode 1 copies it on ctxs[0]'s stream).  A member context in the failed
 * state makes the collective return B2P_EFAILED. */
typedef struct b2p_group b2p_group_t;
int b2p_group_open(b2p_group_t **grp, b2p_ctx_t *const *ctxs, int n, int mode);
/* b2p_group_open with a time limit (ms, > 0) on the RCCL communicator setup
 * and on every b2p_group_sync: setup runs non-blocking
 * (ncclCommInitRankConfig with blocking = 0, rccl.h:204) and is polled;
 * past the limit, or on an asynchronous RCCL error, the communicators are
 * aborted (ncclCommAbort, rccl.h:271) and the call returns B2P_ETIMEDOUT /
 * B2P_EHIP instead of hanging.  b2p_group_open uses 60 000 ms. */
int b2p_group_open_timed(b2p_group_t **grp, b2p_ctx_t *const *ctxs, int n, int mode, int timeout_ms);
int b2p_group_gather(b2p_group_t *grp, float *const *spectra, float *root_out);
/* nspec consecutive spectra per member (e.g. one b2p_integrate_n batch) in
 * one collective; root_out is member-major: member r's nspec x nout floats
 * at r * nspec * nout.  b2p_group_gather is nspec = 1. */
int b2p_group_gather_n(b2p_group_t *grp, float *const *spectra, uint32_t nspec, float *root_out);
/* The same gather for consumers that keep launches in flight: member r's
 * spectra are read once its fence ticket tickets[r] has passed (b2p_fence
 * after the launch that finalizes them -- with b2p_integrate[_n] that is
 * the NEXT launch, or b2p_sync), on streams of the group's own, so neither
 * the members' streams nor their pending finalizes are touched.  host_out
 * (pinned, optional) receives root_out (nspec x nout x members floats)
 * behind the gather.  *gticket is for b2p_group_wait; up to 8 gathers may be
 * outstanding (a 9th first waits for the oldest, bounded like b2p_group_wait:
 * B2P_ETIMEDOUT past the group's limit).  Call from one thread; the members' threads may keep
 * launching meanwhile. */
int b2p_group_gather_async(b2p_group_t *grp, float *const *spectra, uint32_t nspec, float *root_out,
                           const uint64_t *tickets, float *host_out, uint64_t *gticket);
int b2p_group_wait(b2p_group_t *grp, uint64_t gticket); /* bounded by the group's time limit */
int b2p_group_done(b2p_group_t *grp, uint64_t gticket); /* 1 once finished, 0 while running */
/* Time-split mode (second mode): member r integrated its share
 * of ONE sub-band's samples and emitted exact sums with
 * b2p_finish_partial_async; sums[r] holds `count` uint64 on member r's
 * device.  root_sum (member 0's device) receives their total: RCCL
 * ncclReduce(ncclUint64, ncclSum) in mode 0, peer copies + a sum kernel in
 * mode 1.  Exact, so bit-identical to a single-GPU integration. */
int b2p_group_reduce(b2p_group_t *grp, uint64_t *const *sums, uint64_t count, uint64_t *root_sum);
/* Waits for every member's stream, bounded by the group's time limit
 * (B2P_ETIMEDOUT past it; the group is then unusable). */
int b2p_group_sync(b2p_group_t *grp);
const char *b2p_group_last_error(const b2p_group_t *grp); /* grp may be NULL */
int b2p_group_close(b2p_group_t *grp);

/* ---- measurement ----
 * mode 1: every integrate / finalize launch carries start/stop events on
 *   its own dispatch packet (hipExtLaunchKernel) -> exact per-launch times;
 *   the event plumbing costs a few us between launches.
 * mode 2: one event pair on the context's stream brackets every launch
 *   between set_timing(ctx, 2) and set_timing(ctx, 0); kernel_ms is the
 *   region's elapsed time (inter-launch gaps and finalizes included), i.e.
 *   an upper bound of the summed launch durations, with no per-launch cost.
 *   The opening event goes on the stream with the region's first piece of
 *   work (integrate or assembly launch, staging copy, memset or finalize), so the caller's own time
 *   between set_timing(ctx, 2) and that call is not counted.
 * mode 0: off.  Closing a mode-2 region records its end event and returns
 *   without waiting; b2p_get_stats waits for it and adds the region. */
int b2p_set_timing(b2p_ctx_t *ctx, int mode);
int b2p_get_stats(b2p_ctx_t *ctx, b2p_stats_t *stats); /* synchronises */
int b2p_reset_stats(b2p_ctx_t *ctx);

/* ---- synthetic baseband + device buffers (bench / tests) ----
 * Same generator as oracle/b2p_oracle.c:orc_fill_synthetic, bit for bit. */
int b2p_fill_synthetic(b2p_ctx_t *ctx, void *dev, size_t nbytes, uint64_t seed,
                       uint32_t subband, uint64_t block, uint64_t elem0);
int b2p_dev_alloc(b2p_ctx_t *ctx, void **dev, size_t bytes);

/* ---- TFTFP assembly on the GPU (capture.c:527-547; include/b2p_df.h) ----
 * Scatter a stream of ndf raw 7232-B data frames (64-B header + 7168-B
 * payload, as received; device memory) into a payload-only TFTFP block of
 * block_ndf x nchunk x 7168 B (device memory) at
 * (idf_rel * nchunk + chunk) * 7168, idf_rel computed from each header
 * relative to the reference frame (ref_idf, ref_sec) exactly as
 * capture.c:566 does, chunk = chunk_of_df[i] (device, capture.c:571-584).
 * Frames outside [0, block_ndf) or with chunk >= nchunk are not placed;
 * nchunk is 1..255, so a chunk byte of 255 always means "no chunk".
 * counts (device, nchunk + 3 uint64, accumulated): frames placed per
 * chunk, then frames before the block, after it, with a bad chunk.  Slots
 * no frame reaches keep their previous bytes (as in the capture ring).
 * Enqueued on the context's stream, so a b2p_push of the block is ordered
 * after it. */
int b2p_assemble(b2p_ctx_t *ctx, const void *dfs, uint64_t ndf, uint32_t df_bytes,
                 const uint8_t *chunk_of_df, uint64_t ref_idf, uint64_t ref_sec, void *block,
                 uint64_t block_ndf, uint32_t nchunk, unsigned long long *counts);
int b2p_dev_free(b2p_ctx_t *ctx, void *dev);
/* kind: 1 host->device, 2 device->host, 3 device->device; synchronous */
int b2p_memcpy(b2p_ctx_t *ctx, void *dst, const void *src, size_t bytes, int kind);
/* fill device memory with a byte, ordered on the context's stream behind
 * earlier work (clears a ring block before frames are assembled into it,
 * so lost frames read as zeros rather than stale data) */
int b2p_memset(b2p_ctx_t *ctx, void *dev, int value, size_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* B2P_H */
