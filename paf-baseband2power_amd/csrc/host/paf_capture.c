/*
 * paf_capture -- receive BMF data frames over UDP into a GPU-resident ring
 * (the reference's paf_capture.c:46-189, capture.c,
 * sync.c).
 *
 * The reference runs one thread per port, copies each payload into the host
 * ring block at (idf*NCHK_NIC + chunk)*7168 (capture.c:536-541), parks
 * frames that belong to the next block in a temp buffer
 * (capture.c:464-531) and lets a spin loop switch blocks and advance the
 * reference header (sync.c:95-175).  Here one receive thread gathers frames
 * (recvmmsg over every port) and decodes each header on the host only to
 * sort it by time (capture.c:562-568 frame index): frames of the current
 * block go to a pinned batch, frames of later blocks to a spill buffer (the
 * temp buffer's role), frames of past blocks are dropped (capture.c:464-466).
 * The GPU places the payloads: each batch is uploaded once and scattered by
 * b2p_assemble into the current block of a dada_db -g ring.  When the block
 * switches, the spill is sorted again against the new reference.
 *
 *   paf_capture -a key -f header_file [-g epoch_file] [-i freq] [-c rbuf_ndf]
 *               [-j seconds | -n blocks] [-e nic | -I ip] [-P 17100] [-N 6]
 *               [-m ip | -m freq:F0] [-x ref_idf -s ref_sec] [-t idle_s] [-k dir] [-Z]
 *   paf_capture -o frames.df -O chunks.u8 ...      (no GPU: record what arrives)
 *
 * Address: -e NIC binds 10.17.<node>.<NIC>, <node> the 8th character of
 * the host name, as the reference derives it (paf_capture.c:88-90,115-118;
 * HN_LEN 8, paf_capture.h:5); -I gives the address directly (default any).
 *
 * Chunk of a frame: -m ip (default) derives it from the sender address as
 * acquire_ifreq does (capture.c:570-584); -m freq:F0 uses round(freq - F0)
 * from the frame header (test senders on one host).  The reference time is
 * the first frame received unless -x/-s give it.  A block is closed once a
 * frame arrives TBUF_NDF (256, capture.h:35) frames past its end, or when
 * the stream goes idle.
 *
 * Header: written when the first data frame arrives, as the reference does
 * (capture.c:300-312): the template (-f), then UTC_START and PICOSECONDS of
 * the first block's reference frame from the epoch file (-g; restated
 * acquire_start_time, capture.c:791-843, b2p_df_start_time) and FREQ from
 * -i (register_header, capture.c:727-789).  An epoch file that cannot be
 * read, or does not list the frames' epoch, stops the capture.
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include <arpa/inet.h>
#include <errno.h>
#include <getopt.h>
#include <inttypes.h>
#include <math.h>
#include <netinet/in.h>
#include <poll.h>
#include <pthread.h>
#include <signal.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "b2p.h"
#include "b2p_dada.h"
#include "b2p_df.h"

/* the GPU holding ring db's blocks, -1 for a host ring */
static int ring_device_of(ipcbuf_t *db) {
#if defined(B2P_TEST_HOST_RING_AS_DEVICE)
  /* test build only (tests/test_frames_stub.py): a host ring takes the
   * GPU-resident path, driven by the CPU test double tests/c/b2p_cpu_stub.c,
   * so this host runs under ThreadSanitizer on a machine with no GPU */
  (void)db;
  return 0;
#else
  return ipcbuf_get_device(db);
#endif
}

#define MAXPORT 16
#define RECV_BATCH 64
#define TBUF_NDF 256 /* capture.h:35 */
#define RX_SLOTS 32  /* batches in flight per receive thread */

/* SIGINT / SIGTERM: stop receiving, deliver the block being filled and end
 * the ring's transfer cleanly (the reference's capture stopped on a quit
 * flag polled without atomics, capture.c:32-39, 443-446) */
static atomic_int g_stop; /* lock-free: set by the signal handler, read by every thread */
static void on_stop(int sig) {
  (void)sig;
  g_stop = 1;
}

/* the reference's NIC address: 10.17.<node>.<nic>, node = the host name's
 * character HN_LEN - 1 (paf_capture.c:115-118; HN_LEN 8, paf_capture.h:5) */
static int nic_address(int nic, char *ip, size_t len) {
  char hn[256] = "";
  if (gethostname(hn, sizeof hn - 1) < 0 || strlen(hn) < 8 || hn[7] < '0' || hn[7] > '9') {
    fprintf(stderr, "paf_capture: -e %d: host name '%s' has no node digit at its 8th character "
                    "(the reference's 10.17.<node>.<nic> rule); give the address with -I\n", nic, hn);
    return -1;
  }
  snprintf(ip, len, "10.17.%d.%d", hn[7] - '0', nic);
  return 0;
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

typedef struct cap_t {
  /* ring / GPU */
  dada_hdu_t *hdu;
  b2p_ctx_t *ctx;
  char *blk;
  uint64_t bufsz, block_ndf, nblk_done, nblk_max;
  int nchunk, nozero;
  void *d_frames, *d_chunks; /* the uploaded batch */
  unsigned long long *d_cnt;
  uint64_t placed_all, dropped_late, dropped_spill, dropped_far;
  uint64_t far_run; /* consecutive frames at or past far_rel */
  int64_t far_rel;  /* block_ndf + max(block_ndf, 2 x TBUF_NDF) */
  /* host: frames of the current block, and of later ones */
  unsigned char *hf, *hc, *sf, *sc;
  uint64_t hn, cap_frames, sn, spill_cap;
  /* time */
  b2p_df_hdr_t ref; /* reference of the current block */
  int have_ref;
  int64_t max_rel;  /* furthest frame seen, relative to ref */
  multilog_t *log;
  /* ring header, written at the first data frame (capture.c:300-312) */
  const char *hfile, *efile;
  double freq;
  int have_freq, hdr_done;
} cap_t;

/* template + UTC_START / PICOSECONDS of the start frame + FREQ
 * (register_header, capture.c:727-789; acquire_start_time, :791-843) */
static int write_header(cap_t *c, const b2p_df_hdr_t *start) {
  char utc[64] = "";
  uint64_t ps = 0;
  if (c->efile) {
    double days = 0;
    const int e = b2p_df_epoch_days(c->efile, start->epoch, &days);
    if (e == -1) {
      multilog(c->log, LOG_ERR, "cannot open epoch file %s (capture.c:798-805)", c->efile);
      return -1;
    }
    if (e == -2) {
      multilog(c->log, LOG_ERR, "epoch %d is not in epoch file %s", start->epoch, c->efile);
      return -1;
    }
    if (b2p_df_start_time(start, days, utc, sizeof utc, &ps) != 0) {
      multilog(c->log, LOG_ERR, "start time of idf %" PRIu64 " sec %" PRIu64 " does not convert",
               start->idf, start->sec);
      return -1;
    }
    multilog(c->log, LOG_INFO, "SEC_START %" PRIu64 ", IDF_START %" PRIu64 ", epoch %d: UTC_START %s, "
             "PICOSECONDS %" PRIu64, start->sec, start->idf, start->epoch, utc, ps);
  } else {
    multilog(c->log, LOG_WARNING, "no epoch file (-g): UTC_START and PICOSECONDS stay as in %s",
             c->hfile);
  }
  char *hb = ipcbuf_get_next_write(c->hdu->header_block);
  if (!hb || fileread(c->hfile, hb, DADA_DEFAULT_HEADER_SIZE) < 0) {
    multilog(c->log, LOG_ERR, "cannot pass header %s", c->hfile);
    return -1;
  }
  if ((c->efile && (ascii_header_set(hb, "UTC_START", "%s", utc) < 0 ||
                    ascii_header_set(hb, "PICOSECONDS", "%" PRIu64, ps) < 0)) ||
      (c->have_freq && ascii_header_set(hb, "FREQ", "%.1lf", c->freq) < 0)) {
    multilog(c->log, LOG_ERR, "cannot set UTC_START / PICOSECONDS / FREQ in the header");
    return -1;
  }
  if (ipcbuf_mark_filled(c->hdu->header_block, DADA_DEFAULT_HEADER_SIZE) < 0) {
    multilog(c->log, LOG_ERR, "cannot mark the header block filled");
    return -1;
  }
  c->hdr_done = 1;
  return 0;
}

/* ---- receive threads ---------------------------------------------------
 * One per port by default (the reference's capture threads, capture.c:
 * 405-560): each drains its ports with recvmmsg into a ring of batch slots
 * (single producer, single consumer) and never touches the ring block; the
 * main thread takes the batches in order, sorts every frame by time and
 * files it (so block switching stays on one thread, the role of sync.c's
 * loop).  A full slot ring makes the thread wait: frames queue in the
 * socket's 256 MiB receive buffer meanwhile. */
typedef struct rx_slot {
  int n;                         /* frames in the batch                    */
  uint32_t len[RECV_BATCH];      /* datagram length (0: truncated)         */
  uint32_t addr[RECV_BATCH];     /* sender, sin_addr.s_addr                */
  int port[RECV_BATCH];          /* port index the frame arrived on        */
  unsigned char *buf;            /* RECV_BATCH x 7232 B                    */
} rx_slot_t;

typedef struct rxq {
  pthread_t th;
  int started, joined, nport;
  int port[MAXPORT], sock[MAXPORT];
  rx_slot_t slot[RX_SLOTS];
  _Atomic uint64_t head, tail; /* head: slots filled; tail: slots consumed */
  atomic_int *stop;
} rxq_t;

typedef struct port_stat {
  uint64_t frames;
  uint64_t chunks[4]; /* chunk bytes seen on the port (bitmask) */
} port_stat_t;

static atomic_int rx_stop;

static void *rx_main(void *arg) {
  rxq_t *q = (rxq_t *)arg;
  struct pollfd pfd[MAXPORT];
  for (int i = 0; i < q->nport; i++) pfd[i] = (struct pollfd){q->sock[i], POLLIN, 0};
  while (!atomic_load(q->stop)) {
    const uint64_t head = atomic_load_explicit(&q->head, memory_order_relaxed);
    if (head - atomic_load_explicit(&q->tail, memory_order_acquire) >= RX_SLOTS) {
      usleep(20); /* the sorter is behind: the socket buffers hold the stream */
      continue;
    }
    if (poll(pfd, (nfds_t)q->nport, 20) <= 0) continue;
    for (int i = 0; i < q->nport; i++) {
      if (!(pfd[i].revents & POLLIN)) continue;
      const uint64_t h = atomic_load_explicit(&q->head, memory_order_relaxed);
      if (h - atomic_load_explicit(&q->tail, memory_order_acquire) >= RX_SLOTS) break;
      rx_slot_t *sl = &q->slot[h % RX_SLOTS];
      struct mmsghdr msg[RECV_BATCH];
      struct iovec iov[RECV_BATCH];
      struct sockaddr_in from[RECV_BATCH];
      for (unsigned k = 0; k < RECV_BATCH; k++) {
        iov[k].iov_base = sl->buf + (size_t)k * B2P_DF_BYTES;
        iov[k].iov_len = B2P_DF_BYTES;
        memset(&msg[k], 0, sizeof msg[k]);
        msg[k].msg_hdr.msg_iov = &iov[k];
        msg[k].msg_hdr.msg_iovlen = 1;
        msg[k].msg_hdr.msg_name = &from[k];
        msg[k].msg_hdr.msg_namelen = sizeof from[k];
      }
      const int r = recvmmsg(q->sock[i], msg, RECV_BATCH, MSG_DONTWAIT, NULL);
      if (r <= 0) continue;
      for (int k = 0; k < r; k++) {
        sl->len[k] = (msg[k].msg_hdr.msg_flags & MSG_TRUNC) ? 0 : msg[k].msg_len;
        sl->addr[k] = (uint32_t)from[k].sin_addr.s_addr;
        sl->port[k] = q->port[i];
      }
      sl->n = r;
      atomic_store_explicit(&q->head, h + 1, memory_order_release);
    }
  }
  return NULL;
}

/* stop every receive thread and join it (idempotent) */
static void stop_rx(rxq_t *q, int n) {
  atomic_store(&rx_stop, 1);
  for (int t = 0; t < n; t++)
    if (q[t].started && !q[t].joined) {
      pthread_join(q[t].th, NULL);
      q[t].joined = 1;
    }
}

/* upload the batch and scatter it into the current block */
static int flush_batch(cap_t *c) {
  if (!c->hn) return 0;
  if (b2p_memcpy(c->ctx, c->d_frames, c->hf, c->hn * B2P_DF_BYTES, 1) != B2P_OK ||
      b2p_memcpy(c->ctx, c->d_chunks, c->hc, c->hn, 1) != B2P_OK) {
    multilog(c->log, LOG_ERR, "block %" PRIu64 ": uploading %" PRIu64 " frames: %s", c->nblk_done, c->hn,
             b2p_last_error(c->ctx));
    return -1;
  }
  const int rc = b2p_assemble(c->ctx, c->d_frames, c->hn, B2P_DF_BYTES, c->d_chunks, c->ref.idf,
                              c->ref.sec, c->blk, c->block_ndf, (uint32_t)c->nchunk, c->d_cnt);
  c->hn = 0;
  if (rc != B2P_OK)
    multilog(c->log, LOG_ERR, "block %" PRIu64 ": assemble: %s", c->nblk_done, b2p_last_error(c->ctx));
  return rc == B2P_OK ? 0 : -1;
}

/* file one received frame by its index relative to the current block */
static int file_frame(cap_t *c, const unsigned char *df, unsigned char chunk, int64_t rel) {
  if (rel < 0) {
    c->dropped_late++; /* behind the block (capture.c:464-466) */
  } else if (rel < (int64_t)c->block_ndf || !c->spill_cap) {
    if (c->hn == c->cap_frames && flush_batch(c) < 0) return -1; /* a full batch goes first */
    memcpy(c->hf + c->hn * B2P_DF_BYTES, df, B2P_DF_BYTES);
    c->hc[c->hn++] = chunk;
  } else if (c->sn < c->spill_cap) {
    memcpy(c->sf + c->sn * B2P_DF_BYTES, df, B2P_DF_BYTES);
    c->sc[c->sn++] = chunk;
  } else {
    c->dropped_spill++; /* too far ahead: the reference forces a switch first */
  }
  return 0;
}

static int open_block(cap_t *c) {
  uint64_t bid;
  c->blk = ipcio_open_block_write(c->hdu->data_block, &bid);
  if (!c->blk) {
    multilog(c->log, LOG_ERR, "block %" PRIu64 ": no block to write in the ring", c->nblk_done);
    return -1;
  }
  /* a failure from here on leaves the open block unfilled: the end of the
   * transfer (dada_hdu_unlock_write) marks it as the 0-byte end-of-data
   * block, so no reader integrates a half-assembled block */
  if ((!c->nozero && b2p_memset(c->ctx, c->blk, 0, c->bufsz) != B2P_OK) ||
      b2p_memset(c->ctx, c->d_cnt, 0, (c->nchunk + 3) * sizeof(unsigned long long)) != B2P_OK) {
    multilog(c->log, LOG_ERR, "block %" PRIu64 ": clearing: %s", c->nblk_done, b2p_last_error(c->ctx));
    return -1;
  }
  /* the spill, sorted again against this block's reference */
  const uint64_t n = c->sn;
  c->sn = 0;
  c->max_rel = -1;
  for (uint64_t i = 0; i < n; i++) {
    const unsigned char *df = c->sf + i * B2P_DF_BYTES;
    b2p_df_hdr_t h;
    b2p_df_decode(df, &h);
    const int64_t rel = b2p_df_index(&h, &c->ref);
    if (rel > c->max_rel) c->max_rel = rel;
    if (rel >= (int64_t)c->block_ndf) { /* still ahead: compact in place */
      memmove(c->sf + c->sn * B2P_DF_BYTES, df, B2P_DF_BYTES);
      c->sc[c->sn++] = c->sc[i];
    } else if (file_frame(c, df, c->sc[i], rel) < 0) {
      return -1;
    }
  }
  return 0;
}

static int close_block(cap_t *c) {
  if (flush_batch(c) < 0) return -1;
  unsigned long long cnt[256 + 3];
  if (b2p_sync(c->ctx) != B2P_OK ||
      b2p_memcpy(c->ctx, cnt, c->d_cnt, (c->nchunk + 3) * sizeof(unsigned long long), 2) != B2P_OK) {
    multilog(c->log, LOG_ERR, "block %" PRIu64 ": assembly: %s", c->nblk_done, b2p_last_error(c->ctx));
    return -1;
  }
  uint64_t placed = 0;
  for (int i = 0; i < c->nchunk; i++) placed += cnt[i];
  const uint64_t expect = c->block_ndf * (uint64_t)c->nchunk;
  multilog(c->log, LOG_INFO, "block %" PRIu64 ": %" PRIu64 " of %" PRIu64 " frames (%.3f%% lost), %llu with a "
           "bad chunk", c->nblk_done, placed, expect, 100.0 * (double)(expect - placed) / (double)expect,
           cnt[c->nchunk + 2]);
  c->placed_all += placed;
  ipcio_close_block_write(c->hdu->data_block, c->bufsz);
  c->blk = NULL;
  c->nblk_done++;
  b2p_df_ref_advance(&c->ref, c->block_ndf); /* sync.c:119-125 */
  return 0;
}

int main(int argc, char **argv) {
  key_t key = 0;
  int have_key = 0, port0 = 17100, nport = 6, arg, nozero = 0;
  const char *hfile = NULL, *ip = "0.0.0.0", *mapping = "ip", *ofile = NULL, *ocfile = NULL,
             *logdir = NULL, *efile = NULL;
  uint64_t rbuf_ndf = 8192, nblocks = 0, ref_idf = 0, ref_sec = 0;
  int have_ref = 0, have_freq = 0, nrx_req = 0, sod = -1;
  double length = 0, idle_s = 2.0, freq = 0;
  int nic = -1;
  char nic_ip[32] = "";
  while ((arg = getopt(argc, argv, "a:b:c:d:e:f:g:i:j:k:I:P:N:R:m:x:s:n:t:o:O:Zh")) != -1) {
    switch (arg) {
      case 'a': have_key = sscanf(optarg, "%x", (unsigned *)&key) == 1; break;
      case 'b': /* start of data (paf_capture.c:75-77, capture.c:622-639) */
        if (sscanf(optarg, "%d", &sod) != 1) {
          fprintf(stderr, "paf_capture: -b takes 0 or 1, not %s\n", optarg);
          return EXIT_FAILURE;
        }
        break;
      case 'd': { /* record headers (paf_capture.c:83-85, capture.c:216,222) */
        int hdr = 0;
        if (sscanf(optarg, "%d", &hdr) != 1 || hdr != 0) {
          fprintf(stderr, "paf_capture: -d %s: only payload-only blocks (-d 0) are recorded; the "
                          "stage integrates TFTFP payload, not frames with their headers\n", optarg);
          return EXIT_FAILURE;
        }
        break;
      }
      case 'c': rbuf_ndf = strtoull(optarg, NULL, 10); break;
      case 'e': /* which NIC (paf_capture.c:88-90) */
        if (sscanf(optarg, "%d", &nic) != 1 || nic < 0 || nic > 255) {
          fprintf(stderr, "paf_capture: -e takes a NIC number 0..255, not %s\n", optarg);
          return EXIT_FAILURE;
        }
        break;
      case 'f': hfile = optarg; break;
      case 'g': efile = optarg; break;
      case 'i':
        if (sscanf(optarg, "%lf", &freq) != 1) {
          fprintf(stderr, "paf_capture: -i takes the centre frequency in MHz, not %s\n", optarg);
          return EXIT_FAILURE;
        }
        have_freq = 1;
        break;
      case 'j': length = atof(optarg); break;
      case 'k': logdir = optarg; break;
      case 'I': ip = optarg; break;
      case 'P': port0 = atoi(optarg); break;
      case 'N': nport = atoi(optarg); break;
      case 'R': nrx_req = atoi(optarg); break;
      case 'm': mapping = optarg; break;
      case 'x': ref_idf = strtoull(optarg, NULL, 10); have_ref = 1; break;
      case 's': ref_sec = strtoull(optarg, NULL, 10); have_ref = 1; break;
      case 'n': nblocks = strtoull(optarg, NULL, 10); break;
      case 't': idle_s = atof(optarg); break;
      case 'o': ofile = optarg; break;
      case 'O': ocfile = optarg; break;
      case 'Z': nozero = 1; break;
      default:
        fprintf(stdout,
                "paf_capture -a key -f header [-g epoch_file] [-i freq] [-b sod] [-d 0] [-c rbuf_ndf] [-j seconds | -n blocks]\n"
                "            [-e nic | -I ip] [-P port0] [-N nports] [-R rx_threads] [-m ip|freq:F0] [-x ref_idf -s ref_sec]\n"
                "            [-t idle_s] [-k dir] [-Z]\n"
                "paf_capture -o frames.df -O chunks.u8 [-I ip] [-P port0] [-N nports] [-m ...] [-t idle_s]\n");
        return EXIT_FAILURE;
    }
  }
  if (nic >= 0 && !strcmp(ip, "0.0.0.0")) { /* -I wins over -e */
    if (nic_address(nic, nic_ip, sizeof nic_ip) < 0) return EXIT_FAILURE;
    ip = nic_ip;
  }
  const int record = ofile != NULL;
  if ((!record && (!have_key || !hfile)) || (record && !ocfile) || nport < 1 || nport > MAXPORT ||
      nrx_req < 0) {
    fprintf(stderr, "paf_capture: -a and -f (or -o and -O) are required, 1 <= -N <= %d\n", MAXPORT);
    return EXIT_FAILURE;
  }
  double freq0 = 0;
  const int by_freq = !strncmp(mapping, "freq:", 5);
  if (by_freq) freq0 = atof(mapping + 5);
  else if (strcmp(mapping, "ip")) {
    fprintf(stderr, "paf_capture: -m ip or -m freq:F0\n");
    return EXIT_FAILURE;
  }
  if (!record) {
    /* the header goes out with the first data frame, whose start time it
     * carries (capture.c:300-312); the template and the epoch file are
     * checked now, so a bad one fails before any ring or frame is touched */
    FILE *th = fopen(hfile, "r");
    if (!th) {
      fprintf(stderr, "paf_capture: cannot open header template %s\n", hfile);
      return EXIT_FAILURE;
    }
    fclose(th);
    if (efile) {
      FILE *te = fopen(efile, "r");
      if (!te) {
        fprintf(stderr, "paf_capture: cannot open epoch file %s (capture.c:798-805)\n", efile);
        return EXIT_FAILURE;
      }
      fclose(te);
    }
  }

  cap_t c;
  memset(&c, 0, sizeof c);
  c.hfile = hfile;
  c.efile = efile;
  c.freq = freq;
  c.have_freq = have_freq;
  c.log = multilog_open("paf_capture", 0);
  {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sigemptyset(&sa.sa_mask);
    sa.sa_handler = on_stop;
    sigaction(SIGINT, &sa, NULL);
    sigaction(SIGTERM, &sa, NULL);
  }
  multilog_add(c.log, stderr);
  FILE *logf = NULL;
  if (logdir) {
    char p[4096];
    snprintf(p, sizeof p, "%s/paf_capture.log", logdir);
    if ((logf = fopen(p, "w"))) multilog_add(c.log, logf);
  }
  int status = EXIT_FAILURE, locked = 0;
  int socks[MAXPORT];
  for (int p = 0; p < nport; p++) socks[p] = -1;
  FILE *fo = NULL, *fco = NULL;
  port_stat_t pstat[MAXPORT];
  memset(pstat, 0, sizeof pstat);

  /* sockets: one per port (capture.c:146-176), large receive buffers */
  for (int p = 0; p < nport; p++) {
    socks[p] = socket(AF_INET, SOCK_DGRAM, 0);
    int rcv = 256 << 20;
    setsockopt(socks[p], SOL_SOCKET, SO_RCVBUF, &rcv, sizeof rcv);
    struct sockaddr_in sa;
    memset(&sa, 0, sizeof sa);
    sa.sin_family = AF_INET;
    sa.sin_port = htons((uint16_t)(port0 + p));
    if (inet_pton(AF_INET, ip, &sa.sin_addr) != 1 || bind(socks[p], (struct sockaddr *)&sa, sizeof sa) < 0) {
      multilog(c.log, LOG_ERR, "cannot bind %s:%d (%s)", ip, port0 + p, strerror(errno));
      goto done;
    }
  }

  if (record) {
    fo = fopen(ofile, "wb");
    fco = fopen(ocfile, "wb");
    if (!fo || !fco) {
      multilog(c.log, LOG_ERR, "cannot open %s / %s (%s)", ofile, ocfile, strerror(errno));
      goto done;
    }
  } else {
    c.hdu = dada_hdu_create(c.log);
    dada_hdu_set_key(c.hdu, key);
    if (dada_hdu_connect(c.hdu) < 0 || dada_hdu_lock_write(c.hdu) < 0) {
      multilog(c.log, LOG_ERR, "cannot attach/lock ring %x %s", (unsigned)key, dada_device_error());
      goto done;
    }
    locked = 1;
    ipcbuf_t *db = &c.hdu->data_block->buf;
    /* -b 1: the readers see data from the first block written (the
     * reference's enable_sod(db, 0, 0), which assumes a fresh ring, as
     * enable_sod at the ring's next block); -b 0: blocks are written with the
     * start of data disabled, invisible to readers (capture.c:633); no -b:
     * the start of data is the first block written (PSRDADA's default) */
    if ((sod == 1 && ipcbuf_enable_sod(db, ipcbuf_get_write_count(db), 0) < 0) ||
        (sod == 0 && ipcbuf_disable_sod(db) < 0)) {
      multilog(c.log, LOG_ERR, "Can not write data before start (capture.c:626)");
      goto done;
    }
    if (ring_device_of(db) < 0) {
      multilog(c.log, LOG_ERR, "ring %x is not GPU-resident (dada_db -g)", (unsigned)key);
      goto done;
    }
    c.bufsz = ipcbuf_get_bufsz(db);
    c.nchunk = (int)(c.bufsz / ((uint64_t)rbuf_ndf * B2P_DF_PAYLOAD_BYTES));
    if (!c.nchunk || c.nchunk > 255 || c.bufsz != rbuf_ndf * (uint64_t)c.nchunk * B2P_DF_PAYLOAD_BYTES) {
      multilog(c.log, LOG_ERR, "ring block %" PRIu64 " B is not %" PRIu64 " frames x chunks x 7168 B",
               c.bufsz, rbuf_ndf);
      goto done;
    }
    c.block_ndf = rbuf_ndf;
    c.far_rel = (int64_t)(rbuf_ndf + (rbuf_ndf > 2 * TBUF_NDF ? rbuf_ndf : 2 * TBUF_NDF));
    c.nozero = nozero;
    c.nblk_max = nblocks ? nblocks
                         : (length > 0 ? (uint64_t)ceil(length / (rbuf_ndf * B2P_DF_TSAMP_SEC)) : UINT64_MAX);
    b2p_geom_t g;
    b2p_geom_bmf(&g);
    g.nchunk = (uint32_t)c.nchunk;
    g.nsamp_int = rbuf_ndf * g.nsamp_df;
    if (b2p_open(&c.ctx, &g, ring_device_of(db)) != B2P_OK) {
      multilog(c.log, LOG_ERR, "b2p_open: %s", b2p_last_error(NULL));
      goto done;
    }
    if (b2p_dev_alloc(c.ctx, &c.d_frames, rbuf_ndf * c.nchunk * B2P_DF_BYTES) != B2P_OK ||
        b2p_dev_alloc(c.ctx, &c.d_chunks, rbuf_ndf * c.nchunk) != B2P_OK ||
        b2p_dev_alloc(c.ctx, (void **)&c.d_cnt, (c.nchunk + 3) * sizeof(unsigned long long)) != B2P_OK) {
      multilog(c.log, LOG_ERR, "device batch of %" PRIu64 " frames: %s", rbuf_ndf * c.nchunk,
               b2p_last_error(c.ctx));
      goto done;
    }
  }
  /* host batch: one block's worth of frames at most (GPU mode), pinned */
  c.cap_frames = record ? 4096 : rbuf_ndf * (uint64_t)c.nchunk;
  c.hf = malloc(c.cap_frames * B2P_DF_BYTES);
  c.hc = malloc(c.cap_frames);
  /* spill: frames up to the forced switch plus slack, for every chunk */
  c.spill_cap = record ? 0 : (uint64_t)(2 * TBUF_NDF) * (uint64_t)c.nchunk;
  c.sf = c.spill_cap ? malloc(c.spill_cap * B2P_DF_BYTES) : NULL;
  c.sc = c.spill_cap ? malloc(c.spill_cap) : NULL;
  if (!c.hf || !c.hc || (c.spill_cap && (!c.sf || !c.sc))) {
    multilog(c.log, LOG_ERR, "cannot allocate the host batch (%" PRIu64 " frames) and spill", c.cap_frames);
    goto done;
  }
  if (c.ctx) b2p_register_host(c.ctx, c.hf, c.cap_frames * B2P_DF_BYTES);
  if (have_ref) { /* the first block opens with the first frame, after the header */
    c.ref.idf = ref_idf;
    c.ref.sec = ref_sec;
    c.have_ref = 1;
  }

  {
    /* receive threads: port p is drained by thread p % nrx (the reference
     * runs one capture thread per port, capture.c:405-560); each hands
     * batches of raw frames to this thread, which sorts them by time */
    int nrx = nrx_req > 0 ? nrx_req : nport, rx_failed = 0, rx_ok = 0;
    if (nrx > nport) nrx = nport;
    rxq_t *rxq = calloc((size_t)nrx, sizeof *rxq);
    if (!rxq) {
      multilog(c.log, LOG_ERR, "cannot allocate %d receive queues", nrx);
      goto done;
    }
    int rx_started = 0;
    for (int t = 0; t < nrx; t++) {
      rxq[t].stop = &rx_stop;
      for (int p = t; p < nport; p += nrx) {
        rxq[t].port[rxq[t].nport] = p;
        rxq[t].sock[rxq[t].nport++] = socks[p];
      }
      for (int k = 0; k < RX_SLOTS && rxq[t].nport; k++)
        if (!(rxq[t].slot[k].buf = malloc((size_t)RECV_BATCH * B2P_DF_BYTES))) {
          multilog(c.log, LOG_ERR, "receive thread %d: cannot allocate its batch slots", t);
          goto rx_end;
        }
      if (pthread_create(&rxq[t].th, NULL, rx_main, &rxq[t]) != 0) {
        multilog(c.log, LOG_ERR, "cannot start receive thread %d", t);
        goto rx_end;
      }
      rxq[t].started = 1;
      rx_started++;
    }
    multilog(c.log, LOG_INFO, "%d receive thread(s) over %d port(s)", rx_started, nport);
    {
    uint64_t got_all = 0, bad = 0;
    double last_rx = now_s(), t_first = 0;
    const double start_s = idle_s * 5 > 30 ? idle_s * 5 : 30; /* first frame within */
    int stop = 0, jumped = 0, stopped = 0;
    while (!stop) {
      if (g_stop) {
        multilog(c.log, LOG_INFO, "stopped by a signal: delivering the current block");
        stopped = 1;
        break;
      }
      int any = 0;
      /* one batch per thread per round: the ports advance together in time,
       * so no port's frames fall behind a block another port has already
       * closed (a full slot ring is 256 frame times of one port) */
      for (int t = 0; t < nrx && !stop; t++) {
        rxq_t *q = &rxq[t];
        uint64_t tail = atomic_load_explicit(&q->tail, memory_order_relaxed);
        if (!stop && tail < atomic_load_explicit(&q->head, memory_order_acquire)) {
          rx_slot_t *sl = &q->slot[tail % RX_SLOTS];
          any = 1;
          for (int i = 0; i < sl->n; i++) {
            if (sl->len[i] != B2P_DF_BYTES) { /* not a data frame (short, long or truncated) */
              bad++;
              continue;
            }
            const unsigned char *df = sl->buf + (size_t)i * B2P_DF_BYTES;
            b2p_df_hdr_t h;
            b2p_df_decode(df, &h);
            int chunk = by_freq ? (int)lround(h.freq - freq0) : b2p_df_chunk_from_ip(sl->addr[i]);
            const unsigned char ck = (unsigned char)(chunk < 0 || chunk > 255 ? 255 : chunk);
            got_all++;
            port_stat_t *ps = &pstat[sl->port[i]];
            ps->frames++;
            ps->chunks[ck >> 6] |= 1ull << (ck & 63);
            if (record) {
              if (fwrite(df, B2P_DF_BYTES, 1, fo) != 1 || fwrite(&ck, 1, 1, fco) != 1) {
                multilog(c.log, LOG_ERR, "writing %s / %s failed (%s)", ofile, ocfile, strerror(errno));
                goto rx_fail;
              }
              continue;
            }
            if (t_first == 0) t_first = now_s();
            if (!c.hdr_done) { /* the first frame: reference, start time, header, block 0 */
              if (!c.have_ref) { /* the first frame fixes the reference (align_df role) */
                c.ref = h;
                c.have_ref = 1;
              }
              c.ref.epoch = h.epoch; /* -x/-s give idf and sec; the epoch is the stream's */
              multilog(c.log, LOG_INFO, "reference: idf %" PRIu64 ", sec %" PRIu64 ", epoch %d", c.ref.idf,
                       c.ref.sec, c.ref.epoch);
              if (write_header(&c, &c.ref) < 0 || open_block(&c) < 0) goto rx_fail;
            }
            const int64_t rel = b2p_df_index(&h, &c.ref);
            /* far ahead of the current block: the reference quits the
             * capture at two blocks ahead (capture.c:491-508); frames between
             * block_ndf + TBUF_NDF and there force a block switch (:510-524).
             * With blocks shorter than 2 x TBUF_NDF (tests) the far limit is
             * kept past the spill's reach, block_ndf + 2 x TBUF_NDF.  One far
             * frame (a corrupt timestamp) is dropped and must not drive block
             * switches; a run of them, more than one per chunk, means the
             * stream really jumped ahead, and the capture stops, as there */
            if (rel >= c.far_rel) {
              c.dropped_far++;
              if (++c.far_run > (uint64_t)c.nchunk) {
                multilog(c.log, LOG_ERR, "%" PRIu64 " consecutive frames %" PRId64 "+ frames ahead of "
                         "the current block: the stream jumped, stopping (capture.c:491-508)", c.far_run,
                         c.far_rel);
                stop = jumped = 1;
                break;
              }
              continue;
            }
            c.far_run = 0;
            if (rel > c.max_rel) c.max_rel = rel;
            if (file_frame(&c, df, ck, rel) < 0) goto rx_fail;
            /* forced switch as soon as a frame runs TBUF_NDF past the block
             * (capture.c:510-524), before the spill can overflow */
            while (c.blk && c.max_rel >= (int64_t)(c.block_ndf + TBUF_NDF)) {
              if (close_block(&c) < 0) goto rx_fail;
              if (c.nblk_done >= c.nblk_max) {
                stop = 1;
                break;
              }
              if (open_block(&c) < 0) goto rx_fail;
            }
            if (stop) break;
          }
          atomic_store_explicit(&q->tail, ++tail, memory_order_release);
        }
      }
      if (stop) break;
      const double t = now_s();
      if (any) last_rx = t;
      else usleep(100);
      if (record) {
        if (got_all && t - last_rx > idle_s) stop = 1;
        continue;
      }
      if (!got_all) { /* nothing yet: wait for the stream to start */
        if (t - last_rx > start_s) {
          multilog(c.log, LOG_ERR, "no data frame in %.1f s", start_s);
          goto rx_fail;
        }
        continue;
      }
      const int idle = t - last_rx > idle_s;
      if (c.hn == c.cap_frames || (c.hn && !any)) /* a full batch, or the sockets ran dry */
        if (flush_batch(&c) < 0) goto rx_fail;
      /* the block is over once frames run TBUF_NDF past its end (the
       * reference's forced switch, capture.c:510-524) or the stream stops */
      while (c.blk && (c.max_rel >= (int64_t)(c.block_ndf + TBUF_NDF) || idle)) {
        if (close_block(&c) < 0) goto rx_fail;
        if (c.nblk_done >= c.nblk_max || (idle && !c.sn)) {
          stop = 1;
          break;
        }
        if (open_block(&c) < 0) goto rx_fail;
        if (idle) { /* drain what the spill still holds, then stop */
          if (flush_batch(&c) < 0) goto rx_fail;
        }
      }
    }
    if (0) {
    rx_fail:
      rx_failed = 1;
    }
    stop_rx(rxq, nrx);
    if (rx_failed) goto rx_end;
    if ((jumped || stopped) && !record && c.blk && close_block(&c) < 0)
      goto rx_end; /* deliver what arrived */
    const double el = t_first > 0 ? last_rx - t_first : 0.0;
    multilog(c.log, LOG_INFO, "capture: %" PRIu64 " frames received (%" PRIu64 " not frames), %" PRIu64
             " blocks, %" PRIu64 " frames placed, %" PRIu64 " behind their block, %" PRIu64
             " past the spill, %" PRIu64 " far ahead, %.3f s from the first frame to the last", got_all,
             bad, c.nblk_done, c.placed_all, c.dropped_late, c.dropped_spill, c.dropped_far, record ? 0.0 : el);
    /* per-port table (capture.c:700-725): frames expected = chunks seen on
     * the port x frames per chunk over the blocks delivered */
    multilog(c.log, LOG_INFO, "port\tchunks\tframes\texpected\tloss");
    for (int p = 0; p < nport; p++) {
      int nck = 0;
      for (int w = 0; w < 4; w++) nck += __builtin_popcountll(pstat[p].chunks[w]);
      const uint64_t expect = record ? 0 : (uint64_t)nck * c.nblk_done * c.block_ndf;
      if (expect)
        multilog(c.log, LOG_INFO, "%d\t%d\t%" PRIu64 "\t%" PRIu64 "\t%.1E", port0 + p, nck, pstat[p].frames,
                 expect, (double)((int64_t)expect - (int64_t)pstat[p].frames) / (double)expect);
      else
        multilog(c.log, LOG_INFO, "%d\t%d\t%" PRIu64 "\t-\t-", port0 + p, nck, pstat[p].frames);
    }
    if (jumped) goto rx_end; /* EXIT_FAILURE: the stream left the capture window */
    rx_ok = 1;
    }
  rx_end:
    stop_rx(rxq, nrx);
    for (int t = 0; t < nrx; t++)
      for (int k = 0; k < RX_SLOTS; k++) free(rxq[t].slot[k].buf);
    free(rxq);
    if (!rx_ok) goto done;
  }
  status = EXIT_SUCCESS;

done:
  if (locked && !c.hdr_done) { /* no frame ever came: readers still get a header, then EOD */
    c.efile = NULL;
    write_header(&c, &c.ref);
  }
  /* the context first: closing it drains its stream, so no clear or
   * assembly a failure left in flight still writes into a ring block once
   * the ring is detached (its IPC mapping closed) */
  if (c.ctx) {
    if (c.d_frames) b2p_dev_free(c.ctx, c.d_frames);
    if (c.d_chunks) b2p_dev_free(c.ctx, c.d_chunks);
    if (c.d_cnt) b2p_dev_free(c.ctx, c.d_cnt);
    if (c.hf) b2p_unregister_host(c.ctx, c.hf);
    b2p_close(c.ctx);
  }
  if (locked) dada_hdu_unlock_write(c.hdu);
  if (c.hdu) dada_hdu_destroy(c.hdu);
  for (int p = 0; p < nport; p++)
    if (socks[p] >= 0) close(socks[p]);
  if (fo) fclose(fo);
  if (fco) fclose(fco);
  free(c.hf);
  free(c.hc);
  free(c.sf);
  free(c.sc);
  multilog_close(c.log);
  if (logf) fclose(logf);
  return status;
}
