/*
 * paf_dfsend -- replay a BMF data-frame stream over UDP: the sender side the
 * reference's capture receives from (capture.c:405-560, ports from
 * PORT_BASE 17100, capture.h:22-24).  A test source for paf_capture.
 *
 *   paf_dfsend -i frames.df -k chunks.u8 [-H 127.0.0.1] [-P 17100] [-N 6]
 *              [-r MB/s] [-l loops] [-T threads]
 * Frame i goes to port P + (chunk_i mod N) as one 7232-B datagram, in file
 * order; -r paces the stream (0: as fast as the socket takes it).  -T T
 * sends from T threads, thread t taking the ports p with p mod T == t (its
 * frames still in file order), each paced at rate / T: one sender thread
 * saturates near 5 GB/s on loopback, several NICs' worth needs more.
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include <arpa/inet.h>
#include <getopt.h>
#include <inttypes.h>
#include <netinet/in.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "b2p_df.h"

#define MAXPORT 16
#define BATCH 32

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

typedef struct sender {
  pthread_t th;
  int t, nthr, nport, loops, rc;
  double rate;              /* MB/s for this thread, 0: unpaced */
  const unsigned char *frames, *chunk;
  uint64_t n, sent;
  const struct sockaddr_in *dst;
} sender_t;

static void *send_main(void *arg) {
  sender_t *w = (sender_t *)arg;
  int sock = socket(AF_INET, SOCK_DGRAM, 0);
  int sndbuf = 64 << 20;
  setsockopt(sock, SOL_SOCKET, SO_SNDBUF, &sndbuf, sizeof sndbuf);
  const double t0 = now_s();
  for (int l = 0; l < w->loops && !w->rc; l++) {
    for (uint64_t i = 0; i < w->n;) {
      struct mmsghdr msg[BATCH];
      struct iovec iov[BATCH];
      int m = 0;
      for (; m < BATCH && i < w->n; i++) {
        const int port = w->chunk[i] % w->nport;
        if (port % w->nthr != w->t) continue; /* another thread's port */
        iov[m].iov_base = (void *)(w->frames + i * B2P_DF_BYTES);
        iov[m].iov_len = B2P_DF_BYTES;
        memset(&msg[m], 0, sizeof msg[m]);
        msg[m].msg_hdr.msg_iov = &iov[m];
        msg[m].msg_hdr.msg_iovlen = 1;
        msg[m].msg_hdr.msg_name = (void *)&w->dst[port];
        msg[m].msg_hdr.msg_namelen = sizeof(struct sockaddr_in);
        m++;
      }
      for (int off = 0; off < m;) {
        const int done = sendmmsg(sock, msg + off, (unsigned)(m - off), 0);
        if (done < 0) {
          perror("paf_dfsend: sendmmsg");
          w->rc = 1;
          break;
        }
        off += done;
      }
      if (w->rc) break;
      w->sent += (uint64_t)m;
      if (w->rate > 0) { /* pace: sent bytes may not run ahead of rate * elapsed */
        const double ahead = w->sent * (double)B2P_DF_BYTES / (w->rate * 1e6) - (now_s() - t0);
        if (ahead > 0) {
          struct timespec ts = {(time_t)ahead, (long)((ahead - (time_t)ahead) * 1e9)};
          nanosleep(&ts, NULL);
        }
      }
    }
  }
  close(sock);
  return NULL;
}

int main(int argc, char **argv) {
  const char *dfile = NULL, *cfile = NULL, *host = "127.0.0.1";
  int port0 = 17100, nport = 6, loops = 1, nthr = 1, arg;
  double rate = 0;
  while ((arg = getopt(argc, argv, "i:k:H:P:N:r:l:T:h")) != -1) {
    switch (arg) {
      case 'i': dfile = optarg; break;
      case 'k': cfile = optarg; break;
      case 'H': host = optarg; break;
      case 'P': port0 = atoi(optarg); break;
      case 'N': nport = atoi(optarg); break;
      case 'r': rate = atof(optarg); break;
      case 'l': loops = atoi(optarg); break;
      case 'T': nthr = atoi(optarg); break;
      default:
        fprintf(stdout, "paf_dfsend -i frames.df -k chunks.u8 [-H host] [-P port0] [-N nports] "
                        "[-r MB/s] [-l loops] [-T threads]\n");
        return EXIT_FAILURE;
    }
  }
  if (nthr > nport) nthr = nport;
  if (!dfile || !cfile || nport < 1 || nport > MAXPORT || nthr < 1) {
    fprintf(stderr, "paf_dfsend: -i and -k are required, 1 <= -N <= %d\n", MAXPORT);
    return EXIT_FAILURE;
  }
  FILE *fd = fopen(dfile, "rb"), *fc = fopen(cfile, "rb");
  if (!fd || !fc) {
    perror("paf_dfsend: open");
    return EXIT_FAILURE;
  }
  fseek(fd, 0, SEEK_END);
  const long long fsz = ftell(fd);
  fseek(fd, 0, SEEK_SET);
  const uint64_t n = (uint64_t)fsz / B2P_DF_BYTES;
  unsigned char *frames = malloc(n * B2P_DF_BYTES + 1), *chunk = malloc(n + 1);
  if (!frames || !chunk || fread(frames, B2P_DF_BYTES, n, fd) != n || fread(chunk, 1, n, fc) != n) {
    fprintf(stderr, "paf_dfsend: cannot read %" PRIu64 " frames and chunk ids\n", n);
    return EXIT_FAILURE;
  }
  fclose(fd);
  fclose(fc);
  struct sockaddr_in dst[MAXPORT];
  for (int p = 0; p < nport; p++) {
    memset(&dst[p], 0, sizeof dst[p]);
    dst[p].sin_family = AF_INET;
    dst[p].sin_port = htons((uint16_t)(port0 + p));
    if (inet_pton(AF_INET, host, &dst[p].sin_addr) != 1) {
      fprintf(stderr, "paf_dfsend: bad host %s\n", host);
      return EXIT_FAILURE;
    }
  }
  const double t0 = now_s();
  uint64_t sent = 0;
  sender_t w[MAXPORT];
  int rc = 0;
  for (int t = 0; t < nthr; t++) {
    w[t] = (sender_t){0};
    w[t].t = t;
    w[t].nthr = nthr;
    w[t].nport = nport;
    w[t].loops = loops;
    w[t].rate = rate / nthr;
    w[t].frames = frames;
    w[t].chunk = chunk;
    w[t].n = n;
    w[t].dst = dst;
    if (pthread_create(&w[t].th, NULL, send_main, &w[t]) != 0) {
      fprintf(stderr, "paf_dfsend: cannot start sender thread %d\n", t);
      return EXIT_FAILURE;
    }
  }
  for (int t = 0; t < nthr; t++) {
    pthread_join(w[t].th, NULL);
    sent += w[t].sent;
    rc |= w[t].rc;
  }
  if (rc) return EXIT_FAILURE;
  const double el = now_s() - t0;
  fprintf(stderr, "paf_dfsend: %" PRIu64 " frames in %.3f s (%.1f MB/s)\n", sent, el,
          el > 0 ? sent * (double)B2P_DF_BYTES / el / 1e6 : 0.0);
  free(frames);
  free(chunk);
  return EXIT_SUCCESS;
}
