/*
 * ascii_header.c -- DADA "KEY value  # comment" headers (4096 B,
 * header_baseband2power.txt:1-45), get/set as used at capture.c:758-778.
 * A key matches only at the start of a line and only as a whole word.
 */
#include <fcntl.h>
#include <inttypes.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "b2p_dada.h"

/* start of the line holding `keyword` as its first word, or NULL */
static const char *find_key(const char *header, const char *keyword) {
  const size_t kl = strlen(keyword);
  if (!kl) return NULL;
  const char *line = header;
  while (line && *line) {
    const char *p = line;
    while (*p == ' ' || *p == '\t') p++;
    if (strncmp(p, keyword, kl) == 0 && (p[kl] == ' ' || p[kl] == '\t'))
      return line;
    line = strchr(line, '\n');
    if (line) line++;
  }
  return NULL;
}

int ascii_header_get(const char *header, const char *keyword, const char *format, ...) {
  if (!header || !keyword || !format) return -1;
  const char *line = find_key(header, keyword);
  if (!line) return -1;
  const char *v = line;
  while (*v == ' ' || *v == '\t') v++;
  v += strlen(keyword);
  while (*v == ' ' || *v == '\t') v++;
  /* scan only up to end of line / comment */
  size_t n = strcspn(v, "\n#");
  char val[1024];
  if (n >= sizeof val) n = sizeof val - 1;
  memcpy(val, v, n);
  val[n] = 0;
  va_list ap;
  va_start(ap, format);
  int rc = vsscanf(val, format, ap);
  va_end(ap);
  return rc >= 1 ? rc : -1;
}

int ascii_header_set(char *header, const char *keyword, const char *format, ...) {
  if (!header || !keyword || !format) return -1;
  char value[1024];
  va_list ap;
  va_start(ap, format);
  int vn = vsnprintf(value, sizeof value, format, ap);
  va_end(ap);
  if (vn < 0 || (size_t)vn >= sizeof value) return -1;

  const char *cline = find_key(header, keyword);
  if (!cline) {
    /* append before the terminating NUL, on a fresh line */
    size_t hl = strlen(header);
    const char *sep = (hl && header[hl - 1] != '\n') ? "\n" : "";
    sprintf(header + hl, "%s%-12s %s\n", sep, keyword, value);
    return 0;
  }
  char *line = header + (cline - header);
  char *eol = strchr(line, '\n');
  size_t line_len = eol ? (size_t)(eol - line) : strlen(line);
  /* keep leading indent, the key, its separator width and any comment */
  char *p = line;
  while (*p == ' ' || *p == '\t') p++;
  p += strlen(keyword);
  char *vstart = p;
  while (*vstart == ' ' || *vstart == '\t') vstart++;
  char *hash = memchr(vstart, '#', line_len - (size_t)(vstart - line));
  char newline[2048];
  int nl;
  if (hash) {
    int field = (int)(hash - vstart);
    int pad = field > vn ? field - vn : 1;
    nl = snprintf(newline, sizeof newline, "%.*s%s%*s%.*s", (int)(vstart - line), line, value,
                  pad, "", (int)(line + line_len - hash), hash);
  } else {
    nl = snprintf(newline, sizeof newline, "%.*s%s", (int)(vstart - line), line, value);
  }
  if (nl < 0 || (size_t)nl >= sizeof newline) return -1;
  size_t tail = strlen(line + line_len) + 1; /* rest incl. NUL */
  memmove(line + nl, line + line_len, tail);
  memcpy(line, newline, (size_t)nl);
  return 0;
}

int ascii_header_del(char *header, const char *keyword) {
  if (!header || !keyword) return -1;
  const char *cline = find_key(header, keyword);
  if (!cline) return -1;
  char *line = header + (cline - header);
  char *eol = strchr(line, '\n');
  if (eol)
    memmove(line, eol + 1, strlen(eol + 1) + 1);
  else
    *line = 0;
  return 0;
}

/* ascii_header_find (@0x4081e0): the keyword itself, where it starts the
 * header or follows a newline (or a backslash) and is followed by a blank;
 * NULL if absent.  As PSRDADA's, an occurrence at the very start of the
 * header is taken without looking at what follows it. */
char *ascii_header_find(const char *header, const char *keyword) {
  if (!header || !keyword || !*keyword) return NULL;
  const size_t kl = strlen(keyword);
  const char *k = strstr(header, keyword);
  while (k && k > header) {
    if ((k[-1] == '\n' || k[-1] == '\\') && (k[kl] == '\t' || k[kl] == ' ')) break;
    k = strstr(k + 1, keyword);
  }
  return (char *)k;
}

/* HDR_SIZE of the header at the start of an open file: one page read from
 * offset 0, the file offset put back to 0 (@0x408660); (size_t)-1 if the
 * page cannot be read or holds no HDR_SIZE */
size_t ascii_header_get_size_fd(int fd) {
  const long page = sysconf(_SC_PAGESIZE);
  size_t hdr_size = (size_t)-1;
  char *buf = page > 0 ? malloc((size_t)page + 1) : NULL;
  if (!buf) {
    fprintf(stderr, "ascii_header_get_size: failed to allocate %ld bytes\n", page + 1);
    return hdr_size;
  }
  lseek(fd, 0, SEEK_SET);
  if (read(fd, buf, (size_t)page) != (ssize_t)page) {
    fprintf(stderr, "ascii_header_get_size: failed to read %ld bytes from file\n", page);
  } else {
    buf[page] = 0;
    uint64_t v;
    if (ascii_header_get(buf, "HDR_SIZE", "%" SCNu64, &v) == 1)
      hdr_size = (size_t)v;
    else
      fprintf(stderr, "ascii_header_get_size: failed to read HDR_SIZE from header\n");
  }
  lseek(fd, 0, SEEK_SET);
  free(buf);
  return hdr_size;
}

size_t ascii_header_get_size(char *filename) {  /* @0x408790 */
  const int fd = filename ? open(filename, O_RDONLY) : -1;
  if (fd < 0) {
    fprintf(stderr, "ascii_header_get_size: failed to open %s for reading\n", filename ? filename : "(null)");
    return (size_t)-1;
  }
  const size_t n = ascii_header_get_size_fd(fd);
  close(fd);
  return n;
}
