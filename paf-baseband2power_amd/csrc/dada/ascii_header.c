/*
 * ascii_header.c -- DADA "KEY value  # comment" headers (4096 B,
 * header_baseband2power.txt:1-45), get/set as used at capture.c:758-778.
 * A key matches only at the start of a line and only as a whole word.
 */
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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
