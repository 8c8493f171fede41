/* declarations only -- see README.txt */
#ifndef __MULTILOG_H
#define __MULTILOG_H
#include <stdio.h>
#include <syslog.h>
typedef struct multilog_t multilog_t;
multilog_t *multilog_open(const char *program_name, char syslog);
int multilog_close(multilog_t *m);
int multilog_add(multilog_t *m, FILE *fptr);
int multilog(multilog_t *m, int priority, const char *format, ...);
#endif
