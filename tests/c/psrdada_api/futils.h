/* declarations only -- see README.txt */
#ifndef __FUTILS_H
#define __FUTILS_H
#include <stdint.h>
long fileread(const char *filename, char *buffer, unsigned bufsz);
#endif
