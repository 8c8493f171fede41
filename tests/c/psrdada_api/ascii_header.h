/* declarations only -- see README.txt */
#ifndef __ASCII_HEADER_H
#define __ASCII_HEADER_H
int ascii_header_set(char *header, const char *keyword, const char *code, ...);
int ascii_header_get(const char *header, const char *keyword, const char *code, ...);
#endif
