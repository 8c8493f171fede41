/* declarations only -- see README.txt */
#ifndef __DADA_DEF_H
#define __DADA_DEF_H
#define DADA_DEFAULT_HEADER_SIZE 4096
#endif
