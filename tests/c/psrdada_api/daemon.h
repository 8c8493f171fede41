/* declarations only -- see README.txt (included by the reference's hosts) */
#ifndef __DAEMON_H
#define __DAEMON_H
int be_a_daemon(void);
#endif
