/* io_util.h -- gathered positional writes that survive short writes and
 * EINTR (internal to liblzo_mi355x.so; plain C, also linked into the CPU test
 * harness tests/native/split_mock.c, which drives it with a writer that
 * writes a few bytes at a time). */
#ifndef POM_IO_UTIL_H
#define POM_IO_UTIL_H 1

#include <sys/types.h>
#include <sys/uio.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef ssize_t (*pom_pwritev_fn)(int fd, const struct iovec *iov, int iovcnt, off_t off);

/* Writes all bytes of iov[0..n) at file offset off with fn (pwritev when
 * NULL), resuming after short writes from a cursor (iovec index + offset)
 * and retrying on EINTR.  iov[] is modified.  Returns 0 or -errno (-EIO when
 * fn wrote nothing). */
int pom_pwritev_all(int fd, struct iovec *iov, int n, off_t off, pom_pwritev_fn fn);

#ifdef __cplusplus
}
#endif

#endif
