/* io_util.c -- see io_util.h.  Used by the MDSL append file (itb_codec.c,
 * the mdsl/storage.c:455-519 write path). */
#define _GNU_SOURCE
#include <errno.h>
#include <stdint.h>
#include <sys/uio.h>

#include "io_util.h"

int pom_pwritev_all(int fd, struct iovec *iov, int n, off_t off, pom_pwritev_fn fn)
{
    if (!fn)
        fn = pwritev;
    int i = 0;
    while (i < n && iov[i].iov_len == 0)
        i++;
    while (i < n) {
        const ssize_t w = fn(fd, iov + i, n - i, off);
        if (w < 0) {
            if (errno == EINTR)
                continue;
            return -errno;
        }
        if (w == 0)
            return -EIO;
        off += w;
        /* advance the cursor by w bytes: whole iovecs, then into the next */
        size_t adv = (size_t)w;
        while (i < n && adv >= iov[i].iov_len) {
            adv -= iov[i].iov_len;
            i++;
        }
        if (adv) {
            iov[i].iov_base = (uint8_t *)iov[i].iov_base + adv;
            iov[i].iov_len -= adv;
        }
        while (i < n && iov[i].iov_len == 0)
            i++;
    }
    return 0;
}
