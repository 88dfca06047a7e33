"""Client column-data codec (include/pom_column.h): [u64 length][LZO1X-1 stream]
with raw fallback, as api/api.c:6509-6541 (hvfs_fwrite), :6652-6689
(hvfs_fwritev) and :6427-6446 (read side) use it."""
from __future__ import annotations

import ctypes
from typing import List, Sequence, Tuple

from . import lzo

_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_bound = False


def _lib() -> ctypes.CDLL:
    global _bound
    lib = lzo.load()
    if not _bound:
        lib.pom_col_zip_bound.restype = _sz
        lib.pom_col_zip_bound.argtypes = [_sz]
        lib.pom_col_zip_batch.restype = ctypes.c_int
        lib.pom_col_zip_batch.argtypes = [_vp, _vp, _sz, _vp, _vp, _vp, _vp]
        lib.pom_col_zipv.restype = ctypes.c_int
        lib.pom_col_zipv.argtypes = [_vp, _vp, _sz, _vp, _sz, ctypes.POINTER(_sz),
                                     ctypes.POINTER(ctypes.c_int)]
        lib.pom_col_unzip_batch.restype = ctypes.c_int
        lib.pom_col_unzip_batch.argtypes = [_vp, _vp, _sz, _vp, _vp, _vp, _vp]
        _bound = True
    return lib


def zip_bound(n: int) -> int:
    return int(_lib().pom_col_zip_bound(n))


def _arr(bufs):
    a = (_vp * len(bufs))()
    for i, b in enumerate(bufs):
        a[i] = ctypes.cast(b, _vp).value
    return a


def zip_batch(columns: Sequence[bytes], caps: Sequence[int] = None
              ) -> Tuple[List[bytes], List[int]]:
    """-> (zipped bytes or b"" when raw, compressed flags)."""
    lib = _lib()
    n = len(columns)
    caps = list(caps) if caps is not None else [zip_bound(len(c)) for c in columns]
    src = [ctypes.create_string_buffer(bytes(c), max(len(c), 1)) for c in columns]
    dst = [ctypes.create_string_buffer(max(c, 1)) for c in caps]
    ln = (_sz * n)(*[len(c) for c in columns])
    cp = (_sz * n)(*caps)
    zl = (_sz * n)()
    comp = (ctypes.c_int * n)()
    rc = lib.pom_col_zip_batch(_arr(src), ln, n, _arr(dst), cp, zl, comp)
    if rc != 0:
        raise RuntimeError(f"pom_col_zip_batch: {rc}")
    return [dst[i].raw[: zl[i]] for i in range(n)], list(comp)


def zipv(iov: Sequence[bytes], cap: int) -> Tuple[bytes, int]:
    lib = _lib()
    bufs = [ctypes.create_string_buffer(bytes(b), max(len(b), 1)) for b in iov]
    lens = (_sz * len(iov))(*[len(b) for b in iov])
    out = ctypes.create_string_buffer(max(cap, 1))
    zl = _sz(0)
    comp = ctypes.c_int(0)
    rc = lib.pom_col_zipv(_arr(bufs), lens, len(iov), out, cap, ctypes.byref(zl),
                          ctypes.byref(comp))
    if rc != 0:
        raise RuntimeError(f"pom_col_zipv: {rc}")
    return out.raw[: zl.value], comp.value


def unzip_batch(zipped: Sequence[bytes], caps: Sequence[int]) -> Tuple[List[bytes], List[int]]:
    """-> (decoded bytes, err codes: 0 = decoded to exactly the recorded length)."""
    lib = _lib()
    n = len(zipped)
    src = [ctypes.create_string_buffer(bytes(z), max(len(z), 1)) for z in zipped]
    out = [ctypes.create_string_buffer(max(c, 1)) for c in caps]
    zl = (_sz * n)(*[len(z) for z in zipped])
    cp = (_sz * n)(*caps)
    ol = (_sz * n)()
    err = (ctypes.c_int * n)()
    rc = lib.pom_col_unzip_batch(_arr(src), zl, n, _arr(out), cp, ol, err)
    if rc != 0:
        raise RuntimeError(f"pom_col_unzip_batch: {rc}")
    return [out[i].raw[: ol[i]] for i in range(n)], list(err)
