"""ITB record codec and MDSL append-file loopback (include/pom_itb.h).

Python mirror of the reference's per-ITB operations, batched on the GPU:
  compress_batch   <- itb_lzo_compress   (mds/itb.c:2904-2945)
  decompress_batch <- itb_lzo_decompress (mds/itb.c:2949-2980, mdsl/gc.c:755-786)
  AppendFile       <- append_buf_write / append_buf_flush_remap (mdsl/storage.c:384-519)
  read_record      <- the header-then-payload ITB read (mdsl/storage.c:2507-2640)
"""
from __future__ import annotations

import ctypes
import os
import struct
from typing import List, Sequence, Tuple

import numpy as np

from . import lzo, synth

ITBH_SIZE = 264
LEN_OFF, ZLEN_OFF, ALGO_OFF = 240, 244, 248
COMPR_NONE, COMPR_LZO = 0, 1
PAYLOAD_MIN, PAYLOAD_MAX = 12416, 536192
ITB_FULL = ITBH_SIZE + PAYLOAD_MAX      # sizeof(struct itb) + ITB_SIZE * sizeof(struct ite)

_vp = ctypes.c_void_p
_bound = False


class _Abuf(ctypes.Structure):
    _fields_ = [("fd", ctypes.c_int), ("win", ctypes.c_size_t), ("addr", _vp),
                ("file_offset", ctypes.c_uint64), ("offset", ctypes.c_size_t),
                ("falloc_end", ctypes.c_uint64), ("acclen", ctypes.c_uint64)]


def _lib() -> ctypes.CDLL:
    global _bound
    lib = lzo.load()
    if not _bound:
        lib.pom_itb_lzo_compress_batch.restype = ctypes.c_int
        lib.pom_itb_lzo_compress_batch.argtypes = [_vp] * 5 + [ctypes.c_size_t]
        lib.pom_itb_lzo_compress_append_batch.restype = ctypes.c_int
        lib.pom_itb_lzo_compress_append_batch.argtypes = [_vp] * 5 + [ctypes.c_size_t,
                                                                      ctypes.POINTER(_Abuf), _vp]
        lib.pom_itb_lzo_decompress_batch.restype = ctypes.c_int
        lib.pom_itb_lzo_decompress_batch.argtypes = [_vp] * 4 + [ctypes.c_size_t]
        lib.pom_abuf_open.restype = ctypes.c_int
        lib.pom_abuf_open.argtypes = [ctypes.POINTER(_Abuf), ctypes.c_char_p, ctypes.c_size_t]
        lib.pom_abuf_append.restype = ctypes.c_int
        lib.pom_abuf_append.argtypes = [ctypes.POINTER(_Abuf), _vp, ctypes.c_size_t,
                                        ctypes.POINTER(ctypes.c_uint64)]
        lib.pom_abuf_append_batch.restype = ctypes.c_int
        lib.pom_abuf_append_batch.argtypes = [ctypes.POINTER(_Abuf), _vp, _vp, ctypes.c_size_t, _vp]
        lib.pom_abuf_close.restype = ctypes.c_int
        lib.pom_abuf_close.argtypes = [ctypes.POINTER(_Abuf)]
        lib.pom_itb_read.restype = ctypes.c_int
        lib.pom_itb_read.argtypes = [ctypes.c_int, ctypes.c_uint64, _vp, ctypes.c_size_t,
                                     ctypes.POINTER(ctypes.c_size_t)]
        lib.pom_itb_read_lzo_decompress_batch.restype = ctypes.c_int
        lib.pom_itb_read_lzo_decompress_batch.argtypes = [ctypes.c_int, _vp, ctypes.c_size_t] + [_vp] * 6
        lib.pom_itb_read_batch.restype = ctypes.c_int
        lib.pom_itb_read_batch.argtypes = [ctypes.c_int, _vp, ctypes.c_size_t, _vp, _vp, _vp, _vp]
        _bound = True
    return lib


def header_fields(rec) -> Tuple[int, int, int]:
    """(len, zlen, compress_algo) of an ITB record."""
    ln, zl = struct.unpack_from("<II", rec, LEN_OFF)
    (algo,) = struct.unpack_from("<H", rec, ALGO_OFF)
    return ln, zl, algo


def make_record(seed: int, n_ites: int, model: int = synth.ITB) -> bytearray:
    """A synthetic ITB record: a 264-byte header (random fields, len = 264 +
    payload, zlen 0, COMPR_NONE) and a payload of 11904 + 512 * n_ites bytes
    (SURVEY.md Appendix B), in a full-size ITB buffer."""
    n = 11904 + 512 * n_ites
    rng = np.random.default_rng(seed)
    rec = bytearray(ITB_FULL)
    rec[:ITBH_SIZE] = rng.integers(0, 256, ITBH_SIZE, dtype=np.uint8).tobytes()
    struct.pack_into("<II", rec, LEN_OFF, ITBH_SIZE + n, 0)
    struct.pack_into("<H", rec, ALGO_OFF, COMPR_NONE)
    rec[ITBH_SIZE:ITBH_SIZE + n] = synth.block(model, seed, n)
    return rec


def _ptrs(bufs: Sequence[bytearray]):
    arr = (_vp * len(bufs))()
    keep = []
    for i, b in enumerate(bufs):
        c = (ctypes.c_char * len(b)).from_buffer(b)
        keep.append(c)
        arr[i] = ctypes.addressof(c)
    return arr, keep


def compress_batch(ins: List[bytearray], tmps: List[bytearray]) -> Tuple[List[int], List[int]]:
    """pom_itb_lzo_compress_batch: returns (which[b]: 0 = oi is in[b], 1 = tmp[b];
    err[b])."""
    lib = _lib()
    n = len(ins)
    pin, k1 = _ptrs(ins)
    ptmp, k2 = _ptrs(tmps)
    caps = (ctypes.c_size_t * n)(*[len(t) for t in tmps])
    oi = (_vp * n)()
    err = (ctypes.c_int * n)()
    rc = lib.pom_itb_lzo_compress_batch(pin, ptmp, caps, oi, err, n)
    if rc != 0:
        raise RuntimeError(f"pom_itb_lzo_compress_batch: {rc}")
    which = [0 if oi[b] == pin[b] else 1 for b in range(n)]
    return which, list(err)


def compress_append_batch(ins: List[bytearray], tmps: List[bytearray], af: "AppendFile"):
    """pom_itb_lzo_compress_append_batch: compresses the records and appends
    each (compressed or kept) to the append file af as soon as its chunk is
    done.  Returns (which[b], err[b], location[b]) as compress_batch and
    AppendFile.append_batch do."""
    lib = _lib()
    n = len(ins)
    pin, k1 = _ptrs(ins)
    ptmp, k2 = _ptrs(tmps)
    caps = (ctypes.c_size_t * n)(*[len(t) for t in tmps])
    oi = (_vp * n)()
    err = (ctypes.c_int * n)()
    locs = (ctypes.c_uint64 * max(n, 1))()
    rc = lib.pom_itb_lzo_compress_append_batch(pin, ptmp, caps, oi, err, n, ctypes.byref(af.ab), locs)
    if rc != 0:
        raise RuntimeError(f"pom_itb_lzo_compress_append_batch: {rc}")
    which = [0 if oi[b] == pin[b] else 1 for b in range(n)]
    return which, list(err), list(locs[:n])


def decompress_batch(ins: List[bytearray]) -> Tuple[List[int], List[int]]:
    """pom_itb_lzo_decompress_batch in place: (err[b], len_ok[b])."""
    lib = _lib()
    n = len(ins)
    pin, keep = _ptrs(ins)
    caps = (ctypes.c_size_t * n)(*[len(b) for b in ins])
    err = (ctypes.c_int * n)()
    ok = (ctypes.c_int * n)()
    rc = lib.pom_itb_lzo_decompress_batch(pin, caps, err, ok, n)
    if rc != 0:
        raise RuntimeError(f"pom_itb_lzo_decompress_batch: {rc}")
    return list(err), list(ok)


class AppendFile:
    """MDSL ITB append file (pom_abuf_*)."""

    def __init__(self, path: str, win: int = 64 << 20):
        self.lib = _lib()
        self.ab = _Abuf()
        rc = self.lib.pom_abuf_open(ctypes.byref(self.ab), path.encode(), win)
        if rc:
            raise OSError(-rc, os.strerror(-rc), path)

    def append(self, rec, length: "int | None" = None) -> int:
        """Appends the first `length` bytes (default all) of rec: bytes, or a
        writable buffer (bytearray, memoryview) passed without a copy."""
        loc = ctypes.c_uint64(0)
        n = len(rec) if length is None else length
        if isinstance(rec, bytes):
            ptr, keep = rec, None
        else:
            keep = (ctypes.c_char * len(rec)).from_buffer(rec)
            ptr = ctypes.addressof(keep)
        rc = self.lib.pom_abuf_append(ctypes.byref(self.ab), ptr, n, ctypes.byref(loc))
        del keep
        if rc:
            raise OSError(-rc, os.strerror(-rc))
        return loc.value

    def append_batch(self, recs, lengths=None) -> list:
        """Appends the first lengths[i] bytes (default all) of each record in
        one call (pom_abuf_append_batch): the file and the locations equal
        those of append() called in order."""
        n = len(recs)
        ptrs = (ctypes.c_void_p * max(n, 1))()
        lens = (ctypes.c_size_t * max(n, 1))()
        locs = (ctypes.c_uint64 * max(n, 1))()
        keep = []
        for i, r in enumerate(recs):
            if isinstance(r, bytes):
                ptrs[i] = ctypes.cast(ctypes.c_char_p(r), ctypes.c_void_p).value
                keep.append(r)
            else:
                c = (ctypes.c_char * len(r)).from_buffer(r)
                keep.append(c)
                ptrs[i] = ctypes.addressof(c)
            lens[i] = len(r) if lengths is None else int(lengths[i])
            if lens[i] > len(r):
                raise ValueError(f"record {i}: length {lens[i]} > buffer {len(r)}")
        rc = self.lib.pom_abuf_append_batch(ctypes.byref(self.ab), ptrs, lens, n, locs)
        del keep
        if rc:
            raise OSError(-rc, os.strerror(-rc))
        return list(locs[:n])

    def close(self) -> None:
        rc = self.lib.pom_abuf_close(ctypes.byref(self.ab))
        if rc:
            raise OSError(-rc, os.strerror(-rc))


def read_batch(fd: int, locations, outs) -> list:
    """pom_itb_read_batch: record i at locations[i] into outs[i] (writable
    buffers, len = cap), read on up to 8 threads.  Returns outs; raises
    OSError for the first record that failed."""
    lib = _lib()
    n = len(locations)
    loc = (ctypes.c_uint64 * max(n, 1))(*locations)
    keep = [(ctypes.c_char * len(o)).from_buffer(o) for o in outs]
    ptrs = (ctypes.c_void_p * max(n, 1))(*[ctypes.addressof(c) for c in keep])
    caps = (ctypes.c_size_t * max(n, 1))(*[len(o) for o in outs])
    lens = (ctypes.c_size_t * max(n, 1))()
    errs = (ctypes.c_int * max(n, 1))()
    rc = lib.pom_itb_read_batch(fd, loc, n, ptrs, caps, lens, errs)
    del keep
    if rc:
        raise OSError(-rc, os.strerror(-rc))
    for i in range(n):
        if errs[i]:
            raise OSError(-errs[i], f"record {i}: " + os.strerror(-errs[i]))
    return list(outs)


def read_record(fd: int, location: int, cap: int = ITB_FULL,
                out: "bytearray | None" = None) -> bytearray:
    """pom_itb_read into `out` (reused, len(out) is the cap) or a new buffer."""
    lib = _lib()
    buf = bytearray(cap) if out is None else out
    cap = len(buf)
    c = (ctypes.c_char * cap).from_buffer(buf)
    ln = ctypes.c_size_t(0)
    rc = lib.pom_itb_read(fd, location, ctypes.addressof(c), cap, ctypes.byref(ln))
    del c
    if rc:
        raise OSError(-rc, os.strerror(-rc))
    return buf


def read_decompress_batch(fd: int, locations, outs):
    """pom_itb_read_lzo_decompress_batch: record i at locations[i] into outs[i]
    (writable buffers, len = cap), LZO records decoded in place as their
    chunks are read.  Returns (outs, err, derr, len_ok)."""
    lib = _lib()
    n = len(locations)
    loc = (ctypes.c_uint64 * max(n, 1))(*locations)
    pbuf, keep = _ptrs(outs)
    caps = (ctypes.c_size_t * max(n, 1))(*[len(o) for o in outs])
    lens = (ctypes.c_size_t * max(n, 1))()
    err = (ctypes.c_int * max(n, 1))()
    derr = (ctypes.c_int * max(n, 1))()
    ok = (ctypes.c_int * max(n, 1))()
    rc = lib.pom_itb_read_lzo_decompress_batch(fd, loc, n, pbuf, caps, lens, err, derr, ok)
    del keep
    if rc != 0:
        raise RuntimeError(f"pom_itb_read_lzo_decompress_batch: {rc}")
    return outs, list(err[:n]), list(derr[:n]), list(ok[:n])
