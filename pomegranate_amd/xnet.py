"""xnet wire framing of ITB messages (include/pom_xnet.h).

Python mirror of the reference's per-message ITB transfer, batched:
  frame / parse  <- struct xnet_msg_tx + tx.len data bytes, the magic check
                    (include/xnet.h:27-67, xnet/xnet_simple.c:480-587)
  reply_batch    <- __mdsl_send_rpy_data(..., flag 1): XNET_RPY_DATA_ITB
                    (mdsl/m2ml.c:87-120)
  wb_batch       <- txg_wb_itb: itb_lzo_compress + the write-back REQ
                    (mds/txg.c:548-584, :733-770)
  recv_batch     <- the MDS ITB load path (mds/itb.c:140-168)
"""
from __future__ import annotations

import ctypes
import errno
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

from . import itb, lzo

TX_SIZE = 72
MSG_REQ, MSG_RPY = 1, 2
NEED_DATA_FREE = 0x0004
RPY_DATA, RPY_DATA_ITB = 0x03, 0x04
MDS2MDSL_WBTXG = 0x0000000080030000
WBTXG_ITB = 0x0002

_vp = ctypes.c_void_p
_bound = False


class Tx(ctypes.Structure):
    """struct xnet_msg_tx (72 bytes on LP64)."""
    _fields_ = [("vm", ctypes.c_uint8), ("type", ctypes.c_uint8), ("flag", ctypes.c_uint16),
                ("err", ctypes.c_int32), ("ssite_id", ctypes.c_uint64),
                ("dsite_id", ctypes.c_uint64), ("cmd", ctypes.c_uint64),
                ("arg0", ctypes.c_uint64), ("arg1", ctypes.c_uint64),
                ("reqno", ctypes.c_uint32), ("len", ctypes.c_uint32),
                ("handle", ctypes.c_uint64), ("reserved", ctypes.c_uint64)]

    @property
    def magic(self) -> int:
        return self.vm >> 4


class _Frame(ctypes.Structure):
    _fields_ = [("tx", Tx), ("data", _vp), ("dropped", ctypes.c_int)]


class Req(ctypes.Structure):
    _fields_ = [("ssite_id", ctypes.c_uint64), ("reqno", ctypes.c_uint32),
                ("handle", ctypes.c_uint64)]


class Wb(ctypes.Structure):
    _fields_ = [("dsite_id", ctypes.c_uint64), ("vid", ctypes.c_uint64)]


assert ctypes.sizeof(Tx) == TX_SIZE


@dataclass
class Frame:
    tx: Tx
    offset: int             # of the data in the wire buffer
    dropped: bool


def _lib() -> ctypes.CDLL:
    global _bound
    lib = lzo.load()
    if not _bound:
        lib.pom_xnet_frame.restype = ctypes.c_size_t
        lib.pom_xnet_frame.argtypes = [_vp, ctypes.c_size_t, ctypes.POINTER(Tx), _vp,
                                       ctypes.c_uint32]
        lib.pom_xnet_parse.restype = ctypes.c_int
        lib.pom_xnet_parse.argtypes = [_vp, ctypes.c_size_t, ctypes.c_uint8, ctypes.POINTER(_Frame),
                                       ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
                                       ctypes.POINTER(ctypes.c_size_t)]
        lib.pom_xnet_itb_reply_batch.restype = ctypes.c_int
        lib.pom_xnet_itb_reply_batch.argtypes = [_vp, ctypes.POINTER(Req), ctypes.c_size_t,
                                                 ctypes.c_uint64, ctypes.c_uint8, _vp,
                                                 ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        lib.pom_xnet_itb_wb_batch.restype = ctypes.c_int
        lib.pom_xnet_itb_wb_batch.argtypes = [_vp, _vp, _vp, ctypes.POINTER(Wb), ctypes.c_size_t,
                                              ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint8, _vp,
                                              ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t), _vp]
        lib.pom_xnet_itb_recv_batch.restype = ctypes.c_int
        lib.pom_xnet_itb_recv_batch.argtypes = [ctypes.POINTER(_Frame), ctypes.c_size_t, _vp,
                                                ctypes.c_size_t, _vp]
        _bound = True
    return lib


def _addr(buf: bytearray) -> Tuple[int, object]:
    c = (ctypes.c_char * len(buf)).from_buffer(buf)
    return ctypes.addressof(c), c


def frame(wire: bytearray, offset: int, hdr: Tx, data: bytes) -> int:
    """pom_xnet_frame at wire[offset:]: bytes written (0: no room)."""
    lib = _lib()
    base, keep = _addr(wire)
    d = bytes(data)
    return lib.pom_xnet_frame(base + offset, len(wire) - offset, ctypes.byref(hdr), d, len(d))


def parse(wire: bytearray, length: Optional[int] = None, magic: int = 0,
          max_frames: int = 1 << 16) -> Tuple[List[Frame], int]:
    """pom_xnet_parse: (frames, bytes consumed)."""
    lib = _lib()
    length = len(wire) if length is None else length
    base, keep = _addr(wire)
    fr = (_Frame * max_frames)()
    nf, used = ctypes.c_size_t(0), ctypes.c_size_t(0)
    lib.pom_xnet_parse(base, length, magic, fr, max_frames, ctypes.byref(nf), ctypes.byref(used))
    out = [Frame(Tx.from_buffer_copy(fr[i].tx), fr[i].data - base, bool(fr[i].dropped))
           for i in range(nf.value)]
    return out, used.value


def reply_batch(recs: Sequence[bytearray], reqs: Sequence[Tuple[int, int, int]], site_id: int,
                magic: int, wire: bytearray) -> Tuple[int, int]:
    """pom_xnet_itb_reply_batch; reqs = (ssite_id, reqno, handle).  (rc, wire_len)."""
    lib = _lib()
    n = len(recs)
    ptr, k1 = itb._ptrs(list(recs))
    rq = (Req * max(n, 1))(*[Req(s, r, h) for s, r, h in reqs])
    base, k2 = _addr(wire)
    wl = ctypes.c_size_t(0)
    rc = lib.pom_xnet_itb_reply_batch(ptr, rq, n, site_id, magic, base, len(wire), ctypes.byref(wl))
    return rc, wl.value


def wb_batch(recs: Sequence[bytearray], tmps: Sequence[bytearray], dests: Sequence[Tuple[int, int]],
             site_id: int, txg: int, magic: int, wire: bytearray) -> Tuple[int, int, List[int]]:
    """pom_xnet_itb_wb_batch; dests = (dsite_id, vid).  (rc, wire_len, err)."""
    lib = _lib()
    n = len(recs)
    pin, k1 = itb._ptrs(list(recs))
    ptmp, k2 = itb._ptrs(list(tmps))
    caps = (ctypes.c_size_t * max(n, 1))(*[len(t) for t in tmps])
    wb = (Wb * max(n, 1))(*[Wb(d, v) for d, v in dests])
    base, k3 = _addr(wire)
    wl = ctypes.c_size_t(0)
    err = (ctypes.c_int * max(n, 1))()
    rc = lib.pom_xnet_itb_wb_batch(pin, ptmp, caps, wb, n, site_id, txg, magic, base, len(wire),
                                   ctypes.byref(wl), err)
    if rc not in (0, -errno.ENOSPC):
        raise RuntimeError(f"pom_xnet_itb_wb_batch: {rc}")
    return rc, wl.value, list(err)[:n]


def recv_batch(wire: bytearray, frames: Sequence[Frame], bufs: Sequence[bytearray]) -> List[int]:
    """pom_xnet_itb_recv_batch: frames of `wire` into whole-ITB buffers (all of
    one size).  err[b] (0, -EBADMSG, -EIO, -EFAULT)."""
    lib = _lib()
    n = len(frames)
    base, k1 = _addr(wire)
    fr = (_Frame * max(n, 1))()
    for i, f in enumerate(frames):
        fr[i].tx = f.tx
        fr[i].data = base + f.offset
        fr[i].dropped = int(f.dropped)
    pb, k2 = itb._ptrs(list(bufs))
    err = (ctypes.c_int * max(n, 1))()
    cap = len(bufs[0]) if n else 0
    rc = lib.pom_xnet_itb_recv_batch(fr, n, pb, cap, err)
    if rc != 0:
        raise RuntimeError(f"pom_xnet_itb_recv_batch: {rc}")
    return list(err)[:n]
