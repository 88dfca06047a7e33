"""Helpers for GPU tests: pack host blocks into device batches and run the
device-resident C-ABI (lzo_mi355x_compress_dev / _decompress_dev)."""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

from pomegranate_amd import lzo


def _offsets(sizes, align=16):
    sizes = np.asarray(sizes, dtype=np.uint64)
    padded = (sizes + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
    off = np.zeros(len(sizes), dtype=np.uint64)
    if len(sizes) > 1:
        off[1:] = np.cumsum(padded[:-1])
    total = int(padded.sum()) if len(sizes) else 0
    return off, total


def device_batch(torch, blocks: Sequence[bytes], dev, shift: int = 0):
    """Pack blocks (each 16-B aligned + shift) into one HBM arena."""
    sizes = [len(b) for b in blocks]
    off, total = _offsets([s + shift for s in sizes])
    off = off + np.uint64(shift)
    host = np.zeros(max(total + shift, 1), dtype=np.uint8)
    for b, o in zip(blocks, off):
        host[int(o): int(o) + len(b)] = np.frombuffer(b, dtype=np.uint8)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return lzo.DeviceBatch(t(host), t(off.view(np.int64)),
                           t(np.asarray(sizes, np.uint32).view(np.int32)))


def empty_batch(torch, caps: Sequence[int], dev, fill: int = 0):
    off, total = _offsets(caps)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    arena = torch.full((max(total, 1),), fill, dtype=torch.uint8, device=dev)
    return lzo.DeviceBatch(arena, t(off.view(np.int64)),
                           t(np.asarray(caps, np.uint32).view(np.int32)))


def gpu_compress(torch, blocks: Sequence[bytes], dev, shift: int = 0, scratch: bool = False):
    """Device-batch compress.  Without scratch: the LDS-dictionary encoder;
    with scratch: the global-dictionary one-wave encoder the bench times
    (lzo1x_encode_gdict1_kernel)."""
    src = device_batch(torch, blocks, dev, shift)
    dst = empty_batch(torch, [lzo.worst_compress(len(b)) for b in blocks], dev, fill=0xA5)
    n = len(blocks)
    olen = torch.zeros(n, dtype=torch.int32, device=dev)
    st = torch.full((n,), 99, dtype=torch.int32, device=dev)
    scr = torch.zeros(lzo.compress_scratch_bytes(n), dtype=torch.uint8, device=dev) if scratch else None
    lzo.compress_dev(src, dst, olen, st, scratch=scr)
    torch.cuda.synchronize()
    return fetch(dst, olen), st.cpu().numpy().tolist()


def gpu_decompress(torch, comps: Sequence[bytes], caps: Sequence[int], dev, shift: int = 0):
    src = device_batch(torch, comps, dev, shift)
    dst = empty_batch(torch, caps, dev, fill=0x5A)
    n = len(comps)
    olen = torch.zeros(n, dtype=torch.int32, device=dev)
    st = torch.full((n,), 99, dtype=torch.int32, device=dev)
    nscr = lzo.decompress_scratch_bytes(n)
    scratch = torch.empty(max(nscr, 1), dtype=torch.uint8, device=dev) if nscr else None
    lzo.decompress_dev(src, dst, olen, st, scratch)
    torch.cuda.synchronize()
    outs = fetch(dst, olen, cap=caps)
    return outs, st.cpu().numpy().tolist(), dst


def gpu_decompress_fast(torch, comps: Sequence[bytes], caps: Sequence[int], dev):
    """gpu_decompress plus the number of blocks the throughput decoder handed
    to the exact decoder (the fallback list count at the head of scratch)."""
    src = device_batch(torch, comps, dev)
    dst = empty_batch(torch, caps, dev, fill=0x5A)
    n = len(comps)
    olen = torch.zeros(n, dtype=torch.int32, device=dev)
    st = torch.full((n,), 99, dtype=torch.int32, device=dev)
    scratch = torch.zeros(lzo.decompress_scratch_bytes(n), dtype=torch.uint8, device=dev)
    lzo.decompress_dev(src, dst, olen, st, scratch)
    torch.cuda.synchronize()
    fallbacks = int(scratch[:4].view(torch.int32).item())
    return fetch(dst, olen, cap=caps), st.cpu().numpy().tolist(), fallbacks


def fetch(batch, olen, cap=None) -> List[bytes]:
    host = batch.arena.cpu().numpy()
    off = batch.off.cpu().numpy()
    ol = olen.cpu().numpy().astype(np.int64)
    res = []
    for i in range(len(off)):
        n = int(ol[i]) if cap is None else min(int(ol[i]), int(cap[i]))
        res.append(host[int(off[i]): int(off[i]) + n].tobytes())
    return res


def gpu_decompress_win(torch, comps: Sequence[bytes], caps: Sequence[int], dev, kind: str = "win"):
    """The windowed decoder alone (lzo_mi355x_launch_decompress_win), without
    the exact decoder behind it.  Returns the outputs, statuses and the ids of
    the blocks it handed over (fallback list)."""
    import ctypes
    lib = lzo.load()
    fn = getattr(lib, f"lzo_mi355x_launch_decompress_{kind}")
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p] * 10 + [ctypes.c_uint32, ctypes.c_void_p]
    src = device_batch(torch, comps, dev)
    dst = empty_batch(torch, caps, dev, fill=0x5A)
    n = len(comps)
    olen = torch.zeros(n, dtype=torch.int32, device=dev)
    st = torch.full((n,), 99, dtype=torch.int32, device=dev)
    head = torch.zeros(64, dtype=torch.int32, device=dev)
    ids = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)
    p = lambda x: x.data_ptr()
    rc = fn(p(src.arena), p(src.off), p(src.length), p(dst.arena), p(dst.off), p(dst.length),
            p(olen), p(st), p(head), p(ids), n, torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    nfb = int(head[0].item())
    return fetch(dst, olen, cap=caps), st.cpu().numpy().tolist(), sorted(ids[:nfb].cpu().numpy().tolist())


def gpu_decompress_lat(torch, comps: Sequence[bytes], caps: Sequence[int], dev, group: int = 1):
    """The latency decoder (lzo1x_decode_lat.hip) alone, without the exact
    decoder behind it: one block per pipeline (group 1,
    lzo_mi355x_launch_decompress_lat) or up to `group` blocks side by side in
    one pipeline (lzo_mi355x_launch_decompress_lat_n).  Returns the outputs,
    statuses and the ids of the blocks it handed over; blocks outside its range
    (the launcher returns -1) are reported with status None."""
    import ctypes
    lib = lzo.load()
    one = lib.lzo_mi355x_launch_decompress_lat
    one.restype = ctypes.c_int
    one.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                    ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    many = lib.lzo_mi355x_launch_decompress_lat_n
    many.restype = ctypes.c_int
    many.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_uint32] + [ctypes.c_void_p] * 4 + \
        [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    sz = lib.lzo_mi355x_decompress_lat_scratch
    sz.restype = ctypes.c_size_t
    sz.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
    szn = lib.lzo_mi355x_decompress_lat_scratch_n
    szn.restype = ctypes.c_size_t
    szn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
    src = device_batch(torch, comps, dev)
    dst = empty_batch(torch, caps, dev, fill=0x5A)
    n = len(comps)
    olen = torch.zeros(n, dtype=torch.int32, device=dev)
    st = torch.full((n,), 99, dtype=torch.int32, device=dev)
    head = torch.zeros(64, dtype=torch.int32, device=dev)
    ids = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)
    p = lambda x: x.data_ptr()
    s = torch.cuda.current_stream().cuda_stream
    soff = src.off.cpu().numpy().astype(np.uint64)
    doff = dst.off.cpu().numpy().astype(np.uint64)
    launched = [False] * n
    for g0 in range(0, n, group):
        g1 = min(n, g0 + group)
        if group == 1:
            z, cap = comps[g0], int(caps[g0])
            need = int(sz(len(z), cap)) if len(z) else 0
            scratch = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
            rc = one(p(src.arena) + int(soff[g0]), len(z), p(dst.arena) + int(doff[g0]), cap,
                     p(olen), p(st), p(head), p(ids), g0, p(scratch), need, s)
        else:
            so = np.ascontiguousarray(soff[g0:g1] - soff[g0])
            do = np.ascontiguousarray(doff[g0:g1] - doff[g0])
            zz = np.array([len(c) for c in comps[g0:g1]], dtype=np.uint32)
            cc = np.array([int(c) for c in caps[g0:g1]], dtype=np.uint32)
            need = int(szn(so.ctypes.data, zz.ctypes.data, cc.ctypes.data, g1 - g0))
            scratch = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
            rc = many(p(src.arena) + int(soff[g0]), so.ctypes.data, zz.ctypes.data,
                      p(dst.arena) + int(doff[g0]), do.ctypes.data, cc.ctypes.data, g1 - g0,
                      p(olen), p(st), p(head), p(ids), g0, p(scratch), need, s)
        torch.cuda.synchronize()
        for i in range(g0, g1):
            launched[i] = rc == 0
    nfb = int(head[0].item())
    sts = [x if ok else None for x, ok in zip(st.cpu().numpy().tolist(), launched)]
    return fetch(dst, olen, cap=caps), sts, sorted(ids[:nfb].cpu().numpy().tolist())
