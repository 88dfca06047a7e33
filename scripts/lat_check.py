"""Latency decoder (lzo1x_decode_lat.hip) on lone ITB blocks: pipeline time by
HIP events (median of 7) and output check, beside the windowed decoder's
kernel on the same block.  GPU box.  Usage: python scripts/lat_check.py"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pomegranate_amd import lzo, synth  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
lib = lzo.load()
lat = lib.lzo_mi355x_launch_decompress_lat
lat.restype = ctypes.c_int
lat.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                ctypes.c_size_t, ctypes.c_void_p]
sz = lib.lzo_mi355x_decompress_lat_scratch
sz.restype = ctypes.c_size_t
sz.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
win = lib.lzo_mi355x_launch_decompress_win
win.restype = ctypes.c_int
win.argtypes = [ctypes.c_void_p] * 10 + [ctypes.c_uint32, ctypes.c_void_p]
p = lambda x: x.data_ptr()
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def timed(fn, reps=7):
    s = torch.cuda.current_stream()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        fn(s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


for n in (12416, 32768, 65536, 262144, 536192):
    data = synth.block(synth.ITB, 4242 + n, n)
    src = t(np.frombuffer(data, dtype=np.uint8))
    cap = lzo.worst_compress(n)
    zb = lzo.DeviceBatch(torch.zeros(cap + 256, dtype=torch.uint8, device=dev), t(np.zeros(1, np.int64)),
                         t(np.array([cap], np.int32)))
    zl = torch.zeros(1, dtype=torch.int32, device=dev)
    zs = torch.zeros_like(zl)
    lzo.compress_dev(lzo.DeviceBatch(src, t(np.zeros(1, np.int64)), t(np.array([n], np.int32))), zb, zl, zs)
    torch.cuda.synchronize()
    zlen = int(zl.item())
    out = torch.zeros(n + 256, dtype=torch.uint8, device=dev)
    ol = torch.zeros(1, dtype=torch.int32, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    head = torch.zeros(64, dtype=torch.int32, device=dev)
    ids = torch.zeros(1, dtype=torch.int32, device=dev)
    need = int(sz(zlen, n))
    scr = torch.empty(need, dtype=torch.uint8, device=dev)

    def run_lat(s):
        head.zero_()
        assert lat(p(zb.arena), zlen, p(out), n, p(ol), p(st), p(head), p(ids), 0, p(scr), need, s) == 0

    ms = timed(run_lat)
    ok = int(st.item()) == 0 and int(ol.item()) == n and torch.equal(out[:n], src)
    so = t(np.zeros(1, np.int64))
    sl = t(np.array([zlen], np.int32))
    dc = t(np.array([n], np.int32))

    def run_win(s):
        head.zero_()
        assert win(p(zb.arena), p(so), p(sl), p(out), p(so), p(dc), p(ol), p(st), p(head), p(ids), 1, s) == 0

    out.zero_()
    mw = timed(run_win)
    okw = int(st.item()) == 0 and torch.equal(out[:n], src)
    print(f"{n} B (z {zlen}): latency decoder {ms:.3f} ms exact {ok} (scratch {need / 2**20:.1f} MiB); "
          f"windowed {mw:.3f} ms exact {okw}", flush=True)
