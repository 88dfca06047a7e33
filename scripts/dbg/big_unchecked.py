import os, sys, ctypes
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
from pomegranate_amd import lzo, synth
lib = lzo.load()
for n in (65536, 262144, 262145, 300000, 536192):
    d = bytearray(n)
    for i in range(3712, n - 16, 512):
        d[i:i + 8] = (i * 2654435761 % (1 << 64)).to_bytes(8, "little")
    d = bytes(d)
    rc, z = lzo.lzo1x_1_compress(d)
    src = ctypes.create_string_buffer(z, len(z))
    out = ctypes.create_string_buffer(n + 64)
    olen = ctypes.c_ulong(0)
    rc2 = lib.lzo1x_decompress(src, len(z), out, ctypes.byref(olen), None)
    got = out.raw[:olen.value]
    bad = next((i for i in range(min(len(got), n)) if got[i] != d[i]), None)
    print(n, "z", len(z), "rc", rc, rc2, "olen", olen.value, "first diff", bad, flush=True)
