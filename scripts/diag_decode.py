"""Diagnostic: phase breakdown of the fast decoder (s_memtime stamps build).
Usage: python scripts/diag_decode.py [--blocks N] [--model itb]"""
import argparse, ctypes, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from pomegranate_amd import lzo, synth

ap = argparse.ArgumentParser()
ap.add_argument("--blocks", type=int, default=4096)
ap.add_argument("--model", default="itb")
ap.add_argument("--bytes", type=int, default=65536)
ap.add_argument("--lib", default=None, help="alternative liblzo_mi355x.so build")
ap.add_argument("--nostamps", action="store_true", help="timing only (no stamps build run)")
a = ap.parse_args()
if a.lib:
    lzo.LIB_PATH = a.lib
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
lib = lzo.load()
model = {v: k for k, v in synth.MODEL_NAMES.items()}[a.model]
arena, offs, lens = synth.batch(model, 0, [a.bytes] * a.blocks, threads=16)
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
nb = a.blocks
src = lzo.DeviceBatch(t(arena), t(offs.view(np.int64)), t(lens.view(np.int32)))
caps = np.array([lzo.worst_compress(int(n)) for n in lens], dtype=np.uint32)
zo = np.zeros(nb, dtype=np.uint64); zo[1:] = np.cumsum((caps[:-1].astype(np.uint64) + 255) // 256 * 256)
za = torch.zeros(int(zo[-1]) + int(caps[-1]) + 256, dtype=torch.uint8, device=dev)
zb = lzo.DeviceBatch(za, t(zo.view(np.int64)), t(caps.view(np.int32)))
zl = torch.zeros(nb, dtype=torch.int32, device=dev); zs = torch.zeros_like(zl)
lzo.compress_dev(src, zb, zl, zs); torch.cuda.synchronize()
zsrc = lzo.DeviceBatch(za, zb.off, zl)
out = torch.zeros_like(src.arena); ob = lzo.DeviceBatch(out, src.off, src.length)
ol = torch.zeros_like(zl); os_ = torch.zeros_like(zl)
head = torch.zeros(64 + 2048, dtype=torch.int32, device=dev)   # fallback count, op-set pool
fb = head[:1]
ids = torch.zeros(nb, dtype=torch.int32, device=dev)
lib.lzo_mi355x_fast_resident_blocks.restype = ctypes.c_uint32
nsets = min(nb, int(lib.lzo_mi355x_fast_resident_blocks()))
ring = torch.zeros(nsets, dtype=torch.int64, device=dev)
lib.lzo_mi355x_fast_ops_bytes_per_block.restype = ctypes.c_size_t
opsbuf = torch.empty(nsets * lib.lzo_mi355x_fast_ops_bytes_per_block(), dtype=torch.uint8, device=dev)
SLOTS = 40
stamps = torch.zeros(nb * SLOTS, dtype=torch.int64, device=dev)
fn = lib.lzo_mi355x_debug_decompress_fast_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p] * 13 + [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
fast = lib.lzo_mi355x_launch_decompress_fast
fast.restype = ctypes.c_int
fast.argtypes = [ctypes.c_void_p] * 13 + [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
p = lambda x: x.data_ptr()
sh = torch.cuda.current_stream().cuda_stream
def run(stamp):
    head.zero_(); ring.zero_()
    args = (p(zsrc.arena), p(zsrc.off), p(zsrc.length), p(out), p(ob.off), p(ob.length), p(ol), p(os_),
            p(head), p(ids), p(head) + 256, p(ring), p(opsbuf), nsets, nb)
    if stamp:
        fn(*args, p(stamps), sh)
    else:
        fast(*args, None, sh)
for stamp in ((False,) if a.nostamps else (False, True)):
    run(stamp); torch.cuda.synchronize()
    ts = []
    for _ in range(1 if stamp else 10):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(); run(stamp); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(f"stamps={stamp}: kernel {float(np.median(ts)):.3f} ms (median of {len(ts)}, min {min(ts):.3f}), "
          f"fallback {int(fb[0].item())}, equal {torch.equal(out, src.arena)}")
    if not stamp and int(fb[0].item()):
        olr = ol.cpu().numpy().astype(np.uint32)
        fbb = np.nonzero((olr >> 16) == 0xFA11)[0]
        print("  fast-path refusals (block, reason):", [(int(x), int(olr[x] & 15)) for x in fbb[:8]])
        per = opsbuf.numel() // nsets   # (op-set contents; the set a block used is not recorded)
        for x in fbb[:4]:
            blk = opsbuf[int(x) * per: (int(x) + 1) * per].cpu().numpy()
            zs_ = za[int(zb.off[int(x)].item()): int(zb.off[int(x)].item()) + int(zl[int(x)].item())].cpu().numpy()
            np.savez(os.path.join(ROOT, "gpurun_out", f"dead_b{int(x)}.npz"), ops=blk, z=zs_)
if a.nostamps:
    sys.exit(0)
st = stamps.view(nb, SLOTS).double().cpu().numpy()
# order of the kernel's PH_* / CN_* enum (lzo1x_decode_fast.hip)
phases = ["stage", "pass1", "pwalk", "merge", "count", "write", "p_slotwait", "p_duty",
          "e_wait", "wload", "wscan", "src_issue", "fwd", "src_commit+wop", "batch",
          "space", "flags", "gather", "publish"]
counts = ["walks", "it_pass1", "it_pwalk", "it_walk", "it_count", "it_write", "pieces",
          "windows", "src_windows", "src_miss", "batches", "steps", "fwd_rounds", "wide_batches", "narrow_gop",
          "narrow_period", "reason"]
PARSER = 8   # phases [0, 8) belong to the parser wave, the rest to the executor
ptot = st[:, :PARSER].sum(1); etot = st[:, PARSER:len(phases)].sum(1)
print("parser cycles/block (mean):", {n: int(st[:, i].mean()) for i, n in enumerate(phases[:PARSER])},
      "total", int(ptot.mean()))
print("executor cycles/block (mean):", {n: int(st[:, PARSER + i].mean()) for i, n in enumerate(phases[PARSER:])},
      "total", int(etot.mean()))
print("counts/block (mean):", {n: round(float(st[:, len(phases) + i].mean()), 1)
                               for i, n in enumerate(counts)})
print("zlen mean", float(zl.double().mean()))
rsf = stamps.view(nb, SLOTS)[:, len(phases) + counts.index("reason")].cpu().numpy()
rs = (rsf & 15).astype(int)
for b in np.nonzero(rs)[0][:4]:
    q, w0 = int((rsf[b] >> 4) & 0xFFFFFFF), int(rsf[b] >> 32)
    per = opsbuf.numel() // nsets   # (op-set contents; the set a block used is not recorded)
    slot = opsbuf[b * per: (b + 1) * per].view(torch.int32).view(-1, 2).cpu().numpy()
    kslots = 8
    ops_q = slot[(q % kslots) * (len(slot) // kslots): (q % kslots + 1) * (len(slot) // kslots)]
    np.save(os.path.join(ROOT, "gpurun_out", f"refused_b{b}_q{q}.npy"), ops_q)
    print("refused block", int(b), "reason", int(rs[b]), "piece", q, "window", w0)
names = ["none", "off_end", "bad", "ops", "dead", "ewait", "overrun", "lookbehind", "space", "landed", "head",
         "writer"]
print("refusals:", {names[r]: int((rs == r).sum()) for r in np.unique(rs) if r})
