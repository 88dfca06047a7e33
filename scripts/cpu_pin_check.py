"""CPU baseline placement check (GPU box): the native harness oracle/cpu_bench on
512 ITB blocks at 1 and 16 threads, pinned to the first CPUs of the affinity
set, spread over it, and not pinned.  Prints one line per run."""
import ctypes, json, os, struct, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pomegranate_amd import synth
lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libminilzo_ref.so"))
lib.lzo1x_1_compress.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p,
                                 ctypes.POINTER(ctypes.c_ulong), ctypes.c_void_p]
getattr(lib, "__lzo_init_v2")(0x2040, 2, 4, 8, 4, 8, 8, 8, 8, 48)
wrk = ctypes.create_string_buffer(131072)
z = ctypes.create_string_buffer(70000)
path = "/dev/shm/pom_pin_sample.bin"
with open(path, "wb") as f:
    f.write(struct.pack("<I", 512))
    for b in range(512):
        d = synth.block(synth.ITB, b, 65536)
        zl = ctypes.c_ulong(0)
        ctypes.memset(wrk, 0, 131072)
        lib.lzo1x_1_compress(d, len(d), z, ctypes.byref(zl), wrk)
        f.write(struct.pack("<II", len(d), zl.value)); f.write(d); f.write(z.raw[:zl.value])
secs = sys.argv[1] if len(sys.argv) > 1 else "4"
for threads in (1, 16):
    for pin in ("1", "spread", "0"):
        r = subprocess.run([os.path.join(ROOT, "oracle", "cpu_bench"), os.path.join(ROOT, "oracle", "_ref", "libminilzo_ref.so"),
                            path, str(threads), secs, pin], capture_output=True, text=True)
        j = json.loads(r.stdout)
        print(json.dumps({"threads": threads, "pin": pin, "compress_GiBps": round(j["compress_Bps"] / 2**30, 3),
                          "decompress_GiBps": round(j["decompress_Bps"] / 2**30, 3), "cpus": j["cpus"][:16]}), flush=True)
os.unlink(path)
