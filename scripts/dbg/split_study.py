# driver for split_study.c: gcc -O2 -shared -fPIC -o /tmp/split_study.so scripts/dbg/split_study.c
import ctypes, sys
sys.path.insert(0, '/root/repo')
from pomegranate_amd import synth
m = ctypes.CDLL('/tmp/split_study.so')
for model in (synth.ITB, synth.TEXT, synth.LZLIKE):
    for D in (0xC000, 0xC000 + 1024, 0xC000 + 8192):
        tot = [0, 0, 0]
        for seed in range(3):
            data = synth.block(model, 500 + seed, 536192)
            o = (ctypes.c_long * 4)()
            m.study(data, len(data), ctypes.c_size_t(65536), ctypes.c_size_t(D), o)
            tot[0] += o[0]; tot[1] += o[1]; tot[2] += o[2]
        print(synth.MODEL_NAMES[model], "D", D, "verified", tot[0], "/", tot[1], "mean sync offset", tot[2] // 3)
