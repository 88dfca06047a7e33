"""CPU: the drop-in C-ABI library loads and exports every function include/*.h
declares; the reference call sites compile against include/minilzo.h; without
a GPU the codec refuses loudly (no CPU fallback)."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT
from pomegranate_amd import lzo

INCLUDE = os.path.join(ROOT, "include")


def declared_functions():
    """Function prototypes of include/*.h, via gcc -aux-info."""
    names = set()
    for hdr in sorted(os.listdir(INCLUDE)):
        if not hdr.endswith(".h"):
            continue
        aux = f"/tmp/pom_aux_{os.getpid()}_{hdr}.txt"
        subprocess.run(["gcc", "-fsyntax-only", "-x", "c", f"-aux-info={aux}",
                        os.path.join(INCLUDE, hdr)], check=True)
        with open(aux) as f:
            for line in f:
                if f"/include/{hdr}:" not in line:
                    continue
                m = re.search(r"\*/\s*(?:extern\s+)?[^;(]*?\b(\w+)\s*\(", line)
                if m:
                    names.add(m.group(1))
        os.unlink(aux)
    return names


def test_headers_declare_exactly_the_exports():
    assert declared_functions() == set(lzo.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(lzo.LIB_PATH)
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", lzo.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    defined = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert declared_functions() <= defined


def test_library_has_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readobj", "--sections", lzo.LIB_PATH],
                         capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip("llvm-readobj unavailable")
    assert ".hip_fatbin" in out.stdout
    blob = open(lzo.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_no_oracle_in_product_library():
    """The product library never links or names the oracle (no CPU fallback)."""
    blob = open(lzo.LIB_PATH, "rb").read()
    assert b"oracle" not in blob
    out = subprocess.run(["ldd", lzo.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out and "minilzo_ref" not in out


def test_constants_match_reference_values():
    assert lzo.LZO1X_1_MEM_COMPRESS == 131072
    assert lzo.worst_compress(65536) == lzo.load().lzo_mi355x_worst_compress(65536)
    lib = lzo.load()
    assert lib.lzo_version() == 0x2040
    assert lib.lzo_version_string() == b"2.04"
    for name in ("_lzo_version_string", "_lzo_version_date", "lzo_version_date"):
        getattr(lib, name).restype = ctypes.c_char_p
    assert lib._lzo_version_string() == b"2.04"
    assert lib._lzo_version_date() == lib.lzo_version_date() == b"Oct 31 2010"
    assert lib._lzo_config_check() == 0
    # the header's macros, evaluated by the C compiler (lib/minilzo.h:79-81)
    src = (f'#include "minilzo.h"\n#include <stdio.h>\nint main(void){{char b[64];'
           f'printf("%lu %lu %d %lu\\n",(unsigned long)LZO1X_MEM_COMPRESS,'
           f'(unsigned long)LZO1X_1_MEM_COMPRESS,LZO1X_MEM_DECOMPRESS,'
           f'(unsigned long)(LZO_PTR_ALIGN_UP(b+1,16)-b));return 0;}}')
    exe = f"/tmp/pom_consts_{os.getpid()}"
    subprocess.run(["gcc", "-x", "c", "-", f"-I{INCLUDE}", f"-L{os.path.dirname(lzo.LIB_PATH)}",
                    "-llzo_mi355x", f"-Wl,-rpath,{os.path.dirname(lzo.LIB_PATH)}", "-o", exe],
                   input=src, text=True, check=True)
    out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()
    os.unlink(exe)
    assert out[:3] == ["131072", "131072", "0"]
    assert int(out[3]) % 16 == 0 and 1 <= int(out[3]) <= 16


REF_LIB = os.path.join(ROOT, "oracle", "_ref", "libminilzo_ref.so")


def test_exports_cover_reference_minilzo():
    """Every function the reference's lib/minilzo.c exports is exported here
    too (the list is what `nm -D` shows for oracle/_ref, the reference compiled
    in place; fixed below for boxes without it)."""
    ref = {"__lzo_align_gap", "__lzo_init_v2", "__lzo_ptr_linear", "_lzo_config_check",
           "_lzo_version_date", "_lzo_version_string", "lzo1x_1_compress", "lzo1x_decompress",
           "lzo1x_decompress_safe", "lzo_adler32", "lzo_copyright", "lzo_memcmp", "lzo_memcpy",
           "lzo_memmove", "lzo_memset", "lzo_version", "lzo_version_date", "lzo_version_string"}
    if os.path.exists(REF_LIB):
        out = subprocess.run(["nm", "-D", "--defined-only", REF_LIB], capture_output=True,
                             text=True, check=True).stdout
        assert {ln.split()[-1] for ln in out.splitlines() if " T " in ln} == ref
    assert ref <= set(lzo.EXPORTS)


def test_host_utilities_match_reference():
    """lzo_adler32 / lzo_memcmp / __lzo_align_gap against zlib's Adler-32 and,
    when present, the reference's own functions (oracle/_ref)."""
    import random
    import zlib
    lib = lzo.load()
    lib.lzo_adler32.restype = ctypes.c_uint32
    lib.lzo_adler32.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_ulong]
    ref = None
    if os.path.exists(REF_LIB):
        ref = ctypes.CDLL(REF_LIB)
        ref.lzo_adler32.restype = ctypes.c_uint32
        ref.lzo_adler32.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_ulong]
    rng = random.Random(6)
    for n in (0, 1, 15, 16, 17, 5551, 5552, 5553, 65536, 200003):
        data = bytes([255] * n) if n % 2 else bytes(rng.getrandbits(8) for _ in range(n))
        for seed in (1, 0x12345678):
            got = lib.lzo_adler32(seed, data, n)
            assert got == zlib.adler32(data, seed), (n, seed)
            if ref is not None:
                assert got == ref.lzo_adler32(seed, data, n), (n, seed)
    assert lib.lzo_adler32(7, None, 5) == 1
    lib.lzo_memcmp.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong]
    assert lib.lzo_memcmp(b"abc", b"abd", 3) < 0 and lib.lzo_memcmp(b"abc", b"abd", 2) == 0
    lib.__lzo_align_gap.argtypes = [ctypes.c_void_p, ctypes.c_ulong]
    lib.__lzo_align_gap.restype = ctypes.c_uint
    for p, size in ((4096, 16), (4097, 16), (4111, 8), (12, 1)):
        assert lib.__lzo_align_gap(p, size) == (-p) % size


def _build_callsite():
    exe = f"/tmp/pom_itb_callsite_{os.getpid()}"
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", f"-I{INCLUDE}",
                    os.path.join(ROOT, "tests", "c", "itb_callsite.c"),
                    f"-L{os.path.dirname(lzo.LIB_PATH)}", "-llzo_mi355x",
                    f"-Wl,-rpath,{os.path.dirname(lzo.LIB_PATH)}", "-o", exe], check=True)
    return exe


def test_reference_call_sites_compile_against_header():
    exe = _build_callsite()
    assert os.path.exists(exe)
    os.unlink(exe)


def _gpu_present():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.mark.skipif(_gpu_present(), reason="checks the no-GPU refusal")
def test_no_gpu_fails_loudly():
    exe = _build_callsite()
    r = subprocess.run([exe], capture_output=True, text=True)
    os.unlink(exe)
    assert r.returncode == 2
    assert "no usable GPU" in r.stderr
    assert lzo.lzo_init() == lzo.LZO_E_ERROR
    assert lzo.lzo1x_1_compress(b"abc")[0] == lzo.LZO_E_ERROR


@pytest.mark.gpu
@pytest.mark.skipif(not _gpu_present(), reason="needs a GPU")
def test_reference_call_sites_round_trip_on_gpu():
    exe = _build_callsite()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    os.unlink(exe)
    assert r.returncode == 0, r.stderr
    assert "column data ok" in r.stdout
