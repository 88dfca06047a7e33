"""Shared fixtures.  The oracle (oracle/) is loaded ONLY here, as the checker."""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


def _ensure_built():
    need = [os.path.join(ROOT, "pomegranate_amd", "liblzo_mi355x.so"),
            os.path.join(ROOT, "pomegranate_amd", "libpom_synth.so"),
            os.path.join(ROOT, "oracle", "liboracle.so"),
            os.path.join(ROOT, "tests", "native", "libsplit_mock.so")]
    if not all(os.path.exists(p) for p in need):
        import __graft_entry__
        __graft_entry__.build()


_ensure_built()


@pytest.fixture(autouse=True)
def _debug_keys_follow_env():
    """The library reads POM_LZO_DEBUG once (lzo_host.c); tests that set it
    (monkeypatch) get it re-read before and after them."""
    from pomegranate_amd import lzo
    lib = lzo.load()
    lib.lzo_mi355x_debug_reload()
    yield
    lib.lzo_mi355x_debug_reload()


class Oracle:
    """ctypes view of oracle/liboracle.so (the CPU restatement)."""

    def __init__(self):
        self.lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
        self.lib.oracle_lzo1x_1_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t,
                                                     ctypes.c_void_p,
                                                     ctypes.POINTER(ctypes.c_size_t)]
        for fn in ("oracle_lzo1x_decompress_safe", "oracle_lzo1x_decompress_unchecked"):
            getattr(self.lib, fn).argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                              ctypes.POINTER(ctypes.c_size_t)]

    def compress(self, data: bytes) -> bytes:
        n = len(data)
        src = ctypes.create_string_buffer(data, max(n, 1))
        out = ctypes.create_string_buffer(n + n // 16 + 67)
        ol = ctypes.c_size_t(0)
        self.lib.oracle_lzo1x_1_compress(src, n, out, ctypes.byref(ol))
        return out.raw[: ol.value]

    def decompress_safe(self, comp: bytes, cap: int):
        src = ctypes.create_string_buffer(comp, max(len(comp), 1))
        out = ctypes.create_string_buffer(max(cap, 1))
        ol = ctypes.c_size_t(cap)
        rc = self.lib.oracle_lzo1x_decompress_safe(src, len(comp), out, ctypes.byref(ol))
        return rc, out.raw[: ol.value]

    def decompress_unchecked(self, comp: bytes, room: int = 1 << 22):
        """lzo1x_decompress semantics (no input checks; room = output buffer)."""
        src = ctypes.create_string_buffer(comp, max(len(comp), 1))
        out = ctypes.create_string_buffer(max(room, 1))
        ol = ctypes.c_size_t(room)
        rc = self.lib.oracle_lzo1x_decompress_unchecked(src, len(comp), out, ctypes.byref(ol))
        return rc, out.raw[: ol.value]


@pytest.fixture(scope="session")
def oracle():
    return Oracle()


@pytest.fixture(scope="session")
def ref_lib():
    """The reference's own lib/minilzo.c, compiled in place (absent on the GPU box)."""
    path = os.path.join(ROOT, "oracle", "_ref", "libminilzo_ref.so")
    if not os.path.exists(path):
        pytest.skip("oracle/_ref not built here")
    from tests.golden.make_golden import Ref
    return Ref(path)


def _unpack(data, off):
    return [data[off[i]: off[i + 1]].tobytes() for i in range(len(off) - 1)]


@pytest.fixture(scope="session")
def edge():
    z = np.load(os.path.join(GOLDEN, "edge.npz"))
    return {"names": [str(s) for s in z["names"]],
            "inputs": _unpack(z["in_data"], z["in_off"]),
            "comps": _unpack(z["z_data"], z["z_off"])}


@pytest.fixture(scope="session")
def malformed():
    z = np.load(os.path.join(GOLDEN, "malformed.npz"))
    return {"streams": _unpack(z["s_data"], z["s_off"]), "caps": [int(c) for c in z["cap"]],
            "rc": [int(r) for r in z["rc"]], "outs": _unpack(z["out_data"], z["out_off"])}


@pytest.fixture(scope="session")
def unchecked():
    """The reference's UNCHECKED lzo1x_decompress on valid, trailing-byte,
    concatenated and EOF-cut streams (tests/golden/make_golden.py)."""
    z = np.load(os.path.join(GOLDEN, "unchecked.npz"))
    return {"kinds": [str(k) for k in z["kind"]], "streams": _unpack(z["s_data"], z["s_off"]),
            "rc": [int(r) for r in z["rc"]], "out_len": [int(n) for n in z["out_len"]],
            "sha": [str(h) for h in z["out_sha256"]]}


@pytest.fixture(scope="session")
def fwritev_columns():
    """Columns as the reference's hvfs_fwritev writes them (api/api.c:6652-6689):
    [u64 length] + one reference lzo1x_1_compress stream per iovec, with what
    the reference's read side returns on them (tests/golden/make_golden.py)."""
    z = np.load(os.path.join(GOLDEN, "column.npz"))
    n_iov = [int(n) for n in z["n_iov"]]
    flat = [int(n) for n in z["iov_len"]]
    sizes, at = [], 0
    for n in n_iov:
        sizes.append(flat[at: at + n])
        at += n
    return {"names": [str(s) for s in z["names"]], "iov_len": sizes,
            "data": _unpack(z["data"], z["data_off"]), "zips": _unpack(z["z_data"], z["z_off"]),
            "read_rc": [int(r) for r in z["read_rc"]],
            "read_len": [int(n) for n in z["read_len"]]}


@pytest.fixture(scope="session")
def longext():
    """Streams with one length extension of 16,843,008-16,843,010 zero bytes
    (255 per zero passes 2^32) and what the reference's lzo1x_decompress_safe
    returns on them (tests/golden/make_golden.py longext_cases); the streams
    are rebuilt from the spec."""
    from tests.golden.make_golden import longext_stream
    with open(os.path.join(GOLDEN, "longext.json")) as f:
        cases = json.load(f)["cases"]
    return [dict(c, stream=longext_stream(c["kind"], c["zeros"])) for c in cases]


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)["batches"]


def batch_sizes(entry):
    s = entry["sizes"]
    return s if isinstance(s, list) else [s] * entry["nblocks"]
