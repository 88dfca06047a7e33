"""Python mirror of Pomegranate's LZO1X call surface, bound to liblzo_mi355x.so.

The reference calls three C functions (finding 2):
``lzo_init`` (lib/lzoconf.h:331-335), ``lzo1x_1_compress``
(lib/minilzo.c:3159-3207) and ``lzo1x_decompress`` (lib/minilzo.c:3308-3699);
``lzo1x_decompress_safe`` (lib/minilzo.c:3703-4190) is also exported.  The
functions below keep those names, argument meanings and ``LZO_E_*`` return
codes, and call the C-ABI of ``include/minilzo.h`` / ``include/lzo_mi355x.h``
directly -- every byte of coding happens in the HIP kernels.  There is no
Python or CPU codec here: if the library cannot be loaded an ImportError-like
``RuntimeError`` is raised, and without a GPU every call returns LZO_E_ERROR.

Device-resident batches (the path the benchmark measures) take torch tensors
already in HBM and enqueue on the current HIP stream.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblzo_mi355x.so")
SYNTH_PATH = os.path.join(_HERE, "libpom_synth.so")

LZO_E_OK = 0
LZO_E_ERROR = -1
LZO_E_OUT_OF_MEMORY = -2
LZO_E_NOT_COMPRESSIBLE = -3
LZO_E_INPUT_OVERRUN = -4
LZO_E_OUTPUT_OVERRUN = -5
LZO_E_LOOKBEHIND_OVERRUN = -6
LZO_E_EOF_NOT_FOUND = -7
LZO_E_INPUT_NOT_CONSUMED = -8

LZO1X_1_MEM_COMPRESS = 16384 * 8          # lib/minilzo.h:80 on LP64
LZO_VERSION = 0x2040

# Exported symbols, exactly those declared in include/*.h.
EXPORTS = (
    "__lzo_init_v2", "lzo_version", "lzo_version_string", "lzo_version_date",
    "_lzo_version_string", "_lzo_version_date", "lzo_copyright",
    "lzo_memcmp", "lzo_memcpy", "lzo_memmove", "lzo_memset", "lzo_adler32",
    "_lzo_config_check", "__lzo_ptr_linear", "__lzo_align_gap",
    "lzo1x_1_compress", "lzo1x_decompress", "lzo1x_decompress_safe",
    "lzo_mi355x_worst_compress", "lzo_mi355x_device_count", "lzo_mi355x_debug_reload",
    "lzo_mi355x_decoded_length",
    "lzo_mi355x_compress_dev", "lzo_mi355x_decompress_dev",
    "lzo_mi355x_decompress_scratch", "lzo_mi355x_decompress_fallbacks", "lzo_mi355x_decoded_length_dev",
    "lzo_mi355x_compress_scratch",
    "lzo_mi355x_compress_batch", "lzo_mi355x_decompress_batch",
    "lzo_mi355x_decompress_concat_batch",
    # include/pom_itb.h
    "pom_itb_lzo_compress_batch", "pom_itb_lzo_compress_append_batch", "pom_itb_lzo_decompress_batch",
    "pom_abuf_open", "pom_abuf_append", "pom_abuf_append_batch", "pom_abuf_close", "pom_itb_read",
    "pom_itb_read_batch", "pom_itb_read_lzo_decompress_batch",
    # include/pom_column.h
    "pom_col_zip_bound", "pom_col_zip_batch", "pom_col_zipv", "pom_col_unzip_batch",
    # include/pom_xnet.h
    "pom_xnet_frame", "pom_xnet_parse", "pom_xnet_itb_reply_batch", "pom_xnet_itb_wb_batch",
    "pom_xnet_itb_recv_batch",
)

_lib: Optional[ctypes.CDLL] = None
_synth: Optional[ctypes.CDLL] = None

_u8p = ctypes.c_void_p
_ulong = ctypes.c_ulong
_size = ctypes.c_size_t


def debug_reload() -> None:
    """Have the library re-read POM_LZO_DEBUG (it reads it once; see
    include/lzo_mi355x.h lzo_mi355x_debug_reload)."""
    load().lzo_mi355x_debug_reload()


def load() -> ctypes.CDLL:
    """Load liblzo_mi355x.so (built in-tree by __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: run __graft_entry__.build(); the LZO1X "
            "path has no CPU fallback")
    # torch bundles its own HIP runtime.  Loading it first lets this library
    # bind to that same libamdhip64 (by soname); loaded the other way round the
    # process holds two HIP runtimes, and the one initialised second sees no
    # GPU (hipGetDeviceCount = 0 on the GPU box).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    lib.__lzo_init_v2.restype = ctypes.c_int
    lib.__lzo_init_v2.argtypes = [ctypes.c_uint] + [ctypes.c_int] * 9
    for name in ("lzo1x_1_compress", "lzo1x_decompress", "lzo1x_decompress_safe"):
        fn = getattr(lib, name)
        fn.restype = ctypes.c_int
        fn.argtypes = [_u8p, _ulong, _u8p, ctypes.POINTER(_ulong), _u8p]
    lib.lzo_version.restype = ctypes.c_uint
    lib.lzo_version_string.restype = ctypes.c_char_p
    lib.lzo_version_date.restype = ctypes.c_char_p
    lib.lzo_mi355x_decoded_length.restype = ctypes.c_int
    lib.lzo_mi355x_decoded_length.argtypes = [_u8p, _ulong, ctypes.POINTER(_ulong)]
    lib.lzo_mi355x_worst_compress.restype = _size
    lib.lzo_mi355x_worst_compress.argtypes = [_size]
    lib.lzo_mi355x_device_count.restype = ctypes.c_int
    dev_args = [_u8p, _u8p, _u8p, _u8p, _u8p, _u8p, _u8p, _u8p, ctypes.c_uint32]
    lib.lzo_mi355x_compress_dev.restype = ctypes.c_int
    lib.lzo_mi355x_compress_dev.argtypes = dev_args + [_u8p, _u8p]
    lib.lzo_mi355x_compress_scratch.restype = _size
    lib.lzo_mi355x_compress_scratch.argtypes = [ctypes.c_uint32]
    lib.lzo_mi355x_decompress_dev.restype = ctypes.c_int
    lib.lzo_mi355x_decompress_dev.argtypes = dev_args + [_u8p, _u8p]
    lib.lzo_mi355x_decompress_scratch.restype = _size
    lib.lzo_mi355x_decompress_scratch.argtypes = [ctypes.c_uint32]
    lib.lzo_mi355x_decompress_fallbacks.restype = ctypes.c_int
    lib.lzo_mi355x_decompress_fallbacks.argtypes = [_u8p, ctypes.POINTER(ctypes.c_uint32), _u8p]
    lib.lzo_mi355x_decoded_length_dev.restype = ctypes.c_int
    lib.lzo_mi355x_decoded_length_dev.argtypes = [_u8p] * 5 + [ctypes.c_uint32, _u8p]
    for name in ("lzo_mi355x_compress_batch", "lzo_mi355x_decompress_batch",
                 "lzo_mi355x_decompress_concat_batch"):
        fn = getattr(lib, name)
        fn.restype = ctypes.c_int
        fn.argtypes = [_u8p, _u8p, _u8p, _u8p, _u8p, _size]
    _lib = lib
    return lib


def worst_compress(n: int) -> int:
    return n + n // 16 + 64 + 3


# ---------------------------------------------------------------------------
# The reference's call surface
# ---------------------------------------------------------------------------
def lzo_init() -> int:
    """lzo_init() macro of lib/lzoconf.h:331-335 with LP64 type sizes."""
    return load().__lzo_init_v2(LZO_VERSION, 2, 4, 8, 4, 8, 8, 8, 8, 48)


def lzo1x_1_compress(src: bytes, wrkmem: Optional[bytearray] = None) -> Tuple[int, bytes]:
    """lzo1x_1_compress(src, len, dst, &dst_len, wrkmem) -> (rc, dst[:dst_len])."""
    lib = load()
    n = len(src)
    out = ctypes.create_string_buffer(worst_compress(n))
    olen = _ulong(0)
    rc = lib.lzo1x_1_compress(_bytes_ptr(src), n, out, ctypes.byref(olen), None)
    return rc, out.raw[: olen.value] if rc == LZO_E_OK else b""


def lzo1x_decompress(src: bytes) -> Tuple[int, bytes]:
    """Unchecked decoder: *dst_len is ignored on input (lib/minilzo.c:3326).

    Like every reference caller, the destination is sized by the caller; here
    it is sized from the GPU's decoded-length pre-scan
    (lzo_mi355x_decoded_length), then lzo1x_decompress fills it.
    """
    lib = load()
    need = _ulong(0)
    rc = lib.lzo_mi355x_decoded_length(_bytes_ptr(src), len(src), ctypes.byref(need))
    if rc == LZO_E_ERROR:
        return rc, b""
    buf = ctypes.create_string_buffer(max(need.value, 1))
    olen = _ulong(0)
    rc = lib.lzo1x_decompress(_bytes_ptr(src), len(src), buf, ctypes.byref(olen), None)
    return rc, buf.raw[: olen.value]


def lzo1x_decompress_safe(src: bytes, dst_cap: int) -> Tuple[int, bytes]:
    """lzo1x_decompress_safe with capacity dst_cap -> (rc, produced bytes)."""
    lib = load()
    out = ctypes.create_string_buffer(max(dst_cap, 1))
    olen = _ulong(dst_cap)
    rc = lib.lzo1x_decompress_safe(_bytes_ptr(src), len(src), out, ctypes.byref(olen), None)
    return rc, out.raw[: olen.value]


def _bytes_ptr(b: bytes):
    # ctypes passes bytes as a read-only char*; the library never writes src.
    return ctypes.c_char_p(b) if len(b) else ctypes.c_char_p(b"\0")


# ---------------------------------------------------------------------------
# Host-resident batches (pinned staging + hipMemcpyAsync inside the library)
# ---------------------------------------------------------------------------
def _ptr_array(bufs):
    arr = (ctypes.c_void_p * len(bufs))()
    for i, b in enumerate(bufs):
        arr[i] = ctypes.cast(b, ctypes.c_void_p).value
    return arr


def compress_batch(blocks: Sequence[bytes]) -> Tuple[int, List[int], List[bytes]]:
    lib = load()
    nb = len(blocks)
    srcs = [ctypes.create_string_buffer(bytes(b), max(len(b), 1)) for b in blocks]
    dsts = [ctypes.create_string_buffer(worst_compress(len(b))) for b in blocks]
    slen = (_size * nb)(*[len(b) for b in blocks])
    dlen = (_size * nb)()
    st = (ctypes.c_int * nb)()
    rc = lib.lzo_mi355x_compress_batch(_ptr_array(srcs), slen, _ptr_array(dsts), dlen, st, nb)
    return rc, list(st), [dsts[i].raw[: dlen[i]] for i in range(nb)]


def decompress_batch(blocks: Sequence[bytes], caps: Sequence[int], concat: bool = False
                     ) -> Tuple[int, List[int], List[bytes]]:
    """concat: blocks of consecutive streams (lzo_mi355x_decompress_concat_batch)."""
    lib = load()
    nb = len(blocks)
    srcs = [ctypes.create_string_buffer(bytes(b), max(len(b), 1)) for b in blocks]
    dsts = [ctypes.create_string_buffer(max(c, 1)) for c in caps]
    slen = (_size * nb)(*[len(b) for b in blocks])
    dlen = (_size * nb)(*caps)
    st = (ctypes.c_int * nb)()
    fn = lib.lzo_mi355x_decompress_concat_batch if concat else lib.lzo_mi355x_decompress_batch
    rc = fn(_ptr_array(srcs), slen, _ptr_array(dsts), dlen, st, nb)
    return rc, list(st), [dsts[i].raw[: min(dlen[i], caps[i])] for i in range(nb)]


# ---------------------------------------------------------------------------
# Device-resident batches (torch tensors in HBM; torch is plumbing only)
# ---------------------------------------------------------------------------
@dataclass
class DeviceBatch:
    """SoA batch descriptor in HBM: block b = arena[off[b] : off[b] + len[b]]."""
    arena: "object"      # torch.uint8 tensor on the GPU
    off: "object"        # torch.int64 (used as uint64)
    length: "object"     # torch.int32 (used as uint32)

    @property
    def nblocks(self) -> int:
        return int(self.off.numel())


def _ptr(t) -> int:
    return int(t.data_ptr())


def _stream_handle(torch, stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def compress_dev(src: DeviceBatch, dst: DeviceBatch, out_len, status, stream=None, *,
                 scratch="auto") -> None:
    """Enqueue LZO1X-1 compression of every block of src into dst (dst.length = capacity).

    stream: the HIP stream (torch.cuda.Stream) to enqueue on; default the current one.
    scratch (keyword only): device tensor of compress_scratch_bytes(nblocks) bytes
    for the per-workgroup match dictionaries (16 blocks per CU parse at once),
    None for LDS dictionaries (4 per CU), or "auto" to allocate one for this
    call.  An "auto" tensor is allocated on, and recorded against, the stream
    the kernel runs on, so the caching allocator cannot hand its memory to
    another tensor while the encoder still uses it."""
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    if isinstance(scratch, str):
        if scratch != "auto":
            raise ValueError(f"scratch: a tensor, None or 'auto', not {scratch!r}")
        nbytes = compress_scratch_bytes(src.nblocks)
        with torch.cuda.stream(s):
            scratch = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=src.arena.device)
        scratch.record_stream(s)
    rc = load().lzo_mi355x_compress_dev(
        _ptr(src.arena), _ptr(src.off), _ptr(src.length), _ptr(dst.arena), _ptr(dst.off),
        _ptr(dst.length), _ptr(out_len), _ptr(status), src.nblocks,
        _ptr(scratch) if scratch is not None else None, int(s.cuda_stream))
    if rc != 0:
        raise RuntimeError("lzo_mi355x_compress_dev launch failed")


def compress_scratch_bytes(nblocks: int) -> int:
    return int(load().lzo_mi355x_compress_scratch(nblocks))


def decompress_dev(src: DeviceBatch, dst: DeviceBatch, out_len, status, scratch=None,
                   stream=None) -> None:
    """Enqueue LZO1X decompression (safe semantics, capacity dst.length)."""
    import torch
    scr = _ptr(scratch) if scratch is not None else None
    rc = load().lzo_mi355x_decompress_dev(
        _ptr(src.arena), _ptr(src.off), _ptr(src.length), _ptr(dst.arena), _ptr(dst.off),
        _ptr(dst.length), _ptr(out_len), _ptr(status), src.nblocks, scr,
        _stream_handle(torch, stream))
    if rc != 0:
        raise RuntimeError("lzo_mi355x_decompress_dev launch failed")


def decompress_fallbacks(scratch, stream=None) -> int:
    """Blocks the last decompress_dev() on `scratch` handed to the exact decoder
    (waits for `stream`)."""
    import torch
    n = ctypes.c_uint32(0)
    rc = load().lzo_mi355x_decompress_fallbacks(_ptr(scratch), ctypes.byref(n),
                                                _stream_handle(torch, stream))
    if rc != 0:
        raise RuntimeError("lzo_mi355x_decompress_fallbacks failed")
    return int(n.value)


def decompress_scratch_bytes(nblocks: int) -> int:
    return int(load().lzo_mi355x_decompress_scratch(nblocks))


def decoded_length_dev(src: DeviceBatch, out_len, status, stream=None) -> None:
    import torch
    rc = load().lzo_mi355x_decoded_length_dev(
        _ptr(src.arena), _ptr(src.off), _ptr(src.length), _ptr(out_len), _ptr(status),
        src.nblocks, _stream_handle(torch, stream))
    if rc != 0:
        raise RuntimeError("lzo_mi355x_decoded_length_dev launch failed")
