"""Client column-data codec (api/api.c:6509-6541, :6652-6689, :6427-6446):
[u64 length][LZO1X-1 stream], raw when that does not pay, decoded only when
the stream yields exactly the recorded length.  The payload stream is checked
against the oracle (the checker)."""
from __future__ import annotations

import struct

import numpy as np
import pytest

from pomegranate_amd import column, lzo, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _columns():
    rng = np.random.default_rng(9)
    cols = [synth.block(synth.ITB, 700 + i, int(n)) for i, n in
            enumerate(rng.integers(4096, 12289, 6))]            # small-file column data
    cols += [synth.block(synth.TEXT, 800, 3000), synth.block(synth.ZEROS, 801, 9000)]
    cols += [synth.block(synth.RANDOM, 802, 5000), b"abc", b"x" * 9]
    return cols


def test_zip_format_and_raw_fallback(oracle):
    cols = _columns()
    zips, comp = column.zip_batch(cols)
    for c, z, k in zip(cols, zips, comp):
        zc = oracle.compress(c)
        if len(zc) + 8 >= len(c):                  # api/api.c:6525-6538: raw
            assert k == 0 and z == b""
        else:
            assert k == 1 and z == struct.pack("<Q", len(c)) + zc


def test_zip_never_overruns_small_capacity(oracle):
    """The reference's zip buffer is len + 8 (api/api.c:6512); incompressible
    data compresses to more than that.  Here such a column goes raw and the
    buffer is never written past its capacity."""
    c = synth.block(synth.RANDOM, 803, 8192)
    assert len(oracle.compress(c)) > len(c) + 8 - 8
    zips, comp = column.zip_batch([c], caps=[len(c) + 8])
    assert comp == [0] and zips == [b""]


def test_unzip_round_trip_and_length_check():
    cols = [c for c in _columns() if len(c) > 100]
    zips, comp = column.zip_batch(cols)
    zc = [z for z, k in zip(zips, comp) if k]
    want = [c for c, k in zip(cols, comp) if k]
    outs, err = column.unzip_batch(zc, [len(c) + 8 for c in want])
    assert err == [0] * len(zc) and outs == want
    bad = bytearray(zc[0])
    bad[:8] = struct.pack("<Q", len(want[0]) + 1)            # olen != olen_cmp
    outs, err = column.unzip_batch([bytes(bad), zc[1][:-4]], [len(want[0]) + 16, len(want[1])])
    assert err[0] != 0 and err[1] != 0


def test_zipv_is_one_decodable_stream(oracle):
    """hvfs_fwritev: the iovecs zip as one column that the read side decodes."""
    iov = [synth.block(synth.ITB, 810 + i, 4096) for i in range(5)]
    z, k = column.zipv(iov, column.zip_bound(sum(map(len, iov))))
    flat = b"".join(iov)
    assert k == 1 and z == struct.pack("<Q", len(flat)) + oracle.compress(flat)
    outs, err = column.unzip_batch([z], [len(flat)])
    assert err == [0] and outs == [flat]


def test_unzip_reads_reference_fwritev_columns(fwritev_columns):
    """Columns the reference's hvfs_fwritev wrote (api/api.c:6666-6680, one
    stream per iovec; reference-generated fixtures) decode to their data,
    where the reference's own read side stops after the first stream."""
    fx = fwritev_columns
    outs, err = column.unzip_batch(fx["zips"], [len(d) for d in fx["data"]])
    assert err == [0] * len(outs)
    assert outs == fx["data"]
    # mixed with single-stream columns and in a tight capacity
    zips, comp = column.zip_batch([fx["data"][2], fx["data"][4]])
    assert comp == [1, 1]
    outs, err = column.unzip_batch([zips[0], fx["zips"][4], zips[1], fx["zips"][6]],
                                   [len(fx["data"][i]) for i in (2, 4, 4, 6)])
    assert err == [0] * 4 and outs == [fx["data"][i] for i in (2, 4, 4, 6)]


def test_unzip_fwritev_columns_errors(fwritev_columns):
    """Damaged multi-stream columns fail like a damaged single stream: the
    last stream cut short, too little room, or a recorded length that the
    streams do not add up to."""
    fx = fwritev_columns
    i = fx["names"].index("fuse_pages")
    z, d = fx["zips"][i], fx["data"][i]
    bad_len = struct.pack("<Q", len(d) + 1) + z[8:]
    outs, err = column.unzip_batch([z[:-2], z, bad_len], [len(d), len(d) - 1, len(d) + 1])
    assert err[0] != 0 and err[1] == -5 and err[2] != 0
    assert outs[1] == d[:len(d) - 1][: len(outs[1])]


def test_concat_batch_matches_per_stream_decodes(fwritev_columns):
    """lzo_mi355x_decompress_concat_batch: each stream decodes as its own
    lzo1x_decompress_safe call would; the status is the last stream's."""
    fx = fwritev_columns
    payloads = [z[8:] for z in fx["zips"]]
    rc, st, outs = lzo.decompress_batch(payloads, [len(d) for d in fx["data"]], concat=True)
    assert rc == 0 and st == [0] * len(payloads) and outs == fx["data"]
    # trailing junk after the last stream: INPUT_NOT_CONSUMED is not a stream start
    rc, st, outs = lzo.decompress_batch([payloads[1] + b"\x00"], [len(fx["data"][1]) + 64],
                                        concat=True)
    assert rc == 0 and st[0] != 0
