"""CPU: pin the oracle (oracle/lzo1x_oracle.c) to the reference's golden vectors.

Every fixture under tests/golden/ is the output of the reference's own
lib/minilzo.c (tests/golden/make_golden.py).  The GPU parity tests trust the
oracle only because these pass.
"""
from __future__ import annotations

import hashlib
import random

import numpy as np
import pytest

from conftest import batch_sizes
from pomegranate_amd import synth


def test_oracle_compress_matches_reference_edge_vectors(oracle, edge):
    bad = [n for n, d, z in zip(edge["names"], edge["inputs"], edge["comps"])
           if oracle.compress(d) != z]
    assert not bad, f"{len(bad)} mismatches, first: {bad[:5]}"
    assert len(edge["names"]) > 1500


def test_oracle_decompress_edge_vectors(oracle, edge):
    for name, d, z in zip(edge["names"], edge["inputs"], edge["comps"]):
        rc, out = oracle.decompress_safe(z, len(d))
        assert rc == 0 and out == d, name


def test_oracle_safe_decoder_error_codes(oracle, malformed):
    codes = set()
    for i, (s, cap, rc, out) in enumerate(zip(malformed["streams"], malformed["caps"],
                                              malformed["rc"], malformed["outs"])):
        got_rc, got = oracle.decompress_safe(s, cap)
        assert (got_rc, got) == (rc, out), f"case {i}: {got_rc} vs {rc}"
        codes.add(rc)
    # every lzo1x_decompress_safe outcome is represented (lib/lzoconf.h:309-318)
    assert codes >= {0, -4, -5, -6, -7, -8}


def test_oracle_matches_unchecked_decoder(oracle, unchecked):
    """The oracle's unchecked mode returns what the reference's unchecked
    lzo1x_decompress returns (lib/minilzo.c:3676-3680): LZO_E_OK,
    INPUT_NOT_CONSUMED after the first EOF (trailing bytes, the
    api/api.c:6666-6680 concatenated layout) or INPUT_OVERRUN (EOF cut short),
    with the same *out_len and bytes."""
    kinds = set()
    for i, (k, s, rc, n, sha) in enumerate(zip(unchecked["kinds"], unchecked["streams"],
                                               unchecked["rc"], unchecked["out_len"],
                                               unchecked["sha"])):
        got_rc, got = oracle.decompress_unchecked(s)
        assert (got_rc, len(got), hashlib.sha256(got).hexdigest()) == (rc, n, sha), (i, k)
        kinds.add((k, rc))
    assert {("valid", 0), ("trailing", -8), ("concat2", -8), ("eof_cut", -4)} <= kinds


def test_oracle_long_extensions_past_32_bits(oracle, longext):
    """A length extension whose 255-per-zero sum passes 2^32: the oracle keeps
    the reference's 64-bit t (lib/minilzo.c:3805, :3862-3871, :3993-3998,
    :4037-4042) and refuses it as the reference does."""
    for c in longext:
        s = c["stream"]
        assert (len(s), hashlib.sha256(s).hexdigest()) == (c["stream_len"], c["stream_sha256"])
        rc, out = oracle.decompress_safe(s, c["cap"])
        assert (rc, len(out), hashlib.sha256(out).hexdigest()) == \
            (c["rc"], c["out_len"], c["out_sha256"]), (c["kind"], c["zeros"])


def test_oracle_pins_fwritev_columns(oracle, fwritev_columns):
    """The reference's hvfs_fwritev columns (api/api.c:6666-6680): the payload
    is the oracle's per-iovec streams back to back, and the reference's read
    side (one unchecked lzo1x_decompress, :6438-6446) stops after the first
    stream with INPUT_NOT_CONSUMED whenever there is more than one."""
    fx = fwritev_columns
    for name, sizes, data, z, rc, n in zip(fx["names"], fx["iov_len"], fx["data"], fx["zips"],
                                           fx["read_rc"], fx["read_len"]):
        assert int.from_bytes(z[:8], "little") == len(data) == sum(sizes), name
        iov, at = [], 0
        for s in sizes:
            iov.append(data[at: at + s])
            at += s
        assert z[8:] == b"".join(oracle.compress(v) for v in iov), name
        assert (rc, n) == ((0, len(data)) if len(sizes) == 1 else (-8, sizes[0])), name
        got_rc, got = oracle.decompress_unchecked(z[8:])
        assert (got_rc, got) == (rc, data[:n]), name


@pytest.mark.parametrize("name", ["C2C3", "C4_sample", "itb_max", "random_300k",
                                  "models64k_random", "models64k_itb", "models64k_zeros",
                                  "models64k_alpha4", "models64k_lzlike", "models64k_text"])
def test_oracle_manifest_batches(oracle, manifest, name):
    entry = next(e for e in manifest if e["name"] == name)
    arena, offs, lens = synth.batch(entry["model_id"], entry["seed0"], batch_sizes(entry))
    hz, hi = hashlib.sha256(), hashlib.sha256()
    zl = []
    for b in range(len(lens)):
        d = arena[int(offs[b]): int(offs[b]) + int(lens[b])].tobytes()
        z = oracle.compress(d)
        hi.update(d)
        hz.update(z)
        zl.append(len(z))
    assert hi.hexdigest() == entry["sha256_input"], "synthetic generator drifted"
    assert zl == entry["zlens"]
    assert hz.hexdigest() == entry["sha256_z"]


def test_oracle_manifest_c4_order_sample(oracle, manifest):
    """C4_order (8,192 mixed blocks, ~1 GiB) is slow on the CPU: the input
    hash of the whole batch and the first 256 blocks' compressed lengths."""
    entry = next(e for e in manifest if e["name"] == "C4_order")
    sizes = batch_sizes(entry)
    arena, offs, lens = synth.batch(entry["model_id"], entry["seed0"], sizes[:256])
    for b in range(256):
        d = arena[int(offs[b]): int(offs[b]) + int(lens[b])].tobytes()
        assert len(oracle.compress(d)) == entry["zlens"][b]


def test_oracle_manifest_c1_sample(oracle, manifest):
    """C1 (1K random 64 KiB) is slow on the CPU; check the first 64 block lengths."""
    entry = next(e for e in manifest if e["name"] == "C1")
    arena, offs, lens = synth.batch(entry["model_id"], entry["seed0"], [65536] * 64)
    for b in range(64):
        d = arena[int(offs[b]): int(offs[b]) + int(lens[b])].tobytes()
        assert len(oracle.compress(d)) == entry["zlens"][b]


def test_oracle_vs_reference_fuzz(oracle, ref_lib):
    """Extra pin where the reference is compiled here: random sizes and models."""
    rng = random.Random(11)
    for i in range(300):
        n = rng.randrange(0, 70000)
        d = synth.block(i % 6, 50000 + i, n)
        assert oracle.compress(d) == ref_lib.compress(d), (i, n)
    for i in range(300):
        n = rng.randrange(0, 2000)
        z = bytearray(ref_lib.compress(synth.block(i % 6, 60000 + i, n)))
        for _ in range(rng.randrange(0, 3)):
            if z:
                z[rng.randrange(len(z))] = rng.getrandbits(8)
        cap = rng.randrange(0, n + 40)
        assert oracle.decompress_safe(bytes(z), cap) == ref_lib.decompress_safe(bytes(z), cap)


def test_generated_full_grammar_streams(oracle, ref_lib):
    """tests/lzo_streams.py (M1 forms, long extensions, far M4, short first
    runs) decodes to its known output under the oracle and the reference."""
    import lzo_streams
    for seed in range(120):
        z, out = lzo_streams.stream(seed, [50, 300, 5000, 40000][seed % 4])
        assert oracle.decompress_safe(z, len(out)) == (0, out), seed
        assert ref_lib.decompress_safe(z, len(out)) == (0, out), seed


def test_oracle_matches_reference_past_32_mib(oracle, ref_lib):
    """The oracle's encoder on a block past 32 MiB (the general GPU encoder's
    rebased positions are checked against it) equals lib/minilzo.c itself."""
    rng = np.random.default_rng(32)
    period = rng.integers(0, 256, (13 << 20) + 7, dtype=np.uint8).tobytes()
    blk = period * 3 + bytes(20 << 20) + synth.block(synth.ITB, 33, 2 << 20)
    assert oracle.compress(blk) == ref_lib.compress(blk)
