"""pomegranate_amd -- MI355X-native LZO1X block codec for Pomegranate.

The hot path: LZO1X-1 compress / LZO1X decompress of
ITB-sized blocks, as HIP kernels for gfx950 behind the reference's lib/minilzo.h
call surface (liblzo_mi355x.so, include/minilzo.h) and a batch C-ABI
(include/lzo_mi355x.h).  ``lzo`` is the Python mirror of that surface.
"""
__all__ = ["lzo", "synth"]
