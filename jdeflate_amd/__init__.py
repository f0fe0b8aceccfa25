"""jdeflate_amd -- MI355X-native deflate/inflate engine with the jdeflate C API.

The product is the C-ABI library ``jdeflate_amd/lib/libjdeflate_amd.so``
(headers in ``include/jdeflate``); this package only holds its sources
(``csrc/``) and thin ctypes bindings (``engine``) used by the tests and the
benchmark.  See DESIGN.md.
"""
from .engine import (  # noqa: F401
    BLOCKSIZE, DEFLT_END, DEFLT_FLUSH, DEFLT_NOFLUSH, Deflator, EngineUnavailable,
    EXPORTS, Inflator, available, bound, corpus_mixed, corpus_text, deflate_blocks,
    deflate_device, deflate_stream, inflate_blocks, inflate_device, inflate_stream,
    deflate_multi, inflate_multi,
    load_library, nblocks,
    prof_enable, prof_read, KERNELS, ZStrm, checksums, crc32_combine,
)

__version__ = "0.4.0+mi355x"
