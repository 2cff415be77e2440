"""lstore_amd -- MI355X-native erasure-coding engine behind LStore's erasure plan API.

The product is ``liblstore_ec.so`` (C ABI declared in ``include/lstore_ec.h``), built
in-tree from ``lstore_amd/csrc`` for gfx950.  This package is the Python mirror of the
plan service (``lstore_amd.erasure``), used by the tests and by ``bench.py``.
"""
from .erasure import (  # noqa: F401
    BLAUM_ROTH,
    CAUCHY_GOOD,
    CAUCHY_ORIG,
    JE_METHOD_NAMES,
    LIBER8TION,
    LIBERATION,
    RAID4,
    REED_SOL_R6_OP,
    REED_SOL_VAN,
    ErasureError,
    Plan,
    build_library,
    lib,
    library_path,
)
