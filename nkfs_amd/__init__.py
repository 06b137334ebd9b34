"""nkfs_amd -- MI355X-native N-K erasure code + XXH64 integrity path of
irqlevel/nkfs (crt/nk8.c, crt/xxhash.c, crt/csum.c).

The product is the C-ABI library nkfs_amd/lib/libnkfs_crt.so (host C over
hand-written gfx950 HIP kernels in nkfs_amd/csrc/); this package holds its
sources, a ctypes loader (_lib), the Python mirror of the reference
interface (crt), the torch-tensor batch wrappers (batch) and the seeded
workload definition (synth).
"""
from ._lib import LIB_PATH, build, lib  # noqa: F401

__all__ = ["LIB_PATH", "build", "lib"]
