"""Loader for nkfs_amd/lib/libnkfs_crt.so -- the MI355X C-ABI library.

There is no fallback: if the library is missing this raises, and on a host
without a GPU the library's own entry points return -ENODEV / -EAGAIN.

torch (when installed) is imported first so that the library binds to the
same HIP runtime as torch (both carry the SONAME libamdhip64.so.7); streams
and device pointers can then be shared with torch tensors.
"""
from __future__ import annotations

import ctypes as C
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
# NKFS_LIB: test tooling may point at another build of the same library
# (nkfs_amd/lib/debug/libnkfs_crt.so, `make DEBUG_BOUNDS=1`); the product
# path loads the in-tree build.
LIB_PATH = os.environ.get("NKFS_LIB") or os.path.join(HERE, "lib", "libnkfs_crt.so")
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")

try:  # share torch's HIP runtime when torch is present
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the C-ABI
    torch = None

u8p = C.POINTER(C.c_uint8)
vp = C.c_void_p


class Tune(C.Structure):
    """struct nkfs_tune (include/nkfs_gpu.h): kernel choice and launch shape."""
    _fields_ = [(f, C.c_int) for f in ("enc_kernel", "dec_kernel", "enc_waves_per_cu", "dec_waves_per_cu",
                                       "dec_units", "enc_nib", "enc_units", "size_order", "enc_prefetch",
                                       "enc_fused_waves_per_cu", "dec_wave_waves_per_cu", "dec_run_units",
                                       "enc_ws_prefetch", "enc_big_fused", "dec_pair_stage",
                                       "host_depth", "host_lanes", "enc_ragged_split", "enc_ws_waves",
                                       "dec_pair_waves", "enc_few_max", "enc_ws_hash_waves", "enc_persist", "dec_bign", "enc_bign",
                                       "dec_pair_pipe")]


ENC = {"auto": 0, "walk": 1, "fused": 2, "ws": 3, "generic": 4, "wide": 5, "big": 6, "wide_ws": 7, "wsp": 8}
DEC = {"auto": 0, "slice": 1, "wave": 2, "generic": 3, "wide": 4, "big": 5, "run": 6, "pair": 7}

# name -> (restype, argtypes)
_SIGS = {
    "nk8_init": (C.c_int, []),
    "nk8_release": (None, []),
    "nk8_split_block": (C.c_int, [u8p, C.c_uint32, C.c_int, C.c_int, C.POINTER(C.POINTER(u8p)), C.POINTER(u8p)]),
    "nk8_assemble_block": (C.c_int, [C.POINTER(u8p), u8p, C.c_int, C.c_int, u8p, C.c_uint32]),
    "XXH64": (C.c_ulonglong, [vp, C.c_size_t, C.c_ulonglong]),
    "XXH64_createState": (vp, []),
    "XXH64_freeState": (C.c_int, [vp]),
    "XXH64_reset": (C.c_int, [vp, C.c_ulonglong]),
    "XXH64_update": (C.c_int, [vp, vp, C.c_size_t]),
    "XXH64_digest": (C.c_ulonglong, [vp]),
    "csum_reset": (None, [vp]),
    "csum_update": (None, [vp, vp, C.c_size_t]),
    "csum_digest": (None, [vp, vp]),
    "csum_u64": (C.c_uint64, [vp]),
    "crt_malloc": (vp, [C.c_size_t]),
    "crt_free": (None, [vp]),
    "nkfs_gpu_init": (C.c_int, [C.c_int]),
    "nkfs_gpu_ready": (C.c_int, []),
    "nkfs_tune_get": (None, [C.POINTER(Tune)]),
    "nkfs_tune_set": (C.c_int, [C.POINTER(Tune)]),
    "nkfs_part_size": (C.c_uint32, [C.c_uint32, C.c_int]),
    "nkfs_part_pitch": (C.c_uint64, [C.c_uint32, C.c_int]),
    "nkfs_nk8_encode": (C.c_int, [vp, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int, C.c_int, vp, vp, C.c_uint64,
                                  vp, vp]),
    "nkfs_nk8_encode_ragged": (C.c_int, [vp, vp, vp, C.c_uint32, C.c_uint32, C.c_int, C.c_int, vp, vp, vp, vp, vp]),
    "nkfs_decode_workspace": (C.c_uint64, [C.c_uint32, C.c_int]),
    "nkfs_nk8_decode": (C.c_int, [vp, C.c_uint64, C.c_int, vp, vp, C.c_int, C.c_int, C.c_uint32, vp, C.c_uint64,
                                  C.c_uint32, vp, vp, vp]),
    "nkfs_nk8_decode_verify": (C.c_int, [vp, C.c_uint64, C.c_int, vp, vp, C.c_int, C.c_int, C.c_uint32, vp,
                                         C.c_uint64, C.c_uint32, vp, vp, vp, vp, vp]),
    "nkfs_nk8_decode_ragged": (C.c_int, [vp, vp, C.c_int, vp, vp, C.c_int, C.c_int, vp, vp, vp, C.c_uint32,
                                         C.c_uint32, vp, vp, vp]),
    "nkfs_nk8_encode_ragged_host": (C.c_int, [vp, vp, vp, C.c_uint32, C.c_uint32, C.c_int, C.c_int, vp, vp, vp, vp,
                                              C.c_uint64]),
    "nkfs_xxh64_batch": (C.c_int, [vp, vp, vp, C.c_uint32, C.c_uint64, vp, vp]),
    "nkfs_clu_sum_batch": (C.c_int, [vp, C.c_uint64, C.c_uint32, C.c_uint32, vp, vp, vp, vp]),
    "nkfs_pages_dsum_batch": (C.c_int, [vp, vp, vp, C.c_uint32, C.c_uint32, vp, vp]),
    "nkfs_nk8_encode_host": (C.c_int, [vp, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int, C.c_int, vp, vp,
                                       C.c_uint64, vp, C.c_uint64]),
    "nkfs_nk8_decode_ragged_verify": (C.c_int, [vp, vp, C.c_int, vp, vp, C.c_int, C.c_int, vp, vp, vp, C.c_uint32,
                                                C.c_uint32, vp, vp, vp, vp, vp]),
    "nkfs_nk8_encode_pages": (C.c_int, [vp, C.c_uint32, vp, vp, C.c_uint32, C.c_uint32, C.c_int, C.c_int, vp, vp,
                                        vp, vp, C.c_uint64]),
    "nkfs_nk8_decode_host": (C.c_int, [vp, C.c_uint64, C.c_int, vp, vp, C.c_int, C.c_int, C.c_uint32, vp,
                                       C.c_uint64, C.c_uint32, vp, vp, vp, C.c_uint64]),
    "nkfs_nk8_decode_ragged_host": (C.c_int, [vp, vp, C.c_int, vp, vp, C.c_int, C.c_int, vp, vp, vp, C.c_uint32,
                                              C.c_uint32, vp, vp, vp, C.c_uint64]),
    "nkfs_nk8_decode_pages": (C.c_int, [vp, vp, C.c_int, vp, vp, C.c_int, C.c_int, vp, C.c_uint32, vp, vp,
                                        C.c_uint32, C.c_uint32, vp, vp, vp, C.c_uint64]),
    "nkfs_host_register": (C.c_int, [vp, C.c_size_t]),
    "nkfs_host_unregister": (C.c_int, [vp]),
    "nkfs_gpu_device": (C.c_int, []),
    "nkfs_gpu_count": (C.c_int, []),
    "nkfs_gpu_set_devices": (C.c_int, [C.POINTER(C.c_int), C.c_int]),
    "nkfs_gpu_get_devices": (C.c_int, [C.POINTER(C.c_int), C.c_int]),
    "nkfs_synth_ragged": (C.c_int, [vp, vp, vp, C.c_uint32, C.c_uint64, C.c_uint64, vp]),
    "nkfs_synth_blocks": (C.c_int, [vp, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint64, vp]),
    "nkfs_dev_alloc": (vp, [C.c_size_t]),
    "nkfs_dev_free": (None, [vp]),
    "nkfs_memcpy_h2d": (C.c_int, [vp, vp, C.c_size_t]),
    "nkfs_memcpy_d2h": (C.c_int, [vp, vp, C.c_size_t]),
    "nkfs_stream_sync": (C.c_int, [vp]),
    "nkfs_pipeline_check": (C.c_int, [C.c_int, vp, vp, C.c_uint32, C.c_uint32, C.c_int, C.c_int, C.c_int, vp,
                                      C.c_uint32, C.c_uint64, C.c_char_p, C.c_size_t]),
    "nkfs_host_lane_plan": (C.c_int, [vp, C.c_int, C.c_int, vp, C.c_int]),
    "nkfs_host_state": (C.c_int, [vp, C.c_int]),
    "nkfs_percall_service": (C.c_int, [C.c_int]),
}

_lib = None


def build() -> None:
    import subprocess

    jobs = str(min(16, os.cpu_count() or 4))
    out = subprocess.run(["make", "-C", CSRC, "-j", jobs], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("libnkfs_crt build failed:\n" + out.stdout[-4000:] + out.stderr[-4000:])


def lib():
    """The loaded library (ctypes.CDLL) with prototypes set."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make -C {CSRC}` (hipcc, gfx950); "
                              "there is no CPU fallback for the nkfs GPU path")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def header_functions() -> list[str]:
    """Function names declared in include/*.h (the C-ABI contract)."""
    names: list[str] = []
    for h in sorted(os.listdir(INCLUDE)):
        if not h.endswith(".h"):
            continue
        text = open(os.path.join(INCLUDE, h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b([A-Za-z_]\w*)\s*\(([^;{]*?)\)\s*;", text, flags=re.M):
            if m.group(1) not in names:
                names.append(m.group(1))
    return names


def get_tune() -> Tune:
    t = Tune()
    lib().nkfs_tune_get(C.byref(t))
    return t


class tuned:
    """Context manager: run a block with some nkfs_tune fields replaced, e.g.
    ``with tuned(enc_kernel=ENC["fused"]): ...`` (tests pin kernels this way;
    the library reads no environment variable to choose one)."""

    def __init__(self, **fields):
        self.fields = fields
        self.saved = None

    def __enter__(self):
        self.saved = get_tune()
        t = get_tune()
        for k, v in self.fields.items():
            setattr(t, k, v)
        check(lib().nkfs_tune_set(C.byref(t)), "nkfs_tune_set")
        return t

    def __exit__(self, *exc):
        lib().nkfs_tune_set(C.byref(self.saved))
        return False


def check(rc: int, what: str = "nkfs") -> int:
    if rc < 0:
        raise OSError(-rc, f"{what}: {os.strerror(-rc)}")
    return rc
