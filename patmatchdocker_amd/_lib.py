"""ctypes binding of ``libpatmatch_hip.so`` (the C ABI in include/patmatch_hip.h).

The library is built in-tree by :func:`patmatchdocker_amd.build.build`.  There
is deliberately no fallback: if the shared object is missing or cannot be
loaded, every scan raises :class:`EngineUnavailable`.
"""

from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PM_LIB_AB") or os.path.join(_HERE, "libpatmatch_hip.so")   # PM_LIB_AB: A/B runs only

PM_ALPHA_NUC = 0
PM_ALPHA_BYTE = 1
PM_E_ARG, PM_E_HIP, PM_E_NODEV = -1, -2, -3
PM_E_UNSUPPORTED = -4
PM_MAX_K = 15                 # errors, general patterns (<= 7 above 128 positions)
PM_MAX_POSITIONS = 256        # automaton positions, general patterns
PM_MAX_LINEAR_K = 3           # substitutions, fixed-length kernel
PM_MAX_LINEAR_POSITIONS = 64  # pattern length, fixed-length kernel
PM_ERR_INS, PM_ERR_DEL, PM_ERR_SUB = 1, 2, 4
PM_REPORT_ALL, PM_REPORT_NRGREP, PM_ANCHOR_START, PM_ANCHOR_END, PM_KEEP_HEADERS = 0, 1, 2, 4, 8
PM_CROSS_LINES = 16
PM_SCAN_BYTES = 256           # BYTE databases: scan the byte copy, not the 5-bit residue planes
PM_ESIMPLE = 64               # a class sequence at k > 0: nrgrep's esimple report
PM_EXTENDED = 128             # classes with '?*+': nrgrep's extended / eextended report
PM_REGULAR = 512              # '|' / repeated groups: nrgrep's regular report (pm_scan_nfa_tree)
PM_PIPELINED = 1024           # automaton scans: the report pass is queued, the count resolves on first use

# every symbol declared in include/patmatch_hip.h
EXPORTED = (
    "pm_last_error", "pm_version", "pm_device_count", "pm_db_create",
    "pm_db_create_synthetic", "pm_db_destroy", "pm_db_info", "pm_db_decode",
    "pm_scan_linear", "pm_scan_nfa", "pm_hits_count", "pm_hits_copy",
    "pm_hits_kernel_ms", "pm_hits_destroy", "pm_hits_device", "pm_hits_copy_device", "pm_hits_record_use",
    "pm_linear_jit_compile", "pm_scan_nfa_errs", "pm_scan_linear_async", "pm_scan_nfa_wide",
    "pm_ids_jit_compile", "pm_esimple_plan", "pm_db_set_regions", "pm_db_regions",
    "pm_extended_plan", "pm_eextended_plan", "pm_db_residue_codes", "pm_scan_nfa_tree",
    "pm_regular_plan",
    "pm_eregular_plan", "pm_merge_parts",
)
PM_NRGREP_BUFFER = 1600000    # nrgrep_coords -b 1600000 (bytes: patmatch.py:733-743)


class EngineUnavailable(RuntimeError):
    """The HIP scan library is missing or no GPU is present."""


class EngineError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__("patmatch_hip error %d: %s" % (code, message))
        self.code = code


class UnsupportedOnGPU(NotImplementedError):
    """The pattern/option combination has no GPU kernel yet (fails loudly)."""


_lib = None

P = ctypes.c_void_p
PP = ctypes.POINTER(ctypes.c_void_p)
u64 = ctypes.c_uint64
pu64 = ctypes.POINTER(ctypes.c_uint64)


def _declare(lib):
    lib.pm_last_error.restype = ctypes.c_char_p
    lib.pm_version.restype = ctypes.c_char_p
    lib.pm_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
    lib.pm_db_create.argtypes = [ctypes.c_char_p, u64, ctypes.c_int, ctypes.c_int, P, PP]
    lib.pm_db_create_synthetic.argtypes = [u64, u64, u64, ctypes.c_int, P, PP]
    lib.pm_db_destroy.argtypes = [P]
    lib.pm_db_info.argtypes = [P, pu64, ctypes.POINTER(ctypes.c_int), pu64, pu64]
    lib.pm_db_decode.argtypes = [P, u64, ctypes.c_uint32, ctypes.c_char_p]
    lib.pm_db_residue_codes.argtypes = [P, ctypes.POINTER(ctypes.c_int), P]
    lib.pm_db_set_regions.argtypes = [P, u64, P, P]
    lib.pm_db_regions.argtypes = [P, u64, P, P, pu64]
    lib.pm_scan_linear.argtypes = [P, ctypes.c_int, P, P, ctypes.c_int, P, P, P, ctypes.c_int, ctypes.c_int, PP]
    lib.pm_scan_linear_async.argtypes = lib.pm_scan_linear.argtypes
    lib.pm_scan_nfa.argtypes = [P, ctypes.c_int, P, P, u64, u64, ctypes.c_int, ctypes.c_int,
                                ctypes.c_int, PP]
    lib.pm_scan_nfa_errs.argtypes = [P, ctypes.c_int, P, P, u64, u64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, PP]
    lib.pm_scan_nfa_wide.argtypes = [P, ctypes.c_int, ctypes.c_int, P, P, P, P, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, PP]
    lib.pm_scan_nfa_tree.argtypes = lib.pm_scan_nfa_wide.argtypes[:-1] + [ctypes.c_int, P, P, PP]
    lib.pm_regular_plan.argtypes = [ctypes.c_int, ctypes.c_int, P, ctypes.c_int, P, P, P, P]
    lib.pm_eregular_plan.argtypes = [ctypes.c_int, ctypes.c_int, P, ctypes.c_int, P, P, ctypes.c_int, P, P]
    lib.pm_ids_jit_compile.argtypes = [ctypes.c_int, P, ctypes.c_int, ctypes.c_int, pu64]
    lib.pm_extended_plan.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, P]
    lib.pm_eextended_plan.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, ctypes.c_int, P]
    lib.pm_hits_count.argtypes = [P, pu64]
    lib.pm_hits_copy.argtypes = [P, P, P, P, u64]
    lib.pm_hits_kernel_ms.argtypes = [P, ctypes.POINTER(ctypes.c_double)]
    lib.pm_hits_destroy.argtypes = [P]
    lib.pm_hits_device.argtypes = [P, PP, PP, pu64]
    lib.pm_hits_record_use.argtypes = [P, P]
    lib.pm_hits_copy_device.argtypes = [P, P, P, u64, P]
    lib.pm_merge_parts.argtypes = [P, P, P, P, ctypes.c_int, ctypes.c_int, P, P, P, P, pu64, ctypes.c_int, P]
    lib.pm_esimple_plan.argtypes = [ctypes.c_int, ctypes.c_int, P, ctypes.c_int, ctypes.POINTER(ctypes.c_int32)]
    lib.pm_linear_jit_compile.argtypes = [ctypes.c_int, P, P, ctypes.c_int, P, P, ctypes.c_int, pu64]
    for name in EXPORTED:
        if name not in ("pm_last_error", "pm_version"):
            getattr(lib, name).restype = ctypes.c_int
    return lib


def load():
    """Load (once) and return the library handle; raise if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise EngineUnavailable(
                "%s is missing: run `python -m patmatchdocker_amd.build` (no CPU fallback exists)" % LIB_PATH)
        try:
            _lib = _declare(ctypes.CDLL(LIB_PATH))
        except OSError as exc:  # pragma: no cover - depends on the box
            raise EngineUnavailable("cannot load %s: %s" % (LIB_PATH, exc)) from exc
    return _lib


def check(rc: int):
    if rc != 0:
        msg = load().pm_last_error().decode("utf-8", "replace")
        if rc == PM_E_UNSUPPORTED:
            raise UnsupportedOnGPU(msg)
        if rc == -3:
            raise EngineUnavailable(msg)
        raise EngineError(rc, msg)


def device_count() -> int:
    c = ctypes.c_int(0)
    check(load().pm_device_count(ctypes.byref(c)))
    return c.value
