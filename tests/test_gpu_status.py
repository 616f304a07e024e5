"""The C-ABI entries and a HIP status left pending on the caller's thread.

HIP keeps an error on the thread until hipGetLastError() reads it; a later
successful call does not reset it (tools/micro/status_probe.hip).  So a
launch check inside an entry would report a failure of some earlier,
unchecked call -- round 5's one suite failure ("operation not permitted
when stream is capturing" in a test_gpu_p5 launch check) read such a code.
Each entry (guarded(), pm_internal.h) therefore starts by reading the
thread's status: hipErrorStreamCaptureUnsupported (what a capture-unsafe
call returns while a stream captures in global mode) is cleared and the
entry runs; any other pending code is reported as the entry's failure
(PM_E_HIP, the code in pm_last_error) and cleared, so the next call runs."""
import ctypes

import pytest

pytestmark = pytest.mark.gpu

HIP_ERROR_INVALID_DEVICE = 101
HIP_ERROR_STREAM_CAPTURE_UNSUPPORTED = 900
HIP_STREAM_CAPTURE_MODE_GLOBAL = 0
HIP_STREAM_NON_BLOCKING = 1


def _hip():
    """The HIP runtime this process already loaded (torch's and the
    library's), by its path in /proc/self/maps: the same instance, so its
    thread-local status is the one the library reads."""
    with open("/proc/self/maps") as fh:
        paths = {ln.split()[-1] for ln in fh if "libamdhip64.so" in ln}
    assert paths, "libamdhip64 not loaded"
    return ctypes.CDLL(sorted(paths)[0])


@pytest.fixture(scope="module")
def engine():
    from patmatchdocker_amd import engine as eng
    from patmatchdocker_amd import _lib
    _lib.load()
    assert _lib.device_count() > 0, "no GPU visible"
    return eng


@pytest.fixture()
def small_db(engine):
    db = engine.SequenceDatabase.from_bytes(b">s1\n" + b"ACGTTGCA" * 64 + b"\n", alphabet=engine.NUC)
    yield db
    db.close()


def _info_rc(db):
    from patmatchdocker_amd import _lib
    n = ctypes.c_uint64()
    return _lib.load().pm_db_info(db.handle, ctypes.byref(n), None, None, None), n.value


def test_entry_clears_a_pending_capture_status(small_db):
    hip = _hip()
    hip.hipGetLastError()
    stream = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(stream), HIP_STREAM_NON_BLOCKING) == 0
    try:
        assert hip.hipStreamBeginCapture(stream, HIP_STREAM_CAPTURE_MODE_GLOBAL) == 0
        p = ctypes.c_void_p()
        # capture-unsafe while this thread captures: fails, its code stays pending
        rc_unsafe = hip.hipMalloc(ctypes.byref(p), 64)
        pending = hip.hipPeekAtLastError()
        # an entry that makes no HIP call of its own (host-side info)
        rc, n = _info_rc(small_db)
        after = hip.hipPeekAtLastError()
        graph = ctypes.c_void_p()
        hip.hipStreamEndCapture(stream, ctypes.byref(graph))
        if graph.value:
            hip.hipGraphDestroy(graph)
        hip.hipGetLastError()
    finally:
        hip.hipStreamDestroy(stream)
        hip.hipGetLastError()
    assert rc_unsafe == HIP_ERROR_STREAM_CAPTURE_UNSUPPORTED and pending == HIP_ERROR_STREAM_CAPTURE_UNSUPPORTED
    assert rc == 0 and n == len(small_db)
    assert after == 0   # read (cleared) by the entry


def test_entry_reports_any_other_pending_status_then_runs(small_db, engine):
    from patmatchdocker_amd import _lib
    from patmatchdocker_amd.convert import convert
    from patmatchdocker_amd.regex import compile_pattern
    hip = _hip()
    hip.hipGetLastError()
    assert hip.hipSetDevice(4096) == HIP_ERROR_INVALID_DEVICE   # left unread
    rc, _ = _info_rc(small_db)
    assert rc == _lib.PM_E_HIP
    msg = _lib.load().pm_last_error().decode()
    assert "pending" in msg and "invalid device" in msg.lower()
    # read by the failing entry: the next calls run, a scan included
    assert _info_rc(small_db)[0] == 0
    res, _ = engine.scan(small_db, [compile_pattern(convert("-n", "ACGTTGCA"))], k=0, types="")
    assert len(res[0][0]) == 64
