"""The C-ABI library loads and exports every symbol include/patmatch_hip.h
declares (no GPU calls; those are in the gpu-marked tests)."""
import ctypes
import os
import re

from patmatchdocker_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "patmatch_hip.h")).read()
    return sorted(set(re.findall(r"\b(pm_[a-z_]+)\s*\(", text)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(_lib.EXPORTED)


def test_library_exports_every_symbol():
    from patmatchdocker_amd import build
    build.build()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared_symbols():
        assert hasattr(lib, name), name


def test_version_without_gpu():
    lib = _lib.load()
    assert b"gfx950" in lib.pm_version()


def test_no_fallback_when_library_missing(monkeypatch):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libpatmatch_hip.so")
    try:
        _lib.load()
    except _lib.EngineUnavailable:
        pass
    else:
        raise AssertionError("missing library must fail loudly")


def test_specialized_kernel_compiles_without_gpu():
    """hipRTC generation + gfx950 compile of the pattern-specialized kernel."""
    from patmatchdocker_amd import engine
    from patmatchdocker_amd.convert import convert
    from patmatchdocker_amd.regex import compile_pattern
    fwd = convert("-n", "TGCTGASTCAGCANW")
    progs = [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
    for k in (0, 2):
        assert engine.jit_compile(progs, k) > 1000
    long_pat = [compile_pattern(convert("-n", "ACGT" * 12))]
    assert engine.jit_compile(long_pat, 1) > 1000


import pytest  # noqa: E402


@pytest.mark.parametrize("pat", ["GAATTC", "TATAWAWR", "TGCTGASTCAGCANW",
                                 "YYYYYYYYYYYYYYYYYYYYRRRRRRRRRRRRRRRRRRRRNNNNNNNNNNNNNNNNNNNNNNNN"])
@pytest.mark.parametrize("k", [0, 1, 2, 3])
def test_specialized_kernel_matrix_compiles(pat, k):
    """Every (pattern, k, strands) shape the GPU parity tests run generates
    valid gfx950 code (hipRTC, no GPU)."""
    from patmatchdocker_amd import engine
    from patmatchdocker_amd.convert import convert
    from patmatchdocker_amd.regex import compile_pattern
    fwd = convert("-n", pat)
    progs = [compile_pattern(fwd), compile_pattern(convert("-c", fwd))]
    assert engine.jit_compile(progs, k) > 1000
    assert engine.jit_compile(progs[:1], k) > 1000


SHARED_BLOCK_BATCH = ["ACGGTCATTGCAGT", "TTACGGTCATTGCA", "GGTCATTGCAGTCCAA", "ACGGTCATTGCAGT"]


def test_specialized_kernel_shares_strand_blocks(tmp_path, monkeypatch):
    """The generator builds one carry-save block per row for patterns that
    agree on a run of classes at a small offset: both strands of the
    near-palindromic bench motif (13 positions at offset 2) and a batch of
    shifted copies (offsets -2, +2, 0); unrelated strands share nothing."""
    from patmatchdocker_amd import engine
    from patmatchdocker_amd.convert import convert
    from patmatchdocker_amd.regex import compile_pattern

    def n_blocks(pats, k, strands):
        dump = tmp_path / "k.hip"
        monkeypatch.setenv("PM_JIT_DUMP", str(dump))
        fwd = [convert("-n", p) for p in pats]
        progs = [compile_pattern(f) for f in fwd]
        if strands:
            progs += [compile_pattern(convert("-c", f)) for f in fwd]
        assert engine.jit_compile(progs, k) > 1000
        return dump.read_text().count("// shared block")

    # the shifted partner: 8 blocks per wave, plus 2 in the first wave (its
    # lane 0, bit 0 words 0..1) -- was 4 waves x (8 + 2)
    for k in (0, 1, 2, 3):
        assert n_blocks(["TGCTGASTCAGCANW"], k, True) == 34
    assert n_blocks(SHARED_BLOCK_BATCH, 2, False) > 0
    assert n_blocks(["AAAAAACCCCCC"], 2, True) == 0   # strands agree nowhere


def test_route_indels():
    """-k with insertions/deletions routes to the Glushkov kernels, deletions
    with k >= the shortest match included; only sizes past the automaton
    kernels' limits are refused, loudly (no CPU fallback)."""
    from patmatchdocker_amd import engine
    from patmatchdocker_amd._lib import UnsupportedOnGPU
    from patmatchdocker_amd.regex import compile_pattern
    lin = compile_pattern("(GAATTC)")
    assert engine.route(lin, engine.NUC, 2, "s") == "linear"
    assert engine.route(lin, engine.NUC, 2, "ids") == "nfa"
    assert engine.route(lin, engine.NUC, 2, "i") == "nfa"
    assert engine.route(lin, engine.NUC, 0, "") == "linear"
    assert engine.parse_error_types(2, "") == "ids"
    assert engine.error_mask("ids") == 7 and engine.error_mask("d") == 2
    # deletions with k >= the shortest match: class sequences, extended and
    # regular patterns (the esimple / eextended / eregular walks over every
    # line); regular patterns over 63 positions at k > 0 route too (round 6:
    # the multi-word eregular verify)
    assert engine.route(compile_pattern("(RGD)"), engine.BYTE, 3, "d") == "nfa"
    assert engine.route(compile_pattern("(RG?D)"), engine.BYTE, 2, "d") == "nfa"
    assert engine.route(compile_pattern("(R(GK)?D)"), engine.BYTE, 2, "d") == "nfa"
    assert engine.route(compile_pattern("(R(GK)?D" + "A" * 60 + ")"), engine.BYTE, 2, "d") == "nfa"
    assert engine.route(compile_pattern("(RGD)"), engine.BYTE, 2, "d") == "nfa"
    with pytest.raises(UnsupportedOnGPU):   # beyond the automaton kernels' 256 positions
        engine.route(compile_pattern("(R(GK)?D" + "A" * 260 + ")"), engine.BYTE, 1, "s")


def test_flag_values_match_the_header():
    import re
    text = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                             "patmatch_hip.h")).read()
    for name in ("PM_REPORT_NRGREP", "PM_KEEP_HEADERS", "PM_CROSS_LINES", "PM_ESIMPLE", "PM_EXTENDED",
                 "PM_SCAN_BYTES", "PM_REGULAR", "PM_PIPELINED"):
        m = re.search(r"#define %s (\d+)" % name, text)
        assert m and int(m.group(1)) == getattr(_lib, name), name
