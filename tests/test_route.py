"""Kernel routing (engine.route): which shapes run on which kernel, and what
is refused (UnsupportedOnGPU, no CPU fallback).  No GPU needed."""
import pytest

from patmatchdocker_amd import _lib, engine
from patmatchdocker_amd.regex import compile_pattern


def prog(p):
    return compile_pattern(p, ignore_case=True)


def test_fixed_length_kernel_for_short_substitution_patterns():
    assert engine.route(prog("TGCTGA[GC]TCAGCA.[AT]"), engine.NUC, 2, "s") == "linear"
    assert engine.route(prog("A" * 64), engine.NUC, 3, "s") == "linear"


def test_automaton_kernels_take_long_patterns_and_many_errors():
    assert engine.route(prog("ACGT" * 25), engine.NUC, 0, "s") == "nfa"       # 100-nt oligo
    assert engine.route(prog("ACGT" * 25), engine.NUC, 5, "ids") == "nfa"
    assert engine.route(prog("TGCTGA[GC]TCAGCA.[AT]"), engine.NUC, 4, "s") == "nfa"
    assert engine.route(prog("TGCTGA[GC]TCAGCA.[AT]"), engine.NUC, 15, "is") == "nfa"
    # N{10,200} as patmatch_to_nrgrep.pl unrolls it: 202 positions
    assert engine.route(prog("C" + "." * 10 + ".?" * 190 + "C"), engine.BYTE, 0, "s") == "nfa"
    assert engine.route(prog("A" * 256), engine.NUC, 7, "s") == "nfa"


def test_refusals_left():
    with pytest.raises(_lib.UnsupportedOnGPU):
        engine.route(prog("A" * 257), engine.NUC, 0, "s")
    with pytest.raises(_lib.UnsupportedOnGPU):
        engine.route(prog("A" * 200), engine.NUC, 8, "s")
    with pytest.raises(_lib.UnsupportedOnGPU):
        engine.route(prog("ACG"), engine.NUC, 16, "s")
    # every position deletable: class sequences run the esimple walk over
    # every line (pm_esimple.hip), extended patterns the eextended walk,
    # regular patterns the eregular walk (pm_regular.hip)
    assert engine.route(prog("ACG"), engine.NUC, 3, "ids") == "nfa"
    assert engine.route(prog("AC?G"), engine.NUC, 2, "ids") == "nfa"
    assert engine.route(prog("A(TC)?G"), engine.NUC, 2, "ids") == "nfa"
    # the eregular restatement covers more than 64 states too (round 6)
    assert engine.route(prog("A(TC)?G" + "A" * 59), engine.NUC, 1, "ids") == "nfa"
    assert engine.route(prog("A(TC)?G" + "A" * 60), engine.NUC, 0, "") == "nfa"
    assert engine.route(prog("A(TC)?G" + "A" * 60), engine.NUC, 1, "ids") == "nfa"
    assert engine.route(prog("A(TC)?G" + "A" * 200), engine.NUC, 7, "ids") == "nfa"
    with pytest.raises(_lib.UnsupportedOnGPU):   # 4 words: at most 7 errors
        engine.route(prog("A(TC)?G" + "A" * 200), engine.NUC, 8, "ids")


def test_nfa_words():
    assert [engine.nfa_words(m) for m in (1, 64, 65, 128, 129, 256)] == [1, 1, 2, 2, 4, 4]
