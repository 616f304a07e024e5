"""nrgrep-syntax compiler: Glushkov structure, bounds, classes, errors."""
import pytest

from patmatchdocker_amd.regex import RegexSyntaxError, compile_pattern


def test_linear_pattern():
    p = compile_pattern("(GAA[CT]TC)")
    assert p.linear and p.m == 6 and p.min_len == p.max_len == 6
    assert p.first == 1 and p.last == 1 << 5
    assert p.follow == [2, 4, 8, 16, 32, 0]
    assert p.classes[3] == frozenset(b"CT")


def test_optional_and_groups():
    p = compile_pattern("(GA(TC)(TC)?A)")
    assert not p.linear and (p.min_len, p.max_len) == (5, 7)
    assert p.follow[3] == (1 << 4) | (1 << 6)


def test_star_unbounded():
    p = compile_pattern("(A(CG)*T)")
    assert p.max_len is None and p.min_len == 2
    assert p.follow[2] & (1 << 1)          # loop back G -> C


def test_case_folding_and_classes():
    p = compile_pattern("(a[^c].)")
    assert ord("A") in p.classes[0] and ord("a") not in p.classes[0]
    assert ord("C") not in p.classes[1] and ord("G") in p.classes[1]
    assert 10 in p.classes[2]              # '.' sets all 256 bytes (getAclass 0x4198c0)
    assert 10 in p.classes[1]              # so does a negated class (0x419988)


def test_escapes_and_ranges():
    p = compile_pattern(r"(\x41[0-2]\t\()")
    assert p.classes[0] == frozenset([0x41])
    assert p.classes[1] == frozenset(b"012")
    assert p.classes[2] == frozenset([9]) and p.classes[3] == frozenset(b"(")


def test_anchor_characters():
    # a trailing '$' / leading '^' are anchors (nrgrep main 0x4012a1/0x4012bd),
    # elsewhere ordinary characters
    p = compile_pattern("(ACG)$")
    assert p.m == 3 and p.anchor_end and not p.anchor_start
    q = compile_pattern("(A$C^G)")
    assert q.m == 5 and q.classes[1] == frozenset(b"$") and q.classes[3] == frozenset(b"^")


@pytest.mark.parametrize("bad", ["", "()", "(A", "A)", "(*)", "[AC", "(A|)"])
def test_syntax_errors(bad):
    with pytest.raises(RegexSyntaxError):
        compile_pattern(bad)


@pytest.mark.parametrize("pat, want", [("(?A)", "A"), ("(*AC)", "AC"), ("(GAATTC.?.?)", "GAATTC"), ("(A+CG)", "ACG"),
                                       ("(CGA+)", "CGA"), ("(A|C|G)", "[ACG]"), ("(AT(AT)?)", "AT")])
def test_nrgrep_simplify(pat, want):
    """parseConc makes an empty leaf where an operand is missing (0x41a830),
    and simplify (0x41a170) drops nullable edges, a '+' at an edge and merges
    a '|' of single classes: what nrgrep searches is the simpler pattern."""
    assert compile_pattern(pat).classes == compile_pattern("(" + want + ")").classes
    assert compile_pattern(pat).kind == "simple"


def test_long_patterns_compile():
    # nrgrep takes long patterns (multi-word masks); the GPU route decides
    # what runs (engine.route, tests/test_route.py)
    p = compile_pattern("(" + "A" * 300 + ")")
    assert p.m == 300 and p.linear
    with pytest.raises(RegexSyntaxError):   # the parser's own bound
        compile_pattern("A" * 5000)
