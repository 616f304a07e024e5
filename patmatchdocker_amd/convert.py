"""PatMatch pattern syntax -> nrgrep regular-expression syntax.

Behavioural restatement of ``www/bin/patmatch_to_nrgrep.pl`` (the reference's
pattern converter, invoked from ``www/FlaskApp/FlaskApp/patmatch.py:291`` and
``:296``).  The reference runs the Perl script through ``os.popen``; here it is
an in-process function with the same three modes:

    ``-n``  nucleotide pattern            (patmatch_to_nrgrep.pl:51-54)
    ``-p``  peptide pattern               (:55-58)
    ``-c``  reverse-complement nucleotide (:59-62)

The pipeline is the Perl one, stage for stage (``process_pattern``, :83-91):
strip whitespace + upper-case (+ reverse complement for ``-c``), wildcards
``N``/``X`` -> ``.``, ``{m,n}`` repetitions -> unrolled copies with ``?``/``*``,
IUPAC / ambiguity letters -> bracket classes, flattening of nested brackets,
and finally wrapping in ``( )`` with anchors.  Quirks of the Perl code are
kept on purpose because the hits the reference reports depend on them, e.g.
the reverse complement moves a postfix ``?``/``*`` in front of its atom
(``CA.?G`` -> ``C?.TG``), and Perl ``split`` drops trailing empty fields.

Malformed input that makes the Perl script loop forever (unbalanced ``}`` or
``)``) raises :class:`PatternSyntaxError` instead.
"""

from __future__ import annotations

import re

__all__ = ["PatternSyntaxError", "convert", "reverse_complement_pattern"]


class PatternSyntaxError(ValueError):
    """Raised where the reference converter would hang or produce garbage."""


INFINITE = -1

# complement_nucleotides (patmatch_to_nrgrep.pl:564-578)
_COMPLEMENT = str.maketrans("ATCGRYSWMKVHDB", "TAGCYRSWKMBDHV")

# sub_characters (patmatch_to_nrgrep.pl:430-455); order matters only for
# documentation -- no replacement text contains a later key.
_PEPTIDE_CLASSES = (("J", "[IFVLWMAGCY]"), ("O", "[TSHEDQNKR]"),
                    ("B", "[DN]"), ("Z", "[EQ]"))
_NUCLEOTIDE_CLASSES = (("R", "[AG]"), ("Y", "[CT]"), ("S", "[GC]"),
                       ("W", "[AT]"), ("M", "[AC]"), ("K", "[GT]"),
                       ("V", "[ACG]"), ("H", "[ACT]"), ("D", "[AGT]"),
                       ("B", "[CGT]"))

_CLOSER_TO_OPENER = {")": "(", "]": "[", "}": "{"}


def _perl_num(text) -> int:
    """Perl's numeric conversion of a string: leading integer, else 0."""
    m = re.match(r"\s*([+-]?\d+)", str(text))
    return int(m.group(1)) if m else 0


def _pop(stack: list, what: str):
    if not stack:
        raise PatternSyntaxError("unbalanced %s in pattern" % what)
    return stack.pop()


# ---------------------------------------------------------------------------
# reverse complement (get_reverse_complement / reverse_pattern / extract_group,
# patmatch_to_nrgrep.pl:540-700)
# ---------------------------------------------------------------------------

def _read_group_backwards(closer: str, rest: list) -> str:
    """Consume, from the tail of ``rest``, the group that ``closer`` ends.

    Brackets/parentheses come back with their content reversed; a ``{..}``
    repetition comes back with its count in order and the atom (or group) it
    applies to placed in front of it (extract_group, :632-700).
    """
    opener = _CLOSER_TO_OPENER[closer]
    if closer == "}":
        count = []
        while True:
            ch = _pop(rest, "'}'")
            if ch == "{":
                break
            if ch in _CLOSER_TO_OPENER:
                # a group nested inside a count is consumed and dropped: the
                # Perl collects it in a list it never emits for '}' (:676-680)
                _read_group_backwards(ch, rest)
            else:
                count.insert(0, ch)
        atom = rest.pop() if rest else ""     # Perl: undef -> ""
        if atom in (")", "]"):
            atom = _read_group_backwards(atom, rest)
        return atom + "{" + "".join(count) + "}"
    inner = []
    while True:
        ch = _pop(rest, repr(closer))
        if ch == opener:
            return opener + "".join(inner) + closer
        if ch in _CLOSER_TO_OPENER:
            inner.append(_read_group_backwards(ch, rest))
        else:
            inner.append(ch)


def reverse_complement_pattern(pattern: str) -> str:
    """Complement every nucleotide code, then reverse element by element."""
    text = pattern.translate(_COMPLEMENT)
    if text.startswith("<"):
        text = ">" + text[1:]
    if text.endswith(">"):
        text = text[:-1] + "<"
    rest = list(text)
    out = []
    while rest:
        ch = rest.pop()
        out.append(_read_group_backwards(ch, rest) if ch in _CLOSER_TO_OPENER else ch)
    return "".join(out)


# ---------------------------------------------------------------------------
# repetitions (fix_repetitions & helpers, patmatch_to_nrgrep.pl:160-395)
# ---------------------------------------------------------------------------

def _repeat_bounds(info: str):
    """process_repeat_info (:340-368) incl. Perl split's trailing-field drop."""
    fields = info.split(",")
    while fields and fields[-1] == "":
        fields.pop()
    if re.match(r",\d+", info):
        return 0, _perl_num(fields[1])
    if re.search(r"\d+,$", info):
        return _perl_num(fields[0]), INFINITE
    if re.fullmatch(r"\d+\n?", info):
        return _perl_num(info), _perl_num(info)
    if re.fullmatch(r"\d+,\d+\n?", info):
        return _perl_num(fields[0]), _perl_num(fields[1])
    return 0, 0


def _take_repeated_element(elements: list) -> str:
    """extract_repeat_pattern (:270-320): the element a ``{..}`` applies to."""
    if not elements:
        return ""            # Perl pops undef here and carries on with ""
    last = elements.pop()
    if last not in (")", "]"):
        return last
    opener = "(" if last == ")" else "["
    depth, taken = 1, [last]
    while depth:
        el = _pop(elements, repr(last))
        taken.insert(0, el)
        if el == last:
            depth += 1
        elif el == opener:
            depth -= 1
    return "".join(taken)


def _unroll(lower: int, upper: int, unit: str) -> str:
    """build_nrgrep_repeat (:380-395)."""
    text = unit * max(lower, 0)
    if upper == INFINITE:
        return text + unit + "*"
    return text + (unit + "?") * max(upper - lower, 0)


def _expand_repetitions(pattern: str) -> str:
    if "{" not in pattern:
        return pattern
    elements: list = []
    for ch in pattern:
        if ch != "}":
            elements.append(ch)
            continue
        info = []
        while True:
            el = _pop(elements, "'}'")
            if el == "{":
                break
            info.insert(0, el)
        unit = _take_repeated_element(elements)
        lower, upper = _repeat_bounds("".join(info))
        elements.append(_unroll(lower, upper, unit))
    return "".join(elements)


# ---------------------------------------------------------------------------
# classes (sub_characters / remove_nested_brackets, :420-520)
# ---------------------------------------------------------------------------

def _flatten_brackets(pattern: str) -> str:
    """Drop inner brackets and repeated members inside an outer class."""
    out, depth, seen = [], 0, set()
    for ch in pattern:
        if ch == "[":
            if depth == 0:
                out.append(ch)
            depth += 1
        elif ch == "]":
            depth = max(depth - 1, 0)
            if depth == 0:
                out.append(ch)
                seen = set()
        elif depth == 0:
            out.append(ch)
        elif ch not in seen:
            out.append(ch)
            seen.add(ch)
    return "".join(out)


def _anchor_and_wrap(pattern: str) -> str:
    """finalize_pattern (:530-555): '<' / '>' become '^' / '$' outside '( )'."""
    begins, ends = pattern.startswith("<"), bool(re.search(r">\n?$", pattern))
    if begins and ends:
        return "^(" + pattern.replace("<", "", 1).replace(">", "", 1) + ")$"
    if begins:
        return "^(" + pattern.replace("<", "", 1) + ")"
    if ends:
        return "(" + pattern.replace(">", "", 1) + ")$"
    return "(" + pattern + ")"


def convert(mode: str, pattern: str) -> str:
    """Convert ``pattern`` exactly as ``patmatch_to_nrgrep.pl <mode> <pattern>``.

    ``mode`` is ``"-n"``, ``"-p"`` or ``"-c"`` (or ``"n"``/``"p"``/``"c"``).
    """
    kind = mode.lstrip("-")
    if kind not in ("n", "p", "c"):
        raise ValueError("Invalid class.")
    text = re.sub(r"\s", "", pattern).upper()
    if kind == "c":
        text = reverse_complement_pattern(text)
    text = text.replace("X", ".") if kind == "p" else text.replace("N", ".").replace("X", ".")
    text = _expand_repetitions(text)
    for letter, cls in (_PEPTIDE_CLASSES if kind == "p" else _NUCLEOTIDE_CLASSES):
        text = text.replace(letter, cls)
    text = _flatten_brackets(text)
    return _anchor_and_wrap(text)
