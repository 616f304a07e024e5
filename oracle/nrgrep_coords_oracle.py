#!/usr/bin/env python3
"""CPU oracle behind an nrgrep_coords-style command line.  TEST INFRASTRUCTURE
ONLY: used by tests/golden/make_e2e.py to run the reference's own Python
pipeline (www/FlaskApp/FlaskApp/patmatch.py run_test) with this oracle in
place of the prebuilt binary.  Prints what the binary prints:
the engine banner searchPreproc puts() ("SIMPLE search", ...), then one
"[beg, end]: match" line per reported match (record.c 0x402327-0x402383;
the output separator OptRecSep defaults to "" at 0x41cdd5)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import oracle  # noqa: E402
from patmatchdocker_amd.regex import RegexSyntaxError, compile_pattern, engine_banner  # noqa: E402


def main():
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("-i", action="store_true")
    ap.add_argument("-b")
    ap.add_argument("-k", default="0")
    ap.add_argument("pattern")
    ap.add_argument("files", nargs="+")
    a = ap.parse_args()
    k = int("".join(ch for ch in a.k if ch.isdigit()) or 0)
    types = "".join(ch for ch in a.k if ch in "idst") or "idst"
    try:
        prog = compile_pattern(a.pattern)
    except RegexSyntaxError:
        print("Syntax error in pattern %s" % a.pattern, file=sys.stderr)
        return 1
    print(engine_banner(prog, k))
    for path in a.files:
        text = open(path, "rb").read()
        for b, e in oracle.scan_reported(text, prog, k, types):
            sys.stdout.write("[%d, %d]: %s\n" % (b, e, text[b:e].decode("latin-1")))
    return 0


if __name__ == "__main__":
    sys.exit(main())
