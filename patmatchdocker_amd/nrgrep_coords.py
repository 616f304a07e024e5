"""`nrgrep_coords`-compatible command line on the GPU engine.

Drop-in for the prebuilt binary the reference shells out to
(www/FlaskApp/FlaskApp/patmatch.py:733-742):

    nrgrep_coords -i -b <bufsize> -k <err>[idst] '<nrgrep pattern>' <file>...

prints the engine banner line ("SIMPLE search", ...) and one
"[beg, end]: <match>" line per reported match (the binary's own format
string "[%d, %d]: "), in increasing `beg` -- DESIGN.md §1.  Supported options are the ones
the reference passes: -i (required: the database is case-folded), -b
(accepted, ignored: records are never split here), -k.  An invalid pattern
prints nrgrep's "Syntax error in pattern" to stderr and exits 1 with no
output, like the binary; unsupported option combinations fail loudly.
"""

from __future__ import annotations

import argparse
import sys

from . import engine
from .regex import RegexSyntaxError, compile_pattern, engine_banner
from .service import _format_hits, parse_error_option


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="nrgrep_coords", add_help=False)
    ap.add_argument("-i", action="store_true")
    ap.add_argument("-b", type=int, default=None)
    ap.add_argument("-k", default="0")
    ap.add_argument("pattern")
    ap.add_argument("files", nargs="+")
    args = ap.parse_args(argv)
    if not args.i:
        print("nrgrep_coords (GPU): only case-insensitive search (-i) is supported", file=sys.stderr)
        return 2
    try:
        prog = compile_pattern(args.pattern, ignore_case=True)
    except RegexSyntaxError:
        print("Syntax error in pattern %s" % args.pattern, file=sys.stderr)
        return 1
    k, types = parse_error_option(args.k)
    out = sys.stdout
    out.write(engine_banner(prog, k) + "\n")   # searchPreproc's puts(), before any hit
    for path in args.files:
        db = engine.SequenceDatabase.from_file(path)
        try:
            (res,), _ = engine.scan(db, [prog], k=k, types=types)
            out.write(_format_hits(db, *res))
        finally:
            db.close()
    out.flush()
    return 0


if __name__ == "__main__":
    sys.exit(main())
