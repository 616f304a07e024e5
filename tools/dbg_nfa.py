import sys; sys.path.insert(0, ".")
from patmatchdocker_amd import engine
from patmatchdocker_amd.regex import compile_pattern
from oracle import oracle
for pat in ["(GA(TC)(TC)?A)", "(GATC(TC)?A)", "(GATCA)", "(GA(TC)A)", "(A...?TC)", "(GAT.?A)", "((GA)?TC)", "(GA(T)(TC)?A)"]:
    prog = compile_pattern(pat)
    for text in [b"GATCA\n", b"xxGATCTCAxx\n", b">h\nGATCAGATCTCA\n"]:
        for alpha in (engine.NUC, engine.BYTE):
            db = engine.SequenceDatabase.from_bytes(text, alphabet=alpha)
            r = engine.scan_nfa(db, prog, 0)
            got = list(zip(r.beg.tolist(), r.end.tolist()))
            want = oracle.scan(text, prog, 0, "s", skip_headers=True)
            print("OK " if got == want else "BAD", pat, text, alpha, got, want, "m=%d first=%x last=%x maxlen=%s" % (prog.m, prog.first, prog.last, prog.max_len), prog.follow)
            db.close()
