import sys; sys.path.insert(0, ".")
from patmatchdocker_amd import engine
from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern
from oracle import oracle
from tests.fastagen import dna_fasta
text = dna_fasta(1, n_records=5, max_len=4000, width=None)
prog = compile_pattern("(GA(TC)(TC)?A)")
want = oracle.scan(text, prog, 0, "s", skip_headers=True)
print("n", len(text), "want", want)
for alpha in (engine.NUC, engine.BYTE):
    db = engine.SequenceDatabase.from_bytes(text, alphabet=alpha)
    r = engine.scan_nfa(db, prog, 0)
    print(alpha, "fresh", list(zip(r.beg.tolist(), r.end.tolist())))
    r = engine.scan_nfa(db, prog, 0)
    print(alpha, "again", list(zip(r.beg.tolist(), r.end.tolist())))
    p2 = compile_pattern("(A...?TC)")
    r = engine.scan_nfa(db, p2, 0)
    print(alpha, "other", len(r.beg), len(oracle.scan(text, p2, 0, "s", skip_headers=True)))
    for i in range(3):
        r = engine.scan_nfa(db, prog, 0)
        print(alpha, "after", list(zip(r.beg.tolist(), r.end.tolist())))
    # sub-texts
    db.close()
for cut in (2000, 2200, 3000, 6000):
    t = text[:cut]
    db = engine.SequenceDatabase.from_bytes(t, alphabet=engine.NUC)
    r = engine.scan_nfa(db, prog, 0)
    print("cut", cut, list(zip(r.beg.tolist(), r.end.tolist())), oracle.scan(t, prog, 0, "s", skip_headers=True))
    db.close()
