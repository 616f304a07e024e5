"""Regenerate the golden fixtures from the REFERENCE itself (run in the dev
container, where /root/reference exists; the GPU box never runs this).

* converter.json  -- `perl www/bin/patmatch_to_nrgrep.pl <mode> <pattern>` for
                     curated + seeded-random patterns (modes -n, -p, -c and the
                     -c-of-converted chain patmatch.py:296 uses);
* index.json      -- `perl www/bin/generate_sequence_index.pl < file`;
* host_logic.json -- the reference's own Python functions
                     (www/FlaskApp/FlaskApp/patmatch.py) imported from
                     /root/reference: check_pattern, cleanup_pattern,
                     find_exclusion_offset, get_name_offset, set_seq_length,
                     process_pattern (which itself shells out to the Perl
                     converter) and process_output on synthetic hit text.

Only data (inputs and outputs) is written; no reference source is copied.
"""
import importlib.util
import json
import os
import random
import shutil
import subprocess
import sys
import tempfile

REF = "/root/reference"
PERL_CONV = REF + "/www/bin/patmatch_to_nrgrep.pl"
PERL_INDEX = REF + "/www/bin/generate_sequence_index.pl"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))

from tests.fastagen import dna_fasta, pep_fasta  # noqa: E402

CURATED = ["GAATTC", "TATAWAWR", "<ATG", "TAA>", "<ATGNNN>", "CX{2,4}CX{3}[LIVMFYWC]", "(CA){2,3}", "A{3,}",
           "[RY]N{,4}GG", "acg tnn", "(TA[CT]A){2}", "GAN{2,3}TC", "A[^P]C", "[^P]CX{2}", "J{2}OBZ", "MKVHDB",
           "(A{2}T){2}", "[A[AG]]", "TA[ATAG]", "X{0,3}ACG", "((AT)G){1,2}", "TGANTCAGNNNTGAC", "C-X(2,4)-C",
           "NXS", "RGD", "[ST]X[RK]", "LXXLL", "KDEL>", "W{1,3}Y", "P[^P]G", "GA(TC){1,2}A", "TTNNNN{0,3}AA",
           "YYYRRRNNN", "{7V]A}", "{R9}D6C{Y", " {8}[K{[)"]


def perl(args, stdin=None):
    return subprocess.run(["perl"] + args, input=stdin, capture_output=True, timeout=1).stdout


def converter_vectors():
    rng = random.Random(20260227)
    pats = list(CURATED)
    alpha_n = "ACGTNRYSWMKVHDBX[](){},0123456789<> ^"
    alpha_p = "ACDEFGHIKLMNPQRSTVWYXJOBZ[](){},234<>^"
    for alpha in (alpha_n, alpha_p):
        for _ in range(120):
            pats.append("".join(rng.choice(alpha) for _ in range(rng.randint(1, 12))))
    out = []
    for pat in pats:
        for mode in ("-n", "-p", "-c"):
            try:
                res = perl([PERL_CONV, mode, pat]).decode("latin-1")
            except subprocess.TimeoutExpired:
                res = None          # the Perl loops forever on this input
            out.append({"mode": mode, "pattern": pat, "output": res})
            if mode == "-n" and res is not None:
                try:
                    comp = perl([PERL_CONV, "-c", res]).decode("latin-1")
                except subprocess.TimeoutExpired:
                    comp = None
                out.append({"mode": "-c", "pattern": res, "output": comp})
    return out


def index_vectors():
    files = [dna_fasta(1, 4, max_len=300), pep_fasta(2, 5, max_len=100),
             b">a\n\n>b desc\nACGT\n> not header\nAC\n>\n>c\tx\nGG", b"ACGT\n>x\nA", b"",
             dna_fasta(3, 3, max_len=200, width=50)]
    out = []
    for data in files:
        text = perl([PERL_INDEX], stdin=data).decode("latin-1")
        out.append({"fasta": data.decode("latin-1"), "index": text})
    return out


def load_reference_module(tmp):
    spec = importlib.util.spec_from_file_location("ref_patmatch", REF + "/www/FlaskApp/FlaskApp/patmatch.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod._set_dirs_for_test(REF, tmp + "/")
    mod.tmpDir = tmp + "/"
    return mod


def host_vectors():
    tmp = tempfile.mkdtemp()
    try:
        ref = load_reference_module(tmp)
        rng = random.Random(7)
        vec = {"check_pattern": [], "cleanup_pattern": [], "find_exclusion_offset": [], "get_name_offset": [],
               "process_pattern": [], "set_seq_length": [], "process_output": []}
        for pat in CURATED + ["AC", "ACG", "A(C)", "[AC]G", "(AC)", "u", "U", "AUG", "ELF", "{A}", "A{2}"]:
            for st in ("pep", "protein", "dna", "nuc", "DNA", None):
                vec["check_pattern"].append({"pattern": pat, "seqtype": st, "out": ref.check_pattern(pat, st)})
        for pat in ["%28A%29%7B2%2C3%7D%5BCG%5D%5E", "A%2CB", "plain"]:
            vec["cleanup_pattern"].append({"pattern": pat, "out": ref.cleanup_pattern(pat)})
        for pat in ["(A[^P]C)", "([^P]CX)", "(AB{2}[^P])", "(A*B+C?[^Q])", "(A{,3}B{2,}[^R][^S])", "(ABC)",
                    "([LIV]X{2}[^P])", "A.?B[^C]", "((G)[^T]A)", "XY{3,5}Z[^W]"]:
            vec["find_exclusion_offset"].append({"pattern": pat, "out": ref.find_exclusion_offset(pat)})
        for _ in range(60):
            n = rng.randint(1, 12)
            lst = sorted(rng.sample(range(0, 500), n))
            for _ in range(8):
                off = rng.randint(lst[0], 520)
                vec["get_name_offset"].append({"offset": off, "list": lst, "out": ref.get_name_offset(off, lst)})
        strands = [None, "Both strands", "Watson strand", "Reverse complement", "Crick complement"]
        for pat in ["GAATTC", "TATAWAWR", "GAN{2,3}TC", "CX{2,4}C", "NXS", "<ATG", "[^P]C"]:
            for st in ("dna", "pep", None, "nuc", "protein"):
                for strand in strands:
                    for ins, dele, sub, mm in ((None, None, None, None), ("insertion", None, None, "1"),
                                               (None, "deletion", "substitution", "2"), (None, None, "substitution", 0)):
                        res = ref.process_pattern(pat, st, strand, ins, dele, sub, mm)
                        vec["process_pattern"].append({"args": [pat, st, strand, ins, dele, sub, mm], "out": list(res)})
        fastas = {"orf_dna.seq": dna_fasta(5, 6, max_len=400), "orf_pep.seq": pep_fasta(6, 8, max_len=150),
                  "chrs.seq": dna_fasta(8, 3, max_len=500, width=60)}
        for name, data in fastas.items():
            with open(os.path.join(tmp, name), "wb") as fh:
                fh.write(data)
            lengths = {}
            stops = ref.set_seq_length(lengths, os.path.join(tmp, name))
            vec["set_seq_length"].append({"fasta": data.decode("latin-1"), "lengths": lengths, "stops": stops})
        with open(os.path.join(tmp, "locus.txt"), "w") as fh:
            for r in range(8):
                fh.write("YP%04d\tGENE%d\tS%06d\tdescription %d\n" % (r, r, r, r))
            fh.write("seq1\tseq1\tS000001\n")
        locus = open(os.path.join(tmp, "locus.txt")).read()
        # process_output on synthetic nrgrep_coords output
        for name, data in fastas.items():
            datafile = os.path.join(tmp, name)
            offsets, names = ref.get_record_offset(datafile)
            for trial in range(12):
                lines = []
                for _ in range(rng.randint(0, 40)):
                    b = rng.randrange(0, max(1, len(data) - 8))
                    e = b + rng.randint(1, 8)
                    lines.append("[%d, %d]: %s" % (b, e, data[b:e].decode("latin-1").replace("\n", "")))
                output = "\n".join(lines)
                beg, end = (1, 0) if trial % 4 == 1 else ((0, 1) if trial % 4 == 2 else (0, 0))
                maxhits = [None, "5", "no limit", "abc", 3, "100"][trial % 6]
                pattern = ["(GAATTC)", "(A[^C]G)", "(XY[^P][^Q])", "(ACG)"][trial % 4]
                dl = os.path.join(tmp, "dl.txt")
                res = ref.process_output(offsets, names, output, datafile, maxhits, beg, end, dl, pattern)
                vec["process_output"].append({
                    "fasta_name": name, "fasta": data.decode("latin-1"), "locus": locus, "output": output,
                    "maxhits": maxhits, "begMatch": beg, "endMatch": end, "pattern": pattern,
                    "result": [res[0], res[1], res[2], res[3]], "file": open(dl).read()})
        return vec
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    with open(os.path.join(OUT, "converter.json"), "w") as fh:
        json.dump(converter_vectors(), fh, indent=0)
    with open(os.path.join(OUT, "index.json"), "w") as fh:
        json.dump(index_vectors(), fh, indent=0)
    with open(os.path.join(OUT, "host_logic.json"), "w") as fh:
        json.dump(host_vectors(), fh, indent=0)


if __name__ == "__main__":
    main()
