"""End-to-end fixtures: the REFERENCE's run_test (www/FlaskApp/FlaskApp/
patmatch.py:768-838, its Perl converter and generate_sequence_index.pl, its
process_output) with oracle/nrgrep_coords_oracle.py standing in for the
prebuilt nrgrep_coords binary.  Run in the dev container (needs
/root/reference); writes tests/golden/e2e.json (inputs + outputs only)."""
import importlib.util
import json
import os
import shutil
import sys
import tempfile

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from tests.fastagen import dna_fasta, pep_fasta  # noqa: E402

QUERIES = [
    # pattern, seqtype, strand, insertion, deletion, substitution, mismatch, max_hits
    ("GAATTC", "dna", None, None, None, None, None, 500),
    ("TATAWAWR", "dna", "Both strands", None, None, None, None, "no limit"),
    ("GAN{2,3}TC", "dna", None, None, None, None, None, 50),
    ("<ATG", "dna", None, None, None, None, None, 500),
    ("TAA>", "dna", None, None, None, None, None, 500),
    ("CCAAT", "dna", "Watson strand", None, None, "substitution", "1", 100),
    ("TGANTCA", "dna", "Reverse complement", None, None, "substitution", "2", 100),
    ("GGNCC", "dna", None, None, None, "substitution", "1", 7),
    ("CX{2,4}CX{3}[LIVMFYWC]", "pep", None, None, None, None, None, 500),
    ("NXS", "pep", None, None, None, None, None, "no limit"),
    ("[^P]CX", "pep", None, None, None, None, None, 500),
    ("KDEL>", "pep", None, None, None, None, None, 500),
    ("<MSK", "protein", None, None, None, None, None, 20),
    ("<ATGNNN", "dna", "Both strands", None, None, None, None, 500),
    ("NNNTAA>", "dna", None, None, None, None, None, 500),
    ("RGD", "pep", None, None, None, "substitution", "1", 200),
    # insertions / deletions (-k <k><ids>; no checkbox = all three, patmatch.py:308)
    ("GAATTC", "dna", None, None, None, None, "1", 300),
    ("TATAWAWR", "dna", "Both strands", "insertion", "deletion", None, "1", "no limit"),
    ("CCAAT", "dna", None, None, "deletion", "substitution", "1", 100),
    ("GGNCC", "dna", "Watson strand", "insertion", None, None, "2", 50),
    ("CX{2,4}CX{3}[LIVMFYWC]", "pep", None, "insertion", None, None, "1", 500),
    ("RGD", "pep", None, None, None, None, "2", 200),
    ("KDEL>", "pep", None, None, "deletion", None, "1", 500),
    # unbounded repeats ({m,} -> nrgrep '*')
    ("GA{2,}TC", "dna", None, None, None, None, None, 500),
    ("CX{3,}C", "pep", None, None, None, "substitution", "1", 300),
    # the extended engine's window away from the pattern start (nearest
    # start from the window) and nrgrep's simplify at the pattern edges
    ("AN{0,3}GAATTC", "dna", "Both strands", None, None, None, None, 500),
    ("TTN{0,3}NNNAA", "dna", None, None, None, None, None, 500),
    ("N{0,3}GAATTCN{0,3}", "dna", None, None, None, None, None, 500),
    ("CX{1,3}CX{2}C", "pep", None, None, None, None, None, 500),
    # ranges at k > 0: nrgrep's eextended engine (configs[3] at -k 1ids)
    ("CX{2,4}CX{3}[LIVMFYWC]", "pep", None, None, None, None, "1", 500),
    ("GAN{2,3}TC", "dna", None, None, None, None, "1", 300),
    ("AN{0,3}GAATTC", "dna", "Both strands", None, None, "substitution", "2", 300),
    ("CX{1,3}CK", "pep", None, "insertion", "deletion", None, "2", 300),
    # repeated groups: nrgrep's regular engine (k = 0) and eregular engine
    # (k > 0); the -c strand of a group repeat is an extended pattern
    ("GA(TC){1,2}A", "dna", None, None, None, None, None, 500),
    ("GA(TC){1,2}A", "dna", None, None, None, None, "1", 500),
    ("G(TATA){2,}C", "dna", "Watson strand", None, None, "substitution", "1", 300),
    ("(CA){2,4}GT", "dna", None, "insertion", "deletion", None, "2", 300),
    ("C(AG){1,3}L", "pep", None, None, None, None, "1", 300),
    ("K(RK){1,2}XXC", "pep", None, None, None, "substitution", "2", 300),
    # group repeats past 63 positions at k > 0 (round 6: the multi-word
    # eregular verify, its sliced transition tables included)
    ("(CA){37,38}G", "dna", None, None, None, None, "1", 300),
    ("(GATC){8,16}T", "dna", "Both strands", None, None, None, "1", 300),
    ("(CA){20,40}GT", "dna", None, "insertion", "deletion", None, "1", 300),
    ("AC", "pep", None, None, None, None, None, 500),          # below MIN_TOKEN
    ("EFL", "dna", None, None, None, None, None, 500),        # invalid nucleotide
]


def main():
    tmp = tempfile.mkdtemp()
    try:
        files = {"orf_dna.seq": dna_fasta(101, 12, max_len=2500, noise=True)
                 + b">orfA orfA desc\nATGAAACCCGGGAATTCTTTTAA\n>orfB\nATGCATGCTAA\n>orfC x\natgtataaaagtaa\n"
                 + b">orfR repeats\nTT" + b"CA" * 38 + b"GTTA" + b"GATC" * 9 + b"TAA" + b"CA" * 25 + b"GT"
                 + b"CC" + b"CA" * 18 + b"GCA" + b"CA" * 18 + b"GTT\n",
                 "orf_pep.seq": pep_fasta(102, 60, max_len=500)
                 + b">YPX1 X SGDID:S1, p\nMSKCAACGGGCLNASKDEL*\n>YPX2\nMSKDEL\n"}
        for name, data in files.items():
            open(os.path.join(tmp, name), "wb").write(data)
        locus = "".join("YP%04d\tG%d\tS%06d\tprotein %d\n" % (r, r, r, r) for r in range(60))
        locus += "".join("seq%d\tGENE%d\tS9%05d\tdna record %d\n" % (r, r, r, r) for r in range(0, 12, 2))
        open(os.path.join(tmp, "locus.txt"), "w").write(locus)
        spec = importlib.util.spec_from_file_location("ref_patmatch", REF + "/www/FlaskApp/FlaskApp/patmatch.py")
        ref = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(ref)
        ref.dataDir = tmp + "/"
        ref.tmpDir = tmp + "/"
        ref.patternConvertScript = REF + "/www/bin/patmatch_to_nrgrep.pl"
        ref.seqIndexCreateScript = REF + "/www/bin/generate_sequence_index.pl"
        ref.searchScript = os.path.join(ROOT, "oracle", "nrgrep_coords_oracle.py")
        cases = []
        for q in QUERIES:
            pattern, seqtype, strand, ins, dele, sub, mm, maxhits = q
            res = ref.run_test(pattern, seqtype=seqtype, strand=strand, insertion=ins, deletion=dele,
                               substitution=sub, mismatch=mm, max_hits=maxhits)
            dl = os.path.join(tmp, "patmatch.6688")
            cases.append({"query": list(q), "result": list(res),
                          "file": open(dl).read() if os.path.exists(dl) else None})
            if os.path.exists(dl):
                os.remove(dl)
        json.dump({"files": {k: v.decode("latin-1") for k, v in files.items()}, "locus": locus, "cases": cases},
                  open(os.path.join(HERE, "e2e.json"), "w"), indent=0)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
