"""Seeded synthetic FASTA generators for the parity tests."""
import random

DNA = b"ACGT"
PEP = b"ACDEFGHIKLMNPQRSTVWY"


def dna_fasta(seed, n_records=6, min_len=0, max_len=3000, noise=True, width=None):
    rng = random.Random(seed)
    out = bytearray()
    for r in range(n_records):
        out += b">seq%d some description %d\n" % (r, rng.randint(0, 99))
        n = rng.randint(min_len, max_len)
        s = bytearray(rng.choice(DNA) for _ in range(n))
        if noise and n:
            for _ in range(max(1, n // 200)):
                i = rng.randrange(n)
                s[i] = rng.choice(b"NnacgtRY")
            if rng.random() < 0.5:
                i = rng.randrange(n)
                s[i:i + 40] = b"N" * len(s[i:i + 40])
        if width:
            for i in range(0, len(s), width):
                out += s[i:i + width] + b"\n"
        else:
            out += s + b"\n"
    return bytes(out)


def pep_fasta(seed, n_records=20, max_len=600):
    rng = random.Random(seed)
    out = bytearray()
    for r in range(n_records):
        out += b">YP%04d G%d SGDID:S%06d, protein\n" % (r, r, r)
        n = rng.randint(0, max_len)
        s = bytes(rng.choice(PEP) for _ in range(n))
        out += s + (b"*" if rng.random() < 0.7 else b"") + b"\n"
    return bytes(out)
