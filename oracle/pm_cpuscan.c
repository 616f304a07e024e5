/*
 * pm_cpuscan.c -- bit-parallel CPU scan for the bench's CPU baseline.
 *
 * MEASUREMENT INFRASTRUCTURE ONLY (like pm_oracle.c): bench.py's cpu_baseline
 * leg times it and tests/ check it; the product path never loads it.
 *
 * What the reference does on the host: nrgrep_coords (patmatch.py:733-743)
 * scans with bit-parallel automata -- for a class sequence with k errors its
 * esimple engine (nrgrep 1.1, disassembled: esimpleScan 0x4136d0) runs a
 * forward bit-parallel automaton or a piece filter, one machine word of state
 * per text character.  This file restates that family for substitutions:
 * Shift-Add (Baeza-Yates & Gonnet 1992).  One 64-bit state word holds, for
 * every pattern position i, the mismatch count of pattern[0..i] against the
 * text ending at the current character, in fields of b bits (2^(b-1) > k);
 * per character: S = (S << b) + T[c]; overflow bits move to O.  A window
 * ends at the current character iff field m-1 is <= k with no overflow.
 * ~6 ALU ops per character and pattern, no branches in the inner loop.
 *
 * Semantics match pmo_scan2 for fixed-length class sequences:
 * k > 0 (esimple) windows stay inside a line (the state resets at '\n');
 * k = 0 (simple) windows may span it; the report rule keeps the first
 * window found and resumes at its end.
 */
#include <stdint.h>
#include <string.h>

static inline uint8_t fold(uint8_t c) { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; }

/* B[c] bit j: byte c (folded) is in class j.  Returns the number of reported
 * windows (beg written to out_beg while < cap), or -1 if m * b > 64. */
int64_t pmc_shiftadd(const uint8_t* text, int64_t n, const uint64_t* B, int m, int k, int icase,
                     int64_t* out_beg, int64_t cap) {
    int b = 1;
    while ((1 << (b - 1)) <= k) ++b;            /* 2^(b-1) > k */
    if (m < 1 || m * b > 64) return -1;
    const uint64_t mask = (m * b == 64) ? ~0ull : ((1ull << (m * b)) - 1);
    uint64_t H = 0;                              /* high bit of every field */
    for (int i = 0; i < m; ++i) H |= 1ull << (i * b + b - 1);
    uint64_t T[256];
    for (int c = 0; c < 256; ++c) {
        const uint8_t f = icase ? fold((uint8_t)c) : (uint8_t)c;
        uint64_t t = 0;
        for (int i = 0; i < m; ++i)
            if (!((B[f] >> i) & 1)) t |= 1ull << (i * b);
        T[c] = t;
    }
    const int sh_last = (m - 1) * b;
    const uint64_t last_val = ((1ull << (b - 1)) - 1) << sh_last;   /* value bits of field m-1 */
    const uint64_t last_ovf = 1ull << (sh_last + b - 1);
    const int line_bounded = k > 0;
    uint64_t S = 0, O = mask;                   /* nothing matched yet: every field overflowed */
    int64_t count = 0, R = 0;
    for (int64_t p = 0; p < n; ++p) {
        const uint8_t c = text[p];
        if (line_bounded && c == '\n') {         /* no window spans the delimiter */
            S = 0;
            O = mask;
            continue;
        }
        S = (S << b) + T[c];
        O = ((O << b) | (S & H)) & mask;
        S &= ~H & mask;
        if (!(O & last_ovf) && (uint64_t)((S & last_val) >> sh_last) <= (uint64_t)k) {
            const int64_t s = p - m + 1;
            if (s >= R) {                        /* report rule: resume at the match end */
                if (count < cap) out_beg[count] = s;
                ++count;
                R = p + 1;
            }
        }
    }
    return count;
}
