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
#include <stdlib.h>
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

/*
 * pmc_ids_scan -- bit-parallel scan with insertions / deletions /
 * substitutions (`-k <k>ids`) for a class sequence, line-bounded, reported
 * as nrgrep_coords prints (first found wins, the scan resumes at its end).
 * The Wu-Manber recurrence nrgrep's e* engines run, one 64-bit word per
 * error row: a reverse pass over each line finds every start of a match
 * (the automaton of the reversed pattern, the same recurrence as the GPU
 * start pass k_nfa_rev / pm_ids.hip), a forward pass from each start finds
 * its shortest end, then the report rule.  B[c] bit j: byte c (folded) is
 * in class j.  errs: 1 = insertion, 2 = deletion, 4 = substitution.
 * Returns the number of reported matches (written while < cap), -1 if the
 * shape is not covered (m > 64, k > 15, deletions with k >= m).
 */
#define PMC_MAXK 15

int64_t pmc_ids_scan(const uint8_t* text, int64_t n, const uint64_t* B, int m, int k, int errs, int icase,
                     int64_t* out_beg, int64_t* out_end, int64_t cap) {
    if (m < 1 || m > 64 || k < 0 || k > PMC_MAXK || ((errs & 2) && k >= m)) return -1;
    const int ins = errs & 1, del = errs & 2, sub = errs & 4;
    const uint64_t last = 1ull << (m - 1), first = 1ull;
    const uint64_t mmask = m == 64 ? ~0ull : ((1ull << m) - 1);
    uint64_t T[256];
    for (int c = 0; c < 256; ++c) T[c] = c == '\n' ? 0 : B[icase ? fold((uint8_t)c) : (uint8_t)c];
    /* start configurations (pm_nfa.hip scan_nfa): reverse injected rows and
     * the forward deletion closure of the start */
    uint64_t rev_pre[PMC_MAXK + 1], rev_ins[PMC_MAXK + 1], fwd_del[PMC_MAXK + 1];
    {
        uint64_t S = 0, F = 0;
        for (int j = 0; j <= k; ++j) {
            rev_ins[j] = S;
            rev_pre[j] = (S >> 1) | ((j == 0 || ins) ? last : 0);
            fwd_del[j] = F;
            if (del) {
                S = (S >> 1) | ((j == 0 || ins) ? last : 0);
                F = ((F << 1) & mmask) | (j == 0 ? first : 0);
            }
        }
    }
    int64_t count = 0, R = 0;
    int64_t* starts = 0;
    int64_t scap = 0;
    int64_t ls = 0;
    while (ls <= n) {
        int64_t le = ls;
        while (le < n && text[le] != '\n') ++le;
        /* reverse pass over [ls, le): candidate starts, right to left */
        int64_t ns = 0;
        uint64_t Rr[PMC_MAXK + 1], A[PMC_MAXK + 1], N[PMC_MAXK + 1];
        for (int j = 0; j <= k; ++j) Rr[j] = 0;
        for (int64_t p = le; p-- > ls;) {
            const uint64_t bc = T[text[p]];
            for (int j = 0; j <= k; ++j) A[j] = (Rr[j] >> 1) | rev_pre[j];
            for (int j = 0; j <= k; ++j) {
                N[j] = A[j] & bc;
                if (j > 0) {
                    if (sub) N[j] |= A[j - 1];
                    if (ins) N[j] |= Rr[j - 1] | rev_ins[j - 1];
                }
            }
            if (del)
                for (int j = 0; j < k; ++j) N[j + 1] |= (N[j] >> 1) | ((j >= 1 && ins) ? last : 0);
            uint64_t any = 0;
            for (int j = 0; j <= k; ++j) {
                Rr[j] = N[j];
                any |= N[j];
            }
            if (any & first) {
                if (ns == scap) {
                    scap = scap ? 2 * scap : 1024;
                    starts = (int64_t*)realloc(starts, (size_t)scap * sizeof(int64_t));
                }
                starts[ns++] = p;
            }
        }
        /* forward verify + report rule, left to right */
        for (int64_t q = ns; q-- > 0;) {
            const int64_t s = starts[q];
            if (s < R) continue;
            uint64_t F[PMC_MAXK + 1], Af[PMC_MAXK + 1], Nf[PMC_MAXK + 1];
            int init[PMC_MAXK + 1], ninit[PMC_MAXK + 1];
            for (int j = 0; j <= k; ++j) {
                F[j] = fwd_del[j];
                init[j] = j == 0;
            }
            int64_t e = -1;
            for (int64_t p = s; p < le; ++p) {
                const uint64_t bc = T[text[p]];
                for (int j = 0; j <= k; ++j) Af[j] = ((F[j] << 1) & mmask) | (init[j] ? first : 0);
                for (int j = 0; j <= k; ++j) {
                    Nf[j] = Af[j] & bc;
                    ninit[j] = 0;
                    if (j > 0) {
                        if (sub) Nf[j] |= Af[j - 1];
                        if (ins) {
                            Nf[j] |= F[j - 1];
                            ninit[j] = init[j - 1];
                        }
                    }
                }
                if (del)
                    for (int j = 0; j < k; ++j) Nf[j + 1] |= ((Nf[j] << 1) & mmask) | (ninit[j] ? first : 0);
                uint64_t any = 0;
                int alive = 0;
                for (int j = 0; j <= k; ++j) {
                    F[j] = Nf[j];
                    init[j] = ninit[j];
                    any |= Nf[j];
                    alive |= ninit[j];
                }
                if (any & last) {
                    e = p + 1;
                    break;
                }
                if (!any && !alive) break;
            }
            if (e < 0) continue;   /* cannot happen for a start of the reverse pass */
            if (count < cap) {
                out_beg[count] = s;
                out_end[count] = e;
            }
            ++count;
            R = e;
        }
        ls = le + 1;
    }
    free(starts);
    return count;
}
