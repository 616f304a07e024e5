/*
 * pm_oracle.c -- CPU restatement of the PatMatch scan ("nrgrep_coords").
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the
 * checker.  The product path (patmatchdocker_amd) never touches it.
 *
 * What it restates.  The reference runs, for every query and strand,
 *     nrgrep_coords -i -b 1600000 -k <k><ids> '<pattern>' '<datafile>'
 * (www/FlaskApp/FlaskApp/patmatch.py:733-742, run_test :818-828) and parses
 * lines "[beg, end]: <match>" (format string of the binary; parsed at
 * patmatch.py:505-516).  The binary is prebuilt (www/bin/nrgrep_coords,
 * nrgrep 1.1 by G. Navarro + coordinate printing) and is never run here; its
 * source is not in the reference.  The semantics below are this project's
 * restatement of it (see DESIGN.md "Scan semantics"):
 *
 *   - records are the text between '\n' delimiters; no match spans one;
 *   - -i: ASCII letters compare case-insensitively;
 *   - for every start s of a record, in increasing order, report the
 *     SHORTEST non-empty text[s, e) whose edit distance to the pattern's
 *     language is <= k, counting only the allowed operations
 *     (i = extra text char, d = missing pattern char, s = substitution);
 *   - beg = s (0-based byte offset in the file), end = e (exclusive).
 *
 * Parity status: pinned against the reference's converter and host logic
 * (tests/golden), UNPINNED against the nrgrep_coords binary itself, which
 * cannot be run.  The pattern is given as its compiled position automaton
 * (patmatchdocker_amd/regex.py): B[256] byte masks, first/last masks and
 * follow[m], m <= 64.  This file deliberately uses a different algorithm
 * (per-start forward simulation, O(n * alive-length)) from the GPU kernels.
 */
#include <stdint.h>
#include <string.h>

#define PMO_ERR_INS 1
#define PMO_ERR_DEL 2
#define PMO_ERR_SUB 4
#define PMO_MAXK 16

static inline uint8_t fold(uint8_t c) { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; }

static inline uint64_t follow_of(uint64_t set, const uint64_t* follow) {
    uint64_t out = 0;
    while (set) {
        int i = __builtin_ctzll(set);
        out |= follow[i];
        set &= set - 1;
    }
    return out;
}

/* One start: returns e (> s) or -1.  Rows R[j] = positions active with j
 * errors; init[j] = the "before the first pattern character" state with j
 * errors (kept alive by insertions). */
static int64_t match_from(const uint8_t* t, int64_t s, int64_t rec_end,
                          const uint64_t* B, uint64_t first, uint64_t last,
                          const uint64_t* follow, int k, int errs, int icase) {
    uint64_t R[PMO_MAXK + 1], N[PMO_MAXK + 1];
    int init[PMO_MAXK + 1], ninit[PMO_MAXK + 1];
    for (int j = 0; j <= k; ++j) { R[j] = 0; init[j] = (j == 0); }
    /* deletion closure of the start configuration */
    if (errs & PMO_ERR_DEL)
        for (int j = 0; j < k; ++j)
            R[j + 1] |= follow_of(R[j], follow) | (init[j] ? first : 0);
    for (int64_t p = s; p < rec_end; ++p) {
        uint8_t c = icase ? fold(t[p]) : t[p];
        uint64_t bc = B[c];
        int alive = 0;
        for (int j = 0; j <= k; ++j) {
            uint64_t adv = follow_of(R[j], follow) | (init[j] ? first : 0);
            N[j] = adv & bc;
            ninit[j] = 0;
            if (j > 0) {
                if (errs & PMO_ERR_SUB)
                    N[j] |= follow_of(R[j - 1], follow) | (init[j - 1] ? first : 0);
                if (errs & PMO_ERR_INS) {
                    N[j] |= R[j - 1];
                    ninit[j] = init[j - 1];
                }
            }
        }
        if (errs & PMO_ERR_DEL)
            for (int j = 0; j < k; ++j)
                N[j + 1] |= follow_of(N[j], follow) | (ninit[j] ? first : 0);
        for (int j = 0; j <= k; ++j) {
            R[j] = N[j];
            init[j] = ninit[j];
            if (R[j] & last) return p + 1;
            alive |= (R[j] != 0) | init[j];
        }
        if (!alive) return -1;
    }
    return -1;
}

/* Scan the whole text.  Writes up to cap hits; returns the total number of
 * hits (which may exceed cap: call again with a bigger buffer). */
int64_t pmo_scan(const uint8_t* text, int64_t n, const uint64_t* B, uint64_t first,
                 uint64_t last, const uint64_t* follow, int m, int k, int errs,
                 int icase, int64_t* out_beg, int64_t* out_end, int64_t cap) {
    (void)m;
    if (k < 0 || k > PMO_MAXK) return -1;
    int64_t count = 0;
    int64_t rec_start = 0;
    while (rec_start <= n) {
        const uint8_t* nl = rec_start < n ? memchr(text + rec_start, '\n', (size_t)(n - rec_start)) : 0;
        int64_t rec_end = nl ? (int64_t)(nl - text) : n;
        for (int64_t s = rec_start; s < rec_end; ++s) {
            int64_t e = match_from(text, s, rec_end, B, first, last, follow, k, errs, icase);
            if (e > s) {
                if (count < cap) { out_beg[count] = s; out_end[count] = e; }
                ++count;
            }
        }
        rec_start = rec_end + 1;
    }
    return count;
}

/* Record index restatement (www/bin/generate_sequence_index.pl): for every
 * line matching /^>(\S+)/ emit (offset of the line, ">name") and (offset of
 * the next line, "name").  Returns the number of header lines found; for
 * each it stores the header-line offset and the name's [start, len). */
int64_t pmo_index(const uint8_t* text, int64_t n, int64_t* hdr_off, int64_t* data_off,
                  int64_t* name_beg, int64_t* name_len, int64_t cap) {
    int64_t count = 0, p = 0;
    while (p < n) {
        const uint8_t* nl = memchr(text + p, '\n', (size_t)(n - p));
        int64_t end = nl ? (int64_t)(nl - text) + 1 : n;   /* includes '\n' */
        if (text[p] == '>' && p + 1 < end) {
            int64_t q = p + 1;
            while (q < end && !(text[q] == ' ' || text[q] == '\t' || text[q] == '\n' ||
                                text[q] == '\r' || text[q] == '\f' || text[q] == '\v'))
                ++q;
            if (q > p + 1) {
                if (count < cap) {
                    hdr_off[count] = p; data_off[count] = end;
                    name_beg[count] = p + 1; name_len[count] = q - p - 1;
                }
                ++count;
            }
        }
        p = end;
    }
    return count;
}
