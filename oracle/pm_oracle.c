/*
 * pm_oracle.c -- CPU restatement of the PatMatch scan ("nrgrep_coords").
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the
 * checker.  The product path (patmatchdocker_amd) never touches it.
 *
 * What it restates.  (Round 2: the report rules below were read from the
 * binary's disassembly -- objdump -d, never executed; DESIGN.md §1 cites the
 * addresses.  pmo_scan2 implements them, pmo_scan keeps the candidate list.)
 *
 * The reference runs, for every query and strand,
 *     nrgrep_coords -i -b 1600000 -k <k><ids> '<pattern>' '<datafile>'
 * (www/FlaskApp/FlaskApp/patmatch.py:733-742, run_test :818-828) and parses
 * lines "[beg, end]: <match>" (format string of the binary; parsed at
 * patmatch.py:505-516).  The binary is prebuilt (www/bin/nrgrep_coords,
 * nrgrep 1.1 by G. Navarro + coordinate printing) and is never run here; its
 * source is not in the reference.  The semantics below are this project's
 * restatement of it (see DESIGN.md "Scan semantics"):
 *
 *   - candidates (pmo_scan): for every start s of a record (the text
 *     between '\n' delimiters), the SHORTEST non-empty text[s, e) whose edit
 *     distance to the pattern's language is <= k, counting only the allowed
 *     operations (i = extra text char, d = missing pattern char, s =
 *     substitution); -i: ASCII letters compare case-insensitively;
 *   - k = 0 and a fixed-length class sequence (nrgrep's "simple" engine):
 *     the window [s, s+m) is checked against the whole text, line breaks
 *     and header bytes included (simple checkMatch 0x416790 never calls
 *     recGetRecord: simplePreproc sets its flag at 0x417f73);
 *   - reported (pmo_scan2, PMO_NRGREP): scanning regions [R, n) from R = 0,
 *     the first candidate with s >= R is printed and R = its end
 *     (recSearchFile 0x402250: searchScan, printf "[%d, %d]: " at 0x402356,
 *     resume at the match end 0x4022de-0x4022f4) -- matches never overlap;
 *   - '$' (PMO_END): e == n or text[e] == '\n'; '^' (PMO_START): s == 0,
 *     text[s-1] == '\n' or s == R (recCheckLeftContext 0x402170 compares
 *     with the region start);
 *   - beg = s (0-based byte offset in the file), end = e (exclusive).
 *
 * Parity status: the report rules and the simple engine are pinned by the
 * binary's code.  For variable-length patterns and k > 0
 * the binary reports, among overlapping candidates, the one its filter
 * finds first (factor/piece order chosen by a cost model, e.g.
 * simpleFindBest 0x416a10) with the latest start / earliest end around it;
 * this restatement takes the leftmost start and its shortest end -- equal
 * whenever candidates do not overlap, UNPINNED otherwise.  The pattern is given as its compiled position automaton
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
static int64_t match_from_e(const uint8_t* t, int64_t s, int64_t rec_end,
                            const uint64_t* B, uint64_t first, uint64_t last,
                            const uint64_t* follow, int k, int errs, int icase, int to_end) {
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
            /* '$' (to_end): nrgrep's forward verification keeps extending
             * while the right context fails (extended checkMatch 0x411eb0):
             * the end is the line end */
            if ((R[j] & last) && (!to_end || p + 1 == rec_end)) return p + 1;
            alive |= (R[j] != 0) | init[j];
        }
        if (!alive) return -1;
    }
    return -1;
}

static int64_t match_from(const uint8_t* t, int64_t s, int64_t rec_end,
                          const uint64_t* B, uint64_t first, uint64_t last,
                          const uint64_t* follow, int k, int errs, int icase) {
    return match_from_e(t, s, rec_end, B, first, last, follow, k, errs, icase, 0);
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

#define PMO_NRGREP 1
#define PMO_START 2
#define PMO_END 4
#define PMO_SIMPLE 8

/* k = 0 simple engine: window [s, s+m) against the whole text.  B holds
 * bit j for position j of the class sequence. */
static int simple_window(const uint8_t* t, int64_t s, int m, const uint64_t* B, int icase) {
    for (int j = 0; j < m; ++j) {
        const uint8_t c = icase ? fold(t[s + j]) : t[s + j];
        if (!((B[c] >> j) & 1)) return 0;
    }
    return 1;
}

/* What nrgrep_coords prints for one pattern (see the header comment).
 * mode: PMO_* bits.  Returns the number of hits (may exceed cap). */
int64_t pmo_scan2(const uint8_t* text, int64_t n, const uint64_t* B, uint64_t first,
                  uint64_t last, const uint64_t* follow, int m, int k, int errs,
                  int icase, int mode, int64_t* out_beg, int64_t* out_end, int64_t cap) {
    if (k < 0 || k > PMO_MAXK) return -1;
    int64_t count = 0, R = 0;
    int64_t rec_start = 0;
    const int simple = (mode & PMO_SIMPLE) != 0;
    if (simple && k != 0) return -1;
    while (rec_start <= n) {
        const uint8_t* nl = rec_start < n ? memchr(text + rec_start, '\n', (size_t)(n - rec_start)) : 0;
        int64_t rec_end = nl ? (int64_t)(nl - text) : n;
        /* the simple engine's windows may start on the delimiter itself */
        const int64_t s_end = simple ? (nl ? rec_end + 1 : n) : rec_end;
        for (int64_t s = rec_start; s < s_end; ++s) {
            int64_t e;
            if (simple) {
                e = (s + m <= n && simple_window(text, s, m, B, icase)) ? s + m : -1;
            } else {
                e = match_from_e(text, s, rec_end, B, first, last, follow, k, errs, icase, (mode & PMO_END) != 0);
            }
            if (e <= s) continue;
            if ((mode & PMO_END) && !(e == n || text[e] == '\n')) continue;
            if (mode & PMO_NRGREP) {
                if (s < R) continue;
                if ((mode & PMO_START) && !(s == R || s == 0 || text[s - 1] == '\n')) continue;
                R = e;
            } else if ((mode & PMO_START) && !(s == 0 || text[s - 1] == '\n')) {
                continue;
            }
            if (count < cap) { out_beg[count] = s; out_end[count] = e; }
            ++count;
        }
        rec_start = (nl ? rec_end : n) + 1;
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
