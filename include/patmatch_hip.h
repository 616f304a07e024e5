/*
 * patmatch_hip.h -- C ABI of the MI355X PatMatch scan engine (libpatmatch_hip.so).
 *
 * The reference's only boundary on this path is a process boundary: the
 * Flask service shells out to the prebuilt nrgrep_coords binary
 *     nrgrep_coords -i -b 1600000 -k <k><ids> '<nrgrep pattern>' '<datafile>'
 * (www/FlaskApp/FlaskApp/patmatch.py:733-742 for run_patmatch and :818-828
 * for run_test) and parses its "[beg, end]: <match>" lines (:505-516).
 * The entry points below replace that binary.  Pattern compilation (PatMatch
 * syntax -> nrgrep syntax -> position automaton -> per-character bitmasks)
 * stays on the host (patmatchdocker_amd/convert.py, regex.py); this library
 * owns the device-resident sequence database and the scan kernels.
 *
 * Conventions: every function returns 0 on success and a negative PM_E_*
 * code on failure; pm_last_error() then describes the failure (per thread).
 * Positions are 0-based byte offsets into the FASTA file that was loaded,
 * "end" is exclusive -- the same numbers nrgrep_coords prints.
 * No function takes or returns framework (torch) types.
 */
#ifndef PATMATCH_HIP_H
#define PATMATCH_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PM_OK 0
#define PM_E_ARG (-1)      /* bad argument / unsupported shape            */
#define PM_E_HIP (-2)      /* HIP runtime error                           */
#define PM_E_NODEV (-3)    /* no usable GPU                               */
#define PM_E_UNSUPPORTED (-4)

#define PM_ALPHA_NUC 0     /* 2-bit A/C/G/T planes + sparse exceptions    */
#define PM_ALPHA_BYTE 1    /* one folded byte per residue (peptides)      */

#define PM_MAX_POSITIONS 256        /* automaton positions (pm_scan_nfa_wide)   */
#define PM_MAX_K 15                 /* errors (pm_scan_nfa_wide; <= 7 above 128 positions) */
#define PM_MAX_LINEAR_POSITIONS 64  /* pattern length of pm_scan_linear          */
#define PM_MAX_LINEAR_K 3           /* substitutions of pm_scan_linear           */

typedef struct pm_db pm_db;        /* device-resident sequence database   */
typedef struct pm_hits pm_hits;    /* device/host hit list of one scan    */

const char* pm_last_error(void);
const char* pm_version(void);
int pm_device_count(int* count);

/* --- database ----------------------------------------------------------
 * Replaces nrgrep's per-call read of '<datafile>' (the file is uploaded once
 * and stays in HBM).  `fasta` is the raw file content.  Header lines
 * (/^>\S/, generate_sequence_index.pl:33) and '\n' become record breaks.
 * `stream` is a hipStream_t (NULL = the library's own stream).          */
int pm_db_create(const uint8_t* fasta, uint64_t n, int alphabet, int device,
                 void* stream, pm_db** out);
/* Synthetic nucleotide database generated on the device: n_records records
 * laid out like a FASTA file (">r%08u\n" header line, rec_len random bases,
 * "\n"), bases from a counter-based hash of (seed, position); every record
 * holds one run of 50..499 N and IUPAC letters at ~1e-5 of its bases, so
 * scans exercise the exception path as on a real genome.               */
int pm_db_create_synthetic(uint64_t n_records, uint64_t rec_len, uint64_t seed,
                           int device, void* stream, pm_db** out);
/* nrgrep reads '<datafile>' in buffers of -b BYTES (patmatch.py:733-743
 * passes -b 1600000; main() stores atoi(optarg) in OptBufSize, 0x401162, and
 * bufCreate allocates that many bytes, 0x41bb6b -- the help text's "Kb"
 * is not applied).  Each buffer that is not the file's last is searched up
 * to and including its last line break, and the next buffer starts at that
 * line break (recSearchFile 0x402450-0x402497, bufLoad 0x41bbf0); a buffer without one
 * is searched whole.  These search regions matter to what is printed: no
 * match spans a region end, the report rule restarts at each region start,
 * and '^' passes there.  pm_db_create* set the regions of the loaded text
 * read with PM_NRGREP_BUFFER; pm_db_set_regions replaces them (a piece of a
 * larger file takes the file's regions, shifted; `count` = 1, [0, n): none).
 * Region r = [starts[r], ends[r]), starts increasing from 0.             */
#define PM_NRGREP_BUFFER 1600000ull
int pm_db_set_regions(pm_db* db, uint64_t count, const uint64_t* starts, const uint64_t* ends);
/* The current regions: *count of them, the first `cap` copied out.       */
int pm_db_regions(const pm_db* db, uint64_t cap, uint64_t* starts, uint64_t* ends, uint64_t* count);
int pm_db_destroy(pm_db* db);
int pm_db_info(const pm_db* db, uint64_t* n_positions, int* alphabet,
               uint64_t* n_exception_words, uint64_t* device_bytes);
/* BYTE databases (peptides): the folded bytes are also held as 5-bit
 * residue codes in five bit-planes (north_star's 5-bit packing: 0.625 byte
 * per residue); code 0 = a header byte or the padding, 1 = '\n', 2..31 =
 * the file's other distinct bytes in increasing order.  pm_scan_linear
 * scans the planes (one lane per 32 window starts, bit-parallel class
 * tests; windows over header text are re-checked on the file's bytes)
 * unless PM_SCAN_BYTES is set.  *n_codes = the highest code in use, 0 when
 * there are no planes (a nucleotide database, or more than 30 distinct
 * bytes besides '\n': the byte copy is scanned);
 * code_of_byte (256 entries, may be NULL) gets each byte's code.  Replaces
 * nothing in the reference (nrgrep reads the file's bytes).            */
int pm_db_residue_codes(const pm_db* db, int* n_codes, uint8_t* code_of_byte);
/* Decode positions [beg, beg+len) back to folded text (bench/debug). */
int pm_db_decode(pm_db* db, uint64_t beg, uint32_t len, uint8_t* out);

/* --- what a scan reports (the `flags` argument) ---------------------------
 * The kernels find candidates: every start with a match.  nrgrep_coords
 * prints a subset (from the binary's own code): the scan of a
 * region [R, end of text) returns the first match it finds, prints it and
 * resumes at the match's end (record.c recSearchFile), so reported matches
 * never overlap.  PM_REPORT_NRGREP applies that selection (the drop-in
 * behaviour); PM_REPORT_ALL keeps every candidate.  A pattern whose first
 * character was '^' / last was '$' is searched with the anchor stripped
 * and PM_ANCHOR_START / PM_ANCHOR_END set (nrgrep main(): OptStartLine /
 * OptEndLine): the match must start at a line start or where the previous
 * report ended / end at a line end.  Hits starting on a header line are
 * not returned (process_output discards them, patmatch.py:548) unless
 * PM_KEEP_HEADERS is set: a caller that joins the scans of consecutive
 * pieces of one file needs them, since they take part in the report rule
 * (patmatchdocker_amd/shards.py).                                         */
#define PM_REPORT_ALL 0
#define PM_REPORT_NRGREP 1
#define PM_ANCHOR_START 2
#define PM_ANCHOR_END 4
#define PM_KEEP_HEADERS 8
/* pm_scan_nfa_wide only: nrgrep's simple engine (k = 0, a class sequence):
 * windows are checked against the file's own bytes and may span a line
 * break (pm_scan_linear decides this by itself).                          */
#define PM_CROSS_LINES 16
/* pm_scan_linear on a BYTE database: scan the byte copy instead of the
 * 5-bit residue planes (A/B and tests; same hits).                        */
#define PM_SCAN_BYTES 256
/* pm_scan_nfa_errs / _wide / _tree: return once the report pass is queued
 * (no host wait for it); the list's count resolves on first use, as for
 * pm_scan_linear_async, so a caller launches its next scan (the other
 * strand) while this one's report runs.  Same results.                  */
#define PM_PIPELINED 1024
/* The pattern is a class sequence (nrgrep's detClass() == 1) searched with
 * k > 0 errors: nrgrep_coords runs its "esimple" engine (searchPreproc
 * 0x402710), whose own candidate order and two-phase verification decide
 * which overlapping match is printed.  pm_scan_linear sets it
 * by itself for k > 0; pm_scan_nfa_wide takes it from the caller.        */
#define PM_ESIMPLE 64
/* The scan plan nrgrep's esimplePreproc (0x415540) derives from the classes
 * of a class sequence with k errors (cost model over its letterProb table):
 * out[0] = 1 (k+1 pieces, BNDM), 2 (a window, ABNDM) or 3 (the prefix,
 * forward shift-or); out[1] = piece length; out[2..3] = simpleFindBest's
 * window; out[4] = number of pieces P; out[5 .. 5+P) = pattern positions
 * left of each piece / window.  byte_mask as in pm_scan_nfa_wide (the folded
 * byte's positions; classes hold both cases, as `-i` builds them).  Host
 * only, no GPU needed.  out must hold 5 + k + 1 ints.                    */
int pm_esimple_plan(int m, int words, const uint64_t* byte_mask, int k, int32_t* out);
/* The pattern is a sequence of classes each with an optional '?', '*' or '+'
 * (nrgrep's detClass() == 2): nrgrep_coords runs its "extended" engine at
 * k = 0 (searchPreproc 0x4026b7) and its "eextended" engine at k > 0
 * (0x402710), whose scanners and nearest-boundary verification decide which
 * overlapping match is printed.  pm_scan_nfa_wide only; the
 * optional / repeatable positions are read off first / follow / last
 * (PM_E_ARG if the automaton has another shape).                          */
#define PM_EXTENDED 128
/* The scan plan nrgrep's extendedPreproc (0x413260) derives for such a
 * pattern: out[0] = 2 (a window scanned backward) or 3 (the prefix scanned
 * forward); out[1] = the window's non-optional positions (0: no window);
 * out[2..3] = the window / prefix [beg, end); out[4] = pattern positions
 * left of the candidate; out[5] = 1 when the window holds no '?*+'.
 * opt_mask / rep_mask: `words` words of optional / repeatable positions.
 * Host only, no GPU needed.  out must hold 6 ints.                       */
int pm_extended_plan(int m, int words, const uint64_t* byte_mask, const uint64_t* opt_mask,
                     const uint64_t* rep_mask, int32_t* out);
/* The plan nrgrep's eextendedPreproc (0x40fe30) derives for such a pattern
 * at k errors (1..PM_MAX_K): out[0] = 1 (k + 1 pieces searched exactly), 2
 * (a window backward with k errors) or 3 (the prefix forward with k
 * errors); out[1] = 1 when the scanned positions hold no '?*+' (nrgrep then
 * runs its esimple scanners); out[2] = P, the pieces (1 for types 2 and 3);
 * out[3] = the pieces' length in characters (type 1) or the window's
 * non-optional positions; out[4..5] = extendedFindBest's window [beg, end);
 * out[6 + 2i], out[7 + 2i] = piece i's [off, end) (the window / prefix for
 * types 2 and 3).  Host only, no GPU needed.  out must hold 6 + 2 (k + 1)
 * ints.                                                                   */
int pm_eextended_plan(int m, int words, const uint64_t* byte_mask, const uint64_t* opt_mask,
                      const uint64_t* rep_mask, int k, int32_t* out);

/* --- fixed-length patterns: bit-sliced Hamming scan (nucleotide DB) -----
 * A batch of P linear patterns (sequences of classes, no ? * + |), matched
 * with at most k substitutions.  The classes are numbered 0..n_classes-1:
 *   class_acgt[c]     4-bit subset of {A,C,G,T} (bit0=A .. bit3=T)
 *   class_bytes[8*c]  256-bit membership over folded bytes (for non-ACGT
 *                     text bytes such as N)
 *   class_is_any[c]   1 if the class is '.' (accepts every byte)
 * pos_class[64*p + j] is the class of position j of pattern p, lengths[p]
 * its length (1..64).  Hits are (pattern, beg) with end = beg + lengths[p].
 * k = 0 is nrgrep's "simple" engine: a window is checked against the whole
 * text, so with a class that accepts '\n' ('.', '[^..]', '#') a match may
 * span a line break; k > 0 ("esimple") matches stay inside one line.
 * Replaces one nrgrep_coords run per pattern (per strand).              */
int pm_scan_linear(pm_db* db, int n_patterns, const int32_t* lengths,
                   const uint8_t* pos_class, int n_classes, const uint8_t* class_acgt,
                   const uint32_t* class_bytes, const uint8_t* class_is_any, int k,
                   int flags, pm_hits** out);

/* pm_scan_linear without a host synchronization: launches the scan and
 * returns a hit list that resolves on first use (pm_hits_count, _copy*,
 * _device, _kernel_ms wait for it; pm_hits_destroy does not).  A server
 * launches query i+1 before collecting query i, so host-side work overlaps
 * the GPU scan.  Same results as pm_scan_linear: when the hit counts
 * overflow the speculative layout, resolution re-runs the query
 * synchronously.  The database must outlive the list's resolution
 * (pm_db_destroy resolves pending lists first).                       */
int pm_scan_linear_async(pm_db* db, int n_patterns, const int32_t* lengths,
                         const uint8_t* pos_class, int n_classes, const uint8_t* class_acgt,
                         const uint32_t* class_bytes, const uint8_t* class_is_any, int k,
                         int flags, pm_hits** out);

/* Generates and compiles (hipRTC, gfx950) the pattern-specialized linear
 * kernel for up to 8 patterns without launching it: a host-only check that
 * needs no GPU (used by the CPU tests and to pre-warm the code cache). */
int pm_linear_jit_compile(int n_patterns, const int32_t* lengths, const uint8_t* pos_class,
                          int n_classes, const uint8_t* class_acgt, const uint8_t* class_is_any,
                          int k, uint64_t* code_bytes);

/* --- general patterns: Glushkov automaton (both alphabets) -------------
 * m positions (1..64); byte_mask[256] = positions accepting each folded
 * byte; follow[m] / first / last as produced by regex.py; max_len = the
 * longest match, 0 = unbounded (`*`, `+`: a match may run to the end of
 * its record).  Candidates: for every start with a match of <= k
 * substitutions, the shortest end; reported as PM_REPORT_NRGREP selects.
 * Hits carry pattern id `pattern_id`. */
int pm_scan_nfa(pm_db* db, int m, const uint64_t* byte_mask, const uint64_t* follow,
                uint64_t first, uint64_t last, int max_len, int k, int pattern_id,
                pm_hits** out);

/* Error types of nrgrep's `-k <k>[ids]` (patmatch.py:299-314 builds the
 * letters; all three when none is chosen). */
#define PM_ERR_INS 1       /* i: an extra text character                  */
#define PM_ERR_DEL 2       /* d: a pattern position with no text character */
#define PM_ERR_SUB 4       /* s: a substituted character                  */

/* pm_scan_nfa with an explicit error-type mask `errs` (PM_ERR_*) -- the
 * general `nrgrep_coords -k <k><ids>` scan.  min_len = the shortest match
 * length of the pattern (regex.py); with PM_ERR_DEL it must exceed k
 * (otherwise PM_E_UNSUPPORTED) unless the report is nrgrep's -- a class
 * sequence with PM_ESIMPLE or an extended pattern with PM_EXTENDED, whose
 * walks then take every line.  Insertions let a match run to
 * max_len + k characters.  pm_scan_nfa(...) == pm_scan_nfa_errs(..., 0, k,
 * PM_ERR_SUB, ...). */
int pm_scan_nfa_errs(pm_db* db, int m, const uint64_t* byte_mask, const uint64_t* follow,
                     uint64_t first, uint64_t last, int max_len, int min_len, int k, int errs,
                     int pattern_id, int flags, pm_hits** out);

/* pm_scan_nfa_errs for automata of up to PM_MAX_POSITIONS positions and up
 * to PM_MAX_K errors (a long oligo, an unrolled x(m,n), `-k 5`): position
 * sets are `words` 64-bit words (position i = bit i % 64 of word i / 64):
 * byte_mask[256 * words], follow[m * words], first[words], last[words].
 * words = ceil(m / 64) <= 4; k <= 7 when words == 4.  max_len is not
 * bounded.  flags may add PM_CROSS_LINES. */
int pm_scan_nfa_wide(pm_db* db, int m, int words, const uint64_t* byte_mask, const uint64_t* follow,
                     const uint64_t* first, const uint64_t* last, int max_len, int min_len, int k,
                     int errs, int pattern_id, int flags, pm_hits** out);

/* The pattern is a general regular expression -- '|' or a repeated group
 * (nrgrep's detClass() == 3): nrgrep_coords runs its "regular" engine at
 * k = 0 (searchPreproc -> regularPreproc 0x40c880), whose plan is priced
 * over its parse tree (regularFindBest 0x40a500 / minCost 0x409940) and
 * whose window scanner and nearest-boundary checkMatch (0x408ec0) decide
 * which overlapping match is printed.  A pattern whose best
 * window is a class sequence or an extended sequence prints nothing at all
 * (the state word checkMatch reads is only set by regularScan).  Replaces
 * one nrgrep_coords run on such a pattern (www/FlaskApp/FlaskApp/patmatch.py:
 * 733-743; GA(TC){1,2}A -> (GA(TC)(TC)?A), www/bin/patmatch_to_nrgrep.pl:
 * 307-348, 462-495).                                                      */
#define PM_REGULAR 512
/* pm_scan_nfa_wide plus nrgrep's simplified parse tree (regex.py
 * Program.tree): node i = tree[4i .. 4i+3] = (type 0 leaf / 1 '*' / 2 '|' /
 * 3 concatenation / 4 '?' / 5 '+', left child, right child, the leaf's
 * position), preorder, node 0 the root; tree_nullable[i] = the node's
 * parse-time nullable flag.  With PM_REGULAR (and PM_REPORT_NRGREP) the
 * report is the regular engine's at k = 0 and the eregular engine's at
 * k > 0 (eregularPreproc 0x406a20: k + 1 exact pieces, a window with k
 * errors or the automaton forward; checkMatch 0x406010; the sliced
 * transition tables of fwdCheck / bwdCheck beyond 64 states restated;
 * deletions with k >= min_len are answered, every line walked).  A k > 0 plan whose first window is an
 * extended sequence prints nothing (eregularPreproc dies, 0x4081ed).      */
int pm_scan_nfa_tree(pm_db* db, int m, int words, const uint64_t* byte_mask, const uint64_t* follow,
                     const uint64_t* first, const uint64_t* last, int max_len, int min_len, int k,
                     int errs, int pattern_id, int flags, int nodes, const int32_t* tree,
                     const int32_t* tree_nullable, pm_hits** out);
/* The plan nrgrep's regularPreproc derives (host only, no GPU needed):
 * out[0] = 2 (a window of out[1] characters scanned backward) or 3 (the
 * automaton scanned forward), out[2] = detClass of the window (1 / 2: the
 * engine prints nothing), out[3] = the window's states (with the initial
 * one); masks[0..4] / [5..9] / [10..14] = the window's states, its initial
 * and its final states in nrgrep's numbering (position + 1).  out must
 * hold 4 ints, masks 15 words.                                            */
int pm_regular_plan(int m, int words, const uint64_t* byte_mask, int nodes, const int32_t* tree,
                    const int32_t* tree_nullable, int32_t* out, uint64_t* masks);
/* The plan nrgrep's eregularPreproc derives at k errors (host only):
 * out[0] = 1 (k + 1 pieces of out[1] characters found exactly), 2 (a window
 * of out[1] characters scanned backward with k errors) or 3 (the automaton
 * forward), out[2] = detClass of the first window (1: esimple's scanners,
 * 2: the binary dies, 3: eregularScan), out[3] = 0 when the binary would
 * read memory it never wrote for this plan, out[4] = the windows;
 * masks[(3i + j) * 5 .. + 4] = window i (j = 0), its initial (1) and its
 * final (2) states, 5 words each; masks[48 * 5] = checkMatch's state word
 * for class 1.  out: 5 ints, masks: 245 words.  PM_E_UNSUPPORTED when a
 * window union exceeds 64 states or a transition-table slice would lie
 * past the state set (regularMakeDet / SLICE, pm_regular.hip).           */
int pm_eregular_plan(int m, int words, const uint64_t* byte_mask, int nodes, const int32_t* tree,
                     const int32_t* tree_nullable, int k, int32_t* out, uint64_t* masks);

/* Generates and compiles (hipRTC, gfx950) the bit-sliced start pass that
 * pm_scan_nfa_errs / _wide use for a class sequence with insertions /
 * deletions on a nucleotide database (m * (k + 1) <= 64), without
 * launching it: a host-only check that needs no GPU. */
int pm_ids_jit_compile(int m, const uint64_t* byte_mask, int k, int errs, uint64_t* code_bytes);

/* --- hits --------------------------------------------------------------- */
int pm_hits_count(const pm_hits* h, uint64_t* count);
/* Copies hits sorted by (pattern, beg).  Any pointer may be NULL. */
int pm_hits_copy(const pm_hits* h, int32_t* pattern, int64_t* beg, int64_t* end,
                 uint64_t max_count);
/* Milliseconds of the main scan kernel(s), measured with hipEvents on the
 * stream the kernels were launched on. */
int pm_hits_kernel_ms(const pm_hits* h, double* ms);
int pm_hits_destroy(pm_hits* h);

/* Copies sorted keys (pattern<<48 | beg) and match lengths into caller-owned
 * device buffers (e.g. a framework's tensors used for the cross-GPU gather);
 * `stream` = hipStream_t to order the copy on (NULL = synchronous).      */
int pm_hits_copy_device(const pm_hits* h, uint64_t* keys_dst, uint32_t* lens_dst,
                        uint64_t max_count, void* stream);

/* Raw device pointers of a hit list (uint64 keys = pattern<<48 | beg, and
 * uint32 lengths), for a caller that gathers hits across GPUs itself.   */
int pm_hits_device(const pm_hits* h, void** keys, void** lens, uint64_t* count);

/* The caller's last use of the buffers pm_hits_device returned: work queued
 * on `stream` (hipStream_t) up to now.  pm_hits_destroy then recycles the
 * buffers only after that work (e.g. tensors wrapping them, freed while a
 * framework's kernels still read them).  Like pm_hits_copy_device's use. */
int pm_hits_record_use(const pm_hits* h, void* stream);

/* The serving rank's merge of the ranks' hit lists (sharded scans, one rank
 * per GPU: replaces the order of one nrgrep_coords process's output over
 * the whole file, patmatch.py:733-743).  Part r = keys[part_beg[r] ..
 * part_beg[r] + part_len[r]) (host arrays, up to 64 parts), each sorted by
 * key (pattern << 48 | position) and covering its own position range, the
 * ranges increasing with r; out_keys receives every key sorted by key (per
 * pattern the parts' slices in part order: no sort).  out_lens (may be
 * NULL) receives each key's length: lens[i] moved with its key, or, with
 * lens NULL, len_of_pattern[pattern] (a device array of n_patterns entries:
 * fixed-length patterns).  Every key's pattern must be < n_patterns.  All
 * arrays but part_beg / part_len are device memory.  `work` (device,
 * *work_bytes bytes; NULL = size query: *work_bytes is set) holds the
 * slices' starts and destinations.  Enqueued on `stream` (hipStream_t;
 * NULL = the null stream, synchronous).                                   */
int pm_merge_parts(const uint64_t* keys, const int32_t* lens, const uint64_t* part_beg,
                   const uint64_t* part_len, int nparts, int n_patterns,
                   const int32_t* len_of_pattern, uint64_t* out_keys, int32_t* out_lens,
                   void* work, uint64_t* work_bytes, int device, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PATMATCH_HIP_H */
