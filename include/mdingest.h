/*
 * mdingest.h — native reader of metadamage count tables (C-ABI).
 *
 * Replaces the parsing step of the reference's count ingest
 * (/root/reference/metadamage/counts.py:229-235: dask read_csv of the
 * 22-column headerless table, columns counts.py:37-45) with a multi-threaded,
 * memory-mapped parser.  Also reads the 20-column headed files shipped in
 * data/input/ (#taxid Nalignments Direction Pos AA..TT).  Everything after
 * parsing (reference counts, error rates, positions, y_sum_total, the cut,
 * the sort, downcasting: counts.py:86-209) is vectorised on the host
 * (metadamage_amd/counts.py); the GPU fit consumes the packed result.
 *
 * Returns 0 on success, a negative MDI_E_* code on error (message from
 * mdi_last_error(), thread-local).
 */
#ifndef MDINGEST_H
#define MDINGEST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MDI_E_IO (-1)     /* open / map failed */
#define MDI_E_PARSE (-2)  /* malformed row (message names line and column) */
#define MDI_E_ARG (-3)
#define MDI_E_RANGE (-4)  /* a kept count above uint32 (utils.py:338-339 "too large values") */
#define MDI_E_LAYOUT (-5) /* mdi_used_codes: the distinct categories among codes[n] (pd.unique of a
 * categorical column, utils.py:121-130; the present groups of fits.py:736-744):
 * used[k] = 1 where code k (< n_cat) occurs, *n_missing (nullable) = the codes
 * < 0 (missing values); returns the number of used codes, MDI_E_ARG on a code
 * >= n_cat.  Parallel over row ranges. */
int64_t mdi_used_codes(int64_t n, const int32_t* codes, int32_t n_cat, int n_threads, uint8_t* used,
                       int64_t* n_missing);

/* mdi_pack_dense: the table is not in the usual layout */

/* string columns, interned: codes index the table's string list (first
 * appearance order) */
#define MDI_STR_NAME 0   /* tax_name (22-column format only) */
#define MDI_STR_RANK 1   /* tax_rank (22-column format only) */
#define MDI_STR_STRAND 2 /* strand: "5'" / "3'" */

typedef struct mdi_table mdi_table;

/* Map `path`, detect its format, cut it into one chunk per thread
 * (`n_threads` <= 0: hardware concurrency) and count the rows. */
int mdi_open(const char* path, int n_threads, mdi_table** out);

/* 22 (headerless reference table) or 20 (headed data/input table). */
int mdi_format(const mdi_table* t);
int64_t mdi_rows(const mdi_table* t);

/* Parse every row straight into the caller's arrays (mdi_rows entries each;
 * counts16 is column-major int64[16][rows] in AA AC .. TT order; the codes
 * index the string tables).  Once per table. */
int mdi_parse_into(mdi_table* t, int64_t* tax_id, int64_t* n_alignments, int64_t* position,
                   int64_t* counts16, int32_t* name_code, int32_t* rank_code, int32_t* strand_code);

/* String table `which`: number of strings, total bytes, and the strings
 * packed into buf (bytes) with offsets[n + 1]. */
int64_t mdi_n_strings(const mdi_table* t, int which);
int64_t mdi_string_bytes(const mdi_table* t, int which);
int mdi_strings(const mdi_table* t, int which, char* buf, int64_t* offsets);

void mdi_free(mdi_table* t);
const char* mdi_last_error(void);

/* ---- the count pipeline on parsed rows (counts.py:86-209) ----------------
 * Stateless: the arguments are the columns mdi_parse_into filled; the strand
 * of row r is forward iff code_is_fwd[strand_code[r]] ("5'").  sub_fwd /
 * sub_rev name the substitutions ("CT", "GA").
 *
 * mdi_select replaces add_y_sum_counts + the cut + sort_by_alignments
 * (counts.py:167-209): taxon[r] = first-appearance index of tax_id[r],
 * y_sum_total[r] = that taxon's substitution-count sum, and perm[0..n) = the
 * kept rows (N_alignments >= min_alignments, y_sum_total >= min_y_sum) in
 * N_alignments, tax_id, z order (all descending, ties in file order).
 * uniq (nullable, `rows` entries) receives the tax_id of each taxon index and
 * n_taxa (nullable) their number.  Parallel over row ranges (n_threads <= 0:
 * mdi_default_threads()).  Returns n (>= 0) or a negative MDI_E_* code.
 * taxon, y_sum_total and perm hold `rows` entries. */
int64_t mdi_select(int64_t rows, const int64_t* tax_id, const int64_t* n_alignments, const int64_t* position,
                   const int64_t* counts16, const int32_t* strand_code, const uint8_t* code_is_fwd,
                   int32_t n_codes, const char* sub_fwd, const char* sub_rev, int64_t min_alignments,
                   int64_t min_y_sum, int n_threads, int32_t* taxon, int64_t* y_sum_total, int64_t* perm,
                   int64_t* uniq, int64_t* n_taxa);

/* mdi_gather writes the numeric columns of the counts table for the rows
 * perm[0..n_keep), downcast as utils.py:329-356 (add_reference_counts,
 * add_error_rates, positions: counts.py:86-126): N_alignments, position
 * (1-indexed, reverse negative, int8), the 16 pair counts ([16][n_keep]),
 * the two reference-base sums ([2][n_keep], forward then reverse), the two
 * error rates f = count / reference (0/0 -> 0, x/0 -> inf; [2][n_keep]) and
 * y_sum_total.  n_threads <= 0: hardware concurrency.  MDI_E_RANGE if a
 * kept integer exceeds uint32. */
int mdi_gather(int64_t rows, const int64_t* perm, int64_t n_keep, const int64_t* n_alignments,
               const int64_t* position, const int64_t* counts16, const int32_t* strand_code,
               const uint8_t* code_is_fwd, int32_t n_codes, const char* sub_fwd, const char* sub_rev,
               const int64_t* y_sum_total, int n_threads, uint32_t* o_nal, int8_t* o_position,
               uint32_t* o_counts16, uint32_t* o_ref2, float* o_f2, uint32_t* o_y_sum_total);

/* mdi_noise: add_noise_estimates (fits.py:359-376) of n_taxa packed taxa on
 * the host, so the 1,440 B/taxon of mismatch counts need not cross PCIe:
 * mm = uint32[n_taxa][30][12] (columns AC AG AT CA CG CT GA GC GT TA TC TG,
 * rows z = 1..15 then -1..-15, the layout of include/mdfit.h), out3 =
 * double[n_taxa][3] = (normalized_noise, _forward, _reverse): per column the
 * counts over its mean (CT forward / GA reverse excluded), then the
 * population sd over all / forward / reverse rows (NaN when empty).
 * n_threads <= 0: hardware concurrency. */
int mdi_noise(const uint32_t* mm, int64_t n_taxa, int n_threads, double* out3);

/* mdi_codes / mdi_remap: the categorical columns of the kept rows
 * (astype("category") of tax_id, tax_name, tax_rank, strand; utils.py:329-356)
 * without a per-row pass in Python.  mdi_codes, for each of n_cols int32 code
 * columns in[c][rows]: out[c][i] = in[c][perm[i]] (i < n_keep) and used[c][k]
 * = 1 where code k (< n_table[c]) occurs among them (used zeroed here).  The
 * caller orders the used values (the sorted categories) and mdi_remap then
 * rewrites every code in place: codes[c][i] = remap[c][codes[c][i]].  Both
 * parallel over row ranges; n_threads <= 0: hardware concurrency. */
int mdi_codes(int64_t n_keep, const int64_t* perm, int n_cols, const int32_t* const* in, const int32_t* n_table,
              int n_threads, int32_t* const* out, uint8_t* const* used);
int mdi_remap(int64_t n, int n_cols, int32_t* const* codes, const int32_t* const* remap, int n_threads);

/* mdi_first_index / mdi_interleave: the packing of group_to_numpyro_data
 * (fits.py:398-419) for fits.pack_counts.  mdi_first_index numbers the
 * categories of codes[n] (< n_cat) in first-appearance order (pd.factorize):
 * taxon[i] = that number, first[t] = the first row of taxon t; returns the
 * number of taxa T (first holds n entries at most), -1 on a bad code.
 * mdi_interleave writes out[i][c] = cols[c][i] (n rows, n_cols <= 64 uint32
 * columns: the [T][30][12] mismatch block), parallel over row ranges. */
int64_t mdi_first_index(int64_t n, const int32_t* codes, int32_t n_cat, int64_t* taxon, int64_t* first);
int mdi_interleave(int64_t n, int n_cols, const uint32_t* const* cols, uint32_t* out, int n_threads);

/* mdi_pack_dense: fits.pack_counts in one parallel pass for the usual table --
 * n = 30 T rows, taxon t on rows 30t..30t+29 with positions 1..15, -1..-15 and
 * one tax_id code (< n_cat) per block, no code in two blocks.  cols: 16 uint32
 * columns, the 12 mismatch columns (fits.MM_COLUMNS order) then y forward,
 * y reverse, N forward, N reverse.  Writes y, N (uint32[T][ld], columns >= 30
 * zeroed) and mm (uint32[T][30][12]); returns T, MDI_E_LAYOUT when the table
 * is not in that layout (the outputs are then partly written: the caller's general path
 * rewrites them), MDI_E_ARG on bad arguments. */
int64_t mdi_pack_dense(int64_t n, const int32_t* codes, int32_t n_cat, const int8_t* position,
                       const uint32_t* const* cols, int ld, int n_threads, uint32_t* y, uint32_t* N, uint32_t* mm);

/* Worker threads the library uses when a call passes n_threads <= 0: the
 * process's CPU share -- OMP_NUM_THREADS when set (a GPU box grants 16 cores
 * per GPU and sets it), else the CPUs of the affinity mask -- never the whole
 * machine's hardware_concurrency (256 on an 8-GPU node: oversubscription). */
int mdi_default_threads(void);

/* message of the last failed mdi_select / mdi_gather on this thread */
const char* mdi_counts_error(void);

#ifdef __cplusplus
}
#endif

#endif /* MDINGEST_H */
