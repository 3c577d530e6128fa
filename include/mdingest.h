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

#ifdef __cplusplus
}
#endif

#endif /* MDINGEST_H */
