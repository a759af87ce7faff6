/*
 * imgrec_ingest.h — native decoding of the reference's vector BLOBs.
 *
 * The reference stores every feature vector as pickle.dumps(np.ndarray float32, protocol=5)
 * (/root/reference/vector_scripts/create_vector_base.py:144) and decodes each with pickle.loads +
 * np.concatenate per row, twice per build (/root/reference/main/create_index.py:160-189, 285, 306).
 * These functions decode the protocol-5 ndarray layout directly (validating every byte of the
 * opcode stream they rely on) and concatenate the parts of a row into one float32 row; a BLOB in
 * any other layout is reported so the caller can fall back to pickle.loads.
 */
#ifndef IMGREC_INGEST_H
#define IMGREC_INGEST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define INGEST_NOT_FAST (-1)   /* not the numpy protocol-5 float32 layout: use pickle.loads */
#define INGEST_TOO_SMALL (-2)  /* more elements than the output capacity */

/* Decode one BLOB into out[0..cap).  Returns the element count or a negative INGEST_* code. */
int64_t ingest_parse_f32(const uint8_t* blob, int64_t len, float* out, int64_t cap);

/* Decode nrows rows of nparts BLOBs each (blobs/lens row-major [row][part]) into
 * out[row * sum(part_dims) ...], parts concatenated in the given order (create_index.py:188).
 * status[row] = 0 decoded, 1 needs the pickle fallback (some part not in the fast layout),
 * 2 dimension mismatch.  Returns the number of rows with status 0. */
int64_t ingest_concat_rows(const uint8_t* const* blobs, const int64_t* lens, int64_t nrows,
                           int nparts, const int64_t* part_dims, float* out, int8_t* status);

/* Same, with all BLOBs packed back to back in one buffer: BLOB (row, part) occupies
 * buf[offsets[row*nparts+part] .. + lens[row*nparts+part]) (a length < 0 marks a NULL BLOB). */
int64_t ingest_concat_packed(const uint8_t* buf, const int64_t* offsets, const int64_t* lens,
                             int64_t nrows, int nparts, const int64_t* part_dims, float* out,
                             int8_t* status);

/* Native scan of the index builder's query (the reference's _batch_records + _process_batch,
 * /root/reference/main/create_index.py:136-189, in one pass): `sql` = "SELECT id, blob_1 .. blob_P
 * FROM ..." is run read-only on db_path through the system SQLite library (libsqlite3.so.0,
 * dlopen'd: the library Python's sqlite3 module uses, hence the same plan and row order), and
 * every row's BLOBs are parsed in place.  ingest_scan_next fills up to cap rows: ids[i], the
 * concatenated float32 row out[i * sum(part_dims) ...] and status[i] as ingest_concat_rows (rows
 * with status != 0 are left to the caller's pickle fallback).  Returns the rows filled, 0 at the
 * end, < 0 on an SQLite error (message: ingest_scan_error). */
typedef struct ingest_scan ingest_scan_t;
int ingest_scan_open(const char* db_path, const char* sql, int nparts, const int64_t* part_dims,
                     ingest_scan_t** out);
int64_t ingest_scan_next(ingest_scan_t* scan, int64_t cap, int64_t* ids, float* out,
                         int8_t* status);
int ingest_scan_close(ingest_scan_t* scan);
const char* ingest_scan_error(void);

#ifdef __cplusplus
}
#endif

#endif /* IMGREC_INGEST_H */
