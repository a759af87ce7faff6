"""Batch decoding of the vector tables' pickle BLOBs into one float32 matrix (§8f row 1).

Restates FAISSIndexBuilderDB._process_batch (/root/reference/main/create_index.py:160-189): for
each row (id, blob_1..blob_P) every BLOB is unpickled, converted to a flat float32 vector and the
parts are concatenated in the caller's order; a row whose part fails to load is skipped with the
warning "ID {id}: error loading {type}: {exc}".  Here the whole batch is decoded by one native call
(``ingest_concat_packed``: the protocol-5 ndarray layout parsed and copied in C); only BLOBs in
another layout (torch tensors, float64, ...) take the reference's ``pickle.loads`` path.
"""
from __future__ import annotations

import ctypes as C
import logging
import pickle
from typing import Callable, Sequence

import numpy as np

from . import _lib


def _bytes_data_offset() -> int:
    """Offset of a CPython bytes object's data from its address (PyBytesObject.ob_sval:
    bytes.__basicsize__ - 1), verified once; 0 = unknown layout (the copying path is used)."""
    off = bytes.__basicsize__ - 1
    probe = b"imgrec-ingest-probe"
    try:
        return off if C.string_at(id(probe) + off, len(probe)) == probe else 0
    except Exception:   # noqa: BLE001
        return 0


_BYTES_DATA_OFFSET = _bytes_data_offset()


def _reference_decode(blob) -> np.ndarray:
    """create_index.py:176-179: pickle.loads, .cpu().numpy() for tensors, float32 ravel."""
    vec = pickle.loads(blob)
    if hasattr(vec, "cpu"):
        vec = vec.cpu().numpy()
    return np.asarray(vec, dtype="float32").ravel()


def decode_rows(rows: Sequence[tuple], vector_types: Sequence[str],
                part_dims: list[int] | None = None,
                log: Callable[[str, str], None] | None = None):
    """Decode a batch of (id, blob...) rows.

    Returns (ids, matrix, part_dims): the ids and float32 rows (n, sum(part_dims)) of the rows that
    decoded, in input order, and the per-part dimensions (taken from the first decodable row when
    not given).  Rows with a failing part are skipped and reported through ``log``.
    """
    log = log or (lambda msg, level="warning": logging.warning(msg))
    nparts = len(vector_types)
    n = len(rows)
    if n == 0:
        return [], np.zeros((0, sum(part_dims or [0])), np.float32), part_dims
    if part_dims is None:
        part_dims = _probe_dims(rows, vector_types)
        if part_dims is None:
            for rec_id, *blobs in rows:
                _fallback_row(rec_id, blobs, vector_types, log)
            return [], np.zeros((0, 0), np.float32), None
    lib = _lib.load()
    blobs = [b for _, *bs in rows for b in bs]
    lens = np.fromiter((len(b) if b is not None else -1 for b in blobs), np.int64, len(blobs))
    D = int(sum(part_dims))
    out = np.empty((n, D), np.float32)
    status = np.empty(n, np.int8)
    pd = np.asarray(part_dims, np.int64)
    if _BYTES_DATA_OFFSET and all(type(b) is bytes or b is None for b in blobs):
        # sqlite3 hands BLOBs over as bytes objects: pass their buffers in place (no copy; the
        # list keeps them alive across the call)
        ptrs = np.fromiter((id(b) + _BYTES_DATA_OFFSET if b is not None else 0 for b in blobs),
                           np.uint64, len(blobs))
        lib.ingest_concat_rows(ptrs.ctypes.data_as(C.POINTER(C.c_void_p)), lens.ctypes.data_as(
            C.POINTER(C.c_int64)), n, nparts, pd.ctypes.data_as(C.POINTER(C.c_int64)),
            out.ctypes.data, status.ctypes.data)
    else:
        offs = np.zeros(len(blobs), np.int64)
        if len(blobs) > 1:
            np.cumsum(np.maximum(lens[:-1], 0), out=offs[1:])
        buf = b"".join(bytes(b) for b in blobs if b is not None)
        lib.ingest_concat_packed(buf, offs.ctypes.data, lens.ctypes.data, n, nparts,
                                 pd.ctypes.data, out.ctypes.data, status.ctypes.data)
    keep = status == 0
    ids = [rows[i][0] for i in range(n) if keep[i]]
    if keep.all():
        return ids, out, part_dims
    # rows needing the reference's pickle path (status 1) or with mismatched dims (status 2)
    extra = {}
    for i in np.nonzero(~keep)[0]:
        rec_id, *bl = rows[i]
        vec = _fallback_row(rec_id, bl, vector_types, log)
        if vec is None:
            continue
        if vec.shape[0] != D:
            log(f"ID {rec_id}: vector length {vec.shape[0]} != index dimension {D}, skipped",
                "warning")
            continue
        extra[i] = vec
    order = [i for i in range(n) if keep[i] or i in extra]
    mat = np.empty((len(order), D), np.float32)
    for j, i in enumerate(order):
        mat[j] = out[i] if keep[i] else extra[i]
    return [rows[i][0] for i in order], mat, part_dims


def _fallback_row(rec_id, blobs, vector_types, log):
    parts = []
    for vt, blob in zip(vector_types, blobs):
        try:
            parts.append(_reference_decode(blob))
        except Exception as e:   # noqa: BLE001 - same catch-all as the reference
            log(f"ID {rec_id}: error loading {vt}: {e}", "warning")
            return None
    return np.concatenate(parts)


def _probe_dims(rows, vector_types):
    for _, *blobs in rows:
        dims = []
        for blob in blobs:
            try:
                dims.append(int(_reference_decode(blob).shape[0]))
            except Exception:   # noqa: BLE001
                dims = None
                break
        if dims is not None:
            return dims
    return None


def scan_native(db_path: str, sql: str, vector_types: Sequence[str], part_dims: Sequence[int],
                batch: int, refetch: Callable[[list], list],
                log: Callable[[str, str], None] | None = None):
    """The builder's scan + decode in native code (include/imgrec_ingest.h ingest_scan_*): yields
    (ids, float32 matrix) per batch of up to `batch` rows, in the query's row order.

    Rows whose BLOBs are not the fast protocol-5 float32 layout are re-read through `refetch`
    (a list of ids -> (id, blob...) rows) and decoded by decode_rows' pickle fallback, which logs
    and skips undecodable rows exactly as the reference's _process_batch does.  Raises
    NotImplementedError when the system SQLite library cannot be loaded (callers then use the
    Python scan).
    """
    lib = _lib.load()
    pd = np.asarray(part_dims, np.int64)
    D = int(pd.sum())
    h = C.c_void_p()
    rc = lib.ingest_scan_open(str(db_path).encode(), sql.encode(), len(pd),
                              pd.ctypes.data_as(C.POINTER(C.c_int64)), C.byref(h))
    if rc == -5:
        raise NotImplementedError(lib.ingest_scan_error().decode())
    if rc != 0:
        raise RuntimeError(f"ingest_scan_open: {lib.ingest_scan_error().decode()}")
    try:
        while True:
            ids = np.empty(batch, np.int64)
            out = np.empty((batch, D), np.float32)
            status = np.empty(batch, np.int8)
            n = lib.ingest_scan_next(h, batch, ids.ctypes.data, out.ctypes.data, status.ctypes.data)
            if n < 0:
                raise RuntimeError(f"ingest_scan_next: {lib.ingest_scan_error().decode()}")
            if n == 0:
                return
            ids, out, status = ids[:n], out[:n], status[:n]
            bad = np.nonzero(status != 0)[0]
            if len(bad) == 0:
                yield ids.tolist(), out
                continue
            rows = {r[0]: r for r in refetch(ids[bad].tolist())}
            fixed_ids, fixed, _ = decode_rows([rows[int(i)] for i in ids[bad] if int(i) in rows],
                                              vector_types, list(part_dims), log=log)
            ok = dict(zip(fixed_ids, fixed))
            keep = [j for j in range(n) if status[j] == 0 or int(ids[j]) in ok]
            mat = np.empty((len(keep), D), np.float32)
            for r, j in enumerate(keep):
                mat[r] = out[j] if status[j] == 0 else ok[int(ids[j])]
            yield [int(ids[j]) for j in keep], mat
    finally:
        lib.ingest_scan_close(h)
