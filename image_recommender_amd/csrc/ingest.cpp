// ingest.cpp — protocol-5 numpy BLOB decoder (include/imgrec_ingest.h).
//
// Layout written by pickle.dumps(np.float32 ndarray, protocol=5) on numpy 2.x (numpy 1.x writes
// "numpy.core.numeric"), as produced by /root/reference/vector_scripts/create_vector_base.py:144:
//   80 05                      PROTO 5
//   95 <u64>                   FRAME
//   8c <n> numpy[._]core.numeric 94   8c 0b _frombuffer 94   93 94   28 (MARK)
//   96 <u64 nbytes> <payload>  BYTEARRAY8 (raw little-endian float32)
//   [95 <u64>]                 FRAME (only when the payload was written out of band)
//   94 8c 05 numpy 94 8c 05 dtype 94 93 94 8c 02 f4 94 89 88 87 94 52 94
//   28 4b 03 8c 01 3c 94 4e 4e 4e 4a ff ff ff ff 4a ff ff ff ff 4b 00 74 94 62
//   <shape ints: K u8 | M u16 | J i32 ...> 85|86   94 8c 01 (C|F) 94 74 94 52 94 2e
// Every byte is checked; anything else (torch tensors, other dtypes, big-endian) is reported as
// INGEST_NOT_FAST so the caller falls back to pickle.loads, as the reference does.

#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <string>

#include "../../include/imgrec_ingest.h"

namespace {

struct Cursor {
    const uint8_t* p;
    const uint8_t* end;
    bool ok = true;
    bool need(int64_t n) {
        if (!ok || end - p < n) ok = false;
        return ok;
    }
    bool lit(const void* s, int64_t n) {
        if (!need(n) || memcmp(p, s, (size_t)n) != 0) return ok = false;
        p += n;
        return true;
    }
    bool byte(uint8_t b) { return lit(&b, 1); }
    uint64_t u64() {
        if (!need(8)) return 0;
        uint64_t v;
        memcpy(&v, p, 8);
        p += 8;
        return v;
    }
    bool short_str(const char* s) {
        const int64_t n = (int64_t)strlen(s);
        return byte(0x8c) && byte((uint8_t)n) && lit(s, n);
    }
    // BININT1 / BININT2 / BININT
    bool small_int(int64_t* v) {
        if (!need(1)) return false;
        const uint8_t op = *p++;
        if (op == 0x4b && need(1)) { *v = *p; p += 1; return true; }
        if (op == 0x4d && need(2)) { uint16_t x; memcpy(&x, p, 2); p += 2; *v = x; return true; }
        if (op == 0x4a && need(4)) { int32_t x; memcpy(&x, p, 4); p += 4; *v = x; return x >= 0; }
        return ok = false;
    }
};

const uint8_t kDtypeTail[] = {0x94, 0x89, 0x88, 0x87, 0x94, 0x52, 0x94, 0x28, 0x4b, 0x03,
                              0x8c, 0x01, 0x3c, 0x94, 0x4e, 0x4e, 0x4e, 0x4a, 0xff, 0xff,
                              0xff, 0xff, 0x4a, 0xff, 0xff, 0xff, 0xff, 0x4b, 0x00, 0x74,
                              0x94, 0x62};

// Returns payload pointer/bytes and element count, or false.
bool parse(const uint8_t* blob, int64_t len, const uint8_t** payload, int64_t* nbytes,
           int64_t* nelem) {
    Cursor c{blob, blob + len};
    if (!(c.byte(0x80) && c.byte(0x05) && c.byte(0x95))) return false;
    c.u64();
    if (!c.need(2)) return false;
    // "numpy._core.numeric" (numpy >= 2) or "numpy.core.numeric" (numpy 1.x)
    if (c.p[0] == 0x8c && c.p[1] == 19) {
        if (!c.short_str("numpy._core.numeric")) return false;
    } else if (!c.short_str("numpy.core.numeric")) {
        return false;
    }
    if (!(c.byte(0x94) && c.short_str("_frombuffer") && c.byte(0x94) && c.byte(0x93) &&
          c.byte(0x94) && c.byte(0x28) && c.byte(0x96)))
        return false;
    const uint64_t nb = c.u64();
    if (!c.ok || nb % 4 != 0 || (uint64_t)(c.end - c.p) < nb) return false;
    *payload = c.p;
    *nbytes = (int64_t)nb;
    c.p += nb;
    if (c.need(1) && *c.p == 0x95) { c.p += 1; c.u64(); }   // new frame after out-of-band payload
    if (!(c.byte(0x94) && c.short_str("numpy") && c.byte(0x94) && c.short_str("dtype") &&
          c.byte(0x94) && c.byte(0x93) && c.byte(0x94) && c.short_str("f4") &&
          c.lit(kDtypeTail, sizeof(kDtypeTail))))
        return false;
    int64_t prod = 1, v = 0;
    int nd = 0;
    while (c.ok && c.need(1) && (*c.p == 0x4b || *c.p == 0x4d || *c.p == 0x4a) && nd < 3) {
        if (!c.small_int(&v)) return false;
        // a shape holding more elements than the payload is rejected before the product can
        // overflow (shape ints come from an untrusted BLOB; found by tests/test_ingest_fuzz_cpu.py)
        if (v > 0 && prod > (int64_t)(nb / 4) / v) return false;
        prod *= v;
        ++nd;
    }
    const uint8_t tup = nd == 1 ? 0x85 : (nd == 2 ? 0x86 : (nd == 3 ? 0x87 : 0));
    if (!tup || !c.byte(tup) || !c.byte(0x94) || !c.byte(0x8c) || !c.byte(0x01)) return false;
    if (!c.need(1) || (*c.p != 'C' && *c.p != 'F')) return false;
    const bool fortran = *c.p == 'F';
    c.p += 1;
    if (fortran && nd > 1) {
        // a column-major 2-D (1, d) or (d, 1) array is still contiguous; anything else is not
        // reproduced by a plain copy
        return false;
    }
    if (!(c.byte(0x94) && c.byte(0x74) && c.byte(0x94) && c.byte(0x52) && c.byte(0x94) &&
          c.byte(0x2e)))
        return false;
    if (c.p != c.end) return false;
    if (prod * 4 != (int64_t)nb) return false;
    *nelem = prod;
    return true;
}

}  // namespace

extern "C" {

int64_t ingest_parse_f32(const uint8_t* blob, int64_t len, float* out, int64_t cap) {
    if (!blob || len <= 0) return INGEST_NOT_FAST;
    const uint8_t* pl;
    int64_t nb, ne;
    if (!parse(blob, len, &pl, &nb, &ne)) return INGEST_NOT_FAST;
    if (ne > cap) return INGEST_TOO_SMALL;
    if (ne > 0) memcpy(out, pl, (size_t)nb);
    return ne;
}

int64_t ingest_concat_rows(const uint8_t* const* blobs, const int64_t* lens, int64_t nrows,
                           int nparts, const int64_t* part_dims, float* out, int8_t* status) {
    int64_t D = 0;
    for (int j = 0; j < nparts; ++j) D += part_dims[j];
    int64_t good = 0;
    for (int64_t r = 0; r < nrows; ++r) {
        float* o = out + r * D;
        int8_t st = 0;
        for (int j = 0; j < nparts && st == 0; ++j) {
            const uint8_t* pl;
            int64_t nb, ne;
            const int64_t k = r * nparts + j;
            if (!blobs[k] || !parse(blobs[k], lens[k], &pl, &nb, &ne)) {
                st = 1;
            } else if (ne != part_dims[j]) {
                st = 2;
            } else {
                memcpy(o, pl, (size_t)nb);
                o += ne;
            }
        }
        status[r] = st;
        if (st == 0) ++good;
    }
    return good;
}

int64_t ingest_concat_packed(const uint8_t* buf, const int64_t* offsets, const int64_t* lens,
                             int64_t nrows, int nparts, const int64_t* part_dims, float* out,
                             int8_t* status) {
    int64_t D = 0;
    for (int j = 0; j < nparts; ++j) D += part_dims[j];
    int64_t good = 0;
    for (int64_t r = 0; r < nrows; ++r) {
        float* o = out + r * D;
        int8_t st = 0;
        for (int j = 0; j < nparts && st == 0; ++j) {
            const uint8_t* pl;
            int64_t nb, ne;
            const int64_t k = r * nparts + j;
            if (lens[k] < 0 || !parse(buf + offsets[k], lens[k], &pl, &nb, &ne)) {
                st = 1;
            } else if (ne != part_dims[j]) {
                st = 2;
            } else {
                memcpy(o, pl, (size_t)nb);
                o += ne;
            }
        }
        status[r] = st;
        if (st == 0) ++good;
    }
    return good;
}

}  // extern "C"

// -----------------------------------------------------------------------------------------------
// Native scan of the builder's SELECT (include/imgrec_ingest.h ingest_scan_*): the system SQLite
// library (the one Python's sqlite3 module links, so the same query plan and row order) is opened
// with dlopen and driven from C: sqlite3_step per row, the BLOB columns parsed in place
// (sqlite3_column_blob, no copy) and written into the caller's float32 batch.
// -----------------------------------------------------------------------------------------------
namespace {

struct Sqlite {
    void* h = nullptr;
    int (*open_v2)(const char*, void**, int, const char*);
    int (*prepare_v2)(void*, const char*, int, void**, const char**);
    int (*step)(void*);
    int64_t (*column_int64)(void*, int);
    const void* (*column_blob)(void*, int);
    int (*column_bytes)(void*, int);
    int (*column_type)(void*, int);
    int (*finalize)(void*);
    int (*close)(void*);
    const char* (*errmsg)(void*);
    bool ok = false;
};

Sqlite* sqlite_lib() {
    static Sqlite s;
    static std::once_flag once;
    std::call_once(once, [] {
        for (const char* name : {"libsqlite3.so.0", "libsqlite3.so"}) {
            s.h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (s.h) break;
        }
        if (!s.h) return;
#define IMGREC_SYM(field, sym) s.field = reinterpret_cast<decltype(s.field)>(dlsym(s.h, sym))
        IMGREC_SYM(open_v2, "sqlite3_open_v2");
        IMGREC_SYM(prepare_v2, "sqlite3_prepare_v2");
        IMGREC_SYM(step, "sqlite3_step");
        IMGREC_SYM(column_int64, "sqlite3_column_int64");
        IMGREC_SYM(column_blob, "sqlite3_column_blob");
        IMGREC_SYM(column_bytes, "sqlite3_column_bytes");
        IMGREC_SYM(column_type, "sqlite3_column_type");
        IMGREC_SYM(finalize, "sqlite3_finalize");
        IMGREC_SYM(close, "sqlite3_close");
        IMGREC_SYM(errmsg, "sqlite3_errmsg");
#undef IMGREC_SYM
        s.ok = s.open_v2 && s.prepare_v2 && s.step && s.column_int64 && s.column_blob &&
               s.column_bytes && s.column_type && s.finalize && s.close && s.errmsg;
    });
    return s.ok ? &s : nullptr;
}

thread_local std::string g_scan_err;

constexpr int kSqliteOpenReadonly = 0x1, kSqliteRow = 100, kSqliteDone = 101, kSqliteNull = 5;

}  // namespace

struct ingest_scan {
    void* db = nullptr;
    void* stmt = nullptr;
    int nparts = 0;
    int64_t dim = 0;
    int64_t part_dims[64] = {};
    bool done = false;
};

extern "C" {

const char* ingest_scan_error(void) { return g_scan_err.c_str(); }

int ingest_scan_open(const char* db_path, const char* sql, int nparts, const int64_t* part_dims,
                     ingest_scan_t** out) {
    if (!out || !db_path || !sql || nparts < 1 || nparts > 64 || !part_dims) {
        g_scan_err = "bad arguments";
        return -1;
    }
    *out = nullptr;
    Sqlite* L = sqlite_lib();
    if (!L) {
        g_scan_err = "libsqlite3.so.0 not found or incomplete";
        return -5;
    }
    ingest_scan* s = new ingest_scan();
    s->nparts = nparts;
    for (int j = 0; j < nparts; ++j) {
        s->part_dims[j] = part_dims[j];
        s->dim += part_dims[j];
    }
    if (L->open_v2(db_path, &s->db, kSqliteOpenReadonly, nullptr) != 0) {
        g_scan_err = std::string("sqlite3_open_v2: ") + (s->db ? L->errmsg(s->db) : "failed");
        if (s->db) L->close(s->db);
        delete s;
        return -4;
    }
    if (L->prepare_v2(s->db, sql, -1, &s->stmt, nullptr) != 0 || !s->stmt) {
        g_scan_err = std::string("sqlite3_prepare_v2: ") + L->errmsg(s->db);
        L->close(s->db);
        delete s;
        return -4;
    }
    *out = s;
    return 0;
}

int64_t ingest_scan_next(ingest_scan_t* s, int64_t cap, int64_t* ids, float* out, int8_t* status) {
    if (!s || cap <= 0 || !ids || !out || !status) {
        g_scan_err = "bad arguments";
        return -1;
    }
    Sqlite* L = sqlite_lib();
    int64_t n = 0;
    while (n < cap && !s->done) {
        const int rc = L->step(s->stmt);
        if (rc == kSqliteDone) {
            s->done = true;
            break;
        }
        if (rc != kSqliteRow) {
            g_scan_err = std::string("sqlite3_step: ") + L->errmsg(s->db);
            return -4;
        }
        ids[n] = L->column_int64(s->stmt, 0);
        float* o = out + n * s->dim;
        int8_t st = 0;
        for (int j = 0; j < s->nparts && st == 0; ++j) {
            const uint8_t* pl;
            int64_t nb, ne;
            const int col = j + 1;
            const uint8_t* b = L->column_type(s->stmt, col) == kSqliteNull
                                   ? nullptr
                                   : static_cast<const uint8_t*>(L->column_blob(s->stmt, col));
            const int64_t len = b ? L->column_bytes(s->stmt, col) : 0;
            if (!b || !parse(b, len, &pl, &nb, &ne)) {
                st = 1;
            } else if (ne != s->part_dims[j]) {
                st = 2;
            } else {
                memcpy(o, pl, (size_t)nb);
                o += ne;
            }
        }
        status[n] = st;
        ++n;
    }
    return n;
}

int ingest_scan_close(ingest_scan_t* s) {
    if (!s) return 0;
    Sqlite* L = sqlite_lib();
    if (L) {
        if (s->stmt) L->finalize(s->stmt);
        if (s->db) L->close(s->db);
    }
    delete s;
    return 0;
}

}  // extern "C"
