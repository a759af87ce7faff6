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

#include <stdint.h>
#include <string.h>

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
