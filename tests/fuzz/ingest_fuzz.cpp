// ingest_fuzz.cpp — sanitizer harness for csrc/ingest.cpp (the untrusted-BLOB decoder), built by
// tests/test_ingest_fuzz_cpu.py with -fsanitize=address,undefined -fno-sanitize-recover=all and
// linked against the decoder's source.  Reads records from stdin, one per call:
//   u8 kind | u32 a | u32 b | u64 len0 | bytes | u64 len1 | bytes
//   kind 0: ingest_parse_f32(blob0, len0, out, cap = a)
//   kind 1: ingest_concat_rows / ingest_concat_packed over one row of two parts (dims a, b)
// and prints "<rc> <fnv1a-64 of the output bytes>" per record (flushes after each).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/imgrec_ingest.h"

static bool read_all(void* p, size_t n) { return fread(p, 1, n, stdin) == n; }

static uint64_t fnv(const void* p, size_t n) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

static bool read_blob(std::vector<uint8_t>* v) {
    uint64_t n = 0;
    if (!read_all(&n, 8) || n > (1u << 26)) return false;
    v->resize(n);
    return n == 0 || read_all(v->data(), n);
}

int main() {
    for (;;) {
        uint8_t kind;
        uint32_t a, b;
        if (!read_all(&kind, 1)) return 0;
        if (!read_all(&a, 4) || !read_all(&b, 4)) return 2;
        std::vector<uint8_t> b0, b1;
        if (!read_blob(&b0) || !read_blob(&b1)) return 2;
        // exact-size heap copies: any read past the end of a BLOB is an ASan report
        uint8_t* p0 = static_cast<uint8_t*>(malloc(b0.size() ? b0.size() : 1));
        uint8_t* p1 = static_cast<uint8_t*>(malloc(b1.size() ? b1.size() : 1));
        for (size_t i = 0; i < b0.size(); ++i) p0[i] = b0[i];
        for (size_t i = 0; i < b1.size(); ++i) p1[i] = b1[i];
        if (kind == 0) {
            std::vector<float> out(a ? a : 1);
            const int64_t rc = ingest_parse_f32(p0, (int64_t)b0.size(), out.data(), a);
            printf("%lld %llu\n", (long long)rc,
                   (unsigned long long)fnv(out.data(), rc > 0 ? (size_t)rc * 4 : 0));
        } else {
            const int64_t dims[2] = {a, b};
            std::vector<float> out((size_t)a + b + 1), out2((size_t)a + b + 1);
            const uint8_t* blobs[2] = {p0, p1};
            const int64_t lens[2] = {(int64_t)b0.size(), (int64_t)b1.size()};
            int8_t st = -1, st2 = -1;
            const int64_t good = ingest_concat_rows(blobs, lens, 1, 2, dims, out.data(), &st);
            std::vector<uint8_t> packed(b0.begin(), b0.end());
            packed.insert(packed.end(), b1.begin(), b1.end());
            uint8_t* pk = static_cast<uint8_t*>(malloc(packed.size() ? packed.size() : 1));
            for (size_t i = 0; i < packed.size(); ++i) pk[i] = packed[i];
            const int64_t offs[2] = {0, (int64_t)b0.size()};
            const int64_t good2 = ingest_concat_packed(pk, offs, lens, 1, 2, dims, out2.data(), &st2);
            free(pk);
            if (good != good2 || st != st2) return 3;
            printf("%lld %llu\n", (long long)(good ? 0 : -st),
                   (unsigned long long)fnv(out.data(), good ? (size_t)(a + b) * 4 : 0));
        }
        fflush(stdout);
        free(p0);
        free(p1);
    }
}
