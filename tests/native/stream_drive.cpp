#include <cstdio>
#include <cstdint>
#include <vector>
#include "s2c.h"
// Host-only driver of streamed batches with pipelined snapshots (detach → snapshot / shard /
// retain → attach, as stream._sorted_items drives them, here on one thread) for the sanitizer
// test (tests/test_host.py::test_host_code_under_sanitizers).
int main(int argc, char **argv) {
    if (argc < 2) return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<char> buf(1 << 20);
    s2c_parser *p; s2c_parser_new(1, 150, &p);
    s2c_parser_set_tile_width(p, 256);
    s2c_parser *d = nullptr;
    size_t pending = 0; int nb = 0, rc = 0;
    for (;;) {
        size_t n = fread(buf.data(), 1, buf.size(), f);
        if (!n) break;
        if ((rc = s2c_parser_feed(p, buf.data(), n))) { printf("feed rc %d %s\n", rc, s2c_last_error()); break; }
        pending += n;
        if (pending < (4u << 20)) continue;
        pending = 0;
        if (d) { s2c_parser_attach(p, d); d = nullptr; }
        if ((rc = s2c_parser_detach(p, &d))) { printf("detach rc %d\n", rc); break; }
        s2c_batch *b = nullptr;
        if (s2c_parser_snapshot(d, &b) == 0) {
            int64_t st[4]; s2c_parser_stream_state(d, st);
            s2c_batch_info I; s2c_batch_info_get(b, &I);
            if (st[1] >= 0 && I.n_tiles > 2) {   // (the first half of the tiles run; the reads reaching the rest kept)
                s2c_batch_arrays A;
                s2c_batch_arrays_get(b, &A);
                const int64_t cut = A.tiles[(size_t)(I.n_tiles / 2) * S2C_TILE_WORDS];
                s2c_batch *sub = nullptr;
                if (s2c_batch_shard(b, 0, I.n_tiles / 2, &sub) == 0) s2c_batch_free(sub);
                s2c_parser_retain(d, cut);
            }
            s2c_batch_free(b);
            nb++;
        }
    }
    if (d) s2c_parser_attach(p, d);
    s2c_batch *b = nullptr;
    rc = s2c_parser_finish(p, &b);
    s2c_batch_info I{}; if (!rc) s2c_batch_info_get(b, &I);
    printf("rc %d snapshots %d reads %lld\n", rc, nb, (long long)I.reads_mapped);
    fclose(f);
    if (b) s2c_batch_free(b);
    s2c_parser_free(p);
    return 0;
}
