// Host-only driver of the file parse (s2c_parser_feed_file → s2c_parser_finish) for the
// sanitizer test (tests/test_host.py::test_host_code_under_sanitizers).
#include <cstdio>
#include "s2c.h"
int main(int argc, char **argv) {
    if (argc < 2) return 2;
    s2c_parser *p;
    s2c_parser_new(1, 150, &p);
    int rc = s2c_parser_feed_file(p, argv[1]);
    s2c_batch *b = nullptr;
    if (!rc) rc = s2c_parser_finish(p, &b);
    s2c_batch_info I{};
    if (!rc) s2c_batch_info_get(b, &I);
    printf("rc %d reads %lld tiles %lld\n", rc, (long long)I.reads_mapped, (long long)I.n_tiles);
    if (b) s2c_batch_free(b);
    s2c_parser_free(p);
    return rc ? 1 : 0;
}
