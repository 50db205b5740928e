// Test harness (tests/test_decoder_fuzz.py): decodes every file named on the
// command line with the product's texture decoder, built with ASan + UBSan.
// Prints one "<rc> <w>x<h>" line per file; any memory error aborts.
#include <stdio.h>

#include <string>
#include <vector>

#include "host/rt_host.h"

void rt_set_error(const char *, ...) {}

int main(int argc, char **argv)
{
    for (int i = 1; i < argc; ++i) {
        std::vector<uint8_t> rgba;
        int w = 0, h = 0;
        std::string err;
        const int rc = rt_host::decode_image_file(argv[i], rgba, w, h, err);
        if (rc == 0 && rgba.size() != (size_t)w * h * 4) {
            fprintf(stderr, "%s: size mismatch\n", argv[i]);
            return 2;
        }
        printf("%d %dx%d\n", rc, w, h);
    }
    return 0;
}
