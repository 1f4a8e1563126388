// Host driver for the AddressSanitizer / UndefinedBehaviorSanitizer build of the blob validator
// (tools/sanitize_blob.py; tests/test_blob_sanitize.py). Each argument is a blob file; it is read into a heap
// buffer of exactly its size (an over-read past the end is an ASan report) and passed to spef_validate_blob,
// the host-only entry point that runs the same parse_blob checks as spef_load_weights[_device].
// Prints one line per file: "<rc> <dtype> <message>". Exit status 0 unless a file cannot be read.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "spef.h"

int main(int argc, char** argv) {
  for (int i = 1; i < argc; ++i) {
    FILE* f = fopen(argv[i], "rb");
    if (!f) {
      fprintf(stderr, "cannot open %s\n", argv[i]);
      return 2;
    }
    fseek(f, 0, SEEK_END);
    const long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    // exactly n bytes (malloc(0) for an empty file): ASan poisons everything past the end
    unsigned char* buf = (unsigned char*)malloc(n > 0 ? (size_t)n : 1);
    if (n > 0 && fread(buf, 1, (size_t)n, f) != (size_t)n) {
      fprintf(stderr, "short read %s\n", argv[i]);
      return 2;
    }
    fclose(f);
    if (getenv("BLOB_CHECK_SELFTEST")) {   // proves the sanitizer is live: one byte past the buffer must abort
      volatile unsigned char past = buf[n > 0 ? n : 1];
      printf("selftest read %d\n", (int)past);
    }
    int dt = -1, head = -1, n0 = -1, n1 = -1;
    const int rc = spef_validate_blob(buf, (size_t)n, &dt, &head, &n0, &n1);
    printf("%d %d %s\n", rc, dt, rc ? spef_last_error() : "ok");
    free(buf);
  }
  return 0;
}
