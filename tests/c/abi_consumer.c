/* A plain C99 consumer of include/pfscdc.h, as cgo would compile it: no C++, no HIP headers,
 * only the header and -lpfscdc.  Exercises the host-side entry points (no GPU needed) and
 * prints their results one per line for tests/test_abi.py to check against the oracle.
 *
 * usage: abi_consumer SEED PATH...   (prints the table of SEED, Go Int63s of SEED, the
 * in-memory store's behaviour, every knob, and fileset.Clean of each PATH) */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pfscdc.h"

#define CHECK(cond)                                                   \
  do {                                                                \
    if (!(cond)) {                                                    \
      fprintf(stderr, "check failed at line %d: %s\n", __LINE__, #cond); \
      return 1;                                                       \
    }                                                                 \
  } while (0)

int main(int argc, char** argv) {
  pfscdc_params p;
  uint64_t table[256];
  int64_t r[8];
  int i;
  int64_t seed;

  CHECK(argc >= 2);
  seed = strtoll(argv[1], NULL, 10);

  pfscdc_default_params(&p);
  printf("params %u %" PRId64 " %" PRId64 " %" PRId64 "\n", p.average_bits, p.seed, p.min_chunk,
         p.max_chunk);

  CHECK(pfscdc_table(seed, table) == PFSCDC_OK);
  printf("table");
  for (i = 0; i < 256; i++) printf(" %016" PRIx64, table[i]);
  printf("\n");

  CHECK(pfscdc_go_int63(seed, r, 8) == PFSCDC_OK);
  printf("int63");
  for (i = 0; i < 8; i++) printf(" %" PRId64, r[i]);
  printf("\n");

  /* the chunk store: put, dedup by id, get, a missing id */
  {
    pfscdc_store* s = NULL;
    uint8_t id[32], other[32];
    const char* body = "ciphertext bytes";
    const void* got = NULL;
    uint64_t n = 0;
    memset(id, 0xab, sizeof id);
    memset(other, 0xcd, sizeof other);
    CHECK(pfscdc_store_create(&s) == PFSCDC_OK && s != NULL);
    CHECK(pfscdc_store_put(s, id, body, strlen(body)) == PFSCDC_OK);
    CHECK(pfscdc_store_put(s, id, body, strlen(body)) == PFSCDC_OK);
    CHECK(pfscdc_store_get(s, id, &got, &n) == PFSCDC_OK);
    CHECK(n == strlen(body) && memcmp(got, body, n) == 0);
    printf("store count %" PRIu64 " missing %d\n", pfscdc_store_count(s),
           pfscdc_store_get(s, other, &got, &n));
    CHECK(pfscdc_store_destroy(s) == PFSCDC_OK);
  }

  /* bad arguments are refused without a GPU */
  {
    pfscdc_ctx* c = NULL;
    printf("ctx_null %d\n", pfscdc_ctx_create(NULL, 0, &c));
    printf("unknown_knob %d\n", pfscdc_set_knob("PFSCDC_NO_SUCH_KNOB", 1));
  }

  /* every knob: name, range, default; set to its default and read back */
  for (i = 0;; i++) {
    int64_t lo, hi, def, v = -12345;
    const char* name = pfscdc_knob_info(i, &lo, &hi, &def);
    if (!name) break;
    CHECK(pfscdc_set_knob(name, def) == PFSCDC_OK);
    CHECK(pfscdc_get_knob(name, &v) == PFSCDC_OK && v == def);
    if (hi < INT64_MAX) CHECK(pfscdc_set_knob(name, hi + 1) == PFSCDC_EINVAL);
    printf("knob %s %" PRId64 " %" PRId64 " %" PRId64 "\n", name, lo, hi, def);
  }

  for (i = 2; i < argc; i++) {
    char out[4096];
    int dir;
    for (dir = 0; dir < 2; dir++) {
      CHECK(pfscdc_path_clean(argv[i], dir, out, sizeof out) == PFSCDC_OK);
      printf("clean %d %s\n", dir, out);
    }
  }
  return 0;
}
