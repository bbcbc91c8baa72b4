/* A plain C99 process driving the GPU path through include/pfscdc.h alone: no Python, no
 * torch, no HIP headers in the process (the library brings its own HIP runtime), as a cgo
 * binary in pachd would.  tests/test_gpu_parity.py builds it, runs it on the GPU and checks
 * every line against the oracle over the bytes it writes out.
 *
 * usage: abi_gpu_consumer DATA_OUT BITS SEED MIN MAX BATCH_BYTES LEN...
 *   Generates one file per LEN (xorshift bytes), writes their concatenation to DATA_OUT, then
 *   1. pfscdc_scan of the batch from host memory with PFSCDC_OPT_REF_IDS:
 *        seg FILE OFFSET SIZE FLAGS HASH ID DEK
 *   2. a chunk.Writer mirror (one annotation per file, each file in two writes):
 *        cb N                 (one callback with N annotations)
 *        ann USER HAS IDX SIZE EDGE ID DEK HASH OFF SIZE
 *        counts CHUNKS ANNOTATIONS */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pfscdc.h"

static void hex(const uint8_t* b, int n) {
  int i;
  putchar(' ');
  for (i = 0; i < n; i++) printf("%02x", b[i]);
}

static int on_chunk(void* user, const pfscdc_chunk_ref* c, const pfscdc_annotation_out* a,
                    uint32_t n) {
  uint32_t i;
  (void)user;
  printf("cb %u\n", n);
  for (i = 0; i < n; i++) {
    printf("ann %" PRIu64 " %d", a[i].user, a[i].has_data_ref);
    if (a[i].has_data_ref) {
      printf(" %" PRIu64 " %" PRId64 " %d", c->chunk_index, c->size_bytes, c->edge);
      hex(c->ref.id, 32);
      hex(c->ref.dek, 32);
      hex(a[i].data_ref.hash, 32);
      printf(" %" PRId64 " %" PRId64, a[i].data_ref.offset_bytes, a[i].data_ref.size_bytes);
    }
    printf("\n");
  }
  return 0;
}

#define DIE(msg, ctx)                                                              \
  do {                                                                             \
    fprintf(stderr, "%s: %s\n", msg, (ctx) ? pfscdc_last_error(ctx) : "");         \
    return 1;                                                                      \
  } while (0)

int main(int argc, char** argv) {
  pfscdc_params p;
  pfscdc_ctx *scan_ctx = NULL, *wctx = NULL;
  pfscdc_writer* w = NULL;
  uint32_t nfiles, f;
  uint64_t *offs, total = 0, k, s = 0x9e3779b97f4a7c15ull;
  uint8_t* data;
  FILE* out;

  if (argc < 8) {
    fprintf(stderr, "usage: %s DATA_OUT BITS SEED MIN MAX BATCH_BYTES LEN...\n", argv[0]);
    return 2;
  }
  pfscdc_default_params(&p);
  p.average_bits = (uint32_t)strtoul(argv[2], NULL, 10);
  p.seed = strtoll(argv[3], NULL, 10);
  p.min_chunk = strtoll(argv[4], NULL, 10);
  p.max_chunk = strtoll(argv[5], NULL, 10);
  nfiles = (uint32_t)(argc - 7);
  offs = (uint64_t*)calloc(nfiles + 1, sizeof *offs);
  for (f = 0; f < nfiles; f++) offs[f + 1] = offs[f] + strtoull(argv[7 + f], NULL, 10);
  total = offs[nfiles];
  data = (uint8_t*)malloc(total ? total : 1);
  if (!offs || !data) return 1;
  for (k = 0; k < total; k++) {  /* xorshift64: the bytes are written out for the oracle */
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    data[k] = (uint8_t)(s >> 56);
  }
  out = fopen(argv[1], "wb");
  if (!out || fwrite(data, 1, total, out) != total || fclose(out) != 0) return 1;

  /* 1. one batch, one annotation per file */
  if (pfscdc_ctx_create(&p, 0, &scan_ctx) != PFSCDC_OK) DIE("ctx_create", scan_ctx);
  if (pfscdc_set_options(scan_ctx, PFSCDC_OPT_REF_IDS) != PFSCDC_OK) DIE("options", scan_ctx);
  if (pfscdc_scan(scan_ctx, data, total, 0, offs, nfiles) != PFSCDC_OK) DIE("scan", scan_ctx);
  {
    const pfscdc_segment* seg = pfscdc_segments(scan_ctx);
    const pfscdc_ref* ref = pfscdc_refs(scan_ctx);
    uint64_t i, n = pfscdc_num_segments(scan_ctx);
    for (i = 0; i < n; i++) {
      printf("seg %u %" PRIu64 " %" PRIu64 " %u", seg[i].file, seg[i].offset, seg[i].size,
             seg[i].flags);
      hex(seg[i].hash, 32);
      hex(ref[i].id, 32);
      hex(ref[i].dek, 32);
      printf("\n");
    }
  }

  /* 2. the chunk.Writer mirror over the same files */
  if (pfscdc_ctx_create(&p, 0, &wctx) != PFSCDC_OK) DIE("ctx_create", wctx);
  if (pfscdc_set_options(wctx, PFSCDC_OPT_REF_IDS) != PFSCDC_OK) DIE("options", wctx);
  if (pfscdc_writer_create(wctx, on_chunk, NULL, strtoull(argv[6], NULL, 10), &w) != PFSCDC_OK)
    DIE("writer_create", wctx);
  for (f = 0; f < nfiles; f++) {
    uint64_t len = offs[f + 1] - offs[f], half = len / 2;
    if (pfscdc_writer_annotate(w, f) != PFSCDC_OK) DIE("annotate", wctx);
    if (pfscdc_writer_write(w, data + offs[f], half) != PFSCDC_OK) DIE("write", wctx);
    if (pfscdc_writer_write(w, data + offs[f] + half, len - half) != PFSCDC_OK) DIE("write", wctx);
  }
  if (pfscdc_writer_close(w) != PFSCDC_OK) DIE("close", wctx);
  printf("counts %" PRId64 " %" PRId64 "\n", pfscdc_writer_chunk_count(w),
         pfscdc_writer_annotation_count(w));
  if (pfscdc_writer_destroy(w) != PFSCDC_OK || pfscdc_ctx_destroy(wctx) != PFSCDC_OK ||
      pfscdc_ctx_destroy(scan_ctx) != PFSCDC_OK)
    return 1;
  free(data);
  free(offs);
  return 0;
}
