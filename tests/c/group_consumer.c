/* A plain C99 process driving a device group through include/pfscdc.h alone, as a cgo pachd
 * would drive the GPUs of its node: one process, NDEV member contexts.  On a one-GPU box
 * every member is device 0 (several contexts on one GPU), which runs the same dealing,
 * per-member scans and peer-copy gather as distinct devices.
 *
 * usage: group_consumer DATA_OUT NDEV BITS SEED MIN MAX MEM_THRESHOLD INFLIGHT LEN...
 *   Generates one file per LEN (xorshift bytes), writes their concatenation to DATA_OUT, then
 *   1. pfscdc_group_scan of the batch from host memory with PFSCDC_OPT_REF_IDS, compared
 *      field by field with pfscdc_scan on one ctx; prints the group's dealing and records:
 *        part K BEGIN END
 *        seg FILE OFFSET SIZE FLAGS HASH ID DEK
 *   1b. the whole batch as one stream, pfscdc_group_scan_stream against pfscdc_scan of one
 *      file:
 *        stream SEGMENTS
 *   2. pfscdc_uw_create_group (Puts of every file as /f%05u) against pfscdc_uw_create on one
 *      ctx: the one ctx writes groups of INFLIGHT bytes, the group INFLIGHT * NDEV split over
 *      NDEV members, so both form the same groups; the ordered event streams and every
 *      fileset's roots must be byte-identical:
 *        uw EVENTS FILESETS
 *   Any difference exits non-zero with a message on stderr. */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pfscdc.h"

#define DIE(msg, err)                                 \
  do {                                                \
    fprintf(stderr, "%s: %s\n", msg, (err) ? (err) : ""); \
    return 1;                                         \
  } while (0)

static void hex(const uint8_t* b, int n) {
  int i;
  putchar(' ');
  for (i = 0; i < n; i++) printf("%02x", b[i]);
}

/* an event log: every event serialized into one growing byte buffer */
typedef struct {
  uint8_t* p;
  size_t n, cap;
  uint64_t events;
} log_t;

static int put_bytes(log_t* l, const void* b, size_t n) {
  if (l->n + n > l->cap) {
    size_t c = l->cap ? l->cap : 4096;
    uint8_t* q;
    while (c < l->n + n) c *= 2;
    q = (uint8_t*)realloc(l->p, c);
    if (!q) return 1;
    l->p = q;
    l->cap = c;
  }
  memcpy(l->p + l->n, b, n);
  l->n += n;
  return 0;
}

static int on_event(void* user, const pfscdc_uw_event* ev) {
  log_t* l = (log_t*)user;
  int32_t head[4];
  head[0] = ev->kind;
  head[1] = ev->index;
  head[2] = ev->level;
  head[3] = (int32_t)ev->fileset;
  l->events++;
  if (put_bytes(l, head, sizeof head)) return 1;
  if (ev->kind == PFSCDC_EV_CHUNK)
    return put_bytes(l, &ev->chunk, sizeof ev->chunk);
  return put_bytes(l, &ev->len, sizeof ev->len) || put_bytes(l, ev->bytes, (size_t)ev->len);
}

/* Puts every file into w, Closes, appends every fileset's Primitive to l */
static int run_uw(pfscdc_uwriter* w, const uint8_t* data, const uint64_t* offs, uint32_t nfiles,
                  log_t* l, uint32_t* nfs) {
  uint32_t f, i;
  char path[32];
  for (f = 0; f < nfiles; f++) {
    sprintf(path, "/f%05u", f);
    if (pfscdc_uw_put(w, path, "", 0, data + offs[f], offs[f + 1] - offs[f]) != PFSCDC_OK)
      return 1;
    if (f % 13 == 12) {
      sprintf(path, "/f%05u", f - 5);
      if (pfscdc_uw_delete(w, path, "") != PFSCDC_OK) return 1;
    }
  }
  if (pfscdc_uw_close(w) != PFSCDC_OK) return 1;
  *nfs = pfscdc_uw_num_filesets(w);
  for (i = 0; i < *nfs; i++) {
    pfscdc_fileset_info fi;
    if (pfscdc_uw_fileset(w, i, &fi) != PFSCDC_OK) return 1;
    if (put_bytes(l, &fi.size_bytes, 8) || put_bytes(l, &fi.num_files, 4) ||
        put_bytes(l, &fi.num_deletes, 4) || put_bytes(l, &fi.additive_root_len, 8) ||
        put_bytes(l, &fi.deletive_root_len, 8))
      return 1;
    if (fi.additive_root && put_bytes(l, fi.additive_root, (size_t)fi.additive_root_len)) return 1;
    if (fi.deletive_root && put_bytes(l, fi.deletive_root, (size_t)fi.deletive_root_len)) return 1;
  }
  return 0;
}

int main(int argc, char** argv) {
  pfscdc_params p;
  pfscdc_ctx *one = NULL, *uctx = NULL;
  pfscdc_group* g = NULL;
  pfscdc_uwriter *w1 = NULL, *wg = NULL;
  uint32_t nfiles, f, ndev, k, nfs1 = 0, nfsg = 0;
  int* devs;
  int64_t thr, inflight;
  uint64_t *offs, total, i, s = 0x9e3779b97f4a7c15ull;
  uint8_t* data;
  FILE* out;
  log_t l1 = {0}, lg = {0};

  if (argc < 10) {
    fprintf(stderr, "usage: %s DATA_OUT NDEV BITS SEED MIN MAX MEM_THRESHOLD INFLIGHT LEN...\n",
            argv[0]);
    return 2;
  }
  ndev = (uint32_t)strtoul(argv[2], NULL, 10);
  pfscdc_default_params(&p);
  p.average_bits = (uint32_t)strtoul(argv[3], NULL, 10);
  p.seed = strtoll(argv[4], NULL, 10);
  p.min_chunk = strtoll(argv[5], NULL, 10);
  p.max_chunk = strtoll(argv[6], NULL, 10);
  thr = strtoll(argv[7], NULL, 10);
  inflight = strtoll(argv[8], NULL, 10);
  nfiles = (uint32_t)(argc - 9);
  offs = (uint64_t*)calloc(nfiles + 1, sizeof *offs);
  devs = (int*)calloc(ndev ? ndev : 1, sizeof *devs);
  if (!offs || !devs || ndev == 0) return 1;
  for (f = 0; f < nfiles; f++) offs[f + 1] = offs[f] + strtoull(argv[9 + f], NULL, 10);
  total = offs[nfiles];
  data = (uint8_t*)malloc(total ? total : 1);
  if (!data) return 1;
  for (i = 0; i < total; i++) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    data[i] = (uint8_t)(s >> 56);
  }
  out = fopen(argv[1], "wb");
  if (!out || fwrite(data, 1, total, out) != total || fclose(out) != 0) return 1;

  /* 1. the batch: one ctx against the group */
  if (pfscdc_ctx_create(&p, 0, &one) != PFSCDC_OK) DIE("ctx_create", "");
  if (pfscdc_set_options(one, PFSCDC_OPT_REF_IDS) != PFSCDC_OK) DIE("options", pfscdc_last_error(one));
  if (pfscdc_scan(one, data, total, 0, offs, nfiles) != PFSCDC_OK) DIE("scan", pfscdc_last_error(one));
  if (pfscdc_group_create(&p, devs, ndev, PFSCDC_OPT_REF_IDS, &g) != PFSCDC_OK)
    DIE("group_create", "");
  if (pfscdc_group_size(g) != ndev) DIE("group_size", "");
  if (pfscdc_group_scan(g, data, total, offs, nfiles) != PFSCDC_OK)
    DIE("group_scan", pfscdc_group_last_error(g));
  {
    const uint64_t n = pfscdc_group_num_segments(g);
    const pfscdc_segment* seg = pfscdc_group_segments(g);
    const pfscdc_ref* ref = pfscdc_group_refs(g);
    const uint32_t* pb = pfscdc_group_part_begin(g);
    const pfscdc_segment* dseg = NULL;
    int idev = -1;
    if (n != pfscdc_num_segments(one)) DIE("segment count differs", "");
    if (n && (memcmp(seg, pfscdc_segments(one), n * sizeof *seg) != 0 ||
              memcmp(ref, pfscdc_refs(one), n * sizeof *ref) != 0))
      DIE("records differ", "");
    if (memcmp(pfscdc_group_file_segment_begin(g), pfscdc_file_segment_begin(one),
               (nfiles + 1) * sizeof(uint64_t)) != 0)
      DIE("file ranges differ", "");
    if (pfscdc_group_index_device(g, &dseg, NULL, &idev) != PFSCDC_OK || idev != 0 ||
        (n && !dseg))
      DIE("index_device", "");
    for (k = 0; k < ndev; k++) printf("part %u %u %u\n", k, pb[k], pb[k + 1]);
    for (i = 0; i < n; i++) {
      printf("seg %u %" PRIu64 " %" PRIu64 " %u", seg[i].file, seg[i].offset, seg[i].size,
             seg[i].flags);
      hex(seg[i].hash, 32);
      hex(ref[i].id, 32);
      hex(ref[i].dek, 32);
      printf("\n");
    }
  }

  /* 1b. the whole batch as one stream split across the group, against one ctx */
  {
    uint64_t one_offs[2] = {0, total};
    if (pfscdc_scan(one, data, total, 0, one_offs, 1) != PFSCDC_OK)
      DIE("scan stream", pfscdc_last_error(one));
    if (pfscdc_group_scan_stream(g, data, total) != PFSCDC_OK)
      DIE("group_scan_stream", pfscdc_group_last_error(g));
    if (pfscdc_group_num_segments(g) != pfscdc_num_segments(one) ||
        (pfscdc_num_segments(one) &&
         memcmp(pfscdc_group_segments(g), pfscdc_segments(one),
                pfscdc_num_segments(one) * sizeof(pfscdc_segment)) != 0))
      DIE("stream records differ", "");
    printf("stream %" PRIu64 "\n", pfscdc_group_num_segments(g));
  }

  /* 2. the unordered writer: one ctx against the group */
  if (pfscdc_set_knob("PFSCDC_UW_INFLIGHT", inflight) != PFSCDC_OK) DIE("knob", "");
  if (pfscdc_ctx_create(&p, 0, &uctx) != PFSCDC_OK) DIE("ctx_create", "");
  if (pfscdc_set_options(uctx, PFSCDC_OPT_REF_IDS) != PFSCDC_OK) DIE("options", "");
  if (pfscdc_uw_create(uctx, thr, NULL, on_event, &l1, &w1) != PFSCDC_OK) DIE("uw_create", "");
  if (run_uw(w1, data, offs, nfiles, &l1, &nfs1)) DIE("one ctx", pfscdc_uw_last_error(w1));
  if (pfscdc_set_knob("PFSCDC_UW_INFLIGHT", inflight * (int64_t)ndev) != PFSCDC_OK) DIE("knob", "");
  if (pfscdc_uw_create_group(g, thr, NULL, on_event, &lg, &wg) != PFSCDC_OK)
    DIE("uw_create_group", "");
  if (run_uw(wg, data, offs, nfiles, &lg, &nfsg)) DIE("group", pfscdc_uw_last_error(wg));
  if (nfs1 != nfsg || l1.events != lg.events || l1.n != lg.n || memcmp(l1.p, lg.p, l1.n) != 0)
    DIE("unordered writer output differs", "");
  printf("uw %" PRIu64 " %u\n", lg.events, nfsg);

  if (pfscdc_uw_destroy(w1) != PFSCDC_OK || pfscdc_uw_destroy(wg) != PFSCDC_OK ||
      pfscdc_ctx_destroy(uctx) != PFSCDC_OK || pfscdc_ctx_destroy(one) != PFSCDC_OK ||
      pfscdc_group_destroy(g) != PFSCDC_OK)
    return 1;
  free(l1.p);
  free(lg.p);
  free(data);
  free(offs);
  free(devs);
  return 0;
}
