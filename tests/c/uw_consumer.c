/* A plain C99 driver of the host-heavy entry points, for the host-sanitizer run
 * (tools/host_sanitize.sh): the UnorderedWriter (Put, append, Delete, directory deletes,
 * grouped background fileset writes), the chunk store, Writer.Copy of another writer's
 * DataRefs, MergeFileReader.Hash, four threads scanning at once, each on its own ctx, and a
 * device group (its member threads and its unordered writer).  Parity of these paths is tested from Python against the
 * oracle; this program only has to drive them through a sanitized library and print a
 * summary.  usage: uw_consumer NFILES SEED */
#include <inttypes.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "pfscdc.h"

/* Under LeakSanitizer (tools/host_sanitize.sh) the leak check runs here, before the HIP
 * runtime's own teardown, and the process then leaves with _exit: at exit, ROCm's ASan device
 * allocator CHECK-fails freeing HSA runtime objects after that runtime has unloaded
 * (profiles/r5/sanitize/).  Weak: a build without the sanitizers links without it. */
extern void __lsan_do_leak_check(void) __attribute__((weak));

#define OK(call, ctx)                                                                  \
  do {                                                                                 \
    int rc_ = (call);                                                                  \
    if (rc_ != PFSCDC_OK) {                                                            \
      fprintf(stderr, "%s -> %d: %s\n", #call, rc_, (ctx) ? pfscdc_last_error(ctx) : ""); \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

static uint64_t rng_state;
static uint64_t next_u64(void) {
  uint64_t z = (rng_state += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

static uint64_t uw_events, uw_index_events;
static int on_uw(void* user, const pfscdc_uw_event* ev) {
  (void)user;
  uw_events++;
  if (ev->kind == PFSCDC_EV_INDEX) uw_index_events++;
  return 0;
}

/* the first writer's DataRefs, in annotation order */
static pfscdc_full_dataref* refs;
static uint32_t* ref_file;
static uint32_t nrefs, cap_refs;
static uint64_t copies_seen, chunks_seen;

static int on_chunk(void* user, const pfscdc_chunk_ref* c, const pfscdc_annotation_out* a,
                    uint32_t n) {
  uint32_t i;
  int record = user != NULL;
  chunks_seen++;
  if (c->copied) copies_seen++;
  for (i = 0; record && i < n; i++) {
    if (!a[i].has_data_ref) continue;
    if (nrefs == cap_refs) {
      cap_refs = cap_refs ? 2 * cap_refs : 64;
      refs = (pfscdc_full_dataref*)realloc(refs, cap_refs * sizeof *refs);
      ref_file = (uint32_t*)realloc(ref_file, cap_refs * sizeof *ref_file);
      if (!refs || !ref_file) return 1;
    }
    memset(&refs[nrefs], 0, sizeof refs[nrefs]);
    refs[nrefs].ref = c->ref;
    refs[nrefs].ref_size = c->size_bytes;
    refs[nrefs].edge = c->edge;
    refs[nrefs].data = a[i].data_ref;
    ref_file[nrefs] = (uint32_t)a[i].user;
    nrefs++;
  }
  return 0;
}

/* distinct ctxs may run concurrently (pfscdc.h): each thread scans the same batch twice */
typedef struct {
  const uint8_t* data;
  const uint64_t* offs;
  uint32_t nfiles;
  uint64_t nsegs;
  uint8_t digest0[32];
  int rc;
} scan_job;

static void* scan_thread(void* arg) {
  scan_job* j = (scan_job*)arg;
  pfscdc_params p;
  pfscdc_ctx* c = NULL;
  int r;
  pfscdc_default_params(&p);
  p.average_bits = 12;
  p.min_chunk = 2000;
  p.max_chunk = 30000;
  j->rc = pfscdc_ctx_create(&p, 0, &c);
  for (r = 0; r < 2 && j->rc == PFSCDC_OK; r++) {
    j->rc = pfscdc_scan(c, j->data, j->offs[j->nfiles], 0, j->offs, j->nfiles);
    if (j->rc == PFSCDC_OK) {
      j->nsegs = pfscdc_num_segments(c);
      if (j->nsegs) memcpy(j->digest0, pfscdc_segments(c)[0].hash, 32);
    }
  }
  if (c) pfscdc_ctx_destroy(c);
  return NULL;
}

int main(int argc, char** argv) {
  pfscdc_params p, ip;
  pfscdc_ctx* ctx = NULL;
  pfscdc_uwriter* uw = NULL;
  pfscdc_store* store = NULL;
  pfscdc_writer* w = NULL;
  uint32_t nfiles, f, i;
  uint64_t *lens, total = 0, k;
  uint8_t* data;
  char path[64];

  if (argc < 3) return 2;
  nfiles = (uint32_t)strtoul(argv[1], NULL, 10);
  rng_state = strtoull(argv[2], NULL, 10);
  lens = (uint64_t*)calloc(nfiles + 1, sizeof *lens);
  for (f = 0; f < nfiles; f++) {
    lens[f] = next_u64() % 90000;
    if (f % 9 == 4) lens[f] = 0;
    total += lens[f];
  }
  data = (uint8_t*)malloc(total + 1);
  if (!lens || !data) return 1;
  for (k = 0; k < total; k++) data[k] = (uint8_t)(next_u64() >> 56);

  pfscdc_default_params(&p);
  p.average_bits = 12;
  p.min_chunk = 2000;
  p.max_chunk = 30000;
  ip = p;
  ip.average_bits = 13;
  ip.seed = 0;
  ip.min_chunk = 3000;
  ip.max_chunk = 60000;
  OK(pfscdc_ctx_create(&p, 0, &ctx), ctx);
  OK(pfscdc_set_options(ctx, PFSCDC_OPT_REF_IDS), ctx);

  /* 1. UnorderedWriter: small memThreshold, two group writers, small groups */
  OK(pfscdc_set_knob("PFSCDC_UW_WORKERS", 2), NULL);
  OK(pfscdc_set_knob("PFSCDC_UW_INFLIGHT", 400000), NULL);
  OK(pfscdc_uw_create(ctx, 300000, &ip, on_uw, NULL, &uw), ctx);
  for (f = 0, k = 0; f < nfiles; k += lens[f], f++) {
    snprintf(path, sizeof path, "/d%u/f%05u", (unsigned)(next_u64() % 4), f);
    OK(pfscdc_uw_put(uw, path, (f % 3) ? "" : "t1", 0, data + k, lens[f]), ctx);
    if (f % 11 == 5) OK(pfscdc_uw_put(uw, path, "", 1, data, lens[f] / 2), ctx); /* append */
    if (f % 13 == 7) OK(pfscdc_uw_delete(uw, path, NULL), ctx);
    if (f == nfiles / 2) OK(pfscdc_uw_delete(uw, "/d3/", NULL), ctx); /* a directory */
  }
  OK(pfscdc_uw_close(uw), ctx);
  printf("uw filesets %u events %" PRIu64 " index %" PRIu64 "\n", pfscdc_uw_num_filesets(uw),
         uw_events, uw_index_events);
  for (i = 0; i < pfscdc_uw_num_filesets(uw); i++) {
    pfscdc_fileset_info fi;
    OK(pfscdc_uw_fileset(uw, i, &fi), ctx);
    printf("fileset %u %" PRId64 " %u %u %" PRIu64 " %" PRIu64 "\n", i, fi.size_bytes,
           fi.num_files, fi.num_deletes, fi.additive_root_len, fi.deletive_root_len);
  }
  OK(pfscdc_uw_destroy(uw), ctx);

  /* 2. a writer uploading into a store, then a second writer copying its DataRefs */
  OK(pfscdc_store_create(&store), NULL);
  OK(pfscdc_writer_create(ctx, on_chunk, (void*)1, 100000, &w), ctx);
  OK(pfscdc_writer_set_store(w, store, 1), ctx);
  for (f = 0, k = 0; f < nfiles; k += lens[f], f++) {
    OK(pfscdc_writer_annotate(w, f), ctx);
    OK(pfscdc_writer_write(w, data + k, lens[f]), ctx);
  }
  OK(pfscdc_writer_close(w), ctx);
  OK(pfscdc_writer_destroy(w), ctx);
  printf("writer chunks %" PRIu64 " stored %" PRIu64 " datarefs %u\n", chunks_seen,
         pfscdc_store_count(store), nrefs);

  chunks_seen = 0;
  OK(pfscdc_writer_create(ctx, on_chunk, NULL, 100000, &w), ctx);
  OK(pfscdc_writer_set_store(w, store, 0), ctx);
  OK(pfscdc_writer_prefetch(w, refs, nrefs), ctx);
  for (i = 0; i < nrefs; i++) {
    if (i == 0 || ref_file[i] != ref_file[i - 1]) OK(pfscdc_writer_annotate(w, ref_file[i]), ctx);
    OK(pfscdc_writer_copy(w, &refs[i]), ctx);
  }
  OK(pfscdc_writer_close(w), ctx);
  printf("copy chunks %" PRIu64 " cheap %" PRIu64 "\n", chunks_seen, copies_seen);
  OK(pfscdc_writer_destroy(w), ctx);

  /* 3. MergeFileReader.Hash over every DataRef as one file */
  {
    uint8_t h[32];
    OK(pfscdc_merge_file_hash(ctx, store, refs, nrefs, h), ctx);
    printf("merge_hash");
    for (i = 0; i < 32; i++) printf("%02x", h[i]);
    printf("\n");
  }
  OK(pfscdc_store_destroy(store), NULL);

  /* 4. four threads, four ctxs, the same batch */
  {
    pthread_t th[4];
    scan_job jobs[4];
    uint64_t* offs = (uint64_t*)calloc(nfiles + 1, sizeof *offs);
    if (!offs) return 1;
    for (f = 0; f < nfiles; f++) offs[f + 1] = offs[f] + lens[f];
    for (i = 0; i < 4; i++) {
      memset(&jobs[i], 0, sizeof jobs[i]);
      jobs[i].data = data;
      jobs[i].offs = offs;
      jobs[i].nfiles = nfiles;
      if (pthread_create(&th[i], NULL, scan_thread, &jobs[i]) != 0) return 1;
    }
    for (i = 0; i < 4; i++) pthread_join(th[i], NULL);
    for (i = 0; i < 4; i++) {
      if (jobs[i].rc != PFSCDC_OK || jobs[i].nsegs != jobs[0].nsegs ||
          memcmp(jobs[i].digest0, jobs[0].digest0, 32) != 0) {
        fprintf(stderr, "thread %u: rc %d, %" PRIu64 " segments\n", i, jobs[i].rc, jobs[i].nsegs);
        return 1;
      }
    }
    printf("threads 4 segments %" PRIu64 "\n", jobs[0].nsegs);
    free(offs);
  }
  /* 5. a device group of four ctxs on device 0: the batch dealt over them and gathered, then
   * an unordered writer over the group (four group writers, events released in group order) */
  {
    int devs[4] = {0, 0, 0, 0};
    pfscdc_group* g = NULL;
    pfscdc_uwriter* gw = NULL;
    uint64_t* offs = (uint64_t*)calloc(nfiles + 1, sizeof *offs);
    if (!offs) return 1;
    for (f = 0; f < nfiles; f++) offs[f + 1] = offs[f] + lens[f];
    OK(pfscdc_group_create(&p, devs, 4, PFSCDC_OPT_REF_IDS, &g), NULL);
    OK(pfscdc_group_scan(g, data, total, offs, nfiles), NULL);
    printf("group segments %" PRIu64 "\n", pfscdc_group_num_segments(g));
    uw_events = uw_index_events = 0;
    OK(pfscdc_uw_create_group(g, 300000, &ip, on_uw, NULL, &gw), NULL);
    for (f = 0, k = 0; f < nfiles; k += lens[f], f++) {
      snprintf(path, sizeof path, "/g/f%05u", f);
      OK(pfscdc_uw_put(gw, path, "", 0, data + k, lens[f]), NULL);
    }
    OK(pfscdc_uw_close(gw), NULL);
    printf("group uw filesets %u events %" PRIu64 "\n", pfscdc_uw_num_filesets(gw), uw_events);
    OK(pfscdc_uw_destroy(gw), NULL);
    OK(pfscdc_group_destroy(g), NULL);
    free(offs);
  }
  {
    uint64_t freed = 0;
    uint32_t ctxs = 0;
    OK(pfscdc_ctx_destroy(ctx), NULL);
    OK(pfscdc_uw_trim_cache(-1, &freed, &ctxs), NULL);
  }
  free(refs);
  free(ref_file);
  free(data);
  free(lens);
  printf("done\n");
  fflush(stdout);
  if (__lsan_do_leak_check) {
    __lsan_do_leak_check();
    fflush(stderr);
    _exit(0);
  }
  return 0;
}
