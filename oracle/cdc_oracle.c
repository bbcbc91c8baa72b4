/*
 * cdc_oracle.c — C restatement of the reference chunker (TEST INFRASTRUCTURE / CPU BASELINE).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this library
 * (oracle/_build/liboracle.so).  It is the checker and the CPU column, never the product.
 *
 * Restated from (paths under /root/reference):
 *   src/internal/storage/chunk/writer.go:100-103   resetHash: Reset + Write(64 zero bytes)
 *   src/internal/storage/chunk/writer.go:118-130   Annotate: reset hash + seglen per file
 *   src/internal/storage/chunk/writer.go:163-189   roll: per-byte Roll, Sum64 & mask, min/max
 *   src/internal/storage/chunk/writer.go:240,301-312  DataRef.Hash = BLAKE2b-256(segment)
 *   src/internal/pachhash/hash.go:27-30            blake2b.Sum256 (x/crypto, RFC 7693)
 *   third-party buzhash64 v4.0.0 Roll: sum = rotl(sum,1) ^ rotl(T[out], 64%64) ^ T[in]
 *
 * The rolling loop is the literal per-byte recurrence (a ring of the last 64 bytes), one
 * stream per file exactly like one chunk.Writer per annotation; files are spread over
 * pthreads the way independent writers run on independent goroutines.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

/* ---------------- BLAKE2b-256 (RFC 7693), unkeyed ---------------- */

static const uint64_t B2_IV[8] = {
    0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
    0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
    0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

static const uint8_t B2_SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

static inline uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

static void b2_compress(uint64_t h[8], const uint8_t blk[128], uint64_t t, int last) {
    uint64_t v[16], m[16];
    for (int i = 0; i < 16; i++) {
        uint64_t w = 0;
        for (int b = 7; b >= 0; b--) w = (w << 8) | blk[8 * i + b];
        m[i] = w;
    }
    for (int i = 0; i < 8; i++) { v[i] = h[i]; v[i + 8] = B2_IV[i]; }
    v[12] ^= t;          /* counter low word; high word stays 0 below 2^64 bytes */
    if (last) v[14] = ~v[14];
#define G(a, b, c, d, x, y)                      \
    do {                                         \
        v[a] = v[a] + v[b] + (x);                \
        v[d] = rotr64(v[d] ^ v[a], 32);          \
        v[c] = v[c] + v[d];                      \
        v[b] = rotr64(v[b] ^ v[c], 24);          \
        v[a] = v[a] + v[b] + (y);                \
        v[d] = rotr64(v[d] ^ v[a], 16);          \
        v[c] = v[c] + v[d];                      \
        v[b] = rotr64(v[b] ^ v[c], 63);          \
    } while (0)
    for (int r = 0; r < 12; r++) {
        const uint8_t *s = B2_SIGMA[r];
        G(0, 4, 8, 12, m[s[0]], m[s[1]]);
        G(1, 5, 9, 13, m[s[2]], m[s[3]]);
        G(2, 6, 10, 14, m[s[4]], m[s[5]]);
        G(3, 7, 11, 15, m[s[6]], m[s[7]]);
        G(0, 5, 10, 15, m[s[8]], m[s[9]]);
        G(1, 6, 11, 12, m[s[10]], m[s[11]]);
        G(2, 7, 8, 13, m[s[12]], m[s[13]]);
        G(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
#undef G
    for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[i + 8];
}

void oracle_blake2b256(const uint8_t *data, uint64_t n, uint8_t out[32]) {
    uint64_t h[8];
    memcpy(h, B2_IV, sizeof h);
    h[0] ^= 0x01010000ULL ^ 32; /* digest 32, no key, fanout 1, depth 1 */
    uint64_t off = 0;
    while (n - off > 128) {
        b2_compress(h, data + off, off + 128, 0);
        off += 128;
    }
    uint8_t last[128];
    memset(last, 0, sizeof last);
    memcpy(last, data + off, (size_t)(n - off));
    b2_compress(h, last, n, 1);
    for (int i = 0; i < 4; i++)
        for (int b = 0; b < 8; b++) out[8 * i + b] = (uint8_t)(h[i] >> (8 * b));
}

/* ---------------- CDC segmentation (writer.go:163-189) ---------------- */

typedef struct {
    uint32_t average_bits;
    uint32_t _pad;
    int64_t min_chunk;
    int64_t max_chunk;
} oracle_params;

typedef struct {
    uint64_t offset;  /* within the file */
    uint64_t size;
    uint32_t file;
    uint32_t flags;   /* bit0: valid, bit1: ends at a cut */
    uint8_t hash[32];
} oracle_seg;          /* 56 bytes, same layout as pfscdc_segment */

static inline uint64_t rotl1(uint64_t x) { return (x << 1) | (x >> 63); }

/* Segments one annotation exactly like a chunk.Writer that has just been Annotate()d:
 * hash reset to the 64-zero window, seglen counted from the file start. */
static uint64_t segment_file(const uint8_t *x, uint64_t n, const uint64_t T[256],
                             const oracle_params *p, uint32_t file, int do_hash,
                             oracle_seg *out) {
    const uint64_t mask = (1ULL << p->average_bits) - 1;
    uint8_t win[64];
    memset(win, 0, sizeof win);
    uint64_t h = 0;
    for (int j = 0; j < 64; j++) h = rotl1(h) ^ T[0];  /* Write(initialWindow) */
    unsigned oldest = 0;
    uint64_t segstart = 0, nseg = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint8_t b = x[i];
        uint64_t ho = T[win[oldest]];
        win[oldest] = b;
        oldest = (oldest + 1) & 63;
        h = rotl1(h) ^ ho ^ T[b];                      /* rotl(ho, 64%64) == ho (E4) */
        uint64_t seglen = i + 1 - segstart;
        int cut;
        if ((h & mask) == 0)
            cut = seglen >= (uint64_t)p->min_chunk;
        else
            cut = seglen >= (uint64_t)p->max_chunk;
        if (cut) {
            oracle_seg *s = &out[nseg++];
            s->offset = segstart;
            s->size = seglen;
            s->file = file;
            s->flags = 3;
            if (do_hash) oracle_blake2b256(x + segstart, seglen, s->hash);
            segstart = i + 1;
            memset(win, 0, sizeof win);               /* createChunk -> resetHash */
            h = 0;
            for (int j = 0; j < 64; j++) h = rotl1(h) ^ T[0];
            oldest = 0;
        }
    }
    if (segstart < n) {
        oracle_seg *s = &out[nseg++];
        s->offset = segstart;
        s->size = n - segstart;
        s->file = file;
        s->flags = 1;
        if (do_hash) oracle_blake2b256(x + segstart, n - segstart, s->hash);
    }
    return nseg;
}

typedef struct {
    const uint8_t *data;
    const uint64_t *offsets;
    const uint64_t *seg_base;
    const uint64_t *T;
    const oracle_params *p;
    oracle_seg *out;
    uint64_t *nseg;
    uint32_t nfiles;
    uint32_t nthreads;
    uint32_t tid;
    int do_hash;
} job_t;

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    for (uint32_t f = j->tid; f < j->nfiles; f += j->nthreads) {
        uint64_t a = j->offsets[f], b = j->offsets[f + 1];
        j->nseg[f] = segment_file(j->data + a, b - a, j->T, j->p, f, j->do_hash,
                                  j->out + j->seg_base[f]);
    }
    return NULL;
}

/* Upper bound on segments of a file of n bytes: every segment but the last is >= min. */
uint64_t oracle_max_segments(uint64_t n, int64_t min_chunk) {
    return n == 0 ? 0 : n / (uint64_t)min_chunk + 1;
}

/* Segments every file of a batch independently (one fresh writer per annotation).
 * out must hold sum_f oracle_max_segments(len_f); seg_base[f] gives file f's slot range and
 * nseg[f] receives its count.  Returns 0, or -1 on bad arguments. */
int oracle_segment_files(const uint8_t *data, const uint64_t *offsets, uint32_t nfiles,
                         const uint64_t *table, const oracle_params *p, int nthreads,
                         int do_hash, const uint64_t *seg_base, oracle_seg *out,
                         uint64_t *nseg) {
    if (p->min_chunk < 1 || p->max_chunk < p->min_chunk || p->average_bits > 63) return -1;
    if (nthreads < 1) nthreads = 1;
    if ((uint32_t)nthreads > nfiles && nfiles > 0) nthreads = (int)nfiles;
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    job_t *jobs = (job_t *)calloc((size_t)nthreads, sizeof(job_t));
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (job_t){data, offsets, seg_base, table, p, out, nseg, nfiles,
                          (uint32_t)nthreads, (uint32_t)t, do_hash};
        if (nthreads == 1) worker(&jobs[t]);
        else pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
    return 0;
}

/* Candidate positions of one stream (h_i & mask == 0, i >= 63), literal rolling from a reset
 * at position 0 and never reset again; used to check the GPU candidate scan. */
uint64_t oracle_candidates(const uint8_t *x, uint64_t n, const uint64_t *T,
                           uint32_t average_bits, uint64_t *out, uint64_t cap) {
    const uint64_t mask = (1ULL << average_bits) - 1;
    uint8_t win[64];
    memset(win, 0, sizeof win);
    uint64_t h = 0, cnt = 0;
    for (int j = 0; j < 64; j++) h = rotl1(h) ^ T[0];
    unsigned oldest = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t ho = T[win[oldest]];
        win[oldest] = x[i];
        oldest = (oldest + 1) & 63;
        h = rotl1(h) ^ ho ^ T[x[i]];
        if ((h & mask) == 0 && i >= 63) {
            if (cnt < cap) out[cnt] = i;
            cnt++;
        }
    }
    return cnt;
}
