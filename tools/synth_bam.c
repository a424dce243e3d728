/*
 * synth_bam.c -- deterministic synthetic BAM generator for the benchmark shapes and
 * parity corpora (BASELINE.json configs B-E).  Test/bench
 * input generation only; not part of the product path.
 *
 * Records are a pure function of (seed, record index), so any record range can be
 * generated independently (multi-rank shards regenerate their neighbours' halo).
 * The uncompressed stream is cut into BGZF blocks of `payload` bytes (htsjdk-style
 * 65498 B; 65280 B for stored level-0 blocks so they fit BSIZE) and compressed with
 * zlib raw deflate on a thread pool.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#define SHAPE_SHORT 0
#define SHAPE_LONG 1
#define SHAPE_ADVERSARIAL 2

typedef struct {
  uint64_t seed;
  int32_t shape;       /* SHAPE_*                                               */
  int32_t level;       /* zlib level; -1 = per-block random of {0, 1, 9}        */
  int32_t payload;     /* uncompressed bytes per BGZF block (<= 65498)          */
  int32_t threads;
  int32_t empty_every; /* insert an empty BGZF block after every k blocks; 0=no */
  int32_t pad;
} synth_params;

static const char *CONTIG_NAMES[25] = {"1", "2", "3", "4", "5", "6", "7", "8", "9",
                                       "10", "11", "12", "13", "14", "15", "16", "17",
                                       "18", "19", "20", "21", "22", "X", "Y", "MT"};
/* GRCh37 primary contigs (check/src/test/.../header/ContigLengthsTest.scala:18-42) */
static const int32_t CONTIG_LENS[25] = {
    249250621, 243199373, 198022430, 191154276, 180915260, 171115067, 159138663,
    146364022, 141213431, 135534747, 135006516, 133851895, 115169878, 107349540,
    102531392, 90354753,  81195210,  78077248,  59128983,  63025520,  48129895,
    51304566,  155270560, 59373566,  16569};
#define N_CONTIGS 25
#define GENOME_LEN 3095693983LL

typedef struct { uint64_t s; } rng_t;
static inline uint64_t splitmix(uint64_t *x) {
  uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static inline uint64_t rnd(rng_t *r) { return splitmix(&r->s); }
static inline uint32_t rndu(rng_t *r, uint32_t n) { return (uint32_t)((rnd(r) >> 32) * n >> 32); }

static inline void put32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
static inline void put16(uint8_t *p, uint32_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }

/* SAM spec reg2bin */
static int reg2bin(int beg, int end) {
  --end;
  if (beg >> 14 == end >> 14) return ((1 << 15) - 1) / 7 + (beg >> 14);
  if (beg >> 17 == end >> 17) return ((1 << 12) - 1) / 7 + (beg >> 17);
  if (beg >> 20 == end >> 20) return ((1 << 9) - 1) / 7 + (beg >> 20);
  if (beg >> 23 == end >> 23) return ((1 << 6) - 1) / 7 + (beg >> 23);
  if (beg >> 26 == end >> 26) return ((1 << 3) - 1) / 7 + (beg >> 26);
  return 0;
}

static void locate(int64_t g, int32_t *ref, int32_t *pos) {
  g %= GENOME_LEN;
  for (int i = 0; i < N_CONTIGS; ++i) {
    if (g < CONTIG_LENS[i] - 60000) { *ref = i; *pos = (int32_t)g; return; }
    g -= CONTIG_LENS[i] - 60000;
  }
  *ref = 0; *pos = 0;
}

/* Header: BAM\1, l_text, text, n_ref, refs (SAM spec 4.2) */
int64_t synth_header(uint8_t *out, int64_t cap) {
  char text[4096];
  int t = snprintf(text, sizeof text, "@HD\tVN:1.6\tSO:coordinate\n");
  for (int i = 0; i < N_CONTIGS; ++i)
    t += snprintf(text + t, sizeof text - (size_t)t, "@SQ\tSN:%s\tLN:%d\n", CONTIG_NAMES[i], CONTIG_LENS[i]);
  t += snprintf(text + t, sizeof text - (size_t)t, "@RG\tID:rg1\tSM:synthetic\tPL:ILLUMINA\n");
  int64_t n = 12 + t;
  for (int i = 0; i < N_CONTIGS; ++i) n += 8 + (int64_t)strlen(CONTIG_NAMES[i]) + 1;
  if (!out) return n;
  if (cap < n) return -1;
  uint8_t *p = out;
  memcpy(p, "BAM\1", 4); p += 4;
  put32(p, (uint32_t)t); p += 4;
  memcpy(p, text, (size_t)t); p += t;
  put32(p, N_CONTIGS); p += 4;
  for (int i = 0; i < N_CONTIGS; ++i) {
    uint32_t l = (uint32_t)strlen(CONTIG_NAMES[i]) + 1;
    put32(p, l); p += 4;
    memcpy(p, CONTIG_NAMES[i], l); p += l;
    put32(p, (uint32_t)CONTIG_LENS[i]); p += 4;
  }
  return n;
}

static const char NT16[] = "=ACMGRSVTWYHKDBN";

/* Writes record `idx` to out (or only sizes it when out == NULL); returns its size
 * including the 4-byte block_size field. */
static int64_t make_record(const synth_params *P, int64_t idx, uint8_t *out) {
  rng_t r = {P->seed ^ ((uint64_t)idx * 0xD1B54A32D192ED03ull)};
  rnd(&r);
  int shape = P->shape;
  int32_t l_seq;
  int32_t n_cig;
  uint32_t cig[512];
  uint32_t flag;
  int unmapped_mid = 0, zero_seq = 0;
  if (shape == SHAPE_LONG) {
    l_seq = 10000 + (int32_t)rndu(&r, 40001);
    n_cig = 50 + (int32_t)rndu(&r, 451);
  } else {
    l_seq = 100;
    uint32_t u = rndu(&r, 100);
    n_cig = u < 85 ? 1 : 2 + (int32_t)rndu(&r, 3);
  }
  uint32_t mate = (uint32_t)(idx & 1);
  flag = 0x1 | 0x2 | (mate ? 0x80 : 0x40) | (rndu(&r, 2) ? 0x10 : 0x20);
  uint32_t u100 = rndu(&r, 100);
  if (u100 < 2) { flag |= 0x4; flag &= ~0x2u; n_cig = 0; }
  if (shape == SHAPE_ADVERSARIAL) {
    uint32_t a = rndu(&r, 100);
    if (a < 3) { flag = 0x4; n_cig = 0; unmapped_mid = 1; }           /* refID = pos = -1 */
    else if (a < 6) { flag = 0x4 | 0x1 | 0x40; n_cig = 0; zero_seq = 1; } /* l_seq = 0 */
    if (zero_seq) l_seq = 0;
  }
  /* cigar */
  if (n_cig == 1) cig[0] = ((uint32_t)l_seq << 4) | 0; /* 100M */
  else if (n_cig > 1) {
    int32_t left = l_seq;
    for (int i = 0; i < n_cig; ++i) {
      int last = i == n_cig - 1;
      uint32_t op = (i & 1) ? (rndu(&r, 3) == 0 ? 2 : (rndu(&r, 2) ? 1 : 4)) : 0; /* M/I/D/S */
      int32_t len = last ? left : 1 + (int32_t)rndu(&r, (uint32_t)(left / (n_cig - i) + 1));
      if (op == 2) len = 1 + (int32_t)rndu(&r, 20); /* D consumes no query */
      if (last && op != 0 && op != 1 && op != 4) op = 0;
      if (op != 2) { if (len > left) len = left; left -= len; }
      if (last && left > 0) len += left;
      cig[i] = ((uint32_t)(len > 0 ? len : 1) << 4) | op;
    }
  }
  /* read name "SYN:<run>:<lane>:<tile>:<x>:<y>" (pairs share a name) */
  char name[96];
  int64_t pair = idx >> 1;
  rng_t rn = {P->seed ^ ((uint64_t)pair * 0x9E3779B97F4A7C15ull) ^ 0x5A5A};
  int nl = snprintf(name, sizeof name, "SYN:%u:%u:%u:%u:%u", 1 + rndu(&rn, 9), 1 + rndu(&rn, 8),
                    1101 + rndu(&rn, 1200), rndu(&rn, 30000), rndu(&rn, 200000));
  int32_t l_name = nl + 1;
  /* coordinates: monotone in idx (coordinate-sorted) */
  int32_t ref, pos;
  locate(idx * (shape == SHAPE_LONG ? 900 : 3) + rndu(&r, 3), &ref, &pos);
  int32_t next_ref = ref, next_pos = pos + 150 + (int32_t)rndu(&r, 300);
  int32_t tlen = (mate ? -1 : 1) * (next_pos - pos + l_seq);
  if (unmapped_mid) { ref = -1; pos = -1; next_ref = -1; next_pos = -1; tlen = 0; }
  uint32_t mapq = (flag & 4) ? 0 : rndu(&r, 61);
  int32_t bin = reg2bin(pos < 0 ? 0 : pos, (pos < 0 ? 0 : pos) + (l_seq > 0 ? l_seq : 1));
  if (unmapped_mid) bin = 4680;
  /* tags */
  char md[32];
  int mdl = snprintf(md, sizeof md, "%d", l_seq);
  int64_t tag_bytes = (3 + 1) /*NM:c*/ + (3 + mdl + 1) /*MD:Z*/ + (3 + 4) /*RG:Z:rg1*/ +
                      (3 + 1) /*AS:C*/ + (3 + 1) /*XS:C*/;
  int bait = shape == SHAPE_ADVERSARIAL && rndu(&r, 100) < 20;
  int64_t bait_bytes = bait ? (3 + 1 + 4 + 48) : 0; /* XB:B:C,<48 bytes> */
  int64_t size = 4 + 32 + l_name + 4 * (int64_t)n_cig + (l_seq + 1) / 2 + l_seq + tag_bytes + bait_bytes;
  if (!out) return size;
  uint8_t *p = out;
  put32(p, (uint32_t)(size - 4));
  put32(p + 4, (uint32_t)ref);
  put32(p + 8, (uint32_t)pos);
  put32(p + 12, ((uint32_t)bin << 16) | (mapq << 8) | (uint32_t)l_name);
  put32(p + 16, (flag << 16) | (uint32_t)n_cig);
  put32(p + 20, (uint32_t)l_seq);
  put32(p + 24, (uint32_t)next_ref);
  put32(p + 28, (uint32_t)next_pos);
  put32(p + 32, (uint32_t)tlen);
  p += 36;
  memcpy(p, name, (size_t)l_name); p += l_name;
  for (int i = 0; i < n_cig; ++i) { put32(p, cig[i]); p += 4; }
  /* seq: 4-bit ACGT (N at ~1/1024), 2 random bits per base from a 64-bit pool */
  uint64_t pool = 0;
  int bits = 0;
  for (int i = 0; i < (l_seq + 1) / 2; ++i) {
    if (bits < 24) { pool = rnd(&r); bits = 64; }
    uint32_t a = 1u << (pool & 3), b = 1u << ((pool >> 2) & 3);
    if (((pool >> 4) & 1023) == 0) a = 15;
    pool >>= 14; bits -= 14;
    if (2 * i + 1 >= l_seq) b = 0;
    *p++ = (uint8_t)((a << 4) | b);
  }
  (void)NT16;
  /* qual: Phred 2..41, random walk (Illumina-like, compressible-ish) */
  int q = 30 + (int)rndu(&r, 10);
  bits = 0;
  for (int i = 0; i < l_seq; ++i) {
    if (bits < 8) { pool = rnd(&r); bits = 64; }
    uint32_t u = (uint32_t)(pool & 15), v = (uint32_t)((pool >> 4) & 7);
    pool >>= 7; bits -= 7;
    if (u == 0) q -= 1 + (int)v;
    else if (u == 1) q += 1 + (int)(v & 3);
    if (q < 2) q = 2;
    if (q > 41) q = 41;
    *p++ = (uint8_t)q;
  }
  memcpy(p, "NMc", 3); p[3] = (uint8_t)rndu(&r, 4); p += 4;
  memcpy(p, "MDZ", 3); memcpy(p + 3, md, (size_t)mdl + 1); p += 3 + mdl + 1;
  memcpy(p, "RGZrg1", 7); p += 7;
  memcpy(p, "ASC", 3); p[3] = (uint8_t)(80 + rndu(&r, 21)); p += 4;
  memcpy(p, "XSC", 3); p[3] = (uint8_t)rndu(&r, 80); p += 4;
  if (bait) {
    /* False-positive bait: bytes shaped like a plausible record start (valid refID/pos,
     * name length, flags) embedded in a byte array; later checks/chain fail. */
    memcpy(p, "XBBC", 4); put32(p + 4, 48); p += 8;
    uint8_t *b = p;
    memset(b, 0, 48);
    put32(b + 0, 200 + rndu(&r, 200));         /* block_size */
    put32(b + 4, (uint32_t)ref);                /* refID      */
    put32(b + 8, (uint32_t)pos);                /* pos        */
    put32(b + 12, (4680u << 16) | (30u << 8) | 6u);
    put32(b + 16, (0x4u << 16) | 0u);          /* unmapped, no cigar */
    put32(b + 20, 10);
    put32(b + 24, (uint32_t)ref);
    put32(b + 28, (uint32_t)pos);
    memcpy(b + 36, "bait!", 6);                 /* NUL-terminated name */
    p += 48;
  }
  return size;
}

/* Sizes of records [a, b) (prefix-summable); returns total bytes. */
int64_t synth_records_size(const synth_params *P, int64_t a, int64_t b) {
  int64_t t = 0;
  for (int64_t i = a; i < b; ++i) t += make_record(P, i, NULL);
  return t;
}

/* Number of records starting in [0, target_bytes) of the record stream. */
int64_t synth_records_for_bytes(const synth_params *P, int64_t target_bytes) {
  int64_t t = 0, i = 0;
  while (t < target_bytes) t += make_record(P, i++, NULL);
  return i;
}

typedef struct {
  const synth_params *P;
  int64_t a, b, off;
  uint8_t *out;
  int pass;
} rjob;

static void *rworker(void *arg) {
  rjob *j = (rjob *)arg;
  if (j->pass == 0) {
    j->off = synth_records_size(j->P, j->a, j->b);
  } else {
    int64_t t = j->off;
    for (int64_t i = j->a; i < j->b; ++i) t += make_record(j->P, i, j->out + t);
  }
  return NULL;
}

/* Writes records [a, b) to out (parallel over P->threads); returns bytes written
 * (or -1 if cap is too small). */
int64_t synth_records(const synth_params *P, int64_t a, int64_t b, uint8_t *out, int64_t cap) {
  int T = P->threads > 0 ? P->threads : 1;
  if (b - a < 1024) T = 1;
  pthread_t *th = (pthread_t *)calloc((size_t)T, sizeof *th);
  rjob *jobs = (rjob *)calloc((size_t)T, sizeof *jobs);
  for (int pass = 0; pass < 2; ++pass) {
    for (int i = 0; i < T; ++i) {
      jobs[i].P = P; jobs[i].out = out; jobs[i].pass = pass;
      jobs[i].a = a + (b - a) * i / T; jobs[i].b = a + (b - a) * (i + 1) / T;
      pthread_create(&th[i], NULL, rworker, &jobs[i]);
    }
    for (int i = 0; i < T; ++i) pthread_join(th[i], NULL);
    if (pass == 0) { /* exclusive prefix sum of chunk sizes */
      int64_t t = 0;
      for (int i = 0; i < T; ++i) { int64_t s = jobs[i].off; jobs[i].off = t; t += s; }
      if (t > cap) { free(th); free(jobs); return -1; }
    }
  }
  int64_t total = jobs[T - 1].off + synth_records_size(P, jobs[T - 1].a, jobs[T - 1].b);
  free(th); free(jobs);
  return total;
}

/* ------------------------------------------------------------------------- */
/* BGZF compression */
static const uint8_t BGZF_EOF[28] = {0x1f, 0x8b, 0x08, 0x04, 0, 0, 0, 0, 0, 0xff, 0x06, 0,
                                     0x42, 0x43, 0x02, 0, 0x1b, 0, 0x03, 0, 0, 0, 0, 0, 0, 0, 0, 0};

static int block_level(const synth_params *P, int64_t k) {
  if (P->level >= 0) return P->level;
  uint64_t x = P->seed ^ ((uint64_t)k * 0xA24BAED4963EE407ull);
  static const int L[3] = {0, 1, 9};
  return L[splitmix(&x) % 3];
}

/* Compress one BGZF block into out (>= 65536 B); returns its size or -1. */
static int compress_block(const uint8_t *src, int32_t n, int level, uint8_t *out) {
  z_stream zs;
  memset(&zs, 0, sizeof zs);
  if (deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return -1;
  zs.next_in = (Bytef *)src;
  zs.avail_in = (uInt)n;
  zs.next_out = out + 18;
  zs.avail_out = 65536 - 26;
  int zr = deflate(&zs, Z_FINISH);
  int32_t clen = (int32_t)(65536 - 26 - zs.avail_out);
  deflateEnd(&zs);
  if (zr != Z_STREAM_END) return -1;
  int32_t bsize = clen + 26;
  memcpy(out, BGZF_EOF, 16);
  put16(out + 16, (uint32_t)(bsize - 1));
  put32(out + 18 + clen, (uint32_t)crc32(crc32(0, Z_NULL, 0), src, (uInt)n));
  put32(out + 22 + clen, (uint32_t)n);
  return bsize;
}

typedef struct {
  const synth_params *P;
  const uint8_t *U;
  const int64_t *bstart; /* uncompressed start of each block */
  const int32_t *blen;
  int64_t k0, k1, kbase;
  uint8_t *buf;
  int64_t used;
  int err;
} cjob;

static void *cworker(void *arg) {
  cjob *j = (cjob *)arg;
  for (int64_t k = j->k0; k < j->k1; ++k) {
    int c = compress_block(j->U + j->bstart[k], j->blen[k], block_level(j->P, j->kbase + k), j->buf + j->used);
    if (c < 0) { j->err = 1; return NULL; }
    j->used += c;
    if (j->P->empty_every > 0 && ((j->kbase + k + 1) % j->P->empty_every) == 0) {
      memcpy(j->buf + j->used, BGZF_EOF, 28); /* empty block mid-file */
      j->used += 28;
    }
  }
  return NULL;
}

/* BGZF-compress U[0, n) into out.  Block k (global index kbase + k) gets the level
 * of block_level(); payload P->payload (65280 for stored blocks).  Appends the EOF
 * block when add_eof.  Returns compressed bytes or -1.  *n_blocks receives the data
 * block count. */
int64_t synth_bgzf(const synth_params *P, const uint8_t *U, int64_t n, int64_t kbase,
                   int add_eof, uint8_t *out, int64_t cap, int64_t *n_blocks) {
  int64_t nb_cap = n / 32768 + 16, nb = 0;
  int64_t *bstart = (int64_t *)malloc((size_t)nb_cap * sizeof(int64_t));
  int32_t *blen = (int32_t *)malloc((size_t)nb_cap * sizeof(int32_t));
  for (int64_t u = 0; u < n;) {
    int lvl = block_level(P, kbase + nb);
    int32_t pl = P->payload > 0 ? P->payload : 65498;
    if (lvl == 0 && pl > 65280) pl = 65280;
    if (u + pl > n) pl = (int32_t)(n - u);
    bstart[nb] = u;
    blen[nb] = pl;
    ++nb;
    u += pl;
  }
  int T = P->threads > 0 ? P->threads : 1;
  if (T > nb) T = nb > 0 ? (int)nb : 1;
  pthread_t *th = (pthread_t *)calloc((size_t)T, sizeof *th);
  cjob *jobs = (cjob *)calloc((size_t)T, sizeof *jobs);
  int64_t total = 0;
  int err = 0;
  for (int i = 0; i < T; ++i) {
    cjob *j = &jobs[i];
    j->P = P; j->U = U; j->bstart = bstart; j->blen = blen; j->kbase = kbase;
    j->k0 = nb * i / T; j->k1 = nb * (i + 1) / T;
    j->buf = (uint8_t *)malloc((size_t)(j->k1 - j->k0) * (65536 + 28) + 64);
    pthread_create(&th[i], NULL, cworker, j);
  }
  for (int i = 0; i < T; ++i) {
    pthread_join(th[i], NULL);
    cjob *j = &jobs[i];
    if (j->err || total + j->used > cap) err = 1;
    if (!err) memcpy(out + total, j->buf, (size_t)j->used);
    total += j->used;
    free(j->buf);
  }
  if (add_eof && !err) {
    if (total + 28 > cap) err = 1;
    else { memcpy(out + total, BGZF_EOF, 28); total += 28; }
  }
  free(th); free(jobs); free(bstart); free(blen);
  if (n_blocks) *n_blocks = nb;
  return err ? -1 : total;
}

/* Whole file: header + records [0, n_records), BGZF-compressed with EOF block.
 * out must hold at least synth_bam_bound(). Returns compressed size or -1. */
int64_t synth_bam_bound(const synth_params *P, int64_t n_records) {
  int64_t u = synth_header(NULL, 0) + synth_records_size(P, 0, n_records);
  return u + (u / 32768 + 2) * 128 + 1024;
}

int64_t synth_bam(const synth_params *P, int64_t n_records, uint8_t *out, int64_t cap,
                  int64_t *usize_out, int64_t *n_blocks) {
  int64_t h = synth_header(NULL, 0);
  int64_t rs = synth_records_size(P, 0, n_records);
  uint8_t *U = (uint8_t *)malloc((size_t)(h + rs));
  if (!U) return -1;
  synth_header(U, h);
  synth_records(P, 0, n_records, U + h, rs);
  int64_t c = synth_bgzf(P, U, h + rs, 0, 1, out, cap, n_blocks);
  free(U);
  if (usize_out) *usize_out = h + rs;
  return c;
}
