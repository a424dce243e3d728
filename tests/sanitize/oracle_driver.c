/* ASan/UBSan driver for the CPU-side C code (SURVEY.md §5 "sanitizers"): runs the oracle
 * restatement (oracle/sbam_oracle.c) over a BAM file -- whole-stream inflate, eager and full
 * checks at every position, splits at several sizes, FindBlockStart at every 997th offset,
 * the threaded CPU-baseline path -- so that an out-of-bounds read, an overflow or a data race
 * in the checker aborts the sanitized build.  Test infrastructure only. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sbam_oracle.h"

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 2;
  fseek(f, 0, SEEK_END);
  const long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t *data = malloc((size_t)n);
  if (!data || fread(data, 1, (size_t)n, f) != (size_t)n) return 2;
  fclose(f);
  or_stream *s = or_stream_open(data, n, 0);
  if (or_stream_load_all(s) != OR_OK && or_stream_size(s) == 0) return 3;
  int32_t cl[4096];
  int64_t hend = 0;
  const int32_t nref = or_parse_header(s, cl, 4096, &hend);
  const int64_t fs = or_stream_size(s);
  const int32_t nc = nref > 0 ? nref : 0;
  uint8_t *bits = calloc((size_t)(fs + 7) / 8 + 1, 1);
  const int64_t nt = or_eager_range(s, 0, fs, cl, nc, 10, bits);
  int64_t counts[21 * 19], rbe[21 * 64];
  memset(counts, 0, sizeof counts);
  memset(rbe, 0, sizeof rbe);
  uint32_t *words = malloc(sizeof(uint32_t) * (size_t)(fs + 1));
  const int64_t ns = or_full_range(s, 0, fs, cl, nc, 10, words, counts, rbe);
  const int64_t nrec = hend > 0 ? or_record_chain(s, hend, fs, NULL, 0) : 0;
  int64_t nsplit_total = 0;
  const int64_t sizes[3] = {20000, 100000, n};
  for (int k = 0; k < 3; ++k) {
    const int64_t m = or_file_splits(n, sizes[k], NULL, NULL, 0);
    int64_t *st = malloc(sizeof(int64_t) * (size_t)m), *en = malloc(sizeof(int64_t) * (size_t)m);
    or_file_splits(n, sizes[k], st, en, m);
    for (int64_t i = 0; i < m; ++i) {
      uint64_t v = 0;
      int64_t c = 0;
      if (or_split(data, n, st[i], en[i], cl, nc, 5, 10, 100000000, &v, &c) == OR_OK) nsplit_total += c;
    }
    free(st);
    free(en);
  }
  for (int64_t off = 0; off < n; off += 997) {
    int64_t out = 0;
    (void)or_find_block_start(data, n, off, 5, &out);
  }
  or_block blocks[4096];
  const int64_t nb = or_stream_blocks(s, blocks, 4096);
  int64_t pos = 0, tr = 0;
  (void)or_bench_inflate_check(data, n, blocks, 0, nb < 16 ? nb : 16, cl, nc, 10, 4, &pos, &tr);
  printf("flat %lld true %lld success %lld records %lld split-records %lld bench-positions %lld\n", (long long)fs,
         (long long)nt, (long long)ns, (long long)nrec, (long long)nsplit_total, (long long)pos);
  free(words);
  free(bits);
  or_stream_close(s);
  free(data);
  return 0;
}
