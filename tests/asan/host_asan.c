/*
 * host_asan.c -- TEST HARNESS: the engine's host C layer (csrc/host/*.c)
 * built alone with AddressSanitizer + UBSan (gcc), driven over the golden
 * fixtures: index load / transforms / save, the host builder with SA samples,
 * query and result I/O, sample files, and the error paths (missing, wrong-tag
 * and truncated files), and searchIndexCPU on every tag against the
 * reference searchers' result files.  The HIP layer is replaced by the stubs
 * below (the handles never reach a device here).
 *
 *   host_asan <golden_dir> <tmp_dir> <case> <k> <d> <m> <num>
 * Prints "OK <checks>" and exits 0 when every check passes.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../../k-step_fm-index_amd/csrc/kfmi_internal.h"

/* ---- stubs for the HIP layer (csrc/hip) ---- */
int32_t freeIndexGPU(void **index) { (void) index; return KFMI_SUCCESS; }
int32_t kfmi_host_entries(kfmi_fmi_t *f) { return f->h_index ? KFMI_SUCCESS : KFMI_E_NOT_ON_DEVICE; }
void kfmi_free_dev_entries(kfmi_fmi_t *f) { f->d_entries = NULL; }
int32_t freeQueriesGPU(void **q) { (void) q; return KFMI_SUCCESS; }
int32_t freeResultsGPU(void **r) { (void) r; return KFMI_SUCCESS; }
kfmi_backend_t kfmi_backend(void) { return KFMI_BK_TASK_MID; }
uint32_t kfmi_backend_tag(kfmi_backend_t b) { (void) b; return 101u; }
int32_t kfmi_device_count(void) { return 0; }
int32_t kfmi_build_index_gpu_sa(const char *t, uint64_t n, uint32_t k, uint32_t d, uint32_t r, void **i)
{ (void) t; (void) n; (void) k; (void) d; (void) r; (void) i; return KFMI_E_NO_DEVICE; }
int32_t kfmi_build_index_gpu(const char *t, uint64_t n, uint32_t k, uint32_t d, int32_t h, void **i)
{ (void) h; return kfmi_build_index_gpu_sa(t, n, k, d, 0, i); }
static __thread int32_t last_error;
void kfmi_set_last_error(int32_t e) { last_error = e; }
int32_t kfmi_last_error(void) { return last_error; }

static int checks = 0, failures = 0;
#define CHECK(cond, ...) do { checks++; if (!(cond)) { failures++; fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
  fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); } } while (0)

static unsigned char *slurp(const char *fn, size_t *len)
{
  FILE *fp = fopen(fn, "rb");
  unsigned char *b;
  long n;
  if (!fp) return NULL;
  fseek(fp, 0, SEEK_END); n = ftell(fp); fseek(fp, 0, SEEK_SET);
  b = (unsigned char *) malloc((size_t) n + 1);
  if (fread(b, 1, (size_t) n, fp) != (size_t) n) { free(b); fclose(fp); return NULL; }
  fclose(fp);
  *len = (size_t) n;
  return b;
}

static int same_image(void *index, const char *fn)
{
  size_t len = 0;
  const void *img; uint64_t bytes;
  unsigned char *want = slurp(fn, &len);
  int ok = want && kfmi_index_image(index, &img, &bytes) == 0 && bytes == len && !memcmp(img, want, len);
  free(want);
  return ok;
}

int main(int argc, char **argv)
{
  char p[1024], q[1024];
  const char *g, *tmp, *cs;
  uint32_t k, d, m, num, tag;
  void *idx = NULL, *t101 = NULL, *t200 = NULL, *t201 = NULL, *re = NULL;
  if (argc < 8) { fprintf(stderr, "usage\n"); return 2; }
  g = argv[1]; tmp = argv[2]; cs = argv[3];
  k = (uint32_t) atoi(argv[4]); d = (uint32_t) atoi(argv[5]); m = (uint32_t) atoi(argv[6]); num = (uint32_t) atoi(argv[7]);

  /* 1. every tag loads byte-identically; transforms reproduce the reference files */
  for (tag = 100; tag <= 201; tag += (tag == 101 ? 99 : 1)) {
    void *x = NULL;
    snprintf(p, sizeof p, "%s/%s/k%u_d%u.%u.fmi", g, cs, k, d, tag);
    CHECK(loadIndex(p, &x) == 0 && same_image(x, p), "load %s", p);
    freeIndex(&x);
  }
  snprintf(p, sizeof p, "%s/%s/k%u_d%u.100.fmi", g, cs, k, d);
  CHECK(loadIndex(p, &idx) == 0, "load 100");
  CHECK(kfmi_transform_interleave(idx, &t101) == 0, "interleave");
  CHECK(kfmi_transform_ac(idx, &t200, &t201) == 0, "ac");
  snprintf(q, sizeof q, "%s/%s/k%u_d%u.101.fmi", g, cs, k, d); CHECK(same_image(t101, q), "101 bytes");
  snprintf(q, sizeof q, "%s/%s/k%u_d%u.200.fmi", g, cs, k, d); CHECK(same_image(t200, q), "200 bytes");
  snprintf(q, sizeof q, "%s/%s/k%u_d%u.201.fmi", g, cs, k, d); CHECK(same_image(t201, q), "201 bytes");
  CHECK(kfmi_transform_interleave(t101, &re) == KFMI_INDEX_VER_BASELINE, "transform needs tag 100");
  /* the inverse of the AltCounters transform: both AC files back to the .fmi */
  CHECK(kfmi_transform_plain(t200, &re) == 0 && same_image(re, p), "200 -> 100 bytes");
  freeIndex(&re);
  CHECK(kfmi_transform_plain(t201, &re) == 0 && same_image(re, p), "201 -> 100 bytes");
  freeIndex(&re);
  CHECK(kfmi_transform_plain(idx, &re) == KFMI_INDEX_VER_BASELINE_AC && re == NULL, "inverse needs tag 200/201");

  /* 2. save + reload round trip under the reference file names */
  snprintf(q, sizeof q, "%s/x.fmi", tmp);
  CHECK(saveIndex(q, t201) == 0, "save 201");
  snprintf(q, sizeof q, "%s/x.fmi.interleaving.ac", tmp);
  CHECK(loadIndex(q, &re) == 0 && same_image(re, q), "reload 201");
  freeIndex(&re);

  /* 3. strict loader and broken files */
  CHECK(kfmi_load_index_tag(p, 101, &re) == 101 && re == NULL, "strict tag");
  snprintf(q, sizeof q, "%s/missing.fmi", tmp);
  CHECK(loadIndex(q, &re) == KFMI_E_OPENING_INDEX_FILE, "missing file");
  {
    size_t len = 0;
    unsigned char *b = slurp(p, &len);
    FILE *fp;
    snprintf(q, sizeof q, "%s/trunc.fmi", tmp);
    fp = fopen(q, "wb"); fwrite(b, 1, len / 2, fp); fclose(fp);
    CHECK(loadIndex(q, &re) == KFMI_E_READING_FMI && re == NULL, "truncated body");
    fp = fopen(q, "wb"); fwrite(b, 1, 10, fp); fclose(fp);
    CHECK(loadIndex(q, &re) != 0 && re == NULL, "truncated header");
    CHECK(kfmi_index_from_image(b, 20, &re) != 0 && re == NULL, "short image");
    b[0] = 77;
    CHECK(kfmi_index_from_image(b, len, &re) != 0 && re == NULL, "bad tag");
    free(b);
  }

  /* 4. host builder (SA-IS) equals the reference builder's file; SA samples; sample file */
  {
    size_t len = 0, i, n = 0;
    char *fa, *text;
    snprintf(q, sizeof q, "%s/%s/ref.fa", g, cs);
    fa = (char *) slurp(q, &len);
    CHECK(fa != NULL, "ref.fa");
    text = (char *) malloc(len + 1);
    for (i = 0; fa && i < len && fa[i] != '\n'; i++) {}
    for (; fa && i < len; i++) if (fa[i] != '\n') text[n++] = fa[i];
    CHECK(kfmi_build_index_ex(text, n, k, d, 8, 0, &re) == 0 && same_image(re, p), "host builder");
    {
      const uint32_t *sa; uint64_t cnt; uint32_t rate;
      void *x = NULL;
      CHECK(kfmi_index_sa(re, &sa, &cnt, &rate) == 0 && rate == 8 && cnt == (n + 1 + 7) / 8 && sa[0] == n, "sa");
      snprintf(q, sizeof q, "%s/x.sa", tmp);
      CHECK(kfmi_save_sa(q, re) == 0, "save sa");
      CHECK(loadIndex(p, &x) == 0 && kfmi_load_sa(q, x) == 0, "load sa");
      { const uint32_t *sb; uint64_t c2; uint32_t r2;
        kfmi_index_sa(x, &sb, &c2, &r2);
        CHECK(c2 == cnt && r2 == rate && !memcmp(sa, sb, 4 * cnt), "sa roundtrip"); }
      CHECK(kfmi_load_sa(p, x) == KFMI_E_READING_FMI, "not a sample file");
      freeIndex(&x);
    }
    freeIndex(&re);
    CHECK(kfmi_build_index_ex(text, n, k, d, 3, 0, &re) == KFMI_E_BAD_ARGUMENT && re == NULL, "rate 3");
    CHECK(kfmi_build_index_ex("ACGN", 4, k, d, 0, 0, &re) != 0 && re == NULL, "non-ACGT");
    CHECK(kfmi_build_index_ex(text, n, k, d, 0, 1, &re) == KFMI_E_NO_DEVICE, "no device");
    /* tiny and odd texts, every K, a few d */
    for (uint32_t kk = 1; kk <= 4; kk++)
      for (uint32_t dd = 32; dd <= 96; dd += 32)
        for (size_t nn = 1; nn < 70 && nn <= n; nn += 7) {
          int e = kfmi_build_index_ex(text, nn, kk, dd, 2, 0, &re);
          CHECK(nn + 1 < kk ? e != 0 : e == 0, "tiny build k=%u d=%u n=%zu -> %d", kk, dd, nn, e);
          freeIndex(&re);
        }
    free(text);
    free(fa);
  }

  /* 5. queries, results */
  {
    void *qs = NULL, *rs = NULL, *rl = NULL;
    snprintf(q, sizeof q, "%s/%s/q%u.qry", g, cs, m);
    CHECK(loadQueries(q, m, num, &qs) == 0, "queries");
    freeQueries(&qs);
    CHECK(loadQueries(q, m + 1, num, &qs) != 0 && qs == NULL, "wrong length");
    CHECK(loadQueries(q, m, num + 1, &qs) != 0 && qs == NULL, "too few reads");
    snprintf(q, sizeof q, "%s/%s/k%u_d%u.q%u.cpu.res", g, cs, k, d, m);
    CHECK(loadResults(q, &rs) == 0, "results");
    snprintf(p, sizeof p, "%s/out", tmp);
    CHECK(saveResults(p, rs, NULL) == 0, "save results");
    snprintf(p, sizeof p, "%s/out.res.gpu", tmp);
    {
      size_t l1 = 0, l2 = 0;
      unsigned char *a = slurp(q, &l1), *b = slurp(p, &l2);
      CHECK(a && b && l1 == l2 && !memcmp(a, b, l1), "results bytes");
      free(a); free(b);
    }
    CHECK(loadResults(p, &rl) == 0, "reload results");
    freeResults(&rs); freeResults(&rl);
  }
  /* 6. host query packing on exactly-sized buffers, every length 1..300 */
  for (uint32_t mm = 1; mm <= 300; mm++) {
    const uint32_t nr = 3, nw = (mm + 15) / 16;
    char *a = malloc((size_t) nr * mm);
    uint32_t *w = malloc((size_t) nw * nr * 4);
    for (uint32_t i = 0; i < nr * mm; i++) a[i] = "ACGTNacgt"[(i * 7u + mm) % 9u];
    CHECK(a && w && kfmi_pack_queries(a, nr, mm, w) == 0, "pack m=%u", mm);
    /* base 0 of read 1 (reversed index mm-1) sits at bits 2(mm-1) of its string */
    const uint32_t r = mm - 1, c = base2index((uint32_t) (unsigned char) a[mm]);
    CHECK(((w[(r / 16) * nr + 1] >> (2 * (r % 16))) & 3u) == c, "pack first base m=%u", mm);
    CHECK(r % 16 == 15 || (w[(r / 16) * nr + 1] >> (2 * (r % 16) + 2)) == 0, "pack zero tail m=%u", mm);
    free(a);
    free(w);
  }
  CHECK(kfmi_pack_queries(NULL, 1, 4, NULL) == KFMI_E_BAD_ARGUMENT, "pack null");

  /* 7. searchIndexCPU on every tag: results files equal the reference searchers' */
  for (tag = 100; tag <= 201; tag += (tag == 101 ? 99 : 1)) {
    void *x = NULL, *qs = NULL, *rs = NULL;
    size_t l1 = 0, l2 = 0;
    unsigned char *a, *b;
    snprintf(p, sizeof p, "%s/%s/k%u_d%u.%u.fmi", g, cs, k, d, tag);
    snprintf(q, sizeof q, "%s/%s/q%u.qry", g, cs, m);
    CHECK(loadIndex(p, &x) == 0 && loadQueries(q, m, num, &qs) == 0 && initResults(num, &rs) == 0, "cpu inputs");
    CHECK(kfmi_search_cpu(x, qs, rs, 3) == 0, "searchIndexCPU tag %u", tag);
    snprintf(p, sizeof p, "%s/cpu%u", tmp, tag);
    CHECK(saveResults(p, rs, x) == 0, "save cpu results");
    snprintf(p, sizeof p, "%s/cpu%u.res.cpu", tmp, tag);
    snprintf(q, sizeof q, "%s/%s/k%u_d%u.q%u.%s.res", g, cs, k, d, m, tag < 200 ? "cpu" : "cpuac");
    a = slurp(q, &l1); b = slurp(p, &l2);
    CHECK(a && b && l1 == l2 && !memcmp(a, b, l1), "cpu results bytes tag %u", tag);
    free(a); free(b);
    freeResults(&rs); freeQueries(&qs); freeIndex(&x);
  }

  /* 8. big host buffers: below 64 MB calloc, from 64 MB a 2 MB-aligned mapping
   *    (unless KFMI_HUGEPAGES=0); zeroed, writable to the last byte, freed by
   *    kfmi_big_free either way (and NULL is a no-op) */
  {
    const uint64_t sizes[3] = {1000, (64ull << 20) + 12345, (80ull << 20)};
    int t;
    for (t = 0; t < 3; ++t) {
      unsigned char *bp = (unsigned char *) kfmi_big_alloc(sizes[t]);
      uint64_t j, nz = 0;
      CHECK(bp != NULL, "big alloc %llu", (unsigned long long) sizes[t]);
      if (!bp) continue;
      if (sizes[t] >= (64ull << 20))
        CHECK(((uintptr_t) bp & ((2u << 20) - 1)) == 0, "big alloc 2 MB aligned");
      for (j = 0; j < sizes[t]; j += 4093) nz += bp[j] != 0;
      nz += bp[sizes[t] - 1] != 0;
      CHECK(nz == 0, "big alloc zeroed");
      memset(bp, 0x5a, sizes[t]);
      kfmi_big_free(bp);
    }
    kfmi_big_free(NULL);
  }

  /* 9. damaged headers: every tag's image with one header word replaced (the
   *    size fields, a '$' row or its code; the body cut to what the header then
   *    asks for) either fails to load or loads, searches and transforms inside
   *    its own buffers -- ASan reports any read or write outside them */
  {
    void *qs = NULL;
    uint32_t lcg = 12345u + k * 7u + d;
    snprintf(q, sizeof q, "%s/%s/q%u.qry", g, cs, m);
    CHECK(loadQueries(q, m, num < 64 ? num : 64, &qs) == 0, "fuzz queries");
    for (tag = 100; tag <= 201; tag += (tag == 101 ? 99 : 1)) {
      size_t len = 0;
      unsigned char *img;
      uint32_t trial, loaded = 0;
      snprintf(p, sizeof p, "%s/%s/k%u_d%u.%u.fmi", g, cs, k, d, tag);
      img = slurp(p, &len);
      CHECK(img != NULL, "fuzz image %u", tag);
      if (!img) continue;
      for (trial = 0; trial < 600; trial++) {
        uint32_t h[6 + 2 * KFMI_MAX_STEPS], word, val, steps = ((uint32_t *) img)[1];
        unsigned char *b = (unsigned char *) malloc(len);
        uint64_t blen = len, need;
        void *x = NULL, *y = NULL, *z = NULL, *rs = NULL;
        memcpy(b, img, len);
        memcpy(h, img, 4 * (6 + 2 * steps));
        lcg = lcg * 1664525u + 1013904223u;
        word = (lcg >> 8) % 5;   /* bwtsize, nentries, a '$' row, a '$' code, two fields */
        lcg = lcg * 1664525u + 1013904223u;
        switch ((lcg >> 4) % 6) {
          case 0: val = 0; break;
          case 1: val = 1; break;
          case 2: val = 0xFFFFFFFFu - (lcg >> 28); break;
          case 3: val = h[2] + (lcg >> 20) % (3 * d) - (3 * d) / 2; break;
          case 4: val = h[4] + (lcg >> 24) % 5 - 2; break;
          default: val = lcg >> 7; break;
        }
        if (word == 0) h[2] = val;
        else if (word == 1) h[4] = val;
        else if (word == 2) h[6 + (lcg >> 3) % steps] = val;
        else if (word == 3) h[6 + steps + (lcg >> 3) % steps] = val % 7u;
        else { h[2] = val; h[6 + (lcg >> 3) % steps] = val - (lcg >> 29); }
        memcpy(b, h, 4 * (6 + 2 * steps));
        need = 4ull * (6 + 2 * steps) + 4ull * kfmi_entry_words(tag, steps, d) * h[4];
        if (need < blen) blen = need;   /* a smaller nentries: the file ends there */
        if (kfmi_index_from_image(b, blen, &x) == 0) {
          loaded++;
          if (initResults(num < 64 ? num : 64, &rs) == 0) {
            (void) kfmi_search_cpu(x, qs, rs, 2);
            freeResults(&rs);
          }
          if (tag == 100) {
            if (kfmi_transform_interleave(x, &y) == 0) freeIndex(&y);
            if (kfmi_transform_ac(x, &y, &z) == 0) { freeIndex(&y); freeIndex(&z); }
          } else if (tag >= 200 && kfmi_transform_plain(x, &y) == 0) {
            freeIndex(&y);
          }
          freeIndex(&x);
        }
        free(b);
      }
      CHECK(loaded > 0, "fuzz: some damaged %u headers still load", tag);
      free(img);
    }
    freeQueries(&qs);
  }

  /* 9b. damaged bodies: every tag's image with 1-16 entry words (counters or
   *     bit planes) replaced by 0, 0xFFFFFFFF, 2^31 or a random word -- every
   *     such file loads, and the host search and the transforms stay inside
   *     their buffers whatever the counters say (cs_lf's padding entry) */
  {
    void *qs = NULL;
    uint32_t lcg = 4242u + k * 13u + d;
    snprintf(q, sizeof q, "%s/%s/q%u.qry", g, cs, m);
    CHECK(loadQueries(q, m, num < 64 ? num : 64, &qs) == 0, "body fuzz queries");
    for (tag = 100; tag <= 201; tag += (tag == 101 ? 99 : 1)) {
      size_t len = 0;
      unsigned char *img;
      uint32_t trial, loaded = 0;
      snprintf(p, sizeof p, "%s/%s/k%u_d%u.%u.fmi", g, cs, k, d, tag);
      img = slurp(p, &len);
      CHECK(img != NULL, "body fuzz image %u", tag);
      if (!img) continue;
      for (trial = 0; trial < 300; trial++) {
        const uint32_t steps = ((uint32_t *) img)[1];
        const uint64_t hw = 6 + 2 * steps, words = len / 4;
        unsigned char *b = (unsigned char *) malloc(len);
        uint32_t *w = (uint32_t *) b, nw, j;
        void *x = NULL, *y = NULL, *z = NULL, *rs = NULL;
        memcpy(b, img, len);
        lcg = lcg * 1664525u + 1013904223u;
        nw = 1 + (lcg >> 12) % 16u;
        for (j = 0; j < nw && words > hw; j++) {
          uint32_t val;
          lcg = lcg * 1664525u + 1013904223u;
          switch ((lcg >> 4) % 4) {
            case 0: val = 0; break;
            case 1: val = 0xFFFFFFFFu; break;
            case 2: val = 0x80000000u; break;
            default: val = lcg * 2654435761u; break;
          }
          lcg = lcg * 1664525u + 1013904223u;
          w[hw + (lcg >> 3) % (words - hw)] = val;
        }
        if (kfmi_index_from_image(b, len, &x) == 0) {
          loaded++;
          if (initResults(num < 64 ? num : 64, &rs) == 0) {
            (void) kfmi_search_cpu(x, qs, rs, 2);
            freeResults(&rs);
          }
          if (tag == 100) {
            if (kfmi_transform_interleave(x, &y) == 0) freeIndex(&y);
            if (kfmi_transform_ac(x, &y, &z) == 0) { freeIndex(&y); freeIndex(&z); }
          } else if (tag >= 200 && kfmi_transform_plain(x, &y) == 0) {
            freeIndex(&y);
          }
          freeIndex(&x);
        }
        free(b);
      }
      CHECK(loaded == 300, "body fuzz: every damaged %u body loads (%u)", tag, loaded);
      free(img);
    }
    freeQueries(&qs);
  }

  /* 10. damaged text files: random bytes drawn mostly from ">\n\rACGTN" (and
   *     any byte now and then), 0-5000 of them, through loadQueries, loadRef
   *     and loadResults with random sizes -- each either fails or returns a
   *     buffer of the size asked, never reading or writing outside */
  {
    uint32_t lcg = 777u + k + d, trial, okq = 0, okr = 0;
    static const char alpha[] = ">\n\r\nACGTNacgt 0123456789";
    snprintf(q, sizeof q, "%s/junk.txt", tmp);
    for (trial = 0; trial < 400; trial++) {
      uint32_t len, i, mq, nq, nr;
      FILE *fp = fopen(q, "wb");
      void *qs = NULL, *ref = NULL, *rs = NULL;
      lcg = lcg * 1664525u + 1013904223u;
      len = (lcg >> 8) % 5001u;
      for (i = 0; i < len; i++) {
        lcg = lcg * 1664525u + 1013904223u;
        fputc((lcg >> 24) < 8 ? (int) (lcg >> 16) & 0xff : alpha[(lcg >> 16) % (sizeof alpha - 1)], fp);
      }
      fclose(fp);
      lcg = lcg * 1664525u + 1013904223u;
      mq = 1 + (lcg >> 8) % 40u;
      nq = 1 + (lcg >> 16) % 50u;
      nr = 1 + (lcg >> 4) % 3000u;
      if (loadQueries(q, mq, nq, &qs) == 0) { okq++; freeQueries(&qs); }
      if (loadRef(q, nr, &ref) == 0) { okr++; freeReference(&ref, NULL); }
      if (loadResults(q, &rs) == 0) freeResults(&rs);
    }
    CHECK(trial == 400, "junk files");
    (void) okq; (void) okr;
  }

  freeIndex(&idx); freeIndex(&t101); freeIndex(&t200); freeIndex(&t201);
  printf("%s %d checks, %d failures\n", failures ? "FAILED" : "OK", checks, failures);
  return failures ? 1 : 0;
}
