/*
 * common.c -- host I/O and helpers of the k-step FM-index engine.
 *
 * Behavioural restatement of /root/reference/common/common.c (queries,
 * results, reference text, error strings, timer) with 64-bit sizes (B7),
 * no fixed line buffers, and no 32-query interleave: the device packs
 * queries itself (csrc/hip/kfmi_search.hip, pack kernel), so queries stay in
 * the plain layout `q*size` (common.c:163-173 without -DINTERLEAVING_QUERIES).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>
#include "../kfmi_internal.h"

/* common.c:28-33 (monotonic instead of CLOCK_REALTIME) */
double sampleTime(void)
{
  struct timespec tv;
  clock_gettime(CLOCK_MONOTONIC, &tv);
  return (double) tv.tv_sec + (double) tv.tv_nsec / 1e9;
}

/* genFMindex.c:71-84: A/a=0 C/c=1 G/g=2 T/t=3, N->2, by ASCII bits 1..2 */
uint32_t base2index(uint32_t base)
{
  uint32_t f2 = base & 0x02u, b1 = base & 0x04u;
  uint32_t b0 = b1 ? (f2 ^ 0x02u) : f2;
  return (b1 | b0) >> 1;
}

/* ----------------------------------------------------------------------- */
/* reference text (common.c:42-130)                                        */
/* ----------------------------------------------------------------------- */

/* Reads the first `refsize` sequence characters of a (multi-)FASTA file; the
 * first line must be a '>' header (common.c:59-62); later lines are
 * concatenated with their line terminator removed. */
static int32_t read_ref(const char *fn, uint64_t refsize, char **out, uint64_t *got)
{
  FILE *fp = fopen(fn, "rb");
  char *ref, *line = NULL;
  size_t cap = 0;
  ssize_t len;
  uint64_t pos = 0;
  if (!fp) return KFMI_E_OPENING_REFERENCE_FILE;
  ref = (char *) malloc(refsize ? refsize : 1);
  if (!ref) { fclose(fp); return KFMI_E_ALLOCATING_REFERENCE; }
  len = getline(&line, &cap, fp);
  if (len <= 0) { free(ref); free(line); fclose(fp); return KFMI_E_READING_REFERENCE_FILE; }
  if (line[0] != '>') { free(ref); free(line); fclose(fp); return KFMI_E_READING_MFASTA_FILE; }
  while (pos < refsize && (len = getline(&line, &cap, fp)) > 0) {
    while (len > 0 && (line[len - 1] == '\n' || line[len - 1] == '\r')) len--;
    if (len > 0 && line[0] == '>') continue;
    if ((uint64_t) len > refsize - pos) len = (ssize_t) (refsize - pos);
    memcpy(ref + pos, line, (size_t) len);
    pos += (uint64_t) len;
  }
  free(line);
  fclose(fp);
  *out = ref;
  *got = pos;
  return KFMI_SUCCESS;
}

/* The reference's readRef exactly (common.c:42-76), for KFMI_ALPHABET=ref: the
 * file read in fgets pieces of at most 255 bytes; after the first line every
 * piece contributes strlen - 1 bytes -- its newline dropped, or, for a line of
 * 255 bytes or more, its last data byte -- header lines included. */
static int32_t read_ref_exact(const char *fn, uint64_t refsize, char **out, uint64_t *got)
{
  FILE *fp = fopen(fn, "rb");
  char piece[256], *ref;
  uint64_t pos = 0;
  if (!fp) return KFMI_E_OPENING_REFERENCE_FILE;
  ref = (char *) malloc(refsize ? refsize : 1);
  if (!ref) { fclose(fp); return KFMI_E_ALLOCATING_REFERENCE; }
  if (!fgets(piece, sizeof(piece), fp)) { free(ref); fclose(fp); return KFMI_E_READING_REFERENCE_FILE; }
  if (piece[0] != '>') { free(ref); fclose(fp); return KFMI_E_READING_MFASTA_FILE; }
  while (pos < refsize && fgets(piece, sizeof(piece), fp)) {
    uint64_t l = strlen(piece);
    if (l) l--;
    if (l > refsize - pos) l = refsize - pos;
    memcpy(ref + pos, piece, l);
    pos += l;
  }
  fclose(fp);
  *out = ref;
  *got = pos;
  return KFMI_SUCCESS;
}

int32_t loadRef(const char *fn, uint32_t refsize, void **reference)
{
  kfmi_ref_t *ref = (kfmi_ref_t *) calloc(1, sizeof(*ref));
  uint64_t got = 0;
  int32_t err;
  if (!ref) return KFMI_E_ALLOCATING_REFERENCE;
  err = kfmi_alphabet_mode() == KFMI_ALPHA_REF ? read_ref_exact(fn, refsize, &ref->h_reference, &got)
                                               : read_ref(fn, refsize, &ref->h_reference, &got);
  if (err) { free(ref); return err; }
  if (got != refsize) { free(ref->h_reference); free(ref); return KFMI_E_READING_REFERENCE_FILE; }
  ref->size = got;
  *reference = ref;
  return KFMI_SUCCESS;
}

/* common.c:88-130: "<fn>.<size>.fa", header "> <size>", 70-column lines */
int32_t saveRef(const char *fn, void *reference)
{
  kfmi_ref_t *ref = (kfmi_ref_t *) reference;
  char name[1024];
  FILE *fp;
  uint64_t i;
  snprintf(name, sizeof(name), "%s.%llu.fa", fn, (unsigned long long) ref->size);
  fp = fopen(name, "wb");
  if (!fp) return KFMI_E_OPENING_REFERENCE_FILE;
  fprintf(fp, "> %llu", (unsigned long long) ref->size);
  for (i = 0; i < ref->size; i += 70) {
    uint64_t l = ref->size - i < 70 ? ref->size - i : 70;
    fputc('\n', fp);
    fwrite(ref->h_reference + i, 1, l, fp);
  }
  fputc('\n', fp);
  fclose(fp);
  return KFMI_SUCCESS;
}

/* common.c:313-322 frees the text and keeps the handle (its ref_t leaks); here
 * both are freed and the handle cleared */
int32_t freeReference(void **reference, void **index)
{
  kfmi_ref_t *ref = reference ? (kfmi_ref_t *) *reference : NULL;
  (void) index;
  if (!ref) return KFMI_SUCCESS;
  free(ref->h_reference);
  free(ref);
  *reference = NULL;
  return KFMI_SUCCESS;
}

/* ----------------------------------------------------------------------- */
/* queries (common.c:132-199)                                              */
/* ----------------------------------------------------------------------- */

/* Multi-FASTA reads: '>' lines are skipped, every other line is one read of
 * exactly `sizequery` characters (common.c:167-173 copies strlen-1 bytes per
 * line; a line of another length is an error here instead of silently
 * shifting every following read).  Reads beyond `numqueries` are ignored;
 * fewer reads than `numqueries` is an error.
 *
 * The reference reads line by line with fgets on one thread into 32-bit
 * offsets (common.c:132-199, :163, :167).  Here a regular file is mapped and
 * parsed by kfmi_host_threads() threads (KFMI_HOST_THREADS) in two passes
 * over contiguous byte ranges: count the read lines of each range (and note the
 * first malformed one), then -- after a prefix sum gives every range its first
 * read number -- copy each read to q * size.  Same semantics as the
 * line-by-line loop (load_queries_stream, kept for pipes and KFMI_LOAD_MMAP=0). */

static int32_t load_queries_stream(FILE *fp, kfmi_qrys_t *q, uint64_t numqueries, uint32_t sizequery)
{
  char *line = NULL;
  size_t cap = 0;
  ssize_t len;
  uint64_t i = 0;
  while (i < numqueries && (len = getline(&line, &cap, fp)) > 0) {
    if (line[0] == '>') continue;
    while (len > 0 && (line[len - 1] == '\n' || line[len - 1] == '\r')) len--;
    if ((uint64_t) len != sizequery) { free(line); return KFMI_E_READING_MFASTA_FILE; }
    memcpy(q->h_queries + i * sizequery, line, sizequery);
    i++;
  }
  free(line);
  return i == numqueries ? KFMI_SUCCESS : KFMI_E_READING_MFASTA_FILE;
}

typedef struct {
  const char *base;
  uint64_t size, b, e;      /* lines whose first byte lies in [b, e) */
  uint32_t m;
  int pass;                 /* 1: count, 2: copy */
  uint64_t nseq;            /* pass 1: read lines in the range */
  uint64_t first_bad;       /* pass 1: range ordinal of the first malformed read line, or UINT64_MAX */
  uint64_t first;           /* pass 2: global number of the range's first read */
  uint64_t limit;           /* numqueries */
  char *out;
} lq_range;

/* first line start at or after x */
static uint64_t line_start(const char *base, uint64_t size, uint64_t x)
{
  const char *nl;
  if (x == 0) return 0;
  if (x >= size) return size;
  nl = (const char *) memchr(base + x - 1, '\n', size - (x - 1));
  return nl ? (uint64_t) (nl - base) + 1 : size;
}

static void *lq_worker(void *arg)
{
  lq_range *r = (lq_range *) arg;
  const char *base = r->base;
  uint64_t pos = line_start(base, r->size, r->b), end = line_start(base, r->size, r->e), k = 0;
  r->nseq = 0;
  if (r->pass == 1) r->first_bad = UINT64_MAX;
  while (pos < end) {
    const char *ls = base + pos;
    const char *nl = (const char *) memchr(ls, '\n', r->size - pos);
    uint64_t len = nl ? (uint64_t) (nl - ls) : r->size - pos;
    const uint64_t next = pos + len + (nl ? 1 : 0);
    if (ls[0] != '>') {
      while (len > 0 && ls[len - 1] == '\r') len--;
      if (r->pass == 1) {
        if (len != r->m && r->first_bad == UINT64_MAX) r->first_bad = k;
      } else {
        const uint64_t g = r->first + k;
        if (g >= r->limit) break;
        memcpy(r->out + g * r->m, ls, r->m);
      }
      k++;
    }
    pos = next;
  }
  r->nseq = k;
  return NULL;
}

/* Host threads of the parallel paths (this loader, the streamed search's
 * packers and staging copies, the device loader's reads): KFMI_HOST_THREADS,
 * else the CPUs this process may use -- its affinity mask capped by the cgroup
 * CPU quota (the GPU boxes show 256 cores but grant 16) -- divided among the
 * ranks torchrun started on this host (LOCAL_WORLD_SIZE), 2 to 16.  Eight
 * ranks of 16 threads each on a 16-CPU quota would oversubscribe it 8x. */
int32_t kfmi_process_cpus(void)
{
  long cpus = sysconf(_SC_NPROCESSORS_ONLN);
  cpu_set_t set;
  FILE *fp;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) == 0 && CPU_COUNT(&set) > 0 && CPU_COUNT(&set) < cpus)
    cpus = CPU_COUNT(&set);
  if ((fp = fopen("/sys/fs/cgroup/cpu.max", "r")) != NULL) {
    char q[32] = {0};
    long long per = 0;
    if (fscanf(fp, "%31s %lld", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0) {
      long long quota = (atoll(q) + per - 1) / per;
      if (quota > 0 && quota < cpus) cpus = (long) quota;
    }
    fclose(fp);
  }
  return (int32_t) (cpus < 1 ? 1 : cpus);
}

/* Big-buffer registry: the mappings kfmi_big_alloc made (pointer, length), so
 * kfmi_big_free can tell them from calloc'd buffers.  Index images, query and
 * result buffers use it: on 2 MB pages a 1 GB read buffer takes 512 first-touch
 * faults instead of 262,144 (loadQueries 0.14 -> 0.085 s for 0.9 GB here). */
static pthread_mutex_t big_mu = PTHREAD_MUTEX_INITIALIZER;
static struct { void *p; uint64_t len; } *big_tab;
static size_t big_n, big_cap;

#define KFMI_HUGE (2ull << 20)

void *kfmi_big_alloc(uint64_t bytes)
{
  uint64_t len;
  uint8_t *raw, *p;
  const char *e = getenv("KFMI_HUGEPAGES");   /* 0: plain calloc (measurements) */
  if (bytes < (64ull << 20) || (e && !atoi(e))) return calloc(1, bytes ? bytes : 1);
  len = (bytes + KFMI_HUGE - 1) & ~(KFMI_HUGE - 1);
  raw = (uint8_t *) mmap(NULL, len + KFMI_HUGE, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (raw == MAP_FAILED) return calloc(1, bytes);
  p = (uint8_t *) (((uintptr_t) raw + KFMI_HUGE - 1) & ~(uintptr_t) (KFMI_HUGE - 1));
  if (p > raw) munmap(raw, (size_t) (p - raw));
  if (raw + len + KFMI_HUGE > p + len) munmap(p + len, (size_t) (raw + len + KFMI_HUGE - (p + len)));
  (void) madvise(p, len, MADV_HUGEPAGE);   /* a hint: without THP the pages stay 4 KB */
  pthread_mutex_lock(&big_mu);
  if (big_n == big_cap) {
    size_t nc = big_cap ? 2 * big_cap : 16;
    void *t = realloc(big_tab, nc * sizeof(*big_tab));
    if (!t) {
      pthread_mutex_unlock(&big_mu);
      munmap(p, len);
      return calloc(1, bytes);
    }
    big_tab = t;
    big_cap = nc;
  }
  big_tab[big_n].p = p;
  big_tab[big_n].len = len;
  ++big_n;
  pthread_mutex_unlock(&big_mu);
  return p;
}

void kfmi_big_free(void *p)
{
  size_t i;
  if (!p) return;
  pthread_mutex_lock(&big_mu);
  for (i = 0; i < big_n; ++i)
    if (big_tab[i].p == p) {
      const uint64_t len = big_tab[i].len;
      big_tab[i] = big_tab[--big_n];
      pthread_mutex_unlock(&big_mu);
      munmap(p, len);
      return;
    }
  pthread_mutex_unlock(&big_mu);
  free(p);
}

int32_t kfmi_host_threads(void)
{
  const char *e = getenv("KFMI_HOST_THREADS");
  long cpus, ranks = 1;
  if (e) {
    int v = atoi(e);
    return v < 1 ? 1 : (v > 64 ? 64 : v);
  }
  cpus = kfmi_process_cpus();
  if ((e = getenv("LOCAL_WORLD_SIZE")) != NULL && atoi(e) > 0) ranks = atoi(e);
  cpus /= ranks;
  return (int32_t) (cpus < 2 ? 2 : (cpus > 16 ? 16 : cpus));
}

static int host_threads(void) { return kfmi_host_threads(); }

static int32_t load_queries_mapped(const char *base, uint64_t size, kfmi_qrys_t *q, uint64_t numqueries,
                                   uint32_t sizequery)
{
  int nt = host_threads(), t;
  lq_range r[64];
  pthread_t th[64];
  uint64_t acc = 0;
  if (size < (4u << 20)) nt = 1;
  for (t = 0; t < nt; t++) {
    r[t].base = base;
    r[t].size = size;
    r[t].b = size * (uint64_t) t / (uint64_t) nt;
    r[t].e = size * (uint64_t) (t + 1) / (uint64_t) nt;
    r[t].m = sizequery;
    r[t].limit = numqueries;
    r[t].out = q->h_queries;
  }
  for (int pass = 1; pass <= 2; pass++) {
    for (t = 0; t < nt; t++) r[t].pass = pass;
    for (t = 1; t < nt; t++)
      if (pthread_create(&th[t], NULL, lq_worker, &r[t])) {
        for (int u = 1; u < t; u++) pthread_join(th[u], NULL);
        return KFMI_E_ALLOCATING_MFASTA;
      }
    lq_worker(&r[0]);
    for (t = 1; t < nt; t++) pthread_join(th[t], NULL);
    if (pass == 1) {
      /* a malformed read line before the numqueries-th read is what the line
       * loop would stop at; too few reads is an error as well */
      for (t = 0; t < nt; t++) {
        if (r[t].first_bad != UINT64_MAX && acc + r[t].first_bad < numqueries) return KFMI_E_READING_MFASTA_FILE;
        r[t].first = acc;
        acc += r[t].nseq;
      }
      if (acc < numqueries) return KFMI_E_READING_MFASTA_FILE;
    }
  }
  return KFMI_SUCCESS;
}

int32_t loadQueries(const char *fn, uint32_t sizequery, uint32_t numqueries, void **queries)
{
  kfmi_qrys_t *q;
  FILE *fp;
  struct stat sb;
  const char *mm = getenv("KFMI_LOAD_MMAP");
  int32_t err = KFMI_E_READING_MFASTA_FILE;
  int done = 0;
  if (sizequery == 0) return KFMI_E_BAD_ARGUMENT;
  fp = fopen(fn, "rb");
  if (!fp) return KFMI_E_OPENING_MFASTA_FILE;
  q = (kfmi_qrys_t *) calloc(1, sizeof(*q));
  if (!q) { fclose(fp); return KFMI_E_ALLOCATING_MFASTA; }
  q->num = numqueries;
  q->size = sizequery;
  q->h_queries = (char *) kfmi_big_alloc((uint64_t) numqueries * sizequery + 1);
  if (!q->h_queries) { free(q); fclose(fp); return KFMI_E_ALLOCATING_MFASTA; }
  if ((!mm || atoi(mm)) && fstat(fileno(fp), &sb) == 0 && S_ISREG(sb.st_mode) && sb.st_size > 0) {
    void *base = mmap(NULL, (size_t) sb.st_size, PROT_READ, MAP_PRIVATE, fileno(fp), 0);
    if (base != MAP_FAILED) {
      (void) madvise(base, (size_t) sb.st_size, MADV_WILLNEED);
      err = load_queries_mapped((const char *) base, (uint64_t) sb.st_size, q, numqueries, sizequery);
      munmap(base, (size_t) sb.st_size);
      done = 1;
    }
  }
  if (!done) err = load_queries_stream(fp, q, numqueries, sizequery);
  fclose(fp);
  if (err) { kfmi_big_free(q->h_queries); free(q); return err; }
  *queries = q;
  return KFMI_SUCCESS;
}

int32_t kfmi_queries_from_buffer(const char *ascii, uint64_t num, uint32_t size, void **queries)
{
  kfmi_qrys_t *q;
  if (size == 0 || (!ascii && num)) return KFMI_E_BAD_ARGUMENT;
  q = (kfmi_qrys_t *) calloc(1, sizeof(*q));
  if (!q) return KFMI_E_ALLOCATING_MFASTA;
  q->num = num;
  q->size = size;
  q->h_queries = (char *) kfmi_big_alloc(num * size + 1);
  if (!q->h_queries) { free(q); return KFMI_E_ALLOCATING_MFASTA; }
  if (num) memcpy(q->h_queries, ascii, num * size);
  *queries = q;
  return KFMI_SUCCESS;
}

/* common.c:262-270 (also releases the handle) */
int32_t freeQueries(void **queries)
{
  kfmi_qrys_t *q = queries ? (kfmi_qrys_t *) *queries : NULL;
  if (!q) return KFMI_SUCCESS;
  if (q->dev || q->grp) freeQueriesGPU(queries);
  kfmi_big_free(q->h_queries);
  free(q);
  *queries = NULL;
  return KFMI_SUCCESS;
}

/* ----------------------------------------------------------------------- */
/* results (common.c:201-260, 324-341)                                     */
/* ----------------------------------------------------------------------- */

int32_t kfmi_results_alloc(uint64_t num, void **results)
{
  kfmi_res_t *r = (kfmi_res_t *) calloc(1, sizeof(*r));
  if (!r) return KFMI_E_ALLOCATING_RESULTS;
  r->num = num;
  r->h_results = (uint32_t *) kfmi_big_alloc((2 * (uint64_t) num + 1) * sizeof(uint32_t));
  if (!r->h_results) { free(r); return KFMI_E_ALLOCATING_RESULTS; }
  *results = r;
  return KFMI_SUCCESS;
}

int32_t initResults(uint32_t numresults, void **results)
{
  return kfmi_results_alloc(numresults, results);
}

uint32_t *kfmi_results_host(void *results) { return results ? ((kfmi_res_t *) results)->h_results : NULL; }
uint64_t  kfmi_results_num(void *results)  { return results ? ((kfmi_res_t *) results)->num : 0; }

int32_t freeResults(void **results)
{
  kfmi_res_t *r = results ? (kfmi_res_t *) *results : NULL;
  if (!r) return KFMI_SUCCESS;
  if (r->d_results || r->grp) freeResultsGPU(results);
  kfmi_big_free(r->h_results);
  free(r);
  *results = NULL;
  return KFMI_SUCCESS;
}

static char *put_u32(char *p, uint32_t v)
{
  char tmp[12];
  int n = 0;
  do { tmp[n++] = (char) ('0' + v % 10); v /= 10; } while (v);
  while (n) *p++ = tmp[--n];
  return p;
}

static int32_t write_results64(const char *fn, const uint32_t *res, uint64_t num)
{
  FILE *fp = fopen(fn, "wb");
  char *buf, *p;
  const size_t chunk = 1u << 20;
  uint64_t i;
  if (!fp) return KFMI_E_OPENING_RESULTS_FILE;
  buf = (char *) malloc(chunk * 24 + 32);
  if (!buf) { fclose(fp); return KFMI_E_ALLOCATING_RESULTS; }
  p = buf;
  p += sprintf(p, "%llu\n", (unsigned long long) num);
  for (i = 0; i < num; i++) {
    p = put_u32(p, res[2 * i]); *p++ = ' ';
    p = put_u32(p, res[2 * i + 1]); *p++ = '\n';
    if ((size_t) (p - buf) >= chunk * 22) { fwrite(buf, 1, (size_t) (p - buf), fp); p = buf; }
  }
  fwrite(buf, 1, (size_t) (p - buf), fp);
  free(buf);
  fclose(fp);
  return KFMI_SUCCESS;
}

/* common.c:201-220: "N\n" then "L R\n" per query */
int32_t writeResults(const char *fn, uint32_t *results, uint32_t numqueries)
{
  return write_results64(fn, results, numqueries);
}

/* common.c:222-246 */
int32_t loadResults(const char *fn, void **results)
{
  FILE *fp = fopen(fn, "rb");
  unsigned long long n;
  uint64_t i;
  kfmi_res_t *r;
  int32_t err;
  if (!fp) return KFMI_E_OPENING_RESULTS_FILE;
  if (fscanf(fp, "%llu", &n) != 1) { fclose(fp); return KFMI_E_READING_RESULTS_FILE; }
  err = kfmi_results_alloc(n, (void **) &r);
  if (err) { fclose(fp); return err; }
  for (i = 0; i < n; i++) {
    if (fscanf(fp, "%u %u", &r->h_results[2 * i], &r->h_results[2 * i + 1]) != 2) {
      fclose(fp); freeResults((void **) &r); return KFMI_E_READING_RESULTS_FILE;
    }
  }
  fclose(fp);
  *results = r;
  return KFMI_SUCCESS;
}

/* common.c:324-341: "<fn>.res.gpu" as the reference's GPU build names it, or
 * "<fn>.res.cpu" (its CPU build) when searchIndexCPU wrote these results last */
int32_t saveResults(const char *fn, void *results, void *index)
{
  kfmi_res_t *r = (kfmi_res_t *) results;
  char name[1024];
  (void) index;
  if (!r) return KFMI_E_BAD_ARGUMENT;
  snprintf(name, sizeof(name), "%s.res.%s", fn, r->origin == KFMI_RES_FROM_CPU ? "cpu" : "gpu");
  return write_results64(name, r->h_results, r->num);
}

/* common.c:282-310 */
char *errorCommon(int32_t e)
{
  switch (e) {
    case KFMI_SUCCESS:                  return "No error";
    case KFMI_E_OPENING_INDEX_FILE:     return "Cannot open index file";
    case KFMI_E_ALLOCATING_BWT:         return "Cannot allocate memory for bwt";
    case KFMI_E_ALLOCATING_FMI:         return "Cannot allocate memory for counters";
    case KFMI_E_READING_BWT:            return "Error reading index bwt";
    case KFMI_E_READING_FMI:            return "Error reading index counters";
    case KFMI_E_SAVING_INDEX_FILE:      return "Cannot open index file for save";
    case KFMI_E_SAVING_BWT_FILE:        return "Cannot open bwt file for save";
    case KFMI_E_BUILDING_BWT:           return "Error building bwt";
    case KFMI_E_BUILDING_FMI:           return "Error building FMI, cannot allocate memory for bwt";
    case KFMI_E_OPENING_REFERENCE_FILE: return "Cannot open reference file";
    case KFMI_E_ALLOCATING_REFERENCE:   return "Cannot allocate reference";
    case KFMI_E_READING_MFASTA_FILE:    return "Reference file isn't MFASTA format";
    case KFMI_E_READING_REFERENCE_FILE: return "Error reading reference file";
    case KFMI_E_OPENING_MFASTA_FILE:    return "Cannot open MFASTS queries file";
    case KFMI_E_ALLOCATING_MFASTA:      return "Cannot allocate MFASTA queries";
    case KFMI_E_ALLOCATING_RESULTS:     return "Cannot allocate results";
    case KFMI_E_OPENING_RESULTS_FILE:   return "Cannot open results file for load intervals";
    case KFMI_E_READING_RESULTS_FILE:   return "Error reading results";
    case KFMI_E_NOT_IMPLEMENTED:        return "Not implemented";
    case KFMI_E_NO_DEVICE:              return "No usable HIP device (HIP runtime error)";
    case KFMI_E_DEVICE_ALLOC:           return "Cannot allocate device memory";
    case KFMI_E_KERNEL:                 return "HIP kernel launch or execution failed";
    case KFMI_E_BAD_ARGUMENT:           return "Unsupported argument (K, d, query size or backend)";
    case KFMI_E_NOT_ON_DEVICE:          return "Index/queries/results not transferred to the device";
    case KFMI_INDEX_VER_BASELINE:       return "Error in the index type, use gfmiBaseLine_*Bases_*Step to generate an index_name.fmi type";
    case KFMI_INDEX_VER_INTERLEAVE:     return "Error in the index type, use tfmiBMP_*Bases_*Step to generate an index_name.fmi.interleaving type";
    case KFMI_INDEX_VER_BASELINE_AC:    return "Error in the index type, use tfmiAC_*Bases_*Step to generate an index_name.fmi.ac type";
    case KFMI_INDEX_VER_INTERLEAVE_AC:  return "Error in the index type, use tfmiAC_*Bases_*Step to generate an index_name.fmi.interleaving.ac type";
    default:                            return "Unknown error";
  }
}
