/*
 * oracle/fmi_oracle.c -- TEST INFRASTRUCTURE, NOT PRODUCT CODE.
 *
 * A plain-C restatement of the reference CPU backward search
 *   /root/reference/src/fmIndexCPUBaseline.c:157-292            (plain counters, tags 100/101)
 *   /root/reference/src/fmIndexCPUBaseline-AltCounters.c:145-310 (alternate counters, tags 200/201)
 * used only as the parity checker in tests/, in __graft_entry__.smoke() and as
 * bench.py's cpu_baseline ("port").  The product (k-step_fm-index_amd/) never
 * links or calls this file.
 *
 * Parity is pinned (tests/test_oracle.py) against result files produced by the
 * reference binaries themselves (oracle/_ref, built by oracle/Makefile from the
 * reference sources) and committed under tests/golden/.
 *
 * Differences from the reference that do not change any result:
 *   - one binary handles every (K, d) and every index tag (the reference
 *     fixes K/d/tag at compile time, fmIndexCPUBaseline.c:30-41);
 *   - tags 101/201 are read with their own bit-plane order
 *     (transformIndexBitmaps.c:278-279), giving the result the reference
 *     oracle gives on the equivalent tag 100/200 file;
 *   - 64-bit query offsets (the reference uses u32, B7);
 *   - shift-by-32 UB of `mask << (32-shift)` (fmIndexCPUBaseline.c:235) avoided;
 *   - the _mm_prefetch hints (:205-211) are omitted;
 *   - m % K != 0 is rejected (the reference reads query[-1], B6).
 * Optional statistic: the number of distinct d-blocks the search touches
 * (1 per step when L/d == R/d, else 2) -- the dedup-aware algorithmic byte
 * count of SURVEY.md 8(d).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

#define OR_OK            0
#define OR_E_HEADER      5   /* E_READING_FMI, common.h:41 */
#define OR_E_BADARG      99  /* E_NOT_IMPLEMENTED */
#define OR_E_UNDEFINED   98  /* a step reads past the index: the reference's result is undefined */

typedef struct {
  uint32_t tag, steps, bwtsize, ncounters, nentries, chunk;
  uint32_t dpos[4], dbase[4], dblk[4];
  uint32_t nb;          /* 32-bit words per bit-plane row = d/32 */
  uint32_t nc;          /* full counter count 4^K */
  uint32_t ew;          /* u32 words per entry */
  uint32_t cnt_off;     /* first counter word inside an entry */
  uint32_t bmp_off;     /* first bitmap word inside an entry */
  int      ac;          /* alternate counters (tags 200/201) */
  int      inter;       /* interleaved bit planes (tags 101/201) */
  const uint32_t *e;    /* entries */
} ofmi_t;

/* Header layout: genFMindex.c:167-178 (tag, steps, bwtsize, ncounters,
 * nentries, chunk, dollarPositionBWT[steps], dollarBaseBWT[steps]). */
static int parse(const void *image, uint64_t bytes, ofmi_t *f)
{
  const uint32_t *h = (const uint32_t *) image;
  uint32_t s;
  if (bytes < 24) return OR_E_HEADER;
  f->tag = h[0]; f->steps = h[1]; f->bwtsize = h[2];
  f->ncounters = h[3]; f->nentries = h[4]; f->chunk = h[5];
  if (f->steps < 1 || f->steps > 4 || f->chunk == 0 || (f->chunk % 32) != 0) return OR_E_HEADER;
  if (bytes < 24 + 8ull * f->steps) return OR_E_HEADER;
  for (s = 0; s < f->steps; s++) {
    f->dpos[s]  = h[6 + s];
    f->dbase[s] = h[6 + f->steps + s];
    f->dblk[s]  = f->dpos[s] / f->chunk;     /* modposdollarBWT, fmIndexCPUBaseline.c:119-122 */
  }
  f->nb = f->chunk / 32;
  f->nc = 1u << (2 * f->steps);
  switch (f->tag) {
    case 100: f->ac = 0; f->inter = 0; break;
    case 101: f->ac = 0; f->inter = 1; break;
    case 200: f->ac = 1; f->inter = 0; break;
    case 201: f->ac = 1; f->inter = 1; break;
    default: return OR_E_HEADER;
  }
  if (f->ncounters != (f->ac ? f->nc / 2 : f->nc)) return OR_E_HEADER;
  f->ew = 2 * f->nb * f->steps + f->ncounters;
  /* tag 100/101: [bitmap | cnt] (genFMindex.c:42-45); tag 200/201: [cnt | bitmap]
   * (fmIndexCPUBaseline-AltCounters.c:49-52). */
  f->bmp_off = f->ac ? f->ncounters : 0;
  f->cnt_off = f->ac ? 0 : 2 * f->nb * f->steps;
  if (bytes < 24 + 8ull * f->steps + 4ull * f->ew * f->nentries) return OR_E_HEADER;
  f->e = h + 6 + 2 * f->steps;
  return OR_OK;
}

/* Bit plane (step s, code bit t, word w) of an entry.
 * tag 100/200: s*2NB + t*NB + w   (genFMindex.c:436, bwt2bin)
 * tag 101/201: w*2K  + 2s + t     (transformIndexBitmaps.c:278-279)          */
static inline uint32_t plane(const ofmi_t *f, const uint32_t *ent, uint32_t s, uint32_t t, uint32_t w)
{
  uint32_t i = f->inter ? (w * 2 * f->steps + 2 * s + t) : (s * 2 * f->nb + t * f->nb + w);
  return ent[f->bmp_off + i];
}

/* masked popcount of the rows whose K-mer code equals `code`, over the first
 * `shift` rows of the block (inverted mask when `inv`), fmIndexCPUBaseline.c:231-250
 * and -AltCounters.c:232-252. */
static inline int32_t count_block(const ofmi_t *f, const uint32_t *ent, uint32_t code,
                                  int32_t shift, int inv)
{
  int32_t cnt = 0;
  uint32_t n, s;
  for (n = 0; n < f->nb; n++) {
    uint32_t m;
    if (shift >= 32) m = 0xFFFFFFFFu;
    else if (shift > 0) m = 0xFFFFFFFFu << (32 - shift);
    else m = 0u;
    if (inv) m = ~m;
    for (s = 0; s < f->steps; s++) {
      uint32_t cs = (code >> (2 * s)) & 3u;
      uint32_t b0 = plane(f, ent, s, 0, n);
      uint32_t b1 = plane(f, ent, s, 1, n);
      m &= ((cs & 1u) ? b0 : ~b0) & ((cs & 2u) ? b1 : ~b1);
    }
    cnt += __builtin_popcount(m);
    shift -= 32;
  }
  return cnt;
}

/* base2index, fmIndexCPUBaseline.c:213-226 / genFMindex.c:71-84:
 * A/a=0 C/c=1 G/g=2 T/t=3, N->2, anything else by ASCII bits 1..2. */
static inline uint32_t code_of(uint8_t x)
{
  uint32_t b1 = x & 4u, f2 = x & 2u;
  uint32_t b0 = b1 ? (f2 ^ 2u) : f2;
  return (b1 | b0) >> 1;
}

/* One LF step of one interval end.  An entry past the image (the reference
 * reads past its file there) sets *oob and returns 0 instead. */
static inline uint32_t lf_step(const ofmi_t *f, uint32_t X, uint32_t code, int *oob)
{
  uint32_t d = f->chunk, b = X / d, s;
  int32_t shift = (int32_t) (X % d);
  if (b >= f->nentries || (f->ac && b + 1 >= f->nentries && (((b & 1u) != 0) == (code < f->nc / 2)))) {
    *oob = 1;
    return 0;
  }
  if (!f->ac) {
    /* fmIndexCPUBaseline.c:227-257 */
    const uint32_t *ent = f->e + (uint64_t) b * f->ew;
    int32_t bc = count_block(f, ent, code, shift, 0);
    for (s = 0; s < f->steps; s++)
      if (f->dblk[s] == b && code == f->dbase[s] && X > f->dpos[s]) bc--;
    return ent[f->cnt_off + code] + (uint32_t) bc;
  } else {
    /* fmIndexCPUBaseline-AltCounters.c:218-266 */
    uint32_t half = f->nc / 2;
    int e = ((b & 1u) && code < half) || (!(b & 1u) && code >= half);
    const uint32_t *ent = f->e + (uint64_t) b * f->ew;
    const uint32_t *cen = f->e + (uint64_t) (b + (uint32_t) e) * f->ew;
    uint32_t cnt = cen[code & (half - 1)];
    int32_t bc = count_block(f, ent, code, shift, e);
    for (s = 0; s < f->steps; s++) {
      if (f->dblk[s] == b && code == f->dbase[s]) {
        if (!e && X > f->dpos[s]) bc--;
        if (e && X <= f->dpos[s]) bc--;
      }
    }
    return e ? cnt - (uint32_t) bc : cnt + (uint32_t) bc;
  }
}

/* searchIndexCPU restated (fmIndexCPUBaseline.c:157-292):
 *  L=0, R=bwtsize; for j=m-1 downto 0 step K: c = sum_i code(P[j-i]) << 2i;
 *  L=LF(L,c); R=LF(R,c).  No early exit on an empty interval.
 *  results[2q]=L, results[2q+1]=R. */
int32_t oracle_search(const void *image, uint64_t image_bytes, const char *queries,
                      uint64_t num, uint32_t m, uint32_t *results, int32_t nthreads,
                      uint64_t *blocks_out)
{
  ofmi_t f;
  int32_t err = parse(image, image_bytes, &f);
  uint64_t blocks = 0;
  int oob = 0;
  if (err) return err;
  if (m == 0 || (m % f.steps) != 0) return OR_E_BADARG;
  if (nthreads > 0) omp_set_num_threads(nthreads);

  #pragma omp parallel for schedule(static) reduction(+:blocks) reduction(|:oob)
  for (int64_t q = 0; q < (int64_t) num; q++) {
    const uint8_t *p = (const uint8_t *) queries + (uint64_t) q * m;
    uint32_t L = 0, R = f.bwtsize;
    for (int64_t j = (int64_t) m - 1; j >= 0; j -= f.steps) {
      uint32_t code = 0, i;
      for (i = 0; i < f.steps; i++) code |= code_of(p[j - i]) << (2 * i);
      blocks += (L / f.chunk == R / f.chunk) ? 1 : 2;
      L = lf_step(&f, L, code, &oob);
      R = lf_step(&f, R, code, &oob);
    }
    results[2 * q] = L;
    results[2 * q + 1] = R;
  }
  if (blocks_out) *blocks_out = blocks;
  return oob ? OR_E_UNDEFINED : OR_OK;
}

/* Header fields for the Python side: out[0..5] = tag, steps, bwtsize,
 * ncounters, nentries, chunk; out[6..9] = dollarPositionBWT; out[10..13] =
 * dollarBaseBWT. */
int32_t oracle_header(const void *image, uint64_t image_bytes, uint32_t *out)
{
  ofmi_t f;
  int32_t err = parse(image, image_bytes, &f), s;
  if (err) return err;
  memset(out, 0, 14 * sizeof(uint32_t));
  out[0] = f.tag; out[1] = f.steps; out[2] = f.bwtsize;
  out[3] = f.ncounters; out[4] = f.nentries; out[5] = f.chunk;
  for (s = 0; s < (int32_t) f.steps; s++) { out[6 + s] = f.dpos[s]; out[10 + s] = f.dbase[s]; }
  return OR_OK;
}

int32_t oracle_max_threads(void) { return omp_get_max_threads(); }
