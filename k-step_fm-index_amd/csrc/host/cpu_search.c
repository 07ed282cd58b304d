/*
 * cpu_search.c -- searchIndexCPU (interface.h:30): the k-step backward search
 * on the host, for the reference's CPU driver (common/searchQueries.c:84-95)
 * and for callers without a GPU.
 *
 * Contract: the driver opens `#pragma omp parallel` and every
 * thread of the team calls searchIndexCPU(index, queries, results); the
 * function shares the queries out with an orphaned worksharing loop
 * (fmIndexCPUBaseline.c:195 `omp for schedule(static)`), so this file is
 * compiled with gcc -fopenmp and the library links libgomp -- the runtime the
 * driver's own parallel region belongs to.  Called outside a parallel region
 * it searches every query on the calling thread; kfmi_search_cpu() opens its
 * own region.
 *
 * Results are the reference searchers' integers, bit for bit:
 *   tag 100 / 101  fmIndexCPUBaseline.c:197-290 (plain counters),
 *   tag 200 / 201  fmIndexCPUBaseline-AltCounters.c:186-303 (alternate
 *                  counters: entry b or b+1 by block parity and code half,
 *                  the inverted mask, the "X <= D_s" '$' rule).
 * Where the reference reads past its own index (B5: a step with L or R in
 * block nentries when (n+1) % d == 0) the plain step reads a padding entry,
 * as every GPU layout does: the end counters (kfmi_search.hip end_counters:
 * the next block the builder would write, a '$' row two D_s share excluded
 * once) and rows that read as code 0 -- on a 'ref'-mode index
 * whose walk is not a permutation a step can land past n+1
 * (tests/test_alphabet.py dup_dollar_last_block_indexes) -- and the AltCounters step
 * reads zero planes and counters past the sentinel S and is capped at
 * (S+2)*d - 1 rows, as the GPU's AltCounters backends do (kfmi_device.h
 * ac_clamp).  Reads with m % K != 0 take
 * their last m % K bases from a remainder table (the true suffix-array
 * interval, as every plain GPU backend); the AltCounters tags
 * reject them (kfmi_last_error 33), the reference reads query[-1] (B6).
 *
 * Speed: the reference walks one query at a time, so each LF waits for its
 * DRAM line (~90 ns).  Here every thread steps a batch of KFMI_CPU_BATCH
 * queries (default 32) together: first the lines of all their L and R ends
 * are prefetched, then the LFs are computed, so ~2 x batch misses are in
 * flight per core instead of 2.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>
#include "../kfmi_internal.h"

#define CS_MAX_BATCH 256

typedef struct {
  const uint32_t *ent;       /* entry 0 */
  uint32_t ew;               /* u32 words per entry */
  uint32_t K, NB, NC, d;
  uint32_t cnt_off, pl_off;  /* word offsets of the counters and the planes in an entry */
  int      inter;            /* planes in tag-101 order (w * 2K + 2s + t) */
  int      ac;               /* AltCounters semantics (tags 200, 201) */
  uint32_t nent, bwtsize;
  uint32_t dpos[KFMI_MAX_STEPS], dbase[KFMI_MAX_STEPS], dblk[KFMI_MAX_STEPS];
  uint32_t endc[1u << (2 * KFMI_MAX_STEPS)];   /* the padding entry's counters (plain tags) */
} cs_idx_t;

static inline uint32_t cs_code(uint8_t x)   /* base2index, fmIndexCPUBaseline.c:213-222 */
{
  const uint32_t b1 = x & 4u, b0 = b1 ? ((x & 2u) ^ 2u) : (x & 2u);
  return (b1 | b0) >> 1;
}

/* The hot functions take the geometry (K, NB = d / 32, plane order, counter
 * semantics) as arguments and are always inlined into cs_batch_impl, whose
 * instances below fix them at compile time: the plane offsets, d and the
 * loops are then constants, as in the reference's -D build. */
#define CS_INLINE static inline __attribute__((always_inline))

CS_INLINE uint32_t cs_plane(uint32_t K, uint32_t NB, int inter, uint32_t s, uint32_t t, uint32_t w)
{
  return inter ? w * 2u * K + 2u * s + t : s * 2u * NB + t * NB + w;
}

/* cs_top_bits[k]: the k most significant bits of a word (row p of a 32-row
 * word is bit 31 - p, MSB first) */
static const uint32_t cs_top_bits[33] = {
  0x00000000u, 0x80000000u, 0xC0000000u, 0xE0000000u, 0xF0000000u, 0xF8000000u, 0xFC000000u, 0xFE000000u,
  0xFF000000u, 0xFF800000u, 0xFFC00000u, 0xFFE00000u, 0xFFF00000u, 0xFFF80000u, 0xFFFC0000u, 0xFFFE0000u,
  0xFFFF0000u, 0xFFFF8000u, 0xFFFFC000u, 0xFFFFE000u, 0xFFFFF000u, 0xFFFFF800u, 0xFFFFFC00u, 0xFFFFFE00u,
  0xFFFFFF00u, 0xFFFFFF80u, 0xFFFFFFC0u, 0xFFFFFFE0u, 0xFFFFFFF0u, 0xFFFFFFF8u, 0xFFFFFFFCu, 0xFFFFFFFEu,
  0xFFFFFFFFu};

/* rows of code c among the first o rows of the block at pl (or among the
 * others when inv): the bit-plane count of the reference's inner loop.
 * sel(p, bit) = bit ? p : ~p is p ^ (bit - 1). */
CS_INLINE uint32_t cs_count(uint32_t K, uint32_t NB, int inter, const uint32_t *pl, uint32_t o, uint32_t c, int inv)
{
  uint32_t pop = 0, w, s;
  for (w = 0; w < NB; ++w) {
    /* the top clamp(o - 32w, 0, 32) bits, from a table: no branch on the
     * (random) offset, which a compare-and-shift turns into one */
    const int32_t sh = (int32_t) o - 32 * (int32_t) w;
    uint32_t m = cs_top_bits[sh < 0 ? 0 : (sh > 32 ? 32 : sh)];
    if (inv) m = ~m;
    for (s = 0; s < K; ++s) {
      const uint32_t cs = (c >> (2u * s)) & 3u;
      m &= (pl[cs_plane(K, NB, inter, s, 0, w)] ^ ((cs & 1u) - 1u)) &
           (pl[cs_plane(K, NB, inter, s, 1, w)] ^ (((cs >> 1) & 1u) - 1u));
    }
    pop += (uint32_t) __builtin_popcount(m);
  }
  return pop;
}

/* AltCounters: the entry whose counter serves (b, c) is b + e */
CS_INLINE uint32_t cs_ac_e(uint32_t K, uint32_t b, uint32_t c)
{
  const uint32_t half = (1u << (2u * K)) >> 1;
  return ((b & 1u) && c < half) || (!(b & 1u) && c >= half);
}

CS_INLINE const uint32_t *cs_entry(const cs_idx_t *ix, uint32_t b)
{
  return ix->ent + (uint64_t) b * ix->ew;
}

/* the lines one LF of end X with code c reads: planes of block b, its counter */
CS_INLINE void cs_prefetch(const cs_idx_t *ix, uint32_t K, uint32_t NB, int ac, uint32_t X, uint32_t c)
{
  uint32_t b = X / (32u * NB), bc;
  if (b >= ix->nent) b = ix->nent - 1;
  bc = b;
  if (ac) {
    bc = b + cs_ac_e(K, b, c);
    if (bc >= ix->nent) bc = b;
    c &= ((1u << (2u * K)) >> 1) - 1u;
  }
  __builtin_prefetch(cs_entry(ix, b) + ix->pl_off, 0, 3);
  __builtin_prefetch(cs_entry(ix, bc) + ix->cnt_off + c, 0, 3);
}

CS_INLINE uint32_t cs_lf(const cs_idx_t *ix, uint32_t K, uint32_t NB, int inter, int ac, uint32_t X, uint32_t c)
{
  const uint32_t d = 32u * NB;
  uint32_t b = X / d, o = X % d, s, pop;
  int corr = 0;
  if (!ac) {
    if (b >= ix->nent) {   /* B5: the padding entry -- end counters, its rows read as code 0 */
      const uint32_t past = X - ix->nent * d;
      return ix->endc[c] + (c == 0 ? (past < d ? past : d) : 0u);
    }
    pop = cs_count(K, NB, inter, cs_entry(ix, b) + ix->pl_off, o, c, 0);
    for (s = 0; s < K; ++s)
      corr += (ix->dblk[s] == b && ix->dbase[s] == c && X > ix->dpos[s]);
    return cs_entry(ix, b)[ix->cnt_off + c] + pop - (uint32_t) corr;
  } else {
    const uint32_t e = cs_ac_e(K, b, c), half = (1u << (2u * K)) >> 1;
    const uint32_t cnt = b + e < ix->nent ? cs_entry(ix, b + e)[ix->cnt_off + (c & (half - 1u))] : 0u;
    const uint64_t cap = (((uint64_t) ix->bwtsize + d - 1u) / d + 2u) * d - 1u;   /* kfmi_device.h ac_clamp */
    uint32_t v;
    if (b < ix->nent)
      pop = cs_count(K, NB, inter, cs_entry(ix, b) + ix->pl_off, o, c, (int) e);
    else   /* block S+1, past the sentinel: zero planes, rows of code 0 (the GPU layouts' padding) */
      pop = c == 0 ? (e ? d - o : o) : 0u;
    for (s = 0; s < K; ++s)
      if (ix->dblk[s] == b && ix->dbase[s] == c)
        corr += e ? (X <= ix->dpos[s]) : (X > ix->dpos[s]);
    v = e ? cnt - (pop - (uint32_t) corr) : cnt + (pop - (uint32_t) corr);
    return v > cap ? (uint32_t) cap : v;
  }
}

/* K-mer code of the bases P[j-K+1 .. j]: P[j - i] at bits 2i (fmIndexCPUBaseline.c:202-226) */
CS_INLINE uint32_t cs_kmer(const uint8_t *p, int64_t j, uint32_t K)
{
  uint32_t c = 0, i;
  for (i = 0; i < K; ++i) c |= cs_code(p[j - (int64_t) i]) << (2u * i);
  return c;
}

/* Remainder table for r = m % K (0 < r < K): [L, R) of every r-base string x
 * (its last base at bits 0-1), from two K-steps out of [0, n+1) -- R of
 * x.T^(K-r), L of x.A^(K-r) less the suffixes x.A^j.$ (j < K - r), which sort
 * below x.A^(K-r) inside x's range; the text ends with x.A^j iff row 0 (the
 * suffix "$") has that K-mer code in its low bits.  DESIGN.md 5e. */
static void cs_rem_table(const cs_idx_t *ix, uint32_t r, uint32_t *tab)
{
  const uint32_t pad = 2u * (ix->K - r), n = ix->bwtsize - 1u;
  uint32_t tail = 0, s, x, j;
  const uint32_t *pl = cs_entry(ix, 0) + ix->pl_off;
  for (s = 0; s < ix->K; ++s) {   /* code of row 0: bit 31 of word 0 of each plane */
    const uint32_t b0 = pl[cs_plane(ix->K, ix->NB, ix->inter, s, 0, 0)] >> 31;
    const uint32_t b1 = pl[cs_plane(ix->K, ix->NB, ix->inter, s, 1, 0)] >> 31;
    tail |= (b0 | (b1 << 1)) << (2u * s);
  }
  for (x = 0; x < (1u << (2u * r)); ++x) {
    const uint32_t cA = x << pad, cT = cA | ((1u << pad) - 1u);
    uint32_t L = cs_lf(ix, ix->K, ix->NB, ix->inter, ix->ac, 0u, cA);
    const uint32_t R = cs_lf(ix, ix->K, ix->NB, ix->inter, ix->ac, ix->bwtsize, cT);
    for (j = 0; j + r < ix->K; ++j)
      if (j + r <= n && (tail & ((1u << (2u * j)) - 1u)) == 0u && ((tail >> (2u * j)) & ((1u << (2u * r)) - 1u)) == x)
        --L;
    tab[2 * x] = L;
    tab[2 * x + 1] = R;
  }
}

static int32_t cs_setup(kfmi_fmi_t *f, const kfmi_qrys_t *q, const kfmi_res_t *r, cs_idx_t *ix)
{
  uint32_t s;
  if (!f || !q || !r || !f->h_index) return KFMI_E_BAD_ARGUMENT;
  if (f->steps < 1 || f->steps > KFMI_MAX_STEPS || f->chunk < 32 || f->chunk % 32 || f->nentries < 1)
    return KFMI_E_BAD_ARGUMENT;
  if (r->num < q->num || (q->num && (!q->h_queries || !r->h_results))) return KFMI_E_BAD_ARGUMENT;
  memset(ix, 0, sizeof(*ix));
  ix->ent = f->h_index;
  ix->ew = f->entry_words;
  ix->K = f->steps;
  ix->NB = f->chunk / 32u;
  ix->NC = 1u << (2u * f->steps);
  ix->d = f->chunk;
  ix->nent = f->nentries;
  ix->bwtsize = f->bwtsize;
  switch (f->tag) {
    case KFMI_INDEX_VER_BASELINE:     ix->cnt_off = 2u * ix->NB * ix->K; break;
    case KFMI_INDEX_VER_INTERLEAVE:   ix->cnt_off = 2u * ix->NB * ix->K; ix->inter = 1; break;
    case KFMI_INDEX_VER_BASELINE_AC:  ix->pl_off = ix->NC / 2u; ix->ac = 1; break;
    case KFMI_INDEX_VER_INTERLEAVE_AC: ix->pl_off = ix->NC / 2u; ix->ac = 1; ix->inter = 1; break;
    default: return KFMI_E_BAD_ARGUMENT;
  }
  if (ix->ac && ix->K < 1) return KFMI_E_BAD_ARGUMENT;
  if (ix->ac && q->size % ix->K) return KFMI_E_BAD_ARGUMENT;   /* no AltCounters remainder rule */
  for (s = 0; s < ix->K; ++s) {
    ix->dpos[s] = f->dollarPositionBWT[s];
    ix->dbase[s] = f->dollarBaseBWT[s];
    ix->dblk[s] = f->dollarPositionBWT[s] / f->chunk;
  }
  if (!ix->ac) {
    /* counters at row n+1: the last entry's, plus its rows below n+1, less
     * each distinct '$' row there once, as the builder's counters exclude them
     * (kfmi_search.hip end_counters: what every GPU layout's padding entry
     * holds) */
    const uint32_t last = ix->nent - 1, rows = ix->bwtsize - last * ix->d;
    for (uint32_t c = 0; c < ix->NC; ++c) {
      uint32_t v = cs_entry(ix, last)[ix->cnt_off + c] +
                   cs_count(ix->K, ix->NB, ix->inter, cs_entry(ix, last) + ix->pl_off, rows, c, 0);
      for (s = 0; s < ix->K; ++s) {
        int first = 1;
        for (uint32_t t = 0; t < s; ++t) first = first && ix->dpos[t] != ix->dpos[s];
        v -= (first && ix->dblk[s] == last && ix->dbase[s] == c && ix->bwtsize > ix->dpos[s]);
      }
      ix->endc[c] = v;
    }
  }
  return KFMI_SUCCESS;
}

static int cs_batch_size(void)
{
  const char *e = getenv("KFMI_CPU_BATCH");
  int v = e ? atoi(e) : 32;
  return v < 1 ? 1 : (v > CS_MAX_BATCH ? CS_MAX_BATCH : v);
}

/* queries [q0, q1): step the batch together, prefetching every end's lines
 * before the LFs that need them */
CS_INLINE void cs_batch_impl(const cs_idx_t *ix, const kfmi_qrys_t *qr, uint32_t *res, uint64_t q0, uint64_t q1,
                             const uint32_t *rtab, uint32_t K, uint32_t NB, int inter, int ac)
{
  const uint32_t m = qr->size, rem = m % K, nq = (uint32_t) (q1 - q0);
  uint32_t L[CS_MAX_BATCH], R[CS_MAX_BATCH], C[CS_MAX_BATCH], i;
  int64_t j;
  for (i = 0; i < nq; ++i) {
    const uint8_t *p = (const uint8_t *) qr->h_queries + (q0 + i) * (uint64_t) m;
    L[i] = 0;
    R[i] = ix->bwtsize;
    if (rem) {
      const uint32_t x = cs_kmer(p, (int64_t) m - 1, rem);
      L[i] = rtab[2 * x];
      R[i] = rtab[2 * x + 1];
    }
  }
  for (j = (int64_t) m - 1 - rem; j >= 0; j -= K) {
    for (i = 0; i < nq; ++i) {
      const uint8_t *p = (const uint8_t *) qr->h_queries + (q0 + i) * (uint64_t) m;
      C[i] = cs_kmer(p, j, K);
      cs_prefetch(ix, K, NB, ac, L[i], C[i]);
      cs_prefetch(ix, K, NB, ac, R[i], C[i]);
    }
    for (i = 0; i < nq; ++i) {
      L[i] = cs_lf(ix, K, NB, inter, ac, L[i], C[i]);
      R[i] = cs_lf(ix, K, NB, inter, ac, R[i], C[i]);
    }
  }
  for (i = 0; i < nq; ++i) {
    res[2 * (q0 + i)] = L[i];
    res[2 * (q0 + i) + 1] = R[i];
  }
}

typedef void (*cs_batch_fn)(const cs_idx_t *, const kfmi_qrys_t *, uint32_t *, uint64_t, uint64_t, const uint32_t *);

static void cs_batch_any(const cs_idx_t *ix, const kfmi_qrys_t *qr, uint32_t *res, uint64_t q0, uint64_t q1,
                         const uint32_t *rtab)
{
  cs_batch_impl(ix, qr, res, q0, q1, rtab, ix->K, ix->NB, ix->inter, ix->ac);
}

/* compile-time geometries: K = 1..4 at d = 64 (NB 2) and d = 192 (NB 6), both
 * plane orders, both counter semantics; anything else runs cs_batch_any */
#define CS_FN(K, NB, IN, AC)                                                                            \
  static void cs_batch_##K##_##NB##_##IN##_##AC(const cs_idx_t *ix, const kfmi_qrys_t *qr, uint32_t *res, \
                                                uint64_t q0, uint64_t q1, const uint32_t *rtab)          \
  { cs_batch_impl(ix, qr, res, q0, q1, rtab, K, NB, IN, AC); }
#define CS_FN4(K, NB) CS_FN(K, NB, 0, 0) CS_FN(K, NB, 0, 1) CS_FN(K, NB, 1, 0) CS_FN(K, NB, 1, 1)
CS_FN4(1, 2) CS_FN4(2, 2) CS_FN4(3, 2) CS_FN4(4, 2)
CS_FN4(1, 6) CS_FN4(2, 6)
#define CS_ROW(K, NB) { cs_batch_##K##_##NB##_0_0, cs_batch_##K##_##NB##_0_1, \
                        cs_batch_##K##_##NB##_1_0, cs_batch_##K##_##NB##_1_1 }

static cs_batch_fn cs_pick(const cs_idx_t *ix)
{
  static const cs_batch_fn nb2[4][4] = { CS_ROW(1, 2), CS_ROW(2, 2), CS_ROW(3, 2), CS_ROW(4, 2) };
  static const cs_batch_fn nb6[2][4] = { CS_ROW(1, 6), CS_ROW(2, 6) };
  const int v = 2 * ix->inter + ix->ac;
  if (ix->NB == 2 && ix->K >= 1 && ix->K <= 4) return nb2[ix->K - 1][v];
  if (ix->NB == 6 && ix->K >= 1 && ix->K <= 2) return nb6[ix->K - 1][v];
  return cs_batch_any;
}

/* The body every thread of the caller's team runs (orphaned worksharing). */
static void cs_search_team(kfmi_fmi_t *f, kfmi_qrys_t *q, kfmi_res_t *r)
{
  int32_t err = KFMI_SUCCESS;
  cs_idx_t ix;
  uint32_t rtab[2 * 64];
  uint64_t nb, bi;
  int batch;
  cs_batch_fn fn;
  /* an index built on the device without a host image: fetched once, by one thread */
#pragma omp single copyprivate(err)
  {
    err = f ? kfmi_host_entries(f) : KFMI_E_BAD_ARGUMENT;
    if (!err && r) r->origin = KFMI_RES_FROM_CPU;
  }
  if (!err) err = cs_setup(f, q, r, &ix);
  kfmi_set_last_error(err);
  if (err) return;
  if (q->size % ix.K) cs_rem_table(&ix, q->size % ix.K, rtab);
  batch = cs_batch_size();
  fn = cs_pick(&ix);
  nb = (q->num + (uint64_t) batch - 1) / (uint64_t) batch;
#pragma omp for schedule(static)
  for (bi = 0; bi < nb; ++bi) {
    const uint64_t q0 = bi * (uint64_t) batch, q1 = q0 + (uint64_t) batch < q->num ? q0 + (uint64_t) batch : q->num;
    fn(&ix, q, r->h_results, q0, q1, rtab);
  }
}

/* interface.h:30 / fmIndexCPUBaseline.c:157-292 */
void searchIndexCPU(void *index, void *queries, void *resIntervals)
{
  cs_search_team((kfmi_fmi_t *) index, (kfmi_qrys_t *) queries, (kfmi_res_t *) resIntervals);
}

int32_t kfmi_search_cpu(void *index, void *queries, void *results, int32_t nthreads)
{
  int32_t err = KFMI_SUCCESS;
  const int nt = nthreads > 0 ? nthreads : (getenv("OMP_NUM_THREADS") ? omp_get_max_threads() : kfmi_process_cpus());
#pragma omp parallel num_threads(nt)
  {
    cs_search_team((kfmi_fmi_t *) index, (kfmi_qrys_t *) queries, (kfmi_res_t *) results);
#pragma omp master
    err = kfmi_last_error();
  }
  kfmi_set_last_error(err);
  return err;
}
