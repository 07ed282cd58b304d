/*
 * fmi_build.c -- host index builder (the reference's genFMindex.c:457-543,
 * restated on a suffix array instead of libdivsufsort + an LF walk).
 *
 * Construction (bit-exact with genFMindex.c output, pinned by md5 in tests):
 *   SA       : suffix array of T$ ('$' lowest), own SA-IS below
 *   BWT_s[r] : (T$)[(SA[r] - 1 - s) mod (n+1)]          (generateOthersBWTs :327-400)
 *   D_s      : the row with SA[r] == s                  (dollarPositionBWT)
 *   '$' is stored as A in every BWT_s                    (:505-509)
 *   c(r)     : sum_s code(BWT_s[r]) << 2s
 *   cnt_b[c] : C'[c] + #{r < b*d : r not in D, c(r) == c}  (precalculateBasesKSteps :184-260)
 *   C'[c]    : sum_{c'<c} total(c') + #{s : (c(D_s) & (~0 << 2s)) <= c}
 *   planes   : bit 31-p of plane (s,t,w) of entry b = bit t of code(BWT_s[b*d+32w+p]),
 *              rows >= n+1 are 0 (bwt2bin :402-455)
 *   dollarBaseBWT[s] = c(D_s)
 * Alphabet modes (KFMI_ALPHABET or kfmi_set_alphabet; the reference has one):
 *   "acgt" (default): the text must be A/C/G/T only -- the reference builder's
 *          LF walk only counts those four letters (precalculateBasesPreviousBWT
 *          :283-309) and produces a broken index for anything else.
 *   "map": every byte goes through base2index first (N -> G, lowercase ->
 *          uppercase, genFMindex.c:71-84) and the index is the consistent
 *          index of that 4-letter text; searches return true suffix-array
 *          intervals of the mapped text (reads are mapped the same way).
 *   "ref": byte-compatible with the reference tool on any text: suffixes
 *          sorted by raw bytes as divbwt64 sorts them (genFMindex.c:482), codes
 *          and counters through base2index (:86-99, :184-260, :402-424), and for
 *          K >= 2 the reference's own LF walk (generateOthersBWTs :327-400),
 *          which for non-ACGT text is not a permutation: rows it never visits
 *          keep whatever malloc returned there (:342).  This builder writes
 *          a defined byte there (0, base2index -> A); the reference run under
 *          glibc's MALLOC_PERTURB_=p holds p ^ 0xff, which pins its output
 *          (tests/golden/alpha; the test harness patches our image with that
 *          byte, tests/ref_fill.py).  For ACGT-only text the three modes agree.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../kfmi_internal.h"

#define EMPTY 0xFFFFFFFFu

/* ----------------------------------------------------------------------- */
/* SA-IS (Nong, Zhang & Chan 2009) over 32-bit indexes.                    */
/* T has n symbols in [0, alpha) and T[n-1] == 0 is a unique sentinel.     */
/* ----------------------------------------------------------------------- */

typedef struct {
  const void *t;
  int wide;            /* 0: uint8_t symbols, 1: uint32_t symbols */
} sym_t;

static inline uint32_t SYM(const sym_t *s, uint32_t i)
{
  return s->wide ? ((const uint32_t *) s->t)[i] : ((const uint8_t *) s->t)[i];
}

#define TGET(tb, i) (((tb)[(i) >> 3] >> ((i) & 7)) & 1u)
#define TSET(tb, i, v) ((tb)[(i) >> 3] = (uint8_t) (((tb)[(i) >> 3] & ~(1u << ((i) & 7))) | ((v) << ((i) & 7))))
#define IS_LMS(tb, i) ((i) > 0 && TGET(tb, i) && !TGET(tb, (i) - 1))

static void buckets(const sym_t *s, uint32_t n, uint32_t *bkt, uint32_t alpha, int ends)
{
  uint32_t i, sum = 0;
  memset(bkt, 0, sizeof(uint32_t) * (alpha + 1));
  for (i = 0; i < n; i++) bkt[SYM(s, i)]++;
  for (i = 0; i < alpha; i++) {
    sum += bkt[i];
    bkt[i] = ends ? sum : sum - bkt[i];
  }
}

static void induce(const sym_t *s, const uint8_t *tb, uint32_t *sa, uint32_t n, uint32_t *bkt, uint32_t alpha)
{
  uint32_t i, j;
  buckets(s, n, bkt, alpha, 0);
  for (i = 0; i < n; i++) {
    j = sa[i];
    if (j != EMPTY && j > 0 && !TGET(tb, j - 1)) sa[bkt[SYM(s, j - 1)]++] = j - 1;
  }
  buckets(s, n, bkt, alpha, 1);
  for (i = n; i-- > 0;) {
    j = sa[i];
    if (j != EMPTY && j > 0 && TGET(tb, j - 1)) sa[--bkt[SYM(s, j - 1)]] = j - 1;
  }
}

static int sais_rec(const sym_t *s, uint32_t *sa, uint32_t n, uint32_t alpha)
{
  uint8_t *tb;
  uint32_t *bkt;
  uint32_t i, j, n1, name, prev;
  if (n == 1) { sa[0] = 0; return 0; }
  tb = (uint8_t *) calloc(n / 8 + 1, 1);
  bkt = (uint32_t *) malloc(sizeof(uint32_t) * (alpha + 1));
  if (!tb || !bkt) { free(tb); free(bkt); return -1; }

  /* S/L types: T[n-1] is S; T[i] is S iff T[i] < T[i+1] or equal and T[i+1] is S */
  TSET(tb, n - 1, 1u);
  for (i = n - 1; i-- > 0;) {
    uint32_t a = SYM(s, i), b = SYM(s, i + 1);
    TSET(tb, i, (a < b || (a == b && TGET(tb, i + 1))) ? 1u : 0u);
  }

  /* stage 1: sort the LMS substrings by induction */
  buckets(s, n, bkt, alpha, 1);
  for (i = 0; i < n; i++) sa[i] = EMPTY;
  for (i = 1; i < n; i++)
    if (IS_LMS(tb, i)) sa[--bkt[SYM(s, i)]] = i;
  induce(s, tb, sa, n, bkt, alpha);

  /* compact the sorted LMS positions into sa[0..n1) */
  n1 = 0;
  for (i = 0; i < n; i++)
    if (IS_LMS(tb, sa[i])) sa[n1++] = sa[i];

  /* name the LMS substrings (equal substrings get equal names) */
  for (i = n1; i < n; i++) sa[i] = EMPTY;
  name = 0;
  prev = EMPTY;
  for (i = 0; i < n1; i++) {
    uint32_t pos = sa[i], d;
    int diff = 0;
    for (d = 0;; d++) {
      if (prev == EMPTY || pos + d >= n || prev + d >= n || SYM(s, pos + d) != SYM(s, prev + d) ||
          TGET(tb, pos + d) != TGET(tb, prev + d)) {
        diff = 1;
        break;
      }
      if (d > 0 && (IS_LMS(tb, pos + d) || IS_LMS(tb, prev + d))) break;
    }
    if (diff) { name++; prev = pos; }
    sa[n1 + pos / 2] = name - 1;
  }
  for (i = n, j = n; i-- > n1;)
    if (sa[i] != EMPTY) sa[--j] = sa[i];

  /* stage 2: sort the reduced string (recursively if names repeat) */
  {
    uint32_t *s1 = sa + n - n1;
    if (name < n1) {
      sym_t r = {s1, 1};
      if (sais_rec(&r, sa, n1, name)) { free(tb); free(bkt); return -1; }
    } else {
      for (i = 0; i < n1; i++) sa[s1[i]] = i;
    }
    /* stage 3: induce the full SA from the sorted LMS suffixes */
    for (i = 1, j = 0; i < n; i++)
      if (IS_LMS(tb, i)) s1[j++] = i;
    for (i = 0; i < n1; i++) sa[i] = s1[sa[i]];
    for (i = n1; i < n; i++) sa[i] = EMPTY;
    buckets(s, n, bkt, alpha, 1);
    for (i = n1; i-- > 0;) {
      j = sa[i];
      sa[i] = EMPTY;
      sa[--bkt[SYM(s, j)]] = j;
    }
  }
  induce(s, tb, sa, n, bkt, alpha);
  free(tb);
  free(bkt);
  return 0;
}

/* SA of text_codes[0..n) where text_codes[n-1] == 0 is the unique sentinel. */
int32_t kfmi_sais(const uint8_t *text_codes, uint32_t *sa, uint32_t n, uint32_t alpha)
{
  sym_t s = {text_codes, 0};
  if (n == 0) return KFMI_SUCCESS;
  return sais_rec(&s, sa, n, alpha) ? KFMI_E_BUILDING_BWT : KFMI_SUCCESS;
}

/* ----------------------------------------------------------------------- */
/* tag-100 index from the suffix array of T$                               */
/* ----------------------------------------------------------------------- */

/* codes: T as 2-bit codes (0..3), n symbols; sa: n+1 rows of T$ (sa[0] == n) */
int32_t kfmi_index_from_sa(const uint8_t *codes, const uint32_t *sa, uint64_t n, uint32_t k, uint32_t d,
                           kfmi_fmi_t **out)
{
  const uint64_t rows = n + 1;
  const uint32_t nc = 1u << (2 * k), nb = d / 32;
  uint32_t nentries, s, c, dpos[KFMI_MAX_STEPS], dbase[KFMI_MAX_STEPS];
  uint64_t *total, r;
  uint32_t *cprime;
  kfmi_fmi_t *f;
  int32_t err;
  /* n + 1 >= k: every D_s exists and (SA - 1 - s) wraps at most once */
  if (k < 1 || k > KFMI_MAX_STEPS || d == 0 || d % 32 || rows > 0xFFFFFFFFull || rows < k)
    return KFMI_E_BAD_ARGUMENT;
  nentries = (uint32_t) ((rows + d - 1) / d);
  for (s = 0; s < k; s++) { dpos[s] = 0; dbase[s] = 0; }
  err = kfmi_index_alloc(100, k, (uint32_t) rows, nentries, d, NULL, NULL, &f);
  if (err) return err;
  total = (uint64_t *) calloc(nc, sizeof(uint64_t));
  cprime = (uint32_t *) calloc(nc, sizeof(uint32_t));
  if (!total || !cprime) { free(total); free(cprime); freeIndex((void **) &f); return KFMI_E_ALLOCATING_FMI; }

  /* D_s first (rows whose suffix starts at s): needed to exclude them while counting */
  for (r = 0; r < rows; r++)
    if (sa[r] < k) dpos[sa[r]] = (uint32_t) r;

  {
    uint32_t *run = (uint32_t *) calloc(nc, sizeof(uint32_t));
    const uint32_t ew = f->entry_words, nbw = 2 * nb * k;
    if (!run) { free(total); free(cprime); freeIndex((void **) &f); return KFMI_E_ALLOCATING_FMI; }
    for (r = 0; r < rows; r++) {
      const uint64_t b = r / d;
      const uint32_t off = (uint32_t) (r % d), w = off / 32, p = off % 32;
      uint32_t *ent = f->h_index + b * ew;
      uint32_t code = 0, isd = 0;
      if (off == 0) memcpy(ent + nbw, run, sizeof(uint32_t) * nc);   /* Occ before block b */
      for (s = 0; s < k; s++) {
        /* BWT_s[r] = (T$)[(SA[r]-1-s) mod (n+1)], '$' -> A */
        int64_t pos = (int64_t) sa[r] - 1 - (int64_t) s;
        uint32_t cs;
        if (pos < 0) pos += (int64_t) rows;
        cs = ((uint64_t) pos == n) ? 0u : codes[pos];
        code |= cs << (2 * s);
        if (cs & 1u) ent[kfmi_plane_index(100, k, nb, s, 0, w)] |= 1u << (31 - p);
        if (cs & 2u) ent[kfmi_plane_index(100, k, nb, s, 1, w)] |= 1u << (31 - p);
      }
      for (s = 0; s < k; s++) if (dpos[s] == r) { isd = 1; dbase[s] = code; }
      if (!isd) { run[code]++; total[code]++; }
    }
    free(run);
  }
  /* C'[c] = sum_{c'<c} total(c') + #{s : (c(D_s) & (~0 << 2s)) <= c} */
  {
    uint64_t acc = 0;
    for (c = 0; c < nc; c++) { cprime[c] = (uint32_t) acc; acc += total[c]; }
    for (s = 0; s < k; s++) {
      uint32_t masked = dbase[s] & (0xFFFFFFFFu << (2 * s));
      for (c = masked; c < nc; c++) cprime[c]++;
    }
  }
  {
    const uint32_t ew = f->entry_words, nbw = 2 * nb * k;
    uint64_t b;
    for (b = 0; b < nentries; b++) {
      uint32_t *cnt = f->h_index + b * ew + nbw;
      for (c = 0; c < nc; c++) cnt[c] += cprime[c];
    }
  }
  for (s = 0; s < k; s++) {
    f->dollarPositionBWT[s] = dpos[s];
    f->dollarBaseBWT[s] = dbase[s];
    f->modposdollarBWT[s] = dpos[s] / d;
  }
  {
    const void *img; uint64_t bytes;
    kfmi_index_image(f, &img, &bytes);   /* refresh header words */
  }
  free(total);
  free(cprime);
  *out = f;
  return KFMI_SUCCESS;
}

/* ----------------------------------------------------------------------- */
/* alphabet modes (see the header comment)                                   */
/* ----------------------------------------------------------------------- */

static int g_alpha = -1;   /* -1: KFMI_ALPHABET */

int kfmi_alphabet_mode(void)
{
  const char *e;
  if (g_alpha >= 0) return g_alpha;
  e = getenv("KFMI_ALPHABET");
  if (e && !strcmp(e, "map")) return KFMI_ALPHA_MAP;
  if (e && !strcmp(e, "ref")) return KFMI_ALPHA_REF;
  return KFMI_ALPHA_ACGT;
}

int32_t kfmi_set_alphabet(const char *name)
{
  if (!name) { g_alpha = -1; return KFMI_SUCCESS; }
  if (!strcmp(name, "acgt")) g_alpha = KFMI_ALPHA_ACGT;
  else if (!strcmp(name, "map")) g_alpha = KFMI_ALPHA_MAP;
  else if (!strcmp(name, "ref")) g_alpha = KFMI_ALPHA_REF;
  else return KFMI_E_BAD_ARGUMENT;
  return KFMI_SUCCESS;
}

/* 2-bit codes of the text: exact A/C/G/T only (acgt; -1 on any other byte), or
 * base2index of every byte (map, ref; ref rejects NUL, which would tie with
 * the '$' sentinel of the raw-byte sort).  *acgt_only: no byte outside A/C/G/T. */
static int text_to_codes(const char *text, uint64_t n, uint8_t *codes, int mode, int *acgt_only)
{
  uint64_t i;
  int pure = 1;
  for (i = 0; i < n; i++) {
    const uint8_t x = (uint8_t) text[i];
    switch (x) {
      case 'A': codes[i] = 0; break;
      case 'C': codes[i] = 1; break;
      case 'G': codes[i] = 2; break;
      case 'T': codes[i] = 3; break;
      default:
        if (mode == KFMI_ALPHA_ACGT || (mode == KFMI_ALPHA_REF && x == 0)) return -1;
        codes[i] = (uint8_t) base2index(x);
        pure = 0;
    }
  }
  if (acgt_only) *acgt_only = pure;
  return 0;
}

/* ----------------------------------------------------------------------- */
/* "ref" mode, K >= 2: the reference builder's own LF walk                  */
/* ----------------------------------------------------------------------- */

static inline int64_t ref_mod(int64_t x, int64_t m) { return (x % m + m) % m; }   /* genFMindex.c:60-62 */

/* Tag-100 index of `text` (n raw bytes) from its raw-byte suffix array sa
 * (n + 1 rows of T$, sa[0] == n) the way genFMindex.c:457-543 builds it:
 * BWT_0 from the sort, BWT_1..BWT_{k-1} by the walk of generateOthersBWTs
 * (:327-400) on the chunk-32 counters of precalculateBasesPreviousBWT
 * (:262-325, exact 'A'/'C'/'G'/'T' only; any other byte sends the walk to row
 * 0 + its in-chunk count), rows the walk never writes holding 0 (the
 * reference: uninitialised memory, :342); '$' -> A
 * at every D_s (:505-509); then counters, planes and dollarBaseBWT through
 * base2index (precalculateBasesKSteps :184-260, bwt2bin :427-455, :518-520). */
int32_t kfmi_index_ref_walk(const char *text, const uint32_t *sa, uint64_t n, uint32_t k, uint32_t d,
                            kfmi_fmi_t **out)
{
  const uint64_t rows = n + 1;
  const uint32_t nc = 1u << (2 * k), nb = d / 32, nchunk = (uint32_t) ((rows + 31) / 32);
  uint8_t *bwt[KFMI_MAX_STEPS] = {NULL, NULL, NULL, NULL};
  uint32_t (*cnt32)[4] = NULL;
  uint32_t nentries, s, c, dpos[KFMI_MAX_STEPS], dbase[KFMI_MAX_STEPS];
  uint64_t r, tot[4] = {0, 0, 0, 0}, *total = NULL;
  uint32_t *cprime = NULL, *run = NULL;
  int64_t position, refpos;
  kfmi_fmi_t *f = NULL;
  int32_t err = KFMI_E_ALLOCATING_BWT;
  /* rows up to the builders' own limit (n + 1 <= 2^32 - 2): positions are
   * int64 and the chunk counters u32.  The reference's int32 mod() (B8) goes
   * wrong above 2^31 rows only for the last K - 1 walk steps, where it reads
   * ref[-1] into a '$' row that :505-509 overwrites with 'A' -- the bytes
   * ref_mod gives -- so no cap of its own is needed here. */
  if (k < 1 || k > KFMI_MAX_STEPS || d == 0 || d % 32 || rows > 0xFFFFFFFEull || rows < k) return KFMI_E_BAD_ARGUMENT;
  for (s = 0; s < k; s++) {
    bwt[s] = (uint8_t *) malloc(rows);
    if (!bwt[s]) goto done;
    if (s) memset(bwt[s], 0, rows);   /* a defined byte where the walk never writes */
  }
  for (s = 0; s < k; s++) { dpos[s] = 0; dbase[s] = 0; }
  /* BWT_0 with '$' at its primary index (:482-494) */
  for (r = 0; r < rows; r++) {
    bwt[0][r] = sa[r] == 0 ? (uint8_t) '$' : (uint8_t) text[sa[r] - 1];
    if (sa[r] == 0) dpos[0] = (uint32_t) r;
  }
  if (k > 1) {
    /* precalculateBasesPreviousBWT, chunk 32 (:262-325) */
    cnt32 = (uint32_t (*)[4]) malloc(sizeof(*cnt32) * nchunk);
    if (!cnt32) goto done;
    for (r = 0; r < rows; r++) {
      if (r % 32 == 0)
        for (c = 0; c < 4; c++) cnt32[r / 32][c] = (uint32_t) tot[c];
      switch (bwt[0][r]) {
        case 'A': tot[0]++; break;
        case 'C': tot[1]++; break;
        case 'G': tot[2]++; break;
        case 'T': tot[3]++; break;
        default: break;
      }
    }
    {
      const uint32_t acc[4] = {1u, (uint32_t) (1 + tot[0]), (uint32_t) (1 + tot[0] + tot[1]),
                               (uint32_t) (1 + tot[0] + tot[1] + tot[2])};
      uint32_t j;
      for (j = 0; j < nchunk; j++)
        for (c = 0; c < 4; c++) cnt32[j][c] += acc[c];
    }
    /* generateOthersBWTs (:347-391) */
    position = dpos[0];
    for (refpos = (int64_t) rows - 1; refpos >= 0; refpos--) {
      const int64_t desp = position % 32, posb = position - desp;
      uint8_t base;
      int64_t j;
      if (refpos >= (int64_t) k - 1) {
        for (s = 1; s < k; s++) bwt[s][position] = (uint8_t) text[refpos - s];
      } else {
        for (s = 1; s < k; s++) {
          const int64_t m = ref_mod(refpos - (int64_t) s, (int64_t) rows);
          bwt[s][position] = m == (int64_t) rows - 1 ? (uint8_t) '$' : (uint8_t) text[m];
        }
        dpos[refpos + 1] = (uint32_t) position;
      }
      base = bwt[0][position];
      switch (base) {
        case 'A': position = cnt32[position / 32][0]; break;
        case 'C': position = cnt32[position / 32][1]; break;
        case 'G': position = cnt32[position / 32][2]; break;
        case 'T': position = cnt32[position / 32][3]; break;
        default: position = 0; break;
      }
      for (j = 0; j < desp; j++)
        if (bwt[0][posb + j] == base) position++;
    }
  }
  for (s = 0; s < k; s++) bwt[s][dpos[s]] = 'A';   /* :505-509 */

  /* precalculateBasesKSteps (:184-260) and bwt2bin (:427-455) */
  nentries = (uint32_t) ((rows + d - 1) / d);
  err = kfmi_index_alloc(100, k, (uint32_t) rows, nentries, d, NULL, NULL, &f);
  if (err) goto done;
  err = KFMI_E_ALLOCATING_FMI;
  total = (uint64_t *) calloc(nc, sizeof(uint64_t));
  cprime = (uint32_t *) calloc(nc, sizeof(uint32_t));
  run = (uint32_t *) calloc(nc, sizeof(uint32_t));
  if (!total || !cprime || !run) goto done;
  {
    const uint32_t ew = f->entry_words, nbw = 2 * nb * k;
    for (r = 0; r < rows; r++) {
      const uint64_t b = r / d;
      const uint32_t off = (uint32_t) (r % d), w = off / 32, p = off % 32;
      uint32_t *ent = f->h_index + b * ew, code = 0, isd = 0;
      if (off == 0) memcpy(ent + nbw, run, sizeof(uint32_t) * nc);
      for (s = 0; s < k; s++) {
        const uint32_t cs = base2index(bwt[s][r]);
        code |= cs << (2 * s);
        if (cs & 1u) ent[kfmi_plane_index(100, k, nb, s, 0, w)] |= 1u << (31 - p);
        if (cs & 2u) ent[kfmi_plane_index(100, k, nb, s, 1, w)] |= 1u << (31 - p);
      }
      for (s = 0; s < k; s++) if (dpos[s] == r) isd = 1;   /* checkPositionBWT (:114-121) */
      if (!isd) { run[code]++; total[code]++; }
    }
    for (s = 0; s < k; s++) {   /* index2BaseBWT at D_s (:518-520) */
      uint32_t code = 0, t;
      for (t = 0; t < k; t++) code |= base2index(bwt[t][dpos[s]]) << (2 * t);
      dbase[s] = code;
    }
    {
      uint64_t acc = 0;
      for (c = 0; c < nc; c++) { cprime[c] = (uint32_t) acc; acc += total[c]; }
      for (s = 0; s < k; s++) {   /* dollar2BaseBWT adjustments (:246-250) */
        const uint32_t masked = dbase[s] & (0xFFFFFFFFu << (2 * s));
        for (c = masked; c < nc; c++) cprime[c]++;
      }
    }
    for (r = 0; r < nentries; r++) {
      uint32_t *cn = f->h_index + r * ew + nbw;
      for (c = 0; c < nc; c++) cn[c] += cprime[c];
    }
  }
  for (s = 0; s < k; s++) {
    f->dollarPositionBWT[s] = dpos[s];
    f->dollarBaseBWT[s] = dbase[s];
    f->modposdollarBWT[s] = dpos[s] / d;
  }
  {
    const void *img; uint64_t bytes;
    kfmi_index_image(f, &img, &bytes);   /* refresh header words */
  }
  *out = f;
  f = NULL;
  err = KFMI_SUCCESS;
done:
  if (f) freeIndex((void **) &f);
  for (s = 0; s < k; s++) free(bwt[s]);
  free(cnt32);
  free(total);
  free(cprime);
  free(run);
  return err;
}

int32_t kfmi_build_index_cpu(const char *text, uint64_t n, uint32_t k, uint32_t d, void **index)
{
  return kfmi_build_index_cpu_sa(text, n, k, d, 0, index);
}

/* Tag-100 index plus, when sa_rate != 0, the row-sampled suffix array
 * SA[i * sa_rate] (locate). */
int32_t kfmi_build_index_cpu_sa(const char *text, uint64_t n, uint32_t k, uint32_t d, uint32_t sa_rate,
                                void **index)
{
  uint8_t *codes, *sym;
  uint32_t *sa;
  uint64_t i;
  int32_t err;
  const int mode = kfmi_alphabet_mode();
  int acgt_only = 1;
  if (n == 0 || n + 1 < k || n + 1 > 0xFFFFFFFEull) return KFMI_E_BAD_ARGUMENT;
  if (k < 1 || k > KFMI_MAX_STEPS || d == 0 || d % 32) return KFMI_E_BAD_ARGUMENT;
  if (sa_rate && !kfmi_sa_rate_ok(sa_rate)) return KFMI_E_BAD_ARGUMENT;
  /* on 2 MB pages (kfmi_big_alloc): SA-IS scatters over the whole of sa */
  codes = (uint8_t *) kfmi_big_alloc(n);
  sym = (uint8_t *) kfmi_big_alloc(n + 1);
  sa = (uint32_t *) kfmi_big_alloc(sizeof(uint32_t) * (n + 1));
  if (!codes || !sym || !sa) {
    kfmi_big_free(codes); kfmi_big_free(sym); kfmi_big_free(sa);
    return KFMI_E_ALLOCATING_BWT;
  }
  if (text_to_codes(text, n, codes, mode, &acgt_only)) {
    kfmi_big_free(codes); kfmi_big_free(sym); kfmi_big_free(sa);
    return KFMI_E_BUILDING_BWT;
  }
  if (mode == KFMI_ALPHA_REF && !acgt_only) {
    for (i = 0; i < n; i++) sym[i] = (uint8_t) text[i];        /* raw bytes, as divbwt64 sorts them */
    sym[n] = 0;
    err = kfmi_sais(sym, sa, (uint32_t) (n + 1), 256);
  } else {
    for (i = 0; i < n; i++) sym[i] = (uint8_t) (codes[i] + 1);   /* '$' = 0 < A..T = 1..4 */
    sym[n] = 0;
    err = kfmi_sais(sym, sa, (uint32_t) (n + 1), 5);
  }
  kfmi_big_free(sym);
  if (!err) {
    if (mode == KFMI_ALPHA_REF && !acgt_only && k > 1)
      err = kfmi_index_ref_walk(text, sa, n, k, d, (kfmi_fmi_t **) index);
    else
      err = kfmi_index_from_sa(codes, sa, n, k, d, (kfmi_fmi_t **) index);
  }
  if (!err && sa_rate) {
    kfmi_fmi_t *f = (kfmi_fmi_t *) *index;
    err = kfmi_sa_alloc(f, sa_rate);
    if (err) freeIndex(index);
    else
      for (i = 0; i < f->sa_count; i++) f->h_sa[i] = sa[i * sa_rate];
  }
  kfmi_big_free(codes);
  kfmi_big_free(sa);
  return err;
}

int32_t kfmi_build_index_ex(const char *text, uint64_t n, uint32_t k, uint32_t d, uint32_t sa_rate,
                            int32_t on_device, void **index)
{
  if (sa_rate && !kfmi_sa_rate_ok(sa_rate)) return KFMI_E_BAD_ARGUMENT;
  if (on_device) return kfmi_build_index_gpu_sa(text, n, k, d, sa_rate, index);
  return kfmi_build_index_cpu_sa(text, n, k, d, sa_rate, index);
}

/* interface.h:35: K, d from KFMI_K / KFMI_D (the reference: -DK_STEPS, -DNUM_CHUNK);
 * KFMI_SA_RATE > 0 also keeps the row-sampled suffix array (locate). */
int32_t buildIndex(void *reference, void **index)
{
  kfmi_ref_t *ref = (kfmi_ref_t *) reference;
  const char *ek = getenv("KFMI_K"), *ed = getenv("KFMI_D"), *eg = getenv("KFMI_BUILD_GPU");
  const char *es = getenv("KFMI_SA_RATE");
  uint32_t k = ek ? (uint32_t) atoi(ek) : 2, d = ed ? (uint32_t) atoi(ed) : 64;
  uint32_t rate = es ? (uint32_t) atoi(es) : 0;
  int use_gpu = eg ? atoi(eg) : (kfmi_device_count() > 0);
  if (!ref) return KFMI_E_BAD_ARGUMENT;
  return kfmi_build_index_ex(ref->h_reference, ref->size, k, d, rate, use_gpu, index);
}
