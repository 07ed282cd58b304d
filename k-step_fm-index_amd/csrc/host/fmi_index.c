/*
 * fmi_index.c -- index files: load / save / in-memory images and the two
 * offline layout transforms.
 *
 * File format (all u32 little-endian, genFMindex.c:167-178):
 *   tag, steps(K), bwtsize(n+1), ncounters, nentries, chunk(d),
 *   dollarPositionBWT[K], dollarBaseBWT[K], then nentries entries.
 * Entry layouts (NB = d/32, NC = 4^K):
 *   100 .fmi                 [bitmap[2*NB*K] | cnt[NC]]   plane(s,t,w) = s*2NB + t*NB + w
 *   101 .fmi.interleaving    same sizes                    plane(s,t,w) = w*2K + 2s + t
 *   200 .fmi.ac              [cnt[NC/2] | bitmap]          tag-100 plane order, nentries+1
 *   201 .fmi.interleaving.ac [cnt[NC/2] | bitmap]          tag-101 plane order, nentries+1
 * (transformIndexBitmaps.c:269-295, transformIndexAlternateCounters.c:387-479).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../kfmi_internal.h"

uint32_t kfmi_entry_words(uint32_t tag, uint32_t steps, uint32_t chunk)
{
  uint32_t nb = chunk / 32, nc = 1u << (2 * steps);
  return 2 * nb * steps + ((tag == 200 || tag == 201) ? nc / 2 : nc);
}

uint32_t kfmi_plane_index(uint32_t tag, uint32_t steps, uint32_t nb, uint32_t s, uint32_t t, uint32_t w)
{
  if (tag == 101 || tag == 201) return w * 2 * steps + 2 * s + t;
  return s * 2 * nb + t * nb + w;
}

static int valid_geometry(uint32_t tag, uint32_t steps, uint32_t chunk, uint32_t ncounters)
{
  uint32_t nc;
  if (steps < 1 || steps > KFMI_MAX_STEPS) return 0;
  if (chunk == 0 || chunk % 32) return 0;
  nc = 1u << (2 * steps);
  switch (tag) {
    case 100: case 101: return ncounters == nc;
    case 200: case 201: return ncounters == nc / 2;
    default: return 0;
  }
}

/* A header the reference's tools could have written: nentries = ceil(bwtsize /
 * chunk) (genFMindex.c:477), one more for the AltCounters tags' sentinel
 * (transformIndexAlternateCounters.c:138), every '$' row inside [0, bwtsize)
 * and every '$' code a K-mer code.  The reference's loaders take any header and
 * read past their buffers on a damaged one; here it is KFMI_E_READING_FMI. */
static int consistent_header(const uint32_t *h)
{
  const uint32_t tag = h[0], steps = h[1], bwtsize = h[2], nentries = h[4], chunk = h[5];
  const uint64_t want = ((uint64_t) bwtsize + chunk - 1) / chunk + (tag >= 200 ? 1u : 0u);
  uint32_t s;
  if (bwtsize < 2 || nentries != want) return 0;
  for (s = 0; s < steps; s++)
    if (h[6 + s] >= bwtsize || h[6 + steps + s] >= (1u << (2 * steps))) return 0;
  return 1;
}

int32_t kfmi_index_alloc(uint32_t tag, uint32_t steps, uint32_t bwtsize, uint32_t nentries,
                         uint32_t chunk, const uint32_t *dpos, const uint32_t *dbase,
                         kfmi_fmi_t **out)
{
  return kfmi_index_alloc_ex(tag, steps, bwtsize, nentries, chunk, dpos, dbase, 1, out);
}

/* with_entries = 0: header only (h_index NULL), for indexes whose entries stay
 * on the device until asked for (kfmi_host_entries). */
int32_t kfmi_index_alloc_ex(uint32_t tag, uint32_t steps, uint32_t bwtsize, uint32_t nentries,
                            uint32_t chunk, const uint32_t *dpos, const uint32_t *dbase,
                            int with_entries, kfmi_fmi_t **out)
{
  kfmi_fmi_t *f;
  uint32_t s, *h;
  uint32_t nc = 1u << (2 * steps);
  uint32_t ncounters = (tag == 200 || tag == 201) ? nc / 2 : nc;
  if (!valid_geometry(tag, steps, chunk, ncounters)) return KFMI_E_BAD_ARGUMENT;
  f = (kfmi_fmi_t *) calloc(1, sizeof(*f));
  if (!f) return KFMI_E_ALLOCATING_FMI;
  {
    pthread_rwlockattr_t at;
    pthread_rwlockattr_init(&at);
    pthread_rwlockattr_setkind_np(&at, PTHREAD_RWLOCK_PREFER_WRITER_NONRECURSIVE_NP);
    pthread_rwlock_init(&f->rw, &at);
    pthread_rwlockattr_destroy(&at);
  }
  f->tag = tag; f->steps = steps; f->bwtsize = bwtsize; f->ncounters = ncounters;
  f->nentries = nentries; f->chunk = chunk; f->nbitmaps = chunk / 32;
  f->entry_words = kfmi_entry_words(tag, steps, chunk);
  f->header_bytes = 24 + 8 * steps;
  f->image_bytes = f->header_bytes + 4ull * f->entry_words * nentries;
  f->image = (uint8_t *) kfmi_big_alloc((with_entries ? f->image_bytes : f->header_bytes) + 64);
  if (!f->image) { pthread_rwlock_destroy(&f->rw); free(f); return KFMI_E_ALLOCATING_FMI; }
  h = (uint32_t *) f->image;
  h[0] = tag; h[1] = steps; h[2] = bwtsize; h[3] = ncounters; h[4] = nentries; h[5] = chunk;
  for (s = 0; s < steps; s++) {
    f->dollarPositionBWT[s] = dpos ? dpos[s] : 0;
    f->dollarBaseBWT[s] = dbase ? dbase[s] : 0;
    f->modposdollarBWT[s] = f->dollarPositionBWT[s] / chunk;
    h[6 + s] = f->dollarPositionBWT[s];
    h[6 + steps + s] = f->dollarBaseBWT[s];
  }
  f->h_index = with_entries ? (uint32_t *) (f->image + f->header_bytes) : NULL;
  *out = f;
  return KFMI_SUCCESS;
}

static void refresh_header(kfmi_fmi_t *f)
{
  uint32_t *h = (uint32_t *) f->image, s;
  for (s = 0; s < f->steps; s++) {
    h[6 + s] = f->dollarPositionBWT[s];
    h[6 + f->steps + s] = f->dollarBaseBWT[s];
    f->modposdollarBWT[s] = f->dollarPositionBWT[s] / f->chunk;
  }
}

/* Parse and copy a full file image.  fmIndexCPUBaseline.c:71-143 semantics,
 * any tag; `required_tag` != 0 rejects other tags by returning the required
 * one (fmIndexCPUBaseline.c:138-142). */
static int32_t from_image(const uint8_t *img, uint64_t bytes, uint32_t required_tag, kfmi_fmi_t **out)
{
  const uint32_t *h = (const uint32_t *) img;
  uint32_t tag, steps, chunk, ncounters, nentries, ew, hb;
  kfmi_fmi_t *f;
  int32_t err;
  if (bytes < 24) return KFMI_E_READING_FMI;
  tag = h[0]; steps = h[1]; ncounters = h[3]; nentries = h[4]; chunk = h[5];
  if (required_tag && tag != required_tag) return (int32_t) required_tag;
  if (!valid_geometry(tag, steps, chunk, ncounters)) return KFMI_E_READING_FMI;
  hb = 24 + 8 * steps;
  if (bytes < hb || !consistent_header(h)) return KFMI_E_READING_FMI;
  ew = kfmi_entry_words(tag, steps, chunk);
  if (bytes < hb + 4ull * ew * nentries) return KFMI_E_READING_FMI;
  err = kfmi_index_alloc(tag, steps, h[2], nentries, chunk, h + 6, h + 6 + steps, &f);
  if (err) return err;
  memcpy(f->h_index, img + hb, 4ull * ew * nentries);
  *out = f;
  return KFMI_SUCCESS;
}

int32_t kfmi_index_from_image(const void *image, uint64_t bytes, void **index)
{
  return from_image((const uint8_t *) image, bytes, 0, (kfmi_fmi_t **) index);
}

static int32_t load_file(const char *fn, uint32_t required_tag, void **index)
{
  FILE *fp = fopen(fn, "rb");
  uint32_t hdr[6 + 2 * KFMI_MAX_STEPS];
  kfmi_fmi_t *f;
  uint32_t steps, hb, ew;
  uint64_t body;
  int32_t err;
  if (!fp) return KFMI_E_OPENING_INDEX_FILE;
  if (fread(hdr, 4, 6, fp) != 6) { fclose(fp); return KFMI_E_READING_FMI; }
  if (required_tag && hdr[0] != required_tag) { fclose(fp); return (int32_t) required_tag; }
  steps = hdr[1];
  if (!valid_geometry(hdr[0], steps, hdr[5], hdr[3])) { fclose(fp); return KFMI_E_READING_FMI; }
  if (fread(hdr + 6, 4, 2 * steps, fp) != 2 * steps || !consistent_header(hdr)) {
    fclose(fp);
    return KFMI_E_READING_FMI;
  }
  err = kfmi_index_alloc(hdr[0], steps, hdr[2], hdr[4], hdr[5], hdr + 6, hdr + 6 + steps, &f);
  if (err) { fclose(fp); return err; }
  hb = f->header_bytes;
  ew = f->entry_words;
  body = 4ull * ew * f->nentries;
  (void) hb;
  if (fread(f->h_index, 1, body, fp) != body) {
    fclose(fp); kfmi_big_free(f->image); pthread_rwlock_destroy(&f->rw); free(f); return KFMI_E_READING_FMI;
  }
  fclose(fp);
  snprintf(f->src_name, sizeof(f->src_name), "%s", fn);
  *index = f;
  return KFMI_SUCCESS;
}

int32_t kfmi_load_index_tag(const char *fn, uint32_t required_tag, void **index)
{
  return load_file(fn, required_tag, index);
}

/* interface.h:27.  Any tag, unless KFMI_STRICT_TAG=1 asks for the reference
 * behaviour of the selected backend. */
int32_t loadIndex(const char *fn, void **index)
{
  const char *st = getenv("KFMI_STRICT_TAG");
  uint32_t req = (st && atoi(st)) ? kfmi_backend_tag(kfmi_backend()) : 0;
  return load_file(fn, req, index);
}

int32_t kfmi_index_image(void *index, const void **image, uint64_t *bytes)
{
  kfmi_fmi_t *f = (kfmi_fmi_t *) index;
  int32_t err;
  if (!f || !f->image) return KFMI_E_BAD_ARGUMENT;
  if ((err = kfmi_host_entries(f)) != KFMI_SUCCESS) return err;
  refresh_header(f);
  *image = f->image;
  *bytes = f->image_bytes;
  return KFMI_SUCCESS;
}

int32_t kfmi_index_header(void *index, uint32_t *out)
{
  kfmi_fmi_t *f = (kfmi_fmi_t *) index;
  uint32_t s;
  if (!f) return KFMI_E_BAD_ARGUMENT;
  memset(out, 0, 14 * sizeof(uint32_t));
  out[0] = f->tag; out[1] = f->steps; out[2] = f->bwtsize;
  out[3] = f->ncounters; out[4] = f->nentries; out[5] = f->chunk;
  for (s = 0; s < f->steps; s++) { out[6 + s] = f->dollarPositionBWT[s]; out[10 + s] = f->dollarBaseBWT[s]; }
  return KFMI_SUCCESS;
}

/* genFMindex.c:155-181 naming for tag 100 ("<fn>.<n>.<d>fmi<K>steps.fmi"),
 * the transforms' naming for the others (transformIndexBitmaps.c:96-123,
 * transformIndexAlternateCounters.c saveIndexCPU/GPU). */
int32_t saveIndex(const char *fn, void *index)
{
  kfmi_fmi_t *f = (kfmi_fmi_t *) index;
  char name[1024];
  FILE *fp;
  if (!f) return KFMI_E_BAD_ARGUMENT;
  if (kfmi_host_entries(f) != KFMI_SUCCESS) return KFMI_E_SAVING_INDEX_FILE;
  switch (f->tag) {
    case 100: snprintf(name, sizeof(name), "%s.%u.%ufmi%usteps.fmi", fn, f->bwtsize - 1, f->chunk, f->steps); break;
    case 101: snprintf(name, sizeof(name), "%s.interleaving", fn); break;
    case 200: snprintf(name, sizeof(name), "%s.ac", fn); break;
    default:  snprintf(name, sizeof(name), "%s.interleaving.ac", fn); break;
  }
  refresh_header(f);
  fp = fopen(name, "wb");
  if (!fp) return KFMI_E_SAVING_INDEX_FILE;
  if (fwrite(f->image, 1, f->image_bytes, fp) != f->image_bytes) { fclose(fp); return KFMI_E_SAVING_INDEX_FILE; }
  fclose(fp);
  return KFMI_SUCCESS;
}

/* fmIndexCPUBaseline.c:145-155; also releases device copies and the handle. */
int32_t freeIndex(void **index)
{
  kfmi_fmi_t *f = index ? (kfmi_fmi_t *) *index : NULL;
  if (!f) return KFMI_SUCCESS;
  if (f->dev || f->grp) freeIndexGPU(index);
  if (f->d_entries) kfmi_free_dev_entries(f);
  free(f->h_sa);
  kfmi_big_free(f->image);
  kfmi_big_free(f->image_retired);
  pthread_rwlock_destroy(&f->rw);
  free(f);
  *index = NULL;
  return KFMI_SUCCESS;
}

/* ----------------------------------------------------------------------- */
/* sampled suffix array (locate; not in the reference)      */
/* File: u32 magic "KSA1", rate, bwtsize, 0; u64 count; u32 samples[count]. */
/* ----------------------------------------------------------------------- */

#define KFMI_SA_MAGIC 0x3141534Bu   /* "KSA1" little-endian */

int kfmi_sa_rate_ok(uint32_t rate)
{
  return rate != 0 && (rate & (rate - 1)) == 0 && rate <= (1u << 16);
}

int32_t kfmi_sa_alloc(kfmi_fmi_t *f, uint32_t rate)
{
  uint64_t count;
  if (!f || !kfmi_sa_rate_ok(rate)) return KFMI_E_BAD_ARGUMENT;
  count = ((uint64_t) f->bwtsize + rate - 1) / rate;
  free(f->h_sa);
  f->h_sa = (uint32_t *) malloc(4 * count + 4);
  f->sa_gen++;
  if (!f->h_sa) { f->sa_rate = 0; f->sa_count = 0; return KFMI_E_ALLOCATING_FMI; }
  f->sa_rate = rate;
  f->sa_count = count;
  return KFMI_SUCCESS;
}

int32_t kfmi_index_sa(void *index, const uint32_t **sa, uint64_t *count, uint32_t *rate)
{
  kfmi_fmi_t *f = (kfmi_fmi_t *) index;
  if (!f) return KFMI_E_BAD_ARGUMENT;
  if (sa) *sa = f->h_sa;
  if (count) *count = f->h_sa ? f->sa_count : 0;
  if (rate) *rate = f->h_sa ? f->sa_rate : 0;
  return KFMI_SUCCESS;
}

int32_t kfmi_save_sa(const char *fn, void *index)
{
  kfmi_fmi_t *f = (kfmi_fmi_t *) index;
  uint32_t h[4];
  FILE *fp;
  if (!f || !fn || !f->h_sa) return KFMI_E_BAD_ARGUMENT;
  h[0] = KFMI_SA_MAGIC; h[1] = f->sa_rate; h[2] = f->bwtsize; h[3] = 0;
  fp = fopen(fn, "wb");
  if (!fp) return KFMI_E_SAVING_INDEX_FILE;
  if (fwrite(h, 4, 4, fp) != 4 || fwrite(&f->sa_count, 8, 1, fp) != 1 ||
      fwrite(f->h_sa, 4, f->sa_count, fp) != f->sa_count) {
    fclose(fp);
    return KFMI_E_SAVING_INDEX_FILE;
  }
  fclose(fp);
  return KFMI_SUCCESS;
}

/* Attaches the samples of `fn` to an index of the same text (bwtsize checked). */
int32_t kfmi_load_sa(const char *fn, void *index)
{
  kfmi_fmi_t *f = (kfmi_fmi_t *) index;
  uint32_t h[4];
  uint64_t count;
  int32_t err;
  FILE *fp;
  if (!f || !fn) return KFMI_E_BAD_ARGUMENT;
  fp = fopen(fn, "rb");
  if (!fp) return KFMI_E_OPENING_INDEX_FILE;
  if (fread(h, 4, 4, fp) != 4 || fread(&count, 8, 1, fp) != 1 || h[0] != KFMI_SA_MAGIC ||
      !kfmi_sa_rate_ok(h[1]) || h[2] != f->bwtsize || count != ((uint64_t) f->bwtsize + h[1] - 1) / h[1]) {
    fclose(fp);
    return KFMI_E_READING_FMI;
  }
  err = kfmi_sa_alloc(f, h[1]);
  if (err) { fclose(fp); return err; }
  if (fread(f->h_sa, 4, count, fp) != count) {
    free(f->h_sa); f->h_sa = NULL; f->sa_rate = 0; f->sa_count = 0;
    fclose(fp);
    return KFMI_E_READING_FMI;
  }
  fclose(fp);
  return KFMI_SUCCESS;
}

/* ----------------------------------------------------------------------- */
/* transforms                                                              */
/* ----------------------------------------------------------------------- */

/* tag 100 -> 101: transformIndexBitmaps.c:269-295 */
int32_t kfmi_transform_interleave(void *index100, void **index101)
{
  kfmi_fmi_t *f = (kfmi_fmi_t *) index100, *g;
  uint32_t nb, K, i, w, s, t, c, nbw;
  int32_t err;
  if (!f || f->tag != 100) return KFMI_INDEX_VER_BASELINE;
  if ((err = kfmi_host_entries(f)) != KFMI_SUCCESS) return err;
  err = kfmi_index_alloc(101, f->steps, f->bwtsize, f->nentries, f->chunk,
                         f->dollarPositionBWT, f->dollarBaseBWT, &g);
  if (err) return err;
  nb = f->nbitmaps; K = f->steps; nbw = 2 * nb * K;
  for (i = 0; i < f->nentries; i++) {
    const uint32_t *src = f->h_index + (uint64_t) i * f->entry_words;
    uint32_t *dst = g->h_index + (uint64_t) i * g->entry_words;
    for (w = 0; w < nb; w++)
      for (s = 0; s < K; s++)
        for (t = 0; t < 2; t++)
          dst[kfmi_plane_index(101, K, nb, s, t, w)] = src[kfmi_plane_index(100, K, nb, s, t, w)];
    for (c = 0; c < f->ncounters; c++) dst[nbw + c] = src[nbw + c];
  }
  *index101 = g;
  return KFMI_SUCCESS;
}

/* countEntry, transformIndexAlternateCounters.c:91-127: rows of `code` among
 * the first `position` rows of a tag-100 entry, read from the bit planes (a
 * '$' row counts as its stored code, padding as A). */
static uint32_t count_entry100(const kfmi_fmi_t *f, uint32_t entry, uint32_t code, int32_t position)
{
  const uint32_t *e = f->h_index + (uint64_t) entry * f->entry_words;
  uint32_t n, s, cnt = 0, nb = f->nbitmaps;
  for (n = 0; n < nb; n++) {
    uint32_t m = position >= 32 ? 0xFFFFFFFFu : position > 0 ? 0xFFFFFFFFu << (32 - position) : 0u;
    for (s = 0; s < f->steps; s++) {
      uint32_t cs = (code >> (2 * s)) & 3u;
      uint32_t b0 = e[kfmi_plane_index(f->tag, f->steps, nb, s, 0, n)];   /* tag 100 or 101 */
      uint32_t b1 = e[kfmi_plane_index(f->tag, f->steps, nb, s, 1, n)];
      m &= ((cs & 1u) ? b0 : ~b0) & ((cs & 2u) ? b1 : ~b1);
    }
    cnt += (uint32_t) __builtin_popcount(m);
    position -= 32;
  }
  return cnt;
}

/* The counters the AltCounters searcher reads past the last real block:
 * entry E-1 (its plain counters), the sentinel E (the last entry's counters
 * plus its first (n+1) mod d rows counted from the bit planes plus the padding
 * rows for code 0, transformIndexAlternateCounters.c:420-431, exactly as
 * kfmi_transform_ac below) and E+1 (zero, as the AC device layout's padding).
 * All NC codes; the searcher only reads the half each entry's parity keeps. */
int32_t kfmi_ac_tail(const kfmi_fmi_t *f, uint32_t *out, uint32_t *first)
{
  uint32_t c, nc, nbw, rem, last;
  const uint32_t *src;
  if (!f || !out || (f->tag != 100 && f->tag != 101) || !f->nentries) return KFMI_E_BAD_ARGUMENT;
  /* a device-resident index fetches its host image on demand (a cache owned by the handle) */
  if (kfmi_host_entries((kfmi_fmi_t *) f) != KFMI_SUCCESS) return KFMI_E_NOT_ON_DEVICE;
  nc = f->ncounters;
  nbw = 2 * f->nbitmaps * f->steps;
  last = f->nentries;
  rem = f->bwtsize % f->chunk;
  src = f->h_index + (uint64_t) (last - 1) * f->entry_words;
  for (c = 0; c < nc; c++) {
    out[c] = src[nbw + c];
    out[nc + c] = src[nbw + c] + (c == 0 ? f->chunk - rem : 0u) +
                  (rem ? count_entry100(f, f->bwtsize / f->chunk, c, (int32_t) rem) : 0u);
    out[2 * nc + c] = 0;
  }
  if (first) *first = last - 1;
  return KFMI_SUCCESS;
}

/* tag 100 -> 200 and 201: transformIndexAlternateCounters.c:387-479.
 * Even entries keep cnt[0..NC/2), odd entries cnt[NC/2..NC); one sentinel
 * entry with zero bitmaps is appended whose counters are the last entry's
 * plus a count of its first (n+1) mod d rows from the bit planes, plus the
 * padding rows for code 0.  (n+1) mod d == 0 reads past the end in the
 * reference (B5); here the partial count is 0, the value the masked read
 * yields there. */
int32_t kfmi_transform_ac(void *index100, void **index200, void **index201)
{
  kfmi_fmi_t *f = (kfmi_fmi_t *) index100, *g[2] = {NULL, NULL};
  uint32_t nb, K, nc, half, i, s, t, w, c, nbw, last, rem;
  uint32_t *lastCnt;
  int32_t err, v;
  if (!f || f->tag != 100) return KFMI_INDEX_VER_BASELINE;
  if ((err = kfmi_host_entries(f)) != KFMI_SUCCESS) return err;
  nb = f->nbitmaps; K = f->steps; nc = f->ncounters; half = nc / 2; nbw = 2 * nb * K;
  last = f->nentries;          /* index of the sentinel entry */
  rem = f->bwtsize % f->chunk;
  lastCnt = (uint32_t *) calloc(nc, sizeof(uint32_t));
  if (!lastCnt) return KFMI_E_ALLOCATING_FMI;
  lastCnt[0] += f->chunk - rem;
  for (c = 0; c < nc; c++)
    lastCnt[c] += rem ? count_entry100(f, f->bwtsize / f->chunk, c, (int32_t) rem) : 0;
  for (v = 0; v < 2; v++) {
    uint32_t tag = v ? 201 : 200;
    err = kfmi_index_alloc(tag, K, f->bwtsize, f->nentries + 1, f->chunk,
                           f->dollarPositionBWT, f->dollarBaseBWT, &g[v]);
    if (err) { free(lastCnt); if (v) freeIndex((void **) &g[0]); return err; }
    for (i = 0; i < last; i++) {
      const uint32_t *src = f->h_index + (uint64_t) i * f->entry_words;
      uint32_t *dst = g[v]->h_index + (uint64_t) i * g[v]->entry_words;
      for (w = 0; w < nb; w++)
        for (s = 0; s < K; s++)
          for (t = 0; t < 2; t++)
            dst[half + kfmi_plane_index(tag, K, nb, s, t, w)] = src[kfmi_plane_index(100, K, nb, s, t, w)];
      for (c = 0; c < half; c++) dst[c] = src[nbw + (i & 1u) * half + c];
    }
    {
      const uint32_t *src = f->h_index + (uint64_t) (last - 1) * f->entry_words;
      uint32_t *dst = g[v]->h_index + (uint64_t) last * g[v]->entry_words;
      uint32_t off = (last & 1u) * half;
      for (c = 0; c < half; c++) dst[c] = src[nbw + off + c] + lastCnt[off + c];
      /* bitmaps of the sentinel stay zero (calloc) */
    }
  }
  free(lastCnt);
  if (index200) *index200 = g[0]; else freeIndex((void **) &g[0]);
  if (index201) *index201 = g[1]; else freeIndex((void **) &g[1]);
  return KFMI_SUCCESS;
}

/* tag 200 / 201 -> 100: kfmi_transform_ac undone, so that an AltCounters file
 * (the input of the reference's -AC searchers) feeds the layouts built from
 * plain counters.  Entry i keeps cnt_i of its parity's half; the other half
 * is the next entry's (cnt_{i+1}) less block i's rows of each code -- every
 * row read from the planes, a '$' row once however many D_s share it, as the
 * plain counters exclude it -- and, for the last real entry E-1, the
 * sentinel's less exactly what the transform added to it (its first
 * (n+1) mod d rows from the planes, the padding rows as code 0).  Byte-equal
 * to the tag-100 file the transform was run on (tests/test_host.py). */
int32_t kfmi_transform_plain(void *index_ac, void **index100)
{
  kfmi_fmi_t *f = (kfmi_fmi_t *) index_ac, *g;
  uint32_t nb, K, nc, half, i, s, t, w, c, nbw, last, rem, j, k;
  int32_t err;
  if (!f || !index100 || (f->tag != 200 && f->tag != 201)) return KFMI_INDEX_VER_BASELINE_AC;
  if (f->nentries < 2) return KFMI_E_READING_FMI;
  if ((err = kfmi_host_entries(f)) != KFMI_SUCCESS) return err;
  nb = f->nbitmaps; K = f->steps; nc = 1u << (2 * K); half = nc / 2; nbw = 2 * nb * K;
  if (f->ncounters != half) return KFMI_E_READING_FMI;
  last = f->nentries - 1;      /* the sentinel */
  rem = f->bwtsize % f->chunk;
  err = kfmi_index_alloc(100, K, f->bwtsize, last, f->chunk, f->dollarPositionBWT, f->dollarBaseBWT, &g);
  if (err) return err;
  for (i = 0; i < last; i++) {   /* planes and the stored half */
    const uint32_t *src = f->h_index + (uint64_t) i * f->entry_words;
    uint32_t *dst = g->h_index + (uint64_t) i * g->entry_words;
    for (w = 0; w < nb; w++)
      for (s = 0; s < K; s++)
        for (t = 0; t < 2; t++)
          dst[kfmi_plane_index(100, K, nb, s, t, w)] = src[half + kfmi_plane_index(f->tag, K, nb, s, t, w)];
    for (c = 0; c < half; c++) dst[nbw + (i & 1u) * half + c] = src[c];
  }
  for (i = 0; i < last; i++) {   /* the other half, from entry i+1 (or the sentinel) */
    const uint32_t off = ((i + 1) & 1u) * half;
    const uint32_t *nxt = f->h_index + (uint64_t) (i + 1) * f->entry_words;
    uint32_t *dst = g->h_index + (uint64_t) i * g->entry_words;
    for (c = 0; c < half; c++) {
      const uint32_t code = off + c;
      uint32_t sub;
      if (i + 1 < last) {
        sub = count_entry100(g, i, code, (int32_t) f->chunk);
        for (j = 0; j < K; j++) {   /* '$' rows of block i with this stored code, each row once */
          const uint32_t p = f->dollarPositionBWT[j];
          int seen = 0;
          for (k = 0; k < j; k++) seen |= f->dollarPositionBWT[k] == p;
          if (!seen && p / f->chunk == i && count_entry100(g, i, code, (int32_t) (p % f->chunk) + 1) !=
                                                   count_entry100(g, i, code, (int32_t) (p % f->chunk)))
            sub--;
        }
      } else {
        sub = (code == 0 ? f->chunk - rem : 0u) + (rem ? count_entry100(g, f->bwtsize / f->chunk, code, (int32_t) rem) : 0u);
      }
      dst[nbw + code] = nxt[c] - sub;
    }
  }
  *index100 = g;
  return KFMI_SUCCESS;
}
