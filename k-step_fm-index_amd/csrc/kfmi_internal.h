/*
 * kfmi_internal.h -- host structures shared by the C host layer (csrc/host)
 * and the HIP layer (csrc/hip).  Not part of the public ABI: callers only
 * see opaque `void *` handles (include/kstep_fmi.h).
 *
 * Field meanings follow the reference handles (fmIndexCPUBaseline.c:54-69,
 * common.h:64-81) with 64-bit sizes where the reference overflows (B7).
 */
#ifndef KFMI_INTERNAL_H_
#define KFMI_INTERNAL_H_

#include <stdint.h>
#include <stddef.h>
#include <pthread.h>
#include "../../include/kstep_fmi.h"

#ifdef __cplusplus
extern "C" {
#endif

#define KFMI_MAX_STEPS 4

struct kfmi_dev_index;   /* device-resident layouts, defined in csrc/hip */
struct kfmi_dev_queries;

typedef struct {
  /* header, genFMindex.c:167-178 */
  uint32_t tag, steps, bwtsize, ncounters, nentries, chunk;
  uint32_t dollarPositionBWT[KFMI_MAX_STEPS];
  uint32_t dollarBaseBWT[KFMI_MAX_STEPS];
  uint32_t modposdollarBWT[KFMI_MAX_STEPS];   /* = dollarPositionBWT / chunk */
  uint32_t nbitmaps;       /* 32-bit words per bit-plane row = chunk / 32 */
  uint32_t entry_words;    /* u32 words per entry for this tag */
  /* file image: header followed by nentries entries, one allocation */
  uint8_t  *image;
  uint64_t  image_bytes;
  uint8_t  *image_retired; /* the header-only image an on-demand fetch replaced (kfmi_host_entries):
                              kept until freeIndex, so a reader holding it never sees it freed */
  uint32_t  header_bytes;
  uint32_t *h_index;       /* = (uint32_t *)(image + header_bytes), may be unaligned to 16;
                              NULL while the entries live only on the device (d_entries) */
  /* entries of an index built on the device without a host image
   * (kfmi_build_index_gpu, want_host_image = 0): uploads relayout them on the
   * device; the host image is fetched only when something asks for it
   * (kfmi_host_entries).  Owned by the handle, freed by freeIndex. */
  uint32_t *d_entries;
  int       d_entries_dev;
  struct kfmi_dev_index *dev;
  char      src_name[512]; /* file the index came from (for saveIndex/saveResults naming) */
  /* row-sampled suffix array for locate (not in the reference):
   * h_sa[i] = SA[i * sa_rate] for i < sa_count = ceil(bwtsize / sa_rate);
   * sa_rate 0 = none, else a power of two (1 = the full SA).  sa_gen changes
   * whenever the samples do, so a stale device copy is re-uploaded. */
  uint32_t  sa_rate;
  uint32_t  sa_gen;
  uint64_t  sa_count;
  uint32_t *h_sa;
  void     *grp;           /* replicas on a device group (KFMI_DEVICES, kfmi_set_devices) */
  /* guards dev / grp (kfmi_runtime.h index_lock): searches hold it shared,
   * uploads that replace the device copy and freeIndexGPU exclusively;
   * writer-preferring, one per handle (so unrelated handles never wait on
   * each other); initialised by kfmi_index_alloc_ex, destroyed by freeIndex */
  pthread_rwlock_t rw;
} kfmi_fmi_t;

typedef struct {
  uint64_t num;
  uint32_t size;
  char    *h_queries;      /* num*size ASCII, query q at q*size (plain layout) */
  struct kfmi_dev_queries *dev;
  void    *grp;            /* per-device slices on a device group */
} kfmi_qrys_t;

typedef struct {
  uint64_t  num;
  uint32_t *h_results;     /* 2*num: [L0,R0,L1,R1,...] */
  uint32_t *d_results;     /* device copy (hipMalloc), NULL until transfer */
  int32_t   d_device;      /* device holding d_results (valid while d_results != NULL) */
  void     *grp;           /* per-device slices on a device group */
  int32_t   origin;        /* who wrote h_results last: KFMI_RES_FROM_GPU (transferGPUtoCPU) or
                              KFMI_RES_FROM_CPU (searchIndexCPU); saveResults names the file by it */
} kfmi_res_t;
enum { KFMI_RES_FROM_GPU = 0, KFMI_RES_FROM_CPU = 1 };

/* CPUs this process may use: the affinity mask capped by the cgroup quota (common.c) */
int32_t kfmi_process_cpus(void);
/* Index images, query and result buffers: zeroed buffers that, from 64 MB,
 * are 2 MB-aligned anonymous mappings marked MADV_HUGEPAGE (the host search's
 * random LFs walk 2 MB pages; first touches fault 512x less often);
 * kfmi_big_free releases either kind (common.c). */
void *kfmi_big_alloc(uint64_t bytes);
void kfmi_big_free(void *p);

typedef struct {
  uint64_t size;
  char    *h_reference;
} kfmi_ref_t;

/* fmi_index.c */
/* Host entries of an index whose entries are only on the device (fetched once,
 * then kept); KFMI_SUCCESS at once when the host image exists (kfmi_build.hip). */
int32_t kfmi_host_entries(kfmi_fmi_t *f);
void kfmi_free_dev_entries(kfmi_fmi_t *f);
int32_t kfmi_index_alloc(uint32_t tag, uint32_t steps, uint32_t bwtsize, uint32_t nentries,
                         uint32_t chunk, const uint32_t *dpos, const uint32_t *dbase,
                         kfmi_fmi_t **out);
int32_t kfmi_index_alloc_ex(uint32_t tag, uint32_t steps, uint32_t bwtsize, uint32_t nentries,
                            uint32_t chunk, const uint32_t *dpos, const uint32_t *dbase,
                            int with_entries, kfmi_fmi_t **out);
uint32_t kfmi_entry_words(uint32_t tag, uint32_t steps, uint32_t chunk);
uint32_t kfmi_plane_index(uint32_t tag, uint32_t steps, uint32_t nb, uint32_t s, uint32_t t, uint32_t w);

/* backend registry, fmi_backend.c */
typedef enum {
  KFMI_BK_TASK = 0, KFMI_BK_COOP, KFMI_BK_TASK_AC, KFMI_BK_COOP_AC,
  KFMI_BK_TASK_MID, KFMI_BK_COOP_MID, KFMI_BK_TASK_AC_MID, KFMI_BK_COOP_AC_MID,
  KFMI_BK_TASK_GRP, KFMI_BK_COOP_GRP, KFMI_BK_COUNT   /* packed and ac128 retired in round 6 */
} kfmi_backend_t;
kfmi_backend_t kfmi_backend(void);
uint32_t       kfmi_backend_tag(kfmi_backend_t b);   /* 101 or 201 */
int32_t        kfmi_current_device(void);
void           kfmi_set_last_error(int32_t e);

/* AltCounters tail of a tag-100/101 index (fmi_index.c): out[3 * NC] = the
 * tag-201 counters of entries E-1, E (the tfmiAC sentinel) and E+1 (zero) for
 * every code, E = nentries; *first = E-1 */
int32_t kfmi_ac_tail(const kfmi_fmi_t *f, uint32_t *out, uint32_t *first);

/* sampled suffix array (fmi_index.c): (re)allocates h_sa for `rate` */
int32_t kfmi_sa_alloc(kfmi_fmi_t *f, uint32_t rate);

/* qpack.c: ASCII rows -> word-major 2-bit code words (word w of row q at
 * out[w * ostride + q]; ceil(m/16) words per row) */
void kfmi_pack_rows(const uint8_t *ascii, uint64_t n, uint32_t m, uint32_t *out, uint64_t ostride);
/* the same for reads whose last rem = m % K bases come from the remainder table:
 * the stream of bases 0 .. m-rem-1, then one word row of remainder codes */
void kfmi_pack_rows_rem(const uint8_t *ascii, uint64_t n, uint32_t m, uint32_t rem, uint32_t *out,
                        uint64_t ostride);
int     kfmi_sa_rate_ok(uint32_t rate);

/* builders with SA sampling (fmi_build.c, kfmi_build.hip) */
int32_t kfmi_build_index_cpu_sa(const char *text, uint64_t n, uint32_t k, uint32_t d, uint32_t sa_rate,
                                void **index);
int32_t kfmi_build_index_gpu_sa(const char *text, uint64_t n, uint32_t k, uint32_t d, uint32_t sa_rate,
                                void **index);

/* alphabet modes of the builders (fmi_build.c; KFMI_ALPHABET / kfmi_set_alphabet) */
enum { KFMI_ALPHA_ACGT = 0, KFMI_ALPHA_MAP = 1, KFMI_ALPHA_REF = 2 };
int     kfmi_alphabet_mode(void);
int32_t kfmi_index_ref_walk(const char *text, const uint32_t *sa, uint64_t n, uint32_t k, uint32_t d,
                            kfmi_fmi_t **out);

/* suffix array construction, fmi_build.c */
int32_t kfmi_sais(const uint8_t *text_codes, uint32_t *sa, uint32_t n, uint32_t alpha);
int32_t kfmi_index_from_sa(const uint8_t *codes, const uint32_t *sa, uint64_t n,
                           uint32_t k, uint32_t d, kfmi_fmi_t **out);

#ifdef __cplusplus
}
#endif

#endif /* KFMI_INTERNAL_H_ */
