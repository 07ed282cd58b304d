/*
 * kfmi_runtime.h -- host-side runtime shared by the library's translation
 * units: kfmi_search.hip (backends, devices, uploads, the reference's entry
 * points), kfmi_group.hip (device groups), kfmi_locate.hip (locate) and
 * kfmi_stream.hip (streamed search, host worker pool).
 */
#ifndef KFMI_RUNTIME_H_
#define KFMI_RUNTIME_H_

#include <hip/hip_runtime.h>
#include <atomic>
#include <stdint.h>
#include <stdio.h>
#include <mutex>
#include <shared_mutex>
#include <pthread.h>

#include "../kfmi_internal.h"
#include "kfmi_devguard.h"
#include "kfmi_kernels.h"

#define HIP_OK(x)                                                                   \
  do {                                                                              \
    hipError_t _e = (x);                                                            \
    if (_e != hipSuccess) {                                                         \
      fprintf(stderr, "kstepfmi: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(_e), \
              __FILE__, __LINE__);                                                  \
      return KFMI_E_KERNEL;                                                         \
    }                                                                               \
  } while (0)

/* ------------------------------------------------------------------------ */
/* device-side handles                                                      */
/* ------------------------------------------------------------------------ */

struct kfmi_dev_index {
  int device = -1;
  int backend = -1;
  int layout = -1;
  uint32_t K = 0, d = 0, nb = 0, bwtsize = 0, nentries = 0;
  kfmi::DollarArgs dl{};
  uint32_t* ent = nullptr;     /* device entries */
  uint64_t ent_bytes = 0;
  uint32_t* sa = nullptr;      /* locate: row-sampled suffix array */
  /* every LF_K walk ends at a '$' row (check_lf_walks), checked once before
   * the first locate walk or derivation: -1 not yet, 0 no (refused), 1 yes */
  std::atomic<int> lf_perm{-1};
  uint64_t sa_bytes = 0;
  uint32_t sa_log2 = 0, sa_gen = 0;
  /* jump-start tables, one per base count (built on first use, then immutable
   * until the index leaves the device, so concurrent searches with different
   * kfmi_set_ftab values never free a table another kernel reads) */
  uint2* ftab[17] = {};
  std::mutex ftab_mu;
  /* remainder tables: [L, R) of every r-base read suffix, r = m % K in 1..3
   * (same lifetime rule as the ftabs, same mutex) */
  uint2* rtab[4] = {};
  uint32_t* ac_tail = nullptr; /* AltCounters layouts, 4 x NC: (LAY_MIDAC) the counters of entries E-1, E,
                                 E+1; row 3 the locate walk's sentinel correction (ac_locate_fix) */
  uint32_t ac_tail_b0 = 0xFFFFFFFFu;
};

struct kfmi_dev_queries {
  int device = -1;
  uint8_t* ascii = nullptr;    /* num*size bytes, plain layout; null when the host packed the
                                  reads on upload (`packed` is then already valid) */
  uint32_t* packed = nullptr;  /* (nwords + 1) x num u32 codes; row nwords: remainder codes */
  uint64_t num = 0;
  /* m = size = rem + K * steps: the last rem (< K) bases of a read are resolved
   * by one remainder-table lookup before its K-steps (query_geometry) */
  uint32_t size = 0, K = 0, steps = 0, nwords = 0, rem = 0;
  uint32_t packed_rows = 0;    /* rows allocated in `packed` (>= nwords + 1) */
};

namespace kfmi {

/* Guards the device copies of one index handle (f->dev, f->grp): searches,
 * locates, block counts and streamed searches hold it shared for as long as
 * they use the device copy; an upload that replaces it (another backend or
 * device, a new device group) or freeIndexGPU holds it exclusively, so a
 * search running on another thread never sees its tables freed.  One
 * writer-preferring lock per handle (kfmi_fmi_t::rw), so a writer is not
 * starved by a stream of searches and unrelated handles never wait on each
 * other.  RwLock is that pthread lock seen as a SharedMutex. */
struct RwLock {
  pthread_rwlock_t rw;
  void lock() { pthread_rwlock_wrlock(&rw); }
  void unlock() { pthread_rwlock_unlock(&rw); }
  bool try_lock() { return pthread_rwlock_trywrlock(&rw) == 0; }
  void lock_shared() { pthread_rwlock_rdlock(&rw); }
  void unlock_shared() { pthread_rwlock_unlock(&rw); }
  bool try_lock_shared() { return pthread_rwlock_tryrdlock(&rw) == 0; }
};
RwLock& index_lock(const void* f);

/* One non-blocking stream per device, shared by the threads that use it (their
 * work is serialised on it).  Timing events are per calling thread. */
struct DevCtx {
  bool init = false;
  hipStream_t st = nullptr;
  /* pinned chunk buffers of host-packed query uploads (upload_queries) and of
   * device-parsed FASTA loads (fa_upload), kept between calls.  One user at a
   * time per device holds up_mu for its whole pass -- a FASTA load holds it
   * through its file reads too, so a host-packed upload on the same device
   * waits for that load to finish (both are bulk host -> device streams that
   * would share the one link anyway) */
  std::mutex up_mu;
  void* up_buf[2] = {nullptr, nullptr};
  hipEvent_t up_ev[2] = {nullptr, nullptr};
  uint64_t up_cap = 0;
};
void release_upload_staging();   /* kfmi_stream_release */
/* ctx's pinned chunk buffers grown to `need` bytes each (caller holds up_mu) */
hipError_t upload_staging(DevCtx* ctx, uint64_t need);
int32_t ctx_for(int dev, DevCtx** out);   /* selects `dev`, creates its stream once */
/* The calling thread's three timing events on device `dev` (current device). */
hipEvent_t* thread_events(int dev);
/* The calling thread's search stream on device `dev` (current device). */
hipStream_t thread_stream(int dev);

/* per calling thread (kfmi_search.hip) */
extern thread_local int t_device;
extern thread_local int32_t t_last_error;
extern thread_local double t_ms[3];   /* kfmi_last_timing: total, pack, lf (ms) */
uint32_t ftab_bases(void);

/* backends and kernel dispatch (kfmi_search.hip) */
bool is_coop(int backend);
int backend_for(uint32_t K);   /* the selected backend, or coop-grp for K = 4 under the implicit default */
int fused_maxw(int backend, uint32_t bases);   /* bases = K * steps of the batch */
int32_t check_lf_walks(kfmi_dev_index* di, hipStream_t st);   /* sets di->lf_perm (kfmi_search.hip) */
hipError_t dispatch(Op op, uint32_t K, uint32_t nb, int lay, const SearchLaunch& a,
                    unsigned long long* d_total = nullptr);
IdxArgs idx_args(const kfmi_dev_index* di);
int32_t use_ftab(kfmi_dev_index* di, hipStream_t st, IdxArgs& ix, uint32_t bases);
/* reads with m % K = rem != 0: layouts that take the remainder
 * table, and the table of an index (built on first use; clears the ftab) */
bool rem_supported(int layout);
int32_t use_rtab(kfmi_dev_index* di, hipStream_t st, IdxArgs& ix, uint32_t rem);
hipError_t launch_pack(const kfmi_dev_queries* dq, hipStream_t st);

/* uploads (kfmi_search.hip) */
int32_t upload_index(kfmi_fmi_t* f, int backend, int dev, DevCtx* ctx, kfmi_dev_index** out = nullptr);
/* the 2K-step index of a K-step one, derived on `dev` (kfmi_derive.hip) */
int32_t derive_index(kfmi_fmi_t* f, uint32_t k_out, int dev, bool host_image, kfmi_fmi_t** out);
/* K of the handle's device copy (a K = 2 file on the grouped layout searches
 * a derived K = 4 index), else of the file: the K queries are packed for */
uint32_t device_steps(const kfmi_fmi_t* f);
int32_t upload_sa(const kfmi_fmi_t* f, kfmi_dev_index* di, DevCtx* ctx);
int32_t upload_queries(kfmi_qrys_t* q, uint32_t K, int dev, DevCtx* ctx);
void query_geometry(kfmi_dev_queries* dq, uint32_t K);
void free_dev_index(kfmi_dev_index* di);
void free_dev_queries(kfmi_dev_queries* dq);
hipError_t h2d(void* dst, const void* src, uint64_t bytes, hipStream_t st);

/* one device batch: queue pack + LF bracketed by ev[0..2], then wait (kfmi_search.hip) */
int32_t search_enqueue(kfmi_dev_index* di, kfmi_dev_queries* dq, uint32_t* d_res, hipStream_t st, hipEvent_t* ev,
                       uint32_t ftab);
int32_t search_finish(hipStream_t st, hipEvent_t* ev, double* ms);

/* host memory helpers (kfmi_stream.hip) */
bool host_pinned(const void* p);
void par_copy(void* dst, const void* src, uint64_t bytes);
/* n ASCII rows of `size` bases -> word-major 2-bit code words (row stride n;
 * row ceil((size - rem) / 16) holds the remainder codes), over the host workers;
 * K in {1, 2, 4} (qpack.c) */
void par_pack(const char* src, uint64_t n, uint32_t size, uint32_t rem, uint32_t* out);
bool par_pread(int fd, void* dst, uint64_t off, uint64_t bytes);

/* device groups (kfmi_group.hip) */
constexpr int KFMI_MAX_GROUP = 16;
struct GroupIndex {
  int n = 0, backend = -1;
  int dev[KFMI_MAX_GROUP] = {};
  kfmi_dev_index* di[KFMI_MAX_GROUP] = {};
  hipStream_t st[KFMI_MAX_GROUP] = {};
  hipEvent_t ev[KFMI_MAX_GROUP][3] = {};
};

/* queries or results of a group: one contiguous slice per member */
struct GroupSlices {
  int n = 0;
  int dev[KFMI_MAX_GROUP] = {};
  uint64_t q0[KFMI_MAX_GROUP] = {}, num[KFMI_MAX_GROUP] = {};
  kfmi_dev_queries* dq[KFMI_MAX_GROUP] = {};
  uint32_t* d_res[KFMI_MAX_GROUP] = {};
};
int group_devices(int* devs);   /* the KFMI_DEVICES / kfmi_set_devices list */
int32_t group_transfer(kfmi_fmi_t* f, kfmi_qrys_t* q, kfmi_res_t* r, const int* devs, int n);
int32_t group_search(kfmi_fmi_t* f, kfmi_qrys_t* q, kfmi_res_t* r);
int32_t group_to_host(kfmi_res_t* r);
void group_free_index(kfmi_fmi_t* f);
void group_free_queries(kfmi_qrys_t* q);
void group_free_results(kfmi_res_t* r);

}  // namespace kfmi

#endif  // KFMI_RUNTIME_H_
