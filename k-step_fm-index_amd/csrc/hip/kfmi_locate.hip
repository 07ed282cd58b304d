/*
 * kfmi_locate.hip -- locate: the [L, R) of every query to
 * text positions via the row-sampled suffix array: per-query counts, an
 * exclusive scan for the offsets, slot owners by a max-scan, then the LF_K
 * walk of kfmi_locate.h (locate_kernel) to a sampled or '$' row.
 */
#include <stdlib.h>
#include <string.h>
#include <new>
#include <rocprim/device/device_scan.hpp>

#include "kfmi_runtime.h"

struct kfmi_locations {
  uint64_t num = 0, total = 0;
  uint64_t* h_off = nullptr;   /* num + 1 */
  uint32_t* h_pos = nullptr;   /* total */
};

namespace kfmi {

/* locate bookkeeping kernels (slot counts, owners, first rows); the walk itself
 * is locate_kernel in kfmi_locate.h */
// Positions each query reports: min(min(R, n+1) - L, max_occ) (max_occ 0 =
// all; rows from n+1 on hold no suffix -- an AltCounters interval can reach
// past the sentinel, §3).  The count array has num + 1 slots and the last one
// is 0, so the exclusive scan's last element is the total.
static __global__ __launch_bounds__(256) void loc_count_kernel(const uint32_t* __restrict__ res, uint64_t num,
                                                        uint32_t max_occ, uint32_t nrows,
                                                        uint64_t* __restrict__ cnt)
{
  const uint64_t q = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (q > num) return;
  uint64_t c = 0;
  if (q < num) {
    const uint2 lr = *reinterpret_cast<const uint2*>(res + 2 * q);
    const uint32_t hi = lr.y < nrows ? lr.y : nrows;
    c = hi > lr.x ? (uint64_t) (hi - lr.x) : 0u;
    if (max_occ && c > max_occ) c = max_occ;
  }
  cnt[q] = c;
}

// Owner of each output slot without a per-slot search: every query with at
// least one position writes its id at its first slot (owner[] zeroed first),
// and an inclusive max-scan spreads it over the query's slots.
static __global__ __launch_bounds__(256) void loc_heads_kernel(const uint64_t* __restrict__ cnt,
                                                        const uint64_t* __restrict__ off, uint64_t num,
                                                        uint32_t* __restrict__ owner)
{
  const uint64_t q = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (q < num && cnt[q]) owner[off[q]] = (uint32_t) q;
}

// First row of every output slot, in place over the owner array:
// rows[i] = L of its query + the slot's rank inside the query.
static __global__ __launch_bounds__(256) void loc_rows_kernel(const uint32_t* __restrict__ res,
                                                       const uint64_t* __restrict__ off, uint64_t total,
                                                       uint32_t* __restrict__ own_rows)
{
  for (uint64_t i = (uint64_t) blockIdx.x * 256 + threadIdx.x; i < total; i += (uint64_t) gridDim.x * 256) {
    const uint32_t q = own_rows[i];   /* grid-stride: a batch may hold more than 2^32 positions */
    own_rows[i] = res[2 * (uint64_t) q] + (uint32_t) (i - off[q]);
  }
}

/* ------------------------------------------------------------------------ */
/* locate: [L, R) of every query -> text positions          */
/* ------------------------------------------------------------------------ */


extern "C" int32_t kfmi_locations_free(void** locations)
{
  kfmi_locations* L = locations ? (kfmi_locations*) *locations : nullptr;
  if (L) {   /* host memory only */
    free(L->h_off);
    free(L->h_pos);
    delete L;
    *locations = nullptr;
  }
  return KFMI_SUCCESS;
}

extern "C" uint64_t kfmi_locations_total(void* locations)
{
  return locations ? ((kfmi_locations*) locations)->total : 0;
}

extern "C" const uint64_t* kfmi_locations_offsets(void* locations)
{
  return locations ? ((kfmi_locations*) locations)->h_off : nullptr;
}

extern "C" const uint32_t* kfmi_locations_positions(void* locations)
{
  return locations ? ((kfmi_locations*) locations)->h_pos : nullptr;
}

/* Locate of the `num` results at d_res (device of di) into *locations. */
static int32_t locate_on(kfmi_fmi_t* f, kfmi_dev_index* di, uint32_t* d_res, uint64_t num, uint32_t max_occ,
                         kfmi_locations** locations)
{
  DevCtx* ctx = nullptr;
  int32_t err = ctx_for(di->device, &ctx);
  if (err) return err;
  hipEvent_t* ev = thread_events(di->device);
  if (!ev) return KFMI_E_NO_DEVICE;
  if (!di->sa || di->sa_gen != f->sa_gen) {
    err = upload_sa(f, di, ctx);
    if (err) return err;
  }
  if (di->lf_perm.load() < 0) {   /* once per device copy */
    err = check_lf_walks(di, ctx->st);
    if (err) return err;
  }
  /* an LF_K cycle that misses every '$' row would keep a slot walking for up
   * to n/K dependent loads before walk_lost gives up */
  if (di->lf_perm.load() == 0) return KFMI_E_BUILDING_FMI;
  kfmi_locations* L = new (std::nothrow) kfmi_locations();
  if (!L) return KFMI_E_ALLOCATING_RESULTS;
  L->num = num;
  L->h_off = (uint64_t*) malloc(8 * (num + 1));
  if (!L->h_off) {
    kfmi_locations_free((void**) &L);
    return KFMI_E_ALLOCATING_RESULTS;
  }
  uint64_t *d_cnt = nullptr, *d_off = nullptr;
  uint32_t *d_pos = nullptr, *d_own = nullptr;
  void *tmp = nullptr, *tmp2 = nullptr;
  size_t tb = 0, tb2 = 0;
  uint64_t total = 0;
  auto done = [&](int32_t code) {
    if (d_cnt) (void) hipFree(d_cnt);
    if (d_off) (void) hipFree(d_off);
    if (d_pos) (void) hipFree(d_pos);
    if (d_own) (void) hipFree(d_own);
    if (tmp) (void) hipFree(tmp);
    if (tmp2) (void) hipFree(tmp2);
    if (code) kfmi_locations_free((void**) &L);
    else *locations = L;
    return code;
  };
  const hipStream_t st = ctx->st;
  bool ok = hipMalloc((void**) &d_cnt, 8 * (num + 1)) == hipSuccess &&
            hipMalloc((void**) &d_off, 8 * (num + 1)) == hipSuccess &&
            rocprim::exclusive_scan(nullptr, tb, d_cnt, d_off, (uint64_t) 0, (size_t) (num + 1),
                                    rocprim::plus<uint64_t>(), st) == hipSuccess &&
            hipMalloc(&tmp, tb ? tb : 1) == hipSuccess;
  if (!ok) return done(KFMI_E_DEVICE_ALLOC);
  if (hipEventRecord(ev[0], st) != hipSuccess) return done(KFMI_E_KERNEL);
  hipLaunchKernelGGL(loc_count_kernel, dim3((uint32_t) ((num + 1 + 255) / 256)), dim3(256), 0, st, d_res, num,
                     max_occ, di->bwtsize, d_cnt);
  ok = hipGetLastError() == hipSuccess &&
       rocprim::exclusive_scan(tmp, tb, d_cnt, d_off, (uint64_t) 0, (size_t) (num + 1), rocprim::plus<uint64_t>(),
                               st) == hipSuccess &&
       hipMemcpyAsync(&total, d_off + num, 8, hipMemcpyDeviceToHost, st) == hipSuccess &&
       hipStreamSynchronize(st) == hipSuccess;
  if (!ok) return done(KFMI_E_KERNEL);
  L->total = total;
  L->h_pos = (uint32_t*) malloc(4 * total + 4);
  if (!L->h_pos) return done(KFMI_E_ALLOCATING_RESULTS);
  if (hipMalloc((void**) &d_pos, 4 * total + 4) != hipSuccess ||
      hipMalloc((void**) &d_own, 4 * total + 4) != hipSuccess ||
      rocprim::inclusive_scan(nullptr, tb2, d_pos, d_own, (size_t) total, rocprim::maximum<uint32_t>(), st) !=
          hipSuccess ||
      hipMalloc(&tmp2, tb2 ? tb2 : 1) != hipSuccess)
    return done(KFMI_E_DEVICE_ALLOC);
  if (total) {   /* owner[i] = query of slot i: heads at each query's first slot, then a max-scan */
    if (hipMemsetAsync(d_pos, 0, 4 * total, st) != hipSuccess) return done(KFMI_E_KERNEL);   /* heads in d_pos */
    hipLaunchKernelGGL(loc_heads_kernel, dim3((uint32_t) ((num + 255) / 256)), dim3(256), 0, st, d_cnt, d_off, num,
                       d_pos);
    if (hipGetLastError() != hipSuccess ||
        rocprim::inclusive_scan(tmp2, tb2, d_pos, d_own, (size_t) total, rocprim::maximum<uint32_t>(), st) !=
            hipSuccess)
      return done(KFMI_E_KERNEL);
    const uint64_t rb = (total + 255) / 256;
    hipLaunchKernelGGL(loc_rows_kernel, dim3(grid_blocks(rb, 1u << 20)), dim3(256), 0, st,
                       d_res, d_off, total, d_own);   /* owner -> first row of each slot, in place */
    if (hipGetLastError() != hipSuccess) return done(KFMI_E_KERNEL);
  }
  SearchLaunch a{};
  a.st = st;
  a.ix = idx_args(di);
  a.res = d_res;
  a.num = num;
  a.sa = di->sa;
  a.sa_log2 = di->sa_log2;
  a.off = d_off;
  a.owner = d_own;
  a.total = total;
  a.pos = d_pos;
  /* The cooperative walk takes its slots from a queue (counts are spent: word 0
   * of d_cnt is the queue's counter) when walks are long enough for the lanes'
   * ends to drift apart, SA rate >= 8 (rate 8: 2.3 -> 2.0-2.1 ms, rate 32:
   * 8.5-8.9 -> 7.3-7.9 ms; rate 1, one round per slot: 0.30 -> 0.56 ms,
   * profiles/r02/locate_r2av.jsonl); KFMI_LOCATE_QUEUE=0/1 forces it. */
  const char* qe = getenv("KFMI_LOCATE_QUEUE");
  const bool queue = qe ? atoi(qe) != 0 : (1u << di->sa_log2) >= 8;
  a.slot_ctr = queue ? reinterpret_cast<unsigned long long*>(d_cnt) : nullptr;
  const char* ce = getenv("KFMI_LOCATE_CHUNK");   /* slots per queue take; >= 64 keeps one take enough per wave */
  const long cv = ce ? atol(ce) : (long) SLOT_CHUNK;
  a.slot_chunk = (uint32_t) (cv < 64 ? 64 : (cv > 4096 ? 4096 : cv));
  ok = hipMemsetAsync(d_cnt, 0, 8, st) == hipSuccess && hipEventRecord(ev[1], st) == hipSuccess &&
       (total == 0 || dispatch(Op::Locate, di->K, di->nb, di->layout, a) == hipSuccess) &&
       hipEventRecord(ev[2], st) == hipSuccess &&
       hipMemcpyAsync(L->h_off, d_off, 8 * (num + 1), hipMemcpyDeviceToHost, st) == hipSuccess &&
       (total == 0 || hipMemcpyAsync(L->h_pos, d_pos, 4 * total, hipMemcpyDeviceToHost, st) == hipSuccess) &&
       hipStreamSynchronize(st) == hipSuccess;
  if (!ok) return done(KFMI_E_KERNEL);
  float ms01 = 0, ms12 = 0;
  (void) hipEventElapsedTime(&ms01, ev[0], ev[1]);
  (void) hipEventElapsedTime(&ms12, ev[1], ev[2]);
  t_ms[0] = ms01 + ms12;   /* scan + walk (the host read of the total sits between) */
  t_ms[1] = ms01;
  t_ms[2] = ms12;          /* the locate kernel alone */
  return done(KFMI_SUCCESS);
}

extern "C" int32_t kfmi_locate(void* index, void* results, uint32_t max_occ, void** locations)
{
  kfmi_fmi_t* f = (kfmi_fmi_t*) index;
  kfmi_res_t* r = (kfmi_res_t*) results;
  if (!locations) return KFMI_E_BAD_ARGUMENT;
  *locations = nullptr;
  if (!f || !r) return KFMI_E_BAD_ARGUMENT;
  if (!f->h_sa || !f->sa_rate) return KFMI_E_BAD_ARGUMENT;   /* index built without SA samples */
  DeviceGuard dg;
  /* the handle's lock shared; exclusive when a device copy still needs this
   * index's samples (locate_on uploads them into the copy) */
  RwLock& mu = index_lock(f);
  std::shared_lock<RwLock> sl(mu);
  std::unique_lock<RwLock> ul;
  auto stale = [&] {
    const GroupIndex* g = (const GroupIndex*) f->grp;
    if (!g) return f->dev && (!f->dev->sa || f->dev->sa_gen != f->sa_gen);
    for (int i = 0; i < g->n; ++i)
      if (!g->di[i]->sa || g->di[i]->sa_gen != f->sa_gen) return true;
    return false;
  };
  if (stale()) {
    sl.unlock();
    ul = std::unique_lock<RwLock>(mu);
  }
  if (!f->grp && !r->grp) {
    if (!f->dev || !r->d_results) return KFMI_E_NOT_ON_DEVICE;
    if (r->d_device != f->dev->device) return KFMI_E_BAD_ARGUMENT;
    return locate_on(f, f->dev, r->d_results, r->num, max_occ, (kfmi_locations**) locations);
  }
  /* device group: every member locates its slice, the lists are concatenated */
  GroupIndex* gi = (GroupIndex*) f->grp;
  GroupSlices* gr = (GroupSlices*) r->grp;
  if (!gi || !gr) return KFMI_E_NOT_ON_DEVICE;
  if (gr->n != gi->n) return KFMI_E_BAD_ARGUMENT;
  kfmi_locations* part[KFMI_MAX_GROUP] = {};
  int32_t err = KFMI_SUCCESS;
  double ms[3] = {0, 0, 0};
  uint64_t total = 0;
  for (int i = 0; i < gi->n && !err; ++i) {
    if (gr->dev[i] != gi->dev[i]) err = KFMI_E_BAD_ARGUMENT;
    if (!err) err = locate_on(f, gi->di[i], gr->d_res[i], gr->num[i], max_occ, &part[i]);
    if (!err) {
      total += part[i]->total;
      for (int k = 0; k < 3; ++k) ms[k] += t_ms[k];
    }
  }
  kfmi_locations* L = err ? nullptr : new (std::nothrow) kfmi_locations();
  if (!err && !L) err = KFMI_E_ALLOCATING_RESULTS;
  if (!err) {
    L->num = r->num;
    L->total = total;
    L->h_off = (uint64_t*) malloc(8 * (r->num + 1));
    L->h_pos = (uint32_t*) malloc(4 * total + 4);
    if (!L->h_off || !L->h_pos) err = KFMI_E_ALLOCATING_RESULTS;
  }
  if (!err) {
    uint64_t base = 0;
    for (int i = 0; i < gi->n; ++i) {
      for (uint64_t j = 0; j < gr->num[i]; ++j) L->h_off[gr->q0[i] + j] = base + part[i]->h_off[j];
      if (part[i]->total) memcpy(L->h_pos + base, part[i]->h_pos, 4 * part[i]->total);
      base += part[i]->total;
    }
    L->h_off[r->num] = total;
    *locations = L;
    for (int k = 0; k < 3; ++k) t_ms[k] = ms[k];
  } else if (L) {
    kfmi_locations_free((void**) &L);
  }
  for (int i = 0; i < gi->n; ++i)
    if (part[i]) kfmi_locations_free((void**) &part[i]);
  return err;
}

}  // namespace kfmi
