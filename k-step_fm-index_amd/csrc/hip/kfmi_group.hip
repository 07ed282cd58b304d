/*
 * kfmi_group.hip -- device groups: the reference's handles spread over
 * several GPUs (SURVEY 8(b) device selection, 8(e) query slicing).
 */
#include <stdlib.h>
#include <chrono>
#include <new>
#include <thread>
#include <vector>

#include "kfmi_runtime.h"

namespace kfmi {

/* ------------------------------------------------------------------------ */
/* device groups (SURVEY 8(b) device selection, 8(e) partitioning).  The     */
/* reference fixes one GPU at compile time (-DDEVICE); KFMI_DEVICES=0,1,...  */
/* or kfmi_set_devices spreads the same handles over several: the index      */
/* replicated on every device, the queries cut into contiguous slices        */
/* (multiples of 64 reads), each device searching its slice on its own       */
/* stream, results copied back into disjoint slices of h_results.  No        */
/* exchange between devices on the data path.                               */
/* ------------------------------------------------------------------------ */

static thread_local int t_ngroup = -1;   /* -1: read KFMI_DEVICES */
static thread_local int t_group[KFMI_MAX_GROUP];

/* The device list (0 or 1 entry: single-device mode). */
int group_devices(int* devs)
{
  if (t_ngroup < 0) {
    t_ngroup = 0;
    const char* p = getenv("KFMI_DEVICES");
    while (p && *p && t_ngroup < KFMI_MAX_GROUP) {
      char* end = nullptr;
      const long v = strtol(p, &end, 10);
      if (end == p) break;
      t_group[t_ngroup++] = (int) v;
      p = end;
      while (*p == ',' || *p == ' ') ++p;
    }
  }
  for (int i = 0; i < t_ngroup; ++i) devs[i] = t_group[i];
  return t_ngroup;
}

static GroupSlices* group_slices(uint64_t num, const int* devs, int n)
{
  GroupSlices* g = new (std::nothrow) GroupSlices();
  if (!g) return nullptr;
  g->n = n;
  uint64_t per = (num + n - 1) / n;
  per = (per + 63) & ~63ull;
  for (int i = 0; i < n; ++i) {
    g->dev[i] = devs[i];
    const uint64_t a = per * i < num ? per * i : num, b = per * (i + 1) < num ? per * (i + 1) : num;
    g->q0[i] = a;
    g->num[i] = b - a;
  }
  return g;
}

void group_free_index(kfmi_fmi_t* f)
{
  GroupIndex* g = (GroupIndex*) f->grp;
  if (!g) return;
  for (int i = 0; i < g->n; ++i) {
    (void) hipSetDevice(g->dev[i]);
    if (g->st[i]) (void) hipStreamSynchronize(g->st[i]);
    free_dev_index(g->di[i]);
    for (int k = 0; k < 3; ++k)
      if (g->ev[i][k]) (void) hipEventDestroy(g->ev[i][k]);
    if (g->st[i]) (void) hipStreamDestroy(g->st[i]);
  }
  delete g;
  f->grp = nullptr;
}

void group_free_queries(kfmi_qrys_t* q)
{
  GroupSlices* g = (GroupSlices*) q->grp;
  if (!g) return;
  for (int i = 0; i < g->n; ++i) free_dev_queries(g->dq[i]);
  delete g;
  q->grp = nullptr;
}

void group_free_results(kfmi_res_t* r)
{
  GroupSlices* g = (GroupSlices*) r->grp;
  if (!g) return;
  for (int i = 0; i < g->n; ++i)
    if (g->d_res[i]) {
      (void) hipSetDevice(g->dev[i]);
      (void) hipFree(g->d_res[i]);
    }
  delete g;
  r->grp = nullptr;
}

/* A replica of `src` on device `dev`: same geometry, device buffers copied
 * device-to-device on `st` (hipMemcpyPeerAsync: over xGMI between GPUs, a
 * local copy when `dev` is src's own device).  Returns with the copies queued. */
static int32_t replicate_index(const kfmi_dev_index* src, int dev, hipStream_t st, kfmi_dev_index** out)
{
  kfmi_dev_index* di = new (std::nothrow) kfmi_dev_index();
  if (!di) return KFMI_E_ALLOCATING_FMI;
  di->device = dev;
  di->backend = src->backend;
  di->layout = src->layout;
  di->K = src->K;
  di->d = src->d;
  di->nb = src->nb;
  di->bwtsize = src->bwtsize;
  di->nentries = src->nentries;
  di->dl = src->dl;
  di->ent_bytes = src->ent_bytes;
  di->sa_bytes = src->sa_bytes;
  di->sa_log2 = src->sa_log2;
  di->sa_gen = src->sa_gen;
  di->lf_perm.store(src->lf_perm.load());
  di->ac_tail_b0 = src->ac_tail_b0;
  struct Buf { uint32_t* const* from; uint32_t** to; uint64_t bytes; };
  const Buf bufs[3] = {{&src->ent, &di->ent, src->ent_bytes},
                       {&src->sa, &di->sa, src->sa ? src->sa_bytes + 4 : 0},
                       {&src->ac_tail, &di->ac_tail, src->ac_tail ? 16ull * (1u << (2 * src->K)) : 0}};
  for (const Buf& b : bufs) {
    if (!*b.from || !b.bytes) continue;
    if (hipMalloc((void**) b.to, b.bytes) != hipSuccess) {
      *b.to = nullptr;
      free_dev_index(di);
      return KFMI_E_DEVICE_ALLOC;
    }
    if (hipMemcpyPeerAsync(*b.to, dev, *b.from, src->device, b.bytes, st) != hipSuccess) {
      free_dev_index(di);
      return KFMI_E_KERNEL;
    }
  }
  *out = di;
  return KFMI_SUCCESS;
}

/* fn(i) for every member i on its own host thread (hipSetDevice is per thread),
 * first error wins. */
template <class F>
static int32_t each_member(int n, F fn)
{
  std::vector<int32_t> errs(n, KFMI_SUCCESS);
  std::vector<std::thread> th;
  th.reserve(n);
  for (int i = 0; i < n; ++i) th.emplace_back([&, i] { errs[i] = fn(i); });
  for (auto& t : th) t.join();
  for (int32_t e : errs)
    if (e) return e;
  return KFMI_SUCCESS;
}

/* Reads [q0, q0 + n) of device-resident reads `src` (any device) as their own
 * device batch on `dev`: the ASCII rows copied device to device (a local copy
 * on src's own device, hipMemcpyPeerAsync over xGMI otherwise). */
static int32_t slice_device_queries(const kfmi_dev_queries* src, uint64_t q0, uint64_t n, uint32_t K, int dev,
                                    DevCtx* ctx, kfmi_dev_queries** out)
{
  *out = nullptr;
  kfmi_dev_queries* dq = new (std::nothrow) kfmi_dev_queries();
  if (!dq) return KFMI_E_ALLOCATING_MFASTA;
  dq->device = dev;
  dq->num = n;
  dq->size = src->size;
  query_geometry(dq, K);
  const uint64_t bytes = n * (uint64_t) src->size;
  if (hipMalloc((void**) &dq->ascii, bytes + 16) != hipSuccess ||
      hipMalloc((void**) &dq->packed, 4ull * (dq->nwords + 1) * (n ? n : 1)) != hipSuccess) {
    free_dev_queries(dq);
    return KFMI_E_DEVICE_ALLOC;
  }
  dq->packed_rows = dq->nwords + 1;
  if (bytes) {
    int can = 0;
    if (dev != src->device && hipDeviceCanAccessPeer(&can, dev, src->device) == hipSuccess && can &&
        hipDeviceEnablePeerAccess(src->device, 0) != hipSuccess)
      (void) hipGetLastError();   /* already enabled: fine; else the runtime stages the copy */
    const uint8_t* from = src->ascii + q0 * src->size;
    const hipError_t ce = dev == src->device
                              ? hipMemcpyAsync(dq->ascii, from, bytes, hipMemcpyDeviceToDevice, ctx->st)
                              : hipMemcpyPeerAsync(dq->ascii, dev, from, src->device, bytes, ctx->st);
    if (ce != hipSuccess || hipStreamSynchronize(ctx->st) != hipSuccess) {
      free_dev_queries(dq);
      return KFMI_E_KERNEL;
    }
  }
  *out = dq;
  return KFMI_SUCCESS;
}

int32_t group_transfer(kfmi_fmi_t* f, kfmi_qrys_t* q, kfmi_res_t* r, const int* devs, int n)
{
  const int backend = f ? backend_for(f->steps) : kfmi_backend();
  int32_t err = KFMI_SUCCESS;
  if (f) {
    GroupIndex* g = (GroupIndex*) f->grp;
    bool same = g && g->backend == backend && g->n == n;
    for (int i = 0; same && i < n; ++i) same = g->dev[i] == devs[i];
    if (!same) {
      using clk = std::chrono::steady_clock;
      auto ms_since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
      const auto t0 = clk::now();
      double setup_ms = 0;
      group_free_index(f);
      g = new (std::nothrow) GroupIndex();
      if (!g) return KFMI_E_ALLOCATING_FMI;
      g->n = n;
      g->backend = backend;
      f->grp = g;
      /* the layout is built once, on the first member (host -> device upload and
       * the relayout kernels), then fanned out device-to-device to the others,
       * every copy queued on its destination's stream before any is waited for
       * (one-time replication over xGMI, no host round trip) */
      for (int i = 0; i < n && !err; ++i) {
        g->dev[i] = devs[i];
        DevCtx* ctx = nullptr;
        const auto ts = clk::now();
        err = ctx_for(devs[i], &ctx);
        if (!err && hipStreamCreateWithFlags(&g->st[i], hipStreamNonBlocking) != hipSuccess) err = KFMI_E_NO_DEVICE;
        for (int k = 0; k < 3 && !err; ++k)
          if (hipEventCreate(&g->ev[i][k]) != hipSuccess) err = KFMI_E_NO_DEVICE;
        setup_ms += ms_since(ts);
        if (!err && i == 0) err = upload_index(f, backend, devs[0], ctx, &g->di[0]);
      }
      const auto tf = clk::now();
      for (int i = 1; i < n && !err; ++i) {
        int can = 0;
        (void) hipSetDevice(devs[i]);
        if (devs[i] != devs[0] && hipDeviceCanAccessPeer(&can, devs[i], devs[0]) == hipSuccess && can &&
            hipDeviceEnablePeerAccess(devs[0], 0) != hipSuccess)
          (void) hipGetLastError();   /* already enabled: fine; else the copy is staged by the runtime */
        err = replicate_index(g->di[0], devs[i], g->st[i], &g->di[i]);
      }
      for (int i = 1; i < n; ++i)
        if (g->st[i]) {
          (void) hipSetDevice(devs[i]);
          if (hipStreamSynchronize(g->st[i]) != hipSuccess && !err) err = KFMI_E_KERNEL;
        }
      if (err) {
        group_free_index(f);
        return err;
      }
      /* kfmi_last_timing after a group upload: total = the index setup, pack =
       * the members' stream + event creation, lf = the replica fan-out
       * (allocations + device-to-device copies of members 1..n-1) */
      t_ms[0] = ms_since(t0);
      t_ms[1] = setup_ms;
      t_ms[2] = ms_since(tf);
    }
    if (f->dev) {   /* one mode per handle: the single-device copy goes */
      free_dev_index(f->dev);
      f->dev = nullptr;
    }
  }
  if (q) {
    if (!f) return KFMI_E_BAD_ARGUMENT;
    /* reads parsed on a device (kfmi_load_queries_gpu) have no host copy: the
     * members take their slices device to device from the parsing device, and
     * that copy (q->dev) stays with the handle */
    const bool parsed = !q->h_queries && q->num;
    if (parsed && !q->dev) return KFMI_E_NOT_ON_DEVICE;
    group_free_queries(q);
    if (q->dev && !parsed) {
      free_dev_queries(q->dev);
      q->dev = nullptr;
    }
    GroupSlices* g = group_slices(q->num, devs, n);
    if (!g) return KFMI_E_ALLOCATING_MFASTA;
    q->grp = g;
    /* every slice over its own device's PCIe link (or xGMI link) at the same time */
    err = each_member(n, [&](int i) {
      DevCtx* ctx = nullptr;
      int32_t e = ctx_for(devs[i], &ctx);
      if (!e && parsed) {
        e = slice_device_queries(q->dev, g->q0[i], g->num[i], device_steps(f), devs[i], ctx, &g->dq[i]);
        return e;
      }
      kfmi_qrys_t sh{};
      sh.num = g->num[i];
      sh.size = q->size;
      sh.h_queries = q->h_queries + g->q0[i] * q->size;
      if (!e) e = upload_queries(&sh, device_steps(f), devs[i], ctx);
      g->dq[i] = sh.dev;
      return e;
    });
    if (err) {
      group_free_queries(q);
      return err;
    }
  }
  if (r) {
    group_free_results(r);
    if (r->d_results) {
      (void) hipFree(r->d_results);
      r->d_results = nullptr;
    }
    GroupSlices* g = group_slices(r->num, devs, n);
    if (!g) return KFMI_E_ALLOCATING_RESULTS;
    r->grp = g;
    for (int i = 0; i < n && !err; ++i) {
      DevCtx* ctx = nullptr;
      err = ctx_for(devs[i], &ctx);
      if (!err && hipMalloc((void**) &g->d_res[i], 8ull * (g->num[i] ? g->num[i] : 1)) != hipSuccess) {
        g->d_res[i] = nullptr;
        err = KFMI_E_DEVICE_ALLOC;
      }
      if (!err && (hipMemsetAsync(g->d_res[i], 0, 8ull * g->num[i], ctx->st) != hipSuccess ||
                   hipStreamSynchronize(ctx->st) != hipSuccess))
        err = KFMI_E_KERNEL;
    }
    if (err) {
      group_free_results(r);
      return err;
    }
  }
  return KFMI_SUCCESS;
}

/* Every member queues its slice, then all are waited for; the timings are the
 * slowest member's. */
int32_t group_search(kfmi_fmi_t* f, kfmi_qrys_t* q, kfmi_res_t* r)
{
  GroupIndex* gi = (GroupIndex*) f->grp;
  GroupSlices* gq = (GroupSlices*) q->grp;
  GroupSlices* gr = (GroupSlices*) r->grp;
  if (!gi || !gq || !gr) return KFMI_E_NOT_ON_DEVICE;   /* handles moved to different modes */
  if (gq->n != gi->n || gr->n != gi->n) return KFMI_E_BAD_ARGUMENT;
  for (int i = 0; i < gi->n; ++i)
    if (gq->dev[i] != gi->dev[i] || gr->dev[i] != gi->dev[i] || gq->num[i] != gr->num[i]) return KFMI_E_BAD_ARGUMENT;
  const uint32_t ftab = ftab_bases();
  int32_t err = KFMI_SUCCESS;
  int queued = 0;
  for (int i = 0; i < gi->n && !err; ++i) {
    if (hipSetDevice(gi->dev[i]) != hipSuccess) {
      err = KFMI_E_NO_DEVICE;
      break;
    }
    err = search_enqueue(gi->di[i], gq->dq[i], gr->d_res[i], gi->st[i], gi->ev[i], ftab);
    if (!err) ++queued;
  }
  double worst[3] = {0, 0, 0};
  for (int i = 0; i < queued; ++i) {
    (void) hipSetDevice(gi->dev[i]);
    double ms[3] = {0, 0, 0};
    const int32_t e = search_finish(gi->st[i], gi->ev[i], ms);
    if (e && !err) err = e;
    for (int k = 0; k < 3; ++k) worst[k] = ms[k] > worst[k] ? ms[k] : worst[k];
  }
  for (int k = 0; k < 3; ++k) t_ms[k] = worst[k];
  return err;
}

int32_t group_to_host(kfmi_res_t* r)
{
  GroupSlices* g = (GroupSlices*) r->grp;
  for (int i = 0; i < g->n; ++i) {
    DevCtx* ctx = nullptr;
    int32_t err = ctx_for(g->dev[i], &ctx);
    if (err) return err;
    if (g->num[i])
      HIP_OK(hipMemcpyAsync(r->h_results + 2 * g->q0[i], g->d_res[i], 8ull * g->num[i], hipMemcpyDeviceToHost,
                            ctx->st));
  }
  for (int i = 0; i < g->n; ++i) {
    DevCtx* ctx = nullptr;
    int32_t err = ctx_for(g->dev[i], &ctx);
    if (err) return err;
    HIP_OK(hipStreamSynchronize(ctx->st));
  }
  return KFMI_SUCCESS;
}

extern "C" int32_t kfmi_set_devices(const int32_t* devices, int32_t n)
{
  if (n < 0 || n > KFMI_MAX_GROUP || (n && !devices)) return KFMI_E_BAD_ARGUMENT;
  const int avail = kfmi_device_count();
  for (int i = 0; i < n; ++i)
    if (devices[i] < 0 || devices[i] >= avail) return KFMI_E_NO_DEVICE;
  for (int i = 0; i < n; ++i) t_group[i] = devices[i];
  t_ngroup = n;
  if (n == 1) t_device = devices[0];
  return KFMI_SUCCESS;
}

extern "C" int32_t kfmi_get_devices(int32_t* devices, int32_t cap)
{
  int devs[KFMI_MAX_GROUP];
  const int n = group_devices(devs);
  for (int i = 0; i < n && i < cap && devices; ++i) devices[i] = devs[i];
  return n;
}

}  // namespace kfmi
