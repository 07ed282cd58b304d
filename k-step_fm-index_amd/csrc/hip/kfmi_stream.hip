/*
 * kfmi_stream.hip -- streamed search from host memory and
 * the host worker pool shared with the staged uploads.
 */
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "kfmi_runtime.h"

namespace kfmi {

/* ------------------------------------------------------------------------ */
/* streamed search from host memory: query H2D, packing, LF  */
/* and result D2H of successive chunks overlap on a few HIP streams.  By   */
/* default the host packs each chunk to 2-bit code words (qpack.c) while    */
/* the GPU works on the previous ones, so PCIe carries 4 bytes per 16 bases */
/* (KFMI_STREAM_HOSTPACK=0: ASCII H2D and packing on the device).  Pinned   */
/* ASCII is DMA'd directly; pageable goes through pinned staging.           */
/* ------------------------------------------------------------------------ */

/* slots in flight: enough that the host keeps packing while ASCII chunks
 * queue on the link (KFMI_STREAM_SLOTS, 2..8, default 6) */
constexpr int NSLOT_MAX = 8;
static int stream_slots(void)
{
  const char* e = getenv("KFMI_STREAM_SLOTS");
  const int v = e ? atoi(e) : 6;
  return v < 2 ? 2 : v > NSLOT_MAX ? NSLOT_MAX : v;
}

/* Pageable callers' buffers taken by the DMA engines directly instead of
 * through pinned staging copies on the host pool (KFMI_STREAM_DIRECT, read
 * once: bit 0 = the reads, bit 1 = the results; default 0).  On this ROCm a
 * pageable hipMemcpyAsync runs at the pinned rate (DESIGN.md 6a'), so a
 * direct ASCII chunk costs the host nothing -- what matters when 8 ranks share
 * a 16-CPU quota and each has ~2 host threads to pack or stage with. */
static int stream_direct(void)
{
  static const int v = [] {
    const char* e = getenv("KFMI_STREAM_DIRECT");
    return e ? (atoi(e) & 3) : 0;
  }();
  return v;
}

struct StreamSlot {
  hipStream_t st = nullptr;
  hipEvent_t done = nullptr;
  hipEvent_t x0 = nullptr, x1 = nullptr;   /* bracket the chunk's H2D (link time of its mode) */
  bool packed_mode = false;                /* this chunk's reads went over PCIe as host-packed words */
  kfmi_dev_queries dq;         /* device ascii + packed of one chunk */
  uint32_t* d_res = nullptr;
  uint8_t* h_in = nullptr;     /* pinned staging */
  uint32_t* h_out = nullptr;
  uint32_t* h_pk = nullptr;    /* pinned host-packed code words */
  uint64_t cap_q = 0, cap_in = 0, cap_words = 0;
  uint64_t q0 = 0, n = 0;
  bool busy = false;
};

struct StreamPool {
  bool init = false;
  StreamSlot slot[NSLOT_MAX];
  /* adaptive transfer mode: measured costs in ms per byte, kept across calls
   * (0 = not measured yet).  Host: EMA of packing / staging time per ASCII
   * byte.  Link: the fastest H2D seen per byte sent (the events bracketing a
   * copy also count time queued behind other slots' copies) -- an idle-link
   * figure, which the model multiplies by the processes that share this
   * device's link (KFMI_LINK_SHARERS, default 1: one GPU per rank; ranks
   * rehearsing on one card set it; profiles/r04/stream_contention_r4*.jsonl). */
  double r_pack = 0, r_stage = 0, r_xa = 0, r_xp = 0;
};
/* One pool per (device, group member): a single-device search uses member 0;
 * the members of a device group stream from pools of their own, so two
 * replicas listed on one GPU overlap like replicas on two GPUs do. */
static StreamPool g_pool[64][KFMI_MAX_GROUP];
static thread_local double t_stream_packed_frac = 0;   /* share of the last streamed batch packed on the host */
/* one streamed search per pool at a time; searches on other pools (one host
 * thread each) and every other entry point run concurrently with it */
static std::mutex g_pool_mu[64][KFMI_MAX_GROUP];

static void pool_free(int dev, int member)
{
  StreamPool& p = g_pool[dev][member];
  if (!p.init) return;
  (void) hipSetDevice(dev);
  for (StreamSlot& s : p.slot) {
    if (s.st) (void) hipStreamSynchronize(s.st);
    if (s.dq.ascii) (void) hipFree(s.dq.ascii);
    if (s.dq.packed) (void) hipFree(s.dq.packed);
    if (s.d_res) (void) hipFree(s.d_res);
    if (s.h_in) (void) hipHostFree(s.h_in);
    if (s.h_out) (void) hipHostFree(s.h_out);
    if (s.h_pk) (void) hipHostFree(s.h_pk);
    if (s.done) (void) hipEventDestroy(s.done);
    if (s.x0) (void) hipEventDestroy(s.x0);
    if (s.x1) (void) hipEventDestroy(s.x1);
    if (s.st) (void) hipStreamDestroy(s.st);
    s = StreamSlot();
  }
  p.init = false;
}

/* Grows slot buffers to hold `cq` queries of `size` bytes packed in `words` words. */
static int32_t slot_reserve(StreamSlot& s, uint64_t cq, uint32_t size, uint32_t words, bool stage_in, bool stage_out,
                     bool host_pack)
{
  if (!s.st) {
    if (hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreate(&s.x0) != hipSuccess || hipEventCreate(&s.x1) != hipSuccess)
      return KFMI_E_NO_DEVICE;
  }
  const uint64_t in = cq * size + 16;
  if (in > s.cap_in) {
    if (s.dq.ascii) (void) hipFree(s.dq.ascii);
    if (s.h_in) { (void) hipHostFree(s.h_in); s.h_in = nullptr; }
    s.dq.ascii = nullptr;
    s.cap_in = 0;
    if (hipMalloc((void**) &s.dq.ascii, in) != hipSuccess) return KFMI_E_DEVICE_ALLOC;
    s.cap_in = in;
  }
  if (stage_in && !s.h_in && hipHostMalloc((void**) &s.h_in, s.cap_in, hipHostMallocDefault) != hipSuccess)
    return KFMI_E_ALLOCATING_MFASTA;
  if (cq > s.cap_q || (uint64_t) words * cq > s.cap_words) {
    if (s.dq.packed) (void) hipFree(s.dq.packed);
    if (s.d_res) (void) hipFree(s.d_res);
    if (s.h_out) { (void) hipHostFree(s.h_out); s.h_out = nullptr; }
    if (s.h_pk) { (void) hipHostFree(s.h_pk); s.h_pk = nullptr; }
    s.dq.packed = nullptr;
    s.d_res = nullptr;
    s.cap_q = s.cap_words = 0;
    if (hipMalloc((void**) &s.dq.packed, 4ull * words * cq) != hipSuccess ||
        hipMalloc((void**) &s.d_res, 8ull * cq) != hipSuccess)
      return KFMI_E_DEVICE_ALLOC;
    s.cap_q = cq;
    s.cap_words = (uint64_t) words * cq;
  }
  if (stage_out && !s.h_out && hipHostMalloc((void**) &s.h_out, 8ull * s.cap_q, hipHostMallocDefault) != hipSuccess)
    return KFMI_E_ALLOCATING_RESULTS;
  if (host_pack && !s.h_pk && hipHostMalloc((void**) &s.h_pk, 4ull * s.cap_words, hipHostMallocDefault) != hipSuccess)
    return KFMI_E_ALLOCATING_MFASTA;
  return KFMI_SUCCESS;
}

bool host_pinned(const void* p)
{
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void) hipGetLastError();
    return false;
  }
  return at.type == hipMemoryTypeHost;
}

/* Persistent host workers for the streamed search (a chunk every few hundred
 * microseconds: spawning threads per chunk would cost as much as the work).
 * kfmi_host_threads() threads including the caller (KFMI_HOST_THREADS, else
 * the process's CPU share split among this host's ranks, common.c). */
class HostPool {
 public:
  static HostPool& get()
  {
    static HostPool p;
    return p;
  }
  int size() const { return (int) th_.size() + 1; }
  /* fn(i) for i in [0, n) over the workers and the caller; returns when all are
   * done.  Calls from several host threads (one per device) take turns. */
  void run(int n, const std::function<void(int)>& fn)
  {
    if (n <= 1 || th_.empty()) {
      for (int i = 0; i < n; ++i) fn(i);
      return;
    }
    std::lock_guard<std::mutex> turn(run_mu_);
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_ = n;
      next_ = 0;
      left_ = n;
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return left_ == 0; });
    fn_ = nullptr;
  }

 private:
  HostPool()
  {
    const int v = kfmi_host_threads();
    for (int i = 0; i + 1 < v; ++i) th_.emplace_back([this] { loop(); });
  }
  ~HostPool()
  {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void loop()
  {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
    }
  }
  void work()
  {
    for (;;) {
      const std::function<void(int)>* f;
      int i;
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (!fn_ || next_ >= n_) return;
        i = next_++;
        f = fn_;
      }
      (*f)(i);
      std::lock_guard<std::mutex> lk(mu_);
      if (--left_ == 0) done_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_ = 0, next_ = 0, left_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

/* memcpy split over the host workers (pageable <-> pinned staging) */
void par_copy(void* dst, const void* src, uint64_t bytes)
{
  HostPool& hp = HostPool::get();
  const int nt = hp.size();
  /* a streamed chunk's results (8 B x 2^19 reads = 4 MB) are copied here one
   * by one: one thread at ~8 GB/s made them 10 of the 21 ms a 10M-read
   * pageable batch took (profiles/r04/bench_r4c.json end_to_end) */
  if (nt == 1 || bytes < (1u << 20)) {
    memcpy(dst, src, bytes);
    return;
  }
  const uint64_t part = ((bytes + nt - 1) / nt + 4095) & ~4095ull;
  hp.run(nt, [&](int t) {
    const uint64_t b = part * t;
    if (b >= bytes) return;
    const uint64_t len = bytes - b < part ? bytes - b : part;
    memcpy((uint8_t*) dst + b, (const uint8_t*) src + b, len);
  });
}

/* pread of [off, off + bytes) of fd into dst, split over the host workers
 * (page-cache reads run at memcpy speed per thread); false on a short read */
bool par_pread(int fd, void* dst, uint64_t off, uint64_t bytes)
{
  HostPool& hp = HostPool::get();
  const int nt = bytes < (4u << 20) ? 1 : hp.size();
  const uint64_t part = ((bytes + nt - 1) / nt + 4095) & ~4095ull;
  std::atomic<bool> ok{true};
  hp.run(nt, [&](int t) {
    uint64_t b = part * t;
    const uint64_t e = b + part < bytes ? b + part : bytes;
    while (b < e) {
      const ssize_t r = pread(fd, (uint8_t*) dst + b, (size_t) (e - b), (off_t) (off + b));
      if (r <= 0) { ok = false; return; }
      b += (uint64_t) r;
    }
  });
  return ok;
}

/* ASCII rows -> word-major code words of one chunk, over the host workers */
void par_pack(const char* src, uint64_t n, uint32_t size, uint32_t rem, uint32_t* out)
{
  HostPool& hp = HostPool::get();
  const int parts = n < 4096 ? 1 : hp.size();
  hp.run(parts, [&](int t) {
    const uint64_t r0 = n * t / parts, r1 = n * (t + 1) / parts;
    kfmi_pack_rows_rem((const uint8_t*) src + r0 * size, r1 - r0, size, rem, out + r0, n);
  });
}

extern "C" double kfmi_stream_hostpacked_fraction(void) { return t_stream_packed_frac; }

extern "C" int32_t kfmi_host_alloc(uint64_t bytes, void** p)
{
  if (!p) return KFMI_E_BAD_ARGUMENT;
  *p = nullptr;
  DeviceGuard dg;
  if (hipSetDevice(kfmi_current_device()) != hipSuccess) return KFMI_E_NO_DEVICE;
  if (hipHostMalloc(p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return KFMI_E_ALLOCATING_MFASTA;
  return KFMI_SUCCESS;
}

extern "C" int32_t kfmi_host_free(void* p)
{
  if (p && hipHostFree(p) != hipSuccess) return KFMI_E_BAD_ARGUMENT;
  return KFMI_SUCCESS;
}

/* Frees the pools of every device (not only the caller's current one: the
 * pools belong to the devices the searched indexes live on). */
extern "C" int32_t kfmi_stream_release(void)
{
  DeviceGuard dg;
  for (int dev = 0; dev < 64; ++dev)
    for (int m = 0; m < KFMI_MAX_GROUP; ++m) {
      std::lock_guard<std::mutex> lk(g_pool_mu[dev][m]);
      pool_free(dev, m);
    }
  release_upload_staging();
  return KFMI_SUCCESS;
}

/* One device's streamed search of `num` reads (the whole batch, or one member's
 * slice of a device group).  ms3 = {wall, host packing/staging, blocked on
 * the GPU}; *npacked = reads sent as host-packed words. */
static int32_t stream_on(kfmi_dev_index* di, int member, const char* ascii, uint64_t num, uint32_t size,
                         uint32_t* results, uint64_t chunk, uint32_t ftab, double* ms3, uint64_t* npacked_out)
{
  const uint32_t K = di->K;
  DevCtx* ctx = nullptr;
  int32_t err = ctx_for(di->device, &ctx);
  if (err) return err;
  ms3[0] = ms3[1] = ms3[2] = 0;
  *npacked_out = 0;
  if (num == 0) return KFMI_SUCCESS;
  /* KFMI_STREAM_HOSTPACK: 1 = every chunk packed on the host, 0 = every chunk
   * sent as ASCII (packed on the device), 3 = alternate (testing), unset / 2 =
   * adaptive: per chunk, whichever mode a two-resource model (host thread
   * pool, PCIe link) says finishes first, with per-read costs measured on the
   * previous chunks -- on a box whose host packs slower than the link carries
   * ASCII, part of the batch goes as ASCII while the host packs the rest.
   * (A batch-level balance -- pack the share that equalises host and link
   * time -- measured no better than packing everything: host packing and the
   * DMA of pinned ASCII draw on the same host DRAM bandwidth, so the two
   * "resources" are not independent; profiles/r02/e2e_modes_r2al.jsonl.) */
  const char* hp = getenv("KFMI_STREAM_HOSTPACK");
  /* K = 3: the host packer writes 16 bases per word, the K = 3 kernels read 5
   * K-steps per word -- every chunk goes as ASCII (packed in the kernel) */
  const int mode = K == 3 ? 0 : (hp ? atoi(hp) : 2);
  const bool any_pack = mode != 0, any_ascii = mode != 1;
  const uint64_t def_chunk = any_pack ? (1ull << 19) : (1ull << 16);   /* profiles/r01/e2e_sweep*.jsonl */
  if (chunk == 0) {
    const char* e = getenv("KFMI_STREAM_CHUNK");
    chunk = e ? strtoull(e, nullptr, 10) : def_chunk;
  }
  if (chunk == 0) chunk = def_chunk;
  if (chunk > num) chunk = num;
  /* reads with m % K = rem != 0: K-steps over bases 0 .. m-rem-1, the last rem
   * bases from the remainder table; code-word row nwords holds their codes
   * (written by the host packer or by the pack kernel, read by the fused ones
   * from the ASCII) -- the layout kfmi_search uses */
  const uint32_t rem = size % K;
  const uint32_t steps = (size - rem) / K, spw = 32 / (2 * K), nwords = (steps + spw - 1) / spw;
  const uint32_t rows = nwords + (rem ? 1u : 0u);   /* code-word rows per read */
  const int direct = stream_direct();
  /* pinned, or taken directly from pageable memory: no staging either way */
  const bool pin_in = host_pinned(ascii) || (direct & 1), pin_out = host_pinned(results) || (direct & 2);

  std::lock_guard<std::mutex> lk(g_pool_mu[di->device][member]);
  StreamPool& pool = g_pool[di->device][member];
  pool.init = true;
  const int nslot = stream_slots();
  for (int k = 0; k < nslot; ++k) {
    StreamSlot& s = pool.slot[k];
    err = slot_reserve(s, chunk, size, rows, !pin_in && any_ascii, !pin_out, any_pack);
    if (err) return err;
    s.busy = false;
  }
  /* cost model: pool.r_* per byte (see StreamPool) -> ms per read */
  const double abytes = (double) size, pbytes = 4.0 * rows;
  const char* ls = getenv("KFMI_LINK_SHARERS");
  const double sharers = ls && atoi(ls) > 1 ? (double) atoi(ls) : 1.0;
  uint64_t npacked = 0;
  double t_host = 0, t_link = 0;                      /* model clocks of this call */
  auto ema = [](double& v, double x) { v = v > 0 ? 0.6 * v + 0.4 * x : x; };
  auto keep_min = [](double& v, double x) { v = (v > 0 && v < x) ? v : x; };
  const auto t0 = std::chrono::steady_clock::now();
  const Op op = is_coop(di->backend) ? Op::Coop : Op::Task;
  IdxArgs ix = idx_args(di);
  err = use_ftab(di, ctx->st, ix, ftab);   /* the caller's setting (member threads have their own) */
  if (!err) err = use_rtab(di, ctx->st, ix, rem);   /* rem != 0: the table, no ftab (as kfmi_search) */
  if (err) return err;
  int32_t status = KFMI_SUCCESS;
  using clk = std::chrono::steady_clock;
  double host_ms = 0, wait_ms = 0;   /* host packing/staging; blocked on the GPU */
  auto since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
  auto retire = [&](StreamSlot& s) {
    if (!s.busy) return;
    const auto tw = clk::now();
    const bool ok = hipEventSynchronize(s.done) == hipSuccess;
    wait_ms += since(tw);
    if (!ok) status = KFMI_E_KERNEL;
    else {
      if (!pin_out) par_copy(results + 2 * s.q0, s.h_out, 8ull * s.n);
      float x = 0;
      if (hipEventElapsedTime(&x, s.x0, s.x1) == hipSuccess && s.n && x > 0) {
        if (s.packed_mode) keep_min(pool.r_xp, x / (s.n * pbytes));
        else keep_min(pool.r_xa, x / (s.n * abytes));
      }
    }
    s.busy = false;
  };
  const uint64_t nchunks = (num + chunk - 1) / chunk;
  for (uint64_t i = 0; i < nchunks && status == KFMI_SUCCESS; ++i) {
    StreamSlot& s = pool.slot[i % nslot];
    retire(s);
    if (status) break;
    s.q0 = i * chunk;
    s.n = num - s.q0 < chunk ? num - s.q0 : chunk;
    const char* src = ascii + s.q0 * size;
    const uint64_t bytes = s.n * size;
    const void* hsrc = src;
    bool host_pack;
    if (mode == 0 || mode == 1) host_pack = mode == 1;
    else if (mode == 3) host_pack = (i & 1) == 0;
    else if (pool.r_pack <= 0 || pool.r_xp <= 0) host_pack = true;      /* measure packing first */
    else if (pool.r_xa <= 0 || (!pin_in && pool.r_stage <= 0)) host_pack = false;   /* then ASCII */
    else {
      const double dn = (double) s.n;
      const double hp_ms = pool.r_pack * abytes * dn, st_ms = pin_in ? 0.0 : pool.r_stage * abytes * dn;
      const double xp = pool.r_xp * sharers, xa = pool.r_xa * sharers;
      const double done_p = std::max(t_host + hp_ms, t_link) + xp * pbytes * dn;
      const double done_a = std::max(t_host + st_ms, t_link) + xa * abytes * dn;
      host_pack = done_p <= done_a;
      t_host += host_pack ? hp_ms : st_ms;
      t_link = host_pack ? done_p : done_a;
    }
    s.packed_mode = host_pack;
    npacked += host_pack ? s.n : 0;
    const auto th = clk::now();
    if (host_pack) par_pack(src, s.n, size, rem, s.h_pk);
    else if (!pin_in) {
      par_copy(s.h_in, src, bytes);
      hsrc = s.h_in;
    }
    const double hms = since(th);
    host_ms += hms;
    if (s.n && (host_pack || !pin_in)) ema(host_pack ? pool.r_pack : pool.r_stage, hms / (s.n * abytes));
    s.dq.device = di->device;
    s.dq.num = s.n;
    s.dq.size = size;
    s.dq.K = K;
    s.dq.steps = steps;
    s.dq.nwords = nwords;
    s.dq.rem = rem;
    s.dq.packed_rows = rows;
    SearchLaunch a;
    a.st = s.st;
    a.ix = ix;
    a.qp = s.dq.packed;
    a.ascii = s.dq.ascii;
    a.m = size;
    a.maxw = host_pack ? 0 : fused_maxw(di->backend, K * steps);
    a.num = s.n;
    a.steps = steps;
    a.nwords = nwords;
    a.res = s.d_res;
    void* hdst = pin_out ? (void*) (results + 2 * s.q0) : (void*) s.h_out;
    const bool up_ok = hipEventRecord(s.x0, s.st) == hipSuccess &&
                       (host_pack ? hipMemcpyAsync(s.dq.packed, s.h_pk, 4ull * rows * s.n, hipMemcpyHostToDevice,
                                                   s.st) == hipSuccess
                                  : hipMemcpyAsync(s.dq.ascii, hsrc, bytes, hipMemcpyHostToDevice, s.st) == hipSuccess) &&
                       hipEventRecord(s.x1, s.st) == hipSuccess &&
                       (host_pack || a.maxw || launch_pack(&s.dq, s.st) == hipSuccess);
    if (!up_ok || dispatch(op, K, di->nb, di->layout, a) != hipSuccess ||
        hipMemcpyAsync(hdst, s.d_res, 8ull * s.n, hipMemcpyDeviceToHost, s.st) != hipSuccess ||
        hipEventRecord(s.done, s.st) != hipSuccess) {
      status = KFMI_E_KERNEL;
      break;
    }
    s.busy = true;
  }
  for (int k = 0; k < nslot; ++k) retire(pool.slot[k]);
  ms3[0] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  ms3[1] = host_ms;   /* host packing or staging copies */
  ms3[2] = wait_ms;   /* blocked on chunks in flight */
  *npacked_out = npacked;
  return status;
}

/* Streamed search of host reads into host results.  On a device group
 * (KFMI_DEVICES / kfmi_set_devices, index transferred to the group) the batch
 * is cut into one contiguous slice per member (multiples of 64 reads) and
 * every member streams its slice on its own replica from its own host thread;
 * the members' host packing shares the one worker pool (taking turns), their
 * copies and kernels overlap on their devices.  Timings: the slowest member. */
extern "C" int32_t kfmi_search_stream(void* index, const char* ascii, uint64_t num, uint32_t size,
                                      uint32_t* results, uint64_t chunk)
{
  kfmi_fmi_t* f = (kfmi_fmi_t*) index;
  if (!f || (!ascii && num) || (!results && num)) return KFMI_E_BAD_ARGUMENT;
  DeviceGuard dg;
  std::shared_lock<RwLock> lk(index_lock(f));
  GroupIndex* g = (GroupIndex*) f->grp;
  if (!g && !f->dev) return KFMI_E_NOT_ON_DEVICE;
  const kfmi_dev_index* d0 = g ? g->di[0] : f->dev;
  const uint32_t K = d0->K;
  /* m % K != 0 takes the remainder table, like kfmi_search: not on the
   * AltCounters layouts (their semantics differ there) */
  if (size == 0) return KFMI_E_BAD_ARGUMENT;
  if (size % K && !rem_supported(d0->layout)) return KFMI_E_BAD_ARGUMENT;
  double ms[KFMI_MAX_GROUP][3] = {};
  uint64_t np[KFMI_MAX_GROUP] = {};
  int32_t err = KFMI_SUCCESS;
  const uint32_t ftab = ftab_bases();
  if (!g) {
    err = stream_on(f->dev, 0, ascii, num, size, results, chunk, ftab, ms[0], &np[0]);
  } else {
    const int n = g->n;
    uint64_t per = (num + n - 1) / n;
    per = (per + 63) & ~63ull;
    int32_t errs[KFMI_MAX_GROUP] = {};
    std::vector<std::thread> th;
    th.reserve(n);
    for (int i = 0; i < n; ++i) {
      const uint64_t a = per * i < num ? per * i : num, b = per * (i + 1) < num ? per * (i + 1) : num;
      th.emplace_back([&, i, a, b] {
        errs[i] = stream_on(g->di[i], i, ascii + a * size, b - a, size, results + 2 * a, chunk, ftab, ms[i], &np[i]);
      });
    }
    for (auto& t : th) t.join();
    for (int i = 0; i < n && !err; ++i) err = errs[i];
    for (int i = 1; i < n; ++i) {
      for (int k = 0; k < 3; ++k) ms[0][k] = std::max(ms[0][k], ms[i][k]);
      np[0] += np[i];
    }
  }
  for (int k = 0; k < 3; ++k) t_ms[k] = ms[0][k];
  t_stream_packed_frac = num ? (double) np[0] / (double) num : 0.0;
  return err;
}

}  // namespace kfmi
