/*
 * kfmi_probe.hip -- replay probe (diagnostic; DESIGN.md 5 "The ceiling,
 * measured on the kernel's own requests").  Is the LF kernel at the memory
 * system's request ceiling, or is it held below it by its dependent chain?
 *
 * gather_probe measures uniformly random lines; the LF kernel's requests are
 * a mix (its first K-steps touch a few thousand lines that stay in L2, the
 * next ones ~10^5-10^6 lines that live in the Infinity Cache, the rest are
 * HBM).  This probe replays that exact mix: a trace launch walks the batch with
 * the search's own LF and records, for every (K-step, read), the MID128 line
 * each end reads (kfmi_probe_replay, MID layouts at K = 2, d = 64 only); the
 * replay launch then issues the same loads per line as the task kernel (both
 * 16-byte plane chunks and the counter word), with the addresses read from
 * the trace instead of computed from the previous step -- no dependence, and
 * `unroll` K-steps of loads in flight per lane.  Its line rate bounds what any
 * issue order can get from the request stream the search must make.
 *
 * Trace entry (u32 per end): line index (bits 0-24), block parity (25), code
 * c (26-29), bit 31 = R in L's block (the kernel loads nothing for it).
 * Layout [step][read][end]: 8 bytes per read per K-step, read coalesced by the
 * replay (a sequential stream beside the random lines; its requests are
 * reported as trace_bytes).
 */
#include <hip/hip_runtime.h>

#include "kfmi_runtime.h"

namespace kfmi {
namespace {

using GM = Geo<2, 2, LAY_MID>;
constexpr uint32_t LINE_BITS = 25;

__global__ __launch_bounds__(256) void trace_lines_kernel(IdxArgs ix, const uint32_t* __restrict__ qp, uint64_t num,
                                                          uint32_t steps, uint32_t* __restrict__ trace)
{
  const uint64_t q = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (q >= num) return;
  uint32_t L = 0, R = ix.bwtsize;
  for (uint32_t t = 0; t < steps; ++t) {
    const uint32_t word = qp[(uint64_t) (t / GM::SPW) * num + q];
    const uint32_t c = (word >> (2 * GM::K * (t % GM::SPW))) & (uint32_t) (GM::NC - 1);
    const uint32_t bl = L / (uint32_t) GM::D, br = R / (uint32_t) GM::D;
    uint2 e;
    e.x = (bl >> 1) | ((bl & 1u) << LINE_BITS) | (c << 26);
    e.y = (br >> 1) | ((br & 1u) << LINE_BITS) | (c << 26) | (br == bl ? 0x80000000u : 0u);
    reinterpret_cast<uint2*>(trace)[(uint64_t) t * num + q] = e;
    uint32_t sx[2 * GM::K];
    plane_xor<GM::K>(c, sx);
    L = lf_stream<GM>(ix, L, c, sx);
    R = lf_stream<GM>(ix, R, c, sx);
  }
}

/* the task kernel's loads for one end: block b's two 16-B plane chunks and the
 * counter word of code c in its MID128 line */
__device__ __forceinline__ uint32_t replay_end(const uint32_t* __restrict__ ent, uint32_t e)
{
  const uint32_t* line = ent + (uint64_t) (e & ((1u << LINE_BITS) - 1u)) * GM::EW;
  const uint32_t* pl = line + ((e >> LINE_BITS) & 1u) * GM::BMW;
  const uint4 a = *reinterpret_cast<const uint4*>(pl);
  const uint4 b = *reinterpret_cast<const uint4*>(pl + 4);
  const uint32_t cnt = line[GM::MIDCNT + ((e >> 26) & 15u)];
  return a.x ^ a.w ^ b.y ^ b.z ^ cnt;
}

template <int U>
__global__ __launch_bounds__(256) void replay_lines_kernel(const uint32_t* __restrict__ ent,
                                                           const uint32_t* __restrict__ trace, uint64_t num,
                                                           uint32_t steps, uint32_t* __restrict__ sink)
{
  const uint64_t q = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (q >= num) return;
  const uint2* tr = reinterpret_cast<const uint2*>(trace);
  uint32_t acc = 0;
  for (uint32_t t = 0; t < steps; t += U) {
    uint2 e[U];
#pragma unroll
    for (int u = 0; u < U; ++u) e[u] = t + u < steps ? tr[(uint64_t) (t + u) * num + q] : make_uint2(0u, 0x80000000u);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc ^= replay_end(ent, e[u].x);
      if (!(e[u].y >> 31)) acc ^= replay_end(ent, e[u].y);
    }
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;   /* keeps the loads; practically never stored */
}

template <int U>
hipError_t launch_replay(const uint32_t* ent, const uint32_t* trace, uint64_t num, uint32_t steps, uint32_t* sink,
                         hipStream_t st)
{
  const uint64_t blocks = (num + 255) / 256;
  hipLaunchKernelGGL((replay_lines_kernel<U>), dim3((uint32_t) blocks), dim3(256), 0, st, ent, trace, num, steps, sink);
  return hipGetLastError();
}

}  // namespace
}  // namespace kfmi

using namespace kfmi;

/* Diagnostic (not in the reference): replays the MID128 line requests of a
 * search of `queries` on `index` (uploaded for task-mid or coop-mid, K = 2,
 * d = 64, m % K == 0).  `unroll` (1, 2, 4 or 8): K-steps of loads in flight
 * per lane; `reps` timed launches after one warm-up.  Out: mean replay launch
 * time (ms), the lines the replay fetches per launch (L's line every step, R's
 * where it lies in another block -- the fetches of the task kernel), and the
 * trace bytes it streams beside them. */
extern "C" int32_t kfmi_probe_replay(void* index, void* queries, int32_t unroll, int32_t reps, double* ms,
                                     uint64_t* lines, uint64_t* trace_bytes)
{
  kfmi_fmi_t* f = (kfmi_fmi_t*) index;
  kfmi_qrys_t* q = (kfmi_qrys_t*) queries;
  if (!f || !q || !ms || !lines || !trace_bytes || reps < 1) return KFMI_E_BAD_ARGUMENT;
  if (unroll != 1 && unroll != 2 && unroll != 4 && unroll != 8) return KFMI_E_BAD_ARGUMENT;
  DeviceGuard dg;
  std::shared_lock<RwLock> lk(index_lock(f));
  if (!f->dev || !q->dev || f->grp || q->grp) return KFMI_E_NOT_ON_DEVICE;
  kfmi_dev_index* di = f->dev;
  kfmi_dev_queries* dq = q->dev;
  if (di->layout != LAY_MID || di->K != 2 || di->nb != 2 || dq->K != 2 || dq->rem) return KFMI_E_BAD_ARGUMENT;
  if (dq->device != di->device || di->ent_bytes / (GM::EW * 4) >= (1ull << LINE_BITS)) return KFMI_E_BAD_ARGUMENT;
  DevCtx* ctx = nullptr;
  int32_t err = ctx_for(di->device, &ctx);
  if (err) return err;
  const uint64_t num = dq->num, steps = dq->steps, tbytes = 8ull * steps * num;
  uint32_t* trace = nullptr;
  uint32_t* sink = nullptr;
  unsigned long long* d_total = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  HIP_OK(hipMalloc((void**) &trace, tbytes ? tbytes : 8));
  bool ok = hipMalloc((void**) &sink, 4) == hipSuccess && hipMalloc((void**) &d_total, 8) == hipSuccess &&
            hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess &&
            hipMemsetAsync(d_total, 0, 8, ctx->st) == hipSuccess && launch_pack(dq, ctx->st) == hipSuccess;
  const IdxArgs ix = idx_args(di);
  const uint64_t blocks = (num + 255) / 256;
  if (ok && num) {
    hipLaunchKernelGGL(trace_lines_kernel, dim3((uint32_t) blocks), dim3(256), 0, ctx->st, ix, dq->packed, num,
                       (uint32_t) steps, trace);
    /* the fetched lines: count_blocks' distinct blocks (L's, and R's when it differs) */
    SearchLaunch a{};
    a.st = ctx->st;
    a.ix = ix;
    a.qp = dq->packed;
    a.num = num;
    a.steps = dq->steps;
    a.nwords = dq->nwords;
    ok = hipGetLastError() == hipSuccess && dispatch(Op::Count, 2, 2, LAY_MID, a, d_total) == hipSuccess;
  }
  auto run = [&]() -> bool {
    switch (unroll) {
      case 1: return launch_replay<1>(di->ent, trace, num, (uint32_t) steps, sink, ctx->st) == hipSuccess;
      case 2: return launch_replay<2>(di->ent, trace, num, (uint32_t) steps, sink, ctx->st) == hipSuccess;
      case 4: return launch_replay<4>(di->ent, trace, num, (uint32_t) steps, sink, ctx->st) == hipSuccess;
      default: return launch_replay<8>(di->ent, trace, num, (uint32_t) steps, sink, ctx->st) == hipSuccess;
    }
  };
  float total_ms = 0.f;
  unsigned long long total = 0;
  if (ok && num) {
    ok = run() && hipEventRecord(e0, ctx->st) == hipSuccess;
    for (int i = 0; ok && i < reps; ++i) ok = run();
    ok = ok && hipEventRecord(e1, ctx->st) == hipSuccess && hipEventSynchronize(e1) == hipSuccess &&
         hipEventElapsedTime(&total_ms, e0, e1) == hipSuccess &&
         hipMemcpy(&total, d_total, 8, hipMemcpyDeviceToHost) == hipSuccess;
  }
  if (e0) (void) hipEventDestroy(e0);
  if (e1) (void) hipEventDestroy(e1);
  (void) hipFree(d_total);
  (void) hipFree(sink);
  (void) hipFree(trace);
  if (!ok) return KFMI_E_KERNEL;
  *ms = (double) total_ms / reps;
  *lines = total;
  *trace_bytes = tbytes;
  return KFMI_SUCCESS;
}
