/*
 * kfmi_ingest.hip -- multi-FASTA queries parsed on the device (SURVEY 8(f) f2,
 * "FASTA parse ... on the GPU").
 *
 * kfmi_load_queries_gpu reads the file in 64 MB pieces straight into two
 * pinned staging buffers (pread split over the host workers) and DMAs each to
 * the device while the next is read, then does on the device what loadQueries
 * does on the host (reference common/common.c:132-199 semantics, restated in
 * csrc/host/common.c: '>' lines skipped, every other line one read of exactly
 * m bytes after its trailing '\r's, reads past `num` ignored, a malformed read
 * before the num-th or too few reads = KFMI_E_READING_MFASTA_FILE):
 *
 *   fa_count  -- per 64 KiB tile (one workgroup, 256 B per thread, 16-B loads),
 *                the read lines that start in the tile;
 *   rocPRIM exclusive scan of the tile counts -> each tile's first read number;
 *   fa_starts -- the same walk with a workgroup prefix sum: the start offset of
 *                every read, by read number;
 *   fa_rows   -- one thread per 4 output bytes: the reads into the plain
 *                num x m layout the search kernels stage from (coalesced 4-B
 *                stores; the loads walk each read's bytes, near-contiguous in
 *                the file), flagging a read with a '\n' inside its first m bytes
 *                or anything but '\r'* then '\n' / end of file after them.
 *
 * The reads stay on the device (h_queries NULL): transferCPUtoGPU takes them
 * as they are, searchIndexGPU packs them in its kernels as usual.
 */
#include <fcntl.h>
#include <stdlib.h>
#include <sys/stat.h>
#include <unistd.h>
#include <new>

#include <rocprim/device/device_scan.hpp>

#include "kfmi_runtime.h"

namespace kfmi {

constexpr uint32_t FA_TILE = 65536;          /* bytes per workgroup */
constexpr uint32_t FA_SEG = FA_TILE / 256;   /* bytes per thread: 16 x 16-B loads */
constexpr uint64_t FA_PAD = 1024;            /* zero bytes after the file on the device */

/* Read lines starting in this thread's 256 bytes [seg, seg+256); with WRITE,
 * their offsets go to starts[base + k] (k-th such line) while base + k < cap. */
template <bool WRITE>
__device__ __forceinline__ uint32_t fa_walk(const uint8_t* __restrict__ raw, uint64_t n, uint64_t seg,
                                            uint64_t* __restrict__ starts, uint64_t base, uint64_t cap)
{
  uint32_t prev = seg == 0 ? (uint32_t) '\n' : raw[seg - 1];
  uint32_t cnt = 0;
  const uint4* v = reinterpret_cast<const uint4*>(raw + seg);
#pragma unroll 4
  for (int k = 0; k < (int) (FA_SEG / 16); ++k) {
    const uint4 q = v[k];
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int h = 0; h < 4; ++h) {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t cur = (w[h] >> (8 * b)) & 0xFFu;
        const uint64_t i = seg + 16 * k + 4 * h + b;
        if (prev == '\n' && cur != '>' && i < n) {
          if constexpr (WRITE) {
            if (base + cnt < cap) starts[base + cnt] = i;
          }
          ++cnt;
        }
        prev = cur;
      }
    }
  }
  return cnt;
}

__global__ __launch_bounds__(256) void fa_count(const uint8_t* __restrict__ raw, uint64_t n,
                                                uint32_t* __restrict__ tile_cnt)
{
  __shared__ uint32_t part[4];
  const uint64_t seg = (uint64_t) blockIdx.x * FA_TILE + (uint64_t) threadIdx.x * FA_SEG;
  uint32_t c = fa_walk<false>(raw, n, seg, nullptr, 0, 0);
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) tile_cnt[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

__global__ __launch_bounds__(256) void fa_starts(const uint8_t* __restrict__ raw, uint64_t n,
                                                 const uint64_t* __restrict__ tile_base, uint64_t cap,
                                                 uint64_t* __restrict__ starts)
{
  __shared__ uint32_t wsum[4];
  const uint64_t seg = (uint64_t) blockIdx.x * FA_TILE + (uint64_t) threadIdx.x * FA_SEG;
  const uint32_t c = fa_walk<false>(raw, n, seg, nullptr, 0, 0);
  /* exclusive prefix of c over the workgroup: inclusive wave scan + wave offsets */
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t inc = c;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(inc, off);
    if (lane >= (uint32_t) off) inc += y;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  uint32_t woff = 0;
  for (uint32_t k = 0; k < wv; ++k) woff += wsum[k];
  const uint64_t base = tile_base[blockIdx.x] + woff + inc - c;
  if (c && base < cap) fa_walk<true>(raw, n, seg, starts, base, cap);
}

__global__ __launch_bounds__(256) void fa_rows(const uint8_t* __restrict__ raw, uint64_t n,
                                               const uint64_t* __restrict__ starts, uint64_t num, uint32_t m,
                                               uint32_t* __restrict__ out, unsigned long long* __restrict__ first_bad)
{
  const uint64_t total = num * m;
  /* grid-stride: more than 16 GB of reads exceed the 2^32 work-items of one dispatch */
  for (uint64_t w = (uint64_t) blockIdx.x * 256 + threadIdx.x; 4 * w < total; w += (uint64_t) gridDim.x * 256) {
    uint32_t word = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint64_t o = 4 * w + b;
      if (o >= total) break;
      const uint64_t q = o / m;
      const uint32_t j = (uint32_t) (o - q * m);
      const uint64_t s = starts[q] + j;
      const uint32_t ch = s < n ? raw[s] : (uint32_t) '\n';   /* past the end: the read is short */
      bool bad = ch == '\n';
      if (j == m - 1 && !bad) {   /* what follows the read: '\r'* then '\n' or the end of the file */
        /* and the read's last byte is not one of the line's trailing '\r's
         * (the host reader strips those first: "ACG\r" is a 3-base read) */
        uint64_t p = s + 1;
        while (p < n && raw[p] == '\r') ++p;
        bad = ch == '\r' || !(p >= n || raw[p] == '\n');
      }
      if (bad) atomicMin(first_bad, (unsigned long long) q);
      word |= ch << (8 * b);
    }
    out[w] = word;
  }
}

/* The file into device memory at dst (n bytes), through the device's two
 * pinned 64 MB upload buffers (kept between calls: pinning them per call cost
 * 42 ms, copy_probe): the read of one piece overlaps the DMA of the other. */
static int32_t fa_upload(int fd, uint64_t n, uint8_t* dst, DevCtx* ctx)
{
  constexpr uint64_t CH = 64ull << 20;
  const hipStream_t st = ctx->st;
  std::lock_guard<std::mutex> lk(ctx->up_mu);
  if (upload_staging(ctx, CH) != hipSuccess) return KFMI_E_ALLOCATING_MFASTA;
  int32_t err = KFMI_SUCCESS;
  for (uint64_t off = 0, i = 0; off < n && !err; off += CH, ++i) {
    const int b = (int) (i & 1);
    if (i >= 2 && hipEventSynchronize(ctx->up_ev[b]) != hipSuccess) { err = KFMI_E_KERNEL; break; }
    const uint64_t len = n - off < CH ? n - off : CH;
    if (!par_pread(fd, ctx->up_buf[b], off, len)) { err = KFMI_E_READING_MFASTA_FILE; break; }
    if (hipMemcpyAsync(dst + off, ctx->up_buf[b], len, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipEventRecord(ctx->up_ev[b], st) != hipSuccess)
      err = KFMI_E_KERNEL;
  }
  if (hipStreamSynchronize(st) != hipSuccess && !err) err = KFMI_E_KERNEL;   /* buffers free again */
  return err;
}

struct DevMem {
  void* p = nullptr;
  ~DevMem() { if (p) (void) hipFree(p); }
  hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes ? bytes : 1); }
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

extern "C" int32_t kfmi_load_queries_gpu(const char* fn, uint32_t sizequery, uint64_t numqueries, void** queries)
{
  if (!fn || !queries || sizequery == 0) return KFMI_E_BAD_ARGUMENT;
  *queries = nullptr;
  DeviceGuard dg;
  const int dev = kfmi_current_device();
  DevCtx* ctx = nullptr;
  int32_t err = ctx_for(dev, &ctx);
  if (err) return err;
  const hipStream_t st = ctx->st;
  const int fd = open(fn, O_RDONLY);
  if (fd < 0) return KFMI_E_OPENING_MFASTA_FILE;
  struct stat sb;
  if (fstat(fd, &sb) != 0 || !S_ISREG(sb.st_mode)) {
    close(fd);
    return KFMI_E_READING_MFASTA_FILE;
  }
  const uint64_t n = (uint64_t) sb.st_size;
  const uint64_t tiles = (n + FA_TILE - 1) / FA_TILE;
  DevMem raw, tcnt, tbase, starts, bad;
  if (raw.alloc(tiles * FA_TILE + FA_PAD) != hipSuccess || tcnt.alloc(4 * (tiles + 1)) != hipSuccess ||
      tbase.alloc(8 * (tiles + 1)) != hipSuccess || bad.alloc(8) != hipSuccess) {
    close(fd);
    return KFMI_E_DEVICE_ALLOC;
  }
  err = n ? fa_upload(fd, n, raw.as<uint8_t>(), ctx) : KFMI_SUCCESS;
  close(fd);
  if (err) return err;
  /* zero the tail of the last tile and the pad: no line starts there (i < n) */
  HIP_OK(hipMemsetAsync(raw.as<uint8_t>() + n, 0, tiles * FA_TILE + FA_PAD - n, st));
  HIP_OK(hipMemsetAsync(tcnt.p, 0, 4 * (tiles + 1), st));
  if (tiles) {
    hipLaunchKernelGGL(fa_count, dim3((uint32_t) tiles), dim3(256), 0, st, raw.as<uint8_t>(), n, tcnt.as<uint32_t>());
    HIP_OK(hipGetLastError());
  }
  /* tile_base[t] = reads before tile t; tile_base[tiles] = all reads */
  size_t tb = 0;
  HIP_OK(rocprim::exclusive_scan(nullptr, tb, tcnt.as<uint32_t>(), tbase.as<uint64_t>(), (uint64_t) 0,
                                 (size_t) (tiles + 1), rocprim::plus<uint64_t>(), st));
  DevMem tmp;
  HIP_OK(tmp.alloc(tb));
  HIP_OK(rocprim::exclusive_scan(tmp.p, tb, tcnt.as<uint32_t>(), tbase.as<uint64_t>(), (uint64_t) 0,
                                 (size_t) (tiles + 1), rocprim::plus<uint64_t>(), st));
  uint64_t total = 0;
  HIP_OK(hipMemcpyAsync(&total, tbase.as<uint64_t>() + tiles, 8, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  const uint64_t num = numqueries ? numqueries : total;
  if (total < num) return KFMI_E_READING_MFASTA_FILE;
  if (num >= 0xFFFFFFFFull) return KFMI_E_BAD_ARGUMENT;
  kfmi_dev_queries* dq = new (std::nothrow) kfmi_dev_queries();
  if (!dq) return KFMI_E_ALLOCATING_MFASTA;
  dq->device = dev;
  dq->num = num;
  dq->size = sizequery;
  dq->nwords = (sizequery + 15) / 16;   /* K-independent (16 bases per word); K and steps set at transfer */
  const uint64_t abytes = num * (uint64_t) sizequery;
  auto fail = [&](int32_t e) { free_dev_queries(dq); return e; };
  if (hipMalloc((void**) &dq->ascii, ((abytes + 3) & ~3ull) + 16) != hipSuccess ||
      hipMalloc((void**) &dq->packed, 4ull * (dq->nwords + 1) * (num ? num : 1)) != hipSuccess)
    return fail(KFMI_E_DEVICE_ALLOC);
  dq->packed_rows = dq->nwords + 1;
  if (num) {
    if (starts.alloc(8 * num) != hipSuccess) return fail(KFMI_E_DEVICE_ALLOC);
    unsigned long long fb = ~0ull;
    bool ok = hipMemcpyAsync(bad.p, &fb, 8, hipMemcpyHostToDevice, st) == hipSuccess;
    hipLaunchKernelGGL(fa_starts, dim3((uint32_t) tiles), dim3(256), 0, st, raw.as<uint8_t>(), n, tbase.as<uint64_t>(),
                       num, starts.as<uint64_t>());
    ok = ok && hipGetLastError() == hipSuccess;
    const uint64_t words = (abytes + 3) / 4;
    const uint64_t rb = (words + 255) / 256;
    hipLaunchKernelGGL(fa_rows, dim3(grid_blocks(rb, 1u << 22)), dim3(256), 0, st, raw.as<uint8_t>(), n,
                       starts.as<uint64_t>(), num, sizequery, reinterpret_cast<uint32_t*>(dq->ascii),
                       bad.as<unsigned long long>());
    ok = ok && hipGetLastError() == hipSuccess &&
         hipMemcpyAsync(&fb, bad.p, 8, hipMemcpyDeviceToHost, st) == hipSuccess &&
         hipStreamSynchronize(st) == hipSuccess;
    if (!ok) return fail(KFMI_E_KERNEL);
    if (fb < num) return fail(KFMI_E_READING_MFASTA_FILE);
  }
  kfmi_qrys_t* q = (kfmi_qrys_t*) calloc(1, sizeof(kfmi_qrys_t));
  if (!q) return fail(KFMI_E_ALLOCATING_MFASTA);
  q->num = num;
  q->size = sizequery;
  q->h_queries = nullptr;   /* device-resident */
  q->dev = dq;
  *queries = q;
  return KFMI_SUCCESS;
}

}  // namespace kfmi
