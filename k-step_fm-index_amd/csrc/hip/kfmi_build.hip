/*
 * kfmi_build.hip -- GPU index builder for MI355X (reference genFMindex.c:457-543,
 * re-designed for the device; output is bit-identical to the reference
 * builder's tag-100 file, pinned by md5 in tests).
 *
 * Pipeline (all on one device, 3 Gbase K=2 d=64 peaks at ~80 GB of HBM):
 *   1. encode   : ASCII -> 2-bit text, 16 bases per u32 (MSB first); non-ACGT rejected
 *   2. keys     : key(i) = the 32 bases starting at i (bases past the end read as A)
 *   3. sort     : rocPRIM onesweep radix sort of (key, i) pairs, 64-bit keys
 *   4. ties     : equal adjacent keys (repeats >= 32 bases, or short suffixes whose
 *                 padding matches) are re-ordered on the host by full suffix
 *                 comparison ('$' lowest); random genomic text has ~none
 *   5. blocks   : one wave64 per d-block; lane = row.  Each lane derives its row's
 *                 K-mer code from SA (BWT_s[r] = T$[(SA[r]-1-s) mod (n+1)], '$'->A);
 *                 the 2K bit planes are __ballot()s (bit-reversed into the
 *                 MSB-first plane words) and the per-code row counts (with the
 *                 '$' rows excluded) are popcounts of ANDed ballots
 *   6. scan     : per-code exclusive scan over blocks (rocPRIM) -> Occ at block start
 *   7. counters : cnt_b[c] = Occ + C'[c]   (C' on the host from the totals, :237-250)
 */
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

#include "../kfmi_internal.h"

namespace {

#define BHIP(x)                                                                            \
  do {                                                                                     \
    hipError_t _e = (x);                                                                   \
    if (_e != hipSuccess) {                                                                \
      fprintf(stderr, "kstepfmi build: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(_e), \
              __FILE__, __LINE__);                                                         \
      return KFMI_E_BUILDING_BWT;                                                          \
    }                                                                                      \
  } while (0)

__global__ __launch_bounds__(256) void k_encode(const uint8_t* __restrict__ ascii, uint64_t n,
                                                uint32_t* __restrict__ packed, uint64_t nwords,
                                                uint32_t* __restrict__ bad)
{
  const uint64_t w = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (w >= nwords) return;
  uint32_t word = 0, inval = 0;
  const uint64_t i0 = w * 16;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint64_t i = i0 + j;
    uint32_t c = 0;
    if (i < n) {
      const uint8_t x = ascii[i];
      c = x == 'A' ? 0u : x == 'C' ? 1u : x == 'G' ? 2u : x == 'T' ? 3u : 4u;
      if (c == 4u) { inval = 1; c = 0; }
    }
    word |= c << (30 - 2 * j);
  }
  packed[w] = word;
  if (inval) atomicOr(bad, 1u);
}

__device__ __forceinline__ uint32_t base_at(const uint32_t* __restrict__ packed, uint64_t i)
{
  return (packed[i >> 4] >> (30 - 2 * (i & 15))) & 3u;
}

__global__ __launch_bounds__(256) void k_keys(const uint32_t* __restrict__ packed, uint64_t n,
                                              uint64_t* __restrict__ keys, uint32_t* __restrict__ vals)
{
  const uint64_t i = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint64_t w = i >> 4;
  const uint32_t sh = (uint32_t) (i & 15) * 2;
  const uint64_t a = packed[w], b = packed[w + 1], c = packed[w + 2];
  uint64_t k = ((a << 32) | b) << sh;
  if (sh) k |= c >> (32 - sh);
  keys[i] = k;
  vals[i] = (uint32_t) i;
}

__global__ __launch_bounds__(256) void k_ties(const uint64_t* __restrict__ keys, uint64_t n,
                                              uint32_t* __restrict__ list, uint32_t cap,
                                              unsigned long long* __restrict__ count)
{
  const uint64_t i = (uint64_t) blockIdx.x * 256 + threadIdx.x + 1;
  if (i >= n) return;
  if (keys[i] == keys[i - 1]) {
    const unsigned long long slot = atomicAdd(count, 1ull);
    if (slot < cap) list[slot] = (uint32_t) i;
  }
}

__global__ __launch_bounds__(256) void k_dollar(const uint32_t* __restrict__ sa, uint64_t n, uint32_t k,
                                                uint32_t* __restrict__ drow)
{
  const uint64_t j = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const uint32_t v = sa[j];
  if (v < k) drow[v] = (uint32_t) (j + 1);    /* row of T$ = sorted index + 1 ('$' row is 0) */
}

/* One wave per d-block; lane = row inside a 64-row chunk. */
template <int K>
__global__ __launch_bounds__(256) void k_blocks(const uint32_t* __restrict__ sa, const uint32_t* __restrict__ packed,
                                                uint64_t n, uint32_t d, uint32_t nentries, uint32_t d0, uint32_t d1,
                                                uint32_t d2, uint32_t d3, uint32_t* __restrict__ entries,
                                                uint32_t* __restrict__ counts)
{
  constexpr int NC = 1 << (2 * K);
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b = (uint64_t) blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= nentries) return;
  const uint32_t nb = d / 32;
  const uint32_t ew = 2 * nb * K + NC;
  const uint64_t rows = n + 1;
  const uint32_t drows[4] = {d0, d1, d2, d3};
  uint32_t* ent = entries + b * ew;
  constexpr int CPL = (NC + 63) / 64;   /* codes per lane: lane handles c = lane + 64*i */
  uint32_t cnt[CPL];
#pragma unroll
  for (int i = 0; i < CPL; ++i) cnt[i] = 0;
  for (uint32_t base = 0; base < d; base += 64) {
    const uint64_t r = b * d + base + lane;
    const bool valid = (base + lane < d) && (r < rows);
    uint32_t code = 0;
    bool isd = false;
    if (valid) {
      const uint64_t s_a = r == 0 ? n : (uint64_t) sa[r - 1];
#pragma unroll
      for (int s = 0; s < K; ++s) {
        int64_t pos = (int64_t) s_a - 1 - s;
        if (pos < 0) pos += (int64_t) rows;
        const uint32_t cs = ((uint64_t) pos == n) ? 0u : base_at(packed, (uint64_t) pos);
        code |= cs << (2 * s);
      }
#pragma unroll
      for (int s = 0; s < K; ++s) isd |= (drows[s] == (uint32_t) r);
    }
    uint64_t plane[2 * K];
#pragma unroll
    for (int p = 0; p < 2 * K; ++p) plane[p] = __ballot(valid && ((code >> p) & 1u));
    const uint64_t live = __ballot(valid && !isd);
    /* plane words: rows base..base+31 -> word base/32, row p at bit 31-p */
    const uint32_t w0 = base / 32;
    if (lane < 2 * K) {
      const int p = lane;              /* p = 2s + t */
      const int s = p >> 1, t = p & 1;
      const uint32_t lo = __builtin_bitreverse32((uint32_t) plane[p]);
      const uint32_t hi = __builtin_bitreverse32((uint32_t) (plane[p] >> 32));
      ent[s * 2 * nb + t * nb + w0] = lo;
      if (w0 + 1 < nb) ent[s * 2 * nb + t * nb + w0 + 1] = hi;
    }
    /* per-code counts: lane c counts rows whose planes all match c */
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const uint32_t c = lane + 64 * i;
      if (c < (uint32_t) NC) {
        uint64_t m = live;
#pragma unroll
        for (int p = 0; p < 2 * K; ++p) m &= ((c >> p) & 1u) ? plane[p] : ~plane[p];
        cnt[i] += (uint32_t) __popcll(m);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const uint32_t c = lane + 64 * i;
    if (c < (uint32_t) NC) counts[(uint64_t) c * nentries + b] = cnt[i];
  }
}

__global__ __launch_bounds__(256) void k_fill(const uint32_t* __restrict__ occ, uint32_t nentries, uint32_t nc,
                                              uint32_t cntoff, uint32_t ew, const uint32_t* __restrict__ cprime,
                                              uint32_t* __restrict__ entries)
{
  const uint64_t b = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (b >= nentries) return;
  uint32_t* e = entries + b * ew + cntoff;
  for (uint32_t c = 0; c < nc; ++c) e[c] = occ[(uint64_t) c * nentries + b] + cprime[c];
}

/* row-sampled suffix array: out[i] = SA[i * rate] (row 0 is the '$' suffix, SA = n) */
__global__ __launch_bounds__(256) void k_sample(const uint32_t* __restrict__ sa, uint64_t n, uint32_t rate,
                                                uint64_t count, uint32_t* __restrict__ out)
{
  const uint64_t i = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (i >= count) return;
  const uint64_t r = i * rate;
  out[i] = r == 0 ? (uint32_t) n : sa[r - 1];
}

struct DevBuf {
  void* p = nullptr;
  ~DevBuf() { if (p) (void) hipFree(p); }
  hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes ? bytes : 1); }
  template <class T> T* as() { return reinterpret_cast<T*>(p); }
  void release() { if (p) (void) hipFree(p); p = nullptr; }
};

/* '$'-aware full suffix comparison on the host text (the tie breaker). */
struct SuffixLess {
  const char* t;
  uint64_t n;
  bool operator()(uint32_t a, uint32_t b) const
  {
    const uint64_t la = n - a, lb = n - b, l = std::min(la, lb);
    const int c = memcmp(t + a, t + b, l);
    if (c) return c < 0;
    return la < lb;   /* the shorter suffix hits '$' first */
  }
};

int32_t build_gpu(const char* text, uint64_t n, uint32_t k, uint32_t d, uint32_t sa_rate, int dev, kfmi_fmi_t** out)
{
  /* n + 1 >= k: every D_s (s < k) exists -- SA = s is a suffix of T for s < n and
   * the '$' row 0 for s == n -- and (SA - 1 - s) wraps at most once. */
  if (n == 0 || n + 1 < k || n + 1 > 0xFFFFFFFEull || k < 1 || k > 4 || d == 0 || d % 32)
    return KFMI_E_BAD_ARGUMENT;
  /* one thread per base: a dispatch holds at most 2^32 - 1 work-items */
  if (n > 0xFFFFFF00ull) return KFMI_E_NOT_IMPLEMENTED;   /* caller falls back to the host builder */
  BHIP(hipSetDevice(dev));
  hipStream_t st;
  BHIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  struct StreamGuard { hipStream_t s; ~StreamGuard() { (void) hipStreamDestroy(s); } } sg{st};

  const uint64_t rows = n + 1;
  const uint32_t nentries = (uint32_t) ((rows + d - 1) / d);
  const uint32_t nc = 1u << (2 * k), nb = d / 32;
  const uint64_t nwords = (n + 15) / 16 + 4;

  /* 1. encode */
  DevBuf packed, bad;
  BHIP(packed.alloc(nwords * 4));
  BHIP(bad.alloc(4));
  BHIP(hipMemsetAsync(bad.p, 0, 4, st));
  {
    DevBuf ascii;
    BHIP(ascii.alloc(n));
    BHIP(hipMemcpyAsync(ascii.p, text, n, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_encode, dim3((uint32_t) ((nwords + 255) / 256)), dim3(256), 0, st, ascii.as<uint8_t>(), n,
                       packed.as<uint32_t>(), nwords, bad.as<uint32_t>());
    BHIP(hipGetLastError());
    uint32_t hbad = 0;
    BHIP(hipMemcpyAsync(&hbad, bad.p, 4, hipMemcpyDeviceToHost, st));
    BHIP(hipStreamSynchronize(st));
    if (hbad) return KFMI_E_BUILDING_BWT;   /* non-ACGT text (see fmi_build.c) */
  }

  /* 2-3. keys and radix sort */
  DevBuf sa;
  BHIP(sa.alloc(n * 4));
  {
    DevBuf k0, k1, v0, tmp;
    BHIP(k0.alloc(n * 8));
    BHIP(k1.alloc(n * 8));
    BHIP(v0.alloc(n * 4));
    hipLaunchKernelGGL(k_keys, dim3((uint32_t) ((n + 255) / 256)), dim3(256), 0, st, packed.as<uint32_t>(), n,
                       k0.as<uint64_t>(), v0.as<uint32_t>());
    BHIP(hipGetLastError());
    rocprim::double_buffer<uint64_t> kb(k0.as<uint64_t>(), k1.as<uint64_t>());
    rocprim::double_buffer<uint32_t> vb(v0.as<uint32_t>(), sa.as<uint32_t>());
    size_t tbytes = 0;
    BHIP(rocprim::radix_sort_pairs(nullptr, tbytes, kb, vb, (size_t) n, 0, 64, st));
    BHIP(tmp.alloc(tbytes));
    BHIP(rocprim::radix_sort_pairs(tmp.p, tbytes, kb, vb, (size_t) n, 0, 64, st));
    if (vb.current() != sa.as<uint32_t>())
      BHIP(hipMemcpyAsync(sa.p, vb.current(), n * 4, hipMemcpyDeviceToDevice, st));

    /* 4. ties */
    const uint32_t cap = 1u << 24;
    DevBuf list, cntb;
    BHIP(list.alloc((size_t) cap * 4));
    BHIP(cntb.alloc(8));
    BHIP(hipMemsetAsync(cntb.p, 0, 8, st));
    if (n > 1)
      hipLaunchKernelGGL(k_ties, dim3((uint32_t) ((n - 1 + 255) / 256)), dim3(256), 0, st, kb.current(), n,
                         list.as<uint32_t>(), cap, cntb.as<unsigned long long>());
    BHIP(hipGetLastError());
    unsigned long long nties = 0;
    BHIP(hipMemcpyAsync(&nties, cntb.p, 8, hipMemcpyDeviceToHost, st));
    BHIP(hipStreamSynchronize(st));
    if (nties > cap) return KFMI_E_NOT_IMPLEMENTED;   /* too repetitive: caller uses the host builder */
    if (nties) {
      std::vector<uint32_t> idx(nties);
      BHIP(hipMemcpy(idx.data(), list.p, nties * 4, hipMemcpyDeviceToHost));
      std::sort(idx.begin(), idx.end());
      SuffixLess less{text, n};
      size_t i = 0;
      while (i < idx.size()) {
        size_t j = i;
        while (j + 1 < idx.size() && idx[j + 1] == idx[j] + 1) ++j;
        const uint64_t lo = idx[i] - 1, hi = idx[j];   /* run of equal keys [lo, hi] */
        std::vector<uint32_t> grp(hi - lo + 1);
        BHIP(hipMemcpy(grp.data(), sa.as<uint32_t>() + lo, grp.size() * 4, hipMemcpyDeviceToHost));
        std::sort(grp.begin(), grp.end(), less);
        BHIP(hipMemcpy(sa.as<uint32_t>() + lo, grp.data(), grp.size() * 4, hipMemcpyHostToDevice));
        i = j + 1;
      }
    }
  }

  /* 5. '$' rows and blocks */
  uint32_t drow[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  if (n < 4) drow[n] = 0;   /* SA[0] = n: the '$' row */
  {
    DevBuf dd;
    BHIP(dd.alloc(16));
    BHIP(hipMemcpyAsync(dd.p, drow, 16, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_dollar, dim3((uint32_t) ((n + 255) / 256)), dim3(256), 0, st, sa.as<uint32_t>(), n, k,
                       dd.as<uint32_t>());
    BHIP(hipGetLastError());
    BHIP(hipMemcpyAsync(drow, dd.p, 16, hipMemcpyDeviceToHost, st));
    BHIP(hipStreamSynchronize(st));
    /* suffix s < K always exists when n >= K; for n < K the missing ones never match */
  }
  kfmi_fmi_t* f = nullptr;
  int32_t err = kfmi_index_alloc(100, k, (uint32_t) rows, nentries, d, nullptr, nullptr, &f);
  if (err) return err;
  const uint32_t ew = f->entry_words;
  DevBuf ent, counts, occ, cp;
  auto fail = [&](int32_t e) { freeIndex((void**) &f); return e; };
  if (ent.alloc((uint64_t) ew * 4 * nentries) != hipSuccess || counts.alloc((uint64_t) nc * 4 * nentries) != hipSuccess ||
      occ.alloc((uint64_t) nc * 4 * nentries) != hipSuccess || cp.alloc(4 * nc) != hipSuccess)
    return fail(KFMI_E_ALLOCATING_FMI);
  if (hipMemsetAsync(ent.p, 0, (uint64_t) ew * 4 * nentries, st) != hipSuccess) return fail(KFMI_E_BUILDING_FMI);
  {
    const dim3 grid((nentries + 3) / 4);
    hipError_t le;
    switch (k) {
      case 1: hipLaunchKernelGGL((k_blocks<1>), grid, dim3(256), 0, st, sa.as<uint32_t>(), packed.as<uint32_t>(), n, d,
                                 nentries, drow[0], drow[1], drow[2], drow[3], ent.as<uint32_t>(), counts.as<uint32_t>()); break;
      case 2: hipLaunchKernelGGL((k_blocks<2>), grid, dim3(256), 0, st, sa.as<uint32_t>(), packed.as<uint32_t>(), n, d,
                                 nentries, drow[0], drow[1], drow[2], drow[3], ent.as<uint32_t>(), counts.as<uint32_t>()); break;
      case 3: hipLaunchKernelGGL((k_blocks<3>), grid, dim3(256), 0, st, sa.as<uint32_t>(), packed.as<uint32_t>(), n, d,
                                 nentries, drow[0], drow[1], drow[2], drow[3], ent.as<uint32_t>(), counts.as<uint32_t>()); break;
      default: hipLaunchKernelGGL((k_blocks<4>), grid, dim3(256), 0, st, sa.as<uint32_t>(), packed.as<uint32_t>(), n, d,
                                  nentries, drow[0], drow[1], drow[2], drow[3], ent.as<uint32_t>(), counts.as<uint32_t>()); break;
    }
    le = hipGetLastError();
    if (le != hipSuccess) return fail(KFMI_E_BUILDING_FMI);
  }
  if (sa_rate) {   /* locate samples, before the SA is released */
    err = kfmi_sa_alloc(f, sa_rate);
    if (err) return fail(err);
    DevBuf smp;
    if (smp.alloc(4 * f->sa_count) != hipSuccess) return fail(KFMI_E_ALLOCATING_FMI);
    hipLaunchKernelGGL(k_sample, dim3((uint32_t) ((f->sa_count + 255) / 256)), dim3(256), 0, st, sa.as<uint32_t>(), n,
                       sa_rate, f->sa_count, smp.as<uint32_t>());
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(f->h_sa, smp.p, 4 * f->sa_count, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return fail(KFMI_E_BUILDING_FMI);
  }
  sa.release();
  /* 6. per-code exclusive scans over blocks */
  {
    size_t tb = 0;
    if (rocprim::exclusive_scan(nullptr, tb, counts.as<uint32_t>(), occ.as<uint32_t>(), 0u, (size_t) nentries,
                                rocprim::plus<uint32_t>(), st) != hipSuccess)
      return fail(KFMI_E_BUILDING_FMI);
    DevBuf tmp;
    if (tmp.alloc(tb) != hipSuccess) return fail(KFMI_E_ALLOCATING_FMI);
    for (uint32_t c = 0; c < nc; ++c)
      if (rocprim::exclusive_scan(tmp.p, tb, counts.as<uint32_t>() + (uint64_t) c * nentries,
                                  occ.as<uint32_t>() + (uint64_t) c * nentries, 0u, (size_t) nentries,
                                  rocprim::plus<uint32_t>(), st) != hipSuccess)
        return fail(KFMI_E_BUILDING_FMI);
  }
  /* 7. C' and counters */
  std::vector<uint32_t> lastocc(nc), lastcnt(nc), cprime(nc);
  for (uint32_t c = 0; c < nc; ++c) {
    if (hipMemcpyAsync(&lastocc[c], occ.as<uint32_t>() + (uint64_t) c * nentries + nentries - 1, 4,
                       hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(&lastcnt[c], counts.as<uint32_t>() + (uint64_t) c * nentries + nentries - 1, 4,
                       hipMemcpyDeviceToHost, st) != hipSuccess)
      return fail(KFMI_E_BUILDING_FMI);
  }
  if (hipStreamSynchronize(st) != hipSuccess) return fail(KFMI_E_BUILDING_FMI);
  /* dollarBaseBWT[s] = c(D_s): SA[D_s] = s, so BWT_s'[D_s] = T$[(s-1-s') mod (n+1)] */
  uint32_t dbase[4] = {0, 0, 0, 0};
  for (uint32_t s = 0; s < k; ++s) {
    uint32_t code = 0;
    for (uint32_t s2 = 0; s2 < k; ++s2) {
      int64_t pos = (int64_t) s - 1 - (int64_t) s2;
      if (pos < 0) pos += (int64_t) rows;
      uint32_t cs = 0;
      if ((uint64_t) pos != n) {
        const char ch = text[pos];
        cs = ch == 'A' ? 0u : ch == 'C' ? 1u : ch == 'G' ? 2u : 3u;
      }
      code |= cs << (2 * s2);
    }
    dbase[s] = code;
  }
  {
    uint64_t acc = 0;
    for (uint32_t c = 0; c < nc; ++c) {
      cprime[c] = (uint32_t) acc;
      acc += (uint64_t) lastocc[c] + lastcnt[c];
    }
    for (uint32_t s = 0; s < k; ++s) {
      const uint32_t masked = dbase[s] & (0xFFFFFFFFu << (2 * s));
      for (uint32_t c = masked; c < nc; ++c) cprime[c]++;
    }
  }
  if (hipMemcpyAsync(cp.p, cprime.data(), 4 * nc, hipMemcpyHostToDevice, st) != hipSuccess) return fail(KFMI_E_BUILDING_FMI);
  hipLaunchKernelGGL(k_fill, dim3((nentries + 255) / 256), dim3(256), 0, st, occ.as<uint32_t>(), nentries, nc,
                     2 * nb * k, ew, cp.as<uint32_t>(), ent.as<uint32_t>());
  if (hipGetLastError() != hipSuccess ||
      hipMemcpyAsync(f->h_index, ent.p, (uint64_t) ew * 4 * nentries, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return fail(KFMI_E_BUILDING_FMI);
  for (uint32_t s = 0; s < k; ++s) {
    f->dollarPositionBWT[s] = drow[s];
    f->dollarBaseBWT[s] = dbase[s];
    f->modposdollarBWT[s] = drow[s] / d;
  }
  const void* img;
  uint64_t bytes;
  kfmi_index_image(f, &img, &bytes);   /* refresh the header words */
  *out = f;
  return KFMI_SUCCESS;
}

}  // namespace

extern "C" int32_t kfmi_build_index_gpu_sa(const char* text, uint64_t n, uint32_t k, uint32_t d, uint32_t sa_rate,
                                           void** index)
{
  if (sa_rate && !kfmi_sa_rate_ok(sa_rate)) return KFMI_E_BAD_ARGUMENT;
  if (kfmi_device_count() < 1) return KFMI_E_NO_DEVICE;
  int32_t e = build_gpu(text, n, k, d, sa_rate, kfmi_current_device(), (kfmi_fmi_t**) index);
  if (e == KFMI_E_NOT_IMPLEMENTED) {
    fprintf(stderr, "kstepfmi build: text too repetitive for the GPU tie breaker, using the host builder\n");
    return kfmi_build_index_cpu_sa(text, n, k, d, sa_rate, index);
  }
  return e;
}

extern "C" int32_t kfmi_build_index_gpu(const char* text, uint64_t n, uint32_t k, uint32_t d,
                                        int32_t want_host_image, void** index)
{
  (void) want_host_image;   /* the host image is always produced (saveIndex, oracle, md5 pins) */
  return kfmi_build_index_gpu_sa(text, n, k, d, 0, index);
}
