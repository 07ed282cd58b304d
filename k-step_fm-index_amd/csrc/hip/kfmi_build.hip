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
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <mutex>
#include <vector>

#include "../kfmi_internal.h"
#include "kfmi_devguard.h"

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

/* map = 0: A/C/G/T only (anything else flagged in *bad); map = 1: every byte
 * through base2index (genFMindex.c:71-84), the "map" and "ref" alphabets */
__global__ __launch_bounds__(256) void k_encode(const uint8_t* __restrict__ ascii, uint64_t n,
                                                uint32_t* __restrict__ packed, uint64_t nwords,
                                                uint32_t* __restrict__ bad, uint32_t map)
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
      if (c == 4u) {
        if (map) c = (((uint32_t) x >> 1) & 3u) ^ (((uint32_t) x >> 2) & 1u);   /* base2index */
        else { inval = 1; c = 0; }
      }
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

/* "ref" alphabet: the key of suffix i is its first L raw bytes as dense ranks
 * of `bits` bits each (rank 0 past the end, below every byte: '$' sorts
 * lowest), so the radix sort orders suffixes by raw bytes as divbwt64 does
 * (genFMindex.c:482); ties go to the prefix doubling with h0 = L. */
__global__ __launch_bounds__(256) void k_keys_ref(const uint8_t* __restrict__ text, uint64_t n,
                                                  const uint8_t* __restrict__ lut, uint32_t bits, uint32_t L,
                                                  uint64_t* __restrict__ keys, uint32_t* __restrict__ vals)
{
  __shared__ uint8_t rk[256];
  rk[threadIdx.x] = lut[threadIdx.x];
  __syncthreads();
  const uint64_t i = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint64_t k = 0;
  for (uint32_t j = 0; j < L; ++j) k = (k << bits) | (i + j < n ? (uint64_t) rk[text[i + j]] : 0ull);
  keys[i] = k;
  vals[i] = (uint32_t) i;
}

/* number of sorted positions j >= 1 whose 32-base key equals key j-1 (one
 * atomic per wave) */
__global__ __launch_bounds__(256) void k_ties(const uint64_t* __restrict__ keys, uint64_t n,
                                              unsigned long long* __restrict__ count)
{
  const uint64_t i = (uint64_t) blockIdx.x * 256 + threadIdx.x + 1;
  const bool tie = i < n && keys[i] == keys[i - 1];
  const uint64_t b = __ballot(tie);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(count, (unsigned long long) __popcll(b));
}

/* ---- tie resolution by prefix doubling (Manber-Myers / Larsson-Sadakane on
 * the device).  After the 32-base radix sort, positions j with equal keys form
 * groups; rank[i] = group start (a position in SA order) of suffix i.  Round h
 * (h = 32, 64, ...) re-sorts every non-singleton group by the rank of suffix
 * i + h, which holds the order of chars h..2h-1.  Suffixes whose $ falls inside
 * the first h chars (i + h >= n) take n - 1 - i: below every real rank (those
 * are shifted by h) and shortest first -- '$' sorts lowest, and a padded key
 * only ties with a longer suffix that has A where this one ends. */
__device__ __forceinline__ uint64_t dbl_key(const uint32_t* __restrict__ rank, uint64_t n, uint64_t h, uint32_t i)
{
  return (uint64_t) i + h < n ? (uint64_t) rank[i + h] + h : n - 1 - (uint64_t) i;
}

/* Compiler barrier between the loads of element j and its neighbour j - 1:
 * merged, they become one load at half its width's alignment (a 16-byte load
 * of two u64 keys at an 8-mod-16 address), the load form kfmi_device.h
 * load_words keeps out of every kernel.  No instruction. */
__device__ __forceinline__ void apart() { asm volatile("" ::: "memory"); }

/* head value (j if j starts a key group, else 0) for the max-scan of group starts */
__global__ __launch_bounds__(256) void k_head_values(const uint64_t* __restrict__ keys, uint64_t n,
                                                     uint32_t* __restrict__ hv)
{
  const uint64_t j = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const uint64_t kj = keys[j];
  apart();
  hv[j] = (j == 0 || kj != keys[j - 1]) ? (uint32_t) j : 0u;
}

/* rank[sa[j]] = gs[j]; active[j] = j lies in a group of two or more */
__global__ __launch_bounds__(256) void k_rank_init(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ sa,
                                                   const uint32_t* __restrict__ gs, uint64_t n,
                                                   uint32_t* __restrict__ rank, uint8_t* __restrict__ active)
{
  const uint64_t j = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  rank[sa[j]] = gs[j];
  const uint64_t kj = keys[j];
  apart();
  const bool head = j == 0 || kj != keys[j - 1];
  apart();
  const bool last = j + 1 == n || keys[j + 1] != kj;
  active[j] = (head && last) ? 0 : 1;
}

/* round h, step 1: the doubling key and suffix of every active position */
__global__ __launch_bounds__(256) void k_dbl_keys(const uint32_t* __restrict__ act, uint64_t m,
                                                  const uint32_t* __restrict__ sa, const uint32_t* __restrict__ rank,
                                                  uint64_t n, uint64_t h, uint64_t* __restrict__ key2,
                                                  uint32_t* __restrict__ suf)
{
  const uint64_t k = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (k >= m) return;
  const uint32_t i = sa[act[k]];
  key2[k] = dbl_key(rank, n, h, i);
  suf[k] = i;
}

/* step 2: the current group of every suffix (primary key of the stable pass) */
__global__ __launch_bounds__(256) void k_dbl_groups(const uint32_t* __restrict__ suf, uint64_t m,
                                                    const uint32_t* __restrict__ rank, uint32_t* __restrict__ grp)
{
  const uint64_t k = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (k >= m) return;
  grp[k] = rank[suf[k]];
}

/* step 3: write the re-sorted suffixes back into their groups' SA slots (the
 * active positions are in SA order and every group is contiguous there), and
 * mark where a new (group, key) run starts */
__global__ __launch_bounds__(256) void k_dbl_apply(const uint32_t* __restrict__ act, uint64_t m,
                                                   const uint32_t* __restrict__ suf, const uint32_t* __restrict__ grp,
                                                   const uint32_t* __restrict__ rank, uint64_t n, uint64_t h,
                                                   uint32_t* __restrict__ sa, uint32_t* __restrict__ hv,
                                                   uint8_t* __restrict__ head)
{
  const uint64_t k = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (k >= m) return;
  const uint32_t i = suf[k];
  sa[act[k]] = i;
  const uint32_t gk = grp[k];
  apart();
  bool hd = k == 0 || gk != grp[k - 1];
  apart();
  if (!hd) hd = dbl_key(rank, n, h, i) != dbl_key(rank, n, h, suf[k - 1]);
  head[k] = hd ? 1 : 0;
  hv[k] = hd ? act[k] : 0u;
}

/* step 4 (after the max-scan of hv into ngs): new ranks, and which positions
 * stay active (runs of two or more) */
__global__ __launch_bounds__(256) void k_dbl_rank(const uint32_t* __restrict__ suf, const uint32_t* __restrict__ ngs,
                                                  const uint8_t* __restrict__ head, uint64_t m,
                                                  uint32_t* __restrict__ rank, uint8_t* __restrict__ active)
{
  const uint64_t k = (uint64_t) blockIdx.x * 256 + threadIdx.x;
  if (k >= m) return;
  rank[suf[k]] = ngs[k];
  const bool last = k + 1 == m || head[k + 1];
  active[k] = (head[k] && last) ? 0 : 1;
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
                                                const uint8_t* __restrict__ codes, uint64_t n, uint32_t d,
                                                uint32_t nentries, uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3,
                                                uint32_t* __restrict__ entries, uint32_t* __restrict__ counts)
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
    if (valid && codes) {   /* a derived index: the row's K-mer code is given */
      code = codes[r];
    } else if (valid) {
      const uint64_t s_a = r == 0 ? n : (uint64_t) sa[r - 1];
#pragma unroll
      for (int s = 0; s < K; ++s) {
        int64_t pos = (int64_t) s_a - 1 - s;
        if (pos < 0) pos += (int64_t) rows;
        const uint32_t cs = ((uint64_t) pos == n) ? 0u : base_at(packed, (uint64_t) pos);
        code |= cs << (2 * s);
      }
    }
    if (valid) {
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

unsigned long long g_last_ties = 0;   /* diagnostics of the last build (kfmi_build_stats) */
uint32_t g_last_tie_rounds = 0;

/* Sorts every group of equal 32-base keys in `sa` (length n, sorted by the
 * keys in `keys`) into true suffix order; see k_dbl_key. */
int32_t resolve_ties(const uint64_t* keys, uint32_t* sa, uint64_t n, uint64_t h0, hipStream_t st, uint32_t* rounds)
{
  const dim3 gn((uint32_t) ((n + 255) / 256)), blk(256);
  DevBuf rank, gs, hv0, act, flags, cnt;
  BHIP(rank.alloc(4 * n));
  BHIP(gs.alloc(4 * n));
  BHIP(hv0.alloc(4 * n));
  BHIP(act.alloc(4 * n));
  BHIP(flags.alloc(n));
  BHIP(cnt.alloc(8));
  /* group starts, ranks, the active positions */
  {
    hipLaunchKernelGGL(k_head_values, gn, blk, 0, st, keys, n, hv0.as<uint32_t>());
    BHIP(hipGetLastError());
    size_t tb = 0;
    BHIP(rocprim::inclusive_scan(nullptr, tb, hv0.as<uint32_t>(), gs.as<uint32_t>(), (size_t) n,
                                 rocprim::maximum<uint32_t>(), st));
    DevBuf tmp;
    BHIP(tmp.alloc(tb));
    BHIP(rocprim::inclusive_scan(tmp.p, tb, hv0.as<uint32_t>(), gs.as<uint32_t>(), (size_t) n,
                                 rocprim::maximum<uint32_t>(), st));
    hipLaunchKernelGGL(k_rank_init, gn, blk, 0, st, keys, sa, gs.as<uint32_t>(), n, rank.as<uint32_t>(),
                       flags.as<uint8_t>());
    BHIP(hipGetLastError());
  }
  auto compact = [&](const uint32_t* in, bool counting, uint64_t len, uint32_t* outp, uint64_t* m) -> hipError_t {
    size_t tb = 0;
    rocprim::counting_iterator<uint32_t> ci(0);
    hipError_t e = counting ? rocprim::select(nullptr, tb, ci, flags.as<uint8_t>(), outp,
                                              cnt.as<unsigned long long>(), (size_t) len, st)
                            : rocprim::select(nullptr, tb, in, flags.as<uint8_t>(), outp,
                                              cnt.as<unsigned long long>(), (size_t) len, st);
    if (e != hipSuccess) return e;
    DevBuf tmp;
    if ((e = tmp.alloc(tb)) != hipSuccess) return e;
    e = counting ? rocprim::select(tmp.p, tb, ci, flags.as<uint8_t>(), outp, cnt.as<unsigned long long>(),
                                   (size_t) len, st)
                 : rocprim::select(tmp.p, tb, in, flags.as<uint8_t>(), outp, cnt.as<unsigned long long>(),
                                   (size_t) len, st);
    unsigned long long c = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&c, cnt.p, 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    *m = c;
    return e;
  };
  uint64_t m = 0;
  BHIP(compact(nullptr, true, n, act.as<uint32_t>(), &m));
  gs.release();
  hv0.release();
  uint32_t r = 0;
  for (uint64_t h = h0; m > 0; h *= 2, ++r) {
    if (h > 2 * n + 64) return KFMI_E_BUILDING_BWT;   /* cannot happen: all suffixes differ by then */
    const dim3 gm((uint32_t) ((m + 255) / 256));
    DevBuf k2a, k2b, sfa, sfb, ga, gb, hv, ngs, head, nact, tmp;
    BHIP(k2a.alloc(8 * m)); BHIP(k2b.alloc(8 * m));
    BHIP(sfa.alloc(4 * m)); BHIP(sfb.alloc(4 * m));
    BHIP(ga.alloc(4 * m)); BHIP(gb.alloc(4 * m));
    hipLaunchKernelGGL(k_dbl_keys, gm, blk, 0, st, act.as<uint32_t>(), m, sa, rank.as<uint32_t>(), n, h,
                       k2a.as<uint64_t>(), sfa.as<uint32_t>());
    BHIP(hipGetLastError());
    /* LSD: by the doubling key, then stably by the group */
    unsigned kbits = 1;
    while (kbits < 64 && (n + h) >> kbits) ++kbits;
    size_t tb = 0, tb2 = 0;
    BHIP(rocprim::radix_sort_pairs(nullptr, tb, k2a.as<uint64_t>(), k2b.as<uint64_t>(), sfa.as<uint32_t>(),
                                   sfb.as<uint32_t>(), (size_t) m, 0, kbits, st));
    BHIP(rocprim::radix_sort_pairs(nullptr, tb2, ga.as<uint32_t>(), gb.as<uint32_t>(), sfb.as<uint32_t>(),
                                   sfa.as<uint32_t>(), (size_t) m, 0, 32, st));
    BHIP(tmp.alloc(tb > tb2 ? tb : tb2));
    BHIP(rocprim::radix_sort_pairs(tmp.p, tb, k2a.as<uint64_t>(), k2b.as<uint64_t>(), sfa.as<uint32_t>(),
                                   sfb.as<uint32_t>(), (size_t) m, 0, kbits, st));
    k2a.release(); k2b.release();
    hipLaunchKernelGGL(k_dbl_groups, gm, blk, 0, st, sfb.as<uint32_t>(), m, rank.as<uint32_t>(), ga.as<uint32_t>());
    BHIP(hipGetLastError());
    BHIP(rocprim::radix_sort_pairs(tmp.p, tb2, ga.as<uint32_t>(), gb.as<uint32_t>(), sfb.as<uint32_t>(),
                                   sfa.as<uint32_t>(), (size_t) m, 0, 32, st));
    tmp.release(); ga.release(); sfb.release();
    BHIP(hv.alloc(4 * m)); BHIP(head.alloc(m));
    hipLaunchKernelGGL(k_dbl_apply, gm, blk, 0, st, act.as<uint32_t>(), m, sfa.as<uint32_t>(), gb.as<uint32_t>(),
                       rank.as<uint32_t>(), n, h, sa, hv.as<uint32_t>(), head.as<uint8_t>());
    BHIP(hipGetLastError());
    BHIP(ngs.alloc(4 * m));
    BHIP(rocprim::inclusive_scan(nullptr, tb, hv.as<uint32_t>(), ngs.as<uint32_t>(), (size_t) m,
                                 rocprim::maximum<uint32_t>(), st));
    BHIP(tmp.alloc(tb));
    BHIP(rocprim::inclusive_scan(tmp.p, tb, hv.as<uint32_t>(), ngs.as<uint32_t>(), (size_t) m,
                                 rocprim::maximum<uint32_t>(), st));
    hipLaunchKernelGGL(k_dbl_rank, gm, blk, 0, st, sfa.as<uint32_t>(), ngs.as<uint32_t>(), head.as<uint8_t>(), m,
                       rank.as<uint32_t>(), flags.as<uint8_t>());
    BHIP(hipGetLastError());
    BHIP(nact.alloc(4 * m));
    uint64_t m2 = 0;
    BHIP(compact(act.as<uint32_t>(), false, m, nact.as<uint32_t>(), &m2));
    BHIP(hipMemcpyAsync(act.p, nact.p, 4 * m2, hipMemcpyDeviceToDevice, st));
    m = m2;
  }
  BHIP(hipStreamSynchronize(st));
  *rounds = r;
  return KFMI_SUCCESS;
}

/* Steps 5-7: the entries of the K-step index whose row r has the K-mer code
 * codes[r] (derived indexes) or, without codes, the one read from SA and the
 * packed text; drow = the '$' rows D_s, dbase = their stored codes ('$' as A).
 * The suffix array (sa_buf, when given) is released once its samples are
 * taken, before the scans; on success *out owns the index (entries on the
 * device when !host_image). */
static int32_t entries_from_rows(hipStream_t st, DevBuf* sa_buf, const uint32_t* packed, const uint8_t* codes,
                                 uint64_t n, uint32_t k, uint32_t d, const uint32_t* drow, const uint32_t* dbase,
                                 uint32_t sa_rate, int dev, bool host_image, kfmi_fmi_t** out)
{
  const uint64_t rows = n + 1;
  const uint32_t nentries = (uint32_t) ((rows + d - 1) / d);
  const uint32_t nc = 1u << (2 * k), nb = d / 32;
  const uint32_t* sa = sa_buf ? sa_buf->as<uint32_t>() : nullptr;
  kfmi_fmi_t* f = nullptr;
  int32_t err = kfmi_index_alloc_ex(100, k, (uint32_t) rows, nentries, d, nullptr, nullptr, host_image ? 1 : 0, &f);
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
      case 1: hipLaunchKernelGGL((k_blocks<1>), grid, dim3(256), 0, st, sa, packed, codes, n, d,
                                 nentries, drow[0], drow[1], drow[2], drow[3], ent.as<uint32_t>(), counts.as<uint32_t>()); break;
      case 2: hipLaunchKernelGGL((k_blocks<2>), grid, dim3(256), 0, st, sa, packed, codes, n, d,
                                 nentries, drow[0], drow[1], drow[2], drow[3], ent.as<uint32_t>(), counts.as<uint32_t>()); break;
      case 3: hipLaunchKernelGGL((k_blocks<3>), grid, dim3(256), 0, st, sa, packed, codes, n, d,
                                 nentries, drow[0], drow[1], drow[2], drow[3], ent.as<uint32_t>(), counts.as<uint32_t>()); break;
      default: hipLaunchKernelGGL((k_blocks<4>), grid, dim3(256), 0, st, sa, packed, codes, n, d,
                                  nentries, drow[0], drow[1], drow[2], drow[3], ent.as<uint32_t>(), counts.as<uint32_t>()); break;
    }
    le = hipGetLastError();
    if (le != hipSuccess) return fail(KFMI_E_BUILDING_FMI);
  }
  if (sa_rate && sa) {   /* locate samples, before the SA is released */
    err = kfmi_sa_alloc(f, sa_rate);
    if (err) return fail(err);
    DevBuf smp;
    if (smp.alloc(4 * f->sa_count) != hipSuccess) return fail(KFMI_E_ALLOCATING_FMI);
    hipLaunchKernelGGL(k_sample, dim3((uint32_t) ((f->sa_count + 255) / 256)), dim3(256), 0, st, sa, n,
                       sa_rate, f->sa_count, smp.as<uint32_t>());
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(f->h_sa, smp.p, 4 * f->sa_count, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return fail(KFMI_E_BUILDING_FMI);
  }
  if (sa_buf) sa_buf->release();
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
      (host_image &&
       hipMemcpyAsync(f->h_index, ent.p, (uint64_t) ew * 4 * nentries, hipMemcpyDeviceToHost, st) != hipSuccess) ||
      hipStreamSynchronize(st) != hipSuccess)
    return fail(KFMI_E_BUILDING_FMI);
  if (!host_image) {   /* the entries stay in HBM, owned by the handle */
    f->d_entries = ent.as<uint32_t>();
    f->d_entries_dev = dev;
    ent.p = nullptr;
  }
  for (uint32_t s = 0; s < k; ++s) {
    f->dollarPositionBWT[s] = drow[s];
    f->dollarBaseBWT[s] = dbase[s];
    f->modposdollarBWT[s] = drow[s] / d;
  }
  uint32_t* hdr = reinterpret_cast<uint32_t*>(f->image);   /* the header words of the image */
  for (uint32_t s = 0; s < k; ++s) {
    hdr[6 + s] = drow[s];
    hdr[6 + k + s] = dbase[s];
  }
  *out = f;
  return KFMI_SUCCESS;
}


int32_t build_gpu(const char* text, uint64_t n, uint32_t k, uint32_t d, uint32_t sa_rate, int dev, bool host_image,
                  kfmi_fmi_t** out)
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
  const uint64_t nwords = (n + 15) / 16 + 4;

  /* 0. alphabet (fmi_build.c): "ref" on a text with bytes other than A/C/G/T
   * sorts raw bytes -- keys of dense byte ranks, `bits` each -- and for K >= 2
   * leaves BWT_1.. to the reference's LF walk on the host */
  const int mode = kfmi_alphabet_mode();
  bool raw_sort = false;
  uint8_t lut[256] = {0};
  uint32_t kbits = 2, klen = 32;
  if (mode == KFMI_ALPHA_REF) {
    std::vector<uint64_t> hist(256, 0);
    for (uint64_t i = 0; i < n; ++i) hist[(uint8_t) text[i]]++;
    if (hist[0]) return KFMI_E_BUILDING_BWT;   /* NUL would tie with '$' */
    uint32_t sigma = 0;
    for (int b = 1; b < 256; ++b) {
      if (hist[b]) lut[b] = (uint8_t) ++sigma;
      if (hist[b] && b != 'A' && b != 'C' && b != 'G' && b != 'T') raw_sort = true;
    }
    if (raw_sort) {
      kbits = 1;
      while ((1u << kbits) <= sigma) ++kbits;   /* ranks 1..sigma, 0 past the end */
      klen = 64 / kbits;
    }
  }

  /* 1. encode */
  DevBuf packed, bad, ascii;
  BHIP(packed.alloc(nwords * 4));
  BHIP(bad.alloc(4));
  BHIP(hipMemsetAsync(bad.p, 0, 4, st));
  {
    BHIP(ascii.alloc(n));
    BHIP(hipMemcpyAsync(ascii.p, text, n, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_encode, dim3((uint32_t) ((nwords + 255) / 256)), dim3(256), 0, st, ascii.as<uint8_t>(), n,
                       packed.as<uint32_t>(), nwords, bad.as<uint32_t>(), mode == KFMI_ALPHA_ACGT ? 0u : 1u);
    BHIP(hipGetLastError());
    uint32_t hbad = 0;
    BHIP(hipMemcpyAsync(&hbad, bad.p, 4, hipMemcpyDeviceToHost, st));
    BHIP(hipStreamSynchronize(st));
    if (hbad) return KFMI_E_BUILDING_BWT;   /* non-ACGT text in the "acgt" alphabet (see fmi_build.c) */
    if (!raw_sort) ascii.release();
  }

  /* 2-3. keys and radix sort */
  DevBuf sa;
  BHIP(sa.alloc(n * 4));
  {
    DevBuf k0, k1, v0, tmp;
    BHIP(k0.alloc(n * 8));
    BHIP(k1.alloc(n * 8));
    BHIP(v0.alloc(n * 4));
    if (raw_sort) {
      DevBuf dl;
      BHIP(dl.alloc(256));
      BHIP(hipMemcpyAsync(dl.p, lut, 256, hipMemcpyHostToDevice, st));
      hipLaunchKernelGGL(k_keys_ref, dim3((uint32_t) ((n + 255) / 256)), dim3(256), 0, st, ascii.as<uint8_t>(), n,
                         dl.as<uint8_t>(), kbits, klen, k0.as<uint64_t>(), v0.as<uint32_t>());
      BHIP(hipGetLastError());
      BHIP(hipStreamSynchronize(st));
      ascii.release();
    } else {
      hipLaunchKernelGGL(k_keys, dim3((uint32_t) ((n + 255) / 256)), dim3(256), 0, st, packed.as<uint32_t>(), n,
                         k0.as<uint64_t>(), v0.as<uint32_t>());
      BHIP(hipGetLastError());
    }
    rocprim::double_buffer<uint64_t> kb(k0.as<uint64_t>(), k1.as<uint64_t>());
    rocprim::double_buffer<uint32_t> vb(v0.as<uint32_t>(), sa.as<uint32_t>());
    size_t tbytes = 0;
    BHIP(rocprim::radix_sort_pairs(nullptr, tbytes, kb, vb, (size_t) n, 0, 64, st));
    BHIP(tmp.alloc(tbytes));
    BHIP(rocprim::radix_sort_pairs(tmp.p, tbytes, kb, vb, (size_t) n, 0, 64, st));
    if (vb.current() != sa.as<uint32_t>())
      BHIP(hipMemcpyAsync(sa.p, vb.current(), n * 4, hipMemcpyDeviceToDevice, st));

    /* 4. ties: equal 32-base keys (repeats, or suffixes ending within 32 bases
     * of the end), resolved on the device by prefix doubling */
    DevBuf cntb;
    BHIP(cntb.alloc(8));
    BHIP(hipMemsetAsync(cntb.p, 0, 8, st));
    if (n > 1)
      hipLaunchKernelGGL(k_ties, dim3((uint32_t) ((n - 1 + 255) / 256)), dim3(256), 0, st, kb.current(), n,
                         cntb.as<unsigned long long>());
    BHIP(hipGetLastError());
    unsigned long long nties = 0;
    BHIP(hipMemcpyAsync(&nties, cntb.p, 8, hipMemcpyDeviceToHost, st));
    BHIP(hipStreamSynchronize(st));
    g_last_ties = nties;
    g_last_tie_rounds = 0;
    if (nties) {
      int32_t e = resolve_ties(kb.current(), sa.as<uint32_t>(), n, klen, st, &g_last_tie_rounds);
      if (e) return e;
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
  if (raw_sort && k > 1) {
    /* "ref" alphabet, K >= 2, text with bytes other than A/C/G/T: BWT_1.. come
     * from the reference's LF walk (genFMindex.c:327-400), which is not a
     * permutation then -- one dependent chain over the n + 1 rows, on the host
     * (kfmi_index_ref_walk, fmi_build.c) from the device's raw-byte SA */
    std::vector<uint32_t> sa_full(rows);
    sa_full[0] = (uint32_t) n;
    BHIP(hipMemcpyAsync(sa_full.data() + 1, sa.p, 4 * n, hipMemcpyDeviceToHost, st));
    BHIP(hipStreamSynchronize(st));
    sa.release();
    kfmi_fmi_t* f = nullptr;
    int32_t err = kfmi_index_ref_walk(text, sa_full.data(), n, k, d, &f);
    if (err) return err;
    if (sa_rate) {
      err = kfmi_sa_alloc(f, sa_rate);
      if (err) {
        freeIndex((void**) &f);
        return err;
      }
      for (uint64_t i = 0; i < f->sa_count; ++i) f->h_sa[i] = sa_full[i * sa_rate];
    }
    *out = f;
    return KFMI_SUCCESS;
  }
  /* dollarBaseBWT[s] = c(D_s): SA[D_s] = s, so BWT_s'[D_s] = T$[(s-1-s') mod (n+1)] */
  uint32_t dbase[4] = {0, 0, 0, 0};
  for (uint32_t s = 0; s < k; ++s) {
    uint32_t code = 0;
    for (uint32_t s2 = 0; s2 < k; ++s2) {
      int64_t pos = (int64_t) s - 1 - (int64_t) s2;
      if (pos < 0) pos += (int64_t) rows;
      uint32_t cs = 0;
      if ((uint64_t) pos != n) cs = base2index((uint8_t) text[pos]);   /* A/C/G/T, or any byte (map, ref) */
      code |= cs << (2 * s2);
    }
    dbase[s] = code;
  }
  return entries_from_rows(st, &sa, packed.as<uint32_t>(), nullptr, n, k, d, drow, dbase, sa_rate, dev, host_image,
                           out);
}

}  // namespace

namespace kfmi {

/* Steps 5-7 for a 2K-step index derived from a K-step one (kfmi_derive.hip):
 * the rows' K-mer codes are given on the device (d_codes, n + 1 bytes). */
int32_t build_from_codes(const uint8_t* d_codes, uint64_t n, uint32_t k, uint32_t d, const uint32_t* drow,
                         const uint32_t* dbase, int dev, bool host_image, kfmi_fmi_t** out)
{
  if (n == 0 || n + 1 > 0xFFFFFFFEull || k < 1 || k > 4 || d == 0 || d % 32) return KFMI_E_BAD_ARGUMENT;
  BHIP(hipSetDevice(dev));
  hipStream_t st;
  BHIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  struct StreamGuard { hipStream_t s; ~StreamGuard() { (void) hipStreamDestroy(s); } } sg{st};
  return entries_from_rows(st, nullptr, nullptr, d_codes, n, k, d, drow, dbase, 0, dev, host_image, out);
}

}  // namespace kfmi

extern "C" int32_t kfmi_build_index_gpu_sa(const char* text, uint64_t n, uint32_t k, uint32_t d, uint32_t sa_rate,
                                           void** index)
{
  if (sa_rate && !kfmi_sa_rate_ok(sa_rate)) return KFMI_E_BAD_ARGUMENT;
  if (kfmi_device_count() < 1) return KFMI_E_NO_DEVICE;
  kfmi::DeviceGuard dg;
  int32_t e = build_gpu(text, n, k, d, sa_rate, kfmi_current_device(), true, (kfmi_fmi_t**) index);
  if (e == KFMI_E_NOT_IMPLEMENTED) {
    fprintf(stderr, "kstepfmi build: text of %llu bases exceeds one dispatch per base (2^32 - 256), "
                    "using the host builder\n", (unsigned long long) n);
    return kfmi_build_index_cpu_sa(text, n, k, d, sa_rate, index);
  }
  return e;
}

extern "C" int32_t kfmi_build_stats(uint64_t* ties, uint32_t* rounds)
{
  if (ties) *ties = g_last_ties;
  if (rounds) *rounds = g_last_tie_rounds;
  return KFMI_SUCCESS;
}

extern "C" int32_t kfmi_build_index_gpu(const char* text, uint64_t n, uint32_t k, uint32_t d,
                                        int32_t want_host_image, void** index)
{
  if (want_host_image) return kfmi_build_index_gpu_sa(text, n, k, d, 0, index);
  if (kfmi_device_count() < 1) return KFMI_E_NO_DEVICE;
  kfmi::DeviceGuard dg;
  int32_t e = build_gpu(text, n, k, d, 0, kfmi_current_device(), false, (kfmi_fmi_t**) index);
  if (e == KFMI_E_NOT_IMPLEMENTED) return kfmi_build_index_gpu_sa(text, n, k, d, 0, index);   /* host builder */
  return e;
}

/* The host image of an index whose entries are only in HBM: fetched once (one
 * D2H) into a new buffer, then kept beside the device copy.  Nothing a reader
 * may hold moves: the header-only image it replaces is retired (freed by
 * freeIndex), and h_index is published with release order after the bytes
 * are in place, so a thread that sees it non-null sees the whole image. */
extern "C" int32_t kfmi_host_entries(kfmi_fmi_t* f)
{
  if (!f) return KFMI_E_BAD_ARGUMENT;
  if (__atomic_load_n(&f->h_index, __ATOMIC_ACQUIRE)) return KFMI_SUCCESS;
  static std::mutex mu;   /* two threads asking for the same handle's image fetch it once */
  std::lock_guard<std::mutex> lk(mu);
  if (__atomic_load_n(&f->h_index, __ATOMIC_ACQUIRE)) return KFMI_SUCCESS;
  if (!f->d_entries) return KFMI_E_BAD_ARGUMENT;
  const uint64_t body = 4ull * f->entry_words * f->nentries;
  uint8_t* img = (uint8_t*) kfmi_big_alloc(f->header_bytes + body + 64);
  if (!img) return KFMI_E_ALLOCATING_FMI;
  memcpy(img, f->image, f->header_bytes);
  memset(img + f->header_bytes + body, 0, 64);
  kfmi::DeviceGuard dg;
  if (hipSetDevice(f->d_entries_dev) != hipSuccess ||
      hipMemcpy(img + f->header_bytes, f->d_entries, body, hipMemcpyDeviceToHost) != hipSuccess) {
    kfmi_big_free(img);
    return KFMI_E_KERNEL;
  }
  kfmi_big_free(f->image_retired);   /* never set twice: h_index is published once */
  f->image_retired = f->image;
  f->image = img;
  __atomic_store_n(&f->h_index, (uint32_t*) (img + f->header_bytes), __ATOMIC_RELEASE);
  return KFMI_SUCCESS;
}

extern "C" void kfmi_free_dev_entries(kfmi_fmi_t* f)
{
  if (!f || !f->d_entries) return;
  kfmi::DeviceGuard dg;
  (void) hipSetDevice(f->d_entries_dev);
  (void) hipFree(f->d_entries);
  f->d_entries = nullptr;
}
