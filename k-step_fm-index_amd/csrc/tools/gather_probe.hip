/*
 * gather_probe -- random-line gather ceiling of the MI355X memory system for
 * the LF access pattern (dev tool, not part of the engine).
 *
 *   gather_probe [table_GB=3] [lines_M=512]
 *
 * For line sizes of 32/64/128 B it reads `lines` uniformly random, line-aligned
 * lines of a `table_GB` table and reports lines/s and GB/s for:
 *   indep  : every lane issues independent line reads (4 in flight per lane),
 *            one lane per line (dwordx4 loads)
 *   coop   : TPR lanes read one line cooperatively, 16 B each
 *   chain  : dependent chains (next address = f(loaded data)), 1 or 2 chains
 *            per lane -- the LF kernel's shape
 *   mask<G>: as indep / chain1, but each wave issues every gather as G
 *            instructions with 64/G active lanes (fewer distinct pages per
 *            instruction -- the translation-reach question)
 *   PROBE_CPOL=1: the coop 128-B gather with sc0 / sc1 / nt cache-policy
 *            bits on its loads; PROBE_ALLOC=uncached: the table allocated
 *            uncached -- whether any load path beats the random-line
 *            request ceiling
 * Addresses come from a per-lane xorshift generator (no index array traffic).
 */
#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint64_t xs(uint64_t& s)
{
  s ^= s << 13; s ^= s >> 7; s ^= s << 17;
  return s;
}

/* uniform line index in [0, n) without a 64-bit modulo (n < 2^32) */
__device__ __forceinline__ uint64_t pick(uint64_t x, uint64_t n) { return ((x >> 32) * n) >> 32; }

template <int LB>   // line bytes
__global__ __launch_bounds__(256) void k_indep(const uint4* __restrict__ t, uint64_t nlines, uint64_t per_thread,
                                               uint32_t* __restrict__ sink)
{
  constexpr int V = LB / 16;
  uint64_t s = 0x9E3779B97F4A7C15ull ^ ((uint64_t) blockIdx.x * 256 + threadIdx.x) * 0xBF58476D1CE4E5B9ull;
  uint32_t acc = 0;
  for (uint64_t i = 0; i < per_thread; i += 4) {
    uint4 v[4][V];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t l = pick(xs(s), nlines);
#pragma unroll
      for (int k = 0; k < V; ++k) v[j][k] = t[l * V + k];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < V; ++k) acc ^= v[j][k].x ^ v[j][k].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int LB>
__global__ __launch_bounds__(256) void k_coop(const uint4* __restrict__ t, uint64_t nlines, uint64_t per_group,
                                              uint32_t* __restrict__ sink)
{
  constexpr int TPR = LB / 16;
  const int lane = threadIdx.x & 63, k = lane % TPR;
  /* lanes of one group share the generator state: same address */
  uint64_t s = 0x9E3779B97F4A7C15ull ^ (((uint64_t) blockIdx.x * 256 + threadIdx.x) / TPR) * 0xBF58476D1CE4E5B9ull;
  uint32_t acc = 0;
  for (uint64_t i = 0; i < per_group; i += 4) {
    uint4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = t[(pick(xs(s), nlines)) * TPR + k];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc ^= v[j].x ^ v[j].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

/* cooperative 128-B lines with W bytes per lane: 128 / W lanes per line, so
 * one wave instruction touches W / 2 lines (pages) -- 8 (W = 16, k_coop<128>),
 * 4 (W = 8) or 2 (W = 4) */
template <int W>
__global__ __launch_bounds__(256) void k_coopw(const uint8_t* __restrict__ t, uint64_t nlines, uint64_t per_group,
                                               uint32_t* __restrict__ sink)
{
  using E = typename std::conditional<W == 16, uint4, typename std::conditional<W == 8, uint2, uint32_t>::type>::type;
  constexpr int TPR = 128 / W;
  const int lane = threadIdx.x & 63, k = lane % TPR;
  uint64_t s = 0x9E3779B97F4A7C15ull ^ (((uint64_t) blockIdx.x * 256 + threadIdx.x) / TPR) * 0xBF58476D1CE4E5B9ull;
  const E* te = reinterpret_cast<const E*>(t);
  uint32_t acc = 0;
  for (uint64_t i = 0; i < per_group; i += 4) {
    E v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = te[(pick(xs(s), nlines)) * TPR + k];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc ^= reinterpret_cast<const uint32_t*>(&v[j])[0];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int LB, int CH>
__global__ __launch_bounds__(256) void k_chain(const uint4* __restrict__ t, uint64_t nlines, uint32_t steps,
                                               uint32_t* __restrict__ sink)
{
  constexpr int V = LB / 16;
  uint64_t s[CH];
  uint64_t l[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    s[c] = 0x9E3779B97F4A7C15ull ^ (((uint64_t) blockIdx.x * 256 + threadIdx.x) * CH + c) * 0xBF58476D1CE4E5B9ull;
    l[c] = pick(xs(s[c]), nlines);
  }
  uint32_t acc = 0;
  for (uint32_t i = 0; i < steps; ++i) {
    uint4 v[CH][V];
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
      for (int k = 0; k < V; ++k) v[c][k] = t[l[c] * V + k];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      uint32_t x = 0;
#pragma unroll
      for (int k = 0; k < V; ++k) x ^= v[c][k].x ^ v[c][k].y;
      acc ^= x;
      l[c] = pick(xs(s[c]) ^ ((uint64_t) x << 32), nlines);     /* next address depends on the loaded data */
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}


/* indep / chain with every gather issued as G exec-masked instructions of
 * 64/G lanes each: the same requests, at most 64/G distinct pages per
 * instruction */
template <int LB, int G>
__global__ __launch_bounds__(256) void k_masked(const uint4* __restrict__ t, uint64_t nlines, uint64_t per_thread,
                                                uint32_t* __restrict__ sink)
{
  constexpr int V = LB / 16;
  const int grp = (threadIdx.x & 63) / (64 / G);
  uint64_t s = 0x9E3779B97F4A7C15ull ^ ((uint64_t) blockIdx.x * 256 + threadIdx.x) * 0xBF58476D1CE4E5B9ull;
  uint32_t acc = 0;
  for (uint64_t i = 0; i < per_thread; i += 4) {
    uint4 v[4][V];
    uint64_t l[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) l[j] = pick(xs(s), nlines);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (grp == g) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int k = 0; k < V; ++k) v[j][k] = t[l[j] * V + k];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < V; ++k) acc ^= v[j][k].x ^ v[j][k].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int LB, int G>
__global__ __launch_bounds__(256) void k_chain_masked(const uint4* __restrict__ t, uint64_t nlines, uint32_t steps,
                                                      uint32_t* __restrict__ sink)
{
  constexpr int V = LB / 16;
  const int grp = (threadIdx.x & 63) / (64 / G);
  uint64_t s = 0x9E3779B97F4A7C15ull ^ ((uint64_t) blockIdx.x * 256 + threadIdx.x) * 0xBF58476D1CE4E5B9ull;
  uint64_t l = pick(xs(s), nlines);
  uint32_t acc = 0;
  for (uint32_t i = 0; i < steps; ++i) {
    uint4 v[V];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (grp == g) {
#pragma unroll
        for (int k = 0; k < V; ++k) v[k] = t[l * V + k];
      }
    }
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < V; ++k) x ^= v[k].x ^ v[k].y;
    acc ^= x;
    l = pick(xs(s) ^ ((uint64_t) x << 32), nlines);
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

/* coop 128-B gather with explicit cache-policy bits (PROBE_CPOL=1), through
 * raw buffer loads (bounds-checked: an out-of-range offset reads 0, never
 * faults).  aux: sc0 = 1, nt = 2, sc1 = 16.  The table must be < 4 GB. */
typedef unsigned v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t table_rsrc(const void* t, uint64_t bytes)
{
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(t), (short) 0, (int) (uint32_t) bytes, 0x00020000);
}

template <int AUX>
__global__ __launch_bounds__(256) void k_coop_pol(const uint4* __restrict__ t, uint64_t nlines, uint64_t per_group,
                                                  uint32_t* __restrict__ sink)
{
  constexpr int TPR = 8;
  const __amdgpu_buffer_rsrc_t rs = table_rsrc(t, nlines * 128);
  const int lane = threadIdx.x & 63, k = lane % TPR;
  uint64_t s = 0x9E3779B97F4A7C15ull ^ (((uint64_t) blockIdx.x * 256 + threadIdx.x) / TPR) * 0xBF58476D1CE4E5B9ull;
  uint32_t acc = 0;
  for (uint64_t i = 0; i < per_group; i += 4) {
    v4u v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int) (uint32_t) (pick(xs(s), nlines) * 128 + 16 * k), 0, AUX);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc ^= v[j].x ^ v[j].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

/* one buffer load of the table's last 16 B: the descriptor reads real data */
__global__ void k_rsrc_check(const uint4* __restrict__ t, uint64_t bytes, uint32_t* __restrict__ out)
{
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(table_rsrc(t, bytes), (int) (uint32_t) (bytes - 16), 0, 0);
  out[0] = v.x;
}

static float timed(hipEvent_t a, hipEvent_t b)
{
  float ms;
  CHECK(hipEventSynchronize(b));
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

int main(int argc, char** argv)
{
  const double gb = argc > 1 ? atof(argv[1]) : 3.0;
  const uint64_t lines_target = (uint64_t) ((argc > 2 ? atof(argv[2]) : 512.0) * 1e6);
  const uint64_t bytes = (uint64_t) (gb * 1e9) & ~(uint64_t) 127;
  uint4* t;
  uint32_t* sink;
  /* PROBE_ALLOC: default (hipMalloc) | contig (hipDeviceMallocContiguous) |
   * vmm (hipMemCreate + 1 GiB-aligned hipMemAddressReserve) -- translation reach */
  const char* mode = getenv("PROBE_ALLOC") ? getenv("PROBE_ALLOC") : "default";
  if (!strcmp(mode, "contig")) {
    CHECK(hipExtMallocWithFlags((void**) &t, bytes, hipDeviceMallocContiguous));
  } else if (!strcmp(mode, "uncached")) {
    CHECK(hipExtMallocWithFlags((void**) &t, bytes, hipDeviceMallocUncached));
  } else if (!strcmp(mode, "vmm")) {
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gmin = 0, grec = 0;
    CHECK(hipMemGetAllocationGranularity(&gmin, &prop, hipMemAllocationGranularityMinimum));
    CHECK(hipMemGetAllocationGranularity(&grec, &prop, hipMemAllocationGranularityRecommended));
    const size_t g = grec > gmin ? grec : gmin;
    const size_t sz = (bytes + g - 1) / g * g;
    hipMemGenericAllocationHandle_t h;
    CHECK(hipMemCreate(&h, sz, &prop, 0));
    void* va = nullptr;
    CHECK(hipMemAddressReserve(&va, sz, 1ull << 30, nullptr, 0));
    CHECK(hipMemMap(va, sz, 0, h, 0));
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    CHECK(hipMemSetAccess(va, sz, &acc, 1));
    t = (uint4*) va;
    printf("{\"vmm_granularity_min\": %zu, \"recommended\": %zu}\n", gmin, grec);
  } else {
    CHECK(hipMalloc(&t, bytes));
  }
  printf("{\"alloc\": \"%s\"}\n", mode);
  CHECK(hipMalloc(&sink, 4));
  CHECK(hipMemset(t, 0x5a, bytes));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const uint32_t threads = 256 * 256 * 8;   /* 8 blocks of 256 per CU */
  const dim3 grid(threads / 256), blk(256);
  printf("{\"probe\": \"gather\", \"table_bytes\": %llu}\n", (unsigned long long) bytes);

  auto run = [&](const char* name, int lb, auto launch, double nlines) {
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    launch();
    CHECK(hipEventRecord(e1));
    const float ms = timed(e0, e1);
    printf("{\"kind\": \"%s\", \"line_B\": %d, \"ms\": %.3f, \"Glines_s\": %.2f, \"GB_s\": %.1f}\n", name, lb,
           ms, nlines / ms / 1e6, nlines * lb / ms / 1e6);
    fflush(stdout);
  };
  if (getenv("PROBE_CPOL")) {
    if (bytes >= (1ull << 32)) { fprintf(stderr, "PROBE_CPOL: table must be < 4 GB\n"); return 1; }
    uint32_t chk = 0;
    hipLaunchKernelGGL(k_rsrc_check, dim3(1), dim3(1), 0, 0, t, bytes, sink);
    CHECK(hipMemcpy(&chk, sink, 4, hipMemcpyDeviceToHost));
    printf("{\"rsrc_check\": \"0x%08x\", \"ok\": %s}\n", chk, chk == 0x5a5a5a5au ? "true" : "false");
    const uint64_t pg = (lines_target / (threads / 8) + 3) & ~3ull;
    const double nl = (double) pg * (threads / 8);
    run("coop_plain", 128, [&] { hipLaunchKernelGGL((k_coop_pol<0>), grid, blk, 0, 0, t, bytes / 128, pg, sink); }, nl);
    run("coop_sc0", 128, [&] { hipLaunchKernelGGL((k_coop_pol<1>), grid, blk, 0, 0, t, bytes / 128, pg, sink); }, nl);
    run("coop_nt", 128, [&] { hipLaunchKernelGGL((k_coop_pol<2>), grid, blk, 0, 0, t, bytes / 128, pg, sink); }, nl);
    run("coop_sc0_nt", 128, [&] { hipLaunchKernelGGL((k_coop_pol<3>), grid, blk, 0, 0, t, bytes / 128, pg, sink); }, nl);
    run("coop_sc1", 128, [&] { hipLaunchKernelGGL((k_coop_pol<16>), grid, blk, 0, 0, t, bytes / 128, pg, sink); }, nl);
    run("coop_sc0_sc1", 128, [&] { hipLaunchKernelGGL((k_coop_pol<17>), grid, blk, 0, 0, t, bytes / 128, pg, sink); }, nl);
    run("coop_sc1_nt", 128, [&] { hipLaunchKernelGGL((k_coop_pol<18>), grid, blk, 0, 0, t, bytes / 128, pg, sink); }, nl);
    run("coop_sc0_sc1_nt", 128, [&] { hipLaunchKernelGGL((k_coop_pol<19>), grid, blk, 0, 0, t, bytes / 128, pg, sink); }, nl);
    run("coop_ref", 128, [&] { hipLaunchKernelGGL((k_coop<128>), grid, blk, 0, 0, t, bytes / 128, pg, sink); }, nl);
    if (strcmp(mode, "vmm")) CHECK(hipFree(t));
    return 0;
  }
  if (getenv("PROBE_PAGES")) {
    /* lines (pages) per wave instruction for cooperative 128-B lines */
    const uint64_t nl = bytes / 128;
    const uint8_t* tb = reinterpret_cast<const uint8_t*>(t);
    for (int rep = 0; rep < 2; ++rep) {
      const uint64_t g16 = (lines_target / (threads / 8) + 3) & ~3ull;
      const uint64_t g8 = (lines_target / (threads / 16) + 3) & ~3ull;
      const uint64_t g4 = (lines_target / (threads / 32) + 3) & ~3ull;
      run("coopw16_8lines", 128, [&] { hipLaunchKernelGGL((k_coopw<16>), grid, blk, 0, 0, tb, nl, g16, sink); }, (double) g16 * (threads / 8));
      run("coopw8_4lines", 128, [&] { hipLaunchKernelGGL((k_coopw<8>), grid, blk, 0, 0, tb, nl, g8, sink); }, (double) g8 * (threads / 16));
      run("coopw4_2lines", 128, [&] { hipLaunchKernelGGL((k_coopw<4>), grid, blk, 0, 0, tb, nl, g4, sink); }, (double) g4 * (threads / 32));
    }
    if (strcmp(mode, "vmm")) CHECK(hipFree(t));
    return 0;
  }
  if (getenv("PROBE_MASK")) {
    const uint64_t pt = (lines_target / threads + 3) & ~3ull;
    const uint32_t st = (uint32_t) (lines_target / threads);
    run("indep_mask1", 64, [&] { hipLaunchKernelGGL((k_masked<64, 1>), grid, blk, 0, 0, t, bytes / 64, pt, sink); }, (double) pt * threads);
    run("indep_mask2", 64, [&] { hipLaunchKernelGGL((k_masked<64, 2>), grid, blk, 0, 0, t, bytes / 64, pt, sink); }, (double) pt * threads);
    run("indep_mask4", 64, [&] { hipLaunchKernelGGL((k_masked<64, 4>), grid, blk, 0, 0, t, bytes / 64, pt, sink); }, (double) pt * threads);
    run("indep_mask8", 64, [&] { hipLaunchKernelGGL((k_masked<64, 8>), grid, blk, 0, 0, t, bytes / 64, pt, sink); }, (double) pt * threads);
    run("indep_mask16", 64, [&] { hipLaunchKernelGGL((k_masked<64, 16>), grid, blk, 0, 0, t, bytes / 64, pt, sink); }, (double) pt * threads);
    run("chain_mask1", 64, [&] { hipLaunchKernelGGL((k_chain_masked<64, 1>), grid, blk, 0, 0, t, bytes / 64, st, sink); }, (double) st * threads);
    run("chain_mask4", 64, [&] { hipLaunchKernelGGL((k_chain_masked<64, 4>), grid, blk, 0, 0, t, bytes / 64, st, sink); }, (double) st * threads);
    run("chain_mask8", 64, [&] { hipLaunchKernelGGL((k_chain_masked<64, 8>), grid, blk, 0, 0, t, bytes / 64, st, sink); }, (double) st * threads);
    run("indep_mask8", 128, [&] { hipLaunchKernelGGL((k_masked<128, 8>), grid, blk, 0, 0, t, bytes / 128, pt, sink); }, (double) pt * threads);
    run("coop", 128, [&] { const uint64_t pg128 = (lines_target / (threads / 8) + 3) & ~3ull; hipLaunchKernelGGL((k_coop<128>), grid, blk, 0, 0, t, bytes / 128, pg128, sink); }, (double) ((lines_target / (threads / 8) + 3) & ~3ull) * (threads / 8));
    if (strcmp(mode, "vmm")) CHECK(hipFree(t));
    return 0;
  }
  {
    const uint64_t pt = (lines_target / threads + 3) & ~3ull;
    run("indep", 32, [&] { hipLaunchKernelGGL((k_indep<32>), grid, blk, 0, 0, t, bytes / 32, pt, sink); }, (double) pt * threads);
    run("indep", 64, [&] { hipLaunchKernelGGL((k_indep<64>), grid, blk, 0, 0, t, bytes / 64, pt, sink); }, (double) pt * threads);
    run("indep", 128, [&] { hipLaunchKernelGGL((k_indep<128>), grid, blk, 0, 0, t, bytes / 128, pt, sink); }, (double) pt * threads);
  }
  {
    const uint64_t pg32 = (lines_target / (threads / 2) + 3) & ~3ull;
    const uint64_t pg64 = (lines_target / (threads / 4) + 3) & ~3ull;
    const uint64_t pg128 = (lines_target / (threads / 8) + 3) & ~3ull;
    run("coop", 32, [&] { hipLaunchKernelGGL((k_coop<32>), grid, blk, 0, 0, t, bytes / 32, pg32, sink); }, (double) pg32 * (threads / 2));
    run("coop", 64, [&] { hipLaunchKernelGGL((k_coop<64>), grid, blk, 0, 0, t, bytes / 64, pg64, sink); }, (double) pg64 * (threads / 4));
    run("coop", 128, [&] { hipLaunchKernelGGL((k_coop<128>), grid, blk, 0, 0, t, bytes / 128, pg128, sink); }, (double) pg128 * (threads / 8));
  }
  {
    const uint32_t st = (uint32_t) (lines_target / threads);
    run("chain1", 32, [&] { hipLaunchKernelGGL((k_chain<32, 1>), grid, blk, 0, 0, t, bytes / 32, st, sink); }, (double) st * threads);
    run("chain1", 64, [&] { hipLaunchKernelGGL((k_chain<64, 1>), grid, blk, 0, 0, t, bytes / 64, st, sink); }, (double) st * threads);
    run("chain1", 128, [&] { hipLaunchKernelGGL((k_chain<128, 1>), grid, blk, 0, 0, t, bytes / 128, st, sink); }, (double) st * threads);
    const uint32_t st2 = st / 2;
    run("chain2", 64, [&] { hipLaunchKernelGGL((k_chain<64, 2>), grid, blk, 0, 0, t, bytes / 64, st2, sink); }, (double) st2 * threads * 2);
  }
  /* smaller tables: L2 / MALL resident */
  for (double sub : {0.004, 0.2}) {
    const uint64_t sb = (uint64_t) (sub * 1e9) & ~(uint64_t) 127;
    const uint64_t pt = (lines_target / threads + 3) & ~3ull;
    printf("{\"table_bytes\": %llu}\n", (unsigned long long) sb);
    run("indep", 64, [&] { hipLaunchKernelGGL((k_indep<64>), grid, blk, 0, 0, t, sb / 64, pt, sink); }, (double) pt * threads);
  }
  if (strcmp(mode, "vmm")) CHECK(hipFree(t));
  return 0;
}
