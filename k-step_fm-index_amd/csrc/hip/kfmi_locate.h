/*
 * kfmi_locate.h -- SA interval -> text positions on the device (SURVEY.md
 * 8(f) row f4, "SA-interval -> locate").  The reference stops at [L, R)
 * (fmIndexCPUBaseline.c:288-290), so this row has no reference oracle: the
 * tests pin it against brute-force suffix arrays.
 *
 * Index side: a row-sampled suffix array, sa[r >> log2(rate)] = SA[r] for
 * every row r with r % rate == 0 (rate a power of two; rate 1 = the full SA,
 * 12 GB at 3 Gbase, which one MI355X holds beside the 3 GB MID128 lines).
 *
 * Walk: LF_K of a single row X is the ordinary rank step with the row's own
 * K-mer code c(X), read from the bit planes of its block: C'[c] + Occ'(c, X)
 * counts the suffixes smaller than c.S_X, so LF_K(X) is the row of suffix
 * SA[X] - K.  From each row of [L, R) the walk applies LF_K until it reaches
 * a sampled row (SA = sample + K*steps) or a '$' row D_s (SA = s + K*steps;
 * LF_K would wrap there).  SA drops by K per step, so every walk ends within
 * n/K steps, after about `rate` steps on average.
 *
 * Work distribution: one output slot per lane at a time; a lane whose walk
 * ends takes its next slot at once instead of idling until the longest walk
 * of its wave ends.  The per-lane walk takes slots i, i + stride, ...; the
 * cooperative walk (whose waves move in lockstep rounds) takes them from one
 * queue: each wave takes chunks of SLOT_CHUNK consecutive slots from a global
 * counter (one atomic per chunk) and hands them to its lanes as their walks
 * end, so no wave keeps stepping a few long walks while the queue still holds
 * work (a fixed order leaves each lane ~38 walks of geometric length whose
 * sums differ by hundreds of steps).  The slots' first rows are computed
 * without any search: the exclusive scan of
 * min(R - L, max_occ) gives each query's first slot, the query id is written
 * there and spread by an inclusive max-scan, and a coalesced pass turns it
 * into each slot's first row.
 */
#ifndef KFMI_LOCATE_H_
#define KFMI_LOCATE_H_

#include "kfmi_device.h"

namespace kfmi {

// K-mer code of row X itself: bit p = 2s+t of c(X) is bit t of code(BWT_s[X]),
// plane p of X's block at X's row (MSB-first words, genFMindex.c:402-424).
template <class G>
__device__ __forceinline__ uint32_t row_code(const IdxArgs& ix, uint32_t X)
{
  const uint32_t b = X / (uint32_t) G::D;
  const uint32_t o = X - b * (uint32_t) G::D;
  const uint32_t* pl = locate<G>(ix, b, 0u).planes + (o >> 5) * G::PW;
  const uint32_t bit = 31u - (o & 31u);
  /* the word group of row X: aligned to the planes and to its own 4*PW bytes */
  constexpr int A = plane_align<G>() < ((4 * G::PW) & -(4 * G::PW)) ? plane_align<G>() : ((4 * G::PW) & -(4 * G::PW));
  uint32_t w[G::PW];
  load_words<A, G::PW>(pl, w);
  uint32_t c = 0;
#pragma unroll
  for (int p = 0; p < G::PW; ++p) c |= ((w[p] >> bit) & 1u) << p;
  return c;
}

// A walk that cannot end at a suffix: its row is past n+1 (no suffix there --
// rows an AltCounters interval can reach past the sentinel, §3) or it has taken
// more steps than the text is long (a 'ref'-mode index whose BWT is not a
// permutation).  Such a slot reports LOST_POS instead of walking on; on an
// ACGT index every walk from a row below n+1 ends within n/K steps.
constexpr uint32_t LOST_POS = 0xFFFFFFFFu;

__device__ __forceinline__ bool walk_lost(const IdxArgs& ix, uint32_t r, uint32_t steps)
{
  return r >= ix.bwtsize || steps >= ix.bwtsize;
}

// LF_K of one row (X must not be a '$' row D_s).  On the AltCounters layouts
// a step taken backward from the sentinel -- the last real block, the codes
// whose counter sits in the next entry -- differs from the plain LF by a
// constant per code (the sentinel counts that block's '$' rows as their
// stored code, and under B5 its padding, transformIndexAlternateCounters.c:
// 420-431, §3); a walk needs the plain LF, so it is taken off (ac_tail row 3).
template <class G>
__device__ __forceinline__ uint32_t lf_row(const IdxArgs& ix, uint32_t X)
{
  const uint32_t c = row_code<G>(ix, X);
  uint32_t sx[2 * G::K];
  plane_xor<G::K>(c, sx);
  uint32_t v = lf_stream<G>(ix, X, c, sx);
  if constexpr (G::ACRULE || G::LAY == LAY_MIDAC) {
    const uint32_t b = X / (uint32_t) G::D;
    if (b + 1u == (ix.bwtsize + (uint32_t) G::D - 1u) / (uint32_t) G::D && ac_rule_e<G>(b, c))
      v -= ix.ac_tail[3u * (uint32_t) G::NC + c];
  }
  return v;
}

// Wave-level slot queue.  `want` lanes receive the next slots of the wave's
// chunk [cur, end), a new chunk is taken from *ctr when the chunk runs short
// (SLOT_CHUNK >= 64 slots, so one chunk always covers the rest).  Called by
// every lane of the wave (the caller's loop is wave-uniform).  Returns the
// lane's slot, or ~0 when it wants none or the queue is empty; slots a wave
// receives only grow, so once a lane is told "empty" it stays so.
constexpr uint32_t SLOT_CHUNK = 256;   // default chunk (KFMI_LOCATE_CHUNK: 64 .. 4096)

__device__ __forceinline__ uint64_t uniform64(uint64_t x)
{
  return ((uint64_t) __builtin_amdgcn_readfirstlane((uint32_t) (x >> 32)) << 32) |
         (uint64_t) __builtin_amdgcn_readfirstlane((uint32_t) x);
}

struct WaveSlots {
  uint64_t cur = 0, end = 0;   // wave-uniform
  uint64_t fixed = ~0ull;      // ctr == nullptr (KFMI_LOCATE_QUEUE=0): this lane's next slot of i, i + stride, ...
};

__device__ __forceinline__ uint64_t take_slot(bool want, WaveSlots& ws, unsigned long long* ctr, uint64_t total,
                                              uint32_t chunk = SLOT_CHUNK)
{
  if (!ctr) {   // fixed order (A/B reference)
    if (ws.fixed == ~0ull) ws.fixed = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (!want) return ~0ull;
    const uint64_t s = ws.fixed;
    ws.fixed += (uint64_t) gridDim.x * blockDim.x;
    return s < total ? s : ~0ull;
  }
  const uint64_t mask = __ballot(want);
  const uint32_t n = (uint32_t) __popcll(mask);
  if (n == 0) return ~0ull;
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t) (mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) mask, 0u));
  ws.cur = uniform64(ws.cur);   // the same in every lane: keep it (and the branches on it) scalar
  ws.end = uniform64(ws.end);
  const uint64_t have = ws.end - ws.cur;
  uint64_t slot;
  if (have >= n) {
    slot = ws.cur + rank;
    ws.cur += n;
  } else {
    unsigned long long base = ~0ull;   // queue already past its end: no more chunks
    if (ws.end < total) {
      if ((threadIdx.x & 63) == 0) base = atomicAdd(ctr, (unsigned long long) chunk);
      base = __shfl(base, 0);
    }
    slot = rank < have ? ws.cur + rank : (base == ~0ull ? ~0ull : base + (rank - have));
    ws.cur = base == ~0ull ? ws.end : base + (n - have);
    ws.end = base == ~0ull ? ws.end : base + chunk;
  }
  return want && slot < total ? slot : ~0ull;
}

// Each lane walks slot after slot (i, i + stride, ...).  Per iteration a lane
// either reads its row's sample (sampled row), stops at a '$' row, or takes
// one LF_K step; the sample load and the step's line load of the other lanes
// are in flight together, and the next slot's first row is prefetched.  (Fed
// from the slot queue of the cooperative walk below, this walk measured
// 13-20 % slower: profiles/r02/locate_r2au.jsonl.)
template <class G>
__global__ __launch_bounds__(256) void locate_kernel(IdxArgs ix, const uint32_t* __restrict__ sa, uint32_t rate_log2,
                                                     const uint32_t* __restrict__ rows, uint64_t total,
                                                     uint32_t* __restrict__ pos)
{
  const uint32_t mask = (1u << rate_log2) - 1u;
  const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
  uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  uint32_t r = rows[i];
  uint32_t r_next = i + stride < total ? rows[i + stride] : 0u;
  uint32_t steps = 0;
  for (;;) {   // a lane leaves once all its slots are done
    const bool lost = walk_lost(ix, r, steps);
    const bool smp = !lost && (r & mask) == 0u;
    int ds = -1;   /* r = D_s (SA = s): the walk cannot step past it */
#pragma unroll
    for (int s = G::K - 1; s >= 0; --s)
      if (r == ix.dl.dpos[s]) ds = s;
    uint32_t p = 0, nr = 0;
    if (smp) p = sa[r >> rate_log2];
    else if (ds < 0 && !lost) nr = lf_row<G>(ix, r);
    if (smp || ds >= 0 || lost) {
      pos[i] = lost ? LOST_POS : (smp ? p : (uint32_t) ds) + steps;
      i += stride;
      if (i >= total) break;
      r = r_next;
      r_next = i + stride < total ? rows[i + stride] : 0u;
      steps = 0;
    } else {
      r = nr;
      steps += G::K;
    }
  }
}

// ---------------------------------------------------------------------------
// MID128 lines: one round trip per walk step.  A row's K-mer code sits in its
// line's planes and the counter it then needs in the same line, so the
// per-lane walk above pays a line load plus a dependent L2 hit per step.
// Here each wave stages the whole line of every stepping lane HBM -> LDS with
// cooperative 16-byte global_load_lds (TPR lanes per line, one round = 1 KiB,
// as in the coop search kernel) and every lane takes its step from LDS.
// ---------------------------------------------------------------------------
template <class G>
__host__ __device__ constexpr bool locate_coop_ok()
{
  return G::LAY == LAY_MID && G::EW * 4 >= 16 && G::EW * 4 <= 128;
}

// LF_K of row X from its MID line in LDS (the same arithmetic as lf_row on LAY_MID)
template <class G>
__device__ __forceinline__ uint32_t lf_row_line(const IdxArgs& ix, const uint8_t* line, uint32_t X)
{
  const uint32_t* L = reinterpret_cast<const uint32_t*>(line);
  const uint32_t b = X / (uint32_t) G::D;
  const uint32_t o = X - b * (uint32_t) G::D;
  const bool e = (b & 1u) == 0;                     // even block: backward from the midpoint
  const uint32_t* pl = L + (b & 1u) * G::BMW;
  const uint32_t* pw = pl + (o >> 5) * G::PW;
  const uint32_t bit = 31u - (o & 31u);
  uint32_t c = 0;
#pragma unroll
  for (int p = 0; p < G::PW; ++p) c |= ((pw[p] >> bit) & 1u) << p;
  uint32_t sx[2 * G::K];
  plane_xor<G::K>(c, sx);
  uint32_t pop = 0;
#pragma unroll
  for (int w = 0; w < G::NB; ++w) {
    uint32_t m = row_mask((int) o - 32 * w);
    m = e ? ~m : m;
    pop += __popc(m & select_rows<G::K>(&pl[w * G::PW], sx));
  }
  return finish<G>(ix, L[G::MIDCNT + c], pop, b, c, X, e);
}

template <class G>
__global__ __launch_bounds__(256) void locate_coop_kernel(IdxArgs ix, const uint32_t* __restrict__ sa,
                                                          uint32_t rate_log2, const uint32_t* __restrict__ rows,
                                                          uint64_t total, uint32_t* __restrict__ pos,
                                                          unsigned long long* __restrict__ ctr, uint32_t chunk)
{
  constexpr int LB = G::EW * 4;     // line bytes
  constexpr int TPR = LB / 16;      // lanes per line
  constexpr int RPR = 64 / TPR;     // lines per 1 KiB round
  static_assert(locate_coop_ok<G>(), "MID lines of 16..128 bytes");
  __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 64 * LB];   // 32 KiB at 128-B lines: 5 workgroups per CU
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint8_t* wl = lds + wave * 64 * LB;
  const uint8_t* base = reinterpret_cast<const uint8_t*>(ix.ent);
  const uint32_t mask = (1u << rate_log2) - 1u;
  WaveSlots ws;
  uint64_t i = take_slot(true, ws, ctr, total, chunk);
  uint32_t r = i < total ? rows[i] : 0u;
  uint64_t i_n = take_slot(true, ws, ctr, total, chunk);
  uint32_t r_n = i_n < total ? rows[i_n] : 0u;
  bool act = i < total;
  uint32_t steps = 0;
  const int g = lane / TPR, k = lane % TPR;
  while (__ballot(act)) {   // wave-uniform: until every lane of the wave has no slot left
    const bool lost = act && walk_lost(ix, r, steps);
    const bool smp = act && !lost && (r & mask) == 0u;
    int ds = -1;   /* r = D_s (SA = s): the walk cannot step past it */
#pragma unroll
    for (int s = G::K - 1; s >= 0; --s)
      if (r == ix.dl.dpos[s]) ds = s;
    const bool step = act && !smp && ds < 0 && !lost;
    uint32_t p = 0;
    if (smp) p = sa[r >> rate_log2];
    const uint32_t mine = step ? r / (uint32_t) (2 * G::D) : 0xFFFFFFFFu;   // this lane's MID line, or none
#pragma unroll
    for (int rr = 0; rr < 64 / RPR; ++rr) {
      const uint32_t li = __shfl(mine, rr * RPR + g);   // line of lane rr*RPR+g (no LDS table)
      if (li != 0xFFFFFFFFu)
        __builtin_amdgcn_global_load_lds((const void*) (base + (uint64_t) li * LB + 16 * k),
                                         (__attribute__((address_space(3))) void*) (wl + rr * 1024), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t nr = step ? lf_row_line<G>(ix, wl + lane * LB, r) : 0u;
    const bool fin = smp || (act && (ds >= 0 || lost));
    if (fin) {
      pos[i] = lost ? LOST_POS : (smp ? p : (uint32_t) ds) + steps;
      i = i_n;
      r = r_n;
      act = i < total;
      steps = 0;
    } else if (act) {
      r = nr;
      steps += G::K;
    }
    const uint64_t got = take_slot(fin, ws, ctr, total, chunk);
    if (fin) {
      i_n = got;
      r_n = got < total ? rows[got] : 0u;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // LDS reads done before the next round overwrites
  }
}

}  // namespace kfmi

#endif  // KFMI_LOCATE_H_
