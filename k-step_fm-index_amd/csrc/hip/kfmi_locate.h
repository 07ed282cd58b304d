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
 * of its wave ends.  Slots are assigned without any search: the exclusive scan
 * of min(R - L, max_occ) gives each query's first slot, the query id is written
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
  uint32_t c = 0;
#pragma unroll
  for (int p = 0; p < G::PW; ++p) c |= ((pl[p] >> bit) & 1u) << p;
  return c;
}

// LF_K of one row (X must not be a '$' row D_s).
template <class G>
__device__ __forceinline__ uint32_t lf_row(const IdxArgs& ix, uint32_t X)
{
  const uint32_t c = row_code<G>(ix, X);
  uint32_t sx[2 * G::K];
  plane_xor<G::K>(c, sx);
  return lf_stream<G>(ix, X, c, sx);
}

// Each lane walks slot after slot (i, i + stride, ...).  Per iteration a lane
// either reads its row's sample (sampled row), stops at a '$' row, or takes
// one LF_K step; the sample load and the step's line load of the other lanes
// are in flight together, and the next slot's first row is prefetched.
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
    const bool smp = (r & mask) == 0u;
    int ds = -1;   /* r = D_s (SA = s): the walk cannot step past it */
#pragma unroll
    for (int s = G::K - 1; s >= 0; --s)
      if (r == ix.dl.dpos[s]) ds = s;
    uint32_t p = 0, nr = 0;
    if (smp) p = sa[r >> rate_log2];
    else if (ds < 0) nr = lf_row<G>(ix, r);
    if (smp || ds >= 0) {
      pos[i] = (smp ? p : (uint32_t) ds) + steps;
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

}  // namespace kfmi

#endif  // KFMI_LOCATE_H_
