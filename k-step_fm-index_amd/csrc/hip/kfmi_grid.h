/*
 * kfmi_grid.h -- grid sizes of the grid-stride (and persistent) launches.
 */
#ifndef KFMI_GRID_H_
#define KFMI_GRID_H_

#include <stdint.h>
#include <stdlib.h>

namespace kfmi {

/* Workgroups for a grid-stride launch: `want` (one per work tile), capped at
 * the launch's own bound `cap` and, when set, at KFMI_MAX_GRID -- a test knob:
 * with a cap of 1-4 workgroups every grid-stride loop of the library (device
 * FASTA rows, ftab and remainder builds, locate's row fill and walks, the
 * index interleave) runs many iterations at test sizes, the path taken only
 * past 2^32 work-items (more than 16 GB of reads) otherwise. */
static inline uint32_t grid_blocks(uint64_t want, uint64_t cap)
{
  static const uint64_t dbg = [] {
    const char* e = getenv("KFMI_MAX_GRID");
    const long long v = e ? atoll(e) : 0;
    return v > 0 ? (uint64_t) v : 0ull;
  }();
  uint64_t b = want < cap ? want : cap;
  if (dbg && b > dbg) b = dbg;
  return (uint32_t) (b ? b : 1);
}

}  // namespace kfmi

#endif  // KFMI_GRID_H_
