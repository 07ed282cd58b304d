/*
 * searchQueries -- the search driver (reference common/searchQueries.c:34-132):
 *   searchQueries <index> <queries.qry> <qrysize> <numqueries>
 * load index -> load queries -> initResults -> transferCPUtoGPU -> timed
 * searchIndexGPU x iters -> transferGPUtoCPU -> saveResults("<index>.res.gpu").
 * Prints "TIME: <mean seconds per iteration>" like the reference, plus the
 * device-side (HIP event) times of the last iteration.
 * Environment: KFMI_BACKEND (task|coop|task-ac|coop-ac|task-mid|coop-mid|
 * task-ac-mid|coop-ac-mid|task-grp|coop-grp), KFMI_DEVICE, KFMI_ITERS (default 5,
 * the reference's `iter`), KFMI_FTAB.
 * Locate (extension): KFMI_SA_FILE=<samples written by gfmi> also writes
 * "<index>.pos.gpu": per query "<n> <p1> ... <pn>" (text positions, suffix
 * order; at most KFMI_MAX_OCC per query when set).
 */
#include <stdio.h>
#include <stdlib.h>
#include "../../../include/kstep_fmi.h"

#define CHECK(e) do { int32_t _e = (e); if (_e) { fprintf(stderr, "%s\n", errorCommon(_e)); return EXIT_FAILURE; } } while (0)

int main(int argc, char *argv[])
{
  void *index = NULL, *queries = NULL, *results = NULL;
  const char *it = getenv("KFMI_ITERS");
  int iters = it ? atoi(it) : 5, n;
  uint32_t qrysize, numqueries;
  double t0, t1, tot, pack, lf;
  if (argc < 5) {
    fprintf(stderr, "usage: %s <index> <queries> <qrysize> <numqueries>\n", argv[0]);
    return EXIT_FAILURE;
  }
  qrysize = (uint32_t) strtoul(argv[3], NULL, 10);
  numqueries = (uint32_t) strtoul(argv[4], NULL, 10);
  CHECK(loadIndex(argv[1], &index));
  CHECK(loadQueries(argv[2], qrysize, numqueries, &queries));
  CHECK(initResults(numqueries, &results));
  CHECK(transferCPUtoGPU(index, queries, results));
  t0 = sampleTime();
  for (n = 0; n < iters; n++) {
    searchIndexGPU(index, queries, results);
    CHECK(kfmi_last_error());
  }
  t1 = sampleTime();
  if (getenv("KFMI_SA_FILE")) {
    void *loc = NULL;
    const char *mo = getenv("KFMI_MAX_OCC");
    char fn[1100];
    FILE *fp;
    uint32_t q;
    CHECK(kfmi_load_sa(getenv("KFMI_SA_FILE"), index));
    CHECK(kfmi_locate(index, results, mo ? (uint32_t) strtoul(mo, NULL, 10) : 0u, &loc));
    snprintf(fn, sizeof fn, "%s.pos.gpu", argv[1]);
    fp = fopen(fn, "w");
    if (!fp) { fprintf(stderr, "cannot write %s\n", fn); return EXIT_FAILURE; }
    {
      const uint64_t *off = kfmi_locations_offsets(loc);
      const uint32_t *pos = kfmi_locations_positions(loc);
      for (q = 0; q < numqueries; q++) {
        uint64_t i;
        fprintf(fp, "%llu", (unsigned long long) (off[q + 1] - off[q]));
        for (i = off[q]; i < off[q + 1]; i++) fprintf(fp, " %u", pos[i]);
        fputc('\n', fp);
      }
    }
    fclose(fp);
    printf("LOCATE: %llu positions\n", (unsigned long long) kfmi_locations_total(loc));
    kfmi_locations_free(&loc);
  }
  CHECK(transferGPUtoCPU(results));
  CHECK(saveResults(argv[1], results, index));
  CHECK(freeIndexGPU(&index));
  CHECK(freeQueriesGPU(&queries));
  CHECK(freeResultsGPU(&results));
  kfmi_last_timing(&tot, &pack, &lf);
  printf("BACKEND: %s\n", kfmi_get_backend());
  printf("TIME: \t %f \n", iters ? (t1 - t0) / iters : 0.0);
  printf("DEVICE_MS: total %.3f pack %.3f lf %.3f\n", tot, pack, lf);
  freeIndex(&index);
  freeQueries(&queries);
  freeResults(&results);
  return EXIT_SUCCESS;
}
