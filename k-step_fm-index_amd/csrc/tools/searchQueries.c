/*
 * searchQueries -- the search driver (reference common/searchQueries.c:34-132):
 *   searchQueries <index> <queries.qry> <qrysize> <numqueries>
 * load index -> load queries -> initResults -> transferCPUtoGPU -> timed
 * searchIndexGPU x iters -> transferGPUtoCPU -> saveResults("<index>.res.gpu").
 * Prints "TIME: <mean seconds per iteration>" like the reference, plus the
 * device-side (HIP event) times of the last iteration.
 * Environment: KFMI_BACKEND (task|coop|task-ac|coop-ac|task-packed|coop-packed),
 * KFMI_DEVICE, KFMI_ITERS (default 5, the reference's `iter`).
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
