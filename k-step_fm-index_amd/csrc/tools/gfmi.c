/*
 * gfmi -- index builder CLI (reference common/generateIndex.c:30-55):
 *   gfmi <ref.fa> <refsize>     (K, d from KFMI_K / KFMI_D, default 2 / 64)
 * writes "<ref.fa>.<n>.<d>fmi<K>steps.fmi" (tag 100) and "<ref.fa>.<n>.fa".
 * KFMI_BUILD_GPU=0 forces the host builder.
 */
#include <stdio.h>
#include <stdlib.h>
#include "../../../include/kstep_fmi.h"

#define CHECK(e) do { int32_t _e = (e); if (_e) { fprintf(stderr, "%s\n", errorCommon(_e)); return EXIT_FAILURE; } } while (0)

int main(int argc, char *argv[])
{
  void *ref = NULL, *index = NULL;
  if (argc < 3) { fprintf(stderr, "usage: %s <ref.fa> <refsize>\n", argv[0]); return EXIT_FAILURE; }
  CHECK(loadRef(argv[1], (uint32_t) strtoul(argv[2], NULL, 10), &ref));
  CHECK(buildIndex(ref, &index));
  CHECK(saveIndex(argv[1], index));
  CHECK(saveRef(argv[1], ref));
  CHECK(freeIndex(&index));
  CHECK(freeReference(&ref, &index));
  return EXIT_SUCCESS;
}
