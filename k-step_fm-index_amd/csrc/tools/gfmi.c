/*
 * gfmi -- index builder CLI (reference common/generateIndex.c:30-55):
 *   gfmi <ref.fa> <refsize>     (K, d from KFMI_K / KFMI_D, default 2 / 64)
 * writes "<ref.fa>.<n>.<d>fmi<K>steps.fmi" (tag 100) and "<ref.fa>.<n>.fa".
 * KFMI_BUILD_GPU=0 forces the host builder.  KFMI_SA_RATE=r (a power of two)
 * also writes the row-sampled suffix array "<index>.sa" for locate (an
 * extension; the reference has none).
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
  {
    const uint32_t *sa;
    uint64_t count;
    uint32_t rate, h[14];
    char fn[1100];
    CHECK(kfmi_index_sa(index, &sa, &count, &rate));
    if (count) {
      CHECK(kfmi_index_header(index, h));
      snprintf(fn, sizeof fn, "%s.%u.%ufmi%usteps.fmi.sa", argv[1], h[2] - 1, h[5], h[1]);
      CHECK(kfmi_save_sa(fn, index));
    }
  }
  CHECK(saveRef(argv[1], ref));
  CHECK(freeIndex(&index));
  CHECK(freeReference(&ref, &index));
  return EXIT_SUCCESS;
}
